# MI355X serving image: ROCm + PyTorch-ROCm base, in-tree gfx950 HIP kernels
# and the C++ runtime compiled at build time (hipcc --offload-arch=gfx950).
ARG BASE=rocm/pytorch:latest
FROM ${BASE}
ENV PYTORCH_ROCM_ARCH=gfx950 \
    HSA_ENABLE_IPC_MODE_LEGACY=0 \
    PYTHONUNBUFFERED=1
WORKDIR /opt/llm-mcp-amd
COPY . .
RUN python -c "from llm_mcp_amd.build import build_all; build_all(verbose=True)"
EXPOSE 8080 9090 3333
ENTRYPOINT ["python", "-m", "llm_mcp_amd"]
CMD ["serve"]
