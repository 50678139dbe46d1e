#!/bin/bash
# One gpurun session: each GPU step under its own time limit, chained so the
# first failure ends the call.  Usage (on the GPU box, from the repo root):
#   bash tools/gpu_session.sh STEP [STEP...]
# Steps: the case labels below (tests, smoke, bench1, bench20, soak, rehearse*, tp8s, the
# probes and counter passes).  Same-box A/B steps (pf_ab, pf_abab, alloc_ab, sample_ab, ...)
# also run a second package tree under ab/<name> (git-ignored, built on the CPU side before
# the call): a copy of the repo with the older sources checked out and
# `python -c "from llm_mcp_amd import build; build.build_kernels(); build.build_runtime()"`.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[gpu_session] $name: $*" >&2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[gpu_session] $name exit $rc" >&2
  tail -n 3 "gpurun_out/$name.log" >&2
  return $rc
}
for step in "$@"; do
  case $step in
    tests)
      run gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 \
          --timeout-method thread -p no:cacheprovider || exit $? ;;
    bench1)
      run bench1 600 python bench.py --steps 3 --warmup 1 || exit $? ;;
    rehearse2)
      run rehearse2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
          --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 2 --warmup 1 \
          --concurrency 64 --rehearse-on-one-gpu --api-procs 2 || exit $? ;;
    rehearse4)
      run rehearse4 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
          --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 4 --steps 2 --warmup 1 \
          --concurrency 32 --rehearse-on-one-gpu || exit $? ;;
    rehearse4s)
      # the driver's own command path (no launcher: bench.self_launch) at 4 ranks
      run rehearse4s 600 python3 bench.py --gpus 4 --rehearse-on-one-gpu --model llama-3-8b@L8 \
          --steps 2 --warmup 1 --concurrency 64 || exit $? ;;
    rehearse8s)
      run rehearse8s 900 python3 bench.py --gpus 8 --rehearse-on-one-gpu --model llama-3-8b@L8 \
          --steps 2 --warmup 1 --concurrency 32 || exit $? ;;
    tp8s)
      # config 4's launcher shape: one TP-8 engine of the 70B layer shapes (8 layers)
      run tp8s 900 python3 bench.py --gpus 8 --tp 8 --rehearse-on-one-gpu \
          --model llama-3-70b@L8 --steps 2 --warmup 1 --concurrency 32 --max-tokens 64 || exit $? ;;
    dgemm70)
      # every TP = 8 rank projection shape: K11 tiles / splits / stream-K vs the library
      # (rows kept for --from-rows; the table is rewritten on the CPU side)
      run dgemm70 1100 python -u -m llm_mcp_amd.bench.dgemm_bench --model llama-3-70b --tp 8 \
          --only ${DG_ONLY:-qkv,o,gate_up,down} --json gpurun_out/dgemm70_rows.json || exit $? ;;
    rs70)
      # K14 on the TP = 8 rank's gate/up (SwiGLU16) and down at M = 256
      : > gpurun_out/rs70.log
      timeout -k 10 200 tools/labbin/rsgemm_lab 7168 8192 256 3 \
          rs:38:1,rs:38:2,rs:38:4,rs:46:1,rs:46:2,rs:34:2,rs:34:4 >> gpurun_out/rs70.log 2>&1 || exit $?
      timeout -k 10 200 tools/labbin/rsgemm_lab 8192 3584 256 0 \
          rs:38:1,rs:38:2,rs:38:4,rs:46:1,rs:46:2,dg:4:1,dg:8:1 >> gpurun_out/rs70.log 2>&1 || exit $?
      cat gpurun_out/rs70.log ;;
    attn70)
      # one TP = 8 rank's decode attention: 256 rows x 1 kv head x 8 q heads, split-K partitions
      : > gpurun_out/attn70.log
      for parts in 1 2 3 4; do
        timeout -k 10 120 python -u tools/decode_attn_probe.py --layout engine --rope --hq 8 \
            --hkv 1 --batch 256 --ctx-lo 512 --ctx-hi 640 --parts $parts --modes 0,10,4 --pages 100000 \
            --iters 40 >> gpurun_out/attn70.log 2>&1 || exit $?
      done
      cat gpurun_out/attn70.log ;;
    qkv70)
      # the TP = 8 rank's narrow QKV (1280 x 8192): every K11 tile / split / stream-K form
      run qkv70 600 python -u -m llm_mcp_amd.bench.dgemm_bench --model llama-3-70b --tp 8 \
          --only qkv --m ${QKV_MS:-64,128,192,256} --json gpurun_out/qkv70_rows.json || exit $? ;;
    tp8s_la)
      # the same with TP lookahead stepping (every rank samples the all-gathered logits)
      LMX_LOOKAHEAD=1 run tp8s_la 900 python3 bench.py --gpus 8 --tp 8 --rehearse-on-one-gpu \
          --model llama-3-70b@L8 --steps 2 --warmup 1 --concurrency 32 --max-tokens 64 || exit $? ;;
    dgemm_tests)
      run dgemm_tests 600 python -u -m pytest tests/test_kernels_gpu.py -k dgemm -x -q --timeout 120 \
          --timeout-method thread -p no:cacheprovider || exit $? ;;
    dgemm_bench)
      run dgemm_bench 900 python -u -m llm_mcp_amd.bench.dgemm_bench --json gpurun_out/dgemm_rows.json \
          --write || exit $?
      cp llm_mcp_amd/config/dgemm_gfx950.json gpurun_out/ ;;
    prof_engine)
      rm -rf gpurun_out/prof_engine
      run prof_engine 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_engine -o run \
          -- python3 -m llm_mcp_amd.bench.engine_bench --batch 256 --max-tokens 64 || exit $? ;;
    pmc_dgemm)
      # three counter passes over K11 vs the library on one shape (PMC_ARGS="N K M CFG S EPI")
      for pass in \
        "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT" \
        "FETCH_SIZE TCC_HIT_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM GRBM_GUI_ACTIVE" \
        "TCC_MISS_sum TCC_HIT_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum" ; do
        n=$(( ${n:-0} + 1 ))
        rm -rf gpurun_out/pmc_dgemm_$n
        run pmc_dgemm_$n 120 timeout -s KILL 100 rocprofv3 --pmc $pass --kernel-trace -d gpurun_out/pmc_dgemm_$n \
            -o run --output-format csv -- python3 tools/prof_dgemm_probe.py $PMC_ARGS || exit $?
      done ;;
    pmc_engine)
      # counter passes over a short eager engine run (every kernel of prefill + decode)
      n=0
      for pass in \
        "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT" \
        "FETCH_SIZE TCC_HIT_sum SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
        "WRITE_SIZE TCC_MISS_sum TCC_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum" ; do
        n=$(( n + 1 ))
        rm -rf gpurun_out/pmc_engine_$n
        run pmc_engine_$n 300 timeout -s KILL 280 rocprofv3 --pmc $pass --kernel-trace -d gpurun_out/pmc_engine_$n \
            -o run --output-format csv -- python3 -m llm_mcp_amd.bench.engine_bench --batch 128 \
            --prompt-len 512 --max-tokens 8 --no-graphs --max-batched-tokens 16384 || exit $?
      done ;;
    pmc_attn)
      # decode attention at the headline shape (fused rope form, the persistent
      # default and the grid form): LDS share and conflicts, waits, and the
      # HBM read rate, one counter pass each
      n=0
      for pass in \
        "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
        "FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE" \
        "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum TCC_MISS_sum TCC_HIT_sum GRBM_GUI_ACTIVE" ; do
        n=$(( n + 1 ))
        rm -rf gpurun_out/pmc_attn_$n
        run pmc_attn_$n 120 timeout -s KILL 100 rocprofv3 --pmc $pass --kernel-trace -d gpurun_out/pmc_attn_$n \
            -o run --output-format csv -- python3 tools/decode_attn_probe.py --layout engine --rope \
            --modes 0,4 --iters 20 || exit $?
      done
      python tools/pmc_table.py gpurun_out/pmc_attn_1 gpurun_out/pmc_attn_2 gpurun_out/pmc_attn_3 \
          --match paged_decode > gpurun_out/pmc_attn_table.md 2>&1 || true ;;
    pmc_pf)
      # prefill attention (K3), one shape at a time (PF_SHAPES, comma list): MFMA busy,
      # waits, LDS, L2 fetch -- one counter pass each
      for shape in ${PF_SHAPES//,/ }; do
        n=0
        for pass in \
          "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
          "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE" \
          "FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE" ; do
          n=$(( n + 1 ))
          rm -rf gpurun_out/pmc_pf_${shape}_$n
          run pmc_pf_${shape}_$n 120 timeout -s KILL 100 rocprofv3 --pmc $pass --kernel-trace \
              -d gpurun_out/pmc_pf_${shape}_$n -o run --output-format csv -- python3 \
              tools/prefill_attn_probe.py --shapes $shape --waves 4 --iters 10 || exit $?
        done
        python tools/pmc_table.py gpurun_out/pmc_pf_${shape}_1 gpurun_out/pmc_pf_${shape}_2 \
            gpurun_out/pmc_pf_${shape}_3 --match paged_prefill > gpurun_out/pmc_pf_${shape}.md 2>&1 || true
      done ;;
    list_counters)
      run list_counters 120 rocprofv3 -L || exit $? ;;
    tp_tests)
      run tp_tests 600 python -u -m pytest tests/test_00_peer_ar_gpu.py tests/test_00_tp_gpu.py -x -v \
          --timeout 300 --timeout-method thread -p no:cacheprovider || exit $? ;;
    tune70b)
      run tune70b 900 python -u -m llm_mcp_amd.bench.tune_gemms --model llama-3-70b --tp 8 \
          --out gpurun_out/tunableop_70b_tp8.csv --max-ms 40 || exit $? ;;
    dgemm70b)
      run dgemm70b 600 python -u -m llm_mcp_amd.bench.dgemm_bench --model llama-3-70b --tp 8 \
          --json gpurun_out/dgemm_rows_70b.json --write || exit $?
      cp llm_mcp_amd/config/dgemm_gfx950.json gpurun_out/dgemm_gfx950_70b.json ;;
    config5)
      # BASELINE config 5 on one GPU: two workers (chat + embed each) on cuda:0,
      # 256 concurrent mixed jobs + sync chats, injected HIP faults on one worker
      run config5 900 python -u -m llm_mcp_amd.bench.serving_bench mixed --gpus 0 \
          --replicas-per-gpu 2 --fault gpu_error:0.002 --fault-device gpu0.r1 \
          --jobs 1024 --concurrency 256 --sync-every 4 --max-tokens 64 --chars 512 || exit $? ;;
    config5det)
      # config 5 with a FIXED fault schedule (the faulty worker fails at its
      # 300th engine step, every life) and the median of 3 runs; 4096 jobs per
      # run so each run spans several fault/restart cycles (1024-job runs: one
      # fault per ~10 s run, 84-112 jobs/s spread from where it lands)
      run config5det 1100 python -u -m llm_mcp_amd.bench.serving_bench mixed --gpus 0 \
          --replicas-per-gpu 2 --fault gpu_error@300 --fault-device gpu0.r1 --runs 3 \
          --jobs 4096 --concurrency 256 --sync-every 4 --max-tokens 64 --chars 512 || exit $? ;;
    config5r4)
      # round 4's recorded config-5 command (profiles/r4_config5.md): the faulty worker fails
      # once (its first life), then the run waits for its recovery; median of 3 runs
      run config5r4 1100 python -u -m llm_mcp_amd.bench.serving_bench mixed --gpus 0 \
          --replicas-per-gpu 2 --fault gpu_error@300 --fault-device gpu0.r1 --fault-lives 1 \
          --runs 3 --jobs 4096 --concurrency 256 --sync-every 4 --max-tokens 64 --chars 512 \
          --await-recovery 150 || exit $? ;;
    config5b)
      # config 5, round 4: the faulty worker's first life fails at its 300th
      # engine step (LMX_FAULT_LIVES=1), the breaker trips from the released
      # leases, the supervisor restarts the worker; after each 4096-job run
      # the bench waits for the restarted worker to be alive and online again
      run config5b 1150 python -u -m llm_mcp_amd.bench.serving_bench mixed --gpus 0 \
          --replicas-per-gpu 2 --fault gpu_error@300 --fault-device gpu0.r1 --fault-lives 1 \
          --runs 3 --jobs 4096 --concurrency 256 --sync-every 4 --max-tokens 64 --chars 512 \
          --await-recovery 150 || exit $? ;;
    tp_rehearse)
      # BASELINE config 4's launcher on one GPU: bench.py --tp 2 with the 70B
      # layer shapes cut to 8 layers (a plumbing rehearsal, never an N-GPU number)
      run tp_rehearse 480 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
          --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --tp 2 \
          --rehearse-on-one-gpu --model llama-3-70b@L8 --concurrency 64 --max-tokens 128 \
          --steps 2 --warmup 1 || exit $? ;;
    encoder_bench)
      run encoder_bench 600 python -u -m llm_mcp_amd.bench.dgemm_bench --encoder 4096,32768 || exit $? ;;
    prof_bench)
      # the headline bench under a kernel trace; tools/prof_timeline.py splits it into waves/steps
      # (PROF_TAG names the run: a second traced run under another env in the same call;
      # PROF_ARGS adds bench.py options, e.g. another model)
      tag=${PROF_TAG:-prof_bench}
      rm -rf gpurun_out/$tag
      run $tag 900 rocprofv3 --kernel-trace -d gpurun_out/$tag -o run \
          -- python3 bench.py --steps 2 --warmup 1 ${PROF_ARGS:-} || exit $?
      python tools/prof_timeline.py gpurun_out/$tag/run_results.db --waves 2 \
          > gpurun_out/${tag}_timeline.md 2>&1 || true
      rm -rf gpurun_out/$tag ;;   # the trace database alone exceeds what gpurun copies back
    attn_probe)
      run attn_probe 180 python -u tools/decode_attn_probe.py || exit $? ;;
    tp_graph_tests)
      run tp_graph_tests 900 python -u -m pytest tests/test_00_tp_gpu.py -x -v --timeout 400 \
          --timeout-method thread -p no:cacheprovider || exit $? ;;
    smi_dump)
      rocm-smi --showclocks --showpower --showmaxpower --showtemp --json > gpurun_out/smi_dump.json \
          2>&1 || true ;;
    bench_cap16)
      run bench_cap16 600 python bench.py --steps 3 --warmup 1 --mixed-prefill-tokens 16384 \
          || exit $? ;;
    closed_cap16)
      run closed_cap16 600 python bench.py --load closed --duration 30 --closed-warmup 10 \
          --mixed-prefill-tokens 16384 || exit $? ;;
    bench_nocap)
      # the round-4 behaviour (no mixed-step prefill cap) for the A/B
      run bench_nocap 600 python bench.py --steps 3 --warmup 1 --mixed-prefill-tokens 0 || exit $? ;;
    closed_default)
      run closed_default 600 python bench.py --load closed --duration 30 --closed-warmup 10 \
          || exit $? ;;
    conc512)
      run conc512 600 python bench.py --steps 2 --warmup 1 --concurrency 512 || exit $? ;;
    down_norm)
      run down_norm 180 python -u tools/down_norm_probe.py || exit $?
      run down_norm_o 180 python -u tools/down_norm_probe.py --k 4096 || exit $? ;;
    rows_split_probe)
      run rows_split_probe 300 python -u tools/rows_split_probe.py || exit $? ;;
    fill_ab)
      # the headline load, same box: the old K13 rule vs the wave-fill rule (default)
      for i in 1 2; do
        LMX_K13_MIN_FILL=0 LMX_ROWS_SPLIT_MAX=0 run fill_off_$i 600 python bench.py --steps 6 --warmup 2 || exit $?
        run fill_on_$i 600 python bench.py --steps 6 --warmup 2 || exit $?
      done ;;
    conc512_ab)
      # 512 streams, same box: K13 on every >= 512-row product (the old rule) vs the default
      # (hipBLASLt below 60 % K13 wave fill, K14 row pieces for packed-only weights)
      for i in 1 2; do
        LMX_K13_MIN_FILL=0 LMX_ROWS_SPLIT_MAX=0 run conc512_off_$i 600 python bench.py --steps 2 --warmup 1 --concurrency 512 || exit $?
        run conc512_on_$i 600 python bench.py --steps 2 --warmup 1 --concurrency 512 || exit $?
      done ;;
    closed64)
      run closed64 600 python bench.py --load closed --duration 30 --closed-warmup 10 \
          --concurrency 64 || exit $? ;;
    closed_nocap)
      run closed_nocap 600 python bench.py --load closed --duration 30 --closed-warmup 10 \
          --mixed-prefill-tokens 0 || exit $? ;;
    poisson)
      run poisson 600 python bench.py --load poisson --rate ${POISSON_RATE:-60} --duration 30 \
          --closed-warmup 10 || exit $? ;;
    long2k)
      run long2k 900 python bench.py --steps 2 --warmup 1 --prompt-len 2048 --max-tokens 256 \
          || exit $? ;;
    long8k)
      run long8k 900 python bench.py --steps 2 --warmup 1 --prompt-len 7680 --max-tokens 256 \
          --concurrency 64 || exit $? ;;
    proxy70)
      # config 4's per-rank decode on one GPU (llama-3-70b-tp8-rank), under a kernel trace
      rm -rf gpurun_out/proxy70
      run proxy70 900 rocprofv3 --kernel-trace -d gpurun_out/proxy70 -o run \
          -- python3 bench.py --model llama-3-70b-tp8-rank --concurrency 256 --max-tokens 128 \
          --steps 2 --warmup 1 || exit $?
      python tools/prof_timeline.py gpurun_out/proxy70/run_results.db --waves 2 \
          > gpurun_out/proxy70_timeline.md 2>&1 || true
      rm -rf gpurun_out/proxy70 ;;
    peer_tests)
      run peer_tests 600 python -u -m pytest tests/test_00_peer_ar_gpu.py -x -v --timeout 300 \
          --timeout-method thread -p no:cacheprovider || exit $? ;;
    engine_tests)
      run engine_tests 600 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 \
          --timeout-method thread -p no:cacheprovider || exit $? ;;
    pf_probe)
      run pf_probe 300 python -u tools/prefill_attn_probe.py \
          --shapes ${PF_SHAPES:-llama8b,llama8b_2k,llama8b_8k,nomic} --waves 4,8 || exit $? ;;
    pf_tests)
      run pf_tests 400 python -u -m pytest tests/test_kernels_gpu.py -k prefill -x -q \
          --timeout 120 --timeout-method thread -p no:cacheprovider || exit $? ;;
    pf_ab)
      # prefill attention forms A/B: 4- vs 8-wave, 2 vs 3 ring slots
      run pf_ab 400 python -u tools/prefill_attn_probe.py \
          --shapes ${PF_SHAPES:-llama8b,llama8b_2k,llama8b_8k,nomic} --waves 4,8 --stages 0,3 \
          || exit $? ;;
    pf_abab)
      # same-box A/B of two builds (ab/head: the committed tree's package), alternating
      : > gpurun_out/pf_abab.log
      for i in 1 2; do
        for root in ${PF_ROOTS:-ab/head .}; do
          echo "== build $root" >> gpurun_out/pf_abab.log
          timeout -k 10 200 python -u tools/prefill_attn_probe.py --pkg-root $root \
              --shapes ${PF_SHAPES:-llama8b,llama8b_2k,llama8b_8k,nomic} --waves 4 \
              >> gpurun_out/pf_abab.log 2>&1 || exit $?
        done
      done
      grep -E "==|prefill attn" gpurun_out/pf_abab.log ;;
    packed_tests)
      run packed_tests 600 python -u -m pytest tests/test_packed_weights_gpu.py tests/test_engine_gpu.py \
          -x -v --timeout 200 --timeout-method thread -p no:cacheprovider || exit $? ;;
    bench_two_copies)
      LMX_RS_SINGLE=0 run bench_two_copies 600 python bench.py --steps 3 --warmup 1 || exit $? ;;
    l70)
      # Llama-3-70B at TP = 1 (review round 4, item 6): one copy of the MLP weights, K14 decode
      run l70 1000 python bench.py --model llama-3-70b --concurrency 128 --max-tokens 128 \
          --steps 2 --warmup 1 || exit $? ;;
    l70_ab)
      # Llama-3-70B TP = 1 under the round-6 serving defaults vs the round-5 budget / no cap,
      # alternating, twice
      for i in 1 2; do
        run l70_def_$i 600 python bench.py --model llama-3-70b --concurrency 128 --max-tokens 128 \
            --steps 2 --warmup 1 || exit $?
        LMX_MAX_BATCHED_TOKENS=24576 run l70_b24k_$i 600 python bench.py --model llama-3-70b \
            --concurrency 128 --max-tokens 128 --steps 2 --warmup 1 || exit $?
        LMX_MAX_BATCHED_TOKENS=24576 LMX_MIXED_PREFILL_TOKENS=0 run l70_r5_$i 600 python bench.py \
            --model llama-3-70b --concurrency 128 --max-tokens 128 --steps 2 --warmup 1 || exit $?
      done ;;
    l70_two)
      LMX_RS_SINGLE=0 run l70_two 1000 python bench.py --model llama-3-70b --concurrency 128 \
          --max-tokens 128 --steps 2 --warmup 1 || exit $? ;;
    nf_tests)
      run nf_tests 600 python -u -m pytest tests/test_norm_fold_gpu.py tests/test_packed_weights_gpu.py \
          tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "norm or fold or pgemm or packed or engine or prefill or lookahead" \
          -x -q --timeout 200 --timeout-method thread -p no:cacheprovider || exit $? ;;
    bench_nofold)
      LMX_NORM_FOLD=0 run bench_nofold 600 python bench.py --steps 3 --warmup 1 || exit $? ;;
    long8k_nofold)
      LMX_NORM_FOLD=0 run long8k_nofold 900 python bench.py --steps 2 --warmup 1 --prompt-len 7680 \
          --max-tokens 256 --concurrency 64 || exit $? ;;
    qkv70tp1)
      # Llama-3-70B TP = 1 QKV (10240 x 8192) at every decode bucket (M 17-48 were library)
      run qkv70tp1 900 python -u -m llm_mcp_amd.bench.dgemm_bench --model llama-3-70b --tp 1 \
          --only qkv --json gpurun_out/qkv70tp1_rows.json || exit $? ;;
    lm70tp1)
      run lm70tp1 900 python -u -m llm_mcp_amd.bench.dgemm_bench --model llama-3-70b --tp 1 \
          --only lm_head --json gpurun_out/lm70tp1_rows.json || exit $? ;;
    bench20)
      # the driver's own command (20 timed waves after 5 warm-up waves)
      run bench20 900 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $? ;;
    pc_ab)
      # same box, alternating: prefix cache on / off (LMX_PREFIX_CACHE), 12 waves each
      for i in 1 2; do
        LMX_PREFIX_CACHE=1 run pc_ab_on_$i 600 python bench.py --steps 12 --warmup 2 || exit $?
        LMX_PREFIX_CACHE=0 run pc_ab_off_$i 600 python bench.py --steps 12 --warmup 2 || exit $?
      done ;;
    alloc_ab)
      # same box, alternating: KV pages from the min-heap (this tree) / the old LIFO stack
      # (ab/lifo, a copy of the tree with the old block manager), 12 waves each
      for i in 1 2; do
        run alloc_ab_heap_$i 600 python bench.py --steps 12 --warmup 2 || exit $?
        (cd ab/lifo && mkdir -p gpurun_out && run alloc_ab_lifo_$i 600 python bench.py --steps 12 --warmup 2) || exit $?
        cp ab/lifo/gpurun_out/alloc_ab_lifo_$i.log gpurun_out/ || exit $?
      done ;;
    overlap)
      # decode attention under the decode GEMMs: serial vs two streams (tools/overlap_probe.py)
      : > gpurun_out/overlap.log
      for w in gateup down qkv; do
        for m in 128 256; do
          timeout -k 10 120 python -u tools/overlap_probe.py --what $w --rows $m >> gpurun_out/overlap.log 2>&1 || exit $?
        done
      done
      cat gpurun_out/overlap.log ;;
    rs70tp1)
      # K14 (packed) on the 70B TP = 1 QKV (10240 x 8192, bf16 out) and O (8192 x 8192, fp32
      # partials for the slab norm) at the decode buckets, against the K11 entries served today
      : > gpurun_out/rs70tp1.log
      for M in ${RS_MS:-32 64 96 128}; do
        timeout -k 10 200 tools/labbin/rsgemm_lab 10240 8192 $M 0 \
            rs:42:1,rs:42:2,rs:42:4,rs:38:1,rs:38:2,rs:38:4,rs:46:2,dg:106:0,dg:117:0 >> gpurun_out/rs70tp1.log 2>&1 || exit $?
        timeout -k 10 200 tools/labbin/rsgemm_lab 10240 8192 $M 2 \
            rs:42:2,rs:42:4,rs:38:2,rs:38:4 >> gpurun_out/rs70tp1.log 2>&1 || exit $?
        timeout -k 10 200 tools/labbin/rsgemm_lab 8192 8192 $M 2 \
            rs:42:2,rs:42:4,rs:42:8,rs:38:2,rs:38:4,rs:38:8,dg:42:4,dg:63:4 >> gpurun_out/rs70tp1.log 2>&1 || exit $?
      done
      cat gpurun_out/rs70tp1.log ;;
    sample_ab)
      # K6 sampling at the headline shape: this tree vs ab/old (a copy with the previous kernel)
      : > gpurun_out/sample_ab.log
      for i in 1 2; do
        timeout -k 10 120 python -u tools/sample_probe.py >> gpurun_out/sample_ab.log 2>&1 || exit $?
        echo "--- ab/old" >> gpurun_out/sample_ab.log
        (cd ab/old && timeout -k 10 120 python -u tools/sample_probe.py) >> gpurun_out/sample_ab.log 2>&1 || exit $?
        echo "--- this tree" >> gpurun_out/sample_ab.log
      done
      timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "sample or tp8_lm_head" -x -q --timeout 120 \
          --timeout-method thread -p no:cacheprovider >> gpurun_out/sample_ab.log 2>&1 || exit $?
      cat gpurun_out/sample_ab.log ;;
    soak)
      # 10-minute closed-loop window at 256 streams with the shipped defaults: the KV pool
      # fills, the prefix cache evicts, and throughput / latency must hold
      run soak 900 python bench.py --load closed --duration ${SOAK_S:-600} --closed-warmup 10 || exit $? ;;
    attn70tp1)
      # Llama-3-70B TP = 1 decode attention: 128 rows x 8 kv heads x 8-query groups, the bench's
      # contexts (512-640): split-K partitions vs one per segment (1024 segments on 256 CUs)
      : > gpurun_out/attn70tp1.log
      for parts in 1 2 3; do
        for pt in 256 384; do
          timeout -k 10 120 python -u tools/decode_attn_probe.py --layout engine --rope --hq 64 \
              --hkv 8 --batch 128 --ctx-lo 512 --ctx-hi 640 --parts $parts --part-tokens $pt \
              --modes 0,10 --iters 40 >> gpurun_out/attn70tp1.log 2>&1 || exit $?
          [ $parts = 1 ] && break
        done
      done
      cat gpurun_out/attn70tp1.log ;;
    bench20_nopc)
      # the same without the prefix cache (KV pages recycled in place every wave)
      LMX_PREFIX_CACHE=0 run bench20_nopc 900 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $? ;;
    rs_small)
      # K14 on packed weights at every decode batch size vs the K11 entries the
      # table serves today: can one packed copy serve all of decode (one weight copy)?
      : > gpurun_out/rs_small.log
      for M in ${RS_MS:-16 32 64 96 128}; do
        timeout -k 10 200 tools/labbin/rsgemm_lab 28672 4096 $M 3 \
            rs:42:1,rs:42:2,rs:38:1,rs:38:2,dg:48:1,dg:17:1 >> gpurun_out/rs_small.log 2>&1 || exit $?
        timeout -k 10 200 tools/labbin/rsgemm_lab 4096 14336 $M 2 \
            rs:42:8,rs:42:16,rs:38:8,rs:38:16,dg:33:8,dg:53:4 >> gpurun_out/rs_small.log 2>&1 || exit $?
        timeout -k 10 200 tools/labbin/rsgemm_lab 4096 14336 $M 0 \
            rs:42:8,rs:42:16,rs:38:8,rs:38:16,dg:121:0,dg:97:0 >> gpurun_out/rs_small.log 2>&1 || exit $?
      done
      for M in ${RS70_MS:-16 64 128}; do
        timeout -k 10 200 tools/labbin/rsgemm_lab 57344 8192 $M 3 \
            rs:42:1,rs:42:2,rs:38:1,rs:38:2,dg:50:1 >> gpurun_out/rs_small.log 2>&1 || exit $?
        timeout -k 10 200 tools/labbin/rsgemm_lab 8192 28672 $M 2 \
            rs:42:8,rs:42:16,rs:38:8,rs:38:16,dg:38:8 >> gpurun_out/rs_small.log 2>&1 || exit $?
      done
      grep -E "shape|rs cfg|dg cfg|stream" gpurun_out/rs_small.log ;;
    attn_tests)
      run attn_tests 300 python -u -m pytest tests/test_kernels_gpu.py -k paged_decode -x -q \
          --timeout 120 --timeout-method thread -p no:cacheprovider || exit $? ;;
    attn_ring)
      # the rolling register ring (modes 9/10) against the default loop, headline and 70B shapes
      : > gpurun_out/attn_ring.log
      for args in "--layout engine --rope --modes ${ATTN_MODES:-0,10,9,0,10,9}" \
                  "--layout random --modes ${ATTN_MODES:-0,10,0,10}" \
                  "--layout engine --rope --hq 64 --batch 128 --ctx-lo 512 --ctx-hi 640 --modes ${ATTN_MODES:-0,10,0,10}"; do
        timeout -k 10 150 python -u tools/decode_attn_probe.py $args --iters 40 \
            >> gpurun_out/attn_ring.log 2>&1 || exit $?
      done
      cat gpurun_out/attn_ring.log ;;
    attn_layout)
      # kv-head-major cache emulation (each segment one contiguous page run) vs the
      # block-major cache, contiguous and random page placement, default loop form
      : > gpurun_out/attn_layout.log
      for args in "--layout contig" "--layout contig --head-major" "--layout random" \
                  "--layout random --head-major" "--layout engine" "--layout engine --head-major"; do
        timeout -k 10 120 python -u tools/decode_attn_probe.py $args --rope --modes 0,0,0 \
            --iters 30 >> gpurun_out/attn_layout.log 2>&1 || exit $?
      done
      cat gpurun_out/attn_layout.log ;;
    embed_bench)
      run embed_bench 300 python -u -m llm_mcp_amd.bench.embed_engine_bench || exit $? ;;
    embed_http)
      # config 2: /v1/embeddings (HTTP, sync path), 32 concurrent 16-doc requests of 1k-token docs
      run embed_http 600 python -u -m llm_mcp_amd.bench.serving_bench embed --requests 1024 || exit $? ;;
    rope_probe)
      run rope_probe 120 python -u tools/rope_probe.py || exit $? ;;
    config5a)
      # config 5 steady state: the same mixed load with NO fault, 3 fresh runs (the spread
      # is the run-to-run noise of the capacity itself)
      run config5a 1100 python -u -m llm_mcp_amd.bench.serving_bench mixed --gpus 0 \
          --replicas-per-gpu 2 --runs 3 --jobs 4096 --concurrency 256 --sync-every 4 \
          --max-tokens 64 --chars 512 || exit $? ;;
    c5ab)
      # config 5 steady state, shipped default vs no mixed-step cap, 2048 jobs each, alternating
      for i in 1 2; do
        run c5ab_default_$i 400 python -u -m llm_mcp_amd.bench.serving_bench mixed --gpus 0 \
            --replicas-per-gpu 2 --jobs 2048 --concurrency 256 --sync-every 4 --max-tokens 64 \
            --chars 512 || exit $?
        LMX_MIXED_PREFILL_TOKENS=0 run c5ab_nocap_$i 400 python -u -m llm_mcp_amd.bench.serving_bench \
            mixed --gpus 0 --replicas-per-gpu 2 --jobs 2048 --concurrency 256 --sync-every 4 \
            --max-tokens 64 --chars 512 || exit $?
      done ;;
    c5_budget)
      # config 5 steady state (2048 jobs): the shared-GPU prefill budget (8192) vs 16384 / 4096,
      # alternating, twice
      for i in 1 2; do
        for b in 8192 16384 4096; do
          LMX_MAX_BATCHED_TOKENS=$b run c5b_${b}_$i 400 python -u -m llm_mcp_amd.bench.serving_bench \
              mixed --gpus 0 --replicas-per-gpu 2 --jobs 2048 --concurrency 256 --sync-every 4 \
              --max-tokens 64 --chars 512 || exit $?
        done
      done ;;
    prof_c5)
      # config 5 steady state under a kernel trace: GPU busy vs wall per process
      rm -rf gpurun_out/prof_c5
      LMX_STOP_GRACE_S=90 run prof_c5 600 rocprofv3 --kernel-trace -d gpurun_out/prof_c5 -o %pid% -- python3 -u -m \
          llm_mcp_amd.bench.serving_bench mixed --gpus 0 --replicas-per-gpu 2 --jobs 2048 \
          --concurrency 256 --sync-every 4 --max-tokens 64 --chars 512 || exit $?
      # the worker processes finish writing their databases after the bench returns
      for i in $(seq 60); do
        ls gpurun_out/prof_c5/*.db-journal > /dev/null 2>&1 || break
        sleep 2
      done
      find gpurun_out/prof_c5 -name "*.db*" -printf "%s %p\n" || true
      python tools/prof_busy.py gpurun_out/prof_c5 > gpurun_out/prof_c5_busy.md 2>&1 || true
      find gpurun_out/prof_c5 -name "*.db" -delete 2>/dev/null || true ;;
    config5rec)
      # config 5 fault recovery: the faulty worker fails once at its 300th engine step;
      # the bench records the fault -> breaker -> restart -> first-job timeline
      run config5rec 900 python -u -m llm_mcp_amd.bench.serving_bench mixed --gpus 0 \
          --replicas-per-gpu 2 --fault gpu_error@300 --fault-device gpu0.r1 --fault-lives 1 \
          --jobs 4096 --concurrency 256 --sync-every 4 --max-tokens 64 --chars 512 \
          --await-recovery 150 || exit $? ;;
    budget_ab)
      # the wave's prefill step budget: 24576 vs BUDGETS (median request done after
      # 2 full steps from ~33.1k), same box, alternating
      for i in 1 2; do
        for b in 24576 ${BUDGETS:-33280 36864}; do
          run budget_${b}_$i 400 python bench.py --steps 4 --warmup 1 --max-batched-tokens $b \
              || exit $?
        done
      done ;;
    embed_batch)
      # the nomic engine at 32k / 64k tokens per batch
      : > gpurun_out/embed_batch.log
      for bt in 32768 65536; do
        timeout -k 10 200 python -u -m llm_mcp_amd.bench.embed_engine_bench --batch-tokens $bt \
            >> gpurun_out/embed_batch.log 2>&1 || exit $?
      done
      # q rotated inside the attention kernel (the rope/cache kernel skips q's write-back)
      LMX_FUSED_ENCODER_ROPE=1 timeout -k 10 200 python -u -m llm_mcp_amd.bench.embed_engine_bench \
          --batch-tokens 65536 >> gpurun_out/embed_batch.log 2>&1 || exit $?
      grep emb_per_s gpurun_out/embed_batch.log ;;
    budget_trace)
      # one run per budget with the engine's step trace (bench.py logs each wave's steps)
      for b in ${BUDGETS:-33280 36864 65664}; do
        LMX_STEP_TRACE=1 run budget_trace_$b 400 python bench.py --steps 3 --warmup 1 \
            --max-batched-tokens $b || exit $?
      done ;;
    embed_rope_ab)
      # nomic at 64k tokens per batch: q rotated in the rope/cache kernel vs inside attention,
      # alternating, 3 pairs
      : > gpurun_out/embed_rope_ab.log
      for i in 1 2 3; do
        for f in 0 1; do
          echo "fused_rope=$f run $i" >> gpurun_out/embed_rope_ab.log
          LMX_FUSED_ENCODER_ROPE=$f timeout -k 10 200 python -u -m llm_mcp_amd.bench.embed_engine_bench \
              --batch-tokens 65536 --docs 2048 >> gpurun_out/embed_rope_ab.log 2>&1 || exit $?
        done
      done
      grep -E "fused_rope|emb_per_s" gpurun_out/embed_rope_ab.log ;;
    ar_norm)
      # fused all-reduce + norm at world 8 on one GPU (local cost), cs 1/2/4, then the peer
      # all-reduce GPU tests (correctness at world 2/4/8, both grids)
      run ar_norm_probe 300 python -u tools/ar_norm_probe.py --worlds 2,8 || exit $?
      cat gpurun_out/ar_norm_probe.log
      run ar_tests 400 python -u -m pytest tests/test_00_peer_ar_gpu.py -x -v --timeout 300 \
          --timeout-method thread -p no:cacheprovider || exit $? ;;
    dgemm_fam)
      # decode GEMM sweep (K11 tiles / splits / stream-K vs the library) for the other chat
      # families' shapes; rows kept, the table is rebuilt on the CPU side (new shapes only)
      for m in ${DG_MODELS:-qwen3-8b qwen2.5-7b}; do
        run dg_$m 1000 python -u -m llm_mcp_amd.bench.dgemm_bench --model $m --tp ${DG_TP:-1} \
            --json gpurun_out/dg_$m.json || exit $?
      done ;;
    split_tests)
      run split_tests 600 python -u -m pytest tests/test_engine_gpu.py tests/test_norm_fold_gpu.py \
          -k "rows_split or row_pieces or norm" -x -v --timeout 300 --timeout-method thread \
          -p no:cacheprovider || exit $? ;;
    fam_tests)
      run fam_tests 600 python -u -m pytest tests/test_engine_gpu.py -k "family or llama3_8b" -x -v \
          --timeout 300 --timeout-method thread -p no:cacheprovider || exit $? ;;
    copies_ab)
      # Llama-3-8B one packed copy of the MLP weights (LMX_RS_SINGLE=1: K14 at every batch)
      # vs the default for its size (auto: two copies, K11 up to 128 rows, K13 prefill on
      # the packed copy), alternating, twice
      for i in 1 2; do
        for c in ${COPIES_C:-64 256}; do
          LMX_RS_SINGLE=1 run cp1_${c}_$i 400 python bench.py --steps 3 --warmup 1 \
              --concurrency $c || exit $?
          run cp2_${c}_$i 400 python bench.py --steps 3 --warmup 1 --concurrency $c || exit $?
        done
      done ;;
    families)
      # the other chat model families at the headline load (256 streams x 512-token prompts,
      # 256 out), one wave-bench each, and the other embedding encoders
      for m in ${FAMILIES:-qwen3-8b qwen2.5-7b llama-3.2-3b llama-3.2-1b qwen3-32b}; do
        run fam_$m 600 python bench.py --model $m --steps 2 --warmup 1 || exit $?
      done
      for m in mxbai-embed-large bge-base-en-v1.5; do
        timeout -k 10 300 python -u -m llm_mcp_amd.bench.embed_engine_bench --model $m \
            --doc-len 512 > gpurun_out/fam_$m.log 2>&1 || exit $?
        tail -1 gpurun_out/fam_$m.log
      done ;;
    race_tests)
      run race_tests 400 python -u -m pytest tests/test_00_peer_ar_gpu.py tests/test_kernels_gpu.py \
          -k "race or sharded or sample" -x -v --timeout 300 --timeout-method thread \
          -p no:cacheprovider || exit $? ;;
    prof_embed)
      # nomic engine at 1k-token docs under a kernel trace: the kernel-class split
      rm -rf gpurun_out/prof_embed
      run prof_embed 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_embed -o run \
          -- python3 -m llm_mcp_amd.bench.embed_engine_bench || exit $?
      python tools/prof_summary.py gpurun_out/prof_embed/run_results.db --top 30 \
          > gpurun_out/prof_embed_summary.md 2>&1 || true
      find gpurun_out/prof_embed -name "*.db" -delete 2>/dev/null || true ;;
    closed_cap)
      # closed loop at 256 streams with a mixed-step cap of CAP tokens (burst-aware:
      # LMX_MIXED_LATER_STEPS) -- the per-token gap p99 against the uncapped default
      LMX_MIXED_PREFILL_TOKENS=${CAP:-2048} run closed_cap_${CAP:-2048} 600 python bench.py \
          --load closed --duration ${CLOSED_S:-40} --closed-warmup 10 || exit $? ;;
    closed_nocap0)
      LMX_MIXED_PREFILL_TOKENS=0 run closed_nocap0 600 python bench.py --load closed \
          --duration ${CLOSED_S:-40} --closed-warmup 10 || exit $? ;;
    bench_cap)
      LMX_MIXED_PREFILL_TOKENS=${CAP:-2048} run bench_cap_${CAP:-2048} 600 python bench.py \
          --steps 6 --warmup 1 || exit $? ;;
    bench6)
      run bench6 600 python bench.py --steps 6 --warmup 1 || exit $? ;;
    smoke)
      run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    *)
      echo "unknown step $step" >&2; exit 2 ;;
  esac
done
