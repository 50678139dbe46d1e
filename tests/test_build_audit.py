"""The build's code-object audit of the inline-asm ring kernels:
a K14 weight-ring or decode-attention K/V-ring instantiation that spills or uses
scratch could move an inline-asm load destination before its data lands, so
build.py compiles those sources with -Rpass-analysis=kernel-resource-usage and
fails on any spill; this test re-checks the table the last build recorded."""
import json

from llm_mcp_amd import build


REMARKS = """\
rsgemm.hip:165:1: remark: Function Name: _ZN3lmx13rsgemm_kernelILi3ELi4ELi3ELi1ELi0ELi128EEEvPtPKtS3_PfPjiiillli [-Rpass-analysis=kernel-resource-usage]
rsgemm.hip:165:1: remark:     VGPRs: 228 [-Rpass-analysis=kernel-resource-usage]
rsgemm.hip:165:1: remark:     ScratchSize [bytes/lane]: 0 [-Rpass-analysis=kernel-resource-usage]
rsgemm.hip:165:1: remark:     SGPRs Spill: 0 [-Rpass-analysis=kernel-resource-usage]
rsgemm.hip:165:1: remark:     VGPRs Spill: 0 [-Rpass-analysis=kernel-resource-usage]
rsgemm.hip:165:1: remark: Function Name: _ZN3lmx13rsgemm_kernelILi3ELi6ELi4ELi0ELi0ELi256EEEvPtPKtS3_PfPjiiillli [-Rpass-analysis=kernel-resource-usage]
rsgemm.hip:165:1: remark:     VGPRs: 256 [-Rpass-analysis=kernel-resource-usage]
rsgemm.hip:165:1: remark:     ScratchSize [bytes/lane]: 20 [-Rpass-analysis=kernel-resource-usage]
rsgemm.hip:165:1: remark:     SGPRs Spill: 0 [-Rpass-analysis=kernel-resource-usage]
rsgemm.hip:165:1: remark:     VGPRs Spill: 8 [-Rpass-analysis=kernel-resource-usage]
"""


def test_parse_and_audit_flags_spills():
    u = build.parse_resource_usage(REMARKS)
    assert len(u) == 2
    k = "_ZN3lmx13rsgemm_kernelILi3ELi6ELi4ELi0ELi0ELi256EEEvPtPKtS3_PfPjiiillli"
    assert u[k] == {"vgprs": 256, "scratch": 20, "sgpr_spill": 0, "vgpr_spill": 8}
    bad = build.audit_asm_rings({"rsgemm.hip": u, "attention.hip": {}})
    assert any("Li256E" in b and "spills" in b for b in bad)
    assert any("attention.hip" in b for b in bad)          # no ring kernel reported at all


def test_built_ring_kernels_have_no_spills():
    build.build_kernels()                  # no-op when up to date; raises on a spill
    usage = json.loads((build.BUILD / "kernels" / "resource_usage.json").read_text())
    assert build.audit_asm_rings(usage) == []
    n = sum(1 for src in build.ASM_RING_KERNELS for k in usage[src]
            if "rsgemm_kernel" in k or "ELi9E" in k)
    assert n >= 20
