"""Find reads / writes of in-flight load destinations in a hipcc -S listing.

Kernels with inline-asm load rings (rsgemm.hip K14 / K14W) count vmcnt by
hand: the compiler believes an asm load's output is ready at once, so it may
copy, move or reuse that register before the data lands -- silent
corruption (or, when the register later serves as an address, a memory
fault).  This walks each kernel's instructions in listing order with a FIFO
of outstanding vector-memory ops (vmcnt retires in order): ``s_waitcnt
vmcnt(N)`` retires the oldest down to N; any other instruction that names a
register an outstanding load writes is reported.

    python -m llm_mcp_amd.utils.vmem_audit file.s [kernel-regex]

build.py runs it on every inline-asm ring source (ASM_RING_KERNELS) and fails
the build on a finding.
"""
import re
import sys

LOAD = re.compile(r"^\s*(global_load|buffer_load|flat_load|scratch_load)(?!_lds)\w*\s+(\S+?),")
VMEM = re.compile(r"^\s*(global_|buffer_|flat_|scratch_)\w+")
WAIT = re.compile(r"s_waitcnt\s.*vmcnt\((\d+)\)")
REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        kind = m.group(1)
        if m.group(4) is not None:
            out.add((kind, int(m.group(4))))
        else:
            out.update((kind, r) for r in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def audit(body: str):
    q = []            # outstanding VMEM ops in issue order: set of dest regs (empty: no dest)
    issues = []
    for ln, raw in enumerate(body.split("\n")):
        line = raw.split(";")[0].strip()
        if not line or line.endswith(":") or line.startswith("."):
            continue
        w = WAIT.search(line)
        if w:
            n = int(w.group(1))
            while len(q) > n:
                q.pop(0)
            continue
        pending = set().union(*q) if q else set()
        m = LOAD.match(line)
        if m:
            dst = regs(m.group(2))
            src = regs(line[m.end():])
            bad = (dst | src) & pending
            if bad:
                issues.append((ln, line, sorted(bad)[:4]))
            q.append(dst)
            continue
        used = regs(line)
        bad = used & pending
        if bad:
            issues.append((ln, line, sorted(bad)[:4]))
        if VMEM.match(line):
            q.append(set())          # stores / LDS-DMA: count, write no register
    return issues


def audit_listing(text: str, pattern: str = "") -> dict:
    """{kernel: hazards} for the kernels of a -S listing whose name matches
    the regex ``pattern``."""
    out = {}
    for m in re.finditer(r"\n([_A-Za-z]\w+):[^\n]*\n(.*?)\.Lfunc_end", text, re.S):
        name, body = m.group(1), m.group(2)
        if pattern and not re.search(pattern, name):
            continue
        out[name] = audit(body)
    return out


def main():
    s = open(sys.argv[1]).read()
    res = audit_listing(s, sys.argv[2] if len(sys.argv) > 2 else "")
    for name, iss in res.items():
        print(f"{name[:90]}: {len(iss)} hazard(s)")
        for ln, line, r in iss[:8]:
            print(f"    line {ln}: {line}   {r}")
    sys.exit(1 if any(res.values()) else 0)

if __name__ == "__main__":
    main()
