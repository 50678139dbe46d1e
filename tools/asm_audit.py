"""Audit the steady-state loop of kernels in a hipcc -S listing: register
count, MFMA count, waits and moves in the longest backward-branch loop.
    python tools/asm_audit.py file.s [name-substring]"""
import re
import sys
from collections import Counter


def main():
    s = open(sys.argv[1]).read()
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    for m in re.finditer(r'\n([_A-Za-z]\w+):[^\n]*\n(.*?)\.Lfunc_end', s, re.S):
        name, body = m.group(1), m.group(2)
        if sub not in name or "kernel" not in name:
            continue
        meta = s[m.end():m.end() + 20000]
        vg = re.search(r'NumVgprs:\s*(\d+)', meta)
        lines = body.split('\n')
        labels = {l.split(':')[0]: i for i, l in enumerate(lines) if re.match(r'^\.LBB\w+:', l)}
        best = None
        for i, l in enumerate(lines):
            mm = re.search(r's_cbranch_\w+\s+(\.LBB\w+)', l)
            if mm and mm.group(1) in labels and labels[mm.group(1)] < i:
                st = labels[mm.group(1)]
                if best is None or i - st > best[1] - best[0]:
                    best = (st, i)
        if best is None:
            print(name, "no loop")
            continue
        xs = [x.strip() for x in lines[best[0]:best[1] + 1]
              if x.strip() and not x.strip().startswith(';')]
        ops = Counter(x.split()[0] for x in xs)
        waits = Counter(x for x in xs if x.startswith('s_waitcnt'))
        print(f"{name[:70]} vgpr {vg.group(1) if vg else '?'} loop {len(xs)} "
              f"mfma {sum(v for k, v in ops.items() if 'mfma' in k)} "
              f"ds_read {sum(v for k, v in ops.items() if k.startswith('ds_read'))} "
              f"v_mov {ops.get('v_mov_b32', 0)} accvgpr {sum(v for k, v in ops.items() if 'accvgpr' in k)}")
        print("   waits", waits.most_common(8))


if __name__ == "__main__":
    main()
