"""The mixed-step prefill cap (native Scheduler.set_mixed_prefill_cap): a
burst's rows never cap each other (a wave keeps the full token budget), but
streams already running when LATER requests arrive get bounded steps."""
import numpy as np

from llm_mcp_amd import native


def _run(later, extra_after=6):
    rt = native.runtime()
    s = rt.Scheduler(1000, 32, 64, 256, 4096, True)
    s.set_mixed_prefill_cap(64, 2, later)
    for i in range(8):           # one burst: 8 distinct 100-token prompts
        s.add(i, list(range(i * 1000, i * 1000 + 100)), 50, [], True, 0)

    def step():
        p = s.schedule(16)
        s.update(np.full(len(p["sample_seq"]), 5, dtype=np.int32))
        return int(p["num_decode"]), int(p["num_prefill_tokens"])
    burst = [step() for _ in range(extra_after)]
    for i in range(8, 12):       # later arrivals while the burst's rows decode
        s.add(i, list(range(i * 1000, i * 1000 + 200)), 10, [], True, 0)
    later_steps = [step() for _ in range(4)]
    return burst, later_steps


def test_burst_keeps_full_budget_later_arrivals_are_capped():
    burst, late = _run(later=2)
    # the burst: full 256-token steps while prompts remain, decodes riding along
    assert burst[1] == (2, 254) and burst[2] == (5, 251)
    # later arrivals: every step carries the 8 running streams + <= 64 prompt tokens
    assert all(nd == 8 and pf == 64 for nd, pf in late), late


def test_later_steps_zero_caps_every_mixed_step():
    burst, late = _run(later=0)
    assert burst[1] == (2, 64)          # the burst's own rows trigger the cap
    assert all(pf <= 64 for _, pf in burst[1:] + late)
