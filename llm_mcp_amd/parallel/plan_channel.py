"""Leader -> follower step-plan channel for a tensor-parallel group (X4).

Every rank of a TP group runs the same forward on its weight shard, so every
rank needs the leader's scheduling decision for the step (token ids,
positions, KV slots, block tables, prefill tiles, decode-graph bucket).  The
group always lives on one node (TP over xGMI), so the plan travels through a
shared-memory mailbox instead of a device collective: the followers never
have to synchronise with their GPU to learn the step's shapes, and the
leader pays one memcpy per step.

Layout of the mailbox file (``/dev/shm``):
    [0:8)    seq     (u64) -- bumped by the leader after the payload is written
    [8:16)   nbytes  (u64)
    [16:24)  beat    (u64) -- leader heartbeat, wall-clock ns, rewritten every
                              ``BEAT_S`` by a leader thread (also while idle)
    [24:32)  pid     (u64) -- leader process id
    [64 + 8r) ack[r] (u64) -- last seq follower r has copied out
    [4096:)  payload (msgpack)
The leader waits until every follower acked the previous message before
overwriting the payload (single slot, so at most one plan in flight -- the
followers' GPU work still runs asynchronously behind it).
"""
from __future__ import annotations

import os
import tempfile
import threading
import time

import msgpack
import numpy as np

_HDR = 4096
PLAN_KEYS = ("input_ids", "positions", "slots", "context_lens", "cu_q", "block_tables",
             "prefill_tiles", "sample_rows", "seq_ids", "temp", "topk", "topp", "seeds", "offs")
PLAN_INTS = ("num_decode", "max_blocks", "num_tokens", "num_prefill_tokens", "max_context")
# present when the followers sample too (lookahead TP): pending-input rows and
# the penalty windows of the step
PLAN_OPT_KEYS = ("input_src", "pen_window", "pen_ngen", "pen_params")
PLAN_OPT_INTS = ("num_pending_inputs", "any_penalty")
BEAT_S = 1.0


class LeaderLost(RuntimeError):
    """The TP leader died or stopped beating: the follower must exit so its
    launcher can tear the group down (and the supervisor start a new one)."""


def _pid_alive(pid: int) -> bool:
    """True while ``pid`` runs (a zombie -- exited, not yet reaped by its
    parent -- counts as dead)."""
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[0] != "Z"
    except (OSError, IndexError):
        return True


def leader_timeout_s() -> float:
    return float(os.environ.get("LMX_TP_LEADER_TIMEOUT_S", "30"))


def encode_plan(plan: dict, bucket: int | None, full: bool = False) -> dict:
    """``full``: also the keys the followers need to sample (lookahead TP)."""
    msg = {"cmd": "step", "bucket": bucket or 0}
    keys = PLAN_KEYS + (PLAN_OPT_KEYS if full else ())
    for k in keys:
        if k not in plan:
            continue
        a = np.ascontiguousarray(plan[k]).reshape(-1)
        msg[k] = (a.dtype.str, a.shape[0], a.tobytes())
    for k in PLAN_INTS + (PLAN_OPT_INTS if full else ()):
        if k in plan:
            msg[k] = int(plan[k])
    return msg


def decode_plan(msg: dict) -> tuple[dict, int | None]:
    plan = {}
    for k in PLAN_KEYS + PLAN_OPT_KEYS:
        if k not in msg:
            continue
        dt, n, b = msg[k]
        plan[k] = np.frombuffer(b, dtype=np.dtype(dt), count=n)
    for k in PLAN_INTS + PLAN_OPT_INTS:
        if k in msg:
            plan[k] = msg[k]
    plan["sample_seq"] = np.arange(len(plan["sample_rows"]), dtype=np.int32)
    return plan, (msg["bucket"] or None)


def mailbox_path(tag: str) -> str:
    base = "/dev/shm" if os.path.isdir("/dev/shm") else tempfile.gettempdir()
    return os.path.join(base, f"lmx-tp-{tag}")


class PlanChannel:
    def __init__(self, path: str, rank: int, size: int, capacity: int = 64 << 20,
                 create: bool | None = None):
        self.path, self.rank, self.size = path, rank, size
        create = (rank == 0) if create is None else create
        total = _HDR + capacity
        if create:
            with open(path, "wb") as f:
                f.truncate(total)
        else:
            deadline = time.time() + 120
            while not os.path.exists(path) or os.path.getsize(path) < total:
                if time.time() > deadline:
                    raise TimeoutError(f"plan mailbox {path} never appeared")
                time.sleep(0.01)
        self.mm = np.memmap(path, dtype=np.uint8, mode="r+", shape=(total,))
        self.ctl = self.mm[:_HDR].view(np.uint64)
        self.capacity = capacity
        self.owner = create
        # a follower may attach after the leader already published: resume
        # from its own ack slot (0 on a fresh mailbox), not from the head
        self._seq = int(self.ctl[0]) if create else int(self.ctl[8 + rank])
        self._beat_stop = threading.Event()
        self._beat_thread = None
        if create:
            self.ctl[3] = os.getpid()
            self.ctl[2] = time.time_ns()
            self._beat_thread = threading.Thread(target=self._beat, daemon=True, name="tp-beat")
            self._beat_thread.start()

    def _beat(self):
        while not self._beat_stop.wait(BEAT_S):
            try:
                self.ctl[2] = time.time_ns()
            except (TypeError, ValueError, AttributeError):
                return   # mailbox closed

    def leader_alive(self, timeout_s: float | None = None) -> tuple[bool, str]:
        """Follower-side liveness of the leader: its pid exists and its
        heartbeat is younger than ``timeout_s``."""
        pid = int(self.ctl[3])
        if pid and not _pid_alive(pid):
            return False, f"leader pid {pid} is gone"
        age = (time.time_ns() - int(self.ctl[2])) / 1e9
        lim = leader_timeout_s() if timeout_s is None else timeout_s
        if int(self.ctl[2]) and age > lim:
            return False, f"leader heartbeat is {age:.1f}s old (limit {lim:.0f}s)"
        return True, ""

    # ---------------------------------------------------------- leader ----
    def publish(self, msg: dict, timeout: float = 300.0) -> None:
        data = msgpack.packb(msg, use_bin_type=True)
        if len(data) > self.capacity:
            raise RuntimeError("plan exceeds mailbox capacity")
        deadline = time.monotonic() + timeout
        spins = 0
        while any(int(self.ctl[8 + r]) < self._seq for r in range(1, self.size)):
            spins += 1
            if spins > 2000:
                time.sleep(0.0002)
                if time.monotonic() > deadline:
                    raise TimeoutError("TP follower stopped acknowledging plans")
        self.mm[_HDR:_HDR + len(data)] = np.frombuffer(data, dtype=np.uint8)
        self.ctl[1] = len(data)
        self._seq += 1
        self.ctl[0] = self._seq   # x86-64 stores are not reordered after the payload

    # -------------------------------------------------------- follower ----
    def receive(self, idle_sleep: float = 0.0005, timeout_s: float | None = None) -> dict:
        """Next plan.  Raises ``LeaderLost`` when the leader process is gone or
        its heartbeat is older than ``timeout_s`` (LMX_TP_LEADER_TIMEOUT_S),
        so a crashed leader never strands the followers' GPUs."""
        spins = 0
        next_check = 0.0
        while int(self.ctl[0]) == self._seq:
            spins += 1
            if spins > 5000:
                time.sleep(idle_sleep)
                now = time.monotonic()
                if now >= next_check:
                    next_check = now + 0.5
                    ok, why = self.leader_alive(timeout_s)
                    if not ok:
                        raise LeaderLost(why)
        self._seq = int(self.ctl[0])
        n = int(self.ctl[1])
        data = bytes(self.mm[_HDR:_HDR + n])
        self.ctl[8 + self.rank] = self._seq
        return msgpack.unpackb(data, raw=False)

    def close(self):
        self._beat_stop.set()
        if self._beat_thread is not None:
            self._beat_thread.join(timeout=5)
        del self.ctl
        self.mm._mmap.close()
        if self.owner:
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass
