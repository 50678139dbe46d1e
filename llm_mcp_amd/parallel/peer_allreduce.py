"""Peer-memory all-reduce for decode-sized TP messages (X1/X2 over xGMI).

Wraps csrc/kernels/allreduce.hip.  Every rank allocates one uncached device
region, exports it with ``hipIpcGetMemHandle``, the handles are exchanged
over the TP process group (``all_gather_object``), and every rank maps all
peer regions with ``hipIpcOpenMemHandle``.  A call is then ONE kernel launch
with no host involvement, so it is captured into the decode hipGraphs like
any other op.  RCCL stays the path for messages larger than a slot (prefill)
and for anything the kernel does not cover (non-bf16, unaligned).

Selection: one-shot (every rank reads all W inputs) up to ``oneshot_max``
bytes, two-shot (reduce-scatter + all-gather through peer memory) above.
The crossover and the slot size are env-tunable (LMX_AR_ONESHOT_MAX,
LMX_AR_SLOT_MB); the defaults come from the per-link arithmetic in
SURVEY §2.3 (one-shot moves (W-1) x S per rank, two-shot 2 (W-1)/W x S, both
over all W-1 links at once, vs a ring's 2 (W-1)/W x S over one link).

A self-test against the process group's own all-reduce runs at setup; a
mismatch, a bounded-wait timeout (error word set by the kernel) or any HIP
error disables the path and the group falls back to RCCL.
"""
from __future__ import annotations

import logging
import os

import torch
import torch.distributed as dist

from ..native import kernels as native

log = logging.getLogger("lmx.tp")

MAX_WORLD, MAX_BLOCKS = 8, 64
NORM_BLOCKS = 128       # fused norm grid cap (allreduce.hip AR_MAX_BLOCKS)


class PeerAllReduce:
    def __init__(self, group, rank: int, world: int, device: torch.device,
                 slot_bytes: int | None = None, oneshot_max: int | None = None,
                 spin_max: int | None = None):
        if not 2 <= world <= MAX_WORLD:
            raise ValueError(f"peer all-reduce supports 2..{MAX_WORLD} ranks, got {world}")
        self.group, self.rank, self.world, self.device = group, rank, world, device
        self.slot = int(slot_bytes or float(os.environ.get("LMX_AR_SLOT_MB", "16")) * (1 << 20))
        self.slot -= self.slot % (16 * world)
        self.oneshot_max = int(oneshot_max or os.environ.get("LMX_AR_ONESHOT_MAX", 512 << 10))
        # bounded waits: ~2^25 polls of s_sleep(1) is a few seconds, longer than
        # any scheduling skew between healthy ranks (the old 2^22 bound, ~0.2 s,
        # could expire while a follower process was descheduled); a timed-out
        # kernel sets the error word, which check_async / failed() surface
        self.spin_max = int(spin_max or os.environ.get("LMX_AR_SPIN", 1 << 25))
        # column chunks per row of the fused all-reduce + norm (1: one block per row)
        self.norm_max_cs = max(1, int(os.environ.get("LMX_AR_NORM_CS", "2")))
        self._err_h = None
        self.k = native()
        self.own, self.peers, self.calls = None, [], 0
        # every rank reaches the handle exchange, even when its own
        # allocation failed, so a local failure cannot strand the others
        mine, why = b"", ""
        try:
            self.own = self.k.ar_alloc(self.slot)
            mine = self.k.ar_ipc_handle(self.own)
        except RuntimeError as ex:
            why = str(ex)
        # ranks sharing this rank's GPU (a one-GPU rehearsal puts them all on
        # one card): their fused-norm grids must be co-resident together, so the
        # per-rank grid shrinks with it (norm_plan)
        import socket
        key = (socket.gethostname(), os.environ.get("HIP_VISIBLE_DEVICES", ""),
               os.environ.get("ROCR_VISIBLE_DEVICES", ""), device.index)
        handles = [None] * world
        dist.all_gather_object(handles, (mine, key), group=group)
        keys = [h[1] for h in handles]
        handles = [h[0] for h in handles]
        self.co_resident = max(keys.count(k) for k in keys)
        if not all(handles):
            self.close()
            raise RuntimeError(f"peer all-reduce: a rank could not export its region ({why})")
        try:
            for q in range(world):
                self.peers.append(self.own if q == rank else self.k.ar_ipc_open(handles[q]))
        except Exception:
            self.close()
            raise

    # ------------------------------------------------------------------ api --
    def supports(self, t: torch.Tensor) -> bool:
        n = t.numel() * t.element_size()
        return (t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous()
                and 0 < n <= self.slot and n % 16 == 0 and t.data_ptr() % 16 == 0)

    def plan(self, nbytes: int) -> tuple[int, int]:
        """(two_shot, blocks) for a message of nbytes."""
        n8 = nbytes // 16
        two = int(nbytes > self.oneshot_max and n8 % self.world == 0)
        per_rank = nbytes // self.world if two else nbytes
        blocks = max(1, min(MAX_BLOCKS, per_rank // (16 << 10)))
        return two, blocks

    def __call__(self, t: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """Sum of ``t`` over the group, in place unless ``out`` is given."""
        out = t if out is None else out
        n = t.numel() * t.element_size()
        two, blocks = self.plan(n)
        self.k.allreduce(out.data_ptr(), t.data_ptr(), n, self.rank, self.world, self.peers,
                         self.slot, two, blocks, self.spin_max,
                         torch.cuda.current_stream(t.device).cuda_stream)
        self.calls += 1
        return out

    def norm_supports(self, t: torch.Tensor, residual: torch.Tensor) -> bool:
        """``t`` [T, cols] can take the fused all-reduce + residual + RMSNorm."""
        return (self.supports(t) and t.dim() == 2 and t.shape[1] % 8 == 0
                and t.shape[1] <= 16384 and self.world in (2, 4, 8)
                and t.numel() * 2 + t.shape[0] * 16 <= self.slot
                and residual.is_contiguous() and residual.shape == t.shape
                and residual.dtype == torch.bfloat16 and residual.data_ptr() % 16 == 0)

    def norm_plan(self, T: int, cols: int, two: int) -> tuple[int, int]:
        """(row groups, column chunks) of the fused norm's grid: a row's 16-B
        columns split over up to NORM_MAX_CS blocks (>= 256 per block) while
        the grid stays within NORM_BLOCKS, so the few rows a rank owns at
        decode (T / W at two-shot) still spread over many CUs."""
        rows = -(-T // self.world) if two else T
        # every block of every rank on a card must be resident at once (they
        # wait on each other): 128 per rank alone on its GPU, 32 per rank when
        # a rehearsal shares one GPU between up to 8 ranks
        cap = max(32, min(NORM_BLOCKS, 256 // max(1, getattr(self, "co_resident", 1))))
        d8, cs = cols // 8, 1
        while (cs * 2 <= self.norm_max_cs and d8 % (cs * 2) == 0 and d8 // (cs * 2) >= 256
               and min(rows, cap // (cs * 2)) * cs * 2 > min(rows, cap // cs) * cs):
            cs *= 2
        return max(1, min(rows, cap // cs)), cs

    def all_reduce_norm(self, t: torch.Tensor, w: torch.Tensor, eps: float,
                        residual: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """One kernel for a TP sub-layer's tail: residual += sum over the group
        of ``t`` (bf16-rounded like ``__call__``), returns rmsnorm(residual) * w
        -- the residual bitwise what the all-reduce followed by
        ``ops.rms_norm(..., residual=)`` gives, h up to the order of the row's
        sum of squares.  One-shot up to ``oneshot_max`` bytes, else
        row-sharded two-shot."""
        T, cols = t.shape
        if out is None:
            out = torch.empty_like(t)
        n = T * cols * 2
        two = int(n > self.oneshot_max and T >= self.world)
        groups, cs = self.norm_plan(T, cols, two)
        self.k.allreduce_norm(out.data_ptr(), residual.data_ptr(), t.data_ptr(), w.data_ptr(),
                              T, cols, float(eps), self.rank, self.world, self.peers, self.slot,
                              two, groups, cs, self.spin_max,
                              torch.cuda.current_stream(t.device).cuda_stream)
        self.calls += 1
        return out

    def gather_supports(self, t: torch.Tensor) -> bool:
        """``t`` can be all-gathered through the slots (bf16, 16-B rows)."""
        return self.supports(t)

    def all_gather(self, t: torch.Tensor, out: torch.Tensor | None,
                   to_all: bool = True) -> torch.Tensor | None:
        """Concatenation of every rank's ``t`` (flattened) in rank order:
        ``out`` [world * t.numel()] elements.  ``to_all`` False: only rank 0
        receives (``out`` may be None elsewhere); the others only publish."""
        n = t.numel() * t.element_size()
        if out is None:
            out = torch.empty(self.world * t.numel(), dtype=t.dtype, device=t.device) \
                if (to_all or self.rank == 0) else t
        blocks = max(1, min(MAX_BLOCKS, n // (16 << 10)))
        self.k.allreduce(out.data_ptr(), t.data_ptr(), n, self.rank, self.world, self.peers,
                         self.slot, 2 if to_all else 3, blocks, self.spin_max,
                         torch.cuda.current_stream(t.device).cuda_stream)
        self.calls += 1
        return out if (to_all or self.rank == 0) else None

    def check_async(self, stream) -> None:
        """Enqueue a copy of the error word into pinned host memory (after a
        step's collectives, no synchronisation); ``failed`` reads it."""
        if self.own is None:
            return
        if self._err_h is None:
            self._err_h = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self.k.ar_error_async(self.own, self._err_h.data_ptr(), stream.cuda_stream)

    def failed(self) -> bool:
        """A kernel of this rank gave up waiting for a peer (its result was
        wrong): as of the last copy ``check_async`` enqueued that has landed."""
        return self._err_h is not None and int(self._err_h[0]) != 0

    def error(self, clear: bool = False) -> int:
        """Non-zero when a kernel gave up waiting for a peer (synchronous)."""
        return self.k.ar_error(self.own, int(clear))

    def close(self) -> None:
        if self.own is None:
            return
        if self.peers:
            torch.cuda.synchronize(self.device)
        for q, p in enumerate(self.peers):
            if q != self.rank:
                try:
                    self.k.ar_ipc_close(p)
                except RuntimeError:
                    pass
        self.peers = []
        self.k.ar_free(self.own)
        self.own = None

    # ------------------------------------------------------------ self-test --
    def self_test(self, reference_all_reduce, sizes=(4096, 64 << 10, 1 << 20),
                  reference_all_gather=None) -> bool:
        """Compare against ``reference_all_reduce`` (the group's RCCL / gloo
        path) -- and the all-gather against ``reference_all_gather`` when
        given -- on seeded data; every rank must agree on the verdict."""
        ok = True
        g = torch.Generator(device="cpu").manual_seed(1234 + self.rank)
        for n in sizes:
            n = min(n, self.slot)
            x = (torch.randn(n // 2, generator=g) * (self.rank + 1)).to(
                torch.bfloat16).to(self.device)
            want = reference_all_reduce(x.clone()).float()
            try:
                got = self(x.clone()).float()
                torch.cuda.synchronize(self.device)
                err = (got - want).abs().max().item()
                timed_out = self.error(clear=True)
            except RuntimeError as ex:
                err, timed_out = float("inf"), str(ex)
            tol = 2e-2 * max(1.0, want.abs().max().item())
            if not (err <= tol) or timed_out:
                log.warning("peer all-reduce self-test failed at %d B (max err %.3g, %s)", n,
                            err, timed_out or "no timeout")
                ok = False
            if reference_all_gather is not None:
                want_g = reference_all_gather(x.clone())
                try:
                    got_g = self.all_gather(x.clone(), None)
                    torch.cuda.synchronize(self.device)
                    same = bool(torch.equal(got_g.view(-1), want_g.view(-1)))
                    timed_out = self.error(clear=True)
                except RuntimeError as ex:
                    same, timed_out = False, str(ex)
                if not same or timed_out:
                    log.warning("peer all-gather self-test failed at %d B (%s)", n,
                                timed_out or "mismatch")
                    ok = False
        return ok


_CPU_GROUPS: dict = {}


def _cpu_group(group):
    """A gloo twin of ``group`` for host-side control values."""
    if dist.get_backend(group) == "gloo":
        return group
    key = id(group)
    if key not in _CPU_GROUPS:
        _CPU_GROUPS[key] = dist.new_group(backend="gloo")
    return _CPU_GROUPS[key]


def _agree(ok: bool, tp) -> bool:
    flag = torch.tensor([int(ok)], dtype=torch.int32)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN,
                    group=getattr(tp, "cpu_group", None) or _cpu_group(tp.group))
    return bool(flag.item())


def setup(tp, device: torch.device) -> PeerAllReduce | None:
    """Enable the peer all-reduce on a TP context when possible (LMX_CUSTOM_AR=0
    disables it).  Collective: every rank of the group must call it."""
    if tp.size < 2 or device.type != "cuda" or os.environ.get("LMX_CUSTOM_AR", "1") == "0":
        return None
    ar, ok = None, True
    try:
        ar = PeerAllReduce(tp.group, tp.rank, tp.size, device)
    except Exception as ex:   # IPC unavailable (no peer access, old driver ...)
        log.warning("peer all-reduce unavailable: %s", ex)
        ok = False
    if not _agree(ok, tp):          # symmetric: everyone built it, or nobody uses it
        if ar is not None:
            ar.close()
        return None
    def ref_gather(x):
        saved, tp.peer = tp.peer, None
        try:
            return tp.all_gather_rows(x.view(1, -1)).view(-1)
        finally:
            tp.peer = saved
    if not _agree(ar.self_test(tp.all_reduce, reference_all_gather=ref_gather), tp):
        ar.close()
        return None
    tp.peer = ar
    log.info("peer all-reduce enabled: world %d, slot %d MB, one-shot <= %d KB",
             tp.size, ar.slot >> 20, ar.oneshot_max >> 10)
    return ar
