"""Front-door load shared by the API processes of one node.

Several API processes serve one port (SO_REUSEPORT, api/serve.py).  The
kernel hashes client connections over them unevenly, and each process that
balanced only its own streams would hand its remainder (share mod replicas)
to the same first replicas as every other process: with 4 processes and 8
engines one engine can receive mean + 3 streams.  At a fixed per-engine slot
count (``max_num_seqs``) the overflow waits for a whole generation -- the
slowest engine then sets the node's wave time.

``SharedLoad`` keeps one in-flight counter per (API process, replica slot) in
a small shared-memory file (``/dev/shm``): every process writes only its own
row, selection reads the column sums, and the pick plus its increment run
under an exclusive ``flock`` so two processes never take the same last slot.
A restarted process zeroes its own row (the streams it held died with it).
"""
from __future__ import annotations

import fcntl
import mmap
import os
from contextlib import contextmanager

import numpy as np

_HDR = 16   # magic u32, rows u32, cols u32, pad


class SharedLoad:
    MAGIC = 0x4C4D584C   # "LMXL"

    def __init__(self, path: str, row: int, rows: int, cols: int):
        if not (0 <= row < rows and cols > 0):
            raise ValueError(f"shared load: row {row} of {rows}, {cols} cols")
        self.path, self.row, self.rows, self.cols = path, row, rows, cols
        size = _HDR + rows * cols * 8
        self._fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o600)
        with self._locked():
            if os.fstat(self._fd).st_size < size:
                os.ftruncate(self._fd, size)
            self._mm = mmap.mmap(self._fd, size)
            hdr = np.frombuffer(self._mm, dtype=np.uint32, count=4)
            if hdr[0] != self.MAGIC:
                hdr[:] = (self.MAGIC, rows, cols, 0)
            elif (int(hdr[1]), int(hdr[2])) != (rows, cols):
                raise ValueError(f"{path}: shaped {int(hdr[1])}x{int(hdr[2])}, "
                                 f"not {rows}x{cols}")
            self._arr = np.frombuffer(self._mm, dtype=np.int64, offset=_HDR,
                                      count=rows * cols).reshape(rows, cols)
            self._arr[row, :] = 0

    @contextmanager
    def _locked(self):
        fcntl.flock(self._fd, fcntl.LOCK_EX)
        try:
            yield
        finally:
            fcntl.flock(self._fd, fcntl.LOCK_UN)

    @contextmanager
    def locked(self):
        """Hold the lock across a read of ``totals`` and a following ``add``."""
        with self._locked():
            yield self

    def totals(self) -> np.ndarray:
        return self._arr.sum(axis=0)

    def add(self, col: int, d: int) -> None:
        """Own row only; call inside ``locked`` when it follows a selection."""
        self._arr[self.row, col] += d

    def release(self, col: int) -> None:
        with self._locked():
            self._arr[self.row, col] -= 1

    def close(self) -> None:
        try:
            with self._locked():
                self._arr[self.row, :] = 0
        finally:
            del self._arr
            self._mm.close()
            os.close(self._fd)
