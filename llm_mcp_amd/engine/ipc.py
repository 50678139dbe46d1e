"""Engine <-> API process link (Unix domain socket, length-prefixed msgpack).

A GPU worker process owns the engine (and, under TP, leads its rank group);
the API process ("core") owns HTTP, tokenisation and SSE.  Splitting them
keeps the Python GIL of the HTTP/SSE hot loop away from the engine step loop.
The link is the in-tree, binary, batched equivalent of the reference's
core -> Ollama ``/api/chat`` NDJSON hop (core/internal/api/handlers.go:2427):

  API -> engine   {"op": "submit", "rid", "prompt", "params", "priority"}
                  {"op": "abort", "rid"}        {"op": "info", "tag"}
                  {"op": "embed", "tag", "ids": int32 bytes, "lens", "dims"}
  engine -> API   {"op": "ev", "ev": [[rid, token, logprob, finish], ...]}
                  (ONE message per engine step per connection)
                  {"op": "info", "tag", "info": {...}}
                  {"op": "emb", "tag", "vec": float32 bytes, "shape", "error"}

``EngineClient`` exposes the same ``generate()`` async-iterator interface as
``AsyncEngine``, so the API layer does not care where the engine lives.
"""
from __future__ import annotations

import asyncio
import dataclasses
import itertools
import logging
import os
import socket
import struct
import threading

import msgpack
import numpy as np

from .async_engine import RequestStats, StreamItem
from .engine import GenRequest, SamplingParams, TokenEvent

log = logging.getLogger("lmx.ipc")
_HDR = struct.Struct("<I")


def _pack(obj) -> bytes:
    b = msgpack.packb(obj, use_bin_type=True)
    return _HDR.pack(len(b)) + b


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("peer closed")
        buf += chunk
    return bytes(buf)


class _Conn:
    def __init__(self, sock: socket.socket):
        self.sock = sock
        self.lock = threading.Lock()
        self.alive = True

    def send(self, obj) -> None:
        data = _pack(obj)
        with self.lock:
            if self.alive:
                try:
                    self.sock.sendall(data)
                except OSError:
                    self.alive = False


class EngineServer:
    """Serves one LLMEngine over a Unix socket (runs in the GPU process)."""

    def __init__(self, engine, path: str, info: dict | None = None, embed_engine=None,
                 fallback_sink=None):
        self.engine = engine
        self.embed_engine = embed_engine
        # events of requests not submitted over IPC (e.g. the worker's own job
        # runner, an AsyncEngine on the same engine) go to the fallback sink
        self.fallback_sink = fallback_sink
        self.path = path
        self.info = dict(info or {})
        self._conns: dict[int, _Conn] = {}
        self._req_conn: dict[int, tuple[int, int]] = {}   # engine id -> (conn id, client rid)
        self._ids = itertools.count(1)
        self._lock = threading.Lock()
        if engine is not None:
            engine.event_sink = self._sink
        self._sock: socket.socket | None = None

    def start(self) -> None:
        if os.path.exists(self.path):
            os.unlink(self.path)
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        s.bind(self.path)
        s.listen(16)
        self._sock = s
        threading.Thread(target=self._accept, daemon=True, name="ipc-accept").start()
        if self.engine is not None:
            self.engine.start()
        if self.embed_engine is not None:
            self.embed_engine.start()

    def stop(self) -> None:
        if self.engine is not None:
            self.engine.stop()
        if self.embed_engine is not None:
            self.embed_engine.stop()
        if self._sock is not None:
            self._sock.close()
        if os.path.exists(self.path):
            os.unlink(self.path)

    def _accept(self):
        while True:
            try:
                s, _ = self._sock.accept()
            except OSError:
                return
            cid = next(self._ids)
            c = _Conn(s)
            with self._lock:
                self._conns[cid] = c
            threading.Thread(target=self._reader, args=(cid, c), daemon=True,
                             name=f"ipc-conn-{cid}").start()

    def _reader(self, cid: int, c: _Conn):
        try:
            while True:
                n = _HDR.unpack(_recv_exact(c.sock, 4))[0]
                msg = msgpack.unpackb(_recv_exact(c.sock, n), raw=False)
                op = msg.get("op")
                if op == "submit":
                    p = SamplingParams(**msg["params"])
                    req = GenRequest(list(msg["prompt"]), p, priority=msg.get("priority", 0))
                    req.id = next(self.engine._ids)
                    with self._lock:
                        self._req_conn[req.id] = (cid, msg["rid"])
                    self.engine.submit(req)
                elif op == "abort":
                    eid = None
                    with self._lock:
                        for k, (cc, rr) in self._req_conn.items():
                            if cc == cid and rr == msg["rid"]:
                                eid = k
                                break
                    if eid is not None:
                        self.engine.abort(eid)
                elif op == "embed":
                    self._embed(c, msg)
                elif op == "info":
                    info = dict(self.info)
                    info.update(self.engine_info())
                    c.send({"op": "info", "tag": msg.get("tag"), "info": info})
        except (ConnectionError, OSError):
            pass
        finally:
            c.alive = False
            with self._lock:
                self._conns.pop(cid, None)
                dead = [k for k, (cc, _) in self._req_conn.items() if cc == cid]
                for k in dead:
                    self._req_conn.pop(k, None)
            for k in dead:
                self.engine.abort(k)

    def _embed(self, c: _Conn, msg: dict):
        """Queue an embedding request on the batching embed engine; the reply
        is sent from a helper thread once the batch containing it is done."""
        if self.embed_engine is None:
            c.send({"op": "emb", "tag": msg.get("tag"), "error": "no embedding model"})
            return
        from .embed_engine import EmbedRequest
        if "ids" in msg:
            # binary form: one int32 buffer + lengths in, float32 rows out (no
            # per-token Python objects on either side of the socket)
            flat = np.frombuffer(msg["ids"], dtype=np.int32)
            seqs = np.split(flat, np.cumsum(msg["lens"])[:-1]) if msg["lens"] else []
        else:
            seqs = msg["seqs"]
        binary = "ids" in msg
        req = EmbedRequest(self.embed_engine._truncate(seqs), msg.get("dims"))
        self.embed_engine._q.put(req)

        def reply():
            req.done.wait()
            out = {"op": "emb", "tag": msg.get("tag"), "error": req.error}
            if req.error is None:
                v = np.ascontiguousarray(np.asarray(req.result, dtype=np.float32))
                if binary:
                    out.update(vec=v.tobytes(), shape=list(v.shape))
                else:
                    out["vectors"] = v.tolist()
            c.send(out)
        threading.Thread(target=reply, daemon=True).start()

    def engine_info(self) -> dict:
        e = self.engine
        if e is None:
            return {"stats": dict(self.embed_engine.stats) if self.embed_engine else {}}
        s = e.sched

        def skeys(d):
            # msgpack peers unpack with strict_map_key: message-size keys as str
            return {str(k): skeys(v) if isinstance(v, dict) else v for k, v in d.items()}
        return {"running": s.num_running, "waiting": s.num_waiting, "kv_usage": s.kv_usage,
                "kv_free_blocks": s.kv_free_blocks, "stats": dict(e.stats),
                "tp_comm": skeys(getattr(e, "tp_comm", {}) or {}),
                "tp_comm_live": skeys(getattr(e, "tp_comm_live", {}) or {})}

    # engine thread: one message per connection per step
    def _sink(self, evs: list[TokenEvent]):
        per: dict[int, list] = {}
        other = []
        with self._lock:
            for e in evs:
                m = self._req_conn.get(e.req.id)
                if m is None:
                    other.append(e)
                    continue
                per.setdefault(m[0], []).append([m[1], e.token, e.logprob, e.finish])
                if e.finish is not None:
                    self._req_conn.pop(e.req.id, None)
            conns = {cid: self._conns.get(cid) for cid in per}
        for cid, lst in per.items():
            c = conns.get(cid)
            if c is not None:
                c.send({"op": "ev", "ev": lst})
        if other and self.fallback_sink is not None:
            self.fallback_sink(other)


class EngineClient:
    """API-process side; same ``generate`` interface as AsyncEngine."""

    def __init__(self, path: str):
        self.path = path
        self._queues: dict[int, asyncio.Queue] = {}
        self._ids = itertools.count(1)
        self._writer: asyncio.StreamWriter | None = None
        self._reader_task = None
        self._info_waiters: dict[int, asyncio.Future] = {}
        self.connected = asyncio.Event()

    async def connect(self, retry_s: float = 0.5, timeout: float | None = None):
        loop = asyncio.get_running_loop()
        t_end = None if timeout is None else loop.time() + timeout
        while True:
            try:
                reader, writer = await asyncio.open_unix_connection(self.path)
                break
            except (FileNotFoundError, ConnectionRefusedError):
                if t_end is not None and loop.time() > t_end:
                    raise
                await asyncio.sleep(retry_s)
        self._writer = writer
        self._reader_task = asyncio.create_task(self._read_loop(reader))
        self.connected.set()

    async def _read_loop(self, reader: asyncio.StreamReader):
        try:
            while True:
                hdr = await reader.readexactly(4)
                msg = msgpack.unpackb(await reader.readexactly(_HDR.unpack(hdr)[0]), raw=False)
                op = msg.get("op")
                if op == "ev":
                    for rid, tok, lp, fin in msg["ev"]:
                        q = self._queues.get(rid)
                        if q is not None:
                            q.put_nowait(StreamItem(tok, lp, fin))
                elif op == "info":
                    f = self._info_waiters.pop(msg.get("tag"), None)
                    if f is not None and not f.done():
                        f.set_result(msg["info"])
                elif op == "emb":
                    f = self._info_waiters.pop(msg.get("tag"), None)
                    if f is not None and not f.done():
                        if msg.get("error"):
                            f.set_exception(RuntimeError(msg["error"]))
                        elif "vec" in msg:
                            f.set_result(np.frombuffer(msg["vec"], dtype=np.float32)
                                         .reshape(msg["shape"]))
                        else:
                            f.set_result(msg["vectors"])
        except (asyncio.IncompleteReadError, ConnectionError):
            pass
        finally:
            self.connected.clear()
            for q in self._queues.values():
                q.put_nowait(StreamItem(-1, 0.0, "error:engine_disconnected"))
            for f in self._info_waiters.values():
                if not f.done():
                    f.set_exception(ConnectionError("engine disconnected"))
            self._info_waiters.clear()

    async def wait_closed(self) -> None:
        """Return once the link to the engine process is gone (the worker
        died or closed its socket); pending streams have been failed by then."""
        if self._reader_task is not None:
            await asyncio.wait([self._reader_task])

    def _send(self, obj):
        if self._writer is None or not self.connected.is_set():
            raise ConnectionError("engine not connected")
        self._writer.write(_pack(obj))

    async def info(self, timeout: float = 5.0) -> dict:
        tag = next(self._ids)
        f = asyncio.get_running_loop().create_future()
        self._info_waiters[tag] = f
        self._send({"op": "info", "tag": tag})
        return await asyncio.wait_for(f, timeout)

    async def embed(self, seqs, dims=None) -> np.ndarray:
        tag = next(self._ids)
        f = asyncio.get_running_loop().create_future()
        self._info_waiters[tag] = f
        lens = [len(s) for s in seqs]
        flat = np.concatenate([np.asarray(s, dtype=np.int32) for s in seqs]) if seqs else \
            np.zeros(0, np.int32)
        self._send({"op": "embed", "tag": tag, "ids": flat.tobytes(), "lens": lens, "dims": dims})
        return await f

    async def complete(self, prompt_ids, params, priority=0):
        toks, lps, fin = [], [], None
        async for it in self.generate(prompt_ids, params, priority):
            if it.token >= 0:
                toks.append(it.token)
                lps.append(it.logprob)
            fin = it.finish
        return toks, lps, fin

    async def generate(self, prompt_ids, params: SamplingParams, priority: int = 0,
                       stats: RequestStats | None = None):
        rid = next(self._ids)
        q: asyncio.Queue = asyncio.Queue()
        self._queues[rid] = q
        self._send({"op": "submit", "rid": rid, "prompt": list(prompt_ids),
                    "params": dataclasses.asdict(params), "priority": priority})
        done = False
        try:
            while True:
                item = await q.get()
                yield item
                if item.finish is not None:
                    done = True
                    return
        finally:
            self._queues.pop(rid, None)
            if not done and self.connected.is_set():
                try:
                    self._send({"op": "abort", "rid": rid})
                except ConnectionError:
                    pass

    async def close(self):
        if self._writer is not None:
            self._writer.close()
        if self._reader_task is not None:
            self._reader_task.cancel()
