"""Decode projection GEMM (K11, csrc/kernels/dgemm.hip) against hipBLASLt.

For every projection shape of a model and every decode-graph batch bucket M,
times each kernel configuration (tile BM x BN, split-K S) and the library
(torch F.linear -> hipBLASLt with the served TunableOp table) on COLD
weights: the weight operand rotates over enough copies (> the 256 MB
Infinity Cache) that every call streams it from HBM, as in a decode step
where 15 GB of other weights pass between two reads of one layer.  The
activation operand stays warm (it was just produced).  Each configuration is
checked against the library result before it is timed.  The fastest
``NT_TOP`` configurations are timed again with the non-temporal weight stream
(cfg id | ops.DGEMM_NT).

  python -m llm_mcp_amd.bench.dgemm_bench [--model llama-3-8b] [--write]

``--write`` stores the configurations that beat the library by more than
``--margin`` into config/dgemm_gfx950.json (read by ops.dgemm_choice).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import torch

from .. import ops
from ..models.weights import vocab_shard

BUCKETS = [16, 32, 48, 64, 80, 96, 112, 128, 160, 192, 224, 256]
NT_TOP = 4      # configurations re-timed with the non-temporal weight stream (cfg | DGEMM_NT)


def shapes(model: str, tp: int = 1) -> dict:
    from ..models import config as mc
    c = mc.resolve(model)
    d, hd = c.hidden_size, c.head_dim
    qkv = (c.num_heads // tp + 2 * max(1, c.num_kv_heads // tp)) * hd
    inter = c.intermediate_size // tp
    return {"qkv": (qkv, d, 0), "o": (d, c.num_heads // tp * hd, 0),
            "gate_up": (2 * inter, d, 1), "down": (d, inter, 0),
            "lm_head": (vocab_shard(c.vocab_size, tp), d, 0)}


# projections whose output feeds the fused residual-add RMSNorm (TP = 1):
# candidates for the partials-only form (epi 2), timed together with the norm
DEFERRED = ("o", "down")


def _time(fn, iters: int) -> float:
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn(0)
    torch.cuda.synchronize()
    s.record()
    for i in range(iters):
        fn(i)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def interleave(w: torch.Tensor, block: int) -> torch.Tensor:
    I2, d = w.shape
    I = I2 // 2
    return w.view(2, I // block, block, d).transpose(0, 1).reshape(I2, d).contiguous()


def run(model: str, tp: int, ms: list[int], margin: float, only: str = "",
        swiglu16: bool = True) -> list[dict]:
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfgs = ops.native().dgemm_configs()
    rows = []
    best_entries = []
    for name, (N, K, epi) in shapes(model, tp).items():
        if only and name not in only.split(","):
            continue
        # gate/up: the in-register SwiGLU over 16-column pairs (epi 3, one
        # weight layout for every tile) unless --no-swiglu16 (epi 1, BN/2 blocks)
        if epi == 1 and swiglu16:
            epi = 3
        nbytes = N * K * 2
        ncopy = max(2, math.ceil((640 << 20) / nbytes))
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(ncopy)]
        wil = {}
        for M in ms:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            iters = max(ncopy, 40)
            if epi == 3:
                if 16 not in wil:
                    wil[16] = [interleave(w, ops.SWIGLU16) for w in ws]

                def lib(i):
                    ops.silu_mul(torch.nn.functional.linear(x, wil[16][i % ncopy]),
                                 block=ops.SWIGLU16)
            elif epi:
                def lib(i):
                    ops.silu_mul(torch.nn.functional.linear(x, ws[i % ncopy]))
            else:
                def lib(i):
                    torch.nn.functional.linear(x, ws[i % ncopy])
            t_lib = _time(lib, iters)
            ref = torch.nn.functional.linear(x, ws[0]).float()
            if epi:
                I = N // 2
                ref = torch.nn.functional.silu(ref[:, :I]) * ref[:, I:]
            best = None
            timed = []

            def attempt(cfg, s, bm, bn):
                if epi == 3:
                    wv = wil[16]
                elif epi:
                    if bn not in wil:
                        wil[bn] = [interleave(w, bn // 2) for w in ws]
                    wv = wil[bn]
                else:
                    wv = ws
                out = ops.dgemm(x, wv[0], cfg, s, epi)
                err = (out.float() - ref).abs().max().item()
                tol = 2e-2 * ref.abs().max().item() + 1e-3
                if not err <= tol:
                    print(f"  !! {name} M={M} cfg={cfg} s={s}: max err {err:.4g} > {tol:.4g}",
                          file=sys.stderr)
                    rows.append({"shape": name, "M": M, "cfg": cfg, "splits": s, "error": err})
                    return None
                t = _time(lambda i: ops.dgemm(x, wv[i % ncopy], cfg, s, epi, out=out), iters)
                rows.append({"shape": name, "M": M, "N": N, "K": K, "epi": epi, "cfg": cfg,
                             "bm": bm, "bn": bn, "splits": s, "us": round(t, 2),
                             "lib_us": round(t_lib, 2)})
                return t

            for cfg, (bm, bn) in enumerate(cfgs):
                if N % bn or (epi == 3 and not ops.swiglu16_ok(cfg)):
                    continue
                tiles = -(-M // bm) * (N // bn)
                if bm > 2 * max(64, M) and bm > 64:
                    continue
                for s in (1, 2, 4, 8, 16):
                    nwg = tiles * s
                    bk = 128 if cfg in ops.DGEMM_BK128 else 64
                    if K % (bk * s) or nwg < 32 or nwg > 1536 or (s > 1 and K // s < 256):
                        continue
                    t = attempt(cfg, s, bm, bn)
                    if t is not None:
                        timed.append((t, cfg, s, bm, bn))
            # the fastest few again with the non-temporal weight stream
            for t0, cfg, s, bm, bn in sorted(timed)[:NT_TOP]:
                t = attempt(cfg | ops.DGEMM_NT, s, bm, bn)
                if t is not None:
                    timed.append((t, cfg | ops.DGEMM_NT, s, bm, bn))
            # the stream-K form (one workgroup per CU, pieces summed by a
            # second kernel) of every tile, non-temporal weights, plain epilogue
            if epi == 0:
                for cfg, (bm, bn) in enumerate(cfgs):
                    if N % bn or (bm > 2 * max(64, M) and bm > 64):
                        continue
                    t = attempt(cfg | ops.DGEMM_SK | ops.DGEMM_NT, 0, bm, bn)
                    if t is not None:
                        timed.append((t, cfg | ops.DGEMM_SK | ops.DGEMM_NT, 0, bm, bn))
            if timed:
                best = min(timed)
            line = f"{name:8s} M={M:4d} lib {t_lib:7.1f} us ({nbytes / t_lib / 1e6:5.2f} TB/s)"
            if best:
                t, cfg, s, bm, bn = best
                line += (f" | best dgemm cfg {cfg} ({bm}x{bn}) S={s}: {t:7.1f} us "
                         f"({nbytes / t / 1e6:5.2f} TB/s) x{t_lib / t:.2f}")
            if best and best[0] * (1 + margin) < t_lib:
                t, cfg, s, bm, bn = best
                best_entries.append({"N": N, "K": K, "epi": epi, "m_max": M, "cfg": cfg,
                                     "splits": s, "bn": bn, "us": round(t, 2),
                                     "lib_us": round(t_lib, 2), "shape": name})
            else:   # the library keeps this bucket
                best_entries.append({"N": N, "K": K, "epi": epi, "m_max": M, "cfg": -1,
                                     "splits": 0, "bn": 0, "us": None,
                                     "lib_us": round(t_lib, 2), "shape": name})
            print(line, flush=True)
            if name in DEFERRED and tp == 1:
                best_entries.append(deferred(name, N, K, M, x, ws, ncopy, iters, cfgs, margin,
                                             rows))
        del ws, wil
        torch.cuda.empty_cache()
    return rows, best_entries


def deferred(name, N, K, M, x, ws, ncopy, iters, cfgs, margin, rows) -> dict:
    """Projection + residual-add RMSNorm: library GEMM + norm, K11 + norm,
    and K11 partials (epi 2) summed inside the norm (rmsnorm_slabs)."""
    dev = x.device
    lnw = (1.0 + 0.1 * torch.randn(N, device=dev)).to(torch.bfloat16)
    res0 = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    res = res0.clone()
    normed = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

    def lib(i):
        ops.rms_norm(torch.nn.functional.linear(x, ws[i % ncopy]), lnw, 1e-5, residual=res,
                     out=normed)
    t_lib = _time(lib, iters)
    r_ref = res0.clone()
    ref = ops.rms_norm(torch.nn.functional.linear(x, ws[0]), lnw, 1e-5, residual=r_ref)
    timed = []

    def attempt(cfg, s_, bm, bn):
        r2 = res0.clone()
        got = ops.rms_norm(ops.dgemm_partials(x, ws[0], cfg, s_), lnw, 1e-5, residual=r2)
        err = (got.float() - ref.float()).abs().max().item()
        if not err <= 5e-2 * ref.float().abs().max().item() + 1e-2:
            print(f"  !! {name}+norm M={M} cfg={cfg} s={s_}: err {err:.4g}", file=sys.stderr)
            return None
        t = _time(lambda i: ops.rms_norm(ops.dgemm_partials(x, ws[i % ncopy], cfg, s_), lnw,
                                         1e-5, residual=res, out=normed), iters)
        rows.append({"shape": name + "+norm", "M": M, "N": N, "K": K, "epi": 2, "cfg": cfg,
                     "bm": bm, "bn": bn, "splits": s_, "us": round(t, 2),
                     "lib_us": round(t_lib, 2)})
        return t

    for cfg, (bm, bn) in enumerate(cfgs):
        if N % bn or (bm > 2 * max(64, M) and bm > 64):
            continue
        tiles = -(-M // bm) * (N // bn)
        for s_ in (1, 2, 4, 8, 16):
            nwg = tiles * s_
            bk = 128 if cfg in ops.DGEMM_BK128 else 64
            if K % (bk * s_) or nwg < 32 or nwg > 1536 or (s_ > 1 and K // s_ < 256):
                continue
            t = attempt(cfg, s_, bm, bn)
            if t is not None:
                timed.append((t, cfg, s_, bm, bn))
    for t0, cfg, s_, bm, bn in sorted(timed)[:NT_TOP]:
        t = attempt(cfg | ops.DGEMM_NT, s_, bm, bn)
        if t is not None:
            timed.append((t, cfg | ops.DGEMM_NT, s_, bm, bn))
    best = min(timed) if timed else None
    line = f"{name + '+norm':12s} M={M:4d} lib+norm {t_lib:7.1f} us"
    e = {"N": N, "K": K, "epi": 2, "m_max": M, "cfg": -1, "splits": 0, "bn": 0, "us": None,
         "lib_us": round(t_lib, 2), "shape": name + "+norm"}
    if best:
        t, cfg, s_, bm, bn = best
        line += f" | partials cfg {cfg} ({bm}x{bn}) S={s_} + norm: {t:7.1f} us x{t_lib / t:.2f}"
        if t * (1 + margin) < t_lib:
            e.update(cfg=cfg, splits=s_, bn=bn, us=round(t, 2))
    print(line, flush=True)
    return e


def _consistent_bn(entries: list[dict]) -> list[dict]:
    """The fused-SwiGLU weights can be interleaved one way only: keep the
    epi=1 entries of the most common BN per (N, K)."""
    out, by = [], {}
    for e in entries:
        if e["epi"] == 1 and e["cfg"] >= 0:
            by.setdefault((e["N"], e["K"]), []).append(e)
        else:
            out.append(e)
    for lst in by.values():
        bns = [e["bn"] for e in lst]
        keep = max(set(bns), key=lambda b: sum(e["lib_us"] - e["us"] for e in lst if e["bn"] == b))
        for e in lst:
            if e["bn"] != keep:
                e.update(cfg=-1, splits=0, bn=0, us=None)
        out += lst
    return out


def table_from_rows(rows: list[dict], margin: float) -> list[dict]:
    """Rebuild the dispatch entries from saved timing rows (--json output)."""
    best: dict = {}
    for r in rows:
        if "us" not in r:
            continue
        key = (r["shape"], r["N"], r["K"], r["epi"], r["M"])
        if key not in best or r["us"] < best[key]["us"]:
            best[key] = r
    out = []
    for (shape, N, K, epi, M), r in sorted(best.items()):
        e = {"N": N, "K": K, "epi": epi, "m_max": M, "cfg": -1, "splits": 0, "bn": 0,
             "us": None, "lib_us": r["lib_us"], "shape": shape}
        if r["us"] * (1 + margin) < r["lib_us"]:
            e.update(cfg=r["cfg"], splits=r["splits"], bn=r["bn"], us=r["us"])
        out.append(e)
    return _consistent_bn(out)


SWIGLU_SHAPES = ("nomic.gate_up", "l8b.gate_up")


def encoder(ms: list[int], write: bool = False, k11: bool = False) -> None:
    """Prefill / encoder shapes (nomic-bert, BERT-large, Llama-3-8B prefill):
    hipBLASLt vs K13 (the large-M GEMM, ops.pgemm), warm operands (uniform
    [-1, 1)), TFLOP/s; the gate/up shapes also as the fused SwiGLU forms
    (library GEMM + GLU kernel vs K13's SwiGLU epilogue, FLOPs of the GEMM).
    ``k11``: also sweep every K11 configuration and gemm_nt (the round-2 table).
    ``write`` merges the numbers of the largest M into config/dgemm_gfx950.json
    "encoder" (read by ops.encoder_backend / ops.large_gemm_backend)."""
    shapes = {"nomic.qkv": (2304, 768), "nomic.o": (768, 768), "nomic.gate_up": (6144, 768),
              "nomic.down": (768, 3072), "l8b.qkv": (6144, 4096), "l8b.o": (4096, 4096),
              "l8b.gate_up": (28672, 4096), "l8b.down": (4096, 14336), "bert.qkv": (3072, 1024),
              "bert.o": (1024, 1024), "bert.w1": (4096, 1024), "bert.w2": (1024, 4096)}
    cfgs = ops.native().dgemm_configs()
    path = os.path.join(os.path.dirname(os.path.dirname(__file__)), "config", "dgemm_gfx950.json")
    with open(path) as f:
        doc = json.load(f)
    table = {(e["N"], e["K"]): e for e in doc.get("encoder", [])}
    for M in ms:
        for name, (N, K) in shapes.items():
            if name.startswith("l8b") and M < 8192:
                continue
            x = torch.rand(M, K, device="cuda", dtype=torch.bfloat16) * 2 - 1
            w = (torch.rand(N, K, device="cuda", dtype=torch.bfloat16) * 2 - 1) * K ** -0.5
            fl = 2.0 * M * N * K
            iters = max(5, min(50, int(2e12 / fl)))
            ref = torch.nn.functional.linear(x, w).float()
            t_lib = _time(lambda i: torch.nn.functional.linear(x, w), iters)
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            ops.pgemm(x, w, out=out)
            assert (out.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item(), name
            t_k13 = _time(lambda i: ops.pgemm(x, w, out=out), iters)
            e = table.setdefault((N, K), {"N": N, "K": K})
            e.update({"M": M, "lib_tflops": round(fl / t_lib / 1e6, 1),
                      "k13_tflops": round(fl / t_k13 / 1e6, 1)})
            line = (f"{name:13s} M={M:6d} lib {fl / t_lib / 1e6:6.0f} TF | "
                    f"K13 {fl / t_k13 / 1e6:6.0f} TF ({t_lib / t_k13:.3f}x)")
            if name in SWIGLU_SHAPES:
                wil = ops.interleave_gate_up(w, ops.SWIGLU16)
                g = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
                t_lg = _time(lambda i: ops.silu_mul(torch.nn.functional.linear(x, wil),
                                                    block=ops.SWIGLU16), iters)
                t_ks = _time(lambda i: ops.pgemm(x, wil, act=ops.ACT_SWIGLU, out=g), iters)
                e.update({"lib_glu_tflops": round(fl / t_lg / 1e6, 1),
                          "k13_swiglu_tflops": round(fl / t_ks / 1e6, 1)})
                line += (f" | SwiGLU: lib+glu {fl / t_lg / 1e6:6.0f} TF, K13 "
                         f"{fl / t_ks / 1e6:6.0f} TF ({t_lg / t_ks:.3f}x)")
            if k11:
                t_nt = _time(lambda i: ops.gemm_nt(x, w), iters) \
                    if ops.gemm_nt_supported(N, K) else None
                best = None
                for cfg, (bm, bn) in enumerate(cfgs):
                    if N % bn:
                        continue
                    o11 = ops.dgemm(x, w, cfg, 1)
                    if not (o11.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item():
                        continue
                    t = _time(lambda i: ops.dgemm(x, w, cfg, 1, out=o11), iters)
                    if best is None or t < best[0]:
                        best = (t, cfg, bm, bn)
                if best:
                    e.update({"cfg": best[1], "bn": best[3],
                              "tflops": round(fl / best[0] / 1e6, 1)})
                    line += f" | K11 cfg {best[1]} {fl / best[0] / 1e6:6.0f} TF"
                if t_nt:
                    e["gemm_nt_tflops"] = round(fl / t_nt / 1e6, 1)
            print(line, flush=True)
    if write:
        doc["encoder"] = sorted(table.values(), key=lambda e: (e["N"], e["K"]))
        with open(path, "w") as f:
            json.dump(doc, f, indent=1)
        print(f"wrote {len(table)} encoder entries to {path}")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--encoder", default="", help="comma list of M: prefill/encoder shapes")
    ap.add_argument("--k11", action="store_true", help="--encoder: also sweep K11 and gemm_nt")
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--m", default=",".join(map(str, BUCKETS)))
    ap.add_argument("--only", default="", help="comma list of qkv,o,gate_up,down")
    ap.add_argument("--margin", type=float, default=0.03)
    ap.add_argument("--no-swiglu16", action="store_true",
                    help="gate/up with the LDS hand-off epilogue (epi 1) instead of epi 3")
    ap.add_argument("--write", action="store_true")
    ap.add_argument("--json", default="", help="also dump every timing row here")
    ap.add_argument("--from-rows", default="",
                    help="no GPU run: rebuild the table from a saved --json file")
    a = ap.parse_args(argv)
    if a.from_rows:
        with open(a.from_rows) as f:
            best = table_from_rows(json.load(f), a.margin)
        _write(best, "from " + os.path.basename(a.from_rows))
        return
    ops.native()
    os.environ.setdefault("LMX_DGEMM", "0")
    if a.encoder:
        encoder([int(v) for v in a.encoder.split(",")], a.write, a.k11)
        return
    from ..engine.engine import _load_gemm_tuning
    _load_gemm_tuning()       # the library as served: hipBLASLt with the TunableOp table
    ms = [int(v) for v in a.m.split(",") if v]
    rows, best = run(a.model, a.tp, ms, a.margin, a.only, swiglu16=not a.no_swiglu16)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)
    if a.write:
        _write(best, torch.cuda.get_device_name(0))


def _write(best: list[dict], device: str) -> None:
    path = os.path.join(os.path.dirname(os.path.dirname(__file__)), "config",
                        "dgemm_gfx950.json")
    old = {"entries": []}
    if os.path.exists(path):
        with open(path) as f:
            old = json.load(f)
    keys = {(e["N"], e["K"], e["epi"]) for e in best}
    kept = [e for e in old.get("entries", []) if (e["N"], e["K"], e.get("epi", 0)) not in keys]
    doc = dict(old)          # other sections (the "encoder" table) are kept
    doc.update({"device": device,
                "note": "decode GEMM dispatch measured by bench/dgemm_bench.py (cold weights); "
                        "cfg -1 = the library keeps the bucket",
                "entries": kept + best})
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)
    print(f"wrote {len(doc['entries'])} entries to {path}")


if __name__ == "__main__":
    main()
