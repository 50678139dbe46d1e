"""In-tree build of the native parts of llm_mcp_amd.

Two shared objects are produced next to this file (so they travel with the
repository snapshot to the GPU box and are visibly loaded from the tree):

* ``_lmx_kernels*.so``  -- the gfx950 HIP kernels (hipcc --offload-arch=gfx950)
  with their pybind11 bindings.  Linked against the HIP runtime that PyTorch
  already loaded (same soname, ``libamdhip64.so.7``) so kernels and torch share
  one runtime, one device context and the same streams.
* ``_lmx_runtime*.so``  -- the CPU-side native runtime (C++17): lease job
  queue, paged-KV block manager and continuous-batching scheduler.

Usage: ``python -m llm_mcp_amd.build`` (or ``build_all()``); sources are
rebuilt only when newer than their output.
"""
from __future__ import annotations

import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = PKG / "build"
ARCH = os.environ.get("LMX_OFFLOAD_ARCH", "gfx950")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"

KERNEL_SOURCES = ["norm.hip", "rope_cache.hip", "attention.hip", "sampling.hip",
                  "elementwise.hip", "gemm.hip", "dgemm.hip", "pgemm.hip",
                  "rsgemm.hip", "allreduce.hip"]
RUNTIME_SOURCES = ["job_queue.cpp", "block_manager.cpp", "scheduler.cpp", "bindings.cpp"]


def _py_includes() -> list[str]:
    import pybind11
    inc = {sysconfig.get_paths()["include"], sysconfig.get_paths()["platinclude"],
           pybind11.get_include()}
    return [f"-I{p}" for p in sorted(inc)]


def _torch_libdir() -> str | None:
    try:
        import importlib.util
        spec = importlib.util.find_spec("torch")
        if spec and spec.origin:
            d = Path(spec.origin).parent / "lib"
            if (d / "libamdhip64.so").exists():
                return str(d)
    except Exception:
        pass
    return None


def _run(cmd: list[str]) -> str:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r.stderr


# Kernels that keep inline-asm load destinations in flight across code the
# compiler schedules (hand-counted vmcnt rings): a spill or scratch use of such
# a register before its data lands is silent corruption, so every
# instantiation must compile with no VGPR spill and no scratch.  The compile of
# these sources adds -Rpass-analysis=kernel-resource-usage and the build fails
# on a violation; the parsed table is kept in build/kernels/resource_usage.json.
ASM_RING_KERNELS = {"rsgemm.hip": r"rsgemm4?_kernel",
                    "attention.hip": r"paged_decode_\w*kernelILi\d+ELi9E"}


def parse_resource_usage(text: str) -> dict:
    """{kernel: {"vgpr_spill": n, "sgpr_spill": n, "scratch": bytes, "vgprs": n}}
    from hipcc -Rpass-analysis=kernel-resource-usage remarks."""
    import re
    out, cur = {}, None
    for line in text.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = out.setdefault(m.group(1), {})
            continue
        if cur is None:
            continue
        for key, pat in (("vgpr_spill", r"VGPRs Spill: (\d+)"), ("sgpr_spill", r"SGPRs Spill: (\d+)"),
                         ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                         ("vgprs", r"remark:\s+VGPRs: (\d+)")):
            m = re.search(pat, line)
            if m:
                cur[key] = int(m.group(1))
    return out


def audit_asm_rings(usage: dict[str, dict]) -> list[str]:
    """Violations (empty list: clean) of the no-spill / no-scratch rule."""
    import re
    bad = []
    for src, pat in ASM_RING_KERNELS.items():
        fns = {k: v for k, v in usage.get(src, {}).items() if re.search(pat, k)}
        if not fns:
            bad.append(f"{src}: no kernel matching {pat} in the resource report")
        for k, v in fns.items():
            if v.get("vgpr_spill", 0) or v.get("scratch", 0) or v.get("sgpr_spill", 0):
                bad.append(f"{src}: {k} spills (vgpr {v.get('vgpr_spill')}, "
                           f"sgpr {v.get('sgpr_spill')}, scratch {v.get('scratch')} B/lane)")
    return bad


def _stale(out: Path, deps: list[Path]) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps if d.exists())


def kernels_path() -> Path:
    return PKG / f"_lmx_kernels{EXT}"


def runtime_path() -> Path:
    return PKG / f"_lmx_runtime{EXT}"


def build_kernels(force: bool = False, verbose: bool = False) -> Path:
    kdir = CSRC / "kernels"
    out = kernels_path()
    headers = list(kdir.glob("*.h"))
    srcs = [kdir / s for s in KERNEL_SOURCES]
    objdir = BUILD / "kernels"
    objdir.mkdir(parents=True, exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    common = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
              "-munsafe-fp-atomics", f"-I{kdir}"]
    objs = []
    jobs = []
    audit_file = objdir / "resource_usage.json"
    audit_srcs = []
    for s in srcs:
        o = objdir / (s.stem + ".o")
        objs.append(o)
        ring = s.name in ASM_RING_KERNELS
        if force or _stale(o, [s] + headers) or (ring and _stale(audit_file, [s] + headers)):
            extra = ["-Rpass-analysis=kernel-resource-usage"] if ring else []
            jobs.append(common + extra + ["-c", str(s), "-o", str(o)])
            if ring:
                audit_srcs.append((len(jobs) - 1, s.name))
                # the device listing for the in-flight-register audit below
                jobs.append(common + ["--cuda-device-only", "-S", str(s), "-o",
                                      str(objdir / (s.stem + ".s"))])
    bo = objdir / "bindings.o"
    objs.append(bo)
    bsrc = kdir / "bindings.cpp"
    if force or _stale(bo, [bsrc]):
        jobs.append([hipcc, "-O2", "-std=c++17", "-fPIC", "-x", "hip", f"--offload-arch={ARCH}",
                     *_py_includes(), "-c", str(bsrc), "-o", str(bo)])
    if jobs:
        with ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
            logs = list(ex.map(_run, jobs))
        if audit_srcs:
            import json
            usage = json.loads(audit_file.read_text()) if audit_file.exists() else {}
            for i, name in audit_srcs:
                usage[name] = parse_resource_usage(logs[i])
            bad = audit_asm_rings(usage)
            # no instruction may touch an inline-asm load's destination while
            # the load is in flight (the compiler cannot see those loads)
            from .utils.vmem_audit import audit_listing
            for _, name in audit_srcs:
                lst = (objdir / (Path(name).stem + ".s")).read_text()
                for fn, iss in audit_listing(lst, ASM_RING_KERNELS[name]).items():
                    if iss:
                        bad.append(f"{name}: {fn[:80]} touches in-flight load registers "
                                   f"({len(iss)}x, first: {iss[0][1]})")
            if bad:
                for i, _ in audit_srcs:
                    Path(jobs[i][jobs[i].index("-o") + 1]).unlink(missing_ok=True)
                raise RuntimeError("inline-asm ring kernels spill:\n  " + "\n  ".join(bad))
            audit_file.write_text(json.dumps(usage, indent=1, sort_keys=True))
    if force or jobs or _stale(out, objs):
        link = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(out),
                *[str(o) for o in objs]]
        tl = _torch_libdir()
        if tl:
            # resolve libamdhip64.so.7 to the copy torch loads (one HIP runtime per process)
            link += [f"-L{tl}", f"-Wl,-rpath,{tl}"]
        link += ["-lamdhip64"]
        _run(link)
        if verbose:
            print(f"[build] {out.name}")
    return out


def build_runtime(force: bool = False, verbose: bool = False) -> Path:
    rdir = CSRC / "runtime"
    out = runtime_path()
    srcs = [rdir / s for s in RUNTIME_SOURCES]
    headers = list(rdir.glob("*.h"))
    if force or _stale(out, srcs + headers):
        cxx = os.environ.get("CXX", "g++")
        cmd = [cxx, "-O2", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-pthread",
               f"-I{rdir}", *_py_includes(), *[str(s) for s in srcs], "-o", str(out)]
        _run(cmd)
        if verbose:
            print(f"[build] {out.name}")
    return out


SANITIZERS = {"tsan": ["-fsanitize=thread"],
              "asan": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer"]}


def sanitize_runtime(which=("tsan", "asan"), verbose: bool = False) -> dict[str, str]:
    """Build the runtime stress test (csrc/runtime/tests/stress.cpp) with host
    sanitizers and run it; raises on any report.  Host code only -- GPU
    sanitizers are not used on this hardware pool."""
    rdir = CSRC / "runtime"
    srcs = [rdir / s for s in RUNTIME_SOURCES if s != "bindings.cpp"]
    out_dir = BUILD / "sanitize"
    out_dir.mkdir(parents=True, exist_ok=True)
    # ROCm's clang: its TSan runtime intercepts pthread_cond_clockwait (GCC 11's
    # does not and reports a false "double lock" on condition-variable waits)
    cxx = os.environ.get("LMX_SAN_CXX", "/opt/rocm/llvm/bin/clang++")
    logs = {}
    for name in which:
        exe = out_dir / f"stress_{name}"
        _run([cxx, "-O1", "-g", "-std=c++17", "-pthread", *SANITIZERS[name], f"-I{rdir}",
              *[str(s) for s in srcs], str(rdir / "tests" / "stress.cpp"), "-o", str(exe)])
        env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
                   ASAN_OPTIONS="detect_leaks=1:halt_on_error=1",
                   UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
        r = subprocess.run([str(exe), "1500", "2000"], capture_output=True, text=True, env=env,
                           timeout=600)
        logs[name] = r.stdout + r.stderr
        if r.returncode != 0 or "ERROR: " in r.stderr or "runtime error" in r.stderr:
            raise RuntimeError(f"{name} stress failed (rc {r.returncode}):\n{logs[name][-4000:]}")
        if verbose:
            print(f"[sanitize] {name}: {r.stdout.strip().splitlines()[-1]}")
    return logs


def build_all(force: bool = False, verbose: bool = False) -> None:
    with ThreadPoolExecutor(max_workers=2) as ex:
        fk = ex.submit(build_kernels, force, verbose)
        fr = ex.submit(build_runtime, force, verbose)
        fk.result()
        fr.result()


if __name__ == "__main__":
    if "--sanitize-runtime" in sys.argv:
        sanitize_runtime(verbose=True)
    else:
        build_all(force="--force" in sys.argv, verbose=True)
