"""ROCm GPU enumerator -- replaces the reference's Tailscale + Ollama
``/api/tags`` probing (core/internal/discovery/discovery.go:79-384).

Sources, in order (none of them initialises the HIP runtime, so the enumerator
is safe to call from the API process and before forking GPU workers):
  1. ``LMX_FAKE_GPUS`` (tests / CPU plumbing): "N[:hbm_gb[:gfx]]";
  2. the KFD topology in sysfs (/sys/class/kfd/kfd/topology/nodes/*):
     gfx_target_version, simd/CU counts, HBM bank sizes, xGMI io_links;
  3. ``rocm-smi --showproductname --showmeminfo vram --json``.
"""
from __future__ import annotations

import json
import os
import re
import shutil
import socket
import subprocess
from dataclasses import asdict, dataclass, field

KFD = "/sys/class/kfd/kfd/topology/nodes"


@dataclass
class GpuInfo:
    index: int
    gfx: str = ""
    name: str = ""
    hbm_gb: float = 0.0
    cus: int = 0
    node_id: int = -1
    pci_bus: str = ""
    xgmi_peers: list[int] = field(default_factory=list)
    temp_c: float | None = None
    hbm_used_gb: float | None = None

    def to_dict(self):
        return asdict(self)


def _props(path: str) -> dict:
    out = {}
    try:
        with open(path) as f:
            for line in f:
                p = line.split()
                if len(p) == 2:
                    try:
                        out[p[0]] = int(p[1])
                    except ValueError:
                        out[p[0]] = p[1]
    except OSError:
        pass
    return out


def _gfx_from_version(v: int) -> str:
    # gfx_target_version 90500 -> gfx950
    major, minor, step = v // 10000, (v // 100) % 100, v % 100
    return f"gfx{major}{minor:x}{step:x}" if v else ""


def from_kfd(root: str = KFD) -> list[GpuInfo]:
    if not os.path.isdir(root):
        return []
    gpus = []
    for n in sorted(os.listdir(root), key=lambda x: int(x) if x.isdigit() else 1 << 30):
        if not n.isdigit():
            continue
        pr = _props(os.path.join(root, n, "properties"))
        if not pr.get("simd_count"):
            continue  # CPU node
        mem = 0
        mb = os.path.join(root, n, "mem_banks")
        if os.path.isdir(mb):
            for b in os.listdir(mb):
                mem += int(_props(os.path.join(mb, b, "properties")).get("size_in_bytes", 0))
        peers = []
        il = os.path.join(root, n, "io_links")
        if os.path.isdir(il):
            for l in os.listdir(il):
                lp = _props(os.path.join(il, l, "properties"))
                if lp.get("type") == 11:  # HSA_IOLINKTYPE_XGMI
                    peers.append(int(lp.get("node_to", -1)))
        simd = int(pr.get("simd_count", 0))
        per_cu = int(pr.get("simd_per_cu", 4) or 4)
        gpus.append(GpuInfo(index=len(gpus), gfx=_gfx_from_version(int(pr.get(
            "gfx_target_version", 0))), name=str(pr.get("device_id", "")),
            hbm_gb=round(mem / 2 ** 30, 1), cus=simd // per_cu, node_id=int(n),
            pci_bus=str(pr.get("location_id", "")), xgmi_peers=peers))
    # translate peer KFD node ids into GPU indices
    node_to_idx = {g.node_id: g.index for g in gpus}
    for g in gpus:
        g.xgmi_peers = sorted(node_to_idx[p] for p in g.xgmi_peers if p in node_to_idx)
    return gpus


def from_rocm_smi() -> list[GpuInfo]:
    exe = shutil.which("rocm-smi") or ("/opt/rocm/bin/rocm-smi"
                                       if os.path.exists("/opt/rocm/bin/rocm-smi") else None)
    if not exe:
        return []
    try:
        r = subprocess.run([exe, "--showproductname", "--showmeminfo", "vram", "--showtemp",
                            "--json"], capture_output=True, text=True, timeout=20)
        data = json.loads(r.stdout or "{}")
    except Exception:
        return []
    gpus = []
    for k in sorted(data, key=lambda s: int(re.sub(r"\D", "", s) or 0)):
        if not k.startswith("card"):
            continue
        v = data[k]
        tot = float(v.get("VRAM Total Memory (B)", 0) or 0)
        used = float(v.get("VRAM Total Used Memory (B)", 0) or 0)
        temp = None
        for tk, tv in v.items():
            if "Temperature" in tk and "junction" in tk.lower():
                try:
                    temp = float(tv)
                except ValueError:
                    pass
        gpus.append(GpuInfo(index=len(gpus), gfx=str(v.get("GFX Version", "")).lower(),
                            name=str(v.get("Card Series", v.get("Card SKU", ""))),
                            hbm_gb=round(tot / 2 ** 30, 1), temp_c=temp,
                            hbm_used_gb=round(used / 2 ** 30, 1) if used else None))
    return gpus


def from_fake(spec: str) -> list[GpuInfo]:
    parts = spec.split(":")
    n = int(parts[0])
    hbm = float(parts[1]) if len(parts) > 1 else 288.0
    gfx = parts[2] if len(parts) > 2 else "gfx950"
    return [GpuInfo(index=i, gfx=gfx, name="AMD Instinct MI355X (fake)", hbm_gb=hbm, cus=256,
                    xgmi_peers=[j for j in range(n) if j != i]) for i in range(n)]


def enumerate_gpus() -> list[GpuInfo]:
    fake = os.environ.get("LMX_FAKE_GPUS")
    if fake:
        return from_fake(fake)
    gpus = from_kfd()
    if not gpus:
        gpus = from_rocm_smi()
    else:
        smi = {g.index: g for g in from_rocm_smi()}
        for g in gpus:
            s = smi.get(g.index)
            if s:
                g.temp_c, g.hbm_used_gb = s.temp_c, s.hbm_used_gb
                g.name = s.name or g.name
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    if vis:
        keep = [int(x) for x in vis.split(",") if x.strip().isdigit()]
        gpus = [g for g in gpus if g.index in keep]
    return gpus


def gpu_telemetry(drm_root: str = "/sys/class/drm") -> dict[int, dict]:
    """Cheap live GPU counters from the amdgpu DRM sysfs (no subprocess):
    {gpu index: {"busy_pct", "hbm_used_bytes"}}.  Cards are matched to the
    enumeration by PCI location (KFD location_id = bus << 8 | dev << 3 | fn),
    falling back to card order.  Empty where the files do not exist."""
    cards = []
    try:
        names = sorted((n for n in os.listdir(drm_root) if re.fullmatch(r"card\d+", n)),
                       key=lambda n: int(n[4:]))
    except OSError:
        return {}
    for n in names:
        dev = os.path.join(drm_root, n, "device")
        try:
            with open(os.path.join(dev, "vendor")) as f:
                if f.read().strip() != "0x1002":
                    continue
        except OSError:
            continue
        rec = {}
        for key, fname in (("busy_pct", "gpu_busy_percent"), ("hbm_used_bytes", "mem_info_vram_used")):
            try:
                with open(os.path.join(dev, fname)) as f:
                    rec[key] = int(f.read().strip())
            except (OSError, ValueError):
                pass
        loc = None
        m = re.search(r"([0-9a-f]{2}):([0-9a-f]{2})\.([0-7])$", os.path.realpath(dev))
        if m:
            loc = (int(m.group(1), 16) << 8) | (int(m.group(2), 16) << 3) | int(m.group(3))
        if rec:
            cards.append((loc, rec))
    by_loc = {}
    for g in from_kfd():
        try:
            by_loc[int(g.pci_bus)] = g.index
        except ValueError:
            pass
    out = {}
    for i, (loc, rec) in enumerate(cards):
        out[by_loc.get(loc, i) if loc is not None else i] = rec
    return out


def gpu_clock_snapshot(timeout_s: float = 15.0) -> dict:
    """Clocks, power and temperature of every card, for benchmark records
    (two runs of the same commit on two boxes differ by a few percent; the
    record says whether a box ran slower or the code regressed):
    {card: {"sclk_mhz", "mclk_mhz", "power_w", "power_cap_w", "temp_c": {...}}}
    parsed tolerantly from ``rocm-smi --json``; {"error": ...} when unavailable."""
    exe = shutil.which("rocm-smi") or ("/opt/rocm/bin/rocm-smi"
                                       if os.path.exists("/opt/rocm/bin/rocm-smi") else None)
    if exe is None:
        return {"error": "rocm-smi not found"}
    try:
        r = subprocess.run([exe, "--showclocks", "--showpower", "--showmaxpower", "--showtemp",
                            "--json"], capture_output=True, text=True, timeout=timeout_s)
        data = json.loads(r.stdout or "{}")
    except (subprocess.SubprocessError, OSError, ValueError) as ex:
        return {"error": str(ex)[:200]}
    return parse_clock_snapshot(data) or {"error": (r.stderr or "no card")[:200]}


def parse_clock_snapshot(data: dict) -> dict:
    def num(v):
        m = re.search(r"-?\d+(?:\.\d+)?", str(v))
        return float(m.group(0)) if m else None
    out = {}
    for card, kv in data.items():
        if not isinstance(kv, dict) or not card.lower().startswith("card"):
            continue
        rec: dict = {"temp_c": {}}
        for k, v in kv.items():
            kl = k.lower()
            if ("sclk" in kl or "mclk" in kl) and "mhz" not in str(v).lower():
                continue              # clock *level* indices, not frequencies
            if "sclk" in kl:
                rec["sclk_mhz"] = num(v)
            elif "mclk" in kl:
                rec["mclk_mhz"] = num(v)
            elif "power" in kl and "max" in kl:
                rec["power_cap_w"] = num(v)
            elif "power" in kl and "(w)" in kl:
                rec["power_w"] = num(v)
            elif "temperature" in kl:
                sensor = re.search(r"sensor ([a-z0-9 ]+)\)", kl)
                rec["temp_c"][sensor.group(1).strip() if sensor else kl] = num(v)
        out[card] = rec
    return out


def host_id() -> str:
    return os.environ.get("LMX_NODE_ID") or socket.gethostname()


def device_id(gpu_index: int, host: str | None = None) -> str:
    return f"{host or host_id()}:gpu{gpu_index}"
