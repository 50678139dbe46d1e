"""Discovery runner (reference: core/internal/discovery/discovery.go:79-174
and offline_handler.go).

Per run:
  1. enumerate this node's GPUs (rocm_enum) and upsert ``devices`` rows
     ``<host>:gpu<i>`` with tags {engine, rocm, gfx, hbm_gb, cus, xgmi_peers,
     engine_addr, capacity, models}; TP groups served by a multi-GPU engine are
     registered as pseudo-devices ``<host>:tp<N>:gpu<a>-<b>``;
  2. sync ``models`` / ``device_models`` from the local model registry
     (metadata from the architecture, not the name) and mark models no longer
     served as unavailable;
  3. devices of this host that disappeared go offline and their running
     jobs' leases are released so they can be reclaimed at once (the reference's
     "60 s -> <5 s" recovery, offline_handler.go:12-38);
  4. peer nodes are polled at ``GET /v1/discovery/local`` (concurrently, 2 s
     timeout) and their devices upserted with the peer's URL as
     ``engine_addr``; an unreachable peer's devices go offline with their
     leases released.  Peer sources, as the reference's mesh scan
     (discovery.go:88-174, 299-420, 755-877):
       * ``LMX_PEER_NODES`` -- explicit core URLs;
       * ``DISCOVERY_EXTRA_ENDPOINTS`` (alias ``OLLAMA_EXTRA_ENDPOINTS``) --
         ``host:port`` list;
       * Tailscale -- ``tailscale status --json`` Self/Peers (online ones are
         probed on every ``LMX_PEER_PORTS`` port, default 8080; nodes the mesh
         reports offline have their devices taken offline at once);
       * ``DISCOVERY_SCAN_SUBNETS=1`` + ``DISCOVERY_SUBNETS`` (CIDR list, at
         most 1024 hosts) -- LAN scan on the same ports.
"""
from __future__ import annotations

import ipaddress
import json
import logging
import os
import re
import shutil
import subprocess
import threading
import time
import urllib.request
from concurrent.futures import ThreadPoolExecutor

from ..policy.inference import model_record
from . import rocm_enum

log = logging.getLogger("lmx.discovery")


def tp_members(dev: str, host: str) -> tuple[int, list[str]]:
    """``<host>:tp8:gpu0-7`` -> (8, [<host>:gpu0, ..., <host>:gpu7])."""
    m = re.search(r":tp(\d+):gpu(\d+)-(\d+)$", dev)
    if not m:
        return 0, []
    tp, a, b = (int(x) for x in m.groups())
    return tp, [rocm_enum.device_id(i, host) for i in range(a, b + 1)]


class DiscoveryRunner:
    def __init__(self, store, registry=None, metrics=None, engine_addrs: dict | None = None):
        self.store = store
        self.registry = registry
        self.metrics = metrics
        self.engine_addrs = engine_addrs or {}
        self._lock = threading.Lock()
        self._last_run: float | None = None
        self.last_result: dict = {}

    def last_run(self) -> float | None:
        with self._lock:
            return self._last_run

    def local_devices(self) -> list[dict]:
        """This node's device records (also served to peers)."""
        host = rocm_enum.host_id()
        out = []
        served: dict[str, list] = {}
        if self.registry is not None:
            for m in self.registry.all():
                served.setdefault(m.device_id, []).append(m)
        gpus = rocm_enum.enumerate_gpus()
        for g in gpus:
            did = rocm_enum.device_id(g.index, host)
            ms = served.get(did, []) + served.get(f"gpu{g.index}", [])
            out.append({
                "id": did, "name": g.name or f"GPU {g.index}", "platform": "rocm",
                "arch": g.gfx or "gfx950", "host": host,
                "tags": {"engine": bool(ms) or True, "rocm": True, "gfx": g.gfx,
                         "hbm_gb": g.hbm_gb, "cus": g.cus, "gpu_index": g.index,
                         "xgmi_peers": g.xgmi_peers, "pci_bus": g.pci_bus,
                         "temp_c": g.temp_c, "hbm_used_gb": g.hbm_used_gb,
                         "engine_addr": self.engine_addrs.get(did, ""),
                         "capacity": max([m.capacity for m in ms] or [0]) or None,
                         "models": sorted({m.model_id for m in ms})},
                "models": [(m.model_id, m.cfg, m.max_model_len) for m in ms]})
        # extra workers on one GPU (``serve --replicas-per-gpu``: gpuN.rk)
        for dev, ms in served.items():
            base, _, rep = dev.rpartition(".r")
            if rep.isdigit() and ":gpu" in base and not any(d["id"] == dev for d in out):
                out.append({"id": dev, "name": dev, "platform": "rocm", "arch": "gfx950",
                            "host": host, "tags": {"engine": True, "rocm": True,
                                                   "replica_of": base,
                                                   "models": sorted({m.model_id for m in ms}),
                                                   "capacity": max(m.capacity for m in ms)},
                            "models": [(m.model_id, m.cfg, m.max_model_len) for m in ms]})
        # multi-GPU (TP) engines registered under a group id
        for dev, ms in served.items():
            if ":tp" in dev and not any(d["id"] == dev for d in out):
                tp, members = tp_members(dev, host)
                out.append({"id": dev, "name": dev, "platform": "rocm", "arch": "gfx950",
                            "host": host, "tags": {"engine": True, "rocm": True, "tp_group": True,
                                                   "tp": tp, "members": members,
                                                   "models": sorted({m.model_id for m in ms}),
                                                   "capacity": max(m.capacity for m in ms)},
                            "models": [(m.model_id, m.cfg, m.max_model_len) for m in ms]})
        return out

    def run(self) -> dict:
        t0 = time.time()
        status = "ok"
        seen = []
        try:
            host = rocm_enum.host_id()
            for d in self.local_devices():
                self.store.upsert_device(d["id"], d["name"], d["platform"], d["arch"],
                                         d["host"], d["tags"], "online", merge_tags=True)
                seen.append(d["id"])
                present = []
                for mid, cfg, mml in d["models"]:
                    rec = model_record(mid, cfg)
                    self.store.upsert_model(mid, **rec)
                    self.store.upsert_device_model(d["id"], mid, True,
                                                   max_context_k=mml // 1024)
                    present.append(mid)
                self.store.mark_absent_models(d["id"], present)
            gone = []
            for d in self.store.list_devices():
                if d.get("host") == host and d["id"] not in seen and d.get("status") == "online" \
                        and (d.get("tags") or {}).get("rocm"):
                    self.store.set_device_status(d["id"], "offline",
                                                 {"last_error": "device disappeared",
                                                  "last_error_at": time.time()})
                    self.store.release_device_leases(d["id"])
                    gone.append(d["id"])
            peers = self._poll_peers()
            res = {"devices": seen, "offline": gone, "peers": peers}
        except Exception as e:  # discovery must not take the core down
            log.exception("discovery failed")
            status = "error"
            res = {"error": str(e)}
        dt = time.time() - t0
        if self.metrics is not None:
            self.metrics.discovery_runs.labels(status).inc()
            self.metrics.discovery_duration.observe(dt)
            self.metrics.devices_online.set(sum(1 for d in self.store.list_devices()
                                                if d.get("status") == "online"))
        with self._lock:
            self._last_run = time.time()
            self.last_result = res
        return res

    # ------------------------------------------------------------- mesh --
    @staticmethod
    def _ports() -> list[int]:
        return [int(p) for p in os.environ.get("LMX_PEER_PORTS", "8080").split(",") if p.strip()]

    def _tailscale_status(self) -> dict | None:
        """``tailscale status --json`` (LMX_TAILSCALE_STATUS_FILE overrides it
        with a saved status document, used by tests and air-gapped setups)."""
        path = os.environ.get("LMX_TAILSCALE_STATUS_FILE", "")
        try:
            if path:
                with open(path) as f:
                    return json.load(f)
            if os.environ.get("LMX_DISCOVERY_TAILSCALE", "1") == "0":
                return None
            exe = shutil.which("tailscale")
            if not exe:
                return None
            out = subprocess.run([exe, "status", "--json"], capture_output=True, timeout=10,
                                 check=True).stdout
            return json.loads(out)
        except (OSError, ValueError, subprocess.SubprocessError) as e:
            log.warning("tailscale status unavailable: %s", e)
            return None

    def _peer_urls(self) -> tuple[list[str], list[str]]:
        """(urls to probe, hosts the mesh reports offline)."""
        urls = [p.strip().rstrip("/") for p in os.environ.get("LMX_PEER_NODES", "").split(",")
                if p.strip()]
        extra = os.environ.get("DISCOVERY_EXTRA_ENDPOINTS") or os.environ.get(
            "OLLAMA_EXTRA_ENDPOINTS", "")
        for ep in (e.strip() for e in extra.split(",")):
            if ep:
                urls.append(ep.rstrip("/") if "://" in ep else "http://" + ep)
        offline_hosts: list[str] = []
        st = self._tailscale_status()
        if st:
            for node in (st.get("Peer") or {}).values():
                name = (node.get("DNSName") or "").rstrip(".") or node.get("HostName", "")
                ips = node.get("TailscaleIPs") or []
                addr = ips[0] if ips else name       # mesh IPs route without MagicDNS
                if not addr:
                    continue
                if not node.get("Online", False):
                    offline_hosts += [h for h in (name, node.get("HostName", "")) if h]
                    continue
                urls += [f"http://{addr}:{p}" for p in self._ports()]
        if os.environ.get("DISCOVERY_SCAN_SUBNETS", "0") == "1":
            hosts: list[str] = []
            for cidr in os.environ.get("DISCOVERY_SUBNETS", "").split(","):
                if not cidr.strip():
                    continue
                try:
                    net = ipaddress.ip_network(cidr.strip(), strict=False)
                except ValueError:
                    log.warning("bad subnet %r", cidr)
                    continue
                hs = list(net.hosts()) or [net.network_address]
                hosts += [str(h) for h in hs[:1024 - len(hosts)]]
                if len(hosts) >= 1024:
                    break
            urls += [f"http://{h}:{p}" for h in hosts for p in self._ports()]
        return list(dict.fromkeys(urls)), offline_hosts

    @staticmethod
    def _probe(url: str) -> dict | None:
        try:
            with urllib.request.urlopen(url + "/v1/discovery/local", timeout=2) as r:
                data = json.loads(r.read())
            return data if isinstance(data, dict) and "devices" in data else None
        except Exception:
            return None

    def _take_offline(self, pred, reason: str) -> None:
        for d in self.store.list_devices():
            if d.get("status") == "online" and pred(d):
                self.store.set_device_status(d["id"], "offline",
                                             {"last_error": reason, "last_error_at": time.time()})
                self.store.release_device_leases(d["id"])

    def _poll_peers(self) -> list[str]:
        urls, offline_hosts = self._peer_urls()
        if offline_hosts:
            dead = set(offline_hosts)
            self._take_offline(lambda d: d.get("host") in dead, "mesh reports node offline")
        if not urls:
            return []
        with ThreadPoolExecutor(max_workers=min(32, len(urls))) as ex:
            results = list(ex.map(self._probe, urls))
        ok = []
        me = rocm_enum.host_id()
        for url, data in zip(urls, results):
            if data is None:
                self._take_offline(lambda d, u=url: (d.get("tags") or {}).get("peer") == u,
                                   "peer unreachable")
                continue
            for d in data.get("devices", []):
                if d.get("host") == me:
                    continue          # our own core answering through the mesh
                tags = dict(d.get("tags") or {})
                tags.update(peer=url, engine_addr=url)
                self.store.upsert_device(d["id"], d.get("name", ""), d.get("platform", "rocm"),
                                         d.get("arch", ""), d.get("host", ""), tags, "online")
                for mid in tags.get("models", []):
                    self.store.upsert_model(mid, **model_record(mid))
                    self.store.upsert_device_model(d["id"], mid, True)
            ok.append(url)
        return ok
