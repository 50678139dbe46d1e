"""Multi-node discovery sources (reference discovery.go:88-174 Tailscale mesh,
:755-877 subnet scan / extra endpoints, offline_handler.go lease release)
against a stub peer core serving ``/v1/discovery/local``."""
import json
import threading
from http.server import BaseHTTPRequestHandler, HTTPServer

import pytest

from llm_mcp_amd.devices.discovery import DiscoveryRunner
from llm_mcp_amd.store.memory import MemoryStore

PEER_DEV = {"id": "peerhost:gpu0", "name": "MI355X", "platform": "rocm", "arch": "gfx950",
            "host": "peerhost", "tags": {"engine": True, "models": ["llama-3-8b"]}}


@pytest.fixture
def peer():
    class H(BaseHTTPRequestHandler):
        def do_GET(self):
            if self.path != "/v1/discovery/local":
                self.send_response(404)
                self.end_headers()
                return
            body = json.dumps({"devices": [PEER_DEV]}).encode()
            self.send_response(200)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass

    srv = HTTPServer(("127.0.0.1", 0), H)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    yield srv.server_address[1]
    srv.shutdown()


@pytest.fixture(autouse=True)
def _env(monkeypatch):
    for k in ("LMX_PEER_NODES", "DISCOVERY_EXTRA_ENDPOINTS", "OLLAMA_EXTRA_ENDPOINTS",
              "DISCOVERY_SCAN_SUBNETS", "DISCOVERY_SUBNETS", "LMX_TAILSCALE_STATUS_FILE"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("LMX_DISCOVERY_TAILSCALE", "0")
    monkeypatch.setenv("LMX_FAKE_GPUS", "1:288")
    monkeypatch.setenv("LMX_NODE_ID", "node1")


def _online(store):
    return {d["id"] for d in store.list_devices() if d["status"] == "online"}


def test_tailscale_peers_and_offline_nodes(peer, tmp_path, monkeypatch):
    st = MemoryStore()
    # a node the mesh will report offline, holding a running lease
    st.upsert_device("deadhost:gpu0", "MI355X", "rocm", "gfx950", "deadhost", {}, "online")
    jid = st.submit_job("k", {"device_id": "deadhost:gpu0"})
    assert st.claim_job("w", [], 60, "deadhost:gpu0")["id"] == jid
    status = {"Self": {"HostName": "node1", "Online": True},
              "Peer": {"a": {"HostName": "peerhost", "DNSName": "", "Online": True,
                             "TailscaleIPs": ["127.0.0.1"]},
                       "b": {"HostName": "deadhost", "DNSName": "deadhost.tail.ts.net.",
                             "Online": False, "TailscaleIPs": ["100.64.0.9"]}}}
    f = tmp_path / "ts.json"
    f.write_text(json.dumps(status))
    monkeypatch.setenv("LMX_TAILSCALE_STATUS_FILE", str(f))
    monkeypatch.setenv("LMX_PEER_PORTS", str(peer))
    res = DiscoveryRunner(st).run()
    assert res["peers"] == [f"http://127.0.0.1:{peer}"]
    on = _online(st)
    assert "peerhost:gpu0" in on and "node1:gpu0" in on and "deadhost:gpu0" not in on
    assert st.get_job(jid)["lease_until"] is None          # reclaimable at once
    d = st.get_device("peerhost:gpu0")
    assert d["tags"]["engine_addr"] == f"http://127.0.0.1:{peer}"


def test_extra_endpoints_subnet_scan_and_unreachable(peer, monkeypatch):
    st = MemoryStore()
    monkeypatch.setenv("OLLAMA_EXTRA_ENDPOINTS", f"127.0.0.1:{peer}")
    assert DiscoveryRunner(st).run()["peers"] == [f"http://127.0.0.1:{peer}"]
    assert "peerhost:gpu0" in _online(st)

    st2 = MemoryStore()
    monkeypatch.delenv("OLLAMA_EXTRA_ENDPOINTS")
    monkeypatch.setenv("DISCOVERY_SCAN_SUBNETS", "1")
    monkeypatch.setenv("DISCOVERY_SUBNETS", "127.0.0.1/32")
    monkeypatch.setenv("LMX_PEER_PORTS", f"{peer},1")       # port 1: nothing listens
    assert DiscoveryRunner(st2).run()["peers"] == [f"http://127.0.0.1:{peer}"]
    assert "peerhost:gpu0" in _online(st2)

    # the peer goes away: its devices go offline on the next run
    monkeypatch.setenv("DISCOVERY_SUBNETS", "")
    monkeypatch.setenv("LMX_PEER_NODES", f"http://127.0.0.1:{peer}")
    r = DiscoveryRunner(st2)
    r._probe = staticmethod(lambda url: None)
    r.run()
    assert "peerhost:gpu0" not in _online(st2)
