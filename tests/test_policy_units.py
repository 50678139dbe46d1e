"""Unit-level parity with the reference's Go tests:
core/internal/routing/router_test.go (token estimate, message flattening,
payload model/device parsing, circuit-breaker state machine with a moved
clock, quality tables), core/internal/limits/limits_test.go (derived limit
thresholds, string lists) and core/internal/api/helpers_test.go (JSON / error
contract / SSE framing / number coercion); plus the discovery name heuristics
(core/internal/discovery/discovery.go:482-649) and the HBM admission branch."""
import json

import pytest

from llm_mcp_amd.api import helpers
from llm_mcp_amd.models.tokenizer import messages_to_prompt
from llm_mcp_amd.policy import inference as inf
from llm_mcp_amd.policy import limits as lim
from llm_mcp_amd.policy import router as rt
from llm_mcp_amd.policy.circuit import CircuitBreaker
from llm_mcp_amd.store.memory import MemoryStore


# ---------------------------------------------------------------- tokens ----
def test_estimate_tokens_prompt_only_and_floor():
    assert rt.estimate_tokens("x" * 4000) == 1000
    assert rt.estimate_tokens("") == 256                 # floor for empty input
    assert rt.estimate_tokens("hello") == 256


def test_estimate_tokens_messages_and_mixed():
    msgs = [{"role": "user", "content": "Hello"}, {"role": "assistant", "content": "Hi there"}]
    assert rt.estimate_tokens(messages=msgs) == 256
    assert rt.estimate_tokens("a" * 2000, [{"role": "user", "content": "b" * 2000}]) == 1000
    assert rt.estimate_tokens("a" * 400000) == 100000


def test_messages_to_prompt():
    assert messages_to_prompt([{"role": "user", "content": "Hello"},
                               {"role": "assistant", "content": "Hi"}]) == "user: Hello\nassistant: Hi"
    assert messages_to_prompt([]) == ""
    assert messages_to_prompt(None) == ""
    assert messages_to_prompt([{"role": "", "content": ""},
                               {"role": "user", "content": "test"}]) == "user: test"


@pytest.mark.parametrize("payload,expect", [
    ({"model": "qwen3:1.7b", "device_id": "dev-1"}, ("qwen3:1.7b", "dev-1")),
    ({"model": "llama3"}, ("llama3", "")),
    ({}, ("", "")),
    ("{not json", ("", "")),
    (None, ("", "")),
    ({"model": " qwen3 ", "device_id": " dev-2 "}, ("qwen3", "dev-2")),
    ({"model": 5, "device_id": ["x"]}, ("", "")),
])
def test_parse_payload_model_device(payload, expect):
    assert rt.parse_payload_model_device(payload) == expect


# --------------------------------------------------------------- circuit ----
class Clock:
    def __init__(self):
        self.t = 1000.0

    def __call__(self):
        return self.t


def test_circuit_initial_and_one_failure():
    cb = CircuitBreaker(clock=Clock())
    assert not cb.is_degraded("gpu0") and cb.status("gpu0") == "ok"
    cb.record("gpu0", False)
    assert not cb.is_degraded("gpu0") and cb.status("gpu0") == "ok"
    assert cb.snapshot()["gpu0"]["failures"] == 1


def test_circuit_three_failures_degrade_success_resets():
    cb = CircuitBreaker(clock=Clock())
    for _ in range(3):
        cb.record("gpu0", False)
    assert cb.is_degraded("gpu0") and cb.status("gpu0") == "degraded"
    cb.record("gpu0", True)
    assert not cb.is_degraded("gpu0") and "gpu0" not in cb.snapshot()


def test_circuit_trips_count_transitions():
    cb = CircuitBreaker(clock=Clock())
    for _ in range(5):
        cb.record("gpu0", False)
    assert cb.trips == {"gpu0": 1}          # one ok -> degraded transition
    cb.record("gpu0", True)
    for _ in range(3):
        cb.record("gpu0", False)
    assert cb.trips == {"gpu0": 2}


def test_circuit_probe_after_five_minutes():
    clk = Clock()
    cb = CircuitBreaker(clock=clk)
    for _ in range(3):
        cb.record("gpu0", False)
    clk.t += 299
    assert cb.status("gpu0") == "degraded"
    clk.t += 2
    assert cb.status("gpu0") == "probe" and not cb.is_degraded("gpu0")
    # the reference's own test writes the state with a skewed clock (DegradedAt = now - 6 min)
    cb._set("gpu1", 3, clk.t - 360)
    assert cb.status("gpu1") == "probe"
    cb.record("gpu1", False)   # a failed probe re-arms the degraded window
    assert cb.status("gpu1") == "degraded"


def test_circuit_empty_device_and_isolation():
    cb = CircuitBreaker(clock=Clock())
    cb.record("", False)
    assert cb.snapshot() == {}
    for _ in range(3):
        cb.record("gpu0", False)
    cb.record("gpu1", False)
    assert cb.is_degraded("gpu0") and not cb.is_degraded("gpu1")


def test_quality_tables_cover_every_quality():
    q = {"turbo", "economy", "standard", "premium", "ultra", "max"}
    assert set(rt.QUALITY_TIERS) == q
    assert set(rt.CLOUD_FALLBACK_TIERS) == q
    assert set(rt.QUALITY_TIMEOUTS) == q
    assert all(len(v) == 3 for v in rt.QUALITY_TIERS.values())   # <=4K, 4-32K, >32K
    assert rt.QUALITY_TIMEOUTS["turbo"] == 15 and rt.QUALITY_TIMEOUTS["max"] == 180


# ---------------------------------------------------------------- limits ----
def test_derive_limits_from_ram_thresholds():
    s = lim.derive_device_limits({"ram_gb": 4})
    assert (s["max_params_b"], s["max_context_k"], s["max_size_gb"]) == (5.0, 4096, 3.2)
    s = lim.derive_device_limits({"ram_gb": 16})
    assert (s["max_params_b"], s["max_context_k"]) == (12.0, 8192)
    s = lim.derive_device_limits({"ram_gb": 64})
    assert (s["max_params_b"], s["max_context_k"]) == (48.0, 16384)


def test_derive_limits_vram_priority_presets_and_none():
    assert lim.derive_device_limits({"vram_gb": 8, "ram_gb": 32})["max_params_b"] == 5.0
    s = lim.derive_device_limits({"ram_gb": 8, "max_params_b": 99, "max_size_gb": 99,
                                  "max_context_k": 99999})
    assert (s["max_params_b"], s["max_size_gb"], s["max_context_k"]) == (99, 99, 99999)
    s = lim.derive_device_limits({})
    assert all(s.get(k) is None for k in ("max_params_b", "max_size_gb", "max_context_k"))


def test_derive_limits_hbm_and_tp_groups():
    s = lim.derive_device_limits({"hbm_gb": 288})
    assert s["max_params_b"] == 122.0        # 0.85 * 288 GB / 2 B per bf16 param
    assert s["vram_gb"] == 288
    s8 = lim.derive_device_limits({"hbm_gb": 288, "tp": 8})
    assert s8["max_params_b"] > 900 and s8["max_size_gb"] == pytest.approx(1958.4)


def test_string_lists():
    assert lim._list('["a","b"]') == ["a", "b"]
    assert lim._list(["a", " ", " b "]) == ["a", "b"]
    assert lim._list("") == [] and lim._list(None) == [] and lim._list("{bad") == []


def test_model_allowed_reasons():
    st = MemoryStore()
    st.upsert_device("gpu0", name="gpu0")
    st.upsert_model("llama-3-8b", kind="chat", params_b=8.0, size_gb=16.0, context_k=8)
    st.upsert_model("mystery", kind="chat")
    st.upsert_device_model("gpu0", "llama-3-8b", True)
    st.upsert_device_model("gpu0", "mystery", True)
    assert lim.model_allowed(st, "gpu0", "nope") == (False, "model_not_on_device")
    assert lim.model_allowed(st, "gpu0", "llama-3-8b") == (True, "")
    st.upsert_device_limits("gpu0", {"max_params_b": 5})
    assert lim.model_allowed(st, "gpu0", "llama-3-8b") == (False, "model_params_too_large")
    assert lim.model_allowed(st, "gpu0", "mystery", strict=False) == (True, "")
    assert lim.model_allowed(st, "gpu0", "mystery", strict=True) == (False, "model_params_unknown")
    st.upsert_device_limits("gpu0", {"allow_models": ["other"]})
    assert lim.model_allowed(st, "gpu0", "llama-3-8b") == (False, "model_not_in_allowlist")
    st.upsert_device_limits("gpu0", {"deny_models": ["llama-3-8b"]})
    assert lim.model_allowed(st, "gpu0", "llama-3-8b") == (False, "model_denied")
    st.upsert_device_model("gpu0", "llama-3-8b", False)
    assert lim.model_allowed(st, "gpu0", "llama-3-8b") == (False, "model_not_available")


def test_device_limit_specs_from_env(tmp_path):
    specs, default = lim.load_device_limit_specs(
        {"DEVICE_LIMITS_JSON": json.dumps({"*": {"ram_gb": 8}, "gpu0": {"hbm_gb": 288}})})
    assert default == {"ram_gb": 8} and specs == {"gpu0": {"hbm_gb": 288}}
    f = tmp_path / "limits.json"
    f.write_text(json.dumps({"gpu1": {"max_params_b": 70}}))
    specs, default = lim.load_device_limit_specs({"DEVICE_LIMITS_FILE": str(f)})
    assert specs == {"gpu1": {"max_params_b": 70}} and default is None
    assert lim.load_device_limit_specs({}) == ({}, None)


# ------------------------------------------------------------- discovery ----
@pytest.mark.parametrize("raw,expect", [("8B", 8.0), ("137M", 0.137), ("1.5b", 1.5),
                                        ("500K", 0.0005), ("", None), (None, None), ("xB", None)])
def test_parse_params_b(raw, expect):
    got = inf.parse_params_b(raw)
    assert got == (pytest.approx(expect) if expect is not None else None)


@pytest.mark.parametrize("b,name,tier", [(0.5, "qwen3:0.6b", "tiny"), (1.2, "x", "tiny"),
                                         (1.7, "x", "small"), (3.0, "x", "medium"),
                                         (8.0, "llama3", "large"), (70.0, "llama3:70b", "xl"),
                                         (0.137, "nomic-embed-text", "embed"), (None, "x", "")])
def test_infer_tier(b, name, tier):
    assert inf.infer_tier(b, name) == tier


def test_infer_thinking_context_kind():
    assert inf.infer_thinking("qwen3:8b") and inf.infer_thinking("deepseek-r1:7b")
    assert not inf.infer_thinking("llama3.2:3b")
    assert inf.infer_context_k("qwen2.5:7b") == 32 and inf.infer_context_k("llama3.2:3b") == 128
    assert inf.infer_context_k("tinyllama") == 2 and inf.infer_context_k("unknown") == 4
    assert inf.infer_kind("nomic-embed-text") == "embed" and inf.infer_kind("llama3") == "chat"


# --------------------------------------------------------------- helpers ----
def test_write_json_and_error_contract():
    r = helpers.write_json(200, {"status": "ok"})
    assert r.status == 200 and r.content_type == "application/json"
    assert json.loads(r.text) == {"status": "ok"}
    r = helpers.write_error(404, "not_found", "job not found")
    assert r.status == 404 and json.loads(r.text) == {"error": "not_found",
                                                      "message": "job not found"}
    r = helpers.write_error(500, "db_error", "boom", "details here")
    assert json.loads(r.text) == {"error": "db_error", "message": "boom",
                                  "details": "details here"}


def test_sse_frame_format():
    assert helpers.sse_frame("status", {"a": 1}) == b'event: status\ndata: {"a":1}\n\n'
    assert helpers.sse_frame(None, "[DONE]") == b"data: [DONE]\n\n"


@pytest.mark.parametrize("v,expect", [(3.0, 3), (7, 7), ("42", 42), ("2.5", 2), (None, None),
                                      ("abc", None), (True, None)])
def test_to_int(v, expect):
    assert helpers.to_int(v) == expect


def test_clock_snapshot_parser():
    """bench.py records sclk / mclk / power / temperature per card at the start
    and end of the timed region (rocm-smi --json, parsed tolerantly)."""
    from llm_mcp_amd.devices.rocm_enum import parse_clock_snapshot
    data = {"card0": {"sclk clock level:": "1", "mclk clock level:": "0",
                      "sclk clock speed:": "(2100Mhz)", "mclk clock speed:": "(1900Mhz)",
                      "Current Socket Graphics Package Power (W)": "1012.0",
                      "Max Graphics Package Power (W)": "1400.0",
                      "Temperature (Sensor junction) (C)": "71.0",
                      "Temperature (Sensor memory) (C)": "60.0"},
            "system": {"Driver version": "x"}}
    got = parse_clock_snapshot(data)
    assert got == {"card0": {"sclk_mhz": 2100.0, "mclk_mhz": 1900.0, "power_w": 1012.0,
                             "power_cap_w": 1400.0,
                             "temp_c": {"junction": 71.0, "memory": 60.0}}}
