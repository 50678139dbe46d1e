import pytest

from llm_mcp_amd import settings


def test_settings_types_defaults_and_validation(monkeypatch):
    assert settings.get("WORKER_LEASE_SECONDS") == 60
    monkeypatch.setenv("WORKER_LEASE_SECONDS", "30")
    assert settings.get("WORKER_LEASE_SECONDS") == 30
    monkeypatch.setenv("LMX_TP", "eight")
    with pytest.raises(settings.SettingsError):
        settings.validate()
    monkeypatch.delenv("LMX_TP")
    monkeypatch.setenv("LLM_MCP_VERSION", "9.9")
    assert settings.get("CORE_VERSION") == "9.9"
    monkeypatch.setenv("DB_DSN", "postgres://u:secret@h/db")
    t = settings.table()
    assert "secret" not in t and "`DB_DSN`" in t


def test_every_env_read_in_the_package_is_registered():
    """Keeps the settings table the single documented source of env vars."""
    import pathlib
    import re
    root = pathlib.Path(settings.__file__).parent
    names = set()
    for f in root.rglob("*.py"):
        names |= set(re.findall(r'environ(?:\.get)?\(\s*"([A-Z][A-Z0-9_]+)"', f.read_text()))
        names |= set(re.findall(r'environ\[\s*"([A-Z][A-Z0-9_]+)"\s*\]', f.read_text()))
    launcher = {"RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR",
                "HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "PGUSER", "PGPASSWORD", "HIPCC",
                "CXX", "LMX_SAN_CXX", "REPORT_CHAT_ID", "LLM_MCP_VERSION", "OPENAI_MODEL",
                "OPENROUTER_MODEL", "LMX_FAULT_HANG_S", "LMX_HTTP_HOST", "LMX_HTTP_PORT"}
    missing = sorted(n for n in names - launcher if n not in settings._BY_NAME)
    assert not missing, missing


def test_debug_sync_wrapper_names_the_faulting_kernel(monkeypatch):
    import torch

    from llm_mcp_amd import ops

    class Mod:
        answer = 42

        @staticmethod
        def good(x):
            return x + 1

        @staticmethod
        def bad():
            return None

    calls = []
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)

    def sync():
        calls.append(1)
        if len(calls) == 2:
            raise RuntimeError("HIP error: an illegal memory access")
    monkeypatch.setattr(torch.cuda, "synchronize", sync)
    k = ops._SyncedKernels(Mod())
    assert k.answer == 42 and k.good(1) == 2 and calls == [1]
    try:
        k.bad()
        raise AssertionError("expected the fault")
    except RuntimeError as e:
        assert "lmx kernel bad faulted" in str(e)
