"""Catalogue planner: ranking rows from category listings, curated sync into
the store, retention purge (no network: catalogue JSON is synthetic, in the
shape of OpenRouter's /models response)."""
from llm_mcp_amd.planner.catalog import (RetentionPlanner, apply_curated, load_curated,
                                         rankings_from_catalog)
from llm_mcp_amd.store.memory import MemoryStore

CAT = [{"id": "a/m1", "name": "M1", "context_length": 131072,
        "pricing": {"prompt": "0.0000005", "completion": "0.0000015"},
        "architecture": {"input_modalities": ["text", "image"]},
        "supported_parameters": ["tools", "temperature"]},
       {"id": "b/m2", "name": "M2", "context_length": 32768,
        "pricing": {"prompt": "0", "completion": "0"}}]


def test_rankings_merge_categories():
    rows = rankings_from_catalog({"programming": CAT, "finance": CAT[:1]})
    assert rows["a/m1"]["category_scores"] == {"programming": 75, "finance": 75}
    assert rows["a/m1"]["price_in_1m"] == 0.5 and rows["a/m1"]["price_out_1m"] == 1.5
    assert rows["a/m1"]["supports_tools"] and rows["a/m1"]["supports_vision"]
    assert rows["b/m2"]["category_scores"] == {"programming": 75}


def test_curated_sync_and_snapshot(tmp_path):
    st = MemoryStore()
    ids = load_curated("llm_mcp_amd/config/curated_cloud_models.yaml")
    assert "z-ai/glm-4.7" in ids
    res = apply_curated(st, ["a/m1", "zz/missing"], CAT, str(tmp_path))
    assert res["synced"] == ["a/m1"] and res["missing"] == ["zz/missing"]
    assert st.get_model("a/m1")["context_k"] == 128
    assert st.get_pricing("a/m1") == (0.5, 1.5)
    assert (tmp_path / res["snapshot"].split("/")[-1]).exists()


def test_retention_planner_purges_old_finished_jobs():
    t = [1000.0]
    st = MemoryStore(clock=lambda: t[0])
    jid = st.submit_job("echo", {})
    j = st.claim_job("w", [], 30)
    st.complete_job(jid, "w", {"ok": True}, {}, j["attempt_id"])
    keep = st.submit_job("echo", {})
    t[0] += 2 * 86400
    r = RetentionPlanner(st, retention_days=1).tick()
    assert r["purged"] == 1
    assert st.get_job(jid) is None and st.get_job(keep) is not None
