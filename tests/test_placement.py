"""`serve` placement planner (SURVEY §5.6 LMX_MODEL_REGISTRY): which worker
process serves which model / TP group on which GPUs."""
import pytest

from llm_mcp_amd.__main__ import plan_placement


def test_default_dp_and_embed_subset():
    p = plan_placement([0, 1, 2], "llama-3-8b", "nomic-embed-text", [1])
    assert [w["gpus"] for w in p] == [[0], [1], [2]]
    assert all(w["chat"] == "llama-3-8b" and w["tp"] == 1 for w in p)
    assert [w["embed"] for w in p] == ["", "nomic-embed-text", ""]


def test_default_tp_groups():
    p = plan_placement(list(range(8)), "llama-3-70b", tp=4)
    assert [w["gpus"] for w in p] == [[0, 1, 2, 3], [4, 5, 6, 7]]
    assert all(w["tp"] == 4 and w["chat"] == "llama-3-70b" for w in p)
    with pytest.raises(ValueError):
        plan_placement([0, 1, 2], "llama-3-70b", tp=2)


def test_registry_mixed_node():
    p = plan_placement(list(range(8)), registry=(
        "0-3:llama-3-8b; 4-7:tp4:llama-3-70b; 0,1:embed:nomic-embed-text; 2:embed:mxbai"))
    singles = [w for w in p if w["tp"] == 1]
    assert [w["gpus"][0] for w in singles] == [0, 1, 2, 3]
    assert [w["embed"] for w in singles] == ["nomic-embed-text", "nomic-embed-text", "mxbai", ""]
    assert all(w["chat"] == "llama-3-8b" for w in singles)
    grp = [w for w in p if w["tp"] > 1]
    assert grp == [{"gpus": [4, 5, 6, 7], "tp": 4, "chat": "llama-3-70b", "embed": ""}]
    # embed-only GPU
    p = plan_placement([0, 1], registry="0:llama-3-8b;1:embed:nomic-embed-text")
    assert p[1] == {"gpus": [1], "tp": 1, "chat": "", "embed": "nomic-embed-text"}


@pytest.mark.parametrize("reg", [
    "0-3:llama-3-8b;2:qwen2.5-7b",              # two chat engines on GPU 2
    "0-3:tp4:llama-3-70b;1:embed:nomic",         # embedder on a TP rank
    "0:llama-3-8b;0-1:tp2:llama-3-70b",          # chat engine + TP rank
    "0-2:tp2:llama-3-70b",                       # 3 GPUs into TP=2
    "9:llama-3-8b",                              # GPU not served
    "0:foo:llama-3-8b",                          # unknown role
    "llama-3-8b",                                # no GPU set
])
def test_registry_rejects_conflicts(reg):
    with pytest.raises(ValueError):
        plan_placement(list(range(4)), registry=reg)
