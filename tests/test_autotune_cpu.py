"""ops/autotune.py: the node cache and the margin a non-default candidate must win by."""
import json
import os

import pytest

from k8s_amd.ops import autotune


@pytest.fixture
def fresh(monkeypatch):
    monkeypatch.setattr(autotune, "_cache", {})
    monkeypatch.setattr(autotune, "_loaded", False)
    monkeypatch.setenv("K8S_AMD_AUTOTUNE_CACHE", "none")
    return autotune


def test_node_cache_round_trip(fresh, monkeypatch, tmp_path):
    p = tmp_path / "cache.json"
    monkeypatch.setenv("K8S_AMD_AUTOTUNE_CACHE", str(p))
    p.write_text(json.dumps({"op|x": "b"}))
    fresh._load_cache()
    assert fresh.choices() == {"op|x": "b"}
    assert fresh.choose("op|x", [("a", lambda: 0), ("b", lambda: 0)]) == "b"


def test_no_vendor_seed_tables_ship():
    """Round 2 retired MIOpen / hipBLASLt from the dispatch: nothing may pin a vendor kernel per shape."""
    assert not os.path.exists(os.path.join(os.path.dirname(autotune.__file__), "tuned"))


def test_candidate_needs_margin(fresh, monkeypatch):
    monkeypatch.setattr(fresh.torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(fresh, "_time", lambda fn, reps=5: fn())
    assert fresh.choose("op|a", [("hip", lambda: 1.0), ("aten", lambda: 0.98)]) == "hip"  # within 3 %
    assert fresh.choose("op|b", [("hip", lambda: 1.0), ("aten", lambda: 0.90)]) == "aten"
    assert fresh.choose("op|c", [("hip", lambda: 1.0), ("aten", lambda: 2.0)]) == "hip"
    # cached: the candidates are not timed again
    assert fresh.choose("op|b", [("hip", lambda: 0.1), ("aten", lambda: 9.0)]) == "aten"
    # a cached name that is no longer a candidate is re-tuned
    fresh._cache["op|d"] = "gone"
    assert fresh.choose("op|d", [("hip", lambda: 1.0), ("blas", lambda: 0.5)]) == "blas"
