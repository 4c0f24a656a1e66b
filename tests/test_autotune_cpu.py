"""ops/autotune.py: the shipped gfx950 seed table and the margin a vendor candidate must win by."""
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


def test_seed_table_loaded_for_gfx950(fresh, monkeypatch):
    monkeypatch.setattr(fresh, "_arch", lambda: "gfx950")
    seed = json.load(open(os.path.join(fresh.SEED_DIR, "gfx950.json")))
    assert any(k.startswith("conv_fwd|256x56x56x64|") for k in seed)  # the ResNet-50 b256 benchmark shapes
    assert set(seed.values()) <= {"hip", "aten", "blas"}
    fresh._load_cache()
    assert all(fresh._cache[k] == v for k, v in seed.items())


def test_seed_can_be_disabled(fresh, monkeypatch):
    monkeypatch.setattr(fresh, "_arch", lambda: "gfx950")
    monkeypatch.setenv("K8S_AMD_AUTOTUNE_SEED", "0")
    fresh._load_cache()
    assert fresh._cache == {}


def test_vendor_needs_margin(fresh, monkeypatch):
    monkeypatch.setattr(fresh.torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(fresh, "_time", lambda fn, reps=5: fn())
    monkeypatch.setattr(fresh, "_arch", lambda: "")
    assert fresh.choose("op|a", [("hip", lambda: 1.0), ("aten", lambda: 0.98)]) == "hip"  # within 3 %
    assert fresh.choose("op|b", [("hip", lambda: 1.0), ("aten", lambda: 0.90)]) == "aten"
    assert fresh.choose("op|c", [("hip", lambda: 1.0), ("aten", lambda: 2.0)]) == "hip"
    # cached: the candidates are not timed again
    assert fresh.choose("op|b", [("hip", lambda: 0.1), ("aten", lambda: 9.0)]) == "aten"
    # a cached name that is no longer a candidate is re-tuned
    fresh._cache["op|d"] = "gone"
    assert fresh.choose("op|d", [("hip", lambda: 1.0), ("blas", lambda: 0.5)]) == "blas"
