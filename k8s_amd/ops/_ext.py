"""Loader for the in-tree gfx950 extension ``k8s_amd._C``.

The HIP path is the ONLY GPU path: if the extension is missing on a machine
with a GPU, every op raises instead of silently falling back to eager
PyTorch. CPU tensors use the reference implementations in
``k8s_amd.ops.reference`` (the numerics oracles the GPU tests compare
against), which keeps the CPU-only test tier meaningful.
"""
from __future__ import annotations

import importlib
import os

_C = None
_ERR = None


def load(build_if_missing: bool = False):
    """Return the compiled module, raising with a build hint if it is absent."""
    global _C, _ERR
    if _C is not None:
        return _C
    try:
        from k8s_amd.utils.debug import maybe_wrap

        _C = maybe_wrap(importlib.import_module("k8s_amd._C"))
        return _C
    except ImportError as e:  # pragma: no cover - depends on build state
        _ERR = e
        if build_if_missing or os.environ.get("K8S_AMD_AUTOBUILD") == "1":
            from k8s_amd import _build

            _build.build_kernels()
            from k8s_amd.utils.debug import maybe_wrap

            _C = maybe_wrap(importlib.import_module("k8s_amd._C"))
            return _C
        raise ImportError(
            "k8s_amd native kernels are not built (k8s_amd/_C*.so missing): run "
            "`python -m k8s_amd._build` (hipcc --offload-arch=gfx950). Original error: %s" % e
        ) from e


def available() -> bool:
    try:
        load()
        return True
    except ImportError:
        return False


def ext():
    return load()
