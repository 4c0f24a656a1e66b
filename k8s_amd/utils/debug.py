"""Kernel debug mode ("a HIP-side bounds/NaN checking debug mode for kernels").

GPU AddressSanitizer is not available for gfx950 work here, so the checks sit at the op boundary:

* ``K8S_AMD_CHECK_NUMERICS=1`` -- after every call into the native extension, every floating tensor it
  returned (or, for in-place ops that return nothing, every floating tensor argument it may have written) is
  checked for NaN / +Inf; the first offender raises ``NumericsError`` naming the op and the argument.
  ``-Inf`` is allowed (attention uses it as the masked-row log-sum-exp).
* ``K8S_AMD_SYNC_OPS=1`` -- synchronise the device after every native op, so an asynchronous fault
  (out-of-bounds access, illegal instruction) is reported against the op that launched it instead of some
  later, unrelated call.

Both wrap the extension module returned by ``k8s_amd.ops._ext.load()``; with neither set the raw module is
used and there is no overhead.
"""
from __future__ import annotations

import functools
import os

import torch


class NumericsError(RuntimeError):
    pass


def enabled_flags():
    return (os.environ.get("K8S_AMD_CHECK_NUMERICS", "0") == "1", os.environ.get("K8S_AMD_SYNC_OPS", "0") == "1")


def _bad(t: torch.Tensor) -> int:
    if not (torch.is_tensor(t) and t.is_floating_point() and t.numel()):
        return 0
    return int(torch.isnan(t).sum().item() + torch.isposinf(t).sum().item())


def _tensors(obj, prefix):
    if torch.is_tensor(obj):
        yield prefix, obj
    elif isinstance(obj, (list, tuple)):
        for i, o in enumerate(obj):
            yield from _tensors(o, "%s[%d]" % (prefix, i))


class CheckedExtension:
    """Proxy over the native module: every callable attribute is wrapped with the enabled checks."""

    def __init__(self, mod, check_numerics: bool, sync: bool):
        self._mod = mod
        self._check = check_numerics
        self._sync = sync
        self._cache = {}

    def __getattr__(self, name):
        attr = getattr(self._mod, name)
        if not callable(attr):
            return attr
        fn = self._cache.get(name)
        if fn is None:
            fn = self._wrap(name, attr)
            self._cache[name] = fn
        return fn

    def _wrap(self, name, f):
        @functools.wraps(f)
        def call(*args, **kwargs):
            try:
                out = f(*args, **kwargs)
                if self._sync and torch.cuda.is_available():
                    torch.cuda.synchronize()
            except RuntimeError as e:
                raise RuntimeError("k8s_amd native op %s failed: %s" % (name, e)) from e
            if self._check:
                targets = list(_tensors(out, "out")) if out is not None else []
                if not targets:  # in-place op: the outputs are among the arguments
                    targets = list(_tensors(list(args), "arg"))
                for label, t in targets:
                    n = _bad(t)
                    if n:
                        raise NumericsError("k8s_amd native op %s: %s %s %s has %d NaN/+Inf element(s)"
                                            % (name, label, tuple(t.shape), t.dtype, n))
            return out

        return call


def maybe_wrap(mod):
    check, sync = enabled_flags()
    if not (check or sync):
        return mod
    return CheckedExtension(mod, check, sync)
