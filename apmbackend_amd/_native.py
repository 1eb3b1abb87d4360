"""Loader for the in-tree native extension (``_apm_native*.so``).

``torch`` is imported first on purpose: the extension links ``libamdhip64.so.7`` and must bind
to the HIP runtime torch already loaded, so device pointers, streams and RCCL communicators are
shared by one runtime in the process.

On a machine with a GPU the extension is mandatory: ``load()`` raises instead of falling back,
so a GPU test can never silently pass on a CPU path.
"""
from __future__ import annotations

import glob
import importlib
import os

import torch  # noqa: F401  (see module docstring)

_mod = None


def _so_present() -> bool:
    here = os.path.dirname(os.path.abspath(__file__))
    return bool(glob.glob(os.path.join(here, "_apm_native*.so")))


def load(build_if_missing: bool = True):
    global _mod
    if _mod is not None:
        return _mod
    if not _so_present() and build_if_missing:
        from .build_native import build
        build(verbose=False)
    try:
        mod = importlib.import_module("apmbackend_amd._apm_native")
    except ImportError as e:  # pragma: no cover - exercised only on broken installs
        raise RuntimeError(
            "apmbackend_amd native extension is missing or failed to load; run "
            "`python -m apmbackend_amd.build_native` (hipcc, gfx950)") from e
    check_provenance(mod)
    _mod = mod
    return _mod


def check_provenance(mod, strict=None):
    """The .so carries the sha256 of the csrc/ tree it was linked from.  A mismatch with the
    sources next to it (a stale build shipped with a newer tree) is an error on a GPU box -- the
    tests and the bench must run the code at HEAD -- and a warning elsewhere.  APM_ALLOW_STALE_NATIVE=1
    downgrades it (A/B experiments with a deliberately old build)."""
    from .build_native import CSRC, csrc_hash
    embedded = mod.csrc_hash() if hasattr(mod, "csrc_hash") else "<none>"
    if not os.path.isdir(CSRC):  # an installed package without sources: nothing to compare
        return embedded
    here = csrc_hash()
    if embedded == here:
        return embedded
    msg = (f"stale native extension: {mod.__file__} was built from csrc hash {embedded}, the sources here "
           f"hash to {here}; rebuild with `python -m apmbackend_amd.build_native`")
    if strict is None:
        strict = torch.cuda.is_available() and os.environ.get("APM_ALLOW_STALE_NATIVE") != "1"
    if strict:
        raise RuntimeError(msg)
    import warnings
    warnings.warn(msg)
    return embedded


def gpu_available() -> bool:
    return torch.cuda.is_available()
