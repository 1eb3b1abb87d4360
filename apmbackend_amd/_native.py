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
        _mod = importlib.import_module("apmbackend_amd._apm_native")
    except ImportError as e:  # pragma: no cover - exercised only on broken installs
        raise RuntimeError(
            "apmbackend_amd native extension is missing or failed to load; run "
            "`python -m apmbackend_amd.build_native` (hipcc, gfx950)") from e
    return _mod


def gpu_available() -> bool:
    return torch.cuda.is_available()
