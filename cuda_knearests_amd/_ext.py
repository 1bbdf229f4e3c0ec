"""Loader for the in-tree native extension (``_C``) and the standalone C library.

The extension is built by ``python -m cuda_knearests_amd._build`` (``__graft_entry__.build``)
and lives next to this file so it is visible to the GPU box snapshot. It is never silently
replaced by a Python fallback: GPU entry points raise if it is missing.
"""
from __future__ import annotations

import ctypes
import importlib
import os
from pathlib import Path

_HERE = Path(__file__).resolve().parent
_C = None
_ERR: Exception | None = None


def load():
    """Return the ``_C`` module (building it first if the .so is absent and KN_AUTOBUILD=1)."""
    global _C, _ERR
    if _C is not None:
        return _C
    import torch  # noqa: F401  (libtorch / torch's HIP runtime must be loaded first)

    name = "cuda_knearests_amd._C_checked" if os.environ.get("KN_CHECKED") == "1" else "cuda_knearests_amd._C"
    if os.environ.get("KN_C_VARIANT"):  # A/B of compile-time variants (_build.build_variant)
        name = "cuda_knearests_amd._C_" + os.environ["KN_C_VARIANT"]
    try:
        _C = importlib.import_module(name)
    except ImportError as e:  # pragma: no cover - exercised only without a build
        if os.environ.get("KN_AUTOBUILD", "1") == "1":
            from . import _build

            _build.build(verbose=False)
            _C = importlib.import_module(name)
        else:
            _ERR = e
            raise RuntimeError(
                "cuda_knearests_amd native extension is not built; run "
                "`python -m cuda_knearests_amd._build`"
            ) from e
    return _C


def libknearests_path() -> Path:
    return _HERE / "lib" / "libknearests.so"


def load_capi() -> ctypes.CDLL:
    """ctypes handle on the standalone C API (knearests.h)."""
    p = libknearests_path()
    if not p.exists():
        from . import _build

        _build.build(verbose=False)
    import torch  # noqa: F401  share torch's HIP runtime (same soname) when both are used

    return ctypes.CDLL(str(p))
