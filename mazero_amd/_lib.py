"""Loader of the product library mazero_amd/_build/libmzmcts.so.

There is no fallback: if the HIP library is missing or cannot be loaded, this raises.  torch is
imported first when available so that the HIP runtime torch ships (libamdhip64.so.7, same
soname) is the one the library binds to -- one HIP runtime per process.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

from . import _capi
from .build import LIB, LIB_STAMPS

ABI = 2  # MZ_ABI_VERSION of include/mzmcts.h
_lock = threading.Lock()
_lib = None


def load() -> C.CDLL:
    """The product library; MZ_STAMPS=1 in the environment selects the diagnostic build
    (MZ_LIB_OVERRIDE=<path> loads an experiment build of the same source instead)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = LIB_STAMPS if os.environ.get("MZ_STAMPS") == "1" else LIB
        # experiment builds of the same source (scripts/, diagnostics only)
        path = os.environ.get("MZ_LIB_OVERRIDE") or path
        try:
            import torch  # noqa: F401  (plumbing: share torch's HIP runtime)
        except Exception:
            pass
        if not os.path.exists(path):
            raise RuntimeError(
                f"MI355X library not built: {path} is missing (run `python -m mazero_amd.build` "
                "or __graft_entry__.build())"
            )
        lib = _capi.bind(C.CDLL(path, mode=C.RTLD_LOCAL))
        if lib.mz_abi_version() != ABI or lib.mz_backend() != b"hip-gfx950":
            raise RuntimeError(f"{path} is not the hip-gfx950 backend of ABI {ABI}")
        _lib = lib
        return lib


def trim_caches() -> int:
    """Free the device arenas and pinned stages that destroyed handles left in the library's
    process-wide caches (mz_trim_caches, include/mzdriver.h); returns the bytes released.  A
    process that has not loaded the library has nothing cached: 0, without loading it."""
    with _lock:
        lib = _lib
    if lib is None:
        return 0
    n = C.c_int64(0)
    rc = lib.mz_trim_caches(C.byref(n))
    if rc != 0:
        raise RuntimeError(f"mz_trim_caches: {lib.mz_last_error().decode(errors='replace')}")
    return int(n.value)
