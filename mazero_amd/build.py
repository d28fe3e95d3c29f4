"""Build the product HIP library in-tree: mazero_amd/_build/libmzmcts.so (gfx950).

    python -m mazero_amd.build          # or __graft_entry__.build()

Flags that matter for parity with the reference CPU tree (SURVEY.md §7 hard part 3):
  -ffp-contract=off                          no FMA contraction of `a*b + c` (the reference's x86-64
                                             -O2 build has no FMA instructions)
  -fhip-fp32-correctly-rounded-divide-sqrt   IEEE f32 division (value = ws/tw, normalisation)
  no -ffast-math, no denormal flushing
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRCS = [os.path.join(HERE, "csrc", f) for f in ("mzmcts.hip", "mzdriver.hip", "mzconsume.hip")]
SRC = SRCS[0]
OUT_DIR = os.path.join(HERE, "_build")
LIB = os.path.join(OUT_DIR, "libmzmcts.so")
LIB_STAMPS = os.path.join(OUT_DIR, "libmzmcts_stamps.so")  # diagnostic build (MZ_STAMPS=1)
ARCH = os.environ.get("MZ_OFFLOAD_ARCH", "gfx950")

FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-shared",
    "-ffp-contract=off",
    "-fhip-fp32-correctly-rounded-divide-sqrt",
    "-fno-fast-math",
    "-Wall",
    "-Wno-unused-function",
    # the first 16 dwords of scalar kernel arguments arrive in SGPRs at wave launch
    "-mllvm",
    "-amdgpu-kernarg-preload-count=16",
]


def hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the MI355X library cannot be built")


def needs_build(lib: str = LIB) -> bool:
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    deps = [*SRCS, os.path.join(HERE, "csrc", "mz_internal.h"), os.path.join(HERE, "csrc", "mt_seed.inc"), os.path.join(HERE, "csrc", "mzhbm.inc"), os.path.join(ROOT, "include", "mzmcts.h"),
            os.path.join(ROOT, "include", "mzdriver.h"), os.path.join(ROOT, "include", "mzconsume.h"), __file__]
    return any(os.path.getmtime(p) > t for p in deps)


def build(force: bool = False, verbose: bool = True, stamps: bool = False) -> str:
    lib = LIB_STAMPS if stamps else LIB
    if not force and not needs_build(lib):
        return lib
    os.makedirs(OUT_DIR, exist_ok=True)
    tmp = lib + ".tmp"
    # MZ_STAMPS_LEVEL=2: wave 1's node updates in detail instead of the expansion's phases (k_tree)
    extra = ["-DMZ_STAMPS=" + os.environ.get("MZ_STAMPS_LEVEL", "1")] if stamps else []
    cmd = [hipcc(), *FLAGS, *extra, "-I", os.path.join(ROOT, "include"), *SRCS, "-o", tmp]
    if verbose:
        print("[mazero_amd] " + " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, lib)
    return lib


def build_all(force: bool = False, verbose: bool = True) -> None:
    build(force=force, verbose=verbose)
    build(force=force, verbose=verbose, stamps=True)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
