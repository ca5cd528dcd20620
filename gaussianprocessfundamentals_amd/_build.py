"""In-tree build of libgpk.so (hand-written HIP for gfx950) with hipcc.

The shared object lands next to this file so that it travels with the repository snapshot to
the GPU box; nothing is installed into site-packages and nothing is JIT-compiled at import.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
LIB_NAME = "libgpk.so"
LIB_PATH = os.path.join(HERE, LIB_NAME)
SOURCES = ("gpk_assemble.hip", "gpk_diag.hip", "gpk_potrf.hip", "gpk_approx.hip", "gpk_eig.hip", "gpk_flat.hip",
           "gpk_abi.hip")
ARCH = "gfx950"


def _hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP toolchain is required to build libgpk.so")


def _inputs():
    """Every file the build reads: the sources, every header under csrc/ and include/."""
    files = [os.path.join(CSRC, s) for s in SOURCES]
    for d in (CSRC, INCLUDE):
        files += sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith((".h", ".hpp", ".inc")))
    return files


def is_stale() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    return any(os.path.getmtime(f) > t for f in _inputs())


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile every HIP source for gfx950 into one shared object (returns its path)."""
    if not force and not is_stale():
        return LIB_PATH
    tmp = LIB_PATH + ".tmp.%d" % os.getpid()
    cmd = [_hipcc(), "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-result", "-I" + INCLUDE, "-I" + CSRC]
    cmd += [os.path.join(CSRC, s) for s in SOURCES]
    cmd += ["-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError("hipcc failed (%d):\n%s\n%s" % (res.returncode, res.stdout, res.stderr))
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
