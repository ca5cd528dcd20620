"""In-tree build of libgpk.so (hand-written HIP for gfx950) with hipcc.

The shared object lands next to this file so that it travels with the repository snapshot to
the GPU box; nothing is installed into site-packages and nothing is JIT-compiled at import.
Every source compiles to its own object under ``_obj/`` (in parallel; only the sources whose
inputs changed are recompiled), then one link step.  The sources share no device symbols, so
the objects are exactly what one hipcc call over all sources would produce.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
OBJ = os.path.join(HERE, "_obj")
LIB_NAME = "libgpk.so"
LIB_PATH = os.path.join(HERE, LIB_NAME)
SOURCES = ("gpk_assemble.hip", "gpk_diag.hip", "gpk_potrf.hip", "gpk_approx.hip", "gpk_eig.hip", "gpk_flat.hip",
           "gpk_abi.hip")
ARCH = "gfx950"
FLAGS = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result", "-Wno-unused-value"]


def _hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP toolchain is required to build libgpk.so")


def _headers():
    files = []
    for d in (CSRC, INCLUDE):
        files += sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith((".h", ".hpp", ".inc")))
    return files


def _inputs():
    """Every file the build reads: the sources, every header under csrc/ and include/."""
    return [os.path.join(CSRC, s) for s in SOURCES] + _headers()


def _newest(paths) -> float:
    return max((os.path.getmtime(p) for p in paths), default=0.0)


def is_stale() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    return any(os.path.getmtime(f) > t for f in _inputs())


def _obj_path(src: str) -> str:
    return os.path.join(OBJ, os.path.splitext(src)[0] + ".o")


def _compile(src: str, extra, verbose: bool) -> str:
    obj = _obj_path(src)
    tmp = obj + ".tmp.%d" % os.getpid()
    cmd = [_hipcc()] + FLAGS + list(extra) + ["-I" + INCLUDE, "-I" + CSRC, "-c", os.path.join(CSRC, src), "-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError("hipcc failed on %s (%d):\n%s\n%s" % (src, res.returncode, res.stdout, res.stderr))
    os.replace(tmp, obj)
    return obj


def build(force: bool = False, verbose: bool = False, extra=(), out: str = None, jobs: int = None) -> str:
    """Compile every HIP source for gfx950 into one shared object (returns its path).  ``extra``: more hipcc
    flags (variant builds, e.g. -D switches; those go to ``out`` and a separate object directory)."""
    global OBJ
    target = out or LIB_PATH
    if not force and not extra and out is None and not is_stale():
        return LIB_PATH
    obj_dir = OBJ if not extra else os.path.join(HERE, "_obj_" + "_".join(
        "".join(c for c in e if c.isalnum()) for e in extra)[:80])
    os.makedirs(obj_dir, exist_ok=True)
    saved, OBJ = OBJ, obj_dir
    try:
        hdr_t = _newest(_headers())
        todo = []
        for s in SOURCES:
            o = _obj_path(s)
            if force or not os.path.exists(o) or os.path.getmtime(o) < max(hdr_t, os.path.getmtime(os.path.join(CSRC, s))):
                todo.append(s)
        # the largest translation units first (gpk_assemble takes ~2 min, the rest ~1 min or less)
        todo.sort(key=lambda s: -os.path.getsize(os.path.join(CSRC, s)))
        n = jobs or max(1, min(len(todo), os.cpu_count() or 1, 8))
        if todo:
            with ThreadPoolExecutor(max_workers=n) as ex:
                list(ex.map(lambda s: _compile(s, extra, verbose), todo))
        objs = [_obj_path(s) for s in SOURCES]
    finally:
        OBJ = saved
    tmp = target + ".tmp.%d" % os.getpid()
    cmd = [_hipcc(), "--offload-arch=" + ARCH, "-shared", "-fPIC"] + objs + ["-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError("link failed (%d):\n%s\n%s" % (res.returncode, res.stdout, res.stderr))
    os.replace(tmp, target)
    return target


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if a != "--force"]
    out = None
    if "-o" in args:
        i = args.index("-o")
        out = os.path.abspath(args[i + 1])
        del args[i:i + 2]
    print(build(force="--force" in sys.argv, verbose=True, extra=args, out=out))
