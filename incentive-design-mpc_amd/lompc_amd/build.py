"""Build the HIP extension in-tree: csrc/*.hip -> lompc_amd/liblompc_amd.so (gfx950)."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(ROOT, "csrc")
OUT = os.path.join(PKG, "liblompc_amd.so")
SOURCES = ["lompc_kernels.hip", "lompc_plan.hip", "lompc_price.cpp", "lompc_bimpc.cpp", "lompc_comm.cpp",
           "lompc_loop.hip", "lompc_levels.hip"]
# every header under csrc/ (not a hand-kept list: an edit to any included header must rebuild the
# pushed .so; tests/test_build_deps.py checks each `#include "…"` resolves to a DEPS entry)
DEPS = SOURCES + sorted(f for f in os.listdir(CSRC) if f.endswith((".hpp", ".h"))) + \
    [os.path.join("..", "..", "include", "lompc_amd.h")]
ARCH = os.environ.get("LOMPC_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def up_to_date() -> bool:
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(os.path.join(CSRC, d)) <= t for d in DEPS)


# host-only sources (the BiMPC interior point, the price QP, RCCL glue): AVX2 + FMA, which every
# x86-64 host of an MI355X node has
HOST_FLAGS = ["-mavx2", "-mfma"]


def _compile(src: str, obj: str, flags: list, verbose: bool) -> None:
    extra = HOST_FLAGS if src.endswith(".cpp") else []
    cmd = [_hipcc()] + flags + extra + ["-c", os.path.join(CSRC, src), "-o", obj + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(obj + ".tmp", obj)


def build(force: bool = False, verbose: bool = False, out: str = OUT, defines: tuple = ()) -> str:
    """Compile the extension (one object per source, in parallel, then one link); ``defines``
    (e.g. ("LOMPC_K1_STATS",)) builds a diagnostic variant into ``out`` (never the product
    library)."""
    if not force and out == OUT and up_to_date():
        return OUT
    flags = ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-Wno-unused-result"] + \
        [f"-D{d}" for d in defines]
    tag = "_".join(d.replace("=", "-") for d in defines) or "product"
    odir = os.path.join(ROOT, "build", tag)
    os.makedirs(odir, exist_ok=True)
    deps_t = max(os.path.getmtime(os.path.join(CSRC, d)) for d in DEPS)
    objs, todo = [], []
    for s in SOURCES:
        o = os.path.join(odir, os.path.splitext(s)[0] + ".o")
        objs.append(o)
        if force or not os.path.exists(o) or os.path.getmtime(o) < deps_t:
            todo.append((s, o))
    if todo:
        from concurrent.futures import ThreadPoolExecutor

        jobs = max(1, min(len(todo), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
        with ThreadPoolExecutor(jobs) as ex:
            for f in [ex.submit(_compile, s, o, flags, verbose) for s, o in todo]:
                f.result()
    tmp = out + ".tmp"
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-fPIC", "-shared"] + objs + ["-ldl", "-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
