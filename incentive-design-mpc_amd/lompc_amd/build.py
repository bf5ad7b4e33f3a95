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
           "lompc_loop.hip"]
DEPS = SOURCES + ["lompc_qp.hpp", "lompc_wave.hpp", "lompc_pricewave.hpp", "lompc_agg.hpp", "lompc_dense.hpp", "lompc_ctx.hpp",
                  os.path.join("..", "..", "include", "lompc_amd.h")]
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


def build(force: bool = False, verbose: bool = False, out: str = OUT, defines: tuple = ()) -> str:
    """Compile the extension; ``defines`` (e.g. ("LOMPC_K1_STATS",)) builds a diagnostic
    variant into ``out`` (never the product library)."""
    if not force and out == OUT and up_to_date():
        return OUT
    tmp = out + ".tmp"
    cmd = [_hipcc(), "-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-result"] + [f"-D{d}" for d in defines] + \
        [os.path.join(CSRC, s) for s in SOURCES] + ["-ldl", "-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
