"""Diagnostics: build compile-time variants of the extension (never the product library).

    python scripts/build_variant.py NAME DEFINE[=V] [DEFINE[=V] ...]   -> lompc_amd/liblompc_amd_NAME.so

e.g. `python scripts/build_variant.py ru2 EVAL_RU=2`; scripts/step_probe.py times them on the GPU.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "incentive-design-mpc_amd"))
from lompc_amd import build  # noqa: E402

name, defines = sys.argv[1], tuple(sys.argv[2:])
out = os.path.join(ROOT, "incentive-design-mpc_amd", "lompc_amd", f"liblompc_amd_{name}.so")
print(build.build(force=True, out=out, defines=defines))
