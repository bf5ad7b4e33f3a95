"""CPU tests of the drop-in boundary: the C-ABI library builds for gfx950,
loads, and exports exactly the symbols include/lompc_amd.h declares (no
compute calls — there is no GPU here)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "lompc_amd.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(lompc_\w+)\s*\(", src, flags=re.M)


@pytest.fixture(scope="module")
def libpath():
    from lompc_amd import build

    return build.build()


def test_header_declares_entry_points():
    fns = header_functions()
    for f in ("lompc_create", "lompc_set_params", "lompc_solve_batch", "lompc_solve_host", "lompc_destroy",
              "lompc_plan_create", "lompc_plan_run", "lompc_plan_destroy"):
        assert f in fns


def test_library_exports_every_declared_symbol(libpath):
    out = subprocess.run(["nm", "-D", "--defined-only", libpath], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\s[TW]\s(lompc_\w+)$", out, flags=re.M))
    assert set(header_functions()) <= exported


def test_ctypes_signatures_cover_header(libpath):
    from lompc_amd import _lib

    names = {n for n, _, _ in _lib.SIGNATURES}
    assert names == set(header_functions())
    lib = _lib.load()
    assert lib.lompc_abi_version() == _lib.ABI_VERSION
    assert lib.lompc_status_string(_lib.LOMPC_ERR_INVALID_ARG) == b"invalid argument"


def test_header_constants_match_python():
    from lompc_amd import _lib

    src = open(HEADER).read()
    for name in ("LOMPC_OK", "LOMPC_ERR_INVALID_ARG", "LOMPC_ERR_NOT_CONVERGED", "LOMPC_QP_REPAIRED",
                 "LOMPC_STAT_MAX_ERR", "LOMPC_SET_STATS", "LOMPC_MAX_N", "LOMPC_MODE_DIRECT", "LOMPC_PLAN_MAX_CTX",
                 "LOMPC_PLAN_WARM_START", "LOMPC_ABI_VERSION", "LOMPC_PLAN_K_PATH", "LOMPC_PLAN_K_EVAL",
                 "LOMPC_PLAN_K_FINAL", "LOMPC_PLAN_KERNELS", "LOMPC_PLAN_DIAG_REPAIR",
                 "LOMPC_PLAN_CLOSE_IN_EVAL", "LOMPC_PLAN_SORTED_GAMMA", "LOMPC_COMM_ID_BYTES", "LOMPC_LOOP_PROF_ITERS", "LOMPC_LOOP_PROF_WALL",
                 "LOMPC_LOOP_PROF_ISSUE", "LOMPC_LOOP_PROF_WAIT", "LOMPC_LOOP_PROF_GPU", "LOMPC_LOOP_PROF_STEP",
                 "LOMPC_LOOP_PROF_HOST", "LOMPC_LOOP_PROF", "LOMPC_LOOP_AHEAD", "LOMPC_PLAN_CLOSE_IN_FINALIZE",
                 "LOMPC_PLAN_CELLS_SHIFT", "LOMPC_STEPS_PER_KERNEL", "LOMPC_STEPS_SPAN_EVENTS"):
        m = re.search(rf"#define {name}\s+(\d+)", src)
        attr = "ABI_VERSION" if name == "LOMPC_ABI_VERSION" else name
        assert m and int(m.group(1)) == getattr(_lib, attr), name


def test_gfx950_code_object(libpath):
    """The bundle carries gfx950 device code (hipcc --offload-arch=gfx950)."""
    data = open(libpath, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_create_without_device_fails_loudly():
    """No CPU fallback: with no HIP device the engine refuses to run."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a device is visible")
    from lompc_amd import LoMPC, LoMPCConstants

    with pytest.raises(RuntimeError):
        LoMPC(24, LoMPCConstants(0.05, 10, 0.9, 0.25, "small"))
