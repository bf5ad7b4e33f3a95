import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "incentive-design-mpc_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN_DIR, "lompc_golden.json")) as f:
        meta = json.load(f)
    arr = np.load(os.path.join(GOLDEN_DIR, "lompc_golden.npz"), allow_pickle=False)
    cases = []
    for c in meta["cases"]:
        k = c["id"]
        d = dict(c)
        for name in ("lmbd", "gamma", "w_ref", "w", "cost", "state", "w0"):
            d[name] = arr[f"c{k}_{name}"]
        cases.append(d)
    return cases


def oracle_consts(case):
    import lompc_oracle as O

    return O.OracleConstants(case["delta"], case["theta"], case["y_max"], case["w_max"], case["ev_type"])


@pytest.fixture(scope="session")
def gpu():
    import torch

    # gpu-marked tests must not pass silently without the device: fail loudly
    assert torch.cuda.is_available(), "gpu-marked test run without a HIP device (use -m 'not gpu')"
    torch.cuda.set_device(0)
    return torch.device("cuda:0")
