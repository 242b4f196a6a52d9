import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, os.path.join(REPO, "incubator-pinot_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

from pinot_amd.segment import build_segment  # noqa: E402

# BaseSingleValueQueriesTest schema (PT/queries/BaseSingleValueQueriesTest.java:93-101)
SV_SCHEMA = [("column1", "INT"), ("column3", "INT"), ("column5", "STRING"), ("column6", "INT"),
             ("column7", "INT"), ("column9", "INT"), ("column11", "STRING"), ("column12", "STRING"),
             ("column17", "INT"), ("column18", "INT"), ("daysSinceEpoch", "INT")]
SV_INVERTED = ("column6", "column7", "column11", "column17", "column18")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device) and the built libpinot_gpu.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def load_sv_columns():
    z = np.load(os.path.join(GOLDEN, "test_data_sv.npz"))
    return {n: (t, z[n].tolist()) for n, t in SV_SCHEMA}


@pytest.fixture(scope="session")
def sv_segment():
    return build_segment("testTable_126164076_167572854", load_sv_columns(), inverted_columns=SV_INVERTED)


@pytest.fixture(scope="session")
def simple_segments():
    z = np.load(os.path.join(GOLDEN, "simple_data.npz"))
    cols = {n: ("INT", z[n].tolist()) for n in ("dim0", "dim1", "met")}
    return [build_segment("testTable_%d" % i, cols) for i in range(2)]


@pytest.fixture(scope="session")
def kats():
    import json
    with open(os.path.join(GOLDEN, "reference_kats.json")) as f:
        return json.load(f)


def has_gpu():
    try:
        import torch  # noqa: F401  (device count only; no GPU init)
        return torch.cuda.device_count() > 0
    except Exception:
        return False
