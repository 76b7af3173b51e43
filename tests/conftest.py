import os
import re
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def golden(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle_ctypes
    oracle_ctypes.lib()
    return oracle_ctypes


def run_fail_msg(r):
    """a torchrun child's failure, readable: every rank's traceback lines first (torchrun
    prefixes them with [rankN]:), then the tail of the output"""
    out = (r.stdout or "") + (r.stderr or "")
    lines = out.splitlines()
    ranks = [ln for ln in lines if re.match(r"\s*\[rank\d+\]:", ln) or "Error" in ln]
    return "\n".join(ranks[:200]) + "\n---- tail ----\n" + out[-3000:]
