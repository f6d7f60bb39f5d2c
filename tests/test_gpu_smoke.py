"""The driver's round-end entry point: __graft_entry__.smoke() (one small two-pass solve
on cuda:0, bitwise against the device-order oracle) must run as the driver calls it."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_graft_entry_smoke():
    tpl_amd = pytest.importorskip("tpl_amd")
    if tpl_amd.device_count() < 1:
        pytest.skip("no GPU visible")
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import __graft_entry__
    __graft_entry__.smoke()
