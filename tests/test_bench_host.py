"""bench.py's host-side arithmetic (CPU): the all-reduce exposure model the N > 1 line reports."""
import importlib.util
import os

import pytest

from conftest import ROOT


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_exposure_model_serialises_buckets():
    b = _bench()
    # two 1 GB buckets at W = 2 (wire bytes = bytes): 1 GB at 100 GB/s = 10 ms each
    bk = [(-30.0, 1e9), (-5.0, 1e9)]
    # first: -30 -> -20; second starts at max(-5, -20) = -5 -> +5 ms exposed
    assert b.exposure_model(bk, 2, 100.0) == pytest.approx(5.0)
    # ready long before the end and fast links: nothing exposed
    assert b.exposure_model(bk, 2, 1000.0) == 0.0
    # a late first bucket delays the second (serialised on one stream)
    assert b.exposure_model([(-1.0, 1e9), (-0.5, 1e9)], 2, 100.0) == pytest.approx(19.0)
    # W = 8: 2 * 7 / 8 of the bytes on the wire
    assert b.exposure_model([(0.0, 8e9)], 8, 1000.0) == pytest.approx(14.0)
    assert b.exposure_model([], 8, 300.0) == 0.0
