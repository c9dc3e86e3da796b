"""CPU positive controls for the guard-band checker of tests/test_gpu_guard_bands.py: a store one
row before a buffer, one past it, and data in a layer output's pad columns are all reported; a
declared composite-output column and zero-filled pad columns are not."""
import pytest
import torch

import test_gpu_guard_bands as G


def _alloc(gt, shape):
    return gt._guarded(shape, torch.float32, torch.device("cpu"))


def _check(gt, regions, extra=()):
    orig = torch.cuda.synchronize
    torch.cuda.synchronize = lambda: None      # CPU buffers: nothing to wait for
    try:
        return G._check(gt, regions, extra)
    finally:
        torch.cuda.synchronize = orig


def test_clean_buffers_pass():
    gt = G._GuardedTorch()
    t = _alloc(gt, (8, 260))
    t[:, :257] = 1.0
    t[:, 257:] = 0.0
    assert _check(gt, [("f", 0, t.data_ptr(), 8, 260, 257)]) == 1


@pytest.mark.parametrize("where", ["before", "after"])
def test_store_outside_buffer_is_reported(where):
    gt = G._GuardedTorch()
    t = _alloc(gt, (8, 64))
    buf, off, nbytes = gt.allocs[0]
    buf[off - 16 if where == "before" else off + nbytes + 4] = 0
    with pytest.raises(AssertionError, match="outside their buffers"):
        _check(gt, [])


def test_data_in_pad_columns_is_reported_unless_declared():
    gt = G._GuardedTorch()
    t = _alloc(gt, (8, 260))
    t[:, :256] = 1.0
    t[3, 256] = 2.5                           # a stray value in a pad column
    with pytest.raises(AssertionError, match="pad columns"):
        _check(gt, [("f", 0, t.data_ptr(), 8, 260, 256)])
    # the same column declared as another output of the launch (density-gradient rows)
    assert _check(gt, [("f", 0, t.data_ptr(), 8, 260, 256)], [(t.data_ptr() + 4 * 256, 260)]) == 1
