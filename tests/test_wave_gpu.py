"""GPU: the DPP wave64 primitives (wave.cuh) behave as the kernels assume."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_wave_primitives(gpu, lib):
    import torch
    rng = np.random.default_rng(3)
    for trial in range(4):
        v = rng.integers(0, 1 << 20, size=64, dtype=np.uint32)
        if trial == 1:
            v[:] = np.arange(64)[::-1]
        din = torch.from_numpy(v.astype(np.int64).astype(np.int32)).to(gpu)
        dout = torch.zeros(8 * 64, dtype=torch.int32, device=gpu)
        lib.jfs_selftest_wave.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        assert lib.jfs_selftest_wave(din.data_ptr(), dout.data_ptr()) == 0
        o = dout.cpu().numpy().astype(np.uint32).reshape(8, 64)
        x = v.astype(np.uint64)
        assert (o[0] == np.cumsum(x).astype(np.uint32)).all(), "scan add"
        assert (o[1] == np.maximum.accumulate(v)).all(), "scan max"
        assert (o[2] == np.minimum.accumulate(v)).all(), "scan min"
        sh = np.concatenate([[12345], v[:-1]]).astype(np.uint32)
        assert (o[3] == sh).all(), "shift up"
        assert (o[4] == v.min()).all() and (o[5] == v.max()).all()
        assert (o[6] == np.uint32(x.sum() & 0xFFFFFFFF)).all()
        assert (o[7] == (np.cumsum(x) - x).astype(np.uint32)).all(), "exclusive scan"
