"""GPU: the RCCL sharded probe front-end (stage_probe_sharded) on a one-rank communicator
returns exactly what the direct probe returns (routing, all-to-all-v to self, unpermute)."""
import ctypes

import numpy as np
import pytest

import stage
from stage._lib import check

pytestmark = pytest.mark.gpu


def test_sharded_world1_equals_direct(gpu):
    tab = stage.Table(key_width=8)
    tab.load_ycsb(0, 1_000_000, 8, mode=1)
    tab.sync()
    L = stage.lib()
    uid = (ctypes.c_uint8 * 128)()
    check(L.stage_comm_unique_id(uid), "uid")
    check(L.stage_comm_init(tab.h, uid, 0, 1), "init")
    try:
        keys = np.random.default_rng(0).integers(0, 1_100_000, 300_000).astype(np.uint64)
        rids = np.random.default_rng(1).integers(0, 1 << 32, keys.size).astype(np.uint32)
        d_keys = stage.DeviceBuffer.from_numpy(keys)
        d_rids = stage.DeviceBuffer.from_numpy(rids)
        d_out = stage.DeviceBuffer(keys.size * 32)
        d_rec = stage.DeviceBuffer(keys.size * tab.stride)
        for _ in range(2):  # second call reuses the grown scratch buffers
            check(L.stage_probe_sharded(tab.h, d_keys.ptr, d_rids.ptr, keys.size, d_out.ptr, d_rec.ptr, None), "sh")
            check(L.stage_device_sync(), "sync")
        out = d_out.to_numpy(stage.PROBE_OUT_DTYPE, keys.size)
        rows = d_rec.to_numpy(np.uint8, keys.size * tab.stride).reshape(keys.size, tab.stride)
        ref_out, ref_rows = tab.probe(keys, read_ids=rids)
        assert (out == ref_out).all()
        assert (rows == ref_rows).all()
    finally:
        check(L.stage_comm_destroy(tab.h), "destroy")
