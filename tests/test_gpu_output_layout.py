"""GPU parity of stage_set_output_layout: 1008-B row strides and 16-B status records
(stage_probe_out16) carry the same answers as the default layout -- every row's first
key pad + payload bytes and the status / flags / hops / cstamp / copy_sstamp / rec_cstamp of
each probe -- on a table with in-flight copies and version chains."""
import numpy as np
import pytest

import oracle_lib as O
import stage
from test_gpu_parity import check_probe

pytestmark = pytest.mark.gpu


def test_lean_layouts_equal_default(gpu):
    n = 200000
    tab = stage.Table(key_width=8)
    tab.load_ycsb(0, n, 8, mode=1)
    orc = O.OracleTree()
    orc.load_ycsb(0, n, 8, 1)
    rng = np.random.default_rng(5)
    hot = rng.choice(n, 3000, replace=False).astype(np.uint64)
    for ep in range(2):
        d = np.full((hot.size, 16), 0x40 + ep, np.uint8)
        tab.update_batch(hot, 16 * ep, d, 10 + 10 * ep, 11 + 10 * ep)
        for k in hot:
            orc.update(int(k), 8, 16 * ep, bytes([0x40 + ep]) * 16, 10 + 10 * ep)
            orc.commit_update(int(k), 8, 11 + 10 * ep, 11 + 10 * ep)
    for k in hot[:300]:  # in flight: COPY reads
        assert tab.update(int(k), 100, b"\x77" * 4, 40) == orc.update(int(k), 8, 100, b"\x77" * 4, 40)
    tab.sync()
    keys = np.concatenate([rng.integers(0, n + 500, 70000), hot]).astype(np.uint64)
    rids = rng.integers(0, 45, keys.size).astype(np.uint32)
    check_probe(tab, orc, keys[:20000], 8, read_ids=rids[:20000])
    out, rows = tab.probe(keys, read_ids=rids)
    assert set(np.unique(out["status"])) >= {stage.ST_LATEST, stage.ST_COPY, stage.ST_OLD, stage.ST_NOT_FOUND}
    for stride, sb in [(1008, 32), (0, 16), (1008, 16)]:
        tab.set_output_layout(stride, sb)
        assert tab.stride == (stride or 1024)
        o2, r2 = tab.probe(keys, read_ids=rids)
        assert (r2[:, :1008] == rows[:, :1008]).all(), (stride, sb)
        if sb == 32:
            assert (o2 == out).all()
        else:
            assert o2.dtype == stage.PROBE_OUT16_DTYPE
            for f in ("status", "flags", "hops", "cstamp", "copy_sstamp", "rec_cstamp"):
                assert (o2[f] == out[f]).all(), f
    tab.set_output_layout(0, 32)
    o3, r3 = tab.probe(keys[:1000], read_ids=rids[:1000])
    assert (o3 == out[:1000]).all() and (r3 == rows[:1000]).all()
