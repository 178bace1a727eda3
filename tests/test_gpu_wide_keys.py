"""GPU parity for tables with keys above 8 bytes (TPC-C composite keys):
point probes with visibility, range scans and incremental publication, against the oracle.
Leaves of small TPC-C rows hold up to ~600 records: device leaves of up to 1024 slots."""
import numpy as np
import pytest

import oracle_lib as O
import stage
from test_wide_keys import build, composite_keys, tpcc_like

pytestmark = pytest.mark.gpu


def check_wide(tab, orc, keys, rids=None):
    out, rows = tab.probe(keys, read_ids=rids)
    o_out, o_rec = orc.read_batch_k(keys, rids)
    for f in ("status", "hops", "cstamp", "rec_cstamp", "copy_sstamp"):
        assert (out[f] == o_out[f]).all(), f
    assert ((out["flags"] & 1) == o_out["copy_present"]).all()
    assert (rows[:, :orc.row] == o_rec).all()
    return out


@pytest.mark.parametrize("width,payload", [(16, 320), (24, 600), (32, 60), (16, 40)])
def test_wide_probe_and_scan(gpu, width, payload):
    keys = tpcc_like(width)
    tab, orc, _ = build(width, payload, keys)
    tab.sync()
    assert tab.leaf_capacity >= 64
    rng = np.random.default_rng(width + payload)
    probe = np.concatenate([keys[rng.choice(keys.shape[0], 20000)],
                            rng.integers(0, 256, (2000, width), dtype=np.uint8),
                            keys[:50] ^ np.uint8(1)])
    out = check_wide(tab, orc, probe)
    assert (out["status"][:20000] == stage.ST_LATEST).all()
    starts = np.concatenate([keys[rng.choice(keys.shape[0], 300)], keys[-3:], keys[:2]])
    for size in (1, 10, 100):
        counts, rows = tab.range_scan(starts, size)
        o_counts, o_rows = orc.scan_batch_k(starts, size)
        assert (counts == o_counts).all(), size
        for i in range(starts.shape[0]):
            assert (rows[i, :counts[i], :orc.row] == o_rows[i, :counts[i]]).all(), (size, i)
    # resolve on the device == host traversal
    assert (tab.resolve(probe) == tab.traverse(probe)).all()
    assert (tab.resolve(probe, le_child=False) == tab.traverse(probe, le_child=False)).all()


def test_wide_versions_and_incremental_publish(gpu):
    keys = tpcc_like(32)
    tab, orc, _ = build(32, 60, keys)
    tab.sync()
    rng = np.random.default_rng(9)
    hot = keys[rng.choice(keys.shape[0], 3000, replace=False)]
    cid = 10
    for ep in range(3):
        for k in hot[: 3000 - 800 * ep]:
            d = bytes([ep + 1]) * 8
            assert tab.update_key(k.tobytes(), 8 * ep, d, cid) == orc.update(k.tobytes(), 32, 8 * ep, d, cid)
            assert tab.commit_update_key(k.tobytes(), cid + 1, cid + 1) == orc.commit_update(k.tobytes(), 32, cid + 1,
                                                                                             cid + 1)
        cid += 5
        for k in hot[:100]:  # in flight
            if ep == 2:
                assert tab.update_key(k.tobytes(), 40, b"\x55" * 4, cid) == orc.update(k.tobytes(), 32, 40,
                                                                                       b"\x55" * 4, cid)
        tab.sync()
        assert tab.sync_info()["incremental"]
        sel = np.concatenate([hot, keys[rng.choice(keys.shape[0], 5000)]])
        for rid in (0, 11, 16, 21, cid + 1, 0xFFFFFFFE):
            check_wide(tab, orc, sel, np.full(sel.shape[0], rid, np.uint32))
