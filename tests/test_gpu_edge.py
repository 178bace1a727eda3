"""GPU edge cases of the boundary: empty batches, scan_size 0, scans over deleted and in-flight
records, probes of the extreme keys, an index scan on a table without history -- each
against the oracle or the reference's stated behaviour."""
import numpy as np
import pytest

import oracle_lib as O
import stage

pytestmark = pytest.mark.gpu


def test_empty_batches_and_zero_scan_size(gpu):
    tab = stage.Table(key_width=8)
    tab.load_ycsb(0, 1000, 8)
    tab.sync()
    out, rows = tab.probe(np.zeros(0, np.uint64))
    assert out.size == 0
    counts, rows = tab.range_scan(np.array([5, 10], np.uint64), 0)
    assert (counts == 0).all()
    counts, rows, st = tab.index_scan(np.array([5], np.uint64), 0)
    assert (counts == 0).all()
    assert tab.resolve(np.zeros(0, np.uint64)).size == 0


def test_scans_over_deleted_and_inflight_records(gpu):
    n = 60000
    tab = stage.Table(key_width=8)
    orc = O.OracleTree()
    tab.load_ycsb(0, n, 8, mode=1)
    orc.load_ycsb(0, n, 8, 1)
    rng = np.random.default_rng(44)
    for k in rng.choice(n, 2000, replace=False):
        assert tab.delete(int(k), 3) == orc.delete(int(k), 8, 3)
    for k in rng.choice(n, 2000, replace=False):
        d = b"\x33" * 16
        assert tab.update(int(k), 64, d, 5) == orc.update(int(k), 8, 64, d, 5)  # in flight
    tab.sync()
    starts = np.concatenate([rng.integers(0, n, 300), [0, n - 1, n + 5]]).astype(np.uint64)
    for size in (1, 7, 64, 300):
        counts, rows = tab.range_scan(starts, size)
        oc, orows = orc.scan_batch(starts, 8, size)
        assert (counts == oc).all()
        for i in range(starts.size):
            assert (rows[i, :counts[i], :orc.row] == orows[i, :counts[i]]).all()
    # index scans (visibility per record) at several read ids
    for rid in (0, 4, 6, 0xFFFFFFFE):
        counts, rows, st = tab.index_scan(starts[:100], 20, read_ids=np.full(100, rid, np.uint32))
        for i in range(100):
            c, orow, ost = orc.index_scan(int(starts[i]), 8, 20, rid)
            assert counts[i] == c and (st[i, :c] == ost).all()
            assert (rows[i, :c, :orc.row] == orow).all()


def test_extreme_keys(gpu):
    keys = np.array([0, 1, 0x7F, 0x80, 0xFF, (1 << 63) - 1, 1 << 63, (1 << 64) - 1], np.uint64)
    tab = stage.Table(key_width=8)
    tab.load_keys(keys, 8, mode=1)
    tab.sync()
    orc = O.OracleTree()
    orc.load_keys(keys, 8, 1)
    probe = np.concatenate([keys, keys ^ np.uint64(1), np.array([2, 0x81, (1 << 64) - 2], np.uint64)])
    out, rows = tab.probe(probe)
    o_out, o_rec = orc.read_batch(probe, 8)
    assert (out["status"] == o_out["status"]).all() and (rows[:, :orc.row] == o_rec).all()
    counts, rows = tab.range_scan(probe, 8)
    oc, orows = orc.scan_batch(probe, 8, 8)
    assert (counts == oc).all()
    for i in range(probe.size):
        assert (rows[i, :counts[i], :orc.row] == orows[i, :counts[i]]).all()
