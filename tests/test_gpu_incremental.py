"""GPU parity of incremental publication (stage_sync without a split since the last one).

Between two publishes the host write path (update / commit / finalize / delete / insert
into an existing leaf) only changes slot words and heads of the written leaves; the sync
patches those in place on the device (patch_kernel) and appends the new record-heap rows
and copy/version headers.  After every publish the device must answer exactly like the
oracle, and a split must fall back to a full re-publish.
"""
import numpy as np
import pytest

import oracle_lib as O
import stage
from test_gpu_parity import check_probe

pytestmark = pytest.mark.gpu


def check_all(tab, orc, keys, rng, cid_hi, key_size=8):
    for rid in (0, 1, cid_hi // 2, cid_hi, 0xFFFFFFFE):
        check_probe(tab, orc, keys, key_size, read_ids=np.full(keys.size, rid, np.uint32))
    check_probe(tab, orc, keys, key_size, read_ids=rng.integers(0, cid_hi + 2, keys.size).astype(np.uint32))
    starts = rng.choice(keys, 200)
    counts, rows = tab.range_scan(starts, 50)
    o_counts, o_rows = orc.scan_batch(starts, key_size, 50)
    assert (counts == o_counts).all()
    for i in range(starts.size):
        assert (rows[i, :counts[i], :orc.row] == o_rows[i, :counts[i]]).all()


def test_incremental_epochs_match_oracle(gpu):
    n = 200000
    base = np.arange(n, dtype=np.uint64) * 4  # gaps for inserts into existing leaves
    tab = stage.Table(key_width=8)
    orc = O.OracleTree()
    tab.load_keys(base, 8, mode=1)
    orc.load_keys(base, 8, 1)
    tab.sync()
    assert not tab.sync_info()["incremental"]
    leaves0 = tab.stats()["leaves"]
    rng = np.random.default_rng(31)
    cid = 10
    for epoch in range(4):
        m = 20000
        keys = rng.choice(base, m)
        deltas = rng.integers(0, 256, (m, 24), dtype=np.uint8)
        commit = np.where(rng.random(m) < 0.85, cid + 1, 0).astype(np.uint32)
        rc, _ = tab.update_batch(keys, 40 * epoch, deltas, cid, commit)
        for i in range(m):
            r = orc.update(int(keys[i]), 8, 40 * epoch, deltas[i].tobytes(), cid)
            if r == stage.RC_OK and commit[i]:
                r = orc.commit_update(int(keys[i]), 8, int(commit[i]), int(commit[i]))
            assert r == rc[i]
        if epoch == 2:
            for k in rng.choice(base, 300, replace=False):
                assert tab.delete(int(k), cid) == orc.delete(int(k), 8, cid)
        if epoch == 3:
            # a few inserts into gaps of distinct leaves: no split
            for k in rng.choice(base, 40, replace=False) + 1:
                pay = rng.integers(0, 256, 1000, dtype=np.uint8).tobytes()
                assert tab.insert(int(k), 8, pay, commit_id=cid) == orc.insert(int(k), 8, pay, cid)
        tab.sync()
        info = tab.sync_info()
        assert tab.stats()["leaves"] == leaves0
        assert info["incremental"] and info["slots"] > 0 and info["leaves"] > 0, info
        probe = np.concatenate([rng.choice(base, 30000), keys[:5000], base[:64] + 1,
                                rng.integers(0, 4 * n + 100, 3000).astype(np.uint64)])
        check_all(tab, orc, probe, rng, cid + 2)
        cid += 5

    # in-flight updates then FinalizeUpdate (next keeps pointing at the copy)
    for k in rng.choice(base, 500, replace=False):
        assert tab.update(int(k), 0, b"\x77" * 8, cid) == orc.update(int(k), 8, 0, b"\x77" * 8, cid)
        assert tab.finalize_update(int(k), cid + 1) == orc.finalize_update(int(k), 8, cid + 1)
    tab.sync()
    assert tab.sync_info()["incremental"]
    check_all(tab, orc, rng.choice(base, 20000), rng, cid + 2)

    # enough inserts to split leaves: full re-publish, still identical
    extra = np.arange(n, dtype=np.uint64) * 4 + 2
    tab.load_keys(extra[: n // 2], 8, mode=1)
    orc.load_keys(extra[: n // 2], 8, 1)
    tab.sync()
    assert not tab.sync_info()["incremental"] and tab.stats()["leaves"] > leaves0
    check_all(tab, orc, np.concatenate([rng.choice(base, 20000), rng.choice(extra, 20000)]), rng, cid + 2)
    # and incremental again afterwards
    keys = rng.choice(extra[: n // 2], 5000)
    rc, _ = tab.update_batch(keys, 500, np.full((keys.size, 4), 0xAB, np.uint8), cid + 3, cid + 4)
    for i, k in enumerate(keys):
        r = orc.update(int(k), 8, 500, b"\xab" * 4, cid + 3)
        if r == stage.RC_OK:
            r = orc.commit_update(int(k), 8, cid + 4, cid + 4)
        assert r == rc[i]
    tab.sync()
    assert tab.sync_info()["incremental"]
    check_all(tab, orc, keys, rng, cid + 6)
