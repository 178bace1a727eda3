"""CPU: the oracle's CPU-baseline machinery (test infrastructure timed by bench.py).

* orc_load_ycsb_parallel builds the single loader's leaves (every meta word, key, sorted
  count) with several threads; only the inner levels are rebuilt, and they route every key
  (both le_child modes) to the same leaf -- so reads and scans answer identically.
* orc_ycsb_txn_timed (full-txn mode: RunMixed read-only transactions + Index-SSN read side)
  commits every transaction of a read-only mix and its reads see what BTree::Read sees.
* orc_update_batch == orc_update / orc_commit_update applied op by op.
"""
import numpy as np
import pytest

import oracle_lib as O


@pytest.mark.parametrize("key_size,threads", [(8, 4), (4, 3), (8, 16)])
def test_parallel_load_has_the_single_loaders_leaves(key_size, threads):
    n = 400_000
    a = O.OracleTree()
    a.load_ycsb(0, n, key_size, 1)
    b = O.OracleTree()
    assert b.load_ycsb_parallel(0, n, key_size, 1, threads) == n
    sa, sb = a.stats(), b.stats()
    for k in ("leaves", "records", "sorted", "unsorted", "max_count", "height"):
        assert sa[k] == sb[k], k
    for x, y in zip(a.export_leaves(64), b.export_leaves(64)):
        assert (x == y).all()
    rng = np.random.default_rng(key_size * 7 + threads)
    keys = rng.integers(0, n + 500, 20000).astype(np.uint64)
    oa, ra = a.read_batch(keys, key_size)
    ob, rb = b.read_batch(keys, key_size)
    assert (oa == ob).all() and (ra == rb).all()
    ca, xa = a.scan_batch(keys[:200], key_size, 100)
    cb, xb = b.scan_batch(keys[:200], key_size, 100)
    assert (ca == cb).all() and (xa == xb).all()
    for k in keys[:1500]:
        for le in (True, False):
            assert a.traverse(int(k), key_size, le) == b.traverse(int(k), key_size, le)


def test_parallel_load_small_tables_fall_back_to_the_single_loader():
    a = O.OracleTree()
    a.load_ycsb(0, 5000, 8, 0)
    b = O.OracleTree()
    assert b.load_ycsb_parallel(0, 5000, 8, 0, 8) == 5000
    for x, y in zip(a.export_leaves(64), b.export_leaves(64)):
        assert (x == y).all()


def test_full_txn_mode_commits_read_only_mix():
    t = O.OracleTree()
    t.load_ycsb(0, 1000, 4, 0)
    keys = np.random.default_rng(5).integers(0, 1100, 50_000).astype(np.uint64)  # ~9 % absent
    for threads in (1, 4):
        sec, commits, aborts, checksum = t.ycsb_txn_timed(keys, 4, 10, threads)
        assert commits == 5000 and aborts == 0 and sec > 0
    # the checksum adds byte 4 + op of each read's tuple in the latest framing [key 4][pad 4]
    # [payload] (executor.h:396-401): pad bytes for ops 0..3, payload byte = rowid & 0xFF after
    s1 = t.ycsb_txn_timed(keys, 4, 10, 1)[3]
    s4 = t.ycsb_txn_timed(keys, 4, 10, 4)[3]
    k = keys.reshape(-1, 10)[:, 4:]
    assert s1 == s4 and s1 == int(((k & 0xFF) * (k < 1000)).sum())


def test_full_txn_mode_reads_in_flight_copies():
    t = O.OracleTree()
    t.load_ycsb(0, 2000, 8, 0)
    for k in range(0, 2000, 10):
        assert t.update(k, 8, 0, bytes([7]) * 100, 5) == 1  # left in flight (writer 5)
    keys = np.arange(0, 2000, 2, dtype=np.uint64)
    sec, commits, aborts, _ = t.ycsb_txn_timed(keys, 8, 10, 2, first_tid=100)
    assert commits + aborts == 100 and commits > 0


def test_update_batch_equals_op_by_op():
    n = 50_000
    a, b = O.OracleTree(), O.OracleTree()
    a.load_ycsb(0, n, 8, 1)
    b.load_ycsb(0, n, 8, 1)
    rng = np.random.default_rng(9)
    m = 4000
    keys = np.concatenate([rng.integers(0, n + 100, m - 200), rng.integers(0, 50, 200)]).astype(np.uint64)
    deltas = rng.integers(0, 256, (m, 24), dtype=np.uint8)
    deltas[-200:] = 3
    wid = (10 + 2 * np.arange(m)).astype(np.uint32)
    cid = (wid + 1).astype(np.uint32)
    cid[rng.random(m) < 0.1] = 0
    rc, ok = a.update_batch(keys, 8, 5, deltas, wid, cid)
    exp = np.zeros(m, np.uint8)
    for i in range(m):
        r = b.update(int(keys[i]), 8, 5, deltas[i].tobytes(), int(wid[i]))
        if r == 1 and cid[i]:
            r = b.commit_update(int(keys[i]), 8, int(cid[i]), int(cid[i]))
        exp[i] = r
    assert (rc == exp).all() and ok == int((exp == 1).sum())
    assert len(set(rc.tolist())) >= 3
    probe = rng.integers(0, n, 3000).astype(np.uint64)
    rids = rng.integers(0, 2 * m + 20, 3000).astype(np.uint32)
    oa, ra = a.read_batch(probe, 8, rids)
    ob, rb = b.read_batch(probe, 8, rids)
    assert (oa == ob).all() and (ra == rb).all()


@pytest.mark.parametrize("threads", [2, 7, 16])
def test_update_batch_mt_equals_single_writer(threads):
    """bench.py's C3 CPU leg runs the last epoch's updates on T writers (orc_update_batch_mt):
    every rc, every later read (latest / copy / old versions at any read id) and the number of
    retired versions equal the single writer's replay of the same epoch."""
    n = 60_000
    a, b = O.OracleTree(), O.OracleTree()
    a.load_ycsb(0, n, 8, 1)
    b.load_ycsb(0, n, 8, 1)
    rng = np.random.default_rng(threads)
    for ep in range(3):
        m = 6000
        # hot keys repeated many times in one epoch (RunMixed's Zipf stream), absent keys too
        keys = np.concatenate([rng.integers(0, n + 100, m - 1500), rng.integers(0, 40, 1500)]).astype(np.uint64)
        rng.shuffle(keys)
        deltas = np.repeat(rng.integers(0, 4, (m, 1), dtype=np.uint8), 100, 1)
        wid = (10 + 2 * m * ep + 2 * np.arange(m)).astype(np.uint32)
        cid = (wid + 1).astype(np.uint32)
        cid[(rng.random(m) < 0.05) & (keys > 40)] = 0  # left in flight
        rc1, ok1 = a.update_batch(keys, 8, 0, deltas, wid, cid)
        rc2, ok2, sec = b.update_batch_mt(keys, 8, 0, deltas, wid, cid, threads)
        assert (rc1 == rc2).all() and ok1 == ok2 and sec > 0
        assert len(set(rc1.tolist())) >= 3
    assert a.stats()["versions"] == b.stats()["versions"] > 0
    probe = np.concatenate([rng.integers(0, n, 4000), rng.integers(0, 40, 2000)]).astype(np.uint64)
    rids = rng.integers(0, 2 * 6000 * 3 + 20, probe.size).astype(np.uint32)
    oa, ra = a.read_batch(probe, 8, rids)
    ob, rb = b.read_batch(probe, 8, rids)
    assert (oa["status"] == ob["status"]).all() and (ra == rb).all()
    assert len(set(oa["status"].tolist())) >= 3
