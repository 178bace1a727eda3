"""BASELINE.json configs[1] / [3] at their full size (100M rows, 8-byte keys, 1000-byte payloads,
loaded as LoadYCSBRows does, ycsb_loader.cpp:144-172): the oracle cannot hold 134 GB of
64 KiB leaves, so parity here is through size-independent properties of the reference's
semantics --
  * every present key reads back LATEST with its own row ([key][rowid & 0xFF x 1000],
    Record::New framing b_tree.h:407-428), every absent key NOT_FOUND (BTree::Read nullptr);
  * the device separator tree resolves every probe to the leaf the host router picks
    (BTree::TraverseToLeaf, b_tree.cpp:1804-1846), and a probe fed the host's leaf ids writes
    the same bytes as the device-traversal probe;
  * scans equal the reference's scan semantics restated over the exported slot arrays
    (tests/scan_semantics.py, pinned to the oracle on CPU): RangeScanBySize's slot-order cut
    and Iterator's re-traversal (b_tree.cpp:1261-1315, b_tree.h:883-953) -- KeyCompare order
    is signed bytes of the little-endian key, and the cut skips keys, so this is not "the
    next 100 keys";
  * the same batch probed twice writes identical bytes.
Runs in about a minute (load ~25 s, leaf export and the scan restatement ~20 s)."""
import numpy as np
import pytest

import stage
from scan_semantics import LeafScanner

pytestmark = pytest.mark.gpu

N = 100_000_000


@pytest.fixture(scope="module")
def full(gpu):
    tab = stage.Table(key_width=8)
    assert tab.load_ycsb(0, N, 8, 0) == N
    tab.sync()
    yield tab
    tab.close()


def expect_rows(rows, keys):
    got = rows[:, :8].copy().view(np.uint64).ravel()
    bad = np.flatnonzero(got != keys)
    assert bad.size == 0, (f"{bad.size} of {keys.size} keys differ, first at {bad[0]}: "
                           f"got {got[bad[:6]].tolist()} want {keys[bad[:6]].tolist()}")
    assert (rows[:, 8:1008] == (keys & np.uint64(0xFF)).astype(np.uint8)[:, None]).all()


def test_full_size_shape(full):
    st = full.stats()
    assert st["records"] == N
    assert st["sorted"] + st["unsorted"] == N
    assert st["max_count"] <= 63  # ycsb split threshold: at most 63 records per 64 KiB leaf
    assert st["leaves"] * 63 >= N and st["leaves"] < N // 40


def test_full_size_probe(full):
    rng = np.random.default_rng(2024)
    present = np.concatenate([stage.zipf_draws(N - 1, 0.9, 0x5EED, 1 << 21, nthreads=16),
                              rng.integers(0, N, 1 << 18).astype(np.uint64),
                              np.array([0, 1, N // 2, N - 2, N - 1], np.uint64)])
    absent = np.concatenate([np.arange(N, N + 1000, dtype=np.uint64),
                             rng.integers(N, 1 << 62, 1000).astype(np.uint64),
                             np.array([np.iinfo(np.uint64).max], np.uint64)])
    keys = np.concatenate([present, absent])
    out, rows = full.probe(keys)
    m = present.size
    assert (out["status"][:m] == stage.ST_LATEST).all()
    expect_rows(rows[:m], present)
    assert (out["status"][m:] == stage.ST_NOT_FOUND).all()
    # device traversal == host router, and the host-leaf-id probe writes the same bytes
    sample = keys[:: max(1, keys.size // (1 << 16))]
    leaves = full.traverse(sample)
    o1, r1 = full.probe(sample)
    o2, r2 = full.probe(sample, leaf_ids=leaves)
    assert (o1["leaf"] == leaves).all()
    assert o1.tobytes() == o2.tobytes() and r1.tobytes() == r2.tobytes()
    # idempotence
    o3, r3 = full.probe(sample)
    assert o1.tobytes() == o3.tobytes() and r1.tobytes() == r3.tobytes()


def test_full_size_scans(full):
    """Exact parity with the reference's scan semantics at 100M rows: tests/scan_semantics.py
    (pinned to the oracle by test_scan_semantics.py) over the exported slot arrays."""
    ls = LeafScanner(full)
    rng = np.random.default_rng(7)
    last = ls.keyw[-1, :int(ls.rc[-1])]
    starts = np.concatenate([rng.integers(0, N, 600), [0, 1, N - 100, N - 1, N, N + 12345, 0x7F7F7F7F, 0x80808080],
                             last[:2], last[-2:]]).astype(np.uint64)
    for L in (100, 7):
        counts, rows = full.range_scan(starts, L)
        for i, s in enumerate(starts):
            want = ls.scan(int(s), L)
            assert counts[i] == want.size, (int(s), L, int(counts[i]), want.size)
            if want.size:
                expect_rows(rows[i, :want.size], want)


def test_full_size_device_epoch(full):
    """BASELINE configs[2] at full size: one YCSB-B shaped epoch (Zipf 0.99 keys, 100-B column
    patches, ids from one counter, some left in flight) on the device write path of the 100M-row
    table.  A key's outcome depends only on its own record, so the oracle holding just the
    touched keys (same rows: LoadYCSBRows payloads) is the reference: every return code and
    every read of the touched keys at old, middle and current read ids must match it.
    Runs last: it writes to the shared table."""
    from test_gpu_parity import check_probe
    from test_gpu_write_path import oracle_epoch
    import oracle_lib as O

    rng = np.random.default_rng(5)
    m = 1 << 19
    keys = np.concatenate([stage.zipf_draws(N - 1, 0.99, 0x5EED + 77, m - 16, nthreads=16),
                           np.arange(N + 3, N + 19, dtype=np.uint64)])  # a few absent keys
    deltas = np.repeat(((keys + np.uint64(1)) & np.uint64(0xFF)).astype(np.uint8)[:, None], 100, 1)
    rand = rng.random(m) < 0.3  # a third with fresh bytes: hot keys take several versions
    deltas[rand] = rng.integers(0, 256, (int(rand.sum()), 100), dtype=np.uint8)
    wid = (10 + 2 * np.arange(m)).astype(np.uint32)
    cid = (wid + 1).astype(np.uint32)
    cid[rng.random(m) < 0.05] = 0  # left in flight: later ops on the key see DIRTY
    rc, ok = full.update_batch_device(keys, 0, deltas, wid, cid)
    touched = np.unique(keys[keys < N])
    orc = O.OracleTree()
    assert orc.load_keys(touched, 8, 0) == touched.size
    exp = oracle_epoch(orc, keys, 8, 0, deltas, wid, cid)
    bad = np.flatnonzero(rc != exp)
    assert bad.size == 0, (bad[:5], rc[bad[:5]], exp[bad[:5]], keys[bad[:5]])
    assert ok == int((exp == stage.RC_OK).sum()) and len(set(exp.tolist())) >= 3
    hi = int(cid.max()) + 2
    probe = np.concatenate([touched[rng.choice(touched.size, min(touched.size, 60000), replace=False)],
                            keys[:2000]]).astype(np.uint64)
    for r in (0, 1, hi // 3, hi, 0xFFFFFFFE):
        check_probe(full, orc, probe, 8, read_ids=np.full(probe.size, r, np.uint32))
    check_probe(full, orc, probe, 8, read_ids=rng.integers(0, hi, probe.size).astype(np.uint32))
