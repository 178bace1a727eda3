"""8-byte keys with small rows (CH / TPC-C ITEM-like tables: 40..200-byte payloads, 300..1500
records per 64 KiB leaf): device leaves of 256..1024 slots through the wide-key kernel
instances (KW = 1).  CPU: host layout, images and traversal equal the oracle's.  GPU: probes with
visibility, range scans of 1..300 records, device traversal and a device write epoch equal the
oracle's."""
import numpy as np
import pytest

import oracle_lib as O
import stage
from test_wide_keys import build

CASES = [(200, "asc"), (100, "rand"), (40, "rand")]


def keys8(order, n=60000, seed=2):
    rng = np.random.default_rng(seed)
    k = np.arange(n, dtype=np.int64) * 3 + 1
    if order == "rand":
        k = rng.permutation(k)
    return np.ascontiguousarray(k).view(np.uint8).reshape(-1, 8)


@pytest.mark.parametrize("payload,order", CASES)
def test_small_rows_layout_matches_oracle(payload, order):
    keys = keys8(order, n=20000)
    tab, orc, _ = build(8, payload, keys)
    assert tab.leaf_capacity > 128
    assert tab.stats()["leaves"] == orc.stats()["leaves"] > 1
    b, sk, sl = tab.export_leaf_images()
    ob, osk, osl = orc.export_leaf_images(kwords=1)
    assert (b == ob).all() and (sl == osl).all() and (sk == osk).all()
    rng = np.random.default_rng(4)
    probe = np.concatenate([keys[rng.choice(keys.shape[0], 300)], rng.integers(0, 256, (100, 8), dtype=np.uint8)])
    for le in (True, False):
        assert (tab.traverse(probe, le_child=le) ==
                np.array([orc.traverse(k.tobytes(), 8, le) for k in probe])).all()


@pytest.mark.gpu
@pytest.mark.parametrize("payload,order", CASES)
def test_small_rows_device_parity(gpu, payload, order):
    from test_gpu_wide_keys import check_wide
    from test_gpu_write_path import oracle_epoch
    keys = keys8(order)
    tab, orc, _ = build(8, payload, keys)
    tab.sync()
    rng = np.random.default_rng(payload)
    probe = np.concatenate([keys[rng.choice(keys.shape[0], 20000)], rng.integers(0, 256, (2000, 8), dtype=np.uint8)])
    out = check_wide(tab, orc, probe)
    assert (out["status"][:20000] == stage.ST_LATEST).all()
    assert (tab.resolve(probe) == tab.traverse(probe)).all()
    assert (tab.resolve(probe, le_child=False) == tab.traverse(probe, le_child=False)).all()
    starts = np.concatenate([keys[rng.choice(keys.shape[0], 200)], rng.integers(0, 256, (20, 8), dtype=np.uint8)])
    for size in (1, 10, 63, 100, 300):
        counts, rows = tab.range_scan(starts, size)
        o_counts, o_rows = orc.scan_batch_k(starts, size)
        assert (counts == o_counts).all(), size
        for i in range(starts.shape[0]):
            assert (rows[i, :counts[i], :orc.row] == o_rows[i, :counts[i]]).all(), (size, i)
    # one device write epoch (hot keys repeat; some left in flight), then reads at old and new ids
    m = 6000
    ek = keys[rng.choice(keys.shape[0], m)]
    deltas = rng.integers(0, 256, (m, 16), dtype=np.uint8)
    wid = (10 + 2 * np.arange(m)).astype(np.uint32)
    cid = (wid + 1).astype(np.uint32)
    cid[rng.random(m) < 0.1] = 0
    rc, ok = tab.update_batch_device(ek, 4, deltas, wid, cid)
    exp = oracle_epoch(orc, [k.tobytes() for k in ek], 8, 4, deltas, wid, cid)
    assert (rc == exp).all() and ok == int((exp == stage.RC_OK).sum())
    for r in (5, int(cid.max()) // 2, 0xFFFFFFFE):
        check_wide(tab, orc, ek[:3000], np.full(3000, r, np.uint32))
