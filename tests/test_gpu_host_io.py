"""GPU parity of the host-buffer entry points: stage_probe_host (chunked, three streams) and the
single-key readers (stage_reader_*, the BTree::Read adapter of SURVEY §8(b)) -- the coalescing
one and the resident one (a device-resident polling loop over a request ring) -- against the
oracle and against the device-buffer probe."""
import threading

import numpy as np
import pytest

import oracle_lib as O
import stage
from test_gpu_parity import check_probe

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def chains(gpu):
    n = 300000
    tab = stage.Table(key_width=8)
    orc = O.OracleTree()
    tab.load_ycsb(0, n, 8, mode=1)
    orc.load_ycsb(0, n, 8, 1)
    rng = np.random.default_rng(41)
    hot = rng.choice(n, 5000, replace=False).astype(np.uint64)
    for ep in range(3):
        d = np.full((hot.size, 16), 0x30 + ep, np.uint8)
        rc, _ = tab.update_batch(hot, 16 * ep, d, 10 + 10 * ep, 11 + 10 * ep)
        for k in hot:
            orc.update(int(k), 8, 16 * ep, bytes([0x30 + ep]) * 16, 10 + 10 * ep)
            orc.commit_update(int(k), 8, 11 + 10 * ep, 11 + 10 * ep)
    for k in hot[:500]:
        assert tab.update(int(k), 100, b"\x99" * 4, 40) == orc.update(int(k), 8, 100, b"\x99" * 4, 40)
    tab.sync()
    return tab, orc, hot, n


def test_probe_host_matches_device_and_oracle(chains):
    tab, orc, hot, n = chains
    rng = np.random.default_rng(42)
    # > 3 chunks of 2^17 so every lane is reused
    keys = np.concatenate([rng.integers(0, n + 1000, 450000), hot]).astype(np.uint64)
    rids = rng.integers(0, 45, keys.size).astype(np.uint32)
    out_h, rows_h = tab.probe_host(keys, read_ids=rids)
    out_d, rows_d = tab.probe(keys, read_ids=rids)
    assert (out_h == out_d).all()
    assert (rows_h == rows_d).all()
    sel = rng.choice(keys.size, 60000, replace=False)
    check_probe(tab, orc, keys[sel], 8, read_ids=rids[sel])
    # outputs only, no rows
    out2, none = tab.probe_host(keys[:1000], read_ids=rids[:1000], records=False)
    assert none is None and (out2 == out_h[:1000]).all()


def test_probe_host_lean_layout_into_pinned_buffers(chains):
    """bench.py's end-to-end leg: stage_set_output_layout(1008, 16) applies to stage_probe_host
    (packed 16-B stage_probe_out16 records, 1008-B rows) and the results land in caller-owned
    pinned arrays; equal to the device-buffer probe of the same keys in the same layout and, in
    the fields both layouts carry, to the default layout."""
    tab, orc, hot, n = chains
    rng = np.random.default_rng(44)
    keys = np.concatenate([rng.integers(0, n + 1000, 300000), hot]).astype(np.uint64)
    rids = rng.integers(0, 45, keys.size).astype(np.uint32)
    out32, rows32 = tab.probe_host(keys, read_ids=rids)
    try:
        tab.set_output_layout(1008, 16)
        assert tab.stride == 1008
        pk = stage.pinned_empty(keys.size, np.uint64)
        pk[:] = keys
        out = stage.pinned_empty(keys.size, stage.PROBE_OUT16_DTYPE)
        rows = stage.pinned_empty((keys.size, 1008), np.uint8)
        o2, r2 = tab.probe_host(pk, read_ids=rids, out=out, rows=rows)
        assert o2 is out and r2 is rows
        od, rd = tab.probe(keys, read_ids=rids)
        assert od.dtype == stage.PROBE_OUT16_DTYPE
        assert (out == od).all() and (rows == rd).all()
        for f in ("status", "flags", "hops", "cstamp", "rec_cstamp", "copy_sstamp"):
            assert (out[f] == out32[f]).all(), f
        assert (rows == rows32[:, :1008]).all()
    finally:
        tab.set_output_layout(0, 32)


@pytest.mark.parametrize("resident", [False, True])
def test_reader_concurrent_threads_match_oracle(chains, resident):
    tab, orc, hot, n = chains
    rng = np.random.default_rng(43)
    keys = np.concatenate([rng.integers(0, n + 100, 6000), rng.choice(hot, 2000)]).astype(np.uint64)
    rids = rng.integers(0, 45, keys.size).astype(np.uint32)
    o_out, o_rec = orc.read_batch(keys, 8, rids)
    # resident: a 256-slot ring laps ~30 times; 4 waves
    r = tab.reader(max_batch=64, max_wait_us=200, resident=True, ring_slots=256, waves=4) if resident else \
        tab.reader(max_batch=64, max_wait_us=200)
    got_out = np.zeros(keys.size, stage.PROBE_OUT_DTYPE)
    got_rec = np.zeros((keys.size, orc.row), np.uint8)
    T = 16
    errs = []

    def work(t):
        try:
            for i in range(t, keys.size, T):
                got_out[i], got_rec[i] = r.read(int(keys[i]), int(rids[i]))
        except Exception as e:  # surfaced below
            errs.append(e)

    th = [threading.Thread(target=work, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs
    for f in ("status", "hops", "cstamp", "rec_cstamp", "copy_sstamp"):
        assert (got_out[f] == o_out[f]).all(), f
    assert ((got_out["flags"] & 1) == o_out["copy_present"]).all()
    assert (got_rec == o_rec).all()
    st = r.stats()
    assert st["reads"] == keys.size
    assert st["batches"] < keys.size  # coalesced batches / resident instances
    r.close()


def test_reader_single_caller_and_stale_image(gpu):
    tab = stage.Table(key_width=4)
    tab.load_ycsb(0, 1000, 4)
    tab.sync()
    r = tab.reader(max_batch=8, max_wait_us=10)
    out, row = r.read(7)
    assert out["status"] == stage.ST_LATEST and row[0] == 7 and (row[8:1008] == 7).all()
    out, row = r.read(5000)
    assert out["status"] == stage.ST_NOT_FOUND
    assert tab.update(7, 0, b"\x01", 5) == stage.RC_OK
    with pytest.raises(RuntimeError):
        r.read(7)  # host wrote since the last publish
    tab.sync()
    out, row = r.read(7, read_id=10)
    assert out["status"] == stage.ST_COPY and row[8] == 7
    r.close()


def test_resident_reader_single_caller_lifetimes_and_stale_image(gpu):
    tab = stage.Table(key_width=4)
    tab.load_ycsb(0, 1000, 4)
    tab.sync()
    orc = O.OracleTree()
    orc.load_ycsb(0, 1000, 4, 0)
    # 1-ms instances: reads cross many instance boundaries (positions carried over)
    r = tab.reader(resident=True, ring_slots=128, waves=2, life_us=1000)
    keys = np.array(list(range(0, 1200, 3)), np.uint64)
    o_out, o_rec = orc.read_batch(keys, 4, np.full(keys.size, 0xFFFFFFFE, np.uint32))
    for i, k in enumerate(keys):
        out, row = r.read(int(k))
        assert out["status"] == o_out["status"][i] and (row == o_rec[i]).all(), int(k)
    assert r.stats()["reads"] == keys.size
    assert tab.update(7, 0, b"\x01", 5) == stage.RC_OK
    import time
    time.sleep(0.05)  # the keeper sees the unpublished write at its next relaunch
    with pytest.raises(RuntimeError):
        r.read(7)
    r.close()
    tab.sync()
    r = tab.reader(resident=True, ring_slots=64, waves=1)
    out, row = r.read(7, read_id=10)
    assert out["status"] == stage.ST_COPY and row[8] == 7
    r.close()
    with pytest.raises(RuntimeError):  # ring size must be a multiple of 64 * waves
        tab.reader(resident=True, ring_slots=192, waves=2)


def test_resident_reader_variable_length_keys(gpu):
    tab = stage.Table(payload_size=8, leaf_node_size=4096, split_threshold=3072, merge_threshold=1024, key_width=0)
    keys = [b"a", b"ab", b"abc", b"b", b"zz", b"k000", b"k001"]
    for i, k in enumerate(keys):
        assert tab.insert_key(k, bytes([i]) * 8, commit_id=1) == stage.RC_OK
    tab.sync()
    r = tab.reader(resident=True, ring_slots=64, waves=1)
    for i, k in enumerate(keys):
        out, row = r.read(int.from_bytes(k, "little"), key_size=len(k))
        assert out["status"] == stage.ST_LATEST and row[8] == i, k
    out, _ = r.read(int.from_bytes(b"abcd", "little"), key_size=4)
    assert out["status"] == stage.ST_NOT_FOUND
    r.close()
