"""GPU: BTree::Read(..., is_for_update = true) -- a transaction reading its own record -- through
stage_probe_batch_ex and both single-key readers, against the oracle's orc_read_fu, bit-exact.

Reference rule (b_tree.cpp:2066-2129, executor.h:374-454): the overwrite-copy branch of
BTree::Read is taken only when `meta->IsInserting() && !is_for_update` (:2087), so a for-update
read of an in-flight record gets the leaf's patched image (Record::New, cstamp = the reader's id,
no AddReader, :2114-2120) -- also for an uncommitted insert, which the ordinary rule returns as
nothing -- and the executor skips PerformRead (:388).  The device marks such records with
STAGE_FLAG_FOR_UPDATE; records that are not in flight give the ordinary outcome.  The
reference's own assertions on this path are MVCCTest's (tests/golden, test_gpu_scenarios.py)."""
import numpy as np
import pytest

import oracle_lib as O
import stage

pytestmark = pytest.mark.gpu
FU = 2  # STAGE_FLAG_FOR_UPDATE


def key8(k):
    return int(k).to_bytes(8, "little")


@pytest.fixture(scope="module")
def states(gpu):
    """50K rows in every state a for-update read distinguishes: committed chains, in-flight
    updates (copy present) on top of chains, in-flight updates patched again in place by their
    writer, uncommitted inserts (no copy) and their owner's in-place patches, deleted records."""
    n = 50000
    tab = stage.Table(key_width=8, payload_size=200)
    orc = O.OracleTree(payload_size=200)
    tab.load_ycsb(0, n, 8, mode=1)
    orc.load_ycsb(0, n, 8, 1)
    rng = np.random.default_rng(51)
    hot = rng.choice(n, 4000, replace=False)
    cid = 10
    for rnd in range(3):
        for k in hot[: 4000 - 1000 * rnd]:
            d = bytes([rnd * 29 + 5]) * 40
            assert tab.update(int(k), 40 * rnd, d, cid) == orc.update(int(k), 8, 40 * rnd, d, cid)
            assert tab.commit_update(int(k), cid + 1, cid + 1) == orc.commit_update(int(k), 8, cid + 1, cid + 1)
        cid += 5
    inflight = hot[:1500]
    for k in inflight:
        d = bytes([0xEE]) * 30
        assert tab.update(int(k), 7, d, cid) == orc.update(int(k), 8, 7, d, cid) == stage.RC_OK
    for k in inflight[:500]:  # the writer patches its own in-flight record again (is_for_update)
        d = bytes([0x5A]) * 12
        assert tab.update_key_owned(key8(k), 90, d, cid) == orc.update_owned(int(k), 8, 90, d, cid) == stage.RC_OK
    ins = np.arange(n + 10, n + 1010, dtype=np.uint64)
    for k in ins:  # uncommitted inserts of writer cid + 1
        p = bytes([int(k) & 0xFF]) * 200
        assert tab.insert_key_inflight(key8(k), p, cid + 1) == orc.insert_inflight(int(k), 8, p, cid + 1)
    for k in ins[:300]:
        d = bytes([0x33]) * 16
        assert tab.update_key_owned(key8(k), 0, d, cid + 1) == orc.update_owned(int(k), 8, 0, d, cid + 1)  # 1 or 7
    for k in rng.choice(n, 300, replace=False):
        assert tab.delete(int(k), cid) == orc.delete(int(k), 8, cid)
    tab.sync()
    keys = np.concatenate([hot, ins, rng.integers(0, n + 2000, 6000)]).astype(np.uint64)
    return tab, orc, keys, cid


def oracle_reads(orc, keys, rids, fu):
    o_out = np.zeros(len(keys), O.READ_OUT_DTYPE)
    o_rec = np.zeros((len(keys), orc.row), np.uint8)
    for i, k in enumerate(keys):
        o_out[i], o_rec[i] = orc.read(int(k), 8, int(rids[i]), for_update=bool(fu[i]))
    return o_out, o_rec


def compare(out, rows, o_out, o_rec, fu, row_bytes):
    for f in ("status", "hops", "cstamp", "rec_cstamp", "copy_sstamp"):
        bad = np.nonzero(out[f] != o_out[f])[0]
        assert bad.size == 0, (f, bad[:5], out[f][bad[:5]], o_out[f][bad[:5]], fu[bad[:5]])
    assert ((out["flags"] & 1) == o_out["copy_present"]).all()
    assert (((out["flags"] & FU) != 0) == (np.asarray(fu) != 0)).all()
    bad = np.nonzero((rows[:, :row_bytes] != o_rec).any(axis=1))[0]
    assert bad.size == 0, (bad[:5], out["status"][bad[:5]], fu[bad[:5]])


def test_probe_batch_for_update_matches_oracle(states):
    tab, orc, keys, cid = states
    rng = np.random.default_rng(52)
    for rid_mode in ("newest", "writer", "mixed"):
        if rid_mode == "newest":
            rids = np.full(keys.size, 0xFFFFFFFE, np.uint32)
        elif rid_mode == "writer":
            rids = np.full(keys.size, cid + 1, np.uint32)
        else:
            rids = rng.integers(0, cid + 4, keys.size).astype(np.uint32)
        fu = (rng.random(keys.size) < 0.5).astype(np.uint8)
        out, rows = tab.probe(keys, read_ids=rids, for_update=fu)
        o_out, o_rec = oracle_reads(orc, keys, rids, fu)
        compare(out, rows, o_out, o_rec, fu, orc.row)
    # the cases that differ from the ordinary read actually occur
    fu = np.ones(keys.size, np.uint8)
    rids = np.full(keys.size, cid + 1, np.uint32)
    out, _ = tab.probe(keys, read_ids=rids, for_update=fu)
    plain, _ = tab.probe(keys, read_ids=rids)
    copy_to_latest = np.count_nonzero((plain["status"] == stage.ST_COPY) & (out["status"] == stage.ST_LATEST))
    assert copy_to_latest >= 1500, copy_to_latest  # every in-flight update (keys may repeat)
    ins = slice(4000, 5000)  # the uncommitted inserts: nothing for others, the record for its writer
    assert (plain["status"][ins] == stage.ST_NOT_FOUND).all() and (out["status"][ins] == stage.ST_LATEST).all()


def test_probe_batch_for_update_all_off_equals_plain(states):
    tab, orc, keys, cid = states
    rids = np.random.default_rng(53).integers(0, cid + 4, keys.size).astype(np.uint32)
    a, ra = tab.probe(keys, read_ids=rids, for_update=np.zeros(keys.size, np.uint8))
    b, rb = tab.probe(keys, read_ids=rids)
    assert (a == b).all() and (ra == rb).all()


def test_probe_batch_for_update_ragged_and_empty(states):
    tab, orc, keys, cid = states
    for n in (0, 1, 63, 64, 65, 257):
        k = keys[:n]
        fu = np.ones(n, np.uint8)
        rids = np.full(n, cid + 1, np.uint32)
        out, rows = tab.probe(k, read_ids=rids, for_update=fu)
        o_out, o_rec = oracle_reads(orc, k, rids, fu)
        if n:
            compare(out, rows, o_out, o_rec, fu, orc.row)


def test_for_update_needs_32_byte_records(gpu):
    tab = stage.Table(key_width=8)  # the YCSB geometry (16-B records need 64-slot leaves)
    tab.load_ycsb(0, 1000, 8)
    tab.sync()
    tab.set_output_layout(0, 16)
    with pytest.raises(RuntimeError):
        tab.probe(np.arange(10, dtype=np.uint64), for_update=np.ones(10, np.uint8))


@pytest.mark.parametrize("resident", [False, True])
def test_reader_for_update_matches_oracle(states, resident):
    tab, orc, keys, cid = states
    rng = np.random.default_rng(54)
    sample = rng.choice(keys, 600, replace=False)
    rids = rng.integers(0, cid + 4, sample.size).astype(np.uint32)
    fu = (rng.random(sample.size) < 0.5).astype(np.uint8)
    r = tab.reader(max_batch=64, max_wait_us=20, resident=resident, ring_slots=256, waves=4, life_us=2000) \
        if resident else tab.reader(max_batch=64, max_wait_us=20)
    try:
        out = np.zeros(sample.size, stage.PROBE_OUT_DTYPE)
        rows = np.zeros((sample.size, orc.row), np.uint8)
        for i, k in enumerate(sample):
            o, row, ident = r.read_ex(int(k), int(rids[i]), bool(fu[i]))
            out[i], rows[i] = o, row[:orc.row]
    finally:
        r.close()
    o_out, o_rec = oracle_reads(orc, sample, rids, fu)
    compare(out, rows, o_out, o_rec, fu, orc.row)
