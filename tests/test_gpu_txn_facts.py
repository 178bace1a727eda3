"""GPU: the facts the kept transaction manager reads through a Record, on device results
(include/stage_hip.h "what the kept transaction manager reads"; VERDICT r03 "What's missing" #1):

* stage_probe_identify and both single-key readers (stage_reader_read_ident) report the hit
  record's RecordLocation handle and next handle -- the loc_ptr / next_ptr BTree::Read puts into
  the Record (b_tree.cpp:2083, 2099) -- equal to the oracle's for latest, in-flight (overwrite
  copy), committed (TupleHeader) and aborted records;
* the location cells (RecordLocation::record_meta_ptr) follow records through splits and writes;
* the overwrite copies' transaction state (writer id, stamps, readers, dependency count,
  waiting) follows AddReader / IncreaseWRCount / DecreaseWRCount / UpdatePs and the writer's
  commit / abort -- also for copies the device write path created (their writer ids come back
  with the epoch's adoption)."""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
import stage
from stage.table import IDENT_DTYPE, NEXT_COPY, NEXT_INDEX_MASK, NEXT_KIND_MASK, NEXT_VERSION

pytestmark = pytest.mark.gpu

N = 20000


def scenario(tab, orc):
    """key 3 updated and committed, key 5 in flight (writer 8), key 7 updated then aborted, key 9
    updated twice (second in flight)"""
    for t, o in ((tab, None), (None, orc)):
        upd = (lambda k, b, w: t.update(k, 0, bytes([b]) * 100, w)) if t else \
              (lambda k, b, w: o.update(k, 8, 0, bytes([b]) * 100, w))
        com = (lambda k, c: t.commit_update(k, c, c)) if t else (lambda k, c: o.commit_update(k, 8, c, c))
        abt = (lambda k: t.abort_update_key(int(k).to_bytes(8, "little"))) if t else (lambda k: o.abort_update(k, 8))
        assert upd(3, 7, 1) == 1 and com(3, 2) == 1
        assert upd(5, 55, 8) == 1
        assert upd(7, 77, 10) == 1 and abt(7) == 1
        assert upd(9, 90, 11) == 1 and com(9, 12) == 1 and upd(9, 91, 13) == 1


@pytest.fixture(scope="module")
def tables(gpu):
    tab = stage.Table(key_width=8)
    tab.load_ycsb(0, N, 8, mode=0)
    tab.enable_location_cells()
    orc = O.OracleTree()
    orc.load_ycsb(0, N, 8, 0)
    scenario(tab, orc)
    tab.sync()
    return tab, orc


KEYS = [3, 5, 7, 9, 11, 123, N + 5]
RIDS = [0xFFFFFFFE, 20, 20, 20, 1, 20, 20]


def oracle_idents(orc, keys, rids):
    want = np.zeros(len(keys), IDENT_DTYPE)
    st = []
    for i, (k, r) in enumerate(zip(keys, rids)):
        o, _, _, loc, nxt = orc.read_ident(k, 8, r)
        want[i] = (loc, nxt)
        st.append(int(o["status"]))
    return want, st


def test_identify_matches_oracle(tables):
    tab, orc = tables
    out, ident = tab.identify(np.array(KEYS, np.uint64), np.array(RIDS, np.uint32))
    want, st = oracle_idents(orc, KEYS, RIDS)
    assert out["status"].tolist() == st
    assert (ident == want).all(), (ident, want)
    kinds = [int(x) & NEXT_KIND_MASK for x in ident["next"]]
    assert kinds[1] == NEXT_COPY and kinds[3] == NEXT_COPY  # in flight: the overwrite copy
    assert kinds[0] == NEXT_VERSION                          # committed: the newest TupleHeader
    assert ident["loc"][-1] == 0 and ident["next"][-1] == 0  # absent key


@pytest.mark.parametrize("resident", [False, True])
def test_readers_report_the_same_identity(tables, resident):
    tab, orc = tables
    want, _ = oracle_idents(orc, KEYS, RIDS)
    r = stage.Reader(tab, resident=resident, max_batch=64, ring_slots=1024, waves=4, life_us=2000)
    try:
        for i, (k, rid) in enumerate(zip(KEYS, RIDS)):
            out, _, ident = r.read_ident(k, rid)
            assert (int(ident["loc"]), int(ident["next"])) == (int(want[i]["loc"]), int(want[i]["next"])), (k, resident)
    finally:
        r.close()


def test_location_cells_follow_writes_and_splits(gpu):
    tab = stage.Table(key_width=8)
    tab.load_ycsb(0, 5000, 8, mode=0)
    tab.enable_location_cells()
    orc = O.OracleTree()
    orc.load_ycsb(0, 5000, 8, 0)
    scenario(tab, orc)
    # committed inserts next to hot keys: their leaves split after the cells were built
    for j in range(2000):
        k = ((5000 + j) << 8) | (j % 12)
        assert tab.insert(k, commit_id=0) == orc.insert(k, 8, bytes([k & 0xFF]) * 1000, 0)
    nloc = orc.location_count()
    for h in range(1, nloc + 1):
        meta, nxt = orc.location_meta(h)
        assert tab.location_cell(h) == (meta, nxt, h), h
    for k in (3, 5, 7, 9, 1000):  # the cell a key's Record names is the record's current metadata
        meta, loc, nxt = tab.record_meta(k)
        assert tab.location_cell(loc) == (meta, nxt, loc)


def test_copy_state_follows_the_pool_calls(tables):
    tab, orc = tables
    _, loc, nxt = tab.record_meta(5)
    assert nxt & NEXT_KIND_MASK == NEXT_COPY
    cid = nxt & NEXT_INDEX_MASK
    s = tab.copy_state(cid)
    assert (s["cstamp"], s["pstamp"], s["rstamp"], s["sstamp"], s["waiting"]) == (8, 8, 0, 0xFFFFFFFF, 0)
    assert s["reader_ids"] == [] and s["count"] == 0
    L = stage.lib()
    ok = ctypes.c_int(0)
    for rid in (21, 22):
        stage.table.check(L.stage_copy_add_reader(tab.h, cid, rid), "add_reader")
        stage.table.check(L.stage_copy_wr_count(tab.h, cid, 1, ctypes.byref(ok)), "wr+")
        assert ok.value == 1
    stage.table.check(L.stage_copy_wr_count(tab.h, cid, -1, ctypes.byref(ok)), "wr-")
    stage.table.check(L.stage_copy_update_ps(tab.h, cid, 30), "ps")
    s = tab.copy_state(cid)
    assert s["reader_ids"] == [21, 22] and s["readers"] == 2 and s["count"] == 1 and s["pstamp"] == 30
    # the oracle's pool agrees on the same header after the same calls
    ocid = nxt & NEXT_INDEX_MASK
    L2 = O.lib()
    for rid in (21, 22):
        L2.orc_copy_add_reader(orc.t, ocid, rid)
        L2.orc_copy_wr_count(orc.t, ocid, 1)
    L2.orc_copy_wr_count(orc.t, ocid, -1)
    L2.orc_copy_update_ps(orc.t, ocid, 30)
    assert orc.copy_state(ocid) == (s["cstamp"], 30, s["rstamp"], s["sstamp"], 2, 1, 0)
    assert orc.copy_readers(ocid) == [21, 22]
    # the aborted update's header stays in the pool, waiting: IncreaseWRCount is refused
    s7 = [s for s in (tab.copy_state(c) for c in range(cid + 3)) if s["cstamp"] == 10]
    assert len(s7) == 1 and s7[0]["waiting"] == 1 and s7[0]["sstamp"] == 0xFFFFFFFF


def test_device_epoch_copies_carry_their_writer_ids(gpu):
    tab = stage.Table(key_width=8)
    tab.load_ycsb(0, 50000, 8, mode=0)
    tab.sync()
    rng = np.random.default_rng(7)
    keys = rng.choice(50000, 3000, replace=False).astype(np.uint64)
    wid = (1000 + 2 * np.arange(keys.size)).astype(np.uint32)
    cid = np.where(np.arange(keys.size) % 3 == 0, 0, wid + 1).astype(np.uint32)  # every third in flight
    deltas = np.full((keys.size, 100), 0xAB, np.uint8)
    rc, ok = tab.update_batch_device(keys, 0, deltas, wid, cid)
    assert ok == int((rc == stage.RC_OK).sum()) > keys.size * 0.9  # NotNeeded where a row already holds 0xAB
    check = 0
    for i in range(0, keys.size, 7):
        if rc[i] != stage.RC_OK:
            continue
        meta, loc, nxt = tab.record_meta(int(keys[i]))
        if cid[i] == 0:  # in flight: the record names its copy, whose writer is this op's
            assert nxt & NEXT_KIND_MASK == NEXT_COPY
            s = tab.copy_state(nxt & NEXT_INDEX_MASK)
            assert s["cstamp"] == wid[i] and s["pstamp"] == wid[i] and s["waiting"] == 0
            check += 1
        else:            # committed in the epoch: the newest TupleHeader
            assert nxt & NEXT_KIND_MASK == NEXT_VERSION and meta & 0xFFFFFFFF == cid[i]
    assert check > 100
