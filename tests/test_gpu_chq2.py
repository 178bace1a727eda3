"""GPU parity of CH-benCHmark Q2 (RunQuery2, benchmark/tpcc/tpcc_new_order.cpp:608-982) through
the path: stage_ch_query2 against the oracle's restatement (orc_ch_query2) on identically
loaded REGION / NATION / SUPPLIER / ITEM / STOCK tables -- visited suppliers, the stock each
one keeps, the I_DATA and quantity tests, aborts under version-chain visibility, and the
committed stock updates read back through both.  Since round 5 the selection (regions, nations,
suppliers, map segments) runs on the device and a batch synchronises once; the records land in
a page-locked `out` from the finishing kernel, or are copied once the count is known."""
import numpy as np
import pytest

import stage
from ch_data import ChTables

pytestmark = pytest.mark.gpu

FIELDS = ["supp_key", "s_w_id", "s_i_id", "s_quantity", "s_ytd", "s_order_cnt", "s_remote_cnt", "item_has_b",
          "update"]


def same(dev, orc):
    assert dev.size == orc.size
    a, b = np.sort(dev, order="supp_key"), np.sort(orc, order="supp_key")
    for f in FIELDS:
        bad = np.flatnonzero(a[f] != b[f])
        assert bad.size == 0, (f, a[bad[:3]], b[bad[:3]])


@pytest.fixture(scope="module")
def ch(gpu):
    c = ChTables(W=2, I=20000, qty=(1, 100))
    c.sync()
    return c


def test_q2_matches_oracle_all_regions(ch):
    for target in range(5):
        recs, ab = ch.query2(target)
        orecs, oab = ch.query2_oracle(target)
        assert ab == oab and not ab
        same(recs, orecs)
    assert recs.size > 1000 and recs["update"].sum() > 0 and recs["item_has_b"].sum() > 0


@pytest.mark.parametrize("pinned", [False, True])
def test_q2_batch_equals_single_queries(ch, pinned):
    rids = np.array([10, 0xFFFFFFFE, 3, 25, 0xFFFFFFFE, 7], np.uint32)
    # pinned: a page-locked `out` the records are copied into straight from the device
    out = stage.pinned_empty((rids.size, 1 << 14), stage.Q2_REC_DTYPE) if pinned else None
    for target in (0, 3):
        if out is not None:
            out[...] = np.zeros(1, stage.Q2_REC_DTYPE)[0]
        recs, ab = ch.query2_batch(rids, target, out=out)
        assert recs.shape[0] == rids.size
        if out is not None:
            assert recs.base is not None and np.shares_memory(recs, out)
        for q, r in enumerate(rids):
            one, ab1 = ch.query2(target, read_id=int(r))
            assert ab[q] == ab1
            if not ab1:
                same(recs[q], one)
                orecs, oab = ch.query2_oracle(target, int(r))
                assert not oab
                same(recs[q], orecs)


def test_q2_visibility_and_commit(ch):
    ostock = ch.orc["stock"]
    stock = ch.tables["stock"]
    recs, _ = ch.query2(3, read_id=10)
    # committed updates of some kept stocks (writer 20, commit 21), one left in flight (writer 30)
    kept = recs[recs["s_i_id"] > 0][:40]
    for r in kept[:39]:
        k = np.array([r["s_w_id"], r["s_i_id"]], np.int64).tobytes()
        d = np.array([int(r["s_quantity"]) % 7 + 1], np.int32).tobytes()
        assert stock.update_key(k, 0, d, 20) == ostock.update(k, 16, 0, d, 20) == stage.RC_OK
        assert stock.commit_update_key(k, 21, 21) == ostock.commit_update(k, 16, 21, 21)
    r = kept[39]
    k = np.array([r["s_w_id"], r["s_i_id"]], np.int64).tobytes()
    assert stock.update_key(k, 4, b"\x05\x00\x00\x00", 30) == ostock.update(k, 16, 4, b"\x05\x00\x00\x00", 30)
    stock.sync()
    brecs, babort = ch.query2_batch(np.array([10, 25, 40, 0xFFFFFFFE], np.uint32), 3)
    pout = stage.pinned_empty((4, 1 << 14), stage.Q2_REC_DTYPE)
    precs, pabort = ch.query2_batch(np.array([10, 25, 40, 0xFFFFFFFE], np.uint32), 3, out=pout)
    assert (pabort == babort).all() and precs.shape == brecs.shape
    for q in range(4):
        if not babort[q]:
            assert (precs[q] == brecs[q]).all()
    for q, rid in enumerate((10, 25, 40, 0xFFFFFFFE)):  # rid 10: retired versions with begin 0 -> FAILURE -> abort
        recs, ab = ch.query2(3, read_id=rid)
        orecs, oab = ch.query2_oracle(3, read_id=rid)
        assert ab == oab == babort[q], rid
        if not ab:
            same(recs, orecs)
            same(brecs[q], orecs)
    assert ch.query2(3, read_id=10)[1]  # the abort case is exercised
    # commit path: the transaction's updates through the device write path, mirrored on the oracle
    rid, cid = 50, 51
    recs, ab = ch.query2(3, read_id=rid, commit_id=cid)
    assert not ab
    upd = recs[recs["update"] == 1]
    assert upd.size > 0
    for r in upd:
        k = np.array([r["s_w_id"], r["s_i_id"]], np.int64).tobytes()
        d = np.array([r["s_quantity"] + 50, r["s_ytd"], r["s_order_cnt"], r["s_remote_cnt"]], np.int32).tobytes()
        rc = ostock.update(k, 16, 0, d, rid)
        if rc == stage.RC_OK:
            rc = ostock.commit_update(k, 16, cid, cid)
        assert rc == r["update_rc"], (r, rc)
    keys = np.stack([upd["s_w_id"], upd["s_i_id"]], 1).astype(np.int64)
    kb = np.ascontiguousarray(keys).view(np.uint8).reshape(-1, 16)
    for read_id in (40, 60):
        out, rows = stock.probe(kb, read_ids=np.full(len(kb), read_id, np.uint32))
        o_out, o_rec = ostock.read_batch_k(kb, np.full(len(kb), read_id, np.uint32))
        assert (out["status"] == o_out["status"]).all()
        assert (rows[:, :ostock.row] == o_rec).all()
    recs2, ab2 = ch.query2(3, read_id=60)
    orecs2, oab2 = ch.query2_oracle(3, read_id=60)
    assert ab2 == oab2
    if not ab2:
        same(recs2, orecs2)


def test_q2_batch_many_read_ids(ch):
    """40 queries: the folded revisit evaluates read ids 16 at a time per probe (three groups, the
    last partial); every query's records and abort flag equal its single-query run's."""
    rng = np.random.default_rng(5)
    rids = rng.choice(np.array([3, 10, 25, 40, 60, 0xFFFFFFFE], np.uint32), 40)
    out = stage.pinned_empty((rids.size, 1 << 14), stage.Q2_REC_DTYPE)
    recs, ab = ch.query2_batch(rids, 3, out=out)
    seen = {}
    for q, r in enumerate(rids):
        if int(r) not in seen:
            seen[int(r)] = ch.query2(3, read_id=int(r))
        one, ab1 = seen[int(r)]
        assert ab[q] == ab1, (q, r)
        if not ab1:
            same(recs[q], one)


def test_q2_batch_async_two_in_flight(ch):
    """stage_ch_query2_batch_async: two batches in flight (slots 0 and 1, different targets and
    read ids), waited for out of order, each equal to the synchronous batch of the same queries;
    a busy slot, a pageable `out` and a wait on an idle slot are refused."""
    ra = np.array([10, 0xFFFFFFFE, 25], np.uint32)
    rb = np.array([40, 3, 0xFFFFFFFE, 60], np.uint32)
    oa = stage.pinned_empty((ra.size, 1 << 14), stage.Q2_REC_DTYPE)
    ob = stage.pinned_empty((rb.size, 1 << 14), stage.Q2_REC_DTYPE)
    for rep in range(3):  # the third round replays both slots' graphs
        oa[...] = np.zeros(1, stage.Q2_REC_DTYPE)[0]  # the records must come from this round's emit
        ob[...] = np.zeros(1, stage.Q2_REC_DTYPE)[0]
        ja = ch.query2_batch_async(ra, oa, 0, 3)
        jb = ch.query2_batch_async(rb, ob, 1, 0)
        with pytest.raises(stage.StageError):
            ch.query2_batch_async(ra, oa, 0, 3)
        recs_b, ab_b = jb.wait()
        recs_a, ab_a = ja.wait()
        for rids, target, recs, ab in ((ra, 3, recs_a, ab_a), (rb, 0, recs_b, ab_b)):
            srecs, sab = ch.query2_batch(rids, target)
            assert (ab == sab).all() and recs.shape == srecs.shape, rep
            for q in range(rids.size):
                if not ab[q]:
                    same(recs[q], srecs[q])
    with pytest.raises(stage.StageError):
        ch.query2_batch_async(ra, np.zeros((ra.size, 1 << 14), stage.Q2_REC_DTYPE), 0, 3)
    with pytest.raises(stage.StageError):
        stage.table.Q2Batch(ch.tables["stock"], 1, ob, rb.size).wait()


def test_q2_async_split_emit_sizes(ch):
    """Async batches finish their records into the slot's device buffer and emit them to the
    page-locked `out` from a side stream, the emit's grid shaped by the last call's count: a batch
    with more suppliers than the previous one (target 3 after 0 ... and back), one query and many,
    and a narrow `out` (max_per_query below the count) each equal the synchronous batch."""
    for rids, targets, width in ((np.array([25], np.uint32), (1, 3, 0, 3), 1 << 14),
                                 (np.arange(3, 43, dtype=np.uint32), (3, 2), 1 << 14),
                                 (np.array([10, 0xFFFFFFFE], np.uint32), (3,), 100)):
        out = stage.pinned_empty((rids.size, width), stage.Q2_REC_DTYPE)
        for t in targets:
            out[...] = np.zeros(1, stage.Q2_REC_DTYPE)[0]
            recs, ab = ch.query2_batch_async(rids, out, 1, t).wait()
            srecs, sab = ch.query2_batch(rids, t)
            assert (ab == sab).all()
            n = min(srecs.shape[1], width)
            assert recs.shape[1] == n and np.shares_memory(recs, out)
            for q in range(rids.size):
                if not ab[q]:  # the same records in the same (visit) order, the first n of them
                    for f in FIELDS:
                        assert (recs[q][f] == srecs[q][:n][f]).all(), (t, q, f)


def test_q2_place_forms_agree(ch, monkeypatch):
    """The one-launch selection placement (q2_place, SUPPLIER tables of up to 1024 chunks) and the
    three-kernel form larger tables take (q2_sel_start, q2_sel_place, q2_gather;
    STAGE_Q2_PLACE_CHUNKS=0 forces it here) give the same records, synchronous and batched."""
    rids = np.array([10, 0xFFFFFFFE, 25], np.uint32)
    got = {}
    for lim in ("1024", "0"):
        monkeypatch.setenv("STAGE_Q2_PLACE_CHUNKS", lim)
        got[lim] = [ch.query2(t) for t in (0, 3)] + [ch.query2_batch(rids, 3)]
    for (ra, aa), (rb, ab) in zip(got["1024"], got["0"]):
        assert np.all(np.asarray(aa) == np.asarray(ab)) and ra.shape == rb.shape
        assert (ra == rb).all()


def test_q2_batches_on_different_streams(ch):
    """The two async slots and a synchronous batch share the tables' device scratch:
    batches enqueued on different streams while another is in flight wait for it on the device,
    so each still equals its batch run alone."""
    ra = np.array([10, 0xFFFFFFFE, 25], np.uint32)
    rb = np.array([40, 3, 0xFFFFFFFE, 60], np.uint32)
    rc = np.array([25, 0xFFFFFFFE], np.uint32)
    ref = {k: ch.query2_batch(r, t) for k, (r, t) in {"a": (ra, 3), "b": (rb, 0), "c": (rc, 1)}.items()}
    s1, s2, s3 = stage.Stream(), stage.Stream(), stage.Stream()
    oa = stage.pinned_empty((ra.size, 1 << 14), stage.Q2_REC_DTYPE)
    ob = stage.pinned_empty((rb.size, 1 << 14), stage.Q2_REC_DTYPE)
    for rep in range(3):
        oa[...] = np.zeros(1, stage.Q2_REC_DTYPE)[0]
        ob[...] = np.zeros(1, stage.Q2_REC_DTYPE)[0]
        ja = ch.query2_batch_async(ra, oa, 1, 3, stream=s1.ptr)
        got_c = ch.query2_batch(rc, 1, stream=s3.ptr)  # synchronous (slot 0), slot 1 busy on s1
        jb = ch.query2_batch_async(rb, ob, 0, 0, stream=s2.ptr)  # slot 1 may still be busy on s1
        got = {"b": jb.wait(), "a": ja.wait(), "c": got_c}
        for k, (recs, ab) in got.items():
            srecs, sab = ref[k]
            assert (ab == sab).all() and recs.shape == srecs.shape, (rep, k)
            for q in range(ab.size):
                if not ab[q]:
                    same(recs[q], srecs[q])
