"""CPU: the RecordLocation mapping (record_location.h:13-42) of SURVEY §8(f) row 3.

The product's host table names every record by its RecordLocation handle (the reference's
indirection offset + 1: one location per Insert attempt, BTree::RecordIndirectLocation
b_tree.cpp:1865-1866) and repoints it on every split (LeafNode::CopyFrom b_tree.cpp:1520-1527).
Checked against the oracle, which keeps the reference's location objects: the handles of the
leaf images' loc_ptr, handle -> (leaf, slot) after the load, again after further inserts split
the leaves (every record still found under its handle: the key at the resolved slot is the
record's key), after deletes (a split drops a deleted record and its location dangles), after
an aborted insert, and through an export -> import round trip.
"""
import numpy as np

import oracle_lib as O
import stage
from test_leaf_images import assert_same_images


def _check_same(tab, orc, handles):
    lf, sl = tab.resolve_locations(handles)
    olf, osl = orc.resolve_locations(handles)
    assert (lf == olf).all() and (sl == osl).all()
    return lf, sl


def _key_at(tab, lf, sl):
    rc, sc, meta, keyw = tab.export_leaves()
    ok = lf != 0xFFFFFFFF
    out = np.full(lf.size, ~np.uint64(0), np.uint64)
    out[ok] = keyw[lf[ok], sl[ok]]
    live = np.zeros(lf.size, bool)
    live[ok] = meta[lf[ok], sl[ok]] != 0
    return out, live


def test_handles_follow_records_through_splits():
    rng = np.random.default_rng(5)
    base = np.arange(0, 400_000, 4, dtype=np.uint64)
    tab, orc = stage.Table(key_width=8), O.OracleTree()
    assert tab.load_keys(base, 8, mode=1) == base.size
    assert orc.load_keys(base, 8, 1) == base.size
    h, lf, sl = tab.export_locations()
    assert h.size == base.size and orc.location_count() >= h.size
    olf, osl = orc.resolve_locations(h)
    assert (lf == olf).all() and (sl == osl).all()
    keys0, live0 = _key_at(tab, lf, sl)
    assert live0.all()
    # leaf images carry the handles as loc_ptr, byte-identical to the oracle's
    assert_same_images(tab, orc)
    # more inserts split most leaves; every old handle still names its record
    more = rng.permutation(np.arange(1, 400_000, 4, dtype=np.uint64))[:60_000]
    for k in more:
        assert tab.insert(int(k), 8, gen_rowid=int(k), mode=1) == orc.insert(int(k), 8, O.payload(int(k), 1).tobytes())
    lf2, sl2 = _check_same(tab, orc, h)
    keys2, live2 = _key_at(tab, lf2, sl2)
    assert (keys2 == keys0).all() and live2.all()
    assert (lf2 != lf).mean() > 0.5  # most records moved
    # deletes: a deleted record keeps its slot until a split drops it (its location dangles)
    dels = rng.choice(base, 3000, replace=False)
    for k in dels:
        assert tab.delete(int(k), 9) == orc.delete(int(k), 8, 9)
    more2 = rng.permutation(np.arange(2, 400_000, 4, dtype=np.uint64))[:60_000]
    for k in more2:
        assert tab.insert(int(k), 8, gen_rowid=int(k), mode=1) == orc.insert(int(k), 8, O.payload(int(k), 1).tobytes())
    lf3, sl3 = _check_same(tab, orc, h)
    gone = lf3 == 0xFFFFFFFF
    assert gone.sum() > 0 and np.isin(base[gone], dels).all()
    keys3, live3 = _key_at(tab, lf3, sl3)
    assert (keys3[live3] == keys0[live3]).all()
    assert np.isin(base[~live3], dels).all()  # dangling or still in its slot with meta 0
    assert_same_images(tab, orc)
    # all live handles of both sides agree
    ha, la, sa = tab.export_locations()
    olf, osl = orc.resolve_locations(ha)
    assert (la == olf).all() and (sa == osl).all()


def test_aborted_insert_loses_its_location():
    tab, orc = stage.Table(key_width=8), O.OracleTree()
    tab.load_ycsb(0, 1000, 8)
    orc.load_ycsb(0, 1000, 8)
    k = (5000).to_bytes(8, "little")
    assert tab.insert_key(k, bytes(1000), 7) == 1 and orc.insert(k, 8, bytes(1000), 7) == 1
    h, lf, sl = tab.export_locations()
    new = h.max()
    assert tab.abort_insert_key(k) == 1 and orc.abort_insert(k, 8) == 1
    lf2, sl2 = _check_same(tab, orc, np.array([new], np.uint64))
    assert lf2[0] == 0xFFFFFFFF and sl2[0] == 0xFFFF


def test_locations_survive_export_import():
    orc = O.OracleTree()
    orc.load_ycsb(0, 200_000, 8, 1)
    rng = np.random.default_rng(2)
    for k in rng.choice(200_000, 2000, replace=False):
        orc.delete(int(k), 8, 3)
    blocks, seps, lens = orc.export_leaf_images()
    tab = stage.Table(key_width=8)
    tab.import_leaf_images(blocks, seps, lens)
    h, lf, sl = tab.export_locations()
    olf, osl = orc.resolve_locations(h)
    assert (lf == olf).all() and (sl == osl).all()
    assert h.size >= 198_000
    assert_same_images(tab, orc)
