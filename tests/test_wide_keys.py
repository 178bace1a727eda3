"""CPU: tables with keys above 8 bytes (TPC-C composite keys).

TPC-C keys are structs of int64 fields (tpcc_record.h: DistrictKey 16 B, CustomerKey 24 B,
OrderLineKey 32 B) compared by the reference's signed-byte KeyCompare over the raw bytes.  The
product's host table must lay such tables out exactly like the oracle (BTree insert/split
path), export the same reference-format leaf blocks and route every key to the same leaf.
"""
import numpy as np
import pytest

import oracle_lib as O
import stage
from test_host_layout import compare_layout


def composite_keys(fields):
    """rows of int64 fields -> (n, 8*len(fields)) uint8 key bytes (little-endian structs)"""
    a = np.ascontiguousarray(np.asarray(fields, dtype=np.int64))
    return a.view(np.uint8).reshape(a.shape[0], -1)


def tpcc_like(width, n_w=2, seed=0):
    rng = np.random.default_rng(seed)
    if width == 16:    # StockKey {S_W_ID, S_I_ID}, loader order: warehouse, item
        f = [(w, i) for w in range(1, n_w + 1) for i in range(1, 8001)]
    elif width == 24:  # CustomerKey {C_W_ID, C_D_ID, C_ID}
        f = [(w, d, c) for w in range(1, n_w + 1) for d in range(1, 11) for c in range(1, 601)]
    else:              # OrderLineKey {W, D, O, NUMBER}
        f = [(w, d, o, ln) for w in range(1, n_w + 1) for d in range(1, 11) for o in range(1, 151)
             for ln in range(1, 1 + int(rng.integers(5, 16)))]
    return composite_keys(f)


def build(width, payload_size, keys, seed=1):
    rng = np.random.default_rng(seed)
    pays = rng.integers(0, 256, (keys.shape[0], payload_size), dtype=np.uint8)
    tab = stage.Table(payload_size=payload_size, key_width=width)
    rc, ins = tab.load_rows(keys, pays, commit_id=0)
    assert ins == keys.shape[0], np.unique(rc, return_counts=True)
    orc = O.OracleTree(payload_size=payload_size, key_pad=(width + 7) // 8 * 8)
    for k, p in zip(keys, pays):
        assert orc.insert(k.tobytes(), width, p.tobytes()) == stage.RC_OK
    return tab, orc, pays


@pytest.mark.parametrize("width,payload", [(16, 320), (24, 600), (32, 60)])
def test_wide_layout_and_images_match_oracle(width, payload):
    keys = tpcc_like(width)
    tab, orc, _ = build(width, payload, keys)
    assert tab.stats()["leaves"] == orc.stats()["leaves"] > 1
    compare_layout(tab, orc)
    b, sk, sl = tab.export_leaf_images()
    ob, osk, osl = orc.export_leaf_images(kwords=tab.key_words)
    assert (b == ob).all() and (sl == osl).all() and (sk == osk).all()


@pytest.mark.parametrize("width,payload", [(16, 320), (32, 60)])
def test_wide_traversal_matches_oracle(width, payload):
    keys = tpcc_like(width, n_w=1)
    tab, orc, _ = build(width, payload, keys)
    rng = np.random.default_rng(3)
    probe = np.concatenate([keys[rng.choice(keys.shape[0], 400)],
                            rng.integers(0, 256, (200, width), dtype=np.uint8)])
    for le in (True, False):
        got = tab.traverse(probe, le_child=le)
        exp = np.array([orc.traverse(k.tobytes(), width, le) for k in probe])
        assert (got == exp).all()


def test_wide_writes_and_snapshot_round_trip():
    keys = tpcc_like(16)
    tab, orc, _ = build(16, 320, keys)
    rng = np.random.default_rng(4)
    for k in keys[rng.choice(keys.shape[0], 500, replace=False)]:
        d = rng.integers(0, 256, 8, dtype=np.uint8).tobytes()
        assert tab.update_key(k.tobytes(), 4, d, 7) == orc.update(k.tobytes(), 16, 4, d, 7)
        assert tab.commit_update_key(k.tobytes(), 8, 8) == orc.commit_update(k.tobytes(), 16, 8, 8)
    for k in keys[rng.choice(keys.shape[0], 40, replace=False)]:
        assert tab.delete_key(k.tobytes(), 9) == orc.delete(k.tobytes(), 16, 9)
    # more rows (new warehouse) force splits
    more = composite_keys([(3, i) for i in range(1, 3001)])
    pays = rng.integers(0, 256, (more.shape[0], 320), dtype=np.uint8)
    tab.load_rows(more, pays)
    for k, p in zip(more, pays):
        orc.insert(k.tobytes(), 16, p.tobytes())
    compare_layout(tab, orc)
    blocks, sk, sl = orc.export_leaf_images(kwords=2)
    t2 = stage.Table(payload_size=320, key_width=16)
    assert t2.import_leaf_images(blocks, sk, sl) > 0
    compare_layout(t2, orc)
    b2, sk2, sl2 = t2.export_leaf_images()
    assert (b2 == blocks).all() and (sk2 == sk).all() and (sl2 == sl).all()


def test_wide_key_width_is_enforced():
    tab = stage.Table(payload_size=64, key_width=16)
    assert tab.insert_key(b"x" * 15, b"\0" * 64) == stage.RC_INVALID
    assert tab.insert_key(b"x" * 16, b"\0" * 64) == stage.RC_OK
    assert tab.insert_key(b"x" * 16, b"\0" * 64) == stage.RC_KEY_EXISTS
    with pytest.raises(stage.StageError):
        stage.Table(payload_size=64, key_width=33)
