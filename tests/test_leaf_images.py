"""CPU: leaf-level snapshot in the reference's block format.

The product exports its host layout as reference LeafNode blocks (header, StatusWord,
RecordMetadata array, records growing down); the oracle exports its own byte-level leaves in
the same canonical form (pointers zeroed, dead record bytes zeroed).  They must be equal byte
for byte, separators included.  Importing the oracle's blocks into an empty product table must
reproduce the same layout, and the host write path must continue identically afterwards.
No GPU is touched.
"""
import numpy as np
import pytest

import oracle_lib as O
import stage
from test_host_layout import compare_layout


def both_images(tab, orc):
    b, sk, sl = tab.export_leaf_images()
    ob, osk, osl = orc.export_leaf_images()
    return (b, sk, sl), (ob, osk, osl)


def assert_same_images(tab, orc):
    (b, sk, sl), (ob, osk, osl) = both_images(tab, orc)
    assert b.shape == ob.shape
    bad = np.nonzero((b != ob).any(axis=1))[0]
    assert bad.size == 0, (bad[:5], np.nonzero(b[bad[0]] != ob[bad[0]])[0][:16] if bad.size else None)
    assert (sl == osl).all() and (sk == osk).all()
    assert sl[-1] == 0xFFFF
    return ob, osk, osl


@pytest.mark.parametrize("n,ks,mode", [(1, 8, 0), (64, 8, 1), (100000, 4, 0), (60000, 8, 1)])
def test_export_matches_oracle_bytes(n, ks, mode):
    tab = stage.Table(key_width=ks)
    orc = O.OracleTree()
    tab.load_ycsb(0, n, ks, mode)
    orc.load_ycsb(0, n, ks, mode)
    blocks, _, _ = assert_same_images(tab, orc)
    # reference header facts: is_leaf, size, record count in the StatusWord
    assert (blocks[:, 8] == 1).all()
    assert (blocks[:, 16:20].copy().view(np.uint32).ravel() == 65536).all()
    counts = (blocks[:, 32:40].copy().view(np.uint64).ravel() >> np.uint64(44)) & np.uint64(0xFFFF)
    assert counts.sum() == n and counts.max() <= 63


def test_export_after_updates_deletes_random_order():
    rng = np.random.default_rng(51)
    keys = rng.choice(np.arange(1, 3000000, dtype=np.uint64) * 2654435761 % (1 << 62), 40000, replace=False)
    tab = stage.Table(key_width=8)
    orc = O.OracleTree()
    tab.load_keys(keys, 8, 1)
    orc.load_keys(keys, 8, 1)
    for k in keys[::13]:
        d = rng.integers(0, 256, 24, dtype=np.uint8).tobytes()
        assert tab.update(int(k), 8, d, 5) == orc.update(int(k), 8, 8, d, 5)
        if int(k) % 3:
            assert tab.commit_update(int(k), 6, 6) == orc.commit_update(int(k), 8, 6, 6)
    for k in keys[5::101]:
        assert tab.delete(int(k), 7) == orc.delete(int(k), 8, 7)
    assert_same_images(tab, orc)


def test_export_varlen_btreetest_geometry():
    tab = stage.Table(payload_size=8, leaf_node_size=4096, split_threshold=3072, merge_threshold=1024, key_width=0)
    orc = O.OracleTree(4096, 3072, 8, 1024)
    for i in range(20000):
        k = str(i).encode()
        kv = int.from_bytes(k, "little")
        assert tab.insert(kv, len(k), int(i).to_bytes(8, "little"), commit_id=1005) == stage.RC_OK
        orc.insert(k, len(k), int(i).to_bytes(8, "little"), 1005)
    assert_same_images(tab, orc)


@pytest.mark.parametrize("explicit_seps", [True, False])
def test_import_oracle_snapshot_then_continue_writing(explicit_seps):
    orc = O.OracleTree()
    orc.load_ycsb(0, 80000, 8, 1)
    blocks, sk, sl = orc.export_leaf_images()
    tab = stage.Table(key_width=8)
    if explicit_seps:
        assert tab.import_leaf_images(blocks, sk, sl) == 80000
    else:
        assert tab.import_leaf_images(blocks) == 80000
    compare_layout(tab, orc)
    b2, sk2, sl2 = tab.export_leaf_images()
    assert (b2 == blocks).all()
    if explicit_seps:
        assert (sk2 == sk).all() and (sl2 == sl).all()
    # traversal of present, absent and separator keys equals the oracle's
    probes = np.concatenate([np.arange(0, 90000, 7), sk[:-1]]).astype(np.uint64)
    if explicit_seps:
        for le in (True, False):
            got = tab.traverse(probes, le_child=le)
            exp = np.array([orc.traverse(int(k), 8, le) for k in probes])
            assert (got == exp).all()
        # the host write path continues exactly like the reference after the import
        more = np.arange(80000, 120000, dtype=np.uint64)
        tab.load_keys(more, 8, 1)
        orc.load_keys(more, 8, 1)
        for k in range(0, 120000, 17):
            d = bytes([k & 0xFF]) * 10
            assert tab.update(k, 30, d, 9) == orc.update(k, 8, 30, d, 9)
        compare_layout(tab, orc)
        assert_same_images(tab, orc)


def test_import_rejects_malformed_snapshots():
    orc = O.OracleTree()
    orc.load_ycsb(0, 5000, 8, 0)
    blocks, sk, sl = orc.export_leaf_images()

    def expect_fail(bl, k=sk, l=sl, table=None):
        t = table or stage.Table(key_width=8)
        with pytest.raises(stage.StageError):
            t.import_leaf_images(bl, k, l)

    expect_fail(blocks[:, :4096])                      # block size != leaf_node_size
    b = blocks.copy(); b[3, 8] = 0; expect_fail(b)     # not a leaf
    b = blocks.copy(); b[2, 39] |= 0x10; expect_fail(b)  # frozen bit 60 of the StatusWord
    b = blocks.copy(); b[1, 47] |= 0x80; expect_fail(b)  # control bit of slot 0's meta (in flight)
    k = sk.copy(); k[[4, 5]] = k[[5, 4]]; expect_fail(blocks, k, sl)  # separators out of order
    k = sk.copy(); k[3] = 0; expect_fail(blocks, k, sl)  # leaf 3's keys above its separator
    t = stage.Table(key_width=8); t.load_ycsb(0, 10, 8)
    expect_fail(blocks, table=t)                       # table not empty
    expect_fail(blocks, table=stage.Table(key_width=4))  # key width differs
