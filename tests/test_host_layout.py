"""CPU: the product's host write path reproduces the reference leaf layout exactly.

Compares stage (libstage_hip.so host table) with the oracle leaf by leaf: record counts,
sorted counts, every RecordMetadata word (offsets, key lengths, cstamps) and key bytes, and
the host traversal (BTree::TraverseToLeaf) leaf index for present, absent and separator keys.
No GPU is touched.
"""
import numpy as np
import pytest

import oracle_lib as O
import stage


def compare_layout(tab, orc):
    cap = tab.leaf_capacity
    rc, sc, meta, keyw = tab.export_leaves(cap)
    orc_rc, orc_sc, orc_meta, orc_keyw = orc.export_leaves(cap)
    assert rc.size == orc_rc.size
    assert (rc == orc_rc).all()
    assert (sc == orc_sc).all()
    assert (meta == orc_meta).all()
    assert (keyw == orc_keyw).all()


@pytest.mark.parametrize("n,ks", [(1, 4), (63, 8), (64, 8), (5000, 4), (200000, 8), (1000000, 4)])
def test_ycsb_layout_matches_oracle(n, ks):
    tab = stage.Table(key_width=ks)
    assert tab.load_ycsb(0, n, ks) == n
    orc = O.OracleTree()
    assert orc.load_ycsb(0, n, ks) == n
    compare_layout(tab, orc)
    s, so = tab.stats(), orc.stats()
    for k in ("leaves", "records", "sorted", "unsorted", "max_count"):
        assert s[k] == so[k]


def test_random_order_layout_matches_oracle():
    rng = np.random.default_rng(7)
    keys = rng.permutation(np.arange(300000, dtype=np.uint64) * 3 + 11)
    tab = stage.Table(key_width=8)
    orc = O.OracleTree()
    assert tab.load_keys(keys, 8, 1) == keys.size
    assert orc.load_keys(keys, 8, 1) == keys.size
    compare_layout(tab, orc)


def test_duplicate_insert_is_key_exists():
    tab = stage.Table(key_width=8)
    tab.load_ycsb(0, 1000, 8)
    assert tab.insert(5, 8) == stage.RC_KEY_EXISTS
    assert tab.insert(1000, 8) == stage.RC_OK
    assert tab.insert(1 << 40, 4) == stage.RC_INVALID  # wrong key width for a fixed-width table


def test_varlen_btreetest_layout():
    # BTreeTest parameters (testing_btree.cpp:365): variable-length ASCII keys, 8-byte payloads
    tab = stage.Table(payload_size=8, leaf_node_size=4096, split_threshold=3072, merge_threshold=1024, key_width=0)
    orc = O.OracleTree(4096, 3072, 8, 1024)
    assert tab.leaf_capacity == 128
    for i in range(20000):
        k = str(i).encode()
        kv = int.from_bytes(k, "little")
        pay = int(i).to_bytes(8, "little")
        assert tab.insert(kv, len(k), pay, commit_id=1005) == stage.RC_OK
        assert orc.insert(k, len(k), pay, 1005) == 1
    compare_layout(tab, orc)


def test_traverse_matches_oracle():
    tab = stage.Table(key_width=4)
    tab.load_ycsb(0, 200000, 4)
    orc = O.OracleTree()
    orc.load_ycsb(0, 200000, 4)
    # separators are the last keys of left leaves: collect them from the layout
    rc, sc, meta, keyw = tab.export_leaves(64)
    seps = []
    for li in range(rc.size - 1):
        ks = keyw[li, : rc[li]].astype(np.uint32)
        # max key of the leaf under the reference order = last key after sorting by order key
        ok = [int.from_bytes(bytes(b ^ 0x80 for b in int(k).to_bytes(4, "little")), "big") for k in ks]
        seps.append(int(ks[int(np.argmax(ok))]))
    rng = np.random.default_rng(3)
    probes = np.concatenate([rng.integers(0, 400000, 3000), np.array(seps[:500], np.int64)]).astype(np.uint64)
    for le in (True, False):
        got = tab.traverse(probes, le_child=le)
        exp = np.array([orc.traverse(int(k), 4, le) for k in probes])
        assert (got == exp).all()


def test_updates_and_deletes_keep_layout():
    tab = stage.Table(key_width=8)
    orc = O.OracleTree()
    tab.load_ycsb(0, 20000, 8)
    orc.load_ycsb(0, 20000, 8)
    for k in range(0, 20000, 37):
        d = bytes([k & 0xFF ^ 0x5A]) * 100
        assert tab.update(k, 0, d, writer_id=10) == orc.update(k, 8, 0, d, 10)
        if k % 2:
            assert tab.commit_update(k, 11, 11) == orc.commit_update(k, 8, 11, 11)
    for k in range(5, 20000, 1001):
        assert tab.delete(k, 12) == orc.delete(k, 8, 12)
    # more inserts force splits that drop deleted records and copy in-flight ones
    more = np.arange(20000, 60000, dtype=np.uint64)
    tab.load_keys(more, 8, 0)
    orc.load_keys(more, 8, 0)
    compare_layout(tab, orc)


@pytest.mark.parametrize("n", [4000, 20000])  # 20000: the parallel batched path
def test_update_batch_matches_per_key_oracle(n):
    # one YCSB-B writer epoch through the batched entry point (stage_update_batch), with
    # duplicate keys, absent keys, no-op deltas and stale writer ids, against the oracle's
    # per-key LeafNode::Update + CommitTransaction calls
    tab = stage.Table(key_width=8)
    orc = O.OracleTree()
    tab.load_ycsb(0, 30000, 8, mode=1)
    orc.load_ycsb(0, 30000, 8, 1)
    rng = np.random.default_rng(21)
    for epoch in range(3):
        keys = np.concatenate([rng.integers(0, 30000, n - 50), rng.integers(30000, 40000, 50)]).astype(np.uint64)
        deltas = rng.integers(0, 256, (n, 16), dtype=np.uint8)
        deltas[::97] = 0  # payload mode 1 words are random: zero patches still change bytes
        wid = np.full(n, 100 + 10 * epoch, np.uint32)
        wid[::53] = 1  # stale writers -> NOT_NEEDED_UPDATE once a key has a newer cstamp
        cid = np.where(np.arange(n) % 5 == 4, 0, 101 + 10 * epoch).astype(np.uint32)  # 20% stay in flight
        off = 8 * epoch
        rc, ok = tab.update_batch(keys, off, deltas, wid, cid)
        exp = np.zeros(n, np.uint8)
        for i in range(n):
            r = orc.update(int(keys[i]), 8, off, deltas[i].tobytes(), int(wid[i]))
            if r == stage.RC_OK and cid[i]:
                r = orc.commit_update(int(keys[i]), 8, int(cid[i]), int(cid[i]))
            exp[i] = r
        assert (rc == exp).all(), np.nonzero(rc != exp)[0][:5]
        assert ok == int((exp == stage.RC_OK).sum())
        assert len(set(rc.tolist())) >= 3
    compare_layout(tab, orc)
