"""Pins the oracle (CPU restatement) to the reference's own outputs.

Fixtures: tests/golden/reference_facts.json (observed on the reference build, SURVEY.md
Appendix B), tests/golden/murmur64a_kat.json (the reference's MurmurHash2.cpp), and the
assertions of the reference's own BTreeTest suite (test/testing_btree.cpp:331-675).
"""
import json
import os

import numpy as np
import pytest

import oracle_lib as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def facts():
    with open(os.path.join(GOLD, "reference_facts.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def ycsb_1m():
    f = facts()["ycsb_1m_tree"]
    t = O.OracleTree(f["leaf_node_size"], f["split_threshold"], f["payload_size"])
    assert t.load_ycsb(0, f["rows"], f["key_size"], 0) == f["rows"]
    return t


def test_tree_shape_matches_reference(ycsb_1m):
    f = facts()["ycsb_1m_tree"]
    s = ycsb_1m.stats()
    assert s["height"] == f["height"]
    assert s["inner"] == f["inner_nodes_including_root"]
    assert s["leaves"] == f["leaves"]
    assert s["sorted"] == f["sorted_slots"]
    assert s["unsorted"] == f["unsorted_slots"]
    assert s["max_count"] == f["max_records_per_leaf"]
    assert s["records"] == f["rows"]


def test_scans_match_reference(ycsb_1m):
    for sc in facts()["ycsb_1m_scans"]:
        c, recs = ycsb_1m.scan(sc["start"], 4, sc["scan_size"])
        assert c == sc["count"]
        keys = recs[:, :4].copy().view(np.uint32).ravel()
        assert list(keys[: len(sc["first_keys"])]) == sc["first_keys"]
        # payload = memset(rowid) (ycsb_loader.cpp:149-150)
        assert (recs[:, 8:] == (keys & 0xFF)[:, None]).all()


def test_point_reads_every_row(ycsb_1m):
    keys = np.arange(0, 1000000, 997, dtype=np.uint64)
    outs, recs = ycsb_1m.read_batch(keys, 4)
    assert (outs["status"] == 1).all()
    assert (recs[:, :4].copy().view(np.uint32).ravel() == keys).all()
    assert (recs[:, 8:] == (keys & 0xFF).astype(np.uint8)[:, None]).all()
    # read_id defaults to MAX-1 -> cstamp handed to PerformRead is the reader id
    assert (outs["cstamp"] == 0xFFFFFFFE).all()
    miss, _ = ycsb_1m.read_batch(np.array([1000000, 2000000], np.uint64), 4)
    assert (miss["status"] == 0).all()


def test_key_compare_signed_bytes():
    for kc in facts()["key_compare"]:
        a = int(kc["k1_u32"]).to_bytes(4, "little")
        b = int(kc["k2_u32"]).to_bytes(4, "little")
        assert np.sign(O.key_compare(a, b)) == kc["sign"]
    assert O.key_compare(b"12", b"123") < 0  # equal prefix -> shorter first
    assert O.key_compare(b"\x80", b"\x7f") < 0  # signed char


def test_version_chain_reference_scenario():
    vc = facts()["version_chain"]
    t = O.OracleTree()
    t.load_ycsb(0, 10, 4, 0)
    key = vc["key"]
    for u in vc["updates"]:
        delta = bytes([u["byte"]]) * vc["column_bytes"]
        assert t.update(key, 4, vc["column_offset"], delta, u["read_id"]) == 1
        # single writer: t_sstamp = min(MAX_CID, t_cstamp) (transaction_manager.cpp:113-121)
        assert t.commit_update(key, 4, u["commit_id"], u["commit_id"]) == 1
    names = {"FAILURE": 4, "OLD": 3, "LATEST": 1}
    for r in vc["reads"]:
        out, rec = t.read(key, 4, r["read_id"])
        assert out["status"] == names[r["result"]], r
        if "payload_prefix_byte" in r:
            assert (rec[8:8 + vc["column_bytes"]] == r["payload_prefix_byte"]).all()
            assert (rec[8 + vc["column_bytes"]:] == r["payload_rest_byte"]).all()
            assert rec[0] == key


def _u64(i):
    return int(i).to_bytes(8, "little")


def btree_test_tree():
    p = facts()["btree_unit_test"]["params"]
    return O.OracleTree(p["leaf_node_size"], p["split_threshold"], p["payload_size"], p["merge_threshold"])


def insert_dummy(t, commit=0):
    for i in range(0, 100, 10):
        assert t.insert(str(i).encode(), len(str(i)), _u64(i), commit) == 1


def test_btreetest_insert_and_read_back():
    # TEST_F(BTreeTest, Insert): testing_btree.cpp:389-439
    t = btree_test_tree()
    n = facts()["btree_unit_test"]["insert_keys"]
    for i in range(n):
        k = str(i).encode()
        assert t.insert(k, len(k), _u64(i), 1005) == 1
        out, rec = t.read(k, len(k), 1005)
        assert out["status"] == 1 and int.from_bytes(rec[8:16].tobytes(), "little") == i
    for i in range(0, n, 7):
        k = str(i).encode()
        out, rec = t.read(k, len(k), 1007)
        assert out["status"] == 1 and int.from_bytes(rec[8:16].tobytes(), "little") == i


def test_btreetest_read_update_upsert_delete():
    # TEST_F(BTreeTest, Read) testing_btree.cpp:442-470
    t = btree_test_tree()
    assert t.read(b"10", 2, 2007)[0]["status"] == 0
    insert_dummy(t)
    out, rec = t.read(b"10", 2, 2007)
    assert out["status"] == 1 and rec[8] == 10
    assert t.read(b"11", 2, 2007)[0]["status"] == 0
    # TEST_F(BTreeTest, Update) testing_btree.cpp:472-516
    assert t.read(b"20", 2, 5000)[1][8] == 20
    assert t.update(b"20", 2, 0, _u64(21), 5000) == 1
    out, rec = t.read(b"20", 2, 5005)  # in flight: copy of the old image
    assert out["status"] == 2 and rec[8] == 20
    assert t.finalize_update(b"20", 2, 5005) == 1
    out, rec = t.read(b"20", 2, 5006)
    assert out["status"] == 1 and rec[8] == 21
    # TEST_F(BTreeTest, Upsert) testing_btree.cpp:518-583 (insert branch)
    assert t.read(b"abc", 3, 6000)[0]["status"] == 0
    assert t.insert(b"abc", 3, _u64(42), 6000) == 1
    assert t.read(b"abc", 3, 6000)[1][8] == 42


def test_btreetest_delete():
    # TEST_F(BTreeTest, Delete) testing_btree.cpp:585-627
    t = btree_test_tree()
    for i in range(50):
        k = str(i).encode()
        assert t.insert(k, len(k), _u64(i), 7001) == 1
    for i in range(40):
        k = str(i).encode()
        assert t.delete(k, len(k), 7002) == 1
        assert t.read(k, len(k), 7003)[0]["status"] == 0
    assert t.read(b"45", 2, 7003)[0]["status"] == 1


def test_btreetest_range_scan_by_size():
    # TEST_F(BTreeTest, RangeScanBySize) testing_btree.cpp:630-675
    t = btree_test_tree()
    for i in range(1000, 10000):
        k = str(i).encode()
        assert t.insert(k, 4, _u64(i), 8001) == 1
    for size in facts()["btree_unit_test"]["scan_sizes"]:
        c, recs = t.scan(b"9000", 4, size)
        assert c == size
        keys = [bytes(r[:4]).decode() for r in recs]
        assert keys == sorted(keys)  # KeyCompare order == ascii order for digits
        assert keys[0] == "9000"


def test_murmur_kat_reference():
    with open(os.path.join(GOLD, "murmur64a_kat.json")) as f:
        kat = json.load(f)
    for v in kat["vectors"]:
        assert O.murmur64a(bytes.fromhex(v["hex"]), v["seed"]) == v["hash"]


def test_murmur_against_reference_build():
    ref = O.ref_murmur_lib()
    if ref is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    rng = np.random.default_rng(1)
    for ln in range(0, 40):
        data = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
        assert ref.ref_murmur64a(data, ln, 7) == O.murmur64a(data, 7)


def test_key_compare_wide_branch_is_libc_memcmp():
    """KeyCompare's branch for keys of 16 bytes and more calls the C library's memcmp
    (b_tree.h:126-128: `cmp = memcmp(key1, key2, min(size1, size2))`; shorter keys go through
    the signed-char my_memcmp, :99-106).  The dependency is libc itself (glibc 2.35 in this image):
    its published contract is an unsigned-byte lexicographic comparison.  The oracle's
    restatement is pinned here against the real libc memcmp on random keys of 16-40 bytes
    whose bytes straddle 0x80 (where signed and unsigned order disagree), equal prefixes of
    different lengths included; and the < 16-byte branch against a signed-char restatement."""
    import ctypes
    libc = ctypes.CDLL(None)
    libc.memcmp.restype = ctypes.c_int
    libc.memcmp.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]
    rng = np.random.default_rng(21)
    checked_flip = 0
    for _ in range(4000):
        la, lb = (int(x) for x in rng.integers(16, 41, 2))
        a = bytearray(rng.integers(0, 256, la, dtype=np.uint8).tobytes())
        b = bytearray(rng.integers(0, 256, lb, dtype=np.uint8).tobytes())
        cut = int(rng.integers(0, min(la, lb) + 1))  # shared prefix of random length
        b[:cut] = a[:cut]
        if cut < min(la, lb) and rng.random() < 0.5:  # first difference across the sign bit
            a[cut], b[cut] = 0x7F, 0x80
            checked_flip += 1
        a, b = bytes(a), bytes(b)
        c = libc.memcmp(a, b, min(la, lb))
        exp = np.sign(c) if c != 0 else np.sign(la - lb)
        assert np.sign(O.key_compare(a, b)) == exp, (a.hex(), b.hex())
    assert checked_flip > 500
    for _ in range(2000):  # the signed-char branch: min(size) < 16
        la = int(rng.integers(1, 16))
        lb = int(rng.integers(la, 24))
        a = rng.integers(0, 256, la, dtype=np.uint8).tobytes()
        b = a[:int(rng.integers(0, la + 1))] + rng.integers(0, 256, lb, dtype=np.uint8).tobytes()
        b = b[:lb]
        sa = np.frombuffer(a, np.int8).astype(int)
        sb = np.frombuffer(b, np.int8).astype(int)
        m = min(la, lb)
        d = np.nonzero(sa[:m] != sb[:m])[0]
        exp = np.sign(sa[d[0]] - sb[d[0]]) if d.size else np.sign(la - lb)
        assert np.sign(O.key_compare(a, b)) == exp
