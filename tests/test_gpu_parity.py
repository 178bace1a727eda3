"""GPU parity: the HIP path (through the C-ABI) against the oracle, bit-exact.

Every comparison covers the canonical outcome (status, copy flag, hops, cstamps) and the
full tuple row [key padded to 8][payload].  Sizes are ones the oracle finishes in seconds;
full-size properties live in test_gpu_fullsize.py.
"""
import json
import os

import numpy as np
import pytest

import oracle_lib as O
import stage

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def check_probe(tab, orc, keys, key_size, read_ids=None, lens=None, leaf_ids=None):
    out, rows = tab.probe(keys, read_ids=read_ids, lens=lens, leaf_ids=leaf_ids)
    if lens is None:
        o_out, o_rec = orc.read_batch(keys, key_size, read_ids)
    else:
        o_out = np.zeros(len(keys), O.READ_OUT_DTYPE)
        o_rec = np.zeros((len(keys), orc.row), np.uint8)
        for i, (k, ln) in enumerate(zip(keys, lens)):
            o_out[i], o_rec[i] = orc.read(int(k).to_bytes(8, "little")[:ln], int(ln),
                                          0xFFFFFFFE if read_ids is None else int(read_ids[i]))
    for f in ("status", "hops", "cstamp", "rec_cstamp", "copy_sstamp"):
        bad = np.nonzero(out[f] != o_out[f])[0]
        assert bad.size == 0, (f, bad[:5], out[f][bad[:5]], o_out[f][bad[:5]], keys[bad[:5]])
    assert ((out["flags"] & 1) == o_out["copy_present"]).all()
    bad = np.nonzero((rows[:, :orc.row] != o_rec).any(axis=1))[0]
    assert bad.size == 0, (bad[:5], keys[bad[:5]], out["status"][bad[:5]])
    assert (rows[:, orc.row:] == 0).all()
    # the hit slot's whole RecordMetadata word (meta_hi << 32 | rec_cstamp) == the oracle leaf's
    # (when the oracle holds the same table: same leaves and records)
    found = np.nonzero(out["status"] != 0)[0]
    os_, ts = orc.stats(), tab.stats()
    if found.size and os_["leaves"] < 400_000 and (os_["leaves"], os_["records"]) == (ts["leaves"], ts["records"]):
        meta = orc.export_leaves(tab.leaf_capacity)[2]
        m = meta[out["leaf"][found], out["slot"][found]]
        dm = (out["meta_hi"][found].astype(np.uint64) << np.uint64(32)) | out["rec_cstamp"][found].astype(np.uint64)
        bad = np.nonzero(m != dm)[0]
        assert bad.size == 0, ("meta", bad[:5], m[bad[:5]], dm[bad[:5]])
    return out, rows


@pytest.fixture(scope="module")
def ycsb4(gpu):
    tab = stage.Table(key_width=4)
    tab.load_ycsb(0, 1000000, 4, mode=0)
    tab.sync()
    orc = O.OracleTree()
    orc.load_ycsb(0, 1000000, 4, 0)
    return tab, orc


@pytest.fixture(scope="module")
def rand8(gpu):
    rng = np.random.default_rng(11)
    keys = rng.choice(np.arange(1, 4000000, dtype=np.uint64) * 7919, 300000, replace=False)
    tab = stage.Table(key_width=8)
    tab.load_keys(keys, 8, mode=1)
    tab.sync()
    orc = O.OracleTree()
    orc.load_keys(keys, 8, 1)
    return tab, orc, keys


def test_probe_ycsb_1m_all_hits_and_misses(ycsb4):
    tab, orc = ycsb4
    rng = np.random.default_rng(1)
    keys = np.concatenate([rng.integers(0, 1000000, 150000), np.arange(999000, 1001000),
                           rng.integers(1000000, 1 << 32, 5000)]).astype(np.uint64)
    out, rows = check_probe(tab, orc, keys, 4)
    hit = keys < 1000000
    assert (out["status"][hit] == stage.ST_LATEST).all() and (out["status"][~hit] == stage.ST_NOT_FOUND).all()


def test_probe_host_traversal_path(ycsb4):
    tab, orc = ycsb4
    keys = np.random.default_rng(2).integers(0, 1100000, 20000).astype(np.uint64)
    leaf = tab.traverse(keys)
    assert (tab.resolve(keys) == leaf).all()
    check_probe(tab, orc, keys, 4, leaf_ids=leaf)


def test_resolve_matches_oracle_traversal(ycsb4):
    tab, orc = ycsb4
    keys = np.random.default_rng(3).integers(0, 1100000, 2000).astype(np.uint64)
    # add every separator-adjacent case: leaf maxima are separators
    rc, sc, meta, keyw = tab.export_leaves(64)
    seps = []
    for li in range(0, rc.size - 1, 37):
        ks = keyw[li, : rc[li]].astype(np.uint32)
        ok = [int.from_bytes(bytes(b ^ 0x80 for b in int(k).to_bytes(4, "little")), "big") for k in ks]
        seps.append(int(ks[int(np.argmax(ok))]))
    keys = np.concatenate([keys, np.array(seps, np.uint64)])
    for le in (True, False):
        got = tab.resolve(keys, le_child=le)
        exp = np.array([orc.traverse(int(k), 4, le) for k in keys])
        assert (got == exp).all()


def test_probe_random_keys_strong_payload(rand8):
    tab, orc, keys = rand8
    rng = np.random.default_rng(4)
    probe = np.concatenate([rng.choice(keys, 100000), rng.integers(0, 1 << 40, 20000).astype(np.uint64),
                            np.array([0, 1, (1 << 64) - 1, 0x7F7F7F7F7F7F7F7F, 0x8080808080808080], np.uint64)])
    check_probe(tab, orc, probe, 8)


def test_scan_matches_oracle(ycsb4):
    tab, orc = ycsb4
    rng = np.random.default_rng(5)
    starts = np.concatenate([rng.integers(0, 1000000, 300), np.array([0, 999900, 999999, 1000000, 1 << 31])])
    starts = starts.astype(np.uint64)
    for size in (1, 2, 10, 100, 1000):
        counts, rows = tab.range_scan(starts, size)
        o_counts, o_rows = orc.scan_batch(starts, 4, size)
        assert (counts == o_counts).all(), size
        for i in range(starts.size):
            c = o_counts[i]
            assert (rows[i, :c, :orc.row] == o_rows[i, :c]).all(), (size, starts[i])


def test_scan_reference_facts(ycsb4):
    tab, _ = ycsb4
    facts = json.load(open(os.path.join(GOLD, "reference_facts.json")))
    for sc in facts["ycsb_1m_scans"]:
        counts, rows = tab.range_scan(np.array([sc["start"]], np.uint64), sc["scan_size"])
        assert counts[0] == sc["count"]
        keys = rows[0, :, :4].copy().view(np.uint32).ravel()
        assert list(keys[: len(sc["first_keys"])]) == sc["first_keys"]


def test_scan_random_order_8byte(rand8):
    tab, orc, keys = rand8
    starts = np.concatenate([np.random.default_rng(6).choice(keys, 200),
                             np.random.default_rng(7).integers(0, 1 << 40, 100).astype(np.uint64)])
    counts, rows = tab.range_scan(starts, 100)
    o_counts, o_rows = orc.scan_batch(starts, 8, 100)
    assert (counts == o_counts).all()
    for i in range(starts.size):
        assert (rows[i, :counts[i], :orc.row] == o_rows[i, :counts[i]]).all()


def test_visibility_version_chains(gpu):
    tab = stage.Table(key_width=8)
    orc = O.OracleTree()
    n = 50000
    tab.load_ycsb(0, n, 8, mode=1)
    orc.load_ycsb(0, n, 8, 1)
    rng = np.random.default_rng(8)
    hot = rng.choice(n, 3000, replace=False)
    cid = 10
    for rnd in range(4):  # several committed updates per key -> chains of length 1..4
        for k in hot[: 3000 - 600 * rnd]:
            d = bytes([rnd * 17 + 3]) * 100
            assert tab.update(int(k), 100 * rnd, d, cid) == orc.update(int(k), 8, 100 * rnd, d, cid)
            assert tab.commit_update(int(k), cid + 1, cid + 1) == orc.commit_update(int(k), 8, cid + 1, cid + 1)
        cid += 5
    inflight = hot[:700]
    for k in inflight:  # in-flight updates: readers see the copy or walk from its chain
        d = bytes([0xEE]) * 50
        assert tab.update(int(k), 7, d, cid) == orc.update(int(k), 8, 7, d, cid)
    for k in hot[2900:2950]:  # BTree::FinalizeUpdate style (next keeps pointing at the copy)
        orc_rc = orc.update(int(k), 8, 300, b"\x01" * 8, cid)
        assert tab.update(int(k), 300, b"\x01" * 8, cid) == orc_rc
        assert tab.finalize_update(int(k), cid + 2) == orc.finalize_update(int(k), 8, cid + 2)
    for k in rng.choice(n, 200, replace=False):
        assert tab.delete(int(k), cid) == orc.delete(int(k), 8, cid)
    tab.sync()
    keys = np.concatenate([hot, rng.integers(0, n + 100, 5000)]).astype(np.uint64)
    for rid in (0, 1, 10, 11, 12, 15, 16, 20, 21, 26, 27, cid, cid + 1, cid + 3, 0xFFFFFFFE):
        out, _ = check_probe(tab, orc, keys, 8, read_ids=np.full(keys.size, rid, np.uint32))
    mixed = rng.integers(0, cid + 4, keys.size).astype(np.uint32)
    out, _ = check_probe(tab, orc, keys, 8, read_ids=mixed)
    seen = set(np.unique(out["status"]).tolist())
    assert {stage.ST_LATEST, stage.ST_COPY, stage.ST_OLD, stage.ST_FAIL_INVALID_TS, stage.ST_NOT_FOUND} <= seen


def test_reference_version_chain_scenario(gpu):
    vc = json.load(open(os.path.join(GOLD, "reference_facts.json")))["version_chain"]
    tab = stage.Table(key_width=4)
    tab.load_ycsb(0, 10, 4)
    for u in vc["updates"]:
        assert tab.update(vc["key"], vc["column_offset"], bytes([u["byte"]]) * vc["column_bytes"],
                          u["read_id"]) == stage.RC_OK
        assert tab.commit_update(vc["key"], u["commit_id"], u["commit_id"]) == stage.RC_OK
    tab.sync()
    names = {"FAILURE": stage.ST_FAIL_INVALID_TS, "OLD": stage.ST_OLD, "LATEST": stage.ST_LATEST}
    for r in vc["reads"]:
        out, rows = tab.probe(np.array([vc["key"]], np.uint64), read_ids=np.array([r["read_id"]], np.uint32))
        assert out["status"][0] == names[r["result"]]
        if "payload_prefix_byte" in r:
            assert (rows[0, 8:8 + vc["column_bytes"]] == r["payload_prefix_byte"]).all()
            assert (rows[0, 8 + vc["column_bytes"]:1008] == r["payload_rest_byte"]).all()


def test_btreetest_scenarios_on_device(gpu):
    # testing_btree.cpp:389-439 (Insert) and :630-675 (RangeScanBySize) through the device path
    tab = stage.Table(payload_size=8, leaf_node_size=4096, split_threshold=3072, merge_threshold=1024, key_width=0)
    orc = O.OracleTree(4096, 3072, 8, 1024)
    keys, lens = [], []
    for i in range(100000):
        k = str(i).encode()
        kv = int.from_bytes(k, "little")
        assert tab.insert(kv, len(k), int(i).to_bytes(8, "little"), commit_id=1005) == stage.RC_OK
        orc.insert(k, len(k), int(i).to_bytes(8, "little"), 1005)
        keys.append(kv)
        lens.append(len(k))
    tab.sync()
    keys = np.array(keys, np.uint64)
    lens = np.array(lens, np.uint16)
    out, rows = tab.probe(keys, read_ids=np.full(keys.size, 1007, np.uint32), lens=lens)
    assert (out["status"] == stage.ST_LATEST).all()
    assert (rows[:, 8:16].copy().view(np.uint64).ravel() == np.arange(100000)).all()
    sel = np.random.default_rng(9).choice(keys.size, 3000, replace=False)
    check_probe(tab, orc, keys[sel], 8, read_ids=np.full(sel.size, 1007, np.uint32), lens=lens[sel])
    start = np.array([int.from_bytes(b"9000", "little")], np.uint64)
    for size in (100, 1000):
        counts, rows = tab.range_scan(start, size, lens=np.array([4], np.uint16))
        assert counts[0] == size
        oc, orow = orc.scan(b"9000", 4, size)
        assert oc == size
        assert (rows[0, :size, :16] == orow).all()


def test_murmur_device_matches_reference_kat(gpu):
    kat = json.load(open(os.path.join(GOLD, "murmur64a_kat.json")))
    eight = [v for v in kat["vectors"] if len(bytes.fromhex(v["hex"])) == 8 and v["seed"] == 0]
    keys = np.array([int.from_bytes(bytes.fromhex(v["hex"]), "little") for v in eight], np.uint64)
    got = stage.murmur64a_device(keys, 8, 0)
    assert [int(x) for x in got] == [v["hash"] for v in eight]
    rnd = np.random.default_rng(10).integers(0, 1 << 63, 100000).astype(np.uint64)
    for ln in (8, 4, 3):
        assert (stage.murmur64a_device(rnd, ln, 5) == O.murmur64a_keys(rnd, ln, 5)).all()


def test_tiny_tables(gpu):
    for n in (0, 1, 2, 63, 64):
        tab = stage.Table(key_width=8)
        tab.load_ycsb(0, n, 8, mode=1)
        tab.sync()
        orc = O.OracleTree()
        orc.load_ycsb(0, n, 8, 1)
        keys = np.arange(0, 70, dtype=np.uint64)
        check_probe(tab, orc, keys, 8)
        counts, rows = tab.range_scan(keys[:10], 5)
        o_counts, o_rows = orc.scan_batch(keys[:10], 8, 5)
        assert (counts == o_counts).all()


def test_imported_snapshot_on_device(gpu):
    # reference-format leaf blocks (oracle export) -> empty table -> HBM: probes and scans
    # equal the oracle's on the tree the blocks came from
    rng = np.random.default_rng(12)
    keys = rng.choice(np.arange(1, 2000000, dtype=np.uint64) * 40503, 150000, replace=False)
    orc = O.OracleTree()
    orc.load_keys(keys, 8, 1)
    for k in keys[::29]:
        orc.update(int(k), 8, 0, b"\x5a" * 32, 3)
        orc.commit_update(int(k), 8, 4, 4)
    for k in keys[7::211]:
        orc.delete(int(k), 8, 5)
    blocks, sk, sl = orc.export_leaf_images()
    tab = stage.Table(key_width=8)
    tab.import_leaf_images(blocks, sk, sl)
    tab.sync()
    probe = np.concatenate([rng.choice(keys, 60000), rng.integers(0, 1 << 37, 5000).astype(np.uint64)])
    # read ids at/after the last commit: version chains are not part of the snapshot format
    check_probe(tab, orc, probe, 8, read_ids=np.full(probe.size, 10, np.uint32))
    starts = rng.choice(keys, 300)
    counts, rows = tab.range_scan(starts, 100)
    o_counts, o_rows = orc.scan_batch(starts, 8, 100)
    assert (counts == o_counts).all()
    for i in range(starts.size):
        assert (rows[i, :counts[i], :orc.row] == o_rows[i, :counts[i]]).all()


def test_config1_ycsb_c_1000_rows(gpu):
    # BASELINE configs[0] (YCSB-C -k 1000 -b 1 -o 10 -u 0 -z 0, the reference's CPU case) as
    # a parity case: 1000 rows of 4-byte keys loaded as LoadYCSBRows does, uniform keys,
    # 10 reads per transaction, 10^5 transactions
    tab = stage.Table(key_width=4)
    assert tab.load_ycsb(0, 1000, 4, mode=0) == 1000
    tab.sync()
    orc = O.OracleTree()
    orc.load_ycsb(0, 1000, 4, 0)
    keys = (stage.fastrandom(12345, 1_000_000) % np.uint64(1000)).astype(np.uint64)
    out, rows = check_probe(tab, orc, keys, 4)
    assert (out["status"] == stage.ST_LATEST).all()
    assert (rows[:, 8:1008] == (keys & np.uint64(0xFF)).astype(np.uint8)[:, None]).all()
