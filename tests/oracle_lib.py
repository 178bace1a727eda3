"""ctypes binding of the test oracle (oracle/stage_oracle.c) -- TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of the reference path; tests use it as the checker.
"""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "_build", "libstage_oracle.so")
REF_MURMUR_SO = os.path.join(ORACLE_DIR, "_ref", "libref_murmur.so")

READ_OUT_DTYPE = np.dtype([("status", "u1"), ("copy_present", "u1"), ("hops", "u2"), ("cstamp", "u4"),
                           ("rec_cstamp", "u4"), ("copy_sstamp", "u4")])

vp = ctypes.c_void_p
u32, u64 = ctypes.c_uint32, ctypes.c_uint64

_SIG = {
    "orc_tree_new": (vp, [u32, u32, u32]),
    "orc_tree_set_merge_threshold": (None, [vp, u32]),
    "orc_tree_free": (None, [vp]),
    "orc_insert": (ctypes.c_int, [vp, vp, u32, vp, u32]),
    "orc_insert_inflight": (ctypes.c_int, [vp, vp, u32, vp, u32]),
    "orc_commit_insert": (ctypes.c_int, [vp, vp, u32, u32]),
    "orc_load_ycsb": (u64, [vp, u64, u64, u32, ctypes.c_int]),
    "orc_load_keys": (u64, [vp, vp, u64, u32, ctypes.c_int]),
    "orc_read": (ctypes.c_int, [vp, vp, u32, u32, vp, vp]),
    "orc_read_fu": (ctypes.c_int, [vp, vp, u32, u32, ctypes.c_int, vp, vp]),
    "orc_update_owned": (ctypes.c_int, [vp, vp, u32, u32, vp, u32, u32]),
    "orc_delete_owned": (ctypes.c_int, [vp, vp, u32]),
    "orc_read_batch": (ctypes.c_int, [vp, vp, u32, vp, u64, vp, vp, ctypes.c_int]),
    "orc_read_batch_timed": (u64, [vp, vp, u32, vp, u64, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]),
    "orc_scan": (u32, [vp, vp, u32, u32, vp]),
    "orc_scan_batch": (u64, [vp, vp, u32, u64, u32, vp, vp, ctypes.c_int]),
    "orc_scan_batch_timed": (u64, [vp, vp, u32, u64, u32, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]),
    "orc_traverse_leaf_index": (ctypes.c_int64, [vp, vp, u32, ctypes.c_int]),
    "orc_update": (ctypes.c_int, [vp, vp, u32, u32, vp, u32, u32]),
    "orc_commit_update": (ctypes.c_int, [vp, vp, u32, u32, u32]),
    "orc_finalize_update": (ctypes.c_int, [vp, vp, u32, u32]),
    "orc_delete": (ctypes.c_int, [vp, vp, u32, u32]),
    "orc_stats": (None, [vp, vp]),
    "orc_export_leaves": (ctypes.c_int64, [vp, u32, u64, vp, vp, vp, vp]),
    "orc_export_leaf_images": (ctypes.c_int64, [vp, u64, vp, vp, vp]),
    "orc_export_leaf_images_k": (ctypes.c_int64, [vp, u64, vp, vp, u32, vp]),
    "orc_tree_set_key_pad": (None, [vp, u32]),
    "orc_index_scan": (u32, [vp, vp, u32, u32, u32, vp, vp]),
    "orc_load_rows": (u64, [vp, vp, u32, u32, vp, u32, u64]),
    "orc_stock_level": (ctypes.c_int32, [vp, vp, vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, u32]),
    "orc_stock_level_batch": (None, [vp, vp, vp, vp, vp, vp, vp, u64, vp, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_double)]),
    "orc_ch_query2": (ctypes.c_int64, [vp, vp, vp, vp, vp, vp, vp, vp, ctypes.c_int, u32, vp, u64,
                                       ctypes.POINTER(ctypes.c_int)]),
    "orc_ch_query2_timed": (u64, [vp, vp, vp, vp, vp, vp, vp, vp, ctypes.c_int, u32, u64, ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_double)]),
    "orc_read_batch_k": (ctypes.c_int, [vp, vp, u32, u32, vp, u64, vp, vp, ctypes.c_int]),
    "orc_scan_batch_k": (u64, [vp, vp, u32, u32, u64, u32, vp, vp, ctypes.c_int]),
    "orc_ycsb_txn_timed": (None, [vp, vp, u32, u32, u64, ctypes.c_int, u32, ctypes.POINTER(ctypes.c_double), vp]),
    "orc_abort_update": (ctypes.c_int, [vp, vp, u32]),
    "orc_abort_insert": (ctypes.c_int, [vp, vp, u32]),
    "orc_update_batch": (u64, [vp, vp, u32, u64, u32, vp, u32, vp, vp, vp]),
    "orc_update_batch_mt": (u64, [vp, vp, u32, u64, u32, vp, u32, vp, vp, vp, ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_double)]),
    "orc_tree_set_bulk": (None, [vp, ctypes.c_int]),
    "orc_load_ycsb_parallel": (u64, [vp, u64, u64, u32, ctypes.c_int, ctypes.c_int]),
    "orc_resolve_locations": (None, [vp, vp, u64, vp, vp]),
    "orc_location_count": (u64, [vp]),
    "orc_key_compare": (ctypes.c_int, [vp, u32, vp, u32]),
    "orc_murmur64a": (u64, [vp, ctypes.c_int, u64]),
    "orc_murmur64a_batch": (None, [vp, u64, ctypes.c_int, u64, vp]),
    "orc_payload_word": (u64, [u64, u32]),
    "orc_fill_payload": (None, [u64, ctypes.c_int, vp, u32]),
    "orc_read_ident": (ctypes.c_int, [vp, vp, u32, u32, vp, vp, vp, vp, vp]),
    "orc_location_meta": (ctypes.c_int, [vp, u64, vp, vp]),
    "orc_record_meta": (ctypes.c_int, [vp, vp, u32, vp, vp, vp]),
    "orc_copy_state": (ctypes.c_int, [vp, u32, vp]),
    "orc_copy_readers": (u32, [vp, u32, vp, u32]),
    "orc_copy_add_reader": (ctypes.c_int, [vp, u32, u32]),
    "orc_copy_wr_count": (ctypes.c_int, [vp, u32, ctypes.c_int]),
    "orc_copy_update_ps": (ctypes.c_int, [vp, u32, u32]),
}

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build()
        L = ctypes.CDLL(ORACLE_SO)
        for name, (res, args) in _SIG.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def key_bytes(key, size):
    return np.array([int(key)], np.uint64).tobytes()[:size] if isinstance(key, (int, np.integer)) else bytes(key)


class OracleTree:
    def __init__(self, leaf_node_size=64 * 1024, split_threshold=16 * 1024, payload_size=1000,
                 merge_threshold=32 * 1024, key_pad=8):
        self.t = lib().orc_tree_new(leaf_node_size, split_threshold, payload_size)
        lib().orc_tree_set_merge_threshold(self.t, merge_threshold)
        lib().orc_tree_set_key_pad(self.t, key_pad)
        self.payload_size = payload_size
        self.leaf_node_size = leaf_node_size
        self.key_pad = key_pad
        self.row = key_pad + payload_size

    def __del__(self):
        try:
            lib().orc_tree_free(self.t)
        except Exception:
            pass

    def insert(self, key, key_size, payload, commit_id=0):
        kb = key_bytes(key, key_size)
        pb = bytes(payload)
        assert len(pb) == self.payload_size
        return lib().orc_insert(self.t, kb, key_size, pb, commit_id)

    def insert_inflight(self, key, key_size, payload, writer_id):
        """an uncommitted transaction's insert (PrepareForInsert, cstamp = writer id)"""
        pb = bytes(payload)
        assert len(pb) == self.payload_size
        return lib().orc_insert_inflight(self.t, key_bytes(key, key_size), key_size, pb, writer_id)

    def commit_insert(self, key, key_size, commit_id):
        """CommitTransaction INSERT entry (FinalizeForInsert(t_cstamp))"""
        return lib().orc_commit_insert(self.t, key_bytes(key, key_size), key_size, commit_id)

    def load_ycsb(self, begin, end, key_size, mode=0):
        return lib().orc_load_ycsb(self.t, begin, end, key_size, mode)

    def load_ycsb_bulk(self, begin, end, key_size, mode=0):
        """LoadYCSBRows without CheckUnique (distinct keys): the same leaves, built faster"""
        lib().orc_tree_set_bulk(self.t, 1)
        try:
            return lib().orc_load_ycsb(self.t, begin, end, key_size, mode)
        finally:
            lib().orc_tree_set_bulk(self.t, 0)

    def load_ycsb_parallel(self, begin, end, key_size, mode=0, nthreads=8):
        """LoadYCSBRows by nthreads threads: the single loader's leaves, inner levels rebuilt
        bottom-up (same routing) -- the CPU baseline's large tables"""
        lib().orc_tree_set_bulk(self.t, 1)
        try:
            return lib().orc_load_ycsb_parallel(self.t, begin, end, key_size, mode, nthreads)
        finally:
            lib().orc_tree_set_bulk(self.t, 0)

    def ycsb_txn_timed(self, keys, key_size, ops_per_txn, nthreads=1, first_tid=1):
        """full-txn CPU baseline: len(keys) // ops_per_txn read-only RunMixed transactions;
        returns (seconds, commits, aborts, checksum)"""
        keys = np.ascontiguousarray(keys, np.uint64)
        n_txns = keys.size // ops_per_txn
        sec = ctypes.c_double()
        res = np.zeros(3, np.uint64)
        lib().orc_ycsb_txn_timed(self.t, keys.ctypes.data, key_size, ops_per_txn, n_txns, nthreads, first_tid,
                                 ctypes.byref(sec), res.ctypes.data)
        return sec.value, int(res[0]), int(res[1]), int(res[2])

    def load_keys(self, keys, key_size, mode=0):
        keys = np.ascontiguousarray(keys, np.uint64)
        return lib().orc_load_keys(self.t, keys.ctypes.data, keys.size, key_size, mode)

    def read(self, key, key_size, read_id=0xFFFFFFFE, for_update=False):
        kb = key_bytes(key, key_size)
        out = np.zeros(1, READ_OUT_DTYPE)
        rec = np.zeros(self.row, np.uint8)
        lib().orc_read_fu(self.t, kb, key_size, read_id, 1 if for_update else 0, out.ctypes.data, rec.ctypes.data)
        return out[0], rec

    def read_ident(self, key, key_size, read_id=0xFFFFFFFE):
        """orc_read + the hit slot's meta word, location handle and next handle"""
        kb = key_bytes(key, key_size)
        out = np.zeros(1, READ_OUT_DTYPE)
        rec = np.zeros(self.row, np.uint8)
        meta, loc, nxt = ctypes.c_uint64(), ctypes.c_uint32(), ctypes.c_uint32()
        lib().orc_read_ident(self.t, kb, key_size, read_id, out.ctypes.data, rec.ctypes.data, ctypes.byref(meta),
                             ctypes.byref(loc), ctypes.byref(nxt))
        return out[0], rec, meta.value, loc.value, nxt.value

    def location_meta(self, handle):
        meta, nxt = ctypes.c_uint64(), ctypes.c_uint32()
        lib().orc_location_meta(self.t, handle, ctypes.byref(meta), ctypes.byref(nxt))
        return meta.value, nxt.value

    def copy_state(self, copy_id):
        """(cstamp, pstamp, rstamp, sstamp, readers, count, waiting) or None"""
        st = np.zeros(7, np.uint32)
        if lib().orc_copy_state(self.t, copy_id, st.ctypes.data) != 0:
            return None
        return tuple(int(x) for x in st)

    def copy_readers(self, copy_id):
        buf = np.zeros(4096, np.uint32)
        n = lib().orc_copy_readers(self.t, copy_id, buf.ctypes.data, buf.size)
        return buf[:min(n, buf.size)].tolist()

    def read_batch(self, keys, key_size, read_ids=None, records=True, nthreads=8):
        keys = np.ascontiguousarray(keys, np.uint64)
        n = keys.size
        rids = None if read_ids is None else np.ascontiguousarray(read_ids, np.uint32)
        outs = np.zeros(n, READ_OUT_DTYPE)
        recs = np.zeros((n, self.row), np.uint8) if records else None
        lib().orc_read_batch(self.t, keys.ctypes.data, key_size, rids.ctypes.data if rids is not None else None, n,
                             outs.ctypes.data, recs.ctypes.data if recs is not None else None, nthreads)
        return outs, recs

    def load_rows(self, keys, payloads):
        keys = np.ascontiguousarray(keys, np.uint8)
        payloads = np.ascontiguousarray(payloads, np.uint8)
        return lib().orc_load_rows(self.t, keys.ctypes.data, keys.shape[1], keys.shape[1], payloads.ctypes.data,
                                   payloads.shape[1], keys.shape[0])

    def read_batch_k(self, keys, read_ids=None, records=True, nthreads=8):
        """keys: (n, width) uint8 key bytes"""
        keys = np.ascontiguousarray(keys, np.uint8)
        n = keys.shape[0]
        rids = None if read_ids is None else np.ascontiguousarray(read_ids, np.uint32)
        outs = np.zeros(n, READ_OUT_DTYPE)
        recs = np.zeros((n, self.row), np.uint8) if records else None
        lib().orc_read_batch_k(self.t, keys.ctypes.data, keys.shape[1], keys.shape[1],
                               rids.ctypes.data if rids is not None else None, n, outs.ctypes.data,
                               recs.ctypes.data if recs is not None else None, nthreads)
        return outs, recs

    def scan_batch_k(self, keys, scan_size, nthreads=8):
        keys = np.ascontiguousarray(keys, np.uint8)
        n = keys.shape[0]
        counts = np.zeros(n, np.uint32)
        recs = np.zeros((n, scan_size, self.row), np.uint8)
        lib().orc_scan_batch_k(self.t, keys.ctypes.data, keys.shape[1], keys.shape[1], n, scan_size,
                               counts.ctypes.data, recs.ctypes.data, nthreads)
        return counts, recs

    def index_scan(self, key, key_size, scan_size, read_id):
        """IndexScanExecutor range branch: (consumed, rows[consumed], status[consumed])"""
        kb = key_bytes(key, key_size)
        recs = np.zeros((max(scan_size, 1), self.row), np.uint8)
        st = np.zeros(max(scan_size, 1), np.uint8)
        c = lib().orc_index_scan(self.t, kb, key_size, scan_size, read_id, recs.ctypes.data, st.ctypes.data)
        return c, recs[:c], st[:c]

    def scan(self, key, key_size, scan_size):
        kb = key_bytes(key, key_size)
        recs = np.zeros((max(scan_size, 1), self.row), np.uint8)
        c = lib().orc_scan(self.t, kb, key_size, scan_size, recs.ctypes.data)
        return c, recs[:c]

    def scan_batch(self, keys, key_size, scan_size, nthreads=8):
        keys = np.ascontiguousarray(keys, np.uint64)
        counts = np.zeros(keys.size, np.uint32)
        recs = np.zeros((keys.size, scan_size, self.row), np.uint8)
        lib().orc_scan_batch(self.t, keys.ctypes.data, key_size, keys.size, scan_size, counts.ctypes.data,
                             recs.ctypes.data, nthreads)
        return counts, recs

    def traverse(self, key, key_size, le_child=True):
        return lib().orc_traverse_leaf_index(self.t, key_bytes(key, key_size), key_size, int(le_child))

    def update(self, key, key_size, payload_off, delta, writer_id):
        d = bytes(delta)
        return lib().orc_update(self.t, key_bytes(key, key_size), key_size, payload_off, d, len(d), writer_id)

    def update_owned(self, key, key_size, payload_off, delta, writer_id):
        d = bytes(delta)
        return lib().orc_update_owned(self.t, key_bytes(key, key_size), key_size, payload_off, d, len(d), writer_id)

    def delete_owned(self, key, key_size):
        return lib().orc_delete_owned(self.t, key_bytes(key, key_size), key_size)

    def update_batch(self, keys, key_size, payload_off, deltas, wid, cid):
        """orc_update_batch: returns (rc[n], n_ok)"""
        keys = np.ascontiguousarray(keys, np.uint64)
        deltas = np.ascontiguousarray(deltas, np.uint8).reshape(keys.size, -1)
        wid = np.ascontiguousarray(wid, np.uint32)
        cid = np.ascontiguousarray(cid, np.uint32)
        rc = np.zeros(keys.size, np.uint8)
        ok = lib().orc_update_batch(self.t, keys.ctypes.data, key_size, keys.size, payload_off, deltas.ctypes.data,
                                    deltas.shape[1], wid.ctypes.data, cid.ctypes.data, rc.ctypes.data)
        return rc, int(ok)

    def update_batch_mt(self, keys, key_size, payload_off, deltas, wid, cid, nthreads):
        """orc_update_batch_mt (nthreads concurrent writers): returns (rc[n], n_ok, seconds)"""
        keys = np.ascontiguousarray(keys, np.uint64)
        deltas = np.ascontiguousarray(deltas, np.uint8).reshape(keys.size, -1)
        wid = np.ascontiguousarray(wid, np.uint32)
        cid = np.ascontiguousarray(cid, np.uint32)
        rc = np.zeros(keys.size, np.uint8)
        sec = ctypes.c_double()
        ok = lib().orc_update_batch_mt(self.t, keys.ctypes.data, key_size, keys.size, payload_off, deltas.ctypes.data,
                                       deltas.shape[1], wid.ctypes.data, cid.ctypes.data, rc.ctypes.data,
                                       int(nthreads), ctypes.byref(sec))
        return rc, int(ok), sec.value

    def commit_update(self, key, key_size, commit_id, sstamp):
        return lib().orc_commit_update(self.t, key_bytes(key, key_size), key_size, commit_id, sstamp)

    def abort_update(self, key, key_size):
        return lib().orc_abort_update(self.t, key_bytes(key, key_size), key_size)

    def abort_insert(self, key, key_size):
        return lib().orc_abort_insert(self.t, key_bytes(key, key_size), key_size)

    def finalize_update(self, key, key_size, commit_id):
        return lib().orc_finalize_update(self.t, key_bytes(key, key_size), key_size, commit_id)

    def delete(self, key, key_size, commit_id=0):
        return lib().orc_delete(self.t, key_bytes(key, key_size), key_size, commit_id)

    def stats(self):
        s = np.zeros(8, np.uint64)
        lib().orc_stats(self.t, s.ctypes.data)
        keys = ["height", "inner", "leaves", "records", "sorted", "unsorted", "max_count", "versions"]
        return {k: int(v) for k, v in zip(keys, s)}

    def export_leaf_images(self, kwords=1):
        nl = self.stats()["leaves"]
        blocks = np.zeros((nl, self.leaf_node_size), np.uint8)
        sk = np.zeros(nl * kwords, np.uint64)
        sl = np.zeros(nl, np.uint16)
        got = lib().orc_export_leaf_images_k(self.t, nl, blocks.ctypes.data, sk.ctypes.data, kwords, sl.ctypes.data)
        assert got == nl
        return blocks, (sk if kwords == 1 else sk.reshape(nl, kwords)), sl

    def resolve_locations(self, handles):
        handles = np.ascontiguousarray(handles, np.uint64)
        lf = np.zeros(handles.size, np.uint32)
        sl = np.zeros(handles.size, np.uint16)
        lib().orc_resolve_locations(self.t, handles.ctypes.data, handles.size, lf.ctypes.data, sl.ctypes.data)
        return lf, sl

    def location_count(self):
        return int(lib().orc_location_count(self.t))

    def export_leaves(self, cap):
        nl = self.stats()["leaves"]
        rc = np.zeros(nl, np.uint32)
        sc = np.zeros(nl, np.uint32)
        meta = np.zeros(nl * cap, np.uint64)
        keyw = np.zeros(nl * cap, np.uint64)
        got = lib().orc_export_leaves(self.t, cap, nl, rc.ctypes.data, sc.ctypes.data, meta.ctypes.data,
                                      keyw.ctypes.data)
        assert got == nl
        return rc, sc, meta.reshape(nl, cap), keyw.reshape(nl, cap)


def stock_level_batch(dist, ol, stock, w, d, thr, rids=None, nthreads=8):
    """TPC-C stock-level over three oracle trees; returns (results, seconds)."""
    w = np.ascontiguousarray(w, np.int64)
    d = np.ascontiguousarray(d, np.int64)
    thr = np.ascontiguousarray(thr, np.int32)
    r = None if rids is None else np.ascontiguousarray(rids, np.uint32)
    res = np.zeros(w.size, np.int32)
    sec = ctypes.c_double()
    lib().orc_stock_level_batch(dist.t, ol.t, stock.t, w.ctypes.data, d.ctypes.data, thr.ctypes.data,
                                r.ctypes.data if r is not None else None, w.size, res.ctypes.data, nthreads,
                                ctypes.byref(sec))
    return res, sec.value


def key_compare(k1, k2):
    a, b = bytes(k1), bytes(k2)
    return lib().orc_key_compare(a, len(a), b, len(b))


def murmur64a(data, seed=0):
    b = bytes(data)
    return lib().orc_murmur64a(b, len(b), seed)


def murmur64a_keys(keys, length=8, seed=0):
    keys = np.ascontiguousarray(keys, np.uint64)
    out = np.zeros(keys.size, np.uint64)
    lib().orc_murmur64a_batch(keys.ctypes.data, keys.size, length, seed, out.ctypes.data)
    return out


def payload(rowid, mode, size=1000):
    out = np.zeros(size, np.uint8)
    lib().orc_fill_payload(rowid, mode, out.ctypes.data, size)
    return out


def ref_murmur_lib():
    """The reference's own MurmurHash64A compiled from /root/reference (oracle/_ref), if present."""
    if not os.path.exists(REF_MURMUR_SO):
        return None
    L = ctypes.CDLL(REF_MURMUR_SO)
    L.ref_murmur64a.restype = u64
    L.ref_murmur64a.argtypes = [vp, ctypes.c_int, u64]
    return L
