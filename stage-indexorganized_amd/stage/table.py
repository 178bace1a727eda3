"""Host-side mirror of the reference's table interface over the C-ABI.

`Table` plays the role of the reference's `BTree` (include/vstore/b_tree.h:789-880) for the
read path: `read`/`probe` = BTree::Read + IndexScanExecutor point lookup (batched),
`range_scan` = RangeScanBySize + Iterator + TableScanExecutor, `insert`/`update`/... = the
host write path.  Numpy arrays in, numpy arrays out; device buffers are managed here.
"""
import ctypes

import numpy as np

from ._lib import StageParams, c_vp, check, lib

PROBE_OUT_DTYPE = np.dtype([
    ("status", "u1"), ("flags", "u1"), ("hops", "u2"), ("leaf", "u4"), ("slot", "u2"), ("key_len", "u2"),
    ("cstamp", "u4"), ("rec_cstamp", "u4"), ("copy_sstamp", "u4"), ("image", "u4"), ("meta_hi", "u4"),
])
assert PROBE_OUT_DTYPE.itemsize == 32
PROBE_OUT16_DTYPE = np.dtype([("status", "u1"), ("flags", "u1"), ("hops", "u2"), ("cstamp", "u4"),
                              ("copy_sstamp", "u4"), ("rec_cstamp", "u4")])
assert PROBE_OUT16_DTYPE.itemsize == 16
# stage_probe_ident: the hit record's RecordLocation handle and next handle
IDENT_DTYPE = np.dtype([("loc", "u4"), ("next", "u4")])
NEXT_COPY, NEXT_VERSION, NEXT_KIND_MASK, NEXT_INDEX_MASK = 0x40000000, 0x80000000, 0xC0000000, 0x3FFFFFFF
# stage_copy_state
COPY_STATE_DTYPE = np.dtype([("cstamp", "u4"), ("pstamp", "u4"), ("rstamp", "u4"), ("sstamp", "u4"),
                             ("readers", "u4"), ("count", "u2"), ("waiting", "u1"), ("pad", "u1")])

ST_NOT_FOUND, ST_LATEST, ST_COPY, ST_OLD, ST_FAIL_INVALID_TS, ST_CHAIN_MISS = range(6)
Q2_REC_DTYPE = np.dtype([
    ("supp_key", "i8"), ("s_w_id", "i8"), ("s_i_id", "i8"), ("s_quantity", "i4"), ("s_ytd", "i4"),
    ("s_order_cnt", "i4"), ("s_remote_cnt", "i4"), ("item_has_b", "u1"), ("update", "u1"), ("update_rc", "u1"),
    ("pad", "u1", (5,)),
])
assert Q2_REC_DTYPE.itemsize == 48
RC_INVALID, RC_OK, RC_KEY_EXISTS, RC_NOT_FOUND = 0, 1, 2, 3
RC_NOT_NEEDED_UPDATE, RC_DIRTY = 7, 9


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


class DeviceBuffer:
    """A hipMalloc'd buffer owned by Python."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        p = c_vp()
        check(lib().stage_dev_alloc(max(self.nbytes, 16), ctypes.byref(p)), "stage_dev_alloc")
        self.ptr = p.value

    @classmethod
    def from_numpy(cls, arr, stream=None):
        arr = np.ascontiguousarray(arr)
        b = cls(arr.nbytes)
        if arr.nbytes:
            check(lib().stage_memcpy_h2d(b.ptr, arr.ctypes.data, arr.nbytes, stream), "h2d")
        return b

    def to_numpy(self, dtype, count, stream=None, offset=0):
        """count elements from byte `offset` of the buffer."""
        out = np.empty(count, dtype=dtype)
        if out.nbytes:
            check(lib().stage_memcpy_d2h(out.ctypes.data, self.ptr + offset, out.nbytes, stream), "d2h")
        return out

    def memset(self, value=0, stream=None):
        """Fill the buffer; completes before returning (the library's streams are non-blocking,
        so an asynchronous fill on another stream could land after a later kernel's writes)."""
        check(lib().stage_dev_memset(self.ptr, value, self.nbytes, stream), "memset")
        check(lib().stage_stream_sync(stream) if stream else lib().stage_device_sync(), "memset sync")

    def free(self):
        if self.ptr:
            lib().stage_dev_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class _PinnedBlock:
    """stage_host_alloc memory kept alive by the numpy arrays viewing it."""

    def __init__(self, nbytes):
        p = c_vp()
        check(lib().stage_host_alloc(max(int(nbytes), 16), ctypes.byref(p)), "stage_host_alloc")
        self.ptr = p.value

    def __del__(self):
        try:
            if self.ptr:
                lib().stage_host_free(self.ptr)
        except Exception:
            pass


def pinned_empty(shape, dtype):
    """A numpy array in page-locked host memory (stage_host_alloc): result arrays the library
    can copy into straight from the device (e.g. ch_query2_batch's `out`)."""
    dtype = np.dtype(dtype)
    count = int(np.prod(shape)) if np.ndim(shape) else int(shape)
    blk = _PinnedBlock(count * dtype.itemsize)
    buf = (ctypes.c_uint8 * max(count * dtype.itemsize, 1)).from_address(blk.ptr)
    buf._stage_block = blk  # the block lives as long as an array viewing it
    return np.frombuffer(buf, dtype=dtype, count=count).reshape(shape)


class Stream:
    def __init__(self):
        p = c_vp()
        check(lib().stage_stream_create(ctypes.byref(p)), "stream")
        self.ptr = p.value

    def sync(self):
        check(lib().stage_stream_sync(self.ptr), "stream sync")

    def __del__(self):
        try:
            lib().stage_stream_destroy(self.ptr)
        except Exception:
            pass


class Event:
    def __init__(self):
        p = c_vp()
        check(lib().stage_event_create(ctypes.byref(p)), "event")
        self.ptr = p.value

    def record(self, stream):
        check(lib().stage_event_record(self.ptr, stream.ptr if stream else None), "event record")

    def elapsed_ms(self, other):
        ms = ctypes.c_float()
        check(lib().stage_event_elapsed(self.ptr, other.ptr, ctypes.byref(ms)), "event elapsed")
        return ms.value

    def __del__(self):
        try:
            lib().stage_event_destroy(self.ptr)
        except Exception:
            pass


class Table:
    """One index-organized table.  Defaults = the YCSB table (ycsb.cpp:72, ycsb_loader.cpp:27-57)."""

    def __init__(self, payload_size=1000, leaf_node_size=64 * 1024, split_threshold=16 * 1024,
                 merge_threshold=32 * 1024, key_width=8, device=0):
        p = StageParams(split_threshold, merge_threshold, leaf_node_size, payload_size, key_width, device)
        h = c_vp()
        check(lib().stage_table_create(ctypes.byref(p), ctypes.byref(h)), "stage_table_create")
        self.h = h.value
        self.payload_size = payload_size
        self.leaf_node_size = leaf_node_size
        self.key_width = key_width
        self.device = device

    def close(self):
        if self.h:
            lib().stage_table_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- properties
    @property
    def stride(self):
        return lib().stage_record_stride(self.h)

    @property
    def leaf_capacity(self):
        return lib().stage_leaf_capacity(self.h)

    def stats(self):
        s = np.zeros(8, np.uint64)
        check(lib().stage_stats(self.h, s.ctypes.data), "stats")
        keys = ["height", "inner", "leaves", "records", "sorted", "unsorted", "max_count", "versions"]
        return {k: int(v) for k, v in zip(keys, s)}

    # ---------------------------------------------------------------- host write path
    def insert(self, key, key_size=None, payload=None, gen_rowid=0, mode=0, commit_id=0):
        ks = key_size or self.key_width
        rc = ctypes.c_uint8()
        buf = None
        if payload is not None:
            buf = np.frombuffer(bytes(payload), np.uint8)
            assert buf.size == self.payload_size
        check(lib().stage_insert(self.h, int(key), ks, _ptr(buf), gen_rowid, mode, commit_id, ctypes.byref(rc)),
              "insert")
        return rc.value

    def load_ycsb(self, begin, end, key_size=None, mode=0):
        n = ctypes.c_uint64()
        check(lib().stage_load_ycsb(self.h, begin, end, key_size or self.key_width, mode, ctypes.byref(n)),
              "load_ycsb")
        return n.value

    def load_keys(self, keys, key_size=None, mode=0):
        keys = np.ascontiguousarray(keys, np.uint64)
        n = ctypes.c_uint64()
        check(lib().stage_load_keys(self.h, keys.ctypes.data, keys.size, key_size or self.key_width, mode,
                                    ctypes.byref(n)), "load_keys")
        return n.value

    def update(self, key, payload_off, delta, writer_id, key_size=None):
        d = np.frombuffer(bytes(delta), np.uint8)
        rc = ctypes.c_uint8()
        check(lib().stage_update(self.h, int(key), key_size or self.key_width, payload_off, d.ctypes.data, d.size,
                                 writer_id, ctypes.byref(rc)), "update")
        return rc.value

    def commit_update(self, key, commit_id, sstamp, key_size=None):
        rc = ctypes.c_uint8()
        check(lib().stage_commit_update(self.h, int(key), key_size or self.key_width, commit_id, sstamp,
                                        ctypes.byref(rc)), "commit_update")
        return rc.value

    def update_batch(self, keys, payload_off, deltas, writer_ids, commit_ids=None, sstamps=None, key_size=None):
        """Batched update (+ commit where commit_ids[i] != 0); returns (rc per key, number OK).

        ``deltas`` is an (n, delta_len) uint8 array, one patch per key."""
        keys = np.ascontiguousarray(keys, np.uint64)
        n = keys.size
        deltas = np.ascontiguousarray(deltas, np.uint8).reshape(n, -1) if n else np.zeros((0, 0), np.uint8)
        wid = np.ascontiguousarray(np.broadcast_to(np.asarray(writer_ids, np.uint32), (n,)))
        cid = None if commit_ids is None else np.ascontiguousarray(np.broadcast_to(np.asarray(commit_ids, np.uint32),
                                                                                    (n,)))
        sst = None if sstamps is None else np.ascontiguousarray(np.broadcast_to(np.asarray(sstamps, np.uint32), (n,)))
        rc = np.zeros(n, np.uint8)
        ok = ctypes.c_uint64()
        check(lib().stage_update_batch(self.h, keys.ctypes.data, 8, n, key_size or self.key_width, payload_off,
                                       deltas.ctypes.data, deltas.shape[1] if n else 0, wid.ctypes.data,
                                       cid.ctypes.data if cid is not None else None,
                                       sst.ctypes.data if sst is not None else None, rc.ctypes.data,
                                       ctypes.byref(ok)), "update_batch")
        return rc, ok.value

    def update_batch_device(self, keys, payload_off, deltas, writer_ids, commit_ids=None, sstamps=None, lens=None):
        """stage_update_batch_device: the same epoch applied by the device to the published
        image (keys as for probe: integers, or (n, width) uint8 key bytes); returns (rc, n_ok)."""
        words, n = self.key_buffer(keys)
        deltas = np.ascontiguousarray(deltas, np.uint8).reshape(n, -1) if n else np.zeros((0, 0), np.uint8)
        wid = np.ascontiguousarray(np.broadcast_to(np.asarray(writer_ids, np.uint32), (n,)))
        bufs = [DeviceBuffer.from_numpy(words) if n else DeviceBuffer(8),
                DeviceBuffer.from_numpy(deltas.reshape(-1)) if deltas.size else DeviceBuffer(8),
                DeviceBuffer.from_numpy(wid) if n else DeviceBuffer(8)]
        opt = []
        for a, dt in ((commit_ids, np.uint32), (sstamps, np.uint32), (lens, np.uint16)):
            if a is None or not n:
                opt.append(None)
            else:
                bufs.append(DeviceBuffer.from_numpy(np.ascontiguousarray(np.broadcast_to(np.asarray(a, dt), (n,)))))
                opt.append(bufs[-1].ptr)
        d_rc = DeviceBuffer(max(n, 1))
        ok = ctypes.c_uint64()
        check(lib().stage_update_batch_device(self.h, bufs[0].ptr, opt[2], n, payload_off, bufs[1].ptr,
                                              deltas.shape[1] if n else 0, bufs[2].ptr, opt[0], opt[1], d_rc.ptr,
                                              ctypes.byref(ok), None), "update_batch_device")
        rc = d_rc.to_numpy(np.uint8, n) if n else np.zeros(0, np.uint8)
        return rc, ok.value

    def finalize_update(self, key, commit_id, key_size=None):
        rc = ctypes.c_uint8()
        check(lib().stage_finalize_update(self.h, int(key), key_size or self.key_width, commit_id, ctypes.byref(rc)),
              "finalize_update")
        return rc.value

    def delete(self, key, commit_id=0, key_size=None):
        rc = ctypes.c_uint8()
        check(lib().stage_delete(self.h, int(key), key_size or self.key_width, commit_id, ctypes.byref(rc)), "delete")
        return rc.value

    def sync(self):
        check(lib().stage_sync(self.h), "stage_sync")

    def sync_info(self):
        """What the last sync did: {'incremental', 'leaves', 'slots', 'seconds'}."""
        sec = ctypes.c_double()
        info = np.zeros(3, np.uint64)
        check(lib().stage_sync_info(self.h, ctypes.byref(sec), info.ctypes.data), "sync_info")
        return {"incremental": bool(info[0]), "leaves": int(info[1]), "slots": int(info[2]), "seconds": sec.value}

    def export_leaves(self, cap=None):
        cap = cap or self.leaf_capacity
        nl = self.stats()["leaves"]
        rc = np.zeros(nl, np.uint32)
        sc = np.zeros(nl, np.uint32)
        meta = np.zeros(nl * cap, np.uint64)
        keyw = np.zeros(nl * cap, np.uint64)
        got = lib().stage_export_leaves(self.h, cap, nl, rc.ctypes.data, sc.ctypes.data, meta.ctypes.data,
                                        keyw.ctypes.data)
        if got < 0:
            raise RuntimeError("export_leaves failed")
        return rc, sc, meta.reshape(nl, cap), keyw.reshape(nl, cap)

    def export_leaf_images(self):
        """Reference-format leaf blocks in key order + upper separators (key_le, len; 0xFFFF = +inf)."""
        nl = self.stats()["leaves"]
        kw = self.key_words
        blocks = np.zeros((nl, self.leaf_node_size), np.uint8)
        sk = np.zeros(nl * kw, np.uint64)
        sl = np.zeros(nl, np.uint16)
        got = lib().stage_export_leaf_images(self.h, nl, blocks.ctypes.data, sk.ctypes.data, sl.ctypes.data)
        if got < 0:
            check(int(got), "export_leaf_images")
        return blocks[:got], (sk[:got] if kw == 1 else sk.reshape(nl, kw)[:got]), sl[:got]

    def import_leaf_images(self, blocks, sep_keys=None, sep_lens=None):
        blocks = np.ascontiguousarray(blocks, np.uint8)
        n = ctypes.c_uint64()
        sk = None if sep_keys is None else np.ascontiguousarray(sep_keys, np.uint64).reshape(-1)
        sl = None if sep_lens is None else np.ascontiguousarray(sep_lens, np.uint16)
        check(lib().stage_import_leaf_images(self.h, blocks.ctypes.data, blocks.shape[0], blocks.shape[1], _ptr(sk),
                                             _ptr(sl), ctypes.byref(n)), "import_leaf_images")
        return n.value

    def export_locations(self):
        """RecordLocation handles of every live record -> (handles, leaf in key order, slot)"""
        n = lib().stage_export_locations(self.h, 0, None, None, None)
        if n < 0:
            raise RuntimeError("export_locations failed")
        h = np.zeros(n, np.uint64)
        lf = np.zeros(n, np.uint32)
        sl = np.zeros(n, np.uint16)
        if n:
            lib().stage_export_locations(self.h, n, h.ctypes.data, lf.ctypes.data, sl.ctypes.data)
        return h, lf, sl

    def resolve_locations(self, handles):
        """where each RecordLocation handle's record is now: (leaf, slot); 0xFFFFFFFF / 0xFFFF = gone"""
        handles = np.ascontiguousarray(handles, np.uint64)
        lf = np.zeros(handles.size, np.uint32)
        sl = np.zeros(handles.size, np.uint16)
        check(lib().stage_resolve_locations(self.h, handles.ctypes.data, handles.size, lf.ctypes.data, sl.ctypes.data),
              "resolve_locations")
        return lf, sl

    @property
    def key_words(self):
        return int(lib().stage_key_words(self.h))

    def key_buffer(self, keys):
        """Keys -> (u64 words, count): 1-D integer keys (tables of <= 8-byte keys) or a 2-D uint8
        array of key bytes (n, width), zero padded to stage_key_words() words per key."""
        kw = self.key_words
        a = np.asarray(keys)
        if a.ndim == 2:
            a = np.ascontiguousarray(a, np.uint8)
            buf = np.zeros((a.shape[0], kw * 8), np.uint8)
            buf[:, :a.shape[1]] = a
            return buf.view(np.uint64).reshape(-1), a.shape[0]
        assert kw == 1, "tables with keys above 8 bytes take (n, width) uint8 key arrays"
        a = np.ascontiguousarray(a, np.uint64).reshape(-1)
        return a, a.size

    def traverse(self, keys, lens=None, le_child=True):
        words, n = self.key_buffer(keys)
        lens = None if lens is None else np.ascontiguousarray(lens, np.uint16)
        out = np.zeros(n, np.uint32)
        check(lib().stage_traverse_batch(self.h, words.ctypes.data, _ptr(lens), n, int(le_child),
                                         out.ctypes.data), "traverse")
        return out

    # ---------------------------------------------------------------- byte-key write path
    def insert_key(self, key, payload, commit_id=0):
        k = np.frombuffer(bytes(key), np.uint8)
        p = np.frombuffer(bytes(payload), np.uint8)
        assert p.size == self.payload_size
        rc = ctypes.c_uint8()
        check(lib().stage_insert_key(self.h, k.ctypes.data, k.size, p.ctypes.data, commit_id, ctypes.byref(rc)),
              "insert_key")
        return rc.value

    def insert_key_inflight(self, key, payload, writer_id):
        """stage_insert_key_inflight: an uncommitted transaction's insert (PrepareForInsert)"""
        k = np.frombuffer(bytes(key), np.uint8)
        p = np.frombuffer(bytes(payload), np.uint8)
        assert p.size == self.payload_size
        rc = ctypes.c_uint8()
        check(lib().stage_insert_key_inflight(self.h, k.ctypes.data, k.size, p.ctypes.data, writer_id,
                                              ctypes.byref(rc)), "insert_key_inflight")
        return rc.value

    def commit_insert_key(self, key, commit_id):
        """stage_commit_insert_key: CommitTransaction INSERT entry (FinalizeForInsert(t_cstamp))"""
        k = np.frombuffer(bytes(key), np.uint8)
        rc = ctypes.c_uint8()
        check(lib().stage_commit_insert_key(self.h, k.ctypes.data, k.size, commit_id, ctypes.byref(rc)),
              "commit_insert_key")
        return rc.value

    def load_rows(self, keys, payloads, commit_id=0):
        """keys (n, width) uint8, payloads (n, payload_size) uint8 -> (rc per row, inserted)."""
        keys = np.ascontiguousarray(keys, np.uint8)
        payloads = np.ascontiguousarray(payloads, np.uint8)
        n = keys.shape[0]
        assert payloads.shape == (n, self.payload_size)
        rc = np.zeros(n, np.uint8)
        ins = ctypes.c_uint64()
        check(lib().stage_load_rows(self.h, keys.ctypes.data, keys.shape[1], keys.shape[1], payloads.ctypes.data,
                                    payloads.shape[1], n, commit_id, rc.ctypes.data, ctypes.byref(ins)), "load_rows")
        return rc, ins.value

    def update_key(self, key, payload_off, delta, writer_id):
        k = np.frombuffer(bytes(key), np.uint8)
        d = np.frombuffer(bytes(delta), np.uint8)
        rc = ctypes.c_uint8()
        check(lib().stage_update_key(self.h, k.ctypes.data, k.size, payload_off, d.ctypes.data, d.size, writer_id,
                                     ctypes.byref(rc)), "update_key")
        return rc.value

    def update_key_owned(self, key, payload_off, delta, writer_id):
        """LeafNode::Update with is_for_update = true: in place, no copy (b_tree.cpp:1101-1104)"""
        k = np.frombuffer(bytes(key), np.uint8)
        d = np.frombuffer(bytes(delta), np.uint8)
        rc = ctypes.c_uint8()
        check(lib().stage_update_key_owned(self.h, k.ctypes.data, k.size, payload_off, d.ctypes.data, d.size,
                                           writer_id, ctypes.byref(rc)), "update_key_owned")
        return rc.value

    def delete_key_owned(self, key):
        """LeafNode::Delete with is_for_update = true: meta := 0 (b_tree.cpp:1210-1220)"""
        k = np.frombuffer(bytes(key), np.uint8)
        rc = ctypes.c_uint8()
        check(lib().stage_delete_key_owned(self.h, k.ctypes.data, k.size, ctypes.byref(rc)), "delete_key_owned")
        return rc.value

    def commit_update_key(self, key, commit_id, sstamp):
        k = np.frombuffer(bytes(key), np.uint8)
        rc = ctypes.c_uint8()
        check(lib().stage_commit_update_key(self.h, k.ctypes.data, k.size, commit_id, sstamp, ctypes.byref(rc)),
              "commit_update_key")
        return rc.value

    def delete_key(self, key, commit_id=0):
        k = np.frombuffer(bytes(key), np.uint8)
        rc = ctypes.c_uint8()
        check(lib().stage_delete_key(self.h, k.ctypes.data, k.size, commit_id, ctypes.byref(rc)), "delete_key")
        return rc.value

    def abort_update_key(self, key):
        """AbortTransaction UPDATE entry (transaction_manager.cpp:846-921) for one key"""
        k = np.frombuffer(bytes(key), np.uint8)
        rc = ctypes.c_uint8()
        check(lib().stage_abort_update_key(self.h, k.ctypes.data, k.size, ctypes.byref(rc)), "abort_update_key")
        return rc.value

    def abort_insert_key(self, key):
        """AbortTransaction INSERT entry (transaction_manager.cpp:949-979) for one key"""
        k = np.frombuffer(bytes(key), np.uint8)
        rc = ctypes.c_uint8()
        check(lib().stage_abort_insert_key(self.h, k.ctypes.data, k.size, ctypes.byref(rc)), "abort_insert_key")
        return rc.value

    # ---------------------------------------------------------------- device read path
    def probe_device(self, d_keys, n, d_out, d_records=None, d_read_ids=None, d_lens=None, d_leaf_ids=None,
                     stream=None):
        check(lib().stage_probe_batch(self.h, d_keys, d_lens, d_read_ids, d_leaf_ids, n, d_out, d_records,
                                      stream), "stage_probe_batch")

    def probe(self, keys, read_ids=None, lens=None, leaf_ids=None, records=True, for_update=None):
        """Batched BTree::Read + visibility.  Returns (out[n] PROBE_OUT_DTYPE, rows[n, stride] or None).
        for_update: per-probe is_for_update flags (stage_probe_batch_ex)."""
        words, n = self.key_buffer(keys)
        bufs = [DeviceBuffer.from_numpy(words) if n else DeviceBuffer(8)]
        d_rids = d_lens = d_leaf = None
        d_fu = None
        if for_update is not None:
            bufs.append(DeviceBuffer.from_numpy(np.ascontiguousarray(for_update, np.uint8)) if n else DeviceBuffer(8))
            d_fu = bufs[-1].ptr
        if read_ids is not None:
            bufs.append(DeviceBuffer.from_numpy(np.ascontiguousarray(read_ids, np.uint32)))
            d_rids = bufs[-1].ptr
        if lens is not None:
            bufs.append(DeviceBuffer.from_numpy(np.ascontiguousarray(lens, np.uint16)))
            d_lens = bufs[-1].ptr
        if leaf_ids is not None:
            bufs.append(DeviceBuffer.from_numpy(np.ascontiguousarray(leaf_ids, np.uint32)))
            d_leaf = bufs[-1].ptr
        dt = PROBE_OUT16_DTYPE if getattr(self, "status_bytes", 32) == 16 else PROBE_OUT_DTYPE
        d_out = DeviceBuffer(n * dt.itemsize)
        d_rec = DeviceBuffer(n * self.stride) if records else None
        if d_fu is None:
            self.probe_device(bufs[0].ptr, n, d_out.ptr, d_rec.ptr if d_rec else None, d_rids, d_lens, d_leaf)
        else:
            check(lib().stage_probe_batch_ex(self.h, bufs[0].ptr, d_lens, d_rids, d_leaf, d_fu, n, d_out.ptr,
                                             d_rec.ptr if d_rec else None, None), "stage_probe_batch_ex")
        check(lib().stage_device_sync(), "sync")
        out = d_out.to_numpy(dt, n)
        rows = d_rec.to_numpy(np.uint8, n * self.stride).reshape(n, self.stride) if d_rec else None
        return out, rows

    def identify(self, keys, read_ids=None):
        """stage_probe_batch + stage_probe_identify: (out[n], ident[n] IDENT_DTYPE) -- each hit's
        RecordLocation handle and next handle (the Record's loc_ptr / next_ptr)"""
        words, n = self.key_buffer(keys)
        bufs = [DeviceBuffer.from_numpy(words) if n else DeviceBuffer(8)]
        d_rids = None
        if read_ids is not None:
            bufs.append(DeviceBuffer.from_numpy(np.ascontiguousarray(read_ids, np.uint32)))
            d_rids = bufs[-1].ptr
        d_out = DeviceBuffer(max(1, n) * 32)
        d_id = DeviceBuffer(max(1, n) * 8)
        self.probe_device(bufs[0].ptr, n, d_out.ptr, None, d_rids)
        check(lib().stage_probe_identify(self.h, d_out.ptr, n, d_id.ptr, None), "stage_probe_identify")
        check(lib().stage_device_sync(), "sync")
        return d_out.to_numpy(PROBE_OUT_DTYPE, n), d_id.to_numpy(IDENT_DTYPE, n)

    def record_meta(self, key, key_size=None):
        """stage_record_meta_key: (meta word, location handle, next handle) or None"""
        kb = np.array([int(key)], np.uint64).tobytes()[:key_size or self.key_width]
        meta = ctypes.c_uint64()
        ident = np.zeros(1, IDENT_DTYPE)
        rc = ctypes.c_uint8()
        check(lib().stage_record_meta_key(self.h, kb, len(kb), ctypes.byref(meta), ident.ctypes.data, ctypes.byref(rc)),
              "record_meta_key")
        return None if rc.value != RC_OK else (meta.value, int(ident[0]["loc"]), int(ident[0]["next"]))

    def enable_location_cells(self):
        check(lib().stage_location_cells(self.h), "location_cells")

    def location_cell(self, handle):
        """the 24-B RecordMetadata {meta, next_ptr, loc_ptr} location `handle` points at now"""
        p = ctypes.c_void_p()
        check(lib().stage_location_cell(self.h, handle, ctypes.byref(p)), "location_cell")
        return tuple(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint64))[i] for i in range(3))

    def copy_state(self, copy_id):
        """stage_copy_get + stage_copy_readers: dict of the overwrite copy's transaction state"""
        st = np.zeros(1, COPY_STATE_DTYPE)
        ids = np.array([copy_id], np.uint32)
        check(lib().stage_copy_get(self.h, ids.ctypes.data, 1, st.ctypes.data), "copy_get")
        d = {k: int(st[0][k]) for k in COPY_STATE_DTYPE.names if k != "pad"}
        buf = np.zeros(max(1, d["readers"]), np.uint32)
        cnt = ctypes.c_uint32()
        check(lib().stage_copy_readers(self.h, copy_id, buf.ctypes.data, buf.size, ctypes.byref(cnt)), "copy_readers")
        d["reader_ids"] = buf[:cnt.value].tolist()
        return d

    def set_write_overlap(self, on):
        """stage_set_write_overlap: a device write-path epoch's kernels up to its publish run beside
        the caller's later work (inputs must be complete when update_batch_device is called)."""
        check(lib().stage_set_write_overlap(self.h, int(on)), "set_write_overlap")

    def set_output_layout(self, row_stride=0, status_bytes=32):
        """stage_set_output_layout: probe row stride (0 = default) and 32- or 16-B status records."""
        check(lib().stage_set_output_layout(self.h, row_stride, status_bytes), "set_output_layout")
        self.status_bytes = status_bytes

    def probe_host(self, keys, read_ids=None, lens=None, records=True, out=None, rows=None):
        """stage_probe_host: the same probe with host-memory inputs and outputs (pipelined).
        `out` / `rows`: caller-owned result arrays (e.g. pinned_empty) to fill instead of new ones;
        status records are 16 B after set_output_layout(.., 16)."""
        keys, n = self.key_buffer(keys)
        rids = None if read_ids is None else np.ascontiguousarray(read_ids, np.uint32)
        ln = None if lens is None else np.ascontiguousarray(lens, np.uint16)
        dt = PROBE_OUT16_DTYPE if getattr(self, "status_bytes", 32) == 16 else PROBE_OUT_DTYPE
        if out is None:
            out = np.zeros(n, dt)
        assert out.dtype == dt and out.size >= n, "out: n status records of the table's layout"
        if rows is None and records:
            rows = np.zeros((n, self.stride), np.uint8)
        assert rows is None or (rows.shape[0] >= n and rows.shape[1] == self.stride and rows.flags.c_contiguous)
        check(lib().stage_probe_host(self.h, keys.ctypes.data, _ptr(ln), _ptr(rids), n, out.ctypes.data, _ptr(rows)),
              "probe_host")
        return out, rows

    def reader(self, max_batch=1024, max_wait_us=50, **resident):
        return Reader(self, max_batch, max_wait_us, **resident)

    def range_scan(self, start_keys, scan_size, lens=None):
        """TableScanExecutor over RangeScanBySize/Iterator.  Returns (counts[n], rows[n, scan_size, stride])."""
        keys, n = self.key_buffer(start_keys)
        d_keys = DeviceBuffer.from_numpy(keys)
        d_lens = DeviceBuffer.from_numpy(np.ascontiguousarray(lens, np.uint16)) if lens is not None else None
        d_cnt = DeviceBuffer(n * 4)
        d_rec = DeviceBuffer(max(1, n * scan_size * self.stride))
        d_rec.memset(0)
        check(lib().stage_scan_batch(self.h, d_keys.ptr, d_lens.ptr if d_lens else None, n, scan_size, d_cnt.ptr,
                                     d_rec.ptr, None), "stage_scan_batch")
        check(lib().stage_device_sync(), "sync")
        counts = d_cnt.to_numpy(np.uint32, n)
        rows = d_rec.to_numpy(np.uint8, n * scan_size * self.stride).reshape(n, scan_size, self.stride)
        return counts, rows

    def index_scan(self, start_keys, scan_size, read_ids=None, lens=None):
        """IndexScanExecutor range branch: (counts[n], rows[n, scan_size, stride], status[n, scan_size])."""
        keys, n = self.key_buffer(start_keys)
        d_keys = DeviceBuffer.from_numpy(keys)
        d_lens = DeviceBuffer.from_numpy(np.ascontiguousarray(lens, np.uint16)) if lens is not None else None
        d_rid = DeviceBuffer.from_numpy(np.ascontiguousarray(read_ids, np.uint32)) if read_ids is not None else None
        d_cnt = DeviceBuffer(n * 4)
        d_rec = DeviceBuffer(max(1, n * scan_size * self.stride))
        d_st = DeviceBuffer(max(1, n * scan_size))
        d_rec.memset(0)
        d_st.memset(0)
        check(lib().stage_index_scan_batch(self.h, d_keys.ptr, d_lens.ptr if d_lens else None,
                                           d_rid.ptr if d_rid else None, n, scan_size, d_cnt.ptr, d_rec.ptr,
                                           d_st.ptr, None), "stage_index_scan_batch")
        check(lib().stage_device_sync(), "sync")
        counts = d_cnt.to_numpy(np.uint32, n)
        rows = d_rec.to_numpy(np.uint8, n * scan_size * self.stride).reshape(n, scan_size, self.stride)
        st = d_st.to_numpy(np.uint8, n * scan_size).reshape(n, scan_size)
        return counts, rows, st

    def index_scan_first(self, start_keys, scan_size, prefix_words, read_ids=None):
        """index_scan consumed up to its first LATEST / OLD tuple carrying the start key's first
        prefix_words fields: (image[n] heap rows, status[n])."""
        keys, n = self.key_buffer(start_keys)
        d_keys = DeviceBuffer.from_numpy(keys)
        d_rid = DeviceBuffer.from_numpy(np.ascontiguousarray(read_ids, np.uint32)) if read_ids is not None else None
        d_img = DeviceBuffer(max(4, n * 4))
        d_st = DeviceBuffer(max(1, n))
        check(lib().stage_index_scan_first_batch(self.h, d_keys.ptr, d_rid.ptr if d_rid else None, n, scan_size,
                                                 prefix_words, d_img.ptr, d_st.ptr, None),
              "stage_index_scan_first_batch")
        check(lib().stage_device_sync(), "sync")
        return d_img.to_numpy(np.uint32, n), d_st.to_numpy(np.uint8, n)

    def resolve(self, keys, lens=None, le_child=True):
        keys, n = self.key_buffer(keys)
        d_keys = DeviceBuffer.from_numpy(keys)
        d_lens = DeviceBuffer.from_numpy(np.ascontiguousarray(lens, np.uint16)) if lens is not None else None
        d_out = DeviceBuffer(n * 4)
        check(lib().stage_resolve_batch(self.h, d_keys.ptr, d_lens.ptr if d_lens else None, n,
                                        int(le_child), d_out.ptr, None), "resolve")
        check(lib().stage_device_sync(), "sync")
        return d_out.to_numpy(np.uint32, n)


class Reader:
    """stage_reader: thread-safe single-key BTree::Read adapter (calls are coalesced into
    device batches).  ``read`` releases the GIL inside the library, so Python threads
    calling it concurrently are batched together.  ``resident=True``: the device side stays
    resident and polls a request ring (stage_reader_create_resident)."""

    def __init__(self, table, max_batch=1024, max_wait_us=50, resident=False, ring_slots=4096, waves=16,
                 life_us=5000):
        self.table = table
        self.resident = resident
        h = ctypes.c_void_p()
        if resident:
            check(lib().stage_reader_create_resident(table.h, ring_slots, waves, life_us, ctypes.byref(h)),
                  "reader_create_resident")
        else:
            check(lib().stage_reader_create(table.h, max_batch, max_wait_us, ctypes.byref(h)), "reader_create")
        self.h = h

    def read(self, key, read_id=0xFFFFFFFE, key_size=None, record=True):
        out = np.zeros(1, PROBE_OUT_DTYPE)
        row = np.zeros(8 + self.table.payload_size, np.uint8) if record else None
        check(lib().stage_reader_read(self.h, int(key), key_size or self.table.key_width, read_id, out.ctypes.data,
                                      _ptr(row)), "reader_read")
        return out[0], row

    def read_ex(self, key, read_id=0xFFFFFFFE, for_update=False, key_size=None):
        """stage_reader_read_ex: (out, row, ident) of BTree::Read(.., is_for_update)"""
        out = np.zeros(1, PROBE_OUT_DTYPE)
        row = np.zeros(8 + self.table.payload_size, np.uint8)
        ident = np.zeros(1, IDENT_DTYPE)
        check(lib().stage_reader_read_ex(self.h, int(key), key_size or self.table.key_width, read_id,
                                         1 if for_update else 0, out.ctypes.data, row.ctypes.data,
                                         ident.ctypes.data), "reader_read_ex")
        return out[0], row, ident[0]

    def read_ident(self, key, read_id=0xFFFFFFFE, key_size=None):
        """stage_reader_read_ident: (out, row, ident)"""
        out = np.zeros(1, PROBE_OUT_DTYPE)
        row = np.zeros(8 + self.table.payload_size, np.uint8)
        ident = np.zeros(1, IDENT_DTYPE)
        check(lib().stage_reader_read_ident(self.h, int(key), key_size or self.table.key_width, read_id,
                                            out.ctypes.data, row.ctypes.data, ident.ctypes.data), "reader_read_ident")
        return out[0], row, ident[0]

    def stats(self):
        s = np.zeros(3, np.uint64)
        check(lib().stage_reader_stats(self.h, s.ctypes.data), "reader_stats")
        return {"batches": int(s[0]), "reads": int(s[1]), "full_batches": int(s[2])}

    def close(self):
        if self.h:
            lib().stage_reader_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


REPLY_ROWS, REPLY_OWNER, REPLY_PEER, REPLY_DIRECT = 0, 1, 2, 3  # stage_hip.h STAGE_REPLY_*


def owner_rows(table, loopback=True):
    """(device pointer, row count) of the rows an owner-reply sharded probe left on `table`."""
    p = ctypes.c_void_p()
    n = ctypes.c_uint64()
    check(lib().stage_sharded_owner_rows(table.h, int(loopback), ctypes.byref(p), ctypes.byref(n)), "owner_rows")
    return p.value, n.value


def set_shard_dedupe(table, on):
    """stage_set_shard_dedupe: request coalescing of the sharded front-end (-1 = env default)."""
    check(lib().stage_set_shard_dedupe(table.h, int(on)), "set_shard_dedupe")


def set_shard_key_bits(table, bits):
    """stage_set_shard_key_bits: the coalescing sort reads the low `bits` key bits (0 = 64);
    same results for any value, fewer radix passes when every key is < 2^bits."""
    check(lib().stage_set_shard_key_bits(table.h, int(bits)), "set_shard_key_bits")


def rccl_info():
    """stage_rccl_info: {"runtime": ncclGetVersion, "headers": the version libstage_hip was built
    against, "path": the file that provided ncclGetVersion in this process}."""
    rt, hd = ctypes.c_int(), ctypes.c_int()
    buf = ctypes.create_string_buffer(512)
    check(lib().stage_rccl_info(ctypes.byref(rt), ctypes.byref(hd), buf, 512), "rccl_info")
    return {"runtime": rt.value, "headers": hd.value, "path": buf.value.decode()}


def sharded_stats_ex(table, loopback=False):
    """stage_sharded_stats_ex: {keys, routed, remote, received} of the last sharded probe --
    caller keys, requests routed after coalescing, of those owned by other ranks, and the
    requests this rank probed as owner."""
    v = (ctypes.c_uint64 * 4)()
    check(lib().stage_sharded_stats_ex(table.h, int(loopback), v, 4), "sharded_stats_ex")
    return dict(zip(("keys", "routed", "remote", "received"), (int(x) for x in v)))


def comm_allreduce(table, values, op="sum"):
    """stage_comm_allreduce_f64 over the table's communicator (op: sum / max / min)."""
    v = np.ascontiguousarray(values, np.float64).copy()
    check(lib().stage_comm_allreduce_f64(table.h, v.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), v.size,
                                         {"sum": 0, "max": 1, "min": 2}[op]), "comm_allreduce")
    return v


def comm_allgather(table, values, world):
    """stage_comm_allgather_f64: [world, n] array of every rank's values."""
    v = np.ascontiguousarray(values, np.float64)
    out = np.zeros((world, v.size), np.float64)
    check(lib().stage_comm_allgather_f64(table.h, v.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), v.size,
                                         out.ctypes.data_as(ctypes.POINTER(ctypes.c_double))), "comm_allgather")
    return out


def sharded_stats(table, loopback=True):
    """stage_sharded_stats: (caller keys, routed requests, remote requests) of the last sharded probe."""
    v = [ctypes.c_uint64() for _ in range(3)]
    check(lib().stage_sharded_stats(table.h, int(loopback), *[ctypes.byref(x) for x in v]), "sharded_stats")
    return tuple(x.value for x in v)


def probe_sharded_loopback(tables, keys_per_rank, read_ids_per_rank=None, records=True, reply=REPLY_ROWS):
    """stage_probe_sharded_loopback: rank r's keys are routed across the shard tables (all on
    one device) exactly as stage_probe_sharded routes them over RCCL; returns per-rank
    (out, rows) in each rank's own key order."""
    W = len(tables)
    keep = []
    k_ptrs, r_ptrs, o_ptrs, rec_ptrs, ns = [], [], [], [], []
    stride = tables[0].stride
    for r in range(W):
        k = np.ascontiguousarray(keys_per_rank[r], np.uint64)
        n = k.size
        dk = DeviceBuffer.from_numpy(k) if n else DeviceBuffer(8)
        do = DeviceBuffer(max(n, 1) * 32)
        dr = DeviceBuffer(max(n, 1) * stride) if records else None
        keep.append((dk, do, dr))
        k_ptrs.append(dk.ptr)
        o_ptrs.append(do.ptr)
        rec_ptrs.append(dr.ptr if dr else None)
        ns.append(n)
        if read_ids_per_rank is not None:
            ri = np.ascontiguousarray(read_ids_per_rank[r], np.uint32)
            drid = DeviceBuffer.from_numpy(ri) if n else DeviceBuffer(4)
            keep.append((drid,))
            r_ptrs.append(drid.ptr)
    arr = lambda v: (ctypes.c_void_p * W)(*v)
    hs = (ctypes.c_void_p * W)(*[t.h for t in tables])
    n_arr = (ctypes.c_uint64 * W)(*ns)
    check(lib().stage_probe_sharded_loopback(hs, W, arr(k_ptrs), arr(r_ptrs) if r_ptrs else None, n_arr, arr(o_ptrs),
                                             arr(rec_ptrs), reply, None), "probe_sharded_loopback")
    check(lib().stage_device_sync(), "sync")
    res = []
    trip = [x for x in keep if len(x) == 3]
    for r in range(W):
        n = ns[r]
        _, do, dr = trip[r]
        out = do.to_numpy(PROBE_OUT_DTYPE, n) if n else np.zeros(0, PROBE_OUT_DTYPE)
        rows = (dr.to_numpy(np.uint8, n * stride).reshape(n, stride) if n else np.zeros((0, stride), np.uint8)) \
            if records else None
        res.append((out, rows))
    return res


def murmur64a_device(keys, key_len=8, seed=0):
    keys = np.ascontiguousarray(keys, np.uint64)
    d_keys = DeviceBuffer.from_numpy(keys)
    d_out = DeviceBuffer(keys.size * 8)
    check(lib().stage_murmur64a_batch(d_keys.ptr, key_len, 8, seed, keys.size, d_out.ptr, None), "murmur")
    check(lib().stage_device_sync(), "sync")
    return d_out.to_numpy(np.uint64, keys.size)


def zipf_draws(n, theta, seed, count, nthreads=8):
    out = np.empty(count, np.uint64)
    check(lib().stage_zipf_draws(n, theta, seed, count, out.ctypes.data, nthreads), "zipf")
    return out


def zipf_zeta(n, theta):
    out = np.zeros(1, np.float64)
    check(lib().stage_zipf_zeta(n, theta, out.ctypes.data), "zeta")
    return float(out[0])


def fastrandom(seed, count):
    out = np.empty(count, np.uint64)
    check(lib().stage_fastrandom_next(seed, count, out.ctypes.data), "fastrandom")
    return out


def ycsb_ops(seed, count, update_ratio):
    """RunMixed's per-op stream (ycsb_mixed.cpp:26-44): (is_update bool[count], delta byte u8[count])"""
    upd = np.empty(count, np.uint8)
    chr_ = np.empty(count, np.uint8)
    check(lib().stage_ycsb_ops(seed, count, update_ratio, upd.ctypes.data, chr_.ctypes.data), "ycsb_ops")
    return upd.astype(bool), chr_


def device_count():
    c = ctypes.c_int(0)
    rc = lib().stage_device_count(ctypes.byref(c))
    return c.value if rc == 0 else 0


def ch_query2(region, nation, supplier, item, stock, map_off, d_map_keys, target_region=3, read_id=0xFFFFFFFE,
              commit_id=0, max_out=1 << 14, stream=None, out=None):
    """stage_ch_query2 (RunQuery2): returns (records Q2_REC_DTYPE[n], aborted); `out` (a
    Q2_REC_DTYPE array) is reused when given."""
    map_off = np.ascontiguousarray(map_off, np.uint32)
    if out is None:
        out = np.zeros(max_out, Q2_REC_DTYPE)
    max_out = out.size
    n = ctypes.c_uint64()
    ab = ctypes.c_int32()
    check(lib().stage_ch_query2(region.h, nation.h, supplier.h, item.h, stock.h, map_off.ctypes.data, d_map_keys,
                                int(target_region), int(read_id), int(commit_id), out.ctypes.data, max_out,
                                ctypes.byref(n), ctypes.byref(ab), stream), "ch_query2")
    return out[:min(n.value, max_out)], bool(ab.value)


def ch_query2_batch(region, nation, supplier, item, stock, map_off, d_map_keys, read_ids, target_region=3,
                    max_per_query=1 << 14, stream=None, out=None):
    """stage_ch_query2_batch: nq read-only Q2s in one pass -> (records [nq, n] Q2_REC_DTYPE, aborted[nq]).
    out: a caller-owned [nq, max_per_query] Q2_REC_DTYPE array to fill (the result is a view of it)."""
    map_off = np.ascontiguousarray(map_off, np.uint32)
    rids = np.ascontiguousarray(read_ids, np.uint32)
    nq = rids.size
    if out is None:
        out = np.zeros((nq, max_per_query), Q2_REC_DTYPE)
    else:
        assert out.dtype == Q2_REC_DTYPE and out.flags.c_contiguous and out.shape[0] == nq
        max_per_query = out.shape[1]
    ab = np.zeros(nq, np.int32)
    n = ctypes.c_uint64()
    check(lib().stage_ch_query2_batch(region.h, nation.h, supplier.h, item.h, stock.h, map_off.ctypes.data,
                                      d_map_keys, int(target_region), rids.ctypes.data, nq, out.ctypes.data,
                                      max_per_query, ctypes.byref(n), ab.ctypes.data, stream), "ch_query2_batch")
    return out[:, :min(n.value, max_per_query)], ab.astype(bool)


class Q2Batch:
    """An enqueued stage_ch_query2_batch_async batch (slot 0 or 1); wait() -> (records [nq, n],
    aborted[nq]).  `out` is a page-locked [nq, max_per_query] Q2_REC_DTYPE array (pinned_empty)
    left untouched until wait() returns."""

    def __init__(self, stock, slot, out, nq):
        self.stock, self.slot, self.out, self.nq, self.done = stock, slot, out, nq, None

    def wait(self):
        if self.done is None:
            n = ctypes.c_uint64()
            ab = np.zeros(self.nq, np.int32)
            check(lib().stage_ch_query2_wait(self.stock.h, self.slot, ctypes.byref(n), ab.ctypes.data),
                  "ch_query2_wait")
            self.done = (self.out[:, :min(n.value, self.out.shape[1])], ab.astype(bool))
        return self.done


def ch_query2_batch_async(region, nation, supplier, item, stock, map_off, d_map_keys, read_ids, out, slot=0,
                          target_region=3, stream=None):
    """stage_ch_query2_batch_async: ch_query2_batch without the wait (two slots may be in flight)."""
    map_off = np.ascontiguousarray(map_off, np.uint32)
    rids = np.ascontiguousarray(read_ids, np.uint32)
    nq = rids.size
    assert out.dtype == Q2_REC_DTYPE and out.flags.c_contiguous and out.ndim == 2 and out.shape[0] == nq
    check(lib().stage_ch_query2_batch_async(region.h, nation.h, supplier.h, item.h, stock.h, map_off.ctypes.data,
                                            d_map_keys, int(target_region), rids.ctypes.data, nq, out.ctypes.data,
                                            out.shape[1], int(slot), stream), "ch_query2_batch_async")
    return Q2Batch(stock, slot, out, nq)
