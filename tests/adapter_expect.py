"""Expected bytes of the reference-side adapter (include/stage_btree_adapter.hpp), stated
independently in Python from the reference's definitions and computed from the ORACLE:

  Record   (b_tree.h:400-448): RecordMeta{RecordMetadata{meta, next_ptr, loc_ptr} 24 B,
           total_size u32 (+4 pad), next_tuple_ptr u64, cstamp u32 (+4 pad)} = 48 B, then
           tuple_data_ = [cstamp u32][key padded to 8][payload]
  outcome  (executor.h:374-454): ResultType FAILURE only for a chain hit on an INVALID_CID
           begin/end; PerformRead for latest / copy reads; a tuple for latest / copy / old
  YCSBTupleInt (ycsb_configuration.h:38-40, 1004 B): latest / copy = the first 1004 B of
           [key padded to 8][payload]; retired = [key 4][payload 0..999]

Also: the tool's result-file parser and the stage_probe_out records built from the oracle.
"""
import os
import struct
import subprocess

import numpy as np

import oracle_lib as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(REPO, "stage-indexorganized_amd", "lib", "adapter_drive")
PAYLOAD, ROW = 1000, 1008
PROBE_OUT = np.dtype([("status", "u1"), ("flags", "u1"), ("hops", "u2"), ("leaf", "u4"), ("slot", "u2"),
                      ("key_len", "u2"), ("cstamp", "u4"), ("rec_cstamp", "u4"), ("copy_sstamp", "u4"),
                      ("image", "u4"), ("meta_hi", "u4")])
IDENT = np.dtype([("loc", "u4"), ("next", "u4")])  # stage_probe_ident

# the scenario `adapter_drive probe` writes (tools/adapter_drive.cpp)
QUERIES = [(3, 0xFFFFFFFE), (3, 4), (3, 1), (3, 0), (5, 10), (5, 3), (9042, 5), (9042, 11), (9042, 13), (77, 100),
           (123456, 7), (4999, 1)]


def scenario_oracle():
    t = O.OracleTree()
    t.load_ycsb(0, 5000, 4, 0)
    assert t.update(3, 4, 0, bytes([7]) * 100, 1) == 1 and t.commit_update(3, 4, 2, 2) == 1
    assert t.update(3, 4, 0, bytes([9]) * 100, 5) == 1 and t.commit_update(3, 4, 6, 6) == 1
    assert t.update(5, 4, 0, bytes([55]) * 100, 8) == 1
    assert t.insert(9042, 4, bytes([0x42]) * PAYLOAD, 10) == 1
    assert t.update(9042, 4, 0, bytes([11]) * 100, 11) == 1 and t.commit_update(9042, 4, 12, 12) == 1
    return t


def hit_slot(t, key, ks, cache):
    """(leaf, slot, meta) of the first visible equal key in slot order (SearchRecordMeta)"""
    if "leaves" not in cache:
        cache["leaves"] = t.export_leaves(64)
    rc, sc, meta, keyw = cache["leaves"]
    leaf = t.traverse(key, ks, True)
    for s in range(int(rc[leaf])):
        m = int(meta[leaf, s])
        if m and (m >> 62) & 1 and int(keyw[leaf, s]) == key:
            return leaf, s, m
    return None


def oracle_probe_out(t, queries, ks=4):
    """stage_probe_out records + stage_probe_ident records + rows the C-ABI would return, from the
    oracle"""
    cache = {}
    outs = np.zeros(len(queries), PROBE_OUT)
    idents = np.zeros(len(queries), IDENT)
    rows = np.zeros((len(queries), ROW), np.uint8)
    for i, (k, rid) in enumerate(queries):
        o, rec, _, loc, nxt = t.read_ident(k, ks, rid)
        idents[i]["loc"], idents[i]["next"] = loc, nxt
        outs[i]["status"] = o["status"]
        outs[i]["flags"] = o["copy_present"]
        outs[i]["hops"] = o["hops"]
        outs[i]["cstamp"] = o["cstamp"]
        outs[i]["rec_cstamp"] = o["rec_cstamp"]
        outs[i]["copy_sstamp"] = o["copy_sstamp"]
        outs[i]["slot"] = 0xFFFF
        h = hit_slot(t, k, ks, cache)
        if h is not None and o["status"] != 0:
            outs[i]["leaf"], outs[i]["slot"] = h[0], h[1]
            outs[i]["meta_hi"] = h[2] >> 32
            outs[i]["key_len"] = (h[2] >> 48) & 0x2FFF
        rows[i, :t.row] = rec
    return outs, idents, rows


def expected(out, row, ident):
    """(ReturnCode, ResultType, perform_read, tuple, retired, via_copy, record bytes, 1004 tuple
    bytes).  The Record's RecordMetadata carries next_ptr = the next handle and loc_ptr = the
    location handle (the frame tool maps handles to themselves)."""
    st = int(out["status"])
    rc = 3 if st == 0 else 1
    result = 2 if st == 4 else 1
    perform = st in (1, 2)
    tup = st in (1, 2, 3)
    retired = st == 3
    meta_w = (int(out["meta_hi"]) << 32) | int(out["rec_cstamp"])
    inserting = (meta_w >> 62) & 1 and (meta_w >> 63) & 1
    via_copy = bool(st != 0 and inserting and (int(ident["next"]) & 0xC0000000) == 0x40000000)
    rec = b""
    if st in (1, 2):
        meta = (int(out["meta_hi"]) << 32) | int(out["rec_cstamp"])
        kl = (meta >> 48) & 0x2FFF
        kp = (kl + 7) // 8 * 8
        handle = int(ident["loc"])
        nxt = int(ident["next"])
        rec = struct.pack("<QQQIIQII", meta, nxt, handle, kp + PAYLOAD, 0, 0, int(out["cstamp"]), 0)
        rec += struct.pack("<I", int(out["cstamp"])) + bytes(row[:kp]) + bytes(row[max(kp, 8):max(kp, 8) + PAYLOAD])
    t = np.zeros(1004, np.uint8)
    if tup:
        t[:] = row[:1004] if not retired else np.concatenate([row[:4], row[8:1008]])
    return rc, result, perform, tup, retired, via_copy, rec, bytes(t)


def parse(path):
    b = open(path, "rb").read()
    n = struct.unpack_from("<Q", b, 0)[0]
    off, res = 8, []
    for _ in range(n):
        key, rid = struct.unpack_from("<QI", b, off)
        off += 12
        st, rc, result, perform, tup, retired, via_copy = b[off:off + 7]
        off += 7
        ln = struct.unpack_from("<H", b, off)[0]
        off += 2
        rec = b[off:off + ln]
        off += ln
        tb = b[off:off + 1004]
        off += 1004
        res.append((key, rid, st, rc, result, bool(perform), bool(tup), bool(retired), bool(via_copy), rec, tb))
    assert off == len(b)
    return res


def run_tool(*args):
    p = subprocess.run([TOOL] + list(args), capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
