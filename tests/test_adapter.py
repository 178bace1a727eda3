"""CPU: the reference-side adapter (include/stage_btree_adapter.hpp, compiled into
stage-indexorganized_amd/lib/adapter_drive) frames stage_probe_out results exactly as the
reference's Record (b_tree.h:400-448), IndexScanExecutor outcome (executor.h:374-454) and
YCSBTupleInt copy (executor.h:396-401, 424) would be: the C++ adapter's bytes equal an
independent Python statement of those definitions, on probe records built from the oracle for
every status (latest, copy, old, INVALID-begin failure, chain miss, not found).
The same check on real device results is tests/test_gpu_adapter.py."""
import os
import struct

import numpy as np

import adapter_expect as A


def test_adapter_frames_oracle_results(tmp_path):
    t = A.scenario_oracle()
    outs, idents, rows = A.oracle_probe_out(t, A.QUERIES)
    assert set(outs["status"].tolist()) == {0, 1, 2, 3, 4, 5}
    keys = np.array([q[0] for q in A.QUERIES], np.uint64)
    rids = np.array([q[1] for q in A.QUERIES], np.uint32)
    src = tmp_path / "in.bin"
    with open(src, "wb") as f:
        f.write(struct.pack("<Q", keys.size) + keys.tobytes() + rids.tobytes() + outs.tobytes() + idents.tobytes() +
                rows.tobytes())
    dst = tmp_path / "out.bin"
    A.run_tool("frame", str(src), str(dst))
    got = A.parse(str(dst))
    assert len(got) == len(A.QUERIES)
    for i, g in enumerate(got):
        exp = A.expected(outs[i], rows[i], idents[i])
        assert g[0] == keys[i] and g[1] == rids[i] and g[2] == outs[i]["status"]
        assert g[3:] == exp, (i, A.QUERIES[i], g[3:9], exp[:6])
    # the reference framing quirks on this scenario: key 3 at read id 4 is the retired version
    # holding the first update's 100 bytes of 7, in the retired framing [key 4][payload]
    old = got[1]
    assert old[2] == 3 and old[10][:4] == (3).to_bytes(4, "little") and old[10][4:104] == bytes([7]) * 100
    latest = got[0]
    assert latest[10][4:8] == bytes(4) and latest[10][8:108] == bytes([9]) * 100  # [key 4][pad 4][payload]
    assert len(latest[9]) == 48 + 4 + 8 + 1000
    # the in-flight key 5 is read from its overwrite copy: the Record's next_ptr names the copy
    # (STAGE_NEXT_COPY | copy id) and BTree::Read registers the reader (via_copy); loc_ptr is the
    # record's RecordLocation handle, not a (leaf, slot)
    copy_read = got[4]
    assert copy_read[2] == 2 and copy_read[8]
    assert struct.unpack_from("<Q", copy_read[9], 8)[0] & 0xC0000000 == 0x40000000
    assert struct.unpack_from("<Q", copy_read[9], 16)[0] == idents[4]["loc"] != 0


def test_adapter_tool_is_built():
    assert os.access(A.TOOL, os.X_OK)
