"""CPU: the oracle's C CH-benCHmark Q2 (orc_ch_query2, the checker and CPU baseline of the Q2
measurement) equals RunQuery2 (benchmark/tpcc/tpcc_new_order.cpp:608-982) composed in Python
from the oracle's primitives -- REGION / NATION TableScans, the SUPPLIER leaves in ScanLeafNode
order (exported slot arrays), STOCK / ITEM point reads with visibility -- record for record and
in visiting order, including the kept-last-stock quirk, the I_DATA test and aborts."""
import numpy as np

import oracle_lib as O
from ch_data import REGIONS, ChTables


def composed_q2(ch, target, rid):
    o = ch.orc
    zero = np.zeros(1, np.uint64)
    rc, rr = o["region"].scan_batch(zero, 8, 6)
    nc, nn = o["nation"].scan_batch(zero, 8, 65)
    sup = []
    rcount, _, meta, keyw = o["supplier"].export_leaves(512)
    for leaf in range(rcount.size):
        for s in range(rcount[leaf]):
            if meta[leaf, s]:
                out, rec = o["supplier"].read(int(keyw[leaf, s]), 8, rid)
                sup.append((int(keyw[leaf, s]), int(rec[8:16].view(np.int64)[0])))
    recs = []
    for r in rr[0, :rc[0]]:
        if bytes(r[8:63]).split(b"\0")[0].decode() != REGIONS[target]:
            continue
        rkey = int(r[:8].view(np.int64)[0])
        for nrow in nn[0, :nc[0]]:
            if int(nrow[8:16].view(np.int64)[0]) != rkey:
                continue
            nkey = int(nrow[:8].view(np.int64)[0])
            for sk, nat in sup:
                if nat != nkey:
                    continue
                w0 = i0 = 0
                q = [0, 0, 0, 0]
                for e in range(ch.map_off[sk], ch.map_off[sk + 1]):
                    k = np.array([ch.map_w[e], ch.map_i[e]], np.int64).tobytes()
                    out, rec = o["stock"].read(k, 16, rid)
                    if int(np.ravel(out["status"])[0]) not in (1, 2, 3):
                        return recs, True
                    w0, i0 = (int(x) for x in rec[:16].view(np.int64))
                    q = [int(x) for x in rec[16:32].view(np.int32)]
                out, rec = o["item"].read(i0, 8, rid)
                if int(np.ravel(out["status"])[0]) not in (1, 2, 3):
                    return recs, True
                idata = bytes(rec[8 + 44:8 + 108]).split(b"\0")[0]
                has_b = b"b" in idata
                recs.append((sk, w0, i0, q[0], q[1], q[2], q[3], int(has_b), int(not has_b and q[0] < 10)))
    return recs, False


def test_c_query2_equals_composed():
    ch = ChTables(W=2, I=3000, qty=(1, 100), seed=5)
    ostock = ch.orc["stock"]
    for i in range(0, 3000, 7):  # history: committed updates (20 -> 21), some left in flight (30)
        k = np.array([i % 2, i], np.int64).tobytes()
        if ostock.update(k, 16, 0, np.int32(i % 13).tobytes(), 20) == 1:
            ostock.commit_update(k, 16, 21, 21)
    for i in range(3, 3000, 97):
        ostock.update(np.array([1, i], np.int64).tobytes(), 16, 4, b"\x07\x00\x00\x00", 30)
    fields = ["supp_key", "s_w_id", "s_i_id", "s_quantity", "s_ytd", "s_order_cnt", "s_remote_cnt", "item_has_b",
              "update"]
    seen_abort = seen_ok = False
    for target in range(5):
        for rid in (10, 25, 0xFFFFFFFE):
            recs, ab = ch.query2_oracle(target, rid)
            exp, eab = composed_q2(ch, target, rid)
            assert ab == eab, (target, rid)
            if not ab:
                got = [tuple(int(r[f]) for f in fields) for r in recs]
                assert got == exp, (target, rid)
                seen_ok = True
            seen_abort |= ab
    assert seen_ok and seen_abort
