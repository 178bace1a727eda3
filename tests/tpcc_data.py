"""Small TPC-C DISTRICT / ORDER_LINE / STOCK tables with the reference's key and payload layouts
(tpcc_record.h: keys are int64 fields, payload columns in GetData order), loaded identically
into the product and the oracle, plus the oracle-composed stock-level transaction
(tpcc_stock_level.cpp:37-180) used as the checker."""
import numpy as np

import oracle_lib as O
import stage

D_PAYLOAD = 4 + 16 + 32 + 32 + 32 + 2 + 9 + 8 + 8          # District::GetPayloadSize = 143
OL_PAYLOAD = 4 + 4 + 8 + 4 + 8 + 32                       # OrderLine::GetPayloadSize = 60
S_PAYLOAD = 4 * 4 + 10 * 32 + 64                          # Stock::GetPayloadSize = 400


def key(*fields):
    return np.array(fields, dtype=np.int64).tobytes()


def i32(b):
    return int(np.frombuffer(bytes(b[:4]), np.int32)[0])


def i64(b):
    return int(np.frombuffer(bytes(b[:8]), np.int64)[0])


class TpccTables:
    """key_order: load each batch sorted by its key bytes (the tables' memcmp order) instead of
    the loader's numeric order -- every leaf's keys then increase in slot order."""

    def __init__(self, n_w=2, n_d=10, n_o=40, n_items=1000, seed=7, key_order=False):
        rng = np.random.default_rng(seed)
        self.key_order = key_order
        self.n_w, self.n_d, self.n_o, self.n_items = n_w, n_d, n_o, n_items
        self.dist = stage.Table(payload_size=D_PAYLOAD, key_width=16)
        self.ol = stage.Table(payload_size=OL_PAYLOAD, key_width=32)
        self.stock = stage.Table(payload_size=S_PAYLOAD, key_width=16)
        self.odist = O.OracleTree(payload_size=D_PAYLOAD, key_pad=16)
        self.ool = O.OracleTree(payload_size=OL_PAYLOAD, key_pad=32)
        self.ostock = O.OracleTree(payload_size=S_PAYLOAD, key_pad=16)
        for w in range(1, n_w + 1):  # loader order: stock, districts, orders/order lines
            keys, pays = [], []
            for i in range(1, n_items + 1):
                p = rng.integers(0, 256, S_PAYLOAD, dtype=np.uint8)
                p[:4] = np.frombuffer(np.int32(rng.integers(10, 101)).tobytes(), np.uint8)  # S_QUANTITY
                keys.append(np.frombuffer(key(w, i), np.uint8))
                pays.append(p)
            self._load(self.stock, self.ostock, 16, keys, pays)
            keys, pays = [], []
            for d in range(1, n_d + 1):
                p = rng.integers(0, 256, D_PAYLOAD, dtype=np.uint8)
                p[:4] = np.frombuffer(np.int32(n_o + 1).tobytes(), np.uint8)  # D_NEXT_O_ID
                keys.append(np.frombuffer(key(w, d), np.uint8))
                pays.append(p)
            self._load(self.dist, self.odist, 16, keys, pays)
            keys, pays = [], []
            for d in range(1, n_d + 1):
                for o in range(1, n_o + 1):
                    for ln in range(1, int(rng.integers(5, 16)) + 1):
                        p = rng.integers(0, 256, OL_PAYLOAD, dtype=np.uint8)
                        p[:4] = np.frombuffer(np.int32(rng.integers(1, n_items + 1)).tobytes(), np.uint8)  # OL_I_ID
                        keys.append(np.frombuffer(key(w, d, o, ln), np.uint8))
                        pays.append(p)
            self._load(self.ol, self.ool, 32, keys, pays)

    def _load(self, tab, orc, width, keys, pays):
        keys = np.stack(keys)
        pays = np.stack(pays)
        if self.key_order:
            order = np.lexsort(keys.T[::-1])
            keys, pays = keys[order], pays[order]
        rc, ins = tab.load_rows(keys, pays)
        assert ins == keys.shape[0]
        assert orc.load_rows(keys, pays) == keys.shape[0]

    def update(self, which, k, off, delta, writer, commit=None):
        tab, orc, width = {"dist": (self.dist, self.odist, 16), "ol": (self.ol, self.ool, 32),
                           "stock": (self.stock, self.ostock, 16)}[which]
        a = tab.update_key(k, off, delta, writer)
        assert a == orc.update(k, width, off, delta, writer)
        if commit is not None and a == stage.RC_OK:
            assert tab.commit_update_key(k, commit, commit) == orc.commit_update(k, width, commit, commit)
        return a

    def sync(self):
        for t in (self.dist, self.ol, self.stock):
            t.sync()

    def stock_level_oracle(self, w, d, threshold, rid=0xFFFFFFFE):
        out, rec = self.odist.read(key(w, d), 16, rid)
        if out["status"] not in (1, 2, 3):
            return -1
        nxt = i32(rec[16:20])
        items = set()
        for o in range(nxt - 20, nxt):
            c, rows, st = self.ool.index_scan(key(w, d, o, 5), 32, 10, rid)
            ids = [i32(rows[j][32:36]) for j in range(c)
                   if st[j] in (1, 3) and i64(rows[j][16:24]) == o and i64(rows[j][0:8]) == w
                   and i64(rows[j][8:16]) == d]
            if not ids:
                continue
            sout, srec = self.ostock.read(key(w, ids[0]), 16, rid)
            if sout["status"] == 4:
                return -1
            if sout["status"] not in (1, 2, 3):
                continue
            if i32(srec[16:20]) < threshold:
                items.add(int(np.int64(i64(srec[8:16])).astype(np.int32)))
        return len(items)


def stock_level_device(tt, w, d, thr, rids=None):
    n = len(w)
    bufs = [stage.DeviceBuffer.from_numpy(np.asarray(w, np.int64)), stage.DeviceBuffer.from_numpy(np.asarray(d, np.int64)),
            stage.DeviceBuffer.from_numpy(np.asarray(thr, np.int32))]
    d_rid = stage.DeviceBuffer.from_numpy(np.asarray(rids, np.uint32)) if rids is not None else None
    d_res = stage.DeviceBuffer(4 * n)
    from stage._lib import check
    check(stage.lib().stage_tpcc_stock_level(tt.dist.h, tt.ol.h, tt.stock.h, bufs[0].ptr, bufs[1].ptr, bufs[2].ptr,
                                             d_rid.ptr if d_rid else None, n, d_res.ptr, None), "stock level")
    check(stage.lib().stage_device_sync(), "sync")
    return d_res.to_numpy(np.int32, n)
