"""CH-benCHmark tables for Q2 with the reference's key and payload layouts (tpcc_record.h:160-200
ITEM, 417-500 STOCK, 773-880 REGION / NATION / SUPPLIER; payload columns in GetData order) and
the loader's value rules (tpcc_loader.cpp: BuildRegionTuple / BuildNationTuple /
BuildSupplierTuple / BuildItemTuple / BuildStockTuple, :949-1017, :1330-1372; keys from 0,
stock {w, i} with w < W, i < I; GetRandomAlphaNumericString(n) = n copies of ONE character
drawn from the 62 alphanumerics and the terminating NUL, :849-860), plus the driver's
supplier -> stocks map (tpcc_workload.cpp:398-404) as CSR.  Loaded identically into the
product and, optionally, the oracle."""
import numpy as np

import stage

R_PAYLOAD = 55 + 152                       # Region::GetPayloadSize
N_PAYLOAD = 8 + 25 + 152                   # Nation::GetPayloadSize
SU_PAYLOAD = 8 + 8 + 25 + 40 + 15 + 15     # Supplier::GetPayloadSize
I_PAYLOAD = 4 + 32 + 8 + 64                # Item::GetPayloadSize
S_PAYLOAD = 4 * 4 + 10 * 32 + 64           # Stock::GetPayloadSize
REGIONS = ["AFRICA", "AMERICA", "ASIA", "EUROPE", "MIDDLE EAST"]
# N_REGIONKEY of nations[0..61] (tpcc_record.h:869-930), the table's rows are keyed 0..61
NATION_REGION = [0, 1, 1, 1, 4, 0, 3, 3, 2, 2, 4, 4, 2, 4, 0, 0, 0, 1, 2, 3, 4, 2, 3, 3, 1, 2, 2, 2, 1, 2, 2,
                 3, 0, 2, 1, 3, 3, 3, 0, 2, 2, 1, 2, 2, 2, 2, 0, 0, 4, 0, 0, 2, 3, 3, 2, 3, 3, 3, 4, 3, 2, 3]
ALNUM = np.frombuffer(b"0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz\0", np.uint8)


def rep_string(rng, n, length, width):
    """n GetRandomAlphaNumericString(length) results strncpy'd into char[width] fields."""
    c = ALNUM[rng.integers(0, ALNUM.size, n)]
    out = np.zeros((n, width), np.uint8)
    out[:, :min(length, width)] = c[:, None]
    return out


def text(s, width):
    b = np.zeros(width, np.uint8)
    raw = s.encode()[:width]
    b[:len(raw)] = np.frombuffer(raw, np.uint8)
    return b


def supp_stock_map(W, I):
    """CSR of supp_stock_map[w * i % 10000] += (w - 1, i - 1), w in 1..W outer, i in 1..I."""
    w = np.repeat(np.arange(1, W + 1, dtype=np.int64), I)
    i = np.tile(np.arange(1, I + 1, dtype=np.int64), W)
    supp = (w * i) % 10000
    order = np.argsort(supp, kind="stable")
    off = np.zeros(10001, np.uint32)
    np.cumsum(np.bincount(supp, minlength=10000), out=off[1:])
    return off, (w - 1)[order].astype(np.int32), (i - 1)[order].astype(np.int32)


class ChTables:
    def __init__(self, W=2, I=1000, seed=11, qty=(10, 100), oracle=True):
        rng = np.random.default_rng(seed)
        self.W, self.I = W, I
        if len(NATION_REGION) != 62:
            raise AssertionError("nations[] has 62 entries")
        rows = {}
        k = np.arange(5, dtype=np.int64)
        p = np.zeros((5, R_PAYLOAD), np.uint8)
        for r in range(5):
            p[r, :55] = text(REGIONS[r], 55)
        p[:, 55:] = rep_string(rng, 5, 64, 152)
        rows["region"] = (k, p)
        k = np.arange(62, dtype=np.int64)
        p = np.zeros((62, N_PAYLOAD), np.uint8)
        p[:, :8] = np.array(NATION_REGION, np.int64).view(np.uint8).reshape(62, 8)
        p[:, 33:] = rep_string(rng, 62, 64, 152)
        rows["nation"] = (k, p)
        k = np.arange(10000, dtype=np.int64)
        p = rng.integers(0, 256, (10000, SU_PAYLOAD), dtype=np.uint8)
        p[:, :8] = rng.integers(0, 62, 10000).astype(np.int64).view(np.uint8).reshape(-1, 8)  # SU_NATIONKEY
        rows["supplier"] = (k, p)
        k = np.arange(I, dtype=np.int64)
        p = np.zeros((I, I_PAYLOAD), np.uint8)
        p[:, :4] = (k * 10).astype(np.int32).view(np.uint8).reshape(-1, 4)  # I_IM_ID
        p[:, 4:36] = rep_string(rng, I, 24, 32)
        p[:, 36:44] = rng.integers(0x30, 0x3A, (I, 8), dtype=np.uint8)
        p[:, 44:] = rep_string(rng, I, 64, 64)  # I_DATA
        rows["item"] = (k, p)
        wi = np.stack(np.meshgrid(np.arange(W), np.arange(I), indexing="ij"), -1).reshape(-1, 2).astype(np.int64)
        p = rng.integers(0, 256, (W * I, S_PAYLOAD), dtype=np.uint8)
        p[:, :16] = 0  # S_YTD, S_ORDER_CNT, S_REMOTE_CNT = 0
        p[:, :4] = rng.integers(qty[0], qty[1] + 1, W * I).astype(np.int32).view(np.uint8).reshape(-1, 4)
        rows["stock"] = (wi, p)
        self.rows = rows
        self.tables, self.orc = {}, {}
        import oracle_lib as O
        for name, (keys, pays) in rows.items():
            width = 16 if name == "stock" else 8
            kb = np.ascontiguousarray(keys).view(np.uint8).reshape(-1, width)
            t = stage.Table(payload_size=pays.shape[1], key_width=width)
            _, ins = t.load_rows(kb, pays)
            assert ins == kb.shape[0]
            self.tables[name] = t
            if oracle:
                o = O.OracleTree(payload_size=pays.shape[1], key_pad=width)
                assert o.load_rows(kb, pays) == kb.shape[0]
                self.orc[name] = o
        self.map_off, self.map_w, self.map_i = supp_stock_map(W, I)
        self.d_map = None

    def sync(self):
        for t in self.tables.values():
            t.sync()
        keys = np.stack([self.map_w.astype(np.int64), self.map_i.astype(np.int64)], 1).astype(np.uint64)
        self.d_map = stage.DeviceBuffer.from_numpy(np.ascontiguousarray(keys))

    def query2(self, target=3, read_id=0xFFFFFFFE, commit_id=0):
        t = self.tables
        if getattr(self, "_out", None) is None:
            self._out = np.zeros(1 << 14, stage.Q2_REC_DTYPE)
            self._map_off = np.ascontiguousarray(self.map_off, np.uint32)
        recs, ab = stage.ch_query2(t["region"], t["nation"], t["supplier"], t["item"], t["stock"], self._map_off,
                                   self.d_map.ptr, target, read_id, commit_id, out=self._out)
        return recs.copy(), ab

    def query2_batch(self, read_ids, target=3, out=None, stream=None):
        t = self.tables
        return stage.ch_query2_batch(t["region"], t["nation"], t["supplier"], t["item"], t["stock"], self.map_off,
                                     self.d_map.ptr, read_ids, target, out=out, stream=stream)

    def query2_batch_async(self, read_ids, out, slot=0, target=3, stream=None):
        t = self.tables
        return stage.ch_query2_batch_async(t["region"], t["nation"], t["supplier"], t["item"], t["stock"],
                                           self.map_off, self.d_map.ptr, read_ids, out, slot, target, stream=stream)

    def query2_oracle(self, target=3, read_id=0xFFFFFFFE):
        import ctypes

        import oracle_lib as O
        o = self.orc
        out = np.zeros(1 << 16, stage.Q2_REC_DTYPE)
        ab = ctypes.c_int()
        n = O.lib().orc_ch_query2(o["region"].t, o["nation"].t, o["supplier"].t, o["item"].t, o["stock"].t,
                                  self.map_off.ctypes.data, self.map_w.ctypes.data, self.map_i.ctypes.data, target,
                                  read_id, out.ctypes.data, out.size, ctypes.byref(ab))
        return out[:n], bool(ab.value)
