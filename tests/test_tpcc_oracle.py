"""CPU: the oracle's C TPC-C stock-level (orc_stock_level, the CPU baseline of the TPC-C
measurement) equals the transaction composed from the oracle's primitives in Python
(tests/tpcc_data.py: point read, IndexScanExecutor range scan, point read), with history and
in-flight updates, read ids before, between and after commits, and aborts."""
import numpy as np

import oracle_lib as O
from tpcc_data import TpccTables, key


def test_c_stock_level_equals_composed():
    tt = TpccTables(n_o=30, n_items=500)
    rng = np.random.default_rng(3)
    for cid in (10, 20):
        for i in rng.choice(500, 150, replace=False) + 1:
            tt.update("stock", key(1, int(i)), 0, np.int32(rng.integers(1, 40)).tobytes(), cid, cid + 1)
        for o in range(10, 31):
            tt.update("ol", key(2, 4, o, 5), 8, np.int64(cid).tobytes(), cid, cid + 1)
    tt.update("dist", key(1, 2), 0, np.int32(26).tobytes(), 30)
    n = 300
    w = rng.integers(1, 4, n)  # warehouse 3 does not exist -> abort
    d = rng.integers(1, 11, n)
    thr = rng.integers(10, 21, n)
    rids = rng.choice(np.array([0, 11, 15, 21, 31, 0xFFFFFFFE], np.uint32), n)
    res, _ = O.stock_level_batch(tt.odist, tt.ool, tt.ostock, w, d, thr, rids, nthreads=4)
    exp = np.array([tt.stock_level_oracle(int(a), int(b), int(c), int(r)) for a, b, c, r in zip(w, d, thr, rids)])
    assert (res == exp).all()
    assert (res[w == 3] == -1).all() and (res > 0).any()
