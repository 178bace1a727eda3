import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "stage-indexorganized_amd"))
import numpy as np
import oracle_lib as O
import stage
tab = stage.Table(key_width=4)
tab.load_ycsb(0, 1000000, 4, mode=0)
tab.sync()
orc = O.OracleTree()
orc.load_ycsb(0, 1000000, 4, 0)
rng = np.random.default_rng(5)
starts = np.concatenate([rng.integers(0, 1000000, 300), np.array([0, 999900, 999999, 1000000, 1 << 31])]).astype(np.uint64)
for size in (100, 1000, 1000):
    counts, rows = tab.range_scan(starts, size)
    oc, orows = orc.scan_batch(starts, 4, size)
    nbad = 0
    for i in range(starts.size):
        c = oc[i]
        bad = np.nonzero((rows[i, :c, :1008] != orows[i, :c]).any(axis=1))[0]
        nbad += bad.size > 0
    print("size", size, "scans with bad rows", nbad, "count mismatches", int((counts != oc).sum()))
    for i in range(starts.size):
        c = oc[i]
        bad = np.nonzero((rows[i, :c, :1008] != orows[i, :c]).any(axis=1))[0]
        pk = rows[i, :c, :4].copy().view(np.uint32).ravel()
        ok_ = orows[i, :c, :4].copy().view(np.uint32).ravel()
        if bad.size:
            print("start", starts[i], "count", counts[i], c, "bad rows", bad.size, bad[:10])
            j = bad[0]
            print(" prod keys", pk[max(0, j-3):j+5])
            print(" orc  keys", ok_[max(0, j-3):j+5])
            print(" prod row bytes", rows[i, j, :16], rows[i, j, 1000:1010])
            print(" orc  row bytes", orows[i, j, :16], orows[i, j, 1000:1008])
            break
