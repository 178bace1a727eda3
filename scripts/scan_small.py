"""Device time of one small TableScan (CH-Q2's NATION scan of 65 and REGION scan of 6) by scan
size and row tuning: where a single-wave scan's time goes.  Same tables as `bench.py --config
chq2`."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stage-indexorganized_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402

import stage  # noqa: E402
from ch_data import ChTables  # noqa: E402

ch = ChTables(W=2, I=1000, seed=11, oracle=False)
ch.sync()
L = stage.lib()
s = stage.Stream()
for name in ("nation", "region", "supplier"):
    t = ch.tables[name]
    d_key = stage.DeviceBuffer.from_numpy(np.zeros(1, np.uint64))
    d_cnt = stage.DeviceBuffer(4)
    for size in (6, 30, 62, 63, 64, 65, 128):
        d_rec = stage.DeviceBuffer(size * t.stride)
        for _ in range(20):
            L.stage_scan_batch(t.h, d_key.ptr, None, 1, size, d_cnt.ptr, d_rec.ptr, s.ptr)
        e0, e1 = stage.Event(), stage.Event()
        reps = 200
        e0.record(s)
        for _ in range(reps):
            L.stage_scan_batch(t.h, d_key.ptr, None, 1, size, d_cnt.ptr, d_rec.ptr, s.ptr)
        e1.record(s)
        s.sync()
        cnt = d_cnt.to_numpy(np.uint32, 1)[0]
        print(f"{name:8s} stride {t.stride:4d} scan {size:4d}: {e0.elapsed_ms(e1) / reps * 1e3:7.1f} us per scan "
              f"({cnt} rows)", flush=True)
