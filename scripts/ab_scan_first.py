"""A/B of the first-tuple ORDER_LINE scans (stage_index_scan_first_batch, the stock-level scans)
on the bench's TPC-C ORDER_LINE table, for the kernel variant in STAGE_SL_SCANS (read when the
table is created), over two start-key batches of 2^22 scans of (w, d, o, 5), scan size 10,
prefix 3 words:
  hot     -- o among each district's last 20 orders (what stock-level asks: 3200 distinct keys
             at 16 warehouses),
  uniform -- o uniform over all 3000 orders.
Prints one JSON line: mean kernel milliseconds per launch (hipEvents) and the status counts."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stage-indexorganized_amd"))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import stage  # noqa: E402
from stage._lib import check  # noqa: E402

a = bench.parse(["--config", "tpcc"])
data = bench.tpcc_tables(a)
k, p = data["order_line"]
tab = stage.Table(payload_size=60, key_width=32)
tab.load_rows(k, p)
tab.sync()
n = 1 << 22
rng = np.random.default_rng(5)
w = rng.integers(1, a.warehouses + 1, n)
d = rng.integers(1, 11, n)
res = {"variant": os.environ.get("STAGE_SL_SCANS", "0"), "scans": n}
for name, o in (("hot", rng.integers(2981, 3001, n)), ("uniform", rng.integers(1, 3001, n))):
    keys = np.stack([w, d, o, np.full(n, 5)], 1).astype(np.int64).view(np.uint64)
    dk = stage.DeviceBuffer.from_numpy(np.ascontiguousarray(keys))
    di = stage.DeviceBuffer(n * 4)
    ds = stage.DeviceBuffer(n)
    s = stage.Stream()
    ms = []
    for it in range(6):
        e0, e1 = stage.Event(), stage.Event()
        e0.record(s)
        check(stage.lib().stage_index_scan_first_batch(tab.h, dk.ptr, None, n, 10, 3, di.ptr, ds.ptr, s.ptr), "scan")
        e1.record(s)
        s.sync()
        if it:
            ms.append(e0.elapsed_ms(e1))
    st = ds.to_numpy(np.uint8, n)
    res[name] = {"ms": round(float(np.mean(ms)), 4), "scans_per_s": round(n / (np.mean(ms) * 1e-3), 1),
                 "status_counts": {int(v): int(c) for v, c in zip(*np.unique(st, return_counts=True))}}
print(json.dumps(res), flush=True)
