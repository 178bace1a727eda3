"""Where a batched CH-Q2 step's wall time goes: the Python wrapper vs the C++ call (whose own
phases STAGE_Q2_TRACE=1 prints).  Same tables as `bench.py --config chq2`."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stage-indexorganized_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

import bench  # noqa: E402
import stage  # noqa: E402
from ch_data import ChTables  # noqa: E402

args = bench.parse(["--config", "chq2", "--no-cpu-baseline"])
ch = ChTables(W=args.warehouses, I=args.items, seed=args.seed & 0xFFFF, oracle=False)
ch.sync()
nq = args.q2_batch
rids = (0xFFFFFFFE - np.arange(nq)).astype(np.uint32)
out = (stage.pinned_empty if os.environ.get("Q2_PINNED", "1") == "1" else np.zeros)((nq, 1 << 14), stage.Q2_REC_DTYPE)
for _ in range(5):
    ch.query2_batch(rids, 3, out=out)
t = ch.tables
L = stage.lib()
import ctypes  # noqa: E402
map_off = np.ascontiguousarray(ch.map_off, np.uint32)
ab = np.zeros(nq, np.int32)
n = ctypes.c_uint64()
reps = 50
t0 = time.perf_counter()
for _ in range(reps):
    ch.query2_batch(rids, 3, out=out)
wrap = (time.perf_counter() - t0) / reps
t0 = time.perf_counter()
for _ in range(reps):
    L.stage_ch_query2_batch(t["region"].h, t["nation"].h, t["supplier"].h, t["item"].h, t["stock"].h,
                            map_off.ctypes.data, ch.d_map.ptr, 3, rids.ctypes.data, nq, out.ctypes.data,
                            out.shape[1], ctypes.byref(n), ab.ctypes.data, None)
raw = (time.perf_counter() - t0) / reps
print(f"q2 batch of {nq}: wrapper {wrap * 1e6:.1f} us, raw ctypes call {raw * 1e6:.1f} us, suppliers {n.value}")
