"""The HBM side of one rank's sharded step at W ranks, on one GPU: W shard tables of
ROWS / W rows each (the keys MurmurHash64A(key, 8, 0) % W == r of 0..ROWS-1, as bench.py
loads a shard), and W callers of BATCH / W Zipf-0.9 lookups each over all ROWS keys, run through
stage_probe_sharded_loopback -- the same plan as the RCCL path with device copies for the
transfers.  One loopback step does the HBM work all W ranks do (probes, fan-out probes of own
requests, result copies, fan-out of returned results) for BATCH lookups in total, i.e. what ONE
rank does per step at W ranks for its BATCH lookups (trees of ROWS / W rows instead of ROWS;
no xGMI).  Prints one JSON line: step ms (hipEvents), full reply (rows copied back), peer reply
(rows read from the owners' buffers), direct reply (rows written by the owners into the callers'
outputs, duplicates copied by the caller) and owner reply, and the request counts.  Env: ROWS (100M), W (8), BATCH (2^24), STEPS (5), CHUNKS (4)."""
import ctypes
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

rows = int(os.environ.get("ROWS", 100_000_000))
W = int(os.environ.get("W", 8))
batch = int(os.environ.get("BATCH", 1 << 24))
steps = int(os.environ.get("STEPS", 5))
chunks = int(os.environ.get("CHUNKS", 4))
L = stage.lib()
tabs = []
for r in range(W):
    t = stage.Table(key_width=8)
    t.load_keys(bench.owned_keys(rows, W, r), 8, mode=0)
    t.sync()
    check(L.stage_set_shard_chunks(t.h, chunks), "chunks")
    tabs.append(t)
per = batch // W
bufs = []
for r in range(W):
    k = stage.zipf_draws(rows - 1, 0.9, 0x5EED + r, per, nthreads=16)
    bufs.append((stage.DeviceBuffer.from_numpy(k), stage.DeviceBuffer(per * 32), stage.DeviceBuffer(per * tabs[0].stride)))
arr = lambda v: (ctypes.c_void_p * W)(*v)
hs = (ctypes.c_void_p * W)(*[t.h for t in tabs])
n_arr = (ctypes.c_uint64 * W)(*([per] * W))
s = stage.Stream()
res = {"rows": rows, "world": W, "batch_total": batch, "chunks": chunks, "steps": steps}
modes = (("full_reply", stage.REPLY_ROWS), ("peer_reply", stage.REPLY_PEER), ("direct_reply", stage.REPLY_DIRECT),
         ("owner_reply", stage.REPLY_OWNER))
only = os.environ.get("MODES")  # e.g. MODES=peer_reply
for name, reply in [m for m in modes if not only or m[0] in only.split(",")]:
    ms = []
    for it in range(steps + 1):
        e0, e1 = stage.Event(), stage.Event()
        e0.record(s)
        check(L.stage_probe_sharded_loopback(hs, W, arr([b[0].ptr for b in bufs]), None, n_arr,
                                             arr([b[1].ptr for b in bufs]),
                                             arr([b[2].ptr for b in bufs]), reply, s.ptr), "loopback")
        e1.record(s)
        s.sync()
        if it:
            ms.append(e0.elapsed_ms(e1))
    res[name] = {"ms": round(float(np.mean(ms)), 3), "min_ms": round(float(np.min(ms)), 3)}
st = [stage.sharded_stats(t, True) for t in tabs]
res["requests"] = {"keys": int(sum(x[0] for x in st)), "routed": int(sum(x[1] for x in st)),
                   "remote": int(sum(x[2] for x in st))}
print(json.dumps(res), flush=True)
