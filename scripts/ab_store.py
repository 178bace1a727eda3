"""A/B of the probe's output store policy (stage_set_probe_store) on the bench workload: one
100M-row table, interleaved rounds in one process, each policy's launch timed with events.
Checks that every policy writes identical outputs.  Prints one JSON line per policy."""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stage-indexorganized_amd"))
import stage  # noqa: E402
from stage._lib import check  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=100_000_000)
ap.add_argument("--batch", type=int, default=1 << 24)
ap.add_argument("--rounds", type=int, default=6)
ap.add_argument("--theta", type=float, default=0.9)
ap.add_argument("--policies", default="1,2,0")
args = ap.parse_args()

tab = stage.Table(key_width=8)
tab.load_ycsb(0, args.rows, 8, 0)
tab.sync()
keys = stage.zipf_draws(args.rows - 1, args.theta, 0x5EED, args.batch, nthreads=16)
s = stage.Stream()
dk = stage.DeviceBuffer.from_numpy(keys)
do = stage.DeviceBuffer(args.batch * 32)
dr = stage.DeviceBuffer(args.batch * tab.stride)
pols = [int(p) for p in args.policies.split(",")]
res = {p: [] for p in pols}
digest = {}
e0, e1 = stage.Event(), stage.Event()
for r in range(args.rounds):
    for p in pols:
        check(stage.lib().stage_set_probe_store(tab.h, p), "store policy")
        tab.probe_device(dk.ptr, args.batch, do.ptr, dr.ptr, stream=s.ptr)
        e0.record(s)
        tab.probe_device(dk.ptr, args.batch, do.ptr, dr.ptr, stream=s.ptr)
        e1.record(s)
        s.sync()
        res[p].append(e0.elapsed_ms(e1))
        if r == 0:
            n = 1 << 20
            digest[p] = (do.to_numpy(np.uint8, n * 32).tobytes(), dr.to_numpy(np.uint8, n * tab.stride).tobytes())
same = all(digest[p] == digest[pols[0]] for p in pols)
for p in pols:
    ms = np.array(res[p])
    print(json.dumps({"store": p, "median_ms": float(np.median(ms)), "min_ms": float(ms.min()),
                      "glookups_s": args.batch / np.median(ms) / 1e6,
                      "frac_2100B": 2100 * args.batch / (np.median(ms) * 1e-3) / 8e12, "outputs_identical": same}),
          flush=True)
