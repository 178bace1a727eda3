"""Tuning sweep for probe_kernel on one GPU: one table, several launch shapes, interleaved
rounds in one process (cdna_hip_programming.md §5.4 rule 24).  Prints one JSON line per shape."""
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
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--theta", type=float, default=0.9)
ap.add_argument("--shapes", default="4:4096,1:4096,2:4096,8:4096,4:1024,4:2048,4:8192,8:8192")
args = ap.parse_args()

tab = stage.Table(key_width=8)
tab.load_ycsb(0, args.rows, 8, 0)
tab.sync()
keys = stage.zipf_draws(args.rows - 1, args.theta, 0x5EED, args.batch, nthreads=16)
s = stage.Stream()
dk = stage.DeviceBuffer.from_numpy(keys)
do = stage.DeviceBuffer(args.batch * 32)
dr = stage.DeviceBuffer(args.batch * tab.stride)
shapes = [tuple(int(v) for v in x.split(":")) for x in args.shapes.split(",")]
res = {sh: [] for sh in shapes}
e0, e1 = stage.Event(), stage.Event()
for r in range(args.rounds):
    for sh in shapes:
        check(stage.lib().stage_set_probe_tuning(tab.h, sh[0], sh[1]), "tune")
        tab.probe_device(dk.ptr, args.batch, do.ptr, dr.ptr, stream=s.ptr)
        e0.record(s)
        tab.probe_device(dk.ptr, args.batch, do.ptr, dr.ptr, stream=s.ptr)
        e1.record(s)
        s.sync()
        res[sh].append(e0.elapsed_ms(e1))
for sh in shapes:
    ms = np.array(res[sh])
    print(json.dumps({"group": sh[0], "max_blocks": sh[1], "median_ms": float(np.median(ms)),
                      "min_ms": float(ms.min()), "glookups_s": args.batch / np.median(ms) / 1e6,
                      "frac_2100B": 2100 * args.batch / (np.median(ms) * 1e-3) / 8e12}))
