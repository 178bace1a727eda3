"""A/B of the probe across builds: each --pkg is a package directory (holding stage/ and
lib/libstage_hip.so, e.g. a copy of an older commit's build); the bench workload (100M rows,
2^24 Zipf-0.9 lookups) is timed with events, one process per package, so each run gets its
own table.  Prints one JSON line with the median launch time and an output digest."""
import argparse
import hashlib
import json
import os
import sys

import numpy as np

ap = argparse.ArgumentParser()
ap.add_argument("--pkg", required=True)
ap.add_argument("--rows", type=int, default=100_000_000)
ap.add_argument("--batch", type=int, default=1 << 24)
ap.add_argument("--rounds", type=int, default=10)
ap.add_argument("--theta", type=float, default=0.9)
ap.add_argument("--mode", choices=["probe", "scan"], default="probe")
ap.add_argument("--scan-size", type=int, default=100)
args = ap.parse_args()
if args.mode == "scan" and args.batch == 1 << 24:
    args.batch = 1 << 18

sys.path.insert(0, os.path.abspath(args.pkg))
import stage  # noqa: E402
from stage._lib import check  # noqa: E402

tab = stage.Table(key_width=8)
tab.load_ycsb(0, args.rows, 8, 0)
tab.sync()
s = stage.Stream()
e0, e1 = stage.Event(), stage.Event()
ms = []
if args.mode == "probe":
    keys = stage.zipf_draws(args.rows - 1, args.theta, 0x5EED, args.batch, nthreads=16)
    dk = stage.DeviceBuffer.from_numpy(keys)
    do = stage.DeviceBuffer(args.batch * 32)
    dr = stage.DeviceBuffer(args.batch * tab.stride)
    def step():
        tab.probe_device(dk.ptr, args.batch, do.ptr, dr.ptr, stream=s.ptr)
    n_out, per_unit = 1 << 20, 2100
else:
    starts = (stage.fastrandom(0x5EED, args.batch) % np.uint64(args.rows)).astype(np.uint64)
    dk = stage.DeviceBuffer.from_numpy(starts)
    do = stage.DeviceBuffer(args.batch * 4)
    dr = stage.DeviceBuffer(args.batch * args.scan_size * tab.stride)
    L = stage.lib()
    def step():
        check(L.stage_scan_batch(tab.h, dk.ptr, None, args.batch, args.scan_size, do.ptr, dr.ptr, s.ptr), "scan")
    n_out, per_unit = 1 << 12, 201868
step()
for r in range(args.rounds):
    e0.record(s)
    step()
    e1.record(s)
    s.sync()
    ms.append(e0.elapsed_ms(e1))
h = hashlib.sha1(do.to_numpy(np.uint8, n_out * (32 if args.mode == "probe" else 4)).tobytes() +
                 dr.to_numpy(np.uint8, n_out * tab.stride * (1 if args.mode == "probe" else args.scan_size)).tobytes())
med = float(np.median(ms))
print(json.dumps({"pkg": args.pkg, "mode": args.mode, "median_ms": med, "min_ms": float(min(ms)),
                  "units_per_s": args.batch / med * 1e3, "frac_of_8TBs": per_unit * args.batch / (med * 1e-3) / 8e12,
                  "digest": h.hexdigest()}), flush=True)
