"""A/B of the probe's output layout (stage_set_output_layout) on the bench workload: one 100M-row
table, interleaved rounds in one process, each layout's launch timed with events.  Layouts:
default (1024-B rows, 32-B status), 1008-B rows, 16-B status, both.  Checks that every layout
writes the same bytes (rows: the first 1008 of each; status: the 16-B record's fields).
Prints one JSON line per layout."""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stage-indexorganized_amd"))
import stage  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=100_000_000)
ap.add_argument("--batch", type=int, default=1 << 24)
ap.add_argument("--rounds", type=int, default=6)
ap.add_argument("--theta", type=float, default=0.9)
args = ap.parse_args()

tab = stage.Table(key_width=8)
tab.load_ycsb(0, args.rows, 8, 0)
tab.sync()
keys = stage.zipf_draws(args.rows - 1, args.theta, 0x5EED, args.batch, nthreads=16)
s = stage.Stream()
dk = stage.DeviceBuffer.from_numpy(keys)
do = stage.DeviceBuffer(args.batch * 32)
dr = stage.DeviceBuffer(args.batch * 1024)
layouts = [(0, 32), (1008, 32), (0, 16), (1008, 16)]
res = {l: [] for l in layouts}
e0, e1 = stage.Event(), stage.Event()
check_n = 1 << 20
ref = None
same = True
for r in range(args.rounds):
    for lay in layouts:
        tab.set_output_layout(*lay)
        stride = tab.stride
        tab.probe_device(dk.ptr, args.batch, do.ptr, dr.ptr, stream=s.ptr)
        e0.record(s)
        tab.probe_device(dk.ptr, args.batch, do.ptr, dr.ptr, stream=s.ptr)
        e1.record(s)
        s.sync()
        res[lay].append(e0.elapsed_ms(e1))
        if r == 0:
            dt = stage.PROBE_OUT16_DTYPE if lay[1] == 16 else stage.PROBE_OUT_DTYPE
            out = do.to_numpy(dt, check_n)
            rows = dr.to_numpy(np.uint8, check_n * stride).reshape(check_n, stride)[:, :1008]
            if ref is None:
                ref = (out, rows)
            else:
                same &= bool((rows == ref[1]).all())
                for f in ("status", "flags", "hops", "cstamp", "copy_sstamp", "rec_cstamp"):
                    same &= bool((out[f] == ref[0][f]).all())
tab.set_output_layout(0, 32)
for lay in layouts:
    ms = np.array(res[lay])
    written = (1008 if lay[0] else 1024) + lay[1]
    print(json.dumps({"row_stride": lay[0] or 1024, "status_bytes": lay[1], "median_ms": float(np.median(ms)),
                      "min_ms": float(ms.min()), "glookups_s": args.batch / np.median(ms) / 1e6,
                      "frac_2100B": 2100 * args.batch / (np.median(ms) * 1e-3) / 8e12,
                      "bytes_written_per_lookup": written, "outputs_identical": same}), flush=True)
