"""Minimal profiling target: one 100M-row table, W+K probe launches of the bench workload
(used under rocprofv3 so counter passes do not pay for the CPU baseline)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stage-indexorganized_amd"))
import stage  # noqa: E402

rows = int(os.environ.get("ROWS", 100_000_000))
batch = int(os.environ.get("BATCH", 1 << 24))
launches = int(os.environ.get("LAUNCHES", 3))
tab = stage.Table(key_width=8)
tab.load_ycsb(0, rows, 8, 0)
tab.sync()
keys = stage.zipf_draws(rows - 1, 0.9, 0x5EED, batch, nthreads=16)
s = stage.Stream()
dk = stage.DeviceBuffer.from_numpy(keys)
do = stage.DeviceBuffer(batch * 32)
dr = stage.DeviceBuffer(batch * tab.stride)
for _ in range(launches):
    tab.probe_device(dk.ptr, batch, do.ptr, dr.ptr, stream=s.ptr)
s.sync()
print("done", launches, "launches")
