"""Minimal profiling target for C4 (configs[3]): one 100M-row table, W+K launches of the bench's
scan workload (2^18 uniform start keys, 100-key ranges, stage_scan_batch), so that the rocprofv3
--pmc passes do not pay for the bench's other legs.  Same start keys as bench.py c4_leg (seed
0x5EED, rank 0)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stage-indexorganized_amd"))
import stage  # noqa: E402

rows = int(os.environ.get("ROWS", 100_000_000))
batch = int(os.environ.get("BATCH", 1 << 18))
size = int(os.environ.get("SCAN_SIZE", 100))
launches = int(os.environ.get("LAUNCHES", 3))
tab = stage.Table(key_width=8)
tab.load_ycsb(0, rows, 8, 0)
tab.sync()
starts = (stage.fastrandom(0x5EED, batch) % np.uint64(rows)).astype(np.uint64)
s = stage.Stream()
L = stage.lib()
dk = stage.DeviceBuffer.from_numpy(starts)
dc = stage.DeviceBuffer(batch * 4)
dr = stage.DeviceBuffer(batch * size * tab.stride)
for _ in range(launches):
    assert L.stage_scan_batch(tab.h, dk.ptr, None, batch, size, dc.ptr, dr.ptr, s.ptr) == 0
s.sync()
print("done", launches, "launches of", batch, "scans")
