"""Probe time vs key skew on the C2 table (100M rows, 2^24 lookups): how much of the Zipf
batch's locality the caches already catch.  uniform / Zipf 0.5 / 0.9 / 0.99, plus the 0.9
batch sorted by key (the locality upper bound of any batch reordering)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stage-indexorganized_amd"))
import numpy as np

import stage

ROWS, B = 100_000_000, 1 << 24
tab = stage.Table(key_width=8)
tab.load_ycsb(0, ROWS, 8, mode=0)
tab.sync()
L = stage.lib()
s = stage.Stream()
d_keys = stage.DeviceBuffer(B * 8)
d_out = stage.DeviceBuffer(B * 32)
d_rec = stage.DeviceBuffer(B * tab.stride)
batches = {"uniform": np.random.default_rng(1).integers(0, ROWS, B).astype(np.uint64)}
for th in (0.5, 0.9, 0.99):
    batches[f"zipf{th}"] = stage.zipf_draws(ROWS - 1, th, 7, B, nthreads=16)
batches["zipf0.9_sorted"] = np.sort(batches["zipf0.9"])
for name, keys in batches.items():
    L.stage_memcpy_h2d(d_keys.ptr, keys.ctypes.data, keys.nbytes, None)
    evs = [stage.Event() for _ in range(12)]
    for i in range(6):
        evs[2 * i].record(s)
        tab.probe_device(d_keys.ptr, B, d_out.ptr, d_rec.ptr, stream=s.ptr)
        evs[2 * i + 1].record(s)
    s.sync()
    ms = np.mean([evs[2 * i].elapsed_ms(evs[2 * i + 1]) for i in range(1, 6)])
    print(f"{name:16s} unique {np.unique(keys).size / B:.3f}  {ms:.3f} ms  "
          f"{B / ms / 1e6:.3f} G lookups/s  {2100 * B / ms / 1e6:.0f} GB/s algorithmic", flush=True)
