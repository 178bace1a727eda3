"""Profiling target for configs[2] (YCSB-B): the 100M-row table, EPOCHS epochs applied by the
device write path, then LAUNCHES probes of the last epoch's read share at its read ids (the
last LAUNCHES probe_kernel dispatches of the run; scripts/pmc_summary.py --last)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stage-indexorganized_amd"))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import stage  # noqa: E402

args = bench.parse(["--config", "c3", "--no-cpu-baseline"])
args.rows = int(os.environ.get("ROWS", args.rows))
epochs = int(os.environ.get("EPOCHS", 3))
launches = int(os.environ.get("LAUNCHES", 3))
tab = stage.Table(key_width=8)
tab.load_ycsb(0, args.rows, 8, 0)
tab.sync()
y = bench.YcsbB(tab, args, 16, 0.99)
for _ in range(epochs):
    ep = y.make_epoch()
    y.upload(ep)
    y.apply(ep)
s = stage.Stream()
dr = stage.DeviceBuffer(args.batch * tab.stride)
hops = 0
for _ in range(launches):
    tab.probe_device(ep["d"]["reads"].ptr, ep["reads"].size, ep["d"]["out"].ptr, dr.ptr,
                     d_read_ids=ep["d"]["rids"].ptr, stream=s.ptr)
s.sync()
o = ep["d"]["out"].to_numpy(stage.PROBE_OUT_DTYPE, ep["reads"].size)
print(f"done {launches} launches of {ep['reads'].size} reads, mean hops {o['hops'].mean():.4f}")
