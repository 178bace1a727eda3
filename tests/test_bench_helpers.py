"""CPU: bench.py's host-side helpers -- the multi-GPU xGMI roofline (only reached at N > 1 on
the driver's 8-GPU node) and the default arguments of the driver's N = 1 run."""
import sys

import bench


def test_xgmi_roofline_fields():
    hbm = {"bound": "hbm", "frac": 0.5}
    r = bench.xgmi_roofline(1 << 24, 8, 1024, 0.02, hbm)
    remote = (1 << 24) * 7 / 8
    assert r["bound"] == "xgmi" and r["hbm"] is hbm and r["unit"] == "GB/s"
    assert r["peak"] == 7 * bench.XGMI_LINK_GBS
    assert abs(r["achieved"] - remote * (16 + 32 + 1024) / 0.02 / 1e9) < 0.1
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert r["units_per_launch"] == round(remote) and r["avg_launch_ms"] == 20.0
    r2 = bench.xgmi_roofline(1000, 2, 1024, 1.0, hbm)
    assert r2["peak"] == bench.XGMI_LINK_GBS and r2["units_per_launch"] == 500
    # coalesced requests: the bytes of the remote requests actually routed
    r3 = bench.xgmi_roofline(1 << 24, 8, 1024, 0.02, hbm, remote=7_900_000)
    assert r3["units_per_launch"] == 7_900_000
    assert abs(r3["achieved"] - 7_900_000 * (16 + 32 + 1024) / 0.02 / 1e9) < 0.1


def test_default_args_are_the_c2_bench(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert (a.config, a.gpus, a.rows, a.batch, a.steps, a.warmup, a.theta) == ("c2", 1, 100_000_000, 1 << 24, 20, 3, 0.9)
