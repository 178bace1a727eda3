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


def test_sharded_workload_names_world_and_rows():
    import json
    import os
    base = json.load(open(os.path.join(os.path.dirname(bench.__file__), "BASELINE.json")))
    assert bench.sharded_workload(8, 100_000_000) == base["configs"][4]
    assert bench.sharded_workload(2, 100_000_000) == \
        "YCSB-C 200M rows sharded 2 ways, RCCL all-to-all key routing over xGMI, 2×MI355X"
    assert bench.sharded_workload(4, 100_000_000) != base["configs"][4]
    assert "rehearsal" in bench.sharded_workload(1, 100_000_000)


def test_sharded_hbm_bytes_counts_what_moves():
    # world 1: everything is own -- owners' probes of the coalesced requests + every caller row
    st = {"keys": 1000, "routed": 600, "remote": 0, "received": 600}
    b, parts = bench.sharded_hbm_bytes(st, 1024)
    assert parts["owner_probes"] == 600 * 1088 and parts["caller_rows"] == 1000 * 1012
    assert parts["remote_results"] == parts["returned_results"] == parts["key_records"] == 0
    assert b == 600 * 1088 + 1000 * 1012
    # world > 1: 500 of 600 requests go out, 480 other-rank requests come in (+ 100 own)
    st = {"keys": 1000, "routed": 600, "remote": 500, "received": 580}
    b, parts = bench.sharded_hbm_bytes(st, 1024)
    assert parts["remote_results"] == 480 * 2 * 1012 and parts["returned_results"] == 500 * 2 * 1012
    assert parts["key_records"] == (500 + 480) * 32 and b == sum(parts.values())


def test_cpu_legs_c3_times_concurrent_writers():
    """The C3 CPU leg replays the GPU's epochs on the oracle and times the last epoch's updates
    on T concurrent writers (orc_update_batch_mt) beside its reads: the fields the line carries,
    no one-thread update timing left."""
    import types

    import numpy as np
    rows = 30_000
    orc = bench.CpuOracle(rows, 4)
    args = types.SimpleNamespace(seed=3, cpu_seconds=0.05, scan_size=100, rows=rows)
    rng = np.random.default_rng(0)
    record = []
    counter = 1
    for ep in range(3):
        m = 3000
        keys = rng.integers(0, rows, m).astype(np.uint64)
        rid = (counter + 2 * np.arange(m)).astype(np.uint32)
        counter += 2 * m
        record.append({"keys": keys, "colb": rng.integers(0, 4, m).astype(np.uint8), "rid": rid,
                       "cid": (rid + 1).astype(np.uint32)})
    reads = rng.integers(0, rows, 20_000).astype(np.uint64)
    rids = np.full(reads.size, counter, np.uint32)
    res = {"cpu_model": "test", "nproc": 8}
    out = bench.cpu_legs(orc, args, res, 4, c3={"record": record, "reads": reads, "rids": rids})
    c3 = out["c3"]
    assert "last_epoch_update_s_1_thread" not in c3
    assert c3["update_writers"] == 4 and c3["last_epoch_update_ops"] == 3000
    assert 0 < c3["last_epoch_updates_ok"] <= 3000 and c3["updates_per_s"] > 0
    assert c3["updates_replayed"] >= c3["last_epoch_updates_ok"]
    assert c3["value"] > 0 and c3["reads_per_s"] > 0
