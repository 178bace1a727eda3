"""CPU: bench.py's multi-rank launcher and CPU-baseline plumbing (no GPU).

`bench.py --gpus N` outside torch.distributed starts N ranks itself; the ranks' control plane
(gloo rendezvous, barrier, max-over-ranks timing, rank 0's single JSON line) is exercised with
--dry-run, which skips every device call.  Under torch.distributed a world size different
from --gpus is refused instead of being reported as a scaling point.
"""
import json
import os
import subprocess
import sys

import numpy as np

import bench
import oracle_lib as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=300):
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=e, cwd=REPO)


def _dry_line(world):
    p = _run(["--gpus", str(world), "--dry-run", "--steps", "2", "--cpu-seconds", "0.2", "--cpu-threads", "2"],
             timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [s for s in p.stdout.splitlines() if s.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def _check_sharded_line(r, world):
    rows = 200_000
    assert r["n_gpus"] == world and r["ranks"] == list(range(world)) and r["dry_run"] and r["self_check"]
    assert sum(r["rows_per_rank"]) == world * rows and min(r["rows_per_rank"]) > 0
    assert r["config"]["parallelism"] == f"hash-shard x{world}"
    # the workload names the real world and rows (configs[4]'s string only for 8 x 100M)
    assert r["config"]["workload"] == bench.sharded_workload(world, rows)
    assert r["config"]["workload"].startswith(f"YCSB-C {world * rows // 1000}K rows sharded {world} ways")
    # every N > 1 line carries the per-shard CPU baseline (rank 0, the oracle)
    cpu = r["cpu_baseline"]
    assert cpu and cpu["kind"] == "port" and cpu["value"] > 0 and cpu["rows"] == rows and cpu["cores"] >= 1
    assert "per shard" in cpu["scope"] and cpu["full_txn"]["value"] > 0
    # per-rank setup phases and host memory, for diagnosing a timeout or OOM from the record
    assert [p["rank"] for p in r["per_rank"]] == list(range(world))
    assert all(p["host_peak_rss_gib"] > 0 and set(p["setup_s"]) >= {"owned_keys", "load"} for p in r["per_rank"])


def test_launcher_starts_two_ranks():
    _check_sharded_line(_dry_line(2), 2)


def test_launcher_starts_eight_ranks():
    _check_sharded_line(_dry_line(8), 8)


def test_world_size_mismatch_is_refused():
    env = {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "1"}
    p = _run(["--gpus", "4", "--dry-run"], env=env, timeout=120)
    assert p.returncode == 2
    assert "refusing" in p.stderr
    assert not [s for s in p.stdout.splitlines() if s.startswith("{")]


def test_numpy_router_hash_matches_oracle_murmur():
    keys = np.random.default_rng(3).integers(0, 2**63, 5000, dtype=np.uint64)
    assert (bench.murmur64a_u64(keys) == O.murmur64a_keys(keys, 8, 0)).all()


def test_cpu_resources_and_rows():
    res = bench.cpu_resources()
    assert res["threads"] >= 1 and res["threads"] <= res["affinity_cpus"] <= (res["nproc"] or 1 << 20)
    assert res["mem_total_gib"] > 0
    a = bench.parse([])
    n = bench.cpu_rows_for(a, res, a.rows)
    assert 1_000_000 <= n <= a.rows and n % 1_000_000 == 0
    # a host that holds the whole table gets the whole table
    big = dict(res, _avail=400 * 2**30)
    assert bench.cpu_rows_for(a, big, a.rows) == a.rows
    a2 = bench.parse(["--cpu-rows", "3000000"])
    assert bench.cpu_rows_for(a2, res, a2.rows) == 3_000_000


def test_default_args_carry_the_nested_legs():
    a = bench.parse([])
    assert not a.no_extras and a.c3_epochs >= 1 and a.scan_batch == 1 << 18 and a.inflight_share > 0
    assert a.cpu_rows == 0 and a.cpu_threads == 0


def test_tpcc_tables_small():
    a = bench.parse(["--config", "tpcc", "--warehouses", "1", "--items", "200"])
    d = bench.tpcc_tables(a)
    assert d["stock"][0].shape == (200, 16) and d["district"][0].shape == (10, 16)
    assert d["order_line"][0].shape[1] == 32 and d["order_line"][1].shape[1] == 60
    assert callable(bench.run_tpcc) and callable(bench.run_chq2) and callable(bench.c3_leg) and callable(bench.c4_leg)


def test_share_gpu_rehearsal_labels_and_env(monkeypatch):
    # STAGE_RANKS_SHARE_GPU=1: ranks get distinct NCCL host ids (RCCL's socket transport between
    # ranks on one device) and the line names the rehearsal instead of an xGMI / scaling point
    for k in ("NCCL_HOSTID", "NCCL_SOCKET_IFNAME", "NCCL_NET", "NCCL_IB_DISABLE", bench.SHARE_GPU_ENV):
        monkeypatch.delenv(k, raising=False)
    assert not bench.share_gpu_rehearsal(0, 2)  # off unless asked for
    monkeypatch.setenv(bench.SHARE_GPU_ENV, "1")
    assert not bench.share_gpu_rehearsal(0, 1)  # nothing to share at world 1
    ids = set()
    for r in range(3):
        assert bench.share_gpu_rehearsal(r, 3)
        ids.add(os.environ["NCCL_HOSTID"])
    assert len(ids) == 3 and os.environ["NCCL_NET"] == "Socket" and os.environ["NCCL_SOCKET_IFNAME"] == "lo"
    w = bench.sharded_workload(2, 2_000_000, shared=True)
    assert "4M rows sharded 2 ways" in w and "sharing 1×MI355X" in w and "not an xGMI or scaling point" in w
    assert bench.sharded_workload(8, 100_000_000) == bench.WORKLOADS["c5"]
