#!/usr/bin/env python3
"""bench.py -- YCSB-C batched point lookup on MI355X (BASELINE.json configs[1]).

Workload (one "step" = one pass of the hot path over one batch):
  table  : N rows per GPU loaded as LoadYCSBRows does (key = rowid, here 8-byte keys,
           payload = memset(rowid) 1000 B), reference leaf layout (64 KiB leaves, 63 slots)
  batch  : B = 2^24 Zipf(theta=0.9) draws over [1, N_total-1] (ZipfDistribution of
           benchmark_common.h, seed 0x5EED + rank), read_id = MAX_CID-1
  step   : device traversal + leaf probe + visibility + 1008-B tuple copy for all B keys
           (stage_probe_batch); with --gpus > 1 every key is routed to shard
           MurmurHash64A(key, 8, 0) % world and answered over RCCL (stage_probe_sharded)
value = lookups completed by all ranks / max-over-ranks wall time of the K timed steps.

The CPU baseline leg (rank 0, one GPU only) times the test oracle -- the C restatement of
the reference's BTree::Read + executor copy -- on a bounded 2M-row sample (the reference's
own default pools cap a YCSB table at ~2-2.5M rows).
"""
import argparse
import ctypes
import json
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "stage-indexorganized_amd"))
import stage  # noqa: E402  (load libstage_hip.so before anything else binds a HIP runtime)
from stage._lib import check  # noqa: E402

METRIC = "YCSB ops/sec at 1/2/4/8 GPU + achieved HBM GB/s vs peak; CPU ref ops/sec"
WORKLOAD = "YCSB-C 100M rows uint64 keys, zipf 0.9, batched point-lookup on 1×MI355X"
WORKLOAD_MULTI = "YCSB-C 800M rows sharded 8 ways, RCCL all-to-all key routing over xGMI, 8×MI355X"
BYTES_PER_LOOKUP = 2100  # 8 key + 64 key-column line + 16 slot word + 1000 payload + 1008 out + 4
HBM_PEAK_GBS = 8000.0    # MI355X_MICROARCH.md: 8.0 TB/s HBM3E spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--rows", type=int, default=100_000_000, help="rows per GPU")
    p.add_argument("--batch", type=int, default=1 << 24, help="lookups per GPU per step")
    p.add_argument("--theta", type=float, default=0.9)
    p.add_argument("--seed", type=int, default=0x5EED)
    p.add_argument("--cpu-rows", type=int, default=2_000_000)
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--host-traversal", action="store_true", help="leaf ids from the host router instead")
    return p.parse_args()


def owned_keys(total_rows, world, rank):
    """Keys of this shard: MurmurHash64A(key, 8, 0) % world == rank, ascending (loaded in order)."""
    parts = []
    chunk = 1 << 24
    for b in range(0, total_rows, chunk):
        k = np.arange(b, min(total_rows, b + chunk), dtype=np.uint64)
        h = stage.murmur64a_device(k, 8, 0)
        parts.append(k[(h % np.uint64(world)) == np.uint64(rank)])
    return np.concatenate(parts)


def traffic_from_profile(batch, rows):
    """Per-launch HBM bytes of probe_kernel from a committed rocprofv3 --pmc pass (see
    profiles/README.md), if one exists for this configuration."""
    path = os.path.join(REPO, "profiles", "pmc_probe.json")
    if not os.path.exists(path):
        return None, None
    try:
        d = json.load(open(path))
        if d.get("batch") == batch and d.get("rows") == rows:
            return d["hbm_bytes_per_launch"], os.path.relpath(path, REPO)
    except Exception:
        pass
    return None, None


def cpu_baseline(args, threads):
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib as O  # the checker, timed here as the reference CPU path
    n = args.cpu_rows
    t0 = time.time()
    orc = O.OracleTree()
    orc.load_ycsb(0, n, 8, 0)
    build_s = time.time() - t0
    keys = stage.zipf_draws(n - 1, args.theta, args.seed, 400_000, nthreads=threads)
    secs = ctypes.c_double()
    O.lib().orc_read_batch_timed(orc.t, keys.ctypes.data, 8, None, keys.size, threads, ctypes.byref(secs))
    rate = keys.size / max(secs.value, 1e-9)
    count = int(min(max(rate * args.cpu_seconds, 100_000), 50_000_000))
    keys = stage.zipf_draws(n - 1, args.theta, args.seed + 1, count, nthreads=threads)
    O.lib().orc_read_batch_timed(orc.t, keys.ctypes.data, 8, None, keys.size, threads, ctypes.byref(secs))
    value = keys.size / secs.value
    cpu = platform.processor() or "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(value, 1), "unit": "ops/s", "cores": threads, "kind": "port",
            "sample": f"oracle BTree::Read+copy, {n} rows (8-B keys, 1000-B payload, build {build_s:.1f}s), "
                      f"{count} zipf-{args.theta} lookups, {threads} threads on {cpu}, {secs.value:.1f}s"}


def main():
    args = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        tdist.init_process_group("gloo")  # control plane only; the data path is RCCL in the library
        dist = tdist
    nthreads = min(16, os.cpu_count() or 8)
    check(stage.lib().stage_set_device(local), "set device")

    total_rows = args.rows * world
    t0 = time.time()
    tab = stage.Table(key_width=8, device=local)
    if world == 1:
        loaded = tab.load_ycsb(0, total_rows, 8, mode=0)
    else:
        keys = owned_keys(total_rows, world, rank)
        loaded = tab.load_keys(keys, 8, mode=0)
        del keys
    t_load = time.time() - t0
    t0 = time.time()
    tab.sync()
    t_sync = time.time() - t0
    st = tab.stats()
    log(f"[rank {rank}] loaded {loaded} rows in {t_load:.1f}s, sync {t_sync:.1f}s, leaves {st['leaves']}")

    B = args.batch
    draws = stage.zipf_draws(total_rows - 1, args.theta, args.seed + rank, B, nthreads=nthreads)
    stream = stage.Stream()
    d_keys = stage.DeviceBuffer.from_numpy(draws)
    d_out = stage.DeviceBuffer(B * 32)
    d_rec = stage.DeviceBuffer(B * tab.stride)
    d_leaf = None
    if args.host_traversal and world == 1:
        d_leaf = stage.DeviceBuffer.from_numpy(tab.traverse(draws))

    L = stage.lib()
    if world > 1:
        uid = (ctypes.c_uint8 * 128)()
        if rank == 0:
            check(L.stage_comm_unique_id(uid), "unique id")
        obj = [bytes(uid)]
        dist.broadcast_object_list(obj, src=0)
        uid = (ctypes.c_uint8 * 128).from_buffer_copy(obj[0])
        check(L.stage_comm_init(tab.h, uid, rank, world), "comm init")

    def step():
        if world == 1:
            tab.probe_device(d_keys.ptr, B, d_out.ptr, d_rec.ptr, d_leaf_ids=d_leaf.ptr if d_leaf else None,
                             stream=stream.ptr)
        else:
            check(L.stage_probe_sharded(tab.h, d_keys.ptr, None, B, d_out.ptr, d_rec.ptr, stream.ptr), "sharded")

    for _ in range(args.warmup):
        step()
    stream.sync()
    if dist:
        dist.barrier()
    check(L.stage_device_sync(), "sync")
    evs = [stage.Event() for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    evs[0].record(stream)
    for i in range(args.steps):
        step()
        evs[i + 1].record(stream)
    stream.sync()
    check(L.stage_device_sync(), "sync")
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = t1 - t0
    if dist:
        import torch
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    step_ms = [evs[i].elapsed_ms(evs[i + 1]) for i in range(args.steps)]
    kern_ms = float(np.mean(step_ms))

    # self-check outside the timed region: every lookup hit, tuple = [key][memset(key)]
    sample = min(B, 65536)
    outs = d_out.to_numpy(stage.PROBE_OUT_DTYPE, sample)
    rows = d_rec.to_numpy(np.uint8, sample * tab.stride).reshape(sample, tab.stride)
    ok = bool((outs["status"] == stage.ST_LATEST).all() and
              (rows[:, :8].copy().view(np.uint64).ravel() == draws[:sample]).all() and
              (rows[:, 8:1008] == (draws[:sample] & np.uint64(0xFF)).astype(np.uint8)[:, None]).all())
    if not ok:
        log(f"[rank {rank}] SELF-CHECK FAILED")

    total = B * world * args.steps
    value = total / elapsed
    result = None
    if rank == 0:
        achieved = BYTES_PER_LOOKUP * B / (kern_ms * 1e-3) / 1e9
        traffic, tsrc = traffic_from_profile(B, args.rows)
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "kernel": "probe_kernel" if world == 1 else "sharded step (route+RCCL+probe_kernel)",
                "bytes_per_lookup": BYTES_PER_LOOKUP, "avg_launch_ms": round(kern_ms, 4)}
        if tsrc:
            roof["traffic_source"] = tsrc
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args, nthreads)
        result = {
            "metric": METRIC, "value": round(value, 1), "unit": "ops/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic (LoadYCSBRows keys/payloads)",
            "config": {"workload": WORKLOAD if world == 1 else WORKLOAD_MULTI, "rows_per_gpu": args.rows,
                       "rows_total": total_rows, "batch_per_gpu": B, "theta": args.theta, "key_bytes": 8,
                       "payload_bytes": 1000, "leaf_bytes": 65536, "parallelism": f"hash-shard x{world}",
                       "traversal": "host" if d_leaf else "device"},
            "roofline": roof, "cpu_baseline": cpu, "self_check": ok,
            "setup_s": {"load": round(t_load, 1), "sync": round(t_sync, 1)},
        }
        print(json.dumps(result), flush=True)
    if dist:
        dist.barrier()
        check(L.stage_comm_destroy(tab.h), "comm destroy")
        dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
