#!/usr/bin/env python3
"""bench.py -- YCSB on MI355X through the index-organized probe/scan path.

Default (`--config c2`, BASELINE.json configs[1]): YCSB-C batched point lookup.
  table : N rows per GPU loaded as LoadYCSBRows does (key = rowid, 8-byte keys, payload =
          memset(rowid) 1000 B), reference leaf layout (64 KiB leaves, <= 63 records)
  step  : one pass of the hot path over a batch of B = 2^24 Zipf(0.9) lookups over
          [1, N_total-1] (ZipfDistribution of benchmark_common.h, seed 0x5EED + rank):
          device traversal + leaf probe + visibility + 1008-B tuple copy (stage_probe_batch);
          with --gpus > 1 each key goes to shard MurmurHash64A(key, 8, 0) % world and is
          answered over RCCL (stage_probe_sharded, run_sharded) -- configs[4] at 8 GPUs
  value = lookups completed by all ranks / max-over-ranks wall time of the K timed steps.
  After the headline the same 100M-row table runs configs[3] (C4, 100-key scans) and then
  configs[2] (C3, YCSB-B epochs; last, since it mutates the table); their lines are nested
  under "extras" and do not change value / metric / config.
`--config c3` / `--config c4` make those the headline instead.

`--gpus N` (N > 1) without a torch.distributed environment starts N ranks itself (a child
`python -m torch.distributed.run`, before any GPU call) and forwards rank 0's JSON line; under
torch.distributed the world size must equal --gpus.

The CPU baseline leg (rank 0; at N > 1 the per-shard C2 leg) times the test oracle -- the C restatement of the
reference's BTree::Read + executor copy ("lookup" mode) and of RunMixed's read-only
transactions with the Index-SSN read side ("full-txn" mode) -- on the largest table the host
RAM holds (up to the GPU's N; built in parallel with the same leaves as the single loader,
while the GPU leg runs), with the threads this process may use (affinity and cgroup quota).
"""
import argparse
import ctypes
import json
import math
import os
import platform
import resource
import socket
import subprocess
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "stage-indexorganized_amd"))
import stage  # noqa: E402  (libstage_hip.so is loaded lazily, on the first library call)
from stage._lib import check  # noqa: E402

METRIC = "YCSB ops/sec at 1/2/4/8 GPU + achieved HBM GB/s vs peak; CPU ref ops/sec"
WORKLOADS = {
    "c2": "YCSB-C 100M rows uint64 keys, zipf 0.9, batched point-lookup on 1×MI355X",
    "c3": "YCSB-B 100M rows, update_ratio 0.05, zipf 0.99 (version-chain visibility on GPU), 1×MI355X",
    "c4": "YCSB scan_mode, 100M rows, 100-key ranges (leaf range-scan + gather), 1×MI355X",
    "c5": "YCSB-C 800M rows sharded 8 ways, RCCL all-to-all key routing over xGMI, 8×MI355X",
}
# algorithmic bytes
BYTES_PER_LOOKUP = 2100  # 8 key + 64 key-column line + 16 slot word + 1000 payload + 1008 out + 4
HOP_BYTES = 64           # C3: one TupleHeader (version) line per chain hop taken
HBM_PEAK_GBS = 8000.0    # MI355X_MICROARCH.md: 8.0 TB/s HBM3E spec
XGMI_LINK_GBS = 153.0    # per xGMI link of an MI355X (7 links per GPU, point to point)
ORACLE_BYTES_PER_ROW = 1800  # oracle tree host memory per YCSB row (64 KiB leaves, ~38-48 rows each, + inner)
GPU_HOST_BYTES_PER_ROW = 210  # host peak of a rank per row (19.5 GiB at 100M rows, sharded world 1, round 3)
# the reference itself, measured in the survey container and the oracle in
# the same container type: calibration of the port
REF_C1_OPS = 1533428.0       # YCSB-C -k 1000 -o 10, 1 thread
REF_READ_NS_1M = 1786.0      # BTree::Read, 1M rows, 1 thread
REF_TXN_OPS_1M = 428817.0    # YCSB-C 1M rows, 1 thread, full driver


def scan_bytes(L, S=48.8):
    """B_scan = 8 + 64*(ceil(L/S)+1) + L*(8+1000) + L*1008 + 4."""
    return 8 + 64 * (math.ceil(L / S) + 1) + L * (8 + 1000) + L * 1008 + 4


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1,
                   help="ranks (one per GPU); > 1 without torch.distributed env: launch them")
    p.add_argument("--steps", type=int, default=None)
    p.add_argument("--warmup", type=int, default=None)
    p.add_argument("--config", choices=["c2", "c3", "c4", "tpcc", "chq2"], default="c2")
    p.add_argument("--warehouses", type=int, default=16, help="tpcc: warehouses (10 districts, 3000 orders each)")
    p.add_argument("--items", type=int, default=100_000, help="tpcc: items (stock rows per warehouse)")
    p.add_argument("--q2-batch", type=int, default=16, help="chq2: Q2 transactions per step (stage_ch_query2_batch)")
    p.add_argument("--q2-async", type=int, default=1, choices=[0, 1],
                   help="chq2: 1 = two batches in flight (stage_ch_query2_batch_async, slots 0/1 alternating: "
                        "the host stages batch k+1 while the device runs batch k); 0 = one synchronous batch "
                        "per step (stage_ch_query2_batch)")
    p.add_argument("--rows", type=int, default=100_000_000, help="rows per GPU")
    p.add_argument("--batch", type=int, default=None, help="lookups (c2/c3) or scans (c4) per GPU per step")
    p.add_argument("--theta", type=float, default=None)
    p.add_argument("--scan-size", type=int, default=100)
    p.add_argument("--scan-batch", type=int, default=1 << 18, help="scans per step of the C4 leg")
    p.add_argument("--update-ratio", type=float, default=0.05)
    p.add_argument("--old-share", type=float, default=0.25,
                   help="c3: share of reads at an older snapshot (0: every read at the newest id)")
    p.add_argument("--reader-window", type=int, default=1280,
                   help="c3: older-snapshot readers trail the newest id by up to this many ids (RunMixed: "
                        "64 threads x 10 ops x 2 ids)")
    p.add_argument("--inflight-share", type=float, default=0.02,
                   help="c3: share of the update ops left in flight (uncommitted; keys beyond the 10^4 hottest) "
                        "so reads of them take the overwrite-copy (COPY) branch")
    p.add_argument("--c3-epochs", type=int, default=16,
                   help="timed YCSB-B epochs of the nested C3 leg (the write pipeline's fill and the last "
                        "epoch's host adoption are inside the timed loop, amortised over these; round 6: 8 -> 16)")
    p.add_argument("--write-path", choices=["device", "host"], default="device",
                   help="c3: apply each epoch's updates on the device (stage_update_batch_device) or on the "
                        "host write path + incremental publish (stage_update_batch + stage_sync)")
    p.add_argument("--seed", type=int, default=0x5EED)
    p.add_argument("--cpu-rows", type=int, default=0, help="oracle rows of the CPU leg (0 = the largest that fits)")
    p.add_argument("--cpu-seconds", type=float, default=6.0, help="target CPU time of each timed CPU sample")
    p.add_argument("--cpu-threads", type=int, default=0, help="0 = the CPUs this process may use")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extras", action="store_true", help="c2: skip the nested C4 / C3 legs")
    p.add_argument("--host-traversal", action="store_true", help="leaf ids from the host router instead")
    p.add_argument("--no-e2e", action="store_true", help="c2: skip the end-to-end (host-buffer) leg")
    p.add_argument("--e2e-passes", type=int, default=2, help="c2: passes over the batch of the end-to-end leg")
    p.add_argument("--write-overlap", type=int, choices=[0, 1], default=1,
                   help="device write path: 1 = an epoch's kernels up to its publish run beside the previous "
                        "epoch's read probe (stage_set_write_overlap; the epoch inputs are resident beforehand)")
    p.add_argument("--out-stride", type=int, default=0,
                   help="caller row stride in bytes (stage_set_output_layout; 0 = the 1008-B canonical row)")
    p.add_argument("--reply", choices=["auto", "rows", "peer", "direct"], default="auto",
                   help="N > 1: how remote rows reach the caller -- rows: back over RCCL; peer: read by the caller's "
                        "fan-out from the owners' IPC-mapped row buffers (STAGE_REPLY_PEER); direct: written by the "
                        "owners into the callers' IPC-mapped outputs (STAGE_REPLY_DIRECT); auto: peer, falling back "
                        "to rows when the runtime refuses the mapping, then times rows and direct too and reports the "
                        "fastest full reply whose sample check passed on every rank as the line's value, the others "
                        "beside it (same results either way)")
    p.add_argument("--force-sharded", action="store_true",
                   help="run the multi-GPU (RCCL) code path even with one rank -- a rehearsal, not a config")
    p.add_argument("--dry-run", action="store_true",
                   help="control plane only (no GPU): ranks rendezvous over gloo, load their shard's host "
                        "table, time a routing step; for CPU tests of the launcher")
    a = p.parse_args(argv)
    a.steps = a.steps if a.steps is not None else (10 if a.config in ("c3", "tpcc") else 20)
    a.warmup = a.warmup if a.warmup is not None else (1 if a.config == "c3" else 3)
    a.theta = a.theta if a.theta is not None else (0.99 if a.config == "c3" else 0.9)
    a.batch = a.batch if a.batch is not None else ((1 << 18) if a.config in ("c4", "tpcc") else (1 << 24))
    return a


# ------------------------------------------------------------------------ multi-rank launch
def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv):
    """--gpus N > 1 outside torch.distributed: run N ranks as a child torch.distributed.run
    (this process never touches the GPU and never execs), forward rank 0's JSON line, and
    fail unless it reports n_gpus == N."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "8")
    log(f"[launcher] {' '.join(cmd)}")
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    line = None
    for raw in p.stdout:
        s = raw.strip()
        if s.startswith("{") and '"metric"' in s:
            line = s
        else:
            log(raw.rstrip())
    rc = p.wait()
    if line is None:
        log(f"[launcher] no result line from the ranks (exit {rc})")
        return rc or 1
    print(line, flush=True)
    n = json.loads(line).get("n_gpus")
    if n != args.gpus:
        log(f"[launcher] ranks reported n_gpus={n}, expected {args.gpus}")
        return 1
    return rc


def murmur64a_u64(keys, seed=0):
    """MurmurHash64A of 8-byte little-endian keys (misc/murmur/MurmurHash2.cpp:99-147), numpy:
    the router's hash for the host-only --dry-run (the GPU path uses murmur_kernel)."""
    m, r = np.uint64(0xC6A4A7935BD1E995), np.uint64(47)
    with np.errstate(over="ignore"):
        h = np.full(keys.shape, np.uint64(seed) ^ (np.uint64(8) * m), np.uint64)
        k = keys.astype(np.uint64) * m
        k ^= k >> r
        k *= m
        h ^= k
        h *= m
        h ^= h >> r
        h *= m
        h ^= h >> r
    return h


def dry_run(args, rank, world, dist):
    """Control-plane rehearsal without a GPU: the ranks of the launcher rendezvous (gloo), each
    loads its shard (MurmurHash64A(key) % world) into a host table, routes a probe batch to its
    owners with an all-to-all, and the step is timed with the bench's barrier / max-over-ranks
    rule; rank 0 times the per-shard CPU leg (the oracle, as the sharded GPU run does) and
    prints the result line with the same workload label and per-rank report as a GPU run."""
    import torch
    res = cpu_resources()
    threads = min(4, args.cpu_threads or res["threads"])
    rows = min(args.rows, 200_000)
    keys = np.arange(rows * world, dtype=np.uint64)
    t0 = time.time()
    mine = keys[murmur64a_u64(keys) % np.uint64(world) == np.uint64(rank)]
    t_owned = time.time() - t0
    t0 = time.time()
    tab = stage.Table(key_width=8)
    loaded = tab.load_keys(mine, 8, 0)
    t_load = time.time() - t0
    probes = stage.zipf_draws(rows * world - 1, args.theta, args.seed + rank, 1 << 14, nthreads=2)
    dest = (murmur64a_u64(probes) % np.uint64(world)).astype(np.int64)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        order = np.argsort(dest, kind="stable")
        scount = torch.tensor(np.bincount(dest, minlength=world), dtype=torch.int64)
        rcount = torch.zeros(world, dtype=torch.int64)
        dist.all_to_all_single(rcount, scount)
        recv = torch.zeros(int(rcount.sum()), dtype=torch.int64)
        dist.all_to_all_single(recv, torch.from_numpy(probes[order].view(np.int64).copy()), rcount.tolist(),
                               scount.tolist())
    elapsed = time.perf_counter() - t0
    got = recv.numpy().view(np.uint64)
    ok = bool((murmur64a_u64(got) % np.uint64(world) == np.uint64(rank)).all())
    tt = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    mine_report = rank_report(rank, loaded, {"owned_keys": t_owned, "load": t_load}, ok)
    reports = [torch.zeros(len(mine_report), dtype=torch.float64) for _ in range(world)]
    dist.all_gather(reports, torch.tensor(mine_report, dtype=torch.float64))
    dist.barrier()
    if rank == 0:
        per_rank = per_rank_reports(np.stack([r.numpy() for r in reports]))
        cpu = cpu_leg_sharded(args, res, world, threads, rows, rows, None)
        total = float(tt.item())
        print(json.dumps({"metric": METRIC, "value": round(probes.size * args.steps * world / total, 1),
                          "unit": "routed keys/s (dry run, no GPU)", "n_gpus": world, "steps": args.steps,
                          "warmup": 0, "ms_per_step": round(total / args.steps * 1e3, 4), "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
                          "dry_run": True, "ranks": [p["rank"] for p in per_rank],
                          "rows_per_rank": [p["rows"] for p in per_rank], "per_rank": per_rank,
                          "self_check": all(p["self_check"] for p in per_rank),
                          "config": {"workload": sharded_workload(world, rows), "rows_per_gpu": rows,
                                     "rows_total": rows * world, "parallelism": f"hash-shard x{world}",
                                     "control_plane": "gloo (dry run)"},
                          "cpu_baseline": cpu}), flush=True)
    return 0


RANK_REPORT = ("rank", "rows", "owned_keys_s", "load_s", "sync_s", "comm_init_s", "host_peak_rss_gib", "self_check")


def rank_report(rank, rows, setup, ok):
    """one rank's setup phases, peak host RSS and self-check as a float vector (gathered over ranks)"""
    rss = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20
    return [float(rank), float(rows), setup.get("owned_keys", 0.0), setup.get("load", 0.0), setup.get("sync", 0.0),
            setup.get("comm_init", 0.0), rss, 1.0 if ok else 0.0]


def per_rank_reports(mat):
    out = []
    for row in mat:
        d = dict(zip(RANK_REPORT, (float(x) for x in row)))
        out.append({"rank": int(d["rank"]), "rows": int(d["rows"]), "self_check": d["self_check"] > 0.5,
                    "host_peak_rss_gib": round(d["host_peak_rss_gib"], 2),
                    "setup_s": {k[:-2]: round(d[k], 2) for k in ("owned_keys_s", "load_s", "sync_s", "comm_init_s")}})
    return out


def cpu_leg_sharded(args, res, world, threads, cpu_rows, gpu_rows, c2_check):
    """The CPU baseline of a sharded line (C2's per-shard CPU number): rank 0
    builds the oracle table (LoadYCSBRows, the largest that fits beside the world's device tables
    on this node, <= one shard's rows) after the GPU timing and times C2's lookup and full-txn
    modes on it; GPU samples with keys inside the oracle's range are checked against it."""
    if args.no_cpu_baseline:
        return None
    orc = CpuOracle(cpu_rows, threads)
    legs = cpu_legs(orc, args, res, threads, c2_check=c2_check, legs=("c2",))
    c2 = legs["c2"]
    c2["scope"] = (f"per shard: one rank's share of the work on {cpu_rows} rows (a shard holds {gpu_rows}); "
                   f"compare with the line's value / n_gpus")
    return c2


def owned_keys(total_rows, world, rank):
    """Keys of this shard: MurmurHash64A(key, 8, 0) % world == rank, ascending (loaded in order)."""
    parts = []
    chunk = 1 << 24
    for b in range(0, total_rows, chunk):
        k = np.arange(b, min(total_rows, b + chunk), dtype=np.uint64)
        h = stage.murmur64a_device(k, 8, 0)
        parts.append(k[(h % np.uint64(world)) == np.uint64(rank)])
    return np.concatenate(parts)


class RcclControl:
    """Control plane of the GPU ranks over their own RCCL communicator (no second collective
    library in the process): the 128-byte unique id goes from rank 0 to the others through a
    file on the node (the ranks of one torch.distributed.run share a parent and a /tmp), then
    barrier / max-over-ranks / gather are small allreduces on the communicator."""

    def __init__(self, tab, rank, world):
        self.tab, self.rank, self.world = tab, rank, world
        L = stage.lib()
        tag = f"{os.environ.get('MASTER_ADDR', '127.0.0.1')}_{os.environ.get('MASTER_PORT', '0')}_{os.getppid()}"
        self.path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"stage_rccl_uid_{tag}.bin")
        uid = (ctypes.c_uint8 * 128)()
        if rank == 0:
            check(L.stage_comm_unique_id(uid), "unique id")
            tmp = f"{self.path}.{os.getpid()}.tmp"
            with open(tmp, "wb") as f:
                f.write(bytes(uid))
            os.replace(tmp, self.path)
        else:
            deadline = time.time() + 600
            while True:
                try:
                    with open(self.path, "rb") as f:
                        b = f.read()
                    if len(b) == 128:
                        break
                except OSError:
                    pass
                if time.time() > deadline:
                    raise RuntimeError(f"rank {rank}: no RCCL unique id from rank 0 at {self.path}")
                time.sleep(0.05)
            uid = (ctypes.c_uint8 * 128).from_buffer_copy(b)
        check(L.stage_comm_init(tab.h, uid, rank, world), "comm init")

    def barrier(self):
        stage.comm_allreduce(self.tab, [1.0])

    def max(self, x):
        return float(stage.comm_allreduce(self.tab, [x], "max")[0])

    def gather(self, vec):
        return stage.comm_allgather(self.tab, vec, self.world)

    def close(self):
        if self.rank == 0:
            try:
                os.remove(self.path)
            except OSError:
                pass
        check(stage.lib().stage_comm_destroy(self.tab.h), "comm destroy")


SHARE_GPU_ENV = "STAGE_RANKS_SHARE_GPU"


def share_gpu_rehearsal(rank, world):
    """STAGE_RANKS_SHARE_GPU=1 with world > 1: every rank runs on device 0 of a one-GPU box and
    RCCL is told the ranks live on different hosts (a per-rank NCCL_HOSTID; RCCL refuses two
    ranks of one host on one device), so the exchange runs over its socket transport on the
    loopback interface.  That executes the real multi-rank RCCL calls of the sharded step (the
    counts all-to-all, grouped send/recv with peers, the control plane) on hardware this pool
    hands out; xGMI bandwidth is not what it measures, and the line says so.  Must run before
    the first RCCL call of the process."""
    if world <= 1 or os.environ.get(SHARE_GPU_ENV) != "1":
        return False
    os.environ["NCCL_HOSTID"] = f"stage-rehearsal-{os.getppid()}-rank{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_NET", "Socket")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    return True


def rank_device(local):
    """The device of local rank `local`: device `local` when every GPU of the node is visible;
    device 0 when a launcher left each rank exactly one visible GPU (HIP_VISIBLE_DEVICES /
    ROCR_VISIBLE_DEVICES per rank)."""
    ndev = stage.device_count()
    if local < ndev:
        return local
    if ndev == 1:
        log(f"[local rank {local}] one visible GPU: using device 0")
        return 0
    raise SystemExit(f"local rank {local} but only {ndev} visible GPUs")


def run_sharded(args, rank, world, local):
    """configs[4] (C5) and its 1/2/4 smaller points: every rank holds the keys with
    MurmurHash64A(key, 8, 0) % world == rank (rows_per_gpu each, weak scaling), originates its own
    2^24 Zipf-0.9 lookups over all world x rows keys, and stage_probe_sharded answers them in its
    order over RCCL.  This process loads no other HIP runtime or RCCL than libstage_hip's (no
    torch: the control plane is the communicator itself, RcclControl)."""
    shared = share_gpu_rehearsal(rank, world)
    if shared:
        local = 0
    else:
        local = rank_device(local)
    res = cpu_resources()
    nthreads = args.cpu_threads or res["threads"]
    L = stage.lib()
    rccl = stage.rccl_info()
    check(L.stage_set_device(local), "set device")
    total_rows = args.rows * world
    # the CPU leg's table size is fixed before the ranks' host tables exist (MemAvailable then
    # still holds them), for all `world` tables of this node
    cpu_rows = cpu_rows_for(args, res, args.rows, world) if rank == 0 and not args.no_cpu_baseline else 0
    setup = {}
    t0 = time.time()
    keys = owned_keys(total_rows, world, rank)
    setup["owned_keys"] = time.time() - t0
    t0 = time.time()
    tab = stage.Table(key_width=8, device=local)
    loaded = tab.load_keys(keys, 8, mode=0)
    del keys
    setup["load"] = time.time() - t0
    t0 = time.time()
    tab.sync()
    setup["sync"] = time.time() - t0
    log(f"[rank {rank}] loaded {loaded} rows: owned_keys {setup['owned_keys']:.1f}s load {setup['load']:.1f}s "
        f"sync {setup['sync']:.1f}s; RCCL {rccl}")
    if args.out_stride:
        tab.set_output_layout(args.out_stride)
    t0 = time.time()
    ctl = RcclControl(tab, rank, world)
    setup["comm_init"] = time.time() - t0
    # every key is < world x rows: the coalescing sorts read only those bits (same results)
    stage.set_shard_key_bits(tab, max(1, int(total_rows - 1).bit_length()))

    B = args.batch
    stream = stage.Stream()
    draws = stage.zipf_draws(total_rows - 1, args.theta, args.seed + rank, B, nthreads=nthreads)
    d_keys = stage.DeviceBuffer(B * 8)
    check(L.stage_memcpy_h2d(d_keys.ptr, draws.ctypes.data, draws.nbytes, None), "h2d")
    d_out = stage.DeviceBuffer(B * 32)
    d_rec = stage.DeviceBuffer(B * tab.stride)

    def call(reply):
        return L.stage_probe_sharded_ex(tab.h, d_keys.ptr, None, B, d_out.ptr,
                                        None if reply == stage.REPLY_OWNER else d_rec.ptr, reply, stream.ptr)

    # the reply mode of the headline: peer (rows read in place from the owners' exported buffers)
    # unless refused; the library makes every rank agree on a refusal, so all ranks fall back
    # together at the same call
    reply_mode = {"rows": stage.REPLY_ROWS, "peer": stage.REPLY_PEER, "direct": stage.REPLY_DIRECT}.get(
        args.reply, stage.REPLY_PEER if world > 1 else stage.REPLY_ROWS)
    reply_note = None
    if reply_mode in (stage.REPLY_PEER, stage.REPLY_DIRECT):
        rc = call(reply_mode)
        if rc != 0:
            err = L.stage_last_error().decode(errors="replace")
            if args.reply in ("peer", "direct"):
                raise SystemExit(f"[rank {rank}] {args.reply} reply: {err}")
            reply_note = f"peer reply refused, rows over RCCL instead: {err}"
            log(f"[rank {rank}] {reply_note}")
            reply_mode = stage.REPLY_ROWS
        stream.sync()

    def sample_check():
        """8 windows of 8192 lookups spread over the batch (every exchange chunk), each against
        its key's LoadYCSBRows row: (ok, status windows, row windows, key windows)"""
        sample = min(B, 8192)
        outs_w, rows_w, keys_w = [], [], []
        for w in range(8 if B > 8 * sample else 1):
            o = (B - sample) * w // 7 if B > 8 * sample else 0
            outs_w.append(d_out.to_numpy(stage.PROBE_OUT_DTYPE, sample, offset=o * 32))
            rows_w.append(d_rec.to_numpy(np.uint8, sample * tab.stride, offset=o * tab.stride).reshape(sample, tab.stride))
            keys_w.append(draws[o:o + sample])
        outs, rows, kw = np.concatenate(outs_w), np.concatenate(rows_w), np.concatenate(keys_w)
        good = bool((outs["status"] == stage.ST_LATEST).all() and
                    (rows[:, :8].copy().view(np.uint64).ravel() == kw).all() and
                    (rows[:, 8:1008] == (kw & np.uint64(0xFF)).astype(np.uint8)[:, None]).all())
        return good, outs_w, rows_w, keys_w

    def step(reply=None):
        check(call(reply_mode if reply is None else reply), "sharded")

    for _ in range(args.warmup):
        step()
    stream.sync()
    check(L.stage_device_sync(), "sync")
    ctl.barrier()
    evs = [stage.Event() for _ in range(2 * args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        evs[2 * i].record(stream)
        step()
        evs[2 * i + 1].record(stream)
    stream.sync()
    check(L.stage_device_sync(), "sync")
    elapsed = time.perf_counter() - t0
    ctl.barrier()
    elapsed = ctl.max(elapsed)
    kern_ms = float(np.mean([evs[2 * i].elapsed_ms(evs[2 * i + 1]) for i in range(args.steps)]))
    st = stage.sharded_stats_ex(tab)
    # the same steps with STAGE_REPLY_OWNER: rows stay in the owner's HBM, only the 32-B status
    # records return -- the HBM-side scaling without the xGMI tuple return
    for _ in range(max(1, args.warmup)):
        step(stage.REPLY_OWNER)
    stream.sync()
    ctl.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(stage.REPLY_OWNER)
    stream.sync()
    t_own = ctl.max(time.perf_counter() - t0)
    owner = {"value": round(B * args.steps * world / t_own, 1), "ms_per_step": round(t_own / args.steps * 1e3, 4),
             "reply": "32-B status records to the caller, tuple rows materialised on the owner"}
    other_mode = None
    others = {}  # the full-reply modes timed beside the line's, by name
    if reply_mode == stage.REPLY_PEER:  # the same steps with the rows back over RCCL, for comparison
        for _ in range(max(1, args.warmup)):
            step(stage.REPLY_ROWS)
        stream.sync()
        ctl.barrier()
        t0 = time.perf_counter()
        for i in range(args.steps):
            evs[2 * i].record(stream)
            step(stage.REPLY_ROWS)
            evs[2 * i + 1].record(stream)
        stream.sync()
        t_rows = ctl.max(time.perf_counter() - t0)
        kern_rows = float(np.mean([evs[2 * i].elapsed_ms(evs[2 * i + 1]) for i in range(args.steps)]))
        peer_fig = {"value": round(B * args.steps * world / elapsed, 1), "ms_per_step": round(elapsed / args.steps * 1e3, 4),
                    "reply": "status records over RCCL, rows read by the caller from the owners' IPC-mapped buffers"}
        rows_fig = {"value": round(B * args.steps * world / t_rows, 1), "ms_per_step": round(t_rows / args.steps * 1e3, 4),
                    "reply": "status records and rows back over RCCL, fanned out from the receive buffer"}
        # auto: the faster of the two full-reply implementations is the line's value (same
        # results; which one wins depends on the fabric), the other one is reported beside it
        if args.reply == "auto" and t_rows < elapsed:
            reply_mode, elapsed, kern_ms, other_mode = stage.REPLY_ROWS, t_rows, kern_rows, ("peer_reply", peer_fig)
        else:
            other_mode = ("rows_reply", rows_fig)
        others[other_mode[0]] = other_mode[1]
        if args.reply == "auto" and world > 1:
            # and the owners writing into the callers' outputs (STAGE_REPLY_DIRECT): timed, then
            # checked on the sample windows; the line takes it only when every rank's check passed
            d_out.memset(0)  # the check must see what the direct reply wrote (owners write only after
            d_rec.memset(0)  # this rank's keys reached them, i.e. after these fills)
            direct_rc = call(stage.REPLY_DIRECT)
            stream.sync()
            direct_ok = direct_rc == 0 and sample_check()[0]
            if direct_rc != 0:
                log(f"[rank {rank}] direct reply refused: {L.stage_last_error().decode(errors='replace')}")
            if ctl.max(0.0 if direct_ok else 1.0) == 0.0:
                for _ in range(max(1, args.warmup)):
                    step(stage.REPLY_DIRECT)
                stream.sync()
                ctl.barrier()
                t0 = time.perf_counter()
                for i in range(args.steps):
                    evs[2 * i].record(stream)
                    step(stage.REPLY_DIRECT)
                    evs[2 * i + 1].record(stream)
                stream.sync()
                t_dir = ctl.max(time.perf_counter() - t0)
                kern_dir = float(np.mean([evs[2 * i].elapsed_ms(evs[2 * i + 1]) for i in range(args.steps)]))
                direct_fig = {"value": round(B * args.steps * world / t_dir, 1),
                              "ms_per_step": round(t_dir / args.steps * 1e3, 4),
                              "reply": "owners write each remote row into the caller's IPC-mapped output, the "
                                       "caller copies duplicates; 16-B tokens over RCCL"}
                if t_dir < elapsed:
                    mine = ("peer_reply" if reply_mode == stage.REPLY_PEER else "rows_reply",
                            {"value": round(B * args.steps * world / elapsed, 1),
                             "ms_per_step": round(elapsed / args.steps * 1e3, 4),
                             "reply": peer_fig["reply"] if reply_mode == stage.REPLY_PEER else rows_fig["reply"]})
                    others[mine[0]] = mine[1]
                    reply_mode, elapsed, kern_ms = stage.REPLY_DIRECT, t_dir, kern_dir
                else:
                    others["direct_reply"] = direct_fig
            else:
                others["direct_reply"] = {"note": "not timed: refused or its sample check failed on some rank"}
    direct = None
    if world == 1:  # the one-rank rehearsal against the direct probe of the same batch on the same table
        for _ in range(max(1, args.warmup)):
            tab.probe_device(d_keys.ptr, B, d_out.ptr, d_rec.ptr, stream=stream.ptr)
        stream.sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            tab.probe_device(d_keys.ptr, B, d_out.ptr, d_rec.ptr, stream=stream.ptr)
        stream.sync()
        direct = round((time.perf_counter() - t0) / args.steps * 1e3, 4)
    d_out.memset(0)  # the self-check reads what the line's mode writes, not an earlier mode's rows
    d_rec.memset(0)
    step()  # full reply again, so the self-check reads full rows
    stream.sync()
    ok, outs_w, rows_w, keys_w = sample_check()
    c2_check = (draws[:4096].copy(), outs_w[0]["status"][:4096].copy(), rows_w[0][:4096].copy())
    reports = ctl.gather(rank_report(rank, loaded, setup, ok) + [float(st[k]) for k in
                                                                   ("keys", "routed", "remote", "received")])
    for b in (d_keys, d_out, d_rec):
        b.free()
    ctl.barrier()
    ctl.close()
    if rank != 0:
        return 0 if ok else 1
    per_rank = per_rank_reports(reports[:, :len(RANK_REPORT)])
    stats = [dict(zip(("keys", "routed", "remote", "received"), (int(x) for x in r[len(RANK_REPORT):])))
             for r in reports]
    for p, sx in zip(per_rank, stats):
        p["requests"] = sx
    step_s = elapsed / args.steps
    # HBM roofline of the step: the bytes that move on each rank (owners' probes, caller rows,
    # result copies), the busiest rank over the step time
    hb = [sharded_hbm_bytes(sx, tab.stride, peer=reply_mode == stage.REPLY_PEER, direct=reply_mode == stage.REPLY_DIRECT)
          for sx in stats]
    hmax = max(b for b, _ in hb)
    hbm = {"bound": "hbm", "achieved": round(hmax / step_s / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(hmax / step_s / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
           "kernel": "sharded step: owners' probes (fan-out for own requests) + result returns + fan-out copies",
           "algorithmic_bytes_per_launch": hmax, "bytes_by_part_rank0": hb[0][1],
           "avg_launch_ms": round(step_s * 1e3, 4), "event_ms_per_step_rank0": round(kern_ms, 4),
           "algorithmic_bytes": "bench.sharded_hbm_bytes (per rank, what moves)"}
    if shared:  # the exchange ran over host sockets: no xGMI figure to price it against
        roof = dict(hbm, note="ranks share one GPU (rehearsal): HBM bytes of the busiest rank, all ranks' "
                              "kernels contend for the same HBM")
    elif world > 1:
        roof = xgmi_roofline(B, world, tab.stride, step_s, hbm, remote=max(sx["remote"] for sx in stats))
    else:
        roof = hbm
    cpu = cpu_leg_sharded(args, res, world, nthreads, cpu_rows, args.rows, c2_check)
    routed = sum(sx["routed"] for sx in stats)
    result = {
        "metric": METRIC, "value": round(B * args.steps * world / elapsed, 1), "unit": "ops/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic (LoadYCSBRows keys/payloads)",
        "config": {"workload": sharded_workload(world, args.rows, shared), "theta": args.theta, "traversal": "device",
                   "rows_per_gpu": args.rows, "rows_total": total_rows, "batch_per_gpu": B, "key_bytes": 8,
                   "payload_bytes": 1000, "leaf_bytes": 65536, "parallelism": f"hash-shard x{world}",
                   "exchange_chunks": int(os.environ.get("STAGE_SHARD_CHUNKS", 4 if world > 1 else 1)),
                   "control_plane": "the RCCL communicator (file rendezvous of the unique id)"},
        "roofline": roof, "cpu_baseline": cpu, "self_check": all(p["self_check"] for p in per_rank),
        "reply": {stage.REPLY_PEER: "peer", stage.REPLY_ROWS: "rows", stage.REPLY_DIRECT: "direct"}[reply_mode],
        **({"reply_note": reply_note} if reply_note else {}),
        **others,
        "owner_reply": owner,
        **({"world1_vs_direct": {"sharded_ms_per_step": round(step_s * 1e3, 4), "owner_reply_ms_per_step":
                                 owner["ms_per_step"], "direct_probe_ms_per_step": direct,
                                 "note": "same table and batch: stage_probe_sharded_ex at world 1 (coalescing, "
                                         "routing, fan-out probe) vs stage_probe_batch"}} if direct else {}),
        "coalescing": {"keys": sum(sx["keys"] for sx in stats), "requests_routed": routed,
                       "remote_requests": sum(sx["remote"] for sx in stats),
                       "routed_share": round(routed / max(1, sum(sx["keys"] for sx in stats)), 4),
                       "note": "equal (key, read id) requests of the batch travel and are probed once, whatever exchange chunk they fall in; own requests are "
                               "probed straight into their caller positions (fan-out probe)"},
        "rccl": rccl, "per_rank": per_rank,
        "setup_s": {k: round(max(p["setup_s"][k] for p in per_rank), 2) for k in per_rank[0]["setup_s"]},
        "host_peak_rss_gib": max(p["host_peak_rss_gib"] for p in per_rank),
    }
    print(json.dumps(result), flush=True)
    return 0 if result["self_check"] else 1


def traffic_from_profile(batch, rows, name="pmc_probe.json"):
    """Per-launch HBM bytes of the dominant kernel from a committed rocprofv3 --pmc pass (see
    profiles/README.md), if one exists for this configuration."""
    path = os.path.join(REPO, "profiles", name)
    if not os.path.exists(path):
        return None, None
    try:
        d = json.load(open(path))
        if d.get("batch") == batch and d.get("rows") == rows:
            src = os.path.relpath(path, REPO)
            prof = d.get("profiled")
            if prof:  # where the counter pass ran: another box / tree than this run's
                src += f" (profiled on {prof.get('host')} {prof.get('date')}, tree {prof.get('tree')})"
            return d["hbm_bytes_per_launch"], src
    except Exception:
        pass
    return None, None


def cpu_name():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def _read(path):
    try:
        return open(path).read().strip()
    except OSError:
        return None


def cpu_resources():
    """What this process may use: affinity CPUs, the cgroup CPU quota (cpu.max), host memory
    (MemTotal / MemAvailable) and the cgroup memory limit (memory.max)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    q = _read("/sys/fs/cgroup/cpu.max")
    if q and not q.startswith("max"):
        a, b = q.split()[:2]
        quota = max(1, int(math.floor(int(a) / int(b))))
    mem = {}
    for line in (_read("/proc/meminfo") or "").splitlines():
        k, v = line.split(":", 1)
        mem[k] = int(v.split()[0]) * 1024
    cg = _read("/sys/fs/cgroup/memory.max")
    cg_mem = int(cg) if cg and cg.isdigit() else None
    threads = min(aff, quota) if quota else aff
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpus": quota, "threads": threads,
            "cpu_model": cpu_name(), "mem_total_gib": round(mem.get("MemTotal", 0) / 2**30, 1),
            "mem_available_gib": round(mem.get("MemAvailable", 0) / 2**30, 1),
            "cgroup_mem_gib": round(cg_mem / 2**30, 1) if cg_mem else None,
            "_avail": min(x for x in (mem.get("MemAvailable", 0), cg_mem, 250 * 2**30) if x)}


def cpu_rows_for(args, res, gpu_rows, world=1):
    """Largest oracle table (rows) that fits beside the host memory of the `world` ranks' device
    tables on this node, <= one GPU's N."""
    if args.cpu_rows:
        return args.cpu_rows
    budget = res["_avail"] - 24 * 2**30 - world * gpu_rows * GPU_HOST_BYTES_PER_ROW
    fit = int(budget // ORACLE_BYTES_PER_ROW) // 1_000_000 * 1_000_000
    return max(1_000_000, min(gpu_rows, fit))


def xgmi_roofline(batch, world, stride, step_s, hbm_roof, remote=None):
    """Roofline of the multi-GPU step, bound by the xGMI exchange: per rank and step every
    remote request sends its 16-B key record out and gets a 32-B status record + a stride-byte
    row back; peak = the W-1 links a rank uses.  remote = the requests this rank routed to other
    ranks (after coalescing, stage_sharded_stats); default the hash-uniform (W-1)/W of the batch."""
    if remote is None:
        remote = batch * (world - 1) / world
    unit = 16 + 32 + stride
    achieved = remote * unit / step_s / 1e9
    peak = XGMI_LINK_GBS * (world - 1)
    return {"bound": "xgmi", "achieved": round(achieved, 1), "peak": peak, "unit": "GB/s",
            "frac": round(achieved / peak, 4), "traffic": None,
            "kernel": "sharded step (coalesce + route + RCCL all-to-all-v + probe_kernel + fan-out)",
            "algorithmic_bytes_per_unit": unit, "units_per_launch": round(remote),
            "avg_launch_ms": round(step_s * 1e3, 4),
            "peak_source": f"{XGMI_LINK_GBS:.0f} GB/s per xGMI link (7 per MI355X), {world - 1} links per rank",
            "hbm": hbm_roof}


def fmt_rows(n):
    """100000000 -> '100M' (the BASELINE.json spelling of row counts)"""
    for div, suf in ((10**9, "B"), (10**6, "M"), (10**3, "K")):
        if n % div == 0:
            return f"{n // div}{suf}"
    return str(n)


def sharded_workload(world, rows_per_gpu, shared=False):
    """config.workload of a sharded run, naming its real world size and rows: at 8 ranks of
    100M rows this is BASELINE.json configs[4] verbatim; any other world / size names itself."""
    if shared:
        return (f"YCSB-C {fmt_rows(world * rows_per_gpu)} rows sharded {world} ways, RCCL all-to-all key routing "
                f"over its socket transport, {world} ranks sharing 1×MI355X (multi-rank rehearsal, "
                f"{SHARE_GPU_ENV}=1; not an xGMI or scaling point)")
    s = (f"YCSB-C {fmt_rows(world * rows_per_gpu)} rows sharded {world} way{'s' if world != 1 else ''}, "
         f"RCCL all-to-all key routing over xGMI, {world}×MI355X")
    if world == 1:
        s += " (one-rank rehearsal of the multi-GPU path, --force-sharded)"
    return s


def sharded_hbm_bytes(st, stride, row_bytes=1008, peer=False, direct=False):
    """Algorithmic HBM bytes of one sharded step on one rank, counting what actually moves
    (stage_sharded_stats_ex after the step: n caller keys, `routed` requests after coalescing,
    `remote` of them owned by other ranks, `received` requests this rank probed as owner):
      owner probes      received x (8 key + 64 fingerprint line + 16 slot word + 1000 payload)
      caller rows       n x (row_bytes + 4): every caller position's row + status (as C2)
      remote results    (received - own) x 2 x (row_bytes + 4): written for the return, read by RCCL
      returned results  remote x 2 x (row_bytes + 4): written by RCCL, read by the fan-out
      key records       (remote + received - own) x 2 x 16: sent (read) and received (written)
    Peer reply (STAGE_REPLY_PEER): the remote results are written once into this rank's exported
    row buffer and read once by the requesting rank's fan-out (from this rank's HBM, over the
    fabric) -- the same 2 x per row here; the returned results are only status records
    (remote x 2 x 32), their rows are read from the owners' HBM.
    Direct reply (STAGE_REPLY_DIRECT): the owner writes each remote result once, straight into its
    caller's output (counted there, in caller_rows) -- no result buffers, no returned rows; the
    caller reads the first position's row once per duplicate caller of a remote request, estimated
    as the batch's duplicates (n - routed) in the remote share of the requests.
    The coalescing sorts and the routing's own scratch traffic are not counted (not algorithmic)."""
    n, routed, remote, received = st["keys"], st["routed"], st["remote"], st["received"]
    own = routed - remote
    recv_remote = received - own
    out = row_bytes + 4
    if direct:
        parts = {"owner_probes": received * (8 + 64 + 16 + 1000), "caller_rows": n * out,
                 "duplicate_reads": round((n - routed) * remote / max(routed, 1)) * out,
                 "key_records": (remote + recv_remote) * 32}
        return sum(parts.values()), parts
    parts = {"owner_probes": received * (8 + 64 + 16 + 1000), "caller_rows": n * out,
             "remote_results": recv_remote * 2 * out, "returned_results": remote * 2 * (32 if peer else out),
             "key_records": (remote + recv_remote) * 32}
    return sum(parts.values()), parts


def hbm_roofline(per_unit, units_per_launch, kern_ms, kernel, traffic=None, tsrc=None):
    achieved = per_unit * units_per_launch / (kern_ms * 1e-3) / 1e9
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": kernel,
            "algorithmic_bytes_per_unit": round(per_unit, 2), "units_per_launch": units_per_launch,
            "algorithmic_bytes_per_launch": round(per_unit * units_per_launch),
            "avg_launch_ms": round(kern_ms, 4)}
    if traffic:
        roof["traffic_source"] = tsrc
        roof["traffic_over_algorithmic"] = round(traffic / (per_unit * units_per_launch), 4)
    return roof


class YcsbB:
    """configs[2]: YCSB-B epochs.  Each epoch is the update share of a batch applied on the
    write path (LeafNode::Update + CommitTransaction UPDATE entry, read / commit ids from one
    counter as tid_counter does) -- on the device (stage_update_batch_device) or on the host
    (stage_update_batch + incremental publish) -- and its read share with read ids: 75 %
    current, 25 % drawn from the last --reader-window ids (readers concurrent with the newest
    writers: older snapshots a few commits back).  A share of the
    update ops (--inflight-share, keys beyond the 10^4 hottest) stays in flight (commit id 0),
    so later reads of those keys take the overwrite-copy (COPY) branch.
    Epochs are generated and their inputs uploaded to HBM before the timed loop (like the C2
    keys); every epoch is recorded so the CPU leg can replay it on the oracle."""

    def __init__(self, tab, args, nthreads, theta):
        self.tab, self.args, self.nthreads, self.theta = tab, args, nthreads, theta
        self.counter = 1
        self.epoch = 0
        self.record = []

    def make_epoch(self):
        a = self.args
        draws = stage.zipf_draws(a.rows - 1, self.theta, a.seed + 1000 * self.epoch, a.batch, nthreads=self.nthreads)
        rng = np.random.default_rng(a.seed + self.epoch)
        # RunMixed's op stream (ycsb_mixed.cpp:26-44): NextUniform() < update_ratio makes an
        # update whose 100-B delta is memset to the next_char() drawn right after it
        is_upd, chr_ = stage.ycsb_ops(a.seed * 1_000_003 + self.epoch, a.batch, a.update_ratio)
        keys = draws[is_upd]
        m = keys.size
        rid = (self.counter + 2 * np.arange(m, dtype=np.uint64)).astype(np.uint32)
        cid = rid + np.uint32(1)
        cand = np.nonzero(keys > 10_000)[0]
        k_in = min(cand.size, int(round(a.inflight_share * m)))
        if k_in:
            cid[rng.choice(cand, k_in, replace=False)] = 0  # left in flight
        self.counter += 2 * m
        colb = np.ascontiguousarray(chr_[is_upd])
        reads = np.ascontiguousarray(draws[~is_upd])
        rids = np.full(reads.size, self.counter, np.uint32)
        old = rng.random(reads.size) < a.old_share
        # an older snapshot is a reader running beside the writers (RunMixed's threads): its id
        # trails the newest commit by at most the ids its concurrent transactions take, not by
        # the whole run -- with RunMixed's update stream every update adds a version, so a hot
        # key's chain grows by ~10^4 per epoch and a reader at a random historical id would walk it
        win = max(2, min(self.counter, a.reader_window))
        rids[old] = (self.counter - rng.integers(1, win, int(old.sum()))).astype(np.uint32)
        ep = {"keys": keys, "colb": colb, "rid": rid, "cid": cid, "inflight": int(k_in), "reads": reads, "rids": rids}
        self.record.append(ep)
        self.epoch += 1
        return ep

    def upload(self, ep):
        """the epoch's inputs into HBM: update keys, 100-B column patches, ids; read keys, ids"""
        cols = np.repeat(ep["colb"], 100)
        ep["d"] = {k: stage.DeviceBuffer.from_numpy(x) for k, x in
                   (("keys", ep["keys"]), ("cols", cols), ("rid", ep["rid"]), ("cid", ep["cid"]),
                    ("reads", ep["reads"]), ("rids", ep["rids"]))}
        ep["d"]["rc"] = stage.DeviceBuffer(max(1, ep["keys"].size))
        ep["d"]["out"] = stage.DeviceBuffer(32 * ep["reads"].size)

    def apply(self, ep, stream=None):
        """the epoch's write share on the write path; returns the successful updates.  With a
        stream (device write path) the kernels are only enqueued on it -- no host wait; the
        successes are counted afterwards from the per-op return codes (count_ok)."""
        m = ep["keys"].size
        if self.args.write_path == "device":
            ok = ctypes.c_uint64()
            if m:
                d = ep["d"]
                check(stage.lib().stage_update_batch_device(self.tab.h, d["keys"].ptr, None, m, 0, d["cols"].ptr, 100,
                                                            d["rid"].ptr, d["cid"].ptr, None, d["rc"].ptr,
                                                            None if stream is not None else ctypes.byref(ok),
                                                            stream.ptr if stream is not None else None),
                      "update_batch_device")
            return ok.value
        # host write path: LeafNode::Update + commit on the host table, then the incremental
        # publish of the touched leaves (stage_update_batch + stage_sync)
        cols = np.repeat(ep["colb"][:, None], 100, 1)
        ep["rc_host"], ok = self.tab.update_batch(ep["keys"], 0, cols, ep["rid"], ep["cid"])
        self.tab.sync()
        return ok

    RC_NAMES = {stage.RC_OK: "ok", stage.RC_NOT_NEEDED_UPDATE: "not_needed_update", stage.RC_DIRTY: "dirty",
                stage.RC_NOT_FOUND: "not_found", stage.RC_INVALID: "invalid"}

    @staticmethod
    def rc_counts(ep):
        """the epoch's update return codes by name (LeafNode::Update's ReturnCode)"""
        m = ep["keys"].size
        if not m:
            return {}
        rc = ep["rc_host"] if "rc_host" in ep else ep["d"]["rc"].to_numpy(np.uint8, m)
        v, c = np.unique(rc, return_counts=True)
        return {YcsbB.RC_NAMES.get(int(x), f"rc{int(x)}"): int(k) for x, k in zip(v, c)}

    @staticmethod
    def count_ok(ep):
        """successful updates of an epoch applied on the device (return code RC_OK)"""
        m = ep["keys"].size
        return int((ep["d"]["rc"].to_numpy(np.uint8, m) == stage.RC_OK).sum()) if m else 0

    def release(self, ep):
        for b in ep.pop("d", {}).values():
            b.free()


class CpuOracle:
    """The CPU leg's oracle table (test oracle = the reference path restated in C), built in a
    background thread while the GPU leg runs: LoadYCSBRows of `rows` rows with the single
    loader's leaves (orc_load_ycsb_parallel)."""

    def __init__(self, rows, threads):
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_lib as O  # the checker, timed here as the reference CPU path
        self.O = O
        self.rows, self.threads = rows, threads
        self.tree = None
        self.build_s = None
        self.err = None
        self.th = threading.Thread(target=self._build, daemon=True)
        self.th.start()

    def _build(self):
        try:
            t0 = time.time()
            t = self.O.OracleTree()
            t.load_ycsb_parallel(0, self.rows, 8, 0, self.threads)
            self.tree = t
            self.build_s = time.time() - t0
        except Exception as e:  # reported in the result line
            self.err = repr(e)

    def wait(self):
        self.th.join()
        if self.err:
            raise RuntimeError(f"oracle build failed: {self.err}")
        return self.tree


def cpu_sample_count(rate, seconds, lo, hi):
    return int(min(max(rate * seconds, lo), hi))


def cpu_calibration(O, threads):
    """The port against the reference's own numbers: C1 (1000 rows, 4-byte
    keys, 10 reads/txn, 1 thread, full-txn) and 1-thread BTree::Read + copy at 1M rows."""
    t = O.OracleTree()
    t.load_ycsb(0, 1000, 4, 0)
    keys = np.random.default_rng(1).integers(0, 1000, 1_000_000).astype(np.uint64)
    sec, com, ab, _ = t.ycsb_txn_timed(keys, 4, 10, 1)
    c1 = keys.size / sec
    del t
    t = O.OracleTree()
    t.load_ycsb_parallel(0, 1_000_000, 4, 0, threads)
    keys = np.random.default_rng(2).integers(0, 1_000_000, 1_000_000).astype(np.uint64)
    s = ctypes.c_double()
    O.lib().orc_read_batch_timed(t.t, keys.ctypes.data, 4, None, keys.size, 1, ctypes.byref(s))
    ns = s.value / keys.size * 1e9
    sec, _, _, _ = t.ycsb_txn_timed(keys, 4, 10, 1)
    txn_ops = keys.size / sec
    del t
    return {"c1_full_txn_ops_s": round(c1, 1), "c1_aborts": ab, "c1_vs_reference_1533428": round(c1 / REF_C1_OPS, 3),
            "read_ns_1m_1thread": round(ns, 1), "read_vs_reference_1786ns": round(REF_READ_NS_1M / ns, 3),
            "txn_ops_s_1m_1thread": round(txn_ops, 1), "txn_vs_reference_428817": round(txn_ops / REF_TXN_OPS_1M, 3),
            "note": "reference numbers were measured on the survey container (8-core Xeon); ratios > 1 = the port "
                    "is faster on this host; BASELINE.md §3 has the same-host ratios"}


def cpu_legs(orc, args, res, threads, c2_check=None, c4_check=None, c3=None, legs=("c2", "c4", "c3")):
    """Times the oracle on the GPU box's host cores: C2 lookup mode + full-txn mode, C4 scans,
    C3 reads on the replayed epochs' snapshot with the GPU's read ids; checks GPU samples
    against it (the oracle is the checker).  Returns {leg: cpu_baseline dict}."""
    O = orc.O
    tree = orc.wait()
    n = orc.rows
    L = O.lib()
    secs = ctypes.c_double()
    out = {}
    host = {k: v for k, v in res.items() if not k.startswith("_")}
    common = {"cores": threads, "threads": threads, "kind": "port", "rows": n, "host": host,
              "build_s": round(orc.build_s, 1)}
    # C2, lookup mode
    keys = stage.zipf_draws(n - 1, 0.9, args.seed, 400_000, nthreads=threads)
    L.orc_read_batch_timed(tree.t, keys.ctypes.data, 8, None, keys.size, threads, ctypes.byref(secs))
    count = cpu_sample_count(keys.size / max(secs.value, 1e-9), args.cpu_seconds, 100_000, 400_000_000)
    keys = stage.zipf_draws(n - 1, 0.9, args.seed + 1, count, nthreads=threads)
    L.orc_read_batch_timed(tree.t, keys.ctypes.data, 8, None, keys.size, threads, ctypes.byref(secs))
    c2 = {"value": round(count / secs.value, 1), "unit": "ops/s", "mode": "lookup", **common,
          "sample": f"oracle BTree::Read + executor copy, {count} zipf-0.9 lookups over {n} rows (8-B keys, "
                    f"1000-B payload), {threads} threads on {res['cpu_model']}, {secs.value:.1f}s"}
    # C2, full-txn mode (RunMixed read-only transactions of 10 reads, Index-SSN read side)
    keys = stage.zipf_draws(n - 1, 0.9, args.seed + 2, 400_000, nthreads=threads)
    sec, com, ab, _ = tree.ycsb_txn_timed(keys, 8, 10, threads)
    count = cpu_sample_count(keys.size / max(sec, 1e-9), args.cpu_seconds * 0.6, 100_000, 200_000_000) // 10 * 10
    keys = stage.zipf_draws(n - 1, 0.9, args.seed + 3, count, nthreads=threads)
    sec, com, ab, _ = tree.ycsb_txn_timed(keys, 8, 10, threads)
    c2["full_txn"] = {"value": round(count / sec, 1), "unit": "ops/s", "commits": com, "aborts": ab,
                      "sample": f"{count // 10} read-only RunMixed txns x 10 reads (PerformRead rw-set, "
                                f"CommitTransaction FindMinSstamp/FindMaxPstamp, active_tids), {sec:.1f}s"}
    if c2_check is not None:
        ck, st, rows = c2_check
        sel = ck < n
        o_out, o_rec = tree.read_batch(ck[sel], 8, nthreads=threads)
        c2["gpu_check"] = {"compared": int(sel.sum()),
                           "equal": bool((o_out["status"] == st[sel]).all() and
                                         (rows[sel][:, :tree.row] == o_rec).all())}
    out["c2"] = c2
    if "c4" not in legs:
        return out
    # C4, scan mode (TableScanExecutor over RangeScanBySize/Iterator)
    # the first short sample runs cold (its rate underestimates the steady one), so the sample
    # is re-sized until it lasts at least 0.6 of its target time
    target = args.cpu_seconds * 0.6
    count = 20_000
    for attempt in range(4):
        starts = (stage.fastrandom(args.seed + attempt, count) % np.uint64(n)).astype(np.uint64)
        L.orc_scan_batch_timed(tree.t, starts.ctypes.data, 8, starts.size, args.scan_size, threads, ctypes.byref(secs))
        if attempt and (secs.value >= 0.6 * target or count >= 20_000_000):
            break
        count = cpu_sample_count(count / max(secs.value, 1e-9), target, 10_000, 20_000_000)
    count = starts.size
    c4 = {"value": round(count / secs.value, 1), "unit": "scans/s", "mode": "scan", **common,
          "sample": f"oracle TableScanExecutor over Iterator, {count} scans of {args.scan_size} over {n} rows, "
                    f"{threads} threads, {secs.value:.1f}s"}
    if c4_check is not None:
        ck, cnt, recs = c4_check
        sel = np.nonzero(ck < n)[0][:256]
        oc, orows = tree.scan_batch(ck[sel], 8, args.scan_size, nthreads=threads)
        # scans near the top of a smaller CPU table stop earlier: compare the common prefix
        eq = all((orows[i, :min(oc[i], cnt[j]), :tree.row] == recs[j, :min(oc[i], cnt[j]), :tree.row]).all()
                 for i, j in enumerate(sel))
        c4["gpu_check"] = {"compared": int(sel.size), "equal": bool(eq)}
    out["c4"] = c4
    # C3: replay the GPU's epochs on the oracle, then the last epoch's reads with its read ids
    if c3 is not None:
        t0 = time.time()
        applied = 0
        upd_s, upd_ops, upd_n = 0.0, 0, 0
        record = c3["record"]
        for i, ep in enumerate(record):
            sel = ep["keys"] < n
            deltas = np.repeat(ep["colb"][sel][:, None], 100, 1)
            if i + 1 < len(record):  # earlier epochs: the snapshot the timed epoch starts from
                _, ok = tree.update_batch(ep["keys"][sel], 8, 0, deltas, ep["rid"][sel], ep["cid"][sel])
            else:  # the timed epoch: RunMixed's writers run concurrently (LeafNode::Update CASes)
                _, ok, upd_s = tree.update_batch_mt(ep["keys"][sel], 8, 0, deltas, ep["rid"][sel], ep["cid"][sel],
                                                    threads)
                upd_ops, upd_n = int(ok), int(sel.sum())
            applied += ok
        replay_s = time.time() - t0 - upd_s
        reads, rids = c3["reads"], c3["rids"]
        sel = reads < n
        reads, rids = np.ascontiguousarray(reads[sel]), np.ascontiguousarray(rids[sel])
        L.orc_read_batch_timed(tree.t, reads.ctypes.data, 8, rids.ctypes.data, reads.size, threads,
                               ctypes.byref(secs))
        # value: the last epoch's reads and its successful updates, each on T threads (the
        # updates on T concurrent writers, each key's ops on one writer in order), over the
        # summed times -- the GPU's C3 value counts the same two shares over its whole loop
        c3o = {"value": round((reads.size + upd_ops) / (secs.value + upd_s), 1), "unit": "ops/s",
               "mode": "lookup at read ids + the last epoch's updates", **common,
               "reads_per_s": round(reads.size / secs.value, 1),
               "updates_per_s": round(upd_ops / max(upd_s, 1e-9), 1),
               "last_epoch_update_ops": upd_n, "last_epoch_updates_ok": upd_ops,
               "last_epoch_update_s": round(upd_s, 4), "update_writers": threads,
               "updates_replayed": applied, "replay_s_untimed": round(replay_s, 1),
               "sample": f"oracle BTree::Read + visibility (latest / copy / TupleHeader chain) + copy, the GPU's "
                         f"last-epoch reads and read ids ({reads.size}) on the same snapshot, and that epoch's "
                         f"{upd_n} update ops (LeafNode::Update + commit) on {threads} concurrent writers "
                         f"({len(record)} epochs replayed), {threads} threads, {secs.value + upd_s:.1f}s"}
        if c3.get("check") is not None:
            ck_keys, ck_rids, st, rows = c3["check"]
            s2 = ck_keys < n
            o_out, o_rec = tree.read_batch(ck_keys[s2], 8, ck_rids[s2], nthreads=threads)
            c3o["gpu_check"] = {"compared": int(s2.sum()), "snapshot_equal_rows": bool(n == args.rows),
                                "equal": bool((o_out["status"] == st[s2]).all() and
                                              (rows[s2][:, :tree.row] == o_rec).all())}
        out["c3"] = c3o
    return out


def tpcc_tables(args, seed=7):
    """DISTRICT / ORDER_LINE / STOCK rows with the reference's key and payload layouts
    (tpcc_record.h), generated vectorised: W warehouses x 10 districts x 3000 orders of 5..15
    lines, `items` stock rows per warehouse.  First payload columns: D_NEXT_O_ID, OL_I_ID,
    S_QUANTITY (int32)."""
    rng = np.random.default_rng(seed)
    W, I, D, O = args.warehouses, args.items, 10, 3000
    out = {}
    wi = np.stack(np.meshgrid(np.arange(1, W + 1), np.arange(1, I + 1), indexing="ij"), -1).reshape(-1, 2)
    sk = np.ascontiguousarray(wi.astype(np.int64)).view(np.uint8).reshape(-1, 16)
    sp = rng.integers(0, 256, (sk.shape[0], 400), dtype=np.uint8)
    sp[:, :4] = rng.integers(10, 101, sk.shape[0]).astype(np.int32).view(np.uint8).reshape(-1, 4)
    out["stock"] = (sk, sp)
    wd = np.stack(np.meshgrid(np.arange(1, W + 1), np.arange(1, D + 1), indexing="ij"), -1).reshape(-1, 2)
    dk = np.ascontiguousarray(wd.astype(np.int64)).view(np.uint8).reshape(-1, 16)
    dp = rng.integers(0, 256, (dk.shape[0], 143), dtype=np.uint8)
    dp[:, :4] = np.full(dk.shape[0], O + 1, np.int32).view(np.uint8).reshape(-1, 4)
    out["district"] = (dk, dp)
    wdo = np.stack(np.meshgrid(np.arange(1, W + 1), np.arange(1, D + 1), np.arange(1, O + 1), indexing="ij"),
                   -1).reshape(-1, 3)
    nl = rng.integers(5, 16, wdo.shape[0])
    rep = np.repeat(wdo, nl, axis=0)
    ln = np.arange(rep.shape[0]) - np.repeat(np.cumsum(nl) - nl, nl) + 1
    ok = np.ascontiguousarray(np.concatenate([rep, ln[:, None]], 1).astype(np.int64)).view(np.uint8).reshape(-1, 32)
    op = rng.integers(0, 256, (ok.shape[0], 60), dtype=np.uint8)
    op[:, :4] = rng.integers(1, I + 1, ok.shape[0]).astype(np.int32).view(np.uint8).reshape(-1, 4)
    out["order_line"] = (ok, op)
    return out


def run_tpcc(args):
    """TPC-C stock-level through the path (stage_tpcc_stock_level), one GPU."""
    L = stage.lib()
    t0 = time.time()
    data = tpcc_tables(args)
    gen_s = time.time() - t0
    widths = {"district": (16, 143), "order_line": (32, 60), "stock": (16, 400)}
    tabs = {}
    t0 = time.time()
    for name, (k, p) in data.items():
        t = stage.Table(payload_size=widths[name][1], key_width=widths[name][0])
        _, ins = t.load_rows(k, p)
        assert ins == k.shape[0]
        tabs[name] = t
    load_s = time.time() - t0
    t0 = time.time()
    for t in tabs.values():
        t.sync()
    sync_s = time.time() - t0
    B = args.batch
    rng = np.random.default_rng(args.seed)
    w = rng.integers(1, args.warehouses + 1, B).astype(np.int64)
    d = rng.integers(1, 11, B).astype(np.int64)
    thr = rng.integers(10, 21, B).astype(np.int32)  # stock_min/max_threshold
    dw, dd, dt = (stage.DeviceBuffer.from_numpy(x) for x in (w, d, thr))
    dres = stage.DeviceBuffer(4 * B)
    stream = stage.Stream()

    def step():
        check(L.stage_tpcc_stock_level(tabs["district"].h, tabs["order_line"].h, tabs["stock"].h, dw.ptr, dd.ptr,
                                       dt.ptr, None, B, dres.ptr, stream.ptr), "stock level")

    for _ in range(args.warmup):
        step()
    stream.sync()
    t0 = time.perf_counter()
    ev0, ev1 = stage.Event(), stage.Event()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    stream.sync()
    elapsed = time.perf_counter() - t0
    ms = ev0.elapsed_ms(ev1) / args.steps
    res = dres.to_numpy(np.int32, B)
    value = B * args.steps / elapsed
    # algorithmic bytes per transaction (what the fused transaction must touch; no tuple is
    # materialised): a point probe reads key + 64 (fingerprint line) + 32 (slot word) + 64 (the
    # sector holding the column it needs); a 10-record scan reads its 32-B start key, the key
    # words + slot word of the <= 11 records RangeScanBySize collects, and one 64-B sector of the
    # tuple it keeps; plus 4 B result
    probe = lambda kb: kb + 64 + 32 + 64
    per_txn = probe(16) + 20 * (32 + 11 * (32 + 32) + 64) + 20 * probe(16) + 4
    achieved = per_txn * B / (ms * 1e-3) / 1e9
    cpu = None
    if not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_lib as O
        t1 = time.time()
        orcs = {}
        for name, (k, p) in data.items():
            o = O.OracleTree(payload_size=widths[name][1], key_pad=widths[name][0])
            o.load_rows(k, p)
            orcs[name] = o
        build = time.time() - t1
        threads = args.cpu_threads or cpu_resources()["threads"]
        n0 = 20_000
        r0, sec = O.stock_level_batch(orcs["district"], orcs["order_line"], orcs["stock"], w[:n0], d[:n0], thr[:n0],
                                      None, threads)
        assert (r0 == res[:n0]).all(), "stock-level results differ from the oracle"
        n1 = int(min(B, max(n0, n0 / max(sec, 1e-9) * args.cpu_seconds)))
        r1, sec = O.stock_level_batch(orcs["district"], orcs["order_line"], orcs["stock"], w[:n1], d[:n1], thr[:n1],
                                      None, threads)
        cpu = {"value": round(n1 / sec, 1), "unit": "txns/s", "cores": threads, "kind": "port",
               "sample": f"oracle orc_stock_level (DISTRICT read, 20 IndexScanExecutor range scans, STOCK reads), "
                         f"{n1} txns, same tables (build {build:.1f}s), {threads} threads on {cpu_name()}, {sec:.1f}s"}
        del orcs
    result = {
        "metric": "TPC-C stock-level txns/s through the index-organized path (supplementary to "
                  + METRIC + ")",
        "value": round(value, 1), "unit": "txns/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int64 keys / bytes", "data": "synthetic TPC-C rows (tpcc_record.h layouts)",
        "config": {"workload": "TPC-C stock-level (tpcc_stock_level.cpp), batched", "warehouses": args.warehouses,
                   "items": args.items, "districts_per_wh": 10, "orders_per_district": 3000,
                   "order_lines": int(data["order_line"][0].shape[0]), "txns_per_step": B,
                   "aborted": int((res < 0).sum()), "mean_low_stock": round(float(res[res >= 0].mean()), 3)},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel": "stock-level step (district probe + 20 index scans + 20 stock probes)",
                     "algorithmic_bytes_per_unit": per_txn, "units_per_launch": B, "avg_launch_ms": round(ms, 4)},
        "cpu_baseline": cpu, "self_check": bool((res >= -1).all()),
        "setup_s": {"generate": round(gen_s, 1), "load": round(load_s, 1), "sync": round(sync_s, 1)},
    }
    print(json.dumps(result), flush=True)
    return 0


def run_chq2(args):
    """CH-benCHmark Q2 through the path (stage_ch_query2), one GPU: one read-only Q2 transaction
    (target region EUROPE, the reference's fixed choice) per step over W warehouses' STOCK."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from ch_data import ChTables  # the CH table generator (data only; the oracle trees only for the CPU leg)
    t0 = time.time()
    ch = ChTables(W=args.warehouses, I=args.items, seed=args.seed & 0xFFFF, oracle=not args.no_cpu_baseline)
    load_s = time.time() - t0
    t0 = time.time()
    ch.sync()
    sync_s = time.time() - t0
    nq = args.q2_batch
    rids = (0xFFFFFFFE - np.arange(nq)).astype(np.uint32)  # nq transactions per step, one read id each

    state = {}
    # the records land in one reused page-locked array (only the last step's are read): the
    # library copies them there straight from the device (a fresh 12-MiB pageable array per step
    # would cost the step its page faults and a staging copy)
    out_buf = stage.pinned_empty((nq, 1 << 14), stage.Q2_REC_DTYPE)

    use_async = bool(args.q2_async) and nq > 1
    # async: step k enqueues its batch into slot k % 2, then waits for step k-1's (one batch is
    # always in flight while the host stages the next); each slot has its own page-locked out
    outs = [out_buf, stage.pinned_empty((nq, 1 << 14), stage.Q2_REC_DTYPE)] if use_async else [out_buf]
    inflight = []

    def step():
        if nq == 1:
            return ch.query2(3)
        if use_async:
            slot = state.get("k", 0) % 2
            state["k"] = state.get("k", 0) + 1
            inflight.append(ch.query2_batch_async(rids, outs[slot], slot, 3))
            if len(inflight) < 2:
                return None, None
            recs_q, ab_q = inflight.pop(0).wait()
        else:
            recs_q, ab_q = ch.query2_batch(rids, 3, out=out_buf)
        state["all"] = (recs_q, ab_q)
        return recs_q[0], bool(ab_q.any())

    def drain():
        if inflight:
            recs_q, ab_q = inflight.pop(0).wait()
            state["all"] = (recs_q, ab_q)
            return recs_q[0], bool(ab_q.any())
        return None

    for _ in range(args.warmup):
        recs, ab = step()
    check(stage.lib().stage_device_sync(), "sync")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        recs, ab = step()
    last = drain()  # the last batch's results are part of the timed work
    if last is not None:
        recs, ab = last
    elapsed = time.perf_counter() - t0
    ms = elapsed / args.steps * 1e3
    same = True
    if nq > 1:  # every query of the batch must read what query 0 read (the visited suppliers and
        # the kept stocks do not depend on the read id on an update-free table)
        recs_q, ab_q = state["all"]
        same = bool(all((recs_q[q] == recs_q[0]).all() for q in range(nq)) and (ab_q == ab_q[0]).all())
    # the single-transaction commit path (stage_ch_query2 with a commit id: the marked STOCK
    # updates go through stage_update_batch_device), after the read-only batch
    commit = None
    if nq > 1:
        n1 = max(3, args.steps // 2)
        t1 = time.perf_counter()
        for i in range(n1):
            rid = 0x7FFF0000 + 2 * i
            r1, a1 = ch.query2(3, read_id=rid, commit_id=rid + 1)
        dt = time.perf_counter() - t1
        commit = {"value": round(n1 / dt, 2), "unit": "q2/s", "txns": n1, "ms_per_txn": round(dt / n1 * 1e3, 4),
                  "updates_last": int(r1["update"].sum()), "aborted_last": bool(a1),
                  "what": "one Q2 per call with its STOCK updates committed (RunQuery2 incl. the write)"}
    nsupp = int(recs.size)
    nstock = int(sum(int(ch.map_off[k + 1] - ch.map_off[k]) for k in recs["supp_key"]))
    # algorithmic bytes per step: the three scans read and write their rows (once per step); each
    # distinct STOCK / ITEM key is probed once per step -- its key, the 64-B fingerprint sector,
    # the 32-B slot word, a 32-B status record.  In a batch: each STOCK probe's status record and
    # slot word are read once more for all read ids together (the abort check), and per query the
    # supplier's last stock and its item are revisited at that read id (status record and slot
    # word read, a 32-B record written, each), the kept stock's and the item's column sectors read
    # (64 B each) and the 48-B output record written.  (Up to round 5's first lines the model
    # charged every STOCK lookup's revisit per query -- bytes the folded revisit never moves.)
    scans = 10000 * (8 + 111 + 128) + 62 * (8 + 185 + 192) + 5 * (8 + 207 + 224)
    probes = nstock * (16 + 64 + 32 + 32) + nsupp * (8 + 64 + 32 + 32)
    if nq > 1:
        probes += nstock * (32 + 32)
        per_query = nsupp * (64 + 64 + 96 + 96 + 48)
    else:
        per_query = nsupp * (64 + 64)
    per_step = scans + probes + nq * per_query
    achieved = per_step / (ms * 1e-3) / 1e9
    cpu, ok = None, not ab and same
    if not args.no_cpu_baseline:
        import ctypes

        import oracle_lib as O
        orecs, oab = ch.query2_oracle(3)
        a, b = np.sort(recs, order="supp_key"), np.sort(orecs, order="supp_key")
        ok = ok and same and oab == ab and a.size == b.size and all((a[f] == b[f]).all() for f in
                                                            ("supp_key", "s_w_id", "s_i_id", "s_quantity",
                                                             "item_has_b", "update"))
        threads = args.cpu_threads or cpu_resources()["threads"]
        o = ch.orc
        sec = ctypes.c_double()
        args_ = (o["region"].t, o["nation"].t, o["supplier"].t, o["item"].t, o["stock"].t, ch.map_off.ctypes.data,
                 ch.map_w.ctypes.data, ch.map_i.ctypes.data, 3, 0xFFFFFFFE)
        O.lib().orc_ch_query2_timed(*args_, threads, threads, ctypes.byref(sec))
        count = int(max(threads, threads / max(sec.value, 1e-9) * args.cpu_seconds))
        O.lib().orc_ch_query2_timed(*args_, count, threads, ctypes.byref(sec))
        cpu = {"value": round(count / sec.value, 2), "unit": "q2/s", "cores": threads, "kind": "port",
               "sample": f"oracle orc_ch_query2 (RunQuery2 restated), {count} read-only Q2s, same tables, "
                         f"{threads} threads on {cpu_name()}, {sec.value:.1f}s"}
    result = {
        "metric": ("CH-benCHmark Q2 txns/s, read-only batched (" + str(nq) + " Q2s per pass, no STOCK updates), "
                   if nq > 1 else "CH-benCHmark Q2 txns/s (with its updates), ") +
                  "through the index-organized path (supplementary to " + METRIC + ")",
        "value": round(args.steps * nq / elapsed, 2), "unit": "q2/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int64 keys / bytes", "data": "synthetic CH rows (tpcc_record.h layouts, "
                                                                      "tpcc_loader.cpp value rules)",
        "config": {"workload": "CH-benCHmark Q2 (tpcc_new_order.cpp RunQuery2), region EUROPE",
                   "warehouses": args.warehouses, "items": args.items, "q2_per_step": nq,
                   "suppliers_visited": nsupp,
                   "stock_lookups": nstock, "aborted": bool(ab), "updates": int(recs["update"].sum()),
                   "read_only_batch": nq > 1, "queries_equal_query0": same,
                   "batches_in_flight": 2 if use_async else 1,
                   "batch_lookups": "the batch's queries look up the same STOCK / ITEM keys (the visited suppliers do "
                                    "not depend on the read id): each key is probed once and its hit slot's "
                                    "visibility evaluated at every query's read id" if nq > 1 else None},
        "single_q2_commit_path": commit,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel": "Q2 step (3 scans + batched STOCK / ITEM probes of q2_per_step transactions)",
                     "algorithmic_bytes_per_launch": per_step, "q2_per_launch": nq, "avg_launch_ms": round(ms, 4)},
        "cpu_baseline": cpu, "self_check": bool(ok),
        "setup_s": {"load": round(load_s, 1), "sync": round(sync_s, 1)},
    }
    print(json.dumps(result), flush=True)
    return 0 if ok else 1


PCIE_PEAK_GBS = 63.0  # PCIe Gen5 x16 per direction (MI355X_MICROARCH.md, host link)


def end_to_end_leg(tab, args, draws):
    """C2 delivered to host memory (SURVEY §8(d) timing rule: H2D / D2H included): the same 2^24
    Zipf keys through stage_probe_host from a pinned key array, each call's status records and
    rows landing in a pinned result ring the caller consumes (2^22 lookups per call), for
    --e2e-passes passes over the batch.  Two output layouts: the default (32-B stage_probe_out,
    1024-B rows) and the lean one a host caller asks for with stage_set_output_layout(1008, 16)
    (16-B stage_probe_out16, packed 1008-B [key][payload] rows: what IndexScanExecutor copies
    out, executor.h:396-397).  The last call's first 4096 results are compared with the
    device-buffer probe (stage_probe_batch) of the same keys on the same table state.  It runs
    after the other device legs: pinning and releasing its 4-GB ring slowed the C3 leg that
    followed it by ~7 % (round-6 A/B, profiles/r06/e2eorder)."""
    B = draws.size
    chunk = min(B, 1 << 22)
    keys = stage.pinned_empty(B, np.uint64)
    keys[:] = draws
    layouts = (("default", 0, 32), ("lean", 1008, 16))
    res = {}
    last = (B // chunk - 1) * chunk
    k = min(4096, chunk)
    tab.set_output_layout(0, 32)
    ref_out, ref_rows = tab.probe(draws[last:last + k])
    ref_st, ref_rows = ref_out["status"], ref_rows[:, :1008]
    for name, stride, sb in layouts:
        tab.set_output_layout(stride, sb)
        dt = stage.PROBE_OUT16_DTYPE if sb == 16 else stage.PROBE_OUT_DTYPE
        out = stage.pinned_empty(chunk, dt)
        rows = stage.pinned_empty((chunk, tab.stride), np.uint8)
        tab.probe_host(keys[:chunk], out=out, rows=rows)  # warm: the pipe's device buffers
        t0 = time.perf_counter()
        for _ in range(args.e2e_passes):
            for b in range(0, B - chunk + 1, chunk):
                tab.probe_host(keys[b:b + chunk], out=out, rows=rows)
        sec = time.perf_counter() - t0
        n = args.e2e_passes * (B // chunk) * chunk
        d2h = sb + tab.stride
        eq = bool((out["status"][:k] == ref_st).all() and (rows[:k, :1008] == ref_rows).all())
        res[name] = {"value": round(n / sec, 1), "unit": "ops/s", "lookups": n, "seconds": round(sec, 4),
                     "bytes_per_lookup": {"h2d": 8, "d2h": d2h}, "status_bytes": sb, "row_stride": tab.stride,
                     "pcie_d2h_gbs": round(n * d2h / sec / 1e9, 2), "pcie_h2d_gbs": round(n * 8 / sec / 1e9, 3),
                     "pcie_d2h_frac": round(n * d2h / sec / 1e9 / PCIE_PEAK_GBS, 3), "check_equal": eq}
        del out, rows
    tab.set_output_layout(args.out_stride or 0, 32)
    del keys
    lean = res["lean"]
    return {**lean, "layout": "stage_set_output_layout(1008, 16): 16-B status records + packed 1008-B rows",
            "pcie_peak_gbs": PCIE_PEAK_GBS, "default_layout": res["default"],
            "timed": f"{args.e2e_passes} passes over the C2 batch, {chunk} lookups per stage_probe_host call, keys "
                     "in pinned host memory before the timed region, results into a pinned ring the caller "
                     "reuses; H2D of keys, probe and D2H of status records + rows all inside"}


def c4_leg(tab, args, total_rows, rank, stream, steps, warmup):
    """configs[3]: B uniform start keys, L-key range scans (stage_scan_batch); returns the leg's
    measured dict and a sample for the oracle check."""
    L = stage.lib()
    B = args.scan_batch if args.config == "c2" else args.batch
    starts = (stage.fastrandom(args.seed + rank, B) % np.uint64(total_rows)).astype(np.uint64)
    d_keys = stage.DeviceBuffer.from_numpy(starts)
    d_cnt = stage.DeviceBuffer(B * 4)
    d_rec = stage.DeviceBuffer(B * args.scan_size * tab.stride)

    def step():
        check(L.stage_scan_batch(tab.h, d_keys.ptr, None, B, args.scan_size, d_cnt.ptr, d_rec.ptr, stream.ptr), "scan")

    for _ in range(warmup):
        step()
    stream.sync()
    evs = [stage.Event() for _ in range(2 * steps)]
    t0 = time.perf_counter()
    for i in range(steps):
        evs[2 * i].record(stream)
        step()
        evs[2 * i + 1].record(stream)
    stream.sync()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([evs[2 * i].elapsed_ms(evs[2 * i + 1]) for i in range(steps)]))
    cnt = d_cnt.to_numpy(np.uint32, B)
    ok = bool((cnt > 0).all() and (cnt == args.scan_size).mean() > 0.99)
    ns = min(B, 256)
    recs = d_rec.to_numpy(np.uint8, ns * args.scan_size * tab.stride).reshape(ns, args.scan_size, tab.stride)
    traffic, tsrc = traffic_from_profile(B, args.rows, "pmc_scan.json")
    d = {"value": round(B * steps / elapsed, 1), "unit": "scans/s", "steps": steps, "warmup": warmup,
         "ms_per_step": round(elapsed / steps * 1e3, 4), "self_check": ok,
         "config": {"workload": WORKLOADS["c4"], "scans_per_step": B, "scan_size": args.scan_size,
                    "starts": "uniform over [0, N)"},
         "roofline": hbm_roofline(scan_bytes(args.scan_size), B, kern_ms, "scan_kernel", traffic, tsrc)}
    for b in (d_keys, d_cnt, d_rec):
        b.free()
    return d, (starts[:ns], cnt[:ns], recs)


def c3_leg(tab, args, stream, nthreads, steps, warmup):
    """configs[2]: YCSB-B epochs.  Timed loop, per epoch: the write share on the write path,
    then the device probe of the read share at the epoch's read ids.  value = reads / the
    probes' time (device write path: the probes' stream time between events; host write path:
    their wall time); ops_per_s_incl_writes = (reads + updates) / the whole loop's wall time
    (device write path: each epoch's kernels are enqueued on the probe's stream without a host
    wait, the host table adopts the epoch on a background thread while the probe runs, and the
    next epoch's call waits for that adoption)."""
    L = stage.lib()
    B = args.batch
    theta = args.theta if args.config == "c3" else 0.99
    ycsb_b = YcsbB(tab, args, nthreads, theta)
    t0 = time.time()
    warm = max(1, warmup)
    epochs = [ycsb_b.make_epoch() for _ in range(warm + steps)]
    if args.write_path == "device":
        for ep in epochs:
            ycsb_b.upload(ep)
    else:
        for ep in epochs:
            ep["d"] = {"reads": stage.DeviceBuffer.from_numpy(ep["reads"]),
                       "rids": stage.DeviceBuffer.from_numpy(ep["rids"]),
                       "out": stage.DeviceBuffer(32 * ep["reads"].size)}
    prep_s = time.time() - t0
    d_rec = stage.DeviceBuffer(B * tab.stride)
    if args.write_path == "device":
        tab.set_write_overlap(args.write_overlap)

    def probe(ep):
        d = ep["d"]
        tab.probe_device(d["reads"].ptr, ep["reads"].size, d["out"].ptr, d_rec.ptr, d_read_ids=d["rids"].ptr,
                         stream=stream.ptr)

    for ep in epochs[:warm]:  # untimed: first-call allocations of the write path
        ycsb_b.apply(ep)
        probe(ep)
    stream.sync()
    check(L.stage_device_sync(), "sync")
    check(L.stage_settle(tab.h), "settle")  # the warmup epochs' host adoption stays out of the timed loop
    evs = [stage.Event() for _ in range(2 * steps)]
    device_wp = args.write_path == "device"
    elapsed, write_s, updates, ops_done = 0.0, 0.0, 0, 0
    t_loop = time.perf_counter()
    timed = epochs[warm:]
    for i, ep in enumerate(timed):
        tw = time.perf_counter()
        # device write path: the epoch's kernels are enqueued on the probe's stream (the reads
        # follow the epoch's writes in stream order; no host wait in between); host write path:
        # applied and published before the probe
        updates += ycsb_b.apply(ep, stream if device_wp else None)
        write_s += time.perf_counter() - tw
        tr = time.perf_counter()
        evs[2 * i].record(stream)
        probe(ep)
        evs[2 * i + 1].record(stream)
        if not device_wp:
            stream.sync()
            elapsed += time.perf_counter() - tr
        ops_done += ep["reads"].size
    stream.sync()
    # the last epoch's host adoption (a background thread of the device write path) is part of
    # the write work: settle it before the loop's clock stops
    check(L.stage_settle(tab.h), "settle")
    loop_s = time.perf_counter() - t_loop
    probe_ms = [evs[2 * i].elapsed_ms(evs[2 * i + 1]) for i in range(steps)]
    if device_wp:  # the probes' device time (start event -> end event on the stream)
        elapsed = sum(probe_ms) / 1e3
        check(L.stage_device_sync(), "sync")
        updates = sum(YcsbB.count_ok(ep) for ep in epochs[warm:])
    kern_ms = float(np.mean(probe_ms))
    rc_hist = {}
    for ep in epochs[warm:]:
        for k, v in YcsbB.rc_counts(ep).items():
            rc_hist[k] = rc_hist.get(k, 0) + v
    hist = np.zeros(6, np.int64)
    hops = 0
    for ep in epochs[warm:]:
        o = ep["d"]["out"].to_numpy(stage.PROBE_OUT_DTYPE, ep["reads"].size)
        hist += np.bincount(o["status"], minlength=6)[:6]
        hops += int(o["hops"].astype(np.int64).sum())
    mean_hops = hops / max(ops_done, 1)
    last = epochs[-1]
    ns = min(last["reads"].size, 4096)
    rows = d_rec.to_numpy(np.uint8, ns * tab.stride).reshape(ns, tab.stride)
    st = last["d"]["out"].to_numpy(stage.PROBE_OUT_DTYPE, ns)["status"]
    check_sample = (last["reads"][:ns].copy(), last["rids"][:ns].copy(), st, rows)
    # every outcome the read-id model produces occurred (no OLD reads when every read is at the
    # newest id: --old-share 0)
    ok = bool(hist[stage.ST_LATEST] > 0 and hist[stage.ST_COPY] > 0 and (hist[stage.ST_OLD] > 0 or args.old_share == 0))
    per_unit = BYTES_PER_LOOKUP + HOP_BYTES * mean_hops
    # value: the YCSB-B ops/s of configs[2] -- reads and successful updates over the whole loop
    # (write path + probes); reads_per_s: the read probes alone (their stream time), the figure
    # the probe's roofline is about (round 4 reported that one as `value`)
    d = {"value": round((ops_done + updates) / loop_s, 1), "unit": "ops/s", "steps": steps, "warmup": warm,
         "ms_per_step": round(loop_s / steps * 1e3, 4), "self_check": ok,
         "value_is": "reads + successful updates per second over the timed loop (write path + read probes)",
         "reads_per_s": round(ops_done / elapsed, 1), "read_probe_ms_per_step": round(elapsed / steps * 1e3, 4),
         "ops_per_s_incl_writes": round((ops_done + updates) / loop_s, 1),
         "config": {"workload": WORKLOADS["c3"], "theta": theta, "update_ratio": args.update_ratio,
                    "update_stream": "RunMixed: FastRandom NextUniform() < update_ratio, delta = 100 x next_char() "
                                     "(ycsb_mixed.cpp:26-44)",
                    "inflight_share": args.inflight_share, "updates_applied": updates,
                    "read_ids": f"{100 - round(100 * args.old_share)} % the newest id, {round(100 * args.old_share)} % "
                                f"up to {args.reader_window} ids older (concurrent readers; round 4 on: not comparable "
                                f"with round-3 C3 figures, which drew older ids from the whole run)",
                    "update_ops": int(sum(ep["keys"].size for ep in epochs[warm:])),
                    "updates_in_flight": int(sum(ep["inflight"] for ep in epochs[warm:])),
                    # why update ops fail: not_needed_update = the column already holds the value
                    # (RunMixed's delta byte is a fresh next_char() per update: a 1/256 chance) or a
                    # newer committed writer; dirty = the record is in flight (an uncommitted
                    # update earlier in the epoch)
                    "update_rc_counts": rc_hist,
                    "write_path": args.write_path,
                    "write_overlap": bool(args.write_overlap) and args.write_path == "device", "write_call_s": round(write_s, 4), "loop_s": round(loop_s, 4),
                    "epoch_prep_s_untimed": round(prep_s, 2), "mean_chain_hops": round(mean_hops, 4),
                    # copies / versions / heap images are append-only (no GC, as the reference
                    # with its cleaner off): each successful update takes one of each, and the
                    # 30-bit indices end the write path after about this many more updates
                    "write_capacity_updates_left": int((1 << 30) - 1 - tab.stats()["records"] -
                                                       tab.stats()["versions"] -
                                                       sum(ep["keys"].size for ep in epochs)),
                    "read_status_counts": {"latest": int(hist[1]), "copy": int(hist[2]), "old": int(hist[3]),
                                           "fail": int(hist[4]), "chain_miss": int(hist[5]),
                                           "not_found": int(hist[0])},
                    "timed": "value = ops_per_s_incl_writes: the whole loop (write path + probes); reads_per_s: "
                             "the device probes of the read shares; epoch inputs resident in HBM beforehand" +
                             ("; write overlap: each probe runs beside the next epoch's write-path kernels "
                              "(its time includes that contention)" if device_wp and args.write_overlap else "")},
         "roofline": hbm_roofline(per_unit, ops_done / steps, kern_ms, "probe_kernel (read ids, chain walks)",
                                  *traffic_from_profile(args.batch, args.rows, "pmc_probe_c3.json"))}
    d["roofline"]["algorithmic_bytes"] = f"{BYTES_PER_LOOKUP} + {HOP_BYTES} x mean hops ({mean_hops:.4f})"
    rec = {"record": ycsb_b.record, "reads": last["reads"], "rids": last["rids"], "check": check_sample}
    for ep in epochs:
        ycsb_b.release(ep)
    d_rec.free()
    return d, rec


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    in_dist = "WORLD_SIZE" in os.environ
    if args.gpus > 1 and not in_dist:
        return launch_ranks(args, argv)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if in_dist and world != args.gpus:
        log(f"[rank {rank}] WORLD_SIZE={world} but --gpus {args.gpus}: refusing to report a mislabelled point")
        return 2
    if args.config == "tpcc":
        return run_tpcc(args)
    if args.config == "chq2":
        return run_chq2(args)
    sharded = world > 1 or args.force_sharded
    if (sharded or args.dry_run) and args.config != "c2":
        raise SystemExit("multi-GPU runs use the point-lookup config (c2 -> configs[4])")
    if args.dry_run:
        import torch.distributed as tdist
        tdist.init_process_group("gloo")  # CPU rehearsal of the control plane only
        try:
            return dry_run(args, rank, world, tdist)
        finally:
            tdist.destroy_process_group()
    if sharded:
        return run_sharded(args, rank, world, local)
    res = cpu_resources()
    nthreads = args.cpu_threads or res["threads"]
    check(stage.lib().stage_set_device(local), "set device")

    total_rows = args.rows
    orc = None
    cpu_leg = not args.no_cpu_baseline
    if cpu_leg:  # the oracle table builds on the host while the GPU leg runs
        orc = CpuOracle(cpu_rows_for(args, res, args.rows), nthreads)
    t0 = time.time()
    tab = stage.Table(key_width=8, device=local)
    loaded = tab.load_ycsb(0, total_rows, 8, mode=0)
    t_load = time.time() - t0
    t0 = time.time()
    tab.sync()
    t_sync = time.time() - t0
    if args.out_stride:
        tab.set_output_layout(args.out_stride)
    st = tab.stats()
    log(f"[rank {rank}] loaded {loaded} rows in {t_load:.1f}s, sync {t_sync:.1f}s, leaves {st['leaves']}")

    B = args.batch
    L = stage.lib()
    stream = stage.Stream()
    extras, samples = {}, {}
    if args.config == "c4":
        head, samples["c4"] = c4_leg(tab, args, total_rows, rank, stream, args.steps, args.warmup)
    elif args.config == "c3":
        head, samples["c3"] = c3_leg(tab, args, stream, nthreads, args.steps, args.warmup)
    else:
        head = None
    if head is None:  # C2: the headline
        draws = stage.zipf_draws(total_rows - 1, args.theta, args.seed + rank, B, nthreads=nthreads)
        d_keys = stage.DeviceBuffer(B * 8)
        check(L.stage_memcpy_h2d(d_keys.ptr, draws.ctypes.data, draws.nbytes, None), "h2d")
        d_out = stage.DeviceBuffer(B * 32)
        d_rec = stage.DeviceBuffer(B * tab.stride)
        d_leaf = None
        if args.host_traversal:
            d_leaf = stage.DeviceBuffer.from_numpy(tab.traverse(draws))

        def step():
            tab.probe_device(d_keys.ptr, B, d_out.ptr, d_rec.ptr, d_leaf_ids=d_leaf.ptr if d_leaf else None,
                             stream=stream.ptr)

        for _ in range(args.warmup):
            step()
        stream.sync()
        check(L.stage_device_sync(), "sync")
        evs = [stage.Event() for _ in range(2 * args.steps)]
        t0 = time.perf_counter()
        for i in range(args.steps):
            evs[2 * i].record(stream)
            step()
            evs[2 * i + 1].record(stream)
        stream.sync()
        check(L.stage_device_sync(), "sync")
        elapsed = time.perf_counter() - t0
        kern_ms = float(np.mean([evs[2 * i].elapsed_ms(evs[2 * i + 1]) for i in range(args.steps)]))
        # self-check: 8 windows of 8192 lookups spread over the batch, each against its key's
        # LoadYCSBRows row
        sample = min(B, 8192)
        outs_w, rows_w, keys_w = [], [], []
        for w in range(8 if B > 8 * sample else 1):
            o = (B - sample) * w // 7 if B > 8 * sample else 0
            outs_w.append(d_out.to_numpy(stage.PROBE_OUT_DTYPE, sample, offset=o * 32))
            rows_w.append(d_rec.to_numpy(np.uint8, sample * tab.stride, offset=o * tab.stride).reshape(sample, tab.stride))
            keys_w.append(draws[o:o + sample])
        outs, rows, kw = np.concatenate(outs_w), np.concatenate(rows_w), np.concatenate(keys_w)
        ok = bool((outs["status"] == stage.ST_LATEST).all() and
                  (rows[:, :8].copy().view(np.uint64).ravel() == kw).all() and
                  (rows[:, 8:1008] == (kw & np.uint64(0xFF)).astype(np.uint8)[:, None]).all())
        samples["c2"] = (draws[:4096].copy(), outs_w[0]["status"][:4096].copy(), rows_w[0][:4096].copy())
        traffic, tsrc = traffic_from_profile(B, args.rows, "pmc_probe.json")
        roof = hbm_roofline(BYTES_PER_LOOKUP, B, kern_ms, "probe_kernel", traffic, tsrc)
        roof["timing_note"] = ("achieved uses this run's hipEvent time of the probe; traffic comes from a separate "
                               "rocprofv3 --pmc pass (traffic_source), whose box and kernel time can differ by a few %")
        head = {"value": round(B * args.steps / elapsed, 1), "unit": "ops/s",
                "ms_per_step": round(elapsed / args.steps * 1e3, 4), "self_check": ok, "roofline": roof,
                "config": {"workload": WORKLOADS["c2"], "theta": args.theta,
                           "traversal": "host" if d_leaf else "device"}}
        for b in (d_keys, d_out, d_rec) + ((d_leaf,) if d_leaf else ()):
            b.free()
        if not args.no_extras:
            # the other single-GPU configs on the same loaded table: C4, then C3 (mutates it)
            log(f"[rank {rank}] C2: {head['value'] / 1e9:.3f} G lookups/s; C4 leg")
            extras["c4"], samples["c4"] = c4_leg(tab, args, total_rows, rank, stream, 5, 1)
            log(f"[rank {rank}] C4: {extras['c4']['value'] / 1e6:.1f} M scans/s; C3 leg")
            extras["c3"], samples["c3"] = c3_leg(tab, args, stream, nthreads, args.c3_epochs, 1)
            log(f"[rank {rank}] C3: {extras['c3']['value'] / 1e9:.3f} G ops/s incl. writes "
                f"({extras['c3']['reads_per_s'] / 1e9:.3f} G reads/s)")
        if not args.no_e2e:  # last: its pinned ring disturbs the legs after it
            head["end_to_end"] = end_to_end_leg(tab, args, draws)
            head["end_to_end"]["table_state"] = ("as the C4 and C3 legs left it (C3's updates applied)"
                                                 if not args.no_extras else "as loaded (the C2 table)")
            log(f"[rank {rank}] C2 end to end (host buffers): {head['end_to_end']['value'] / 1e6:.1f} M lookups/s, "
                f"{head['end_to_end']['pcie_d2h_gbs']} GB/s D2H")
    if not head["self_check"]:
        log(f"[rank {rank}] SELF-CHECK FAILED")

    cpu = None
    if cpu_leg:
        log(f"[rank {rank}] CPU legs ({nthreads} threads)")
        legs = cpu_legs(orc, args, res, nthreads, c2_check=samples.get("c2"), c4_check=samples.get("c4"),
                        c3=samples.get("c3"))
        legs["c2"]["calibration"] = cpu_calibration(orc.O, nthreads)
        cpu = legs[args.config]
        if "end_to_end" in head:
            head["end_to_end"]["vs_cpu_baseline"] = round(head["end_to_end"]["value"] / cpu["value"], 2)
        for k, v in extras.items():
            v["cpu_baseline"] = legs.get(k)
    config = {**head["config"], "rows_per_gpu": args.rows, "rows_total": total_rows,
              "batch_per_gpu": B if args.config != "c4" else args.batch, "key_bytes": 8, "payload_bytes": 1000,
              "leaf_bytes": 65536, "parallelism": "single GPU"}
    result = {
        "metric": METRIC, "value": head["value"], "unit": head["unit"], "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": head["ms_per_step"], "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic (LoadYCSBRows keys/payloads)",
        "config": config, "roofline": head["roofline"], "cpu_baseline": cpu, "self_check": head["self_check"],
        **({k: head[k] for k in ("value_is", "reads_per_s", "read_probe_ms_per_step", "ops_per_s_incl_writes")
            if k in head}),
        **({"end_to_end": head["end_to_end"]} if "end_to_end" in head else {}),
        **({"extras": extras} if extras else {}),
        "setup_s": {"load": round(t_load, 1), "sync": round(t_sync, 1)},
        "host_peak_rss_gib": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20, 1),
    }
    print(json.dumps(result), flush=True)
    ok = head["self_check"] and all(v["self_check"] for v in extras.values())
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
