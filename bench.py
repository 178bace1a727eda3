#!/usr/bin/env python3
"""bench.py -- YCSB on MI355X through the index-organized probe/scan path.

Default (`--config c2`, BASELINE.json configs[1]): YCSB-C batched point lookup.
  table : N rows per GPU loaded as LoadYCSBRows does (key = rowid, 8-byte keys, payload =
          memset(rowid) 1000 B), reference leaf layout (64 KiB leaves, <= 63 records)
  step  : one pass of the hot path over a batch of B = 2^24 Zipf(0.9) lookups over
          [1, N_total-1] (ZipfDistribution of benchmark_common.h, seed 0x5EED + rank):
          device traversal + leaf probe + visibility + 1008-B tuple copy (stage_probe_batch);
          with --gpus > 1 each key goes to shard MurmurHash64A(key, 8, 0) % world and is
          answered over RCCL (stage_probe_sharded) -- configs[4] at 8 GPUs
  value = lookups completed by all ranks / max-over-ranks wall time of the K timed steps.
`--config c3` (configs[2]): YCSB-B epochs -- 5 % updates (zipf 0.99) applied between steps
  by the device write path (stage_update_batch_device; `--write-path host` = host write path +
  incremental publish), the step probes the reads (25 % at older snapshots -> version chains
  on the device).  `--config c4` (configs[3]): 100-key range scans.

The CPU baseline leg (rank 0, one GPU) times the test oracle -- the C restatement of the
reference's BTree::Read + executor copy (or TableScanExecutor) -- on a bounded 2M-row sample
(the reference's own default pools cap a YCSB table at ~2-2.5M rows).
"""
import argparse
import ctypes
import json
import math
import os
import platform
import resource
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "stage-indexorganized_amd"))
import stage  # noqa: E402  (load libstage_hip.so before anything else binds a HIP runtime)
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
HBM_PEAK_GBS = 8000.0    # MI355X_MICROARCH.md: 8.0 TB/s HBM3E spec
XGMI_LINK_GBS = 153.0    # per xGMI link of an MI355X (7 links per GPU, point to point)


def scan_bytes(L, S=48.8):
    """B_scan = 8 + 64*(ceil(L/S)+1) + L*(8+1000) + L*1008 + 4."""
    return 8 + 64 * (math.ceil(L / S) + 1) + L * (8 + 1000) + L * 1008 + 4


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=None)
    p.add_argument("--warmup", type=int, default=None)
    p.add_argument("--config", choices=["c2", "c3", "c4", "tpcc", "chq2"], default="c2")
    p.add_argument("--warehouses", type=int, default=16, help="tpcc: warehouses (10 districts, 3000 orders each)")
    p.add_argument("--items", type=int, default=100_000, help="tpcc: items (stock rows per warehouse)")
    p.add_argument("--q2-batch", type=int, default=16, help="chq2: Q2 transactions per step (stage_ch_query2_batch)")
    p.add_argument("--rows", type=int, default=100_000_000, help="rows per GPU")
    p.add_argument("--batch", type=int, default=None, help="lookups (c2/c3) or scans (c4) per GPU per step")
    p.add_argument("--theta", type=float, default=None)
    p.add_argument("--scan-size", type=int, default=100)
    p.add_argument("--update-ratio", type=float, default=0.05)
    p.add_argument("--write-path", choices=["device", "host"], default="device",
                   help="c3: apply each epoch's updates on the device (stage_update_batch_device) or on the "
                        "host write path + incremental publish (stage_update_batch + stage_sync)")
    p.add_argument("--seed", type=int, default=0x5EED)
    p.add_argument("--cpu-rows", type=int, default=2_000_000)
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--host-traversal", action="store_true", help="leaf ids from the host router instead")
    p.add_argument("--force-sharded", action="store_true",
                   help="run the multi-GPU (RCCL) code path even with one rank -- a rehearsal, not a config")
    a = p.parse_args()
    a.steps = a.steps if a.steps is not None else (5 if a.config == "c3" else 20)
    a.warmup = a.warmup if a.warmup is not None else (1 if a.config == "c3" else 3)
    a.theta = a.theta if a.theta is not None else (0.99 if a.config == "c3" else 0.9)
    a.batch = a.batch if a.batch is not None else ((1 << 18) if a.config in ("c4", "tpcc") else (1 << 24))
    if a.config == "tpcc":
        a.steps = a.steps if a.steps is not None else 10
    return a


def owned_keys(total_rows, world, rank):
    """Keys of this shard: MurmurHash64A(key, 8, 0) % world == rank, ascending (loaded in order)."""
    parts = []
    chunk = 1 << 24
    for b in range(0, total_rows, chunk):
        k = np.arange(b, min(total_rows, b + chunk), dtype=np.uint64)
        h = stage.murmur64a_device(k, 8, 0)
        parts.append(k[(h % np.uint64(world)) == np.uint64(rank)])
    return np.concatenate(parts)


def traffic_from_profile(batch, rows, name="pmc_probe.json"):
    """Per-launch HBM bytes of the dominant kernel from a committed rocprofv3 --pmc pass (see
    profiles/README.md), if one exists for this configuration."""
    path = os.path.join(REPO, "profiles", name)
    if not os.path.exists(path):
        return None, None
    try:
        d = json.load(open(path))
        if d.get("batch") == batch and d.get("rows") == rows:
            return d["hbm_bytes_per_launch"], os.path.relpath(path, REPO)
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


def xgmi_roofline(batch, world, stride, step_s, hbm_roof):
    """Roofline of the multi-GPU step, bound by the xGMI exchange: per rank and step the remote
    share of the batch ((W-1)/W of it, hash-uniform) sends its 16-B key record out and gets a
    32-B status record + a stride-byte row back; peak = the W-1 links a rank uses."""
    remote = batch * (world - 1) / world
    unit = 16 + 32 + stride
    achieved = remote * unit / step_s / 1e9
    peak = XGMI_LINK_GBS * (world - 1)
    return {"bound": "xgmi", "achieved": round(achieved, 1), "peak": peak, "unit": "GB/s",
            "frac": round(achieved / peak, 4), "traffic": None,
            "kernel": "sharded step (route + RCCL all-to-all-v + probe_kernel + un-permute)",
            "algorithmic_bytes_per_unit": unit, "units_per_launch": round(remote),
            "avg_launch_ms": round(step_s * 1e3, 4),
            "peak_source": f"{XGMI_LINK_GBS:.0f} GB/s per xGMI link (7 per MI355X), {world - 1} links per rank",
            "hbm": hbm_roof}


def cpu_baseline(args, threads):
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib as O  # the checker, timed here as the reference CPU path
    n = args.cpu_rows
    t0 = time.time()
    orc = O.OracleTree()
    orc.load_ycsb(0, n, 8, 0)
    build_s = time.time() - t0
    secs = ctypes.c_double()
    if args.config == "c4":
        starts = (stage.fastrandom(args.seed, 20_000) % np.uint64(n)).astype(np.uint64)
        O.lib().orc_scan_batch_timed(orc.t, starts.ctypes.data, 8, starts.size, args.scan_size, threads,
                                     ctypes.byref(secs))
        rate = starts.size / max(secs.value, 1e-9)
        count = int(min(max(rate * args.cpu_seconds, 10_000), 5_000_000))
        starts = (stage.fastrandom(args.seed + 1, count) % np.uint64(n)).astype(np.uint64)
        O.lib().orc_scan_batch_timed(orc.t, starts.ctypes.data, 8, starts.size, args.scan_size, threads,
                                     ctypes.byref(secs))
        value = count / secs.value
        what = f"oracle TableScanExecutor over Iterator, {count} scans of {args.scan_size}"
        unit = "scans/s"
    else:
        keys = stage.zipf_draws(n - 1, args.theta, args.seed, 400_000, nthreads=threads)
        O.lib().orc_read_batch_timed(orc.t, keys.ctypes.data, 8, None, keys.size, threads, ctypes.byref(secs))
        rate = keys.size / max(secs.value, 1e-9)
        count = int(min(max(rate * args.cpu_seconds, 100_000), 300_000_000))
        keys = stage.zipf_draws(n - 1, args.theta, args.seed + 1, count, nthreads=threads)
        O.lib().orc_read_batch_timed(orc.t, keys.ctypes.data, 8, None, keys.size, threads, ctypes.byref(secs))
        value = count / secs.value
        what = f"oracle BTree::Read+copy, {count} zipf-{args.theta} lookups"
        unit = "ops/s"
    return {"value": round(value, 1), "unit": unit, "cores": threads, "kind": "port",
            "sample": f"{what}, {n} rows (8-B keys, 1000-B payload, build {build_s:.1f}s), {threads} threads "
                      f"on {cpu_name()}, {secs.value:.1f}s"}


class PinnedArray:
    """numpy view of a pinned host buffer (stage_host_alloc): full-rate PCIe copies."""

    def __init__(self, count, dtype):
        self.nbytes = max(1, count * np.dtype(dtype).itemsize)
        self.p = ctypes.c_void_p()
        check(stage.lib().stage_host_alloc(self.nbytes, ctypes.byref(self.p)), "host alloc")
        raw = (ctypes.c_uint8 * self.nbytes).from_address(self.p.value)
        self.a = np.frombuffer(raw, np.uint8).view(dtype)[:count]

    def free(self):
        if self.p:
            stage.lib().stage_host_free(self.p)
            self.p = None


class YcsbB:
    """configs[2]: each epoch applies the update share of a YCSB-B batch on the write path
    (LeafNode::Update + CommitTransaction UPDATE entry, read/commit ids from one counter as
    tid_counter does) -- on the device (stage_update_batch_device) or on the host
    (stage_update_batch + incremental publish) -- and returns the read share with read ids:
    75 % current, 25 % drawn from the ids of this run so far (older snapshots).
    Timed as the write path (`write_s`): the update share's transfer to the device and the call
    (device) or the host update + publish (host); generating the synthetic epoch is not."""

    def __init__(self, tab, args, nthreads):
        self.tab, self.args, self.nthreads = tab, args, nthreads
        self.counter = 1
        self.epoch = 0
        self.updates = 0
        self.prep_s = 0.0
        self.write_s = 0.0
        self.sync_s = 0.0
        self.last_sync = None
        if args.write_path == "device":
            B = args.batch  # the update share of a batch never exceeds it
            self.h = {k: PinnedArray(B * w, dt) for k, (w, dt) in
                      {"keys": (1, np.uint64), "cols": (100, np.uint8), "rid": (1, np.uint32),
                       "cid": (1, np.uint32)}.items()}
            self.d = {k: stage.DeviceBuffer(v.nbytes) for k, v in self.h.items()}
            self.d_rc = stage.DeviceBuffer(B)

    def next_batch(self):
        a = self.args
        n = a.rows
        t0 = time.time()
        draws = stage.zipf_draws(n - 1, a.theta, a.seed + 1000 * self.epoch, a.batch, nthreads=self.nthreads)
        rng = np.random.default_rng(a.seed + self.epoch)
        is_upd = rng.random(a.batch) < a.update_ratio
        keys = draws[is_upd]
        m = keys.size
        # read id / commit id pairs from one counter (tid_counter), one 100-B column patch each
        rid = (self.counter + 2 * np.arange(m, dtype=np.uint64)).astype(np.uint32)
        cid = rid + np.uint32(1)
        self.counter += 2 * m
        cols = np.repeat(((keys + np.uint64(self.epoch + 1)) & np.uint64(0xFF)).astype(np.uint8)[:, None], 100, 1)
        if a.write_path == "device":
            for k, x in (("keys", keys), ("cols", cols.reshape(-1)), ("rid", rid), ("cid", cid)):
                self.h[k].a[:x.size] = x
        self.prep_s += time.time() - t0
        tu = time.time()
        if a.write_path == "device":
            # keys / ids / column patches over PCIe, then the epoch runs on the published image
            L = stage.lib()
            ok = ctypes.c_uint64()
            if m:
                for k, w in (("keys", 8), ("cols", 100), ("rid", 4), ("cid", 4)):
                    check(L.stage_memcpy_h2d(self.d[k].ptr, self.h[k].p, m * w, None), "h2d")
                check(L.stage_update_batch_device(self.tab.h, self.d["keys"].ptr, None, m, 0, self.d["cols"].ptr, 100,
                                                  self.d["rid"].ptr, self.d["cid"].ptr, None, self.d_rc.ptr,
                                                  ctypes.byref(ok), None),
                      "update_batch_device")
            ok = ok.value
        else:
            _, ok = self.tab.update_batch(keys, 0, cols, rid, cid)
            t1 = time.time()
            self.tab.sync()
            self.sync_s += time.time() - t1
            self.last_sync = self.tab.sync_info()
        self.write_s += time.time() - tu
        self.updates += ok
        t0 = time.time()
        reads = draws[~is_upd]
        rids = np.full(reads.size, self.counter, np.uint32)
        old = rng.random(reads.size) < 0.25
        rids[old] = rng.integers(1, max(2, self.counter), int(old.sum())).astype(np.uint32)
        self.epoch += 1
        self.prep_s += time.time() - t0
        return reads, rids


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
        threads = min(16, os.cpu_count() or 8)
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

    def step():
        if nq == 1:
            return ch.query2(3)
        recs_q, ab_q = ch.query2_batch(rids, 3)
        return recs_q[0], bool(ab_q.any())

    for _ in range(args.warmup):
        recs, ab = step()
    check(stage.lib().stage_device_sync(), "sync")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        recs, ab = step()
    elapsed = time.perf_counter() - t0
    ms = elapsed / args.steps * 1e3
    nsupp = int(recs.size)
    nstock = int(sum(int(ch.map_off[k + 1] - ch.map_off[k]) for k in recs["supp_key"]))
    # algorithmic bytes per Q2: each STOCK / ITEM point lookup reads its key, the 64-B fingerprint
    # sector and the 32-B slot word and writes its 32-B status record; the kept stock's and the
    # item's column sectors (64 B each); the three scans read and write their rows
    per_q2 = nstock * (16 + 64 + 32 + 32) + nsupp * (8 + 64 + 32 + 32 + 64 + 64) + \
        10000 * (8 + 111 + 128) + 62 * (8 + 185 + 192) + 5 * (8 + 207 + 224)
    achieved = per_q2 * nq / (ms * 1e-3) / 1e9
    cpu, ok = None, not ab
    if not args.no_cpu_baseline:
        import ctypes

        import oracle_lib as O
        orecs, oab = ch.query2_oracle(3)
        a, b = np.sort(recs, order="supp_key"), np.sort(orecs, order="supp_key")
        ok = ok and oab == ab and a.size == b.size and all((a[f] == b[f]).all() for f in
                                                            ("supp_key", "s_w_id", "s_i_id", "s_quantity",
                                                             "item_has_b", "update"))
        threads = min(16, os.cpu_count() or 8)
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
        "metric": "CH-benCHmark Q2 txns/s through the index-organized path (supplementary to " + METRIC + ")",
        "value": round(args.steps * nq / elapsed, 2), "unit": "q2/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int64 keys / bytes", "data": "synthetic CH rows (tpcc_record.h layouts, "
                                                                      "tpcc_loader.cpp value rules)",
        "config": {"workload": "CH-benCHmark Q2 (tpcc_new_order.cpp RunQuery2), region EUROPE",
                   "warehouses": args.warehouses, "items": args.items, "q2_per_step": nq,
                   "suppliers_visited": nsupp,
                   "stock_lookups": nstock, "aborted": bool(ab), "updates": int(recs["update"].sum())},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel": "Q2 step (3 scans + batched STOCK / ITEM probes of q2_per_step transactions)",
                     "algorithmic_bytes_per_unit": per_q2, "units_per_launch": nq, "avg_launch_ms": round(ms, 4)},
        "cpu_baseline": cpu, "self_check": bool(ok),
        "setup_s": {"load": round(load_s, 1), "sync": round(sync_s, 1)},
    }
    print(json.dumps(result), flush=True)
    return 0 if ok else 1


def main():
    args = parse()
    if args.config == "tpcc":
        return run_tpcc(args)
    if args.config == "chq2":
        return run_chq2(args)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    dist = None
    sharded = world > 1 or args.force_sharded
    if sharded:
        import torch.distributed as tdist
        tdist.init_process_group("gloo")  # control plane only; the data path is RCCL in the library
        dist = tdist
        if args.config != "c2":
            raise SystemExit("multi-GPU runs use the point-lookup config (c2 -> configs[4])")
    nthreads = min(16, os.cpu_count() or 8)
    check(stage.lib().stage_set_device(local), "set device")

    total_rows = args.rows * world
    t0 = time.time()
    tab = stage.Table(key_width=8, device=local)
    if not sharded:
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
    L = stage.lib()
    stream = stage.Stream()
    ycsb_b = None
    if args.config == "c4":
        starts = (stage.fastrandom(args.seed + rank, B) % np.uint64(total_rows)).astype(np.uint64)
        d_keys = stage.DeviceBuffer.from_numpy(starts)
        d_cnt = stage.DeviceBuffer(B * 4)
        d_rec = stage.DeviceBuffer(B * args.scan_size * tab.stride)
        draws = starts
    else:
        if args.config == "c3":
            ycsb_b = YcsbB(tab, args, nthreads)
            # epoch 0 is the warm-up (first-call allocations of the write path), untimed; every
            # timed step applies one more epoch
            draws, rids = ycsb_b.next_batch()
            ycsb_b.updates, ycsb_b.write_s, ycsb_b.sync_s = 0, 0.0, 0.0
            n_ops = draws.size
        else:
            draws = stage.zipf_draws(total_rows - 1, args.theta, args.seed + rank, B, nthreads=nthreads)
            rids = None
            n_ops = B
        d_keys = stage.DeviceBuffer(B * 8)
        check(L.stage_memcpy_h2d(d_keys.ptr, draws.ctypes.data, draws.nbytes, None), "h2d")
        d_rid = None
        if rids is not None:  # YCSB-B: the read share varies per epoch, buffers hold a whole batch
            d_rid = stage.DeviceBuffer(B * 4)
            check(L.stage_memcpy_h2d(d_rid.ptr, rids.ctypes.data, rids.nbytes, None), "h2d")
        d_out = stage.DeviceBuffer(B * 32)
        d_rec = stage.DeviceBuffer(B * tab.stride)
    d_leaf = None
    if args.host_traversal and world == 1 and args.config == "c2":
        d_leaf = stage.DeviceBuffer.from_numpy(tab.traverse(draws))

    if sharded:
        uid = (ctypes.c_uint8 * 128)()
        if rank == 0:
            check(L.stage_comm_unique_id(uid), "unique id")
        obj = [bytes(uid)]
        dist.broadcast_object_list(obj, src=0)
        uid = (ctypes.c_uint8 * 128).from_buffer_copy(obj[0])
        check(L.stage_comm_init(tab.h, uid, rank, world), "comm init")

    def step():
        if args.config == "c4":
            check(L.stage_scan_batch(tab.h, d_keys.ptr, None, B, args.scan_size, d_cnt.ptr, d_rec.ptr, stream.ptr),
                  "scan")
        elif not sharded:
            tab.probe_device(d_keys.ptr, n_ops, d_out.ptr, d_rec.ptr, d_read_ids=d_rid.ptr if d_rid else None,
                             d_leaf_ids=d_leaf.ptr if d_leaf else None, stream=stream.ptr)
        else:
            check(L.stage_probe_sharded(tab.h, d_keys.ptr, None, B, d_out.ptr, d_rec.ptr, stream.ptr), "sharded")

    for _ in range(args.warmup):
        step()
    stream.sync()
    if dist:
        dist.barrier()
    check(L.stage_device_sync(), "sync")
    evs = [stage.Event() for _ in range(2 * args.steps)]
    elapsed = 0.0
    status_hist = np.zeros(6, np.int64)
    ops_done = 0
    if ycsb_b is None:
        t0 = time.perf_counter()
        for i in range(args.steps):
            evs[2 * i].record(stream)
            step()
            evs[2 * i + 1].record(stream)
        stream.sync()
        check(L.stage_device_sync(), "sync")
        elapsed = time.perf_counter() - t0
        ops_done = B * args.steps
    else:
        # each step: one epoch's write share on the write path (timed apart, in write_s) ->
        # timed device probe of its read share
        for i in range(args.steps):
            draws, rids = ycsb_b.next_batch()
            n_ops = draws.size
            check(L.stage_memcpy_h2d(d_keys.ptr, draws.ctypes.data, draws.nbytes, None), "h2d")
            check(L.stage_memcpy_h2d(d_rid.ptr, rids.ctypes.data, rids.nbytes, None), "h2d")
            check(L.stage_device_sync(), "sync")
            t0 = time.perf_counter()
            evs[2 * i].record(stream)
            step()
            evs[2 * i + 1].record(stream)
            stream.sync()
            elapsed += time.perf_counter() - t0
            ops_done += n_ops
            o = d_out.to_numpy(stage.PROBE_OUT_DTYPE, n_ops)
            status_hist += np.bincount(o["status"], minlength=6)[:6]
    owner = None
    if dist:
        dist.barrier()
        import torch
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        # the same steps with STAGE_REPLY_OWNER: rows stay in the owner's HBM, only the 32-B
        # status records return -- the HBM-side scaling without the xGMI tuple return
        for _ in range(max(1, args.warmup)):
            check(L.stage_probe_sharded_ex(tab.h, d_keys.ptr, None, B, d_out.ptr, None, stage.REPLY_OWNER, stream.ptr),
                  "sharded owner")
        stream.sync()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            check(L.stage_probe_sharded_ex(tab.h, d_keys.ptr, None, B, d_out.ptr, None, stage.REPLY_OWNER, stream.ptr),
                  "sharded owner")
        stream.sync()
        t_own = time.perf_counter() - t0
        tt = torch.tensor([t_own], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_own = float(tt.item())
        owner = {"value": round(B * args.steps * world / t_own, 1), "ms_per_step": round(t_own / args.steps * 1e3, 4),
                 "reply": "32-B status records to the caller, tuple rows materialised on the owner"}
    step_ms = [evs[2 * i].elapsed_ms(evs[2 * i + 1]) for i in range(args.steps)]
    kern_ms = float(np.mean(step_ms))

    # self-check outside the timed region
    ok = True
    if args.config == "c4":
        cnt = d_cnt.to_numpy(np.uint32, B)
        ok = bool((cnt > 0).all() and (cnt == args.scan_size).mean() > 0.99)
    elif args.config == "c2":
        sample = min(B, 65536)
        outs = d_out.to_numpy(stage.PROBE_OUT_DTYPE, sample)
        rows = d_rec.to_numpy(np.uint8, sample * tab.stride).reshape(sample, tab.stride)
        ok = bool((outs["status"] == stage.ST_LATEST).all() and
                  (rows[:, :8].copy().view(np.uint64).ravel() == draws[:sample]).all() and
                  (rows[:, 8:1008] == (draws[:sample] & np.uint64(0xFF)).astype(np.uint8)[:, None]).all())
    else:
        ok = bool(status_hist[stage.ST_LATEST] > 0 and status_hist[stage.ST_OLD] > 0)
    if not ok:
        log(f"[rank {rank}] SELF-CHECK FAILED")

    total = ops_done * world
    value = total / elapsed
    if rank == 0:
        if args.config == "c4":
            per_unit = scan_bytes(args.scan_size)
            unit = "scans/s"
            kernel = "scan_kernel"
        else:
            per_unit = BYTES_PER_LOOKUP
            unit = "ops/s"
            kernel = "probe_kernel" if not sharded else "sharded step (route + RCCL + probe_kernel)"
        units_per_launch = ops_done / args.steps
        achieved = per_unit * units_per_launch / (kern_ms * 1e-3) / 1e9
        traffic, tsrc = None, None
        if not sharded and args.config in ("c2", "c4"):
            traffic, tsrc = traffic_from_profile(B, args.rows, "pmc_probe.json" if args.config == "c2" else
                                                 "pmc_scan.json")
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": kernel,
                "algorithmic_bytes_per_unit": per_unit, "units_per_launch": units_per_launch,
                "algorithmic_bytes_per_launch": round(per_unit * units_per_launch),
                "avg_launch_ms": round(kern_ms, 4)}
        if tsrc:
            roof["traffic_source"] = tsrc
        if sharded and world > 1:
            roof = xgmi_roofline(B, world, tab.stride, elapsed / args.steps, roof)
        cpu = None
        if not sharded and not args.no_cpu_baseline:
            cpu = cpu_baseline(args, nthreads)
        wl = WORKLOADS[args.config] if not sharded else WORKLOADS["c5"]
        config = {"workload": wl, "rows_per_gpu": args.rows, "rows_total": total_rows, "batch_per_gpu": B,
                  "key_bytes": 8, "payload_bytes": 1000, "leaf_bytes": 65536,
                  "parallelism": f"hash-shard x{world}", "traversal": "host" if d_leaf else "device"}
        if args.config == "c4":
            config.update({"scan_size": args.scan_size, "starts": "uniform over [0, N)"})
        else:
            config["theta"] = args.theta
        if ycsb_b is not None:
            config.update({"update_ratio": args.update_ratio, "updates_applied": ycsb_b.updates,
                           "write_path": args.write_path,
                           "write_s": round(ycsb_b.write_s, 3), "publish_s": round(ycsb_b.sync_s, 3),
                           "epoch_prep_s_untimed": round(ycsb_b.prep_s, 2),
                           "last_publish": ycsb_b.last_sync,
                           "ops_per_s_incl_writes": round((ops_done + ycsb_b.updates) /
                                                               (elapsed + ycsb_b.write_s), 1),
                           "read_status_counts": {"latest": int(status_hist[1]), "copy": int(status_hist[2]),
                                                  "old": int(status_hist[3]), "fail": int(status_hist[4]),
                                                  "chain_miss": int(status_hist[5]),
                                                  "not_found": int(status_hist[0])},
                           "timed": "device probe of the read share; the epoch's write path between steps excluded "
                                    "(it is in ops_per_s_incl_writes: update share over PCIe + write path)"})
        result = {
            "metric": METRIC, "value": round(value, 1), "unit": unit, "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic (LoadYCSBRows keys/payloads)",
            "config": config, "roofline": roof, "cpu_baseline": cpu, "self_check": ok,
            **({"owner_reply": owner} if owner else {}),
            "setup_s": {"load": round(t_load, 1), "sync": round(t_sync, 1)},
            "host_peak_rss_gib": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20, 1),
        }
        print(json.dumps(result), flush=True)
    if dist:
        dist.barrier()
        check(L.stage_comm_destroy(tab.h), "comm destroy")
        dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
