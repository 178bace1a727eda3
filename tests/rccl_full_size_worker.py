"""One rank of BASELINE.json configs[4]'s data path at size over a REAL 8-rank RCCL communicator
on one GPU (driven by tests/test_gpu_rccl_full_size.py; not a test module itself).

Rank r loads its shard -- the keys k < N with MurmurHash64A(k, 8, 0) % W == r, LoadYCSBRows rows
(memset(rowid) payloads) -- and probes its 2^21-key Zipf-0.9 batch (drawn over all N keys, as a
C5 rank draws it) through stage_probe_sharded_ex, rows back to the caller and rows left at the
owner.  The reference is ONE N-row table's direct probe of the same keys, taken by the parent
before any rank started and saved to OUTDIR: the 32-B status records and a 64-bit digest per
row.  Every status field and every row digest must match (owner mode: the row each status
record names in its owner's buffer, whose digests every owner saves).  Ranks share device 0 with
their own NCCL_HOSTID (RCCL's socket transport on the loopback interface), as
tests/rccl_rank_worker.py.  Writes OUTDIR/rank{r}.json with the per-step times.

Env: RANK, WORLD_SIZE, OUTDIR, N."""
import ctypes
import json
import os
import sys
import time
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if __name__ == "__main__":  # a rank (the test module imports digest() only)
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    outdir = os.environ["OUTDIR"]
    os.environ["NCCL_HOSTID"] = f"stage-c5-{os.getppid()}-rank{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_NET", "Socket")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
sys.path.insert(0, os.path.join(REPO, "stage-indexorganized_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402

import stage  # noqa: E402
from progress import say  # noqa: E402
from stage._lib import check  # noqa: E402

FIELDS = ("status", "flags", "hops", "key_len", "cstamp", "rec_cstamp", "copy_sstamp")


def digest(rows):
    """64-bit digest per row (u64 words times odd weights, wrapping) -- the parent's function"""
    w = rows.view(np.uint64)
    weights = (np.arange(w.shape[1], dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)) | np.uint64(1)
    return (w * weights).sum(axis=1, dtype=np.uint64)


def wait_file(path, timeout=600):
    t_end = time.time() + timeout
    while not os.path.exists(path):
        if time.time() > t_end:
            raise RuntimeError(f"rank {rank}: timed out waiting for {path}")
        time.sleep(0.05)


def main():
    n = int(os.environ["N"])
    t0 = time.time()
    L = stage.lib()
    check(L.stage_set_device(0), "device")
    keys = np.arange(n, dtype=np.uint64)
    own = keys[(stage.murmur64a_device(keys, 8, 0) % np.uint64(world)) == np.uint64(rank)]
    del keys
    shard = stage.Table(key_width=8)
    assert shard.load_keys(own, 8, mode=0) == own.size
    shard.sync()
    say(f"rank {rank}: shard of {own.size} rows loaded", t0)
    uid = (ctypes.c_uint8 * 128)()
    uid_path = os.path.join(outdir, "uid.bin")
    if rank == 0:
        check(L.stage_comm_unique_id(uid), "uid")
        with open(uid_path + ".tmp", "wb") as f:
            f.write(bytes(uid))
        os.replace(uid_path + ".tmp", uid_path)
    else:
        wait_file(uid_path)
        uid = (ctypes.c_uint8 * 128).from_buffer_copy(open(uid_path, "rb").read())
    check(L.stage_comm_init(shard.h, uid, rank, world), "comm init")
    stage.set_shard_key_bits(shard, max(1, int(n).bit_length()))
    stage.set_shard_dedupe(shard, 1)
    report = {"rank": rank, "world": world, "rows": int(own.size), "rccl": stage.rccl_info(), "cases": []}
    k = np.load(os.path.join(outdir, f"keys{rank}.npy"))
    ref_out = np.load(os.path.join(outdir, f"out{rank}.npy"))
    ref_dig = np.load(os.path.join(outdir, f"dig{rank}.npy"))
    nk = k.size
    d_keys = stage.DeviceBuffer.from_numpy(k)
    d_out = stage.DeviceBuffer(nk * 32)
    d_rec = stage.DeviceBuffer(nk * shard.stride)
    ok = True
    for reply in (stage.REPLY_ROWS, stage.REPLY_OWNER, stage.REPLY_PEER, stage.REPLY_DIRECT):
        name = {stage.REPLY_OWNER: "owner", stage.REPLY_PEER: "peer", stage.REPLY_DIRECT: "direct"}.get(reply, "rows")
        times = []
        for it in range(3):  # the first call grows the exchange buffers; all three are checked alike
            stage.comm_allreduce(shard, [1.0])  # barrier
            ts = time.perf_counter()
            check(L.stage_probe_sharded_ex(shard.h, d_keys.ptr, None, nk, d_out.ptr,
                                           d_rec.ptr if reply != stage.REPLY_OWNER else None, reply, None), "sharded")
            check(L.stage_device_sync(), "sync")
            times.append(time.perf_counter() - ts)
        st = stage.sharded_stats_ex(shard)
        out = d_out.to_numpy(stage.PROBE_OUT_DTYPE, nk)
        case = {"reply": name, "keys": int(nk), "step_s": [round(x, 4) for x in times],
                "stats": {kk: int(v) for kk, v in st.items()}}
        good = True
        for f in (FIELDS if reply != stage.REPLY_OWNER else ("status", "cstamp", "rec_cstamp")):
            if not (out[f] == ref_out[f]).all():
                good = False
                case.setdefault("mismatch", []).append(f)
        if reply != stage.REPLY_OWNER:
            rows = d_rec.to_numpy(np.uint8, nk * shard.stride).reshape(nk, shard.stride)
            if not (digest(rows) == ref_dig).all():
                good = False
                case.setdefault("mismatch", []).append("rows")
            del rows
        else:
            ptr, cnt = stage.owner_rows(shard, loopback=False)
            buf = np.zeros(cnt * shard.stride, np.uint8)
            if cnt:
                check(L.stage_memcpy_d2h(buf.ctypes.data, ptr, buf.nbytes, None), "d2h")
            np.save(os.path.join(outdir, f"owner_dig{rank}.npy"), digest(buf.reshape(cnt, shard.stride)))
            del buf
            stage.comm_allreduce(shard, [1.0])  # every owner's digests are on disk
            kh = (stage.murmur64a_device(k, 8, 0) % np.uint64(world)).astype(np.int64)
            hit = out["status"] != stage.ST_NOT_FOUND
            for o in range(world):
                od = np.load(os.path.join(outdir, f"owner_dig{o}.npy"))
                sel = np.nonzero((kh == o) & hit)[0]
                if not (od[out["meta_hi"][sel]] == ref_dig[sel]).all():
                    good = False
                    case.setdefault("mismatch", []).append(f"owner rows from rank {o}")
        case["ok"] = good
        ok &= good
        report["cases"].append(case)
        say(f"rank {rank}: {name} reply {'ok' if good else 'MISMATCH'}, steps {case['step_s']} s, {case['stats']}", t0)
    report["all_ranks_ok"] = bool(stage.comm_allreduce(shard, [1.0 if ok else 0.0], "min")[0] > 0.5)
    stage.comm_allreduce(shard, [1.0])
    check(L.stage_comm_destroy(shard.h), "destroy")
    report["ok"] = ok
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump(report, f)
    return 0 if ok else 1


if __name__ == "__main__":
    try:
        sys.exit(main())
    except Exception:
        traceback.print_exc()
        with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
            json.dump({"rank": rank, "ok": False, "error": traceback.format_exc()}, f)
        sys.exit(1)
