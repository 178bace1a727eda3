"""One rank of a real multi-rank RCCL run of the sharded probe (driven by
tests/test_gpu_rccl_ranks.py; not a test module itself).

Every rank runs on device 0 of a one-GPU box: RCCL refuses two ranks of one host on one device,
so each rank gets its own NCCL_HOSTID and the exchange runs over RCCL's socket transport on the
loopback interface.  The calls are the real ones of the multi-GPU path -- the counts
ncclAllToAll, grouped ncclSend / ncclRecv with peers, the control-plane allreduce / allgather --
which the one-device loopback tests replace by device copies.

Rank r loads its shard (MurmurHash64A(key, 8, 0) % W == r of N keys, version chains on a set of
hot keys) and one table holding every key, probes its own batch (missing keys, hot keys, read
ids) through stage_probe_sharded in several settings, and compares every status field and row
with the full table's direct probe.  Owner-reply rows are checked across processes through
files in OUTDIR.  Writes OUTDIR/rank{r}.json; exit status 0 iff every check passed.

Env: RANK, WORLD_SIZE, OUTDIR (shared by the ranks), N (keys, default 300000)."""
import ctypes
import json
import os
import sys
import time
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
outdir = os.environ["OUTDIR"]
# before the first RCCL call of this process (see bench.share_gpu_rehearsal)
os.environ["NCCL_HOSTID"] = f"stage-test-{os.getppid()}-rank{rank}"
os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
os.environ.setdefault("NCCL_NET", "Socket")
os.environ.setdefault("NCCL_IB_DISABLE", "1")
sys.path.insert(0, os.path.join(REPO, "stage-indexorganized_amd"))

import numpy as np  # noqa: E402

import stage  # noqa: E402
from stage._lib import check  # noqa: E402

FIELDS = ("status", "flags", "hops", "key_len", "cstamp", "rec_cstamp", "copy_sstamp")


def wait_file(path, timeout=300):
    t_end = time.time() + timeout
    while not os.path.exists(path):
        if time.time() > t_end:
            raise RuntimeError(f"rank {rank}: timed out waiting for {path}")
        time.sleep(0.05)


def main():
    n = int(os.environ.get("N", 300_000))
    L = stage.lib()
    check(L.stage_set_device(0), "device")
    keys = np.arange(n, dtype=np.uint64)
    h = stage.murmur64a_device(keys, 8, 0)
    own_mask = (h % np.uint64(world)) == np.uint64(rank)
    shard = stage.Table(key_width=8)
    shard.load_keys(keys[own_mask], 8, mode=1)
    full = stage.Table(key_width=8)
    full.load_keys(keys, 8, mode=1)
    rng_hot = np.random.default_rng(4242)  # same hot keys on every rank
    hot = rng_hot.choice(n, 2000, replace=False).astype(np.uint64)
    for k in hot:
        tabs = [full] + ([shard] if own_mask[int(k)] else [])
        for t in tabs:
            assert t.update(int(k), 16, b"\x42" * 32, 10) == stage.RC_OK
            assert t.commit_update(int(k), 11, 11) == stage.RC_OK
    shard.sync()
    full.sync()

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
    stage.set_shard_key_bits(shard, max(1, int(n + 30_000).bit_length()))
    report = {"rank": rank, "world": world, "rccl": stage.rccl_info(), "cases": []}

    def barrier():
        stage.comm_allreduce(shard, [1.0])

    rng = np.random.default_rng(1000 + rank)
    ok = True
    # (chunks, dedupe, read ids, reply, batch size): rank world-1 probes nothing in one case (it
    # still takes part in every exchange)
    # STAGE_REPLY_PEER: rows read through the owners' IPC-mapped row buffers (two parities: the
    # case runs its probe twice, as every case does); STAGE_REPLY_DIRECT: the owners write into
    # the callers' IPC-mapped outputs (each case allocates new ones: the mappings move with them)
    cases = [(1, 1, True, stage.REPLY_ROWS, 60_000), (4, 1, True, stage.REPLY_ROWS, 90_000),
             (3, 0, False, stage.REPLY_ROWS, 40_000), (4, 1, False, stage.REPLY_OWNER, 50_000),
             (2, 1, True, stage.REPLY_ROWS, 0 if rank == world - 1 else 30_000),
             (4, 1, True, stage.REPLY_PEER, 80_000), (2, 0, False, stage.REPLY_PEER, 0 if rank == 0 else 35_000),
             (4, 1, True, stage.REPLY_DIRECT, 80_000), (2, 0, False, stage.REPLY_DIRECT, 0 if rank == 1 else 35_000),
             (3, 1, False, stage.REPLY_DIRECT, 45_000)]
    for ci, (chunks, dedupe, use_rids, reply, size) in enumerate(cases):
        print(f"[case {ci}] reply {reply}, chunks {chunks}, dedupe {dedupe}, keys {size}", flush=True)
        check(L.stage_set_shard_chunks(shard.h, chunks), "chunks")
        stage.set_shard_dedupe(shard, dedupe)
        if size:
            k = np.concatenate([rng.integers(0, n + 30_000, size), rng.choice(hot, 2000),
                                np.repeat(rng.integers(0, n, 8), 300)]).astype(np.uint64)
            k = k[rng.permutation(k.size)]
        else:
            k = np.zeros(0, np.uint64)
        rids = rng.integers(0, 14, k.size).astype(np.uint32) if use_rids else None
        nk = k.size
        d_keys = stage.DeviceBuffer.from_numpy(k) if nk else None
        d_rids = stage.DeviceBuffer.from_numpy(rids) if (use_rids and nk) else None
        d_out = stage.DeviceBuffer(max(nk, 1) * 32)
        d_rec = stage.DeviceBuffer(max(nk, 1) * shard.stride) if reply != stage.REPLY_OWNER else None
        for _ in range(2):  # the second call reuses grown scratch buffers
            check(L.stage_probe_sharded_ex(shard.h, d_keys.ptr if d_keys else None, d_rids.ptr if d_rids else None,
                                           nk, d_out.ptr, d_rec.ptr if d_rec else None, reply, None), "sharded")
            check(L.stage_device_sync(), "sync")
        st = stage.sharded_stats_ex(shard)
        case = {"case": ci, "chunks": chunks, "dedupe": dedupe, "read_ids": use_rids,
                "reply": {stage.REPLY_OWNER: "owner", stage.REPLY_PEER: "peer",
                          stage.REPLY_DIRECT: "direct"}.get(reply, "rows"), "keys": nk,
                "stats": {kk: int(v) for kk, v in st.items()} if isinstance(st, dict) else str(st)}
        good = True
        if nk:
            out = d_out.to_numpy(stage.PROBE_OUT_DTYPE, nk)
            ref_out, ref_rows = full.probe(k, read_ids=rids)
            for f in FIELDS if reply != stage.REPLY_OWNER else ("status", "cstamp"):
                if not (out[f] == ref_out[f]).all():
                    good = False
                    case.setdefault("mismatch", []).append(f)
            if reply != stage.REPLY_OWNER:
                rows = d_rec.to_numpy(np.uint8, nk * shard.stride).reshape(nk, shard.stride)
                if not (rows == ref_rows).all():
                    good = False
                    case.setdefault("mismatch", []).append("rows")
        if reply == stage.REPLY_OWNER:
            # every owner publishes the rows it kept; callers read them at the index the status
            # record carries (meta_hi), owner = the key's shard
            ptr, cnt = stage.owner_rows(shard, loopback=False)
            buf = np.zeros(cnt * shard.stride, np.uint8)
            if cnt:
                check(L.stage_memcpy_d2h(buf.ctypes.data, ptr, buf.nbytes, None), "d2h")
            np.save(os.path.join(outdir, f"owner{ci}_{rank}.npy"), buf.reshape(cnt, shard.stride))
            barrier()
            if nk:
                owners = [np.load(os.path.join(outdir, f"owner{ci}_{o}.npy")) for o in range(world)]
                kh = (stage.murmur64a_device(k, 8, 0) % np.uint64(world)).astype(np.int64)
                for o in range(world):
                    sel = np.nonzero(kh == o)[0]
                    hit = out["status"][sel] != stage.ST_NOT_FOUND
                    got = owners[o][out["meta_hi"][sel][hit]]
                    if not (got == ref_rows[sel][hit]).all():
                        good = False
                        case.setdefault("mismatch", []).append(f"owner rows from rank {o}")
            barrier()
        case["ok"] = good
        ok &= good
        report["cases"].append(case)
        for b in (d_keys, d_rids, d_out, d_rec):
            if b is not None:
                b.free()
    # every rank agrees on the outcome
    report["all_ranks_ok"] = bool(stage.comm_allreduce(shard, [1.0 if ok else 0.0], "min")[0] > 0.5)
    barrier()
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
