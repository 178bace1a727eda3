"""CPU, world_size 2 over gloo: the multi-GPU front-end's partition and routing logic.

Each rank owns the keys with MurmurHash64A(key, 8, 0) % world == rank (the router of
csrc/dist.hip), loads them in ascending order into its own host table, and answers the
keys routed to it by an all-to-all.  Checks: shards are disjoint and cover the key space,
every routed key lands on the rank whose table holds it, and the per-shard leaf layout is
what a single loader would build for that shard (against the oracle).  No GPU is touched.
"""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

# torch is imported inside the (spawned) workers only, not at collection: a `pytest -m gpu` run
# collects this module too, and a torch imported there would bring its own HIP runtime and RCCL
# into the process before libstage_hip's (stage_rccl_info / stage_comm_init check the RCCL)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, q):
    import sys

    import torch
    import torch.distributed as dist
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(repo, "stage-indexorganized_amd"))
    sys.path.insert(0, os.path.join(repo, "tests"))
    import oracle_lib as O
    import stage
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        keys = np.arange(total, dtype=np.uint64)
        h = O.murmur64a_keys(keys, 8, 0)
        mine = keys[(h % np.uint64(world)) == np.uint64(rank)]
        tab = stage.Table(key_width=8)
        assert tab.load_keys(mine, 8, 0) == mine.size
        counts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(counts, torch.tensor([mine.size]))
        assert sum(int(c) for c in counts) == total
        # route a probe batch (including absent keys) with an all-to-all, as dist.hip does
        probes = np.random.default_rng(100 + rank).integers(0, total + total // 10, 20000).astype(np.uint64)
        dest = (O.murmur64a_keys(probes, 8, 0) % np.uint64(world)).astype(np.int64)
        order = np.argsort(dest, kind="stable")
        send = torch.from_numpy(probes[order].view(np.int64).copy())
        scount = torch.tensor(np.bincount(dest, minlength=world), dtype=torch.int64)
        rcount = torch.zeros(world, dtype=torch.int64)
        dist.all_to_all_single(rcount, scount)
        recv = torch.zeros(int(rcount.sum()), dtype=torch.int64)
        dist.all_to_all_single(recv, send, rcount.tolist(), scount.tolist())
        got = recv.numpy().view(np.uint64)
        # every routed key that exists must be in this rank's shard; insert reports KEY_EXISTS
        present = got < total
        for k in got[present][:2000]:
            assert tab.insert(int(k), 8) == stage.RC_KEY_EXISTS
        assert ((O.murmur64a_keys(got, 8, 0) % np.uint64(world)) == np.uint64(rank)).all()
        # shard layout == a single loader's layout for the shard
        orc = O.OracleTree()
        orc.load_keys(mine, 8, 0)
        rc, sc, meta, keyw = tab.export_leaves(64)
        orc_rc, orc_sc, orc_meta, orc_keyw = orc.export_leaves(64)
        assert (rc == orc_rc).all() and (meta == orc_meta).all() and (keyw == orc_keyw).all()
        q.put((rank, "ok"))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_two_rank_routing_gloo():
    world, total = 2, 200_000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    res = dict(q.get(timeout=5) for _ in range(world))
    assert res == {0: "ok", 1: "ok"}, res
    assert all(p.exitcode == 0 for p in procs)
