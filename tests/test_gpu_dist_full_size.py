"""BASELINE.json configs[4] (YCSB-C sharded 8 ways over RCCL, MurmurHash64A(key, 8, 0) % 8) at
size on ONE device: the multi-GPU data path (request coalescing of the whole batch, routing,
count exchange, chunked key / result exchange, the owners' fan-out probes, the fan-out of
returned rows) run by stage_probe_sharded_loopback over W = 8 shard tables of 12.5M rows each
(100M rows in all, the keys each rank of C5 owns), fed a 2^24-key Zipf-0.9 batch (2^21 keys per
rank, drawn over all 100M keys as C5's ranks draw them), must return byte for byte what ONE
100M-row table returns for the same keys -- in the three reply modes (rows back to the caller,
rows read by the caller from the owners' row buffers, rows left at the owner), coalescing on.  The direct probe's results are taken first and the
100M-row table is released before the shards are built (both at once would not leave room for
the exchange buffers in 288 GB).  Reference semantics: executor.h:374-454 (IndexScanExecutor
point lookup) through BTree::Read (b_tree.cpp:2066-2129) on every shard."""
import sys
import time

import numpy as np
import pytest

import oracle_lib as O
import stage
from progress import say

pytestmark = pytest.mark.gpu

N = 100_000_000
W = 8
PER_RANK = 1 << 21  # 2^24 keys in all


def _say(t0, what):  # progress (stderr + gpurun_out/progress.log): each phase takes tens of seconds
    say(f"[c5 at size] {what}", t0)


@pytest.mark.timeout(900)
def test_c5_loopback_at_size_equals_one_table(gpu):
    t0 = time.time()
    rng = np.random.default_rng(0xC5)
    per_keys = []
    for r in range(W):
        k = stage.zipf_draws(N - 1, 0.9, 0x5EED + r, PER_RANK - 64, nthreads=16)
        absent = rng.integers(N, N + 10_000_000, 64).astype(np.uint64)
        k = np.concatenate([k, absent])
        per_keys.append(k[rng.permutation(k.size)].astype(np.uint64))
    # 1. the direct probe of one 100M-row table (LoadYCSBRows rows)
    _say(t0, "batches drawn")
    full = stage.Table(key_width=8)
    assert full.load_ycsb(0, N, 8, 0) == N
    full.sync()
    _say(t0, "100M-row table loaded")
    ref = [full.probe(k) for k in per_keys]
    _say(t0, "direct probes done")
    full.close()
    del full
    # 2. the shards: rank r holds the keys with MurmurHash64A(key, 8, 0) % 8 == r, ascending
    keys = np.arange(N, dtype=np.uint64)
    own = O.murmur64a_keys(keys, 8, 0) % np.uint64(W)
    tabs = []
    for r in range(W):
        t = stage.Table(key_width=8)
        mine = keys[own == np.uint64(r)]
        assert t.load_keys(mine, 8, mode=0) == mine.size
        t.sync()
        tabs.append(t)
        _say(t0, f"shard {r} loaded ({mine.size} rows)")
    del keys, own
    for t in tabs:
        stage.set_shard_dedupe(t, 1)
    fields = ("status", "flags", "hops", "key_len", "cstamp", "rec_cstamp", "copy_sstamp")
    # 3. rows back to the caller
    res = stage.probe_sharded_loopback(tabs, per_keys, None)
    _say(t0, "sharded probe, rows mode")
    routed = 0
    for r in range(W):
        out, rows = res[r]
        ref_out, ref_rows = ref[r]
        for f in fields:
            assert (out[f] == ref_out[f]).all(), (r, f)
        assert (rows == ref_rows).all(), r
        nk, rt, remote = stage.sharded_stats(tabs[r])
        assert nk == per_keys[r].size and remote < rt < 0.8 * nk  # Zipf duplicates coalesced
        routed += rt
    assert (np.concatenate([o["status"] for o, _ in res]) == stage.ST_LATEST).sum() == W * (PER_RANK - 64)
    del res
    # 3b. peer reply: status records back, rows read from the owners' row buffers (STAGE_REPLY_PEER)
    res = stage.probe_sharded_loopback(tabs, per_keys, None, reply=stage.REPLY_PEER)
    _say(t0, "sharded probe, peer mode")
    for r in range(W):
        out, rows = res[r]
        ref_out, ref_rows = ref[r]
        for f in fields:
            assert (out[f] == ref_out[f]).all(), (r, f)
        assert (rows == ref_rows).all(), r
    del res
    # 3c. direct reply: each owner writes its rows into the callers' outputs (STAGE_REPLY_DIRECT)
    res = stage.probe_sharded_loopback(tabs, per_keys, None, reply=stage.REPLY_DIRECT)
    _say(t0, "sharded probe, direct mode")
    for r in range(W):
        out, rows = res[r]
        ref_out, ref_rows = ref[r]
        for f in fields:
            assert (out[f] == ref_out[f]).all(), (r, f)
        assert (rows == ref_rows).all(), r
    del res
    # 4. rows left at their owners, status records back (each carries the owner-local row index)
    res = stage.probe_sharded_loopback(tabs, per_keys, None, records=True, reply=stage.REPLY_OWNER)
    _say(t0, "sharded probe, owner mode")
    owner_rows = []
    for t in tabs:
        ptr, cnt = stage.owner_rows(t, loopback=True)
        buf = np.zeros(cnt * t.stride, np.uint8)
        stage.table.check(stage.lib().stage_memcpy_d2h(buf.ctypes.data, ptr, buf.nbytes, None), "d2h")
        owner_rows.append(buf.reshape(cnt, t.stride))
    assert sum(b.shape[0] for b in owner_rows) == routed
    for r in range(W):
        out, _ = res[r]
        ref_out, ref_rows = ref[r]
        for f in ("status", "cstamp", "rec_cstamp"):
            assert (out[f] == ref_out[f]).all(), (r, f)
        o = (O.murmur64a_keys(per_keys[r], 8, 0) % np.uint64(W)).astype(np.int64)
        hit = out["status"] != stage.ST_NOT_FOUND
        for w in range(W):
            sel = np.nonzero((o == w) & hit)[0]
            assert (owner_rows[w][out["meta_hi"][sel]] == ref_rows[sel]).all(), (r, w)
    for t in tabs:
        stage.set_shard_dedupe(t, -1)
        t.close()
