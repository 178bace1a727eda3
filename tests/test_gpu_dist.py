"""GPU: the sharded probe front-end.  stage_probe_sharded on a one-rank RCCL communicator
returns exactly what the direct probe returns (coalescing, routing, the fan-out probe of own
requests); the same data path with W = 2, 3, 8 shards on one device
(stage_probe_sharded_loopback) returns what one table holding every key returns -- with and
without coalescing, hot keys beyond one request's 64 callers, read ids interleaved with keys,
and tables outside the fan-out probe's geometry (probed, then fanned out by fan_copy)."""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
import stage
from stage._lib import check

pytestmark = pytest.mark.gpu


def test_sharded_world1_equals_direct(gpu):
    tab = stage.Table(key_width=8)
    tab.load_ycsb(0, 1_000_000, 8, mode=1)
    tab.sync()
    L = stage.lib()
    uid = (ctypes.c_uint8 * 128)()
    check(L.stage_comm_unique_id(uid), "uid")
    check(L.stage_comm_init(tab.h, uid, 0, 1), "init")
    try:
        keys = np.random.default_rng(0).integers(0, 1_100_000, 300_000).astype(np.uint64)
        rids = np.random.default_rng(1).integers(0, 1 << 32, keys.size).astype(np.uint32)
        d_keys = stage.DeviceBuffer.from_numpy(keys)
        d_rids = stage.DeviceBuffer.from_numpy(rids)
        d_out = stage.DeviceBuffer(keys.size * 32)
        d_rec = stage.DeviceBuffer(keys.size * tab.stride)
        for _ in range(2):  # second call reuses the grown scratch buffers
            check(L.stage_probe_sharded(tab.h, d_keys.ptr, d_rids.ptr, keys.size, d_out.ptr, d_rec.ptr, None), "sh")
            check(L.stage_device_sync(), "sync")
        out = d_out.to_numpy(stage.PROBE_OUT_DTYPE, keys.size)
        rows = d_rec.to_numpy(np.uint8, keys.size * tab.stride).reshape(keys.size, tab.stride)
        ref_out, ref_rows = tab.probe(keys, read_ids=rids)
        assert (out == ref_out).all()
        assert (rows == ref_rows).all()
    finally:
        check(L.stage_comm_destroy(tab.h), "destroy")


def shard_tables(keys, world, mode=1, payload=1000):
    """Rank r's shard: the keys with MurmurHash64A(key, 8, 0) % world == r, in ascending order."""
    h = O.murmur64a_keys(keys, 8, 0)
    tabs = []
    for r in range(world):
        t = stage.Table(key_width=8, payload_size=payload)
        t.load_keys(keys[(h % np.uint64(world)) == np.uint64(r)], 8, mode=mode)
        tabs.append(t)
    return tabs, h


@pytest.mark.parametrize("world,chunks,dedupe,reply", [(2, 1, 1, 0), (3, 4, 1, 0), (8, 7, 1, 0), (3, 4, 0, 0),
                                                        (2, 1, 1, 2), (3, 4, 1, 2), (8, 7, 1, 2), (3, 4, 0, 2),
                                                        (2, 1, 1, 3), (3, 4, 1, 3), (8, 7, 1, 3), (3, 4, 0, 3)])
def test_sharded_data_path_loopback_equals_single_table(gpu, world, chunks, dedupe, reply):
    # reply 2 = STAGE_REPLY_PEER: status records travel back, each row is read by the caller's
    # fan-out where its owner left it (here: the other shard's row buffer in place of an IPC map);
    # reply 3 = STAGE_REPLY_DIRECT: each owner probes a remote request straight into its
    # caller's output at the request's first caller position, the caller copies the duplicates
    # the multi-GPU data path (routing, count exchange, all-to-all-v offsets, local probes,
    # reverse exchange, un-permutation) with W shards on one device, against one table
    # holding every key; version chains on some keys so statuses and rows vary
    n = 400_000
    keys = np.arange(n, dtype=np.uint64)
    tabs, h = shard_tables(keys, world)
    full = stage.Table(key_width=8)
    full.load_keys(keys, 8, mode=1)
    orc = O.OracleTree(payload_size=1000)  # the same table in the oracle: a direct pin
    orc.load_ycsb_bulk(0, n, 8, 1)
    rng = np.random.default_rng(world)
    hot = rng.choice(n, 3000, replace=False).astype(np.uint64)
    for k in hot:
        owner = tabs[int(h[int(k)] % np.uint64(world))]
        for t in (owner, full):
            assert t.update(int(k), 16, b"\x42" * 32, 10) == stage.RC_OK
            assert t.commit_update(int(k), 11, 11) == stage.RC_OK
        assert orc.update(int(k), 8, 16, b"\x42" * 32, 10) == stage.RC_OK
        assert orc.commit_update(int(k), 8, 11, 11) == stage.RC_OK
    for t in tabs + [full]:
        t.sync()
    for t in tabs:
        check(stage.lib().stage_set_shard_chunks(t.h, chunks), "chunks")
        stage.set_shard_dedupe(t, dedupe)
    sizes = [int(x) for x in rng.integers(1, 120_000, world)]
    sizes[-1] = 0  # a rank with nothing to probe still takes part in the exchange
    per_keys = [np.concatenate([rng.integers(0, n + 20_000, s), rng.choice(hot, min(s, 500))]).astype(np.uint64)
                if s else np.zeros(0, np.uint64) for s in sizes]
    per_rids = [rng.integers(0, 14, k.size).astype(np.uint32) for k in per_keys]
    res = stage.probe_sharded_loopback(tabs, per_keys, per_rids, reply=reply)
    if reply in (stage.REPLY_PEER, stage.REPLY_DIRECT):  # a second call: the other parity / fresh buffers
        res = stage.probe_sharded_loopback(tabs, per_keys, per_rids, reply=reply)
    for r in range(world):
        out, rows = res[r]
        if per_keys[r].size == 0:
            assert out.size == 0
            continue
        ref_out, ref_rows = full.probe(per_keys[r], read_ids=per_rids[r])
        for f in ("status", "flags", "hops", "key_len", "cstamp", "rec_cstamp", "copy_sstamp"):
            assert (out[f] == ref_out[f]).all(), (world, r, f)
        assert (rows == ref_rows).all(), (world, r)
        for i in rng.choice(per_keys[r].size, min(400, per_keys[r].size), replace=False):  # and the oracle's
            o, rec = orc.read(int(per_keys[r][i]), 8, int(per_rids[r][i]))
            assert (out["status"][i], out["cstamp"][i]) == (o["status"], o["cstamp"]), (world, r, i)
            assert (rows[i, :orc.row] == rec).all(), (world, r, i)
    # and a second round reuses the grown scratch buffers, without rows
    res2 = stage.probe_sharded_loopback(tabs, per_keys, None, records=False)
    for r in range(world):
        if per_keys[r].size:
            ref_out, _ = full.probe(per_keys[r], records=False)
            assert (res2[r][0]["status"] == ref_out["status"]).all()


@pytest.mark.parametrize("dedupe", [1, 0])
def test_owner_reply_mode_loopback(gpu, dedupe):
    # STAGE_REPLY_OWNER: only status records travel back; each row stays in its owner's result
    # buffer at the index the record carries.  Repeated keys: coalesced, a caller's request may
    # sit in any exchange chunk (the status records are expanded once every chunk is back)
    world, n = 4, 200_000
    keys = np.arange(n, dtype=np.uint64)
    tabs, h = shard_tables(keys, world)
    full = stage.Table(key_width=8)
    full.load_keys(keys, 8, mode=1)
    for t in tabs + [full]:
        t.sync()
    rng = np.random.default_rng(77)
    for t in tabs:
        stage.set_shard_dedupe(t, dedupe)
    per_keys = []
    for r in range(world):
        k = np.concatenate([rng.integers(0, n + 5000, 30_000 + 1000 * r), np.repeat(rng.integers(0, n, 20), 150)])
        per_keys.append(k[rng.permutation(k.size)].astype(np.uint64))
    res = stage.probe_sharded_loopback(tabs, per_keys, None, records=True, reply=stage.REPLY_OWNER)
    owner_bufs = []
    for t in tabs:
        ptr, cnt = stage.owner_rows(t, loopback=True)
        buf = np.zeros(cnt * t.stride, np.uint8)
        check(stage.lib().stage_memcpy_d2h(buf.ctypes.data, ptr, buf.nbytes, None), "d2h")
        owner_bufs.append(buf.reshape(cnt, t.stride))
    # one owner row per routed request (equal keys of the batch are coalesced)
    routed = [stage.sharded_stats(t)[1] for t in tabs]
    assert sum(b.shape[0] for b in owner_bufs) == sum(routed) <= sum(k.size for k in per_keys)
    assert (sum(routed) < sum(k.size for k in per_keys)) == bool(dedupe)
    for r in range(world):
        out, rows = res[r]
        ref_out, ref_rows = full.probe(per_keys[r])
        assert (out["status"] == ref_out["status"]).all() and (out["cstamp"] == ref_out["cstamp"]).all()
        own = (O.murmur64a_keys(per_keys[r], 8, 0) % np.uint64(world)).astype(np.int64)
        for o in range(world):
            sel = np.nonzero(own == o)[0]
            got = owner_bufs[o][out["meta_hi"][sel]]
            hit = out["status"][sel] != stage.ST_NOT_FOUND
            assert (got[hit] == ref_rows[sel][hit]).all()
    for t in tabs:
        stage.set_shard_dedupe(t, -1)


@pytest.mark.parametrize("read_ids", [False, True])
def test_request_coalescing_zipf_batch(gpu, read_ids):
    # a Zipf batch is about half duplicates: equal (key, read id) requests of the batch travel
    # and are probed once (whatever exchange chunk they fall in), every caller position gets its request's result -- identical to the
    # uncoalesced path and to one table holding every key
    world, n = 4, 300_000
    keys = np.arange(n, dtype=np.uint64)
    tabs, h = shard_tables(keys, world)
    full = stage.Table(key_width=8)
    full.load_keys(keys, 8, mode=1)
    rng = np.random.default_rng(5)
    hot = rng.choice(n, 500, replace=False).astype(np.uint64)
    for k in hot:  # version chains on some hot keys: results depend on the read id
        owner = tabs[int(h[int(k)] % np.uint64(world))]
        for t in (owner, full):
            assert t.update(int(k), 16, b"\x17" * 24, 10) == stage.RC_OK
            assert t.commit_update(int(k), 11, 11) == stage.RC_OK
    for t in tabs + [full]:
        t.sync()
    per_keys = [np.concatenate([stage.zipf_draws(n + 999, 0.9, 40 + r, 60_000, nthreads=2), hot[:300]])
                for r in range(world)]
    per_rids = [rng.integers(9, 13, k.size).astype(np.uint32) for k in per_keys] if read_ids else None
    got = {}
    for dd in (1, 0):
        for t in tabs:
            stage.set_shard_dedupe(t, dd)
        got[dd] = stage.probe_sharded_loopback(tabs, per_keys, per_rids)
        stats = [stage.sharded_stats(t) for t in tabs]
        for r in range(world):
            nk, routed, remote = stats[r]
            assert nk == per_keys[r].size and remote <= routed
            pairs = per_keys[r] if per_rids is None else \
                (per_keys[r] << np.uint64(8)) | per_rids[r].astype(np.uint64)
            if dd:
                # the distinct (key, read id) requests of the batch, plus the cuts of the sorted
                # batch every 64 positions (a run of > 64 callers travels as several requests)
                assert np.unique(pairs).size <= routed <= min(nk, np.unique(pairs).size + nk // 64 + 1)
                assert routed < 0.8 * nk
            else:
                assert routed == nk
    for r in range(world):
        ref_out, ref_rows = full.probe(per_keys[r], read_ids=None if per_rids is None else per_rids[r])
        for dd in (1, 0):
            out, rows = got[dd][r]
            for f in ("status", "flags", "hops", "key_len", "cstamp", "rec_cstamp", "copy_sstamp"):
                assert (out[f] == ref_out[f]).all(), (dd, r, f)
            assert (rows == ref_rows).all(), (dd, r)
    for t in tabs:
        stage.set_shard_dedupe(t, -1)


@pytest.mark.parametrize("world,chunks,payload,reply", [(2, 1, 1000, 0), (3, 3, 1000, 0), (3, 2, 100, 0),
                                                         (3, 3, 1000, 2), (3, 2, 100, 2), (2, 1, 1000, 3),
                                                         (3, 3, 1000, 3), (3, 2, 100, 3)])
def test_hot_keys_and_other_geometries_loopback(gpu, world, chunks, payload, reply):
    # one key asked 10,000 times in a batch (its run is cut into requests of <= 64 callers, each
    # fanned out), a few keys a few hundred times, read ids interleaved; payload 100 = leaves of
    # > 64 slots, outside the fan-out probe: own requests are probed, then fanned out (fan_copy)
    n = 150_000
    keys = np.arange(n, dtype=np.uint64)
    tabs, h = shard_tables(keys, world, payload=payload)
    full = stage.Table(key_width=8, payload_size=payload)
    full.load_keys(keys, 8, mode=1)
    for t in tabs + [full]:
        t.sync()
    for t in tabs:
        check(stage.lib().stage_set_shard_chunks(t.h, chunks), "chunks")
        stage.set_shard_dedupe(t, 1)
    rng = np.random.default_rng(world * 10 + chunks)
    per_keys, per_rids = [], []
    for r in range(world):
        k = np.concatenate([np.full(10_000, 4242 + r, np.uint64), np.repeat(rng.integers(0, n, 5), 300),
                            rng.integers(0, n + 1000, 20_000)]).astype(np.uint64)
        perm = rng.permutation(k.size)
        per_keys.append(k[perm])
        per_rids.append(rng.integers(1, 4, k.size).astype(np.uint32))
    if reply == stage.REPLY_DIRECT and payload != 1000:  # outside the fan-out probe's geometry: refused
        with pytest.raises(stage.StageError):
            stage.probe_sharded_loopback(tabs, per_keys, per_rids, reply=reply)
        for t in tabs:
            stage.set_shard_dedupe(t, -1)
        return
    res = stage.probe_sharded_loopback(tabs, per_keys, per_rids, reply=reply)
    for r in range(world):
        out, rows = res[r]
        ref_out, ref_rows = full.probe(per_keys[r], read_ids=per_rids[r])
        for f in ("status", "flags", "hops", "key_len", "cstamp", "rec_cstamp", "copy_sstamp"):
            assert (out[f] == ref_out[f]).all(), (r, f)
        assert (rows == ref_rows).all(), r
        nk, routed, remote = stage.sharded_stats(tabs[r])
        # the 10,000 callers of one key (3 read ids) travel as ~160 requests of <= 64 callers
        assert routed < 0.7 * nk
    for t in tabs:
        stage.set_shard_dedupe(t, -1)


@pytest.mark.parametrize("bits,wide", [(18, False), (12, False), (18, True)])
def test_narrow_coalescing_sort(gpu, bits, wide):
    # a coalescing width of <= 32 bits sorts the keys' low words (stage_set_shard_key_bits, as
    # the bench sets it from the row count): exact grouping when every key fits 32 bits; a
    # width below the keys' (12 of 18 bits) or keys above 2^32 in the batch (gathered back by
    # position) only coalesce less -- every caller still gets the one-table result
    world, n = 3, 200_000
    keys = np.arange(n, dtype=np.uint64)
    tabs, _ = shard_tables(keys, world)
    full = stage.Table(key_width=8)
    full.load_keys(keys, 8, mode=1)
    for t in tabs + [full]:
        t.sync()
    rng = np.random.default_rng(bits + wide)
    per_keys = []
    for r in range(world):
        k = np.concatenate([stage.zipf_draws(n + 99, 0.9, 70 + r, 50_000, nthreads=2),
                            np.full(3000, 77 + r, np.uint64)])
        if wide:  # absent keys above 2^32, some sharing low words with present keys
            k = np.concatenate([k, (np.uint64(1) << np.uint64(32 + r)) + rng.integers(0, n, 2000).astype(np.uint64)])
        per_keys.append(k[rng.permutation(k.size)].astype(np.uint64))
    for t in tabs:
        stage.set_shard_dedupe(t, 1)
        stage.set_shard_key_bits(t, bits)
    try:
        res = stage.probe_sharded_loopback(tabs, per_keys, None)
        for r in range(world):
            out, rows = res[r]
            ref_out, ref_rows = full.probe(per_keys[r])
            for f in ("status", "flags", "hops", "key_len", "cstamp", "rec_cstamp", "copy_sstamp"):
                assert (out[f] == ref_out[f]).all(), (r, f)
            assert (rows == ref_rows).all(), r
            nk, routed, _ = stage.sharded_stats(tabs[r])
            u = np.unique(per_keys[r]).size
            assert u <= routed <= nk
            if bits == 18 and not wide:  # exact grouping: distinct keys + the 64-caller cuts
                assert routed <= u + nk // 64 + 1
        own = stage.probe_sharded_loopback(tabs, per_keys, None, records=True, reply=stage.REPLY_OWNER)
        for r in range(world):
            ref_out, _ = full.probe(per_keys[r])
            for f in ("status", "cstamp", "rec_cstamp"):
                assert (own[r][0][f] == ref_out[f]).all(), (r, f)
    finally:
        for t in tabs:
            stage.set_shard_dedupe(t, -1)
            stage.set_shard_key_bits(t, 0)


@pytest.mark.parametrize("world", [2, 3])
def test_peer_reply_row_stride_raised_between_calls(gpu, world):
    """STAGE_REPLY_PEER row buffers are sized in rows of the call's stride: raising the output
    stride (stage_set_output_layout) between peer calls re-plans and reallocates every shard's
    buffers, so the owners' rows never land past their end.  Each call also rewrites
    the same buffer parity with different rows (the keys change), so a stale row would show."""
    n = 200_000
    keys = np.arange(n, dtype=np.uint64)
    tabs, h = shard_tables(keys, world)
    full = stage.Table(key_width=8)
    full.load_keys(keys, 8, mode=1)
    for t in tabs + [full]:
        t.sync()
    rng = np.random.default_rng(100 + world)
    for call, stride in enumerate((0, 0, 1152, 1152, 1008, 2048)):
        for t in tabs + [full]:
            t.set_output_layout(stride, 32)
        per_keys = [rng.integers(0, n + 5000, int(rng.integers(20_000, 60_000))).astype(np.uint64)
                    for _ in range(world)]
        res = stage.probe_sharded_loopback(tabs, per_keys, None, reply=stage.REPLY_PEER)
        for r in range(world):
            out, rows = res[r]
            ref_out, ref_rows = full.probe(per_keys[r])
            assert rows.shape[1] == full.stride == (stride or 1024)
            assert (out["status"] == ref_out["status"]).all(), (call, r)
            assert (rows == ref_rows).all(), (call, r, stride)
            # past the 1024-B heap row the output row is zero (not the next heap row)
            assert not rows[:, 1024:].any()
    for t in tabs + [full]:
        t.set_output_layout(0, 32)
