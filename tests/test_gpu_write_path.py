"""GPU parity of the device write path (stage_update_batch_device).

Each epoch is applied by the device to the published image; the reference semantics are the
oracle's LeafNode::Update + CommitTransaction UPDATE entry applied op by op in batch order.
After every epoch the device must return the oracle's return codes and answer every read
(latest, in-flight copy, retired versions at old read ids, range scans) like the oracle, and
host-side writes after a device epoch must still behave like the reference.
"""
import numpy as np
import pytest

import oracle_lib as O
import stage
from stage._lib import check
from test_gpu_incremental import check_all
from test_gpu_parity import check_probe
from test_leaf_images import assert_same_images

pytestmark = pytest.mark.gpu


def oracle_epoch(orc, keys, key_size, off, deltas, wid, cid):
    rc = np.zeros(len(keys), np.uint8)
    for i in range(len(keys)):
        k = keys[i] if isinstance(keys[i], bytes) else int(keys[i])
        r = orc.update(k, key_size, off, deltas[i].tobytes(), int(wid[i]))
        if r == stage.RC_OK and cid[i]:
            r = orc.commit_update(k, key_size, int(cid[i]), int(cid[i]))
        rc[i] = r
    return rc


def epoch_ops(rng, base, hot, m, counter):
    """keys: uniform, a hot set with repeats, absent keys; deltas: random, or one per hot key
    (its repeats are NotNeededUpdate); ids from one counter; ~12 % left in flight."""
    kind = rng.random(m)
    keys = np.where(kind < 0.6, rng.choice(base, m), rng.choice(hot, m))
    keys = np.where(kind > 0.93, rng.choice(base, m) + 1, keys).astype(np.uint64)  # absent
    deltas = rng.integers(0, 256, (m, 24), dtype=np.uint8)
    fixed = (kind >= 0.6) & (kind < 0.8)
    deltas[fixed] = (keys[fixed] % 251).astype(np.uint8)[:, None]
    wid = (counter + 2 * np.arange(m)).astype(np.uint32)
    wid[rng.random(m) < 0.03] = 1  # older writer than the committed record -> NotNeededUpdate
    cid = (wid + 1).astype(np.uint32)
    cid[rng.random(m) < 0.12] = 0
    return keys, deltas, wid, cid


def test_device_epochs_match_oracle(gpu):
    n = 120000
    base = np.arange(n, dtype=np.uint64) * 4
    tab = stage.Table(key_width=8)
    orc = O.OracleTree()
    tab.load_keys(base, 8, mode=1)
    orc.load_keys(base, 8, 1)
    tab.sync()
    rng = np.random.default_rng(41)
    hot = rng.choice(base, 40, replace=False)
    counter = 10
    seen = set()
    for epoch in range(4):
        m = 12000
        keys, deltas, wid, cid = epoch_ops(rng, base, hot, m, counter)
        counter += 2 * m + 2
        off = 100 * epoch + 3
        rc, ok = tab.update_batch_device(keys, off, deltas, wid, cid)
        exp = oracle_epoch(orc, keys, 8, off, deltas, wid, cid)
        bad = np.nonzero(rc != exp)[0]
        assert bad.size == 0, (epoch, bad[:5], rc[bad[:5]], exp[bad[:5]], keys[bad[:5]])
        assert ok == int(((exp == stage.RC_OK)).sum())
        seen |= set(rc.tolist())
        if epoch == 1:  # host writes after a device epoch (device rows materialised first)
            for k in rng.choice(hot, 5, replace=False):
                d = rng.integers(0, 256, 16, dtype=np.uint8)
                assert tab.update(int(k), 7, d, counter) == orc.update(int(k), 8, 7, d.tobytes(), counter)
            for k in rng.choice(base, 200, replace=False):
                assert tab.delete(int(k), counter) == orc.delete(int(k), 8, counter)
            tab.sync()
            assert tab.sync_info()["incremental"]
        if epoch == 2:  # the host batch path on top of device epochs
            k2, d2, w2, c2 = epoch_ops(rng, base, hot, 3000, counter)
            counter += 6002
            rc2, _ = tab.update_batch(k2, 11, d2, w2, c2)
            assert (rc2 == oracle_epoch(orc, k2, 8, 11, d2, w2, c2)).all()
            tab.sync()
        probe = np.concatenate([hot, rng.choice(keys, 3000), rng.choice(base, 2000)]).astype(np.uint64)
        check_all(tab, orc, probe, rng, counter)
    assert {stage.RC_OK, stage.RC_NOT_FOUND, stage.RC_NOT_NEEDED_UPDATE, stage.RC_DIRTY} <= seen
    assert_same_images(tab, orc)


def test_device_epoch_equals_host_epoch_zipf(gpu):
    """YCSB-B shaped epoch (Zipf 0.99, one delta per key per epoch: a hot key's repeats are
    NotNeededUpdate): codes and every read equal the host write path's."""
    n = 400000
    a, b = stage.Table(key_width=8), stage.Table(key_width=8)
    for t in (a, b):
        t.load_ycsb(0, n, 8, mode=0)
        t.sync()
    counter = 1
    for epoch in range(3):
        keys = stage.zipf_draws(n - 1, 0.99, 77 + epoch, 100000)
        m = keys.size
        wid = (counter + 2 * np.arange(m)).astype(np.uint32)
        cid = (wid + 1).astype(np.uint32)
        counter += 2 * m
        cols = np.repeat(((keys + np.uint64(epoch + 1)) & np.uint64(0xFF)).astype(np.uint8)[:, None], 100, 1)
        rc_a, ok_a = a.update_batch(keys, 0, cols, wid, cid)
        a.sync()
        rc_b, ok_b = b.update_batch_device(keys, 0, cols, wid, cid)
        assert ok_a == ok_b and (rc_a == rc_b).all()
        assert (rc_b == stage.RC_NOT_NEEDED_UPDATE).sum() > m // 4  # long groups were finished
        probe = np.unique(keys)
        for rid in (0, counter // 3, counter // 2, 0xFFFFFFFE):
            rids = np.full(probe.size, rid, np.uint32)
            oa, ra = a.probe(probe, read_ids=rids)
            ob, rb = b.probe(probe, read_ids=rids)
            for f in ("status", "flags", "hops", "leaf", "slot", "cstamp", "rec_cstamp", "copy_sstamp"):
                assert (oa[f] == ob[f]).all(), (epoch, rid, f)
            assert (ra == rb).all()


def test_device_epoch_wide_keys(gpu):
    """16-byte composite keys (TPC-C StockKey layout, unsigned memcmp order)."""
    rng = np.random.default_rng(5)
    wi = np.stack(np.meshgrid(np.arange(1, 5), np.arange(1, 6001), indexing="ij"), -1).reshape(-1, 2)
    keys = np.ascontiguousarray(wi.astype(np.int64)).view(np.uint8).reshape(-1, 16)
    pays = rng.integers(0, 256, (keys.shape[0], 400), dtype=np.uint8)
    tab = stage.Table(payload_size=400, key_width=16)
    tab.load_rows(keys, pays)
    tab.sync()
    orc = O.OracleTree(payload_size=400, key_pad=16)
    orc.load_rows(keys, pays)
    counter = 5
    for epoch in range(3):
        m = 3000
        idx = rng.integers(0, keys.shape[0] + 200, m)  # some absent
        uk = np.zeros((m, 16), np.uint8)
        present = idx < keys.shape[0]
        uk[present] = keys[idx[present]]
        uk[~present] = np.ascontiguousarray(np.stack([np.full((~present).sum(), 9), idx[~present]], 1)
                                            .astype(np.int64)).view(np.uint8).reshape(-1, 16)
        deltas = rng.integers(0, 256, (m, 4), dtype=np.uint8)
        deltas[::7] = 1
        wid = (counter + 2 * np.arange(m)).astype(np.uint32)
        cid = (wid + 1).astype(np.uint32)
        cid[::9] = 0
        counter += 2 * m
        rc, _ = tab.update_batch_device(uk, 0, deltas, wid, cid)
        exp = oracle_epoch(orc, [bytes(r) for r in uk], 16, 0, deltas, wid, cid)
        assert (rc == exp).all()
        for rid in (0, counter // 2, 0xFFFFFFFE):
            out, rows = tab.probe(uk, read_ids=np.full(m, rid, np.uint32))
            o_out, o_rec = orc.read_batch_k(uk, np.full(m, rid, np.uint32))
            for f in ("status", "hops", "cstamp", "rec_cstamp", "copy_sstamp"):
                assert (out[f] == o_out[f]).all(), (epoch, rid, f)
            assert (rows[:, :orc.row] == o_rec).all()


def test_device_epoch_edge_cases(gpu):
    tab = stage.Table(key_width=8)
    tab.load_ycsb(0, 5000, 8, mode=0)
    tab.sync()
    orc = O.OracleTree()
    orc.load_ycsb(0, 5000, 8, 0)
    # empty batch
    rc, ok = tab.update_batch_device(np.zeros(0, np.uint64), 0, np.zeros((0, 8), np.uint8), [])
    assert rc.size == 0 and ok == 0
    # window past the payload: every op Invalid
    k = np.array([1, 2, 2], np.uint64)
    rc, ok = tab.update_batch_device(k, 995, np.ones((3, 8), np.uint8), 3, 4)
    assert ok == 0 and (rc == oracle_epoch(orc, k, 8, 995, np.ones((3, 8), np.uint8), [3] * 3, [4] * 3)).all()
    # one key many times, alternating deltas, no commits: first OK, then Dirty (in flight)
    k = np.full(200, 7, np.uint64)
    d = np.where(np.arange(200)[:, None] % 2 == 0, 1, 2).astype(np.uint8).repeat(8, 1)
    w = np.arange(10, 210, dtype=np.uint32)
    rc, ok = tab.update_batch_device(k, 0, d, w, None)
    assert (rc == oracle_epoch(orc, k, 8, 0, d, w, np.zeros(200, np.uint32))).all() and ok == 1
    # all commits, alternating deltas: every op succeeds (a 200-version chain)
    k = np.full(200, 9, np.uint64)
    w = np.arange(1000, 1400, 2, dtype=np.uint32)
    rc, ok = tab.update_batch_device(k, 0, d, w, w + 1)
    assert (rc == oracle_epoch(orc, k, 8, 0, d, w, w + 1)).all() and ok == 200
    # a table that was written on the host but not published is refused
    tab.update(11, 0, b"x" * 8, 5000)
    with pytest.raises(stage.StageError):
        tab.update_batch_device(np.array([12], np.uint64), 0, np.ones((1, 8), np.uint8), 6000)
    orc.update(11, 8, 0, b"x" * 8, 5000)
    tab.sync()
    keys = np.array([1, 2, 7, 9, 11, 4999, 5000], np.uint64)
    for rid in (0, 5, 1100, 1399, 0xFFFFFFFE):
        check_probe(tab, orc, keys, 8, read_ids=np.full(keys.size, rid, np.uint32))


@pytest.mark.parametrize("alphabet,old_writers,head_fails,adjacent", [(3, True, False, False), (256, True, False, False),
                                                                       (3, False, False, False), (256, False, False, False),
                                                                       (62, False, True, False), (3, False, False, True),
                                                                       (62, False, True, True)])
def test_hot_key_groups_finished_by_workgroups(gpu, alphabet, old_writers, head_fails, adjacent):
    """Groups longer than the workgroup finisher's threshold (2048 ops from the first failure):
    three hot keys hammered ~6000 times each in one epoch with a 3-letter delta alphabet
    (NotNeededUpdate and successes interleave) or RunMixed's 256 / 62 (successes with sparse
    failures), a few left in flight (the rest of that group DIRTY) -- return codes, versions and
    reads equal to the oracle applied op by op.  Without writers older than the record the groups
    are finished by pointer jumping (wp_jump_links / _chain / _codes); with them (NotNeededUpdate by cstamp) the
    chain is not known locally and the walk finishes them.  head_fails: every hot group's first op
    repeats the record's current column (NotNeededUpdate against the epoch-start state), so the
    chain starts behind a failed head.  adjacent: two hot keys in neighbouring slots, so their
    groups meet inside one 64-position chunk (the grid-wide jump phases key the chain's per-chunk
    record by group)."""
    n = 20000
    tab = stage.Table(key_width=8)
    tab.load_ycsb(0, n, 8, mode=1)
    tab.sync()
    orc = O.OracleTree()
    orc.load_ycsb(0, n, 8, 1)
    rng = np.random.default_rng(12)
    counter = 10
    for epoch in range(2):
        m = 24000
        hot = np.array([3, 4, 19999] if adjacent else [3, 1000, 19999], np.uint64)
        keys = np.where(rng.random(m) < 0.75, rng.choice(hot, m), rng.integers(0, n + 50, m)).astype(np.uint64)
        deltas = rng.integers(0, alphabet, (m, 1), dtype=np.uint8).repeat(16, 1)
        if head_fails:  # the first op of each hot key writes what its row already holds there
            for h in hot:
                first = int(np.nonzero(keys == h)[0][0])
                _, row = orc.read(int(h), 8)
                deltas[first] = row[8 + 40 * epoch: 8 + 40 * epoch + 16]
        wid = (counter + 2 * np.arange(m)).astype(np.uint32)
        if old_writers:
            wid[rng.random(m) < 0.02] = 1
        cid = (wid + 1).astype(np.uint32)
        cid[(keys == hot[2]) & (rng.random(m) < 0.002)] = 0  # the third hot key goes in flight
        counter += 2 * m + 2
        off = 40 * epoch
        rc, ok = tab.update_batch_device(keys, off, deltas, wid, cid)
        exp = oracle_epoch(orc, keys, 8, off, deltas, wid, cid)
        bad = np.nonzero(rc != exp)[0]
        assert bad.size == 0, (epoch, bad[:5], rc[bad[:5]], exp[bad[:5]], keys[bad[:5]])
        assert ok == int((exp == stage.RC_OK).sum())
        assert (keys == hot[0]).sum() > 4096
        if alphabet == 3:
            assert (exp[keys == hot[0]] == stage.RC_NOT_NEEDED_UPDATE).sum() > 1000
        else:
            assert (exp[keys == hot[0]] == stage.RC_OK).sum() > 4000
            assert (exp[keys == hot[0]] != stage.RC_OK).sum() > (50 if old_writers else 10)
        if head_fails:
            assert all(exp[int(np.nonzero(keys == h)[0][0])] == stage.RC_NOT_NEEDED_UPDATE for h in hot[:2])
        probe = np.concatenate([hot, rng.integers(0, n, 2000).astype(np.uint64)])
        for rid in (0, counter // 3, counter // 2, counter - 5, 0xFFFFFFFE):
            check_probe(tab, orc, probe, 8, read_ids=np.full(probe.size, rid, np.uint32))


@pytest.mark.parametrize("dlen,off", [(150, 5), (133, 0), (3, 1)])
def test_long_and_ragged_windows(gpu, dlen, off):
    """Windows longer than one 32-lane team pass (wp_classify loops), lengths that are not a
    word multiple and unaligned offsets; an A-B-A delta pattern per key (equal contents in
    different runs: the byte comparison behind a fingerprint match)."""
    n = 3000
    tab = stage.Table(key_width=8)
    tab.load_ycsb(0, n, 8, mode=1)
    tab.sync()
    orc = O.OracleTree()
    orc.load_ycsb(0, n, 8, 1)
    rng = np.random.default_rng(dlen)
    counter = 10
    for epoch in range(2):
        m = 5000
        keys = np.where(rng.random(m) < 0.5, rng.integers(0, 8, m), rng.integers(0, n + 20, m)).astype(np.uint64)
        deltas = rng.integers(0, 3, (m, 1), dtype=np.uint8).repeat(dlen, 1)
        deltas[:, -1] ^= rng.integers(0, 2, m, dtype=np.uint8)  # a difference in the last (ragged) byte only
        wid = (counter + 2 * np.arange(m)).astype(np.uint32)
        cid = (wid + 1).astype(np.uint32)
        counter += 2 * m + 2
        rc, ok = tab.update_batch_device(keys, off, deltas, wid, cid)
        exp = oracle_epoch(orc, keys, 8, off, deltas, wid, cid)
        bad = np.nonzero(rc != exp)[0]
        assert bad.size == 0, (epoch, bad[:5], rc[bad[:5]], exp[bad[:5]], keys[bad[:5]])
        assert (exp == stage.RC_NOT_NEEDED_UPDATE).sum() > 100 and ok > 100
        probe = np.arange(0, 40, dtype=np.uint64)
        for rid in (0, counter // 2, 0xFFFFFFFE):
            check_probe(tab, orc, probe, 8, read_ids=np.full(probe.size, rid, np.uint32))


def test_pipelined_epochs_without_waits(gpu):
    """Epochs enqueued back to back on one stream with no host wait: each epoch's adoption runs
    in the background while the next epoch's kernels are enqueued (device-side append counters,
    double-buffered outputs); a large epoch in the middle grows the header arrays and the heap
    (settling first).  Codes, reads and the host table after settling equal the oracle's."""
    n = 30000
    tab = stage.Table(key_width=8)
    tab.load_ycsb(0, n, 8, mode=1)
    tab.sync()
    orc = O.OracleTree()
    orc.load_ycsb(0, n, 8, 1)
    rng = np.random.default_rng(8)
    s = stage.Stream()
    counter, epochs = 10, []
    for m in (2000, 500, 9000, 120000, 700, 3000, 1):
        keys = np.where(rng.random(m) < 0.3, rng.integers(0, 50, m), rng.integers(0, n + 100, m)).astype(np.uint64)
        deltas = rng.integers(0, 4, (m, 1), dtype=np.uint8).repeat(12, 1)
        wid = (counter + 2 * np.arange(m)).astype(np.uint32)
        cid = np.where(rng.random(m) < 0.05, 0, wid + 1).astype(np.uint32)
        counter += 2 * m + 2
        d = [stage.DeviceBuffer.from_numpy(x) for x in (keys, deltas.reshape(-1), wid, cid)]
        rcb = stage.DeviceBuffer(m)
        check(stage.lib().stage_update_batch_device(tab.h, d[0].ptr, None, m, 16, d[1].ptr, 12, d[2].ptr, d[3].ptr,
                                                    None, rcb.ptr, None, s.ptr), "update_batch_device")
        epochs.append((keys, deltas, wid, cid, rcb, d))
    s.sync()
    for keys, deltas, wid, cid, rcb, _ in epochs:
        rc = rcb.to_numpy(np.uint8, keys.size)
        exp = oracle_epoch(orc, keys, 8, 16, deltas, wid, cid)
        bad = np.nonzero(rc != exp)[0]
        assert bad.size == 0, (keys.size, bad[:5], rc[bad[:5]], exp[bad[:5]])
    probe = np.concatenate([np.arange(60), rng.integers(0, n, 3000)]).astype(np.uint64)
    check_all(tab, orc, probe, rng, counter)
    # the host table (settled) agrees too: host-side writes on top, then a publish
    for k in range(0, 50, 7):
        dd = rng.integers(0, 256, 8, dtype=np.uint8)
        assert tab.update(k, 3, dd, counter) == orc.update(k, 8, 3, dd.tobytes(), counter)
    tab.sync()
    check_all(tab, orc, probe, rng, counter + 1)
    assert_same_images(tab, orc)


def test_write_overlap_epochs_with_probes_between(gpu):
    """stage_set_write_overlap: epoch e + 1's kernels up to its publish run beside epoch e's read
    probe (same caller stream, no host waits).  Each epoch's probe -- enqueued right after that
    epoch's call, at old and current read ids over hot and cold keys -- must read exactly the
    oracle's state after that epoch (not the next one's, not the previous one's); codes equal the
    oracle's; a growth in the middle and a host write + publish between overlapped epochs are
    ordered too."""
    n = 30000
    tab = stage.Table(key_width=8)
    tab.load_ycsb(0, n, 8, mode=1)
    tab.sync()
    tab.set_write_overlap(1)
    orc = O.OracleTree()
    orc.load_ycsb(0, n, 8, 1)
    rng = np.random.default_rng(31)
    s = stage.Stream()
    base, hot = np.arange(0, n, 2, dtype=np.uint64), np.arange(0, 40, dtype=np.uint64)
    counter, epochs = 10, []
    probe_keys = np.concatenate([hot, rng.integers(0, n + 50, 6000)]).astype(np.uint64)
    for e, m in enumerate((3000, 800, 9000, 90000, 1500, 4000, 2)):
        keys, deltas, wid, cid = epoch_ops(rng, base, hot, m, counter)
        counter += 2 * m + 2
        if e == 5:  # a host-side write + publish between two overlapped epochs
            s.sync()
            check(stage.lib().stage_settle(tab.h), "settle")
            k0 = int(hot[3])
            dd = rng.integers(0, 256, 8, dtype=np.uint8)
            ep_host = (k0, dd, counter, tab.update(k0, 3, dd, counter))
            counter += 2
            tab.sync()
        else:
            ep_host = None
        d = [stage.DeviceBuffer.from_numpy(x) for x in (keys, deltas.reshape(-1), wid, cid)]
        rcb = stage.DeviceBuffer(m)
        check(stage.lib().stage_update_batch_device(tab.h, d[0].ptr, None, m, 16, d[1].ptr, 24, d[2].ptr, d[3].ptr,
                                                    None, rcb.ptr, None, s.ptr), "update_batch_device")
        rids = np.where(rng.random(probe_keys.size) < 0.5, rng.integers(0, counter, probe_keys.size),
                        0xFFFFFFFE).astype(np.uint32)
        pk, pr = stage.DeviceBuffer.from_numpy(probe_keys), stage.DeviceBuffer.from_numpy(rids)
        pout, prow = stage.DeviceBuffer(probe_keys.size * 32), stage.DeviceBuffer(probe_keys.size * tab.stride)
        tab.probe_device(pk.ptr, probe_keys.size, pout.ptr, prow.ptr, d_read_ids=pr.ptr, stream=s.ptr)
        epochs.append((keys, deltas, wid, cid, rcb, d, rids, pk, pr, pout, prow, ep_host))
    s.sync()
    for keys, deltas, wid, cid, rcb, _, rids, _, _, pout, prow, ep_host in epochs:
        if ep_host is not None:
            k0, dd, c0, rc0 = ep_host
            assert orc.update(k0, 8, 3, dd.tobytes(), c0) == rc0
        exp = oracle_epoch(orc, keys, 8, 16, deltas, wid, cid)
        rc = rcb.to_numpy(np.uint8, keys.size)
        bad = np.nonzero(rc != exp)[0]
        assert bad.size == 0, (keys.size, bad[:5], rc[bad[:5]], exp[bad[:5]])
        out = pout.to_numpy(stage.PROBE_OUT_DTYPE, probe_keys.size)
        rows = prow.to_numpy(np.uint8, probe_keys.size * tab.stride).reshape(probe_keys.size, tab.stride)
        o_out, o_rec = orc.read_batch(probe_keys, 8, rids)
        for f in ("status", "hops", "cstamp", "rec_cstamp", "copy_sstamp"):
            badf = np.nonzero(out[f] != o_out[f])[0]
            assert badf.size == 0, (keys.size, f, badf[:5], out[f][badf[:5]], o_out[f][badf[:5]])
        assert not (rows[:, :orc.row] != o_rec).any(axis=1).any(), keys.size
    check_all(tab, orc, probe_keys, rng, counter)
    assert_same_images(tab, orc)


def test_overlap_epochs_reuse_input_buffers(gpu):
    """Write-overlap mode 1 with ONE set of device input buffers (keys, deltas, writer and commit
    ids) for every epoch: each next epoch's inputs are copied into them on the caller's stream
    right behind the call -- after the epoch's publish in stream order, which is the header's
    contract (inputs unmodified until the work enqueued behind the call has run; ADVICE r05 on
    the retired deferred-publish mode) -- and probes enqueued between epochs see each epoch.
    Codes, statuses and rows equal the oracle's; the host table agrees at the end."""
    n = 30000
    tab = stage.Table(key_width=8)
    tab.load_ycsb(0, n, 8, mode=1)
    tab.sync()
    tab.set_write_overlap(1)
    with pytest.raises(stage.StageError):
        tab.set_write_overlap(2)  # retired
    orc = O.OracleTree()
    orc.load_ycsb(0, n, 8, 1)
    rng = np.random.default_rng(37)
    s = stage.Stream()
    base, hot = np.arange(0, n, 2, dtype=np.uint64), np.arange(0, 40, dtype=np.uint64)
    counter, epochs = 10, []
    probe_keys = np.concatenate([hot, rng.integers(0, n + 50, 5000)]).astype(np.uint64)
    cap = 60000
    dk, dd, dw, dc = (stage.DeviceBuffer(cap * w) for w in (8, 24, 4, 4))
    L = stage.lib()

    def refill(keys, deltas, wid, cid):  # stream-ordered H2D into the shared input buffers
        for buf, x in ((dk, keys), (dd, deltas.reshape(-1)), (dw, wid), (dc, cid)):
            x = np.ascontiguousarray(x)
            check(L.stage_memcpy_h2d(buf.ptr, x.ctypes.data, x.nbytes, s.ptr), "h2d")
        return x

    def enqueue_probe():
        rids = np.where(rng.random(probe_keys.size) < 0.5, rng.integers(0, counter, probe_keys.size),
                        0xFFFFFFFE).astype(np.uint32)
        pk, pr = stage.DeviceBuffer.from_numpy(probe_keys), stage.DeviceBuffer.from_numpy(rids)
        pout, prow = stage.DeviceBuffer(probe_keys.size * 32), stage.DeviceBuffer(probe_keys.size * tab.stride)
        tab.probe_device(pk.ptr, probe_keys.size, pout.ptr, prow.ptr, d_read_ids=pr.ptr, stream=s.ptr)
        return rids, (pk, pr), pout, prow

    sizes = (3000, 800, 9000, 60000, 1500, 4000, 2)
    ops = []
    for m in sizes:
        ops.append(epoch_ops(rng, base, hot, m, counter))
        counter += 2 * m + 2
    host_src = [refill(*ops[0])]  # the first epoch's inputs; the arrays stay alive until s is done
    s.sync()
    for e, m in enumerate(sizes):
        keys, deltas, wid, cid = ops[e]
        rcb = stage.DeviceBuffer(m)
        check(L.stage_update_batch_device(tab.h, dk.ptr, None, m, 16, dd.ptr, 24, dw.ptr, dc.ptr, None, rcb.ptr,
                                          None, s.ptr), "update_batch_device")
        after = enqueue_probe()
        if e + 1 < len(sizes):
            host_src.append(refill(*ops[e + 1]))  # behind the epoch's publish and probe on s
            s.sync()  # the next call's inputs are complete when it is made
        epochs.append((keys, deltas, wid, cid, rcb, after))
    s.sync()

    def compare(probe):
        rids, _, pout, prow = probe
        out = pout.to_numpy(stage.PROBE_OUT_DTYPE, probe_keys.size)
        rows = prow.to_numpy(np.uint8, probe_keys.size * tab.stride).reshape(probe_keys.size, tab.stride)
        o_out, o_rec = orc.read_batch(probe_keys, 8, rids)
        for f in ("status", "hops", "cstamp", "rec_cstamp", "copy_sstamp"):
            badf = np.nonzero(out[f] != o_out[f])[0]
            assert badf.size == 0, (f, badf[:5], out[f][badf[:5]], o_out[f][badf[:5]])
        assert not (rows[:, :orc.row] != o_rec).any(axis=1).any()

    for keys, deltas, wid, cid, rcb, after in epochs:
        exp = oracle_epoch(orc, keys, 8, 16, deltas, wid, cid)
        rc = rcb.to_numpy(np.uint8, keys.size)
        bad = np.nonzero(rc != exp)[0]
        assert bad.size == 0, (keys.size, bad[:5], rc[bad[:5]], exp[bad[:5]])
        compare(after)
    check_all(tab, orc, probe_keys, rng, counter)
    assert_same_images(tab, orc)
