"""CPU: the C-ABI library loads and exports every symbol include/stage_hip.h declares;
host-only entry points behave (errors, generators).  No compute is launched."""
import ctypes
import os
import re

import numpy as np

import stage
from stage._lib import LIB_PATH, SIGNATURES

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "stage_hip.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(stage_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_exported():
    names = declared_functions()
    assert len(names) >= 40
    L = ctypes.CDLL(LIB_PATH)
    for n in names:
        assert hasattr(L, n), f"{n} declared in stage_hip.h but not exported"
        assert n in SIGNATURES, f"{n} has no ctypes signature"
    assert set(SIGNATURES) == set(names)


def test_version_and_errors():
    L = stage.lib()
    assert b"gfx950" in L.stage_version()
    # null table -> STAGE_E_ARG with a message
    assert L.stage_sync(None) == -1
    assert len(L.stage_last_error()) > 0
    t = stage.Table(key_width=8)
    t.load_ycsb(0, 100, 8)
    # device entry points refuse a stale image instead of computing anything on the host
    out = ctypes.c_void_p(16)
    rc = L.stage_probe_batch(t.h, out, None, None, None, 1, out, None, None)
    assert rc == -4 and b"stage_sync" in L.stage_last_error()


def test_bad_params_rejected():
    import pytest
    with pytest.raises(stage.StageError):
        stage.Table(payload_size=0)
    with pytest.raises(stage.StageError):
        stage.Table(payload_size=1000, leaf_node_size=1024)  # fewer than 3 records per leaf


def _fastrandom_py(seed, count):
    # benchmark_common.h:12-64 (Java LCG)
    m48 = (1 << 48) - 1
    s = (seed ^ 0x5DEECE66D) & m48
    out = []

    def nxt(bits):
        nonlocal s
        s = (s * 0x5DEECE66D + 0xB) & m48
        return s >> (48 - bits)

    for _ in range(count):
        hi = nxt(32)
        lo = nxt(32)
        out.append(((hi << 32) + lo) & ((1 << 64) - 1))
    return out


def test_fastrandom_matches_lcg():
    for seed in (0, 1, 0x5EED, 123456789):
        assert list(stage.fastrandom(seed, 50)) == _fastrandom_py(seed, 50)


def test_zipf_draws_deterministic_and_threads_agree():
    a = stage.zipf_draws(1000000, 0.9, 0x5EED, 200000, nthreads=1)
    b = stage.zipf_draws(1000000, 0.9, 0x5EED, 200000, nthreads=8)
    assert (a == b).all()
    assert a.min() >= 1 and a.max() <= 1000000
    # skew: key 1 is the most frequent and carries a few percent of the draws at theta 0.9
    counts = np.bincount(a.astype(np.int64))
    assert counts.argmax() == 1
    assert 0.01 < counts[1] / a.size < 0.2


def test_q2_async_arguments():
    """stage_ch_query2_batch_async / _wait refuse bad calls before anything reaches a device:
    a slot outside 0..1, an empty batch, no `out`, a wait on a slot with nothing in flight, and
    unsynced tables (no device image: STAGE_E_STATE, as every device entry point)."""
    L = stage.lib()
    t = stage.Table(key_width=8)
    n = ctypes.c_uint64()
    ab = (ctypes.c_int32 * 4)()
    assert L.stage_ch_query2_wait(t.h, 2, ctypes.byref(n), ab) == -1
    assert L.stage_ch_query2_wait(t.h, 0, ctypes.byref(n), ab) == -4
    assert b"in flight" in L.stage_last_error()
    rids = (ctypes.c_uint32 * 4)(1, 2, 3, 4)
    out = ctypes.create_string_buffer(4 * 48 * 8)
    moff = (ctypes.c_uint32 * 10001)()
    h = t.h
    assert L.stage_ch_query2_batch_async(h, h, h, h, h, moff, None, 3, rids, 0, out, 8, 0, None) == -1
    assert L.stage_ch_query2_batch_async(h, h, h, h, h, moff, None, 3, rids, 4, None, 8, 0, None) == -1
    # one table for every role: its scratch would serve the batch buffers and both scan rows
    assert L.stage_ch_query2_batch_async(h, h, h, h, h, moff, ctypes.c_void_p(16), 3, rids, 4, out, 8, 0,
                                         None) == -1
    assert b"scratch alias" in L.stage_last_error()
    ts = [stage.Table(key_width=8) for _ in range(5)]
    assert L.stage_ch_query2_batch_async(*[x.h for x in ts], moff, ctypes.c_void_p(16), 3, rids, 4, out, 8, 0,
                                         None) == -4
