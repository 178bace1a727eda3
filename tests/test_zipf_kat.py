"""CPU: the harness's YCSB stream generators equal the reference's own (row a13).

tests/golden/zipf_kat.json holds outputs of the reference's FastRandom and ZipfDistribution
(benchmark/benchmark_common.h:10-98) compiled from the reference checkout by
tests/golden/make_zipf_kat.py: FastRandom(seed).next() streams, the zeta(n, theta) sums
bit for bit, and GetNextNumber() draws with the generator seeded FastRandom(seed), over the
drivers' key ranges ZipfDistribution(scale_factor - 1, theta) (ycsb_workload.cpp:88) at 1000,
1M and 100M rows.
"""
import json
import os
import struct

import numpy as np
import pytest

import stage

KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "zipf_kat.json")))


def _bits(x):
    return "%016x" % struct.unpack("<Q", struct.pack("<d", x))[0]


@pytest.mark.parametrize("case", KAT["fastrandom"], ids=lambda c: "seed%d" % c["seed"])
def test_fastrandom_stream(case):
    got = stage.fastrandom(case["seed"], len(case["next"]))
    assert got.tolist() == case["next"]


@pytest.mark.parametrize("case", KAT["zipf"], ids=lambda c: "n%d_t%g" % (c["n"], c["theta"]))
def test_zipf_zeta_bit_identical(case):
    assert _bits(stage.zipf_zeta(case["n"], case["theta"])) == case["zeta_n_bits"]
    assert _bits(stage.zipf_zeta(2, case["theta"])) == case["zeta_2_bits"]


@pytest.mark.parametrize("case", KAT["zipf"], ids=lambda c: "n%d_t%g" % (c["n"], c["theta"]))
@pytest.mark.parametrize("nthreads", [1, 8])
def test_zipf_draws(case, nthreads):
    want = np.array(case["draws"], np.uint64)
    # the threaded generator jumps each thread's FastRandom ahead; pad the count so 8 threads split it
    count = max(len(want), 8192)
    got = stage.zipf_draws(case["n"], case["theta"], case["seed"], count, nthreads=nthreads)
    assert (got[:len(want)] == want).all()
    if nthreads > 1:  # the other threads' jumped streams continue the same sequence
        assert (got == stage.zipf_draws(case["n"], case["theta"], case["seed"], count, nthreads=1)).all()
    assert got.min() >= 1 and got.max() <= case["n"]


@pytest.mark.parametrize("case", KAT["ops"], ids=lambda c: "seed%d_u%g" % (c["seed"], c["update_ratio"]))
def test_ycsb_op_stream(case):
    """RunMixed's op stream (ycsb_mixed.cpp:26-44): which ops update, and each update's
    next_char() delta byte, equal the reference's FastRandom draws."""
    want = np.array(case["ops"])
    upd, chr_ = stage.ycsb_ops(case["seed"], case["count"], case["update_ratio"])
    assert (upd == (want >= 0)).all()
    assert (chr_[upd] == want[want >= 0]).all()
    assert (chr_[~upd] == 0).all()
