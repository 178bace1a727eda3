"""Pins tests/scan_semantics.py (the restatement the full-size GPU scan test checks against)
to the oracle: over the host mirror's exported leaves it must reproduce the oracle's
TableScanExecutor output exactly, including the keys RangeScanBySize's slot-order cut skips."""
import numpy as np
import pytest

import oracle_lib as O
import stage
from scan_semantics import LeafScanner, order_key


@pytest.mark.parametrize("n", [300_000])
def test_restatement_equals_oracle(n):
    orc = O.OracleTree()
    orc.load_ycsb(0, n, 8, 0)
    tab = stage.Table(key_width=8)
    tab.load_ycsb(0, n, 8, 0)
    ls = LeafScanner(tab)
    rng = np.random.default_rng(11)
    last = ls.keyw[-1, :int(ls.rc[-1])]
    starts = np.concatenate([rng.integers(0, n, 300), [0, 1, n - 1, n, n + 5], last[:2], last[-2:]]).astype(np.uint64)
    ordered = np.sort(order_key(np.arange(n, dtype=np.uint64)))
    pos = np.searchsorted(ordered, order_key(starts))
    for L in (1, 7, 64, 100):
        c, r = orc.scan_batch(starts, 8, L)
        not_successors = 0
        for i, s in enumerate(starts):
            e = ls.scan(int(s), L)
            got = r[i, :c[i], :8].copy().view(np.uint64).ravel()
            assert e.size == c[i] and (e == got).all(), (int(s), L)
            succ = order_key(ordered[pos[i]:pos[i] + L])
            not_successors += int(e.size != succ.size or not (e == succ).all())
        if L == 100:  # the slot-order cut is exercised: many scans skip keys
            assert not_successors > 50
    tab.close()
