"""GPU: the reference-side adapter on real device results -- `adapter_drive probe` builds a
YCSB table through the C-ABI (version chains, an in-flight update, an inserted-then-updated
key), publishes, probes with stage_probe_batch + stage_probe_identify and frames every result through
include/stage_btree_adapter.hpp; each Record / outcome / YCSBTupleInt must equal the bytes
stated from the reference's definitions over the oracle's answer for the same scenario."""
import pytest

import adapter_expect as A

pytestmark = pytest.mark.gpu


def test_adapter_on_device_results(gpu, tmp_path):
    dst = tmp_path / "probe.bin"
    A.run_tool("probe", str(dst))
    got = A.parse(str(dst))
    t = A.scenario_oracle()
    outs, idents, rows = A.oracle_probe_out(t, A.QUERIES)
    assert [(g[0], g[1]) for g in got] == A.QUERIES
    for i, g in enumerate(got):
        assert g[2] == outs[i]["status"], (i, A.QUERIES[i], g[2], outs[i]["status"])
        assert g[3:] == A.expected(outs[i], rows[i], idents[i]), (i, A.QUERIES[i])
