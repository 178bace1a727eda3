"""CPU: the reference's transaction-level unit tests on the visibility path, restated as op
sequences (tests/golden/reference_test_scenarios.json, made by tests/golden/make_scenarios.py
from testing_execute.cpp BasicTransactionTest incl. Lookup-Old, AbortVersionChainTest,
ConcurrentTransactionTest, MultiTransactionTest, DirtyWriteTest (observer reads), DirtyReadTest,
FuzzyReadTest, MVCCTest and testing_btree.cpp Update / Upsert):

* the oracle meets every expected outcome the reference tests assert;
* the product's host write path (insert / update / commit / abort / delete on the C-ABI)
  leaves every leaf identical to the oracle's after each write (the device reads of the same
  scenarios are tests/test_gpu_scenarios.py).

Round 5: MVCCTest is restated in full (its three schedules), including the writer's own-record
operations with is_for_update = true -- reads (results[4] == 1, :1425; 4, :1440; -1 / -1 / 2 / 3,
:1466-1469), in-place updates and deletes (stage_update_key_owned / stage_delete_key_owned).
"""
import pytest

import scenarios as S
import stage
from test_host_layout import compare_layout

SCEN = S.load()


@pytest.mark.parametrize("sc", SCEN, ids=[s["name"] for s in SCEN])
def test_oracle_meets_reference_assertions(sc):
    assert S.run(sc, S.OracleBackend) == []


@pytest.mark.parametrize("sc", SCEN, ids=[s["name"] for s in SCEN])
def test_host_write_path_matches_oracle_layout(sc):
    g = S.geometry(sc["table"])
    o = S.OracleBackend(g)
    h = S.DeviceBackend(g)  # host side only: no sync, no device call
    for op in sc["ops"]:
        if op["op"] in ("read", "scan"):
            continue
        assert h.write(op) == o.write(op), op
        compare_layout(h.t, o.t)


def test_fixture_covers_the_cited_assertions():
    names = {s["name"] for s in SCEN}
    assert {"ExecuteTest.BasicTransactionTest", "ExecuteTest.AbortVersionChainTest", "ExecuteTest.MVCCTest",
            "BTreeTest.Update", "BTreeTest.Upsert"} <= names
    srcs = " ".join(op["src"] for s in SCEN for op in s["ops"])
    for cited in (":371-418 Lookup-Old", ":525-529", ":536-540", ":1414", ":557-565", ":569-575"):
        assert cited in srcs
    # round 3: the other-transaction read path of the scheduler tests
    assert {"ExecuteTest.ConcurrentTransactionTest/insert", "ExecuteTest.ConcurrentTransactionTest/update",
            "ExecuteTest.MultiTransactionTest", "ExecuteTest.DirtyReadTest/commit", "ExecuteTest.DirtyReadTest/abort",
            "ExecuteTest.FuzzyReadTest/reader-first", "ExecuteTest.FuzzyReadTest/writer-first"} <= names
    assert sum(n.startswith("ExecuteTest.DirtyWriteTest/") for n in names) == 6
    for cited in (":832", ":836", ":865", ":866", ":905", ":925", ":943", ":965", ":970", ":971", ":995", ":998",
                  ":1038", ":1072", ":1107", ":1142", ":1178", ":1215", ":1258", ":1259", ":1295", ":1296",
                  ":1338", ":1339", ":1341", ":1382", ":1383", ":1384", ":1387"):
        assert f"assert {cited}" in srcs, cited
    # round 5: MVCCTest's is_for_update operations (testing_execute.cpp:1414-1469)
    for cited in (":1425", ":1426", ":1427", ":1440", ":1466", ":1467", ":1468", ":1469"):
        assert f"{cited})" in srcs, cited
    fu = [op for s in SCEN for op in s["ops"] if op.get("for_update")]
    assert len(fu) == 7 and {op["op"] for s in SCEN for op in s["ops"]} >= {"update_owned", "delete_owned"}
    assert stage.RC_NOT_NEEDED_UPDATE == 7
