"""Writes tests/golden/reference_txn_schedules.json: the reference's TransactionScheduler tests
(test/testing_execute.cpp) whose operations are point reads, point updates, commits and aborts,
with the assertions each test makes on txn_result and on the values its reads returned.

These are the reference's own known answers for the Index-SSN transaction manager the north
star keeps on the host (FindMinSstamp / FindMaxPstamp / PerformRead / PerformUpdate,
transaction_manager.cpp): tests/test_txn_schedules.py runs the schedules through the manager's
restatement (oracle/ssn_txn.hpp, `oracle/_build/txn_parity sched ...`) over the oracle (CPU) and
over the device path through the adapter (GPU), and holds both to these assertions.

Every expected value is an assert in the cited test (read here as text).  Ops are listed in the
order the test enqueues them (TransactionScheduler::sequence, testing_transaction_util.h:
375-413); Read / Update default is_for_update = false (:386, :396).  Tests that insert, delete or
scan are covered at the storage level by make_scenarios.py and are not listed here.

Directives (txn_parity's input): "table new N" = TestingTransactionUtil::CreateTable(N)
(testing_transaction_util.cpp:21-70: keys 0..N-1, value 0, one committed transaction);
"table same" = the previous schedule's table and manager (several schedulers over one table);
"tick N" = N tid-counter values taken by transactions this file does not restate.
Run `python tests/golden/make_txn_schedules.py` to regenerate.
"""
import json
import os

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_txn_schedules.json")


def R(t, key, fu=False):
    return f"op {t} read {key} {int(fu)}"


def U(t, key, value, fu=False):
    return f"op {t} update {key} {value} {int(fu)}"


def C(t):
    return f"op {t} commit"


def A(t):
    return f"op {t} abort"


def sched(name, source, ops, expect, table="table new 10"):
    """expect: {txn: {"result": "SUCCESS"|"ABORTED"|None, "results": {index: value}, "src": "..."}}"""
    return {"name": name, "source": source, "ops": [table] + ops,
            "expect": {str(t): v for t, v in expect.items()}}


def dirty_write():
    out = []
    cases = [  # (ops of T0 / T1 after both updated key 0, asserted results, lines)
        ([C(0), C(1)], ("SUCCESS", "ABORTED", 1), "1019-1038"),
        ([C(1), C(0)], ("SUCCESS", "ABORTED", 1), "1054-1072"),
        ([A(0), C(1)], ("ABORTED", "ABORTED", 0), "1087-1107"),
        ([C(1), A(0)], ("ABORTED", "ABORTED", 0), "1122-1142"),
        ([A(0), A(1)], ("ABORTED", "ABORTED", 0), "1158-1178"),
        ([A(1), A(0)], ("ABORTED", "ABORTED", 0), "1194-1215"),
    ]
    for i, (tail, (r0, r1, obs), lines) in enumerate(cases):
        ops = [U(0, 0, 1), U(1, 0, 2)] + tail + [R(2, 0), C(2)]
        out.append(sched(f"DirtyWriteTest/{i + 1}", f"test/testing_execute.cpp:{lines}", ops, {
            0: {"result": r0, "results": {}}, 1: {"result": r1, "results": {}},
            2: {"result": None, "results": {0: obs}}}))
    return out


def dirty_read():
    return [
        sched("DirtyReadTest/commit", "test/testing_execute.cpp:1237-1259",
              [U(0, 0, 1), R(1, 0), C(0), C(1), R(2, 0), C(2)],
              {0: {"result": "SUCCESS", "results": {}}, 1: {"result": "SUCCESS", "results": {0: 0}},
               2: {"result": None, "results": {0: 1}}}),
        sched("DirtyReadTest/abort", "test/testing_execute.cpp:1274-1296",
              [U(0, 0, 1), R(1, 0), A(0), C(1), R(2, 0), C(2)],
              {0: {"result": "ABORTED", "results": {}}, 1: {"result": "SUCCESS", "results": {0: 0}},
               2: {"result": None, "results": {0: 0}}}),
    ]


def fuzzy_read():
    return [
        sched("FuzzyReadTest/reader-first", "test/testing_execute.cpp:1316-1341",
              [R(0, 0), U(1, 0, 1), C(1), R(0, 0), C(0), R(2, 0), C(2)],
              {0: {"result": "SUCCESS", "results": {0: 0, 1: 0}}, 1: {"result": "SUCCESS", "results": {}},
               2: {"result": None, "results": {0: 1}}}),
        sched("FuzzyReadTest/writer-first", "test/testing_execute.cpp:1356-1387",
              [R(1, 0), R(0, 0), U(1, 0, 1), C(1), R(0, 0), C(0), R(2, 0), C(2)],
              {0: {"result": "SUCCESS", "results": {0: 0, 1: 0}}, 1: {"result": "SUCCESS", "results": {0: 0}},
               2: {"result": None, "results": {0: 1}}}),
    ]


def abort_version_chain():
    return [sched("AbortVersionChainTest/1", "test/testing_execute.cpp:526-533",
                  [U(0, 1, 100), A(0), R(1, 1), C(1)],
                  {0: {"result": None, "results": {}}, 1: {"result": None, "results": {0: 0}}})]


def single_transaction():
    return [
        sched("SingleTransactionTest/1", "test/testing_execute.cpp:564-576",
              [U(0, 0, 1), U(0, 0, 2, True), U(0, 0, 3, True), U(0, 0, 4, True), R(0, 0, True), C(0)],
              {0: {"result": "SUCCESS", "results": {0: 4}}}),
        sched("SingleTransactionTest2/2", "test/testing_execute.cpp:664-689",
              [R(0, 0), R(0, 0), R(0, 0), R(0, 0), U(0, 0, 1), R(0, 0, True), R(0, 100), C(0)],
              {0: {"result": "SUCCESS", "results": {0: 0, 1: 0, 2: 0, 3: 0, 4: 1, 5: -1}}}),
        sched("SingleTransactionTest2/3", "test/testing_execute.cpp:696-720",
              [U(0, 0, 1), R(0, 0, True), U(0, 0, 2, True), R(0, 0, True), U(0, 0, 3, True), R(0, 0, True),
               U(0, 0, 4, True), R(0, 0, True), C(0)],
              {0: {"result": "SUCCESS", "results": {0: 1, 1: 2, 2: 3, 3: 4}}}),
    ]


def concurrent():
    return [sched("ConcurrentTransactionTest/2", "test/testing_execute.cpp:841-866",
                  [U(0, 0, 1), R(1, 0), R(0, 0, True), C(0), R(1, 0), C(1)],
                  {0: {"result": "SUCCESS", "results": {0: 1}}, 1: {"result": "SUCCESS", "results": {0: 0, 1: 0}}})]


def multi_transaction():
    # :888-926 (two schedulers of scans: 3 + 2 transactions, 2 + 1 + 1 begin / commit / abort ids
    # each) ran on this table first; their ids are taken with "tick"
    return [
        sched("MultiTransactionTest/3", "test/testing_execute.cpp:932-943",
              ["tick 10", R(0, 0), A(0), R(1, 0), C(1)],
              {0: {"result": "ABORTED", "results": {}}, 1: {"result": "SUCCESS", "results": {0: 0}}}),
        sched("MultiTransactionTest/4", "test/testing_execute.cpp:948-971",
              [R(0, 0), R(0, 0), R(0, 0), R(0, 0), U(0, 0, 1), R(0, 0, True), R(0, 100, True), C(0), R(1, 0), C(1)],
              {0: {"result": "SUCCESS", "results": {0: 0, 1: 0, 2: 0, 3: 0, 4: 1, 5: -1}},
               1: {"result": "SUCCESS", "results": {0: 1}}}, table="table same"),
        sched("MultiTransactionTest/5", "test/testing_execute.cpp:975-998",
              [R(0, 3), R(0, 4), U(0, 3, 1), A(0), R(1, 3), R(1, 4), U(1, 3, 2), C(1), R(2, 3), R(2, 4), C(2)],
              {0: {"result": "ABORTED", "results": {}}, 1: {"result": "SUCCESS", "results": {0: 0, 1: 0}},
               2: {"result": "SUCCESS", "results": {0: 2, 1: 0}}}, table="table same"),
    ]


def mvcc():
    return [
        sched("MVCCTest/1", "test/testing_execute.cpp:1407-1427",
              [R(0, 0), R(0, 0), R(0, 0), R(0, 0), U(0, 0, 1), R(0, 0, True), R(0, 100, True), C(0), R(1, 0), C(1)],
              {0: {"result": None, "results": {0: 0, 1: 0, 2: 0, 3: 0, 4: 1, 5: -1}},
               1: {"result": None, "results": {0: 1}}}),
        sched("MVCCTest/2", "test/testing_execute.cpp:1431-1440",
              [U(0, 0, 1), U(0, 0, 2, True), U(0, 0, 3, True), U(0, 0, 4, True), R(0, 0, True), C(0)],
              {0: {"result": None, "results": {0: 4}}}, table="table same"),
    ]


def main():
    ss = dirty_write() + dirty_read() + fuzzy_read() + abort_version_chain() + single_transaction() + \
        concurrent() + multi_transaction() + mvcc()
    doc = {"generator": "tests/golden/make_txn_schedules.py", "schedules": ss}
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
    n = sum(1 for s in ss for v in s["expect"].values() if v["result"]) + \
        sum(len(v["results"]) for s in ss for v in s["expect"].values())
    print(f"wrote {OUT}: {len(ss)} schedules, {n} asserted values")


if __name__ == "__main__":
    main()
