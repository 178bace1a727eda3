"""The kept transaction manager against the reference's own assertions (the SSN
restatement was only ever compared with itself).

tests/golden/reference_txn_schedules.json holds the reference's TransactionScheduler tests whose
operations are point reads, point updates, commits and aborts (DirtyWrite, DirtyRead, FuzzyRead,
AbortVersionChain, SingleTransaction, ConcurrentTransaction, MultiTransaction, MVCCTest: 20
schedules), each with the asserts the test makes on txn_result and on its reads' values
(testing_execute.cpp, cited per schedule).  `oracle/_build/txn_parity sched` runs them through
oracle/ssn_txn.hpp -- the restatement of SSNTransactionManager's BeginTransaction, PerformRead,
PerformUpdate, FindMinSstamp, FindMaxPstamp, CommitTransaction and AbortTransaction -- with the
scheduler's rules (testing_transaction_util.h:203-309: begin at the first op, skip after an
abort, a failed executor aborts on the spot, an explicit Abort takes a counter value).

CPU: over the oracle, every asserted value holds.  GPU: over the device path through the
reference-side adapter (probes, for-update probes, owned updates, location cells, overwrite-copy
pool) the same, and the manager's trace equals the oracle-driven one step for step.

Where the reference's sequential driver would wait forever -- a commit that spins in
FindMaxPstamp on a reader that has no commit id yet (DirtyReadTest: the writer commits while its
reader is still open) -- the commit is parked and finished once the reader has committed; the
assertions describe that outcome.  Each such schedule reports its parked commits in the trace."""
import json
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(REPO, "oracle", "_build", "txn_parity")
GOLD = os.path.join(REPO, "tests", "golden", "reference_txn_schedules.json")


def schedules():
    with open(GOLD) as f:
        return json.load(f)["schedules"]


def program(ss):
    lines = []
    for s in ss:
        lines.append(f"schedule {s['name']}")
        lines += s["ops"]
        lines.append("end")
    return "\n".join(lines) + "\n"


def run(mode):
    p = subprocess.run([TOOL, "sched", mode], input=program(schedules()), capture_output=True, text=True,
                       timeout=600)
    return p.returncode, p.stdout, p.stderr


def parse(out):
    res, cur = {}, None
    for line in out.splitlines():
        w = line.split()
        if not w:
            continue
        if w[0] == "schedule":
            cur = res.setdefault(w[1], {})
        elif w[0] == "txn":
            r = w[2].split("=", 1)[1]
            vals = w[3].split("=", 1)[1]
            cur[w[1]] = (r, [int(v) for v in vals.split(",")] if vals else [])
    return res


def check(got):
    ss = schedules()
    assert set(got) == {s["name"] for s in ss}
    n = 0
    for s in ss:
        g = got[s["name"]]
        for t, exp in s["expect"].items():
            result, results = g[t]
            assert result != "BLOCKED", (s["name"], t)
            if exp["result"] is not None:
                assert result == exp["result"], (s["name"], s["source"], t, result)
                n += 1
            for i, v in exp["results"].items():
                assert int(i) < len(results) and results[int(i)] == v, (s["name"], s["source"], t, results)
                n += 1
    return n


def test_golden_schedules_cover_the_manager():
    ss = schedules()
    assert len(ss) == 20
    assert sum(1 for s in ss for v in s["expect"].values() if v["result"]) >= 30


def test_oracle_manager_meets_the_reference_assertions():
    assert os.access(TOOL, os.X_OK), "oracle/_build/txn_parity not built (make -C oracle)"
    rc, out, err = run("oracle")
    assert rc == 0, err
    assert check(parse(out)) >= 80


@pytest.mark.gpu
def test_device_manager_meets_the_reference_assertions(gpu):
    rc, out, err = run("both")
    lines = out.splitlines()
    assert rc == 0 and lines[0] == "MATCH", (out[-4000:], err[-2000:])
    assert check(parse(out)) >= 80
