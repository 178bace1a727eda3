"""Writes tests/golden/reference_test_scenarios.json: the reference's own transaction-level
unit tests on the visibility path, restated as op sequences with expected outcomes.

Source of every expected value: the assertion in the reference test it cites (read here as
text; the reference's execute tests cannot pass as shipped -- its point lookups never fill
GetResults(), testing_execute.cpp:305 / executor.h:396 vs :549 -- so the assertions state
the intended semantics, which the fixture pins).  Ids follow the reference's tid counter
(transaction_manager.cpp:14, :287 BeginTransaction read_id = counter++, :552 commit id =
counter++, aborts take no commit id); the counter starts at TID0 = 1 here (the reference's
process-wide counter starts at INVALID_CID = 0 and keeps counting across tests).

Op vocabulary (keys: "key" = u64 little-endian of key_size bytes, "key_str" = ASCII bytes):
  insert        key, payload_u64 (payload = those u64 words), cid: Insert + FinalizeInsert
                (InsertExecutor + CommitTransaction INSERT: FinalizeForInsert(t_cstamp))
  insert_abort  key, payload_u64, wid: Insert by an aborting txn + AbortTransaction INSERT
  update        key, off, payload_u64, wid: LeafNode::Update (PointUpdateExecutor), expect_rc
  commit_update key, cid: CommitTransaction UPDATE entry (sstamp = cid, single writer)
  abort_update  key: AbortTransaction UPDATE entry
  finalize_update key, cid: BTree::FinalizeUpdate (BTreeTest style)
  delete        key, cid: PointDeleteExecutor + CommitTransaction DELETE
  read          key, rid, expect: {"found": false} | {"found": true, "payload_u64": [...]}
                (IndexScanExecutor point lookup at read id rid; canonical payload)
  scan          key, size, expect_keys (TableScanExecutor over RangeScanBySize/Iterator)
Run `python tests/golden/make_scenarios.py` to regenerate.
"""
import json
import os

TID0 = 1
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_test_scenarios.json")


class Counter:
    def __init__(self, start=TID0):
        self.c = start

    def next(self):
        v = self.c
        self.c += 1
        return v


def basic_transaction_test():
    """TEST_F(ExecuteTest, BasicTransactionTest), test/testing_execute.cpp:102-514: a table of
    (u64 key, 10 u64 columns), ParameterSet(64K, 32K, 64K, 80) (:105), n_txns = 10 (:132)."""
    n = 10
    tid = Counter()
    ops = []
    vals = lambda v: [v] * 10
    # :136-166 insert then abort, every key
    for i in range(n):
        r = tid.next()
        ops.append({"op": "insert_abort", "key": i, "payload_u64": vals(i), "wid": r, "src": ":136-166"})
    # :168-201 empty lookups: nothing visible (res.size() == 0, :194)

    def lookup_empty(src):
        for i in range(n):
            r = tid.next()
            ops.append({"op": "read", "key": i, "rid": r, "expect": {"found": False}, "src": src})
            tid.next()  # commit

    lookup_empty(":168-201 (assert :194)")
    # :238-270 committed inserts, values[j] = i
    for i in range(n):
        tid.next()
        c = tid.next()
        ops.append({"op": "insert", "key": i, "payload_u64": vals(i), "cid": c, "src": ":238-270"})
    # :205-235 table scans of 10 from key 0 (printed, not asserted; order per KeyCompare)
    for _ in range(n):
        tid.next()
        ops.append({"op": "scan", "key": 0, "size": 10, "expect_keys": list(range(n)), "src": ":205-235 (derived)"})
        tid.next()

    def lookup_check(inc, src):
        for i in range(n):
            r = tid.next()
            ops.append({"op": "read", "key": i, "rid": r, "expect": {"found": True, "payload_u64": vals(i + inc)},
                        "src": src})
            tid.next()

    lookup_check(0, ":274-312 lookup_check(0) (asserts :304-305)")
    snapshot = tid.c - 1  # :315 GetCurrentTidCounter() - 1
    # :316-367 update every column to i+1, committed
    for i in range(n):
        r = tid.next()
        ops.append({"op": "update", "key": i, "off": 0, "payload_u64": vals(i + 1), "wid": r, "expect_rc": 1,
                    "src": ":316-367"})
        c = tid.next()
        ops.append({"op": "commit_update", "key": i, "cid": c, "src": ":361"})
    lookup_check(1, ":369 lookup_check(1)")
    # :371-418 Lookup-Old: read at snapshot_tid sees the pre-update values (asserts :406-407)
    for i in range(n):
        tid.next()
        ops.append({"op": "read", "key": i, "rid": snapshot, "expect": {"found": True, "payload_u64": vals(i)},
                    "src": ":371-418 Lookup-Old (asserts :406-407)"})
        tid.next()
    # :420-466 "duplicate update": all ten up_col entries are column 1, so the executor writes
    # column 1 ten times with the delta's ten words, i.e. column 1 = i+1 -- equal to its value:
    # ComparePayload -> NotNeededUpdate; the txn aborts with nothing in flight
    for i in range(n):
        r = tid.next()
        ops.append({"op": "update", "key": i, "off": 0, "payload_u64": [i + 1], "wid": r, "expect_rc": 7,
                    "src": ":420-466"})
    lookup_check(1, ":468 lookup_check(1) after the aborted duplicate updates")
    # :470-499 committed deletes, then :501 lookup_empty_check
    for i in range(n):
        tid.next()
        c = tid.next()
        ops.append({"op": "delete", "key": i, "cid": c, "expect_rc": 1, "src": ":470-499"})
    lookup_empty(":501 lookup_empty_check")
    return {"name": "ExecuteTest.BasicTransactionTest", "source": "test/testing_execute.cpp:102-514",
            "table": {"key_size": 8, "payload_size": 80, "split_threshold": 65536, "merge_threshold": 32768,
                      "leaf_node_size": 65536}, "ops": ops}


def create_table(tid, num_key=10):
    """TestingTransactionUtil::CreateTable, test/testing_transaction_util.cpp:21-70: keys
    0..num_key-1 with value 0, one committed transaction, ParameterSet(64K, 32K, 64K, 8)."""
    tid.next()
    c = tid.next()
    return [{"op": "insert", "key": i, "payload_u64": [0], "cid": c, "src": "testing_transaction_util.cpp:63-68"}
            for i in range(num_key)]


CT_TABLE = {"key_size": 8, "payload_size": 8, "split_threshold": 65536, "merge_threshold": 32768,
            "leaf_node_size": 65536}


def abort_version_chain_test():
    """TEST_F(ExecuteTest, AbortVersionChainTest), test/testing_execute.cpp:516-551.  The
    TransactionScheduler runs serially; a txn begins at its first op
    (testing_transaction_util.h:210-219)."""
    tid = Counter()
    ops = create_table(tid)
    r0 = tid.next()  # Txn(0).Update(1, 100) ; Txn(0).Abort()
    ops.append({"op": "update", "key": 1, "off": 0, "payload_u64": [100], "wid": r0, "expect_rc": 1, "src": ":523"})
    ops.append({"op": "abort_update", "key": 1, "expect_rc": 1, "src": ":524"})
    r1 = tid.next()  # Txn(1).Read(1) -> 0
    ops.append({"op": "read", "key": 1, "rid": r1, "expect": {"found": True, "payload_u64": [0]},
                "src": ":525-529 (assert results[0] == 0)"})
    tid.next()
    r0 = tid.next()  # Txn(0).Insert(100, 0) ; Abort
    ops.append({"op": "insert_abort", "key": 100, "payload_u64": [0], "wid": r0, "src": ":534-535"})
    r1 = tid.next()  # Txn(1).Read(100) -> -1
    ops.append({"op": "read", "key": 100, "rid": r1, "expect": {"found": False},
                "src": ":536-540 (assert results[0] == -1)"})
    tid.next()
    return {"name": "ExecuteTest.AbortVersionChainTest", "source": "test/testing_execute.cpp:516-551",
            "table": CT_TABLE, "ops": ops}


def mvcc_test():
    """TEST_F(ExecuteTest, MVCCTest) first schedule, test/testing_execute.cpp:1397-1424: Txn0
    reads key 0 four times, updates it to 1, reads key 100, commits; then Txn1 reads key 0.
    Not restated: Txn0's own-write read of key 0 (is_for_update = true, results[4] == 1) and
    the later schedules of own-write re-updates / insert-delete within one txn -- the writer's
    own path, kept on the host (north star)."""
    tid = Counter()
    ops = create_table(tid)
    r0 = tid.next()
    for k in range(4):
        ops.append({"op": "read", "key": 0, "rid": r0, "expect": {"found": True, "payload_u64": [0]},
                    "src": f":1406 (assert results[{k}] == 0)"})
    ops.append({"op": "update", "key": 0, "off": 0, "payload_u64": [1], "wid": r0, "expect_rc": 1, "src": ":1410"})
    ops.append({"op": "read", "key": 100, "rid": r0, "expect": {"found": False},
                "src": ":1412 (assert results[5] == -1)"})
    c0 = tid.next()
    ops.append({"op": "commit_update", "key": 0, "cid": c0, "src": ":1413"})
    r1 = tid.next()
    ops.append({"op": "read", "key": 0, "rid": r1, "expect": {"found": True, "payload_u64": [1]},
                "src": ":1414 (assert schedules[1].results[0] == 1)"})
    # a reader that began before Txn0 committed still reads the old version
    ops.append({"op": "read", "key": 0, "rid": r0, "expect": {"found": True, "payload_u64": [0]},
                "src": "derived: read id r0 < commit id, inclusive [begin, end] (executor.h:407-449)"})
    tid.next()
    return {"name": "ExecuteTest.MVCCTest", "source": "test/testing_execute.cpp:1397-1424", "table": CT_TABLE,
            "ops": ops}


BT_TABLE = {"key_size": 0, "payload_size": 8, "split_threshold": 3072, "merge_threshold": 1024,
            "leaf_node_size": 4096}


def insert_dummy():
    """BTreeTest::InsertDummy, test/testing_btree.cpp:340-352: keys "0","10",..,"90", payload i,
    commit id = txn_conxt->GetCommitId() = 0 (TransactionContext(0, ..., 0, 0), :355)."""
    return [{"op": "insert", "key_str": str(i), "payload_u64": [i], "cid": 0, "src": "testing_btree.cpp:340-352"}
            for i in range(0, 100, 10)]


def btree_update_test():
    """TEST_F(BTreeTest, Update), test/testing_btree.cpp:472-516."""
    ops = insert_dummy()
    ops += [
        {"op": "read", "key_str": "20", "rid": 5000, "expect": {"found": True, "payload_u64": [20]},
         "src": ":479-481 (assert payload == 20)"},
        {"op": "update", "key_str": "20", "off": 0, "payload_u64": [21], "wid": 5000, "expect_rc": 1, "src": ":486-492"},
        {"op": "read", "key_str": "20", "rid": 5005, "expect": {"found": True, "payload_u64": [20]},
         "src": ":494-500 in flight (assert payload == 20)"},
        {"op": "finalize_update", "key_str": "20", "cid": 5005, "src": ":504"},
        {"op": "read", "key_str": "20", "rid": 5006, "expect": {"found": True, "payload_u64": [21]},
         "src": ":505-510 (assert payload == 21)"},
    ]
    return {"name": "BTreeTest.Update", "source": "test/testing_btree.cpp:472-516", "table": BT_TABLE, "ops": ops}


def btree_upsert_test():
    """TEST_F(BTreeTest, Upsert), test/testing_btree.cpp:518-583: the insert branch (key "abc")
    and the update branch (key "20": in flight reads 20, after FinalizeUpdate 21)."""
    ops = insert_dummy()
    ops += [
        {"op": "read", "key_str": "abc", "rid": 6000, "expect": {"found": False}, "src": ":523-527"},
        {"op": "insert", "key_str": "abc", "payload_u64": [42], "cid": 6000, "src": ":529-539 Upsert insert branch"},
        {"op": "read", "key_str": "abc", "rid": 6000, "expect": {"found": True, "payload_u64": [42]},
         "src": ":541-545 (assert payload_0 == 42)"},
        {"op": "update", "key_str": "20", "off": 0, "payload_u64": [21], "wid": 6001, "expect_rc": 1,
         "src": ":550-556 Upsert update branch"},
        {"op": "read", "key_str": "20", "rid": 6001, "expect": {"found": True, "payload_u64": [20]},
         "src": ":557-565 in flight (assert payload_1 == 20)"},
        {"op": "finalize_update", "key_str": "20", "cid": 6001, "src": ":567-568"},
        {"op": "read", "key_str": "20", "rid": 6002, "expect": {"found": True, "payload_u64": [21]},
         "src": ":569-575 (assert payload_1 == 21)"},
    ]
    return {"name": "BTreeTest.Upsert", "source": "test/testing_btree.cpp:518-583", "table": BT_TABLE, "ops": ops}


def main():
    scen = [basic_transaction_test(), abort_version_chain_test(), mvcc_test(), btree_update_test(),
            btree_upsert_test()]
    doc = {"generator": "tests/golden/make_scenarios.py", "tid0": TID0, "scenarios": scen}
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
    print(f"wrote {OUT}: {sum(len(s['ops']) for s in scen)} ops in {len(scen)} scenarios")


if __name__ == "__main__":
    main()
