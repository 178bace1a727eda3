"""Writes tests/golden/reference_test_scenarios.json: the reference's own transaction-level
unit tests on the visibility path, restated as op sequences with expected outcomes.

Source of every expected value: the assertion in the reference test it cites (read here as
text; the reference's execute tests cannot pass as shipped -- its point lookups never fill
GetResults(), testing_execute.cpp:305 / executor.h:396 vs :549 -- so the assertions state
the intended semantics, which the fixture pins).  Ids follow the reference's tid counter
(transaction_manager.cpp:14, :287 BeginTransaction read_id = counter++, :552 commit id =
counter++, aborts take no commit id); the counter starts at TID0 = 1 here (the reference's
process-wide counter starts at INVALID_CID = 0 and keeps counting across tests).
TransactionScheduler tests (testing_transaction_util.h:203-309) run their ops one at a time in
the written order; a txn begins (read id = counter++) at its first op; an explicit Abort() op
takes a counter value (GetNextCurrentTidCounter, :275); a txn whose op failed (e.g. an update
of a record another txn is updating: Dirty) is aborted on the spot without one, and its later
ops are skipped (:221-224, :302-308).  Since round 5 the ops with is_for_update = true (the
writer's reads, updates and deletes of its own record, MVCCTest) are restated too.

Op vocabulary (keys: "key" = u64 little-endian of key_size bytes, "key_str" = ASCII bytes):
  insert        key, payload_u64 (payload = those u64 words), cid: Insert + FinalizeInsert
                (InsertExecutor + CommitTransaction INSERT: FinalizeForInsert(t_cstamp))
  insert_abort  key, payload_u64, wid: Insert by an aborting txn + AbortTransaction INSERT
  insert_inflight key, payload_u64, wid: Insert by a txn that has not committed (the record
                stays PrepareForInsert, b_tree.cpp:860-864)
  commit_insert key, cid: CommitTransaction INSERT entry (FinalizeForInsert(t_cstamp), :677-695)
  update        key, off, payload_u64, wid: LeafNode::Update (PointUpdateExecutor), expect_rc
  commit_update key, cid: CommitTransaction UPDATE entry (sstamp = cid, single writer)
  abort_update  key: AbortTransaction UPDATE entry
  finalize_update key, cid: BTree::FinalizeUpdate (BTreeTest style)
  delete        key, cid: PointDeleteExecutor + CommitTransaction DELETE
  update_owned  key, off, payload_u64, wid: LeafNode::Update with is_for_update = true (in place)
  delete_owned  key: LeafNode::Delete with is_for_update = true (meta := 0)
  read          key, rid, expect: {"found": false} | {"found": true, "payload_u64": [...]}
                (IndexScanExecutor point lookup at read id rid; canonical payload);
                for_update: true = BTree::Read(.., is_for_update = true), PerformRead skipped
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
    tid.next()  # the explicit Abort() takes a counter value
    r1 = tid.next()  # Txn(1).Read(1) -> 0
    ops.append({"op": "read", "key": 1, "rid": r1, "expect": {"found": True, "payload_u64": [0]},
                "src": ":525-529 (assert results[0] == 0)"})
    tid.next()
    r0 = tid.next()  # Txn(0).Insert(100, 0) ; Abort
    ops.append({"op": "insert_abort", "key": 100, "payload_u64": [0], "wid": r0, "src": ":534-535"})
    tid.next()  # Abort()
    r1 = tid.next()  # Txn(1).Read(100) -> -1
    ops.append({"op": "read", "key": 100, "rid": r1, "expect": {"found": False},
                "src": ":536-540 (assert results[0] == -1)"})
    tid.next()
    return {"name": "ExecuteTest.AbortVersionChainTest", "source": "test/testing_execute.cpp:516-551",
            "table": CT_TABLE, "ops": ops}


def mvcc_test():
    """TEST_F(ExecuteTest, MVCCTest), test/testing_execute.cpp:1397-1470, all three schedules.
    Schedule 1 (:1405-1428): Txn0 reads key 0 four times, updates it to 1, reads it back for
    update (its own in-flight update: BTree::Read(.., is_for_update = true) reads the leaf, not the
    copy -- b_tree.cpp:2087, 2114-2120 -- and the executor skips PerformRead, executor.h:388), reads
    key 100 for update, commits; then Txn1 reads key 0.  Schedule 2 (:1430-1441): one txn updates
    key 0 to 1 (already 1: NotNeededUpdate), then to 2, 3, 4 with is_for_update = true (LeafNode::
    Update's in-place branch, b_tree.cpp:1101-1104) and reads 4 back for update.  Schedule 3
    (:1443-1470): one txn inserts key 1000, deletes it for update (meta := 0, b_tree.cpp:1210-1220),
    reads nothing, again, then inserts it, reads 2, updates it in place to 3 and reads 3."""
    tid = Counter()
    ops = create_table(tid)
    # schedule 1
    r0 = tid.next()
    for k in range(4):
        ops.append({"op": "read", "key": 0, "rid": r0, "expect": {"found": True, "payload_u64": [0]},
                    "src": f":{1409 + k} (assert results[{k}] == 0, :{1421 + k})"})
    ops.append({"op": "update", "key": 0, "off": 0, "payload_u64": [1], "wid": r0, "expect_rc": 1, "src": ":1413"})
    ops.append({"op": "read", "key": 0, "rid": r0, "for_update": True, "expect": {"found": True, "payload_u64": [1]},
                "src": ":1414 Read(0, true) (assert results[4] == 1, :1425)"})
    ops.append({"op": "read", "key": 100, "rid": r0, "for_update": True, "expect": {"found": False},
                "src": ":1415 Read(100, true) (assert results[5] == -1, :1426)"})
    c0 = tid.next()
    ops.append({"op": "commit_update", "key": 0, "cid": c0, "src": ":1416"})
    r1 = tid.next()
    ops.append({"op": "read", "key": 0, "rid": r1, "expect": {"found": True, "payload_u64": [1]},
                "src": ":1417 (assert schedules[1].results[0] == 1, :1427)"})
    # a reader that began before Txn0 committed still reads the old version
    ops.append({"op": "read", "key": 0, "rid": r0, "expect": {"found": True, "payload_u64": [0]},
                "src": "derived: read id r0 < commit id, inclusive [begin, end] (executor.h:407-449)"})
    tid.next()
    # schedule 2
    r2 = tid.next()
    ops.append({"op": "update", "key": 0, "off": 0, "payload_u64": [1], "wid": r2, "expect_rc": 7,
                "src": ":1433 Update(0, 1, false): the value is already 1 (ComparePayload -> NotNeededUpdate)"})
    for v, line in ((2, 1434), (3, 1435), (4, 1436)):
        ops.append({"op": "update_owned", "key": 0, "off": 0, "payload_u64": [v], "wid": r2, "expect_rc": 1,
                    "src": f":{line} Update(0, {v}, true) (LeafNode::Update in place, b_tree.cpp:1101-1104)"})
    ops.append({"op": "read", "key": 0, "rid": r2, "for_update": True, "expect": {"found": True, "payload_u64": [4]},
                "src": ":1437 Read(0, true) (assert results[0] == 4, :1440)"})
    tid.next()  # Commit(): nothing in the rw-set (the updates were for update, the first NotNeeded)
    r = tid.next()
    ops.append({"op": "read", "key": 0, "rid": r, "expect": {"found": True, "payload_u64": [4]},
                "src": "derived: an in-place update keeps the record's cstamp; a later reader sees 4"})
    tid.next()
    # schedule 3
    r3 = tid.next()
    for n, v in enumerate((0, 1)):
        ops.append({"op": "insert_inflight", "key": 1000, "payload_u64": [v], "wid": r3,
                    "src": f":{1448 + 4 * n} Insert(1000, {v}) (InsertExecutor: BTree::Insert at the read id)"})
        ops.append({"op": "delete_owned", "key": 1000, "expect_rc": 1,
                    "src": f":{1449 + 4 * n} Delete(1000, true) (LeafNode::Delete: meta := 0, b_tree.cpp:1210-1220)"})
        ops.append({"op": "read", "key": 1000, "rid": r3, "for_update": True, "expect": {"found": False},
                    "src": f":{1450 + 4 * n} Read(1000, true) (assert results[{n}] == -1, :{1466 + n})"})
    ops.append({"op": "insert_inflight", "key": 1000, "payload_u64": [2], "wid": r3, "src": ":1456 Insert(1000, 2)"})
    ops.append({"op": "read", "key": 1000, "rid": r3, "for_update": True, "expect": {"found": True, "payload_u64": [2]},
                "src": ":1457 Read(1000, true) (assert results[2] == 2, :1468)"})
    ops.append({"op": "update_owned", "key": 1000, "off": 0, "payload_u64": [3], "wid": r3, "expect_rc": 1,
                "src": ":1459 Update(1000, 3, true)"})
    ops.append({"op": "read", "key": 1000, "rid": r3, "for_update": True, "expect": {"found": True, "payload_u64": [3]},
                "src": ":1460 Read(1000, true) (assert results[3] == 3, :1469)"})
    # an other transaction's read of the uncommitted insert returns nothing (b_tree.cpp:2087-2095)
    ops.append({"op": "read", "key": 1000, "rid": r3, "expect": {"found": False},
                "src": "derived: not for update, the in-flight insert has no copy -> nullptr"})
    c3 = tid.next()
    ops.append({"op": "commit_insert", "key": 1000, "cid": c3,
                "src": ":1462 Commit() (CommitTransaction INSERT: FinalizeForInsert(t_cstamp) on the live record)"})
    r = tid.next()
    ops.append({"op": "read", "key": 1000, "rid": r, "expect": {"found": True, "payload_u64": [3]},
                "src": "derived: after the commit another reader sees 3"})
    tid.next()
    return {"name": "ExecuteTest.MVCCTest", "source": "test/testing_execute.cpp:1397-1470", "table": CT_TABLE,
            "ops": ops}


def read(key, rid, value, src):
    """a point lookup of another transaction; value None = no tuple (-1)"""
    exp = {"found": False} if value is None else {"found": True, "payload_u64": [value]}
    return {"op": "read", "key": key, "rid": rid, "expect": exp, "src": src}


def upd(key, value, wid, src, rc=1):
    """TestingTransactionUtil::ExecuteUpdate: column 1 (the value) := value (testing_transaction_util.cpp:139-160)"""
    return {"op": "update", "key": key, "off": 0, "payload_u64": [value], "wid": wid, "expect_rc": rc, "src": src}


def concurrent_transaction_tests():
    """TEST_F(ExecuteTest, ConcurrentTransactionTest), test/testing_execute.cpp:808-871, two
    schedules on fresh tables.  Not restated: Txn 0's own-write reads (Read(.., true))."""
    out = []
    # :819-836 Txn0 inserts key 100; Txn1 reads it in flight and after Txn0's commit: both -1
    tid = Counter()
    ops = create_table(tid)
    r0 = tid.next()
    ops.append({"op": "insert_inflight", "key": 100, "payload_u64": [1], "wid": r0, "src": ":819 Insert(100, 1)"})
    r1 = tid.next()
    ops.append(read(100, r1, None, ":820 (assert :832 schedules[1].results[0] == -1): an uncommitted insert"))
    c0 = tid.next()
    ops.append({"op": "commit_insert", "key": 100, "cid": c0, "src": ":822 Txn(0).Commit()"})
    ops.append(read(100, r1, None, ":823 (assert :836 results[1] == -1): committed after Txn1 began (no version)"))
    tid.next()  # Txn1 commit
    ops.append(read(100, tid.next(), 1, "derived: a txn that begins after the commit reads it (latest)"))
    out.append({"name": "ExecuteTest.ConcurrentTransactionTest/insert", "source": "test/testing_execute.cpp:810-839",
                "table": CT_TABLE, "ops": ops})
    # :849-866 Txn0 updates key 0 to 1; Txn1 reads it in flight and after the commit: both 0
    tid = Counter()
    ops = create_table(tid)
    r0 = tid.next()
    ops.append(upd(0, 1, r0, ":849 Update(0, 1)"))
    r1 = tid.next()
    ops.append(read(0, r1, 0, ":850 (assert :865 results[0] == 0): the overwrite copy"))
    c0 = tid.next()
    ops.append({"op": "commit_update", "key": 0, "cid": c0, "src": ":852"})
    ops.append(read(0, r1, 0, ":853 (assert :866 results[1] == 0): the retired version"))
    tid.next()
    out.append({"name": "ExecuteTest.ConcurrentTransactionTest/update", "source": "test/testing_execute.cpp:841-869",
                "table": CT_TABLE, "ops": ops})
    return out


def multi_transaction_test():
    """TEST_F(ExecuteTest, MultiTransactionTest), test/testing_execute.cpp:873-1004: five
    schedules on one table.  Scan(-1) passes the 4-byte int -1 as an 8-byte key
    (testing_transaction_util.cpp:182, the upper 4 bytes are whatever follows it): its first
    byte 0xFF is -1 under KeyCompare's signed bytes, below every key, so the 20-record scan
    returns all 10 rows -- results.size() == 10.  The upper bytes are taken as 0 here."""
    tid = Counter()
    ops = create_table(tid)
    start = 0xFFFFFFFF
    keys = list(range(10))
    scan = lambda src: {"op": "scan", "key": start, "size": 20, "expect_keys": keys, "src": src}
    # :889-905
    tid.next()
    ops.append(scan(":890 Txn(0).Scan(-1, true) (assert :905 results.size() == 10)"))
    tid.next()
    ops.append(scan(":891 Txn(1).Scan(-1)"))
    tid.next()  # Txn1 commit
    tid.next()
    ops.append(scan(":893 Txn(2).Scan(-1, true)"))
    tid.next()
    tid.next()
    # :913-925
    tid.next()
    ops.append(scan(":914 Txn(0).Scan(-1, true)"))
    tid.next()  # Abort()
    tid.next()
    ops.append(scan(":916 Txn(1).Scan(-1, true) (assert :925 results.size() == 10)"))
    tid.next()
    # :933-943
    r0 = tid.next()
    ops.append(read(0, r0, 0, ":934 Txn(0).Read(0)"))
    tid.next()  # Abort()
    r1 = tid.next()
    ops.append(read(0, r1, 0, ":936 (assert :943 results.size() == 1; key 0 holds 0)"))
    tid.next()
    # :949-971
    r0 = tid.next()
    for k, line in enumerate((950, 951, 952, 953)):
        ops.append(read(0, r0, 0, f":{line} (assert :{965 + k} results[{k}] == 0)"))
    ops.append(upd(0, 1, r0, ":954 Update(0, 1)"))
    ops.append(read(100, r0, None, ":956 Read(100, true) of a missing key (assert :970 results[5] == -1)"))
    c0 = tid.next()
    ops.append({"op": "commit_update", "key": 0, "cid": c0, "src": ":957"})
    r1 = tid.next()
    ops.append(read(0, r1, 1, ":958 (assert :971 schedules[1].results[0] == 1)"))
    tid.next()
    # :977-998 commit / abort with part of the read tuples updated
    r0 = tid.next()
    ops.append(read(3, r0, 0, ":978"))
    ops.append(read(4, r0, 0, ":979"))
    ops.append(upd(3, 1, r0, ":980 Update(3, 1)"))
    ops.append({"op": "abort_update", "key": 3, "expect_rc": 1, "src": ":981 Abort()"})
    tid.next()
    r1 = tid.next()
    ops.append(read(3, r1, 0, ":982 (assert :995 results[0] == 0)"))
    ops.append(read(4, r1, 0, ":983 (assert :996 results[1] == 0)"))
    ops.append(upd(3, 2, r1, ":984 Update(3, 2)"))
    c1 = tid.next()
    ops.append({"op": "commit_update", "key": 3, "cid": c1, "src": ":985"})
    r2 = tid.next()
    ops.append(read(3, r2, 2, ":986 (assert :997 schedules[2].results[0] == 2)"))
    ops.append(read(4, r2, 0, ":987 (assert :998 results[1] == 0)"))
    tid.next()
    return {"name": "ExecuteTest.MultiTransactionTest", "source": "test/testing_execute.cpp:873-1004",
            "table": CT_TABLE, "ops": ops}


def dirty_write_tests():
    """TEST_F(ExecuteTest, DirtyWriteTest), test/testing_execute.cpp:1007-1225: Txn0 and Txn1
    update key 0 one after the other; Txn1's update meets Txn0's in-flight record (Dirty), so
    Txn1 is aborted on the spot (asserted ABORTED in every schedule) and its Commit / Abort op is
    skipped; the observer Txn2 reads what Txn0's end left."""
    out = []
    cases = [("T0 commit, T1 commit", "commit", 1, ":1018-1038"), ("T1 commit, T0 commit", "commit", 1, ":1053-1072"),
             ("T0 abort, T1 commit", "abort", 0, ":1086-1107"), ("T1 commit, T0 abort", "abort", 0, ":1126-1142"),
             ("T0 abort, T1 abort", "abort", 0, ":1157-1178"), ("T1 abort, T0 abort", "abort", 0, ":1194-1215")]
    for name, t0_end, value, src in cases:
        tid = Counter()
        ops = create_table(tid)
        r0 = tid.next()
        ops.append(upd(0, 1, r0, "Txn(0).Update(0, 1)"))
        r1 = tid.next()
        ops.append(upd(0, 2, r1, "Txn(1).Update(0, 2): Dirty, Txn1 aborted", rc=9))
        if t0_end == "commit":
            ops.append({"op": "commit_update", "key": 0, "cid": tid.next(), "src": "Txn(0).Commit()"})
        else:
            ops.append({"op": "abort_update", "key": 0, "expect_rc": 1, "src": "Txn(0).Abort()"})
            tid.next()
        r2 = tid.next()
        last = src.split("-")[1]
        ops.append(read(0, r2, value, f"observer Txn(2).Read(0) (assert :{last} results[0] == {value})"))
        tid.next()
        out.append({"name": f"ExecuteTest.DirtyWriteTest/{name}", "source": f"test/testing_execute.cpp{src}",
                    "table": CT_TABLE, "ops": ops})
    return out


def dirty_read_tests():
    """TEST_F(ExecuteTest, DirtyReadTest), test/testing_execute.cpp:1227-1304: Txn1 reads key 0
    while Txn0's update is in flight -- the overwrite copy (old value) -- then Txn0 commits or
    aborts and the observer reads the outcome."""
    out = []
    for name, t0_end, value, src, a1, a2 in (("commit", "commit", 1, ":1229-1264", 1258, 1259),
                                            ("abort", "abort", 0, ":1266-1301", 1295, 1296)):
        tid = Counter()
        ops = create_table(tid)
        r0 = tid.next()
        ops.append(upd(0, 1, r0, "Txn(0).Update(0, 1)"))
        r1 = tid.next()
        ops.append(read(0, r1, 0, f"Txn(1).Read(0) during the update (assert :{a1} results[0] == 0)"))
        if t0_end == "commit":
            ops.append({"op": "commit_update", "key": 0, "cid": tid.next(), "src": "Txn(0).Commit()"})
        else:
            ops.append({"op": "abort_update", "key": 0, "expect_rc": 1, "src": "Txn(0).Abort()"})
            tid.next()
        tid.next()  # Txn1 commit
        r2 = tid.next()
        ops.append(read(0, r2, value, f"observer (assert :{a2} results[0] == {value})"))
        tid.next()
        out.append({"name": f"ExecuteTest.DirtyReadTest/{name}", "source": f"test/testing_execute.cpp{src}",
                    "table": CT_TABLE, "ops": ops})
    return out


def fuzzy_read_tests():
    """TEST_F(ExecuteTest, FuzzyReadTest), test/testing_execute.cpp:1306-1395: a reader that
    began before a concurrent update commits keeps reading the old version (TupleHeader chain)."""
    out = []
    # :1315-1341: T0 begins first
    tid = Counter()
    ops = create_table(tid)
    r0 = tid.next()
    ops.append(read(0, r0, 0, ":1322 (assert :1338 results[0] == 0)"))
    r1 = tid.next()
    ops.append(upd(0, 1, r1, ":1323 Txn(1).Update(0, 1)"))
    ops.append({"op": "commit_update", "key": 0, "cid": tid.next(), "src": ":1324"})
    ops.append(read(0, r0, 0, ":1325 should read the old version (assert :1339 results[1] == 0)"))
    tid.next()
    ops.append(read(0, tid.next(), 1, "observer (assert :1341 results[0] == 1)"))
    tid.next()
    out.append({"name": "ExecuteTest.FuzzyReadTest/reader-first", "source": "test/testing_execute.cpp:1308-1346",
                "table": CT_TABLE, "ops": ops})
    # :1355-1387: T1 begins first, reads, T0 reads, T1 updates + commits, T0 reads again
    tid = Counter()
    ops = create_table(tid)
    r1 = tid.next()
    ops.append(read(0, r1, 0, ":1363 (assert :1384 schedules[1].results[0] == 0)"))
    r0 = tid.next()
    ops.append(read(0, r0, 0, ":1364 (assert :1382 results[0] == 0)"))
    ops.append(upd(0, 1, r1, ":1365 Txn(1).Update(0, 1)"))
    ops.append({"op": "commit_update", "key": 0, "cid": tid.next(), "src": ":1366"})
    ops.append(read(0, r0, 0, ":1367 (assert :1383 results[1] == 0)"))
    tid.next()
    ops.append(read(0, tid.next(), 1, "observer (assert :1387 results[0] == 1)"))
    tid.next()
    out.append({"name": "ExecuteTest.FuzzyReadTest/writer-first", "source": "test/testing_execute.cpp:1348-1392",
                "table": CT_TABLE, "ops": ops})
    return out


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
            btree_upsert_test()] + concurrent_transaction_tests() + [multi_transaction_test()] + \
        dirty_write_tests() + dirty_read_tests() + fuzzy_read_tests()
    doc = {"generator": "tests/golden/make_scenarios.py", "tid0": TID0, "scenarios": scen}
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
    print(f"wrote {OUT}: {sum(len(s['ops']) for s in scen)} ops in {len(scen)} scenarios")


if __name__ == "__main__":
    main()
