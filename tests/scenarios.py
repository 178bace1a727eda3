"""Runner of tests/golden/reference_test_scenarios.json (the reference's transaction-level
unit tests restated as op sequences, see tests/golden/make_scenarios.py) against a backend:
the oracle (CPU) or the HIP path through the C-ABI (host write path + stage_sync + device
probes / scans)."""
import json
import os

import numpy as np

import oracle_lib as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_test_scenarios.json")
ST_NOT_FOUND, ST_LATEST, ST_COPY, ST_OLD, ST_FAIL, ST_CHAIN_MISS = range(6)


def load():
    return json.load(open(GOLD))["scenarios"]


def geometry(table):
    """The table geometry both backends run.  The device holds at most 1024 slots per leaf (128
    for variable-length keys); the reference's CreateTable geometry (64 KiB leaves, 8-B payload)
    holds 1637 records per leaf, so its leaf size is halved until the leaf fits -- on BOTH
    backends, and the scenarios never hold more than 11 rows, so no leaf splits in either
    geometry and every expected outcome is unaffected."""
    t = dict(table)
    kpad = 8 if t["key_size"] <= 8 else (t["key_size"] + 7) // 8 * 8
    limit = 128 if t["key_size"] == 0 else 1024
    while (t["leaf_node_size"] - 40) // (24 + kpad + t["payload_size"]) >= limit:
        t["leaf_node_size"] //= 2
        t["split_threshold"] = min(t["split_threshold"], t["leaf_node_size"])
        t["merge_threshold"] = min(t["merge_threshold"], t["leaf_node_size"] // 2)
    return t


def key_of(op, key_size):
    if "key_str" in op:
        b = op["key_str"].encode()
        return b, len(b)
    return int(op["key"]).to_bytes(8, "little")[:key_size], key_size


def payload(op, size):
    p = np.zeros(size, np.uint8)
    w = np.array(op["payload_u64"], np.uint64).view(np.uint8)
    p[:w.size] = w
    return p


class OracleBackend:
    def __init__(self, table):
        self.ks = table["key_size"]
        self.ps = table["payload_size"]
        self.t = O.OracleTree(table["leaf_node_size"], table["split_threshold"], table["payload_size"],
                              table["merge_threshold"])

    def write(self, op):
        k, ks = key_of(op, self.ks)
        o = op["op"]
        if o == "insert":
            return self.t.insert(k, ks, payload(op, self.ps).tobytes(), op["cid"])
        if o == "insert_abort":
            rc = self.t.insert(k, ks, payload(op, self.ps).tobytes(), op["wid"])
            assert rc == 1, rc
            return self.t.abort_insert(k, ks)
        if o == "insert_inflight":
            return self.t.insert_inflight(k, ks, payload(op, self.ps).tobytes(), op["wid"])
        if o == "commit_insert":
            return self.t.commit_insert(k, ks, op["cid"])
        if o == "update":
            d = np.array(op["payload_u64"], np.uint64).view(np.uint8).tobytes()
            return self.t.update(k, ks, op["off"], d, op["wid"])
        if o == "commit_update":
            return self.t.commit_update(k, ks, op["cid"], op["cid"])
        if o == "abort_update":
            return self.t.abort_update(k, ks)
        if o == "finalize_update":
            return self.t.finalize_update(k, ks, op["cid"])
        if o == "delete":
            return self.t.delete(k, ks, op["cid"])
        if o == "update_owned":
            d = np.array(op["payload_u64"], np.uint64).view(np.uint8).tobytes()
            return self.t.update_owned(k, ks, op["off"], d, op["wid"])
        if o == "delete_owned":
            return self.t.delete_owned(k, ks)
        raise ValueError(o)

    def read(self, op):
        k, ks = key_of(op, self.ks)
        out, rec = self.t.read(k, ks, op["rid"], for_update=op.get("for_update", False))
        return int(out["status"]), rec[8:8 + self.ps]

    def scan(self, op):
        k, ks = key_of(op, self.ks)
        c, rows = self.t.scan(k, ks, op["size"])
        return [int.from_bytes(r[:8].tobytes(), "little") for r in rows[:c]]


class DeviceBackend:
    """Writes on the host write path (the reference keeps writes on the host), then every read
    or scan publishes (stage_sync, incremental) and runs on the device."""

    def __init__(self, table):
        import stage
        self.stage = stage
        self.ks = table["key_size"]
        self.ps = table["payload_size"]
        self.t = stage.Table(payload_size=self.ps, leaf_node_size=table["leaf_node_size"],
                             split_threshold=table["split_threshold"], merge_threshold=table["merge_threshold"],
                             key_width=self.ks)

    def write(self, op):
        k, ks = key_of(op, self.ks)
        t = self.t
        o = op["op"]
        if o == "insert":
            return t.insert_key(k, payload(op, self.ps).tobytes(), op["cid"])
        if o == "insert_abort":
            rc = t.insert_key(k, payload(op, self.ps).tobytes(), op["wid"])
            assert rc == 1, rc
            return t.abort_insert_key(k)
        if o == "insert_inflight":
            return t.insert_key_inflight(k, payload(op, self.ps).tobytes(), op["wid"])
        if o == "commit_insert":
            return t.commit_insert_key(k, op["cid"])
        if o == "update":
            d = np.array(op["payload_u64"], np.uint64).view(np.uint8).tobytes()
            return t.update_key(k, op["off"], d, op["wid"])
        if o == "commit_update":
            return t.commit_update_key(k, op["cid"], op["cid"])
        if o == "abort_update":
            return t.abort_update_key(k)
        if o == "finalize_update":
            return t.finalize_update(int.from_bytes(k, "little"), op["cid"], key_size=ks)
        if o == "delete":
            return t.delete_key(k, op["cid"])
        if o == "update_owned":
            d = np.array(op["payload_u64"], np.uint64).view(np.uint8).tobytes()
            return t.update_key_owned(k, op["off"], d, op["wid"])
        if o == "delete_owned":
            return t.delete_key_owned(k)
        raise ValueError(o)

    def _key(self, op):
        k, ks = key_of(op, self.ks)
        return np.array([int.from_bytes(k, "little")], np.uint64), np.array([ks], np.uint16)

    def read(self, op):
        """A read for update goes through stage_probe_batch_ex, whose status record must carry
        STAGE_FLAG_FOR_UPDATE (the executor skips PerformRead, executor.h:388); -1 = flag missing."""
        self.t.sync()
        keys, lens = self._key(op)
        fu = op.get("for_update", False)
        out, rows = self.t.probe(keys, read_ids=np.array([op["rid"]], np.uint32),
                                 lens=lens if self.ks == 0 else None,
                                 for_update=np.array([1], np.uint8) if fu else None)
        flag = (int(out["flags"][0]) & 2) != 0
        if flag != fu:
            return -1, rows[0, 8:8 + self.ps]
        return int(out["status"][0]), rows[0, 8:8 + self.ps]

    def scan(self, op):
        self.t.sync()
        keys, lens = self._key(op)
        counts, rows = self.t.range_scan(keys, op["size"], lens=lens if self.ks == 0 else None)
        return [int.from_bytes(rows[0, j, :8].tobytes(), "little") for j in range(int(counts[0]))]


def run(scenario, backend_cls):
    """Applies every op; returns the list of mismatches (empty = the scenario holds)."""
    b = backend_cls(geometry(scenario["table"]))
    bad = []
    for n, op in enumerate(scenario["ops"]):
        o = op["op"]
        if o == "read":
            st, pay = b.read(op)
            exp = op["expect"]
            if not exp["found"]:
                ok = st in (ST_NOT_FOUND, ST_CHAIN_MISS)
            else:
                ok = st in (ST_LATEST, ST_COPY, ST_OLD) and (pay == payload(exp, len(pay))).all()
            if not ok:
                bad.append((n, op["src"], op, st, pay[:16].tolist()))
        elif o == "scan":
            got = b.scan(op)
            if got != op["expect_keys"]:
                bad.append((n, op["src"], op, got))
        else:
            rc = b.write(op)
            want = op.get("expect_rc", 1)
            if rc != want:
                bad.append((n, op["src"], op, rc))
    return bad
