"""Debug helper: the write-path edge-case sequence, chain of key 9 after each step."""
import sys
import numpy as np
sys.path.insert(0, "stage-indexorganized_amd")
sys.path.insert(0, "tests")
import stage
import oracle_lib as O

tab = stage.Table(key_width=8)
tab.load_ycsb(0, 5000, 8, mode=0)
tab.sync()
orc = O.OracleTree()
orc.load_ycsb(0, 5000, 8, 0)
rids = np.array([0, 1001, 1201, 0xFFFFFFFE], np.uint32)


def show(what):
    out, rows = tab.probe(np.full(rids.size, 9, np.uint64), read_ids=rids)
    o, _ = orc.read_batch(np.full(rids.size, 9, np.uint64), 8, rids)
    print(what, "dev", out["status"].tolist(), out["hops"].tolist(), "orc", o["status"].tolist(), o["hops"].tolist())


rc, ok = tab.update_batch_device(np.zeros(0, np.uint64), 0, np.zeros((0, 8), np.uint8), [])
k = np.array([1, 2, 2], np.uint64)
rc, ok = tab.update_batch_device(k, 995, np.ones((3, 8), np.uint8), 3, 4)
print("invalid", rc.tolist(), ok)
for i in range(3):
    print(orc.update(int(k[i]), 8, 995, bytes(8 * [1]), 3))
show("after invalid")
k = np.full(200, 7, np.uint64)
d = np.where(np.arange(200)[:, None] % 2 == 0, 1, 2).astype(np.uint8).repeat(8, 1)
w = np.arange(10, 210, dtype=np.uint32)
rc, ok = tab.update_batch_device(k, 0, d, w, None)
for i in range(200):
    orc.update(7, 8, 0, d[i].tobytes(), int(w[i]))
show("after key7")
k = np.full(200, 9, np.uint64)
w = np.arange(1000, 1400, 2, dtype=np.uint32)
rc, ok = tab.update_batch_device(k, 0, d, w, w + 1)
for i in range(200):
    r = orc.update(9, 8, 0, d[i].tobytes(), int(w[i]))
    if r == 1:
        orc.commit_update(9, 8, int(w[i]) + 1, int(w[i]) + 1)
show("after key9")
print("host update", tab.update(11, 0, b"x" * 8, 5000), orc.update(11, 8, 0, b"x" * 8, 5000))
tab.sync()
show("after sync")
