import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "stage-indexorganized_amd"))
import numpy as np
import stage
from test_wide_keys import build, tpcc_like
for nk in (3000, 6000, 8000, 16000):
    keys = tpcc_like(16)[:nk]
    tab, orc, pays = build(16, 320, keys)
    tab.sync()
    tr = tab.traverse(keys); rs = tab.resolve(keys)
    out, rows = tab.probe(keys)
    bad = np.nonzero(out["status"] != 1)[0]
    print(nk, "leaves", tab.stats()["leaves"], "resolve!=traverse", int((tr != rs).sum()), "notfound", bad.size,
          bad[:5], keys[bad[:2]].view(np.int64) if bad.size else "")
    if bad.size:
        print(" leaf", out["leaf"][bad[:5]], "traverse", tr[bad[:5]])
