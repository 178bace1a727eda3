"""GPU: BASELINE.json configs[4] (YCSB-C 800M rows sharded 8 ways, RCCL key routing) as close as
one MI355X allows -- the data path at C5's per-rank batch over a REAL 8-rank RCCL communicator.

8 processes share device 0 (each its own NCCL_HOSTID: RCCL's socket transport on the loopback
interface, tests/rccl_rank_worker.py) and form one communicator; rank r holds the 12.5M rows of
a 100M-key table with MurmurHash64A(key, 8, 0) % 8 == r and probes its 2^21-key Zipf-0.9 batch
(drawn over all 100M keys) with stage_probe_sharded_ex -- the counts ncclAllToAll, the 8-peer
grouped ncclSend / ncclRecv and the fan-out of returned rows all execute -- in the four reply
modes (rows back over RCCL, rows left at the owner, rows read by the caller from the owner's
IPC-mapped row buffers: STAGE_REPLY_PEER, rows written by the owner into the caller's
IPC-mapped output: STAGE_REPLY_DIRECT).
The reference is ONE 100M-row table's direct probe of the same keys, taken first (in this
process, then released) and saved: every status field and every row (64-bit digest) must match.
Per-rank step times are in the reports; they are not a scaling point (8 ranks share one GPU and
exchange over TCP loopback, not xGMI).  Reference semantics per shard: executor.h:374-454."""
import json
import os
import sys
import tempfile
import time

import numpy as np
import pytest

import stage
from progress import say
from test_gpu_rccl_ranks import rank_env, run_group

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(REPO, "tests", "rccl_full_size_worker.py")
N = 100_000_000
W = 8
PER_RANK = 1 << 21


@pytest.mark.timeout(1000)
def test_c5_rccl_8_ranks_at_size(gpu):
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from rccl_full_size_worker import digest
    t0 = time.time()
    rng = np.random.default_rng(0xC5)
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
        full = stage.Table(key_width=8)
        assert full.load_ycsb(0, N, 8, 0) == N
        full.sync()
        say("100M-row table loaded", t0)
        for r in range(W):
            k = stage.zipf_draws(N - 1, 0.9, 0x5EED + r, PER_RANK - 64, nthreads=16)
            k = np.concatenate([k, rng.integers(N, N + 10_000_000, 64).astype(np.uint64)])
            k = k[rng.permutation(k.size)].astype(np.uint64)
            out, rows = full.probe(k)
            np.save(os.path.join(d, f"keys{r}.npy"), k)
            np.save(os.path.join(d, f"out{r}.npy"), out)
            np.save(os.path.join(d, f"dig{r}.npy"), digest(rows))
            del rows
        full.close()
        del full
        say("direct probes saved; starting 8 ranks", t0)
        envs = [rank_env(r, W, OUTDIR=d, N=str(N)) for r in range(W)]
        rcs, outs = run_group([[sys.executable, "-u", WORKER]] * W, envs, timeout=900)
        reports = []
        for r in range(W):
            path = os.path.join(d, f"rank{r}.json")
            assert os.path.exists(path), f"rank {r} wrote no report (exit {rcs[r]}):\n{outs[r][-3000:]}"
            reports.append(json.load(open(path)))
        say("ranks done", t0)
        for r, rep in enumerate(reports):
            assert rep.get("ok"), (r, rep.get("error"), [c for c in rep.get("cases", []) if not c["ok"]],
                                   outs[r][-2000:])
            assert rep["all_ranks_ok"] and rcs[r] == 0
        for rep in reports:
            assert [c["reply"] for c in rep["cases"]] == ["rows", "owner", "peer", "direct"]
            rows_case = rep["cases"][0]
            assert rows_case["stats"]["remote"] > 0 and rows_case["stats"]["received"] > 0
            print(json.dumps({"rank": rep["rank"], "rows": rep["rows"],
                              "cases": [(c["reply"], c["step_s"], c["stats"]) for c in rep["cases"]]}))
        assert sum(rep["rows"] for rep in reports) == N
