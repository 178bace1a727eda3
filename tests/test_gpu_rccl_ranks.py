"""GPU: the sharded probe over a REAL multi-rank RCCL communicator.

The one-device loopback tests (test_gpu_dist.py) run the multi-GPU data path with device copies
in place of RCCL; here W separate processes form one RCCL communicator and exchange through it.
A one-GPU box cannot give each rank its own device, so all ranks share device 0 and each
declares its own host (NCCL_HOSTID): RCCL then connects them over its socket transport on the
loopback interface (it refuses two ranks of one host on one device).  The counts ncclAllToAll,
the grouped ncclSend / ncclRecv with real peers, the control-plane allreduce / allgather and the
bench's N > 1 code path all execute; xGMI bandwidth is the one thing not exercised.

Every rank compares its results with a table holding every key (tests/rccl_rank_worker.py);
the bench rehearsal checks its own self-check and its N > 1 line."""
import json
import os
import signal
import subprocess
import sys
import tempfile

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(REPO, "tests", "rccl_rank_worker.py")


def run_group(cmds, envs, timeout):
    """start every rank in its own process group; kill them all if any is still running at
    the timeout; returns (return codes, outputs)"""
    procs = []
    for cmd, env in zip(cmds, envs):
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                                      start_new_session=True))
    outs, rcs = [], []
    try:
        for p in procs:
            o, _ = p.communicate(timeout=timeout)
            outs.append(o)
            rcs.append(p.returncode)
    except subprocess.TimeoutExpired:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
        for p in procs:
            p.wait()
        pytest.fail(f"ranks still running after {timeout}s")
    return rcs, outs


def rank_env(rank, world, **extra):
    env = dict(os.environ)
    env.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": "0",
                "HSA_ENABLE_IPC_MODE_LEGACY": "0", "NCCL_DEBUG": os.environ.get("NCCL_DEBUG", "WARN"), **extra})
    return env


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_probe_over_rccl_ranks(gpu, world):
    with tempfile.TemporaryDirectory() as d:
        envs = [rank_env(r, world, OUTDIR=d) for r in range(world)]
        rcs, outs = run_group([[sys.executable, "-u", WORKER]] * world, envs, timeout=300)
        reports = []
        for r in range(world):
            path = os.path.join(d, f"rank{r}.json")
            assert os.path.exists(path), f"rank {r} wrote no report (exit {rcs[r]}):\n{outs[r][-3000:]}"
            reports.append(json.load(open(path)))
        # every failing rank's last error line and its library diagnostics, not only the first rank's
        bad = [(r, (rep.get("error") or "").strip().splitlines()[-1:], [c for c in rep.get("cases", []) if not c["ok"]],
                [ln for ln in outs[r].splitlines() if ln.startswith("[") or "IPC" in ln][-6:])
               for r, rep in enumerate(reports) if not rep.get("ok")]
        assert not bad, bad
        for r, rep in enumerate(reports):
            assert rep["all_ranks_ok"]
            assert rcs[r] == 0
        # the exchange carried requests between the processes
        for rep in reports:
            for c in rep["cases"]:
                if c["keys"]:
                    assert c["stats"]["remote"] > 0 and c["stats"]["received"] > 0
            print(json.dumps({"rank": rep["rank"], "rccl": rep["rccl"],
                              "cases": [(c["case"], c["stats"]) for c in rep["cases"]]}))


def test_bench_multi_rank_line_over_rccl(gpu):
    # the bench's own N > 1 path (launcher, torch.distributed.run ranks, RCCL control plane,
    # sharded steps in both reply modes, self-check, the line's fields) at 2 ranks, small tables
    env = dict(os.environ, STAGE_RANKS_SHARE_GPU="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--rows", "2000000", "--batch", "1048576",
           "--steps", "3", "--warmup", "1", "--no-cpu-baseline"]
    rcs, outs = run_group([cmd], [env], timeout=300)
    lines = [s for s in outs[0].splitlines() if s.startswith("{") and '"metric"' in s]
    assert rcs[0] == 0 and lines, outs[0][-4000:]
    line = json.loads(lines[-1])
    assert line["n_gpus"] == 2 and line["self_check"]
    assert "sharing 1×MI355X" in line["config"]["workload"] and "rehearsal" in line["config"]["workload"]
    assert [p["rank"] for p in line["per_rank"]] == [0, 1] and all(p["self_check"] for p in line["per_rank"])
    assert line["coalescing"]["remote_requests"] > 0
    assert line["rccl"]["runtime"] > 0
    # auto: every full-reply mode was timed (or its refusal noted); the line names the fastest
    replies = {"peer": "peer_reply", "rows": "rows_reply", "direct": "direct_reply"}
    assert line["reply"] in replies and all(v in line for k, v in replies.items() if k != line["reply"]), line
    print(json.dumps({k: line.get(k) for k in ("value", "ms_per_step", "reply", "peer_reply", "rows_reply",
                                               "direct_reply", "owner_reply", "coalescing", "rccl")}))
