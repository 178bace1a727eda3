#!/bin/bash
# Round-5 validation call (one GPU box): the new parity tests (SSN schedules, peer reply, CH-Q2
# one-sync batch), the CH-Q2 bench and its trace, and a 2-rank shared-GPU rehearsal of the N > 1
# bench (peer reply).  Each GPU step has its own time limit; the first failure ends the script.
set -e
out=gpurun_out/q2p
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_txn_schedules.py tests/test_txn_parity.py tests/test_gpu_dist.py tests/test_gpu_rccl_ranks.py \
    tests/test_gpu_chq2.py tests/test_gpu_tpcc.py tests/test_gpu_wide_keys.py tests/test_small_rows.py \
    > $out/tests.log 2>&1
timeout -k 10 120 python -u bench.py --config chq2 --steps 300 > $out/bench_chq2.log 2>&1
STAGE_Q2_TRACE=1 timeout -k 10 120 python -u bench.py --config chq2 --steps 50 > $out/trace.log 2>&1
STAGE_RANKS_SHARE_GPU=1 timeout -k 10 300 python -u bench.py --gpus 2 --rows 20000000 --steps 5 --warmup 2 \
    --no-cpu-baseline > $out/bench_g2.log 2>&1
STAGE_Q2_TRACE=1 timeout -k 10 120 python -u bench.py --config chq2 --steps 20 > $out/trace2.log 2>&1
bash scripts/profile_r05.sh q2_trace > $out/prof_q2.log 2>&1
