#!/bin/bash
# Round-6 evidence run on one GPU box, from one tree: the -m gpu suite, smoke, the default bench
# line, the f4 legs (CH-Q2, TPC-C stock-level), C3 alone, the 2-rank shared-GPU rehearsal of the
# the first failure ends it.
set -e
out=${OUT:-gpurun_out/final6c}
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests --durations=20 > $out/tests.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 480 python -u bench.py > $out/bench_default.log 2>&1
timeout -k 10 200 python -u bench.py --config chq2 --steps 300 > $out/bench_chq2.log 2>&1
timeout -k 10 200 python -u bench.py --config tpcc > $out/bench_tpcc.log 2>&1
timeout -k 10 200 python -u bench.py --config c3 --no-cpu-baseline > $out/bench_c3.log 2>&1
STAGE_RANKS_SHARE_GPU=1 timeout -k 10 300 python -u bench.py --gpus 2 --rows 20000000 --steps 5 --warmup 2 \
    --no-cpu-baseline > $out/bench_g2_rehearsal.log 2>&1
