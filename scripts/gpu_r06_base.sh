#!/bin/bash
# Round-6 baseline on one GPU box: the -m gpu suite, smoke and the default bench line.
set -e
out=gpurun_out/r06base
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests --durations=30 > $out/tests.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 420 python -u bench.py > $out/bench_default.log 2>&1
