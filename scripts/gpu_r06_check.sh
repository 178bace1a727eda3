#!/bin/bash
# Round-6 check after the variant retirement: the -m gpu suite, smoke and the default bench line
# (with the end-to-end leg and the threaded C3 CPU leg).
set -e
out=gpurun_out/r06check
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests --durations=20 > $out/tests.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 480 python -u bench.py > $out/bench_default.log 2>&1
