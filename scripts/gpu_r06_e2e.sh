#!/bin/bash
# Round-6: the host-buffer probe tests and the default bench line (with its end-to-end leg).
set -e
out=gpurun_out/r06e2e
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_host_io.py > $out/tests.log 2>&1
timeout -k 10 480 python -u bench.py > $out/bench_default.log 2>&1
