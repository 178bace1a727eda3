#!/bin/bash
# Round-6 C3 iteration: the write-path tests, C3 alone and its kernel trace.
set -e
out=gpurun_out/r06c3
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_write_path.py tests/test_gpu_bench_legs.py tests/test_gpu_incremental.py > $out/tests.log 2>&1
B="python3 -u bench.py --no-cpu-baseline --no-e2e"
timeout -k 10 200 $B --config c3 > $out/c3.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c3_trace -o c3 -- $B --config c3 --steps 5 --warmup 1 > $out/c3_trace.log 2>&1
