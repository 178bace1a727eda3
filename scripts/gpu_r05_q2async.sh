#!/bin/bash
# CH-Q2: the CH-Q2 GPU tests, the chq2 bench (one / two batches in flight), a kernel trace
set -e
out=gpurun_out/q2async
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_chq2.py tests/test_gpu_tpcc.py > $out/tests.log 2>&1
for a in 0 1 0 1; do
  timeout -k 10 200 python -u bench.py --config chq2 --steps 300 --no-cpu-baseline --q2-async $a >> $out/bench.log 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o q2 -- python3 -u bench.py --config chq2 --steps 20 --warmup 2 --no-cpu-baseline > $out/trace.log 2>&1
