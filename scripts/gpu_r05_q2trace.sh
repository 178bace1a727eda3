#!/bin/bash
# CH-Q2 host phases per batch (STAGE_Q2_TRACE) and a kernel trace, two batches in flight
set -e
out=gpurun_out/q2trace
mkdir -p $out
export TMPDIR=/tmp
STAGE_Q2_TRACE=1 timeout -k 10 200 python -u bench.py --config chq2 --steps 40 --warmup 4 --no-cpu-baseline > $out/trace.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $out/kt -o q2 -- python3 -u bench.py --config chq2 --steps 40 --warmup 4 --no-cpu-baseline > $out/kt.log 2>&1
