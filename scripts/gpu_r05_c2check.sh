#!/bin/bash
# the default bench line twice on one box (box-to-box HBM variance check)
set -e
out=gpurun_out/c2check
mkdir -p $out
for k in 1 2; do
  timeout -k 10 420 python -u bench.py --no-cpu-baseline > $out/bench_$k.log 2>&1
done
