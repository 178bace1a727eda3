#!/bin/bash
# CH-Q2 two batches in flight: hipGraph replay (default) against plain enqueue (STAGE_Q2_GRAPH=0)
set -e
out=gpurun_out/q2graph
mkdir -p $out
for g in 1 0 1 0; do
  echo "== graph $g" >> $out/bench.log
  STAGE_Q2_GRAPH=$g timeout -k 10 200 python -u bench.py --config chq2 --steps 300 --no-cpu-baseline >> $out/bench.log 2>&1
done
