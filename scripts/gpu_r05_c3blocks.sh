#!/bin/bash
# C3: the read probe's grid cap (STAGE_PROBE_MAX_BLOCKS) against the write chain's overlap --
# a capped grid leaves room on every CU for the high-priority write stream's kernels
set -e
out=gpurun_out/c3blocks
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_write_path.py > $out/tests.log 2>&1
for mb in ${BLOCKS:-0 1024 1536 2048 3072 0 1536}; do
  echo "== max_blocks $mb" >> $out/c3.log
  STAGE_PROBE_MAX_BLOCKS=$mb timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline >> $out/c3.log 2>&1
done
