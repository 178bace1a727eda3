#!/bin/bash
# C3: the read probe's grid cap (STAGE_PROBE_MAX_BLOCKS) against the write chain's overlap --
# shorter-lived probe workgroups free CUs for the high-priority write stream more often
set -e
out=gpurun_out/c3blocks
mkdir -p $out
for mb in 0 65536 0 65536 4096; do
  echo "== max_blocks $mb" >> $out/c3.log
  STAGE_PROBE_MAX_BLOCKS=$mb timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline >> $out/c3.log 2>&1
done
