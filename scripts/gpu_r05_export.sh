#!/bin/bash
# C3: the export kernel's grid (STAGE_WP_EXPORT_BLOCKS; it runs beside the next probe)
set -e
out=gpurun_out/export
mkdir -p $out
for b in 32 8 16 64 32 16; do
  echo "== blocks $b" >> $out/c3.log
  STAGE_WP_EXPORT_BLOCKS=$b timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline >> $out/c3.log 2>&1
done
