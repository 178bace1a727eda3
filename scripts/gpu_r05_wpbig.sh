#!/bin/bash
# C3: the big-group threshold (STAGE_WP_BIG: ops from a group's first failure on that send it to
# the grid-wide jump kernels instead of wp_finish_groups), a kernel trace per setting
set -e
out=gpurun_out/wpbig
mkdir -p $out
export TMPDIR=/tmp
for b in 256 64 32 128; do
  STAGE_WP_BIG=$b timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/t$b -o c3 -- python3 -u bench.py --config c3 --no-cpu-baseline --steps 6 --warmup 1 > $out/b$b.log 2>&1
done
