#!/bin/bash
# probe_lane_kernel with the separator tree's top levels in LDS: the wide-key parity tests, then
# CH-Q2 and stock-level with STAGE_LANE_LDS=1 / 0 alternating, then a CH-Q2 kernel trace
set -e
out=gpurun_out/lanelds
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chq2.py tests/test_gpu_tpcc.py tests/test_gpu_wide_keys.py > $out/tests.log 2>&1
for v in 1 0 1 0; do
  echo "== lds $v" >> $out/bench.log
  STAGE_LANE_LDS=$v timeout -k 10 200 python -u bench.py --config chq2 --steps 300 --no-cpu-baseline >> $out/bench.log 2>&1
  STAGE_LANE_LDS=$v timeout -k 10 200 python -u bench.py --config tpcc --no-cpu-baseline >> $out/bench.log 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o q2 -- python3 -u bench.py --config chq2 --steps 20 --warmup 2 --no-cpu-baseline > $out/trace.log 2>&1
