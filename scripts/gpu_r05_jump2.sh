#!/bin/bash
# Grid-wide jump phases: the write-path tests, then C3 with the new finisher against
# STAGE_WP_FINISH=jump1 (the per-group kernel) in the same call, then a C3 kernel trace
set -e
out=gpurun_out/jump2
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_write_path.py tests/test_gpu_bench_legs.py > $out/tests.log 2>&1
for m in new jump1 new jump1; do
  echo "== $m" >> $out/c3.log
  if [ $m = new ]; then
    timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline >> $out/c3.log 2>&1
  else
    STAGE_WP_FINISH=jump1 timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline >> $out/c3.log 2>&1
  fi
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o c3 -- python3 -u bench.py --config c3 --no-cpu-baseline --steps 5 --warmup 1 > $out/trace.log 2>&1
