#!/bin/bash
# the write-path tests under the A/B finishing modes (STAGE_WP_FINISH=walk / jump1)
set -e
out=gpurun_out/wpmodes
mkdir -p $out
for m in walk jump1; do
  STAGE_WP_FINISH=$m timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_write_path.py > $out/tests_$m.log 2>&1
done
