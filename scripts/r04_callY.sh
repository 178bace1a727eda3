#!/bin/bash
# Round-4 call: write-path tests, the C3 leg with the write-path trace, the C5 data path at size
# on one GPU (8 x 12.5M-row shards vs one 100M-row table), and the remaining counter passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_steps.sh \
  "300 wp_tests python -u -m pytest tests/test_gpu_write_path.py tests/test_gpu_bench_legs.py -m gpu -v --timeout 240 --timeout-method thread" \
  "200 c3 env STAGE_WP_TRACE=1 python -u bench.py --config c3 --no-cpu-baseline --steps 8" \
  "700 c5_full python -u -m pytest tests/test_gpu_dist_full_size.py -m gpu -v -s --timeout 680 --timeout-method thread" || exit $?
TREE=${TREE:-unknown} bash scripts/profile_r04.sh q2_sq q2_fetch sl_fetch
