#!/bin/bash
# Round-4 call: the write-path tests on the success-heavy stream, the C3 leg with the write-path
# trace, then the profile set's trace and counter passes (scripts/profile_r04.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_steps.sh \
  "300 wp_tests python -u -m pytest tests/test_gpu_write_path.py tests/test_gpu_bench_legs.py tests/test_gpu_incremental.py tests/test_gpu_txn_facts.py -m gpu -v --timeout 240 --timeout-method thread" \
  "200 c3 env STAGE_WP_TRACE=1 python -u bench.py --config c3 --no-cpu-baseline --steps 8" || exit $?
TREE=${TREE:-unknown} bash scripts/profile_r04.sh c2_trace c2_fetch c2_write c3_trace c3_fetch c3_write fs_trace q2_trace q2s_trace sl_trace sl_sq
