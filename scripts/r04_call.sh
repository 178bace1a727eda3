#!/bin/bash
# Round-4 GPU call: the new and changed tests, the full -m gpu suite, then the bench lines
# (default; world-1 sharded rehearsal with the coalescing sort at 8 / 10 / 11 radix bits;
# CH-Q2; stock-level with the default, 6-wave split and probe-first scan kernels).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_steps.sh \
  "300 new_tests python -u -m pytest tests/test_gpu_txn_facts.py tests/test_txn_parity.py tests/test_gpu_adapter.py tests/test_gpu_bench_legs.py tests/test_gpu_chq2.py tests/test_gpu_dist.py tests/test_gpu_tpcc.py -m gpu -v --timeout 240 --timeout-method thread" \
  "420 gpu_tests python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_dist_full_size.py --deselect tests/test_gpu_txn_facts.py --deselect tests/test_txn_parity.py --deselect tests/test_gpu_adapter.py --deselect tests/test_gpu_bench_legs.py --deselect tests/test_gpu_chq2.py --deselect tests/test_gpu_dist.py --deselect tests/test_gpu_tpcc.py" \
  "200 bench python -u bench.py" \
  "120 fs8 python -u bench.py --force-sharded --no-cpu-baseline --steps 10" \
  "120 fs10 env STAGE_DD_RADIX_BITS=10 python -u bench.py --force-sharded --no-cpu-baseline --steps 10" \
  "120 fs11 env STAGE_DD_RADIX_BITS=11 python -u bench.py --force-sharded --no-cpu-baseline --steps 10" \
  "150 chq2 python -u bench.py --config chq2" \
  "100 tpcc0 python -u bench.py --config tpcc --no-cpu-baseline" \
  "100 tpcc11 env STAGE_SL_SCANS=-11 python -u bench.py --config tpcc --no-cpu-baseline" \
  "120 chq2s env STAGE_Q2_SORT=1 python -u bench.py --config chq2 --no-cpu-baseline" \
  "100 tpcc10 env STAGE_SL_SCANS=-10 python -u bench.py --config tpcc --no-cpu-baseline"
