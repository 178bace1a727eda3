#!/bin/bash
# Round-4 closing GPU call: the whole -m gpu suite, smoke, the default bench line, the CH-Q2 and
# stock-level lines, and the CH-Q2 kernel trace on the final tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_steps.sh \
  "600 gpu_tests python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "120 smoke python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "240 bench python -u bench.py" \
  "150 chq2 python -u bench.py --config chq2 --steps 300" \
  "120 tpcc0 python -u bench.py --config tpcc --no-cpu-baseline" \
  "200 q2prof bash scripts/profile_r04.sh q2_trace"
