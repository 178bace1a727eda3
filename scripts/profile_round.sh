#!/bin/bash
# Round profile set (kernel traces + PMC passes, each pass its own run; PMC never combined
# with trace domains).  Output: gpurun_out/prof_$TAG/<pass>/...  Usage: scripts/profile_round.sh TAG
set -o pipefail
TAG=${1:-v3}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
run() {  # name limit cmd...
  local name=$1 limit=$2; shift 2
  echo "=== $name"
  timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping"; exit $rc; fi
  return 0
}
run c2_trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c2_trace -o c2 -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline
run c2_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/c2_fetch -o c2 -- python scripts/profile_probe.py
run c2_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/c2_write -o c2 -- python scripts/profile_probe.py
run c4_trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4_trace -o c4 -- python bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline
run c4_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/c4_fetch -o c4 -- python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline
run c4_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/c4_write -o c4 -- python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline
run tpcc_trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tpcc_trace -o tpcc -- python bench.py --config tpcc --steps 5 --warmup 1 --no-cpu-baseline
find $OUT -name "*.csv" | sort
