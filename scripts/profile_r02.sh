#!/bin/bash
# Round-2 profile set: kernel traces and PMC passes, each pass its own run under its own time
# limit (PMC never combined with trace domains; at most 8 SQ / 4 TCC / 2 GRBM counters a pass).
# A pass that ends by a signal or its limit (exit >= 124) stops the script.
# Output: gpurun_out/prof_$TAG/<pass>/...   Usage: scripts/profile_r02.sh TAG [PASS...]
set -o pipefail
TAG=${1:-r02}
shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
WANT=" $* "
run() {  # name limit cmd...
  local name=$1 limit=$2; shift 2
  if [ "$WANT" != "  " ] && [[ "$WANT" != *" $name "* ]]; then return 0; fi
  echo "=== $name"
  timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 3 $OUT/$name.log
  if [ $rc -ge 124 ]; then echo "stopping"; exit $rc; fi
  return 0
}
CAL=stage-indexorganized_amd/lib/fetch_calib
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
INSTS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"
run calib_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/calib_fetch -o calib -- $CAL 32 2
run calib_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/calib_write -o calib -- $CAL 32 2
run c2_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c2_trace -o c2 -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras
run c2_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/c2_fetch -o c2 -- python scripts/profile_probe.py
run c2_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/c2_write -o c2 -- python scripts/profile_probe.py
run c3_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3_trace -o c3 -- python bench.py --config c3 --steps 3 --no-cpu-baseline
run c3_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/c3_fetch -o c3 -- python scripts/profile_c3.py
run c3_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/c3_write -o c3 -- python scripts/profile_c3.py
run c4_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4_trace -o c4 -- python bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline
run tpcc_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tpcc_trace -o tpcc -- python bench.py --config tpcc --steps 5 --warmup 1 --no-cpu-baseline
run tpcc_sq 300 rocprofv3 --pmc $SQ --output-format csv -d $OUT/tpcc_sq -o tpcc -- python bench.py --config tpcc --steps 2 --warmup 1 --no-cpu-baseline
run tpcc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/tpcc_fetch -o tpcc -- python bench.py --config tpcc --steps 2 --warmup 1 --no-cpu-baseline
run tpcc_insts 300 rocprofv3 --pmc $INSTS --output-format csv -d $OUT/tpcc_insts -o tpcc -- python bench.py --config tpcc --steps 2 --warmup 1 --no-cpu-baseline
run c2_sq 300 rocprofv3 --pmc $SQ --output-format csv -d $OUT/c2_sq -o c2 -- python scripts/profile_probe.py
find $OUT -name "*.csv" | sort
