#!/bin/bash
# Stock-level scan kernels, round 3: kernel trace + counter passes (one rocprofv3 --pmc pass per
# counter group, each its own short run) for the default (scan_first_mono_kernel) and
# STAGE_SL_SCANS=-8 (scan_first_split_kernel).  Output: gpurun_out/prof_tpcc_r03/<variant>_<pass>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_tpcc_r03
mkdir -p $OUT
B="python3 -u bench.py --config tpcc --no-cpu-baseline --steps 3 --warmup 1"
run() {  # name limit args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
for V in 0 -8; do
  export STAGE_SL_SCANS=$V
  run v${V}_sq 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $OUT/v${V}_sq -o p -- $B
  run v${V}_fetch 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/v${V}_fetch -o p -- $B
  run v${V}_tcc 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_LDS --output-format csv -d $OUT/v${V}_tcc -o p -- $B
done
