#!/bin/bash
# C3 with the write path's 64-bit-key sort built scratch-free (radix_sort.hpp): the write-path
# tests, then C3 A/B against the library before the change (libstage_hip_base.so), interleaved,
# then a kernel trace (does the sort now run beside the read probe?).
set -e
out=gpurun_out/r06c3sort
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_write_path.py tests/test_gpu_bench_legs.py tests/test_gpu_incremental.py > $out/tests.log 2>&1
base=$PWD/stage-indexorganized_amd/lib/libstage_hip_base.so
B="python3 -u bench.py --no-cpu-baseline --no-e2e --config c3"
for r in 1 2; do
  timeout -k 10 200 $B > $out/c3_new_$r.log 2>&1
  STAGE_LIB=$base timeout -k 10 200 $B > $out/c3_base_$r.log 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c3_trace -o c3 -- $B --steps 5 --warmup 1 > $out/c3_trace.log 2>&1
