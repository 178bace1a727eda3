#!/bin/bash
# Round-6 A/B on one box: C4 and C2 with the current library against libstage_hip_base.so (the
# library without the heap_chunk bound), CH-Q2 with the LDS-staged q2_finish, and a kernel trace
# of C3 (the tile-pass write path beside the read probe).
set -e
out=gpurun_out/r06ab
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
BASE=$PWD/stage-indexorganized_amd/lib/libstage_hip_base.so
B="python3 -u bench.py --no-cpu-baseline --no-e2e"
timeout -k 10 200 $B --config c4 --steps 10 > $out/c4_cur.log 2>&1
STAGE_LIB=$BASE timeout -k 10 200 $B --config c4 --steps 10 > $out/c4_base.log 2>&1
timeout -k 10 200 $B --config c4 --steps 10 > $out/c4_cur2.log 2>&1
timeout -k 10 200 python -u bench.py --config chq2 --steps 300 --no-cpu-baseline > $out/chq2_cur.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c3_trace -o c3 -- $B --config c3 --steps 5 --warmup 1 > $out/c3_trace.log 2>&1
