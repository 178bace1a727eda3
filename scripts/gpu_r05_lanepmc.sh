#!/bin/bash
# probe_lane_kernel (CH-Q2's STOCK probe) counters: wave waits vs texture-pipe busy
set -e
out=gpurun_out/lanepmc
mkdir -p $out
export TMPDIR=/tmp
B="python3 -u bench.py --config chq2 --steps 20 --warmup 2 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $out/sq -o q2 -- $B > $out/sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $out/ta -o q2 -- $B > $out/ta.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d $out/tcp -o q2 -- $B > $out/tcp.log 2>&1
