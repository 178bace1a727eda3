#!/bin/bash
# wp_jump_chain's phase-B timing (STAGE_WP_CHAIN_DEBUG: the hottest group's first fill, walk and
# span totals from wall_clock64, printed per epoch).  The instrumentation was a temporary
# build (wp_finish_jump follow-up); on later trees this only runs C3.
set -e
out=gpurun_out/chaindbg
mkdir -p $out
STAGE_WP_CHAIN_DEBUG=1 timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline --steps 4 --warmup 1 > $out/c3.log 2>&1
