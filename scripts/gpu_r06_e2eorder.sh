#!/bin/bash
# Does the end-to-end leg (host-buffer probes into 4 GB of pinned memory) slow the C4 / C3 legs
# that follow it in the default run?  The default line without CPU legs, with and without it.
set -e
out=gpurun_out/r06e2eorder
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/with_e2e.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e > $out/without_e2e.log 2>&1
