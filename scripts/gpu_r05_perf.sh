#!/bin/bash
# Round-5 measurement call (one GPU box), after scripts/gpu_r05_validate.sh passed: the default
# bench line, C3 with every read at the newest id beside the default read-id model,
# and the CH-Q2 kernel trace of this tree.  Each step has its own time limit; the first failure
# ends the script.
set -e
out=gpurun_out/perf
mkdir -p $out
timeout -k 10 420 python -u bench.py > $out/bench_default.log 2>&1
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > $out/c3_default.log 2>&1
timeout -k 10 300 python -u bench.py --config c3 --old-share 0 --no-cpu-baseline > $out/c3_newest.log 2>&1
bash scripts/profile_r05.sh q2_trace > $out/prof.log 2>&1
