#!/bin/bash
# CH-Q2 chain folding (round 6): the REGION / NATION scans in one launch, q2_sel_start over a
# visit-major count layout, the per-supplier last-stock and item revisits inside q2_reduce /
# q2_finish, the stock probe's miss pass folded into the probe, and async batches' records
# emitted from a side stream.  The -m gpu suite, then the bench A/B against the library built
# before the change (libstage_hip_base.so), interleaved, then kernel traces.
set -e
out=gpurun_out/r06q2fold4
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $out/tests.log 2>&1
base=$PWD/stage-indexorganized_amd/lib/libstage_hip_base.so
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --config chq2 --steps 300 --no-cpu-baseline > $out/chq2_new_$r.log 2>&1
  STAGE_LIB=$base timeout -k 10 200 python -u bench.py --config chq2 --steps 300 --no-cpu-baseline > $out/chq2_base_$r.log 2>&1
done
timeout -k 10 200 python -u bench.py --config tpcc --no-cpu-baseline > $out/tpcc_new.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_graph -o q2 -- python3 -u bench.py --no-cpu-baseline --no-e2e --config chq2 --steps 20 --warmup 2 > $out/trace_graph.log 2>&1
