#!/bin/bash
# Round-6 check: the -m gpu suite, smoke, the default bench line (end-to-end leg, threaded C3 CPU
# leg, tile-pass write path), then CH-Q2 and stock-level with the cooperative descent against
# the library built without it (STAGE_LIB=libstage_hip_base.so, when present).
set -e
out=gpurun_out/r06check
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests --durations=20 > $out/tests.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 480 python -u bench.py > $out/bench_default.log 2>&1
timeout -k 10 200 python -u bench.py --config chq2 --steps 300 --no-cpu-baseline > $out/chq2_coop.log 2>&1
timeout -k 10 200 python -u bench.py --config tpcc --no-cpu-baseline > $out/tpcc_coop.log 2>&1
if [ -f stage-indexorganized_amd/lib/libstage_hip_base.so ]; then
  STAGE_LIB=$PWD/stage-indexorganized_amd/lib/libstage_hip_base.so timeout -k 10 200 python -u bench.py --config chq2 --steps 300 --no-cpu-baseline > $out/chq2_base.log 2>&1
  STAGE_LIB=$PWD/stage-indexorganized_amd/lib/libstage_hip_base.so timeout -k 10 200 python -u bench.py --config tpcc --no-cpu-baseline > $out/tpcc_base.log 2>&1
fi
