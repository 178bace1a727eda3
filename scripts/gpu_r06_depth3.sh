# three write-path epochs in flight: the write-path / CH-Q2 / for-update tests, C3 twice, its
# write-path trace, and the default line (its nested C3 leg)
set -e
out=gpurun_out/r06depth3
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -k "write or chq2 or epoch or for_update or bench_legs" tests > $out/tests.log 2>&1
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-e2e --config c3 > $out/c3_$r.log 2>&1
done
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-e2e --config c3 --steps 16 > $out/c3_16.log 2>&1
STAGE_WP_TRACE=1 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-e2e --config c3 --steps 16 > $out/c3_wptrace.log 2>&1
