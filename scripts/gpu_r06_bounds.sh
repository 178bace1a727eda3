set -e
out=gpurun_out/r06bounds
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -k "write" tests > $out/tests.log 2>&1
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-e2e --config c3 > $out/c3_$r.log 2>&1
done
