set -e
out=gpurun_out/r06c3ab16b
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
base=$PWD/stage-indexorganized_amd/lib/libstage_hip_base.so
B="python3 -u bench.py --no-cpu-baseline --no-e2e --config c3 --steps 16"
for r in 1 2; do
  timeout -k 10 300 $B > $out/c3_new_$r.log 2>&1
  STAGE_LIB=$base timeout -k 10 300 $B > $out/c3_base_$r.log 2>&1
done
STAGE_WP_TRACE=1 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-e2e --config c3 --steps 16 > $out/c3_wptrace.log 2>&1
