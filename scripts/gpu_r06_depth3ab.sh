# A/B on one box: write-path pipeline depth 3 (libstage_hip.so) vs depth 2 (libstage_hip_base.so),
# 16-epoch C3, alternating
set -e
out=gpurun_out/r06depth3ab
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
base=$PWD/stage-indexorganized_amd/lib/libstage_hip_base.so
B="python3 -u bench.py --no-cpu-baseline --no-e2e --config c3 --steps 16"
for r in 1 2 3; do
  timeout -k 10 300 $B > $out/c3_d3_$r.log 2>&1
  STAGE_LIB=$base timeout -k 10 300 $B > $out/c3_d2_$r.log 2>&1
done
