# A/B of the 2-rank shared-GPU rehearsal, direct reply: own requests in the chunk's launch
# (libstage_hip.so) vs on a side stream (libstage_hip_base.so), alternating
set -e
out=gpurun_out/r06g2ab
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
base=$PWD/stage-indexorganized_amd/lib/libstage_hip_base.so
B="python -u bench.py --gpus 2 --rows 20000000 --steps 5 --warmup 2 --no-cpu-baseline --reply direct"
for r in 1 2; do
  STAGE_RANKS_SHARE_GPU=1 timeout -k 10 240 $B > $out/new_$r.log 2>&1
  STAGE_LIB=$base STAGE_RANKS_SHARE_GPU=1 timeout -k 10 240 $B > $out/old_$r.log 2>&1
done
