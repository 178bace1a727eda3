# direct reply with the world-size rule (own requests merged from 4 ranks on): the sharded-path
# tests, the W = 8 loopback, and the 2-rank rehearsal against the side-stream form
set -e
out=gpurun_out/r06direct3
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_dist.py tests/test_gpu_dist_full_size.py tests/test_gpu_rccl_ranks.py tests/test_gpu_rccl_full_size.py --durations=5 > $out/tests.log 2>&1
BATCH=16777216 STEPS=5 MODES=direct_reply timeout -k 10 300 python -u scripts/loopback_w8.py > $out/loopback_w8_2p24.log 2>&1
base=$PWD/stage-indexorganized_amd/lib/libstage_hip_base.so
B="python -u bench.py --gpus 2 --rows 20000000 --steps 5 --warmup 2 --no-cpu-baseline --reply direct"
for r in 1 2; do
  STAGE_RANKS_SHARE_GPU=1 timeout -k 10 240 $B > $out/g2_new_$r.log 2>&1
  STAGE_LIB=$base STAGE_RANKS_SHARE_GPU=1 timeout -k 10 240 $B > $out/g2_old_$r.log 2>&1
done
