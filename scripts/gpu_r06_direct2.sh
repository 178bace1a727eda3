#!/bin/bash
# STAGE_REPLY_DIRECT (owners write rows into the callers' outputs): the sharded-path tests
# (loopback W = 2/3/8, the C5 loopback at size, real RCCL ranks sharing one GPU incl. the
# 8-rank C5 run), then the W = 8 loopback HBM side in every reply mode at 2^24 and 2^25.
set -e
out=gpurun_out/r06direct2
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_dist.py tests/test_gpu_dist_full_size.py tests/test_gpu_rccl_ranks.py tests/test_gpu_rccl_full_size.py --durations=10 > $out/tests.log 2>&1
BATCH=16777216 STEPS=5 timeout -k 10 300 python -u scripts/loopback_w8.py > $out/loopback_w8_2p24.log 2>&1
BATCH=33554432 STEPS=5 timeout -k 10 300 python -u scripts/loopback_w8.py > $out/loopback_w8_2p25.log 2>&1
CHUNKS=2 BATCH=16777216 STEPS=5 timeout -k 10 300 python -u scripts/loopback_w8.py > $out/loopback_w8_2p24_c2.log 2>&1
