#!/bin/bash
# CH-Q2 async records: emitted by a kernel on the side stream vs a 2-D DMA copy (STAGE_Q2_EMIT=dma)
set -e
out=gpurun_out/r06q2emit
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_chq2.py > $out/tests_kernel.log 2>&1
STAGE_Q2_EMIT=dma timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_chq2.py > $out/tests_dma.log 2>&1
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --config chq2 --steps 300 --no-cpu-baseline > $out/chq2_kernel_$r.log 2>&1
  STAGE_Q2_EMIT=dma timeout -k 10 200 python -u bench.py --config chq2 --steps 300 --no-cpu-baseline > $out/chq2_dma_$r.log 2>&1
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_kernel -o q2 -- python3 -u bench.py --no-cpu-baseline --no-e2e --config chq2 --steps 20 --warmup 2 > $out/trace_kernel.log 2>&1
STAGE_Q2_EMIT=dma timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $out/trace_dma -o q2 -- python3 -u bench.py --no-cpu-baseline --no-e2e --config chq2 --steps 20 --warmup 2 > $out/trace_dma.log 2>&1
