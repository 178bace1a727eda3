#!/bin/bash
# Round-6: which guest workgroups get dispatched beside a CU-filling HBM-bound kernel
# (stage-indexorganized_amd/tools/dispatch_probe.hip, built in-tree).
set -e
out=gpurun_out/r06dispatch
mkdir -p $out
timeout -k 10 120 stage-indexorganized_amd/lib/dispatch_probe > $out/dispatch.log 2>&1
