#!/bin/bash
# Single-key reader latency / throughput: the coalescing reader and the resident reader at
# 1 / 16 / 64 caller threads (tools/reader_drive.cpp), 20M rows, Zipf 0.9.  Each run has its
# own time limit; a run that ends by a signal or its limit stops the script.
# Output: gpurun_out/reader/<name>.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/reader
mkdir -p $OUT
BIN=stage-indexorganized_amd/lib/reader_drive
run() {  # name args...
  local name=$1; shift
  timeout -k 10 120 $BIN "$@" > $OUT/$name.json 2> $OUT/$name.err
  local rc=$?
  echo "$name rc=$rc $(cat $OUT/$name.json)"
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
W=${WAVES:-16}
for T in ${THREADS:-1 16 64}; do
  [ -n "$SKIP_COALESCING" ] || run coalescing_t$T 20000000 3 $T 1024 100 1048576 0.9 0
  run resident_w${W}_t$T${TAG} 20000000 3 $T 1024 100 1048576 0.9 $W
done
