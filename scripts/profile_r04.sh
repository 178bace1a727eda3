#!/bin/bash
# Round-4 profile set on one box, from one tree: kernel traces (C2, C3, the world-1 sharded step,
# CH-Q2, TPC-C stock-level) and PMC passes (C2 probe FETCH_SIZE / WRITE_SIZE -> pmc_probe.json;
# C3 read probe FETCH_SIZE / WRITE_SIZE on the reference update stream -> pmc_probe_c3.json;
# CH-Q2 and stock-level SQ + FETCH_SIZE), each pass its own run, PMC never combined with trace
# domains.  Output: gpurun_out/prof_r04/<pass>/...
# Usage: TREE=<git head> scripts/profile_r04.sh [pass ...]   (no pass names: all of them)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_r04
mkdir -p $OUT
want() { [ $# -eq 0 ] && return 0; for p in $PASSES; do [ "$p" = "$1" ] && return 0; done; return 1; }
PASSES="$*"
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  if [ -n "$PASSES" ] && ! want "$name"; then return 0; fi
  echo "=== $name"
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 3 $OUT/$name.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
B="python3 -u bench.py --no-cpu-baseline"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
run c2_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c2_trace -o c2 -- $B --steps 5 --warmup 1 --no-extras
run c2_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/c2_fetch -o c2 -- python3 scripts/profile_probe.py
run c2_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/c2_write -o c2 -- python3 scripts/profile_probe.py
run c3_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3_trace -o c3 -- $B --config c3 --steps 5 --warmup 1
run c3_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/c3_fetch -o c3 -- python3 scripts/profile_c3.py
run c3_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/c3_write -o c3 -- python3 scripts/profile_c3.py
run fs_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/fs_trace -o fs -- $B --force-sharded --steps 5 --warmup 1
run q2_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/q2_trace -o q2 -- $B --config chq2 --steps 3 --warmup 1
run q2_sq 300 rocprofv3 --pmc $SQ --output-format csv -d $OUT/q2_sq -o q2 -- $B --config chq2 --steps 3 --warmup 1
run q2_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/q2_fetch -o q2 -- $B --config chq2 --steps 3 --warmup 1
export STAGE_Q2_SORT=1
run q2s_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/q2s_trace -o q2s -- $B --config chq2 --steps 3 --warmup 1
unset STAGE_Q2_SORT
run sl_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/sl_trace -o sl -- $B --config tpcc --steps 5 --warmup 1
run sl_sq 300 rocprofv3 --pmc $SQ --output-format csv -d $OUT/sl_sq -o sl -- $B --config tpcc --steps 3 --warmup 1
run sl_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/sl_fetch -o sl -- $B --config tpcc --steps 3 --warmup 1
stamp() {  # file: add where / what the counters came from
  python3 - "$1" "${TREE:-unknown}" "$2" <<'PY'
import json, socket, subprocess, sys, time
path, tree, trace = sys.argv[1:4]
p = json.load(open(path))
try:
    gpu = subprocess.run(["rocm-smi", "--showproductname"], capture_output=True, text=True, timeout=30).stdout
    gpu = [l.split(":", 2)[-1].strip() for l in gpu.splitlines() if "Card Series" in l or "Card SKU" in l][:2]
except Exception:
    gpu = []
p["profiled"] = {"host": socket.gethostname(), "gpu": gpu, "date": time.strftime("%Y-%m-%d"), "tree": tree,
                 "kernel_trace": trace}
json.dump(p, open(path, "w"), indent=1)
print(json.dumps(p["profiled"]))
PY
}
if [ -f $OUT/c2_fetch/c2_counter_collection.csv ] && [ -f $OUT/c2_write/c2_counter_collection.csv ]; then
  python3 scripts/pmc_summary.py $OUT/c2_fetch/c2_counter_collection.csv $OUT/c2_write/c2_counter_collection.csv \
    probe_kernel 16777216 100000000 $OUT/pmc_probe.json 0 1024 > $OUT/pmc_summary.log 2>&1 &&
    stamp $OUT/pmc_probe.json "prof_r04/c2_trace (same call)"
fi
if [ -f $OUT/c3_fetch/c3_counter_collection.csv ] && [ -f $OUT/c3_write/c3_counter_collection.csv ]; then
  U=$(grep -o "launches of [0-9]* reads" $OUT/c3_fetch.log | grep -o "[0-9]*" | tail -1)
  python3 scripts/pmc_summary.py $OUT/c3_fetch/c3_counter_collection.csv $OUT/c3_write/c3_counter_collection.csv \
    probe_kernel "$U" 100000000 $OUT/pmc_probe_c3.json 3 1024 16777216 >> $OUT/pmc_summary.log 2>&1 &&
    stamp $OUT/pmc_probe_c3.json "prof_r04/c3_trace (same call)"
fi
find $OUT -name "*.csv" | sort
