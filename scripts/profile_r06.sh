#!/bin/bash
# Round-6 profile set on one box, from one tree: kernel traces (C2, C4, C3, CH-Q2) and the PMC
# passes the bench line's `traffic` fields come from -- C2 probe FETCH_SIZE / WRITE_SIZE ->
# pmc_probe.json, C4 scan -> pmc_scan.json, C3 read probe on the reference update stream ->
# pmc_probe_c3.json -- each pass its own run, PMC never combined with trace domains.
# Output: gpurun_out/prof_r06/<pass>/...
# Usage: TREE=<git head> scripts/profile_r06.sh [pass ...]   (no pass names: all of them)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_r06
mkdir -p $OUT
PASSES="$*"
want() { [ -z "$PASSES" ] && return 0; for p in $PASSES; do [ "$p" = "$1" ] && return 0; done; return 1; }
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  want "$name" || return 0
  echo "=== $name"
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 3 $OUT/$name.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
B="python3 -u bench.py --no-cpu-baseline --no-e2e"
run c2_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c2_trace -o c2 -- $B --steps 5 --warmup 1 --no-extras
run c2_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/c2_fetch -o c2 -- python3 scripts/profile_probe.py
run c2_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/c2_write -o c2 -- python3 scripts/profile_probe.py
run c4_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4_trace -o c4 -- $B --config c4 --steps 5 --warmup 1
run c4_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/c4_fetch -o c4 -- python3 scripts/profile_scan.py
run c4_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/c4_write -o c4 -- python3 scripts/profile_scan.py
run c3_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3_trace -o c3 -- $B --config c3 --steps 5 --warmup 1
run c3_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/c3_fetch -o c3 -- python3 scripts/profile_c3.py
run c3_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/c3_write -o c3 -- python3 scripts/profile_c3.py
run q2_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/q2_trace -o q2 -- $B --config chq2 --steps 3 --warmup 1
stamp() {  # file trace: add where / what the counters came from
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
# C2: the probe's heap rows as 1024-B wide reads (as round 4), the rest counted once
if [ -f $OUT/c2_fetch/c2_counter_collection.csv ] && [ -f $OUT/c2_write/c2_counter_collection.csv ]; then
  python3 scripts/pmc_summary.py $OUT/c2_fetch/c2_counter_collection.csv $OUT/c2_write/c2_counter_collection.csv \
    probe_kernel 16777216 100000000 $OUT/pmc_probe.json 0 1024 > $OUT/pmc_summary_c2.log 2>&1 &&
    stamp $OUT/pmc_probe.json "prof_r06/c2_trace (same call)"
fi
# C4: 100 heap rows of 1024 B + the key columns of about 3 leaves per scan counted wide
if [ -f $OUT/c4_fetch/c4_counter_collection.csv ] && [ -f $OUT/c4_write/c4_counter_collection.csv ]; then
  python3 scripts/pmc_summary.py $OUT/c4_fetch/c4_counter_collection.csv $OUT/c4_write/c4_counter_collection.csv \
    scan_kernel 262144 100000000 $OUT/pmc_scan.json 0 103936 > $OUT/pmc_summary_c4.log 2>&1 &&
    stamp $OUT/pmc_scan.json "prof_r06/c4_trace (same call)"
fi
# C3: the last 3 read-probe launches of the last epoch (scripts/profile_c3.py)
if [ -f $OUT/c3_fetch/c3_counter_collection.csv ] && [ -f $OUT/c3_write/c3_counter_collection.csv ]; then
  U=$(grep -o "launches of [0-9]* reads" $OUT/c3_fetch.log | grep -o "[0-9]*" | tail -1)
  python3 scripts/pmc_summary.py $OUT/c3_fetch/c3_counter_collection.csv $OUT/c3_write/c3_counter_collection.csv \
    probe_kernel "$U" 100000000 $OUT/pmc_probe_c3.json 3 1024 16777216 > $OUT/pmc_summary_c3.log 2>&1 &&
    stamp $OUT/pmc_probe_c3.json "prof_r06/c3_trace (same call)"
fi
find $OUT -name "*.csv" | sort
