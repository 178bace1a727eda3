#!/bin/bash
# Round-3 profile set on one box, from one tree: kernel traces (C2, C3, the world-1 sharded step,
# CH-Q2) and PMC passes (C2 probe FETCH_SIZE / WRITE_SIZE -> pmc_probe.json; CH-Q2 SQ and
# FETCH_SIZE), each pass its own run, PMC never combined with trace domains.
# Output: gpurun_out/prof_r03/<pass>/...   Usage: TREE=<git head> scripts/profile_r03.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_r03
mkdir -p $OUT
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 3 $OUT/$name.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
B="python3 -u bench.py --no-cpu-baseline"
run c2_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c2_trace -o c2 -- $B --steps 5 --warmup 1 --no-extras
run c2_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/c2_fetch -o c2 -- python3 scripts/profile_probe.py
run c2_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/c2_write -o c2 -- python3 scripts/profile_probe.py
run c3_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3_trace -o c3 -- $B --config c3 --steps 5 --warmup 1
run fs_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/fs_trace -o fs -- $B --force-sharded --steps 5 --warmup 1
run q2_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/q2_trace -o q2 -- $B --config chq2 --steps 3 --warmup 1
run q2_sq 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $OUT/q2_sq -o q2 -- $B --config chq2 --steps 3 --warmup 1
run q2_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/q2_fetch -o q2 -- $B --config chq2 --steps 3 --warmup 1
python3 scripts/pmc_summary.py $OUT/c2_fetch/c2_counter_collection.csv $OUT/c2_write/c2_counter_collection.csv \
  probe_kernel 16777216 100000000 $OUT/pmc_probe.json 0 1024 > $OUT/pmc_summary.log 2>&1
python3 - "$OUT" "${TREE:-unknown}" <<'PY'
import json, socket, subprocess, sys, time
out, tree = sys.argv[1], sys.argv[2]
p = json.load(open(f"{out}/pmc_probe.json"))
try:
    gpu = subprocess.run(["rocm-smi", "--showproductname"], capture_output=True, text=True, timeout=30).stdout
    gpu = [l.split(":", 2)[-1].strip() for l in gpu.splitlines() if "Card Series" in l or "Card SKU" in l][:2]
except Exception:
    gpu = []
p["profiled"] = {"host": socket.gethostname(), "gpu": gpu, "date": time.strftime("%Y-%m-%d"), "tree": tree,
                 "kernel_trace": "prof_r03/c2_trace (same call)"}
json.dump(p, open(f"{out}/pmc_probe.json", "w"), indent=1)
print(json.dumps(p["profiled"]))
PY
find $OUT -name "*.csv" | sort
