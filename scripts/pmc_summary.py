"""Turns rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes for one kernel.

Calibration (profiles/r02/fetch_calibration.json, tools/fetch_calib.hip on gfx950): FETCH_SIZE
reports 1/2 of the bytes of 128-B-line reads (wide coalesced streams, random 128-B lines,
random 1024-B rows) and the exact bytes of random 64-B sectors; a random 32-B read is tallied
as one 64-B request (what the memory moves).  WRITE_SIZE is exact for 16-B-per-lane stores,
streaming or random 32-B records.  So

    read bytes = 2 x wide + 1 x (FETCH - wide),   wide = min(FETCH, WIDE_PER_UNIT x units / 2)

where WIDE_PER_UNIT is the bytes a unit reads in whole 128-B lines (a probe's 1024-B heap row;
attributed first, so the estimate is an upper one), and the r01 rule (2 x FETCH for
everything) is reported beside it as `read_bytes_uncalibrated`.  Counters are in KiB.
usage: python scripts/pmc_summary.py FETCH.csv WRITE.csv KERNEL_SUBSTR UNITS ROWS OUT.json
       [LAST] [WIDE_PER_UNIT] [BATCH]
  LAST: average only the kernel's last LAST dispatches (the read probes of
  scripts/profile_c3.py, after the write path's locate probes); BATCH: the bench batch the
  file is matched on (default UNITS)
"""
import csv
import json
import sys


def per_launch(path, counter, kernel, last=0):
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0)))
    vals = [float(r["Counter_Value"]) for r in rows][-last if last else 0:]
    return sum(vals) / len(vals), len(vals)


def main():
    fpath, wpath, kernel, units, rows, out = sys.argv[1:7]
    last = int(sys.argv[7]) if len(sys.argv) > 7 else 0
    wide_per_unit = float(sys.argv[8]) if len(sys.argv) > 8 else 0.0
    batch = int(sys.argv[9]) if len(sys.argv) > 9 else int(units)
    units = int(units)
    fetch, nf = per_launch(fpath, "FETCH_SIZE", kernel, last)
    write, nw = per_launch(wpath, "WRITE_SIZE", kernel, last)
    fb = fetch * 1024
    wide = min(fb, wide_per_unit * units / 2) if wide_per_unit else fb
    read_b = 2 * wide + (fb - wide)
    write_b = write * 1024
    d = {"kernel": kernel, "batch": batch, "units_per_launch": units, "rows": int(rows), "launches": [nf, nw],
         "fetch_size_kib": fetch, "write_size_kib": write, "read_bytes_calibrated": read_b,
         "read_bytes_uncalibrated": 2 * fb, "write_bytes": write_b, "hbm_bytes_per_launch": read_b + write_b,
         "bytes_per_unit": (read_b + write_b) / units,
         "bytes_per_unit_uncalibrated": (2 * fb + write_b) / units,
         "correction": f"read = 2 x wide + 1 x rest of FETCH_SIZE, wide = min(FETCH, {wide_per_unit} B x units / 2) "
                       "(profiles/r02/fetch_calibration.json); write = WRITE_SIZE; KiB -> bytes"}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
