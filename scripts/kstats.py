"""Prints a rocprofv3 kernel_stats.csv compactly: short name, calls, average and total time."""
import csv
import re
import sys

for path in sys.argv[1:]:
    print(path)
    for r in csv.DictReader(open(path)):
        n = r["Name"].replace("stage::(anonymous namespace)::", "").replace("void ", "")
        n = re.sub(r"rocprim::ROCPRIM_\w+::detail::", "rocprim::", n)
        short = n.split("(")[0] if not n.startswith("rocprim") else n[:90]
        print(f"  {short[:90]:90s} {int(r['Calls']):5d} avg {float(r['AverageNs']) / 1e3:9.1f} us"
              f"  total {float(r['TotalDurationNs']) / 1e6:8.2f} ms")
