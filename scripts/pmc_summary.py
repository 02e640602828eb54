"""Per-kernel averages of rocprofv3 --pmc counter_collection.csv files
(counters summed over the dispatch's instances, averaged over dispatches).
usage: pmc_summary.py <csv>... [--kernel substr]"""
import csv
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
ksub = None
if "--kernel" in sys.argv:
    ksub = sys.argv[sys.argv.index("--kernel") + 1]
    args = [a for a in args if a != ksub]
acc = defaultdict(lambda: defaultdict(dict))  # kernel -> counter -> dispatch -> value
for path in args:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0]
        if ksub and ksub not in k:
            continue
        d = acc[k][r["Counter_Name"]]
        d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
for k in sorted(acc):
    print(f"== {k}")
    for c in sorted(acc[k]):
        v = acc[k][c]
        print(f"  {c:24s} {sum(v.values()) / len(v):16.4g}  (dispatches {len(v)})")
