"""Per-kernel average of every PMC counter in rocprofv3 counter_collection CSVs (dispatch-summed over
XCD/SE instances first).  python tools/pmc_summary.py <dir> [<dir> ...]"""
import collections
import csv
import glob
import sys

per = collections.defaultdict(float)
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/run_counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            per[(row["Kernel_Name"].split("(")[0][:40], row["Counter_Name"], row["Dispatch_Id"])] += float(row["Counter_Value"])
acc = collections.defaultdict(list)
for (k, c, _), v in per.items():
    acc[(k, c)].append(v)
kernels = sorted({k for k, _ in acc})
for k in kernels:
    print(k)
    for (kk, c), v in sorted(acc.items()):
        if kk == k:
            print(f"    {c:24s} {sum(v) / len(v):16.1f}  (n={len(v)})")
