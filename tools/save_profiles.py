"""Copy a gpu_measure.sh run's summaries from gpurun_out/ into profiles/ (tracked):
kernel stats, bench JSON line, per-kernel PMC averages, and the K1 traffic entry.
  python tools/save_profiles.py r01"""
import collections
import csv
import json
import shutil
import subprocess
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = "gpurun_out"
name = "config3_fp32_huber_pair"
shutil.copy(f"{src}/{tag}_prof_stats/run_kernel_stats.csv", f"profiles/{tag}_kernel_stats_{name}.csv")
line = open(f"{src}/{tag}_bench.json").read().strip().splitlines()[-1]
json.loads(line)
open(f"profiles/{tag}_bench.json", "w").write(line + "\n")
with open(f"profiles/{tag}_pmc_summary_{name}.csv", "w") as out:
    out.write("counter,kernel,dispatches,avg_kib\n")
    for tagp, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        per = collections.defaultdict(float)
        for row in csv.DictReader(open(f"{src}/{tag}_pmc_{tagp}/run_counter_collection.csv")):
            if row["Counter_Name"] == ctr:
                per[(row["Kernel_Name"].split("(")[0], row["Dispatch_Id"])] += float(row["Counter_Value"])
        acc = collections.defaultdict(list)
        for (k, _), v in per.items():
            acc[k].append(v)
        for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
            out.write(f"{ctr},\"{k}\",{len(v)},{sum(v) / len(v):.1f}\n")
shutil.copy(f"{src}/{tag}_k1_traffic.json", "profiles/k1_traffic.json")  # the file the bench line read
shutil.copy(f"{src}/{tag}_pmc_calib.json", f"profiles/{tag}_pmc_calib.json")
print("saved", tag)
