"""Counter bytes / true bytes per access width from tools/pmc_calib.bin's two PMC passes.
  python tools/pmc_calib_summary.py FETCH_DIR WRITE_DIR [OUT_JSON]"""
import collections
import csv
import glob
import json
import os
import sys

TRUE_BYTES = 1 << 30


def per_kernel(d, counter):
    disp = collections.defaultdict(float)
    names = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == counter:
                k = (row["Process_Id"], row["Dispatch_Id"])
                disp[k] += float(row["Counter_Value"])
                names[k] = row["Kernel_Name"]
    acc = collections.defaultdict(list)
    for k, v in disp.items():
        acc[names[k]].append(v * 1024.0)  # KiB -> bytes
    return acc


def label(name):
    for key, lab in (("k_write16", "write 16 B/lane"), ("HIP_vector_type<unsigned int, 2u>", "read 8 B/lane"),
                     ("HIP_vector_type<unsigned int, 4u>", "read 16 B/lane"), ("unsigned char", "read 1 B/lane"),
                     ("unsigned int", "read 4 B/lane")):
        if key in name:
            return lab
    return name[:40]


def main():
    fe = per_kernel(sys.argv[1], "FETCH_SIZE")
    wr = per_kernel(sys.argv[2], "WRITE_SIZE")
    res = {}
    for name in sorted(set(fe) | set(wr)):
        if not name.startswith("void k_") and "k_write16" not in name:
            continue
        lab = label(name)
        f = fe.get(name, [0.0])
        w = wr.get(name, [0.0])
        if lab == "read 8 B/lane":  # dispatches 1-2: 1 GiB streams; 3-5: the cache-resident 128 MiB table
            res["read 8 B/lane, 128 MiB table, 3rd pass"] = {"fetch_over_true": f[-1] / (TRUE_BYTES / 8)}
            print(f"{'8 B/lane, resident 128 MiB':26s} FETCH/true {f[-1] / (TRUE_BYTES / 8):6.3f}")
            f = f[:2]
        res[lab] = {"fetch_over_true": f[-1] / TRUE_BYTES, "write_over_true": w[-1] / TRUE_BYTES,
                    "dispatches": len(f)}
        print(f"{lab:26s} FETCH/true {f[-1] / TRUE_BYTES:6.3f}  WRITE/true {w[-1] / TRUE_BYTES:6.3f}")
    if len(sys.argv) > 3:
        json.dump(res, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
