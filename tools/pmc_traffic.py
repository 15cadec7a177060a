"""Per-launch HBM traffic of a kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

FETCH_SIZE / WRITE_SIZE are in KiB (rocprofv3 derived counters).  On gfx950 FETCH_SIZE reports half of
the bytes of wide coalesced streaming reads (MI355X_MICROARCH.md, HBM section), so the read bytes are
2 x FETCH_SIZE; WRITE_SIZE is taken as is.  Writes a JSON entry keyed like bench.py's --traffic-json.
  python tools/pmc_traffic.py FETCH_DIR WRITE_DIR KERNEL_SUBSTR KEY OUT_JSON [MIN_KIB] [GRID_SIZE]
MIN_KIB drops dispatches with less traffic (the device-driven LM's speculative launches that exit at
once: K2 after the solve's last decision); GRID_SIZE keeps only dispatches of that grid (threads): one
problem's launches when the profiled run also solves others (bench.py's config-4 and stream legs).
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter, kernel, grid=0):
    """Summed counter per dispatch of the kernel.  `kernel` is a substring of the kernel name -- name the
    instantiation (e.g. `k_linearize<float, 1>`): the bench also runs the fp64 leg, whose K1 moves 1.8x the
    bytes."""
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = row["Kernel_Name"]
            if row["Counter_Name"] == counter and kernel in name and (not grid or int(row["Grid_Size"]) == grid):
                k = (row["Process_Id"], row["Dispatch_Id"])
                vals[k] = vals.get(k, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    fdir, wdir, kernel, key, out = sys.argv[1:6]
    min_kib = float(sys.argv[6]) if len(sys.argv) > 6 else 0.0
    grid = int(sys.argv[7]) if len(sys.argv) > 7 else 0
    fe = [x for x in per_dispatch(fdir, "FETCH_SIZE", kernel, grid) if x >= min_kib]
    wr = [x for x in per_dispatch(wdir, "WRITE_SIZE", kernel, grid) if x >= min_kib / 64]
    if not fe or not wr:
        raise SystemExit(f"no dispatches of {kernel}: fetch {len(fe)} write {len(wr)}")
    fkib = sum(fe) / len(fe)
    wkib = sum(wr) / len(wr)
    entry = {"kernel": kernel, "grid_size": grid or None, "launches_fetch_pass": len(fe), "launches_write_pass": len(wr),
             "fetch_size_kib_avg": fkib, "write_size_kib_avg": wkib,
             "read_bytes_corrected": 2 * fkib * 1024, "write_bytes": wkib * 1024,
             "hbm_bytes_per_launch": 2 * fkib * 1024 + wkib * 1024,
             "correction": "read = 2 x FETCH_SIZE, write = WRITE_SIZE (calibrated with tools/pmc_calib.hip: "
                           "FETCH_SIZE = 0.5 x bytes for 1/4/8/16-B coalesced loads, cache-resident or not; "
                           "WRITE_SIZE = bytes for 16-B stores)"}
    db = json.load(open(out)) if os.path.exists(out) else {}
    db[key] = entry
    json.dump(db, open(out, "w"), indent=1)
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
