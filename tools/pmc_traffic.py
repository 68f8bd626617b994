#!/usr/bin/env python3
"""Per-kernel HBM traffic from two separate rocprofv3 PMC passes
(--pmc FETCH_SIZE, --pmc WRITE_SIZE; MI355X_MICROARCH.md "rocprofv3 PMC
slots": they do not fit one pass).  Values are in KiB per dispatch.

usage: pmc_traffic.py <fetch_dir> <write_dir> <out.json> <tag>
Writes/updates profiles/traffic.json[tag] with the dominant kernel's
per-launch bytes (what bench.py reports as roofline.traffic) and a per-kernel
table.  Correction (MI355X_MICROARCH.md §HBM, calibrated for our access widths
by tools/pmc_calib.hip, profiles/r01/pmc_calib.txt): FETCH_SIZE reports half the
bytes of coalesced 8-B and 16-B per lane reads, so reads count x2; WRITE_SIZE
is exact for coalesced 8-B stores and counts a scattered 4-B store as a ~32-B
partial-line write (7.56 x the bytes on the calibration pattern) -- real
memory-side write requests, so it is kept as is."""
import collections
import csv
import json
import pathlib
import sys


def per_kernel(d):
    agg = collections.defaultdict(list)
    files = sorted(pathlib.Path(d).rglob("*counter_collection.csv"))
    for f in files:
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    fetch, write, out, tag = sys.argv[1:5]
    f, w = per_kernel(fetch), per_kernel(write)
    table = {k: {"fetch_kib": round(f.get(k, 0.0), 1), "write_kib": round(w.get(k, 0.0), 1),
                 "bytes": round((2.0 * f.get(k, 0.0) + w.get(k, 0.0)) * 1024)} for k in sorted(set(f) | set(w))}
    scan = [k for k in table if "bin_kernel" in k] or [k for k in table if "scan_insert_kernel" in k]
    p = pathlib.Path(out)
    doc = json.loads(p.read_text()) if p.exists() else {}
    doc[tag] = {"hbm_bytes_per_launch": table[scan[0]]["bytes"] if scan else None,
                "kernel": scan[0] if scan else None,
                "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes, KiB*1024; "
                          "bytes = 2 x FETCH (calibrated: coalesced 8/16-B reads count half) + WRITE "
                          "(exact for coalesced stores; scattered 4-B stores as 32-B partial writes)",
                "per_kernel": table}
    p.write_text(json.dumps(doc, indent=1) + "\n")
    for k, v in sorted(table.items(), key=lambda x: -x[1]["bytes"]):
        print(f"{k:45s} {v['bytes'] / 1e9:8.3f} GB  (fetch {v['fetch_kib'] / 1e6:.3f} GiB-ish, write {v['write_kib'] / 1e6:.3f})")


if __name__ == "__main__":
    main()
