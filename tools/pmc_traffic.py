#!/usr/bin/env python3
"""Per-kernel HBM traffic from two separate rocprofv3 PMC passes
(--pmc FETCH_SIZE, --pmc WRITE_SIZE; MI355X_MICROARCH.md "rocprofv3 PMC
slots": they do not fit one pass).  Values are in KiB per dispatch.

usage: pmc_traffic.py <fetch_dir> <write_dir> <out.json> <tag>
Writes/updates profiles/traffic.json[tag] with the scan_insert kernel's
per-launch bytes (what bench.py reports as roofline.traffic) and a per-kernel
table.  Calibration caveat (guide §HBM): FETCH_SIZE counts half the bytes of a
16-B/lane coalesced streaming read; the random 8-16 B probes of scan_insert are
an uncalibrated access width, so the raw value is reported as is."""
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
                 "bytes": round((f.get(k, 0.0) + w.get(k, 0.0)) * 1024)} for k in sorted(set(f) | set(w))}
    scan = [k for k in table if "bin_kernel" in k] or [k for k in table if "scan_insert_kernel" in k]
    p = pathlib.Path(out)
    doc = json.loads(p.read_text()) if p.exists() else {}
    doc[tag] = {"hbm_bytes_per_launch": table[scan[0]]["bytes"] if scan else None,
                "kernel": scan[0] if scan else None,
                "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes, "
                          "KiB*1024, raw (uncalibrated access width, see tools/pmc_traffic.py)",
                "per_kernel": table}
    p.write_text(json.dumps(doc, indent=1) + "\n")
    for k, v in sorted(table.items(), key=lambda x: -x[1]["bytes"]):
        print(f"{k:45s} {v['bytes'] / 1e9:8.3f} GB  (fetch {v['fetch_kib'] / 1e6:.3f} GiB-ish, write {v['write_kib'] / 1e6:.3f})")


if __name__ == "__main__":
    main()
