#!/usr/bin/env python3
"""Per-kernel HBM traffic from two separate rocprofv3 PMC passes
(--pmc FETCH_SIZE, --pmc WRITE_SIZE; MI355X_MICROARCH.md "rocprofv3 PMC
slots": they do not fit one pass).  Counter values are KiB per dispatch.

usage: pmc_traffic.py <fetch_dir> <write_dir> <out.json> <tag> [--skip-gen]

Every kernel's dispatches are split into the COLD first dispatch (a fresh
context: nothing learned yet -- the first bench warmup step) and the STEADY
ones (every later dispatch; the mean is reported, with min/max).  Writes
out.json[tag]: the roofline kernel's steady per-launch bytes (what bench.py
reports as roofline.traffic), its cold bytes, and a per-kernel table.

Correction (MI355X_MICROARCH.md §HBM, calibrated for our access widths by
tools/pmc_calib.hip, profiles/pmc_calib.txt): FETCH_SIZE reports half the
bytes of coalesced 8-B and 16-B per-lane reads, so reads count x2; WRITE_SIZE
is exact for coalesced 8-B/16-B stores and counts a scattered 4-B store as a
~32-B partial-line write (7.56 x its bytes on the calibration pattern) -- real
memory-side write requests, so it is kept as is."""
import collections
import csv
import json
import pathlib
import sys


def dispatches(d):
    """kernel -> [KiB per dispatch] in dispatch order"""
    rows = []
    for f in sorted(pathlib.Path(d).rglob("*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"].split("(")[0], float(r["Counter_Value"])))
    agg = collections.defaultdict(list)
    for _, k, v in sorted(rows):
        agg[k].append(v)
    return agg


def split(v):
    steady = v[1:] or v
    return v[0], sum(steady) / len(steady), min(steady), max(steady), len(steady)


def main():
    fetch, write, out, tag = sys.argv[1:5]
    f, w = dispatches(fetch), dispatches(write)
    table = {}
    for k in sorted(set(f) | set(w)):
        fc, fs, fmin, fmax, n = split(f.get(k, [0.0]))
        wc, ws, wmin, wmax, _ = split(w.get(k, [0.0]))
        table[k] = {"dispatches": n + 1,
                    "steady": {"fetch_kib": round(fs, 1), "write_kib": round(ws, 1),
                               "bytes": round((2.0 * fs + ws) * 1024),
                               "bytes_min": round((2.0 * fmin + wmin) * 1024),
                               "bytes_max": round((2.0 * fmax + wmax) * 1024)},
                    "cold": {"fetch_kib": round(fc, 1), "write_kib": round(wc, 1),
                             "bytes": round((2.0 * fc + wc) * 1024)}}
    # (the bin kernel variant with the most dispatches: ranked bins run
    # bin_kernel_ranked, the cold pass the plain one)
    roof = sorted([k for k in table if "bin_kernel" in k], key=lambda k: -table[k]["dispatches"]) or \
        [k for k in table if "scan_insert_kernel" in k]
    # the bin phase as one "kernel" (bench.py's roofline kernel when heavy bins
    # dominate: C3, C5): every kernel between the bucket ordering and the lists
    phase = [k for k in table if any(x in k for x in ("bin_kernel", "flat_count_kernel", "flat_scan_kernel",
                                                        "flat_scatter_kernel", "flat_scatter_lds_kernel",
                                                        "bin_parts_kernel",
                                                        "bins_final_kernel"))]
    if phase:
        # (of the bin kernel's variants only the most dispatched counts: the
        # plain bin_kernel runs the passes before ranked bins are enabled --
        # the cold one -- and bin_kernel_ranked every later one)
        bk = [k for k in phase if "bin_kernel" in k]
        main_bk = max(bk, key=lambda k: table[k]["dispatches"]) if bk else None
        steady_m = [k for k in phase if "bin_kernel" not in k or k == main_bk]
        first_bk = min(bk, key=lambda k: table[k]["dispatches"]) if bk else None  # (ran the cold pass)
        cold_m = [k for k in phase if "bin_kernel" not in k or k == first_bk]
        table["bin phase"] = {"dispatches": min(table[k]["dispatches"] for k in steady_m or phase),
                              "members": sorted(phase),
                              "steady": {"bytes": sum(table[k]["steady"]["bytes"] for k in steady_m)},
                              "cold": {"bytes": sum(table[k]["cold"]["bytes"] for k in cold_m)}}
    p = pathlib.Path(out)
    doc = json.loads(p.read_text()) if p.exists() else {}
    doc[tag] = {"hbm_bytes_per_launch": table[roof[0]]["steady"]["bytes"] if roof else None,
                "cold_hbm_bytes": table[roof[0]]["cold"]["bytes"] if roof else None,
                "kernel": roof[0] if roof else None,
                "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes, KiB*1024; "
                          "bytes = 2 x FETCH (calibrated: coalesced 8/16-B reads count half) + WRITE "
                          "(exact for coalesced stores; scattered 4-B stores as 32-B partial writes); "
                          "steady = mean over every dispatch after the first, cold = the first",
                "per_kernel": table}
    p.write_text(json.dumps(doc, indent=1) + "\n")
    step = sum(v["steady"]["bytes"] for k, v in table.items() if k != "bin phase")
    print(f"{tag}: steady-state bytes per step (all kernels) {step / 1e9:.3f} GB")
    for k, v in sorted(table.items(), key=lambda x: -x[1]["steady"]["bytes"]):
        print(f"{k:45s} steady {v['steady']['bytes'] / 1e9:8.3f} GB  cold {v['cold']['bytes'] / 1e9:8.3f} GB"
              f"  (x{v['dispatches']})")


if __name__ == "__main__":
    main()
