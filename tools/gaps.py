"""Idle gaps between the kernels of one finalize, from a rocprofv3 kernel trace.

    python tools/gaps.py gpurun_out/<dir>/kt/<host>/<pid>_kernel_trace.csv

A finalize starts at clear_kernel; for the last few complete finalizes it
prints the span (first kernel start to last kernel end), the summed kernel
time, and every gap above 2 us with the kernels either side."""
import csv
import glob
import sys


def main(path):
    if "*" in path:
        path = sorted(glob.glob(path))[0]
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    starts = [i for i, k in enumerate(ks) if k[2].startswith("kb::clear_kernel")]
    fins = [(a, b) for a, b in zip(starts, starts[1:] + [len(ks)])]
    for a, b in fins[-4:-1]:
        seq = ks[a:b]
        span = seq[-1][1] - seq[0][0]
        busy = sum(e - s for s, e, _ in seq)
        print(f"finalize: {len(seq)} kernels, span {span / 1e3:.1f} us, kernels {busy / 1e3:.1f} us, "
              f"idle {(span - busy) / 1e3:.1f} us")
        for (s0, e0, n0), (s1, e1, n1) in zip(seq, seq[1:]):
            g = s1 - e0
            if g > 2000:
                print(f"   gap {g / 1e3:7.1f} us  after {n0[:48]:48s} before {n1[:48]}")
        for s, e, n in seq:
            print(f"      {(e - s) / 1e3:8.1f} us  {n[:70]}")


if __name__ == "__main__":
    main(sys.argv[1])
