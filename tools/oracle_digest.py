"""Compute a full-size workload's kb_digest with the CPU oracle (VERDICT r04
item 2) and record it as a golden fixture: tests/golden/oracle_digests.json.

The reads are the device generator's (oracle.gen_reads: the CPU twin of
kb_generate_reads_device_at, pinned to the device by
tests/test_gpu_scale.py::test_generator_twin), ids = read index, binned by the
oracle's own scan (kb_oracle.c scan_read: binning.c:902-1076) with the prune
(binning.c:1085-1144), and digested as kb_digest does -- without holding the
12 G-id result (oracle.gen_stream_digest).  bench.py's capacity leg asserts
its GPU digest against this file.

    python tools/oracle_digest.py c3 [--workers 8] [--cap-log2 27]

C3 (100 M x 150 bp, 12 G k-mers): about 45 min on 8 cores, ~30 GB of RAM.
"""
import argparse
import json
import pathlib
import sys
import time

REPO = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "oracle"))
sys.path.insert(0, str(REPO))

import oracle  # noqa: E402

OUT = REPO / "tests" / "golden" / "oracle_digests.json"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workload", choices=["c2", "c3", "c4", "c5"])
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--cap-log2", type=int, default=27)
    ap.add_argument("--reads", type=int, default=0, help="a prefix of the workload's reads (0: all)")
    a = ap.parse_args()
    import bench  # (the workload table and its seeds; bench imports torch lazily enough for this)
    wl = bench.WORKLOADS[a.workload]
    n = a.reads or wl["reads"]
    seed = bench.gen_seed(wl["seed"])
    t0 = time.time()
    dig, nk = oracle.gen_stream_digest(n, wl["read_len"], wl["genome"], wl["err_ppm"], seed, wl["K"], wl["M"],
                                       cutoff=1, prune=True, read_base=0, id0=0, workers=a.workers,
                                       cap_log2=a.cap_log2)
    dt = time.time() - t0
    rec = {"workload": a.workload, "reads": n, "read_len": wl["read_len"], "genome": wl["genome"],
           "err_ppm": wl["err_ppm"], "seed": seed, "K": wl["K"], "M": wl["M"], "cutoff": 1, "prune": True,
           "ids": "read index", "kmers": nk, "digest": [hex(x) for x in dig], "seconds": round(dt, 1),
           "workers": a.workers, "source": "oracle.gen_stream_digest (oracle/kb_oracle.c)"}
    print(json.dumps(rec))
    data = json.loads(OUT.read_text()) if OUT.exists() else {}
    data[f"{a.workload}" if not a.reads else f"{a.workload}_prefix{n}"] = rec
    OUT.write_text(json.dumps(data, indent=1, sort_keys=True) + "\n")


if __name__ == "__main__":
    main()
