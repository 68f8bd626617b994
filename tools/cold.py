#!/usr/bin/env python3
"""Cold vs warm passes of one workload (diagnostic): per finalize, wall time
and the engine's phase timing, from a fresh context.  Prints one line per pass.
    python tools/cold.py --workload c5 --steps 2"""
import argparse
import pathlib
import sys
import time

REPO = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "genome-assembly_amd"))
import torch  # noqa: E402
import kbin  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c5")
ap.add_argument("--steps", type=int, default=2)
ap.add_argument("--reads", type=int, default=None)
ap.add_argument("--prewarm", type=int, default=0, help="first bin this many reads on a throw-away context")
a = ap.parse_args()
wl = bench.WORKLOADS[a.workload]
n, L, K, M, P = a.reads or wl["reads"], wl["read_len"], wl["K"], wl["M"], wl["parts"]
wpr = (L + 31) // 32
w = torch.empty(n * wpr, dtype=torch.int64, device="cuda")
ln = torch.empty(n, dtype=torch.int32, device="cuda")
kbin.generate_reads_device(w.data_ptr(), ln.data_ptr(), n, L, wl["genome"], wl["err_ppm"], bench.gen_seed(wl["seed"]))
torch.cuda.synchronize()
if a.prewarm:
    with kbin.Engine(K, M, cutoff=1, max_read_len=L) as tmp:
        t0 = time.perf_counter()
        tmp.submit_packed_device(w.data_ptr(), ln.data_ptr(), a.prewarm, wpr, 0)
        tmp.finalize(True)
        torch.cuda.synchronize()
        print(f"prewarm {a.prewarm} reads: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
tcr = time.perf_counter()
with kbin.Engine(K, M, cutoff=1, max_read_len=L) as eng:
    print(f"create: {(time.perf_counter() - tcr) * 1e3:.2f} ms", flush=True)
    eng.set_timing(True)
    for s in range(a.steps):
        eng.reset()
        eng.submit_packed_device(w.data_ptr(), ln.data_ptr(), n, wpr, 0)
        for p in range(P):
            if P > 1:
                eng.set_partition(p, P)
            t0 = time.perf_counter()
            eng.finalize(True)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) * 1e3
            t = eng.timing()
            print(f"step {s} pass {p}: wall {dt:9.2f} ms  scan {t['scan_insert_ms']:8.2f} sort {t['sort_ms']:8.2f} "
                  f"runs {t['runs_ms']:8.2f} bin_kernel {t['bin_kernel_ms']:8.2f} emit {t['emit_ms']:8.2f} "
                  f"bins {t['n_bins']}", flush=True)
