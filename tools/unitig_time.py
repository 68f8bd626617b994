#!/usr/bin/env python3
"""Wall time of the reference program's own unitig extension (binning.c:477-783)
on GPU-materialised tables, and byte-identity of the
drop-in program against the reference program as shipped at the C2 read
shape (READ_LENGTH 152, oracle/build_ref.sh KB_REF_READ_LENGTH).

For each read count n: the C2 generator's first n reads go to a file, one per
line; dropin_k31_m7_c1_rl152 (reference main, GPU process_read/prune_data)
and, when asked, full_k31_m7_c1_rl152 (the reference as shipped) run on it.
stdout is hashed as it streams.  The drop-in's KBH_TRACE lines give
prune_data's and expand_read_id_list's own times (the drop-in replaces both),
so the rest of the wall is the read loop, the extension, print_kmers and the
exit.  Prints one JSON line per run."""
import argparse
import hashlib
import json
import os
import pathlib
import subprocess
import sys
import tempfile
import time

REPO = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "genome-assembly_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import kbin  # noqa: E402
import bench  # noqa: E402


def run(exe, path, timeout, env=None):
    t0 = time.perf_counter()
    p = subprocess.Popen([str(exe), str(path)], stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env)
    h, nbytes = hashlib.sha256(), 0
    deadline = t0 + timeout
    beat = t0
    while True:
        b = p.stdout.read(1 << 20)
        if not b:
            break
        if time.perf_counter() - beat > 20:  # (a heartbeat: the box kills runs silent for 3 min)
            beat = time.perf_counter()
            print(f"  {exe.name}: {nbytes >> 20} MiB out, {beat - t0:.0f} s", file=sys.stderr, flush=True)
        h.update(b)
        nbytes += len(b)
        if time.perf_counter() > deadline:
            p.kill()
            return {"timeout_s": timeout}
    t_eof = time.monotonic()  # (CLOCK_MONOTONIC, as the shim's trace stamps)
    err = p.stderr.read().decode(errors="replace")
    rc = p.wait()
    wall = time.perf_counter() - t0
    out = {"rc": rc, "wall_s": round(wall, 3), "stdout_bytes": nbytes, "sha256": h.hexdigest()[:16]}
    for ln in err.splitlines():
        if ln.startswith("{\"prune_data_ms\""):
            out["prune_data"] = json.loads(ln)
        elif ln.startswith("{\"expand_ms\""):  # the shim's expand_read_id_list (binning.c:857-888)
            out["expand"] = json.loads(ln)
        elif ln.startswith("{\"find_kmer_extensions_ms\""):  # the exact replay (host/unitig.c)
            out.setdefault("find_kmer_extensions", []).append(json.loads(ln))
        elif ln.startswith("{\"t_exit_s\""):  # exit() started: the reference's main has returned
            out["t_exit_s"] = json.loads(ln)["t_exit_s"]
    if "expand" in out and "t_exit_s" in out:
        # after the expansion: find_kmer_extensions x2 + print_kmers; after exit(): teardown
        out["after_expand_to_exit_s"] = round(out["t_exit_s"] - out["expand"]["t_end_s"], 3)
        out["exit_to_eof_s"] = round(t_eof - out.pop("t_exit_s"), 3)
    if "prune_data" in out and "expand" in out:
        pd = out["prune_data"]["prune_data_ms"] / 1e3
        out["rest_s"] = round(wall - pd - out["expand"]["expand_ms"] / 1e3, 3)  # read loop, extension, print, exit
    return out


ap = argparse.ArgumentParser()
ap.add_argument("--reads", type=int, nargs="+", default=[100_000, 1_000_000])
ap.add_argument("--full-max", type=int, default=1_000_000, help="run the reference as shipped up to this many reads")
ap.add_argument("--timeout", type=int, default=500)
ap.add_argument("--M", type=int, default=7, help="MMER_SIZE of the binaries (4: the reference as shipped, "
                                                 "where the unitig extension is live)")
ap.add_argument("--walk-ref", action="store_true",
                help="also run dropinw (the drop-in with the reference's own find_kmer_extensions)")
a = ap.parse_args()
wl = bench.WORKLOADS["c2"]
L = wl["read_len"]
nmax = max(a.reads)
wpr = (L + 31) // 32
w = torch.empty(nmax * wpr, dtype=torch.int64, device="cuda")
ln = torch.empty(nmax, dtype=torch.int32, device="cuda")
kbin.generate_reads_device(w.data_ptr(), ln.data_ptr(), nmax, L, wl["genome"], wl["err_ppm"], bench.gen_seed(wl["seed"]))
torch.cuda.synchronize()
bases, _ = kbin.unpack_reads_to_host(w.data_ptr(), ln.data_ptr(), nmax, wpr, nmax * L)
raw = np.frombuffer(bases, dtype=np.uint8).reshape(nmax, L)
ref = REPO / "oracle" / "_ref"
for n in a.reads:
    with tempfile.NamedTemporaryFile(suffix=".txt", dir="/tmp") as f:
        f.write(np.concatenate([raw[:n], np.full((n, 1), 10, np.uint8)], axis=1).tobytes())
        f.flush()
        row = {"reads": n, "read_len": L}
        row["M"] = a.M
        row["dropin"] = run(ref / f"dropin_k31_m{a.M}_c1_rl152", f.name, a.timeout, dict(os.environ, KBH_TRACE="1"))
        if a.walk_ref:
            row["dropin_refwalk"] = run(ref / f"dropinw_k31_m{a.M}_c1_rl152", f.name, a.timeout,
                                        dict(os.environ, KBH_TRACE="1"))
        if n <= a.full_max:
            row["reference"] = run(ref / f"full_k31_m{a.M}_c1_rl152", f.name, a.timeout)
            if "sha256" in row["reference"] and "sha256" in row["dropin"]:
                row["identical"] = row["reference"]["sha256"] == row["dropin"]["sha256"]
        print(json.dumps(row), flush=True)
