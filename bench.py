#!/usr/bin/env python3
"""Headline benchmark: canonical k-mers binned per second (BASELINE.json).

One step = one full pass of the hot path over one resident batch of synthetic
reads: k-mer offsets -> fused signature scan + (mmer,kmer) table insert/count
-> low-abundance prune + compaction -> read-id placement -> per-key id order.
Inputs are generated on the device before the timed region (seeded, SURVEY
§8(d) C2 at N=1: 1M x 150 bp, genome 5 Mbp, 0.1% substitutions, seed 2,
K=31 M=7, cutoff 1); outputs stay device-resident (CSR).

N>1 (torchrun, one rank per GPU): rank r generates reads [r n, (r+1) n) of
the workload's ONE genome (weak scaling: n reads per GPU; coverage grows with
N) and k-mers are routed to the GPU that owns their canonical mmer with an
RCCL all-to-all (genome-assembly_amd/kbin/dist.py).

Prints ONE JSON line on rank 0 (contract in the task statement); extra
objects: "roofline" for the dominant kernel (bin_kernel; scan_insert_kernel
on the table engine) and "cpu_baseline" (the compiled reference, with the C
port beside it, on a bounded sample of the same workload, rank 0 only).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import pathlib
import sys
import time

REPO = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "genome-assembly_amd"))


import numpy as np  # noqa: E402
import torch  # noqa: E402  (loaded before libkbin: one HIP runtime per process)

import kbin  # noqa: E402

METRIC = "canonical k-mers binned/sec, 150bp k=31, at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


# SURVEY.md §8(d) configurations (per GPU: C4/C5 are the per-rank shares of
# the 8-GPU runs; at N>1 every rank bins its own share, routed by mmer owner)
WORKLOADS = {
    "c2": {"reads": 1_000_000, "read_len": 150, "K": 31, "M": 7, "err_ppm": 1000,
           "genome": 5_000_000, "seed": 2, "parts": 1, "name": "C2"},
    # 12G occurrences: the 32-bit occurrence index of one finalize caps a pass
    # at 2^32, so the step bins disjoint mmer partitions in turn
    "c3": {"reads": 100_000_000, "read_len": 150, "K": 31, "M": 7, "err_ppm": 1000,
           "genome": 5_000_000, "seed": 3, "parts": 4, "name": "C3"},
    # 1B x 150 bp over 8 GPUs: 125M reads (15G occurrences) per GPU
    "c4": {"reads": 125_000_000, "read_len": 150, "K": 31, "M": 7, "err_ppm": 1000,
           "genome": 3_100_000_000, "seed": 4, "parts": 5, "name": "C4 (per-GPU share)"},
    # 500M x 250 bp, K63 two-word k-mers, 1% errors, over 8 GPUs: 62.5M reads per GPU
    "c5": {"reads": 62_500_000, "read_len": 250, "K": 63, "M": 7, "err_ppm": 10000,
           "genome": 3_100_000_000, "seed": 5, "parts": 4, "name": "C5 (per-GPU share)"},
}


def gen_seed(seed: int) -> int:
    """generator seed of workload seed `seed` (rank 0's stream of round 1, so
    the C3 digest recorded in DESIGN.md stays comparable)"""
    return seed * 1000003


def algorithmic_bytes_per_read(L: int, K: int) -> float:
    """ceil(L/4) (2-bit read) + n_k * (Kb + 12) per read, Kb = 8 B
    (K<=32) or 16 B: per k-mer a slot-key read, a 4-B count read + 4-B write,
    a 4-B occurrence/id write."""
    nk = max(0, L - K + 1)
    kb = 8 if K <= 32 else 16
    return (L + 3) // 4 + nk * (kb + 12)


def host_cores() -> int:
    """CPU threads this process may use on the host: the affinity mask, capped
    by OMP_NUM_THREADS where the box sets it (the GPU box's per-GPU share)"""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(omp))) if omp.isdigit() else n


def _run_ref(binary, path, L, timeout=300):
    """one reference harness run in timing mode: (k-mers, seconds of the fgets +
    process_read loop and prune_data)"""
    import subprocess
    out = subprocess.run([str(binary), path, str(L + 2), "1", "time"], capture_output=True, text=True,
                         timeout=timeout, check=True).stdout
    kv = dict(t.split("=") for t in out.split())
    return int(kv["kmers"]), float(kv["bin_s"]), float(kv["prune_s"])


def cpu_baseline(words, lens, n_avail, n_sample, wpr, L, K, M, cutoff, ref_sample):
    """CPU baseline on the host cores of this box (BASELINE.md's CPU plan).

    kind "reference": the reference's own binning.c/zhash.c/llist.c, compiled
    in the build container by oracle/build_ref.sh into oracle/_ref/ (the
    binaries travel with the tree), timed by its harness over the fgets +
    process_read loop and prune_data (BASELINE.md's timed region), reads
    written one per line (READ_LENGTH = L + 2, no split).  The headline value
    is the AGGREGATE of C independent reference processes (C = host_cores())
    on C disjoint shards of the workload's reads, run at once -- an upper
    bound for the reference on this host, since the shards' tables are never
    merged.  Beside it: one core at -O2 on the first ref_sample
    reads, one core with the makefile's flags (-g, no -O) on half of them,
    and the clean-room C port (oracle/kb_oracle.c) on n_sample reads
    ("port", the baseline when no reference binary is present).
    """
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle  # test-infrastructure checker, used here only as the CPU baseline leg
    import subprocess
    import tempfile
    cores = host_cores()
    n_host = min(n_avail, max(n_sample, ref_sample * 4))
    bases, hl = kbin.unpack_reads_to_host(words.data_ptr(), lens.data_ptr(), n_host, wpr, n_host * L)
    buf = np.frombuffer(bases, dtype=np.uint8) if not isinstance(bases, np.ndarray) else bases
    t0 = time.perf_counter()
    r = oracle.bin_reads(buf[:n_sample * L].tobytes(), hl[:n_sample], K, M, cutoff, True)
    dt = time.perf_counter() - t0
    port = {"value": r.n_kmers / dt, "unit": "k-mers/s", "cores": 1, "kind": "port",
            "sample": f"first {n_sample} reads of the bench workload ({r.n_kmers} k-mers), "
                      f"oracle/kb_oracle.c single-threaded, {dt:.2f} s"}
    ref = REPO / "oracle" / "_ref" / f"ref_k{K}_m{M}_c{cutoff}"
    refg = REPO / "oracle" / "_ref" / f"refg_k{K}_m{M}_c{cutoff}"
    if not (ref_sample > 0 and ref.is_file() and os.access(ref, os.X_OK)):
        return {**port, "note": "reference binary absent: clean-room port only"}
    assert all(int(x) == L for x in hl[:n_host]), "fixed-length reads expected"

    def write(d, name, a, b):  # reads [a, b) as lines
        p = os.path.join(d, name)
        lines = np.concatenate([buf[a * L:b * L].reshape(b - a, L), np.full((b - a, 1), 10, np.uint8)], axis=1)
        with open(p, "wb") as f:
            f.write(lines.tobytes())
        return p

    rows = {}
    try:
        with tempfile.TemporaryDirectory() as d:
            m = min(ref_sample, n_host)
            km, bs, ps = _run_ref(ref, write(d, "one.txt", 0, m), L)
            rows["ref_1core_O2"] = {"value": km / (bs + ps), "cores": 1,
                                    "sample": f"first {m} reads ({km} k-mers): process_read loop {bs:.2f} s "
                                              f"+ prune_data {ps:.2f} s, gcc -O2"}
            if refg.is_file():
                mg = max(1, m // 2)
                km, bs, ps = _run_ref(refg, write(d, "g.txt", 0, mg), L)
                rows["ref_1core_g"] = {"value": km / (bs + ps), "cores": 1,
                                       "sample": f"first {mg} reads ({km} k-mers), makefile flags (-g, no -O): "
                                                 f"{bs + ps:.2f} s"}
            # C independent processes on C disjoint shards, all at once
            sh = max(1, min(n_host // cores, m))
            paths = [write(d, f"s{i}.txt", i * sh, (i + 1) * sh) for i in range(cores)]
            tw = time.perf_counter()
            procs = [subprocess.Popen([str(ref), p, str(L + 2), "1", "time"], stdout=subprocess.PIPE, text=True)
                     for p in paths]
            outs = [pr.communicate(timeout=300)[0] for pr in procs]
            wall = time.perf_counter() - tw
            if any(pr.returncode for pr in procs):
                raise subprocess.CalledProcessError(1, str(ref))
            kvs = [dict(t.split("=") for t in o.split()) for o in outs]
            kms = sum(int(kv["kmers"]) for kv in kvs)
            # the timed region of every process (fgets + process_read + prune_data),
            # all running at once: the slowest one sets the aggregate
            slow = max(float(kv["bin_s"]) + float(kv["prune_s"]) for kv in kvs)
    except (subprocess.SubprocessError, OSError, ValueError, KeyError) as e:
        if not rows:
            port["note"] = f"reference binary failed ({type(e).__name__}); port reported"
            return port
        one = rows["ref_1core_O2"]
        return {"value": one["value"], "unit": "k-mers/s", "cores": 1, "kind": "reference",
                "sample": one["sample"], "rows": rows, "port": port,
                "note": f"aggregate run failed ({type(e).__name__})"}
    return {"value": kms / slow, "unit": "k-mers/s", "cores": cores, "kind": "reference",
            "sample": f"{cores} independent reference processes (gcc -O2) run at once on {cores} disjoint "
                      f"shards of {sh} reads of the bench workload ({kms} k-mers): the slowest one's "
                      f"fgets + process_read + prune_data took {slow:.2f} s (process wall {wall:.2f} s); "
                      f"the shards' tables are never merged, and a {sh}-read shard keeps each "
                      f"process's tables far smaller than one table over the whole workload (faster "
                      f"zhash chains, fewer rehashes): the shard size is part of why this is an upper "
                      f"bound (one core on the first {m} reads: {rows['ref_1core_O2']['value'] / 1e6:.2f} M "
                      f"k-mers/s); "
                      f"host nproc={os.cpu_count()}",
            "rows": rows, "port": port}


def host_input_leg(words, lens, n, wpr, L, K, M, cutoff, device, batch=1 << 16, reps=3):
    """The host-ingest path (H2D of input and D2H of output
    reported separately): the workload's reads as host ASCII go through
    kb_submit in batches (pinned double-buffered staging, H2D + pack on the
    context's stream), then kb_finalize, then kb_export (D2H of the CSR into
    pinned buffers).  Best of `reps` runs; not the bench value."""
    bases, hl = kbin.unpack_reads_to_host(words.data_ptr(), lens.data_ptr(), n, wpr, n * L, device=device)
    raw = np.frombuffer(bases, dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(hl.astype(np.int64))])
    chunks = [(bytes(raw[offs[a]:offs[min(a + batch, n)]]), hl[a:a + batch], a) for a in range(0, n, batch)]
    best = None
    with kbin.Engine(K, M, cutoff=cutoff, max_read_len=L, device=device) as eng:
        for _ in range(reps + 1):  # (the first run sizes the pool and buffers)
            eng.reset()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for b, ln, a in chunks:
                eng.submit(bases=b, lens=ln, first_id=int(a))
            t_ret = time.perf_counter()
            torch.cuda.synchronize()  # every H2D copy and pack done
            t1 = time.perf_counter()
            eng.finalize(prune=True)
            t2 = time.perf_counter()
            csr = kbin.kb_csr()  # kb_export alone: the D2H into its pinned buffers, no Python copies
            rc = eng.lib.kb_export(eng._h, ctypes.byref(csr))
            t3 = time.perf_counter()
            if rc:
                raise RuntimeError(f"kb_export failed: {rc}")
            row = {"ingest_ms": (t1 - t0) * 1e3, "submit_return_ms": (t_ret - t0) * 1e3,
                   "finalize_ms": (t2 - t1) * 1e3, "export_ms": (t3 - t2) * 1e3,
                   "end_to_end_ms": (t3 - t0) * 1e3}
            if best is None or row["end_to_end_ms"] < best["end_to_end_ms"]:
                best = row
        out_bytes = int(csr.n_entries) * (4 + 8 + 8 + 4 + 8) + 8 + int(csr.n_ids) * 4
    in_bytes = len(raw) + n * 4
    kmers = n * max(0, L - K + 1)
    return {"batch_reads": batch, "reads": n,
            **{k: round(v, 3) for k, v in best.items()},
            "h2d_GBps": round(in_bytes / best["ingest_ms"] / 1e6, 2),
            "d2h_GBps": round(out_bytes / best["export_ms"] / 1e6, 2),
            "end_to_end_kmers_per_s": round(kmers / best["end_to_end_ms"] * 1e3, 1),
            "note": "host ASCII reads -> kb_submit batches (H2D + 2-bit pack) -> kb_finalize -> kb_export "
                    "(D2H of the CSR); ingest_ms includes the pack kernel, export_ms the whole CSR copy"}


def dropin_leg(words, lens, n, wpr, L, K, M, cutoff, device):
    """The reference surface end to end: kbin_main is
    binning.c's main up to the prune -- fgets loop, process_read per read,
    prune_data -- over libkbin_host (the process_read / prune_data shim) and
    libkbin.so, on the workload's reads written one per line.  prune_data
    finalises on the GPU, exports the CSR and materialises the reference's
    ZHashTable / ll_node tables (first-occurrence insertion order), then
    prunes them; its phases come from kbh_last_times.  Not the bench value."""
    import subprocess
    import tempfile
    exe = REPO / "genome-assembly_amd" / "lib" / "kbin_main"
    if not exe.is_file():
        return {"note": "kbin_main not built"}
    bases, hl = kbin.unpack_reads_to_host(words.data_ptr(), lens.data_ptr(), n, wpr, n * L, device=device)
    raw = np.frombuffer(bases, dtype=np.uint8).reshape(n, L)
    with tempfile.NamedTemporaryFile(suffix=".txt") as f:
        f.write(np.concatenate([raw, np.full((n, 1), 10, np.uint8)], axis=1).tobytes())
        f.flush()
        env = dict(os.environ, KBH_TIMING="1", KBH_NODUMP="1")
        t0 = time.perf_counter()
        r = subprocess.run([str(exe), f.name, str(K), str(M), str(L + 2), str(cutoff), "1", str(device)],
                           capture_output=True, text=True, timeout=600, env=env)
        wall = time.perf_counter() - t0
    if r.returncode:
        return {"note": f"kbin_main failed rc={r.returncode}: {r.stderr[-300:]}"}
    row = json.loads(r.stderr.strip().splitlines()[-1])
    row["process_wall_ms"] = round(wall * 1e3, 1)
    row["kmers_per_s"] = round(row["kmers"] / row["total_ms"] * 1e3, 1)
    row["note"] = ("kbin_main: fgets + process_read loop (async batched kb_submit) -> prune_data "
                   "(kb_finalize, kb_export, direct zhash layout: every table's insertion/rehash history "
                   "replayed on integer codes, only surviving entries and their ll_node lists allocated); "
                   "total_ms = read loop + prune_data; process_wall_ms adds process start, HIP init and "
                   "the file read")
    return row


def load_traffic(tag: str, kernel: str):
    """Per-launch HBM bytes of the roofline kernel from the committed rocprofv3
    --pmc passes (profiles/traffic.json, written by tools/pmc_traffic.py):
    the steady-state launches (every dispatch after the first) and the cold
    first one, reported separately."""
    p = REPO / "profiles" / "traffic.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text()).get(tag)
        if not d:
            return None
        k = "bin phase" if kernel.startswith("bin phase") else kernel.split("<")[0]
        pk = d.get("per_kernel", {})
        # (the tag's roofline kernel is its most-dispatched variant: ranked bins
        # run bin_kernel_ranked, the cold pass the plain bin_kernel)
        row = pk.get(d.get("kernel")) if k != "bin phase" and k in (d.get("kernel") or "") else None
        row = row or next((v for name, v in pk.items() if k in name), None)
        if not row or "steady" not in row:
            return None
        return {"hbm_bytes_per_launch": row["steady"]["bytes"], "cold_bytes": row["cold"]["bytes"],
                "source": f"profiles/traffic.json[{tag}]"}
    except Exception:
        return None


def single_gpu_runner(K, M, L, cutoff, n, wpr, P, local, reads, pass_log, scan_once=True):
    """The single-GPU step of a workload: (engine, step(digest=False)).  P > 1:
    one super-k-mer pass over the reads (kb_split_passes) fills the P passes'
    regions and each pass bins its region (no rescans) -- or, when the regions
    would not fit beside the passes' buffers (or scan_once is off), every pass
    rescans the reads with kb_set_partition.  step() appends (export_device,
    timing, None) of every pass to pass_log and returns the digest summed over
    the passes when asked."""
    eng = kbin.Engine(K, M, cutoff=cutoff, max_read_len=L, device=local)
    # Super-k-mers per read: about 2 (L - K + 1) / (K - M + 2) (a sticky
    # signature holds for half a window on average; ~10 at 150 bp K31 M7,
    # ~7 at 250 bp K63 M7), with a margin; the partition hash splits them
    # evenly, and a short region is retried bigger.  Gated on the HBM: the
    # regions sit beside the pass's own buffers
    per_read = 2.0 * max(1, L - K + 1) / (K - M + 2) * 1.25 + 1.0
    split = {"cap": int(n * per_read / P * 1.1) + 4096, "buf": None, "counts": None}
    split_bytes = P * split["cap"] * (1 + (2 * K - M + 31) // 32) * 8
    scan_once = (P > 1 and scan_once
                 and split_bytes < 0.15 * torch.cuda.get_device_properties(local).total_memory)
    sender = kbin.Engine(K, M, cutoff=cutoff, max_read_len=L, device=local) if scan_once else None
    rw = eng.record_words()

    def scan():
        sender.reset()
        w, ln = reads()
        sender.submit_packed_device(w.data_ptr(), ln.data_ptr(), n, wpr, first_id=0)
        for _ in range(3):
            need = P * split["cap"] * rw
            if split["buf"] is None or split["buf"].numel() < need:
                split["buf"] = None  # (free the old one first)
                split["buf"] = torch.empty(need, dtype=torch.int64, device="cuda")
            ok, counts = sender.split_passes(P, split["buf"].data_ptr(), split["cap"])
            if ok:
                split["counts"] = [int(c) for c in counts]
                return
            split["cap"] = int(int(counts.max()) * 1.1) + 1024
        raise RuntimeError("kb_split_passes: region capacity not converging")

    dbg = os.environ.get("BENCH_DEBUG") == "1"

    def step(digest=False):
        pass_log.clear()
        dig = [0, 0, 0, 0]
        t0 = time.perf_counter()
        if scan_once:
            scan()
            if dbg:
                torch.cuda.synchronize()
                print(f"[bench] scan {1e3 * (time.perf_counter() - t0):.1f} ms (cap {split['cap']})",
                      file=sys.stderr, flush=True)
        for p in range(P):
            eng.reset()
            if scan_once:
                eng.set_partition(p, P)
                eng.submit_superkmers_device(split["buf"][p * split["cap"] * rw:].data_ptr(),
                                             split["counts"][p])
            else:
                w, ln = reads()
                eng.submit_packed_device(w.data_ptr(), ln.data_ptr(), n, wpr, first_id=0)
                if P > 1:
                    eng.set_partition(p, P)
            eng.finalize(prune=True)
            if dbg:
                print(f"[bench] pass {p} done at {1e3 * (time.perf_counter() - t0):.1f} ms", file=sys.stderr,
                      flush=True)
            # (one pass: its export is the same shape every step -- read once
            # after the timed steps; the timing struct converted after them too)
            pass_log.append((eng.export_device() if P > 1 else None, eng.timing_raw(), None))
            if digest:
                dig = [(a + b) % (1 << 64) for a, b in zip(dig, eng.digest())]
        return dig

    return eng, step


def roofline(passes, L, K, world, kmers_scanned_per_s, tag):
    """roofline of the dominant kernel: SURVEY.md 8(d)'s algorithmic bytes per
    k-mer occurrence x the occurrences one launch processes / the launch's
    device time (HIP events on the engine stream, inside the timed loop).
    Binned: bin_kernel alone (events right around it) while it does most of
    the bin phase (light bins, C2); when heavy bins dominate (C3) it only
    publishes them, and the roofline kernel is the whole bin phase (runs_ms:
    bin_kernel, the heavy-bin kernels, bins_final)."""
    tim = [t for _, t in passes]
    bpk = algorithmic_bytes_per_read(L, K) / max(1, L - K + 1)
    binned = int(tim[-1]["engine"]) == kbin.KB_ENG_BINNED
    kname = "bin_kernel" if binned else ("scan_insert_kernel<1>" if K <= 31 else "scan_insert_kernel<2>")
    # (runs_ms 0: the pass ran with bin_kernel's events only -- a light-bin
    # workload, see main)
    bin_alone = binned and all(0 < t.get("bin_kernel_ms", 0) and t["bin_kernel_ms"] >= 0.5 * t["runs_ms"]
                               for t in tim)
    if binned and not bin_alone:
        kname = "bin phase (bin_kernel + heavy-bin kernels)"
    launch_ms = [(t["bin_kernel_ms"] if bin_alone else t["runs_ms"]) if binned
                 else t["scan_insert_ms"] / max(1, t["scan_insert_launches"]) for t in tim]
    avg_kernel_ms = float(np.mean(launch_ms))
    kmers_per_launch = float(np.mean([int(d["n_kmers"]) for d, _ in passes]))
    achieved = kmers_per_launch * bpk / (avg_kernel_ms * 1e-3) / 1e9  # GB/s, per launch
    traffic = load_traffic(tag, kname)
    return {"bound": "hbm", "kernel": kname,
            "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic.get("hbm_bytes_per_launch") if traffic else None,
            **({"traffic_cold_launch": traffic["cold_bytes"], "traffic_source": traffic["source"]}
               if traffic else {}),
            "kernel_ms": round(avg_kernel_ms, 4),
            "kmers_per_launch": int(kmers_per_launch),
            "bytes_per_kmer": round(bpk, 3),
            "path_frac": round(kmers_scanned_per_s * bpk / (world * HBM_PEAK_GBS * 1e9), 4)}


def path_counters(passes):
    """which bin-phase paths the passes took (kb_timing path counters, summed)"""
    keys = ("n_bins", "split_mmers", "heavy_bins", "split_bins", "partitions", "offset_partitions",
            "flat_partitions", "overflow_redos", "prefiltered", "long_lists", "clustered_lists",
            "tail_reruns", "light_prefilter_bins", "ranked_bins", "bitmap_partitions")
    out = {k: int(sum(int(t.get(k, 0)) for _, t in passes)) for k in keys}
    out["max_depth"] = int(max(int(t.get("max_depth", 0)) for _, t in passes))
    return out


# C3's digest over its 4 passes (kb_digest summed): entries, ids, key sum,
# list sum -- computed by the CPU oracle over the same generated reads
# (tools/oracle_digest.py c3: oracle/kb_oracle.c's scan, 12 G k-mers, 52 min
# on 8 cores), not taken from a GPU run
C3_DIGEST = tuple(json.loads((REPO / "tests" / "golden" / "oracle_digests.json").read_text())["c3"]["digest"])


def capacity_leg(local, steps=2, warmup=1):
    """SURVEY 8(d) C3 on one GPU (the largest single-GPU BASELINE config:
    100M x 150 bp, 12 G k-mer occurrences, P = 4 mmer-partitioned passes, one
    super-k-mer scan for all passes): ms per step, the bin phase's roofline, the
    paths taken, and the full result's digest checked against the committed
    one.  Not the bench value (the headline is C2)."""
    wl = WORKLOADS["c3"]
    n, L, K, M, P = wl["reads"], wl["read_len"], wl["K"], wl["M"], wl["parts"]
    wpr = (L + 31) // 32
    w = torch.empty(n * wpr, dtype=torch.int64, device="cuda")
    ln = torch.empty(n, dtype=torch.int32, device="cuda")
    kbin.generate_reads_device(w.data_ptr(), ln.data_ptr(), n, L, wl["genome"], wl["err_ppm"],
                               gen_seed(wl["seed"]), device=local, read_base=0)
    torch.cuda.synchronize()
    pass_log = []
    eng, step = single_gpu_runner(K, M, L, 1, n, wpr, P, local, lambda off=0: (w, ln), pass_log)
    eng.set_timing(True)
    tc = time.perf_counter()
    step()
    torch.cuda.synchronize()
    cold_ms = (time.perf_counter() - tc) * 1e3
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    log = []
    for _ in range(steps):
        step()
        log.extend((d, kbin.timing_dict(t)) for d, t, *_ in pass_log)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    kmers = n * (L - K + 1)
    dig = tuple(hex(x) for x in step(digest=True))
    torch.cuda.synchronize()
    del eng, step
    out = {"workload": f"C3: {n} x {L}bp reads, genome {wl['genome']} bp, {wl['err_ppm'] / 1e4:.2f}% "
                       f"substitutions, seed {wl['seed']}, K={K} M={M}, prune cutoff 1, {P} mmer-partitioned "
                       f"passes (one super-k-mer scan)",
           "value": round(kmers / dt, 1), "unit": "k-mers/s", "ms_per_step": round(dt * 1e3, 3),
           "steps": steps, "cold_first_step_ms": round(cold_ms, 1),
           "roofline": roofline(log, L, K, 1, kmers / dt, f"n{n}_L{L}_K{K}_M{M}_P{P}"),
           "phases_ms": {k: round(float(sum(t[k] for _, t in log)) / steps, 3)
                         for k in ("scan_insert_ms", "sort_ms", "runs_ms", "emit_ms", "total_ms")},
           "paths": path_counters(log[-P:]),
           "digest": list(dig), "digest_expected": list(C3_DIGEST), "digest_ok": dig == C3_DIGEST}
    if not out["digest_ok"]:
        print(f"capacity leg: C3 digest {dig} != committed {C3_DIGEST}", file=sys.stderr)
    return out


def routed_runner(K, M, L, cutoff, n, wpr, P, local, rank, reads, pass_log, pipeline=True, cur=None):
    """one rank of the mmer-sharded job (kbin.dist over the C-ABI group: C
    routing, RCCL exchange from C under an nccl process group; torch
    collectives under gloo): rank r bins reads(off) = its n reads (ids r n ..)
    together with every other rank's, P mmer-partitioned passes a step.
    Returns (runner, engine, step, drain)."""
    from kbin import dist as kdist
    # (KB_ROUTED_TRANSPORT=c|torch: the exchange's transport; default the C
    # group under nccl, torch collectives under gloo -- a gloo rehearsal of
    # the C group's plumbing sets c)
    runner = kdist.ShardedBinner(K, M, cutoff, L, device=local, group=None,
                                 transport=os.environ.get("KB_ROUTED_TRANSPORT") or None)
    eng = runner.engine
    pending = []  # pipelined: the next unit, already scattered, its records in flight

    def send(p, off=0):
        w, ln = reads(off)
        return runner.send(w, ln, n, wpr, first_id=rank * n, part=p, n_parts=P)

    def step(digest=False):
        pass_log.clear()
        dig = [0, 0, 0, 0]
        for p in range(P):
            if pipeline:
                # unit (step, pass p): its records were sent with the last
                # unit (or now, at the start); the next unit's -- the next
                # pass, or the next step's first -- go out before it is binned
                unit = pending.pop() if pending else send(p)
                pending.append(send((p + 1) % P, 1 if p + 1 == P else 0))
                runner.receive(unit)
            else:
                w, ln = reads()
                runner.step(w, ln, n, wpr, first_id=rank * n, part=p, n_parts=P)
            pass_log.append((eng.export_device() if P > 1 else None, eng.timing_raw(), runner.last_times,
                             runner.last_counts))
            if digest:
                dig = [(a + b) % (1 << 64) for a, b in zip(dig, eng.digest())]
        if cur is not None:
            cur[0] += 1
        return dig

    def drain():
        # no unit crosses into the timed region: the timed steps send their
        # own first unit (and one last prefetch goes unused -- counted in)
        while pending:
            runner.discard(pending.pop())

    return runner, eng, step, drain


def multi_capacity_leg(name, rank, world, local, dist, backend, steps=2, warmup=1, scale=1):
    """N > 1: one of BASELINE's multi-GPU configurations AS SPECIFIED (SURVEY
    8(d)): C4 -- 125 M x 150 bp reads per rank (1 B over 8 GPUs) of ONE
    3.1-Gbp genome, K31 M7, P = 5 passes; C5 -- 62.5 M x 250 bp per rank, 1 %
    errors, K63 M7, P = 4 -- routed by owner(mmer) over the C group (RCCL
    all-to-all from C) and binned by the owners.  ms per step (max over
    ranks), whole-job k-mers/s, the bin phase's roofline, and the exchange:
    the records this rank sent to its peers per step and their rate per peer
    link (xGMI is point-to-point: one link per peer).  scale > 1 divides the
    reads (a rehearsal of the plumbing, e.g. gloo ranks sharing one GPU)."""
    wl = WORKLOADS[name]
    n, L, K, M, P = wl["reads"] // scale, wl["read_len"], wl["K"], wl["M"], wl["parts"]
    wpr = (L + 31) // 32
    w = torch.empty(n * wpr, dtype=torch.int64, device="cuda")
    ln = torch.empty(n, dtype=torch.int32, device="cuda")
    kbin.generate_reads_device(w.data_ptr(), ln.data_ptr(), n, L, wl["genome"], wl["err_ppm"],
                               gen_seed(wl["seed"]), device=local, read_base=rank * n)
    torch.cuda.synchronize()
    pass_log = []
    runner, eng, step, drain = routed_runner(K, M, L, 1, n, wpr, P, local, rank, lambda off=0: (w, ln), pass_log)
    eng.set_timing(True)

    def barrier():
        dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x):
        tt = torch.tensor([x], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    barrier()
    tc = time.perf_counter()
    step()
    barrier()
    cold_ms = max_over_ranks((time.perf_counter() - tc) * 1e3)
    for _ in range(warmup):
        step()
    drain()
    barrier()
    t0 = time.perf_counter()
    log, sent = [], []
    for _ in range(steps):
        step()
        log.extend((d if d is not None else eng.export_device(), kbin.timing_dict(t)) for d, t, _, _ in pass_log)
        # records this rank sent to each peer this step (its row of every pass's counts)
        row = np.zeros(world, dtype=np.float64)
        for _, _, _, c in pass_log:
            if c is not None:
                row += np.asarray(c[0], dtype=np.float64)
        sent.append(row)
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    drain()
    dt = elapsed / steps
    kmers = n * (L - K + 1) * world
    rec_bytes = runner.rec_words * 8
    row = np.mean(sent, axis=0)
    off_rank = float(row.sum() - row[rank]) * rec_bytes
    phases = {k: round(float(sum(t[k] for _, t in log)) / steps, 3)
              for k in ("scan_insert_ms", "sort_ms", "runs_ms", "emit_ms", "total_ms")}
    route = pass_log[-1][2] if pass_log else {}
    out = {"workload": f"{wl['name'].split(' ')[0]} as specified: {n * world} x {L}bp reads over {world} GPUs "
                       f"({n} per GPU), genome {wl['genome']} bp, {wl['err_ppm'] / 1e4:.2f}% substitutions, "
                       f"seed {wl['seed']}, K={K} M={M}, prune cutoff 1, {P} mmer-partitioned passes, "
                       f"mmer-sharded (owner(mmer)), records routed over the group",
           "value": round(kmers / dt, 1), "unit": "k-mers/s", "ms_per_step": round(dt * 1e3, 3), "steps": steps,
           "cold_first_step_ms": round(cold_ms, 1),
           "roofline": roofline(log, L, K, world, kmers / dt, f"n{n}_L{L}_K{K}_M{M}_P{P}"),
           "phases_ms_rank0": phases,
           "exchange": {"bytes_sent_off_rank_per_step": int(off_rank), "record_bytes": rec_bytes,
                        "peer_links": world - 1,
                        "per_link_GBps_over_step": round(off_rank / max(1, world - 1) / dt / 1e9, 3),
                        "route_ms_last_pass": {k: round(float(v), 3) for k, v in route.items()}
                        if isinstance(route, dict) else route}}
    if scale > 1:
        out["rehearsal_scale"] = scale
    del runner, eng, step, w, ln
    torch.cuda.empty_cache()
    return out


def main():
    # stdout carries exactly ONE JSON line (rank 0): native libraries print to
    # fd 1 (RCCL's version banner, gloo's connection notes), so fd 1 points at
    # stderr for the run and the result goes to a private copy of the real stdout
    result_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2",
                    help="SURVEY §8(d) configuration (c2: the headline 1M x 150 bp; c3: "
                         "100M x 150 bp on one GPU in mmer-partitioned passes; c4/c5: the "
                         "per-GPU shares of the 8-GPU configurations)")
    ap.add_argument("--reads", type=int, default=None, help="reads per GPU")
    ap.add_argument("--read-len", type=int, default=None)
    ap.add_argument("--K", type=int, default=None)
    ap.add_argument("--M", type=int, default=None)
    ap.add_argument("--cutoff", type=int, default=1)
    ap.add_argument("--genome", type=int, default=None)
    ap.add_argument("--err-ppm", type=int, default=None)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--parts", type=int, default=None,
                    help="mmer partitions (kb_set_partition passes) per step")
    ap.add_argument("--digest", action="store_true",
                    help="after timing, one more step reporting kb_digest summed over the passes")
    ap.add_argument("--cpu-sample", type=int, default=300_000,
                    help="reads timed on the CPU oracle (0 = skip)")
    ap.add_argument("--ref-sample", type=int, default=120_000,
                    help="reads timed on the compiled reference (oracle/_ref; 0 = port only)")
    ap.add_argument("--input", choices=("auto", "fresh", "replay"), default="auto",
                    help="fresh: every step bins new reads of the same genome (all sets generated before "
                         "timing); replay: the same reads every step; auto: fresh when the sets fit in "
                         "5%% of the HBM")
    ap.add_argument("--host-input", dest="host_input", action="store_true", default=True,
                    help=argparse.SUPPRESS)  # (the host leg is on by default; kept for older command lines)
    ap.add_argument("--no-host-input", dest="host_input", action="store_false",
                    help="N=1: skip the host-ingest leg (kb_submit of host ASCII, finalize, kb_export, "
                         "H2D and D2H reported separately; on by default)")
    ap.add_argument("--no-capacity", dest="capacity", action="store_false",
                    help="N=1: skip the C3 capacity leg (100M x 150 bp in 4 passes, digest-checked; on by "
                         "default)")
    ap.add_argument("--multi-legs", action="store_true",
                    help="N=1 with --routed: run the N > 1 run's C4 and C5 legs through the one-rank group "
                         "(a full-size rehearsal of their memory and time)")
    ap.add_argument("--dropin", action="store_true",
                    help="N=1: also time the reference surface (kbin_main: fgets + process_read loop, "
                         "prune_data with materialised zhash tables) on the workload's reads")
    ap.add_argument("--no-scan-once", action="store_true",
                    help="P>1 on one GPU: every pass rescans the reads (kb_set_partition) instead of "
                         "one kb_split_passes scan into the passes' regions")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="N>1: no overlap of the next unit's record exchange with this unit's binning")
    ap.add_argument("--timing-all", action="store_true",
                    help="every phase event in the timed steps too (by default light-bin workloads record only "
                         "bin_kernel's two events there)")
    ap.add_argument("--routed", action="store_true",
                    help="N=1 through the multi-GPU path (route, all-to-all over a 1-rank group, "
                         "receive): measures the routing overhead on one GPU")
    args = ap.parse_args()
    wl = WORKLOADS[args.workload]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    genome_given = args.genome is not None
    for k in ("reads", "genome", "seed", "parts", "read_len", "K", "M", "err_ppm"):
        if getattr(args, k) is None:
            setattr(args, k, wl[k])
    if args.workload == "c2" and not genome_given:
        # weak scaling of the headline: N ranks bin N x 1M reads of ONE genome of
        # N x 5 Mbp -- per GPU the same reads, coverage (30x) and owned key count
        # as C2; C4/C5 keep their fixed 3.1-Gbp genome
        args.genome *= world

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    # one rank per GPU; KB_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs
    backend = os.environ.get("KB_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    local = local % ndev if backend == "gloo" else local
    torch.cuda.set_device(local)
    dist = None
    if args.routed and world == 1:
        import socket
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if world > 1 or args.routed:
        import torch.distributed as tdist
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            tdist.init_process_group(backend)
        dist = tdist

    L, K, M = args.read_len, args.K, args.M
    wpr = (L + 31) // 32
    n = args.reads
    # ONE genome per workload (seeded by the workload seed), one read stream:
    # rank r holds reads [r n, (r + 1) n) of it (kb_generate_reads_device_at),
    # so the N-rank job bins the first N n reads of that genome -- C4's shape
    # (1B reads of one 3.1-Gbp genome split by id range); every
    # rank owns 1/N of the canonical mmers and receives its keys from all ranks.
    # Fresh input: step i bins the i-th such batch of the same stream
    # (reads [(i N + r) n, (i N + r + 1) n)), every set generated and resident
    # before the timed region; replay: set 0 every step.
    set_bytes = n * wpr * 8 + n * 4
    n_sets = args.warmup + args.steps + 1
    hbm = torch.cuda.get_device_properties(local).total_memory
    fresh = args.input == "fresh" or (args.input == "auto" and n_sets * set_bytes <= 0.05 * hbm)
    if not fresh:
        n_sets = 1
    sets = []
    for i in range(n_sets):
        w_i = torch.empty(n * wpr, dtype=torch.int64, device="cuda")
        l_i = torch.empty(n, dtype=torch.int32, device="cuda")
        kbin.generate_reads_device(w_i.data_ptr(), l_i.data_ptr(), n, L, args.genome, args.err_ppm,
                                   gen_seed(args.seed), device=local, read_base=(i * world + rank) * n)
        sets.append((w_i, l_i))
    torch.cuda.synchronize()
    cur = [0]  # the set the next step bins
    pinned = [False]  # replay leg and digest: set 0 every step

    def reads(off=0):
        return sets[0] if pinned[0] else sets[(cur[0] + off) % n_sets]

    P = args.parts
    pass_log = []  # (export_device, timing[, route times]) of every pass of the last step
    if world > 1 or args.routed:
        runner, eng, step, drain = routed_runner(K, M, L, args.cutoff, n, wpr, P, local, rank, reads, pass_log,
                                                 not args.no_pipeline, cur)
    else:
        eng, step = single_gpu_runner(K, M, L, args.cutoff, n, wpr, P, local, reads, pass_log,
                                      scan_once=not args.no_scan_once)

        def drain():
            pass

    if world == 1 and not args.routed:
        _step1 = step

        def step(digest=False):
            d = _step1(digest)
            cur[0] += 1
            return d

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    eng.set_timing(True)
    cold_ms = None
    for i in range(args.warmup):
        if i == 0:  # the first step of fresh contexts: nothing learned yet
            barrier()
            tc = time.perf_counter()
            step()
            barrier()
            cold_ms = (time.perf_counter() - tc) * 1e3
        else:
            step()
    drain()
    # Every phase event idles the GPU for ~5 us (seven per finalize: ~35 us of
    # a 2-ms C2 step).  Where bin_kernel is the bin phase (light bins) the
    # timed steps record only its two events (the roofline's kernel time) and
    # the phases come from one more step after them; heavy-bin workloads keep
    # every event (their roofline kernel is the whole bin phase)
    phase_log = [(d, kbin.timing_dict(t)) for d, t, *_ in pass_log] if args.warmup else []
    light = bool(phase_log) and not args.timing_all and all(int(t["engine"]) == kbin.KB_ENG_BINNED and t["bin_kernel_ms"] > 0
                                    and t["bin_kernel_ms"] >= 0.5 * t["runs_ms"] for _, t in phase_log)
    if dist is not None:  # (every rank takes the same branch: the phase step runs collectives)
        lt = torch.tensor([1 if light else 0], dtype=torch.int32, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(lt, op=dist.ReduceOp.MIN)
        light = bool(lt.item())
    if light:
        eng.set_timing("kernel")

    steps_log = []  # per step: [(export_device, timing)] of each finalize (pass)
    barrier()
    t0 = time.perf_counter()
    route_t = []
    for _ in range(args.steps):
        step()
        steps_log.append([(d, t) for d, t, *_ in pass_log])  # (converted after the timed steps)
        if world > 1 or args.routed:
            rts = [r for _, _, r, *_ in pass_log]
            route_t.append({k: sum(r[k] for r in rts) for k in rts[0]})
    barrier()
    elapsed = time.perf_counter() - t0
    drain()
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64,
                          device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    # the Python side of the timed steps kept raw structs: convert them now, and
    # read a one-pass step's export (the same shape every step) from the last
    ex_last = eng.export_device()
    if light:  # the phases: one untimed step with every phase event
        eng.set_timing(True)
        step()
        drain()
        phase_log = [(d, kbin.timing_dict(t)) for d, t, *_ in pass_log]
        eng.set_timing("kernel")
    steps_log = [[(d if d is not None else ex_last, kbin.timing_dict(t)) for d, t in st] for st in steps_log]
    last = steps_log[-1]  # the passes of the last step, added up
    dev = {k: sum(int(d[k]) for d, _ in last) for k in ("n_kmers", "n_entries", "n_ids", "n_distinct")}
    n_kmers = dev["n_kmers"]               # occurrences this rank inserted (owned)
    scanned = n * max(0, L - K + 1)         # occurrences this rank scanned
    total_scanned = scanned * world
    value = total_scanned * args.steps / elapsed

    passes = [pt for st in steps_log for pt in st]
    tim = [t for _, t in passes]
    tag = f"n{n}_L{L}_K{K}_M{M}" + (f"_P{args.parts}" if args.parts > 1 else "")
    roof = roofline(passes, L, K, world, total_scanned * args.steps / elapsed, tag)
    # device time per step (all passes of a step added up): the timed steps',
    # or -- timed with bin_kernel's events only -- the last warmup step's
    phases = {k: round(float(np.mean([sum(t[k] for _, t in st) for st in ([phase_log] if light else steps_log)])), 4)
              for k in ("scan_insert_ms", "sort_ms", "runs_ms", "emit_ms", "total_ms")}
    phases["source"] = "one untimed step after the timed ones (all phase events)" if light else "timed steps"
    replay = None
    if fresh and args.steps:
        # the same number of steps replaying one set (round 1's headline mode)
        drain()
        barrier()
        tr = time.perf_counter()
        pinned[0] = True
        for _ in range(args.steps):
            step()
        barrier()
        t_rep = time.perf_counter() - tr
        drain()
        if dist is not None:
            tt = torch.tensor([t_rep], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            t_rep = float(tt.item())
        replay = {"value": round(total_scanned * args.steps / t_rep, 1),
                  "ms_per_step": round(t_rep / args.steps * 1e3, 4)}
    digest = None
    if args.digest:  # this rank's share of set 0 (ranks own disjoint mmers: shares add up)
        drain()
        pinned[0] = True
        digest = [hex(x) for x in step(digest=True)]
        drain()

    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "k-mers/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
        "config": {"workload": f"{WORKLOADS[args.workload]['name']}: {n} x {L}bp reads per GPU, genome {args.genome} bp, "
                               f"{args.err_ppm / 1e4:.2f}% substitutions, seed {args.seed}, "
                               f"K={K} M={M}, prune cutoff {args.cutoff}",
                   "reads_per_gpu": n, "read_len": L, "K": K, "M": M, "cutoff": args.cutoff,
                   "genome_len": args.genome, "err_ppm": args.err_ppm,
                   **({"mmer_partitions": args.parts} if args.parts > 1 else {}),
                   "parallelism": (f"mmer-sharded x{world}" if world > 1 else
                                   ("single GPU, routed path" if args.routed else "single GPU"))
                                  + (", pipelined exchange" if (world > 1 or args.routed)
                                     and not args.no_pipeline else "")},
        "input": {"mode": "fresh" if fresh else "replay",
                  "note": ("every step bins the next n reads of the same genome, all sets resident before "
                           "the timed region" if fresh else "every step re-bins the same resident reads"),
                  "cold_first_step_ms": None if cold_ms is None else round(cold_ms, 3),
                  **({"replay": replay} if replay else {})},
        "roofline": roof,
        "phases_ms": phases,
        "paths": path_counters(steps_log[-1]),
        **({"route_ms": {k: round(float(np.mean([r[k] for r in route_t])), 4) for k in route_t[0]}}
           if route_t else {}),
        "result": {**({"digest": digest} if digest else {}),
                   "entries": int(dev["n_entries"]), "ids": int(dev["n_ids"]),
                   "distinct": int(dev["n_distinct"]), "kmers_owned": n_kmers,
                   "table_slots": int(tim[-1]["table_slots"]),
                   "engine": {1: "table", 2: "binned"}.get(int(tim[-1]["engine"]), "?"),
                   "bins": int(tim[-1]["n_bins"]), "superkmers": int(tim[-1]["n_superkmers"])},
    }
    legs = (world > 1 or (args.routed and args.multi_legs)) and args.capacity and args.workload == "c2"
    if legs:
        # BASELINE's multi-GPU configurations as specified (the headline stays
        # C2 weak scaling: the same per-GPU work at every N); the main leg's
        # contexts and read sets go first
        del runner, eng, step, sets
        torch.cuda.empty_cache()
        scale = max(1, int(os.environ.get("KB_CAPACITY_SCALE", "1")))
        out["capacity"] = {}
        for name in ("c4", "c5"):
            out["capacity"][name] = multi_capacity_leg(name, rank, world, local, dist, backend, scale=scale)
            if rank == 0:
                print(json.dumps({name: out["capacity"][name]}), file=sys.stderr, flush=True)
    if world == 1 and args.host_input and P == 1 and not legs:
        out["host_input"] = host_input_leg(sets[0][0], sets[0][1], n, wpr, L, K, M, args.cutoff, local)
    if world == 1 and args.capacity and args.workload == "c2" and not args.routed:
        out["capacity"] = capacity_leg(local)
    if rank == 0 and world == 1 and args.dropin and P == 1 and not legs:
        out["dropin"] = dropin_leg(sets[0][0], sets[0][1], n, wpr, L, K, M, args.cutoff, local)
    if rank == 0 and world == 1 and args.cpu_sample > 0 and not legs:
        out["cpu_baseline"] = cpu_baseline(sets[0][0], sets[0][1], n, min(args.cpu_sample, n), wpr, L, K, M,
                                           args.cutoff, args.ref_sample)
    if rank == 0:
        print(json.dumps(out), file=result_out, flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
