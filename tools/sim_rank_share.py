"""What one rank of the N-GPU C2 weak-scaling run bins, measured on one GPU.

bench.py --gpus N gives rank r the reads [(i N + r) n, (i N + r + 1) n) of one
genome of N x 5 Mbp and routes every super-k-mer to owner(mmer): each rank
then bins 1/N of the mmers of N n reads -- the same k-mer count as C2 at
N = 1, but N-times larger mmer bins (the genome is N times longer).  This
script routes the N shards (kb_route_scatter, each rank's sender), then bins
what the most and the least loaded rank receive alone on the GPU, a few times so the
bucket maps are learned, and prints the finalize phases (kb timing) -- the
per-rank compute of the driver's N-GPU run, without the peer traffic and
without other ranks sharing the GPU.

    python tools/sim_rank_share.py --ranks 1 2 4 8 --steps 3
"""
import argparse
import json
import pathlib
import sys
import time

REPO = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "genome-assembly_amd"))
sys.path.insert(0, str(REPO))


def main():
    import torch
    import kbin
    import bench
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--reads", type=int, default=1_000_000)
    a = ap.parse_args()
    wl = bench.WORKLOADS["c2"]
    n, L, K, M = a.reads, wl["read_len"], wl["K"], wl["M"]
    wpr = (L + 31) // 32
    seed = bench.gen_seed(wl["seed"])
    for G in a.ranks:
        genome = wl["genome"] * G
        sets = []
        for r in range(G):
            w = torch.empty(n * wpr, dtype=torch.int64, device="cuda")
            ln = torch.empty(n, dtype=torch.int32, device="cuda")
            kbin.generate_reads_device(w.data_ptr(), ln.data_ptr(), n, L, genome, wl["err_ppm"], seed,
                                       read_base=r * n)
            sets.append((w, ln))
        torch.cuda.synchronize()
        rows = []
        # route every shard (kb_route_scatter, as each rank's sender does)
        rw = 3
        cap = n * 12 // G + 65536
        regions, counts = [], []
        for r, (w, ln) in enumerate(sets):
            reg = torch.empty(G * cap * rw, dtype=torch.int64, device="cuda")
            with kbin.Engine(K, M, cutoff=1, max_read_len=L) as snd:
                snd.submit_packed_device(w.data_ptr(), ln.data_ptr(), n, wpr, first_id=r * n)
                ok, cnt = snd.route_scatter(G, reg.data_ptr(), cap)
                assert ok
            regions.append(reg)
            counts.append([int(c) for c in cnt])
        torch.cuda.synchronize()
        del sets
        per_dest = [sum(c[d] for c in counts) for d in range(G)]
        heavy = max(range(G), key=lambda d: per_dest[d])
        light = min(range(G), key=lambda d: per_dest[d])
        for d in sorted({light, heavy}):
            # what rank d receives, concatenated by source rank, binned alone
            recv = torch.cat([regions[r][d * cap * rw:(d * cap + counts[r][d]) * rw] for r in range(G)])
            nrec = sum(c[d] for c in counts)
            with kbin.Engine(K, M, cutoff=1, max_read_len=L) as own:
                own.set_timing(True)
                for s in range(a.steps):
                    own.reset()
                    own.submit_superkmers_device(recv.data_ptr(), nrec)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    own.finalize(True)
                    torch.cuda.synchronize()
                    t = own.timing()
                    rows.append({"rank": d, "step": s, "records": nrec,
                                 "finalize_ms": round((time.perf_counter() - t0) * 1e3, 3),
                                 "total_ms": round(t["total_ms"], 3), "scan_ms": round(t["scan_insert_ms"], 3),
                                 "bin_ms": round(t["runs_ms"], 3), "bin_kernel_ms": round(t["bin_kernel_ms"], 3),
                                 "bins": int(t["n_bins"]), "heavy": int(t["heavy_bins"]),
                                 "flat": int(t["flat_partitions"]), "split": int(t["split_bins"])})
            del recv
        print(json.dumps({"ranks": G, "genome": genome, "reads_per_rank": n, "records_per_rank": per_dest,
                          "max_over_mean": round(max(per_dest) * G / max(1, sum(per_dest)), 4), "rows": rows}),
              flush=True)
        del regions
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
