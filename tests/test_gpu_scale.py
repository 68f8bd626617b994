"""Parity at the BASELINE configurations' own workloads (SURVEY.md §8(d):
"Parity for C3-C5 is checked against cpu_ref on a deterministic sub-sample:
the first 1M reads").  Reads come from the bench's device generator with the
bench's seeds (bench.gen_seed), are unpacked to ASCII and binned by the CPU
oracle (oracle/kb_oracle.c, pinned to the compiled reference); the HIP path
runs the same route the bench times:

  C2  1M x 150 bp, K31 M7, seed 2, in full -- one finalize;
  C3  its first 1M reads (seed 3), kb_split_passes into P = 4 passes (the
      bench's scan-once path) and kb_set_partition rescans;
  C4  two ranks' read ranges of ONE 3.1-Gbp genome (seed 4, read_base = r n),
      routed by owner(mmer) with kb_route_scatter, union over the receivers;
  C5  its first 300K reads (L250, K63 M7, 1 % errors, seed 5) in P = 4
      partitioned passes, with and without the prune;
  C2  a 30K-read prefix against the compiled reference binary itself
      (oracle/_ref/ref_k31_m7_c1, built in the build container; skipped where
      it was not built).

Bit-exact on every key, count and read-id list (assert_same), or -- for the
56M-key unpruned C5 result -- on kb_digest against the oracle's digest."""
import hashlib
import subprocess
import tempfile

import numpy as np
import pytest

import bench
import kbin
import kbin.dist
import oracle
from test_gpu_parity import assert_csr, assert_same

pytestmark = [pytest.mark.gpu]


def _generate(n, L, genome, err_ppm, seed, read_base=0):
    import torch
    wpr = (L + 31) // 32
    words = torch.empty(n * wpr, dtype=torch.int64, device="cuda")
    lens = torch.empty(n, dtype=torch.int32, device="cuda")
    kbin.generate_reads_device(words.data_ptr(), lens.data_ptr(), n, L, genome, err_ppm, seed,
                               read_base=read_base)
    torch.cuda.synchronize()
    return words, lens, wpr


def _unpack(words, lens, n, wpr, L):
    bases, hl = kbin.unpack_reads_to_host(words.data_ptr(), lens.data_ptr(), n, wpr, n * L)
    assert (hl == L).all()
    return bases, hl


def _add(a, b):
    return [(x + y) % (1 << 64) for x, y in zip(a, b)]


@pytest.mark.timeout(600)
def test_c2_full_vs_oracle():
    """BASELINE C2 in full: 1M x 150 bp, genome 5 Mbp, 0.1 % errors, K31 M7,
    cutoff 1 -- the bench's headline workload, bit-exact against the oracle"""
    wl = bench.WORKLOADS["c2"]
    n, L = wl["reads"], wl["read_len"]
    words, lens, wpr = _generate(n, L, wl["genome"], wl["err_ppm"], bench.gen_seed(wl["seed"]))
    with kbin.Engine(31, 7, cutoff=1, max_read_len=L) as eng:
        eng.set_timing(True)
        eng.submit_packed_device(words.data_ptr(), lens.data_ptr(), n, wpr, 0)
        eng.finalize(True)
        t = eng.timing()
        dig = eng.digest()
        res = eng.export()
    bases, hl = _unpack(words, lens, n, wpr, L)
    ora = oracle.bin_reads(bases, hl, 31, 7, 1, True)
    assert res.n_kmers == ora.n_kmers == n * (L - 31 + 1)
    assert ora.n_entries > 5_000_000  # the workload really is C2-sized
    assert_same(res, ora)
    assert tuple(dig) == kbin.result_digest(ora)
    # the default path at C2: context sub-bins for the big mmers, offset
    # partitions for the bins still over one table
    assert t["engine"] == kbin.KB_ENG_BINNED
    assert t["split_mmers"] > 100 and t["n_bins"] > 2500, t
    assert t["offset_partitions"] > 0, t


@pytest.mark.timeout(600)
def test_c3_prefix_split_passes():
    """BASELINE C3's first 1M reads (seed 3): the bench's scan-once path
    (kb_split_passes into P = 4 regions, each bound to a partitioned pass) and
    the rescanning kb_set_partition path; both unions equal the oracle"""
    wl = bench.WORKLOADS["c3"]
    n, L, P = 1_000_000, wl["read_len"], wl["parts"]
    words, lens, wpr = _generate(n, L, wl["genome"], wl["err_ppm"], bench.gen_seed(wl["seed"]))
    import torch
    parts, dig = [], [0] * 4
    with kbin.Engine(31, 7, cutoff=1, max_read_len=L) as sender, \
            kbin.Engine(31, 7, cutoff=1, max_read_len=L) as eng:
        rw = eng.record_words()
        sender.submit_packed_device(words.data_ptr(), lens.data_ptr(), n, wpr, 0)
        cap = n * 12 // P + 4096
        regions = torch.empty(P * cap * rw, dtype=torch.int64, device="cuda")
        ok, counts = sender.split_passes(P, regions.data_ptr(), cap)
        assert ok and int(counts.min()) > 0
        for p in range(P):
            eng.reset()
            eng.set_partition(p, P)
            eng.submit_superkmers_device(regions[p * cap * rw:].data_ptr(), int(counts[p]))
            eng.finalize(True)
            parts.append(eng.export())
            dig = _add(dig, eng.digest())
        rescans, dig2 = [], [0] * 4
        eng.reset()
        eng.submit_packed_device(words.data_ptr(), lens.data_ptr(), n, wpr, 0)
        for p in range(P):
            eng.set_partition(p, P)
            eng.finalize(True)
            rescans.append(eng.export())
            dig2 = _add(dig2, eng.digest())
    bases, hl = _unpack(words, lens, n, wpr, L)
    ora = oracle.bin_reads(bases, hl, 31, 7, 1, True)
    want = kbin.result_digest(ora)
    for r in parts + rescans:
        assert_csr(r)
    assert tuple(dig) == want and tuple(dig2) == want
    assert sum(r.n_kmers for r in parts) == ora.n_kmers
    assert_same(kbin.Result.concat(parts), ora)
    assert_same(kbin.Result.concat(rescans), ora)


@pytest.mark.timeout(600)
def test_c4_two_ranks_one_genome():
    """BASELINE C4's shape: ranks hold consecutive read-id ranges of ONE genome
    (kb_generate_reads_device_at, read_base = r n); each rank routes its
    super-k-mers to owner(mmer) (kb_route_scatter), each owner bins what it
    receives; the union equals the oracle on all 2n reads, pruned and not"""
    import torch
    wl = bench.WORKLOADS["c4"]
    n, L, G = 150_000, wl["read_len"], 2
    seed = bench.gen_seed(wl["seed"])
    shards = [_generate(n, L, wl["genome"], wl["err_ppm"], seed, read_base=r * n) for r in range(G)]
    whole, wl_lens, wpr = _generate(G * n, L, wl["genome"], wl["err_ppm"], seed)
    # the ranks' streams are slices of the one stream
    torch.testing.assert_close(torch.cat([s[0] for s in shards]), whole, rtol=0, atol=0)
    bases, hl = _unpack(whole, wl_lens, G * n, wpr, L)
    for prune in (False, True):
        ora = oracle.bin_reads(bases, hl, 31, 7, 1, prune)
        rw = 3
        cap = n * 12
        regions = [torch.empty(G * cap * rw, dtype=torch.int64, device="cuda") for _ in range(G)]
        counts = []
        for r, (w, ln, _) in enumerate(shards):
            with kbin.Engine(31, 7, cutoff=1, max_read_len=L) as snd:
                assert snd.record_words() == rw
                snd.submit_packed_device(w.data_ptr(), ln.data_ptr(), n, wpr, first_id=r * n)
                ok, cnt = snd.route_scatter(G, regions[r].data_ptr(), cap)
                assert ok
                counts.append(cnt)
        torch.cuda.synchronize()
        parts = []
        for d in range(G):
            # what rank d receives: every sender's region d, concatenated by source rank
            recv = torch.cat([regions[r][d * cap * rw:(d * cap + int(counts[r][d])) * rw] for r in range(G)])
            with kbin.Engine(31, 7, cutoff=1, max_read_len=L) as own:
                own.submit_superkmers_device(recv.data_ptr(), int(sum(int(c[d]) for c in counts)))
                own.finalize(prune)
                parts.append(own.export())
        for d, r in enumerate(parts):
            assert all(kbin.dist.owner_of(int(m), G) == d for m in np.unique(r.mmer))
        assert_same(kbin.Result.concat(parts), ora)


@pytest.mark.timeout(900)
def test_c5_prefix_partitioned():
    """BASELINE C5's first 300K reads: 250 bp, K63 M7 (two-word k-mers), 1 %
    substitutions, 3.1-Gbp genome -- nearly every k-mer a singleton.  P = 4
    partitioned passes (the bench's C5 path) pruned: bit-exact; unpruned (the
    ~56M-key table the prune then thins): digest-exact; and the scan-once
    kb_split_passes route pruned: bit-exact"""
    import torch
    wl = bench.WORKLOADS["c5"]
    n, L, P = 300_000, wl["read_len"], wl["parts"]
    words, lens, wpr = _generate(n, L, wl["genome"], wl["err_ppm"], bench.gen_seed(wl["seed"]))
    bases, hl = _unpack(words, lens, n, wpr, L)
    for prune in (True, False):
        ora = oracle.bin_reads(bases, hl, 63, 7, 1, prune)
        parts, dig = [], [0] * 4
        with kbin.Engine(63, 7, cutoff=1, max_read_len=L) as eng:
            eng.set_timing(True)
            eng.submit_packed_device(words.data_ptr(), lens.data_ptr(), n, wpr, 0)
            for p in range(P):
                eng.set_partition(p, P)
                eng.finalize(prune)
                assert eng.timing()["engine"] == kbin.KB_ENG_BINNED
                dig = _add(dig, eng.digest())
                if prune:
                    parts.append(eng.export())
        assert tuple(dig) == kbin.result_digest(ora)
        if prune:
            assert_same(kbin.Result.concat(parts), ora)
            with kbin.Engine(63, 7, cutoff=1, max_read_len=L) as snd, \
                    kbin.Engine(63, 7, cutoff=1, max_read_len=L) as eng:
                rw = eng.record_words()
                snd.submit_packed_device(words.data_ptr(), lens.data_ptr(), n, wpr, 0)
                cap = n * 30 // P + 4096
                regions = torch.empty(P * cap * rw, dtype=torch.int64, device="cuda")
                ok, counts = snd.split_passes(P, regions.data_ptr(), cap)
                assert ok
                split = []
                for p in range(P):
                    eng.reset()
                    eng.set_partition(p, P)
                    eng.submit_superkmers_device(regions[p * cap * rw:].data_ptr(), int(counts[p]))
                    eng.finalize(True)
                    split.append(eng.export())
            assert_same(kbin.Result.concat(split), ora)
        del ora


def test_c2_prefix_vs_reference_binary():
    """the first 30K reads of the C2 workload against the compiled reference
    program itself (oracle/_ref/ref_k31_m7_c1: binning.c + zhash.c + llist.c,
    fgets loop, prune_data, canonical dump): sha256 of the sorted dumps"""
    ref = kbin.REPO_ROOT / "oracle" / "_ref" / "ref_k31_m7_c1"
    if not ref.is_file():
        pytest.skip("reference binary not built (needs /root/reference at build time)")
    wl = bench.WORKLOADS["c2"]
    n, L = 30_000, wl["read_len"]
    words, lens, wpr = _generate(n, L, wl["genome"], wl["err_ppm"], bench.gen_seed(wl["seed"]))
    bases, hl = _unpack(words, lens, n, wpr, L)
    with tempfile.NamedTemporaryFile(suffix=".txt") as f:
        buf = np.frombuffer(bases, dtype=np.uint8).reshape(n, L)
        f.write(np.concatenate([buf, np.full((n, 1), ord("\n"), np.uint8)], axis=1).tobytes())
        f.flush()
        out = subprocess.run([str(ref), f.name, str(L + 2), "1"], check=True, capture_output=True,
                             timeout=300).stdout
    want = hashlib.sha256(b"".join(sorted(out.splitlines(keepends=True)))).hexdigest()
    with kbin.Engine(31, 7, cutoff=1, max_read_len=L) as eng:
        eng.submit_packed_device(words.data_ptr(), lens.data_ptr(), n, wpr, 0)
        eng.finalize(True)
        res = eng.export()
    assert res.n_entries > 1000
    h = hashlib.sha256()
    for line in kbin.dump_lines(res, 31, 7):
        h.update(line.encode())
    assert h.hexdigest() == want


@pytest.mark.parametrize("wl_name,read_base", [("c2", 0), ("c3", 0), ("c3", 99_950_000), ("c4", 875_000_000),
                                               ("c5", 62_450_000)])
def test_generator_twin(wl_name, read_base):
    """the oracle's CPU twin of the device generator
    (oracle.gen_reads, kb_oracle.c kbo_gen_reads) gives the same reads as
    kb_generate_reads_device_at -- at the start of each workload's stream and
    at its far end (C3's last reads, C4 rank 7's range, C5's last share reads)
    -- so the oracle-computed full-size digests (tests/golden/
    oracle_digests.json) are of the bench's own reads"""
    wl = bench.WORKLOADS[wl_name]
    n, L = 20_000, wl["read_len"]
    seed = bench.gen_seed(wl["seed"])
    words, lens, wpr = _generate(n, L, wl["genome"], wl["err_ppm"], seed, read_base=read_base)
    bases, _ = _unpack(words, lens, n, wpr, L)
    assert oracle.gen_reads(n, L, wl["genome"], wl["err_ppm"], seed, read_base) == bases


@pytest.mark.timeout(600)
def test_c2_full_oracle_digest():
    """C2 in full against the oracle-computed digest fixture (tools/
    oracle_digest.py c2): the same check bench.py's C3 leg makes, on a size
    the fixture script computes in 30 s"""
    import json
    fx = json.loads((bench.REPO / "tests" / "golden" / "oracle_digests.json").read_text())["c2"]
    wl = bench.WORKLOADS["c2"]
    n, L = wl["reads"], wl["read_len"]
    assert fx["reads"] == n and fx["seed"] == bench.gen_seed(wl["seed"])
    words, lens, wpr = _generate(n, L, wl["genome"], wl["err_ppm"], fx["seed"])
    with kbin.Engine(wl["K"], wl["M"], cutoff=1, max_read_len=L) as eng:
        eng.submit_packed_device(words.data_ptr(), lens.data_ptr(), n, wpr, 0)
        eng.finalize(True)
        dig = [hex(x) for x in eng.digest()]
    assert dig == fx["digest"]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("wl_name", ["c4", "c5"])
def test_c4_c5_prefix_oracle_digest(wl_name):
    """VERDICT r05 weak #6 (full-size C4 / C5 parity was GPU-only): the first
    4 M reads of the C4 and C5 share streams (480 M and 752 M k-mers, 13x and
    2x the largest earlier oracle checks of these configurations) binned by
    bench.py itself -- P mmer-partitioned passes, the one-scan split path --
    and its digest summed over the passes equal to the CPU oracle's
    (tools/oracle_digest.py c4|c5 --reads 4000000: 146 s / 243 s on 8 cores)"""
    import json
    import os
    import sys
    fx = json.loads((bench.REPO / "tests" / "golden" / "oracle_digests.json").read_text())[f"{wl_name}_prefix4000000"]
    wl = bench.WORKLOADS[wl_name]
    assert fx["seed"] == bench.gen_seed(wl["seed"]) and fx["K"] == wl["K"] and fx["read_len"] == wl["read_len"]
    env = dict(os.environ)
    env.pop("KB_ENGINE", None)
    r = subprocess.run([sys.executable, str(bench.REPO / "bench.py"), "--workload", wl_name, "--reads", str(fx["reads"]),
                        "--steps", "1", "--warmup", "0", "--digest", "--cpu-sample", "0", "--no-host-input"],
                       capture_output=True, text=True, env=env, timeout=540)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["result"]["kmers_owned"] == fx["kmers"]
    assert line["result"]["digest"] == fx["digest"]
