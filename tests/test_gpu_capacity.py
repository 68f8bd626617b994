"""Parity in the CAPACITY regimes at default knobs,
with the engine's path counters (kb_timing) asserting that the paths those
configurations run were actually taken:

  C3  coverage ~3000x (the C3 generator, 0.1 % errors, on a genome shrunk so
      1M-4M reads reach C3's depth): long read-id lists (> 256 ids), heavy
      bins with flat per-partition lists, offset partitions, table-overflow
      redos -- checked against the oracle restricted to one mmer partition
      (kbo_bin_masked), including a kb_set_partition pass of P = 8;
  C5  the C5 generator (250 bp, K63 M7, 1 % errors): heavy bins and, on the
      context's second pass, the singleton pre-filter (its "learned from the
      last finalize" switch), pre-filtered keys > 0 asserted, bit-exact;
  C4  the C4 generator's read ranges of G = 8 ranks routed by owner(mmer)
      (kb_route_scatter), the union of the 8 receivers against the oracle.

The reference semantics these pin: binning.c:1042-1069 (insert / prepend,
duplicates kept) and 1085-1123 (prune at the cutoff)."""
import numpy as np
import pytest

import bench
import kbin
import kbin.dist
import oracle
from test_gpu_parity import assert_same
from test_gpu_scale import _generate, _unpack

pytestmark = [pytest.mark.gpu]

PART_SALT = 0x9E3779B97F4A7C15  # kbin_bins.hip in_part (kb_set_partition)


def part_mask(M, part, n_parts):
    """uint8 per canonical mmer code: 1 if in_part(m, part, n_parts)"""
    m = np.arange(1 << (2 * M), dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = kbin._mix64_np(m + np.uint64(PART_SALT)) >> np.uint64(32)
    return (h % np.uint64(n_parts) == np.uint64(part)).astype(np.uint8)


def subset(res, mask):
    """the entries of a result whose mmer is in mask"""
    keep = mask[res.mmer.astype(np.int64)].astype(bool)
    idx = np.flatnonzero(keep)
    cnt = res.count[idx]
    off = np.zeros(len(idx) + 1, dtype=np.uint64)
    np.cumsum(cnt, out=off[1:])
    starts = res.offset[:-1][idx].astype(np.int64)
    take = np.repeat(starts - off[:-1].astype(np.int64), cnt.astype(np.int64)) + \
        np.arange(int(off[-1]), dtype=np.int64)
    return kbin.Result(res.mmer[idx], res.kmer_hi[idx], res.kmer_lo[idx], cnt, off, res.ids[take],
                       res.n_kmers, res.n_distinct)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("n,genome,P,p", [(1_000_000, 50_000, 1, 0), (4_000_000, 200_000, 8, 3)])
def test_c3_coverage_regime(n, genome, P, p):
    """C3's generator at ~3000x coverage: one pass (the whole input, or
    partition p of P via kb_set_partition) at default knobs takes the long-list,
    heavy/flat, offset-partition and overflow paths; the pass's mmers (a
    partition of 2 for the P = 1 case, to keep the oracle quick) are bit-exact
    against the oracle filtered to the same mmers"""
    wl = bench.WORKLOADS["c3"]
    L, K, M = wl["read_len"], wl["K"], wl["M"]
    words, lens, wpr = _generate(n, L, genome, wl["err_ppm"], bench.gen_seed(wl["seed"]))
    with kbin.Engine(K, M, cutoff=1, max_read_len=L) as eng:
        eng.set_timing(True)
        eng.submit_packed_device(words.data_ptr(), lens.data_ptr(), n, wpr, 0)
        if P > 1:
            eng.set_partition(p, P)
        eng.finalize(True)
        t = eng.timing()
        res = eng.export()
    assert t["engine"] == kbin.KB_ENG_BINNED
    assert t["long_lists"] > 1000, t           # lists of > 256 ids (C3: 5.2M per step)
    assert t["offset_partitions"] > 0, t
    assert t["overflow_redos"] > 0, t
    assert t["heavy_bins"] > 0 and t["flat_partitions"] > 0, t
    mask = part_mask(M, p, P) if P > 1 else part_mask(M, 0, 2)
    bases, hl = _unpack(words, lens, n, wpr, L)
    ora = oracle.bin_reads(bases, hl, K, M, 1, True, mmer_mask=mask)
    assert ora.n_kmers == n * (L - K + 1)
    got = subset(res, mask) if P == 1 else res
    assert got.n_entries > 10_000
    assert int(got.count.max()) > 1000  # C3-depth lists really are in the checked part
    assert_same(got, ora)


@pytest.mark.timeout(1200)
def test_c3_repeated_finalizes_default_knobs():
    """the path C3 really runs -- ranking switched on by
    the LAST finalize's mean list length (>= 64 ids), the sticky long-list
    regime's finer sub-bins from the maps learned on it, bitmap emission with
    KB_BIN_RANK_MERGE -- at default knobs over repeated finalizes of one
    context: partition 3 of 8 of the C3 generator at ~3000x coverage (4 M reads
    over 200 Kbp), finalized three times (cold; then ranked, on learned maps),
    each bit-exact against the oracle on the same mmers, the later two
    asserted ranked and bitmap-emitted"""
    wl = bench.WORKLOADS["c3"]
    n, genome, P, p = 4_000_000, 200_000, 8, 3
    L, K, M = wl["read_len"], wl["K"], wl["M"]
    words, lens, wpr = _generate(n, L, genome, wl["err_ppm"], bench.gen_seed(wl["seed"]))
    mask = part_mask(M, p, P)
    bases, hl = _unpack(words, lens, n, wpr, L)
    ora = oracle.bin_reads(bases, hl, K, M, 1, True, mmer_mask=mask)
    del bases
    tim = []
    with kbin.Engine(K, M, cutoff=1, max_read_len=L) as eng:
        eng.set_timing(True)
        for f in range(3):
            eng.reset()
            eng.submit_packed_device(words.data_ptr(), lens.data_ptr(), n, wpr, 0)
            eng.set_partition(p, P)
            eng.finalize(True)
            tim.append(eng.timing())
            assert_same(eng.export(), ora)
    assert tim[0]["ranked_bins"] == 0, tim[0]  # (no last finalize to learn from)
    for t in tim[1:]:
        assert t["ranked_bins"] > 100 and t["bitmap_partitions"] > 100, t


_C5_ORACLE = {}  # (n, p, P) -> the oracle's partition result: both variants bin the same reads


@pytest.mark.timeout(900)
@pytest.mark.parametrize("light", ["1", "0"])
def test_c5_singleton_prefilter_default_knobs(light, monkeypatch):
    """the C5 generator (L250, K63 M7, 1 % errors): pass 0 of 2 learns the
    singleton ratio, pass 1 runs with the pre-filter (default knobs): its
    would-be heavy bins stay light behind a per-bin sketch (KB_BIN_PF_LIGHT=1,
    the default) or take the pre-filtered flat lists (0); both passes
    bit-exact against the oracle on their partitions"""
    monkeypatch.setenv("KB_BIN_PF_LIGHT", light)
    wl = bench.WORKLOADS["c5"]
    n, L, K, M, P = 2_000_000, wl["read_len"], wl["K"], wl["M"], 2
    words, lens, wpr = _generate(n, L, wl["genome"], wl["err_ppm"], bench.gen_seed(wl["seed"]))
    out, tim = [], []
    with kbin.Engine(K, M, cutoff=1, max_read_len=L) as eng:
        eng.set_timing(True)
        eng.submit_packed_device(words.data_ptr(), lens.data_ptr(), n, wpr, 0)
        for p in range(P):
            eng.set_partition(p, P)
            eng.finalize(True)
            tim.append(eng.timing())
            out.append(eng.export())
    assert tim[0]["heavy_bins"] > 0, tim
    assert tim[1]["prefiltered"] > 0, tim[1]
    if light == "1":
        assert tim[1]["light_prefilter_bins"] > 0, tim[1]
    else:
        assert tim[1]["heavy_bins"] > 0 and tim[1]["light_prefilter_bins"] == 0, tim[1]
    bases, hl = _unpack(words, lens, n, wpr, L)
    for p in range(P):
        if (n, p, P) not in _C5_ORACLE:
            _C5_ORACLE[(n, p, P)] = oracle.bin_reads(bases, hl, K, M, 1, True, mmer_mask=part_mask(M, p, P))
        assert_same(out[p], _C5_ORACLE[(n, p, P)])
    if light == "0":  # (the last variant: free the cached results)
        _C5_ORACLE.clear()


@pytest.mark.timeout(600)
def test_c4_eight_ranks_routed():
    """C4's shape at G = 8: eight ranks' consecutive read ranges of one
    3.1-Gbp genome, each routed to owner(mmer) by kb_route_scatter, each owner
    binning what it receives; the union equals the oracle"""
    import torch
    wl = bench.WORKLOADS["c4"]
    n, L, G = 40_000, wl["read_len"], 8
    seed = bench.gen_seed(wl["seed"])
    shards = [_generate(n, L, wl["genome"], wl["err_ppm"], seed, read_base=r * n) for r in range(G)]
    rw, cap = 3, n * 4
    regions = [torch.empty(G * cap * rw, dtype=torch.int64, device="cuda") for _ in range(G)]
    counts = []
    for r, (w, ln, wpr) in enumerate(shards):
        with kbin.Engine(31, 7, cutoff=1, max_read_len=L) as snd:
            assert snd.record_words() == rw
            snd.submit_packed_device(w.data_ptr(), ln.data_ptr(), n, wpr, first_id=r * n)
            ok, cnt = snd.route_scatter(G, regions[r].data_ptr(), cap)
            assert ok
            counts.append(cnt)
    torch.cuda.synchronize()
    parts = []
    for d in range(G):
        recv = torch.cat([regions[r][d * cap * rw:(d * cap + int(counts[r][d])) * rw] for r in range(G)])
        with kbin.Engine(31, 7, cutoff=1, max_read_len=L) as own:
            own.submit_superkmers_device(recv.data_ptr(), int(sum(int(c[d]) for c in counts)))
            own.finalize(True)
            parts.append(own.export())
    for d, r in enumerate(parts):
        assert all(kbin.dist.owner_of(int(m), G) == d for m in np.unique(r.mmer))
        assert r.n_entries > 0
    whole, wl_lens, wpr = _generate(G * n, L, wl["genome"], wl["err_ppm"], seed)
    bases, hl = _unpack(whole, wl_lens, G * n, wpr, L)
    ora = oracle.bin_reads(bases, hl, 31, 7, 1, True)
    assert_same(kbin.Result.concat(parts), ora)
