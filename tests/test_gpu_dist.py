"""GPU side of the multi-GPU path on ONE device with G virtual shards
(SURVEY §4.5): the HIP route kernels pack exactly the records of the format
restatement (tests/skmer_ref.py), every shard bins its records through the
receiver kernels, and the union of the shards equals the oracle."""
import numpy as np
import pytest
import torch

import kbin
import kbin.dist
import oracle
import skmer_ref
from conftest import GOLDEN

# every case runs on both engines (conftest.engine), senders and receivers alike
pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("engine")]


def _reads(n=700, rl=102):
    bases, lens = oracle.read_fgets(GOLDEN / "reads.txt", rl)
    off = np.concatenate([[0], np.cumsum(lens.astype(np.int64))]).astype(np.int64)
    rng = np.random.default_rng(3)
    extra = [rng.choice(np.frombuffer(b"ACGT", np.uint8), int(rng.integers(0, 200))).tobytes()
             for _ in range(100)] + [b"A" * 120, b"ACGT" * 40, b""]
    reads = [bases[off[i]:off[i + 1]] for i in range(n)] + extra
    return reads


def _result_dict(res):
    c = res.canonical()
    out = {}
    for e in range(c.n_entries):
        key = (int(c.mmer[e]), (int(c.kmer_hi[e]) << 64) | int(c.kmer_lo[e]))
        out[key] = [int(x) for x in c.ids[int(c.offset[e]):int(c.offset[e + 1])]]
    return out


@pytest.mark.parametrize("K,M,G", [(31, 7, 1), (31, 7, 2), (31, 7, 3), (21, 5, 8), (63, 7, 4),
                                   (40, 6, 5)])
def test_virtual_shards(K, M, G):
    reads = _reads()
    bases, lens = kbin.pack_reads(reads)
    ids = np.arange(len(reads), dtype=np.int32) * 2 + 5  # increasing, not ordinals
    rw = skmer_ref.rec_words(K, M)
    with kbin.Engine(K, M, cutoff=1, max_read_len=300) as eng:
        assert eng.record_words() == rw
        eng.submit(bases=bases, lens=lens, ids=ids)
        counts = eng.route_plan(G)
        total = int(counts.sum())
        send = torch.zeros(max(1, total * rw), dtype=torch.int64, device="cuda")
        eng.route_pack(send.data_ptr())
        torch.cuda.synchronize()
        got = send.cpu().numpy().view(np.uint64)[: total * rw]
    want, wcounts = skmer_ref.encode(reads, ids.tolist(), K, M, G)
    assert counts.tolist() == wcounts
    np.testing.assert_array_equal(got, want)

    ora = skmer_ref.oracle_dict(oracle.bin_reads(bases, lens, K, M, 1, True, ids=ids))
    union = {}
    edges = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
    for d in range(G):
        seg = send[int(edges[d]) * rw:int(edges[d + 1]) * rw]
        with kbin.Engine(K, M, cutoff=1, max_read_len=300) as shard:
            shard.submit_superkmers_device(seg.data_ptr(), int(counts[d]))
            shard.finalize(prune=True)
            part = _result_dict(shard.export())
        assert all(kbin.dist.owner_of(mm, G, K, M) == d for mm, _ in part)
        assert not (set(part) & set(union))
        union.update(part)
    assert union == ora


@pytest.mark.parametrize("K,M,G", [(31, 7, 1), (31, 7, 3), (21, 5, 8), (15, 7, 4), (63, 7, 4), (40, 6, 3)])
def test_route_scatter(K, M, G, engine):
    """one-pass sender: per destination the same multiset of records as
    plan/pack (order is free), a too-small region reports KB_EOVERFLOW and
    ships nothing, and the receivers' union equals the oracle"""
    reads = _reads()
    bases, lens = kbin.pack_reads(reads)
    ids = np.arange(len(reads), dtype=np.int32) * 2 + 5
    rw = skmer_ref.rec_words(K, M)
    want, wcounts = skmer_ref.encode(reads, ids.tolist(), K, M, G)
    want = np.asarray(want, dtype=np.uint64).reshape(-1, rw)
    with kbin.Engine(K, M, cutoff=1, max_read_len=300) as eng:
        eng.submit(bases=bases, lens=lens, ids=ids)
        if engine == "table":  # the one-pass sender is the binned engine's
            with pytest.raises(kbin.KbError) as ei:
                eng.route_scatter(G, 0, 0)
            assert ei.value.code == kbin.KB_EINVAL
            return
        small = torch.zeros(G * 8 * rw, dtype=torch.int64, device="cuda")
        ok, need = eng.route_scatter(G, small.data_ptr(), 8)
        assert not ok and need.tolist() == wcounts
        cap = int(need.max())
        regions = torch.zeros(G * cap * rw, dtype=torch.int64, device="cuda")
        ok, counts = eng.route_scatter(G, regions.data_ptr(), cap)
        assert ok and counts.tolist() == wcounts
        torch.cuda.synchronize()
    got = regions.cpu().numpy().view(np.uint64).reshape(G, cap, rw)
    edges = np.concatenate([[0], np.cumsum(np.asarray(wcounts, dtype=np.int64))])
    ora = skmer_ref.oracle_dict(oracle.bin_reads(bases, lens, K, M, 1, True, ids=ids))
    union = {}
    for d in range(G):
        mine = got[d, :wcounts[d]]
        ref = want[edges[d]:edges[d + 1]]
        order = lambda a: a[np.lexsort(a.T[::-1])]  # noqa: E731
        np.testing.assert_array_equal(order(mine), order(ref))
        with kbin.Engine(K, M, cutoff=1, max_read_len=300) as shard:
            seg = regions[d * cap * rw:]
            shard.submit_superkmers_device(seg.data_ptr(), int(wcounts[d]))
            shard.finalize(prune=True)
            part = _result_dict(shard.export())
        assert not (set(part) & set(union))
        union.update(part)
    assert union == ora


@pytest.mark.parametrize("sub", ["4", "0"])
def test_receiver_learned_map(sub, engine, monkeypatch):
    """a receiver reused over passes learns its bucket map from its own bins
    (few mmers per shard: large ones split into context sub-bins) and converts
    received records by it, cutting them at the edge -- every pass equals the
    oracle's share"""
    if engine != "binned":
        pytest.skip("binned engine only")
    monkeypatch.setenv("KB_BIN_BALANCE_MIN", "0")
    monkeypatch.setenv("KB_BIN_SUB", sub)
    K, M, G = 31, 7, 4
    reads = _reads()
    bases, lens = kbin.pack_reads(reads)
    ids = np.arange(len(reads), dtype=np.int32)
    rw = skmer_ref.rec_words(K, M)
    with kbin.Engine(K, M, cutoff=1, max_read_len=300) as eng:
        eng.submit(bases=bases, lens=lens, ids=ids)
        small = torch.zeros(G * 8 * rw, dtype=torch.int64, device="cuda")
        ok, need = eng.route_scatter(G, small.data_ptr(), 8)
        cap = int(need.max())
        regions = torch.zeros(G * cap * rw, dtype=torch.int64, device="cuda")
        ok, counts = eng.route_scatter(G, regions.data_ptr(), cap)
        assert ok
        torch.cuda.synchronize()
    ora = skmer_ref.oracle_dict(oracle.bin_reads(bases, lens, K, M, 1, True, ids=ids))
    union = {}
    for d in range(G):
        with kbin.Engine(K, M, cutoff=1, max_read_len=300) as shard:
            first = None
            for _ in range(3):  # the first pass learns the map, the next ones use it
                shard.reset()
                shard.submit_superkmers_device(regions[d * cap * rw:].data_ptr(), int(counts[d]))
                shard.finalize(prune=True)
                part = _result_dict(shard.export())
                if first is None:
                    first = part
                assert part == first
        union.update(part)
    assert union == ora


@pytest.mark.parametrize("K,M,P", [(31, 7, 3), (63, 7, 4), (21, 5, 2)])
def test_split_passes(K, M, P, engine):
    """kb_split_passes: ONE super-k-mer pass into the regions of P
    kb_set_partition passes; a context set to pass p bins region p -- equal to
    the direct partitioned pass, and the union equals the oracle"""
    if engine != "binned":
        pytest.skip("binned engine only")
    reads = _reads()
    bases, lens = kbin.pack_reads(reads)
    ids = np.arange(len(reads), dtype=np.int32)
    rw = skmer_ref.rec_words(K, M)
    with kbin.Engine(K, M, cutoff=1, max_read_len=300) as eng:
        eng.submit(bases=bases, lens=lens, ids=ids)
        small = torch.zeros(P * 8 * rw, dtype=torch.int64, device="cuda")
        ok, need = eng.split_passes(P, small.data_ptr(), 8)
        assert not ok
        cap = int(need.max())
        regions = torch.zeros(P * cap * rw, dtype=torch.int64, device="cuda")
        ok, counts = eng.split_passes(P, regions.data_ptr(), cap)
        assert ok and counts.tolist() == need.tolist()
        torch.cuda.synchronize()
    ora = skmer_ref.oracle_dict(oracle.bin_reads(bases, lens, K, M, 1, True, ids=ids))
    union = {}
    with kbin.Engine(K, M, cutoff=1, max_read_len=300) as rx, \
            kbin.Engine(K, M, cutoff=1, max_read_len=300) as direct:
        for p in range(P):
            rx.reset()
            rx.set_partition(p, P)
            rx.submit_superkmers_device(regions[p * cap * rw:].data_ptr(), int(counts[p]))
            rx.finalize(prune=True)
            part = _result_dict(rx.export())
            direct.reset()
            direct.submit(bases=bases, lens=lens, ids=ids)
            direct.set_partition(p, P)
            direct.finalize(prune=True)
            assert part == _result_dict(direct.export())
            assert not (set(part) & set(union))
            union.update(part)
    assert union == ora


@pytest.mark.parametrize("P,K,M", [(2, 31, 7), (5, 31, 7), (3, 63, 7), (4, 40, 6)])
def test_partitioned_routing(P, K, M, engine):
    """kb_set_partition on the sender: each pass routes (ordered plan/pack on
    even passes, one-pass scatter on odd ones) only its mmer slice; the
    per-destination counts add up to the single pass and the union over
    passes and shards equals the oracle.  Two-word k-mers (K > 31) plan/pack
    through route_kernel, which filters by partition as the binned sender does"""
    if engine != "binned":
        pytest.skip("partitioned passes are the binned engine's")
    G = 3
    reads = _reads()
    bases, lens = kbin.pack_reads(reads)
    ids = np.arange(len(reads), dtype=np.int32) * 2 + 5
    rw = skmer_ref.rec_words(K, M)
    # (each pass routes to its own owner table: kb_owner_table)
    pcounts = [skmer_ref.encode(reads, ids.tolist(), K, M, G, p, P)[1] for p in range(P)]
    wcounts = np.sum(pcounts, axis=0).tolist()
    ora = skmer_ref.oracle_dict(oracle.bin_reads(bases, lens, K, M, 1, True, ids=ids))
    union = {}
    tot = np.zeros(G, dtype=np.int64)
    with kbin.Engine(K, M, cutoff=1, max_read_len=300) as eng:
        eng.submit(bases=bases, lens=lens, ids=ids)
        for p in range(P):
            eng.set_partition(p, P)
            if p % 2 == 0:
                counts = eng.route_plan(G)
                send = torch.zeros(max(1, int(counts.sum()) * rw), dtype=torch.int64, device="cuda")
                eng.route_pack(send.data_ptr())
                edges = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
                segs = [(send, int(edges[d]) * rw) for d in range(G)]
            else:
                cap = int(max(pcounts[p])) + 16
                regions = torch.zeros(G * cap * rw, dtype=torch.int64, device="cuda")
                ok, counts = eng.route_scatter(G, regions.data_ptr(), cap)
                assert ok
                segs = [(regions, d * cap * rw) for d in range(G)]
            torch.cuda.synchronize()
            assert counts.tolist() == list(pcounts[p])
            tot += counts.astype(np.int64)
            for d in range(G):
                buf, o = segs[d]
                with kbin.Engine(K, M, cutoff=1, max_read_len=300) as shard:
                    if counts[d]:
                        shard.submit_superkmers_device(buf[o:].data_ptr(), int(counts[d]))
                    shard.finalize(prune=True)
                    part = _result_dict(shard.export())
                assert all(kbin.dist.owner_of(mm, G, K, M, p, P) == d for mm, _ in part)
                assert not (set(part) & set(union))
                union.update(part)
    assert tot.tolist() == list(wcounts)
    assert union == ora


def test_track_first_through_routing():
    """first occurrence (id << 16 | position) survives the exchange"""
    reads = _reads(300)
    bases, lens = kbin.pack_reads(reads)
    ids = np.arange(len(reads), dtype=np.int32)
    K, M, G = 31, 7, 3
    rw = skmer_ref.rec_words(K, M)
    with kbin.Engine(K, M, max_read_len=300, flags=kbin.KB_TRACK_FIRST) as whole:
        whole.submit(bases=bases, lens=lens, ids=ids)
        whole.finalize(prune=False)
        ref = whole.export().canonical()
    firsts = {(int(ref.mmer[e]), int(ref.kmer_lo[e])): int(ref.first[e]) for e in range(ref.n_entries)}
    with kbin.Engine(K, M, max_read_len=300) as eng:
        eng.submit(bases=bases, lens=lens, ids=ids)
        counts = eng.route_plan(G)
        send = torch.zeros(max(1, int(counts.sum()) * rw), dtype=torch.int64, device="cuda")
        eng.route_pack(send.data_ptr())
        torch.cuda.synchronize()
    edges = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
    seen = 0
    for d in range(G):
        with kbin.Engine(K, M, max_read_len=300, flags=kbin.KB_TRACK_FIRST) as shard:
            shard.submit_superkmers_device(send[int(edges[d]) * rw:].data_ptr(), int(counts[d]))
            shard.finalize(prune=False)
            r = shard.export()
            for e in range(r.n_entries):
                assert firsts[(int(r.mmer[e]), int(r.kmer_lo[e]))] == int(r.first[e])
                seen += 1
    assert seen == ref.n_entries


@pytest.mark.parametrize("transport", ["torch", "c"])
def test_ranks_rehearsal(tmp_path, transport):
    """Two real ranks (torch.distributed.run, gloo rehearsal on one GPU) run
    kbin.dist.ShardedBinner end to end, stepwise and pipelined; the union of
    what they own equals a single-GPU engine over both shards' reads.
    transport "c" (VERDICT r04 item 6): GroupBinner, i.e. the C group's
    routing, count and offset bookkeeping and async sender thread, with the
    counts and records moved by gloo host collectives
    (kb_group_create_rank_host) instead of RCCL, which refuses two ranks on
    one device."""
    import socket
    import subprocess
    import sys
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    n, L, K, M = 20000, 150, 31, 7
    env = dict(__import__("os").environ, KB_DIST_BACKEND="gloo", KB_DIST_TRANSPORT=transport)
    worker = kbin.REPO_ROOT / "tests" / "dist_worker.py"
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                    "--master-addr", "127.0.0.1", "--master-port", str(port), str(worker),
                    str(tmp_path), str(n), str(L), str(K), str(M)], check=True, env=env, timeout=300)
    wpr = (L + 31) // 32
    words = np.concatenate([np.load(tmp_path / f"words{r}.npy") for r in range(2)])
    dw = torch.from_numpy(words).cuda()
    dl = torch.full((2 * n,), L, dtype=torch.int32, device="cuda")
    with kbin.Engine(K, M, cutoff=1, max_read_len=L) as eng:
        eng.submit_packed_device(dw.data_ptr(), dl.data_ptr(), 2 * n, wpr, 0)
        eng.finalize(True)
        want = _result_dict(eng.export())
    union = {}
    for r in range(2):
        z = np.load(tmp_path / f"rank{r}.npz")
        res = kbin.Result(z["mmer"], z["hi"], z["lo"], z["count"], z["offset"], z["ids"], 0, 0)
        part = _result_dict(res)
        zp = np.load(tmp_path / f"rank{r}_pipe.npz")  # pipelined send / receive: the same share
        assert _result_dict(kbin.Result(zp["mmer"], zp["hi"], zp["lo"], zp["count"], zp["offset"],
                                        zp["ids"], 0, 0)) == part
        assert all(kbin.dist.owner_of(mm, 2) == r for mm, _ in part)
        assert not (set(part) & set(union))
        union.update(part)
        assert z["sent"].sum() > 0 and z["recv"].sum() > 0
    assert union == want


# ---- multi-GPU groups through the C-ABI (kb_group_*: routing, exchange over
# RCCL or device copies, receivers -- all in C; kbin.h "multi-GPU groups")

def _group_union(grp, G_local, K=31, M=7, p=0, P=1):
    union = {}
    for g in range(G_local):
        part = _result_dict(grp.ctx(g).export())
        assert all(kbin.dist.owner_of(mm, grp.n_ranks, K, M, p, P) == grp.rank0 + g for mm, _ in part)
        assert not (set(part) & set(union))
        union.update(part)
    return union


@pytest.mark.parametrize("K,M,G", [(31, 7, 2), (31, 7, 4), (31, 7, 8), (21, 5, 3), (63, 7, 4), (40, 6, 2)])
def test_group_virtual_shards(K, M, G, engine):
    """G ranks in this process on one device (virtual shards: the device-copy
    transport on the same C routing code): each rank gets a contiguous slice
    of the reads, and the union of the receivers equals the oracle, pruned
    and not; every rank owns exactly its owner(mmer) share"""
    reads = _reads()
    bases, lens = kbin.pack_reads(reads)
    ids = np.arange(len(reads), dtype=np.int32) * 2 + 5  # increasing with the call order
    off = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
    cuts = np.linspace(0, len(reads), G + 1).astype(int)
    with kbin.Group(K, M, cutoff=1, max_read_len=300, devices=[0] * G) as grp:
        assert grp.transport == kbin.KB_TRANSPORT_LOCAL and grp.n_ranks == G == grp.n_local
        for prune in (True, False):
            grp.reset()
            for g in range(G):
                a, b = cuts[g], cuts[g + 1]
                grp.submit(g, bases=bases[off[a]:off[b]], lens=lens[a:b], ids=ids[a:b])
            grp.finalize(prune)
            want = skmer_ref.oracle_dict(oracle.bin_reads(bases, lens, K, M, 1, prune, ids=ids))
            assert _group_union(grp, G, K, M) == want


def _c2_prefix(n):
    import bench
    wl = bench.WORKLOADS["c2"]
    L = wl["read_len"]
    wpr = (L + 31) // 32
    w = torch.empty(n * wpr, dtype=torch.int64, device="cuda")
    ln = torch.empty(n, dtype=torch.int32, device="cuda")
    kbin.generate_reads_device(w.data_ptr(), ln.data_ptr(), n, L, wl["genome"], wl["err_ppm"],
                               bench.gen_seed(wl["seed"]))
    torch.cuda.synchronize()
    bases, lens = kbin.unpack_reads_to_host(w.data_ptr(), ln.data_ptr(), n, wpr, n * L)
    return w, ln, wpr, L, bases, lens


@pytest.mark.parametrize("api", ["create", "create_rank", "self_rccl_pieces"])
def test_group_rccl_c2_prefix(api, engine, monkeypatch):
    """G = 1 through RCCL itself (ncclCommInitAll / ncclCommInitRank with a
    unique id; counts all-gathered), bit-exact against the oracle on the C2
    generator's first 40 K reads.  A rank's own records are a device copy;
    self_rccl_pieces sends them through RCCL in 32-KB pieces instead -- the
    piecewise exchange every peer message takes (a single multi-GB RCCL
    message delivered about half of its records, round 6)"""
    if api == "self_rccl_pieces":
        monkeypatch.setenv("KB_GROUP_SELF_RCCL", "1")
        monkeypatch.setenv("KB_GROUP_CHUNK", "4096")
    n = 40_000
    w, ln, wpr, L, bases, lens = _c2_prefix(n)
    kw = dict(cutoff=1, max_read_len=L)
    if api != "create_rank":
        grp = kbin.Group(31, 7, devices=[0], **kw)
    else:
        grp = kbin.Group(31, 7, rank=0, n_ranks=1, unique_id=kbin.group_unique_id(), device=0, **kw)
    with grp:
        assert grp.transport == kbin.KB_TRANSPORT_RCCL
        grp.submit_packed_device(0, w.data_ptr(), ln.data_ptr(), n, wpr, 0)
        counts = grp.send()
        assert counts.shape == (1, 1) and int(counts[0, 0]) > 0
        grp.receive(True)
        got = grp.ctx(0).export()
    assert_same_as_oracle(got, oracle.bin_reads(bases, lens, 31, 7, 1, True))


def assert_same_as_oracle(res, ora):
    c = res.canonical()
    assert c.n_entries == ora.n_entries
    for f in ("mmer", "kmer_hi", "kmer_lo", "count", "offset", "ids"):
        np.testing.assert_array_equal(getattr(c, f), getattr(ora, f))


def test_group_pipelined_partitions(engine):
    """two units in flight (send, send, receive, receive ...) over partitioned
    passes of the same reads: the passes' union over 4 virtual ranks equals
    the oracle; a third unit in flight is KB_ESTATE; a discarded unit is
    dropped unbinned"""
    if engine != "binned":
        pytest.skip("partitioned passes are the binned engine's")
    n = 12_000
    w, ln, wpr, L, bases, lens = _c2_prefix(n)
    G, P = 4, 3
    cuts = np.linspace(0, n, G + 1).astype(int)
    union = {}
    with kbin.Group(31, 7, cutoff=1, max_read_len=L, devices=[0] * G) as grp:
        for g in range(G):
            a = int(cuts[g])
            grp.submit_packed_device(g, w[a * wpr:].data_ptr(), ln[a:].data_ptr(), int(cuts[g + 1]) - a, wpr, a)
        grp.set_partition(0, P)
        grp.send()
        grp.set_partition(1, P)
        grp.send()
        with pytest.raises(kbin.KbError) as ei:
            grp.send()
        assert ei.value.code == kbin.KB_ESTATE
        grp.discard()
        grp.discard()
        grp.set_partition(0, P)
        grp.send()
        for p in range(P):
            if p + 1 < P:
                grp.set_partition(p + 1, P)
                grp.send()
            grp.receive(True)
            part = _group_union(grp, G, p=p, P=P)
            assert not (set(part) & set(union))
            union.update(part)
    assert union == skmer_ref.oracle_dict(oracle.bin_reads(bases, lens, 31, 7, 1, True))


def test_group_discard_reports_failed_unit(engine):
    """kb_group_discard returns the unit's failure, as kb_group_receive does
    (ADVICE r05): a unit whose routing fails (a read byte outside ACGT on one
    rank: kb_route_plan's ingest check) is discarded with KB_EALPHABET, not
    silently dropped with zero counts; after kb_group_reset the group bins
    the next unit bit-exact"""
    if engine != "binned":
        pytest.skip("routing is engine-independent")
    good = _reads(300)
    bad = list(good[:100])
    bad[7] = bad[7][:20] + b"N" + bad[7][21:]
    K, M = 31, 7
    with kbin.Group(K, M, cutoff=1, max_read_len=300, devices=[0, 0]) as grp:
        grp.submit(0, bad, first_id=0)
        grp.submit(1, good[100:], first_id=100)
        grp.send_async()
        with pytest.raises(kbin.KbError) as ei:
            grp.discard()
        assert ei.value.code == kbin.KB_EALPHABET
        grp.reset()
        grp.submit(0, good[:100], first_id=0)
        grp.submit(1, good[100:], first_id=100)
        grp.finalize(True)
        union = {}
        for g in range(2):
            union.update(_result_dict(grp.ctx(g).export()))
    bases, lens = kbin.pack_reads(good)
    assert union == skmer_ref.oracle_dict(oracle.bin_reads(bases, lens, K, M, 1, True))


def test_group_track_first(engine):
    """first occurrences through a group (the drop-in's multi-GPU mode): the
    sender switches to plan/pack (read order), receivers keep (id << 16 |
    position) of every key exactly as one engine over all reads does"""
    reads = _reads(400)
    bases, lens = kbin.pack_reads(reads)
    ids = np.arange(len(reads), dtype=np.int32)
    K, M, G = 31, 7, 3
    with kbin.Engine(K, M, max_read_len=300, flags=kbin.KB_TRACK_FIRST) as whole:
        whole.submit(bases=bases, lens=lens, ids=ids)
        whole.finalize(prune=False)
        ref = whole.export().canonical()
    firsts = {(int(ref.mmer[e]), int(ref.kmer_lo[e])): int(ref.first[e]) for e in range(ref.n_entries)}
    want = _result_dict(ref)
    off = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
    cuts = np.linspace(0, len(reads), G + 1).astype(int)
    with kbin.Group(K, M, max_read_len=300, devices=[0] * G, flags=kbin.KB_TRACK_FIRST) as grp:
        for g in range(G):
            a, b = cuts[g], cuts[g + 1]
            grp.submit(g, bases=bases[off[a]:off[b]], lens=lens[a:b], ids=ids[a:b])
        grp.finalize(False)
        seen = 0
        union = {}
        for g in range(G):
            r = grp.ctx(g).export()
            for e in range(r.n_entries):
                assert firsts[(int(r.mmer[e]), int(r.kmer_lo[e]))] == int(r.first[e])
                seen += 1
            union.update(_result_dict(r))
    assert seen == ref.n_entries and union == want


@pytest.mark.parametrize("transport", ["torch", "c"])
def test_bench_multi_gpu_capacity_rehearsal(tmp_path, engine, transport):
    """bench.py at N = 2 (gloo rehearsal: two ranks on one GPU) runs the
    headline C2 weak-scaling leg and then BASELINE's multi-GPU configurations
    as specified -- C4 (K31, 150 bp, one 3.1-Gbp genome, P = 5) and C5 (K63,
    250 bp, 1 % errors, P = 4) -- routed between the ranks; here at 1/400 of
    their reads (KB_CAPACITY_SCALE) to test the legs' plumbing: the one JSON
    line carries both legs with their timings, rooflines and exchange bytes.
    transport c: the legs through the C group (kb_group_create_rank_host over
    gloo), the object the driver's RCCL run uses (GroupBinner)"""
    if engine != "binned":
        pytest.skip("bench picks its engine itself")
    import json
    import os
    import socket
    import subprocess
    import sys
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, KB_DIST_BACKEND="gloo", KB_CAPACITY_SCALE="400", KB_ROUTED_TRANSPORT=transport)
    env.pop("KB_ENGINE", None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), str(kbin.REPO_ROOT / "bench.py"),
                        "--gpus", "2", "--steps", "2", "--warmup", "1", "--reads", "100000"],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["value"] > 0
    for name, K in (("c4", 31), ("c5", 63)):
        leg = line["capacity"][name]
        assert leg["value"] > 0 and leg["ms_per_step"] > 0, leg
        assert f"K={K}" in leg["workload"] and leg["rehearsal_scale"] == 400
        assert leg["exchange"]["bytes_sent_off_rank_per_step"] > 0
        assert 0 < leg["roofline"]["frac"] < 1


def test_bench_multi_legs_one_rank_rccl(engine):
    """bench.py --routed --multi-legs: the N > 1 run's C4 and C5 legs through
    a one-rank RCCL group (GroupBinner: the object the driver's multi-GPU run
    uses), here at 1/400 of their reads -- the full-size run of the same
    command is the legs' memory and time rehearsal"""
    if engine != "binned":
        pytest.skip("bench picks its engine itself")
    import json
    import os
    import subprocess
    import sys
    env = dict(os.environ, KB_CAPACITY_SCALE="400")
    env.pop("KB_ENGINE", None)
    env.pop("KB_DIST_BACKEND", None)
    r = subprocess.run([sys.executable, str(kbin.REPO_ROOT / "bench.py"), "--routed", "--multi-legs", "--steps", "2",
                        "--warmup", "1", "--reads", "100000", "--cpu-sample", "0", "--no-host-input"],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["value"] > 0
    for name, K in (("c4", 31), ("c5", 63)):
        leg = line["capacity"][name]
        assert leg["value"] > 0 and leg["ms_per_step"] > 0, leg
        assert f"K={K}" in leg["workload"] and leg["rehearsal_scale"] == 400
        assert leg["exchange"]["record_bytes"] == (24 if K == 31 else 40)
        assert 0 < leg["roofline"]["frac"] < 1


def _k_below_2m_reads(K, M):
    rng = np.random.default_rng(K * 1000 + M + 7)
    genome = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=3000)
    reads = []
    for _ in range(1200):
        L = int(rng.integers(0, 260))
        s = int(rng.integers(0, 3000 - L))
        r = genome[s:s + L].copy()
        m = rng.random(L) < 0.01
        r[m] = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=int(m.sum()))
        reads.append(r.tobytes())
    return reads


@pytest.mark.parametrize("K,M", [(10, 6), (5, 4), (7, 4), (13, 7), (15, 8), (3, 2)])
@pytest.mark.parametrize("mode", ["split3", "scatter4", "plan2", "group2", "group4"])
def test_k_below_2m_routed(K, M, mode, engine):
    """K < 2M beyond one GPU: the routed records carry the
    complement flag (kbin_internal.h ROUTED_REV_BIT) -- the live incremental
    branch's is_rev (binning.c:992-1021) is no function of the span -- so
    kb_split_passes (P = 3), kb_route_scatter (4 shards), kb_route_plan/pack
    (2 shards) and the C group (2 and 4 virtual ranks) all take these
    configurations; every union is bit-exact against the oracle"""
    if engine != "binned":
        pytest.skip("K < 2M runs on the binned engine")
    reads = _k_below_2m_reads(K, M)
    bases, lens = kbin.pack_reads(reads)
    ids = np.arange(len(reads), dtype=np.int32)
    rw = skmer_ref.rec_words(K, M)
    ora = skmer_ref.oracle_dict(oracle.bin_reads(bases, lens, K, M, 1, True, ids=ids))
    union = {}
    if mode.startswith("group"):
        G = int(mode[5:])
        off = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
        cuts = np.linspace(0, len(reads), G + 1).astype(int)
        with kbin.Group(K, M, cutoff=1, max_read_len=300, devices=[0] * G) as grp:
            for g in range(G):
                a, b = cuts[g], cuts[g + 1]
                grp.submit(g, bases=bases[off[a]:off[b]], lens=lens[a:b], ids=ids[a:b])
            grp.finalize(True)
            for g in range(G):
                part = _result_dict(grp.ctx(g).export())
                assert not (set(part) & set(union))
                union.update(part)
        assert union == ora
        return
    with kbin.Engine(K, M, cutoff=1, max_read_len=300) as eng:
        eng.submit(bases=bases, lens=lens, ids=ids)
        if mode == "plan2":
            G = 2
            counts = eng.route_plan(G)
            total = int(counts.sum())
            send = torch.zeros(max(1, total * rw), dtype=torch.int64, device="cuda")
            eng.route_pack(send.data_ptr())
            edges = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
            segs = [(send[int(edges[d]) * rw:].data_ptr(), int(counts[d]), None) for d in range(G)]
        else:
            P = 3 if mode == "split3" else 4
            fn = eng.split_passes if mode == "split3" else eng.route_scatter
            small = torch.zeros(P * 8 * rw, dtype=torch.int64, device="cuda")
            ok, need = fn(P, small.data_ptr(), 8)
            cap = int(need.max()) + 1
            regions = torch.zeros(P * cap * rw, dtype=torch.int64, device="cuda")
            ok, counts = fn(P, regions.data_ptr(), cap)
            assert ok
            segs = [(regions[p * cap * rw:].data_ptr(), int(counts[p]), p if mode == "split3" else None)
                    for p in range(P)]
        torch.cuda.synchronize()
        for ptr, cnt, p in segs:
            with kbin.Engine(K, M, cutoff=1, max_read_len=300) as rx:
                if p is not None:
                    rx.set_partition(p, 3)
                rx.submit_superkmers_device(ptr, cnt)
                rx.finalize(prune=True)
                part = _result_dict(rx.export())
            assert not (set(part) & set(union))
            union.update(part)
    assert union == ora
