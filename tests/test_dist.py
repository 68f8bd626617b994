"""World-size-2 test of the multi-GPU path on CPU (gloo): each rank encodes
its half of the reads into super-k-mer records, the product's exchange
(kbin.dist.exchange_records) moves them, each rank bins what it owns; the
union over ranks must equal the single-process oracle, with disjoint keys
owned by owner(mmer)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
import skmer_ref
from conftest import GOLDEN
from kbin.dist import exchange_records, owner_of

K, M = 21, 5


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _reads():
    bases, lens = oracle.read_fgets(GOLDEN / "reads.txt", 102)
    off = np.concatenate([[0], np.cumsum(lens.astype(np.int64))]).astype(np.int64)
    n = 600
    return [bases[off[i]:off[i + 1]] for i in range(n)], bases[:off[n]], lens[:n]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        reads, _, _ = _reads()
        cuts = np.linspace(0, len(reads), world + 1).astype(int)
        mine = list(range(cuts[rank], cuts[rank + 1]))
        recs, counts = skmer_ref.encode([reads[i] for i in mine], mine, K, M, world)
        rw = skmer_ref.rec_words(K, M)
        send = torch.from_numpy(recs.view(np.int64).copy())
        recv, rc = exchange_records(send, counts, rw, None)
        occ = skmer_ref.decode(recv.numpy().view(np.uint64), K, M)
        mine_res = skmer_ref.bin_occurrences(occ)
        # every key this rank holds is owned by this rank
        assert all(owner_of(mm, world, K, M) == rank for mm, _ in mine_res)
        gathered = [None] * world
        dist.all_gather_object(gathered, mine_res)
        if rank == 0:
            q.put(gathered)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_union_equals_single(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    gathered = None
    for _ in range(240):
        try:
            gathered = q.get(timeout=1)
            break
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                break
    for p in procs:
        if gathered is None:
            p.kill()
        p.join(timeout=60)
        assert p.exitcode == 0
    assert gathered is not None
    _, bases, lens = _reads()
    want = skmer_ref.oracle_dict(oracle.bin_reads(bases, lens, K, M, 1, True))
    union = {}
    for part in gathered:
        assert not (set(part) & set(union)), "a key landed on two ranks"
        union.update(part)
    assert union == want
    assert all(len(p) > 0 for p in gathered)


def test_owner_balance():
    """owner(mmer) (kb_owner_table): every pass's canonical mmers packed onto
    the ranks by their expected signature frequency -- the busiest rank's
    expected load within 1 % of the mean at 2-8 ranks (or within one mmer of
    it), in one pass and in every pass of 4 and 5 (the hash it replaced: up to 1.20x in one pass at
    8 ranks, 1.4-1.7x inside C4's and C5's passes); the same table from every
    call; K < 2M codes (not canonical) keep the spread of the owner hash"""
    import kbin
    from kbin.dist import _mix64
    for KK, MM in ((31, 7), (63, 7), (21, 5)):
        half = 1 << (2 * MM - 1)
        w = ((np.arange(half) + 1) / half) ** (KK - MM)
        for G in (2, 4, 8):
            for P in (1, 4, 5):
                for p in range(P):
                    t = kbin.owner_table(KK, MM, G, p, P)
                    assert (t == kbin.owner_table(KK, MM, G, p, P)).all() and t.max() < G
                    mine = np.array([P == 1 or (_mix64(half + i + 0x9E3779B97F4A7C15) >> 32) % P == p
                                     for i in range(half)])
                    load = np.bincount(t[mine], weights=w[mine], minlength=G)
                    # (LPT: within 1 % of the mean, or one mmer above it when a
                    # single mmer outweighs a rank's share -- M = 5 at 8 ranks)
                    assert load.max() <= max(1.01 * load.mean(), load.mean() + w[mine].max()), (KK, MM, G, P, p)
                    assert all(owner_of(half + i, G, KK, MM, p, P) == t[i] for i in range(0, half, 97))
    rng = np.random.default_rng(0)
    mm = rng.integers(0, 1 << 14, 20000)
    for G in (2, 4, 8):
        cnt = np.bincount([owner_of(int(x), G, 9, 7) for x in mm], minlength=G)  # (K < 2M: the hash)
        assert cnt.max() / cnt.mean() < 1.1


def test_encoder_roundtrip_single_rank():
    reads, bases, lens = _reads()
    recs, counts = skmer_ref.encode(reads, range(len(reads)), K, M, 1)
    got = skmer_ref.bin_occurrences(skmer_ref.decode(recs, K, M))
    want = skmer_ref.oracle_dict(oracle.bin_reads(bases, lens, K, M, 1, True))
    assert got == want


def _host_worker(rank, world, port, q):
    import ctypes as C
    from kbin.dist import HostCollectives
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hc = HostCollectives()
        # counts rows (G counts + a status word, as kbin_group.hip sends them)
        row = (C.c_uint64 * (world + 1))(*([10 * rank + d for d in range(world)] + [0]))
        out = (C.c_uint64 * ((world + 1) * world))()
        assert hc.allgather(None, row, world + 1, out) == 0, hc.errors
        # records: rank r sends (r + 1)(d + 1) 8-B words to rank d, each word r << 8 | d
        sw = [(rank + 1) * (d + 1) for d in range(world)]
        rw_ = [(s + 1) * (rank + 1) for s in range(world)]
        send = np.concatenate([np.full(n, (rank << 8) | d, np.uint64) for d, n in enumerate(sw)])
        recv = np.zeros(sum(rw_), np.uint64)
        sb = (C.c_uint64 * world)(*[8 * n for n in sw])
        rb = (C.c_uint64 * world)(*[8 * n for n in rw_])
        assert hc.alltoallv(None, send.ctypes.data, sb, recv.ctypes.data, rb) == 0, hc.errors
        if rank == 1:
            q.put((list(out), recv.tolist()))
    finally:
        dist.destroy_process_group()


def test_group_host_collectives():
    """kbin.dist.HostCollectives -- the host transport the C group
    (kb_group_create_rank_host) calls for its counts all-gather and record
    all-to-all under a gloo process group -- at world size 2 on CPU"""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_host_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rows, recv = got
    assert rows == [0, 1, 0, 10, 11, 0]
    # rank 1 receives 2 words from rank 0 (0 << 8 | 1), then 4 from itself (1 << 8 | 1)
    assert recv == [1, 1] + [257] * 4
