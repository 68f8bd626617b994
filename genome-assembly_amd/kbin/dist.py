"""Multi-GPU binning: one process per GPU, the canonical-mmer space sharded
over the ranks.

The reference has no distributed mode; FAQ.md:11 only asks how bins would be
merged across nodes.  Here the level-1 key of binning.c (the mmer,
binning.c:1045) is the shard key: every (mmer, kmer) entry lives on rank
owner(mmer), so per-rank results are disjoint and their union is the
single-GPU result.  The one exchange step is an all-to-all of super-k-mer
records (a run of consecutive k-mers of a read that share one signature,
~10 per 150-bp read at k31/m7 -- about 2 B per k-mer on the wire instead of
a 12-16 B per-k-mer record) over RCCL (torch.distributed "nccl") / xGMI.

Data path (one process per GPU, torch.distributed "nccl"): the exchange is
the C-ABI's multi-GPU group (kbin.h kb_group_create_rank; kbin.Group):
routing, the counts all-gather and the records' grouped ncclSend/ncclRecv
all run in C (csrc/kbin_group.hip) on an RCCL communicator of its own, and
torch.distributed only hands every rank the group's unique id.  The torch
exchange below stays for the gloo rehearsal (KB_DIST_BACKEND=gloo: several
ranks sharing a GPU, or CPU tests), where RCCL cannot run.

Per step on every rank, wherever the binned engine applies (K <= 31 on any
read length; K <= 63 on reads of <= 512 bp -- the default; kbin.h
KB_ENGINE_BINNED):
  kb_route_scatter (one pass: records straight into per-destination regions)
  ->  all_to_all_single of the counts, all_to_all of the region slices  ->
  kb_submit_superkmers_device (one batch per source rank)  ->  kb_finalize.
Otherwise (the table engine: forced, or two-word k-mers on reads > 512 bp):
  kb_route_plan (counts per destination)  ->  kb_route_pack (dest-major send
  buffer, read order)  ->  all_to_all_single (counts, then records)  ->
  kb_submit_superkmers_device (received, concatenated by source rank)  ->
  kb_finalize.  Both senders honour kb_set_partition (only the pass's mmer
  partition is counted and shipped), so step(part, n_parts) is valid on
  either; the receivers' union equals the single-GPU result in every case.
Read ids must increase with the global call order (rank r's ids below rank
r+1's): they are the reverse-call-order key of every id list.
"""
from __future__ import annotations

import ctypes as C
import time

import numpy as np

import torch
import torch.distributed as dist

from . import Engine, Group, group_unique_id

_MIX_SALT = 0x5851F42D4C957F2D
_M64 = (1 << 64) - 1


def _mix64(x: int) -> int:
    x &= _M64
    x ^= x >> 30
    x = (x * 0xBF58476D1CE4E5B9) & _M64
    x ^= x >> 27
    x = (x * 0x94D049BB133111EB) & _M64
    x ^= x >> 31
    return x


_OWNER_TABLES = {}


def owner_of(mmer_code: int, n_dest: int, K: int = 31, M: int = 7, part: int = 0, n_parts: int = 1) -> int:
    """Owning rank of a mmer among n_dest ranks in pass (part, n_parts): the
    routing kernels' owner -- kb_owner_table (include/kbin.h) for a canonical
    code at K >= 2M, the owner hash (owner_of() in csrc/kbin_kernels.hip)
    for any other code"""
    half = 1 << (2 * M - 1)
    if K < 2 * M or not half <= mmer_code < 2 * half:
        return (_mix64(mmer_code + _MIX_SALT) >> 32) % n_dest
    key = (K, M, n_dest, part if n_parts > 1 else 0, max(1, n_parts))
    t = _OWNER_TABLES.get(key)
    if t is None:
        from . import owner_table
        t = _OWNER_TABLES[key] = owner_table(K, M, n_dest, key[3], key[4])
    return int(t[mmer_code - half])


def exchange_records(send: torch.Tensor, counts, rec_words: int, group=None):
    """All-to-all of fixed-size records.  `send` holds sum(counts) records
    (rec_words int64 each), destination-major; returns (received records
    concatenated by source rank, per-source counts).  Device-agnostic: RCCL
    for cuda tensors, gloo for cpu tensors."""
    dev = send.device
    if dev.type == "cuda" and dist.get_backend(group) == "gloo":
        # rehearsal mode (several ranks sharing one GPU, gloo): stage via host
        recv, rc = exchange_records(send[: int(sum(counts)) * rec_words].cpu(), counts, rec_words,
                                    group)
        return recv.to(dev), rc
    cnt = torch.tensor([int(c) for c in counts], dtype=torch.int64, device=dev)
    rcnt = torch.empty_like(cnt)
    dist.all_to_all_single(rcnt, cnt, group=group)
    rc = [int(x) for x in rcnt.cpu().tolist()]
    recv = torch.empty(sum(rc) * rec_words, dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv, send[: int(sum(counts)) * rec_words].contiguous(),
                           output_split_sizes=[c * rec_words for c in rc],
                           input_split_sizes=[int(c) * rec_words for c in counts], group=group)
    return recv, rc


def exchange_regions(regions: torch.Tensor, counts, cap: int, rec_words: int, group=None):
    """All-to-all of per-destination record regions (destination d's records
    at regions[d*cap*rec_words:], counts[d] of them; kb_route_scatter's
    layout).  Returns (one received tensor per source rank, per-source
    counts).  RCCL moves each region slice directly (no packing pass); the
    gloo rehearsal of cuda tensors stages through the host."""
    dev = regions.device
    G = len(counts)
    sends = [regions[d * cap * rec_words:(d * cap + int(counts[d])) * rec_words] for d in range(G)]
    if dev.type == "cuda" and dist.get_backend(group) == "gloo":
        flat = torch.cat(sends).cpu()
        recv, rc = exchange_records(flat, [int(c) for c in counts], rec_words, group)
        recv = recv.to(dev)
        edges = [0]
        for c in rc:
            edges.append(edges[-1] + c * rec_words)
        return [recv[edges[i]:edges[i + 1]] for i in range(G)], rc
    cnt = torch.tensor([int(c) for c in counts], dtype=torch.int64, device=dev)
    rcnt = torch.empty_like(cnt)
    dist.all_to_all_single(rcnt, cnt, group=group)
    rc = [int(x) for x in rcnt.cpu().tolist()]
    recvs = [torch.empty(c * rec_words, dtype=torch.int64, device=dev) for c in rc]
    dist.all_to_all(recvs, sends, group=group)
    return recvs, rc


def exchange_records_async(send: torch.Tensor, counts, rec_words: int, group=None):
    """exchange_records with the record all-to-all left in flight: returns
    ([received tensor], per-source counts, work handle or None)"""
    dev = send.device
    if dev.type == "cuda" and dist.get_backend(group) == "gloo":
        recv, rc = exchange_records(send, counts, rec_words, group)
        return [recv], rc, None
    cnt = torch.tensor([int(c) for c in counts], dtype=torch.int64, device=dev)
    rcnt = torch.empty_like(cnt)
    dist.all_to_all_single(rcnt, cnt, group=group)
    rc = [int(x) for x in rcnt.cpu().tolist()]
    recv = torch.empty(sum(rc) * rec_words, dtype=torch.int64, device=dev)
    work = dist.all_to_all_single(recv, send[: int(sum(counts)) * rec_words],
                                  output_split_sizes=[c * rec_words for c in rc],
                                  input_split_sizes=[int(c) * rec_words for c in counts], group=group,
                                  async_op=True)
    return [recv], rc, work


def exchange_regions_async(regions: torch.Tensor, counts, cap: int, rec_words: int, group=None):
    """exchange_regions with the record all-to-all left in flight: returns
    (received tensors, per-source counts, work handle or None).  The counts
    exchange synchronises; the records land when work.wait() returns (the
    gloo rehearsal completes at once)."""
    dev = regions.device
    if dev.type == "cuda" and dist.get_backend(group) == "gloo":
        recvs, rc = exchange_regions(regions, counts, cap, rec_words, group)
        return recvs, rc, None
    G = len(counts)
    sends = [regions[d * cap * rec_words:(d * cap + int(counts[d])) * rec_words] for d in range(G)]
    cnt = torch.tensor([int(c) for c in counts], dtype=torch.int64, device=dev)
    rcnt = torch.empty_like(cnt)
    dist.all_to_all_single(rcnt, cnt, group=group)
    rc = [int(x) for x in rcnt.cpu().tolist()]
    recvs = [torch.empty(c * rec_words, dtype=torch.int64, device=dev) for c in rc]
    work = dist.all_to_all(recvs, sends, group=group, async_op=True)
    return recvs, rc, work


class ShardedBinner:
    """One rank's share of a mmer-sharded binning job.  transport "c" (the
    default under an nccl process group): the C-ABI group does the routing
    and the RCCL exchange; "torch": the exchange through torch.distributed
    collectives (the gloo rehearsal)."""

    def __new__(cls, *a, transport: str | None = None, **kw):
        if cls is ShardedBinner:
            group = kw.get("group")
            if transport is None:
                transport = "c" if dist.get_backend(group) == "nccl" else "torch"
            if transport == "c":
                return super().__new__(GroupBinner)
        return super().__new__(cls)

    def __init__(self, K: int, M: int, cutoff: int, max_read_len: int, device: int = 0,
                 group=None, flags: int = 0, transport: str | None = None):
        self.engine = Engine(K, M, cutoff=cutoff, max_read_len=max_read_len, device=device,
                             flags=flags)
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.rec_words = self.engine.record_words()
        self.device = torch.device("cuda", device)
        self._send = torch.empty(0, dtype=torch.int64, device=self.device)
        self._recv = None
        self.last_counts = None
        self.last_times = {}
        self._regions = torch.empty(0, dtype=torch.int64, device=self.device)
        self._cap = 0
        self._wcap = 0  # the region capacity of the last scatter (its layout)
        self.scatter = True  # one-pass sender while the engine accepts it
        # pipelined steps (send / receive): a sender context of its own and
        # two region buffers, so one unit's records can be in flight while
        # the previous unit is binned
        self._engine_args = (K, M, cutoff, max_read_len, device, flags)
        self._sender = None
        self._pregions = [torch.empty(0, dtype=torch.int64, device=self.device) for _ in range(2)]
        self._slot = 0

    def _scatter(self, n_reads: int, engine=None, slot=None):
        """kb_route_scatter with a learned region capacity; None when the
        engine cannot take this path (the caller plans and packs instead).
        slot: one of the pipelined region buffers instead of self._regions."""
        from . import KB_EINVAL, KbError
        engine = engine or self.engine
        if self._cap == 0:  # ~10 records per 150-bp read, spread over the ranks
            self._cap = int(n_reads * 12 / self.world * 1.25) + 4096
        for _ in range(2):
            need = self.world * self._cap * self.rec_words
            buf = self._regions if slot is None else self._pregions[slot]
            if buf.numel() < need:
                buf = torch.empty(need, dtype=torch.int64, device=self.device)
                if slot is None:
                    self._regions = buf
                else:
                    self._pregions[slot] = buf
            try:
                ok, counts = engine.route_scatter(self.world, buf.data_ptr(), self._cap)
            except KbError as e:
                if e.code != KB_EINVAL:
                    raise
                self.scatter = False
                return None
            if ok:
                # the layout this call wrote (destination d at d * cap) is the
                # exchange's; the raised headroom is the next unit's
                self._wcap = self._cap
                self._cap = max(self._cap, int(int(counts.max()) * 1.1) + 1024)
                return counts
            self._cap = int(int(counts.max()) * 1.2) + 1024  # retry once with room for all
        raise RuntimeError("kb_route_scatter: region capacity not converging")

    def _send_buffer(self, words: int) -> torch.Tensor:
        if self._send.numel() < words:
            self._send = torch.empty(int(words * 1.25) + 1024, dtype=torch.int64, device=self.device)
        return self._send

    def step(self, words: torch.Tensor, lens: torch.Tensor, n_reads: int, words_per_read: int,
             first_id: int, prune: bool = True, part: int = 0, n_parts: int = 1) -> None:
        """Bin this rank's resident packed reads (ids first_id..first_id+n-1)
        together with every other rank's; the result this rank owns stays in
        self.engine (export / export_device).  n_parts > 1: only the keys of
        mmer partition `part` (kb_set_partition) -- every rank passes the same
        (part, n_parts), and the n_parts steps together bin everything."""
        eng = self.engine
        t = [time.perf_counter()]
        eng.reset()
        eng.submit_packed_device(words.data_ptr(), lens.data_ptr(), n_reads, words_per_read,
                                 first_id)
        if n_parts > 1:
            eng.set_partition(part, n_parts)
        counts = self._scatter(n_reads) if self.scatter else None
        if counts is not None:  # one pass: records straight into destination regions
            t.append(time.perf_counter())
            t.append(t[-1])
            recvs, rc = exchange_regions(self._regions, counts.tolist(), self._wcap, self.rec_words,
                                         self.group)
        else:  # plan / pack: destination-major, read order (any engine)
            counts = eng.route_plan(self.world)  # synchronises the engine stream
            t.append(time.perf_counter())
            total = int(counts.sum())
            send = self._send_buffer(total * self.rec_words)
            eng.route_pack(send.data_ptr())  # synchronises the engine stream
            t.append(time.perf_counter())
            recv, rc = exchange_records(send, counts.tolist(), self.rec_words, self.group)
            recvs = [recv]
        torch.cuda.current_stream(self.device).synchronize()
        t.append(time.perf_counter())
        self._recv = recvs  # referenced by the engine until the next reset
        self.last_counts = (counts.tolist(), rc)
        for r in recvs:
            if r.numel():
                eng.submit_superkmers_device(r.data_ptr(), r.numel() // self.rec_words)
        eng.finalize(prune=prune)
        t.append(time.perf_counter())
        # host wall time per stage (each ends in a stream synchronisation)
        self.last_times = {k: (t[i + 1] - t[i]) * 1e3
                           for i, k in enumerate(("plan_ms", "pack_ms", "exchange_ms", "receive_ms"))}

    # ---- pipelined steps: the record exchange of the next unit overlaps the
    # binning of this one.  send() scatters a unit on the sender context and
    # starts its all-to-all; receive() waits for it and bins on self.engine.
    # Every rank must call them in the same order (the collectives pair up).
    def send(self, words: torch.Tensor, lens: torch.Tensor, n_reads: int, words_per_read: int,
             first_id: int, part: int = 0, n_parts: int = 1):
        if self._sender is None:
            K, M, cutoff, max_read_len, device, flags = self._engine_args
            self._sender = Engine(K, M, cutoff=cutoff, max_read_len=max_read_len, device=device,
                                  flags=flags)
        eng = self._sender
        t0 = time.perf_counter()
        eng.reset()
        eng.submit_packed_device(words.data_ptr(), lens.data_ptr(), n_reads, words_per_read,
                                 first_id)
        if n_parts > 1:
            eng.set_partition(part, n_parts)
        slot = self._slot
        self._slot ^= 1  # (the other buffer may still be in flight)
        counts = self._scatter(n_reads, engine=eng, slot=slot) if self.scatter else None
        if counts is not None:  # one pass: records straight into destination regions
            t1 = time.perf_counter()
            recvs, rc, work = exchange_regions_async(self._pregions[slot], counts.tolist(), self._wcap,
                                                     self.rec_words, self.group)
        else:  # plan / pack (table engine): destination-major, read order
            counts = eng.route_plan(self.world)
            words_needed = int(counts.sum()) * self.rec_words
            if self._pregions[slot].numel() < words_needed:
                self._pregions[slot] = torch.empty(int(words_needed * 1.25) + 1024, dtype=torch.int64,
                                                   device=self.device)
            eng.route_pack(self._pregions[slot].data_ptr())  # synchronises the engine stream
            t1 = time.perf_counter()
            recvs, rc, work = exchange_records_async(self._pregions[slot], counts.tolist(), self.rec_words,
                                                     self.group)
        t2 = time.perf_counter()
        return {"recvs": recvs, "rc": rc, "work": work, "part": part, "n_parts": n_parts,
                "counts": counts.tolist(), "times": (t1 - t0, t2 - t1)}

    def wait(self, unit) -> None:
        """the unit's records have landed (receive may follow)"""
        if unit["work"] is not None:
            unit["work"].wait()
            unit["work"] = None
        torch.cuda.current_stream(self.device).synchronize()

    def discard(self, unit) -> None:
        """drop a unit nobody receives (its records land, unbinned)"""
        self.wait(unit)

    def receive(self, unit, prune: bool = True) -> None:
        eng = self.engine
        t0 = time.perf_counter()
        self.wait(unit)
        t1 = time.perf_counter()
        eng.reset()
        if unit["n_parts"] > 1:
            eng.set_partition(unit["part"], unit["n_parts"])
        self._recv = unit["recvs"]  # referenced by the engine until the next reset
        self.last_counts = (unit["counts"], unit["rc"])
        for r in unit["recvs"]:
            if r.numel():
                eng.submit_superkmers_device(r.data_ptr(), r.numel() // self.rec_words)
        eng.finalize(prune=prune)
        t2 = time.perf_counter()
        self.last_times = {"plan_ms": unit["times"][0] * 1e3, "pack_ms": 0.0,
                           "exchange_ms": unit["times"][1] * 1e3 + (t1 - t0) * 1e3,
                           "receive_ms": (t2 - t1) * 1e3}


class HostCollectives:
    """The host transport of a C group (kb_group_create_rank_host) over a
    torch.distributed gloo process group of its own (the group's sender thread
    calls these while the caller's thread may run collectives of its own on
    the default group): the counts all-gather and the records' all-to-all, on
    CPU tensors.  Exceptions become a failed unit (non-zero return)."""

    def __init__(self, group=None):
        ranks = list(range(dist.get_world_size(group))) if group is None else dist.get_process_group_ranks(group)
        self.pg = dist.new_group(ranks=ranks, backend="gloo")
        self.world = len(ranks)
        self.errors = []

    def allgather(self, user, mine, n, out) -> int:
        try:
            t = torch.from_numpy(np.ctypeslib.as_array(mine, shape=(n,)).view(np.int64).copy())
            got = [torch.empty(n, dtype=torch.int64) for _ in range(self.world)]
            dist.all_gather(got, t, group=self.pg)
            np.ctypeslib.as_array(out, shape=(n * self.world,)).view(np.int64)[:] = torch.cat(got).numpy()
            return 0
        except Exception as e:  # (reported by the unit's receive)
            self.errors.append(repr(e))
            return 1

    def alltoallv(self, user, send, send_bytes, recv, recv_bytes) -> int:
        try:
            sb = [int(x) for x in np.ctypeslib.as_array(send_bytes, shape=(self.world,))]
            rb = [int(x) for x in np.ctypeslib.as_array(recv_bytes, shape=(self.world,))]
            inp = torch.from_numpy(np.ctypeslib.as_array(C.cast(send, C.POINTER(C.c_uint8)), shape=(max(1, sum(sb)),))
                                   [:sum(sb)].copy())
            out = torch.empty(sum(rb), dtype=torch.uint8)
            dist.all_to_all_single(out, inp, output_split_sizes=rb, input_split_sizes=sb, group=self.pg)
            if sum(rb):
                C.memmove(recv, out.data_ptr(), sum(rb))
            return 0
        except Exception as e:
            self.errors.append(repr(e))
            return 1


class GroupBinner(ShardedBinner):
    """ShardedBinner over the C-ABI multi-GPU group: kb_group_create_rank on
    this rank's device (torch.distributed broadcasts the 128-byte RCCL unique
    id, nothing else), then per unit kb_group_send (route, counts all-gather,
    records by grouped ncclSend/ncclRecv -- left in flight) and
    kb_group_receive (bin on the receiver).  Same interface: step, send /
    receive / wait, engine (the receiver context), last_times, last_counts."""

    def __init__(self, K: int, M: int, cutoff: int, max_read_len: int, device: int = 0,
                 group=None, flags: int = 0, transport: str | None = None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = torch.device("cuda", device)
        if dist.get_backend(group) == "nccl":
            box = [group_unique_id() if self.rank == 0 else None]
            dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                       group=group)
            self.grp = Group(K, M, cutoff=cutoff, max_read_len=max_read_len, rank=self.rank, n_ranks=self.world,
                             unique_id=box[0], device=device, flags=flags)
        else:  # (gloo: the C group over host collectives -- the rehearsal of the RCCL path's bookkeeping)
            self._host = HostCollectives(group)
            self.grp = Group(K, M, cutoff=cutoff, max_read_len=max_read_len, rank=self.rank, n_ranks=self.world,
                             device=device, flags=flags, host=(self._host.allgather, self._host.alltoallv))
        self.engine = self.grp.ctx(0)
        self.rec_words = self.engine.record_words()  # (the routed record's int64 words: exchange accounting)
        self.last_counts = None
        self.last_times = {}
        self._prune = True
        self._units = []  # units in flight, oldest first

    def _load(self, words, lens, n_reads, words_per_read, first_id, part, n_parts):
        self.grp.reset()
        self.grp.submit_packed_device(0, words.data_ptr(), lens.data_ptr(), n_reads, words_per_read, first_id)
        if n_parts > 1:
            self.grp.set_partition(part, n_parts)

    def step(self, words: torch.Tensor, lens: torch.Tensor, n_reads: int, words_per_read: int,
             first_id: int, prune: bool = True, part: int = 0, n_parts: int = 1) -> None:
        unit = self.send(words, lens, n_reads, words_per_read, first_id, part, n_parts)
        self.receive(unit, prune)

    def send(self, words: torch.Tensor, lens: torch.Tensor, n_reads: int, words_per_read: int,
             first_id: int, part: int = 0, n_parts: int = 1):
        """queue the unit (kb_group_send_async): its routing and exchange run
        on the group's sender thread while the caller receives the last one"""
        t0 = time.perf_counter()
        self._load(words, lens, n_reads, words_per_read, first_id, part, n_parts)
        self.grp.send_async()
        unit = {"counts": None, "part": part, "n_parts": n_parts, "times": (time.perf_counter() - t0, 0.0)}
        self._units.append(unit)
        return unit

    def wait(self, unit) -> None:
        """ShardedBinner.wait's contract (the unit may still be received):
        kb_group_receive waits for the unit's send stage and records itself,
        so nothing is to be done here"""
        assert unit in self._units, "a unit in flight"

    def discard(self, unit) -> None:
        """drop a unit nobody receives (its records land, unbinned); the
        unit's counts are then known (unit["counts"])"""
        assert self._units and self._units[0] is unit, "units leave in the order they were sent"
        self._units.pop(0)
        self.grp.discard()
        unit["counts"] = self.grp.unit_counts()

    def receive(self, unit, prune: bool = True) -> None:
        assert self._units and self._units[0] is unit, "units are received in the order they were sent"
        t0 = time.perf_counter()
        self._units.pop(0)
        self.grp.receive(prune)
        c = unit["counts"] = self.grp.unit_counts()
        self.last_counts = (c[self.rank].tolist(), c[:, self.rank].tolist())
        self.last_times = {"plan_ms": unit["times"][0] * 1e3, "pack_ms": 0.0, "exchange_ms": 0.0,
                           "receive_ms": (time.perf_counter() - t0) * 1e3}
