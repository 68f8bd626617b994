"""ctypes binding of libkbin.so -- the MI355X k-mer binning engine.

Mirrors the reference operator surface (binning.c process_read / prune_data)
for Python callers: an :class:`Engine` is one two-level mmer->kmer table
(binning.c:1151 zcreate_hash_table), :meth:`Engine.submit` stands for the
stream of process_read calls (binning.c:1165) and :meth:`Engine.finalize`
for prune_data (binning.c:1169).  Results come back as a :class:`Result`
CSR.  The engine is HIP-only: importing works anywhere, but creating an
Engine without the built library or a GPU raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib
from dataclasses import dataclass

import numpy as np

_HERE = pathlib.Path(__file__).resolve().parent
PKG_ROOT = _HERE.parent                       # genome-assembly_amd/
REPO_ROOT = PKG_ROOT.parent
LIB_DIR = PKG_ROOT / "lib"
LIB_PATH = LIB_DIR / "libkbin.so"
HOST_LIB_PATH = LIB_DIR / "libkbin_host.so"
INCLUDE_DIR = REPO_ROOT / "include"

KB_OK, KB_EINVAL, KB_ENOMEM, KB_EDEVICE, KB_EALPHABET, KB_ETOOLONG, KB_ESTATE, KB_EOVERFLOW = range(8)
_ERRNAMES = {0: "KB_OK", 1: "KB_EINVAL", 2: "KB_ENOMEM", 3: "KB_EDEVICE", 4: "KB_EALPHABET",
             5: "KB_ETOOLONG", 6: "KB_ESTATE", 7: "KB_EOVERFLOW"}

# symbols include/kbin.h declares (tests check every one is exported)
EXPORTED = [
    "kb_create", "kb_destroy", "kb_submit", "kb_submit_ids", "kb_submit_packed_device",
    "kb_finalize", "kb_export", "kb_export_device", "kb_reset", "kb_set_timing",
    "kb_get_timing", "kb_generate_reads_device", "kb_generate_reads_device_at", "kb_unpack_reads_to_host", "kb_stream",
    "kb_last_error", "kb_abi_version", "kb_record_words", "kb_route_plan", "kb_route_pack",
    "kb_submit_superkmers_device", "kb_route_scatter", "kb_split_passes", "kb_set_partition", "kb_digest",
    "kb_group_unique_id", "kb_group_create", "kb_group_create_rank", "kb_group_destroy", "kb_group_info",
    "kb_group_submit_ids", "kb_group_submit_packed_device", "kb_group_set_partition", "kb_group_send",
    "kb_group_receive", "kb_group_finalize", "kb_group_discard", "kb_group_reset", "kb_group_ctx",
    "kb_group_send_async", "kb_group_unit_counts", "kb_group_create_rank_host", "kb_owner_table",
]
KB_TRANSPORT_RCCL, KB_TRANSPORT_LOCAL = 1, 2


class KbError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{_ERRNAMES.get(code, code)}: {msg}")
        self.code = code


class kb_params(C.Structure):
    _fields_ = [("K", C.c_int32), ("M", C.c_int32), ("cutoff", C.c_int32),
                ("max_read_len", C.c_int32), ("device", C.c_int32), ("flags", C.c_int32),
                ("table_slots", C.c_uint64)]


class kb_csr(C.Structure):
    _fields_ = [("n_entries", C.c_uint64), ("n_ids", C.c_uint64), ("n_kmers", C.c_uint64),
                ("n_distinct", C.c_uint64),
                ("mmer", C.POINTER(C.c_uint32)), ("kmer_hi", C.POINTER(C.c_uint64)),
                ("kmer_lo", C.POINTER(C.c_uint64)), ("count", C.POINTER(C.c_uint32)),
                ("offset", C.POINTER(C.c_uint64)), ("ids", C.POINTER(C.c_int32)),
                ("first", C.POINTER(C.c_uint64))]


KB_TRACK_FIRST = 1
KB_ENGINE_TABLE = 2
KB_ENGINE_BINNED = 4
KB_ENG_TABLE, KB_ENG_BINNED = 1, 2


class kb_timing(C.Structure):
    _fields_ = [("scan_insert_ms", C.c_float), ("sort_ms", C.c_float),
                ("runs_ms", C.c_float), ("emit_ms", C.c_float), ("total_ms", C.c_float),
                ("scan_insert_launches", C.c_uint32), ("sort_passes", C.c_uint32),
                ("table_slots", C.c_uint64), ("engine", C.c_uint32), ("n_bins", C.c_uint32),
                ("n_superkmers", C.c_uint64), ("bin_kernel_ms", C.c_float),
                # path counters (kbin.h): which bin-phase paths the finalize took
                ("heavy_bins", C.c_uint32), ("split_bins", C.c_uint32), ("partitions", C.c_uint64),
                ("offset_partitions", C.c_uint64), ("flat_partitions", C.c_uint64),
                ("max_depth", C.c_uint32), ("overflow_redos", C.c_uint32), ("prefiltered", C.c_uint64),
                ("long_lists", C.c_uint32), ("clustered_lists", C.c_uint32),
                ("split_mmers", C.c_uint32), ("tail_reruns", C.c_uint32),
                ("light_prefilter_bins", C.c_uint32), ("ranked_bins", C.c_uint32),
                ("bitmap_partitions", C.c_uint32)]


_lib = None


def load_library(path: os.PathLike | str | None = None) -> C.CDLL:
    """Load libkbin.so (raises if it is not built -- no fallback)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # KB_LIB_PATH: load an alternative build (A/B experiments)
    p = pathlib.Path(path) if path else pathlib.Path(os.environ.get("KB_LIB_PATH", LIB_PATH))
    # One HIP runtime per process: torch ships its own libamdhip64.so (same
    # SONAME as /opt/rocm's).  If torch is importable it must be loaded first so
    # libkbin.so binds to that copy instead of pulling in a second runtime.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    if not p.exists():
        raise FileNotFoundError(f"{p} not built; run `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(str(p))
    vp, u64, u32, i32 = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int32
    lib.kb_create.argtypes = [C.POINTER(kb_params), C.POINTER(vp)]
    lib.kb_destroy.argtypes = [vp]
    lib.kb_destroy.restype = None
    lib.kb_submit.argtypes = [vp, C.c_char_p, C.POINTER(u32), u64, i32]
    lib.kb_submit_ids.argtypes = [vp, C.c_char_p, C.POINTER(u32), u64, C.POINTER(i32)]
    lib.kb_submit_packed_device.argtypes = [vp, vp, vp, u64, u32, i32]
    lib.kb_finalize.argtypes = [vp, C.c_int]
    lib.kb_export.argtypes = [vp, C.POINTER(kb_csr)]
    lib.kb_export_device.argtypes = [vp, C.POINTER(kb_csr)]
    lib.kb_reset.argtypes = [vp]
    lib.kb_set_timing.argtypes = [vp, C.c_int]
    lib.kb_get_timing.argtypes = [vp, C.POINTER(kb_timing)]
    lib.kb_generate_reads_device.argtypes = [C.c_int, vp, vp, u64, u32, u64, u32, u64]
    lib.kb_generate_reads_device_at.argtypes = [C.c_int, vp, vp, u64, u32, u64, u32, u64, u64]
    lib.kb_unpack_reads_to_host.argtypes = [C.c_int, vp, vp, u64, u32, C.c_char_p, C.POINTER(u32)]
    lib.kb_record_words.argtypes = [vp, C.POINTER(u32)]
    lib.kb_owner_table.argtypes = [C.c_int, C.c_int, u32, u32, u32, C.POINTER(C.c_uint8)]
    lib.kb_route_plan.argtypes = [vp, u32, C.POINTER(u64)]
    lib.kb_route_pack.argtypes = [vp, vp]
    lib.kb_submit_superkmers_device.argtypes = [vp, vp, u64]
    lib.kb_route_scatter.argtypes = [vp, C.c_uint32, vp, u64, C.POINTER(C.c_uint64)]
    lib.kb_split_passes.argtypes = [vp, C.c_uint32, vp, u64, C.POINTER(C.c_uint64)]
    lib.kb_set_partition.argtypes = [vp, u32, u32]
    lib.kb_digest.argtypes = [vp, C.POINTER(u64)]
    lib.kb_stream.argtypes = [vp]
    lib.kb_stream.restype = vp
    lib.kb_last_error.argtypes = []
    lib.kb_last_error.restype = C.c_char_p
    lib.kb_abi_version.restype = C.c_int
    lib.kb_group_unique_id.argtypes = [vp, C.c_size_t]
    lib.kb_group_create.argtypes = [C.POINTER(kb_params), C.c_int, C.POINTER(C.c_int), C.POINTER(vp)]
    lib.kb_group_create_rank.argtypes = [C.POINTER(kb_params), C.c_int, C.c_int, vp, C.c_size_t, C.POINTER(vp)]
    lib.kb_group_destroy.argtypes = [vp]
    lib.kb_group_destroy.restype = None
    lib.kb_group_info.argtypes = [vp] + [C.POINTER(C.c_int)] * 4
    lib.kb_group_submit_ids.argtypes = [vp, C.c_int, C.c_char_p, C.POINTER(u32), u64, C.POINTER(i32)]
    lib.kb_group_submit_packed_device.argtypes = [vp, C.c_int, vp, vp, u64, u32, i32]
    lib.kb_group_set_partition.argtypes = [vp, u32, u32]
    lib.kb_group_send.argtypes = [vp, C.POINTER(u64)]
    # (A/B builds of an earlier tree -- KB_LIB_PATH -- may lack the newest calls)
    for name, at in (("kb_group_send_async", [vp]), ("kb_group_unit_counts", [vp, C.POINTER(u64)]),
                     ("kb_group_create_rank_host", [C.POINTER(kb_params), C.c_int, C.c_int,
                                                    C.POINTER(kb_group_host_transport), C.POINTER(vp)])):
        if hasattr(lib, name):
            getattr(lib, name).argtypes = at
    lib.kb_group_receive.argtypes = [vp, C.c_int]
    lib.kb_group_finalize.argtypes = [vp, C.c_int]
    lib.kb_group_reset.argtypes = [vp]
    lib.kb_group_discard.argtypes = [vp]
    lib.kb_group_ctx.argtypes = [vp, C.c_int]
    lib.kb_group_ctx.restype = vp
    for name in EXPORTED:
        if name not in ("kb_destroy", "kb_stream", "kb_last_error", "kb_group_destroy", "kb_group_ctx") and \
                hasattr(lib, name):  # (test_abi checks that every one is exported)
            getattr(lib, name).restype = C.c_int
    if path is None:
        _lib = lib
    return lib


def _check(lib, rc: int) -> None:
    if rc != KB_OK:
        raise KbError(rc, lib.kb_last_error().decode(errors="replace"))


@dataclass
class Result:
    """Post-prune CSR: entry e is the key (mmer[e], kmer_hi[e]:kmer_lo[e]) with
    count[e] read ids ids[offset[e]:offset[e+1]] in reverse call order."""
    mmer: np.ndarray
    kmer_hi: np.ndarray
    kmer_lo: np.ndarray
    count: np.ndarray
    offset: np.ndarray
    ids: np.ndarray
    n_kmers: int
    n_distinct: int
    first: np.ndarray | None = None  # (ordinal << 16 | i) with KB_TRACK_FIRST

    @property
    def n_entries(self) -> int:
        return int(self.mmer.shape[0])

    def canonical(self) -> "Result":
        """Entries in canonical dump order: bytewise (mmer, kmer) ascending,
        i.e. descending codes (A=3 > C=2 > G=1 > T=0)."""
        order = np.lexsort((self.kmer_lo, self.kmer_hi, self.mmer))[::-1]
        cnt = self.count[order]
        off = np.zeros(len(order) + 1, dtype=np.uint64)
        np.cumsum(cnt, out=off[1:])
        if len(order):
            starts = self.offset[:-1][order].astype(np.int64)
            idx = np.repeat(starts - off[:-1].astype(np.int64), cnt.astype(np.int64)) + \
                np.arange(int(off[-1]), dtype=np.int64)
            ids = self.ids[idx]
        else:
            ids = self.ids[:0]
        return Result(self.mmer[order], self.kmer_hi[order], self.kmer_lo[order], cnt, off, ids,
                      self.n_kmers, self.n_distinct,
                      None if self.first is None else self.first[order])


    @staticmethod
    def concat(parts) -> "Result":
        """union of disjoint results (the passes of kb_set_partition): entries
        concatenated, each part's offsets shifted past the ids before it"""
        parts = list(parts)
        base = np.cumsum([0] + [len(r.ids) for r in parts])
        off = [np.zeros(1, dtype=np.uint64)] + [r.offset[1:].astype(np.uint64) + np.uint64(b)
                                                 for r, b in zip(parts, base[:-1])]
        cat = lambda f, dt: np.concatenate([getattr(r, f) for r in parts]).astype(dt)  # noqa: E731
        first = None if any(r.first is None for r in parts) else cat("first", np.uint64)
        return Result(cat("mmer", np.uint32), cat("kmer_hi", np.uint64), cat("kmer_lo", np.uint64),
                      cat("count", np.uint32), np.concatenate(off), cat("ids", np.int32),
                      sum(r.n_kmers for r in parts), sum(r.n_distinct for r in parts), first)


def _mix64_np(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser, uint64 wrap-around (kbin_device.h mix64)"""
    x = x.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(30)
        x *= np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(27)
        x *= np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(31)
    return x


def result_digest(res: "Result") -> tuple:
    """kb_digest (kbin.h) of a host result: (entries, ids, key sum, list sum)"""
    key = _mix64_np(_mix64_np(_mix64_np(res.mmer.astype(np.uint64)) ^ res.kmer_hi.astype(np.uint64))
                    ^ res.kmer_lo.astype(np.uint64))
    cnt = res.count.astype(np.uint64)
    dk = int(_mix64_np(key ^ (cnt << np.uint64(1))).sum(dtype=np.uint64))
    n = len(res.ids)
    if n:
        e_of = np.repeat(np.arange(res.n_entries), res.count.astype(np.int64))
        j = np.arange(n, dtype=np.int64) - res.offset[:-1].astype(np.int64)[e_of] + 1
        ids = res.ids.astype(np.int64) & 0xFFFFFFFF
        t = key[e_of] ^ ((j.astype(np.uint64) << np.uint64(32)) | ids.astype(np.uint64))
        dl = int(_mix64_np(t).sum(dtype=np.uint64))
    else:
        dl = 0
    return res.n_entries, n, dk, dl


_BP = np.frombuffer(b"TGCA", dtype=np.uint8)  # getbp (binning.c:69-88)


def decode(code_hi: int, code_lo: int, n: int) -> str:
    """Key string of an n-base code (first base most significant)."""
    v = (int(code_hi) << 64) | int(code_lo)
    out = bytearray(n)
    for j in range(n - 1, -1, -1):
        out[j] = _BP[v & 3]
        v >>= 2
    return out.decode()


def dump_lines(res: Result, K: int, M: int):
    """Canonical dump lines: mmer\\tkmer\\tcount\\tids."""
    r = res.canonical()
    for e in range(r.n_entries):
        ids = r.ids[int(r.offset[e]):int(r.offset[e + 1])]
        yield "%s\t%s\t%d\t%s\n" % (decode(0, r.mmer[e], M), decode(r.kmer_hi[e], r.kmer_lo[e], K),
                                    int(r.count[e]), ",".join(str(int(x)) for x in ids))


def pack_reads(reads) -> tuple[bytes, np.ndarray]:
    """list of str/bytes reads -> (concatenated bytes, uint32 lengths)."""
    bs = [r.encode() if isinstance(r, str) else bytes(r) for r in reads]
    lens = np.fromiter((len(b) for b in bs), dtype=np.uint32, count=len(bs))
    return b"".join(bs), lens


class Engine:
    """One binning context on one GPU (C-ABI kb_ctx)."""

    def __init__(self, K: int, M: int, cutoff: int = 1, max_read_len: int = 1024,
                 device: int = 0, table_slots: int = 0, flags: int = 0, lib_path=None):
        self.lib = load_library(lib_path)
        self.K, self.M, self.cutoff = K, M, cutoff
        p = kb_params(K=K, M=M, cutoff=cutoff, max_read_len=max_read_len, device=device,
                      flags=flags, table_slots=table_slots)
        h = C.c_void_p()
        _check(self.lib, self.lib.kb_create(C.byref(p), C.byref(h)))
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None):
            self.lib.kb_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def submit(self, reads=None, *, bases: bytes | None = None, lens=None, first_id: int = 0,
               ids=None) -> None:
        """Append reads (list of strings, or bases+lens).  Read r gets id
        first_id + r unless `ids` is given (process_read's read_id)."""
        if reads is not None:
            bases, lens = pack_reads(reads)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        n = int(lens.shape[0])
        lp = lens.ctypes.data_as(C.POINTER(C.c_uint32))
        if ids is not None:
            ids = np.ascontiguousarray(ids, dtype=np.int32)
            _check(self.lib, self.lib.kb_submit_ids(self._h, bases, lp, n,
                                                    ids.ctypes.data_as(C.POINTER(C.c_int32))))
        else:
            _check(self.lib, self.lib.kb_submit(self._h, bases, lp, n, int(first_id)))

    def submit_packed_device(self, words_ptr: int, lens_ptr: int, n_reads: int,
                             words_per_read: int, first_id: int = 0) -> None:
        _check(self.lib, self.lib.kb_submit_packed_device(self._h, C.c_void_p(words_ptr),
                                                          C.c_void_p(lens_ptr), n_reads,
                                                          words_per_read, int(first_id)))

    # ---- multi-GPU routing (include/kbin.h; driven by kbin.dist) ----
    def record_words(self) -> int:
        w = C.c_uint32()
        _check(self.lib, self.lib.kb_record_words(self._h, C.byref(w)))
        return int(w.value)

    def route_plan(self, n_dest: int) -> np.ndarray:
        """super-k-mer records per destination for the reads submitted so far"""
        cnt = np.zeros(n_dest, dtype=np.uint64)
        _check(self.lib, self.lib.kb_route_plan(self._h, n_dest,
                                                cnt.ctypes.data_as(C.POINTER(C.c_uint64))))
        return cnt

    def route_pack(self, send_ptr: int) -> None:
        _check(self.lib, self.lib.kb_route_pack(self._h, C.c_void_p(send_ptr)))

    def route_scatter(self, n_dest: int, regions_ptr: int, region_cap: int):
        """one-pass sender: records into per-destination regions of region_cap
        records each; returns (ok, counts) -- ok False means a destination
        needs more room (counts say how much; nothing was shipped)"""
        cnt = np.zeros(n_dest, dtype=np.uint64)
        rc = self.lib.kb_route_scatter(self._h, n_dest, C.c_void_p(regions_ptr), int(region_cap),
                                       cnt.ctypes.data_as(C.POINTER(C.c_uint64)))
        if rc == KB_EOVERFLOW:
            return False, cnt
        _check(self.lib, rc)
        return True, cnt

    def split_passes(self, n_parts: int, regions_ptr: int, region_cap: int):
        """kb_split_passes: one super-k-mer pass into the regions of the
        n_parts kb_set_partition passes; (ok, counts) as route_scatter"""
        cnt = np.zeros(n_parts, dtype=np.uint64)
        rc = self.lib.kb_split_passes(self._h, n_parts, C.c_void_p(regions_ptr), int(region_cap),
                                      cnt.ctypes.data_as(C.POINTER(C.c_uint64)))
        if rc == KB_EOVERFLOW:
            return False, cnt
        _check(self.lib, rc)
        return True, cnt

    def submit_superkmers_device(self, recs_ptr: int, n_records: int) -> None:
        _check(self.lib, self.lib.kb_submit_superkmers_device(self._h, C.c_void_p(recs_ptr),
                                                              int(n_records)))

    def finalize(self, prune: bool = True) -> None:
        _check(self.lib, self.lib.kb_finalize(self._h, 1 if prune else 0))

    def reset(self) -> None:
        _check(self.lib, self.lib.kb_reset(self._h))

    def digest(self) -> tuple:
        """kb_digest of the last result: (entries, ids, key sum, list sum)"""
        out = (C.c_uint64 * 4)()
        _check(self.lib, self.lib.kb_digest(self._h, out))
        return tuple(int(x) for x in out)

    def set_partition(self, part: int, n_parts: int) -> None:
        """next finalize/route covers mmer partition `part` of `n_parts` only
        (kbin.h: partitioned passes; the read batches are kept)"""
        _check(self.lib, self.lib.kb_set_partition(self._h, int(part), int(n_parts)))

    def set_timing(self, on=True) -> None:
        """True / 1: every phase event; "kernel" / 2: only bin_kernel's (binned
        engine: no idle gaps from the phase events); False / 0: off"""
        mode = 2 if on == "kernel" else int(on)
        _check(self.lib, self.lib.kb_set_timing(self._h, mode))

    def timing_raw(self) -> "kb_timing":
        """the kb_timing struct itself (one call; timing_dict() converts it)"""
        t = kb_timing()
        _check(self.lib, self.lib.kb_get_timing(self._h, C.byref(t)))
        return t

    def timing(self) -> dict:
        return timing_dict(self.timing_raw())

    def stream(self) -> int:
        return self.lib.kb_stream(self._h) or 0

    def export(self) -> Result:
        c = kb_csr()
        _check(self.lib, self.lib.kb_export(self._h, C.byref(c)))
        n, m = int(c.n_entries), int(c.n_ids)

        def arr(ptr, count, dt):
            if count == 0:
                return np.zeros(0, dtype=dt)
            return np.ctypeslib.as_array(ptr, shape=(count,)).astype(dt, copy=True)

        return Result(arr(c.mmer, n, np.uint32), arr(c.kmer_hi, n, np.uint64),
                      arr(c.kmer_lo, n, np.uint64), arr(c.count, n, np.uint32),
                      arr(c.offset, n + 1, np.uint64), arr(c.ids, m, np.int32),
                      int(c.n_kmers), int(c.n_distinct),
                      arr(c.first, n, np.uint64) if bool(c.first) else None)

    def export_device(self) -> dict:
        c = kb_csr()
        _check(self.lib, self.lib.kb_export_device(self._h, C.byref(c)))
        return {f: (getattr(c, f) if f.startswith("n_") else C.cast(getattr(c, f), C.c_void_p).value)
                for f, _ in kb_csr._fields_}


class _CtxView(Engine):
    """a context owned by something else (a group's receiver): the Engine
    result/timing methods, no ownership"""

    def __init__(self, lib, handle: int, K: int, M: int, cutoff: int):
        self.lib, self._h = lib, C.c_void_p(handle)
        self.K, self.M, self.cutoff = K, M, cutoff

    def close(self) -> None:
        self._h = None


def group_unique_id() -> bytes:
    """128-byte RCCL unique id for kb_group_create_rank (made once, by one
    process, and handed to every rank by the caller)"""
    lib = load_library()
    buf = C.create_string_buffer(128)
    _check(lib, lib.kb_group_unique_id(buf, 128))
    return buf.raw


KB_TRANSPORT_HOST = 3
HOST_ALLGATHER = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.c_uint64, C.POINTER(C.c_uint64))
HOST_ALLTOALLV = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_void_p,
                             C.POINTER(C.c_uint64))


class kb_group_host_transport(C.Structure):
    _fields_ = [("user", C.c_void_p), ("allgather", HOST_ALLGATHER), ("alltoallv", HOST_ALLTOALLV)]


class Group:
    """A multi-GPU binning group (kbin.h "multi-GPU groups"): G ranks sharded
    by canonical mmer; records exchanged over RCCL from C (or device copies
    for virtual shards on one device).  devices: every rank in this process
    (kb_group_create); rank/n_ranks/unique_id: this process is one rank
    (kb_group_create_rank on `device`); rank/n_ranks/host=(allgather,
    alltoallv): one rank whose counts and records move through the caller's
    host-memory collectives (kb_group_create_rank_host; kbin.dist builds them
    on a gloo process group)."""

    def __init__(self, K: int, M: int, cutoff: int = 1, max_read_len: int = 1024, *, devices=None,
                 rank: int | None = None, n_ranks: int | None = None, unique_id: bytes | None = None,
                 device: int = 0, flags: int = 0, lib_path=None, host=None):
        self.lib = load_library(lib_path)
        self.K, self.M, self.cutoff = K, M, cutoff
        p = kb_params(K=K, M=M, cutoff=cutoff, max_read_len=max_read_len, device=device, flags=flags,
                      table_slots=0)
        h = C.c_void_p()
        if rank is None:
            devs = list(devices) if devices is not None else [device]
            arr = (C.c_int * len(devs))(*devs)
            _check(self.lib, self.lib.kb_group_create(C.byref(p), len(devs), arr, C.byref(h)))
        elif host is not None:
            # (the callbacks live as long as the group: the sender thread calls them)
            self._ht = kb_group_host_transport(None, HOST_ALLGATHER(host[0]), HOST_ALLTOALLV(host[1]))
            _check(self.lib, self.lib.kb_group_create_rank_host(C.byref(p), int(rank), int(n_ranks),
                                                                C.byref(self._ht), C.byref(h)))
        else:
            _check(self.lib, self.lib.kb_group_create_rank(C.byref(p), int(rank), int(n_ranks), unique_id,
                                                           len(unique_id), C.byref(h)))
        self._h = h
        n, nl, r0, tr = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        _check(self.lib, self.lib.kb_group_info(self._h, C.byref(n), C.byref(nl), C.byref(r0), C.byref(tr)))
        self.n_ranks, self.n_local, self.rank0, self.transport = n.value, nl.value, r0.value, tr.value

    def close(self) -> None:
        if getattr(self, "_h", None):
            self.lib.kb_group_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def submit(self, local: int, reads=None, *, bases: bytes | None = None, lens=None, ids=None,
               first_id: int = 0) -> None:
        if reads is not None:
            bases, lens = pack_reads(reads)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        n = int(lens.shape[0])
        if ids is None:
            ids = np.arange(first_id, first_id + n, dtype=np.int32)
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        _check(self.lib, self.lib.kb_group_submit_ids(self._h, int(local), bases,
                                                      lens.ctypes.data_as(C.POINTER(C.c_uint32)), n,
                                                      ids.ctypes.data_as(C.POINTER(C.c_int32))))

    def submit_packed_device(self, local: int, words_ptr: int, lens_ptr: int, n_reads: int,
                             words_per_read: int, first_id: int = 0) -> None:
        _check(self.lib, self.lib.kb_group_submit_packed_device(self._h, int(local), C.c_void_p(words_ptr),
                                                                C.c_void_p(lens_ptr), n_reads, words_per_read,
                                                                int(first_id)))

    def set_partition(self, part: int, n_parts: int) -> None:
        _check(self.lib, self.lib.kb_group_set_partition(self._h, int(part), int(n_parts)))

    def send(self) -> np.ndarray:
        """route + start the exchange; returns the G x G record counts"""
        c = np.zeros(self.n_ranks * self.n_ranks, dtype=np.uint64)
        _check(self.lib, self.lib.kb_group_send(self._h, c.ctypes.data_as(C.POINTER(C.c_uint64))))
        return c.reshape(self.n_ranks, self.n_ranks)

    def send_async(self) -> None:
        """queue the unit on the group's sender thread (kb_group_send_async):
        returns at once; receive() / discard() report its failure"""
        _check(self.lib, self.lib.kb_group_send_async(self._h))

    def unit_counts(self) -> np.ndarray:
        """G x G record counts of the last unit received or discarded"""
        c = np.zeros(self.n_ranks * self.n_ranks, dtype=np.uint64)
        _check(self.lib, self.lib.kb_group_unit_counts(self._h, c.ctypes.data_as(C.POINTER(C.c_uint64))))
        return c.reshape(self.n_ranks, self.n_ranks)

    def receive(self, prune: bool = True) -> None:
        _check(self.lib, self.lib.kb_group_receive(self._h, 1 if prune else 0))

    def finalize(self, prune: bool = True) -> None:
        _check(self.lib, self.lib.kb_group_finalize(self._h, 1 if prune else 0))

    def reset(self) -> None:
        """drop the submitted reads (units in flight keep their records)"""
        _check(self.lib, self.lib.kb_group_reset(self._h))

    def discard(self) -> None:
        """wait for the oldest unit in flight and drop it unbinned"""
        _check(self.lib, self.lib.kb_group_discard(self._h))

    def ctx(self, local: int) -> Engine:
        """local rank's receiver context (export / digest / timing)"""
        h = self.lib.kb_group_ctx(self._h, int(local))
        if not h:
            raise KbError(KB_EINVAL, f"no local rank {local}")
        return _CtxView(self.lib, h, self.K, self.M, self.cutoff)


def timing_dict(t: "kb_timing") -> dict:
    return {f: getattr(t, f) for f, _ in kb_timing._fields_ if f != "reserved"}


def owner_table(K: int, M: int, n_dest: int, part: int = 0, n_parts: int = 1) -> np.ndarray:
    """kb_owner_table: the owner rank of every canonical mmer 2^(2M-1) + i
    (index i) for n_dest ranks in pass (part, n_parts) -- host only"""
    lib = load_library()
    out = np.zeros(1 << (2 * M - 1), dtype=np.uint8)
    _check(lib, lib.kb_owner_table(K, M, n_dest, part, n_parts, out.ctypes.data_as(C.POINTER(C.c_uint8))))
    return out


def generate_reads_device(words_ptr: int, lens_ptr: int, n_reads: int, read_len: int,
                          genome_len: int, err_per_million: int, seed: int, device: int = 0,
                          read_base: int = 0) -> None:
    """reads read_base .. read_base + n_reads - 1 of the stream `seed` defines
    (one genome per seed; kb_generate_reads_device_at)"""
    lib = load_library()
    _check(lib, lib.kb_generate_reads_device_at(device, C.c_void_p(words_ptr), C.c_void_p(lens_ptr),
                                                n_reads, read_len, genome_len, err_per_million, seed,
                                                int(read_base)))


def unpack_reads_to_host(words_ptr: int, lens_ptr: int, n_reads: int, words_per_read: int,
                         total_bases: int, device: int = 0) -> tuple[bytes, np.ndarray]:
    lib = load_library()
    buf = C.create_string_buffer(max(total_bases, 1))
    lens = np.zeros(n_reads, dtype=np.uint32)
    _check(lib, lib.kb_unpack_reads_to_host(device, C.c_void_p(words_ptr), C.c_void_p(lens_ptr),
                                            n_reads, words_per_read, buf,
                                            lens.ctypes.data_as(C.POINTER(C.c_uint32))))
    return buf.raw[:int(lens.sum())], lens
