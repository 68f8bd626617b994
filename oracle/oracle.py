"""TEST INFRASTRUCTURE ONLY -- ctypes binding of the parity oracle
(oracle/liboracle.so, a clean-room C restatement of binning.c's process_read
+ prune_data; see kb_oracle.c for the file:line map).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
"""
from __future__ import annotations

import ctypes as C
import pathlib
import subprocess

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"
REF_DIR = HERE / "_ref"


class kbo_result(C.Structure):
    _fields_ = [("n_entries", C.c_uint64), ("mmer", C.POINTER(C.c_uint32)),
                ("kmer_hi", C.POINTER(C.c_uint64)), ("kmer_lo", C.POINTER(C.c_uint64)),
                ("count", C.POINTER(C.c_uint32)), ("offset", C.POINTER(C.c_uint64)),
                ("ids", C.POINTER(C.c_int32)), ("n_kmers", C.c_uint64), ("alphabet_ok", C.c_int),
                ("first", C.POINTER(C.c_uint64))]


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        l = C.CDLL(str(LIB))
        l.kbo_bin.argtypes = [C.c_char_p, C.POINTER(C.c_uint64), C.c_uint64, C.POINTER(C.c_int32),
                              C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(kbo_result)]
        l.kbo_bin.restype = C.c_int
        l.kbo_bin_masked.argtypes = [C.c_char_p, C.POINTER(C.c_uint64), C.c_uint64, C.POINTER(C.c_int32),
                                     C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint8),
                                     C.POINTER(kbo_result)]
        l.kbo_bin_masked.restype = C.c_int
        l.kbo_free.argtypes = [C.POINTER(kbo_result)]
        l.kbo_free.restype = None
        l.kbo_read_fgets.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.POINTER(C.c_char)),
                                     C.POINTER(C.POINTER(C.c_uint64)), C.POINTER(C.c_uint64)]
        l.kbo_read_fgets.restype = C.c_int
        l.kbo_free_reads.argtypes = [C.c_void_p, C.c_void_p]
        l.kbo_free_reads.restype = None
        l.kbo_gen_reads.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint64,
                                    C.c_char_p]
        l.kbo_gen_reads.restype = None
        l.kbo_stream_digest.argtypes = [C.c_char_p, C.c_uint64, C.c_uint32, C.c_int, C.c_int, C.c_int, C.c_int,
                                        C.c_int32, C.c_int, C.c_int, C.POINTER(C.c_uint64)]
        l.kbo_stream_digest.restype = C.c_int
        l.kbo_gen_stream_digest.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint64,
                                            C.c_int, C.c_int, C.c_int, C.c_int, C.c_int32, C.c_int, C.c_int,
                                            C.POINTER(C.c_uint64)]
        l.kbo_gen_stream_digest.restype = C.c_int
        _lib = l
    return _lib


class OracleResult:
    """Same field names as kbin.Result, already in canonical order."""

    def __init__(self, mmer, kmer_hi, kmer_lo, count, offset, ids, n_kmers, alphabet_ok, first=None):
        self.mmer, self.kmer_hi, self.kmer_lo = mmer, kmer_hi, kmer_lo
        self.count, self.offset, self.ids = count, offset, ids
        self.n_kmers, self.alphabet_ok = n_kmers, alphabet_ok
        self.first = first  # per entry: call ordinal << 16 | k-mer position of its first occurrence

    @property
    def n_entries(self):
        return int(self.mmer.shape[0])


def bin_reads(bases: bytes, lens, K: int, M: int, cutoff: int = 1, prune: bool = True,
              ids=None, mmer_mask=None) -> OracleResult:
    """Run the oracle on concatenated reads (mmer_mask: uint8 per canonical
    mmer code, keys of unmasked mmers dropped -- one partition of a big input)."""
    l = lib()
    lens = np.asarray(lens, dtype=np.uint64)
    off = np.zeros(len(lens) + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    idp = None
    if ids is not None:
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        idp = ids.ctypes.data_as(C.POINTER(C.c_int32))
    r = kbo_result()
    maskp = None
    if mmer_mask is not None:
        mmer_mask = np.ascontiguousarray(mmer_mask, dtype=np.uint8)
        assert mmer_mask.size == 1 << (2 * M)
        maskp = mmer_mask.ctypes.data_as(C.POINTER(C.c_uint8))
    rc = l.kbo_bin_masked(bases, off.ctypes.data_as(C.POINTER(C.c_uint64)), len(lens), idp, K, M, cutoff,
                          1 if prune else 0, maskp, C.byref(r))
    if rc:
        raise RuntimeError(f"kbo_bin failed: {rc}")
    n = int(r.n_entries)
    try:
        def arr(p, cnt, dt):
            if cnt == 0:
                return np.zeros(0, dtype=dt)
            return np.ctypeslib.as_array(p, shape=(cnt,)).astype(dt, copy=True)
        off_a = arr(r.offset, n + 1, np.uint64)
        out = OracleResult(arr(r.mmer, n, np.uint32), arr(r.kmer_hi, n, np.uint64),
                           arr(r.kmer_lo, n, np.uint64), arr(r.count, n, np.uint32), off_a,
                           arr(r.ids, int(off_a[-1]) if n else 0, np.int32), int(r.n_kmers),
                           bool(r.alphabet_ok), arr(r.first, n, np.uint64))
    finally:
        l.kbo_free(C.byref(r))
    return out


def read_fgets(path, read_length: int) -> tuple[bytes, np.ndarray]:
    """binning.c:1150-1166 read loop restated (oracle side)."""
    l = lib()
    bp = C.POINTER(C.c_char)()
    op = C.POINTER(C.c_uint64)()
    n = C.c_uint64()
    rc = l.kbo_read_fgets(str(path).encode(), read_length, C.byref(bp), C.byref(op), C.byref(n))
    if rc:
        raise OSError(f"kbo_read_fgets({path}) failed: {rc}")
    try:
        nr = int(n.value)
        off = np.ctypeslib.as_array(op, shape=(nr + 1,)).copy()
        bases = C.string_at(bp, int(off[-1])) if off[-1] else b""
    finally:
        l.kbo_free_reads(C.cast(bp, C.c_void_p), C.cast(op, C.c_void_p))
    return bases, np.diff(off).astype(np.uint32)


def ref_binary(K: int, M: int, cutoff: int = 1) -> pathlib.Path | None:
    """oracle/_ref/ref_k*_m*_c* if it can be built here (reference present)."""
    p = REF_DIR / f"ref_k{K}_m{M}_c{cutoff}"
    if not p.exists():
        subprocess.run(["bash", str(HERE / "build_ref.sh"), str(K), str(M), str(cutoff)],
                       check=False, capture_output=True)
    return p if p.exists() else None


def gen_reads(n_reads: int, read_len: int, genome_len: int, err_ppm: int, seed: int, read_base: int = 0) -> bytes:
    """the device generator's reads (kb_generate_reads_device_at) on the CPU:
    n_reads x read_len ASCII bytes (oracle/kb_oracle.c kbo_gen_reads)"""
    buf = C.create_string_buffer(max(1, n_reads * read_len))
    lib().kbo_gen_reads(n_reads, read_len, genome_len, err_ppm, seed, read_base, buf)
    return buf.raw[:n_reads * read_len]


def _digest_out(rc, out):
    if rc:
        raise RuntimeError(f"kbo stream digest failed: {rc}")
    return tuple(int(x) for x in out[:4]), int(out[4])


def stream_digest(bases: bytes, n_reads: int, read_len: int, K: int, M: int, cutoff: int = 1, prune: bool = True,
                  id0: int = 0, workers: int = 4, cap_log2: int = 20):
    """kb_digest (entries, ids, key sum, list sum) of binning fixed-length
    reads, computed by the oracle's scan without holding the result; and the
    k-mers scanned"""
    out = (C.c_uint64 * 5)()
    rc = lib().kbo_stream_digest(bases, n_reads, read_len, K, M, cutoff, 1 if prune else 0, id0, workers, cap_log2,
                                 out)
    return _digest_out(rc, out)


def gen_stream_digest(n_reads: int, read_len: int, genome_len: int, err_ppm: int, seed: int, K: int, M: int,
                      cutoff: int = 1, prune: bool = True, read_base: int = 0, id0: int = 0, workers: int = 8,
                      cap_log2: int = 24):
    """stream_digest over gen_reads' reads (generated inside, 2-bit packed)"""
    out = (C.c_uint64 * 5)()
    rc = lib().kbo_gen_stream_digest(n_reads, read_len, genome_len, err_ppm, seed, read_base, K, M, cutoff,
                                     1 if prune else 0, id0, workers, cap_log2, out)
    return _digest_out(rc, out)
