"""TEST INFRASTRUCTURE: a pure-Python restatement of the super-k-mer record
format of the multi-GPU path (include/kbin.h "multi-GPU routing",
csrc/kbin_kernels.hip route_kernel / insert_sk_kernel), small inputs only.

Used (a) by the world_size-2 gloo test to drive the product's exchange code
(kbin.dist.exchange_records) on CPU, and (b) pinned byte-for-byte against the
records the HIP route kernel packs (tests/test_gpu_dist.py)."""
from __future__ import annotations

import numpy as np

from kbin.dist import owner_of

V = {ord("T"): 0, ord("G"): 1, ord("C"): 2, ord("A"): 3}  # getval, binning.c:91-111


def superkmers(read: bytes, K: int, M: int):
    """(i0, n, sig_off, canonical mmer) per signature segment of one read:
    sticky chain of binning.c:922 -- a fresh leftmost-argmax signature at the
    first k-mer past the previous one."""
    L = len(read)
    nK = L - K + 1
    if nK <= 0:
        return []
    v = [V[b] for b in read]
    mask = (1 << (2 * M)) - 1
    s = [0] * (L - M + 1)
    for p in range(L - M + 1):
        x = 0
        for j in range(M):
            x = x * 4 + v[p + j]
        s[p] = x
    c = [max(x, mask - x) for x in s]
    out = []
    lo = 0
    while lo < nK:
        best = lo
        for p in range(lo, lo + K - M + 1):
            if c[p] > c[best]:
                best = p
        n = min(best, nK - 1) - lo + 1
        out.append((lo, n, best - lo, c[best]))
        lo = best + 1
    return out


def rec_words(K: int, M: int) -> int:
    return 1 + (2 * K - M + 31) // 32


def _word(v, p):
    """32 bases from position p, first base in the MSBs, zeros past the end"""
    w = 0
    for j in range(32):
        w = (w << 2) | (v[p + j] if p + j < len(v) else 0)
    return w


def _in_part(mmer: int, part: int, n_parts: int) -> bool:
    """kb_set_partition membership (route_in_part, csrc/kbin_kernels.hip)"""
    from kbin.dist import _mix64
    return n_parts <= 1 or (_mix64(mmer + 0x9E3779B97F4A7C15) >> 32) % n_parts == part


def encode(reads, ids, K: int, M: int, G: int, part: int = 0, n_parts: int = 1):
    """dest-major record buffer (uint64) + per-destination counts, in read
    order; n_parts > 1: only pass `part`'s records, to that pass's owners"""
    rw = rec_words(K, M)
    per = [[] for _ in range(G)]
    for read, rid in zip(reads, ids):
        v = [V[b] for b in read]
        for i0, n, so, cm in superkmers(read, K, M):
            sm = 0
            for b in v[i0 + so:i0 + so + M]:
                sm = sm * 4 + b
            rev = 1 if sm < (1 << (2 * M - 1)) else 0  # the complement flag (kbin_internal.h ROUTED_REV_BIT)
            rec = [int(rid) | (i0 << 32) | (n << 48) | (so << 54) | (rev << 60)]
            for w in range(rw - 1):
                p = i0 + 32 * w
                rec.append(_word(v, p) if p < len(v) else 0)
            if not _in_part(cm, part, n_parts):
                continue
            per[owner_of(cm, G, K, M, part, n_parts)].append(rec)
    counts = [len(x) for x in per]
    flat = [w for d in per for rec in d for w in rec]
    return np.array(flat, dtype=np.uint64).reshape(-1), counts


def decode(recs: np.ndarray, K: int, M: int):
    """(mmer, kmer_code, id) per k-mer occurrence of received records"""
    rw = rec_words(K, M)
    recs = np.asarray(recs, dtype=np.uint64).reshape(-1, rw)
    mask = (1 << (2 * M)) - 1
    kmask = (1 << (2 * K)) - 1
    out = []
    for rec in recs:
        h = int(rec[0])
        rid, i0, n, so = h & 0xFFFFFFFF, (h >> 32) & 0xFFFF, (h >> 48) & 63, (h >> 54) & 63
        bits = 0
        for w in rec[1:]:
            bits = (bits << 64) | int(w)
        nb = 32 * (rw - 1)

        def sub(p, m):
            return (bits >> (2 * (nb - p - m))) & ((1 << (2 * m)) - 1)

        sm = sub(so, M)
        rev = sm < (1 << (2 * M - 1))
        mm = mask - sm if rev else sm
        for j in range(n):
            km = sub(j, K)
            if rev:
                km ^= kmask
            out.append((mm, km, rid))
    return out


def bin_occurrences(occ, cutoff=1, prune=True):
    """{(mmer, kmer): [ids in reverse call order]} (ids increase with call order)"""
    d = {}
    for mm, km, rid in occ:
        d.setdefault((mm, km), []).append(rid)
    res = {}
    for k, v in d.items():
        if not prune or len(v) > cutoff:
            res[k] = sorted(v, reverse=True)
    return res


def oracle_dict(ora):
    res = {}
    for e in range(ora.n_entries):
        key = (int(ora.mmer[e]), (int(ora.kmer_hi[e]) << 64) | int(ora.kmer_lo[e]))
        res[key] = [int(x) for x in ora.ids[int(ora.offset[e]):int(ora.offset[e + 1])]]
    return res
