"""The drop-in's DIRECT table layout (binning_gpu.c materialise_direct: the
zhash history replayed on integer codes, survivors only allocated) against the
REPLAY (zhash_set of every key in first-occurrence order, then the prune's
unlinks, zhash.c:53-76/184-214, binning.c:1085-1144) on synthetic CSRs:
identical size steps, bucket chains, chain order, keys and lists
(kbh_layout_digest).  No GPU: the CSR is host memory built here."""
import ctypes as C
import os
import pathlib

import numpy as np
import pytest

import kbin


def host_lib():
    lib = C.CDLL(str(kbin.HOST_LIB_PATH))
    lib.zcreate_hash_table.restype = C.c_void_p
    lib.kbh_materialise_csr.argtypes = [C.c_void_p, C.POINTER(kbin.kb_csr), C.c_int, C.c_int]
    lib.kbh_layout_digest.argtypes = [C.c_void_p]
    lib.kbh_layout_digest.restype = C.c_uint64
    lib.kbh_dump_table.argtypes = [C.c_void_p, C.c_void_p]
    return lib


def synthetic_csr(rng, n, K, M, heavy=0):
    """n distinct (mmer, kmer) keys with unique first-occurrence stamps,
    counts 1..4 (a third at 1: pruned at cutoff 1), `heavy` keys piled on one
    mmer (a table that climbs many ladder steps)"""
    nm = 1 << (2 * M)
    mmer = rng.integers(0, nm, n, dtype=np.uint64).astype(np.uint32)
    mmer[:heavy] = 5 % nm
    bits = 2 * K
    lo = rng.integers(0, 2**63, n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, n, dtype=np.uint64)
    hi = rng.integers(0, 2**63, n, dtype=np.uint64)
    if bits < 64:
        lo &= np.uint64((1 << bits) - 1)
        hi[:] = 0
    elif bits < 128:
        hi &= np.uint64((1 << (bits - 64)) - 1)
    lo[:] = lo ^ np.arange(n, dtype=np.uint64) << np.uint64(min(bits, 64) - 24)  # distinct keys
    if bits < 64:
        lo &= np.uint64((1 << bits) - 1)
    key = np.stack([mmer.astype(np.uint64), hi, lo], 1)
    assert len(np.unique(key, axis=0)) == n
    count = rng.choice([1, 1, 2, 3, 4], n).astype(np.uint32)
    offset = np.zeros(n + 1, np.uint64)
    offset[1:] = np.cumsum(count)
    ids = rng.integers(0, 1 << 30, int(offset[-1])).astype(np.int32)
    first = (rng.permutation(n).astype(np.uint64) << np.uint64(16)) | rng.integers(0, 300, n, dtype=np.uint64)
    arrays = dict(mmer=mmer, kmer_hi=hi, kmer_lo=lo, count=count, offset=offset, ids=ids, first=first)
    c = kbin.kb_csr()
    c.n_entries, c.n_ids = n, int(offset[-1])
    for f, a in arrays.items():
        setattr(c, f, a.ctypes.data_as(dict(kbin.kb_csr._fields_)[f]))
    return c, arrays


@pytest.mark.parametrize("n,K,M,heavy", [(0, 31, 7, 0), (1, 31, 7, 0), (3000, 31, 7, 0), (40000, 21, 3, 0),
                                         (20000, 31, 7, 12000), (20000, 63, 7, 3000), (5000, 32, 4, 0),
                                         (30000, 27, 6, 30000)])
@pytest.mark.parametrize("prune", [1, 0])
def test_direct_layout_equals_replay(n, K, M, heavy, prune):
    lib = host_lib()
    rng = np.random.default_rng(n + K + M + heavy)
    csr, keep = synthetic_csr(rng, n, K, M, heavy)
    assert lib.kbh_configure(K, M, 1, 0) == 0
    a, b = lib.zcreate_hash_table(), lib.zcreate_hash_table()
    assert lib.kbh_materialise_csr(a, C.byref(csr), prune, 1) == 0
    assert lib.kbh_materialise_csr(b, C.byref(csr), prune, 0) == 0
    assert lib.kbh_layout_digest(a) == lib.kbh_layout_digest(b)
    del keep


class _Node(C.Structure):
    pass


_Node._fields_ = [("next", C.POINTER(_Node)), ("item", C.c_void_p)]


class _Entry(C.Structure):
    pass


_Entry._fields_ = [("key", C.c_char_p), ("val", C.c_void_p), ("next", C.POINTER(_Entry))]


class _Table(C.Structure):
    _fields_ = [("size_index", C.c_size_t), ("entry_count", C.c_size_t), ("entries", C.POINTER(C.POINTER(_Entry)))]


LADDER = [53, 101, 211, 503, 1553, 3407, 6803, 12503, 25013, 50261, 104729, 250007, 500009, 1000003]


def _entries(tab_addr):
    t = _Table.from_address(tab_addr)
    for b in range(LADDER[t.size_index]):
        e = t.entries[b]
        while e:
            yield e.contents
            e = e.contents.next


def _chain(head_addr):
    """(node address, read id) of an ll_node list"""
    out = []
    p = head_addr
    while p:
        nd = _Node.from_address(p)
        out.append((p, C.c_int.from_address(p + 8).value))
        p = C.cast(nd.next, C.c_void_p).value
    return out


@pytest.mark.parametrize("threads", ["1", "5"])
@pytest.mark.parametrize("n,K,M", [(0, 31, 7), (600, 31, 7), (900, 21, 3), (300, 63, 7)])
def test_expand_read_id_list(n, K, M, threads, monkeypatch):
    """expand_read_id_list (binning.c:857-888) on materialised tables: every
    kmer entry's value becomes strlen(key) = K outer nodes (create_node_item,
    llist.c:13-18); the first holds the ORIGINAL list (same nodes), the other
    K - 1 hold fresh copies (duplicate_llist, llist.c:83-99): same ids in the
    same order, every node a distinct block.  Tables and keys are untouched."""
    monkeypatch.setenv("KBH_THREADS", threads)
    lib = host_lib()
    lib.expand_read_id_list.argtypes = [C.c_void_p]
    rng = np.random.default_rng(n + K)
    csr, keep = synthetic_csr(rng, n, K, M)
    assert lib.kbh_configure(K, M, 1, 0) == 0
    h = lib.zcreate_hash_table()
    assert lib.kbh_materialise_csr(h, C.byref(csr), 1, 0) == 0
    before = {}
    for me in _entries(h):
        for ke in _entries(me.val):
            before[(me.key, ke.key)] = (ke.val, _chain(ke.val))
    layout = lib.kbh_layout_digest(h)  # (walks the lists: taken before the expansion)
    lib.expand_read_id_list(h)
    seen = set()
    n_after = 0
    for me in _entries(h):
        for ke in _entries(me.val):
            head, ids = before[(me.key, ke.key)]
            outer = _chain(ke.val)
            assert len(outer) == len(ke.key) == K
            items = [C.c_void_p.from_address(a + 8).value for a, _ in outer]
            assert items[0] == head
            assert _chain(items[0]) == ids  # the original list, untouched
            for it in items[1:]:
                cp = _chain(it)
                assert [i for _, i in cp] == [i for _, i in ids]
                for a, _ in cp:
                    assert a not in seen
                    seen.add(a)
            for a, _ in outer:
                assert a not in seen
                seen.add(a)
            n_after += 1
    assert n_after == len(before)
    for _, ids in before.values():
        assert not any(a in seen for a, _ in ids)
    del keep, layout


@pytest.mark.parametrize("threads", ["1", "8"])
def test_node_arena(tmp_path, threads):
    """The drop-in's list-node arena (binning_gpu.c node_new): a program
    linked like the drop-in (its free() is the library's) gets arena nodes,
    KBH_NODE_ARENA=0 malloc'd ones; the expanded lists are identical and
    every node can be freed one by one as free_llist does (llist.c:101-108).
    Loaded through ctypes (this process) the arena stays off."""
    import subprocess
    repo = pathlib.Path(__file__).resolve().parents[1]
    lib = repo / "genome-assembly_amd" / "lib"
    exe = tmp_path / "node_arena_check"
    subprocess.run(["gcc", "-O2", "-pthread", str(repo / "tests" / "helpers" / "node_arena_check.c"),
                    f"-L{lib}", "-lkbin_host", "-lkbin", f"-Wl,-rpath,{lib}", "-o", str(exe)], check=True)
    out = {}
    for arena in ("1", "0"):
        env = dict(os.environ, KBH_NODE_ARENA=arena, KBH_THREADS=threads)
        r = subprocess.run([str(exe), "30000"], env=env, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        f = r.stdout.split()
        out[arena] = (f[1], f[3], f[5], f[7])
    assert out["1"][:3] == out["0"][:3]
    assert int(out["1"][1]) > 0 and int(out["1"][2]) > 0
    assert out["1"][3] == "1" and out["0"][3] == "0"
    assert host_lib().kbh_node_arena_active() == 0
