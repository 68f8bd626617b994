"""The unitig extension, find_kmer_extensions (binning.c:659-783), replayed
exactly by genome-assembly_amd/host/unitig.c.

CPU tests, three ways of pinning it:
  * test_unitig_goldens_via_oracle -- no reference and no GPU needed: the
    oracle's unpruned CSR (with first-occurrence stamps) is materialised into
    the reference's exact zhash layout (kbh_materialise_csr, the drop-in's
    prune_data path), expanded, extended forward and backward, and printed
    (kbh_print_kmers = print_kmers, binning.c:827-843); the stdout's sha256
    equals the reference program's own on every tests/golden/unitigs.json
    configuration, including the C2 generator's first 20 000 reads at the
    reference's shipped M = 4 (the reference took 13 min on them);
  * test_unitig_vs_reference_random -- the compiled reference (this container
    only): random inputs at small K and M (many candidates, multiple-candidate
    breaks, resumed static cursors), the reference program as shipped against
    the same program with only find_kmer_extensions replaced
    (oracle/build_ref.sh unitig): stdout byte-identical whenever the
    reference exits 0; where it crashes (SIGSEGV: the use-after-free of
    binning.c:721-731) the replay reports the event (u1_events);
  * the GPU suite runs kbin_main --unitigs (GPU binning + this replay) on the
    same goldens (tests/test_gpu_parity.py::test_kbin_main_unitigs).
"""
import ctypes as C
import hashlib
import json
import os
import pathlib
import random
import subprocess
import tempfile

import numpy as np
import pytest

import kbin
import oracle

REPO = pathlib.Path(__file__).resolve().parent.parent
GOLDEN = REPO / "tests" / "golden"


def _host():
    lib = C.CDLL(str(kbin.HOST_LIB_PATH))
    lib.zcreate_hash_table.restype = C.c_void_p
    lib.kbh_materialise_csr.argtypes = [C.c_void_p, C.POINTER(kbin.kb_csr), C.c_int, C.c_int]
    lib.expand_read_id_list.argtypes = [C.c_void_p]
    lib.find_kmer_extensions.argtypes = [C.c_void_p, C.c_bool]
    lib.kbh_print_kmers.argtypes = [C.c_void_p, C.c_void_p]
    return lib


class _Stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("calls", "queries", "unitigs", "merges", "multiple", "resumes",
                                          "candidates", "deleted", "inserted", "set_existing", "u1_events")] + \
               [("index_ms", C.c_double), ("walk_ms", C.c_double)]


def _libc():
    libc = C.CDLL(None)
    libc.fopen.restype = C.c_void_p
    libc.fopen.argtypes = [C.c_char_p, C.c_char_p]
    libc.fclose.argtypes = [C.c_void_p]
    return libc


def unitigs_via_oracle(bases: bytes, lens, K: int, M: int, cutoff: int = 1):
    """the reference's main after the read loop (binning.c:1169-1180) over the
    oracle's keys: prune_data's exact tables, expand, extend x2, print"""
    res = oracle.bin_reads(bases, lens, K, M, cutoff, prune=False)
    lib = _host()
    arrays = dict(mmer=res.mmer, kmer_hi=res.kmer_hi, kmer_lo=res.kmer_lo, count=res.count,
                  offset=res.offset, ids=res.ids, first=res.first)
    arrays = {k: np.ascontiguousarray(v) for k, v in arrays.items()}
    csr = kbin.kb_csr()
    csr.n_entries, csr.n_ids = res.n_entries, int(res.offset[-1]) if res.n_entries else 0
    for f, a in arrays.items():
        setattr(csr, f, a.ctypes.data_as(dict(kbin.kb_csr._fields_)[f]))
    assert lib.kbh_configure(K, M, cutoff, 0) == 0
    lib.kbh_unitig_reset()
    table = lib.zcreate_hash_table()
    assert lib.kbh_materialise_csr(table, C.byref(csr), 1, 0) == 0
    lib.expand_read_id_list(table)
    lib.find_kmer_extensions(table, True)
    lib.find_kmer_extensions(table, False)
    st = _Stats()
    lib.kbh_unitig_stats_get(C.byref(st))
    libc = _libc()
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "out.txt")
        f = libc.fopen(path.encode(), b"w")
        assert f
        assert lib.kbh_print_kmers(table, f) == 0
        libc.fclose(f)
        out = pathlib.Path(path).read_bytes()
    del arrays
    return out, st


def golden_input(case):
    """(bases, lens) as the reference's read loop chunks the input"""
    src = case["input"]
    rl = case.get("read_length", 101)
    if src.startswith("c2:"):  # the C2 generator's first n reads, one per line (tools/unitig_golden.py)
        n = int(src.split(":")[1])
        raw = oracle.gen_reads(n, 150, 5_000_000, 1000, 2 * 1000003)
        d = tempfile.mkdtemp()
        p = os.path.join(d, "reads.txt")
        with open(p, "wb") as f:
            for i in range(n):
                f.write(raw[i * 150:(i + 1) * 150] + b"\n")
        bases, lens = oracle.read_fgets(p, rl)
        os.unlink(p)
        os.rmdir(d)
        return bases, lens
    return oracle.read_fgets(str(GOLDEN / src), rl)


CASES = json.loads((GOLDEN / "unitigs.json").read_text())


@pytest.mark.parametrize("case", CASES, ids=[f"{c['input']}-k{c['K']}m{c['M']}" for c in CASES])
def test_unitig_goldens_via_oracle(case):
    bases, lens = golden_input(case)
    out, st = unitigs_via_oracle(bases, lens, case["K"], case["M"], case["cutoff"])
    assert out.count(b"\n") == case["lines"]
    assert hashlib.sha256(out).hexdigest() == case["sha256"]
    assert st.u1_events == 0
    if case["M"] <= 4:  # (the extension is live: score_limit 65 M >= 2 * 4^(M-1), binning.c:672)
        assert st.merges > 0


def test_unitig_paths_exercised():
    """reads.txt at K6 M3: multiple-candidate breaks and resumed cursors"""
    bases, lens = oracle.read_fgets(str(GOLDEN / "reads.txt"), 101)
    _, st = unitigs_via_oracle(bases, lens, 6, 3)
    assert st.multiple > 1000 and st.resumes > 50 and st.merges > 500


def test_unitig_noop_at_m5():
    """M >= 5: the reference's loop never runs (binning.c:672-678); the tables
    are left untouched and print as the dump's keys"""
    bases, lens = oracle.read_fgets(str(GOLDEN / "synth_a.txt"), 101)
    out, st = unitigs_via_oracle(bases, lens, 21, 5)
    assert st.merges == 0 and st.queries == 0
    res = oracle.bin_reads(bases, lens, 21, 5, 1, prune=True)
    assert out.count(b"\n") == res.n_entries


# ---- against the compiled reference (this container only) ----

def _ref_bin(mode, K, M):
    p = REPO / "oracle" / "_ref" / f"{mode}_k{K}_m{M}_c1"
    r = subprocess.run(["bash", str(REPO / "oracle" / "build_ref.sh"), mode, str(K), str(M)],
                       capture_output=True, text=True)
    if r.returncode or not p.exists():
        pytest.skip(f"reference not buildable here: {r.stderr[-200:]}")
    return p


RANDOM_CFGS = [(5, 1), (5, 2), (6, 2), (7, 3), (8, 3), (9, 4), (12, 4), (4, 4), (3, 2), (10, 3), (15, 4),
               (6, 3), (21, 4), (31, 4), (31, 3), (2, 1), (4, 2)]


@pytest.mark.skipif(not (pathlib.Path("/root/reference") / "binning.c").exists(), reason="no reference here")
@pytest.mark.parametrize("seed", range(4))
def test_unitig_vs_reference_random(seed, tmp_path):
    rng = random.Random(1000 + seed)
    for it in range(12):
        K, M = rng.choice(RANDOM_CFGS)
        full, ours = _ref_bin("full", K, M), _ref_bin("unitig", K, M)
        glen = rng.choice([20, 50, 200, 1000, 5000])
        g = "".join(rng.choice("ACGT") for _ in range(glen))
        lines = []
        for _ in range(rng.choice([10, 50, 200, 1000])):
            L = rng.randint(1, 99)
            if L >= glen:
                s = list(g)
            else:
                st = rng.randint(0, glen - L)
                s = list(g[st:st + L])
            for j in range(len(s)):
                if rng.random() < 0.01:
                    s[j] = rng.choice("ACGT")
            lines.append("".join(s))
        p = tmp_path / f"in_{it}.txt"
        p.write_text("\n".join(lines) + "\n")
        a = subprocess.run([str(full), str(p)], capture_output=True, timeout=600)
        b = subprocess.run([str(ours), str(p)], capture_output=True, timeout=600, env=dict(os.environ, KBH_TRACE="1"))
        assert b.returncode == 0, b.stderr[-500:]
        u1 = sum(json.loads(ln)["u1_events"] for ln in b.stderr.decode().splitlines()
                 if ln.startswith('{"find_kmer_extensions_ms"') and json.loads(ln)["forward"] == 0)
        if a.returncode == 0:
            assert a.stdout == b.stdout, (seed, it, K, M)
            assert u1 == 0
        else:  # the reference's use-after-free (binning.c:721-731) -- and only that
            assert a.returncode == -11 and u1 > 0, (seed, it, K, M, a.returncode)
