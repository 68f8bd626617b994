"""CPU tests of the parity oracle (oracle/): pinned to the reference's known
answers (tests/golden/digests.json, produced by the compiled reference) and,
where the reference is buildable (this container), to the reference binary on
fresh seeded inputs -- including K < 2M, where the reference's incremental
branch (binning.c:992-1021) is live."""
import hashlib
import pathlib
import subprocess

import numpy as np
import pytest

import oracle


def dump_bytes(res, K, M) -> bytes:
    bp = b"TGCA"

    def s(hi, lo, n):
        v = (int(hi) << 64) | int(lo)
        out = bytearray(n)
        for j in range(n - 1, -1, -1):
            out[j] = bp[v & 3]
            v >>= 2
        return bytes(out)

    lines = []
    for e in range(res.n_entries):
        ids = res.ids[int(res.offset[e]):int(res.offset[e + 1])]
        lines.append(b"%s\t%s\t%d\t%s\n" % (s(0, res.mmer[e], M), s(res.kmer_hi[e], res.kmer_lo[e], K),
                                             int(res.count[e]), b",".join(b"%d" % x for x in ids)))
    return b"".join(lines)


def test_known_answer_digests(digests, golden_dir):
    for row in digests:
        bases, lens = oracle.read_fgets(golden_dir / row["input"], row["read_length"])
        res = oracle.bin_reads(bases, lens, row["K"], row["M"], row["cutoff"], row["prune"])
        d = dump_bytes(res, row["K"], row["M"])
        assert res.n_entries == row["entries"], row
        assert hashlib.sha256(d).hexdigest() == row["sha256"], row


def test_full_dump_line_level(golden_dir):
    bases, lens = oracle.read_fgets(golden_dir / "input.txt", 101)
    res = oracle.bin_reads(bases, lens, 6, 3, 1, True)
    assert dump_bytes(res, 6, 3) == (golden_dir / "input_k6m3_prune.tsv").read_bytes()
    # first sorted lines
    assert dump_bytes(res, 6, 3).startswith(b"ACC\tACCACG\t2\t15,8\nACC\tACCCAG\t2\t7,0\n")


def test_fgets_chunking(tmp_path):
    """binning.c:1158-1166: 100-bp lines with READ_LENGTH 101 split into a
    99-bp read + an empty read; a last line without newline loses a base."""
    p = tmp_path / "r.txt"
    p.write_bytes(b"A" * 100 + b"\n" + b"C" * 10 + b"\n" + b"G" * 5)
    _, lens = oracle.read_fgets(p, 101)
    assert lens.tolist() == [99, 0, 10, 4]
    _, lens = oracle.read_fgets(p, 40)
    assert lens.tolist() == [38, 38, 22, 10, 4]


def test_hand_trace_read0():
    """SURVEY §8(c) hand trace of input.txt read 0 at k=6 m=3."""
    r = b"CAGCCGCTGGGTCCG"
    res = oracle.bin_reads(r, [len(r)], 6, 3, 1, False)
    d = dump_bytes(res, 6, 3).decode().splitlines()
    keys = {tuple(x.split("\t")[:2]) for x in d}
    for mm, km in [("AGC", "CAGCCG"), ("AGC", "AGCCGC"), ("CCG", "GCCGCT"), ("CCG", "CCGCTG"),
                   ("ACC", "GCGACC"), ("ACC", "CGACCC"), ("ACC", "GACCCA"), ("ACC", "ACCCAG"),
                   ("AGG", "CCCAGG"), ("AGG", "CCAGGC")]:
        assert (mm, km) in keys


def _ref_or_skip(K, M, c=1):
    exe = oracle.ref_binary(K, M, c)
    if exe is None:
        pytest.skip("reference not buildable here (no /root/reference)")
    return exe


# (13, 7), (15, 8), (3, 2), (1, 1): K < 2M pairs whose incremental branch
# (binning.c:992-1021) overflows the reference's int differently
@pytest.mark.parametrize("K,M,rl", [(31, 7, 152), (6, 3, 101), (10, 6, 80), (5, 4, 60), (40, 8, 130),
                                    (63, 7, 260), (13, 7, 90), (15, 8, 100), (3, 2, 50), (1, 1, 30)])
def test_oracle_vs_reference_binary(tmp_path, K, M, rl):
    exe = _ref_or_skip(K, M)
    rng = np.random.default_rng(K * 31 + M)
    g = rng.choice(np.frombuffer(b"ACGT", np.uint8), 2500)
    lines = []
    for _ in range(300):
        L = int(rng.integers(0, rl + 30))
        s = int(rng.integers(0, 2500 - L))
        r = g[s:s + L].copy()
        m = rng.random(L) < 0.02
        r[m] = rng.choice(np.frombuffer(b"ACGT", np.uint8), int(m.sum()))
        lines.append(r.tobytes())
    p = tmp_path / "reads.txt"
    p.write_bytes(b"\n".join(lines) + b"\n")
    for prune in (0, 1):
        out = subprocess.run([str(exe), str(p), str(rl), str(prune)], check=True,
                             capture_output=True).stdout
        ref = b"".join(sorted(out.splitlines(keepends=True)))
        bases, lens = oracle.read_fgets(p, rl)
        res = oracle.bin_reads(bases, lens, K, M, 1, bool(prune))
        assert dump_bytes(res, K, M) == ref


@pytest.mark.parametrize("K,M,prune", [(31, 7, True), (63, 7, False), (21, 5, True)])
def test_masked_oracle_is_a_partition(K, M, prune):
    """kbo_bin_masked (the capacity tests' partition filter) returns exactly
    the full result's entries whose mmer is in the mask, lists included, and
    still counts every k-mer"""
    rng = np.random.default_rng(K)
    n, L = 3000, 150
    genome = rng.integers(0, 4, 20000)
    st = rng.integers(0, len(genome) - L, n)
    raw = np.frombuffer(b"TGCA", dtype=np.uint8)[genome[st[:, None] + np.arange(L)]].reshape(-1)
    lens = np.full(n, L, np.uint32)
    full = oracle.bin_reads(raw.tobytes(), lens, K, M, 1, prune)
    mask = (rng.random(1 << (2 * M)) < 0.3).astype(np.uint8)
    part = oracle.bin_reads(raw.tobytes(), lens, K, M, 1, prune, mmer_mask=mask)
    keep = mask[full.mmer].astype(bool)
    assert part.n_kmers == full.n_kmers and 0 < part.n_entries == int(keep.sum()) < full.n_entries
    for f in ("mmer", "kmer_hi", "kmer_lo", "count"):
        np.testing.assert_array_equal(getattr(part, f), getattr(full, f)[keep])
    lists = [full.ids[full.offset[e]:full.offset[e + 1]] for e in np.flatnonzero(keep)]
    np.testing.assert_array_equal(part.ids, np.concatenate(lists))


@pytest.mark.parametrize("K,M,err", [(31, 7, 1000), (63, 7, 10000), (21, 5, 0), (6, 3, 2000)])
def test_stream_digest_matches_result(K, M, err):
    """oracle.stream_digest (the full-size digests' path, kb_oracle.c
    kbo_stream_digest: scan_read into per-worker count tables, then the list
    positions counted down in a second scan) equals kbin.result_digest of the
    oracle's own result, pruned and not, over several workers"""
    import kbin
    n, L = 2500, 150
    bases = oracle.gen_reads(n, L, 30000, err, 4242)
    lens = np.full(n, L, np.uint32)
    for prune in (True, False):
        ora = oracle.bin_reads(bases, lens, K, M, 1, prune)
        want = tuple(int(x) for x in kbin.result_digest(ora))
        got, nk = oracle.stream_digest(bases, n, L, K, M, 1, prune, workers=3, cap_log2=19)
        assert got == want and nk == ora.n_kmers


def test_gen_reads_stream():
    """kbo_gen_reads: reads read_base .. of one stream (any slice of it agrees
    with the whole), ACGT only, substitutions at the asked rate"""
    a = oracle.gen_reads(400, 150, 100000, 10000, 77)
    b = oracle.gen_reads(100, 150, 100000, 10000, 77, read_base=250)
    assert a[250 * 150:350 * 150] == b
    assert set(a) <= set(b"ACGT")
    clean = oracle.gen_reads(400, 150, 100000, 0, 77)
    diff = sum(x != y for x, y in zip(a, clean)) / len(a)
    assert 0.006 < diff < 0.014  # 1 % substitutions


def test_full_size_digest_fixtures():
    """tests/golden/oracle_digests.json (tools/oracle_digest.py) holds the
    bench workloads' own parameters; its C2 entry recomputes in seconds"""
    import json
    import bench
    fx = json.loads((pathlib.Path(__file__).parent / "golden" / "oracle_digests.json").read_text())
    for name in ("c2", "c3"):
        wl, f = bench.WORKLOADS[name], fx[name]
        assert (f["reads"], f["read_len"], f["genome"], f["err_ppm"], f["K"], f["M"]) == \
            (wl["reads"], wl["read_len"], wl["genome"], wl["err_ppm"], wl["K"], wl["M"])
        assert f["seed"] == bench.gen_seed(wl["seed"]) and f["kmers"] == wl["reads"] * (wl["read_len"] - wl["K"] + 1)
    assert tuple(fx["c3"]["digest"]) == bench.C3_DIGEST
    f = fx["c2"]
    dig, nk = oracle.gen_stream_digest(f["reads"], f["read_len"], f["genome"], f["err_ppm"], f["seed"], f["K"], f["M"],
                                       workers=8, cap_log2=23)
    assert [hex(x) for x in dig] == f["digest"] and nk == f["kmers"]
