"""The invariant behind the binned engine's offset partitions (bin_body in
csrc/kbin_bins.hip): for every k-mer occurrence, the offset of
its signature inside the k-mer equals the FIRST occurrence of the key's mmer
string in the key's k-mer (both complemented together, binning.c:1029-1040).
So the offset is a function of the key, and partitioning a bin by offset
ranges puts every key in exactly one partition.

Pure Python over the closed form of SURVEY.md §8(a) (sticky leftmost strict
argmax, binning.c:922-989); no GPU.  Small inputs: the bundled reads and
seeded random reads with errors."""
import pathlib
import random

import pytest

GOLD = pathlib.Path(__file__).parent / "golden"
VAL = {"T": 0, "G": 1, "C": 2, "A": 3}
COMP = {"A": "T", "T": "A", "C": "G", "G": "C"}


def occurrences(read, K, M):
    """(mmer key, kmer key, signature offset) per k-mer, binning.c:918-1040"""
    full = 4 ** M - 1
    L = len(read)
    sc = []
    for p in range(L - M + 1):
        s = 0
        for c in read[p:p + M]:
            s = s * 4 + VAL[c]
        sc.append(s)
    sig = -1
    for i in range(L - K + 1):
        if i > sig:
            best = -1
            for p in range(i, i + K - M + 1):
                c = max(sc[p], full - sc[p])
                if c > best:
                    best, sig = c, p
        mm, km = read[sig:sig + M], read[i:i + K]
        if sc[sig] < full - sc[sig]:
            mm = "".join(COMP[c] for c in mm)
            km = "".join(COMP[c] for c in km)
        yield mm, km, sig - i


def random_reads(n, L, glen, err, seed):
    rng = random.Random(seed)
    g = "".join(rng.choice("ACGT") for _ in range(glen))
    out = []
    for _ in range(n):
        s = rng.randrange(glen - L)
        r = list(g[s:s + L])
        for j in range(L):
            if rng.random() < err:
                r[j] = rng.choice([c for c in "ACGT" if c != r[j]])
        out.append("".join(r))
    return out


@pytest.mark.parametrize("K,M", [(31, 7), (21, 5), (6, 3), (63, 7), (31, 8)])
def test_signature_offset_is_first_occurrence(K, M):
    reads = [ln.strip() for ln in open(GOLD / "reads.txt")][:150]
    reads = [r for r in reads if len(r) >= K] + random_reads(150, max(150, K + 40), 20000, 0.01, K * 100 + M)
    seen = {}
    n = 0
    for r in reads:
        for mm, km, o in occurrences(r, K, M):
            assert km.find(mm) == o, (r, mm, km, o)
            assert seen.setdefault((mm, km), o) == o  # one offset per key
            n += 1
    assert n > 10000
