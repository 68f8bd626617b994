#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ (run in the build container,
where /root/reference exists; the GPU box only reads the committed outputs).

Fixtures = data, never reference source:
  input.txt, reads.txt   the reference's own bundled inputs (copied verbatim)
  synth_*.txt            seeded random read files written by this script
  digests.json           for each case: entries, sum of counts, distinct mmers
                         and the sha256 of the canonical dump,
                         produced by the COMPILED REFERENCE (oracle/_ref, built
                         by oracle/build_ref.sh from /root/reference sources)
  input_k6m3_prune.tsv   one full canonical dump, for line-level diffs
"""
import hashlib
import json
import pathlib
import subprocess
import sys

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO / "oracle"))
import oracle  # noqa: E402


def ref_dump(path, K, M, rl, prune, cutoff=1) -> bytes:
    exe = oracle.ref_binary(K, M, cutoff)
    if exe is None:
        raise SystemExit("reference not buildable here (needs /root/reference)")
    out = subprocess.run([str(exe), str(path), str(rl), "1" if prune else "0"],
                         check=True, capture_output=True).stdout
    lines = out.splitlines(keepends=True)
    lines.sort()  # bytewise == LC_ALL=C sort
    return b"".join(lines)


def summarize(dump: bytes) -> dict:
    lines = dump.splitlines()
    mmers = {ln.split(b"\t", 1)[0] for ln in lines}
    return {"entries": len(lines), "sum_count": sum(int(ln.split(b"\t")[2]) for ln in lines),
            "mmers": len(mmers), "sha256": hashlib.sha256(dump).hexdigest()}


def synth(name, n, lo, hi, seed, genome=4000, err=0.01, homopolymer=False):
    """Seeded random reads: substrings of an iid genome (generate_reads.py:93-112
    concept), random lengths in [lo, hi], substitutions at rate err, plus edge
    cases (short reads, exactly-K reads, homopolymers, repeated k-mers)."""
    rng = np.random.default_rng(seed)
    g = rng.choice(list(b"ACGT"), size=genome).astype(np.uint8)
    lines = []
    for _ in range(n):
        L = int(rng.integers(lo, hi + 1))
        s = int(rng.integers(0, genome - L))
        r = g[s:s + L].copy()
        flips = rng.random(L) < err
        r[flips] = rng.choice(list(b"ACGT"), size=int(flips.sum()))
        lines.append(bytes(r))
    if homopolymer:
        lines += [b"A" * hi, b"T" * hi, b"C" * hi, b"G" * hi, b"ACGT" * (hi // 4),
                  b"AC" * (hi // 2), b"", b"A", (b"ACGTTGCA" * hi)[:hi]]
    p = HERE / f"{name}.txt"
    p.write_bytes(b"\n".join(lines) + b"\n")
    return p


CASES = [
    # (file, K, M, READ_LENGTH, prune) -- the SURVEY §8(c) known-answer table
    ("input.txt", 6, 3, 101, False),
    ("input.txt", 6, 3, 101, True),
    ("reads.txt", 6, 3, 101, False),
    ("reads.txt", 6, 3, 101, True),
    ("reads.txt", 31, 4, 101, True),
    ("reads.txt", 31, 7, 101, True),
    ("reads.txt", 31, 7, 102, True),
    ("reads.txt", 63, 7, 101, True),
]


def main():
    synth("synth_a", 400, 20, 150, seed=11, homopolymer=True)
    synth("synth_b", 300, 60, 250, seed=12, genome=2000, err=0.02, homopolymer=True)
    synth("synth_c", 200, 8, 40, seed=13, genome=300, err=0.0, homopolymer=True)
    cases = list(CASES) + [
        ("synth_a.txt", 31, 7, 152, True), ("synth_a.txt", 21, 5, 152, False),
        ("synth_a.txt", 16, 8, 152, True), ("synth_a.txt", 32, 8, 152, True),
        ("synth_b.txt", 63, 7, 252, True), ("synth_b.txt", 40, 6, 252, True),
        ("synth_b.txt", 33, 1, 252, False), ("synth_b.txt", 31, 7, 101, True),
        ("synth_c.txt", 6, 3, 42, False), ("synth_c.txt", 9, 4, 42, True),
        ("synth_c.txt", 2, 1, 42, False),
    ]
    out = []
    for f, K, M, rl, prune in cases:
        d = ref_dump(HERE / f, K, M, rl, prune)
        row = {"input": f, "K": K, "M": M, "read_length": rl, "cutoff": 1, "prune": prune}
        row.update(summarize(d))
        out.append(row)
        print(row)
        if (f, K, M, rl, prune) == ("input.txt", 6, 3, 101, True):
            (HERE / "input_k6m3_prune.tsv").write_bytes(d)
    (HERE / "digests.json").write_text(json.dumps(out, indent=1) + "\n")

    # whole-program outputs of the reference as shipped (binning.c main: bin,
    # prune, expand, unitig extension, print_kmers; READ_LENGTH 101) -- the
    # drop-in test runs the same program with the GPU process_read/prune_data
    uni = []
    for f, K, M in [("reads.txt", 31, 4), ("input.txt", 6, 3), ("reads.txt", 6, 3),
                    ("reads.txt", 31, 7), ("synth_a.txt", 21, 5), ("reads.txt", 63, 7)]:
        subprocess.run(["bash", str(REPO / "oracle" / "build_ref.sh"), "full", str(K), str(M), "1"],
                       check=True, capture_output=True)
        exe = REPO / "oracle" / "_ref" / f"full_k{K}_m{M}_c1"
        outb = subprocess.run([str(exe), str(HERE / f)], check=True, capture_output=True).stdout
        row = {"input": f, "K": K, "M": M, "cutoff": 1, "lines": outb.count(b"\n"),
               "sha256": hashlib.sha256(outb).hexdigest()}
        print(row)
        uni.append(row)
    (HERE / "unitigs.json").write_text(json.dumps(uni, indent=1) + "\n")


if __name__ == "__main__":
    main()
