#!/usr/bin/env python3
"""Adds whole-program goldens of the reference AS SHIPPED (its main: bin,
prune, expand, unitig extension, print_kmers) on the C2 generator's first n
reads (bench.py C2: seed 2, generator stream gen_seed(2) = 2000006), one
150-bp read per line, READ_LENGTH 152, at the reference's own MMER_SIZE 4
(binning.c:10) -- where its unitig extension is live and
quadratic (20 000 reads: ~13 min on one core here).  Runs only where
/root/reference is (oracle/build_ref.sh full); writes tests/golden/unitigs.json
entries {"input": "c2:<n>", "read_length": 152, ...}.

    python tools/unitig_golden.py 20000
"""
import hashlib
import json
import os
import pathlib
import subprocess
import sys
import tempfile
import time

REPO = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "oracle"))
import oracle  # noqa: E402

GOLDEN = REPO / "tests" / "golden" / "unitigs.json"


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    K, M = 31, 4
    env = dict(os.environ, KB_REF_READ_LENGTH="152")
    subprocess.run(["bash", str(REPO / "oracle" / "build_ref.sh"), "full", str(K), str(M), "1"], env=env,
                   check=True, capture_output=True)
    exe = REPO / "oracle" / "_ref" / f"full_k{K}_m{M}_c1_rl152"
    raw = oracle.gen_reads(n, 150, 5_000_000, 1000, 2 * 1000003)
    with tempfile.TemporaryDirectory() as d:
        p = pathlib.Path(d) / "reads.txt"
        with open(p, "wb") as f:
            for i in range(n):
                f.write(raw[i * 150:(i + 1) * 150] + b"\n")
        t0 = time.time()
        out = subprocess.run([str(exe), str(p)], check=True, capture_output=True).stdout
        wall = time.time() - t0
    row = {"input": f"c2:{n}", "K": K, "M": M, "cutoff": 1, "read_length": 152, "lines": out.count(b"\n"),
           "sha256": hashlib.sha256(out).hexdigest(), "reference_wall_s": round(wall, 1)}
    print(row)
    rows = [r for r in json.loads(GOLDEN.read_text()) if r["input"] != row["input"]]
    rows.append(row)
    GOLDEN.write_text(json.dumps(rows, indent=1) + "\n")


if __name__ == "__main__":
    main()
