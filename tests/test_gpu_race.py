"""Barrier-ordering stress of the bin kernel.

Round 4's r4f6 SQ pass returned KB_EDEVICE (5 650 k-mers uncounted, +10 030
distinct keys) on C2.  Cause (kbin_bins.hip, bin_body's partition loop): a
partition's loop left on an empty stack read from LDS without a barrier after
the last one, and the next partition's start (tid 0, no barrier before it)
rewrote that same word to 1.  A wave released late from the barrier could read
the new partition's 1, run one more loop body of the old partition and stay a
barrier out of step with the rest of the block: table zeroing under live
counts, keys claimed twice.  The fix keeps the stack depth in one word per
partition parity.

The diagnostic build (lib/abl, KB_BIN_ABL) lets one wave arrive ~60 K cycles
late at every partition-loop top (KB_DIAG_SKEW = wave + 1): with the old
single word that wave reads the next partition's depth every time a bin has a
second partition.  Evidence (gpurun_out/r5g3, profiles/r05/race/): round 4's
single word (tools/race_ab.sh) under this stress ended its first finalize in
an illegal memory access -- the out-of-step wave runs on stale cursors -- so
that mutation check is NOT part of the suite (a faulting kernel risks the
box); the fixed build stays bit-exact under it in every case below.  Inputs use 1024-slot tables (KB_BIN_TS_LOG2=10) so
that most bins take several offset / hash partitions and overflow redos.
"""
import json
import os
import pathlib
import subprocess
import sys

import pytest

REPO = pathlib.Path(__file__).resolve().parent.parent
ABL = REPO / "genome-assembly_amd" / "lib" / "abl" / "libkbin.so"

pytestmark = pytest.mark.gpu


def run_worker(lib: pathlib.Path, skew: int, n_reads=60000, glen=2_000_000, seed=7, err=0.0, extra=None):
    env = dict(os.environ, KB_LIB_PATH=str(lib), KB_DIAG_SKEW=str(skew), KB_BIN_TS_LOG2="10", KB_ENGINE="binned")
    env.update(extra or {})
    p = subprocess.run([sys.executable, str(REPO / "tests" / "race_worker.py"), str(n_reads), str(glen), str(seed),
                        str(err)],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.mark.skipif(not ABL.exists(), reason="diagnostic build lib/abl not built (make -C genome-assembly_amd/csrc abl)")
@pytest.mark.parametrize("skew", [0, 6, 16])
def test_partition_loop_skew(skew):
    """a late wave at every partition-loop top changes nothing: bit-exact on
    every finalize (cold, learned, KB_TIMING_KERNEL)"""
    out = run_worker(ABL, skew)
    assert out["ok"], out
    paths = out["paths"]
    # the input really takes the multi-partition paths the race needs
    assert paths.get("offset_partitions", 0) > 0 or paths.get("partitions", 0) > paths.get("n_bins", 0), paths


@pytest.mark.skipif(not ABL.exists(), reason="diagnostic build lib/abl not built")
def test_partition_loop_skew_ranked():
    """the same late wave in the ranked kernel (long lists: bitmaps, ranks)"""
    out = run_worker(ABL, 6, n_reads=40000, glen=3000, seed=9, err=0.005,
                     extra={"KB_BIN_RANK": "2", "KB_BIN_TS_LOG2": "13"})
    assert out["ok"], out
    assert out["paths"].get("ranked_bins", 0) > 0, out["paths"]

