"""debug: K < 2M through a 4-rank virtual group -- which keys land twice"""
import sys, pathlib
REPO = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO / "tests"), str(REPO / "genome-assembly_amd"), str(REPO / "oracle")]
import numpy as np
import kbin, oracle, skmer_ref
from test_gpu_dist import _k_below_2m_reads, _result_dict
for K, M, G in [(15, 8, 4), (13, 7, 4), (15, 8, 2), (15, 8, 3)]:
    reads = _k_below_2m_reads(K, M)
    bases, lens = kbin.pack_reads(reads)
    ids = np.arange(len(reads), dtype=np.int32)
    ora = skmer_ref.oracle_dict(oracle.bin_reads(bases, lens, K, M, 1, True, ids=ids))
    off = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
    cuts = np.linspace(0, len(reads), G + 1).astype(int)
    try:
        with kbin.Group(K, M, cutoff=1, max_read_len=300, devices=[0] * G) as grp:
            for g in range(G):
                a, b = cuts[g], cuts[g + 1]
                grp.submit(g, bases=bases[off[a]:off[b]], lens=lens[a:b], ids=ids[a:b])
            grp.finalize(True)
            print(K, M, G, "counts", grp.unit_counts().tolist(), flush=True)
            parts = [_result_dict(grp.ctx(g).export()) for g in range(G)]
    except Exception as e:
        print(K, M, G, "ERR", e, flush=True)
        continue
    seen = {}
    for g, p in enumerate(parts):
        for k in p:
            seen.setdefault(k, []).append(g)
    dup = {k: v for k, v in seen.items() if len(v) > 1}
    print(K, M, G, "keys", len(seen), "oracle", len(ora), "dup", len(dup), flush=True)
    for k, v in list(dup.items())[:5]:
        print("  key", k, "ranks", v, "owner", kbin.dist.owner_of(k[0], G, K, M), [parts[g][k] for g in v], "ora", ora.get(k))
    wrong = sum(1 for g, p in enumerate(parts) for k in p if kbin.dist.owner_of(k[0], G, K, M) != g)
    print("  keys at a non-owner rank:", wrong)
