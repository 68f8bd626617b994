"""GPU probe: which engine paths (kb_timing path counters) a workload takes
at default knobs -- used to size the capacity-regime parity tests."""
import json
import sys

import torch

sys.path.insert(0, "genome-assembly_amd")
import kbin  # noqa: E402

KEYS = ("n_bins", "split_mmers", "heavy_bins", "partitions", "offset_partitions", "flat_partitions",
        "overflow_redos", "prefiltered", "long_lists", "clustered_lists", "max_depth")


def probe(n, L, K, M, genome, err, seed, P):
    wpr = (L + 31) // 32
    words = torch.empty(n * wpr, dtype=torch.int64, device="cuda")
    lens = torch.empty(n, dtype=torch.int32, device="cuda")
    kbin.generate_reads_device(words.data_ptr(), lens.data_ptr(), n, L, genome, err, seed)
    torch.cuda.synchronize()
    out = []
    with kbin.Engine(K, M, cutoff=1, max_read_len=L) as eng:
        eng.submit_packed_device(words.data_ptr(), lens.data_ptr(), n, wpr, 0)
        for p in range(P):
            if P > 1:
                eng.set_partition(p, P)
            eng.finalize(True)
            t = eng.timing()
            out.append({k: t[k] for k in KEYS})
    return out


for spec in sys.argv[1:]:
    n, L, K, M, genome, err, seed, P = (int(x) for x in spec.split(","))
    r = probe(n, L, K, M, genome, err, seed, P)
    print(json.dumps({"spec": spec, "passes": r}), flush=True)
