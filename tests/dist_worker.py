"""Rank body for tests/test_gpu_dist.py::test_ranks_rehearsal (launched by
torch.distributed.run).  Each rank generates its shard of synthetic reads on
the GPU, runs kbin.dist.ShardedBinner and saves the entries it owns."""
import os
import pathlib
import sys

REPO = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "genome-assembly_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import kbin  # noqa: E402
from kbin.dist import ShardedBinner  # noqa: E402


def main():
    out_dir = pathlib.Path(sys.argv[1])
    n, L, K, M = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    backend = os.environ.get("KB_DIST_BACKEND", "gloo")
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    dist.init_process_group(backend)
    wpr = (L + 31) // 32
    words = torch.empty(n * wpr, dtype=torch.int64, device="cuda")
    lens = torch.empty(n, dtype=torch.int32, device="cuda")
    # one genome, reads split by id range (C4's shape): rank r holds reads [r n, (r + 1) n)
    kbin.generate_reads_device(words.data_ptr(), lens.data_ptr(), n, L, 300000, 2000, 77,
                               device=dev, read_base=rank * n)
    torch.cuda.synchronize()
    # (KB_DIST_TRANSPORT=c under gloo: the C group -- its routing, counts and
    # offsets -- over host collectives; default: the torch exchange)
    sb = ShardedBinner(K, M, 1, L, device=dev, transport=os.environ.get("KB_DIST_TRANSPORT") or None)
    for _ in range(2):  # twice: buffers and contexts are reused across steps
        sb.step(words, lens, n, wpr, first_id=rank * n)
    r = sb.engine.export()
    np.savez(out_dir / f"rank{rank}.npz", mmer=r.mmer, hi=r.kmer_hi, lo=r.kmer_lo, count=r.count,
             offset=r.offset, ids=r.ids, sent=np.array(sb.last_counts[0]),
             recv=np.array(sb.last_counts[1]))
    # the pipelined path (send / receive, the next unit's exchange in flight
    # while a unit is binned): three units, and a last prefetch nobody receives
    unit = sb.send(words, lens, n, wpr, first_id=rank * n)
    for _ in range(3):
        nxt = sb.send(words, lens, n, wpr, first_id=rank * n)
        sb.receive(unit)
        unit = nxt
    sb.discard(unit)
    r = sb.engine.export()
    np.savez(out_dir / f"rank{rank}_pipe.npz", mmer=r.mmer, hi=r.kmer_hi, lo=r.kmer_lo, count=r.count,
             offset=r.offset, ids=r.ids)
    # also the rank's raw reads, for the single-GPU reference run
    np.save(out_dir / f"words{rank}.npy", words.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
