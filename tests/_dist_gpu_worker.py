"""Worker of tests/test_gpu_distributed.py (launched by torch.distributed.run, one process per rank, all on
cuda:0, gloo collectives): every rank holds a contiguous shard of a seeded corpus in a ShardedIndexCorpus,
answers the same query batch (progressive search: local scan + exact re-rank, records all-gather, R-way
hq_progressive_final merge; and the brute-force / frame modes), and rank 0 writes the results next to the
unsharded IndexCorpus's for the test to compare."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hilbert-quantization_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main(out_path):
    from hq_mi355x.core.search_engine import IndexCorpus
    from hq_mi355x.distributed import ShardedIndexCorpus, shard_range
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    comm = None
    if os.environ.get("HQ_DIST_RCCL"):
        # one GPU per rank, RCCL: the records all-gather through the C-ABI (hq_allgather_topk)
        from hq_mi355x.rccl import Communicator
        local = int(os.environ.get("LOCAL_RANK", rank))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        comm = Communicator.from_process_group()
    else:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo")
    rng = np.random.default_rng(123)
    N, L = 20_011, 64
    C = rng.standard_normal((N, L)).cumsum(1) * 0.1
    C[15_000:15_006] = C[17]          # duplicates in another shard: ties follow global ids
    C[40, :32] = 0.5                  # zero-variance level-0 segment
    Q = np.concatenate([C[[17, 40, 9_999, 20_010]], C[100:160] + rng.normal(0, 0.02, (60, L)),
                        rng.standard_normal((3, L))])
    a, b = shard_range(N, rank, world)
    sh = ShardedIndexCorpus(C[a:b], id_base=a, n_total=N, comm=comm)
    got = {}
    ids, ov, lv, cnt = sh.progressive(Q, 10, 0.1, 20)
    got["progressive"] = [x.cpu().numpy() for x in (ids, ov, lv, cnt)]
    # the sharded forms also return the per-query counts: (ids, overall, levels, count), (ids, scores, count)
    got["brute_force"] = [x.cpu().numpy() for x in sh.brute_force(Q, 10)[:3]]
    got["frame_search"] = [x.cpu().numpy() for x in sh.frame_search(Q, 10, 0.1)[:2]]
    if rank == 0:
        full = IndexCorpus(C)
        want = {"progressive": [x.cpu().numpy() for x in full.progressive(Q, 10, 0.1, 20)],
                "brute_force": [x.cpu().numpy() for x in full.brute_force(Q, 10)],
                "frame_search": [x.cpu().numpy() for x in full.frame_search(Q, 10, 0.1)]}
        res = {}
        for k in got:
            gi, wi = got[k][0], want[k][0]
            ok = [bool(np.array_equal(gi, wi))]
            valid = wi >= 0  # scores / records compared on the filled slots (padding conventions differ)
            for x, y in zip(got[k][1:3], want[k][1:3]):
                ok.append(bool(np.array_equal(x[valid], y[valid])))
            res[k] = ok
        np.savez(out_path, C=C, Q=Q, ids=got["progressive"][0], ov=got["progressive"][1],
                 cnt=got["progressive"][3])
        with open(out_path + ".json", "w") as f:
            json.dump({"world": world, "equal": res}, f)
    dist.barrier()
    if comm is not None:
        comm.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
