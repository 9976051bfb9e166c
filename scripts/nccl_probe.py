"""Can the RCCL ("nccl") backend run here?  Two ranks, launched by
torch.distributed.run, all-gather a tensor and all-reduce the EI shard result the
way ShardedScorer / bench --gpus N do.  With one GPU visible both ranks share
cuda:0; RCCL may refuse two ranks on one device, which is reported, not hidden.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port 29641 scripts/nccl_probe.py
"""
import os
import time

import torch
import torch.distributed as dist


def main():
    rank, ws = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", rank % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    x = torch.full((4,), float(rank), dtype=torch.float64, device=dev)
    g = torch.empty(ws * 4, dtype=torch.float64, device=dev)
    dist.all_gather_into_tensor(g, x)
    t = torch.tensor([rank + 1.0], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(20):
        dist.all_gather_into_tensor(g, x)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / 20
    ok = g.view(ws, 4)[:, 0].tolist() == [float(r) for r in range(ws)] and float(t.item()) == float(ws)
    if rank == 0:
        print(f"nccl backend: {ws} ranks on {torch.cuda.device_count()} visible GPU(s), all_gather / all_reduce "
              f"{'correct' if ok else 'WRONG'}, {dt * 1e6:.1f} us per 32-byte all_gather", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
