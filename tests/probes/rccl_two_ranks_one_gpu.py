"""Probe: can two RCCL ranks share one GPU (the one-GPU box)?  If RCCL accepts it, the product
UlyssesGroup runs at world size 2 over real RCCL collectives; prints the outcome either way."""
import os
import sys
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker(rank, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=2, device_id=torch.device("cuda:0"))
    x = torch.full((4,), float(rank), device="cuda")
    y = torch.empty_like(x)
    dist.all_to_all_single(y, x)
    torch.cuda.synchronize()
    print(f"rank {rank}: all_to_all {y.tolist()}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    import socket
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    mp.start_processes(worker, args=(port,), nprocs=2, start_method="spawn")
