"""Probe: an in-place RCCL all-gather (the data-parallel exchange, rae/dist.py) captured into a
HIP graph and replayed, on a 1-rank "nccl" process group -- the only RCCL communicator a
one-GPU box can form.  Checks the capture path bench.py uses at N>1 before the driver's
multi-GPU run.   usage: python tools/rccl_graph_probe.py"""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "relation-autoencoder_amd"))


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    n = 1288 * 100
    buf = torch.arange(n, dtype=torch.float32, device=dev)

    def exchange(b):
        dist.all_gather_into_tensor(b, b[:n], group=None)

    exchange(buf)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.graph(g, stream=s):
        for _ in range(64):
            buf.mul_(1.0)
            exchange(buf)
    torch.cuda.current_stream(dev).wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(buf, torch.arange(n, dtype=torch.float32, device=dev))
    t0 = time.perf_counter()
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / 640 * 1e6
    print(f"captured in-place all_gather_into_tensor (1 rank) replayed: {us:.2f} us per "
          f"exchange+mul step, rccl {torch.cuda.nccl.version()}")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
