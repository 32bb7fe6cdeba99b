"""Probe (diagnostic): can an RCCL all-reduce (torch.distributed "nccl" = RCCL) be captured in a HIP graph
(world size 1 on the test box)?  Prints the replayed results."""
import os
import sys

import torch
import torch.distributed as dist


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    t = torch.ones(1 << 20, device="cuda")
    side = torch.cuda.Stream()
    # warm-up outside capture (communicator init)
    dist.all_reduce(t, op=dist.ReduceOp.AVG)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=s):
        t.mul_(3.0)
        side.wait_stream(s)
        with torch.cuda.stream(side):
            dist.all_reduce(t, op=dist.ReduceOp.AVG)
        s.wait_stream(side)
        t.add_(1.0)
    torch.cuda.synchronize()
    t.fill_(2.0)
    g.replay()
    torch.cuda.synchronize()
    print("after replay:", float(t[0]), "(want 7.0)", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print("after 2nd replay:", float(t[0]), "(want 22.0)", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
