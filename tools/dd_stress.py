"""Diagnostic: repeat the multi-rank (ranks on one GPU, gloo transport) action
and PCG of sem_dd; report run-to-run differences, plans and iteration counts."""
import os
import socket
import sys

import numpy as np
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, world, port, check, tag):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from spectralelementmethod_amd.distributed import OverlappedOperator, StripPartition
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    p, nex, ney = 8, 12, 6
    part = StripPartition(nex, ney, p, world, rank)
    nodes, e2n = part.local_mesh(0.05)
    op = OverlappedOperator(p, nodes, e2n, part.neighbors, 1, dev, owned=part.owned,
                            transport="torch", world=world, rank=rank)
    plans = [(o.plan_info()["atomic_groups"], o.plan_info()["colours"]) for o in op.ops]
    g = torch.Generator(device=dev).manual_seed(21)
    u = torch.randn(op.ndof, dtype=torch.float64, device=dev, generator=g)
    y0 = op.apply(u)
    torch.cuda.synchronize()
    md = 0.0
    for _ in range(20):
        y = op.apply(u)
        md = max(md, ((y - y0).abs().max() / y0.abs().max()).item())
    d0 = op.diag()
    dd = 0.0
    for _ in range(10):
        dd = max(dd, ((op.diag() - d0).abs().max() / d0.abs().max()).item())
    x_n = torch.from_numpy(nodes[0]).to(dev)
    y_n = torch.from_numpy(nodes[1]).to(dev)
    xs = torch.sin(0.5 * np.pi * x_n) * torch.cos(0.5 * np.pi * y_n) + x_n * y_n
    on = (torch.abs(x_n.abs() - 1) < 1e-9) | (torch.abs(y_n.abs() - 1) < 1e-9)
    b = op.apply(xs)
    res = []
    for t in range(4):
        x = torch.where(on, xs, torch.zeros_like(xs))
        try:
            x, its, rel = op.pcg_solve(b, x, on, rtol=1e-12, check_every=check)
            res.append(its)
        except Exception as e:
            res.append(str(e)[:40])
    print("%s check=%d rank %d: plans %s action max rel diff %.2e, diag %.2e, pcg its %s" % (
        tag, check, rank, plans, md, dd, res), flush=True)
    op.close()
    dist.destroy_process_group()


def run(check, tag):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.start_processes(worker, args=(2, port, check, tag), nprocs=2, start_method="spawn")


if __name__ == "__main__":
    tag = sys.argv[1] if len(sys.argv) > 1 else "base"
    for check in (1, 4, 16, 4):
        run(check, tag)
