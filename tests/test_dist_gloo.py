"""Multi-process (world size 2, gloo, CPU) check of the distributed 2-hop
combine (dist.py): shard-local histograms → reduce-scatter → dot → all-reduce
must equal the single-process closed form bit-exactly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, scale, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import capf_import  # noqa: F401
    from capf_amd.dist import combine_two_hop, edge_range, padded_nodes
    from oracle import cmodel
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = 16 << scale
    n = 1 << scale
    lo, hi = edge_range(m, rank, world)
    src, dst = cmodel.rmat(scale, first=lo, count=hi - lo)
    i, o, loops = cmodel.degree_hists(src, dst, 0, n)
    npad = padded_nodes(n, world)
    ti = torch.zeros(npad, dtype=torch.int32)
    to = torch.zeros(npad, dtype=torch.int32)
    ti[:n] = torch.from_numpy(i.astype(np.int32))
    to[:n] = torch.from_numpy(o.astype(np.int32))
    dot = lambda a, b: int((a.numpy().astype(np.int64) * b.numpy().astype(np.int64)).sum())
    total = combine_two_hop(ti, to, loops, dot)
    q.put((rank, total))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_two_hop_combine(world):
    scale = 10
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, scale, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    import capf_import  # noqa: F401
    from oracle import cmodel
    src, dst = cmodel.rmat(scale)
    expect = cmodel.count_2hop(src, dst, 1 << scale)
    assert all(v == expect for v in res.values()), (res, expect)
