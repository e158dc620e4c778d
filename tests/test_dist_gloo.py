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


def _sharded_worker(rank, world, port, scale, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import capf_import  # noqa: F401
    from oracle import cmodel, nodemix
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 1 << scale
    src, dst = cmodel.rmat(scale)
    # this rank's copies (capf_table_node_partition): rels it owns the target / source of
    in_dst = dst[nodemix.owner(dst, n, world) == rank]
    out_mask = nodemix.owner(src, n, world) == rank
    out_src, out_dst = src[out_mask], dst[out_mask]
    ein = np.bincount(in_dst, minlength=n).astype(np.int64)
    eout = np.bincount(out_src, minlength=n).astype(np.int64)
    partial = int((ein * eout).sum()) - int((out_src == out_dst).sum())
    t = torch.tensor([partial], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)  # the one collective of the sharded count
    q.put((rank, int(t.item())))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_node_partitioned_two_hop(world):
    """Node-partitioned layout (dist.gpu_two_hop_count_sharded): per-rank
    partials over the owned nodes, one int64 all-reduce, equal the closed form."""
    scale = 18  # 4 buckets of 64 Ki: uneven bucket ranges at world 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, scale, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    import capf_import  # noqa: F401
    from oracle import cmodel
    src, dst = cmodel.rmat(scale)
    expect = cmodel.count_2hop(src, dst, 1 << scale)
    assert all(v == expect for v in res.values()), (res, expect)
