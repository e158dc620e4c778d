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
    """One rank of the node-partitioned count with the product's host side
    (capf_amd.dist: owned_buckets = the split capf_table_node_partition uses,
    sum_partials = the one collective) and the oracle's partial in place of
    the GPU kernel (no GPU here; tests/test_dist_gpu.py runs the kernels)."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import capf_import  # noqa: F401
    from capf_amd import dist as cdist
    from oracle import cmodel, nodemix
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 1 << scale
    src, dst = cmodel.rmat(scale)
    b0, b1 = cdist.owned_buckets(n, world, rank)
    k = cdist.hist_bits(n)
    own = lambda x: ((nodemix.node_mix(x, k) >> 16) >= b0) & ((nodemix.node_mix(x, k) >> 16) < b1)  # noqa: E731
    in_dst = dst[own(dst)]
    out_mask = own(src)
    out_src, out_dst = src[out_mask], dst[out_mask]
    ein = np.bincount(in_dst, minlength=n).astype(np.int64)
    eout = np.bincount(out_src, minlength=n).astype(np.int64)
    partial = int((ein * eout).sum()) - int((out_src == out_dst).sum())
    t = torch.tensor([partial], dtype=torch.int64)
    cdist.sum_partials(t)
    q.put((rank, int(t.item()), len(in_dst)))
    dist.destroy_process_group()


def test_owned_buckets_match_owner():
    """dist.owned_buckets (host) and the oracle's owner() (restating the
    device owner_of) give every node exactly one owner, for world sizes that do
    and do not divide the bucket count."""
    import capf_import  # noqa: F401
    from capf_amd import dist as cdist
    from oracle import nodemix
    for scale in (16, 18, 20):
        n = 1 << scale
        x = np.arange(n)
        for world in (1, 2, 3, 5, 8):
            own = nodemix.owner(x, n, world)
            k = cdist.hist_bits(n)
            b = nodemix.node_mix(x, k) >> 16
            for r in range(world):
                b0, b1 = cdist.owned_buckets(n, world, r)
                assert np.array_equal((b >= b0) & (b < b1), own == r), (scale, world, r)


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
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    import capf_import  # noqa: F401
    from oracle import cmodel
    src, dst = cmodel.rmat(scale)
    expect = cmodel.count_2hop(src, dst, 1 << scale)
    assert all(v == expect for _, v, _ in res), (res, expect)
    assert sum(r[2] for r in res) == len(src)
