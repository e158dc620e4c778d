"""The multi-process product path on the GPU: two freshly spawned ranks on
cuda:0, each with its own GpuSession (libcapf_gpu.so), its own node-partitioned
copies (capf_table_node_partition) and its own sharded partial
(capf_chain2_sharded_count), summed by the real all-reduce of dist.py
(gloo here: RCCL refuses two ranks on one device; the driver's N-GPU bench
runs the same code over RCCL).  Both the host-read step and the pipelined
async step of bench.py are exercised; the sum must equal the committed
fixture (s20) / closed form."""
import json
import os
import socket

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, scale, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import capf_import  # noqa: F401
    from capf_amd.dist import (gpu_two_hop_count_sharded, gpu_two_hop_count_sharded_async,
                               node_partitioned_copies)
    from capf_amd.synthetic import rmat_seed, thresholds
    from capf_amd.table import GpuSession
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        s = GpuSession.on_torch_stream(0)
        n, m = 1 << scale, 16 << scale
        full = s.rmat_rels(scale, rmat_seed(scale), thresholds(), 0, m)
        in_copy, out_copy = node_partitioned_copies(full, n, world, rank)
        del full
        partial = torch.zeros(1, dtype=torch.int64, device="cuda")
        sync_count = gpu_two_hop_count_sharded(s, in_copy, out_copy, n, partial)
        slots = torch.full((3,), -1, dtype=torch.int64, device="cuda")
        for i in range(3):
            gpu_two_hop_count_sharded_async(s, in_copy, out_copy, n, slots[i:i + 1])
        torch.cuda.synchronize()
        q.put((rank, sync_count, slots.cpu().tolist(), in_copy.size, out_copy.size))
        dist.destroy_process_group()
    except Exception as e:  # report, do not hang the parent
        q.put((rank, repr(e), None, None, None))


@pytest.mark.parametrize("world,scale", [(2, 20), (3, 18), (3, 16)])
def test_sharded_two_hop_multiprocess(world, scale):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, scale, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=100) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    with open(os.path.join(ROOT, "tests", "golden", "rmat_counts.json")) as f:
        counts = json.load(f)
    if str(scale) in counts["full"]:
        expect = counts["full"][str(scale)]["two_hop"]
    else:
        from oracle import cmodel
        expect = cmodel.stream_counts(scale)["two_hop"]
    for rank, c, slots, nin, nout in res:
        assert c == expect, (rank, c, expect)
        assert slots == [expect] * 3, (rank, slots)
    assert sum(r[3] for r in res) == 16 << scale  # in-copies partition the rels
    assert sum(r[4] for r in res) == 16 << scale  # out-copies too
