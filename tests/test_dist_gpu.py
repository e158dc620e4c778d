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


def _spi_worker(rank, world, port, scale, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import traceback
    import torch
    import torch.distributed as dist
    try:
        import capf_import  # noqa: F401
        from capf_amd.dist_table import DistSession, GpuExchange, dist_node_partitioned_graph
        from capf_amd.expr import CountStar
        from capf_amd.graph import ElementTable, ScanGraph
        from capf_amd.planner import Match, NodeP, Query, RelP, Stage, run
        from capf_amd.synthetic import rmat_seed, thresholds
        from capf_amd.table import GpuSession
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        s = GpuSession.on_torch_stream(0)
        n, m = 1 << scale, 16 << scale
        rels = s.rmat_rels(scale, rmat_seed(scale), thresholds(), 0, m)
        nodes = s.range_nodes(0, n, id_col="id")
        full = ScanGraph(s, [ElementTable("node", frozenset(), nodes, {})],
                         [ElementTable("rel", frozenset(["E"]), rels, {})])
        ds = DistSession(s, GpuExchange(s))
        g = dist_node_partitioned_graph(ds, full)
        two = Query([Match([NodeP("a"), NodeP("b"), NodeP("c")], [RelP("r1", "a", "b"), RelP("r2", "b", "c")])],
                    [Stage([("count", CountStar())])])
        s.reset_profile()
        s.set_profiling(True)
        counts = [run(g, two)[0]["count"] for _ in range(3)]
        s.sync()
        s.set_profiling(False)
        kernels = sorted(s.profile())
        q.put((rank, counts, kernels))
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001 - report, do not hang the parent
        q.put((rank, traceback.format_exc(), None))


@pytest.mark.parametrize("world,scale", [(2, 20), (3, 16)])
def test_sharded_two_hop_through_spi_multiprocess(world, scale):
    """MATCH (a)-->(b)-->(c) RETURN count(*) through the unchanged planner on
    a node-partitioned DistTable graph (dist_table.dist_node_partitioned_graph):
    DistTable.group(∅, count(*)) recognises the deferred join chain and runs
    capf_chain2_sharded_count on each rank's copies + ONE all-reduce — the
    c5_* kernels run, no rows move.  Every rank returns the fixture / closed
    form, three queries in a row."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_spi_worker, args=(r, world, port, scale, q)) for r in range(world)]
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
    for rank, got, kernels in res:
        assert kernels is not None, got
        assert got == [expect] * 3, (rank, got, expect)
        assert not any(k.startswith(("route", "pack_rows", "dense_probe", "rj_")) for k in kernels), kernels
    # a rank owning no node_mix bucket (s16 has one bucket of 2^16 keys) launches nothing
    assert any("c5_partition" in k and "c5_gather" in k for _, _, k in res), [k for _, _, k in res]


# ------------------------------------------------ distributed Table layer
def test_hash_route_matches_numpy_router(gpu_session):
    """capf_table_hash_route (csrc/shuffle.hip) puts every row on the owner
    the numpy restatement (oracle/route.py) computes, for INTEGER (plain,
    FOR32, FOR24), FLOAT (−0.0, NaN), BOOL and NULL keys, one and two keys,
    stable inside an owner, every column carried along."""
    import numpy as np
    from ctypes import byref, c_int64, c_void_p
    from capf_amd import _lib
    from capf_amd.expr import T_BOOL, T_FLOAT, T_INT
    from capf_amd.table import GpuTable
    from oracle import route
    rng = np.random.default_rng(7)
    n = 100_003
    ids = rng.integers(0, 1 << 22, n)
    fl = rng.standard_normal(n)
    fl[:5] = [0.0, -0.0, np.nan, -np.nan, 1.5]
    fvalid = rng.random(n) > 0.1
    bo = rng.integers(0, 2, n)
    s = gpu_session
    base = s.table([("k", T_INT, ids, None), ("f", T_FLOAT, fl, fvalid.astype(np.uint8)),
                    ("b", T_BOOL, bo, None), ("row", T_INT, np.arange(n), None)])
    for tab in (base, base.compact(4), base.compact(3)):
        for keys, bits in ((["k"], [route.key_bits("int", ids, np.ones(n, bool))]),
                           (["f", "b"], [route.key_bits("float", fl, fvalid),
                                         route.key_bits("bool", bo, np.ones(n, bool))])):
            for parts in (1, 2, 3, 8):
                want = route.owners(bits, n, parts)
                counts = (c_int64 * parts)()
                h = c_void_p()
                _lib.call("capf_table_hash_route", tab._h, len(keys), _lib.strs(keys), parts, counts, byref(h))
                out = GpuTable(s, h)
                assert list(counts) == np.bincount(want, minlength=parts).tolist()
                rows = np.asarray(out.column_arrays("row")[0])
                assert (rows == np.argsort(want, kind="stable")).all()  # owner order, stable
                assert (out.column_arrays("k")[0] == ids[rows]).all()


def _dist_cases_worker(rank, world, port, q, compact=None, chunk=(0, 1)):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import traceback
    import torch
    import torch.distributed as dist
    try:
        import capf_import  # noqa: F401
        from conftest import case_parts, check_case
        from reference_cases import CASES
        from capf_amd.dist_table import DistSession, GpuExchange, dist_scan_graph
        from capf_amd.graph import ScanGraph
        from capf_amd.planner import run
        from capf_amd.table import GpuSession
        from oracle.create_parser import parse_create
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        s = GpuSession.on_torch_stream(0)
        ds = DistSession(s, GpuExchange(s))
        bad = []
        k, nk = chunk
        mine = CASES[k * len(CASES) // nk:(k + 1) * len(CASES) // nk]
        for compact in ((False, 3) if compact is None else (compact,)):
            for case in mine:
                cid, src, create, query, expected, opts = case_parts(case)
                if opts.get("local_only"):  # LIST property columns are not routed between ranks
                    continue
                full = ScanGraph.from_data(s, parse_create(create), compact=compact)
                try:
                    got = run(dist_scan_graph(ds, full), query, opts.get("params"))
                    ok = check_case(got, expected, opts)
                except Exception as e:  # noqa: BLE001 - reported per case
                    got, ok = repr(e), False
                if not ok:
                    bad.append((cid, compact, str(got)[:300]))
        q.put((rank, bad, len(mine)))
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001 - report, do not hang the parent
        q.put((rank, [("worker", traceback.format_exc())], 0))


@pytest.mark.timeout(400)
@pytest.mark.parametrize("compact", [False, 3], ids=["int64", "for24"])
@pytest.mark.parametrize("chunk", [0, 1])
def test_reference_cases_distributed_on_gpu(compact, chunk):
    """Every reference acceptance case through the unchanged planner on
    DistTable shards of GpuTables (dist_table.py): two spawned ranks on
    cuda:0, rows routed by capf_table_hash_route and moved by
    all_to_all_single (gloo, host-staged: RCCL refuses two ranks on one
    device; the N-GPU path is the same code over RCCL), int64 and FOR24
    element tables."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dist_cases_worker, args=(r, 2, port, q, compact, (chunk, 2))) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=380) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank, bad, n in res:
        assert n > 50 and not bad, f"rank {rank}: {len(bad)} failing: {bad}"
