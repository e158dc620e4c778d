"""The distributed Table layer (capf_amd/dist_table.py) on CPU: world-size 2
and 3 gloo process groups run EVERY reference acceptance case
(tests/golden/reference_cases.py) through the unchanged planner on DistTable
shards — node tables sharded by h(id), rel tables by h(source), joins
co-partitioned / shuffled / broadcast, GROUP BY and DISTINCT shuffled,
global aggregates combined from per-rank partials, ORDER BY / SKIP / LIMIT
on rank 0 — and every rank must return the reference's expected rows.
The shards are numpy oracle tables moved by tests/dist_support.py; the GPU
exchange of the same operators is tests/test_dist_gpu.py."""
import os
import socket
import sys
import traceback

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    try:
        sys.path[:0] = [ROOT, HERE, os.path.join(HERE, "golden")]
        import capf_import  # noqa: F401
        from conftest import case_parts, check_case
        from dist_support import OracleExchange
        from reference_cases import CASES

        from capf_amd.dist_table import DistSession, dist_scan_graph
        from capf_amd.graph import ScanGraph
        from capf_amd.planner import run
        from oracle.create_parser import parse_create
        from oracle.table_np import OracleSession
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        ds = DistSession(OracleSession(), OracleExchange())
        bad = []
        for case in CASES:
            cid, src, create, query, expected, opts = case_parts(case)
            full = ScanGraph.from_data(OracleSession(), parse_create(create))
            try:
                got = run(dist_scan_graph(ds, full), query, opts.get("params"))
                ok = check_case(got, expected, opts)
            except Exception as e:  # noqa: BLE001 - reported per case
                got, ok = repr(e), "raises" in opts
            if not ok:
                bad.append((cid, str(got)[:300]))
        q.put((rank, bad, len(CASES)))
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        q.put((rank, [("worker", traceback.format_exc())], 0))


@pytest.mark.parametrize("world", [2, 3])
def test_reference_cases_distributed_on_oracle(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, bad, n in res:
        assert n > 100 and not bad, f"rank {rank}: {len(bad)} failing cases: {bad[:5]}"


def _two_hop_worker(rank, world, port, q):
    try:
        sys.path[:0] = [ROOT, HERE, os.path.join(HERE, "golden")]
        import capf_import  # noqa: F401
        import numpy as np
        from conftest import bag
        from dist_support import OracleExchange, oracle_count_copies
        from capf_amd.dist_table import DistSession, dist_node_partitioned_graph
        from capf_amd.expr import CountStar, IntegerLit, LessThan, Multiply, Var
        from capf_amd.graph import GraphData, ScanGraph
        from capf_amd.planner import Match, NodeP, Query, RelP, Stage, run
        from oracle import cmodel
        from oracle.table_np import OracleSession
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        scale = 8
        src, dst = cmodel.rmat(scale)
        n = 1 << scale
        data = GraphData([(i + 5, frozenset(), {}) for i in range(n)],
                         [(100000 + k, int(a) + 5, int(b) + 5, "E", {}) for k, (a, b) in enumerate(zip(src, dst))])
        full = ScanGraph.from_data(OracleSession(), data)
        ds = DistSession(OracleSession(), OracleExchange())
        g = dist_node_partitioned_graph(ds, full, count_copies=oracle_count_copies)
        two = Query([Match([NodeP("a"), NodeP("b"), NodeP("c")], [RelP("r1", "a", "b"), RelP("r2", "b", "c")])],
                    [Stage([("count", CountStar())])])
        got = run(g, two)[0]["count"]
        # mirrored pattern (a)<--(b)<--(c): the same chain
        back = Query([Match([NodeP("a"), NodeP("b"), NodeP("c")],
                            [RelP("r1", "a", "b", direction="in"), RelP("r2", "b", "c", direction="in")])],
                     [Stage([("count", CountStar())])])
        got_back = run(g, back)[0]["count"]
        dispatched = len(oracle_count_copies.calls)
        # not the 2-hop count: the deferred operators replay eagerly (shuffles, joins)
        rows = Query([Match([NodeP("a"), NodeP("b")], [RelP("r", "a", "b")])],
                     [Stage([("a", Var("a")), ("b", Var("b"))])])
        got_rows = run(g, rows)
        one = run(g, Query([Match([NodeP("a"), NodeP("b")], [RelP("r", "a", "b")])],
                           [Stage([("count", CountStar())])]))[0]["count"]
        ref_rows = run(full, rows)
        # a WHERE that is not a uniqueness filter: no sharded count, the chain replays
        where = Query([Match([NodeP("a"), NodeP("b"), NodeP("c")], [RelP("r1", "a", "b"), RelP("r2", "b", "c")],
                             where=[LessThan(Var("a"), IntegerLit(40))])],
                      [Stage([("count", CountStar())])])
        got3 = run(g, where)[0]["count"]
        want3 = run(full, where)[0]["count"]
        # the sharded count's host-held row feeding a further projection (moved to
        # the device only then)
        doubled = run(g, Query(two.matches, [Stage([("c", CountStar())]),
                                             Stage([("d", Multiply(Var("c"), IntegerLit(2)))])]))[0]["d"]
        # duplicate rel ids (two rels sharing id 100000) or a NULL endpoint: no
        # node-partitioned layout, the plan replays and matches the single-process one
        extra = []
        for rels in ([(100000 if k == 7 else 100000 + k, int(a) + 5, int(b) + 5, "E", {})
                      for k, (a, b) in enumerate(zip(src, dst))],
                     [(100000 + k, None if k == 3 else int(a) + 5, int(b) + 5, "E", {})
                      for k, (a, b) in enumerate(zip(src, dst))]):
            d2 = GraphData(data.nodes, rels)
            full2 = ScanGraph.from_data(OracleSession(), d2)
            before = len(oracle_count_copies.calls)
            g2 = dist_node_partitioned_graph(DistSession(OracleSession(), OracleExchange()), full2,
                                             count_copies=oracle_count_copies)
            extra.append((run(g2, two)[0]["count"], run(full2, two)[0]["count"],
                          len(oracle_count_copies.calls) - before))
        q.put((rank, got, got_back, dispatched, bag(got_rows) == bag(ref_rows), one,
               got3 == want3 > 0 and doubled == 2 * got and all(a == b and k == 0 for a, b, k in extra),
               cmodel.count_2hop(src, dst, n), len(src)))
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        q.put((rank, traceback.format_exc()) + (None,) * 7)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_two_hop_through_spi(world):
    """The 2-hop count(*) through the unchanged planner on a node-partitioned
    DistTable graph: DistTable.group(∅, count(*)) sees the deferred join
    chain, every rank adds its partial, one all-reduce sums them (no rows
    shuffled); the mirrored pattern is the same chain; other queries on the
    same graph replay the deferred operators eagerly and match the
    single-process plan."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_two_hop_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, got, got_back, dispatched, rows_ok, one, three_ok, want, m in res:
        assert isinstance(got, int), got
        assert got == want and got_back == want, (rank, got, got_back, want)
        assert dispatched == 2, dispatched  # both chains took the sharded count
        assert rows_ok and one == m and three_ok


def _fuzz_worker(rank, world, port, q):
    try:
        sys.path[:0] = [ROOT, HERE, os.path.join(HERE, "golden")]
        import capf_import  # noqa: F401
        from conftest import bag
        from dist_support import OracleExchange
        from test_pattern_fuzz import CASES, graph, query

        from capf_amd.dist_table import DistSession, dist_scan_graph
        from capf_amd.graph import ScanGraph
        from capf_amd.planner import run
        from oracle.table_np import OracleSession
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        ds = DistSession(OracleSession(), OracleExchange())
        bad = []
        for gs, qs in CASES[::3]:
            g, qy = graph(gs), query(qs)
            want = run(ScanGraph.from_data(OracleSession(), g), qy)
            try:
                got = run(dist_scan_graph(ds, ScanGraph.from_data(OracleSession(), g)), qy)
                if bag(got) != bag(want):
                    bad.append((gs, qs, len(got), len(want)))
            except Exception as e:  # noqa: BLE001 - reported per case
                bad.append((gs, qs, repr(e)[:200]))
        q.put((rank, bad))
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        q.put((rank, [("worker", traceback.format_exc())]))


def test_random_patterns_distributed_on_oracle():
    """The 100 seeded pattern cases of tests/test_pattern_fuzz.py (every third)
    over 2 DistTable ranks: the same bags as one session."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fuzz_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, bad in res:
        assert not bad, f"rank {rank}: {len(bad)} failing cases: {bad[:4]}"
