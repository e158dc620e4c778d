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
