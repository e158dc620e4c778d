"""Parity at the BASELINE.json sizes themselves (configs 2-4), against the
committed fixtures of tests/golden/rmat_counts.json.

The fixtures were computed in the dev container by oracle/rmat.c
(make_golden.py): configs 2/3 by streamed closed forms over the same
counter-based R-MAT stream the GPU generates (rmat_stream_counts: Σ in·out −
self-loops; rels with a Person source), config 4 by trace(A³) with
sorted-list intersection (count_triangle_trace, a different algorithm from
csrc/triangle.hip's degree-oriented forward count; both agree with brute
force at s ≤ 10).  Nothing here reads /root/reference or calls the oracle.

These sizes reach code no small case reaches: 256 buckets per side in P1,
hub-split P3 units, the uint16 overflow hand-offs of s24 hubs (in-degree
369,897), the sliced P3 of a node-partitioned rank.
"""
import json
import os

import pytest

from capf_amd.expr import CountStar
from capf_amd.planner import Match, NodeP, Query, RelP, Stage, plan_query, run
from capf_amd.synthetic import rmat_graph, rmat_seed, thresholds

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rmat_counts.json")
with open(GOLDEN) as _f:
    COUNTS = json.load(_f)
FULL = COUNTS["full"]
TRI = COUNTS["triangle"]

TWO_HOP = Query([Match([NodeP("a"), NodeP("b"), NodeP("c")], [RelP("r1", "a", "b"), RelP("r2", "b", "c")])],
                [Stage([("count", CountStar())])])
ONE_HOP_PERSON = Query([Match([NodeP("a", ("Person",)), NodeP("b")], [RelP("r", "a", "b")])],
                       [Stage([("count", CountStar())])])
TRIANGLE = Query([Match([NodeP("a"), NodeP("b"), NodeP("c")],
                        [RelP("r1", "a", "b"), RelP("r2", "b", "c"), RelP("r3", "c", "a")])],
                 [Stage([("count", CountStar())])])


@pytest.mark.parametrize("compact", [3, True, False], ids=["for24", "for32", "int64"])
@pytest.mark.parametrize("scale", [20, 22, 24])
def test_two_hop_headline(gpu_session, scale, compact):
    """Config 3: MATCH (a)-->(b)-->(c) RETURN count(*) — s24 is the headline."""
    g = rmat_graph(gpu_session, scale, compact=compact)
    got = run(g, TWO_HOP)[0]["count"]
    assert gpu_session.last_plan() == "fused_chain2"
    assert got == FULL[str(scale)]["two_hop"]


def test_two_hop_headline_handoff_sync_async(gpu_session):
    """The uint16 P3 counters hand 2^15 off to a log when a hub's counter
    fills (s24 hub in-degree 369,897); the dot kernel folds the log in
    (Σ Δ·other + Σ Δ_in·Δ_out, no overflow launch).  Same fixture
    synchronous and asynchronous."""
    import torch
    g = rmat_graph(gpu_session, 24, compact=3)
    assert run(g, TWO_HOP)[0]["count"] == FULL["24"]["two_hop"]
    slot = torch.full((1,), -1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    plan_query(g, TWO_HOP).table.count_async(slot.data_ptr())
    gpu_session.sync()
    assert slot.item() == FULL["24"]["two_hop"]


@pytest.mark.parametrize("scale", [20, 24])
def test_two_hop_headline_split_runs(gpu_session, monkeypatch, scale):
    """Hub-split P3 units flush with atomic adds into buckets that must start
    at zero.  CAPF_P3_SPLIT=0.5 splits every run above half the mean, so most
    runs split (uint32 bins for split runs, packed pairs for the rest); the
    first unit of each (run, slice) clears its bucket (claim / ready bits) and
    the others wait for it.  Two queries back to back: the second must not see
    the first one's counters."""
    monkeypatch.setenv("CAPF_P3_SPLIT", "0.5")
    monkeypatch.setenv("CAPF_C5_DIRECT", "0")  # (the one-slice pipeline has no split units)
    g = rmat_graph(gpu_session, scale, compact=3)
    for _ in range(2):
        assert run(g, TWO_HOP)[0]["count"] == FULL[str(scale)]["two_hop"]
    assert gpu_session.last_plan() == "fused_chain2"


@pytest.mark.parametrize("direct", ["1", "0"], ids=["no_transpose", "transpose"])
def test_two_hop_headline_s24_both_pipelines(gpu_session, monkeypatch, direct):
    """s24 (one slice): the default pipeline without the transpose and work-list
    kernels (P1 writes run-major meta, one exclusive P3 unit per run, the dot
    sums the self-loops) and the transpose pipeline (CAPF_C5_DIRECT=0) give the
    fixture, twice in a row, synchronously and through count_async."""
    import torch
    monkeypatch.setenv("CAPF_C5_DIRECT", direct)
    g = rmat_graph(gpu_session, 24, compact=3)
    for _ in range(2):
        assert run(g, TWO_HOP)[0]["count"] == FULL["24"]["two_hop"]
    slot = torch.full((1,), -1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    plan_query(g, TWO_HOP).table.count_async(slot.data_ptr())
    gpu_session.sync()
    assert slot.item() == FULL["24"]["two_hop"]


def test_two_hop_headline_async_queue(gpu_session):
    """The pipelined bench mode (capf_table_count_async): 4 in-flight s24
    counts land the fixture in every slot."""
    import torch
    g = rmat_graph(gpu_session, 24, compact=3)
    slots = torch.full((4,), -1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    for i in range(4):
        plan_query(g, TWO_HOP).table.count_async(slots.data_ptr() + 8 * i)
    gpu_session.sync()
    assert slots.cpu().tolist() == [FULL["24"]["two_hop"]] * 4


@pytest.mark.parametrize("parts", [2, 4, 8])
def test_two_hop_headline_node_partitioned(gpu_session, parts):
    """Config 3 across G ranks: every rank's in/out copies and
    its sharded partial, computed one rank after the other on this GPU; the
    partials (what the int64 all-reduce sums) give the fixture."""
    import torch
    from capf_amd.dist import node_partitioned_copies
    from capf_amd.table import chain2_sharded_count_async
    scale = 24
    n, m = 1 << scale, 16 << scale
    full = gpu_session.rmat_rels(scale, rmat_seed(scale), thresholds(), 0, m)
    part = torch.full((parts,), -1, dtype=torch.int64, device="cuda")
    rows = 0
    for p in range(parts):
        in_copy, out_copy = node_partitioned_copies(full, n, parts, p)
        rows += in_copy.size
        chain2_sharded_count_async(gpu_session, in_copy, out_copy, 0, n, parts, p, part.data_ptr() + 8 * p)
        gpu_session.sync()
        del in_copy, out_copy
    assert rows == m  # every rel lands in exactly one in-copy
    assert int(part.sum().item()) == FULL["24"]["two_hop"]


@pytest.mark.parametrize("scale", [20, 22])
def test_one_hop_person_headline(gpu_session, scale):
    """Config 2: MATCH (a:Person)-->(b) RETURN count(*) at s22 (and s20)."""
    g = rmat_graph(gpu_session, scale, person_split=True, compact=True)
    got = run(g, ONE_HOP_PERSON)[0]["count"]
    assert got == FULL[str(scale)]["one_hop_person"]


@pytest.mark.parametrize("scale", [16, 18, 20, 22, 24])
def test_triangle_headline(gpu_session, scale):
    """Config 4: MATCH (a)-->(b)-->(c)-->(a) RETURN count(*)."""
    if str(scale) not in TRI:
        pytest.skip(f"no s{scale} triangle fixture")
    g = rmat_graph(gpu_session, scale, compact=True)
    got = run(g, TRIANGLE)[0]["count"]
    assert gpu_session.last_plan() == "fused_triangle"
    assert got == TRI[str(scale)]


def test_triangle_headline_eight_parts(gpu_session):
    """Config 4 is quoted across 8 GPUs: the 8 row-chunk parts of the s24
    triangle count (capf_triangle_count_part, what each rank computes before
    the int64 all-reduce; computed one after the other on this GPU) sum to the
    committed trace(A³) fixture."""
    import torch
    from capf_amd.table import triangle_count_part_async
    scale, parts = 24, 8
    t = gpu_session.rmat_rels(scale, rmat_seed(scale), thresholds(), 0, 16 << scale)
    d = torch.full((parts,), -1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    for p in range(parts):
        triangle_count_part_async(gpu_session, t, 0, 1 << scale, parts, p, d.data_ptr() + 8 * p)
    gpu_session.sync()
    got = d.cpu().tolist()
    assert all(v >= 0 for v in got)
    assert sum(got) == TRI["24"]
