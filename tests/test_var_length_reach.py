"""Fused config-5 path: the planner sends the unchanged okapi relational plan
(VarLengthExpand join chain + isomorphism filters + UNION ALL, DISTINCT,
GROUP BY — VarLengthExpandPlanner.scala:82-259) through the Table SPI; the
runtime recognises Group(a; count(*)) ∘ Distinct(a, b) ∘ UNION ALL of the
chains in its plan DAG (fused_count.hip::try_fused_reach) and runs the BFS of
csrc/var_length_reach.hip.  Checked against (1) the scipy matrix-power
restatement (oracle/reach.py), (2) the unfused relational plan on the GPU
(CAPF_FUSED_REACH=0) and (3) the isomorphic-path brute force on the
reference's LDBC sample."""
import numpy as np
import pytest

from ldbc import config5_query, ldbc_graph_data

from capf_amd.expr import CountStar, Var
from capf_amd.graph import GraphData, ScanGraph
from capf_amd.planner import Match, NodeP, Query, RelP, Stage, run
from oracle import cmodel
from oracle import reach as oreach


def synthetic(scale, person_frac=0.6, seed=5):
    """R-MAT edges on sparse LDBC-style ids, Person/Other labels, KNOWS plus
    a second rel type that the pattern must ignore."""
    src, dst = cmodel.rmat(scale)
    n = 1 << scale
    rng = np.random.default_rng(seed)
    ids = np.arange(n, dtype=np.int64) * 1000003 + 65 - (n // 2) * 1000003  # negatives too
    person = rng.random(n) < person_frac
    nodes = [(int(ids[i]), frozenset(["Person" if person[i] else "Other"]), {}) for i in range(n)]
    other = rng.random(len(src)) < 0.1
    rels = [(10 ** 12 + k, int(ids[s]), int(ids[d]), "LIKES" if other[k] else "KNOWS", {})
            for k, (s, d) in enumerate(zip(src.tolist(), dst.tolist()))]
    knows = ~other
    return (GraphData(nodes, rels), ids[src[knows]], ids[dst[knows]], ids[person])


def reach_query(upper, direction="out", lower=1):
    return Query([Match([NodeP("a", ("Person",)), NodeP("b", ("Person",))],
                        [RelP("k", "a", "b", ("KNOWS",), direction=direction, length=(lower, upper))])],
                 [Stage([("a", Var("a")), ("b", Var("b"))], distinct=True),
                  Stage([("a", Var("a")), ("reach", CountStar())])])


def test_oracle_on_ldbc_sample():
    g = ldbc_graph_data()
    src = np.array([r[1] for r in g.rels])
    dst = np.array([r[2] for r in g.rels])
    persons = np.array([nd[0] for nd in g.nodes])
    from test_ldbc_config5 import brute_force
    assert oreach.config5_histogram(src, dst, persons, persons) == brute_force()


@pytest.mark.gpu
def test_config5_fused_on_ldbc_sample(gpu_session):
    from test_ldbc_config5 import brute_force
    g = ScanGraph.from_data(gpu_session, ldbc_graph_data())
    gpu_session.reset_profile()
    got = run(g, config5_query())
    assert gpu_session.last_plan() == "fused_var_length_reach"
    assert sorted([r["reach"], r["n"]] for r in got) == brute_force()


@pytest.mark.gpu
@pytest.mark.parametrize("upper", [1, 2, 3, 4])
@pytest.mark.parametrize("compact", [False, True], ids=["int64", "for32"])
def test_reach_vs_matrix_powers(gpu_session, upper, compact):
    data, ks, kd, persons = synthetic(10)
    g = ScanGraph.from_data(gpu_session, data, compact=compact)
    gpu_session.reset_profile()
    got = {r["a"]: r["reach"] for r in run(g, reach_query(upper))}
    assert gpu_session.last_plan() == "fused_var_length_reach"
    assert got == oreach.reach_counts(ks, kd, persons, persons, upper)


@pytest.mark.gpu
def test_reach_incoming_direction(gpu_session):
    data, ks, kd, persons = synthetic(9)
    g = ScanGraph.from_data(gpu_session, data)
    # (a)<-[:KNOWS*1..3]-(b) grouped by b: walks from b along the rels
    q = Query([Match([NodeP("a", ("Person",)), NodeP("b", ("Person",))],
                     [RelP("k", "a", "b", ("KNOWS",), direction="in", length=(1, 3))])],
              [Stage([("a", Var("a")), ("b", Var("b"))], distinct=True),
               Stage([("b", Var("b")), ("reach", CountStar())])])
    got = {r["b"]: r["reach"] for r in run(g, q)}
    assert got == oreach.reach_counts(ks, kd, persons, persons, 3)


@pytest.mark.parametrize("upper", [1, 3])
def test_relational_from_zero_on_oracle(upper):
    """The relational lowering of *0..u (join chains + the copyElement branch,
    DISTINCT, GROUP BY) on the oracle equals the matrix-power restatement with
    the self pair: pins the lower-bound-0 semantics the fused path follows."""
    from oracle.table_np import OracleSession
    data, ks, kd, persons = synthetic(6)
    got = {r["a"]: r["reach"] for r in run(ScanGraph.from_data(OracleSession(), data),
                                           reach_query(upper, lower=0))}
    assert got == oreach.reach_counts(ks, kd, persons, persons, upper, lower=0)


@pytest.mark.gpu
@pytest.mark.parametrize("upper", [1, 3])
@pytest.mark.parametrize("compact", [False, True], ids=["int64", "for32"])
def test_reach_from_zero_vs_matrix_powers(gpu_session, upper, compact):
    data, ks, kd, persons = synthetic(10)
    g = ScanGraph.from_data(gpu_session, data, compact=compact)
    gpu_session.reset_profile()
    got = {r["a"]: r["reach"] for r in run(g, reach_query(upper, lower=0))}
    assert gpu_session.last_plan() == "fused_var_length_reach"
    assert got == oreach.reach_counts(ks, kd, persons, persons, upper, lower=0)


@pytest.mark.gpu
@pytest.mark.parametrize("lower,upper", [(1, 2), (1, 3), (0, 1), (0, 3)])
def test_fused_equals_relational_plan(gpu_session, monkeypatch, lower, upper):
    """The fused operator and the okapi relational lowering (join chain with
    relationship-isomorphism filters, UNION ALL, DISTINCT, GROUP BY) agree
    row for row on the GPU, self-loops and multi-edges included; lower bound
    0 adds the copyElement branch (VarLengthExpandPlanner.scala:180-205):
    every source pairs with itself once."""
    data, *_ = synthetic(6)
    g = ScanGraph.from_data(gpu_session, data)
    q = reach_query(upper, lower=lower)
    q.stages.append(Stage([("reach", Var("reach")), ("n", CountStar())]))
    gpu_session.reset_profile()
    fused = sorted([r["reach"], r["n"]] for r in run(g, q))
    assert gpu_session.last_plan() == "fused_var_length_reach"
    monkeypatch.setenv("CAPF_FUSED_REACH", "0")
    gpu_session.reset_profile()
    plain = sorted([r["reach"], r["n"]] for r in run(g, q))
    assert gpu_session.last_plan() == "none"
    assert fused == plain


# ------------------------------------------------ config 5 at its BASELINE size
def _sf10_graph(session):
    """LDBC-SF10-shaped KNOWS — 2^16 Person nodes,
    R-MAT (Graph500 a/b/c) rels with edge factor 30 (1,966,080), generated in HBM."""
    from capf_amd.graph import ElementTable
    from capf_amd.synthetic import rmat_seed, thresholds
    scale, ef = 16, 30
    rels = session.rmat_rels(scale, rmat_seed(scale), thresholds(), 0, ef << scale)
    nodes = session.range_nodes(0, 1 << scale, id_col="id")
    g = ScanGraph(session, [ElementTable("node", frozenset(["Person"]), nodes, {})],
                  [ElementTable("rel", frozenset(["KNOWS"]), rels, {})])
    return g, rels


def _fixture5():
    import json
    import os
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    with open(os.path.join(here, "rmat_counts.json")) as f:
        summary = json.load(f)["config5"]
    with open(os.path.join(here, summary["histogram_file"])) as f:
        return summary, json.load(f)["histogram"]


def test_config5_fixture_consistent():
    summary, hist = _fixture5()
    assert len(hist) == summary["histogram_rows"]
    assert sum(r * n for r, n in hist) == summary["pairs"]
    assert sum(n for _, n in hist) == summary["sources"]
    assert summary["rels"] == summary["edge_factor"] << summary["scale"]


@pytest.mark.parametrize("scale,ef", [(9, 8), (11, 30)])
def test_c_bitset_bfs_vs_matrix_powers(scale, ef):
    """oracle/rmat.c::reach_bitset (the config-5 fixture's oracle) against the
    scipy matrix powers and against isomorphic-path enumeration."""
    src, dst = cmodel.rmat(scale, ef)
    n = 1 << scale
    p = np.arange(n)
    for upper in (1, 2, 3):
        r = cmodel.reach_bitset(src, dst, n, upper)
        exp = oreach.reach_counts(src, dst, p, p, upper)
        assert {int(a): int(c) for a, c in enumerate(r) if c} == exp
    sample = np.arange(0, n, 5)
    rp, paths = cmodel.reach_paths(src, dst, n, sample, 3)
    assert np.array_equal(rp, cmodel.reach_bitset(src, dst, n, 3)[sample]) and paths > 0


@pytest.mark.gpu
def test_config5_sf10_histogram(gpu_session):
    """The config-5 query at its BASELINE size against the committed fixture
    (C bitset BFS, tests/golden/config5_sf10.json)."""
    summary, hist = _fixture5()
    g, _ = _sf10_graph(gpu_session)
    gpu_session.reset_profile()
    got = sorted([r["reach"], r["n"]] for r in run(g, config5_query()))
    assert gpu_session.last_plan() == "fused_var_length_reach"
    assert got == hist
    assert sum(r * n for r, n in got) == summary["pairs"] == 1819538648


@pytest.mark.gpu
def test_config5_sf10_per_source(gpu_session):
    """reach per source at SF10 size against the C BFS run on the same edges
    (downloaded), and the fixture's weighted checksum."""
    summary, _ = _fixture5()
    g, rels = _sf10_graph(gpu_session)
    got = {r["a"]: r["reach"] for r in run(g, reach_query(3))}
    src, _ = rels.column_arrays("source")
    dst, _ = rels.column_arrays("target")
    exp = cmodel.reach_bitset(src, dst, 1 << 16, 3)
    assert got == {a: int(c) for a, c in enumerate(exp) if c}
    w = sum((a + 1) * c for a, c in got.items()) % (1 << 63)
    assert w == summary["weighted"]


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{}, {"CAPF_VR_COUNT": "0"}, {"CAPF_VR_BUDGET": "4e7"},
                                 {"CAPF_VR_BUDGET": "4e7", "CAPF_VR_COUNT": "0"}],
                         ids=["default", "ballot_count", "batched", "batched_ballot"])
def test_reach_multiblock_paths(gpu_session, monkeypatch, env):
    """More than 4096 sources and node rows (several count blocks on both grid
    axes, cross-block atomics) and — with a small state budget — several
    source batches: both count kernels against the C BFS (scale 13)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    scale = 13
    src, dst = cmodel.rmat(scale, 16)
    n = 1 << scale
    nodes = [(i, frozenset(["Person"]), {}) for i in range(n)]
    rels = [(k, int(s), int(d), "KNOWS", {}) for k, (s, d) in enumerate(zip(src.tolist(), dst.tolist()))]
    g = ScanGraph.from_data(gpu_session, GraphData(nodes, rels))
    got = {r["a"]: r["reach"] for r in run(g, reach_query(3))}
    exp = cmodel.reach_bitset(src, dst, n, 3)
    assert got == {a: int(c) for a, c in enumerate(exp) if c}
