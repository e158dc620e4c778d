"""GPU parity: the HIP backend (through the C-ABI) against the oracle.

 * every reference acceptance case (tests/golden/reference_cases.py) runs
   through planner → GpuTable → libcapf_gpu.so and must equal both the
   reference's expected Bag and the numpy oracle;
 * R-MAT configs 2/3 counts are bit-exact against the C closed forms and the
   Flink-shaped pipelined join (oracle/rmat.c) at small scales, and the fused
   path must be the one that ran;
 * Table operators are checked one by one against the oracle on seeded data.
"""
import numpy as np
import pytest

from conftest import bag, case_parts, check_case
from reference_cases import CASES, ERROR_CASES

from capf_amd import _lib
from capf_amd.expr import (Add, Ands, Avg, BoolLit, Coalesce, Count, CountStar, Divide, ElementProperty,
                           Equals, FloatLit, GreaterThan, IntegerLit, IsNotNull, IsNull, LessThan, Max, Min,
                           Modulo, Multiply, Not, NullLit, Ors, StringLit, Subtract, Sum, ToFloat,
                           ToInteger, Var, T_BOOL, T_FLOAT, T_INT, T_STRING)
from capf_amd.graph import ScanGraph
from capf_amd.header import RecordHeader
from capf_amd.planner import Match, NodeP, Query, RelP, Stage, plan_query, run
from capf_amd.synthetic import rmat_graph
from oracle import cmodel
from oracle.create_parser import parse_create
from oracle.table_np import OracleSession

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("compact", [False, True, 3], ids=["int64", "for32", "for24"])
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_reference_case_on_gpu(gpu_session, case, compact, monkeypatch):
    if compact == 3:  # one encoding runs every reference case through the radix join
        monkeypatch.setenv("CAPF_JOIN", "radix")
    cid, src, create, query, expected, opts = case_parts(case)
    g = ScanGraph.from_data(gpu_session, parse_create(create), compact=compact)
    got = run(g, query, opts.get("params"))
    assert check_case(got, expected, opts), f"{cid} ({src}): {got}"
    og = ScanGraph.from_data(OracleSession(), parse_create(create))
    want = run(og, query, opts.get("params"))
    assert check_case(got, want, {k: v for k, v in opts.items() if k != "row_count"}, reference=False) \
        if "row_count" not in opts else len(got) == len(want)


@pytest.mark.parametrize("case", ERROR_CASES, ids=[c[0] for c in ERROR_CASES])
def test_reference_error_case_on_gpu(gpu_session, case):
    """The exception class the reference test expects (MatchTests.scala:380-418)."""
    cid, src, create, query, exc = case
    with pytest.raises(Exception) as ei:
        run(ScanGraph.from_data(gpu_session, parse_create(create)), query)
    assert type(ei.value).__name__ == exc, f"{cid} ({src}): {ei.value!r}"


def test_union_graph_on_gpu(gpu_session):
    from test_oracle_golden import check_union_graph, check_union_graph_scans, check_union_graph_schema
    check_union_graph(gpu_session)
    check_union_graph_scans(gpu_session)
    check_union_graph_schema(gpu_session)


def test_scan_graph_schema_on_gpu(gpu_session):
    from test_oracle_golden import check_scan_graph_schema
    check_scan_graph_schema(gpu_session)


TWO_HOP = Query([Match([NodeP("a"), NodeP("b"), NodeP("c")], [RelP("r1", "a", "b"), RelP("r2", "b", "c")])],
                [Stage([("count", CountStar())])])
ONE_HOP_PERSON = Query([Match([NodeP("a", ("Person",)), NodeP("b")], [RelP("r", "a", "b")])],
                       [Stage([("count", CountStar())])])


@pytest.mark.parametrize("compact", [False, True, 3], ids=["int64", "for32", "for24"])
@pytest.mark.parametrize("scale", [6, 8, 10, 12, 14, 16, 18])
def test_two_hop_count_rmat(gpu_session, scale, compact):
    g = rmat_graph(gpu_session, scale, compact=compact)
    got = run(g, TWO_HOP)[0]["count"]
    assert gpu_session.last_plan() == "fused_chain2"
    src, dst = cmodel.rmat(scale)
    assert got == cmodel.count_2hop(src, dst, 1 << scale)
    if scale <= 12:
        p = cmodel.Pipeline(np.arange(1 << scale), np.arange(len(src)), src, dst)
        assert got == p.probe(0, len(src), 4)


@pytest.mark.parametrize("variant", ["partitioned", "atomic"])
@pytest.mark.parametrize("compact", [False, True, 3], ids=["int64", "for32", "for24"])
@pytest.mark.parametrize("scale,count,nodes", [(6, None, None), (11, 30001, None), (14, None, None),
                                               (15, 123457, None), (12, None, 3000), (14, 50001, 9999)])
def test_two_hop_partition_variants(gpu_session, monkeypatch, variant, compact, scale, count, nodes):
    """Every histogram path, forced at small and ragged sizes (count not a
    multiple of the 4-rel vector or the tile) and with a node table smaller
    than the id range (range checks + dummy run), must give the closed form."""
    monkeypatch.setenv("CAPF_CHAIN2", variant)
    g = rmat_graph(gpu_session, scale, compact=compact, count=count, n_nodes=nodes)
    got = run(g, TWO_HOP)[0]["count"]
    assert gpu_session.last_plan() == "fused_chain2"
    src, dst = cmodel.rmat(scale, count=count)
    assert got == cmodel.count_2hop(src, dst, nodes or 1 << scale)


@pytest.mark.parametrize("query", ["two_hop", "triangle", "one_hop_person", "grouped"])
def test_count_async_matches_size(gpu_session, query):
    """capf_table_count_async: a queue of in-flight counts (no host wait per
    query) lands the same values as the synchronous records path — fused
    chain2 / triangle on the device, the other shapes through the fallback."""
    import torch
    tri = Query([Match([NodeP("a"), NodeP("b"), NodeP("c")],
                       [RelP("r1", "a", "b"), RelP("r2", "b", "c"), RelP("r3", "c", "a")])],
                [Stage([("count", CountStar())])])
    grouped = Query([Match([NodeP("a"), NodeP("b")], [RelP("r", "a", "b")])],
                    [Stage([("a", Var("a")), ("n", CountStar())])])
    q = {"two_hop": TWO_HOP, "triangle": tri, "one_hop_person": ONE_HOP_PERSON, "grouped": grouped}[query]
    g = rmat_graph(gpu_session, 12, person_split=query == "one_hop_person", compact=True)
    if query == "grouped":
        want = len(run(g, q))  # row count of the grouped table
    else:
        want = run(g, q)[0]["count"]
    slots = torch.full((6,), -1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()  # the fill runs on torch's stream, the counts on the session's
    for i in range(6):
        plan_query(g, q).table.count_async(slots.data_ptr() + 8 * i)
    gpu_session.sync()
    assert slots.cpu().tolist() == [want] * 6
    if query == "two_hop":
        src, dst = cmodel.rmat(12)
        assert want == cmodel.count_2hop(src, dst, 1 << 12)


def test_rmat_generator_bit_exact(gpu_session):
    t = gpu_session.rmat_rels(12, cmodel.rmat_seed(12), cmodel.thresholds(), 1000, 5000)
    src, dst = cmodel.rmat(12, first=1000, count=5000)
    s, _ = t.column_arrays("source")
    d, _ = t.column_arrays("target")
    i, _ = t.column_arrays("id")
    assert np.array_equal(s, src) and np.array_equal(d, dst)
    assert np.array_equal(i, np.arange(1000, 6000))


@pytest.mark.parametrize("compact", [False, True, 3], ids=["int64", "for32", "for24"])
@pytest.mark.parametrize("scale,count", [(8, None), (12, None), (16, None), (12, 40001), (14, 9)])
def test_one_hop_person_count_rmat(gpu_session, scale, count, compact):
    """Config 2; `count` makes the rel table ragged (not a multiple of the
    4-row vector loads of the FOR32 root kernel)."""
    g = rmat_graph(gpu_session, scale, person_split=True, count=count, compact=compact)
    got = run(g, ONE_HOP_PERSON)[0]["count"]
    src, dst = cmodel.rmat(scale, count=count)
    person = cmodel.labels(1 << scale, cmodel.rmat_seed(scale))
    assert got == cmodel.count_1hop(src, dst, 1 << scale, in_a=person)


@pytest.mark.parametrize("semi", ["0", "1"], ids=["probe_rows", "partitioned"])
@pytest.mark.parametrize("compact", [True, 3], ids=["for32", "for24"])
@pytest.mark.parametrize("scale,count", [(16, None), (18, None), (18, 3000001), (20, None)])
def test_one_hop_person_partitioned_semijoin(gpu_session, scale, count, compact, semi, monkeypatch):
    """Config 2 at sizes where the Person bitmap is probed radix-partitioned
    (chain2_partitioned.hip::bits_count_partitioned: keys grouped by bucket,
    the bucket's bitmap slice in LDS) against the row-by-row probes; ragged
    tile counts included.  Both equal the oracle."""
    monkeypatch.setenv("CAPF_SEMI_PART", semi)
    g = rmat_graph(gpu_session, scale, person_split=True, count=count, compact=compact)
    gpu_session.reset_profile()
    gpu_session.set_profiling(True)
    got = run(g, ONE_HOP_PERSON)[0]["count"]
    got2 = run(g, ONE_HOP_PERSON)[0]["count"]  # the second query reuses the cached bitmaps
    gpu_session.set_profiling(False)
    src, dst = cmodel.rmat(scale, count=count)
    person = cmodel.labels(1 << scale, cmodel.rmat_seed(scale))
    want = cmodel.count_1hop(src, dst, 1 << scale, in_a=person)
    assert got == got2 == want
    assert ("semi_count" in gpu_session.profile()) == (semi == "1")


@pytest.mark.parametrize("compact", [False, True, 3], ids=["int64", "for32", "for24"])
@pytest.mark.parametrize("scale,nodes", [(12, 3000), (14, 9999), (16, None)])
def test_one_hop_person_partial_node_range(gpu_session, scale, nodes, compact):
    """Config 2 with a node table narrower than the rel ids (rels whose target
    is not a node drop out): the all-ones message of (b) may only be skipped
    when the target column provably lies in the node range (statistics);
    here it does not, and the count must still be exact.  Plus the
    pipelined async path of the message-passing count."""
    import torch
    g = rmat_graph(gpu_session, scale, person_split=True, compact=compact, n_nodes=nodes)
    got = run(g, ONE_HOP_PERSON)[0]["count"]
    n = nodes or 1 << scale
    src, dst = cmodel.rmat(scale)
    person = cmodel.labels(1 << scale, cmodel.rmat_seed(scale))[:n]
    want = cmodel.count_1hop(src, dst, n, in_a=person)
    assert got == want
    slots = torch.full((3,), -1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    for i in range(3):
        plan_query(g, ONE_HOP_PERSON).table.count_async(slots.data_ptr() + 8 * i)
    gpu_session.sync()
    assert slots.cpu().tolist() == [want] * 3


def test_two_hop_materialized_vs_oracle(gpu_session):
    """The non-fused path: return the joined rows themselves."""
    q = Query([Match([NodeP("a"), NodeP("b"), NodeP("c")], [RelP("r1", "a", "b"), RelP("r2", "b", "c")])],
              [Stage([("a", Var("a")), ("b", Var("b")), ("c", Var("c"))])])
    g = rmat_graph(gpu_session, 7, edge_factor=4)
    got = run(g, q)
    src, dst = cmodel.rmat(7, edge_factor=4)
    og = ScanGraph.from_data(OracleSession(), _graph_data(src, dst, 1 << 7))
    exp = run(og, q)
    assert bag(got) == bag(exp)


def _graph_data(src, dst, n):
    from capf_amd.graph import GraphData
    return GraphData(nodes=[(i, frozenset(["V"]), {}) for i in range(n)],
                     rels=[(i, int(s), int(d), "E", {}) for i, (s, d) in enumerate(zip(src, dst))])


def test_two_hop_general_message_passing(gpu_session):
    """Sparse (non-dense) ids force the hashed message-passing count."""
    rng = np.random.default_rng(7)
    n, m = 300, 3000
    ids = rng.choice(10 ** 12, size=n, replace=False).astype(np.int64)
    s = ids[rng.integers(0, n, m)]
    d = ids[rng.integers(0, n, m)]
    d[:50] = s[:50]  # self-loops
    from capf_amd.graph import GraphData
    gd = GraphData(nodes=[(int(i), frozenset(["V"]), {}) for i in ids],
                   rels=[(10 ** 13 + k, int(a), int(b), "E", {}) for k, (a, b) in enumerate(zip(s, d))])
    g = ScanGraph.from_data(gpu_session, gd)
    got = run(g, TWO_HOP)[0]["count"]
    og = ScanGraph.from_data(OracleSession(), gd)
    assert got == run(og, TWO_HOP)[0]["count"]


# ----------------------------------------------------------------- operators
def _rand_tables(seed=3, n=500):
    rng = np.random.default_rng(seed)
    words = ["alpha", "beta", "gamma", "delta", None]
    cols = [
        ("k", T_INT, [int(x) if rng.random() > 0.1 else None for x in rng.integers(0, 20, n)], None),
        ("f", T_FLOAT, [float(x) if rng.random() > 0.1 else None for x in rng.normal(size=n)], None),
        ("s", T_STRING, [words[i] for i in rng.integers(0, 5, n)], None),
        ("b", T_BOOL, [bool(x) if rng.random() > 0.1 else None for x in rng.integers(0, 2, n)], None),
        ("i", T_INT, list(range(n)), None),
    ]
    return cols


def _both(cols):
    gs = pytest.gpu_session_ref
    g = gs.table(cols)
    if pytest.capf_compact:
        width = 3 if pytest.capf_compact == 3 else 4
        g = g.compact(width)
        for name, t, values, _ in cols:  # every non-empty INTEGER/STRING column is re-encoded
            if t in (T_INT, T_STRING):
                assert g.encoding(name)[0] in ((1, 2) if width == 3 else (1,)), name
    return g, OracleSession().table(cols)


@pytest.fixture(autouse=True)
def _expose(gpu_session):
    pytest.gpu_session_ref = gpu_session
    pytest.capf_compact = False


@pytest.fixture(params=[False, True, 3], ids=["int64", "for32", "for24"])
def encoding(request, _expose):
    """Operator tests run on plain int64 columns and on FOR32 / FOR24-compacted ones."""
    pytest.capf_compact = request.param


H = RecordHeader({Var("k"): "k", Var("f"): "f", Var("s"): "s", Var("b"): "b", Var("i"): "i"})

FILTERS = [
    GreaterThan(Var("k"), IntegerLit(10)),
    Equals(Var("s"), StringLit("beta")),
    Not(Equals(Var("s"), StringLit("beta"))),
    Ands(LessThan(Var("f"), FloatLit(0.5)), Var("b")),
    Ors(IsNull(Var("k")), Equals(Var("b"), BoolLit(False))),
    Equals(Modulo(Var("i"), IntegerLit(7)), IntegerLit(3)),
    GreaterThan(Add(Var("k"), Var("f")), FloatLit(10.0)),
    IsNotNull(Coalesce(Var("k"), Var("f"))),
    Equals(NullLit("INTEGER"), Var("k")),
]


@pytest.mark.parametrize("pred", FILTERS, ids=[str(p) for p in FILTERS])
@pytest.mark.usefixtures("encoding")
def test_filter_parity(pred):
    g, o = _both(_rand_tables())
    assert bag(g.filter(pred, H, {}).rows) == bag(o.filter(pred, H, {}).rows)


JH = RecordHeader({Var("a"): "a", Var("x"): "x", Var("s"): "s", Var("ka"): "ka",
                   Var("b"): "b", Var("y"): "y", Var("t"): "t", Var("kb"): "kb"})
JOIN_FILTERS = [
    Not(Equals(Var("x"), Var("y"))),  # the relational uniqueness filter r_i <> r_j
    Ands(Not(Equals(Var("x"), Var("y"))), GreaterThan(Var("a"), IntegerLit(3))),
    LessThan(Var("x"), Var("y")),
    Ands(Equals(Var("s"), Var("t")), Not(Equals(Var("a"), Var("b")))),
    Ands(Not(Equals(Var("x"), Var("y"))), Not(Equals(Var("a"), Var("b"))), LessThan(Var("b"), IntegerLit(9))),
    Ors(Equals(Var("x"), Var("y")), IsNull(Var("a"))),  # (not a conjunction: the interpreter)
]


@pytest.mark.parametrize("pred", JOIN_FILTERS, ids=[str(p) for p in JOIN_FILTERS])
@pytest.mark.parametrize("paths", ["default", "interpreter_compose"])
@pytest.mark.usefixtures("encoding")
def test_filter_over_join_parity(pred, paths, monkeypatch):
    """WHERE over a join's (lazy) output: conjunctions of comparisons run as
    terms read through the join's row indexes, and the selection writes the
    composed indexes of both sides itself (kernels_basic.hip filter_select);
    CAPF_FILTER_TERMS=0 / CAPF_FILTER_SELECT=0 force the interpreter and the
    selection-index + compose path.  Many-to-many keys, NULL operands."""
    if paths != "default":
        monkeypatch.setenv("CAPF_FILTER_TERMS", "0")
        monkeypatch.setenv("CAPF_FILTER_SELECT", "0")
    rng = np.random.default_rng(11)
    words = ["p", "q", "r", None]
    n = 700
    left = [("a", T_INT, [int(v) if rng.random() > 0.1 else None for v in rng.integers(0, 12, n)], None),
            ("x", T_INT, [int(v) for v in rng.integers(0, 40, n)], None),
            ("s", T_STRING, [words[i] for i in rng.integers(0, 4, n)], None),
            ("ka", T_INT, [int(v) for v in rng.integers(0, 30, n)], None)]
    right = [("b", T_INT, [int(v) if rng.random() > 0.1 else None for v in rng.integers(0, 12, n)], None),
             ("y", T_INT, [int(v) for v in rng.integers(0, 40, n)], None),
             ("t", T_STRING, [words[i] for i in rng.integers(0, 4, n)], None),
             ("kb", T_INT, [int(v) for v in rng.integers(0, 30, n)], None)]
    gl, ol = _both(left)
    gr, orr = _both(right)
    got = gl.join(gr, "inner", ("ka", "kb")).filter(pred, JH, {}).rows
    want = ol.join(orr, "inner", ("ka", "kb")).filter(pred, JH, {}).rows
    assert len(want) > 0
    assert bag(got) == bag(want)


@pytest.mark.parametrize("pred", JOIN_FILTERS, ids=[str(p) for p in JOIN_FILTERS])
@pytest.mark.parametrize("fused", ["1", "0"], ids=["fused", "join_then_filter"])
@pytest.mark.usefixtures("encoding")
def test_filter_fused_into_radix_join(pred, fused, monkeypatch):
    """WHERE over an inner radix join: the join's EMIT evaluates the terms per
    pair and writes only the passing pairs (radix_join.hip radix_join_filtered:
    one pass, failing pairs' slots refilled from the tail); CAPF_RJ_FILTER=0
    joins, then filters.  Same bag as the oracle; the fused kernels ran exactly
    when the predicate is a conjunction of terms.  Many-to-many keys, NULL
    operands, hub keys."""
    monkeypatch.setenv("CAPF_JOIN", "radix")
    monkeypatch.setenv("CAPF_RJ_FILTER", fused)
    rng = np.random.default_rng(13)
    words = ["p", "q", "r", None]
    n = 1500
    kl = [int(v) for v in rng.integers(0, 30, n)]
    kr = [int(v) for v in rng.integers(0, 30, n)]
    kl[:300] = [7] * 300  # a hub key: 300 × (its right rows) pairs, split over sub-items
    kr[:200] = [7] * 200
    left = [("a", T_INT, [int(v) if rng.random() > 0.1 else None for v in rng.integers(0, 12, n)], None),
            ("x", T_INT, [int(v) for v in rng.integers(0, 40, n)], None),
            ("s", T_STRING, [words[i] for i in rng.integers(0, 4, n)], None),
            ("ka", T_INT, kl, None)]
    right = [("b", T_INT, [int(v) if rng.random() > 0.1 else None for v in rng.integers(0, 12, n)], None),
             ("y", T_INT, [int(v) for v in rng.integers(0, 40, n)], None),
             ("t", T_STRING, [words[i] for i in rng.integers(0, 4, n)], None),
             ("kb", T_INT, kr, None)]
    gl, ol = _both(left)
    gr, orr = _both(right)
    gs = pytest.gpu_session_ref
    gs.reset_profile()
    gs.set_profiling(True)
    got = gl.join(gr, "inner", ("ka", "kb")).filter(pred, JH, {}).rows
    gs.set_profiling(False)
    want = ol.join(orr, "inner", ("ka", "kb")).filter(pred, JH, {}).rows
    assert len(want) > 0
    assert ("rj_join_filter_emit" in gs.profile()) == (fused == "1" and not isinstance(pred, Ors))
    assert bag(got) == bag(want)


@pytest.mark.parametrize("fail", ["few", "many"])
@pytest.mark.parametrize("idx", ["int32", "int64"])
def test_filter_fused_radix_holes(gpu_session, monkeypatch, fail, idx):
    """The one-pass filtered EMIT: failing pairs leave holes that the tail's
    pairs fill (a few: the uniqueness filter's self-loop pairs); past 2^20
    holes (here x < y fails on ~1.2 M of 2.56 M hub pairs) the join counts the
    passes per sub-item first and writes them compactly.  Exact pair set
    against numpy (int32 and int64 pair indexes)."""
    monkeypatch.setenv("CAPF_JOIN", "radix")
    monkeypatch.setenv("CAPF_IDX64", "1" if idx == "int64" else "0")
    rng = np.random.default_rng(31)
    n = 1600
    x = rng.integers(0, 40, n).astype(np.int64)
    y = rng.integers(0, 40, n).astype(np.int64)
    if fail == "few":
        y = np.full(n, 1000, dtype=np.int64)  # x < y everywhere but in the right rows set below
        y[::97] = -1
    k = np.full(n, 7, dtype=np.int64)
    gl = gpu_session.table([("x", T_INT, x, None), ("ka", T_INT, k, None), ("li", T_INT, np.arange(n), None)])
    gr = gpu_session.table([("y", T_INT, y, None), ("kb", T_INT, k, None), ("ri", T_INT, np.arange(n), None)])
    hdr = RecordHeader({Var("x"): "x", Var("y"): "y", Var("ka"): "ka", Var("kb"): "kb",
                        Var("li"): "li", Var("ri"): "ri"})
    gpu_session.reset_profile()
    gpu_session.set_profiling(True)
    out = gl.join(gr, "inner", ("ka", "kb")).filter(LessThan(Var("x"), Var("y")), hdr, {})
    li, _ = out.column_arrays("li")
    ri, _ = out.column_arrays("ri")
    gpu_session.set_profiling(False)
    prof = gpu_session.profile()
    assert "rj_join_filter_emit" in prof
    assert ("rj_join_filter_count" in prof) == (fail == "many")
    wl, wr = np.nonzero(x[:, None] < y[None, :])
    got = np.sort(li.astype(np.int64) * n + ri)
    assert np.array_equal(got, np.sort(wl.astype(np.int64) * n + wr))


@pytest.mark.parametrize("jt", ["left_outer", "right_outer", "full_outer"])
@pytest.mark.parametrize("pred", [Not(Equals(Var("x"), Var("y"))), IsNull(Var("c")), IsNotNull(Var("c")),
                                  Ands(Not(Equals(Var("x"), Var("y"))), Equals(Var("c"), IntegerLit(7)))],
                         ids=["neq", "c_null", "c_not_null", "neq_and_c"])
def test_filter_over_outer_join_constant_column(jt, pred):
    """An outer join turns a projected literal of the null-extended side into a
    nullable lazy column over a constant; a WHERE over that join's output must
    compose its index (kernels_basic.hip filter_select), not treat it as a fill
    (the 8-B placeholder selection index was read m times)."""
    rng = np.random.default_rng(12)
    n = 900
    left = [("x", T_INT, [int(v) for v in rng.integers(0, 40, n)], None),
            ("ka", T_INT, [int(v) for v in rng.integers(0, 1500, n)], None)]  # sparse keys: unmatched rows
    right = [("y", T_INT, [int(v) for v in rng.integers(0, 40, n)], None),
             ("kb", T_INT, [int(v) for v in rng.integers(0, 1500, n)], None)]
    hdr = RecordHeader({Var("x"): "x", Var("ka"): "ka", Var("y"): "y", Var("kb"): "kb", Var("c"): "c"})
    gl, ol = _both(left)
    gr, orr = _both(right)
    rh = RecordHeader({Var("y"): "y", Var("kb"): "kb"})
    gr = gr.withColumns((IntegerLit(7), "c"), header=rh, params={})
    orr = orr.withColumns((IntegerLit(7), "c"), header=rh, params={})
    got = gl.join(gr, jt, ("ka", "kb")).filter(pred, hdr, {}).rows
    want = ol.join(orr, jt, ("ka", "kb")).filter(pred, hdr, {}).rows
    assert len(want) > 0 or (jt == "right_outer" and isinstance(pred, IsNull))  # c is never NULL there
    assert bag(got) == bag(want)


EXPRS = [Add(Var("k"), IntegerLit(3)), Multiply(Var("f"), FloatLit(2.5)), Divide(Var("k"), IntegerLit(3)),
         Subtract(Var("i"), Var("k")), ToFloat(Var("k")), ToInteger(Multiply(Var("f"), FloatLit(1e3))),
         Coalesce(Var("k"), IntegerLit(-1)), Divide(Var("i"), Var("k"))]


@pytest.mark.parametrize("e", EXPRS, ids=[str(e) for e in EXPRS])
@pytest.mark.usefixtures("encoding")
def test_with_columns_parity(e):
    g, o = _both(_rand_tables())
    rg = g.withColumns((e, "x"), header=H, params={}).rows
    ro = o.withColumns((e, "x"), header=H, params={}).rows
    assert len(rg) == len(ro)
    for a, b in zip(rg, ro):  # row order is preserved by withColumns
        if isinstance(a["x"], float) or isinstance(b["x"], float):
            assert (a["x"] is None) == (b["x"] is None)
            if a["x"] is not None:
                assert a["x"] == pytest.approx(b["x"], rel=1e-12, abs=0)
        else:
            assert a["x"] == b["x"]


@pytest.fixture(params=["auto", "radix", "hash"])
def join_mode(request, monkeypatch):
    """Both materialising join implementations: the radix-partitioned LDS
    join (radix_join.hip) and the global hash table (kernels_hash.hip)."""
    if request.param != "auto":
        monkeypatch.setenv("CAPF_JOIN", request.param)
    return request.param


@pytest.mark.parametrize("jt", ["inner", "left_outer", "right_outer", "full_outer", "cross"])
@pytest.mark.usefixtures("encoding", "join_mode")
def test_join_parity(jt):
    rng = np.random.default_rng(11)
    n1, n2 = (60, 40) if jt == "cross" else (400, 300)
    a = [("ak", T_INT, [int(x) if rng.random() > 0.1 else None for x in rng.integers(0, 50, n1)], None),
         ("as", T_STRING, [["x", "y", "z"][i] for i in rng.integers(0, 3, n1)], None),
         ("av", T_FLOAT, [float(x) for x in rng.normal(size=n1)], None)]
    b = [("bk", T_INT, [int(x) if rng.random() > 0.1 else None for x in rng.integers(0, 50, n2)], None),
         ("bs", T_STRING, [["x", "y", "z"][i] for i in rng.integers(0, 3, n2)], None),
         ("bv", T_INT, list(range(n2)), None)]
    gs = pytest.gpu_session_ref
    ga, gb = gs.table(a), gs.table(b)
    if pytest.capf_compact:  # mixed encodings: FOR32/FOR24 left keys probe plain right keys
        ga = ga.compact(3 if pytest.capf_compact == 3 else 4)
    oa, ob = OracleSession().table(a), OracleSession().table(b)
    pairs = [] if jt == "cross" else [("ak", "bk"), ("as", "bs")]
    assert bag(ga.join(gb, jt, *pairs).rows) == bag(oa.join(ob, jt, *pairs).rows)
    if jt != "cross":  # one key column: the radix join's shape
        one = [("ak", "bk")]
        assert bag(ga.join(gb, jt, *one).rows) == bag(oa.join(ob, jt, *one).rows)
        st = [("as", "bs")]  # a STRING key (dictionary codes)
        assert bag(ga.join(gb, jt, *st).rows) == bag(oa.join(ob, jt, *st).rows)


@pytest.mark.parametrize("jt", ["inner", "left_outer", "right_outer", "full_outer"])
@pytest.mark.parametrize("sizes", [(0, 500), (500, 0), (3000, 200000), (300000, 5000), (70000, 70000)])
@pytest.mark.parametrize("idx", ["int32", "int64"])
def test_radix_join_large(gpu_session, monkeypatch, jt, sizes, idx):
    """The radix join at sizes that fill many partitions, with skewed keys
    (one key on 20 % of the rows: chunked LDS builds and split probe items),
    NULL keys on both sides, empty sides; checked against numpy.  Both widths
    of the pair list's row indexes (int32 by default below 2^31 rows;
    CAPF_IDX64=1 keeps int64)."""
    monkeypatch.setenv("CAPF_JOIN", "radix")
    monkeypatch.setenv("CAPF_IDX64", "1" if idx == "int64" else "0")
    rng = np.random.default_rng(sum(sizes))
    nl, nr = sizes
    def keys(n, hot):
        k = rng.integers(0, max(n // 3, 1) + 7, n).astype(np.int64)
        if hot:  # the larger side: one key on 20 % of its rows
            k[: n // 5] = 42
        return k
    lk, rk = keys(nl, nl >= nr), keys(nr, nr > nl)
    lv = np.ones(nl, dtype=np.uint8)
    lv[::97] = 0
    rv = np.ones(nr, dtype=np.uint8)
    rv[::89] = 0
    ga = gpu_session.table([("lk", T_INT, lk, lv), ("li", T_INT, np.arange(nl), None)])
    gb = gpu_session.table([("rk", T_INT, rk, rv), ("ri", T_INT, np.arange(nr), None)])
    out = ga.join(gb, jt, ("lk", "rk"))
    li, lok = out.column_arrays("li")
    ri, rok = out.column_arrays("ri")
    got = sorted(zip(np.where(lok, li, -1).tolist(), np.where(rok, ri, -1).tolist()))
    # numpy reference: pairs of non-null equal keys, plus unmatched rows of outer sides
    lval, rval = np.nonzero(lv)[0], np.nonzero(rv)[0]
    from collections import defaultdict
    byk = defaultdict(list)
    for j in rval:
        byk[int(rk[j])].append(int(j))
    pairs, lm, rm = [], set(), set()
    for i in lval:
        for j in byk.get(int(lk[i]), ()):
            pairs.append((int(i), j))
            lm.add(int(i))
            rm.add(j)
    if jt in ("left_outer", "full_outer"):
        pairs += [(i, -1) for i in range(nl) if i not in lm]
    if jt in ("right_outer", "full_outer"):
        pairs += [(-1, j) for j in range(nr) if j not in rm]
    assert got == sorted(pairs)


@pytest.mark.parametrize("jt", ["inner", "left_outer", "right_outer", "full_outer"])
@pytest.mark.parametrize("sizes", [(3000, 200000), (300000, 5000), (70000, 70001), (1, 1000), (50000, 1)])
def test_radix_join_unique_build(gpu_session, monkeypatch, jt, sizes):
    """The radix join (forced) whose smaller (build) side has every non-NULL
    key once — including a one-row build side — through the run-based COUNT
    and the ranges EMIT: sparse int64 keys, misses on both sides, NULL keys on
    both; checked against numpy."""
    monkeypatch.setenv("CAPF_JOIN", "radix")
    rng = np.random.default_rng(sum(sizes) + 5)
    nl, nr = sizes
    nb, npr = min(nl, nr), max(nl, nr)
    bkeys = rng.permutation(np.arange(2 * nb + 3, dtype=np.int64))[:nb] * 1000003 + 7  # unique, sparse
    pkeys = rng.integers(0, 2 * nb + 3, npr).astype(np.int64) * 1000003 + 7           # some miss
    bv = np.ones(nb, dtype=np.uint8)
    bv[1::53] = 0  # (row 0 keeps its key: the one-row build side joins a real key)
    pv = np.ones(npr, dtype=np.uint8)
    pv[::61] = 0
    lk, lv, rk, rv = (bkeys, bv, pkeys, pv) if nl < nr else (pkeys, pv, bkeys, bv)
    ga = gpu_session.table([("lk", T_INT, lk, lv), ("li", T_INT, np.arange(nl), None)])
    gb = gpu_session.table([("rk", T_INT, rk, rv), ("ri", T_INT, np.arange(nr), None)])
    gpu_session.reset_profile()
    gpu_session.set_profiling(True)
    out = ga.join(gb, jt, ("lk", "rk"))
    li, lok = out.column_arrays("li")
    ri, rok = out.column_arrays("ri")
    gpu_session.set_profiling(False)
    assert "rj_partition1" in gpu_session.profile()  # the radix path ran
    got = sorted(zip(np.where(lok, li, -1).tolist(), np.where(rok, ri, -1).tolist()))
    byk = {int(rk[j]): int(j) for j in np.nonzero(rv)[0]} if nl >= nr else None
    pairs, lm, rm = [], set(), set()
    if byk is not None:
        for i in np.nonzero(lv)[0]:
            j = byk.get(int(lk[i]))
            if j is not None:
                pairs.append((int(i), j)); lm.add(int(i)); rm.add(j)
    else:
        byl = {int(lk[i]): int(i) for i in np.nonzero(lv)[0]}
        for j in np.nonzero(rv)[0]:
            i = byl.get(int(rk[j]))
            if i is not None:
                pairs.append((i, int(j))); lm.add(i); rm.add(int(j))
    if jt in ("left_outer", "full_outer"):
        pairs += [(i, -1) for i in range(nl) if i not in lm]
    if jt in ("right_outer", "full_outer"):
        pairs += [(-1, j) for j in range(nr) if j not in rm]
    assert got == sorted(pairs)


def test_join_overlapping_columns_raises():
    g, _ = _both(_rand_tables())
    with pytest.raises(_lib.IllegalArgumentException):
        g.join(g, "inner", ("k", "k"))


@pytest.mark.usefixtures("encoding")
def test_union_distinct_parity():
    g, o = _both(_rand_tables())
    g2 = g.select("i", "k", "s", "f", "b")  # different column order: matched by name
    o2 = o.select("i", "k", "s", "f", "b")
    assert bag(g.unionAll(g2).rows) == bag(o.unionAll(o2).rows)
    # union of a FOR32 and a plain table (different bases) decodes to int64
    gp = pytest.gpu_session_ref.table(_rand_tables(seed=5))
    op = OracleSession().table(_rand_tables(seed=5))
    assert bag(g.unionAll(gp).rows) == bag(o.unionAll(op).rows)
    assert bag(g.select("k", "s").distinct().rows) == bag(o.select("k", "s").distinct().rows)
    # distinct(cols): one row per distinct value of cols
    rg = g.distinct("s").rows
    ro = o.distinct("s").rows
    assert sorted(map(repr, [r["s"] for r in rg])) == sorted(map(repr, [r["s"] for r in ro]))


@pytest.mark.usefixtures("encoding")
def test_group_parity():
    g, o = _both(_rand_tables(n=2000))
    aggs = {"cnt": CountStar(), "cf": Count(Var("f")), "sk": Sum(Var("k")), "mn": Min(Var("f")),
            "mx": Max(Var("k")), "av": Avg(Var("f")), "ai": Avg(Var("k")), "sf": Sum(Var("f")),
            "cd": Count(Var("k"), True)}
    by = [Var("s"), Var("b")]
    rg = {(r["s"], r["b"]): r for r in g.group(by, aggs, header=H, params={}).rows}
    ro = {(r["s"], r["b"]): r for r in o.group(by, aggs, header=H, params={}).rows}
    assert rg.keys() == ro.keys()
    for key in rg:
        for c in aggs:
            x, y = rg[key][c], ro[key][c]
            if isinstance(y, float):
                assert x == pytest.approx(y, rel=1e-12, abs=1e-12), (key, c)
            else:
                assert x == y, (key, c)
    # global aggregation (no keys), including over an empty input
    assert g.group([], {"c": CountStar()}, header=H).rows == [{"c": 2000}]
    e = g.filter(BoolLit(False), H, {})
    assert e.group([], {"c": CountStar(), "s": Sum(Var("k"))}, header=H).rows == [{"c": 0, "s": None}]


@pytest.mark.parametrize("nulls", [False, True], ids=["dense", "with_nulls"])
def test_fp64_sum_avg_exact_at_size(gpu_session, nulls):
    """FLOAT sum / avg (FlinkSQLExprMapper.scala:281-287) at 1.2e7 rows against
    math.fsum (exactly rounded): mixed signs over 12 decades, ±1e15 pairs that
    cancel exactly inside groups (an uncompensated fp64 running sum loses the
    low bits there), a few huge groups and many small ones, and the global
    aggregate.  North-star tolerance 1e-12 relative; two runs bit-identical
    (kernels_hash.hip fp64_sum_groups: fixed order, double-double)."""
    import math
    rng = np.random.default_rng(2026)
    n = 12_000_000
    k = np.where(rng.random(n) < 0.4, rng.integers(0, 3, n), rng.integers(3, 4003, n)).astype(np.int64)
    f = rng.standard_normal(n) * 10.0 ** rng.integers(-6, 7, n)
    big = rng.choice(n, 20000, replace=False)
    f[big[:10000]] = 1e15
    f[big[10000:]] = -1e15
    k[big[10000:]] = k[big[:10000]]  # each +1e15 has a −1e15 partner in its group
    valid = None
    if nulls:
        valid = (rng.random(n) > 0.05).astype(np.uint8)
        valid[big] = 1
    t = gpu_session.table([("k", T_INT, k, None), ("f", T_FLOAT, f, valid)])
    hdr = RecordHeader({Var("k"): "k", Var("f"): "f"})
    aggs = {"s": Sum(Var("f")), "a": Avg(Var("f")), "c": Count(Var("f"))}
    out = t.group([Var("k")], aggs, header=hdr, params={})
    ks, _ = out.column_arrays("k")
    sv, _ = out.column_arrays("s")
    av, _ = out.column_arrays("a")
    cv, _ = out.column_arrays("c")
    keep = np.ones(n, bool) if valid is None else valid.astype(bool)
    order = np.argsort(k[keep], kind="stable")
    kk, ff = k[keep][order], f[keep][order]
    bounds = np.flatnonzero(np.diff(kk)) + 1
    starts = np.concatenate([[0], bounds])
    ends = np.concatenate([bounds, [len(kk)]])
    exact = {int(kk[a]): (math.fsum(ff[a:b].tolist()), b - a) for a, b in zip(starts, ends)}
    assert len(ks) == len(exact)
    worst = 0.0
    for key, s_, a_, c_ in zip(ks.tolist(), sv.tolist(), av.tolist(), cv.tolist()):
        es, ec = exact[key]
        assert c_ == ec
        worst = max(worst, abs(s_ - es) / abs(es), abs(a_ - es / ec) / abs(es / ec))
    assert worst <= 1e-12, worst
    # bit-identical on a second run
    sv2, _ = t.group([Var("k")], aggs, header=hdr, params={}).column_arrays("s")
    assert np.array_equal(sv.view(np.uint64), sv2.view(np.uint64))
    # the global aggregate
    g = t.group([], {"s": Sum(Var("f")), "a": Avg(Var("f"))}, header=hdr, params={}).rows[0]
    es = math.fsum(f[keep].tolist())
    assert abs(g["s"] - es) <= 1e-12 * abs(es)
    assert abs(g["a"] - es / keep.sum()) <= 1e-12 * abs(es / keep.sum())


@pytest.mark.usefixtures("encoding")
def test_order_skip_limit_parity():
    g, o = _both(_rand_tables())
    for items in ([(Var("k"), "asc"), (Var("i"), "desc")], [(Var("f"), "desc"), (Var("i"), "asc")]):
        rg = g.orderBy(*items, header=H, params={}).skip(13).limit(100).rows
        ro = o.orderBy(*items, header=H, params={}).skip(13).limit(100).rows
        assert [r["i"] for r in rg] == [r["i"] for r in ro]


def test_compact_for24_roundtrip(gpu_session):
    """FOR24 (3-byte offsets): values, NULLs, a base near 2^62, ragged row
    counts (not a multiple of the 4-row group), the widest 24-bit range, and
    columns too wide for 24 bits (FOR32) or 32 bits (plain)."""
    big = 2 ** 62
    for n in (1, 3, 4, 5, 1027):
        vals = [big + (i * 7919) % (1 << 24) if i % 5 else None for i in range(n)]
        vals[0] = big  # min
        if n > 1:
            vals[-1] = big + (1 << 24) - 1  # max: range exactly 2^24 - 1
        cols = [("a", T_INT, vals, None), ("w", T_INT, [i << 24 for i in range(n)], None)]
        t = gpu_session.table(cols).compact(3)
        assert t.encoding("a") == (2, big), n
        assert t.encoding("w")[0] == (2 if n == 1 else 1 if n - 1 < 256 else 0), n
        assert t.column_values("a") == vals
        assert t.column_values("w") == [i << 24 for i in range(n)]
        # gather (filter) and concat (union) of a FOR24 column
        ha = RecordHeader({Var("a"): "a"})
        f = t.filter(GreaterThan(Var("a"), IntegerLit(big + 1000)), ha, {})
        assert f.column_values("a") == [v for v in vals if v is not None and v > big + 1000]
        u = t.select("a").unionAll(gpu_session.table([("a", T_INT, [5, None], None)]))
        assert u.column_values("a") == vals + [5, None]


def test_compact_roundtrip(gpu_session):
    big = 10 ** 15
    cols = [("a", T_INT, [big + 7, big, None, big + 2 ** 32 - 1], None),
            ("w", T_INT, [0, 2 ** 40, 1, 2], None),          # range > 2^32: stays plain
            ("n", T_INT, [None, None, None, None], None)]    # all null: stays plain
    t = gpu_session.table(cols).compact()
    assert t.encoding("a") == (1, big)
    assert t.encoding("w")[0] == 0 and t.encoding("n")[0] == 0
    assert t.column_values("a") == [big + 7, big, None, big + 2 ** 32 - 1]
    assert t.column_values("w") == [0, 2 ** 40, 1, 2]
    ha = RecordHeader({Var("a"): "a"})
    assert t.filter(GreaterThan(Var("a"), IntegerLit(big + 3)), ha, {}).column_values("a") == \
        [big + 7, big + 2 ** 32 - 1]


def test_unit_and_empty(gpu_session):
    assert gpu_session.unit().size == 1
    e = gpu_session.empty(["a", "b"], [T_INT, T_STRING])
    assert e.size == 0 and e.physicalColumns == ["a", "b"]
    assert e.columnType == {"a": "INTEGER", "b": "STRING"}


@pytest.mark.parametrize("variant", ["partitioned", "atomic"])
@pytest.mark.parametrize("compact", [False, True, 3], ids=["int64", "for32", "for24"])
@pytest.mark.parametrize("scale,base", [(10, 0), (13, 5), (16, 0)])
def test_local_hists_hashed_layout(gpu_session, monkeypatch, variant, compact, scale, base):
    """capf_chain2_local_hists: every counter of the node_mix-indexed in/out
    histograms equals the oracle's degree count (partitioned and atomic paths
    share the layout), and the self-loop count matches."""
    import torch
    from capf_amd.table import chain2_hist_len
    from oracle import nodemix
    monkeypatch.setenv("CAPF_CHAIN2", variant)
    m = 16 << scale
    t = gpu_session.rmat_rels(scale, cmodel.rmat_seed(scale), cmodel.thresholds(), 0, m)
    if compact:
        t = t.compact()
    n = (1 << scale) - base  # node range [base, 2^scale): rels touching ids < base drop out
    hl = chain2_hist_len(n)
    assert hl == 1 << nodemix.hist_bits(n)
    hi = torch.full((hl,), 7, dtype=torch.int32, device="cuda")  # garbage: all must be written
    ho = torch.full((hl,), 7, dtype=torch.int32, device="cuda")
    loops = t.chain2_local_hists("source", "target", base, n, hi.data_ptr(), ho.data_ptr())
    src, dst = cmodel.rmat(scale)
    ok = (src >= base) & (dst >= base)
    s, d = src[ok] - base, dst[ok] - base
    k = nodemix.hist_bits(n)
    ein = np.bincount(nodemix.node_mix(d, k), minlength=hl)
    eout = np.bincount(nodemix.node_mix(s, k), minlength=hl)
    assert np.array_equal(hi.cpu().numpy().astype(np.int64), ein)
    assert np.array_equal(ho.cpu().numpy().astype(np.int64), eout)
    assert loops == int((s == d).sum())


@pytest.mark.parametrize("n", [1 << 17, 100000], ids=["in_range", "checked"])
@pytest.mark.parametrize("compact", [False, True, 3], ids=["int64", "for32", "for24"])
def test_two_hop_hub_overflow(gpu_session, monkeypatch, n, compact):
    """Hubs with in/out degree far above 2^16 in one P3 unit: the packed
    uint16 LDS counters hand off 2^15 per overflow (k_c3_overflow) and the
    hub runs are split into atomically flushed units; the count stays exact."""
    from capf_amd.graph import ElementTable, ScanGraph as SG
    from capf_amd.expr import T_INT
    monkeypatch.setenv("CAPF_CHAIN2", "partitioned")
    rng = np.random.default_rng(11)
    m = 1 << 20
    src = rng.integers(0, 1 << 17, m)  # ids ≥ n (checked case) fall outside the node table
    dst = rng.integers(0, 1 << 17, m)
    src[: 300000] = 5            # out-hub
    dst[100000: 400000] = 9      # in-hub
    dst[500000: 600000] = 70000  # second in-hub in another bucket
    src[590000: 700000] = 70000
    dst[650000: 660000] = src[650000: 660000]  # self-loops
    rels = gpu_session.table([("id", T_INT, np.arange(m), None), ("source", T_INT, src, None),
                              ("target", T_INT, dst, None)])
    nodes = gpu_session.range_nodes(0, n, id_col="id")
    if compact:
        rels, nodes = rels.compact(), nodes.compact()
    g = SG(gpu_session, [ElementTable("node", frozenset(["V"]), nodes, {})],
           [ElementTable("rel", frozenset(["E"]), rels, {})])
    got = run(g, TWO_HOP)[0]["count"]
    assert gpu_session.last_plan() == "fused_chain2"
    assert got == cmodel.count_2hop(src.astype(np.int64), dst.astype(np.int64), n)


@pytest.mark.parametrize("compact", [False, True, 3], ids=["int64", "for32", "for24"])
@pytest.mark.parametrize("scale,parts", [(10, 2), (16, 1), (16, 3), (18, 4), (18, 3), (20, 8)])
def test_sharded_two_hop_partials(gpu_session, compact, scale, parts):
    """Node-partitioned layout (dist.py): every part's in/out copies hold
    exactly the rels whose target/source it owns, each part's on-device
    partial Σ_{owned b} in·out − owned loops equals the oracle's, and the
    partials sum to the closed-form 2-hop count (what the all-reduce forms).
    A rank's P3: S static tile ranges per run into histogram slices + the dot
    (packed slices with their hand-off log when S ≥ 2)."""
    import torch
    from capf_amd.dist import node_partitioned_copies
    from capf_amd.table import chain2_sharded_count_async
    from oracle import nodemix
    m = 16 << scale
    n = 1 << scale
    t = gpu_session.rmat_rels(scale, cmodel.rmat_seed(scale), cmodel.thresholds(), 0, m)
    if not compact:
        t = t.select("id", "source", "target")
    src, dst = cmodel.rmat(scale)
    own_s = nodemix.owner(src, n, parts)
    own_d = nodemix.owner(dst, n, parts)
    total = 0
    for p in range(parts):
        in_copy, out_copy = node_partitioned_copies(t, n, parts, p, compact=compact)
        if not compact:  # keep the copies int64 (node_partitioned_copies compacts)
            in_copy = t.node_partition("target", 0, n, parts, p)
            out_copy = t.node_partition("source", 0, n, parts, p)
        assert in_copy.size == int((own_d == p).sum())
        assert out_copy.size == int((own_s == p).sum())
        assert sorted(out_copy.column_arrays("id")[0].tolist()) == np.nonzero(own_s == p)[0].tolist()
        nd = getattr(out_copy, "n_diag", -1)
        if nd >= 0:  # 2-D order: the rels whose target p owns too come first
            ids = out_copy.column_arrays("id")[0]
            assert nd == int(((own_s == p) & (own_d == p)).sum())
            assert (own_d[ids[:nd]] == p).all() and (own_d[ids[nd:]] != p).all()
        part = torch.full((1,), -1, dtype=torch.int64, device="cuda")
        chain2_sharded_count_async(gpu_session, in_copy, out_copy, 0, n, parts, p, part.data_ptr())
        gpu_session.sync()
        ein = np.bincount(dst[own_d == p], minlength=n).astype(np.int64)
        eout = np.bincount(src[own_s == p], minlength=n).astype(np.int64)
        loops = int(((src == dst) & (own_s == p)).sum())
        expect = int((ein * eout).sum()) - loops
        assert int(part.item()) == expect, (p, int(part.item()), expect)
        total += expect
    assert total == cmodel.count_2hop(src, dst, n)


def _triangle_query():
    return Query([Match([NodeP("a"), NodeP("b"), NodeP("c")],
                        [RelP("r1", "a", "b"), RelP("r2", "b", "c"), RelP("r3", "c", "a")])],
                 [Stage([("count", CountStar())])])


@pytest.mark.parametrize("compact", [False, True, 3], ids=["int64", "for32", "for24"])
@pytest.mark.parametrize("scale", [6, 8, 10, 12])
def test_triangle_count_rmat(gpu_session, scale, compact):
    """MATCH (a)-->(b)-->(c)-->(a) RETURN count(*) through the planner (Expand,
    Expand, ExpandInto + uniqueness) runs as the fused triangle kernel and
    equals the oracle's trace(A^3) count (pinned by brute force at s <= 10)."""
    g = rmat_graph(gpu_session, scale, compact=compact)
    got = run(g, _triangle_query())[0]["count"]
    assert gpu_session.last_plan() == "fused_triangle"
    src, dst = cmodel.rmat(scale)
    expect = cmodel.count_triangle_formula(src, dst, 1 << scale)
    if scale <= 10:
        assert expect == cmodel.count_triangle_brute(src, dst, 1 << scale)
    assert got == expect


def test_triangle_self_loops_multi_edges(gpu_session):
    """Hand-made edge cases: 4 self-loops at one node (3 distinct loops needed),
    loops beside 2-cycles, parallel edges both ways, a triangle with
    multiplicities, an isolated 2-cycle, ids outside the node table."""
    from capf_amd.graph import ElementTable, ScanGraph as SG
    from capf_amd.expr import T_INT
    e = [(0, 0)] * 4 + [(1, 1), (1, 2), (2, 1), (2, 1)] + [(3, 4), (3, 4), (4, 5), (5, 3), (5, 3),
                                                             (3, 5), (5, 4)] + [(6, 7), (7, 6)] + [(8, 99), (99, 8)]
    src = np.array([x for x, _ in e], dtype=np.int64)
    dst = np.array([y for _, y in e], dtype=np.int64)
    n = 10
    rels = gpu_session.table([("id", T_INT, np.arange(len(e)), None), ("source", T_INT, src, None),
                              ("target", T_INT, dst, None)])
    nodes = gpu_session.range_nodes(0, n, id_col="id")
    g = SG(gpu_session, [ElementTable("node", frozenset(["V"]), nodes, {})],
           [ElementTable("rel", frozenset(["E"]), rels, {})])
    got = run(g, _triangle_query())[0]["count"]
    assert gpu_session.last_plan() == "fused_triangle"
    ok = (src < n) & (dst < n)
    assert got == cmodel.count_triangle_brute(src[ok], dst[ok], n) == cmodel.count_triangle_formula(src, dst, n)


@pytest.mark.parametrize("n", [40, (1 << 24) + 40], ids=["packed", "unpacked"])
def test_triangle_heavy_multi_edges(gpu_session, n):
    """Pairs with 15+ parallel rels in either direction (the packed column
    word's multiplicity nibbles saturate and the count reads vals through the
    sorted copy's escape words), beside pairs of 1-14; checked against brute
    force and trace(A^3).  A node range past 2^24 takes the unpacked kernel."""
    from capf_amd.graph import ElementTable, ScanGraph as SG
    from capf_amd.expr import T_INT
    big = n > 1000
    rng = np.random.default_rng(5)
    k = 40
    e = []
    for _ in range(120):
        x, y = rng.integers(0, k, 2)
        e += [(int(x), int(y))] * int(rng.choice([1, 2, 3, 14, 15, 16, 23]))
    e += [(0, 1)] * 17 + [(1, 2)] * 15 + [(2, 0)] * 16 + [(1, 0)] * 19  # one heavy triangle both ways
    if big:  # a triangle through the top of the range
        e += [(n - 1, 3), (3, 7), (7, n - 1)] * 2
    src = np.array([x for x, _ in e], dtype=np.int64)
    dst = np.array([y for _, y in e], dtype=np.int64)
    rels = gpu_session.table([("id", T_INT, np.arange(len(e)), None), ("source", T_INT, src, None),
                              ("target", T_INT, dst, None)])
    nodes = gpu_session.range_nodes(0, n, id_col="id")
    g = SG(gpu_session, [ElementTable("node", frozenset(["V"]), nodes, {})],
           [ElementTable("rel", frozenset(["E"]), rels, {})])
    got = run(g, _triangle_query())[0]["count"]
    assert gpu_session.last_plan() == "fused_triangle"
    remap = {v: i for i, v in enumerate(sorted(set(src.tolist()) | set(dst.tolist())))}
    s2 = np.array([remap[v] for v in src.tolist()], dtype=np.int64)
    d2 = np.array([remap[v] for v in dst.tolist()], dtype=np.int64)
    want = cmodel.count_triangle_brute(s2, d2, len(remap))
    assert got == want == cmodel.count_triangle_formula(s2, d2, len(remap))


def test_triangle_top_id_escape_word(gpu_session):
    """Node id 2^24 − 1 in a pair saturated both ways: its packed column word
    would be 0xFFFFFFFF — the count kernels' end-of-batch marker — unless the
    pack step clears b when f saturates; with the pair in triangles both ways."""
    from capf_amd.graph import ElementTable, ScanGraph as SG
    from capf_amd.expr import T_INT
    T, U = (1 << 24) - 1, (1 << 24) - 2
    rng = np.random.default_rng(11)
    e = [(T, U)] * 17 + [(U, T)] * 16 + [(U, 5)] * 15 + [(5, T)] * 20 + [(T, 5)] * 3 + [(5, U)] * 2
    for _ in range(300):
        x, y = (int(v) for v in rng.integers(0, 60, 2))
        e += [(x, y)] * int(rng.choice([1, 2, 15, 16]))
        e += [(x, T), (U, y)]
    src = np.array([x for x, _ in e], dtype=np.int64)
    dst = np.array([y for _, y in e], dtype=np.int64)
    n = 1 << 24
    rels = gpu_session.table([("id", T_INT, np.arange(len(e)), None), ("source", T_INT, src, None),
                              ("target", T_INT, dst, None)])
    nodes = gpu_session.range_nodes(0, n, id_col="id")
    g = SG(gpu_session, [ElementTable("node", frozenset(["V"]), nodes, {})],
           [ElementTable("rel", frozenset(["E"]), rels, {})])
    got = run(g, _triangle_query())[0]["count"]
    assert gpu_session.last_plan() == "fused_triangle"
    assert got == cmodel.count_triangle_brute(src, dst, n)


@pytest.mark.parametrize("qtile", ["12", "14", "18", "26"])
@pytest.mark.parametrize("scale", [10, 13])
def test_triangle_qtiled(gpu_session, monkeypatch, qtile, scale):
    """Pass A over q-tiled work items (CAPF_TRI_QTILE = log2 words per tile;
    small tiles cut most rows into several items, some rows longer than the
    LDS copy) gives the trace(A^3) count, alone and as 3 parts."""
    import torch
    from capf_amd.table import triangle_count_part_async
    monkeypatch.setenv("CAPF_TRI_QTILE", qtile)
    g = rmat_graph(gpu_session, scale, compact=True)
    got = run(g, _triangle_query())[0]["count"]
    assert gpu_session.last_plan() == "fused_triangle"
    src, dst = cmodel.rmat(scale)
    want = cmodel.count_triangle_formula(src, dst, 1 << scale)
    assert got == want
    t = gpu_session.rmat_rels(scale, cmodel.rmat_seed(scale), cmodel.thresholds(), 0, 16 << scale)
    d = torch.zeros(3, dtype=torch.int64, device="cuda")
    for p in range(3):
        triangle_count_part_async(gpu_session, t, 0, 1 << scale, 3, p, d.data_ptr() + 8 * p)
    gpu_session.sync()
    assert int(d.sum().item()) == want


@pytest.mark.parametrize("parts", [1, 2, 3, 5])
def test_triangle_partials_sum(gpu_session, parts):
    """capf_triangle_count_part: the parts (row chunks dealt round-robin, loop
    terms in part 0) sum to the count — what the multi-GPU all-reduce forms."""
    import torch
    from capf_amd.table import triangle_count_part_async
    scale = 11
    t = gpu_session.rmat_rels(scale, cmodel.rmat_seed(scale), cmodel.thresholds(), 0, 16 << scale)
    d = torch.zeros(parts, dtype=torch.int64, device="cuda")
    for p in range(parts):
        triangle_count_part_async(gpu_session, t, 0, 1 << scale, parts, p, d.data_ptr() + 8 * p)
    gpu_session.sync()
    src, dst = cmodel.rmat(scale)
    assert int(d.sum().item()) == cmodel.count_triangle_formula(src, dst, 1 << scale)


def _collect_graph(n=3000, seed=11):
    """Nodes with an integer key (some NULL), a float and a string value
    (some NULL) — collect / collect DISTINCT inputs with repeats."""
    from capf_amd.graph import GraphData
    rng = np.random.default_rng(seed)
    g = GraphData()
    for i in range(n):
        props = {}
        if rng.random() > 0.1:
            props["key"] = int(rng.integers(0, 40))
        if rng.random() > 0.2:
            props["val"] = float(rng.integers(0, 25)) / 4.0
        if rng.random() > 0.3:
            props["s"] = "w%d" % rng.integers(0, 12)
        g.nodes.append((i, frozenset(["N"]), props))
    return g


@pytest.mark.parametrize("distinct", [False, True])
@pytest.mark.parametrize("what", ["val", "s", "key"])
def test_collect_grouped_sorted_limited(gpu_session, distinct, what):
    """collect over 40 groups (+ the NULL group), then ORDER BY key, SKIP and
    LIMIT: the list column is gathered twice (sort permutation, slice) —
    lists.hip gather_list — and must equal the oracle's lists as bags."""
    from capf_amd.expr import Collect
    P = lambda k: ElementProperty(Var("n", "NODE"), k)  # noqa: E731
    q = Query([Match([NodeP("n")])],
              [Stage([("key", P("key")), ("col", Collect(P(what), distinct=distinct)), ("c", CountStar())],
                     order_by=[("key", "desc")], skip=3, limit=30)])
    data = _collect_graph()
    got = run(ScanGraph.from_data(gpu_session, data, compact=True), q)
    want = run(ScanGraph.from_data(OracleSession(), data), q)
    assert len(got) == 30
    assert [bag([r]) for r in got] == [bag([r]) for r in want]
    if distinct:
        assert all(len(r["col"]) == len(set(r["col"])) for r in got)


def test_collect_list_ops_fail_loudly(gpu_session):
    """A list column can be projected, not keyed or compared: DISTINCT over it
    is NotImplementedException (as a MULTISET key is in Flink)."""
    from capf_amd.expr import Collect
    P = lambda k: ElementProperty(Var("n", "NODE"), k)  # noqa: E731
    q = Query([Match([NodeP("n")])], [Stage([("col", Collect(P("val")))], distinct=True)])
    with pytest.raises(_lib.NotImplementedException):
        run(ScanGraph.from_data(gpu_session, _collect_graph(200)), q)


def _stat_table(session, n, ng, seed, nulls, ints=False):
    """n rows in ng groups: values X / 2^20 with integer X near 2^39 (mean
    about 5e5, spread below 1: a naive one-pass variance loses ~12 digits),
    one group holding most rows, optional NULLs; returns (table, header,
    gid, X, valid)."""
    rng = np.random.default_rng(seed)
    gid = rng.integers(0, ng, n)
    gid[rng.random(n) < 0.3] = 0  # a huge group
    X = (1 << 39) + rng.integers(0, 1 << 20, n) * (1 + (gid % 5))
    if ints:
        X = rng.integers(-(1 << 40), 1 << 40, n)
    valid = rng.random(n) > 0.05 if nulls else np.ones(n, bool)
    vals = X.astype(np.float64) / 2.0 ** 20 if not ints else X
    t = session.table([("k", T_INT, gid, None), ("v", T_INT if ints else T_FLOAT, vals, valid.astype(np.uint8))])
    h = RecordHeader({Var("k"): "k", Var("v"): "v"})
    return t, h, gid, X, valid


def _isum(a):
    """Exact sum of an int64 array as a Python int (chunks far below 2^63)."""
    return sum(int(c.sum()) for c in np.array_split(a, len(a) // 500_000 + 1)) if len(a) else 0


def _exact_stdev_groups(gid, X, valid, ng, scale, samp):
    """Exact per-group standard deviation of X / scale with integer
    arithmetic: var = (n·ΣX² − (ΣX)²) / (n·(n − 1)) / scale², one rounding in
    a 60-digit Decimal square root."""
    from decimal import Decimal, localcontext
    s1 = np.zeros(ng, dtype=object)
    s2 = np.zeros(ng, dtype=object)
    cnt = np.bincount(gid[valid], minlength=ng)
    for g in range(ng):
        xs = X[(gid == g) & valid]
        hi, lo = xs >> 20, xs & ((1 << 20) - 1)  # exact squares from 20-bit halves
        s1[g] = _isum(xs)
        s2[g] = (_isum(hi * hi) << 40) + (_isum(2 * hi * lo) << 20) + _isum(lo * lo)
    out = []
    for g in range(ng):
        n = int(cnt[g])
        if n < (2 if samp else 1):
            out.append(None)
            continue
        num = n * s2[g] - s1[g] * s1[g]
        den = n * (n - 1 if samp else n) * scale * scale
        with localcontext() as ctx:
            ctx.prec = 60
            out.append(float((Decimal(num) / Decimal(den)).sqrt()))
    return out


@pytest.mark.parametrize("nulls", [False, True])
def test_stdev_exact_at_size(gpu_session, nulls):
    """Grouped stDev / stDevP over 1e7 rows against the exact value within
    the north star's 1e-12 (the reference's stddevSamp / stddevPop,
    FlinkSQLExprMapper.scala:223-224); bit-identical run to run."""
    from capf_amd.expr import StDev, StDevP
    n, ng = 10_000_000, 1009
    t, h, gid, X, valid = _stat_table(gpu_session, n, ng, 7, nulls)
    for samp in (True, False):
        agg = StDev(Var("v")) if samp else StDevP(Var("v"))
        out = t.group([Var("k")], {"s": agg}, header=h)
        keys, vals = out.column_values("k"), out.column_values("s")
        want = _exact_stdev_groups(gid, X, valid, ng, 1 << 20, samp)
        for k, v in zip(keys, vals):
            w = want[k]
            assert (v is None) == (w is None), (k, v, w)
            if w is not None:
                assert abs(v - w) <= 1e-12 * w, (k, v, w, abs(v - w) / w)
        again = t.group([Var("k")], {"s": agg}, header=h).column_values("s")
        assert again == vals
    # the global aggregate, and INTEGER values (exact integers, no scaling)
    g = t.group([], {"s": StDev(Var("v"))}, header=h).column_values("s")[0]
    w = _exact_stdev_groups(np.zeros(n, np.int64), X, valid, 1, 1 << 20, True)[0]
    assert abs(g - w) <= 1e-12 * w
    ti, hi_, gi, Xi, vi = _stat_table(gpu_session, 200_000, 17, 9, nulls, ints=True)
    got = ti.group([Var("k")], {"s": StDevP(Var("v"))}, header=hi_)
    assert got.capf_type("s") == T_FLOAT
    want = _exact_stdev_groups(gi, Xi, vi, 17, 1, False)
    for k, v in zip(got.column_values("k"), got.column_values("s")):
        assert abs(v - want[k]) <= 1e-12 * want[k]


@pytest.mark.parametrize("kind", ["PercentileCont", "PercentileDisc"])
@pytest.mark.parametrize("p", [0.0, 0.05, 0.5, 0.62, 1.0])
@pytest.mark.parametrize("ints", [False, True])
def test_percentiles_parity(gpu_session, kind, p, ints):
    """percentileCont / percentileDisc grouped over 3e5 rows (NULLs, ties,
    one huge group) bit-exact against the oracle's restatement of the Spark
    UDAFs (PercentileUdafs.scala:59-96), in every encoding of the values."""
    import capf_amd.expr as ex
    rng = np.random.default_rng(int(p * 100) + ints)
    n, ng = 300_000, 777
    gid = rng.integers(0, ng, n)
    gid[rng.random(n) < 0.4] = 3
    vals = rng.integers(-50, 50, n) if ints else np.round(rng.normal(0, 1e3, n), 3)
    valid = (rng.random(n) > 0.1).astype(np.uint8)
    cols = [("k", T_INT, gid, None), ("v", T_INT if ints else T_FLOAT, vals, valid)]
    h = RecordHeader({Var("k"): "k", Var("v"): "v"})
    agg = {"q": getattr(ex, kind)(Var("v"), ex.FloatLit(p))}
    gt = gpu_session.table(cols)
    ot = OracleSession().table([(c, t, [x if ok else None for x, ok in zip(v, valid)] if c == "v" else v.tolist(),
                                 None) for c, t, v, _ in cols])
    for table in ([gt, gt.compact(3)] if ints else [gt]):
        got = table.group([Var("k")], agg, header=h)
        want = ot.group([Var("k")], agg, header=h)
        assert got.capf_type("q") == want.capf_type("q")
        assert sorted(zip(got.column_values("k"), got.column_values("q"))) == \
            sorted(zip(want.column_values("k"), want.column_values("q")))


def test_unwind_on_gpu(gpu_session):
    """UNWIND (RelationalPlanner.scala:99-101): a literal list over a scan (NULL
    elements kept, INTEGER/FLOAT widened), a parameter list, an empty list, and
    a collected LIST column; against the oracle."""
    from capf_amd.expr import Collect, FloatLit, ListLit
    from capf_amd.planner import Unwind, plan_query, plan_stage, plan_unwind, records
    create = "CREATE ({v: 1, s: 'a'}), ({v: 2, s: 'b'}), ({v: 2})"
    P = lambda k: ElementProperty(Var("n", "NODE"), k)  # noqa: E731
    queries = [
        Query([Match([NodeP("n")]), Unwind(ListLit(IntegerLit(3), NullLit(), FloatLit(4.5)), "x")],
              [Stage([("x", Var("x")), ("v", P("v"))])]),
        Query([Unwind(ListLit(), "x"), Match([NodeP("n")])], [Stage([("x", Var("x"))])]),
        Query([Unwind(ListLit(StringLit("p"), StringLit("q")), "x"), Match([NodeP("n")])],
              [Stage([("x", Var("x")), ("c", CountStar())])]),
    ]
    for q in queries:
        got = run(ScanGraph.from_data(gpu_session, parse_create(create)), q, {})
        want = run(ScanGraph.from_data(OracleSession(), parse_create(create)), q, {})
        assert bag(got) == bag(want), (got, want)
    from capf_amd.expr import Param
    q = Query([Unwind(Param("xs"), "x")], [Stage([("x", Var("x"))])])
    got = run(ScanGraph.from_data(gpu_session, parse_create(create)), q, {"xs": [5, 6, 7]})
    assert sorted(r["x"] for r in got) == [5, 6, 7]
    for sess in (gpu_session, OracleSession()):
        g = ScanGraph.from_data(sess, parse_create(create))
        op = plan_query(g, Query([Match([NodeP("n")])], [Stage([("k", P("s")), ("xs", Collect(P("v")))])]))
        op = plan_stage(plan_unwind(op, Unwind(Var("xs"), "y")), Stage([("k", Var("k")), ("y", Var("y"))]))
        rows = records(op, ["k", "y"])
        assert sorted((r["k"] or "", r["y"]) for r in rows) == [("", 2), ("a", 1), ("b", 2)]


def test_unwind_and_list_type_read_off_the_plan(gpu_session):
    """capf_table_explode_list and the type-only capf_table_list_info
    take a LIST column's element type from the plan (collect's argument type, a
    list literal's widened type, labels() → STRING, passed through select /
    filter / join / union / sort) instead of running the child while the plan is
    built — no upstream kernel (the filter's) runs before the result is asked
    for — and the unwound rows match the oracle."""
    from capf_amd.expr import Collect, Explode, ListLit
    cols = [("k", T_INT, [1, 1, 2, 3, 3, 3], None), ("x", T_INT, [4, 5, 6, 7, 8, 9], None),
            ("f", T_FLOAT, [0.5, 1.5, 2.5, 3.5, 4.5, 5.5], None)]
    h = RecordHeader({Var(c): c for c in ["k", "x", "f", "xs", "ys", "e", "l"]})

    def plans(sess):
        t = sess.table(cols).filter(GreaterThan(Var("x"), IntegerLit(4)), h, {})
        g = t.group([Var("k")], {"xs": Collect(Var("x")), "ys": Collect(Var("f"))}, header=h)
        lit = t.withColumns((ListLit(Var("x"), Var("f")), "l"), header=h, params={})
        return {
            "collect": g.withColumns((Explode(Var("xs")), "e"), header=h, params={}),
            "collect_sorted_renamed": g.orderBy((Var("k"), "desc"), header=h, params={})
                                       .select(("ys", "xs"), ("k", "k"))
                                       .withColumns((Explode(Var("xs")), "e"), header=h, params={}),
            "union": g.select(("k", "k"), ("xs", "xs")).unionAll(g.select(("k", "k"), ("xs", "xs")))
                      .withColumns((Explode(Var("xs")), "e"), header=h, params={}),
            "list_literal": lit.withColumns((Explode(Var("l")), "e"), header=h, params={}),
        }, g, lit

    want, _, _ = plans(OracleSession())
    gpu_session.reset_profile()
    gpu_session.set_profiling(True)
    try:
        got, g, lit = plans(gpu_session)
        assert g.list_elem_type("xs") == T_INT and g.list_elem_type("ys") == T_FLOAT
        assert lit.list_elem_type("l") == T_FLOAT  # INTEGER and FLOAT elements widen
        ran = [k for k in gpu_session.profile() if k.startswith("filter")]
        assert not ran, f"the plan ran while it was being built: {ran}"
        for name, t in got.items():
            assert t.capf_type("e") == want[name].capf_type("e"), name
            # (k, element) pairs: the order inside a collected list is not part of the contract
            assert bag({"k": r["k"], "e": r["e"]} for r in t.rows) == \
                bag({"k": r["k"], "e": r["e"]} for r in want[name].rows), name
        assert any(k.startswith("filter") for k in gpu_session.profile())
    finally:
        gpu_session.set_profiling(False)


MATH = ["Round", "Abs", "Ceil", "Floor", "Sign", "Sqrt", "Log", "Log10", "Exp", "Sin", "Cos", "Tan", "Asin",
        "Acos", "Atan", "Degrees", "Radians", "Cot", "Haversin"]


@pytest.mark.parametrize("fn", MATH)
def test_math_functions_parity(gpu_session, fn):
    """FlinkSQLExprMapper.scala:199-221 on the GPU against the oracle: exact for
    round / abs / ceil / floor / sign / degrees / radians, within 1e-15
    relative (the device libm against numpy's) for the transcendental ones."""
    import capf_amd.expr as ex
    rng = np.random.default_rng(len(fn))
    n = 4096
    f = np.concatenate([rng.normal(0, 10, n - 12), [0.5, -0.5, 1.5, -2.5, 2.4999999999999996, 0.0, -0.0, 1e300,
                                                    -1e-300, np.inf, -np.inf, np.nan]])
    iv = rng.integers(-1000, 1000, n)
    valid = (rng.random(n) > 0.1).astype(np.uint8)
    cols = [("f", T_FLOAT, f, valid), ("i", T_INT, iv, valid)]
    h = RecordHeader({Var("f"): "f", Var("i"): "i"})
    ot = OracleSession().table([(c, t, [x if ok else None for x, ok in zip(v.tolist(), valid)], None)
                                for c, t, v, _ in cols])
    for src in ("f", "i"):
        e = getattr(ex, fn)(Var(src))
        got = gpu_session.table(cols).withColumns((e, "o"), header=h)
        want = ot.withColumns((e, "o"), header=h)
        assert got.capf_type("o") == want.capf_type("o"), (fn, src)
        gv, wv = got.column_values("o"), want.column_values("o")
        exact = fn in ("Round", "Abs", "Ceil", "Floor", "Sign", "Degrees", "Radians")
        for a, b in zip(gv, wv):
            if a is None or b is None or (isinstance(b, float) and (b != b or b in (np.inf, -np.inf))):
                assert (a is None) == (b is None) and (b is None or repr(a) == repr(b) or (a != a and b != b))
            elif exact:
                assert a == b and repr(a) == repr(b), (fn, src, a, b)
            else:
                # haversin = (1 - cos x) / 2 cancels near x = 0: a 1-ulp difference
                # of the two cos implementations is an absolute 1e-16 there
                scale = max(abs(a), abs(b), 1.0 if fn == "Haversin" else 0.0)
                assert abs(a - b) <= 1e-15 * scale + 1e-300, (fn, src, a, b)


def test_case_atan2_toboolean_parity(gpu_session):
    """CASE (FlinkSQLExprMapper.scala:242-260, numeric branches widened),
    atan2 (:207), toBoolean over strings (:185), e() / pi(), startNode(r)."""
    import capf_amd.expr as ex
    rng = np.random.default_rng(5)
    n = 2000
    x = rng.normal(0, 3, n)
    y = rng.integers(-5, 5, n)
    words = ["true", "FALSE", " True ", "yes", "", "false"]
    s = [words[i % len(words)] if i % 7 else None for i in range(n)]
    cols = [("x", T_FLOAT, x.tolist(), None), ("y", T_INT, y.tolist(), None), ("s", T_STRING, s, None)]
    h = RecordHeader({Var("x"): "x", Var("y"): "y", Var("s"): "s"})
    exprs = [
        ex.CaseExpr([(GreaterThan(Var("x"), FloatLit(1.0)), Var("y")), (LessThan(Var("y"), IntegerLit(0)), Var("x"))],
                    ex.NullLit("FLOAT")),
        ex.CaseExpr([(Equals(Var("y"), IntegerLit(2)), IntegerLit(20))], Var("y")),
        ex.CaseExpr([(IsNull(Var("s")), StringLit("none"))], Var("s")),
        ex.CaseExpr([(GreaterThan(Var("y"), IntegerLit(3)), IntegerLit(1))]),
        ex.Atan2(Var("x"), Var("y")),
        ex.ToBoolean(Var("s")),
        Add(Var("x"), ex.Pi), Multiply(ex.E, Var("y")),
        # a widened CASE (INTEGER and FLOAT branches) inside an enclosing
        # operator: the chosen INTEGER branch is already a FLOAT there (1 / 2 =
        # 0.5, not integer division) — ADVICE r5
        ex.Divide(ex.CaseExpr([(GreaterThan(Var("x"), FloatLit(1.0)), IntegerLit(1))], FloatLit(2.5)),
                  IntegerLit(2)),
        ex.Modulo(ex.CaseExpr([(LessThan(Var("y"), IntegerLit(0)), Var("y"))], Var("x")), IntegerLit(2)),
        ex.Divide(ex.CaseExpr([(GreaterThan(Var("y"), IntegerLit(0)), Var("y"))], FloatLit(0.5)), Var("y")),
    ]
    gt = gpu_session.table(cols)
    ot = OracleSession().table(cols)
    for e in exprs:
        got = gt.withColumns((e, "o"), header=h)
        want = ot.withColumns((e, "o"), header=h)
        assert got.capf_type("o") == want.capf_type("o"), e
        for a, b in zip(got.column_values("o"), want.column_values("o")):
            assert a == b or (isinstance(a, float) and abs(a - b) <= 1e-15 * abs(b)), (str(e), a, b)


@pytest.mark.parametrize("hot", ["sampled", "none", "owned", "foreign", "dup", "range"])
def test_sharded_heavy_hitter_hints(gpu_session, hot):
    """Heavy-hitter hints of the sharded 2-hop count (dist.heavy_hitters, a
    sampled plan hint): whatever ids are passed — the sampled hubs, none, other
    owned nodes, nodes another rank owns, duplicates, ids outside the node
    range — every partial equals the oracle's (self-loops at a hub included)."""
    import torch
    from capf_amd.dist import node_partitioned_copies
    from capf_amd.table import chain2_sharded_count_async
    from oracle import nodemix
    scale, parts = 18, 3
    m, n = 16 << scale, 1 << scale
    t = gpu_session.rmat_rels(scale, cmodel.rmat_seed(scale), cmodel.thresholds(), 0, m)
    src, dst = cmodel.rmat(scale)
    own_s, own_d = nodemix.owner(src, n, parts), nodemix.owner(dst, n, parts)
    deg = np.bincount(src, minlength=n) + np.bincount(dst, minlength=n)
    total = 0
    for p in range(parts):
        in_copy, out_copy = node_partitioned_copies(t, n, parts, p, compact=3)
        mine = np.nonzero(nodemix.owner(np.arange(n), n, parts) == p)[0]
        top = mine[np.argsort(-deg[mine])[:2]].tolist()
        other = np.nonzero(nodemix.owner(np.arange(n), n, parts) != p)[0][:2].tolist()
        out_copy.hot_ids = {"sampled": out_copy.hot_ids, "none": [], "owned": mine[5:7].tolist(),
                            "foreign": other, "dup": top[:1] * 2, "range": [-5, n + 3]}[hot]
        if hot == "sampled":  # a sampled hint: ids of nodes this rank owns
            assert set(out_copy.hot_ids) <= set(mine.tolist())
        part = torch.full((1,), -1, dtype=torch.int64, device="cuda")
        chain2_sharded_count_async(gpu_session, in_copy, out_copy, 0, n, parts, p, part.data_ptr())
        gpu_session.sync()
        ein = np.bincount(dst[own_d == p], minlength=n).astype(np.int64)
        eout = np.bincount(src[own_s == p], minlength=n).astype(np.int64)
        expect = int((ein * eout).sum()) - int(((src == dst) & (own_s == p)).sum())
        assert int(part.item()) == expect, (p, hot, out_copy.hot_ids)
        total += expect
    assert total == cmodel.count_2hop(src, dst, n)


@pytest.mark.usefixtures("encoding")
@pytest.mark.parametrize("case", ["ints", "ints_with_null", "strings", "param_ids", "short"])
def test_in_long_list_set_lookup(case):
    """x IN a long list (≥ 17 elements, FlinkSQLExprMapper.scala:114-118): one
    binary search per row in a sorted session literal set (CAPF_OP_IN_SET)
    instead of an OR of equalities per element; three-valued as the OR — a NULL
    x, or a miss when the list holds a NULL, is NULL.  Same rows as the oracle,
    a second query reuses the memoised program, and the program carries the
    set opcode exactly for the long lists."""
    from capf_amd.expr import In, ListLit, Param, OP_IN_SET, compile_program
    rng = np.random.default_rng(17)
    n = 4000
    ids = [int(x) if rng.random() > 0.05 else None for x in rng.integers(0, 3000, n)]
    words = [f"w{int(x)}" if rng.random() > 0.05 else None for x in rng.integers(0, 60, n)]
    cols = [("k", T_INT, ids, None), ("s", T_STRING, words, None), ("i", T_INT, list(range(n)), None)]
    g, o = _both(cols)
    h = RecordHeader({Var("k"): "k", Var("s"): "s", Var("i"): "i"})
    params = {}
    if case == "ints":
        pred = In(Var("k"), ListLit(*[IntegerLit(int(v)) for v in rng.integers(0, 3000, 40)]))
    elif case == "ints_with_null":
        pred = Not(In(Var("k"), ListLit(*([IntegerLit(int(v)) for v in rng.integers(0, 3000, 30)]
                                                    + [NullLit("INTEGER")]))))
    elif case == "strings":
        pred = In(Var("s"), ListLit(*[StringLit(f"w{int(v)}") for v in rng.integers(0, 80, 25)]))
    elif case == "param_ids":
        params = {"ids": [int(v) for v in rng.integers(0, 3000, 1000)]}
        pred = In(Var("k"), Param("ids"))
    else:  # below the threshold: the OR of equalities
        pred = In(Var("k"), ListLit(*[IntegerLit(int(v)) for v in rng.integers(0, 3000, 5)]))
    for _ in range(2):
        got = g.filter(pred, h, params).rows
        want = o.filter(pred, h, params).rows
        assert bag(got) == bag(want)
    prog = compile_program(pred, h, set(g.physicalColumns), params, g.session.intern, g.capf_type,
                           g.session.literal_set)
    assert (OP_IN_SET in prog[0]) == (case != "short")


def test_distinct_flag_on_every_aggregator(gpu_session):
    """capf_table_group_ex honours the DISTINCT flag of every aggregator (the
    okapi IR carries it on count / collect only, Expr.scala:1077, 1136; the
    C-ABI takes one per aggregation): sum / avg / min / max over the distinct
    (group, value) pairs."""
    from dataclasses import dataclass
    from capf_amd.expr import Avg, Max, Min, Sum, T_INT, Var
    from capf_amd.header import RecordHeader

    def distinct(cls):
        @dataclass(frozen=True)
        class D(cls):
            distinct = True
        return D

    k = [0, 0, 0, 1, 1, 1, 1, 2]
    v = [5, 5, 7, 1, 1, None, 3, 4]
    t = gpu_session.table([("k", T_INT, k, None), ("v", T_INT, v, None)])
    h = RecordHeader({Var("k"): "k", Var("v"): "v"})
    aggs = {"s": distinct(Sum)(Var("v")), "a": distinct(Avg)(Var("v")), "lo": distinct(Min)(Var("v")),
            "hi": distinct(Max)(Var("v"))}
    rows = sorted((r["k"], r["s"], r["a"], r["lo"], r["hi"]) for r in t.group([Var("k")], aggs, header=h, params={}).rows)
    assert rows == [(0, 12, 6.0, 5, 7), (1, 4, 2.0, 1, 3), (2, 4, 4.0, 4, 4)]
