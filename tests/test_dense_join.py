"""GPU parity of the direct-address join (csrc/dense_join.hip): the Expand
join shape node.id = start(r) / end(r) (RelationalPlanner.scala:130-165,
FlinkTable.join FlinkTable.scala:171-187) when one key column is a dense
unique id column.  Every case is checked against the numpy oracle and must
have run the dense path (its probe kernel shows up in the profile), with ids
in order (no slot table) and shuffled (slot table), keys that miss, NULL
keys, every join type (build-side outer / FULL OUTER fall back), both sides
as the dense one, and FOR32 / FOR24 encodings."""
import numpy as np
import pytest

from conftest import bag

from capf_amd.expr import T_INT, T_STRING
from capf_amd.planner import Match, NodeP, Query, RelP, Stage, plan_query
from capf_amd.synthetic import rmat_graph
from capf_amd.expr import Var
from oracle.table_np import OracleSession

pytestmark = pytest.mark.gpu


def _tables(n_nodes, n_rels, order, misses, nulls, seed):
    rng = np.random.default_rng(seed)
    base = 1000
    ids = np.arange(base, base + n_nodes, dtype=np.int64)
    if order == "shuffled":
        ids = rng.permutation(ids)
    lo, hi = (base - 5, base + n_nodes + 5) if misses else (base, base + n_nodes)
    src = rng.integers(lo, hi, n_rels).astype(np.int64)
    sv = None
    if nulls:
        sv = np.ones(n_rels, dtype=np.uint8)
        sv[::13] = 0
    nodes = [("id", T_INT, ids, None), ("name", T_STRING, [f"n{int(i) % 7}" for i in ids], None)]
    rels = [("rid", T_INT, np.arange(n_rels, dtype=np.int64), None), ("src", T_INT, src, sv)]
    return nodes, rels


@pytest.mark.parametrize("jt", ["inner", "left_outer", "right_outer", "full_outer"])
@pytest.mark.parametrize("dense_left", [True, False], ids=["nodes_left", "nodes_right"])
@pytest.mark.parametrize("order", ["ordered", "shuffled"])
@pytest.mark.parametrize("misses,nulls", [(False, False), (True, False), (True, True)],
                         ids=["all_match", "misses", "misses_nulls"])
@pytest.mark.parametrize("compact", [False, 4, 3], ids=["int64", "for32", "for24"])
def test_dense_join_parity(gpu_session, jt, dense_left, order, misses, nulls, compact):
    nodes, rels = _tables(3000, 20000, order, misses, nulls, seed=len(jt) * 7 + int(dense_left))
    gn, gr = gpu_session.table(nodes), gpu_session.table(rels)
    if compact:
        gn, gr = gn.compact(compact), gr.compact(compact)
    on, orl = OracleSession().table(nodes), OracleSession().table(rels)
    gpu_session.reset_profile()
    gpu_session.set_profiling(True)
    if dense_left:
        got = gn.join(gr, jt, ("id", "src")).rows
        want = on.join(orl, jt, ("id", "src")).rows
    else:
        got = gr.join(gn, jt, ("src", "id")).rows
        want = orl.join(on, jt, ("src", "id")).rows
    gpu_session.set_profiling(False)
    assert bag(got) == bag(want)
    # the dense path runs unless the dense side must keep its unmatched rows
    dense_is_outer = jt == "full_outer" or (jt == "left_outer" and dense_left) or \
        (jt == "right_outer" and not dense_left)
    assert ("dense_probe" in gpu_session.profile()) == (not dense_is_outer)


def test_dense_join_key_alias_and_forced_paths(gpu_session, monkeypatch):
    """Inner dense join: the build key column of the output is the probe key
    column (same values on every row); CAPF_JOIN=radix/hash give the same bag."""
    nodes, rels = _tables(5000, 40000, "shuffled", True, True, seed=3)
    gn, gr = gpu_session.table(nodes), gpu_session.table(rels)
    out = gr.join(gn, "inner", ("src", "id"))
    a, _ = out.column_arrays("src")
    b, _ = out.column_arrays("id")
    assert np.array_equal(a, b)
    dense = bag(out.rows)
    for mode in ("radix", "hash"):
        monkeypatch.setenv("CAPF_JOIN", mode)
        assert bag(gr.join(gn, "inner", ("src", "id")).rows) == dense


@pytest.mark.parametrize("compact", [True, 3], ids=["for32", "for24"])
def test_one_hop_rows_rmat(gpu_session, compact):
    """MATCH (a)-->(b) RETURN a, b on R-MAT s12: one row per rel, (a, b) =
    (source, target) of that rel — the two Expand joins run dense."""
    from oracle import cmodel
    g = rmat_graph(gpu_session, 12, compact=compact)
    q = Query([Match([NodeP("a"), NodeP("b")], [RelP("r", "a", "b")])],
              [Stage([("a", Var("a", "NODE")), ("b", Var("b", "NODE"))])])
    gpu_session.reset_profile()
    gpu_session.set_profiling(True)
    t = plan_query(g, q).table
    cols = t.physicalColumns
    cols = cols() if callable(cols) else cols
    ka = next(c for c in cols if c.lstrip("_") == "a")
    kb = next(c for c in cols if c.lstrip("_") == "b")
    a, _ = t.column_arrays(ka)
    b, _ = t.column_arrays(kb)
    gpu_session.set_profiling(False)
    src, dst = cmodel.rmat(12)
    assert sorted(zip(a.tolist(), b.tolist())) == sorted(zip(src.tolist(), dst.tolist()))
    # both node scans hold only their id (the join key): every rel endpoint lies
    # in the dense id range (cached statistics), so no build row index is ever
    # read and neither dense probe runs — the rel rows pass through
    assert "dense_probe" not in gpu_session.profile()


@pytest.mark.parametrize("misses", [False, True], ids=["all_match", "misses"])
def test_dense_join_unread_build_side(gpu_session, misses):
    """Inner dense join whose build side is its key plus a constant (label)
    column: when every probe key provably matches (probe statistics inside the
    dense id range) the probe is skipped — the key column is the probe key, the
    label a fill; with keys that miss, the probe runs.  Same bag as the oracle
    either way."""
    from capf_amd.expr import BoolLit
    from capf_amd.header import RecordHeader
    nodes, rels = _tables(4000, 30000, "shuffled", misses, False, seed=11)
    nodes = nodes[:1]  # the id column only
    gn = gpu_session.table(nodes).compact(4)
    gn = gn.withColumns((BoolLit(True), "n:Person"), header=RecordHeader({}), params={})
    gr = gpu_session.table(rels).compact(4)
    on = OracleSession().table(nodes).withColumns((BoolLit(True), "n:Person"), header=RecordHeader({}),
                                                  params={})
    orl = OracleSession().table(rels)
    gpu_session.reset_profile()
    gpu_session.set_profiling(True)
    got = gr.join(gn, "inner", ("src", "id")).rows
    gpu_session.set_profiling(False)
    assert bag(got) == bag(orl.join(on, "inner", ("src", "id")).rows)
    assert ("dense_probe" in gpu_session.profile()) == misses


def _sparse_tables(n_nodes, n_rels, misses, nulls, dups, seed):
    """Node ids spread over a sparse domain (v·1000003 − 2^40, negative ones
    included: no dense range), shuffled; rel keys drawn from those ids (plus
    absent ids when `misses`); `dups` repeats a node id (no unique index)."""
    rng = np.random.default_rng(seed)
    ids = rng.permutation(np.arange(n_nodes, dtype=np.int64) * 1000003 - (1 << 40))
    if dups:
        ids[7] = ids[8]
    src = ids[rng.integers(0, n_nodes, n_rels)]
    if misses:
        src[::11] += 1  # not a node id
    sv = None
    if nulls:
        sv = np.ones(n_rels, dtype=np.uint8)
        sv[::13] = 0
    nodes = [("id", T_INT, ids, None), ("name", T_STRING, [f"n{int(i) % 7}" for i in ids], None)]
    rels = [("rid", T_INT, np.arange(n_rels, dtype=np.int64), None), ("src", T_INT, src, sv)]
    return nodes, rels


@pytest.mark.parametrize("jt", ["inner", "left_outer", "right_outer", "full_outer"])
@pytest.mark.parametrize("index_left", [True, False], ids=["nodes_left", "nodes_right"])
@pytest.mark.parametrize("misses,nulls", [(False, False), (True, True)], ids=["all_match", "misses_nulls"])
@pytest.mark.parametrize("dups", [False, True], ids=["unique", "dup_key"])
def test_hashed_index_join_parity(gpu_session, jt, index_left, misses, nulls, dups):
    """Unique sparse node ids: the hashed unique-key index (one 16-B slot load
    per probe) replaces the direct-address table; a repeated id disables it
    (the radix / hash joins run) — the same bag as the oracle either way."""
    nodes, rels = _sparse_tables(3000, 20000, misses, nulls, dups, seed=len(jt) * 5 + int(index_left))
    gn, gr = gpu_session.table(nodes), gpu_session.table(rels)
    on, orl = OracleSession().table(nodes), OracleSession().table(rels)
    gpu_session.reset_profile()
    gpu_session.set_profiling(True)
    if index_left:
        got = gn.join(gr, jt, ("id", "src")).rows
        want = on.join(orl, jt, ("id", "src")).rows
    else:
        got = gr.join(gn, jt, ("src", "id")).rows
        want = orl.join(on, jt, ("src", "id")).rows
    gpu_session.set_profiling(False)
    assert bag(got) == bag(want)
    index_is_outer = jt == "full_outer" or (jt == "left_outer" and index_left) or \
        (jt == "right_outer" and not index_left)
    assert ("hidx_probe" in gpu_session.profile()) == (not index_is_outer and not dups)
    assert "dense_probe" not in gpu_session.profile()


@pytest.mark.parametrize("misses,nulls", [(False, False), (True, False), (False, True)],
                         ids=["all_match", "misses", "nulls"])
@pytest.mark.parametrize("index_left", [True, False], ids=["nodes_left", "nodes_right"])
def test_hashed_index_key_only_build_side(gpu_session, misses, nulls, index_left):
    """Inner join on a sparse-id node table holding only its key: the matches
    are counted first (no build row written per probe row) and, when every
    probe key has its node, the probe rows pass through with the key as the
    node id; a missing key or a NULL falls back to the full probe.  Same bag as
    the oracle either way."""
    nodes, rels = _sparse_tables(3000, 20000, misses, nulls, False, seed=5 + int(misses) + 2 * int(nulls))
    nodes = nodes[:1]  # the id column only
    gn, gr = gpu_session.table(nodes), gpu_session.table(rels)
    on, orl = OracleSession().table(nodes), OracleSession().table(rels)
    if index_left:
        got, want = gn.join(gr, "inner", ("id", "src")).rows, on.join(orl, "inner", ("id", "src")).rows
    else:
        got, want = gr.join(gn, "inner", ("src", "id")).rows, orl.join(on, "inner", ("src", "id")).rows
    assert len(want) == 20000 or misses or nulls
    assert bag(got) == bag(want)


@pytest.mark.parametrize("compact", [False, True], ids=["int64", "for32"])
def test_one_hop_rows_rmat_sparse_ids(gpu_session, compact):
    """MATCH (a)-->(b) RETURN a, b on R-MAT s12 with node ids v·1000003 + 7:
    both Expand joins probe the hashed index; (a, b) = the rel's endpoints."""
    from oracle import cmodel
    stride = 1000003
    g = rmat_graph(gpu_session, 12, compact=compact, id_stride=stride)
    q = Query([Match([NodeP("a"), NodeP("b")], [RelP("r", "a", "b")])],
              [Stage([("a", Var("a", "NODE")), ("b", Var("b", "NODE"))])])
    gpu_session.reset_profile()
    gpu_session.set_profiling(True)
    t = plan_query(g, q).table
    cols = t.physicalColumns
    cols = cols() if callable(cols) else cols
    ka = next(c for c in cols if c.lstrip("_") == "a")
    kb = next(c for c in cols if c.lstrip("_") == "b")
    a, _ = t.column_arrays(ka)
    b, _ = t.column_arrays(kb)
    gpu_session.set_profiling(False)
    src, dst = cmodel.rmat(12)
    want = sorted(zip((src * stride + 7).tolist(), (dst * stride + 7).tolist()))
    assert sorted(zip(a.tolist(), b.tolist())) == want
    assert gpu_session.profile()["hidx_probe"]["launches"] == 2
