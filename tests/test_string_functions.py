"""String functions of the expression mapper (FlinkSQLExprMapper.scala:120-128
concatenation, :184 toString, :187-195 trim / lTrim / rTrim / toUpper /
toLower / replace / substring).

On the GPU a function of one STRING operand with literal arguments is a code
map of the session dictionary (CAPF_OP_STR_MAP: the function applied per
dictionary string on the host, the results interned, one table lookup per
row).  The oracle restates the JVM semantics independently
(oracle/table_np.py).  The Flink test suites hold no case for these functions,
so parity here is against the oracle's restatement only (parity unpinned by
reference fixtures).
"""
import numpy as np
import pytest

from capf_amd import _lib
from capf_amd.expr import (Add, BoolLit, Equals, FloatLit, GreaterThan, GreaterThanOrEqual, IntegerLit, LessThan,
                           LessThanOrEqual, LTrim, NullLit, Param, Replace, RTrim,
                           StringLit, Substring, ToLower, ToString, ToUpper, Trim, Var, T_BOOL, T_FLOAT, T_INT,
                           T_STRING, java_double_str, string_fn)
from capf_amd.header import RecordHeader
from oracle.table_np import OracleSession, _jstr

WORDS = ["alpha", "  Beta ", "GAMMA  ", " delta", "", "straße", "ÉCOLE", "a-b-a", "x\U0001F600yz", None]


def _cols(n=400, seed=5):
    rng = np.random.default_rng(seed)
    return [("s", T_STRING, [WORDS[i] for i in rng.integers(0, len(WORDS), n)], None),
            ("t", T_STRING, [WORDS[i] for i in rng.integers(0, len(WORDS), n)], None),
            ("k", T_INT, [int(x) if rng.random() > 0.1 else None for x in rng.integers(-50, 50, n)], None),
            ("b", T_BOOL, [bool(x) if rng.random() > 0.1 else None for x in rng.integers(0, 2, n)], None),
            ("f", T_FLOAT, [float(x) if rng.random() > 0.1 else None
                            for x in np.concatenate([rng.normal(0, 1e4, n - 8),
                                                     [0.0, -0.0, 1e7, 1e-4, 0.001, 1e21, 2.5, -7.0]])], None)]


H = RecordHeader({Var("s"): "s", Var("t"): "t", Var("k"): "k", Var("b"): "b", Var("f"): "f"})

EXPRS = [
    ToUpper(Var("s")), ToLower(Var("s")), Trim(Var("s")), LTrim(Var("s")), RTrim(Var("s")),
    Substring(Var("s"), IntegerLit(1), IntegerLit(3)), Substring(Var("s"), IntegerLit(0)),
    Substring(Var("s"), IntegerLit(2), IntegerLit(100)), Substring(Var("s"), IntegerLit(-3), IntegerLit(2)),
    Replace(Var("s"), StringLit("a"), StringLit("<>")), Replace(Var("s"), StringLit("[a-c]"), StringLit("")),
    Add(Var("s"), StringLit("!")), Add(StringLit(">"), Var("s")), Add(Var("s"), IntegerLit(7)),
    Add(FloatLit(1.5), Var("s")), Add(Var("s"), NullLit("STRING")),
    ToUpper(Trim(Var("s"))), Add(ToLower(Var("t")), StringLit("?")),
    ToString(Var("s")), ToString(Var("b")), ToString(IntegerLit(42)), ToString(FloatLit(1e7)),
    ToString(BoolLit(False)), ToUpper(StringLit("lit")), ToUpper(NullLit("STRING")),
    Add(StringLit("a"), IntegerLit(1)), ToUpper(Param("p")),
    # a new string per distinct value / value pair (value maps)
    ToString(Var("k")), ToString(Var("f")), Add(Var("s"), Var("t")), Add(Var("s"), Var("k")),
    Add(Var("f"), Var("s")), Add(ToUpper(Var("s")), ToString(Var("k"))),
]


def test_java_double_to_string_known_answers():
    """Double.toString as the JVM prints it (the cast of a FLOAT to STRING)."""
    known = [(1.0, "1.0"), (0.001, "0.001"), (1e-4, "1.0E-4"), (1e7, "1.0E7"), (9999999.0, "9999999.0"),
             (123456.789, "123456.789"), (12345678.9, "1.23456789E7"), (-0.5, "-0.5"), (1e21, "1.0E21"),
             (1.5e-10, "1.5E-10"), (0.0, "0.0"), (-0.0, "-0.0"), (float("inf"), "Infinity")]
    for d, want in known:
        assert java_double_str(d) == want
        assert _jstr(d, T_FLOAT) == want


def test_string_fn_semantics():
    """Calcite SUBSTRING (1-based, UTF-16 units, clipped), SQL TRIM of ' ' only,
    REGEXP_REPLACE, concatenation."""
    assert string_fn(("substring", 1, 3), "alpha") == "alp"
    assert string_fn(("substring", 3, 100), "alpha") == "pha"
    assert string_fn(("substring", 9, 2), "alpha") == ""
    assert string_fn(("substring", -2, 2), "alpha") == "ha"  # from the end (Calcite)
    assert string_fn(("substring", 2, 2), "x\U0001F600yz") == "\U0001F600"  # a surrogate pair is 2 units
    assert string_fn(("trim",), "\t a \t") == "\t a \t"  # only the space character
    assert string_fn(("trim",), "  a  ") == "a"
    assert string_fn(("replace", "[a-c]", ""), "abcd") == "d"
    assert string_fn(("concat_l", "x"), "y") == "xy"


@pytest.mark.parametrize("e", EXPRS, ids=[str(e) for e in EXPRS])
def test_oracle_string_functions_run(e):
    o = OracleSession().table(_cols())
    rows = o.withColumns((e, "x"), header=H, params={"p": "param"}).rows
    assert len(rows) == 400


@pytest.mark.gpu
@pytest.mark.parametrize("e", EXPRS, ids=[str(e) for e in EXPRS])
def test_string_functions_gpu_parity(gpu_session, e):
    """withColumns of each function: the GPU column equals the oracle's row by
    row (NULLs, unicode, empty strings, surrogate pairs)."""
    cols = _cols()
    g, o = gpu_session.table(cols), OracleSession().table(cols)
    rg = g.withColumns((e, "x"), header=H, params={"p": "param"}).rows
    ro = o.withColumns((e, "x"), header=H, params={"p": "param"}).rows
    assert [r["x"] for r in rg] == [r["x"] for r in ro]


@pytest.mark.gpu
def test_string_function_in_filter_and_memo(gpu_session):
    """A string function inside a WHERE, planned twice (the program memo reuses
    the code map) and again after new strings entered the dictionary (the map
    is extended)."""
    cols = _cols()
    pred = Equals(ToUpper(Trim(Var("s"))), StringLit("BETA"))
    o = OracleSession().table(cols)
    want = len(o.filter(pred, H, {}).rows)
    assert want > 0
    g = gpu_session.table(cols)
    assert len(g.filter(pred, H, {}).rows) == want
    assert len(g.filter(pred, H, {}).rows) == want
    more = [("s", T_STRING, ["  beta", "zeta", "BeTa  "], None), ("t", T_STRING, ["a", "b", "c"], None),
            ("k", T_INT, [1, 2, 3], None), ("b", T_BOOL, [True, False, True], None)]
    g2 = gpu_session.table(more)
    assert len(g2.filter(pred, H, {}).rows) == 2


@pytest.mark.gpu
@pytest.mark.parametrize("e", [Substring(Var("s"), Var("k")), Replace(Var("s"), StringLit("a"), StringLit("$1")),
                               Add(Var("s"), Var("b"))],
                         ids=["substring_column_start", "replace_group_ref", "concat_boolean"])
def test_string_shapes_not_on_gpu_raise(gpu_session, e):
    """Shapes outside the mapping (per-row function arguments, Java regex
    replacement groups, a BOOLEAN operand) raise instead of running elsewhere."""
    g = gpu_session.table(_cols())
    with pytest.raises(_lib.NotImplementedException):
        g.withColumns((e, "x"), header=H, params={}).rows


# labels(n) / keys(n) (FlinkSQLExprMapper.scala:136-153, GetLabels / GetKeys at
# :310-329): the planner's RETURN through withColumns → capf_table_name_list.
LK_CREATE = ("CREATE (:A:B {name: 'x', age: 3}), (:A {name: 'y'}), (:B {age: 7, flag: true}), (), "
             "(:C {name: null, age: 1})")


def _lk_query():
    from capf_amd.expr import Keys, Labels
    from capf_amd.planner import Match, NodeP, Query, Stage
    return Query([Match([NodeP("n")], [])],
                 [Stage([("l", Labels(Var("n", "NODE"))), ("k", Keys(Var("n", "NODE")))])])


def _canon(rows):
    return sorted((tuple(r["l"]), tuple(r["k"])) for r in rows)


def test_labels_keys_oracle():
    """Per node: its labels and the keys of its non-NULL properties, each sorted
    by name; never NULL (GetKeys itself lists only properties whose value is
    TRUE — a reference UDF bug not reproduced: keys(n) lists every property
    holding a value, Cypher's semantics)."""
    from capf_amd.graph import ScanGraph
    from capf_amd.planner import run
    from oracle.create_parser import parse_create
    og = ScanGraph.from_data(OracleSession(), parse_create(LK_CREATE))
    got = _canon(run(og, _lk_query()))
    assert got == sorted([(("A", "B"), ("age", "name")), (("A",), ("name",)), (("B",), ("age", "flag")),
                          ((), ()), (("C",), ("age",))])


@pytest.mark.gpu
@pytest.mark.parametrize("compact", [False, True], ids=["int64", "for32"])
def test_labels_keys_gpu(gpu_session, compact):
    from capf_amd.graph import ScanGraph
    from capf_amd.planner import run
    from oracle.create_parser import parse_create
    g = ScanGraph.from_data(gpu_session, parse_create(LK_CREATE), compact=compact)
    og = ScanGraph.from_data(OracleSession(), parse_create(LK_CREATE))
    assert _canon(run(g, _lk_query())) == _canon(run(og, _lk_query()))


@pytest.mark.gpu
def test_value_map_cap_raises(gpu_session, monkeypatch):
    """More distinct operand values than VALUE_MAP_MAX: NotImplementedException
    (no host string per value of a huge column)."""
    import capf_amd.table as tb
    monkeypatch.setattr(tb, "VALUE_MAP_MAX", 10)
    g = gpu_session.table(_cols())
    with pytest.raises(_lib.NotImplementedException):
        g.withColumns((ToString(Var("k")), "x"), header=H, params={}).rows


# ------------------------------------------------------- string ordering
# <, <=, >, >= on STRINGs (FlinkSQLExprMapper.scala:91-94, Flink compares
# VARCHARs as java.lang.String.compareTo: UTF-16 code units) and ORDER BY on a
# STRING key: on the GPU each string's rank in the session dictionary
# (CAPF_OP_STR_RANK, a device table rebuilt when the dictionary grows).  An
# INTEGER against a STRING orders to NULL (PredicateTests.scala:197-207).
ORD_WORDS = ["alpha", "Alpha", "", "b", "ab", "abc", "Z", "straße", "strasse", "x\U0001F600", "x�",
             "x", "é", "e", None]


def _ord_cols(n=300, seed=11):
    rng = np.random.default_rng(seed)
    return [("s", T_STRING, [ORD_WORDS[i] for i in rng.integers(0, len(ORD_WORDS), n)], None),
            ("t", T_STRING, [ORD_WORDS[i] for i in rng.integers(0, len(ORD_WORDS), n)], None),
            ("k", T_INT, [int(x) for x in rng.integers(0, 1000, n)], None)]


def test_java_string_compare_known_answers():
    from oracle.table_np import _jcmp
    assert _jcmp("a", "b") < 0 and _jcmp("B", "a") < 0 and _jcmp("", "a") < 0 and _jcmp("ab", "ab") == 0
    assert _jcmp("abc", "ab") > 0 and _jcmp("straße", "strasse") > 0
    # a supplementary character is a surrogate pair (D83D ..) and sorts below U+E000..U+FFFF
    assert _jcmp("x\U0001F600", "x") < 0 and _jcmp("x\U0001F600", "x�") < 0
    assert _jcmp("x\U0001F600", "xé") > 0


ORD_PREDS = [LessThan(Var("s"), Var("t")), LessThanOrEqual(Var("s"), StringLit("b")),
             GreaterThan(Var("s"), StringLit("x")), GreaterThanOrEqual(StringLit("alpha"), Var("t")),
             LessThan(ToUpper(Var("s")), Var("t")), LessThan(Var("s"), NullLit("STRING"))]


@pytest.mark.parametrize("e", ORD_PREDS + [LessThan(Var("s"), Var("k"))], ids=str)
def test_oracle_string_order_runs(e):
    rows = OracleSession().table(_ord_cols()).withColumns((e, "x"), header=OH, params={}).rows
    assert len(rows) == 300


OH = RecordHeader({Var("s"): "s", Var("t"): "t", Var("k"): "k"})


@pytest.mark.gpu
@pytest.mark.parametrize("e", ORD_PREDS + [LessThan(Var("s"), Var("k")), GreaterThanOrEqual(Var("k"), Var("t"))],
                         ids=str)
def test_string_order_predicates_gpu_parity(gpu_session, e):
    """Each comparison as a column (TRUE / FALSE / NULL per row) and as a
    filter: equal to the oracle's String.compareTo, row by row."""
    cols = _ord_cols()
    g, o = gpu_session.table(cols), OracleSession().table(cols)
    rg = g.withColumns((e, "x"), header=OH, params={}).rows
    ro = o.withColumns((e, "x"), header=OH, params={}).rows
    assert [r["x"] for r in rg] == [r["x"] for r in ro]
    assert g.filter(e, OH, {}).rows == o.filter(e, OH, {}).rows


@pytest.mark.gpu
@pytest.mark.parametrize("desc", [False, True], ids=["asc", "desc"])
def test_order_by_string_gpu_parity(gpu_session, desc):
    """ORDER BY s, k (and ORDER BY toUpper(t), k): the same row order as the
    oracle, NULLs where the ascending / descending sort puts them; again after
    new strings entered the dictionary (the rank table is rebuilt)."""
    cols = _ord_cols()
    d = "desc" if desc else "asc"
    for keys in ([(Var("s"), d), (Var("k"), "asc")], [(ToUpper(Var("t")), d), (Var("k"), "asc")]):
        g, o = gpu_session.table(cols), OracleSession().table(cols)
        assert g.orderBy(*keys, header=OH).rows == o.orderBy(*keys, header=OH).rows
    more = [("s", T_STRING, ["zz", "aa", "m", None, "abd"], None), ("t", T_STRING, ["q"] * 5, None),
            ("k", T_INT, [1, 2, 3, 4, 5], None)]
    g, o = gpu_session.table(more), OracleSession().table(more)
    keys = [(Var("s"), d)]
    assert g.orderBy(*keys, header=OH).rows == o.orderBy(*keys, header=OH).rows


@pytest.mark.gpu
def test_string_functions_over_distinct_values(gpu_session, monkeypatch):
    """Past CODE_MAP_MAX dictionary strings a string function maps the distinct
    values of its operand in the table (a value map) instead of the whole
    dictionary — a code map over a large dictionary interns a result per
    string and grows the dictionary the next map must cover.  Same rows as the
    oracle either way."""
    import capf_amd.table as tb
    monkeypatch.setattr(tb, "CODE_MAP_MAX", 0)
    cols = _cols()
    bad = []
    for e in EXPRS:
        g, o = gpu_session.table(cols), OracleSession().table(cols)
        rg = g.withColumns((e, "x"), header=H, params={"p": "param"}).rows
        ro = o.withColumns((e, "x"), header=H, params={"p": "param"}).rows
        if [r["x"] for r in rg] != [r["x"] for r in ro]:
            bad.append(str(e))
    assert not bad, bad


@pytest.mark.gpu
def test_code_map_grows_in_place():
    """a code map extended after the dictionary grew replaces its
    device table under the same id (capf_session_code_map_extend) rather than
    registering one more table per growth; a map two functions share (equal
    contents) stays as it is and the growing function gets a map of its own;
    a program planned before the growth evaluates right after it."""
    from capf_amd.table import GpuSession
    s = GpuSession(0)
    try:
        h = RecordHeader({Var("s"): "s"})
        up, tr = ToUpper(Var("s")), Trim(Var("s"))

        def col(t, e):
            return [r["x"] for r in t.withColumns((e, "x"), header=h, params={}).rows]

        t1 = s.table([("s", T_STRING, ["AB", "CD"], None)])
        assert col(t1, up) == ["AB", "CD"] and col(t1, tr) == ["AB", "CD"]
        before = {k: v[2] for k, v in s._maps.items()}
        assert before[("upper",)] == before[("trim",)]  # identity on this dictionary: one shared map
        early = t1.withColumns((up, "x"), header=h, params={})  # planned now, evaluated below
        t2 = s.table([("s", T_STRING, ["ef ", " G", None], None)])
        assert col(t2, up) == ["EF ", " G", None]
        grown = s._maps[("upper",)][2]
        assert grown != before[("upper",)]  # the shared map was not touched ...
        assert col(t2, tr) == ["ef", "G", None]  # ... and trim's grows in place (its only user now)
        assert s._maps[("trim",)][2] == before[("trim",)]
        t3 = s.table([("s", T_STRING, ["hi", "jk "], None)])
        assert col(t3, up) == ["HI", "JK "] and s._maps[("upper",)][2] == grown  # in place
        assert [r["x"] for r in early.rows] == ["AB", "CD"]
    finally:
        s.close()
