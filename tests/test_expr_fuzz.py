"""Randomised expression parity: seeded, well-typed expression trees over a
table with NULLs in every column type, evaluated as a projection
(withColumns) and as a predicate (filter) on the GPU interpreter and on the
oracle's independent restatement (oracle/table_np.py), row for row.

The generator covers the lowered operator set of FlinkSQLExprMapper.scala
:78-260 (comparisons, three-valued AND / OR / NOT, IS [NOT] NULL, IN lists,
+ - * / % with Java integer semantics, casts, CASE, coalesce, math functions,
string functions, string ordering), nested to depth 4, with INTEGER / FLOAT
operands mixed the way okapi types them.  Integer divisors are non-zero
literals (Flink's integer division by zero fails the job; that error path has
its own test).  FLOAT results compare within the north-star tolerance 1e-12
(relative), everything else exactly.
"""
import math
import random

import numpy as np
import pytest

from capf_amd.expr import (Abs, Add, Ands, BoolLit, CaseExpr, Ceil, Coalesce, Cos, Divide, Equals, Floor, FloatLit,
                           GreaterThan, GreaterThanOrEqual, In, IntegerLit, IsNotNull, IsNull, LessThan,
                           LessThanOrEqual, ListLit, Modulo, Multiply, Negate, Not, Ors, Round, Sign, Sin, Size,
                           Sqrt, StringLit, Substring, Subtract, ToFloat, ToInteger, ToLower, ToUpper, Trim, Var,
                           T_BOOL, T_FLOAT, T_INT, T_STRING)
from capf_amd.header import RecordHeader
from oracle.table_np import OracleSession

WORDS = ["alpha", "Beta", " gamma ", "", "delta", "ÉCOLE", "straße", "x\U0001F600", "Zeta", None]
N = 240
COLS = {"i": T_INT, "j": T_INT, "f": T_FLOAT, "g": T_FLOAT, "b": T_BOOL, "s": T_STRING, "t": T_STRING}
H = RecordHeader({Var(c): c for c in COLS})


def _table_cols(seed=17):
    rng = np.random.default_rng(seed)
    nul = lambda: rng.random() < 0.15  # noqa: E731
    return [("i", T_INT, [None if nul() else int(x) for x in rng.integers(-40, 40, N)], None),
            ("j", T_INT, [int(x) for x in rng.integers(-1000, 1000, N)], None),
            ("f", T_FLOAT, [None if nul() else float(x) for x in np.round(rng.normal(0, 20, N), 3)], None),
            ("g", T_FLOAT, [float(x) for x in rng.uniform(-5, 5, N)], None),
            ("b", T_BOOL, [None if nul() else bool(x) for x in rng.integers(0, 2, N)], None),
            ("s", T_STRING, [WORDS[k] for k in rng.integers(0, len(WORDS), N)], None),
            ("t", T_STRING, [WORDS[k] for k in rng.integers(0, len(WORDS) - 1, N)], None)]


class Gen:
    def __init__(self, seed):
        self.r = random.Random(seed)

    def pick(self, *xs):
        return self.r.choice(xs)

    def num(self, d):
        return self.int_(d) if self.r.random() < 0.5 else self.float_(d)

    def int_(self, d):
        r = self.r
        if d <= 0 or r.random() < 0.25:
            return self.pick(Var("i"), Var("j"), IntegerLit(r.randint(-9, 9)))
        k = r.randrange(10)
        if k == 0:
            return self.pick(Add, Subtract, Multiply)(self.int_(d - 1), self.int_(d - 1))
        if k == 1:
            return Divide(self.int_(d - 1), IntegerLit(self.pick(-7, -3, 2, 5, 11)))
        if k == 2:
            return Modulo(self.int_(d - 1), IntegerLit(self.pick(-4, 3, 7)))
        if k == 3:
            return self.pick(Abs, Sign, Negate, Ceil, Floor)(self.int_(d - 1))
        if k == 4:
            return CaseExpr([(self.bool_(d - 1), self.int_(d - 1))], self.pick(None, self.int_(d - 1)))
        if k == 5:
            return Coalesce(self.int_(d - 1), self.int_(d - 1))
        if k == 6:
            return Size(self.str_(d - 1))
        if k == 7:
            return ToInteger(Multiply(self.float_(d - 1), FloatLit(0.5)))
        return self.pick(Var("i"), Var("j"))

    def float_(self, d):
        r = self.r
        if d <= 0 or r.random() < 0.25:
            return self.pick(Var("f"), Var("g"), FloatLit(round(r.uniform(-3, 3), 2)))
        k = r.randrange(8)
        if k == 0:
            return self.pick(Add, Subtract, Multiply)(self.float_(d - 1), self.num(d - 1))
        if k == 1:
            return Divide(self.num(d - 1), self.float_(d - 1))
        if k == 2:
            return ToFloat(self.int_(d - 1))
        if k == 3:
            return self.pick(Round, Abs, Ceil, Floor, Sign, Negate)(self.float_(d - 1))
        if k == 4:
            return self.pick(Sin, Cos)(self.num(d - 1))
        if k == 5:
            return Sqrt(Abs(self.float_(d - 1)))
        if k == 6:
            return CaseExpr([(self.bool_(d - 1), self.float_(d - 1))], self.float_(d - 1))
        return Coalesce(self.float_(d - 1), self.float_(d - 1))

    def str_(self, d):
        r = self.r
        if d <= 0 or r.random() < 0.35:
            return self.pick(Var("s"), Var("t"), StringLit(self.pick("alpha", "Zeta", "x", "")))
        k = r.randrange(5)
        if k == 0:
            return self.pick(ToUpper, ToLower, Trim)(self.str_(d - 1))
        if k == 1:
            return Substring(self.str_(d - 1), IntegerLit(r.randint(0, 3)), IntegerLit(r.randint(0, 4)))
        if k == 2:
            return Add(self.str_(d - 1), StringLit(self.pick("!", "-x")))
        if k == 3:
            return CaseExpr([(self.bool_(d - 1), self.str_(d - 1))], self.str_(d - 1))
        return Coalesce(self.str_(d - 1), StringLit("none"))

    def bool_(self, d):
        r = self.r
        if d <= 0 or r.random() < 0.2:
            return self.pick(Var("b"), BoolLit(r.random() < 0.5))
        k = r.randrange(9)
        cmp = self.pick(Equals, LessThan, LessThanOrEqual, GreaterThan, GreaterThanOrEqual)
        if k == 0:
            return cmp(self.int_(d - 1), self.int_(d - 1))
        if k == 1:
            return cmp(self.num(d - 1), self.num(d - 1))
        if k == 2:
            return cmp(self.str_(d - 1), self.str_(d - 1))
        if k == 3:
            return self.pick(Ands, Ors)(self.bool_(d - 1), self.bool_(d - 1))
        if k == 4:
            return Not(self.bool_(d - 1))
        if k == 5:
            return self.pick(IsNull, IsNotNull)(self.pick(self.int_, self.float_, self.str_, self.bool_)(d - 1))
        if k == 6:
            return In(self.int_(d - 1), ListLit(*[IntegerLit(r.randint(-9, 9)) for _ in range(r.randint(0, 4))]))
        if k == 7:
            return CaseExpr([(self.bool_(d - 1), self.bool_(d - 1))], self.bool_(d - 1))
        return Equals(self.bool_(d - 1), self.bool_(d - 1))

    def any_(self, d):
        return self.pick(self.int_, self.float_, self.str_, self.bool_)(d)


def expressions(n=240, seed=2024):
    g = Gen(seed)
    return [g.any_(4) for _ in range(n)]


def _same(x, y):
    if x is None or y is None:
        return x is None and y is None
    if isinstance(x, float) or isinstance(y, float):
        if not (isinstance(x, float) and isinstance(y, float)):
            return False
        if math.isnan(x) or math.isnan(y):
            return math.isnan(x) and math.isnan(y)
        return x == y or abs(x - y) <= 1e-12 * max(abs(x), abs(y))
    return type(x) is type(y) and x == y


def _eval(session, e):
    t = session.table(_table_cols())
    return [r["x"] for r in t.withColumns((e, "x"), header=H, params={}).rows]


def test_generator_is_deterministic_and_oracle_evaluates():
    es = expressions(60)
    assert [str(e) for e in es] == [str(e) for e in expressions(60)]
    o = OracleSession()
    for e in es:
        assert len(_eval(o, e)) == N


@pytest.mark.gpu
def test_random_expressions_gpu_vs_oracle(gpu_session):
    bad = []
    for k, e in enumerate(expressions()):
        want = _eval(OracleSession(), e)
        got = _eval(gpu_session, e)
        rows = [r for r, (x, y) in enumerate(zip(got, want)) if not _same(x, y)]
        if rows or len(got) != len(want):
            bad.append((k, str(e), rows[:3], [got[r] for r in rows[:3]], [want[r] for r in rows[:3]]))
    assert not bad, f"{len(bad)} of 240 expressions differ: {bad[:4]}"


@pytest.mark.gpu
def test_random_predicates_gpu_vs_oracle(gpu_session):
    g = Gen(77)
    bad = []
    for k in range(120):
        p = g.bool_(4)
        want = OracleSession().table(_table_cols()).filter(p, H, {}).rows
        got = gpu_session.table(_table_cols()).filter(p, H, {}).rows
        if got != want:
            bad.append((k, str(p), len(got), len(want)))
    assert not bad, f"{len(bad)} of 120 predicates differ: {bad[:4]}"


# ------------------------------------------------- random grouped aggregates
def groups(n=60, seed=99):
    """(group key vars, {column: aggregator}) pairs over the fuzz table:
    count(*), count([DISTINCT] e), sum / min / max / avg of numeric
    expressions, min / max of strings, collect([DISTINCT] e) (FlinkTable.scala:123-150,
    FlinkSQLExprMapper.scala:281-287)."""
    from capf_amd.expr import Avg, Collect, Count, CountStar, Max, Min, Sum
    g = Gen(seed)
    out = []
    for _ in range(n):
        keys = g.r.sample([Var("i"), Var("s"), Var("b")], g.r.randint(0, 2))
        aggs = {}
        for k in range(g.r.randint(1, 3)):
            kind = g.r.randrange(7)
            if kind == 0:
                a = CountStar()
            elif kind == 1:
                a = Count(g.any_(2), g.r.random() < 0.4)
            elif kind == 2:
                a = g.pick(Sum, Min, Max)(g.int_(2))
            elif kind == 3:
                a = g.pick(Sum, Avg, Min, Max)(g.float_(2))
            elif kind == 4:
                a = Avg(g.int_(2))
            elif kind == 5:
                a = Collect(g.pick(g.int_, g.str_)(2), g.r.random() < 0.4)
            else:  # String.compareTo order (CAPF_OP_STR_RANK, ranks mapped back to codes)
                a = g.pick(Min, Max)(g.str_(2))
            aggs[f"a{k}"] = a
        out.append((keys, aggs))
    return out


def _norm(v):
    return sorted((repr(x) for x in v)) if isinstance(v, list) else v


def _group_rows(session, keys, aggs):
    t = session.table(_table_cols())
    rows = t.group(keys, aggs, header=H, params={}).rows
    names = [k.vname for k in keys] + list(aggs)
    return sorted((tuple(_norm(r[c]) for c in names) for r in rows), key=repr)


def test_group_generator_runs_on_oracle():
    for keys, aggs in groups(20):
        assert _group_rows(OracleSession(), keys, aggs) is not None


@pytest.mark.gpu
def test_random_groups_gpu_vs_oracle(gpu_session):
    bad = []
    for k, (keys, aggs) in enumerate(groups()):
        want = _group_rows(OracleSession(), keys, aggs)
        got = _group_rows(gpu_session, keys, aggs)
        ok = len(got) == len(want) and all(len(x) == len(y) and all(_same(a, b) or a == b for a, b in zip(x, y))
                                           for x, y in zip(got, want))
        if not ok:
            bad.append((k, [str(v) for v in keys], {c: str(a) for c, a in aggs.items()}, got[:2], want[:2]))
    assert not bad, f"{len(bad)} of 60 groupings differ: {bad[:3]}"
