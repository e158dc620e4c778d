"""Randomised LIST parity: seeded chains of Table SPI calls that make LIST
columns and take them apart again — collect / collect(DISTINCT) under a
grouping (FlinkTable.scala:123-150), a list literal of per-row elements
(FlinkSQLExprMapper.scala:71), then select / rename, filter, orderBy, a
self-unionAll (:152-169) — followed by UNWIND (RelationalPlanner.scala:99-101,
capf_table_explode_list), size(xs) and xs[i] (:262-269), and a closing
aggregation.  The element type of the exploded column is read off the plan
(capf_table_explode_list / capf_table_list_info no longer evaluate the child
while the plan is built), so these chains check that derivation against the
oracle's independent restatement (oracle/table_np.py) on every shape.
Compared as bags of (key, value) rows: the order inside a collected list is
not part of the contract, so lists are only ever observed through UNWIND,
size() and sorted element sets.
"""
import random

import pytest

from capf_amd.expr import (Collect, ContainerIndex, CountStar, Explode, GreaterThan, IntegerLit, ListLit, Max, Min,
                           Size, Sum, Var, T_FLOAT, T_INT, T_STRING)
from capf_amd.header import RecordHeader
from conftest import bag
from oracle.table_np import OracleSession

N = 60
WORDS = ["ant", "bee", "cat", "dog", None]


def _cols(seed):
    r = random.Random(seed)
    return [("k", T_INT, [r.randint(0, 5) for _ in range(N)], None),
            ("x", T_INT, [r.choice([None, r.randint(-9, 9)]) if r.random() < 0.2 else r.randint(-9, 9)
                          for _ in range(N)], None),
            ("f", T_FLOAT, [round(r.uniform(-4, 4), 2) for _ in range(N)], None),
            ("s", T_STRING, [r.choice(WORDS) for _ in range(N)], None)]


H = RecordHeader({Var(c): c for c in ["k", "x", "f", "s", "xs", "l", "e", "n", "m", "z", "i0"]})


def chain(sess, seed):
    """One random chain; returns the final table (columns k and a value)."""
    r = random.Random(seed * 7919 + 3)
    t = sess.table(_cols(seed))
    if r.random() < 0.5:
        t = t.filter(GreaterThan(Var("f"), IntegerLit(r.randint(-3, 1))), H, {})
    src = r.choice(["x", "f", "s"])
    literal = r.random() >= 0.7
    if not literal:  # LIST from an aggregation
        t = t.group([Var("k")], {"xs": Collect(Var(src), r.random() < 0.4)}, header=H)
    else:  # LIST literal of per-row elements (no NULL elements: non-null operands)
        t = t.select(("k", "k"), ("f", "f")).withColumns((ListLit(Var("f"), Var("k"), IntegerLit(7)), "xs"),
                                                          header=H, params={})
    for _ in range(r.randint(0, 3)):  # plumbing the LIST column passes through
        op = r.randrange(4)
        if op == 0:
            t = t.select(("k", "k"), ("xs", "xs"))
        elif op == 1:
            t = t.orderBy((Var("k"), r.choice(["asc", "desc"])), header=H, params={})
        elif op == 2:
            t = t.filter(GreaterThan(Var("k"), IntegerLit(r.randint(-1, 3))), H, {})
        else:
            t = t.select(("k", "k"), ("xs", "xs"))
            t = t.unionAll(t)
    shape = r.randrange(3)
    if shape == 0:  # UNWIND, then an aggregation over the elements
        t = t.withColumns((Explode(Var("xs")), "e"), header=H, params={})
        agg = r.choice([CountStar(), Min(Var("e")), Max(Var("e"))] +
                       ([Sum(Var("e"))] if src == "x" and not literal else []))  # (exact: INTEGER sums)
        return t.group([Var("k")], {"z": agg}, header=H)
    if shape == 1:  # size(xs)
        return t.withColumns((Size(Var("xs")), "z"), header=H, params={}).select(("k", "k"), ("z", "z"))
    # xs[i] (an index past the end is NULL); observed only on list literals,
    # whose element order is defined
    t = t.withColumns((ContainerIndex(Var("xs"), IntegerLit(r.randint(0, 3))), "i0"), header=H, params={})
    return t.select(("k", "k"), ("i0", "z")) if literal else \
        t.withColumns((Size(Var("xs")), "z"), header=H, params={}).select(("k", "k"), ("z", "z"))


def rows(t):
    return bag({"k": x["k"], "z": x["z"]} for x in t.rows)


CASES = list(range(80))


def test_list_chains_run_on_oracle():
    for seed in CASES[:30]:
        assert rows(chain(OracleSession(), seed)) is not None


@pytest.mark.gpu
def test_list_chains_gpu_vs_oracle(gpu_session):
    bad = []
    for seed in CASES:
        want = rows(chain(OracleSession(), seed))
        try:
            got = rows(chain(gpu_session, seed))
        except Exception as e:  # noqa: BLE001 - reported with the case
            bad.append((seed, repr(e)[:200]))
            continue
        if got != want:
            bad.append((seed, "rows differ"))
    assert not bad, f"{len(bad)} of {len(CASES)} chains differ: {bad[:4]}"
