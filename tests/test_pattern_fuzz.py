"""Randomised pattern parity: seeded small property graphs (labels, types,
NULL properties, self-loops, parallel rels) and seeded MATCH shapes — chains
of two or three hops with any mix of directions (Expand, RelationalPlanner
.scala:130-165, undirected as the UNION of both orientations), label / type
constraints (ScanGraph.scala:59-105), a bounded var-length rel
(VarLengthExpandPlanner.scala:82-259, lower bound 0 or 1), a closing rel
(ExpandInto :167-189), OPTIONAL MATCH (:222-246), a WHERE over properties and
a DISTINCT / grouped / row RETURN — planned by the same planner over the GPU
Table SPI and over the oracle's tables, compared as bags.  Every
materialising join kind, the uniqueness filters, unionAll, distinct, group
and the fused counts see random inputs.
"""
import random

import pytest

from capf_amd.expr import (Add, Ands, CountStar, ElementProperty, Equals, GreaterThan, Id, IntegerLit, IsNotNull,
                           LessThan, Not, Ors, StringLit, Var)
from capf_amd.graph import GraphData, ScanGraph
from capf_amd.planner import Match, NodeP, Query, RelP, Stage, run
from conftest import bag
from oracle.table_np import OracleSession

LABELS = [(), ("A",), ("B",), ("A", "B")]
NAMES = ["ann", "bob", "cy", "dee", None]


def graph(seed):
    r = random.Random(seed)
    nodes = []
    for i in range(r.randint(6, 24)):
        props = {}
        if r.random() < 0.8:
            props["val"] = r.randint(0, 5)
        nm = r.choice(NAMES)
        if nm is not None:
            props["name"] = nm
        nodes.append((i, frozenset(r.choice(LABELS)), props))
    n = len(nodes)
    rels = []
    for k in range(r.randint(0, 3 * n)):
        s = r.randrange(n)
        t = s if r.random() < 0.08 else r.randrange(n)
        props = {"w": r.randint(0, 3)} if r.random() < 0.7 else {}
        rels.append((n + k, s, t, r.choice(["R", "R", "S"]), props))
    return GraphData(nodes, rels)


def P(v, k):
    return ElementProperty(Var(v, "NODE"), k)


def query(seed):
    r = random.Random(seed)
    hops = r.randint(1, 3)
    vs = ["a", "b", "c", "d"][:hops + 1]
    nodes = [NodeP(v, r.choice([(), (), ("A",), ("B",)])) for v in vs]
    rels = []
    vl = r.randrange(hops) if r.random() < 0.3 else -1
    for i in range(hops):
        types = r.choice([(), ("R",), ("S",), ("R", "S")])
        direction = r.choice(["out", "out", "in", "both"])
        length = (r.choice([0, 1]), r.choice([1, 2])) if i == vl else None
        rels.append(RelP(f"r{i}", vs[i], vs[i + 1], types, direction, length))
    if hops >= 2 and vl < 0 and r.random() < 0.25:  # close a cycle: the ExpandInto rel
        rels.append(RelP("rc", vs[-1], vs[0], r.choice([(), ("R",)]), "out"))
    where = []
    if r.random() < 0.5:
        a, b = r.sample(vs, 2)
        where.append(r.choice([
            GreaterThan(P(a, "val"), IntegerLit(r.randint(0, 4))),
            Equals(P(a, "name"), StringLit(r.choice(NAMES[:-1]))),
            Ors(LessThan(P(a, "val"), P(b, "val")), Not(IsNotNull(P(b, "name")))),
            Ands(IsNotNull(P(a, "val")), Equals(Add(P(a, "val"), IntegerLit(1)), P(b, "val"))),
        ]))
    matches = [Match(nodes, rels, where)]
    if r.random() < 0.25:  # OPTIONAL MATCH from the last node
        o = "o"
        matches.append(Match([NodeP(vs[-1]), NodeP(o, r.choice([(), ("A",)]))],
                             [RelP("ro", vs[-1], o, r.choice([(), ("S",)]), r.choice(["out", "in"]))],
                             optional=True))
        vs = vs + [o]
    kind = r.randrange(4)
    if kind == 0:
        stages = [Stage([("n", CountStar())])]
    elif kind == 1:
        stages = [Stage([("k", P(vs[0], "val")), ("n", CountStar())])]
    elif kind == 2:
        stages = [Stage([(f"{v}.name", P(v, "name")) for v in r.sample(vs, min(2, len(vs)))], distinct=True)]
    else:
        stages = [Stage([(f"id_{v}", Id(Var(v, "NODE"))) for v in vs] +
                        [(f"{vs[-1]}.val", P(vs[-1], "val"))])]
    return Query(matches, stages)


CASES = [(s, s * 7919 + 11) for s in range(300)]


def test_pattern_generator_runs_on_oracle():
    for gs, qs in CASES[:40]:
        run(ScanGraph.from_data(OracleSession(), graph(gs)), query(qs))


@pytest.mark.gpu
@pytest.mark.parametrize("compact,join", [(False, None), (3, None), (True, "radix")],
                         ids=["int64", "for24", "for32-radix"])
def test_random_patterns_gpu_vs_oracle(gpu_session, monkeypatch, compact, join):
    """(for32-radix: every join through the radix-partitioned path, which the
    planner otherwise keeps for large inputs.)"""
    if join:
        monkeypatch.setenv("CAPF_JOIN", join)
    bad = []
    for gs, qs in CASES:
        g, q = graph(gs), query(qs)
        want = run(ScanGraph.from_data(OracleSession(), g), q)
        try:
            got = run(ScanGraph.from_data(gpu_session, g, compact=compact), q)
        except Exception as e:  # noqa: BLE001 - reported with the case
            bad.append((gs, qs, repr(e)[:200]))
            continue
        if bag(got) != bag(want):
            bad.append((gs, qs, len(got), len(want)))
    assert not bad, f"{len(bad)} of {len(CASES)} differ: {bad[:4]}"
