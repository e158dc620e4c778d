"""Config 5 (BASELINE.json): LDBC-SNB-shaped KNOWS var-length + DISTINCT + GROUP BY.

MATCH (a:Person)-[:KNOWS*1..3]->(b:Person)
WITH DISTINCT a, b
WITH a, count(*) AS reach
RETURN reach, count(*) AS n
"""
import json
import os

import capf_import  # noqa: F401
from capf_amd.expr import CountStar, Var
from capf_amd.graph import GraphData
from capf_amd.planner import Match, NodeP, Query, RelP, Stage

HERE = os.path.dirname(os.path.abspath(__file__))


def config5_query(upper=3):
    return Query([Match([NodeP("a", ("Person",)), NodeP("b", ("Person",))],
                        [RelP("k", "a", "b", ("KNOWS",), length=(1, upper))])],
                 [Stage([("a", Var("a")), ("b", Var("b"))], distinct=True),
                  Stage([("a", Var("a")), ("reach", CountStar())]),
                  Stage([("reach", Var("reach")), ("n", CountStar())])])


def ldbc_graph_data():
    with open(os.path.join(HERE, "ldbc_sample.json")) as f:
        d = json.load(f)
    nodes = [(p, frozenset(["Person"]), {}) for p in d["persons"]]
    rels = [(10 ** 15 + i, s, t, "KNOWS", {}) for i, (s, t) in enumerate(d["knows"])]
    return GraphData(nodes, rels)
