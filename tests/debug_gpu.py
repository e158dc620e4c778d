"""Ad-hoc GPU diagnostics (not collected by pytest)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import capf_import  # noqa
from capf_amd.table import GpuSession
from capf_amd.synthetic import rmat_graph
from capf_amd.planner import Match, NodeP, Query, RelP, Stage, run, plan_query
from capf_amd.expr import CountStar, Var
from oracle import cmodel

s = GpuSession(0)
for scale in (6, 8, 10, 12):
    g = rmat_graph(s, scale)
    rel = g.rel_tables[0].table
    src, _ = rel.column_arrays("source"); dst, _ = rel.column_arrays("target")
    cs, cd = cmodel.rmat(scale)
    print("scale", scale, "gen equal", np.array_equal(src, cs), np.array_equal(dst, cd))
    q = Query([Match([NodeP("a"), NodeP("b"), NodeP("c")], [RelP("r1", "a", "b"), RelP("r2", "b", "c")])],
              [Stage([("count", CountStar())])])
    got = run(g, q)[0]["count"]
    print("  fused", got, s.last_plan(), "closed", cmodel.count_2hop(cs, cd, 1 << scale))
    # materialised pieces
    from capf_amd import planner as P
    m = Match([NodeP("a"), NodeP("b"), NodeP("c")], [RelP("r1", "a", "b"), RelP("r2", "b", "c")])
    op = P.plan_match(g, m, None)
    print("  materialised size", op.table.size)
    qq = Query([m], [Stage([("a", Var("a")), ("b", Var("b")), ("c", Var("c")), ("r1", Var("r1")), ("r2", Var("r2"))])])
    op2 = plan_query(g, qq)
    cols = {k: np.array(op2.table.column_values(op2.header.column(Var(k)))) for k in ("a", "b", "c", "r1", "r2")}
    n = len(cols["a"])
    ok1 = np.array_equal(cs[cols["r1"]], cols["a"]) and np.array_equal(cd[cols["r1"]], cols["b"])
    ok2 = np.array_equal(cs[cols["r2"]], cols["b"]) and np.array_equal(cd[cols["r2"]], cols["c"])
    print("  rows", n, "consistent", ok1, ok2, "r1==r2 rows", int((cols["r1"] == cols["r2"]).sum()),
          "distinct (r1,r2)", len(set(zip(cols["r1"].tolist(), cols["r2"].tolist()))))
