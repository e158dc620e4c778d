import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import capf_import  # noqa
from capf_amd.table import GpuSession
from capf_amd.synthetic import rmat_graph
from capf_amd import planner as P
from capf_amd.expr import Var, StartNode, EndNode, Not, Equals, CountStar
from oracle import cmodel

s = GpuSession(0)
scale = int(sys.argv[1]) if len(sys.argv) > 1 else 12
g = rmat_graph(s, scale)
cs, cd = cmodel.rmat(scale)
a, b, c, r1, r2 = (Var("a", "NODE"), Var("b", "NODE"), Var("c", "NODE"), Var("r1", "RELATIONSHIP"), Var("r2", "RELATIONSHIP"))
Sa, Sb, Sc = g.node_scan("a"), g.node_scan("b"), g.node_scan("c")
R1, R2 = g.rel_scan("r1"), g.rel_scan("r2")

def check(name, op, pairs):
    n = op.table.size
    cols = {}
    for e in set(x for p in pairs for x in p):
        v, ok = op.table.column_arrays(op.header.column(e))
        cols[e] = v
    bad = {f"{x}={y}": int((cols[x] != cols[y]).sum()) for x, y in pairs}
    print(name, "rows", n, "mismatch", bad, flush=True)
    return cols

J1 = P.join(Sa, R1, [(a, StartNode(r1))]); check("J1", J1, [(a, StartNode(r1))])
J2 = P.join(J1, Sb, [(EndNode(r1), b)]); check("J2", J2, [(a, StartNode(r1)), (EndNode(r1), b)])
J3 = P.join(J2, R2, [(b, StartNode(r2))]); cols = check("J3", J3, [(a, StartNode(r1)), (EndNode(r1), b), (b, StartNode(r2))])
ind = np.bincount(cd, minlength=1 << scale); outd = np.bincount(cs, minlength=1 << scale)
print("J3 expect", int((ind * outd).sum()))
rr1 = cols[StartNode(r1)]
J4 = P.join(J3, Sc, [(EndNode(r2), c)]); check("J4", J4, [(a, StartNode(r1)), (EndNode(r1), b), (b, StartNode(r2)), (EndNode(r2), c)])
F = P.filter_(J4, Not(Equals(r1, r2))); check("F", F, [(a, StartNode(r1)), (EndNode(r1), b), (b, StartNode(r2)), (EndNode(r2), c)])
print("closed", cmodel.count_2hop(cs, cd, 1 << scale))
