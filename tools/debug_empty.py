"""Bisect a host crash on graphs without relationships (not a test)."""
import faulthandler
import os
import sys

faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
import torch  # noqa: E402,F401
import capf_import  # noqa: E402,F401
from capf_amd.expr import CountStar, Var  # noqa: E402
from capf_amd.graph import ScanGraph  # noqa: E402
from capf_amd.planner import Match, NodeP, Query, RelP, Stage, run  # noqa: E402
from capf_amd.table import GpuSession  # noqa: E402
from oracle.create_parser import parse_create  # noqa: E402

s = GpuSession(0)
g = ScanGraph.from_data(s, parse_create("CREATE (s {val: 1})"))
N = lambda v: Var(v, "NODE")  # noqa: E731
variants = [
    ("scan b NonExistent", Query([Match([NodeP("b", ("NonExistent",))])], [Stage([("b", N("b"))])])),
    ("count a-->b", Query([Match([NodeP("a"), NodeP("b")], [RelP("r", "a", "b")])], [Stage([("n", CountStar())])])),
    ("rows a-->b", Query([Match([NodeP("a"), NodeP("b")], [RelP("r", "a", "b")])], [Stage([("b", N("b"))])])),
    ("rows a-->b:NonExistent", Query([Match([NodeP("a"), NodeP("b", ("NonExistent",))], [RelP("r", "a", "b")])],
                                     [Stage([("b", N("b"))])])),
    ("one optional", Query([Match([NodeP("a")]), Match([NodeP("a"), NodeP("b", ("NonExistent",))],
                                                        [RelP("r1", "a", "b")], optional=True)],
                           [Stage([("b", N("b"))])])),
]
for name, q in variants:
    print("variant:", name, flush=True)
    print("  ->", run(g, q), flush=True)
print("all ok", flush=True)
