"""CPU-only checks: the C-ABI library loads and exports every declared symbol,
the oracle's generators and closed forms agree with independent restatements,
and the planner's 2-hop plan on the numpy oracle reproduces the closed form."""
import ctypes
import os
import re

import numpy as np
import pytest

from capf_amd import _lib
from capf_amd.expr import CountStar
from capf_amd.graph import GraphData, ScanGraph
from capf_amd.planner import Match, NodeP, Query, RelP, Stage, run
from oracle import cmodel, rmat_np
from oracle.table_np import OracleSession

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "capf_gpu.h")).read()
    return sorted(set(re.findall(r"\b(capf_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert declared_symbols() == _lib.EXPORTED_SYMBOLS


def test_library_exports_every_symbol():
    assert os.path.exists(_lib.LIB_PATH), "libcapf_gpu.so not built (run __graft_entry__.build())"
    lib = ctypes.CDLL(_lib.LIB_PATH)  # loading must not need a GPU
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert _lib.load().capf_abi_version() == 1


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(ImportError):
        _lib.load(str(tmp_path / "nope.so"))


@pytest.mark.parametrize("scale", [4, 8, 11])
def test_rmat_c_matches_numpy(scale):
    s1, d1 = cmodel.rmat(scale, first=123, count=4000)
    s2, d2 = rmat_np.rmat(scale, cmodel.rmat_seed(scale), cmodel.thresholds(), 123, 4000)
    assert np.array_equal(s1, s2) and np.array_equal(d1, d2)


def test_rmat_degree_skew():
    # Graph500 parameters: the low-id quadrant dominates
    s, d = cmodel.rmat(12)
    assert (s < 1 << 11).mean() == pytest.approx(0.76, abs=0.02)
    assert (d < 1 << 11).mean() == pytest.approx(0.76, abs=0.02)


TWO_HOP = Query([Match([NodeP("a"), NodeP("b"), NodeP("c")], [RelP("r1", "a", "b"), RelP("r2", "b", "c")])],
                [Stage([("count", CountStar())])])


@pytest.mark.parametrize("scale", [5, 7])
def test_two_hop_three_ways(scale):
    """closed form == Flink-shaped pipeline == materialising planner on the oracle table."""
    src, dst = cmodel.rmat(scale, edge_factor=8)
    n = 1 << scale
    closed = cmodel.count_2hop(src, dst, n)
    pipe = cmodel.Pipeline(np.arange(n), np.arange(len(src)), src, dst, threads=2).probe(0, len(src), 2)
    gd = GraphData(nodes=[(i, frozenset(["V"]), {}) for i in range(n)],
                   rels=[(i, int(a), int(b), "E", {}) for i, (a, b) in enumerate(zip(src, dst))])
    planned = run(ScanGraph.from_data(OracleSession(), gd), TWO_HOP)[0]["count"]
    assert closed == pipe == planned


def test_one_hop_label_closed_form():
    scale = 8
    src, dst = cmodel.rmat(scale, edge_factor=4)
    n = 1 << scale
    person = cmodel.labels(n, 99)
    gd = GraphData(nodes=[(i, frozenset(["Person"] if person[i] else ["Other"]), {}) for i in range(n)],
                   rels=[(i, int(a), int(b), "E", {}) for i, (a, b) in enumerate(zip(src, dst))])
    q = Query([Match([NodeP("a", ("Person",)), NodeP("b")], [RelP("r", "a", "b")])], [Stage([("c", CountStar())])])
    assert run(ScanGraph.from_data(OracleSession(), gd), q)[0]["c"] == cmodel.count_1hop(src, dst, n, in_a=person)


@pytest.mark.parametrize("k", [15, 16, 20, 24])
def test_node_mix_is_a_bijection(k):
    from oracle import nodemix
    h = nodemix.node_mix(np.arange(1 << k), k)
    assert h.min() == 0 and h.max() == (1 << k) - 1
    assert len(np.unique(h)) == 1 << k


def test_node_mix_balances_rmat_runs():
    # the raw top bits of R-MAT ids are skewed (run 0 holds ~8 % of keys at 9
    # run bits); the mixed ones are near-uniform
    from oracle import nodemix
    s, d = cmodel.rmat(20, count=1 << 20)
    raw = np.bincount(d >> 15, minlength=32)
    mixed = np.bincount(nodemix.node_mix(d, 20) >> 15, minlength=32)
    assert raw.max() / raw.mean() > 4
    assert mixed.max() / mixed.mean() < 1.5


def test_bag_is_type_exact():
    """The test Bag follows typed CypherValue equality: an INTEGER result is
    not a FLOAT result (the avg-of-integers hazard, Expr.scala:1058-1066),
    large int64 ids do not collapse through float rounding, NULL is neither
    0 nor false, and the multiset counts duplicates."""
    from conftest import bag
    assert bag([{"a": 4}]) != bag([{"a": 4.0}])
    assert bag([{"a": 2 ** 60}]) != bag([{"a": 2 ** 60 + 1}])
    assert bag([{"a": None}]) != bag([{"a": 0}])
    assert bag([{"a": False}]) != bag([{"a": 0}])
    assert bag([{"a": 1}, {"a": 1}]) != bag([{"a": 1}])
    assert bag([{"a": 0.1 + 0.2}]) == bag([{"a": 0.3}])  # 1e-12 relative tolerance
    assert bag([{"a": float("nan")}]) == bag([{"a": float("nan")}])
    assert bag([{"a": [1, 2]}]) != bag([{"a": [1.0, 2.0]}])
    assert bag([{"a": 1, "b": "x"}, {"a": 2, "b": None}]) == bag([{"b": None, "a": 2}, {"b": "x", "a": 1}])
