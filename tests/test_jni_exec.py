"""The JNI adapter EXECUTED, not only type-checked.

integration/jni/capf_jni.cpp is built into tests/jni_fake/libcapf_jni_fake.so
against the stub jni.h with the in-process fake JVM (tests/jni_fake/
fake_jvm.cpp: JNI strings, arrays, fields, direct ByteBuffers, exceptions).
tests/jni_route.py then routes every C-ABI call of the unchanged planner →
GpuTable stack through the adapter's Native methods, so the queries below run
through the JNI marshalling — String[] / int[] / long[] / boolean[] arguments,
Program objects, direct buffers for uploads and downloads, out-arrays, and the
CapfNativeException → okapi-exception rethrow of Native.scala — and must match
the direct ctypes path row for row.

CPU tests: the library builds and exports one symbol per @native method; the
adapter's own argument checks (mismatched arrays, a heap buffer where a direct
one is needed) raise IllegalArgumentException before any device call; a C-ABI
error surfaces as the exception class of its kind.
GPU tests (-m gpu): config 1 (TeamDataFixture) and the 2-hop count, plus every
reference case, through the adapter against the ctypes path.
"""
import ctypes
import os
import re
import shutil
from ctypes import c_int64, c_void_p

import pytest

from conftest import bag, case_parts, check_case

from capf_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "integration", "scala", "org", "opencypher", "gpu", "Native.scala")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")


@pytest.fixture(scope="module")
def route():
    import jni_route
    jni_route.build()  # make: a no-op when up to date (the GPU box has g++ too)
    return jni_route.JniRoute()


def test_adapter_builds_and_exports_every_native_method(route):
    import jni_route
    scala = set(re.findall(r"@native def (\w+)\(", open(NATIVE).read()))
    for m in scala:
        assert hasattr(route.lib, jni_route.PREFIX + m), m
    assert len(scala) >= 80


def test_abi_and_error_accessors_through_jni(route):
    assert route.native("abiVersion", ctypes.c_int32) == _lib.load().capf_abi_version()


def test_group_with_mismatched_arrays_is_illegal_argument(route):
    """tableGroupEx checks its arrays against the aggregation count before any
    device call: two kinds, one name → IllegalArgumentException."""
    L, I = ctypes.c_int64, ctypes.c_int32
    kinds = (ctypes.c_int32 * 2)(0, 0)
    names = (ctypes.c_char_p * 1)(b"n")
    by = (ctypes.c_char_p * 1)()
    with pytest.raises(_lib.IllegalArgumentException, match="one entry per aggregation"):
        route.native("tableGroupEx", L, (L, 0), route.jstrs(by, 0), route.jints(kinds, 2),
                     route.lib.fj_objects(None, 0, b"org/opencypher/gpu/Program"),
                     route.jbools(kinds, 2), route.jdoubles((ctypes.c_double * 2)(), 2),
                     route.jstrs(names, 1))
    route.done()


def test_from_host_with_mismatched_arrays_is_illegal_argument(route):
    L = ctypes.c_int64
    names = (ctypes.c_char_p * 2)(b"a", b"b")
    types = (ctypes.c_int32 * 1)(1)
    with pytest.raises(_lib.IllegalArgumentException, match="one entry per column"):
        route.native("tableFromHost", L, (L, 0), route.jstrs(names, 2), route.jints(types, 1),
                     route.objects((c_void_p * 2)(), 2), None, (L, 0))
    route.done()


def test_session_copy_needs_a_direct_buffer(route):
    L, I = ctypes.c_int64, ctypes.c_int32
    with pytest.raises(_lib.IllegalArgumentException, match="direct buffer"):
        route.native("sessionCopy", None, (L, 0), (L, 0), route.lib.fj_heap_buffer(), (L, 8), (I, 2))
    buf = (ctypes.c_uint8 * 4)()
    with pytest.raises(_lib.IllegalArgumentException, match="direct buffer"):  # capacity 4 < 8 bytes
        route.native("sessionCopy", None, (L, 0), (L, 0), route.direct(ctypes.addressof(buf), 4), (L, 8), (I, 2))
    route.done()


def test_value_map_with_mismatched_arrays_is_illegal_argument(route):
    L = ctypes.c_int64
    k = (c_int64 * 3)(1, 2, 3)
    with pytest.raises(_lib.IllegalArgumentException, match="same length"):
        route.native("sessionValueMap", ctypes.c_int32, (L, 0), route.jlongs(k, 3), None, route.jlongs(k, 2))
    route.done()


def test_capf_error_rethrown_by_kind(route):
    """A failing C-ABI status becomes CapfNativeException(kind, message) in the
    adapter and the okapi exception of that kind above it (Native.scala):
    a NULL communicator is an IllegalArgumentException (kind -1)."""
    L = ctypes.c_int64
    with pytest.raises(_lib.IllegalArgumentException, match="null communicator"):
        route.native("commRank", ctypes.c_int32, (L, 0))
    route.done()


def test_all_to_all_needs_one_entry_per_rank(route):
    L = ctypes.c_int64
    k = (c_int64 * 1)(0)
    with pytest.raises(_lib.IllegalArgumentException, match="null communicator"):  # checked first
        route.native("commAllToAllBytes", None, (L, 0), (L, 0), route.jlongs(k, 1), (L, 0), route.jlongs(k, 1))
    route.done()


# ---------------------------------------------------------------- GPU
def _run_both(route, build_graph, query, params=None):
    """The query through the ctypes path, then through the JNI adapter."""
    from capf_amd.planner import run
    from capf_amd.table import GpuSession
    direct = run(build_graph(GpuSession(0)), query, params)
    before = route.jni_calls
    routed = route.install()
    try:
        via_jni = run(build_graph(GpuSession(0)), query, params)
    finally:
        route.uninstall()
    return direct, via_jni, route.jni_calls - before, routed


@pytest.mark.gpu
def test_config1_through_jni(route):
    """Config 1: MATCH (a:Person)-[:KNOWS]->(b) RETURN a.name, b.name over
    TeamDataFixture — every upload, join, projection and download through the
    adapter; identical rows to the ctypes path and to the reference's."""
    from reference_cases import CASES
    from capf_amd.graph import ScanGraph
    from oracle.create_parser import parse_create
    cid, src, create, query, expected, opts = case_parts(next(c for c in CASES if c[0] == "team_knows"))
    direct, via, calls, routed = _run_both(route, lambda s: ScanGraph.from_data(s, parse_create(create)), query)
    assert via == direct or bag(via) == bag(direct)
    assert bag(via) == bag(expected)
    assert calls > 20, calls
    assert "capf_table_join" in routed and "capf_table_download" in routed


@pytest.mark.gpu
@pytest.mark.parametrize("compact", [False, 3], ids=["int64", "for24"])
def test_two_hop_count_through_jni(route, compact):
    from capf_amd.expr import CountStar
    from capf_amd.planner import Match, NodeP, Query, RelP, Stage
    from capf_amd.synthetic import rmat_graph
    from oracle import cmodel
    q = Query([Match([NodeP("a"), NodeP("b"), NodeP("c")], [RelP("r1", "a", "b"), RelP("r2", "b", "c")])],
              [Stage([("count", CountStar())])])
    direct, via, calls, _ = _run_both(route, lambda s: rmat_graph(s, 14, compact=compact), q)
    src, dst = cmodel.rmat(14)
    assert via == direct == [{"count": cmodel.count_2hop(src, dst, 1 << 14)}]
    assert calls > 5


@pytest.mark.gpu
def test_reference_cases_through_jni(route):
    """Every transcribed reference case through the adapter: the same bag as
    the ctypes path (expressions as Program objects, group / order / explode /
    name lists, string dictionary round trips)."""
    from reference_cases import CASES
    from capf_amd.graph import ScanGraph
    from capf_amd.planner import run
    from capf_amd.table import GpuSession
    from oracle.create_parser import parse_create
    s_direct = GpuSession(0)
    bad = []
    for case in CASES:
        cid, src, create, query, expected, opts = case_parts(case)
        want = run(ScanGraph.from_data(s_direct, parse_create(create)), query, opts.get("params"))
        route.install()
        try:
            got = run(ScanGraph.from_data(GpuSession(0), parse_create(create)), query, opts.get("params"))
        finally:
            route.uninstall()
        same = check_case(got, expected, opts) if "rand" in opts else bag(got) == bag(want)
        if not same:  # (rand(): a fresh draw per evaluation — checked against its range)
            bad.append((cid, got, want))
    assert not bad, bad[:3]


@pytest.mark.gpu
def test_device_error_surfaces_as_mapped_exception(route):
    """An illegal argument detected inside the C-ABI (a join on a column the
    table lacks) crosses the adapter as CapfNativeException(kind -1) and
    reaches the caller as IllegalArgumentException — as through ctypes."""
    from capf_amd.expr import T_INT
    from capf_amd.table import GpuSession
    route.install()
    try:
        s = GpuSession(0)
        t = s.table([("x", T_INT, [1, 2, 3], None)])
        with pytest.raises(_lib.IllegalArgumentException, match="not found"):
            t.join(t.select(("x", "y")), "inner", ("nope", "y")).size
        assert t.column_values("x") == [1, 2, 3]  # the session stays usable
    finally:
        route.uninstall()


@pytest.mark.gpu
def test_random_programs_and_list_chains_through_jni(route):
    """Seeded expression trees (tests/test_expr_fuzz.py: projections, WHERE
    predicates, grouped aggregates) and LIST chains (tests/test_list_fuzz.py)
    through the adapter — Program objects of every opcode the generators emit,
    session code / value maps registered over JNI, LIST columns in and out —
    against the same calls over ctypes."""
    import test_expr_fuzz as ef
    import test_list_fuzz as lf
    from capf_amd.table import GpuSession
    s_direct = GpuSession(0)

    def run_all(s):
        out = [ef._eval(s, e) for e in ef.expressions(60, seed=31)]
        g = ef.Gen(5)
        out += [s.table(ef._table_cols()).filter(g.bool_(3), ef.H, {}).rows for _ in range(30)]
        out += [ef._group_rows(s, keys, aggs) for keys, aggs in ef.groups(20, seed=7)]
        out += [lf.rows(lf.chain(s, seed)) for seed in range(30)]
        return out

    want = run_all(s_direct)
    route.install()
    try:
        got = run_all(GpuSession(0))
    finally:
        route.uninstall()
    bad = [i for i, (x, y) in enumerate(zip(got, want)) if x != y and not (
        isinstance(x, list) and len(x) == len(y) and all(ef._same(a, b) or a == b for a, b in zip(x, y)))]
    assert len(got) == len(want) and not bad, bad[:5]
