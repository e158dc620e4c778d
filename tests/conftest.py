import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
if GOLDEN not in sys.path:
    sys.path.insert(0, GOLDEN)

# torch first: it ships its own HIP runtime, which cannot enumerate the GPU
# once libcapf_gpu.so's runtime has initialised it in the same process
import torch  # noqa: E402,F401

import capf_import  # noqa: E402,F401


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: larger parity sizes")


def cypher_value_key(v):
    """A hashable, type-exact key of one CypherValue for Bag comparison.

    CypherValue equality (okapi-api .../api/value/CypherValue.scala) is typed:
    CypherInteger(4) != CypherFloat(4.0), so ints and floats stay distinct
    and ints compare exactly (no float rounding of ids above 2^53).  Floats
    are compared at 12 significant digits: the north-star tolerance for
    floating-point aggregates (1e-12 relative) absorbs summation order.
    NaN equals NaN here (one canonical key); NULL is its own kind.  Lists
    (collect) compare as bags: Flink's COLLECT is a MULTISET
    (FlinkSQLExprMapper.scala:283) and the reference tests compare collected
    lists with .toBag; nodes / relationships by identity, labels/type and
    properties."""
    if v is None:
        return ("null",)
    if isinstance(v, bool):
        return ("bool", v)
    if isinstance(v, int):
        return ("int", v)
    if isinstance(v, float):
        if v != v:
            return ("float", "nan")
        return ("float", float(f"{v:.12g}"))
    if isinstance(v, str):
        return ("str", v)
    if isinstance(v, (list, tuple)):
        return ("list", tuple(sorted((cypher_value_key(x) for x in v), key=repr)))
    if isinstance(v, dict):
        return ("map", tuple(sorted((k, cypher_value_key(x)) for k, x in v.items())))
    if isinstance(v, (frozenset, set)):
        return ("set", tuple(sorted(v)))
    from capf_amd.planner import CypherNode, CypherRelationship
    if isinstance(v, CypherNode):
        return ("node", v.id, tuple(sorted(v.labels)),
                tuple((k, cypher_value_key(x)) for k, x in sorted(v.properties)))
    if isinstance(v, CypherRelationship):
        return ("relationship", v.id, v.source, v.target, v.rel_type,
                tuple((k, cypher_value_key(x)) for k, x in sorted(v.properties)))
    try:
        import numpy as np
        if isinstance(v, np.integer):
            return ("int", int(v))
        if isinstance(v, np.floating):
            return cypher_value_key(float(v))
    except ImportError:
        pass
    raise TypeError(f"no Cypher value kind for {type(v).__name__}: {v!r}")


def check_case(got, expected, opts):
    """A reference case's assertion: Bag equality (OT/Bag.scala), or the
    ordered row list ({"ordered": True}), or only the row count."""
    if "row_count" in opts:
        return len(got) == opts["row_count"]
    if opts.get("ordered"):
        return [bag([r]) for r in got] == [bag([r]) for r in expected]
    return bag(got) == bag(expected)


def case_parts(case):
    cid, src, create, query, expected = case[:5]
    return cid, src, create, query, expected, (case[5] if len(case) > 5 else {})


def bag(rows):
    """okapi-testing Bag (OT/Bag.scala:29-51): multiset equality of records,
    each record a CypherMap compared with typed CypherValue equality."""
    return sorted(tuple(sorted((k, cypher_value_key(v)) for k, v in r.items())) for r in rows)


@pytest.fixture(scope="session")
def gpu_session():
    from capf_amd.table import GpuSession
    s = GpuSession(0)
    yield s
