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
    keep their exact value here; Bag equality compares them with the
    north-star tolerance, |a − b| ≤ 1e-12 · max(|a|, |b|) (FLOAT_REL).
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
            return ("float", 1, 0.0)
        return ("float", 0, v)
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


def check_case(got, expected, opts, reference=True):
    """A reference case's assertion: Bag equality (OT/Bag.scala), or the
    ordered row list ({"ordered": True}), or only the row count.

    reference=True: against the reference test's expectation, typed (an
    INTEGER / FLOAT slip fails), except the cases marked {"coop": True}: the
    reference test's Bag of CypherMaps compares by Scala Map equality over the
    unwrapped values (okapi-api/.../value/CypherValue.scala:199-203, 301-302),
    where numeric values compare by value (CypherMap("res" -> 4) equals the 4.0
    that avg over INTEGER values is) — the only three cases whose expectation
    differs from the result in type (avg_ints*).  ({"typed": True} marks the
    cases whose reference test compares CypherValues directly.)
    reference=False (backend against oracle): typed, always."""
    if "row_count" in opts:
        return len(got) == opts["row_count"]
    if "rand" in opts:  # rand(): one FLOAT per row in [0, 1) (FunctionTests.scala:1422-1429)
        col = opts["rand"]
        return len(got) == len(expected) and all(
            isinstance(r[col], float) and 0.0 <= r[col] < 1.0 for r in got)
    coop = reference and bool(opts.get("coop")) and not opts.get("typed")
    if opts.get("ordered"):
        return [bag([r], coop) for r in got] == [bag([r], coop) for r in expected]
    return bag(got, coop) == bag(expected, coop)


def case_parts(case):
    cid, src, create, query, expected = case[:5]
    return cid, src, create, query, expected, (case[5] if len(case) > 5 else {})


FLOAT_REL = 1e-12  # north-star tolerance for floating-point results (relative)


def _close(a, b):
    """Typed key equality with floats within FLOAT_REL (relative)."""
    if isinstance(a, float) and isinstance(b, float):
        return a == b or abs(a - b) <= FLOAT_REL * max(abs(a), abs(b))
    if (isinstance(a, float) or isinstance(b, float)) and isinstance(a, (int, float)) \
            and isinstance(b, (int, float)) and not isinstance(a, bool) and not isinstance(b, bool):
        # coop keys: 4 == 4.0 (the kind tag was already compared); ints stay exact
        return a == b or abs(a - b) <= FLOAT_REL * max(abs(a), abs(b))
    if isinstance(a, tuple) and isinstance(b, tuple):
        return len(a) == len(b) and all(_close(x, y) for x, y in zip(a, b))
    return type(a) is type(b) and a == b


class Bag(list):
    """okapi-testing Bag (OT/Bag.scala:29-51): multiset equality of records,
    each record a CypherMap compared with typed CypherValue equality; floats
    match within FLOAT_REL.  Rows are compared in sorted order; when two
    near-equal floats sort differently on the two sides, rows are matched
    one by one instead."""

    def __eq__(self, other):
        if not isinstance(other, list) or len(self) != len(other):
            return False
        if all(_close(a, b) for a, b in zip(self, other)):
            return True
        if len(self) > 20000:
            return False
        left = list(other)
        for a in self:
            for i, b in enumerate(left):
                if _close(a, b):
                    del left[i]
                    break
            else:
                return False
        return True

    def __ne__(self, other):
        return not self.__eq__(other)

    __hash__ = None


def _coop(key):
    """A value key under Scala's numeric equality: INTEGER and FLOAT values
    share one kind ("num"), compared by value."""
    if isinstance(key, tuple) and key and key[0] == "int":
        return ("num", 0, key[1])
    if isinstance(key, tuple) and key and key[0] == "float":
        return ("num",) + key[1:]
    if isinstance(key, tuple):
        return tuple(_coop(x) for x in key)
    return key


def bag(rows, coop=False):
    """Test Bag of result rows: typed CypherValue equality, or with
    coop=True Scala's numeric Map equality (see check_case)."""
    keys = (tuple(sorted((k, cypher_value_key(v)) for k, v in r.items())) for r in rows)
    if coop:
        keys = (_coop(k) for k in keys)
    return Bag(sorted(keys))


@pytest.fixture(scope="session")
def gpu_session():
    from capf_amd.table import GpuSession
    s = GpuSession(0)
    yield s
