"""The JVM drop-in (integration/scala) against the okapi API it
plugs into.  No scalac exists in this image, so the sources are checked
against the okapi names, case-class arities and inherited members recorded
from the reference's own Scala sources (tests/golden/okapi_api.json, built
by tests/golden/make_okapi_api.py):

  * every okapi name the sources import exists there;
  * every extractor pattern `case X(a, b)` on an okapi case class (or
    extractor object) uses its arity, and every bare `case X =>` names a case object (e.g. CountStar,
    Expr.scala:1071);
  * every `override` in a class extending okapi types names a member that
    one of its (transitive) parents declares;
  * GpuCypherSession extends RelationalCypherSession[GpuTable] and supplies
    its three factories (RelationalCypherSession.scala:101-105).
"""
import json
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import okapi_scala_scan as sc  # noqa: E402

FIXTURE = os.path.join(HERE, "golden", "okapi_api.json")
REFERENCE = "/root/reference"
# members every JVM class has, or that non-okapi parents (Function1,
# Runnable, AutoCloseable) declare
UNIVERSAL = {"toString", "equals", "hashCode", "apply", "run", "close"}


@pytest.fixture(scope="module")
def api():
    with open(FIXTURE) as f:
        return json.load(f)


def _okapi_names(srcs, api):
    explicit = {}
    for text in srcs.values():
        for prefix, name in sc.imports(text):
            if name != "_":
                explicit[name] = f"{prefix}.{name}"
    wild = {n: f"{p}.{n}" for p, names in api["wildcard_packages"].items() for n in names}
    return {**wild, **explicit}


def test_imports_resolve(api):
    missing = []
    for f, text in sc.integration_sources().items():
        for prefix, name in sc.imports(text):
            if name == "_":
                assert prefix in api["wildcard_packages"] and api["wildcard_packages"][prefix], (f, prefix)
            elif not api["names"].get(f"{prefix}.{name}"):
                missing.append((f, f"{prefix}.{name}"))
    assert not missing, f"imported names the okapi sources do not define: {missing}"


def test_extractor_arities(api):
    srcs = sc.integration_sources()
    okapi = _okapi_names(srcs, api)
    bad = []
    for f, text in srcs.items():
        calls, bare = sc.patterns(text)
        for name, n in calls:
            q = okapi.get(name)
            if q is None:
                continue
            defs = api["names"].get(q, [])
            if not any(k in ("case class", "object") and a == n for k, a in defs):
                bad.append((f, f"case {name}({n} args)", defs))
        for name in bare:
            q = okapi.get(name)
            if q is None:
                continue
            defs = api["names"].get(q, [])
            if not any(k in ("case object", "object", "val") for k, _ in defs):
                bad.append((f, f"case {name} =>", defs))
    assert not bad, bad


def test_overrides_exist_in_parents(api):
    srcs = sc.integration_sources()
    okapi = _okapi_names(srcs, api)
    local = {}
    for text in srcs.values():
        local.update(sc.classes(text))

    def members(parent, seen):
        if parent in seen:
            return set()
        seen.add(parent)
        out = set()
        if parent in api["members"]:
            out |= set(api["members"][parent]["members"])
            for q in api["members"][parent]["parents"]:
                out |= members(q, seen)
        elif parent in local:
            ps, over = local[parent]
            out |= set(over)
            for q in ps:
                out |= members(q, seen)
        return out

    bad = []
    checked = 0
    for f, text in srcs.items():
        for cls, (parents, over) in sc.classes(text).items():
            if not any(p in okapi or p in local for p in parents):
                continue
            avail = set(UNIVERSAL)
            for p in parents:
                avail |= members(p, set())
            for m in over:
                checked += 1
                if m not in avail:
                    bad.append((f, cls, m))
    assert checked >= 40, checked
    assert not bad, f"overrides of members no parent declares: {bad}"


def test_session_is_a_relational_cypher_session():
    srcs = sc.integration_sources()
    parents, over = sc.classes(srcs["GpuCypherSession.scala"])["GpuCypherSession"]
    assert "RelationalCypherSession" in parents
    assert {"records", "graphs", "elementTables", "Records", "Result"} <= set(over)
    recs = sc.classes(srcs["GpuRecords.scala"])
    assert "RelationalCypherRecordsFactory" in recs["GpuRecordsFactory"][0]
    assert {"unit", "empty", "fromElementTable", "from"} <= set(recs["GpuRecordsFactory"][1])
    assert "ElementTable" in sc.classes(srcs["GpuElementTable.scala"])["GpuElementTable"][0]
    # the relationship's end id comes from the END column (rowToCypherMap.scala:98-99 bug not copied)
    assert "header.endNodeFor(v)" in srcs["GpuRecords.scala"]


def test_removed_non_okapi_names():
    text = sc.strip_comments(sc.integration_sources()["GpuExprMapper.scala"])
    assert "Modulo" not in text  # okapi-ir defines no Modulo
    assert "CountStar(" not in text  # CountStar is a case object (Expr.scala:1071)


@pytest.mark.skipif(not os.path.isdir(REFERENCE), reason="reference sources absent")
def test_fixture_matches_reference():
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_okapi_api
    with open(FIXTURE) as f:
        assert make_okapi_api.build(REFERENCE) == json.load(f)


def test_fs_graph_source_twin_matches_python_layout():
    """GpuFSGraphSource.scala reads and writes the files capf_amd/fs_source.py
    does: same file / directory names, canonical key columns, GPU LONG parser
    for all-INTEGER tables, okapi's own schema JSON and name encoding."""
    from capf_amd import fs_source as fs
    text = sc.strip_comments(sc.integration_sources()["GpuFSGraphSource.scala"])
    for const, value in [("SchemaFile", fs.SCHEMA_FILE), ("MetaDataFile", fs.META_FILE),
                         ("NodesDir", fs.NODES_DIR), ("RelsDir", fs.RELS_DIR),
                         ("IdKey", "id"), ("SourceKey", "source"), ("TargetKey", "target")]:
        assert f'val {const} = "{value}"' in text, const
    assert "Native.csvReadLongs(" in text and "gpu.fromHost(" in text
    assert "PropertyGraphSchema.fromJson(" in text and "schema.toJson" in text
    assert "encodeSpecialCharacters" in text and "toPropertyColumnName" in text
    parents, over = sc.classes(text)["GpuFSGraphSource"]
    assert "PropertyGraphDataSource" in parents
    assert {"hasGraph", "graph", "schema", "store", "delete", "graphNames"} <= set(over)
