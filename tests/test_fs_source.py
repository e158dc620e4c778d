"""FS graph source (capf_amd/fs_source.py, FSGraphSource.scala:47-148 over CSV):
the reference's own CSV graph (flink-cypher/src/main/resources/csv/products,
committed as tests/golden/fs/products) read into element tables, queried
through the planner and checked against a join computed straight from the CSV
text; the directory layout and names of DefaultGraphDirectoryStructure
(GraphDirectoryStructure.scala:35-98); store → read round trips; the GPU CSV
reader (capf_csv_read_longs) on an all-LONG R-MAT relationship table."""
import csv
import json
import os

import numpy as np
import pytest

from conftest import bag, case_parts, check_case

import capf_import  # noqa: F401
from capf_amd.expr import ElementProperty, Var
from capf_amd.fs_source import FSGraphSource, decode_special, encode_special, node_table_dir
from capf_amd.graph import ScanGraph
from capf_amd.planner import Match, NodeP, Query, RelP, Stage, run
from oracle.create_parser import parse_create
from oracle.table_np import OracleSession

HERE = os.path.dirname(os.path.abspath(__file__))
FS_ROOT = os.path.join(HERE, "golden", "fs")


def _p(v, k):
    return ElementProperty(Var(v, "NODE"), k, "ANY")


BOUGHT_QUERY = Query([Match([NodeP("c", ("Customer",)), NodeP("p", ("Product",))],
                            [RelP("b", "c", "p", ("BOUGHT",))])],
                     [Stage([("name", _p("c", "name")), ("title", _p("p", "title")),
                             ("rating", ElementProperty(Var("b", "RELATIONSHIP"), "rating", "ANY"))])])
CUSTOMERS = Query([Match([NodeP("c", ("Customer",))])], [Stage([("name", _p("c", "name"))])])


def _csv_rows(*path):
    with open(os.path.join(FS_ROOT, "products", *path)) as f:
        return list(csv.reader(f))


def expected_bought():
    """The BOUGHT join computed from the CSV text alone (canonical column
    order: id, properties sorted by column name — Customer: name; Product:
    category, rank, title; BOUGHT: id, source, target, helpful, rating, votes)."""
    cust = {int(r[0]): r[1] for r in _csv_rows("nodes", "Customer", "table.csv")}
    prod = {int(r[0]): r[3] for r in _csv_rows("nodes", "Product", "table.csv")}
    out = []
    for r in _csv_rows("relationships", "BOUGHT", "table.csv"):
        s, t, rating = int(r[1]), int(r[2]), int(r[4])
        if s in cust and t in prod:
            out.append({"name": cust[s], "title": prod[t], "rating": rating})
    return out


def test_directory_structure_names():
    # StringEncodingUtilities.encodeSpecialCharacters: letters, digits, '_' kept
    assert encode_special("Person_1") == "Person_1"
    assert encode_special("a b.c") == "a@0020b@002ec"
    assert encode_special("ä") == "@00e4"
    for s in ("a b.c", "KNOWS", "名前", "x@y", "😀"):
        assert decode_special(encode_special(s)) == s
    assert node_table_dir({"Person", "German"}) == "German_Person"
    src = FSGraphSource(OracleSession(), FS_ROOT)
    assert src.graph_names() == {"products"} and src.has_graph("products")
    assert src.metadata("products") == {"tableStorageFormat": "csv", "tags": [0]}
    nodes, rels = src.schema("products")
    assert set(nodes) == {frozenset(["Customer"]), frozenset(["Product"])}
    assert rels == {"BOUGHT": {"rating": "INTEGER", "helpful": "INTEGER", "votes": "INTEGER"}}


def test_products_graph_on_oracle():
    g = FSGraphSource(OracleSession(), FS_ROOT).graph("products")
    sizes = {tuple(sorted(t.labels)): t.table.size for t in g.node_tables + g.rel_tables}
    assert sizes == {("Customer",): 12, ("Product",): 16, ("BOUGHT",): 8}
    prod = next(t for t in g.node_tables if "Product" in t.labels).table
    assert prod.column_values("p_title")[0] == "1984" and prod.column_values("p_rank")[0] == 246
    assert bag(run(g, BOUGHT_QUERY)) == bag(expected_bought())
    assert len(run(g, CUSTOMERS)) == 12  # CsvDemo (Demo.scala:143-157)


ROUND_TRIP = """
CREATE (a:Person:German {name: "Stefan", age: 42, score: 1.5, ok: true})
CREATE (b:Person {name: "Mats", age: 23})
CREATE (c:`Odd Label` {x: 1})
CREATE (a)-[:KNOWS {since: 2016}]->(b)
CREATE (b)-[:KNOWS {since: 2017, weight: 0.25}]->(c)
CREATE (c)-[:`HAS ONE` ]->(a)
"""


def test_store_read_round_trip(tmp_path):
    from reference_cases import CASES
    s = OracleSession()
    src = FSGraphSource(s, str(tmp_path))
    g = ScanGraph.from_data(s, parse_create(ROUND_TRIP))
    src.store("social.v1", g)
    assert (tmp_path / "social" / "v1" / "propertyGraphSchema.json").is_file()
    assert (tmp_path / "social" / "v1" / "nodes" / "German_Person").is_dir()
    assert (tmp_path / "social" / "v1" / "nodes" / "Odd@0020Label").is_dir()
    assert (tmp_path / "social" / "v1" / "relationships" / "HAS@0020ONE").is_dir()
    js = json.loads((tmp_path / "social" / "v1" / "propertyGraphSchema.json").read_text())
    assert {tuple(e["labels"]) for e in js["labelPropertyMap"]} == {("German", "Person"), ("Person",),
                                                                   ("Odd Label",)}
    with pytest.raises(ValueError):
        src.store("social.v1", g)
    back = FSGraphSource(OracleSession(), str(tmp_path)).graph("social.v1")
    q = Query([Match([NodeP("a"), NodeP("b")], [RelP("r", "a", "b")])],
              [Stage([("a", _p("a", "name")), ("b", _p("b", "name")), ("x", _p("b", "x")),
                      ("s", _p("a", "score"))])])
    assert bag(run(back, q)) == bag(run(g, q))
    # every reference acceptance case survives store → read
    for case in CASES[:40]:
        cid, _, create, query, expected, opts = case_parts(case)
        gg = ScanGraph.from_data(s, parse_create(create))
        name = "c" + cid.replace("-", "_")
        src.store(name, gg)
        got = run(FSGraphSource(OracleSession(), str(tmp_path)).graph(name), query, opts.get("params"))
        assert check_case(got, expected, opts), cid
    src.delete("social.v1")
    assert not src.has_graph("social.v1")


def test_short_row_fails(tmp_path):
    import shutil
    shutil.copytree(os.path.join(FS_ROOT, "products"), tmp_path / "products", copy_function=shutil.copyfile)
    with open(tmp_path / "products" / "nodes" / "Product" / "table.csv", "a") as f:
        f.write("1017,Book\n")
    with pytest.raises(ValueError, match="too short"):
        FSGraphSource(OracleSession(), str(tmp_path)).graph("products")


# ----------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_products_graph_on_gpu(gpu_session):
    g = FSGraphSource(gpu_session, FS_ROOT).graph("products")
    assert bag(run(g, BOUGHT_QUERY)) == bag(expected_bought())
    rel = g.rel_tables[0].table
    assert rel.column_values("p_rating") == [int(r[4]) for r in _csv_rows("relationships", "BOUGHT", "table.csv")]


NULLABLE_INT = """
CREATE (a:Person {name: 'A', age: 30})
CREATE (b:Person {name: 'B'})
CREATE (c:Person {name: 'C', age: 7})
CREATE (a)-[:KNOWS {since: 2010}]->(b)
CREATE (b)-[:KNOWS]->(c)
"""


@pytest.mark.gpu
def test_store_read_nullable_integer_on_gpu(gpu_session, tmp_path):
    """A nullable INTEGER property ('INTEGER?') with a missing value is stored
    as an empty CSV field and reads back as NULL on the GPU session too."""
    g = ScanGraph.from_data(gpu_session, parse_create(NULLABLE_INT))
    FSGraphSource(gpu_session, str(tmp_path)).store("nulls", g)
    back = FSGraphSource(gpu_session, str(tmp_path)).graph("nulls")
    q = Query([Match([NodeP("a"), NodeP("b")], [RelP("r", "a", "b")])],
              [Stage([("a", _p("a", "name")), ("age", _p("a", "age")), ("b_age", _p("b", "age")),
                      ("since", _p("r", "since"))])])
    got = bag(run(back, q))
    assert got == bag(run(g, q))
    assert got == bag([{"a": "A", "age": 30, "b_age": None, "since": 2010},
                       {"a": "B", "age": None, "b_age": 7, "since": None}])


@pytest.mark.gpu
@pytest.mark.parametrize("compact", [False, 3])
def test_rmat_csv_graph_on_gpu(gpu_session, tmp_path, compact):
    """An R-MAT s16 graph stored as CSV tables (all-LONG: read by the GPU
    parser), read back, 2-hop count = the committed fixture."""
    from capf_amd.graph import ElementTable
    from capf_amd.planner import Match as M
    from capf_amd.expr import CountStar
    from oracle import cmodel
    scale = 16
    src, dst = cmodel.rmat(scale)
    n = 1 << scale
    gdir = tmp_path / "rmat"
    (gdir / "nodes" / "V").mkdir(parents=True)
    (gdir / "relationships" / "E").mkdir(parents=True)
    (gdir / "capsGraphMetaData.json").write_text(json.dumps({"tableStorageFormat": "csv", "tags": [0]}))
    (gdir / "propertyGraphSchema.json").write_text(json.dumps(
        {"version": "1.0", "labelPropertyMap": [{"labels": ["V"], "properties": {}}],
         "relTypePropertyMap": [{"relType": "E", "properties": {"w": "INTEGER"}}]}))
    np.savetxt(gdir / "nodes" / "V" / "table.csv", np.arange(n), fmt="%d")
    m = len(src)
    rows = np.stack([np.arange(m), src, dst, (src * 7 + dst) % 1000 - 500], axis=1)
    half = m // 2  # two files per table directory
    np.savetxt(gdir / "relationships" / "E" / "part-0.csv", rows[:half], fmt="%d", delimiter=",")
    np.savetxt(gdir / "relationships" / "E" / "part-1.csv", rows[half:], fmt="%d", delimiter=",")
    g = FSGraphSource(gpu_session, str(tmp_path)).graph("rmat", compact=compact)
    assert g.rel_tables[0].table.size == m
    w = np.asarray(g.rel_tables[0].table.column_arrays("p_w")[0])
    assert (np.sort(w) == np.sort(rows[:, 3])).all()
    q = Query([M([NodeP("a"), NodeP("b"), NodeP("c")], [RelP("r1", "a", "b"), RelP("r2", "b", "c")])],
              [Stage([("count", CountStar())])])
    with open(os.path.join(HERE, "golden", "rmat_counts.json")) as f:
        want = json.load(f)["rmat"][str(scale)]["two_hop"]
    assert run(g, q)[0]["count"] == want


@pytest.mark.gpu
def test_csv_longs_parse_errors(gpu_session):
    from capf_amd import _lib
    names = ["id", "source", "target"]
    t = gpu_session.csv_parse_longs(b"1,2,3\n4,5,6,extra\r\n-7,8,9", ",", names)
    assert t.column_values("id") == [1, 4, -7] and t.column_values("target") == [3, 6, 9]
    for bad, why in ((b"1,2,3\n4,5\n", "too short"), (b"1,2,3\n4,,6\n", "empty"),
                     (b"1,2,x\n", "illegal"), (b"1,2,99999999999999999999\n", "range")):
        with pytest.raises(_lib.IllegalArgumentException, match=why):
            gpu_session.csv_parse_longs(bad, ",", names).size
