"""Edge-list ingest: EdgeListDataSource
(flink-cypher/.../api/io/edgelist/EdgeListDataSource.scala:43-92) parsed on the
GPU (csrc/edge_list.hip) against the CPU restatement (oracle/edgelist.py).

CPU tests pin the oracle on the reference's own EdgeListDataSourceTest data
(morpheus-testing/.../api/io/edgelist/EdgeListDataSourceTest.scala:39-82) and
hand-checked rows; GPU tests compare the parsed columns bit-exactly with the
oracle on seeded CSVs (separators, CRLF, comments, long lines across the
16 KiB parse chunks, int64 extremes) and run the 2-hop count over an R-MAT
graph loaded from CSV.
"""
import numpy as np
import pytest

from oracle import cmodel
from oracle import edgelist as oel

# EdgeListDataSourceTest.scala:39-45 (its blank first / whitespace last
# lines are Spark-CSV artefacts; Flink's CsvInputFormat rejects such rows)
MORPHEUS_EDGES = b"0 1\n0 2\n1 2\n1 3\n"


def test_oracle_reference_fixture():
    ids, src, dst = oel.parse(MORPHEUS_EDGES, " ", "#")
    assert len(ids) == 4 and len(oel.nodes(src, dst)) == 4  # EdgeListDataSourceTest.scala:78-82
    assert src.tolist() == [0, 0, 1, 1] and dst.tolist() == [1, 2, 2, 3]


def test_oracle_rows():
    data = b"# header\r\n-5,7\r\n9223372036854775807,-9223372036854775808,x y\r\n#c\n3,4"
    ids, src, dst = oel.parse(data, ",", "#")
    assert ids.tolist() == [0, 1, 2]
    assert src.tolist() == [-5, 2 ** 63 - 1, 3] and dst.tolist() == [7, -2 ** 63, 4]


@pytest.mark.parametrize("bad,line", [(b"1,2\n3\n", 2), (b"1,2\n\n3,4\n", 2), (b"1, 2\n", 1),
                                      (b"1,2\n3,9223372036854775808\n", 2), (b"-,1\n", 1),
                                      (b"1,2\n,3\n", 2), (b"1;2\n", 1)])
def test_oracle_rejects(bad, line):
    with pytest.raises(oel.ParseError) as e:
        oel.parse(bad, ",", "#")
    assert e.value.line == line


def test_oracle_vs_numpy_loadtxt():
    rng = np.random.default_rng(7)
    s, d = rng.integers(-10 ** 12, 10 ** 12, size=(2, 5000))
    data = oel.write_csv(s, d, sep="\t")
    _, src, dst = oel.parse(data, "\t", "#")
    ref = np.loadtxt(data.decode().splitlines(), dtype=np.int64, delimiter="\t")
    assert np.array_equal(src, ref[:, 0]) and np.array_equal(dst, ref[:, 1])


# ----------------------------------------------------------------- GPU


def _cases():
    rng = np.random.default_rng(11)
    out = []
    for k, (sep, crlf, trail, ncom, m) in enumerate([(",", False, True, 0, 1000), (" ", True, False, 5, 3000),
                                                      ("\t", False, False, 40, 70000), ("|", True, True, 1, 1),
                                                      ("::", False, True, 300, 20000)]):
        s = rng.integers(-2 ** 62, 2 ** 62, size=m)
        d = rng.integers(0, 1 << 20, size=m)
        s[: min(m, 3)] = [2 ** 63 - 1, -2 ** 63, 0][: min(m, 3)]
        coms = [(int(rng.integers(0, m + 1)), "#" + "c" * int(rng.integers(0, 50))) for _ in range(ncom)]
        if k == 2:  # a comment longer than two parse chunks (16 KiB each)
            coms.append((m // 2, "#" + "x" * 40000))
        out.append((oel.write_csv(s, d, sep=sep, crlf=crlf, comments=coms, trailing_newline=trail), sep))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(5))
def test_edge_list_parse_parity(gpu_session, k):
    data, sep = _cases()[k]
    t = gpu_session.edge_list(data, sep, "#")
    ids, src, dst = oel.parse(data, sep, "#")
    assert t.size == len(ids)
    for col, ref in (("id", ids), ("source", src), ("target", dst)):
        got, _ = t.column_arrays(col)
        assert np.array_equal(got, ref), col


@pytest.mark.gpu
@pytest.mark.parametrize("bad,line", [(b"1,2\n3\n", 2), (b"1,2\n\n3,4\n", 2), (b"1, 2\n", 1),
                                      (b"1,2\n3,9223372036854775808\n", 2), (b"-,1\n", 1),
                                      (b"1,2\n,3\n", 2), (b"1;2\n", 1)])
def test_edge_list_rejects(gpu_session, bad, line):
    from capf_amd._lib import IllegalArgumentException
    with pytest.raises(IllegalArgumentException, match=f"line {line} "):
        gpu_session.edge_list(bad, ",", "#")


@pytest.mark.gpu
def test_edge_list_empty_and_comments_only(gpu_session):
    assert gpu_session.edge_list(b"", ",", "#").size == 0
    assert gpu_session.edge_list(b"# a\n# b\n", ",", "#").size == 0


@pytest.mark.gpu
def test_edge_list_data_source_reference_fixture(gpu_session, tmp_path):
    from capf_amd.edgelist import EdgeListDataSource, UnsupportedOperationException
    p = tmp_path / "edges.txt"
    p.write_bytes(MORPHEUS_EDGES)
    ds = EdgeListDataSource(gpu_session, str(p), {"sep": " ", "comment": "#"})
    assert ds.hasGraph("graph") and not ds.hasGraph("foo") and ds.graphNames() == {"graph"}
    with pytest.raises(UnsupportedOperationException):
        ds.delete("graph")
    with pytest.raises(UnsupportedOperationException):
        ds.store("foo", None)
    g = ds.graph("graph")
    assert g.node_scan("n", ("V",)).table.size == 4  # EdgeListDataSourceTest.scala:78-82
    assert g.rel_scan("r", ("E",)).table.size == 4
    ids, _ = g.node_tables[0].table.column_arrays("id")
    assert sorted(ids.tolist()) == [0, 1, 2, 3]


@pytest.mark.gpu
@pytest.mark.parametrize("compact", [False, True], ids=["int64", "for32"])
def test_two_hop_over_csv_rmat(gpu_session, tmp_path, compact):
    from capf_amd.edgelist import EdgeListDataSource
    from capf_amd.expr import CountStar
    from capf_amd.planner import Match, NodeP, Query, RelP, Stage, run
    scale = 12
    src, dst = cmodel.rmat(scale)
    p = tmp_path / "rmat.csv"
    p.write_bytes(oel.write_csv(src, dst, sep=",", comments=[(0, "# R-MAT s12")]))
    g = EdgeListDataSource(gpu_session, str(p), {"sep": ",", "comment": "#"}, compact=compact).graph()
    q = Query([Match([NodeP("a"), NodeP("b"), NodeP("c")], [RelP("r1", "a", "b"), RelP("r2", "b", "c")])],
              [Stage([("count", CountStar())])])
    assert run(g, q)[0]["count"] == cmodel.count_2hop(src, dst, 1 << scale)
    assert gpu_session.last_plan() == "fused_chain2"
    assert g.node_tables[0].table.size == len(oel.nodes(src, dst))
