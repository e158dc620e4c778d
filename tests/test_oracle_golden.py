"""Pin the oracle: the numpy restatement + planner reproduce the expected
results of the reference's own acceptance tests (tests/golden/reference_cases.py)."""
import pytest

from conftest import bag
from reference_cases import CASES

from capf_amd.graph import ScanGraph
from capf_amd.planner import run
from oracle.create_parser import parse_create
from oracle.table_np import OracleSession


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_reference_case_on_oracle(case):
    cid, src, create, query, expected = case
    g = ScanGraph.from_data(OracleSession(), parse_create(create))
    got = run(g, query)
    assert bag(got) == bag(expected), f"{cid} ({src}): {got}"


def test_create_parser_ids():
    # CreateQueryParser.scala:150-200: one counter, chain processed left-nested
    g = parse_create("CREATE (a:N)-[:R]->(b:N)-[:R]->(c:N)")
    assert [n[0] for n in g.nodes] == [0, 1, 3]
    assert [(r[0], r[1], r[2]) for r in g.rels] == [(2, 0, 1), (4, 1, 3)]
    g = parse_create("CREATE (a)<-[:R]-(b)")
    assert g.rels == [(2, 1, 0, "R", {})]
