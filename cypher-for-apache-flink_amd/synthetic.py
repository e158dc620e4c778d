"""Synthetic benchmark graphs resident in HBM (BASELINE.json configs 2-4).

R-MAT with Graph500 parameters a/b/c/d = .57/.19/.19/.05, edge factor 16,
seed 0x5EED0000 + scale; generated on the GPU by
capf_rmat_rel_table.  The graph is exposed as a ScanGraph with one node
label combination per table, exactly like EdgeListDataSource
(flink-cypher/.../api/io/edgelist/EdgeListDataSource.scala:56-92: label `V`,
type `E`), or with the config-2 `Person` / `Other` split.
"""
from .expr import BoolLit, Equals, Var
from .graph import ElementTable, ScanGraph
from .header import RecordHeader
from .table import compact_as

A, B, C = 0.57, 0.19, 0.19


def thresholds(a=A, b=B, c=C):
    t = lambda x: min(int(x * 2 ** 32), 2 ** 32 - 1)
    return t(a), t(a + b), t(a + b + c)


def rmat_seed(scale):
    return 0x5EED0000 + scale


def rmat_graph(session, scale, edge_factor=16, seed=None, person_split=False, first=0, count=None,
               node_base=0, n_nodes=None, compact=False, id_stride=1):
    """ScanGraph over an R-MAT edge table (optionally a shard [first, first+count)).

    compact=True stores the id columns FOR32-encoded (GpuTable.compact),
    compact=3 FOR24 (3 B per id where the range fits 24 bits).  id_stride > 1
    spreads the node ids to v·id_stride + 7 (rel source/target alike): a sparse
    id domain with no dense range, so joins on node ids cannot address directly."""
    seed = rmat_seed(scale) if seed is None else seed
    m = edge_factor << scale
    count = m - first if count is None else count
    n = (1 << scale) if n_nodes is None else n_nodes
    rels = session.rmat_rels(scale, seed, thresholds(), first, count, id_base=0)
    if id_stride != 1:
        rels = _spread_ids(rels, ("source", "target"), id_stride)
    rels = compact_as(rels, compact)
    rel_tables = [ElementTable("rel", frozenset(["E"]), rels, {})]
    if person_split:
        nodes = session.range_nodes(node_base, n, seed=seed, id_col="id", label_col="person")
        nodes = compact_as(nodes, compact)
        h = RecordHeader({Var("person"): "person"})
        person = nodes.filter(Equals(Var("person"), BoolLit(True)), h, {}).select("id")
        other = nodes.filter(Equals(Var("person"), BoolLit(False)), h, {}).select("id")
        if compact:
            # one element table per label combination, built at ingest
            # (ScanGraph.scala:115-128): materialised here, not re-filtered per query
            person, other = compact_as(person, compact), compact_as(other, compact)
        node_tables = [ElementTable("node", frozenset(["Person"]), person, {}),
                       ElementTable("node", frozenset(["Other"]), other, {})]
    else:
        nodes = session.range_nodes(node_base, n, id_col="id")
        if id_stride != 1:
            nodes = _spread_ids(nodes, ("id",), id_stride)
        nodes = compact_as(nodes, compact)
        node_tables = [ElementTable("node", frozenset(["V"]), nodes, {})]
    return ScanGraph(session, node_tables, rel_tables)


def _spread_ids(table, cols, stride):
    """The table with each of `cols` replaced by col·stride + 7 (materialised)."""
    from .expr import Add, IntegerLit, Multiply
    h = RecordHeader({Var(c): c for c in table.physicalColumns})
    spread = table.withColumns(*[(Add(Multiply(Var(c), IntegerLit(stride)), IntegerLit(7)), "_s_" + c)
                                 for c in cols], header=h)
    keep = [(c, c) if c not in cols else ("_s_" + c, c) for c in table.physicalColumns]
    return spread.select(*keep).cache()
