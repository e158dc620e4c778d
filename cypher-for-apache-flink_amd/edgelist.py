"""EdgeListDataSource over the GPU backend (graph ingest).

Mirror of flink-cypher/src/main/scala/org/opencypher/flink/api/io/edgelist/
EdgeListDataSource.scala:43-92:
 * one graph, `graph` (:49, :59, :91), with schema node label `V`, rel type `E`
   and no properties (:45-54, :83);
 * relationships = the CSV's two LONG fields (source, target) with field
   delimiter options["sep"] and comment prefix options["comment"] (:62-68),
   plus a unique LONG id per row (safeAddIdColumn, :72) — parsed on the GPU by
   capf_edge_list_read / capf_edge_list_parse (csrc/edge_list.hip);
 * nodes = distinct(source ∪ target) as `id` (:74-77), computed with the
   Table SPI itself (select, unionAll, distinct on the GPU);
 * store / delete raise UnsupportedOperationException (:85-89).
Both options are required, as in the reference (`options.get(..).get`).
"""
from ._lib import CypherException, IllegalArgumentException
from .graph import ElementTable, ScanGraph

NODE_LABEL = "V"
REL_TYPE = "E"
GRAPH_NAME = "graph"


class UnsupportedOperationException(CypherException):
    pass


class EdgeListDataSource:
    def __init__(self, session, path, options, compact=False):
        """`path`: a file path, or the file's bytes.  compact=True stores the
        id columns FOR32 (GpuTable.compact; values unchanged)."""
        for k in ("sep", "comment"):
            if k not in options:
                raise IllegalArgumentException(f"EdgeListDataSource: option `{k}` is required")
        self.session = session
        self.path = path
        self.options = dict(options)
        self.compact = compact

    def hasGraph(self, name):
        return name == GRAPH_NAME

    def graphNames(self):
        return {GRAPH_NAME}

    def schema(self, name):
        return {"nodes": {frozenset([NODE_LABEL]): {}}, "rels": {REL_TYPE: {}}}

    def graph(self, name=GRAPH_NAME):
        if not self.hasGraph(name):
            raise IllegalArgumentException(f"EdgeListDataSource has no graph {name!r}")
        rels = self.session.edge_list(self.path, self.options["sep"], self.options["comment"] or None)
        nodes = rels.select(("source", "id")).unionAll(rels.select(("target", "id"))).distinct()
        if self.compact:
            rels, nodes = rels.compact(), nodes.compact()
        return ScanGraph(self.session,
                         [ElementTable("node", frozenset([NODE_LABEL]), nodes, {})],
                         [ElementTable("rel", frozenset([REL_TYPE]), rels, {})])

    def store(self, name, graph):
        raise UnsupportedOperationException("Storing an edge list is not supported")

    def delete(self, name):
        raise UnsupportedOperationException("Deleting an edge list is not supported")
