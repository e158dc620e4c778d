/*
 * GpuEdgeListDataSource.scala — the edge-list PropertyGraphDataSource on the
 * MI355X backend: the drop-in for EdgeListDataSource
 * (flink-cypher/src/main/scala/org/opencypher/flink/api/io/edgelist/EdgeListDataSource.scala:43-92).
 * The file is read and parsed natively (capf_edge_list_read: rel ids = data-line
 * ordinals, one valid zipWithUniqueId assignment); the node table is
 * distinct(source ∪ target) through the Table SPI, as the reference builds it
 * with Flink tables (:74-77).  One label `V`, one relationship type `E`.
 */
package org.opencypher.gpu

import org.opencypher.okapi.api.graph.{GraphName, PropertyGraph}
import org.opencypher.okapi.api.io.PropertyGraphDataSource
import org.opencypher.okapi.api.io.conversion.{NodeMappingBuilder, RelationshipMappingBuilder}
import org.opencypher.okapi.api.schema.{PropertyGraphSchema, PropertyKeys}
import org.opencypher.okapi.impl.exception.UnsupportedOperationException

object GpuEdgeListDataSource {
  val NODE_LABEL = "V"
  val REL_TYPE = "E"
  val GRAPH_NAME = GraphName("graph")

  val SCHEMA: PropertyGraphSchema = PropertyGraphSchema.empty
    .withNodePropertyKeys(Set(NODE_LABEL), PropertyKeys.empty)
    .withRelationshipPropertyKeys(REL_TYPE, PropertyKeys.empty)
}

case class GpuEdgeListDataSource(path: String, options: Map[String, String] = Map.empty)
  (implicit gpu: GpuCypherSession) extends PropertyGraphDataSource {

  import GpuEdgeListDataSource._

  override def hasGraph(name: GraphName): Boolean = name == GRAPH_NAME

  override def graph(name: GraphName): PropertyGraph = {
    // columns id, source, target (int64); separator and comment prefix as the
    // reference's CsvTableSource options
    val rels = gpu.edgeList(path, options.getOrElse("sep", ","), options.getOrElse("comment", "#"))
    val nodes = rels.select("source" -> "id").unionAll(rels.select("target" -> "id")).distinct
    val nodeMapping = NodeMappingBuilder.on("id").withImpliedLabels(NODE_LABEL).build
    val relMapping = RelationshipMappingBuilder.on("id").from("source").to("target").withRelType(REL_TYPE).build
    gpu.graphs.create(gpu.elementTables.elementTable(nodeMapping, nodes), gpu.elementTables.elementTable(relMapping, rels))
  }

  override def schema(name: GraphName): Option[PropertyGraphSchema] = Some(SCHEMA)

  override def store(name: GraphName, graph: PropertyGraph): Unit =
    throw UnsupportedOperationException("Storing an edge list is not supported")

  override def delete(name: GraphName): Unit =
    throw UnsupportedOperationException("Deleting an edge list is not supported")

  override def graphNames: Set[GraphName] = Set(GRAPH_NAME)
}
