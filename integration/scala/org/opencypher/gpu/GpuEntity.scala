/*
 * GpuEntity.scala — the node and relationship values returned by GpuRecords:
 * the counterparts of CAPFNode / CAPFRelationship
 * (flink-cypher/src/main/scala/org/opencypher/flink/api/value/CAPFEntity.scala:31-58)
 * over okapi's Node[Long] / Relationship[Long] (okapi-api/.../api/value/CypherValue.scala:382-470).
 */
package org.opencypher.gpu

import org.opencypher.okapi.api.value.CypherValue.{CypherMap, Node, Relationship}

case class GpuNode(
  override val id: Long,
  override val labels: Set[String] = Set.empty,
  override val properties: CypherMap = CypherMap.empty
) extends Node[Long] {

  override type I = GpuNode

  override def copy(id: Long = id, labels: Set[String] = labels, properties: CypherMap = properties): GpuNode =
    GpuNode(id, labels, properties)
}

case class GpuRelationship(
  override val id: Long,
  override val startId: Long,
  override val endId: Long,
  override val relType: String,
  override val properties: CypherMap = CypherMap.empty
) extends Relationship[Long] {

  override type I = GpuRelationship

  override def copy(
    id: Long = id,
    source: Long = startId,
    target: Long = endId,
    relType: String = relType,
    properties: CypherMap = properties): GpuRelationship =
    GpuRelationship(id, source, target, relType, properties)
}
