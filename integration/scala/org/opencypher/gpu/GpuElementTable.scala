/*
 * GpuElementTable.scala — node / relationship element tables over GpuTable:
 * the drop-in for CAPFElementTable and CAPFElementTableFactory
 * (flink-cypher/src/main/scala/org/opencypher/flink/api/io/CAPFTable.scala:41-83)
 * implementing okapi's ElementTable[T] (okapi-relational/.../api/io/ElementTable.scala:41-125).
 * `create` keeps only the mapping's id and property columns (a metadata-only
 * select on the backend); `verify` requires INTEGER id columns, as
 * CAPFTable.scala:68-72 does.
 */
package org.opencypher.gpu

import org.opencypher.okapi.api.io.conversion.ElementMapping
import org.opencypher.okapi.api.types.CTInteger
import org.opencypher.okapi.relational.api.io.ElementTable
import org.opencypher.okapi.relational.api.table.RelationalElementTableFactory

case class GpuElementTableFactory(session: GpuCypherSession) extends RelationalElementTableFactory[GpuTable] {
  override def elementTable(elementMapping: ElementMapping, table: GpuTable): ElementTable[GpuTable] =
    GpuElementTable.create(elementMapping, table)(session)
}

case class GpuElementTable private[gpu] (
  override val mapping: ElementMapping,
  override val table: GpuTable
)(implicit val gpu: GpuCypherSession) extends ElementTable[GpuTable] with GpuRecordBehaviour {

  override type Records = GpuElementTable

  /** The records view of this element table (CAPFElementTable.records). */
  private[gpu] def records: GpuRecords = gpu.records.fromElementTable(this)

  override def cache(): GpuElementTable = copy(table = table.cache())

  override protected def verify(): Unit = {
    mapping.idKeys.values.toSeq.flatten.foreach {
      case (_, column) => table.verifyColumnType(column, CTInteger, "id key")
    }
  }
}

object GpuElementTable {
  /** The mapping's id columns, then its property columns (CAPFElementTable.create). */
  def create(mapping: ElementMapping, table: GpuTable)(implicit gpu: GpuCypherSession): GpuElementTable = {
    val columns = mapping.allSourceIdKeys ++ mapping.allSourcePropertyKeys
    GpuElementTable(mapping, table.select(columns: _*))
  }
}
