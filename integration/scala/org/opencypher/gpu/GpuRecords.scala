/*
 * GpuRecords.scala — records over GpuTable: the drop-in for CAPFRecords /
 * CAPFRecordsFactory (flink-cypher/src/main/scala/org/opencypher/flink/impl/CAPFRecords.scala:47-145)
 * and for the row → CypherMap conversion of
 * flink-cypher/.../impl/convert/rowToCypherMap.scala:40-131.
 *
 * Materialisation: `collect` / `iterator` download the table's columns once
 * (GpuRows.download: one capf_table_download per column) and assemble every
 * row's return items.  Nodes and relationships are reassembled from their
 * columns as GpuNode / GpuRelationship (labels = the true label flags,
 * properties = the non-null property columns).  The relationship's end id is
 * read from its END node column; rowToCypherMap.scala:98-99 reads the start
 * column twice, a reference bug that is not reproduced.
 */
package org.opencypher.gpu

import org.opencypher.okapi.api.types.{CTList, CTNode, CTRelationship, CypherType}
import org.opencypher.okapi.api.value.CypherValue.{CypherBoolean, CypherInteger, CypherList, CypherMap, CypherNull, CypherValue}
import org.opencypher.okapi.impl.exception.UnsupportedOperationException
import org.opencypher.okapi.ir.api.expr.{Expr, ListSegment, Var}
import org.opencypher.okapi.relational.api.io.ElementTable
import org.opencypher.okapi.relational.api.table.{RelationalCypherRecords, RelationalCypherRecordsFactory}
import org.opencypher.okapi.relational.impl.table.RecordHeader

/** RelationalCypherRecordsFactory[GpuTable] (RelationalCypherRecords.scala:43-54). */
case class GpuRecordsFactory()(implicit gpu: GpuCypherSession) extends RelationalCypherRecordsFactory[GpuTable] {

  override type Records = GpuRecords

  /** One row, no columns: the driving table of a query without input. */
  override def unit(): GpuRecords = GpuRecords(RecordHeader.empty, gpu.unitTable())

  /** No rows; one column per distinct header column, typed from its expressions. */
  override def empty(initialHeader: RecordHeader = RecordHeader.empty): GpuRecords = {
    val columns = initialHeader.exprToColumn.toSeq
      .groupBy { case (_, column) => column }
      .toSeq
      .sortBy { case (column, _) => column }
      .map { case (column, exprs) => column -> GpuTypes.fromCypher(exprs.head._1.cypherType) }
    GpuRecords(initialHeader, gpu.emptyTable(columns))
  }

  override def fromElementTable(elementTable: ElementTable[GpuTable]): GpuRecords =
    GpuRecords(elementTable.header, elementTable.table)

  /** The result records of a query (RelationalCypherResult.getRecords): the
    * display names default to the header's variables, as in CAPFRecordsFactory.from. */
  override def from(header: RecordHeader, table: GpuTable, maybeDisplayNames: Option[Seq[String]]): GpuRecords = {
    val displayNames = maybeDisplayNames.orElse(Some(header.vars.map(_.withoutType).toSeq))
    GpuRecords(header, table, displayNames)
  }
}

case class GpuRecords(
  header: RecordHeader,
  table: GpuTable,
  override val logicalColumns: Option[Seq[String]] = None
)(implicit val gpu: GpuCypherSession) extends RelationalCypherRecords[GpuTable] with GpuRecordBehaviour {

  override type Records = GpuRecords

  /** Table.cache is the identity on the backend (tables are immutable, results memoised). */
  override def cache(): GpuRecords = copy(table = table.cache())

  override def toString: String =
    if (header.isEmpty) "GpuRecords.empty" else s"GpuRecords(header: $header)"
}

/** What CAPF's RecordBehaviour provides (CAPFRecords.scala:121-145), over GpuTable. */
trait GpuRecordBehaviour extends RelationalCypherRecords[GpuTable] {

  override lazy val columnType: Map[String, CypherType] = table.columnType

  override def rows: Iterator[String => CypherValue] = table.rows

  override def iterator: Iterator[CypherMap] = toCypherMaps.iterator

  override def collect: Array[CypherMap] = toCypherMaps

  def toLocalIterator: Iterator[CypherMap] = iterator

  /** Every row as a CypherMap of the header's return items. */
  def toCypherMaps: Array[CypherMap] = {
    val convert = GpuRowToCypherMap(header)
    table.rows.map(convert).toArray
  }
}

/** rowToCypherMap (rowToCypherMap.scala:40-131) over a downloaded row
  * (column name → value). */
final case class GpuRowToCypherMap(header: RecordHeader) extends ((String => CypherValue) => CypherMap) {

  private val items = header.returnItems.toSeq

  override def apply(row: String => CypherValue): CypherMap =
    CypherMap(items.map(v => v.name -> value(row, v)): _*)

  private def value(row: String => CypherValue, v: Var): CypherValue = v.cypherType.material match {
    case _: CTNode => node(row, v)
    case _: CTRelationship => relationship(row, v)
    case CTList(_) if !header.exprToColumn.contains(v) => segments(row, v)
    case _ => row(header.column(v))
  }

  private def id(row: String => CypherValue, e: Expr, what: String): Option[Long] = row(header.column(e)) match {
    case CypherNull => None
    case i: CypherInteger => Some(i.value)
    case other => throw UnsupportedOperationException(s"$what id has to be an INTEGER instead of $other")
  }

  private def properties(row: String => CypherValue, v: Var): CypherMap =
    CypherMap(header.propertiesFor(v).toSeq
      .map(p => p.key.name -> row(header.column(p)))
      .filterNot { case (_, value) => value.isNull }: _*)

  private def flagged(row: String => CypherValue, flag: Expr): Boolean = row(header.column(flag)) match {
    case b: CypherBoolean => b.value
    case _ => false
  }

  private def node(row: String => CypherValue, v: Var): CypherValue = id(row, v, "node") match {
    case None => CypherNull
    case Some(i) =>
      val labels = header.labelsFor(v).collect { case l if flagged(row, l) => l.label.name }
      GpuNode(i, labels, properties(row, v))
  }

  private def relationship(row: String => CypherValue, v: Var): CypherValue = id(row, v, "relationship") match {
    case None => CypherNull
    case Some(i) =>
      val start = id(row, header.startNodeFor(v), "start node").getOrElse(-1L)
      val end = id(row, header.endNodeFor(v), "end node").getOrElse(-1L)   // END column (cf. rowToCypherMap.scala:99)
      val relType = header.typesFor(v).collectFirst { case t if flagged(row, t) => t.relType.name }
        .getOrElse(throw UnsupportedOperationException(s"relationship $i without a type flag"))
      GpuRelationship(i, start, end, relType, properties(row, v))
  }

  /** A list assembled from its ListSegment columns (collectComplexList, :125-131). */
  private def segments(row: String => CypherValue, v: Var): CypherList = {
    val parts = header.ownedBy(v).collect { case s: ListSegment => s }.toSeq.sortBy(_.index)
    CypherList(parts.map(s => value(row, s)).filterNot(_ == CypherNull): _*)
  }
}
