/*
 * GpuTable.scala — `Table[GpuTable]` over the MI355X backend: the drop-in for
 * FlinkTable (flink-cypher/src/main/scala/org/opencypher/flink/impl/table/FlinkTable.scala:49-199).
 * Every SPI method is one JNI call (Native.scala → integration/jni/capf_jni.cpp
 * → include/capf_gpu.h).  Handles are immutable and reference counted: each
 * wrapper owns one reference, released by a Cleaner when it is unreachable.
 */
package org.opencypher.gpu

import java.lang.ref.Cleaner

import org.opencypher.okapi.api.types.CypherType
import org.opencypher.okapi.api.value.CypherValue._
import org.opencypher.okapi.impl.exception.{IllegalArgumentException, NotImplementedException}
import org.opencypher.okapi.ir.api.expr._
import org.opencypher.okapi.relational.api.table.Table
import org.opencypher.okapi.relational.impl.planning._
import org.opencypher.okapi.relational.impl.table.RecordHeader

object GpuTable {
  private val cleaner: Cleaner = Cleaner.create()

  private final class Release(handle: Long) extends Runnable {
    override def run(): Unit = Native.tableRelease(handle)
  }

  /** Takes ownership of a handle returned by a native call. */
  def apply(handle: Long)(implicit session: GpuCypherSession): GpuTable = new GpuTable(handle)

  def joinTypeCode(joinType: JoinType): Int = joinType match {   // PhysicalConstants.scala:29-35
    case InnerJoin => Native.JoinInner
    case LeftOuterJoin => Native.JoinLeftOuter
    case RightOuterJoin => Native.JoinRightOuter
    case FullOuterJoin => Native.JoinFullOuter
    case CrossJoin => Native.JoinCross
  }
}

final class GpuTable private (private[gpu] val handle: Long)(implicit val session: GpuCypherSession)
  extends Table[GpuTable] {

  GpuTable.cleaner.register(this, new GpuTable.Release(handle))

  private def wrap(h: => Long): GpuTable = GpuTable(Native.guard(h))

  // ---------------------------------------------------------------- CypherTable
  override def physicalColumns: Seq[String] = Native.guard(Native.tableColumns(handle)).toSeq  // CypherTable.scala:48

  override def columnType: Map[String, CypherType] =                                          // CypherTable.scala:58
    physicalColumns.map(c => c -> GpuTypes.toCypher(Native.guard(Native.tableColumnType(handle, c)))).toMap

  override def rows: Iterator[String => CypherValue] = GpuRows.download(this)                 // CypherTable.scala:63

  override def size: Long = Native.guard(Native.tableSize(handle))                            // CypherTable.scala:68

  // ---------------------------------------------------------------- Table[T]
  override def cache(): GpuTable = wrap(Native.tableCache(handle))                            // Table.scala:52

  override def select(col: (String, String), cols: (String, String)*): GpuTable = {         // Table.scala:71
    val all = col +: cols
    wrap(Native.tableSelect(handle, all.map(_._1).toArray, all.map(_._2).toArray))
  }

  override def filter(expr: Expr)(implicit header: RecordHeader, parameters: CypherMap): GpuTable = // :81
    wrap(Native.tableFilter(handle, GpuExprMapper.program(expr, header, this, parameters)))

  override def drop(cols: String*): GpuTable = wrap(Native.tableDrop(handle, cols.toArray))   // :89

  override def join(other: GpuTable, joinType: JoinType, joinCols: (String, String)*): GpuTable = { // :99
    // disjoint column sets, as FlinkTable.join asserts (FlinkTable.scala:173-174); the
    // backend raises CAPF_ERR_ILLEGAL_ARGUMENT for an overlap as well
    wrap(Native.tableJoin(handle, other.handle, GpuTable.joinTypeCode(joinType),
      joinCols.map(_._1).toArray, joinCols.map(_._2).toArray))
  }

  override def unionAll(other: GpuTable): GpuTable = wrap(Native.tableUnionAll(handle, other.handle)) // :107

  override def orderBy(sortItems: (Expr, Order)*)(implicit header: RecordHeader, parameters: CypherMap): GpuTable = // :115
    wrap(Native.tableOrderBy(handle,
      sortItems.map { case (e, _) => GpuExprMapper.program(e, header, this, parameters) }.toArray,
      sortItems.map { case (_, o) => o == Descending }.toArray))

  override def skip(n: Long): GpuTable = wrap(Native.tableSkip(handle, n))                   // :123

  override def limit(n: Long): GpuTable = wrap(Native.tableLimit(handle, n))                 // :131

  override def distinct: GpuTable = wrap(Native.tableDistinct(handle))                       // :138

  override def distinct(cols: String*): GpuTable = wrap(Native.tableDistinctCols(handle, cols.toArray)) // :146

  override def group(by: Set[Var], aggregations: Map[String, Aggregator])                      // :158-159
    (implicit header: RecordHeader, parameters: CypherMap): GpuTable = {
    // grouping columns: every column owned by a grouping var (FlinkTable.scala:129-135)
    val byCols = by.toSeq.flatMap(v => header.ownedBy(v).toSeq.map(header.column)).distinct
    val aggs = aggregations.toSeq
    val lowered = aggs.map { case (_, agg) => GpuExprMapper.aggregator(agg, header, this, parameters) }
    wrap(Native.tableGroupEx(handle, byCols.toArray, lowered.map(_._1).toArray, lowered.map(_._2).toArray,
      lowered.map(_._3).toArray, lowered.map(_._4).toArray, aggs.map(_._1).toArray))
  }

  override def withColumns(columns: (Expr, String)*)(implicit header: RecordHeader, parameters: CypherMap): GpuTable = { // :170
    val (literalLists, others) = columns.partition { case (e, _) => listItems(e, parameters).isDefined }
    if (literalLists.nonEmpty) {  // [x, y, ...] / $list (FlinkSQLExprMapper.scala:71, 75): capf_table_list_columns
      val base = if (others.isEmpty) this else withColumns(others: _*)
      val keep = base.physicalColumns
      val built = literalLists.zipWithIndex.foldLeft(base) { case (t, ((e, col), i)) =>
        val items = listItems(e, parameters).get
        val tmp = items.indices.map(j => s"\u0003le$i.$j")
        val withItems = if (items.isEmpty) t else t.withColumns(items.zip(tmp): _*)
        wrap(Native.tableListColumns(withItems.handle, tmp.toArray, col))
      }
      return built.select(keep ++ literalLists.map(_._2): _*)
    }
    val (lists, rest) = columns.partition { case (e, _) => e.isInstanceOf[Labels] || e.isInstanceOf[Keys] }
    val (explodes, plain) = rest.partition { case (e, _) => e.isInstanceOf[Explode] }
    val base =
      if (plain.isEmpty) this
      else wrap(Native.tableWithColumns(handle,
        plain.map { case (e, _) => GpuExprMapper.program(e, header, this, parameters) }.toArray,
        plain.map(_._2).toArray))
    val withLists = lists.foldLeft(base) { case (t, (e, col)) => t.nameList(e, col, header) }
    explodes.foldLeft(withLists) { case (t, (Explode(list), col)) => t.explode(list, col, header, parameters) }
  }

  /** The element expressions of a list literal, or of a parameter holding a list. */
  private def listItems(e: Expr, parameters: CypherMap): Option[Seq[Expr]] = e match {
    case ListLit(items) => Some(items)
    case Param(p) => parameters.value.get(p) match {
      case Some(CypherList(vs)) => Some(vs.map {
        case CypherNull => NullLit()
        case CypherInteger(v) => IntegerLit(v)
        case CypherFloat(v) => FloatLit(v)
        case CypherString(v) => StringLit(v)
        case CypherBoolean(v) => if (v) TrueLit else FalseLit
        case other => throw NotImplementedException(s"GPU list element $other")
      })
      case _ => None
    }
    case _ => None
  }

  /** labels(n) / keys(n) (FlinkSQLExprMapper.scala:136-153): the label flag columns
    * (TRUE) or property columns (any value) of n, sorted by name, as a LIST<STRING>
    * column.  keys lists every property holding a value (GetKeys, :321-329, matches
    * `case (key, true)` on the VALUE — a reference bug not reproduced). */
  private def nameList(e: Expr, col: String, header: RecordHeader): GpuTable = {
    val present = physicalColumns.toSet
    val (found, kind) = e match {
      case Labels(v) => (header.labelsFor(v.owner.get).toSeq.map(l => l.label.name -> header.column(l)), 0)
      case Keys(v) => (header.propertiesFor(v.owner.get).toSeq.map(p => p.key.name -> header.column(p)), 1)
      case other => throw NotImplementedException(s"GPU list function $other")
    }
    val cols = found.filter { case (_, c) => present(c) }.sortBy(_._1)
    wrap(Native.tableNameList(handle, cols.map(_._2).toArray, Array.fill(cols.size)(kind),
      cols.map { case (n, _) => session.intern(n) }.toArray, col))
  }

  /** UNWIND list AS item = add(Explode(list) as item) (RelationalPlanner.scala:99-101). */
  private def explode(list: Expr, col: String, header: RecordHeader, parameters: CypherMap): GpuTable = {
    val literal: Option[Seq[CypherValue]] = list match {
      case ListLit(items) => Some(items.map {
        case NullLit(_) => CypherNull
        case IntegerLit(v) => CypherInteger(v)
        case FloatLit(v) => CypherFloat(v)
        case StringLit(v) => CypherString(v)
        case TrueLit => CypherBoolean(true)
        case FalseLit => CypherBoolean(false)
        case Param(p) => parameters(p)
        case other => throw NotImplementedException(s"GPU UNWIND element $other")
      })
      case Param(p) => parameters(p) match {
        case CypherList(vs) => Some(vs)
        case CypherNull => Some(Seq.empty)
        case other => throw NotImplementedException(s"GPU UNWIND of $other")
      }
      case NullLit(_) => Some(Seq.empty)
      case _ => None
    }
    literal match {
      case Some(vs) => wrap(GpuRows.explodeValues(this, col, vs))
      case None if header.contains(list) => wrap(Native.tableExplodeList(handle, header.column(list), col))
      case None => throw NotImplementedException(s"GPU UNWIND of $list")
    }
  }

  override def show(rows: Int): Unit = Native.guard(Native.tableShow(handle, rows))        // :177

  // ---------------------------------------------------------------- beyond the SPI
  /** Count into device memory without the host wait (capf_table_count_async). */
  def countAsync(dCount: Long): Unit = Native.guard(Native.tableCountAsync(handle, dCount))

  /** Re-encode INTEGER columns narrower (FOR32 / FOR24); values unchanged. */
  def compact(width: Int = 4): GpuTable = wrap(Native.tableCompactWidth(handle, width))
}

object GpuTypes {
  import org.opencypher.okapi.api.types._

  /** FlinkConversions.scala:43-117: LONG → CTInteger, DOUBLE → CTFloat, … (nullable: the
    * backend tracks validity per column, FlinkTable reports nullable types too). */
  def toCypher(code: Int): CypherType = code match {
    case Native.TypeInt64 => CTInteger.nullable
    case Native.TypeFloat64 => CTFloat.nullable
    case Native.TypeBool => CTBoolean.nullable
    case Native.TypeString => CTString.nullable
    case Native.TypeNull => CTNull
    case Native.TypeList => CTList(CTAny).nullable   // element type: Native.tableListInfo
    case other => throw IllegalArgumentException("a capf column type", other)
  }

  def fromCypher(t: CypherType): Int = t.material match {
    case CTInteger | _: CTNode | _: CTRelationship | CTIdentity => Native.TypeInt64
    case CTFloat => Native.TypeFloat64
    case CTBoolean => Native.TypeBool
    case CTString => Native.TypeString
    case CTNull | CTVoid => Native.TypeNull
    case other => throw org.opencypher.okapi.impl.exception.NotImplementedException(s"GPU column of type $other")
  }
}
