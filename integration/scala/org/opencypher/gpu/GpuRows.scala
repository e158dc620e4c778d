/*
 * GpuRows.scala — CypherTable.rows (CypherTable.scala:63) over downloaded
 * columns: one capf_table_download per column into direct buffers, then rows as
 * `String => CypherValue`, the shape CAPFRecords' materialisation consumes
 * (flink-cypher/.../impl/CAPFRecords.scala:142-144, rowToCypherMap.scala:40-131).
 * The session, records and element tables that consume it live in
 * GpuCypherSession.scala, GpuRecords.scala and GpuElementTable.scala.
 */
package org.opencypher.gpu

import java.nio.{ByteBuffer, ByteOrder}

import org.opencypher.okapi.api.value.CypherValue._

object GpuRows {
  def download(t: GpuTable): Iterator[String => CypherValue] = {
    val n = t.size
    require(n <= Int.MaxValue / 8, s"rows: $n rows do not fit one host buffer")
    val cols = t.physicalColumns
    val data: Map[String, Int => CypherValue] = cols.map { c =>
      val ty = Native.guard(Native.tableColumnType(t.handle, c))
      if (ty == Native.TypeList) c -> lists(t, c, n) else {
      val width = if (ty == Native.TypeBool) 1 else 8
      val values = ByteBuffer.allocateDirect(math.max(1, (n * width).toInt)).order(ByteOrder.nativeOrder())
      val valid = ByteBuffer.allocateDirect(math.max(1, n.toInt))
      if (ty != Native.TypeNull) Native.guard(Native.tableDownload(t.handle, c, values, valid))
      val get: Int => CypherValue = ty match {
        case Native.TypeNull => _ => CypherNull
        case Native.TypeInt64 => i => if (valid.get(i) == 0) CypherNull else CypherInteger(values.getLong(8 * i))
        case Native.TypeFloat64 => i => if (valid.get(i) == 0) CypherNull else CypherFloat(values.getDouble(8 * i))
        case Native.TypeBool => i => if (valid.get(i) == 0) CypherNull else CypherBoolean(values.get(i) != 0)
        case Native.TypeString => i =>
          if (valid.get(i) == 0) CypherNull
          else CypherString(Native.guard(Native.stringLookup(t.session.handle, values.getLong(8 * i))))
      }
      c -> get
    }}.toMap
    Iterator.range(0, n.toInt).map(i => (c: String) => data(c)(i))
  }

  /** UNWIND of a literal / parameter list (capf_table_explode_values): the
    * elements as one typed buffer — INTEGER and FLOAT widen to FLOAT, NULL
    * elements kept — returns the new handle. */
  def explodeValues(t: GpuTable, col: String, vs: Seq[CypherValue]): Long = {
    val present = vs.filter(_ != CypherNull)
    val ty =
      if (present.isEmpty) Native.TypeNull
      else if (present.forall(v => v.isInstanceOf[CypherInteger])) Native.TypeInt64
      else if (present.forall(v => v.isInstanceOf[CypherInteger] || v.isInstanceOf[CypherFloat])) Native.TypeFloat64
      else if (present.forall(_.isInstanceOf[CypherBoolean])) Native.TypeBool
      else if (present.forall(_.isInstanceOf[CypherString])) Native.TypeString
      else throw new UnsupportedOperationException(s"UNWIND of a list of mixed types: $vs")
    val n = vs.size
    val width = if (ty == Native.TypeBool) 1 else 8
    val values = ByteBuffer.allocateDirect(math.max(1, n * width)).order(ByteOrder.nativeOrder())
    val valid = ByteBuffer.allocateDirect(math.max(1, n))
    vs.zipWithIndex.foreach { case (v, i) =>
      valid.put(i, if (v == CypherNull) 0.toByte else 1.toByte)
      v match {
        case CypherInteger(x) if ty == Native.TypeFloat64 => values.putDouble(8 * i, x.toDouble)
        case CypherInteger(x) => values.putLong(8 * i, x)
        case CypherFloat(x) => values.putDouble(8 * i, x)
        case CypherBoolean(b) => values.put(i, if (b) 1.toByte else 0.toByte)
        case CypherString(s) => values.putLong(8 * i, Native.guard(Native.stringIntern(t.session.handle, s)))
        case _ =>
      }
    }
    Native.guard(Native.tableExplodeValues(t.handle, col, ty, n.toLong,
      if (ty == Native.TypeNull) null else values, valid))
  }

  /** A LIST column (collect): offsets + elements (capf_table_download_list). */
  private def lists(t: GpuTable, c: String, n: Long): Int => CypherValue = {
    val nv = Array(0L)
    val elem = Native.guard(Native.tableListInfo(t.handle, c, nv))
    val width = if (elem == Native.TypeBool) 1 else 8
    val offsets = ByteBuffer.allocateDirect(8 * (n.toInt + 1)).order(ByteOrder.nativeOrder())
    val values = ByteBuffer.allocateDirect(math.max(1, (nv(0) * width).toInt)).order(ByteOrder.nativeOrder())
    val valid = ByteBuffer.allocateDirect(math.max(1, n.toInt))
    Native.guard(Native.tableDownloadList(t.handle, c, offsets, values, valid))
    def value(k: Int): CypherValue = elem match {
      case Native.TypeInt64 => CypherInteger(values.getLong(8 * k))
      case Native.TypeFloat64 => CypherFloat(values.getDouble(8 * k))
      case Native.TypeBool => CypherBoolean(values.get(k) != 0)
      case Native.TypeString => CypherString(Native.guard(Native.stringLookup(t.session.handle, values.getLong(8 * k))))
      case _ => CypherNull
    }
    i =>
      if (valid.get(i) == 0) CypherNull
      else CypherList((offsets.getLong(8 * i).toInt until offsets.getLong(8 * (i + 1)).toInt).map(value): _*)
  }
}
