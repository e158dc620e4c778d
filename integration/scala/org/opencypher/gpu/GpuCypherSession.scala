/*
 * GpuCypherSession.scala — the RelationalCypherSession[GpuTable] of the MI355X
 * backend: the drop-in for CAPFSession
 * (flink-cypher/src/main/scala/org/opencypher/flink/api/CAPFSession.scala:47-91).
 *
 * The okapi pipeline (parser → IR → logical planner → RelationalPlanner →
 * RelationalOptimizer) is inherited unchanged from RelationalCypherSession
 * (okapi-relational/.../api/graph/RelationalCypherSession.scala:63-199); this
 * class only supplies the three backend factories that class leaves abstract
 * (:101-105): `records`, `graphs` and `elementTables`.  Where CAPFSession
 * holds a Flink ExecutionEnvironment + BatchTableEnvironment, this holds one
 * capf_session (a HIP stream on one GPU, its stream-ordered memory pool and
 * the string dictionary).
 */
package org.opencypher.gpu

import org.opencypher.okapi.relational.api.graph.{RelationalCypherGraph, RelationalCypherGraphFactory, RelationalCypherSession}
import org.opencypher.okapi.relational.api.planning.RelationalCypherResult

final class GpuCypherSession private (val device: Int, hipStream: Long)
  extends RelationalCypherSession[GpuTable] with AutoCloseable {

  override type Result = RelationalCypherResult[GpuTable]

  override type Records = GpuRecords

  protected implicit val gpu: GpuCypherSession = this

  /** The native session (capf_session_create, include/capf_gpu.h). */
  private[gpu] val handle: Long = Native.guard(Native.sessionCreate(device, hipStream))

  private val strings = scala.collection.mutable.HashMap.empty[String, Long]

  /** Set by DistGpuTable.nodePartitioned: inner joins between projections of
    * the base shards are recorded (the 2-hop count dispatch looks at them). */
  @volatile private[gpu] var deferJoins: Boolean = false

  // the factories RelationalCypherSession.scala:101-105 leaves abstract
  override val records: GpuRecordsFactory = GpuRecordsFactory()

  override val graphs: GpuGraphFactory = GpuGraphFactory()

  override val elementTables: GpuElementTableFactory = GpuElementTableFactory(this)

  /** Dictionary code of a string value (STRING columns hold codes). */
  def intern(s: String): Long = strings.synchronized {
    strings.getOrElseUpdate(s, Native.guard(Native.stringIntern(handle, s)))
  }

  private val sets = scala.collection.mutable.HashMap.empty[Seq[Long], String]

  /** Program name of the session literal set of `values` (CAPF_OP_IN_SET). */
  def literalSet(values: Seq[Long]): String = sets.synchronized {
    val key = values.distinct.sorted
    sets.getOrElseUpdate(key, "\u0001set:" + Native.sessionLiteralSet(handle, key.toArray))
  }

  private val maps = scala.collection.mutable.HashMap.empty[Seq[Any], (Long, Array[Long], String)]

  /** Program name of the session code map of string function `key` (CAPF_OP_STR_MAP,
    * GpuStringFunctions.apply): the function applied to every dictionary string
    * with the JVM's own String semantics, the results interned; extended in
    * place when the dictionary has grown since (the shim's twin of
    * table.py GpuSession.string_map). */
  def stringMap(key: Seq[Any]): Option[String] = maps.synchronized {
    val n = { val d = new Array[Long](2); Native.guard(Native.stringDigest(handle, d)); d(0) }
    if (n > GpuCypherSession.CodeMapMax) None  // a large dictionary: the caller's value map
    else maps.get(key) match {
      case Some((m, _, name)) if m >= n => Some(name)
      case prev =>
        val old = prev.map(_._2).getOrElse(Array.empty[Long])
        val codes = old ++ (old.length.toLong until n).map { c =>
          GpuStringFunctions(key, Native.stringLookup(handle, c)).map(intern).getOrElse(-1L)
        }
        val id = Native.guard(prev match {  // a grown map replaces its table in place (capf_session_code_map_extend)
          case Some((_, _, was)) => Native.sessionCodeMapExtend(handle, was.stripPrefix("\u0001map:").toInt, codes)
          case None => Native.sessionCodeMap(handle, codes)
        })
        val name = "\u0001map:" + id
        maps.update(key, (n, codes, name))
        Some(name)
    }
  }

  // ------------------------------------------------------------ table sources
  /** The one-row, zero-column table (RelationalCypherRecordsFactory.unit). */
  def unitTable(): GpuTable = GpuTable(Native.guard(Native.tableUnit(handle)))

  /** An empty table with the given (column, capf type) schema. */
  def emptyTable(columns: Seq[(String, Int)]): GpuTable =
    GpuTable(Native.guard(Native.tableEmpty(handle, columns.map(_._1).toArray, columns.map(_._2).toArray)))

  /** A table from host columns (the input side of CAPFElementTable.create,
    * CAPFTable.scala:76-83): direct buffers of 8 B (INT64 / FLOAT64 / STRING
    * codes) or 1 B (BOOL) per row, validity bytes or null. */
  def fromHost(columns: Seq[(String, Int, java.nio.ByteBuffer, java.nio.ByteBuffer)], nrows: Long): GpuTable =
    GpuTable(Native.guard(Native.tableFromHost(handle, columns.map(_._1).toArray, columns.map(_._2).toArray,
      columns.map(_._3).toArray, columns.map(_._4).toArray, nrows)))

  /** Relationship table of an edge-list file parsed on the GPU
    * (EdgeListDataSource.scala:56-92: rel ids = line ordinals). */
  def edgeList(path: String, sep: String = " ", comment: String = "#"): GpuTable =
    GpuTable(Native.guard(Native.edgeListRead(handle, path, sep, comment, "id", "source", "target")))

  /** Waits for every operation enqueued on the session's stream. */
  def sync(): Unit = Native.guard(Native.sessionSync(handle))

  override def close(): Unit = Native.guard(Native.sessionDestroy(handle))
}

object GpuCypherSession {

  /** String functions run over the whole dictionary (a code map) only while it
    * holds at most this many strings (table.py CODE_MAP_MAX). */
  final val CodeMapMax: Long = 1L << 16

  /** A session on one GPU (CAPFSession.local(), CAPFSession.scala:79): device 0
    * by default, the backend's own stream. */
  def local(device: Int = 0): GpuCypherSession = new GpuCypherSession(device, 0L)

  /** A session whose work is ordered on an existing HIP stream (e.g. one that
    * RCCL or another library also uses). */
  def onStream(device: Int, hipStream: Long): GpuCypherSession = new GpuCypherSession(device, hipStream)
}

/** RelationalCypherGraphFactory[GpuTable] (CAPFGraphFactory.scala:33-35): the
  * generic ScanGraph / UnionGraph / PrefixedGraph of okapi-relational over
  * GpuTable element tables. */
case class GpuGraphFactory()(implicit val session: GpuCypherSession)
  extends RelationalCypherGraphFactory[GpuTable] {
  override type Graph = RelationalCypherGraph[GpuTable]
}
