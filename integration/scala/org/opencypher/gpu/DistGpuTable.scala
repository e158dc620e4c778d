/*
 * DistGpuTable.scala — `Table[DistGpuTable]`: the okapi Table SPI over G ranks,
 * one JVM per GPU, each holding a shard as a GpuTable.  The JVM twin of
 * cypher-for-apache-flink_amd/dist_table.py::DistTable (the Python layer the
 * multi-process tests run): the same placements, operator rules, deferral and
 * count dispatch, with the exchange on the C-ABI's rank communicator
 * (capf_comm_*: RCCL over xGMI, ordered on the session stream).
 *
 * What it replaces: Flink repartitions the inputs of every join / groupBy /
 * distinct by a hash of the key (or broadcasts a small side) before the local
 * operator (flink-cypher/.../impl/table/FlinkTable.scala:123-196); SURVEY §8(e)
 * prescribes the same for the GPU node: graph hash-partitioned by node id,
 * frontier rows shuffled by join key, a global count an int64 all-reduce.
 *
 * Placements
 *   Hashed      rows spread over the ranks; `part` = columns whose equal values
 *               sit on one rank (the last shuffle's key and its aliases)
 *   Root        every row on rank 0 (ORDER BY results, global aggregates, unit)
 *   Replicated  every rank holds every row (a broadcast side; a count's result)
 * Rules: select / drop / filter / withColumns local; join local when
 * co-partitioned on a key pair, else the right side broadcast when
 * |right|·G < |left| (inner / left outer), else both sides shuffled; group with
 * keys shuffled by the keys, without keys two-phase (count / sum / min / max /
 * avg) or gathered to rank 0; distinct shuffled; orderBy / skip / limit on
 * rank 0.
 *
 * Deferral (node-partitioned graphs, DistGpuGraph.nodePartitioned): inner joins
 * between projections of the base shards and the filters / projections over
 * them are recorded; `group(∅, count(*))` — what the Aggregate operator calls
 * (RelationalOperator.scala:334-346 → Table.scala:158-159) — first looks at the
 * record: S_a ⋈ R1 ⋈ S_b ⋈ R2 ⋈ S_c (RelationalPlanner.scala:130-165) with
 * NOT(r1 = r2) runs capf_chain2_sharded_count_diag on the rank's in / out copies
 * plus ONE 8-byte all-reduce; anything that reads rows replays the record.
 */
package org.opencypher.gpu

import java.nio.{ByteBuffer, ByteOrder}

import org.opencypher.okapi.api.types.{CTInteger, CypherType}
import org.opencypher.okapi.api.value.CypherValue._
import org.opencypher.okapi.impl.exception.{IllegalStateException, NotImplementedException}
import org.opencypher.okapi.ir.api.expr._
import org.opencypher.okapi.relational.api.table.Table
import org.opencypher.okapi.relational.impl.planning._
import org.opencypher.okapi.relational.impl.table.RecordHeader

/** One rank's view of the job: its session, the communicator, rank and world
  * (capf_comm_init with the id rank 0 created). */
final class GpuRankContext(val session: GpuCypherSession, val comm: Long) extends AutoCloseable {
  val rank: Int = Native.guard(Native.commRank(comm))
  val world: Int = Native.guard(Native.commWorld(comm))
  private val s = session.handle
  private val scratchLongs = 4096
  private val scratch: Long = Native.guard(Native.sessionAlloc(s, 8L * scratchLongs * world))

  private def host(n: Int): ByteBuffer = ByteBuffer.allocateDirect(math.max(8 * n, 8)).order(ByteOrder.nativeOrder())

  /** In-place all-reduce of host int64 values (CAPF_COMM_SUM / CAPF_COMM_MAX) through the scratch slot. */
  def allReduce(vals: Array[Long], op: Int): Array[Long] = {
    require(vals.length <= scratchLongs, "too many values for one all-reduce")
    val b = host(vals.length)
    vals.zipWithIndex.foreach { case (v, i) => b.putLong(8 * i, v) }
    Native.guard(Native.sessionCopy(s, scratch, b, 8L * vals.length, 1))
    Native.guard(Native.commAllReduceI64(comm, scratch, vals.length, op))
    Native.guard(Native.sessionCopy(s, scratch, b, 8L * vals.length, 2))
    Array.tabulate(vals.length)(i => b.getLong(8 * i))
  }

  def allSum(v: Long): Long = allReduce(Array(v), Native.CommSum)(0)

  /** Every rank's `vals` (same length everywhere), rank-major. */
  def allGather(vals: Array[Long]): Array[Array[Long]] = {
    val n = vals.length
    require(n * world <= scratchLongs * world && n <= scratchLongs, "too many values for one all-gather")
    val b = host(n * world)
    vals.zipWithIndex.foreach { case (v, i) => b.putLong(8 * i, v) }
    val send = Native.guard(Native.sessionAlloc(s, 8L * math.max(n, 1)))
    try {
      Native.guard(Native.sessionCopy(s, send, b, 8L * n, 1))
      Native.guard(Native.commAllGatherBytes(comm, send, 8L * n, scratch))
      Native.guard(Native.sessionCopy(s, scratch, b, 8L * n * world, 2))
    } finally Native.guard(Native.sessionFree(s, send))
    Array.tabulate(world, n)((r, i) => b.getLong(8 * (r * n + i)))
  }

  // ------------------------------------------------------------------ rows
  /** Rows of `t` grouped by owner h(keys) (capf_table_hash_route) and the count per owner. */
  def route(t: GpuTable, keys: Seq[String]): (GpuTable, Array[Long]) = {
    val counts = new Array[Long](world)
    val h = Native.guard(Native.tableHashRoute(t.handle, keys.take(8).toArray, world, counts))
    (GpuTable(h)(session), counts)
  }

  def shuffle(t: GpuTable, keys: Seq[String]): GpuTable = {
    val (routed, counts) = route(t, keys)
    send(routed, counts, repeat = false)
  }

  /** The rows this rank owns of a table every rank holds in full (ingest sharding, no exchange). */
  def ownShare(t: GpuTable, keys: Seq[String]): GpuTable = {
    val (routed, counts) = route(t, keys)
    routed.skip(counts.take(rank).sum).limit(counts(rank)).cache()
  }

  def toRoot(t: GpuTable): GpuTable = {
    val n = t.size
    send(t, Array.tabulate(world)(p => if (p == 0) n else 0L), repeat = false)
  }

  def replicate(t: GpuTable): GpuTable = send(t, Array.fill(world)(t.size), repeat = true)

  /** The wire layout every rank agrees on in ONE max all-reduce (dist_table.py
    * GpuExchange._layout): per column the width of (value − base) — 3 / 4 where
    * the range over all ranks fits 24 / 32 bits — and a validity byte where
    * some rank has NULLs; STRING codes need equal dictionaries (digest check). */
  private def layout(t: GpuTable): (Array[String], Array[Int], Array[Int], Array[Long], Array[Int]) = {
    val cols = t.physicalColumns.toArray
    val types = cols.map(c => Native.guard(Native.tableColumnType(t.handle, c)))
    if (types.contains(Native.TypeList)) throw NotImplementedException("LIST columns are not moved between ranks")
    val k = cols.length
    val big = Long.MaxValue
    val has = cols.map(c => if (Native.guard(Native.tableHasNulls(t.handle, c))) 1L else 0L)
    val ranges = cols.zip(types).map { case (c, ty) =>
      if (ty == Native.TypeInt64 || ty == Native.TypeString) {
        val r = new Array[Long](3)
        Native.guard(Native.tableColumnRange(t.handle, c, r))
        if (r(2) > 0) (-r(0), r(1)) else (-big, -big)
      } else (-big, -big)
    }
    val check =
      if (!types.contains(Native.TypeString)) Array.empty[Long]
      else {
        val d = new Array[Long](2)
        Native.guard(Native.stringDigest(session.handle, d))
        Array(d(0), -d(0), d(1), if (d(1) == Long.MinValue) big else -d(1))
      }
    val got = allReduce(has ++ ranges.map(_._1) ++ ranges.map(_._2) ++ check, Native.CommMax)
    if (check.nonEmpty) {
      val c0 = 3 * k
      if (got(c0) != -got(c0 + 1) || (got(c0 + 2) != -got(c0 + 3) && check(2) != Long.MinValue))
        throw IllegalStateException("string dictionaries differ between ranks: STRING columns cannot move as codes")
    }
    val nullable = Array.tabulate(k)(j => if (got(j) != 0 && types(j) != Native.TypeNull) 1 else 0)
    val (width, base) = Array.tabulate(k) { j =>
      types(j) match {
        case Native.TypeNull => (0, 0L)
        case Native.TypeBool => (1, 0L)
        case Native.TypeInt64 | Native.TypeString =>
          val (gmin, gmax) = (-got(k + j), got(2 * k + j))
          if (gmax < gmin) (3, 0L)
          else if (gmax - gmin < (1L << 24)) (3, gmin)
          else if (gmax - gmin < (1L << 32)) (4, gmin)
          else (8, 0L)
        case _ => (8, 0L)
      }
    }.unzip
    (cols, types, width, base, nullable)
  }

  /** Rows [off_p, off_p + counts(p)) of `t` go to rank p (every row to every
    * rank when `repeat`); the rows this rank receives, in sender order, packed
    * on the GPU (capf_table_pack_rows) and moved by one all-to-all. */
  def send(t: GpuTable, counts: Array[Long], repeat: Boolean): GpuTable = {
    val (cols, types, width, base, nullable) = layout(t)
    val n = t.size
    val w = width.sum + nullable.sum
    val packed = Native.guard(Native.sessionAlloc(s, math.max(n * w, 1L)))
    val sendBuf = if (repeat) Native.guard(Native.sessionAlloc(s, math.max(n * w * world, 1L))) else packed
    try {
      val wb = Native.guard(Native.tablePackRows(t.handle, cols, width, base, nullable, packed))
      require(wb == w, s"packed row width $wb, expected $w")
      if (repeat) (0 until world).foreach(p => Native.guard(Native.sessionCopyDevice(s, sendBuf + p * n * w, packed, n * w)))
      val recvCounts = allGather(counts).map(_(rank))
      val m = recvCounts.sum
      val recv = Native.guard(Native.sessionAlloc(s, math.max(m * w, 1L)))
      try {
        if (w > 0) Native.guard(Native.commAllToAllBytes(comm, sendBuf, counts.map(_ * w), recv, recvCounts.map(_ * w)))
        GpuTable(Native.guard(Native.tableFromPackedRows(s, cols, types, width, base, nullable,
          if (m > 0 && w > 0) recv else 0L, m)))(session)
      } finally Native.guard(Native.sessionFree(s, recv))
    } finally {
      Native.guard(Native.sessionFree(s, packed))
      if (repeat) Native.guard(Native.sessionFree(s, sendBuf))
    }
  }

  override def close(): Unit = {
    Native.guard(Native.sessionFree(s, scratch))
    Native.guard(Native.commDestroy(comm))
  }
}

object GpuRankContext {
  /** Rank 0 calls this and hands the bytes to every rank out of band. */
  def uniqueId(): Array[Byte] = Native.guard(Native.commUniqueId())

  def apply(session: GpuCypherSession, world: Int, rank: Int, id: Array[Byte]): GpuRankContext =
    new GpuRankContext(session, Native.guard(Native.commInit(session.handle, world, rank, id)))
}

/** Graph-level facts of a node-partitioned base shard (dist_table.py Prov). */
final case class ShardInfo(kind: String, graph: AnyRef, idCol: String, srcCol: String, dstCol: String,
                           complete: Boolean, count: () => Long)

final case class Prov(info: ShardInfo, cols: Map[String, String]) {
  def renamed(pairs: Seq[(String, String)]): Option[Prov] = {
    val c = pairs.collect { case (from, to) if cols.contains(from) => to -> cols(from) }.toMap
    if (c.isEmpty) None else Some(copy(cols = c))
  }
  def without(names: Set[String]): Option[Prov] = {
    val c = cols.filterNot { case (k, _) => names(k) }
    if (c.isEmpty) None else Some(copy(cols = c))
  }
}

sealed trait Placement
case object Hashed extends Placement
case object Root extends Placement
case object Replicated extends Placement

/** A recorded operator of a deferred table, replayed when rows are read. */
sealed trait Deferred
final case class DJoin(l: DistGpuTable, r: DistGpuTable, jt: JoinType, cols: Seq[(String, String)]) extends Deferred
final case class DSelect(t: DistGpuTable, cols: Seq[(String, String)]) extends Deferred
final case class DFilter(t: DistGpuTable, e: Expr, h: RecordHeader, p: CypherMap) extends Deferred
final case class DWithColumns(t: DistGpuTable, cols: Seq[(Expr, String)], h: RecordHeader, p: CypherMap)
  extends Deferred
final case class DDrop(t: DistGpuTable, cols: Seq[String]) extends Deferred
final case class DHostRows(names: Seq[String], values: Seq[Long]) extends Deferred

final class DistGpuTable private[gpu] (
  private var localT: GpuTable,
  private var partCols: Set[String],
  private var place: Placement,
  val prov: Option[Prov],
  private var deferred: Option[Deferred],
  deferredCols: Seq[String]
)(implicit val ctx: GpuRankContext) extends Table[DistGpuTable] {

  private implicit val session: GpuCypherSession = ctx.session

  private def force(): Unit = deferred.foreach { d =>
    val out = d match {
      case DHostRows(names, values) =>
        val cols = names.zip(values).map { case (nm, v) =>
          val b = ByteBuffer.allocateDirect(8).order(ByteOrder.nativeOrder())
          b.putLong(0, v)
          (nm, Native.TypeInt64, b, null: ByteBuffer)
        }
        new DistGpuTable(session.fromHost(cols, 1), Set.empty, Replicated, None, None, Seq.empty)
      case DJoin(l, r, jt, cols) => l.joinEager(r, jt, cols)
      case DSelect(t, cols) => t.selectEager(cols)
      case DFilter(t, e, h, p) => t.wrap(t.local.filter(e)(h, p), t.part)
      case DWithColumns(t, cols, h, p) => t.withColumnsEager(cols, h, p)
      case DDrop(t, cols) => t.dropEager(cols)
    }
    localT = out.local
    partCols = out.part
    place = out.placement
    deferred = None
  }

  private[gpu] def deferredOp: Option[Deferred] = deferred

  def local: GpuTable = { force(); localT }
  def part: Set[String] = { force(); partCols }
  def placement: Placement = { force(); place }

  private def rank0 = ctx.rank == 0
  private[gpu] def wrap(t: GpuTable, p: Set[String] = Set.empty, pl: Placement = null,
                        pv: Option[Prov] = None): DistGpuTable =
    new DistGpuTable(t, if ((if (pl == null) placement else pl) == Hashed) p else Set.empty,
      if (pl == null) placement else pl, pv, None, Seq.empty)
  private def defer(d: Deferred, cols: Seq[String]): DistGpuTable =
    new DistGpuTable(null, Set.empty, Hashed, None, Some(d), cols)
  private def deferrable: Boolean = deferred.isDefined || prov.isDefined
  private def rooted: GpuTable = placement match {
    case Root => local
    case Replicated => if (rank0) local else local.limit(0)
    case Hashed => ctx.toRoot(local)
  }

  // ---------------------------------------------------------------- CypherTable
  override def physicalColumns: Seq[String] =                                           // CypherTable.scala:48
    if (deferred.isDefined) deferredCols else local.physicalColumns

  override def columnType: Map[String, CypherType] = local.columnType                    // :58

  /** All rows on every rank (the result a driver reads back). */
  override def rows: Iterator[String => CypherValue] =                                 // :63
    if (placement == Replicated) local.rows else ctx.replicate(rooted).rows

  override def size: Long = if (placement == Replicated) local.size else ctx.allSum(local.size) // :68

  // ---------------------------------------------------------------- Table[T]
  override def cache(): DistGpuTable =                                                   // Table.scala:52
    if (deferred.isDefined) this else wrap(local.cache(), part, pv = prov)

  override def select(col: (String, String), cols: (String, String)*): DistGpuTable = {  // :71
    val all = col +: cols
    if (deferred.isDefined) defer(DSelect(this, all), all.map(_._2)) else selectEager(all)
  }

  private[gpu] def selectEager(all: Seq[(String, String)]): DistGpuTable =
    wrap(local.select(all.head, all.tail: _*), all.collect { case (c, a) if part(c) => a }.toSet,
      pv = prov.flatMap(_.renamed(all)))

  override def filter(expr: Expr)(implicit header: RecordHeader, parameters: CypherMap): DistGpuTable = // :81
    if (deferred.isDefined) defer(DFilter(this, expr, header, parameters), deferredCols)
    else wrap(local.filter(expr), part)

  override def drop(cols: String*): DistGpuTable =                                       // :89
    if (deferred.isDefined) defer(DDrop(this, cols), deferredCols.filterNot(cols.contains)) else dropEager(cols)

  private[gpu] def dropEager(cols: Seq[String]): DistGpuTable =
    wrap(local.drop(cols: _*), part -- cols, pv = prov.flatMap(_.without(cols.toSet)))

  override def withColumns(columns: (Expr, String)*)                                     // :170
    (implicit header: RecordHeader, parameters: CypherMap): DistGpuTable =
    if (columns.exists(_._1.isInstanceOf[Explode]))  // UNWIND multiplies each rank's rows in place
      wrap(local.withColumns(columns: _*), part -- columns.map(_._2))
    else if (deferred.isDefined)
      defer(DWithColumns(this, columns, header, parameters), (deferredCols ++ columns.map(_._2)).distinct)
    else withColumnsEager(columns, header, parameters)

  private[gpu] def withColumnsEager(columns: Seq[(Expr, String)], h: RecordHeader, p: CypherMap): DistGpuTable = {
    val written = columns.map(_._2).toSet
    wrap(local.withColumns(columns: _*)(h, p), part -- written, pv = prov.flatMap(_.without(written)))
  }

  override def unionAll(other: DistGpuTable): DistGpuTable = {                           // :107
    if (placement == Replicated || other.placement == Replicated)
      throw IllegalStateException("union of a broadcast table")
    if (placement == Root && other.placement == Root) wrap(local.unionAll(other.local), pl = Root)
    else {  // rank 0's root rows join its shard: the union is hash placed, unpartitioned
      val p = if (placement == Hashed && other.placement == Hashed) part & other.part else Set.empty[String]
      wrap(local.unionAll(other.local), p, Hashed)
    }
  }

  override def join(other: DistGpuTable, joinType: JoinType, joinCols: (String, String)*): DistGpuTable = // :99
    if (session.deferJoins && joinType == InnerJoin && deferrable && other.deferrable)
      defer(DJoin(this, other, joinType, joinCols), physicalColumns ++ other.physicalColumns)
    else joinEager(other, joinType, joinCols)

  private[gpu] def joinEager(other: DistGpuTable, jt: JoinType, cols: Seq[(String, String)]): DistGpuTable = {
    def localJoin(l: GpuTable, r: GpuTable, p: Set[String], pl: Placement) =
      wrap(l.join(r, jt, cols: _*), p, pl)
    if (jt == CrossJoin) return localJoin(local, ctx.replicate(other.rooted), part, placement)
    if (placement == Root && other.placement == Root) return localJoin(local, other.local, Set.empty, Root)
    if (other.placement == Replicated && (jt == InnerJoin || jt == LeftOuterJoin))
      return localJoin(local, other.local, part, placement)
    val colocated = placement == Hashed && other.placement == Hashed &&
      cols.exists { case (l, r) => part(l) && other.part(r) }
    if (colocated) {
      val keys = cols.collect { case (l, r) if part(l) && other.part(r) => Set(l, r) }.flatten.toSet
      return localJoin(local, other.local, part ++ other.part ++ keys, Hashed)
    }
    val (ln, rn) = (size, other.size)
    if ((jt == InnerJoin || jt == LeftOuterJoin) && rn * ctx.world < ln && placement == Hashed)
      return localJoin(local, ctx.replicate(other.rooted), part, Hashed)
    val (l0, r0) = cols.head
    val lt = if (placement == Hashed && part(l0)) local else ctx.shuffle(movedRows, Seq(l0))
    val rt = if (other.placement == Hashed && other.part(r0)) other.local else ctx.shuffle(other.movedRows, Seq(r0))
    localJoin(lt, rt, Set(l0, r0), Hashed)
  }

  /** This rank's share of the rows for a shuffle (a replicated table's rows once, on rank 0). */
  private def movedRows: GpuTable = placement match {
    case Replicated => if (rank0) local else local.limit(0)
    case _ => local
  }

  override def orderBy(sortItems: (Expr, Order)*)                                       // :115
    (implicit header: RecordHeader, parameters: CypherMap): DistGpuTable =
    wrap(rooted.orderBy(sortItems: _*), pl = Root)

  override def skip(n: Long): DistGpuTable = wrap(rooted.skip(n), pl = Root)            // :123

  override def limit(n: Long): DistGpuTable = wrap(rooted.limit(n), pl = Root)          // :131

  override def distinct: DistGpuTable = distinct(physicalColumns: _*)                   // :138

  override def distinct(cols: String*): DistGpuTable = {                                // :146
    val keys = if (cols.isEmpty) physicalColumns else cols
    if (placement == Root || keys.isEmpty) wrap(rooted.distinct(cols: _*), pl = Root)
    else if (placement == Hashed && keys.exists(part)) wrap(local.distinct(cols: _*), part & keys.toSet)
    else wrap(ctx.shuffle(movedRows, keys).distinct(cols: _*), if (keys.size == 1) keys.toSet else Set.empty, Hashed)
  }

  override def group(by: Set[Var], aggregations: Map[String, Aggregator])               // :158-159
    (implicit header: RecordHeader, parameters: CypherMap): DistGpuTable = {
    val sharded =
      if (deferred.isDefined && by.isEmpty && aggregations.nonEmpty && aggregations.values.forall(_ == CountStar))
        DistGpuTable.shardedTwoHop(this)
      else None
    sharded match {
      case Some(count) =>
        // every rank holds the all-reduced count: one replicated row, kept on the
        // host until an operator needs it on the device
        val names = aggregations.keys.toSeq
        new DistGpuTable(null, Set.empty, Replicated, None, Some(DHostRows(names, names.map(_ => count))), names)
      case None => groupRows(by, aggregations)
    }
  }

  private def groupRows(by: Set[Var], aggregations: Map[String, Aggregator])
    (implicit header: RecordHeader, parameters: CypherMap): DistGpuTable = {
    val keys = by.toSeq.flatMap(v => header.ownedBy(v).toSeq.map(header.column)).distinct
      .filter(physicalColumns.contains)
    if (placement == Root) {
      val out = local.group(by, aggregations)
      wrap(if (keys.isEmpty && !rank0) out.limit(0) else out, pl = Root)
    } else if (keys.nonEmpty) {
      if (placement == Hashed && keys.exists(part)) wrap(local.group(by, aggregations), part & keys.toSet)
      else wrap(ctx.shuffle(movedRows, keys).group(by, aggregations), if (keys.size == 1) keys.toSet else Set.empty,
        Hashed)
    } else if (placement == Replicated) {
      wrap(if (rank0) local.group(by, aggregations) else local.group(by, aggregations).limit(0), pl = Root)
    } else globalAggregate(aggregations)
  }

  /** Two phases for count / sum / min / max / avg (avg = Σ sum / Σ count, a
    * FLOAT); every other aggregator over the rows gathered to rank 0. */
  private def globalAggregate(aggs: Map[String, Aggregator])
    (implicit header: RecordHeader, parameters: CypherMap): DistGpuTable = {
    val decomposable = aggs.values.forall {
      case CountStar | Sum(_) | Min(_) | Max(_) | Avg(_) => true
      case Count(_, distinct) => !distinct
      case _ => false
    }
    if (!decomposable) {
      val out = ctx.toRoot(local).group(Set.empty, aggs)
      return wrap(if (rank0) out else out.limit(0), pl = Root)
    }
    val names = aggs.keys.toSeq
    def v(c: String, t: CypherType = CTInteger) = Var(c)(t)
    val partial = scala.collection.mutable.LinkedHashMap.empty[String, Aggregator]
    val fin = scala.collection.mutable.LinkedHashMap.empty[String, Aggregator]
    val avgs = scala.collection.mutable.ArrayBuffer.empty[(String, String, String)]
    names.zipWithIndex.foreach { case (name, i) =>
      val p = s"__dist_p$i"
      aggs(name) match {
        case Avg(e) =>
          partial(p) = Sum(e)
          partial(s"__dist_c$i") = Count(e, distinct = false)
          fin(s"__dist_s$i") = Sum(v(p))
          fin(s"__dist_n$i") = Sum(v(s"__dist_c$i"))
          avgs += ((name, s"__dist_s$i", s"__dist_n$i"))
        case Min(_) => partial(p) = aggs(name); fin(name) = Min(v(p))
        case Max(_) => partial(p) = aggs(name); fin(name) = Max(v(p))
        case other => partial(p) = other; fin(name) = Sum(v(p))
      }
    }
    val loc = local.group(Set.empty, partial.toMap)
    val rows = ctx.toRoot(loc)
    val h2 = RecordHeader(partial.keys.map(p => (v(p): Expr) -> p).toMap)
    var out = rows.group(Set.empty, fin.toMap)(h2, CypherMap.empty)
    if (avgs.nonEmpty) {
      val h3 = RecordHeader(out.physicalColumns.map(c => (v(c): Expr) -> c).toMap)
      out = out.withColumns(avgs.map { case (name, s, n) => (Divide(ToFloat(v(s)), v(n)): Expr, name) }: _*)(h3,
        CypherMap.empty)
    }
    val sel = names.map(n => (n, n))
    out = out.select(sel.head, sel.tail: _*)
    wrap(if (rank0) out else out.limit(0), pl = Root)
  }

  override def show(rows: Int): Unit = { val r = rooted; if (rank0) r.show(rows) }       // :177
}

object DistGpuTable {
  /** A table every rank holds in full (rank 0 keeps the rows). */
  def fromFull(t: GpuTable)(implicit ctx: GpuRankContext): DistGpuTable =
    new DistGpuTable(if (ctx.rank == 0) t else t.limit(0), Set.empty, Root, None, None, Seq.empty)

  /** A table every rank holds in full, hash-partitioned by `key` at ingest (no exchange). */
  def shard(t: GpuTable, key: String, prov: Option[Prov] = None)(implicit ctx: GpuRankContext): DistGpuTable =
    new DistGpuTable(ctx.ownShare(t, Seq(key)), Set(key), Hashed, prov, None, Seq.empty)

  def unit()(implicit ctx: GpuRankContext): DistGpuTable = fromFull(ctx.session.unitTable())

  private final class NoMatch extends RuntimeException

  /** Column → (leaf, base column) of a deferred join tree; join keys into eqs,
    * NOT(r_i = r_j) filters into neqs (dist_table.py _tree_refs). */
  private def treeRefs(t: DistGpuTable, leaves: scala.collection.mutable.ArrayBuffer[Prov],
                       eqs: scala.collection.mutable.ArrayBuffer[((Int, String), (Int, String))],
                       neqs: scala.collection.mutable.ArrayBuffer[((Int, String), (Int, String))])
  : Map[String, (Int, String)] = t.deferredOp match {
    case None =>
      val p = t.prov.getOrElse(throw new NoMatch)
      leaves += p
      p.cols.map { case (c, b) => c -> (leaves.size - 1, b) }
    case Some(DHostRows(_, _)) => throw new NoMatch
    case Some(DJoin(l, r, _, cols)) =>
      val lr = treeRefs(l, leaves, eqs, neqs)
      val rr = treeRefs(r, leaves, eqs, neqs)
      cols.foreach { case (x, y) =>
        if (!lr.contains(x) || !rr.contains(y)) throw new NoMatch
        eqs += ((lr(x), rr(y)))
      }
      lr ++ rr
    case Some(DSelect(c, cols)) =>
      val refs = treeRefs(c, leaves, eqs, neqs)
      cols.collect { case (x, a) if refs.contains(x) => a -> refs(x) }.toMap
    case Some(DDrop(c, cols)) => treeRefs(c, leaves, eqs, neqs) -- cols
    case Some(DWithColumns(c, cols, _, _)) => treeRefs(c, leaves, eqs, neqs) -- cols.map(_._2)
    case Some(DFilter(c, e, h, _)) =>
      val refs = treeRefs(c, leaves, eqs, neqs)
      val terms = e match {
        case Ands(xs) => xs.toSeq
        case other => Seq(other)
      }
      terms.foreach {
        case Not(Equals(a, b)) =>  // relationship uniqueness (CypherParser.scala:72)
          val (x, y) = (h.column(a), h.column(b))
          if (!refs.contains(x) || !refs.contains(y)) throw new NoMatch
          neqs += ((refs(x), refs(y)))
        case _ => throw new NoMatch
      }
      refs
  }

  /** count(*) of the 2-hop chain over a node-partitioned graph: this rank's
    * partial + ONE all-reduce (the rel shard's `count`), or None when the
    * deferred record is not S_a ⋈ R1 ⋈ S_b ⋈ R2 ⋈ S_c with NOT(r1 = r2). */
  private[gpu] def shardedTwoHop(t: DistGpuTable): Option[Long] = {
    val leaves = scala.collection.mutable.ArrayBuffer.empty[Prov]
    val eqs = scala.collection.mutable.ArrayBuffer.empty[((Int, String), (Int, String))]
    val neqs = scala.collection.mutable.ArrayBuffer.empty[((Int, String), (Int, String))]
    try treeRefs(t, leaves, eqs, neqs) catch { case _: NoMatch => return None }
    val rels = leaves.indices.filter(i => leaves(i).info.kind == "rel")
    val nodes = leaves.indices.filter(i => leaves(i).info.kind == "node")
    if (rels.size != 2 || nodes.size != 3 || eqs.size != 4 || neqs.size != 1) return None
    val info = leaves(rels(0)).info
    if (!(leaves(rels(1)).info eq info) || !nodes.forall(i => leaves(i).info.complete)) return None
    if (nodes.exists(i => !(leaves(i).info.graph eq info.graph))) return None
    val ends = scala.collection.mutable.HashMap.empty[(Int, String), Int]
    for ((a, b) <- eqs) {
      val (x, y) = if (leaves(a._1).info.kind == "rel") (b, a) else (a, b)
      if (leaves(x._1).info.kind != "node" || leaves(y._1).info.kind != "rel" || x._2 != leaves(x._1).info.idCol)
        return None
      val side = if (y._2 == info.srcCol) "src" else if (y._2 == info.dstCol) "dst" else return None
      if (ends.contains((y._1, side))) return None
      ends((y._1, side)) = x._1
    }
    val (x, y) = neqs.head
    if (Set(x._1, y._1) != rels.toSet || x._2 != info.idCol || y._2 != info.idCol) return None
    val (r1, r2) = if (ends((rels(0), "dst")) == ends((rels(1), "src"))) (rels(0), rels(1)) else (rels(1), rels(0))
    val b = ends((r1, "dst"))
    if (ends((r2, "src")) != b || Set(ends((r1, "src")), b, ends((r2, "dst"))).size != 3) return None
    Some(info.count())
  }

  /** The node-partitioned layout of SURVEY §8(e) for the 2-hop count over a
    * graph of one node table (ids exactly [lo, lo + n)) and one rel table:
    * relational shards (nodes by h(id), rels by h(source)) with provenance,
    * plus this rank's in / out copies (capf_table_node_partition_diag) whose
    * count runs as capf_chain2_sharded_count_diag + one all-reduce.  Rel ids
    * must be unique and endpoints non-NULL (else the plain shards are returned:
    * Σ in·out − self-loops equals NOT(r1 = r2) only for unique ids). */
  def nodePartitioned(nodes: GpuTable, nodeId: String, rels: GpuTable, relId: String, src: String, dst: String)
    (implicit ctx: GpuRankContext): (DistGpuTable, DistGpuTable) = {
    val s = ctx.session
    def range(t: GpuTable, c: String) = { val r = new Array[Long](3); Native.guard(Native.tableColumnRange(t.handle, c, r)); r }
    val Array(lo, hi, n) = range(nodes, nodeId)
    val m = rels.size
    val ok = n > 0 && hi - lo + 1 == n && nodes.size == n &&
      Seq(src, dst).forall { c => val r = range(rels, c); r(0) >= lo && r(1) <= hi && r(2) == m } &&
      range(rels, relId)(2) == m && rels.select((relId, relId)).distinct.size == m
    if (!ok) return (shard(nodes, nodeId), shard(rels, src))
    val nd = new Array[Long](1)
    val out = GpuTable(Native.guard(Native.tableNodePartitionDiag(rels.handle, src, dst, lo, n, ctx.world, ctx.rank,
      nd)))(s).compact(3)
    val in = GpuTable(Native.guard(Native.tableNodePartition(rels.handle, dst, lo, n, ctx.world, ctx.rank)))(s)
      .compact(3)
    val slot = Native.guard(Native.sessionAlloc(s.handle, 8))
    val count = () => {
      Native.guard(Native.chain2ShardedCountDiag(s.handle, in.handle, dst, out.handle, src, dst, nd(0),
        Array.empty[Long], lo, n, ctx.world, ctx.rank, slot))
      Native.guard(Native.commAllReduceI64(ctx.comm, slot, 1, Native.CommSum))  // ONE 8-byte all-reduce
      val b = ByteBuffer.allocateDirect(8).order(ByteOrder.nativeOrder())
      Native.guard(Native.sessionCopy(s.handle, slot, b, 8, 2))
      b.getLong(0)
    }
    val graph = new Object
    val nodeInfo = ShardInfo("node", graph, nodeId, "", "", complete = true, () => 0L)
    val relInfo = ShardInfo("rel", graph, relId, src, dst, complete = false, count)
    s.deferJoins = true
    (shard(nodes, nodeId, Some(Prov(nodeInfo, nodes.physicalColumns.map(c => c -> c).toMap))),
      shard(rels, src, Some(Prov(relInfo, rels.physicalColumns.map(c => c -> c).toMap))))
  }
}
