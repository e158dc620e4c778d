/*
 * Native.scala — the JVM declarations of integration/jni/capf_jni.cpp, one
 * @native method per entry point of include/capf_gpu.h, plus the exception
 * mapping.  Source a maintainer adds next to flink-cypher (no JVM in this
 * image: it is not compiled here; the C++ half is type-checked by
 * tests/test_jni_shim.py, which also checks that every method below has its
 * JNI symbol in capf_jni.cpp).
 */
package org.opencypher.gpu

import java.nio.ByteBuffer

import org.opencypher.okapi.impl.exception.{IllegalArgumentException, IllegalStateException, NotImplementedException}

/** Thrown by the JNI layer; `kind` is the capf status (CAPF_ERR_*). */
final class CapfNativeException(val kind: Int, msg: String) extends RuntimeException(msg)

/** Postfix expression program (capf_expr): what GpuExprMapper lowers an okapi Expr to. */
final class Program(val ops: Array[Int], val iargs: Array[Long], val fargs: Array[Double],
                    val names: Array[String])

object Program {
  val empty: Program = new Program(Array.empty, Array.empty, Array.empty, Array.empty)
}

object Native {
  System.loadLibrary("capf_jni") // libcapf_jni.so, linked against libcapf_gpu.so

  // status codes and enums of include/capf_gpu.h
  final val ErrIllegalArgument = -1
  final val ErrNotImplemented = -2
  final val ErrInternal = -3
  final val ErrHip = -4
  final val ErrOom = -5

  final val TypeNull = 0
  final val TypeInt64 = 1
  final val TypeFloat64 = 2
  final val TypeBool = 3
  final val TypeString = 4
  final val TypeList = 5

  final val JoinInner = 0
  final val JoinLeftOuter = 1
  final val JoinRightOuter = 2
  final val JoinFullOuter = 3
  final val JoinCross = 4

  final val AggCountStar = 0
  final val AggCount = 1
  final val AggSum = 2
  final val AggMin = 3
  final val AggMax = 4
  final val AggAvg = 5
  final val AggCollect = 6
  final val AggStDev = 7            // stddevSamp (FlinkSQLExprMapper.scala:223)
  final val AggStDevPop = 8         // stddevPop (:224)
  final val AggPercentileCont = 9   // PercentileUdafs.scala:83-96 (Spark backend semantics)
  final val AggPercentileDisc = 10  // PercentileUdafs.scala:59-81

  /** Runs a native call, rethrowing its failure as the okapi exception of that kind
    * (okapi-api/.../impl/exception/InternalException.scala:36-65). */
  def guard[A](body: => A): A =
    try body
    catch {
      case e: CapfNativeException =>
        e.kind match {
          case ErrIllegalArgument => throw IllegalArgumentException("a valid GPU table operation", e.getMessage)
          case ErrNotImplemented => throw NotImplementedException(e.getMessage)
          case _ => throw IllegalStateException(e.getMessage, Some(e))
        }
    }

  // errors / ABI
  @native def lastError(): String
  @native def lastErrorKind(): Int
  @native def abiVersion(): Int

  // session (RelationalCypherSession.scala:63-111)
  @native def sessionCreate(device: Int, hipStream: Long): Long
  @native def sessionDestroy(session: Long): Unit
  @native def sessionSync(session: Long): Unit
  @native def sessionSetProfiling(session: Long, on: Boolean): Unit
  @native def sessionResetProfile(session: Long): Unit
  @native def sessionProfileCount(session: Long): Int
  @native def sessionProfileEntry(session: Long, i: Int, launchesOut: Array[Long], msBytesOut: Array[Double]): String
  @native def sessionLastPlan(session: Long): String
  @native def stringIntern(session: Long, s: String): Long
  @native def stringLookup(session: Long, code: Long): String
  @native def stringDigest(session: Long, out: Array[Long]): Unit

  // construction (CAPFTable.scala:76-83, CAPFRecords.scala:47-100, RelationalCypherRecords.scala:43-54)
  @native def tableFromHost(session: Long, names: Array[String], types: Array[Int], data: Array[ByteBuffer],
                            valid: Array[ByteBuffer], nrows: Long): Long
  @native def tableFromDevice(session: Long, names: Array[String], types: Array[Int], data: Array[Long],
                              valid: Array[Long], nrows: Long, copy: Boolean): Long
  @native def tableUnit(session: Long): Long
  @native def tableEmpty(session: Long, names: Array[String], types: Array[Int]): Long
  @native def tableRetain(table: Long): Unit
  @native def tableRelease(table: Long): Unit

  // CypherTable (CypherTable.scala:41-70)
  @native def tableColumns(table: Long): Array[String]
  @native def tableNumColumns(table: Long): Int
  @native def tableColumnName(table: Long, i: Int): String
  @native def tableColumnType(table: Long, col: String): Int
  @native def tableSize(table: Long): Long
  @native def tableCountAsync(table: Long, dCount: Long): Unit
  @native def tableDownload(table: Long, col: String, values: ByteBuffer, valid: ByteBuffer): Unit
  @native def tableListInfo(table: Long, col: String, nValuesOut: Array[Long]): Int
  @native def tableDownloadList(table: Long, col: String, offsets: ByteBuffer, values: ByteBuffer,
                                valid: ByteBuffer): Unit
  @native def tableDeviceColumn(table: Long, col: String, out: Array[Long]): Unit
  @native def tableCompact(table: Long): Long
  @native def tableCompactWidth(table: Long, width: Int): Long
  @native def tableColumnEncoding(table: Long, col: String, baseOut: Array[Long]): Int

  // Table[T] (Table.scala:43-178)
  @native def tableCache(table: Long): Long
  @native def tableMaterialize(table: Long): Unit
  @native def tableSelect(table: Long, cols: Array[String], aliases: Array[String]): Long
  @native def tableFilter(table: Long, pred: Program): Long
  @native def tableDrop(table: Long, cols: Array[String]): Long
  @native def tableJoin(l: Long, r: Long, joinType: Int, lcols: Array[String], rcols: Array[String]): Long
  @native def tableUnionAll(l: Long, r: Long): Long
  @native def tableOrderBy(table: Long, keys: Array[Program], descending: Array[Boolean]): Long
  @native def tableSkip(table: Long, n: Long): Long
  @native def tableLimit(table: Long, n: Long): Long
  @native def tableDistinct(table: Long): Long
  @native def tableDistinctCols(table: Long, cols: Array[String]): Long
  @native def tableGroup(table: Long, by: Array[String], kinds: Array[Int], args: Array[Program],
                         distinct: Array[Boolean], names: Array[String]): Long
  @native def tableGroupEx(table: Long, by: Array[String], kinds: Array[Int], args: Array[Program],
                           distinct: Array[Boolean], params: Array[Double], names: Array[String]): Long
  @native def tableWithColumns(table: Long, exprs: Array[Program], names: Array[String]): Long
  // UNWIND: withColumns(Explode(list) as item) (RelationalPlanner.scala:99-101)
  @native def tableExplodeValues(table: Long, name: String, elemType: Int, n: Long, values: java.nio.ByteBuffer,
                                 valid: java.nio.ByteBuffer): Long
  @native def tableExplodeList(table: Long, listCol: String, name: String): Long
  // a LIST property column (CTList) from direct buffers: offsets, element values, list validity
  @native def tableAddList(table: Long, name: String, elemType: Int, offsets: java.nio.ByteBuffer,
                           values: java.nio.ByteBuffer, valid: java.nio.ByteBuffer): Long
  @native def tableNameList(table: Long, cols: Array[String], kinds: Array[Int], codes: Array[Long], name: String): Long
  @native def tableListColumns(table: Long, cols: Array[String], name: String): Long
  @native def tableShow(table: Long, rows: Int): Unit

  // graph inputs (EdgeListDataSource.scala:56-92; synthetic R-MAT / node ranges)
  @native def rmatRelTable(session: Long, scale: Int, seed: Long, tA: Int, tAB: Int, tABC: Int, first: Long,
                           count: Long, idBase: Long, idCol: String, srcCol: String, dstCol: String): Long
  @native def rangeNodeTable(session: Long, base: Long, n: Long, seed: Long, idCol: String, labelCol: String): Long
  @native def edgeListParse(session: Long, bytes: ByteBuffer, nbytes: Long, sep: String, comment: String,
                            idCol: String, srcCol: String, dstCol: String): Long
  @native def edgeListRead(session: Long, path: String, sep: String, comment: String, idCol: String,
                           srcCol: String, dstCol: String): Long

  // fused var-length reach (VarLengthExpandPlanner.scala:82-259 → Distinct → Aggregate)
  @native def varLengthReach(session: Long, rels: Long, srcCol: String, dstCol: String, sources: Long,
                             sourceId: String, targets: Long, targetId: String, lower: Int, upper: Int,
                             outSource: String, outReach: String): Long

  // multi-GPU building blocks (one JVM per GPU; the caller all-reduces the device partials)
  @native def tableNodePartition(table: Long, keyCol: String, nodeBase: Long, nNodes: Long, parts: Int,
                                 part: Int): Long
  @native def chain2ShardedCount(session: Long, inCopy: Long, inDst: String, outCopy: Long, outSrc: String,
                                 outDst: String, nodeBase: Long, nNodes: Long, parts: Int, part: Int,
                                 dPartial: Long): Unit
  @native def tableNodePartitionDiag(table: Long, srcCol: String, dstCol: String, nodeBase: Long, nNodes: Long,
                                     parts: Int, part: Int, nDiagOut: Array[Long]): Long
  @native def chain2ShardedCountDiag(session: Long, inCopy: Long, inDst: String, outCopy: Long, outSrc: String,
                                     outDst: String, nDiag: Long, hotIds: Array[Long], nodeBase: Long,
                                     nNodes: Long, parts: Int, part: Int, dPartial: Long): Unit
  @native def triangleCountPart(session: Long, rels: Long, srcCol: String, dstCol: String, nodeBase: Long,
                                nNodes: Long, parts: Int, part: Int, dCount: Long): Unit
  @native def chain2HistLen(nNodes: Long): Long
  @native def chain2LocalHists(session: Long, rels: Long, srcCol: String, dstCol: String, nodeBase: Long,
                               nNodes: Long, dIn: Long, dOut: Long): Long
  @native def dotU32(session: Long, dA: Long, dB: Long, n: Long): Long
  // FS graph source: all-LONG CSV tables (FSGraphSource.scala:80-84) parsed on the GPU
  @native def csvReadLongs(session: Long, path: String, sep: String, names: Array[String]): Long
  @native def csvParseLongs(session: Long, bytes: java.nio.ByteBuffer, nBytes: Long, sep: String,
                            names: Array[String]): Long
  // distributed Table layer (dist_table.py): rows grouped by owner h(keys), counts per owner
  @native def tableHashRoute(table: Long, keys: Array[String], parts: Int, countsOut: Array[Long]): Long
  @native def tableDownloadDevice(table: Long, col: String, dValues: Long, dValid: Long): Unit
  @native def tableHasNulls(table: Long, col: String): Boolean
  @native def tableColumnRange(table: Long, col: String, out: Array[Long]): Unit
  @native def tablePackRows(table: Long, cols: Array[String], width: Array[Int], base: Array[Long],
                            nullable: Array[Int], dOut: Long): Int
  @native def tableFromPackedRows(session: Long, names: Array[String], types: Array[Int], width: Array[Int],
                                  base: Array[Long], nullable: Array[Int], dRows: Long, nrows: Long): Long

  // rank communicator (RCCL over xGMI, capf_comm_*) and session device buffers
  final val CommSum = 0
  final val CommMax = 2
  @native def commUniqueId(): Array[Byte]
  @native def commInit(session: Long, world: Int, rank: Int, id: Array[Byte]): Long
  @native def commDestroy(comm: Long): Unit
  @native def commRank(comm: Long): Int
  @native def commWorld(comm: Long): Int
  @native def commAllReduceI64(comm: Long, dBuf: Long, n: Long, op: Int): Unit
  @native def commAllGatherBytes(comm: Long, dSend: Long, bytes: Long, dRecv: Long): Unit
  @native def commAllToAllBytes(comm: Long, dSend: Long, sendBytes: Array[Long], dRecv: Long,
                                recvBytes: Array[Long]): Unit
  @native def sessionAlloc(session: Long, bytes: Long): Long
  @native def sessionFree(session: Long, d: Long): Unit
  @native def sessionCopy(session: Long, d: Long, host: ByteBuffer, bytes: Long, kind: Int): Unit
  @native def sessionCopyDevice(session: Long, dst: Long, src: Long, bytes: Long): Unit
  @native def sessionLiteralSet(session: Long, values: Array[Long]): Int
  @native def sessionCodeMap(session: Long, codes: Array[Long]): Int
  @native def sessionCodeMapExtend(session: Long, mapId: Int, codes: Array[Long]): Int
  @native def sessionValueMap(session: Long, keys: Array[Long], keys2: Array[Long], codes: Array[Long]): Int
}
