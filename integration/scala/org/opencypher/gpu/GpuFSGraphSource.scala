/*
 * GpuFSGraphSource.scala — the file-system PropertyGraphDataSource (CSV
 * storage format) on the MI355X backend: the drop-in for FSGraphSource
 * (flink-cypher/src/main/scala/org/opencypher/flink/api/io/fs/FSGraphSource.scala:47-148)
 * with the graph / store logic of AbstractPropertyGraphDataSource
 * (flink-cypher/.../api/io/AbstractPropertyGraphDataSource.scala:87-155) and
 * the layout of DefaultGraphDirectoryStructure (api/io/fs/GraphDirectoryStructure.scala:35-98):
 *
 *   <root>/<graph name, '.' → '/'>/propertyGraphSchema.json   PropertyGraphSchema.toJson
 *                                 /capsGraphMetaData.json      {"tableStorageFormat":"csv","tags":[0]}
 *                                 /nodes/<labels sorted, '_'-joined, encoded>/<files>
 *                                 /relationships/<rel type, encoded>/<files>
 *
 * Every table has the canonical field list of CAPFGraphExport
 * (api/io/util/CAPFGraphExport.scala:45-63): `id` (nodes) or `id, source,
 * target` (relationships), then the properties sorted by their column name
 * `property_<encoded key>`; no header, ',' between fields (CsvTableSource
 * defaults, FSGraphSource.scala:80-84).  A table whose fields are all
 * non-nullable INTEGERs (ids and INTEGER properties — every R-MAT / LDBC edge
 * table) is parsed on the GPU (capf_csv_read_longs); any other table is parsed
 * on the JVM and uploaded column by column (capf_table_from_host, strings as
 * dictionary codes).  The JVM twin of capf_amd/fs_source.py, which the parity
 * tests drive (tests/test_fs_source.py); the two read and write the same files.
 */
package org.opencypher.gpu

import java.io.File
import java.nio.charset.StandardCharsets
import java.nio.file.{Files, Paths}
import java.nio.{ByteBuffer, ByteOrder}

import org.opencypher.okapi.api.graph.{GraphName, PropertyGraph}
import org.opencypher.okapi.api.io.PropertyGraphDataSource
import org.opencypher.okapi.api.io.conversion.{NodeMappingBuilder, RelationshipMappingBuilder}
import org.opencypher.okapi.api.schema.PropertyGraphSchema
import org.opencypher.okapi.api.types.{CTBoolean, CTFloat, CTInteger, CTNode, CTRelationship, CTString, CypherType}
import org.opencypher.okapi.api.value.CypherValue._
import org.opencypher.okapi.impl.exception.{GraphNotFoundException, IllegalArgumentException, UnsupportedOperationException}
import org.opencypher.okapi.impl.util.StringEncodingUtilities._
import org.opencypher.okapi.ir.api.expr.Var
import org.opencypher.okapi.relational.api.graph.RelationalCypherGraph

import scala.collection.JavaConverters._

object GpuFSGraphSource {
  val SchemaFile = "propertyGraphSchema.json"       // GraphDirectoryStructure.scala:61
  val MetaDataFile = "capsGraphMetaData.json"       // :63
  val NodesDir = "nodes"                            // :65
  val RelsDir = "relationships"                     // :67
  val IdKey = "id"                                  // GraphElement.sourceIdKey
  val SourceKey = "source"                          // Relationship.sourceStartNodeKey
  val TargetKey = "target"                          // Relationship.sourceEndNodeKey

  /** GraphSources.fs(root).csv (api/GraphSources.scala:7-27). */
  def csv(rootPath: String)(implicit gpu: GpuCypherSession): GpuFSGraphSource = GpuFSGraphSource(rootPath)

  /** A canonical field: its column name, capf type and whether the schema
    * types it nullable (then an empty CSV field is NULL). */
  private[gpu] case class Field(name: String, capfType: Int, nullable: Boolean)

  private[gpu] def fieldOf(column: String, ct: CypherType): Field = Field(column, ct.material match {
    case CTInteger => Native.TypeInt64
    case CTFloat => Native.TypeFloat64
    case CTBoolean => Native.TypeBool
    case CTString => Native.TypeString
    case other => throw UnsupportedOperationException(s"CSV column $column of type $other")
  }, ct.isNullable)

  /** One CSV field → its value in a host column (no quoting, FlinkConversions'
    * LONG / DOUBLE / BOOLEAN / STRING; an empty field is NULL). */
  private def parse(s: String, f: Field, path: String, line: Int): Option[Any] =
    if (s.isEmpty) None
    else try Some(f.capfType match {
      case Native.TypeInt64 =>
        if (s.startsWith("+")) throw new NumberFormatException(s)
        java.lang.Long.parseLong(s)
      case Native.TypeFloat64 =>
        if (s.trim != s) throw new NumberFormatException(s)
        java.lang.Double.parseDouble(s)
      case Native.TypeBool => s.toLowerCase match {
        case "true" => true
        case "false" => false
        case _ => throw new NumberFormatException(s)
      }
      case _ => s
    }) catch {
      case _: NumberFormatException =>
        throw IllegalArgumentException(s"a ${f.name} value", s"$path: line $line could not be parsed: '$s'")
    }

  private def format(v: CypherValue): String = v match {
    case CypherNull => ""
    case CypherBoolean(b) => if (b) "true" else "false"
    case other => other.unwrap.toString
  }
}

case class GpuFSGraphSource(rootPath: String)(implicit gpu: GpuCypherSession) extends PropertyGraphDataSource {

  import GpuFSGraphSource._

  private var schemaCache = Map.empty[GraphName, PropertyGraphSchema]

  // -------------------------------------------- DefaultGraphDirectoryStructure
  private def graphDir(name: GraphName): File =                                      // :79-81
    new File(rootPath, name.value.replace(".", File.separator))

  private def nodeTableDir(name: GraphName, labels: Set[String]): File =             // :69, :91-93
    new File(new File(graphDir(name), NodesDir), labels.toSeq.sorted.mkString("_").encodeSpecialCharacters)

  private def relTableDir(name: GraphName, relType: String): File =                  // :71, :95-97
    new File(new File(graphDir(name), RelsDir), relType.encodeSpecialCharacters)

  // ------------------------------------------------------------------ catalog
  override def graphNames: Set[GraphName] = {                                       // FSGraphSource.scala:109-111
    val root = new File(rootPath)
    Option(root.listFiles).map(_.filter(_.isDirectory).map(d => GraphName(d.getName)).toSet).getOrElse(Set.empty)
  }

  override def hasGraph(name: GraphName): Boolean = new File(graphDir(name), SchemaFile).isFile

  override def delete(name: GraphName): Unit = {                                    // AbstractPropertyGraphDataSource.scala:81-85
    schemaCache -= name
    def rm(f: File): Unit = { Option(f.listFiles).foreach(_.foreach(rm)); f.delete() }
    rm(graphDir(name))
  }

  override def schema(name: GraphName): Option[PropertyGraphSchema] =               // :110-118
    schemaCache.get(name).orElse {
      val f = new File(graphDir(name), SchemaFile)
      if (!f.isFile) None else {
        val s = PropertyGraphSchema.fromJson(new String(Files.readAllBytes(f.toPath), StandardCharsets.UTF_8))
        schemaCache += name -> s
        Some(s)
      }
    }

  // --------------------------------------------------------------------- read
  override def graph(name: GraphName): PropertyGraph = {                           // :87-108
    if (!hasGraph(name)) throw GraphNotFoundException(s"Graph with name '$name'")
    val meta = new String(Files.readAllBytes(new File(graphDir(name), MetaDataFile).toPath), StandardCharsets.UTF_8)
    if (!meta.replaceAll("\\s", "").contains("\"tableStorageFormat\":\"csv\""))
      throw UnsupportedOperationException(s"graph $name: only the CSV storage format is readable here")
    val schema = this.schema(name).get
    val nodeTables = schema.allCombinations.toSeq.sortBy(_.toSeq.sorted.mkString("_")).map { combo =>
      val props = schema.nodePropertyKeys(combo).toSeq.map { case (k, ct) => k.toPropertyColumnName -> (k, ct) }.sortBy(_._1)
      val fields = Field(IdKey, Native.TypeInt64, nullable = false) +: props.map { case (c, (_, ct)) => fieldOf(c, ct) }
      val mapping = props.foldLeft(NodeMappingBuilder.on(IdKey).withImpliedLabels(combo.toSeq: _*)) {
        case (b, (c, (k, _))) => b.withPropertyKey(k -> c)
      }.build
      gpu.elementTables.elementTable(mapping, readTable(nodeTableDir(name, combo), fields))
    }
    val relTables = schema.relationshipTypes.toSeq.sorted.map { relType =>
      val props = schema.relationshipPropertyKeys(relType).toSeq.map { case (k, ct) => k.toPropertyColumnName -> (k, ct) }.sortBy(_._1)
      val fields = Seq(IdKey, SourceKey, TargetKey).map(Field(_, Native.TypeInt64, nullable = false)) ++
        props.map { case (c, (_, ct)) => fieldOf(c, ct) }
      val mapping = props.foldLeft(RelationshipMappingBuilder.on(IdKey).from(SourceKey).to(TargetKey).withRelType(relType)) {
        case (b, (c, (k, _))) => b.withPropertyKey(k -> c)
      }.build
      gpu.elementTables.elementTable(mapping, readTable(relTableDir(name, relType), fields))
    }
    if (nodeTables.isEmpty) gpu.graphs.empty
    else gpu.graphs.create(Some(schema), nodeTables.head, (nodeTables.tail ++ relTables): _*)
  }

  /** The data files of a table directory (hidden / '_' files skipped), each
    * read as one table, then unionAll'd (CsvTableSource over a directory). */
  private def readTable(dir: File, fields: Seq[Field]): GpuTable = {
    val files = Option(dir.listFiles).map(_.toSeq.filter(f => f.isFile && !f.getName.startsWith(".") &&
      !f.getName.startsWith("_")).sortBy(_.getName)).getOrElse(Seq.empty)
    val longsOnly = fields.forall(f => f.capfType == Native.TypeInt64 && !f.nullable)
    val parts = files.map { f =>
      if (longsOnly) GpuTable(Native.guard(Native.csvReadLongs(gpu.handle, f.getPath, ",", fields.map(_.name).toArray)))
      else hostTable(f, fields)
    }
    if (parts.isEmpty) gpu.emptyTable(fields.map(f => f.name -> f.capfType))
    else parts.reduce(_ unionAll _)
  }

  /** A table parsed on the JVM: rows split on ',' (trailing '\r' stripped,
    * fields past the declared ones ignored, a short row fails the read), then
    * one direct value buffer + validity buffer per column. */
  private def hostTable(file: File, fields: Seq[Field]): GpuTable = {
    val lines = Files.readAllLines(file.toPath, StandardCharsets.UTF_8).asScala.toIndexedSeq
    val n = lines.size
    val cols = fields.map { f =>
      val width = if (f.capfType == Native.TypeBool) 1 else 8
      (ByteBuffer.allocateDirect(math.max(1, n * width)).order(ByteOrder.nativeOrder()), ByteBuffer.allocateDirect(math.max(1, n)))
    }
    lines.zipWithIndex.foreach { case (raw, i) =>
      val line = if (raw.endsWith("\r")) raw.dropRight(1) else raw
      val parts = line.split(",", -1)
      if (parts.length < fields.size)
        throw IllegalArgumentException(s"${fields.size} fields", s"${file.getPath}: line ${i + 1} could not be parsed: Row too short")
      fields.zip(cols).zipWithIndex.foreach { case ((f, (values, valid)), j) =>
        parse(parts(j), f, file.getPath, i + 1) match {
          case None => valid.put(i, 0.toByte)
          case Some(v) =>
            valid.put(i, 1.toByte)
            v match {
              case x: Long => values.putLong(8 * i, x)
              case x: Double => values.putDouble(8 * i, x)
              case x: Boolean => values.put(i, if (x) 1.toByte else 0.toByte)
              case x: String => values.putLong(8 * i, gpu.intern(x))
            }
        }
      }
    }
    gpu.fromHost(fields.zip(cols).map { case (f, (values, valid)) => (f.name, f.capfType, values, valid) }, n.toLong)
  }

  // -------------------------------------------------------------------- write
  override def store(name: GraphName, graph: PropertyGraph): Unit = {              // :120-155
    if (hasGraph(name))
      throw UnsupportedOperationException(s"A graph with name $name is already stored in this graph data source.")
    val g = graph match {
      case r: RelationalCypherGraph[GpuTable @unchecked] => r
      case other => throw UnsupportedOperationException(s"storing a ${other.getClass.getSimpleName}")
    }
    val schema = g.schema
    val dir = graphDir(name)
    dir.mkdirs()
    Files.write(new File(dir, MetaDataFile).toPath,
      "{\"tableStorageFormat\":\"csv\",\"tags\":[0]}".getBytes(StandardCharsets.UTF_8))
    Files.write(new File(dir, SchemaFile).toPath, schema.toJson.getBytes(StandardCharsets.UTF_8))
    schemaCache += name -> schema
    schema.labelCombinations.combos.foreach { combo =>                                 // CAPFGraphExport.scala:68-83
      val v = Var("n")(CTNode(combo))
      val records = g.nodes(v.name, CTNode(combo), exactLabelMatch = true)
      val h = records.header
      val props = h.propertiesFor(v).toSeq.map(p => h.column(p) -> p.key.name.toPropertyColumnName).sortBy(_._2)
      writeTable(nodeTableDir(name, combo), records.table, (h.column(v) -> IdKey) +: props)
    }
    schema.relationshipTypes.foreach { relType =>                                      // :85-102
      val v = Var("r")(CTRelationship(relType))
      val records = g.relationships(v.name, CTRelationship(relType))
      val h = records.header
      val props = h.propertiesFor(v).toSeq.map(p => h.column(p) -> p.key.name.toPropertyColumnName).sortBy(_._2)
      writeTable(relTableDir(name, relType), records.table,
        Seq(h.column(v) -> IdKey, h.column(h.startNodeFor(v)) -> SourceKey, h.column(h.endNodeFor(v)) -> TargetKey) ++ props)
    }
  }

  /** One CSV file of the canonical columns (CsvTableSink, FSGraphSource.scala:100-107):
    * NULL as an empty field, no quoting. */
  private def writeTable(dir: File, table: GpuTable, columns: Seq[(String, String)]): Unit = {
    dir.mkdirs()
    val canonical = table.select(columns.head, columns.tail: _*)
    val names = columns.map(_._2)
    val out = canonical.rows.map(row => names.map(c => format(row(c))).mkString(",") + "\n").mkString
    Files.write(Paths.get(dir.getPath, "part-00000.csv"), out.getBytes(StandardCharsets.UTF_8))
  }
}
