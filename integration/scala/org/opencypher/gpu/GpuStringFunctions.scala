package org.opencypher.gpu

import org.opencypher.okapi.api.value.CypherValue._

/** The string functions Flink's lowering gives okapi's string expressions
  * (flink-cypher/.../impl/FlinkSQLExprMapper.scala:120-128, 184-195), applied
  * per dictionary string by GpuCypherSession.stringMap with the JVM's own
  * String semantics (the shim's twin of expr.py string_fn). */
object GpuStringFunctions {

  /** key = (name, literal arguments…); None = NULL. */
  def apply(key: Seq[Any], s: String): Option[String] = key match {
    case Seq("upper") => Some(s.toUpperCase)
    case Seq("lower") => Some(s.toLowerCase)
    case Seq("trim") => Some(trimSpaces(s, leading = true, trailing = true))     // SQL TRIM(BOTH ' ')
    case Seq("ltrim") => Some(trimSpaces(s, leading = true, trailing = false))
    case Seq("rtrim") => Some(trimSpaces(s, leading = false, trailing = true))
    case Seq("substring", from: Long, len: Long) => Some(substring(s, from, len))
    case Seq("replace", regex: String, replacement: String) => Some(s.replaceAll(regex, replacement))
    case Seq("regex", pattern: String) => Some(if (s.matches(pattern)) "true" else "false")  // s =~ pattern
    case Seq("concat_r", lit: String) => Some(s + lit)
    case Seq("concat_l", lit: String) => Some(lit + s)
    case other => throw new IllegalArgumentException(s"unknown string function $other")
  }

  private def trimSpaces(s: String, leading: Boolean, trailing: Boolean): String = {
    var b = 0
    var e = s.length
    if (leading) while (b < e && s.charAt(b) == ' ') b += 1
    if (trailing) while (e > b && s.charAt(e - 1) == ' ') e -= 1
    s.substring(b, e)
  }

  /** Calcite SqlFunctions.substring(s, from, for): 1-based, clipped. */
  private def substring(s: String, from0: Long, len: Long): String = {
    val lc = s.length.toLong
    val from = if (from0 < 0) from0 + lc + 1 else from0
    val end = from + len
    if (from > lc || end < 1) ""
    else s.substring((math.max(from, 1L) - 1).toInt, (math.min(end, lc + 1) - 1).toInt)
  }

  /** CAST(v AS VARCHAR). */
  def cast(v: CypherValue): String = v match {
    case CypherString(s) => s
    case CypherInteger(i) => java.lang.Long.toString(i)
    case CypherFloat(d) => java.lang.Double.toString(d)
    case CypherBoolean(b) => if (b) "true" else "false"
    case other => throw new IllegalArgumentException(s"cast of $other to STRING")
  }
}
