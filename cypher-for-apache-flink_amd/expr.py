"""Cypher IR expressions used by the relational layer, and their lowering to
the GPU expression program of the C-ABI.

The classes mirror the okapi IR (okapi-ir/src/main/scala/org/opencypher/okapi/
ir/api/expr/Expr.scala): the subset that FlinkSQLExprMapper can lower
(flink-cypher/src/main/scala/org/opencypher/flink/impl/FlinkSQLExprMapper.scala:
48-294).  `compile_program` is the counterpart of `asFlinkSQLExpr`:

 * Var / HasLabel / HasType / StartNode / EndNode resolve to their physical
   column (`expression_for`, CAPFFunctions.scala:63-73); a header expression
   whose column is missing from the table lowers to a NULL literal;
 * ElementProperty not in the header lowers to a NULL literal
   (FlinkSQLExprMapper.scala:102-112);
 * Param is substituted by its value (FlinkSQLExprMapper.scala:80);
 * anything else raises NotImplementedException (:289-290).
"""
from dataclasses import dataclass, field
from typing import Tuple

# capf column types (include/capf_gpu.h)
T_NULL, T_INT, T_FLOAT, T_BOOL, T_STRING, T_LIST = 0, 1, 2, 3, 4, 5

CT_TO_CAPF = {
    "NULL": T_NULL, "INTEGER": T_INT, "FLOAT": T_FLOAT, "BOOLEAN": T_BOOL, "STRING": T_STRING,
    "NODE": T_INT, "RELATIONSHIP": T_INT, "ANY": T_NULL,
    # CTList properties (LIST columns: int64 offsets + an element column)
    "LIST(INTEGER)": T_LIST, "LIST(FLOAT)": T_LIST, "LIST(BOOLEAN)": T_LIST, "LIST(STRING)": T_LIST,
}
CAPF_TO_CT = {T_NULL: "NULL", T_INT: "INTEGER", T_FLOAT: "FLOAT", T_BOOL: "BOOLEAN", T_STRING: "STRING",
              T_LIST: "LIST"}

# opcodes
OP_COL, OP_LIT_INT, OP_LIT_FLOAT, OP_LIT_BOOL, OP_LIT_STRING, OP_LIT_NULL = 1, 2, 3, 4, 5, 6
OP_EQ, OP_NEQ, OP_LT, OP_LE, OP_GT, OP_GE = 10, 11, 12, 13, 14, 15
OP_NOT, OP_AND, OP_OR, OP_IS_NULL, OP_IS_NOT_NULL = 20, 21, 22, 23, 24
OP_ADD, OP_SUB, OP_MUL, OP_DIV, OP_MOD, OP_NEG = 30, 31, 32, 33, 34, 35
OP_TO_FLOAT, OP_TO_INTEGER, OP_COALESCE = 40, 41, 50
OP_STR_LEN, OP_LIST_SIZE, OP_IF = 60, 61, 62
OP_ROUND, OP_ABS, OP_CEIL, OP_FLOOR, OP_SIGN, OP_SQRT, OP_LOG, OP_LOG10, OP_EXP = 70, 71, 72, 73, 74, 75, 76, 77, 78
OP_SIN, OP_COS, OP_TAN, OP_ASIN, OP_ACOS, OP_ATAN, OP_DEGREES, OP_RADIANS = 79, 80, 81, 82, 83, 84, 85, 86
OP_ATAN2, OP_TO_BOOLEAN, OP_IN_SET, OP_STR_MAP, OP_VALUE_MAP = 87, 88, 89, 90, 91
OP_STR_TO_NUM, OP_RAND, OP_LIST_INDEX, OP_STR_RANK = 92, 93, 94, 95
IN_SET_MIN = 17  # list length from which IN runs as a session-set lookup (shorter: an OR of equalities)

# aggregators
AGG_COUNT_STAR, AGG_COUNT, AGG_SUM, AGG_MIN, AGG_MAX, AGG_AVG, AGG_COLLECT = 0, 1, 2, 3, 4, 5, 6
AGG_STDEV, AGG_STDEV_POP, AGG_PERCENTILE_CONT, AGG_PERCENTILE_DISC = 7, 8, 9, 10


class Expr:
    children: Tuple = ()

    def name(self):
        return str(self)


@dataclass(frozen=True)
class Var(Expr):
    vname: str
    ctype: str = field(default="ANY", compare=False)

    def __str__(self):
        return self.vname


@dataclass(frozen=True)
class ElementProperty(Expr):
    owner: Var
    key: str
    ctype: str = field(default="ANY", compare=False)

    def __str__(self):
        return f"{self.owner}.{self.key}"


Property = ElementProperty


@dataclass(frozen=True)
class HasLabel(Expr):
    owner: Var
    label: str

    def __str__(self):
        return f"{self.owner}:{self.label}"


@dataclass(frozen=True)
class HasType(Expr):
    owner: Var
    rel_type: str

    def __str__(self):
        return f"{self.owner}:{self.rel_type}"


@dataclass(frozen=True)
class StartNode(Expr):
    rel: Var

    def __str__(self):
        return f"source({self.rel})"


@dataclass(frozen=True)
class EndNode(Expr):
    rel: Var

    def __str__(self):
        return f"target({self.rel})"


@dataclass(frozen=True)
class IntegerLit(Expr):
    v: int

    def __str__(self):
        return str(self.v)


@dataclass(frozen=True)
class FloatLit(Expr):
    v: float

    def __str__(self):
        return repr(self.v)


@dataclass(frozen=True)
class StringLit(Expr):
    v: str

    def __str__(self):
        return repr(self.v)


@dataclass(frozen=True)
class BoolLit(Expr):
    v: bool

    def __str__(self):
        return "true" if self.v else "false"


TrueLit = BoolLit(True)
FalseLit = BoolLit(False)


@dataclass(frozen=True)
class NullLit(Expr):
    ctype: str = "NULL"

    def __str__(self):
        return "null"


@dataclass(frozen=True)
class Param(Expr):
    pname: str

    def __str__(self):
        return "$" + self.pname


def _binary(name, sym):
    def __str__(self):
        return f"({self.lhs} {sym} {self.rhs})"

    cls = dataclass(frozen=True)(type(name, (Expr,), {"__annotations__": {"lhs": Expr, "rhs": Expr},
                                                       "__str__": __str__}))
    return cls


Equals = _binary("Equals", "=")
LessThan = _binary("LessThan", "<")
LessThanOrEqual = _binary("LessThanOrEqual", "<=")
GreaterThan = _binary("GreaterThan", ">")
GreaterThanOrEqual = _binary("GreaterThanOrEqual", ">=")
Add = _binary("Add", "+")
Subtract = _binary("Subtract", "-")
Multiply = _binary("Multiply", "*")
Divide = _binary("Divide", "/")
Modulo = _binary("Modulo", "%")
# lhs =~ rhs (okapi RegexMatch, Expr.scala:418): Cypher's whole-string Java
# regex match.  Flink lowers it to child0.regexpExtract(child1)
# (FlinkSQLExprMapper.scala:99) — a STRING, which a WHERE cannot take; the
# backend evaluates the predicate the reference expectations pin
# (ExpressionTests.scala:246-312, NullTests.scala:93).
RegexMatch = _binary("RegexMatch", "=~")


def _unary(name, fmt):
    def __str__(self):
        return fmt.format(self.expr)

    return dataclass(frozen=True)(type(name, (Expr,), {"__annotations__": {"expr": Expr},
                                                        "__str__": __str__}))


Not = _unary("Not", "NOT {}")
IsNull = _unary("IsNull", "{} IS NULL")
IsNotNull = _unary("IsNotNull", "{} IS NOT NULL")
ToFloat = _unary("ToFloat", "toFloat({})")
ToInteger = _unary("ToInteger", "toInteger({})")
Negate = _unary("Negate", "-{}")


@dataclass(frozen=True)
class Ands(Expr):
    exprs: Tuple[Expr, ...]

    def __init__(self, *exprs):
        object.__setattr__(self, "exprs", tuple(exprs))

    def __str__(self):
        return "(" + " AND ".join(map(str, self.exprs)) + ")"


@dataclass(frozen=True)
class Ors(Expr):
    exprs: Tuple[Expr, ...]

    def __init__(self, *exprs):
        object.__setattr__(self, "exprs", tuple(exprs))

    def __str__(self):
        return "(" + " OR ".join(map(str, self.exprs)) + ")"


@dataclass(frozen=True)
class Coalesce(Expr):
    exprs: Tuple[Expr, ...]

    def __init__(self, *exprs):
        object.__setattr__(self, "exprs", tuple(exprs))

    def __str__(self):
        return "coalesce(" + ", ".join(map(str, self.exprs)) + ")"


@dataclass(frozen=True)
class ListLit(Expr):
    """[e1, e2, …] (okapi ListLit): literal elements only on the GPU."""
    items: Tuple[Expr, ...]

    def __init__(self, *items):
        object.__setattr__(self, "items", tuple(items))

    def __str__(self):
        return "[" + ", ".join(map(str, self.items)) + "]"


@dataclass(frozen=True)
class In(Expr):
    """lhs IN rhs (okapi In; FlinkSQLExprMapper.scala:114-118): rhs a list
    literal or a list parameter.  SQL IN semantics: NULL when lhs is NULL or
    when nothing matches and the list holds a NULL; an empty list is FALSE."""
    lhs: Expr
    rhs: Expr

    def __str__(self):
        return f"({self.lhs} IN {self.rhs})"


# Mathematical functions (okapi Expr.scala UnaryMathematicalFunctionExpr …;
# FlinkSQLExprMapper.scala:199-221).  Round: half away from zero, a FLOAT (the
# Spark mapping round(x).cast(Double), SparkSQLExprMapper.scala:286 — Flink's
# own case is `child0.round(???)`, which throws).
Round = _unary("Round", "round({})")
Abs = _unary("Abs", "abs({})")
Ceil = _unary("Ceil", "ceil({})")
Floor = _unary("Floor", "floor({})")
Sign = _unary("Sign", "sign({})")
Sqrt = _unary("Sqrt", "sqrt({})")
Log = _unary("Log", "log({})")
Log10 = _unary("Log10", "log10({})")
Exp = _unary("Exp", "exp({})")
Sin = _unary("Sin", "sin({})")
Cos = _unary("Cos", "cos({})")
Tan = _unary("Tan", "tan({})")
Asin = _unary("Asin", "asin({})")
Acos = _unary("Acos", "acos({})")
Atan = _unary("Atan", "atan({})")
Degrees = _unary("Degrees", "degrees({})")
Radians = _unary("Radians", "radians({})")
Cot = _unary("Cot", "cot({})")            # Divide(1, Tan(e)) (:208)
Haversin = _unary("Haversin", "haversin({})")  # Divide(Subtract(1, Cos(e)), 2) (:210)
Atan2 = _binary("Atan2", ",")             # atan2(y, x) (:207)
ToBoolean = _unary("ToBoolean", "toBoolean({})")  # cast to BOOLEAN (:185)
ToString = _unary("ToString", "toString({})")     # cast to STRING (:184): not on the GPU
# startNode(r) / endNode(r): the rel's start / end node column (:179-180)
StartNodeFunction = _unary("StartNodeFunction", "startNode({})")
EndNodeFunction = _unary("EndNodeFunction", "endNode({})")
# UNWIND's Explode(list) (RelationalPlanner.scala:99-101; Explode, :101): a
# withColumns item whose value is each element of the list in turn
Explode = _unary("Explode", "explode({})")


@dataclass(frozen=True)
class E_(Expr):
    """e() (okapi E, FlinkSQLExprMapper.scala:196): Math.E"""

    def __str__(self):
        return "e()"


@dataclass(frozen=True)
class Pi_(Expr):
    """pi() (okapi Pi, FlinkSQLExprMapper.scala:197): Math.PI"""

    def __str__(self):
        return "pi()"


@dataclass(frozen=True)
class Rand_(Expr):
    """rand() (okapi Rand, FlinkSQLExprMapper.scala:207: Flink rand()): a
    uniform double in [0, 1), drawn per row and per evaluation."""

    def __str__(self):
        return "rand()"


E = E_()
Pi = Pi_()
Rand = Rand_()


@dataclass(frozen=True)
class CaseExpr(Expr):
    """CASE WHEN p1 THEN v1 … [ELSE d] END (okapi CaseExpr; FlinkSQLExprMapper
    .scala:242-260: a chain of If(pred, value, rest), the last rest the default
    or a NULL)."""
    alternatives: Tuple[Tuple[Expr, Expr], ...]
    default: object = None

    def __init__(self, alternatives, default=None):
        object.__setattr__(self, "alternatives", tuple(tuple(a) for a in alternatives))
        object.__setattr__(self, "default", default)

    def __str__(self):
        alts = " ".join(f"WHEN {p} THEN {v}" for p, v in self.alternatives)
        return f"CASE {alts}{'' if self.default is None else f' ELSE {self.default}'} END"


# String functions (FlinkSQLExprMapper.scala:187-195): one STRING operand and
# literal arguments — on the GPU a code map of the session dictionary
# (CAPF_OP_STR_MAP), the function applied per dictionary string on the host.
ToUpper = _unary("ToUpper", "toUpper({})")  # upperCase (:190)
ToLower = _unary("ToLower", "toLower({})")  # lowerCase (:191)
Trim = _unary("Trim", "trim({})")           # trim(): SQL TRIM(BOTH ' ') (:187)
LTrim = _unary("LTrim", "lTrim({})")        # (:188)
RTrim = _unary("RTrim", "rTrim({})")        # (:189)


@dataclass(frozen=True)
class Substring(Expr):
    """substring(s, start[, length]) (okapi Substring; FlinkSQLExprMapper.scala
    :195: child0.substring(child1 + 1, child2 — or 1 when absent)): Calcite's
    1-based SUBSTRING over UTF-16 units."""
    expr: Expr
    start: Expr
    length: object = None

    def __str__(self):
        return f"substring({self.expr}, {self.start}{'' if self.length is None else f', {self.length}'})"


@dataclass(frozen=True)
class Replace(Expr):
    """replace(s, search, replacement) (okapi Replace; FlinkSQLExprMapper.scala:
    193: child0.regexpReplace(child1, child2) — `search` is a Java regex)."""
    expr: Expr
    search: Expr
    replacement: Expr

    def __str__(self):
        return f"replace({self.expr}, {self.search}, {self.replacement})"


def java_long_str(v):
    """Long.toString."""
    return str(int(v))


def java_double_str(d):
    """Double.toString: the shortest digits that round-trip, decimal notation for
    1e-3 <= |d| < 1e7 (at least one fractional digit), else d.dddE<exp>."""
    import math
    if math.isnan(d):
        return "NaN"
    if math.isinf(d):
        return "Infinity" if d > 0 else "-Infinity"
    if d == 0:
        return "-0.0" if math.copysign(1.0, d) < 0 else "0.0"
    sign = "-" if d < 0 else ""
    digits, exp = _shortest_digits(abs(d))  # value = 0.d1d2… × 10^exp
    if 1e-3 <= abs(d) < 1e7:
        if exp <= 0:
            txt = "0." + "0" * (-exp) + digits
        elif exp >= len(digits):
            txt = digits + "0" * (exp - len(digits)) + ".0"
        else:
            txt = digits[:exp] + "." + digits[exp:]
        return sign + txt
    mant = digits[0] + "." + (digits[1:] or "0")
    return f"{sign}{mant}E{exp - 1}"


def _shortest_digits(a):
    r = repr(a)  # shortest round-trip (as the JDK's since 19)
    if "e" in r or "E" in r:
        m, e = r.lower().split("e")
        e = int(e)
    else:
        m, e = r, 0
    if "." in m:
        ip, fp = m.split(".")
    else:
        ip, fp = m, ""
    ds = (ip + fp).lstrip("0")
    lead = len(ip.lstrip("0")) if ip.strip("0") else -(len(fp) - len(fp.lstrip("0")))
    ds = ds.rstrip("0") or "0"
    return ds, lead + e


def cypher_to_string(v):
    """A literal cast to STRING (Flink CAST(x AS VARCHAR))."""
    if v is None:
        return None
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return java_long_str(v)
    if isinstance(v, float):
        return java_double_str(v)
    return v


def _utf16(sv):
    return sv.encode("utf-16-le", "surrogatepass")


def _from_utf16(b):
    return b.decode("utf-16-le", "surrogatepass")


def string_fn(key, sv):
    """The string function `key` (a tuple: name, literal args) of the string sv,
    with the JVM semantics Flink's lowering gives it (None: NULL)."""
    import re
    name = key[0]
    if name == "upper":
        return sv.upper()
    if name == "lower":
        return sv.lower()
    if name in ("trim", "ltrim", "rtrim"):  # SQL TRIM of ' ' (not all whitespace)
        return sv.strip(" ") if name == "trim" else sv.lstrip(" ") if name == "ltrim" else sv.rstrip(" ")
    if name == "substring":  # Calcite SqlFunctions.substring(s, from, for), UTF-16 units
        u = _utf16(sv)
        lc = len(u) // 2
        frm, ln = key[1], key[2]
        if frm < 0:
            frm += lc + 1
        e = frm + ln
        if frm > lc or e < 1:
            return ""
        s1, e1 = max(frm, 1), min(e, lc + 1)
        return _from_utf16(u[2 * (s1 - 1):2 * (e1 - 1)])
    if name == "replace":  # REGEXP_REPLACE(s, regex, replacement)
        return re.sub(key[1], lambda m: key[2], sv)
    if name == "regex":  # s =~ pattern: 'true' / 'false' (then cast to BOOLEAN)
        return "true" if re.fullmatch(key[1], sv) else "false"
    if name == "concat_r":  # s + literal
        return sv + key[1]
    if name == "concat_l":  # literal + s
        return key[1] + sv
    raise ValueError(f"unknown string function {key}")


_STR_FUNCS = {"ToUpper": "upper", "ToLower": "lower", "Trim": "trim", "LTrim": "ltrim", "RTrim": "rtrim"}


@dataclass(frozen=True)
class ContainerIndex(Expr):
    """container[index] (okapi ContainerIndex, Expr.scala:1240; Flink
    `container.at(index)`, FlinkSQLExprMapper.scala:262-269) on a list: the
    element at the 0-based index (negative from the end), NULL out of range —
    Cypher's indexing, which the reference expectations pin
    (ExpressionTests.scala:863-918).  Flink's ARRAY `at` is 1-based, so the
    Flink path returns the next element (a hazard)."""
    container: Expr
    index: Expr

    def __str__(self):
        return f"{self.container}[{self.index}]"


@dataclass(frozen=True)
class MapExpression(Expr):
    """{k1: e1, k2: e2, …} (okapi MapExpression, Expr.scala:511; Flink
    MapConstructor, FlinkSQLExprMapper.scala:271-278).  A MAP value is held as
    a struct of columns: the planner projects one column per entry plus a
    presence flag (planner.py `_map_entries`); `m.k` / `m['k']` read the
    entry's column (ElementProperty on the MAP variable), records() rebuilds
    the Python dict."""
    items: Tuple[Tuple[str, Expr], ...]

    def __init__(self, items=()):
        pairs = items.items() if isinstance(items, dict) else items
        object.__setattr__(self, "items", tuple((str(k), v) for k, v in pairs))

    def __str__(self):
        return "{" + ", ".join(f"{k}: {v}" for k, v in self.items) + "}"


# properties(x) (okapi Properties, Expr.scala:851; FlinkSQLExprMapper.scala:167-177):
# the MAP of a node's / relationship's property columns (every key of its
# header, NULL values included), or a MAP itself
Properties = _unary("Properties", "properties({})")


# labels(n) / keys(n) (FlinkSQLExprMapper.scala:136-153): a LIST of the label names
# whose flag column is TRUE / of the property keys holding a value, sorted by
# name — a table operation (capf_table_name_list), as a withColumns item only
Labels = _unary("Labels", "labels({})")
Keys = _unary("Keys", "keys({})")


def name_list_columns(e, header, columns):
    """(columns, kinds, names) of labels(v) / keys(v) over the header: the
    label flag columns (kind 0) or property columns (kind 1) of v, by name."""
    v = e.expr
    is_labels = type(e).__name__ == "Labels"
    found = []
    for h, c in (header.items() if header is not None else ()):
        if c not in columns:
            continue
        if is_labels and isinstance(h, HasLabel) and h.owner == v:
            found.append((h.label, c))
        elif not is_labels and isinstance(h, ElementProperty) and h.owner == v:
            found.append((h.key, c))
    found.sort()
    return [c for _, c in found], [0 if is_labels else 1] * len(found), [nm for nm, _ in found]


Id = _unary("Id", "id({})")            # FlinkSQLExprMapper.scala:134: the element's id column
Exists = _unary("Exists", "exists({})")  # exists(n.prop) → IS NOT NULL (:90)
Size = _unary("Size", "size({})")      # charLength / cardinality (:80-85)
Type = _unary("Type", "type({})")      # the relationship's type name (:152-160)


def java_length(v):
    """Java String.length: UTF-16 code units."""
    return len(v.encode("utf-16-le", "surrogatepass")) // 2


class ExistsPattern(Expr):
    """EXISTS((a)-->()-->(b)) — a pattern predicate (okapi ExistsPatternExpr,
    okapi-ir/.../api/expr/Expr.scala).  `pattern` is a planner Match over
    variables of the enclosing clause; the relational planner turns it into
    an ExistsSubQuery (RelationalPlanner.scala:224-247) whose boolean target
    column then stands for this expression in the header (the Flink mapper
    lowers ExistsPatternExpr to its target field, FlinkSQLExprMapper.scala:226).
    Identity-hashed: two EXISTS with the same text are two sub-queries."""

    def __init__(self, pattern):
        self.pattern = pattern

    def __str__(self):
        return f"exists#{id(self) & 0xFFFFFF:06x}"

    def __hash__(self):
        return id(self)

    def __eq__(self, other):
        return self is other


# ----------------------------------------------------------------- aggregators
class Aggregator(Expr):
    kind = -1
    distinct = False


@dataclass(frozen=True)
class CountStar(Aggregator):
    kind = AGG_COUNT_STAR

    def __str__(self):
        return "count(*)"


@dataclass(frozen=True)
class Count(Aggregator):
    expr: Expr
    distinct: bool = False
    kind = AGG_COUNT

    def __str__(self):
        return f"count({'DISTINCT ' if self.distinct else ''}{self.expr})"


@dataclass(frozen=True)
class Sum(Aggregator):
    expr: Expr
    kind = AGG_SUM

    def __str__(self):
        return f"sum({self.expr})"


@dataclass(frozen=True)
class Min(Aggregator):
    expr: Expr
    kind = AGG_MIN

    def __str__(self):
        return f"min({self.expr})"


@dataclass(frozen=True)
class Max(Aggregator):
    expr: Expr
    kind = AGG_MAX

    def __str__(self):
        return f"max({self.expr})"


@dataclass(frozen=True)
class Avg(Aggregator):
    expr: Expr
    kind = AGG_AVG

    def __str__(self):
        return f"avg({self.expr})"


# --------------------------------------------------------------- lowering
_BIN_OPS = {
    "Equals": OP_EQ, "LessThan": OP_LT, "LessThanOrEqual": OP_LE, "GreaterThan": OP_GT,
    "GreaterThanOrEqual": OP_GE, "Add": OP_ADD, "Subtract": OP_SUB, "Multiply": OP_MUL,
    "Divide": OP_DIV, "Modulo": OP_MOD,
}
_ORDERED = ("LessThan", "LessThanOrEqual", "GreaterThan", "GreaterThanOrEqual")
_CMP_NAMES = ("Equals",) + _ORDERED
_UN_OPS = {"Not": OP_NOT, "IsNull": OP_IS_NULL, "IsNotNull": OP_IS_NOT_NULL, "ToFloat": OP_TO_FLOAT,
           "ToInteger": OP_TO_INTEGER, "Negate": OP_NEG, "Exists": OP_IS_NOT_NULL,
           "Round": OP_ROUND, "Abs": OP_ABS, "Ceil": OP_CEIL, "Floor": OP_FLOOR, "Sign": OP_SIGN,
           "Sqrt": OP_SQRT, "Log": OP_LOG, "Log10": OP_LOG10, "Exp": OP_EXP, "Sin": OP_SIN, "Cos": OP_COS,
           "Tan": OP_TAN, "Asin": OP_ASIN, "Acos": OP_ACOS, "Atan": OP_ATAN, "Degrees": OP_DEGREES,
           "Radians": OP_RADIANS, "ToBoolean": OP_TO_BOOLEAN}
# math functions whose result is a FLOAT whatever the operand (Calcite's
# DOUBLE-returning functions)
_FLOAT_FUNCS = {"Round", "Sqrt", "Log", "Log10", "Exp", "Sin", "Cos", "Tan", "Asin", "Acos", "Atan", "Degrees",
                "Radians", "Cot", "Haversin", "Atan2"}


def _value_type(v):
    """capf type of a literal / parameter value (None: not a scalar)."""
    if v is None:
        return T_NULL
    if isinstance(v, bool):
        return T_BOOL
    if isinstance(v, int):
        return T_INT
    if isinstance(v, float):
        return T_FLOAT
    if isinstance(v, str):
        return T_STRING
    return None


def literal_expr(v):
    """The literal expression of a host value (a list parameter's element)."""
    if v is None:
        return NullLit()
    if isinstance(v, bool):
        return BoolLit(v)
    if isinstance(v, int):
        return IntegerLit(v)
    if isinstance(v, float):
        return FloatLit(v)
    if isinstance(v, str):
        return StringLit(v)
    from ._lib import NotImplementedException
    raise NotImplementedException(f"a list element {v!r} of type {type(v).__name__}")


def _comparable(a, b):
    """Could values of capf types a and b be equal?  (None: unknown.)"""
    if a is None or b is None or T_NULL in (a, b):
        return True
    num = (T_INT, T_FLOAT)
    return a == b or (a in num and b in num)


def list_values(e, params):
    """The Python values of a list literal / list parameter, or None."""
    if isinstance(e, ListLit):
        out = []
        for x in e.items:
            if isinstance(x, NullLit):
                out.append(None)
            elif isinstance(x, (IntegerLit, FloatLit, StringLit, BoolLit)):
                out.append(x.v)
            elif isinstance(x, Param):
                out.append((params or {}).get(x.pname))
            else:
                return None
        return out
    if isinstance(e, Param):
        v = (params or {}).get(e.pname)
        return list(v) if isinstance(v, (list, tuple)) else None
    return None


def explode_values(e, params):
    """(capf element type, python values) of a literal / parameter list to
    UNWIND, or None when `e` is not one.  INTEGER and FLOAT elements widen to
    FLOAT together; NULL elements stay; other mixes are NotImplemented."""
    vals = list_values(e, params)
    if vals is None:
        if isinstance(e, NullLit) or (isinstance(e, Param) and (params or {}).get(e.pname) is None):
            return T_NULL, []  # UNWIND null: no rows (Spark explode of a NULL array)
        return None
    kinds = {_value_type(v) for v in vals if v is not None}
    if None in kinds:
        from ._lib import NotImplementedException
        raise NotImplementedException(f"UNWIND of nested lists / maps: {e}")
    if not kinds:
        return T_NULL, vals
    if kinds <= {T_INT, T_FLOAT}:
        if T_FLOAT in kinds:
            return T_FLOAT, [None if v is None else float(v) for v in vals]
        return T_INT, vals
    if len(kinds) == 1:
        return kinds.pop(), vals
    from ._lib import NotImplementedException
    raise NotImplementedException(f"UNWIND of a list of mixed types: {e}")


def resolve_column(expr, header, columns):
    """Physical column of a header expression or None (→ NULL literal)."""
    col = header.get(expr) if header is not None else None
    if col is not None and col in columns:
        return col
    return None


_MISSING = object()
_PROGRAM_MEMO = {}  # repr(expr) -> (lookups made while compiling it, program)


def _memo_key(expr):
    """repr(expr), kept on the instance: unlike Expr equality it tells 1 from
    True and 1 from 1.0 inside literals, which lower to different programs."""
    d = expr.__dict__
    k = d.get("_mk")
    if k is None:
        k = d["_mk"] = repr(expr)
    return k


class _Lookups:
    """Recording views of compile_program's inputs: every header / column /
    type / parameter / string-code lookup and its answer, so a later call with
    the same expression reuses the program when every answer is the same."""
    __slots__ = ("log", "cacheable", "h", "cols", "par", "intern_fn", "type_fn")

    def __init__(self, header, columns, params, intern, coltype):
        self.log, self.cacheable = [], True
        self.h, self.cols, self.par = header, columns, params or {}
        self.intern_fn, self.type_fn = intern, coltype

    # header view
    def get(self, e, default=None):
        v = self.h.get(e, _MISSING)
        self.log.append((0, e, v))
        return default if v is _MISSING else v

    def __contains__(self, e):
        return self.get(e, _MISSING) is not _MISSING

    def items(self):  # the whole header: not recorded, the program is not reused
        self.cacheable = False
        return self.h.items()


class _ColumnsView:
    __slots__ = ("rec",)

    def __init__(self, rec):
        self.rec = rec

    def __contains__(self, c):
        v = c in self.rec.cols
        self.rec.log.append((1, c, v))
        return v


class _ParamsView:
    __slots__ = ("rec",)

    def __init__(self, rec):
        self.rec = rec

    def __bool__(self):
        return True

    def get(self, k, default=None):
        v = self.rec.par.get(k, _MISSING)
        self.rec.log.append((2, k, _MISSING if v is _MISSING else repr(v)))
        return default if v is _MISSING else v

    def __getitem__(self, k):
        v = self.get(k, _MISSING)
        if v is _MISSING:
            raise KeyError(k)
        return v


def _lookups_hold(log, header, columns, params, intern, coltype, lset=None, smap=None):
    params = params or {}
    for kind, k, v in log:
        if kind == 0:
            if header.get(k, _MISSING) != v:
                return False
        elif kind == 1:
            if (k in columns) != v:
                return False
        elif kind == 2:
            w = params.get(k, _MISSING)
            if (_MISSING if w is _MISSING else repr(w)) != v:
                return False
        elif kind == 3:
            if coltype is None or coltype(k) != v:
                return False
        elif kind == 5:
            if lset is None or lset(k) != v:
                return False
        elif kind == 6:
            if smap is None or smap(k) != v:
                return False
        elif intern is None or intern(k) != v:
            return False
    return True


def compile_program(expr, header, columns, params=None, intern=None, coltype=None, lset=None, smap=None,
                    vmap=None):
    """Lower `expr` to (ops, iargs, fargs, names) for the C-ABI — memoised per
    expression: a program is reused when every lookup its compilation made
    (header columns, column presence and types, parameters, string codes)
    gives the same answer again (the planner re-plans the same predicates and
    aggregates query after query).  Programs are immutable once returned."""
    try:
        key = _memo_key(expr)
    except AttributeError:  # not an Expr instance: compile every time
        return _compile_program(expr, header, columns, params, intern, coltype, lset, smap, vmap)
    ent = _PROGRAM_MEMO.get(key)
    if ent is not None and header is not None and ent[0] is not None and \
            _lookups_hold(ent[0], header, columns, params, intern, coltype, lset, smap):
        return ent[1]
    if header is None:
        return _compile_program(expr, header, columns, params, intern, coltype, lset, smap, vmap)
    rec = _Lookups(header, columns, params, intern, coltype)

    def rec_type(c):
        v = coltype(c)
        rec.log.append((3, c, v))
        return v

    def rec_intern(x):
        v = intern(x)
        rec.log.append((4, x, v))
        return v

    def rec_lset(vals):
        v = lset(vals)
        rec.log.append((5, vals, v))
        return v

    def rec_smap(k):
        v = smap(k)
        rec.log.append((6, k, v))
        return v

    def rec_vmap(kind, exprs):  # depends on the table's data: never memoised
        rec.cacheable = False
        return vmap(kind, exprs)

    prog = _compile_program(expr, rec, _ColumnsView(rec), _ParamsView(rec),
                            rec_intern if intern is not None else None,
                            rec_type if coltype is not None else None,
                            rec_lset if lset is not None else None,
                            rec_smap if smap is not None else None,
                            rec_vmap if vmap is not None else None)
    prog = (tuple(prog[0]), tuple(prog[1]), tuple(prog[2]), tuple(prog[3]))
    if rec.cacheable:
        if len(_PROGRAM_MEMO) >= 4096:
            _PROGRAM_MEMO.clear()
        _PROGRAM_MEMO[key] = (rec.log, prog)
    return prog


def _compile_program(expr, header, columns, params=None, intern=None, coltype=None, lset=None, smap=None,
                     vmap=None):
    """Lower `expr` to (ops, iargs, fargs, names) for the C-ABI.

    header: dict Expr -> physical column; columns: set of the table's columns;
    intern: str -> int64 code (session string dictionary); coltype: column ->
    capf type (for size() and IN, whose lowering depends on the operand type).
    """
    params = params or {}
    ops, ia, fa, names = [], [], [], []
    name_idx = {}

    def emit(op, i=0, f=0.0):
        ops.append(op)
        ia.append(int(i))
        fa.append(float(f))

    def lit(v):
        if v is None:
            emit(OP_LIT_NULL, T_NULL)
        elif isinstance(v, bool):
            emit(OP_LIT_BOOL, 1 if v else 0)
        elif isinstance(v, int):
            emit(OP_LIT_INT, v)
        elif isinstance(v, float):
            emit(OP_LIT_FLOAT, 0, v)
        elif isinstance(v, str):
            if intern is None:
                raise ValueError("string literal without a string dictionary")
            emit(OP_LIT_STRING, intern(v))
        else:
            from ._lib import NotImplementedException
            raise NotImplementedException(f"literal {v!r} of type {type(v).__name__}")

    def name_of(name):
        if name not in name_idx:
            name_idx[name] = len(names)
            names.append(name)
        return name_idx[name]

    def col(name):
        emit(OP_COL, name_of(name))

    def column_of(e):
        return resolve_column(e, header, columns) if header is not None and e in header else None

    def static_type(e):
        """capf type of e when known without evaluating it, else None."""
        c = column_of(e)
        if c is not None:
            return coltype(c) if coltype is not None else CT_TO_CAPF.get(getattr(e, "ctype", "ANY"))
        if isinstance(e, (IntegerLit, FloatLit, StringLit, BoolLit)):
            return _value_type(e.v)
        if isinstance(e, NullLit):
            return T_NULL
        if isinstance(e, Param):
            return _value_type((params or {}).get(e.pname))
        if isinstance(e, (Var, ElementProperty)):  # no column: a NULL literal
            return T_NULL
        if isinstance(e, (ToFloat,)) or type(e).__name__ in _FLOAT_FUNCS or isinstance(e, (E_, Pi_, Rand_)):
            return T_FLOAT
        if type(e).__name__ in ("Labels", "Keys") and isinstance(e.expr, NullLit):
            return T_NULL
        if isinstance(e, (ToInteger, Size, Id)):
            return T_INT
        if isinstance(e, ToBoolean) or type(e).__name__ == "RegexMatch":
            return T_BOOL
        if type(e).__name__ in _STR_FUNCS or isinstance(e, (Substring, Replace, ToString)):
            return T_STRING
        name = type(e).__name__
        if name in ("Add", "Subtract", "Multiply", "Divide", "Modulo"):
            ta, tb = static_type(e.lhs), static_type(e.rhs)
            if name == "Add" and T_STRING in (ta, tb):
                return T_STRING
            if ta in (T_INT, T_FLOAT) and tb in (T_INT, T_FLOAT):
                return T_FLOAT if T_FLOAT in (ta, tb) else T_INT
            return None
        if name in ("Negate", "Abs", "Ceil", "Floor", "Sign"):
            t = static_type(e.expr)
            return t if t in (T_INT, T_FLOAT) else None
        if name in _CMP_NAMES or isinstance(e, (Ands, Ors, In)) or name in ("Not", "IsNull", "IsNotNull", "Exists"):
            return T_BOOL
        if isinstance(e, (Coalesce, CaseExpr)):  # the branches' common type (INTEGER and FLOAT: FLOAT)
            parts = list(e.exprs) if isinstance(e, Coalesce) else \
                [v for _, v in e.alternatives] + ([e.default] if e.default is not None else [])
            ts = {static_type(x) for x in parts} - {T_NULL}
            if None in ts or not ts:
                return None if None in ts else T_NULL
            if ts == {T_INT, T_FLOAT}:
                return T_FLOAT
            return ts.pop() if len(ts) == 1 else None
        return None

    def literal_value(x):
        """(True, value) of a literal / parameter operand — string concatenations
        of literals folded ('l' + 'l', FunctionTests.scala:480-487) — else
        (False, None)."""
        if isinstance(x, (IntegerLit, FloatLit, StringLit, BoolLit)):
            return True, x.v
        if isinstance(x, NullLit):
            return True, None
        if isinstance(x, Param):
            return True, (params or {}).get(x.pname)
        if type(x).__name__ == "Add":
            la, va = literal_value(x.lhs)
            lb, vb = literal_value(x.rhs)
            if la and lb and (isinstance(va, str) or isinstance(vb, str)):
                if va is None or vb is None:
                    return True, None
                if not all(isinstance(v, (str, int, float)) and not isinstance(v, bool) for v in (va, vb)):
                    return False, None
                return True, cypher_to_string(va) + cypher_to_string(vb)
        return False, None

    def no_memo():
        """The program depends on more than its lookups (rand()'s seed)."""
        if isinstance(header, _Lookups):
            header.cacheable = False

    def string_map(x, key):
        """f(x) for a STRING operand x: folded for a literal, else a code map."""
        isl, v = literal_value(x)
        if isl:
            if v is not None and not isinstance(v, str):
                not_impl(x)
            lit(None if v is None else string_fn(key, v))
            return
        t = static_type(x)
        if t == T_NULL:
            emit(OP_LIT_NULL, T_STRING)
            return
        if t != T_STRING or (smap is None and vmap is None):
            not_impl(x)
        go(x)
        nm = smap(key) if smap is not None else None
        if nm is not None:  # a code map of the whole (small) dictionary
            emit(OP_STR_MAP, name_of(nm))
        elif vmap is not None:
            # f over the operand's DISTINCT values in this table (a value map):
            # a code map over a large dictionary would apply f to every string
            # and intern every result, and each such map grows the dictionary
            # the next one must cover
            emit(OP_VALUE_MAP, name_of(vmap(("fn", key), (x,))), 0.0)
        else:
            not_impl(x)

    def not_impl(what):
        from ._lib import NotImplementedException
        raise NotImplementedException(f"No support for converting Cypher expression {what} to a GPU expression")

    def container_index(e):
        """xs[i] (FlinkSQLExprMapper.scala:262-269), Cypher's 0-based indexing:
        a literal / parameter list with a literal index folds; with a column
        index it is a chain of IFs over the index values; a LIST column is
        CAPF_OP_LIST_INDEX (the element type from the column)."""
        from ._lib import IllegalArgumentException
        if isinstance(e.container, Var) and e.container.ctype == "MAP":
            # m['k'] on a MAP held as a struct of columns: the entry's column
            okk, key = literal_value(e.index)
            if not okk or not isinstance(key, (str, type(None))):
                not_impl(e)  # a per-row key
            if key is None:
                emit(OP_LIT_NULL, T_NULL)
            else:
                go(ElementProperty(e.container, key))
            return
        isl, iv = literal_value(e.index)
        if isl and (isinstance(iv, bool) or not isinstance(iv, (int, type(None)))):
            raise IllegalArgumentException(f"a list index must be an INTEGER, got {e.index}")
        vals = list_values(e.container, params) if isinstance(e.container, (ListLit, Param)) else None
        if vals is not None:
            kinds = {_value_type(v) for v in vals if v is not None}
            if None in kinds:
                not_impl(e)  # nested lists / maps
            t = (T_FLOAT if kinds <= {T_INT, T_FLOAT} and T_FLOAT in kinds else
                 kinds.pop() if len(kinds) == 1 else T_NULL if not kinds else None)
            if t is None:
                not_impl(e)  # a list of mixed types
            conv = (lambda v: None if v is None else float(v)) if t == T_FLOAT else (lambda v: v)
            n = len(vals)
            if isl:
                k = None if iv is None else (iv + n if iv < 0 else iv)
                if k is None or not 0 <= k < n:
                    emit(OP_LIT_NULL, t)
                else:
                    lit(conv(vals[k]))
                return
            emit(OP_LIT_NULL, t)  # acc: out of range
            for k in reversed(range(n)):  # IF(i = k OR i = k − n, v_k, acc)
                go(e.index)
                lit(k)
                emit(OP_EQ)
                go(e.index)
                lit(k - n)
                emit(OP_EQ)
                emit(OP_OR, 2)
                lit(conv(vals[k]))
                emit(OP_IF)
            return
        if isinstance(e.container, NullLit):
            emit(OP_LIT_NULL, T_NULL)
            return
        c = column_of(e.container)
        if c is None or static_type(e.container) != T_LIST or coltype is None:
            not_impl(e)
        et = coltype(("elem", c))
        go(e.index)
        emit(OP_LIST_INDEX, name_of(c), float(et))

    def go(e):
        cls = type(e).__name__
        if isinstance(e, (Var, HasLabel, HasType, StartNode, EndNode, ElementProperty)):
            c = resolve_column(e, header, columns)
            if c is None:
                ct = getattr(e, "ctype", "BOOLEAN" if isinstance(e, (HasLabel, HasType)) else "INTEGER")
                emit(OP_LIT_NULL, CT_TO_CAPF.get(ct, T_NULL))
            else:
                col(c)
            return
        c = resolve_column(e, header, columns) if header is not None and e in header else None
        if c is not None:  # an already-projected expression (e.g. an alias column)
            col(c)
            return
        if isinstance(e, IntegerLit):
            emit(OP_LIT_INT, e.v)
        elif isinstance(e, FloatLit):
            emit(OP_LIT_FLOAT, 0, e.v)
        elif isinstance(e, BoolLit):
            emit(OP_LIT_BOOL, 1 if e.v else 0)
        elif isinstance(e, StringLit):
            lit(e.v)
        elif isinstance(e, NullLit):
            emit(OP_LIT_NULL, CT_TO_CAPF.get(e.ctype, T_NULL))
        elif isinstance(e, Param):
            lit(params[e.pname])
        elif cls == "Add" and T_STRING in (static_type(e.lhs), static_type(e.rhs)):
            # string concatenation (:120-128): concat with the other side cast to
            # STRING; on the GPU one side must be a literal (a code map of the other)
            la, va = literal_value(e.lhs)
            lb, vb = literal_value(e.rhs)
            if la and lb:
                lit(None if va is None or vb is None else cypher_to_string(va) + cypher_to_string(vb))
            elif lb:
                if vb is None:
                    emit(OP_LIT_NULL, T_STRING)
                else:
                    string_map(e.lhs, ("concat_r", cypher_to_string(vb)))
            elif la:
                if va is None:
                    emit(OP_LIT_NULL, T_STRING)
                else:
                    string_map(e.rhs, ("concat_l", cypher_to_string(va)))
            else:  # two columns: a new string per distinct value pair (a value map)
                ta, tb = static_type(e.lhs), static_type(e.rhs)
                if vmap is None or not {ta, tb} <= {T_STRING, T_INT, T_FLOAT}:
                    not_impl(e)
                go(e.lhs)
                go(e.rhs)
                emit(OP_VALUE_MAP, name_of(vmap("concat", (e.lhs, e.rhs))), 1.0)
        elif cls == "RegexMatch":
            # a code map of the dictionary: each string's match as 'true' / 'false',
            # then the session's string → BOOLEAN table (CAPF_OP_TO_BOOLEAN)
            okp, pat = literal_value(e.rhs)
            if not okp or not isinstance(pat, (str, type(None))):
                not_impl(e)  # a per-row pattern
            if pat is None:
                emit(OP_LIT_NULL, T_BOOL)
                return
            import re
            try:
                re.compile(pat)
            except re.error as err:
                from ._lib import IllegalArgumentException
                raise IllegalArgumentException(f"invalid regular expression {pat!r}: {err}")
            okl, sv = literal_value(e.lhs)
            if okl:  # a literal subject folds
                if sv is not None and not isinstance(sv, str):
                    not_impl(e)
                if sv is None:
                    emit(OP_LIT_NULL, T_BOOL)
                else:
                    emit(OP_LIT_BOOL, 1 if re.fullmatch(pat, sv) else 0)
                return
            t = static_type(e.lhs)
            if t == T_NULL:
                emit(OP_LIT_NULL, T_BOOL)
                return
            if t != T_STRING or vmap is None:
                not_impl(e)
            # the match of each DISTINCT subject value of this table (a value map
            # over STRING codes) — not of the whole dictionary, where one long
            # unrelated string can make a backtracking pattern exponential
            go(e.lhs)
            emit(OP_VALUE_MAP, name_of(vmap(("regex", pat), (e.lhs,))), 0.0)
            emit(OP_TO_BOOLEAN)
        elif cls in _ORDERED:
            # FlinkSQLExprMapper.scala:91-94.  STRINGs order by their rank in
            # the session dictionary (CAPF_OP_STR_RANK, String.compareTo);
            # operands of incomparable types compare to NULL (Cypher: 1 < 'a'
            # is null, so a WHERE drops the row — PredicateTests.scala:195)
            ta, tb = static_type(e.lhs), static_type(e.rhs)
            if None not in (ta, tb) and T_NULL not in (ta, tb) and not _comparable(ta, tb):
                emit(OP_LIT_NULL, T_BOOL)
                return
            strs = T_STRING in (ta, tb)
            go(e.lhs)
            if strs:
                emit(OP_STR_RANK)
            go(e.rhs)
            if strs:
                emit(OP_STR_RANK)
            emit(_BIN_OPS[cls])
        elif cls in _BIN_OPS:
            go(e.lhs)
            go(e.rhs)
            emit(_BIN_OPS[cls])
        elif cls in _STR_FUNCS:
            string_map(e.expr, (_STR_FUNCS[cls],))
        elif isinstance(e, Substring):
            ok1, st = literal_value(e.start)
            ok2, ln = literal_value(e.length) if e.length is not None else (True, 1)
            if not (ok1 and ok2) or any(isinstance(v, bool) or not isinstance(v, (int, type(None))) for v in (st, ln)):
                not_impl(e)
            if st is None or ln is None:
                emit(OP_LIT_NULL, T_STRING)
            elif ln < 0:
                from ._lib import IllegalArgumentException
                raise IllegalArgumentException(f"negative substring length {ln}")
            else:
                string_map(e.expr, ("substring", int(st) + 1, int(ln)))
        elif isinstance(e, Replace):
            ok1, se = literal_value(e.search)
            ok2, rp = literal_value(e.replacement)
            if not (ok1 and ok2) or not all(isinstance(v, (str, type(None))) for v in (se, rp)):
                not_impl(e)
            if se is None or rp is None:
                emit(OP_LIT_NULL, T_STRING)
            elif "$" in rp or "\\" in rp:
                not_impl(e)  # Java regex replacement groups
            else:
                string_map(e.expr, ("replace", se, rp))
        elif isinstance(e, ToString):  # cast to STRING (:184)
            isl, v = literal_value(e.expr)
            t = static_type(e.expr)
            if isl:
                lit(cypher_to_string(v))
            elif t == T_STRING:
                go(e.expr)
            elif t == T_NULL:
                emit(OP_LIT_NULL, T_STRING)
            elif t == T_BOOL:  # NULL ← IF(NOT x, 'false', ·) ← IF(x, 'true', ·)
                emit(OP_LIT_NULL, T_STRING)
                go(e.expr)
                emit(OP_NOT)
                lit("false")
                emit(OP_IF)
                go(e.expr)
                lit("true")
                emit(OP_IF)
            elif t in (T_INT, T_FLOAT) and vmap is not None:  # a new string per distinct value
                go(e.expr)
                emit(OP_VALUE_MAP, name_of(vmap("tostring", (e.expr,))), 0.0)
            else:
                not_impl(e)
        elif cls in ("ToFloat", "ToInteger") and static_type(e.expr) == T_STRING:
            # CAST(string AS DOUBLE / INT) (FlinkSQLExprMapper.scala:182-183): the
            # dictionary strings parsed once per session (a device table)
            go(e.expr)
            emit(OP_STR_TO_NUM, 1 if cls == "ToFloat" else 0)
        elif cls in ("Labels", "Keys") and isinstance(e.expr, NullLit):
            emit(OP_LIT_NULL, T_NULL)  # labels(null) / keys(null) is NULL (MTa/NullTests.scala:50, 53)
        elif cls in _UN_OPS:
            go(e.expr)
            emit(_UN_OPS[cls])
        elif isinstance(e, Rand_):  # a fresh seed per compilation: never memoised
            import os
            no_memo()
            emit(OP_RAND, int.from_bytes(os.urandom(8), "little") >> 1)
        elif isinstance(e, Ands):
            if not e.exprs:
                emit(OP_LIT_BOOL, 1)
                return
            for x in e.exprs:
                go(x)
            emit(OP_AND, len(e.exprs))
        elif isinstance(e, Ors):
            if not e.exprs:
                emit(OP_LIT_BOOL, 0)
                return
            for x in e.exprs:
                go(x)
            emit(OP_OR, len(e.exprs))
        elif isinstance(e, Coalesce):
            for x in e.exprs:
                go(x)
            emit(OP_COALESCE, len(e.exprs))
        elif cls == "Id":
            go(e.expr)  # the id column (FlinkSQLExprMapper.scala:134)
        elif cls in ("StartNodeFunction", "EndNodeFunction"):
            v = e.expr  # header.startNodeFor / endNodeFor of the rel var (:179-180)
            if isinstance(v, NullLit):
                emit(OP_LIT_NULL, T_INT)  # startNode(null) is NULL (MTa/NullTests.scala:53-54)
                return
            if not isinstance(v, Var):
                not_impl(e)
            go(StartNode(v) if cls == "StartNodeFunction" else EndNode(v))
        elif isinstance(e, E_):
            emit(OP_LIT_FLOAT, 0, 2.718281828459045)
        elif isinstance(e, Pi_):
            emit(OP_LIT_FLOAT, 0, 3.141592653589793)
        elif cls == "Cot":  # Divide(IntegerLit(1), Tan(e)) (:208)
            emit(OP_LIT_INT, 1)
            go(e.expr)
            emit(OP_TAN)
            emit(OP_DIV)
        elif cls == "Haversin":  # Divide(Subtract(1, Cos(e)), 2) (:210)
            emit(OP_LIT_INT, 1)
            go(e.expr)
            emit(OP_COS)
            emit(OP_SUB)
            emit(OP_LIT_INT, 2)
            emit(OP_DIV)
        elif cls == "Atan2":  # atan2(child0, child1) (:207)
            go(e.lhs)
            go(e.rhs)
            emit(OP_ATAN2)
        elif isinstance(e, CaseExpr):
            if not e.alternatives:
                not_impl(e)
            # If(p1, v1, If(p2, v2, … default)): innermost first in postfix
            if e.default is None:
                emit(OP_LIT_NULL, T_INT)  # expressions.Null(Types.LONG) (:256)
            else:
                go(e.default)
            for p, v in reversed(e.alternatives):
                go(p)
                go(v)
                emit(OP_IF)
        elif isinstance(e, In):
            vals = list_values(e.rhs, params)
            if vals is None and literal_value(e.rhs) == (True, None):
                emit(OP_LIT_NULL, T_BOOL)  # x IN null: the rhs type is not a list (:117)
                return
            if vals is None:
                not_impl(e)
            if not vals:
                emit(OP_LIT_BOOL, 0)  # CTList(CTVoid) → FALSE (:115)
                return
            lt = static_type(e.lhs)
            cand = [v for v in vals if _value_type(v) is not None and _comparable(lt, _value_type(v))]
            if any(_value_type(v) is None for v in vals):
                not_impl(e)  # nested lists / maps
            if not cand:
                emit(OP_LIT_NULL, T_BOOL)  # no element could be of lhs's type (:117)
                return
            vals_nn = [v for v in cand if v is not None]
            same = (lt == T_INT and all(_value_type(v) == T_INT for v in vals_nn)) or \
                (lt == T_STRING and intern is not None and all(isinstance(v, str) for v in vals_nn))
            if lset is not None and same and len(cand) >= IN_SET_MIN:
                # a long list: one binary search per row in a sorted session set
                # (an element NULL → a miss is NULL, as the OR of equalities gives)
                codes = tuple(sorted(set(intern(v) if lt == T_STRING else int(v) for v in vals_nn)))
                go(e.lhs)
                emit(OP_IN_SET, name_of(lset(codes)), 1.0 if len(vals_nn) < len(cand) else 0.0)
                return
            # left-folded 3-valued OR of equalities: stack depth 3 whatever the list length
            for k, v in enumerate(cand):
                go(e.lhs)
                lit(v)
                emit(OP_EQ)
                if k:
                    emit(OP_OR, 2)
        elif isinstance(e, ContainerIndex):
            container_index(e)
        elif cls == "Size" and type(e.expr).__name__ in ("Labels", "Keys") and isinstance(e.expr.expr, Var):
            # size(labels(n)) / size(keys(n)): the number of TRUE label flags /
            # of property columns holding a value, summed per row
            cols, kinds, _ = name_list_columns(e.expr, header, columns)
            emit(OP_LIT_INT, 0)
            for c, k in zip(cols, kinds):
                emit(OP_LIT_INT, 0)  # else
                col(c)
                if k == 1:
                    emit(OP_IS_NOT_NULL)
                emit(OP_LIT_INT, 1)  # then
                emit(OP_IF)
                emit(OP_ADD)
        elif cls == "Size":
            x = e.expr
            vals = list_values(x, params) if isinstance(x, (ListLit, Param)) else None
            if vals is not None:
                emit(OP_LIT_INT, len(vals))
                return
            if isinstance(x, StringLit) or (isinstance(x, Param) and isinstance((params or {}).get(x.pname), str)):
                emit(OP_LIT_INT, java_length(x.v if isinstance(x, StringLit) else params[x.pname]))
                return
            if isinstance(x, (NullLit, Param)):
                emit(OP_LIT_NULL, T_INT)
                return
            c = column_of(x)
            t = static_type(x)
            if c is not None and t == T_LIST:
                emit(OP_LIST_SIZE, name_of(c))
            elif t == T_STRING:
                go(x)
                emit(OP_STR_LEN)
            elif t == T_NULL:
                emit(OP_LIT_NULL, T_INT)
            else:
                not_impl(e)
        elif cls == "Type":
            v = e.expr
            if isinstance(v, NullLit):
                emit(OP_LIT_NULL, T_STRING)  # type(null) is null (MTa/NullTests.scala:49)
                return
            if not isinstance(v, Var):
                not_impl(e)  # only variables (:161-162)
            types = sorted((h.rel_type, c) for h, c in (header.items() if header is not None else ())
                           if isinstance(h, HasType) and h.owner == v and c in columns)
            emit(OP_LIT_NULL, T_STRING)
            for ty, c in types:  # acc ← HasType(v, ty) ? 'ty' : acc
                col(c)
                lit(ty)
                emit(OP_IF)
        else:
            from ._lib import NotImplementedException
            raise NotImplementedException(
                f"No support for converting Cypher expression {e} to a GPU expression")

    go(expr)
    return ops, ia, fa, names


@dataclass(frozen=True)
class Collect(Aggregator):
    """collect(e) / collect(DISTINCT e) (okapi Expr.scala Collect; Flink
    child0.collect, FlinkSQLExprMapper.scala:283): the non-NULL values of the
    group as a list.  Flink's COLLECT is a MULTISET, so element order is not
    part of the result (tests compare lists as bags)."""
    expr: Expr
    distinct: bool = False
    kind = AGG_COLLECT

    def __str__(self):
        return f"collect({'DISTINCT ' if self.distinct else ''}{self.expr})"


@dataclass(frozen=True)
class StDev(Aggregator):
    """stDev(e) (Expr.scala:1120-1123): Flink child0.stddevSamp
    (FlinkSQLExprMapper.scala:223) — the sample standard deviation of the
    non-NULL values as a FLOAT, NULL with fewer than two values."""
    expr: Expr
    kind = AGG_STDEV

    def __str__(self):
        return f"stDev({self.expr})"


@dataclass(frozen=True)
class StDevP(Aggregator):
    """stDevP(e) (Expr.scala:1125-1128): Flink child0.stddevPop (:224),
    NULL without values."""
    expr: Expr
    kind = AGG_STDEV_POP

    def __str__(self):
        return f"stDevP({self.expr})"


def percentile_value(p, params=None):
    """The percentile argument: a float / integer literal or parameter (the
    Spark backend requires a literal, SparkSQLExprMapper.scala:451-462)."""
    from ._lib import IllegalArgumentException
    v = p
    if isinstance(p, (FloatLit, IntegerLit)):
        v = p.v
    elif isinstance(p, Param):
        v = (params or {}).get(p.pname)
    if isinstance(v, bool) or not isinstance(v, (int, float)):
        raise IllegalArgumentException(f"Literal as percentage for percentile, got {p}")
    v = float(v)
    if not 0.0 <= v <= 1.0:
        raise IllegalArgumentException(f"percentile must be between 0.0 and 1.0, got {v}")
    return v


@dataclass(frozen=True)
class PercentileCont(Aggregator):
    """percentileCont(e, p) (Expr.scala:1096-1106), the Spark backend's UDAF
    semantics (PercentileUdafs.scala:83-96): linear interpolation, a FLOAT."""
    expr: Expr
    percentile: object
    kind = AGG_PERCENTILE_CONT

    def __str__(self):
        return f"percentileCont({self.expr}, {self.percentile})"


@dataclass(frozen=True)
class PercentileDisc(Aggregator):
    """percentileDisc(e, p) (Expr.scala:1108-1118; PercentileUdafs.scala:
    59-81): the value at rank round(n·p), in the input's type."""
    expr: Expr
    percentile: object
    kind = AGG_PERCENTILE_DISC

    def __str__(self):
        return f"percentileDisc({self.expr}, {self.percentile})"


def aggregators_in(e):
    """Aggregator sub-expressions of a projection item, outermost first
    (RETURN round(stDev(x) * 1000) / 1000.0 aggregates stDev(x), then
    projects the rest over it)."""
    if isinstance(e, Aggregator):
        return [e]
    out = []
    for name in ("lhs", "rhs", "expr"):
        c = getattr(e, name, None)
        if isinstance(c, Expr):
            out += aggregators_in(c)
    for c in getattr(e, "exprs", ()) or ():
        if isinstance(c, Expr):
            out += aggregators_in(c)
    if isinstance(e, CaseExpr):
        for p, v in e.alternatives:
            out += aggregators_in(p) + aggregators_in(v)
        if isinstance(e.default, Expr):
            out += aggregators_in(e.default)
    return out


def replace_exprs(e, m):
    """`e` with every sub-expression found in the dict m replaced."""
    if e in m:
        return m[e]
    import dataclasses
    if isinstance(e, CaseExpr):
        return CaseExpr([(replace_exprs(p, m), replace_exprs(v, m)) for p, v in e.alternatives],
                        None if e.default is None else replace_exprs(e.default, m))
    if isinstance(e, (Ands, Ors, Coalesce)):
        return type(e)(*[replace_exprs(x, m) for x in e.exprs])
    if dataclasses.is_dataclass(e) and not isinstance(e, (Var, ElementProperty)):
        ch = {f.name: replace_exprs(getattr(e, f.name), m) for f in dataclasses.fields(e)
              if isinstance(getattr(e, f.name), Expr)}
        if ch:
            return dataclasses.replace(e, **ch)
    return e


# ----------------------------------------------------------- hash caching
# Expressions are immutable and are looked up in RecordHeader dicts many times
# per plan: each one's hash is computed once and kept on the instance (never
# pickled — str hashes differ between processes).
def _cached_hash(gen):
    def __hash__(self):
        try:
            return self.__dict__["_hc"]
        except KeyError:
            h = gen(self)
            self.__dict__["_hc"] = h
            return h
    return __hash__


def _expr_getstate(self):
    d = dict(self.__dict__)
    d.pop("_hc", None)
    d.pop("_mk", None)
    return d


def _all_subclasses(cls):
    for c in cls.__subclasses__():
        yield c
        yield from _all_subclasses(c)


Expr.__getstate__ = _expr_getstate
for _cls in list(_all_subclasses(Expr)):
    if "__dataclass_fields__" in _cls.__dict__ and _cls.__dict__.get("__hash__") is not None:
        _cls.__hash__ = _cached_hash(_cls.__dict__["__hash__"])
