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

# aggregators
AGG_COUNT_STAR, AGG_COUNT, AGG_SUM, AGG_MIN, AGG_MAX, AGG_AVG, AGG_COLLECT = 0, 1, 2, 3, 4, 5, 6


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


Id = _unary("Id", "id({})")            # FlinkSQLExprMapper.scala:134: the element's id column
Exists = _unary("Exists", "exists({})")  # exists(n.prop) → IS NOT NULL (:90)
Size = _unary("Size", "size({})")      # charLength / cardinality (:80-85)
Type = _unary("Type", "type({})")      # the relationship's type name (:152-160)


def java_length(v):
    """Java String.length: UTF-16 code units."""
    return len(v.encode("utf-16-le")) // 2


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
_UN_OPS = {"Not": OP_NOT, "IsNull": OP_IS_NULL, "IsNotNull": OP_IS_NOT_NULL, "ToFloat": OP_TO_FLOAT,
           "ToInteger": OP_TO_INTEGER, "Negate": OP_NEG, "Exists": OP_IS_NOT_NULL}


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


def resolve_column(expr, header, columns):
    """Physical column of a header expression or None (→ NULL literal)."""
    col = header.get(expr) if header is not None else None
    if col is not None and col in columns:
        return col
    return None


def compile_program(expr, header, columns, params=None, intern=None, coltype=None):
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
        if isinstance(e, (ToFloat,)):
            return T_FLOAT
        if isinstance(e, (ToInteger, Size, Id)):
            return T_INT
        return None

    def not_impl(what):
        from ._lib import NotImplementedException
        raise NotImplementedException(f"No support for converting Cypher expression {what} to a GPU expression")

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
        elif cls in _BIN_OPS:
            go(e.lhs)
            go(e.rhs)
            emit(_BIN_OPS[cls])
        elif cls in _UN_OPS:
            go(e.expr)
            emit(_UN_OPS[cls])
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
        elif isinstance(e, In):
            vals = list_values(e.rhs, params)
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
            # left-folded 3-valued OR of equalities: stack depth 3 whatever the list length
            for k, v in enumerate(cand):
                go(e.lhs)
                lit(v)
                emit(OP_EQ)
                if k:
                    emit(OP_OR, 2)
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


# Aggregators of the okapi IR that the Flink backend does not map
# (FlinkSQLExprMapper.scala:281-290 has no case for them): planning them raises
# NotImplementedException, as the reference does.
@dataclass(frozen=True)
class StDev(Aggregator):
    expr: Expr

    def __str__(self):
        return f"stDev({self.expr})"


@dataclass(frozen=True)
class StDevP(Aggregator):
    expr: Expr

    def __str__(self):
        return f"stDevP({self.expr})"


@dataclass(frozen=True)
class PercentileCont(Aggregator):
    expr: Expr
    percentile: float

    def __str__(self):
        return f"percentileCont({self.expr}, {self.percentile})"


@dataclass(frozen=True)
class PercentileDisc(Aggregator):
    expr: Expr
    percentile: float

    def __str__(self):
        return f"percentileDisc({self.expr}, {self.percentile})"


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
    return d


def _all_subclasses(cls):
    for c in cls.__subclasses__():
        yield c
        yield from _all_subclasses(c)


Expr.__getstate__ = _expr_getstate
for _cls in list(_all_subclasses(Expr)):
    if "__dataclass_fields__" in _cls.__dict__ and _cls.__dict__.get("__hash__") is not None:
        _cls.__hash__ = _cached_hash(_cls.__dict__["__hash__"])
