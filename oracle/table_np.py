"""numpy restatement of the Flink Table[T] semantics — TEST INFRASTRUCTURE ONLY.

OracleTable implements the same SPI as the product GpuTable
(okapi-relational/.../api/table/Table.scala:43-178) with the semantics of
FlinkTable (flink-cypher/.../impl/table/FlinkTable.scala:49-199):

 * select / drop: projection (FlinkTable.scala:63-74, 100-103);
 * filter: expression lowered as FlinkSQLExprMapper.asFlinkSQLExpr
   (FlinkSQLExprMapper.scala:48-294) under SQL three-valued logic; only TRUE
   rows survive (FlinkTable.scala:76-78);
 * join: equi-join, `true && l1 === r1 && ...` — NULL keys never match
   (FlinkTable.scala:171-187); disjoint columns asserted (:173-174);
 * unionAll: bag union, rhs columns matched by name (FlinkTable.scala:152-169);
 * distinct(cols): one row per distinct value of cols (Spark dropDuplicates,
   morpheus-spark-cypher/.../SparkTable.scala:198-200; the Flink version is
   broken);
 * group: GROUP BY the owned columns with NULL as its own group; aggregators
   per FlinkSQLExprMapper.scala:281-287 (count(*) counts rows; count(e)
   non-null; sum/min/max/avg ignore NULL and are NULL on no input; avg of an
   INTEGER column is an INTEGER, Java long division — Expr.scala:1058-1066);
 * collect: the group's non-NULL values as a list (DISTINCT drops repeats);
   Flink's COLLECT is a MULTISET (FlinkSQLExprMapper.scala:283), so the
   element order is not part of the result;
 * orderBy: NULL sorts as the largest value;
 * withColumns: replace in place or append (FlinkTable.scala:86-98).

Everything materialises with numpy; sizes are the small parity cases.
"""
import numpy as np

import math
import re
from decimal import Decimal, localcontext
from fractions import Fraction

from capf_amd.expr import (T_BOOL, T_FLOAT, T_INT, T_LIST, T_NULL, T_STRING, CAPF_TO_CT, CT_TO_CAPF,
                           Aggregator, Ands, BoolLit, CaseExpr, Coalesce, E_, ElementProperty, EndNode, Explode,
                           FloatLit, HasLabel, HasType, IntegerLit, ListLit, NullLit, Ors, Param, Pi_, StartNode,
                           StringLit, Var, AGG_AVG, AGG_COLLECT, AGG_COUNT, AGG_COUNT_STAR, AGG_MAX, AGG_MIN,
                           AGG_PERCENTILE_CONT, AGG_PERCENTILE_DISC, AGG_STDEV, AGG_STDEV_POP, AGG_SUM,
                           explode_values, percentile_value)


def list_values(e, params):
    """Values of a list literal or list parameter (None: not one)."""
    if isinstance(e, ListLit):
        out = []
        for x in e.items:
            if isinstance(x, NullLit):
                out.append(None)
            elif isinstance(x, Param):
                out.append((params or {}).get(x.pname))
            elif isinstance(x, (IntegerLit, FloatLit, StringLit, BoolLit)):
                out.append(x.v)
            else:
                return None
        return out
    if isinstance(e, Param):
        v = (params or {}).get(e.pname)
        return list(v) if isinstance(v, (list, tuple)) else None
    return None


def java_length(v):
    """java.lang.String.length(): UTF-16 code units."""
    return len(v.encode("utf-16-le", "surrogatepass")) // 2


class Col:
    __slots__ = ("t", "v", "ok")

    def __init__(self, t, v, ok):
        self.t = t
        self.v = v
        self.ok = np.asarray(ok, dtype=bool)

    def take(self, idx):
        idx = np.asarray(idx, dtype=np.int64)
        neg = idx < 0
        safe = np.where(neg, 0, idx)
        if len(self.v) == 0:
            v = np.zeros(len(idx), dtype=self.v.dtype) if self.v.dtype != object else np.full(len(idx), None, dtype=object)
            return Col(self.t, v, np.zeros(len(idx), dtype=bool))
        return Col(self.t, self.v[safe], np.where(neg, False, self.ok[safe]))


_NP = {T_INT: np.int64, T_FLOAT: np.float64, T_BOOL: np.bool_, T_STRING: object, T_NULL: np.int64,
       T_LIST: object}


def _empty_vals(t, n):
    if t in (T_STRING, T_LIST):
        return np.full(n, None, dtype=object)
    return np.zeros(n, dtype=_NP[t])


class OracleSession:
    def table(self, columns, nrows=None):
        cols = {}
        order = []
        n = nrows
        for name, t, values, valid in columns:
            lst = list(values)
            m = len(lst)
            n = m if n is None else n
            ok = np.array([x is not None for x in lst], dtype=bool) if valid is None else np.asarray(valid, bool)
            if t == T_STRING:
                v = np.array(lst, dtype=object)
            elif t == T_LIST:  # one Python list per row (np.array would build a 2-D array)
                v = np.empty(m, dtype=object)
                for i, x in enumerate(lst):
                    v[i] = list(x) if x is not None else []
            elif t == T_NULL:
                v = np.zeros(m, dtype=np.int64)
                ok = np.zeros(m, dtype=bool)
            else:
                v = np.array([x if x is not None else 0 for x in lst], dtype=_NP[t])
            cols[name] = Col(t, v, ok)
            order.append(name)
        return OracleTable(order, cols, n or 0)

    def unit(self):
        return OracleTable([], {}, 1)

    def empty(self, names, types):
        return OracleTable(list(names), {c: Col(t, _empty_vals(t, 0), []) for c, t in zip(names, types)}, 0)

    def intern(self, s):
        return s


# ------------------------------------------------------------ expressions
class Val:
    """Vectorised value: type, values, validity."""
    __slots__ = ("t", "v", "ok")

    def __init__(self, t, v, ok):
        self.t, self.v, self.ok = t, v, np.asarray(ok, dtype=bool)


def _num(x):
    if x.t == T_FLOAT:
        return x.v.astype(np.float64)
    if x.t == T_BOOL:
        return x.v.astype(np.int64)
    return x.v


def _jcmp(x, y):
    """java.lang.String.compareTo sign: UTF-16 code-unit order."""
    kx, ky = x.encode("utf-16-be", "surrogatepass"), y.encode("utf-16-be", "surrogatepass")
    return (kx > ky) - (kx < ky)


def _cmp(a, b, op):
    ok = a.ok & b.ok
    if a.t == T_NULL or b.t == T_NULL:
        return Val(T_BOOL, np.zeros(len(ok), bool), np.zeros(len(ok), bool))
    if a.t == T_STRING or b.t == T_STRING:
        if a.t != b.t:
            if op not in ("eq", "ne"):  # Cypher: incomparable operands order to NULL
                return Val(T_BOOL, np.zeros(len(ok), bool), np.zeros(len(ok), bool))
            raise TypeError("cannot compare STRING with non-string")
        if op not in ("eq", "ne"):  # String.compareTo: UTF-16 code units (= UTF-16-BE bytes)
            f = {"lt": lambda c: c < 0, "le": lambda c: c <= 0, "gt": lambda c: c > 0, "ge": lambda c: c >= 0}[op]
            r = np.array([f(_jcmp(x, y)) if (p and q) else False for x, y, p, q in zip(a.v, b.v, a.ok, b.ok)],
                         dtype=bool)
            return Val(T_BOOL, r, ok)
        r = np.array([(x == y) if (p and q) else False for x, y, p, q in zip(a.v, b.v, a.ok, b.ok)], dtype=bool)
        return Val(T_BOOL, r if op == "eq" else ~r, ok)
    if (a.t == T_BOOL) != (b.t == T_BOOL) and op not in ("eq", "ne"):
        return Val(T_BOOL, np.zeros(len(ok), bool), np.zeros(len(ok), bool))
    x, y = _num(a), _num(b)
    with np.errstate(invalid="ignore"):
        r = {"eq": x == y, "ne": x != y, "lt": x < y, "le": x <= y, "gt": x > y, "ge": x >= y}[op]
    return Val(T_BOOL, np.asarray(r, bool), ok)


def _arith(a, b, op):
    n = len(a.ok)
    ok = a.ok & b.ok
    fl = a.t == T_FLOAT or b.t == T_FLOAT
    if a.t in (T_STRING, T_BOOL) or b.t in (T_STRING, T_BOOL):
        raise NotImplementedError("arithmetic on non-numeric values")
    if fl:
        x, y = _num(a).astype(np.float64), _num(b).astype(np.float64)
        with np.errstate(all="ignore"):
            r = {"add": x + y, "sub": x - y, "mul": x * y, "div": x / y, "mod": np.fmod(x, y)}[op]
        return Val(T_FLOAT, r, ok)
    x, y = a.v.astype(np.int64), b.v.astype(np.int64)
    r = np.zeros(n, dtype=np.int64)
    with np.errstate(all="ignore"):
        if op == "add":
            r = x + y
        elif op == "sub":
            r = x - y
        elif op == "mul":
            r = x * y
        else:
            zero = y == 0
            ok = ok & ~zero
            ys = np.where(zero, 1, y)
            # Java long division truncates toward zero
            q = np.abs(x) // np.abs(ys) * np.sign(x) * np.sign(ys)
            r = q if op == "div" else x - q * ys
    return Val(T_INT, r, ok)


def evaluate(e, table, header, params):
    n = table._n
    cols = table._cols

    def const(t, value, valid=True):
        if t == T_STRING:
            return Val(t, np.full(n, value, dtype=object), np.full(n, valid))
        return Val(t, np.full(n, value if value is not None else 0, dtype=_NP[t]), np.full(n, valid))

    def col_of(x):
        c = header.get(x) if header is not None else None
        if c is not None and c in cols:
            k = cols[c]
            return Val(k.t, k.v, k.ok)
        return None

    def go(x):
        if isinstance(x, (Var, HasLabel, HasType, StartNode, EndNode, ElementProperty)):
            v = col_of(x)
            if v is not None:
                return v
            ct = getattr(x, "ctype", "BOOLEAN" if isinstance(x, (HasLabel, HasType)) else "INTEGER")
            t = CT_TO_CAPF.get(ct, T_NULL)
            return const(t, None, False)
        v = col_of(x) if header is not None and x in header else None
        if v is not None:
            return v
        name = type(x).__name__
        if isinstance(x, IntegerLit):
            return const(T_INT, x.v)
        if isinstance(x, FloatLit):
            return const(T_FLOAT, x.v)
        if isinstance(x, BoolLit):
            return const(T_BOOL, x.v)
        if isinstance(x, StringLit):
            return const(T_STRING, x.v)
        if isinstance(x, NullLit):
            return const(CT_TO_CAPF.get(x.ctype, T_NULL), None, False)
        if isinstance(x, ListLit) or (isinstance(x, Param) and isinstance(params.get(x.pname), (list, tuple))):
            # a list value per row (FlinkSQLExprMapper.scala:71 array(...), :75):
            # INTEGER elements widen to FLOAT beside a FLOAT one
            items = [go(y) for y in x.items] if isinstance(x, ListLit) else None
            vals = list(params[x.pname]) if items is None else None
            out = np.empty(n, dtype=object)
            for i in range(n):
                row = vals if items is None else [(y.v[i].item() if hasattr(y.v[i], "item") else y.v[i])
                                                  if y.ok[i] else None for y in items]
                if any(isinstance(v, float) for v in row):
                    row = [float(v) if isinstance(v, int) and not isinstance(v, bool) else v for v in row]
                out[i] = list(row)
            return Val(T_LIST, out, np.ones(n, bool))
        if isinstance(x, Param):
            p = params[x.pname]
            if p is None:
                return const(T_NULL, None, False)
            t = T_BOOL if isinstance(p, bool) else T_INT if isinstance(p, int) else T_FLOAT if isinstance(p, float) else T_STRING
            return const(t, p)
        cmp_ops = {"Equals": "eq", "LessThan": "lt", "LessThanOrEqual": "le", "GreaterThan": "gt",
                   "GreaterThanOrEqual": "ge"}
        if name in cmp_ops:
            return _cmp(go(x.lhs), go(x.rhs), cmp_ops[name])
        if name == "Add":  # string concatenation (FlinkSQLExprMapper.scala:120-128)
            a, b = go(x.lhs), go(x.rhs)
            if T_STRING in (a.t, b.t):
                if {a.t, b.t} - {T_STRING, T_INT, T_FLOAT, T_NULL}:
                    raise NotImplementedError(f"oracle: {x}")
                out = np.array([_jstr(u, a.t) + _jstr(v, b.t) if oa and ob else None
                                for u, v, oa, ob in zip(a.v, b.v, a.ok, b.ok)], dtype=object)
                return Val(T_STRING, out, a.ok & b.ok)
        ar_ops = {"Add": "add", "Subtract": "sub", "Multiply": "mul", "Divide": "div", "Modulo": "mod"}
        if name in ar_ops:
            return _arith(go(x.lhs), go(x.rhs), ar_ops[name])
        if name == "Not":
            a = go(x.expr)
            return Val(T_BOOL, ~a.v.astype(bool), a.ok)
        if name == "IsNull":
            a = go(x.expr)
            return Val(T_BOOL, ~a.ok, np.ones(n, bool))
        if name == "IsNotNull":
            a = go(x.expr)
            return Val(T_BOOL, a.ok.copy(), np.ones(n, bool))
        if name == "Negate":
            a = go(x.expr)
            return Val(a.t, -a.v, a.ok)
        if name in ("ToFloat", "ToInteger") and x.expr is not None:
            a = go(x.expr)
            if a.t == T_STRING:  # CAST(string AS DOUBLE / INT): see _parse_double / _parse_int
                f = _parse_double if name == "ToFloat" else _parse_int
                vals = [f(v) if ok else None for v, ok in zip(a.v, a.ok)]
                t = T_FLOAT if name == "ToFloat" else T_INT
                return Val(t, np.array([0 if v is None else v for v in vals], dtype=_NP[t]),
                           np.array([v is not None for v in vals], bool))
        if name == "ContainerIndex" and isinstance(x.container, Var) and x.container.ctype == "MAP":
            # m[key] on a MAP held as a struct of columns: the entry's column
            key = x.index.v if isinstance(x.index, StringLit) else (
                params.get(x.index.pname) if isinstance(x.index, Param) else None)
            if key is None and not isinstance(x.index, (StringLit, Param, NullLit)):
                raise NotImplementedError("oracle: a per-row map key")
            return go(ElementProperty(x.container, key)) if key is not None else const(T_NULL, None, False)
        if name == "ContainerIndex":  # xs[i], 0-based, negative from the end, NULL out of range
            ix = go(x.index)
            lits = list_values(x.container, params) if isinstance(x.container, (ListLit, Param)) else None
            if lits is not None:
                rows = [lits] * n
                okc = np.ones(n, bool)
            else:
                c = go(x.container)
                if c.t == T_NULL:
                    return const(T_NULL, None, False)
                if c.t != T_LIST:
                    raise NotImplementedError(f"oracle: index into {CAPF_TO_CT[c.t]}")
                rows, okc = list(c.v), c.ok
            elems = [v for r in rows for v in r if v is not None]
            t = (T_FLOAT if any(isinstance(v, float) for v in elems) else
                 T_BOOL if elems and isinstance(elems[0], bool) else
                 T_STRING if elems and isinstance(elems[0], str) else T_INT if elems else T_NULL)
            out, ok = [], []
            for r, rok, i, iok in zip(rows, okc, ix.v, ix.ok):
                k = int(i) + len(r) if iok and int(i) < 0 else int(i)
                hit = bool(rok and iok and 0 <= k < len(r) and r[k] is not None)
                v = r[k] if hit else None
                out.append(float(v) if hit and t == T_FLOAT else v)
                ok.append(hit)
            if t == T_STRING:
                return Val(t, np.array(out, dtype=object), np.array(ok, bool))
            return Val(t, np.array([0 if v is None else v for v in out], dtype=_NP[t]), np.array(ok, bool))
        if name == "RegexMatch":  # whole-string regex match (Java String.matches)
            a, pt = go(x.lhs), go(x.rhs)
            if a.t not in (T_STRING, T_NULL) or pt.t not in (T_STRING, T_NULL):
                raise NotImplementedError("oracle: =~ of non-strings")
            hit = [bool(ao and po and re.fullmatch(p_, v) is not None)
                   for v, p_, ao, po in zip(a.v, pt.v, a.ok, pt.ok)]
            return Val(T_BOOL, np.array(hit, bool), a.ok & pt.ok)
        if name == "Rand_":  # rand(): uniform in [0, 1) per row
            return Val(T_FLOAT, np.random.default_rng().random(n), np.ones(n, bool))
        if name in ("Labels", "Keys") and isinstance(x.expr, NullLit):
            return const(T_NULL, None, False)
        if name == "ToFloat":
            a = go(x.expr)
            if a.t == T_BOOL:
                return const(T_FLOAT, None, False)
            return Val(T_FLOAT, _num(a).astype(np.float64), a.ok)
        if name == "ToInteger":
            # Flink: cast to INT (32 bit), FlinkSQLExprMapper.scala:183
            a = go(x.expr)
            if a.t == T_BOOL:
                return const(T_INT, None, False)
            if a.t == T_FLOAT:
                f = np.nan_to_num(a.v.astype(np.float64), nan=0.0)
                r = np.clip(np.trunc(f), -2 ** 31, 2 ** 31 - 1).astype(np.int64)
            else:
                r = a.v.astype(np.int64).astype(np.int32).astype(np.int64)
            return Val(T_INT, r, a.ok)
        if isinstance(x, (Ands, Ors)):
            vals = [go(y) for y in x.exprs]
            is_and = isinstance(x, Ands)
            if not vals:
                return const(T_BOOL, is_and)
            dom = np.zeros(n, bool)
            anynull = np.zeros(n, bool)
            for a in vals:
                b = a.v.astype(bool)
                dom |= a.ok & (~b if is_and else b)
                anynull |= ~a.ok
            res = np.full(n, not is_and) if True else None
            res = np.where(dom, not is_and, is_and)
            ok = dom | ~anynull
            return Val(T_BOOL, res.astype(bool), ok)
        if name == "Id":  # the element's id column (FlinkSQLExprMapper.scala:134)
            return go(x.expr)
        if name == "Exists":  # exists(n.prop) (:90)
            a = go(x.expr)
            return Val(T_BOOL, a.ok.copy(), np.ones(n, bool))
        if name == "In":  # SQL IN over a literal / parameter list (:114-118)
            items = list_values(x.rhs, params)
            if items is None and (isinstance(x.rhs, NullLit) or
                                  (isinstance(x.rhs, Param) and params.get(x.rhs.pname) is None)):
                return const(T_BOOL, None, False)  # x IN null (MTa/NullTests.scala:98)
            if items is None:
                raise NotImplementedError(f"oracle: IN over {x.rhs}")
            if not items:
                return const(T_BOOL, False)
            a = go(x.lhs)
            kind = lambda v: (None if v is None else "num" if isinstance(v, (int, float)) and not isinstance(v, bool)  # noqa: E731
                              else type(v).__name__)
            lk = {T_INT: "num", T_FLOAT: "num", T_STRING: "str", T_BOOL: "bool"}.get(a.t)
            cand = [v for v in items if v is None or lk is None or kind(v) == lk]
            if not cand:
                return const(T_BOOL, None, False)
            hit = np.zeros(n, bool)
            vals = a.v
            for v in cand:
                if v is not None:
                    hit |= np.array([ok and (u == v) for u, ok in zip(vals, a.ok)], dtype=bool)
            has_null = any(v is None for v in cand)
            ok = a.ok & (hit | (not has_null))
            return Val(T_BOOL, hit, ok)
        if name == "Size":  # charLength / cardinality (:80-85)
            items = list_values(x.expr, params) if isinstance(x.expr, (ListLit, Param)) else None
            if items is not None:
                return const(T_INT, len(items))
            a = go(x.expr)
            if a.t == T_NULL:
                return const(T_INT, None, False)
            if a.t == T_STRING:
                r = np.array([java_length(v) if ok else 0 for v, ok in zip(a.v, a.ok)], dtype=np.int64)
            elif a.t == T_LIST:
                r = np.array([len(v) if ok else 0 for v, ok in zip(a.v, a.ok)], dtype=np.int64)
            else:
                raise NotImplementedError(f"oracle: size of {CAPF_TO_CT[a.t]}")
            return Val(T_INT, r, a.ok.copy())
        if name == "Type":  # the type whose HasType column is true (:152-160)
            if isinstance(x.expr, NullLit):
                return const(T_STRING, None, False)
            out = np.full(n, None, dtype=object)
            ok = np.zeros(n, bool)
            for h, c in (header.items() if header is not None else ()):
                if isinstance(h, HasType) and h.owner == x.expr and c in cols:
                    k = cols[c]
                    t = k.ok & k.v.astype(bool)
                    out[t] = h.rel_type
                    ok |= t
            return Val(T_STRING, out, ok)
        if name in _MATH1:
            return _math1(name, go(x.expr), n)
        if name == "Atan2":  # atan2(child0, child1) (FlinkSQLExprMapper.scala:207)
            y, z = go(x.lhs), go(x.rhs)
            with np.errstate(all="ignore"):
                return Val(T_FLOAT, np.arctan2(_num(y).astype(np.float64), _num(z).astype(np.float64)), y.ok & z.ok)
        if name == "Cot":  # Divide(IntegerLit(1), Tan(e)) (:208)
            t = _math1("Tan", go(x.expr), n)
            return _arith(const(T_INT, 1), t, "div")
        if name == "Haversin":  # Divide(Subtract(1, Cos(e)), 2) (:210)
            c = _math1("Cos", go(x.expr), n)
            return _arith(_arith(const(T_INT, 1), c, "sub"), const(T_INT, 2), "div")
        if isinstance(x, E_):
            return const(T_FLOAT, math.e)
        if isinstance(x, Pi_):
            return const(T_FLOAT, math.pi)
        if name in ("StartNodeFunction", "EndNodeFunction"):  # (:179-180)
            return go(StartNode(x.expr) if name == "StartNodeFunction" else EndNode(x.expr))
        if name == "ToBoolean":  # cast to BOOLEAN (:185)
            a = go(x.expr)
            if a.t in (T_BOOL, T_NULL):
                return Val(T_BOOL, a.v.astype(bool), a.ok.copy())
            if a.t != T_STRING:
                raise NotImplementedError(f"oracle: toBoolean of {CAPF_TO_CT[a.t]}")
            parsed = [(str(v).strip().lower() if ok else None) for v, ok in zip(a.v, a.ok)]
            return Val(T_BOOL, np.array([p == "true" for p in parsed], bool),
                       np.array([p in ("true", "false") for p in parsed], bool))
        if name in _STR1 or name in ("Substring", "Replace"):  # (:187-195)
            a = go(x.expr)
            if a.t == T_NULL:
                return const(T_STRING, None, False)
            if a.t != T_STRING:
                raise NotImplementedError(f"oracle: {name} of {CAPF_TO_CT[a.t]}")
            if name == "Substring":
                st = go(x.start)
                ln = go(x.length) if x.length is not None else const(T_INT, 1)  # (:195: default 1)
                args = [(int(u), int(w), ou and ow) for u, w, ou, ow in zip(st.v, ln.v, st.ok, ln.ok)]
                out = [_substring(v, u + 1, w) if ok and aok else None for v, aok, (u, w, ok) in zip(a.v, a.ok, args)]
            elif name == "Replace":
                se, rp = go(x.search), go(x.replacement)
                out = [re.sub(p1, lambda m, r=p2: r, v) if ok and o1 and o2 else None
                       for v, ok, p1, p2, o1, o2 in zip(a.v, a.ok, se.v, rp.v, se.ok, rp.ok)]
            else:
                f = _STR1[name]
                out = [f(v) if ok else None for v, ok in zip(a.v, a.ok)]
            ok = np.array([v is not None for v in out], bool)
            return Val(T_STRING, np.array(out, dtype=object), ok)
        if name in ("Labels", "Keys"):  # GetLabels / GetKeys (FlinkSQLExprMapper.scala:136-153, 310-329)
            found = []
            for h, c in (header.items() if header is not None else ()):
                if c not in cols:
                    continue
                if name == "Labels" and isinstance(h, HasLabel) and h.owner == x.expr:
                    found.append((h.label, cols[c], True))
                elif name == "Keys" and isinstance(h, ElementProperty) and h.owner == x.expr:
                    found.append((h.key, cols[c], False))
            found.sort(key=lambda f: f[0])
            out = np.empty(n, dtype=object)
            for i in range(n):
                out[i] = [nm for nm, k, flag in found if k.ok[i] and (bool(k.v[i]) if flag else True)]
            return Val(T_LIST, out, np.ones(n, bool))
        if name == "ToString":  # cast to STRING (:184)
            a = go(x.expr)
            if a.t == T_NULL:
                return const(T_STRING, None, False)
            out = np.array([_jstr(v, a.t) if ok else None for v, ok in zip(a.v, a.ok)], dtype=object)
            return Val(T_STRING, out, a.ok.copy())
        if isinstance(x, CaseExpr):  # If(p1, v1, If(p2, v2, … default)) (:242-260)
            acc = go(x.default) if x.default is not None else const(T_INT, None, False)
            for p, v in reversed(x.alternatives):
                c, val = go(p), go(v)
                take = c.ok & c.v.astype(bool)
                t = val.t if val.t != T_NULL else acc.t
                if T_NULL not in (val.t, acc.t) and val.t != acc.t:
                    if {val.t, acc.t} <= {T_INT, T_FLOAT}:
                        t = T_FLOAT
                    else:
                        raise TypeError("branches of different types")
                vv = _num(val).astype(np.float64) if t == T_FLOAT else val.v
                av = _num(acc).astype(np.float64) if t == T_FLOAT else acc.v
                if t == T_NULL:
                    acc = Val(T_NULL, np.zeros(n, np.int64), np.zeros(n, bool))
                    continue
                if val.t == T_NULL:
                    vv = _empty_vals(t, n)
                if acc.t == T_NULL:
                    av = _empty_vals(t, n)
                acc = Val(t, np.where(take, vv, av), np.where(take, val.ok, acc.ok))
            return acc
        if isinstance(x, Coalesce):
            vals = [go(y) for y in x.exprs]
            t = T_NULL
            for a in vals:
                if a.t != T_NULL:
                    t = T_FLOAT if (t == T_INT and a.t == T_FLOAT) or (t == T_FLOAT and a.t == T_INT) else (a.t if t == T_NULL else t)
            out = _empty_vals(t, n)
            ok = np.zeros(n, bool)
            for a in vals:
                take = ~ok & a.ok
                if t == T_FLOAT:
                    out[take] = _num(a)[take]
                else:
                    out[take] = a.v[take]
                ok |= a.ok
            return Val(t, out, ok)
        raise NotImplementedError(f"oracle: unsupported expression {x}")

    return go(e)


# Flink's string functions as the JVM runs them (FlinkSQLExprMapper.scala:187-191):
# upperCase / lowerCase, SQL TRIM of the space character
_STR1 = {"ToUpper": str.upper, "ToLower": str.lower, "Trim": lambda v: v.strip(" "),
         "LTrim": lambda v: v.lstrip(" "), "RTrim": lambda v: v.rstrip(" ")}


_DOUBLE_RE = re.compile(r"[+-]?(NaN|Infinity|((\d+\.?\d*|\.\d+)([eE][+-]?\d+)?)[fFdD]?)")
_INT_RE = re.compile(r"[+-]?\d+(\.\d*)?")


def _jtrim(v):
    """java.lang.String.trim: strip chars <= ' '."""
    b, e = 0, len(v)
    while b < e and v[b] <= " ":
        b += 1
    while e > b and v[e - 1] <= " ":
        e -= 1
    return v[b:e]


def _parse_double(v):
    """toFloat(string): Double.valueOf(s.trim()) — decimal / exponent forms,
    NaN, Infinity, an optional f / d suffix; anything else NULL (Flink's CAST
    throws there, the reference expectation is NULL: FunctionTests.scala)."""
    t = _jtrim(v)
    if not _DOUBLE_RE.fullmatch(t):
        return None
    t = t.rstrip("fFdD") if t[-1:] in "fFdD" and "Infinity" not in t else t
    return float(t.replace("Infinity", "inf"))


def _parse_int(v):
    """toInteger(string): the decimal integer, a fractional part truncated
    ('82.9' -> 82, FunctionTests.scala:1117-1127), NULL when unparsable or
    outside INT (32 bit: Flink casts to INT, FlinkSQLExprMapper.scala:183)."""
    t = _jtrim(v)
    if not _INT_RE.fullmatch(t):
        return None
    r = int(t.split(".")[0])
    return r if -2 ** 31 <= r < 2 ** 31 else None


def _substring(v, frm, ln):
    """Calcite SqlFunctions.substring(s, from, for): 1-based, UTF-16 units."""
    u = v.encode("utf-16-le", "surrogatepass")
    n = len(u) // 2
    if ln < 0:
        raise ValueError("negative substring length")
    if frm < 0:
        frm += n + 1
    end = frm + ln
    if frm > n or end < 1:
        return ""
    lo, hi = max(frm, 1), min(end, n + 1)
    return u[2 * (lo - 1):2 * (hi - 1)].decode("utf-16-le", "surrogatepass")


def _jstr(v, t):
    """CAST(v AS VARCHAR) on the JVM: Long.toString, Double.toString, 'true'/'false'."""
    if t == T_STRING:
        return v
    if t == T_BOOL:
        return "true" if v else "false"
    if t == T_INT:
        return str(int(v))
    if t == T_FLOAT:
        d = float(v)
        if d != d:
            return "NaN"
        if d in (math.inf, -math.inf):
            return "Infinity" if d > 0 else "-Infinity"
        if d == 0:
            return "-0.0" if math.copysign(1, d) < 0 else "0.0"
        if 1e-3 <= abs(d) < 1e7:
            r = repr(d)
            if "e" in r:  # repr's exponent form inside the decimal range (e.g. 1e-03)
                r = format(Decimal(r), "f")
            return r if "." in r else r + ".0"
        m, e = f"{d:.17e}".split("e")
        # the shortest round-trip mantissa digits, Java's d.dddE<exp>
        digits = Decimal(repr(d)).normalize()
        sign, dg, ex = digits.as_tuple()
        ds = "".join(map(str, dg))
        exp10 = len(dg) + ex - 1
        mant = ds[0] + "." + (ds[1:] or "0")
        return ("-" if sign else "") + f"{mant}E{exp10}"
    raise NotImplementedError(f"oracle: toString of {CAPF_TO_CT[t]}")


_MATH1 = {"Round", "Abs", "Ceil", "Floor", "Sign", "Sqrt", "Log", "Log10", "Exp", "Sin", "Cos", "Tan", "Asin",
          "Acos", "Atan", "Degrees", "Radians"}


def _math1(name, a, n):
    """FlinkSQLExprMapper.scala:199-221 over doubles (Java Math); ROUND half
    away from zero as a FLOAT (Spark's round(x).cast(Double)); ABS / CEIL /
    FLOOR / SIGN keep an INTEGER operand's type (Calcite ARG0)."""
    keeps = name in ("Abs", "Ceil", "Floor", "Sign")
    if a.t == T_NULL:
        return Val(T_FLOAT, np.zeros(n), np.zeros(n, bool))
    if a.t not in (T_INT, T_FLOAT):
        raise NotImplementedError(f"oracle: {name} of {CAPF_TO_CT[a.t]}")
    if a.t == T_INT and keeps:
        v = a.v.astype(np.int64)
        r = {"Abs": np.abs(v), "Ceil": v, "Floor": v, "Sign": np.sign(v)}[name]
        return Val(T_INT, r.astype(np.int64), a.ok.copy())
    x = _num(a).astype(np.float64)
    with np.errstate(all="ignore"):
        if name == "Round":
            r = np.trunc(x)
            f = x - r
            r = np.where(f >= 0.5, r + 1.0, np.where(f <= -0.5, r - 1.0, r))
        elif name == "Sign":
            r = np.where(x > 0, 1.0, np.where(x < 0, -1.0, x))
        elif name == "Degrees":
            r = x * 180.0 / math.pi
        elif name == "Radians":
            r = x / 180.0 * math.pi
        else:
            r = {"Abs": np.abs, "Ceil": np.ceil, "Floor": np.floor, "Sqrt": np.sqrt, "Log": np.log,
                 "Log10": np.log10, "Exp": np.exp, "Sin": np.sin, "Cos": np.cos, "Tan": np.tan, "Asin": np.arcsin,
                 "Acos": np.arccos, "Atan": np.arctan}[name](x)
    return Val(T_FLOAT, np.asarray(r, dtype=np.float64), a.ok.copy())


def _exact_stdev(vals, samp):
    """The exact standard deviation of floats, rounded once: Fraction mean
    and squared deviations, a 60-digit square root."""
    n = len(vals)
    if n < (2 if samp else 1):
        return None
    fr = [Fraction(v) for v in vals]
    mean = sum(fr) / n
    m2 = sum((f - mean) ** 2 for f in fr) / (n - 1 if samp else n)
    with localcontext() as ctx:
        ctx.prec = 60
        return float((Decimal(m2.numerator) / Decimal(m2.denominator)).sqrt())


def _percentile(vals, p, cont):
    """PercentileUdafs.scala:59-96 (the Spark backend's UDAFs): over the
    ascending values as doubles."""
    sv = sorted(vals)
    n = len(sv)
    if n == 0:
        return None
    if not cont:
        x = n * p
        pos = math.floor(x)
        if x - pos >= 0.5:  # Math.round, ties up
            pos += 1
        return sv[0] if pos == 0 else sv[pos - 1]
    sv = [float(v) for v in sv]
    exact = 1 + ((n - 1) * p)
    prec, succ = math.floor(exact), math.ceil(exact)
    w = succ - exact
    if exact < 1:
        return (1 - w) * sv[succ] + w * sv[prec]
    if exact == succ:
        return sv[prec - 1]
    return (1 - w) * sv[succ - 1] + w * sv[prec - 1]


def _key_codes(cols, null_is_group=True):
    """Joint integer codes of rows over `cols` (NULL → its own code, or -1)."""
    n = len(cols[0].ok) if cols else 0
    parts = []
    anynull = np.zeros(n, bool)
    for c in cols:
        anynull |= ~c.ok
        if c.t == T_LIST:
            raise NotImplementedError("list values as keys")
        if c.t == T_STRING:
            vals = np.array([v if ok else "" for v, ok in zip(c.v, c.ok)], dtype=object)
            _, inv = np.unique(vals.astype(str), return_inverse=True) if n else (None, np.zeros(0, np.int64))
            parts.append(np.asarray(inv, dtype=np.int64))
        elif c.t == T_FLOAT:
            f = np.where(c.ok, c.v.astype(np.float64), 0.0)
            f = np.where(f == 0, 0.0, f)  # -0.0 == 0.0
            parts.append(f.view(np.int64))
        else:
            parts.append(np.where(c.ok, c.v.astype(np.int64), 0))
        parts.append(c.ok.astype(np.int64))
    if n == 0:
        return np.zeros(0, np.int64), anynull
    if not parts:
        return np.zeros(n, np.int64), anynull
    stacked = np.stack(parts, axis=1)
    _, inv = np.unique(stacked, axis=0, return_inverse=True)
    codes = np.asarray(inv, dtype=np.int64).reshape(-1)
    if not null_is_group:
        codes = np.where(anynull, -1, codes)
    return codes, anynull


class OracleTable:
    def __init__(self, order, cols, n):
        self._order = list(order)
        self._cols = dict(cols)
        self._n = int(n)
        if len(set(self._order)) != len(self._order):
            raise ValueError("duplicate column names")

    def _mk(self, order, cols, n):
        return OracleTable(order, cols, n)

    # ----------------------------------------------------------- CypherTable
    @property
    def physicalColumns(self):
        return list(self._order)

    @property
    def columnType(self):
        return {c: CAPF_TO_CT[self._cols[c].t] for c in self._order}

    def capf_type(self, c):
        return self._cols[c].t

    @property
    def size(self):
        return self._n

    def column_values(self, col):
        c = self._cols[col]
        out = []
        for v, ok in zip(c.v.tolist(), c.ok.tolist()):
            if not ok:
                out.append(None)
            elif c.t == T_BOOL:
                out.append(bool(v))
            elif c.t == T_INT:
                out.append(int(v))
            elif c.t == T_FLOAT:
                out.append(float(v))
            elif c.t == T_LIST:
                out.append(list(v))
            else:
                out.append(v)
        return out

    @property
    def rows(self):
        data = {c: self.column_values(c) for c in self._order}
        return [{c: data[c][i] for c in self._order} for i in range(self._n)]

    # ----------------------------------------------------------- Table[T]
    def cache(self):
        return self

    def select(self, *cols):
        pairs = [(c, c) if isinstance(c, str) else tuple(c) for c in cols]
        for c, _ in pairs:
            if c not in self._cols:
                raise KeyError(c)
        return self._mk([a for _, a in pairs], {a: self._cols[c] for c, a in pairs}, self._n)

    def filter(self, expr, header=None, params=None):
        v = evaluate(expr, self, header, params or {})
        keep = np.nonzero(v.ok & v.v.astype(bool))[0]
        return self._take(keep)

    def _take(self, idx):
        return self._mk(self._order, {c: k.take(idx) for c, k in self._cols.items()}, len(idx))

    def drop(self, *cols):
        left = [c for c in self._order if c not in cols]
        return self.select(*left)

    def join(self, other, join_type, *pairs):
        overlap = set(self._order) & set(other._order)
        assert not overlap, f"overlapping columns: {overlap}"
        nl, nr = self._n, other._n
        if join_type == "cross":
            li = np.repeat(np.arange(nl), nr)
            ri = np.tile(np.arange(nr), nl)
        else:
            lk = [self._cols[a] for a, _ in pairs]
            rk = [other._cols[b] for _, b in pairs]
            # joint codes over the concatenation so equal keys share a code
            both = [Col(a.t if a.t != T_NULL else b.t, np.concatenate([a.v, b.v]) if a.v.dtype == b.v.dtype
                        else np.concatenate([a.v.astype(object), b.v.astype(object)]),
                        np.concatenate([a.ok, b.ok])) for a, b in zip(lk, rk)]
            codes, _ = _key_codes(both, null_is_group=False)
            lc, rc = codes[:nl], codes[nl:]
            order = np.argsort(rc, kind="stable")
            rs = rc[order]
            lo = np.searchsorted(rs, lc, side="left")
            hi = np.searchsorted(rs, lc, side="right")
            cnt = np.where(lc < 0, 0, hi - lo)
            li = np.repeat(np.arange(nl), cnt)
            starts = np.repeat(lo, cnt)
            offs = np.arange(len(li)) - np.repeat(np.cumsum(cnt) - cnt, cnt)
            ri = order[starts + offs] if len(li) else np.zeros(0, np.int64)
            if join_type in ("left_outer", "full_outer"):
                miss = np.nonzero(cnt == 0)[0]
                li = np.concatenate([li, miss])
                ri = np.concatenate([ri, np.full(len(miss), -1)])
            if join_type in ("right_outer", "full_outer"):
                matched = np.zeros(nr, bool)
                matched[ri[ri >= 0]] = True
                miss = np.nonzero(~matched)[0]
                li = np.concatenate([li, np.full(len(miss), -1)])
                ri = np.concatenate([ri, miss])
        cols = {c: k.take(li) for c, k in self._cols.items()}
        cols.update({c: k.take(ri) for c, k in other._cols.items()})
        return self._mk(self._order + other._order, cols, len(li))

    def unionAll(self, other):
        if set(self._order) != set(other._order):
            raise ValueError("unionAll: column sets differ")
        cols = {}
        for c in self._order:
            a, b = self._cols[c], other._cols[c]
            t = a.t if a.t != T_NULL else b.t
            if a.t != b.t and T_NULL not in (a.t, b.t):
                raise ValueError(f"Equal column types for union all: {c}")
            va = a.v if a.t == t else _empty_vals(t, len(a.ok))
            vb = b.v if b.t == t else _empty_vals(t, len(b.ok))
            cols[c] = Col(t, np.concatenate([va, vb]), np.concatenate([a.ok, b.ok]))
        return self._mk(self._order, cols, self._n + other._n)

    def orderBy(self, *sort_items, header=None, params=None):
        idx = np.arange(self._n)
        for e, o in reversed(sort_items):
            v = evaluate(e, self, header, params or {})
            desc = o in ("desc", "Descending", True)
            vals = v.v[idx]
            ok = v.ok[idx]
            if v.t == T_STRING:  # the strings' ranks in String.compareTo order
                enc = [x.encode("utf-16-be", "surrogatepass") if p else b"" for x, p in zip(vals, ok)]
                rank = {k: i for i, k in enumerate(sorted(set(enc)))}
                vals = np.array([rank[k] for k in enc], dtype=np.int64)
            key = vals.astype(np.float64) if v.t == T_FLOAT else vals.astype(np.int64)
            if desc:
                key = -key if v.t == T_FLOAT else ~key
            o1 = np.argsort(key, kind="stable")
            idx = idx[o1]
            ok = ok[o1]
            nulls = ~ok
            o2 = np.argsort(~nulls if desc else nulls, kind="stable")
            idx = idx[o2]
        return self._take(idx)

    def skip(self, n):
        return self._take(np.arange(min(n, self._n), self._n))

    def limit(self, n):
        return self._take(np.arange(min(n, self._n)))

    def distinct(self, *cols):
        keys = [self._cols[c] for c in (cols or self._order)]
        if not keys:
            return self._take(np.arange(min(1, self._n)))
        codes, _ = _key_codes(keys)
        _, first = np.unique(codes, return_index=True)
        return self._take(np.sort(first))

    def group(self, by, aggregations, header=None, params=None):
        gcols = []
        for v in by:
            for e in header.owned_by(v):
                c = header.column(e)
                if c in self._cols and c not in gcols:
                    gcols.append(c)
        if gcols:
            codes, _ = _key_codes([self._cols[c] for c in gcols])
            uniq, first, inv = np.unique(codes, return_index=True, return_inverse=True)
            order = np.argsort(first)
            remap = np.empty_like(order)
            remap[order] = np.arange(len(order))
            gid = remap[np.asarray(inv).reshape(-1)]
            ng = len(uniq)
            reps = np.sort(first)
        else:
            gid = np.zeros(self._n, dtype=np.int64)
            ng = 1
            reps = np.zeros(1, dtype=np.int64)
        out_order = list(gcols)
        cols = {c: self._cols[c].take(reps) for c in gcols}
        for name, agg in aggregations.items():
            cols[name] = self._aggregate(agg, gid, ng, header, params or {})
            out_order.append(name)
        return self._mk(out_order, cols, ng)

    def _aggregate(self, agg, gid, ng, header, params):
        if not isinstance(agg, Aggregator):
            raise TypeError(agg)
        if agg.kind < 0:  # no case in FlinkSQLExprMapper.scala:281-290
            raise NotImplementedError(f"No support for converting Cypher expression {agg}")
        if agg.kind == AGG_COUNT_STAR:
            return Col(T_INT, np.bincount(gid, minlength=ng).astype(np.int64), np.ones(ng, bool))
        v = evaluate(agg.expr, self, header, params)
        sel = v.ok
        if v.t == T_LIST:
            raise NotImplementedError("aggregation of list values")
        if agg.kind == AGG_COLLECT:
            lists = [[] for _ in range(ng)]
            seen = [set() for _ in range(ng)]
            for g, x, ok in zip(gid.tolist(), v.v.tolist(), sel.tolist()):
                if not ok or v.t == T_NULL:
                    continue
                x = bool(x) if v.t == T_BOOL else x
                if agg.distinct:
                    if x in seen[g]:
                        continue
                    seen[g].add(x)
                lists[g].append(x)
            out = np.empty(ng, dtype=object)
            for g in range(ng):
                out[g] = sorted(lists[g])
            return Col(T_LIST, out, np.ones(ng, bool))
        if agg.kind == AGG_COUNT:
            if agg.distinct:  # Spark semantics (Flink ignores DISTINCT)
                seen = set()
                cnt = np.zeros(ng, np.int64)
                for g, x, ok in zip(gid.tolist(), v.v.tolist(), sel.tolist()):
                    if ok and (g, x) not in seen:
                        seen.add((g, x))
                        cnt[g] += 1
                return Col(T_INT, cnt, np.ones(ng, bool))
            return Col(T_INT, np.bincount(gid[sel], minlength=ng).astype(np.int64), np.ones(ng, bool))
        if agg.kind in (AGG_STDEV, AGG_STDEV_POP, AGG_PERCENTILE_CONT, AGG_PERCENTILE_DISC):
            if v.t not in (T_INT, T_FLOAT, T_NULL):
                raise NotImplementedError("stDev / percentile of non-numeric values")
            groups = [[] for _ in range(ng)]
            if v.t != T_NULL:
                for g, x, ok in zip(gid.tolist(), v.v.tolist(), sel.tolist()):
                    if ok:
                        groups[g].append(x)
            if agg.kind in (AGG_STDEV, AGG_STDEV_POP):
                res = [_exact_stdev([float(x) for x in xs], agg.kind == AGG_STDEV) for xs in groups]
                out_t = T_FLOAT
            else:
                p = percentile_value(agg.percentile, params)
                res = [_percentile(xs, p, agg.kind == AGG_PERCENTILE_CONT) for xs in groups]
                out_t = T_FLOAT if agg.kind == AGG_PERCENTILE_CONT or v.t != T_INT else T_INT
            arr = _empty_vals(out_t, ng)
            for g, r in enumerate(res):
                if r is not None:
                    arr[g] = r
            return Col(out_t, arr, np.array([r is not None for r in res], bool))
        if v.t == T_STRING and agg.kind in (AGG_MIN, AGG_MAX):  # String.compareTo order
            best = [None] * ng
            for g, x, ok in zip(gid.tolist(), v.v.tolist(), sel.tolist()):
                if ok and (best[g] is None or (_jcmp(x, best[g]) < 0) == (agg.kind == AGG_MIN)
                           and _jcmp(x, best[g]) != 0):
                    best[g] = x
            return Col(T_STRING, np.array(best, dtype=object), np.array([b is not None for b in best], bool))
        if v.t == T_STRING and agg.kind != AGG_COUNT:
            raise NotImplementedError("aggregate of strings")
        cnt = np.bincount(gid[sel], minlength=ng)
        t = v.t
        out_t = T_FLOAT if agg.kind == AGG_AVG and t == T_INT else t
        res = _empty_vals(out_t if out_t != T_NULL else T_INT, ng)
        # sequential fold in row order (Flink accumulates per group)
        acc = [None] * ng
        for g, x, ok in zip(gid.tolist(), v.v.tolist(), sel.tolist()):
            if not ok:
                continue
            a = acc[g]
            if agg.kind in (AGG_SUM, AGG_AVG):
                acc[g] = x if a is None else a + x
            elif agg.kind == AGG_MIN:
                acc[g] = x if a is None or x < a else a
            else:
                acc[g] = x if a is None or x > a else a
        for g in range(ng):
            a = acc[g]
            if a is None:
                continue
            if agg.kind == AGG_AVG:
                # a FLOAT also over INTEGER values (AggregationTests.scala:852, 876, 921):
                # the exact sum as a double over the count
                a = float(((int(a) + 2 ** 63) % 2 ** 64) - 2 ** 63 if t == T_INT else a) / float(cnt[g])
            elif t == T_INT:
                a = ((int(a) + 2 ** 63) % 2 ** 64) - 2 ** 63  # LONG wrap-around
            res[g] = a
        return Col(out_t if out_t != T_NULL else T_INT, res, cnt > 0)

    def _explode(self, e, name, header, params):
        """UNWIND: Explode(list) AS name (RelationalPlanner.scala:99-101),
        every row repeated per element (Spark explode: a NULL / empty list
        yields no row)."""
        ev = explode_values(e.expr, params)
        if ev is not None:
            t, vals = ev
            k = len(vals)
            idx = np.repeat(np.arange(self._n), k)
            el = np.tile(np.arange(k), self._n)
            ev_col = Col(t, np.array([v if v is not None else (0 if t != T_STRING else None) for v in vals],
                                     dtype=_NP[t]) if k else _empty_vals(t, 0),
                         np.array([v is not None for v in vals], bool))
        else:
            src = header.get(e.expr) if header is not None else None
            if src is None or src not in self._cols:
                if isinstance(e.expr, (Var, NullLit)):
                    return self._mk(self._order + [name], {**{c: k.take([]) for c, k in self._cols.items()},
                                                           name: Col(T_NULL, _empty_vals(T_NULL, 0), [])}, 0)
                raise NotImplementedError(f"oracle: UNWIND of {e.expr}")
            lc = self._cols[src]
            if lc.t == T_NULL:  # every row's list is NULL: no rows
                return self._mk(self._order + [name], {**{c: k.take([]) for c, k in self._cols.items()},
                                                       name: Col(T_NULL, _empty_vals(T_NULL, 0), [])}, 0)
            if lc.t != T_LIST:
                raise ValueError("UNWIND of a non-list column")
            rows, els = [], []
            for i, (lst, ok) in enumerate(zip(lc.v, lc.ok)):
                if ok and lst is not None:
                    rows += [i] * len(lst)
                    els += list(lst)
            idx = np.array(rows, dtype=np.int64)
            el = np.arange(len(els))
            et = T_NULL
            for x in els:
                et = T_FLOAT if isinstance(x, float) else T_BOOL if isinstance(x, bool) else \
                    T_STRING if isinstance(x, str) else T_INT
                break
            ev_col = Col(et, np.array(els, dtype=_NP[et]) if els else _empty_vals(et, 0), np.ones(len(els), bool))
        cols = {c: k.take(idx) for c, k in self._cols.items()}
        cols[name] = ev_col.take(el)
        return self._mk(self._order + [name], cols, len(idx))

    def withColumns(self, *columns, header=None, params=None):
        if any(isinstance(e, Explode) for e, _ in columns):
            t = self
            plain = [(e, c) for e, c in columns if not isinstance(e, Explode)]
            if plain:
                t = t.withColumns(*plain, header=header, params=params)
            for e, c in columns:
                if isinstance(e, Explode):
                    t = t._explode(e, c, header, params)
            return t
        order = list(self._order)
        cols = dict(self._cols)
        for e, name in columns:
            v = evaluate(e, self, header, params or {})
            vals = v.v
            if v.t == T_STRING:
                vals = np.asarray(vals, dtype=object)
            cols[name] = Col(v.t, vals, v.ok)
            if name not in order:
                order.append(name)
        return self._mk(order, cols, self._n)

    def show(self, rows=20):
        for r in self.rows[:rows]:
            print(r)
