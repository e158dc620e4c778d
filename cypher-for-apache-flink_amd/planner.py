"""Relational planning of MATCH patterns onto any Table[T] backend.

This is the caller side of the drop-in boundary: a restatement of the okapi
planning that produces the Table-operation sequences the backend executes —
  * LogicalPlanner.planComponentPattern / planExpansions
    (okapi-logical/.../impl/LogicalPlanner.scala:309-433): node scans, then one
    Expand / ExpandInto / BoundedVarLengthExpand per relationship in pattern
    order, WHERE conjuncts as one Filter each (:211-227);
  * RelationalPlanner Expand / ExpandInto
    (okapi-relational/.../impl/planning/RelationalPlanner.scala:130-189);
  * DirectedVarLengthExpandPlanner
    (okapi-relational/.../impl/planning/VarLengthExpandPlanner.scala:82-259);
  * relationship uniqueness NOT(r_i = r_j) added per MATCH clause by the
    front end (okapi-ir/.../impl/parse/CypherParser.scala:72);
  * projections / aggregation / DISTINCT / ORDER BY / SKIP / LIMIT on top
    (Table.withColumns / group / distinct / orderBy / skip / limit).

Queries are given as small pattern objects (the Cypher parser and IR builder
are out of scope: the front end stays unchanged in the real deployment).
"""
from dataclasses import dataclass, field
from itertools import combinations
from functools import lru_cache
from typing import List, Optional, Sequence, Tuple

from .expr import (Aggregator, Ands, BoolLit, ElementProperty, EndNode, Equals, ExistsPattern, Explode, Expr,
                   HasLabel, HasType, IntegerLit, IsNotNull, Not, NullLit, StartNode, TrueLit, Var,
                   aggregators_in, replace_exprs)
from .header import RecordHeader, owner_of


@dataclass
class Planned:
    """A relational operator's result: backend table + record header."""
    table: object
    header: RecordHeader


# ------------------------------------------------------------- query model
@dataclass
class NodeP:
    name: str
    labels: Tuple[str, ...] = ()


@dataclass
class RelP:
    name: str
    src: str
    dst: str
    types: Tuple[str, ...] = ()
    direction: str = "out"          # out | in | both
    length: Optional[Tuple[int, int]] = None  # (lower, upper) for *l..u


@dataclass
class Match:
    nodes: List[NodeP]
    rels: List[RelP] = field(default_factory=list)
    where: List[Expr] = field(default_factory=list)
    optional: bool = False  # OPTIONAL MATCH


@dataclass
class Stage:
    """A WITH / RETURN projection: items = [(alias, Expr | Aggregator)]."""
    items: List[Tuple[str, Expr]]
    distinct: bool = False
    where: List[Expr] = field(default_factory=list)
    order_by: List[Tuple[str, str]] = field(default_factory=list)  # (alias, asc|desc)
    skip: Optional[int] = None
    limit: Optional[int] = None


@dataclass
class Unwind:
    """UNWIND list AS alias (logical Unwind, RelationalPlanner.scala:99-101:
    `in.add(Explode(list) as item)`); a clause of Query.matches, in order."""
    list: Expr
    alias: str


@dataclass
class Query:
    matches: List[object]  # Match / Unwind clauses in query order
    stages: List[object]   # Stage (WITH / RETURN) and Unwind clauses after the first WITH
    # the driving table of `session.cypher(query, drivingTable = records)`
    # (RelationalCypherSession.scala:122-145): (name, capf type, values, valid)
    # columns, each bound to the variable of its name
    driving: Optional[List[tuple]] = None


@dataclass
class UnionQuery:
    """q1 UNION [ALL] q2 (logical TabularUnionAll, RelationalPlanner.scala:123-124;
    UNION adds a Distinct over the returned fields): both sides return the same
    aliases."""
    left: object   # Query | UnionQuery
    right: Query
    all: bool = False


# ------------------------------------------------------------- relational ops
@lru_cache(maxsize=16384)
def _mk(cls, *args):
    """One shared instance per expression the planner builds for a query's
    variables (Var, StartNode(r), …): its hash is computed once and header
    lookups hit on identity (the same plan is built query after query)."""
    return cls(*args)


def _rename_disjoint(left: Planned, right: Planned) -> Planned:
    """withDisjointColumnNames (RelationalPlanner.scala:366-368, 524-538)."""
    rcols = right.table.physicalColumns
    hcols = left.header.column_frozenset()
    tcols = left.table.physicalColumns
    if hcols.isdisjoint(rcols) and (len(tcols) <= len(hcols) and hcols.issuperset(tcols)
                                    or set(tcols).isdisjoint(rcols)):
        return right
    lcols = set(hcols)
    lcols.update(tcols)
    clash = [c for c in rcols if c in lcols]
    if not clash:
        return right
    ren = {}
    taken = lcols | set(right.table.physicalColumns)
    for c in clash:
        k = 1
        while f"{c}_{k}" in taken:
            k += 1
        ren[c] = f"{c}_{k}"
        taken.add(ren[c])
    tab = right.table.select(*[(c, ren.get(c, c)) for c in right.table.physicalColumns])
    return Planned(tab, right.header.renamed(lambda e, c: ren.get(c, c)))


def join(left: Planned, right: Planned, pairs: Sequence[Tuple[Expr, Expr]], join_type="inner") -> Planned:
    right = _rename_disjoint(left, right)
    cols = [(left.header.column(a), right.header.column(b)) for a, b in pairs]
    return Planned(left.table.join(right.table, join_type, *cols), left.header.union(right.header))


def filter_(op: Planned, expr: Expr, params=None) -> Planned:
    if expr == TrueLit or (isinstance(expr, Ands) and not expr.exprs):
        return op
    return Planned(op.table.filter(expr, op.header, params or {}), op.header)


def union_all(a: Planned, b: Planned) -> Planned:
    """TabularUnionAll: align the right side's columns to the left header."""
    exprs = a.header.expressions
    missing = [e for e in exprs if e not in b.header] + [e for e in b.header.expressions if e not in a.header]
    if missing:
        raise ValueError(f"union of differing headers: {missing}")
    tb = b.table.select(*[(b.header.column(e), a.header.column(e)) for e in exprs])
    ta = a.table.select(*[a.header.column(e) for e in exprs])
    return Planned(ta.unionAll(tb), RecordHeader({e: a.header.column(e) for e in exprs}))


def union_queries(a: Planned, b: Planned) -> Planned:
    """unionAll of two query results (RelationalPlanner.scala:374-391): the
    combined header; each side's elements aligned to it — a label / type the
    side lacks is FALSE, a property it lacks NULL of the other side's type
    (alignExpressions :447-500) — every column renamed to one name per
    expression (alignColumnNames), then TabularUnionAll (RelationalOperator
    .scala:451-482; unequal column types raise there)."""
    from .expr import BoolLit, HasLabel, HasType, NullLit
    target = list(dict.fromkeys(a.header.expressions + b.header.expressions))
    names = {e: f"__u{i}" for i, e in enumerate(target)}

    def align(p: Planned, other: Planned) -> Planned:
        missing = [e for e in target if e not in p.header]
        for e in missing:
            if isinstance(e, Var):
                from ._lib import IllegalArgumentException
                raise IllegalArgumentException(f"UNION: both sides must return the same columns ({e.vname})")
        adds = [(BoolLit(False) if isinstance(e, (HasLabel, HasType)) else NullLit(getattr(e, "ctype", "ANY")),
                 names[e]) for e in missing]
        tab = p.table.select(*[(p.header.column(e), names[e]) for e in target if e in p.header])
        if adds:
            tab = tab.withColumns(*adds, header=RecordHeader({}), params={})
        return Planned(tab.select(*[names[e] for e in target]), RecordHeader(names))

    la, lb = align(a, b), align(b, a)
    return Planned(la.table.unionAll(lb.table), la.header)


def add_into(op: Planned, items: Sequence[Tuple[Expr, Expr]], params=None) -> Planned:
    """AddInto(expr -> target expr) as withColumns (RelationalOperator.scala:219-264)."""
    h = op.header
    cols = []
    for src, tgt in items:
        col = h.get(tgt) or _col_name(tgt)
        cols.append((src, col))
        h = h.with_expr(tgt, col)
    return Planned(op.table.withColumns(*cols, header=op.header, params=params or {}), h)


def _col_name(e):
    return str(e)


def alias_var(op: Planned, old: Var, new: Var) -> Planned:
    """Alias a relationship var's columns to a new var (edgeScan as e_i)."""
    cols, m = [], {}
    for e in op.header.owned_by(old):
        c = op.header.column(e)
        ne = _rewrite_owner(e, old, new)
        nc = str(ne)
        cols.append((c, nc))
        m[ne] = nc
    return Planned(op.table.select(*cols), RecordHeader(m))


def _rewrite_owner(e, old, new):
    if e == old:
        return new
    if isinstance(e, ElementProperty):
        return ElementProperty(new, e.key, e.ctype)
    if isinstance(e, HasLabel):
        return HasLabel(new, e.label)
    if isinstance(e, HasType):
        return HasType(new, e.rel_type)
    if isinstance(e, StartNode):
        return StartNode(new)
    if isinstance(e, EndNode):
        return EndNode(new)
    raise ValueError(e)


# ------------------------------------------------------------- expand
def expand(graph, source: Var, rel: RelP, target: Var, src_op: Planned, tgt_op: Planned,
           direction: str) -> Planned:
    """RelationalPlanner Expand (RelationalPlanner.scala:130-165)."""
    r = _mk(Var, rel.name, "RELATIONSHIP")
    second = graph.rel_scan(rel.name, rel.types)
    start, end = _mk(StartNode, r), _mk(EndNode, r)
    if direction == "out":
        tmp = join(src_op, second, [(source, start)])
        return join(tmp, tgt_op, [(end, target)])
    if direction == "in":
        tmp = join(tgt_op, second, [(target, end)])
        return join(tmp, src_op, [(start, source)])
    # undirected: outgoing ∪ incoming-without-loops
    tmp_out = join(src_op, second, [(source, start)])
    outgoing = join(tmp_out, tgt_op, [(end, target)])
    no_loops = filter_(second, Not(Equals(start, end)))
    tmp_in = join(src_op, no_loops, [(source, end)])
    incoming = join(tmp_in, tgt_op, [(start, target)])
    return union_all(outgoing, incoming)


def expand_into(graph, source: Var, rel: RelP, target: Var, in_op: Planned, direction: str) -> Planned:
    """RelationalPlanner ExpandInto (RelationalPlanner.scala:167-189)."""
    r = Var(rel.name, "RELATIONSHIP")
    rels = graph.rel_scan(rel.name, rel.types)
    start, end = StartNode(r), EndNode(r)
    if direction in ("out", "in"):
        if direction == "in":
            source, target = target, source
        return join(in_op, rels, [(source, start), (target, end)])
    outgoing = join(in_op, rels, [(source, start), (target, end)])
    incoming = join(in_op, graph.rel_scan(rel.name, rel.types), [(target, start), (source, end)])
    return union_all(outgoing, incoming)


def var_length_expand(graph, source: Var, rel: RelP, target: Var, src_op: Planned, tgt_op: Planned,
                      is_expand_into: bool) -> Planned:
    """Directed/UndirectedVarLengthExpandPlanner.plan
    (VarLengthExpandPlanner.scala:246-259, 277-307), join for join."""
    lower, upper = rel.length
    edge = Var(rel.name, "RELATIONSHIP")
    edge_scan = graph.rel_scan(rel.name, rel.types)

    def seg(i):
        return Var(f"{rel.name}_{i}", "RELATIONSHIP")

    existing_rels = [e for e in src_op.header.vars() if e.ctype == "RELATIONSHIP"]

    def iso(new, cands):
        # isomorphismFilter (:178-179); Ands() of nothing is TrueLit → no Filter
        return Ands(*[Not(Equals(e, new)) for e in cands]) if cands else TrueLit

    def init(direction):  # (:82-97)
        e1 = seg(1)
        step = alias_var(edge_scan, edge, e1)
        key = StartNode(e1) if direction == "out" else EndNode(e1)
        return filter_(join(src_op, step, [(source, key)]), iso(e1, existing_rels))

    def expand_step(i, table, dirs, edges):  # (:107-135)
        ei = seg(i)
        step = alias_var(edge_scan, edge, ei)
        last = edges[-1]
        left, right = {
            ("out", "out"): (EndNode(last), StartNode(ei)),
            ("out", "in"): (EndNode(last), EndNode(ei)),
            ("in", "out"): (StartNode(last), EndNode(ei)),
            ("in", "in"): (StartNode(last), StartNode(ei)),
        }[dirs]
        return filter_(join(table, step, [(left, right)]), iso(ei, edges)), ei

    def add_target(p, last, direction):  # addTargetOps (:218-229)
        key = EndNode(last) if direction == "out" else StartNode(last)
        if is_expand_into:
            return filter_(p, Equals(target, key))
        return join(p, tgt_op, [(key, target)])

    with_targets = []
    if rel.direction != "both":
        acc = [(init("out"), [seg(1)])]
        for i in range(2, upper + 1):
            last, edges = acc[-1]
            nxt, ei = expand_step(i, last, ("out", "out"), edges)
            acc.append((nxt, edges + [ei]))
        acc = [(p, es) for p, es in acc if len(es) >= lower] if upper >= 1 else []
        with_targets = [add_target(p, es[-1], "out") for p, es in acc]
    else:
        acc = [((init("out"), init("in")), [seg(1)])]
        for i in range(2, upper + 1):
            (last, last_rev), edges = acc[-1]
            out_out, ei = expand_step(i, last, ("out", "out"), edges)
            out_in, _ = expand_step(i, last, ("out", "in"), edges)
            in_out, _ = expand_step(i, last_rev, ("in", "out"), edges)
            in_in, _ = expand_step(i, last_rev, ("in", "in"), edges)
            acc.append(((union_all(out_out, in_out), union_all(out_in, in_in)), edges + [ei]))
        acc = [(p, es) for p, es in acc if len(es) >= lower] if upper >= 1 else []
        with_targets = [union_all(add_target(o, es[-1], "out"), add_target(n, es[-1], "in"))
                        for (o, n), es in acc]
    if lower == 0:
        with_targets.append(_copy_element(src_op, source, target, tgt_op))
    if not with_targets:
        raise ValueError("empty var-length range")
    return _finalize(with_targets)


def _copy_element(src_op, source, target, tgt_op):
    """copyElement: zero-length paths (VarLengthExpandPlanner.scala:180-205)."""
    items = []
    for e in tgt_op.header.owned_by(target):
        if e == target:
            items.append((source, target))
        elif isinstance(e, HasLabel):
            s = HasLabel(source, e.label)
            items.append((s if s in src_op.header else BoolLit(False), e))
        elif isinstance(e, ElementProperty):
            s = ElementProperty(source, e.key, e.ctype)
            items.append((s if s in src_op.header else NullLit(e.ctype), e))
    return add_into(src_op, items)


def _finalize(paths: List[Planned]) -> Planned:
    """Null-pad shorter paths to the widest header and UNION ALL (:145-170)."""
    widest = max(paths, key=lambda p: len(p.header.columns)).header
    aligned = []
    for p in paths:
        missing = [e for e in widest.expressions if e not in p.header]
        if missing:
            p = add_into(p, [(NullLit(_ctype(e)), e) for e in missing])
        aligned.append(p)
    out = aligned[0]
    for p in aligned[1:]:
        out = union_all(out, p)
    return out


def _ctype(e):
    if isinstance(e, (HasLabel, HasType)):
        return "BOOLEAN"
    if isinstance(e, ElementProperty):
        return e.ctype
    return "INTEGER"


# ------------------------------------------------------------- pattern planning
def plan_match(graph, m: Match, prev: Optional[Planned], params=None) -> Planned:
    """planComponentPattern + planExpansions + planFilter for one MATCH clause."""
    rels = []
    for r in m.rels:  # normalise <-[r]- to -[r]->
        if r.direction == "in":
            r = RelP(r.name, r.dst, r.src, r.types, "out", r.length)
        rels.append(r)
    labels = {}
    for n in m.nodes:
        labels.setdefault(n.name, set()).update(n.labels)
    node_names = [n.name for n in m.nodes]
    for r in rels:
        for v in (r.src, r.dst):
            if v not in labels:
                labels[v] = set()
                node_names.append(v)
    node_names = list(dict.fromkeys(node_names))
    bound = set(v.vname for v in prev.header.vars()) if prev is not None else set()
    plans = []  # (set of vars, Planned)
    solved = [v for v in node_names if v in bound]
    # label constraints on already-bound nodes are row predicates on their
    # label columns (their scans already happened)
    extra_where = [HasLabel(Var(v, "NODE"), l) for v in solved for l in sorted(labels[v])]
    if prev is not None and solved:
        plans.append((set(bound), prev))
        remaining = [v for v in node_names if v not in bound]
    else:
        first = node_names[0]
        scan = graph.node_scan(first, sorted(labels[first]))
        if prev is not None:
            scan = Planned(prev.table.join(scan.table, "cross"), prev.header.union(scan.header))
            plans.append((set(bound) | {first}, scan))
        else:
            plans.append(({first}, scan))
        remaining = node_names[1:]
    for v in remaining:
        plans.append(({v}, graph.node_scan(v, sorted(labels[v]))))

    for r in rels:
        si = next(i for i, (vs, _) in enumerate(plans) if r.src in vs)
        ti = next(i for i, (vs, _) in enumerate(plans) if r.dst in vs)
        s, t = _mk(Var, r.src, "NODE"), _mk(Var, r.dst, "NODE")
        if r.length is not None:
            if si == ti:
                op = var_length_expand(graph, s, r, t, plans[si][1], plans[si][1], True)
                plans[si] = (plans[si][0] | {r.name}, op)
            else:
                op = var_length_expand(graph, s, r, t, plans[si][1], plans[ti][1], False)
                vs = plans[si][0] | plans[ti][0] | {r.name}
                plans = [p for i, p in enumerate(plans) if i not in (si, ti)] + [(vs, op)]
        elif si == ti:
            # a cyclic relationship (a)-[r]-(a) is planned as a directed
            # ExpandInto (LogicalPlanner.scala:407-418, CyclicRelationship)
            d = "both" if r.direction == "both" and r.src != r.dst else "out"
            op = expand_into(graph, s, r, t, plans[si][1], d)
            plans[si] = (plans[si][0] | {r.name}, op)
        else:
            op = expand(graph, s, r, t, plans[si][1], plans[ti][1], r.direction)
            vs = plans[si][0] | plans[ti][0] | {r.name}
            plans = [p for i, p in enumerate(plans) if i not in (si, ti)] + [(vs, op)]
    # disconnected components: cartesian products
    op = plans[0][1]
    for _, p in plans[1:]:
        p = _rename_disjoint(op, p)
        op = Planned(op.table.join(p.table, "cross"), op.header.union(p.header))
    # WHERE conjuncts, then front-end uniqueness predicates, one Filter each
    fixed = [_mk(Var, r.name, "RELATIONSHIP") for r in rels if r.length is None]
    preds = list(m.where) + extra_where + [_mk(Not, _mk(Equals, a, b)) for a, b in combinations(fixed, 2)]
    for p in preds:
        op = plan_subqueries(graph, op, p, params)
        op = filter_(op, p, params)
    return op


def _exists_in(e):
    """ExistsPattern sub-expressions of e, innermost first (planInnerSubquery,
    LogicalPlanner.scala:230-243)."""
    out = []

    def go(x):
        if isinstance(x, ExistsPattern):
            out.append(x)
            return
        for name in ("lhs", "rhs", "expr"):
            c = getattr(x, name, None)
            if isinstance(c, Expr):
                go(c)
        for c in getattr(x, "exprs", ()) or ():
            if isinstance(c, Expr):
                go(c)
    go(e)
    return out


_LEAVES = (Var, StartNode, EndNode, HasLabel, HasType, ElementProperty, IntegerLit, BoolLit, NullLit)


def _may_hold_exists(e):
    """False when `e` provably holds no EXISTS pattern (the common predicates:
    column references, literals and NOT / = over them)."""
    t = type(e)
    if t in _LEAVES:
        return False
    if t is Not:
        return _may_hold_exists(e.expr)
    if t is Equals:
        return _may_hold_exists(e.lhs) or _may_hold_exists(e.rhs)
    return True


def plan_subqueries(graph, op: Planned, expr: Expr, params=None) -> Planned:
    """Plans every EXISTS pattern inside `expr` that the header does not hold yet."""
    if not _may_hold_exists(expr):
        return op
    for ex in _exists_in(expr):
        if ex not in op.header:
            op = plan_exists(graph, ex, op, params)
    return op


def plan_exists(graph, ex: ExistsPattern, lhs: Planned, params=None) -> Planned:
    """ExistsSubQuery (RelationalPlanner.scala:224-247): the pattern is planned
    on its own (rhs, with its own scans of the shared variables), then
      1. the variables common to both headers are the join expressions,
      2. the rhs join-var columns are aliased to fresh names, every other rhs
         expression is dropped,
      3. DISTINCT rows of the aliases,
      4. lhs LEFT OUTER JOIN rhs on (lhs var = alias),
      5. IsNotNull(first alias) is added as the predicate's target column.
    (The reference's rhs keeps its other columns through the Distinct and the
    join; only IsNotNull(alias) is read from them, so they are not carried.)"""
    rhs = plan_match(graph, ex.pattern, None, params)
    lvars = {v.vname: v for v in lhs.header.vars()}
    join_vars = [v for v in rhs.header.vars() if v.vname in lvars]
    if not join_vars:
        from ._lib import NotImplementedException
        raise NotImplementedException("EXISTS pattern sharing no variable with the enclosing clause")
    taken = set(lhs.table.physicalColumns) | set(rhs.table.physicalColumns)
    fresh = []
    for i in range(len(join_vars) + 1):
        c = f"__exists_{len(lhs.header.expressions)}_{i}"
        while c in taken:
            c += "_"
        taken.add(c)
        fresh.append(c)
    target, aliases = fresh[0], fresh[1:]
    rtab = rhs.table.select(*[(rhs.header.column(v), a) for v, a in zip(join_vars, aliases)]).distinct()
    pairs = [(lhs.header.column(lvars[v.vname]), a) for v, a in zip(join_vars, aliases)]
    joined = lhs.table.join(rtab, "left_outer", *pairs)
    joined = joined.withColumns((IsNotNull(Var(aliases[0])), target),
                                header=RecordHeader({Var(aliases[0]): aliases[0]}), params=params or {})
    joined = joined.drop(*aliases)
    return Planned(joined, lhs.header.with_expr(ex, target))


def plan_optional(graph, m: Match, lhs: Planned, params=None) -> Planned:
    """planOptional (RelationalPlanner.scala:298-329): the optional pattern is
    planned on its own (rhs), then
      1. common expressions of both headers; the Vars among them join,
      2. the rhs drops the join vars' other expressions (labels, properties)
         and every other common expression,
      3. the rhs join-var columns get temporary names,
      4. lhs LEFT OUTER JOIN rhs on (lhs var column = temporary column),
      5. the temporary columns are dropped (Select of the header's columns).
    Rows of lhs without a match keep NULLs in every rhs column; a leading
    OPTIONAL MATCH joins the unit table.  Uniqueness
    predicates apply within the optional pattern only (MTa/OptionalMatchTests
    .scala:191-240: e2 may equal e1)."""
    rhs = plan_match(graph, m, None, params)
    if lhs is None:
        # a leading OPTIONAL MATCH: Optional(Start, rhs) — the unit table (one
        # row, no columns) left-outer-joined with no join columns: the rhs
        # rows, or one all-NULL row when the pattern has no match
        # (the empty key list is expressed as one constant key on both sides).
        # The rhs is the PROBE side and the one-row unit the build side
        # (unit RIGHT OUTER rhs ≡ rhs LEFT OUTER unit, mirrored): every rhs row
        # finds the single build row in parallel, and the unmatched unit row
        # still yields the all-NULL row when the pattern has no match.
        taken = set(rhs.table.physicalColumns)
        kl, kr = "__optional_unit", "__optional_unit_r"
        while kl in taken or kr in taken:
            kl, kr = kl + "_", kr + "_"
        unit = graph.session.unit().withColumns((IntegerLit(1), kl), header=RecordHeader({}))
        rtab = rhs.table.withColumns((IntegerLit(1), kr), header=rhs.header, params=params)
        joined = rtab.join(unit, "right_outer", (kr, kl)).drop(kl, kr)
        return Planned(joined, rhs.header)
    common = [e for e in lhs.header.expressions if e in rhs.header]
    join_vars = [e for e in common if isinstance(e, Var)]
    if not join_vars:
        # no shared variable: a left outer join with an EMPTY join list
        # (RelationalPlanner.scala:325 with joinExprs = ∅): every lhs row times
        # every rhs row, or the lhs row with NULLs when the rhs is empty —
        # expressed as one constant key on both sides
        right = _rename_disjoint(lhs, rhs)
        taken = set(lhs.table.physicalColumns) | set(right.table.physicalColumns)
        kl, kr = "__optional_const", "__optional_const_r"
        while kl in taken or kr in taken:
            kl, kr = kl + "_", kr + "_"
        ltab = lhs.table.withColumns((IntegerLit(1), kl), header=lhs.header, params=params)
        rtab = right.table.withColumns((IntegerLit(1), kr), header=right.header, params=params)
        joined = ltab.join(rtab, "left_outer", (kl, kr)).drop(kl, kr)
        return Planned(joined, lhs.header.union(right.header))
    remove = {e for v in join_vars for e in rhs.header.owned_by(v) if e != v} | \
        {e for e in common if not isinstance(e, Var)}
    keep = [e for e in rhs.header.expressions if e not in remove]
    jcol = {rhs.header.column(v): v for v in join_vars}
    taken = set(lhs.table.physicalColumns) | set(rhs.table.physicalColumns)
    tmp = {}
    for i, c in enumerate(jcol):
        t = f"__optional_{i}"
        while t in taken:
            t += "_"
        taken.add(t)
        tmp[c] = t
    rcols = list(dict.fromkeys(rhs.header.column(e) for e in keep))
    rtab = rhs.table.select(*[(c, tmp.get(c, c)) for c in rcols])
    rhead = RecordHeader({e: tmp.get(c, c) for e, c in ((e, rhs.header.column(e)) for e in keep)
                          if not (isinstance(e, Var) and e in jcol.values())})
    right = _rename_disjoint(lhs, Planned(rtab, rhead))
    # the temporary names are fresh, so _rename_disjoint left them alone
    pairs = [(lhs.header.column(v), tmp[c]) for c, v in jcol.items()]
    joined = lhs.table.join(right.table, "left_outer", *pairs)
    joined = joined.drop(*[tmp[c] for c in jcol])
    # rhs expressions that lived in a join-var column now read the lhs column
    inv = {t: c for c, t in tmp.items()}
    head = lhs.header.union(RecordHeader({e: (lhs.header.column(jcol[inv[c]]) if c in inv else c)
                                          for e, c in right.header.items()}))
    return Planned(joined, head)


def plan_unwind(op: Planned, u: Unwind, params=None) -> Planned:
    """Unwind → `add(Explode(list) as item)` (RelationalPlanner.scala:99-101):
    withColumns with the Explode item; the alias var reads the new column."""
    v = Var(u.alias)
    col = op.header.get(v) or "__" + u.alias
    tab = op.table.withColumns((Explode(u.list), col), header=op.header, params=params or {})
    return Planned(tab, op.header.with_expr(v, col))


def _split_aggregates(st: Stage) -> Stage:
    """Items that compute over aggregates (RETURN round(stDev(x) * 1000) /
    1000.0): each aggregator becomes its own item, aggregated first, and the
    item is projected over the aggregate columns by a following stage (the
    okapi IR plans the Aggregate below a Project of the outer expression)."""
    inner = [it for it in st.items if not aggregators_in(it[1]) or isinstance(it[1], Aggregator)]
    nested = [it for it in st.items if it not in inner]
    if not nested:
        return None
    hidden, mapping = [], {}
    for _, e in nested:
        for a in aggregators_in(e):
            if a not in mapping:
                name = f"__agg{len(mapping)}"
                mapping[a] = Var(name)
                hidden.append((name, a))
    first = Stage([(a, e) for a, e in st.items if (a, e) in inner] + hidden)
    outer = [(a, Var(a)) if (a, e) in inner else (a, replace_exprs(e, mapping)) for a, e in st.items]
    second = Stage(outer, distinct=st.distinct, where=st.where, order_by=st.order_by, skip=st.skip,
                   limit=st.limit)
    return first, second


def _map_entries(e, h):
    """(presence expression, [(key, expression)]) of a MAP-valued projection
    item — a map literal (MapExpression) or properties(x) — else None.
    properties(n) of an element lists every property key of its header (NULL
    values included, ExpressionTests.scala:1289-1333); of NULL it is NULL."""
    from .expr import BoolLit, IsNotNull, MapExpression, NullLit
    from ._lib import NotImplementedException
    if isinstance(e, MapExpression):
        for k, x in e.items:
            if isinstance(x, MapExpression) or type(x).__name__ == "Properties":
                raise NotImplementedException(f"nested maps: {e}")
        return BoolLit(True), list(e.items)
    if type(e).__name__ != "Properties":
        return None
    x = e.expr
    if isinstance(x, NullLit):
        return NullLit("BOOLEAN"), []
    if isinstance(x, Var) and x in h:
        props = sorted(((p.key, p) for p in h.owned_by(x) if isinstance(p, ElementProperty)), key=lambda kp: kp[0])
        return IsNotNull(x), props
    raise NotImplementedException(f"properties of {x}")


def plan_stage(op: Planned, st: Stage, params=None, graph=None) -> Planned:
    split = _split_aggregates(st)
    if split is not None:
        return plan_stage(plan_stage(op, split[0], params, graph), split[1], params, graph)
    aggs = [(a, e) for a, e in st.items if isinstance(e, Aggregator)]
    projs = [(a, e) for a, e in st.items if not isinstance(e, Aggregator)]
    for _, e in projs:
        op = plan_subqueries(graph, op, e, params)
    # project non-aggregate items into alias vars (RelationalPlanner Add → withColumns)
    h = op.header
    adds, new_h = [], {}
    for alias, e in projs:
        me = _map_entries(e, h)
        if me is not None:  # a MAP value: a presence flag plus one column per entry
            present, entries = me
            v = Var(alias, "MAP")
            adds.append((present, "__" + alias))
            new_h[v] = "__" + alias
            for k, x in entries:
                c = f"__{alias}.{k}"
                adds.append((x, c))
                new_h[ElementProperty(v, k)] = c
            continue
        owned = [x for x in h.owned_by(e) if x != e] if isinstance(e, Var) and e in h else []
        # startNode(r) / endNode(r) are CTNode (okapi Expr.scala): a node holding
        # only the rel's start / end id column (FlinkSQLExprMapper.scala:179-180)
        v = Var(alias, e.ctype if isinstance(e, Var) else
                "NODE" if type(e).__name__ in ("StartNodeFunction", "EndNodeFunction") else "ANY")
        col = "__" + alias
        adds.append((e, col))
        new_h[v] = col
        # a node / relationship var keeps its labels, type, endpoints and
        # properties under the alias (RETURN n returns the whole element)
        for x in owned:
            nx = _rewrite_owner(x, e, v)
            c = "__" + alias + "." + h.column(x)
            adds.append((x, c))
            new_h[nx] = c
    # aggregation arguments are evaluated against the incoming header
    if adds:
        tab = op.table.withColumns(*adds, header=h, params=params or {})
        h2 = h
        for v, c in new_h.items():
            h2 = h2.with_expr(v, c)
        op = Planned(tab, h2)
    if aggs:
        group_vars = [_mk(Var, a) for a, _ in projs]
        agg_cols = {"__" + a: e for a, e in aggs}
        tab = op.table.group(group_vars, agg_cols, header=op.header, params=params or {})
        hh = dict(new_h)
        hh.update({_mk(Var, a): "__" + a for a, _ in aggs})
        op = Planned(tab, RecordHeader(hh))
    else:
        cols = list(dict.fromkeys(new_h.values()))
        op = Planned(op.table.select(*cols), RecordHeader(new_h))
    if st.distinct:
        op = Planned(op.table.distinct(), op.header)
    for p in st.where:
        op = plan_subqueries(graph, op, p, params)
        op = filter_(op, p, params)
    if st.order_by:
        items = [(Var(a), o) for a, o in st.order_by]
        op = Planned(op.table.orderBy(*items, header=op.header, params=params or {}), op.header)
    if st.skip is not None:
        op = Planned(op.table.skip(_row_count(st.skip, params, "SKIP")), op.header)
    if st.limit is not None:
        op = Planned(op.table.limit(_row_count(st.limit, params, "LIMIT")), op.header)
    return op


def _row_count(e, params, what):
    """Skip / Limit argument: an integer literal or a parameter holding an
    integer (RelationalOperator.scala:362-398); anything else is illegal."""
    from .expr import IntegerLit, Param
    from ._lib import IllegalArgumentException
    if isinstance(e, bool):
        raise IllegalArgumentException(f"{what}: an integer literal or parameter, got {e!r}")
    if isinstance(e, int):
        return e
    if isinstance(e, IntegerLit):
        return e.v
    if isinstance(e, Param):
        v = (params or {}).get(e.pname)
        if isinstance(v, int) and not isinstance(v, bool):
            return v
        raise IllegalArgumentException(f"{what}: parameter ${e.pname} must be a CypherInteger, got {v!r}")
    raise IllegalArgumentException(f"{what}: an integer literal or parameter, got {e}")


def plan_query(graph, q: Query, params=None) -> Planned:
    """The okapi relational plan of `q`, operator for operator.  Physical
    choices (fused counts, the fused var-length reach of config 5) are made by
    the backend below the Table SPI from the plan DAG these calls build."""
    if isinstance(q, UnionQuery):
        op = union_queries(plan_query(graph, q.left, params), plan_query(graph, q.right, params))
        return op if q.all else Planned(op.table.distinct(), op.header)
    op = None
    if q.driving is not None:  # Start over the driving table's records (RelationalPlanner.scala:90)
        op = Planned(graph.session.table(list(q.driving)), RecordHeader({Var(c[0]): c[0] for c in q.driving}))
    if not q.matches and op is None:  # a leading RETURN / WITH: one row of the unit table (Start)
        op = Planned(graph.session.unit(), RecordHeader({}))
    for m in q.matches:
        if isinstance(m, Unwind):
            if op is None:  # a leading UNWIND: over the unit table (Start)
                op = Planned(graph.session.unit(), RecordHeader({}))
            op = plan_unwind(op, m, params)
            continue
        op = plan_optional(graph, m, op, params) if m.optional else plan_match(graph, m, op, params)
    for st in q.stages:  # WITH ... UNWIND list AS x ... RETURN (UnwindTests.scala:82-145)
        op = plan_unwind(op, st, params) if isinstance(st, Unwind) else plan_stage(op, st, params, graph)
    return op


@dataclass(frozen=True)
class CypherNode:
    """A returned node (CAPFNode: id, labels, non-null properties)."""
    id: int
    labels: frozenset
    properties: tuple  # sorted (key, value) pairs

    def props(self):
        return dict(self.properties)


@dataclass(frozen=True)
class CypherRelationship:
    """A returned relationship (CAPFRelationship: id, source, target, type,
    non-null properties)."""
    id: int
    source: int
    target: int
    rel_type: str
    properties: tuple

    def props(self):
        return dict(self.properties)


def _element_values(op: Planned, v: Var, data):
    """rowToCypherMap.collectNode / collectRel (flink-cypher/.../impl/convert/
    rowToCypherMap.scala:77-123) over downloaded columns: a NULL id is a NULL
    element; labels are the true label flags, properties the non-null ones.
    The relationship's target is read from the END node column (the Flink
    code reads startNodeFor twice, :98-99 — a reference bug, not reproduced)."""
    h = op.header
    ids = data(h.column(v))
    owned = h.owned_by(v)
    labels = [(x.label, data(h.column(x))) for x in owned if isinstance(x, HasLabel)]
    types = [(x.rel_type, data(h.column(x))) for x in owned if isinstance(x, HasType)]
    props = [(x.key, data(h.column(x))) for x in owned if isinstance(x, ElementProperty)]
    is_rel = v.ctype == "RELATIONSHIP" or StartNode(v) in h
    src = data(h.column(StartNode(v))) if is_rel else None
    dst = data(h.column(EndNode(v))) if is_rel else None
    out = []
    for i, ident in enumerate(ids):
        if ident is None:
            out.append(None)
            continue
        pr = tuple(sorted((k, vals[i]) for k, vals in props if vals[i] is not None))
        if is_rel:
            ty = [t for t, flags in types if flags[i]]
            out.append(CypherRelationship(ident, src[i], dst[i], ty[0] if ty else None, pr))
        else:
            out.append(CypherNode(ident, frozenset(l for l, flags in labels if flags[i]), pr))
    return out


def records(op: Planned, aliases: Sequence[str]):
    """RelationalCypherResult.records.toMaps: list of {alias: value}; node and
    relationship variables come back as CypherNode / CypherRelationship."""
    cache = {}

    def data(c):
        if c not in cache:
            cache[c] = op.table.column_values(c)
        return cache[c]

    out_cols = {}
    for a in aliases:
        v = next((e for e in op.header.vars() if e.vname == a), Var(a))
        if v.ctype == "MAP":  # a struct of columns: presence flag + one column per entry
            present = data(op.header.column(v))
            ents = [(x.key, data(op.header.column(x))) for x in op.header.owned_by(v)
                    if isinstance(x, ElementProperty)]
            out_cols[a] = [None if p is None else {k: vals[i] for k, vals in ents}
                           for i, p in enumerate(present)]
        elif v.ctype in ("NODE", "RELATIONSHIP") and len(op.header.owned_by(v)) >= 1:
            out_cols[a] = _element_values(op, v, data)
        else:
            out_cols[a] = data(op.header.column(v))
    if not out_cols:
        return [{} for _ in range(op.table.size)]
    cols = [out_cols[a] for a in aliases]
    # one dict display per row (dict(zip(...)) per row costs ~3x as much on
    # large results, e.g. config 5's histogram)
    if len(aliases) == 1:
        (k0,), (c0,) = aliases, cols
        return [{k0: x} for x in c0]
    if len(aliases) == 2:
        k0, k1 = aliases
        return [{k0: x, k1: y} for x, y in zip(*cols)]
    if len(aliases) == 3:
        k0, k1, k2 = aliases
        return [{k0: x, k1: y, k2: z} for x, y, z in zip(*cols)]
    return [dict(zip(aliases, row)) for row in zip(*cols)]


def _aliases(q):
    return _aliases(q.left) if isinstance(q, UnionQuery) else [a for a, _ in q.stages[-1].items]


def run(graph, q: Query, params=None):
    op = plan_query(graph, q, params)
    return records(op, _aliases(q))
