"""Element tables and the scan graph over any Table[T] backend.

Mirrors the okapi-relational graph layer that sits directly above the Table SPI:
 * element tables — one node table per label combination, one relationship
   table per type, all ids int64 (CAPFElementTable.create,
   flink-cypher/.../api/io/CAPFTable.scala:76-83; CAPFScanGraphFactory,
   flink-cypher-testing/.../support/creation/graphs/CAPFScanGraphFactory.scala:24-158);
 * ScanGraph.scanOperator — pick the element tables whose label set ⊇ the
   requested labels (okapi-api/.../api/graph/Pattern.scala:95-111), align them
   to the var's header with constant label columns and NULL property columns
   (RelationalPlanner.scala:447-515) and UNION ALL them
   (okapi-relational/.../impl/graph/ScanGraph.scala:59-105).

A label constraint in a pattern is therefore a table-selection decision, not
a row predicate.

The backend `session` only needs `table(columns)` and `empty(names, types)`;
tables need the Table[T] methods.  The same code drives GpuTable (product)
and the numpy oracle table (tests).
"""
from dataclasses import dataclass, field
from typing import Dict, FrozenSet, List, Tuple

from .expr import (CT_TO_CAPF, T_BOOL, T_FLOAT, T_INT, T_NULL, T_STRING, BoolLit, ElementProperty,
                   EndNode, HasLabel, HasType, NullLit, StartNode, Var)
from .header import RecordHeader
from .table import compact_as


@dataclass
class GraphData:
    """An in-memory property graph (okapi-testing InMemoryTestGraph)."""
    nodes: List[Tuple[int, FrozenSet[str], Dict]] = field(default_factory=list)
    rels: List[Tuple[int, int, int, str, Dict]] = field(default_factory=list)


def ctype_of(v):
    if isinstance(v, bool):
        return "BOOLEAN"
    if isinstance(v, int):
        return "INTEGER"
    if isinstance(v, float):
        return "FLOAT"
    if isinstance(v, str):
        return "STRING"
    if isinstance(v, (list, tuple)):  # CTList: the join of the element types
        et = None
        for x in v:
            if x is not None:
                et = _join_type(et, ctype_of(x))
        return f"LIST({et or 'INTEGER'})"
    raise NotImplementedError(f"property value {v!r} of type {type(v).__name__}")


def _join_type(a, b):
    if a is None:
        return b
    if b is None or a == b:
        return a
    if {a, b} == {"INTEGER", "FLOAT"}:
        return "FLOAT"
    if {a, b} == {"LIST(INTEGER)", "LIST(FLOAT)"}:
        return "LIST(FLOAT)"
    # a property schema conflict (MatchTests.scala:380-418 expect an
    # IllegalArgumentException; Flink's unionAll rejects unequal column types)
    from ._lib import IllegalArgumentException
    raise IllegalArgumentException(f"property with conflicting types {a} / {b}")


def _check_schema(node_tables, rel_tables):
    """CAPFSchema.asCapf (flink-cypher/.../schema/CAPFSchema.scala:42-72) over
    the schema of these element tables: the property types of one label
    combination / relationship type are joined across its tables (a union
    graph's members), and any two label combinations that share a label must
    agree on the keys they share — one column per property key and label.
    A conflict is okapi's SchemaException, worded as CAPF words it."""
    from ._lib import IllegalArgumentException, SchemaException

    def fmt(combo):
        return "[" + ", ".join(sorted(combo)) + "]"

    def merged(tables):
        out = {}
        for t in tables:
            keys = out.setdefault(t.labels, {})
            for k, ct in t.props.items():
                try:
                    keys[k] = _join_type(keys.get(k), ct)
                except IllegalArgumentException:
                    raise SchemaException(
                        f"The property type 'UNION({keys[k]}, {ct})' for property '{k}' can not be stored in a "
                        f"Flink column. The unsupported type is specified on label combination "
                        f"{fmt(t.labels)}.") from None
        return out

    combos = merged(node_tables)
    merged(rel_tables)
    for label in sorted(set().union(*combos) if combos else ()):
        with_label = sorted((c for c in combos if label in c), key=sorted)
        for i, c1 in enumerate(with_label):
            for c2 in with_label[i + 1:]:
                for k in sorted(set(combos[c1]) & set(combos[c2])):
                    try:
                        _join_type(combos[c1][k], combos[c2][k])
                    except IllegalArgumentException:
                        raise SchemaException(
                            f"The property type 'UNION({combos[c1][k]}, {combos[c2][k]})' for property '{k}' can "
                            f"not be stored in a Flink column. The conflict appears between label combinations "
                            f"{fmt(c1)} and {fmt(c2)}.") from None


@dataclass
class ElementTable:
    kind: str                 # "node" | "rel"
    labels: FrozenSet[str]    # label combination (node) or {type} (rel)
    table: object             # backend table
    props: Dict[str, str]     # property key -> CypherType name
    # physical column names inside `table`
    id_col: str = "id"
    src_col: str = "source"
    dst_col: str = "target"

    def prop_col(self, key):
        return "p_" + key


class ScanGraph:
    def __init__(self, session, node_tables, rel_tables, validate=True):
        self.session = session
        self.node_tables = list(node_tables)
        self.rel_tables = list(rel_tables)
        # ScanGraph.validate: one table per label combination / rel type
        # (okapi-relational/.../impl/graph/ScanGraph.scala:115-143); a union
        # graph scans every member's tables (UnionGraph.scala:74-115)
        combos = [t.labels for t in self.node_tables]
        if validate and len(combos) != len(set(combos)):
            raise ValueError("more than one node table per label combination")
        types = [t.labels for t in self.rel_tables]
        if validate and len(types) != len(set(types)):
            raise ValueError("more than one relationship table per type")
        # aligned scans per (element tables, labels, properties), built once
        # with canonical column names and renamed per variable by a zero-copy
        # select: the graph is immutable, so a scan (and the statistics of
        # a multi-table UNION ALL behind it) is computed once per graph — the
        # role of okapi's Cache operator (RelationalOptimizer.scala:37-92)
        self._scan_cache = {}
        # planning metadata of a scan per (kind, variable, labels): the header
        # and the column renaming (each call still returns a fresh select)
        self._scan_meta = {}

    @property
    def rel_types(self):
        return sorted(next(iter(t.labels)) for t in self.rel_tables)

    @staticmethod
    def from_data(session, g: GraphData, compact=False):
        """CAPFScanGraphFactory: one element table per label combination / type."""
        by_combo, by_type = {}, {}
        for nid, labels, props in g.nodes:
            by_combo.setdefault(frozenset(labels), []).append((nid, props))
        for rid, s, t, typ, props in g.rels:
            by_type.setdefault(typ, []).append((rid, s, t, props))
        node_tables, rel_tables = [], []
        for combo, rows in sorted(by_combo.items(), key=lambda kv: sorted(kv[0])):
            keys = {}
            for _, props in rows:
                for k, v in props.items():
                    if v is not None:
                        keys[k] = _join_type(keys.get(k), ctype_of(v))
            cols = [("id", T_INT, [r[0] for r in rows], None)]
            for k in sorted(keys):
                vals = [_coerce(r[1].get(k), keys[k]) for r in rows]
                cols.append(("p_" + k, CT_TO_CAPF[keys[k]], vals, None))
            t = session.table(cols, nrows=len(rows))
            node_tables.append(ElementTable("node", combo, compact_as(t, compact), keys))
        for typ, rows in sorted(by_type.items()):
            keys = {}
            for *_, props in rows:
                for k, v in props.items():
                    if v is not None:
                        keys[k] = _join_type(keys.get(k), ctype_of(v))
            cols = [("id", T_INT, [r[0] for r in rows], None),
                    ("source", T_INT, [r[1] for r in rows], None),
                    ("target", T_INT, [r[2] for r in rows], None)]
            for k in sorted(keys):
                vals = [_coerce(r[3].get(k), keys[k]) for r in rows]
                cols.append(("p_" + k, CT_TO_CAPF[keys[k]], vals, None))
            t = session.table(cols, nrows=len(rows))
            rel_tables.append(ElementTable("rel", frozenset([typ]), compact_as(t, compact), keys))
        return ScanGraph(session, node_tables, rel_tables)

    def union_all(self, *others):
        """graph.unionAll(others) (RelationalCypherGraph.scala:124-139): member i
        is PrefixedGraph(g, i) — every element id (and rel endpoint) tagged with
        the graph's index in its top byte (PrefixId; ids are LONGs here, so the
        tag is i << 56 on ids below 2^56) — and the union scans all members'
        tables (UnionGraph.scala:74-115)."""
        from ._lib import IllegalArgumentException
        from .expr import Add, IntegerLit
        nodes, rels = [], []
        for i, g in enumerate((self,) + others):
            if g.session is not self.session:
                raise IllegalArgumentException("union of graphs of different sessions")
            for t in g.node_tables + g.rel_tables:
                cols = [t.id_col] + ([t.src_col, t.dst_col] if t.kind == "rel" else [])
                tab = t.table
                if i:
                    h = RecordHeader({Var(c): c for c in cols})
                    tab = tab.withColumns(*[(Add(Var(c), IntegerLit(i << 56)), c) for c in cols], header=h, params={})
                e = ElementTable(t.kind, t.labels, tab, t.props, t.id_col, t.src_col, t.dst_col)
                (nodes if t.kind == "node" else rels).append(e)
        _check_schema(nodes, rels)  # the union's schema (UnionTests.scala:284-301)
        return ScanGraph(self.session, nodes, rels, validate=False)

    # ------------------------------------------------------------ scans
    def node_scan(self, var_name, labels=()):
        """ScanGraph.scanOperator for NodePattern(CTNode(labels))."""
        key = ("node", var_name, tuple(labels))
        meta = self._scan_meta.get(key)
        if meta is not None:
            return self._scan_from_meta(meta)
        want = frozenset(labels)
        sel = [t for t in self.node_tables if want <= t.labels]
        v = Var(var_name, "NODE")
        all_labels = sorted(set().union(*[t.labels for t in sel])) if sel else sorted(want)
        props = {}
        for t in sel:
            for k, ct in t.props.items():
                props[k] = _join_type(props.get(k), ct)
        header = {v: var_name}
        for l in all_labels:
            header[HasLabel(v, l)] = f"{var_name}:{l}"
        for k in sorted(props):
            header[ElementProperty(v, k, props[k])] = f"{var_name}.{k}"
        h = RecordHeader(header)
        order = [header[e] for e in header]
        types = [T_INT] + [T_BOOL] * len(all_labels) + [CT_TO_CAPF[props[k]] for k in sorted(props)]
        return self._align_union(sel, h, order, types, v, all_labels, props, rel=False, meta_key=key)

    def rel_scan(self, var_name, types=()):
        """ScanGraph.scanOperator for RelationshipPattern(CTRelationship(types))."""
        key = ("rel", var_name, tuple(types))
        meta = self._scan_meta.get(key)
        if meta is not None:
            return self._scan_from_meta(meta)
        want = set(types)
        sel = [t for t in self.rel_tables if not want or (t.labels & want)]
        r = Var(var_name, "RELATIONSHIP")
        all_types = sorted(set().union(*[t.labels for t in sel])) if sel else sorted(want)
        props = {}
        for t in sel:
            for k, ct in t.props.items():
                props[k] = _join_type(props.get(k), ct)
        header = {r: var_name, StartNode(r): f"source({var_name})", EndNode(r): f"target({var_name})"}
        for ty in all_types:
            header[HasType(r, ty)] = f"{var_name}:{ty}"
        for k in sorted(props):
            header[ElementProperty(r, k, props[k])] = f"{var_name}.{k}"
        h = RecordHeader(header)
        order = [header[e] for e in header]
        tys = [T_INT, T_INT, T_INT] + [T_BOOL] * len(all_types) + [CT_TO_CAPF[props[k]] for k in sorted(props)]
        return self._align_union(sel, h, order, tys, r, all_types, props, rel=True, meta_key=key)

    @staticmethod
    def _scan_from_meta(meta):
        # the scan of (var, labels) is an immutable view of the graph's element
        # tables: built once, then handed out again (no select call per query)
        return meta[3]

    def _align_union(self, sel, h, order, types, v, flags, props, rel, meta_key=None):
        from .planner import Planned
        if not sel:
            return Planned(self.session.empty(order, types), h)
        canon = "_scan_"
        canon_order = _scan_columns(canon, flags, props, rel)
        assert len(canon_order) == len(order) and _scan_columns(v.vname, flags, props, rel) == order
        key = (rel, tuple(id(t) for t in sel), tuple(flags), tuple(sorted(props.items())))
        base = self._scan_cache.get(key)
        if base is None:
            base = self._build_union(sel, h, canon_order, Var(canon, v.ctype), flags, props, rel)
            self._scan_cache[key] = base
        pairs = tuple(zip(canon_order, order))
        planned = Planned(base.select(*pairs), h)
        if meta_key is not None:
            self._scan_meta[meta_key] = (base, pairs, h, planned)
        return planned

    def _build_union(self, sel, h, order, v, flags, props, rel):
        name = v.vname
        parts = []
        for t in sel:
            cols = [(t.id_col, name)]
            if rel:
                cols += [(t.src_col, f"source({name})"), (t.dst_col, f"target({name})")]
            present = set()
            for k in sorted(props):
                if k in t.props:
                    cols.append((t.prop_col(k), f"{name}.{k}"))
                    present.add(k)
            tab = t.table.select(*cols)
            adds = []
            for f in flags:
                adds.append((BoolLit(f in t.labels), f"{name}:{f}"))
            for k in sorted(props):
                if k not in present:
                    adds.append((NullLit(props[k]), f"{name}.{k}"))
            if adds:
                tab = tab.withColumns(*adds, header=RecordHeader({}), params={})
            tab = tab.select(*order)
            parts.append(tab)
        out = parts[0]
        for p in parts[1:]:
            out = out.unionAll(p)
        return out


def _planned(table, header):
    from .planner import Planned
    global _planned
    _planned = Planned  # bound once: no import statement per scan
    return Planned(table, header)


def _scan_columns(name, flags, props, rel):
    """Column names of an aligned scan of variable `name` (header order)."""
    cols = [name] + ([f"source({name})", f"target({name})"] if rel else [])
    cols += [f"{name}:{f}" for f in flags]
    cols += [f"{name}.{k}" for k in sorted(props)]
    return cols


def _coerce(v, ct):
    if v is None:
        return None
    if ct == "FLOAT":
        return float(v)
    if ct == "LIST(FLOAT)":
        return [None if x is None else float(x) for x in v]
    return v
