"""RecordHeader: the expression → physical column mapping of a relational table.

Mirrors the parts of okapi's RecordHeader the Table SPI consumes
(okapi-relational/src/main/scala/org/opencypher/okapi/relational/impl/table/
RecordHeader.scala:68-455): `column(expr)`, `ownedBy(var)` (used by
Table.group, FlinkTable.scala:129-135), `startNodeFor`/`endNodeFor`, and
column naming derived from the expression text (:299-318).
"""
from .expr import ElementProperty, EndNode, HasLabel, HasType, StartNode, Var


def owner_of(e):
    if isinstance(e, (ElementProperty, HasLabel, HasType)):
        return e.owner
    if isinstance(e, (StartNode, EndNode)):
        return e.rel
    return None


class RecordHeader:
    __slots__ = ("_m", "_cols", "_cset")

    def __init__(self, mapping=None):
        self._m = dict(mapping) if mapping else {}
        self._cols = None
        self._cset = None

    # dict-like access used by expression lowering
    def get(self, expr, default=None):
        return self._m.get(expr, default)

    def __contains__(self, expr):
        return expr in self._m

    def __iter__(self):
        return iter(self._m)

    def items(self):
        return self._m.items()

    def column(self, expr):
        try:
            return self._m[expr]
        except KeyError:
            raise KeyError(f"{expr} not in header {list(map(str, self._m))}")

    @property
    def expressions(self):
        return list(self._m)

    @property
    def columns(self):
        if self._cols is None:  # immutable: computed once
            self._cols = list(dict.fromkeys(self._m.values()))
        return list(self._cols)

    def column_set(self):
        """The distinct physical columns as a set (planner renaming checks)."""
        return set(self.column_frozenset())

    def column_frozenset(self):
        if self._cset is None:  # immutable: computed once
            self._cset = frozenset(self._m.values())
        return self._cset

    def owned_by(self, var):
        return [e for e in self._m if e == var or owner_of(e) == var]

    def vars(self):
        return [e for e in self._m if isinstance(e, Var)]

    def start_node_for(self, rel):
        return self.column(StartNode(rel))

    def end_node_for(self, rel):
        return self.column(EndNode(rel))

    def with_expr(self, expr, column):
        m = dict(self._m)
        m[expr] = column
        return RecordHeader(m)

    def union(self, other):
        m = dict(self._m)
        m.update(other._m)
        h = RecordHeader.__new__(RecordHeader)
        h._m = m
        h._cols = None
        h._cset = None
        return h

    def without(self, exprs):
        drop = set(exprs)
        return RecordHeader({e: c for e, c in self._m.items() if e not in drop})

    def renamed(self, fn):
        return RecordHeader({e: fn(e, c) for e, c in self._m.items()})

    def __repr__(self):
        return "RecordHeader(" + ", ".join(f"{e}->{c}" for e, c in self._m.items()) + ")"
