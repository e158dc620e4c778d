"""Distributed Table[T]: the okapi Table SPI over G ranks, one shard per GPU.

SURVEY §8(e): the graph is hash-partitioned by node id over the GPUs of a
node and every hop's frontier rows are shuffled by join key with an
all-to-all; GROUP BY / DISTINCT move rows (or partial aggregates) by h(key).
This module is that execution layer for EVERY Table operator, so the
unchanged planner (planner.py, the RelationalPlanner restatement) runs a
whole Cypher query distributed by calling the SPI on `DistTable`s instead
of `GpuTable`s.  It mirrors what Flink does underneath FlinkTable: a DataSet
join / groupBy / distinct repartitions its inputs by a hash of the key (or
broadcasts a small side) before the local operator
(flink-cypher/.../impl/table/FlinkTable.scala:123-196).

Placement of a DistTable's rows:
  "hash"        rows spread over the ranks; `part` = the columns whose equal
                values are known to sit on one rank (the routing key of the
                last shuffle, its aliases, and join partners of it)
  "root"        every row on rank 0 (ORDER BY results, global aggregates,
                the unit table)
  "replicated"  every rank holds all rows (the broadcast side of a join;
                internal, never returned by an SPI call)

Operator rules (local = the rank's GpuTable; no exchange unless stated):
  select / drop / filter / withColumns / cache      local; `part` follows renames
  join inner / left_outer   local if co-partitioned on a key pair; else the
                            right side is BROADCAST when |right|·G < |left|
                            (cheaper than moving the left rows), else both
                            sides are SHUFFLED by the first key pair
  join right_outer / full_outer   co-partitioned (shuffle), never broadcast
  join cross                the right side broadcast
  unionAll                  local (both shards)
  group with keys           SHUFFLE by the key columns unless partitioned on
                            one of them, then local group
  group without keys        count/sum/min/max/avg: local partials, gathered
                            to rank 0 and combined there (avg = Σsum / Σcount);
                            collect / DISTINCT aggregates: rows gathered to rank 0
  distinct                  SHUFFLE by the key columns (unless partitioned)
  orderBy / skip / limit    rows gathered to rank 0, local operator
  size / rows               local, then summed / gathered over the ranks

The exchange itself is pluggable: `GpuExchange` (product) routes rows on the
GPU (capf_table_hash_route, csrc/shuffle.hip) and moves them with ONE
all_to_all_single per shuffle (RCCL over xGMI; host-staged under gloo), the
columns packed row-major; the CPU tests drive the same DistTable logic over
the numpy oracle with their own exchange.
"""
from ctypes import byref, c_int32, c_int64, c_uint64, c_void_p

import torch
import torch.distributed as dist

from . import _lib
from .expr import (AGG_AVG, AGG_COUNT, AGG_COUNT_STAR, AGG_MAX, AGG_MIN, AGG_SUM, T_BOOL, T_INT, T_NULL, T_STRING, Count,
                   Divide, Explode, Max, Min, Sum, ToFloat, Var)
from .header import RecordHeader

ROUTE_MAXK = 8  # routing keys per shuffle (shuffle.hip); a subset of a key tuple routes correctly


class GpuExchange:
    """Row exchange of GpuTable shards over a torch.distributed group: RCCL
    on the GPU tensors (backend "nccl"), host-staged under "gloo"."""

    def __init__(self, session, group=None):
        self.s = session
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.staged = dist.get_backend(group) != "nccl"
        self.dev = torch.device("cuda", torch.cuda.current_device())

    # -- collectives on small host values ------------------------------------
    def all_sum(self, v):
        t = torch.tensor([int(v)], dtype=torch.int64, device="cpu" if self.staged else self.dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return int(t.item())

    def all_max_vec(self, vals):
        t = torch.tensor(list(vals) or [0], dtype=torch.int32, device="cpu" if self.staged else self.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return t.tolist()[:len(vals)]

    def all_gather_obj(self, obj):
        out = [None] * self.world
        dist.all_gather_object(out, obj, group=self.group)
        return out

    # -- row movement -----------------------------------------------------------
    def route(self, table, keys):
        """(table with rows grouped by owner, per-owner row counts)."""
        keys = list(keys)[:ROUTE_MAXK]
        counts = (c_int64 * self.world)()
        h = c_void_p()
        _lib.call("capf_table_hash_route", table._h, len(keys), _lib.strs(keys), self.world, counts, byref(h))
        from .table import GpuTable
        return GpuTable(self.s, h), list(counts)

    def shuffle(self, table, keys):
        routed, counts = self.route(table, keys)
        return self.send(routed, counts)

    def own_share(self, table, keys):
        """Rows of a table every rank holds in full that this rank owns by
        h(keys) (sharding at ingest: no exchange)."""
        routed, counts = self.route(table, keys)
        off = sum(counts[:self.rank])
        return routed.skip(off).limit(counts[self.rank]).cache()

    def to_root(self, table):
        n = table.size
        return self.send(table, [n if p == 0 else 0 for p in range(self.world)])

    def replicate(self, table):
        return self.send(table, [table.size] * self.world, repeat=True)

    def all_max_i64(self, vals):
        t = torch.tensor(list(vals) or [0], dtype=torch.int64, device="cpu" if self.staged else self.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return t.tolist()[:len(vals)]

    def _layout(self, table):
        """One wire layout on every rank (capf_table_pack_rows): per column the
        width of (value − base) — FOR24 / FOR32 where the value range over ALL
        ranks fits 24 / 32 bits, 8 B otherwise — and whether it carries a
        validity byte.  Everything is agreed in ONE int64 MAX all-reduce: the
        local NULL flags, −min and max of every INTEGER / STRING column, and
        (STRING columns travel as dictionary codes) the dictionary size and
        digest with their negations (min == max on every rank)."""
        cols = table.physicalColumns
        types = [table.capf_type(c) for c in cols]
        if any(t not in (0, 1, 2, 3, 4) for t in types):
            raise _lib.NotImplementedException("LIST columns are not moved between ranks")
        k = len(cols)
        has, lo, hi = [], [], []
        big = (1 << 63) - 1
        for c, t in zip(cols, types):
            v = c_int32()
            _lib.call("capf_table_has_nulls", table._h, c.encode(), byref(v))
            has.append(v.value)
            if t in (T_INT, T_STRING):
                mn, mx, nn = c_int64(), c_int64(), c_int64()
                _lib.call("capf_table_column_range", table._h, c.encode(), byref(mn), byref(mx), byref(nn))
                lo.append(-mn.value if nn.value else -big)
                hi.append(mx.value if nn.value else -big)
            else:
                lo.append(-big)
                hi.append(-big)
        check = []
        if T_STRING in types:
            cnt, dig = c_int64(), c_uint64()
            _lib.call("capf_string_digest", self.s._h, byref(cnt), byref(dig))
            d = dig.value - (1 << 64) if dig.value >= (1 << 63) else dig.value
            check = [cnt.value, -cnt.value, d, -d if d != -(1 << 63) else big]
        got = self.all_max_i64(has + lo + hi + check)
        if check:
            c0 = 3 * k
            if got[c0] != -got[c0 + 1] or (got[c0 + 2] != -got[c0 + 3] and check[2] != -(1 << 63)):
                raise _lib.IllegalStateException(
                    "string dictionaries differ between ranks: STRING columns cannot be exchanged as codes")
        # an all-NULL column is rebuilt from its type alone
        nullable = [bool(x) and t != T_NULL for x, t in zip(got[:k], types)]
        width, base = [], []
        for j, t in enumerate(types):
            if t == T_NULL:
                width.append(0), base.append(0)
            elif t == T_BOOL:
                width.append(1), base.append(0)
            elif t in (T_INT, T_STRING):
                gmin, gmax = -got[k + j], got[2 * k + j]
                if gmax < gmin:  # no value anywhere
                    width.append(3), base.append(0)
                elif gmax - gmin < (1 << 24):
                    width.append(3), base.append(gmin)
                elif gmax - gmin < (1 << 32):
                    width.append(4), base.append(gmin)
                else:
                    width.append(8), base.append(0)
            else:
                width.append(8), base.append(0)
        return cols, types, width, base, nullable

    def send(self, table, counts, repeat=False):
        """Rows [off_p, off_p + counts[p]) of `table` go to rank p (every row
        to every rank when repeat); returns the rows this rank receives, in
        sender order.  Rows are packed on the GPU in the narrow wire layout
        (capf_table_pack_rows) and moved by one all_to_all_single."""
        cols, types, width, base, nullable = self._layout(table)
        n = table.size
        k = len(cols)
        arrs = (_lib.strs(cols), (c_int32 * max(k, 1))(*width), (c_int64 * max(k, 1))(*base),
                (c_int32 * max(k, 1))(*[int(x) for x in nullable]))
        W = sum(width) + sum(nullable)
        dev = "cpu" if self.staged else self.dev
        rows = torch.empty(max(n * W, 1), dtype=torch.uint8, device=self.dev)
        wb = c_int32()
        torch.cuda.current_stream().synchronize()
        _lib.call("capf_table_pack_rows", table._h, k, *arrs, byref(wb), c_void_p(rows.data_ptr()))
        assert wb.value == W, (wb.value, W)
        rows = rows[:n * W].view(n, W)
        if repeat:
            rows = rows.repeat(self.world, 1)
        send_counts = torch.tensor(counts, dtype=torch.int64, device=dev)
        recv_counts = torch.empty_like(send_counts)
        dist.all_to_all_single(recv_counts, send_counts, group=self.group)
        rc = recv_counts.tolist()
        m = sum(rc)
        out = torch.empty((max(m, 1), W), dtype=torch.uint8, device=dev)[:m]
        if W > 0:
            src = rows.to(dev) if self.staged else rows
            dist.all_to_all_single(out, src, rc, list(counts), group=self.group)
        if self.staged:
            out = out.to(self.dev)
        torch.cuda.current_stream().synchronize()
        h = c_void_p()
        ty = (c_int32 * max(k, 1))(*types)
        _lib.call("capf_table_from_packed_rows", self.s._h, k, arrs[0], ty, arrs[1], arrs[2], arrs[3],
                  c_void_p(out.data_ptr() if m > 0 and W > 0 else 0), m, byref(h))
        from .table import GpuTable
        return GpuTable(self.s, h)


class DistSession:
    """RelationalCypherSession side of the distributed backend: table
    factories over the rank-local session plus the exchange."""

    def __init__(self, local_session, exchange):
        self.local = local_session
        self.ex = exchange
        # value maps (toString / concatenation of columns) intern the union of
        # every rank's values: the ranks' string dictionaries stay equal
        local_session.value_map_gather = exchange.all_gather_obj
        self.world = exchange.world
        self.rank = exchange.rank
        # deferred inner joins over base shards (set by dist_node_partitioned_graph)
        self.defer = False

    def intern(self, s):
        return self.local.intern(s)

    def lookup(self, code):
        return self.local.lookup(code)

    def unit(self):
        # the one unit row lives on rank 0
        t = self.local.unit() if self.rank == 0 else self.local.empty([], [])
        return DistTable(self, t, placement="root")

    def empty(self, names, types):
        return DistTable(self, self.local.empty(names, types), placement="root")

    def table(self, columns, nrows=None):
        """A table every rank passes in full (same rows, same order): rank 0
        keeps the rows."""
        t = self.local.table(columns, nrows)
        if self.rank != 0:
            t = t.limit(0)
        return DistTable(self, t, placement="root")

    def shard(self, table, key):
        """A table every rank holds in full, hash-partitioned by `key`
        (graph ingest: rank r keeps the rows it owns, no exchange)."""
        return DistTable(self, self.ex.own_share(table, [key]), part={key})


def _dist_key_cols(table, by, header):
    cols = []
    for v in by:
        for e in header.owned_by(v):
            c = header.column(e)
            if c in table.physicalColumns and c not in cols:
                cols.append(c)
    return cols


class Prov:
    """Provenance of a table that is a projection of one base shard of a
    node-partitioned graph (dist_node_partitioned_graph): kind "node" / "rel",
    the shard's graph-level facts (`info`) and physical column → base column.
    Kept through select / withColumns / drop / cache, dropped by anything that
    changes the rows."""
    __slots__ = ("kind", "info", "cols")

    def __init__(self, kind, info, cols):
        self.kind, self.info, self.cols = kind, info, dict(cols)

    def renamed(self, pairs):
        cols = {a: self.cols[c] for c, a in pairs if c in self.cols}
        return Prov(self.kind, self.info, cols) if cols else None

    def without(self, names):
        cols = {c: b for c, b in self.cols.items() if c not in names}
        return Prov(self.kind, self.info, cols) if cols else None


class _NoMatch(Exception):
    pass


class DistTable:
    """Table[DistTable]: the rank's shard (`local`, a backend table) plus its
    placement.  Every method is collective: all ranks call it in the same
    order with the same arguments (the planner is deterministic).

    Deferred evaluation (sessions with `defer` set, i.e. node-partitioned
    graphs): inner joins between projections of base shards, and the filters /
    projections over them, are recorded instead of executed.  The record is
    replayed operator for operator — the same eager decisions, shuffles and
    results — as soon as anything reads the rows; only group(∅, count(*)) looks
    at the whole record first: the 2-hop chain over the rel shard then runs as
    the node-partitioned fused count plus ONE all-reduce (_sharded_two_hop),
    the multi-GPU path of SURVEY §8(e), below the Table SPI."""

    def __init__(self, session, local=None, part=(), placement="hash", prov=None, deferred=None, cols=None):
        self.session = session
        self._local = local
        self._part = frozenset(part) if placement == "hash" else frozenset()
        self._placement = placement
        self.prov = prov
        self._deferred = deferred  # (op, args…) replayed by _force
        self._cols = cols          # physical columns of a deferred table

    @property
    def ex(self):
        return self.session.ex

    def _force(self):
        if self._deferred is None:
            return
        op, *args = self._deferred
        if op == "host_rows":  # the one replicated row of a count held on the host
            names, vals = args
            self._local = self.session.local.table([(n, T_INT, [v], None) for n, v in zip(names, vals)], nrows=1)
            self._part, self._placement, self._deferred = frozenset(), "replicated", None
            return
        if op == "join":
            out = args[0]._join_eager(args[1], args[2], *args[3])
        elif op == "select":
            out = args[0]._select_eager(*args[1])
        elif op == "filter":
            out = args[0]._filter_eager(*args[1:])
        elif op == "withColumns":
            out = args[0]._with_columns_eager(args[1], args[2], args[3])
        else:  # drop
            out = args[0]._drop_eager(*args[1])
        self._local, self._part, self._placement = out.local, out.part, out.placement
        self._deferred = None

    @property
    def local(self):
        if self._deferred is not None:
            self._force()
        return self._local

    @property
    def part(self):
        if self._deferred is not None:
            self._force()
        return self._part

    @property
    def placement(self):
        if self._deferred is not None:
            self._force()
        return self._placement

    def _deferrable(self):
        return self._deferred is not None or self.prov is not None

    def _defer(self, op, cols):
        return DistTable(self.session, deferred=op, cols=list(cols))

    def _wrap(self, local, part=(), placement=None, prov=None):
        return DistTable(self.session, local, part, placement or self.placement, prov)

    # ------------------------------------------------------------- CypherTable
    @property
    def physicalColumns(self):
        if self._deferred is not None:
            return list(self._cols)
        return self.local.physicalColumns

    @property
    def columnType(self):
        return self.local.columnType

    def capf_type(self, col):
        return self.local.capf_type(col)

    @property
    def size(self):
        n = self.local.size
        return n if self.placement == "replicated" else self.ex.all_sum(n)

    def _host_values(self, col):
        """The values of `col` when this table is (a projection of) a count's
        host-held row — read without building or downloading a device table."""
        d = self._deferred
        if d is None:
            return None
        if d[0] == "host_rows":
            names, vals = d[1], d[2]
            return [vals[names.index(col)]] if col in names else None
        if d[0] == "select":
            for c in d[2]:
                src, alias = (c, c) if isinstance(c, str) else tuple(c)
                if alias == col:
                    return d[1]._host_values(src)
        return None

    def column_values(self, col):
        hv = self._host_values(col)
        if hv is not None:
            return hv
        vals = self.local.column_values(col)
        if self.placement == "replicated":
            return vals
        return [x for part in self.ex.all_gather_obj(vals) for x in part]

    @property
    def rows(self):
        cols = self.physicalColumns
        data = [self.column_values(c) for c in cols]
        n = len(data[0]) if data else self.size
        return [{c: data[i][r] for i, c in enumerate(cols)} for r in range(n)]

    # ------------------------------------------------------------- placement moves
    def _shuffled(self, keys):
        return self.ex.shuffle(self.local, keys)

    def _rooted(self):
        if self.placement == "root":
            return self.local
        if self.placement == "replicated":
            return self.local if self.session.rank == 0 else self.local.limit(0)
        return self.ex.to_root(self.local)

    # ------------------------------------------------------------- Table[T]
    def cache(self):
        if self._deferred is not None:
            return self
        return self._wrap(self.local.cache(), self.part, prov=self.prov)

    def select(self, *cols):
        pairs = [(c, c) if isinstance(c, str) else tuple(c) for c in cols]
        if self._deferred is not None:
            return self._defer(("select", self, cols), [a for _, a in pairs])
        return self._select_eager(*cols)

    def _select_eager(self, *cols):
        pairs = [(c, c) if isinstance(c, str) else tuple(c) for c in cols]
        part = {a for c, a in pairs if c in self.part}
        return self._wrap(self.local.select(*cols), part, prov=self.prov.renamed(pairs) if self.prov else None)

    def filter(self, expr, header=None, params=None):
        if self._deferred is not None:
            return self._defer(("filter", self, expr, header, params), self._cols)
        return self._filter_eager(expr, header, params)

    def _filter_eager(self, expr, header=None, params=None):
        return self._wrap(self.local.filter(expr, header, params), self.part)

    def drop(self, *cols):
        if self._deferred is not None:
            return self._defer(("drop", self, cols), [c for c in self._cols if c not in cols])
        return self._drop_eager(*cols)

    def _drop_eager(self, *cols):
        return self._wrap(self.local.drop(*cols), self.part - set(cols),
                          prov=self.prov.without(set(cols)) if self.prov else None)

    def withColumns(self, *columns, header=None, params=None):
        if any(isinstance(e, Explode) for e, _ in columns):
            # UNWIND multiplies each rank's rows in place: the placement stays,
            # the projection provenance does not (rows changed)
            local = self.local.withColumns(*columns, header=header, params=params)
            return self._wrap(local, self.part - {c for _, c in columns})
        if self._deferred is not None:
            out = list(self._cols)
            for _, c in columns:
                if c not in out:
                    out.append(c)
            return self._defer(("withColumns", self, columns, header, params), out)
        return self._with_columns_eager(columns, header, params)

    def _with_columns_eager(self, columns, header=None, params=None):
        written = {c for _, c in columns}
        return self._wrap(self.local.withColumns(*columns, header=header, params=params), self.part - written,
                          prov=self.prov.without(written) if self.prov else None)

    def unionAll(self, other):
        if "replicated" in (self.placement, other.placement):
            raise _lib.IllegalStateException("union of a broadcast table")
        if self.placement == other.placement == "root":
            return self._wrap(self.local.unionAll(other.local), placement="root")
        part = self.part & other.part if self.placement == other.placement == "hash" else ()
        return self._wrap(self.local.unionAll(other.local), part, "hash")

    def join(self, other, join_type, *join_cols):
        if getattr(self.session, "defer", False) and join_type == "inner" and self._deferrable() \
                and other._deferrable():
            return self._defer(("join", self, other, join_type, tuple(join_cols)),
                               self.physicalColumns + other.physicalColumns)
        return self._join_eager(other, join_type, *join_cols)

    def _join_eager(self, other, join_type, *join_cols):
        jt = join_type
        pairs = list(join_cols)
        if self.placement == other.placement == "root":
            return self._wrap(self.local.join(other.local, jt, *pairs), placement="root")
        if jt == "cross":
            right = other.local if other.placement == "replicated" else self.ex.replicate(other.local)
            left = self.local if self.placement != "replicated" else self._rooted()
            place = "root" if self.placement in ("root", "replicated") else "hash"
            return self._wrap(left.join(right, jt, *pairs), self.part, place)
        lpart = self.part if self.placement == "hash" else frozenset()
        rpart = other.part if other.placement == "hash" else frozenset()
        co = next(((l, r) for l, r in pairs if l in lpart and r in rpart), None)
        if co is not None:
            left, right, lp, rp, key = self.local, other.local, lpart, rpart, co
        else:
            if jt in ("inner", "left_outer") and self.placement == "hash":
                nl, nr = self.size, other.size
                if nr * self.session.world < nl:  # broadcast the right side
                    right = other.local if other.placement == "replicated" else self.ex.replicate(other.local)
                    part = set(lpart)
                    if jt == "inner":
                        part |= {r for l, r in pairs if l in lpart}
                    return self._wrap(self.local.join(right, jt, *pairs), part, "hash")
            # co-partition on a pair: keep a side already partitioned on it
            key = next(((l, r) for l, r in pairs if l in lpart), None) or \
                next(((l, r) for l, r in pairs if r in rpart), None) or pairs[0]
            l0, r0 = key
            if l0 in lpart:
                left, lp = self.local, lpart
            else:
                left, lp = self._moved_for_join(self, l0), frozenset([l0])
            if r0 in rpart:
                right, rp = other.local, rpart
            else:
                right, rp = self._moved_for_join(other, r0), frozenset([r0])
        out = left.join(right, jt, *pairs)
        l0, r0 = key
        if jt == "inner":
            part = set(lp) | set(rp) | {l0, r0}
        elif jt == "left_outer":
            part = set(lp)
        elif jt == "right_outer":
            part = set(rp)
        else:
            part = set()
        return self._wrap(out, part, "hash")

    def _moved_for_join(self, t, key):
        if t.placement == "replicated":
            # keep one copy (rank 0's) and route it
            return t.ex.shuffle(t._rooted(), [key])
        return t.ex.shuffle(t.local, [key])

    def orderBy(self, *sort_items, header=None, params=None):
        return self._wrap(self._rooted().orderBy(*sort_items, header=header, params=params), placement="root")

    def skip(self, n):
        return self._wrap(self._rooted().skip(n), placement="root")

    def limit(self, n):
        return self._wrap(self._rooted().limit(n), placement="root")

    def distinct(self, *cols):
        keys = list(cols) or self.physicalColumns
        if self.placement == "root" or not keys:
            base = self._rooted()
            return self._wrap(base.distinct(*cols), placement="root")
        if self.placement == "hash" and any(k in self.part for k in keys):
            return self._wrap(self.local.distinct(*cols), self.part & set(keys))
        moved = self.ex.shuffle(self.local if self.placement == "hash" else self._rooted(), keys)
        part = {keys[0]} if len(keys) == 1 else ()
        return self._wrap(moved.distinct(*cols), part, "hash")

    def group(self, by, aggregations, header=None, params=None):
        if self._deferred is not None and not list(by) and aggregations and \
                all(a.kind == AGG_COUNT_STAR for a in aggregations.values()):
            count = _sharded_two_hop(self)
            if count is not None:
                names = list(aggregations)
                # every rank holds the all-reduced count: the one row is replicated
                # (reading it back needs no gather), and it stays on the host until
                # an operator needs it on the device (records read it directly)
                return DistTable(self.session, deferred=("host_rows", names, [count] * len(names)), cols=names)
        keys = _dist_key_cols(self.local, by, header)
        if self.placement == "root":
            out = self.local.group(by, aggregations, header=header, params=params)
            if not keys and self.session.rank != 0:
                out = out.limit(0)  # the one global row lives on rank 0
            return self._wrap(out, placement="root")
        if keys:
            if self.placement == "hash" and any(k in self.part for k in keys):
                base, part = self.local, self.part & set(keys)
            else:
                src = self.local if self.placement == "hash" else self._rooted()
                base = self.ex.shuffle(src, keys)
                part = {keys[0]} if len(keys) == 1 else set()
            return self._wrap(base.group(by, aggregations, header=header, params=params), part, "hash")
        if self.placement == "replicated":
            base = self._rooted()
            out = base.group(by, aggregations, header=header, params=params)
            return self._wrap(out if self.session.rank == 0 else out.limit(0), placement="root")
        return self._global_aggregate(aggregations, header, params)

    def _global_aggregate(self, aggregations, header, params):
        names = list(aggregations)
        decomposable = all(a.kind in (AGG_COUNT_STAR, AGG_COUNT, AGG_SUM, AGG_MIN, AGG_MAX, AGG_AVG)
                           and not getattr(a, "distinct", False) for a in aggregations.values())
        rank0 = self.session.rank == 0
        if not decomposable:
            base = self.ex.to_root(self.local)
            out = base.group([], aggregations, header=header, params=params)
            return self._wrap(out if rank0 else out.limit(0), placement="root")
        # phase 1: one partial row per rank
        partial, final, avgs = {}, {}, []
        for i, name in enumerate(names):
            a = aggregations[name]
            p = f"__dist_p{i}"
            if a.kind in (AGG_COUNT_STAR, AGG_COUNT):
                partial[p] = a
                final[name] = Sum(Var(p))
            elif a.kind == AGG_SUM:
                partial[p] = a
                final[name] = Sum(Var(p))
            elif a.kind == AGG_MIN:
                partial[p] = a
                final[name] = Min(Var(p))
            elif a.kind == AGG_MAX:
                partial[p] = a
                final[name] = Max(Var(p))
            else:  # avg = Σ sum / Σ count, a FLOAT also over INTEGER values
                pc = f"__dist_c{i}"
                partial[p] = Sum(a.expr)
                partial[pc] = Count(a.expr)
                final[f"__dist_s{i}"] = Sum(Var(p))
                final[f"__dist_n{i}"] = Sum(Var(pc))
                avgs.append((name, f"__dist_s{i}", f"__dist_n{i}"))
        loc = self.local.group([], partial, header=header, params=params)
        rows = self.ex.to_root(loc)
        h2 = RecordHeader({Var(p): p for p in partial})
        out = rows.group([], final, header=h2, params={})
        if avgs:
            h3 = RecordHeader({Var(c): c for c in out.physicalColumns})
            out = out.withColumns(*[(Divide(ToFloat(Var(s)), Var(n)), name) for name, s, n in avgs], header=h3,
                                  params={})
        out = out.select(*names)
        return self._wrap(out if rank0 else out.limit(0), placement="root")

    def show(self, rows=20):
        base = self._rooted()
        if self.session.rank == 0:
            base.show(rows)

    def materialize(self):
        if hasattr(self.local, "materialize"):
            self.local.materialize()
        return self


def dist_scan_graph(dsession, graph):
    """The distributed ScanGraph of a graph every rank built in full
    (graph.ScanGraph.from_data on the rank-local session): node tables sharded
    by h(id), relationship tables by h(source) — SURVEY §8(e): "each rel is
    stored on owner(src)".  Hop 1 (S_a ⋈ R on a = source) is then local."""
    from .graph import ElementTable, ScanGraph
    nodes = [ElementTable(t.kind, t.labels, dsession.shard(t.table, t.id_col), t.props, t.id_col, t.src_col,
                          t.dst_col) for t in graph.node_tables]
    rels = [ElementTable(t.kind, t.labels, dsession.shard(t.table, t.src_col), t.props, t.id_col, t.src_col,
                         t.dst_col) for t in graph.rel_tables]
    return ScanGraph(dsession, nodes, rels)


# ------------------------------------------------------------ sharded 2-hop count
def _tree_refs(t, leaves, eqs, neqs):
    """Column name → (leaf index, base column) for the columns of a deferred
    join tree; join keys into `eqs`, NOT(r_i = r_j) filters into `neqs`."""
    if t._deferred is None:
        if t.prov is None:
            raise _NoMatch
        leaves.append(t.prov)
        return {c: (len(leaves) - 1, b) for c, b in t.prov.cols.items()}
    op, *a = t._deferred
    if op == "host_rows":
        raise _NoMatch
    if op == "join":
        lr = _tree_refs(a[0], leaves, eqs, neqs)
        rr = _tree_refs(a[1], leaves, eqs, neqs)
        for x, y in a[3]:
            if x not in lr or y not in rr:
                raise _NoMatch
            eqs.append((lr[x], rr[y]))
        out = dict(lr)
        out.update(rr)
        return out
    refs = _tree_refs(a[0], leaves, eqs, neqs)
    if op == "select":
        return {al: refs[c] for c, al in ((c, c) if isinstance(c, str) else tuple(c) for c in a[1])
                if c in refs}
    if op == "drop":
        return {c: r for c, r in refs.items() if c not in a[1]}
    if op == "withColumns":
        written = {c for _, c in a[1]}
        return {c: r for c, r in refs.items() if c not in written}
    # filter: relationship uniqueness only (front-end rewrite, CypherParser.scala:72)
    from .expr import Ands, Equals, Not
    expr, header = a[1], a[2]
    for term in (expr.exprs if isinstance(expr, Ands) else (expr,)):
        if not (isinstance(term, Not) and isinstance(term.expr, Equals)):
            raise _NoMatch
        x, y = header.get(term.expr.lhs), header.get(term.expr.rhs)
        if x not in refs or y not in refs:
            raise _NoMatch
        neqs.append((refs[x], refs[y]))
    return refs


def _sharded_two_hop(t):
    """count(*) of MATCH (a)-->(b)-->(c) as lowered by the relational planner
    (RelationalPlanner.scala:130-165: S_a ⋈ R1 ⋈ S_b ⋈ R2 ⋈ S_c, NOT(r1 = r2))
    over a node-partitioned graph: every rank adds its partial
    Σ_{b owned} in[b]·out[b] − owned self-loops (the rel shard's `count_partial`)
    and ONE int64 all-reduce sums them.  None when `t` is not that shape (the
    deferred operators are then replayed as usual)."""
    leaves, eqs, neqs = [], [], []
    try:
        _tree_refs(t, leaves, eqs, neqs)
    except _NoMatch:
        return None
    rels = [i for i, p in enumerate(leaves) if p.kind == "rel"]
    nodes = [i for i, p in enumerate(leaves) if p.kind == "node"]
    if len(rels) != 2 or len(nodes) != 3 or len(eqs) != 4 or len(neqs) != 1:
        return None
    info = leaves[rels[0]].info
    if leaves[rels[1]].info is not info or not all(leaves[i].info.get("complete") for i in nodes):
        return None
    if any(leaves[i].info.get("graph") is not info.get("graph") for i in nodes):
        return None
    ends = {}  # (rel leaf, "src"/"dst") → node leaf
    for x, y in eqs:
        if leaves[x[0]].kind == "rel":
            x, y = y, x
        if leaves[x[0]].kind != "node" or leaves[y[0]].kind != "rel" or x[1] != leaves[x[0]].info["id"]:
            return None
        side = "src" if y[1] == info["src"] else "dst" if y[1] == info["dst"] else None
        if side is None or (y[0], side) in ends:
            return None
        ends[(y[0], side)] = x[0]
    (x, y), = neqs
    if {x[0], y[0]} != set(rels) or x[1] != info["id"] or y[1] != info["id"]:
        return None
    r1, r2 = rels
    if ends[(r1, "dst")] != ends[(r2, "src")]:
        r1, r2 = r2, r1
    b = ends[(r1, "dst")]
    if ends[(r2, "src")] != b or len({ends[(r1, "src")], b, ends[(r2, "dst")]}) != 3:
        return None
    return info["count"]()


def dist_node_partitioned_graph(dsession, graph, count_copies=None, compact=True):
    """dist_scan_graph plus the node-partitioned layout of SURVEY §8(e) for the
    2-hop count: rank r also holds the rels whose target it owns (in-copy) and
    those whose source it owns (out-copy), owner(v) = the rank whose node_mix
    bucket range holds v.  `graph` is the full ScanGraph every rank built (one
    node table whose ids are exactly [base, base + n) — the complete node set
    — and one rel table).  count_copies(dsession, rel element table, n, base,
    compact) → a zero-argument function returning the count: this rank's
    partial summed over the ranks by one all-reduce (default: the GPU copies,
    FOR-compacted per `compact`, and capf_chain2_sharded_count).  Graph-ingest
    work, outside any timed query."""
    g = dist_scan_graph(dsession, graph)
    if len(graph.node_tables) != 1 or len(graph.rel_tables) != 1:
        return g
    nt, rt = graph.node_tables[0], graph.rel_tables[0]
    lo, hi, n = _int_range(nt.table, nt.id_col)
    if n == 0 or hi - lo + 1 != n or nt.table.size != n:
        return g
    m = rt.table.size
    for c in (rt.src_col, rt.dst_col):
        a, b, nn = _int_range(rt.table, c)
        if a < lo or b > hi or nn != m:  # a NULL endpoint: no node-partitioned layout
            return g
    # Σ in·out − self-loops equals the plan's NOT(r1 = r2) filter only when rel
    # ids are unique (a repeated id would also drop pairs of distinct rels):
    # otherwise the chain replays as planned
    if _int_range(rt.table, rt.id_col)[2] != m or rt.table.select(rt.id_col).distinct().size != m:
        return g
    total = (count_copies or _gpu_count_copies)(dsession, rt, n, lo, compact)
    ginfo = object()
    node_info = {"complete": True, "graph": ginfo, "id": nt.id_col}
    rel_info = {"graph": ginfo, "id": rt.id_col, "src": rt.src_col, "dst": rt.dst_col, "count": total}
    gn, gr = g.node_tables[0].table, g.rel_tables[0].table
    gn.prov = Prov("node", node_info, {c: c for c in gn.physicalColumns})
    gr.prov = Prov("rel", rel_info, {c: c for c in gr.physicalColumns})
    dsession.defer = True
    return g


def _int_range(table, col):
    """(min, max, non-null count) of an INTEGER column."""
    if hasattr(table, "_h"):
        mn, mx, nn = c_int64(), c_int64(), c_int64()
        _lib.call("capf_table_column_range", table._h, col.encode(), byref(mn), byref(mx), byref(nn))
        return mn.value, mx.value, nn.value
    vals = [v for v in table.column_values(col) if v is not None]
    return (min(vals), max(vals), len(vals)) if vals else (0, -1, 0)


def _gpu_count_copies(dsession, rt, n, lo, compact=True):
    """This rank's in/out copies (capf_table_node_partition, FOR-compacted) and
    the count: its partial enqueued (capf_chain2_sharded_count) into a device
    int64 on the session stream (= torch's current stream), summed in place by
    ONE all-reduce (RCCL orders it after the kernels on that stream), one host
    read."""
    from .dist import node_partitioned_copies, sum_partials
    from .table import chain2_sharded_count_async
    s, world, rank = dsession.local, dsession.world, dsession.rank
    group = getattr(dsession.ex, "group", None)
    in_copy, out_copy = node_partitioned_copies(rt.table, n, world, rank, lo, rt.src_col, rt.dst_col,
                                                compact=compact)
    buf = torch.zeros(1, dtype=torch.int64, device="cuda")

    def total():
        chain2_sharded_count_async(s, in_copy, out_copy, lo, n, world, rank, buf.data_ptr(),
                                   rt.src_col, rt.dst_col)
        sum_partials(buf, group)
        return int(buf.item())
    total.copies = (in_copy, out_copy)
    return total
