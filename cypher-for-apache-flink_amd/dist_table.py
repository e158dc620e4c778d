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
                   Divide, Max, Min, Sum, Var)
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
        self.world = exchange.world
        self.rank = exchange.rank

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


class DistTable:
    """Table[DistTable]: the rank's shard (`local`, a backend table) plus its
    placement.  Every method is collective: all ranks call it in the same
    order with the same arguments (the planner is deterministic)."""

    def __init__(self, session, local, part=(), placement="hash"):
        self.session = session
        self.local = local
        self.part = frozenset(part) if placement == "hash" else frozenset()
        self.placement = placement

    @property
    def ex(self):
        return self.session.ex

    def _wrap(self, local, part=(), placement=None):
        return DistTable(self.session, local, part, placement or self.placement)

    # ------------------------------------------------------------- CypherTable
    @property
    def physicalColumns(self):
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

    def column_values(self, col):
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
        return self._wrap(self.local.cache(), self.part)

    def select(self, *cols):
        pairs = [(c, c) if isinstance(c, str) else tuple(c) for c in cols]
        part = {a for c, a in pairs if c in self.part}
        return self._wrap(self.local.select(*cols), part)

    def filter(self, expr, header=None, params=None):
        return self._wrap(self.local.filter(expr, header, params), self.part)

    def drop(self, *cols):
        return self._wrap(self.local.drop(*cols), self.part - set(cols))

    def withColumns(self, *columns, header=None, params=None):
        written = {c for _, c in columns}
        return self._wrap(self.local.withColumns(*columns, header=header, params=params), self.part - written)

    def unionAll(self, other):
        if "replicated" in (self.placement, other.placement):
            raise _lib.IllegalStateException("union of a broadcast table")
        if self.placement == other.placement == "root":
            return self._wrap(self.local.unionAll(other.local), placement="root")
        part = self.part & other.part if self.placement == other.placement == "hash" else ()
        return self._wrap(self.local.unionAll(other.local), part, "hash")

    def join(self, other, join_type, *join_cols):
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
            else:  # avg = Σ sum / Σ count, integer avg by Java long division
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
            out = out.withColumns(*[(Divide(Var(s), Var(n)), name) for name, s, n in avgs], header=h3, params={})
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
