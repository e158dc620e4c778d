"""GpuTable / GpuSession: the host-side mirror of the okapi Table SPI over the
MI355X C-ABI (include/capf_gpu.h).

`GpuTable` implements exactly the methods of
  trait Table[T <: Table[T]] extends CypherTable
  (okapi-relational/src/main/scala/org/opencypher/okapi/relational/api/table/Table.scala:43-178)
with the same names and argument meaning as FlinkTable
(flink-cypher/src/main/scala/org/opencypher/flink/impl/table/FlinkTable.scala:49-199),
so a planner written against the SPI (planner.py, mirroring RelationalPlanner)
drives it unchanged.  Every operation returns a new immutable table; nothing
executes on the GPU until `size` / `rows` (lazy, like the Flink Table API).
"""
import ctypes
import os
from ctypes import byref, c_char_p, c_double, c_int32, c_int64, c_uint64, c_void_p

import numpy as np

from . import _lib
from .expr import (AGG_COUNT_STAR, CAPF_TO_CT, T_BOOL, T_FLOAT, T_INT, T_LIST, T_NULL, T_STRING, Aggregator,
                   Explode, Var, compile_program, explode_values, percentile_value)

JOIN_TYPES = {"inner": 0, "left_outer": 1, "right_outer": 2, "full_outer": 3, "cross": 4}

_NP_DTYPE = {T_INT: np.int64, T_FLOAT: np.float64, T_BOOL: np.uint8, T_STRING: np.int64}


class GpuSession:
    """Backend state of a RelationalCypherSession[GpuTable]
    (okapi-relational/.../api/graph/RelationalCypherSession.scala:63-111)."""

    def __init__(self, device=0, stream=None):
        _lib.load()
        h = c_void_p()
        _lib.call("capf_session_create", int(device), stream, byref(h))
        self._h = h
        self._strings = {}
        self._codes = {}
        self._sets = {}
        self._maps = {}

    def literal_set(self, values):
        """Program name of the session literal set of `values` (int64 values
        or string codes) for CAPF_OP_IN_SET: "\x01set:<id>"."""
        key = tuple(sorted(set(values)))
        nm = self._sets.get(key)
        if nm is None:
            arr = (c_int64 * max(len(key), 1))(*key)
            sid = c_int32()
            _lib.call("capf_session_literal_set", self._h, arr, len(key), byref(sid))
            nm = self._sets[key] = "\x01set:%d" % sid.value
        return nm

    def string_map(self, key):
        """Program name of the session code map of string function `key`
        (expr.string_fn) for CAPF_OP_STR_MAP: "\x01map:<id>".  The function runs
        on the host over every dictionary string (results interned); a map is
        extended and re-registered when the dictionary has grown since."""
        from .expr import string_fn
        cnt, dig = c_int64(), c_uint64()
        _lib.call("capf_string_digest", self._h, byref(cnt), byref(dig))
        n = cnt.value
        if n > CODE_MAP_MAX:  # None: the caller maps the operand's distinct values instead
            return None
        ent = self._maps.get(key)
        if ent is not None and ent[0] >= n:
            return ent[2]
        codes = list(ent[1]) if ent is not None else []
        for c in range(len(codes), n):
            r = string_fn(key, self.lookup(c))
            codes.append(-1 if r is None else self.intern(r))
        arr = (c_int64 * max(len(codes), 1))(*codes)
        mid = c_int32()
        if ent is None:
            _lib.call("capf_session_code_map", self._h, arr, len(codes), byref(mid))
        else:  # the same map grown (in place: no device table left behind per growth)
            _lib.call("capf_session_code_map_extend", self._h, int(ent[2].rsplit(":", 1)[1]), arr, len(codes),
                      byref(mid))
        nm = "\x01map:%d" % mid.value
        self._maps[key] = (n, codes, nm)
        return nm

    @classmethod
    def on_torch_stream(cls, device=0):
        """Session whose work is ordered with torch's: a dedicated torch stream
        becomes torch's current stream and the session's (torch's default
        stream is the legacy null stream, which a non-blocking session stream
        would NOT be ordered with — collectives and .item() would race)."""
        import torch
        st = torch.cuda.Stream(device=device)
        torch.cuda.set_stream(st)
        s = cls(device, stream=c_void_p(st.cuda_stream))
        s.torch_stream = st  # keep it alive
        return s

    def close(self):
        if getattr(self, "_h", None):
            _lib.load().capf_session_destroy(self._h)
            self._h = None

    # -- strings ------------------------------------------------------------
    def intern(self, s):
        c = self._codes.get(s)
        if c is None:
            v = c_int64()
            # (surrogatepass: a Java string may hold a lone UTF-16 surrogate, e.g. a
            # substring splitting a pair; the dictionary keeps it as WTF-8 bytes)
            _lib.call("capf_string_intern", self._h, s.encode("utf-8", "surrogatepass"), byref(v))
            c = v.value
            self._codes[s] = c
            self._strings[c] = s
        return c

    def lookup(self, code):
        s = self._strings.get(code)
        if s is None:
            p = c_char_p()
            _lib.call("capf_string_lookup", self._h, int(code), byref(p))
            s = p.value.decode("utf-8", "surrogatepass")
            self._strings[code] = s
        return s

    # -- table factories ----------------------------------------------------
    def table(self, columns, nrows=None):
        """columns: list of (name, capf_type, values, valid-or-None).

        values: sequence of python values (None = NULL) or a numpy array."""
        lists = [c for c in columns if c[1] == T_LIST]
        if lists:  # CTList properties: the scalar columns first, then each LIST column
            t = self.table([c for c in columns if c[1] != T_LIST],
                           nrows=len(lists[0][2]) if nrows is None else nrows)
            for name, _, values, valid in lists:
                t = t.add_list(name, values, valid)
            return t.select(*[c[0] for c in columns])
        names, types, datas, valids, keep = [], [], [], [], []
        n = nrows
        for name, t, values, valid in columns:
            vals = values
            if not isinstance(vals, np.ndarray) or vals.dtype == object:
                lst = list(vals)
                if valid is None and any(v is None for v in lst):
                    valid = np.array([v is not None for v in lst], dtype=np.uint8)
                if t == T_STRING:
                    vals = np.array([self.intern(v) if v is not None else 0 for v in lst], dtype=np.int64)
                elif t == T_NULL:
                    vals = None
                else:
                    vals = np.array([v if v is not None else 0 for v in lst], dtype=_NP_DTYPE[t])
            elif t != T_NULL:
                vals = np.ascontiguousarray(vals.astype(_NP_DTYPE[t], copy=False))
            m = len(values)
            if n is None:
                n = m
            elif n != m:
                raise _lib.IllegalArgumentException("columns of different length")
            names.append(name)
            types.append(t)
            datas.append(vals.ctypes.data if vals is not None and m > 0 else None)
            if valid is not None:
                valid = np.ascontiguousarray(np.asarray(valid, dtype=np.uint8))
                valids.append(valid.ctypes.data if m > 0 else None)
            else:
                valids.append(None)
            keep += [vals, valid]
        n = n or 0
        k = len(names)
        h = c_void_p()
        _lib.call("capf_table_from_host", self._h, k, _lib.strs(names), (c_int32 * max(k, 1))(*types),
                  (c_void_p * max(k, 1))(*datas), (c_void_p * max(k, 1))(*valids), n, byref(h))
        return GpuTable(self, h)

    def unit(self):
        h = c_void_p()
        _lib.call("capf_table_unit", self._h, byref(h))
        return GpuTable(self, h)

    def empty(self, names, types):
        h = c_void_p()
        k = len(names)
        _lib.call("capf_table_empty", self._h, k, _lib.strs(names), (c_int32 * max(k, 1))(*types), byref(h))
        return GpuTable(self, h)

    def rmat_rels(self, scale, seed, thresholds, first, count, id_base=0, cols=("id", "source", "target")):
        h = c_void_p()
        ta, tab, tabc = thresholds
        _lib.call("capf_rmat_rel_table", self._h, int(scale), int(seed), ta, tab, tabc, int(first),
                  int(count), int(id_base), cols[0].encode(), cols[1].encode(), cols[2].encode(), byref(h))
        return GpuTable(self, h)

    def range_nodes(self, base, n, seed=0, id_col="id", label_col=None):
        h = c_void_p()
        _lib.call("capf_range_node_table", self._h, int(base), int(n), int(seed), id_col.encode(),
                  label_col.encode() if label_col else None, byref(h))
        return GpuTable(self, h)

    def edge_list(self, source, sep, comment=None, cols=("id", "source", "target")):
        """Relationship table parsed on the GPU from a CSV edge list: `source`
        is a path (str) or the file's bytes (capf_edge_list_read / _parse)."""
        h = c_void_p()
        com = comment.encode() if comment else None
        names = [c.encode() for c in cols]
        if isinstance(source, (bytes, bytearray, memoryview)):
            buf = bytes(source)
            _lib.call("capf_edge_list_parse", self._h, buf, len(buf), sep.encode(), com, *names, byref(h))
        else:
            _lib.call("capf_edge_list_read", self._h, os.fsencode(source), sep.encode(), com, *names, byref(h))
        return GpuTable(self, h)

    def csv_read_longs(self, path, sep, names):
        """A CSV table whose declared fields are all LONG, parsed on the GPU
        (capf_csv_read_longs; FSGraphSource.readFromCsv)."""
        h = c_void_p()
        _lib.call("capf_csv_read_longs", self._h, os.fsencode(path), sep.encode(), len(names),
                  _lib.strs(list(names)), byref(h))
        return GpuTable(self, h)

    def csv_parse_longs(self, data, sep, names):
        h = c_void_p()
        buf = bytes(data)
        _lib.call("capf_csv_parse_longs", self._h, buf, len(buf), sep.encode(), len(names),
                  _lib.strs(list(names)), byref(h))
        return GpuTable(self, h)

    def var_length_reach(self, rels, src_col, dst_col, sources, source_id_col, targets, target_id_col,
                         lower, upper, out_source_col, out_reach_col):
        """Fused VarLengthExpand → Distinct(a, b) → Aggregate(a, count(*))
        (capf_var_length_reach): one row (a, reach) per source reaching a target."""
        h = c_void_p()
        _lib.call("capf_var_length_reach", self._h, rels._h, src_col.encode(), dst_col.encode(), sources._h,
                  source_id_col.encode(), targets._h, target_id_col.encode(), int(lower), int(upper),
                  out_source_col.encode(), out_reach_col.encode(), byref(h))
        return GpuTable(self, h)

    # -- profiling ----------------------------------------------------------
    def set_profiling(self, on):
        _lib.call("capf_session_set_profiling", self._h, 1 if on else 0)

    def reset_profile(self):
        _lib.call("capf_session_reset_profile", self._h)

    def profile(self):
        n = c_int32()
        _lib.call("capf_session_profile_count", self._h, byref(n))
        out = {}
        for i in range(n.value):
            name, launches, ms, by = c_char_p(), c_int64(), c_double(), c_double()
            _lib.call("capf_session_profile_entry", self._h, i, byref(name), byref(launches), byref(ms), byref(by))
            out[name.value.decode()] = {"launches": launches.value, "total_ms": ms.value, "bytes": by.value}
        return out

    def last_plan(self):
        return _lib.load().capf_session_last_plan(self._h).decode()

    def sync(self):
        _lib.call("capf_session_sync", self._h)


# distinct operand values (pairs) a value map may hold (toString of a number
# column, concatenation of two columns): each becomes a host-built string
VALUE_MAP_MAX = 1 << 22
# a string function runs over the whole dictionary (a code map) only while the
# dictionary holds at most this many strings; beyond, over the distinct values
# of its operand in the table (a value map)
CODE_MAP_MAX = 1 << 16

# encoded argument arrays of select() per column tuple (scans and renames
# repeat the same selections every query)
_SELECT_ARGS = {}


def _program(expr, header, table, params):
    return compile_program(expr, header, set(table.physicalColumns), params, table.session.intern,
                           table._coltype, getattr(table.session, "literal_set", None),
                           getattr(table.session, "string_map", None),
                           lambda kind, exprs: table._value_map(kind, exprs, header, params))


class GpuTable:
    """Table[GpuTable] over an opaque capf_table handle."""

    def __init__(self, session, handle, cols=None):
        self.session = session
        self._h = handle
        self._cols = cols  # physical columns when the operation defines them (else asked once)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib._lib is not None and not _lib._exiting and getattr(self.session, "_h", None):
            _lib._lib.capf_table_release(h)

    def _new(self, fn, *args, cols=None):
        h = c_void_p()
        _lib.call(fn, *args, byref(h))
        return GpuTable(self.session, h, cols)

    # ---------------------------------------------------------- CypherTable
    @property
    def physicalColumns(self):
        if self._cols is None:
            p, nb, n = c_void_p(), c_int64(), c_int32()
            _lib.call("capf_table_columns", self._h, byref(p), byref(nb), byref(n))
            raw = ctypes.string_at(p.value, nb.value) if nb.value else b""
            self._cols = raw.decode().split("\0")[:n.value]
        return list(self._cols)

    def capf_type(self, col):
        t = c_int32()
        _lib.call("capf_table_column_type", self._h, col.encode(), byref(t))
        return t.value

    def _coltype(self, col):
        """capf type of a column; ("elem", col): the element type of a LIST column."""
        if isinstance(col, tuple):
            return self.list_elem_type(col[1])
        return self.capf_type(col)

    def list_elem_type(self, col):
        """Element type of a LIST column (capf_table_list_info without a value
        count: read off the plan when it says, else the table is evaluated)."""
        et = c_int32()
        _lib.call("capf_table_list_info", self._h, col.encode(), byref(et), None)
        return et.value

    @property
    def columnType(self):
        return {c: CAPF_TO_CT[self.capf_type(c)] for c in self.physicalColumns}

    @property
    def size(self):
        n = c_int64()
        _lib.call("capf_table_size", self._h, byref(n))
        return n.value

    def materialize(self):
        """Evaluate the table into device memory (no download)."""
        _lib.call("capf_table_materialize", self._h)
        return self

    def count_async(self, d_count):
        """`size` (or the count(*) of a global group(∅, {count(*)})) written to
        the device int64 at address d_count, without waiting for the GPU."""
        _lib.call("capf_table_count_async", self._h, c_void_p(int(d_count)))

    def column_arrays(self, col):
        """(values ndarray, valid ndarray[bool]) of a column (materialises)."""
        n = self.size
        t = self.capf_type(col)
        valid = np.zeros(n, dtype=np.uint8)
        if t == T_NULL:
            _lib.call("capf_table_download", self._h, col.encode(), None, valid.ctypes.data if n else None)
            return np.zeros(n, dtype=np.int64), valid.astype(bool)
        vals = np.zeros(n, dtype=_NP_DTYPE[t])
        _lib.call("capf_table_download", self._h, col.encode(), vals.ctypes.data if n else None,
                  valid.ctypes.data if n else None)
        return vals, valid.astype(bool)

    def list_values(self, col):
        """Python lists (None for a NULL list) of a LIST column (collect)."""
        et, nv = c_int32(), c_int64()
        _lib.call("capf_table_list_info", self._h, col.encode(), byref(et), byref(nv))
        n = self.size
        offs = np.zeros(n + 1, dtype=np.int64)
        valid = np.zeros(max(n, 1), dtype=np.uint8)
        t = et.value
        vals = np.zeros(max(nv.value, 1), dtype=_NP_DTYPE.get(t, np.int64))
        _lib.call("capf_table_download_list", self._h, col.encode(), offs.ctypes.data,
                  vals.ctypes.data if nv.value and t != T_NULL else None, valid.ctypes.data if n else None)
        out = []
        for i in range(n):
            if not valid[i]:
                out.append(None)
                continue
            xs = vals[offs[i]:offs[i + 1]].tolist()
            if t == T_STRING:
                xs = [self.session.lookup(x) for x in xs]
            elif t == T_BOOL:
                xs = [bool(x) for x in xs]
            out.append(xs)
        return out

    def column_values(self, col):
        """Python values (None for NULL) of one column."""
        t = self.capf_type(col)
        if t == T_LIST:
            return self.list_values(col)
        vals, valid = self.column_arrays(col)
        if t not in (T_STRING, T_BOOL) and valid.all():
            return vals.tolist()  # no NULLs: the values as they are
        out = []
        for v, ok in zip(vals.tolist(), valid.tolist()):
            if not ok:
                out.append(None)
            elif t == T_STRING:
                out.append(self.session.lookup(v))
            elif t == T_BOOL:
                out.append(bool(v))
            else:
                out.append(v)
        return out

    @property
    def rows(self):
        cols = self.physicalColumns
        data = [self.column_values(c) for c in cols]
        if not data:
            return [{} for _ in range(self.size)]
        return [dict(zip(cols, row)) for row in zip(*data)]

    # ---------------------------------------------------------- Table[T]
    def cache(self):
        return self._new("capf_table_cache", self._h)

    def compact(self, width=4):
        """Materialised copy whose INTEGER columns are FOR32-encoded where
        their value range fits 32 bits (same rows; half the id bytes);
        width=3: FOR24 where the range fits 24 bits (3 B per id)."""
        if width == 4:
            return self._new("capf_table_compact", self._h)
        return self._new("capf_table_compact_width", self._h, int(width))

    def encoding(self, col):
        """(encoding, base) of a column: (0, 0) plain, (1, base) FOR32, (2, base) FOR24."""
        e, b = c_int32(), c_int64()
        _lib.call("capf_table_column_encoding", self._h, col.encode(), byref(e), byref(b))
        return e.value, b.value

    def select(self, *cols):
        try:
            enc = _SELECT_ARGS.get(cols)
        except TypeError:  # unhashable (list) pairs
            enc, cols = None, tuple(c if isinstance(c, str) else tuple(c) for c in cols)
        if enc is None:
            pairs = [(c, c) if isinstance(c, str) else tuple(c) for c in cols]
            al = [p[1] for p in pairs]
            enc = (len(pairs), _lib.strs([p[0] for p in pairs]), _lib.strs(al), al)
            if len(_SELECT_ARGS) < 4096:
                _SELECT_ARGS[cols] = enc
        return self._new("capf_table_select", self._h, enc[0], enc[1], enc[2], cols=enc[3])

    def filter(self, expr, header=None, params=None):
        prog = _program(expr, header, self, params)
        e, keep = _lib._keepalive_expr(prog)
        return self._new("capf_table_filter", self._h, byref(e), cols=self._cols)

    def drop(self, *cols):
        gone = set(cols)
        keep = None if self._cols is None else [c for c in self._cols if c not in gone]
        return self._new("capf_table_drop", self._h, len(cols), _lib.strs(list(cols)), cols=keep)

    def join(self, other, join_type, *join_cols):
        jt = JOIN_TYPES[join_type] if isinstance(join_type, str) else int(join_type)
        ls = [l for l, _ in join_cols]
        rs = [r for _, r in join_cols]
        out = None
        if self._cols is not None and other._cols is not None:
            out = self._cols + other._cols  # capf_table_join: left columns, then right
        return self._new("capf_table_join", self._h, other._h, jt, len(join_cols), _lib.strs(ls), _lib.strs(rs),
                         cols=out)

    def unionAll(self, other):
        return self._new("capf_table_union_all", self._h, other._h)

    def orderBy(self, *sort_items, header=None, params=None):
        progs = [_program(e, header, self, params) for e, _ in sort_items]
        arr, keep = _lib.expr_array(progs)
        desc = (c_int32 * max(len(sort_items), 1))(*[1 if o in ("desc", "Descending", True) else 0
                                                     for _, o in sort_items])
        return self._new("capf_table_order_by", self._h, len(progs), arr, desc)

    def skip(self, n):
        return self._new("capf_table_skip", self._h, int(n))

    def limit(self, n):
        return self._new("capf_table_limit", self._h, int(n))

    def distinct(self, *cols):
        if not cols:
            return self._new("capf_table_distinct", self._h)
        return self._new("capf_table_distinct_cols", self._h, len(cols), _lib.strs(list(cols)))

    def group(self, by, aggregations, header=None, params=None):
        """by: iterable of Var (grouping uses every column they own,
        FlinkTable.scala:129-135); aggregations: {column: Aggregator}."""
        cols = []
        for v in by:
            for e in header.owned_by(v):
                c = header.column(e)
                if c in self.physicalColumns and c not in cols:
                    cols.append(c)
        names = list(aggregations)
        kinds, progs, dist, pars = [], [], [], []
        for name in names:
            agg = aggregations[name]
            if not isinstance(agg, Aggregator):
                raise _lib.IllegalArgumentException(f"{agg} is not an aggregator")
            if agg.kind < 0:  # FlinkSQLExprMapper.scala:289-290
                raise _lib.NotImplementedException(
                    f"No support for converting Cypher expression {agg} to a GPU expression")
            kinds.append(agg.kind)
            dist.append(1 if getattr(agg, "distinct", False) else 0)
            pars.append(percentile_value(agg.percentile, params) if hasattr(agg, "percentile") else 0.0)
            progs.append(None if agg.kind == AGG_COUNT_STAR else _program(agg.expr, header, self, params))
        arr, keep = _lib.expr_array(progs)
        k = len(names)
        return self._new("capf_table_group_ex", self._h, len(cols), _lib.strs(cols), k,
                         (c_int32 * max(k, 1))(*kinds), arr, (c_int32 * max(k, 1))(*dist),
                         (c_double * max(k, 1))(*pars), _lib.strs(names))

    def _explode(self, e, col, header, params):
        """UNWIND: withColumns(Explode(list) AS col) — a literal / parameter
        list (capf_table_explode_values) or a LIST column (capf_table_explode_list)."""
        ev = explode_values(e.expr, params)
        if ev is not None:
            t, vals = ev
            n = len(vals)
            valid = None
            if any(v is None for v in vals):
                valid = np.array([v is not None for v in vals], dtype=np.uint8)
            if t == T_NULL:
                data = None
            elif t == T_STRING:
                data = np.array([self.session.intern(v) if v is not None else 0 for v in vals], dtype=np.int64)
            else:
                data = np.array([v if v is not None else 0 for v in vals], dtype=_NP_DTYPE[t])
            return self._new("capf_table_explode_values", self._h, col.encode(), int(t), n,
                             data.ctypes.data if data is not None and n else None,
                             valid.ctypes.data if valid is not None and n else None)
        src = header.get(e.expr) if header is not None else None
        if src is None or src not in self.physicalColumns:
            if isinstance(e.expr, Var) or type(e.expr).__name__ == "NullLit":  # UNWIND null: no rows
                return self._new("capf_table_explode_values", self._h, col.encode(), int(T_NULL), 0, None, None)
            raise _lib.NotImplementedException(f"UNWIND of {e.expr}")
        return self._new("capf_table_explode_list", self._h, src.encode(), col.encode())

    def add_list(self, name, values, valid=None):
        """This table plus LIST column `name` from host lists (None = a NULL
        list): capf_table_add_list.  INTEGER and FLOAT elements widen to FLOAT
        together; NULL elements are NotImplemented (LIST columns hold none)."""
        kinds = set()
        for xs in values:
            for x in xs or ():
                if x is None:
                    raise _lib.NotImplementedException("NULL elements in a LIST property")
                kinds.add(T_BOOL if isinstance(x, bool) else T_INT if isinstance(x, int) else
                          T_FLOAT if isinstance(x, float) else T_STRING if isinstance(x, str) else None)
        if None in kinds or len(kinds - {T_INT, T_FLOAT}) > (0 if kinds & {T_INT, T_FLOAT} else 1):
            raise _lib.NotImplementedException(f"LIST property '{name}' of mixed or nested elements")
        et = T_FLOAT if T_FLOAT in kinds else kinds.pop() if kinds else T_INT
        offs = np.zeros(len(values) + 1, dtype=np.int64)
        flat = []
        for i, xs in enumerate(values):
            flat += list(xs or ())
            offs[i + 1] = len(flat)
        if et == T_STRING:
            data = np.array([self.session.intern(x) for x in flat], dtype=np.int64)
        else:
            data = np.array(flat, dtype=_NP_DTYPE[et]) if flat else np.zeros(1, dtype=_NP_DTYPE[et])
        ok = np.array([xs is not None for xs in values], dtype=np.uint8) if valid is None else \
            np.ascontiguousarray(np.asarray(valid, dtype=np.uint8))
        return self._new("capf_table_add_list", self._h, name.encode(), int(et), offs.ctypes.data,
                         data.ctypes.data, ok.ctypes.data if len(values) else None)

    def _value_map(self, kind, exprs, header, params):
        """Program name of a session value map (CAPF_OP_VALUE_MAP) giving the STRING
        of each distinct value (toString) or value pair (concatenation) the
        operand expressions take over this table: the operands are evaluated
        and their distinct rows downloaded, the strings built with the JVM's
        casts (Long.toString / Double.toString) and interned."""
        import struct
        from .expr import cypher_to_string
        names = [f"\x02vm{i}" for i in range(len(exprs))]
        t = self.withColumns(*zip(exprs, names), header=header, params=params).select(*names)
        types = [t.capf_type(c) for c in names]
        t = t.distinct(*names)
        if t.size > VALUE_MAP_MAX:  # every distinct value becomes a host string and a dictionary entry
            raise _lib.NotImplementedException(
                f"a new string per value over {t.size} distinct values (more than {VALUE_MAP_MAX})")
        cols = [t.column_values(c) for c in names]
        rows = sorted({r for r in zip(*cols) if not any(v is None for v in r)})
        gather = getattr(self.session, "value_map_gather", None)
        if gather is not None:
            # distributed (dist_table.DistSession): every rank interns the union
            # of all ranks' values in one order, so the string dictionaries stay
            # equal and STRING codes can cross ranks
            rows = sorted({r for part in gather(rows) for r in part})

        def key(v, ty):
            if ty == T_FLOAT:
                return struct.unpack("<q", struct.pack("<d", float(v)))[0]
            if ty == T_STRING:
                return self.session.intern(v)
            return int(v)

        entries = []
        for vals in rows:
            if isinstance(kind, tuple) and kind[0] == "regex":  # s =~ pattern, then cast to BOOLEAN
                import re
                txt = "true" if re.fullmatch(kind[1], vals[0]) else "false"
            elif isinstance(kind, tuple) and kind[0] == "fn":  # a string function (expr.string_fn)
                from .expr import string_fn
                txt = string_fn(kind[1], vals[0])
                if txt is None:  # (no entry: the lookup misses, NULL)
                    continue
            else:
                txt = "".join(cypher_to_string(float(v) if ty == T_FLOAT else v) for v, ty in zip(vals, types))
            entries.append((tuple(key(v, ty) for v, ty in zip(vals, types)), self.session.intern(txt)))
        entries.sort()
        n = len(entries)
        k1 = (c_int64 * max(n, 1))(*[e[0][0] for e in entries])
        k2 = (c_int64 * max(n, 1))(*[e[0][1] for e in entries]) if len(exprs) > 1 else None
        cd = (c_int64 * max(n, 1))(*[e[1] for e in entries])
        mid = c_int32()
        _lib.call("capf_session_value_map", self.session._h, k1, k2, cd, n, byref(mid))
        return "\x01vmap:%d" % mid.value

    def withColumns(self, *columns, header=None, params=None):
        lit = [(e, c) for e, c in columns if _list_items(e, params) is not None]
        if lit:  # [x, y, ...] / $list: LIST columns of per-row elements (capf_table_list_columns)
            plain = [(e, c) for e, c in columns if (e, c) not in lit]
            t = self.withColumns(*plain, header=header, params=params) if plain else self
            keep = list(t.physicalColumns)
            for i, (e, c) in enumerate(lit):
                items = _list_items(e, params)
                tmp = [f"\x03le{i}.{j}" for j in range(len(items))]
                if items:
                    t = t.withColumns(*zip(items, tmp), header=header, params=params)
                t = t._new("capf_table_list_columns", t._h, len(tmp), _lib.strs(tmp), c.encode())
                keep.append(c)
            return t.select(*keep)
        is_list = lambda e: type(e).__name__ in ("Labels", "Keys") and type(e.expr).__name__ != "NullLit"  # noqa: E731
        lists = [(e, c) for e, c in columns if is_list(e)]
        if lists:  # labels(n) / keys(n): LIST columns built by capf_table_name_list
            from .expr import name_list_columns
            plain = [(e, c) for e, c in columns if not is_list(e)]
            t = self.withColumns(*plain, header=header, params=params) if plain else self
            for e, c in lists:
                if not isinstance(e.expr, Var):
                    raise _lib.NotImplementedException(f"{e} of a non-variable")
                cols, kinds, names = name_list_columns(e, header, set(t.physicalColumns))
                n = len(cols)
                ka = (c_int32 * max(n, 1))(*kinds)
                ca = (c_int64 * max(n, 1))(*[self.session.intern(x) for x in names])
                t = t._new("capf_table_name_list", t._h, n, _lib.strs(cols), ka, ca, c.encode())
            return t
        if any(isinstance(e, Explode) for e, _ in columns):
            t = self
            plain = [(e, c) for e, c in columns if not isinstance(e, Explode)]
            if plain:
                t = t.withColumns(*plain, header=header, params=params)
            for e, c in columns:
                if isinstance(e, Explode):
                    t = t._explode(e, c, header, params)
            return t
        progs = [_program(e, header, self, params) for e, _ in columns]
        arr, keep = _lib.expr_array(progs)
        return self._new("capf_table_with_columns", self._h, len(columns), arr,
                         _lib.strs([c for _, c in columns]))

    def show(self, rows=20):
        _lib.call("capf_table_show", self._h, int(rows))

    # ---------------------------------------------------------- multi-GPU helpers
    def node_partition(self, key_col, node_base, n_nodes, parts, part):
        """Rows whose key_col node is owned by `part` of `parts` (Multi-GPU)."""
        return self._new("capf_table_node_partition", self._h, key_col.encode(), int(node_base),
                         int(n_nodes), int(parts), int(part))

    def node_partition_diag(self, src_col, dst_col, node_base, n_nodes, parts, part):
        """The out-copy of `part` in 2-D order: rows whose source it owns, those
        whose target it owns too first.  Returns (table, n_diag)."""
        h, nd = c_void_p(), c_int64()
        _lib.call("capf_table_node_partition_diag", self._h, src_col.encode(), dst_col.encode(), int(node_base),
                  int(n_nodes), int(parts), int(part), byref(h), byref(nd))
        return GpuTable(self.session, h), nd.value

    def chain2_local_hists(self, src_col, dst_col, node_base, n_nodes, d_in, d_out):
        loops = c_int64()
        _lib.call("capf_chain2_local_hists", self.session._h, self._h, src_col.encode(), dst_col.encode(),
                  int(node_base), int(n_nodes), c_void_p(d_in), c_void_p(d_out), byref(loops))
        return loops.value


def _list_items(e, params):
    """The element expressions of a list-valued projection item — a list
    literal, or a parameter holding a list (FlinkSQLExprMapper.scala:71, 75) —
    else None."""
    from .expr import ListLit, Param, literal_expr
    if isinstance(e, ListLit):
        return list(e.items)
    if isinstance(e, Param):
        v = (params or {}).get(e.pname)
        if isinstance(v, (list, tuple)):
            return [literal_expr(x) for x in v]
    return None


def compact_as(table, compact):
    """Ingest-time encoding choice of the graph builders: False = plain int64,
    True / 4 = FOR32 where the range fits, 3 = FOR24 where it fits (else FOR32)."""
    if not compact:
        return table
    return table.compact(3 if compact == 3 else 4)


def chain2_sharded_count_async(session, in_copy, out_copy, node_base, n_nodes, parts, part,
                               d_partial, src="source", dst="target"):
    """Enqueue this rank's 2-hop partial (int64 at device address d_partial).
    An out-copy in 2-D order (node_partition_diag) carries `n_diag`: only its
    first n_diag rows are tested for self-loops."""
    hot = list(getattr(out_copy, "hot_ids", ()))[:2]
    _lib.call("capf_chain2_sharded_count_diag", session._h, in_copy._h, dst.encode(), out_copy._h,
              src.encode(), dst.encode(), int(getattr(out_copy, "n_diag", -1)), len(hot),
              (c_int64 * max(len(hot), 1))(*hot), int(node_base), int(n_nodes), int(parts), int(part),
              c_void_p(d_partial))


def triangle_count_part_async(session, rels, node_base, n_nodes, parts, part, d_count,
                              src="source", dst="target"):
    """Enqueue part `part` of `parts` of the directed triangle count (int64 at
    device address d_count); the parts sum to the count."""
    _lib.call("capf_triangle_count_part", session._h, rels._h, src.encode(), dst.encode(), int(node_base),
              int(n_nodes), int(parts), int(part), c_void_p(d_count))


def chain2_hist_len(n_nodes):
    """Counters per histogram written by chain2_local_hists (2^k >= n_nodes)."""
    return int(_lib.load().capf_chain2_hist_len(int(n_nodes)))


def dot_u32(session, d_a, d_b, n):
    out = c_uint64()
    _lib.call("capf_dot_u32", session._h, c_void_p(d_a), c_void_p(d_b), int(n), byref(out))
    return out.value
