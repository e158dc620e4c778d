"""Test infrastructure: route the Python host's C-ABI calls through the JNI
adapter (integration/jni/capf_jni.cpp), executed against the in-process fake
JVM of tests/jni_fake/ (VERDICT r5 item 8).

`JniRoute.install()` replaces the entries of `capf_amd._lib` that
`table.GpuSession` / `table.GpuTable` call (`_lib.call(name, ...)`) by
adapters that do what `org.opencypher.gpu.Native` + `GpuTable.scala` do on the
JVM: build the Java arguments (String / String[] / int[] / long[] / double[] /
boolean[], direct ByteBuffers over host memory, `org.opencypher.gpu.Program`
objects for expressions), call the adapter's
`Java_org_opencypher_gpu_Native_00024_<method>` symbol, and take back its
result (a jlong handle, a String[], values written into long[] / double[]
out-arrays) or its pending exception — `CapfNativeException(kind, message)`
rethrown as the okapi exception of that kind (Native.scala), or the adapter's
own `IllegalArgumentException` for argument arrays that disagree.  The whole
unchanged planner → GpuTable stack then runs through the JNI marshalling.
"""
import ctypes
import os
import subprocess
from ctypes import POINTER, byref, c_char_p, c_double, c_int32, c_int64, c_uint8, c_void_p

from capf_amd import _lib

HERE = os.path.dirname(os.path.abspath(__file__))
FAKE_DIR = os.path.join(HERE, "jni_fake")
FAKE_LIB = os.path.join(FAKE_DIR, "libcapf_jni_fake.so")
PREFIX = "Java_org_opencypher_gpu_Native_00024_"
BIG = 1 << 62  # capacity of a direct buffer over memory the C-ABI sizes itself


def build():
    """make the fake-JVM adapter library (g++; seconds).  __graft_entry__.build()
    builds it on the CPU; where make cannot run (a snapshot whose mtimes make
    it look stale, a read-only tree) the prebuilt library is used as is."""
    r = subprocess.run(["make", "-s"], cwd=FAKE_DIR, capture_output=True, text=True)
    if r.returncode != 0 and not os.path.exists(FAKE_LIB):
        raise RuntimeError(f"building {FAKE_LIB} failed:\n{r.stderr}")
    return FAKE_LIB


class JavaException(RuntimeError):
    """A Java exception other than the mapped ones (e.g. ArrayIndexOutOfBounds)."""


class JniRoute:
    def __init__(self, path=FAKE_LIB):
        _lib.load()  # the adapter links the same libcapf_gpu.so instance
        self.lib = ctypes.CDLL(path)
        fj = self.lib
        for name, res, args in [
                ("fj_env", c_void_p, []), ("fj_reset", None, []), ("fj_calls", c_int64, []),
                ("fj_string", c_void_p, [c_char_p]), ("fj_string_value", c_char_p, [c_void_p]),
                ("fj_ints", c_void_p, [c_void_p, c_int64]), ("fj_longs", c_void_p, [c_void_p, c_int64]),
                ("fj_doubles", c_void_p, [c_void_p, c_int64]), ("fj_bools", c_void_p, [c_void_p, c_int64]),
                ("fj_bytes", c_void_p, [c_void_p, c_int64]),
                ("fj_objects", c_void_p, [POINTER(c_void_p), c_int64, c_char_p]),
                ("fj_direct", c_void_p, [c_void_p, c_int64]), ("fj_heap_buffer", c_void_p, []),
                ("fj_program", c_void_p, [c_void_p, c_void_p, c_void_p, c_void_p]),
                ("fj_length", c_int64, [c_void_p]), ("fj_element", c_void_p, [c_void_p, c_int64]),
                ("fj_get_longs", None, [c_void_p, POINTER(c_int64)]),
                ("fj_get_doubles", None, [c_void_p, POINTER(c_double)]),
                ("fj_take_exception", c_int32, [POINTER(c_char_p), POINTER(c_char_p), POINTER(c_int32)])]:
            f = getattr(fj, name)
            f.restype, f.argtypes = res, args
        self.env = fj.fj_env()
        self._saved = None
        self._keep = []  # C strings handed back as const char* (profile names)
        self.jni_calls = 0  # Native methods invoked through the adapter

    # ------------------------------------------------------------ Java values
    def jstr(self, b):
        if b is None:
            return None
        if isinstance(b, str):
            b = b.encode()
        return self.lib.fj_string(b)

    def jstrs(self, arr, n):
        items = (c_void_p * max(n, 1))(*[self.jstr(arr[i]) for i in range(n)])
        return self.lib.fj_objects(items, n, b"java/lang/String")

    def jints(self, arr, n):
        return self.lib.fj_ints(ctypes.cast(arr, c_void_p) if n else None, n)

    def jlongs(self, arr, n):
        return self.lib.fj_longs(ctypes.cast(arr, c_void_p) if n else None, n)

    def jdoubles(self, arr, n):
        return self.lib.fj_doubles(ctypes.cast(arr, c_void_p) if n else None, n)

    def jbools(self, arr, n):
        b = (c_uint8 * max(n, 1))(*[1 if arr[i] else 0 for i in range(n)])
        return self.lib.fj_bools(b, n)

    def direct(self, ptr, cap=BIG):
        if ptr is None:
            return None
        p = ptr.value if isinstance(ptr, c_void_p) else int(ptr)
        return self.lib.fj_direct(p, cap) if p else None

    def program(self, e):
        n, k = e.n, e.n_names
        return self.lib.fj_program(self.jints(e.ops, n), self.jlongs(e.iargs, n),
                                   self.jdoubles(e.fargs, n) if e.fargs else self.lib.fj_doubles(None, n),
                                   self.jstrs(e.names, k))

    def programs(self, arr, n):
        items = (c_void_p * max(n, 1))(*[self.program(arr[i]) for i in range(n)])
        return self.lib.fj_objects(items, n, b"org/opencypher/gpu/Program")

    def objects(self, ptrs, n):
        items = (c_void_p * max(n, 1))(*[self.direct(ptrs[i]) for i in range(n)])
        return self.lib.fj_objects(items, n, b"java/nio/ByteBuffer")

    # ------------------------------------------------------------ calls
    def native(self, method, restype, *args):
        """Invoke Native.<method> through the adapter: (JNIEnv*, self, args…);
        a pending Java exception is rethrown as Native.scala does."""
        f = getattr(self.lib, PREFIX + method)
        f.restype = restype
        conv = []
        for a in args:
            if isinstance(a, tuple):  # (ctypes type, value)
                conv.append(a[0](a[1]))
            else:
                conv.append(c_void_p(a) if a is not None else c_void_p())
        self.jni_calls += 1
        r = f(c_void_p(self.env), c_void_p(), *conv)
        self.raise_pending()
        return r

    def raise_pending(self):
        cls, msg, code = c_char_p(), c_char_p(), c_int32()
        if self.lib.fj_take_exception(byref(cls), byref(msg), byref(code)):
            c, m = cls.value.decode(), msg.value.decode("utf-8", "replace")
            self.lib.fj_reset()
            if c == "org/opencypher/gpu/CapfNativeException":  # Native.scala: rethrow by kind
                raise _lib._ERRORS.get(code.value, _lib.CypherException)(m)
            if c == "java/lang/IllegalArgumentException":
                raise _lib.IllegalArgumentException(m)
            raise JavaException(f"{c}: {m}")

    def done(self):
        self.lib.fj_reset()
        return 0

    # ------------------------------------------------------------ adapters
    def adapters(self):
        L, I, D, Z = c_int64, c_int32, c_double, c_uint8
        h = lambda p: (L, p.value if isinstance(p, c_void_p) else (p or 0))  # noqa: E731
        out = lambda ref, v: setattr(ref._obj, "value", v)  # noqa: E731
        nat = self.native
        A = {}

        def new_table(method, jargs):
            def f(*a):
                r = nat(method, L, *jargs(*a[:-1]))
                out(a[-1], r)
                return self.done()
            return f

        def session_create(device, stream, ref):
            out(ref, nat("sessionCreate", L, (I, device), (L, stream.value if isinstance(stream, c_void_p)
                                                           else (stream or 0))))
            return self.done()
        A["capf_session_create"] = session_create
        A["capf_session_sync"] = lambda s: (nat("sessionSync", None, h(s)), self.done())[1]
        A["capf_session_set_profiling"] = lambda s, on: (nat("sessionSetProfiling", None, h(s), (Z, on)),
                                                         self.done())[1]
        A["capf_session_reset_profile"] = lambda s: (nat("sessionResetProfile", None, h(s)), self.done())[1]

        def profile_count(s, ref):
            out(ref, nat("sessionProfileCount", I, h(s)))
            return self.done()
        A["capf_session_profile_count"] = profile_count

        def profile_entry(s, i, name, launches, ms, by):
            lo, mb = self.lib.fj_longs(None, 1), self.lib.fj_doubles(None, 2)
            js = nat("sessionProfileEntry", c_void_p, h(s), (I, i), lo, mb)
            buf = ctypes.create_string_buffer(self.lib.fj_string_value(js))
            self._keep.append(buf)
            out(name, ctypes.cast(buf, c_char_p).value)
            lv, dv = (c_int64 * 1)(), (c_double * 2)()
            self.lib.fj_get_longs(lo, lv)
            self.lib.fj_get_doubles(mb, dv)
            out(launches, lv[0])
            out(ms, dv[0])
            out(by, dv[1])
            return self.done()
        A["capf_session_profile_entry"] = profile_entry

        def intern(s, b, ref):
            out(ref, nat("stringIntern", L, h(s), self.jstr(b)))
            return self.done()
        A["capf_string_intern"] = intern

        def lookup(s, code, ref):
            js = nat("stringLookup", c_void_p, h(s), (L, code))
            buf = ctypes.create_string_buffer(self.lib.fj_string_value(js))
            self._keep.append(buf)
            out(ref, buf.value)
            return self.done()
        A["capf_string_lookup"] = lookup

        def digest(s, cnt, dig):
            o = self.lib.fj_longs(None, 2)
            nat("stringDigest", None, h(s), o)
            v = (c_int64 * 2)()
            self.lib.fj_get_longs(o, v)
            out(cnt, v[0])
            out(dig, v[1] & ((1 << 64) - 1))
            return self.done()
        A["capf_string_digest"] = digest

        A["capf_table_from_host"] = new_table(
            "tableFromHost", lambda s, k, names, types, datas, valids, n:
            (h(s), self.jstrs(names, k), self.jints(types, k), self.objects(datas, k), self.objects(valids, k),
             (L, n)))
        A["capf_table_unit"] = new_table("tableUnit", lambda s: (h(s),))
        A["capf_table_empty"] = new_table("tableEmpty", lambda s, k, names, types:
                                          (h(s), self.jstrs(names, k), self.jints(types, k)))

        def columns(t, p, nb, n):
            arr = nat("tableColumns", c_void_p, h(t))
            k = self.lib.fj_length(arr)
            names = [self.lib.fj_string_value(self.lib.fj_element(arr, i)) for i in range(k)]
            raw = b"".join(x + b"\0" for x in names)
            buf = ctypes.create_string_buffer(raw, max(len(raw), 1))
            self._keep.append(buf)
            out(p, ctypes.addressof(buf))
            out(nb, len(raw))
            out(n, k)
            return self.done()
        A["capf_table_columns"] = columns

        def column_type(t, col, ref):
            out(ref, nat("tableColumnType", I, h(t), self.jstr(col)))
            return self.done()
        A["capf_table_column_type"] = column_type

        def size(t, ref):
            out(ref, nat("tableSize", L, h(t)))
            return self.done()
        A["capf_table_size"] = size
        A["capf_table_materialize"] = lambda t: (nat("tableMaterialize", None, h(t)), self.done())[1]
        A["capf_table_count_async"] = lambda t, d: (nat("tableCountAsync", None, h(t), h(d)), self.done())[1]
        A["capf_table_download"] = lambda t, col, vals, valid: (
            nat("tableDownload", None, h(t), self.jstr(col), self.direct(vals), self.direct(valid)), self.done())[1]

        def list_info(t, col, et, nv):
            if nv is None:  # the type alone (a null nValuesOut)
                out(et, nat("tableListInfo", I, h(t), self.jstr(col), None))
                return self.done()
            o = self.lib.fj_longs(None, 1)
            out(et, nat("tableListInfo", I, h(t), self.jstr(col), o))
            v = (c_int64 * 1)()
            self.lib.fj_get_longs(o, v)
            out(nv, v[0])
            return self.done()
        A["capf_table_list_info"] = list_info
        A["capf_table_download_list"] = lambda t, col, offs, vals, valid: (
            nat("tableDownloadList", None, h(t), self.jstr(col), self.direct(offs), self.direct(vals),
                self.direct(valid)), self.done())[1]

        def encoding(t, col, e, b):
            o = self.lib.fj_longs(None, 1)
            out(e, nat("tableColumnEncoding", I, h(t), self.jstr(col), o))
            v = (c_int64 * 1)()
            self.lib.fj_get_longs(o, v)
            out(b, v[0])
            return self.done()
        A["capf_table_column_encoding"] = encoding
        A["capf_table_cache"] = new_table("tableCache", lambda t: (h(t),))
        A["capf_table_compact"] = new_table("tableCompact", lambda t: (h(t),))
        A["capf_table_compact_width"] = new_table("tableCompactWidth", lambda t, w: (h(t), (I, w)))
        A["capf_table_select"] = new_table("tableSelect", lambda t, k, cols, als:
                                           (h(t), self.jstrs(cols, k), self.jstrs(als, k)))
        A["capf_table_filter"] = new_table("tableFilter", lambda t, e: (h(t), self.program(e._obj)))
        A["capf_table_drop"] = new_table("tableDrop", lambda t, k, cols: (h(t), self.jstrs(cols, k)))
        A["capf_table_join"] = new_table("tableJoin", lambda l, r, jt, k, lc, rc:
                                         (h(l), h(r), (I, jt), self.jstrs(lc, k), self.jstrs(rc, k)))
        A["capf_table_union_all"] = new_table("tableUnionAll", lambda l, r: (h(l), h(r)))
        A["capf_table_order_by"] = new_table("tableOrderBy", lambda t, k, progs, desc:
                                             (h(t), self.programs(progs, k), self.jbools(desc, k)))
        A["capf_table_skip"] = new_table("tableSkip", lambda t, n: (h(t), (L, n)))
        A["capf_table_limit"] = new_table("tableLimit", lambda t, n: (h(t), (L, n)))
        A["capf_table_distinct"] = new_table("tableDistinct", lambda t: (h(t),))
        A["capf_table_distinct_cols"] = new_table("tableDistinctCols", lambda t, k, cols:
                                                  (h(t), self.jstrs(cols, k)))
        A["capf_table_group_ex"] = new_table(
            "tableGroupEx", lambda t, nb, by, k, kinds, progs, dist, pars, names:
            (h(t), self.jstrs(by, nb), self.jints(kinds, k), self.programs(progs, k), self.jbools(dist, k),
             self.jdoubles(pars, k), self.jstrs(names, k)))
        A["capf_table_with_columns"] = new_table("tableWithColumns", lambda t, k, progs, names:
                                                 (h(t), self.programs(progs, k), self.jstrs(names, k)))
        A["capf_table_explode_values"] = new_table(
            "tableExplodeValues", lambda t, col, ty, n, vals, valid:
            (h(t), self.jstr(col), (I, ty), (L, n), self.direct(vals), self.direct(valid)))
        A["capf_table_explode_list"] = new_table("tableExplodeList", lambda t, src, col:
                                                 (h(t), self.jstr(src), self.jstr(col)))
        A["capf_table_name_list"] = new_table("tableNameList", lambda t, k, cols, kinds, codes, col:
                                              (h(t), self.jstrs(cols, k), self.jints(kinds, k),
                                               self.jlongs(codes, k), self.jstr(col)))
        A["capf_table_list_columns"] = new_table("tableListColumns", lambda t, k, cols, col:
                                                 (h(t), self.jstrs(cols, k), self.jstr(col)))
        A["capf_table_add_list"] = new_table(
            "tableAddList", lambda t, col, et, offs, vals, valid:
            (h(t), self.jstr(col), (I, et), self.direct(offs), self.direct(vals), self.direct(valid)))
        A["capf_table_show"] = lambda t, rows: (nat("tableShow", None, h(t), (I, rows)), self.done())[1]
        A["capf_rmat_rel_table"] = new_table(
            "rmatRelTable", lambda s, sc, seed, ta, tab, tabc, first, count, base, ic, sc_, dc:
            (h(s), (I, sc), (L, c_int64(seed).value), (I, c_int32(ta).value), (I, c_int32(tab).value),
             (I, c_int32(tabc).value), (L, first), (L, count), (L, base), self.jstr(ic), self.jstr(sc_),
             self.jstr(dc)))
        A["capf_range_node_table"] = new_table(
            "rangeNodeTable", lambda s, base, n, seed, ic, lc:
            (h(s), (L, base), (L, n), (L, c_int64(seed).value), self.jstr(ic), self.jstr(lc)))
        A["capf_var_length_reach"] = new_table(
            "varLengthReach", lambda s, rels, a, b, src, si, tgt, ti, lo, up, os_, or_:
            (h(s), h(rels), self.jstr(a), self.jstr(b), h(src), self.jstr(si), h(tgt), self.jstr(ti), (I, lo),
             (I, up), self.jstr(os_), self.jstr(or_)))

        def id_of(method, jargs):
            def f(*a):
                out(a[-1], nat(method, I, *jargs(*a[:-1])))
                return self.done()
            return f
        A["capf_session_literal_set"] = id_of("sessionLiteralSet", lambda s, arr, n: (h(s), self.jlongs(arr, n)))
        A["capf_session_code_map"] = id_of("sessionCodeMap", lambda s, arr, n: (h(s), self.jlongs(arr, n)))
        A["capf_session_code_map_extend"] = id_of("sessionCodeMapExtend", lambda s, mid, arr, n:
                                                  (h(s), (I, mid), self.jlongs(arr, n)))
        A["capf_session_value_map"] = id_of(
            "sessionValueMap", lambda s, k1, k2, cd, n:
            (h(s), self.jlongs(k1, n), self.jlongs(k2, n) if k2 is not None else None, self.jlongs(cd, n)))
        return A

    def install(self):
        """Route every adapted entry point through the JNI adapter; returns
        the names routed.  `uninstall()` restores the direct ctypes path."""
        self._saved = dict(_lib._FNS)
        routed = self.adapters()
        _lib._FNS.update(routed)
        return sorted(routed)

    def uninstall(self):
        if self._saved is not None:
            _lib._FNS.clear()
            _lib._FNS.update(self._saved)
            self._saved = None
