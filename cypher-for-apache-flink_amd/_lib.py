"""ctypes binding of libcapf_gpu.so (the C-ABI declared in include/capf_gpu.h).

The product path has exactly one implementation: the HIP library.  If the
shared object is missing or fails to load, every entry point raises — there is
no CPU fallback (oracle/ is test infrastructure and is never imported here).

Error mapping mirrors the okapi exception hierarchy the Scala shim would
rethrow (okapi-api/src/main/scala/org/opencypher/okapi/impl/exception/
InternalException.scala:36-65).
"""
import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int32, c_int64, c_uint8, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
# CAPF_LIB_AB (A/B timing of two builds only): an alternative in-tree build
# of the same library, e.g. ab/libcapf_gpu_a.so; never set in production.
LIB_PATH = os.path.join(_HERE, os.environ.get("CAPF_LIB_AB", "libcapf_gpu.so"))


class CypherException(RuntimeError):
    """Base of the okapi exceptions raised through the C-ABI."""


class IllegalArgumentException(CypherException):
    pass


class NotImplementedException(CypherException):
    pass


class SchemaException(CypherException):
    """okapi's SchemaException: a property graph schema whose property types
    cannot share one column (CAPFSchema.asCapf, CAPFSchema.scala:42-72)."""


class IllegalStateException(CypherException):
    pass


class HipRuntimeException(CypherException):
    pass


class DeviceOutOfMemoryException(HipRuntimeException):
    pass


_ERRORS = {
    -1: IllegalArgumentException,
    -2: NotImplementedException,
    -3: IllegalStateException,
    -4: HipRuntimeException,
    -5: DeviceOutOfMemoryException,
}


class CapfExpr(ctypes.Structure):
    _fields_ = [
        ("n", c_int32),
        ("ops", POINTER(c_int32)),
        ("iargs", POINTER(c_int64)),
        ("fargs", POINTER(c_double)),
        ("n_names", c_int32),
        ("names", POINTER(c_char_p)),
    ]


_S = c_void_p  # capf_session*
_T = c_void_p  # capf_table*
_PT = POINTER(c_void_p)
_STRS = POINTER(c_char_p)

# name -> (restype, argtypes)
_SIGS = {
    "capf_last_error": (c_char_p, []),
    "capf_last_error_kind": (c_int32, []),
    "capf_abi_version": (c_int32, []),
    "capf_session_create": (c_int32, [c_int32, c_void_p, _PT]),
    "capf_session_destroy": (c_int32, [_S]),
    "capf_session_sync": (c_int32, [_S]),
    "capf_session_set_profiling": (c_int32, [_S, c_int32]),
    "capf_session_reset_profile": (c_int32, [_S]),
    "capf_session_profile_count": (c_int32, [_S, POINTER(c_int32)]),
    "capf_session_profile_entry": (c_int32, [_S, c_int32, POINTER(c_char_p), POINTER(c_int64),
                                             POINTER(c_double), POINTER(c_double)]),
    "capf_session_last_plan": (c_char_p, [_S]),
    "capf_string_intern": (c_int32, [_S, c_char_p, POINTER(c_int64)]),
    "capf_string_lookup": (c_int32, [_S, c_int64, POINTER(c_char_p)]),
    "capf_string_digest": (c_int32, [_S, POINTER(c_int64), POINTER(c_uint64)]),
    "capf_table_from_host": (c_int32, [_S, c_int32, _STRS, POINTER(c_int32), POINTER(c_void_p),
                                       POINTER(c_void_p), c_int64, _PT]),
    "capf_table_from_device": (c_int32, [_S, c_int32, _STRS, POINTER(c_int32), POINTER(c_void_p),
                                         POINTER(c_void_p), c_int64, c_int32, _PT]),
    "capf_table_unit": (c_int32, [_S, _PT]),
    "capf_table_empty": (c_int32, [_S, c_int32, _STRS, POINTER(c_int32), _PT]),
    "capf_table_retain": (c_int32, [_T]),
    "capf_table_release": (c_int32, [_T]),
    "capf_table_num_columns": (c_int32, [_T, POINTER(c_int32)]),
    "capf_table_column_name": (c_int32, [_T, c_int32, POINTER(c_char_p)]),
    "capf_table_columns": (c_int32, [_T, POINTER(c_void_p), POINTER(c_int64), POINTER(c_int32)]),
    "capf_table_column_type": (c_int32, [_T, c_char_p, POINTER(c_int32)]),
    "capf_table_size": (c_int32, [_T, POINTER(c_int64)]),
    "capf_table_count_async": (c_int32, [_T, c_void_p]),
    "capf_table_download": (c_int32, [_T, c_char_p, c_void_p, c_void_p]),
    "capf_table_list_info": (c_int32, [_T, c_char_p, POINTER(c_int32), POINTER(c_int64)]),
    "capf_table_download_list": (c_int32, [_T, c_char_p, c_void_p, c_void_p, c_void_p]),
    "capf_table_device_column": (c_int32, [_T, c_char_p, POINTER(c_void_p), POINTER(c_void_p),
                                           POINTER(c_int64)]),
    "capf_table_cache": (c_int32, [_T, _PT]),
    "capf_table_compact": (c_int32, [_T, _PT]),
    "capf_table_compact_width": (c_int32, [_T, c_int32, _PT]),
    "capf_table_materialize": (c_int32, [_T]),
    "capf_table_column_encoding": (c_int32, [_T, c_char_p, POINTER(c_int32), POINTER(c_int64)]),
    "capf_table_select": (c_int32, [_T, c_int32, _STRS, _STRS, _PT]),
    "capf_table_filter": (c_int32, [_T, POINTER(CapfExpr), _PT]),
    "capf_table_drop": (c_int32, [_T, c_int32, _STRS, _PT]),
    "capf_table_join": (c_int32, [_T, _T, c_int32, c_int32, _STRS, _STRS, _PT]),
    "capf_table_union_all": (c_int32, [_T, _T, _PT]),
    "capf_table_order_by": (c_int32, [_T, c_int32, POINTER(CapfExpr), POINTER(c_int32), _PT]),
    "capf_table_skip": (c_int32, [_T, c_int64, _PT]),
    "capf_table_limit": (c_int32, [_T, c_int64, _PT]),
    "capf_table_distinct": (c_int32, [_T, _PT]),
    "capf_table_distinct_cols": (c_int32, [_T, c_int32, _STRS, _PT]),
    "capf_table_group": (c_int32, [_T, c_int32, _STRS, c_int32, POINTER(c_int32), POINTER(CapfExpr),
                                   POINTER(c_int32), _STRS, _PT]),
    "capf_table_group_ex": (c_int32, [_T, c_int32, _STRS, c_int32, POINTER(c_int32), POINTER(CapfExpr),
                                      POINTER(c_int32), POINTER(c_double), _STRS, _PT]),
    "capf_table_with_columns": (c_int32, [_T, c_int32, POINTER(CapfExpr), _STRS, _PT]),
    "capf_table_explode_values": (c_int32, [_T, c_char_p, c_int32, c_int64, c_void_p, c_void_p, _PT]),
    "capf_table_explode_list": (c_int32, [_T, c_char_p, c_char_p, _PT]),
    "capf_table_show": (c_int32, [_T, c_int32]),
    "capf_rmat_rel_table": (c_int32, [_S, c_int32, c_uint64, c_uint32, c_uint32, c_uint32, c_int64,
                                      c_int64, c_int64, c_char_p, c_char_p, c_char_p, _PT]),
    "capf_range_node_table": (c_int32, [_S, c_int64, c_int64, c_uint64, c_char_p, c_char_p, _PT]),
    "capf_edge_list_parse": (c_int32, [_S, c_char_p, c_int64, c_char_p, c_char_p, c_char_p, c_char_p,
                                       c_char_p, _PT]),
    "capf_edge_list_read": (c_int32, [_S, c_char_p, c_char_p, c_char_p, c_char_p, c_char_p, c_char_p, _PT]),
    "capf_var_length_reach": (c_int32, [_S, _T, c_char_p, c_char_p, _T, c_char_p, _T, c_char_p, c_int32,
                                        c_int32, c_char_p, c_char_p, _PT]),
    "capf_chain2_hist_len": (c_int64, [c_int64]),
    "capf_chain2_local_hists": (c_int32, [_S, _T, c_char_p, c_char_p, c_int64, c_int64, c_void_p,
                                          c_void_p, POINTER(c_int64)]),
    "capf_table_node_partition_diag": (c_int32, [_T, c_char_p, c_char_p, c_int64, c_int64, c_int32, c_int32, _PT,
                                               POINTER(c_int64)]),
    "capf_chain2_sharded_count_diag": (c_int32, [_S, _T, c_char_p, _T, c_char_p, c_char_p, c_int64, c_int32,
                                               POINTER(c_int64), c_int64, c_int64, c_int32, c_int32, c_void_p]),
    "capf_table_node_partition": (c_int32, [_T, c_char_p, c_int64, c_int64, c_int32, c_int32, _PT]),
    "capf_chain2_sharded_count": (c_int32, [_S, _T, c_char_p, _T, c_char_p, c_char_p, c_int64, c_int64,
                                            c_int32, c_int32, c_void_p]),
    "capf_triangle_count_part": (c_int32, [_S, _T, c_char_p, c_char_p, c_int64, c_int64, c_int32, c_int32,
                                           c_void_p]),
    "capf_csv_parse_longs": (c_int32, [_S, c_char_p, c_int64, c_char_p, c_int32, _STRS, _PT]),
    "capf_csv_read_longs": (c_int32, [_S, c_char_p, c_char_p, c_int32, _STRS, _PT]),
    "capf_table_hash_route": (c_int32, [_T, c_int32, _STRS, c_int32, POINTER(c_int64), _PT]),
    "capf_table_download_device": (c_int32, [_T, c_char_p, c_void_p, c_void_p]),
    "capf_table_has_nulls": (c_int32, [_T, c_char_p, POINTER(c_int32)]),
    "capf_table_column_range": (c_int32, [_T, c_char_p, POINTER(c_int64), POINTER(c_int64), POINTER(c_int64)]),
    "capf_table_pack_rows": (c_int32, [_T, c_int32, POINTER(c_char_p), POINTER(c_int32), POINTER(c_int64),
                                       POINTER(c_int32), POINTER(c_int32), c_void_p]),
    "capf_table_from_packed_rows": (c_int32, [_S, c_int32, POINTER(c_char_p), POINTER(c_int32), POINTER(c_int32),
                                              POINTER(c_int64), POINTER(c_int32), c_void_p, c_int64,
                                              POINTER(_T)]),
    "capf_dot_u32": (c_int32, [_S, c_void_p, c_void_p, c_int64, POINTER(c_uint64)]),
    "capf_comm_unique_id": (c_int32, [c_void_p]),
    "capf_comm_init": (c_int32, [_S, c_int32, c_int32, c_void_p, _PT]),
    "capf_comm_destroy": (c_int32, [c_void_p]),
    "capf_comm_rank": (c_int32, [c_void_p, POINTER(c_int32), POINTER(c_int32)]),
    "capf_comm_all_reduce_i64": (c_int32, [c_void_p, c_void_p, c_int64, c_int32]),
    "capf_comm_all_gather_bytes": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p]),
    "capf_comm_all_to_all_bytes": (c_int32, [c_void_p, c_void_p, POINTER(c_int64), c_void_p, POINTER(c_int64)]),
    "capf_session_alloc": (c_int32, [_S, c_int64, POINTER(c_void_p)]),
    "capf_session_free": (c_int32, [_S, c_void_p]),
    "capf_session_copy": (c_int32, [_S, c_void_p, c_void_p, c_int64, c_int32]),
    "capf_session_literal_set": (c_int32, [_S, POINTER(c_int64), c_int64, POINTER(c_int32)]),
    "capf_session_code_map": (c_int32, [_S, POINTER(c_int64), c_int64, POINTER(c_int32)]),
    "capf_session_code_map_extend": (c_int32, [_S, c_int32, POINTER(c_int64), c_int64, POINTER(c_int32)]),
    "capf_table_add_list": (c_int32, [_T, c_char_p, c_int32, c_void_p, c_void_p, c_void_p, _PT]),
    "capf_table_name_list": (c_int32, [_T, c_int32, _STRS, POINTER(c_int32), POINTER(c_int64), c_char_p, _PT]),
    "capf_table_list_columns": (c_int32, [_T, c_int32, _STRS, c_char_p, _PT]),
    "capf_session_value_map": (c_int32, [_S, POINTER(c_int64), POINTER(c_int64), POINTER(c_int64), c_int64,
                                         POINTER(c_int32)]),
}

EXPORTED_SYMBOLS = sorted(_SIGS)

_lib = None
_exiting = False


def _at_exit():
    # handles still alive at interpreter exit are leaked, not released: the
    # HIP runtime may already be shutting down
    global _exiting
    _exiting = True


import atexit  # noqa: E402

atexit.register(_at_exit)


def load(path=LIB_PATH):
    """Load libcapf_gpu.so (raises if absent — there is no fallback)."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    if not os.path.exists(path):
        raise ImportError(
            f"{path} not found: build the HIP extension first (python -c 'import __graft_entry__ as g; g.build()')")
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path == LIB_PATH:
        _lib = lib
    return lib


def check(status):
    if status != 0:
        lib = load()
        msg = lib.capf_last_error().decode("utf-8", "replace")
        raise _ERRORS.get(status, CypherException)(msg)
    return status


_FNS = {}


def call(name, *args):
    fn = _FNS.get(name)
    if fn is None:
        fn = _FNS[name] = getattr(load(), name)
    status = fn(*args)
    if status != 0:
        check(status)
    return status


_STRS = {}  # encoded name arrays per name tuple (read-only on the C side; plans repeat them)


def strs(values):
    key = tuple(values)
    arr = _STRS.get(key)
    if arr is None:
        arr = (c_char_p * max(len(key), 1))()
        for i, v in enumerate(key):
            arr[i] = v.encode() if isinstance(v, str) else v
        if len(_STRS) < 16384:
            _STRS[key] = arr
    return arr


_EXPR_STRUCTS = {}  # id(program) -> (program, struct, refs): memoised programs are reused


def _keepalive_expr(program):
    """Build a CapfExpr from (ops, iargs, fargs, names); returns (struct, refs).
    Immutable (tuple) programs — compile_program's memoised ones — keep their
    struct: the C-ABI copies a program on every call that takes one."""
    if type(program[0]) is tuple:
        ent = _EXPR_STRUCTS.get(id(program))
        if ent is not None and ent[0] is program:
            return ent[1], ent[2]
        e, refs = _build_expr(program)
        if len(_EXPR_STRUCTS) >= 4096:
            _EXPR_STRUCTS.clear()
        _EXPR_STRUCTS[id(program)] = (program, e, refs)  # holds the program: its id stays its own
        return e, refs
    return _build_expr(program)


def _build_expr(program):
    ops, iargs, fargs, names = program
    n = len(ops)
    o = (c_int32 * n)(*ops)
    i = (c_int64 * n)(*iargs)
    f = (c_double * n)(*fargs)
    nm = strs(names)
    e = CapfExpr(n, o, i, f, len(names), nm)
    return e, (o, i, f, nm)


def expr_array(programs):
    """ctypes array of CapfExpr plus the buffers that must stay alive."""
    arr = (CapfExpr * max(len(programs), 1))()
    keep = []
    for k, p in enumerate(programs):
        if p is None:
            continue
        e, refs = _keepalive_expr(p)
        arr[k] = e
        keep.append(refs)
    return arr, keep
