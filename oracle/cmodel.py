"""ctypes binding of oracle/rmat.c (TEST INFRASTRUCTURE ONLY)."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "build")
SO = os.path.join(BUILD, "liboracle.so")

# Graph500 R-MAT parameters
A, B, C = 0.57, 0.19, 0.19


def thresholds(a=A, b=B, c=C):
    t = lambda x: min(int(x * 2 ** 32), 2 ** 32 - 1)
    return t(a), t(a + b), t(a + b + c)


def rmat_seed(scale):
    return 0x5EED0000 + scale


def build():
    os.makedirs(BUILD, exist_ok=True)
    src = os.path.join(HERE, "rmat.c")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        subprocess.check_call(["gcc", "-O3", "-march=x86-64-v2", "-fPIC", "-shared", "-pthread",
                               src, "-o", SO])
    return SO


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        l = ctypes.CDLL(SO)
        P = ctypes.c_void_p
        i64, u64, u32, i32 = ctypes.c_int64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
        l.rmat_edges.argtypes = [i32, u64, u32, u32, u32, i64, i64, P, P]
        l.rmat_edges.restype = None
        l.node_labels.argtypes = [i64, i64, u64, P]
        l.node_labels.restype = None
        l.count_1hop.argtypes = [P, P, i64, P, P, i64]
        l.count_1hop.restype = u64
        l.count_2hop.argtypes = [P, P, i64, i64]
        l.count_2hop.restype = u64
        l.count_triangle_brute.argtypes = [P, P, i64, i64]
        l.count_triangle_brute.restype = u64
        l.degree_hists.argtypes = [P, P, i64, i64, i64, P, P, P]
        l.degree_hists.restype = None
        l.pipeline_build.argtypes = [P, i64, P, P, P, i64, i32]
        l.pipeline_build.restype = P
        l.pipeline_probe.argtypes = [P, i64, i64, i32]
        l.pipeline_probe.restype = u64
        l.onehop_label_count.argtypes = [P, i64, P, i64, P, P, i64, i32]
        l.onehop_label_count.restype = u64
        l.pipeline_build_pairs.argtypes = [P, i32]
        l.pipeline_build_pairs.restype = None
        l.pipeline_triangles.argtypes = [P, i64, i64, i32, P]
        l.pipeline_triangles.restype = u64
        l.pipeline_free.argtypes = [P]
        l.pipeline_free.restype = None
        l.rmat_stream_counts.argtypes = [i32, u64, u32, u32, u32, i64, i32, P]
        l.rmat_stream_counts.restype = None
        l.count_triangle_trace.argtypes = [P, P, i64, i64, i32]
        l.count_triangle_trace.restype = u64
        l.reach_bitset.argtypes = [P, P, i64, i64, i32, i32, P]
        l.reach_bitset.restype = None
        l.reach_paths.argtypes = [P, P, i64, i64, i32, P, i64, i32, P]
        l.reach_paths.restype = i64
        l.oracle_splitmix64.argtypes = [u64]
        l.oracle_splitmix64.restype = u64
        _lib = l
    return _lib


def rmat(scale, edge_factor=16, seed=None, first=0, count=None):
    seed = rmat_seed(scale) if seed is None else seed
    m = (edge_factor << scale) if count is None else count
    src = np.empty(m, dtype=np.int64)
    dst = np.empty(m, dtype=np.int64)
    ta, tab, tabc = thresholds()
    lib().rmat_edges(scale, seed, ta, tab, tabc, first, m, src.ctypes.data, dst.ctypes.data)
    return src, dst


def labels(n, seed, base=0):
    out = np.empty(n, dtype=np.uint8)
    lib().node_labels(base, n, seed, out.ctypes.data)
    return out


def count_1hop(src, dst, n, in_a=None, in_b=None):
    pa = None if in_a is None else np.ascontiguousarray(in_a, dtype=np.uint8)
    pb = None if in_b is None else np.ascontiguousarray(in_b, dtype=np.uint8)
    return lib().count_1hop(src.ctypes.data, dst.ctypes.data, len(src),
                            None if pa is None else pa.ctypes.data,
                            None if pb is None else pb.ctypes.data, n)


def count_triangle_brute(src, dst, n):
    """(a)-->(b)-->(c)-->(a) with distinct rels, brute force over rels (small scales)."""
    L = lib()
    src = np.ascontiguousarray(src, dtype=np.int64)
    dst = np.ascontiguousarray(dst, dtype=np.int64)
    return int(L.count_triangle_brute(src.ctypes.data, dst.ctypes.data, len(src), n))


def count_triangle_formula(src, dst, n):
    """Same count by linear algebra: trace(A^3) over the multiplicity matrix A
    (closed walks a->b->c->a of rels), minus the walks reusing a rel — only
    three self-loops at one node can coincide: L^3 - L(L-1)(L-2) per node."""
    import scipy.sparse as sp
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    ok = (src >= 0) & (src < n) & (dst >= 0) & (dst < n)
    s, d = src[ok], dst[ok]
    A = sp.csr_matrix((np.ones(len(s), dtype=np.int64), (s, d)), shape=(n, n))
    A.sum_duplicates()
    tr = int((A @ A).multiply(A.T).sum())
    L = np.bincount(s[s == d], minlength=n).astype(object)
    bad = sum(int(x) ** 3 - int(x) * (int(x) - 1) * (int(x) - 2) for x in L if x)
    return tr - bad


def count_triangle_trace(src, dst, n, threads=8):
    """trace(A^3) − self-loop corrections by sorted-list intersection in C
    (threads; an independent method for the larger fixture scales)."""
    src = np.ascontiguousarray(src, dtype=np.int64)
    dst = np.ascontiguousarray(dst, dtype=np.int64)
    return int(lib().count_triangle_trace(src.ctypes.data, dst.ctypes.data, len(src), n, threads))


def stream_counts(scale, edge_factor=16, threads=8):
    """Closed-form counts of the full-size R-MAT graph, streamed (no edge
    arrays): dict(two_hop, self_loops, one_hop_person, max_in, max_out)."""
    res = np.zeros(5, dtype=np.uint64)
    ta, tab, tabc = thresholds()
    lib().rmat_stream_counts(scale, rmat_seed(scale), ta, tab, tabc, edge_factor << scale, threads,
                             res.ctypes.data)
    keys = ("two_hop", "self_loops", "one_hop_person", "max_in", "max_out")
    return {k: int(v) for k, v in zip(keys, res)}


def onehop_label_count(person_ids, node_ids, src, dst, threads=8):
    """Config 2's Flink plan shape on the host (oracle/rmat.c): hash-join
    builds on the Person scan and the all-node scan, rels streamed through both
    probes on `threads` workers."""
    p = np.ascontiguousarray(person_ids, dtype=np.int64)
    a = np.ascontiguousarray(node_ids, dtype=np.int64)
    s = np.ascontiguousarray(src, dtype=np.int64)
    d = np.ascontiguousarray(dst, dtype=np.int64)
    return int(lib().onehop_label_count(p.ctypes.data, len(p), a.ctypes.data, len(a), s.ctypes.data,
                                        d.ctypes.data, len(s), threads))


def count_2hop(src, dst, n):
    return lib().count_2hop(src.ctypes.data, dst.ctypes.data, len(src), n)


def degree_hists(src, dst, base, n):
    i = np.empty(n, dtype=np.uint32)
    o = np.empty(n, dtype=np.uint32)
    loops = ctypes.c_int64()
    lib().degree_hists(src.ctypes.data, dst.ctypes.data, len(src), base, n, i.ctypes.data, o.ctypes.data,
                       ctypes.byref(loops))
    return i, o, loops.value


class Pipeline:
    """Flink-shaped hash-join pipeline of the 2-hop count (CPU baseline)."""

    def __init__(self, node_ids, rel_ids, src, dst, threads=1):
        self._keep = [np.ascontiguousarray(x, dtype=np.int64) for x in (node_ids, rel_ids, src, dst)]
        n, i, s, d = self._keep
        self.m = len(s)
        self._h = lib().pipeline_build(n.ctypes.data, len(n), i.ctypes.data, s.ctypes.data, d.ctypes.data,
                                       len(s), threads)

    def probe(self, lo, hi, threads):
        return lib().pipeline_probe(self._h, lo, hi, threads)

    def build_pairs(self, threads):
        """The (start, end)-keyed R3 table of the triangle's ExpandInto join."""
        lib().pipeline_build_pairs(self._h, threads)

    def triangles(self, lo, hi, threads):
        """(triangle rows, wedge rows) of r1 rows [lo, hi): the relational plan's
        Expand, Expand, ExpandInto with the uniqueness filters."""
        w = ctypes.c_uint64()
        c = lib().pipeline_triangles(self._h, lo, hi, threads, ctypes.byref(w))
        return int(c), int(w.value)

    def close(self):
        if self._h:
            lib().pipeline_free(self._h)
            self._h = None

    def __del__(self):
        self.close()


def reach_bitset(src, dst, n, upper=3, threads=8):
    """reach[a] for every node a in [0, n): distinct nodes at walk distance 1..upper
    (config 5; oracle/rmat.c::reach_bitset)."""
    s = np.ascontiguousarray(src, dtype=np.int64)
    d = np.ascontiguousarray(dst, dtype=np.int64)
    out = np.zeros(n, dtype=np.int64)
    lib().reach_bitset(s.ctypes.data, d.ctypes.data, len(s), n, upper, threads, out.ctypes.data)
    return out


def reach_paths(src, dst, n, sources, upper=3, threads=8):
    """(reach per sampled source, isomorphic paths enumerated): the relational
    plan's shape (join chain + isomorphism filters, DISTINCT, GROUP BY)."""
    s = np.ascontiguousarray(src, dtype=np.int64)
    d = np.ascontiguousarray(dst, dtype=np.int64)
    a = np.ascontiguousarray(sources, dtype=np.int64)
    out = np.zeros(max(len(a), 1), dtype=np.int64)
    paths = lib().reach_paths(s.ctypes.data, d.ctypes.data, len(s), n, upper, a.ctypes.data, len(a), threads,
                              out.ctypes.data)
    return out[:len(a)], int(paths)


def reach_histogram(reach):
    """RETURN reach, count(*) AS n as sorted [reach, n] pairs (sources with reach ≥ 1)."""
    r = np.asarray(reach)
    vals, cnts = np.unique(r[r > 0], return_counts=True)
    return [[int(v), int(c)] for v, c in zip(vals, cnts)]
