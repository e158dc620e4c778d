"""Reachability restatement for the fused config-5 path — TEST INFRASTRUCTURE ONLY.

MATCH (a:L)-[:T*1..u]->(b:L) WITH DISTINCT a, b WITH a, count(*) AS reach
RETURN reach, count(*) AS n  (BASELINE config 5; VarLengthExpandPlanner.scala:82-259
+ FlinkTable.distinct / group).  Independent of the GPU's BFS: boolean sparse
matrix powers R = A ∨ A² ∨ … ∨ A^u (scipy), rows restricted to the sources,
columns to the targets; reach(a) = |row a| for rows with ≥ 1 entry.  (The
relational plan's DISTINCT pairs are the walk-reachable pairs for lower bound
1; tests/test_ldbc_config5.py pins that against an isomorphic-path brute force.)
"""
from collections import Counter

import numpy as np
import scipy.sparse as sp


def reach_counts(src, dst, sources, targets, upper, lower=1):
    """{source id: #distinct targets reachable in 1..upper hops} (> 0 only).
    lower=0 adds the zero-length path of the copyElement branch
    (VarLengthExpandPlanner.scala:180-205): every source also pairs with
    itself, once, whatever its labels — so every source has an entry."""
    ids = np.unique(np.concatenate([src, dst, sources, targets]).astype(np.int64))
    ix = lambda v: np.searchsorted(ids, np.asarray(v, dtype=np.int64))  # noqa: E731
    n = len(ids)
    a = sp.csr_matrix((np.ones(len(src), dtype=np.int8), (ix(src), ix(dst))), shape=(n, n))
    a.data[:] = 1
    a.sum_duplicates()
    a.data = np.minimum(a.data, 1).astype(np.int8)
    s = np.unique(ix(sources))
    r = a[s].astype(np.int32)
    p = r.copy()
    for _ in range(1, upper):
        p = (p @ a).astype(np.int32)
        p.data = np.minimum(p.data, 1)
        p.eliminate_zeros()
        r = r + p
        r.data = np.minimum(r.data, 1)
    tmask = np.zeros(n, dtype=bool)
    tmask[ix(targets)] = True
    r = r.tocsr()
    out = {}
    for row, node in enumerate(s):
        cols = r.indices[r.indptr[row]:r.indptr[row + 1]]
        c = int(tmask[cols].sum())
        if lower == 0 and not (tmask[node] and node in set(cols.tolist())):
            c += 1
        if c:
            out[int(ids[node])] = c
    return out


def config5_histogram(src, dst, sources, targets, upper=3):
    """RETURN reach, count(*) AS n as sorted [reach, n] pairs."""
    return sorted([k, v] for k, v in Counter(reach_counts(src, dst, sources, targets, upper).values()).items())
