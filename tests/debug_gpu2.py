"""Ad-hoc GPU diagnostics: which materialising stage breaks at large sizes."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import capf_import  # noqa
from capf_amd.table import GpuSession
from capf_amd.expr import Equals, Modulo, IntegerLit, Var, T_INT
from capf_amd.header import RecordHeader
from oracle import cmodel

s = GpuSession(0)
for n in (1 << 20, 5 << 20, 20 << 20):
    t = s.table([("i", T_INT, np.arange(n, dtype=np.int64), None)])
    f = t.filter(Equals(Modulo(Var("i"), IntegerLit(3)), IntegerLit(0)), RecordHeader({Var("i"): "i"}), {})
    v, _ = f.column_arrays("i")
    print("filter n", n, "size", len(v), "expect", (n + 2) // 3, "ok", np.array_equal(v, np.arange(0, n, 3)))

# join with skewed keys: probe p (keys), build b (keys with multiplicity)
rng = np.random.default_rng(0)
for nb, np_, nk in ((65536, 65536, 4096), (65536, 1 << 20, 4096), (1 << 20, 1 << 20, 1 << 16)):
    bk = (rng.zipf(1.5, nb) % nk).astype(np.int64)
    pk = (rng.zipf(1.5, np_) % nk).astype(np.int64)
    B = s.table([("bk", T_INT, bk, None), ("bi", T_INT, np.arange(nb, dtype=np.int64), None)])
    P = s.table([("pk", T_INT, pk, None), ("pi", T_INT, np.arange(np_, dtype=np.int64), None)])
    J = P.join(B, "inner", ("pk", "bk"))
    a, _ = J.column_arrays("pk"); b, _ = J.column_arrays("bk")
    pi, _ = J.column_arrays("pi"); bi, _ = J.column_arrays("bi")
    cnt = np.bincount(bk, minlength=nk)
    expect = int(cnt[pk].sum())
    print("join", nb, np_, "rows", len(a), "expect", expect, "keys equal", np.array_equal(a, b),
          "pk consistent", np.array_equal(pk[pi], a), "bk consistent", np.array_equal(bk[bi], b),
          "distinct pairs", len(set(zip(pi.tolist(), bi.tolist()))) if len(a) < 3e7 else -1)
