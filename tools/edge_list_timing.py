"""Edge-list ingest timing on one GPU.

    python tools/edge_list_timing.py [scale] [reps]

Writes the R-MAT edge list of `scale` as a CSV of fixed-width (zero-padded,
valid LONG) fields "SSSSSSSS,DDDDDDDD\n" (18 B/line) to a temp file, then
loads it with EdgeListDataSource's GPU parser (capf_edge_list_read: file read
+ pinned H2D + parse kernels) and reports the parse kernels' device time
(HIP events) and the end-to-end rate.  Checks the parsed columns against the
generator (bit-exact)."""
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import capf_import  # noqa: E402

capf_import.load()
from capf_amd.synthetic import rmat_seed, thresholds  # noqa: E402
from capf_amd.table import GpuSession  # noqa: E402


def fixed_width_csv(src, dst, w=8):
    m = len(src)
    buf = np.empty((m, 2 * w + 2), dtype=np.uint8)
    for col, off in ((src, 0), (dst, w + 1)):
        v = col.astype(np.int64).copy()
        for k in range(w - 1, -1, -1):
            buf[:, off + k] = 48 + (v % 10)
            v //= 10
    buf[:, w] = ord(",")
    buf[:, 2 * w + 1] = ord("\n")
    return buf.tobytes()


def main():
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    s = GpuSession(0)
    m = 16 << scale
    g = s.rmat_rels(scale, rmat_seed(scale), thresholds(), 0, m)
    src, _ = g.column_arrays("source")
    dst, _ = g.column_arrays("target")
    del g
    data = fixed_width_csv(src, dst)
    fd, path = tempfile.mkstemp(suffix=".csv")
    with os.fdopen(fd, "wb") as f:
        f.write(data)
    try:
        t = s.edge_list(path, ",", "#")  # warm-up + check
        a, _ = t.column_arrays("source")
        b, _ = t.column_arrays("target")
        assert np.array_equal(a, src) and np.array_equal(b, dst), "parse mismatch"
        del t, a, b
        s.reset_profile()
        s.set_profiling(True)
        e2e = []
        for _ in range(reps):
            t0 = time.perf_counter()
            t = s.edge_list(path, ",", "#")
            s.sync()
            e2e.append(time.perf_counter() - t0)
            del t
        s.set_profiling(False)
        prof = s.profile()
        print(f"R-MAT s{scale}: {m} rels, CSV {len(data) / 1e9:.3f} GB ({len(data) / m:.0f} B/line)")
        dev = 0.0
        for k in ("el_count", "el_parse"):
            ms = prof[k]["total_ms"] / reps
            dev += ms
            print(f"  {k:9s} {ms:8.3f} ms  {len(data) / (ms * 1e-3) / 1e9:8.1f} GB/s of text")
        # algorithmic bytes: text read once + (source, target, id) written at int64 width
        alg = len(data) + 24.0 * m
        print(f"  parse kernels {dev:.3f} ms: {alg / (dev * 1e-3) / 1e9:.1f} GB/s algorithmic "
              f"(text + 24 B/rel), {m / (dev * 1e-3) / 1e9:.2f} G rels/s")
        best = min(e2e)
        print(f"  end to end (file read + pinned H2D + parse + ids), best of {reps}: {best * 1e3:.1f} ms, "
              f"{len(data) / best / 1e9:.2f} GB/s")
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()
