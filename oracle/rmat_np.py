"""Independent numpy restatement of the R-MAT generator (small scales) —
TEST INFRASTRUCTURE ONLY.  Pins oracle/rmat.c and csrc/graph_gen.hip:
edge e, level l draws u = 32-bit half of splitmix64(key + 32e + l//2) and picks
the Graph500 quadrant by integer thresholds."""
import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def rmat(scale, seed, thresholds, first, count):
    ta, tab, tabc = (np.uint64(t) for t in thresholds)
    key = splitmix64(np.uint64(seed))
    e = np.arange(first, first + count, dtype=np.uint64)
    src = np.zeros(count, dtype=np.uint64)
    dst = np.zeros(count, dtype=np.uint64)
    r = None
    for l in range(scale):
        if l % 2 == 0:
            with np.errstate(over="ignore"):
                r = splitmix64(key + e * np.uint64(32) + np.uint64(l // 2))
        u = (r >> np.uint64(32)) if l % 2 else (r & np.uint64(0xFFFFFFFF))
        q = np.where(u < ta, 0, np.where(u < tab, 1, np.where(u < tabc, 2, 3))).astype(np.uint64)
        bit = np.uint64(scale - 1 - l)
        src |= (q >> np.uint64(1)) << bit
        dst |= (q & np.uint64(1)) << bit
    return src.astype(np.int64), dst.astype(np.int64)
