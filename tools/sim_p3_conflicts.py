"""Simulates the LDS same-word serialisation of P3 (k_c5_gather) on the R-MAT
in-side key stream: per run, the keys in random order are cut into 8-key
pieces, 64 pieces per wave step; atomic instruction e of a step touches word
(key & 0x7FFF) for each lane.  Cost of an instruction = max lanes on one word.
Compares plain adds with "sort the lane's 8 keys, one add per distinct key".

    python tools/sim_p3_conflicts.py [scale]
"""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from oracle import cmodel  # noqa: E402
from oracle.nodemix import hist_bits, node_mix  # noqa: E402


def cost(keys):
    """keys: (steps, 64 lanes, 8) → (plain cost, combined cost, plain instrs)."""
    words = keys & 0x7FFF
    plain = 0
    for e in range(8):
        w = words[:, :, e]
        s = np.sort(w, axis=1)
        # max multiplicity per row
        plain += max_mult(s).sum()
    ks = np.sort(keys, axis=2)
    last = np.ones_like(ks, dtype=bool)
    last[:, :, :-1] = ks[:, :, :-1] != ks[:, :, 1:]
    comb = 0
    for e in range(8):
        w = np.where(last[:, :, e], ks[:, :, e] & 0x7FFF, -1 - np.arange(64)[None, :])
        comb += max_mult(np.sort(w, axis=1)).sum()
    # in place: the first occurrence of a key in the lane's piece adds its
    # multiplicity at its own (random) position
    first = np.ones_like(keys, dtype=bool)
    for e in range(1, 8):
        for f in range(e):
            first[:, :, e] &= keys[:, :, e] != keys[:, :, f]
    inpl = 0
    for e in range(8):
        w = np.where(first[:, :, e], keys[:, :, e] & 0x7FFF, -1 - np.arange(64)[None, :])
        inpl += max_mult(np.sort(w, axis=1)).sum()
    print(f"  atomics: plain {keys.size}, deduped {int(first.sum())}")
    return plain, comb, inpl


def max_mult(s):
    # s sorted along axis 1; longest run of equal values per row
    n = s.shape[1]
    eq = s[:, 1:] == s[:, :-1]
    best = np.ones(s.shape[0], dtype=np.int64)
    run = np.ones(s.shape[0], dtype=np.int64)
    for i in range(n - 1):
        run = np.where(eq[:, i], run + 1, 1)
        best = np.maximum(best, run)
    return best


def main():
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    src, dst = cmodel.rmat(scale)
    n = 1 << scale
    k = hist_bits(n)
    h = node_mix(dst, k)
    rng = np.random.default_rng(1)
    runs = h >> 16
    tp = tc = tq = ti = 0
    for r in np.unique(runs)[:16]:
        keys = h[runs == r] & 0xFFFF
        keys = keys[rng.permutation(len(keys))]
        m = len(keys) // 512 * 512
        kk = keys[:m].reshape(-1, 64, 8)
        p, c, q = cost(kk)
        tp += p
        tc += c
        tq += q
        ti += kk.shape[0] * 8
    print(f"s{scale}: instrs {ti}, plain serial cycles {tp} ({tp / ti:.2f}/instr), "
          f"sorted+combined {tc} ({tc / ti:.2f}/instr), in-place dedup {tq} ({tq / ti:.2f}/instr)")


if __name__ == "__main__":
    main()
