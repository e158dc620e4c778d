"""Ad-hoc (not a test): per-unit timeline of P3 (k_c5_gather) from
CAPF_P3_TRACE dumps.  usage: python tools/p3_trace.py TRACEFILE [max_units]"""
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 4)
a = a[a[:, 0] > 0]
t0 = a[:, 0].astype(np.int64)
t1 = a[:, 1].astype(np.int64)
# dumps are appended per query: split where the start time jumps back / far ahead
order = np.argsort(t0)
a, t0, t1 = a[order], t0[order], t1[order]
gaps = np.nonzero(np.diff(t0) > 100000)[0]  # > 1 ms apart (100 MHz clock)
starts = np.concatenate([[0], gaps + 1])
ends = np.concatenate([gaps + 1, [len(a)]])
for q, (i, j) in enumerate(zip(starts, ends)):
    s0, e0 = t0[i:j], t1[i:j]
    base = s0.min()
    dur = (e0 - s0) / 100.0  # µs
    span = (e0.max() - base) / 100.0
    run = (a[i:j, 3] >> np.uint64(32)).astype(np.int64)
    xcc = (a[i:j, 2] >> np.uint64(32)).astype(np.int64)
    hw = (a[i:j, 2] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    cu = (hw >> 8) & 15
    se = (hw >> 13) & 7
    print(f"query {q}: {j - i} units, span {span:.1f} us, unit dur mean {dur.mean():.1f} "
          f"median {np.median(dur):.1f} max {dur.max():.1f} us; last end − first end "
          f"{(e0.max() - e0.min()) / 100:.1f} us")
    slow = np.argsort(-dur)[:8]
    for k in slow:
        print(f"   run {run[k]:4d} dur {dur[k]:.1f} us start +{(s0[k] - base) / 100:.1f} xcc {xcc[k]} se {se[k]} cu {cu[k]}")
    ends_rel = np.sort((e0 - base) / 100.0)
    print("   end-time percentiles (us):", [round(float(np.percentile(ends_rel, p)), 1) for p in (10, 50, 90, 99, 100)])
    if q >= 1:
        break
