"""numpy restatement of the row routing of csrc/shuffle.hip — TEST
INFRASTRUCTURE ONLY (the checker of capf_table_hash_route and the router of
the CPU tests' oracle exchange, tests/dist_support.py).

owner(row) = ((h >> 32) · parts) >> 32 with
  h = 0x243F6A8885A308D3;  for each key:  h = splitmix64(h ^ bits(key)) + 0x9E3779B97F4A7C15
  bits: INTEGER / STRING code = the int64 value, FLOAT = IEEE bits with
  −0.0 → 0.0 and one NaN, BOOL = 0/1, NULL = 0x6E756C6C6E756C6C.
Strings of the oracle table are Python str (no dictionary codes): they route
by the first 8 bytes of their blake2b digest — consistent across processes,
which is all a router needs (equal keys → equal owner).
"""
import hashlib

import numpy as np

NULL_BITS = np.uint64(0x6E756C6C6E756C6C)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_H0 = np.uint64(0x243F6A8885A308D3)
_GOLD = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x ^ (x >> np.uint64(30))
        x = x * _M1
        x = x ^ (x >> np.uint64(27))
        x = x * _M2
        x = x ^ (x >> np.uint64(31))
    return x


def key_bits(kind, values, valid):
    """uint64 routing image of one key column.  kind: 'int' | 'float' |
    'bool' | 'str' | 'null'."""
    valid = np.asarray(valid, dtype=bool)
    n = len(valid)
    if kind == "null":
        return np.full(n, NULL_BITS, dtype=np.uint64)
    if kind == "float":
        f = np.asarray(values, dtype=np.float64).copy()
        f[f == 0.0] = 0.0
        bits = f.view(np.uint64).copy()
        bits[np.isnan(f)] = np.uint64(0x7FF8000000000000)
    elif kind == "bool":
        bits = (np.asarray(values) != 0).astype(np.uint64)
    elif kind == "str":
        bits = np.array([int.from_bytes(hashlib.blake2b(str(v).encode(), digest_size=8).digest(), "little")
                         if ok else 0 for v, ok in zip(values, valid)], dtype=np.uint64)
    else:
        bits = np.asarray(values, dtype=np.int64).view(np.uint64)
    return np.where(valid, bits, NULL_BITS).astype(np.uint64)


def owners(key_bit_columns, n, parts):
    """Owner (0..parts-1) of each of the n rows."""
    h = np.full(n, _H0, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for b in key_bit_columns:
            h = splitmix64(h ^ b) + _GOLD
        return (((h >> np.uint64(32)) * np.uint64(parts)) >> np.uint64(32)).astype(np.int64)
