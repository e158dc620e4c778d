"""numpy restatement of csrc/device_common.h node_mix — TEST INFRASTRUCTURE ONLY.

The partitioned 2-hop histograms (and capf_chain2_local_hists) index node
offset x = id − lo by node_mix(x) on a 2^k domain, k = max(16, ceil log2 n):
h = (x·0xB5297B) mod 2^k; h ^= h >> k/2.  Tests use it to check the GPU
histograms entry by entry."""
import numpy as np

A = 0xB5297B


def hist_bits(n):
    k = 16
    while (1 << k) < n:
        k += 1
    return k


def node_mix(x, k):
    x = np.asarray(x, dtype=np.uint64)
    mask = np.uint64((1 << k) - 1)
    h = (x * np.uint64(A)) & mask
    return (h ^ (h >> np.uint64(k // 2))).astype(np.int64)


def owner(x, n_nodes, parts):
    """Owner rank of node offsets x under the node-partitioned layout
    (csrc/chain2_partitioned.hip owned_buckets/owner_of): rank p owns the
    64 Ki-index buckets [nb·p/parts, nb·(p+1)/parts) of mix(x)."""
    k = hist_bits(n_nodes)
    nb = (1 << k) >> 16
    b = node_mix(x, k) >> 16
    bounds = np.array([nb * p // parts for p in range(parts + 1)], dtype=np.int64)
    return np.searchsorted(bounds, b, side="right") - 1
