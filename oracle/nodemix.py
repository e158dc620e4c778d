"""numpy restatement of csrc/device_common.h node_mix — TEST INFRASTRUCTURE ONLY.

The partitioned 2-hop histograms (and capf_chain2_local_hists) index node
offset x = id − lo by node_mix(x) on a 2^k domain, k = max(15, ceil log2 n):
h = (x·0x9E3779B1) mod 2^k; h ^= h >> k/2; h = (h·0x85EBCA6B) mod 2^k;
h ^= h >> k/2.  Tests use it to check the GPU histograms entry by entry."""
import numpy as np


def hist_bits(n):
    k = 15
    while (1 << k) < n:
        k += 1
    return k


def node_mix(x, k):
    x = np.asarray(x, dtype=np.uint64)
    mask = np.uint64((1 << k) - 1)
    sh = np.uint64(k // 2)
    h = (x * np.uint64(0x9E3779B1)) & mask
    h ^= h >> sh
    h = (h * np.uint64(0x85EBCA6B)) & mask
    return (h ^ (h >> sh)).astype(np.int64)
