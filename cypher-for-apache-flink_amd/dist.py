"""One process per GPU: the hash-partitioned 2-hop count over RCCL.

Two layouts are implemented.

NODE-PARTITIONED (default, `node_partitioned_copies` + `gpu_two_hop_count_sharded`):
SURVEY §8(e) stores each rel on owner(src) and, for incoming expansion, a copy
on owner(dst), with owner(v) = the rank holding mix(v)'s bucket.  Rank r then
holds every rel that ends at one of its nodes (in-copy) and every rel that
starts at one (out-copy): in[b] and out[b] for its own b are both local, the
count-only frontier never leaves the GPU, and the only collective is ONE int64
all-reduce of the per-rank partials Σ_{b owned} in[b]·out[b] − owned self-loops.

EDGE-RANGE (below): rels sharded by edge index, per-node histograms
reduce-scattered (2·N·4 B per rank).  Kept as the layout for graphs stored
without the in-copy.

SURVEY §8(e): the graph is partitioned over G GPUs and the 2-hop join needs
one exchange keyed by the middle node b.  Because the fused count only needs
per-node path multiplicities (the "count-only frontier"), the exchange is
reduced to per-node histograms:

  1. rank r holds the rel shard E_r (a contiguous edge-index range of the
     R-MAT stream — R-MAT edges are i.i.d., so this is a uniform partition);
     it computes in_r[v] = |{e ∈ E_r : dst = v}|, out_r[v] = |{e ∈ E_r : src = v}|
     and its self-loop count with ONE pass over its shard
     (capf_chain2_local_hists);
  2. reduce-scatter (RCCL over xGMI) gives rank r the global in/out counts of
     the nodes it owns (contiguous node range V_r) — the repartition by join
     key b;
  3. rank r computes Σ_{b ∈ V_r} in[b]·out[b] (capf_dot_u32);
  4. one int64 all-reduce of (partial − local self-loops) gives the count.

Bit-exact: every term is an integer; uint32 histogram sums are exact below
2^32 rels per node.  The exchange volume is 2·N·4 B per rank, independent of
the number of joined rows.
"""
import torch
import torch.distributed as dist


def edge_range(m, rank, world):
    return m * rank // world, m * (rank + 1) // world


def padded_nodes(n, world):
    """Histogram length (capf_chain2_hist_len: 2^k >= n, indexed by the node_mix
    hash) padded so every rank's slice is a multiple of 4 (dwordx4)."""
    from .table import chain2_hist_len
    h = chain2_hist_len(n)
    q = 4 * world
    return (h + q - 1) // q * q


def reduce_scatter(t, world, group=None):
    """Sum `t` over ranks and return this rank's contiguous 1/world slice."""
    out = torch.empty(t.numel() // world, dtype=t.dtype, device=t.device)
    if dist.get_backend(group) == "nccl":
        dist.reduce_scatter_tensor(out, t, op=dist.ReduceOp.SUM, group=group)
    else:  # gloo (CPU tests): all-reduce then slice
        t = t.clone()
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        r = dist.get_rank(group)
        out.copy_(t[r * out.numel():(r + 1) * out.numel()])
    return out


def combine_two_hop(in_hist, out_hist, local_loops, dot_fn, group=None):
    """Steps 2-4: exchange the local histograms and reduce to the count.

    in_hist / out_hist: int32 tensors of padded length; dot_fn(a, b) -> int
    computes Σ a·b exactly (GPU: capf_dot_u32; tests: numpy)."""
    world = dist.get_world_size(group)
    rin = reduce_scatter(in_hist, world, group)
    rout = reduce_scatter(out_hist, world, group)
    partial = dot_fn(rin, rout) - int(local_loops)
    acc = torch.tensor([partial], dtype=torch.int64, device=in_hist.device)
    dist.all_reduce(acc, op=dist.ReduceOp.SUM, group=group)
    return int(acc.item())


def gpu_two_hop_count(session, rels, n_nodes, node_base=0, group=None, hists=None):
    """Distributed 2-hop count(*) for this rank's rel shard `rels` (GpuTable)."""
    from .table import chain2_hist_len, dot_u32
    world = dist.get_world_size(group)
    npad = padded_nodes(n_nodes, world)
    if hists is None:
        hists = (torch.zeros(npad, dtype=torch.int32, device="cuda"),
                 torch.zeros(npad, dtype=torch.int32, device="cuda"))
    in_h, out_h = hists
    loops = rels.chain2_local_hists("source", "target", node_base, n_nodes, in_h.data_ptr(), out_h.data_ptr())
    hlen = chain2_hist_len(n_nodes)
    if npad > hlen:
        in_h[hlen:].zero_()
        out_h[hlen:].zero_()
    return combine_two_hop(in_h, out_h, loops,
                           lambda a, b: dot_u32(session, a.data_ptr(), b.data_ptr(), a.numel()), group)


def node_partitioned_copies(rels, n_nodes, world, rank, node_base=0, src="source", dst="target",
                            compact=True, diag=True):
    """(in_copy, out_copy) of this rank: the rels whose target / source node it
    owns, FOR-compacted (compact=True/4: FOR32, 3: FOR24 where the id range
    fits 24 bits; False: int64).  diag: the out-copy in 2-D order — the rels
    whose target the rank owns too first, their count as `out_copy.n_diag`
    (a block partition of the adjacency matrix by (owner(src), owner(dst)));
    only those can be self-loops, so the count reads the target column of
    1/G of the out-copy instead of all of it.  Graph-ingest step, outside the
    timed query."""
    from .table import compact_as
    if diag:
        out_copy, n_diag = rels.node_partition_diag(src, dst, node_base, n_nodes, world, rank)
    else:
        out_copy, n_diag = rels.node_partition(src, node_base, n_nodes, world, rank), -1
    in_copy = rels.node_partition(dst, node_base, n_nodes, world, rank)
    out_copy = compact_as(out_copy, compact)  # compaction keeps the row order
    out_copy.n_diag = n_diag
    in_copy = compact_as(in_copy, compact)
    out_copy.hot_ids = heavy_hitters(in_copy, dst, out_copy, src)
    return in_copy, out_copy


def heavy_hitters(in_copy, in_key, out_copy, out_key, sample=1 << 18, k=1, min_frac=1.0 / 256):
    """Ingest-time statistic of a rank's copies: the (at most k) node ids that
    hold ≥ min_frac (0.4 %) of a sample of the rank's 2-hop keys (the in-copy's target
    and the out-copy's source column, first `sample` rows of each — R-MAT /
    edge-list rows are in no key order).  A plan hint like a most-common-
    values list: the count is exact for any ids (capf_chain2_sharded_count_diag
    counts the hub's keys in registers instead of partitioning them)."""
    import numpy as np
    vals = []
    for t, c in ((in_copy, in_key), (out_copy, out_key)):
        n = min(t.size, sample)
        if n:
            vals.append(np.asarray(t.limit(n).column_arrays(c)[0]))
    if not vals:
        return []
    v = np.concatenate(vals)
    ids, cnt = np.unique(v, return_counts=True)
    order = np.argsort(-cnt, kind="stable")[:k]
    return [int(ids[i]) for i in order if cnt[i] >= max(2, min_frac * len(v))]


def gpu_two_hop_count_sharded(session, in_copy, out_copy, n_nodes, partial, node_base=0, group=None):
    """Distributed 2-hop count(*) over the node-partitioned copies: the local
    partial is enqueued on the session stream (= torch's current stream) into
    the int64 device tensor `partial`, then ONE all-reduce (RCCL) sums it."""
    gpu_two_hop_count_sharded_async(session, in_copy, out_copy, n_nodes, partial, node_base, group)
    return int(partial.item())


def gpu_two_hop_count_sharded_async(session, in_copy, out_copy, n_nodes, partial, node_base=0,
                                    group=None, async_op=False):
    """gpu_two_hop_count_sharded without the host read: the summed count is
    left in `partial` (ordered on the session/torch stream), so a driver can
    enqueue the next query before this one finishes.  async_op=True returns
    the all-reduce's work handle instead of ordering the stream after it: the
    next query's kernels then overlap this query's all-reduce (RCCL runs on
    its own stream); `partial` holds the sum once the handle is waited on."""
    from .table import chain2_sharded_count_async
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    chain2_sharded_count_async(session, in_copy, out_copy, node_base, n_nodes, world, rank,
                               partial.data_ptr())
    return sum_partials(partial, group, async_op)


def sum_partials(partial, group=None, async_op=False):
    """The one collective of the node-partitioned count: an int64 SUM
    all-reduce of the per-rank partials, in place (RCCL on the GPU; gloo in
    the CPU tests).  async_op: return the work handle (wait before reading)."""
    work = dist.all_reduce(partial, op=dist.ReduceOp.SUM, group=group, async_op=async_op)
    return work if async_op else partial


def hist_bits(n_nodes):
    """k of the node_mix domain 2^k ≥ n_nodes (at least 2^16: one bucket)."""
    k = 16
    while (1 << k) < n_nodes:
        k += 1
    return k


def owned_buckets(n_nodes, world, rank):
    """[b0, b1): the 64 Ki-index buckets of node_mix owned by `rank`
    (capf_table_node_partition / capf_chain2_sharded_count use the same split:
    contiguous bucket ranges, nb·r/G .. nb·(r+1)/G)."""
    nb = (1 << hist_bits(n_nodes)) >> 16
    return nb * rank // world, nb * (rank + 1) // world
