// lists.hip — LIST columns: collect(e) per group and gathers of list rows.
//
// collect is the list-valued aggregator of the reference's Table SPI group
// (Expr.scala Collect, lowered by FlinkSQLExprMapper.scala:283 to Flink's
// COLLECT, a MULTISET).  A LIST column is CSR-shaped: int64 offsets [n + 1] in
// `data` and the elements in `child` (a plain column, no NULL elements).
//   collect: keep the rows whose argument is non-NULL (compact_flags), drop
//   duplicate (group, value) pairs for DISTINCT (group_rows), stable radix sort
//   by (group, value) — elements ascend within a list —, per-group counts with
//   atomics, one exclusive scan over ng + 1 counters → offsets.
//   gather: new lengths, exclusive scan → offsets, one thread per output list
//   writes its child indexes, then the element column is gathered.
#include <algorithm>

#include "capf_internal.h"
#include "device_common.h"

namespace capf {

__global__ void k_valid_flags(const uint8_t *valid, int64_t n, uint8_t *flags) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    flags[i] = valid[i] ? 1 : 0;
}

__global__ void k_group_counts(const int64_t *gid, int64_t n, unsigned long long *counts) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&counts[gid[i]], 1ull);
}

static ColPtr list_column(Session *s, int64_t n, const BufPtr &offsets, const ColPtr &child) {
  auto o = std::make_shared<Column>();
  o->type = Type::List;
  o->n = n;
  o->data = offsets;
  o->child = child;
  (void)s;
  return o;
}

static ColPtr empty_elements(Session *s, Type elem) {
  return elem == Type::Null ? null_column(s, Type::Null, 0) : make_column(s, elem, 0, false);
}

ColPtr collect_lists(Session *s, const Grouping &g, int64_t nrows, const ColPtr &arg,
                     bool distinct) {
  const int64_t ng = g.ngroups;
  BufPtr offsets = s->alloc(8 * (ng + 1));
  HIP_CHECK(hipMemsetAsync(offsets->p, 0, 8 * (ng + 1), s->stream));
  force(arg);
  if (nrows == 0 || ng == 0 || arg->type == Type::Null)
    return list_column(s, ng, offsets, empty_elements(s, arg->type));
  auto gid = std::make_shared<Column>();
  gid->type = Type::Int64;
  gid->n = nrows;
  gid->data = g.group_of_row;
  // rows with a non-NULL argument
  ColPtr gk = gid, vk = arg;
  int64_t k = nrows;
  if (arg->valid) {
    BufPtr flags = s->alloc(nrows);
    hipLaunchKernelGGL(k_valid_flags, dim3(grid_for(nrows, 256)), dim3(256), 0, s->stream,
                       (const uint8_t *)arg->valid->p, nrows, (uint8_t *)flags->p);
    KERNEL_CHECK();
    BufPtr idx = compact_flags(s, (const uint8_t *)flags->p, nrows, &k);
    gk = gather_column(s, gid, (const int64_t *)idx->p, k);
    vk = gather_column(s, arg, (const int64_t *)idx->p, k);
  }
  if (k == 0) return list_column(s, ng, offsets, empty_elements(s, arg->type));
  if (distinct) {  // one row per distinct (group, value)
    Data pairs;
    pairs.nrows = k;
    pairs.cols = {gk, vk};
    Grouping dg = group_rows(s, pairs, {0, 1});
    const int64_t *reps = (const int64_t *)dg.rep_row->p;
    gk = gather_column(s, gk, reps, dg.ngroups);
    vk = gather_column(s, vk, reps, dg.ngroups);
    k = dg.ngroups;
  }
  BufPtr perm = sort_permutation(s, {gk, vk}, {0, 0}, k);
  ColPtr gs = gather_column(s, gk, (const int64_t *)perm->p, k);
  ColPtr vs = decode_column(s, gather_column(s, vk, (const int64_t *)perm->p, k));
  BufPtr counts = s->alloc(8 * (ng + 1));
  HIP_CHECK(hipMemsetAsync(counts->p, 0, 8 * (ng + 1), s->stream));
  hipLaunchKernelGGL(k_group_counts, dim3(grid_for(k, 256)), dim3(256), 0, s->stream,
                     (const int64_t *)gs->data->p, k, (unsigned long long *)counts->p);
  KERNEL_CHECK();
  // counts[ng] = 0, so the exclusive scan's last entry is the element total
  exclusive_scan_i64(s, (const int64_t *)counts->p, (int64_t *)offsets->p, ng + 1);
  auto child = std::make_shared<Column>();
  child->type = vs->type;
  child->n = k;
  child->data = vs->data;  // no NULL elements: validity dropped
  return list_column(s, ng, offsets, child);
}

__global__ void k_list_lengths(const int64_t *off, const int64_t *idx, int64_t m, int64_t *len) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = idx[i];
    len[i] = j < 0 ? 0 : off[j + 1] - off[j];
  }
}

__global__ void k_list_child_idx(const int64_t *off, const int64_t *idx, const int64_t *noff,
                                 int64_t m, int64_t *cidx) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = idx[i];
    if (j < 0) continue;
    const int64_t a = off[j], len = off[j + 1] - a, o = noff[i];
    for (int64_t q = 0; q < len; ++q) cidx[o + q] = a + q;
  }
}

__global__ void k_list_valid(const uint8_t *sval, const int64_t *idx, int64_t m, uint8_t *dval) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = idx[i];
    dval[i] = j < 0 ? 0 : (sval ? sval[j] : 1);
  }
}

ColPtr gather_list(Session *s, const ColPtr &c, const int64_t *d_idx, int64_t m) {
  BufPtr noff = s->alloc(8 * (m + 1));
  HIP_CHECK(hipMemsetAsync(noff->p, 0, 8 * (m + 1), s->stream));
  if (m == 0) return list_column(s, 0, noff, empty_elements(s, c->child->type));
  BufPtr len = s->alloc(8 * (m + 1));
  HIP_CHECK(hipMemsetAsync(len->p, 0, 8 * (m + 1), s->stream));
  const int64_t *off = (const int64_t *)c->data->p;
  hipLaunchKernelGGL(k_list_lengths, dim3(grid_for(m, 256)), dim3(256), 0, s->stream, off, d_idx, m,
                     (int64_t *)len->p);
  KERNEL_CHECK();
  const int64_t total = exclusive_scan_i64(s, (const int64_t *)len->p, (int64_t *)noff->p, m + 1);
  ColPtr child;
  if (total == 0 || c->child->type == Type::Null) {
    child = empty_elements(s, c->child->type);
  } else {
    BufPtr cidx = s->alloc(8 * total);
    hipLaunchKernelGGL(k_list_child_idx, dim3(grid_for(m, 256)), dim3(256), 0, s->stream, off, d_idx,
                       (const int64_t *)noff->p, m, (int64_t *)cidx->p);
    KERNEL_CHECK();
    child = gather_column(s, c->child, (const int64_t *)cidx->p, total);
  }
  ColPtr o = list_column(s, m, noff, child);
  o->valid = s->alloc(m);
  hipLaunchKernelGGL(k_list_valid, dim3(grid_for(m, 256)), dim3(256), 0, s->stream,
                     c->valid ? (const uint8_t *)c->valid->p : nullptr, d_idx, m,
                     (uint8_t *)o->valid->p);
  KERNEL_CHECK();
  return o;
}

}  // namespace capf
