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

// ---------------------------------------------------------------- UNWIND
// withColumns(Explode(list) AS item) (RelationalPlanner.scala:99-101): row i of
// the output is input row i / k with element i % k of the constant list
// (k elements): two index columns, every input column a lazy gather of the
// first, the element column a gather of the second.
__global__ void k_explode_idx(int64_t m, int64_t k, int64_t *row, int64_t *elem) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / k;
    row[i] = r;
    elem[i] = i - r * k;
  }
}

DataPtr explode_values(Session *s, const Data &d, const ColPtr &values) {
  const int64_t k = values->n, m = d.nrows * k;
  auto out = std::make_shared<Data>();
  out->nrows = m;
  BufPtr row = s->alloc(8 * std::max<int64_t>(m, 1)), elem = s->alloc(8 * std::max<int64_t>(m, 1));
  if (m > 0) {
    hipLaunchKernelGGL(k_explode_idx, dim3(grid_for(m, 256)), dim3(256), 0, s->stream, m, k,
                       (int64_t *)row->p, (int64_t *)elem->p);
    KERNEL_CHECK();
  }
  IdxCache cache;
  for (auto &c : d.cols) out->cols.push_back(gather_lazy(s, c, row, m, false, &cache));
  out->cols.push_back(m > 0 ? gather_column(s, values, (const int64_t *)elem->p, m)
                            : (values->type == Type::Null ? null_column(s, Type::Null, 0)
                                                          : make_column(s, values->type, 0, false)));
  return out;
}

// a LIST column: output rows [off[r], off[r+1]) come from input row r and
// hold its elements in order (the element column is the list's child, as is)
__global__ void k_explode_list_rows(const int64_t *off, const uint8_t *valid, int64_t n, int64_t *row) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x) {
    if (valid && !valid[r]) continue;
    for (int64_t q = off[r]; q < off[r + 1]; ++q) row[q] = r;
  }
}
// drop the elements of NULL lists: their element rows keep row = -1
__global__ void k_row_flags(const int64_t *row, int64_t n, uint8_t *flags) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    flags[i] = row[i] >= 0 ? 1 : 0;
}

DataPtr explode_list(Session *s, const Data &d, int list_col) {
  const ColPtr &lc = d.cols[(size_t)list_col];
  auto out = std::make_shared<Data>();
  if (lc->type == Type::Null || d.nrows == 0) {  // nothing to unwind
    out->nrows = 0;
    BufPtr none = s->alloc(8);
    for (auto &c : d.cols) out->cols.push_back(gather_column(s, c, (const int64_t *)none->p, 0, false));
    out->cols.push_back(null_column(s, lc->type == Type::Null ? Type::Null : lc->child->type, 0));
    return out;
  }
  force(lc);
  int64_t total = 0;
  HIP_CHECK(hipMemcpyAsync(&total, (const int64_t *)lc->data->p + d.nrows, 8, hipMemcpyDeviceToHost, s->stream));
  s->sync();
  BufPtr row = s->alloc(8 * std::max<int64_t>(total, 1));
  ColPtr elems = lc->child;
  int64_t m = total;
  if (total > 0) {
    HIP_CHECK(hipMemsetAsync(row->p, 0xFF, 8 * total, s->stream));
    hipLaunchKernelGGL(k_explode_list_rows, dim3(grid_for(d.nrows, 256)), dim3(256), 0, s->stream,
                       (const int64_t *)lc->data->p, lc->valid ? (const uint8_t *)lc->valid->p : nullptr, d.nrows,
                       (int64_t *)row->p);
    KERNEL_CHECK();
    if (lc->valid) {  // elements of NULL lists (if any were stored) are dropped
      BufPtr flags = s->alloc(total);
      hipLaunchKernelGGL(k_row_flags, dim3(grid_for(total, 256)), dim3(256), 0, s->stream,
                         (const int64_t *)row->p, total, (uint8_t *)flags->p);
      KERNEL_CHECK();
      BufPtr keep = compact_flags(s, (const uint8_t *)flags->p, total, &m);
      if (m != total) {
        ColPtr r64 = std::make_shared<Column>();
        r64->type = Type::Int64;
        r64->n = total;
        r64->data = row;
        row = gather_column(s, r64, (const int64_t *)keep->p, m)->data;
        elems = gather_column(s, elems, (const int64_t *)keep->p, m);
      }
    }
  }
  out->nrows = m;
  IdxCache cache;
  for (auto &c : d.cols) out->cols.push_back(gather_lazy(s, c, row, m, false, &cache));
  out->cols.push_back(elems);
  return out;
}

// ---------------------------------------------------------- labels / keys
// labels(n) / keys(n) (FlinkSQLExprMapper.scala:136-153, the GetLabels /
// GetKeys UDFs at :310-329): per row the names (STRING codes, caller-sorted)
// of the label columns holding TRUE (kind 0) or of the property columns
// holding a value (kind 1).  A row with none gets the empty list (the UDFs
// return an empty array, never NULL).  Two passes: per-row counts → offsets
// (exclusive scan) → the codes written in column order.
constexpr int NL_MAX = 64;
struct NameCols {
  ColView c[NL_MAX];
  int32_t kind[NL_MAX];
  int64_t code[NL_MAX];
  int32_t n;
};

__device__ inline bool nl_hit(const NameCols &nc, int j, int64_t r) {
  const ColView &v = nc.c[j];
  if (v.type == CAPF_TYPE_NULL || !v.data || (v.valid && !v.valid[r])) return false;
  return nc.kind[j] ? true : ((const uint8_t *)v.data)[r] != 0;
}

__global__ void k_name_counts(NameCols nc, int64_t n, int64_t *cnt) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    int64_t k = 0;
    for (int j = 0; j < nc.n; ++j) k += nl_hit(nc, j, r) ? 1 : 0;
    cnt[r] = k;
  }
}

__global__ void k_name_fill(NameCols nc, int64_t n, const int64_t *off, int64_t *codes) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    int64_t o = off[r];
    for (int j = 0; j < nc.n; ++j)
      if (nl_hit(nc, j, r)) codes[o++] = nc.code[j];
  }
}

ColPtr name_list_column(Session *s, const Data &d, const std::vector<int> &cols, const std::vector<int32_t> &kinds,
                        const std::vector<int64_t> &codes) {
  if (cols.size() > (size_t)NL_MAX) not_impl("labels / keys over more than 64 columns");
  NameCols nc{};
  nc.n = (int32_t)cols.size();
  for (size_t j = 0; j < cols.size(); ++j) {
    const ColPtr &c = d.cols[(size_t)cols[j]];
    if (kinds[j] == 0 && c->type != Type::Bool && c->type != Type::Null) illegal("label column is not BOOLEAN");
    if (c->type == Type::List) not_impl("keys() over a LIST property");
    nc.c[j] = c->type == Type::Null ? ColView{nullptr, nullptr, CAPF_TYPE_NULL, ENC_PLAIN, 0} : view_of(c);
    nc.kind[j] = kinds[j];
    nc.code[j] = codes[j];
  }
  const int64_t n = d.nrows;
  BufPtr off = s->alloc(8 * (n + 1));
  int64_t total = 0;
  if (n > 0) {
    BufPtr cnt = s->alloc(8 * n);
    hipLaunchKernelGGL(k_name_counts, dim3(grid_for(n, 256)), dim3(256), 0, s->stream, nc, n, (int64_t *)cnt->p);
    KERNEL_CHECK();
    total = exclusive_scan_i64(s, (const int64_t *)cnt->p, (int64_t *)off->p, n);
  }
  HIP_CHECK(hipMemcpyAsync((int64_t *)off->p + n, &total, 8, hipMemcpyHostToDevice, s->stream));
  ColPtr child = make_column(s, Type::String, total, false);
  if (total > 0) {
    hipLaunchKernelGGL(k_name_fill, dim3(grid_for(n, 256)), dim3(256), 0, s->stream, nc, n, (const int64_t *)off->p,
                       (int64_t *)child->data->p);
    KERNEL_CHECK();
  }
  s->sync();  // (the pageable total)
  return list_column(s, n, off, child);
}

// ------------------------------------------------- list literals per row
// Element j of every row: child[i * k + j] = column j's value (an INTEGER
// widened to FLOAT when the list's element type is FLOAT); a NULL element
// raises the flag (LIST columns hold no NULL elements).
__global__ void k_list_elem(ColView c, int64_t n, int32_t k, int32_t j, int32_t elem, void *child,
                            uint32_t *null_seen) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (c.type == CAPF_TYPE_NULL || (c.valid && !c.valid[i])) null_seen[0] = 1u;
    const int64_t o = i * k + j;
    if (elem == CAPF_TYPE_BOOL) {
      ((uint8_t *)child)[o] = c.data ? (((const uint8_t *)c.data)[i] ? 1 : 0) : 0;
    } else if (elem == CAPF_TYPE_FLOAT64) {
      ((double *)child)[o] = !c.data ? 0.0
                             : c.type == CAPF_TYPE_FLOAT64 ? ((const double *)c.data)[i] : (double)ld_int(c, i);
    } else {
      ((int64_t *)child)[o] = c.data ? ld_int(c, i) : 0;
    }
  }
}

__global__ void k_list_offsets_stride(int64_t *off, int64_t n, int32_t k) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += (int64_t)gridDim.x * blockDim.x)
    off[i] = i * k;
}

ColPtr list_from_columns(Session *s, const Data &d, const std::vector<int> &cols, Type elem) {
  const int64_t n = d.nrows;
  const int32_t k = (int32_t)cols.size();
  BufPtr off = s->alloc(8 * (n + 1));
  hipLaunchKernelGGL(k_list_offsets_stride, dim3(grid_for(n + 1, 256)), dim3(256), 0, s->stream,
                     (int64_t *)off->p, n, k);
  KERNEL_CHECK();
  ColPtr child = k == 0 ? empty_elements(s, elem) : make_column(s, elem, n * k, false);
  if (n > 0 && k > 0) {
    BufPtr flag = s->alloc(4);
    HIP_CHECK(hipMemsetAsync(flag->p, 0, 4, s->stream));
    for (int32_t j = 0; j < k; ++j) {
      const ColPtr &c = d.cols[(size_t)cols[(size_t)j]];
      const ColView v = c->type == Type::Null ? ColView{nullptr, nullptr, CAPF_TYPE_NULL, ENC_PLAIN, 0} : view_of(c);
      hipLaunchKernelGGL(k_list_elem, dim3(grid_for(n, 256)), dim3(256), 0, s->stream, v, n, k, j, (int32_t)elem,
                         child->data->p, (uint32_t *)flag->p);
      KERNEL_CHECK();
    }
    uint32_t seen = 0;
    HIP_CHECK(hipMemcpyAsync(&seen, flag->p, 4, hipMemcpyDeviceToHost, s->stream));
    s->sync();
    if (seen) not_impl("a NULL element in a list (LIST columns hold no NULL elements)");
  }
  return list_column(s, n, off, child);
}

}  // namespace capf
