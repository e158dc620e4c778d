// graph_gen.hip — deterministic synthetic graph inputs written straight into HBM.
//
// Graph500-style R-MAT (a, b, c, d quadrant recursion, edge factor given by
// the caller) with a counter-based PRNG so that every edge is a pure function
// of (seed, edge index): the GPU, the C oracle (oracle/rmat.c) and every rank
// of a multi-GPU run generate bit-identical graphs.  Self-loops and
// multi-edges are kept.  This stands in for graph ingest
// (EdgeListDataSource, flink-cypher/.../api/io/edgelist/EdgeListDataSource.scala:56-92).
#include "capf_internal.h"
#include "device_common.h"

namespace capf {

__global__ __launch_bounds__(256) void k_rmat(int scale, uint64_t key, uint32_t ta, uint32_t tab,
                                              uint32_t tabc, int64_t first, int64_t count,
                                              int64_t id_base, int64_t *id, int64_t *src,
                                              int64_t *dst) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < count;
       k += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t e = (uint64_t)(first + k);
    uint64_t s = 0, d = 0, r = 0;
    for (int l = 0; l < scale; ++l) {
      if ((l & 1) == 0) r = splitmix64(key + e * 32ull + (uint64_t)(l >> 1));
      const uint32_t u = (l & 1) ? (uint32_t)(r >> 32) : (uint32_t)r;
      const uint32_t q = u < ta ? 0u : (u < tab ? 1u : (u < tabc ? 2u : 3u));
      const int bit = scale - 1 - l;
      s |= (uint64_t)(q >> 1) << bit;
      d |= (uint64_t)(q & 1) << bit;
    }
    id[k] = id_base + (int64_t)e;
    src[k] = (int64_t)s;
    dst[k] = (int64_t)d;
  }
}

__global__ void k_range_nodes(int64_t base, int64_t n, uint64_t lkey, int64_t *id, uint8_t *label) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
       k += (int64_t)gridDim.x * blockDim.x) {
    id[k] = base + k;
    if (label) label[k] = (uint8_t)(splitmix64(lkey + (uint64_t)(base + k)) >> 63);
  }
}

}  // namespace capf

using namespace capf;

extern "C" capf_status capf_rmat_rel_table(capf_session *cs, int32_t scale, uint64_t seed,
                                           uint32_t t_a, uint32_t t_ab, uint32_t t_abc,
                                           int64_t first, int64_t count, int64_t id_base,
                                           const char *id_col, const char *src_col,
                                           const char *dst_col, capf_table **out) {
  try {
    if (!cs || !out || !id_col || !src_col || !dst_col) illegal("null argument");
    if (scale < 1 || scale > 40) illegal("scale out of range");
    if (count < 0 || first < 0) illegal("negative edge range");
    if (!(t_a <= t_ab && t_ab <= t_abc)) illegal("R-MAT thresholds must be non-decreasing");
    Session *s = &cs->impl;
    auto n = std::make_shared<Node>();
    n->s = s;
    n->kind = Kind::Source;
    n->names = {id_col, src_col, dst_col};
    n->types = {Type::Int64, Type::Int64, Type::Int64};
    auto d = std::make_shared<Data>();
    d->nrows = count;
    for (int i = 0; i < 3; ++i) d->cols.push_back(make_column(s, Type::Int64, count, false));
    if (count > 0) {
      KernelTimer kt(s, "rmat_generate", 24.0 * count);
      hipLaunchKernelGGL(k_rmat, dim3(grid_for(count, 256, 256 * 64)), dim3(256), 0, s->stream,
                         (int)scale, splitmix64(seed), t_a, t_ab, t_abc, first, count, id_base,
                         (int64_t *)d->cols[0]->data->p, (int64_t *)d->cols[1]->data->p,
                         (int64_t *)d->cols[2]->data->p);
      KERNEL_CHECK();
    }
    s->sync();
    n->result = d;
    auto *t = new capf_table;
    t->node = n;
    *out = t;
    return CAPF_OK;
  } catch (const capf::Error &e) {
    return record_error(e.code, e.what());
  }
}

extern "C" capf_status capf_range_node_table(capf_session *cs, int64_t base, int64_t n_nodes,
                                             uint64_t seed, const char *id_col,
                                             const char *label_col, capf_table **out) {
  try {
    if (!cs || !out || !id_col) illegal("null argument");
    if (n_nodes < 0) illegal("negative node count");
    Session *s = &cs->impl;
    auto n = std::make_shared<Node>();
    n->s = s;
    n->kind = Kind::Source;
    n->names = {id_col};
    n->types = {Type::Int64};
    if (label_col) {
      n->names.emplace_back(label_col);
      n->types.push_back(Type::Bool);
    }
    auto d = std::make_shared<Data>();
    d->nrows = n_nodes;
    d->cols.push_back(make_column(s, Type::Int64, n_nodes, false));
    if (label_col) d->cols.push_back(make_column(s, Type::Bool, n_nodes, false));
    if (n_nodes > 0) {
      hipLaunchKernelGGL(k_range_nodes, dim3(grid_for(n_nodes, 256)), dim3(256), 0, s->stream,
                         base, n_nodes, splitmix64(seed ^ 0x1ABE1ull),
                         (int64_t *)d->cols[0]->data->p,
                         label_col ? (uint8_t *)d->cols[1]->data->p : nullptr);
      KERNEL_CHECK();
    }
    s->sync();
    n->result = d;
    auto *t = new capf_table;
    t->node = n;
    *out = t;
    return CAPF_OK;
  } catch (const capf::Error &e) {
    return record_error(e.code, e.what());
  }
}
