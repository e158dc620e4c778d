// capf_internal.h — runtime data structures of the MI355X relational backend.
//
// Columnar SoA tables in HBM, immutable and reference-counted, behind the
// lazy plan DAG that mirrors the okapi RelationalOperator tree
// (okapi-relational/.../impl/operators/RelationalOperator.scala:48-514).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/capf_gpu.h"

namespace capf {

// ----------------------------------------------------------------- errors
struct Error : std::runtime_error {
  int32_t code;
  Error(int32_t c, const std::string &m) : std::runtime_error(m), code(c) {}
};
[[noreturn]] inline void fail(int32_t code, const std::string &m) { throw Error(code, m); }
[[noreturn]] inline void illegal(const std::string &m) { fail(CAPF_ERR_ILLEGAL_ARGUMENT, m); }
[[noreturn]] inline void not_impl(const std::string &m) { fail(CAPF_ERR_NOT_IMPLEMENTED, m); }

#define HIP_CHECK(expr)                                                                  \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      ::capf::fail(_e == hipErrorOutOfMemory ? CAPF_ERR_OOM : CAPF_ERR_HIP,              \
                   std::string(#expr) + ": " + hipGetErrorString(_e));                   \
  } while (0)

// CAPF_DEBUG_SYNC=1: synchronise after every launch so an asynchronous fault
// is reported at the kernel that caused it.
bool debug_sync_enabled();
#define KERNEL_CHECK()                                         \
  do {                                                         \
    HIP_CHECK(hipGetLastError());                              \
    if (::capf::debug_sync_enabled()) HIP_CHECK(hipDeviceSynchronize()); \
  } while (0)

enum class Type : int32_t {
  Null = CAPF_TYPE_NULL,
  Int64 = CAPF_TYPE_INT64,
  Float64 = CAPF_TYPE_FLOAT64,
  Bool = CAPF_TYPE_BOOL,
  String = CAPF_TYPE_STRING,
  List = CAPF_TYPE_LIST  // data = int64 offsets [n + 1], child = the elements
};
inline size_t type_width(Type t) { return t == Type::Bool ? 1 : (t == Type::Null ? 0 : 8); }
const char *type_name(Type t);

struct Session;

// ------------------------------------------------------------- device memory
struct DevBuf {
  void *p = nullptr;
  size_t bytes = 0;
  bool owned = true;
  Session *s = nullptr;
  ~DevBuf();
};
using BufPtr = std::shared_ptr<DevBuf>;

// Column statistics, computed once per column (ingest-time metadata like
// ORC/Parquet min/max), used to pick dense vs hashed join structures.
struct ColStats {
  int64_t non_null = 0;
  int64_t min = 0, max = -1;   // over non-null values (int-like columns)
  bool dense_unique = false;   // values are exactly {min..max}, each once
};

// Physical encodings of an INT64 / STRING-code column.  The logical type is
// unchanged (CTInteger = Flink LONG); ENC_FOR32 is frame-of-reference
// compression chosen at ingest when max - min < 2^32: value = base + u32;
// ENC_FOR24 the same with 3-byte little-endian offsets (max - min < 2^24,
// e.g. node ids of a 16 Mi-node graph): 3 B per id instead of 8.  FOR24
// buffers carry 16 zero bytes past 3·n, so 4-B and 12-B loads at any row
// stay inside the allocation.
enum : int32_t { ENC_PLAIN = 0, ENC_FOR32 = 1, ENC_FOR24 = 2 };

struct Column;
// Late materialisation: a column defined as rows `idx` of `src` (a join side,
// a filter, a sort), gathered only when a kernel or a download reads it
// (force).  Gathers of gathers compose their indexes instead of moving data.
struct LazyGather {
  Session *s = nullptr;
  std::shared_ptr<Column> src;  // never lazy itself
  BufPtr idx;  // int64 [m] (iw 8) or int32 [m] (iw 4), -1 = NULL row (nullable)
  int64_t m = 0;
  bool nullable = false;
  int32_t iw = 8;  // index width in bytes
};

struct Column {
  Type type = Type::Null;
  int64_t n = 0;
  std::shared_ptr<LazyGather> lazy;  // non-null: data/valid/enc/base not yet computed
  int32_t enc = ENC_PLAIN;
  int64_t base = 0;  // ENC_FOR32 reference value
  BufPtr data;   // n * width bytes (4 for ENC_FOR32; nullptr for Type::Null or n == 0)
  BufPtr valid;  // n bytes (1 = present) or nullptr = no nulls
  mutable std::mutex mu;
  mutable std::optional<ColStats> stats;
  // are the non-null values pairwise distinct?  -1 unknown (computed once,
  // like stats: the column is immutable)
  mutable int8_t unique_flag = -1;
  // values of a tiny host-born column (a fused scalar result), kept beside
  // the device copy so `rows` needs no device round trip
  std::vector<int64_t> host_i64;
  // every row holds the same non-NULL value (a literal evaluated over a
  // table, e.g. the label column of a one-label scan): const_bits = its
  // physical bits; a gather of it is a fill (no index read)
  bool is_const = false;
  uint64_t const_bits = 0;
  // Type::List: the element column (never lazy, no NULL elements)
  std::shared_ptr<Column> child;
  // an index derived from this column and a peer column (the triangle
  // count's oriented CSR of (this, peer)), built on first use and kept for
  // the column's lifetime like `stats`: ingest-time work, not per query
  mutable std::shared_ptr<void> index;
  // the direct-address index of a dense unique id column (dense_join.hip)
  mutable std::shared_ptr<void> dense;
  // the var-length reach index of this rel source column (var_length_reach.hip)
  mutable std::shared_ptr<void> vr_index;
  // the membership bitmap of this (unique) key column over [bits_key[0],
  // bits_key[1]] (fused_count.hip message passing)
  mutable std::shared_ptr<void> bits;
  mutable int64_t bits_key[2] = {0, 0};
  mutable std::weak_ptr<Column> index_peer;
  mutable int64_t index_key[2] = {0, 0};
  // provenance of a node-partitioned copy's key column (capf_table_node_partition):
  // every value is a node of [owner[0], owner[0] + owner[1]) owned by part owner[3]
  // of owner[2] — the sharded count then skips its range and ownership tests.
  // owner[3] = −1: no such guarantee.  Kept by compaction (values unchanged).
  int64_t owner[4] = {0, 0, 0, -1};
  bool is_all_null() const { return type == Type::Null; }
};
using ColPtr = std::shared_ptr<Column>;

struct Data {  // a materialised table body
  int64_t nrows = 0;
  std::vector<ColPtr> cols;
};
using DataPtr = std::shared_ptr<Data>;

// ------------------------------------------------------------- expressions
enum Op : int32_t {
  OP_COL = CAPF_OP_COL, OP_LIT_INT = CAPF_OP_LIT_INT, OP_LIT_FLOAT = CAPF_OP_LIT_FLOAT,
  OP_LIT_BOOL = CAPF_OP_LIT_BOOL, OP_LIT_STRING = CAPF_OP_LIT_STRING,
  OP_LIT_NULL = CAPF_OP_LIT_NULL, OP_EQ = CAPF_OP_EQ, OP_NEQ = CAPF_OP_NEQ, OP_LT = CAPF_OP_LT,
  OP_LE = CAPF_OP_LE, OP_GT = CAPF_OP_GT, OP_GE = CAPF_OP_GE, OP_NOT = CAPF_OP_NOT,
  OP_AND = CAPF_OP_AND, OP_OR = CAPF_OP_OR, OP_IS_NULL = CAPF_OP_IS_NULL,
  OP_IS_NOT_NULL = CAPF_OP_IS_NOT_NULL, OP_ADD = CAPF_OP_ADD, OP_SUB = CAPF_OP_SUB,
  OP_MUL = CAPF_OP_MUL, OP_DIV = CAPF_OP_DIV, OP_MOD = CAPF_OP_MOD, OP_NEG = CAPF_OP_NEG,
  OP_TO_FLOAT = CAPF_OP_TO_FLOAT, OP_TO_INTEGER = CAPF_OP_TO_INTEGER,
  OP_COALESCE = CAPF_OP_COALESCE, OP_STR_LEN = CAPF_OP_STR_LEN, OP_LIST_SIZE = CAPF_OP_LIST_SIZE,
  OP_IF = CAPF_OP_IF, OP_ROUND = CAPF_OP_ROUND, OP_ABS = CAPF_OP_ABS, OP_CEIL = CAPF_OP_CEIL,
  OP_FLOOR = CAPF_OP_FLOOR, OP_SIGN = CAPF_OP_SIGN, OP_SQRT = CAPF_OP_SQRT, OP_LOG = CAPF_OP_LOG,
  OP_LOG10 = CAPF_OP_LOG10, OP_EXP = CAPF_OP_EXP, OP_SIN = CAPF_OP_SIN, OP_COS = CAPF_OP_COS,
  OP_TAN = CAPF_OP_TAN, OP_ASIN = CAPF_OP_ASIN, OP_ACOS = CAPF_OP_ACOS, OP_ATAN = CAPF_OP_ATAN,
  OP_DEGREES = CAPF_OP_DEGREES, OP_RADIANS = CAPF_OP_RADIANS, OP_ATAN2 = CAPF_OP_ATAN2,
  OP_TO_BOOLEAN = CAPF_OP_TO_BOOLEAN, OP_IN_SET = CAPF_OP_IN_SET, OP_STR_MAP = CAPF_OP_STR_MAP,
  OP_VALUE_MAP = CAPF_OP_VALUE_MAP, OP_STR_TO_NUM = CAPF_OP_STR_TO_NUM, OP_RAND = CAPF_OP_RAND,
  OP_LIST_INDEX = CAPF_OP_LIST_INDEX, OP_STR_RANK = CAPF_OP_STR_RANK
};
// a program name that refers to a session literal set ("\x01set:<id>"), not a column
inline bool is_literal_set_name(const std::string &nm) { return nm.size() > 5 && nm.compare(0, 5, "\x01set:") == 0; }
// ... or to a session code map of CAPF_OP_STR_MAP ("\x01map:<id>")
inline bool is_code_map_name(const std::string &nm) { return nm.size() > 5 && nm.compare(0, 5, "\x01map:") == 0; }
// ... or to a session value map of CAPF_OP_VALUE_MAP ("\x01vmap:<id>")
inline bool is_value_map_name(const std::string &nm) { return nm.size() > 6 && nm.compare(0, 6, "\x01vmap:") == 0; }
// a program name that is a session table (literal set, code or value map), not a column
inline bool is_session_table_name(const std::string &nm) {
  return is_literal_set_name(nm) || is_code_map_name(nm) || is_value_map_name(nm);
}
// unary math opcodes (one operand, one result)
inline bool is_math1(int32_t op) { return op >= OP_ROUND && op <= OP_RADIANS; }

struct Instr {
  int32_t op;
  int32_t pad;
  int64_t i;
  double f;
};

// An owned copy of a capf_expr with column names kept as strings.
struct Program {
  std::vector<Instr> code;
  std::vector<std::string> names;
  static Program from_c(const capf_expr *e);
  std::vector<std::string> referenced() const;
};

// Device-side view of a column for kernels.
struct ColView {
  const void *data;
  const uint8_t *valid;
  int32_t type;
  int32_t enc;   // ENC_PLAIN / ENC_FOR32 / ENC_FOR24
  int64_t base;  // FOR reference value
};

// 3-byte little-endian offset of row r of a FOR24 buffer.
__host__ __device__ inline uint32_t ld_u24(const void *p, int64_t r) {
  const uint8_t *b = (const uint8_t *)p + 3 * r;
  return (uint32_t)b[0] | (uint32_t)b[1] << 8 | (uint32_t)b[2] << 16;
}

// Integer value of row r of an INT64 / STRING column view (any encoding).
__host__ __device__ inline int64_t ld_int(const ColView &c, int64_t r) {
  return c.enc == ENC_FOR32   ? c.base + (int64_t)((const uint32_t *)c.data)[r]
         : c.enc == ENC_FOR24 ? c.base + (int64_t)ld_u24(c.data, r)
                              : ((const int64_t *)c.data)[r];
}

// A WHERE that is a conjunction of comparisons [NOT] (a op b) — a a column, b
// a column or an integer literal (kernels_basic.hip::ft_compile): evaluated
// without the stack interpreter by filter_select, and per output pair inside
// the radix join's EMIT when it filters the join's output (`side`: the operand
// is a column of the join's left (0) or right (1) input).
constexpr int FT_MAX = 8;
struct FtOperand {
  ColView v;            // the column (or the lazy gather's source)
  const void *idx;      // lazy gather index (int64, or int32 when iw == 4), or null
  int64_t lit;          // literal (v.data == null and lit_ok)
  int32_t is_lit;
  int32_t side;         // join-fused filters: 0 = left input row, 1 = right input row
  int32_t iw;           // idx width in bytes (8 or 4)
  int32_t pad_;
};
struct FtTerm {
  FtOperand a, b;
  int32_t op;   // OP_EQ … OP_GE
  int32_t neg;  // NOT around the comparison
};
struct FtProgram {
  FtTerm t[FT_MAX];
  int32_t nt;
};

// Operand value at row r (false: NULL — a NULL lazy row or an invalid value).
__device__ inline bool ft_load(const FtOperand &o, int64_t r, int64_t &val) {
  if (o.is_lit) {
    val = o.lit;
    return true;
  }
  int64_t row = r;
  if (o.idx) {
    row = o.iw == 4 ? (int64_t)((const int32_t *)o.idx)[r] : ((const int64_t *)o.idx)[r];
    if (row < 0) return false;
  }
  if (o.v.valid && !o.v.valid[row]) return false;
  val = o.v.type == CAPF_TYPE_BOOL ? (((const uint8_t *)o.v.data)[row] ? 1 : 0) : ld_int(o.v, row);
  return true;
}

// ------------------------------------------------------------- plan nodes
enum class Kind {
  Source, Select, Filter, Join, Union, Distinct, Group, WithColumns, OrderBy, Skip, Limit, Explode, NameList,
  ListColumns
};

struct AggSpec {
  int32_t kind;
  bool distinct;
  bool rank_to_code = false;  // min / max of STRINGs: aggregated as ranks, mapped back to codes
  double param = 0;  // percentile fraction (CAPF_AGG_PERCENTILE_*)
  Program arg;  // empty for COUNT_STAR
  std::string name;
  Type out_type;
};

struct Node {
  Session *s;
  Kind kind;
  std::vector<std::string> names;
  std::vector<Type> types;
  std::vector<std::shared_ptr<Node>> kids;
  // Select: source index of each output column
  std::vector<int> sel_index;
  // Filter
  Program pred;
  // Join
  int32_t join_type = CAPF_JOIN_INNER;
  std::vector<std::pair<int, int>> join_keys;  // (left col idx, right col idx)
  // Distinct / Group
  std::vector<int> key_index;
  std::vector<AggSpec> aggs;
  // WithColumns / OrderBy
  std::vector<Program> exprs;
  std::vector<int> target_index;  // WithColumns: output index per expr
  std::vector<int32_t> desc;
  // Skip / Limit
  int64_t count = 0;
  // Explode (UNWIND): a constant list (explode_list_col < 0) or the LIST
  // column explode_list_col of the child; the element column is the last
  // output column
  int explode_list_col = -1;
  ColPtr explode_values;  // the constant list as a column of its elements
  // NameList (labels(n) / keys(n)): the child's columns name_cols, tested per
  // row (kind 0: BOOLEAN TRUE, 1: not NULL), name_codes[j] listed for each hit
  std::vector<int> name_cols;
  std::vector<int32_t> name_kinds;
  std::vector<int64_t> name_codes;
  // ListColumns (a list literal of per-row elements): the child's columns
  // name_cols, row i's list = (col0[i], ..., colk-1[i]) of element type list_elem
  Type list_elem = Type::Null;

  // memoised result
  std::mutex mu;
  DataPtr result;
  // physicalColumns in one call: names joined by '\0' (built on first request)
  std::string joined_names;

  int col_index(const std::string &name) const;  // -1 if absent
  int col_index_or_throw(const std::string &name) const;
};
using NodePtr = std::shared_ptr<Node>;

// ------------------------------------------------------------- session
struct ProfileEntry {
  int64_t launches = 0;
  double total_ms = 0;
  double bytes = 0;
};

struct PendingTiming {
  std::string name;
  double bytes;
  hipEvent_t a, b;
};

// Stream-ordered caching allocator over hipMalloc.  All work of a session is
// issued on its one stream, so a freed block may be handed to the next
// allocation immediately: stream order makes every later use of the block run
// after every earlier one.  (HIP's own stream-ordered pool, hipMallocAsync,
// gave non-deterministic results on this stack under heavy reuse — measured,
// see DESIGN.md.)
struct BlockCache {
  std::multimap<size_t, void *> free_blocks;  // rounded size → block
  std::map<void *, size_t> sizes;             // every block ever allocated
  size_t cached = 0;
  void *get(size_t rounded);
  void put(void *p);
  void release_all();
};

struct Session {
  int device = 0;
  int num_cus = 256;  // compute units of the device (persistent-grid sizing)
  BlockCache cache;
  // buffers handed out by capf_session_alloc (kept alive until capf_session_free)
  std::mutex user_mu;
  std::map<void *, std::shared_ptr<DevBuf>> user_bufs;
  // literal sets of CAPF_OP_IN_SET: sorted unique int64 values on the device
  std::vector<std::pair<std::shared_ptr<DevBuf>, int64_t>> literal_sets;
  // code maps of CAPF_OP_STR_MAP: int64 STRING code per dictionary code (−1 NULL)
  std::vector<std::pair<std::shared_ptr<DevBuf>, int64_t>> code_maps;
  std::vector<int32_t> code_map_refs;  // registrations naming each map (extend in place at 1)
  // value maps of CAPF_OP_VALUE_MAP: [keys n][keys2 n (pairs)][codes n] on the
  // device, n, pair flag
  struct ValueMap {
    std::shared_ptr<DevBuf> buf;
    int64_t n;
    bool pairs;
  };
  std::vector<ValueMap> value_maps;
  // content → id of the code / value maps: a program compiled again over the same
  // dictionary / data re-registers the same map (no device buffer per query)
  std::map<std::vector<int64_t>, int32_t> code_map_ids, value_map_ids;
  std::map<std::vector<int64_t>, int32_t> literal_set_ids;
  std::vector<PendingTiming> pending;   // recorded, not yet resolved
  std::vector<hipEvent_t> event_pool;
  hipEvent_t get_event();
  void resolve_profile();
  hipStream_t stream = nullptr;
  bool own_stream = false;
  bool profiling = false;
  std::map<std::string, ProfileEntry> profile;
  std::string last_plan = "none";
  // string dictionary
  std::mutex str_mu;
  std::vector<std::string> strings;
  std::unordered_map<std::string, int64_t> string_codes;
  // device table of the strings' lengths (CAPF_OP_STR_LEN), grown on demand
  BufPtr d_str_len;
  size_t d_str_len_n = 0;
  // device table of the strings as booleans (CAPF_OP_TO_BOOLEAN): 0 false,
  // 1 true, 2 neither (NULL)
  BufPtr d_str_bool;
  size_t d_str_bool_n = 0;
  // device table of the strings' sort ranks (CAPF_OP_STR_RANK) and its inverse
  BufPtr d_str_rank, d_str_order;
  size_t d_str_rank_n = 0;
  // device table of the strings as numbers (CAPF_OP_STR_TO_NUM)
  BufPtr d_str_num;
  size_t d_str_num_n = 0;
  // small device scratch for scalar results
  int64_t *d_scalars = nullptr;  // 64 slots
  int64_t *h_scalars = nullptr;  // pinned mirror
  // set by capf_table_count_async for the duration of one call: the fused
  // count writes its result to this device int64 and does not wait
  int64_t *async_out = nullptr;

  BufPtr alloc(size_t bytes);
  void sync();
};

// Scoped HIP-event timer around one hot kernel (profiling only).
struct KernelTimer {
  Session *s;
  const char *name;
  double bytes;
  hipEvent_t a = nullptr, b = nullptr;
  KernelTimer(Session *s_, const char *n, double by);
  ~KernelTimer();
};

// ------------------------------------------------------------- helpers
DataPtr materialize(const NodePtr &n);
// One-row INTEGER column holding v (device copy written by a kernel: async,
// no host buffer lifetime) with a host mirror.
ColPtr scalar_i64_column(Session *s, int64_t v);
int64_t node_size(const NodePtr &n);
ColPtr make_column(Session *s, Type t, int64_t n, bool with_valid);
ColPtr null_column(Session *s, Type t, int64_t n);
const ColStats &column_stats(Session *s, const ColPtr &c);
ColView view_of(const ColPtr &c);

// Type inference of a program against a schema (host side).
Type infer_type(const Program &p, const std::vector<std::string> &names,
                const std::vector<Type> &types);

// ---- kernels (implemented in *.hip)
// Evaluate a program over `n` rows; writes a column of type `out_type`.
ColPtr eval_program(Session *s, const Program &p, const std::vector<std::string> &names,
                    const Data &d, Type out_type);
// Predicate → compacted row index list (rows where predicate is TRUE).
BufPtr eval_filter(Session *s, const Program &p, const std::vector<std::string> &names,
                   const Data &d, int64_t *out_count);
// Filter of a table body in one step: the rows passing `p`, its lazy (join
// output) columns composed by the selection kernel itself.
DataPtr filter_select(Session *s, const Program &p, const std::vector<std::string> &names, const Data &d);
// Row index entry i of an index of iw bytes per entry (-1 = NULL row).
__host__ __device__ inline int64_t idx_at(const void *idx, int iw, int64_t i) {
  return iw == 4 ? (int64_t)((const int32_t *)idx)[i] : ((const int64_t *)idx)[i];
}
// Gather rows (int64 indices, -1 = null row) of a column.
ColPtr gather_column(Session *s, const ColPtr &c, const int64_t *d_idx, int64_t n,
                     bool idx_may_be_null = false);
// The same with an index of iw bytes per row (8 = int64, 4 = int32).
ColPtr gather_column_w(Session *s, const ColPtr &c, const void *d_idx, int iw, int64_t n, bool idx_may_be_null);
// Late-materialised gather (LazyGather): rows idx of c, composed with c's own
// index when c is lazy; `cache` shares one composition among the columns of
// a side (keyed by the two index buffers).
struct IdxCache {
  std::vector<std::pair<std::pair<const void *, const void *>, BufPtr>> entries;
};
// iw: bytes per index entry (8, or 4 for a join's int32 pair list).
ColPtr gather_lazy(Session *s, const ColPtr &c, const BufPtr &idx, int64_t n, bool idx_may_be_null,
                   IdxCache *cache, int iw = 8);
// Computes a lazy column in place (no-op otherwise).
void force(const ColPtr &c);
BufPtr iota_index(Session *s, int64_t start, int64_t m);
void cross_index(Session *s, int64_t nl, int64_t nr, BufPtr &li, BufPtr &ri);
// Compact indices of rows whose flag byte is non-zero.
BufPtr compact_flags(Session *s, const uint8_t *d_flags, int64_t n, int64_t *out_count);
// Concatenate columns.
ColPtr concat_columns(Session *s, const ColPtr &a, const ColPtr &b, Type t);
// Exclusive scan of int64 counts; returns total.
int64_t exclusive_scan_i64(Session *s, const int64_t *d_in, int64_t *d_out, int64_t n);
// int64 exclusive scan, the total left in the device int64 d_total (no host sync).
void exclusive_scan_i64_async(Session *s, const int64_t *d_in, int64_t *d_out, int64_t n, int64_t *d_total);
// uint32 exclusive scan (total < 2^32) left on the device, no host sync.
void exclusive_scan_u32_async(Session *s, const uint32_t *d_in, uint32_t *d_out, int64_t n,
                              uint32_t *d_total);
// Hash grouping: group id per row (dense, 0..ngroups-1) and representative row per group.
struct Grouping {
  BufPtr group_of_row;  // int64 [nrows]
  BufPtr rep_row;       // int64 [ngroups]
  int64_t ngroups = 0;
};
Grouping group_rows(Session *s, const Data &d, const std::vector<int> &keys);
// Equi-join of two materialised tables on key columns → (left idx, right idx) pairs.
struct JoinPairs {
  BufPtr left, right;  // int64 [n], -1 for a null-extended side; null = identity (n rows)
  int64_t n = 0;
  int iw = 8;  // bytes per index entry: 4 = int32 (radix join, both sides < 2^31 rows)
  // radix join: the build side's columns in sorted order, indexed by the pairs'
  // build entries (null: those index the build side's own rows)
  std::shared_ptr<Data> build_sorted;
  bool build_is_left = false;
  // inner join whose key values are equal on every output row: 1 = the left
  // key column may be replaced by the right one, 2 = the other way round
  int key_alias = 0;
  // the build side's row index is never read (dense_join: every probe row
  // matches, the build side holds only its key and constant columns): no
  // index for it — 1 = left, 2 = right; its key column is the alias above
  int build_unread = 0;
};
JoinPairs hash_join(Session *s, const Data &l, const Data &r,
                    const std::vector<std::pair<int, int>> &keys, int32_t join_type);
// Direct-address join on a dense unique INTEGER key column (dense_join.hip):
// false when no side qualifies (then radix / hash join).
bool dense_join(Session *s, const Data &l, const Data &r, const std::vector<std::pair<int, int>> &keys,
                int32_t join_type, JoinPairs &out);
// Radix-partitioned equi-join on one key column (radix_join.hip): used for
// large inputs (CAPF_JOIN=radix|hash forces a path).
bool radix_join_applies(const Data &l, const Data &r, const std::vector<std::pair<int, int>> &keys,
                        int32_t join_type);
// A Filter directly over an inner Join that would run as the radix join, whose
// predicate compiles to terms (ft_compile over the join's output columns):
// the join's EMIT evaluates the terms per pair and writes only the passing
// pairs (a count pass, then the write) — no pair list, flags or selection of
// the unfiltered join.  False when the shape does not apply (nothing ran).
bool radix_join_filtered(Session *s, const Program &pred, const std::vector<std::string> &names, const Data &l,
                         const Data &r, const std::vector<std::pair<int, int>> &keys, int32_t join_type,
                         JoinPairs &out);
bool ft_compile(const Program &p, const std::vector<std::string> &names, const Data &d, FtProgram &fp);
bool dense_join_possible(Session *s, const Data &l, const Data &r, const std::vector<std::pair<int, int>> &keys,
                         int32_t join_type);
JoinPairs radix_join(Session *s, const Data &l, const Data &r,
                     const std::vector<std::pair<int, int>> &keys, int32_t join_type,
                     const FtProgram *pred = nullptr);
// Aggregations over a grouping.
ColPtr aggregate(Session *s, const Grouping &g, const Data &d, int64_t nrows, int32_t kind,
                 const ColPtr &arg, Type out_type, double param = 0);
// UNWIND: every row of d repeated per element (explode, kernels_basic.hip)
DataPtr explode_values(Session *s, const Data &d, const ColPtr &values);
// LIST<STRING> column of the names whose column tests true per row (labels / keys, lists.hip)
ColPtr name_list_column(Session *s, const Data &d, const std::vector<int> &cols, const std::vector<int32_t> &kinds,
                        const std::vector<int64_t> &codes);
DataPtr explode_list(Session *s, const Data &d, int list_col);
// LIST column whose row i is (d.cols[cols[0]][i], ..., d.cols[cols[k-1]][i]) (lists.hip)
ColPtr list_from_columns(Session *s, const Data &d, const std::vector<int> &cols, Type elem);
// collect(arg) per group (lists.hip): a Type::List column of g.ngroups lists.
ColPtr collect_lists(Session *s, const Grouping &g, int64_t nrows, const ColPtr &arg,
                     bool distinct);
// Rows d_idx (-1 = NULL list) of a Type::List column.
ColPtr gather_list(Session *s, const ColPtr &c, const int64_t *d_idx, int64_t m);
// Sort permutation (stable) by key columns.
BufPtr sort_permutation(Session *s, const std::vector<ColPtr> &keys,
                        const std::vector<int32_t> &desc, int64_t n);
// Column statistics kernel.
ColStats compute_stats(Session *s, const Column &c);
// m rows of the constant column c's value (c.is_const)
ColPtr const_column(Session *s, const Column &c, int64_t m);
// Frame-of-reference encodings: FOR32 stores an INTEGER column whose value
// range spans < 2^32 as uint32 offsets from `base` (half the HBM bytes).
// encode_column returns the input when the range does not fit.
ColPtr encode_column(Session *s, const ColPtr &c, int width = 4);
ColPtr decode_column(Session *s, const ColPtr &c);

// Device table of the session's string lengths by code (UTF-16 units), for
// CAPF_OP_STR_LEN; *n = strings covered.
const int64_t *string_length_table(Session *s, size_t *n);
// Device table of the session's strings parsed as booleans (CAPF_OP_TO_BOOLEAN).
const uint8_t *string_bool_table(Session *s, size_t *n);
// Device table of each string's rank in UTF-16 code-unit order
// (CAPF_OP_STR_RANK, Java String.compareTo); *n = strings covered.
const int64_t *string_rank_table(Session *s, size_t *n);
// Its inverse: the code of the string of each rank.
const int64_t *string_order_table(Session *s, size_t *n);
// STRING column of the codes of an INTEGER column of ranks (NULLs kept).
ColPtr ranks_to_codes(Session *s, const ColPtr &ranks);
// Device table of the session's strings parsed as numbers (CAPF_OP_STR_TO_NUM):
// [double n][int64 n][uint8 flags n] (bit 0: a DOUBLE, bit 1: an INTEGER).
const void *string_num_table(Session *s, size_t *n);
// Record an error for capf_last_error() (used by entry points outside runtime.cpp).
int32_t record_error(int32_t code, const char *msg);

// Fused counting over lazy inner-join trees (the Expand hot path).
bool try_fused_count(const NodePtr &n, int64_t *out);
// Config 5 below the SPI: Group(a; count(*)) over Distinct(a, b) over the
// UNION ALL of the var-length join chains k = 1..u (fused_count.hip) →
// the (a-keys, reach) rows by multi-source BFS; false: not that shape.
bool try_fused_reach(const NodePtr &grp, DataPtr &out);
// Multi-source BFS reach (var_length_reach.hip): rows (a, #targets reachable
// by a walk of length 1..upper) for every source reaching one; include_self
// (lower bound 0): every source, (a, a) counted once whatever its labels.
DataPtr var_length_reach_rows(Session *s, const ColPtr &rsrc, const ColPtr &rdst, int64_t m,
                              const ColPtr &sid, int64_t ns_in, const ColPtr &tid, int64_t nt, int upper,
                              bool include_self = false);
// Radix-partitioned LDS histograms of the 2-hop count (chain2_partitioned.hip).
// cols = {start(r1), end(r1), start(r2), end(r2)}, all plain or all FOR32.
// Histograms hold chain2_hist_len(hi − lo + 1) counters indexed by
// node_mix(id − lo) (device_common.h) and are fully written (no memset).
// The self-loop count is added to *d_loops (device memory): no host round trip.
// in_range: the columns' statistics put every id inside [lo, hi].
int chain2_hist_bits(int64_t len);
int64_t chain2_hist_len(int64_t len);
__global__ void k_partial_minus_loops(const unsigned long long *acc, int64_t *out);
// Node-partitioned multi-GPU layout (chain2_partitioned.hip)
uint8_t *node_owner_flags(Session *s, const ColView &key, int64_t n, int64_t lo, int64_t n_nodes,
                          int parts, int part, BufPtr &keep);
BufPtr node_partition_diag_index(Session *s, const ColView &src, const ColView &dst, int64_t n, int64_t lo,
                                 int64_t n_nodes, int parts, int part, int64_t *m, int64_t *n_diag);
// n_diag ≥ 0: only out-copy rows [0, n_diag) can be self-loops (2-D layout); −1: any row
// nhot / hot_ids: heavy-hitter node ids (a sampled plan hint; any ids are correct)
bool chain2_sharded(Session *s, const ColView *cols, int64_t n_in, int64_t n_out, int64_t lo,
                    int64_t n_nodes, int parts, int part, int64_t *d_partial, int64_t n_diag = -1,
                    int nhot = 0, const int64_t *hot_ids = nullptr, bool trusted = false);
// Exchange wire format (shuffle.hip): cols packed row-major, `width` bytes of
// (value − base) per column + a validity byte where nullable; *W = row bytes.
void pack_rows(Session *s, const std::vector<ColPtr> &cols, const int32_t *width, const int64_t *base,
               const int32_t *nullable, int64_t n, int *W, void *d_out);
ColPtr unpack_column(Session *s, const void *rows, int64_t n, int W, int off, int width, int voff, int64_t base,
                     Type t);
// Rows of `keys` (n rows) grouped by owner h(key tuple) of `parts` (shuffle.hip):
// the permutation (int64 row indexes) and the row count per owner.
BufPtr route_permutation(Session *s, const std::vector<ColView> &keys, int64_t n, int parts,
                         std::vector<int64_t> &counts);
// Σ_rows bit[key − lo] of a membership bitmap over [lo, hi] into *d_acc,
// radix-partitioned (chain2_partitioned.hip); `mixed_cache` holds the bitmap in
// node_mix order (built when empty).  false: shape not handled, nothing launched.
bool bits_count_partitioned(Session *s, const ColView &key, int64_t n, int64_t lo, int64_t hi,
                            const uint32_t *bits, BufPtr &mixed_cache, unsigned long long *d_acc);
// Directed triangle count (triangle.hip), part `part` of `parts`, to device int64.
// The oriented CSR is cached on `src` (Column::index) for the pair (src, dst).
void triangle_count_async(Session *s, const ColPtr &src, const ColPtr &dst, int64_t m,
                          int64_t lo, uint64_t len, int parts, int part, int64_t *d_out);
// Hand-offs of the partitioned 2-hop histograms (P3's uint16 counters hand
// 2^15 off when a hub's counter fills): (hist index, side | count << 1)
// entries, hist index mod hl = the counter; the dot kernel adds their terms
// (a few dozen entries at R-MAT s24) instead of a separate overflow kernel.
struct C2Spill {
  const uint2 *log = nullptr;
  const uint32_t *n = nullptr;
  uint32_t cap = 0;
  int64_t hl = 0;
  // non-null: bucket layout per run (runs [0, nb) in, [nb, 2·nb) out): split[r] = 0 →
  // packed uint16 pairs in the first 2^15 words of the bucket (word i: bin i low,
  // bin i + 2^15 high), 1 → one uint32 per bin
  const int32_t *split = nullptr;
  int nb = 0;
  // host side: where the count goes (the pinned scalar or the async slot)
  int64_t *fin = nullptr;
  // non-null: P1's per-tile self-loop counts, summed into acc[1] by the dot
  // (the pipeline without a transpose kernel)
  const uint32_t *tile_loops = nullptr;
  int64_t ntiles = 0;
};
// d_acc3 = [Σ in·out, self-loops, done counter] (device): the pipeline writes
// the self-loop total into [1] and clears [0] and [2] itself (no memset needed)
// spill: non-null → the hand-off log is left for the dot kernel (no separate
// overflow kernel); null → the overflow kernel runs.
bool chain2_partitioned(Session *s, const ColView *cols, int64_t n, int64_t lo, int64_t hi,
                        bool in_range, uint32_t *h_in, uint32_t *h_out,
                        unsigned long long *d_acc3, C2Spill *spill = nullptr);

}  // namespace capf

// opaque handle given to C callers
struct capf_table {
  capf::NodePtr node;
};
struct capf_session {
  capf::Session impl;
};
