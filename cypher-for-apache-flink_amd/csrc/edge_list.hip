// edge_list.hip — CSV edge-list ingest straight into HBM.
//
// EdgeListDataSource.graph (flink-cypher/.../api/io/edgelist/EdgeListDataSource.scala:61-81)
// reads a CSV through Flink's CsvTableSource with two LONG fields
// (sourceStartNodeKey, sourceEndNodeKey), a field delimiter and a comment
// prefix (:62-68), then gives every row a unique LONG id with
// `safeAddIdColumn` = DataSet.zipWithUniqueId (flink-cypher/.../impl/TableOps.scala:217-238).
// Here the raw bytes are copied to the device once and parsed there:
//
//   K1 k_el_count  per 16 KiB chunk (1024 threads × 16 B): '\n' count
//   (scan)         chunk → first line index (int64 exclusive scan)
//   K2 k_el_parse  per chunk: the chunk staged in LDS, its newline offsets
//                  found by a block scan, then one thread per line ending in
//                  the chunk parses (start, end) into the line's slot
//   compaction     only when comment lines were skipped
//
// Row semantics follow Flink 1.7's CsvInputFormat / LongParser: a trailing
// '\r' is stripped (line delimiter '\n'); a line starting with the comment
// prefix is skipped; each LONG field is an optional '-' and decimal digits
// up to the (possibly multi-byte) field delimiter; an empty field, any other
// byte (whitespace included), an orphan sign, an int64 overflow or a line
// with fewer than two fields fails the whole read (Flink raises a
// ParseException in the job); text after the second field is not read
// (only two fields are declared).  Rel ids are the data-line ordinals
// 0..M-1: one valid zipWithUniqueId assignment (Flink's ids are unique but
// depend on the task parallelism, so only uniqueness is specified).
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <system_error>
#include <thread>
#include <vector>

#include "capf_internal.h"
#include "device_common.h"

namespace capf {

constexpr int EL_BLOCK = 1024;
constexpr int EL_CHUNK = 16 * EL_BLOCK;  // bytes per workgroup
constexpr int EL_MAX_DELIM = 8;          // field delimiter / comment prefix bytes

enum : uint32_t {
  EL_OK = 0, EL_TOO_SHORT = 1, EL_EMPTY = 2, EL_ILLEGAL_CHAR = 3, EL_OVERFLOW = 4, EL_ORPHAN_SIGN = 5
};

struct ElSpec {
  uint8_t sep[EL_MAX_DELIM];
  uint8_t comment[EL_MAX_DELIM];
  int sep_len, comment_len;
};

// 16-bit mask of the '\n' bytes of a 16-B piece (bit i = byte i).
__device__ inline uint32_t el_newlines(uint4 q) {
  const uint32_t w[4] = {q.x, q.y, q.z, q.w};
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t x = w[k] ^ 0x0A0A0A0Au;
    // exact zero-byte detector (no borrow between bytes): 0x80 per zero byte
    const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
#pragma unroll
    for (int b = 0; b < 4; ++b) m |= ((z >> (8 * b + 7)) & 1u) << (4 * k + b);
  }
  return m;
}

__global__ __launch_bounds__(EL_BLOCK) void k_el_count(const uint4 *text, int64_t *chunk_nl) {
  __shared__ int64_t lds[17];
  const uint4 q = text[(int64_t)blockIdx.x * EL_BLOCK + threadIdx.x];
  const int64_t c = __popc(el_newlines(q));
  const int64_t tot = block_reduce_sum(c, lds);
  if (threadIdx.x == 0) chunk_nl[blockIdx.x] = tot;
}

// Byte at absolute position p.  ElLds: lines inside the staged chunk (the
// common case — the accessor indexes the __shared__ stage directly, so the
// loads are ds_read_u8, not flat loads); ElAny: the first line of a chunk,
// which may start in an earlier chunk (HBM below c0).
struct ElLds {
  const uint8_t *lds;
  int64_t c0;
  __device__ uint8_t operator[](int64_t p) const { return lds[p - c0]; }
};
struct ElAny {
  const uint8_t *g;
  const uint8_t *lds;
  int64_t c0;
  __device__ uint8_t operator[](int64_t p) const { return p >= c0 ? lds[p - c0] : g[p]; }
};

template <int SEP1, class B>
__device__ inline bool el_delim_at(const B &b, int64_t p, int64_t end, const ElSpec &sp) {
  if (SEP1) return p < end && b[p] == sp.sep[0];
  if (p + sp.sep_len > end) return false;
  for (int i = 0; i < sp.sep_len; ++i)
    if (b[p + i] != sp.sep[i]) return false;
  return true;
}

// LongParser.parseField: [p, end) up to the delimiter → value; *p advances
// to the delimiter (or end).  Returns an EL_* code.
template <int SEP1, class B>
__device__ inline uint32_t el_parse_long(const B &b, int64_t &p, int64_t end, const ElSpec &sp,
                                         int64_t &out) {
  if (p >= end || el_delim_at<SEP1>(b, p, end, sp)) return EL_EMPTY;
  bool neg = false;
  if (b[p] == '-') {
    neg = true;
    ++p;
    if (p >= end || el_delim_at<SEP1>(b, p, end, sp)) return EL_ORPHAN_SIGN;
  }
  const uint64_t limit = neg ? 9223372036854775808ull : 9223372036854775807ull;
  uint64_t mag = 0;
  for (; p < end; ++p) {
    const uint8_t ch = b[p];
    if (SEP1 ? ch == sp.sep[0] : el_delim_at<SEP1>(b, p, end, sp)) break;
    const uint32_t d = (uint32_t)ch - '0';
    if (d > 9) return EL_ILLEGAL_CHAR;
    if (mag > (limit - d) / 10) return EL_OVERFLOW;
    mag = mag * 10 + d;
  }
  out = neg ? (int64_t)(0ull - mag) : (int64_t)mag;
  return EL_OK;
}

// One line [start, end): comment test, two LONG fields.
template <int SEP1, class B>
__device__ inline uint32_t el_line(const B &by, int64_t start, int64_t end, const ElSpec &sp,
                                   bool &comment, int64_t &s, int64_t &d) {
  if (end > start && by[end - 1] == '\r') --end;
  comment = sp.comment_len > 0 && end - start >= sp.comment_len;
  for (int i = 0; comment && i < sp.comment_len; ++i) comment = by[start + i] == sp.comment[i];
  s = d = 0;
  if (comment) return EL_OK;
  int64_t p = start;
  uint32_t code = el_parse_long<SEP1>(by, p, end, sp, s);
  if (code != EL_OK) return code;
  if (p >= end) return EL_TOO_SHORT;  // no delimiter before the end of the line
  p += sp.sep_len;
  return p >= end ? EL_TOO_SHORT : el_parse_long<SEP1>(by, p, end, sp, d);
}

template <int SEP1>
__global__ __launch_bounds__(EL_BLOCK) void k_el_parse(const uint4 *text, int64_t n,
                                                       const int64_t *chunk_off, int64_t nchunks,
                                                       int64_t nlines, ElSpec sp, int64_t *src,
                                                       int64_t *dst, uint8_t *keep,
                                                       unsigned long long *err,
                                                       unsigned long long *kept) {
  __shared__ uint4 stage[EL_BLOCK];
  __shared__ uint16_t nlp[EL_CHUNK];
  __shared__ uint32_t lds_scan[17];
  __shared__ unsigned long long lds_kept[17];
  const int64_t b = blockIdx.x, c0 = b * EL_CHUNK;
  const uint4 q = text[b * EL_BLOCK + threadIdx.x];
  stage[threadIdx.x] = q;
  uint32_t m = el_newlines(q), cnt;
  uint32_t idx = block_exclusive_scan((uint32_t)__popc(m), lds_scan, cnt);
  while (m) {
    const int i = __ffs(m) - 1;
    m &= m - 1;
    nlp[idx++] = (uint16_t)(16 * threadIdx.x + i);
  }
  __syncthreads();
  const ElLds fast{(const uint8_t *)stage, c0};
  const int64_t l0 = chunk_off[b];
  // lines ending in this chunk: k < cnt end at a '\n'; the last chunk also
  // owns the unterminated last line (its slot is nlines − 1)
  const bool tail = b == nchunks - 1 && l0 + cnt < nlines;
  const uint32_t items = cnt + (tail ? 1u : 0u);
  unsigned long long mine = 0;
  for (uint32_t k = threadIdx.x; k < items; k += EL_BLOCK) {
    const int64_t gl = l0 + k;
    const int64_t end = k < cnt ? c0 + nlp[k] : n;
    bool comment;
    int64_t s, d;
    uint32_t code;
    if (k > 0) {
      code = el_line<SEP1>(fast, c0 + nlp[k - 1] + 1, end, sp, comment, s, d);
    } else {  // walk back to the previous '\n' (in an earlier chunk)
      const ElAny any{(const uint8_t *)text, (const uint8_t *)stage, c0};
      int64_t start = c0;
      while (start > 0 && any[start - 1] != '\n') --start;
      code = el_line<SEP1>(any, start, end, sp, comment, s, d);
    }
    if (code != EL_OK) atomicMin(err, ((unsigned long long)gl << 8) | code);
    mine += comment ? 0 : 1;
    src[gl] = s;
    dst[gl] = d;
    keep[gl] = comment ? 0 : 1;
  }
  const unsigned long long tot = block_reduce_sum(mine, lds_kept);
  if (threadIdx.x == 0 && tot) atomicAdd(kept, tot);
}

// ------------------------------------------------ K LONG fields per line
// The node / relationship tables of an FS graph source whose declared fields
// are all LONG (FSGraphSource.readFromCsv, FSGraphSource.scala:80-84: a
// CsvTableSource with the canonical field list — id, source, target and
// INTEGER properties, CAPFGraphExport.scala canonical*FieldReference) parse
// with the same row rules, one output column per declared field.
constexpr int CSV_MAXK = 16;
struct CsvOut {
  int64_t *col[CSV_MAXK];
  int k;
};

template <int SEP1, class B>
__device__ inline uint32_t csv_line(const B &by, int64_t start, int64_t end, const ElSpec &sp,
                                    bool &comment, const CsvOut &o, int64_t gl) {
  if (end > start && by[end - 1] == '\r') --end;
  comment = sp.comment_len > 0 && end - start >= sp.comment_len;
  for (int i = 0; comment && i < sp.comment_len; ++i) comment = by[start + i] == sp.comment[i];
  if (comment) {
    for (int f = 0; f < o.k; ++f) o.col[f][gl] = 0;
    return EL_OK;
  }
  int64_t p = start;
  for (int f = 0; f < o.k; ++f) {
    if (f > 0) {
      if (p >= end) return EL_TOO_SHORT;  // no delimiter before the end of the line
      p += sp.sep_len;
      if (p >= end) return EL_TOO_SHORT;
    }
    int64_t v = 0;
    const uint32_t code = el_parse_long<SEP1>(by, p, end, sp, v);
    if (code != EL_OK) return code;
    o.col[f][gl] = v;
  }
  return EL_OK;
}

template <int SEP1>
__global__ __launch_bounds__(EL_BLOCK) void k_csv_parse(const uint4 *text, int64_t n,
                                                        const int64_t *chunk_off, int64_t nchunks,
                                                        int64_t nlines, ElSpec sp, CsvOut o,
                                                        uint8_t *keep, unsigned long long *err,
                                                        unsigned long long *kept) {
  __shared__ uint4 stage[EL_BLOCK];
  __shared__ uint16_t nlp[EL_CHUNK];
  __shared__ uint32_t lds_scan[17];
  __shared__ unsigned long long lds_kept[17];
  const int64_t b = blockIdx.x, c0 = b * EL_CHUNK;
  const uint4 q = text[b * EL_BLOCK + threadIdx.x];
  stage[threadIdx.x] = q;
  uint32_t m = el_newlines(q), cnt;
  uint32_t idx = block_exclusive_scan((uint32_t)__popc(m), lds_scan, cnt);
  while (m) {
    const int i = __ffs(m) - 1;
    m &= m - 1;
    nlp[idx++] = (uint16_t)(16 * threadIdx.x + i);
  }
  __syncthreads();
  const ElLds fast{(const uint8_t *)stage, c0};
  const int64_t l0 = chunk_off[b];
  const bool tail = b == nchunks - 1 && l0 + cnt < nlines;
  const uint32_t items = cnt + (tail ? 1u : 0u);
  unsigned long long mine = 0;
  for (uint32_t k = threadIdx.x; k < items; k += EL_BLOCK) {
    const int64_t gl = l0 + k;
    const int64_t end = k < cnt ? c0 + nlp[k] : n;
    bool comment;
    uint32_t code;
    if (k > 0) {
      code = csv_line<SEP1>(fast, c0 + nlp[k - 1] + 1, end, sp, comment, o, gl);
    } else {
      const ElAny any{(const uint8_t *)text, (const uint8_t *)stage, c0};
      int64_t start = c0;
      while (start > 0 && any[start - 1] != '\n') --start;
      code = csv_line<SEP1>(any, start, end, sp, comment, o, gl);
    }
    if (code != EL_OK) atomicMin(err, ((unsigned long long)gl << 8) | code);
    mine += comment ? 0 : 1;
    keep[gl] = comment ? 0 : 1;
  }
  const unsigned long long tot = block_reduce_sum(mine, lds_kept);
  if (threadIdx.x == 0 && tot) atomicAdd(kept, tot);
}

static const char *el_reason(uint32_t code) {
  switch (code) {
    case EL_TOO_SHORT: return "Row too short (fewer fields than declared)";
    case EL_EMPTY: return "empty LONG field";
    case EL_ILLEGAL_CHAR: return "illegal character in a LONG field";
    case EL_OVERFLOW: return "LONG value out of range";
    case EL_ORPHAN_SIGN: return "orphan sign in a LONG field";
    default: return "unknown parse error";
  }
}

// Parses `nbytes` host bytes into (id, source, target) INT64 columns.
// Parses the device copy `text` (nbytes, zero-padded to whole chunks) into
// (id, source, target) INT64 columns.  last = the file's last byte.
static DataPtr edge_list_parse_device(Session *s, const BufPtr &text, int64_t nbytes, char last,
                                      const ElSpec &sp) {
  auto d = std::make_shared<Data>();
  for (int i = 0; i < 3; ++i) d->cols.push_back(make_column(s, Type::Int64, 0, false));
  if (nbytes == 0) return d;
  const int64_t nchunks = (nbytes + EL_CHUNK - 1) / EL_CHUNK;
  BufPtr cnt = s->alloc(8 * nchunks), off = s->alloc(8 * nchunks);
  {
    KernelTimer kt(s, "el_count", (double)nchunks * EL_CHUNK);
    hipLaunchKernelGGL(k_el_count, dim3((unsigned)nchunks), dim3(EL_BLOCK), 0, s->stream,
                       (const uint4 *)text->p, (int64_t *)cnt->p);
    KERNEL_CHECK();
  }
  const int64_t nl = exclusive_scan_i64(s, (const int64_t *)cnt->p, (int64_t *)off->p, nchunks);
  const int64_t nlines = nl + (last != '\n' ? 1 : 0);
  ColPtr src = make_column(s, Type::Int64, nlines, false);
  ColPtr dst = make_column(s, Type::Int64, nlines, false);
  BufPtr keep = s->alloc(std::max<int64_t>(nlines, 1));
  BufPtr flags = s->alloc(16);
  unsigned long long *d_err = (unsigned long long *)flags->p, *d_kept = d_err + 1;
  const unsigned long long init[2] = {~0ull, 0ull};
  HIP_CHECK(hipMemcpyAsync(d_err, init, 16, hipMemcpyHostToDevice, s->stream));
  if (nlines > 0) {
    KernelTimer kt(s, "el_parse", (double)nchunks * EL_CHUNK + 17.0 * nlines);
    hipLaunchKernelGGL(sp.sep_len == 1 ? k_el_parse<1> : k_el_parse<0>, dim3((unsigned)nchunks),
                       dim3(EL_BLOCK), 0, s->stream,
                       (const uint4 *)text->p, nbytes, (const int64_t *)off->p, nchunks, nlines, sp,
                       (int64_t *)src->data->p, (int64_t *)dst->data->p, (uint8_t *)keep->p, d_err,
                       d_kept);
    KERNEL_CHECK();
  }
  unsigned long long h[2];
  HIP_CHECK(hipMemcpyAsync(h, d_err, 16, hipMemcpyDeviceToHost, s->stream));
  s->sync();
  if (h[0] != ~0ull) {
    const int64_t line = (int64_t)(h[0] >> 8);
    char msg[160];
    snprintf(msg, sizeof msg, "edge list line %lld could not be parsed: %s",
             (long long)line + 1, el_reason((uint32_t)(h[0] & 0xFF)));
    illegal(msg);
  }
  const int64_t m = (int64_t)h[1];
  if (m != nlines) {  // comment lines: compact the data lines
    int64_t got = 0;
    BufPtr idx = compact_flags(s, (const uint8_t *)keep->p, nlines, &got);
    if (got != m) fail(CAPF_ERR_INTERNAL, "edge list: kept-line count mismatch");
    src = gather_column(s, src, (const int64_t *)idx->p, m);
    dst = gather_column(s, dst, (const int64_t *)idx->p, m);
  }
  auto id = std::make_shared<Column>();
  id->type = Type::Int64;
  id->n = m;
  if (m > 0) id->data = iota_index(s, 0, m);
  d->nrows = m;
  d->cols = {id, src, dst};
  s->sync();
  return d;
}

// Parses the device copy `text` into K INT64 columns (one per declared field).
static DataPtr csv_longs_parse_device(Session *s, const BufPtr &text, int64_t nbytes, char last,
                                      const ElSpec &sp, int k) {
  auto d = std::make_shared<Data>();
  for (int i = 0; i < k; ++i) d->cols.push_back(make_column(s, Type::Int64, 0, false));
  if (nbytes == 0) return d;
  const int64_t nchunks = (nbytes + EL_CHUNK - 1) / EL_CHUNK;
  BufPtr cnt = s->alloc(8 * nchunks), off = s->alloc(8 * nchunks);
  {
    KernelTimer kt(s, "el_count", (double)nchunks * EL_CHUNK);
    hipLaunchKernelGGL(k_el_count, dim3((unsigned)nchunks), dim3(EL_BLOCK), 0, s->stream,
                       (const uint4 *)text->p, (int64_t *)cnt->p);
    KERNEL_CHECK();
  }
  const int64_t nl = exclusive_scan_i64(s, (const int64_t *)cnt->p, (int64_t *)off->p, nchunks);
  const int64_t nlines = nl + (last != '\n' ? 1 : 0);
  std::vector<ColPtr> cols;
  CsvOut o{};
  o.k = k;
  for (int i = 0; i < k; ++i) {
    cols.push_back(make_column(s, Type::Int64, nlines, false));
    o.col[i] = nlines > 0 ? (int64_t *)cols[i]->data->p : nullptr;
  }
  BufPtr keep = s->alloc(std::max<int64_t>(nlines, 1));
  BufPtr flags = s->alloc(16);
  unsigned long long *d_err = (unsigned long long *)flags->p, *d_kept = d_err + 1;
  const unsigned long long init[2] = {~0ull, 0ull};
  HIP_CHECK(hipMemcpyAsync(d_err, init, 16, hipMemcpyHostToDevice, s->stream));
  if (nlines > 0) {
    KernelTimer kt(s, "csv_parse", (double)nchunks * EL_CHUNK + 8.0 * k * nlines);
    hipLaunchKernelGGL(sp.sep_len == 1 ? k_csv_parse<1> : k_csv_parse<0>, dim3((unsigned)nchunks),
                       dim3(EL_BLOCK), 0, s->stream, (const uint4 *)text->p, nbytes, (const int64_t *)off->p,
                       nchunks, nlines, sp, o, (uint8_t *)keep->p, d_err, d_kept);
    KERNEL_CHECK();
  }
  unsigned long long h[2];
  HIP_CHECK(hipMemcpyAsync(h, d_err, 16, hipMemcpyDeviceToHost, s->stream));
  s->sync();
  if (h[0] != ~0ull) {
    char msg[160];
    snprintf(msg, sizeof msg, "CSV line %lld could not be parsed: %s", (long long)(h[0] >> 8) + 1,
             el_reason((uint32_t)(h[0] & 0xFF)));
    illegal(msg);
  }
  const int64_t m = (int64_t)h[1];
  if (m != nlines) {  // comment lines
    int64_t got = 0;
    BufPtr idx = compact_flags(s, (const uint8_t *)keep->p, nlines, &got);
    if (got != m) fail(CAPF_ERR_INTERNAL, "csv: kept-line count mismatch");
    for (auto &c : cols) c = gather_column(s, c, (const int64_t *)idx->p, m);
  }
  d->nrows = m;
  d->cols = cols;
  s->sync();
  return d;
}

static BufPtr el_text_buffer(Session *s, int64_t nbytes) {
  const int64_t nchunks = (nbytes + EL_CHUNK - 1) / EL_CHUNK;
  BufPtr text = s->alloc(std::max<int64_t>(nchunks, 1) * EL_CHUNK);
  if (nchunks * EL_CHUNK > nbytes)  // zero padding: never a '\n'
    HIP_CHECK(hipMemsetAsync((char *)text->p + nbytes, 0, nchunks * EL_CHUNK - nbytes, s->stream));
  return text;
}

static DataPtr edge_list_parse(Session *s, const char *bytes, int64_t nbytes, const ElSpec &sp) {
  BufPtr text = el_text_buffer(s, nbytes);
  if (nbytes > 0)
    HIP_CHECK(hipMemcpyAsync(text->p, bytes, nbytes, hipMemcpyHostToDevice, s->stream));
  return edge_list_parse_device(s, text, nbytes, nbytes > 0 ? bytes[nbytes - 1] : '\n', sp);
}

// File → HBM: 64 MiB pieces read by parallel pread()s into two pinned staging
// buffers, each DMA'd while the next piece is read (no whole-file pinning).
constexpr int64_t EL_PIECE = 64ll << 20;
constexpr int EL_READERS = 8;

// File → device text buffer (zero-padded to whole chunks); *len_out / *last_out
// = the file's size and last byte.
static BufPtr read_text_file(Session *s, const char *path, int64_t *len_out, char *last_out) {
  const int fd = open(path, O_RDONLY);
  if (fd < 0) illegal(std::string("cannot open ") + path);
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    illegal(std::string("cannot stat ") + path);
  }
  const int64_t len = (int64_t)st.st_size;
  char *stage[2] = {nullptr, nullptr};
  hipEvent_t done[2] = {nullptr, nullptr};
  auto cleanup = [&]() {
    for (int b = 0; b < 2; ++b) {
      if (done[b]) (void)hipEventDestroy(done[b]);
      if (stage[b]) (void)hipHostFree(stage[b]);
    }
    close(fd);
  };
  try {
    BufPtr text = el_text_buffer(s, len);
    const int64_t piece = std::min<int64_t>(EL_PIECE, std::max<int64_t>(len, 1));
    for (int b = 0; b < 2; ++b) {
      HIP_CHECK(hipHostMalloc((void **)&stage[b], (size_t)piece, hipHostMallocDefault));
      HIP_CHECK(hipEventCreateWithFlags(&done[b], hipEventDisableTiming));
    }
    char last = '\n';
    for (int64_t off = 0, i = 0; off < len; off += piece, ++i) {
      const int b = (int)(i & 1);
      const int64_t n = std::min(piece, len - off);
      HIP_CHECK(hipEventSynchronize(done[b]));  // the DMA that last used this buffer
      std::atomic<bool> bad{false};
      std::vector<std::thread> rd;
      const int64_t part = (n + EL_READERS - 1) / EL_READERS;
      auto read_range = [&, b, off](int64_t lo, int64_t hi) {
        for (int64_t p = lo; p < hi;) {
          const ssize_t r = pread(fd, stage[b] + p, (size_t)(hi - p), (off_t)(off + p));
          if (r <= 0) {
            bad = true;
            return;
          }
          p += r;
        }
      };
      try {
        for (int t = 0; t < EL_READERS; ++t) {
          const int64_t lo = t * part, hi = std::min(n, lo + part);
          if (lo >= hi) break;
          rd.emplace_back(read_range, lo, hi);
        }
      } catch (const std::system_error &) {
        // a reader thread could not be started: the ones that were started
        // are joined below; the remaining ranges are read on this thread
        const int64_t done_to = (int64_t)rd.size() * part;
        read_range(done_to, n);
      }
      for (auto &th : rd) th.join();
      if (bad) illegal(std::string("short read of ") + path);
      last = stage[b][n - 1];
      HIP_CHECK(hipMemcpyAsync((char *)text->p + off, stage[b], (size_t)n, hipMemcpyHostToDevice,
                               s->stream));
      HIP_CHECK(hipEventRecord(done[b], s->stream));
    }
    s->sync();
    cleanup();
    *len_out = len;
    *last_out = last;
    return text;
  } catch (...) {
    s->sync();
    cleanup();
    throw;
  }
}

static DataPtr edge_list_read_file(Session *s, const char *path, const ElSpec &sp) {
  int64_t len = 0;
  char last = '\n';
  BufPtr text = read_text_file(s, path, &len, &last);
  return edge_list_parse_device(s, text, len, last, sp);  // syncs the stream
}

static ElSpec el_spec(const char *sep, const char *comment) {
  ElSpec sp{};
  if (!sep || !*sep) illegal("edge list: the field delimiter (option `sep`) must be non-empty");
  sp.sep_len = (int)strlen(sep);
  sp.comment_len = comment ? (int)strlen(comment) : 0;
  if (sp.sep_len > EL_MAX_DELIM || sp.comment_len > EL_MAX_DELIM)
    illegal("edge list: delimiter / comment prefix longer than 8 bytes");
  if (strchr(sep, '\n') || (comment && strchr(comment, '\n')))
    illegal("edge list: delimiter / comment prefix must not contain the line delimiter");
  memcpy(sp.sep, sep, sp.sep_len);
  if (sp.comment_len) memcpy(sp.comment, comment, sp.comment_len);
  return sp;
}

static capf_table *edge_list_table(Session *s, DataPtr d, const char *id_col, const char *src_col,
                                   const char *dst_col) {
  auto n = std::make_shared<Node>();
  n->s = s;
  n->kind = Kind::Source;
  n->names = {id_col, src_col, dst_col};
  n->types = {Type::Int64, Type::Int64, Type::Int64};
  n->result = d;
  auto *t = new capf_table;
  t->node = n;
  return t;
}

}  // namespace capf

using namespace capf;

extern "C" capf_status capf_edge_list_parse(capf_session *cs, const char *bytes, int64_t nbytes,
                                            const char *sep, const char *comment,
                                            const char *id_col, const char *src_col,
                                            const char *dst_col, capf_table **out) {
  try {
    if (!cs || !out || !id_col || !src_col || !dst_col || (nbytes > 0 && !bytes))
      illegal("null argument");
    if (nbytes < 0) illegal("negative byte count");
    const ElSpec sp = el_spec(sep, comment);
    Session *s = &cs->impl;
    *out = edge_list_table(s, edge_list_parse(s, bytes, nbytes, sp), id_col, src_col, dst_col);
    return CAPF_OK;
  } catch (const capf::Error &e) {
    return record_error(e.code, e.what());
  } catch (const std::exception &e) {  // bad_alloc, system_error, … never cross the C-ABI
    return record_error(CAPF_ERR_INTERNAL, e.what());
  }
}

extern "C" capf_status capf_edge_list_read(capf_session *cs, const char *path, const char *sep,
                                           const char *comment, const char *id_col,
                                           const char *src_col, const char *dst_col,
                                           capf_table **out) {
  try {
    if (!cs || !out || !path || !id_col || !src_col || !dst_col) illegal("null argument");
    const ElSpec sp = el_spec(sep, comment);
    Session *s = &cs->impl;
    DataPtr d = edge_list_read_file(s, path, sp);
    *out = edge_list_table(s, d, id_col, src_col, dst_col);
    return CAPF_OK;
  } catch (const capf::Error &e) {
    return record_error(e.code, e.what());
  } catch (const std::exception &e) {  // bad_alloc, system_error, … never cross the C-ABI
    return record_error(CAPF_ERR_INTERNAL, e.what());
  }
}

static capf_table *csv_table(Session *s, DataPtr d, int32_t ncols, const char *const *names) {
  auto n = std::make_shared<Node>();
  n->s = s;
  n->kind = Kind::Source;
  for (int i = 0; i < ncols; ++i) {
    n->names.emplace_back(names[i]);
    n->types.push_back(Type::Int64);
  }
  n->result = d;
  auto *t = new capf_table;
  t->node = n;
  return t;
}

static void csv_args(capf_session *cs, int32_t ncols, const char *const *names, capf_table **out) {
  if (!cs || !out || !names) illegal("null argument");
  if (ncols < 1 || ncols > CSV_MAXK) illegal("CSV: 1..16 LONG fields");
  for (int i = 0; i < ncols; ++i)
    if (!names[i]) illegal("null column name");
}

extern "C" capf_status capf_csv_parse_longs(capf_session *cs, const char *bytes, int64_t nbytes,
                                            const char *sep, int32_t ncols, const char *const *names,
                                            capf_table **out) {
  try {
    csv_args(cs, ncols, names, out);
    if (nbytes < 0 || (nbytes > 0 && !bytes)) illegal("bad byte buffer");
    const ElSpec sp = el_spec(sep, nullptr);
    Session *s = &cs->impl;
    BufPtr text = el_text_buffer(s, nbytes);
    if (nbytes > 0) HIP_CHECK(hipMemcpyAsync(text->p, bytes, nbytes, hipMemcpyHostToDevice, s->stream));
    DataPtr d = csv_longs_parse_device(s, text, nbytes, nbytes > 0 ? bytes[nbytes - 1] : '\n', sp, ncols);
    *out = csv_table(s, d, ncols, names);
    return CAPF_OK;
  } catch (const capf::Error &e) {
    return record_error(e.code, e.what());
  } catch (const std::exception &e) {
    return record_error(CAPF_ERR_INTERNAL, e.what());
  }
}

extern "C" capf_status capf_csv_read_longs(capf_session *cs, const char *path, const char *sep,
                                           int32_t ncols, const char *const *names, capf_table **out) {
  try {
    csv_args(cs, ncols, names, out);
    if (!path) illegal("null argument");
    const ElSpec sp = el_spec(sep, nullptr);
    Session *s = &cs->impl;
    int64_t len = 0;
    char last = '\n';
    BufPtr text = read_text_file(s, path, &len, &last);
    DataPtr d = csv_longs_parse_device(s, text, len, last, sp, ncols);
    *out = csv_table(s, d, ncols, names);
    return CAPF_OK;
  } catch (const capf::Error &e) {
    return record_error(e.code, e.what());
  } catch (const std::exception &e) {
    return record_error(CAPF_ERR_INTERNAL, e.what());
  }
}
