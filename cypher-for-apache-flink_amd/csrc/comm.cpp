// comm.cpp — the rank communicator of the distributed Table layer: RCCL over
// xGMI, one process per GPU, ordered on the capf session's stream.
//
// The reference's only exchange is Flink's hash repartition between operator
// instances (FlinkTable.scala:123-196 lower join / groupBy / distinct onto
// hash-partitioned DataSet operators).  Here a rank's shuffle is
// capf_table_hash_route → capf_table_pack_rows → capf_comm_all_to_all →
// capf_table_from_packed_rows, and a global count(*) is ONE 8-byte
// capf_comm_all_reduce.  The Python layer (dist_table.py) uses torch.distributed
// for the same collectives; this C-ABI serves hosts without torch (the JVM
// twin, integration/scala/org/opencypher/gpu/DistGpuTable.scala).
//
// RCCL is loaded on first use (dlopen): a process that never builds a
// communicator never maps it, and one whose framework already mapped its own
// RCCL copy (torch) reuses that one (RTLD_NOLOAD first).
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "capf_internal.h"

namespace {

struct Rccl {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};

const Rccl &rccl() {
  static Rccl r;
  static std::once_flag once;
  static std::string err;
  std::call_once(once, [] {
    void *h = nullptr;
    for (const char *name : {"librccl.so", "librccl.so.1"})
      if (!h) h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      err = std::string("RCCL not loadable: ") + dlerror();
      return;
    }
#define CAPF_SYM(field, name) r.field = (decltype(r.field))dlsym(h, name)
    CAPF_SYM(get_unique_id, "ncclGetUniqueId");
    CAPF_SYM(init_rank, "ncclCommInitRank");
    CAPF_SYM(destroy, "ncclCommDestroy");
    CAPF_SYM(all_reduce, "ncclAllReduce");
    CAPF_SYM(all_gather, "ncclAllGather");
    CAPF_SYM(send, "ncclSend");
    CAPF_SYM(recv, "ncclRecv");
    CAPF_SYM(group_start, "ncclGroupStart");
    CAPF_SYM(group_end, "ncclGroupEnd");
    CAPF_SYM(error_string, "ncclGetErrorString");
#undef CAPF_SYM
    if (!r.get_unique_id || !r.init_rank || !r.destroy || !r.all_reduce || !r.all_gather || !r.send || !r.recv ||
        !r.group_start || !r.group_end)
      err = "RCCL lacks a collective this backend uses";
  });
  if (!err.empty()) capf::fail(CAPF_ERR_INTERNAL, err);
  return r;
}

void check(ncclResult_t rc, const char *what) {
  if (rc != ncclSuccess) {
    const Rccl &r = rccl();
    capf::fail(CAPF_ERR_INTERNAL, std::string(what) + ": " + (r.error_string ? r.error_string(rc) : "RCCL error"));
  }
}

}  // namespace

struct capf_comm {
  capf_session *session;
  ncclComm_t comm;
  int world, rank;
};

using namespace capf;

#define COMM_API_BEGIN try {
#define COMM_API_END                                            \
  }                                                             \
  catch (const capf::Error &e) {                                \
    return capf::record_error(e.code, e.what());                \
  }                                                             \
  catch (const std::exception &e) {                             \
    return capf::record_error(CAPF_ERR_INTERNAL, e.what());     \
  }                                                             \
  return CAPF_OK;

static hipStream_t stream_of(capf_comm *c) { return c->session->impl.stream; }

capf_status capf_comm_unique_id(uint8_t *id_out) {
  COMM_API_BEGIN
  if (!id_out) illegal("id_out is null");
  ncclUniqueId id;
  check(rccl().get_unique_id(&id), "ncclGetUniqueId");
  memcpy(id_out, id.internal, CAPF_COMM_ID_BYTES);
  COMM_API_END
}

capf_status capf_comm_init(capf_session *s, int32_t world, int32_t rank, const uint8_t *id, capf_comm **out) {
  COMM_API_BEGIN
  if (!s || !id || !out) illegal("null argument");
  if (world < 1 || rank < 0 || rank >= world) illegal("rank outside [0, world)");
  HIP_CHECK(hipSetDevice(s->impl.device));
  ncclUniqueId uid;
  memcpy(uid.internal, id, CAPF_COMM_ID_BYTES);
  auto *c = new capf_comm{s, nullptr, world, rank};
  ncclResult_t rc = rccl().init_rank(&c->comm, world, uid, rank);
  if (rc != ncclSuccess) {
    delete c;
    check(rc, "ncclCommInitRank");
  }
  *out = c;
  COMM_API_END
}

capf_status capf_comm_destroy(capf_comm *c) {
  COMM_API_BEGIN
  if (!c) return CAPF_OK;
  ncclResult_t rc = rccl().destroy(c->comm);
  delete c;
  check(rc, "ncclCommDestroy");
  COMM_API_END
}

capf_status capf_comm_all_reduce_i64(capf_comm *c, int64_t *d_buf, int64_t n, int32_t op) {
  COMM_API_BEGIN
  if (!c || (!d_buf && n > 0)) illegal("null argument");
  if (op != CAPF_COMM_SUM && op != CAPF_COMM_MAX) illegal("reduction must be CAPF_COMM_SUM or CAPF_COMM_MAX");
  if (n > 0)
    check(rccl().all_reduce(d_buf, d_buf, (size_t)n, ncclInt64, op == CAPF_COMM_SUM ? ncclSum : ncclMax, c->comm,
                            stream_of(c)),
          "ncclAllReduce");
  COMM_API_END
}

capf_status capf_comm_all_gather_bytes(capf_comm *c, const void *d_send, int64_t bytes, void *d_recv) {
  COMM_API_BEGIN
  if (!c || ((!d_send || !d_recv) && bytes > 0)) illegal("null argument");
  if (bytes > 0)
    check(rccl().all_gather(d_send, d_recv, (size_t)bytes, ncclUint8, c->comm, stream_of(c)), "ncclAllGather");
  COMM_API_END
}

capf_status capf_comm_all_to_all_bytes(capf_comm *c, const void *d_send, const int64_t *send_bytes, void *d_recv,
                                       const int64_t *recv_bytes) {
  COMM_API_BEGIN
  if (!c || !send_bytes || !recv_bytes) illegal("null argument");
  const Rccl &r = rccl();
  // one group of point-to-point pairs: RCCL schedules them over the xGMI links
  // together (the shape of an all-to-allv; per-link bound on xGMI)
  // every argument is checked before the group opens: a throw inside the
  // group would leave it open, and the next collective would join it
  int64_t st = 0, rt = 0;
  for (int p = 0; p < c->world; ++p) {
    if (send_bytes[p] < 0 || recv_bytes[p] < 0) illegal("negative byte count");
    st += send_bytes[p];
    rt += recv_bytes[p];
  }
  if ((st > 0 && !d_send) || (rt > 0 && !d_recv)) illegal("null buffer");
  int64_t so = 0, ro = 0;
  check(r.group_start(), "ncclGroupStart");
  ncclResult_t first = ncclSuccess;
  const char *what = nullptr;
  for (int p = 0; p < c->world && first == ncclSuccess; ++p) {
    if (send_bytes[p] > 0) {
      ncclResult_t rc = r.send((const uint8_t *)d_send + so, (size_t)send_bytes[p], ncclUint8, p, c->comm,
                               stream_of(c));
      if (rc != ncclSuccess) first = rc, what = "ncclSend";
    }
    if (first == ncclSuccess && recv_bytes[p] > 0) {
      ncclResult_t rc = r.recv((uint8_t *)d_recv + ro, (size_t)recv_bytes[p], ncclUint8, p, c->comm,
                               stream_of(c));
      if (rc != ncclSuccess) first = rc, what = "ncclRecv";
    }
    so += send_bytes[p];
    ro += recv_bytes[p];
  }
  // the group is always closed, then the first error is raised
  ncclResult_t end = r.group_end();
  if (first != ncclSuccess) check(first, what);
  check(end, "ncclGroupEnd");
  COMM_API_END
}

capf_status capf_comm_rank(capf_comm *c, int32_t *rank, int32_t *world) {
  COMM_API_BEGIN
  if (!c) illegal("null communicator");
  if (rank) *rank = c->rank;
  if (world) *world = c->world;
  COMM_API_END
}
