// comm.hip — the multi-GPU communicator of the landmark-sharded BA (SURVEY
// §8e).  One me_comm per rank (one process per GPU): an RCCL communicator over
// xGMI whose all-reduces are enqueued on the ctx stream with no host round
// trip, or a caller callback (host-staged exchanges: gloo, or several contexts
// of one GPU driven by threads).  The reference has no multi-GPU path; this
// is the exchange `north_star` asks for around BundleAdjuster<4>::optimise
// (include/MotionEstimation/optimisation/BundleAdjuster.h:431-476).
#include <cstring>
#include <rccl/rccl.h>
#include "me_internal.hpp"

static int nccl_err(me_ctx* c, ncclResult_t r, const char* what) {
  return me_set_error(c, ME_ERR_HIP, "%s failed: %s", what, ncclGetErrorString(r));
}

int me_comm_allreduce_impl(me_comm* m, double* buf, long n, int op) {
  me_ctx* c = m->ctx;
  if (n <= 0) return ME_OK;
  if (m->nccl) {
    const ncclResult_t r = ncclAllReduce(buf, buf, (size_t)n, ncclDouble, op == ME_COMM_MAX ? ncclMax : ncclSum,
                                         (ncclComm_t)m->nccl, c->stream);
    if (r != ncclSuccess) return nccl_err(c, r, "ncclAllReduce");
    return ME_OK;
  }
  if (!m->ar) return me_set_error(c, ME_ERR_STATE, "me_comm: no exchange configured");
  ME_CHECK(c, n <= 0x7fffffffL, "me_comm: %ld doubles exceed the callback's int count", n);
  // the callback's contract: sum (n > 0) or max (n < 0) in place, ordered on the ctx stream
  if (m->ar(buf, op == ME_COMM_MAX ? -(int)n : (int)n, m->user) != 0)
    return me_set_error(c, ME_ERR_HIP, "me_comm: all-reduce callback failed");
  return ME_OK;
}

extern "C" {

int me_comm_unique_id(void* id_out, int id_bytes) {
  if (!id_out || id_bytes < (int)sizeof(ncclUniqueId)) return ME_ERR_INVALID;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return ME_ERR_HIP;
  std::memcpy(id_out, &id, sizeof(id));
  return ME_OK;
}

int me_comm_create_rccl(me_ctx* c, int world, int rank, const void* id, me_comm** out) {
  if (!c || !out || !id) return ME_ERR_INVALID;
  *out = nullptr;
  ME_CHECK(c, world >= 1 && rank >= 0 && rank < world, "me_comm_create_rccl: rank %d of %d", rank, world);
  ME_HIP(c, hipSetDevice(c->device));
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  ncclComm_t nc = nullptr;
  const ncclResult_t r = ncclCommInitRank(&nc, world, uid, rank);
  if (r != ncclSuccess) return nccl_err(c, r, "ncclCommInitRank");
  auto* m = new me_comm;
  m->ctx = c;
  m->world = world;
  m->rank = rank;
  m->nccl = nc;
  *out = m;
  return ME_OK;
}

int me_comm_create_callback(me_ctx* c, int world, int rank, me_allreduce_fn ar, void* user, me_comm** out) {
  if (!c || !out || !ar) return ME_ERR_INVALID;
  *out = nullptr;
  ME_CHECK(c, world >= 1 && rank >= 0 && rank < world, "me_comm_create_callback: rank %d of %d", rank, world);
  auto* m = new me_comm;
  m->ctx = c;
  m->world = world;
  m->rank = rank;
  m->ar = ar;
  m->user = user;
  *out = m;
  return ME_OK;
}

void me_comm_destroy(me_comm* m) {
  if (!m) return;
  if (m->nccl) {
    hipSetDevice(m->ctx->device);
    hipStreamSynchronize(m->ctx->stream);
    ncclCommDestroy((ncclComm_t)m->nccl);
  }
  delete m;
}

int me_comm_info(const me_comm* m, int* world, int* rank, int* native) {
  if (!m) return ME_ERR_INVALID;
  if (world) *world = m->world;
  if (rank) *rank = m->rank;
  if (native) *native = m->nccl ? 1 : 0;
  return ME_OK;
}

int me_comm_allreduce(me_comm* m, double* dev_buf, long n, int op) {
  if (!m || (n > 0 && !dev_buf) || (op != ME_COMM_SUM && op != ME_COMM_MAX)) return ME_ERR_INVALID;
  ME_HIP(m->ctx, hipSetDevice(m->ctx->device));
  return me_comm_allreduce_impl(m, dev_buf, n, op);
}

}  // extern "C"
