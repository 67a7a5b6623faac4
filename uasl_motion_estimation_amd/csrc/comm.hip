// comm.hip — the multi-GPU communicator of the landmark-sharded BA (SURVEY
// §8e).  One me_comm per rank (one process per GPU): an RCCL communicator over
// xGMI whose all-reduces are enqueued on the ctx stream with no host round
// trip, or a caller callback (host-staged exchanges: gloo, or several contexts
// of one GPU driven by threads).  The reference has no multi-GPU path; this
// is the exchange `north_star` asks for around BundleAdjuster<4>::optimise
// (include/MotionEstimation/optimisation/BundleAdjuster.h:431-476).
#include <algorithm>
#include <chrono>
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

// Exchange-cost calibration (me_comm_calibrate): wall time per all-reduce
// of the two sizes a sharded LM iteration exchanges, stream-synchronised,
// then the max over the ranks -- the landmark-count gate's input, measured
// on the communicator that will carry the exchanges instead of a constant.
static int comm_calibrate(me_comm* m, int reps) {
  me_ctx* c = m->ctx;
  reps = std::max(1, reps);
  double* d = nullptr;
  ME_HIP(c, hipMalloc(&d, 8 * (size_t)ME_COMM_CAL_SYSTEM));
  int rc = ME_OK;
  double us[2] = {0.0, 0.0};
  auto run = [&]() -> int {
    ME_HIP(c, hipMemsetAsync(d, 0, 8 * (size_t)ME_COMM_CAL_SYSTEM, c->stream));
    // (a callback may order its copies on another stream than the ctx's, e.g.
    // torch's current one: the buffer's contents are settled before each use)
    ME_HIP(c, hipStreamSynchronize(c->stream));
    const long sizes[2] = {ME_COMM_CAL_SYSTEM, 5};
    for (int k = 0; k < 2; ++k) {
      for (int i = 0; i < 3; ++i) ME_TRY(me_comm_allreduce_impl(m, d, sizes[k], ME_COMM_SUM));
      ME_HIP(c, hipStreamSynchronize(c->stream));
      const auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < reps; ++i) ME_TRY(me_comm_allreduce_impl(m, d, sizes[k], ME_COMM_SUM));
      ME_HIP(c, hipStreamSynchronize(c->stream));
      us[k] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
    }
    // the same values on every rank: the max of each over the ranks
    ME_HIP(c, hipMemcpyAsync(d, us, sizeof(us), hipMemcpyHostToDevice, c->stream));
    ME_HIP(c, hipStreamSynchronize(c->stream));
    ME_TRY(me_comm_allreduce_impl(m, d, 2, ME_COMM_MAX));
    ME_HIP(c, hipMemcpyAsync(us, d, sizeof(us), hipMemcpyDeviceToHost, c->stream));
    ME_HIP(c, hipStreamSynchronize(c->stream));
    return ME_OK;
  };
  rc = run();
  (void)hipStreamSynchronize(c->stream);
  (void)hipFree(d);
  if (rc == ME_OK) {
    m->xch_us[0] = us[0];
    m->xch_us[1] = us[1];
  }
  return rc;
}
constexpr int kCalReps = 10;

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
  if (int rc2 = comm_calibrate(m, kCalReps)) {
    me_comm_destroy(m);
    return rc2;
  }
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
  if (int rc = comm_calibrate(m, kCalReps)) {
    me_comm_destroy(m);
    return rc;
  }
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

int me_comm_calibrate(me_comm* m, int reps) {
  if (!m) return ME_ERR_INVALID;
  ME_HIP(m->ctx, hipSetDevice(m->ctx->device));
  return comm_calibrate(m, reps);
}

int me_comm_exchange_us(const me_comm* m, double* system_us, double* scalars_us) {
  if (!m) return ME_ERR_INVALID;
  if (system_us) *system_us = m->xch_us[0];
  if (scalars_us) *scalars_us = m->xch_us[1];
  return ME_OK;
}

int me_ba_shard_worthwhile_comm(const me_comm* m, long n_obs) {
  if (!m) return 0;
  const double x = 0.5 * (m->xch_us[0] + m->xch_us[1]);
  return me_ba_shard_worthwhile(n_obs, m->world, x);
}

int me_comm_allreduce(me_comm* m, double* dev_buf, long n, int op) {
  if (!m || (n > 0 && !dev_buf) || (op != ME_COMM_SUM && op != ME_COMM_MAX)) return ME_ERR_INVALID;
  ME_HIP(m->ctx, hipSetDevice(m->ctx->device));
  return me_comm_allreduce_impl(m, dev_buf, n, op);
}

}  // extern "C"
