// me_internal.hpp — host-side internals of libme_hip.so (context, errors,
// scratch memory, kernel timing).  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdarg>
#include <cstdio>
#include <string>
#include <vector>
#include "../../include/me_hip.h"

struct me_timer_pair {
  hipEvent_t a, b;
  int kernel;
};

struct me_ctx {
  int device = 0;
  int num_cu = 256;  // compute units of the device (grid sizing of streaming kernels)
  int cu_active = 0;  // compute units enabled for the own stream (0: all; me_set_cu_mask)
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  std::string err;
  // growable device scratch slots (allocated outside timed/captured regions)
  std::vector<void*> slot_ptr;
  std::vector<size_t> slot_size;
  // pinned host staging for small scalar read-backs
  void* pinned = nullptr;
  size_t pinned_size = 0;
  // kernel timing
  int timing = 0;  // bitmask of timed kernel families (ME_KT_*)
  std::vector<me_timer_pair> pending;
  std::vector<hipEvent_t> event_pool;
  long launches[ME_KT_COUNT] = {0};
  double total_ms[ME_KT_COUNT] = {0};
  long kt_seen[ME_KT_COUNT] = {0};  // launches of each family since the last reset (sampling)
  int timing_every = 1;             // time every k-th launch of a timed family (me_timing_sample)
  hipEvent_t poll_ev[2] = {nullptr, nullptr};  // device-state read-back events of iterative solves
  // glibc-compatible rand() stream of the RANSAC sampling (vo.hip)
  int32_t rand_st[31] = {0};
  int rand_f = 3, rand_r = 0;
  bool rand_init = false;
  long long dbg[16] = {0};  // diagnostics (last BA solve phase stamps)
  int dbg_solve_flags = 0;        // test hook (me_debug_solve_flags): OR-ed into the camera solve's diagnostic flags
  unsigned dbg_solve_count = 0;  // solves queued since the hook was set (reset by it)
  // asynchronous BA solve in flight (me_ba_solve_async / me_ba_wait, ba.hip):
  // its own pinned staging, so later calls on the ctx cannot overwrite it
  void* ba_async = nullptr;
  void (*ba_async_free)(me_ctx*) = nullptr;
  void* ba_pinned[2] = {nullptr, nullptr};  // staging of the (at most two) queued asynchronous BA solves
  size_t ba_pinned_size[2] = {0, 0};
  int ba_lds_attr = 0;  // dynamic-LDS ceilings of the BA kernels set (plan_build)
  void* scale_mirror = nullptr;  // coherent host page the scale LM control writes its state to
  int scale_gen = 0;             // generation of the last scale LM solve (mirror ownership)
  int scale_lm_cap = -1;         // co-resident workgroups of the persistent scale LM kernel (-1: not queried)
  long scale_counters[4] = {0, 0, 0, 0};  // last solve: residual / normal-equation evaluations, LM rejections, executed residual evaluations
  // MI term tables, one per patch pixel count N (built on first use, mi.hip)
  float* mi_table[256] = {nullptr};
};

// Multi-GPU communicator (comm.hip): RCCL, or a caller callback.
struct me_comm {
  me_ctx* ctx = nullptr;
  int world = 1, rank = 0;
  void* nccl = nullptr;            // ncclComm_t (native RCCL over xGMI)
  me_allreduce_fn ar = nullptr;    // else: caller all-reduce (host-staged)
  void* user = nullptr;
  double xch_us[2] = {0.0, 0.0};   // calibrated us per exchange: packed system, step scalars (max over ranks)
};
// All-reduce of n doubles in place on the ctx stream (op ME_COMM_SUM / ME_COMM_MAX).
int me_comm_allreduce_impl(me_comm* m, double* buf, long n, int op);

// Device table of every MI term value for patches of N pixels (mi.hip).
int me_mi_table(me_ctx* ctx, int npx, const float** out);

int me_set_error(me_ctx* ctx, int code, const char* fmt, ...);

#define ME_HIP(ctx, call)                                                                    \
  do {                                                                                       \
    hipError_t e_ = (call);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      return me_set_error((ctx), ME_ERR_HIP, "%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), \
                          __FILE__, __LINE__);                                               \
  } while (0)

#define ME_CHECK(ctx, cond, ...)                                     \
  do {                                                               \
    if (!(cond)) return me_set_error((ctx), ME_ERR_INVALID, __VA_ARGS__); \
  } while (0)

#define ME_TRY(expr)            \
  do {                          \
    int rc_ = (expr);           \
    if (rc_ != ME_OK) return rc_; \
  } while (0)

// Returns a device buffer of at least `bytes` for scratch slot `slot`.
int me_scratch(me_ctx* ctx, int slot, size_t bytes, void** out);
int me_pinned(me_ctx* ctx, size_t bytes, void** out);
int me_check_launch(me_ctx* ctx, const char* what);

// roctx range (rocprofv3 --marker-trace) around an entry point's host work.
struct me_range {
  explicit me_range(const char* name);
  ~me_range();
};

// RAII event pair around one launch when timing is enabled.
// Family timer around a launch.  ext: the launch itself takes the two events
// (hipExtLaunchKernelGGL: the kernel's own begin / end timestamps, no marker
// packets of their own on the stream); else they are recorded around it.
struct me_ktimer {
  me_ctx* c;
  int k;
  bool ext;
  hipEvent_t a = nullptr, b = nullptr;
  me_ktimer(me_ctx* ctx, int kernel, bool ext_launch = false);
  ~me_ktimer();
};

// Scratch slot ids (one owner per slot)
enum {
  SLOT_IMG_L = 0, SLOT_IMG_R, SLOT_XY_L, SLOT_XY_R, SLOT_MI_OUT, SLOT_RED, SLOT_GENERIC,
  SLOT_SC_TRACKS, SLOT_SC_RES, SLOT_SC_RES2, SLOT_SC_NEQ, SLOT_SC_IMGL, SLOT_SC_IMGR,
  SLOT_KLT_PYR, SLOT_KLT_PTS, SLOT_NMS, SLOT_VO, SLOT_EPI, SLOT_MONO,
  SLOT_COUNT
};
