// extern "C" entry points of libgpk.so (declared in include/gpk.h).
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <initializer_list>
#include <map>
#include <queue>
#include <tuple>
#include <mutex>
#include <string>
#include <vector>

#include "gpk_internal.h"

using namespace gpk;

namespace {

thread_local std::string g_err;

int fail_arg(int idx, const char* what) {
  g_err = std::string("invalid argument: ") + what;
  return -idx;
}

int fail_hip(hipError_t e, const char* where) {
  g_err = std::string(where) + ": " + hipGetErrorString(e);
  return (int)e > 0 ? (int)e : 1;
}

#define GPK_HIP(call, where)                         \
  do {                                               \
    hipError_t e_ = (call);                          \
    if (e_ != hipSuccess) return fail_hip(e_, where); \
  } while (0)

// ------------------------------------------------------------------------------ event timing
struct TimedLaunch {
  int cls;
  hipEvent_t beg, end;
  double flops, bytes;
};

struct Timing {
  std::mutex mu;
  bool on = false;
  std::vector<TimedLaunch> pending;
  std::vector<hipEvent_t> pool;
  double ms[GPK_NUM_CLASSES] = {0};
  int64_t launches[GPK_NUM_CLASSES] = {0};
  double flops[GPK_NUM_CLASSES] = {0};
  double bytes[GPK_NUM_CLASSES] = {0};
};
Timing g_timing;

hipEvent_t take_event() {
  if (!g_timing.pool.empty()) {
    hipEvent_t e = g_timing.pool.back();
    g_timing.pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  hipEventCreate(&e);
  return e;
}

// Run `launch` bracketed by events on stream s when timing is on.
template <typename F>
hipError_t timed(int cls, double flops, double bytes, hipStream_t s, F&& launch) {
  if (!g_timing.on) return launch();
  std::lock_guard<std::mutex> lk(g_timing.mu);
  TimedLaunch t{cls, take_event(), take_event(), flops, bytes};
  hipEventRecord(t.beg, s);
  hipError_t e = launch();
  hipEventRecord(t.end, s);
  g_timing.pending.push_back(t);
  return e;
}

bool valid_kdesc(const gpk_kdesc* kd, int64_t d) {
  if (!kd || kd->n_nodes <= 0 || kd->n_nodes > GPK_MAX_NODES) return false;
  if (kd->n_hyp < 0 || kd->n_hyp > GPK_MAX_HYP || kd->dim != d) return false;
  if (kd->n_ard < 0 || kd->n_ard > GPK_MAX_ARD) return false;
  int sp = 0;
  for (int q = 0; q < kd->n_nodes; ++q) {
    const gpk_node& nd = kd->nodes[q];
    if (nd.op == GPK_OP_ADD || nd.op == GPK_OP_MUL) {
      if (sp < 2) return false;
      sp -= 1;
    } else if (nd.op == GPK_OP_SE || nd.op == GPK_OP_PER || nd.op == GPK_OP_MAT32 ||
               nd.op == GPK_OP_MAT52) {
      const bool ard = (nd.flags & GPK_NODE_ARD) != 0;
      if (ard && (nd.op == GPK_OP_PER || nd.ard_slot < 0 || nd.ard_slot >= kd->n_ard)) return false;
      int need = (nd.op == GPK_OP_PER) ? 2 : (ard ? (int)d : 1);
      if (nd.flags & GPK_NODE_SCALED) need += 1;
      if (nd.hyp_offset < 0 || nd.hyp_offset + need > kd->n_hyp) return false;
      sp += 1;
      if (sp > 8) return false;
    } else {
      return false;
    }
  }
  return sp == 1;
}

size_t elem_size(int dtype) { return dtype == GPK_F64 ? 8 : 4; }

// For every base node of the postfix program: the nodes (subtree roots) whose values multiply
// its value on the way to the root -- the siblings under each MUL ancestor.  d K / d k_node is
// the product of those values (ADD ancestors pass the adjoint through unchanged).
void adjoint_masks(const gpk_kdesc& kd, uint32_t* mask) {
  int left[GPK_MAX_NODES], right[GPK_MAX_NODES], stk[GPK_MAX_NODES];
  int sp = 0;
  for (int q = 0; q < kd.n_nodes; ++q) {
    left[q] = right[q] = -1;
    mask[q] = 0u;
    if (kd.nodes[q].op == GPK_OP_ADD || kd.nodes[q].op == GPK_OP_MUL) {
      right[q] = stk[--sp];
      left[q] = stk[--sp];
    }
    stk[sp++] = q;
  }
  for (int q = kd.n_nodes; q < GPK_MAX_NODES; ++q) mask[q] = 0u;
  // top-down: the root is the last node; children inherit the parent's mask (+ sibling at MUL)
  for (int q = kd.n_nodes - 1; q >= 0; --q) {
    if (left[q] < 0) continue;
    const bool mul = kd.nodes[q].op == GPK_OP_MUL;
    mask[left[q]] = mask[q] | (mul ? (1u << right[q]) : 0u);
    mask[right[q]] = mask[q] | (mul ? (1u << left[q]) : 0u);
  }
}

// Launch-shape thresholds (environment overrides for tuning runs).
struct Tune {
  int64_t upd_t128_min;   // 128 x 128 update tiles when at least this many (else 64 x 64)
  int64_t trsm_t128_min;  // 128-row panel-solve tiles when at least this many (else 64)
  int64_t diag_dbg;       // timing-only ablation flags of the diagonal kernel (never set in production)
  int64_t lookahead;      // 1: panel chain on a high-priority side stream, 0: one stream, 2: auto (default:
                          // on for large matrices, see potrf_impl)
  int64_t la_min_blocks;  // auto look-ahead: on from this many 128-blocks of the augmented matrix
  int64_t fuse_trsm;      // f64: panel solve fused into the diagonal-block launch (1: look-ahead off only,
                          // 2: always; one workgroup per
  int64_t fuse_trsm_max;  //   64-row tile, each factoring the block) while batch x tiles <= fuse_trsm_max
  int64_t reserve_cus;    // CUs kept free of the bulk trailing update for the panel chain (32: single N = 8192
                          // 6.46 -> 6.26 ms, -LML + gradient N = 4096 3.29 -> 3.04 ms, batches of 2 / 8 / 32
                          // without pipelining +1.9 / +0.6 / +0.4 % against 8)
  int64_t group;          // panels per trailing update (K = 128 group)
  int64_t group_first;    // panels of the first group (a short first chain lets the bulk start early)
  int64_t fuse_kbuild;    // gpk_nlml: K build fused into the first trailing update (single-node kernels)
  int64_t upd_band;       // trailing-update tile order: 0 row-major, B > 0 bands of B tile rows
  int64_t skip_zero_rows; // skip the MFMAs of the all-zero 16-row blocks below the y row
  int64_t syevj_abs_tol_e3; // Jacobi: absolute rotation threshold in units of 1e-3 eps max|a_ii|
  int64_t diag_version;   // diagonal-block kernel: 2 look-ahead schedule, 1 phase-serial
  int64_t ingroup;        // in-group updates: 1 left-looking, 2 right-looking, 3 two-level, 0 auto (by batch)
  int64_t rl_max_tiles;   // auto: right-looking while batch x (block rows) stays below this
  int64_t band_skip;      // identity extra rows: leave the zero band's tiles out of the grid
  int64_t group_eye;      // panels per trailing update of identity-augmented factorisations
  int64_t asm_generic;    // K build: interior tiles through the generic loop too (A/B; bitwise equal)
  int64_t panel_stream;   // look-ahead panel chain: 0 high-priority side stream, 1 caller's stream,
                          // 2 normal-priority side stream
  int64_t trd_split_m;    // gpk_syevd: above this m the tridiagonalisation's A22 v runs over the chip (three
                          // launches per column) instead of inside one workgroup per panel
  int64_t chain;          // single f64 factorisations as ONE persistent launch (chain_kernel): 1 auto (default: on
                          // unless a factorisation enqueued on another stream of the device is still in flight --
                          // each persistent launch claims every CU, so overlapped factorisations keep the launch
                          // path: C2 at 4 in flight 1315 vs 779 evals/s), 2 always, 0 off
  int64_t chain_max_p;    //   ... while the augmented matrix has at most this many rows
  int64_t chain_grid;     //   workgroups of that launch (0: one per CU)
  int64_t chain_timeout_ms;  // bound of every wait inside it (then info = -1)
  int64_t chain_group;    //   panels per deferred tile update (1: every tile update one panel deep; 0: auto,
                          //   chain_group_for)
  int64_t chain_max_batch;   // batches of up to this many members run as one persistent launch too ...
  int64_t chain_batch_max_rows;  // ... while batch x (rows of the augmented matrix) stays within this
                                 // (batch x span, persistent vs launch path: N = 2048 x 8 1.15 vs 1.38 ms,
                                 // 4096 x 2 1.87 vs 2.53, 4096 x 4 2.83 vs 3.51; 4096 x 8 5.32 vs 5.07,
                                 // 2048 x 16 2.02 vs 1.94 -- profiles/r04_chain_batch.jsonl)
  int64_t chain_uq;       //   the next diagonal block's update split by 32-column quarter (0: one task per slice)
  int64_t chain_eye;      //   identity-augmented factorisations (the gradient / explicit inverse) too (1: auto as
                          //   above, 0: never)
  int64_t chain_max_p_eye;  // ... while their augmented matrix has at most this many rows
  int64_t asm_feat;       // K build, two-leaf SE + periodic trees on MFMA: per-point features in a pre-pass
                          // (pair_feat_kernel; 0: staged per tile, A/B -- bitwise equal)
  int64_t chain_min_p;    // chain = 1 (auto): the launch path below this many rows (a handful of panels: the
                          // launch path's few launches win -- get_metric N = 128 / 256 / 384 0.119 / 0.165 / 0.216
                          // vs 0.145 / 0.187 / 0.224 ms, equal at 512, the persistent launch ahead from 768,
                          // profiles/r05ak_api_small_n_chain_vs_launch.jsonl)
  int64_t chain_min_p_eye;  // ... and for identity-augmented factorisations (value + gradient): N = 1024 / 1280
                            // 0.554 / 0.657 ms on the launch path vs 0.590 / 0.683, N = 1536 0.809 vs 0.786
                            // (profiles/r05al_api_crossover.jsonl)
  int64_t chain_group_corner;  // identity-augmented plans: panels per deferred update of the corner's tiles (-K^-1,
                               // read by no later task)
  int64_t chain_corner_tail;   //   ... except the last this many panels, which keep chain_group
  int64_t chain_group_la;      // deferred (grouped) tile updates only for block columns at least this many columns
                               // past the group's last panel
  int64_t asm_f32_fast;   // f32 K build of a single SE / MAT32 / MAT52 node: the interior tiles through f32_fast_kernel
                          // (f64 distances, f32 transcendentals; 0: every tile through the general f64 loop, A/B)
  int64_t chain_group_eye;  // identity-augmented plans: panels per deferred tile update (0: chain_group's rule; 8: value +
                            // gradient N = 8192 11.33 vs 11.11 ms best, profiles/r06b_grad_sweep_8192.jsonl)
  int64_t chain_xcd;      // persistent launch: the diagonal chain's tasks as a second list, claimed first by up to
                          // chain_xcd_seats workgroups of XCD 0 (their hand-offs in one L2); 0: one list
  int64_t chain_xcd_seats;
  int64_t asm_f32_chunk;  // f32_fast_kernel: consecutive lower tiles per workgroup (C3: 1 / 2 / 4 / 8 / 16 0.062 / 0.059 /
                          // 0.059 / 0.063 / 0.073 ms, profiles/r06c_kb_c3_chunks.txt)
  int64_t chain_f32;      // f32 factorisations as one persistent launch too (chain_kernel<float>: f32 tile tasks, the
                          // diagonal blocks in f64 as the launch path's); 0: f32 keeps the launch path
  int64_t chain_group_near;  // tile updates of the columns too near the diagonal for the deferred group: in sub-groups
                             // of this many panels (same look-ahead rule; 1: panel by panel)
  int64_t chain_u128;     // the next panel's column below the next diagonal block: one 128 x 128 tile update per block
                          // row instead of four 32-row slice updates (1; 0: slice updates; 2 auto: slice updates only
                          // below 48 diagonal blocks on a grid of more than 2 workgroups per diagonal block)
  int64_t chain_near_la;  // chain_group_near's sub-groups cover the columns at least this many past their last panel
                          // (1: C2 1866 -> 1884 evals/s, C3 474 -> 480, value + gradient N = 8192 10.6 -> 10.43 ms
                          // against 2, profiles/r06u_near_la_ab.txt)
  int64_t chain_s128;     // the panel solves below the next diagonal block: one task per block row (its slices one after
                          // another) instead of one per 32-row slice (1; 0: per slice; 2 auto: on a grid of at most 2
                          // workgroups per diagonal block -- the CU-share launches side by side -- and for
                          // identity-augmented plans of at least 64 diagonal blocks; N = 6144 within the spread either way)
  // (new fields go last: tune() initialises the struct positionally)
};

int64_t env_i64(const char* name, int64_t dflt) {
  const char* v = getenv(name);
  return (v && *v) ? (int64_t)atoll(v) : dflt;
}

Tune& tune() {
  static Tune t = {env_i64("GPK_UPD_T128_MIN", 512), env_i64("GPK_TRSM_T128_MIN", 256),
                         env_i64("GPK_DIAG_DEBUG", 0), env_i64("GPK_LOOKAHEAD", 2), env_i64("GPK_LA_MIN_BLOCKS", 64),
                         env_i64("GPK_FUSE_TRSM", 1), env_i64("GPK_FUSE_TRSM_MAX", 256),
                         env_i64("GPK_RESERVE_CUS", 32), env_i64("GPK_GROUP", 8),
                         env_i64("GPK_GROUP_FIRST", 8), env_i64("GPK_FUSE_KBUILD", 1),
                         env_i64("GPK_UPD_BAND", 0), env_i64("GPK_SKIP_ZERO_ROWS", 1), env_i64("GPK_SYEVJ_ABS_TOL_E3", 0),
                         env_i64("GPK_DIAG_VERSION", 2), env_i64("GPK_INGROUP", 0),
                         env_i64("GPK_RL_MAX_TILES", 256), env_i64("GPK_BAND_SKIP", 1),
                         env_i64("GPK_GROUP_EYE", 4), env_i64("GPK_ASM_GENERIC", 0),
                         env_i64("GPK_PANEL_STREAM", 0), env_i64("GPK_TRD_SPLIT_M", 1024),
                         env_i64("GPK_CHAIN", 1), env_i64("GPK_CHAIN_MAX_P", 12416), env_i64("GPK_CHAIN_GRID", 0),
                         env_i64("GPK_CHAIN_TIMEOUT_MS", 1000), env_i64("GPK_CHAIN_GROUP", 0),
                         env_i64("GPK_CHAIN_MAX_BATCH", 8), env_i64("GPK_CHAIN_BATCH_MAX_ROWS", 17500),
                         env_i64("GPK_CHAIN_UQ", 1), env_i64("GPK_CHAIN_EYE", 1),
                         env_i64("GPK_CHAIN_MAX_P_EYE", 16640), env_i64("GPK_ASM_FEAT", 1),
                         env_i64("GPK_CHAIN_MIN_P", 768), env_i64("GPK_CHAIN_MIN_P_EYE", 3072),
                         env_i64("GPK_CHAIN_GROUP_CORNER", 16), env_i64("GPK_CHAIN_CORNER_TAIL", 8),
                         env_i64("GPK_CHAIN_GROUP_LA", 2), env_i64("GPK_ASM_F32_FAST", 1),
                         env_i64("GPK_CHAIN_GROUP_EYE", 8),
                         env_i64("GPK_CHAIN_XCD", 0), env_i64("GPK_CHAIN_XCD_SEATS", 16),
                         env_i64("GPK_ASM_F32_CHUNK", 4), env_i64("GPK_CHAIN_F32", 1),
                         env_i64("GPK_CHAIN_GROUP_NEAR", 2), env_i64("GPK_CHAIN_U128", 2),
                         env_i64("GPK_CHAIN_NEAR_LA", 1), env_i64("GPK_CHAIN_S128", 2)};
  return t;
}

// Knob names of gpk_tune / gpk_tune_thread.
struct Knob {
  const char* name;
  int64_t Tune::*field;
};
const Knob kKnobs[] = {
    {"lookahead", &Tune::lookahead},         {"reserve_cus", &Tune::reserve_cus},
    {"upd_t128_min", &Tune::upd_t128_min},   {"trsm_t128_min", &Tune::trsm_t128_min},
    {"diag_debug", &Tune::diag_dbg},         {"group", &Tune::group},
    {"group_first", &Tune::group_first},     {"fuse_kbuild", &Tune::fuse_kbuild},
    {"upd_band", &Tune::upd_band},           {"skip_zero_rows", &Tune::skip_zero_rows},
    {"syevj_abs_tol_e3", &Tune::syevj_abs_tol_e3}, {"diag_version", &Tune::diag_version},
    {"ingroup", &Tune::ingroup},             {"rl_max_tiles", &Tune::rl_max_tiles},
    {"band_skip", &Tune::band_skip},         {"group_eye", &Tune::group_eye},
    {"asm_generic", &Tune::asm_generic},     {"panel_stream", &Tune::panel_stream},
    {"la_min_blocks", &Tune::la_min_blocks}, {"fuse_trsm", &Tune::fuse_trsm},
    {"fuse_trsm_max", &Tune::fuse_trsm_max}, {"trd_split_m", &Tune::trd_split_m},
    {"chain", &Tune::chain},                 {"chain_max_p", &Tune::chain_max_p},
    {"chain_grid", &Tune::chain_grid},       {"chain_timeout_ms", &Tune::chain_timeout_ms},
    {"chain_group", &Tune::chain_group},     {"chain_max_batch", &Tune::chain_max_batch},
    {"chain_batch_max_rows", &Tune::chain_batch_max_rows}, {"chain_uq", &Tune::chain_uq},
    {"chain_eye", &Tune::chain_eye},         {"chain_max_p_eye", &Tune::chain_max_p_eye},
    {"asm_feat", &Tune::asm_feat},           {"chain_min_p", &Tune::chain_min_p},
    {"chain_min_p_eye", &Tune::chain_min_p_eye}, {"chain_group_corner", &Tune::chain_group_corner},
    {"chain_corner_tail", &Tune::chain_corner_tail}, {"chain_group_la", &Tune::chain_group_la},
    {"asm_f32_fast", &Tune::asm_f32_fast},
    {"chain_group_eye", &Tune::chain_group_eye}, {"chain_xcd", &Tune::chain_xcd},
    {"chain_xcd_seats", &Tune::chain_xcd_seats}, {"asm_f32_chunk", &Tune::asm_f32_chunk},
    {"chain_f32", &Tune::chain_f32},         {"chain_group_near", &Tune::chain_group_near},
    {"chain_u128", &Tune::chain_u128},         {"chain_near_la", &Tune::chain_near_la},
    {"chain_s128", &Tune::chain_s128},
};

int64_t Tune::*knob_field(const char* key) {
  for (const Knob& k : kKnobs)
    if (!strcmp(key, k.name)) return k.field;
  return nullptr;
}

// Per-host-thread overrides (gpk_tune_thread): a caller that runs its own schedule -- e.g. the
// pipelined sweep's factorisations on several streams -- pins knobs for its own calls without
// changing them for other threads.
thread_local std::vector<std::pair<int64_t Tune::*, int64_t>> t_tune_over;

// The knobs in effect for one call on this thread: one snapshot per call, so a gpk_tune from
// another thread (ctypes releases the GIL during the enqueue) cannot change a decision midway.
Tune tune_now() {
  Tune t = tune();
  for (const auto& o : t_tune_over) t.*(o.first) = o.second;
  return t;
}


// Per host thread and device: the high-priority panel stream, the bulk-update stream (created
// with a CU mask that leaves tune().reserve_cus CUs to the panel chain, so that the
// diagonal-block kernel -- one workgroup of 150 KB LDS per batch member -- never waits for a CU
// to drain) and the fork / join events of gpk_potrf_aug; created on first use.
struct SideStream {
  hipStream_t panel_s = nullptr, bulk_s = nullptr, panel_np = nullptr;
  hipEvent_t fork = nullptr, panel = nullptr, bulk = nullptr, join_p = nullptr, join_b = nullptr;
};

// Every side stream ever created, destroyed by an atexit handler: registered after the HIP
// runtime's own start-up, it runs before the runtime tears down, and a CU-masked queue still
// alive at that point crashes rocprofv3's finalisation.
std::mutex g_side_mu;
std::vector<SideStream*> g_side_all;

void release_side_streams() {
  std::lock_guard<std::mutex> lk(g_side_mu);
  for (SideStream* ss : g_side_all) {
    if (ss->panel_s) hipStreamSynchronize(ss->panel_s);
    if (ss->bulk_s) hipStreamSynchronize(ss->bulk_s);
    if (ss->panel_np) hipStreamSynchronize(ss->panel_np);
    for (hipEvent_t e : {ss->fork, ss->panel, ss->bulk, ss->join_p, ss->join_b})
      if (e) hipEventDestroy(e);
    if (ss->panel_s) hipStreamDestroy(ss->panel_s);
    if (ss->bulk_s) hipStreamDestroy(ss->bulk_s);
    if (ss->panel_np) hipStreamDestroy(ss->panel_np);
    *ss = SideStream();
  }
  g_side_all.clear();
}

SideStream* side_stream() {
  thread_local std::vector<SideStream*> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return nullptr;
  if ((int)cache.size() <= dev) cache.resize(dev + 1, nullptr);
  if (!cache[dev]) {
    std::lock_guard<std::mutex> lk(g_side_mu);
    static bool registered = false;
    if (!registered) {
      std::atexit(release_side_streams);
      registered = true;
    }
    cache[dev] = new SideStream();  // owned by g_side_all (released at exit)
    g_side_all.push_back(cache[dev]);
  }
  SideStream& ss = *cache[dev];
  if (!ss.panel_s) {
    int least = 0, greatest = 0, ncu = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) return nullptr;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return nullptr;
    if (hipStreamCreateWithPriority(&ss.panel_s, hipStreamNonBlocking, greatest) != hipSuccess) return nullptr;
    if (hipStreamCreateWithFlags(&ss.panel_np, hipStreamNonBlocking) != hipSuccess) return nullptr;
    const int64_t r = std::max<int64_t>(0, std::min<int64_t>(tune().reserve_cus, ncu / 2));
    if (r > 0) {
      std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
      for (int c = (int)r; c < ncu; ++c) mask[c / 32] |= 1u << (c % 32);
      if (hipExtStreamCreateWithCUMask(&ss.bulk_s, (uint32_t)mask.size(), mask.data()) != hipSuccess)
        return nullptr;
    } else if (hipStreamCreateWithFlags(&ss.bulk_s, hipStreamNonBlocking) != hipSuccess) {
      return nullptr;
    }
    for (hipEvent_t* e : {&ss.fork, &ss.panel, &ss.bulk, &ss.join_p, &ss.join_b})
      if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) return nullptr;
  }
  return &ss;
}

// Ticket counters of the fused panel solve (DiagArgs::ctr), one block of kFuseCtr per (device,
// stream): launches on one stream never overlap.  Tickets are drawn with atomicInc(ctr, grid - 1), so
// the grid's last draw wraps the counter back to 0 by itself (no reset store).  A handle that stands
// for one stream per host thread (hipStreamPerThread) or a stream being captured does not get
// counters: its panel solve stays a separate launch (fuse_counters returns nullptr).  The null stream
// is one queue per device whatever thread launches on it (torch's default stream), so it keeps them.
constexpr int kFuseCtr = 256;  // members per launch
std::mutex g_ctr_mu;
std::map<std::pair<int, hipStream_t>, int32_t*> g_ctr;

int32_t* fuse_counters(hipStream_t s) {
  if (s == hipStreamPerThread) return nullptr;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_ctr_mu);
  auto it = g_ctr.find({dev, s});
  if (it != g_ctr.end()) return it->second;
  int32_t* p = nullptr;
  if (hipMalloc(&p, kFuseCtr * sizeof(int32_t)) != hipSuccess) return nullptr;
  if (hipMemsetAsync(p, 0, kFuseCtr * sizeof(int32_t), s) != hipSuccess) {
    hipFree(p);
    return nullptr;
  }
  g_ctr[{dev, s}] = p;  // owned for the life of the process
  return p;
}


// ------------------------------------------------------------------------ persistent factorisation
// Task order of chain_kernel (gpk_potrf.hip) for one shape: the task graph (D / S / U32 / BLK, see there)
// list-scheduled on `grid` workers with estimated durations, highest bottom level (longest path to the
// end) first; the order in which the simulation starts the tasks is a topological order, which the
// kernel needs (every task waits only for tasks claimed before it), and puts the diagonal chain ahead
// of the trailing tiles whenever both are ready.
struct ChainPlan {
  int32_t* tasks = nullptr;  // device [ntasks + ntasks_b][4]: list A, then list B (chain_xcd)
  int32_t ntasks = 0, ntasks_b = 0;
  int32_t nblk = 0, nsl = 0, nbc = 0;
};
std::mutex g_chain_mu;
// key: device, n_pad, y_row, grid, members, eye, and every knob chain_order reads (ChainKnobs)
std::map<std::tuple<int, int64_t, int64_t, int, int, int, int, int, int, int, int, int, int, int, int, int>, ChainPlan>
    g_chain_plans;

enum { CHT_D = 0, CHT_S = 1, CHT_U32 = 2, CHT_BLK = 3 };

// chain_xcd: the diagonal chain's tasks -- D, the panel solves of the next diagonal block's slices (S / SQ), its
// quarter updates (UQ) or, without quarters, its per-slice updates (U32 of block column k + 1 on its own rows) --
// move to list B, in their order; the rest stays list A.  Both lists keep the topological order.  Returns nb.
int32_t chain_split_lists(std::vector<int32_t>& ord) {
  std::vector<int32_t> la, lb;
  la.reserve(ord.size());
  for (size_t t = 0; t + 3 < ord.size(); t += 4) {
    const int tyg = ord[t], ty = tyg & 3, g = ((tyg >> 2) & 15) + 1, k = ord[t + 1], r = ord[t + 2], j = ord[t + 3];
    const bool chain = ty == CHT_D || (ty == CHT_S && (r >> 2) == k + 1) ||
                       (ty == CHT_U32 && (g > 1 || (j == k + 1 && (r >> 2) == k + 1)));
    std::vector<int32_t>& dst = chain ? lb : la;
    dst.insert(dst.end(), ord.begin() + t, ord.begin() + t + 4);
  }
  const int32_t nb = (int32_t)(lb.size() / 4);
  ord.assign(la.begin(), la.end());
  ord.insert(ord.end(), lb.begin(), lb.end());
  return nb;
}
// Counter scratch of the persistent launch, per (host thread, device, stream): the counters are zeroed
// by a memset enqueued before each launch, so two threads enqueueing on one stream (torch's null stream
// is shared by every thread) must never share them -- memset A, memset B, launch A, launch B would hand
// launch B counters already past its task count.  A thread's own calls on one stream are stream-ordered.
// The blocks are freed when their thread exits (hipFree waits for the device, so no launch still reads them).
struct ChainCtl {
  std::map<std::pair<int, hipStream_t>, std::pair<int32_t*, size_t>> blocks;
  ~ChainCtl() {
    for (auto& kv : blocks)
      if (kv.second.first) {
        int cur = 0;
        if (hipGetDevice(&cur) == hipSuccess && hipSetDevice(kv.first.first) == hipSuccess) {
          (void)hipFree(kv.second.first);
          (void)hipSetDevice(cur);
        }
      }
  }
};
thread_local ChainCtl t_chain_ctl;
std::atomic<int64_t> g_chain_launches{0};      // persistent launches enqueued
std::atomic<int64_t> g_chain_declined{0};      // auto mode: launch path taken, another stream busy
std::atomic<int64_t> g_chain_force_timeout{0};  // testing: the next N persistent launches time out
thread_local bool t_chain_last = false;         // this thread's last factorisation was the persistent one

// Factorisations in flight per (device, stream): an event recorded on the caller's stream after every
// factorisation this library enqueues.  chain = 1 (auto) takes the launch path while a factorisation on
// another stream of the device has not finished: the persistent launch claims every CU and would
// serialise overlapped factorisations (C2 at 4 in flight: 1315 evals/s on the launch path, 779 with
// persistent launches).
std::mutex g_busy_mu;
std::map<std::pair<int, hipStream_t>, hipEvent_t> g_busy;

bool plain_stream(hipStream_t s) {
  if (s == hipStreamPerThread) return false;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &cap) == hipSuccess && cap == hipStreamCaptureStatusNone;
}

void note_factorisation(hipStream_t s) {
  int dev = 0;
  if (!plain_stream(s) || hipGetDevice(&dev) != hipSuccess) return;
  std::lock_guard<std::mutex> lk(g_busy_mu);
  hipEvent_t& e = g_busy[{dev, s}];
  if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
    e = nullptr;
    return;
  }
  hipEventRecord(e, s);
}

// (entries of other streams whose last factorisation has completed are dropped -- streams come and go, e.g. a
// pipelined sweep's -- once the map holds more than a few; the caller's own entry is kept for its next record)
bool other_stream_busy(hipStream_t s) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return true;
  std::lock_guard<std::mutex> lk(g_busy_mu);
  const bool prune = g_busy.size() > 16;
  bool busy = false;
  for (auto it = g_busy.begin(); it != g_busy.end();) {
    const bool other = !(it->first.first == dev && it->first.second == s);
    const hipError_t q = it->second ? hipEventQuery(it->second) : hipSuccess;
    if (other && it->first.first == dev && q == hipErrorNotReady) busy = true;
    if (prune && other && q != hipErrorNotReady) {
      if (it->second) hipEventDestroy(it->second);
      it = g_busy.erase(it);
    } else {
      ++it;
    }
  }
  return busy;
}
int32_t* g_chain_trace = nullptr;  // GPK_CHAIN_TRACE=1: pinned host words the kernel writes its progress to
uint64_t* g_chain_times = nullptr;  // GPK_CHAIN_TIMES=1: device stamps per task of the last profiled launch
int64_t g_chain_times_n = 0;


// panels per deferred tile update: the knob, or (0) 4 below 80 diagonal blocks and 8 from there -- the deep
// updates' MFMA rate starts to matter more than the columns they hold back (N = 8192 4.46 / 4.49 ms with 4 / 8,
// 10240 7.74 / 7.62, 12288 12.56 / 12.17, profiles/r04af_chain_group_large.jsonl)
int chain_group_for(int64_t knob, int64_t n_pad, bool f32 = false) {
  if (knob > 0) return (int)knob;
  // (f32: 8 -- C3 at 8 persistent launches in flight 426 / 436 / 427 / 417 evals/s at 4 / 8 / 12 / 16,
  // profiles/r06j_c3_f32_chain_sweep.txt)
  return n_pad / NB >= 80 || f32 ? 8 : 4;
}

// Every tuning input of chain_order, resolved once per call from the knobs (and part of the plan cache key, so a
// cached device plan and gpk_chain_plan_ex always agree)
struct ChainKnobs {
  int group, uq, group_corner, corner_tail, group_la, group_near, u128, near_la, s128;
};
ChainKnobs chain_knobs(const Tune& tn, int64_t n_pad, bool eye, bool f32 = false, int grid = 0) {
  ChainKnobs k;
  const int64_t gk = eye && tn.chain_group_eye > 0 ? tn.chain_group_eye : tn.chain_group;
  k.group = std::max(1, std::min(chain_group_for(gk, n_pad, f32), 16));
  // (f32: one U32 task per slice -- chain_kernel<float> has no quarter-task bodies)
  k.uq = f32 ? 0 : (int)std::max<int64_t>(0, std::min<int64_t>(2, tn.chain_uq));
  k.group_corner = (int)std::max<int64_t>(1, std::min<int64_t>(tn.chain_group_corner, 16));
  k.corner_tail = (int)std::max<int64_t>(0, tn.chain_corner_tail);
  k.group_la = (int)std::max<int64_t>(1, tn.chain_group_la);
  k.group_near = (int)std::max<int64_t>(1, std::min<int64_t>(tn.chain_group_near, k.group));
  k.near_la = (int)std::max<int64_t>(1, tn.chain_near_la);
  // (auto: slice updates only for short chains on a full grid -- single N = 4096 on 256 workgroups 1.577 vs 1.595 ms;
  // C2's 64-workgroup launches 1726 -> 1863 evals/s, N = 8192 4.50 -> 4.31 ms, C3 f32 persistent 442 -> 470,
  // profiles/r06r_chain_u128_ab.txt)
  k.u128 = tn.chain_u128 == 1 || (tn.chain_u128 == 2 && (n_pad / NB >= 48 || grid <= 2 * (n_pad / NB))) ? 1 : 0;
  // (auto: the CU-share launches only -- C3 on 8 f32 launches of 64 workgroups 476 -> 495 evals/s, C2 neutral, while a
  // single N = 8192 on 256 workgroups lost 2 %: 4.27 -> 4.37 ms, profiles/r06x_chain_s128_ab.txt)
  // and the long identity-augmented plans (value + gradient N = 8192 10.43-10.48 -> 10.32-10.35 ms)
  k.s128 = tn.chain_s128 == 1 ||
                   (tn.chain_s128 == 2 && ((grid > 0 && grid <= 2 * (n_pad / NB)) || (eye && n_pad / NB >= 64)))
               ? 1 : 0;
  return k;
}

// list-scheduling durations (us) of D / S / U32 / BLK: the measured per-task run times (round 4, profiles/r04y_*;
// UQ: half of U32); GPK_CHAIN_DUR="d,s,u,b" overrides them (A/B), read once per process
const float* chain_durations() {
  static const std::array<float, 4> dur = [] {
    std::array<float, 4> d = {28.f, 6.5f, 12.f, 22.5f};
    if (const char* e = getenv("GPK_CHAIN_DUR")) sscanf(e, "%f,%f,%f,%f", &d[0], &d[1], &d[2], &d[3]);
    return d;
  }();
  return dur.data();
}

// Type word of a task: ty (bits 0..1) | (g - 1) << 2 (BLK over g panels; UQ: quarter + 1, bits 2..5) |
// kChainFirst (bit 6: the (slice, block column) cells the task updates have no earlier update -- its counter
// wait is for 0, not for the task's first panel; identity-augmented lists only) | member << 8.
constexpr int kChainFirst = 1 << 6;
// bit 7 on an S task (chain_uq 2): SQ -- the panel solve of a slice of the next diagonal block followed by the
// slice's lower quarters of that block's update (chain_sq); it publishes sdone after the solve, qdone = 1 at the end
constexpr int kChainSq = 1 << 7;

// eye: identity extra rows (m = n, gpk_potrf_aug_ex GPK_AUG_EXTRA_IDENTITY).  Extra row t (row n_pad + t) of
// E L^-T is zero left of column t, so block i >= nblk (extra block e = i - nblk) is zero in every panel q < e
// (its rows' panel columns are zero until panel e, where its identity entries are solved): the list leaves out
// every task that would only move zeros -- the panel solves of such slices and the tile updates where either
// block is still zero -- so the factorisation does n^3 flops (potrf + trtri + lauum) like the launch path's
// band skip.  The block holding the y row is live in every panel.
// Returns the task words (four per task); empty if the graph exceeds a bound of the device tasks (the caller
// reports that as an error -- never reached for graphs built here, whose in-degrees are bounded by construction).
std::vector<int32_t> chain_order(int64_t n_pad, int64_t y_row, int grid, int nmem, const ChainKnobs& kn,
                                 bool eye = false) {
  const int group = kn.group, chain_uq = kn.uq;
  const int nblk = (int)(n_pad / NB), yb = (int)(y_row / NB), rlast = (int)(y_row / 32);
  // block i holds a nonzero row in the columns of panel q (monotone in q): from panel live_from(i) on
  auto live_from = [&](int i) { return (!eye || i < nblk || i == yb) ? 0 : i - nblk; };
  auto live = [&](int i, int q) { return live_from(i) <= q; };
  // (flat storage: the lists reach 70 000+ tasks for the identity-augmented N = 8192 -- a vector per task's
  // dependencies and a map per tile made the first call of a shape cost ~30 ms of host time there)
  constexpr int MAXDEP = 16;  // D: up to 10 quarter tasks; BLK: 4 + 4 slices + the tile's last update
  struct Task {
    int ty, k, r, j;
    float dur;
    int nd;
    int deps[MAXDEP];
    void dep(int d) {
      if (nd < MAXDEP) deps[nd] = d;
      ++nd;
    }
  };
  std::vector<Task> T;
  T.reserve(4096);
  const int nr = rlast + 1;
  std::vector<int> D(nblk, -1), S((size_t)nblk * nr, -1), U((size_t)nblk * nr, -1);
  const int nbt = yb + 1;
  std::vector<int> last_upd((size_t)nbt * nbt, -1);  // tile (i, j) -> its latest update task so far
  auto mk = [](int ty, int k, int r, int j, float du) {
    Task t;
    t.ty = ty;
    t.k = k;
    t.r = r;
    t.j = j;
    t.dur = du;
    t.nd = 0;
    return t;
  };
  auto s_of = [&](int k, int r) { return S[(size_t)k * nr + r]; };
  auto u_of = [&](int k, int r) { return U[(size_t)k * nr + r]; };
  // list-scheduling durations (chain_durations); a tile update over g panels is estimated at b (0.25 + 0.75 g):
  // the C read / write and the pipeline fill are paid once per task
  const float* dur = chain_durations();
  // Deferred tile updates: the panels of group [q0, q1) (G panels) are applied to a tile of block column j
  // by ONE task of depth 128 (q1 - q0) when j >= q1 + L -- the column is not needed until L steps after
  // the group's last panel solve; the columns nearer the diagonal take each panel on its own (depth 128),
  // so the diagonal chain never waits for a deep update.  G = 1 disables it.
  const int G = group, Gc = kn.group_corner, tail_c = kn.corner_tail, LA = kn.group_la, Gn = kn.group_near;
  bool overflow = false;  // a task with more than MAXDEP dependencies (unreachable: bounded by construction)
  auto add = [&](const Task& t) {
    if (t.nd > MAXDEP) overflow = true;
    T.push_back(t);
    return (int)T.size() - 1;
  };
  // BLK tasks carry ty = 3 | (g - 1) << 2 for an update over the g panels k .. k + g - 1
  auto blk = [&](int q0, int g, int i, int jj) {
    const int ql = q0 + g - 1;  // (S(ql, r) done implies S(q, r) done for every q < ql that has an S task)
    if (!live(i, ql) || !live(jj, ql)) return;  // (identity rows: zero in every panel of the group)
    // (identity rows: the group's leading panels in which either block is still zero are left out -- their
    // products are exact zeros, so the tile's bits are those of the launch path, which includes or skips them)
    const int f = std::max(live_from(i), live_from(jj));
    if (f > q0) {
      g -= f - q0;
      q0 = f;
    }
    Task t = mk(CHT_BLK | ((g - 1) << 2), q0, i, jj, dur[3] * (0.25f + 0.75f * (float)g));
    for (int s = 4 * i; s <= std::min(4 * i + 3, rlast); ++s) t.dep(s_of(ql, s));
    if (jj != i)
      for (int s = 4 * jj; s <= std::min(4 * jj + 3, rlast); ++s) t.dep(s_of(ql, s));
    int& lu = last_upd[(size_t)i * nbt + jj];
    if (lu >= 0)
      t.dep(lu);
    else if (q0 > 0)
      t.ty |= kChainFirst;
    lu = add(t);
  };
  // the next diagonal block's update by panel k, split by 32-column quarter (UQ: U32 with the quarter + 1 in
  // the type word's bits 2..7): 10 tasks of 32 x 32 x 128 on the chain to D(k + 1) instead of 4 of 32 x 128 x
  // 128, each loading 64 KB of panel instead of 160 (chain_uq; 0: one U32 per slice)
  const bool uq = chain_uq != 0, sq = chain_uq == 2;
  std::vector<std::vector<int>> uq_of(nr);  // slice s of diagonal block k + 1 -> its UQ tasks (panel k)
  for (int k = 0; k < nblk; ++k) {
    Task d = mk(CHT_D, k, 0, k, dur[0]);
    if (k > 0)
      for (int s = 4 * k; s <= std::min(4 * k + 3, rlast); ++s) {
        if (uq)
          for (int t : uq_of[s]) d.dep(t);
        else
          d.dep(u_of(k - 1, s));
      }
    D[k] = add(d);
    for (int r = 4 * (k + 1); r <= rlast; ++r) {
      if (!live(r / 4, k)) continue;
      if (kn.s128 && r >= 4 * (k + 2)) {
        // chain_s128: below the next diagonal block, a block row's slices take ONE panel-solve task (S with g = the
        // slice count in the type word's bits 2..5: the slices solved one after another, each as its own S task would)
        if (r % 4 != 0) continue;
        const int g = std::min(4, rlast - r + 1);
        Task t = mk(CHT_S | ((g - 1) << 2), k, r, 0, dur[1] * (0.5f + 0.5f * (float)g));
        t.dep(D[k]);
        if (k > 0 && live(r / 4, k - 1)) {
          for (int s2 = r; s2 < r + g; ++s2) {
            const int u = u_of(k - 1, s2);
            bool dup = false;
            for (int e = 0; e < t.nd && e < MAXDEP; ++e) dup = dup || t.deps[e] == u;
            if (!dup) t.dep(u);
          }
        } else if (k > 0) {
          t.ty |= kChainFirst;
        }
        const int id = add(t);
        for (int s2 = r; s2 < r + g; ++s2) S[(size_t)k * nr + s2] = id;
        continue;
      }
      // chain_uq 2: the next diagonal block's slices take SQ tasks -- the panel solve followed by the slice's lower
      // quarters of that block (chain_sq), which need the siblings' solved rows (claimed before: lower slices first)
      const bool sqt = sq && k + 1 < nblk && r < 4 * (k + 2);
      Task t = mk(CHT_S | (sqt ? kChainSq : 0), k, r, 0, dur[1] + (sqt ? dur[2] * 0.5f : 0.f));
      t.dep(D[k]);
      if (k > 0 && live(r / 4, k - 1))
        t.dep(u_of(k - 1, r));
      else if (k > 0)
        t.ty |= kChainFirst;  // (the slice's first live panel: nothing updated it before)
      if (sqt) {
        const int lu = last_upd[(size_t)(k + 1) * nbt + (k + 1)];
        if (lu >= 0) t.dep(lu);
        for (int q = 4 * (k + 1); q < r; ++q) t.dep(s_of(k, q));
      }
      S[(size_t)k * nr + r] = add(t);
      if (sqt) {
        uq_of[r].push_back(S[(size_t)k * nr + r]);
        U[(size_t)k * nr + r] = S[(size_t)k * nr + r];
      }
    }
    for (int r = 4 * (k + 1); r <= rlast; ++r) {
      if (!live(r / 4, k)) continue;
      if (sq && k + 1 < nblk && r < 4 * (k + 2)) continue;  // (done by the slice's SQ task)
      const int lu = last_upd[(size_t)(r / 4) * nbt + (k + 1)];
      const int first = (lu < 0 && k > 0) ? kChainFirst : 0;
      if (uq && k + 1 < nblk && r < 4 * (k + 2)) {
        const int rl = r - 4 * (k + 1);
        for (int q = 0; q <= rl; ++q) {  // lower quarters of the diagonal block's slice r
          Task t = mk(CHT_U32 | ((q + 1) << 2) | first, k, r, k + 1, dur[2] * 0.5f);
          t.dep(s_of(k, r));
          if (q != rl) t.dep(s_of(k, 4 * (k + 1) + q));
          if (lu >= 0) t.dep(lu);
          uq_of[r].push_back(add(t));
        }
        U[(size_t)k * nr + r] = uq_of[r].back();  // (not read: D(k + 1) waits for every quarter)
        continue;
      }
      if (kn.u128 && r >= 4 * (k + 2)) {
        // chain_u128: below the next diagonal block, the four slices of a block row take ONE 128 x 128 tile update
        // over panel k (a BLK task: the same k-steps, half the CU time of four slice updates); it publishes every
        // slice's counter, so each slice's next panel solve waits for the block row instead of its own slice
        if (r % 4 == 0 || r == 4 * (k + 2)) {
          blk(k, 1, r / 4, k + 1);
          const int bt = last_upd[(size_t)(r / 4) * nbt + (k + 1)];
          for (int s2 = r; s2 <= std::min(4 * (r / 4) + 3, rlast); ++s2) U[(size_t)k * nr + s2] = bt;
        }
        continue;
      }
      Task t = mk(CHT_U32 | first, k, r, k + 1, dur[2]);
      t.dep(s_of(k, r));
      for (int s = 4 * (k + 1); s <= std::min(4 * (k + 1) + 3, rlast); ++s)
        if (s != r) t.dep(s_of(k, s));
      if (lu >= 0) t.dep(lu);
      U[(size_t)k * nr + r] = add(t);
    }
    for (int jj = k + 2; jj <= yb; ++jj) {
      // identity-augmented lists: the corner's columns (jj >= nblk) are read by no later task -- only the
      // read-out and the gradient use -K^-1 -- so their tiles take deeper groups (chain_group_corner)
      // (the corner's last updates wait for the last panel solves and form the factorisation's tail: the last
      // tail_c panels keep depth G)
      const bool corner = eye && jj >= nblk;
      const int qlim = corner ? std::max(0, nblk - tail_c) : 0;
      int q0, q1;
      if (corner && k < qlim) {
        q0 = k / Gc * Gc;
        q1 = std::min(q0 + Gc, qlim);
      } else {
        q0 = qlim + (k - qlim) / G * G;
        q1 = std::min(q0 + G, nblk);
      }
      const bool grouped = q1 - q0 > 1 && jj >= q1 + LA;
      if (grouped && k != q1 - 1) continue;  // the group's one task comes with its last panel
      // the columns too near the diagonal for the group (chain_group_near > 1): sub-groups of Gn panels of the
      // group, under the same rule (a column at least LA past the sub-group's last panel), else panel by panel
      const int p0 = q0 + (k - q0) / Gn * Gn, p1 = std::min(p0 + Gn, q1);
      const bool sub = !grouped && p1 - p0 > 1 && jj >= p1 + kn.near_la;
      if (sub && k != p1 - 1) continue;
      for (int i = jj; i <= yb; ++i) {
        if (grouped)
          blk(q0, q1 - q0, i, jj);
        else if (sub)
          blk(p0, p1 - p0, i, jj);
        else
          blk(k, 1, i, jj);
      }
    }
  }
  // independent members (a small batch): one copy of the graph per member, tagged in the type word's bits
  // 8.. (task fields: ty | (g - 1) << 2 | member << 8), scheduled together so that every member's diagonal
  // chain runs beside the others' tile updates
  if (nmem > 1) {
    const int n1 = (int)T.size();
    T.reserve((size_t)n1 * nmem);
    for (int m = 1; m < nmem; ++m)
      for (int t = 0; t < n1; ++t) {
        Task c = T[t];
        c.ty |= m << 8;
        for (int e = 0; e < c.nd; ++e) c.deps[e] += m * n1;
        T.push_back(c);
      }
  }
  if (overflow) return {};
  const int n = (int)T.size();
  // successors in CSR form, each task's in the order its dependants were built
  std::vector<int> indeg(n, 0), soff(n + 1, 0);
  for (int t = 0; t < n; ++t)
    for (int e = 0; e < T[t].nd; ++e) ++soff[T[t].deps[e] + 1];
  for (int t = 0; t < n; ++t) soff[t + 1] += soff[t];
  std::vector<int> succ(soff[n]), fill(soff.begin(), soff.end() - 1);
  for (int t = 0; t < n; ++t)
    for (int e = 0; e < T[t].nd; ++e) {
      succ[fill[T[t].deps[e]]++] = t;
      ++indeg[t];
    }
  std::vector<float> bl(n, 0.f);
  for (int t = n - 1; t >= 0; --t) {  // the construction order is topological
    float m = 0.f;
    for (int e = soff[t]; e < soff[t + 1]; ++e) m = std::max(m, bl[succ[e]]);
    bl[t] = T[t].dur + m;
  }
  auto cmp = [&](int a, int b) { return bl[a] != bl[b] ? bl[a] < bl[b] : a > b; };
  std::priority_queue<int, std::vector<int>, decltype(cmp)> ready(cmp);
  std::priority_queue<std::pair<float, int>, std::vector<std::pair<float, int>>, std::greater<std::pair<float, int>>> ev;
  for (int t = 0; t < n; ++t)
    if (indeg[t] == 0) ready.push(t);
  std::vector<int32_t> out;
  out.reserve((size_t)n * 4);
  int free = std::max(1, grid);
  float now = 0.f;
  while ((int)out.size() < 4 * n) {
    while (free > 0 && !ready.empty()) {
      const int t = ready.top();
      ready.pop();
      out.insert(out.end(), {T[t].ty, T[t].k, T[t].r, T[t].j});
      ev.push({now + T[t].dur, t});
      --free;
    }
    if (ev.empty()) break;  // (cannot happen for a well-formed graph)
    const auto e = ev.top();
    ev.pop();
    now = e.first;
    ++free;
    for (int x = soff[e.second]; x < soff[e.second + 1]; ++x)
      if (--indeg[succ[x]] == 0) ready.push(succ[x]);
  }
  return out;
}

// chain_kernel applies to one f64 member (or a small batch) without ragged rows -- identity extra rows
// included (chain_eye) --, on a stream that is not being captured (the first call of a shape uploads its task
// list), up to chain_max_p (identity rows: chain_max_p_eye) rows; f32 (chain_f32) without identity rows
bool chain_applies(const gpk_layout* lay, bool eye, const int64_t* n_dev, const int64_t* m_dev, const Tune& tn,
                   hipStream_t s) {
  const bool dt_ok = lay->dtype == GPK_F64 || (lay->dtype == GPK_F32 && tn.chain_f32 != 0 && !eye);
  if (!tn.chain || !dt_ok || (eye && !tn.chain_eye) || n_dev || m_dev) return false;
  if (lay->batch == 1 ? lay->p > (eye ? tn.chain_max_p_eye : tn.chain_max_p)
                      : (lay->batch > tn.chain_max_batch || lay->batch * lay->p > tn.chain_batch_max_rows))
    return false;
  if (tn.diag_dbg != 0 || tn.diag_version == 1) return false;
  if (!plain_stream(s)) return false;
  if (tn.chain == 1 && lay->p < (eye ? tn.chain_min_p_eye : tn.chain_min_p)) return false;
  if (tn.chain == 1 && other_stream_busy(s)) {
    ++g_chain_declined;
    return false;
  }
  return true;
}

int chain_potrf(const gpk_layout* lay, void* W, void* Winv, int32_t* info_dev, const Tune& tn, hipStream_t s,
                bool eye) {
  int dev = 0, ncu = 0;
  GPK_HIP(hipGetDevice(&dev), "device");
  GPK_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev), "device");
  const int grid = tn.chain_grid > 0 ? (int)tn.chain_grid : ncu;
  ChainPlan plan;
  int32_t* ctl = nullptr;
  size_t ctl_ints = 0;
  {
    std::lock_guard<std::mutex> lk(g_chain_mu);
    const ChainKnobs kn = chain_knobs(tn, lay->n_pad, eye, lay->dtype == GPK_F32, grid);
    const int nmem = lay->batch;
    // (two lists need workgroups of both roles: at least 8 per XCD)
    const int xcd = tn.chain_xcd != 0 && grid >= 64 ? 1 : 0;
    auto key = std::make_tuple(dev, lay->n_pad, lay->y_row, grid, nmem, eye ? 1 : 0, kn.group, kn.uq,
                               kn.group_corner, kn.corner_tail, kn.group_la, xcd, kn.group_near, kn.u128,
                               kn.near_la, kn.s128);
    auto it = g_chain_plans.find(key);
    if (it == g_chain_plans.end()) {
      std::vector<int32_t> ord = chain_order(lay->n_pad, lay->y_row, grid, nmem, kn, eye);
      if (ord.empty()) {
        // (an internal failure, not a bad argument: reported like a HIP error, > 0)
        return fail_hip(hipErrorUnknown, "chain_order: a task exceeds the device's dependency bound");
      }
      ChainPlan p;
      p.ntasks_b = xcd ? chain_split_lists(ord) : 0;
      p.ntasks = (int32_t)(ord.size() / 4) - p.ntasks_b;
      p.nblk = (int32_t)(lay->n_pad / NB);
      p.nsl = (int32_t)(lay->y_row / 32 + 1);
      p.nbc = (int32_t)(lay->y_row / NB + 1);
      GPK_HIP(hipMalloc(&p.tasks, ord.size() * sizeof(int32_t)), "chain tasks");
      GPK_HIP(hipMemcpy(p.tasks, ord.data(), ord.size() * sizeof(int32_t), hipMemcpyHostToDevice), "chain tasks");
      it = g_chain_plans.emplace(key, p).first;  // owned for the life of the process
    }
    plan = it->second;
    ctl_ints = 4 + (size_t)lay->batch * (2 * (size_t)plan.nblk + 2 * (size_t)plan.nblk * plan.nsl + (size_t)plan.nsl * plan.nbc);
    ctl_ints = (ctl_ints + 3) / 4 * 4;
  }
  {
    auto& c = t_chain_ctl.blocks[{dev, s}];  // this thread's own (see t_chain_ctl)
    if (c.second < ctl_ints) {
      // (hipFree synchronises the device: no launch of this thread still uses the old block)
      if (c.first) GPK_HIP(hipFree(c.first), "chain scratch");
      c = {nullptr, 0};
      GPK_HIP(hipMalloc(&c.first, ctl_ints * sizeof(int32_t)), "chain scratch");
      c.second = ctl_ints;
    }
    ctl = c.first;
  }
  // every counter starts at zero in every call
  GPK_HIP(hipMemsetAsync(ctl, 0, ctl_ints * sizeof(int32_t), s), "chain memset");
  ChainArgs a;
  memset(&a, 0, sizeof(a));
  a.W = W;
  a.ld = lay->ld;
  a.Winv = Winv;
  a.info = info_dev;
  a.tasks = plan.tasks;
  a.ntasks = env_i64("GPK_CHAIN_MAX_TASKS", 0) > 0 ? (int32_t)std::min<int64_t>(plan.ntasks, env_i64("GPK_CHAIN_MAX_TASKS", 0)) : plan.ntasks;  // (debugging)
  a.ntasks_b = plan.ntasks_b;
  if (a.ntasks_b > 0) a.ntasks = plan.ntasks;  // (GPK_CHAIN_MAX_TASKS: one list only)
  a.xcd_b = plan.ntasks_b > 0 ? 0 : -1;
  a.b_seats = (int32_t)std::max<int64_t>(1, std::min<int64_t>(tn.chain_xcd_seats, grid / 16));
  a.dbg = (int32_t)env_i64("GPK_CHAIN_DBG", 0);
  a.ctl = ctl;
  a.dflag = ctl + 4;
  a.sdone = a.dflag + plan.nblk;
  a.ucnt = a.sdone + (size_t)plan.nblk * plan.nsl;
  a.qdone = a.ucnt + (size_t)plan.nsl * plan.nbc;
  a.hflag = a.qdone + (size_t)plan.nblk * plan.nsl;
  a.nsl = plan.nsl;
  a.nbc = plan.nbc;
  a.nmem = lay->batch;
  a.w_bs = lay->w_batch_stride;
  a.inv_bs = lay->inv_batch_stride;
  a.ctl_stride = 2 * (int64_t)plan.nblk + 2 * (int64_t)plan.nblk * plan.nsl + (int64_t)plan.nsl * plan.nbc;
  a.uq = (int32_t)chain_knobs(tn, lay->n_pad, eye, lay->dtype == GPK_F32, grid).uq;
  // rows of L_kk^-1 behind D's early flag: later (more of the panel solve early) for short chains, where the
  // diagonal chain is all there is; earlier for long ones, where the S tasks' waiting CUs cost tile-update time
  // (N = 4096: 112 rows 1.501 vs 96 rows 1.515 ms; 6144 / 8192 2.42 / 4.44 vs 2.37 / 4.39, profiles/r04ab_*)
  a.half_step = (plan.nblk <= 32 ? GPK_CHAIN_SHALF_ROWS_SMALL : GPK_CHAIN_SHALF_ROWS) / 16;
  a.row_end = lay->y_row + 1;
  a.timeout = std::max<int64_t>(1, tn.chain_timeout_ms) * 100000;  // 100 MHz ticks
  for (int64_t f = g_chain_force_timeout.load(); f > 0;)
    if (g_chain_force_timeout.compare_exchange_weak(f, f - 1)) {
      a.force_abort = 1;
      break;
    }
  if (env_i64("GPK_CHAIN_TIMES", 0)) {
    std::lock_guard<std::mutex> lk(g_chain_mu);
#ifndef GPK_DIAG_PROF
#define GPK_DIAG_PROF 0
#endif
    // (GPK_DIAG_PROF builds: the D tasks' phase stamps follow the task stamps, 8 steps x 8 waves x 6 per block,
    // read back as extra "tasks" of gpk_chain_times)
    const int64_t extra = GPK_DIAG_PROF ? (int64_t)plan.nblk * 8 * 8 : 0;
    const int64_t nt = (int64_t)a.ntasks + a.ntasks_b;
    if (g_chain_times_n < nt + extra) {
      if (g_chain_times) hipFree(g_chain_times);
      GPK_HIP(hipMalloc(&g_chain_times, (size_t)(nt + extra) * 6 * sizeof(uint64_t)), "chain times");
      g_chain_times_n = nt + extra;
    }
    a.times = g_chain_times;
    if (extra) a.dprof = g_chain_times + (size_t)nt * 6;
  }
  if (env_i64("GPK_CHAIN_TRACE", 0)) {
    std::lock_guard<std::mutex> lk(g_chain_mu);
    if (!g_chain_trace) GPK_HIP(hipHostMalloc(&g_chain_trace, 4096 * 32 * sizeof(int32_t), hipHostMallocCoherent), "trace");
    memset(g_chain_trace, 0xff, 4096 * 32 * sizeof(int32_t));
    a.trace = grid <= 4096 ? g_chain_trace : nullptr;
  }
  const double n3 = (double)lay->n_pad;
  GPK_HIP(timed(3, lay->batch * n3 * n3 * n3 / (eye ? 1.0 : 3.0), 0.0, s, [&] { return launch_chain(a, lay->dtype, grid, s); }),
          "chain");
  ++g_chain_launches;
  t_chain_last = true;
  return 0;
}

}  // namespace

namespace gpk {
bool tune_asm_feat() { return tune_now().asm_feat != 0; }
bool tune_asm_f32_fast() { return tune_now().asm_f32_fast != 0; }
int tune_asm_f32_chunk() { return (int)std::max<int64_t>(1, std::min<int64_t>(64, tune_now().asm_f32_chunk)); }
}  // namespace gpk

extern "C" {

int gpk_abi_version(void) { return GPK_ABI_VERSION; }

const char* gpk_last_error(void) { return g_err.c_str(); }

int gpk_plan(int dtype, int32_t batch, int64_t n, int64_t m, int64_t d, gpk_layout* out) {
  if (dtype != GPK_F64 && dtype != GPK_F32) return fail_arg(1, "dtype");
  if (batch <= 0) return fail_arg(2, "batch must be > 0");
  if (n <= 0) return fail_arg(3, "n must be > 0");
  if (m < 0) return fail_arg(4, "m must be >= 0");
  if (d <= 0 || d > GPK_MAX_DIM) return fail_arg(5, "d must be in [1, 16]");
  if (!out) return fail_arg(6, "out");
  gpk_layout L;
  memset(&L, 0, sizeof(L));
  L.dtype = dtype;
  L.batch = batch;
  L.n = n;
  L.m = m;
  L.d = d;
  L.nb = NB;
  L.n_pad = (n + NB - 1) / NB * NB;
  L.y_row = L.n_pad + m;
  L.p = (L.y_row + 1 + NB - 1) / NB * NB;
  L.ld = L.p;
  L.w_batch_stride = L.p * L.ld;
  L.inv_batch_stride = (L.n_pad / NB) * NB * NB;
  L.w_bytes = (size_t)batch * (size_t)L.w_batch_stride * elem_size(dtype);
  L.inv_bytes = (size_t)batch * (size_t)L.inv_batch_stride * elem_size(dtype);
  *out = L;
  return 0;
}

static int check_layout(const gpk_layout* lay) {
  if (!lay) return fail_arg(1, "layout");
  if ((lay->dtype != GPK_F64 && lay->dtype != GPK_F32) || lay->batch <= 0 || lay->nb != NB ||
      lay->n_pad % NB != 0 || lay->p % NB != 0 || lay->ld < lay->p || lay->y_row >= lay->p ||
      lay->n <= 0 || lay->n > lay->n_pad)
    return fail_arg(1, "layout (use gpk_plan)");
  return 0;
}

static int assemble_impl(const gpk_kdesc* kd, const gpk_layout* lay, const double* hyp_dev,
                         int64_t hyp_stride, const double* noise_dev, int64_t noise_stride,
                         const double* X, int64_t x_bstride, const double* Xs, int64_t xs_bstride,
                         const double* E, int64_t e_bstride, const double* y, int64_t y_bstride,
                         void* W, bool eye, const int64_t* n_dev, const int64_t* m_dev, void* stream,
                         int64_t tcol_hi = 0) {
  if (int e = check_layout(lay)) return e;
  if (!valid_kdesc(kd, lay->d)) return fail_arg(1, "kernel descriptor");
  if (!hyp_dev && kd->n_hyp > 0) return fail_arg(3, "hyp_dev");
  if (!noise_dev) return fail_arg(5, "noise_dev");
  if (!X) return fail_arg(7, "X");
  if (eye && lay->m != lay->n) return fail_arg(2, "identity extra rows need a layout planned with m = n");
  if (lay->m > 0 && !Xs && !E && !eye) return fail_arg(9, "Xs or E");
  if (!y) return fail_arg(13, "y");
  if (!W) return fail_arg(15, "W");
  AsmArgs a;
  memset(&a, 0, sizeof(a));
  a.generic = tune_now().asm_generic != 0 ? 1 : 0;
  a.hyp = hyp_dev;
  a.hyp_stride = hyp_stride;
  a.noise = noise_dev;
  a.noise_stride = noise_stride;
  a.X = X;
  a.x_bs = x_bstride;
  a.Xs = Xs ? Xs : X;
  a.xs_bs = xs_bstride;
  a.E = (lay->m > 0) ? E : nullptr;
  a.e_bs = e_bstride;
  a.y = y;
  a.y_bs = y_bstride;
  a.W = W;
  a.ld = lay->ld;
  a.w_bs = lay->w_batch_stride;
  a.n = lay->n;
  a.m = lay->m;
  a.n_pad = lay->n_pad;
  a.y_row = lay->y_row;
  a.p = lay->p;
  a.d = (int32_t)lay->d;
  a.dp = (lay->d % 2 == 0) ? (int32_t)lay->d + 1 : (int32_t)lay->d;
  a.plain = 0;
  a.eye = eye ? 1 : 0;
  a.ntile = lay->p / ATILE;
  a.nb = n_dev;
  a.mb = m_dev;
  a.tcol_hi = tcol_hi;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const double es = (double)elem_size(lay->dtype);
  const double cols = (tcol_hi > 0 && tcol_hi < a.ntile) ? (double)(tcol_hi * ATILE) : (double)lay->p;
  const double bytes = (double)lay->batch *
                       (es * (cols * (double)lay->p - cols * (cols - (double)ATILE) / 2.0) +
                        8.0 * (double)(lay->n + lay->m) * (double)lay->d + 8.0 * (double)lay->n);
  GPK_HIP(timed(0, 0.0, bytes, s, [&] { return launch_assemble(*kd, a, lay->dtype, lay->batch, s); }),
          "assemble");
  return 0;
}

int gpk_assemble(const gpk_kdesc* kd, const gpk_layout* lay, const double* hyp_dev,
                 int64_t hyp_stride, const double* noise_dev, int64_t noise_stride,
                 const double* X, int64_t x_bstride, const double* Xs, int64_t xs_bstride,
                 const double* E, int64_t e_bstride, const double* y, int64_t y_bstride,
                 void* W, void* stream) {
  return assemble_impl(kd, lay, hyp_dev, hyp_stride, noise_dev, noise_stride, X, x_bstride, Xs,
                       xs_bstride, E, e_bstride, y, y_bstride, W, false, nullptr, nullptr, stream);
}

int gpk_assemble_ragged(const gpk_kdesc* kd, const gpk_layout* lay, const double* hyp_dev,
                        int64_t hyp_stride, const double* noise_dev, int64_t noise_stride,
                        const double* X, int64_t x_bstride, const double* Xs, int64_t xs_bstride,
                        const double* y, int64_t y_bstride, const int64_t* n_dev, const int64_t* m_dev,
                        void* W, void* stream) {
  if (!n_dev) return fail_arg(13, "n_dev");
  if (lay && lay->m > 0 && !m_dev) return fail_arg(14, "m_dev (layout planned with m > 0)");
  return assemble_impl(kd, lay, hyp_dev, hyp_stride, noise_dev, noise_stride, X, x_bstride, Xs,
                       xs_bstride, nullptr, 0, y, y_bstride, W, false, n_dev, lay && lay->m > 0 ? m_dev : nullptr,
                       stream);
}

int gpk_assemble_inverse(const gpk_kdesc* kd, const gpk_layout* lay, const double* hyp_dev,
                         int64_t hyp_stride, const double* noise_dev, int64_t noise_stride,
                         const double* X, int64_t x_bstride, const double* y, int64_t y_bstride,
                         void* W, void* stream) {
  return assemble_impl(kd, lay, hyp_dev, hyp_stride, noise_dev, noise_stride, X, x_bstride, nullptr,
                       0, nullptr, 0, y, y_bstride, W, true, nullptr, nullptr, stream);
}

static int potrf_impl(const gpk_layout* lay, void* W, void* Winv, int32_t* info_dev, int32_t flags,
                      const int64_t* n_dev, const int64_t* m_dev, void* stream, const GemmArgs* kb = nullptr) {
  if (int e = check_layout(lay)) return e;
  if (!W) return fail_arg(2, "W");
  if (!Winv) return fail_arg(3, "Winv");
  if (!info_dev) return fail_arg(4, "info_dev");
  if (flags & ~GPK_AUG_EXTRA_IDENTITY) return fail_arg(5, "flags");
  const bool eye = (flags & GPK_AUG_EXTRA_IDENTITY) != 0;
  if (eye && lay->m != lay->n) return fail_arg(1, "identity extra rows need a layout planned with m = n");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int dt = lay->dtype;
  const size_t es = elem_size(dt);
  const int64_t nblk = lay->n_pad / NB;

  // one snapshot of the knobs per call: a gpk_tune from another thread (ctypes releases the GIL during
  // the enqueue) must not change the fuse decision between a panel's diag(k) and trsm(k)
  const Tune tn = tune_now();
  t_chain_last = false;
  // a single evaluation: the whole factorisation as one persistent launch (no K build fused into it)
  if (!kb && chain_applies(lay, eye, n_dev, m_dev, tn, s)) {
    const int e = chain_potrf(lay, W, Winv, info_dev, tn, s, eye);
    if (!e) note_factorisation(s);
    return e;
  }
  // The panel chain (diag, panel solve, thin and look-ahead updates) runs on a high-priority
  // stream, the bulk of each trailing update on a CU-masked stream concurrently with the next
  // panel pair's chain; both fork from and join back into the caller's stream.
  // GPK_LOOKAHEAD=0 puts everything on the caller's stream.
  // Auto (2): on when the augmented matrix has at least la_min_blocks 128-blocks.  Below that the
  // whole factorisation is faster on the caller's stream alone: each launch on the side streams costs
  // ~5 us more than back to back on one queue, more than the overlap of the short trailing updates
  // saves.  ms per call, look-ahead off / on (profiles/r02s_lookahead.txt): one member N = 1024
  // 0.45 / 0.55, 2048 0.92 / 1.09, 4096 2.10 / 2.29, 6144 3.98 / 4.03, 8192 6.53 / 6.40, 12288
  // 15.3 / 14.5; batches of 8 at N = 4096 5.13 / 5.26; the 128-candidate C4 sweep 52.7 / 54.2;
  // -LML + gradient (identity rows: twice the width) N = 4096 3.44 / 3.28.  With the panel solve fused
  // (look-ahead off only): N = 6144 3.89 / 4.02, 7168 5.01 / 5.05, 8192 6.43 / 6.39 -> 64 blocks.
  const bool la = tn.lookahead == 1 || (tn.lookahead == 2 && lay->p / NB >= tn.la_min_blocks);
  SideStream* ss = nullptr;
  if (la) {
    ss = side_stream();
    if (!ss) return fail_hip(hipErrorInvalidValue, "side stream");
  }
  hipStream_t sp = !la ? s : tn.panel_stream == 1 ? s : tn.panel_stream == 2 ? ss->panel_np : ss->panel_s;
  hipStream_t sb = la ? ss->bulk_s : s;

  // extra rows that are nonzero in panel columns left of c: all test rows, or the identity rows
  // t < c (row n_pad + t of E L^-T is zero left of column t)
  auto extra_nonzero = [&](int64_t c) -> double {
    return (double)(eye ? std::min<int64_t>(lay->m, c) : lay->m);
  };
  // Small grids (f64): the panel solve of block k runs inside the diagonal-block launch -- one
  // workgroup per 64-row tile (plus the one that writes L and L^-1), each factoring the block
  // redundantly (the chip is otherwise idle there) and solving its rows against L^-1 in LDS, bitwise
  // the separate gemm<TRSM>; one launch fewer on the chain per panel.
  int32_t* const ctr = (dt == GPK_F64 && tn.fuse_trsm) ? fuse_counters(sp) : nullptr;
  auto fused_tiles = [&](int64_t k) -> int64_t {
    const int64_t rows = lay->p - (k + 1) * NB;
    if (!ctr) return 0;  // no counters for this stream: the separate panel-solve launch
    // (the timing-only ablations of the diagonal kernel skip the writer's counter reset: never fused)
    if (dt != GPK_F64 || !tn.fuse_trsm || tn.diag_version == 1 || tn.diag_dbg != 0 || rows <= 0) return 0;
    if (la && tn.fuse_trsm != 2) return 0;  // beside the look-ahead's bulk updates the extra workgroups
                                             // cost more than the launch saves (N = 8192: 6.39 -> 6.43 ms)
    const int64_t t64 = rows / 64;
    return (t64 + 1) * lay->batch <= tn.fuse_trsm_max && lay->batch <= kFuseCtr ? t64 : 0;
  };
  // diagonal block k: factor + invert
  auto diag = [&](int64_t k) -> hipError_t {
    DiagArgs da;
    memset(&da, 0, sizeof(da));
    da.W = W;
    da.ld = lay->ld;
    da.w_bs = lay->w_batch_stride;
    da.Winv = Winv;
    da.inv_bs = lay->inv_batch_stride;
    da.j0 = k * NB;
    da.kblk = k;
    da.info = info_dev;
    da.dbg = (int32_t)tn.diag_dbg;
    da.version = (int32_t)tn.diag_version;
    da.trsm_tiles = (int32_t)fused_tiles(k);
    double flops = (double)lay->batch * NB * NB * NB / 3.0;
    if (da.trsm_tiles > 0) {
      da.row0 = (k + 1) * NB;
      da.p = lay->p;
      da.n_pad = lay->n_pad;
      da.y_row = lay->y_row;
      da.zlo = eye ? lay->n_pad + da.row0 : 0;  // identity rows t >= j0 + nb are still zero
      da.zhi = eye ? lay->y_row : 0;
      da.nb = n_dev;
      da.mb = m_dev;
      da.ctr = ctr;
      flops += (double)lay->batch * ((double)(lay->n_pad - da.row0) + extra_nonzero(da.row0)) * NB * NB;
    }
    return timed(1, flops, 0.0, sp, [&] { return launch_diag(da, dt, lay->batch, sp); });
  };
  GemmArgs base;
  memset(&base, 0, sizeof(base));
  base.W = W;
  base.ld = lay->ld;
  base.w_bs = lay->w_batch_stride;
  base.inv_bs = lay->inv_batch_stride;
  base.nb = n_dev;
  base.mb = m_dev;
  base.n_pad = lay->n_pad;
  base.y_row = lay->y_row;
  base.p = lay->p;
  base.row_end = tn.skip_zero_rows ? lay->y_row + 1 : 0;  // rows below the y row are zero
  // identity extra rows: the tiles wholly inside the zero band [zlo, zhi) are left out of the grid
  // (launched and exiting at once they would also crowd the live tiles onto a few XCDs, since
  // xcd_remap hands each XCD a contiguous run of tile ids).  c: a tile index from row0 -> its index
  // in the compressed enumeration.
  auto set_band = [&](GemmArgs& ga, int tile) {
    if (!eye || !tn.band_skip) return;
    const int64_t b0 = (ga.zlo - ga.row0) / tile, b1 = (ga.zhi - ga.row0) / tile;
    if (b1 <= b0) return;
    ga.bz0 = (int32_t)b0;
    ga.bzn = (int32_t)(b1 - b0);
  };
  auto compress = [](const GemmArgs& ga, int64_t c) -> int64_t {
    return ga.bzn == 0 || c < ga.bz0 ? c : (c >= (int64_t)ga.bz0 + ga.bzn ? c - ga.bzn : ga.bz0);
  };
  // panel solve of block k: every row below the block (the y / test rows included)
  auto trsm = [&](int64_t k) -> hipError_t {
    if (fused_tiles(k) > 0) return hipSuccess;  // solved by the diagonal-block launch
    GemmArgs ga = base;
    ga.Binv = static_cast<const char*>(Winv) + (size_t)k * NB * NB * es;
    ga.j0 = k * NB;
    ga.row0 = ga.j0 + NB;
    const int64_t rows = lay->p - ga.row0;
    if (rows <= 0) return hipSuccess;
    ga.kdepth = NB;
    if (eye) {  // identity rows t >= j0 + nb are still zero in this panel
      ga.zlo = lay->n_pad + ga.j0 + NB;
      ga.zhi = lay->y_row;
    }
    set_band(ga, 128);
    const int tile = (compress(ga, rows / NB) * lay->batch >= tn.trsm_t128_min) ? 128 : 64;
    ga.bz0 = ga.bzn = 0;
    set_band(ga, tile);
    ga.nt = (int32_t)compress(ga, rows / tile);
    // algorithmic: rows that are nonzero in the panel (K part + extra rows) x nb^2
    const double rK = (double)(lay->n_pad - ga.row0) + extra_nonzero(ga.j0 + NB);
    return timed(2, (double)lay->batch * rK * NB * NB, 0.0, sp,
                 [&] { return launch_gemm(ga, dt, GEMM_TRSM, tile, lay->batch, sp); });
  };
  // trailing update from panel columns [j0, j0 + kdepth) of the lower tiles whose 128-column
  // block lies in [c_lo, c_hi) (relative to row0 = j0 + kdepth; c_hi < 0: to the end)
  auto update = [&](int64_t j0, int kdepth, int64_t c_lo, int64_t c_hi, hipStream_t st,
                    bool fused_k = false) -> hipError_t {
    GemmArgs ga = base;
    if (fused_k && kb) {  // first trailing update: C is evaluated, not loaded (gpk_nlml's fused K build)
      ga.kbuild = 1;
      ga.d = kb->d;
      ga.n = kb->n;
      ga.node = kb->node;
      ga.hyp = kb->hyp;
      ga.hyp_stride = kb->hyp_stride;
      ga.noise = kb->noise;
      ga.noise_stride = kb->noise_stride;
      ga.X = kb->X;
      ga.x_bs = kb->x_bs;
      ga.y = kb->y;
      ga.y_bs = kb->y_bs;
    }
    ga.j0 = j0;
    ga.row0 = j0 + kdepth;
    ga.kdepth = kdepth;
    const int64_t rows = lay->p - ga.row0;
    if (rows <= 0) return hipSuccess;
    const int64_t t128 = rows / NB;
    if (c_hi < 0 || c_hi > t128) c_hi = t128;
    if (c_lo >= c_hi) return hipSuccess;
    if (eye) {  // identity rows t >= j0 + kdepth are zero in the panel columns
      ga.zlo = lay->n_pad + j0 + kdepth;
      ga.zhi = lay->y_row;
    }
    set_band(ga, 128);
    const int64_t w128 = compress(ga, c_hi) - compress(ga, c_lo);
    if (w128 <= 0) return hipSuccess;
    const int64_t tiles128 = w128 * (w128 + 1) / 2 + (compress(ga, t128) - compress(ga, c_hi)) * w128;
    const int tile = (tiles128 * lay->batch >= tn.upd_t128_min) ? 128 : 64;
    const int64_t scale = NB / tile;
    ga.bz0 = ga.bzn = 0;
    set_band(ga, tile);
    ga.nt = (int32_t)compress(ga, rows / tile);
    ga.c_lo = (int32_t)compress(ga, c_lo * scale);
    ga.c_hi = (int32_t)compress(ga, c_hi * scale);
    ga.band = (int32_t)std::max<int64_t>(0, tn.upd_band);
    // algorithmic flops: 2 kdepth x (lower-triangle elements in the column range of the rows that
    // are nonzero in the panel: the K part, then the extra rows, which follow it contiguously)
    const double rK = (double)(lay->n_pad - ga.row0) + extra_nonzero(j0 + kdepth);
    const double cl = std::min(rK, (double)(c_lo * NB)), ch = std::min(rK, (double)(c_hi * NB));
    const double elems = (ch - cl) * rK - (cl + ch - 1.0) * (ch - cl) / 2.0;
    // algorithmic bytes: the updated tiles' elements read + written once (y / test rows too)
    // and the panel rows read once
    const double rA = (double)rows;
    const double ca = (double)(c_lo * NB), cb = (double)(c_hi * NB);
    const double elems_all = (cb - ca) * rA - (ca + cb - 1.0) * (cb - ca) / 2.0;
    const double bytes = (double)lay->batch * (double)es * (2.0 * elems_all + rA * kdepth);
    return timed(3, (double)lay->batch * 2.0 * kdepth * std::max(0.0, elems), bytes, st,
                 [&] { return launch_gemm(ga, dt, GEMM_UPDATE, tile, lay->batch, st); });
  };

  // Groups of G 128-column panels per trailing update (K = 128 G): inside the group, block column k
  // is brought up to date with the group's earlier panels (one left-looking update of depth
  // 128 (k - g0)) and then factored and solved, ..., then update the trailing
  // matrix with all G panels at once -- its first G block columns (look-ahead, on the panel
  // stream: the next group's panels) and the rest (bulk stream, overlapping the next group's
  // panel chain).  A deeper K halves the read-modify-write passes over the trailing matrix per
  // doubling of G.  The first group has G0 <= G panels: its chain is exposed (nothing to overlap
  // yet), so a short one lets the first bulk update start early.
  // identity-augmented (gradient / inverse) factorisations: groups of group_eye panels -- their
  // trailing matrix carries the K^-1 corner, and 4-panel groups measured faster there at every batch
  const int64_t G = std::max<int64_t>(1, std::min<int64_t>(eye ? tn.group_eye : tn.group, 16));
  const int64_t G0 = std::max<int64_t>(1, std::min<int64_t>(tn.group_first, G));
  if (la) {
    GPK_HIP(hipEventRecord(ss->fork, s), "event");
    GPK_HIP(hipStreamWaitEvent(sp, ss->fork, 0), "event");
    GPK_HIP(hipStreamWaitEvent(sb, ss->fork, 0), "event");
  }
  // In-group updates.  Left-looking (throughput): block column k receives the group's earlier
  // panels in ONE update of depth 128 (k - g0) right before its diagonal block is factored
  // (right-looking updates read and write the group's columns once per panel).  Right-looking
  // (latency, small batches whose thin launches cannot fill the chip): after panel k, the group's
  // remaining columns receive panel k at depth 128 -- the chain to diag(k + 1) then carries one
  // short update instead of one of depth up to 128 (G - 1).
  // Two-level left-looking (ingroup 3): the group is split in halves; each half is left-looking
  // within itself, and between the halves ONE update of the second half's columns with the first
  // half's panels (depth 128 G/2) -- the thin launches re-read the half's panels instead of the
  // group's, 36 instead of 42 panel-column reads + writes per group of 8 (they are HBM-bound).
  const int64_t rows128 = lay->p / NB;
  const bool right_looking = tn.ingroup == 2 || (tn.ingroup == 0 && lay->batch * rows128 < tn.rl_max_tiles);
  const bool two_level = !right_looking && (tn.ingroup == 3 || tn.ingroup == 0) && G >= 4;
  bool bulk_pending = false;
  for (int64_t g0 = 0, gsize = G0; g0 < nblk; g0 += gsize, gsize = G) {
    const int64_t gend = std::min(g0 + gsize, nblk);
    const int64_t gmid = two_level ? std::min(g0 + (gend - g0 + 1) / 2, gend) : gend;
    for (int64_t k = g0; k < gend; ++k) {
      const int64_t h0 = k < gmid ? g0 : gmid;  // first panel of k's half
      if (two_level && k == gmid && gmid > g0)
        GPK_HIP(update(g0 * NB, (int)((gmid - g0) * NB), 0, gend - gmid, sp), "update half");
      if (!right_looking && k > h0) GPK_HIP(update(h0 * NB, (int)((k - h0) * NB), 0, 1, sp), "update thin");
      GPK_HIP(diag(k), "diag");
      GPK_HIP(trsm(k), "trsm");
      if (right_looking && k + 1 < gend) GPK_HIP(update(k * NB, NB, 0, gend - k - 1, sp), "update thin");
    }
    const int kd = (int)((gend - g0) * NB);
    if (!la) {
      GPK_HIP(update(g0 * NB, kd, 0, -1, s, g0 == 0), "update");
      continue;
    }
    GPK_HIP(hipEventRecord(ss->panel, sp), "event");      // panels g0 .. gend-1 solved
    if (bulk_pending) GPK_HIP(hipStreamWaitEvent(sp, ss->bulk, 0), "event");
    GPK_HIP(update(g0 * NB, kd, 0, G, sp, g0 == 0), "update look-ahead");
    GPK_HIP(hipStreamWaitEvent(sb, ss->panel, 0), "event");
    GPK_HIP(update(g0 * NB, kd, G, -1, sb, g0 == 0), "update bulk");
    GPK_HIP(hipEventRecord(ss->bulk, sb), "event");
    bulk_pending = true;
  }
  if (la) {
    GPK_HIP(hipEventRecord(ss->join_p, sp), "event");
    GPK_HIP(hipEventRecord(ss->join_b, sb), "event");
    GPK_HIP(hipStreamWaitEvent(s, ss->join_p, 0), "event");
    GPK_HIP(hipStreamWaitEvent(s, ss->join_b, 0), "event");
  }
  note_factorisation(s);
  return 0;
}

int gpk_potrf_aug_ex(const gpk_layout* lay, void* W, void* Winv, int32_t* info_dev, int32_t flags,
                     void* stream) {
  return potrf_impl(lay, W, Winv, info_dev, flags, nullptr, nullptr, stream);
}

int gpk_potrf_aug(const gpk_layout* lay, void* W, void* Winv, int32_t* info_dev, void* stream) {
  return potrf_impl(lay, W, Winv, info_dev, 0, nullptr, nullptr, stream);
}

int gpk_potrf_aug_ragged(const gpk_layout* lay, void* W, void* Winv, int32_t* info_dev,
                         const int64_t* n_dev, const int64_t* m_dev, void* stream) {
  if (!n_dev) return fail_arg(5, "n_dev");
  if (lay && lay->m > 0 && !m_dev) return fail_arg(6, "m_dev (layout planned with m > 0)");
  return potrf_impl(lay, W, Winv, info_dev, 0, n_dev, lay && lay->m > 0 ? m_dev : nullptr, stream);
}

static int finalize_impl(const gpk_layout* lay, const void* W, const int32_t* info_dev, const int64_t* n_dev,
                         double* out_dev, double* mu_dev, double* var_dev, void* stream) {
  if (int e = check_layout(lay)) return e;
  if (!W) return fail_arg(2, "W");
  if (!info_dev) return fail_arg(3, "info_dev");
  if (!out_dev) return fail_arg(4, "out_dev");
  FinArgs f;
  f.W = W;
  f.ld = lay->ld;
  f.w_bs = lay->w_batch_stride;
  f.n = lay->n;
  f.m = lay->m;
  f.n_pad = lay->n_pad;
  f.y_row = lay->y_row;
  f.info = info_dev;
  f.out = out_dev;
  f.mu = mu_dev;
  f.var = var_dev;
  f.nb = n_dev;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  GPK_HIP(timed(4, 0.0, 0.0, s, [&] { return launch_finalize(f, lay->dtype, lay->batch, s); }),
          "finalize");
  return 0;
}

int gpk_finalize(const gpk_layout* lay, const void* W, const int32_t* info_dev, double* out_dev,
                 double* mu_dev, double* var_dev, void* stream) {
  return finalize_impl(lay, W, info_dev, nullptr, out_dev, mu_dev, var_dev, stream);
}

int gpk_finalize_ragged(const gpk_layout* lay, const void* W, const int32_t* info_dev, const int64_t* n_dev,
                        double* out_dev, double* mu_dev, double* var_dev, void* stream) {
  if (!n_dev) return fail_arg(4, "n_dev");
  return finalize_impl(lay, W, info_dev, n_dev, out_dev, mu_dev, var_dev, stream);
}

int gpk_nlml_ragged(const gpk_kdesc* kd, const gpk_layout* lay, const double* hyp_dev, int64_t hyp_stride,
                    const double* noise_dev, int64_t noise_stride, const double* X, int64_t x_bstride,
                    const double* y, int64_t y_bstride, const int64_t* n_dev, void* W, void* Winv,
                    int32_t* info_dev, double* out_dev, void* stream) {
  if (int e = check_layout(lay)) return e;
  if (lay->m != 0) return fail_arg(2, "gpk_nlml_ragged needs a layout planned with m = 0");
  if (!n_dev) return fail_arg(11, "n_dev");
  if (!info_dev) return fail_arg(14, "info_dev");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  GPK_HIP(hipMemsetAsync(info_dev, 0, sizeof(int32_t) * lay->batch, s), "memset info");
  int e = gpk_assemble_ragged(kd, lay, hyp_dev, hyp_stride, noise_dev, noise_stride, X, x_bstride, nullptr, 0,
                              y, y_bstride, n_dev, nullptr, W, stream);
  if (e) return e;
  e = gpk_potrf_aug_ragged(lay, W, Winv, info_dev, n_dev, nullptr, stream);
  if (e) return e;
  return gpk_finalize_ragged(lay, W, info_dev, n_dev, out_dev, nullptr, nullptr, stream);
}

int gpk_nlml(const gpk_kdesc* kd, const gpk_layout* lay, const double* hyp_dev, int64_t hyp_stride,
             const double* noise_dev, int64_t noise_stride, const double* X, int64_t x_bstride,
             const double* y, int64_t y_bstride, void* W, void* Winv, int32_t* info_dev,
             double* out_dev, void* stream) {
  if (int e = check_layout(lay)) return e;
  if (lay->m != 0) return fail_arg(2, "gpk_nlml needs a layout planned with m = 0");
  if (!info_dev) return fail_arg(13, "info_dev");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  GPK_HIP(hipMemsetAsync(info_dev, 0, sizeof(int32_t) * lay->batch, s), "memset info");
  // Fused K build (single-base-node kernels): only the first panel group's block columns are
  // assembled; the first trailing update evaluates its C tiles instead of reading them, so the
  // trailing part of K is never written to HBM and read back.
  const Tune tn = tune_now();
  const int64_t nblk = lay->n_pad / NB;
  const int64_t G = std::max<int64_t>(1, std::min<int64_t>(tn.group, 16));
  const int64_t G0 = std::max<int64_t>(1, std::min<int64_t>(tn.group_first, G));
  const int op0 = kd ? kd->nodes[0].op : 0;
  if (tn.fuse_kbuild && lay->dtype == GPK_F64 && valid_kdesc(kd, lay->d) && kd->n_nodes == 1 && G0 < nblk &&
      !chain_applies(lay, false, nullptr, nullptr, tn, s) &&
      (op0 == GPK_OP_SE || op0 == GPK_OP_MAT32 || op0 == GPK_OP_MAT52)) {
    int e = assemble_impl(kd, lay, hyp_dev, hyp_stride, noise_dev, noise_stride, X, x_bstride, nullptr, 0,
                          nullptr, 0, y, y_bstride, W, false, nullptr, nullptr, stream, G0 * NB / ATILE);
    if (e) return e;
    GemmArgs kb;
    memset(&kb, 0, sizeof(kb));
    kb.d = (int32_t)lay->d;
    kb.n = lay->n;
    kb.node = kd->nodes[0];
    kb.hyp = hyp_dev;
    kb.hyp_stride = hyp_stride;
    kb.noise = noise_dev;
    kb.noise_stride = noise_stride;
    kb.X = X;
    kb.x_bs = x_bstride;
    kb.y = y;
    kb.y_bs = y_bstride;
    e = potrf_impl(lay, W, Winv, info_dev, 0, nullptr, nullptr, stream, &kb);
    if (e) return e;
    return gpk_finalize(lay, W, info_dev, out_dev, nullptr, nullptr, stream);
  }
  int e = gpk_assemble(kd, lay, hyp_dev, hyp_stride, noise_dev, noise_stride, X, x_bstride, nullptr,
                       0, nullptr, 0, y, y_bstride, W, stream);
  if (e) return e;
  e = gpk_potrf_aug(lay, W, Winv, info_dev, stream);
  if (e) return e;
  return gpk_finalize(lay, W, info_dev, out_dev, nullptr, nullptr, stream);
}

// ------------------------------------------------------------- workspace-style convenience entries
// The flat signatures of SURVEY §8(b): the caller hands one scratch buffer instead of a layout and
// W / Winv; the calls carve the augmented layout out of it and run the same kernels.
static size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

size_t gpk_workspace_bytes(int op, int dtype, int64_t n, int64_t m, int32_t batch) {
  (void)m;
  gpk_layout lay;
  if (n <= 0 || batch <= 0) return 0;
  if (op == GPK_WS_NLML) {
    if (gpk_plan(dtype, batch, n, 0, 1, &lay)) return 0;
    return align256(lay.w_bytes) + align256(lay.inv_bytes) + align256((size_t)batch * 4 * sizeof(double));
  }
  if (op == GPK_WS_POTRF) {
    if ((dtype != GPK_F64 && dtype != GPK_F32) || gpk_plan(dtype, 1, n, 0, 1, &lay)) return 0;
    return align256(lay.w_bytes) + align256(lay.inv_bytes) + align256(8 * sizeof(double)) +
           align256((size_t)n * sizeof(double));
  }
  const int64_t n_pad = (n + NB - 1) / NB * NB;
  const size_t winv = align256((size_t)n_pad * NB * sizeof(double));
  if (op == GPK_WS_TRSV) {
    if (dtype != GPK_F64) return 0;
    return winv + align256((size_t)n_pad * sizeof(double));
  }
  if (op == GPK_WS_POSTERIOR) {
    if (dtype != GPK_F64 || m <= 0) return 0;
    return winv + 2 * align256((size_t)n_pad * (size_t)m * sizeof(double)) + align256(8 * sizeof(double));
  }
  return 0;
}

int gpk_nlml_batched(const gpk_kdesc* kd, int32_t batch, const double* hyp_dev, const double* noise_dev, int dtype,
                     const double* X, const double* y, int64_t n, int32_t d, void* work, size_t work_bytes,
                     double* nlml_dev, int32_t* info_dev, void* stream) {
  if (!kd) return fail_arg(1, "kd");
  if (batch <= 0) return fail_arg(2, "batch");
  if (!nlml_dev) return fail_arg(12, "nlml_dev");
  gpk_layout lay;
  if (int e = gpk_plan(dtype, batch, n, 0, d, &lay)) return e;
  if (!work || work_bytes < gpk_workspace_bytes(GPK_WS_NLML, dtype, n, 0, batch)) return fail_arg(11, "work_bytes");
  char* w = reinterpret_cast<char*>(work);
  void* W = w;
  void* Winv = w + align256(lay.w_bytes);
  double* out = reinterpret_cast<double*>(w + align256(lay.w_bytes) + align256(lay.inv_bytes));
  if (int e = gpk_nlml(kd, &lay, hyp_dev, kd->n_hyp, noise_dev, 1, X, 0, y, 0, W, Winv, info_dev, out, stream))
    return e;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  GPK_HIP(hipMemcpy2DAsync(nlml_dev, sizeof(double), out, 4 * sizeof(double), sizeof(double), (size_t)batch,
                           hipMemcpyDeviceToDevice, s),
          "nlml_batched read-out");
  return 0;
}

static int potrf_lower_f32(float* A, int64_t n, int64_t lda, void* work, size_t work_bytes, int32_t* info_dev,
                           double* logdet_dev, void* stream) {
  gpk_layout lay;
  if (int e = gpk_plan(GPK_F32, 1, n, 0, 1, &lay)) return e;
  if (!work || work_bytes < gpk_workspace_bytes(GPK_WS_POTRF, GPK_F32, n, 0, 1)) return fail_arg(6, "work_bytes");
  char* w = reinterpret_cast<char*>(work);
  void* W = w;
  void* Winv = w + align256(lay.w_bytes);
  double* out = reinterpret_cast<double*>(w + align256(lay.w_bytes) + align256(lay.inv_bytes));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  GPK_HIP(hipMemsetAsync(info_dev, 0, sizeof(int32_t), s), "memset info");
  GPK_HIP(launch_pack_lower(GPK_F32, A, lda, n, lay.n_pad, lay.p, W, s), "potrf_lower pack");
  if (int e = gpk_potrf_aug(&lay, W, Winv, info_dev, stream)) return e;
  if (int e = gpk_finalize(&lay, W, info_dev, out, nullptr, nullptr, stream)) return e;
  GPK_HIP(launch_unpack_lower(GPK_F32, W, lay.ld, n, A, lda, s), "potrf_lower unpack");
  if (logdet_dev) GPK_HIP(hipMemcpyAsync(logdet_dev, out + 2, sizeof(double), hipMemcpyDeviceToDevice, s), "logdet");
  return 0;
}

int gpk_potrf_lower(int dtype, void* A, int64_t n, int64_t lda, void* work, size_t work_bytes, int32_t* info_dev,
                    double* logdet_dev, void* stream) {
  if (dtype != GPK_F64 && dtype != GPK_F32) return fail_arg(1, "dtype");
  if (!A) return fail_arg(2, "A");
  if (n <= 0) return fail_arg(3, "n");
  if (lda < n) return fail_arg(4, "lda");
  if (!info_dev) return fail_arg(7, "info_dev");
  if (dtype == GPK_F32)
    return potrf_lower_f32(static_cast<float*>(A), n, lda, work, work_bytes, info_dev, logdet_dev, stream);
  gpk_layout lay;
  if (int e = gpk_plan(GPK_F64, 1, n, 0, 1, &lay)) return e;
  if (!work || work_bytes < gpk_workspace_bytes(GPK_WS_POTRF, GPK_F64, n, 0, 1)) return fail_arg(6, "work_bytes");
  char* w = reinterpret_cast<char*>(work);
  double* W = reinterpret_cast<double*>(w);
  void* Winv = w + align256(lay.w_bytes);
  double* out = reinterpret_cast<double*>(w + align256(lay.w_bytes) + align256(lay.inv_bytes));
  double* zeros = reinterpret_cast<double*>(w + align256(lay.w_bytes) + align256(lay.inv_bytes) +
                                            align256(8 * sizeof(double)));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  GPK_HIP(hipMemsetAsync(out, 0, 8 * sizeof(double), s), "potrf_lower scratch");
  GPK_HIP(hipMemsetAsync(zeros, 0, (size_t)n * sizeof(double), s), "potrf_lower scratch");
  GPK_HIP(hipMemsetAsync(info_dev, 0, sizeof(int32_t), s), "memset info");
  // noise 0 (out[4] is zero), y = 0: the augmented factorisation of A alone
  if (int e = gpk_assemble_dense(&lay, reinterpret_cast<const double*>(A), lda, 0, out + 4, 0, nullptr, 0, 0, zeros, 0,
                                 W, stream))
    return e;
  if (int e = gpk_potrf_aug(&lay, W, Winv, info_dev, stream)) return e;
  if (int e = gpk_finalize(&lay, W, info_dev, out, nullptr, nullptr, stream)) return e;
  GPK_HIP(launch_copy_lower(W, lay.ld, reinterpret_cast<double*>(A), lda, n, s), "potrf_lower copy");
  if (logdet_dev) GPK_HIP(hipMemcpyAsync(logdet_dev, out + 2, sizeof(double), hipMemcpyDeviceToDevice, s), "logdet");
  return 0;
}

size_t gpk_grad_workspace_bytes(const gpk_kdesc* kd, const gpk_layout* lay) {
  if (!kd || !lay || lay->n <= 0 || lay->batch <= 0) return 0;
  const int64_t nt = (lay->n + ATILE - 1) / ATILE;
  return (size_t)lay->batch * (size_t)(nt * (nt + 1) / 2) * (size_t)(kd->n_hyp + 1) * sizeof(double);
}

int gpk_nlml_grad(const gpk_kdesc* kd, const gpk_layout* lay, const double* hyp_dev, int64_t hyp_stride,
                  const double* noise_dev, int64_t noise_stride, const double* X, int64_t x_bstride,
                  const double* y, int64_t y_bstride, void* W, void* Winv, int32_t* info_dev,
                  double* out_dev, double* grad_dev, void* work, size_t work_bytes, void* stream) {
  if (int e = check_layout(lay)) return e;
  if (lay->m != lay->n) return fail_arg(2, "gpk_nlml_grad needs a layout planned with m = n");
  if (!valid_kdesc(kd, lay->d)) return fail_arg(1, "kernel descriptor");
  if (!info_dev) return fail_arg(13, "info_dev");
  if (!out_dev) return fail_arg(14, "out_dev");
  if (grad_dev && (!work || work_bytes < gpk_grad_workspace_bytes(kd, lay)))
    return fail_arg(16, "work (see gpk_grad_workspace_bytes)");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  GPK_HIP(hipMemsetAsync(info_dev, 0, sizeof(int32_t) * lay->batch, s), "memset info");
  int e = gpk_assemble_inverse(kd, lay, hyp_dev, hyp_stride, noise_dev, noise_stride, X, x_bstride, y,
                               y_bstride, W, stream);
  if (e) return e;
  e = gpk_potrf_aug_ex(lay, W, Winv, info_dev, GPK_AUG_EXTRA_IDENTITY, stream);
  if (e) return e;
  e = gpk_finalize(lay, W, info_dev, out_dev, nullptr, nullptr, stream);
  if (e) return e;
  if (!grad_dev) return 0;
  GradArgs g;
  memset(&g, 0, sizeof(g));
  g.W = W;
  g.ld = lay->ld;
  g.w_bs = lay->w_batch_stride;
  g.n = lay->n;
  g.n_pad = lay->n_pad;
  g.y_row = lay->y_row;
  g.hyp = hyp_dev;
  g.hyp_stride = hyp_stride;
  g.X = X;
  g.x_bs = x_bstride;
  g.d = (int32_t)lay->d;
  g.dp = (lay->d % 2 == 0) ? (int32_t)lay->d + 1 : (int32_t)lay->d;
  g.ntile = (lay->n + ATILE - 1) / ATILE;
  g.part = static_cast<double*>(work);
  g.grad = grad_dev;
  g.info = info_dev;
  adjoint_masks(*kd, g.adj_mask);
  GPK_HIP(timed(6, 0.0, 0.0, s, [&] { return launch_grad(*kd, g, lay->dtype, lay->batch, s); }), "grad");
  return 0;
}

int gpk_kernel_matrix(const gpk_kdesc* kd, const double* hyp_dev, int dtype, int uplo,
                      const double* X, int64_t n, const double* Y, int64_t m, int32_t d,
                      double diag_add, void* K, int64_t ldk, void* stream) {
  if (!valid_kdesc(kd, d)) return fail_arg(1, "kernel descriptor");
  if (!hyp_dev && kd->n_hyp > 0) return fail_arg(2, "hyp_dev");
  if (dtype != GPK_F64 && dtype != GPK_F32) return fail_arg(3, "dtype");
  if (uplo != 0 && uplo != 1) return fail_arg(4, "uplo");
  if (!X) return fail_arg(5, "X");
  if (n <= 0) return fail_arg(6, "n");
  if (!Y) return fail_arg(7, "Y");
  if (m <= 0) return fail_arg(8, "m");
  if (d <= 0 || d > GPK_MAX_DIM) return fail_arg(9, "d");
  if (!K) return fail_arg(11, "K");
  if (ldk < m) return fail_arg(12, "ldk");
  AsmArgs a;
  memset(&a, 0, sizeof(a));
  a.hyp = hyp_dev;
  a.noise = nullptr;
  a.X = X;
  a.Xs = Y;
  a.W = K;
  a.ld = ldk;
  a.n = n;
  a.m = m;
  a.d = d;
  a.dp = (d % 2 == 0) ? d + 1 : d;
  a.plain = 1;
  a.uplo = uplo;
  a.diag_add = diag_add;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const double bytes = (double)elem_size(dtype) * (double)n * (double)m;
  GPK_HIP(timed(0, 0.0, bytes, s, [&] { return launch_assemble(*kd, a, dtype, 1, s); }),
          "kernel_matrix");
  return 0;
}

int gpk_trsv(const gpk_layout* lay, int trans, const void* W, const void* Winv, double* x,
             void* stream) {
  if (int e = check_layout(lay)) return e;
  if (trans != 0 && trans != 1) return fail_arg(2, "trans");
  if (!W) return fail_arg(3, "W");
  if (!Winv) return fail_arg(4, "Winv");
  if (!x) return fail_arg(5, "x");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t nblk = lay->n_pad / NB;
  TrsvArgs t;
  t.W = W;
  t.ld = lay->ld;
  t.w_bs = lay->w_batch_stride;
  t.Winv = Winv;
  t.inv_bs = lay->inv_batch_stride;
  t.x = x;
  t.x_bs = lay->n_pad;
  t.n_pad = lay->n_pad;
  t.trans = trans;
  t.n_valid = lay->n_pad;
  for (int64_t i = 0; i < nblk; ++i) {
    t.kblk = (trans == 0) ? i : nblk - 1 - i;
    GPK_HIP(timed(5, 0.0, 0.0, s, [&] { return launch_trsv_diag(t, lay->dtype, lay->batch, s); }),
            "trsv_diag");
    GPK_HIP(timed(5, 0.0, 0.0, s, [&] { return launch_trsv_update(t, lay->dtype, lay->batch, s); }),
            "trsv_update");
  }
  return 0;
}

int gpk_trsv_lower(int dtype, int trans, const double* L, int64_t n, int64_t ldl, double* x, void* work,
                   size_t work_bytes, void* stream) {
  if (dtype != GPK_F64) return fail_arg(1, "dtype (gpk_trsv_lower solves fp64)");
  if (trans != 0 && trans != 1) return fail_arg(2, "trans");
  if (!L) return fail_arg(3, "L");
  if (n <= 0) return fail_arg(4, "n");
  if (ldl < n) return fail_arg(5, "ldl");
  if (!x) return fail_arg(6, "x");
  if (!work || work_bytes < gpk_workspace_bytes(GPK_WS_TRSV, GPK_F64, n, 0, 1))
    return fail_arg(8, "work (gpk_workspace_bytes(GPK_WS_TRSV))");
  const int64_t n_pad = (n + NB - 1) / NB * NB, nblk = n_pad / NB;
  char* w = static_cast<char*>(work);
  double* Winv = reinterpret_cast<double*>(w);
  double* xp = reinterpret_cast<double*>(w + align256((size_t)n_pad * NB * sizeof(double)));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  GPK_HIP(launch_trtri_blocks(L, ldl, n, Winv, s), "trsv_lower diagonal blocks");
  GPK_HIP(hipMemsetAsync(xp, 0, (size_t)n_pad * sizeof(double), s), "trsv_lower x");
  GPK_HIP(hipMemcpyAsync(xp, x, (size_t)n * sizeof(double), hipMemcpyDeviceToDevice, s), "trsv_lower x");
  TrsvArgs t;
  t.W = L;
  t.ld = ldl;
  t.w_bs = 0;
  t.Winv = Winv;
  t.inv_bs = 0;
  t.x = xp;
  t.x_bs = n_pad;
  t.n_pad = n_pad;
  t.trans = trans;
  t.n_valid = n;
  for (int64_t i = 0; i < nblk; ++i) {
    t.kblk = (trans == 0) ? i : nblk - 1 - i;
    GPK_HIP(timed(5, 0.0, 0.0, s, [&] { return launch_trsv_diag(t, GPK_F64, 1, s); }), "trsv_lower diag");
    GPK_HIP(timed(5, 0.0, 0.0, s, [&] { return launch_trsv_update(t, GPK_F64, 1, s); }), "trsv_lower update");
  }
  GPK_HIP(hipMemcpyAsync(x, xp, (size_t)n * sizeof(double), hipMemcpyDeviceToDevice, s), "trsv_lower x");
  return 0;
}

int gpk_posterior(const gpk_kdesc* kd, const double* hyp_dev, int dtype, const double* L, int64_t ldl,
                  const double* alpha, const double* X, int64_t n, const double* Xs, int64_t m, int32_t d,
                  int32_t var_mode, double* mu, double* var, int64_t ldv, void* work, size_t work_bytes,
                  void* stream) {
  if (!valid_kdesc(kd, d)) return fail_arg(1, "kernel descriptor");
  if (dtype != GPK_F64) return fail_arg(3, "dtype (gpk_posterior is fp64)");
  if (!L) return fail_arg(4, "L");
  if (ldl < n) return fail_arg(5, "ldl");
  if (!alpha && mu) return fail_arg(6, "alpha");
  if (!X) return fail_arg(7, "X");
  if (n <= 0) return fail_arg(8, "n");
  if (!Xs) return fail_arg(9, "Xs");
  if (m <= 0) return fail_arg(10, "m");
  if (var_mode != 0 && var_mode != 1) return fail_arg(12, "var_mode");
  if (var && var_mode == 1 && ldv < m) return fail_arg(15, "ldv");
  if (!work || work_bytes < gpk_workspace_bytes(GPK_WS_POSTERIOR, GPK_F64, n, m, 1))
    return fail_arg(16, "work (gpk_workspace_bytes(GPK_WS_POSTERIOR))");
  const int64_t n_pad = (n + NB - 1) / NB * NB, nblk = n_pad / NB;
  char* w = static_cast<char*>(work);
  double* Winv = reinterpret_cast<double*>(w);
  w += align256((size_t)n_pad * NB * sizeof(double));
  double* Ks = reinterpret_cast<double*>(w);
  w += align256((size_t)n_pad * (size_t)m * sizeof(double));
  double* V = reinterpret_cast<double*>(w);
  w += align256((size_t)n_pad * (size_t)m * sizeof(double));
  double* kdiag = reinterpret_cast<double*>(w);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // K_s = k(X, Xs) [n, m], zero padding rows
  if (n_pad > n)
    GPK_HIP(hipMemsetAsync(Ks + n * m, 0, (size_t)(n_pad - n) * (size_t)m * sizeof(double), s), "posterior pad");
  if (int e = gpk_kernel_matrix(kd, hyp_dev, GPK_F64, 0, X, n, Xs, m, d, 0.0, Ks, m, stream)) return e;
  if (mu) {  // mu = K_s^T alpha (S/Auxiliary.py:57-66)
    DgemmArgs g{1, 0, m, 1, n, Ks, m, 0, alpha, 1, 0, mu, 1, 0, 1.0, 0.0};
    GPK_HIP(launch_dgemm(g, 1, s), "posterior mu");
  }
  if (!var) return 0;
  // V = L^-1 K_s, blocked: V_k = L_kk^-1 K_s,k; K_s,below -= L_below,k V_k
  GPK_HIP(launch_trtri_blocks(L, ldl, n, Winv, s), "posterior diagonal blocks");
  for (int64_t kb = 0; kb < nblk; ++kb) {
    const int64_t j0 = kb * NB, nv = std::min<int64_t>(NB, n - j0);
    DgemmArgs g1{0, 0, NB, m, NB, Winv + kb * NB * NB, NB, 0, Ks + j0 * m, m, 0, V + j0 * m, m, 0, 1.0, 0.0};
    GPK_HIP(launch_dgemm(g1, 1, s), "posterior solve");
    if (j0 + NB < n) {
      DgemmArgs g2{0, 0, n - j0 - NB, m, nv, L + (j0 + NB) * ldl + j0, ldl, 0, V + j0 * m, m, 0,
                   Ks + (j0 + NB) * m, m, 0, -1.0, 1.0};
      GPK_HIP(launch_dgemm(g2, 1, s), "posterior update");
    }
  }
  if (var_mode == 1) {  // Sigma = K_ss - V^T V (S/Auxiliary.py:68-93)
    if (int e = gpk_kernel_matrix(kd, hyp_dev, GPK_F64, 0, Xs, m, Xs, m, d, 0.0, var, ldv, stream)) return e;
    DgemmArgs g{1, 0, m, m, n, V, m, 0, V, m, 0, var, ldv, 0, -1.0, 1.0};
    GPK_HIP(launch_dgemm(g, 1, s), "posterior covariance");
  } else {  // diag: k(x*, x*) is the same for every x* (every kernel of the descriptor is stationary)
    if (int e = gpk_kernel_matrix(kd, hyp_dev, GPK_F64, 0, Xs, 1, Xs, 1, d, 0.0, kdiag, 1, stream)) return e;
    GPK_HIP(launch_posterior_var(V, n, m, kdiag, var, s), "posterior variance");
  }
  return 0;
}

int gpk_gemv(const double* A, int64_t n, int64_t m, int64_t lda, const double* x, double* y, double alpha,
             double beta, void* stream) {
  if (!A) return fail_arg(1, "A");
  if (n < 0) return fail_arg(2, "n");
  if (m < 0) return fail_arg(3, "m");
  if (lda < m) return fail_arg(4, "lda");
  if (!x && m > 0) return fail_arg(5, "x");
  if (!y && n > 0) return fail_arg(6, "y");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  GPK_HIP(timed(5, 2.0 * (double)n * (double)m, 8.0 * (double)n * (double)m, s,
                [&] { return launch_gemv(A, n, m, lda, x, y, alpha, beta, s); }),
          "gemv");
  return 0;
}

// ------------------------------------------------------------------ approximation paths (§8f.4)
int gpk_assemble_dense(const gpk_layout* lay, const double* A, int64_t lda, int64_t a_bstride,
                       const double* noise_dev, int64_t noise_stride, const double* E, int64_t e_bstride,
                       int32_t eye, const double* y, int64_t y_bstride, void* W, void* stream) {
  if (int e = check_layout(lay)) return e;
  if (lay->dtype != GPK_F64) return fail_arg(1, "layout dtype (dense mode is fp64)");
  if (!A) return fail_arg(2, "A");
  if (lda < lay->n) return fail_arg(3, "lda");
  if (!noise_dev) return fail_arg(5, "noise_dev");
  if (eye && lay->m != lay->n) return fail_arg(9, "identity extra rows need a layout planned with m = n");
  if (lay->m > 0 && !E && !eye) return fail_arg(7, "E (extra rows) or eye");
  if (!y) return fail_arg(10, "y");
  if (!W) return fail_arg(12, "W");
  gpk_kdesc kd;
  memset(&kd, 0, sizeof(kd));
  kd.n_nodes = 1;
  kd.dim = 1;
  kd.nodes[0].op = GPK_OP_SE;
  AsmArgs a;
  memset(&a, 0, sizeof(a));
  a.noise = noise_dev;
  a.noise_stride = noise_stride;
  a.E = (lay->m > 0 && !eye) ? E : nullptr;
  a.e_bs = e_bstride;
  a.y = y;
  a.y_bs = y_bstride;
  a.W = W;
  a.ld = lay->ld;
  a.w_bs = lay->w_batch_stride;
  a.n = lay->n;
  a.m = lay->m;
  a.n_pad = lay->n_pad;
  a.y_row = lay->y_row;
  a.p = lay->p;
  a.d = 1;
  a.dp = 1;
  a.eye = eye ? 1 : 0;
  a.ntile = lay->p / ATILE;
  a.A = A;
  a.a_ld = lda;
  a.a_bs = a_bstride;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  GPK_HIP(launch_assemble(kd, a, lay->dtype, lay->batch, s), "assemble_dense");
  return 0;
}

int gpk_dgemm(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K, double alpha,
              const double* A, int64_t lda, int64_t a_bstride, const double* B, int64_t ldb, int64_t b_bstride,
              double beta, double* C, int64_t ldc, int64_t c_bstride, int32_t batch, void* stream) {
  if (M < 0) return fail_arg(3, "M");
  if (N < 0) return fail_arg(4, "N");
  if (K < 0) return fail_arg(5, "K");
  if (!A && M > 0 && K > 0) return fail_arg(7, "A");
  if (lda < (trans_a ? M : K)) return fail_arg(8, "lda");
  if (!B && N > 0 && K > 0) return fail_arg(10, "B");
  if (ldb < (trans_b ? K : N)) return fail_arg(11, "ldb");
  if (!C && M > 0 && N > 0) return fail_arg(14, "C");
  if (ldc < N) return fail_arg(15, "ldc");
  if (batch < 0) return fail_arg(17, "batch");
  DgemmArgs g{trans_a ? 1 : 0, trans_b ? 1 : 0, M, N, K, A, lda, a_bstride, B, ldb, b_bstride,
              C, ldc, c_bstride, alpha, beta};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  GPK_HIP(timed(5, 2.0 * (double)M * (double)N * (double)K * batch,
                8.0 * ((double)M * K + (double)K * N + 2.0 * (double)M * N) * batch, s,
                [&] { return launch_dgemm(g, batch, s); }),
          "dgemm");
  return 0;
}

size_t gpk_syevj_workspace_bytes(int64_t m, int32_t batch) {
  if (m <= 0 || batch <= 0) return 8;
  return (size_t)(4 * m * m * (int64_t)batch + 2) * sizeof(double);
}

int gpk_syevj(int64_t m, int32_t batch, const double* A, int64_t lda, int64_t a_bstride, double* V, double* lam,
              void* work, size_t work_bytes, int32_t max_sweeps, int32_t* sweeps_out, void* stream) {
  if (m < 0 || m > (1 << 20)) return fail_arg(1, "m");
  if (batch < 0) return fail_arg(2, "batch");
  if (m == 0 || batch == 0) {
    if (sweeps_out) *sweeps_out = 0;
    return 0;
  }
  if (!A) return fail_arg(3, "A");
  if (lda < m) return fail_arg(4, "lda");
  if (!V) return fail_arg(6, "V");
  if (!lam) return fail_arg(7, "lam");
  if (!work || work_bytes < gpk_syevj_workspace_bytes(m, batch)) return fail_arg(9, "work_bytes");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t blk = m * m * (int64_t)batch;
  double* buf = reinterpret_cast<double*>(work);
  double* Ab[2] = {buf, buf + blk};
  double* Vb[2] = {buf + 2 * blk, buf + 3 * blk};
  int32_t* flag = reinterpret_cast<int32_t*>(buf + 4 * blk);
  GPK_HIP(launch_jacobi_init(A, lda, a_bstride, (int)m, Ab[0], Vb[0], batch, s), "syevj init");
  // optional absolute threshold (gpk_tune("syevj_abs_tol_e3"), default 0 = the relative criterion
  // alone): pairs with |a_pq| below e3 * 1e-3 eps max|a_ii| are not rotated.  Measured on SE Gram
  // matrices (tools/diag_syevj.py): 1 eps saves 1 sweep of 31, 10 eps 7 sweeps with 4x the pinv error
  double* dmax = reinterpret_cast<double*>(flag) + 1;
  GPK_HIP(launch_diag_absmax(Ab[0], (int)m, batch, dmax, s), "syevj scale");
  double host_dmax = 0.0;
  GPK_HIP(hipMemcpyAsync(&host_dmax, dmax, sizeof(double), hipMemcpyDeviceToHost, s), "syevj scale read");
  GPK_HIP(hipStreamSynchronize(s), "syevj sync");
  const double tol_abs = (double)tune_now().syevj_abs_tol_e3 * 1e-3 * 2.220446049250313e-16 * host_dmax;
  const int mm = (int)(m + (m & 1));
  int cur = 0, sweeps = 0;
  for (; sweeps < (max_sweeps > 0 ? max_sweeps : 60); ++sweeps) {
    GPK_HIP(hipMemsetAsync(flag, 0, sizeof(int32_t), s), "syevj flag");
    for (int r = 0; r < mm - 1; ++r) {
      JacobiArgs ja{Ab[cur], Ab[cur ^ 1], Vb[cur], Vb[cur ^ 1], (int32_t)m, mm, flag, tol_abs};
      GPK_HIP(launch_jacobi_round(ja, r, batch, s), "syevj round");
      cur ^= 1;
    }
    int32_t host_flag = 0;
    GPK_HIP(hipMemcpyAsync(&host_flag, flag, sizeof(int32_t), hipMemcpyDeviceToHost, s), "syevj flag read");
    GPK_HIP(hipStreamSynchronize(s), "syevj sync");
    if (!host_flag) {
      ++sweeps;
      break;
    }
  }
  GPK_HIP(launch_jacobi_out(Ab[cur], Vb[cur], (int)m, V, lam, batch, s), "syevj out");
  if (sweeps_out) *sweeps_out = sweeps;
  return 0;
}

// ------------------------------------------------------------------- tridiagonal eigensolver (gpk_eig.hip)
namespace {
constexpr int kEigNb = 32;  // reflectors per compact-WY block of the back-transformation
// m^2 < 2^31: the eigensolver's kernels index a row-major m x m matrix with 32-bit products of two indices
#define GPK_SYEVD_MAX_M 46340

struct EigWs {  // carving of the gpk_syevd workspace
  double *W, *Qg, *U, *d, *e, *tau, *Y, *T1, *T2, *Gs, *S, *PV, *vg, *yg, *Sall;
  DcLevel L;
  size_t bytes;
};

EigWs eig_carve(int64_t m, void* base) {
  EigWs ws;
  memset(&ws, 0, sizeof(ws));
  char* p = static_cast<char*>(base);
  size_t off = 0;
  auto take = [&](size_t n) -> double* {
    double* r = reinterpret_cast<double*>(p ? p + off : nullptr);
    off += (n * sizeof(double) + 255) & ~(size_t)255;
    return r;
  };
  auto itake = [&](size_t n) -> int32_t* { return reinterpret_cast<int32_t*>(take((n + 1) / 2)); };
  const size_t mm = (size_t)m * (size_t)m, hp = (size_t)m / 2 + 1;
  ws.W = take(mm);
  ws.Qg = take(mm);
  ws.U = take(mm);
  ws.d = take(m);
  ws.e = take(m);
  ws.tau = take(m);
  ws.Y = take((size_t)m * kEigNb);
  ws.T1 = take((size_t)m * kEigNb);
  ws.T2 = take((size_t)m * kEigNb);
  ws.Gs = take((size_t)kEigNb * kEigNb);
  ws.S = take((size_t)kEigNb * kEigNb);
  ws.PV = take((size_t)3 * m * kEigNb);
  ws.Sall = take((size_t)(m / kEigNb + 1) * kEigNb * kEigNb);
  ws.vg = take(m);
  ws.yg = take(m);
  DcLevel& L = ws.L;
  L.dK = take(m);
  L.zK = take(m);
  L.rc = take(m);
  L.rs = take(m);
  L.root_t = take(m);
  L.zhat = take(m);
  L.rho = take(hp);
  L.idx = itake(m);
  L.ord = itake(m);
  L.rp = itake(m);
  L.rn = itake(m);
  L.root_o = itake(m);
  L.kcnt = itake(hp);
  L.rcnt = itake(hp);
  L.flip = itake(hp);
  L.gscr = take((size_t)5 * m);
  ws.bytes = off;
  return ws;
}

// C <- alpha op(A) op(B) + beta C (row-major, contiguous leading dimensions)
hipError_t eig_gemm(int ta, int tb, int64_t M, int64_t N, int64_t K, double alpha, const double* A, int64_t lda,
                    const double* B, int64_t ldb, double beta, double* C, int64_t ldc, hipStream_t s) {
  DgemmArgs g{ta, tb, M, N, K, A, lda, 0, B, ldb, 0, C, ldc, 0, alpha, beta};
  return launch_dgemm(g, 1, s);
}
}  // namespace

size_t gpk_syevd_workspace_bytes(int64_t m) {
  if (m <= 0) return 8;
  return eig_carve(m, nullptr).bytes;
}

int gpk_syevd(int64_t m, int32_t batch, const double* A, int64_t lda, int64_t a_bstride, double* V, double* lam,
              void* work, size_t work_bytes, void* stream) {
  if (m < 0 || m > GPK_SYEVD_MAX_M) return fail_arg(1, "m (gpk_syevd: m <= 46340)");
  if (batch < 0) return fail_arg(2, "batch");
  if (m == 0 || batch == 0) return 0;
  if (!A) return fail_arg(3, "A");
  if (lda < m) return fail_arg(4, "lda");
  if (!V) return fail_arg(6, "V");
  if (!lam) return fail_arg(7, "lam");
  if (!work || work_bytes < gpk_syevd_workspace_bytes(m)) return fail_arg(8, "work (gpk_syevd_workspace_bytes)");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  EigWs ws = eig_carve(m, work);
  const Tune tn = tune_now();
  const int mi = (int)m;
  const int64_t mm = m * m;
  for (int32_t b = 0; b < batch; ++b) {
    double* Vb = V + (int64_t)b * mm;
    double* lb = lam + (int64_t)b * m;
    GPK_HIP(launch_sym_copy(A + (int64_t)b * a_bstride, lda, mi, ws.W, s), "syevd copy");
    if (m == 1) {
      GPK_HIP(hipMemcpyAsync(lb, ws.W, sizeof(double), hipMemcpyDeviceToDevice, s), "syevd m=1");
      GPK_HIP(launch_eig_identity(Vb, 1, s), "syevd m=1");
      continue;
    }
    GPK_HIP(launch_eig_tridiag(ws.W, mi, ws.d, ws.e, ws.tau, ws.PV, ws.vg, ws.yg, (int)tn.trd_split_m, s),
            "syevd tridiag");
    // eigenvectors of T into V, eigenvalues into lam
    DcLevel L = ws.L;
    L.lam = lb;
    GPK_HIP(launch_eig_dc(ws.d, ws.e, mi, L, Vb, ws.Qg, ws.U, s), "syevd divide and conquer");
    // V <- Q V, Q = H_0 ... H_{m-2}: blocks of reflectors from the last to the first, V <- V - Y (S (Y^T V))
    if (eig_bt_fused(mi)) {
      GPK_HIP(launch_eig_backtransform(ws.W, ws.tau, mi, ws.Sall, Vb, s), "syevd back-transformation");
      continue;
    }
    const int nref = mi - 1;
    for (int k0 = ((nref - 1) / kEigNb) * kEigNb; k0 >= 0; k0 -= kEigNb) {
      const int nb = std::min(kEigNb, nref - k0);
      GPK_HIP(launch_eig_build_y(ws.W, mi, k0, nb, ws.Y, s), "syevd Y");
      GPK_HIP(eig_gemm(1, 0, nb, nb, m, 1.0, ws.Y, nb, ws.Y, nb, 0.0, ws.Gs, nb, s), "syevd Y^T Y");
      GPK_HIP(launch_eig_larft(ws.Gs, ws.tau, k0, nb, ws.S, s), "syevd larft");
      GPK_HIP(eig_gemm(1, 0, nb, m, m, 1.0, ws.Y, nb, Vb, m, 0.0, ws.T1, m, s), "syevd Y^T V");
      GPK_HIP(eig_gemm(0, 0, nb, m, nb, 1.0, ws.S, nb, ws.T1, m, 0.0, ws.T2, m, s), "syevd S (Y^T V)");
      GPK_HIP(eig_gemm(0, 0, m, m, nb, -1.0, ws.Y, nb, ws.T2, m, 1.0, Vb, m, s), "syevd V update");
    }
  }
  return 0;
}

int gpk_pinv_factor(int64_t m, int32_t batch, const double* V, const double* lam, double rcond, int32_t mode,
                    double* mu, double* U, int32_t* rank_dev, void* stream) {
  if (m <= 0) return fail_arg(1, "m");
  if (batch <= 0) return fail_arg(2, "batch");
  if (!V) return fail_arg(3, "V");
  if (!lam) return fail_arg(4, "lam");
  if (mode < 0 || mode > 2) return fail_arg(6, "mode (0, 1 or 2)");
  if (!mu) return fail_arg(7, "mu");
  if (!U) return fail_arg(8, "U");
  if (!rank_dev) return fail_arg(9, "rank_dev");
  if (rcond < 0.0) rcond = 10.0 * (double)m * 2.220446049250313e-16;  // tf.linalg.pinv's default
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  GPK_HIP(launch_pinv_factor(V, lam, (int)m, rcond, mode, mu, U, rank_dev, batch, s), "pinv_factor");
  return 0;
}

int gpk_pinv_backward_scale(int64_t m, int32_t batch, const double* lam, const double* mu, double* T, void* stream) {
  if (m <= 0) return fail_arg(1, "m");
  if (batch <= 0) return fail_arg(2, "batch");
  if (!lam) return fail_arg(3, "lam");
  if (!mu) return fail_arg(4, "mu");
  if (!T) return fail_arg(5, "T");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  GPK_HIP(launch_pinv_bwd_scale(lam, mu, (int)m, T, batch, s), "pinv_backward_scale");
  return 0;
}

int gpk_ski_weights(const double* X, int64_t n, const double* Z, int64_t m, int32_t d, double* Wm, double* work,
                    void* stream) {
  if (!X) return fail_arg(1, "X");
  if (n <= 0) return fail_arg(2, "n");
  if (!Z) return fail_arg(3, "Z");
  if (m <= 0) return fail_arg(4, "m");
  if (d <= 0 || d > GPK_MAX_DIM) return fail_arg(5, "d");
  if (!Wm) return fail_arg(6, "Wm");
  if (!work) return fail_arg(7, "work");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  GPK_HIP(launch_ski_weights(X, n, Z, m, d, Wm, work, s), "ski_weights");
  return 0;
}

int gpk_distance_matrix(int mode, const double* A, int64_t n, int64_t a_bstride, const double* B, int64_t m,
                        int64_t b_bstride, int32_t d, int32_t batch, double* out, int64_t ldo, int64_t o_bstride,
                        void* stream) {
  if (mode < 0 || mode > 2) return fail_arg(1, "mode (0 expanded-norm euclidean, 1 manhattan, 2 euclidean)");
  if (!A && n > 0) return fail_arg(2, "A");
  if (n < 0) return fail_arg(3, "n");
  if (!B && m > 0) return fail_arg(5, "B");
  if (m < 0) return fail_arg(6, "m");
  if (d <= 0) return fail_arg(8, "d");
  if (batch < 0) return fail_arg(9, "batch");
  if (!out && n > 0 && m > 0) return fail_arg(10, "out");
  if (ldo < m) return fail_arg(11, "ldo");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  GPK_HIP(launch_distance(mode, A, n, a_bstride, B, m, b_bstride, d, batch, out, ldo, o_bstride, s), "distance");
  return 0;
}

size_t gpk_kernel_vjp_workspace_bytes(const gpk_kdesc* kd, int64_t n, int64_t m, int32_t d, int32_t want_z) {
  if (!kd || n <= 0 || m <= 0 || d <= 0) return 0;
  return vjp_workspace_elems(*kd, n, m, d, want_z != 0) * sizeof(double);
}

int gpk_kernel_vjp(const gpk_kdesc* kd, const double* hyp_dev, const double* X, int64_t n, const double* Z, int64_t m,
                   int32_t d, const double* G, int64_t ldg, const double* gu, const double* gv, double* grad_hyp,
                   double* grad_z, void* work, size_t work_bytes, void* stream) {
  if (!valid_kdesc(kd, d)) return fail_arg(1, "kernel descriptor");
  if (!hyp_dev && kd->n_hyp > 0) return fail_arg(2, "hyp_dev");
  if (!X) return fail_arg(3, "X");
  if (n <= 0) return fail_arg(4, "n");
  if (!Z) return fail_arg(5, "Z");
  if (m <= 0) return fail_arg(6, "m");
  if (d <= 0 || d > GPK_MAX_DIM) return fail_arg(7, "d");
  if (!G && !(gu && gv)) return fail_arg(8, "G (or the rank-1 weights gu, gv)");
  if (G && ldg < m) return fail_arg(9, "ldg");
  if (!grad_hyp && kd->n_hyp > 0) return fail_arg(12, "grad_hyp");
  if (!work || work_bytes < gpk_kernel_vjp_workspace_bytes(kd, n, m, d, grad_z != nullptr ? 1 : 0))
    return fail_arg(14, "work (see gpk_kernel_vjp_workspace_bytes)");
  VjpArgs g;
  memset(&g, 0, sizeof(g));
  g.hyp = hyp_dev;
  g.G = G;
  g.ldg = ldg;
  g.gu = gu;
  g.gv = gv;
  g.part_h = static_cast<double*>(work);
  adjoint_masks(*kd, g.adj_mask);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  GPK_HIP(timed(6, 0.0, 8.0 * (double)n * (double)m, s,
                [&] { return launch_vjp(*kd, g, X, n, Z, m, d, grad_hyp, grad_z, s); }),
          "kernel_vjp");
  return 0;
}

int gpk_add_diagonal(double* A, int64_t n, int64_t lda, int64_t a_bstride, int32_t batch, double value,
                     void* stream) {
  if (!A && n > 0) return fail_arg(1, "A");
  if (n < 0) return fail_arg(2, "n");
  if (lda < n) return fail_arg(3, "lda");
  if (batch < 0) return fail_arg(5, "batch");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  GPK_HIP(launch_add_diag(A, n, lda, a_bstride, value, batch, s), "add_diagonal");
  return 0;
}

int gpk_timing_enable(int on) {
  std::lock_guard<std::mutex> lk(g_timing.mu);
  g_timing.on = on != 0;
  return 0;
}

// profiling: the per-task stamps of the last chain launch with GPK_CHAIN_TIMES=1 (synchronises the device)
int gpk_chain_times(uint64_t* out, int64_t ntasks) {
  if (!g_chain_times || !out || ntasks > g_chain_times_n) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  return hipMemcpy(out, g_chain_times, (size_t)ntasks * 6 * sizeof(uint64_t), hipMemcpyDeviceToHost) == hipSuccess ? 0 : -3;
}

// debugging: the progress words of the last traced chain launch (GPK_CHAIN_TRACE=1), host memory only
int gpk_chain_trace(int32_t* out, int64_t n) {
  if (!g_chain_trace || !out) return -1;
  memcpy(out, g_chain_trace, (size_t)std::min<int64_t>(n, 4096 * 32) * sizeof(int32_t));
  return 0;
}

namespace {
// gpk_chain_plan(_ex): ap = the argument positions of (tasks_out, cap, ntasks) in the entry point's own signature,
// so that -i names the caller's i-th argument (gpk.h's convention) for both entry points
int chain_plan_impl(int64_t n_pad, int64_t y_row, int32_t grid, int32_t flags, int32_t* tasks_out, int64_t cap,
                    int64_t* ntasks, int ap_cap, int ap_ntasks) {
  if (n_pad <= 0 || n_pad % NB != 0) return fail_arg(1, "n_pad (a positive multiple of 128)");
  if (y_row < n_pad) return fail_arg(2, "y_row (>= n_pad)");
  if (grid <= 0) return fail_arg(3, "grid");
  if (flags & ~(GPK_AUG_EXTRA_IDENTITY | GPK_CHAIN_PLAN_F32)) return fail_arg(4, "flags");
  const bool eye = (flags & GPK_AUG_EXTRA_IDENTITY) != 0;
  const bool f32 = (flags & GPK_CHAIN_PLAN_F32) != 0;
  if (eye && f32) return fail_arg(4, "flags (f32 plans have no identity rows)");
  if (eye && (y_row - n_pad < 1 || y_row - n_pad > n_pad))
    return fail_arg(2, "y_row (identity extra rows: n_pad + n with 0 < n <= n_pad)");
  if (!ntasks) return fail_arg(ap_ntasks, "ntasks");
  const std::vector<int32_t> ord = chain_order(n_pad, y_row, grid, 1, chain_knobs(tune_now(), n_pad, eye, f32, grid), eye);
  if (ord.empty()) {
    return fail_hip(hipErrorUnknown, "chain_order: a task exceeds the device's dependency bound");
  }
  *ntasks = (int64_t)(ord.size() / 4);
  if (tasks_out) {
    if (cap < *ntasks) return fail_arg(ap_cap, "cap (fewer than ntasks)");
    memcpy(tasks_out, ord.data(), ord.size() * sizeof(int32_t));
  }
  return 0;
}
}  // namespace

int gpk_chain_plan(int64_t n_pad, int64_t y_row, int32_t grid, int32_t* tasks_out, int64_t cap, int64_t* ntasks) {
  return chain_plan_impl(n_pad, y_row, grid, 0, tasks_out, cap, ntasks, 5, 6);
}

int gpk_chain_plan_ex(int64_t n_pad, int64_t y_row, int32_t grid, int32_t flags, int32_t* tasks_out, int64_t cap,
                      int64_t* ntasks) {
  return chain_plan_impl(n_pad, y_row, grid, flags, tasks_out, cap, ntasks, 6, 7);
}

int gpk_tune(const char* key, int64_t value, int64_t* old) {
  if (!key) return fail_arg(1, "key");
  if (!strcmp(key, "chain_force_timeout")) {  // (testing: the next `value` persistent launches time out)
    const int64_t prev = g_chain_force_timeout.exchange(value);
    if (old) *old = prev;
    return 0;
  }
  int64_t Tune::*f = knob_field(key);
  if (!f) return fail_arg(1, "key (unknown tuning knob)");
  Tune& t = tune();
  if (old) *old = t.*f;
  t.*f = value;
  return 0;
}

int gpk_tune_thread(const char* key, int64_t value, int32_t set, int64_t* old_value, int32_t* old_set) {
  if (!key) return fail_arg(1, "key");
  int64_t Tune::*f = knob_field(key);
  if (!f) return fail_arg(1, "key (unknown tuning knob)");
  auto it = std::find_if(t_tune_over.begin(), t_tune_over.end(),
                         [&](const std::pair<int64_t Tune::*, int64_t>& o) { return o.first == f; });
  if (old_set) *old_set = it != t_tune_over.end() ? 1 : 0;
  if (old_value) *old_value = it != t_tune_over.end() ? it->second : tune().*f;
  if (it != t_tune_over.end()) t_tune_over.erase(it);
  if (set) t_tune_over.emplace_back(f, value);
  return 0;
}

int gpk_chain_stats(int64_t* out, int32_t n) {
  if (!out || n < 1) return fail_arg(1, "out");
  const int64_t v[4] = {g_chain_launches.load(), g_chain_declined.load(), t_chain_last ? 1 : 0,
                        g_chain_force_timeout.load()};
  for (int i = 0; i < n && i < 4; ++i) out[i] = v[i];
  if (n >= 5) {  // (a device read: waits for the work enqueued so far on the null stream's device)
    int64_t t = 0;
    GPK_HIP(chain_timeouts_read(&t), "chain timeouts");
    out[4] = t;
  }
  return 0;
}

int gpk_timing_reset(void) {
  std::lock_guard<std::mutex> lk(g_timing.mu);
  for (auto& t : g_timing.pending) {
    hipEventSynchronize(t.end);
    g_timing.pool.push_back(t.beg);
    g_timing.pool.push_back(t.end);
  }
  g_timing.pending.clear();
  for (int c = 0; c < GPK_NUM_CLASSES; ++c) {
    g_timing.ms[c] = 0;
    g_timing.launches[c] = 0;
    g_timing.flops[c] = 0;
    g_timing.bytes[c] = 0;
  }
  return 0;
}

int gpk_timing_read(double* ms_by_class, int64_t* launches_by_class, double* flops_by_class,
                    double* bytes_by_class) {
  std::lock_guard<std::mutex> lk(g_timing.mu);
  for (auto& t : g_timing.pending) {
    hipError_t e = hipEventSynchronize(t.end);
    if (e != hipSuccess) return fail_hip(e, "timing sync");
    float ms = 0.f;
    hipEventElapsedTime(&ms, t.beg, t.end);
    g_timing.ms[t.cls] += ms;
    g_timing.launches[t.cls] += 1;
    g_timing.flops[t.cls] += t.flops;
    g_timing.bytes[t.cls] += t.bytes;
    g_timing.pool.push_back(t.beg);
    g_timing.pool.push_back(t.end);
  }
  g_timing.pending.clear();
  for (int c = 0; c < GPK_NUM_CLASSES; ++c) {
    if (ms_by_class) ms_by_class[c] = g_timing.ms[c];
    if (launches_by_class) launches_by_class[c] = g_timing.launches[c];
    if (flops_by_class) flops_by_class[c] = g_timing.flops[c];
    if (bytes_by_class) bytes_by_class[c] = g_timing.bytes[c];
  }
  return 0;
}

}  // extern "C"
