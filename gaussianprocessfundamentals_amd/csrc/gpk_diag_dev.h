// Device code of the diagonal-block factorisation (128 x 128 block in LDS: potf2 of 16 x 16 pivot tiles,
// f64 MFMA tile operations, the block inverse), shared by the launch-per-block kernels of gpk_diag.hip
// and the persistent factorisation of gpk_potrf.hip (chain_kernel), which runs the same body as one of
// its tasks.  Included by both translation units (anonymous namespace: one copy each).
#pragma once
#include <type_traits>

#include "gpk_internal.h"

namespace gpk {
namespace {

constexpr int DB = 16;            // tile edge
constexpr int NTL = NB / DB;      // tiles per block edge (8)
#ifndef GPK_DIAG_SWIZZLE
#define GPK_DIAG_SWIZZLE 0
#endif
// LDS row stride (doubles).  Default: 130, so the 16 rows of one column that the MFMA operand reads take
// (lanes along rows) sit on distinct banks; the accumulator-layout accesses (lanes along 16 columns x 2
// consecutive rows) are then 2-way conflicted.  GPK_DIAG_SWIZZLE=1: rows of 128 with the columns XOR-swizzled
// per row, c ^ (16 (r & 1) + 2 ((r >> 1) & 7)), conflict-free for both patterns (SQ_LDS_BANK_CONFLICT per LDS
// instruction 2.12 -> 0.75) but slower: the fused diagonal launch at N = 4096 took 44.8 instead of 40.2 us
// (the swizzled addresses split the block load's 16-B LDS stores and add VALU work on the potf2 path).
constexpr int LDA = GPK_DIAG_SWIZZLE ? NB : NB + 2;
constexpr int DT = 512;           // threads (8 waves)
constexpr int LDS_A = NB * LDA;

__device__ __forceinline__ int aidx(int r, int c) {
  return GPK_DIAG_SWIZZLE ? r * LDA + (c ^ (((r & 1) << 4) | (((r >> 1) & 7) << 1))) : r * LDA + c;
}
#ifndef GPK_DINV_LD
#define GPK_DINV_LD 18  // row stride of the inverted pivot tiles: lane (r, k) reads of a tile row hit distinct
#endif              // banks (stride 16: the 16 rows sat on two banks, an 8-way conflict per read)
constexpr int DBS = GPK_DINV_LD;   // Dinv tile row stride (doubles)
constexpr int DTS = DB * DBS;      // Dinv tile stride
constexpr int LDS_DINV = NTL * DTS;
constexpr int LDS_COL = 2 * DB;  // potf2 column broadcast, double-buffered
constexpr size_t DIAG_LDS_BYTES = sizeof(double) * (LDS_A + LDS_DINV + LDS_COL) + 16;

// 1/sqrt(x) from the hardware estimate plus two Newton steps (~1 ulp); NaN for x < 0.
#ifndef GPK_RSQ_NEWTON
#define GPK_RSQ_NEWTON 2  // Newton steps after the hardware estimate (A/B builds only)
#endif
__device__ __forceinline__ double rsqrt_refined(double x) {
  double r = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
#pragma unroll
  for (int i = 0; i < GPK_RSQ_NEWTON; ++i) r = r * fma(-h * r, r, 1.5);
  return r;
}

__device__ __forceinline__ d4 mfma64(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

#ifndef GPK_DIAG_PROF
#define GPK_DIAG_PROF 0
#endif
#ifndef GPK_POTF2_MODE
#define GPK_POTF2_MODE 2  // pivot column broadcast: 2 DPP row_newbcast, 1 v_readlane, 0 LDS (rounds 1-4; A/B builds)
#endif
#define GPK_POTF2_READLANE (GPK_POTF2_MODE == 1)
#ifndef GPK_PIPE_NEWTON
#define GPK_PIPE_NEWTON 1  // Newton steps after v_rsq_f64 in the pipelined potf2 (2: rounds 1-4)
#endif
#ifndef GPK_PIPE_NOINV
#define GPK_PIPE_NOINV 0  // (timing probes only: the inverse half's FMAs left out -- wrong L^-1)
#endif
#ifndef GPK_PIPE_NOBAD
#define GPK_PIPE_NOBAD 0  // (timing probes only: no non-positive pivot bookkeeping)
#endif
#ifndef GPK_POTF2_PIPE
#define GPK_POTF2_PIPE 1  // mode 2: the software-pipelined issue order (potf2_pipelined)
#endif
// lane l's value of v, wave-uniform (two v_readlane_b32 into SGPRs; l a compile-time lane)
__device__ __forceinline__ double bcast_lane(double v, int l) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// Lane C of each 16-lane row of the wave, as a 64-bit DPP move (row_newbcast), and w += (lane C's u) * ng as
// one DPP-sourced f64 FMA.  (s_nop 1: a VALU write of a VGPR needs two wait states before a DPP read of it --
// the compiler's hazard recognizer does not see into inline asm.  Wave 0 runs these with every lane active.)
#ifndef GPK_DPP_VOLATILE
#define GPK_DPP_VOLATILE 0  // 1: the DPP statements in program order (asm volatile); 0: the scheduler interleaves them
#endif
#if GPK_DPP_VOLATILE
#define GPK_DPP_VOL volatile
#else
#define GPK_DPP_VOL
#endif
template <int C>
__device__ __forceinline__ double row_bcast(double v) {
  double r;
  asm GPK_DPP_VOL("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(v), "n"(C));
  return r;
}
template <int C>
__device__ __forceinline__ void fmac_row_bcast(double& w, double u, double ng) {
  asm GPK_DPP_VOL("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(w) : "v"(u), "v"(ng),
      "n"(C));
}
// potf2 pivot J (mode 2): every 16-lane row holds the whole problem -- lane r the tile row r (w) and column r of
// the inverse (v) -- so column J of the tile, entry (c, J) in lane c's w[J], reaches every lane of the row by DPP
// inside the FMAs; the same arithmetic as the other modes: a = x[J] / L[J][J]; x[J] = a; x[c] -= (a / L[J][J]) u[c]
template <int J, int C>
struct Potf2Upd {
  static __device__ __forceinline__ void run(double* w, double* v, double u, double ngw, double ngv) {
    fmac_row_bcast<C>(w[C], u, ngw);
    fmac_row_bcast<C>(v[C], u, ngv);
    Potf2Upd<J, C + 1>::run(w, v, u, ngw, ngv);
  }
};
template <int J>
struct Potf2Upd<J, 16> {
  static __device__ __forceinline__ void run(double*, double*, double, double, double) {}
};
template <int J>
struct Potf2Step {
  static __device__ __forceinline__ void run(double* w, double* v, int& bad) {
    const double u = w[J];
    const double piv = row_bcast<J>(u);
    bad = (bad == 0 && !(piv > 0.0)) ? J + 1 : bad;
    const double ri = rsqrt_refined(piv);  // 1 / L[J][J]
    const double aw = u * ri, av = v[J] * ri;
    const double ngw = -(aw * ri), ngv = -(av * ri);
    w[J] = aw;
    v[J] = av;
    Potf2Upd<J, J + 1>::run(w, v, u, ngw, ngv);
    Potf2Step<J + 1>::run(w, v, bad);
  }
};
template <>
struct Potf2Step<16> {
  static __device__ __forceinline__ void run(double*, double*, int&) {}
};

template <int C>
__device__ __forceinline__ void fmac_bcast_v(double& w, double u, double ng) {
  // (no wait states: u was written many instructions earlier -- tools/isa_dpp_hazard.py checks the binary)
  asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(w) : "v"(u), "v"(ng),
               "n"(C));
}
template <int C>
__device__ __forceinline__ double bcast_v(double v) {
  double r;
  asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(v), "n"(C));
  return r;
}
__device__ __forceinline__ double vmul(double a, double b) {
  double r;
  asm volatile("v_mul_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double vmul_mhalf(double a) {  // a * -0.5
  double r;
  asm volatile("v_mul_f64 %0, %1, -0.5" : "=v"(r) : "v"(a));
  return r;
}
__device__ __forceinline__ double vmul_neg(double a, double b) {  // a * (-b)
  double r;
  asm volatile("v_mul_f64 %0, %1, -%2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double vfma(double a, double b, double c) {
  double r;
  asm volatile("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ double vrsq(double a) {
  double r;
  asm volatile("v_rsq_f64 %0, %1" : "=v"(r) : "v"(a));
  return r;
}
// deferred FMA number D of pivot J - 1 (issued during pivot J): v[J] first (this pivot's a reads it), then
// w[c], v[c] for c = J + 1 .. 15 (w[J] was the previous pivot's critical FMA)
template <int J, int D>
struct DeferOp {
  static __device__ __forceinline__ void run(double* w, double* v, double up, double ngw, double ngv) {
    constexpr int ND = (J == 0) ? 0 : 1 + 2 * (DB - 1 - J);
    if constexpr (D < ND && !(GPK_PIPE_NOINV && (D == 0 || ((D - 1) & 1) != 0))) {  // (NOINV: probe builds only)
      // (entry c takes column entry (c, J - 1), i.e. lane c's u)
      if constexpr (D == 0) {
        fmac_bcast_v<J>(v[J], up, ngv);
      } else {
        constexpr int C = J + 1 + (D - 1) / 2;
        if constexpr (((D - 1) & 1) != 0)
          fmac_bcast_v<C>(v[C], up, ngv);
        else
          fmac_bcast_v<C>(w[C], up, ngw);
      }
    }
  }
};
template <int J, int D0, int D1>
struct DeferRange {
  static __device__ __forceinline__ void run(double* w, double* v, double up, double ngw, double ngv) {
    if constexpr (D0 < D1 && D0 < 2 * DB) {
      DeferOp<J, D0>::run(w, v, up, ngw, ngv);
      DeferRange<J, D0 + 1, D1>::run(w, v, up, ngw, ngv);
    }
  }
};
template <int J>
struct PipeStep {
  static __device__ __forceinline__ void run(double* w, double* v, int& bad, double up, double ngwp, double ngvp,
                                             double c15) {
    if constexpr (J < DB) {
      const double u = w[J];
      const double piv = bcast_v<J>(u);
      if (!GPK_PIPE_NOBAD) bad = (bad == 0 && !(piv > 0.0)) ? J + 1 : bad;
      const double r0 = vrsq(piv);
      const double hn = vmul_mhalf(piv);
      DeferRange<J, 0, 3>::run(w, v, up, ngwp, ngvp);
      double t = vmul(hn, r0);
      DeferRange<J, 3, 4>::run(w, v, up, ngwp, ngvp);
      t = vfma(t, r0, c15);
      DeferRange<J, 4, 5>::run(w, v, up, ngwp, ngvp);
      const double r1 = vmul(r0, t);
      DeferRange<J, 5, 6>::run(w, v, up, ngwp, ngvp);
      double ri = r1;
      if constexpr (GPK_PIPE_NEWTON >= 2) {
        t = vmul(hn, r1);
        DeferRange<J, 6, 7>::run(w, v, up, ngwp, ngvp);
        t = vfma(t, r1, c15);
        DeferRange<J, 7, 8>::run(w, v, up, ngwp, ngvp);
        ri = vmul(r1, t);  // 1 / L[J][J]
        DeferRange<J, 8, 9>::run(w, v, up, ngwp, ngvp);
      }
      const double aw = vmul(u, ri), av = vmul(v[J], ri);
      const double ngw = vmul_neg(aw, ri), ngv = vmul_neg(av, ri);
      if constexpr (J + 1 < DB) fmac_bcast_v<J + 1>(w[J + 1], u, ngw);  // the next pivot's input
      DeferRange<J, (GPK_PIPE_NEWTON >= 2 ? 9 : 6), 2 * DB>::run(w, v, up, ngwp, ngvp);  // the rest of the previous pivot's FMAs
      w[J] = aw;
      v[J] = av;
      PipeStep<J + 1>::run(w, v, bad, u, ngw, ngv, c15);
    }
  }
};
// pivot j's chain: bcast -> rsq -> 2 Newton steps -> a -> -a / L[j][j] -> the FMA of entry j + 1 (the next
// pivot's input), ~110 cycles; its other 2 (15 - j) FMAs go into the latency gaps of pivot j + 1's chain instead
// of in front of it.  Every instruction pinned in that order (asm volatile).  Measured per wave (tools/probe):
// dependent f64 FMA 8 cycles, rsq 20, 64-bit DPP move 16 (with its two wait states), independent f64 FMA issue
// 5, mode 0's LDS round trip 112.  The same operations on the same values as the other modes: the same bits.
__device__ __forceinline__ void potf2_pipelined(double* w, double* v, int& bad) {
  PipeStep<0>::run(w, v, bad, 0.0, 0.0, 0.0, 1.5);
}

// potf2 + inverse of tile (kb, kb), one wave.  Lanes 0..15 hold row r = lane of the tile and
// factor it (right-looking); lanes 16..31 hold column r = lane - 16 of the identity and turn it
// into column r of L^-1 (column-oriented forward substitution).  Both run the SAME update per
// pivot j with w = their 16 values:   a = w[j] / L[j][j];  w[j] = a;  w[c] -= a L[c][j] (c > j)
// (for a row of A, a = L[r][j]; for a column of the inverse, a = (L^-1)[j][r]).  Column j of L is
// broadcast through LDS: written by lanes 0..15, read back by every lane with 8 broadcast
// ds_read_b128.  Lanes 32..63 mirror 0..31 and never store.  (The earlier form -- one readlane
// per element and a separate substitution -- took 2 x 480 readlanes and spilled SGPRs.)
__device__ __forceinline__ void potf2_tile(double* A, double* Dk, double* colbuf, int kb, int lane,
                                           int* flag, int64_t col_base) {
  typedef double dbl2 __attribute__((ext_vector_type(2)));
  const int r = lane & 15;
  const bool inv = (lane & 16) != 0;
  const int c0 = kb * DB;
#if GPK_POTF2_MODE == 2
  {
    (void)inv;
    (void)colbuf;
    double w[DB], v[DB];
#pragma unroll
    for (int c = 0; c < DB; c += 2) {
      const dbl2 t = *reinterpret_cast<const dbl2*>(A + aidx(c0 + r, c0 + c));
      w[c] = t.x;
      w[c + 1] = t.y;
      v[c] = (c == r) ? 1.0 : 0.0;
      v[c + 1] = (c + 1 == r) ? 1.0 : 0.0;
    }
    int bad = 0;
#if GPK_POTF2_PIPE
    potf2_pipelined(w, v, bad);
#else
    Potf2Step<0>::run(w, v, bad);
#endif
#pragma unroll
    for (int c = 0; c < DB; ++c) asm volatile("" : "+v"(w[c]), "+v"(v[c]));  // (computed here, every lane active)
    if (bad != 0 && lane == 0 && *flag == 0) *flag = (int)(col_base + c0 + bad);
    if (lane < DB) {
#pragma unroll
      for (int c = 0; c < DB; ++c) A[aidx(c0 + r, c0 + c)] = (c <= r) ? w[c] : 0.0;
    } else if (lane < 2 * DB) {
#pragma unroll
      for (int rr = 0; rr < DB; ++rr) Dk[rr * DBS + r] = v[rr];  // Dinv[rr][r]
    }
    return;
  }
#endif
  // rows: entries above the diagonal are never used (only c <= r is stored, and column j is
  // read from rows c >= j only), so the tile row is loaded whole
  double w[DB];
#pragma unroll
  for (int c = 0; c < DB; c += 2) {
    const dbl2 t = *reinterpret_cast<const dbl2*>(A + aidx(c0 + r, c0 + c));
    w[c] = inv ? ((c == r) ? 1.0 : 0.0) : t.x;
    w[c + 1] = inv ? ((c + 1 == r) ? 1.0 : 0.0) : t.y;
  }
  int bad = 0;  // first non-positive pivot of this tile (1-based in the tile), wave-uniform
#pragma unroll
  for (int j = 0; j < DB; ++j) {
    double u[DB];
#if GPK_POTF2_READLANE
    // column j, entry (c, j) from lane c (which holds row c), straight into SGPRs: the same values as the
    // LDS form below without its store -> wait -> load round trip on the pivot chain (D task 33 -> ? us)
#pragma unroll
    for (int c = j; c < DB; ++c) u[c] = bcast_lane(w[j], c);
    (void)colbuf;
#else
    double* cb = colbuf + (j & 1) * DB;
    if (lane < DB) cb[lane] = w[j];            // column j: entry (r, j) of row r
    // Other lanes' stores are invisible to the per-thread memory model: without a fence hipcc
    // may serve the reads below from the loads of step j - 2 (same buffer).  The wave's LDS
    // operations retire in order, so a wave-scope fence is all the hardware needs.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int c = j & ~1; c < DB; c += 2) {
      const dbl2 t = *reinterpret_cast<const dbl2*>(cb + c);
      u[c] = t.x;
      u[c + 1] = t.y;
    }
#endif
    const double piv = u[j];
    bad = (bad == 0 && !(piv > 0.0)) ? j + 1 : bad;
    const double ri = rsqrt_refined(piv);      // 1 / L[j][j]
    const double aj = w[j] * ri;
    const double g = aj * ri;  // w[c] -= (w[j] / L[j][j]) (u[c] / L[j][j]): one FMA per entry
    w[j] = aj;
#pragma unroll
    for (int c = j + 1; c < DB; ++c) w[c] = fma(-g, u[c], w[c]);
  }
  if (bad != 0 && lane == 0 && *flag == 0) *flag = (int)(col_base + c0 + bad);
  if (lane < DB) {
#pragma unroll
    for (int c = 0; c < DB; ++c) A[aidx(c0 + r, c0 + c)] = (c <= r) ? w[c] : 0.0;
  } else if (lane < 2 * DB) {
#pragma unroll
    for (int rr = 0; rr < DB; ++rr) Dk[rr * DBS + r] = w[rr];  // Dinv[rr][r]
  }
}

// 16-B vectors of the block loads and stores
template <typename T>
struct Vec16;
template <>
struct Vec16<double> {
  typedef double type __attribute__((ext_vector_type(2)));
};
template <>
struct Vec16<float> {
  typedef float type __attribute__((ext_vector_type(4)));
};

// global-address-space views (the hand-off words and payloads are always global_ accesses, never flat_)
typedef __attribute__((address_space(1))) uint64_t gu64;
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) int32_t gi32;

// Global accesses of the block code.  SC1 (chain_kernel): W / Winv bytes are handed to workgroups on
// other XCDs inside one launch, so every store of them is an agent-scope relaxed atomic (global_store
// ... sc1: written through the XCD's L2), and the consumer reads them with plain loads behind one agent
// acquire (buffer_inv sc1: the CU's L1 and the XCD's L2 drop their stale lines) issued after its waits
// (MI355X guide, inter-workgroup visibility).  (Until round 3's last measurements the loads were
// relaxed 8-byte atomics too -- twice the load instructions for the same bytes.)
template <bool SC1, typename T>
__device__ __forceinline__ typename Vec16<T>::type ldv(const T* p) {
  return *reinterpret_cast<const typename Vec16<T>::type*>(p);
}
#ifdef GPK_CHAIN_SC1LD
constexpr bool kChainSc1Ld = true;  // (A/B: chain tasks read through 16-B sc1 buffer loads, no acquire)
#else
constexpr bool kChainSc1Ld = false;
#endif
// a buffer resource over a wave-uniform base (readfirstlane: the compiler cannot prove it uniform), 1 GiB
// long: an offset of kRsrcBytes or more is out of range -- the load returns 0 and touches no memory
constexpr int kRsrcBytes = 0x40000000;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint64_t uu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(u >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(uu), 0, kRsrcBytes, 0x00020000);
}
// 16-B / 8-B buffer loads: one VGPR offset per lane, the wave-uniform part in soffset (an SGPR), so a
// batch of loads needs no per-load 64-bit address registers (hoisted and spilled in chain_kernel, each
// reload then waited vmcnt(0) -- the diagonal task's 16 block loads went out one at a time).  aux 16: sc1.
constexpr int kLdAux = kChainSc1Ld ? 16 : 0;
__device__ __forceinline__ Vec16<double>::type ld16_buf(__amdgpu_buffer_rsrc_t rs, int vo, int so) {
  return __builtin_bit_cast(Vec16<double>::type, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, so, kLdAux));
}
__device__ __forceinline__ double ld8_buf(__amdgpu_buffer_rsrc_t rs, int vo, int so) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, vo, so, kLdAux));
}
// threadIdx.x behind an empty volatile asm: in chain_kernel's task loop every task body then recomputes
// its per-lane addresses instead of the compiler hoisting them out of the loop for all task types at
// once and spilling them (their scratch reloads waited behind the write-through stores)
__device__ __forceinline__ int opaque_tid() {
  int t = (int)threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}
// Hand-off words of the persistent factorisation (gpk_potrf.hip, chain_kernel): agent-scope relaxed atomics
__device__ __forceinline__ int32_t ld_flag(const int32_t* p) {
  return __hip_atomic_load((gi32*)const_cast<int32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_flag(int32_t* p, int32_t v) {
  __hip_atomic_store((gi32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Persistent launches that timed out, since the library was loaded (one count per launch: the waiter that
// raises the launch's abort word adds it); read by gpk_chain_stats (gpk_potrf.hip, chain_timeouts_read), so
// that a caller that never reads info (the bench's pipelined steps) can still tell whether any run aborted.
// (Per translation unit: only gpk_potrf.hip's chain_kernel waits.)
static __device__ unsigned long long g_chain_timeouts_dev = 0;

// A wait of the persistent launch timed out: raise the launch's abort word (the first to raise it counts the launch in
// g_chain_timeouts_dev) and set info = -1 on every member where no non-positive pivot was found first.  One wave.
__device__ __forceinline__ void chain_report_timeout(int32_t* ctl, int32_t* info, int nmem) {
  const int lane = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  if (lane == __builtin_amdgcn_readfirstlane(lane)) {
    const int32_t was = __hip_atomic_exchange((gi32*)(ctl + 1), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (was == 0) __hip_atomic_fetch_add(&g_chain_timeouts_dev, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  for (int m = 0; m < nmem; ++m) {
    int32_t zero = 0;
    __hip_atomic_compare_exchange_strong((gi32*)(info + m), &zero, -1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
  }
}

// one wave: wait until *p >= v; false on timeout (which it reports) or after another task's timeout.  Plain
// values (the task bodies call it too, and they must not take the kernel argument by reference)
__device__ __forceinline__ bool chain_wait_v(const int32_t* p, int32_t v, int32_t* ctl, int32_t* info, int nmem,
                                             int64_t timeout, int force_abort, uint64_t t0) {
  // (polled values through readfirstlane: the loop is wave-uniform, as every branch of chain_kernel)
  while (force_abort || __builtin_amdgcn_readfirstlane(ld_flag(p)) < v) {
    if (__builtin_amdgcn_readfirstlane(ld_flag(ctl + 1)) != 0) return false;
    if (force_abort || __builtin_amdgcn_s_memrealtime() - t0 > (uint64_t)timeout) {
      chain_report_timeout(ctl, info, nmem);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}
// Workgroup barrier.  SC1: an LDS-only one -- __syncthreads() also waits for every outstanding global
// access of the wave (vmcnt(0)), and with write-through stores in flight each of the block's 17 barriers
// waited for their acknowledgement from beyond the L2.  Nothing in the block body reads back what it
// stored (the persistent kernel drains the stores before it publishes).
#ifndef GPK_DIAG_LDS_BARRIER
#define GPK_DIAG_LDS_BARRIER 0  // 1: the LDS-only barrier in the launch path's diagonal kernels too (A/B)
#endif
template <bool SC1>
__device__ __forceinline__ void wg_sync() {
  if constexpr (SC1 || GPK_DIAG_LDS_BARRIER) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  } else {
    __syncthreads();
  }
}
template <bool SC1, typename T>
__device__ __forceinline__ void stv(T* p, typename Vec16<T>::type v) {
  if constexpr (SC1) {
    struct W2 {
      uint64_t a, b;
    };
    const W2 w = __builtin_bit_cast(W2, v);
    gu64* q = (gu64*)p;
    __hip_atomic_store(q, w.a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 1, w.b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    *reinterpret_cast<typename Vec16<T>::type*>(p) = v;
  }
}
template <bool SC1, typename T>
__device__ __forceinline__ void sts(T* p, T v) {
  if constexpr (SC1 && sizeof(T) == 8) {
    __hip_atomic_store((gu64*)p, __builtin_bit_cast(uint64_t, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if constexpr (SC1) {
    __hip_atomic_store((gu32*)p, __builtin_bit_cast(uint32_t, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    *p = v;
  }
}

// ------------------------------------------------------------------------------------------------
// Look-ahead form (diag_version 2).  The same tile algebra, scheduled so that the potf2 chain -- the
// only inherently sequential part -- is the critical path and everything else runs beside it:
//
//   P_s  wave 0     : potf2 + inverse of tile (s, s)
//        waves 1..7 : trailing update of step s-1 for tile columns j >= s + 1; block row I = s - 1
//                     of L^-1; L's block row s - 1 and L^-1's block row s - 2 to HBM
//   ---- barrier
//   QR_s wave w     : row i = s + 1 + w: X_i = A_{i,s} Dinv_s^T and X_{s+1}, both computed transposed
//                     (Dinv_s A^T), which puts X[r][k = lk + 4q] in the registers of lane (r, lk) --
//                     the MFMA operand layout -- then A_{i,s+1} -= X_i X_{s+1}^T: tile column s + 1
//                     is up to date for potf2(s + 1) without waiting for the rest of the update
//   ---- barrier
// L^-1 lives in the block's upper tiles, which the factorisation never touches: tile (I, J) of L^-1
// (J < I) is stored transposed as tile (J, I), its diagonal tiles stay in Dinv -- so no in-place
// hazard, and each tile of L^-1 goes to HBM from the registers that computed it (the zero tiles in
// P_0, where waves 1..7 are idle).  Two barriers
// per step instead of three, the inverse and every HBM store off the critical path, and 16-B loads of
// the lower tiles only (the upper tiles of the block are never read).
template <typename T, bool SC1 = false>
__device__ __forceinline__ void store_l_rows(const double* A, T* Wb, int64_t ld, int I, int t, int nt) {
  // rows 16 I .. 16 I + 15 of L, columns 0 .. row (lower triangle only, as the phase-serial kernel)
  constexpr int EPC = 16 / (int)sizeof(T);
  typedef T vT __attribute__((ext_vector_type(EPC)));
  const int ppr = (I + 1) * DB / EPC;  // pieces of a row up to the end of its diagonal tile
  for (int e = t; e < DB * ppr; e += nt) {
    const int r = I * DB + e / ppr, pc = e % ppr, c0 = pc * EPC;
    if (c0 + EPC - 1 <= r) {
      vT v;
#pragma unroll
      for (int u = 0; u < EPC; ++u) v[u] = (T)A[aidx(r, c0 + u)];
      stv<SC1, T>(Wb + (int64_t)r * ld + c0, v);
    } else {
#pragma unroll
      for (int u = 0; u < EPC; ++u)
        if (c0 + u <= r) sts<SC1>(Wb + (int64_t)r * ld + c0 + u, (T)A[aidx(r, c0 + u)]);
    }
  }
}

template <typename T, bool SC1 = false>
__device__ __forceinline__ void store_inv_zeros(T* Ib, int t, int nt) {
  // the tiles right of L^-1's diagonal tiles: zeros (read as such by the panel solve's MFMA chunks)
  constexpr int EPC = 16 / (int)sizeof(T);
  typedef T vT __attribute__((ext_vector_type(EPC)));
  constexpr int PPT = DB / EPC;  // pieces per tile row
  for (int e = t; e < NB * NB / EPC; e += nt) {
    const int r = e / (NB / EPC), c0 = (e % (NB / EPC)) * EPC;
    if (c0 / DB > r / DB) {
      vT v;
#pragma unroll
      for (int u = 0; u < EPC; ++u) v[u] = (T)0;
      stv<SC1, T>(Ib + r * NB + c0, v);
    }
  }
  (void)PPT;
}

template <typename T, bool SC1 = false>
__device__ __forceinline__ void store_inv_diag(const double* Dinv, T* Ib, int I, int t, int nt) {
  // diagonal tile I of L^-1 (Dinv_I, zeros above its diagonal)
  for (int e = t; e < DB * DB; e += nt)
    sts<SC1>(Ib + (I * DB + e / DB) * NB + I * DB + e % DB, (T)Dinv[I * DTS + (e / DB) * DBS + e % DB]);
}

// tile (I, J) of L^-1, J < I: -Dinv_I sum_{K=J}^{I-1} L_{I,K} Linv_{K,J}, stored transposed in tile (J, I)
template <typename T, bool SC1 = false>
__device__ __forceinline__ void inverse_tile(double* A, const double* Dinv, T* Ib, int I, int J, int lr, int lk,
                                             bool st = true) {
  d4 tacc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s = 0; s < 4; ++s)  // K = J: the diagonal tile Dinv_J
    tacc = mfma64(A[aidx(I * DB + lr, J * DB + 4 * s + lk)], Dinv[J * DTS + (4 * s + lk) * DBS + lr], tacc);
  for (int K = J + 1; K < I; ++K) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
      tacc = mfma64(A[aidx(I * DB + lr, K * DB + 4 * s + lk)], A[aidx(J * DB + lr, K * DB + 4 * s + lk)], tacc);
  }
  const double* Di = Dinv + I * DTS;
  d4 out = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s = 0; s < 4; ++s) out = mfma64(-Di[lr * DBS + 4 * s + lk], tacc[s], out);
  // out[q] = Linv_{I,J}[lk + 4q][lr]  ->  tile (J, I) [lr][lk + 4q] for the later rows, and straight
  // from the registers to HBM (16 lanes of a row store 128 contiguous bytes)
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    A[aidx(J * DB + lr, I * DB + lk + 4 * q)] = out[q];
    if (st) sts<SC1>(Ib + (I * DB + lk + 4 * q) * NB + J * DB + lr, (T)out[q]);
  }
}

// rows [r0, r1) of member b are zero in the panel columns [j0, j0 + 128) (gpk_potrf.hip's zero_rows
// for a panel solve: identity extra rows past the panel, a ragged member's padding / unused test rows)
__device__ __forceinline__ bool panel_zero_rows(const DiagArgs& a, int b, int64_t r0, int64_t r1) {
  if (r0 >= a.zlo && r1 <= a.zhi) return true;
  if (a.nb == nullptr) return false;
  const int64_t npb = (a.nb[b] + NB - 1) / NB * NB;
  const int64_t jend = a.j0 + NB;
  if (a.j0 >= npb) return r0 >= jend && r1 <= a.p;
  if (r0 >= (npb > jend ? npb : jend) && r1 <= a.n_pad) return true;
  return a.mb != nullptr && r0 >= a.n_pad + a.mb[b] && r1 <= a.y_row;
}

// The end of QR_s without wave 0 (GPK_DIAG_QR_LDSBAR): wave 0's next step needs only its own QR_s result (the pivot
// tile (s + 1, s + 1); the P_s barrier already covered the trailing update of it), so waves 1..7 meet on an LDS counter
// instead of the workgroup barrier (they exchange the X_i of QR_s for P_{s+1}'s trailing tiles) and wave 0 goes on
// into potf2(s + 1) at once.  Its one write that waves 1..7 could still be reading -- X_{s+1} into tile (s + 1, s),
// whose pre-solve values their QR_s reads -- waits for the counter, after the potf2.  Phase-profile (N = 4096,
// r06m): wave 0 waited 600-2550 cycles per step at that barrier for the other waves' longer QR work.
#ifndef GPK_DIAG_QR_LDSBAR
#define GPK_DIAG_QR_LDSBAR 1
#endif
__device__ __forceinline__ void lds_counter_arrive(int* cnt) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");  // (this wave's LDS reads and writes retired first)
  const int lane = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  if (lane == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_counter_wait(int* cnt, int target) {
  while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < target)
    __builtin_amdgcn_s_sleep(0);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// FUSE (f64): a workgroup with ticket t (DiagArgs) also solves the 64 rows R = row0 + 64 t .. +63 of the panel:
// X = A L_kk^-T with the same MFMA k-order as gemm_kernel<TRSM> (k-step s of chunk kc takes k = 16 kc +
// 2 q + 8 (s >> 1) + (s & 1) in lane group q; chunks kc > the column block skipped), so X is bitwise
// the separate panel solve's.  Wave w: 16-row block w & 3, column blocks of half w >> 2 (balanced).  Its A operands (32
// doubles per lane) are loaded during the last step of the factorisation.
template <typename T, bool FUSE, bool SC1 = false>
__device__ __forceinline__ void diag2_body(const DiagArgs& a, int b_in, double* sm) {
  const int b = FUSE ? (int)blockIdx.y : b_in;
  double* A = sm;
  double* Dinv = A + LDS_A;
  double* colbuf = Dinv + LDS_DINV;
  int* flag = reinterpret_cast<int*>(colbuf + LDS_COL);

  const int tid = SC1 ? opaque_tid() : (int)threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15;
  const int lk = lane >> 4;
  int* ticket = flag + 1;
  int* qrcnt = flag + 2;  // (GPK_DIAG_QR_LDSBAR) arrivals of waves 1..7 at the ends of the QR phases
  T* Wb = reinterpret_cast<T*>(a.W) + (int64_t)b * a.w_bs + a.j0 * a.ld + a.j0;
  T* Ib = reinterpret_cast<T*>(a.Winv) + (int64_t)b * a.inv_bs + a.kblk * NB * NB;
  typedef double dbl2 __attribute__((ext_vector_type(2)));
  dbl2 pa[FUSE ? NTL : 1][2];  // A operands: chunk kc, pieces lk and lk + 4 (k-steps 0, 1 and 2, 3)
  // (GPK_DIAG_PROF builds: lane 0 of every wave stamps the shader clock at the phase boundaries of each step --
  // 0 P_s start, 1 P_s work done, 2 QR_s start, 3 QR_s work done; step 0 / 5: block loaded, step 7 / 4: end)
  auto stamp = [&](int s, int ph) {
    if constexpr (GPK_DIAG_PROF != 0) {
      if (a.prof && lane == 0) a.prof[((a.kblk * NTL + s) * 8 + wave) * 6 + ph] = __builtin_amdgcn_s_memtime();
    }
  };
  {
    // the lower 16-tiles of the block, 16 B per load, every load of a thread in flight at once
    constexpr int EPC = 16 / (int)sizeof(T);
    typedef T vT __attribute__((ext_vector_type(EPC)));
    constexpr int PPR = NB / EPC, RPP = DT / PPR, NPASS = NB / RPP;
    const int pc = tid % PPR, r0 = tid / PPR;
    vT v[NPASS];
#pragma unroll
    for (int q = 0; q < NPASS; ++q) {
      const int r = r0 + q * RPP;
      if (pc * EPC <= (r | (DB - 1))) {
        if constexpr (SC1)
          v[q] = __builtin_bit_cast(vT, ld16_buf(uniform_rsrc(Wb), (int)(((int64_t)r0 * a.ld + pc * EPC) * sizeof(T)),
                                                 __builtin_amdgcn_readfirstlane((int)((int64_t)q * RPP * a.ld * sizeof(T)))));
        else
          v[q] = ldv<SC1, T>(Wb + (int64_t)r * a.ld + pc * EPC);
      }
    }
#pragma unroll
    for (int q = 0; q < NPASS; ++q) {
      const int r = r0 + q * RPP;
      if (pc * EPC <= (r | (DB - 1))) {
#pragma unroll
        for (int u = 0; u < EPC; ++u) A[aidx(r, pc * EPC + u)] = (double)v[q][u];
      }
    }
  }
  if (tid == 0) {
    *flag = 0;
    *qrcnt = 0;
  }
  stamp(0, 5);
  wg_sync<SC1>();
  if (FUSE) {
    // the whole block is in LDS (every load retired into the LDS stores above): draw the ticket
    // tickets 0 .. grid - 1; the grid's last draw wraps the counter to 0 for the next launch
    if (tid == 0) *ticket = (int)atomicInc(reinterpret_cast<unsigned*>(&a.ctr[b]), gridDim.x - 1u);
    wg_sync<SC1>();
  }
  // FUSE: the last workgroup to load writes (alone, so its HBM stores never sit in front of a tile's
  // solve); the others solve tile = ticket
  const int tk = FUSE ? *ticket : 0;
  const bool wr = !FUSE || tk == (int)gridDim.x - 1;
  const int64_t R = a.row0 + (int64_t)tk * 64;
  const bool live = FUSE && !wr && !panel_zero_rows(a, b, R, R + 64);

  // FUSE: the panel rows' A operands (32 doubles per lane) are loaded in the last step -- waves 1..7 at its
  // start, wave 0 after its potf2 -- so their latency hides under that step; the last step is peeled off
  // the loop, so they are not live (and do not spill) through the earlier steps
  bool fetched = false;
  auto prefetch = [&]() {
    if (!FUSE || !live) return;
    const double* Ar = reinterpret_cast<const double*>(a.W) + (int64_t)b * a.w_bs +
                       (R + (wave & 3) * DB + lr) * a.ld + a.j0 + 2 * lk;
#pragma unroll
    for (int kc = 0; kc < NTL; ++kc) {
      pa[kc][0] = *reinterpret_cast<const dbl2*>(Ar + kc * DB);
      pa[kc][1] = *reinterpret_cast<const dbl2*>(Ar + kc * DB + 8);
    }
    fetched = true;
  };
  d4 xs = {0.0, 0.0, 0.0, 0.0};  // wave 0: X_{s+1} (operand layout) from QR_s, stored in P_{s+1}
  auto step = [&](int s, auto last) {
    // ---------------------------------------------------------------- P_s
    stamp(s, 0);
    if (decltype(last)::value && wave != 0) prefetch();
    if (wave == 0) {
      if (s > 0 && !GPK_DIAG_QR_LDSBAR) {
#pragma unroll
        for (int q = 0; q < 4; ++q) A[aidx(s * DB + lr, (s - 1) * DB + lk + 4 * q)] = xs[q];
      }
      if (!(a.dbg & 2)) potf2_tile(A, Dinv + s * DTS, colbuf, s, lane, flag, a.j0);  // timing ablation
      if (s > 0 && GPK_DIAG_QR_LDSBAR) {
        lds_counter_wait(qrcnt, (NTL - 1) * s);  // (waves 1..7 are past their QR_{s-1} reads of tile (s, s - 1))
#pragma unroll
        for (int q = 0; q < 4; ++q) A[aidx(s * DB + lr, (s - 1) * DB + lk + 4 * q)] = xs[q];
      }
      if (decltype(last)::value) prefetch();
    } else if (s == 0) {
      if (!(a.dbg & 8) && wr && !a.no_inv_zeros) store_inv_zeros<T, SC1>(Ib, tid - 64, DT - 64);  // waves 1..7 are idle in P_0
    } else {
      const int w = wave - 1;
      const int I = s - 1;
      if (w < I && !(a.dbg & 1)) inverse_tile<T, SC1>(A, Dinv, Ib, I, w, lr, lk, wr);
      if (s < NTL - 1) stamp(s, 5);  // (profiling: inverse tile done)
      // trailing update of step s - 1 for tile columns j >= s + 1 (column s was done in QR_{s-1});
      // the last waves take the first tiles (waves 1..I hold an inverse tile)
      const int m = NTL - 1 - s;
      const int ntri = m * (m + 1) / 2;
      int t = (NTL - 2) - w;
      const int nt_all = (a.dbg & 4) ? 0 : ntri;
      auto tile_of = [&](int tt, int& i, int& j) {
        int ti = 0;
        while ((ti + 1) * (ti + 2) / 2 <= tt) ++ti;
        i = s + 1 + ti;
        j = s + 1 + tt - ti * (ti + 1) / 2;
      };
      for (; t < nt_all; t += NTL - 1) {
        int i, j;
        tile_of(t, i, j);
        d4 acc;
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = A[aidx(i * DB + lk + 4 * q, j * DB + lr)];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          acc = mfma64(-A[aidx(i * DB + lr, (s - 1) * DB + 4 * k + lk)],
                       A[aidx(j * DB + lr, (s - 1) * DB + 4 * k + lk)], acc);
#pragma unroll
        for (int q = 0; q < 4; ++q) A[aidx(i * DB + lk + 4 * q, j * DB + lr)] = acc[q];
      }
      if (s < NTL - 1) stamp(s, 4);  // (profiling: trailing tiles done)
      if (!(a.dbg & 8) && wr) {
        if (!a.defer_l_store) store_l_rows<T, SC1>(A, Wb, a.ld, I, tid - 64, DT - 64);
        store_inv_diag<T, SC1>(Dinv, Ib, I, tid - 64, DT - 64);
      }
    }
    stamp(s, 1);
    if (a.half_flag && s == a.half_step && wave != 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wg_sync<SC1>();
    // ---------------------------------------------------------------- QR_s
    stamp(s, 2);
    // (persistent factorisation: block rows 0 .. half_step - 1 of L^-1 went out in P_1 .. P_half_step and every
    // storing wave drained them before the barrier -- an idle wave of this QR phase publishes them for the panel
    // solves' first column blocks)
    if (a.half_flag && s == a.half_step && wave == NTL - 1) {
      __hip_atomic_store((gi32*)a.half_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    xs = d4{0.0, 0.0, 0.0, 0.0};  // (the old value is dead: nothing keeps it alive across potf2)
    if (s < NTL - 1 && wave < NTL - 1 - s && !(a.dbg & 4)) {
      const int i = s + 1 + wave;
      const double* Dk = Dinv + s * DTS;
      d4 xi = {0.0, 0.0, 0.0, 0.0}, x1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double dv = Dk[lr * DBS + 4 * k + lk];
        xi = mfma64(dv, A[aidx(i * DB + lr, s * DB + 4 * k + lk)], xi);
        if (wave != 0) x1 = mfma64(dv, A[aidx((s + 1) * DB + lr, s * DB + 4 * k + lk)], x1);
      }
      if (wave == 0) x1 = xi;
      // xi[q] = X_i[lr][lk + 4q]: the A operand of k-step q; x1 likewise the B operand
      d4 acc;
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = A[aidx(i * DB + lk + 4 * q, (s + 1) * DB + lr)];
#pragma unroll
      for (int q = 0; q < 4; ++q) acc = mfma64(-xi[q], x1[q], acc);
#pragma unroll
      for (int q = 0; q < 4; ++q) A[aidx(i * DB + lk + 4 * q, (s + 1) * DB + lr)] = acc[q];
      xs = xi;  // wave 0: tile (s + 1, s) is read by every wave of this phase, stored in P_{s+1}
      if (wave != 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) A[aidx(i * DB + lr, s * DB + lk + 4 * q)] = xi[q];
      }
    }
    stamp(s, 3);
    if (GPK_DIAG_QR_LDSBAR && s < NTL - 1) {
      if (wave != 0) {
        lds_counter_arrive(qrcnt);
        lds_counter_wait(qrcnt, (NTL - 1) * (s + 1));
      }
    } else {
      wg_sync<SC1>();
    }
    };
  const int nsteps = (a.dbg & 16) ? 0 : NTL;
#pragma unroll 1
  for (int s = 0; s + 1 < nsteps; ++s) step(s, std::false_type());
  if (nsteps > 0) step(nsteps - 1, std::integral_constant<bool, FUSE>());
  // after P_7: block row 7 of L to HBM, rows 6 and 7 of L^-1
  if (a.dbg & 32) return;  // timing ablation
  if (!fetched) prefetch();  // (only when the step loop was ablated away)
  if (wave >= 1) {
    inverse_tile<T, SC1>(A, Dinv, Ib, NTL - 1, wave - 1, lr, lk, wr);
  } else if (wr) {
    store_inv_diag<T, SC1>(Dinv, Ib, NTL - 1, lane, 64);
  }
  if (wr) {
    if (!a.defer_l_store) store_l_rows<T, SC1>(A, Wb, a.ld, NTL - 1, tid, DT);
    if (tid == 0 && *flag != 0) atomicCAS(&a.info[b], 0, *flag);
  }
  stamp(NTL - 1, 4);
  if (!FUSE) return;
  wg_sync<SC1>();  // block row 7 of L^-1 in LDS
  if (!live) return;
  // Linv[c][k] (c in tile I, k in tile J <= I): tile (J, I) of A transposed for J < I, Dinv_I for J = I
  const int rb = wave & 3, ch = wave >> 2;
  double* Xr = reinterpret_cast<double*>(a.W) + (int64_t)b * a.w_bs + (R + rb * DB + lk) * a.ld + a.j0 + lr;
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    // column block = tile row I of L^-1; block cb takes cb + 1 chunks, so the halves {0, 7, 2, 5} and
    // {1, 6, 3, 4} carry 18 chunks each (contiguous halves: 10 and 26)
    const int cb = (n & 1) ? 7 - 2 * (n >> 1) - ch : 2 * (n >> 1) + ch;
    d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kc = 0; kc < NTL; ++kc) {
      if (kc > cb) break;
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const int x = 2 * lk + 8 * (st >> 1) + (st & 1);  // k within the chunk
        const double bv = (kc < cb) ? A[aidx(kc * DB + x, cb * DB + lr)] : Dinv[cb * DTS + lr * DBS + x];
        acc = mfma64(pa[kc][st >> 1][st & 1], bv, acc);
      }
    }
    // C/D layout: col = lr, row = lk + 4 q
#pragma unroll
    for (int q = 0; q < 4; ++q) Xr[(int64_t)(4 * q) * a.ld + cb * DB] = acc[q];
  }
}

}  // namespace
}  // namespace gpk
