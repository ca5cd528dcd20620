// MFMA GEMM of the blocked Cholesky (panel solve + trailing update), the read-out, and the
// triangular solves.  The diagonal-block factorisation lives in gpk_diag.hip.
//
// Replaces tf.linalg.cholesky / tf.linalg.triangular_solve of
// gpbasics/Statistics/CovarianceMatrix.py:247-265 and the log-determinant / data-fit
// assembly of gpbasics/Metrics/Metrics.py:152-154 and gpbasics/Metrics/LogLikelihood.py:30-65.
//
// Per panel step k (columns j0 = 128k .. j0+127):
//   gemm<TRSM>    rows below the block: W[R, j0:j0+128] <- W[R, j0:j0+128] * L_kk^-T, an MFMA
//                 GEMM against the inverted diagonal block (upper zero blocks skipped); every
//                 row of the augmented matrix, so z = L^-1 y and V^T = Ks^T L^-T come out of it
//   gemm<UPDATE>  lower tiles of the trailing matrix: C -= P P^T, f64 MFMA
//                 (v_mfma_f64_16x16x4_f64) or f32 MFMA (v_mfma_f32_16x16x4_f32)
// Tiles are TM x TN (128 x 128 while the grid fills the chip, 64 x 64 on small trailing
// matrices); a 256-thread workgroup = 2 x 2 waves, double-buffered LDS staging of 16-deep K
// chunks through registers; block ids are remapped so that each XCD (blockIdx % 8) walks runs of
// consecutive tiles, which share panel rows in its L2 (xcd_remap).
#include <math.h>

#include "gpk_diag_dev.h"
#include "gpk_internal.h"
#include "gpk_kernels.h"

namespace gpk {
namespace {

template <typename T>
struct Mfma;
template <>
struct Mfma<double> {
  typedef d4 acc_t;
  static __device__ __forceinline__ acc_t op(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  // c - a b: on the f64 MFMA the blgp field is the neg modifier (neg:[1,0,0] negates A)
  static __device__ __forceinline__ acc_t op_neg(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 1);
  }
  // v_mfma_f64_16x16x4_f64 C/D map: col = lane & 15, row = (lane >> 4) + 4 * reg
  static __device__ __forceinline__ int row(int lane, int reg) { return (lane >> 4) + 4 * reg; }
};
template <>
struct Mfma<float> {
  typedef f4 acc_t;
  static __device__ __forceinline__ acc_t op(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ acc_t op_neg(float a, float b, acc_t c) { return op(-a, b, c); }
  // f32 16x16 C/D map: col = lane & 15, row = 4 * (lane >> 4) + reg
  static __device__ __forceinline__ int row(int lane, int reg) { return 4 * (lane >> 4) + reg; }
};

typedef __attribute__((address_space(3))) void lds_void;

// Waves along N of the 128 x 128 update tile: 2 (4 waves of 64 x 64 each) or 4 (8 waves of 64 x 32:
// 111 VGPRs, so two 512-thread workgroups -- four waves per SIMD -- share a CU; f64 update +2.8 %)
#ifndef GPK_UPD_WN
#define GPK_UPD_WN 4
#endif
#ifndef GPK_UPD_WN_F32
#define GPK_UPD_WN_F32 2
#endif

#ifndef GPK_ABLATE
#define GPK_ABLATE 0  // timing-only ablations (wrong results): 1 no C read, 2 no epilogue, 3 K loop x2,
                      // 4 operands from one L2-resident block, 5 no per-chunk barrier
#endif

constexpr int ROWB = 128;  // bytes of one row of a staged K chunk (8 pieces of 16 B)

// bijective XCD-aware remap of the hardware block order (XCD = blockIdx % 8) to logical tiles.
// run = 0: each XCD walks one contiguous run of tile ids, which share panel rows in its L2 (uniform
// batches: the fewest L2 misses).  run > 0: runs of that many consecutive tiles are dealt round-robin
// over the XCDs -- ragged batches, whose members' padding makes contiguous clusters of structurally
// zero tiles that would otherwise leave some XCDs idle: 1 x 8192 + 15 x 4096 members 18.0 -> 16.2 ms;
// on uniform batches runs of 8 are neutral in time but raise the update's L2 misses by 7-13 %
// (profiles/r02y_xcd_runs.txt).
__device__ __forceinline__ int64_t xcd_remap(int64_t bid, int64_t nblk, int64_t run) {
  if (run > 0) {
    const int64_t full = nblk - nblk % (8 * run);
    if (bid >= full) return bid;
    const int64_t x = bid % 8, pos = bid / 8;
    return ((pos / run) * 8 + x) * run + pos % run;
  }
  const int64_t q = nblk / 8, r = nblk % 8;
  const int64_t x = bid % 8, pos = bid / 8;
  const int64_t base = (x < r) ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + pos;
}

// LDS image of a staged K chunk: one 128-B row per operand row, 16-B piece c of row r stored at
// piece c ^ ((r >> 1) & 7).  The 16 rows a quarter-wave ds_read_b128 touches then fill all 16
// slots of a 256-B bank row (conflict-free), while every global_load_lds wave-instruction still
// writes its 1 KiB lane-linearly (8 rows): the swizzle is applied to the per-lane SOURCE address.
__device__ __forceinline__ int swz(int r, int c) { return c ^ ((r >> 1) & 7); }

// 16 B per lane global -> LDS (wave-uniform LDS base + 16 lane).  The gfx950 builtins sit in
// __device__ helpers so that the host pass still emits the kernels' launch stubs.
__device__ __forceinline__ void glds16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (lds_void*)lds_base, 16, 0, 0);
}
template <int AUX>  // cache-policy bits (16: sc1)
__device__ __forceinline__ void glds16a(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (lds_void*)lds_base, 16, 0, AUX);
}
__device__ __forceinline__ int wave_uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// buffer loads / stores of one element (voffset per lane, soffset wave-uniform)
template <typename T>
struct BufIO;
template <>
struct BufIO<double> {
  typedef decltype(__builtin_amdgcn_raw_buffer_load_b64(__amdgpu_buffer_rsrc_t(), 0, 0, 0)) raw_t;
  static __device__ __forceinline__ double load(__amdgpu_buffer_rsrc_t rs, int vo, int so) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, vo, so, 0));
  }
  static __device__ __forceinline__ void store(__amdgpu_buffer_rsrc_t rs, int vo, int so, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(raw_t, v), rs, vo, so, 0);
  }
  // write-through (sc1): stores another XCD reads inside the same launch (chain_kernel)
  static __device__ __forceinline__ void store_sc1(__amdgpu_buffer_rsrc_t rs, int vo, int so, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(raw_t, v), rs, vo, so, 16);
  }
  // chain_kernel's C reads (kLdAux: sc1 in the GPK_CHAIN_SC1LD A/B builds)
  static __device__ __forceinline__ double load_ch(__amdgpu_buffer_rsrc_t rs, int vo, int so) { return ld8_buf(rs, vo, so); }
};
template <>
struct BufIO<float> {
  static __device__ __forceinline__ float load(__amdgpu_buffer_rsrc_t rs, int vo, int so) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, so, 0));
  }
  static __device__ __forceinline__ void store(__amdgpu_buffer_rsrc_t rs, int vo, int so, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), rs, vo, so, 0);
  }
  static __device__ __forceinline__ void store_sc1(__amdgpu_buffer_rsrc_t rs, int vo, int so, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), rs, vo, so, 16);
  }
  static __device__ __forceinline__ float load_ch(__amdgpu_buffer_rsrc_t rs, int vo, int so) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, so, kLdAux));
  }
};

// Rows [r0, r1) are zero in the panel columns [j0, j0 + kdepth): identity extra rows past the
// panel (zlo / zhi), or, in a ragged batch, member b's identity padding rows below the panel and
// its unused test rows -- and, once the panel lies in the member's padding, every row below it.
__device__ __forceinline__ bool zero_rows(const GemmArgs& a, int b, int64_t r0, int64_t r1) {
  if (r0 >= a.zlo && r1 <= a.zhi) return true;
  if (a.nb == nullptr) return false;
  const int64_t npb = (a.nb[b] + NB - 1) / NB * NB;
  const int64_t jend = a.j0 + a.kdepth;
  if (a.j0 >= npb) return r0 >= jend && r1 <= a.p;
  if (r0 >= (npb > jend ? npb : jend) && r1 <= a.n_pad) return true;
  return a.mb != nullptr && r0 >= a.n_pad + a.mb[b] && r1 <= a.y_row;
}

// One 256-thread workgroup computes a TM x TN tile: acc = A_rows(TM x K) * B_rows(TN x K)^T,
// K = the panel depth.  Waves 2 x 2, each (TM/2) x (TN/2) = MB x NBK blocks of 16 x 16.
// Staging: global_load_lds (16 B per lane, no VGPR round trip) into two LDS stages; the chunk
// kc+1 load is issued before chunk kc's fragment reads and MFMAs and retired by the barrier that
// ends chunk kc.  K is permuted identically for both operands so that one ds_read_b128 yields
// the operands of EPC consecutive MFMA k-steps: in k-step s, lane group q = lane >> 4 uses
// logical piece q + 4 (s / EPC), element s % EPC.
// C value (i, j) of member b's augmented matrix for the fused K build (m = 0 layout): kernel value +
// noise on the diagonal, identity padding, the y row (gpk_assemble.hip's classes for m = 0).  ls:
// the ARD length scales (u = x / ls, the reference kernel with l = 1) or NULL.
template <int OPK>
__device__ __forceinline__ double kbuild_value(const FastNode& fn, const double* ls, const double* X,
                                               const double* y, double noise, int64_t n, int64_t n_pad,
                                               int64_t y_row, int64_t gi, int64_t gj) {
  if (gi < n && gj < n) {
    FastNode f = fn;
    f.op = OPK;  // compile-time kernel: only its branch of fast_value_at is generated
    const int d = fn.d;
    const double* xi = X + gi * d;
    const double* xj = X + gj * d;
    double v;
    if (ls) {
      v = fast_value_at(f, [xi, ls](int k) { return xi[k] / ls[k]; }, [xj, ls](int k) { return xj[k] / ls[k]; });
    } else {
      v = fast_value_at(f, [xi](int k) { return xi[k]; }, [xj](int k) { return xj[k]; });
    }
    return gi == gj ? v + noise : v;
  }
  if (gi < n_pad && gj < n_pad) return gi == gj ? 1.0 : 0.0;
  if (gi == y_row && gj < n) return y[gj];
  return 0.0;
}

template <typename T, int MODE, int TM, int TN, int WN, int KB = 0>
__global__ __launch_bounds__(128 * WN, (WN == 4 && MODE == GEMM_UPDATE) ? 4 : 2) void gemm_kernel(GemmArgs a) {
  constexpr int EPC = 16 / (int)sizeof(T);   // elements per 16-B piece
  constexpr int GBK = ROWB / (int)sizeof(T); // K depth per stage (16 f64, 32 f32)
  constexpr int KS = GBK / 4;                // MFMA k-steps per stage
  constexpr int WM = 2;                      // waves along M (rows); WN along N (columns)
  constexpr int NW = WM * WN;                // waves per workgroup
  constexpr int MB = TM / (16 * WM), NBK = TN / (16 * WN);  // 16 x 16 blocks per wave
  constexpr int STAGE = (TM + TN) * ROWB;    // bytes per stage
  constexpr int PW = (TM + TN) / (8 * NW);   // glds wave-instructions (8 rows each) per wave
  typedef typename Mfma<T>::acc_t acc_t;
  typedef T vec_t __attribute__((ext_vector_type(EPC)));
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  const int b = blockIdx.y;
  const int64_t t = xcd_remap(blockIdx.x, gridDim.x, a.nb != nullptr ? 8 : 0);
  int64_t ti, tj;  // tile coordinates in units of TM (rows) and TN (cols)
  // tiles in row-major lower-triangle order, or banded (a.band > 0, gpk_tune("upd_band"))
  if (MODE == GEMM_UPDATE) {
    const int64_t w = a.c_hi - a.c_lo;
    const int64_t ttri = w * (w + 1) / 2;
    const int64_t B = a.band;
    if (t < ttri && B > 0) {
      // banded order: bands of B tile rows, each walked column by column, so that the tiles one XCD
      // runs at a time (consecutive ids, see xcd_remap) form ~B x B blocks sharing B A- and B
      // B-panels in its L2 (row-major: 1 A- and 64 B-panels)
      int64_t q = 0, start = 0;
      for (;;) {
        const int64_t h = (q * B + B <= w) ? B : w - q * B;
        const int64_t cnt = q * B * h + h * (h + 1) / 2;
        if (t < start + cnt) break;
        start += cnt;
        ++q;
      }
      const int64_t h = (q * B + B <= w) ? B : w - q * B;
      int64_t u = t - start;
      int64_t r, c;
      if (u < q * B * h) {
        c = u / h;
        r = q * B + u % h;
      } else {
        u -= q * B * h;
        int64_t j = 0;
        while (u >= h - j) {
          u -= h - j;
          ++j;
        }
        c = q * B + j;
        r = q * B + j + u;
      }
      ti = a.c_lo + r;
      tj = a.c_lo + c;
    } else if (t < ttri) {
      int64_t r = (int64_t)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
      while (r * (r + 1) / 2 > t) --r;
      while ((r + 1) * (r + 2) / 2 <= t) ++r;
      ti = a.c_lo + r;
      tj = a.c_lo + (t - r * (r + 1) / 2);
    } else {
      const int64_t u = t - ttri;
      ti = a.c_hi + u / w;
      tj = a.c_lo + u % w;
    }
  } else {
    ti = t;
    tj = 0;
  }
  if (a.bzn) {  // skip the band of structurally zero tiles (the grid does not enumerate it)
    if (ti >= a.bz0) ti += a.bzn;
    if (MODE == GEMM_UPDATE && tj >= a.bz0) tj += a.bzn;
  }
  T* W = reinterpret_cast<T*>(a.W) + (int64_t)b * a.w_bs;
  const int64_t R = a.row0 + ti * TM;
  // structurally zero operand rows: the product (and so the update / solve) of the tile is zero
  if (zero_rows(a, b, R, R + TM)) return;
  if (MODE == GEMM_UPDATE && zero_rows(a, b, a.row0 + tj * TN, a.row0 + tj * TN + TN)) return;
  const T* Ag = W + R * a.ld + a.j0;
  const T* Bg;
  int64_t ldb;
  if (GPK_ABLATE == 4 && MODE == GEMM_UPDATE) {
    Ag = reinterpret_cast<const T*>(a.W) + a.row0 * a.ld + a.j0;  // timing-only: L2-resident operands
    Bg = Ag + TM * a.ld;
    ldb = a.ld;
  } else if (MODE == GEMM_UPDATE) {
    Bg = W + (a.row0 + tj * TN) * a.ld + a.j0;
    ldb = a.ld;
  } else {
    Bg = reinterpret_cast<const T*>(a.Binv) + (int64_t)b * a.inv_bs;
    ldb = NB;
  }

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = wave_uniform(tid >> 6);
  const int wr = wid / WN, wc = wid % WN;

  // per-lane source of each of this wave's glds instructions: rows [0, TM) are A, [TM, TM+TN) B
  const T* src[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int g0 = (wid * PW + i) * 8;
    const int r = g0 + (lane >> 3);
    if (g0 < TM)
      src[i] = Ag + (int64_t)r * a.ld + swz(r, lane & 7) * EPC;
    else
      src[i] = Bg + (int64_t)(r - TM) * ldb + swz(r - TM, lane & 7) * EPC;
  }
#define GPK_GLDS(stage, kc)                                                                   \
  {                                                                                           \
    _Pragma("unroll") for (int i = 0; i < PW; ++i)                                            \
        glds16(src[i] + (int64_t)(kc) * GBK, smem + (stage) * STAGE + (wid * PW + i) * 1024);   \
  }

#ifndef GPK_ABLATE_C
#define GPK_ABLATE_C 0  // timing-only (wrong results): 1 = the C-first update starts from zero instead of C
#endif
#ifndef GPK_CFIRST
#define GPK_CFIRST 1  // f64 update: C loaded into the accumulators before the K loop (A negated)
#endif
  // C first: the C read overlaps the first chunk's staging instead of following the last MFMA, and the
  // epilogue is stores only (+3 % update rate at N = 8192; neutral for f32).  Every element then takes its
  // products one k-step after another onto C whatever the panel grouping, so the persistent launch's tile
  // tasks (other groupings) write the same bits -- f32 included (its A negated: exact)
  constexpr bool CFIRST = (MODE == GEMM_UPDATE) && (GPK_CFIRST || KB != 0);
  const int col = lane & 15;
  // C tile through a buffer descriptor: one 32-bit per-lane offset (VGPR) plus, for block (m, n)
  // and register r, the wave-uniform byte offset ((m 16 + r RSTEP) ld + n 16) sizeof(T) in an
  // SGPR (rows of the C/D layout: row(lane, r) = row(lane, 0) + r RSTEP) -- no 64-bit address
  // per access, which the 64 loads and stores of the epilogue would otherwise hold in VGPRs
  T* const C = (MODE == GEMM_UPDATE) ? W + R * a.ld + a.row0 + tj * TN : W + R * a.ld + a.j0;
  const uint64_t cu = reinterpret_cast<uint64_t>(C);
  const uint64_t cuu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(cu >> 32)) << 32) |
                       (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)cu);
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(cuu), 0, (int)(TM * a.ld * (int64_t)sizeof(T)), 0x00020000);
  const int cvo = (int)(((int64_t)(wr * (TM / WM) + Mfma<T>::row(lane, 0)) * a.ld + wc * (TN / WN) + col) *
                        (int64_t)sizeof(T));
  constexpr int RSTEP = sizeof(T) == 8 ? 4 : 1;
  const int ldb_s = wave_uniform((int)(a.ld * (int64_t)sizeof(T)));
#define GPK_CSOFF(m, n, r) (((m) * 16 + (r) * RSTEP) * ldb_s + (n) * 16 * (int)sizeof(T))

  acc_t acc[MB][NBK];
  // fused K build: the first chunk's DMA goes out before the evaluation (which no longer touches the
  // staging LDS) and lands while the lanes evaluate their entries
  if (KB != 0) GPK_GLDS(0, 0);
  if (KB != 0) {
    // fused K build: evaluate this tile's C instead of loading it (the values gpk_assemble would
    // have written; the tile's points are read straight from X, cached in L1 / L2)
    const double* hyp = a.hyp + (int64_t)b * a.hyp_stride;
    const double* Xb = a.X + (int64_t)b * a.x_bs;
    const double* yb = a.y + (int64_t)b * a.y_bs;
    const double noise = a.noise[(int64_t)b * a.noise_stride];
    gpk_node nd;  // register copy (taking the kernel argument's address would put it on the stack)
    nd.op = a.node.op;
    nd.hyp_offset = a.node.hyp_offset;
    nd.ard_slot = a.node.ard_slot;
    nd.flags = a.node.flags;
    const FastNode fn = make_fast_node(nd, hyp, a.d);
    const double* ls = (nd.flags & GPK_NODE_ARD) ? hyp + nd.hyp_offset : nullptr;
    const int64_t nn = a.n, npad = a.n_pad, yrow = a.y_row;
    // every lane evaluates its own accumulator entries (C/D layout: row wr (TM / WM) + 16 m + RSTEP r +
    // row(lane, 0), column wc (TN / WN) + 16 n + col), so each wave evaluates its own eighth of the tile
    // with no LDS round trip and no barrier; the points of a 16-row block's four rows are loaded together.
    // (The earlier form staged two half tiles through LDS, one element per iteration of a rolled loop:
    // ~16 us per tile, 3.3 ms of a 64 x 2 metric step.)
    const int64_t ci = R + wr * (TM / WM) + Mfma<T>::row(lane, 0);
    const int64_t cj = a.row0 + tj * TN + wc * (TN / WN) + col;
    const int64_t cj_tile = a.row0 + tj * TN;
    if (a.d == 1 && ls == nullptr && R + TM <= nn && cj_tile + TN <= nn && R != cj_tile) {
      // interior off-diagonal tile of a one-dimensional kernel (the metric's case): every entry is the
      // kernel value of two training points -- no class branches; the lane's 16 row points and 2
      // column points are loaded together up front.  The same fast_value_at as kbuild_value: same bits.
      FastNode f = fn;
      f.op = KB;
      double xr[MB][4], xc[NBK];
#pragma unroll
      for (int m = 0; m < MB; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) xr[m][r] = Xb[ci + m * 16 + r * RSTEP];
#pragma unroll
      for (int n = 0; n < NBK; ++n) xc[n] = Xb[cj + n * 16];
#pragma unroll
      for (int m = 0; m < MB; ++m)
#pragma unroll
        for (int n = 0; n < NBK; ++n)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const double u = xr[m][r], v = xc[n];
            acc[m][n][r] = (T)fast_value_at(f, [u](int) { return u; }, [v](int) { return v; });
          }
    } else {
#pragma unroll
      for (int m = 0; m < MB; ++m)
#pragma unroll
        for (int n = 0; n < NBK; ++n)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            acc[m][n][r] = (T)kbuild_value<KB>(fn, ls, Xb, yb, noise, nn, npad, yrow, ci + m * 16 + r * RSTEP,
                                               cj + n * 16);
    }
  } else {
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
      for (int n = 0; n < NBK; ++n) {
        if (CFIRST && GPK_ABLATE_C == 0) {
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[m][n][r] = BufIO<T>::load(crs, cvo, GPK_CSOFF(m, n, r));
        } else {
          acc[m][n] = acc_t{0, 0, 0, 0};
        }
      }
  }

  const int q = lane >> 4, lr = lane & 15;
  const int aoff = (wr * (TM / WM) + lr) * ROWB;
  const int boff = (TM + wc * (TN / WN) + lr) * ROWB;
  const int p0 = swz(lr, q) * 16, p1 = swz(lr, q + 4) * 16;

  const int NK0 = (MODE == GEMM_TRSM) ? NB / GBK : a.kdepth / GBK;
  const int NK = (GPK_ABLATE == 3 && MODE == GEMM_UPDATE) ? 2 * NK0 : NK0;
  if (KB == 0) GPK_GLDS(0, 0);
#ifndef GPK_SETPRIO
#define GPK_SETPRIO 0  // 1: static priority 1 for the second-dispatched half of the waves (MI355X guide)
#endif
  if (GPK_SETPRIO && MODE == GEMM_UPDATE && wid >= NW / 2) __builtin_amdgcn_s_setprio(1);
  // 16-row blocks of this wave that hold a nonzero row: rows >= row_end (below the y row) are zero in
  // every panel, so in the tiles of the y row's block most MFMAs would multiply zeros; those tiles
  // take the guarded form of the chunk (wave-uniform, the other tiles are unaffected)
  const int64_t wrow0 = R + wr * (TM / WM);
  const int mact = a.row_end <= 0 ? MB
                 : (int)(a.row_end <= wrow0 ? 0 : ((a.row_end - wrow0 + 15) / 16 < MB ? (a.row_end - wrow0 + 15) / 16 : MB));
  // The K loop is instantiated per MFMA row count (MB, 1, 0 live 16-row blocks) so that each form is
  // one basic block per chunk.  Order inside a chunk: barrier, all fragment reads, the MFMAs of the
  // first half of the k-steps, THEN the next chunk's global_load_lds, then the second half.  hipcc's
  // wait insertion treats an outstanding LDS DMA as pending LDS traffic and waits lgkmcnt(0) for any
  // ds_read issued while one is in flight; with the DMA issued after the first half, the first MFMAs
  // wait only for their own two fragment reads instead of all of them (the second half's lgkmcnt(0)
  // falls on reads long completed), and the DMA still has half a chunk plus the next barrier to land.
  // sched_barrier keeps the scheduler from hoisting the DMA back above the first half.
#ifndef GPK_GLDS_MID
#define GPK_GLDS_MID 1
#endif
#ifndef GPK_GLDS_MID_F32
#define GPK_GLDS_MID_F32 0  // f32 (8 k-steps per chunk): the DMA at the top measured faster (116 vs 112 TF)
#endif
  constexpr bool GMID = sizeof(T) == 8 ? GPK_GLDS_MID : GPK_GLDS_MID_F32;
#define GPK_MFMA_STEPS(S0, S1, MLIM)                                                                     \
  _Pragma("unroll") for (int s = (S0); s < (S1); ++s)                                                    \
  _Pragma("unroll") for (int n = 0; n < NBK; ++n) {                                                      \
    /* TRSM against the lower-triangular inverse: K chunk kc feeds output columns >= kc GBK only */      \
    if (MODE == GEMM_TRSM && kc * GBK > wc * (TN / WN) + n * 16 + 15) continue;                          \
    _Pragma("unroll") for (int m = 0; m < (MLIM); ++m)                                                   \
      acc[m][n] = CFIRST ? Mfma<T>::op_neg(fa[m][s / EPC][s % EPC], fb[n][s / EPC][s % EPC], acc[m][n])   \
                         : Mfma<T>::op(fa[m][s / EPC][s % EPC], fb[n][s / EPC][s % EPC], acc[m][n]);     \
  }
#define GPK_KLOOP(MLIM)                                                                                  \
  for (int kc = 0; kc < NK; ++kc) {                                                                      \
    const int st = kc & 1;                                                                               \
    /* one barrier per chunk, at the top: it retires the chunk kc glds (vmcnt(0)) and frees stage       \
       st ^ 1, read during chunk kc - 1.  The vmcnt(0) is explicit: hipcc's wait insertion does not     \
       always see the LDS write of global_load_lds across the loop back edge. */                       \
    if (GPK_ABLATE != 5) {                                                                               \
      __builtin_amdgcn_s_waitcnt(0x0F70); /* gfx9 encoding: vmcnt(0), expcnt(7), lgkmcnt(15) */        \
      __syncthreads();                                                                                   \
    }                                                                                                    \
    if (!GMID && kc + 1 < NK) GPK_GLDS(st ^ 1, (kc + 1) % NK0);                                  \
    if ((MLIM) > 0) {                                                                                    \
      const char* sb = smem + st * STAGE;                                                                \
      vec_t fa[MB][2], fb[NBK][2];                                                                       \
      /* first-half pieces (k-steps 0 .. KS/2-1) of every fragment first, A0 and B0 leading */          \
      _Pragma("unroll") for (int h = 0; h < 2; ++h) {                                                    \
        fa[0][h] = *reinterpret_cast<const vec_t*>(sb + aoff + (h ? p1 : p0));                           \
        _Pragma("unroll") for (int n = 0; n < NBK; ++n)                                                  \
          fb[n][h] = *reinterpret_cast<const vec_t*>(sb + boff + n * 16 * ROWB + (h ? p1 : p0));         \
        _Pragma("unroll") for (int m = 1; m < (MLIM); ++m)                                               \
          fa[m][h] = *reinterpret_cast<const vec_t*>(sb + aoff + m * 16 * ROWB + (h ? p1 : p0));         \
      }                                                                                                  \
      GPK_MFMA_STEPS(0, KS / 2, MLIM)                                                                    \
      if (GMID) {                                                                                        \
        __builtin_amdgcn_sched_barrier(0);                                                               \
        if (kc + 1 < NK) GPK_GLDS(st ^ 1, (kc + 1) % NK0);                                               \
        __builtin_amdgcn_sched_barrier(0);                                                               \
      }                                                                                                  \
      GPK_MFMA_STEPS(KS / 2, KS, MLIM)                                                                   \
    } else if (GMID && kc + 1 < NK) {                                                                    \
      GPK_GLDS(st ^ 1, (kc + 1) % NK0);                                                                  \
    }                                                                                                    \
  }
  if (mact > 1) {
    GPK_KLOOP(MB)
  } else if (mact == 1) {
    GPK_KLOOP(1)
  } else {
    GPK_KLOOP(0)
  }
#undef GPK_KLOOP
#undef GPK_MFMA_STEPS
#undef GPK_GLDS

  if (GPK_ABLATE == 2 && acc[0][0][0] != (T)12345.678) return;
  if (MODE == GEMM_UPDATE && GPK_ABLATE != 1 && !CFIRST) {
    // every C value is loaded before the first store: interleaved load/store pairs may alias,
    // so hipcc would wait for each load in turn (64 dependent HBM round trips per tile)
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
      for (int n = 0; n < NBK; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[m][n][r] = BufIO<T>::load(crs, cvo, GPK_CSOFF(m, n, r)) - acc[m][n][r];
  }
#pragma unroll
  for (int m = 0; m < MB; ++m)
#pragma unroll
    for (int n = 0; n < NBK; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) BufIO<T>::store(crs, cvo, GPK_CSOFF(m, n, r), acc[m][n][r]);
#undef GPK_CSOFF
}

// ================================================================================ read-out
template <typename T>
__global__ __launch_bounds__(256) void finalize_kernel(FinArgs a) {
  __shared__ double red[256];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const T* W = reinterpret_cast<const T*>(a.W) + (int64_t)b * a.w_bs;
  double s = 0.0;
  for (int64_t i = tid; i < a.n; i += 256) s += log((double)W[i * a.ld + i]);
  red[tid] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w) red[tid] += red[tid + w];
    __syncthreads();
  }
  if (tid == 0) {
    const double logdet = 2.0 * red[0];                          // Metrics.py:153-154
    const double fit = -(double)W[a.y_row * a.ld + a.y_row];     // y^T alpha = z^T z
    const double log2pi = log(2.0 * 3.141592653589793);
    const double nm = (double)(a.nb ? a.nb[b] : a.n);             // padding rows add log 1 = 0
    const double ll = (-0.5 * fit + -0.5 * logdet) + (-0.5 * (nm * log2pi));  // LogLikelihood.py:39-49
    double nl = -ll;
    if (a.info[b] != 0) nl = INFINITY;
    a.out[b * 4 + 0] = nl;
    a.out[b * 4 + 1] = fit;
    a.out[b * 4 + 2] = logdet;
    a.out[b * 4 + 3] = nm;
  }
  // posterior read-out from the Schur complement corner
  for (int64_t t = tid; t < a.m; t += 256) {
    if (a.mu) a.mu[(int64_t)b * a.m + t] = -(double)W[a.y_row * a.ld + a.n_pad + t];
    if (a.var) a.var[(int64_t)b * a.m + t] = (double)W[(a.n_pad + t) * a.ld + a.n_pad + t];
  }
}

// ================================================================================ triangular solve
// trans = 0 (x <- L^-1 x): block k: x_k <- Linv_kk x_k, then rows below: x_i -= L[i, blk k] x_k
// trans = 1 (x <- L^-T x): block k (descending): x_k <- Linv_kk^T x_k, then x_j -= sum_i L[i, j] x_i
template <typename T>
__global__ __launch_bounds__(NB) void trsv_diag_kernel(TrsvArgs a) {
  __shared__ double xs[NB];
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  double* x = a.x + (int64_t)b * a.x_bs + a.kblk * NB;
  const T* Li = reinterpret_cast<const T*>(a.Winv) + (int64_t)b * a.inv_bs + a.kblk * NB * NB;
  xs[t] = x[t];
  __syncthreads();
  double s = 0.0;
  if (a.trans == 0) {
    for (int k = 0; k <= t; ++k) s = fma((double)Li[t * NB + k], xs[k], s);
  } else {
    for (int k = t; k < NB; ++k) s = fma((double)Li[k * NB + t], xs[k], s);
  }
  x[t] = s;
}

template <typename T>
__global__ __launch_bounds__(256) void trsv_update_kernel(TrsvArgs a) {
  __shared__ double xk[NB];
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  double* x = a.x + (int64_t)b * a.x_bs;
  const T* W = reinterpret_cast<const T*>(a.W) + (int64_t)b * a.w_bs;
  const int64_t j0 = a.kblk * NB;
  if (tid < NB) xk[tid] = x[j0 + tid];
  __syncthreads();
  if (a.trans == 0) {
    const int64_t i = j0 + NB + (int64_t)blockIdx.x * 256 + tid;
    if (i >= a.n_valid) return;  // rows past a caller L's n: padding, x stays 0 there
    const T* row = W + i * a.ld + j0;
    const int kn = (int)((a.n_valid - j0) < NB ? (a.n_valid - j0) : NB);
    double s = 0.0;
    for (int k = 0; k < kn; ++k) s = fma((double)row[k], xk[k], s);
    x[i] -= s;
  } else {
    const int64_t j = (int64_t)blockIdx.x * 256 + tid;
    if (j >= j0) return;
    const int kn = (int)((a.n_valid - j0) < NB ? (a.n_valid - j0) : NB);
    double s = 0.0;
    for (int k = 0; k < kn; ++k) s = fma((double)W[(j0 + k) * a.ld + j], xk[k], s);
    x[j] -= s;
  }
}


// ================================================================================ matrix-vector
// y <- alpha A x + beta y, A row-major fp64 [n, m] (ld).  HBM-bound (8 n m bytes): one wave per
// row, lanes stride the row with 16-B loads (two fp64 each), wave reduction by shuffles.  Used by
// the iterative / explicit-inverse numerical handlings (linear_cg, inv(K) y) of the metrics.
__global__ __launch_bounds__(256) void gemv_kernel(const double* __restrict__ A, int64_t n, int64_t m, int64_t lda,
                                                   const double* __restrict__ x, double* __restrict__ y,
                                                   double alpha, double beta) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const double* a = A + row * lda;
  double s0 = 0.0, s1 = 0.0;
  const bool vec = ((lda & 1) == 0) && ((reinterpret_cast<uintptr_t>(A) & 15) == 0) &&
                   ((reinterpret_cast<uintptr_t>(x) & 15) == 0);
  int64_t j = 0;
  if (vec) {
    typedef double dbl2 __attribute__((ext_vector_type(2)));
    for (; j + 2 * 64 <= m; j += 2 * 64) {
      const dbl2 av = *reinterpret_cast<const dbl2*>(a + j + 2 * lane);
      const dbl2 xv = *reinterpret_cast<const dbl2*>(x + j + 2 * lane);
      s0 = fma(av.x, xv.x, s0);
      s1 = fma(av.y, xv.y, s1);
    }
  }
  for (int64_t k = j + lane; k < m; k += 64) s0 = fma(a[k], x[k], s0);
  double sum = s0 + s1;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
  if (lane == 0) y[row] = alpha * sum + (beta == 0.0 ? 0.0 : beta * y[row]);
}

template <typename T, int MODE, int TM, int TN, int WN = 2, int KB = 0>
hipError_t launch_gemm_t(const GemmArgs& a, int32_t batch, hipStream_t s) {
  // a.nt / c_lo / c_hi are in units of this launch's tile sizes
  unsigned nblk;
  if (MODE == GEMM_UPDATE) {
    const int64_t w = a.c_hi - a.c_lo;
    nblk = (unsigned)(w * (w + 1) / 2 + (int64_t)(a.nt - a.c_hi) * w);
  } else {
    nblk = (unsigned)a.nt;
  }
  if (nblk == 0) return hipSuccess;
  hipLaunchKernelGGL((gemm_kernel<T, MODE, TM, TN, WN, KB>), dim3(nblk, batch), dim3(128 * WN), 0, s, a);
  return hipGetLastError();
}


// ================================================================================ persistent factorisation
// chain_kernel: the whole blocked factorisation of ONE augmented matrix (f64) in one launch.  Its
// workgroups (one per CU: the diagonal-block task needs the 150 KB of LDS) claim tasks from a list in
// the order the host computed by list-scheduling the task graph (a topological order, so every task
// waits only for tasks claimed before it: the launch finishes whatever the residency), wait for their
// inputs on per-task counters, and publish their outputs with write-through stores.  Tasks (block =
// 128 rows / columns, slice = 32 rows, panel k = block column k):
//   D(k)          diagonal block k, the diag2 body (factor + inverse) on the block as the earlier tasks
//                 left it; L_kk^-1 to Winv (its lower tiles), hflag[k] once its first half_step block rows are
//                 out, dflag[k] at the end; L_kk to W after the hand-off (no task of the launch reads it)
//   S(k, r)       slice r below block k: X = A(r, k) L_kk^-T, in place; sdone[k][r].  It stages its slice once
//                 the slice's last update is in; on the diagonal chain (r in block k + 1) its first column
//                 blocks start on hflag[k], the others on dflag[k]
//   U32(q, r, j)  slice r of block column j = q + 1: C -= X(r, q) X(j, q)^T; ucnt[r][j] = q + 1
//   UQ(q, r, j, c) the same on the 32-column quarter c only, for the slices r of diagonal block j (round 4);
//                 qdone[q][r] += 1 -- D(j) waits for all of them
//   BLK(q, i, j)  128 x 128 tile (i, j), j >= q + 2: C -= X(i, q..) X(j, q..)^T over g panels q .. q + g - 1
//                 (g = 1 for the columns the diagonal chain needs soon, g = the planner's group for the deferred
//                 ones: the launch path's deep group update); ucnt[r][j] = q + g for the slices r of block i
// Every task polls all its input counters together (chain_wait_set: one round trip per poll).
// The chain D(k) -> S(k, block k + 1) -> UQ(k, block k + 1, k + 1) -> D(k + 1) runs on slices spread
// over CUs (a 128-row panel solve or update on one CU would take ~14 us of f64 MFMA), the BLK tiles of
// older panels fill the rest of the chip -- the look-ahead that launches cannot give a single
// evaluation (persistent factorisation).  Hand-offs (MI355X guide, inter-workgroup
// visibility): every byte of W / Winv that a task writes is stored sc1 (write-through) and, after every
// storing wave's vmcnt(0) and a barrier, one lane sets the counter; D, S and U32 read W / Winv with
// plain loads behind one agent acquire per task.  Every wait is bounded: on timeout
// the task sets ctl[1] and info = -1 and every workgroup drains the list without work.
enum { CH_D = 0, CH_S = 1, CH_U32 = 2, CH_BLK = 3 };
#ifndef GPK_CHAIN_DEFER_L
#define GPK_CHAIN_DEFER_L 1  // D publishes L_kk^-1 first and stores L_kk (read by no task of the launch) afterwards
#endif
#ifndef GPK_CHAIN_SHALF
#define GPK_CHAIN_SHALF 1  // the diagonal chain's S tasks start their first column blocks on D's early flag
#endif

#ifndef GPK_CHAIN_SPREF
#define GPK_CHAIN_SPREF 1  // S stages its slice before waiting for D (0: one wait for both inputs)
#endif
constexpr int CHAIN_SLOT_OFF = (int)((DIAG_LDS_BYTES + 15) / 16 * 16);
constexpr size_t CHAIN_LDS_BYTES = CHAIN_SLOT_OFF + 16;

__device__ __forceinline__ bool chain_wait(const ChainArgs& a, const int32_t* p, int32_t v, uint64_t t0) {
  return chain_wait_v(p, v, a.ctl, a.info, a.nmem, a.timeout, a.force_abort, t0);
}
// the wait of a panel solve's second column half (waves 4..7) for the whole of L_kk^-1
struct HalfWait {
  const int32_t* full;  // NULL: no split (the whole panel solve already waited)
  int32_t* ctl;
  int32_t* info;
  int nmem;
  int64_t timeout;
  int force_abort;
  int split;  // the first column block that waits for all of L^-1 (rows of the early flag / 16)
};

// wave 0: wait until *p[i] >= v[i] for every i -- the N counters polled together (all loads in flight at once,
// one round trip per poll: a task's inputs are usually all published by the time it looks, and polling them one
// after another cost a cross-XCD round trip each); false on timeout (reported) or after another task's timeout
template <int N>
__device__ __forceinline__ bool chain_wait_set(const ChainArgs& a, const int32_t* const (&p)[N], const int32_t (&v)[N],
                                               uint64_t t0) {
  for (;;) {
    int32_t x[N];
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] = ld_flag(p[i]);
    bool all = !a.force_abort;
#pragma unroll
    for (int i = 0; i < N; ++i) all = all && __builtin_amdgcn_readfirstlane(x[i]) >= v[i];
    if (all) return true;
    if (__builtin_amdgcn_readfirstlane(ld_flag(a.ctl + 1)) != 0) return false;
    if (a.force_abort || __builtin_amdgcn_s_memrealtime() - t0 > (uint64_t)a.timeout) {
      chain_report_timeout(a.ctl, a.info, a.nmem);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// C[32 x 128] = A[32 x 128] B^T (SUB false) or C -= A B^T (SUB true), B [128 x 128]; A, C with row
// stride ld, B with ldb.  These tasks are bound by the bytes one CU pulls from the Infinity Cache, so every
// operand byte is fetched once: A (32 rows, 32 KB) is staged into LDS by LDS-DMA (row stride 1040 B: the
// quarter-wave's 16 rows land on distinct bank groups), and each wave owns one column block (16 columns,
// both 16-row blocks), loading its 16 rows of B straight into registers.  In k-step pair j = 0..15 lane group q
// takes the 16-B piece k = 8 j + 2 q (+0, +1), so the four lane groups of a row read one 64-B line.  Pieces
// that contribute nothing -- the upper triangle of L^-1 (S: column block cb needs k <= 16 cb + 15) or a
// column block right of the diagonal (U32, diag_off >= 0: rows diag_off .. +31 of the block whose columns C
// covers) -- are loaded out of the buffer's range (zeros, no memory traffic).  C may alias A (the panel
// solve, in place): A is in LDS behind the barrier before any store.  Plain loads behind the task's
// acquire, sc1 stores.  (The first form -- 2 x 4 waves of 16 x 32, A and B loaded per wave from HBM / L2 --
// moved 384 KB per task: 16 us against 11-12 us for the same work with the zero pieces skipped.)
constexpr int SLAB_LDS_ROW = 1040;
// A rows 4 w .. 4 w + 3 into LDS, one 1-KB row per instruction (the slab's first operand)
__device__ __forceinline__ void slab_stage_a(const double* A, int64_t ld, char* smem) {
  const int tid = opaque_tid();
  const int lane = tid & 63;
  const int w = wave_uniform(tid >> 6);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 4 * w + i;
    glds16a<kLdAux>(A + (int64_t)row * ld + 2 * lane, smem + row * SLAB_LDS_ROW);
  }
}
// KEEP (the SQ task): the result also replaces the staged A rows in LDS (C/D layout -> row-major rows of
// SLAB_LDS_ROW bytes), behind a barrier that lets every wave finish reading A first
template <bool SUB, bool STAGED = false, bool HALF = false, bool KEEP = false>
__device__ __forceinline__ void slab_gemm(const double* A, const double* B, int64_t ldb, double* C, int64_t ld,
                                          int diag_off, uint64_t* st, char* smem, HalfWait hw = HalfWait{}) {
  typedef double dbl2 __attribute__((ext_vector_type(2)));
  const int tid = opaque_tid();
  const int lane = tid & 63;
  const int w = wave_uniform(tid >> 6);
  const int lr = lane & 15, q = lane >> 4;
  // column block of wave w: waves w and w + 4 share a SIMD, so pair the blocks (0, 7), (1, 6), (2, 5),
  // (3, 4) -- S's work per block grows with the block index (the triangle of L^-1)
  const int cb = w < 4 ? w : 11 - w;
  // live row blocks of this wave's column block (U32 on the diagonal block: columns <= the rows' block)
  const bool live0 = diag_off < 0 || cb <= (diag_off >> 4), live1 = diag_off < 0 || cb <= (diag_off >> 4) + 1;
  // (STAGED: the caller issued them already -- the panel solve prefetches its slice before L^-1 is ready)
  if (!STAGED) slab_stage_a(A, ld, smem);
  const __amdgpu_buffer_rsrc_t brs = uniform_rsrc(B), crs = uniform_rsrc(C);
  const int bvo = (int)(((int64_t)(cb * 16 + lr) * ldb + 2 * q) * 8);
  const int cvo = (int)(((int64_t)q * ld + cb * 16 + lr) * 8);  // C/D layout: row q + 4 i, column lr
  const int ldc4 = __builtin_amdgcn_readfirstlane((int)(4 * ld * 8)), ldc16 = __builtin_amdgcn_readfirstlane((int)(16 * ld * 8));
  const int jm = SUB ? (live1 ? 15 : -1) : 2 * cb + 1;
  d4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
  if (SUB) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc0[i] = ld8_buf(crs, cvo, i * ldc4);
      acc1[i] = ld8_buf(crs, cvo, ldc16 + i * ldc4);
    }
  }
  // HALF (S, its slice already in LDS behind the caller's barrier): column blocks below GPK_CHAIN_SHALF_ROWS / 16
  // need only the rows of L^-1 that D publishes before its last steps, and go at once; the others wait for all of it
  if (HALF && cb >= hw.split) {
    if (chain_wait_v(hw.full, 1, hw.ctl, hw.info, hw.nmem, hw.timeout, hw.force_abort,
                     __builtin_amdgcn_s_memrealtime()) && !kChainSc1Ld) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
  }
  dbl2 bv[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) bv[j] = ld16_buf(brs, j <= jm ? bvo + j * 64 : kRsrcBytes, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the LDS-DMA writes are not tracked by hipcc)
  if (!HALF) __syncthreads();
  if (st && w == 0) st[4] = __builtin_amdgcn_s_memrealtime();  // (profiling: operands in place)
  const char* a0 = smem + lr * SLAB_LDS_ROW + q * 16;
  const char* a1 = a0 + 16 * SLAB_LDS_ROW;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    if (j <= jm) {  // (wave-uniform; a break here left bv dynamically indexed, i.e. in scratch)
      const dbl2 x0 = *reinterpret_cast<const dbl2*>(a0 + j * 64);
      const dbl2 x1 = *reinterpret_cast<const dbl2*>(a1 + j * 64);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x0[e], bv[j][e], acc0, 0, 0, SUB ? 1 : 0);
        acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x1[e], bv[j][e], acc1, 0, 0, SUB ? 1 : 0);
      }
    }
  }
  if (st && w == 0) {  // (profiling: wave 0's MFMAs retired -- the readfirstlane waits for the last one)
    const int dep = __builtin_amdgcn_readfirstlane((int)acc0[3] + (int)acc1[3]);
    st[5] = __builtin_amdgcn_s_memrealtime() + (dep == 0x7fffffff ? 1 : 0);
  }
  double* Cr = C + (int64_t)q * ld + cb * 16 + lr;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (live0) sts<true>(Cr + 4 * i * ld, acc0[i]);
    if (live1) sts<true>(Cr + (16 + 4 * i) * ld, acc1[i]);
  }
  if (KEEP) {
    wg_sync<true>();  // (every wave's A reads done; the global stores stay in flight)
    double* xr = reinterpret_cast<double*>(smem + q * SLAB_LDS_ROW) + cb * 16 + lr;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      *reinterpret_cast<double*>(reinterpret_cast<char*>(xr) + 4 * i * SLAB_LDS_ROW) = acc0[i];
      *reinterpret_cast<double*>(reinterpret_cast<char*>(xr) + (16 + 4 * i) * SLAB_LDS_ROW) = acc1[i];
    }
  }
}

// UQ: the 32 x 32 quarter q of slice r in the next diagonal block, C -= A B^T with A = X(r) [32 x 128] and
// B = X(slice q of that block) [32 x 128] (K = 128, panel k): one 16 x 16 block per wave for waves 0..3 (wave w:
// rows 16 (w & 1), columns 16 (w >> 1)), the A rows staged in LDS by all 8 waves as in slab_gemm, the wave's B
// rows straight to registers.  Every accumulator runs slab_gemm's k-steps in its order (the same bits as the
// per-slice U32 and the launch path); on the diagonal quarter the block right of the diagonal is skipped.
// 64 KB of operands per task instead of U32's 160 KB: the update that gates the next diagonal block.
__device__ __forceinline__ void slab_q(const double* A, const double* B, int64_t ld, double* C, bool diag, uint64_t* st,
                                       char* smem) {
  typedef double dbl2 __attribute__((ext_vector_type(2)));
  const int tid = opaque_tid();
  const int lane = tid & 63;
  const int w = wave_uniform(tid >> 6);
  const int lr = lane & 15, q = lane >> 4;
  const int rb = w & 1, cbl = (w >> 1) & 1;
  const bool active = w < 4 && (!diag || cbl <= rb);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 4 * w + i;
    glds16a<kLdAux>(A + (int64_t)row * ld + 2 * lane, smem + row * SLAB_LDS_ROW);
  }
  const __amdgpu_buffer_rsrc_t brs = uniform_rsrc(B), crs = uniform_rsrc(C);
  const int bvo = (int)(((int64_t)(cbl * 16 + lr) * ld + 2 * q) * 8);
  const int cvo = (int)(((int64_t)(rb * 16 + q) * ld + cbl * 16 + lr) * 8);  // C/D layout: row q + 4 i, column lr
  const int ldc4 = __builtin_amdgcn_readfirstlane((int)(4 * ld * 8));
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  if (active) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = ld8_buf(crs, cvo, i * ldc4);
  }
  dbl2 bv[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) bv[j] = ld16_buf(brs, active ? bvo + j * 64 : kRsrcBytes, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the LDS-DMA writes are not tracked by hipcc)
  __syncthreads();
  if (st && w == 0) st[4] = __builtin_amdgcn_s_memrealtime();  // (profiling: operands in place)
  if (active) {
    const char* a0 = smem + (rb * 16 + lr) * SLAB_LDS_ROW + q * 16;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const dbl2 x = *reinterpret_cast<const dbl2*>(a0 + j * 64);
#pragma unroll
      for (int e = 0; e < 2; ++e) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x[e], bv[j][e], acc, 0, 0, 1);
    }
  }
  if (st && w == 0) {
    const int dep = __builtin_amdgcn_readfirstlane((int)acc[3]);
    st[5] = __builtin_amdgcn_s_memrealtime() + (dep == 0x7fffffff ? 1 : 0);
  }
  if (active) {
    double* Cr = C + (int64_t)(rb * 16 + q) * ld + cbl * 16 + lr;
#pragma unroll
    for (int i = 0; i < 4; ++i) sts<true>(Cr + 4 * i * ld, acc[i]);
  }
}

// SQ (chain_uq = 2), second half: slice r = 4 (k + 1) + rl of the next diagonal block, its panel-k rows X(r) in
// LDS rows 0..31 (slab_gemm KEEP), applies panel k to its lower quarters of that block,
//   C(r, q) -= X(r) X(4 (k + 1) + q)^T,  q = 0 .. rl   (32 x 32 x 128 each, on the diagonal one the lower half),
// the siblings' rows X(4 (k + 1) + q), q < rl, published by the SQ tasks claimed before this one, staged by LDS-DMA
// into LDS rows 32 (q + 1) ..  Every 16 x 16 accumulator runs slab_q's k-steps in its order (the same bits as the
// quarter tasks UQ, the per-slice U32 and the launch path).  The 4 rl + 3 live 16 x 16 blocks are dealt to the 8
// waves (block b to wave b % 8).  sib_ok: the siblings' rows were published (false after a timeout: no work).
__device__ __forceinline__ void sq_quarters(double* W, int64_t ld, int k, int r, int rl, bool sib_ok, char* smem) {
  typedef double dbl2 __attribute__((ext_vector_type(2)));
  const int tid = opaque_tid();
  const int lane = tid & 63;
  const int w = wave_uniform(tid >> 6);
  const int lr = lane & 15, lq = lane >> 4;
  if (sib_ok) {
    // siblings: 32 rows each, 4 rows per wave (1 KB per instruction)
    for (int q = 0; q < rl; ++q) {
      const double* X = W + (int64_t)(32 * (4 * (k + 1) + q)) * ld + (int64_t)k * NB;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = 4 * w + i;
        glds16a<kLdAux>(X + (int64_t)row * ld + 2 * lane, smem + (32 * (q + 1) + row) * SLAB_LDS_ROW);
      }
    }
  }
  const int nblk16 = 4 * rl + 3;
  double* const Cq = W + (int64_t)(32 * r) * ld + (int64_t)(k + 1) * NB;
  const __amdgpu_buffer_rsrc_t crs = uniform_rsrc(Cq);
  const int ldc4 = __builtin_amdgcn_readfirstlane((int)(4 * ld * 8));
  d4 acc[2];
  int qq[2], rb[2], cbl[2];
  bool act[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int b = w + 8 * u;
    act[u] = sib_ok && b < nblk16;
    // block b: quarter b / 4, position b % 4 = (rb, cbl) in (0,0), (1,0), (0,1), (1,1); the diagonal quarter
    // (q = rl) has the three blocks (0,0), (1,0), (1,1)
    const int q = b < 4 * rl ? b / 4 : rl;
    const int pos = b < 4 * rl ? b % 4 : (b - 4 * rl == 2 ? 3 : b - 4 * rl);
    qq[u] = q;
    rb[u] = pos & 1;
    cbl[u] = pos >> 1;
    const int cvo = (int)(((int64_t)(rb[u] * 16 + lq) * ld + 32 * q + cbl[u] * 16 + lr) * 8);
    acc[u] = d4{0.0, 0.0, 0.0, 0.0};
    if (act[u]) {
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[u][i] = ld8_buf(crs, cvo, i * ldc4);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the LDS-DMA writes are not tracked by hipcc)
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (act[u]) {
      const char* a0 = smem + (rb[u] * 16 + lr) * SLAB_LDS_ROW + lq * 16;
      const int brow = (qq[u] == rl ? 0 : 32 * (qq[u] + 1)) + cbl[u] * 16 + lr;
      const char* b0 = smem + brow * SLAB_LDS_ROW + lq * 16;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const dbl2 x = *reinterpret_cast<const dbl2*>(a0 + j * 64);
        const dbl2 y = *reinterpret_cast<const dbl2*>(b0 + j * 64);
#pragma unroll
        for (int e = 0; e < 2; ++e) acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(x[e], y[e], acc[u], 0, 0, 1);
      }
      double* Cr = Cq + (int64_t)(rb[u] * 16 + lq) * ld + 32 * qq[u] + cbl[u] * 16 + lr;
#pragma unroll
      for (int i = 0; i < 4; ++i) sts<true>(Cr + 4 * i * ld, acc[u][i]);
    }
  }
}

// ---------------------------------------------------------------------------- f32 slab tasks (chain_kernel<float>)
// The f32 forms of S and U32 (slab_gemm): the 32 x 128 slice staged in LDS, wave w on column block cb (the f64
// pairing), the B rows straight to registers, f32 MFMA (v_mfma_f32_16x16x4_f32).  LDS image: row r of the slice
// in LDS row r & 15 of SLAB_LDS_ROW bytes, at byte 512 (r >> 4) -- rows 0..15 in the first half, 16..31 in the
// second, the f64 row stride (16 rows of one operand read on distinct 16-B bank slots); one DMA wave-instruction
// per LDS row (lanes 0..31 row r, 32..63 row r + 16).  k-steps: 16-B pieces, k = 16 j + 4 q + e for lane group
// q = lane >> 4, piece j = 0..7, element e -- gemm_kernel<float>'s order (chunk kc = j / 2, step 4 (j & 1) + e),
// so X and the updated C are the launch path's bits (U32 C first, as its update).
__device__ __forceinline__ void slab_stage_a32(const float* A, int64_t ld, char* smem) {
  const int tid = opaque_tid();
  const int lane = tid & 63;
  const int w = wave_uniform(tid >> 6);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int lrow = 2 * w + i;
    glds16a<kLdAux>(A + (int64_t)(lrow + 16 * (lane >> 5)) * ld + 4 * (lane & 31), smem + lrow * SLAB_LDS_ROW);
  }
}
__device__ __forceinline__ float ld4_buf(__amdgpu_buffer_rsrc_t rs, int vo, int so) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, so, kLdAux));
}
template <bool SUB, bool STAGED = false, bool HALF = false>
__device__ __forceinline__ void slab_gemm32(const float* A, const float* B, int64_t ldb, float* C, int64_t ld,
                                            int diag_off, uint64_t* st, char* smem, HalfWait hw = HalfWait{}) {
  typedef float flt4 __attribute__((ext_vector_type(4)));
  const int tid = opaque_tid();
  const int lane = tid & 63;
  const int w = wave_uniform(tid >> 6);
  const int lr = lane & 15, q = lane >> 4;
  const int cb = w < 4 ? w : 11 - w;
  const bool live0 = diag_off < 0 || cb <= (diag_off >> 4), live1 = diag_off < 0 || cb <= (diag_off >> 4) + 1;
  if (!STAGED) slab_stage_a32(A, ld, smem);
  const __amdgpu_buffer_rsrc_t brs = uniform_rsrc(B), crs = uniform_rsrc(C);
  const int bvo = (int)(((int64_t)(cb * 16 + lr) * ldb + 4 * q) * 4);
  const int cvo = (int)(((int64_t)(4 * q) * ld + cb * 16 + lr) * 4);  // f32 C/D layout: row 4 q + i, column lr
  const int ldc1 = __builtin_amdgcn_readfirstlane((int)(ld * 4)), ldc16 = __builtin_amdgcn_readfirstlane((int)(16 * ld * 4));
  // pieces j <= jm: L^-1's lower triangle (S: k < 16 (cb + 1); its upper tiles are never written), all (U32)
  const int jm = SUB ? (live1 ? 7 : -1) : cb;
  f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  if (SUB) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc0[i] = ld4_buf(crs, cvo, i * ldc1);
      acc1[i] = ld4_buf(crs, cvo, ldc16 + i * ldc1);
    }
  }
  if (HALF && cb >= hw.split) {
    if (chain_wait_v(hw.full, 1, hw.ctl, hw.info, hw.nmem, hw.timeout, hw.force_abort,
                     __builtin_amdgcn_s_memrealtime()) && !kChainSc1Ld) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
  }
  flt4 bv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
    bv[j] = __builtin_bit_cast(flt4, __builtin_amdgcn_raw_buffer_load_b128(brs, j <= jm ? bvo + j * 64 : kRsrcBytes, 0, kLdAux));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the LDS-DMA writes are not tracked by hipcc)
  if (!HALF) __syncthreads();
  if (st && w == 0) st[4] = __builtin_amdgcn_s_memrealtime();
  const char* a0 = smem + lr * SLAB_LDS_ROW + q * 16;
  const char* a1 = a0 + 512;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (j <= jm) {
      const flt4 x0 = *reinterpret_cast<const flt4*>(a0 + j * 64);
      const flt4 x1 = *reinterpret_cast<const flt4*>(a1 + j * 64);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(SUB ? -x0[e] : x0[e], bv[j][e], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(SUB ? -x1[e] : x1[e], bv[j][e], acc1, 0, 0, 0);
      }
    }
  }
  if (st && w == 0) {
    const int dep = __builtin_amdgcn_readfirstlane((int)acc0[3] + (int)acc1[3]);
    st[5] = __builtin_amdgcn_s_memrealtime() + (dep == 0x7fffffff ? 1 : 0);
  }
  float* Cr = C + (int64_t)(4 * q) * ld + cb * 16 + lr;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (live0) sts<true>(Cr + i * ld, acc0[i]);
    if (live1) sts<true>(Cr + (16 + i) * ld, acc1[i]);
  }
}

// BLK: C(R.., Cc..) -= A(R.., Kc..) B(Cc.., Kc..)^T on a 128 x 128 tile, K = 128 g: gemm_kernel's update
// (8 waves of 64 x 32, LDS-DMA staging of 128-B row chunks -- 16 f64 / 32 f32 deep -- in two stages, C first,
// the next chunk's DMA after the first half of the MFMAs) with write-through C stores.  Rows >= row_end are
// zero.  Every element takes gemm_kernel's k-steps in its order, C first (both dtypes): the launch path's bits.
#ifndef GPK_CH_GMID_F32
#define GPK_CH_GMID_F32 0
#endif
template <typename T>
__device__ __forceinline__ void blk_tile(T* W, int64_t ld, int64_t R, int64_t Cc, int64_t Kc, int g,
                                         int64_t row_end, char* smem) {
  constexpr int TM = 128, TN = 128, WN = 4, WM = 2, NW = 8, MB = 4, NBK = 2;
  constexpr int EPC = 16 / (int)sizeof(T), GBK = ROWB / (int)sizeof(T), KS = GBK / 4;
  constexpr int RSTEP = sizeof(T) == 8 ? 4 : 1;  // C/D rows of one accumulator's registers
  // the next chunk's DMA after the first half of the MFMAs (f64) or at the top of the chunk (f32, gemm_kernel's
  // GPK_GLDS_MID_F32: 8 k-steps per chunk)
  constexpr bool GMID = sizeof(T) == 8 || GPK_CH_GMID_F32 != 0;
  constexpr int STAGE = (TM + TN) * ROWB;
  constexpr int PW = (TM + TN) / (8 * NW);
  const int NK = wave_uniform(g * (NB / GBK));  // depth 128 g: the g panels Kc / 128 .. + g - 1
  typedef T vec_t __attribute__((ext_vector_type(EPC)));
  typedef typename Mfma<T>::acc_t acc_t;
  const int tid = opaque_tid();
  const int lane = tid & 63;
  const int wid = wave_uniform(tid >> 6);
  const int wr = wid / WN, wc = wid % WN;
  const T* Ag = W + R * ld + Kc;
  const T* Bg = W + Cc * ld + Kc;
  const T* src[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int g0 = (wid * PW + i) * 8;
    const int r = g0 + (lane >> 3);
    src[i] = (g0 < TM) ? Ag + (int64_t)r * ld + swz(r, lane & 7) * EPC
                       : Bg + (int64_t)(r - TM) * ld + swz(r - TM, lane & 7) * EPC;
  }
  T* const C = W + R * ld + Cc;
  const uint64_t cu = reinterpret_cast<uint64_t>(C);
  const uint64_t cuu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(cu >> 32)) << 32) |
                       (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)cu);
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(cuu), 0, (int)(TM * ld * (int64_t)sizeof(T)), 0x00020000);
  const int col = lane & 15;
  const int cvo = (int)(((int64_t)(wr * (TM / WM) + Mfma<T>::row(lane, 0)) * ld + wc * (TN / WN) + col) *
                        (int64_t)sizeof(T));
  const int ldb_s = wave_uniform((int)(ld * (int64_t)sizeof(T)));
#define GPK_CH_CSOFF(m, n, r) (((m) * 16 + (r) * RSTEP) * ldb_s + (n) * 16 * (int)sizeof(T))
  acc_t acc[MB][NBK];
#pragma unroll
  for (int m = 0; m < MB; ++m)
#pragma unroll
    for (int n = 0; n < NBK; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[m][n][r] = BufIO<T>::load_ch(crs, cvo, GPK_CH_CSOFF(m, n, r));
  const int q = lane >> 4, lr = lane & 15;
  const int aoff = (wr * (TM / WM) + lr) * ROWB;
  const int boff = (TM + wc * (TN / WN) + lr) * ROWB;
  const int p0 = swz(lr, q) * 16, p1 = swz(lr, q + 4) * 16;
#define GPK_CH_GLDS(stage, kc)                                                                   \
  {                                                                                              \
    _Pragma("unroll") for (int i = 0; i < PW; ++i)                                               \
        glds16a<kLdAux>(src[i] + (int64_t)(kc) * GBK, smem + (stage) * STAGE + (wid * PW + i) * 1024); \
  }
  GPK_CH_GLDS(0, 0);
  const int64_t wrow0 = R + wr * (TM / WM);
  const int mact = row_end <= wrow0 ? 0 : ((row_end - wrow0 + 15) / 16 < MB ? (int)((row_end - wrow0 + 15) / 16) : MB);
#define GPK_CH_STEPS(S0, S1, MLIM)                                                                 \
  _Pragma("unroll") for (int s = (S0); s < (S1); ++s)                                              \
  _Pragma("unroll") for (int n = 0; n < NBK; ++n)                                                  \
  _Pragma("unroll") for (int m = 0; m < (MLIM); ++m)                                               \
    acc[m][n] = Mfma<T>::op_neg(fa[m][s / EPC][s % EPC], fb[n][s / EPC][s % EPC], acc[m][n]);
#define GPK_CH_KLOOP(MLIM)                                                                         \
  for (int kc = 0; kc < NK; ++kc) {                                                                \
    const int st = kc & 1;                                                                         \
    __builtin_amdgcn_s_waitcnt(0x0F70);                                                            \
    __syncthreads();                                                                               \
    if (!GMID && kc + 1 < NK) GPK_CH_GLDS(st ^ 1, kc + 1);                                         \
    if ((MLIM) > 0) {                                                                              \
      const char* sb = smem + st * STAGE;                                                          \
      vec_t fa[MB][2], fb[NBK][2];                                                                 \
      _Pragma("unroll") for (int h = 0; h < 2; ++h) {                                              \
        fa[0][h] = *reinterpret_cast<const vec_t*>(sb + aoff + (h ? p1 : p0));                     \
        _Pragma("unroll") for (int n = 0; n < NBK; ++n)                                            \
          fb[n][h] = *reinterpret_cast<const vec_t*>(sb + boff + n * 16 * ROWB + (h ? p1 : p0));   \
        _Pragma("unroll") for (int m = 1; m < (MLIM); ++m)                                         \
          fa[m][h] = *reinterpret_cast<const vec_t*>(sb + aoff + m * 16 * ROWB + (h ? p1 : p0));   \
      }                                                                                            \
      GPK_CH_STEPS(0, KS / 2, MLIM)                                                                \
      if (GMID) {                                                                                  \
        __builtin_amdgcn_sched_barrier(0);                                                         \
        if (kc + 1 < NK) GPK_CH_GLDS(st ^ 1, kc + 1);                                              \
        __builtin_amdgcn_sched_barrier(0);                                                         \
      }                                                                                            \
      GPK_CH_STEPS(KS / 2, KS, MLIM)                                                               \
    } else if (GMID && kc + 1 < NK) {                                                              \
      GPK_CH_GLDS(st ^ 1, kc + 1);                                                                 \
    }                                                                                              \
  }
  if (mact > 1) {
    GPK_CH_KLOOP(MB)
  } else if (mact == 1) {
    GPK_CH_KLOOP(1)
  } else {
    GPK_CH_KLOOP(0)
  }
#undef GPK_CH_KLOOP
#undef GPK_CH_STEPS
#undef GPK_CH_GLDS
  // (through a scalar-typed parameter: __builtin_bit_cast of the vector element acc[m][n][r] itself
  // compiled to four stores of element 0)
#pragma unroll
  for (int m = 0; m < MB; ++m)
#pragma unroll
    for (int n = 0; n < NBK; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) BufIO<T>::store_sc1(crs, cvo, GPK_CH_CSOFF(m, n, r), acc[m][n][r]);
#undef GPK_CH_CSOFF
}

#ifndef GPK_CHAIN_NOINLINE
#define GPK_CHAIN_FN __device__ __forceinline__
#else
#define GPK_CHAIN_FN __device__ __noinline__
#endif
// The task bodies are separate (not inlined) functions: each gets its own register allocation, so the
// diagonal-block body's 250 VGPRs do not force the others -- or the claim loop -- to spill.  They take
// plain values, never the kernel argument by reference: its address taken, the kernel copies ChainArgs to
// per-lane scratch and every field read becomes a VGPR load -- divergent for the compiler, which then
// turned the claim loop's exit into an exec-mask-controlled loop whose barriers the waves no longer
// executed the same number of times (the deadlock of the first versions).
template <typename T>
GPK_CHAIN_FN void chain_d(T* W, int64_t ld, T* Winv, int32_t* info, int dbg, int k, uint64_t* dprof,
                          int32_t* half_flag, int half_step, double* sm) {
  DiagArgs da{};
  da.W = W;
  da.ld = ld;
  da.Winv = Winv;
  da.j0 = (int64_t)k * NB;
  da.kblk = k;
  da.info = info;
  da.version = 2;
  da.dbg = dbg;  // (GPK_CHAIN_DBG: diag2_body's timing ablations -- wrong results)
  da.prof = dprof;
  da.no_inv_zeros = 1;  // (S reads only the lower 16-tiles of L^-1: slab_gemm's skipped pieces; gpk_trsv likewise)
  da.defer_l_store = GPK_CHAIN_DEFER_L;
  da.half_flag = half_flag;
  da.half_step = half_step;
  diag2_body<T, false, true>(da, 0, sm);
}
GPK_CHAIN_FN void chain_s(double* W, int64_t ld, const double* Winv, int k, int r, uint64_t* st, char* smem) {
  double* X = W + (int64_t)r * 32 * ld + (int64_t)k * NB;
  slab_gemm<false>(X, Winv + (int64_t)k * NB * NB, NB, X, ld, -1, st, smem);
}
GPK_CHAIN_FN void chain_s_staged(double* W, int64_t ld, const double* Winv, int k, int r, uint64_t* st, char* smem) {
  double* X = W + (int64_t)r * 32 * ld + (int64_t)k * NB;
  slab_gemm<false, true>(X, Winv + (int64_t)k * NB * NB, NB, X, ld, -1, st, smem);
}
GPK_CHAIN_FN void chain_s_half(double* W, int64_t ld, const double* Winv, int k, int r, uint64_t* st, char* smem,
                               HalfWait hw) {
  double* X = W + (int64_t)r * 32 * ld + (int64_t)k * NB;
  slab_gemm<false, true, true>(X, Winv + (int64_t)k * NB * NB, NB, X, ld, -1, st, smem, hw);
}
// SQ: the diagonal chain's panel solve S(k, r) of slice r = 4 (k + 1) + rl, whose rows stay in LDS, then -- after
// publishing sdone[k][r] (sd_k = sdone + k nsl) and waiting for its siblings' -- its lower quarters of block k + 1
// (sq_quarters).  hw.full etc.: the panel solve's wait for all of L_kk^-1; slot: an LDS word for the siblings' ok.
GPK_CHAIN_FN void chain_sq(double* W, int64_t ld, const double* Winv, int k, int r, uint64_t* st, char* smem,
                           HalfWait hw, int32_t* sd_k, int32_t* slot) {
  double* X = W + (int64_t)r * 32 * ld + (int64_t)k * NB;
  slab_gemm<false, true, true, true>(X, Winv + (int64_t)k * NB * NB, NB, X, ld, -1, st, smem, hw);
  const int rl = r - 4 * (k + 1);
  const int wave = wave_uniform(opaque_tid() >> 6);
  // publish the rows (every storing wave drains its stores first), then wait for the siblings' rows
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (wave == 0) {
    st_flag(sd_k + r, 1);
    bool ok = true;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int q = 0; q < rl && ok; ++q)
      ok = chain_wait_v(sd_k + 4 * (k + 1) + q, 1, hw.ctl, hw.info, hw.nmem, hw.timeout, hw.force_abort, t0);
    if (ok && !kChainSc1Ld && rl > 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    slot[2] = ok ? 1 : 0;
  }
  __syncthreads();
  sq_quarters(W, ld, k, r, rl, __builtin_amdgcn_readfirstlane(slot[2]) != 0, smem);
}
GPK_CHAIN_FN void chain_s_stage(double* W, int64_t ld, int k, int r, char* smem) {
  slab_stage_a(W + (int64_t)r * 32 * ld + (int64_t)k * NB, ld, smem);
}
GPK_CHAIN_FN void chain_uq(double* W, int64_t ld, int k, int r, int j, int qq, uint64_t* st, char* smem) {
  const int64_t R = (int64_t)r * 32;
  const int64_t J = (int64_t)j * NB;
  const int64_t Bq = J + 32 * qq;  // rows of slice qq of block j = its quarter qq of columns
  slab_q(W + R * ld + (int64_t)k * NB, W + Bq * ld + (int64_t)k * NB, ld, W + R * ld + Bq, R == Bq, st, smem);
}
GPK_CHAIN_FN void chain_u32(double* W, int64_t ld, int q, int r, int j, uint64_t* st, char* smem) {
  const int64_t R = (int64_t)r * 32;
  const int64_t J = (int64_t)j * NB;
  slab_gemm<true>(W + R * ld + (int64_t)q * NB, W + J * ld + (int64_t)q * NB, ld, W + R * ld + J, ld,
                  (R >= J && R < J + NB) ? (int)(R - J) : -1, st, smem);
}

// f32 forms (chain_kernel<float>: no SQ / UQ tasks -- its plans take one U32 per slice, chain_knobs)
GPK_CHAIN_FN void chain_s32(float* W, int64_t ld, const float* Winv, int k, int r, uint64_t* st, char* smem) {
  float* X = W + (int64_t)r * 32 * ld + (int64_t)k * NB;
  slab_gemm32<false>(X, Winv + (int64_t)k * NB * NB, NB, X, ld, -1, st, smem);
}
GPK_CHAIN_FN void chain_s32_staged(float* W, int64_t ld, const float* Winv, int k, int r, uint64_t* st, char* smem) {
  float* X = W + (int64_t)r * 32 * ld + (int64_t)k * NB;
  slab_gemm32<false, true>(X, Winv + (int64_t)k * NB * NB, NB, X, ld, -1, st, smem);
}
GPK_CHAIN_FN void chain_s32_half(float* W, int64_t ld, const float* Winv, int k, int r, uint64_t* st, char* smem,
                                 HalfWait hw) {
  float* X = W + (int64_t)r * 32 * ld + (int64_t)k * NB;
  slab_gemm32<false, true, true>(X, Winv + (int64_t)k * NB * NB, NB, X, ld, -1, st, smem, hw);
}
GPK_CHAIN_FN void chain_s32_stage(float* W, int64_t ld, int k, int r, char* smem) {
  slab_stage_a32(W + (int64_t)r * 32 * ld + (int64_t)k * NB, ld, smem);
}
GPK_CHAIN_FN void chain_u32_f32(float* W, int64_t ld, int q, int r, int j, uint64_t* st, char* smem) {
  const int64_t R = (int64_t)r * 32;
  const int64_t J = (int64_t)j * NB;
  slab_gemm32<true>(W + R * ld + (int64_t)q * NB, W + J * ld + (int64_t)q * NB, ld, W + R * ld + J, ld,
                    (R >= J && R < J + NB) ? (int)(R - J) : -1, st, smem);
}

__device__ __forceinline__ void chain_trace(const ChainArgs& a, int slot, int v) {
  if (a.trace) __hip_atomic_store(a.trace + 32 * blockIdx.x + slot, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One atomic add by lane 0 of the wave, without a lane-divergent branch: the claim loop below keeps every
// branch wave-uniform.  (With "if (tid == 0) claim" the loop's exit became exec-mask controlled: wave 0
// then ran the next iteration's barrier once with lane 0 masked off and once for lane 0 -- one barrier
// more than the other waves -- and the workgroup deadlocked after its first task.)
__device__ __forceinline__ int claim_ticket(int32_t* p) {
  int v;
  uint64_t saved;
  const int one = 1;
  asm volatile(
      "s_mov_b64 %1, exec\n\t"
      "s_mov_b64 exec, 1\n\t"
      "s_nop 1\n\t"
      "global_atomic_add %0, %2, %3, off sc0\n\t"
      "s_waitcnt vmcnt(0)\n\t"
      "s_mov_b64 exec, %1\n\t"
      "s_nop 1"
      : "=&v"(v), "=&s"(saved)
      : "v"(p), "v"(one)
      : "memory");
  return __builtin_amdgcn_readfirstlane(v);
}

// Wave 0 (all its lanes poll the same words: no lane-divergent branch) waits until the task's inputs are
// published; false on timeout (reported) or after another task's timeout.  kprev: the count the previous
// update of the task's cells published (k, or 0 when there is none: the task word's first bit)
__device__ __forceinline__ bool chain_deps(const ChainArgs& a, int ty, int kprev, int k, int r, int j, int g,
                                           int64_t co) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const int32_t* dflag = a.dflag + co;
  const int32_t* sdone = a.sdone + co;
  const int32_t* ucnt = a.ucnt + co;
  // (slots a task does not need keep the first pointer with value 0: always met, loaded in the same batch)
  if (ty == CH_D) {
    if (k == 0) return true;
    const int32_t* p[4];
    int32_t v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int s = 4 * k + i;
      if (a.uq) {
        // every quarter update of panel k - 1 on the block's slices (slice s has s - 4 k + 1 of them; uq 2: one
        // SQ task per slice sets 1 once all of its quarters are stored)
        p[i] = a.qdone + co + (int64_t)(k - 1) * a.nsl + (s < a.nsl ? s : 4 * k);
        v[i] = s < a.nsl ? (a.uq == 2 ? 1 : i + 1) : 0;
      } else {
        p[i] = ucnt + (int64_t)s * a.nbc + k;
        v[i] = k;
      }
    }
    return chain_wait_set<4>(a, p, v, t0);
  } else if (ty == CH_S) {
    // (g > 1, chain_s128: slices r .. r + g - 1 of one block row; unused slots repeat the first, always met)
    const int32_t* p[5] = {dflag + k, dflag + k, dflag + k, dflag + k, dflag + k};
    int32_t v[5] = {1, 1, 1, 1, 1};
    for (int i = 0; i < g; ++i) {
      p[1 + i] = ucnt + (int64_t)(r + i) * a.nbc + k;
      v[1 + i] = kprev;
    }
    return chain_wait_set<5>(a, p, v, t0);
  } else if (ty == CH_U32) {
    const int32_t* sd = sdone + (int64_t)k * a.nsl;
    const int32_t* p[6];
    int32_t v[6];
    p[0] = sd + r;
    v[0] = 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int s = 4 * j + i;
      // g > 1: UQ, quarter g - 2 -- slice 4 j + quarter of the panel only
      const bool need = g > 1 ? (i == g - 2) : (s < a.nsl);
      p[1 + i] = need ? sd + s : sd + r;
      v[1 + i] = need ? 1 : 0;
    }
    p[5] = ucnt + (int64_t)r * a.nbc + j;
    v[5] = kprev;
    return chain_wait_set<6>(a, p, v, t0);
  }
  // BLK over the g panels k .. k + g - 1: the last panel's solves of both blocks' slices (S(q, r) done implies
  // S(q', r) done for q' < q: S(q, r) waited for the update of panel q - 1, which waited for S(q - 1, r)), and the
  // tile's previous update
  const int32_t* sd = sdone + (int64_t)(k + g - 1) * a.nsl;
  const int32_t* p[12];
  int32_t v[12];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int sr = 4 * r + i, sj = 4 * j + i;
    p[i] = sd + (sr < a.nsl ? sr : 4 * r);
    v[i] = sr < a.nsl ? 1 : 0;
    p[4 + i] = sd + (sj < a.nsl ? sj : 4 * j);
    v[4 + i] = sj < a.nsl ? 1 : 0;
    p[8 + i] = ucnt + (int64_t)(sr < a.nsl ? sr : 4 * r) * a.nbc + j;
    v[8 + i] = sr < a.nsl ? kprev : 0;
  }
  return chain_wait_set<12>(a, p, v, t0);
}

// XCD of the executing workgroup (HW_REG_XCC_ID, bits 3:0)
__device__ __forceinline__ int xcc_id() { return (int)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 0xf); }

template <typename T>
__global__ __launch_bounds__(DT) void chain_kernel(ChainArgs a) {
  constexpr bool F64 = sizeof(T) == 8;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  int32_t* slot = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(sm) + CHAIN_SLOT_OFF);
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int total = a.ntasks + a.ntasks_b;
  // Two lists (chain_xcd, a.xcd_b >= 0): up to b_seats workgroups of XCD xcd_b claim list B (the diagonal chain:
  // its hand-offs and operands stay in one L2) and everyone else list A; a workgroup whose own list is exhausted
  // claims from the other.  Both lists are subsequences of one topological order, and a workgroup holds a task of
  // its own list until that list is exhausted, so with at least one workgroup of each role the earliest claimed,
  // unfinished task only ever waits for finished tasks (tests/test_chain_plan.py simulates it).  One list
  // (ntasks_b = 0): list A, then an empty list B.
  int lst = 0;
  if (wave == 0) {
    if (a.xcd_b >= 0 && xcc_id() == a.xcd_b && claim_ticket(a.ctl + 3) < a.b_seats) lst = 1;
    slot[3] = lst;
  }
  __syncthreads();
  lst = __builtin_amdgcn_readfirstlane(slot[3]);
  bool switched = false;
  // every branch of this loop is wave-uniform (wave; the task fields through readfirstlane)
  for (;;) {
    if (wave == 0) {
      int g = total;
      for (;;) {
        const int n = lst ? a.ntasks_b : a.ntasks;
        const int t = claim_ticket(a.ctl + (lst ? 2 : 0));
        if (t < n) {
          g = lst ? a.ntasks + t : t;
          break;
        }
        if (switched) break;  // (both lists exhausted)
        switched = true;
        lst ^= 1;
      }
      if (g < total && __builtin_amdgcn_readfirstlane(ld_flag(a.ctl + 1)) != 0) g = total;  // timed out
      slot[0] = g;
      chain_trace(a, 0, g);
    }
    __syncthreads();
    const int t = __builtin_amdgcn_readfirstlane(slot[0]);
    if (t >= total) break;
    const int tyg = __builtin_amdgcn_readfirstlane(a.tasks[4 * t]);
    // BLK: updates over g panels; U32 with g > 1: the quarter g - 2 task (UQ); first: the cells the task
    // updates have no earlier update (identity-augmented lists: their counter waits are for 0); member
    const int ty = tyg & 3, g = ((tyg >> 2) & 15) + 1, first = (tyg >> 6) & 1, mem = tyg >> 8;
    const bool sq = ty == CH_S && ((tyg >> 7) & 1);  // (chain_uq 2: S + the next block's quarters, chain_sq)
    T* const Wm = reinterpret_cast<T*>(a.W) + (int64_t)mem * a.w_bs;
    T* const Wi = reinterpret_cast<T*>(a.Winv) + (int64_t)mem * a.inv_bs;
    const int64_t co = (int64_t)mem * a.ctl_stride;
    const int k = __builtin_amdgcn_readfirstlane(a.tasks[4 * t + 1]);
    const int r = __builtin_amdgcn_readfirstlane(a.tasks[4 * t + 2]);
    const int j = __builtin_amdgcn_readfirstlane(a.tasks[4 * t + 3]);
    // S (GPK_CHAIN_SPREF): its slice of the panel is final once the slice's last update is published, before
    // L_kk^-1 is: wait for that first, start the slice's LDS-DMA, then wait for D(k) -- the slice's load leaves
    // the critical chain D(k) -> S
    const bool spref = GPK_CHAIN_SPREF && ty == CH_S && g == 1;
    const bool shalf = GPK_CHAIN_SHALF && spref && (r >> 2) == k + 1;  // (the S tasks on the diagonal chain)
    if (wave == 0) {
      if (a.times) a.times[6 * t] = __builtin_amdgcn_s_memrealtime();
      bool ok;
      if (sq && k > 0) {
        // SQ: the slice's panel-k columns and its quarters' block column k + 1, both updated through panel k - 1
        const int32_t* p[2] = {a.ucnt + co + (int64_t)r * a.nbc + k, a.ucnt + co + (int64_t)r * a.nbc + k + 1};
        const int32_t v[2] = {k, k};
        ok = chain_wait_set<2>(a, p, v, __builtin_amdgcn_s_memrealtime());
      } else {
        ok = spref ? (k == 0 || first || chain_wait(a, a.ucnt + co + (int64_t)r * a.nbc + k, k,
                                                    __builtin_amdgcn_s_memrealtime()))
                   : chain_deps(a, ty, first ? 0 : k, k, r, j, g, co);
      }
      if (a.times) {
        a.times[6 * t + 1] = __builtin_amdgcn_s_memrealtime();
        if (ty == CH_D || ty == CH_BLK) a.times[6 * t + 4] = __builtin_amdgcn_s_memtime();  // shader clock
      }
      if (ok && !kChainSc1Ld) {
        // the task reads W / Winv with plain loads (BLK: LDS-DMA / buffer loads): one agent acquire
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      slot[1] = ok ? 1 : 0;
      chain_trace(a, 1, ok ? 2 : -2);
    }
    __syncthreads();
    if (!__builtin_amdgcn_readfirstlane(slot[1])) continue;
    if (spref) {
      if constexpr (F64)
        chain_s_stage(Wm, a.ld, k, r, reinterpret_cast<char*>(sm));
      else
        chain_s32_stage(Wm, a.ld, k, r, reinterpret_cast<char*>(sm));
      if (wave == 0) {
        // (GPK_CHAIN_SHALF: rows 0..63 of L_kk^-1 suffice for the first column half; the rest waits in the body)
        const bool ok = chain_wait(a, (shalf ? a.hflag : a.dflag) + co + k, 1, __builtin_amdgcn_s_memrealtime());
        if (a.times) a.times[6 * t + 1] = __builtin_amdgcn_s_memrealtime();
        if (ok && !kChainSc1Ld) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        slot[1] = ok ? 1 : 0;
      }
      // every wave's own slice rows have landed before the barrier: the panel solve reads all 32 rows from LDS,
      // and its HALF form has no barrier of its own after the operand loads (each wave drains only its own DMA)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (!__builtin_amdgcn_readfirstlane(slot[1])) continue;
    }
    if (ty == CH_D) {
      chain_d<T>(Wm, a.ld, Wi, a.info + mem, a.dbg, k, a.dprof, GPK_CHAIN_SHALF ? a.hflag + co + k : nullptr,
                 a.half_step, sm);
    } else if constexpr (F64) {
      if (sq) {
        chain_sq(Wm, a.ld, Wi, k, r, a.times ? a.times + 6 * t : nullptr, reinterpret_cast<char*>(sm),
                 HalfWait{a.dflag + co + k, a.ctl, a.info, a.nmem, a.timeout, a.force_abort,
                          GPK_CHAIN_SHALF ? a.half_step : 0},
                 a.sdone + co + (int64_t)k * a.nsl, slot);
      } else if (shalf) {
        chain_s_half(Wm, a.ld, Wi, k, r, a.times ? a.times + 6 * t : nullptr, reinterpret_cast<char*>(sm),
                     HalfWait{a.dflag + co + k, a.ctl, a.info, a.nmem, a.timeout, a.force_abort, a.half_step});
      } else if (spref) {
        chain_s_staged(Wm, a.ld, Wi, k, r, a.times ? a.times + 6 * t : nullptr, reinterpret_cast<char*>(sm));
      } else if (ty == CH_S) {
        for (int i = 0; i < g; ++i) {  // (g > 1: a block row's slices, chain_s128)
          if (i > 0) wg_sync<true>();  // (every wave done reading the previous slice's rows in LDS)
          chain_s(Wm, a.ld, Wi, k, r + i, a.times ? a.times + 6 * t : nullptr, reinterpret_cast<char*>(sm));
        }
      } else if (ty == CH_U32 && g > 1) {
        chain_uq(Wm, a.ld, k, r, j, g - 2, a.times ? a.times + 6 * t : nullptr, reinterpret_cast<char*>(sm));
      } else if (ty == CH_U32) {
        chain_u32(Wm, a.ld, k, r, j, a.times ? a.times + 6 * t : nullptr, reinterpret_cast<char*>(sm));
      } else {
        blk_tile<double>(Wm, a.ld, (int64_t)r * NB, (int64_t)j * NB, (int64_t)k * NB, g, a.row_end,
                         reinterpret_cast<char*>(sm));
      }
    } else {
      // (f32 plans hold no SQ / UQ tasks)
      if (shalf) {
        chain_s32_half(Wm, a.ld, Wi, k, r, a.times ? a.times + 6 * t : nullptr, reinterpret_cast<char*>(sm),
                       HalfWait{a.dflag + co + k, a.ctl, a.info, a.nmem, a.timeout, a.force_abort, a.half_step});
      } else if (spref) {
        chain_s32_staged(Wm, a.ld, Wi, k, r, a.times ? a.times + 6 * t : nullptr, reinterpret_cast<char*>(sm));
      } else if (ty == CH_S) {
        for (int i = 0; i < g; ++i) {
          if (i > 0) wg_sync<true>();
          chain_s32(Wm, a.ld, Wi, k, r + i, a.times ? a.times + 6 * t : nullptr, reinterpret_cast<char*>(sm));
        }
      } else if (ty == CH_U32) {
        chain_u32_f32(Wm, a.ld, k, r, j, a.times ? a.times + 6 * t : nullptr, reinterpret_cast<char*>(sm));
      } else {
        blk_tile<float>(Wm, a.ld, (int64_t)r * NB, (int64_t)j * NB, (int64_t)k * NB, g, a.row_end,
                        reinterpret_cast<char*>(sm));
      }
    }
    if (wave == 0 && a.times) {
      a.times[6 * t + 2] = __builtin_amdgcn_s_memrealtime();  // wave 0's body done
      if (ty == CH_D || ty == CH_BLK) a.times[6 * t + 5] = __builtin_amdgcn_s_memtime();
    }
    // publish: every storing wave drains its stores, then wave 0 sets the counter
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (wave == 0) {
      chain_trace(a, 1, 4);
      if (a.times) a.times[6 * t + 3] = __builtin_amdgcn_s_memrealtime();
      if (ty == CH_D) {
        st_flag(a.dflag + co + k, 1);
      } else if (sq) {
        st_flag(a.qdone + co + (int64_t)k * a.nsl + r, 1);  // (its sdone went out before the quarters)
      } else if (ty == CH_S) {
        for (int i = 0; i < g; ++i) st_flag(a.sdone + co + (int64_t)k * a.nsl + r + i, 1);
      } else if (ty == CH_U32 && g > 1) {
        // +1 from lane 0 only (every lane of wave 0 executes this: an add of 1 would count 64; the compiler
        // reduces the lanes' values and issues one atomic)
        __hip_atomic_fetch_add((gi32*)(a.qdone + co + (int64_t)k * a.nsl + r), (threadIdx.x & 63) == 0 ? 1 : 0,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else if (ty == CH_U32) {
        st_flag(a.ucnt + co + (int64_t)r * a.nbc + j, k + 1);
      } else {
        for (int s = 4 * r; s <= 4 * r + 3 && s < a.nsl; ++s) st_flag(a.ucnt + co + (int64_t)s * a.nbc + j, k + g);
      }
    }
    if (GPK_CHAIN_DEFER_L && ty == CH_D) {
      // L_kk from LDS (the block's lower tiles; L^-1 sits in the upper ones) to W, after the hand-off: only the
      // read-out after the launch uses it.  (The next claim's barrier keeps the LDS intact until every wave has
      // read its rows.)
      T* Wb = Wm + (int64_t)k * NB * a.ld + (int64_t)k * NB;
      const int tid = opaque_tid();
#pragma unroll 1
      for (int I = 0; I < NTL; ++I) store_l_rows<T, true>(sm, Wb, a.ld, I, tid, DT);
    }
  }
  if (wave == 0) chain_trace(a, 1, 9);
}

}  // namespace

#ifndef GPK_TRSM_WN
#define GPK_TRSM_WN 2  // waves along N of the f64 128-tile TRSM (4: the update's 8-wave 64 x 32 layout)
#endif

hipError_t launch_gemm(const GemmArgs& a, int dtype, int mode, int tile, int32_t batch, hipStream_t s) {
  if (a.kbuild) {  // first trailing update with the fused K build (SE / MAT32 / MAT52 nodes)
    if (mode != GEMM_UPDATE || dtype != GPK_F64) return hipErrorInvalidValue;
    switch (a.node.op) {
      case GPK_OP_SE:
        return tile == 128 ? launch_gemm_t<double, GEMM_UPDATE, 128, 128, GPK_UPD_WN, GPK_OP_SE>(a, batch, s)
                           : launch_gemm_t<double, GEMM_UPDATE, 64, 64, 2, GPK_OP_SE>(a, batch, s);
      case GPK_OP_MAT32:
        return tile == 128 ? launch_gemm_t<double, GEMM_UPDATE, 128, 128, GPK_UPD_WN, GPK_OP_MAT32>(a, batch, s)
                           : launch_gemm_t<double, GEMM_UPDATE, 64, 64, 2, GPK_OP_MAT32>(a, batch, s);
      case GPK_OP_MAT52:
        return tile == 128 ? launch_gemm_t<double, GEMM_UPDATE, 128, 128, GPK_UPD_WN, GPK_OP_MAT52>(a, batch, s)
                           : launch_gemm_t<double, GEMM_UPDATE, 64, 64, 2, GPK_OP_MAT52>(a, batch, s);
      default:
        return hipErrorInvalidValue;
    }
  }
  if (dtype == GPK_F64) {
    if (mode == GEMM_UPDATE)
      return tile == 128 ? launch_gemm_t<double, GEMM_UPDATE, 128, 128, GPK_UPD_WN>(a, batch, s)
                         : launch_gemm_t<double, GEMM_UPDATE, 64, 64>(a, batch, s);
    return tile == 128 ? launch_gemm_t<double, GEMM_TRSM, 128, 128, GPK_TRSM_WN>(a, batch, s)
                       : launch_gemm_t<double, GEMM_TRSM, 64, 128>(a, batch, s);
  }
  if (mode == GEMM_UPDATE)
    return tile == 128 ? launch_gemm_t<float, GEMM_UPDATE, 128, 128, GPK_UPD_WN_F32>(a, batch, s)
                       : launch_gemm_t<float, GEMM_UPDATE, 64, 64>(a, batch, s);
  return tile == 128 ? launch_gemm_t<float, GEMM_TRSM, 128, 128>(a, batch, s)
                     : launch_gemm_t<float, GEMM_TRSM, 64, 128>(a, batch, s);
}

hipError_t launch_finalize(const FinArgs& a, int dtype, int32_t batch, hipStream_t s) {
  if (dtype == GPK_F64)
    hipLaunchKernelGGL(finalize_kernel<double>, dim3(batch), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(finalize_kernel<float>, dim3(batch), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_trsv_diag(const TrsvArgs& a, int dtype, int32_t batch, hipStream_t s) {
  if (dtype == GPK_F64)
    hipLaunchKernelGGL(trsv_diag_kernel<double>, dim3(batch), dim3(NB), 0, s, a);
  else
    hipLaunchKernelGGL(trsv_diag_kernel<float>, dim3(batch), dim3(NB), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_gemv(const double* A, int64_t n, int64_t m, int64_t lda, const double* x, double* y,
                       double alpha, double beta, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(gemv_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, A, n, m, lda, x, y, alpha, beta);
  return hipGetLastError();
}

hipError_t launch_trsv_update(const TrsvArgs& a, int dtype, int32_t batch, hipStream_t s) {
  const int64_t j0 = a.kblk * NB;
  const int64_t cnt = (a.trans == 0) ? (a.n_pad - j0 - NB) : j0;
  if (cnt <= 0) return hipSuccess;
  dim3 grid((unsigned)((cnt + 255) / 256), batch);
  if (dtype == GPK_F64)
    hipLaunchKernelGGL(trsv_update_kernel<double>, grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(trsv_update_kernel<float>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

__global__ __launch_bounds__(DT) void chain_d_only_kernel(ChainArgs a) {  // (debugging: GPK_CHAIN_DBG=4)
  extern __shared__ __attribute__((aligned(16))) double sm[];
  chain_d<double>(static_cast<double*>(a.W), a.ld, static_cast<double*>(a.Winv), a.info, a.dbg, 0, a.dprof, nullptr, 0,
                  sm);
}

template <typename T>
hipError_t launch_chain_t(const ChainArgs& a, int grid, hipStream_t s) {
  hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(chain_kernel<T>), CHAIN_LDS_BYTES);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(chain_kernel<T>, dim3(grid), dim3(DT), CHAIN_LDS_BYTES, s, a);
  return hipGetLastError();
}

hipError_t launch_chain(const ChainArgs& a, int dtype, int grid, hipStream_t s) {
  if (a.dbg == 4 && dtype == GPK_F64) {
    hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(chain_d_only_kernel), CHAIN_LDS_BYTES);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(chain_d_only_kernel, dim3(1), dim3(DT), CHAIN_LDS_BYTES, s, a);
    return hipGetLastError();
  }
  return dtype == GPK_F32 ? launch_chain_t<float>(a, grid, s) : launch_chain_t<double>(a, grid, s);
}

// persistent launches that timed out on the current device so far (g_chain_timeouts_dev; synchronous copy)
hipError_t chain_timeouts_read(int64_t* out) {
  unsigned long long v = 0;
  hipError_t e = hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_chain_timeouts_dev), sizeof(v), 0, hipMemcpyDeviceToHost);
  if (e == hipSuccess) *out = (int64_t)v;
  return e;
}

}  // namespace gpk
