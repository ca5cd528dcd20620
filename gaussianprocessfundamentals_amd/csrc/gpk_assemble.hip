// Kernel-matrix build (the HBM-write-bound half of the LML hot path).
//
// One 256-thread workgroup writes one 64 x 64 tile.  The tile's 64 row points and 64 column
// points (plus their per-ARD-node rescaled copies) are staged once in LDS; every lane then
// owns one column and walks 16 rows, evaluating the postfix kernel program in registers and
// storing whole 512-B rows (64 consecutive fp64 per wave instruction).  In the augmented
// layout only lower-triangular tiles are launched (the factorisation never reads the upper
// triangle), so the bytes written are p(p+64)/2 elements per batch member.
//
// Two-leaf SE + periodic trees at D = 4 / 8 (the C5 kernel) take three launches instead (launch_assemble):
// pair_feat_kernel (per-point MFMA operands and norms, once per point), pair_fast_kernel (interior tiles whose
// error bounds hold: the dot products on the f64 MFMA, a table exp in ln2 / 32 units; y-row / zero tail tiles
// written directly; every other tile appended to a device list) and the general instantiation over that list.
//
// Reference semantics (paths relative to gpbasics/):
//   SE     KernelBasics/BaseKernels.py:277-294   exp(-0.5 * (dist^2 / l^2)), sg * (..) if scaled
//   PER    KernelBasics/BaseKernels.py:440-457   exp((-2 sin^2(pi * (d1 / p))) / l^2)
//   MAT32  KernelBasics/BaseKernels.py:702-720   (1 + f) e^-f,            f = (sqrt3 d1) / |l|
//   MAT52  KernelBasics/BaseKernels.py:859-880   ((1 + f) + 5 d1^2 / (3 l^2)) e^-f,  f = (sqrt5 d1) / |l|
//   ADD/MUL KernelBasics/Operators.py:207-225, :306-326 (left fold over children)
//   d1 = L1 distance (Auxiliary/Distances.py:10-12); SE distance either the expanded norm of
//   Auxiliary/Distances.py:4-7 (GPK_NODE_SE_EXPANDED) or the direct sum of squares.
//   noise on the training diagonal only: Statistics/CovarianceMatrix.py:197-206; K_ss has none
//   (:218-225); K_s = k(X, X_test) (:277-286).
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>

#include "gpk_internal.h"
#include "gpk_kernels.h"

namespace gpk {
namespace {

#ifndef GPK_ASM_ABLATE
#define GPK_ASM_ABLATE 0  // timing-only: 1 skips the kernel evaluation (wrong results)
#endif

enum { CLS_TRAIN = 0, CLS_PAD = 1, CLS_TEST = 2, CLS_Y = 3, CLS_ZERO = 4 };

// row / column class of index g for a member with n training and m test points
__device__ __forceinline__ int classify(const AsmArgs& a, int64_t g, int64_t n, int64_t m) {
  if (g < n) return CLS_TRAIN;
  if (g < a.n_pad) return CLS_PAD;
  if (g < a.n_pad + m) return CLS_TEST;
  if (g == a.y_row) return CLS_Y;
  return CLS_ZERO;
}

// training / test points of member b (ragged batches: its own counts)
__device__ __forceinline__ int64_t member_n(const AsmArgs& a, int b) { return a.nb ? a.nb[b] : a.n; }
__device__ __forceinline__ int64_t member_m(const AsmArgs& a, int b) { return a.mb ? a.mb[b] : a.m; }

// Stage 64 points (raw + per-ARD-node rescaled copies) of one tile edge into LDS.  sc_slot > 0: also
// sin(pi f) and cos(pi f) of u = x / p (f = u - rint(u)) for the periodic node sc_node(kd) into slots
// sc_slot and sc_slot + 1, clearing *sc_flag if any |u| exceeds SC_MAX_U.
__device__ __forceinline__ void stage_points(const gpk_kdesc& kd, const AsmArgs& a, const double* hyp,
                                             double* dst, int64_t g0, int b, bool rows, int slot_stride,
                                             int sc_slot = 0, double sc_iper = 0.0, int* sc_flag = nullptr) {
  const int tid = threadIdx.x;
  for (int e = tid; e < ATILE * a.d; e += 256) {
    const int pt = e / a.d, k = e - pt * a.d;
    const int64_t g = g0 + pt;
    double v = 0.0;
    if (a.plain) {
      const int64_t lim = rows ? a.n : a.m;
      const double* src = rows ? a.X : a.Xs;
      if (g < lim) v = src[g * a.d + k];
    } else {
      const int c = classify(a, g, member_n(a, b), member_m(a, b));
      if (c == CLS_TRAIN) v = a.X[(int64_t)b * a.x_bs + g * a.d + k];
      else if (c == CLS_TEST && a.E == nullptr && !a.eye) v = a.Xs[(int64_t)b * a.xs_bs + (g - a.n_pad) * a.d + k];
    }
    dst[pt * a.dp + k] = v;
    if (sc_slot > 0) {
      const double u = v * sc_iper;
      if (!(fabs(u) <= SC_MAX_U)) atomicAnd(sc_flag, 0);
      double sv, cv;
      sincospi(u - rint(u), &sv, &cv);
      dst[sc_slot * slot_stride + pt * a.dp + k] = sv;
      dst[(sc_slot + 1) * slot_stride + pt * a.dp + k] = cv;
    }
    // ARD copies: u = x / ls (the reference kernel with l = 1 on rescaled inputs)
    for (int q = 0; q < kd.n_nodes; ++q) {
      const gpk_node nd = kd.nodes[q];
      if (nd.op != GPK_OP_ADD && nd.op != GPK_OP_MUL && (nd.flags & GPK_NODE_ARD))
        dst[(nd.ard_slot + 1) * slot_stride + pt * a.dp + k] = v / hyp[nd.hyp_offset + k];
    }
  }
}

#ifndef GPK_ASM_INTERIOR_TREE
#define GPK_ASM_INTERIOR_TREE 1  // trees of base nodes on the interior path too
#endif
#ifndef GPK_ASM_PAIR_MFMA
#define GPK_ASM_PAIR_MFMA 1  // two-leaf SE + periodic trees on f64 MFMA (pair_mfma_tile; 0: the VALU form, A/B)
#endif
#ifndef GPK_ASM_INTERIOR
#define GPK_ASM_INTERIOR 1  // 0: every tile through the generic loop (A/B)
#endif

// Interior tiles -- every row and column a training point of the member, no dense / E / identity
// rows (all but the tiles along the block edges) -- with the dimension D a compile-time constant: the
// lane's column point (and its ARD copy) is held in registers for its 16 rows, the row point is an LDS
// broadcast, and the D loops unroll; one loop per base-kernel op, the op test hoisted out of it.  Same
// formulas, operation order and contraction (gpk_kernels.h) as the generic path and the fused build,
// so every path writes the same bits.
template <typename TOut, int D>
__device__ __forceinline__ void interior_single_sc(FastNode fn, const double* prow, const double* pcol, int dp, int c,
                                                   int r0, int64_t gi0, int64_t gj, double noise, TOut* W, int64_t ld) {
  double sb[D], cb[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    sb[k] = pcol[fn.sc_sin + c * dp + k];
    cb[k] = pcol[fn.sc_cos + c * dp + k];
  }
  fn.d = D;
  for (int rr = r0; rr < ATILE; rr += 4) {
    const double* ps = prow + fn.sc_sin + rr * dp;
    const double* pc = prow + fn.sc_cos + rr * dp;
    double v = GPK_ASM_ABLATE ? 0.0
                              : per_sc_value(fn, [ps](int k) { return ps[k]; }, [pc](int k) { return pc[k]; },
                                             [&sb](int k) { return sb[k]; }, [&cb](int k) { return cb[k]; });
    const int64_t gi = gi0 + rr;
    if (gi == gj) v += noise;
    W[gi * ld + gj] = (TOut)v;
  }
}

template <typename TOut, int D, int OP>
__device__ __forceinline__ void interior_single(FastNode fn, const double* prow, const double* pcol, int dp, int c,
                                                int r0, int64_t gi0, int64_t gj, double noise, TOut* W, int64_t ld) {
  double cb[D];
#pragma unroll
  for (int k = 0; k < D; ++k) cb[k] = pcol[fn.off + c * dp + k];
  fn.op = OP;
  fn.d = D;
  for (int rr = r0; rr < ATILE; rr += 4) {
    const double* pa = prow + fn.off + rr * dp;
    double v = GPK_ASM_ABLATE ? 0.0 : fast_value_at(fn, [pa](int k) { return pa[k]; }, [&cb](int k) { return cb[k]; });
    const int64_t gi = gi0 + rr;
    if (gi == gj) v += noise;
    W[gi * ld + gj] = (TOut)v;
  }
}

// trees whose base nodes read the raw points or ONE ARD slot (slot offset off1)
template <typename TOut, int D>
__device__ __forceinline__ void interior_tree(const gpk_kdesc& kd, const FastNode* fns, const double* prow,
                                              const double* pcol, int off1, int dp, int c, int r0, int64_t gi0,
                                              int64_t gj, double noise, TOut* W, int64_t ld, int sc_sin, int sc_cos,
                                              bool sc_on) {
  double cb0[D], cb1[D], csb[D], ccb[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    cb0[k] = pcol[c * dp + k];
    cb1[k] = pcol[off1 + c * dp + k];
    csb[k] = sc_on ? pcol[sc_sin + c * dp + k] : 0.0;
    ccb[k] = sc_on ? pcol[sc_cos + c * dp + k] : 0.0;
  }
  for (int rr = r0; rr < ATILE; rr += 4) {
    Stack st;
    st.s0 = 0.0;
    int sp = 0;
    for (int q = 0; q < kd.n_nodes; ++q) {
      const int op = kd.nodes[q].op;
      if (op == GPK_OP_ADD || op == GPK_OP_MUL) {
        const double top = st.get(sp - 1);
        const double below = st.get(sp - 2);
        st.set(sp - 2, op == GPK_OP_ADD ? below + top : below * top);
        sp -= 1;
      } else {
        FastNode f = fns[q];
        f.d = D;
        if (sc_on && f.sc && f.op == GPK_OP_PER) {
          const double* ps = prow + sc_sin + rr * dp;
          const double* pc = prow + sc_cos + rr * dp;
          st.set(sp, per_sc_value(f, [ps](int k) { return ps[k]; }, [pc](int k) { return pc[k]; },
                                  [&csb](int k) { return csb[k]; }, [&ccb](int k) { return ccb[k]; }));
        } else {
          const bool s1 = f.off != 0;
          const double* pa = prow + f.off + rr * dp;
          st.set(sp, fast_value_at(f, [pa](int k) { return pa[k]; },
                                   [&cb0, &cb1, s1](int k) { return s1 ? cb1[k] : cb0[k]; }));
        }
        sp += 1;
      }
    }
    double v = st.s0;
    const int64_t gi = gi0 + rr;
    if (gi == gj) v += noise;
    W[gi * ld + gj] = (TOut)v;
  }
}

// Trees of exactly two base nodes under one ADD / MUL (postfix [leaf, leaf, op]; SURVEY C5's SE-ARD + PER):
// leaf by leaf over the lane's 16 rows -- each leaf's op is tile-uniform, so one specialised loop per leaf
// (its column point, raw / ARD slot / the periodic leaf's sin and cos, in registers) instead of the program
// loop, value stack and op dispatch per element; the 16 row values stay in registers between the leaves.
// Same leaf functions and the same combination (below op top) as eval_tree_fast: the same bits.
template <int D, int OP>
__device__ __forceinline__ void leaf_rows(FastNode f, const double* prow, const double* pcol, int dp, int c, int r0,
                                          int mode, double (&acc)[ATILE / 4]) {
  f.op = OP;  // compile-time op: only its branch of fast_value_at is generated
  f.d = D;
  double cb[D];
#pragma unroll
  for (int k = 0; k < D; ++k) cb[k] = pcol[f.off + c * dp + k];
#pragma unroll
  for (int i = 0; i < ATILE / 4; ++i) {
    const double* pa = prow + f.off + (r0 + 4 * i) * dp;
    const double v = GPK_ASM_ABLATE ? 0.0 : fast_value_at(f, [pa](int k) { return pa[k]; }, [&cb](int k) { return cb[k]; });
    acc[i] = mode == 0 ? v : (mode == 1 ? acc[i] + v : acc[i] * v);
  }
}
template <int D>
__device__ __forceinline__ void leaf_rows_sc(FastNode f, const double* prow, const double* pcol, int dp, int c, int r0,
                                             int mode, double (&acc)[ATILE / 4]) {
  f.d = D;
  double sb[D], cb[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    sb[k] = pcol[f.sc_sin + c * dp + k];
    cb[k] = pcol[f.sc_cos + c * dp + k];
  }
#pragma unroll
  for (int i = 0; i < ATILE / 4; ++i) {
    const double* ps = prow + f.sc_sin + (r0 + 4 * i) * dp;
    const double* pc = prow + f.sc_cos + (r0 + 4 * i) * dp;
    const double v = GPK_ASM_ABLATE ? 0.0
                                    : per_sc_value(f, [ps](int k) { return ps[k]; }, [pc](int k) { return pc[k]; },
                                                   [&sb](int k) { return sb[k]; }, [&cb](int k) { return cb[k]; });
    acc[i] = mode == 0 ? v : (mode == 1 ? acc[i] + v : acc[i] * v);
  }
}
template <int D>
__device__ __forceinline__ void leaf_dispatch(const FastNode& f, bool sc_on, const double* prow, const double* pcol,
                                              int dp, int c, int r0, int mode, double (&acc)[ATILE / 4]) {
  if (sc_on && f.sc && f.op == GPK_OP_PER) {
    leaf_rows_sc<D>(f, prow, pcol, dp, c, r0, mode, acc);
    return;
  }
  switch (f.op) {
    case GPK_OP_SE: leaf_rows<D, GPK_OP_SE>(f, prow, pcol, dp, c, r0, mode, acc); break;
    case GPK_OP_PER: leaf_rows<D, GPK_OP_PER>(f, prow, pcol, dp, c, r0, mode, acc); break;
    case GPK_OP_MAT32: leaf_rows<D, GPK_OP_MAT32>(f, prow, pcol, dp, c, r0, mode, acc); break;
    default: leaf_rows<D, GPK_OP_MAT52>(f, prow, pcol, dp, c, r0, mode, acc); break;
  }
}
template <typename TOut, int D>
__device__ __forceinline__ void interior_pair(const gpk_kdesc& kd, const FastNode* fns, const double* prow,
                                              const double* pcol, int dp, int c, int r0, int64_t gi0, int64_t gj,
                                              double noise, TOut* W, int64_t ld, bool sc_on) {
  double acc[ATILE / 4];
  const FastNode f0 = fns[0], f1 = fns[1];
  leaf_dispatch<D>(f0, sc_on, prow, pcol, dp, c, r0, 0, acc);
  leaf_dispatch<D>(f1, sc_on, prow, pcol, dp, c, r0, kd.nodes[2].op == GPK_OP_MUL ? 2 : 1, acc);
#pragma unroll
  for (int i = 0; i < ATILE / 4; ++i) {
    double v = acc[i];
    const int64_t gi = gi0 + r0 + 4 * i;
    if (gi == gj) v += noise;
    W[gi * ld + gj] = (TOut)v;
  }
}

// ------------------------------------------------------------------ two-leaf SE + periodic trees on f64 MFMA
// SURVEY C5's ADD(SE-ARD, PER standard): the per-dimension sums of both leaves are dot products of per-point
// features, so a tile's 64 x 64 of them are f64 MFMA tiles and only the two exps and a few FMAs per element
// stay on the VALU (the VALU form: 150 instructions per element, VALU-issue-bound at 0.94 ms for C5):
//   SE   ||u_a - u_b||^2 = |u_a|^2 + |u_b|^2 - 2 u_a . u_b                 (u: the leaf's ARD slot or raw points;
//        the reference's expanded norm, Auxiliary/Distances.py:4-7, clamped at 0 as the direct sum never goes
//        negative)
//   PER  sum_k sin^2(pi (u_ak - u_bk)) = D / 2 - 1/2 sum_k (C_ak C_bk + S_ak S_bk),  C = cos 2 pi f, S = sin 2 pi f,
//        from the staged sin(pi f), cos(pi f) (f = u - rint(u), u = x / p): C = 1 - 2 s^2, S = 2 s c
// A point's value against itself (i == j in one point set) takes distance 0 exactly (k(x, x) = sg).  Both forms
// cancel for close points: |d(r^2)| <~ 4 eps (|u_a|^2 + |u_b|^2) and |d(sn)| <~ 2 D eps, relative errors in K of
// half and 2 / l^2 times that.  A tile takes this path only where those stay <~ 1e-13 (kernel-matrix tests: rel
// 1e-12): max |u|^2 of its rows + of its columns <= 512, and D / l_per^2 <= 128, D in {4, 8, 12, 16}; other tiles
// keep the VALU form (per tile, like the sin / cos form itself; the decision is symmetric in rows and columns).
constexpr double PAIR_MFMA_MAX_NORM = 512.0;
constexpr double PAIR_MFMA_MAX_DIL2 = 128.0;

// exp(x) for x <= 0 (the kernel values' exponents): 2^(k / 32) from a 32-entry table in LDS (tab) times a degree-6
// Taylor polynomial on |r| <= ln2 / 64 (truncation <= 4e-18), k = rint(32 x / ln2), r = x - k ln2 / 32 by a two-part
// Cody-Waite reduction (k L1 exact for |k| < 2^21); x clamped at -746 (2^-1076: 0).  <= 1.5 ulp against the correctly
// rounded exp (checked in numpy over [-745, 0]); ~16 VALU operations and one conflict-free LDS read (distinct table
// entries sit on distinct bank pairs) against ~25 for the library exp with its overflow / NaN guards.  NaN input:
// never reaches it (the pair path's tile bounds reject NaN points and hyperparameters).
__device__ const double kExp2Tab32[32] = {
    1.0, 1.0218971486541166, 1.0442737824274138, 1.0671404006768237, 1.0905077326652577, 1.1143867425958924,
    1.1387886347566916, 1.1637248587775775, 1.189207115002721, 1.215247359980469, 1.241857812073484,
    1.2690509571917332, 1.2968395546510096, 1.3252366431597413, 1.3542555469368927, 1.383909881963832,
    1.4142135623730951, 1.4451808069770467, 1.4768261459394993, 1.5091644275934228, 1.5422108254079407,
    1.5759808451078865, 1.6104903319492543, 1.645755478153965, 1.681792830507429, 1.718619298122478,
    1.7562521603732995, 1.7947090750031072, 1.8340080864093424, 1.8741676341103, 1.9152065613971474,
    1.9571441241754002};
#ifndef GPK_FAST_ABLATE
#define GPK_FAST_ABLATE 0  // timing-only ablations of the fast read-out (A/B builds; wrong values)
#endif
#ifndef GPK_ASM_TAB_EXP
#define GPK_ASM_TAB_EXP 1
#endif
__device__ __forceinline__ double exp_neg(double x, const double* tab) {
#pragma clang fp contract(on)
  if (!GPK_ASM_TAB_EXP) return exp(x);
  x = fmax(x, -746.0);
  const double k = rint(x * 46.16624130844683);             // 32 / ln2
  double r = fma(-k, 0.02166084938653512, x);               // L1: ln2 / 32 to 32 significant bits
  r = fma(-k, 5.9631716539705866e-12, r);                   // L2
  double p = 1.0 / 720.0;
  p = fma(p, r, 1.0 / 120.0);
  p = fma(p, r, 1.0 / 24.0);
  p = fma(p, r, 1.0 / 6.0);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  const int ki = (int)k;
  return ldexp(tab[ki & 31] * p, ki >> 5);
}

// 2^(t / 32) = exp(t ln2 / 32) for the pair tile's fast read-out, whose exponents come out in these units (the
// scale folded into its per-tile constants): k = rint(t), s = t - k (exact), 2^(k / 32) from the table times the
// degree-6 Taylor polynomial of exp(s ln2 / 32) with the powers of ln2 / 32 folded into its coefficients -- no
// reduction step.  <= 1.5 ulp against the correctly rounded exp of t ln2 / 32 (numpy / mpmath over [-24000, 80]);
// t >= -2^26 (every exponent the pair bounds admit is >= -512 ln 2 ... -25000 units).  14 VALU operations.
__device__ __forceinline__ double exp2_32(double t, const double* tab) {
#pragma clang fp contract(on)
  const double k = rint(t);
  const double sr = t - k;
  double p = 1.4345655584131934e-13;
  p = fma(p, sr, 3.973709984549416e-11);
  p = fma(p, sr, 9.172562701824643e-09);
  p = fma(p, sr, 1.693850972437182e-06);
  p = fma(p, sr, 0.0002345961982022468);
  p = fma(p, sr, 0.02166084939249829);
  p = fma(p, sr, 1.0);
  const int ki = (int)k;
#if GPK_FAST_ABLATE == 1
  return ldexp(p, ki >> 5);  // (timing-only ablation: no table read)
#endif
  return ldexp(tab[ki & 31] * p, ki >> 5);
}

// per-point feature k0 + kq of the periodic leaf: C_k (k < D), S_{k - D} (k < 2 D); k0 a multiple of 4 (inside the
// unrolled k-step loops a constant, so the branch folds)
template <int D>
__device__ __forceinline__ double per_feature(const double* pts, int pt, int k0, int kq, int dp, int sc_sin, int sc_cos) {
#pragma clang fp contract(on)
  if (k0 < D) {
    const double sv = pts[sc_sin + pt * dp + k0 + kq];
    return fma(-2.0 * sv, sv, 1.0);
  }
  const double sv = pts[sc_sin + pt * dp + k0 - D + kq], cv = pts[sc_cos + pt * dp + k0 - D + kq];
  return 2.0 * (sv * cv);
}

// wave w: rows 16 w .. 16 w + 15 of the tile against its 64 columns (four 16 x 16 MFMA blocks, their k-steps
// interleaved: 4 independent accumulator chains per leaf), then the per-element read-out; interior tiles (every row
// and column a training point) skip the generic loop's classes, edge tiles, test rows and ragged members take them
// (the same values as the generic loop).  D a multiple of 4 (compile-time: the k-steps are whole).
template <typename TOut, int D>
__device__ __forceinline__ void pair_mfma_tile(const gpk_kdesc& kd, const AsmArgs& a, const FastNode* fns, int se_leaf,
                                               const double* prow, const double* pcol, int sc_sin, int sc_cos,
                                               const double* na_r, const double* na_c, const double* tab,
                                               int64_t gi0, int64_t gj0, int b, TOut* W) {
#pragma clang fp contract(on)
  static_assert(D % 4 == 0, "whole k-steps");
  constexpr int SS = D / 4, PS = 2 * D / 4;
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, kq = lane >> 4;
  const int dp = a.dp;
  const FastNode fs = fns[se_leaf], fq = fns[1 - se_leaf];
  auto se_op = [&](const double* P, int pt, int k) { return P[fs.off + pt * dp + k]; };
  auto per_op = [&](const double* P, int pt, int k0) { return per_feature<D>(P, pt, k0, kq, dp, sc_sin, sc_cos); };
  // the row operands (this wave's 16 rows) once; the column operands per block
  double ase[SS], ape[PS];
  const int prow_pt = 16 * w + lr;
#pragma unroll
  for (int t = 0; t < SS; ++t) ase[t] = se_op(prow, prow_pt, 4 * t + kq);
#pragma unroll
  for (int t = 0; t < PS; ++t) ape[t] = per_op(prow, prow_pt, 4 * t);
  const bool mul = kd.nodes[2].op == GPK_OP_MUL;
  const bool same_set = !a.plain || a.X == a.Xs;  // (row i and column i are one point)
  constexpr double halfd = 0.5 * (double)D;
  const double noise = a.plain ? 0.0 : a.noise[(int64_t)b * a.noise_stride];
  const int64_t nm = a.plain ? a.n : member_n(a, b), mm = a.plain ? a.m : member_m(a, b);
  const bool interior = !a.plain && gi0 + ATILE <= nm && gj0 + ATILE <= nm;
  // (workgroup-uniform; every tile of an N = 16384 matrix but the 256 diagonal and edge ones)
  const bool fast_tile =
      __builtin_amdgcn_readfirstlane((int)(interior && fs.sg > 0.0 && fq.sg > 0.0)) != 0;
  const bool diag = gi0 == gj0;
  const double kself = (mul ? fs.sg * fq.sg : fs.sg + fq.sg) + noise;  // (diagonal of K + noise I)
  TOut* const Wt = W + gi0 * a.ld + gj0;
  double nrow[4];
  TOut* wrow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    nrow[i] = na_r[16 * w + kq + 4 * i];
    wrow[i] = Wt + (int64_t)(16 * w + kq + 4 * i) * a.ld;
  }
  const double cse = -0.5 * fs.il2, cpe = -2.0 * fq.il2;  // (exp(-0.5 r^2 / l^2), exp(-2 sn / l^2))
  // the fast read-out's exponents in units of ln2 / 32 (exp2_32), the scales sg inside them:
  //   SE   sg exp(-0.5 il2 (|u_i|^2 + |u_j|^2 - 2 u_i.u_j)) = 2^(ts / 32),  ts = min(a_s dse + hr_i + hc_j, lsg_s)
  //   PER  sg exp(-2 il2 (D / 2 - dpe / 2))                 = 2^(tp / 32),  tp = min(a_p dpe + c_p, lsg_p)
  // (the min: the reference's clamp-free direct forms never exceed sg; neither may the expanded ones)
  constexpr double kU = 46.16624130844683;  // 32 / ln2
  const double lsg_s = fast_tile ? log(fs.sg) * kU : 0.0, lsg_p = fast_tile ? log(fq.sg) * kU : 0.0;
  const double a_s = fs.il2 * kU, a_p = fq.il2 * kU;
  const double c_p = fma(-(double)D, a_p, lsg_p);
  double hr[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) hr[i] = fma(-0.5 * a_s, nrow[i], lsg_s);
  // two column blocks at a time (four accumulators and eight elements' exps live: the register count, i.e. the
  // waves per SIMD, is set by this read-out)
#pragma unroll 1
  for (int cp = 0; cp < 2; ++cp) {
    d4 dse[2], dpe[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      dse[h] = d4{0.0, 0.0, 0.0, 0.0};
      dpe[h] = d4{0.0, 0.0, 0.0, 0.0};
    }
#pragma unroll
    for (int t = 0; t < SS; ++t)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        dse[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(ase[t], se_op(pcol, 16 * (2 * cp + h) + lr, 4 * t + kq),
                                                      dse[h], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < PS; ++t)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const double bv = per_op(pcol, 16 * (2 * cp + h) + lr, 4 * t);
        dpe[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(ape[t], bv, dpe[h], 0, 0, 0);
      }
    if (fast_tile) {
      // interior: no classes; MUL: one exp of the summed exponents.  Diagonal tiles: the symmetric form of the SE
      // exponent (K bitwise symmetric there) and k(x, x) + noise exactly on the diagonal.  pair_fast_kernel's values
      // bit for bit (IEEE addition commutes, so the leaf order is moot).
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int col = 16 * (2 * cp + h) + lr;
        const double ncol = na_c[col];
        const double hc = -0.5 * a_s * ncol;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const double hs = diag ? fma(-0.5 * a_s, nrow[i] + ncol, lsg_s) : hr[i] + hc;
          const double ts = fmin(fma(dse[h][i], a_s, hs), lsg_s);
          const double tp = fmin(fma(dpe[h][i], a_p, c_p), lsg_p);
          const double e1 = exp2_32(mul ? ts + tp : ts, tab);
          const double v = mul ? e1 : e1 + exp2_32(tp, tab);
          wrow[i][col] = (TOut)((diag && 16 * w + kq + 4 * i == col) ? kself : v);
        }
      }
      continue;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int col = 16 * (2 * cp + h) + lr;
      const int64_t gj = gj0 + col;
      const double ncol = na_c[col];
      const int ccls = (a.plain || interior) ? CLS_TRAIN : classify(a, gj, nm, mm);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = 16 * w + kq + 4 * i;
        const int64_t gi = gi0 + row;
        const bool same = same_set && gi == gj;
        double r2 = fma(-2.0, dse[h][i], nrow[i] + ncol);
        double sn = fma(-0.5, dpe[h][i], halfd);
        r2 = same ? 0.0 : fmax(r2, 0.0);
        sn = same ? 0.0 : fmax(sn, 0.0);
        const double vse = fs.sg * exp_neg(r2 * cse, tab);
        const double vper = fq.sg * exp_neg(sn * cpe, tab);
        const double v0 = se_leaf == 0 ? vse : vper, v1 = se_leaf == 0 ? vper : vse;
        double v = mul ? v0 * v1 : v0 + v1;
        if (interior) {
          if (gi == gj) v += noise;
        } else if (a.plain) {
          if (gi >= a.n || gj >= a.m || (a.uplo && gj > gi)) continue;
          if (gi == gj) v += a.diag_add;
        } else {
          const int rcls = classify(a, gi, nm, mm);
          if (rcls == CLS_PAD || ccls == CLS_PAD) {
            v = (gi == gj) ? 1.0 : 0.0;
          } else if (a.eye && rcls == CLS_TEST) {
            v = (ccls == CLS_TRAIN && gj == gi - a.n_pad) ? 1.0 : 0.0;
          } else if (a.E != nullptr && rcls == CLS_TEST) {
            v = (ccls == CLS_TRAIN) ? a.E[(int64_t)b * a.e_bs + (gi - a.n_pad) * a.n + gj] : 0.0;
          } else if ((rcls == CLS_TRAIN || rcls == CLS_TEST) && (ccls == CLS_TRAIN || ccls == CLS_TEST)) {
            if (rcls == CLS_TRAIN && ccls == CLS_TRAIN && gi == gj) v += noise;
          } else if (rcls == CLS_Y && ccls == CLS_TRAIN) {
            v = a.y[(int64_t)b * a.y_bs + gj];
          } else {
            v = 0.0;
          }
        }
        wrow[i][col] = (TOut)v;
      }
    }
  }
}

// TREE: 0 single base node, 1 general tree, 2 two-leaf tree (interior_pair)
template <typename TOut, int D, int TREE>
__device__ __forceinline__ bool interior_d(const gpk_kdesc& kd, const FastNode& fn, const FastNode* fns, bool fast,
                                           const double* prow, const double* pcol, int slot_stride, int dp, int c,
                                           int r0, int64_t gi0, int64_t gj, double noise, TOut* W, int64_t ld,
                                           int sc_sin, int sc_cos, bool sc_on) {
  if (fast) {
    if (sc_on && fn.sc && fn.op == GPK_OP_PER) {
      interior_single_sc<TOut, D>(fn, prow, pcol, dp, c, r0, gi0, gj, noise, W, ld);
      return true;
    }
    switch (fn.op) {
      case GPK_OP_SE: interior_single<TOut, D, GPK_OP_SE>(fn, prow, pcol, dp, c, r0, gi0, gj, noise, W, ld); return true;
      case GPK_OP_PER: interior_single<TOut, D, GPK_OP_PER>(fn, prow, pcol, dp, c, r0, gi0, gj, noise, W, ld); return true;
      case GPK_OP_MAT32: interior_single<TOut, D, GPK_OP_MAT32>(fn, prow, pcol, dp, c, r0, gi0, gj, noise, W, ld); return true;
      case GPK_OP_MAT52: interior_single<TOut, D, GPK_OP_MAT52>(fn, prow, pcol, dp, c, r0, gi0, gj, noise, W, ld); return true;
      default: return false;
    }
  }
  if (TREE == 2) {
    interior_pair<TOut, D>(kd, fns, prow, pcol, dp, c, r0, gi0, gj, noise, W, ld, sc_on);
    return true;
  }
  if (!TREE || GPK_ASM_INTERIOR_TREE == 0 || kd.n_ard > 1 || kd.n_nodes > 8) return false;
  interior_tree<TOut, D>(kd, fns, prow, pcol, slot_stride, dp, c, r0, gi0, gj, noise, W, ld, sc_sin, sc_cos, sc_on);
  return true;
}


// Lower-triangular tile t of an augmented build, row-major; with tcol_hi > 0 only the tile columns [0, tcol_hi):
// their triangle, then the full rows below it.
__device__ __forceinline__ void lower_tile(const AsmArgs& a, int64_t t, int64_t& ti, int64_t& tj) {
  const int64_t w = a.tcol_hi;
  if (w > 0 && t >= w * (w + 1) / 2) {
    const int64_t u = t - w * (w + 1) / 2;
    ti = w + u / w;
    tj = u % w;
  } else {
    int64_t r = (int64_t)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while (r * (r + 1) / 2 > t) --r;
    while ((r + 1) * (r + 2) / 2 <= t) ++r;
    ti = r;
    tj = t - r * (r + 1) / 2;
  }
}

// Per-point features of the two-leaf SE + periodic MFMA path, once per point instead of once per tile (a point's
// sin / cos and ARD quotients were recomputed by each of the ~N / 64 tiles it borders: ~20 of the ~110 VALU
// operations per matrix element at N = 16384, D = 8).  One wave per 64-point block of member b: the feature row
// [u_1..u_D | C_1..C_D | S_1..S_D | |u|^2 | 0] of each point -- u the SE leaf's (ARD-rescaled) coordinates, C_k =
// 1 - 2 sin^2(pi f_k), S_k = 2 sin(pi f_k) cos(pi f_k) of the periodic leaf's f_k = x_k / p - rint(x_k / p), the
// same operations, in the same order, as stage_points + per_feature + the per-tile norm loop -- and the block's
// (max |u|^2, every |x_k / p| <= SC_MAX_U) for the tile kernel's bounds.  Points are classified as in
// stage_points (training rows of X, test rows of Xs, zeros elsewhere).  256 threads per block: the four waves
// split the dimensions (the sin / cos and the ARD quotients), wave 0 then sums the norms in dimension order.
template <int D>
__global__ __launch_bounds__(256) void pair_feat_kernel(gpk_kdesc kd, AsmArgs a, int se_node, int per_node) {
#pragma clang fp contract(on)
  constexpr int FS = 3 * D + 2;
  __shared__ double us[ATILE][D + 1];
  const int b = blockIdx.y;
  const int pt = threadIdx.x & (ATILE - 1), grp = threadIdx.x >> 6;  // point, dimensions grp, grp + 4, ...
  const int64_t g = (int64_t)blockIdx.x * ATILE + pt;
  const double* hyp = a.hyp + (int64_t)b * a.hyp_stride;
  const gpk_node se = kd.nodes[se_node], pq = kd.nodes[per_node];
  const bool ard = (se.flags & GPK_NODE_ARD) != 0;
  const double iper = 1.0 / hyp[pq.hyp_offset + 1];
  const int c = classify(a, g, member_n(a, b), member_m(a, b));
  const double* src = nullptr;
  if (c == CLS_TRAIN) src = a.X + (int64_t)b * a.x_bs + g * a.d;
  else if (c == CLS_TEST && a.E == nullptr && !a.eye) src = a.Xs + (int64_t)b * a.xs_bs + (g - a.n_pad) * a.d;
  double* f = const_cast<double*>(a.feat) + (int64_t)b * a.feat_bs + g * FS;
  bool ok = true;
#pragma unroll
  for (int k = grp; k < D; k += 4) {
    const double v = src ? src[k] : 0.0;
    const double u = ard ? v / hyp[se.hyp_offset + k] : v;
    us[pt][k] = u;
    f[k] = u;
    const double t = v * iper;
    ok = ok && fabs(t) <= SC_MAX_U;
    double sv, cv;
    sincospi(t - rint(t), &sv, &cv);
    f[D + k] = fma(-2.0 * sv, sv, 1.0);
    f[2 * D + k] = 2.0 * (sv * cv);
  }
  const bool all_ok = __syncthreads_and(ok) != 0;
  if (threadIdx.x >= ATILE) return;
  double nrm = 0.0;  // (in dimension order: the staged path's norm bit for bit)
#pragma unroll
  for (int k = 0; k < D; ++k) nrm = fma(us[pt][k], us[pt][k], nrm);
  f[3 * D] = nrm;
  f[3 * D + 1] = 0.0;
  double mx = nrm;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
  if (threadIdx.x == 0) {
    double* x = const_cast<double*>(a.faux) + 2 * ((int64_t)b * gridDim.x + blockIdx.x);
    x[0] = mx;
    x[1] = all_ok ? 1.0 : 0.0;
    if (blockIdx.x == 0) {
      // the member's read-out constants (pair_fast_kernel; the same operations as pair_mfma_tile's): exponents in
      // units of ln2 / 32, the scales inside them; [5] the node-level bounds, [6] the SE leaf's 1 / l^2
      const FastNode fsn = make_fast_node(se, hyp, a.d), fqn = make_fast_node(pq, hyp, a.d);
      const bool node_ok = (double)a.d * fqn.il2 <= PAIR_MFMA_MAX_DIL2 && fsn.sg > 0.0 && fqn.sg > 0.0;
      constexpr double kU = 46.16624130844683;
      double* mc = const_cast<double*>(a.faux) + 2 * (int64_t)gridDim.y * gridDim.x + 8 * b;
      mc[0] = fsn.il2 * kU;
      mc[1] = node_ok ? log(fsn.sg) * kU : 0.0;
      mc[2] = fqn.il2 * kU;
      mc[4] = node_ok ? log(fqn.sg) * kU : 0.0;
      mc[3] = fma(-(double)D, mc[2], mc[4]);
      mc[5] = node_ok ? 1.0 : 0.0;
      mc[6] = fsn.il2;
      mc[7] = kd.nodes[2].op == GPK_OP_MUL ? fsn.sg * fqn.sg : fsn.sg + fqn.sg;  // k(x, x)
      if (b == 0) const_cast<int32_t*>(a.tlist)[0] = 0;
    }
  }
}

// The interior tiles of a two-leaf SE + periodic tree whose bounds hold (and the tail rows), from pair_feat_kernel's
// features: one 256-thread workgroup per chunk of consecutive lower tiles (below).  The tile's 2 x 64 feature rows
// (contiguous in HBM, L2-resident; the row's kept from the previous tile of the same tile row) go to LDS -- row
// stride 3 D + 2 doubles, so that the 16 points x 2 k-lanes of an MFMA operand read hit 32 distinct bank pairs --
// then wave w takes rows 16 w .. 16 w + 15 against the 64 columns: per 16 x 16 block D / 4 MFMAs (u_i . u_j) and
// D / 2 (sum_k C_ik C_jk + S_ik S_jk), then per element
//   ADD  2^(ts / 32) + 2^(tp / 32),  MUL  2^((ts + tp) / 32),
//   ts = min(a_s dse + hr_i + hc_j, lsg_s), tp = min(a_p dpe + c_p, lsg_p)   (pair_feat_kernel's member constants)
// Edge tiles and tiles outside the bounds are appended to the tile list for the general instantiation.  No class
// logic, no staging, no sin / cos: ~31 VALU operations per element with ADD (two exps of 14), ~17 with MUL -- a
// kernel of its own, so that none of the general path's registers weigh on it.
#ifndef GPK_FAST_MINB
#define GPK_FAST_MINB 4  // pair_fast_kernel: workgroups per CU the register allocation must allow (A/B)
#endif
#ifndef GPK_FAST_CHUNK
#define GPK_FAST_CHUNK 8  // pair_fast_kernel: consecutive lower tiles per workgroup (C5 K build 0.465 -> 0.450 ms)
#endif
// Workgroup c of member b walks the lower tiles c * chunk .. c * chunk + chunk - 1 (row-major: mostly one tile row,
// whose feature rows it loads once); each tile as one workgroup per tile would -- the same values bit for bit.
// GPK_FAST_DMA: the column features are double-buffered in LDS and the next tile's are fetched by LDS-DMA
// (global_load_lds, no VGPRs) while the current tile is evaluated -- one barrier per tile instead of two, and the
// feature fetch off the tile's critical path (0: the round-5 form, loaded through VGPRs after the barrier).
#ifndef GPK_FAST_DMA
#define GPK_FAST_DMA 0
#endif
typedef __attribute__((address_space(3))) void asm_lds_void;
template <int D, bool MUL>
__global__ __launch_bounds__(256, GPK_FAST_MINB) void pair_fast_kernel(gpk_kdesc kd, AsmArgs a, int64_t ntl,
                                                                      int chunk) {
#pragma clang fp contract(on)
  constexpr int FS = 3 * D + 2, SS = D / 4, PS = 2 * D / 4;
  constexpr int NPC = ATILE * FS / 2;  // 16-B pieces of one tile edge's feature rows
  __shared__ __attribute__((aligned(16))) double fr[ATILE * FS];
  __shared__ __attribute__((aligned(16))) double fcb[GPK_FAST_DMA ? 2 : 1][ATILE * FS];
  __shared__ double tab[32];
  const int b = blockIdx.y;
  const int64_t nm = member_n(a, b), mm = member_m(a, b);
  const double* mc = a.faux + 2 * (int64_t)gridDim.y * a.ntile + 8 * b;
  const double* fb = a.feat + (int64_t)b * a.feat_bs;
  if (threadIdx.x < 32) tab[threadIdx.x] = kExp2Tab32[threadIdx.x];
  int64_t loaded = -1;  // the tile row whose features are in fr
  const int64_t t_end = std::min<int64_t>(ntl, ((int64_t)blockIdx.x + 1) * chunk);
  // LDS-DMA of tile tt's column features into fcb[buf]: wave w moves 64 pieces per instruction, lane-linear
  auto dma_col = [&](int64_t tt, int buf) {
    int64_t ti2, tj2;
    lower_tile(a, tt, ti2, tj2);
    const char* src = reinterpret_cast<const char*>(fb + tj2 * ATILE * FS);
    char* dst = reinterpret_cast<char*>(fcb[buf]);
    const int lane = (int)threadIdx.x & 63;
    for (int base = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) * 64; base < NPC; base += 256)
      if (base + lane < NPC)
        __builtin_amdgcn_global_load_lds(src + (size_t)(base + lane) * 16, (asm_lds_void*)(dst + base * 16), 16, 0, 0);
  };
  int cur = 0;
  if (GPK_FAST_DMA && (int64_t)blockIdx.x * chunk < t_end) dma_col((int64_t)blockIdx.x * chunk, 0);
  for (int64_t t = (int64_t)blockIdx.x * chunk; t < t_end; ++t, cur ^= (GPK_FAST_DMA ? 1 : 0)) {
    if (GPK_FAST_DMA) {
      // this tile's column features have landed (every wave's DMA: vmcnt, then the barrier), and every wave is done
      // with the previous tile (its LDS reads of fcb[cur ^ 1] and fr); then the next tile's DMA into the other buffer
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t + 1 < t_end) dma_col(t + 1, cur ^ 1);
    }
    double* const fc = fcb[cur];
    // (the lane's offsets recomputed per tile: hoisted out of the loop they would hold registers across it)
    int tid = (int)threadIdx.x;
    asm volatile("" : "+v"(tid));
    int64_t ti, tj;
    lower_tile(a, t, ti, tj);
    const int64_t gi0 = ti * ATILE, gj0 = tj * ATILE;
    if (gi0 >= a.n_pad + mm) {
      // tail tiles (the y row and the zero rows below it): y^T on the y row, zeros elsewhere -- the general loop's
      // values (CLS_Y / CLS_ZERO rows), without its staging
      const int c = tid & 63;
      const int64_t gj = gj0 + c;
      const double yv = gj < nm ? a.y[(int64_t)b * a.y_bs + gj] : 0.0;
      double* const Wc = reinterpret_cast<double*>(a.W) + (int64_t)b * a.w_bs + gj;
      for (int rr = tid >> 6; rr < ATILE; rr += 4) Wc[(gi0 + rr) * a.ld] = gi0 + rr == a.y_row ? yv : 0.0;
      continue;
    }
    const double* xr = a.faux + 2 * ((int64_t)b * a.ntile + ti);
    const double* xc = a.faux + 2 * ((int64_t)b * a.ntile + tj);
    const bool fast = gi0 + ATILE <= nm && gj0 + ATILE <= nm && mc[5] != 0.0 && xr[1] != 0.0 && xc[1] != 0.0 &&
                      (xr[0] + xc[0]) * mc[6] <= PAIR_MFMA_MAX_NORM;
    if (!fast) {
      if (tid == 0) {
        int32_t* tl = const_cast<int32_t*>(a.tlist);
        const int k = atomicAdd(tl, 1);
        tl[1 + 3 * k] = b;
        tl[2 + 3 * k] = (int32_t)ti;
        tl[3 + 3 * k] = (int32_t)tj;
      }
      continue;
    }
    if (GPK_FAST_DMA) {
      if (ti != loaded) {  // (a new tile row: its features through VGPRs, behind a barrier of their own)
        const double2* sr = reinterpret_cast<const double2*>(fb + gi0 * FS);
        double2* dr = reinterpret_cast<double2*>(fr);
        for (int e = tid; e < NPC; e += 256) dr[e] = sr[e];
        loaded = ti;
        __syncthreads();
      }
    } else {
      if (loaded >= 0) __syncthreads();  // (the previous tile's LDS reads are done)
      const double2* sr = reinterpret_cast<const double2*>(fb + gi0 * FS);
      const double2* sc = reinterpret_cast<const double2*>(fb + gj0 * FS);
      double2* dr = reinterpret_cast<double2*>(fr);
      double2* dc = reinterpret_cast<double2*>(fc);
      if (ti != loaded) {
        for (int e = tid; e < NPC; e += 256) {
          dr[e] = sr[e];
          dc[e] = sc[e];
        }
      } else {
        for (int e = tid; e < NPC; e += 256) dc[e] = sc[e];
      }
      loaded = ti;
    }
    const double a_s = mc[0], lsg_s = mc[1], a_p = mc[2], c_p = mc[3], lsg_p = mc[4];
    const bool diag = ti == tj;
    const double kself = mc[7] + (diag ? a.noise[(int64_t)b * a.noise_stride] : 0.0);
    if (!GPK_FAST_DMA) __syncthreads();
    const int lane = tid & 63, w = tid >> 6;
    const int lr = lane & 15, kq = lane >> 4;
    double ase[SS], ape[PS];
    const int prow_pt = 16 * w + lr;
#pragma unroll
    for (int t2 = 0; t2 < SS; ++t2) ase[t2] = fr[prow_pt * FS + 4 * t2 + kq];
#pragma unroll
    for (int t2 = 0; t2 < PS; ++t2) ape[t2] = fr[prow_pt * FS + D + 4 * t2 + kq];
    double hr[4];
    double* wrow[4];
    double* const Wt = reinterpret_cast<double*>(a.W) + (int64_t)b * a.w_bs + gi0 * a.ld + gj0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      hr[i] = fma(-0.5 * a_s, fr[(16 * w + kq + 4 * i) * FS + 3 * D], lsg_s);
      wrow[i] = Wt + (int64_t)(16 * w + kq + 4 * i) * a.ld;
    }
#pragma unroll 1
    for (int cp = 0; cp < 2; ++cp) {
      d4 dse[2], dpe[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        dse[h] = d4{0.0, 0.0, 0.0, 0.0};
        dpe[h] = d4{0.0, 0.0, 0.0, 0.0};
      }
#pragma unroll
      for (int t2 = 0; t2 < SS; ++t2)
#pragma unroll
        for (int h = 0; h < 2; ++h)
          dse[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(ase[t2], fc[(16 * (2 * cp + h) + lr) * FS + 4 * t2 + kq],
                                                        dse[h], 0, 0, 0);
#pragma unroll
      for (int t2 = 0; t2 < PS; ++t2)
#pragma unroll
        for (int h = 0; h < 2; ++h)
          dpe[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(ape[t2], fc[(16 * (2 * cp + h) + lr) * FS + D + 4 * t2 + kq],
                                                        dpe[h], 0, 0, 0);
      if (!diag) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int col = 16 * (2 * cp + h) + lr;
          const double hc = -0.5 * a_s * fc[col * FS + 3 * D];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const double ts = fmin(fma(dse[h][i], a_s, hr[i] + hc), lsg_s);
            const double tp = fmin(fma(dpe[h][i], a_p, c_p), lsg_p);
#if GPK_FAST_ABLATE == 2
            { const double v = MUL ? exp2_32(ts + tp, tab) : exp2_32(ts, tab) + exp2_32(tp, tab);
              if (v == 12345.678) wrow[i][col] = v; }  // (timing-only ablation: no stores)
#elif GPK_FAST_ABLATE == 3
            wrow[i][col] = ts + tp;  // (timing-only ablation: no exps)
#else
            wrow[i][col] = MUL ? exp2_32(ts + tp, tab) : exp2_32(ts, tab) + exp2_32(tp, tab);
#endif
          }
        }
      } else {
        // the diagonal tile: the symmetric form of the SE exponent (K bitwise symmetric), k(x, x) + noise exactly
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int col = 16 * (2 * cp + h) + lr;
          const double ncol = fc[col * FS + 3 * D];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = 16 * w + kq + 4 * i;
            const double ts = fmin(fma(dse[h][i], a_s, fma(-0.5 * a_s, fr[row * FS + 3 * D] + ncol, lsg_s)), lsg_s);
            const double tp = fmin(fma(dpe[h][i], a_p, c_p), lsg_p);
            const double v = MUL ? exp2_32(ts + tp, tab) : exp2_32(ts, tab) + exp2_32(tp, tab);
            wrow[i][col] = row == col ? kself : v;
          }
        }
      }
    }
  }
}

// ------------------------------------------------------------------ f32 K build of a single base node
// C3's precision (fp32 storage + f32 MFMA factorisation): a single SE (direct norm) / Matern-3/2 /
// Matern-5/2 node written as f32.  The general instantiation evaluates every element in f64 (library exp / sqrt,
// ~50 f64 VALU operations) and rounds; here the squared distance stays f64 (the differences of the scaled points,
// as the reference's direct form; no cancellation) and the element's transcendental part runs on the f32 hardware
// instructions (v_sqrt_f32, v_exp_f32: a few operations instead of ~35):
//   SE     sg 2^(s * (-0.5 il2 log2 e))
//   MAT32  sg (1 + f) 2^(-f log2 e),           f = sqrt(3 s il2)
//   MAT52  sg (1 + f + f^2 / 3) 2^(-f log2 e), f = sqrt(5 s il2)      (= ((1 + f) + 5 d^2 / (3 l^2)) e^-f)
// with s the squared Euclidean distance of the (ARD-scaled) points, or f = c d1 il of the L1 distance d1 for the
// reference's L1 Matern forms (K/BaseKernels.py:702-720, :859-880).  Element error against the f64 value: a few f32
// ulps (kernel-matrix tests: 4e-6 of max |K|); K stays exactly symmetric (the f64 differences are antisymmetric, the
// sums run in one order) and its diagonal is (f32)(sg + noise) as in the general path.  One 256-thread workgroup per
// chunk of consecutive lower tiles (the tile row's points kept in LDS between tiles): lane c owns column c (its
// point in registers), wave w the rows 16 w .. 16 w + 15; whole 256-B tile rows per store.  Tiles with test, padding
// or identity rows go to a device list for the general instantiation; y-row / zero tail tiles are written here.
template <int D, int OP, bool L1>
__global__ __launch_bounds__(256) void f32_fast_kernel(gpk_kdesc kd, AsmArgs a, int64_t ntl, int chunk) {
  __shared__ double rp[ATILE * D];
  const int b = blockIdx.y;
  const int64_t nm = member_n(a, b), mm = member_m(a, b);
  const double* hyp = a.hyp + (int64_t)b * a.hyp_stride;
  const gpk_node nd = kd.nodes[0];
  const FastNode fn = make_fast_node(nd, hyp, D);
  const bool ard = (nd.flags & GPK_NODE_ARD) != 0;
  double il[D];
#pragma unroll
  for (int k = 0; k < D; ++k) il[k] = ard ? 1.0 / hyp[nd.hyp_offset + k] : 1.0;
  constexpr double LOG2E = 1.4426950408889634;
  // exponent / distance scales (f64 products, rounded once to f32 per element)
  const double cse = -0.5 * fn.il2 * LOG2E;                              // SE: s -> log2 of the value
  const double cm2 = (OP == GPK_OP_MAT52 ? 5.0 : 3.0) * fn.il2;          // MAT, Euclidean: s -> f^2
  const double cm1 = (OP == GPK_OP_MAT52 ? SQRT5 : SQRT3) * fn.il;       // MAT, L1: d1 -> f
  const float sg = (float)fn.sg;
  const float kself = (float)(fn.sg + a.noise[(int64_t)b * a.noise_stride]);
  float* const Wb = reinterpret_cast<float*>(a.W) + (int64_t)b * a.w_bs;
  const double* Xb = a.X + (int64_t)b * a.x_bs;
  const int tid = (int)threadIdx.x, c = tid & 63, w = tid >> 6;
  int64_t loaded = -1;
  const int64_t t_end = std::min<int64_t>(ntl, ((int64_t)blockIdx.x + 1) * chunk);
  // the lane's column point of the next tile is loaded while the current one is evaluated (clamped to a valid
  // training point: tail / edge tiles ignore it)
  auto col_point = [&](int64_t t, double (&xv)[D]) {
    int64_t ti2, tj2;
    lower_tile(a, t, ti2, tj2);
    const int64_t gjn = std::min<int64_t>(tj2 * ATILE + c, nm - 1);
#pragma unroll
    for (int k = 0; k < D; ++k) xv[k] = Xb[gjn * D + k];
  };
  double xn[D];
  int64_t t = (int64_t)blockIdx.x * chunk;
  if (t < t_end) col_point(t, xn);
  for (; t < t_end; ++t) {
    double xc[D];
#pragma unroll
    for (int k = 0; k < D; ++k) xc[k] = xn[k] * il[k];
    if (t + 1 < t_end) col_point(t + 1, xn);
    int64_t ti, tj;
    lower_tile(a, t, ti, tj);
    const int64_t gi0 = ti * ATILE, gj0 = tj * ATILE;
    if (gi0 >= a.n_pad + mm) {
      // tail tiles: y^T on the y row, zeros elsewhere (the general loop's CLS_Y / CLS_ZERO rows)
      const int64_t gj = gj0 + c;
      const float yv = gj < nm ? (float)a.y[(int64_t)b * a.y_bs + gj] : 0.0f;
      for (int rr = w; rr < ATILE; rr += 4) Wb[(gi0 + rr) * a.ld + gj] = gi0 + rr == a.y_row ? yv : 0.0f;
      continue;
    }
    if (!(gi0 + ATILE <= nm && gj0 + ATILE <= nm)) {
      if (tid == 0 && a.tlist) {  // (NULL only when the host ruled edge tiles out: launch_assemble's no_edges)
        int32_t* tl = const_cast<int32_t*>(a.tlist);
        const int k = atomicAdd(tl, 1);
        tl[1 + 3 * k] = b;
        tl[2 + 3 * k] = (int32_t)ti;
        tl[3 + 3 * k] = (int32_t)tj;
      }
      continue;
    }
    if (ti != loaded) {
      if (loaded >= 0) __syncthreads();  // (every wave done with the previous row points)
      for (int e = tid; e < ATILE * D; e += 256) {
        const int pt = e / D, k = e - pt * D;
        rp[e] = Xb[(gi0 + pt) * D + k] * il[k];
      }
      __syncthreads();
      loaded = ti;
    }
    const int64_t gj = gj0 + c;
    float* const Wc = Wb + gi0 * a.ld + gj;
    const bool diag = ti == tj;
#pragma unroll 4
    for (int i = 0; i < 16; ++i) {
      const int row = 16 * w + i;
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k) {
        const double dlt = rp[row * D + k] - xc[k];
        s = L1 ? s + fabs(dlt) : fma(dlt, dlt, s);
      }
      float v;
      if (OP == GPK_OP_SE) {
        v = sg * __builtin_amdgcn_exp2f((float)(s * cse));
      } else {
        const float f = L1 ? (float)(s * cm1) : __builtin_amdgcn_sqrtf((float)(s * cm2));
        const float e = __builtin_amdgcn_exp2f(-f * (float)LOG2E);
        const float poly = OP == GPK_OP_MAT52 ? fmaf(f, fmaf(f, 1.0f / 3.0f, 1.0f), 1.0f) : 1.0f + f;
        v = sg * (poly * e);
      }
      if (diag && row == c) v = kself;
      Wc[(int64_t)row * a.ld] = v;
    }
  }
}

// TREE: the instantiation for kernel trees (its interior loop holds two column points in registers;
// single-node kernels get the lighter instantiation and keep four waves per SIMD); 3: two-leaf SE + periodic trees
// on MFMA (pair_mfma_tile), tiles outside its error bounds through the generic loop -- an instantiation of its own,
// so that neither path's registers limit the other's occupancy
#ifndef GPK_ASM3_MINB
#define GPK_ASM3_MINB 3  // TREE 3: workgroups per CU the register allocation must allow (A/B)
#endif
template <typename TOut, int TREE>
__device__ __forceinline__ void assemble_tile(const gpk_kdesc& kd, const AsmArgs& a, int64_t ti, int64_t tj, int b,
                                              double* smem, int& sc_flag, unsigned long long* pair_max) {
  const int slot_stride = ATILE * a.dp;
  // slots per tile edge: raw points, one per ARD node, and (periodic node through sin / cos) sin, cos
  const int scq = a.A == nullptr ? sc_node(kd) : -1;
  const int sc_slot = 1 + kd.n_ard;
  const int nslot = sc_slot + (scq >= 0 ? 2 : 0);
  double* hyp_s = smem;                                  // GPK_MAX_HYP
  double* prow = smem + GPK_MAX_HYP;                     // nslot * slot_stride
  double* pcol = prow + nslot * slot_stride;
  const int tid = threadIdx.x;
  const double* hyp_g = a.hyp + (int64_t)b * a.hyp_stride;
  for (int e = tid; e < kd.n_hyp; e += 256) hyp_s[e] = hyp_g[e];
  if (tid == 0) {
    sc_flag = 1;
    pair_max[0] = pair_max[1] = 0ull;
  }
  __syncthreads();
  // per-node constants of a tree (reciprocals of the hyperparameters; single nodes keep theirs in
  // registers below)
  FastNode* fns = reinterpret_cast<FastNode*>(pcol + nslot * slot_stride);
  const int sc_sin = sc_slot * slot_stride, sc_cos = (sc_slot + 1) * slot_stride;
  if (kd.n_nodes > 1 && tid < kd.n_nodes) {
    const gpk_node nd = kd.nodes[tid];
    if (nd.op != GPK_OP_ADD && nd.op != GPK_OP_MUL) {
      FastNode f = make_fast_node(nd, hyp_s, a.d);
      f.off = (nd.flags & GPK_NODE_ARD) ? (nd.ard_slot + 1) * slot_stride : 0;
      if (tid == scq) {
        f.sc = 1;
        f.sc_sin = sc_sin;
        f.sc_cos = sc_cos;
      }
      fns[tid] = f;
    }
  }
  const int64_t gi0 = ti * ATILE, gj0 = tj * ATILE;
  if (a.A == nullptr) {
    const double sc_iper = scq >= 0 ? 1.0 / hyp_s[kd.nodes[scq].hyp_offset + 1] : 0.0;
    stage_points(kd, a, hyp_s, prow, gi0, b, true, slot_stride, scq >= 0 ? sc_slot : 0, sc_iper, &sc_flag);
    stage_points(kd, a, hyp_s, pcol, gj0, b, false, slot_stride, scq >= 0 ? sc_slot : 0, sc_iper, &sc_flag);
  }
  __syncthreads();
  // the sin / cos form for this tile: every staged point within |x / p| <= SC_MAX_U (workgroup-uniform)
  const bool sc_on = scq >= 0 && sc_flag != 0;
  if (TREE == 3 && sc_on && a.A == nullptr && a.d >= 4 && !GPK_ASM_ABLATE) {
    // two-leaf SE + periodic tree: the tile on f64 MFMA (pair_mfma_tile) when its error bounds hold
    const gpk_node n0 = kd.nodes[0], n1 = kd.nodes[1];
    const bool se0 = n0.op == GPK_OP_SE && !(n0.flags & GPK_NODE_SE_EXPANDED);
    const bool se1 = n1.op == GPK_OP_SE && !(n1.flags & GPK_NODE_SE_EXPANDED);
    const int se_leaf = (se0 && n1.op == GPK_OP_PER) ? 0 : ((se1 && n0.op == GPK_OP_PER) ? 1 : -1);
    if (se_leaf >= 0 && fns[1 - se_leaf].sc && (double)a.d * fns[1 - se_leaf].il2 <= PAIR_MFMA_MAX_DIL2) {
      double* na_r = reinterpret_cast<double*>(fns + GPK_MAX_NODES);
      double* na_c = na_r + ATILE;
      double* tab = na_c + ATILE;  // exp_neg's 2^(j / 32)
      if (tid < 32) tab[tid] = kExp2Tab32[tid];
      const FastNode fs = fns[se_leaf];
      if (tid < 2 * ATILE) {
        const double* pts = tid < ATILE ? prow : pcol;
        const int pt = tid & (ATILE - 1);
        double nrm = 0.0;
        for (int k = 0; k < a.d; ++k) {
          const double u = pts[fs.off + pt * a.dp + k];
          nrm = fma(u, u, nrm);
        }
        (tid < ATILE ? na_r : na_c)[pt] = nrm;
        atomicMax(&pair_max[tid < ATILE ? 0 : 1], (unsigned long long)__double_as_longlong(nrm));
      }
      __syncthreads();
      const double bound = (__longlong_as_double((long long)pair_max[0]) + __longlong_as_double((long long)pair_max[1])) *
                           fs.il2;
      if (bound <= PAIR_MFMA_MAX_NORM) {
        TOut* const Wb = reinterpret_cast<TOut*>(a.W) + (int64_t)b * a.w_bs;
        switch (a.d) {
          case 4: pair_mfma_tile<TOut, 4>(kd, a, fns, se_leaf, prow, pcol, sc_sin, sc_cos, na_r, na_c, tab, ti * ATILE, tj * ATILE, b, Wb); return;
          case 8: pair_mfma_tile<TOut, 8>(kd, a, fns, se_leaf, prow, pcol, sc_sin, sc_cos, na_r, na_c, tab, ti * ATILE, tj * ATILE, b, Wb); return;
          // case 12: pair_mfma_tile<TOut, 12>(kd, a, fns, se_leaf, prow, pcol, sc_sin, sc_cos, na_r, na_c, tab, ti * ATILE, tj * ATILE, b, Wb); return;
          // case 16: pair_mfma_tile<TOut, 16>(kd, a, fns, se_leaf, prow, pcol, sc_sin, sc_cos, na_r, na_c, tab, ti * ATILE, tj * ATILE, b, Wb); return;
          default: break;
        }
      }
    }
  }

  const int c = tid & 63;
  const int r0 = tid >> 6;
  const int64_t gj = gj0 + c;
  TOut* W = reinterpret_cast<TOut*>(a.W) + (int64_t)b * a.w_bs;
  if (a.plain) {
    for (int rr = r0; rr < ATILE; rr += 4) {
      const int64_t gi = gi0 + rr;
      if (gi >= a.n || gj >= a.m) continue;
      if (a.uplo && gj > gi) continue;
      double v;
      if (kd.n_nodes == 1) {
        FastNode f1 = make_fast_node(kd.nodes[0], hyp_s, a.d);
        f1.sc = scq == 0 ? 1 : 0;
        f1.sc_sin = sc_sin;
        f1.sc_cos = sc_cos;
        v = fast_value(f1, prow + rr * a.dp + fast_off(kd, slot_stride), pcol + c * a.dp + fast_off(kd, slot_stride),
                       sc_on);
      } else {
        v = eval_tree_fast(kd, fns, prow + rr * a.dp, pcol + c * a.dp, sc_on);
      }
      if (gi == gj) v += a.diag_add;
      W[gi * a.ld + gj] = (TOut)v;
    }
    return;
  }
  const double noise = a.noise[(int64_t)b * a.noise_stride];
  const int64_t nm = member_n(a, b), mm = member_m(a, b);
  const int ccls = classify(a, gj, nm, mm);
  const double yv = (ccls == CLS_TRAIN) ? a.y[(int64_t)b * a.y_bs + gj] : 0.0;
  const bool col_kernel = (ccls == CLS_TRAIN || ccls == CLS_TEST);
  const bool fast = kd.n_nodes == 1;
  FastNode fn = make_fast_node(kd.nodes[0], hyp_s, a.d);
  fn.off = fast_off(kd, slot_stride);
  fn.sc = scq == 0 ? 1 : 0;
  fn.sc_sin = sc_sin;
  fn.sc_cos = sc_cos;
  if (TREE != 3 && GPK_ASM_INTERIOR && !a.generic && a.A == nullptr && gi0 + ATILE <= nm) {  // lower tiles: gj0 <= gi0
    bool done = false;
    switch (a.d) {
      case 1: done = interior_d<TOut, 1, TREE>(kd, fn, fns, fast, prow, pcol, slot_stride, a.dp, c, r0, gi0, gj, noise, W, a.ld, sc_sin, sc_cos, sc_on); break;
      case 2: done = interior_d<TOut, 2, TREE>(kd, fn, fns, fast, prow, pcol, slot_stride, a.dp, c, r0, gi0, gj, noise, W, a.ld, sc_sin, sc_cos, sc_on); break;
      case 3: done = interior_d<TOut, 3, TREE>(kd, fn, fns, fast, prow, pcol, slot_stride, a.dp, c, r0, gi0, gj, noise, W, a.ld, sc_sin, sc_cos, sc_on); break;
      case 4: done = interior_d<TOut, 4, TREE>(kd, fn, fns, fast, prow, pcol, slot_stride, a.dp, c, r0, gi0, gj, noise, W, a.ld, sc_sin, sc_cos, sc_on); break;
      case 8: done = interior_d<TOut, 8, TREE>(kd, fn, fns, fast, prow, pcol, slot_stride, a.dp, c, r0, gi0, gj, noise, W, a.ld, sc_sin, sc_cos, sc_on); break;
      default: break;
    }
    if (done) return;
  }
#ifndef GPK_ASM_UNROLL
#define GPK_ASM_UNROLL 1
#endif
#pragma unroll GPK_ASM_UNROLL
  for (int rr = r0; rr < ATILE; rr += 4) {
    const int64_t gi = gi0 + rr;
    const int rcls = classify(a, gi, nm, mm);
    double v = 0.0;
    if (rcls == CLS_PAD || ccls == CLS_PAD) {
      v = (gi == gj) ? 1.0 : 0.0;
    } else if (a.eye && rcls == CLS_TEST) {
      v = (ccls == CLS_TRAIN && gj == gi - a.n_pad) ? 1.0 : 0.0;
    } else if (a.E != nullptr && rcls == CLS_TEST) {
      v = (ccls == CLS_TRAIN) ? a.E[(int64_t)b * a.e_bs + (gi - a.n_pad) * a.n + gj] : 0.0;
    } else if (a.A != nullptr && rcls == CLS_TRAIN && ccls == CLS_TRAIN) {
      // dense mode: the caller's matrix (lower triangle, mirrored) + noise on the diagonal
      const double* Ab = a.A + (int64_t)b * a.a_bs;
      v = (gj <= gi) ? Ab[gi * a.a_ld + gj] : Ab[gj * a.a_ld + gi];
      if (gi == gj) v += noise;
    } else if ((rcls == CLS_TRAIN || rcls == CLS_TEST) && col_kernel) {
      if (!GPK_ASM_ABLATE)
        v = fast ? fast_value(fn, prow + fn.off + rr * a.dp, pcol + fn.off + c * a.dp, sc_on)
                 : eval_tree_fast(kd, fns, prow + rr * a.dp, pcol + c * a.dp, sc_on);
      if (rcls == CLS_TRAIN && ccls == CLS_TRAIN && gi == gj) v += noise;
    } else if (rcls == CLS_Y && ccls == CLS_TRAIN) {
      v = yv;
    }
    W[gi * a.ld + gj] = (TOut)v;
  }
}

template <typename TOut, int TREE>
__global__ __launch_bounds__(256, TREE == 3 ? GPK_ASM3_MINB : 1) void assemble_kernel(gpk_kdesc kd, AsmArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  __shared__ int sc_flag;
  __shared__ unsigned long long pair_max[2];  // (TREE 3) max |u|^2 of the tile's row / column points, as bits
  // (TREE 4: TREE 3's body over the tile list -- the tiles pair_fast_kernel left: diagonal, edge, outside its
  // bounds -- in a persistent loop; an instantiation of its own without the register bound of TREE 3's, whose
  // occupancy its few tiles do not need)
  // (TREE 5: TREE 0's body over the tile list f32_fast_kernel left)
  constexpr int TB = TREE == 4 ? 3 : TREE == 5 ? 0 : TREE;
  const bool list = TREE >= 4;
  const int cnt = list ? a.tlist[0] : 1;
  for (int e = list ? (int)blockIdx.x : 0; e < cnt; e += list ? (int)gridDim.x : 1) {
    int b;
    int64_t ti, tj;
    if (list) {
      const int32_t* t = a.tlist + 1 + 3 * e;
      b = t[0];
      ti = t[1];
      tj = t[2];
      __syncthreads();  // (the previous tile's LDS reads)
    } else if (a.plain) {
      b = blockIdx.y;
      ti = blockIdx.x / ((a.m + ATILE - 1) / ATILE);
      tj = blockIdx.x - ti * ((a.m + ATILE - 1) / ATILE);
      if (a.uplo && tj > ti) return;
    } else {
      b = blockIdx.y;
      lower_tile(a, blockIdx.x, ti, tj);
    }
    assemble_tile<TOut, TB>(kd, a, ti, tj, b, smem, sc_flag, pair_max);
  }
}

// ================================================================================ LML gradient
// d(-LML)/d theta_p = 1/2 sum_ij (K^-1 - alpha alpha^T)_ij dK_ij/d theta_p: the reverse-mode
// derivative TensorFlow's GradientTape takes through LogLikelihood.get_metric for
// VariationalSgdFitter (gpbasics/Optimizer/Fitter.py:104-158).  K^-1 and alpha come out of ONE
// factorisation of the augmented matrix with identity extra rows: its corner holds -K^-1 (lower
// triangle) and its y row -alpha^T.  Every workgroup takes one 64 x 64 lower tile of the n x n
// training block, re-evaluates the kernel tree there (values of every node, so the adjoint of a
// base node is the product of the node values its ancestors multiply it by -- a host-built mask)
// and reduces the weighted partial derivatives of each base node's hyperparameters; partial sums
// per tile go to a workspace reduced in a fixed order by grad_reduce_kernel (deterministic).

// values of every node of the postfix program (node q's value = its subtree's value) into the
// thread's LDS column v[q * 256]
__device__ __forceinline__ void eval_nodes(const gpk_kdesc& kd, const double* hyp, const double* pa,
                                           const double* pb, int slot_stride, int d, double* v) {
  Stack st;
  st.s0 = 0.0;
  int sp = 0;
#pragma unroll 1
  for (int q = 0; q < kd.n_nodes; ++q) {
    const gpk_node nd = kd.nodes[q];
    if (nd.op == GPK_OP_ADD || nd.op == GPK_OP_MUL) {
      const double top = st.get(sp - 1);
      const double below = st.get(sp - 2);
      st.set(sp - 2, nd.op == GPK_OP_ADD ? below + top : below * top);
      sp -= 1;
    } else {
      const int off = (nd.flags & GPK_NODE_ARD) ? (nd.ard_slot + 1) * slot_stride : 0;
      st.set(sp, base_value(nd, hyp, pa + off, pb + off, d));
      sp += 1;
    }
    v[q * 256] = st.get(sp - 1);
  }
}

constexpr int GNP = GPK_MAX_DIM + 1;  // hyperparameters of one base node, at most (ARD l + sg)

// acc[k] += coef * d k_node / d h[k] for the node's hyperparameters h (reference formulas, see the
// citations at the top of this file; |l| of the Matern kernels differentiates to sign(l)).
__device__ __forceinline__ void base_partials(const gpk_node& nd, const double* __restrict__ hyp,
                                              const double* a, const double* b, int d, double coef,
                                              double (&acc)[GNP]) {
  const int fl = nd.flags;
  const bool ard = (fl & GPK_NODE_ARD) != 0;
  const bool scaled = (fl & GPK_NODE_SCALED) != 0;
  const double* h = hyp + nd.hyp_offset;
  if (nd.op == GPK_OP_SE) {
    double s = 0.0;
    if (fl & GPK_NODE_SE_EXPANDED) {
      double na = 0.0, nb = 0.0, ab = 0.0;
      for (int k = 0; k < d; ++k) {
        na += a[k] * a[k];
        nb += b[k] * b[k];
        ab += a[k] * b[k];
      }
      const double dist = sqrt((na - 2.0 * ab) + nb);
      s = dist * dist;
    } else {
      for (int k = 0; k < d; ++k) {
        const double t = a[k] - b[k];
        s += t * t;
      }
    }
    const int sg_at = ard ? d : 1;
    const double sg = scaled ? h[sg_at] : 1.0;
    if (ard) {
      const double r = exp(-0.5 * s);
#pragma unroll
      for (int k = 0; k < GPK_MAX_DIM; ++k)
        if (k < d) {
          const double t = a[k] - b[k];  // (x_k - y_k) / l_k
          acc[k] += coef * sg * r * (t * t) / h[k];
        }
      if (scaled) acc[GPK_MAX_DIM] += coef * r;
    } else {
      const double l = h[0];
      const double r = exp(-0.5 * (s / (l * l)));
      acc[0] += coef * sg * r * s / (l * l * l);
      if (scaled) acc[1] += coef * r;
    }
    return;
  }
  if (nd.op == GPK_OP_PER) {
    const double l = h[0], per = h[1];
    double sn, tw;  // sum sin^2(theta), sum theta sin(2 theta)
    if (fl & GPK_NODE_STANDARD) {
      sn = 0.0;
      tw = 0.0;
      for (int k = 0; k < d; ++k) {
        const double th = PI * (fabs(a[k] - b[k]) / per);
        const double t = sin(th);
        sn += t * t;
        tw += th * sin(2.0 * th);
      }
    } else {
      double dist = 0.0;
      for (int k = 0; k < d; ++k) dist += fabs(a[k] - b[k]);
      const double th = PI * (dist / per);
      const double t = sin(th);
      sn = t * t;
      tw = th * sin(2.0 * th);
    }
    const double r = exp((-2.0 * sn) / (l * l));
    const double sg = scaled ? h[2] : 1.0;
    acc[0] += coef * sg * r * 4.0 * sn / (l * l * l);
    acc[1] += coef * sg * r * 2.0 * tw / (l * l * per);
    if (scaled) acc[2] += coef * r;
    return;
  }
  // MAT32 / MAT52
  const bool std_form = (fl & GPK_NODE_STANDARD) != 0;
  double dist = 0.0;
  if (std_form) {
    for (int k = 0; k < d; ++k) {
      const double t = a[k] - b[k];
      dist += t * t;
    }
    dist = sqrt(dist);
  } else {
    for (int k = 0; k < d; ++k) dist += fabs(a[k] - b[k]);
  }
  const double c = (nd.op == GPK_OP_MAT52) ? SQRT5 : SQRT3;
  const int sg_at = ard ? d : 1;
  const double sg = scaled ? h[sg_at] : 1.0;
  const double l = ard ? 1.0 : h[0];
  const double f = (c * dist) / fabs(l);
  const double e = exp(-f);
  double r, drdf;  // value and d value / d f
  if (nd.op == GPK_OP_MAT52) {
    r = ((1.0 + f) + f * f / 3.0) * e;
    drdf = -(f / 3.0) * (1.0 + f) * e;
  } else {
    r = (1.0 + f) * e;
    drdf = -f * e;
  }
  if (ard) {
    // f = c dist(u, v), u = x / l: d dist / d l_k = -|u_k - v_k| / l_k (L1) or
    // -(u_k - v_k)^2 / (l_k dist) (Euclidean)
#pragma unroll
    for (int k = 0; k < GPK_MAX_DIM; ++k)
      if (k < d) {
        const double t = a[k] - b[k];
        double dd;
        if (std_form) dd = dist > 0.0 ? -(t * t) / (h[k] * dist) : 0.0;
        else dd = -fabs(t) / h[k];
        acc[k] += coef * sg * drdf * c * dd;
      }
    if (scaled) acc[GPK_MAX_DIM] += coef * r;
  } else {
    acc[0] += coef * sg * drdf * (-f / l);  // d f / d l = -f / l  (f uses |l|)
    if (scaled) acc[1] += coef * r;
  }
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T>
__global__ __launch_bounds__(256) void grad_kernel(gpk_kdesc kd, AsmArgs a, GradArgs g) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int slot_stride = ATILE * a.dp;
  double* hyp_s = smem;                                  // GPK_MAX_HYP
  double* al_r = hyp_s + GPK_MAX_HYP;                    // alpha of the tile rows / columns
  double* al_c = al_r + ATILE;
  double* red = al_c + ATILE;                            // [4 waves][GNP + 1]
  double* prow = red + 4 * (GNP + 1);
  double* pcol = prow + (1 + kd.n_ard) * slot_stride;
  double* vals = pcol + (1 + kd.n_ard) * slot_stride;   // [n_nodes][256] node values (MUL trees)

  const int b = blockIdx.y;
  const int64_t t = blockIdx.x;
  int64_t r = (int64_t)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
  while (r * (r + 1) / 2 > t) --r;
  while ((r + 1) * (r + 2) / 2 <= t) ++r;
  const int64_t ti = r, tj = t - r * (r + 1) / 2;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int np1 = kd.n_hyp + 1;
  double* part = g.part + ((int64_t)b * gridDim.x + t) * np1;

  const double* hyp_g = g.hyp + (int64_t)b * g.hyp_stride;
  for (int e = tid; e < kd.n_hyp; e += 256) hyp_s[e] = hyp_g[e];
  const T* W = reinterpret_cast<const T*>(g.W) + (int64_t)b * g.w_bs;
  const int64_t gi0 = ti * ATILE, gj0 = tj * ATILE;
  if (tid < 2 * ATILE) {
    const int64_t gg = (tid < ATILE ? gi0 : gj0) + (tid & (ATILE - 1));
    // y row of the corner: -alpha^T
    const double v = gg < g.n ? -(double)W[g.y_row * g.ld + g.n_pad + gg] : 0.0;
    (tid < ATILE ? al_r : al_c)[tid & (ATILE - 1)] = v;
  }
  __syncthreads();
  stage_points(kd, a, hyp_s, prow, gi0, b, true, slot_stride);
  stage_points(kd, a, hyp_s, pcol, gj0, b, false, slot_stride);
  __syncthreads();

  const int c = lane;
  const int64_t gj = gj0 + c;
  // weighted (K^-1 - alpha alpha^T)_ij of this thread's 16 elements: weight 2 off the diagonal
  // (the strictly lower triangle stands for both halves), 1 on it; the corner holds -K^-1
  auto qval = [&](int rr) -> double {
    const int64_t gi = gi0 + rr;
    if (gi >= g.n || gj > gi) return 0.0;
    const double qq = -(double)W[(g.n_pad + gi) * g.ld + g.n_pad + gj] - al_r[rr] * al_c[c];
    return gi == gj ? qq : 2.0 * qq;
  };
  double noise_acc = 0.0;  // d K / d noise = I: the diagonal of the weighted matrix
  if (ti == tj && (c & 3) == wave) noise_acc = qval(c);

  for (int qn = 0; qn < kd.n_nodes; ++qn) {
    const gpk_node nd = kd.nodes[qn];
    if (nd.op == GPK_OP_ADD || nd.op == GPK_OP_MUL) continue;
    const uint32_t mask = g.adj_mask[qn];
    const int off = (nd.flags & GPK_NODE_ARD) ? (nd.ard_slot + 1) * slot_stride : 0;
    double acc[GNP];
#pragma unroll
    for (int k = 0; k < GNP; ++k) acc[k] = 0.0;
#pragma unroll 1
    for (int k = 0; k < ATILE / 4; ++k) {
      const int rr = wave + 4 * k;
      const double qk = qval(rr);
      if (qk == 0.0) continue;
      double adj = 1.0;
      if (mask != 0u) {
        eval_nodes(kd, hyp_s, prow + rr * a.dp, pcol + c * a.dp, slot_stride, a.d, vals + tid);
#pragma unroll 1
        for (int q = 0; q < kd.n_nodes; ++q)
          if (mask & (1u << q)) adj *= vals[q * 256 + tid];
      }
      base_partials(nd, hyp_s, prow + off + rr * a.dp, pcol + off + c * a.dp, a.d, qk * adj, acc);
    }
    // hyperparameter slots of this node: ARD l_0..l_{d-1} then sg (stored at acc[GPK_MAX_DIM])
    const bool ard = (nd.flags & GPK_NODE_ARD) != 0;
    const int nshape = ard ? a.d : (nd.op == GPK_OP_PER ? 2 : 1);
    const bool scaled = (nd.flags & GPK_NODE_SCALED) != 0;
    const bool sg_moved = ard && scaled;
    const int np = nshape + (scaled ? 1 : 0);
#pragma unroll
    for (int k = 0; k < GNP; ++k) {
      if (k < np) {
        const double sres = wave_sum((sg_moved && k == a.d) ? acc[GPK_MAX_DIM] : acc[k]);
        if (lane == 0) red[wave * (GNP + 1) + k] = sres;
      }
    }
    __syncthreads();
    if (tid < np)
      part[nd.hyp_offset + tid] = red[tid] + red[(GNP + 1) + tid] + red[2 * (GNP + 1) + tid] +
                                  red[3 * (GNP + 1) + tid];
    __syncthreads();
  }
  const double ns = wave_sum(noise_acc);
  if (lane == 0) red[wave * (GNP + 1) + GNP] = ns;
  __syncthreads();
  if (tid == 0)
    part[kd.n_hyp] = red[GNP] + red[(GNP + 1) + GNP] + red[2 * (GNP + 1) + GNP] + red[3 * (GNP + 1) + GNP];
}

// grad[b][p] = 1/2 sum over tiles (fixed order); NaN where the factorisation failed
__global__ __launch_bounds__(256) void grad_reduce_kernel(GradArgs g, int64_t ntri, int np1) {
  __shared__ double red[256];
  const int p = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const double* part = g.part + (int64_t)b * ntri * np1 + p;
  double s = 0.0;
  for (int64_t t = tid; t < ntri; t += 256) s += part[t * np1];
  red[tid] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w) red[tid] += red[tid + w];
    __syncthreads();
  }
  if (tid == 0) g.grad[(int64_t)b * np1 + p] = g.info[b] != 0 ? NAN : 0.5 * red[0];
}

// ===================================================================== kernel-matrix reverse mode
// gpk_kernel_vjp: for a weight matrix G [n, m] (the adjoint of K(X, Z) = kernel(X, Z), as TensorFlow's
// tape would hand it back from the ops downstream of get_tf_tensor), the hyperparameter adjoints
// sum_ij G_ij dK_ij / d theta_p and the adjoints of the SECOND argument's points, sum_i G_ij dK_ij / d z_jk
// (the inducing inputs of the Nystroem metrics, Optimizer/Fitter.py:76-87,128-130).  A symmetric K(Z, Z)
// is handled by the caller with G + G^T (k(a, b) = k(b, a)).  Derivatives are the analytic ones of the
// reference formulas; at coincident points the distance terms differentiate to 0 (tf.abs' sign(0)
// = 0 for the L1 kernels; for SE the reference's sqrt-then-square, Auxiliary/Distances.py:5-7, would
// give TensorFlow's 0 * inf = NaN there -- the analytic limit 0 is returned instead).

// acc_z[k] += coef * d k_node(a, b) / d b_k in the node's own coordinates (ARD nodes: scaled points)
__device__ __forceinline__ void base_input_partials(const gpk_node& nd, const double* __restrict__ hyp,
                                                    const double* a, const double* b, int d, double coef,
                                                    double (&acc)[GPK_MAX_DIM]) {
  const int fl = nd.flags;
  const bool ard = (fl & GPK_NODE_ARD) != 0;
  const bool scaled = (fl & GPK_NODE_SCALED) != 0;
  const double* h = hyp + nd.hyp_offset;
  const double v = base_value(nd, hyp, a, b, d);  // includes sg
  if (nd.op == GPK_OP_SE) {
    const double l = ard ? 1.0 : h[0];
    const double c = coef * v / (l * l);
#pragma unroll
    for (int k = 0; k < GPK_MAX_DIM; ++k)
      if (k < d) acc[k] += c * (a[k] - b[k]);
    return;
  }
  if (nd.op == GPK_OP_PER) {
    const double l = h[0], per = h[1];
    const double c = coef * v * (-2.0 / (l * l)) * (PI / per);  // d k / d sn * d theta / d |t|
    if (fl & GPK_NODE_STANDARD) {
#pragma unroll
      for (int k = 0; k < GPK_MAX_DIM; ++k)
        if (k < d) {
          const double t = a[k] - b[k];
          const double th = PI * (fabs(t) / per);
          const double sgn = t > 0.0 ? 1.0 : (t < 0.0 ? -1.0 : 0.0);
          acc[k] += c * sin(2.0 * th) * (-sgn);
        }
    } else {
      double dist = 0.0;
      for (int k = 0; k < d; ++k) dist += fabs(a[k] - b[k]);
      const double s2 = sin(2.0 * PI * (dist / per));
#pragma unroll
      for (int k = 0; k < GPK_MAX_DIM; ++k)
        if (k < d) {
          const double t = a[k] - b[k];
          const double sgn = t > 0.0 ? 1.0 : (t < 0.0 ? -1.0 : 0.0);
          acc[k] += c * s2 * (-sgn);
        }
    }
    return;
  }
  // MAT32 / MAT52: k = sg r(f), f = c dist / |l|
  const bool std_form = (fl & GPK_NODE_STANDARD) != 0;
  double dist = 0.0;
  if (std_form) {
    for (int k = 0; k < d; ++k) {
      const double t = a[k] - b[k];
      dist += t * t;
    }
    dist = sqrt(dist);
  } else {
    for (int k = 0; k < d; ++k) dist += fabs(a[k] - b[k]);
  }
  const double cc = (nd.op == GPK_OP_MAT52) ? SQRT5 : SQRT3;
  const double sg = scaled ? h[ard ? d : 1] : 1.0;
  const double l = ard ? 1.0 : fabs(h[0]);
  const double f = (cc * dist) / l;
  const double e = exp(-f);
  const double drdf = (nd.op == GPK_OP_MAT52) ? -(f / 3.0) * (1.0 + f) * e : -f * e;
  const double c = coef * sg * drdf * (cc / l);  // times d dist / d b_k
#pragma unroll
  for (int k = 0; k < GPK_MAX_DIM; ++k)
    if (k < d) {
      const double t = a[k] - b[k];
      double dd;
      if (std_form) dd = dist > 0.0 ? -t / dist : 0.0;
      else dd = -(t > 0.0 ? 1.0 : (t < 0.0 ? -1.0 : 0.0));
      acc[k] += c * dd;
    }
}

// one 64 x 64 tile of K(X, Z) per workgroup (row tile ti = blockIdx.y, column tile tj = blockIdx.x);
// lane = column, wave w = rows w, w + 4, ...; per-tile partial sums to the workspace, reduced in a
// fixed order by vjp_reduce_kernel (deterministic)
__global__ __launch_bounds__(256) void vjp_kernel(gpk_kdesc kd, AsmArgs a, VjpArgs g) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int slot_stride = ATILE * a.dp;
  double* hyp_s = smem;                                  // GPK_MAX_HYP
  double* red = hyp_s + GPK_MAX_HYP;                     // [4 waves][GNP]
  double* zred = red + 4 * GNP;                          // [4 waves][64][d]
  double* prow = zred + 4 * ATILE * a.d;
  double* pcol = prow + (1 + kd.n_ard) * slot_stride;
  double* vals = pcol + (1 + kd.n_ard) * slot_stride;    // [n_nodes][256] node values (MUL trees)

  const int64_t ti = blockIdx.y, tj = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  for (int e = tid; e < kd.n_hyp; e += 256) hyp_s[e] = g.hyp[e];
  __syncthreads();
  const int64_t gi0 = ti * ATILE, gj0 = tj * ATILE;
  stage_points(kd, a, hyp_s, prow, gi0, 0, true, slot_stride);
  stage_points(kd, a, hyp_s, pcol, gj0, 0, false, slot_stride);
  __syncthreads();
  const int c = lane;
  const int64_t gj = gj0 + c;
  double* part = g.part_h + (ti * (int64_t)gridDim.x + tj) * kd.n_hyp;
  double gz[GPK_MAX_DIM];
#pragma unroll
  for (int k = 0; k < GPK_MAX_DIM; ++k) gz[k] = 0.0;
  for (int qn = 0; qn < kd.n_nodes; ++qn) {
    const gpk_node nd = kd.nodes[qn];
    if (nd.op == GPK_OP_ADD || nd.op == GPK_OP_MUL) continue;
    const uint32_t mask = g.adj_mask[qn];
    const bool ard = (nd.flags & GPK_NODE_ARD) != 0;
    const int off = ard ? (nd.ard_slot + 1) * slot_stride : 0;
    double acc[GNP], az[GPK_MAX_DIM];
#pragma unroll
    for (int k = 0; k < GNP; ++k) acc[k] = 0.0;
#pragma unroll
    for (int k = 0; k < GPK_MAX_DIM; ++k) az[k] = 0.0;
#pragma unroll 1
    for (int k = 0; k < ATILE / 4; ++k) {
      const int rr = wave + 4 * k;
      const int64_t gi = gi0 + rr;
      if (gi >= a.n || gj >= a.m) continue;
      const double qk = g.G ? g.G[gi * g.ldg + gj] : g.gu[gi] * g.gv[gj];
      if (qk == 0.0) continue;
      double adj = 1.0;
      if (mask != 0u) {
        eval_nodes(kd, hyp_s, prow + rr * a.dp, pcol + c * a.dp, slot_stride, a.d, vals + tid);
#pragma unroll 1
        for (int q = 0; q < kd.n_nodes; ++q)
          if (mask & (1u << q)) adj *= vals[q * 256 + tid];
      }
      base_partials(nd, hyp_s, prow + off + rr * a.dp, pcol + off + c * a.dp, a.d, qk * adj, acc);
      if (g.want_z) base_input_partials(nd, hyp_s, prow + off + rr * a.dp, pcol + off + c * a.dp, a.d, qk * adj, az);
    }
    // raw coordinates: an ARD node sees z_k / l_k
#pragma unroll
    for (int k = 0; k < GPK_MAX_DIM; ++k)
      if (k < a.d) gz[k] += ard ? az[k] / hyp_s[nd.hyp_offset + k] : az[k];
    const int nshape = ard ? a.d : (nd.op == GPK_OP_PER ? 2 : 1);
    const bool scaled = (nd.flags & GPK_NODE_SCALED) != 0;
    const bool sg_moved = ard && scaled;
    const int np = nshape + (scaled ? 1 : 0);
#pragma unroll
    for (int k = 0; k < GNP; ++k) {
      if (k < np) {
        const double sres = wave_sum((sg_moved && k == a.d) ? acc[GPK_MAX_DIM] : acc[k]);
        if (lane == 0) red[wave * GNP + k] = sres;
      }
    }
    __syncthreads();
    if (tid < np) part[nd.hyp_offset + tid] = red[tid] + red[GNP + tid] + red[2 * GNP + tid] + red[3 * GNP + tid];
    __syncthreads();
  }
  if (!g.want_z) return;
  for (int k = 0; k < a.d; ++k) zred[(wave * ATILE + c) * a.d + k] = gz[k];
  __syncthreads();
  for (int e = tid; e < ATILE * a.d; e += 256) {
    const int cc = e / a.d, k = e - cc * a.d;
    if (gj0 + cc < a.m)
      g.part_z[(ti * a.m + gj0 + cc) * a.d + k] = zred[(0 * ATILE + cc) * a.d + k] + zred[(1 * ATILE + cc) * a.d + k] +
                                                   zred[(2 * ATILE + cc) * a.d + k] + zred[(3 * ATILE + cc) * a.d + k];
  }
}

// out[p] = scale * sum_t part[t * stride + p] over t < nt (fixed order); one workgroup per p
__global__ __launch_bounds__(256) void vjp_reduce_kernel(const double* part, int64_t nt, int64_t stride, double scale,
                                                         double* out) {
  __shared__ double red[256];
  const int64_t p = blockIdx.x;
  const int tid = threadIdx.x;
  double s = 0.0;
  for (int64_t t = tid; t < nt; t += 256) s += part[t * stride + p];
  red[tid] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w) red[tid] += red[tid + w];
    __syncthreads();
  }
  if (tid == 0) out[p] = scale * red[0];
}

}  // namespace

size_t vjp_workspace_elems(const gpk_kdesc& kd, int64_t n, int64_t m, int32_t d, bool want_z) {
  const int64_t tr = (n + ATILE - 1) / ATILE, tc = (m + ATILE - 1) / ATILE;
  return (size_t)(tr * tc * kd.n_hyp) + (want_z ? (size_t)(tr * m * d) : 0);
}

hipError_t launch_vjp(const gpk_kdesc& kd, const VjpArgs& g0, const double* X, int64_t n, const double* Z, int64_t m,
                      int32_t d, double* grad_hyp, double* grad_z, hipStream_t s) {
  AsmArgs a;
  memset(&a, 0, sizeof(a));
  a.hyp = g0.hyp;
  a.X = X;
  a.Xs = Z;
  a.n = n;
  a.m = m;
  a.d = d;
  a.dp = (d % 2 == 0) ? d + 1 : d;
  a.plain = 1;
  VjpArgs g = g0;
  g.want_z = grad_z != nullptr ? 1 : 0;
  const int64_t tr = (n + ATILE - 1) / ATILE, tc = (m + ATILE - 1) / ATILE;
  g.part_z = g.part_h + tr * tc * kd.n_hyp;
  bool has_mul = false;
  for (int q = 0; q < kd.n_nodes; ++q) has_mul |= g.adj_mask[q] != 0u;
  const size_t lds = sizeof(double) * (GPK_MAX_HYP + 4 * GNP + 4 * (size_t)ATILE * d +
                                       2 * (size_t)(1 + kd.n_ard) * ATILE * a.dp +
                                       (has_mul ? (size_t)kd.n_nodes * 256 : 0));
  {
    hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(vjp_kernel), lds);  // (d = 16, two ARD nodes: 118 KB)
    if (e != hipSuccess) return e;
  }
  if (kd.n_hyp > 0) {
    hipLaunchKernelGGL(vjp_kernel, dim3((unsigned)tc, (unsigned)tr), dim3(256), lds, s, kd, a, g);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(vjp_reduce_kernel, dim3((unsigned)kd.n_hyp), dim3(256), 0, s, g.part_h, tr * tc,
                       (int64_t)kd.n_hyp, 1.0, grad_hyp);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  } else if (g.want_z) {
    hipLaunchKernelGGL(vjp_kernel, dim3((unsigned)tc, (unsigned)tr), dim3(256), lds, s, kd, a, g);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (g.want_z) {
    hipLaunchKernelGGL(vjp_reduce_kernel, dim3((unsigned)(m * d)), dim3(256), 0, s, g.part_z, tr, m * (int64_t)d, 1.0,
                       grad_z);
    return hipGetLastError();
  }
  return hipSuccess;
}

hipError_t launch_grad(const gpk_kdesc& kd, const GradArgs& g, int dtype, int32_t batch, hipStream_t s) {
  // the staging helpers read the points through an augmented-layout AsmArgs
  AsmArgs a;
  memset(&a, 0, sizeof(a));
  a.hyp = g.hyp;
  a.hyp_stride = g.hyp_stride;
  a.X = g.X;
  a.x_bs = g.x_bs;
  a.n = g.n;
  a.m = g.n;
  a.n_pad = g.n_pad;
  a.y_row = g.y_row;
  a.d = g.d;
  a.dp = g.dp;
  a.eye = 1;
  const int64_t ntri = g.ntile * (g.ntile + 1) / 2;
  bool has_mul = false;
  for (int q = 0; q < kd.n_nodes; ++q) has_mul |= g.adj_mask[q] != 0u;
  const size_t lds = sizeof(double) * (GPK_MAX_HYP + 2 * ATILE + 4 * (GNP + 1) +
                                       2 * (size_t)(1 + kd.n_ard) * ATILE * a.dp +
                                       (has_mul ? (size_t)kd.n_nodes * 256 : 0));
  dim3 grid((unsigned)ntri, (unsigned)batch, 1);
  {
    hipError_t e = ensure_dyn_lds(dtype == GPK_F64 ? reinterpret_cast<const void*>(grad_kernel<double>)
                                                   : reinterpret_cast<const void*>(grad_kernel<float>), lds);
    if (e != hipSuccess) return e;
  }
  if (dtype == GPK_F64)
    hipLaunchKernelGGL(grad_kernel<double>, grid, dim3(256), lds, s, kd, a, g);
  else
    hipLaunchKernelGGL(grad_kernel<float>, grid, dim3(256), lds, s, kd, a, g);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(grad_reduce_kernel, dim3((unsigned)(kd.n_hyp + 1), (unsigned)batch), dim3(256), 0, s,
                     g, ntri, kd.n_hyp + 1);
  return hipGetLastError();
}

// The K build's stream-ordered scratch (the per-point features of pair_feat_kernel): one pool per device, created
// on first use, that keeps its memory between builds (release threshold: never).
static hipMemPool_t feat_pool() {
  static std::mutex mu;
  static std::map<int, hipMemPool_t> pools;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  auto it = pools.find(dev);
  if (it != pools.end()) return it->second;
  hipMemPoolProps props;
  memset(&props, 0, sizeof(props));
  props.allocType = hipMemAllocationTypePinned;
  props.location.type = hipMemLocationTypeDevice;
  props.location.id = dev;
  hipMemPool_t p = nullptr;
  if (hipMemPoolCreate(&p, &props) != hipSuccess) {
    (void)hipGetLastError();
    p = nullptr;
  } else {
    uint64_t keep = UINT64_MAX;
    (void)hipMemPoolSetAttribute(p, hipMemPoolAttrReleaseThreshold, &keep);
  }
  pools[dev] = p;
  return p;
}

static bool tune_pair_off() {  // GPK_ASM_PAIR=0: two-leaf trees through the general tree instantiation (A/B)
  static const bool off = [] {
    const char* v = getenv("GPK_ASM_PAIR");
    return v && *v == '0';
  }();
  return off;
}

hipError_t launch_assemble(const gpk_kdesc& kd, const AsmArgs& a, int dtype, int32_t batch,
                           hipStream_t s) {
  const int nslot = 1 + kd.n_ard + ((a.A == nullptr && sc_node(kd) >= 0) ? 2 : 0);
  const size_t lds = sizeof(double) * (GPK_MAX_HYP + 2 * (size_t)nslot * ATILE * a.dp) +
                     sizeof(FastNode) * GPK_MAX_NODES + sizeof(double) * (2 * ATILE + 32);  // (+ pair_mfma_tile's)
  dim3 grid;
  if (a.plain) {
    const int64_t tr = (a.n + ATILE - 1) / ATILE, tc = (a.m + ATILE - 1) / ATILE;
    grid = dim3((unsigned)(tr * tc), 1, 1);
  } else if (a.tcol_hi > 0 && a.tcol_hi < a.ntile) {
    const int64_t w = a.tcol_hi;
    grid = dim3((unsigned)(w * (w + 1) / 2 + (a.ntile - w) * w), (unsigned)batch, 1);
  } else {
    grid = dim3((unsigned)(a.ntile * (a.ntile + 1) / 2), (unsigned)batch, 1);
  }
  // instantiation: 0 single base node, 2 two leaves under one ADD / MUL, 3 the two leaves SE (direct norm) and a
  // separable periodic node at D >= 4 (pair_mfma_tile), 1 any other tree
  const bool pair = kd.n_nodes == 3 && (kd.nodes[2].op == GPK_OP_ADD || kd.nodes[2].op == GPK_OP_MUL);
  int tree = kd.n_nodes == 1 ? 0 : (pair && !tune_pair_off() ? 2 : 1);
  if (tree == 2 && GPK_ASM_PAIR_MFMA && a.A == nullptr && a.d % 4 == 0 && dtype == GPK_F64) {
    const int q = sc_node(kd);
    const gpk_node se = kd.nodes[q == 0 ? 1 : 0];
    if ((q == 0 || q == 1) && se.op == GPK_OP_SE && !(se.flags & GPK_NODE_SE_EXPANDED)) tree = 3;
  }
  // tree 3 on an augmented matrix: the per-point features first (pair_feat_kernel), into stream-ordered scratch of
  // the library's pool (freed on the stream after the build; the pool keeps its memory, so after the first call
  // this is a host-side bookkeeping step), then pair_fast_kernel over the grid, then the general instantiation over
  // the tiles it left.  Without the scratch (or with gpk_tune("asm_feat", 0)) the general instantiation takes the
  // grid and stages every tile's points itself (the same values, bit for bit).
  AsmArgs af = a;
  af.feat = nullptr;
  af.faux = nullptr;
  af.tlist = nullptr;
  void* scratch = nullptr;
  if (tree == 3 && !a.plain && (a.d == 4 || a.d == 8) && a.ntile > 0 && tune_asm_feat()) {
    const int fsz = 3 * a.d + 2;
    const int64_t rows = a.ntile * ATILE;
    const size_t ntl = (size_t)grid.x * batch;
    const size_t fdoubles = (size_t)batch * rows * fsz + 2 * (size_t)batch * a.ntile + 8 * (size_t)batch;
    const size_t fbytes = sizeof(double) * fdoubles + sizeof(int32_t) * (1 + 3 * ntl);
    hipMemPool_t pool = feat_pool();
    if (pool && hipMallocFromPoolAsync(&scratch, fbytes, pool, s) == hipSuccess) {
      af.feat = static_cast<const double*>(scratch);
      af.faux = af.feat + (size_t)batch * rows * fsz;
      af.feat_bs = rows * fsz;
      af.feat_fs = fsz;
      af.tlist = reinterpret_cast<const int32_t*>(af.feat + fdoubles);
      const int q = sc_node(kd);
      const bool mul = kd.nodes[2].op == GPK_OP_MUL;
      const dim3 fgrid((unsigned)a.ntile, (unsigned)batch, 1);
      const int64_t tiles = (int64_t)grid.x;  // lower tiles per member
      const int chunk = GPK_FAST_CHUNK;
      const dim3 cgrid((unsigned)((tiles + chunk - 1) / chunk), (unsigned)batch, 1);
      if (a.d == 8) {
        hipLaunchKernelGGL((pair_feat_kernel<8>), fgrid, dim3(256), 0, s, kd, af, 1 - q, q);
        if (mul)
          hipLaunchKernelGGL((pair_fast_kernel<8, true>), cgrid, dim3(256), 0, s, kd, af, tiles, chunk);
        else
          hipLaunchKernelGGL((pair_fast_kernel<8, false>), cgrid, dim3(256), 0, s, kd, af, tiles, chunk);
      } else {
        hipLaunchKernelGGL((pair_feat_kernel<4>), fgrid, dim3(256), 0, s, kd, af, 1 - q, q);
        if (mul)
          hipLaunchKernelGGL((pair_fast_kernel<4, true>), cgrid, dim3(256), 0, s, kd, af, tiles, chunk);
        else
          hipLaunchKernelGGL((pair_fast_kernel<4, false>), cgrid, dim3(256), 0, s, kd, af, tiles, chunk);
      }
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) {
        (void)hipFreeAsync(scratch, s);
        return e;
      }
      // the leftover tiles: ~ one per tile row of the matrix normally (diagonal + edge), all of them at worst
      grid = dim3((unsigned)std::min<size_t>(ntl, 2048), 1, 1);
    } else {
      (void)hipGetLastError();
      scratch = nullptr;
    }
  }
  // f32, one SE (direct) / MAT32 / MAT52 node: f32_fast_kernel over the grid (interior and tail tiles), then the general
  // instantiation over the tiles it left (TREE 5; the list lives in the same pool's stream-ordered scratch)
  if (dtype == GPK_F32 && tree == 0 && !a.plain && !a.generic && a.A == nullptr && a.ntile > 0 && tune_asm_f32_fast() &&
      (a.d == 1 || a.d == 2 || a.d == 3 || a.d == 4 || a.d == 8)) {
    const gpk_node nd = kd.nodes[0];
    const bool se = nd.op == GPK_OP_SE && !(nd.flags & GPK_NODE_SE_EXPANDED);
    const bool mat = nd.op == GPK_OP_MAT32 || nd.op == GPK_OP_MAT52;
    // every tile interior (training rows and columns) or tail (y / zero rows): n = n_pad, no test, identity or
    // dense rows, no ragged members -- then no edge tile can occur and the kernel runs alone (no list, no memset)
    const bool no_edges = a.n == a.n_pad && a.m == 0 && !a.nb && !a.mb && !a.eye && a.E == nullptr &&
                          (a.tcol_hi <= 0 || a.tcol_hi >= a.ntile);
    hipMemPool_t pool = (se || mat) && !no_edges ? feat_pool() : nullptr;
    const size_t ntl = (size_t)grid.x * batch;
    if ((se || mat) &&
        (no_edges || (pool && hipMallocFromPoolAsync(&scratch, sizeof(int32_t) * (1 + 3 * ntl), pool, s) == hipSuccess))) {
      af.tlist = static_cast<const int32_t*>(scratch);
      if (scratch) {
        const hipError_t em = hipMemsetAsync(scratch, 0, sizeof(int32_t), s);
        if (em != hipSuccess) {
          (void)hipFreeAsync(scratch, s);
          return em;
        }
      }
      const int64_t tiles = (int64_t)grid.x;
      const int chunk = tune_asm_f32_chunk();
      const dim3 cgrid((unsigned)((tiles + chunk - 1) / chunk), (unsigned)batch, 1);
      // (L1: the reference's Matern distance beyond D = 1; at D = 1 both forms are |x - y|)
      const bool l1 = mat && !(nd.flags & GPK_NODE_STANDARD) && a.d > 1;
#define GPK_F32_LAUNCH(DD)                                                                                         \
  if (se) hipLaunchKernelGGL((f32_fast_kernel<DD, GPK_OP_SE, false>), cgrid, dim3(256), 0, s, kd, af, tiles, chunk);        \
  else if (nd.op == GPK_OP_MAT32 && l1) hipLaunchKernelGGL((f32_fast_kernel<DD, GPK_OP_MAT32, true>), cgrid, dim3(256), 0, s, kd, af, tiles, chunk); \
  else if (nd.op == GPK_OP_MAT32) hipLaunchKernelGGL((f32_fast_kernel<DD, GPK_OP_MAT32, false>), cgrid, dim3(256), 0, s, kd, af, tiles, chunk); \
  else if (l1) hipLaunchKernelGGL((f32_fast_kernel<DD, GPK_OP_MAT52, true>), cgrid, dim3(256), 0, s, kd, af, tiles, chunk); \
  else hipLaunchKernelGGL((f32_fast_kernel<DD, GPK_OP_MAT52, false>), cgrid, dim3(256), 0, s, kd, af, tiles, chunk);
      switch (a.d) {
        case 1: GPK_F32_LAUNCH(1) break;
        case 2: GPK_F32_LAUNCH(2) break;
        case 3: GPK_F32_LAUNCH(3) break;
        case 4: GPK_F32_LAUNCH(4) break;
        default: GPK_F32_LAUNCH(8) break;
      }
#undef GPK_F32_LAUNCH
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) {
        if (scratch) (void)hipFreeAsync(scratch, s);
        return e;
      }
      if (no_edges) return hipSuccess;
      // (the edge tiles: about one tile row and column per member -- a persistent loop over the list)
      grid = dim3((unsigned)std::min<size_t>(ntl, 256), 1, 1);
      tree = 5;
    } else {
      (void)hipGetLastError();
      scratch = nullptr;
    }
  }
  // (above 64 KB -- e.g. an ARD node beside a standard PER node, whose per-point sin / cos take two more point
  // slots, at d = 16: 71 KB; two ARD nodes: 87 KB -- the kernel's dynamic-LDS limit must be raised first)
  {
    const void* fn = dtype == GPK_F64
                         ? (af.tlist != nullptr ? reinterpret_cast<const void*>(assemble_kernel<double, 4>)
                            : tree == 3 ? reinterpret_cast<const void*>(assemble_kernel<double, 3>)
                            : tree == 2 ? reinterpret_cast<const void*>(assemble_kernel<double, 2>)
                                      : tree == 1 ? reinterpret_cast<const void*>(assemble_kernel<double, 1>)
                                                  : reinterpret_cast<const void*>(assemble_kernel<double, 0>))
                         : (tree == 5 ? reinterpret_cast<const void*>(assemble_kernel<float, 5>)
                            : tree == 2 ? reinterpret_cast<const void*>(assemble_kernel<float, 2>)
                                      : tree == 1 ? reinterpret_cast<const void*>(assemble_kernel<float, 1>)
                                                  : reinterpret_cast<const void*>(assemble_kernel<float, 0>));
    hipError_t e = ensure_dyn_lds(fn, lds);
    if (e != hipSuccess) return e;
  }
  if (af.tlist != nullptr && dtype == GPK_F64) tree = 4;
  if (dtype == GPK_F64) {
    if (tree == 4)
      hipLaunchKernelGGL((assemble_kernel<double, 4>), grid, dim3(256), lds, s, kd, af);
    else if (tree == 3)
      hipLaunchKernelGGL((assemble_kernel<double, 3>), grid, dim3(256), lds, s, kd, af);
    else if (tree == 2)
      hipLaunchKernelGGL((assemble_kernel<double, 2>), grid, dim3(256), lds, s, kd, a);
    else if (tree == 1)
      hipLaunchKernelGGL((assemble_kernel<double, 1>), grid, dim3(256), lds, s, kd, a);
    else
      hipLaunchKernelGGL((assemble_kernel<double, 0>), grid, dim3(256), lds, s, kd, a);
  } else {
    if (tree == 5)
      hipLaunchKernelGGL((assemble_kernel<float, 5>), grid, dim3(256), lds, s, kd, af);
    else if (tree == 2)
      hipLaunchKernelGGL((assemble_kernel<float, 2>), grid, dim3(256), lds, s, kd, a);
    else if (tree == 1)
      hipLaunchKernelGGL((assemble_kernel<float, 1>), grid, dim3(256), lds, s, kd, a);
    else
      hipLaunchKernelGGL((assemble_kernel<float, 0>), grid, dim3(256), lds, s, kd, a);
  }
  hipError_t e = hipGetLastError();
  if (scratch) {
    const hipError_t ef = hipFreeAsync(scratch, s);
    if (e == hipSuccess) e = ef;
  }
  return e;
}

}  // namespace gpk
