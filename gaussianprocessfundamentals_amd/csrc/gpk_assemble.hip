// Kernel-matrix build (the HBM-write-bound half of the LML hot path).
//
// One 256-thread workgroup writes one 64 x 64 tile.  The tile's 64 row points and 64 column
// points (plus their per-ARD-node rescaled copies) are staged once in LDS; every lane then
// owns one column and walks 16 rows, evaluating the postfix kernel program in registers and
// storing whole 512-B rows (64 consecutive fp64 per wave instruction).  In the augmented
// layout only lower-triangular tiles are launched (the factorisation never reads the upper
// triangle), so the bytes written are p(p+64)/2 elements per batch member.
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
                                               const double* na_r, const double* na_c, int64_t gi0, int64_t gj0,
                                               int b, TOut* W) {
#pragma clang fp contract(on)
  static_assert(D % 4 == 0, "whole k-steps");
  constexpr int SS = D / 4, PS = 2 * D / 4;
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, kq = lane >> 4;
  const int dp = a.dp;
  const FastNode fs = fns[se_leaf], fq = fns[1 - se_leaf];
  // the row operands (this wave's 16 rows) once; the column operands per block
  double ase[SS], ape[PS];
  const int prow_pt = 16 * w + lr;
#pragma unroll
  for (int t = 0; t < SS; ++t) ase[t] = prow[fs.off + prow_pt * dp + 4 * t + kq];
#pragma unroll
  for (int t = 0; t < PS; ++t)
    ape[t] = per_feature<D>(prow, prow_pt, 4 * t, kq, dp, sc_sin, sc_cos);
  const bool mul = kd.nodes[2].op == GPK_OP_MUL;
  const bool same_set = !a.plain || a.X == a.Xs;  // (row i and column i are one point)
  constexpr double halfd = 0.5 * (double)D;
  const double noise = a.plain ? 0.0 : a.noise[(int64_t)b * a.noise_stride];
  const int64_t nm = a.plain ? a.n : member_n(a, b), mm = a.plain ? a.m : member_m(a, b);
  const bool interior = !a.plain && gi0 + ATILE <= nm && gj0 + ATILE <= nm;
  // (workgroup-uniform; every tile of an N = 16384 matrix but the 256 diagonal and edge ones)
  const bool fast_tile = __builtin_amdgcn_readfirstlane((int)(interior && gi0 != gj0)) != 0;
  TOut* const Wt = W + gi0 * a.ld + gj0;
  double nrow[4];
  TOut* wrow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    nrow[i] = na_r[16 * w + kq + 4 * i];
    wrow[i] = Wt + (int64_t)(16 * w + kq + 4 * i) * a.ld;
  }
  const double cse = -0.5 * fs.il2, cpe = -2.0 * fq.il2;  // (exp(-0.5 r^2 / l^2), exp(-2 sn / l^2))
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
        dse[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(ase[t], pcol[fs.off + (16 * (2 * cp + h) + lr) * dp + 4 * t + kq],
                                                      dse[h], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < PS; ++t)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const double bv = per_feature<D>(pcol, 16 * (2 * cp + h) + lr, 4 * t, kq, dp, sc_sin, sc_cos);
        dpe[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(ape[t], bv, dpe[h], 0, 0, 0);
      }
    if (fast_tile) {
      // interior, off the diagonal: no classes, no noise, no coincident points
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int col = 16 * (2 * cp + h) + lr;
        const double ncol = na_c[col];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const double r2 = fmax(fma(-2.0, dse[h][i], nrow[i] + ncol), 0.0);
          const double sn = fmax(fma(-0.5, dpe[h][i], halfd), 0.0);
          const double vse = fs.sg * exp(r2 * cse);
          const double vper = fq.sg * exp(sn * cpe);
          const double v0 = se_leaf == 0 ? vse : vper, v1 = se_leaf == 0 ? vper : vse;
          wrow[i][col] = (TOut)(mul ? v0 * v1 : v0 + v1);
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
        const double vse = fs.sg * exp(r2 * cse);
        const double vper = fq.sg * exp(sn * cpe);
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


// TREE: the instantiation for kernel trees (its interior loop holds two column points in registers;
// single-node kernels get the lighter instantiation and keep four waves per SIMD); 3: two-leaf SE + periodic trees
// on MFMA (pair_mfma_tile), tiles outside its error bounds through the generic loop -- an instantiation of its own,
// so that neither path's registers limit the other's occupancy
#ifndef GPK_ASM3_MINB
#define GPK_ASM3_MINB 3  // TREE 3: workgroups per CU the register allocation must allow (A/B)
#endif
template <typename TOut, int TREE>
__global__ __launch_bounds__(256, TREE == 3 ? GPK_ASM3_MINB : 1) void assemble_kernel(gpk_kdesc kd, AsmArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  __shared__ int sc_flag;
  __shared__ unsigned long long pair_max[2];  // (TREE 2) max |u|^2 of the tile's row / column points, as bits
  const int slot_stride = ATILE * a.dp;
  // slots per tile edge: raw points, one per ARD node, and (periodic node through sin / cos) sin, cos
  const int scq = a.A == nullptr ? sc_node(kd) : -1;
  const int sc_slot = 1 + kd.n_ard;
  const int nslot = sc_slot + (scq >= 0 ? 2 : 0);
  double* hyp_s = smem;                                  // GPK_MAX_HYP
  double* prow = smem + GPK_MAX_HYP;                     // nslot * slot_stride
  double* pcol = prow + nslot * slot_stride;

  const int b = blockIdx.y;
  int64_t ti, tj;
  if (a.plain) {
    ti = blockIdx.x / ((a.m + ATILE - 1) / ATILE);
    tj = blockIdx.x - ti * ((a.m + ATILE - 1) / ATILE);
    if (a.uplo && tj > ti) return;
  } else {
    // lower-triangular tile enumeration, row-major; with tcol_hi > 0 only the tile columns
    // [0, tcol_hi): their triangle, then the full rows below it
    const int64_t t = blockIdx.x;
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
          case 4: pair_mfma_tile<TOut, 4>(kd, a, fns, se_leaf, prow, pcol, sc_sin, sc_cos, na_r, na_c, ti * ATILE, tj * ATILE, b, Wb); return;
          case 8: pair_mfma_tile<TOut, 8>(kd, a, fns, se_leaf, prow, pcol, sc_sin, sc_cos, na_r, na_c, ti * ATILE, tj * ATILE, b, Wb); return;
          // case 12: pair_mfma_tile<TOut, 12>(kd, a, fns, se_leaf, prow, pcol, sc_sin, sc_cos, na_r, na_c, ti * ATILE, tj * ATILE, b, Wb); return;
          // case 16: pair_mfma_tile<TOut, 16>(kd, a, fns, se_leaf, prow, pcol, sc_sin, sc_cos, na_r, na_c, ti * ATILE, tj * ATILE, b, Wb); return;
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
                     sizeof(FastNode) * GPK_MAX_NODES + sizeof(double) * 2 * ATILE;  // (+ pair_mfma_tile's norms)
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
  // (above 64 KB -- e.g. an ARD node beside a standard PER node, whose per-point sin / cos take two more point
  // slots, at d = 16: 71 KB; two ARD nodes: 87 KB -- the kernel's dynamic-LDS limit must be raised first)
  {
    const void* fn = dtype == GPK_F64
                         ? (tree == 3 ? reinterpret_cast<const void*>(assemble_kernel<double, 3>)
                            : tree == 2 ? reinterpret_cast<const void*>(assemble_kernel<double, 2>)
                                      : tree == 1 ? reinterpret_cast<const void*>(assemble_kernel<double, 1>)
                                                  : reinterpret_cast<const void*>(assemble_kernel<double, 0>))
                         : (tree == 2 ? reinterpret_cast<const void*>(assemble_kernel<float, 2>)
                                      : tree == 1 ? reinterpret_cast<const void*>(assemble_kernel<float, 1>)
                                                  : reinterpret_cast<const void*>(assemble_kernel<float, 0>));
    hipError_t e = ensure_dyn_lds(fn, lds);
    if (e != hipSuccess) return e;
  }
  if (dtype == GPK_F64) {
    if (tree == 3)
      hipLaunchKernelGGL((assemble_kernel<double, 3>), grid, dim3(256), lds, s, kd, a);
    else if (tree == 2)
      hipLaunchKernelGGL((assemble_kernel<double, 2>), grid, dim3(256), lds, s, kd, a);
    else if (tree == 1)
      hipLaunchKernelGGL((assemble_kernel<double, 1>), grid, dim3(256), lds, s, kd, a);
    else
      hipLaunchKernelGGL((assemble_kernel<double, 0>), grid, dim3(256), lds, s, kd, a);
  } else {
    if (tree == 2)
      hipLaunchKernelGGL((assemble_kernel<float, 2>), grid, dim3(256), lds, s, kd, a);
    else if (tree == 1)
      hipLaunchKernelGGL((assemble_kernel<float, 1>), grid, dim3(256), lds, s, kd, a);
    else
      hipLaunchKernelGGL((assemble_kernel<float, 0>), grid, dim3(256), lds, s, kd, a);
  }
  return hipGetLastError();
}

}  // namespace gpk
