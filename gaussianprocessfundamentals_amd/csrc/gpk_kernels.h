// Device evaluation of the kernel program (shared by the K build in gpk_assemble.hip and the
// fused first trailing update in gpk_potrf.hip).  Reference formulas: see gpk_assemble.hip.
// Multiply-adds are contracted within a source expression only (fp contract(on)): with hipcc's
// default (fast) the fusions across statements depend on the inlining context, so the K build's
// interior / edge loops and the fused build would round a few elements differently.
#pragma once

#include <math.h>

#include "gpk_internal.h"

namespace gpk {
namespace {

constexpr double SQRT3 = 1.7320508075688772;
constexpr double SQRT5 = 2.23606797749979;
constexpr double PI = 3.141592653589793;

// Values of one base node for R row points a[i] against one column point b.  The R evaluations
// are independent, so the compiler interleaves their long f64 chains (exp / sin / sqrt / div).
template <int R>
__device__ __forceinline__ void base_values(const gpk_node& nd, const double* __restrict__ hyp,
                                            const double* const (&a)[R], const double* b, int d, double (&r)[R]) {
#pragma clang fp contract(on)  // fuse within an expression only: every caller rounds alike
  const int fl = nd.flags;
  const bool ard = (fl & GPK_NODE_ARD) != 0;
  const double* h = hyp + nd.hyp_offset;
  int sg_at;
  if (nd.op == GPK_OP_SE) {
    double s[R];
    if (fl & GPK_NODE_SE_EXPANDED) {
#pragma unroll
      for (int i = 0; i < R; ++i) {
        double na = 0.0, nb = 0.0, ab = 0.0;
        for (int k = 0; k < d; ++k) {
          na += a[i][k] * a[i][k];
          nb += b[k] * b[k];
          ab += a[i][k] * b[k];
        }
        const double dist = sqrt((na - 2.0 * ab) + nb);  // NaN on a negative argument, as the reference
        s[i] = dist * dist;
      }
    } else {
#pragma unroll
      for (int i = 0; i < R; ++i) s[i] = 0.0;
      for (int k = 0; k < d; ++k) {
        const double bk = b[k];
#pragma unroll
        for (int i = 0; i < R; ++i) {
          const double t = a[i][k] - bk;
          s[i] += t * t;
        }
      }
    }
    const double l = ard ? 1.0 : h[0];
    const double l2 = l * l;
#pragma unroll
    for (int i = 0; i < R; ++i) r[i] = exp(-0.5 * (s[i] / l2));
    sg_at = ard ? d : 1;
  } else if (nd.op == GPK_OP_PER) {
    const double l = h[0], per = h[1];
    double sn[R];
    if (fl & GPK_NODE_STANDARD) {  // product of 1-D periodic kernels
#pragma unroll
      for (int i = 0; i < R; ++i) sn[i] = 0.0;
      for (int k = 0; k < d; ++k) {
#pragma unroll
        for (int i = 0; i < R; ++i) {
          const double t = sin(PI * (fabs(a[i][k] - b[k]) / per));
          sn[i] += t * t;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < R; ++i) {
        double dist = 0.0;
        for (int k = 0; k < d; ++k) dist += fabs(a[i][k] - b[k]);
        const double t = sin(PI * (dist / per));
        sn[i] = t * t;
      }
    }
#pragma unroll
    for (int i = 0; i < R; ++i) r[i] = exp((-2.0 * sn[i]) / (l * l));
    sg_at = 2;
  } else {  // MAT32 / MAT52
    double dist[R];
#pragma unroll
    for (int i = 0; i < R; ++i) dist[i] = 0.0;
    if (fl & GPK_NODE_STANDARD) {  // Euclidean distance
      for (int k = 0; k < d; ++k) {
#pragma unroll
        for (int i = 0; i < R; ++i) {
          const double t = a[i][k] - b[k];
          dist[i] += t * t;
        }
      }
#pragma unroll
      for (int i = 0; i < R; ++i) dist[i] = sqrt(dist[i]);
    } else {
      for (int k = 0; k < d; ++k) {
#pragma unroll
        for (int i = 0; i < R; ++i) dist[i] += fabs(a[i][k] - b[k]);
      }
    }
    const double l = ard ? 1.0 : fabs(h[0]);
    if (nd.op == GPK_OP_MAT52) {
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const double frac = (SQRT5 * dist[i]) / l;
        const double third = (5.0 * (dist[i] * dist[i])) / (3.0 * (l * l));
        r[i] = ((1.0 + frac) + third) * exp(-frac);
      }
    } else {
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const double frac = (SQRT3 * dist[i]) / l;
        r[i] = (1.0 + frac) * exp(-frac);
      }
    }
    sg_at = ard ? d : 1;
  }
  if (fl & GPK_NODE_SCALED) {
    const double sg = h[sg_at];
#pragma unroll
    for (int i = 0; i < R; ++i) r[i] = sg * r[i];
  }
}

__device__ __forceinline__ double base_value(const gpk_node& nd, const double* __restrict__ hyp,
                                             const double* a, const double* b, int d) {
  const double* aa[1] = {a};
  double r[1];
  base_values<1>(nd, hyp, aa, b, d, r);
  return r[0];
}

// Register stack of the postfix program.  The stack pointer is wave-uniform, so the switch
// lowers to scalar branches and nothing is indexed dynamically (no scratch).
struct Stack {
  double s0, s1, s2, s3, s4, s5, s6, s7;
  __device__ __forceinline__ double get(int i) const {
    switch (i) {
      case 0: return s0; case 1: return s1; case 2: return s2; case 3: return s3;
      case 4: return s4; case 5: return s5; case 6: return s6; default: return s7;
    }
  }
  __device__ __forceinline__ void set(int i, double v) {
    switch (i) {
      case 0: s0 = v; break; case 1: s1 = v; break; case 2: s2 = v; break; case 3: s3 = v; break;
      case 4: s4 = v; break; case 5: s5 = v; break; case 6: s6 = v; break; default: s7 = v; break;
    }
  }
};

// Single-base-node trees (the common case, e.g. every SURVEY config but C5): the node's constants
// are computed once per thread into registers and every division by a hyperparameter becomes a
// multiplication by its reciprocal (|error| <= ~1e-14 relative in K).  Multi-node trees go through
// eval_tree_fast with the same reciprocals and periodic nodes through sin2_pi, so the K build no
// longer keeps the reference's literal operation order anywhere.  The gradient kernel re-evaluates K
// with base_values (divisions, library sin): for trees its K differs from the factorised one by
// ~1e-14 relative, far inside the gradient tests' tolerances.
struct FastNode {
  int op, flags, d, off;
  double il, il2, i3l2, iper, sg;
  // periodic node through the staged sin / cos of its points (sc_node): sin(pi u), cos(pi u) per point and
  // dimension at offsets sc_sin / sc_cos from the point (tiles whose points all have |u| = |x / p| <= 4)
  int sc, sc_sin, sc_cos;
};

// The periodic node whose sin^2(pi (x_k - y_k) / p) terms the K build takes from per-point sin / cos
// (sin(a - b) = sin a cos b - cos a sin b; separable per dimension: the standard form, or D = 1 where the
// reference's L1 form is the same): the first such node of the program, -1 if none.
__host__ __device__ inline int sc_node(const gpk_kdesc& kd) {
  for (int q = 0; q < kd.n_nodes; ++q)
    if (kd.nodes[q].op == GPK_OP_PER && ((kd.nodes[q].flags & GPK_NODE_STANDARD) || kd.dim == 1)) return q;
  return -1;
}
constexpr double SC_MAX_U = 4.0;  // |x / p| bound of a tile for the sin / cos form (phase error <= 8 pi eps)

__device__ __forceinline__ int fast_off(const gpk_kdesc& kd, int slot_stride) {
  return (kd.nodes[0].flags & GPK_NODE_ARD) ? (kd.nodes[0].ard_slot + 1) * slot_stride : 0;
}

__device__ __forceinline__ FastNode make_fast_node(const gpk_node& nd, const double* hyp, int d) {
  FastNode f;
  f.op = nd.op;
  f.flags = nd.flags;
  f.d = d;
  f.off = 0;
  const double* h = hyp + nd.hyp_offset;
  const bool ard = (nd.flags & GPK_NODE_ARD) != 0;
  double l = 1.0;
  int sg_at = 1;
  if (nd.op == GPK_OP_PER) {
    l = h[0];
    f.iper = 1.0 / h[1];
    sg_at = 2;
  } else {
    l = ard ? 1.0 : (nd.op == GPK_OP_SE ? h[0] : fabs(h[0]));
    f.iper = 0.0;
    sg_at = ard ? d : 1;
  }
  f.il = 1.0 / l;
  f.il2 = 1.0 / (l * l);
  f.i3l2 = 1.0 / (3.0 * (l * l));
  f.sg = (nd.flags & GPK_NODE_SCALED) ? h[sg_at] : 1.0;
  f.sc = 0;
  f.sc_sin = f.sc_cos = 0;
  return f;
}

// sin^2 over the dimensions from per-point sin(pi u) / cos(pi u) (u = x / p, reduced by the nearest integer
// before the sincospi: the sign (-1)^n cancels in the square): sin(pi (u_a - u_b)) = s_a c_b - c_a s_b.
// Same contraction everywhere it is used (interior, generic and plain paths write the same bits).  Against the
// reference's sin(pi |x_a - x_b| / p) the phase error is eps (|u_a| + |u_b|) pi <= 8 pi eps on a tile that
// qualifies (SC_MAX_U): 3 VALU operations per dimension instead of the reduced Taylor series' ~25.
template <typename SA, typename CA, typename SB, typename CB>
__device__ __forceinline__ double per_sc_value(const FastNode& f, SA sa, CA ca, SB sb, CB cb) {
#pragma clang fp contract(on)  // fuse within an expression only: every caller rounds alike
  double sn = 0.0;
  for (int k = 0; k < f.d; ++k) {
    // sin(pi (a - b) / p) = sa cb - ca sb, the two products rounded separately (no FMA between them): swapping
    // the points swaps them exactly, so t(b, a) = -t(a, b) and K stays exactly symmetric (a contracted
    // fma(sa, cb, -ca sb) left 1-ulp asymmetries, found by tests/test_gpu_properties.py)
    const double p1 = sa(k) * cb(k);
    const double p2 = ca(k) * sb(k);
    const double t = p1 - p2;
    sn += t * t;
  }
  return f.sg * exp((-2.0 * sn) * f.il2);
}

// sin^2(pi t), t >= 0 (the periodic kernel's sin^2(pi d / p) with t = d / p).  sin^2 has period 1 in
// t, so t is reduced to its fraction (exact in floating point), folded onto [0, 1/2] by
// sin(pi g) = sin(pi (1 - g)) (1 - g exact there), and sin(pi g) is its Taylor series to x^19 on
// [0, pi/2] (truncation <= 2.6e-16): about a third of the library sin's work, with no quadrant
// branches.  The phase error of t itself, |t| ulp, is the reference formula's as well.
__device__ __forceinline__ double sin2_pi(double t) {
#pragma clang fp contract(on)  // fuse within an expression only: every caller rounds alike
  const double f = t - floor(t);
  const double g = fmin(f, 1.0 - f);
  const double x = PI * g;
  const double x2 = x * x;
  double p = -1.0 / 121645100408832000.0;     // -1/19!
  p = fma(p, x2, 1.0 / 355687428096000.0);    //  1/17!
  p = fma(p, x2, -1.0 / 1307674368000.0);     // -1/15!
  p = fma(p, x2, 1.0 / 6227020800.0);         //  1/13!
  p = fma(p, x2, -1.0 / 39916800.0);          // -1/11!
  p = fma(p, x2, 1.0 / 362880.0);             //  1/9!
  p = fma(p, x2, -1.0 / 5040.0);              // -1/7!
  p = fma(p, x2, 1.0 / 120.0);                //  1/5!
  p = fma(p, x2, -1.0 / 6.0);                 // -1/3!
  const double sv = fma(x * x2, p, x);
  return sv * sv;
}

// fast_value over coordinate accessors: a(k), b(k) return coordinate k of the two points
template <typename PA, typename PB>
__device__ __forceinline__ double fast_value_at(const FastNode& f, PA a, PB b) {
#pragma clang fp contract(on)  // fuse within an expression only: every caller rounds alike
  const int d = f.d;
  double r;
  if (f.op == GPK_OP_SE) {
    double s = 0.0;
    if (f.flags & GPK_NODE_SE_EXPANDED) {
      double na = 0.0, nb = 0.0, ab = 0.0;
      for (int k = 0; k < d; ++k) {
        na += a(k) * a(k);
        nb += b(k) * b(k);
        ab += a(k) * b(k);
      }
      const double dist = sqrt((na - 2.0 * ab) + nb);
      s = dist * dist;
    } else {
      for (int k = 0; k < d; ++k) {
        const double t = a(k) - b(k);
        s += t * t;
      }
    }
    r = exp(-0.5 * (s * f.il2));
  } else if (f.op == GPK_OP_PER) {
    double sn = 0.0;
    if (f.flags & GPK_NODE_STANDARD) {
      for (int k = 0; k < d; ++k) sn += sin2_pi(fabs(a(k) - b(k)) * f.iper);
    } else {
      double dist = 0.0;
      for (int k = 0; k < d; ++k) dist += fabs(a(k) - b(k));
      sn = sin2_pi(dist * f.iper);
    }
    r = exp((-2.0 * sn) * f.il2);
  } else {
    double dist = 0.0;
    if (f.flags & GPK_NODE_STANDARD) {
      for (int k = 0; k < d; ++k) {
        const double t = a(k) - b(k);
        dist += t * t;
      }
      dist = sqrt(dist);
    } else {
      for (int k = 0; k < d; ++k) dist += fabs(a(k) - b(k));
    }
    if (f.op == GPK_OP_MAT52) {
      const double frac = (SQRT5 * dist) * f.il;
      r = ((1.0 + frac) + (5.0 * (dist * dist)) * f.i3l2) * exp(-frac);
    } else {
      const double frac = (SQRT3 * dist) * f.il;
      r = (1.0 + frac) * exp(-frac);
    }
  }
  return f.sg * r;
}

__device__ __forceinline__ double fast_value(const FastNode& f, const double* a, const double* b, bool sc_on = false) {
  if (sc_on && f.sc && f.op == GPK_OP_PER) {
    const int so = f.sc_sin, co = f.sc_cos;
    return per_sc_value(f, [a, so](int k) { return a[so + k]; }, [a, co](int k) { return a[co + k]; },
                        [b, so](int k) { return b[so + k]; }, [b, co](int k) { return b[co + k]; });
  }
  return fast_value_at(f, [a](int k) { return a[k]; }, [b](int k) { return b[k]; });
}

// The postfix program with every base node's constants precomputed (fns[q] = make_fast_node of
// node q, fns[q].off its ARD slot offset): the tree form of the single-node fast path -- no division
// by a hyperparameter per element, the periodic nodes through sin2_pi.
__device__ __forceinline__ double eval_tree_fast(const gpk_kdesc& kd, const FastNode* fns, const double* pa,
                                                 const double* pb, bool sc_on = false) {
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
      const FastNode f = fns[q];
      st.set(sp, fast_value(f, pa + f.off, pb + f.off, sc_on));
      sp += 1;
    }
  }
  return st.s0;
}

}  // namespace
}  // namespace gpk
