// Dependent-latency probe (one wave): cycles (s_memtime) per instruction for chains of f64 VALU ops, the
// f64 rsq, 64-bit DPP moves, v_readlane round trips and LDS write->read round trips.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

__global__ void probe(double* out, double seed, unsigned long long* cyc) {
  __shared__ double lds[64];
  double a = seed + threadIdx.x * 1e-3, b = 1.0000001, c = 1e-9;
  unsigned long long t0, t1;
  // 1 fma chain
  t0 = __builtin_amdgcn_s_memtime();
  REP64(asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));)
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
  // 2 mul chain
  t0 = __builtin_amdgcn_s_memtime();
  REP64(asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a) : "v"(b));)
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[1] = t1 - t0;
  // 3 rsq chain (abs keeps it defined)
  t0 = __builtin_amdgcn_s_memtime();
  REP64(asm volatile("v_rsq_f64 %0, |%0|" : "+v"(a));)
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[2] = t1 - t0;
  // 4 dpp mov chain (with the two wait states)
  t0 = __builtin_amdgcn_s_memtime();
  REP64(asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %0 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(a));)
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[3] = t1 - t0;
  // 5 readlane -> fma (sgpr operand) chain
  t0 = __builtin_amdgcn_s_memtime();
  int iv = (int)threadIdx.x;
  REP64(asm volatile("v_readlane_b32 s40, %0, 5\n\tv_add_u32 %0, s40, %0" : "+v"(iv) : : "s40");)
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[4] = t1 - t0;
  // 6 LDS write -> read round trip chain
  t0 = __builtin_amdgcn_s_memtime();
  const unsigned addr = (unsigned)(size_t)(lds + (threadIdx.x & 15));
  REP64(asm volatile("ds_write_b64 %1, %0\n\ts_waitcnt lgkmcnt(0)\n\tds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "+v"(a) : "v"(addr) : "memory");)
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[5] = t1 - t0;
  // 7 independent fma throughput (8 accumulators)
  double q0 = a, q1 = a + 1, q2 = a + 2, q3 = a + 3, q4 = a + 4, q5 = a + 5, q6 = a + 6, q7 = a + 7;
  t0 = __builtin_amdgcn_s_memtime();
  REP8(asm volatile("v_fma_f64 %0, %0, %8, %9\n\tv_fma_f64 %1, %1, %8, %9\n\tv_fma_f64 %2, %2, %8, %9\n\tv_fma_f64 %3, %3, %8, %9\n\t"
                    "v_fma_f64 %4, %4, %8, %9\n\tv_fma_f64 %5, %5, %8, %9\n\tv_fma_f64 %6, %6, %8, %9\n\tv_fma_f64 %7, %7, %8, %9"
                    : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3), "+v"(q4), "+v"(q5), "+v"(q6), "+v"(q7) : "v"(b), "v"(c));)
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[6] = t1 - t0;
  // 9 independent DPP64 fmac (8 accumulators, s_nop 1 each)
  t0 = __builtin_amdgcn_s_memtime();
  REP8(asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %8, %9 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
                    "s_nop 1\n\tv_fmac_f64_dpp %1, %8, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
                    "s_nop 1\n\tv_fmac_f64_dpp %2, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                    "s_nop 1\n\tv_fmac_f64_dpp %3, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
                    "s_nop 1\n\tv_fmac_f64_dpp %4, %8, %9 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
                    "s_nop 1\n\tv_fmac_f64_dpp %5, %8, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
                    "s_nop 1\n\tv_fmac_f64_dpp %6, %8, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
                    "s_nop 1\n\tv_fmac_f64_dpp %7, %8, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf"
                    : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3), "+v"(q4), "+v"(q5), "+v"(q6), "+v"(q7) : "v"(b), "v"(c));)
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[8] = t1 - t0;
  // 10 independent DPP64 fmac without the nops
  t0 = __builtin_amdgcn_s_memtime();
  REP8(asm volatile("v_fmac_f64_dpp %0, %8, %9 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
                    "v_fmac_f64_dpp %1, %8, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
                    "v_fmac_f64_dpp %2, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                    "v_fmac_f64_dpp %3, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
                    "v_fmac_f64_dpp %4, %8, %9 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
                    "v_fmac_f64_dpp %5, %8, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
                    "v_fmac_f64_dpp %6, %8, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
                    "v_fmac_f64_dpp %7, %8, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf"
                    : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3), "+v"(q4), "+v"(q5), "+v"(q6), "+v"(q7) : "v"(b), "v"(c));)
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[9] = t1 - t0;
  // 11 independent readlanes (64, into 8 SGPRs)
  t0 = __builtin_amdgcn_s_memtime();
  REP8(asm volatile("v_readlane_b32 s40, %0, 1\n\tv_readlane_b32 s41, %0, 2\n\tv_readlane_b32 s42, %0, 3\n\tv_readlane_b32 s43, %0, 4\n\t"
                    "v_readlane_b32 s44, %0, 5\n\tv_readlane_b32 s45, %0, 6\n\tv_readlane_b32 s46, %0, 7\n\tv_readlane_b32 s47, %0, 8"
                    : : "v"(iv) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");)
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[10] = t1 - t0;
  // 12 independent f64 fma with an SGPR operand (8 accumulators)
  t0 = __builtin_amdgcn_s_memtime();
  REP8(asm volatile("v_fma_f64 %0, %0, s[40:41], %8\n\tv_fma_f64 %1, %1, s[40:41], %8\n\tv_fma_f64 %2, %2, s[42:43], %8\n\tv_fma_f64 %3, %3, s[42:43], %8\n\t"
                    "v_fma_f64 %4, %4, s[44:45], %8\n\tv_fma_f64 %5, %5, s[44:45], %8\n\tv_fma_f64 %6, %6, s[46:47], %8\n\tv_fma_f64 %7, %7, s[46:47], %8"
                    : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3), "+v"(q4), "+v"(q5), "+v"(q6), "+v"(q7) : "v"(c) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");)
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[11] = t1 - t0;
  // 13 dependent f64 MFMA 16x16x4 (accumulator chain), 14 independent (4 accumulators)
  typedef double d4 __attribute__((ext_vector_type(4)));
  d4 m0 = {a, a, a, a}, m1 = m0, m2 = m0, m3 = m0;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 64; ++i) m0 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, c, m0, 0, 0, 0);
  asm volatile("s_nop 7" ::: "memory");
  const double dep = m0[0];
  asm volatile("" ::"v"(dep));
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[12] = t1 - t0;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 16; ++i) {
    m0 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, c, m0, 0, 0, 0);
    m1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, c, m1, 0, 0, 0);
    m2 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, c, m2, 0, 0, 0);
    m3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, c, m3, 0, 0, 0);
  }
  const double dep2 = m0[0] + m1[1] + m2[2] + m3[3];
  asm volatile("" ::"v"(dep2));
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[13] = t1 - t0;
  a += dep + dep2;
  // 8 s_memtime back to back
  t0 = __builtin_amdgcn_s_memtime();
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[7] = t1 - t0;
  out[threadIdx.x] = iv + a + q0 + q1 + q2 + q3 + q4 + q5 + q6 + q7;
}

int main() {
  double* out;
  unsigned long long* cyc;
  (void)hipMalloc(&out, 64 * sizeof(double));
  (void)hipMalloc(&cyc, 16 * sizeof(unsigned long long));
  unsigned long long h[16];
  for (int it = 0; it < 3; ++it) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, out, 1.5, cyc);
    (void)hipMemcpy(h, cyc, 14 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  }
  const char* nm[8] = {"fma f64 dep", "mul f64 dep", "rsq f64 dep", "dpp64 mov dep (+s_nop 1)", "readlane + add_u32 dep",
                       "lds write+read dep", "fma f64 indep (64 instr)", "memtime overhead"};
  for (int i = 0; i < 7; ++i) printf("%-28s %6.1f cycles per step\n", nm[i], (double)h[i] / 64.0);
  const char* nm2[4] = {"fmac dpp64 indep (+s_nop 1)", "fmac dpp64 indep", "readlane indep", "fma f64 sgpr indep"};
  for (int i = 0; i < 4; ++i) printf("%-28s %6.1f cycles per instr\n", nm2[i], (double)h[8 + i] / 64.0);
  printf("%-28s %6.1f cycles per instr\n", "mfma f64 16x16x4 dep", (double)h[12] / 64.0);
  printf("%-28s %6.1f cycles per instr\n", "mfma f64 16x16x4 indep", (double)h[13] / 64.0);
  printf("%-28s %6llu cycles\n", nm[7], h[7]);
  return 0;
}
