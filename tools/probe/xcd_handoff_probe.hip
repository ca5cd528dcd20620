// Hand-off probe (round 6, DESIGN §12.5 item 1 "XCD-local chain tasks"): what does one producer -> consumer
// hand-off of a chain task's operands cost when both workgroups sit on the same XCD (shared L2) versus on two
// different XCDs?  The producer (workgroup 0, 8 waves) stores 96 KB (an S task's operand volume) the way
// chain_kernel does -- write-through (sc1 = agent-scope) stores, vmcnt(0), barrier, one relaxed agent-scope flag
// store -- or with plain stores and an agent release (buffer_wbl2 sc1) instead.  The consumer polls the flag
// (agent-scope loads), takes an agent acquire (buffer_inv sc1) or none, and loads the 96 KB with plain 16-B loads.
// Stamps (s_memrealtime, 100 MHz): producer store start / drained / flag set, consumer flag seen / data loaded /
// data loaded again.  Workgroup -> XCD from the XCC_ID hardware register.
//
//   hipcc --offload-arch=gfx950 -O3 tools/probe/xcd_handoff_probe.hip -o tools/probe/xcd_handoff_probe
//   tools/probe/xcd_handoff_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

typedef __attribute__((address_space(1))) int gi32;
constexpr int NWG = 64, DT = 512, NDBL = 12288;  // 96 KB

__device__ __forceinline__ unsigned xcc_id() {
  // HW_REG_XCC_ID (id 20), bits 3:0
  return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xf;
}

__global__ __launch_bounds__(DT) void probe(double* buf, int* flag, unsigned long long* st, unsigned* xcc,
                                            int consumer, int mode, double* sink) {
  const int tid = threadIdx.x, wg = blockIdx.x;
  if (tid == 0) xcc[wg] = xcc_id();
  __shared__ double red[DT];
  if (wg == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = tid; i < NDBL; i += DT) {
      const double v = (double)(i + 1) * 0.5 + (double)mode;
      if (mode & 1)
        buf[i] = v;  // plain store (released below)
      else
        __hip_atomic_store(buf + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1 store
    }
    if (mode & 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) {
      __hip_atomic_store((gi32*)flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      st[0] = t0;
      st[1] = t1;
      st[2] = __builtin_amdgcn_s_memrealtime();
    }
  } else if (wg == consumer) {
    __shared__ unsigned long long seen;
    if (tid < 64) {
      while (__builtin_amdgcn_readfirstlane(__hip_atomic_load((gi32*)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0)
        __builtin_amdgcn_s_sleep(1);
      if (!(mode & 2)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      if (tid == 0) seen = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    typedef double d2 __attribute__((ext_vector_type(2)));
    double s = 0.0;
    for (int pass = 0; pass < 2; ++pass) {
      const d2* p = reinterpret_cast<const d2*>(buf);
      d2 v[12];
#pragma unroll
      for (int i = 0; i < 12; ++i) v[i] = p[tid + i * DT];
#pragma unroll
      for (int i = 0; i < 12; ++i) s += v[i][0] + v[i][1];
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) st[4 + pass] = __builtin_amdgcn_s_memrealtime();
    }
    red[tid] = s;
    __syncthreads();
    if (tid == 0) {
      double t = 0.0;
      for (int i = 0; i < DT; ++i) t += red[i];
      sink[0] = t;
      st[3] = seen;
    }
  }
}

int main() {
  double *buf, *sink;
  int* flag;
  unsigned long long* st;
  unsigned* xcc;
  hipMalloc(&buf, NDBL * sizeof(double));
  hipMalloc(&sink, sizeof(double));
  hipMalloc(&flag, sizeof(int));
  hipMalloc(&st, 8 * sizeof(unsigned long long));
  hipMalloc(&xcc, NWG * sizeof(unsigned));
  std::vector<unsigned> hx(NWG);
  const char* mname[4] = {"sc1 stores + acquire", "plain stores + release + acquire", "sc1 stores, no acquire",
                          "plain + release, no acquire"};
  for (int mode = 0; mode < 4; ++mode) {
    for (int consumer : {8, 16, 1, 2, 3}) {
      std::vector<double> hand, load1, load2, drain;
      for (int rep = 0; rep < 25; ++rep) {
        hipMemset(flag, 0, sizeof(int));
        hipMemset(buf, 0, NDBL * sizeof(double));
        hipLaunchKernelGGL(probe, dim3(NWG), dim3(DT), 0, 0, buf, flag, st, xcc, consumer, mode, sink);
        unsigned long long h[8];
        hipMemcpy(h, st, sizeof(h), hipMemcpyDeviceToHost);
        hipMemcpy(hx.data(), xcc, NWG * sizeof(unsigned), hipMemcpyDeviceToHost);
        double chk = 0.0;
        hipMemcpy(&chk, sink, sizeof(double), hipMemcpyDeviceToHost);
        double exp = 0.0;
        for (int i = 0; i < NDBL; ++i) exp += (double)(i + 1) * 0.5 + (double)mode;
        if (chk != 2.0 * exp && rep == 0) printf("  (mode %d consumer %d: checksum %.6g vs %.6g)\n", mode, consumer, chk, 2 * exp);
        drain.push_back((h[1] - h[0]) * 10.0);
        hand.push_back(((long long)h[3] - (long long)h[2]) * 10.0);
        load1.push_back((h[4] - h[3]) * 10.0);
        load2.push_back((h[5] - h[4]) * 10.0);
      }
      auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
      printf("%-34s producer xcc %u consumer wg %2d xcc %u: store+drain %6.0f ns, flag->seen %6.0f ns, "
             "load 96KB %6.0f ns, again %6.0f ns\n", mname[mode], hx[0], consumer, hx[consumer], med(drain), med(hand),
             med(load1), med(load2));
    }
  }
  return 0;
}
