// Cost of a barrier among the workgroups of ONE XCD (same L2), for a
// per-XCD persistent coarse tail: arrive = one L2 atomic per workgroup (after
// s_waitcnt: its stores are in L2), wait = polling loads that bypass the
// vector L1 (sc0), then the vector L1 invalidated (buffer_inv sc0) so later
// loads see the other CUs' stores.  Also checks the workgroup -> XCD map
// (HW_REG_XCC_ID) and times back-to-back empty launches for comparison.
// Build: hipcc --offload-arch=gfx950 -O3 xcd_barrier.hip -o xcd_barrier
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ unsigned long long load_l2(const unsigned long long* p) {
  unsigned long long v;
  asm volatile("global_load_dwordx2 %0, %1, off sc0\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return v;
}

__global__ __launch_bounds__(256) void k_bar(unsigned long long* bar, int rounds, int* xcc, int* err,
                                             long long* t, int* data) {
  const int x = blockIdx.x % 8, j = blockIdx.x / 8, G = gridDim.x / 8;
  if (threadIdx.x == 0) xcc[blockIdx.x] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11)) & 15;
  unsigned long long* b = bar + 16 * x;
  const long long t0 = clock64();
  int bad = 0;
  for (int r = 0; r < rounds; ++r) {
    // each workgroup writes a value the next round's neighbour reads
    if (threadIdx.x == 0) data[x * 4096 + j] = r;
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_s_waitcnt(0);
      __hip_atomic_fetch_add(b, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const unsigned long long target = (unsigned long long)(r + 1) * G;
      long it = 0;
      while (load_l2(b) < target && *(volatile int*)err == 0) {
        __builtin_amdgcn_s_sleep(1);
        if (++it > (1l << 20)) {   // ~1 s: a workgroup is not resident; give up everywhere
          *(volatile int*)err = 1;
          break;
        }
      }
      asm volatile("buffer_inv sc0" ::: "memory");
    }
    __syncthreads();
    if (threadIdx.x == 0 && data[x * 4096 + (j + 1) % G] != r) bad = 1;
  }
  const long long t1 = clock64();
  if (threadIdx.x == 0) {
    t[blockIdx.x] = t1 - t0;
    if (bad) atomicAdd(err + 1, 1);
  }
}

__global__ void k_empty(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 1 << 30) *p = 1;
}

int main() {
  const int G = 32, rounds = 200, nwg = 8 * G;
  unsigned long long* bar;
  int *xcc, *err, *data;
  long long* t;
  hipMalloc(&bar, 8 * 16 * 8);
  hipMalloc(&xcc, nwg * 4);
  hipMalloc(&err, 8);
  hipMalloc(&t, nwg * 8);
  hipMalloc(&data, 8 * 4096 * 4);
  hipMemset(bar, 0, 8 * 16 * 8);
  hipMemset(err, 0, 8);
  hipMemset(data, 0xff, 8 * 4096 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_bar, dim3(nwg), dim3(256), 0, 0, bar, rounds, xcc, err, t, data);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<int> hx(nwg), he(2);
  std::vector<long long> ht(nwg);
  hipMemcpy(hx.data(), xcc, nwg * 4, hipMemcpyDeviceToHost);
  hipMemcpy(he.data(), err, 8, hipMemcpyDeviceToHost);
  hipMemcpy(ht.data(), t, nwg * 8, hipMemcpyDeviceToHost);
  int mism = 0;
  for (int i = 0; i < nwg; ++i) mism += hx[i] != i % 8;
  double tm = 0;
  for (long long v : ht) tm = tm > (double)v ? tm : (double)v;
  printf("per-XCD barrier: %d XCDs x %d workgroups, %d rounds: %.3f ms total, %.2f us per round (wall), "
         "%.0f clock64 per round (slowest wg)\n", 8, G, rounds, ms, 1000.0 * ms / rounds, tm / rounds);
  printf("workgroups off the XCD b %% 8: %d of %d; timeout %d; stale reads %d\n", mism, nwg, he[0], he[1]);
  // back-to-back empty launches
  hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, 0, nullptr);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, 0, nullptr);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  hipEventElapsedTime(&ms, e0, e1);
  printf("empty kernel, 256 workgroups, back to back: %.2f us per launch\n", 1000.0 * ms / 200);
  return 0;
}
