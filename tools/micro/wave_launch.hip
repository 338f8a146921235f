// Wave start spread inside a workgroup (tools/micro, A/B only): every wave
// stamps s_memrealtime (100 MHz) at entry; per config, the spread between the
// first and last wave of workgroup 0 and of the whole grid.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

__global__ void k_stamp(unsigned long long* out, int vg) {
  unsigned long long t = __builtin_amdgcn_s_memrealtime();
  __shared__ double lds[8192];
  if (vg) lds[threadIdx.x] = threadIdx.x;   // some LDS use
  const int w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if ((threadIdx.x & 63) == 0) out[w] = t + (vg ? (unsigned long long)lds[0] : 0ull);
}

int main() {
  unsigned long long* d;
  hipMalloc(&d, 1 << 22);
  for (int bs : {256, 512, 1024})
    for (int g : {1, 272}) {
      const int nw = g * bs / 64;
      std::vector<unsigned long long> h(nw);
      for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_stamp, dim3(g), dim3(bs), 0, 0, d, 1);
        hipDeviceSynchronize();
      }
      hipMemcpy(h.data(), d, nw * 8, hipMemcpyDeviceToHost);
      const int wpg = bs / 64;
      auto mm0 = std::minmax_element(h.begin(), h.begin() + wpg);
      auto mma = std::minmax_element(h.begin(), h.end());
      printf("block %4d grid %3d: WG0 wave-start spread %6.2f us, grid spread %6.2f us\n", bs, g,
             (*mm0.second - *mm0.first) * 0.01, (*mma.second - *mma.first) * 0.01);
    }
  return 0;
}
