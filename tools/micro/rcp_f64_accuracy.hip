// Accuracy of v_rcp_f64 (__builtin_amdgcn_rcp) against the correctly rounded
// 1/x, and of one / two Newton steps (rcp_nr in dwhmc_device.h uses two):
// max |r - 1/x| in ulps of 1/x over random x with spread exponents.
// Build: hipcc --offload-arch=gfx950 -O3 rcp_f64_accuracy.hip -o rcp_f64_accuracy
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

__global__ void k_rcp(const double* x, double* r0, double* r1, double* r2, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double d = x[i];
  double r = __builtin_amdgcn_rcp(d);
  r0[i] = r;
  r = fma(r, fma(-d, r, 1.0), r);
  r1[i] = r;
  r = fma(r, fma(-d, r, 1.0), r);
  r2[i] = r;
}

static double ulps(double a, double ref) {
  int64_t ia, ib;
  std::memcpy(&ia, &a, 8);
  std::memcpy(&ib, &ref, 8);
  return (double)std::llabs(ia - ib);
}

int main() {
  const int n = 1 << 22;
  std::vector<double> h(n);
  uint64_t s = 0x1234567u;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    const double m = 1.0 + (double)(s >> 11) * 0x1.0p-53;   // [1, 2)
    const int e = (int)((s >> 3) % 120) - 60;
    h[i] = std::ldexp(m, e) * ((s & 1) ? -1.0 : 1.0);
  }
  double *x, *r0, *r1, *r2;
  hipMalloc(&x, n * 8);
  hipMalloc(&r0, n * 8);
  hipMalloc(&r1, n * 8);
  hipMalloc(&r2, n * 8);
  hipMemcpy(x, h.data(), n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_rcp, dim3(n / 256), dim3(256), 0, 0, x, r0, r1, r2, n);
  std::vector<double> a(n), b(n), c(n);
  hipMemcpy(a.data(), r0, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(b.data(), r1, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(c.data(), r2, n * 8, hipMemcpyDeviceToHost);
  double m0 = 0, m1 = 0, m2 = 0;
  int64_t e0 = 0, e1 = 0, e2 = 0;
  for (int i = 0; i < n; ++i) {
    const double ref = 1.0 / h[i];
    const double u0 = ulps(a[i], ref), u1 = ulps(b[i], ref), u2 = ulps(c[i], ref);
    m0 = std::fmax(m0, u0);
    m1 = std::fmax(m1, u1);
    m2 = std::fmax(m2, u2);
    e0 += u0 != 0;
    e1 += u1 != 0;
    e2 += u2 != 0;
  }
  printf("x: %d values, |x| in [2^-60, 2^60)\n", n);
  printf("v_rcp_f64          max %.0f ulp, not correctly rounded %.4f\n", m0, (double)e0 / n);
  printf("+ 1 Newton step    max %.0f ulp, not correctly rounded %.4f\n", m1, (double)e1 / n);
  printf("+ 2 Newton steps   max %.0f ulp, not correctly rounded %.4f\n", m2, (double)e2 / n);
  return 0;
}
