#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
__global__ void k(const float* x, float* s, float* c, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x; if (i >= n) return;
  float r = x[i] * 0.15915494309189535f;
  s[i] = __builtin_amdgcn_sinf(r); c[i] = __builtin_amdgcn_cosf(r);
}
int main() {
  const int n = 1 << 20; float *x, *s, *c;
  hipMallocManaged(&x, n * 4); hipMallocManaged(&s, n * 4); hipMallocManaged(&c, n * 4);
  for (int i = 0; i < n; ++i) x[i] = -3.5f + 7.0f * i / n;
  k<<<n / 256, 256>>>(x, s, c, n); hipDeviceSynchronize();
  double es = 0, ec = 0;
  for (int i = 0; i < n; ++i) { es = fmax(es, fabs(s[i] - sin((double)x[i]))); ec = fmax(ec, fabs(c[i] - cos((double)x[i]))); }
  printf("max abs err sin %.3e cos %.3e\n", es, ec);
}
