// What v_cvt_pk_u8_f32 does outside [0, 255] and with fractions (gfx950):
// saturation decides whether the float kernel needs its v_med3_f32 clamp.
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench/cvt_pk_u8.hip -o /tmp/cvt_pk_u8
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

__global__ void k(const float* in, unsigned* out, int n) {
  const int i = threadIdx.x;
  if (i < n) out[i] = __builtin_amdgcn_cvt_pk_u8_f32(in[i], 0, 0u);
}

int main() {
  const float v[] = {-1e9f, -300.f, -5.f, -1.f, -0.5f, -0.0f, 0.f,  0.4f,   0.5f,  0.6f,  1.5f,  2.5f,
                     127.5f, 254.4f, 254.5f, 254.6f, 255.f, 255.4f, 255.5f, 256.f, 300.f, 1e9f, NAN, INFINITY};
  const int n = sizeof(v) / sizeof(v[0]);
  float* din;
  unsigned* dout;
  unsigned h[64];
  if (hipMalloc(&din, sizeof(v)) != hipSuccess || hipMalloc(&dout, n * 4) != hipSuccess) return 1;
  if (hipMemcpy(din, v, sizeof(v), hipMemcpyHostToDevice) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, din, dout, n);
  if (hipMemcpy(h, dout, n * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int i = 0; i < n; ++i) printf("%12g -> %u\n", v[i], h[i] & 0xff);
  return 0;
}
