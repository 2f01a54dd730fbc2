// Probe: what does buffer_load_dword ... lds write to LDS for out-of-range lanes?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const float* x, unsigned bytes, float* out) {
  __shared__ float s[64];
  s[threadIdx.x] = 7.0f;
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), (short)0, (int)bytes, 0x00020000);
  const unsigned voff = threadIdx.x < 48 ? threadIdx.x * 4 : 0x80000000u;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)s, 4, voff, 0, 0, 0);
  __syncthreads();
  out[threadIdx.x] = s[threadIdx.x];
}
int main() {
  float h[64], *dx, *dout;
  for (int i = 0; i < 64; ++i) h[i] = 100.f + i;
  hipMalloc(&dx, 256); hipMalloc(&dout, 256);
  hipMemcpy(dx, h, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dx, 32 * 4, dout);  // 32 in range, 16 beyond bytes, 16 kOOB
  hipMemcpy(h, dout, 256, hipMemcpyDeviceToHost);
  for (int i = 0; i < 64; ++i) printf("%g%c", h[i], i % 16 == 15 ? '\n' : ' ');
  return 0;
}
