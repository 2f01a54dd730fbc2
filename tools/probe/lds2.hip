// Probe: where does buffer_load_ushort ... lds place each lane's 2 bytes?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const unsigned short* x, unsigned short* out) {
  __shared__ unsigned short s[256];
  for (int i = threadIdx.x; i < 256; i += 64) s[i] = 0xEEEE;
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(x), (short)0, 512, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)s, 2, threadIdx.x * 2, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += 64) out[i] = s[i];
}
int main() {
  unsigned short h[256], *dx, *dout;
  for (int i = 0; i < 256; ++i) h[i] = 0x1000 + i;
  hipMalloc(&dx, 512); hipMalloc(&dout, 512);
  hipMemcpy(dx, h, 512, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dx, dout);
  hipMemcpy(h, dout, 512, hipMemcpyDeviceToHost);
  for (int i = 0; i < 160; ++i) printf("%04x%c", h[i], i % 16 == 15 ? '\n' : ' ');
  return 0;
}
