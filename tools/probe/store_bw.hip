// Probe: HBM write rate of the forward's distance-store pattern, without the compute.
// Layout-A tiles: a wave owns 32 consecutive pixels (lane j = pixel, h = lane>>5) and stores,
// per prototype tile, 16 dwords per lane at rows pt*32 + row_of(r) + 4h (stride HW), i.e. two
// 128-B row segments per store instruction. Variants:
//   0 plain buffer_store_dword (as l2_fwd_bf16_kernel)
//   1 same with the nontemporal cache policy
//   2 upper bound: the same bytes as a linear dwordx4 stream
//   3 dwordx4 8-row quads; 4 variant 0 with the XCD-aware order
//   5 / 6 256-B row runs per store (64 pixels per wave), without / with the XCD order
//   7 / 8 512-B / 1-KB row runs (dwordx2 / dwordx4 per lane), XCD order
// plus a read of the same x tile per pixel tile (32 dword loads per lane) in variants 0/1.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr unsigned kOOB = 0x80000000u;
__device__ __forceinline__ int row_of(int r) { return (r & 3) + 8 * (r >> 2); }

// XCD: workgroup i runs as virtual workgroup (i % 8) * (G / 8) + i / 8, so the workgroups one XCD
// holds (dispatch is round-robin over the 8 XCDs) take one contiguous range of tiles per round
template <int POL, int XCD = 0>
__global__ __launch_bounds__(512) void dstore(const float* x, unsigned xb, float* d, unsigned db, int HW, int npix, int P,
                                              int npt, float v0) {
  const rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), (short)0, (int)xb, 0x00020000);
  const rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(d, (short)0, (int)db, 0x00020000);
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5, wave = threadIdx.x >> 6;
  const int ntiles = (npix + 31) / 32;
  const int G = gridDim.x, bid = blockIdx.x;
  const int vb = XCD ? (bid & 7) * (G >> 3) + (bid >> 3) : bid;
  for (int t = vb * 8 + wave; t < ntiles; t += gridDim.x * 8) {
    const int g = t * 32 + j;
    const bool valid = g < npix;
    const int b = valid ? g / HW : 0, n = valid ? g - b * HW : 0;
    float acc = v0;
    const unsigned xo = valid ? static_cast<unsigned>(((b * 64 + 4 * h) * HW + n) * 4) : kOOB;
#pragma unroll
    for (int q = 0; q < 32; ++q)
      acc += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rx, xo, static_cast<unsigned>((8 * (q >> 2) + (q & 3)) * HW * 4), 0));
    const unsigned dbase = valid ? static_cast<unsigned>(((b * P + 4 * h) * HW + n) * 4) : kOOB;
    for (int pt = 0; pt < npt; ++pt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = pt * 32 + row_of(r);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc + r), rd, row < P ? dbase : kOOB,
                                              static_cast<unsigned>(row * HW * 4), POL);
      }
    }
  }
}


// dwordx4 per lane: lane (h, q = j >> 3, i = j & 7) writes pixels 4i .. 4i + 3 of row 4h + q
// (+ 8 s), i.e. each store instruction covers 8 rows x 128 B (the layout a 4x4 quad transpose of
// the 32x32 accumulator gives); rows at HW stride (misaligned 16-B chunks when HW is odd)
__global__ __launch_bounds__(512) void dstore4(const float* x, unsigned xb, float* d, unsigned db, int HW, int npix, int P,
                                               int npt, float v0) {
  const rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), (short)0, (int)xb, 0x00020000);
  const rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(d, (short)0, (int)db, 0x00020000);
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5, wave = threadIdx.x >> 6;
  const int ntiles = (npix + 31) / 32;
  for (int t = blockIdx.x * 8 + wave; t < ntiles; t += gridDim.x * 8) {
    const int g = t * 32 + j;
    const bool valid = g < npix;
    const int b = valid ? g / HW : 0, n = valid ? g - b * HW : 0;
    float acc = v0;
    const unsigned xo = valid ? static_cast<unsigned>(((b * 64 + 4 * h) * HW + n) * 4) : kOOB;
#pragma unroll
    for (int q = 0; q < 32; ++q)
      acc += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rx, xo, static_cast<unsigned>((8 * (q >> 2) + (q & 3)) * HW * 4), 0));
    const int q8 = j >> 3, i8 = j & 7;
    const int g4 = t * 32 + 4 * i8;  // first pixel of the lane's chunk (tile never straddles an image here: probe)
    const int b4 = g4 / HW, n4 = g4 - b4 * HW;
    const unsigned dbase = g4 < npix ? static_cast<unsigned>(((b4 * P + 4 * h + q8) * HW + n4) * 4) : kOOB;
    typedef float f4 __attribute__((ext_vector_type(4)));
    for (int pt = 0; pt < npt; ++pt) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int row = pt * 32 + 8 * s + 4 * h + q8;
        const f4 v = {acc + s, acc, acc, acc};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), rd,
                                               row < P ? dbase : kOOB, static_cast<unsigned>((pt * 32 + 8 * s) * HW * 4), 0);
      }
    }
  }
}

// Long runs: a wave owns 64 * VEC consecutive pixels, lane l the VEC pixels from 64 * ... + l * VEC,
// and each store instruction writes one row's 256 * VEC contiguous bytes (what a permlane32 swap
// of two adjacent tiles' accumulators gives at VEC = 1); x read as in dstore (same bytes)
template <int VEC, int XCD>
__global__ __launch_bounds__(512) void dstore_run(const float* x, unsigned xb, float* d, unsigned db, int HW, int npix,
                                                  int P, int npt, float v0) {
  const rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), (short)0, (int)xb, 0x00020000);
  const rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(d, (short)0, (int)db, 0x00020000);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int units = (npix + 64 * VEC - 1) / (64 * VEC);
  const int G = gridDim.x, bid = blockIdx.x;
  const int vb = XCD ? (bid & 7) * (G >> 3) + (bid >> 3) : bid;
  for (int t = vb * 8 + wave; t < units; t += G * 8) {
    const int g = t * 64 * VEC + lane * VEC;
    const bool valid = g < npix;
    const int b = valid ? g / HW : 0, n = valid ? g - b * HW : 0;
    float acc = v0;
    const unsigned xo = valid ? static_cast<unsigned>((b * 64 * HW + n) * 4) : kOOB;
#pragma unroll
    for (int q = 0; q < 64 * VEC; q += 2 * VEC)  // 32 * VEC dword loads per lane = the same x bytes
      acc += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rx, xo, static_cast<unsigned>((q >> VEC) * HW * 4), 0));
    const unsigned dbase = valid ? static_cast<unsigned>((b * P * HW + n) * 4) : kOOB;
    for (int pt = 0; pt < npt; ++pt) {
#pragma unroll 8
      for (int r = 0; r < 32; ++r) {
        const int row = pt * 32 + r;
        if constexpr (VEC == 1) {
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc + r), rd, row < P ? dbase : kOOB,
                                                static_cast<unsigned>(row * HW * 4), 0);
        } else if constexpr (VEC == 2) {
          typedef unsigned u2 __attribute__((ext_vector_type(2)));
          const u2 v = {__float_as_uint(acc + r), __float_as_uint(acc)};
          __builtin_amdgcn_raw_buffer_store_b64(v, rd, row < P ? dbase : kOOB, static_cast<unsigned>(row * HW * 4), 0);
        } else {
          typedef unsigned u4 __attribute__((ext_vector_type(4)));
          const u4 v = {__float_as_uint(acc + r), __float_as_uint(acc), __float_as_uint(acc), __float_as_uint(acc)};
          __builtin_amdgcn_raw_buffer_store_b128(v, rd, row < P ? dbase : kOOB, static_cast<unsigned>(row * HW * 4), 0);
        }
      }
    }
  }
}

__global__ __launch_bounds__(512) void linear(float4* d, size_t n4, float v0) {
  for (size_t i = blockIdx.x * 512ull + threadIdx.x; i < n4; i += gridDim.x * 512ull) d[i] = make_float4(v0, v0, v0, v0);
}

#include <cstdlib>
int main(int argc, char** argv) {
  const int B = 32, HW = argc > 1 ? atoi(argv[1]) : 65 * 65, P = argc > 2 ? atoi(argv[2]) : 190, npt = (P + 31) / 32;
  printf("HW %d P %d\n", HW, P);
  const int npix = B * HW;
  const size_t dn = static_cast<size_t>(npix) * P, xn = static_cast<size_t>(npix) * 64;
  float *d, *x;
  hipMalloc(&d, dn * 4);
  hipMalloc(&x, xn * 4);
  hipMemset(x, 0, xn * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int grids[] = {256, 512, 1024};
  for (int gi = 0; gi < 3; ++gi) {
    for (int v = 0; v < 9; ++v) {
      float best = 1e9f;
      for (int rep = 0; rep < 20; ++rep) {
        hipEventRecord(a);
        if (v == 0)
          hipLaunchKernelGGL(dstore<0>, dim3(grids[gi]), dim3(512), 0, 0, x, (unsigned)(xn * 4), d, (unsigned)(dn * 4), HW,
                             npix, P, npt, 1.f);
        else if (v == 1)
          hipLaunchKernelGGL(dstore<2>, dim3(grids[gi]), dim3(512), 0, 0, x, (unsigned)(xn * 4), d, (unsigned)(dn * 4), HW,
                             npix, P, npt, 1.f);
        else if (v == 4)
          hipLaunchKernelGGL((dstore<0, 1>), dim3(grids[gi]), dim3(512), 0, 0, x, (unsigned)(xn * 4), d, (unsigned)(dn * 4),
                             HW, npix, P, npt, 1.f);
        else if (v == 5)
          hipLaunchKernelGGL((dstore_run<1, 0>), dim3(grids[gi]), dim3(512), 0, 0, x, (unsigned)(xn * 4), d,
                             (unsigned)(dn * 4), HW, npix, P, npt, 1.f);
        else if (v == 6)
          hipLaunchKernelGGL((dstore_run<1, 1>), dim3(grids[gi]), dim3(512), 0, 0, x, (unsigned)(xn * 4), d,
                             (unsigned)(dn * 4), HW, npix, P, npt, 1.f);
        else if (v == 7)
          hipLaunchKernelGGL((dstore_run<2, 1>), dim3(grids[gi]), dim3(512), 0, 0, x, (unsigned)(xn * 4), d,
                             (unsigned)(dn * 4), HW, npix, P, npt, 1.f);
        else if (v == 8)
          hipLaunchKernelGGL((dstore_run<4, 1>), dim3(grids[gi]), dim3(512), 0, 0, x, (unsigned)(xn * 4), d,
                             (unsigned)(dn * 4), HW, npix, P, npt, 1.f);
        else if (v == 3)
          hipLaunchKernelGGL(dstore4, dim3(grids[gi]), dim3(512), 0, 0, x, (unsigned)(xn * 4), d, (unsigned)(dn * 4), HW,
                             npix, P, npt, 1.f);
        else
          hipLaunchKernelGGL(linear, dim3(grids[gi]), dim3(512), 0, 0, reinterpret_cast<float4*>(d), dn / 4, 1.f);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      const double bytes = dn * 4.0 + (v != 2 ? xn * 4.0 : 0.0);
      printf("grid %4d variant %d: %7.1f us  %6.2f TB/s (%.1f MB)\n", grids[gi], v, best * 1e3, bytes / (best * 1e-3) / 1e12,
             bytes / 1e6);
    }
  }
  return 0;
}
