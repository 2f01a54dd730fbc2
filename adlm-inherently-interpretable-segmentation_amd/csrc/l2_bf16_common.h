// l2_bf16_common.h — pieces shared by the bf16 prototype-layer kernels (l2_bf16.hip: forward,
// x-backward, pw-backward; l2_bwd_fused.hip: the one-kernel backward): the operand-image block
// layout, LDS-DMA helpers and small LDS accessors. Device code only; everything is inline.
#pragma once
#include "bf16_split.h"

namespace protoseg {
namespace bf16l {

constexpr int kC = 64;         // channels of the bf16 family
constexpr int kNQ = kC / 16;   // channel k-steps of 16

// Operand images of the prototypes and the last layer, built once per call by
// l2_prep_bf16_kernel into a global block laid out exactly as the kernels' LDS regions, so each
// workgroup fills its LDS with 16-B LDS-DMA copies (one round trip) instead of re-deriving them.
//   [P image T*Pp*128 B | W^T image T*Pp*64 | ||p||^2 (Pp floats, padded to 1 KiB) |
//    P^T image T*Pp*128 | W image T*Pp*64]      (every region a multiple of 1 KiB)
struct ImgOffsets {
  int p, wt, p2, pt, w, total;
};
__host__ __device__ inline ImgOffsets img_offsets(int Pp, int T) {
  ImgOffsets o;
  o.p = 0;
  o.wt = T * Pp * 128;
  o.p2 = o.wt + T * Pp * 64;
  o.pt = o.p2 + ((Pp * 4 + 1023) & ~1023);
  o.w = o.pt + T * Pp * 128;
  o.total = o.w + T * Pp * 64;
  return o;
}

// v[r] = rows[acc_row(r, h) - 4h] for a 16-B aligned LDS row block (4 x ds_read_b128): the
// per-row scalars of one accumulator tile, read once instead of per element.
__device__ __forceinline__ void load_rows16(const float* rows, float (&v)[16]) {
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    const float4 q = *reinterpret_cast<const float4*>(rows + 8 * g4);
    v[4 * g4] = q.x;
    v[4 * g4 + 1] = q.y;
    v[4 * g4 + 2] = q.z;
    v[4 * g4 + 3] = q.w;
  }
}

// XCD-aware workgroup index. The dispatcher deals workgroups round-robin over the 8 XCDs
// (workgroup i on XCD i % 8), each with its own L2. Workgroup i runs as virtual workgroup
// (i % 8) * (G / 8) + i / 8, so the workgroups of one XCD take neighbouring pixel tiles. A 32-pixel
// tile's NCHW rows start at any 4-B offset (65 x 65 maps), so the line two neighbouring tiles
// share is then written (and read) through one L2 instead of two (store probe: 48.2 -> 42.9 us
// for the forward's distance pattern, tools/probe/store_bw.hip). A grid that is not a multiple
// of 8 keeps the plain order (a bijection either way: only the placement changes).
#ifndef XCD_MAP
#define XCD_MAP 1
#endif
__device__ __forceinline__ int xcd_block() {
  const int G = static_cast<int>(gridDim.x), b = static_cast<int>(blockIdx.x);
  if (!XCD_MAP || (G & 7)) return b;
  return (b & 7) * (G >> 3) + (b >> 3);
}

// Wave index as a provably wave-uniform value (SGPR): threadIdx.x / 64 is uniform but the
// compiler cannot prove it, and a "divergent" LDS-DMA base or buffer soffset derived from it
// makes hipcc wrap every such memory op in a waterfall loop (cdna_hip_programming.md T20).
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6)); }

// Workgroup-wide copy of `bytes` (a multiple of 1 KiB) from global to LDS by 16-B LDS-DMA
// (global_load_lds_dwordx4: one wave-instruction moves 1 KiB, lane-linear). The caller's
// __syncthreads() waits for it.
__device__ __forceinline__ void lds_copy(void* lds, const unsigned char* src, int bytes) {
  const int lane = threadIdx.x & 63, wave = wave_id(), nw = blockDim.x >> 6;
  for (int off = wave * 1024; off < bytes; off += nw * 1024)
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(src + off + lane * 16),
        (__attribute__((address_space(3))) void*)(static_cast<unsigned char*>(lds) + off), 16, 0, 0);
}

template <int PAIR>
__device__ __forceinline__ int pair_off(int row, int col) { return (row >> 1) * PAIR + (row & 1) * 32 + col; }

__device__ __forceinline__ float lds_val(const float* p) { return *p; }
__device__ __forceinline__ float lds_val(const uint32_t* p) { return __uint_as_float(*p << 16); }
// Four consecutive elements (16-B / 8-B aligned).
__device__ __forceinline__ void lds_val4(const float* p, float* v) {
  const float4 q = *reinterpret_cast<const float4*>(p);
  v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
}
__device__ __forceinline__ void lds_val4(const uint32_t* p, float* v) {
  const uint4 q = *reinterpret_cast<const uint4*>(p);
  v[0] = __uint_as_float(q.x << 16), v[1] = __uint_as_float(q.y << 16);
  v[2] = __uint_as_float(q.z << 16), v[3] = __uint_as_float(q.w << 16);
}

// One LDS-DMA wave-instruction: lane l's element (byte offset voff + soff of the buffer) lands
// in the dword at lds + 4 l (zero-extended); out-of-range lanes land as 0.
// Written as inline asm on purpose (cdna_hip_programming.md §5.7): hipcc counts a builtin
// LDS-DMA as an LDS write of unknown extent and drains it (vmcnt(0)) before the next ds_read,
// which here would stall the compute of tile t on the prefetch of tile t+1. The kernel waits
// for its DMA itself (s_waitcnt vmcnt(0) + barrier at the top of each tile). `lds` and `soff`
// must be wave-uniform.
template <typename TX>
__device__ __forceinline__ void dma(rsrc_t r, void* lds, unsigned voff, unsigned soff) {
  const unsigned dst = static_cast<unsigned>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) void*)lds));
  unsigned so = __builtin_amdgcn_readfirstlane(soff);
  asm volatile("" : "+s"(so));  // an SGPR even when soff folds to a constant (no immediate soffset)
  unsigned keep;
  if constexpr (sizeof(TX) == 4)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dword %1, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(__builtin_amdgcn_readfirstlane(dst)), "s"(r), "s"(so)
                 : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_ushort %1, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(__builtin_amdgcn_readfirstlane(dst)), "s"(r), "s"(so)
                 : "memory");
}

// ||x||^2 of one pixel in the bf16 family's fixed order: s_{q,h} = fma chain over the 8
// channels chan_of(q, h, 0..7) starting from 0, u_q = s_{q,0} + s_{q,1}, and
// x2 = (u_0 + u_1) + (u_2 + u_3). Every kernel of the family that needs ||x||^2 (forward,
// x-backward, pw-backward, fused backward) forms exactly this value, so all of them compute
// bit-identical distances and the backward's relu mask is the forward's.
__device__ __forceinline__ float chunk_sq(const float (&v)[8]) {
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) s = fmaf(v[e], v[e], s);
  return s;
}
// Lane layout with the channel half h on lane bit 5 (layout A / per-pixel rows): s[q] = s_{q,h}.
__device__ __forceinline__ float x2_tree_halves(const float (&s)[4]) {
  float u[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) u[q] = s[q] + __shfl_xor(s[q], 32);
  return (u[0] + u[1]) + (u[2] + u[3]);
}

// n / d for 0 <= n < 2^23 and a wave-uniform d >= 1 (the family's pixel indices: bf16_sizes_ok
// keeps B H W below 2^23): a v_rcp_f32 estimate (1 ulp; the quotient estimate is within 0.75 of
// n / d), truncation and one correction step, in place of the ~25-instruction signed division
// the compiler emits for a runtime divisor. Exact, as the integer division.
__device__ __forceinline__ int div_pix(int n, int d) {
  const float r = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(__builtin_amdgcn_rcpf(static_cast<float>(d)))));
  int q = static_cast<int>(static_cast<float>(n) * r);
  const int rem = n - __mul24(q, d);
  q += rem >= d ? 1 : 0;
  q -= rem < 0 ? 1 : 0;
  return q;
}

}  // namespace bf16l
}  // namespace protoseg
