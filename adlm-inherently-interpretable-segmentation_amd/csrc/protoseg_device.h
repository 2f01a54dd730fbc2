// protoseg_device.h — device helpers shared by the prototype-layer and push kernels (gfx950).
//
// MFMA used throughout: v_mfma_f32_32x32x2_f32 (f32 in, f32 accumulate, exact: a k-ordered
// fmaf chain, cdna_hip_programming.md §3 "FP32-input MFMA").  Lane maps (wave64):
//   A operand  lane l: A[i = l&31][k = l>>5]
//   B operand  lane l: B[k = l>>5][j = l&31]
//   C/D        lane l, reg r: col = l&31, row = acc_row(r, l>>5)
// A 32x32 tile therefore lives as: column on the lane (j), 16 rows in registers, the two
// half-waves (h = l>>5) holding interleaved row quads.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace protoseg {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kWave = 64;
constexpr int kTile = 32;

__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }
// The lane-independent part of acc_row: acc_row(r, h) = row_of(r) + 4h. Strided addresses
// are written as (lane base incl. 4h) + row_of(r) * stride so that the per-register offset
// is wave-uniform (SGPR / immediate) instead of a VGPR per register.
__device__ __forceinline__ constexpr int row_of(int r) { return (r & 3) + 8 * (r >> 2); }

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.f;
  return z;
}

// Feature-map element I/O: f32 or bf16 (uint16 bits). bf16 -> f32 is exact.
template <typename T> struct XIO;
template <> struct XIO<float> {
  static __device__ __forceinline__ float load(const float* p, size_t i) { return p[i]; }
  static __device__ __forceinline__ void store(float* p, size_t i, float v) { p[i] = v; }
};
template <> struct XIO<_Float16> {  // IEEE half (PROTOSEG_F16): exact widening, round-to-nearest-even narrowing
  static __device__ __forceinline__ float load(const _Float16* p, size_t i) { return static_cast<float>(p[i]); }
  static __device__ __forceinline__ void store(_Float16* p, size_t i, float v) { p[i] = static_cast<_Float16>(v); }
};
template <> struct XIO<uint16_t> {
  static __device__ __forceinline__ float load(const uint16_t* p, size_t i) {
    return __uint_as_float(static_cast<uint32_t>(p[i]) << 16);
  }
  static __device__ __forceinline__ void store(uint16_t* p, size_t i, float v) {
    uint32_t u = __float_as_uint(v);
    if ((u & 0x7fffffffu) > 0x7f800000u) {  // NaN stays NaN
      p[i] = static_cast<uint16_t>((u >> 16) | 0x40u);
      return;
    }
    u += 0x7fffu + ((u >> 16) & 1u);  // round to nearest even
    p[i] = static_cast<uint16_t>(u >> 16);
  }
};

// model.py:217-219: relu(x2_patch_sum + (-2 * xp + p2)); -2*xp is exact, so the
// expression below rounds exactly where the reference does.
__device__ __forceinline__ float l2_pre_relu(float x2, float p2, float xp) {
  const float inter = p2 - 2.f * xp;
  return x2 + inter;
}
__device__ __forceinline__ float l2_distance(float x2, float p2, float xp) {
  return __builtin_fmaxf(l2_pre_relu(x2, p2, xp), 0.f);  // F.relu (v_max_f32; NaN inputs are out of scope)
}

// model.py:231-237
__device__ __forceinline__ float activation(float d, float eps, int act_kind) {
  if (act_kind == 0) return logf((d + 1.f) / (d + eps));
  return -d;
}

// d activation / d d. For 'log': 1/(d+1) - 1/(d+eps) = (eps-1) / ((d+1)(d+eps)), written
// without the cancellation of the two-term form.
__device__ __forceinline__ float activation_grad(float d, float eps, int act_kind) {
  if (act_kind == 0) return (eps - 1.f) / ((d + 1.f) * (d + eps));
  return -1.f;
}

// Orders this wave's preceding LDS accesses before its following ones, for data that
// crosses lanes of the same wave (the compiler cannot see that dependency).
// A batch of guarded loads: every element is loaded through a clamped (always valid) address,
// then the batch is pinned in VGPRs before the guards select. Left alone, the compiler sinks each
// load into its guard's branch with a wait of its own: one round trip per load, not per batch.
template <int N, typename T>
__device__ __forceinline__ void pin_batch(T (&v)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(v[i]));
}

__device__ __forceinline__ void wave_lds_fence() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// Bitwise OR of a 32-bit value over the 64 lanes of the wave (result in every lane).
__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) v |= __shfl_xor(v, m);
  return v;
}

__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int m) {
  const uint32_t lo = __shfl_xor(static_cast<uint32_t>(v), m);
  const uint32_t hi = __shfl_xor(static_cast<uint32_t>(v >> 32), m);
  return (static_cast<unsigned long long>(hi) << 32) | lo;
}

}  // namespace protoseg
