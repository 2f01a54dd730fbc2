// bf16_split.h — exact-ish f32 products on bf16 MFMA (v_mfma_f32_32x32x16_bf16) by operand
// splitting, plus the XOR-swizzled LDS image helpers shared by the bf16 kernels.
//
// A float v is split into T bf16 terms v = t0 + t1 (+ t2) + e with |e| <= 2^-8T |v| (each
// subtraction below is exact in f32). A product a*b is then the sum of the T(T+1)/2 largest
// cross terms, accumulated in f32 by the MFMA:
//   T = 2: a0b1 + a1b0 + a0b0              (3 MFMAs; |rel err| ~ 3*2^-16 per product)
//   T = 3: a1b1 + a2b0 + a0b2 + a1b0 + a0b1 + a0b0   (6 MFMAs; f32-class accuracy)
// (smallest terms first). At 16x the f32-MFMA rate this is 5.3x / 2.7x cheaper than
// v_mfma_f32_32x32x2_f32 for the same products.
//
// MFMA 32x32x16 bf16 lane maps (cdna_hip_programming.md §3): lane l, h = l>>5:
//   A: A[i = l&31][k = 8h + jj], jj = 0..7 (one 16-B fragment per lane)
//   B: B[k = 8h + jj][j = l&31]
//   C/D: same as every 32x32 shape: col = l&31, row = acc_row(r, h)
// An accumulator used as the next B operand (or A operand, transposed product) supplies,
// for k-step s (s = 0, 1 over the tile's 32 rows), registers 8s..8s+7: element jj of half h
// is row 16s + 8(jj>>2) + 4h + (jj&3) — perm_row(). The other operand must follow it.
#pragma once
#include "protoseg_device.h"

namespace protoseg {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16;

__device__ __forceinline__ f32x16 mfma_bf16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// v -> T bf16 terms, most significant first.
template <int T>
__device__ __forceinline__ void split_terms(float v, bf16 (&t)[T]) {
  float rest = v;
#pragma unroll
  for (int i = 0; i < T; ++i) {
    t[i] = static_cast<bf16>(rest);
    rest = rest - static_cast<float>(t[i]);
  }
}

// 8 floats -> T packed fragments.
template <int T>
__device__ __forceinline__ void split8(const float (&v)[8], bf16x8 (&out)[T]) {
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) {
    bf16 t[T];
    split_terms<T>(v[jj], t);
#pragma unroll
    for (int i = 0; i < T; ++i) out[i][jj] = t[i];
  }
}

template <int T>
__device__ __forceinline__ f32x16 mma_split(const bf16x8 (&a)[T], const bf16x8 (&b)[T], f32x16 acc) {
  if constexpr (T == 1) {
    acc = mfma_bf16(a[0], b[0], acc);
  } else if constexpr (T == 2) {
    acc = mfma_bf16(a[0], b[1], acc);
    acc = mfma_bf16(a[1], b[0], acc);
    acc = mfma_bf16(a[0], b[0], acc);
  } else {
    acc = mfma_bf16(a[1], b[1], acc);
    acc = mfma_bf16(a[2], b[0], acc);
    acc = mfma_bf16(a[0], b[2], acc);
    acc = mfma_bf16(a[1], b[0], acc);
    acc = mfma_bf16(a[0], b[1], acc);
    acc = mfma_bf16(a[0], b[0], acc);
  }
  return acc;
}

// Row of element jj (half h, k-step s) when a 32x32 accumulator is used as an operand.
__device__ __forceinline__ constexpr int perm_row(int s, int h, int jj) {
  return 16 * s + 8 * (jj >> 2) + 4 * h + (jj & 3);
}
// Storage position e (0..31) of a permuted 32-element row -> logical index.
__device__ __forceinline__ constexpr int perm_of(int e) { return perm_row(e >> 4, (e >> 3) & 1, e & 7); }

// Accumulator registers 8s..8s+7 split into T operand fragments.
template <int T>
__device__ __forceinline__ void acc_operand(const f32x16& acc, int s, bf16x8 (&out)[T]) {
  float v[8];
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) v[jj] = acc[8 * s + jj];
  split8<T>(v, out);
}

// XOR swizzle of the 16-B chunk index for an LDS image whose rows hold CPR chunks, making
// ds_read_b128 of 16 different rows at the same logical chunk conflict-free (the four
// 16-lane groups of ds_read_b128, MI355X_MICROARCH.md §LDS).
// CPR 8 (128-B rows, two per 256-B bank period): every ds_read_b128 group holds all 8 even and
// all 8 odd row residues mod 16, so the swizzle must permute 0..7 over each; it is also read
// transposed (ds_read_b64_tr_b16: 4 rows p0..p0+3, p0 = 0 mod 4, 4 chunks per 32-lane half),
// which needs rows p0 and p0+2 (both in one bank half) in disjoint aligned chunk quads, i.e.
// swz(p0) ^ swz(p0+2) with bit 2 set. ((row>>1)&1)<<2 | ((row>>2)&3) does both.
template <int CPR>
__device__ __forceinline__ constexpr int swz(int row) {
  static_assert(CPR == 4 || CPR == 8 || CPR == 16, "row length");
  if constexpr (CPR == 4) return (row >> 2) & 3;
  if constexpr (CPR == 8) return (((row >> 1) & 1) << 2) | ((row >> 2) & 3);
  return row & 15;
}

// Element offset (in bf16 units) of chunk `chunk` of `row` in an image with CPR chunks per row.
template <int CPR>
__device__ __forceinline__ int img_off(int row, int chunk) {
  return row * (CPR * 8) + ((chunk ^ swz<CPR>(row)) << 3);
}

template <int T>
__device__ __forceinline__ void load_frag(const bf16* img, int plane_elems, int off, bf16x8 (&out)[T]) {
#pragma unroll
  for (int t = 0; t < T; ++t) out[t] = *reinterpret_cast<const bf16x8*>(img + t * plane_elems + off);
}

template <int T>
__device__ __forceinline__ void store_frag(bf16* img, int plane_elems, int off, const bf16x8 (&in)[T]) {
#pragma unroll
  for (int t = 0; t < T; ++t) *reinterpret_cast<bf16x8*>(img + t * plane_elems + off) = in[t];
}

}  // namespace protoseg

namespace protoseg {

// ---- buffer-resource memory ops: out-of-range offsets are dropped (stores) or read 0 (loads),
// which replaces per-element exec-mask branches. Descriptors are built from kernel arguments
// (wave-uniform), and every tensor is < 2^31 bytes (checked on the host), so a lane offset of
// kOOB plus any uniform offset stays out of range without wrapping.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr unsigned kOOB = 0x80000000u;

__device__ __forceinline__ rsrc_t make_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), static_cast<short>(0), static_cast<int>(bytes),
                                           0x00020000);
}

template <typename TX> struct BufIO;
template <> struct BufIO<float> {
  static __device__ __forceinline__ float load(rsrc_t r, unsigned voff, unsigned soff) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
  }
  static __device__ __forceinline__ void store(rsrc_t r, float v, unsigned voff, unsigned soff) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, voff, soff, 0);
  }
};
template <> struct BufIO<uint16_t> {
  static __device__ __forceinline__ float load(rsrc_t r, unsigned voff, unsigned soff) {
    return __uint_as_float(static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b16(r, voff, soff, 0)) << 16);
  }
  static __device__ __forceinline__ void store(rsrc_t r, float v, unsigned voff, unsigned soff) {
    const uint16_t b = __builtin_bit_cast(uint16_t, static_cast<bf16>(v));  // RNE, NaN kept
    __builtin_amdgcn_raw_buffer_store_b16(b, r, voff, soff, 0);
  }
};

// Activations of the bf16 family, with their constant factors folded into the operand images
// (l2_prep_bf16_kernel) instead of applied per element:
//   act  = act_unit * act_base(d):   log: ln2 * log2((d+1)/(d+eps))   (ln2 is in the W image)
//                                    linear: 1 * (-d)
//   act' = grad_unit * grad_base(d): log: (eps-1) * 1/((d+1)(d+eps))   ((eps-1) is in W^T)
//                                    linear: -1 * 1                   (-1 is in W^T)
// v_rcp_f32 + v_log_f32 replace the IEEE division and the denormal-safe logf: the ratio
// (d+1)/(d+eps) lies in (1, 1e4], where v_log_f32 is accurate to ~1 ulp. The forward forms the
// ratio as 1 + (1-eps)/(d+eps) (one add, one rcp, one fma: a VALU op fewer per element than
// (d+1) * rcp(d+eps); same absolute rounding, one ulp of the ratio).
constexpr float kLn2 = 0.6931471805599453f;
template <int ACT>
__device__ __forceinline__ float act_base(float d, float eps) {
  if constexpr (ACT == 0) {
    return __builtin_amdgcn_logf(fmaf(1.f - eps, __builtin_amdgcn_rcpf(d + eps), 1.f));
  } else {
    return -d;
  }
}
template <int ACT>
__device__ __forceinline__ float act_grad_base(float d, float eps) {
  if constexpr (ACT == 0) {
    return __builtin_amdgcn_rcpf((d + 1.f) * (d + eps));
  } else {
    return 1.f;
  }
}
// Both at once from one reciprocal (the bwd_pw epilogue needs the pair): with u = d+1 and
// r = 1/(u(d+eps)), (d+1)/(d+eps) = u*u*r — two multiplies instead of a second v_rcp_f32.
template <int ACT>
__device__ __forceinline__ float act_grad_and_base(float d, float eps, float& act) {
  if constexpr (ACT == 0) {
    const float u = d + 1.f;
    const float r = __builtin_amdgcn_rcpf(u * (d + eps));
    act = __builtin_amdgcn_logf((u * u) * r);
    return r;
  } else {
    act = -d;
    return 1.f;
  }
}
// F.relu on an accumulator value as one v_med3_f32 (distances are finite, so the FLT_MAX bound
// never binds). fmaxf(x, 0), or med3 with +inf (folded back to fmaxnum), also emits a NaN-quieting
// v_max_f32 x, x: IEEE mode cannot prove that an MFMA result is not a signalling NaN.
__device__ __forceinline__ float relu_f(float x) { return __builtin_amdgcn_fmed3f(x, 0.f, 3.402823466e38f); }
// The deeplab_simple add-on (model.py:124-128: nn.Sigmoid) applied on the layer's x load when
// the caller passes the pre-activation (PROTOSEG_X_SIGMOID): 1 / (1 + 2^(-x log2 e)) as one
// v_exp_f32 + v_rcp_f32. Forward and backward form it with this one sequence, so the backward's
// recomputed distances (and relu mask) are the forward's bit for bit. Within 2 ulp of torch.
__device__ __forceinline__ float sigmoid_f(float v) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(v * -1.44269504088896341f));
}
__host__ __device__ inline float act_unit(int act_kind) { return act_kind == 0 ? kLn2 : 1.f; }
__host__ __device__ inline float act_grad_unit(int act_kind, float eps) { return act_kind == 0 ? eps - 1.f : -1.f; }

// Channel of k-step q, element jj, half h in the shared channel order of the bf16 family:
// chan_of(q, h, jj) = 32*(q>>1) + perm_row(q&1, h, jj). With it the x fragments a lane loads
// for the distance GEMM hold exactly the channels of its g_x accumulator registers
// (gx[ct] register 8s+jj <-> q = 2ct+s), so no lane movement is needed in the backward.
__device__ __forceinline__ constexpr int chan_of(int q, int h, int jj) { return 32 * (q >> 1) + perm_row(q & 1, h, jj); }
// The lane-independent part (h = 0).
__device__ __forceinline__ constexpr int chan_base(int q, int jj) { return chan_of(q, 0, jj); }

}  // namespace protoseg

// ---- optional per-wave phase timestamps (debug builds: make stamps) --------------------------
// STAMP(slot) records s_memtime for (workgroup, wave, slot) into g_stamps; the host reads them
// with protoseg_debug_stamps(). Compiled out unless PROTOSEG_STAMPS is defined.
#ifdef PROTOSEG_STAMPS
namespace protoseg {
constexpr int kStampSlots = 8;
constexpr int kStampCap = 1 << 17;
__device__ extern unsigned long long g_stamps[kStampCap];
}  // namespace protoseg
// Each translation unit records into its own array (no device-side linking across TUs).
#ifndef PROTOSEG_STAMP_ARRAY
#define PROTOSEG_STAMP_ARRAY ::protoseg::g_stamps
#endif
#define STAMP(slot)                                                                                   \
  do {                                                                                                \
    const unsigned _w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);                          \
    if ((threadIdx.x & 63) == 0 && _w * ::protoseg::kStampSlots + (slot) < ::protoseg::kStampCap)      \
      PROTOSEG_STAMP_ARRAY[_w * ::protoseg::kStampSlots + (slot)] = __builtin_amdgcn_s_memtime();     \
  } while (0)
#define STAMP_RT(slot)                                                                                \
  do {                                                                                                \
    const unsigned _w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);                          \
    if ((threadIdx.x & 63) == 0 && _w * ::protoseg::kStampSlots + (slot) < ::protoseg::kStampCap)      \
      PROTOSEG_STAMP_ARRAY[_w * ::protoseg::kStampSlots + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define STAMP_RT(slot) \
  do {                 \
  } while (0)
#define STAMP(slot) \
  do {              \
  } while (0)
#endif
