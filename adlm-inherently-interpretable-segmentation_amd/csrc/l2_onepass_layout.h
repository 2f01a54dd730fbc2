// l2_onepass_layout.h — the operand block of the one-pass training backward (l2_bwd_onepass.hip)
// and the device code that fills it, shared by that kernel's own prep launch and by the forward's
// prep launch (l2_bf16.hip), which builds it beside the forward's images when the caller will run
// the backward on the same operands (PROTOSEG_OPERANDS_FROM_FWD).
#pragma once
#include "bf16_split.h"
#include "l2_bf16_common.h"

namespace protoseg {
namespace onepass {

constexpr int kT = 2;  // split terms (bf16x3: 3 MFMAs per product)

// Block layout (g = l >> 4, m = l & 15):
//   wt [ptile Pp/16][term]: g_act B fragment (fragment order, 1 KiB, lane l at 16 l): lane (p =
//                           16 ptile + m), classes 8 g + e (grad_unit * W)
//   pi [term][Pp][64 c]:    the (-2P) image, bf16 rows of 128 B, 16-B chunk q (channels 8q ..
//                           8q+7) at q ^ pi_swz(p); copied to LDS as is
//   p2 [Pp]                 ||p||^2 in the family's order (the forward's)
struct Offsets {
  int wt, pi, p2, total;
};
__host__ __device__ constexpr Offsets offsets(int Pp) {
  Offsets o{};
  o.wt = 0;
  o.pi = o.wt + (Pp / 16) * kT * 1024;
  o.p2 = o.pi + kT * Pp * 128;
  o.total = o.p2 + ((Pp * 4 + 1023) & ~1023);
  return o;
}
// (-2P) image swizzle: row p, 16-B chunk q at q ^ pi_swz(p) (tools/lds_swizzle_check.py pimg).
__host__ __device__ __forceinline__ int pi_swz(int p) { return (p & 2) | ((p >> 1) & 4); }

// The (-2P) image: thread tid < Pp * 8 writes row p = tid >> 3, chunk q = tid & 7, both terms.
__device__ __forceinline__ void fill_pi(const float* __restrict__ protos, int P, int Pp, unsigned char* block, int tid) {
  using namespace bf16l;
  if (tid >= Pp * 8) return;
  const Offsets o = offsets(Pp);
  const int p = tid >> 3, q = tid & 7;
  float v[8];
  bf16x8 f[kT];
  const int pc = p < P ? p : P - 1;  // clamped loads, pinned (pin_batch)
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = protos[static_cast<size_t>(pc) * kC + 8 * q + e];
  pin_batch(v);
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = p < P ? -2.f * v[e] : 0.f;
  split8<kT>(v, f);
  const int off = o.pi + p * 128 + ((q ^ pi_swz(p)) & 7) * 16;
#pragma unroll
  for (int t = 0; t < kT; ++t) *reinterpret_cast<bf16x8*>(block + off + t * Pp * 128) = f[t];
}

// The W^T fragments: thread tid = 64 frag + lane, frag < Pp / 16.
__device__ __forceinline__ void fill_wt(const float* __restrict__ w_last, int K, int ldw, int P, int Pp, float wt_scale,
                                        unsigned char* block, int tid) {
  using namespace bf16l;
  const Offsets o = offsets(Pp);
  const int lane = tid & 63, frag = tid >> 6, g = lane >> 4, m = lane & 15;
  if (frag >= Pp / 16) return;
  const int p = 16 * frag + m;
  float v[8] = {};
  bf16x8 f[kT];
  if (w_last && K > 0) {  // clamped loads, pinned (pin_batch)
    const int pc = p < P ? p : P - 1;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = w_last[static_cast<size_t>(8 * g + e < K ? 8 * g + e : K - 1) * ldw + pc];
    pin_batch(v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (p < P && 8 * g + e < K) ? wt_scale * v[e] : 0.f;
  }
  split8<kT>(v, f);
#pragma unroll
  for (int t = 0; t < kT; ++t) *reinterpret_cast<bf16x8*>(block + o.wt + (frag * kT + t) * 1024 + lane * 16) = f[t];
}

}  // namespace onepass
}  // namespace protoseg
