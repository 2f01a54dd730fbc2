// l2_layer.hip — the PPNet prototype layer on gfx950: fused forward and a two-kernel
// backward, all on f32-input MFMA (v_mfma_f32_32x32x2_f32, an exact f32 fma chain).
//
// Reference: model.py:203-221 (_l2_convolution), 231-237 (distance_2_similarity),
// 259-283 (forward_from_conv_features, patch_classification branch), and the autograd
// graph of those ops for the backward.
//
// Index space: pixels are flattened over the batch, g = b*HW + n, and cut into 32-pixel
// tiles; prototypes are padded to Pp = ceil(P/32)*32 (zero rows), classes to 32.
//
//   l2_fwd_kernel      "layout A" tiles S[p][n] (prototype on the register rows, pixel on
//                      the lane) -> D stored NCHW with 128-B row segments; the activation
//                      tile is already the B operand of the last-layer MFMA (rows = p).
//   l2_bwd_x_kernel    layout A again: recompute S, g_act = W^T g_logits, g_s, and
//                      g_x = P^T (-2 g_s) accumulated over p-tiles (sums over rows: no
//                      lane movement), + 2 x sum_p g_s.
//   l2_bwd_pw_kernel   "layout B" tiles S[n][p] (pixel on the rows): g_P^T and g_W sum over
//                      pixels = over rows, so the g_s / act tiles feed the MFMA A/B operands
//                      directly. One workgroup per (p-tile, pixel split); per-workgroup
//                      partial slabs, reduced by l2_bwd_reduce_kernel in a fixed order
//                      (bitwise reproducible, no atomics).
#include "protoseg_device.h"
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <utility>
#include <vector>

#include "bf16_split.h"
#include "l2_launch.h"
#include "protoseg_host.h"

// (defined below, after the kernel families' launch helpers)
bool use_wide(int C, int K, int P);

namespace protoseg {

namespace {

constexpr int kFwdWaves = 8;   // 512-thread workgroups share one LDS prototype image
constexpr int kPwWaves = 4;
constexpr int kLdx = 33;       // padded row of the per-wave X tile in bwd_pw
constexpr int kLdt = 33;       // padded row of a prototype tile [C][33]

// Stage prototypes tile-major as Pt[pt][c][33] (a 32-prototype tile per [C][33] block) and
// p2[p] = sum_c p^2 (model.py:210-211). Every read is conflict-free: lanes over p (distance
// A operand, consecutive words) and lanes over c (g_x A operand, stride 33); and every
// per-register offset is a compile-time immediate on one lane base.
template <int NC>
__device__ void stage_prototypes(float* Pt, float* p2s, const float* __restrict__ protos, int P, int Pp) {
  constexpr int C = NC * 32;
  for (int idx = threadIdx.x; idx < Pp * C; idx += blockDim.x) {
    const int p = idx / C;
    const int c = idx - p * C;
    Pt[((p >> 5) * C + c) * kLdt + (p & 31)] = (p < P) ? protos[static_cast<size_t>(p) * C + c] : 0.f;
  }
  __syncthreads();
  for (int p = threadIdx.x; p < Pp; p += blockDim.x) {
#pragma clang fp contract(off)
    float s = 0.f;
    for (int c = 0; c < C; ++c) {
      const float v = Pt[((p >> 5) * C + c) * kLdt + (p & 31)];
      s += v * v;
    }
    p2s[p] = s;
  }
}

// Same p2 as stage_prototypes, for one prototype row read from global memory.
template <int NC>
__device__ float proto_norm2(const float* __restrict__ protos, int p, bool valid) {
#pragma clang fp contract(off)
  constexpr int C = NC * 32;
  float s = 0.f;
  if (valid) {
    for (int c = 0; c < C; ++c) {
      const float v = protos[static_cast<size_t>(p) * C + c];
      s += v * v;
    }
  }
  return s;
}

// Loads the 32-pixel tile of x for this lane in layout-A order: xv[ct][r] = x[c][pixel j]
// with c = 32ct + acc_row(r, h). Returns the full ||x||^2 of the lane's pixel (both
// half-waves hold the same value).
template <typename TX, int NC>
__device__ __forceinline__ float load_x_tile(const TX* __restrict__ xb, int HW, bool valid, float (&xv)[NC][16]) {
  const int h = (threadIdx.x & 63) >> 5;
  const TX* xh = xb + static_cast<size_t>(4 * h) * HW;
  float x2 = 0.f;
#pragma unroll
  for (int ct = 0; ct < NC; ++ct) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      // channel c = 32ct + acc_row(r, h); unconditional load (invalid lanes read pixel 0
      // of image 0), then select: a conditional load makes hipcc branch and drain vmcnt
      const float v = XIO<TX>::load(xh, static_cast<size_t>(ct * 32 + row_of(r)) * HW);
      xv[ct][r] = valid ? v : 0.f;
      x2 = fmaf(xv[ct][r], xv[ct][r], x2);
    }
  }
  x2 += __shfl_xor(x2, 32);
  return x2;
}

template <typename TX, int NC>
__global__ __launch_bounds__(kFwdWaves * 64) void l2_fwd_kernel(
    const TX* __restrict__ x, int HW, int npix, const float* __restrict__ protos, int P, int Pp,
    const float* __restrict__ w_last, int K, float eps, int act_kind, float* __restrict__ dist,
    float* __restrict__ act_out, float* __restrict__ logits, int ld, int p0, int ldw, int accumulate) {
  // Prototype chunk p0 .. p0 + P of ld in all (ld = P, p0 = 0 for a whole call): distance rows at
  // b * ld + p0 + p, activation columns at g * ld + p0 + p, W columns at stride ldw (w_last
  // points at column p0), logits added to the earlier chunks' when accumulate != 0.
  constexpr int C = NC * 32;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Pt = smem;                      // [Pp/32][C][33]
  float* Wl = Pt + (Pp / 32) * C * kLdt;  // [Pp][32]: W[k][p] at p*32 + k
  float* p2s = Wl + Pp * 32;     // [Pp]
  const bool do_logits = logits != nullptr;
  if (do_logits) {
    for (int idx = threadIdx.x; idx < Pp * 32; idx += blockDim.x) {
      const int p = idx >> 5, k = idx & 31;
      Wl[idx] = (p < P && k < K) ? w_last[static_cast<size_t>(k) * ldw + p] : 0.f;
    }
  }
  stage_prototypes<NC>(Pt, p2s, protos, P, Pp);
  __syncthreads();

  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5, wave = threadIdx.x >> 6;
  const int ntiles = (npix + 31) / 32;
  const int npt = Pp / 32;
  for (int t = blockIdx.x * kFwdWaves + wave; t < ntiles; t += gridDim.x * kFwdWaves) {
    const int g = t * 32 + j;
    const bool valid = g < npix;
    const int b = valid ? g / HW : 0;
    const int n = valid ? g - b * HW : 0;
    float xv[NC][16];
    const float x2 = load_x_tile<TX, NC>(x + static_cast<size_t>(b) * C * HW + n, HW, valid, xv);

    f32x16 lacc = zero16();
#pragma unroll 1
    for (int pt = 0; pt < npt; ++pt) {
      // row p = pt*32 + 4h + row_of(r) of D[b] (clamped to a valid row for padded lanes)
      float* dpt = dist ? dist + (static_cast<size_t>(b) * ld + p0 + pt * 32 + 4 * h) * HW + n : nullptr;
      f32x16 acc = zero16();
      const float* Pa = Pt + pt * C * kLdt + j;
#pragma unroll
      for (int ct = 0; ct < NC; ++ct)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc = mfma32(Pa[(ct * 32 + acc_row(r, h)) * kLdt], xv[ct][r], acc);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int p = pt * 32 + acc_row(r, h);
        const float d = l2_distance(x2, p2s[p], acc[r]);
        const bool st = valid && p < P;
        if (dpt && st) dpt[static_cast<size_t>(row_of(r)) * HW] = d;
        const float a = activation(d, eps, act_kind);
        if (act_out && st) act_out[static_cast<size_t>(g) * ld + p0 + p] = a;
        acc[r] = a;
      }
      if (do_logits) {
        const float* Wa = Wl + pt * 32 * 32 + j;
#pragma unroll
        for (int r = 0; r < 16; ++r) lacc = mfma32(Wa[acc_row(r, h) * 32], acc[r], lacc);
      }
    }
    if (do_logits && valid) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int k = acc_row(r, h);
        if (k < K) {
          float* lp = logits + static_cast<size_t>(g) * K + k;
          *lp = accumulate ? *lp + lacc[r] : lacc[r];
        }
      }
    }
  }
}

template <typename TX, int NC>
__global__ __launch_bounds__(kFwdWaves * 64) void l2_bwd_x_kernel(
    const TX* __restrict__ x, int HW, int npix, const float* __restrict__ protos, int P, int Pp,
    const float* __restrict__ w_last, int K, float eps, int act_kind, const float* __restrict__ g_logits,
    const float* __restrict__ g_dist, TX* __restrict__ g_x, int ld, int p0, int ldw, int accumulate) {
  // chunk conventions as l2_fwd_kernel; g_x of chunk c > 0 is added (a sum over prototypes)
  constexpr int C = NC * 32;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Pt = smem;                      // [Pp/32][C][33]
  float* Wt = Pt + (Pp / 32) * C * kLdt;  // [Pp/32][32][32]: W[k][p] at (p>>5)*1024 + k*32 + (p&31)
  float* p2s = Wt + Pp * 32;     // [Pp]
  if (g_logits) {
    for (int idx = threadIdx.x; idx < Pp * 32; idx += blockDim.x) {
      const int pt = idx >> 10, k = (idx >> 5) & 31, p = pt * 32 + (idx & 31);
      Wt[idx] = (p < P && k < K) ? w_last[static_cast<size_t>(k) * ldw + p] : 0.f;
    }
  }
  stage_prototypes<NC>(Pt, p2s, protos, P, Pp);
  __syncthreads();

  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5, wave = threadIdx.x >> 6;
  const int ntiles = (npix + 31) / 32;
  const int npt = Pp / 32;
  const int KS = (K + 1) / 2;
  for (int t = blockIdx.x * kFwdWaves + wave; t < ntiles; t += gridDim.x * kFwdWaves) {
    const int g = t * 32 + j;
    const bool valid = g < npix;
    const int b = valid ? g / HW : 0;
    const int n = valid ? g - b * HW : 0;
    float xv[NC][16];
    const float x2 = load_x_tile<TX, NC>(x + static_cast<size_t>(b) * C * HW + n, HW, valid, xv);
    // B operand of g_act^T = W^T g_logits^T: lane (h, j) holds g_logits[pixel j][k = 2s+h].
    float gl[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int k = 2 * s + h;
      const bool ok = valid && k < K;
      const float v = g_logits ? g_logits[ok ? static_cast<size_t>(g) * K + k : 0] : 0.f;
      gl[s] = ok ? v : 0.f;
    }

    f32x16 gx[NC];
#pragma unroll
    for (int ct = 0; ct < NC; ++ct) gx[ct] = zero16();
    float gsum = 0.f;
#pragma unroll 1
    for (int pt = 0; pt < npt; ++pt) {
      f32x16 acc = zero16();
      const float* Pa = Pt + pt * C * kLdt + j;
#pragma unroll
      for (int ct = 0; ct < NC; ++ct)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc = mfma32(Pa[(ct * 32 + acc_row(r, h)) * kLdt], xv[ct][r], acc);
      const float* gdpt = g_dist ? g_dist + (static_cast<size_t>(b) * ld + p0 + pt * 32 + 4 * h) * HW + n : nullptr;
      f32x16 gacc = zero16();
      if (g_logits) {
        const float* Wa = Wt + pt * 1024 + j;
#pragma unroll
        for (int s = 0; s < 16; ++s)
          if (s < KS) gacc = mfma32(Wa[(2 * s + h) * 32], gl[s], gacc);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int p = pt * 32 + acc_row(r, h);
        const float d = l2_distance(x2, p2s[p], acc[r]);
        float gd = g_logits ? gacc[r] * activation_grad(d, eps, act_kind) : 0.f;
        if (gdpt) {
          const bool ok = valid && p < P;
          const float v = gdpt[ok ? static_cast<size_t>(row_of(r)) * HW : 0];
          gd += ok ? v : 0.f;
        }
        const float gs = (d > 0.f && p < P) ? gd : 0.f;  // relu backward: grad * (out > 0)
        gsum += gs;
        acc[r] = -2.f * gs;                               // d(-2*xp)/dxp folded into the operand
      }
#pragma unroll
      for (int ct = 0; ct < NC; ++ct) {
        const float* Pc = Pt + (pt * C + ct * 32 + j) * kLdt;
#pragma unroll
        for (int r = 0; r < 16; ++r) gx[ct] = mfma32(Pc[acc_row(r, h)], acc[r], gx[ct]);
      }
    }
    gsum += __shfl_xor(gsum, 32);
    if (valid) {
      TX* gxh = g_x + (static_cast<size_t>(b) * C + 4 * h) * HW + n;
#pragma unroll
      for (int ct = 0; ct < NC; ++ct)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          // channel c = 32ct + acc_row(r, h). conv(x^2, ones) backward then pow backward:
          // gsum * (2x); plus the xp branch accumulated in gx.
          const size_t o = static_cast<size_t>(ct * 32 + row_of(r)) * HW;
          const float v = gx[ct][r] + gsum * (2.f * xv[ct][r]);
          XIO<TX>::store(gxh, o, accumulate ? XIO<TX>::load(gxh, o) + v : v);
        }
    }
  }
}

template <typename TX, int NC>
__global__ __launch_bounds__(kPwWaves * 64) void l2_bwd_pw_kernel(
    const TX* __restrict__ x, int HW, int npix, const float* __restrict__ protos, int P, int Pp,
    const float* __restrict__ w_last, int K, float eps, int act_kind, const float* __restrict__ g_logits,
    const float* __restrict__ g_dist, float* __restrict__ slab_gp, float* __restrict__ slab_gw,
    float* __restrict__ slab_gs) {
  constexpr int C = NC * 32;
  // LDS: Pl[C][32] prototype tile (B operand of S), Wl[32][32] class tile (B operand of
  // g_act), then one Xl[C][33] pixel tile per wave (A operand of S, B operand of g_P).
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Pl = smem;
  float* Wl = Pl + C * 32;
  float* Xall = Wl + 32 * 32;
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5, wave = threadIdx.x >> 6;
  float* Xl = Xall + wave * C * kLdx;
  const int pt = blockIdx.x;
  const int p = pt * 32 + j;  // this lane's prototype column
  const bool pvalid = p < P;

  for (int idx = threadIdx.x; idx < C * 32; idx += blockDim.x) {
    const int c = idx >> 5, pp = pt * 32 + (idx & 31);
    Pl[idx] = pp < P ? protos[static_cast<size_t>(pp) * C + c] : 0.f;
  }
  for (int idx = threadIdx.x; idx < 32 * 32; idx += blockDim.x) {
    const int k = idx >> 5, pp = pt * 32 + (idx & 31);
    Wl[idx] = (g_logits && k < K && pp < P) ? w_last[static_cast<size_t>(k) * P + pp] : 0.f;
  }
  const float p2 = proto_norm2<NC>(protos, p, pvalid);
  const int KS = (K + 1) / 2;
  __syncthreads();

  f32x16 gp[NC];
#pragma unroll
  for (int ct = 0; ct < NC; ++ct) gp[ct] = zero16();
  f32x16 gw = zero16();
  float gsum = 0.f;

  const int ntiles = (npix + 31) / 32;
  for (int t = blockIdx.y * kPwWaves + wave; t < ntiles; t += gridDim.y * kPwWaves) {
    const int g0 = t * 32;
    const int g = g0 + j;  // pixel staged by this lane
    const bool valid = g < npix;
    const int b = valid ? g / HW : 0;
    const int n = valid ? g - b * HW : 0;

    wave_lds_fence();  // the previous tile's reads of Xl are complete
    float x2;
    {
      float xv[NC][16];
      x2 = load_x_tile<TX, NC>(x + static_cast<size_t>(b) * C * HW + n, HW, valid, xv);
#pragma unroll
      for (int ct = 0; ct < NC; ++ct)
#pragma unroll
        for (int r = 0; r < 16; ++r) Xl[(ct * 32 + acc_row(r, h)) * kLdx + j] = xv[ct][r];
    }
    float gl[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int k = 2 * s + h;
      const bool ok = valid && k < K;
      const float v = g_logits ? g_logits[ok ? static_cast<size_t>(g) * K + k : 0] : 0.f;
      gl[s] = ok ? v : 0.f;
    }
    wave_lds_fence();  // Xl writes of every lane are visible

    // S[n][p]: A = x (lane i = pixel, k = channel pair), B = P (lane j = prototype).
    f32x16 acc = zero16();
    {
      const float* Xa = Xl + 4 * h * kLdx + j;
      const float* Pb = Pl + 4 * h * 32 + j;
#pragma unroll
      for (int ct = 0; ct < NC; ++ct)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          acc = mfma32(Xa[(ct * 32 + row_of(r)) * kLdx], Pb[(ct * 32 + row_of(r)) * 32], acc);
    }
    f32x16 gacc = zero16();
    if (g_logits) {
      const float* Wb = Wl + h * 32 + j;
#pragma unroll
      for (int s = 0; s < 16; ++s)
        if (s < KS) gacc = mfma32(gl[s], Wb[2 * s * 32], gacc);
    }

#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int nr = acc_row(r, h);
      const bool rvalid = g0 + nr < npix;
      const float x2n = __shfl(x2, nr);
      const float d = l2_distance(x2n, p2, acc[r]);
      const float a = activation(d, eps, act_kind);
      float gd = g_logits ? gacc[r] * activation_grad(d, eps, act_kind) : 0.f;
      if (g_dist) {  // row nr's (image, pixel) comes from the lane that staged it
        const bool ok = rvalid && pvalid;
        const int br = __shfl(b, nr), nn = __shfl(n, nr);
        const float v = g_dist[ok ? (static_cast<unsigned>(br) * P + p) * static_cast<unsigned>(HW) + nn : 0u];
        gd += ok ? v : 0.f;
      }
      const float gs = (d > 0.f && pvalid && rvalid) ? gd : 0.f;
      gsum += gs;
      acc[r] = -2.f * gs;
      gacc[r] = rvalid ? a : 0.f;
    }

    // g_P^T tile: A = -2 g_s (lane = prototype, k = pixel rows), B = x (lane = channel).
#pragma unroll
    for (int ct = 0; ct < NC; ++ct) {
      const float* Xc = Xl + (ct * 32 + j) * kLdx + 4 * h;
#pragma unroll
      for (int r = 0; r < 16; ++r) gp[ct] = mfma32(acc[r], Xc[row_of(r)], gp[ct]);
    }
    // g_W tile: A = g_logits^T (lane = class), B = act (lane = prototype).
    if (g_logits) {
      const int gh = g0 + 4 * h;
      const float* glh = g_logits + static_cast<unsigned>(gh) * K + j;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const bool ok = gh + row_of(r) < npix && j < K;
        const float v = glh[ok ? row_of(r) * K : 0];
        gw = mfma32(ok ? v : 0.f, gacc[r], gw);
      }
    }
  }

  // Workgroup reduction of the per-wave partials through LDS, fixed wave order.
  __syncthreads();
  float* R = Xall + wave * C * kLdx;  // >= 32*C + 32 floats per wave
#pragma unroll
  for (int ct = 0; ct < NC; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r) R[acc_row(r, h) * C + ct * 32 + j] = gp[ct][r];
  __syncthreads();
  for (int idx = threadIdx.x; idx < 32 * C; idx += blockDim.x) {
    float s = 0.f;
    for (int w = 0; w < kPwWaves; ++w) s += Xall[w * C * kLdx + idx];
    const int pr = idx / C, c = idx - pr * C;
    slab_gp[(static_cast<size_t>(blockIdx.y) * Pp + pt * 32 + pr) * C + c] = s;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) R[acc_row(r, h) * 32 + j] = gw[r];
  gsum += __shfl_xor(gsum, 32);
  if (h == 0) R[1024 + j] = gsum;
  __syncthreads();
  for (int idx = threadIdx.x; idx < 32 * 32 + 32; idx += blockDim.x) {
    float s = 0.f;
    for (int w = 0; w < kPwWaves; ++w) s += Xall[w * C * kLdx + idx];
    if (idx < 1024) {
      const int k = idx >> 5, pc = idx & 31;
      slab_gw[(static_cast<size_t>(blockIdx.y) * 32 + k) * Pp + pt * 32 + pc] = s;
    } else {
      slab_gs[static_cast<size_t>(blockIdx.y) * Pp + pt * 32 + (idx - 1024)] = s;
    }
  }
}

__global__ void l2_bwd_reduce_kernel(const float* __restrict__ slab_gp, const float* __restrict__ slab_gw,
                                     const float* __restrict__ slab_gs, int S, int P, int Pp, int C, int K,
                                     const float* __restrict__ protos, float* __restrict__ g_protos,
                                     float* __restrict__ g_w) {
  const long long e = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (g_protos && e < static_cast<long long>(P) * C) {
    const int p = static_cast<int>(e / C), c = static_cast<int>(e - static_cast<long long>(p) * C);
    float s = 0.f, gs = 0.f;
    for (int si = 0; si < S; ++si) {
      s += slab_gp[(static_cast<size_t>(si) * Pp + p) * C + c];
      gs += slab_gs[static_cast<size_t>(si) * Pp + p];
    }
    // conv weight grad of xp (-2 g_s folded) + pow backward of p2: gs * (2p)
    g_protos[e] = s + gs * (2.f * protos[e]);
  }
  if (g_w && e < static_cast<long long>(K) * P) {
    const int k = static_cast<int>(e / P), p = static_cast<int>(e - static_cast<long long>(k) * P);
    float s = 0.f;
    for (int si = 0; si < S; ++si) s += slab_gw[(static_cast<size_t>(si) * 32 + k) * Pp + p];
    g_w[e] = s;
  }
}

// ---------------------------------------------------------------------------------------
// Host side.

int padded_protos(int P) { return static_cast<int>(ceil_div(P, 32) * 32); }

size_t layer_lds_bytes(int C, int Pp) {
  return (static_cast<size_t>(Pp / 32) * C * kLdt + static_cast<size_t>(Pp) * 32 + Pp) * sizeof(float);
}

int nc_of(int C) { return C == 32 ? 1 : C == 64 ? 2 : C == 128 ? 4 : 0; }

int validate(const void* x, int x_dtype, int B, int C, int H, int W, const float* protos, int P, int K,
             int act_kind, int precision, Geometry* geo) {
  if (!x || !protos) return fail(PROTOSEG_ERR_INVALID, "x and protos must be non-null");
  if (B <= 0 || H <= 0 || W <= 0 || P <= 0 || K < 0)
    return fail(PROTOSEG_ERR_INVALID, "bad shape B=%d H=%d W=%d P=%d K=%d", B, H, W, P, K);
  if (x_dtype != PROTOSEG_F32 && x_dtype != PROTOSEG_BF16 && x_dtype != PROTOSEG_F16)
    return fail(PROTOSEG_ERR_UNSUPPORTED, "x_dtype %d (f32, bf16 or f16 only)", x_dtype);
  if (x_dtype == PROTOSEG_F16 && C > 0 && P > 0 && K >= 0 && !use_wide(C, K, P))
    return fail(PROTOSEG_ERR_UNSUPPORTED, "x_dtype f16: the wide family only (protoseg_l2_x_dtype_supported)");
  if (act_kind != PROTOSEG_ACT_LOG && act_kind != PROTOSEG_ACT_LINEAR)
    return fail(PROTOSEG_ERR_UNSUPPORTED, "act_kind %d", act_kind);
  if (precision < PROTOSEG_PREC_BF16X3 || precision > PROTOSEG_PREC_F32)
    return fail(PROTOSEG_ERR_UNSUPPORTED, "precision %d", precision);
  if (!protoseg_l2_supported(C, P, K))
    return fail(PROTOSEG_ERR_UNSUPPORTED, "C=%d P=%d K=%d outside the kernel family", C, P, K);
  geo->C = C;
  geo->P = P;
  geo->Pp = padded_protos(P);
  geo->K = K;
  geo->HW = H * W;
  const long long npix = static_cast<long long>(B) * H * W;
  const long long big = npix * (C > P ? C : P);
  if (big >= (1LL << 31) - 64)
    return fail(PROTOSEG_ERR_UNSUPPORTED, "B*H*W*max(C,P)=%lld >= 2^31 elements: split the batch", big);
  geo->npix = static_cast<int>(npix);
  geo->ntiles = static_cast<int>(ceil_div(npix, 32));
  geo->ldw = P;
  geo->ldd = P;
  geo->p0 = 0;
  return PROTOSEG_OK;
}

// Grid for the pixel-major kernels: every resident workgroup slot once, no more than the tiles.
int layer_grid(const Geometry& geo) {
  const size_t lds = layer_lds_bytes(geo.C, geo.Pp);
  const int per_cu = static_cast<int>(kMaxLds / lds) > 0 ? static_cast<int>(kMaxLds / lds) : 1;
  const long long want = ceil_div(geo.ntiles, kFwdWaves);
  const long long cap = 256LL * (per_cu < 2 ? per_cu : 2);
  return static_cast<int>(want < cap ? want : cap);
}

// Pixel splits of the bwd_pw grid: ~512 workgroups in all.
int pw_splits(long long ntiles, int Pp) {
  const long long npt = Pp / 32;
  long long s = 512 / npt;
  if (s < 1) s = 1;
  const long long need = ceil_div(ntiles, kPwWaves);
  return static_cast<int>(s < need ? s : need);
}

template <typename TX, int NC>
int launch_fwd(const Geometry& geo, const void* x, const float* protos, const float* w_last, float eps,
               int act_kind, float* dist, float* act, float* logits, hipStream_t stream, int accumulate = 0) {
  if (int st = ensure_lds<l2_fwd_kernel<TX, NC>>()) return st;
  const size_t lds = layer_lds_bytes(geo.C, geo.Pp);
  KernelTimer timer("l2_fwd_kernel", stream);
  hipLaunchKernelGGL((l2_fwd_kernel<TX, NC>), dim3(layer_grid(geo)), dim3(kFwdWaves * 64), lds, stream,
                     static_cast<const TX*>(x), geo.HW, geo.npix, protos, geo.P, geo.Pp, w_last, geo.K, eps,
                     act_kind, dist, act, logits, geo.ldd, geo.p0, geo.ldw, accumulate);
  return check_launch("l2_fwd_kernel");
}

template <typename TX, int NC>
int launch_bwd_x(const Geometry& geo, const void* x, const float* protos, const float* w_last, float eps,
                 int act_kind, const float* g_logits, const float* g_dist, void* g_x, hipStream_t stream,
                 int accumulate = 0) {
  if (int st = ensure_lds<l2_bwd_x_kernel<TX, NC>>()) return st;
  KernelTimer timer("l2_bwd_x_kernel", stream);
  hipLaunchKernelGGL((l2_bwd_x_kernel<TX, NC>), dim3(layer_grid(geo)), dim3(kFwdWaves * 64),
                     layer_lds_bytes(geo.C, geo.Pp), stream, static_cast<const TX*>(x), geo.HW, geo.npix, protos,
                     geo.P, geo.Pp, w_last, geo.K, eps, act_kind, g_logits, g_dist, static_cast<TX*>(g_x), geo.ldd,
                     geo.p0, geo.ldw, accumulate);
  return check_launch("l2_bwd_x_kernel");
}

size_t f32_pw_workspace(const Geometry& geo) {
  const size_t S = static_cast<size_t>(pw_splits(geo.ntiles, geo.Pp));
  return (S * geo.Pp * geo.C + S * 32 * geo.Pp + S * geo.Pp) * sizeof(float);
}

template <typename TX, int NC>
int launch_bwd_pw(const Geometry& geo, const void* x, const float* protos, const float* w_last, float eps,
                  int act_kind, const float* g_logits, const float* g_dist, float* g_protos, float* g_w, float* ws,
                  hipStream_t stream) {
  const int S = pw_splits(geo.ntiles, geo.Pp);
  float* slab_gp = ws;
  float* slab_gw = slab_gp + static_cast<size_t>(S) * geo.Pp * geo.C;
  float* slab_gs = slab_gw + static_cast<size_t>(S) * 32 * geo.Pp;
  const size_t lds = (static_cast<size_t>(geo.C) * 32 + 32 * 32 + static_cast<size_t>(kPwWaves) * geo.C * kLdx) *
                     sizeof(float);
  if (int st = ensure_lds<l2_bwd_pw_kernel<TX, NC>>()) return st;
  {
    KernelTimer timer("l2_bwd_pw_kernel", stream);
    hipLaunchKernelGGL((l2_bwd_pw_kernel<TX, NC>), dim3(geo.Pp / 32, S), dim3(kPwWaves * 64), lds, stream,
                       static_cast<const TX*>(x), geo.HW, geo.npix, protos, geo.P, geo.Pp, w_last, geo.K, eps,
                       act_kind, g_logits, g_dist, slab_gp, slab_gw, slab_gs);
    if (int st = check_launch("l2_bwd_pw_kernel")) return st;
  }
  const long long n = static_cast<long long>(geo.P) * (geo.C > geo.K ? geo.C : geo.K);
  hipLaunchKernelGGL(l2_bwd_reduce_kernel, dim3(static_cast<unsigned>(ceil_div(n, 256))), dim3(256), 0, stream,
                     slab_gp, slab_gw, slab_gs, S, geo.P, geo.Pp, geo.C, geo.K, protos, g_protos,
                     g_logits ? g_w : nullptr);
  return check_launch("l2_bwd_reduce_kernel");
}

template <typename Fn>
int dispatch(int x_dtype, int C, Fn&& fn) {
  const int nc = nc_of(C);
  if (x_dtype == PROTOSEG_F32) {
    if (nc == 1) return fn(static_cast<float*>(nullptr), std::integral_constant<int, 1>());
    if (nc == 2) return fn(static_cast<float*>(nullptr), std::integral_constant<int, 2>());
    if (nc == 4) return fn(static_cast<float*>(nullptr), std::integral_constant<int, 4>());
  } else {
    if (nc == 1) return fn(static_cast<uint16_t*>(nullptr), std::integral_constant<int, 1>());
    if (nc == 2) return fn(static_cast<uint16_t*>(nullptr), std::integral_constant<int, 2>());
    if (nc == 4) return fn(static_cast<uint16_t*>(nullptr), std::integral_constant<int, 4>());
  }
  return fail(PROTOSEG_ERR_UNSUPPORTED, "C=%d", C);
}

// Split terms of the bf16 family for a precision request; 0 = use the f32-MFMA family.
int terms_of(int precision) {
  return precision == PROTOSEG_PREC_BF16X3 ? 2 : precision == PROTOSEG_PREC_BF16X6 ? 3 : 0;
}

Geometry geometry_of(int B, int C, int H, int W, int P, int K) {
  Geometry g;
  g.C = C;
  g.P = P;
  g.Pp = padded_protos(P);
  g.K = K;
  g.HW = H * W;
  g.npix = B * H * W;
  g.ntiles = static_cast<int>(ceil_div(g.npix, 32));
  g.ldw = P;
  g.ldd = P;
  g.p0 = 0;
  return g;
}

}  // namespace

}  // namespace protoseg

using namespace protoseg;

namespace {
// Scratch for the bf16 family's operand images (a few hundred KiB): one block per (device,
// stream), allocated on first use at a size that covers every supported shape, then reused.
// Kernels on one stream are ordered, so a call's prep kernel never overwrites images that an
// earlier call's kernels still read. No per-call allocation: the launch sequence is only
// kernel launches and can be captured in a HIP graph once the block exists.
constexpr size_t kImageBlockMin = 512 * 1024;

// Backward kernel choice for the bf16x3 training backward (C = 64):
//   wave    l2_bwd_wave.hip: 4 waves, one per SIMD, each owning a quarter of the prototypes for
//           every product (P <= 384 per launch, prototype chunks beyond);
//   fused   l2_bwd_fused.hip: 6 owner + 2 g_x waves (P <= 192 per launch).
// Automatic: wave for P > 192, fused below. protoseg_set_backward_kernel("wave" / "fused" / "")
// overrides it (tests and A/B measurement); the initial override is PROTOSEG_BWD, read once.
enum class BwdKernel { kAuto = 0, kWave, kFused };
std::atomic<int> g_bwd_override{-1};  // -1: PROTOSEG_BWD not read yet
BwdKernel bwd_kernel_of_name(const char* e) {
  if (e && !strcmp(e, "wave")) return BwdKernel::kWave;
  if (e && !strcmp(e, "fused")) return BwdKernel::kFused;
  return BwdKernel::kAuto;
}
BwdKernel bwd_kernel(int P) {
  int o = g_bwd_override.load(std::memory_order_relaxed);
  if (o < 0) {
    int expected = -1;
    o = static_cast<int>(bwd_kernel_of_name(getenv("PROTOSEG_BWD")));
    if (!g_bwd_override.compare_exchange_strong(expected, o)) o = expected;
  }
  if (o != static_cast<int>(BwdKernel::kAuto)) return static_cast<BwdKernel>(o);
  // P > 192: the wave-owned kernel (one pass over X for up to 384 prototypes per chunk, the
  // forward's operand images); the fused kernel below (its 192-prototype LDS images)
  return P > 192 ? BwdKernel::kWave : BwdKernel::kFused;
}

int stream_block(size_t need, hipStream_t s, int kind, void** out) {
  return stream_scratch(static_cast<ScratchKind>(kind), need, kImageBlockMin, s, out);
}

struct ImageBlock {
  void* ptr = nullptr;
  // per > 0: the images of ceil(g.P / per) prototype chunks of `per` rows, one prep launch.
  // fwd_only: the forward's images only.
  int build(const Geometry& g, int terms, const float* protos, const float* w_last, int act_kind, float eps,
            hipStream_t s, int per = 0, int fwd_only = 0) {
    const int nchunk = per > 0 ? static_cast<int>(ceil_div(g.P, per)) : 1;
    const size_t need = per > 0 ? nchunk * bf16_image_bytes(geometry_of(1, g.C, 1, 1, per, g.K), terms)
                                : bf16_image_bytes(g, terms);
    if (int st = stream_block(need, s, 0, &ptr)) return st;
    if (per > 0)
      return launch_prep_bf16_chunks(g, per, nchunk, terms, protos, w_last, act_kind, eps, ptr, s, fwd_only);
    return launch_prep_bf16(g, terms, protos, w_last, act_kind, eps, ptr, s, fwd_only);
  }
};

// The training backward's operand images built by the forward into a caller buffer
// (protoseg_l2_fwd_ex / protoseg_l2_bwd_ex): the standard image block the wave (P <= 384) and
// fused (P <= 192) kernels read, the layout the backward's own prep would write.
enum class TrainOperands { kNone, kFused };
}  // namespace

// Largest P the bf16 family serves through prototype chunks (C = 64).
constexpr int kMaxChunkedP = 4096;

bool f32_family_fits(int C, int Pp) { return layer_lds_bytes(C, Pp) <= kMaxLds; }

// Largest P one f32-family launch stages (its LDS holds every prototype of the launch).
int f32_launch_protos(int C) {
  int p = 0;
  while (f32_family_fits(C, p + 32)) p += 32;
  return p;
}

// Bounds of the wide family (l2_wide.hip): every depth / class count the register- and
// LDS-resident families do not hold.
constexpr int kWideMaxC = 4096, kWideMaxP = 65536, kWideMaxK = 4096;

// The C in {32, 64, 128}, K <= 32, P <= 4096 families (bf16 split and f32) vs the wide GEMM family.
bool use_wide(int C, int K, int P) { return nc_of(C) == 0 || K > 32 || P > kMaxChunkedP; }

namespace {
// Which operands a bf16x3 training backward of (C, P, K) reads in one launch; kNone when it
// chunks prototypes or runs another family (the caller's buffer is then not used).
TrainOperands train_operands_kind(int C, int P, int K, int precision) {
  if (terms_of(precision) != 2 || C != 64 || P <= 0 || K < 0 || use_wide(C, K, P)) return TrainOperands::kNone;
  const Geometry g = geometry_of(1, C, 1, 1, P, K);
  switch (bwd_kernel(P)) {
    case BwdKernel::kWave:  // the standard image block (launch_prep_bf16), one chunk
      return P <= 384 && bf16_bwd_wave_fits(g, 2) ? TrainOperands::kFused : TrainOperands::kNone;
    default:
      return P <= 192 && bf16_bwd_fused_fits(g, 2) ? TrainOperands::kFused : TrainOperands::kNone;
  }
}

size_t train_operands_bytes(int C, int P, int K, TrainOperands kind) {
  const Geometry g = geometry_of(1, C, 1, 1, P, K);
  return kind == TrainOperands::kFused ? bf16_image_bytes(g, 2) : 0;
}
}  // namespace

extern "C" int protoseg_set_backward_kernel(const char* name) {
  if (name && *name && strcmp(name, "wave") && strcmp(name, "fused"))
    return fail(PROTOSEG_ERR_INVALID, "backward kernel '%s': \"wave\", \"fused\" or \"\" (automatic)", name);
  g_bwd_override.store(static_cast<int>(bwd_kernel_of_name(name)), std::memory_order_relaxed);
  return PROTOSEG_OK;
}

extern "C" size_t protoseg_l2_train_operands_bytes(int C, int P, int K, int precision) {
  return train_operands_bytes(C, P, K, train_operands_kind(C, P, K, precision));
}

extern "C" int protoseg_l2_adam_prep_supported(int C, int P, int K, int precision) {
  return K >= 0 && K <= 32 && train_operands_kind(C, P, K, precision) == TrainOperands::kFused ? 1 : 0;
}

extern "C" int protoseg_l2_adam_prep(int C, int P, int K, float eps, int act_kind, int precision, float* protos,
                                     const float* g_protos, float* exp_avg_p, float* exp_avg_sq_p, int32_t* state_p,
                                     float lr_p, float weight_decay_p, float* w_last, const float* g_w,
                                     float* exp_avg_w, float* exp_avg_sq_w, int32_t* state_w, float lr_w,
                                     float weight_decay_w, float beta1, float beta2, float adam_eps, void* operands,
                                     size_t operands_bytes, protoseg_stream_t stream) {
  if (!protoseg_l2_adam_prep_supported(C, P, K, precision))
    return fail(PROTOSEG_ERR_UNSUPPORTED, "adam_prep: C = 64, K <= 32, BF16X3 one-chunk shapes only "
                                          "(protoseg_l2_adam_prep_supported)");
  if (act_kind != PROTOSEG_ACT_LOG && act_kind != PROTOSEG_ACT_LINEAR)
    return fail(PROTOSEG_ERR_INVALID, "adam_prep: act_kind LOG or LINEAR");
  if (!(beta1 >= 0.f && beta1 < 1.f && beta2 >= 0.f && beta2 < 1.f && adam_eps >= 0.f))
    return fail(PROTOSEG_ERR_INVALID, "betas in [0, 1), eps >= 0");
  if (!operands || operands_bytes < train_operands_bytes(C, P, K, TrainOperands::kFused))
    return fail(PROTOSEG_ERR_INVALID, "operands %zu B < %zu B (protoseg_l2_train_operands_bytes)", operands_bytes,
                train_operands_bytes(C, P, K, TrainOperands::kFused));
  AdamPrepArgs a{};
  a.p = protos, a.gp = g_protos, a.mp = exp_avg_p, a.vp = exp_avg_sq_p, a.stp = state_p;
  a.w = K > 0 ? w_last : nullptr, a.gw = K > 0 ? g_w : nullptr, a.mw = K > 0 ? exp_avg_w : nullptr;
  a.vw = K > 0 ? exp_avg_sq_w : nullptr, a.stw = K > 0 ? state_w : nullptr;
  a.P = P, a.K = K;
  a.lr_p = lr_p, a.wd_p = weight_decay_p, a.lr_w = lr_w, a.wd_w = weight_decay_w;
  a.beta1 = beta1, a.beta2 = beta2, a.eps = adam_eps;
  a.w_scale = act_unit(act_kind), a.wt_scale = act_grad_unit(act_kind, eps);
  a.block = static_cast<unsigned char*>(operands);
  return launch_adam_prep_bf16(a, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int protoseg_l2_x_dtype_supported(int C, int P, int K, int x_dtype) {
  if (!protoseg_l2_supported(C, P, K)) return 0;
  if (x_dtype == PROTOSEG_F32 || x_dtype == PROTOSEG_BF16) return 1;
  return x_dtype == PROTOSEG_F16 && use_wide(C, K, P) ? 1 : 0;
}

extern "C" int protoseg_l2_supported(int C, int P, int K) {
  if (C <= 0 || P <= 0 || K < 0) return 0;
  if (!use_wide(C, K, P)) return 1;  // beyond one launch's LDS: prototype chunks
  return (C <= kWideMaxC && P <= kWideMaxP && K <= kWideMaxK) ? 1 : 0;
}

extern "C" int protoseg_l2_max_protos(int C, int precision) {
  if (C <= 0 || precision < PROTOSEG_PREC_BF16X3 || precision > PROTOSEG_PREC_F32) return 0;
  return C <= kWideMaxC ? kWideMaxP : 0;  // the wide family beyond the chunked families' 4096
}

// PROTOSEG_X_SIGMOID in act_kind: x is the add-on's pre-activation and the kernels apply the
// sigmoid on load (model.py:124-128). Served by the bf16 forward and the fused backward only.
bool x_sigmoid_path(int B, int C, int H, int W, int P, int K, int precision) {
  if (precision != PROTOSEG_PREC_BF16X3 || C != 64 || P <= 0 || P > kMaxChunkedP || K < 0 || K > 32) return false;  // not wide
  if (B <= 0 || H <= 0 || W <= 0 || static_cast<long long>(B) * H * W >= (1LL << 31)) return false;
  return bf16_sizes_ok(geometry_of(B, C, H, W, P, K));
}

int split_x_sigmoid(int& act_kind, int B, int C, int H, int W, int P, int K, int precision) {
  const int xsig = (act_kind & PROTOSEG_X_SIGMOID) ? 1 : 0;
  act_kind &= ~PROTOSEG_X_SIGMOID;
  if (xsig && !x_sigmoid_path(B, C, H, W, P, K, precision))
    return -fail(PROTOSEG_ERR_UNSUPPORTED,
                 "PROTOSEG_X_SIGMOID needs precision BF16X3, C = 64 and the bf16 size bounds "
                 "(protoseg_l2_x_sigmoid_supported)");
  return xsig;
}

extern "C" int protoseg_l2_x_sigmoid_supported(int B, int C, int H, int W, int P, int K, int precision) {
  return x_sigmoid_path(B, C, H, W, P, K, precision) ? 1 : 0;
}

namespace {
int l2_fwd_impl(const void* x, int x_dtype, int B, int C, int H, int W, const float* protos, int P, const float* w_last,
                int K, float eps, int act_kind, int precision, float* dist_out, float* act_out, float* logits_out,
                void* operands, size_t operands_bytes, protoseg_stream_t stream) {
  const bool ready = (act_kind & PROTOSEG_OPERANDS_READY) != 0;
  act_kind &= ~PROTOSEG_OPERANDS_READY;
  const int xsig = split_x_sigmoid(act_kind, B, C, H, W, P, K, precision);
  if (xsig < 0) return -xsig;
  Geometry geo;
  if (int st = validate(x, x_dtype, B, C, H, W, protos, P, K, act_kind, precision, &geo)) return st;
  geo.xsig = xsig;
  if (logits_out && (!w_last || K <= 0)) return fail(PROTOSEG_ERR_INVALID, "logits_out needs w_last and K > 0");
  const TrainOperands tk = operands ? train_operands_kind(C, P, K, precision) : TrainOperands::kNone;
  if (ready && (tk != TrainOperands::kFused || !protoseg_l2_adam_prep_supported(C, P, K, precision)))
    return fail(PROTOSEG_ERR_INVALID, "PROTOSEG_OPERANDS_READY needs operands of a shape protoseg_l2_adam_prep serves");
  if (tk != TrainOperands::kNone) {
    if (operands_bytes < train_operands_bytes(C, P, K, tk))
      return fail(PROTOSEG_ERR_INVALID, "operands %zu B < %zu B (protoseg_l2_train_operands_bytes)", operands_bytes,
                  train_operands_bytes(C, P, K, tk));
    if (K > 0 && !w_last) return fail(PROTOSEG_ERR_INVALID, "operands need w_last");
  }
  if (!dist_out && !act_out && !logits_out && tk == TrainOperands::kNone) return PROTOSEG_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const float* w_ops = K > 0 ? w_last : nullptr;  // the backward's W images (g_logits) from the real weights
  if (tk == TrainOperands::kFused) {  // the forward runs on the backward's full image block
    if (!ready)
      if (int st = launch_prep_bf16(geo, 2, protos, w_ops, act_kind, eps, operands, s)) return st;
    if (!dist_out && !act_out && !logits_out) return PROTOSEG_OK;
    if (bf16_fwd_fits(geo, 2))
      return launch_fwd_bf16(geo, x_dtype == PROTOSEG_BF16, 2, x, operands, eps, act_kind, dist_out, act_out,
                             logits_out, s);
  }
  if (use_wide(C, K, P)) {  // any C / K: exact f32 GEMMs (l2_wide.hip), every precision request
    if (xsig) return fail(PROTOSEG_ERR_UNSUPPORTED, "PROTOSEG_X_SIGMOID: C = 64, K <= 32 only");
    if (!wide_family_fits(geo)) return fail(PROTOSEG_ERR_UNSUPPORTED, "B*H*W*max(P, C) >= 2^31 elements");
    void* scratch = nullptr;
    if (int st = stream_block(wide_fwd_scratch_bytes(geo, !dist_out && logits_out), s, 2, &scratch)) return st;
    return launch_fwd_wide(geo, x_dtype, x, protos, w_last, eps, act_kind, dist_out, act_out,
                           logits_out, scratch, s, terms_of(precision) == 2);
  }
  const int terms = terms_of(precision);
  if (terms && bf16_fwd_fits(geo, terms)) {
    // one prep launch: the forward's images
    ImageBlock img;
    if (int st = img.build(geo, terms, protos, logits_out ? w_last : nullptr, act_kind, eps, s, 0, 1)) return st;
    if (!dist_out && !act_out && !logits_out) return PROTOSEG_OK;
    return launch_fwd_bf16(geo, x_dtype == PROTOSEG_BF16, terms, x, img.ptr, eps, act_kind, dist_out, act_out,
                           logits_out, s);
  }
  // P beyond the forward's LDS images (Pp > 384, e.g. 30 prototypes/class): prototype chunks of
  // <= 384. Distance / activation rows land at (b * P + p0 + p); the logits are a sum over
  // prototypes, so chunk c > 0 adds to them.
  if (terms && C == 64 && bf16_sizes_ok(geo)) {
    int nchunk = static_cast<int>(ceil_div(P, 384)), per = 0;
    Geometry gc;
    for (;; ++nchunk) {  // fewest chunks whose images fit (fewer rows per chunk at 3 terms)
      per = static_cast<int>(ceil_div(P, nchunk));
      gc = geometry_of(B, C, H, W, per, K);
      if (bf16_fwd_fits(gc, terms) || per <= 32) break;
    }
    if (nchunk > 1 && bf16_fwd_fits(gc, terms)) {
      KernelSpan span("l2_fwd_bf16_kernel", "", s);
      for (int c = 0; c < nchunk; ++c) {
        const int p0 = c * per, pc = P - p0 < per ? P - p0 : per;
        gc = geometry_of(B, C, H, W, pc, K);
        gc.ldw = gc.ldd = P;
        gc.p0 = p0;
        gc.xsig = xsig;
        ImageBlock img;
        if (int st = img.build(gc, terms, protos + static_cast<size_t>(p0) * C, logits_out ? w_last + p0 : nullptr,
                               act_kind, eps, s, 0, 1))
          return st;
        if (int st = launch_fwd_bf16(gc, x_dtype == PROTOSEG_BF16, terms, x, img.ptr, eps, act_kind, dist_out,
                                     act_out, logits_out, s, c > 0))
          return st;
      }
      return PROTOSEG_OK;
    }
  }
  // the f32 family has no sigmoid-on-load: refuse here, as the backward does, rather than
  // return distances of the pre-activation
  if (xsig) return fail(PROTOSEG_ERR_UNSUPPORTED, "PROTOSEG_X_SIGMOID: no bf16 kernel serves this shape");
  // f32 family: prototype chunks of at most one launch's LDS (C = 64: 384 rows); distance and
  // activation rows at (b * P + p0 + p), logits summed over the chunks
  const int fmax = f32_launch_protos(C);
  const int nchunk = static_cast<int>(ceil_div(P, fmax)), per = static_cast<int>(ceil_div(P, nchunk));
  KernelSpan span(nchunk > 1 ? "l2_fwd_kernel" : "", "", s);
  for (int c = 0; c < nchunk; ++c) {
    const int p0 = c * per, pc = P - p0 < per ? P - p0 : per;
    Geometry gc = geo;
    if (nchunk > 1) {
      gc = geometry_of(B, C, H, W, pc, K);
      gc.ldw = gc.ldd = P;
      gc.p0 = p0;
    }
    const int st = dispatch(x_dtype, C, [&](auto tx, auto nc) {
      using TX = std::remove_pointer_t<decltype(tx)>;
      return launch_fwd<TX, decltype(nc)::value>(gc, x, protos + static_cast<size_t>(p0) * C,
                                                 w_last ? w_last + p0 : nullptr, eps, act_kind, dist_out, act_out,
                                                 logits_out, s, c > 0);
    });
    if (st) return st;
  }
  return PROTOSEG_OK;
}
}  // namespace

extern "C" int protoseg_l2_fwd(const void* x, int x_dtype, int B, int C, int H, int W, const float* protos, int P,
                               const float* w_last, int K, float eps, int act_kind, int precision, float* dist_out,
                               float* act_out, float* logits_out, protoseg_stream_t stream) {
  return l2_fwd_impl(x, x_dtype, B, C, H, W, protos, P, w_last, K, eps, act_kind, precision, dist_out, act_out,
                     logits_out, nullptr, 0, stream);
}

extern "C" int protoseg_l2_fwd_ex(const void* x, int x_dtype, int B, int C, int H, int W, const float* protos, int P,
                                  const float* w_last, int K, float eps, int act_kind, int precision, float* dist_out,
                                  float* act_out, float* logits_out, void* operands, size_t operands_bytes,
                                  protoseg_stream_t stream) {
  return l2_fwd_impl(x, x_dtype, B, C, H, W, protos, P, w_last, K, eps, act_kind, precision, dist_out, act_out,
                     logits_out, operands, operands_bytes, stream);
}

extern "C" size_t protoseg_l2_bwd_workspace_size(int B, int C, int H, int W, int P, int K) {
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || P <= 0) return 0;
  if (static_cast<long long>(B) * H * W >= (1LL << 31)) return 0;
  const Geometry g = geometry_of(B, C, H, W, P, K);
  if (use_wide(C, K, P)) return ((wide_bwd_workspace_bytes(g) + 255) / 256) * 256;
  size_t need = f32_pw_workspace(g);
  const size_t b16 = bf16_bwd_pw_workspace(g);
  if (C == 64 && b16 > need) need = b16;
  if (C == 64) {  // wave backward: one slab per workgroup and prototype chunk of <= 384
    const int nchunk = static_cast<int>(ceil_div(P, 384)), per = static_cast<int>(ceil_div(P, nchunk));
    const Geometry gc = geometry_of(B, C, H, W, per, K);
    if (bf16_bwd_wave_fits(gc, 2)) {
      const size_t q = static_cast<size_t>(nchunk) * bf16_bwd_wave_slab_elems(gc) * sizeof(float);
      if (q > need) need = q;
    }
  }
  if (C == 64) {  // fused backward: one slab per workgroup and prototype chunk (fused_chunks)
    const int nchunk = static_cast<int>(ceil_div(P, 192)), per = static_cast<int>(ceil_div(P, nchunk));
    const Geometry gc = geometry_of(B, C, H, W, per, K);
    const size_t fused = static_cast<size_t>(nchunk) * bf16_bwd_fused_grid(gc) *
                         (static_cast<size_t>(gc.Pp) * C + 32 * gc.Pp + gc.Pp) * sizeof(float);
    if (fused > need) need = fused;
  }
  return ((need + 255) / 256) * 256;
}

namespace {
// The compact KLD gradient (protoseg_l2_bwd_kld) is expanded in the owners of the bf16x3 training
// backward (one-pass and fused kernels), f32 x.
// Not on the wide family (K > 32 or P > 4096 run there): its GEMM chain reads a dense g_dist only.
bool kld_compact_path(const Geometry& geo, int x_dtype, int precision, int mpc) {
  return terms_of(precision) == 2 && geo.C == 64 && !use_wide(geo.C, geo.K, geo.P) && x_dtype == PROTOSEG_F32 &&
         bf16_sizes_ok(geo) && mpc >= 1 &&
         mpc <= 32 && static_cast<long long>(geo.npix) * mpc * 4 < (1LL << 31);
}

int l2_bwd_impl(const void* x, int x_dtype, int B, int C, int H, int W, const float* protos, int P, const float* w_last,
                int K, float eps, int act_kind, int precision, const float* g_logits, const float* g_dist,
                const CompactGd& cgd, void* g_x, float* g_protos, float* g_w, void* workspace, size_t workspace_bytes,
                const void* operands, size_t operands_bytes, protoseg_stream_t stream,
                const float* dist_saved = nullptr) {
  const int xsig = split_x_sigmoid(act_kind, B, C, H, W, P, K, precision);
  if (xsig < 0) return -xsig;
  Geometry geo;
  if (int st = validate(x, x_dtype, B, C, H, W, protos, P, K, act_kind, precision, &geo)) return st;
  if (cgd.val) {
    if (g_dist) return fail(PROTOSEG_ERR_INVALID, "a dense g_dist and the compact KLD gradient together");
    if (!kld_compact_path(geo, x_dtype, precision, cgd.mpc) || !(xsig || (g_x && (g_protos || g_w))))
      return fail(PROTOSEG_ERR_UNSUPPORTED, "compact KLD gradient: needs BF16X3, C = 64, f32 x, g_x and g_protos / g_w "
                                            "(protoseg_l2_bwd_kld_supported)");
  }
  if (g_logits && (!w_last || K <= 0)) return fail(PROTOSEG_ERR_INVALID, "g_logits needs w_last and K > 0");
  if (g_w && !g_logits) return fail(PROTOSEG_ERR_INVALID, "g_w needs g_logits");
  if (g_protos || g_w || xsig || use_wide(C, K, P)) {  // slabs (fused kernel, every X_SIGMOID backward; wide family)
    const size_t need = protoseg_l2_bwd_workspace_size(B, C, H, W, P, K);
    if (!workspace || workspace_bytes < need)
      return fail(PROTOSEG_ERR_INVALID, "workspace %zu B < %zu B", workspace_bytes, need);
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!g_logits && !g_dist && !cgd.val) {  // no upstream gradient: every output is zero
    const size_t esz = x_dtype == PROTOSEG_F32 ? 4 : 2;
    if (g_x && hipMemsetAsync(g_x, 0, static_cast<size_t>(geo.npix) * C * esz, s) != hipSuccess)
      return check_launch("memset g_x");
    if (g_protos && hipMemsetAsync(g_protos, 0, static_cast<size_t>(P) * C * 4, s) != hipSuccess)
      return check_launch("memset g_protos");
    return PROTOSEG_OK;
  }
  const int terms = terms_of(precision);
  const bool xb = x_dtype == PROTOSEG_BF16;
  float* ws = static_cast<float*>(workspace);
  // the forward's prep wrote this backward's images (protoseg_l2_fwd_ex): used when the
  // backward runs the kernel they were built for, in one prototype chunk
  const TrainOperands tk = operands ? train_operands_kind(C, P, K, precision) : TrainOperands::kNone;
  if (tk != TrainOperands::kNone && operands_bytes < train_operands_bytes(C, P, K, tk))
    return fail(PROTOSEG_ERR_INVALID, "operands %zu B < %zu B (protoseg_l2_train_operands_bytes)", operands_bytes,
                train_operands_bytes(C, P, K, tk));
  if (use_wide(C, K, P)) {  // any C / K (l2_wide.hip)
    if (xsig) return fail(PROTOSEG_ERR_UNSUPPORTED, "PROTOSEG_X_SIGMOID: C = 64, K <= 32 only");
    if (cgd.val) return fail(PROTOSEG_ERR_UNSUPPORTED, "compact KLD gradient on the wide family (K > 32 or P > 4096)");
    if (!wide_family_fits(geo)) return fail(PROTOSEG_ERR_UNSUPPORTED, "B*H*W*max(P, C) >= 2^31 elements");
    return launch_bwd_wide(geo, x_dtype, x, protos, w_last, eps, act_kind, g_logits, g_dist, g_x, g_protos,
                           g_logits ? g_w : nullptr, workspace, s, terms == 2, dist_saved);
  }
  // Training backward at bf16x3, wave-owned prototypes (l2_bwd_wave.hip): up to 384 prototypes
  // per launch over the standard operand images, prototype chunks beyond (chunk c > 0 adds its
  // g_x), one slab reduce.
  if (terms == 2 && (xsig || (g_x && (g_protos || g_w))) && bwd_kernel(P) == BwdKernel::kWave) {
    const int nchunk = static_cast<int>(ceil_div(P, 384)), per = static_cast<int>(ceil_div(P, nchunk));
    Geometry gc = geometry_of(B, C, H, W, per, K);
    if (bf16_bwd_wave_fits(gc, terms)) {
      KernelSpan span(nchunk > 1 ? "l2_bwd_wave_bf16_kernel" : "", "", s);
      const size_t cb = bf16_image_bytes(gc, terms);
      const size_t chunk_elems = bf16_bwd_wave_slab_elems(gc);
      const int grid = bf16_bwd_wave_grid(gc);
      ImageBlock img;
      if (tk == TrainOperands::kFused && nchunk == 1)
        img.ptr = const_cast<void*>(operands);
      else if (int st = img.build(geo, terms, protos, g_logits ? w_last : nullptr, act_kind, eps, s, per))
        return st;
      for (int c = 0; c < nchunk; ++c) {
        const int p0 = c * per, pc = P - p0 < per ? P - p0 : per;
        Geometry gq = geometry_of(B, C, H, W, pc, K);
        gq.ldw = gq.ldd = P;
        gq.p0 = p0;
        gq.xsig = xsig;
        gq.cgd = cgd;
        gq.protos = protos;
        if (int st = launch_bwd_wave_bf16(gq, xb, x, static_cast<unsigned char*>(img.ptr) + c * cb, eps, act_kind,
                                          g_logits, g_dist, g_x, ws + c * chunk_elems, s, c > 0))
          return st;
      }
      return launch_bwd_reduce_bf16_chunks(geo, per, nchunk, ws, grid, chunk_elems, protos, act_kind, g_protos,
                                           g_logits ? g_w : nullptr, s, 2);
    }
  }
  // Training backward (g_x and g_P / g_W) at bf16x3: one fused kernel per chunk of <= 192
  // prototypes (l2_bwd_fused.hip); chunk c > 0 adds its x-gradient to g_x.
  if (terms == 2 && C == 64 && bf16_sizes_ok(geo) && (xsig || (g_x && (g_protos || g_w)))) {
    const int nchunk = static_cast<int>(ceil_div(P, 192));
    const int per = static_cast<int>(ceil_div(P, nchunk));
    Geometry gc = geometry_of(B, C, H, W, per, K);
    if (bf16_bwd_fused_fits(gc, terms)) {
      // One prep launch for every chunk's images, the chunks' fused kernels (each its own slab
      // region; chunk c > 0 adds its g_x), one reduce launch over all chunks' slabs.
      KernelSpan span(nchunk > 1 ? "l2_bwd_fused_bf16_kernel" : "", "", s);
      const size_t cb = bf16_image_bytes(gc, terms);
      const int grid = bf16_bwd_fused_grid(gc);
      const size_t chunk_elems = static_cast<size_t>(grid) * (static_cast<size_t>(gc.Pp) * C + 32 * gc.Pp + gc.Pp);
      Geometry gall = geometry_of(B, C, H, W, P, K);
      ImageBlock img;
      if (tk == TrainOperands::kFused && nchunk == 1)
        img.ptr = const_cast<void*>(operands);
      else if (int st = img.build(gall, terms, protos, g_logits ? w_last : nullptr, act_kind, eps, s, per))
        return st;
      for (int c = 0; c < nchunk; ++c) {
        const int p0 = c * per, pc = P - p0 < per ? P - p0 : per;
        gc = geometry_of(B, C, H, W, pc, K);
        gc.ldw = gc.ldd = P;
        gc.p0 = p0;
        gc.xsig = xsig;
        gc.cgd = cgd;
        if (int st = launch_bwd_fused_bf16(gc, xb, x, protos + static_cast<size_t>(p0) * C,
                                           static_cast<unsigned char*>(img.ptr) + c * cb, eps, act_kind, g_logits,
                                           g_dist, g_x, nullptr, nullptr, ws + c * chunk_elems, s, c > 0, 0))
          return st;
      }
      return launch_bwd_reduce_bf16_chunks(gall, per, nchunk, ws, grid, chunk_elems, protos, act_kind, g_protos,
                                           g_logits ? g_w : nullptr, s);
    }
  }
  if (xsig) return fail(PROTOSEG_ERR_UNSUPPORTED, "PROTOSEG_X_SIGMOID: no fused backward for this shape");
  if (cgd.val) return fail(PROTOSEG_ERR_UNSUPPORTED, "compact KLD gradient: no fused backward for this shape");
  // P too large for the bf16 backward's LDS images (e.g. P = 361, 19 prototypes/class): run it
  // over prototype chunks of <= 192. g_P rows and g_W columns are per prototype; g_x is a sum
  // over prototypes, so chunk c > 0 adds to it; g_dist rows are read at (b * P + p0 + p).
  if (terms && C == 64 && !bf16_bwd_x_fits(geo, terms)) {
    int nchunk = static_cast<int>(ceil_div(P, 192)), per = 0;
    Geometry gc;
    for (;; ++nchunk) {  // fewest chunks whose images fit (fewer rows per chunk at 3 terms)
      per = static_cast<int>(ceil_div(P, nchunk));
      gc = geometry_of(B, C, H, W, per, K);
      if ((bf16_bwd_x_fits(gc, terms) && bf16_bwd_pw_fits(gc, terms)) || per <= 32) break;
    }
    if (nchunk > 1 && bf16_bwd_x_fits(gc, terms) && bf16_bwd_pw_fits(gc, terms) && bf16_sizes_ok(geo)) {
      KernelSpan span(g_x ? "l2_bwd_x_bf16_kernel" : "", (g_protos || g_w) ? "l2_bwd_pw_bf16_kernel" : "", s);
      for (int c = 0; c < nchunk; ++c) {
        const int p0 = c * per, pc = P - p0 < per ? P - p0 : per;
        gc = geometry_of(B, C, H, W, pc, K);
        gc.ldw = gc.ldd = P;
        gc.p0 = p0;
        const float* wc = g_logits ? w_last + p0 : nullptr;
        ImageBlock img;
        if (int st = img.build(gc, terms, protos + static_cast<size_t>(p0) * C, wc, act_kind, eps, s)) return st;
        if (g_x)
          if (int st = launch_bwd_x_bf16(gc, xb, terms, x, img.ptr, eps, act_kind, g_logits, g_dist, g_x, s, c > 0))
            return st;
        if (g_protos || g_w)
          if (int st = launch_bwd_pw_bf16(gc, xb, terms, x, protos + static_cast<size_t>(p0) * C, img.ptr, eps,
                                          act_kind, g_logits, g_dist,
                                          g_protos ? g_protos + static_cast<size_t>(p0) * C : nullptr,
                                          g_w ? g_w + p0 : nullptr, ws, s))
            return st;
      }
      return PROTOSEG_OK;
    }
  }
  const bool bf16_x = g_x && terms && bf16_bwd_x_fits(geo, terms);
  const bool bf16_pw = (g_protos || g_w) && terms && bf16_bwd_pw_fits(geo, terms);
  ImageBlock img;
  if (bf16_x || bf16_pw)
    if (int st = img.build(geo, terms, protos, g_logits ? w_last : nullptr, act_kind, eps, s)) return st;
  if (g_x) {
    int st;
    if (bf16_x)
      st = launch_bwd_x_bf16(geo, xb, terms, x, img.ptr, eps, act_kind, g_logits, g_dist, g_x, s);
    else {  // f32 family: prototype chunks of one launch's LDS, chunk c > 0 adds to g_x
      const int fmax = f32_launch_protos(C);
      const int nchunk = static_cast<int>(ceil_div(P, fmax)), per = static_cast<int>(ceil_div(P, nchunk));
      KernelSpan span(nchunk > 1 ? "l2_bwd_x_kernel" : "", "", s);
      st = PROTOSEG_OK;
      for (int c = 0; c < nchunk && !st; ++c) {
        const int p0 = c * per, pc = P - p0 < per ? P - p0 : per;
        Geometry gc = geo;
        if (nchunk > 1) {
          gc = geometry_of(B, C, H, W, pc, K);
          gc.ldw = gc.ldd = P;
          gc.p0 = p0;
        }
        st = dispatch(x_dtype, C, [&](auto tx, auto nc) {
          using TX = std::remove_pointer_t<decltype(tx)>;
          return launch_bwd_x<TX, decltype(nc)::value>(gc, x, protos + static_cast<size_t>(p0) * C,
                                                       g_logits ? w_last + p0 : w_last, eps, act_kind, g_logits,
                                                       g_dist, g_x, s, c > 0);
        });
      }
    }
    if (st) return st;
  }
  if (g_protos || g_w) {
    if (bf16_pw)
      return launch_bwd_pw_bf16(geo, xb, terms, x, protos, img.ptr, eps, act_kind, g_logits, g_dist, g_protos, g_w, ws,
                                s);
    return dispatch(x_dtype, C, [&](auto tx, auto nc) {
      using TX = std::remove_pointer_t<decltype(tx)>;
      return launch_bwd_pw<TX, decltype(nc)::value>(geo, x, protos, w_last, eps, act_kind, g_logits, g_dist, g_protos,
                                                    g_w, ws, s);
    });
  }
  return PROTOSEG_OK;
}
}  // namespace

extern "C" int protoseg_l2_bwd(const void* x, int x_dtype, int B, int C, int H, int W, const float* protos, int P,
                               const float* w_last, int K, float eps, int act_kind, int precision,
                               const float* g_logits, const float* g_dist, void* g_x, float* g_protos, float* g_w,
                               void* workspace, size_t workspace_bytes, protoseg_stream_t stream) {
  return l2_bwd_impl(x, x_dtype, B, C, H, W, protos, P, w_last, K, eps, act_kind, precision, g_logits, g_dist,
                     CompactGd{}, g_x, g_protos, g_w, workspace, workspace_bytes, nullptr, 0, stream);
}

extern "C" int protoseg_l2_bwd_reads_dist(int C, int P, int K, int precision) {
  if (precision < PROTOSEG_PREC_BF16X3 || precision > PROTOSEG_PREC_F32) return 0;
  return protoseg_l2_supported(C, P, K) && use_wide(C, K, P) ? 1 : 0;
}

extern "C" int protoseg_l2_bwd_saved(const void* x, int x_dtype, int B, int C, int H, int W, const float* protos,
                                     int P, const float* w_last, int K, float eps, int act_kind, int precision,
                                     const float* dist, const float* g_logits, const float* g_dist, void* g_x,
                                     float* g_protos, float* g_w, void* workspace, size_t workspace_bytes,
                                     protoseg_stream_t stream) {
  if (!dist) return fail(PROTOSEG_ERR_INVALID, "protoseg_l2_bwd_saved: dist is null");
  return l2_bwd_impl(x, x_dtype, B, C, H, W, protos, P, w_last, K, eps, act_kind, precision, g_logits, g_dist,
                     CompactGd{}, g_x, g_protos, g_w, workspace, workspace_bytes, nullptr, 0, stream,
                     protoseg_l2_bwd_reads_dist(C, P, K, precision) ? dist : nullptr);
}

extern "C" int protoseg_l2_bwd_ex(const void* x, int x_dtype, int B, int C, int H, int W, const float* protos, int P,
                                  const float* w_last, int K, float eps, int act_kind, int precision,
                                  const float* g_logits, const float* g_dist, void* g_x, float* g_protos, float* g_w,
                                  void* workspace, size_t workspace_bytes, const void* operands,
                                  size_t operands_bytes, protoseg_stream_t stream) {
  return l2_bwd_impl(x, x_dtype, B, C, H, W, protos, P, w_last, K, eps, act_kind, precision, g_logits, g_dist,
                     CompactGd{}, g_x, g_protos, g_w, workspace, workspace_bytes, operands, operands_bytes, stream);
}

extern "C" int protoseg_l2_bwd_kld_supported(int B, int C, int H, int W, int P, int K, int x_dtype, int precision,
                                             int max_per_class) {
  if (B <= 0 || H <= 0 || W <= 0 || P <= 0 || !protoseg_l2_supported(C, P, K)) return 0;
  if (static_cast<long long>(B) * H * W >= (1LL << 31)) return 0;
  return kld_compact_path(geometry_of(B, C, H, W, P, K), x_dtype, precision, max_per_class) ? 1 : 0;
}

extern "C" int protoseg_l2_bwd_kld(const void* x, int x_dtype, int B, int C, int H, int W, const float* protos, int P,
                                   const float* w_last, int K, float eps, int act_kind, int precision,
                                   const float* g_logits, const float* g_cls, const int32_t* pix_cls,
                                   const int32_t* proto_slot, int max_per_class, void* g_x, float* g_protos,
                                   float* g_w, void* workspace, size_t workspace_bytes, protoseg_stream_t stream) {
  return protoseg_l2_bwd_kld_ex(x, x_dtype, B, C, H, W, protos, P, w_last, K, eps, act_kind, precision, g_logits,
                                g_cls, pix_cls, proto_slot, max_per_class, g_x, g_protos, g_w, workspace,
                                workspace_bytes, nullptr, 0, stream);
}

extern "C" int protoseg_l2_bwd_kld_ex(const void* x, int x_dtype, int B, int C, int H, int W, const float* protos,
                                      int P, const float* w_last, int K, float eps, int act_kind, int precision,
                                      const float* g_logits, const float* g_cls, const int32_t* pix_cls,
                                      const int32_t* proto_slot, int max_per_class, void* g_x, float* g_protos,
                                      float* g_w, void* workspace, size_t workspace_bytes, const void* operands,
                                      size_t operands_bytes, protoseg_stream_t stream) {
  if (!g_cls || !pix_cls || !proto_slot) return fail(PROTOSEG_ERR_INVALID, "g_cls, pix_cls and proto_slot must be non-null");
  CompactGd cgd;
  cgd.val = g_cls;
  cgd.pix = pix_cls;
  cgd.slot = proto_slot;
  cgd.mpc = max_per_class;
  return l2_bwd_impl(x, x_dtype, B, C, H, W, protos, P, w_last, K, eps, act_kind, precision, g_logits, nullptr, cgd,
                     g_x, g_protos, g_w, workspace, workspace_bytes, operands, operands_bytes, stream);
}
