// l2_bf16.hip — the prototype layer on bf16 MFMA with split operands (bf16_split.h), C = 64.
//
// Same math and outputs as the f32-MFMA family in l2_layer.hip (reference model.py:203-237,
// 259-283 and their autograd), at 5.3x (T=2) / 2.7x (T=3) fewer matrix-core cycles, which
// moves the forward from MFMA-bound to HBM-bound (the D write dominates its bytes).
//
//   l2_fwd_bf16_kernel     layout A (rows p, cols n): distances -> NCHW stores, activation in
//                          registers, logits = W . act with the accumulator as B operand.
//   l2_bwd_x_bf16_kernel   layout A: recompute S, g_act = W^T g_logits^T, g_s, and
//                          g_x^T = P^T (-2 g_s) with the accumulator as B operand.
//   l2_bwd_pw_bf16_kernel  layout B (rows n, cols p): one workgroup = S streams x npt waves,
//                          wave (stream, w) owns prototype tile w; each 32-pixel tile is read
//                          from HBM once, staged in LDS as bf16 images, and shared by the
//                          npt waves; g_P^T and g_W accumulate in registers (the accumulator
//                          is their A / B operand), one partial slab per workgroup.
//   l2_bwd_reduce_bf16_kernel  deterministic parallel sum of the slabs (+ 2p * sum g_s).
#include "bf16_split.h"
#include "l2_launch.h"
#include "protoseg_host.h"

namespace protoseg {

namespace {

constexpr int kC = 64;         // channels of the bf16 family
constexpr int kNQ = kC / 16;   // channel k-steps of 16
constexpr int kWavesA = 8;     // layout-A kernels: 8 waves, one 32-pixel tile each at a time
constexpr int kLdf = 33;       // padded fp32 staging rows

template <typename TX>
__device__ __forceinline__ float ldx(const TX* p, size_t i) { return XIO<TX>::load(p, i); }

// P image [T][Pp][64]: row p natural channel chunks (CPR 8) — A operand of S (layout A).
template <int T>
__device__ void stage_p_rows(bf16* img, const float* __restrict__ protos, int P, int Pp) {
  const int plane = Pp * kC;
  for (int idx = threadIdx.x; idx < Pp * 8; idx += blockDim.x) {
    const int p = idx >> 3, q8 = idx & 7;
    float v[8];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) v[jj] = p < P ? protos[static_cast<size_t>(p) * kC + q8 * 8 + jj] : 0.f;
    bf16x8 f[T];
    split8<T>(v, f);
    store_frag<T>(img, plane, img_off<8>(p, q8), f);
  }
}

// P^T image [T][npt][64 c][32 p-permuted] (CPR 4) — A operand of g_x^T = P^T g_s.
template <int T>
__device__ void stage_pt_perm(bf16* img, const float* __restrict__ protos, int P, int Pp) {
  const int plane = Pp * kC;
  for (int idx = threadIdx.x; idx < (Pp / 32) * kC * 4; idx += blockDim.x) {
    const int pt = idx / (kC * 4), c = (idx >> 2) & (kC - 1), e8 = idx & 3;
    float v[8];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const int p = pt * 32 + perm_of(e8 * 8 + jj);
      v[jj] = p < P ? protos[static_cast<size_t>(p) * kC + c] : 0.f;
    }
    bf16x8 f[T];
    split8<T>(v, f);
    store_frag<T>(img, plane, img_off<4>(pt * kC + c, e8), f);
  }
}

// W image [T][npt][32 k][32 p-permuted] (CPR 4) — A operand of logits = W . act.
template <int T>
__device__ void stage_w_perm(bf16* img, const float* __restrict__ w, int K, int P, int Pp) {
  const int plane = Pp * 32;
  for (int idx = threadIdx.x; idx < Pp * 4; idx += blockDim.x) {
    const int row = idx >> 2, e8 = idx & 3;  // row = pt*32 + k
    const int pt = row >> 5, k = row & 31;
    float v[8];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const int p = pt * 32 + perm_of(e8 * 8 + jj);
      v[jj] = (k < K && p < P) ? w[static_cast<size_t>(k) * P + p] : 0.f;
    }
    bf16x8 f[T];
    split8<T>(v, f);
    store_frag<T>(img, plane, img_off<4>(row, e8), f);
  }
}

// W^T image [T][Pp][32 k] natural classes (CPR 4) — A operand of g_act^T = W^T g_logits^T.
template <int T>
__device__ void stage_wt_rows(bf16* img, const float* __restrict__ w, int K, int P, int Pp) {
  const int plane = Pp * 32;
  for (int idx = threadIdx.x; idx < Pp * 4; idx += blockDim.x) {
    const int p = idx >> 2, e8 = idx & 3;
    float v[8];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const int k = e8 * 8 + jj;
      v[jj] = (k < K && p < P) ? w[static_cast<size_t>(k) * P + p] : 0.f;
    }
    bf16x8 f[T];
    split8<T>(v, f);
    store_frag<T>(img, plane, img_off<4>(p, e8), f);
  }
}

// ||p||^2 exactly as the f32 family (sequential, no contraction) so that every kernel
// computes bit-identical distances for the same inputs.
__device__ float proto_norm2_64(const float* __restrict__ protos, int p, bool valid) {
#pragma clang fp contract(off)
  float s = 0.f;
  if (valid) {
    for (int c = 0; c < kC; ++c) {
      const float v = protos[static_cast<size_t>(p) * kC + c];
      s += v * v;
    }
  }
  return s;
}

// Layout-A x tile of this lane: xb[q] = x[16q + 8h + 0..7][pixel j] split in T terms;
// returns ||x||^2 (f32 fma chain over the lane's half of the channels, then the two halves).
template <typename TX, int T>
__device__ __forceinline__ float load_x_frags(const TX* __restrict__ x, int b, int n, int HW, bool valid,
                                              bf16x8 (&xb)[kNQ][T]) {
  const int h = (threadIdx.x & 63) >> 5;
  const TX* xh = x + (static_cast<size_t>(b) * kC + 8 * h) * HW + n;
  float x2 = 0.f;
#pragma unroll
  for (int q = 0; q < kNQ; ++q) {
    float v[8];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const float t = ldx(xh, static_cast<size_t>(16 * q + jj) * HW);
      v[jj] = valid ? t : 0.f;
      x2 = fmaf(v[jj], v[jj], x2);
    }
    split8<T>(v, xb[q]);
  }
  x2 += __shfl_xor(x2, 32);
  return x2;
}

template <typename TX, int T>
__global__ __launch_bounds__(kWavesA * 64) void l2_fwd_bf16_kernel(
    const TX* __restrict__ x, int HW, int npix, const float* __restrict__ protos, int P, int Pp,
    const float* __restrict__ w_last, int K, float eps, int act_kind, float* __restrict__ dist,
    float* __restrict__ act_out, float* __restrict__ logits) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  bf16* Pimg = reinterpret_cast<bf16*>(smem_raw);                // [T][Pp][64]
  bf16* Wimg = Pimg + T * Pp * kC;                               // [T][Pp][32]
  float* p2s = reinterpret_cast<float*>(Wimg + T * Pp * 32);     // [Pp]
  const bool do_logits = logits != nullptr;
  stage_p_rows<T>(Pimg, protos, P, Pp);
  if (do_logits) stage_w_perm<T>(Wimg, w_last, K, P, Pp);
  for (int p = threadIdx.x; p < Pp; p += blockDim.x) p2s[p] = proto_norm2_64(protos, p, p < P);
  __syncthreads();

  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5, wave = threadIdx.x >> 6;
  const int ntiles = (npix + 31) / 32;
  const int npt = Pp / 32;
  for (int t = blockIdx.x * kWavesA + wave; t < ntiles; t += gridDim.x * kWavesA) {
    const int g = t * 32 + j;
    const bool valid = g < npix;
    const int b = valid ? g / HW : 0;
    const int n = valid ? g - b * HW : 0;
    bf16x8 xb[kNQ][T];
    const float x2 = load_x_frags<TX, T>(x, b, n, HW, valid, xb);

    f32x16 lacc = zero16();
#pragma unroll 1
    for (int pt = 0; pt < npt; ++pt) {
      f32x16 acc = zero16();
#pragma unroll
      for (int q = 0; q < kNQ; ++q) {
        bf16x8 pa[T];
        load_frag<T>(Pimg, Pp * kC, img_off<8>(pt * 32 + j, 2 * q + h), pa);
        acc = mma_split<T>(pa, xb[q], acc);
      }
      float* dpt = dist ? dist + (static_cast<size_t>(b) * P + pt * 32 + 4 * h) * HW + n : nullptr;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int p = pt * 32 + acc_row(r, h);
        const float d = l2_distance(x2, p2s[p], acc[r]);
        const bool st = valid && p < P;
        if (dpt && st) dpt[static_cast<size_t>(row_of(r)) * HW] = d;
        const float a = activation(d, eps, act_kind);
        if (act_out && st) act_out[static_cast<size_t>(g) * P + p] = a;
        acc[r] = a;
      }
      if (do_logits) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 ab[T], wa[T];
          acc_operand<T>(acc, s, ab);
          load_frag<T>(Wimg, Pp * 32, img_off<4>(pt * 32 + j, 2 * s + h), wa);
          lacc = mma_split<T>(wa, ab, lacc);
        }
      }
    }
    if (do_logits && valid) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int k = acc_row(r, h);
        if (k < K) logits[static_cast<size_t>(g) * K + k] = lacc[r];
      }
    }
  }
}

template <typename TX, int T>
__global__ __launch_bounds__(kWavesA * 64) void l2_bwd_x_bf16_kernel(
    const TX* __restrict__ x, int HW, int npix, const float* __restrict__ protos, int P, int Pp,
    const float* __restrict__ w_last, int K, float eps, int act_kind, const float* __restrict__ g_logits,
    const float* __restrict__ g_dist, TX* __restrict__ g_x) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  bf16* Pimg = reinterpret_cast<bf16*>(smem_raw);                 // [T][Pp][64]
  bf16* PTimg = Pimg + T * Pp * kC;                               // [T][npt*64][32]
  bf16* WTimg = PTimg + T * Pp * kC;                              // [T][Pp][32]
  float* p2s = reinterpret_cast<float*>(WTimg + T * Pp * 32);     // [Pp]
  stage_p_rows<T>(Pimg, protos, P, Pp);
  stage_pt_perm<T>(PTimg, protos, P, Pp);
  if (g_logits) stage_wt_rows<T>(WTimg, w_last, K, P, Pp);
  for (int p = threadIdx.x; p < Pp; p += blockDim.x) p2s[p] = proto_norm2_64(protos, p, p < P);
  __syncthreads();

  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5, wave = threadIdx.x >> 6;
  const int ntiles = (npix + 31) / 32;
  const int npt = Pp / 32;
  const int KS = (K + 15) / 16;  // class k-steps of 16
  for (int t = blockIdx.x * kWavesA + wave; t < ntiles; t += gridDim.x * kWavesA) {
    const int g = t * 32 + j;
    const bool valid = g < npix;
    const int b = valid ? g / HW : 0;
    const int n = valid ? g - b * HW : 0;
    bf16x8 xb[kNQ][T];
    const float x2 = load_x_frags<TX, T>(x, b, n, HW, valid, xb);
    // B operand of g_act^T: lane (h, j) holds g_logits[pixel j][16s + 8h + jj]
    bf16x8 glb[2][T];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float v[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int k = 16 * s + 8 * h + jj;
        const bool ok = g_logits && valid && k < K;
        const float t0 = g_logits ? g_logits[ok ? static_cast<size_t>(g) * K + k : 0] : 0.f;
        v[jj] = ok ? t0 : 0.f;
      }
      split8<T>(v, glb[s]);
    }

    f32x16 gx[2] = {zero16(), zero16()};
    float gsum = 0.f;
#pragma unroll 1
    for (int pt = 0; pt < npt; ++pt) {
      f32x16 acc = zero16();
#pragma unroll
      for (int q = 0; q < kNQ; ++q) {
        bf16x8 pa[T];
        load_frag<T>(Pimg, Pp * kC, img_off<8>(pt * 32 + j, 2 * q + h), pa);
        acc = mma_split<T>(pa, xb[q], acc);
      }
      f32x16 gacc = zero16();
      if (g_logits) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          if (s < KS) {
            bf16x8 wa[T];
            load_frag<T>(WTimg, Pp * 32, img_off<4>(pt * 32 + j, 2 * s + h), wa);
            gacc = mma_split<T>(wa, glb[s], gacc);
          }
        }
      }
      const float* gdpt = g_dist ? g_dist + (static_cast<size_t>(b) * P + pt * 32 + 4 * h) * HW + n : nullptr;
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
        const float gs = (d > 0.f && p < P) ? gd : 0.f;
        gsum += gs;
        acc[r] = -2.f * gs;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 gsb[T];
        acc_operand<T>(acc, s, gsb);
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          bf16x8 pa[T];
          load_frag<T>(PTimg, Pp * kC, img_off<4>(pt * kC + ct * 32 + j, 2 * s + h), pa);
          gx[ct] = mma_split<T>(pa, gsb, gx[ct]);
        }
      }
    }
    gsum += __shfl_xor(gsum, 32);
    if (valid) {
      const TX* xh = x + (static_cast<size_t>(b) * kC + 4 * h) * HW + n;
      TX* gxh = g_x + (static_cast<size_t>(b) * kC + 4 * h) * HW + n;
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const size_t off = static_cast<size_t>(ct * 32 + row_of(r)) * HW;
          XIO<TX>::store(gxh, off, gx[ct][r] + gsum * (2.f * ldx(xh, off)));
        }
    }
  }
}

// ---- bwd_pw: per-stream LDS staging area ------------------------------------------------
template <int T>
struct PwStage {
  static constexpr int kXf = kC * kLdf;        // fp32 [64][33]
  static constexpr int kGf = 32 * kLdf;        // fp32 [32][33]
  static constexpr int kXA = T * 32 * kC;      // bf16 [T][32 n][64 c]   CPR 8
  static constexpr int kXB = T * kC * 32;      // bf16 [T][64 c][32 n~]  CPR 4, permuted n
  static constexpr int kGA = T * 32 * 32;      // bf16 [T][32 n][32 k]   CPR 4
  static constexpr int kGT = T * 32 * 32;      // bf16 [T][32 k][32 n~]  CPR 4, permuted n
  // byte layout: Xf | Gf | x2[32] | rowb[32] | rown[32] | XA | XB | GA | GT
  static constexpr int kBytes = (kXf + kGf + 32) * 4 + 2 * 32 * 4 + (kXA + kXB + kGA + kGT) * 2;
};

template <int T>
__device__ __forceinline__ void pw_carve(unsigned char* base, float*& Xf, float*& Gf, float*& x2s, int*& rowb,
                                         int*& rown, bf16*& XA, bf16*& XB, bf16*& GA, bf16*& GT) {
  using S = PwStage<T>;
  Xf = reinterpret_cast<float*>(base);
  Gf = Xf + S::kXf;
  x2s = Gf + S::kGf;
  rowb = reinterpret_cast<int*>(x2s + 32);
  rown = rowb + 32;
  XA = reinterpret_cast<bf16*>(rown + 32);
  XB = XA + S::kXA;
  GA = XB + S::kXB;
  GT = GA + S::kGA;
}

template <typename TX, int T>
__global__ __launch_bounds__(768) void l2_bwd_pw_bf16_kernel(
    const TX* __restrict__ x, int HW, int npix, const float* __restrict__ protos, int P, int Pp,
    const float* __restrict__ w_last, int K, float eps, int act_kind, const float* __restrict__ g_logits,
    const float* __restrict__ g_dist, int streams, float* __restrict__ slab) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int npt = Pp / 32;
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5, wave = threadIdx.x >> 6;
  const int stream = wave / npt;                 // which pixel stream this wave works on
  const int w = wave - stream * npt;             // prototype tile owned by this wave
  const int nt_stream = npt * 64;                // threads per stream
  const int tid_s = threadIdx.x - stream * nt_stream;
  // LDS: [P image | W^T image | stream staging areas]. P rows (B operand of S) and W^T rows
  // (B operand of g_act) are read per tile from LDS rather than held in registers.
  bf16* Pimg = reinterpret_cast<bf16*>(smem_raw);      // [T][Pp][64]  CPR 8
  bf16* WTimg = Pimg + T * Pp * kC;                    // [T][Pp][32]  CPR 4
  unsigned char* stage_root = reinterpret_cast<unsigned char*>(WTimg + T * Pp * 32);
  stage_p_rows<T>(Pimg, protos, P, Pp);
  stage_wt_rows<T>(WTimg, w_last, g_logits ? K : 0, P, Pp);
  unsigned char* stage_base = stage_root + static_cast<size_t>(stream) * PwStage<T>::kBytes;
  float *Xf, *Gf, *x2s;
  int *rowb, *rown;
  bf16 *XA, *XB, *GA, *GT;
  pw_carve<T>(stage_base, Xf, Gf, x2s, rowb, rown, XA, XB, GA, GT);

  const int p = w * 32 + j;  // this lane's prototype column
  const bool pvalid = p < P;
  const float p2 = proto_norm2_64(protos, p, pvalid);
  const int KS = (K + 15) / 16;

  f32x16 gp[2] = {zero16(), zero16()};
  f32x16 gw = zero16();
  float gsum = 0.f;

  const int ntiles = (npix + 31) / 32;
  const int total_streams = gridDim.x * streams;
  const int my_stream = blockIdx.x * streams + stream;
  const int iters = (ntiles + total_streams - 1) / total_streams;  // uniform across the workgroup
  for (int it = 0; it < iters; ++it) {
    const int t = my_stream + it * total_streams;
    const bool tile_ok = t < ntiles;
    // ---- stage: global -> fp32 LDS (coalesced along pixels) ----
    __syncthreads();  // previous tile's operand reads are done
    for (int idx = tid_s; idx < kC * 32; idx += nt_stream) {
      const int c = idx >> 5, nn = idx & 31;
      const int g = t * 32 + nn;
      const bool ok = tile_ok && g < npix;
      const int b = ok ? g / HW : 0;
      const int n = ok ? g - b * HW : 0;
      const float v = ldx(x, (static_cast<size_t>(b) * kC + c) * HW + n);
      Xf[c * kLdf + nn] = ok ? v : 0.f;
      if (c == 0) {
        rowb[nn] = ok ? b : -1;
        rown[nn] = n;
      }
    }
    for (int idx = tid_s; idx < 32 * 32; idx += nt_stream) {
      const int nn = idx >> 5, k = idx & 31;
      const int g = t * 32 + nn;
      const bool ok = g_logits && tile_ok && g < npix && k < K;
      const float v = g_logits ? g_logits[ok ? static_cast<size_t>(g) * K + k : 0] : 0.f;
      Gf[nn * kLdf + k] = ok ? v : 0.f;
    }
    __syncthreads();
    // ---- convert to split bf16 operand images ----
    for (int idx = tid_s; idx < 32 * 8; idx += nt_stream) {  // XA: row n, chunk q8
      const int nn = idx >> 3, q8 = idx & 7;
      float v[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) v[jj] = Xf[(q8 * 8 + jj) * kLdf + nn];
      bf16x8 f[T];
      split8<T>(v, f);
      store_frag<T>(XA, 32 * kC, img_off<8>(nn, q8), f);
    }
    for (int idx = tid_s; idx < kC * 4; idx += nt_stream) {  // XB: row c, permuted pixels
      const int c = idx >> 2, e8 = idx & 3;
      float v[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) v[jj] = Xf[c * kLdf + perm_of(e8 * 8 + jj)];
      bf16x8 f[T];
      split8<T>(v, f);
      store_frag<T>(XB, kC * 32, img_off<4>(c, e8), f);
    }
    for (int idx = tid_s; idx < 32 * 4; idx += nt_stream) {  // GA: row n, classes; GT: row k, permuted n
      const int r = idx >> 2, e8 = idx & 3;
      float v[8], u[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        v[jj] = Gf[r * kLdf + e8 * 8 + jj];
        u[jj] = Gf[perm_of(e8 * 8 + jj) * kLdf + r];
      }
      bf16x8 f[T], ft[T];
      split8<T>(v, f);
      split8<T>(u, ft);
      store_frag<T>(GA, 32 * 32, img_off<4>(r, e8), f);
      store_frag<T>(GT, 32 * 32, img_off<4>(r, e8), ft);
    }
    if (tid_s < 32) {  // ||x||^2 per pixel, the same chain as load_x_frags
      const int nn = tid_s;
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int q = 0; q < kNQ; ++q)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          const float a = Xf[(16 * q + jj) * kLdf + nn], c = Xf[(16 * q + 8 + jj) * kLdf + nn];
          s0 = fmaf(a, a, s0);
          s1 = fmaf(c, c, s1);
        }
      x2s[nn] = s0 + s1;
    }
    __syncthreads();

    // ---- compute: this wave's prototype tile against the staged pixel tile ----
    f32x16 acc = zero16();
#pragma unroll
    for (int q = 0; q < kNQ; ++q) {
      bf16x8 xa[T], pb[T];
      load_frag<T>(XA, 32 * kC, img_off<8>(j, 2 * q + h), xa);
      load_frag<T>(Pimg, Pp * kC, img_off<8>(p, 2 * q + h), pb);
      acc = mma_split<T>(xa, pb, acc);
    }
    f32x16 gacc = zero16();
    if (g_logits) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if (s < KS) {
          bf16x8 ga[T], wb[T];
          load_frag<T>(GA, 32 * 32, img_off<4>(j, 2 * s + h), ga);
          load_frag<T>(WTimg, Pp * 32, img_off<4>(p, 2 * s + h), wb);
          gacc = mma_split<T>(ga, wb, gacc);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int nr = acc_row(r, h);
      const int br = rowb[nr];
      const bool rvalid = br >= 0;
      const float d = l2_distance(x2s[nr], p2, acc[r]);
      const float a = activation(d, eps, act_kind);
      float gd = g_logits ? gacc[r] * activation_grad(d, eps, act_kind) : 0.f;
      if (g_dist) {
        const bool ok = rvalid && pvalid;
        const float v = g_dist[ok ? (static_cast<size_t>(br) * P + p) * HW + rown[nr] : 0];
        gd += ok ? v : 0.f;
      }
      const float gs = (d > 0.f && pvalid && rvalid) ? gd : 0.f;
      gsum += gs;
      acc[r] = -2.f * gs;
      gacc[r] = rvalid ? a : 0.f;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 gsa[T], actb[T];
      acc_operand<T>(acc, s, gsa);   // A of g_P^T: lane = prototype, k = pixels (permuted)
      acc_operand<T>(gacc, s, actb); // B of g_W:   lane = prototype, k = pixels (permuted)
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        bf16x8 xbf[T];
        load_frag<T>(XB, kC * 32, img_off<4>(ct * 32 + j, 2 * s + h), xbf);
        gp[ct] = mma_split<T>(gsa, xbf, gp[ct]);
      }
      if (g_logits) {
        bf16x8 gt[T];
        load_frag<T>(GT, 32 * 32, img_off<4>(j, 2 * s + h), gt);
        gw = mma_split<T>(gt, actb, gw);
      }
    }
  }

  // ---- workgroup reduction over streams (fixed order) and slab write ----
  const int E = Pp * kC + 32 * Pp + Pp;
  float* my_slab = slab + static_cast<size_t>(blockIdx.x) * E;
  float* red = reinterpret_cast<float*>(smem_raw);  // [streams-1][npt][32*64 + 32*32 + 32]
  constexpr int kPerWave = 32 * kC + 32 * 32 + 32;
  __syncthreads();
  gsum += __shfl_xor(gsum, 32);
  if (stream > 0) {
    float* dst = red + static_cast<size_t>((stream - 1) * npt + w) * kPerWave;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) dst[acc_row(r, h) * kC + ct * 32 + j] = gp[ct][r];
#pragma unroll
    for (int r = 0; r < 16; ++r) dst[32 * kC + acc_row(r, h) * 32 + j] = gw[r];
    if (h == 0) dst[32 * kC + 1024 + j] = gsum;
  }
  __syncthreads();
  if (stream == 0) {
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int pr = acc_row(r, h);
        float v = gp[ct][r];
        for (int s2 = 1; s2 < streams; ++s2) v += red[static_cast<size_t>((s2 - 1) * npt + w) * kPerWave + pr * kC + ct * 32 + j];
        my_slab[static_cast<size_t>(w * 32 + pr) * kC + ct * 32 + j] = v;
      }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k = acc_row(r, h);
      float v = gw[r];
      for (int s2 = 1; s2 < streams; ++s2) v += red[static_cast<size_t>((s2 - 1) * npt + w) * kPerWave + 32 * kC + k * 32 + j];
      my_slab[static_cast<size_t>(Pp) * kC + static_cast<size_t>(k) * Pp + w * 32 + j] = v;
    }
    if (h == 0) {
      float v = gsum;
      for (int s2 = 1; s2 < streams; ++s2) v += red[static_cast<size_t>((s2 - 1) * npt + w) * kPerWave + 32 * kC + 1024 + j];
      my_slab[static_cast<size_t>(Pp) * kC + 32 * Pp + w * 32 + j] = v;
    }
  }
}

// Slab sum: 64 elements x 4 slab groups per workgroup, groups combined in fixed order.
__global__ __launch_bounds__(256) void l2_bwd_reduce_bf16_kernel(const float* __restrict__ slab, int S, int P,
                                                                  int Pp, int K, const float* __restrict__ protos,
                                                                  float* __restrict__ g_protos,
                                                                  float* __restrict__ g_w) {
  __shared__ float part[4][64];
  __shared__ float gpart[4][64];
  const int E = Pp * kC + 32 * Pp + Pp;
  const int e = blockIdx.x * 64 + (threadIdx.x & 63);
  const int grp = threadIdx.x >> 6;
  const bool is_gp = e < Pp * kC;
  const int p_of_e = is_gp ? e / kC : 0;
  float s = 0.f, gs = 0.f;
  if (e < Pp * kC + 32 * Pp) {
    for (int si = grp; si < S; si += 4) {
      s += slab[static_cast<size_t>(si) * E + e];
      if (is_gp) gs += slab[static_cast<size_t>(si) * E + Pp * kC + 32 * Pp + p_of_e];
    }
  }
  part[grp][threadIdx.x & 63] = s;
  gpart[grp][threadIdx.x & 63] = gs;
  __syncthreads();
  if (grp != 0 || e >= Pp * kC + 32 * Pp) return;
  const int l = threadIdx.x;
  const float tot = ((part[0][l] + part[1][l]) + part[2][l]) + part[3][l];
  if (is_gp) {
    const int c = e - p_of_e * kC;
    if (p_of_e < P && g_protos) {
      const float gst = ((gpart[0][l] + gpart[1][l]) + gpart[2][l]) + gpart[3][l];
      g_protos[static_cast<size_t>(p_of_e) * kC + c] = tot + gst * (2.f * protos[static_cast<size_t>(p_of_e) * kC + c]);
    }
  } else {
    const int e2 = e - Pp * kC;
    const int k = e2 / Pp, pp = e2 - k * Pp;
    if (g_w && k < K && pp < P) g_w[static_cast<size_t>(k) * P + pp] = tot;
  }
}

size_t fwd_lds(const Geometry& g, int terms) { return static_cast<size_t>(g.Pp) * (terms * (kC + 32) * 2 + 4); }
size_t bwd_x_lds(const Geometry& g, int terms) {
  return static_cast<size_t>(g.Pp) * (terms * (2 * kC + 32) * 2 + 4);
}
// Pixel streams per workgroup: 2 when 2*npt waves fit the 768-thread launch bound.
int pw_streams(const Geometry& g) { return (g.Pp / 32) * 2 <= 12 ? 2 : 1; }
size_t pw_lds(const Geometry& g, int terms) {
  const size_t stage = terms == 2 ? PwStage<2>::kBytes : PwStage<3>::kBytes;
  const int streams = pw_streams(g);
  const size_t red = static_cast<size_t>(streams - 1) * (g.Pp / 32) * (32 * kC + 32 * 32 + 32) * sizeof(float);
  const size_t st = static_cast<size_t>(g.Pp) * terms * (kC + 32) * 2 + stage * streams;
  return st > red ? st : red;
}
int pw_grid(const Geometry& g) {
  const int streams = pw_streams(g);
  const int need = static_cast<int>(ceil_div(g.ntiles, streams));
  return need < 256 ? need : 256;
}

template <typename TX, int T>
int fwd_t(const Geometry& g, const void* x, const float* protos, const float* w_last, float eps, int act_kind,
          float* dist, float* act, float* logits, hipStream_t stream) {
  if (int st = ensure_lds<l2_fwd_bf16_kernel<TX, T>>()) return st;
  const size_t lds = fwd_lds(g, T);
  const int per_cu = static_cast<int>(kMaxLds / lds);
  const int cap = 256 * (per_cu < 1 ? 1 : (per_cu > 2 ? 2 : per_cu));
  const int want = static_cast<int>(ceil_div(g.ntiles, kWavesA));
  hipLaunchKernelGGL((l2_fwd_bf16_kernel<TX, T>), dim3(want < cap ? want : cap), dim3(kWavesA * 64), lds, stream,
                     static_cast<const TX*>(x), g.HW, g.npix, protos, g.P, g.Pp, w_last, g.K, eps, act_kind, dist,
                     act, logits);
  return check_launch("l2_fwd_bf16_kernel");
}

template <typename TX, int T>
int bwd_x_t(const Geometry& g, const void* x, const float* protos, const float* w_last, float eps, int act_kind,
            const float* g_logits, const float* g_dist, void* g_x, hipStream_t stream) {
  if (int st = ensure_lds<l2_bwd_x_bf16_kernel<TX, T>>()) return st;
  const size_t lds = bwd_x_lds(g, T);
  const int per_cu = static_cast<int>(kMaxLds / lds);
  const int cap = 256 * (per_cu < 1 ? 1 : (per_cu > 2 ? 2 : per_cu));
  const int want = static_cast<int>(ceil_div(g.ntiles, kWavesA));
  hipLaunchKernelGGL((l2_bwd_x_bf16_kernel<TX, T>), dim3(want < cap ? want : cap), dim3(kWavesA * 64), lds, stream,
                     static_cast<const TX*>(x), g.HW, g.npix, protos, g.P, g.Pp, w_last, g.K, eps, act_kind, g_logits,
                     g_dist, static_cast<TX*>(g_x));
  return check_launch("l2_bwd_x_bf16_kernel");
}

template <typename TX, int T>
int bwd_pw_t(const Geometry& g, const void* x, const float* protos, const float* w_last, float eps, int act_kind,
             const float* g_logits, const float* g_dist, float* g_protos, float* g_w, float* ws, hipStream_t stream) {
  if (int st = ensure_lds<l2_bwd_pw_bf16_kernel<TX, T>>()) return st;
  const int streams = pw_streams(g);
  const int grid = pw_grid(g);
  const int threads = streams * (g.Pp / 32) * 64;
  hipLaunchKernelGGL((l2_bwd_pw_bf16_kernel<TX, T>), dim3(grid), dim3(threads), pw_lds(g, T), stream,
                     static_cast<const TX*>(x), g.HW, g.npix, protos, g.P, g.Pp, w_last, g.K, eps, act_kind, g_logits,
                     g_dist, streams, ws);
  if (int st = check_launch("l2_bwd_pw_bf16_kernel")) return st;
  const int elems = g.Pp * kC + 32 * g.Pp;
  hipLaunchKernelGGL(l2_bwd_reduce_bf16_kernel, dim3(static_cast<unsigned>(ceil_div(elems, 64))), dim3(256), 0,
                     stream, ws, grid, g.P, g.Pp, g.K, protos, g_protos, g_logits ? g_w : nullptr);
  return check_launch("l2_bwd_reduce_bf16_kernel");
}

template <typename Fn>
int by_type(bool x_bf16, int terms, Fn&& fn) {
  if (terms == 2) {
    return x_bf16 ? fn(static_cast<uint16_t*>(nullptr), std::integral_constant<int, 2>())
                  : fn(static_cast<float*>(nullptr), std::integral_constant<int, 2>());
  }
  return x_bf16 ? fn(static_cast<uint16_t*>(nullptr), std::integral_constant<int, 3>())
                : fn(static_cast<float*>(nullptr), std::integral_constant<int, 3>());
}

}  // namespace

bool bf16_fwd_fits(const Geometry& g, int terms) { return g.C == kC && fwd_lds(g, terms) <= kMaxLds; }
bool bf16_bwd_x_fits(const Geometry& g, int terms) { return g.C == kC && bwd_x_lds(g, terms) <= kMaxLds; }
bool bf16_bwd_pw_fits(const Geometry& g, int terms) {
  return g.C == kC && g.Pp <= 384 && pw_lds(g, terms) <= kMaxLds;
}
size_t bf16_bwd_pw_workspace(const Geometry& g) {
  return static_cast<size_t>(pw_grid(g)) * (static_cast<size_t>(g.Pp) * kC + 32 * g.Pp + g.Pp) * sizeof(float);
}

int launch_fwd_bf16(const Geometry& g, bool x_bf16, int terms, const void* x, const float* protos,
                    const float* w_last, float eps, int act_kind, float* dist, float* act, float* logits,
                    hipStream_t stream) {
  return by_type(x_bf16, terms, [&](auto tx, auto tt) {
    using TX = std::remove_pointer_t<decltype(tx)>;
    return fwd_t<TX, decltype(tt)::value>(g, x, protos, w_last, eps, act_kind, dist, act, logits, stream);
  });
}

int launch_bwd_x_bf16(const Geometry& g, bool x_bf16, int terms, const void* x, const float* protos,
                      const float* w_last, float eps, int act_kind, const float* g_logits, const float* g_dist,
                      void* g_x, hipStream_t stream) {
  return by_type(x_bf16, terms, [&](auto tx, auto tt) {
    using TX = std::remove_pointer_t<decltype(tx)>;
    return bwd_x_t<TX, decltype(tt)::value>(g, x, protos, w_last, eps, act_kind, g_logits, g_dist, g_x, stream);
  });
}

int launch_bwd_pw_bf16(const Geometry& g, bool x_bf16, int terms, const void* x, const float* protos,
                       const float* w_last, float eps, int act_kind, const float* g_logits, const float* g_dist,
                       float* g_protos, float* g_w, float* ws, hipStream_t stream) {
  return by_type(x_bf16, terms, [&](auto tx, auto tt) {
    using TX = std::remove_pointer_t<decltype(tx)>;
    return bwd_pw_t<TX, decltype(tt)::value>(g, x, protos, w_last, eps, act_kind, g_logits, g_dist, g_protos, g_w, ws,
                                             stream);
  });
}

}  // namespace protoseg
