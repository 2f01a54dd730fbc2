// l2_bf16.hip — the prototype layer on bf16 MFMA with split operands (bf16_split.h), C = 64.
//
// Same math and outputs as the f32-MFMA family in l2_layer.hip (reference model.py:203-237,
// 259-283 and their autograd), at 5.3x (T=2) / 2.7x (T=3) fewer matrix-core cycles.
//
//   l2_fwd_bf16_kernel     layout A (rows p, cols n): distances -> NCHW stores, activation in
//                          registers, logits = W . act with the accumulator as B operand.
//                          Each wave prefetches its next pixel tile during the current one.
//   l2_bwd_x_bf16_kernel   layout A: recompute S, g_act = W^T g_logits^T, g_s, and
//                          g_x^T = P^T (-2 g_s) with the accumulator as B operand.
//   l2_bwd_pw_bf16_kernel  layout B (rows n, cols p): one workgroup = S streams x npt waves,
//                          wave (stream, w) owns prototype tile w; each 32-pixel tile is read
//                          from HBM once (prefetched into registers one tile ahead), staged in
//                          LDS as bf16 images and shared by the npt waves; g_P^T and g_W
//                          accumulate in registers (the accumulator is their A / B operand),
//                          one partial slab per workgroup.
//   l2_bwd_reduce_bf16_kernel  deterministic parallel sum of the slabs (+ 2p * sum g_s).
//
// Memory ops go through buffer resources (out-of-range lanes read 0 / drop their store), the
// activation is a template parameter, and every kernel uses the channel order chan_of() for
// the distance GEMM, so all three compute bit-identical distances for the same inputs.
#include <type_traits>

#include "adam_update.h"
#include "bf16_split.h"
#include "l2_bf16_common.h"
#include "l2_launch.h"
#include "protoseg_host.h"

namespace protoseg {

namespace {

using namespace bf16l;

constexpr int kWavesA = 8;     // x-backward: 8 waves, one 32-pixel tile each at a time
constexpr int kWavesF = 8;     // forward: 8 waves (12 would need <= 168 VGPRs: 80+ spill today)
// Remainder-tile logits partials go through LDS 4 registers at a time (8 KB for 8 waves), so the
// forward's LDS (P and W images + partials) fits 160 KiB up to Pp = 384 (19 prototypes/class).
constexpr int kFwdPartRegs = 4;

// (-2 P) image [T][Pp][64]: row p, chunk 2q+h = channels chan_of(q, h, 0..7) (CPR 8). Operand
// of the distance GEMM in every kernel: A in layout A (lane = p), B in layout B (lane = p). The
// accumulator starts at ||x||^2 + ||p||^2, so d = relu(acc) directly (the -2 scaling is exact).
template <int T>
__device__ void stage_p_rows(bf16* img, const float* __restrict__ protos, int P, int Pp, int tid, int nth) {
  const int plane = Pp * kC;
  for (int idx = tid; idx < Pp * 8; idx += nth) {
    const int p = idx >> 3, e8 = idx & 7, q = e8 >> 1, h = e8 & 1;
    const int pc = p < P ? p : P - 1;  // clamped: every load is issued unconditionally (pin_batch)
    float v[8];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) v[jj] = protos[static_cast<size_t>(pc) * kC + chan_of(q, h, jj)];
    pin_batch(v);
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) v[jj] = p < P ? -2.f * v[jj] : 0.f;
    bf16x8 f[T];
    split8<T>(v, f);
    store_frag<T>(img, plane, img_off<8>(p, e8), f);
  }
}

// (-2 P)^T image [T][npt][64 c][32 p-permuted] (CPR 4) — A operand of g_x^T = -2 P^T g_s.
template <int T>
__device__ void stage_pt_perm(bf16* img, const float* __restrict__ protos, int P, int Pp, int tid, int nth) {
  const int plane = Pp * kC;
  for (int idx = tid; idx < (Pp / 32) * kC * 4; idx += nth) {
    const int pt = idx / (kC * 4), c = (idx >> 2) & (kC - 1), e8 = idx & 3;
    float v[8];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const int p = pt * 32 + perm_of(e8 * 8 + jj);
      v[jj] = protos[static_cast<size_t>(p < P ? p : P - 1) * kC + c];
    }
    pin_batch(v);
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const int p = pt * 32 + perm_of(e8 * 8 + jj);
      v[jj] = p < P ? -2.f * v[jj] : 0.f;  // -2 folded in (exact)
    }
    bf16x8 f[T];
    split8<T>(v, f);
    store_frag<T>(img, plane, img_off<4>(pt * kC + c, e8), f);
  }
}

// (act_unit W) image [T][npt][32 k][32 p-permuted] (CPR 4) — A operand of logits = W . act.
template <int T>
__device__ void stage_w_perm(bf16* img, const float* __restrict__ w, int K, int P, int ldw, int Pp, float scale,
                             int tid, int nth) {
  const int plane = Pp * 32;
  for (int idx = tid; idx < Pp * 4; idx += nth) {
    const int row = idx >> 2, e8 = idx & 3;  // row = pt*32 + k
    const int pt = row >> 5, k = row & 31;
    float v[8] = {};
    if (K > 0) {  // w is null iff K = 0 (uniform)
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int p = pt * 32 + perm_of(e8 * 8 + jj);
        v[jj] = w[static_cast<size_t>(k < K ? k : 0) * ldw + (p < P ? p : P - 1)];
      }
      pin_batch(v);
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int p = pt * 32 + perm_of(e8 * 8 + jj);
        v[jj] = (k < K && p < P) ? scale * v[jj] : 0.f;
      }
    }
    bf16x8 f[T];
    split8<T>(v, f);
    store_frag<T>(img, plane, img_off<4>(row, e8), f);
  }
}

// (grad_unit W)^T image [T][Pp][32 k] natural classes (CPR 4) — operand of g_act: A in layout A
// (lane = p), B in layout B (lane = p).
template <int T>
__device__ void stage_wt_rows(bf16* img, const float* __restrict__ w, int K, int P, int ldw, int Pp, float scale,
                              int tid, int nth) {
  const int plane = Pp * 32;
  for (int idx = tid; idx < Pp * 4; idx += nth) {
    const int p = idx >> 2, e8 = idx & 3;
    float v[8] = {};
    if (K > 0) {  // w is null iff K = 0 (uniform)
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int k = e8 * 8 + jj;
        v[jj] = w[static_cast<size_t>(k < K ? k : 0) * ldw + (p < P ? p : P - 1)];
      }
      pin_batch(v);
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int k = e8 * 8 + jj;
        v[jj] = (k < K && p < P) ? scale * v[jj] : 0.f;
      }
    }
    bf16x8 f[T];
    split8<T>(v, f);
    store_frag<T>(img, plane, img_off<4>(p, e8), f);
  }
}


// ||p||^2 exactly as the f32 family (sequential, no contraction).
__device__ float proto_norm2_64(const float* __restrict__ protos, int p, bool valid) {
#pragma clang fp contract(off)
  const float* row = protos + static_cast<size_t>(valid ? p : 0) * kC;
  float v[kC];
#pragma unroll
  for (int c = 0; c < kC; ++c) v[c] = row[c];  // all loads in flight, then the ordered sum
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < kC; ++c) s += v[c] * v[c];
  return valid ? s : 0.f;
}


// blockIdx.y selects the image, so the five loops (each a few load round trips) run concurrently;
// blockIdx.z the prototype chunk (rows z*per .. of `P` in all; chunk z's images at z*chunk_bytes),
// so a chunked call builds every chunk's images in one launch.
// fwd_only: the forward's images only (P rows, W, p2: the backward families build their own).
template <int T>
__global__ __launch_bounds__(256) void l2_prep_bf16_kernel(const float* __restrict__ protos, int P, int per,
                                                           const float* __restrict__ w_last, int K, int ldw,
                                                           float w_scale, float wt_scale,
                                                           unsigned char* __restrict__ block, unsigned chunk_bytes,
                                                           int fwd_only) {
  const int p0 = static_cast<int>(blockIdx.z) * per;
  protos += static_cast<size_t>(p0) * kC;
  if (w_last) w_last += p0;
  block += static_cast<size_t>(blockIdx.z) * chunk_bytes;
  P = P - p0 < per ? P - p0 : per;
  const int Pp = (P + 31) & ~31;
  const ImgOffsets o = img_offsets(Pp, T);
  const int tid = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
  switch (blockIdx.y) {
    case 0:
      stage_p_rows<T>(reinterpret_cast<bf16*>(block + o.p), protos, P, Pp, tid, nth);
      break;
    case 1:
      if (!fwd_only)
        stage_wt_rows<T>(reinterpret_cast<bf16*>(block + o.wt), w_last, w_last ? K : 0, P, ldw, Pp, wt_scale, tid, nth);
      break;
    case 2:
      if (!fwd_only) stage_pt_perm<T>(reinterpret_cast<bf16*>(block + o.pt), protos, P, Pp, tid, nth);
      break;
    case 3:
      stage_w_perm<T>(reinterpret_cast<bf16*>(block + o.w), w_last, w_last ? K : 0, P, ldw, Pp, w_scale, tid, nth);
      break;
    default: {
      float* p2 = reinterpret_cast<float*>(block + o.p2);
      const int n1 = (o.pt - o.p2) / 4;
      for (int p = tid; p < n1; p += nth) p2[p] = proto_norm2_64(protos, p, p < P);
    }
  }
}


// Adam step of (prototypes, last layer) fused with the operand prep of the updated values: the
// image block l2_prep_bf16_kernel<2> builds (fwd_only 0, one chunk), so the next forward skips
// its prep launch (PROTOSEG_OPERANDS_READY). One workgroup per 32-prototype tile: it updates rows
// 32 pt .. of the prototypes and the same columns of the last layer (adam_update.h: adam_kernel's
// arithmetic), keeps the new values in LDS, and writes the tile's part of every image region from
// them with the stage_* functions' element order, scaling and zeroing (the same bits). The step
// counts advance once per launch (the last workgroup's ticket, as adam_kernel).
constexpr int kApPitch = kC + 1;  // LDS rows of the tile's prototypes (conflict-free column reads)
// 1024 threads: 2 prototype elements and 1 last-layer element per thread, then one image item
// each (the tile's 768 of them) — 12 workgroups at P = 361 carry the whole step, so the work per
// wave is kept short
constexpr int kApThreads = 1024;
__global__ __launch_bounds__(kApThreads) void l2_adam_prep_kernel(AdamPrepArgs a) {
  __shared__ float sp[32 * kApPitch];
  __shared__ float sw[32 * 33];
  __shared__ float corr[4];
  __shared__ int tk[2], last[2];
  const int pt = blockIdx.x, tid = threadIdx.x, P = a.P, K = a.K;
  const int Pp = (P + 31) & ~31, p0 = pt * 32;
  // this tile's elements: prototypes (row r, channel c) = e, w (class k, column j) = e
  constexpr int kPE = 32 * kC / kApThreads, kWE = 32 * 32 / kApThreads;
  float gi[kPE], pi[kPE], mi[kPE], vi[kPE], gwi[kWE], wi[kWE], mwi[kWE], vwi[kWE];
#pragma unroll
  for (int u = 0; u < kPE; ++u) {
    const int e = tid + kApThreads * u, r = e >> 6;
    const bool ok = p0 + r < P;
    const size_t i = static_cast<size_t>(p0) * kC + e;
    gi[u] = ok ? a.gp[i] : 0.f;
    pi[u] = ok ? a.p[i] : 0.f;
    mi[u] = ok ? a.mp[i] : 0.f;
    vi[u] = ok ? a.vp[i] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < kWE; ++u) {
    const int e = tid + kApThreads * u, k = e >> 5, j = e & 31;
    const bool ok = k < K && p0 + j < P;
    const size_t i = static_cast<size_t>(k) * P + p0 + j;
    gwi[u] = ok ? a.gw[i] : 0.f;
    wi[u] = ok ? a.w[i] : 0.f;
    mwi[u] = ok ? a.mw[i] : 0.f;
    vwi[u] = ok ? a.vw[i] : 0.f;
  }
  if (tid < 2 && (tid == 0 || K > 0)) {
    const AdamCorr ac = tid == 0 ? adam_corr(a.stp, a.lr_p, a.beta1, a.beta2) : adam_corr(a.stw, a.lr_w, a.beta1, a.beta2);
    tk[tid] = ac.t;
    corr[2 * tid] = ac.step_size;
    corr[2 * tid + 1] = ac.bc2_sqrt;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kPE; ++u) {
    const int e = tid + kApThreads * u, r = e >> 6, c = e & 63;
    if (p0 + r < P) {
      adam_update(pi[u], mi[u], vi[u], gi[u], corr[0], corr[1], a.beta1, a.beta2, a.eps, a.wd_p);
      const size_t i = static_cast<size_t>(p0) * kC + e;
      a.mp[i] = mi[u];
      a.vp[i] = vi[u];
      a.p[i] = pi[u];
    }
    sp[r * kApPitch + c] = pi[u];
  }
#pragma unroll
  for (int u = 0; u < kWE; ++u) {
    const int e = tid + kApThreads * u, k = e >> 5, j = e & 31;
    if (k < K && p0 + j < P) {
      adam_update(wi[u], mwi[u], vwi[u], gwi[u], corr[2], corr[3], a.beta1, a.beta2, a.eps, a.wd_w);
      const size_t i = static_cast<size_t>(k) * P + p0 + j;
      a.mw[i] = mwi[u];
      a.vw[i] = vwi[u];
      a.w[i] = wi[u];
    }
    sw[k * 33 + j] = wi[u];
  }
  __syncthreads();
  // the step counts: the last workgroup publishes t (every read of state[0] returned before the
  // tickets, see adam_kernel)
  if (tid < 2 && (tid == 0 || K > 0)) {
    int* st = tid == 0 ? a.stp : a.stw;
    last[tid] = atomicAdd(st + 1, 1) == static_cast<int>(gridDim.x) - 1;
    if (last[tid]) {
      atomicExch(st, tk[tid]);
      atomicExch(st + 1, 0);
    }
  }
  const ImgOffsets o = img_offsets(Pp, 2);
  bf16* img_p = reinterpret_cast<bf16*>(a.block + o.p);
  bf16* img_pt = reinterpret_cast<bf16*>(a.block + o.pt);
  bf16* img_w = reinterpret_cast<bf16*>(a.block + o.w);
  bf16* img_wt = reinterpret_cast<bf16*>(a.block + o.wt);
  if (tid < 256) {  // (-2 P) rows (stage_p_rows): row p0 + (tid >> 3), chunk tid & 7
    const int r = tid >> 3, e8 = tid & 7, q = e8 >> 1, h = e8 & 1, p = p0 + r;
    float v[8];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) v[jj] = p < P ? -2.f * sp[r * kApPitch + chan_of(q, h, jj)] : 0.f;
    bf16x8 f[2];
    split8<2>(v, f);
    store_frag<2>(img_p, Pp * kC, img_off<8>(p, e8), f);
  } else if (tid < 512) {  // (-2 P)^T permuted (stage_pt_perm): channel (tid - 256) >> 2, chunk tid & 3
    const int c = (tid - 256) >> 2, e8 = tid & 3;
    float v[8];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const int r = perm_of(e8 * 8 + jj);
      v[jj] = p0 + r < P ? -2.f * sp[r * kApPitch + c] : 0.f;
    }
    bf16x8 f[2];
    split8<2>(v, f);
    store_frag<2>(img_pt, Pp * kC, img_off<4>(pt * kC + c, e8), f);
  } else if (tid < 640) {  // (act_unit W) permuted (stage_w_perm): class (tid - 512) >> 2, chunk tid & 3
    const int k = (tid - 512) >> 2, e8 = tid & 3;
    float v[8];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const int j = perm_of(e8 * 8 + jj);
      v[jj] = (k < K && p0 + j < P) ? a.w_scale * sw[k * 33 + j] : 0.f;
    }
    bf16x8 f[2];
    split8<2>(v, f);
    store_frag<2>(img_w, Pp * 32, img_off<4>(pt * 32 + k, e8), f);
  } else if (tid < 768) {  // (grad_unit W)^T rows (stage_wt_rows): row p0 + ((tid - 640) >> 2), chunk tid & 3
    const int j = (tid - 640) >> 2, e8 = tid & 3, p = p0 + j;
    float v[8];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const int k = e8 * 8 + jj;
      v[jj] = (k < K && p < P) ? a.wt_scale * sw[k * 33 + j] : 0.f;
    }
    bf16x8 f[2];
    split8<2>(v, f);
    store_frag<2>(img_wt, Pp * 32, img_off<4>(p, e8), f);
  } else if (tid < 800) {  // ||p||^2 as proto_norm2_64: sequential, no contraction
#pragma clang fp contract(off)
    const int r = tid - 768, p = p0 + r;
    float s = 0.f;
    for (int c = 0; c < kC; ++c) {
      const float x = sp[r * kApPitch + c];
      s += x * x;
    }
    reinterpret_cast<float*>(a.block + o.p2)[p] = p < P ? s : 0.f;
  } else if (pt == static_cast<int>(gridDim.x) - 1) {  // the p2 region's padding past Pp
    const int n1 = (o.pt - o.p2) / 4;
    for (int p = Pp + tid - 800; p < n1; p += kApThreads - 800) reinterpret_cast<float*>(a.block + o.p2)[p] = 0.f;
  }
}

// Byte offset of this lane's pixel at channel 4h of image b (layout A lane = pixel j), or kOOB.
template <typename TX>
__device__ __forceinline__ unsigned x_lane_off(int t, int ntiles, int npix, int HW) {
  const int j = threadIdx.x & 31, h = (threadIdx.x & 63) >> 5;
  const int g = t * 32 + j;
  if (t >= ntiles || g >= npix) return kOOB;
  const int b = div_pix(g, HW), n = g - b * HW;
  return static_cast<unsigned>(((b * kC + 4 * h) * HW + n) * static_cast<int>(sizeof(TX)));
}

// Raw layout-A x of one tile: raw[q*8 + jj] = x[chan_of(q, h, jj)][pixel j] (0 when out of range).
template <typename TX>
__device__ __forceinline__ void load_x_raw(rsrc_t rx, unsigned off, unsigned cs, float (&raw)[kNQ * 8]) {
#pragma unroll
  for (int q = 0; q < kNQ; ++q)
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) raw[q * 8 + jj] = BufIO<TX>::load(rx, off, chan_base(q, jj) * cs);
}

// Split fragments + ||x||^2 in the family's fixed order (x2_tree_halves).
template <int T>
__device__ __forceinline__ float x_frags(const float (&raw)[kNQ * 8], bf16x8 (&xb)[kNQ][T]) {
  float sq[kNQ];
#pragma unroll
  for (int q = 0; q < kNQ; ++q) {
    float v[8];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) v[jj] = raw[q * 8 + jj];
    sq[q] = chunk_sq(v);
    split8<T>(v, xb[q]);
  }
  return x2_tree_halves(sq);
}

// ||x||^2 + ||p||^2 - 2 P . X for prototype tile pt (layout A: rows p, cols the wave's 32
// pixels): the accumulator starts at x2 + p2 (per element) and the (-2 P) image does the rest.
template <int T>
__device__ __forceinline__ f32x16 s_tile(const bf16* Pimg, int Pp, int pt, const bf16x8 (&xb)[kNQ][T], float x2,
                                         const float (&p2r)[16]) {
  const int j = threadIdx.x & 31, h = (threadIdx.x & 63) >> 5;
  f32x16 acc;
  typedef float f32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int r = 0; r < 16; r += 2) {  // v_pk_add_f32: two rows per VALU op
    const f32x2 v = f32x2{x2, x2} + f32x2{p2r[r], p2r[r + 1]};
    acc[r] = v.x;
    acc[r + 1] = v.y;
  }
#pragma unroll
  for (int q = 0; q < kNQ; ++q) {
    bf16x8 pa[T];
    load_frag<T>(Pimg, Pp * kC, img_off<8>(pt * 32 + j, 2 * q + h), pa);
    acc = mma_split<T>(pa, xb[q], acc);
  }
  return acc;
}

// Tile schedule shared by the layout-A kernels (forward, x-backward). The ntiles pixel tiles are
// split into R = ntiles / W full rounds (W = resident waves; wave g takes tiles g, g + W, ...,
// every wave the same count) and a remainder of m < W tiles. A remainder tile is processed
// by one whole workgroup, its waves splitting the prototype tiles (wave w: pt = w, w + 8, ...),
// so the remainder costs about one prototype tile of time instead of one pixel tile — with
// one tile per wave per round, a remainder handled the plain way would leave most of the chip
// idle for a whole extra round.
struct TileSchedule {
  int full_end;  // tiles [0, full_end) are done in full rounds
  __device__ TileSchedule(int ntiles, int waves_per_block) {
    const int W = static_cast<int>(gridDim.x) * waves_per_block;
    full_end = (ntiles / W) * W;
  }
};

#ifndef FWD_REM_ROUNDS
#define FWD_REM_ROUNDS 3  // small-batch forward: remainder rounds preferred over one full round
#endif
#ifndef FWD_DIST_CPOL
#define FWD_DIST_CPOL 0  // cache policy of the distance stores (measured variants: tools/gpu_r3aa.sh)
#endif
// Forward, one pixel tile per wave per round: distances (NCHW stores), activation in registers,
// logits = W . act with the accumulator as B operand. Remainder tiles: see TileSchedule; the
// per-wave logits partials are summed in LDS in a fixed order (deterministic).
template <typename TX, int T, int ACT, bool ACTS, bool LOGITS>
__global__ __launch_bounds__(kWavesF * 64) void l2_fwd_bf16_kernel(
    const TX* __restrict__ x, unsigned x_bytes, int HW, int npix, const unsigned char* __restrict__ img, int P, int Pp,
    int K, float eps, float* __restrict__ dist, unsigned d_bytes,
    float* __restrict__ act_out, unsigned a_bytes, float* __restrict__ logits, unsigned l_bytes, int ld, int p0,
    int accumulate, int xsig) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  STAMP(0);
  STAMP_RT(7);
  const ImgOffsets io = img_offsets(Pp, T);
  bf16* Pimg = reinterpret_cast<bf16*>(smem_raw);                // [T][Pp][64]
  bf16* Wimg = Pimg + T * Pp * kC;                               // [T][Pp][32]
  float* p2s = reinterpret_cast<float*>(Wimg + T * Pp * 32);     // [Pp]
  float* lpart = p2s + (io.pt - io.p2) / 4;                      // [kWavesF][kFwdPartRegs][64] remainder logits

  const rsrc_t rx = make_rsrc(x, x_bytes), rd = make_rsrc(dist, d_bytes);
  const rsrc_t ra = make_rsrc(act_out, a_bytes), rl = make_rsrc(logits, l_bytes);
  const unsigned cs = static_cast<unsigned>(HW) * sizeof(TX);
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5, wave = wave_id();
  const int ntiles = (npix + 31) / 32;
  const int npt = Pp / 32;
  const int stride = gridDim.x * kWavesF;
  const TileSchedule sched(ntiles, kWavesF);

  // The first tile's x loads are issued before the operand-image DMA, so the barrier's wait
  // covers both round trips at once instead of one after the other.
  constexpr bool kPrefetch = kWavesF <= 8;
  const int vb = xcd_block();
  int t = vb * kWavesF + wave;
  float raw[kNQ * 8];
  if constexpr (kPrefetch)
    load_x_raw<TX>(rx, x_lane_off<TX>(t < sched.full_end ? t : ntiles, ntiles, npix, HW), cs, raw);
  lds_copy(Pimg, img + io.p, io.wt - io.p);
  if constexpr (LOGITS) lds_copy(Wimg, img + io.w, io.total - io.w);
  lds_copy(p2s, img + io.p2, io.pt - io.p2);
  __syncthreads();
  STAMP(1);

  // Prototype tiles pt0, pt0 + dpt, ... of pixel tile t (x already in raw); returns the
  // tile's logits accumulator over those prototype tiles.
  auto run_tile = [&](int t, const float (&raw)[kNQ * 8], int pt0, int dpt) {
    bf16x8 xb[kNQ][T];
    float xv[kNQ * 8];
    if (xsig) {  // wave-uniform: sigmoid of the pre-activation (model.py:124-128) on the load
#pragma unroll
      for (int i = 0; i < kNQ * 8; ++i) xv[i] = sigmoid_f(raw[i]);
    } else {
#pragma unroll
      for (int i = 0; i < kNQ * 8; ++i) xv[i] = raw[i];
    }
    const float x2 = x_frags<T>(xv, xb);
    const int g = t * 32 + j;
    const bool valid = g < npix;
    const int b = valid ? div_pix(g, HW) : 0;
    const int n = valid ? g - b * HW : 0;
    // ld = prototypes per image / pixel row of the outputs (= P, or the full P for a chunk
    // starting at prototype p0)
    const unsigned dbase = valid ? static_cast<unsigned>(((b * ld + p0 + 4 * h) * HW + n) * 4) : kOOB;
    const unsigned abase = valid ? static_cast<unsigned>((g * ld + p0 + 4 * h) * 4) : kOOB;
    f32x16 lacc = zero16();
    // The (-2P) fragments of the next prototype tile are read from LDS while this tile's
    // epilogue runs (one LDS round trip per tile off the MFMA chain), and the W fragments of the
    // logits before the epilogue's VALU, not after it.
    // (bf16x3 only: the 3-term fragments would not fit the 256 registers beside the logits.)
    constexpr bool kPf = T == 2;
    bf16x8 pf[kNQ][T];
    auto load_pf = [&](int pt) __attribute__((always_inline)) {
#pragma unroll
      for (int q = 0; q < kNQ; ++q) load_frag<T>(Pimg, Pp * kC, img_off<8>(pt * 32 + j, 2 * q + h), pf[q]);
    };
    if (kPf && pt0 < npt) load_pf(pt0);
    // Prototype tiles entirely below P store without a row predicate; only the last one (when
    // P is not a multiple of 32) pays for it. The body is instantiated for both cases.
    auto proto_tile = [&](int pt, auto full_tag) {
      constexpr bool kFull = decltype(full_tag)::value;
      float p2r[16];
      load_rows16(p2s + pt * 32 + 4 * h, p2r);
      f32x16 acc;
      {
        typedef float f32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int r = 0; r < 16; r += 2) {  // v_pk_add_f32: two rows per VALU op
          const f32x2 v = f32x2{x2, x2} + f32x2{p2r[r], p2r[r + 1]};
          acc[r] = v.x;
          acc[r + 1] = v.y;
        }
      }
      if constexpr (!kPf) load_pf(pt);
#pragma unroll
      for (int q = 0; q < kNQ; ++q) acc = mma_split<T>(pf[q], xb[q], acc);
      if (kPf && pt + dpt < npt) load_pf(pt + dpt);
      bf16x8 wa[2][T];
      if constexpr (LOGITS && kPf) {
#pragma unroll
        for (int s = 0; s < 2; ++s) load_frag<T>(Wimg, Pp * 32, img_off<4>(pt * 32 + j, 2 * s + h), wa[s]);
      }
      const int prem = P - pt * 32 - 4 * h;  // rows of this tile (and half) below P
      // No branches per element: a null output has a zero-size buffer resource (its stores are
      // dropped), rows past P get an out-of-range offset.
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float d = relu_f(acc[r]);  // F.relu (model.py:219)
        const unsigned row_ok = (kFull || row_of(r) < prem) ? 0u : kOOB;
#ifndef FWD_ABL_NODIST  // (FWD_ABL_*: timing ablations of development builds; wrong results)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(d), rd, dbase | row_ok,
                                              static_cast<unsigned>((pt * 32 + row_of(r)) * HW * 4), FWD_DIST_CPOL);
#endif
#ifndef FWD_ABL_NOACT
        const float a = act_base<ACT>(d, eps);  // act_unit lives in the W image
#else
        const float a = d;
#endif
        if constexpr (ACTS)
          BufIO<float>::store(ra, a * act_unit(ACT), abase | row_ok, static_cast<unsigned>((pt * 32 + row_of(r)) * 4));
        acc[r] = a;
      }
#ifdef FWD_ABL_NOLOGITS
      if constexpr (false) {
#else
      if constexpr (LOGITS) {
#endif
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 ab[T];
          acc_operand<T>(acc, s, ab);
          if constexpr (!kPf) load_frag<T>(Wimg, Pp * 32, img_off<4>(pt * 32 + j, 2 * s + h), wa[s]);
          lacc = mma_split<T>(wa[s], ab, lacc);
        }
      }
    };
    const int npt_full = P / 32;  // tiles whose 32 rows are all below P
    // Full tiles in a loop of their own and the (at most one) partial tile after it: with both
    // bodies in one loop the logits accumulator lives in different registers on the two paths,
    // and every iteration ended in 16 v_mov (after an s_nop for the last MFMA) to merge them.
    int pt = pt0;
#pragma unroll 1
    for (; pt < npt_full; pt += dpt) proto_tile(pt, std::true_type());
    if (pt < npt) proto_tile(pt, std::false_type());
    return lacc;
  };
  auto store_logits = [&](int t, const f32x16& lacc) {
    const int g = t * 32 + j;
    const unsigned lbase = g < npix ? static_cast<unsigned>((g * K + 4 * h) * 4) : kOOB;
    const int krem = K - 4 * h;
    float old[16];
    if (accumulate) {  // chunk c > 0: the earlier chunks' logits, loaded as one batch (pin_batch)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        old[r] = BufIO<float>::load(rl, row_of(r) < krem ? lbase : kOOB, static_cast<unsigned>(row_of(r) * 4));
      pin_batch(old);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const unsigned off = row_of(r) < krem ? lbase : kOOB;
      float v = lacc[r];
      if (accumulate) v = old[r] + v;
      BufIO<float>::store(rl, v, off, static_cast<unsigned>(row_of(r) * 4));
    }
  };

  // ---- full rounds: one tile per wave per round. At 2 waves per SIMD the next tile's x is
  // prefetched into registers; at 3 the other waves cover the load and the 32 VGPRs go.
  for (; t < sched.full_end; t += stride) {
    float cur[kNQ * 8];
    if constexpr (kPrefetch) {
#pragma unroll
      for (int i = 0; i < kNQ * 8; ++i) cur[i] = raw[i];
      const int tn = t + stride;
      load_x_raw<TX>(rx, x_lane_off<TX>(tn < sched.full_end ? tn : ntiles, ntiles, npix, HW), cs, raw);
    } else {
      load_x_raw<TX>(rx, x_lane_off<TX>(t, ntiles, npix, HW), cs, cur);
    }
    if (t == vb * kWavesF + wave) STAMP(2);
    const f32x16 lacc = run_tile(t, cur, 0, 1);
    if constexpr (LOGITS) store_logits(t, lacc);
    if (t == vb * kWavesF + wave) STAMP(3);
  }
  STAMP(4);

  // ---- remainder: one tile per workgroup, prototype tiles split over the waves
  for (int tt = sched.full_end + vb; tt < ntiles; tt += gridDim.x) {
    float rt[kNQ * 8];
    load_x_raw<TX>(rx, x_lane_off<TX>(tt, ntiles, npix, HW), cs, rt);
    const f32x16 lacc = run_tile(tt, rt, wave, kWavesF);
    if constexpr (LOGITS) {  // fixed-order sum of the waves' partials, kFwdPartRegs registers at a time
      const int nw = npt < kWavesF ? npt : kWavesF;
      float* mine = lpart + wave * kFwdPartRegs * 64;
      f32x16 sum = zero16();
#pragma unroll
      for (int hf = 0; hf < 16 / kFwdPartRegs; ++hf) {
        if (wave < nw)
#pragma unroll
          for (int r = 0; r < kFwdPartRegs; ++r) mine[r * 64 + lane] = lacc[kFwdPartRegs * hf + r];
        __syncthreads();
        if (wave == 0)
          for (int w = 0; w < nw; ++w)
#pragma unroll
            for (int r = 0; r < kFwdPartRegs; ++r)
              sum[kFwdPartRegs * hf + r] += lpart[(w * kFwdPartRegs + r) * 64 + lane];
        __syncthreads();
      }
      if (wave == 0) store_logits(tt, sum);
    }
  }
  STAMP(6);
}

// x-backward (layout A): per pixel tile, recompute S and g_act = W^T g_logits^T for every
// prototype tile, g_s, and g_x^T = (-2 P^T) g_s with the accumulator as B operand (the -2 is
// folded into the P^T image), plus 2x * sum_p g_s. Rows p >= P need no predicate: their W^T
// rows and g_dist reads are zero, so g_s = 0 there. Same tile schedule as the forward; the
// remainder tiles' g_x partials are summed in LDS in a fixed order, 8 registers at a time.
constexpr int kXPartRegs = 8;
template <typename TX, int T, int ACT, bool GD>
__global__ __launch_bounds__(kWavesA * 64) void l2_bwd_x_bf16_kernel(
    const TX* __restrict__ x, unsigned x_bytes, int HW, int npix, const unsigned char* __restrict__ img, int P, int Pp,
    int K, float eps, const float* __restrict__ g_logits, unsigned gl_bytes,
    const float* __restrict__ g_dist, unsigned gd_bytes, int gd_ld, int gd_p0, TX* __restrict__ g_x, int accumulate) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const ImgOffsets io = img_offsets(Pp, T);
  bf16* Pimg = reinterpret_cast<bf16*>(smem_raw);                 // [T][Pp][64]
  bf16* PTimg = Pimg + T * Pp * kC;                               // [T][npt*64][32]
  bf16* WTimg = PTimg + T * Pp * kC;                              // [T][Pp][32]
  float* p2s = reinterpret_cast<float*>(WTimg + T * Pp * 32);     // [Pp]
  float* part = p2s + (io.pt - io.p2) / 4;                        // [kWavesA][kXPartRegs + 1][64]
  const rsrc_t rx = make_rsrc(x, x_bytes), rg = make_rsrc(g_logits, gl_bytes);
  const rsrc_t rgd = make_rsrc(g_dist, gd_bytes), rgx = make_rsrc(g_x, x_bytes);
  const unsigned cs = static_cast<unsigned>(HW) * sizeof(TX);
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5, wave = wave_id();
  const int ntiles = (npix + 31) / 32;
  const int npt = Pp / 32;
  const TileSchedule sched(ntiles, kWavesA);
  // The first tile's x loads go out before the operand-image DMA (one combined wait).
  const int t0 = static_cast<int>(blockIdx.x) * kWavesA + wave;
  float raw[kNQ * 8];
  load_x_raw<TX>(rx, x_lane_off<TX>(t0 < sched.full_end ? t0 : ntiles, ntiles, npix, HW), cs, raw);
  lds_copy(Pimg, img + io.p, io.wt - io.p);
  lds_copy(PTimg, img + io.pt, io.w - io.pt);
  lds_copy(WTimg, img + io.wt, io.p2 - io.wt);
  lds_copy(p2s, img + io.p2, io.pt - io.p2);
  __syncthreads();

  // Prototype tiles pt0, pt0 + dpt, ... of pixel tile t: accumulates this wave's part of
  // (-2 P^T) g_s into gx and of sum_p g_s into gsum (this half-wave's rows only).
  auto run_tile = [&](int t, const float (&raw)[kNQ * 8], int pt0, int dpt, f32x16 (&gx)[2], float& gsum) {
    const int g = t * 32 + j;
    const bool valid = g < npix;
    const int b = valid ? div_pix(g, HW) : 0;
    const int n = valid ? g - b * HW : 0;
    // B operand of g_act^T: lane (h, j) holds g_logits[pixel j][16s + 8h + jj]
    bf16x8 glb[2][T];
    {
      const unsigned gbase = valid ? static_cast<unsigned>((g * K + 8 * h) * 4) : kOOB;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float v[8];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          const float t0 = BufIO<float>::load(rg, gbase, static_cast<unsigned>((16 * s + jj) * 4));
          v[jj] = (16 * s + 8 * h + jj < K) ? t0 : 0.f;
        }
        split8<T>(v, glb[s]);
      }
    }
    bf16x8 xb[kNQ][T];
    const float x2 = x_frags<T>(raw, xb);
    const unsigned gdbase = valid ? static_cast<unsigned>(((b * gd_ld + gd_p0 + 4 * h) * HW + n) * 4) : kOOB;
#pragma unroll 1
    for (int pt = pt0; pt < npt; pt += dpt) {
      float gdv[16];  // upstream distance gradient of this tile, loaded before the MFMAs
      if constexpr (GD) {
        const int prem_gd = P - pt * 32 - 4 * h;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          gdv[r] = BufIO<float>::load(rgd, row_of(r) < prem_gd ? gdbase : kOOB,
                                      static_cast<unsigned>((pt * 32 + row_of(r)) * HW * 4));
      }
      float p2r[16];
      load_rows16(p2s + pt * 32 + 4 * h, p2r);
      f32x16 acc = s_tile<T>(Pimg, Pp, pt, xb, x2, p2r);
      // Both class k-steps always run (W^T rows >= K are zero, g_logits reads 0 when absent).
      f32x16 gacc = zero16();
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 wa[T];
        load_frag<T>(WTimg, Pp * 32, img_off<4>(pt * 32 + j, 2 * s + h), wa);
        gacc = mma_split<T>(wa, glb[s], gacc);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float d = relu_f(acc[r]);
        float gd = gacc[r] * act_grad_base<ACT>(d, eps);  // gacc holds grad_unit * g_act (W^T image)
        if constexpr (GD) gd += gdv[r];
        const float gs = d > 0.f ? gd : 0.f;  // relu backward: grad * (out > 0)
        gsum += gs;
        acc[r] = gs;
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
  };
  // gx[ct] register 8s+jj is channel chan_of(2ct+s, h, jj) — the channel of raw[(2ct+s)*8+jj].
  // conv(x^2, ones) backward then pow backward: gsum * (2x); plus the xp branch in gx.
  auto store_gx = [&](unsigned xoff, const float (&raw)[kNQ * 8], const f32x16 (&gx)[2], float gsum_all) {
    float old[kNQ * 8];
    if (accumulate) {  // prototype chunks: the earlier chunks' g_x, loaded as one batch (pin_batch)
#pragma unroll
      for (int q = 0; q < kNQ; ++q)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) old[q * 8 + jj] = BufIO<TX>::load(rgx, xoff, chan_base(q, jj) * cs);
      pin_batch(old);
    }
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          const int q = 2 * ct + s;
          float v = gx[ct][8 * s + jj] + gsum_all * (2.f * raw[q * 8 + jj]);
          if (accumulate) v = old[q * 8 + jj] + v;
          BufIO<TX>::store(rgx, v, xoff, chan_base(q, jj) * cs);
        }
  };

  // ---- full rounds
  for (int t = t0; t < sched.full_end; t += gridDim.x * kWavesA) {
    const unsigned xoff = x_lane_off<TX>(t, ntiles, npix, HW);
    if (t != t0) load_x_raw<TX>(rx, xoff, cs, raw);
    f32x16 gx[2] = {zero16(), zero16()};
    float gsum = 0.f;
    run_tile(t, raw, 0, 1, gx, gsum);
    store_gx(xoff, raw, gx, gsum + __shfl_xor(gsum, 32));
  }

  // ---- remainder: one tile per workgroup, prototype tiles split over the waves
  const int nw = npt < kWavesA ? npt : kWavesA;
  for (int tt = sched.full_end + static_cast<int>(blockIdx.x); tt < ntiles; tt += gridDim.x) {
    const unsigned xoff = x_lane_off<TX>(tt, ntiles, npix, HW);
    float raw[kNQ * 8];
    load_x_raw<TX>(rx, xoff, cs, raw);
    f32x16 gx[2] = {zero16(), zero16()};
    float gsum = 0.f;
    run_tile(tt, raw, wave, kWavesA, gx, gsum);
    gsum += __shfl_xor(gsum, 32);
    float* mine = part + wave * (kXPartRegs + 1) * 64;
    mine[kXPartRegs * 64 + lane] = gsum;
    f32x16 tot[2] = {zero16(), zero16()};
    float gsum_all = 0.f;
#pragma unroll
    for (int c8 = 0; c8 < 4; ++c8) {  // registers 8*c8 .. 8*c8+7 of (gx[0] | gx[1])
#pragma unroll
      for (int r = 0; r < kXPartRegs; ++r) mine[r * 64 + lane] = gx[c8 >> 1][8 * (c8 & 1) + r];
      __syncthreads();
      if (wave == 0) {
        for (int w = 0; w < nw; ++w) {
          const float* src = part + w * (kXPartRegs + 1) * 64;
#pragma unroll
          for (int r = 0; r < kXPartRegs; ++r) tot[c8 >> 1][8 * (c8 & 1) + r] += src[r * 64 + lane];
          if (c8 == 0) gsum_all += src[kXPartRegs * 64 + lane];
        }
      }
      __syncthreads();
    }
    if (wave == 0) store_gx(xoff, raw, tot, gsum_all);
  }
}

// ---- bwd_pw ----------------------------------------------------------------------------------
// Per pixel stream: the raw tile (x [64 c][32 n] in the input dtype, g_logits [32 n][32 k] f32)
// is brought into LDS by LDS-DMA (buffer_load ... lds: no VGPRs, out-of-range lanes land as 0)
// while the previous tile is computed, then split into the bf16 operand images. Rows are
// stored in pairs (row 2r at +0, 2r+1 at +32 elements, pair stride kPair) so one DMA
// wave-instruction fills one pair; the stride keeps the conversion reads conflict-free.
// A 2-byte LDS-DMA lands zero-extended in a dword per lane, so bf16 x is staged as uint32 words
// holding the bf16 bits in their low half.
template <typename TX>
struct PwRaw {
  using XS = std::conditional_t<sizeof(TX) == 4, float, uint32_t>;
  static constexpr int kPairX = 72;
  static constexpr int kPairG = 72;
  static constexpr int kXs = 32 * kPairX;                    // dwords
  static constexpr int kGs = 16 * kPairG;                    // floats
  static constexpr int kBytes = (kXs + kGs + 64) * 4;        // + x2[32], rowoff[32]
};
template <typename TX, int T>
struct PwStage {
  static constexpr int kXA = T * 32 * kC;   // bf16 [T][32 n][64 c]   CPR 8, chan_of order
  static constexpr int kXB = T * kC * 32;   // bf16 [T][64 c][32 n~]  CPR 4, permuted n, x * -2
  static constexpr int kGA = T * 32 * 32;   // bf16 [T][32 n][32 k]   CPR 4
  static constexpr int kGT = T * 32 * 32;   // bf16 [T][32 k][32 n~]  CPR 4, permuted n
  static constexpr int kBytes = PwRaw<TX>::kBytes + (kXA + kXB + kGA + kGT) * 2;
};



template <typename TX, int T, int ACT, int MAXT, bool GD>
__global__ __launch_bounds__(MAXT) void l2_bwd_pw_bf16_kernel(
    const TX* __restrict__ x, unsigned x_bytes, int HW, int npix, const unsigned char* __restrict__ img, int P, int Pp,
    int K, float eps, const float* __restrict__ g_logits, unsigned gl_bytes,
    const float* __restrict__ g_dist, unsigned gd_bytes, int gd_ld, int gd_p0, int streams,
    float* __restrict__ slab) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  using R = PwRaw<TX>;
  using S = PwStage<TX, T>;
  const int npt = Pp / 32;
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5, wave = wave_id();
  const int stream = wave / npt;                 // which pixel stream this wave computes on
  const int w = wave - stream * npt;             // prototype tile owned by this wave

  // LDS: [P image | W^T image | per stream: Xs | Gs | x2[32] | rowoff[32] | XA | XB | GA | GT]
  const ImgOffsets io = img_offsets(Pp, T);
  bf16* Pimg = reinterpret_cast<bf16*>(smem_raw);      // [T][Pp][64]  CPR 8 (chan_of order)
  bf16* WTimg = Pimg + T * Pp * kC;                    // [T][Pp][32]  CPR 4
  unsigned char* sbase = reinterpret_cast<unsigned char*>(WTimg + T * Pp * 32) + stream * S::kBytes;
  using XS = typename R::XS;
  XS* Xs = reinterpret_cast<XS*>(sbase);
  float* Gs = reinterpret_cast<float*>(sbase + R::kXs * 4);
  float* x2s = Gs + R::kGs;
  unsigned* rowoff = reinterpret_cast<unsigned*>(x2s + 32);
  bf16* XA = reinterpret_cast<bf16*>(rowoff + 32);
  bf16* XB = XA + S::kXA;
  bf16* GA = XB + S::kXB;
  bf16* GT = GA + S::kGA;
  STAMP(0);
  STAMP_RT(7);
  lds_copy(Pimg, img + io.p, io.p2 - io.p);  // P and W^T images are adjacent in the block

  const rsrc_t rx = make_rsrc(x, x_bytes), rg = make_rsrc(g_logits, gl_bytes), rgd = make_rsrc(g_dist, gd_bytes);
  const int p = w * 32 + j;  // this lane's prototype column
  const bool pvalid = p < P;
  const float p2 = reinterpret_cast<const float*>(img + io.p2)[p];

  f32x16 gp[2] = {zero16(), zero16()};
  f32x16 gw = zero16();
  float gsum = 0.f;

  const int ntiles = (npix + 31) / 32;
  const int total_streams = gridDim.x * streams;
  const int iters = (ntiles + total_streams - 1) / total_streams;  // uniform across the workgroup
  const int tid_s = threadIdx.x - stream * npt * 64;
  const int nt_stream = npt * 64;

  // DMA of tile t: instruction i < 32 moves x channels 2i, 2i+1 (lane = pixel l&31 of channel
  // 2i + (l>>5)); instruction 32 + i2 moves g_logits pixels 2i2, 2i2+1 (lane = class l&31).
  // The stream's waves take instructions w, w + npt, ...
  auto dma_tile = [&](int t) {
    const int g = t * 32 + j;
    unsigned xo = kOOB;
    if (t < ntiles && g < npix) {
      const int b = div_pix(g, HW);
      xo = static_cast<unsigned>(((b * kC + h) * HW + (g - b * HW)) * static_cast<int>(sizeof(TX)));
    }
    const int lim = t < ntiles ? min(32, npix - t * 32) : 0;  // valid pixels of this tile
    const unsigned go = j < K ? static_cast<unsigned>(((t * 32 + h) * K + j) * 4) : kOOB;
    for (int i = w; i < 48; i += npt) {
      if (i < 32) {
        dma<TX>(rx, Xs + i * R::kPairX, xo, static_cast<unsigned>(2 * i * HW) * sizeof(TX));
      } else {
        const int i2 = i - 32;
        dma<float>(rg, Gs + i2 * R::kPairG, (2 * i2 + h < lim) ? go : kOOB, static_cast<unsigned>(2 * i2 * K * 4));
      }
    }
  };

  // Raw tile -> split images. Wave 0 of the stream: XA and ||x||^2 (lane = (pixel, half), the
  // family's fixed order, so the distances match the forward bit for bit); the other waves (all
  // of them when npt == 1): XB (x * -2, exact), GA, GT.
  auto convert = [&](int t) {
    if (w == 0) {
      float sq[kNQ];
#pragma unroll
      for (int q = 0; q < kNQ; ++q) {
        float v[8];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) v[jj] = lds_val(Xs + pair_off<R::kPairX>(chan_of(q, h, jj), j));
        sq[q] = chunk_sq(v);
        bf16x8 f[T];
        split8<T>(v, f);
        store_frag<T>(XA, 32 * kC, img_off<8>(j, 2 * q + h), f);
      }
      const float x2 = x2_tree_halves(sq);
      if (h == 0) x2s[j] = x2;
    }
    const int nthr = npt > 1 ? nt_stream - 64 : nt_stream;
    for (int idx = npt > 1 ? tid_s - 64 : tid_s; idx >= 0 && idx < 512; idx += nthr) {
      float v[8];
      if (idx < 256) {  // XB row c, chunk e8 = (s, hp): pixels 16s + 4hp + {0..3} and + 8
        const int c = idx >> 2, e8 = idx & 3, sb = 16 * (e8 >> 1) + 4 * (e8 & 1);
        lds_val4(Xs + pair_off<R::kPairX>(c, sb), v);
        lds_val4(Xs + pair_off<R::kPairX>(c, sb + 8), v + 4);
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) v[jj] *= -2.f;
        bf16x8 f[T];
        split8<T>(v, f);
        store_frag<T>(XB, kC * 32, img_off<4>(c, e8), f);
      } else if (idx < 384) {  // GA row n, classes 8e8..8e8+7
        const int n = (idx - 256) >> 2, e8 = idx & 3;
        lds_val4(Gs + pair_off<R::kPairG>(n, 8 * e8), v);
        lds_val4(Gs + pair_off<R::kPairG>(n, 8 * e8 + 4), v + 4);
        bf16x8 f[T];
        split8<T>(v, f);
        store_frag<T>(GA, 32 * 32, img_off<4>(n, e8), f);
      } else {  // GT row k, permuted pixels
        const int k = (idx - 384) >> 2, e8 = idx & 3;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) v[jj] = Gs[pair_off<R::kPairG>(perm_of(e8 * 8 + jj), k)];
        bf16x8 f[T];
        split8<T>(v, f);
        store_frag<T>(GT, 32 * 32, img_off<4>(k, e8), f);
      }
    }
    if constexpr (GD) {
      if (w == npt - 1 && lane < 32) {  // per-row g_dist offset (b, n) of this tile
        const int g = t * 32 + lane;
        const bool ok = t < ntiles && g < npix;
        const int b = ok ? div_pix(g, HW) : 0;
        rowoff[lane] = ok ? static_cast<unsigned>(((b * gd_ld + gd_p0) * HW + (g - b * HW)) * 4) : kOOB;
      }
    }
  };

  int t = blockIdx.x * streams + stream;
  dma_tile(t);
  STAMP(1);
  for (int it = 0; it < iters; ++it, t += total_streams) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of tile t has landed
    __syncthreads();                                   // ... and every wave's; images are free
    if (it == 1) STAMP(2);
    convert(t);
    __syncthreads();  // images ready; the raw tile area is free
    if (it == 1) STAMP(3);
    if (it + 1 < iters) dma_tile(t + total_streams);  // lands while this tile is computed

    // ---- compute: this wave's prototype tile against the staged pixel tile ----
    // Rows past npix hold x = 0 and g_logits = 0, so they contribute exact zeros to g_P and g_W;
    // columns p >= P have zero W^T rows, so g_s = 0 there.
    float x2r[16], gdv[16];
    load_rows16(x2s + 4 * h, x2r);
    if constexpr (GD) {
      float rof[16];
      load_rows16(reinterpret_cast<const float*>(rowoff) + 4 * h, rof);
      const unsigned pcol = static_cast<unsigned>(p * HW * 4);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const unsigned ro = __float_as_uint(rof[r]);
        gdv[r] = BufIO<float>::load(rgd, (ro != kOOB && pvalid) ? ro + pcol : kOOB, 0);
      }
    }
    f32x16 acc;  // starts at ||x||^2 + ||p||^2; the (-2 P) image does the rest
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = x2r[r] + p2;
#pragma unroll
    for (int q = 0; q < kNQ; ++q) {
      bf16x8 xa[T], pb[T];
      load_frag<T>(XA, 32 * kC, img_off<8>(j, 2 * q + h), xa);
      load_frag<T>(Pimg, Pp * kC, img_off<8>(p, 2 * q + h), pb);
      acc = mma_split<T>(xa, pb, acc);
    }
    f32x16 gacc = zero16();  // both class k-steps always run: zero W^T rows / GA columns past K
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 ga[T], wb[T];
      load_frag<T>(GA, 32 * 32, img_off<4>(j, 2 * s + h), ga);
      load_frag<T>(WTimg, Pp * 32, img_off<4>(p, 2 * s + h), wb);
      gacc = mma_split<T>(ga, wb, gacc);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float d = relu_f(acc[r]);
      float a;
      float gd = gacc[r] * act_grad_and_base<ACT>(d, eps, a);  // grad_unit is in the W^T image
      if constexpr (GD) gd += gdv[r];
      const float gs = d > 0.f ? gd : 0.f;
      gsum += gs;
      acc[r] = gs;  // XB holds -2x
      gacc[r] = a;  // act_unit is applied to g_W in the slab reduce
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
      bf16x8 gt[T];
      load_frag<T>(GT, 32 * 32, img_off<4>(j, 2 * s + h), gt);
      gw = mma_split<T>(gt, actb, gw);
    }
    if (it == 1) STAMP(5);
  }

  // ---- workgroup reduction over streams (fixed order) and slab write ----
  const int E = Pp * kC + 32 * Pp + Pp;
  float* my_slab = slab + static_cast<size_t>(blockIdx.x) * E;
  float* red = reinterpret_cast<float*>(smem_raw);  // [streams-1][npt][32*64 + 32*32 + 32]
  constexpr int kPerWave = 32 * kC + 32 * 32 + 32;
  __syncthreads();
  STAMP(6);
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
        for (int s2 = 1; s2 < streams; ++s2)
          v += red[static_cast<size_t>((s2 - 1) * npt + w) * kPerWave + pr * kC + ct * 32 + j];
        my_slab[static_cast<size_t>(w * 32 + pr) * kC + ct * 32 + j] = v;
      }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k = acc_row(r, h);
      float v = gw[r];
      for (int s2 = 1; s2 < streams; ++s2)
        v += red[static_cast<size_t>((s2 - 1) * npt + w) * kPerWave + 32 * kC + k * 32 + j];
      my_slab[static_cast<size_t>(Pp) * kC + static_cast<size_t>(k) * Pp + w * 32 + j] = v;
    }
    if (h == 0) {
      float v = gsum;
      for (int s2 = 1; s2 < streams; ++s2)
        v += red[static_cast<size_t>((s2 - 1) * npt + w) * kPerWave + 32 * kC + 1024 + j];
      my_slab[static_cast<size_t>(Pp) * kC + 32 * Pp + w * 32 + j] = v;
    }
  }
}

// Slab sum: 64 elements x 4 slab groups per workgroup, groups combined in fixed order; each
// thread keeps 8 independent loads in flight.
// blockIdx.y = prototype chunk: its slabs start at y * chunk_elems, its prototypes at y * per.
#ifndef REDUCE_GROUPS
#define REDUCE_GROUPS 4
#endif
// Slab groups per reduce workgroup: group g adds slabs g, g + kRG, ... (kReduceBatch loads in
// flight per step), then the groups' partials are added in group order.
constexpr int kRG = REDUCE_GROUPS;
__global__ __launch_bounds__(64 * kRG) void l2_bwd_reduce_bf16_kernel(const float* __restrict__ slab, int S, int P,
                                                                  int per, int K, int ldw, const float* __restrict__ protos,
                                                                  float w_unit, float* __restrict__ g_protos,
                                                                  float* __restrict__ g_w, size_t chunk_elems,
                                                                  int gp_t) {
  __shared__ float part[kRG][64];
  __shared__ float gpart[kRG][64];
  const int p0 = static_cast<int>(blockIdx.y) * per;
  slab += blockIdx.y * chunk_elems;
  protos += static_cast<size_t>(p0) * kC;
  if (g_protos) g_protos += static_cast<size_t>(p0) * kC;
  if (g_w) g_w += p0;
  P = P - p0 < per ? P - p0 : per;
  // slab layout: [R][64] g_P | [KR][R] g_W | [R] sum_n g_s with R = Pp rows and KR = 32 class
  // rows; gp_t 1: exact rows R = P, KR = K, and g_P transposed ([64][R]); gp_t 2 (the wave
  // kernel's): as gp_t 1 with rows padded to R = Pp (columns P .. Pp are never written: their sums
  // are formed and dropped, like every p >= P below), and the g_P slabs already hold 2 p sum_n g_s
  // (no sum_n g_s loads, no 2 p term here)
  const int Pp = (P + 31) & ~31;
  const int R = gp_t == 1 ? P : Pp, KR = gp_t ? K : 32;
  const int E = R * kC + KR * R + R;
  const int e = blockIdx.x * 64 + (threadIdx.x & 63);
  const int grp = threadIdx.x >> 6;
  const bool active = e < R * kC + KR * R;
  const bool is_gp = e < R * kC;
  const int p_of_e = is_gp ? (gp_t ? e % R : e / kC) : 0;
  const int gs_e = R * kC + KR * R + p_of_e;
  float s = 0.f, gs = 0.f;
  if (active) {
    // this group's slabs grp, grp + 4, ... added in order, kReduceBatch loads in flight per step;
    // the last step's loads are predicated, not issued one round trip at a time
    constexpr int kReduceBatch = 16;
    for (int si = grp; si < S; si += kRG * kReduceBatch) {
      float v[kReduceBatch], u[kReduceBatch];
#pragma unroll
      for (int k = 0; k < kReduceBatch; ++k) {
        const bool ok = si + kRG * k < S;
        v[k] = ok ? slab[static_cast<size_t>(si + kRG * k) * E + e] : 0.f;
        u[k] = ok && is_gp && gp_t != 2 ? slab[static_cast<size_t>(si + kRG * k) * E + gs_e] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < kReduceBatch; ++k) {
        if (si + kRG * k < S) {
          s += v[k];
          gs += u[k];
        }
      }
    }
  }
  part[grp][threadIdx.x & 63] = s;
  gpart[grp][threadIdx.x & 63] = gs;
  __syncthreads();
  if (grp != 0 || !active) return;
  const int l = threadIdx.x;
  float tot = part[0][l], gst = gpart[0][l];
#pragma unroll
  for (int g2 = 1; g2 < kRG; ++g2) {
    tot += part[g2][l];
    gst += gpart[g2][l];
  }
  if (is_gp) {
    const int c = gp_t ? e / R : e - p_of_e * kC;
    if (p_of_e < P && g_protos) {
      g_protos[static_cast<size_t>(p_of_e) * kC + c] =
          gp_t == 2 ? tot : tot + gst * (2.f * protos[static_cast<size_t>(p_of_e) * kC + c]);
    }
  } else {
    const int e2 = e - R * kC;
    const int k = e2 / R, pp = e2 - k * R;
    if (g_w && k < K && pp < P) g_w[static_cast<size_t>(k) * ldw + pp] = tot * w_unit;  // act = act_unit * act_base
  }
}

// ---- host side ---------------------------------------------------------------------------------
size_t p2_pad(const Geometry& g) { return (static_cast<size_t>(g.Pp) * 4 + 1023) & ~static_cast<size_t>(1023); }
size_t fwd_lds(const Geometry& g, int terms) {
  return static_cast<size_t>(g.Pp) * terms * (kC + 32) * 2 + p2_pad(g) +
         static_cast<size_t>(kWavesF) * kFwdPartRegs * 64 * 4;
}
size_t bwd_x_lds(const Geometry& g, int terms) {
  return static_cast<size_t>(g.Pp) * terms * (2 * kC + 32) * 2 + p2_pad(g) +
         static_cast<size_t>(kWavesA) * (kXPartRegs + 1) * 64 * 4;
}
size_t pw_lds_for(const Geometry& g, int terms, bool x_bf16, int streams) {
  const size_t stage = x_bf16 ? (terms == 2 ? PwStage<uint16_t, 2>::kBytes : PwStage<uint16_t, 3>::kBytes)
                              : (terms == 2 ? PwStage<float, 2>::kBytes : PwStage<float, 3>::kBytes);
  const size_t red = static_cast<size_t>(streams - 1) * (g.Pp / 32) * (32 * kC + 32 * 32 + 32) * sizeof(float);
  const size_t st = static_cast<size_t>(g.Pp) * terms * (kC + 32) * 2 + stage * streams;
  return st > red ? st : red;
}
// Pixel streams per workgroup: 2 when 2*npt waves fit the 768-thread launch bound and LDS.
int pw_streams(const Geometry& g, int terms, bool x_bf16) {
  return (g.Pp / 32) * 2 <= 12 && pw_lds_for(g, terms, x_bf16, 2) <= kMaxLds ? 2 : 1;
}
size_t pw_lds(const Geometry& g, int terms, bool x_bf16) {
  return pw_lds_for(g, terms, x_bf16, pw_streams(g, terms, x_bf16));
}
int pw_grid(const Geometry& g, int streams) {
  const int need = static_cast<int>(ceil_div(g.ntiles, streams));
  return need < 256 ? need : 256;
}

struct Bytes {
  unsigned x, d, a, l, gl, gd;
};

// Grid of the layout-A kernels (TileSchedule): ceil(ntiles / waves) workgroups up to the resident
// cap, except below one full round over the cap, where that grid leaves no full round and every
// tile in the remainder path, rounds deep: then up to FWD_REM_ROUNDS remainder rounds over the
// whole cap, else floor(ntiles / waves) workgroups (one full round, < waves remainder tiles).
static int layout_a_grid(int ntiles, int waves, int cap) {
  if (ntiles <= FWD_REM_ROUNDS * cap) return ntiles < cap ? ntiles : cap;
  if (ntiles < waves * cap) return ntiles / waves;
  const int want = static_cast<int>(ceil_div(ntiles, waves));
  return want < cap ? want : cap;
}

template <typename TX, int T, int ACT, bool ACTS, bool LOGITS>
int fwd_t(const Geometry& g, const Bytes& nb, const void* x, const unsigned char* img, float eps, float* dist,
          float* act, float* logits, int accumulate, hipStream_t stream) {
  if (int st = ensure_lds<l2_fwd_bf16_kernel<TX, T, ACT, ACTS, LOGITS>>()) return st;
  const size_t lds = fwd_lds(g, T);
  // Persistent: one generation of resident workgroups; waves stride over the tiles and
  // prefetch their next tile.
  const int cap = resident_blocks<l2_fwd_bf16_kernel<TX, T, ACT, ACTS, LOGITS>>(kWavesF * 64, lds);
  // Small batches (the drop-in runs 2-4 images per GPU): a full-round tile costs one wave
  // ≈ 2.6x a remainder tile (one workgroup, the prototype tiles split over its waves; stamps in
  // DESIGN.md §5.3), hence layout_a_grid's small-batch rule.
  const int grid = layout_a_grid(g.ntiles, kWavesF, cap);
  KernelTimer timer("l2_fwd_bf16_kernel", stream);
  hipLaunchKernelGGL((l2_fwd_bf16_kernel<TX, T, ACT, ACTS, LOGITS>), dim3(grid), dim3(kWavesF * 64), lds,
                     stream, static_cast<const TX*>(x), nb.x, g.HW, g.npix, img, g.P, g.Pp, g.K, eps, dist, nb.d, act,
                     nb.a, logits, nb.l, g.ldd, g.p0, accumulate, g.xsig);
  return check_launch("l2_fwd_bf16_kernel");
}

template <typename TX, int T, int ACT, bool GD>
int bwd_x_t(const Geometry& g, const Bytes& nb, const void* x, const unsigned char* img, float eps,
            const float* g_logits, const float* g_dist, void* g_x, int accumulate, hipStream_t stream) {
  if (int st = ensure_lds<l2_bwd_x_bf16_kernel<TX, T, ACT, GD>>()) return st;
  const size_t lds = bwd_x_lds(g, T);
  const int cap = resident_blocks<l2_bwd_x_bf16_kernel<TX, T, ACT, GD>>(kWavesA * 64, lds);
  KernelTimer timer("l2_bwd_x_bf16_kernel", stream);
  hipLaunchKernelGGL((l2_bwd_x_bf16_kernel<TX, T, ACT, GD>), dim3(layout_a_grid(g.ntiles, kWavesA, cap)),
                     dim3(kWavesA * 64), lds,
                     stream, static_cast<const TX*>(x), nb.x, g.HW, g.npix, img, g.P, g.Pp, g.K, eps, g_logits, nb.gl,
                     g_dist, nb.gd, g.ldd, g.p0, static_cast<TX*>(g_x), accumulate);
  return check_launch("l2_bwd_x_bf16_kernel");
}

template <typename TX, int T, int ACT, int MAXT, bool GD>
int bwd_pw_launch(const Geometry& g, const Bytes& nb, const void* x, const float* protos, const unsigned char* img,
                  float eps, const float* g_logits, const float* g_dist, float* g_protos, float* g_w, float* ws,
                  int streams, hipStream_t stream) {
  if (int st = ensure_lds<l2_bwd_pw_bf16_kernel<TX, T, ACT, MAXT, GD>>()) return st;
  const int grid = pw_grid(g, streams);
  const int threads = streams * (g.Pp / 32) * 64;
  {
    KernelTimer timer("l2_bwd_pw_bf16_kernel", stream);
    hipLaunchKernelGGL((l2_bwd_pw_bf16_kernel<TX, T, ACT, MAXT, GD>), dim3(grid), dim3(threads),
                       pw_lds(g, T, sizeof(TX) == 2), stream, static_cast<const TX*>(x), nb.x, g.HW, g.npix, img,
                       g.P, g.Pp, g.K, eps, g_logits, nb.gl, g_dist, nb.gd, g.ldd, g.p0, streams, ws);
  }
  if (int st = check_launch("l2_bwd_pw_bf16_kernel")) return st;
  return launch_bwd_reduce_bf16(g, ws, grid, protos, ACT, g_protos, g_logits ? g_w : nullptr, stream);
}

template <typename TX, int T, int ACT, bool GD>
int bwd_pw_t(const Geometry& g, const Bytes& nb, const void* x, const float* protos, const unsigned char* img,
             float eps, const float* g_logits, const float* g_dist, float* g_protos, float* g_w, float* ws,
             hipStream_t stream) {
  const int streams = pw_streams(g, T, sizeof(TX) == 2);
  if (streams * (g.Pp / 32) * 64 > 384)
    return bwd_pw_launch<TX, T, ACT, 768, GD>(g, nb, x, protos, img, eps, g_logits, g_dist, g_protos, g_w, ws, streams,
                                              stream);
  return bwd_pw_launch<TX, T, ACT, 384, GD>(g, nb, x, protos, img, eps, g_logits, g_dist, g_protos, g_w, ws, streams,
                                            stream);
}

template <typename Fn>
int by_type(bool x_bf16, int terms, int act_kind, Fn&& fn) {
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using A0 = std::integral_constant<int, 0>;
  using A1 = std::integral_constant<int, 1>;
  float* f = nullptr;
  uint16_t* b = nullptr;
  if (act_kind == 0) {
    if (terms == 2) return x_bf16 ? fn(b, I2(), A0()) : fn(f, I2(), A0());
    return x_bf16 ? fn(b, I3(), A0()) : fn(f, I3(), A0());
  }
  if (terms == 2) return x_bf16 ? fn(b, I2(), A1()) : fn(f, I2(), A1());
  return x_bf16 ? fn(b, I3(), A1()) : fn(f, I3(), A1());
}

// Buffer-resource sizes; a null tensor gets 0 bytes, so every access through it is dropped
// (stores) or reads 0 (loads) without a branch in the kernel.
Bytes bytes_of(const Geometry& g, bool x_bf16, const void* dist, const void* act, const void* logits,
               const void* g_logits, const void* g_dist) {
  Bytes nb;
  const unsigned long long npix = static_cast<unsigned long long>(g.npix);
  const unsigned d = static_cast<unsigned>(npix * g.ldd * 4), l = static_cast<unsigned>(npix * g.K * 4);
  nb.x = static_cast<unsigned>(npix * kC * (x_bf16 ? 2 : 4));
  nb.d = dist ? d : 0u;
  nb.a = act ? d : 0u;
  nb.l = logits ? l : 0u;
  nb.gl = g_logits ? l : 0u;
  nb.gd = g_dist ? d : 0u;
  return nb;
}

}  // namespace

// Every buffer these kernels address must stay below 2^31 bytes (kOOB arithmetic).
bool bf16_sizes_ok(const Geometry& g) {
  const unsigned long long npix = static_cast<unsigned long long>(g.npix);
  const unsigned long long big = npix * 4ull * static_cast<unsigned long long>(g.P > kC ? g.P : kC);
  return big < (1ull << 31);
}

bool bf16_fwd_fits(const Geometry& g, int terms) {
  return g.C == kC && fwd_lds(g, terms) <= kMaxLds && bf16_sizes_ok(g);
}
bool bf16_bwd_x_fits(const Geometry& g, int terms) {
  return g.C == kC && bwd_x_lds(g, terms) <= kMaxLds && bf16_sizes_ok(g);
}
bool bf16_bwd_pw_fits(const Geometry& g, int terms) {
  return g.C == kC && g.Pp <= 384 && pw_lds(g, terms, false) <= kMaxLds && pw_lds(g, terms, true) <= kMaxLds &&
         bf16_sizes_ok(g);
}
size_t bf16_bwd_pw_workspace(const Geometry& g) {
  // the largest slab count of any stream configuration (one stream per workgroup)
  return static_cast<size_t>(pw_grid(g, 1)) * (static_cast<size_t>(g.Pp) * kC + 32 * g.Pp + g.Pp) * sizeof(float);
}

size_t bf16_image_bytes(const Geometry& g, int terms) {
  return static_cast<size_t>(img_offsets(g.Pp, terms).total);
}

int launch_prep_bf16_chunks(const Geometry& g, int per, int nchunk, int terms, const float* protos,
                            const float* w_last, int act_kind, float eps, void* img, hipStream_t stream, int fwd_only) {
  const int Pp = static_cast<int>(ceil_div(per, 32) * 32);
  const int items = Pp * 8;  // the largest image loop (rows x 8 chunks)
  const dim3 grid(static_cast<unsigned>(ceil_div(items, 256)), 5, static_cast<unsigned>(nchunk));
  unsigned char* blk = static_cast<unsigned char*>(img);
  const unsigned cb = static_cast<unsigned>(img_offsets(Pp, terms).total);
  const float ws = act_unit(act_kind), wts = act_grad_unit(act_kind, eps);
  if (terms == 2)
    hipLaunchKernelGGL(l2_prep_bf16_kernel<2>, grid, dim3(256), 0, stream, protos, g.P, per, w_last, g.K, g.ldw, ws,
                       wts, blk, cb, fwd_only);
  else
    hipLaunchKernelGGL(l2_prep_bf16_kernel<3>, grid, dim3(256), 0, stream, protos, g.P, per, w_last, g.K, g.ldw, ws,
                       wts, blk, cb, fwd_only);
  return check_launch("l2_prep_bf16_kernel");
}

int launch_prep_bf16(const Geometry& g, int terms, const float* protos, const float* w_last, int act_kind, float eps,
                     void* img, hipStream_t stream, int fwd_only) {
  return launch_prep_bf16_chunks(g, g.P, 1, terms, protos, w_last, act_kind, eps, img, stream, fwd_only);
}

int launch_adam_prep_bf16(const AdamPrepArgs& a, hipStream_t stream) {
  if (a.P <= 0 || a.K < 0 || a.K > 32 || !a.p || !a.gp || !a.mp || !a.vp || !a.stp || !a.block ||
      (a.K > 0 && (!a.w || !a.gw || !a.mw || !a.vw || !a.stw)))
    return fail(PROTOSEG_ERR_INVALID, "adam_prep: null tensor or K outside 0..32");
  hipLaunchKernelGGL(l2_adam_prep_kernel, dim3(static_cast<unsigned>(ceil_div(a.P, 32))), dim3(kApThreads), 0, stream, a);
  return check_launch("l2_adam_prep_kernel");
}

int launch_bwd_reduce_bf16_chunks(const Geometry& g, int per, int nchunk, const float* ws, int slabs,
                                  size_t chunk_elems, const float* protos, int act_kind, float* g_protos, float* g_w,
                                  hipStream_t stream, int gp_t) {
  const int Pp = static_cast<int>(ceil_div(per, 32) * 32);
  const int elems = gp_t == 1 ? per * (kC + g.K) : gp_t == 2 ? Pp * (kC + g.K) : Pp * kC + 32 * Pp;
  hipLaunchKernelGGL(l2_bwd_reduce_bf16_kernel, dim3(static_cast<unsigned>(ceil_div(elems, 64)), nchunk), dim3(64 * kRG),
                     0, stream, ws, slabs, g.P, per, g.K, g.ldw, protos, act_unit(act_kind), g_protos, g_w,
                     chunk_elems, gp_t);
  return check_launch("l2_bwd_reduce_bf16_kernel");
}

int launch_bwd_reduce_bf16(const Geometry& g, const float* ws, int slabs, const float* protos, int act_kind,
                           float* g_protos, float* g_w, hipStream_t stream) {
  return launch_bwd_reduce_bf16_chunks(g, g.P, 1, ws, slabs, 0, protos, act_kind, g_protos, g_w, stream);
}

int launch_fwd_bf16(const Geometry& g, bool x_bf16, int terms, const void* x, const void* img, float eps, int act_kind,
                    float* dist, float* act, float* logits, hipStream_t stream, int accumulate) {
  const Bytes nb = bytes_of(g, x_bf16, dist, act, logits, nullptr, nullptr);
  const unsigned char* blk = static_cast<const unsigned char*>(img);
  return by_type(x_bf16, terms, act_kind, [&](auto tx, auto tt, auto aa) {
    using TX = std::remove_pointer_t<decltype(tx)>;
    constexpr int kT = decltype(tt)::value, kA = decltype(aa)::value;
    if (act) {
      if (logits) return fwd_t<TX, kT, kA, true, true>(g, nb, x, blk, eps, dist, act, logits, accumulate, stream);
      return fwd_t<TX, kT, kA, true, false>(g, nb, x, blk, eps, dist, act, logits, accumulate, stream);
    }
    if (logits) return fwd_t<TX, kT, kA, false, true>(g, nb, x, blk, eps, dist, act, logits, accumulate, stream);
    return fwd_t<TX, kT, kA, false, false>(g, nb, x, blk, eps, dist, act, logits, accumulate, stream);
  });
}

int launch_bwd_x_bf16(const Geometry& g, bool x_bf16, int terms, const void* x, const void* img, float eps,
                      int act_kind, const float* g_logits, const float* g_dist, void* g_x, hipStream_t stream,
                      int accumulate) {
  const Bytes nb = bytes_of(g, x_bf16, nullptr, nullptr, nullptr, g_logits, g_dist);
  const unsigned char* blk = static_cast<const unsigned char*>(img);
  return by_type(x_bf16, terms, act_kind, [&](auto tx, auto tt, auto aa) {
    using TX = std::remove_pointer_t<decltype(tx)>;
    constexpr int kT = decltype(tt)::value, kA = decltype(aa)::value;
    if (g_dist) return bwd_x_t<TX, kT, kA, true>(g, nb, x, blk, eps, g_logits, g_dist, g_x, accumulate, stream);
    return bwd_x_t<TX, kT, kA, false>(g, nb, x, blk, eps, g_logits, g_dist, g_x, accumulate, stream);
  });
}

int launch_bwd_pw_bf16(const Geometry& g, bool x_bf16, int terms, const void* x, const float* protos, const void* img,
                       float eps, int act_kind, const float* g_logits, const float* g_dist, float* g_protos,
                       float* g_w, float* ws, hipStream_t stream) {
  const Bytes nb = bytes_of(g, x_bf16, nullptr, nullptr, nullptr, g_logits, g_dist);
  const unsigned char* blk = static_cast<const unsigned char*>(img);
  return by_type(x_bf16, terms, act_kind, [&](auto tx, auto tt, auto aa) {
    using TX = std::remove_pointer_t<decltype(tx)>;
    constexpr int kT = decltype(tt)::value, kA = decltype(aa)::value;
    if (g_dist) return bwd_pw_t<TX, kT, kA, true>(g, nb, x, protos, blk, eps, g_logits, g_dist, g_protos, g_w, ws, stream);
    return bwd_pw_t<TX, kT, kA, false>(g, nb, x, protos, blk, eps, g_logits, g_dist, g_protos, g_w, ws, stream);
  });
}

}  // namespace protoseg

#ifdef PROTOSEG_STAMPS
namespace protoseg {
__device__ unsigned long long g_stamps[kStampCap];
}
// Debug builds only: copy (and clear) the per-wave phase stamps of the last launches.
extern "C" int protoseg_debug_stamps(void* dst, size_t bytes) {
  using protoseg::g_stamps;
  const size_t n = bytes < sizeof(g_stamps) ? bytes : sizeof(g_stamps);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  if (dst && hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_stamps), n, 0, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_stamps)) != hipSuccess) return 3;
  return hipMemset(p, 0, sizeof(g_stamps)) == hipSuccess ? 0 : 3;
}
#endif
