// l2_bwd_onepass.hip — the prototype layer's training backward for up to 384 prototypes in ONE
// pass (bf16x3, C = 64). 19 prototypes/class x 19 classes (P = 361, the metric's config) reads
// X and g_logits once and writes g_x once, where the 192-prototype fused kernel
// (l2_bwd_fused.hip) ran two chunks, each re-reading X, the second adding to g_x. It is the
// autograd of reference model.py:203-221 (_l2_convolution), 231-237 (distance_2_similarity) and
// 259-283 (forward_from_conv_features):
//   S = ||x||^2 + ||p||^2 - 2 X.P^T,  d = relu(S),  act = f(d),  logits = act . W^T
//   g_act = g_logits . W,  g_s = (g_act f'(d) + g_dist) [d > 0]
//   g_x   = 2 x sum_p g_s - 2 g_s . P          g_P = 2 p sum_n g_s - 2 g_s^T . X
//   g_W   = g_logits^T . act
//
// Workgroup = 8 waves (2 per SIMD), one per CU, persistent over 32-pixel tiles; every product
// on v_mfma_f32_16x16x32_bf16 (16 x 16 tiles, 32-deep k-steps). Every wave has the same two
// roles, so the four SIMDs carry equal MFMA and VALU work and each SIMD's two waves cover each
// other's epilogue:
//   phase A (owner): wave w owns prototypes 16 NPT w .. +16 NPT (NPT = 3 at Pp = 384). Layout B
//     (rows = pixels, columns = prototypes: the prototype is on the lane): S with the owned rows
//     of the (-2P) image in LDS as B fragments, g_act with W^T B fragments streamed from the
//     (L2-resident) operand block, the epilogue, then g_P += g_s^T X and g_W += g_logits^T act with the accumulators as the A /
//     B operands (the contraction runs over their rows: k-slot (g, e) of a lane group g is pixel
//     4g + e of n-tile 0 for e < 4, 16 + 4g + e - 4 of n-tile 1 after), so g_P / g_W stay in
//     registers for the launch and go out once as this workgroup's slab. g_s goes to LDS as a
//     [p][n] image.
//   phase B (after a barrier): wave w computes g_x^T for channels 16 (w & 3) .. +15 and pixels
//     16 (w >> 2) .. +15 over ALL prototypes: A from the same (-2P) image by transposed reads
//     (one image in LDS for the launch serves both orientations), B from the g_s image by transposed reads
//     (ds_read_b64_tr_b16). sum_p g_s (the 2 x sum_p g_s term) comes from the same B fragments
//     times a ones A operand, each wave over a quarter of the k-steps; the four partials are
//     added in a fixed order after the second barrier.
// The x / g_logits images and the g_s image carry XOR swizzles found by tools/lds_swizzle_check.py
// that make every access pattern above conflict-free.
#include <type_traits>

#ifdef PROTOSEG_STAMPS
#include <hip/hip_runtime.h>
namespace protoseg {
__device__ unsigned long long g_stamps_onepass[1 << 17];
}
// 16 slots per wave (tools/stamps_onepass.py), fenced so the phases they bracket stay in place
// (debug builds only: production code has neither stamps nor fences).
#define OSTAMP(slot)                                                                                 \
  do {                                                                                               \
    __builtin_amdgcn_sched_barrier(0);                                                               \
    const unsigned _w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);                         \
    if ((threadIdx.x & 63) == 0 && _w * 16 + (slot) < (1u << 17))                                    \
      ::protoseg::g_stamps_onepass[_w * 16 + (slot)] = __builtin_amdgcn_s_memtime();                 \
    __builtin_amdgcn_sched_barrier(0);                                                               \
  } while (0)
#else
#define OSTAMP(slot) \
  do {               \
  } while (0)
#endif
#include "bf16_split.h"
#include "l2_bf16_common.h"
#include "l2_launch.h"
#include "l2_onepass_layout.h"
#include "protoseg_host.h"

namespace protoseg {

namespace {

using namespace bf16l;

constexpr int kOW = 8;  // waves per workgroup
constexpr int kOT = onepass::kT;  // split terms (bf16x3: 3 MFMAs per product)
constexpr int kOThreads = kOW * 64;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// ---- operand block: l2_onepass_layout.h (built by l2_prep_onepass_kernel, or by the forward's
// prep launch beside its own images)
using OneOffsets = onepass::Offsets;
__host__ __device__ constexpr OneOffsets one_offsets(int Pp) { return onepass::offsets(Pp); }
using onepass::pi_swz;

// LDS regions (bytes)
struct OneLds {
  int pimg, gs, xa, ga, x2s, ro, cl, sig, total;
};
__host__ __device__ constexpr OneLds one_lds(int Pp) {
  OneLds o{};
  o.pimg = 0;                         // the (-2P) image (the pi region), Pp x 256 B
  o.gs = o.pimg + kOT * Pp * 128;     // [term][Pp][32 n] bf16, 64-B rows of 8-B slots
  o.xa = o.gs + kOT * Pp * 64;        // [term][32 n][64 c] bf16, 160-B rows (128 B + 32 B pad)
  o.ga = o.xa + kOT * 32 * 160;       // [term][32 n][32 k] bf16, 64-B rows of 16-B chunks
  o.x2s = o.ga + kOT * 32 * 64;       // [32] f32 ||x||^2
  o.ro = o.x2s + 32 * 4;              // [32] u32 g_dist byte offset per pixel
  o.cl = o.ro + 32 * 4;               // [32] int: the pixel's KLD class (compact g_dist, GD = 2)
  o.sig = o.cl + 32 * 4;              // [2 slots][2 pixel halves][4 channel tiles][16] f32
  o.total = o.sig + 2 * 2 * 4 * 16 * 4;
  return o;
}

// Image offsets in bf16 elements (tools/lds_swizzle_check.py checks every access pattern).
// x image: row n (64 channels) at a 160-B stride: the padding, not an XOR swizzle, makes the A
// reads (16 rows x 16 B) and the transposed reads (4 rows x 4 slots per 16-lane group)
// conflict-free, so every n-tile / k-step / channel-tile variant of an access is an immediate
// offset from one per-lane base (no per-variant address registers).
constexpr int kXaRow = 80;  // bf16 elements per x-image row
constexpr int kXaPlane = 32 * kXaRow;
__device__ __forceinline__ int xa_off(int n, int chunk) { return n * kXaRow + (chunk << 3); }
// g_logits image: row n (32 classes), chunk k at (k ^ ((n >> 1) & 2)) & 3.
__device__ __forceinline__ int ga_off(int n, int chunk) { return n * 32 + (((chunk ^ ((n >> 1) & 2)) & 3) << 3); }
// g_s image: row p (32 pixels), 8-B slot s (pixels 4s .. 4s+3) at s ^ (((p >> 2) & 1) | ((p >> 1) & 4)).
__device__ __forceinline__ int gs_off2(int p, int slot) {
  return p * 32 + ((slot ^ (((p >> 2) & 1) | ((p >> 1) & 4))) << 2);
}
// (-2P) image: row p (64 channels), 16-B chunk q at q ^ pi_swz(p) (l2_onepass_layout.h).
__device__ __forceinline__ int pi_off(int p, int chunk) { return p * 64 + (((chunk ^ pi_swz(p)) & 7) << 3); }

__device__ __forceinline__ bf16x8 tr_pair(const bf16* lo, const bf16* hi) {
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(lo));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(hi));
  const s16x8 v = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// a * b for split operands, smallest products first: a0 b1, a1 b0, a0 b0 (the forward's order
// with a = P, b = x; the S product below passes x as a and P as b in the mirrored order)
__device__ __forceinline__ f32x4 mma16_split(const bf16x8 (&a)[kOT], const bf16x8 (&b)[kOT], f32x4 c) {
  c = mfma16(a[0], b[1], c);
  c = mfma16(a[1], b[0], c);
  return mfma16(a[0], b[0], c);
}

// Eight floats -> split fragments (term t) and the 4-element halves as 8-byte LDS stores.
__device__ __forceinline__ void store_half4(bf16* dst, const bf16x8& f, int half) {
  const s16x8 v = __builtin_bit_cast(s16x8, f);
  *reinterpret_cast<s16x4*>(dst) = half ? __builtin_shufflevector(v, v, 4, 5, 6, 7) : __builtin_shufflevector(v, v, 0, 1, 2, 3);
}

#define OSCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#ifndef ONEPASS_PB_FREE
#define ONEPASS_PB_FREE 0  // 1: no scheduling fence per phase-B k-step (measured variant)
#endif
#ifndef ONEPASS_PRIO
#define ONEPASS_PRIO 0  // 1: s_setprio 1 for waves 4..7 (measured variant)
#endif
#ifndef ONEPASS_PIPE
#define ONEPASS_PIPE 1  // owned tile jt + 1's products issued before tile jt's epilogue
#endif
#ifndef PB_DEPTH
#define PB_DEPTH 2  // phase B: k-steps of fragments in flight ahead of the one multiplying (2: -1.1 % vs 1)
#endif

// GD: 0 no distance gradient, 1 a dense g_dist, 2 the KLD loss's compact one (CompactGd).
template <typename TX, int ACT, int GD, bool XSIG, int NPT>
__global__ __launch_bounds__(kOThreads, 1) void l2_bwd_onepass_bf16_kernel(
    const TX* __restrict__ x, unsigned x_bytes, int HW, int npix, const unsigned char* __restrict__ img, int P,
    int K, float eps, const float* __restrict__ g_logits, unsigned gl_bytes, const float* __restrict__ g_dist,
    unsigned gd_bytes, int gd_ld, int gd_p0, CompactGd cg, TX* __restrict__ g_x, int accumulate,
    float* __restrict__ slab) {
  constexpr int Pp = kOW * NPT * 16;  // prototype columns of the images
  constexpr int KS = Pp / 32;         // g_x k-steps (a multiple of 4)
  constexpr int KSQ = KS / 4;         // sum_p g_s k-steps per channel-tile wave
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  constexpr OneLds L = one_lds(Pp);
  constexpr OneOffsets io = one_offsets(Pp);
  const bf16* PI = reinterpret_cast<const bf16*>(smem_raw + L.pimg);
  bf16* GS = reinterpret_cast<bf16*>(smem_raw + L.gs);
  bf16* XA = reinterpret_cast<bf16*>(smem_raw + L.xa);
  bf16* GA = reinterpret_cast<bf16*>(smem_raw + L.ga);
  float* X2S = reinterpret_cast<float*>(smem_raw + L.x2s);
  unsigned* RO = reinterpret_cast<unsigned*>(smem_raw + L.ro);
  int* CL = reinterpret_cast<int*>(smem_raw + L.cl);
  float* SIG = reinterpret_cast<float*>(smem_raw + L.sig);

  const int lane = threadIdx.x & 63, g = lane >> 4, m = lane & 15, wave = wave_id();
  const int ntiles = (npix + 31) / 32;
  const int G = static_cast<int>(gridDim.x);
  const int iters = (ntiles - static_cast<int>(blockIdx.x) + G - 1) / G;
  const unsigned sz = sizeof(TX);
  const unsigned chs = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(HW) * sz);  // one channel plane
  const rsrc_t rx = make_rsrc(x, x_bytes), rg = make_rsrc(g_logits, gl_bytes);
  // GD = 2: g_dist points at the compact values (gd_bytes = npix * mpc * 4)
  const rsrc_t rgd = make_rsrc(GD == 2 ? cg.val : g_dist, gd_bytes), rgx = make_rsrc(g_x, g_x ? x_bytes : 0u);
  const rsrc_t rimg = make_rsrc(img, static_cast<unsigned>(io.total));
  auto tile_of = [&](int i) __attribute__((always_inline)) { return static_cast<int>(blockIdx.x) + i * G; };

  // ---- prologue: the (-2P) image -> LDS (for the launch); the owned ||p||^2 -> registers ------
  lds_copy(smem_raw + L.pimg, img + io.pi, io.p2 - io.pi);

  float p2[NPT];
  int pcls[NPT], pslot[NPT];  // GD = 2: the owned prototypes' class and compact column (bytes)
#pragma unroll
  for (int jt = 0; jt < NPT; ++jt) {
    const int ptile = wave * NPT + jt;
    p2[jt] = reinterpret_cast<const float*>(img + io.p2)[ptile * 16 + m];
    if constexpr (GD == 2) {
      const int pp = ptile * 16 + m;
      const int code = pp < P ? cg.slot[gd_p0 + pp] : 0;
      pcls[jt] = pp < P ? code >> 8 : -2;  // never a pixel class (those are >= -1)
      pslot[jt] = (code & 255) * 4;
    }
  }

  // Lane-derived LDS / buffer addresses are loop-invariant; held across the tile loop they are the
  // first values the allocator spills (a spilled address costs a scratch reload and a vmcnt(0)
  // per tile), so each phase rebuilds them from the lane id plus an opaque zero (a few VALU).
  auto opaque_lane = [&]() __attribute__((always_inline)) {
    int z = 0;
    asm volatile("" : "+v"(z));
    return lane + z;
  };

  // ---- staging: wave w stages pixels 4w .. 4w+3 of a tile. Lanes 0..31: x of pixel 4w + l/8,
  // chunk ch = l & 7 = channels chan_of(ch >> 1, ch & 1, 0..7) (the family's ||x||^2 order);
  // lanes 32..47: 8 classes (8 kc ..) of pixel 4w + (l - 32) / 4. Raw values go to registers
  // first (issued one phase ahead), then split into the images.
  float raw[8];
  int rcl = -1;  // GD = 2, lanes 48 .. 51: the KLD class of pixel 4 wave + lane - 48
  auto load_raw = [&](int t) __attribute__((always_inline)) {
    const int lz = opaque_lane();
    const int sn = 4 * wave + ((lz & 31) >> 3), sch = lz & 7;
    const int gn = 4 * wave + ((lz - 32) >> 2), gkc = lz & 3;
    if (lane < 32) {
      const int gp = t * 32 + sn;
      unsigned off = kOOB;
      if (gp < npix) {
        const int b = div_pix(gp, HW);
        off = static_cast<unsigned>((b * kC) * HW + (gp - b * HW)) * sz;
      }
      // channel chan_of(q, h, e) = lane part (q, h) + element part (e): the lane part goes into
      // the per-lane voffset (a divergent soffset makes hipcc emit a waterfall loop per load),
      // the uniform element part into the soffset, so no per-element offsets stay live
      const unsigned vo = off == kOOB ? kOOB : off + static_cast<unsigned>(chan_of(sch >> 1, sch & 1, 0) * HW) * sz;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        raw[e] = BufIO<TX>::load(rx, vo, __builtin_amdgcn_readfirstlane(static_cast<unsigned>(chan_of(0, 0, e)) * chs));
    } else {
      if constexpr (GD == 2) {
        const int gc = t * 32 + 4 * wave + (lane - 48);
        if (lane >= 48 && lane < 52) rcl = gc < npix ? cg.pix[gc] : -1;
      }
      const int gg = t * 32 + gn;
      const bool ok = lane < 48 && gg < npix;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = 8 * gkc + e;
        raw[e] = BufIO<float>::load(rg, (ok && k < K) ? static_cast<unsigned>((gg * K + k) * 4) : kOOB, 0u);
      }
    }
  };
  auto convert = [&](int t) __attribute__((always_inline)) {
    float v[8];
    bf16x8 f[kOT];
    const int lz = opaque_lane();
    const int sn = 4 * wave + ((lz & 31) >> 3), sch = lz & 7;
    const int gn = 4 * wave + ((lz - 32) >> 2), gkc = lz & 3;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = raw[e];
    if (lane < 32) {
      if constexpr (XSIG) {  // pixels past the map stay 0 (their g_s is 0 anyway)
        const bool ok = t * 32 + sn < npix;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = ok ? sigmoid_f(v[e]) : 0.f;
      }
      split8<kOT>(v, f);
      // element e of the chunk is channel chan_of(q, h, e): e = 0..3 and 4..7 are 4-channel runs
      const int q = sch >> 1, hh = sch & 1;
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int c = chan_of(q, hh, 4 * half);
#pragma unroll
        for (int t2 = 0; t2 < kOT; ++t2)
          store_half4(XA + t2 * kXaPlane + xa_off(sn, c >> 3) + (c & 7), f[t2], half);
      }
      // ||x||^2 in the family's fixed order (chunk fma chains, then pairs, quads, halves)
      float s = chunk_sq(v);
      s += __shfl_xor(s, 1);
      s += __shfl_xor(s, 2);
      s += __shfl_xor(s, 4);
      if (sch == 0) X2S[sn] = s;
    } else if (lane < 48) {
      split8<kOT>(v, f);
#pragma unroll
      for (int t2 = 0; t2 < kOT; ++t2) *reinterpret_cast<bf16x8*>(GA + t2 * 32 * 32 + ga_off(gn, gkc)) = f[t2];
      if constexpr (GD == 1) {
        if (gkc == 0) {
          const int gg = t * 32 + gn;
          const bool ok = gg < npix;
          const int b = ok ? div_pix(gg, HW) : 0;
          RO[gn] = ok ? static_cast<unsigned>(((b * gd_ld + gd_p0) * HW + (gg - b * HW)) * 4) : kOOB;
        }
      }
    } else if (GD == 2 && lane < 52) {  // the pixel's compact row and class
      const int n = 4 * wave + (lane - 48);
      RO[n] = rcl >= 0 ? static_cast<unsigned>((t * 32 + n) * cg.mpc * 4) : kOOB;
      CL[n] = rcl;
    }
  };

  // transposed-read lane roles: lane 4 qq + pp of group g supplies row qq of its 4-row block,
  // 8-B slot pp of the block's 16 columns

  // ---- phase A: owned prototype tile jt (16 prototypes) against the staged 32 pixels ---------
  f32x4 gp[NPT][4], gw[NPT][2];
  float gsum[NPT];
#pragma unroll
  for (int jt = 0; jt < NPT; ++jt) {
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) gp[jt][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
    gw[jt][0] = gw[jt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    gsum[jt] = 0.f;
  }
  // lz: the opaque lane id of this pixel tile's phase A (one per tile, shared by the owned
  // prototype tiles, whose addresses differ by immediates: the swizzles use row bits below 16).
  // An owned tile runs in two halves: the front (S and g_act products, the g_dist loads) and the
  // back (epilogue, g_s image, g_P / g_W products). The main loop issues tile jt + 1's front
  // before tile jt's back, so the epilogue's VALU runs beside the next tile's MFMAs.
  struct Front {
    f32x4 acc[2], gacc[2];
    float gdv[8];
  };
  auto owner_front = [&](int jt, int lz, Front& fr) __attribute__((always_inline)) {
    const int m = lz & 15, g = lz >> 4;
    const int p = (wave * NPT + jt) * 16 + m;
    // the x / g_logits operands are the same for every owned tile: an opaque zero on their image
    // bases makes each tile reload them instead of keeping their fragments live across the tiles
    int zj = 0;
    asm volatile("" : "+v"(zj));
    const bf16* XAj = XA + zj;
    const bf16* GAj = GA + zj;
    f32x4 (&acc)[2] = fr.acc;
    f32x4 (&gacc)[2] = fr.gacc;
    float (&gdv)[8] = fr.gdv;
    bf16x8 psj[2][kOT];  // S B fragments: rows p of the (-2P) image
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int t = 0; t < kOT; ++t)
        psj[ks][t] = *reinterpret_cast<const bf16x8*>(PI + t * Pp * 64 + pi_off(p, 4 * ks + g));
    bf16x8 wtj[kOT];  // this tile's g_act B fragments, streamed from the (L2-resident) operand block
#pragma unroll
    for (int t = 0; t < kOT; ++t)  // lane part in the voffset, the tile's (uniform) part in the soffset
      wtj[t] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                              rimg, static_cast<unsigned>(lz * 16),
                                              static_cast<unsigned>(io.wt + ((wave * NPT + jt) * kOT + t) * 1024), 0));
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const float4 x2 = *reinterpret_cast<const float4*>(X2S + 16 * nt + 4 * g);
      acc[nt] = f32x4{x2.x + p2[jt], x2.y + p2[jt], x2.z + p2[jt], x2.w + p2[jt]};
      // S: x (A) against (-2P) (B) in the forward's product order, k-steps of 32 channels
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 xa[kOT];
#pragma unroll
        for (int t = 0; t < kOT; ++t)
          xa[t] = *reinterpret_cast<const bf16x8*>(XAj + t * kXaPlane + xa_off(16 * nt + m, 4 * ks + g));
        acc[nt] = mfma16(xa[1], psj[ks][0], acc[nt]);
        acc[nt] = mfma16(xa[0], psj[ks][1], acc[nt]);
        acc[nt] = mfma16(xa[0], psj[ks][0], acc[nt]);
      }
      bf16x8 ga[kOT];
#pragma unroll
      for (int t = 0; t < kOT; ++t) ga[t] = *reinterpret_cast<const bf16x8*>(GAj + t * 32 * 32 + ga_off(16 * nt + m, g));
      gacc[nt] = mma16_split(ga, wtj, f32x4{0.f, 0.f, 0.f, 0.f});
    }
    if constexpr (GD == 2) {
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const uint4 ro = *reinterpret_cast<const uint4*>(RO + 16 * nt + 4 * g);
        const int4 cl = *reinterpret_cast<const int4*>(CL + 16 * nt + 4 * g);
        const unsigned rv[4] = {ro.x, ro.y, ro.z, ro.w};
        const int cv[4] = {cl.x, cl.y, cl.z, cl.w};
#pragma unroll
        for (int r = 0; r < 4; ++r)
          gdv[4 * nt + r] = BufIO<float>::load(rgd, cv[r] == pcls[jt] ? rv[r] + pslot[jt] : kOOB, 0);
      }
    } else if constexpr (GD == 1) {
      const unsigned pcol = static_cast<unsigned>(p * HW * 4);
      const bool pvalid = p < P;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const uint4 ro = *reinterpret_cast<const uint4*>(RO + 16 * nt + 4 * g);
        const unsigned rv[4] = {ro.x, ro.y, ro.z, ro.w};
#pragma unroll
        for (int r = 0; r < 4; ++r)
          gdv[4 * nt + r] = BufIO<float>::load(rgd, (rv[r] != kOOB && pvalid) ? rv[r] + pcol : kOOB, 0);
      }
    }
  };
  auto owner_back = [&](int jt, int lz, Front& fr) __attribute__((always_inline)) {
    const int m = lz & 15, g = lz >> 4, qq = (lz >> 2) & 3, pp = lz & 3;
    const int p = (wave * NPT + jt) * 16 + m;
    int zj = 0;
    asm volatile("" : "+v"(zj));
    const bf16* XAj = XA + zj;
    const bf16* GAj = GA + zj;
    const f32x4 (&acc)[2] = fr.acc;
    const f32x4 (&gacc)[2] = fr.gacc;
    const float (&gdv)[8] = fr.gdv;
    // epilogue: element e = 4 nt + r is pixel (16 nt + 4 g + r): the A / B k-slot order
    float gs[8], av[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = relu_f(acc[e >> 2][e & 3]);
      float a;
      float gd = gacc[e >> 2][e & 3] * act_grad_and_base<ACT>(d, eps, a);  // grad_unit is in W^T
      if constexpr (GD) gd += gdv[e];
      gs[e] = d > 0.f ? gd : 0.f;  // relu backward
      gsum[jt] += gs[e];
      av[e] = a;  // act_unit is applied to g_W in the slab reduce
    }
    bf16x8 gsf[kOT], actf[kOT];
    split8<kOT>(gs, gsf);
    split8<kOT>(av, actf);
    // g_s -> [p][n] image: pixels 4g .. 4g+3 (slot g) and 16 + 4g .. (slot 4 + g)
#pragma unroll
    for (int t = 0; t < kOT; ++t) {
      store_half4(GS + t * Pp * 32 + gs_off2(p, g), gsf[t], 0);
      store_half4(GS + t * Pp * 32 + gs_off2(p, 4 + g), gsf[t], 1);
    }
    OSCHED_FENCE();
    // g_P[p][c] += g_s^T X: B = x[n][c] with the k-slot pixels, transposed reads of the x image
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      bf16x8 xb[kOT];
      const int slot = 4 * ct + pp, chunk = slot >> 1, sub = (slot & 1) * 4;
#pragma unroll
      for (int t = 0; t < kOT; ++t)
        xb[t] = tr_pair(XAj + t * kXaPlane + xa_off(4 * g + qq, chunk) + sub, XAj + t * kXaPlane + xa_off(16 + 4 * g + qq, chunk) + sub);
      gp[jt][ct] = mma16_split(gsf, xb, gp[jt][ct]);
    }
    // g_W[k][p] += g_logits^T act: A = g_logits[n][k] transposed (lane = class)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      bf16x8 gl[kOT];
      const int slot = 4 * kt + pp, chunk = slot >> 1, sub = (slot & 1) * 4;
#pragma unroll
      for (int t = 0; t < kOT; ++t)
        gl[t] = tr_pair(GAj + t * 32 * 32 + ga_off(4 * g + qq, chunk) + sub, GAj + t * 32 * 32 + ga_off(16 + 4 * g + qq, chunk) + sub);
      gw[jt][kt] = mma16_split(gl, actf, gw[jt][kt]);
    }
  };

  // ---- phase B: g_x^T of channels 16 ct .. +15, pixels 16 nh .. +15, over all Pp prototypes ----
  const int ct = wave & 3, nh = wave >> 2;
  f32x4 gx;
  float xe[4], olde[4];  // x (and the earlier chunks' g_x) at the lane's output elements
  // output element r: channel 16 ct + 4 g + r, pixel 16 nh + m of the tile
  auto out_off = [&](int t, int m, int g) __attribute__((always_inline)) -> unsigned {
    const int gp = t * 32 + 16 * nh + m;
    if (gp >= npix) return kOOB;
    const int b = div_pix(gp, HW);
    return static_cast<unsigned>((b * kC + 16 * ct + 4 * g) * HW + (gp - b * HW)) * sz;
  };
  auto phase_b = [&](int t, int slot) __attribute__((always_inline)) {
    const int lz = opaque_lane();
    const int m = lz & 15, g = lz >> 4, qq = (lz >> 2) & 3, pp = lz & 3;
    const unsigned o = out_off(t, m, g);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      xe[r] = BufIO<TX>::load(rx, o, static_cast<unsigned>(r * HW) * sz);
      olde[r] = 0.f;
    }
    if (accumulate) {
#pragma unroll
      for (int r = 0; r < 4; ++r) olde[r] = BufIO<TX>::load(rgx, o, static_cast<unsigned>(r * HW) * sz);
    }
    gx = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 sg = f32x4{0.f, 0.f, 0.f, 0.f};
    // g_x: the fully unrolled k-loop reads the fragments of k-step ks + PB_DEPTH while k-step ks
    // multiplies (the LDS latency hides behind the MFMAs instead of being exposed once per
    // k-step); every read is a per-lane base + an immediate offset (the image swizzles depend
    // on row bits below 32, so a k-step moves every address by the same amount).
    const int aslot = 4 * ct + pp, chunk = aslot >> 1, sub = (aslot & 1) * 4, row0 = 8 * g + qq;
    const bf16* pa0 = PI + pi_off(row0, chunk) + sub;  // rebuilt per tile (opaque lane), not held across phase A
    const bf16* pa1 = PI + pi_off(row0 + 4, chunk) + sub;
    const bf16* pb0 = GS + gs_off2(row0, 4 * nh + pp);
    const bf16* pb1 = GS + gs_off2(row0 + 4, 4 * nh + pp);
    auto ldk = [&](int ks, bf16x8 (&a)[kOT], bf16x8 (&b)[kOT]) __attribute__((always_inline)) {
#pragma unroll
      for (int t2 = 0; t2 < kOT; ++t2) {
        a[t2] = tr_pair(pa0 + t2 * Pp * 64 + ks * 32 * 64, pa1 + t2 * Pp * 64 + ks * 32 * 64);
        b[t2] = tr_pair(pb0 + t2 * Pp * 32 + ks * 32 * 32, pb1 + t2 * Pp * 32 + ks * 32 * 32);
      }
    };
    constexpr int D = PB_DEPTH;
    bf16x8 fa[D + 1][kOT], fb[D + 1][kOT];
#pragma unroll
    for (int j = 0; j < D; ++j) ldk(j, fa[j], fb[j]);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + D < KS) ldk(ks + D, fa[(ks + D) % (D + 1)], fb[(ks + D) % (D + 1)]);
      gx = mma16_split(fa[ks % (D + 1)], fb[ks % (D + 1)], gx);
#if !ONEPASS_PB_FREE
      OSCHED_FENCE();
#endif
    }
    // sum_p g_s over this wave's quarter of the prototypes (k-steps ct KSQ ..): the g_s
    // fragments again, times a ones A operand
    const int qoff = ct * KSQ * 32 * 32;
    const unsigned one2 = 0x3F803F80u + static_cast<unsigned>(lz - lane);  // bf16 (1, 1), built per tile, not held
    const bf16x8 ones = __builtin_bit_cast(bf16x8, u32x4{one2, one2, one2, one2});
#pragma unroll
    for (int kk = 0; kk < KSQ; ++kk) {
      bf16x8 b[kOT];
#pragma unroll
      for (int t2 = 0; t2 < kOT; ++t2)
        b[t2] = tr_pair(pb0 + qoff + t2 * Pp * 32 + kk * 32 * 32, pb1 + qoff + t2 * Pp * 32 + kk * 32 * 32);
      sg = mfma16(ones, b[1], sg);
      sg = mfma16(ones, b[0], sg);
    }
    if (lane < 16) SIG[((slot * 2 + nh) * 4 + ct) * 16 + m] = sg[0];
  };
  auto gx_epilogue = [&](int t, int slot) __attribute__((always_inline)) {
    const int lz = opaque_lane();
    const int m = lz & 15, g = lz >> 4;
    const float* sp = SIG + (slot * 2 + nh) * 64 + m;
    const float sn2 = ((sp[0] + sp[16]) + sp[32]) + sp[48];  // fixed order over the channel tiles
    const unsigned o = out_off(t, m, g);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v;
      if constexpr (XSIG) {  // through the sigmoid: g_pre = g_x s (1 - s)
        const float s = sigmoid_f(xe[r]);
        v = (gx[r] + sn2 * (2.f * s)) * (s * (1.f - s));
      } else {
        v = gx[r] + sn2 * (2.f * xe[r]);  // conv(x^2, ones) backward: sum_p g_s * 2x
      }
      BufIO<TX>::store(rgx, accumulate ? olde[r] + v : v, o, static_cast<unsigned>(r * HW) * sz);
    }
  };

  // ---- main loop. Per tile: phase A(i) | barrier | raw loads of tile i+1, phase B(i), the
  // sum_p g_s partial, staging of tile i+1 | barrier | g_x epilogue(i). The raw loads and the
  // epilogue's x live only across phase B, where phase A's working registers are dead.
#if ONEPASS_PRIO
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);  // static priority for the second-dispatched half
#endif
  OSTAMP(0);
  load_raw(tile_of(0));
  convert(tile_of(0));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the (-2P) image DMA
  __syncthreads();
  OSTAMP(1);
  for (int i = 0; i < iters; ++i) {
    const int t = tile_of(i);
    if (i == 2) OSTAMP(2);
    const int lzA = opaque_lane();
#if ONEPASS_PIPE
    Front fr[2];
    owner_front(0, lzA, fr[0]);
#pragma unroll
    for (int jt = 0; jt < NPT; ++jt) {
      if (jt + 1 < NPT) owner_front(jt + 1, lzA, fr[(jt + 1) & 1]);
      owner_back(jt, lzA, fr[jt & 1]);
      if (i == 2) OSTAMP(3 + jt);
    }
    OSCHED_FENCE();
#else
#pragma unroll
    for (int jt = 0; jt < NPT; ++jt) {
      Front fr;
      owner_front(jt, lzA, fr);
      OSCHED_FENCE();
      owner_back(jt, lzA, fr);
      OSCHED_FENCE();
      if (i == 2) OSTAMP(3 + jt);
    }
#endif
    __syncthreads();  // g_s(i) complete; every wave's reads of the x / g_logits images done
    if (i == 2) OSTAMP(6);
    if (i + 1 < iters) load_raw(tile_of(i + 1));
    phase_b(t, i & 1);
    OSCHED_FENCE();
    if (i == 2) OSTAMP(7);
    if (i + 1 < iters) convert(tile_of(i + 1));
    if (i == 2) OSTAMP(8);
    __syncthreads();  // g_s(i) reads done; images(i+1) and every sum_p g_s partial of tile i written
    if (i == 2) OSTAMP(9);
    gx_epilogue(t, i & 1);
    OSCHED_FENCE();
    if (i == 2) OSTAMP(10);
  }
  OSTAMP(13);

  // ---- slab: this workgroup's g_P (x -2: the x image holds +x), g_W, sum_n g_s; stride Ps = P
  // rounded up to 32 (the reduce kernel's layout), rows past it skipped --------------------------
  const int Ps = (P + 31) & ~31;
  const int E = Ps * kC + 32 * Ps + Ps;
  float* my_slab = slab + static_cast<size_t>(blockIdx.x) * E;
#pragma unroll
  for (int jt = 0; jt < NPT; ++jt) {
    const int p0 = (wave * NPT + jt) * 16;
    if (p0 >= Ps) continue;
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4)
#pragma unroll
      for (int r = 0; r < 4; ++r) my_slab[static_cast<size_t>(p0 + 4 * g + r) * kC + 16 * c4 + m] = -2.f * gp[jt][c4][r];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) my_slab[static_cast<size_t>(Ps) * kC + (16 * kt + 4 * g + r) * Ps + p0 + m] = gw[jt][kt][r];
    float s = gsum[jt];
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    if (g == 0) my_slab[static_cast<size_t>(Ps) * kC + 32 * Ps + p0 + m] = s;
  }
}

// ---- prep: the operand block -------------------------------------------------------------------
__device__ float one_norm2(const float* __restrict__ protos, int p, bool valid) {
#pragma clang fp contract(off)
  const float* row = protos + static_cast<size_t>(valid ? p : 0) * kC;
  float v[kC];
#pragma unroll
  for (int c = 0; c < kC; ++c) v[c] = row[c];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < kC; ++c) s += v[c] * v[c];
  return valid ? s : 0.f;
}

// blockIdx.y: 0 = the (-2P) image (one thread per row chunk, both terms), 1 = wt (one thread per
// fragment lane), 2 = p2.
__global__ __launch_bounds__(256) void l2_prep_onepass_kernel(const float* __restrict__ protos, int P, int Pp,
                                                              const float* __restrict__ w_last, int K, int ldw,
                                                              float wt_scale, unsigned char* __restrict__ block) {
  const OneOffsets o = one_offsets(Pp);
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  switch (blockIdx.y) {
    case 0:
      onepass::fill_pi(protos, P, Pp, block, tid);
      break;
    case 1:
      onepass::fill_wt(w_last, K, ldw, P, Pp, wt_scale, block, tid);
      break;
    default: {
      float* p2 = reinterpret_cast<float*>(block + o.p2);
      for (int p = tid; p < (o.total - o.p2) / 4; p += gridDim.x * blockDim.x) p2[p] = one_norm2(protos, p, p < P);
    }
  }
}

template <typename TX, int ACT, int GD, bool XSIG, int NPT>
int onepass_t(const Geometry& g, const void* x, const unsigned char* img, float eps, const float* g_logits,
              const float* g_dist, void* g_x, int accumulate, float* ws, int grid, hipStream_t stream) {
  constexpr int Pp = kOW * NPT * 16;
  constexpr size_t lds = static_cast<size_t>(one_lds(Pp).total);
  static_assert(lds <= kMaxLds, "one-pass backward LDS");
  if (int st = ensure_lds<l2_bwd_onepass_bf16_kernel<TX, ACT, GD, XSIG, NPT>, lds>()) return st;
  const unsigned long long npix = static_cast<unsigned long long>(g.npix);
  const unsigned xb = static_cast<unsigned>(npix * kC * sizeof(TX));
  const unsigned glb = g_logits ? static_cast<unsigned>(npix * g.K * 4) : 0u;
  const unsigned gdb = GD == 2 ? static_cast<unsigned>(npix * g.cgd.mpc * 4)
                               : g_dist ? static_cast<unsigned>(npix * g.ldd * 4) : 0u;
  KernelTimer timer("l2_bwd_onepass_bf16_kernel", stream);
  hipLaunchKernelGGL((l2_bwd_onepass_bf16_kernel<TX, ACT, GD, XSIG, NPT>), dim3(grid), dim3(kOThreads), lds, stream,
                     static_cast<const TX*>(x), xb, g.HW, g.npix, img, g.P, g.K, eps, g_logits, glb, g_dist, gdb,
                     g.ldd, g.p0, g.cgd, static_cast<TX*>(g_x), accumulate, ws);
  return check_launch("l2_bwd_onepass_bf16_kernel");
}

}  // namespace

int bf16_onepass_npt(int P) { return P <= 128 ? 1 : P <= 256 ? 2 : 3; }
int bf16_onepass_pp(int P) { return kOW * bf16_onepass_npt(P) * 16; }

bool bf16_bwd_onepass_fits(const Geometry& g, int terms) {
  return terms == kOT && g.C == kC && g.P > 0 && g.P <= kOW * 3 * 16 && bf16_sizes_ok(g);
}

int bf16_bwd_onepass_grid(const Geometry& g) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  // as many workgroups as the rounds need, no more: at small batches every slab the reduce reads
  // belongs to a workgroup that did work (e.g. 265 tiles: 133 workgroups x 2, not 256 + 9)
  const int rounds = static_cast<int>(ceil_div(g.ntiles, cus));
  return static_cast<int>(ceil_div(g.ntiles, rounds > 0 ? rounds : 1));
}

size_t bf16_onepass_image_bytes(const Geometry& g) {
  return static_cast<size_t>(one_offsets(kOW * bf16_onepass_npt(g.P) * 16).total);
}

size_t bf16_bwd_onepass_slab_elems(const Geometry& g) {
  const size_t Ps = static_cast<size_t>(ceil_div(g.P, 32) * 32);
  return static_cast<size_t>(bf16_bwd_onepass_grid(g)) * (Ps * kC + 32 * Ps + Ps);
}

int launch_prep_onepass(const Geometry& g, const float* protos, const float* w_last, int act_kind, float eps,
                        void* img, hipStream_t stream) {
  const int Pp = kOW * bf16_onepass_npt(g.P) * 16;
  const dim3 grid(static_cast<unsigned>(ceil_div(Pp * 8, 256)), 3);  // the image's Pp x 8 chunks: the largest region
  hipLaunchKernelGGL(l2_prep_onepass_kernel, grid, dim3(256), 0, stream, protos, g.P, Pp, w_last, g.K, g.ldw,
                     act_grad_unit(act_kind, eps), static_cast<unsigned char*>(img));
  return check_launch("l2_prep_onepass_kernel");
}

int launch_bwd_onepass_bf16(const Geometry& g, bool x_bf16, const void* x, const void* img, float eps, int act_kind,
                            const float* g_logits, const float* g_dist, void* g_x, float* ws, hipStream_t stream,
                            int accumulate) {
  const unsigned char* blk = static_cast<const unsigned char*>(img);
  const int grid = bf16_bwd_onepass_grid(g);
  const int npt = bf16_onepass_npt(g.P);
  auto go = [&](auto tx, auto aa, auto gd) __attribute__((always_inline)) {
    using TX = std::remove_pointer_t<decltype(tx)>;
    constexpr int kA = decltype(aa)::value;
    constexpr int kG = decltype(gd)::value;
    auto by_npt = [&](auto xs) __attribute__((always_inline)) {
      constexpr bool kX = decltype(xs)::value;
      if (npt == 3) return onepass_t<TX, kA, kG, kX, 3>(g, x, blk, eps, g_logits, g_dist, g_x, accumulate, ws, grid, stream);
      if (npt == 2) return onepass_t<TX, kA, kG, kX, 2>(g, x, blk, eps, g_logits, g_dist, g_x, accumulate, ws, grid, stream);
      return onepass_t<TX, kA, kG, kX, 1>(g, x, blk, eps, g_logits, g_dist, g_x, accumulate, ws, grid, stream);
    };
    return g.xsig ? by_npt(std::true_type()) : by_npt(std::false_type());
  };
  using A0 = std::integral_constant<int, 0>;
  using A1 = std::integral_constant<int, 1>;
  using G0 = std::integral_constant<int, 0>;
  using G1 = std::integral_constant<int, 1>;
  using G2 = std::integral_constant<int, 2>;
  float* f = nullptr;
  uint16_t* b = nullptr;
  if (g.cgd.val) {  // the compact KLD gradient: f32 x only (bf16_bwd_compact_ok)
    if (x_bf16 || g_dist) return fail(PROTOSEG_ERR_UNSUPPORTED, "compact g_dist: f32 x and no dense g_dist");
    return act_kind == 0 ? go(f, A0(), G2()) : go(f, A1(), G2());
  }
  if (act_kind == 0)
    return x_bf16 ? (g_dist ? go(b, A0(), G1()) : go(b, A0(), G0())) : (g_dist ? go(f, A0(), G1()) : go(f, A0(), G0()));
  return x_bf16 ? (g_dist ? go(b, A1(), G1()) : go(b, A1(), G0())) : (g_dist ? go(f, A1(), G1()) : go(f, A1(), G0()));
}

}  // namespace protoseg

#ifdef PROTOSEG_STAMPS
// Debug builds only: copy (and clear) the one-pass kernel's per-wave phase stamps.
extern "C" int protoseg_debug_stamps_onepass(void* dst, size_t bytes) {
  using protoseg::g_stamps_onepass;
  const size_t n = bytes < sizeof(g_stamps_onepass) ? bytes : sizeof(g_stamps_onepass);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  if (dst && hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_stamps_onepass), n, 0, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_stamps_onepass)) != hipSuccess) return 3;
  return hipMemset(p, 0, sizeof(g_stamps_onepass)) == hipSuccess ? 0 : 3;
}
#endif
