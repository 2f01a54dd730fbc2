// l2_bwd_owner.hip — the prototype layer's training backward from the forward's saved distances
// (bf16x3, C = 64, up to 384 prototypes per launch). It is the autograd of reference
// model.py:203-221 (_l2_convolution), 231-237 (distance_2_similarity) and 259-283
// (forward_from_conv_features) as the reference's autograd runs it: the relu backward and the
// log / division backward read the SAVED distances D = relu(S) (torch saves relu's output), so
// nothing of S = ||x||^2 + ||p||^2 - 2 x.p is recomputed here:
//   act = f(D),  g_act = g_logits . W,  g_s = (g_act f'(D) + g_dist) [D > 0]
//   g_x = 2 x sum_p g_s - 2 g_s . P          g_P = 2 p sum_n g_s - 2 g_s^T . X
//   g_W = g_logits^T . act
//
// Workgroup = 8 waves (2 per SIMD), one per CU, over a CONTIGUOUS run of 32-pixel tiles (the
// distance rows and g_x rows that two neighbouring tiles share meet in one XCD's L2). Every wave
// owns 16 NPT prototypes (NPT = 3 at 384) and does every product of its prototypes — there is no
// second phase over all prototypes:
//   * layout B (rows = pixels, columns = prototypes, 16x16x32 MFMA): D arrives in the
//     accumulator layout straight from HBM (loaded one tile ahead), g_act against W^T fragments
//     streamed from L2, the epilogue, then g_P += g_s^T X and g_W += g_logits^T act with the
//     epilogue values as the A / B operands (registers for the launch; one slab per workgroup);
//   * g_s goes to the wave's own LDS image, is read back transposed (ds_read_b64_tr_b16, no
//     barrier: the wave's own rows) as the B operand of g_x^T partial = (-2P)^T g_s over the
//     owned prototypes on 32x32x16 MFMA (one 16-prototype k-step per owned tile), with the
//     (-2P)^T A fragments held in registers for the launch, and sum_p g_s partial from the same
//     fragments against ones;
//   * the eight partials (64 channels x 32 pixels + 32 sums) meet in LDS; after one barrier every
//     thread sums its four outputs over the waves in a fixed order (deterministic), adds
//     2 x sum_p g_s with x from an f32 copy staged with the tile, and stores g_x (NCHW).
// LDS images: x and g_logits split images (as l2_bwd_onepass.hip), the f32 x copy (double
// buffered), and per wave one region that holds its g_s image, then its g_x partial.
#include <type_traits>

#include "bf16_split.h"
#include "l2_bf16_common.h"
#include "l2_launch.h"
#include "protoseg_host.h"

namespace protoseg {

namespace {

using namespace bf16l;

constexpr int kQW = 8;  // waves per workgroup
constexpr int kQT = 2;  // split terms (bf16x3)
constexpr int kQThreads = kQW * 64;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// ---- operand block (l2_prep_owner_kernel). g = l >> 4, m = l & 15, h = l >> 5.
//   wt [ptile Pp/16][term]: g_act B fragments (16x16x32): lane (p = 16 ptile + m), classes
//                           8 g + jj (grad_unit * W), 1 KiB each
//   pa [ptile][ci 2][term]: g_x A fragments (32x32x16): lane (c = 32 ci + (l & 31)), prototypes
//                           16 ptile + 8 h + jj of (-2P)^T, 1 KiB each
struct QOffsets {
  int wt, pa, total;
};
__host__ __device__ constexpr QOffsets q_offsets(int Pp) {
  QOffsets o{};
  o.wt = 0;
  o.pa = o.wt + (Pp / 16) * kQT * 1024;
  o.total = o.pa + (Pp / 16) * 2 * kQT * 1024;
  return o;
}

// LDS (bytes). The per-wave region holds the wave's g_s image ([term][16 NPT][32] bf16), then
// its g_x partial ([32 n][68] f32) and its 32 pixel sums.
constexpr int kPartRow = 68;                    // floats per partial / x-copy row (64 + 4 pad)
constexpr int kPartBytes = 32 * kPartRow * 4 + 32 * 4;
constexpr int kMaxWtBytes = (kQW * 3 * 16 / 16) * kQT * 1024;  // Pp = 384
struct QLds {
  int xa, ga, xs, wave, wt, ro, cl, total;
};
__host__ __device__ constexpr QLds q_lds() {
  QLds o{};
  o.xa = 0;                              // [term][32 n][80] bf16 (onepass x image)
  o.ga = o.xa + kQT * 32 * 160;          // [term][32 n][32 k] bf16
  o.xs = o.ga + kQT * 32 * 64;           // [2][32 n][68] f32: x (sigmoid(x) with XSIG) per tile
  o.wave = o.xs + 2 * 32 * kPartRow * 4;  // [8][kPartBytes]
  o.wt = o.wave + kQW * kPartBytes;      // the operand block's wt region (W^T fragments), copied once
  o.ro = o.wt + kMaxWtBytes;             // [32] u32 g_dist row offset per pixel
  o.cl = o.ro + 32 * 4;                  // [32] int KLD class per pixel
  o.total = o.cl + 32 * 4;
  return o;
}

constexpr int kXaRow = 80;
constexpr int kXaPlane = 32 * kXaRow;
__device__ __forceinline__ int xa_off(int n, int chunk) { return n * kXaRow + (chunk << 3); }
__device__ __forceinline__ int ga_off(int n, int chunk) { return n * 32 + (((chunk ^ ((n >> 1) & 2)) & 3) << 3); }
// g_s image of one wave: row p (its local prototype), 32 pixels in 8-B slots (4 pixels), slot s
// at s ^ ((p >> 1) & 7): the owners' ds_write_b64 (16 rows x one slot per 16-lane group) and the
// 32x32x16 B-operand transposed reads (4 rows x 8 slots per 32-lane half) are both conflict-free.
__device__ __forceinline__ int gw_off(int p, int slot) { return p * 32 + ((slot ^ ((p >> 1) & 7)) << 2); }

__device__ __forceinline__ bf16x8 tr_pair(const bf16* lo, const bf16* hi) {
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(lo));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(hi));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mma16_split(const bf16x8 (&a)[kQT], const bf16x8 (&b)[kQT], f32x4 c) {
  c = mfma16(a[0], b[1], c);
  c = mfma16(a[1], b[0], c);
  return mfma16(a[0], b[0], c);
}
__device__ __forceinline__ void store_half4(bf16* dst, const bf16x8& f, int half) {
  const s16x8 v = __builtin_bit_cast(s16x8, f);
  *reinterpret_cast<s16x4*>(dst) = half ? __builtin_shufflevector(v, v, 4, 5, 6, 7) : __builtin_shufflevector(v, v, 0, 1, 2, 3);
}
// Timing-only ablations (wrong results; measured variants built by tools/build_var.sh):
//   OWNER_ABL_NO_D: no distance loads; OWNER_ABL_NO_PA: no (-2P)^T fragment loads;
//   OWNER_ABL_NO_GX: no g_x partial / reduce; OWNER_TILES_RR: round-robin tiles instead of runs.
#ifndef OWNER_ABL_NO_D
#define OWNER_ABL_NO_D 0
#endif
#ifndef OWNER_ABL_NO_PA
#define OWNER_ABL_NO_PA 0
#endif
#ifndef OWNER_ABL_NO_GX
#define OWNER_ABL_NO_GX 0
#endif
#ifndef OWNER_TILES_RR
#define OWNER_TILES_RR 0
#endif
#ifndef OWNER_PIPE
#define OWNER_PIPE 0  // 1: owned tile jt+1's g_act products issued before tile jt's epilogue
#endif
__device__ __forceinline__ void mem_fence_compiler() { asm volatile("" ::: "memory"); }

// GD: 0 no distance gradient, 1 a dense g_dist, 2 the KLD loss's compact one (CompactGd).
template <typename TX, int ACT, int GD, bool XSIG, int NPT>
__global__ __launch_bounds__(kQThreads, 1) void l2_bwd_owner_bf16_kernel(
    const TX* __restrict__ x, unsigned x_bytes, int HW, int npix, const float* __restrict__ dist, unsigned d_bytes,
    const unsigned char* __restrict__ img, int P, int K, float eps, const float* __restrict__ g_logits,
    unsigned gl_bytes, const float* __restrict__ g_dist, unsigned gd_bytes, int ld, int p0, CompactGd cg,
    TX* __restrict__ g_x, int accumulate, float* __restrict__ slab) {
  constexpr int Pp = kQW * NPT * 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  constexpr QLds L = q_lds();
  constexpr QOffsets io = q_offsets(Pp);
  bf16* XA = reinterpret_cast<bf16*>(smem_raw + L.xa);
  bf16* GA = reinterpret_cast<bf16*>(smem_raw + L.ga);
  float* XS = reinterpret_cast<float*>(smem_raw + L.xs);
  unsigned* RO = reinterpret_cast<unsigned*>(smem_raw + L.ro);
  int* CL = reinterpret_cast<int*>(smem_raw + L.cl);

  const int lane = threadIdx.x & 63, g = lane >> 4, m = lane & 15, wave = wave_id();
  unsigned char* const WREG = smem_raw + L.wave + wave * kPartBytes;  // this wave's region
  bf16* GW = reinterpret_cast<bf16*>(WREG);                            // [term][16 NPT][32]
  float* PART = reinterpret_cast<float*>(WREG);                        // [32][68] after the g_x products
  float* PSUM = PART + 32 * kPartRow;                                  // [32]
  const bf16* WT = reinterpret_cast<const bf16*>(smem_raw + L.wt);       // wt fragments, 1 KiB each

  const int ntiles = (npix + 31) / 32;
  // contiguous runs: workgroup b takes tiles [first, first + iters)
  const int G = static_cast<int>(gridDim.x), bq = ntiles / G, br = ntiles - bq * G;
  const int bid = static_cast<int>(blockIdx.x);
#if OWNER_TILES_RR
  const int first = bid;  // tile first + i * G (round robin)
  const int iters = (ntiles - bid + G - 1) / G;
  auto tile_at = [&](int i) __attribute__((always_inline)) { return first + i * G; };
#else
  const int first = bid * bq + (bid < br ? bid : br);
  const int iters = bq + (bid < br ? 1 : 0);
  auto tile_at = [&](int i) __attribute__((always_inline)) { return first + i; };
#endif
  const unsigned sz = sizeof(TX);
  const unsigned chs = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(HW) * sz);
  const rsrc_t rx = make_rsrc(x, x_bytes), rg = make_rsrc(g_logits, gl_bytes), rd = make_rsrc(dist, d_bytes);
  const rsrc_t rgd = make_rsrc(GD == 2 ? cg.val : g_dist, gd_bytes), rgx = make_rsrc(g_x, g_x ? x_bytes : 0u);
  const rsrc_t rimg = make_rsrc(img, static_cast<unsigned>(io.total));

  auto opaque_lane = [&]() __attribute__((always_inline)) {
    int z = 0;
    asm volatile("" : "+v"(z));
    return lane + z;
  };

  // ---- the owned (-2P)^T A fragments of g_x, streamed from the (L2-resident) operand block per
  // tile and owned tile (12 KiB per wave: held for the launch they would cost 48 VGPRs)
  auto load_pa = [&](int jt, bf16x8 (&dst)[2][kQT]) __attribute__((always_inline)) {
    if (OWNER_ABL_NO_PA) {
#pragma unroll
      for (int ci = 0; ci < 2; ++ci)
#pragma unroll
        for (int t = 0; t < kQT; ++t) dst[ci][t] = __builtin_bit_cast(bf16x8, u32x4{0x3F803F80u + jt, 0u, 0u, 0u});
      return;
    }
#pragma unroll
    for (int ci = 0; ci < 2; ++ci)
#pragma unroll
      for (int t = 0; t < kQT; ++t)
        dst[ci][t] = __builtin_bit_cast(
            bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                        rimg, static_cast<unsigned>(opaque_lane() * 16),
                        static_cast<unsigned>(io.pa + (((wave * NPT + jt) * 2 + ci) * kQT + t) * 1024), 0));
  };
  int pcls[NPT], pslot[NPT];  // GD = 2: the owned prototypes' class and compact column (bytes)
  if constexpr (GD == 2) {
#pragma unroll
    for (int jt = 0; jt < NPT; ++jt) {
      const int pp = (wave * NPT + jt) * 16 + m;
      const int code = pp < P ? cg.slot[p0 + pp] : 0;
      pcls[jt] = pp < P ? code >> 8 : -2;  // never a pixel class (those are >= -1)
      pslot[jt] = (code & 255) * 4;
    }
  }

  // ---- distances, layout B: lane (p = 16 ptile + m, g) holds D[n][p] for n = 16 nt + 4 g + r ----
  // Fast tiles (inside one image, below npix): two 16-B loads per owned tile, the row part in the
  // voffset (loop-invariant), the tile part in the soffset. Other tiles: one load per element.
  float dv[NPT][8];
  const unsigned drow = static_cast<unsigned>((m * HW + 4 * g) * 4);  // lane part
  auto load_d = [&](int t, int jt) __attribute__((always_inline)) {
    if (OWNER_ABL_NO_D) {
#pragma unroll
      for (int e = 0; e < 8; ++e) dv[jt][e] = static_cast<float>(t & 7) + 0.5f * e;
      return;
    }
    const int gp0 = t * 32;
    const int b0 = div_pix(gp0, HW);
    const int pl = (wave * NPT + jt) * 16;  // the owned tile's first prototype (chunk-local)
    const bool fast = gp0 + 31 < npix && gp0 + 31 - b0 * HW < HW;
    const bool row_ok = pl + m < P;
    if (fast) {
      const unsigned so =
          __builtin_amdgcn_readfirstlane(static_cast<unsigned>(((b0 * ld + p0 + pl) * HW + (gp0 - b0 * HW)) * 4));
      const unsigned vo = row_ok ? drow : kOOB;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rd, vo + 64u * nt, so, 0));
#pragma unroll
        for (int r = 0; r < 4; ++r) dv[jt][4 * nt + r] = v[r];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int gp = gp0 + 16 * (e >> 2) + 4 * g + (e & 3);
        unsigned off = kOOB;
        if (gp < npix && row_ok) {
          const int b = div_pix(gp, HW);
          off = static_cast<unsigned>(((b * ld + p0 + pl + m) * HW + (gp - b * HW)) * 4);
        }
        dv[jt][e] = BufIO<float>::load(rd, off, 0u);
      }
    }
  };

  // ---- staging (as l2_bwd_onepass.hip): wave w stages pixels 4w .. 4w+3. Lanes 0..31: x of
  // pixel 4w + l/8, chunk ch = l & 7 = channels chan_of(ch >> 1, ch & 1, 0..7); lanes 32..47:
  // 8 classes of pixel 4w + (l - 32) / 4. Raw values go to registers first (issued a phase ahead).
  float raw[8];
  int rcl = -1;
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
  auto convert = [&](int t, int buf) __attribute__((always_inline)) {
    float v[8];
    bf16x8 f[kQT];
    const int lz = opaque_lane();
    const int sn = 4 * wave + ((lz & 31) >> 3), sch = lz & 7;
    const int gn = 4 * wave + ((lz - 32) >> 2), gkc = lz & 3;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = raw[e];
    if (lane < 32) {
      if constexpr (XSIG) {
        const bool ok = t * 32 + sn < npix;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = ok ? sigmoid_f(v[e]) : 0.f;
      }
      split8<kQT>(v, f);
      const int q = sch >> 1, hh = sch & 1;
      float* xs = XS + buf * 32 * kPartRow + sn * kPartRow;
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int c = chan_of(q, hh, 4 * half);  // e = 4 half .. +3 are channels c .. c+3
#pragma unroll
        for (int t2 = 0; t2 < kQT; ++t2) store_half4(XA + t2 * kXaPlane + xa_off(sn, c >> 3) + (c & 7), f[t2], half);
        *reinterpret_cast<float4*>(xs + c) = make_float4(v[4 * half], v[4 * half + 1], v[4 * half + 2], v[4 * half + 3]);
      }
    } else if (lane < 48) {
      split8<kQT>(v, f);
#pragma unroll
      for (int t2 = 0; t2 < kQT; ++t2) *reinterpret_cast<bf16x8*>(GA + t2 * 32 * 32 + ga_off(gn, gkc)) = f[t2];
      if constexpr (GD == 1) {
        if (gkc == 0) {
          const int gg = t * 32 + gn;
          const bool ok = gg < npix;
          const int b = ok ? div_pix(gg, HW) : 0;
          RO[gn] = ok ? static_cast<unsigned>(((b * ld + p0) * HW + (gg - b * HW)) * 4) : kOOB;
        }
      }
    } else if (GD == 2 && lane < 52) {
      const int n = 4 * wave + (lane - 48);
      RO[n] = rcl >= 0 ? static_cast<unsigned>((t * 32 + n) * cg.mpc * 4) : kOOB;
      CL[n] = rcl;
    }
  };

  // ---- owner products of tile t, owned tile jt (front: g_act + g_dist loads; back: epilogue,
  // g_s image, g_P / g_W) -------------------------------------------------------------------
  f32x4 gpa[NPT][4], gwa[NPT][2];
  float gsum[NPT];
#pragma unroll
  for (int jt = 0; jt < NPT; ++jt) {
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) gpa[jt][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
    gwa[jt][0] = gwa[jt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    gsum[jt] = 0.f;
  }
  struct Front {
    f32x4 gacc[2];
    float gdv[8];
  };
  auto owner_front = [&](int jt, int lz, Front& fr) __attribute__((always_inline)) {
    const int m = lz & 15, g = lz >> 4;
    const int p = (wave * NPT + jt) * 16 + m;
    int zj = 0;
    asm volatile("" : "+v"(zj));
    const bf16* GAj = GA + zj;
    bf16x8 wtj[kQT];  // from LDS: no vector-memory wait here (the distance prefetch is in flight)
#pragma unroll
    for (int t = 0; t < kQT; ++t)
      wtj[t] = *reinterpret_cast<const bf16x8*>(WT + ((wave * NPT + jt) * kQT + t) * 512 + lz * 8);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      bf16x8 ga[kQT];
#pragma unroll
      for (int t = 0; t < kQT; ++t) ga[t] = *reinterpret_cast<const bf16x8*>(GAj + t * 32 * 32 + ga_off(16 * nt + m, g));
      fr.gacc[nt] = mma16_split(ga, wtj, f32x4{0.f, 0.f, 0.f, 0.f});
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
          fr.gdv[4 * nt + r] = BufIO<float>::load(rgd, cv[r] == pcls[jt] ? rv[r] + pslot[jt] : kOOB, 0);
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
          fr.gdv[4 * nt + r] = BufIO<float>::load(rgd, (rv[r] != kOOB && pvalid) ? rv[r] + pcol : kOOB, 0);
      }
    }
  };
  auto owner_back = [&](int jt, int lz, Front& fr) __attribute__((always_inline)) {
    const int m = lz & 15, g = lz >> 4, qq = (lz >> 2) & 3, pp = lz & 3;
    const int pl = 16 * jt + m;  // the lane's prototype in this wave's g_s image
    int zj = 0;
    asm volatile("" : "+v"(zj));
    const bf16* XAj = XA + zj;
    const bf16* GAj = GA + zj;
    // epilogue: element e = 4 nt + r is pixel 16 nt + 4 g + r (the A / B k-slot order)
    float gs[8], av[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = dv[jt][e];  // relu's output (>= 0)
      float a;
      float gd = fr.gacc[e >> 2][e & 3] * act_grad_and_base<ACT>(d, eps, a);  // grad_unit is in W^T
      if constexpr (GD) gd += fr.gdv[e];
      gs[e] = d > 0.f ? gd : 0.f;  // relu backward (threshold on the saved output)
      gsum[jt] += gs[e];
      av[e] = a;
    }
    bf16x8 gsf[kQT], actf[kQT];
    split8<kQT>(gs, gsf);
    split8<kQT>(av, actf);
#pragma unroll
    for (int t = 0; t < kQT; ++t) {
      store_half4(GW + t * (16 * NPT * 32) + gw_off(pl, g), gsf[t], 0);
      store_half4(GW + t * (16 * NPT * 32) + gw_off(pl, 4 + g), gsf[t], 1);
    }
    // g_P[p][c] += g_s^T X: B = x[n][c] with the k-slot pixels (transposed reads of the x image)
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      bf16x8 xb[kQT];
      const int slot = 4 * ct + pp, chunk = slot >> 1, sub = (slot & 1) * 4;
#pragma unroll
      for (int t = 0; t < kQT; ++t)
        xb[t] = tr_pair(XAj + t * kXaPlane + xa_off(4 * g + qq, chunk) + sub, XAj + t * kXaPlane + xa_off(16 + 4 * g + qq, chunk) + sub);
      gpa[jt][ct] = mma16_split(gsf, xb, gpa[jt][ct]);
    }
    // g_W[k][p] += g_logits^T act
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      bf16x8 gl[kQT];
      const int slot = 4 * kt + pp, chunk = slot >> 1, sub = (slot & 1) * 4;
#pragma unroll
      for (int t = 0; t < kQT; ++t)
        gl[t] = tr_pair(GAj + t * 32 * 32 + ga_off(4 * g + qq, chunk) + sub, GAj + t * 32 * 32 + ga_off(16 + 4 * g + qq, chunk) + sub);
      gwa[jt][kt] = mma16_split(gl, actf, gwa[jt][kt]);
    }
  };

  // ---- g_x^T partial over the owned prototypes (32x32x16): out[c][n], c = 32 ci + row ---------
  auto gx_partial = [&](bf16x8 (&pa0)[2][kQT], auto&& after_loads) __attribute__((always_inline)) {
    const int lz = opaque_lane();
    const int h = lz >> 5, G = (lz >> 4) & 1, q = (lz >> 2) & 3, pq = lz & 3;
    f32x16 acc[2] = {zero16(), zero16()};
    f32x16 sacc = zero16();
    const unsigned one2 = 0x3F803F80u + static_cast<unsigned>(lz - lane);  // bf16 (1, 1)
    const bf16x8 ones = __builtin_bit_cast(bf16x8, u32x4{one2, one2, one2, one2});
    bf16x8 pa[2][2][kQT];
#pragma unroll
    for (int ci = 0; ci < 2; ++ci)
#pragma unroll
      for (int t = 0; t < kQT; ++t) pa[0][ci][t] = pa0[ci][t];
#pragma unroll
    for (int jt = 0; jt < NPT; ++jt) {
      if (jt + 1 < NPT) load_pa(jt + 1, pa[(jt + 1) & 1]);
      // B[k = 8h + jj][n = l & 31] = g_s[prototype 16 jt + 8h + jj][n]: rows 8h + q (+4), slot 4G + pq
      bf16x8 bs[kQT];
      const int row = 16 * jt + 8 * h + q, slot = 4 * G + pq;
#pragma unroll
      for (int t = 0; t < kQT; ++t)
        bs[t] = tr_pair(GW + t * (16 * NPT * 32) + gw_off(row, slot), GW + t * (16 * NPT * 32) + gw_off(row + 4, slot));
#pragma unroll
      for (int ci = 0; ci < 2; ++ci) {
        acc[ci] = mfma_bf16(pa[jt & 1][ci][0], bs[1], acc[ci]);
        acc[ci] = mfma_bf16(pa[jt & 1][ci][1], bs[0], acc[ci]);
        acc[ci] = mfma_bf16(pa[jt & 1][ci][0], bs[0], acc[ci]);
      }
      sacc = mfma_bf16(ones, bs[1], sacc);
      sacc = mfma_bf16(ones, bs[0], sacc);
    }
    // the next tile's distances are issued behind the last fragment load (vmcnt counts in issue
    // order: a wait for the fragments never waits for them), with the fragment registers dead
    __builtin_amdgcn_sched_barrier(0);
    after_loads();
    __builtin_amdgcn_sched_barrier(0);
    // every read of the g_s image (this wave's) is done before the partial overwrites it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int n = lz & 31;
#pragma unroll
    for (int ci = 0; ci < 2; ++ci)
#pragma unroll
      for (int j = 0; j < 4; ++j)  // registers 4j .. 4j+3: channels 32 ci + 8 j + 4 h + 0..3
        *reinterpret_cast<float4*>(PART + n * kPartRow + 32 * ci + 8 * j + 4 * h) =
            make_float4(acc[ci][4 * j], acc[ci][4 * j + 1], acc[ci][4 * j + 2], acc[ci][4 * j + 3]);
    if (lane < 32) PSUM[n] = sacc[0];
  };

  // ---- after the barrier: fixed-order sum of the waves' partials, + 2 x sum_p g_s, NCHW stores.
  // Thread (wave w, lane l): pixel n = l & 31, channels c0 = 8 w + 4 (l >> 5) .. +3.
  auto gx_reduce = [&](int t, int buf) __attribute__((always_inline)) {
    const int lz = opaque_lane();
    const int n = lz & 31, c0 = 8 * wave + 4 * (lz >> 5);
    const float* base = reinterpret_cast<const float*>(smem_raw + L.wave);
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    float ps = 0.f;
#pragma unroll
    for (int w = 0; w < kQW; ++w) {
      const float* pw = base + w * (kPartBytes / 4);
      const float4 v = *reinterpret_cast<const float4*>(pw + n * kPartRow + c0);
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
      ps += pw[32 * kPartRow + n];
    }
    const float4 xv = *reinterpret_cast<const float4*>(XS + buf * 32 * kPartRow + n * kPartRow + c0);
    const float sv[4] = {s.x, s.y, s.z, s.w}, xe[4] = {xv.x, xv.y, xv.z, xv.w};
    const int gp = t * 32 + n;
    if (gp < npix) {
      const int b = div_pix(gp, HW);
      const unsigned o = static_cast<unsigned>((b * kC + c0) * HW + (gp - b * HW)) * sz;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v;
        if constexpr (XSIG) {  // g_pre = g_x s (1 - s), s = sigmoid(pre) (the copy holds s)
          v = (sv[r] + ps * (2.f * xe[r])) * (xe[r] * (1.f - xe[r]));
        } else {
          v = sv[r] + ps * (2.f * xe[r]);  // conv(x^2, ones) backward: sum_p g_s * 2x
        }
        if (accumulate) v += BufIO<TX>::load(rgx, o, static_cast<unsigned>(r * HW) * sz);
        BufIO<TX>::store(rgx, v, o, static_cast<unsigned>(r * HW) * sz);
      }
    }
  };

  // ---- main loop -------------------------------------------------------------------------
  lds_copy(smem_raw + L.wt, img + io.wt, io.pa - io.wt);
  if (iters > 0) {
    load_raw(tile_at(0));
#pragma unroll
    for (int jt = 0; jt < NPT; ++jt) load_d(tile_at(0), jt);
    convert(tile_at(0), 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the wt DMA (and tile 0's distances)
  __syncthreads();
  for (int i = 0; i < iters; ++i) {
    const int t = tile_at(i), tn = tile_at(i + 1);
    const bool more = i + 1 < iters;
    if (more) load_raw(tn);  // x / g_logits of the next tile, converted after the barrier
    const int lzA = opaque_lane();
#if OWNER_PIPE
    Front fr[2];
    owner_front(0, lzA, fr[0]);
#pragma unroll
    for (int jt = 0; jt < NPT; ++jt) {
      if (jt + 1 < NPT) owner_front(jt + 1, lzA, fr[(jt + 1) & 1]);
      owner_back(jt, lzA, fr[jt & 1]);
    }
#else
#pragma unroll
    for (int jt = 0; jt < NPT; ++jt) {
      Front fr;
      owner_front(jt, lzA, fr);
      owner_back(jt, lzA, fr);
    }
#endif
    if (!OWNER_ABL_NO_GX) {
      bf16x8 pa0[2][kQT];
      load_pa(0, pa0);
      mem_fence_compiler();  // the g_s image writes above, the transposed reads below (same wave)
      gx_partial(pa0, [&]() __attribute__((always_inline)) {
        if (more)
#pragma unroll
          for (int jt = 0; jt < NPT; ++jt) load_d(tn, jt);  // dv is consumed: the next tile's go there
      });
    } else if (more) {
#pragma unroll
      for (int jt = 0; jt < NPT; ++jt) load_d(tn, jt);
    }
    __syncthreads();  // every wave's partial written; every read of the x / g_logits images done
    if (!OWNER_ABL_NO_GX) gx_reduce(t, i & 1);
    if (more) convert(tn, (i + 1) & 1);
    __syncthreads();  // images of tile t+1 written; every read of the partials done
  }

  // ---- slab: this workgroup's g_P (x -2: the x image holds +x), g_W, sum_n g_s; stride Ps = P
  // rounded up to 32 (the reduce kernel's layout), rows past it skipped --------------------------
  const int Ps = (P + 31) & ~31;
  const int E = Ps * kC + 32 * Ps + Ps;
  float* my_slab = slab + static_cast<size_t>(blockIdx.x) * E;
#pragma unroll
  for (int jt = 0; jt < NPT; ++jt) {
    const int pb = (wave * NPT + jt) * 16;
    if (pb >= Ps) continue;
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4)
#pragma unroll
      for (int r = 0; r < 4; ++r) my_slab[static_cast<size_t>(pb + 4 * g + r) * kC + 16 * c4 + m] = -2.f * gpa[jt][c4][r];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) my_slab[static_cast<size_t>(Ps) * kC + (16 * kt + 4 * g + r) * Ps + pb + m] = gwa[jt][kt][r];
    float s = gsum[jt];
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    if (g == 0) my_slab[static_cast<size_t>(Ps) * kC + 32 * Ps + pb + m] = s;
  }
}

// ---- prep: the operand block ----------------------------------------------------------------
// blockIdx.y: 0 = wt (one thread per fragment lane), 1 = pa (one thread per fragment lane).
__global__ __launch_bounds__(256) void l2_prep_owner_kernel(const float* __restrict__ protos, int P, int Pp,
                                                            const float* __restrict__ w_last, int K, int ldw,
                                                            float wt_scale, unsigned char* __restrict__ block) {
  const QOffsets o = q_offsets(Pp);
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = tid & 63, frag = tid >> 6;
  float v[8];
  bf16x8 f[kQT];
  if (blockIdx.y == 0) {  // wt[ptile]: lane (p = 16 ptile + m), classes 8 g + jj
    if (frag >= Pp / 16) return;
    const int g = lane >> 4, p = 16 * frag + (lane & 15);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 8 * g + e;
      v[e] = (w_last && p < P && k < K) ? wt_scale * w_last[static_cast<size_t>(k) * ldw + p] : 0.f;
    }
    split8<kQT>(v, f);
#pragma unroll
    for (int t = 0; t < kQT; ++t) *reinterpret_cast<bf16x8*>(block + o.wt + (frag * kQT + t) * 1024 + lane * 16) = f[t];
  } else {  // pa[ptile][ci]: lane (c = 32 ci + (l & 31)), prototypes 16 ptile + 8 h + jj, times -2
    if (frag >= (Pp / 16) * 2) return;
    const int ptile = frag >> 1, ci = frag & 1, h = lane >> 5, c = 32 * ci + (lane & 31);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int p = 16 * ptile + 8 * h + e;
      v[e] = p < P ? -2.f * protos[static_cast<size_t>(p) * kC + c] : 0.f;
    }
    split8<kQT>(v, f);
#pragma unroll
    for (int t = 0; t < kQT; ++t) *reinterpret_cast<bf16x8*>(block + o.pa + (frag * kQT + t) * 1024 + lane * 16) = f[t];
  }
}

template <typename TX, int ACT, int GD, bool XSIG, int NPT>
int owner_t(const Geometry& g, const void* x, const float* dist, const unsigned char* img, float eps,
            const float* g_logits, const float* g_dist, void* g_x, int accumulate, float* ws, int grid,
            hipStream_t stream) {
  constexpr size_t lds = static_cast<size_t>(q_lds().total);
  static_assert(lds <= kMaxLds, "owner backward LDS");
  if (int st = ensure_lds<l2_bwd_owner_bf16_kernel<TX, ACT, GD, XSIG, NPT>, lds>()) return st;
  const unsigned long long npix = static_cast<unsigned long long>(g.npix);
  const unsigned xb = static_cast<unsigned>(npix * kC * sizeof(TX));
  const unsigned db = static_cast<unsigned>(static_cast<unsigned long long>(g.npix) * g.ldd * 4);
  const unsigned glb = g_logits ? static_cast<unsigned>(npix * g.K * 4) : 0u;
  const unsigned gdb = GD == 2 ? static_cast<unsigned>(npix * g.cgd.mpc * 4)
                               : g_dist ? static_cast<unsigned>(npix * g.ldd * 4) : 0u;
  KernelTimer timer("l2_bwd_owner_bf16_kernel", stream);
  hipLaunchKernelGGL((l2_bwd_owner_bf16_kernel<TX, ACT, GD, XSIG, NPT>), dim3(grid), dim3(kQThreads), lds, stream,
                     static_cast<const TX*>(x), xb, g.HW, g.npix, dist, db, img, g.P, g.K, eps, g_logits, glb, g_dist,
                     gdb, g.ldd, g.p0, g.cgd, static_cast<TX*>(g_x), accumulate, ws);
  return check_launch("l2_bwd_owner_bf16_kernel");
}

}  // namespace

int bf16_owner_npt(int P) { return P <= 128 ? 1 : P <= 256 ? 2 : 3; }

bool bf16_bwd_owner_fits(const Geometry& g, int terms) {
  return terms == kQT && g.C == kC && g.P > 0 && g.P <= kQW * 3 * 16 && bf16_sizes_ok(g) &&
         static_cast<unsigned long long>(g.npix) * g.ldd * 4 < (1ULL << 31);
}

int bf16_bwd_owner_grid(const Geometry& g) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int rounds = static_cast<int>(ceil_div(g.ntiles, cus));
  return static_cast<int>(ceil_div(g.ntiles, rounds > 0 ? rounds : 1));
}

size_t bf16_owner_image_bytes(const Geometry& g) {
  return static_cast<size_t>(q_offsets(kQW * bf16_owner_npt(g.P) * 16).total);
}

size_t bf16_bwd_owner_slab_elems(const Geometry& g) {
  const size_t Ps = static_cast<size_t>(ceil_div(g.P, 32) * 32);
  return static_cast<size_t>(bf16_bwd_owner_grid(g)) * (Ps * kC + 32 * Ps + Ps);
}

int launch_prep_owner(const Geometry& g, const float* protos, const float* w_last, int act_kind, float eps, void* img,
                      hipStream_t stream) {
  const int Pp = kQW * bf16_owner_npt(g.P) * 16;
  const dim3 grid(static_cast<unsigned>(ceil_div((Pp / 16) * 2 * 64, 256)), 2);
  hipLaunchKernelGGL(l2_prep_owner_kernel, grid, dim3(256), 0, stream, protos, g.P, Pp, w_last, g.K, g.ldw,
                     act_grad_unit(act_kind, eps), static_cast<unsigned char*>(img));
  return check_launch("l2_prep_owner_kernel");
}

int launch_bwd_owner_bf16(const Geometry& g, bool x_bf16, const void* x, const float* dist, const void* img, float eps,
                          int act_kind, const float* g_logits, const float* g_dist, void* g_x, float* ws,
                          hipStream_t stream, int accumulate) {
  const unsigned char* blk = static_cast<const unsigned char*>(img);
  const int grid = bf16_bwd_owner_grid(g);
  const int npt = bf16_owner_npt(g.P);
  auto go = [&](auto tx, auto aa, auto gd) __attribute__((always_inline)) {
    using TX = std::remove_pointer_t<decltype(tx)>;
    constexpr int kA = decltype(aa)::value;
    constexpr int kG = decltype(gd)::value;
    auto by_npt = [&](auto xs) __attribute__((always_inline)) {
      constexpr bool kX = decltype(xs)::value;
      if (npt == 3)
        return owner_t<TX, kA, kG, kX, 3>(g, x, dist, blk, eps, g_logits, g_dist, g_x, accumulate, ws, grid, stream);
      if (npt == 2)
        return owner_t<TX, kA, kG, kX, 2>(g, x, dist, blk, eps, g_logits, g_dist, g_x, accumulate, ws, grid, stream);
      return owner_t<TX, kA, kG, kX, 1>(g, x, dist, blk, eps, g_logits, g_dist, g_x, accumulate, ws, grid, stream);
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
  if (g.cgd.val) {  // the compact KLD gradient: f32 x only
    if (x_bf16 || g_dist) return fail(PROTOSEG_ERR_UNSUPPORTED, "compact g_dist: f32 x and no dense g_dist");
    return act_kind == 0 ? go(f, A0(), G2()) : go(f, A1(), G2());
  }
  if (act_kind == 0)
    return x_bf16 ? (g_dist ? go(b, A0(), G1()) : go(b, A0(), G0())) : (g_dist ? go(f, A0(), G1()) : go(f, A0(), G0()));
  return x_bf16 ? (g_dist ? go(b, A1(), G1()) : go(b, A1(), G0())) : (g_dist ? go(f, A1(), G1()) : go(f, A1(), G0()));
}

}  // namespace protoseg
