// l2_bwd_wave.hip — the prototype layer's training backward (bf16x3, C = 64, up to 384
// prototypes per launch) with ONE wave per SIMD and every product of a prototype done by the wave
// that owns it. It is the autograd of reference model.py:203-221 (_l2_convolution), 231-237
// (distance_2_similarity) and 259-283 (forward_from_conv_features):
//   S = ||x||^2 + ||p||^2 - 2 X.P^T,  d = relu(S),  act = f(d),  logits = act . W^T
//   g_act = g_logits . W,  g_s = (g_act f'(d) + g_dist) [d > 0]
//   g_x   = 2 x sum_p g_s - 2 g_s . P          g_P = 2 p sum_n g_s - 2 g_s^T . X
//   g_W   = g_logits^T . act
//
// Workgroup = 4 waves, one per SIMD (up to 512 registers each), one workgroup per CU, persistent
// over 32-pixel tiles. Wave w owns NB blocks of 32 prototypes (Pp = 128 NB). Per pixel tile and
// owned block, on v_mfma_f32_32x32x16_bf16 (the 16x16x32 form holds the SIMD's vector issue for
// half of its cycles, this one for a quarter, and the epilogue is VALU-heavy):
//   S [n][p]     = X (A, rows of the x image) . (-2P)^T (B, rows of the (-2P) image), the
//                  accumulator starting at ||x||^2 + ||p||^2, products in the forward's order and
//                  channel order, so d is the forward's distance bit for bit;
//   g_act [n][p] = g_logits (A, rows of the g_logits image) . (grad_unit W) (B, registers);
//   the epilogue (relu mask, f'(d), act, g_s, sum_n g_s) on the accumulators;
//   g_P^T [c][p] += X^T (A, transposed reads of the x image) . g_s (B: the accumulator);
//   g_W [k][p]  += g_logits^T (A, transposed reads) . act (B: the accumulator);
//   g_x^T [c][n] += (-2P)^T (A, transposed reads of the (-2P) image) . g_s^T (B: the wave's own
//                  g_s written to its LDS region and read back transposed), and sum_p g_s from
//                  the same fragments against ones.
// g_P / g_W stay in registers for the launch (one slab per workgroup, summed by the reduce
// kernel); g_x is a sum over the four waves' prototypes: each wave leaves its partial in LDS and,
// after one barrier, wave w adds the four partials of channels 16w .. 16w + 15 in a fixed order
// (bitwise deterministic, no atomics) and stores them. No other hand-off between the waves:
// between the two barriers of a tile every wave runs its own MFMA and VALU work, so the SIMDs
// do not wait on each other's phases.
//
// Staging: wave w loads the x of channels chan_of(w, hh, 0..7) for the tile's 32 pixels (lane
// = pixel: each load instruction reads two 128-B rows) and g_logits classes 8w .. 8w + 7, one
// tile ahead into registers; after the tile's barrier they are split into the bf16 images. The
// x values stay in registers for the g_x epilogue (2 x sum_p g_s), whose stores use the same
// lane map.
#include <type_traits>

#include "bf16_split.h"
#include "l2_bf16_common.h"
#include "l2_launch.h"
#include "protoseg_host.h"

namespace protoseg {

namespace {

using namespace bf16l;

constexpr int kWW = 4;  // waves per workgroup: one per SIMD
constexpr int kWT = 2;  // split terms (bf16x3: 3 MFMAs per product)
constexpr int kWThreads = kWW * 64;

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// g_x partial rows: pixel n, 64 physical columns + sum_p g_s at column 64, padded to 68 floats
// (16-B row accesses of 16 consecutive pixels land on distinct banks).
constexpr int kPartRow = 68 * 4;

// LDS regions (bytes).
struct WaveLds {
  int pimg, xa, ga, raw, raw_gl, raw_cls, x2u, ro, cl, tm, tw, tw_bytes, total;
};
__host__ __device__ constexpr WaveLds wave_lds(int NB) {
  WaveLds o{};
  const int Pp = 128 * NB;
  o.pimg = 0;                          // [T][Pp][64 c] (-2P), CPR 8, chan_of order (the forward's)
  o.xa = o.pimg + kWT * Pp * 128;      // [T][32 n][64 c] bf16, CPR 8, chan_of order
  o.ga = o.xa + kWT * 32 * 128;        // [T][32 n][32 k] bf16, CPR 4
  o.raw = o.ga + kWT * 32 * 64;        // LDS-DMA target: x [64 c][32 n] f32 (bf16 zero-extended)
  o.raw_gl = o.raw + 64 * 32 * 4;      //   g_logits: the tile's [32 n][K] run (K <= 32)
  o.raw_cls = o.raw_gl + 32 * 32 * 4;  //   the tile's KLD pixel classes (GD = 2): 64 dwords
  o.x2u = o.raw_cls + 64 * 4;          // [4 q][32 n] f32: u_q = s_{q,0} + s_{q,1} (||x||^2 pieces)
  o.ro = o.x2u + 4 * 32 * 4;           // [32] u32: g_dist byte offset per pixel (GD)
  o.cl = o.ro + 32 * 4;                // [32] int: the pixel's KLD class (GD = 2)
  o.tm = o.cl + 32 * 4;                // u32: the tile's KLD classes as a bit mask (GD = 2); 256 B
                                       // so the regions below keep their bank alignment
  // per wave: its g_s image for two blocks [T][2][32 p][32 n] bf16 (64-B rows, 8-B slots
  // swizzled), then, in the same bytes, its g_x partial [32 n][64 physical columns | sum_p g_s]
  o.tw = o.tm + 256;
  o.tw_bytes = 32 * kPartRow;         // >= kWT * 2 * 32 * 64 = 8192
  o.total = o.tw + kWW * o.tw_bytes;
  return o;
}

// Channel of physical column u of a CPR-8 image row (chunk u >> 3 holds chan_of(q, h, 0..7)).
__device__ __forceinline__ constexpr int chan_col(int u) { return chan_of(u >> 4, (u >> 3) & 1, u & 7); }

// LDS accesses by 32-bit byte address: a per-lane base register plus a compile-time immediate,
// which the DS instruction's 16-bit offset field absorbs (one address VGPR per access family).
typedef __attribute__((address_space(3))) bf16x8 lds_b128;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) float lds_f32;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ bf16x8 lds_frag(unsigned a) { return *reinterpret_cast<const lds_b128*>(static_cast<uintptr_t>(a)); }
__device__ __forceinline__ float lds_ld(unsigned a) { return *reinterpret_cast<const lds_f32*>(static_cast<uintptr_t>(a)); }
__device__ __forceinline__ uint32_t lds_ldu(unsigned a) { return *reinterpret_cast<const lds_u32*>(static_cast<uintptr_t>(a)); }
__device__ __forceinline__ void lds_st(unsigned a, float v) { *reinterpret_cast<lds_f32*>(static_cast<uintptr_t>(a)) = v; }
__device__ __forceinline__ void lds_stu(unsigned a, uint32_t v) { *reinterpret_cast<lds_u32*>(static_cast<uintptr_t>(a)) = v; }
__device__ __forceinline__ void lds_st_frag(unsigned a, bf16x8 v) { *reinterpret_cast<lds_b128*>(static_cast<uintptr_t>(a)) = v; }
__device__ __forceinline__ void lds_st4(unsigned a, s16x4 v) { *reinterpret_cast<lds_s16x4*>(static_cast<uintptr_t>(a)) = v; }
// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p' supplies the address of row q (4 contiguous
// elements); lane i of the group receives column i of the 4 rows (cdna_hip_programming.md T10).
// The two reads of one fragment give elements 0..3 and 4..7.
__device__ __forceinline__ bf16x8 lds_tr(unsigned lo, unsigned hi) {
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16(reinterpret_cast<lds_s16x4*>(static_cast<uintptr_t>(lo)));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16(reinterpret_cast<lds_s16x4*>(static_cast<uintptr_t>(hi)));
  const s16x8 v = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// The barrier between the phases of a tile: LDS visibility only. __syncthreads() would also wait
// for every outstanding global load and store, which the barrier does not need.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// WAVE_FENCE (development builds): a scheduling fence between the steps. Measured: the compiler's
// own schedule across the steps is 4% faster (no spills: 245 AGPRs vs 256 + 2 spilled VGPRs).
#ifdef WAVE_FENCE
#define WSCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define WSCHED_FENCE()
#endif

// WAVE_STAMP (diagnostic builds only): per-wave s_memtime deltas per phase, summed over the
// tiles, into a buffer of their own (read by protoseg_dev_wave_stamps); nothing else reads it.
#ifdef WAVE_STAMP
__device__ unsigned long long g_wave_stamp[1024 * 16];
#define WSTAMP(k)                                                  \
  do {                                                             \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    st_acc[k] += now_ - st_last;                                   \
    st_last = now_;                                                \
  } while (0)
#else
#define WSTAMP(k) \
  do {            \
  } while (0)
#endif

__device__ __forceinline__ uint32_t pack_bf16(float lo, float hi) {
  return static_cast<uint32_t>(__builtin_bit_cast(uint16_t, static_cast<bf16>(lo))) |
         (static_cast<uint32_t>(__builtin_bit_cast(uint16_t, static_cast<bf16>(hi))) << 16);
}

// GD: 0 no distance gradient, 1 a dense g_dist, 2 the KLD loss's compact one (CompactGd).
// NB: 32-prototype blocks per wave (Pp = 128 NB).
template <typename TX, int ACT, int GD, bool XSIG, int NB>
__global__ __launch_bounds__(kWThreads, 1) void l2_bwd_wave_bf16_kernel(
    const TX* __restrict__ x, unsigned x_bytes, int HW, int npix, const unsigned char* __restrict__ img, int P,
    int K, float eps, const float* __restrict__ g_logits, unsigned gl_bytes, const float* __restrict__ g_dist,
    unsigned gd_bytes, int gd_ld, int gd_p0, CompactGd cg, TX* __restrict__ g_x, int accumulate,
    float* __restrict__ slab, const float* __restrict__ protos) {
  constexpr int Pp = 128 * NB;  // prototype rows of the LDS image
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  constexpr WaveLds L = wave_lds(NB);
  const int Pi = (P + 31) & ~31;  // rows of the operand block's images (its Pp)
  const ImgOffsets io = img_offsets(Pi, kWT);
  const unsigned S0 = static_cast<unsigned>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) void*)smem_raw));

  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5, wave = wave_id();
  const int ntiles = (npix + 31) / 32;
#ifdef WAVE_STAMP
  unsigned long long st_acc[16] = {}, st_last = __builtin_amdgcn_s_memtime();
#endif
  const int G = static_cast<int>(gridDim.x);
  const int vb = xcd_block();  // neighbouring tiles on one XCD (l2_bf16_common.h); slab vb as well,
                               // so the reduce's fixed slab order sums the same tiles as before
  const int iters = (ntiles - vb + G - 1) / G;
  const unsigned sz = sizeof(TX);
  const unsigned chs = static_cast<unsigned>(HW) * sz;  // one channel plane
  const rsrc_t rx = make_rsrc(x, x_bytes), rg = make_rsrc(g_logits, gl_bytes);
  // GD = 2: g_dist points at the compact values (gd_bytes = npix * mpc * 4)
  const rsrc_t rgd = make_rsrc(GD == 2 ? cg.val : g_dist, gd_bytes), rgx = make_rsrc(g_x, g_x ? x_bytes : 0u);
  const rsrc_t rimg = make_rsrc(img, static_cast<unsigned>(io.total));
  const rsrc_t rpc = make_rsrc(cg.pix, GD == 2 ? static_cast<unsigned>(npix) * 4u : 0u);
  auto tile_of = [&](int i) __attribute__((always_inline)) { return vb + i * G; };
  const unsigned TWw = S0 + L.tw + wave * L.tw_bytes;  // this wave's g_s image / g_x partial

  // ---- prologue: the (-2P) image -> LDS (for the launch; term t of the block's Pi rows at term t
  // of the LDS image). Rows Pi .. Pp (blocks past the last prototype) are zero, as are their W
  // fragments (out-of-range loads) and ||p||^2, so their g_s is 0: every wave runs all NB blocks
  // without branches (the critical path is NB blocks per wave either way).
#pragma unroll
  for (int t = 0; t < kWT; ++t) lds_copy(smem_raw + L.pimg + t * Pp * 128, img + io.p + t * Pi * 128, Pi * 128);
  for (int i = Pi * 8 + static_cast<int>(threadIdx.x); i < Pp * 8; i += kWThreads)
#pragma unroll
    for (int t = 0; t < kWT; ++t)
      reinterpret_cast<u32x4*>(smem_raw + L.pimg + t * Pp * 128)[i] = u32x4{0u, 0u, 0u, 0u};
  // per owned block: the g_act B fragments (grad_unit W)[k = 16 s + 8 h + e][p] (rows of the W^T
  // image, registers for the launch), ||p||^2 as a bf16 pair (the B operand of the k-step that
  // adds ||x||^2 + ||p||^2, below) and (GD = 2) the class / compact column
  bf16x8 wreg[NB][2][kWT];
  uint32_t p2pk[NB][2];
  int pcls[NB], pslot[NB];
  uint32_t bmask[NB];  // (GD = 2) the classes of block jb's prototypes as a bit mask (K <= 32), uniform
#pragma unroll
  for (int jb = 0; jb < NB; ++jb) {
    const int p = 32 * (NB * wave + jb) + j;
    const unsigned wb = p < Pi ? static_cast<unsigned>(io.wt) : kOOB;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int t = 0; t < kWT; ++t)
        wreg[jb][s][t] = __builtin_bit_cast(
            bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                        rimg, wb + static_cast<unsigned>((t * Pi * 32 + img_off<4>(p, 2 * s + h)) * 2), 0, 0));
    const float p2 = __uint_as_float(
        __builtin_amdgcn_raw_buffer_load_b32(rimg, p < Pi ? static_cast<unsigned>(io.p2 + 4 * p) : kOOB, 0, 0));
    // three bf16 terms hold the f32 exactly (hi, mid, lo: 8 + 8 + 8 significant bits)
    const float p2h = static_cast<float>(static_cast<bf16>(p2));
    const float p2m = static_cast<float>(static_cast<bf16>(p2 - p2h));
    p2pk[jb][0] = h == 0 ? pack_bf16(1.f, p2h) : 0u;
    p2pk[jb][1] = h == 0 ? pack_bf16(p2m, (p2 - p2h) - p2m) : 0u;
    pcls[jb] = -2;  // never a pixel class (those are >= -1)
    pslot[jb] = 0;
    if constexpr (GD == 2) {
      const int code = p < P ? cg.slot[gd_p0 + p] : 0;
      pcls[jb] = p < P ? code >> 8 : -2;
      pslot[jb] = (code & 255) * 4;
      uint32_t m = pcls[jb] >= 0 && pcls[jb] < 32 ? 1u << pcls[jb] : 0u;  // (bucket K never matches a pixel)
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) m |= static_cast<uint32_t>(__shfl_xor(static_cast<int>(m), o));
      bmask[jb] = __builtin_amdgcn_readfirstlane(m);
    }
  }
  // bf16 (1, 1) in the k-steps' first dword for the lanes of half 0 (k = 0..7), 0 for half 1
  const uint32_t one2 = h == 0 ? 0x3F803F80u : 0u;

  // ---- staging: tile t's raw x, g_logits (and pixel classes) land in the raw region by LDS-DMA
  // (buffer_load ... lds: no registers; out-of-range lanes land as 0). x piece k (channels 2k,
  // 2k + 1: [c][n] rows, lane = pixel) for k = 8 wave .. 8 wave + 7; g_logits pieces of the
  // tile's contiguous 32 K floats m = wave, wave + 4, ...
  struct Stage {
    unsigned off;  // the lane's x offset (kOOB past the map)
    int lim;       // valid floats of the tile's g_logits run
  };
  auto stage_of = [&](int t) __attribute__((always_inline)) -> Stage {
    const int n = lane & 31, gp = t * 32 + n;
    Stage st{kOOB, t < ntiles ? min(32, npix - t * 32) * K : 0};
    if (t < ntiles && gp < npix) {
      const int b = div_pix(gp, HW);
      st.off = static_cast<unsigned>((b * kC + (lane >> 5)) * HW + (gp - b * HW)) * sz;
    }
    return st;
  };
  // piece m of tile t: m = 0..7 x pieces, 8..11 g_logits pieces (16 pieces of 64 floats cover
  // 32 K <= 1024; pieces past the run land zeros), 12 the pixel classes (GD = 2, wave 3)
  auto stage_piece = [&](int t, const Stage& st, int m) __attribute__((always_inline)) {
    if (m < 8) {
      const int k = 8 * wave + m;
      dma<TX>(rx, smem_raw + L.raw + k * 256, st.off, static_cast<unsigned>(2 * k) * chs);
    } else if (m < 12) {
      const int mg = wave + kWW * (m - 8);
      dma<float>(rg, smem_raw + L.raw_gl + mg * 256, mg * 64 + lane < st.lim ? static_cast<unsigned>(lane * 4) : kOOB,
                 static_cast<unsigned>((t * 32 * K + mg * 64) * 4));
    } else if constexpr (GD == 2) {
      if (wave == kWW - 1) {
        const int valid = t < ntiles ? min(32, npix - t * 32) : 0;
        dma<float>(rpc, smem_raw + L.raw_cls, lane < valid ? static_cast<unsigned>(lane * 4) : kOOB,
                   static_cast<unsigned>(t * 32 * 4));
      }
    }
  };
  constexpr int kPieces = GD == 2 ? 13 : 12;
  auto stage_dma = [&](int t) __attribute__((always_inline)) {
    const Stage st = stage_of(t);
#pragma unroll
    for (int m = 0; m < kPieces; ++m) stage_piece(t, st, m);
  };
  // Raw tile -> split images. Lane (n = j, hh = h) of wave w: x channels chan_of(w, hh, 0..7) of
  // pixel n (chunk 2w + hh of the x image row n), the chunk's ||x||^2 piece in the family's fixed
  // order (chunk fma chain, the pair (q, 0) + (q, 1) here, the q pairs in compute_tile); lanes
  // h = 0 also g_logits classes 8w .. 8w + 7 of pixel n (chunk w of the g_logits image row n).
  const unsigned a_xrow = S0 + L.xa + j * 128 + (((2 * wave + h) ^ swz<8>(j)) << 4);  // XA chunk (2w + h), row j
  auto convert = [&](int t) __attribute__((always_inline)) {
    const int gp = t * 32 + j;
    const bool ok = gp < npix;
    const unsigned a_raw = S0 + L.raw + (chan_of(wave, h, 0) * 32 + j) * 4;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if constexpr (sizeof(TX) == 4) v[e] = lds_ld(a_raw + chan_of(0, 0, e) * 128);
      else v[e] = __uint_as_float(lds_ldu(a_raw + chan_of(0, 0, e) * 128) << 16);
    }
    if constexpr (XSIG) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = ok ? sigmoid_f(v[e]) : 0.f;  // pixels past the map stay 0
    }
    bf16x8 f[kWT];
    split8<kWT>(v, f);
    lds_st_frag(a_xrow, f[0]);
    lds_st_frag(a_xrow + 32 * 128, f[1]);
    float sq = chunk_sq(v);
    sq += __shfl_xor(sq, 32);
    if (h == 0) {
      lds_st(S0 + L.x2u + (wave * 32 + j) * 4, sq);
      const unsigned a_gl = S0 + L.raw_gl + (j * K + 8 * wave) * 4;
      float g[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] = lds_ld(a_gl + 4 * e);  // in the region for every k < 32
      pin_batch(g);  // loaded together, then the classes past K zeroed (no branch per load)
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] = 8 * wave + e < K ? g[e] : 0.f;
      split8<kWT>(g, f);
      const unsigned a_ga = S0 + L.ga + j * 64 + ((wave ^ swz<4>(j)) << 4);
      lds_st_frag(a_ga, f[0]);
      lds_st_frag(a_ga + 32 * 64, f[1]);
    } else {
      // lanes h = 1: GD bookkeeping of the pixel (one wave writes each array)
      if constexpr (GD == 1) {
        if (wave == 1) {
          const int b = ok ? div_pix(gp, HW) : 0;
          lds_stu(S0 + L.ro + 4 * j, ok ? static_cast<unsigned>(((b * gd_ld + gd_p0) * HW + (gp - b * HW)) * 4) : kOOB);
        }
      } else if constexpr (GD == 2) {
        if (wave == 0) {
          const int cl = ok ? static_cast<int>(lds_ldu(S0 + L.raw_cls + 4 * j)) : -1;
          lds_stu(S0 + L.ro + 4 * j, cl >= 0 ? static_cast<unsigned>(gp * cg.mpc * 4) : kOOB);
          lds_stu(S0 + L.cl + 4 * j, static_cast<uint32_t>(cl));
          uint32_t m = cl >= 0 ? 1u << cl : 0u;  // (lanes 32..63: the shuffles stay in the half)
#pragma unroll
          for (int o = 1; o < 32; o <<= 1) m |= static_cast<uint32_t>(__shfl_xor(static_cast<int>(m), o));
          if (j == 0) lds_stu(S0 + L.tm, m);
        }
      }
    }
  };

  // ---- per-lane LDS address bases (loop-invariant; every other access of a family is an
  // immediate offset from its base: k-steps, terms, blocks and the wave's rows) -----------------
  // transposed-read lane roles: lane 16 gg + 4 qq + pq supplies row qq of its group's 4-row
  // block, columns 4 pq .. 4 pq + 3 of the group's 16 (gg & 1 selects which 16)
  const int gg = lane >> 4, qq = (lane >> 2) & 3, pq = lane & 3;
  const int tr_c16 = 2 * (gg & 1) + (pq >> 1);  // 16-B chunk within a 32-column tile
  const int tr_sub2 = 8 * (pq & 1);             // byte offset inside the chunk
  unsigned a_row[kNQ];                           // x / (-2P) row reads: row j, chunk 2q + h
#pragma unroll
  for (int q = 0; q < kNQ; ++q) a_row[q] = static_cast<unsigned>(j * 128 + (((2 * q + h) ^ swz<8>(j)) << 4));
  const unsigned pi_wave = S0 + L.pimg + static_cast<unsigned>(32 * NB * wave * 128);  // this wave's first row
  unsigned a_ga[2];  // g_logits row reads: row j, chunk 2s + h
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) a_ga[s2] = S0 + L.ga + j * 64 + (((2 * s2 + h) ^ swz<4>(j)) << 4);
  // X^T / g_logits^T transposed reads: rows 16 s + 4 h + qq (+ 8 i2); the swizzle does not depend on s
  unsigned a_xt[2][2], a_glt[2];
#pragma unroll
  for (int i2 = 0; i2 < 2; ++i2) {
    const int row = 4 * h + qq + 8 * i2;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
      a_xt[i2][ct] = S0 + L.xa + row * 128 + (((4 * ct + tr_c16) ^ swz<8>(row)) << 4) + tr_sub2;
    a_glt[i2] = S0 + L.ga + row * 64 + ((tr_c16 ^ swz<4>(row)) << 4) + tr_sub2;
  }
  // g_s image: 8-B slot s of row p at s ^ ((p >> 1) & 7) (stores: 16 consecutive rows per 16-lane
  // group, one slot; transposed reads: 4 rows x 64 B per 32-lane half: both conflict-free)
  unsigned a_tw[2][2];  // stores of row j: slot 4s + h + 2 half
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) a_tw[s2][hf] = TWw + j * 64 + (((4 * s2 + h + 2 * hf) ^ ((j >> 1) & 7)) << 3);
  unsigned a_bt[2];  // transposed reads: rows 16 s + 8 h + qq (+ 4 i4), slot 4 (gg & 1) + pq
#pragma unroll
  for (int i4 = 0; i4 < 2; ++i4) {
    const int row = 8 * h + qq + 4 * i4;
    a_bt[i4] = TWw + row * 64 + (((4 * (gg & 1) + pq) ^ ((row >> 1) & 7)) << 3);
  }
  unsigned a_pa[2][2];  // (-2P)^T transposed reads: rows p0 + 16 s + 8 h + qq (+ 4 i4)
#pragma unroll
  for (int i4 = 0; i4 < 2; ++i4) {
    const int row = 8 * h + qq + 4 * i4;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) a_pa[i4][ct] = pi_wave + row * 128 + (((4 * ct + tr_c16) ^ swz<8>(row)) << 4) + tr_sub2;
  }

  // ---- accumulators for the launch ------------------------------------------------------------
  f32x16 gp[NB][2], gw[NB];
  float gsum[NB];
#pragma unroll
  for (int jb = 0; jb < NB; ++jb) {
    gp[jb][0] = gp[jb][1] = gw[jb] = zero16();
    gsum[jb] = 0.f;
  }
  // sum_p g_s per pixel: a 16x16x32 product of a selector A against the g_x product's B fragments
  // (lane l: pixel l & 31, prototypes 16 s + 8 (l >> 5) + e), read as 16x16x32 operands (column
  // l & 15, k = 8 (l >> 4) + e): A row 0 is one on k-groups 0 and 2 (pixels 0..15), row 1 on
  // groups 1 and 3 (pixels 16..31), i.e. lanes 0, 32 and 17, 49
  bf16x8 onesel;
  {
    const bf16 v = static_cast<bf16>(lane == 0 || lane == 32 || lane == 17 || lane == 49 ? 1.f : 0.f);
#pragma unroll
    for (int e = 0; e < 8; ++e) onesel[e] = v;
  }

  // ---- one tile. One wave per SIMD: nothing else fills the matrix pipe, so the instruction
  // stream itself puts VALU work between the MFMAs. The program order is a software pipeline over
  // the wave's blocks: a fill (block 0's S / g_act products beside the next tile's staging DMA),
  // then per block jb six steps, each pairing a step of block jb's epilogue (VALU) with products
  // of other blocks (block jb+1's front, block jb-1's g_x, g_P / g_W pieces of blocks jb-1 and
  // jb), then a drain (the last block's g_x and g_P / g_W k-step 1) and the partial into the
  // wave's LDS region. The compiler schedules within that order (WAVE_FENCE: per step).
  auto compute_tile = [&](int tn) __attribute__((always_inline)) {
    // the A operand of the ||x||^2 + ||p||^2 k-step: row n = j holds (x2_hi, x2_mid, x2_lo, 1, 1,
    // 1) in k = 0..5 (half 0); its B operand per block (1, 1, 1, p2_hi, p2_mid, p2_lo): three bf16
    // terms hold each f32 exactly, so the MFMA adds the f32 x2 + p2 to every element and the S
    // accumulator starts from zero (no per-element initialisation)
    u32x4 ax2;
    {
      const unsigned a = S0 + L.x2u + 4 * j;
      const float x2 = (lds_ld(a) + lds_ld(a + 128)) + (lds_ld(a + 256) + lds_ld(a + 384));
      const float x2h = static_cast<float>(static_cast<bf16>(x2));
      const float x2m = static_cast<float>(static_cast<bf16>(x2 - x2h));
      ax2 = h == 0 ? u32x4{pack_bf16(x2h, x2m), pack_bf16((x2 - x2h) - x2m, 1.f), one2, 0u} : u32x4{0u, 0u, 0u, 0u};
    }
    const bf16x8 ax2f = __builtin_bit_cast(bf16x8, ax2);
    // (GD = 2) the tile's class mask: blocks with none of its classes skip their g_dist loads
    const uint32_t tmask = GD == 2 ? __builtin_amdgcn_readfirstlane(lds_ldu(S0 + L.tm)) : 0u;

    struct Front {
      f32x16 acc, gacc;
      float gdv[16];
    };
    // g_dist values of block jb, accumulator rows 8 hf .. 8 hf + 7 (epilogue steps 3 hf, 3 hf + 1)
    auto front_gd = [&](int jb, Front& fr, int hf) __attribute__((always_inline)) {
      const int p = 32 * (NB * wave + jb) + j;
      if constexpr (GD == 2) {
        if ((tmask & bmask[jb]) == 0u) {  // no pixel of the tile has a class of the block: all 0
#pragma unroll
          for (int e = 8 * hf; e < 8 * hf + 8; ++e) fr.gdv[e] = 0.f;
          return;
        }
#pragma unroll
        for (int g4 = 2 * hf; g4 < 2 * hf + 2; ++g4) {
          const u32x4 ro = __builtin_bit_cast(u32x4, lds_frag(S0 + L.ro + 16 * h + 32 * g4));
          const u32x4 cl = __builtin_bit_cast(u32x4, lds_frag(S0 + L.cl + 16 * h + 32 * g4));
          const unsigned rv[4] = {ro[0], ro[1], ro[2], ro[3]};
          const int cv[4] = {static_cast<int>(cl[0]), static_cast<int>(cl[1]), static_cast<int>(cl[2]), static_cast<int>(cl[3])};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            fr.gdv[4 * g4 + e] = BufIO<float>::load(rgd, cv[e] == pcls[jb] ? rv[e] + pslot[jb] : kOOB, 0);
        }
      } else if constexpr (GD == 1) {
        const unsigned pcol = static_cast<unsigned>(p * HW * 4);
        const bool pvalid = p < P;
#pragma unroll
        for (int g4 = 2 * hf; g4 < 2 * hf + 2; ++g4) {
          const u32x4 ro = __builtin_bit_cast(u32x4, lds_frag(S0 + L.ro + 16 * h + 32 * g4));
          const unsigned rv[4] = {ro[0], ro[1], ro[2], ro[3]};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            fr.gdv[4 * g4 + e] = BufIO<float>::load(rgd, (rv[e] != kOOB && pvalid) ? rv[e] + pcol : kOOB, 0);
        }
      }
    };
    // front product step k (0..5) of block jb: operands, MFMAs. k = 0..3: S channel k-step k
    // (x (A) against (-2P) (B), smallest products first); k = 4, 5: g_act class k-step (W^T rows
    // / g_logits columns past K are zero)
    struct FrontOps {
      bf16x8 a[kWT], b[kWT];
    };
    auto front_load = [&](int jb, int k, FrontOps& o) __attribute__((always_inline)) {
      if (k < 4) {
        o.a[0] = lds_frag(S0 + L.xa + a_row[k]);
        o.a[1] = lds_frag(S0 + L.xa + a_row[k] + 32 * 128);
        o.b[0] = lds_frag(pi_wave + a_row[k] + jb * 4096);
        o.b[1] = lds_frag(pi_wave + a_row[k] + jb * 4096 + Pp * 128);
      } else {
        o.a[0] = lds_frag(a_ga[k - 4]);
        o.a[1] = lds_frag(a_ga[k - 4] + 32 * 64);
      }
    };
    auto front_mfma = [&](int jb, int k, Front& fr, const FrontOps& o) __attribute__((always_inline)) {
      if (k == 0) {
        const bf16x8 bp2 = __builtin_bit_cast(bf16x8, u32x4{one2, p2pk[jb][0], p2pk[jb][1], 0u});
        fr.acc = mfma_bf16(ax2f, bp2, zero16());
      }
      if (k < 4) {
        fr.acc = mfma_bf16(o.a[1], o.b[0], fr.acc);
        fr.acc = mfma_bf16(o.a[0], o.b[1], fr.acc);
        fr.acc = mfma_bf16(o.a[0], o.b[0], fr.acc);
      } else {
        fr.gacc = mma_split<kWT>(o.a, wreg[jb][k - 4], k == 4 ? zero16() : fr.gacc);
      }
    };
    // epilogue step e (0..5) of block jb: e = 0, 1, 3, 4 rows 4(e - e/3) .. +3 (g_s, act,
    // sum_n g_s); e = 2, 5 the split fragments of k-step s = e / 3 (the B operands of g_P / g_W)
    // and g_s into the wave's [p][n] image (buffer jb & 1): fragment elements 0..3 are rows
    // 16s + 4h + 0..3 (slot 4s + h), elements 4..7 rows 16s + 8 + 4h + 0..3 (slot 4s + 2 + h).
    float gsv[16], av[16];
    auto epi_step = [&](int jb, int e, const Front& fr, bf16x8 (&gsf)[2][kWT], bf16x8 (&actf)[2][kWT])
        __attribute__((always_inline)) {
      if (e != 2 && e != 5) {
        const int r0 = 4 * (e - e / 3);
#pragma unroll
        for (int r = r0; r < r0 + 4; ++r) {
          const float d = relu_f(fr.acc[r]);
          float a;
          float gd = fr.gacc[r] * act_grad_and_base<ACT>(d, eps, a);  // grad_unit is in the W^T image
          if constexpr (GD) gd += fr.gdv[r];
          const float g = d > 0.f ? gd : 0.f;  // relu backward
          gsum[jb] += g;
          gsv[r] = g;
          av[r] = a;  // act_unit is applied to g_W in the slab reduce
        }
      } else {
        const int sk = e / 3;
        float v[8], w8[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          v[i] = gsv[8 * sk + i];
          w8[i] = av[8 * sk + i];
        }
        split8<kWT>(v, gsf[sk]);
        split8<kWT>(w8, actf[sk]);
#pragma unroll
        for (int t = 0; t < kWT; ++t) {
          const s16x8 q = __builtin_bit_cast(s16x8, gsf[sk][t]);
          const unsigned o = (jb & 1) * 2048 + t * 4096;
          lds_st4(a_tw[sk][0] + o, __builtin_shufflevector(q, q, 0, 1, 2, 3));
          lds_st4(a_tw[sk][1] + o, __builtin_shufflevector(q, q, 4, 5, 6, 7));
        }
      }
    };
    // g_P^T += X^T g_s, g_W += g_logits^T act (the accumulators are the B operands); X^T and
    // g_logits^T by transposed reads, k = n in the accumulator's row order; step s = 0, 1
    // piece pc of k-step s: pc = 0, 1 g_P^T channel tile pc, pc = 2 g_W
    struct WOps {
      bf16x8 a[kWT];
    };
    auto w_load = [&](int s, int pc, WOps& o) __attribute__((always_inline)) {
#pragma unroll
      for (int t = 0; t < kWT; ++t)
        o.a[t] = pc < 2 ? lds_tr(a_xt[0][pc] + s * 2048 + t * 4096, a_xt[1][pc] + s * 2048 + t * 4096)
                        : lds_tr(a_glt[0] + s * 1024 + t * 2048, a_glt[1] + s * 1024 + t * 2048);
    };
    auto w_mfma = [&](int jb, int s, int pc, const WOps& o, const bf16x8 (&gsf)[2][kWT], const bf16x8 (&actf)[2][kWT])
        __attribute__((always_inline)) {
      if (pc < 2) gp[jb][pc] = mma_split<kWT>(o.a, gsf[s], gp[jb][pc]);
      else gw[jb] = mma_split<kWT>(o.a, actf[s], gw[jb]);
    };
    // g_x^T [c][n] += (-2P)^T [c][p] g_s^T [p][n] over block jb's 32 prototypes (natural k
    // order: k = 8h + e is prototype 16s + 8h + e), sum_p g_s against ones; step (s, half):
    // half 0 = the g_s fragments + channel tile 0, half 1 = channel tile 1 + the ones products
    struct GxOps {
      bf16x8 bt[kWT], pa[kWT];
    };
    auto gx_load = [&](int jb, int s, int half, GxOps& o) __attribute__((always_inline)) {
      if (half == 0) {
#pragma unroll
        for (int t = 0; t < kWT; ++t) {
          const unsigned ob = (jb & 1) * 2048 + s * 1024 + t * 4096;
          o.bt[t] = lds_tr(a_bt[0] + ob, a_bt[1] + ob);
        }
      }
#pragma unroll
      for (int t = 0; t < kWT; ++t) {
        const unsigned op = jb * 4096 + s * 2048 + t * Pp * 128;
        o.pa[t] = lds_tr(a_pa[0][half] + op, a_pa[1][half] + op);
      }
    };
    auto gx_mfma = [&](int half, const GxOps& o, const bf16x8 (&bt)[kWT], f32x16 (&gx)[2], f32x4& sg)
        __attribute__((always_inline)) {
      gx[half] = mma_split<kWT>(o.pa, bt, gx[half]);
      if (half == 1) {
        sg = __builtin_amdgcn_mfma_f32_16x16x32_bf16(onesel, bt[1], sg, 0, 0, 0);
        sg = __builtin_amdgcn_mfma_f32_16x16x32_bf16(onesel, bt[0], sg, 0, 0, 0);
      }
    };

    Front fr[2];
    bf16x8 gsf[2][kWT], actf[2][kWT];
    f32x16 gx[2] = {zero16(), zero16()};
    f32x4 sg = {0.f, 0.f, 0.f, 0.f};
    bf16x8 bt[kWT];
    // fill: block 0's front, the next tile's staging pieces beside it (their issue cost hides
    // behind the MFMAs; the raw region is free: this tile is converted). The g_dist rows of a
    // block load in two halves: rows 0..7 a period ahead, rows 8..15 (used from epilogue step 3)
    // at the start of the block's own period, so at most 16 of them are live at a time.
    front_gd(0, fr[0], 0);
    {
      const Stage st = stage_of(tn);
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        FrontOps o;
        front_load(0, k, o);
        stage_piece(tn, st, 2 * k);
        stage_piece(tn, st, 2 * k + 1);
        if (k == 5 && kPieces > 12) stage_piece(tn, st, 12);
        front_mfma(0, k, fr[0], o);
        WSCHED_FENCE();
      }
    }
    WSTAMP(1);
    // period jb, six steps; step k: the LDS operands of the step, block jb's epilogue step k, then
    // the products: block jb+1's front k-step k, block jb-1's g_x half step k (k < 4), and the
    // g_P / g_W pieces: block jb-1's k-step 1 (k < 3: its split fragments live until epilogue
    // step 5 rewrites them) and block jb's k-step 0 (k >= 3: written by epilogue step 2)
#pragma unroll
    for (int jb = 0; jb < NB; ++jb) {
      const bool nxt = jb + 1 < NB, prv = jb >= 1;
      Front& cur = fr[jb & 1];
      Front& fn = fr[(jb + 1) & 1];
      front_gd(jb, cur, 1);
      if (nxt) front_gd(jb + 1, fn, 0);
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        FrontOps o;
        GxOps xo;
        WOps wo;
        if (nxt) front_load(jb + 1, k, o);
        if (prv && k < 4) gx_load(jb - 1, k >> 1, k & 1, xo);
        if (prv && k < 3) w_load(1, k, wo);
        if (k >= 3) w_load(0, k - 3, wo);
        epi_step(jb, k, cur, gsf, actf);
        if (nxt) front_mfma(jb + 1, k, fn, o);
        if (prv && k < 4) {
          if ((k & 1) == 0) {
#pragma unroll
            for (int t = 0; t < kWT; ++t) bt[t] = xo.bt[t];
          }
          gx_mfma(k & 1, xo, bt, gx, sg);
        }
        if (prv && k < 3) w_mfma(jb - 1, 1, k, wo, gsf, actf);
        if (k >= 3) w_mfma(jb, 0, k - 3, wo, gsf, actf);
        WSCHED_FENCE();
      }
      WSTAMP(2 + jb);
    }
    // drain: the last block's g_x products and its g_P / g_W k-step 1
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      GxOps xo;
      WOps wo;
      gx_load(NB - 1, k >> 1, k & 1, xo);
      if (k < 3) w_load(1, k, wo);
      if ((k & 1) == 0) {
#pragma unroll
        for (int t = 0; t < kWT; ++t) bt[t] = xo.bt[t];
      }
      gx_mfma(k & 1, xo, bt, gx, sg);
      if (k < 3) w_mfma(NB - 1, 1, k, wo, gsf, actf);
      WSCHED_FENCE();
    }
    WSCHED_FENCE();
    WSTAMP(8);
    // the partial (row: pixel j, columns: physical channel columns 32 ct + acc_row, 4 consecutive
    // per 16-B store) and sum_p g_s (column 64) into this wave's region (the g_s image's bytes;
    // the wave's own LDS operations run in order)
    asm volatile("" ::: "memory");
    const unsigned a_part = TWw + j * kPartRow + 16 * h;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
        *reinterpret_cast<__attribute__((address_space(3))) f32x4*>(static_cast<uintptr_t>(a_part + (32 * ct + 8 * g4) * 4)) =
            f32x4{gx[ct][4 * g4], gx[ct][4 * g4 + 1], gx[ct][4 * g4 + 2], gx[ct][4 * g4 + 3]};
    if (lane < 16) {  // sum_p g_s of pixels j and j + 16 (rows 0, 1 of the 16x16 product)
      lds_st(TWw + j * kPartRow + 64 * 4, sg[0]);
      lds_st(TWw + (j + 16) * kPartRow + 64 * 4, sg[1]);
    }
    WSTAMP(9);
  };

  // ---- g_x epilogue of a tile: wave w adds the four partials of its rows (physical columns
  // 16 w + 8 hh + e = channels chan_of(w, hh, e)) in a fixed order, + 2 x sum_p g_s, x from the
  // x image (hi + lo: within 2^-17 of x) ------------------------------------------------------
  auto pix_off = [&](int t) __attribute__((always_inline)) -> unsigned {
    const int gp = t * 32 + j;
    if (gp >= npix) return kOOB;
    const int b = div_pix(gp, HW);
    return static_cast<unsigned>((b * kC) * HW + (gp - b * HW)) * sz +
           static_cast<unsigned>(chan_of(wave, h, 0) * HW) * sz;
  };
  auto reduce_store = [&](int t) __attribute__((always_inline)) {
    const unsigned pb = S0 + L.tw + j * kPartRow;
    constexpr int ps = L.tw_bytes;  // bytes between the waves' regions
    const float sgt = ((lds_ld(pb + 256) + lds_ld(pb + ps + 256)) + lds_ld(pb + 2 * ps + 256)) + lds_ld(pb + 3 * ps + 256);
    const unsigned vo = pix_off(t);
    float old[8] = {};
    if (accumulate) {  // (wave-uniform: a single-chunk call issues no loads and waits on none)
#pragma unroll
      for (int e = 0; e < 8; ++e) old[e] = BufIO<TX>::load(rgx, vo, static_cast<unsigned>(chan_of(0, 0, e)) * chs);
    }
    const u32x4 xh = __builtin_bit_cast(u32x4, lds_frag(a_xrow)), xl = __builtin_bit_cast(u32x4, lds_frag(a_xrow + 32 * 128));
    // the 8 physical columns 16 w + 8 h .. + 7 of each wave's partial: two 16-B reads each
    const unsigned pr = pb + (16 * wave + 8 * h) * 4;
    typedef __attribute__((address_space(3))) f32x4 lds_f32x4;
    f32x4 pq[kWW][2];
#pragma unroll
    for (int q = 0; q < kWW; ++q)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) pq[q][hf] = *reinterpret_cast<const lds_f32x4*>(static_cast<uintptr_t>(pr + q * ps + 16 * hf));
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float tot = ((pq[0][e >> 2][e & 3] + pq[1][e >> 2][e & 3]) + pq[2][e >> 2][e & 3]) + pq[3][e >> 2][e & 3];
      const unsigned sh = (e & 1) ? 0u : 16u;
      const float xv = __uint_as_float((xh[e >> 1] << sh) & 0xFFFF0000u) + __uint_as_float((xl[e >> 1] << sh) & 0xFFFF0000u);
      float v;
      if constexpr (XSIG) {  // through the sigmoid: g_pre = g_x s (1 - s)
        v = (tot + sgt * (2.f * xv)) * (xv * (1.f - xv));
      } else {
        v = tot + sgt * (2.f * xv);  // conv(x^2, ones) backward: sum_p g_s * 2x
      }
      if (accumulate) v = old[e] + v;
      BufIO<TX>::store(rgx, v, vo, static_cast<unsigned>(chan_of(0, 0, e)) * chs);
    }
  };

  // ---- main loop. Per tile: [the next tile's LDS-DMA | compute(i) | partial] barrier
  // [g_x(i) epilogue | staging of tile i+1 from the raw region] barrier.
  if (iters > 0) stage_dma(tile_of(0));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the (-2P) image and tile 0's raw DMA
  __syncthreads();
  if (iters > 0) convert(tile_of(0));
  lds_barrier();
  WSTAMP(14);
  // (no branches in the loop body: past the last tile, the staging loads land zeros)
  for (int i = 0; i < iters; ++i) {
    const int t = tile_of(i);
    WSTAMP(0);
#ifndef WAVE_ABL_NOCOMPUTE  // (WAVE_ABL_*: timing ablations of development builds; wrong results)
    compute_tile(tile_of(i + 1));  // (+ the staging DMA of tile i + 1)
#else
    stage_dma(tile_of(i + 1));
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of tile i + 1 has landed
    lds_barrier();  // every partial of tile i and every raw piece of tile i + 1 written; images read
    WSTAMP(10);
#ifndef WAVE_ABL_NOREDCONV
    reduce_store(t);
    WSTAMP(11);
    convert(tile_of(i + 1));
    WSTAMP(12);
#else
    (void)t;
#endif
    lds_barrier();  // images(i+1) written; every partial read
    WSTAMP(13);
  }

  // ---- slab: this workgroup's g_P^T = -2 X^T g_s + 2 p sum_n g_s (x -2: the x image holds +x;
  // the conv(x^2, ones) term's 2 p sum g_s is added per workgroup, so the reduce sums g_P slabs
  // alone) and g_W in the reduce kernel's layout (gp_t 2): [64][Pi] g_P^T | [K][Pi] g_W | [Pi]
  // unused, rows padded to Pi = 32 ceil(P / 32) prototypes so that every half-wave store is one
  // whole aligned 128-B line (rows past P and classes past K are not written)
  const int E = Pi * kC + K * Pi + Pi;
  float* my_slab = slab + static_cast<size_t>(vb) * E;
#ifdef WAVE_ABL_NOSLAB
  if (npix != -7) return;
#endif
#pragma unroll
  for (int jb = 0; jb < NB; ++jb) {
    if (32 * (NB * wave + jb) >= P) continue;  // blocks past the last prototype
    const int p = 32 * (NB * wave + jb) + j;
    float s = gsum[jb];
    s += __shfl_xor(s, 32);
    if (p < P) {
      const float s2 = 2.f * s;
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int c = chan_col(32 * ct + acc_row(r, h));
          my_slab[static_cast<size_t>(c) * Pi + p] = fmaf(s2, protos[static_cast<size_t>(p) * kC + c], -2.f * gp[jb][ct][r]);
        }
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (acc_row(r, h) < K) my_slab[static_cast<size_t>(Pi) * kC + acc_row(r, h) * Pi + p] = gw[jb][r];
    }
  }
#ifdef WAVE_STAMP
  WSTAMP(15);
  if (lane < 16) {
    unsigned long long v = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) v = lane == k ? st_acc[k] : v;
    g_wave_stamp[(blockIdx.x * kWW + wave) * 16 + lane] = v;
  }
#endif
}

template <typename TX, int ACT, int GD, bool XSIG, int NB>
int wave_t(const Geometry& g, const void* x, const unsigned char* img, float eps, const float* g_logits,
           const float* g_dist, void* g_x, int accumulate, float* ws, int grid, hipStream_t stream) {
  constexpr size_t lds = static_cast<size_t>(wave_lds(NB).total);
  static_assert(lds <= kMaxLds, "wave backward LDS");
  if (int st = ensure_lds<l2_bwd_wave_bf16_kernel<TX, ACT, GD, XSIG, NB>, lds>()) return st;
  const unsigned long long npix = static_cast<unsigned long long>(g.npix);
  const unsigned xb = static_cast<unsigned>(npix * kC * sizeof(TX));
  const unsigned glb = g_logits ? static_cast<unsigned>(npix * g.K * 4) : 0u;
  const unsigned gdb = GD == 2 ? static_cast<unsigned>(npix * g.cgd.mpc * 4)
                               : g_dist ? static_cast<unsigned>(npix * g.ldd * 4) : 0u;
  KernelTimer timer("l2_bwd_wave_bf16_kernel", stream);
  hipLaunchKernelGGL((l2_bwd_wave_bf16_kernel<TX, ACT, GD, XSIG, NB>), dim3(grid), dim3(kWThreads), lds, stream,
                     static_cast<const TX*>(x), xb, g.HW, g.npix, img, g.P, g.K, eps, g_logits, glb, g_dist, gdb,
                     g.ldd, g.p0, g.cgd, static_cast<TX*>(g_x), accumulate, ws, g.protos + static_cast<size_t>(g.p0) * kC);
  return check_launch("l2_bwd_wave_bf16_kernel");
}

}  // namespace

int bf16_wave_nb(int P) { return P <= 128 ? 1 : P <= 256 ? 2 : 3; }

bool bf16_bwd_wave_fits(const Geometry& g, int terms) {
  return terms == kWT && g.C == kC && g.P > 0 && g.P <= kWW * 3 * 32 && g.K <= 32 && bf16_sizes_ok(g);
}

int bf16_bwd_wave_grid(const Geometry& g) {
  const int cus = device_cus();
  // as many workgroups as the rounds need, no more (every slab the reduce reads did work)
  const int rounds = static_cast<int>(ceil_div(g.ntiles, cus));
  return static_cast<int>(ceil_div(g.ntiles, rounds > 0 ? rounds : 1));
}

size_t bf16_bwd_wave_slab_elems(const Geometry& g) {
  const size_t P = static_cast<size_t>(g.P + 31) & ~static_cast<size_t>(31);  // padded rows (the slab write)
  return static_cast<size_t>(bf16_bwd_wave_grid(g)) * (P * kC + static_cast<size_t>(g.K) * P + P);
}

int launch_bwd_wave_bf16(const Geometry& g, bool x_bf16, const void* x, const void* img, float eps, int act_kind,
                         const float* g_logits, const float* g_dist, void* g_x, float* ws, hipStream_t stream,
                         int accumulate) {
  const unsigned char* blk = static_cast<const unsigned char*>(img);
  const int grid = bf16_bwd_wave_grid(g);
  const int nb = bf16_wave_nb(g.P);
  if (!g.protos) return fail(PROTOSEG_ERR_INVALID, "wave backward: Geometry::protos (the slab's 2 p sum g_s) is null");
  auto go = [&](auto tx, auto aa, auto gd) __attribute__((always_inline)) {
    using TX = std::remove_pointer_t<decltype(tx)>;
    constexpr int kA = decltype(aa)::value;
    constexpr int kG = decltype(gd)::value;
    auto by_nb = [&](auto xs) __attribute__((always_inline)) {
      constexpr bool kX = decltype(xs)::value;
      if (nb == 3) return wave_t<TX, kA, kG, kX, 3>(g, x, blk, eps, g_logits, g_dist, g_x, accumulate, ws, grid, stream);
      if (nb == 2) return wave_t<TX, kA, kG, kX, 2>(g, x, blk, eps, g_logits, g_dist, g_x, accumulate, ws, grid, stream);
      return wave_t<TX, kA, kG, kX, 1>(g, x, blk, eps, g_logits, g_dist, g_x, accumulate, ws, grid, stream);
    };
    return g.xsig ? by_nb(std::true_type()) : by_nb(std::false_type());
  };
  using A0 = std::integral_constant<int, 0>;
  using A1 = std::integral_constant<int, 1>;
  using G0 = std::integral_constant<int, 0>;
  using G1 = std::integral_constant<int, 1>;
  using G2 = std::integral_constant<int, 2>;
  float* f = nullptr;
  uint16_t* b = nullptr;
#ifdef WAVE_DEV_ONE  // development builds: the headline instantiation only
  if (g.cgd.val || x_bf16 || g_dist || act_kind != 0 || g.xsig || nb != WAVE_DEV_ONE)
    return fail(PROTOSEG_ERR_UNSUPPORTED, "WAVE_DEV_ONE build");
  return wave_t<float, 0, 0, false, WAVE_DEV_ONE>(g, x, blk, eps, g_logits, g_dist, g_x, accumulate, ws, grid, stream);
#else
  if (g.cgd.val) {  // the compact KLD gradient: f32 x only (bf16_bwd_compact_ok)
    if (x_bf16 || g_dist) return fail(PROTOSEG_ERR_UNSUPPORTED, "compact g_dist: f32 x and no dense g_dist");
    return act_kind == 0 ? go(f, A0(), G2()) : go(f, A1(), G2());
  }
  if (act_kind == 0)
    return x_bf16 ? (g_dist ? go(b, A0(), G1()) : go(b, A0(), G0())) : (g_dist ? go(f, A0(), G1()) : go(f, A0(), G0()));
  return x_bf16 ? (g_dist ? go(b, A1(), G1()) : go(b, A1(), G0())) : (g_dist ? go(f, A1(), G1()) : go(f, A1(), G0()));
#endif
}

}  // namespace protoseg

#ifdef WAVE_STAMP
extern "C" int protoseg_dev_wave_stamps(unsigned long long* host, int n) {
  return static_cast<int>(hipMemcpyFromSymbol(host, HIP_SYMBOL(protoseg::g_wave_stamp), sizeof(unsigned long long) * n));
}
#endif
