// l2_bwd_fused.hip — the prototype layer's backward as ONE kernel on bf16 MFMA with 2-term
// split operands (bf16x3, C = 64, up to 192 prototypes per launch; larger P runs as prototype
// chunks). It is the autograd of reference model.py:203-221 (_l2_convolution), 231-237
// (distance_2_similarity) and 259-283 (forward_from_conv_features), which has no explicit
// backward upstream:
//   S = ||x||^2 + ||p||^2 - 2 X.P^T,  d = relu(S),  act = f(d),  logits = act . W^T
//   g_act = g_logits . W,  g_s = (g_act f'(d) + g_dist) [d > 0]
//   g_x   = 2 x sum_p g_s - 2 g_s . P          g_P = 2 p sum_n g_s - 2 g_s^T . X
//   g_W   = g_logits^T . act
// The two-kernel form (l2_bf16.hip: bwd_x + bwd_pw) computes S, g_act and the epilogue twice;
// here every (pixel tile, prototype tile) block computes them once.
//
// Workgroup = 8 waves, one per CU (LDS), persistent over 32-pixel tiles:
//   waves 0..5 ("owners"): wave w owns prototype tile w. Layout B (rows = pixels n, columns =
//     prototypes p, so the prototype is on the lane): S and g_act on MFMA, the epilogue, then
//     g_P^T += g_s^T X and g_W += g_logits^T act with the accumulators as operands (the
//     contraction is over their row index n), so g_P / g_W stay in registers for the whole
//     launch: one slab per workgroup, summed by l2_bwd_reduce_bf16_kernel. g_s also goes to LDS
//     as a [p][n] bf16 image (8-byte stores, no shuffles).
//   waves 6, 7 ("x waves"): x wave c owns channel tile c of g_x. g_x^T[c][n] = (-2P)^T g_s^T sums
//     over p, the accumulator's column index, so it reads both operands transposed
//     (ds_read_b64_tr_b16) from the (-2P) image and the g_s image; sum_p g_s comes from the same
//     fragments times a ones matrix. Output lane = pixel: coalesced NCHW stores.
// The owners also stage the tiles (register loads one tile ahead, conversion to the split bf16
// images + ||x||^2 one tile ahead). One barrier per iteration; the x, g_logits and g_s images
// are double-buffered, so owners work on tile i while the x waves finish g_x of tile i-1.
#include <type_traits>

#ifdef PROTOSEG_STAMPS
#define PROTOSEG_STAMP_ARRAY ::protoseg::g_stamps_fused
#include <hip/hip_runtime.h>
namespace protoseg {
__device__ unsigned long long g_stamps_fused[1 << 17];
}
// 16 slots per wave (tools/stamps_fused.py); each stamp is fenced so the phases it brackets are
// not reordered across it (debug builds only: production code has neither stamps nor fences).
#define FSTAMP(slot)                                                                                 \
  do {                                                                                               \
    __builtin_amdgcn_sched_barrier(0);                                                               \
    const unsigned _w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);                         \
    if ((threadIdx.x & 63) == 0 && _w * 16 + (slot) < (1u << 17))                                    \
      ::protoseg::g_stamps_fused[_w * 16 + (slot)] =                                                 \
          (slot) == 14 ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime();            \
    __builtin_amdgcn_sched_barrier(0);                                                               \
  } while (0)
#else
#define FSTAMP(slot) \
  do {               \
  } while (0)
#endif
#include "bf16_split.h"
#include "l2_bf16_common.h"
#include "l2_launch.h"
#include "protoseg_host.h"

namespace protoseg {

namespace {

using namespace bf16l;

constexpr int kT = 2;                       // split terms (bf16x3: 3 MFMAs per product)
constexpr int kOwners = 6;                  // prototype-tile waves
constexpr int kXWaves = 2;                  // channel-tile waves (64 channels = 2 x 32)
constexpr int kThreads = (kOwners + kXWaves) * 64;
constexpr int kMaxPp = kOwners * 32;        // prototypes per launch

// Raw tile slot (LDS-DMA target, dwords): x as [32 pieces][2 rows c][32 n] with a 68-dword piece
// stride (rows c and c + 4, read together by the ||x||^2 chains, fall in different banks; bf16 x
// lands zero-extended in a dword), then g_logits as the tile's flat [32 n][K] run (K <= 32).
constexpr int kRawPiece = 68;
constexpr int kRawXDw = 32 * kRawPiece;
// + 64 dwords: the tile's KLD pixel classes (compact g_dist, GD = 2; one 64-lane DMA)
constexpr int kRawClsDw = kRawXDw + 32 * 32;
constexpr int kRawSlot = (kRawClsDw + 64) * 4;  // 13,056 B
__device__ __forceinline__ constexpr int raw_x(int c, int n) { return (c >> 1) * kRawPiece + (c & 1) * 32 + n; }

// LDS regions (bytes). The (-2P) and W^T images are adjacent, as in the operand-image block,
// so one LDS-DMA copy fills both.
struct FusedLds {
  int pimg, wtimg, xa, ga, x2s, rowoff, rcls, gs, raw, total;
};
__host__ __device__ inline FusedLds fused_lds(int Pp) {
  FusedLds o;
  o.pimg = 0;                           // [T][Pp][64] (-2P), CPR 8, chan_of order
  o.wtimg = kT * Pp * 128;              // [T][Pp][32] (grad_unit W)^T, CPR 4
  o.xa = o.wtimg + kT * Pp * 64;        // [2 slots][T][32 n][64 c] bf16, CPR 8
  o.ga = o.xa + 2 * kT * 32 * 64 * 2;   // [2 slots][T][32 n][32 k] bf16, CPR 4
  o.x2s = o.ga + 2 * kT * 32 * 32 * 2;  // [2 slots][32] f32: ||x||^2 per pixel
  o.rowoff = o.x2s + 2 * 32 * 4;        // [2 slots][32] u32: g_dist byte offset per pixel
  o.rcls = o.rowoff + 2 * 32 * 4;       // [2 slots][32] int: KLD pixel class (GD = 2)
  o.gs = o.rcls + 2 * 32 * 4;           // [2 slots][T][Pp][32 n] bf16, 8-B slots swizzled
  o.total = o.gs + 2 * kT * Pp * 64;
  // Raw tiles (LDS-DMA targets, 2 slots). The operand images are read into registers in the
  // prologue, so their region is free afterwards and holds the raw slots when it is big enough.
  if (o.xa - o.pimg >= 2 * kRawSlot) {
    o.raw = o.pimg;
  } else {
    o.raw = o.total;
    o.total += 2 * kRawSlot;
  }
  return o;
}

// Keeps the scheduler from hoisting a later phase's LDS loads above this point (register
// pressure: every phase's operand fragments in flight at once would spill).
#define SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p' supplies the address of row q (4 contiguous
// elements); lane i of the group receives column i of the 4 rows (cdna_hip_programming.md T10).
// The two reads of one fragment give elements 0..3 and 4..7.
__device__ __forceinline__ bf16x8 tr_frag(const bf16* lo, const bf16* hi) {
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(lo));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(hi));
  const s16x8 v = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// g_s image: [Pp rows p][32 n] bf16, 64-B rows of eight 8-B slots (4 pixels each), slot
// swizzle (p >> 1) & 7: the owners' 8-byte stores (16 rows per lane group) and the x waves'
// transposed reads (4 rows x 64 B per 32-lane half) are both conflict-free.
__device__ __forceinline__ int gs_off(int row, int slot) { return row * 32 + ((slot ^ ((row >> 1) & 7)) << 2); }

// Channel of physical column u of a CPR-8 image row (chunk u>>3 holds chan_of(q, h, 0..7)).
__device__ __forceinline__ constexpr int chan_of_col(int u) { return chan_of(u >> 4, (u >> 3) & 1, u & 7); }

// XSIG: x is the add-on's pre-activation (PROTOSEG_X_SIGMOID): a template parameter, so the
// plain instantiations carry no trace of it (registers, scheduling). NPT: prototype tiles of
// the launch when known at compile time (6: Pp = 192, every chunk at P = 190 / 361 / 570), else
// 0 (read from Pp): with it the x waves' g_x loop is one straight-line block instead of a
// branch per prototype tile (each branch a scheduling boundary with its own s_waitcnt).
// GD: 0 no distance gradient, 1 a dense g_dist, 2 the KLD loss's compact one (CompactGd).
template <typename TX, int ACT, int GD, bool XSIG, int NPT>
__global__ __launch_bounds__(kThreads) void l2_bwd_fused_bf16_kernel(
    const TX* __restrict__ x, unsigned x_bytes, int HW, int npix, const unsigned char* __restrict__ img, int P, int Pp,
    int K, float eps, const float* __restrict__ g_logits, unsigned gl_bytes, const float* __restrict__ g_dist,
    unsigned gd_bytes, int gd_ld, int gd_p0, CompactGd cg, TX* __restrict__ g_x, int accumulate,
    float* __restrict__ slab) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const FusedLds L = fused_lds(Pp);
  const ImgOffsets io = img_offsets(Pp, kT);
  bf16* Pimg = reinterpret_cast<bf16*>(smem_raw + L.pimg);
  bf16* WTimg = reinterpret_cast<bf16*>(smem_raw + L.wtimg);
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5, wave = wave_id();
  const int ntiles = (npix + 31) / 32;
  const int npt = NPT ? NPT : Pp / 32;
  const int vb = xcd_block();  // neighbouring tiles on one XCD (l2_bf16_common.h); slab vb as well
  const int iters = (ntiles - vb + static_cast<int>(gridDim.x) - 1) / static_cast<int>(gridDim.x);
  const bool owner = wave < kOwners;
  const int xw = wave - kOwners;  // x wave index (channel tile), valid when !owner
  const unsigned sz = sizeof(TX);
  const rsrc_t rx = make_rsrc(x, x_bytes), rg = make_rsrc(g_logits, gl_bytes);
  // GD = 2: g_dist points at the compact values (gd_bytes = npix * mpc * 4)
  const rsrc_t rgd = make_rsrc(GD == 2 ? cg.val : g_dist, gd_bytes), rgx = make_rsrc(g_x, g_x ? x_bytes : 0u);
  const rsrc_t rpc = make_rsrc(cg.pix, GD == 2 ? static_cast<unsigned>(npix) * 4u : 0u);
  auto tile_of = [&](int i) __attribute__((always_inline)) { return vb + i * static_cast<int>(gridDim.x); };
  auto xa_slot = [&](int sb) __attribute__((always_inline)) { return reinterpret_cast<bf16*>(smem_raw + L.xa) + sb * kT * 32 * kC; };
  auto ga_slot = [&](int sb) __attribute__((always_inline)) { return reinterpret_cast<bf16*>(smem_raw + L.ga) + sb * kT * 32 * 32; };
  auto x2_slot = [&](int sb) __attribute__((always_inline)) { return reinterpret_cast<float*>(smem_raw + L.x2s) + sb * 32; };
  auto ro_slot = [&](int sb) __attribute__((always_inline)) { return reinterpret_cast<unsigned*>(smem_raw + L.rowoff) + sb * 32; };
  auto cl_slot = [&](int sb) __attribute__((always_inline)) { return reinterpret_cast<int*>(smem_raw + L.rcls) + sb * 32; };
  auto gs_slot = [&](int sb) __attribute__((always_inline)) { return reinterpret_cast<bf16*>(smem_raw + L.gs) + sb * kT * Pp * 32; };

  // ---- staging (all 8 waves) ------------------------------------------------------------------
  // Tile t's raw x and g_logits land in raw slot rs by LDS-DMA (no registers, whole cache lines):
  // x piece k (rows 2k, 2k + 1: lane = pixel) for k = 4 wave .. 4 wave + 3, and g_logits pieces
  // m = wave, wave + 8, ... of the tile's contiguous 32 K floats. Out-of-range lanes land as 0.
  using XS = std::conditional_t<sizeof(TX) == 4, float, uint32_t>;
  auto raw_slot = [&](int rs) __attribute__((always_inline)) { return reinterpret_cast<XS*>(smem_raw + L.raw + rs * kRawSlot); };
  auto stage_dma = [&](int t, int rs) __attribute__((always_inline)) {
    XS* R = raw_slot(rs);
    const int n = lane & 31, g = t * 32 + n;
    unsigned off = kOOB;
    if (t < ntiles && g < npix) {
      const int b = div_pix(g, HW);
      off = static_cast<unsigned>((b * kC + (lane >> 5)) * HW + (g - b * HW)) * sz;
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int k = 4 * wave + m;
      dma<TX>(rx, R + k * kRawPiece, off, static_cast<unsigned>(2 * k * HW) * sz);
    }
    const int lim = t < ntiles ? min(32, npix - t * 32) * K : 0;  // valid floats of the tile's run
    float* RG = reinterpret_cast<float*>(R + kRawXDw);
    for (int m = wave; m * 64 < 32 * K; m += 8)
      dma<float>(rg, RG + m * 64, m * 64 + lane < lim ? static_cast<unsigned>(lane * 4) : kOOB,
                 static_cast<unsigned>((t * 32 * K + m * 64) * 4));
    if constexpr (GD == 2) {  // the tile's 32 contiguous pixel classes (lanes past them land 0)
      if (wave == kOwners + kXWaves - 1) {
        const int valid = t < ntiles ? min(32, npix - t * 32) : 0;
        dma<float>(rpc, R + kRawClsDw, lane < valid ? static_cast<unsigned>(lane * 4) : kOOB,
                   static_cast<unsigned>(t * 32 * 4));
      }
    }
  };
  // Raw slot rs -> split images of slot sb, pixels 4 wave .. 4 wave + 3 per wave: lanes 0..31
  // the 8 XA chunks of a pixel (lane = 8 (pixel) + chunk 2q + hh: channels chan_of(q, hh, 0..7)),
  // lanes 32..47 its 4 GA chunks (classes 8 kc .. 8 kc + 7). ||x||^2 in the family's fixed order
  // (chunk_sq per lane, then chunk pairs (q, 0)+(q, 1), q pairs, halves: three butterflies over
  // the pixel's 8 lanes), so the distances match the forward's bit for bit.
  auto convert = [&](int t, int rs, int sb) __attribute__((always_inline)) {
    const XS* R = raw_slot(rs);
    float v[8];
    bf16x8 f[kT];
    // lane-derived addresses rebuilt per tile from an opaque lane id: held across the loop they
    // are what the allocator spills first (a scratch reload + vmcnt(0) per tile)
    int z = 0;
    asm volatile("" : "+v"(z));
    const int lz = lane + z;
    if (lane < 32) {
      const int n = 4 * wave + (lz >> 3), ch = lz & 7;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = lds_val(R + raw_x(chan_of(ch >> 1, ch & 1, e), n));
      if constexpr (XSIG) {  // pixels past the map stay 0 (their g_s is 0 anyway)
        const bool ok = t < ntiles && t * 32 + n < npix;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = ok ? sigmoid_f(v[e]) : 0.f;
      }
      split8<kT>(v, f);
      store_frag<kT>(xa_slot(sb), 32 * kC, img_off<8>(n, ch), f);
      float s = chunk_sq(v);
      s += __shfl_xor(s, 1);
      s += __shfl_xor(s, 2);
      s += __shfl_xor(s, 4);
      if (ch == 0) x2_slot(sb)[n] = s;
    } else if (lane < 48) {
      const int n = 4 * wave + ((lz - 32) >> 2), kc = lz & 3;
      const float* RG = reinterpret_cast<const float*>(R + kRawXDw);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 8 * kc + e < K ? RG[n * K + 8 * kc + e] : 0.f;
      split8<kT>(v, f);
      store_frag<kT>(ga_slot(sb), 32 * 32, img_off<4>(n, kc), f);
      if constexpr (GD == 1) {
        if (kc == 0) {
          const int g = t * 32 + n;
          const bool ok = t < ntiles && g < npix;
          const int b = ok ? div_pix(g, HW) : 0;
          ro_slot(sb)[n] = ok ? static_cast<unsigned>(((b * gd_ld + gd_p0) * HW + (g - b * HW)) * 4) : kOOB;
        }
      } else if constexpr (GD == 2) {
        if (kc == 0) {  // the pixel's compact row and class
          const int g = t * 32 + n;
          const int cl = (t < ntiles && g < npix) ? reinterpret_cast<const int*>(R + kRawClsDw)[n] : -1;
          ro_slot(sb)[n] = cl >= 0 ? static_cast<unsigned>(g * cg.mpc * 4) : kOOB;
          cl_slot(sb)[n] = cl;
        }
      }
    }
  };

  // Per-lane parts of the transposed-read addresses: lane 16G + 4qq + pp supplies row qq of
  // its group's 4-row block, columns 4pp..4pp+3 of the group's 16 (G & 1 selects which 16).
  const int G = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
  const int tr_c16 = 2 * (G & 1) + (pp >> 1);  // 16-B chunk within a 32-column tile
  const int tr_sub = 4 * (pp & 1);             // element offset inside the chunk

  // ---- owners: one prototype tile against one pixel tile --------------------------------------
  f32x16 gp[2] = {zero16(), zero16()};  // sum_n g_s x  (rows p, cols: physical x columns)
  f32x16 gw = zero16();                 // g_logits^T act (rows k, cols p)
  float gsum = 0.f;                     // sum_n g_s, this half-wave's rows
  const int p = (owner ? wave : 0) * 32 + j;
  const bool pvalid = p < P;
  const float p2 = owner ? reinterpret_cast<const float*>(img + io.p2)[p] : 0.f;
  int pcls = -2, pslot = 0;  // GD = 2: this lane's prototype's class (-2: none) and compact column
  if constexpr (GD == 2) {
    if (owner && pvalid) {
      const int code = cg.slot[gd_p0 + p];
      pcls = code >> 8;
      pslot = (code & 255) * 4;
    }
  }
  // this wave's prototype-tile B fragments of S and g_act (registers, loaded in the prologue)
  bf16x8 preg[kNQ][kT], wreg[2][kT];
  auto owner_tile = [&](int sb, bool stamp) __attribute__((always_inline)) {
    const bf16* XA = xa_slot(sb);
    const bf16* GA = ga_slot(sb);
    float x2r[16], gdv[16];
    load_rows16(x2_slot(sb) + 4 * h, x2r);
    if constexpr (GD == 2) {  // four rows at a time: the row offsets / classes are not all live at once
      const unsigned* ros = ro_slot(sb) + 4 * h;
      const int* cls = cl_slot(sb) + 4 * h;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const uint4 ro = *reinterpret_cast<const uint4*>(ros + 8 * g4);
        const int4 cl = *reinterpret_cast<const int4*>(cls + 8 * g4);
        const unsigned rv[4] = {ro.x, ro.y, ro.z, ro.w};
        const int cv[4] = {cl.x, cl.y, cl.z, cl.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) gdv[4 * g4 + e] = BufIO<float>::load(rgd, cv[e] == pcls ? rv[e] + pslot : kOOB, 0);
      }
    } else if constexpr (GD == 1) {
      float rof[16];
      load_rows16(reinterpret_cast<const float*>(ro_slot(sb)) + 4 * h, rof);
      const unsigned pcol = static_cast<unsigned>(p * HW * 4);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const unsigned ro = __float_as_uint(rof[r]);
        gdv[r] = BufIO<float>::load(rgd, (ro != kOOB && pvalid) ? ro + pcol : kOOB, 0);
      }
    }
    f32x16 acc;  // ||x||^2 + ||p||^2, then the (-2P) image does the rest
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = x2r[r] + p2;
#pragma unroll
    for (int q = 0; q < kNQ; ++q) {
      bf16x8 xa[kT];
      load_frag<kT>(XA, 32 * kC, img_off<8>(j, 2 * q + h), xa);
      acc = mma_split<kT>(xa, preg[q], acc);
    }
    if (stamp) FSTAMP(7);
    f32x16 gacc = zero16();  // both class k-steps run: W^T rows / GA columns past K are zero
    SCHED_FENCE();
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 ga[kT];
      load_frag<kT>(GA, 32 * 32, img_off<4>(j, 2 * s + h), ga);
      gacc = mma_split<kT>(ga, wreg[s], gacc);
    }
    if (stamp) FSTAMP(8);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float d = relu_f(acc[r]);
      float a;
      float gd = gacc[r] * act_grad_and_base<ACT>(d, eps, a);  // grad_unit is in the W^T image
      if constexpr (GD) gd += gdv[r];
      const float gs = d > 0.f ? gd : 0.f;  // relu backward
      gsum += gs;
      acc[r] = gs;
      gacc[r] = a;  // act_unit is applied to g_W in the slab reduce
    }
    SCHED_FENCE();
    if (stamp) FSTAMP(9);
    bf16x8 gsf[2][kT], actf[2][kT];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      acc_operand<kT>(acc, s, gsf[s]);
      acc_operand<kT>(gacc, s, actf[s]);
    }
    // g_s -> [p][n] image: fragment elements 0..3 are rows 16s + 4h + 0..3 (slot 4s + h),
    // elements 4..7 rows 16s + 8 + 4h + 0..3 (slot 4s + 2 + h).
    bf16* GS = gs_slot(sb);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int t = 0; t < kT; ++t) {
        const s16x8 v = __builtin_bit_cast(s16x8, gsf[s][t]);
        *reinterpret_cast<s16x4*>(GS + t * Pp * 32 + gs_off(p, 4 * s + h)) = __builtin_shufflevector(v, v, 0, 1, 2, 3);
        *reinterpret_cast<s16x4*>(GS + t * Pp * 32 + gs_off(p, 4 * s + 2 + h)) =
            __builtin_shufflevector(v, v, 4, 5, 6, 7);
      }
    SCHED_FENCE();
    if (stamp) FSTAMP(10);
    // g_P^T += g_s^T X: B = x[n][c] with k = n in the accumulator's order, from XA transposed.
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int r1 = 16 * s + 4 * h + qq, r2 = r1 + 8;
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        bf16x8 xt[kT];
        const int c16 = 4 * ct + tr_c16;
#pragma unroll
        for (int t = 0; t < kT; ++t)
          xt[t] = tr_frag(XA + t * 32 * kC + r1 * kC + ((c16 ^ swz<8>(r1)) << 3) + tr_sub,
                          XA + t * 32 * kC + r2 * kC + ((c16 ^ swz<8>(r2)) << 3) + tr_sub);
        gp[ct] = mma_split<kT>(gsf[s], xt, gp[ct]);
      }
      if (stamp && s == 1) FSTAMP(11);
      // g_W += g_logits^T act: A = g_logits[n][k] transposed (lane = class).
      bf16x8 glt[kT];
#pragma unroll
      for (int t = 0; t < kT; ++t)
        glt[t] = tr_frag(GA + t * 32 * 32 + r1 * 32 + ((tr_c16 ^ swz<4>(r1)) << 3) + tr_sub,
                         GA + t * 32 * 32 + r2 * 32 + ((tr_c16 ^ swz<4>(r2)) << 3) + tr_sub);
      gw = mma_split<kT>(glt, actf[s], gw);
    }
  };

  // ---- x waves: g_x of one tile from the g_s image of slot sb ---------------------------------
  // D[c][n] = sum_p (-2P)^T[c][p] g_s^T[p][n] (c = physical column 32 xw + row), and
  // s[n] = sum_p g_s[n][p]; g_x = D + 2 x s. Register r of half h holds channel
  // 32 xw + 16 (r >> 3) + 4 ((r >> 2) & 1) + (r & 3) + 8h (chan_of of its column).
  // s[n]: the g_s fragments of k-steps 0 and 1 exchanged by v_permlane16_swap so that every
  // lane holds pixel (lane & 15) (first) or 16 + (lane & 15) (second), then one
  // v_mfma_f32_16x16x32_bf16 against ones per term and pixel half: 32 prototypes per MFMA at
  // half the cycles of the 32x32x16 form.
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = static_cast<bf16>(1.f);
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  // The (-2P)^T fragments of this wave's channel tile are the same for every pixel tile: read
  // once into registers (kMaxPp / 16 k-steps x T terms x 4 VGPRs = 96); per prototype tile only
  // the g_s fragments come from LDS (8 transposed reads, one tile ahead).
  constexpr int kMaxNpt = kMaxPp / 32;
  bf16x8 pa[kMaxNpt][2][kT];
  auto gs_frags = [&](const bf16* GS, int pt, bf16x8 (&b)[2][kT]) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int r1 = 32 * pt + 16 * s + 8 * h + qq, r2 = r1 + 4;
#pragma unroll
      for (int t2 = 0; t2 < kT; ++t2)
        b[s][t2] = tr_frag(GS + t2 * Pp * 32 + gs_off(r1, 4 * (G & 1) + pp), GS + t2 * Pp * 32 + gs_off(r2, 4 * (G & 1) + pp));
    }
  };
  auto gx_tile = [&](int t, int sb, bool stamp) __attribute__((always_inline)) {
    const bf16* GS = gs_slot(sb);
    const int g = t * 32 + j;
    unsigned pix = kOOB;
    if (g < npix) {
      const int b = div_pix(g, HW);
      pix = static_cast<unsigned>((b * kC + 32 * xw + 8 * h) * HW + (g - b * HW)) * sz;
    }
    // x (for the 2 x s term) and, for chunk c > 0, the earlier chunks' g_x: loads issued before
    // the MFMA loop so their latency hides under it.
    float xr[16], old[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const unsigned co = static_cast<unsigned>((16 * (r >> 3) + 4 * ((r >> 2) & 1) + (r & 3)) * HW) * sz;
      xr[r] = BufIO<TX>::load(rx, pix, co);
      old[r] = BufIO<TX>::load(rgx, accumulate ? pix : kOOB, co);
    }
    f32x16 acc = zero16();
#ifdef FUSED_XACC2
    f32x16 acc1 = zero16();  // second chain: k-step 1 of every prototype tile
#endif
    f32x4 s_lo = {0.f, 0.f, 0.f, 0.f}, s_hi = {0.f, 0.f, 0.f, 0.f};
    bf16x8 b0[2][kT], b1[2][kT];
    auto step = [&](int pt, bf16x8 (&b)[2][kT]) __attribute__((always_inline)) {
      acc = mma_split<kT>(pa[pt][0], b[0], acc);
#ifdef FUSED_XACC2
      acc1 = mma_split<kT>(pa[pt][1], b[1], acc1);
#else
      acc = mma_split<kT>(pa[pt][1], b[1], acc);
#endif
#ifndef FUSED_NO_ONES
#pragma unroll
      for (int t2 = 0; t2 < kT; ++t2) {
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        u32x4 f0 = __builtin_bit_cast(u32x4, b[0][t2]), f1 = __builtin_bit_cast(u32x4, b[1][t2]);
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const auto r = __builtin_amdgcn_permlane16_swap(f0[v], f1[v], false, false);
          f0[v] = r[0];
          f1[v] = r[1];
        }
        s_lo = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, __builtin_bit_cast(bf16x8, f0), s_lo, 0, 0, 0);
        s_hi = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, __builtin_bit_cast(bf16x8, f1), s_hi, 0, 0, 0);
      }
#endif
    };
    // Ping-pong over prototype tiles: tile pt + 1's reads (8, within the 15 LDS operations a
    // wave keeps in flight) are issued, pinned by a scheduling barrier, before tile pt's MFMAs.
    gs_frags(GS, 0, b0);
#pragma unroll
    for (int pt = 0; pt < kMaxNpt; pt += 2) {
      if (pt < npt) {
        if (pt + 1 < npt) gs_frags(GS, pt + 1, b1);
        SCHED_FENCE();
        step(pt, b0);
        SCHED_FENCE();
      }
      if (pt + 1 < npt) {
        if (pt + 2 < npt) gs_frags(GS, pt + 2, b0);
        SCHED_FENCE();
        step(pt + 1, b1);
        SCHED_FENCE();
      }
    }
    if (stamp) FSTAMP(6);
#ifdef FUSED_XACC2
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] += acc1[r];
#endif
    const float sn = j < 16 ? s_lo[0] : s_hi[0];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const unsigned co = static_cast<unsigned>((16 * (r >> 3) + 4 * ((r >> 2) & 1) + (r & 3)) * HW) * sz;
      float v;
      if constexpr (XSIG) {  // through the sigmoid: g_pre = g_x s (1 - s)
        const float s = sigmoid_f(xr[r]);
        v = (acc[r] + sn * (2.f * s)) * (s * (1.f - s));
      } else {
        v = acc[r] + sn * (2.f * xr[r]);  // conv(x^2, ones) backward: sum_p g_s * 2x
      }
      BufIO<TX>::store(rgx, accumulate ? old[r] + v : v, pix, co);  // chunk c > 0 adds
    }
  };

  // ---- prologue + main loop ------------------------------------------------------------------
  // Operand images -> LDS -> registers (owners: their tile's S / g_act B fragments; x waves:
  // their channel tile's (-2P)^T fragments); then the image region becomes the raw slots:
  // tiles 0 and 1 land by DMA, tile 0 is converted.
  FSTAMP(0);
  FSTAMP(14);
  lds_copy(Pimg, img + io.p, io.p2 - io.p);  // (-2P) and W^T images
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // The rest of the prologue and the main loop are written once per role (the role is
  // wave-uniform; both paths run the same barriers), so neither role's register-resident
  // operands or loop-carried values are live in the other's code.
  auto prologue_tail = [&]() __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // image reads done before the DMA reuses it
    __syncthreads();
    stage_dma(tile_of(0), 0);
    if (iters > 1) stage_dma(tile_of(1), 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    convert(tile_of(0), 0, 0);
    __syncthreads();
    FSTAMP(1);
  };
  // Main loop: all waves convert tile i+1 (raw slot (i+1)&1, landed last iteration) and start
  // tile i+2's DMA into raw slot i&1 (converted last iteration); then owners work on tile i and
  // the x waves finish g_x of tile i-1.
  if (owner) {
#pragma unroll
    for (int q = 0; q < kNQ; ++q) load_frag<kT>(Pimg, Pp * kC, img_off<8>(p, 2 * q + h), preg[q]);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) load_frag<kT>(WTimg, Pp * 32, img_off<4>(p, 2 * s2 + h), wreg[s2]);
    prologue_tail();
    // Unrolled by two so the image slot of every LDS access is a compile-time constant.
    auto owner_iter = [&](int i, auto slot) __attribute__((always_inline)) {
      constexpr int sb = decltype(slot)::value;
      if (i == 2) FSTAMP(2);
      // Owners 4, 5 share their SIMDs with owners 0, 1 (waves w and w + 4 pair up): they stage
      // after their tile instead of before it, so the two waves of a SIMD are in different
      // phases (one's MFMAs beside the other's conversion VALU / LDS traffic).
#ifndef FUSED_NO_STAGGER
      const bool late = wave >= 4;
#else
      const bool late = false;
#endif
      if (!late) {
        if (i + 1 < iters) convert(tile_of(i + 1), sb ^ 1, sb ^ 1);
        if (i == 2) FSTAMP(5);
        if (i + 2 < iters) stage_dma(tile_of(i + 2), sb);
        if (i == 2) FSTAMP(6);
      }
      if (i < iters && wave < npt) owner_tile(sb, i == 2);
      if (late) {
        if (i + 1 < iters) convert(tile_of(i + 1), sb ^ 1, sb ^ 1);
        if (i + 2 < iters) stage_dma(tile_of(i + 2), sb);
      }
      if (i == 2) FSTAMP(3);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of tile i+2
      __syncthreads();
      if (i == 2) FSTAMP(4);
    };
    for (int i = 0; i <= iters; i += 2) {
      owner_iter(i, std::integral_constant<int, 0>());
      if (i + 1 <= iters) owner_iter(i + 1, std::integral_constant<int, 1>());
    }
  } else {
    {
      const int c16 = 4 * xw + tr_c16;
#pragma unroll
      for (int pt = 0; pt < kMaxNpt; ++pt)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int r1 = (pt < npt ? 32 * pt : 0) + 16 * s + 8 * h + qq, r2 = r1 + 4;
#pragma unroll
          for (int t2 = 0; t2 < kT; ++t2)
            pa[pt][s][t2] = tr_frag(Pimg + t2 * Pp * kC + r1 * kC + ((c16 ^ swz<8>(r1)) << 3) + tr_sub,
                                    Pimg + t2 * Pp * kC + r2 * kC + ((c16 ^ swz<8>(r2)) << 3) + tr_sub);
        }
    }
    prologue_tail();
#ifdef FUSED_XPRIO
    __builtin_amdgcn_s_setprio(FUSED_XPRIO);  // the x waves are the loop's critical path
#endif
    for (int i = 0; i <= iters; ++i) {
      if (i == 2) FSTAMP(2);
#ifndef FUSED_NO_XSTAGE
      if (i + 1 < iters) convert(tile_of(i + 1), (i + 1) & 1, (i + 1) & 1);
      if (i == 2) FSTAMP(5);
      if (i + 2 < iters) stage_dma(tile_of(i + 2), i & 1);
#endif
      // g_x's x loads are issued after the DMA and waited for before its stores, so the DMA has
      // landed by then (vector-memory operations retire in issue order); without g_x, wait here.
      if (i >= 1) {
        gx_tile(tile_of(i - 1), (i - 1) & 1, i == 2);
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if (i == 2) FSTAMP(7);
      if (i == 2) FSTAMP(3);
      __syncthreads();
      if (i == 2) FSTAMP(4);
    }
  }
  FSTAMP(13);

  // ---- slab: this workgroup's g_P (x -2: XA holds +x), g_W, sum_n g_s -------------------------
  if (owner && wave < npt) {
    const int E = Pp * kC + 32 * Pp + Pp;
    float* my_slab = slab + static_cast<size_t>(vb) * E;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        my_slab[static_cast<size_t>(wave * 32 + acc_row(r, h)) * kC + chan_of_col(32 * ct + j)] = -2.f * gp[ct][r];
#pragma unroll
    for (int r = 0; r < 16; ++r) my_slab[static_cast<size_t>(Pp) * kC + acc_row(r, h) * Pp + wave * 32 + j] = gw[r];
    gsum += __shfl_xor(gsum, 32);
    if (h == 0) my_slab[static_cast<size_t>(Pp) * kC + 32 * Pp + wave * 32 + j] = gsum;
  }
}

template <typename TX, int ACT, int GD, bool XSIG, int NPT>
int fused_t(const Geometry& g, const void* x, const unsigned char* img, float eps, const float* g_logits,
            const float* g_dist, void* g_x, int accumulate, float* ws, int grid, hipStream_t stream) {
  if (int st = ensure_lds<l2_bwd_fused_bf16_kernel<TX, ACT, GD, XSIG, NPT>>()) return st;
  const unsigned long long npix = static_cast<unsigned long long>(g.npix);
  const unsigned xb = static_cast<unsigned>(npix * kC * sizeof(TX));
  const unsigned glb = g_logits ? static_cast<unsigned>(npix * g.K * 4) : 0u;
  const unsigned gdb = GD == 2 ? static_cast<unsigned>(npix * g.cgd.mpc * 4)
                               : g_dist ? static_cast<unsigned>(npix * g.ldd * 4) : 0u;
  KernelTimer timer("l2_bwd_fused_bf16_kernel", stream);
  hipLaunchKernelGGL((l2_bwd_fused_bf16_kernel<TX, ACT, GD, XSIG, NPT>), dim3(grid), dim3(kThreads),
                     static_cast<size_t>(fused_lds(g.Pp).total), stream, static_cast<const TX*>(x), xb, g.HW, g.npix, img,
                     g.P, g.Pp, g.K, eps, g_logits, glb, g_dist, gdb, g.ldd, g.p0, g.cgd, static_cast<TX*>(g_x), accumulate,
                     ws);
  return check_launch("l2_bwd_fused_bf16_kernel");
}

}  // namespace

bool bf16_bwd_fused_fits(const Geometry& g, int terms) {
  return terms == kT && g.C == kC && g.Pp <= kMaxPp && static_cast<size_t>(fused_lds(g.Pp).total) <= kMaxLds &&
         bf16_sizes_ok(g);
}

// as many workgroups as the rounds of 256 need (fewer slabs for the reduce at small batches)
int bf16_bwd_fused_grid(const Geometry& g) {
  const int rounds = static_cast<int>(ceil_div(g.ntiles, 256));
  return static_cast<int>(ceil_div(g.ntiles, rounds > 0 ? rounds : 1));
}

int launch_bwd_fused_bf16(const Geometry& g, bool x_bf16, const void* x, const float* protos, const void* img,
                          float eps, int act_kind, const float* g_logits, const float* g_dist, void* g_x,
                          float* g_protos, float* g_w, float* ws, hipStream_t stream, int accumulate, int reduce) {
  const unsigned char* blk = static_cast<const unsigned char*>(img);
  const int grid = bf16_bwd_fused_grid(g);
  auto go = [&](auto tx, auto aa, auto gd) __attribute__((always_inline)) {
    using TX = std::remove_pointer_t<decltype(tx)>;
    constexpr int kA = decltype(aa)::value;
    constexpr int kG = decltype(gd)::value;
    const bool six = g.Pp == 6 * 32;
    if (g.xsig)
      return six ? fused_t<TX, kA, kG, true, 6>(g, x, blk, eps, g_logits, g_dist, g_x, accumulate, ws, grid, stream)
                 : fused_t<TX, kA, kG, true, 0>(g, x, blk, eps, g_logits, g_dist, g_x, accumulate, ws, grid, stream);
    return six ? fused_t<TX, kA, kG, false, 6>(g, x, blk, eps, g_logits, g_dist, g_x, accumulate, ws, grid, stream)
               : fused_t<TX, kA, kG, false, 0>(g, x, blk, eps, g_logits, g_dist, g_x, accumulate, ws, grid, stream);
  };
  using A0 = std::integral_constant<int, 0>;
  using A1 = std::integral_constant<int, 1>;
  using GT = std::integral_constant<int, 1>;
  using GF = std::integral_constant<int, 0>;
  using GC = std::integral_constant<int, 2>;
  float* f = nullptr;
  uint16_t* b = nullptr;
  int st;
  if (g.cgd.val) {  // the compact KLD gradient: f32 x only
    if (x_bf16 || g_dist) return fail(PROTOSEG_ERR_UNSUPPORTED, "compact g_dist: f32 x and no dense g_dist");
    st = act_kind == 0 ? go(f, A0(), GC()) : go(f, A1(), GC());
  } else if (act_kind == 0)
    st = x_bf16 ? (g_dist ? go(b, A0(), GT()) : go(b, A0(), GF())) : (g_dist ? go(f, A0(), GT()) : go(f, A0(), GF()));
  else
    st = x_bf16 ? (g_dist ? go(b, A1(), GT()) : go(b, A1(), GF())) : (g_dist ? go(f, A1(), GT()) : go(f, A1(), GF()));
  if (st || !reduce) return st;
  return launch_bwd_reduce_bf16(g, ws, grid, protos, act_kind, g_protos, g_logits ? g_w : nullptr, stream);
}

}  // namespace protoseg

#ifdef PROTOSEG_STAMPS
// Debug builds only: copy (and clear) the fused kernel's per-wave phase stamps.
extern "C" int protoseg_debug_stamps_fused(void* dst, size_t bytes) {
  using protoseg::g_stamps_fused;
  const size_t n = bytes < sizeof(g_stamps_fused) ? bytes : sizeof(g_stamps_fused);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  if (dst && hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_stamps_fused), n, 0, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_stamps_fused)) != hipSuccess) return 3;
  return hipMemset(p, 0, sizeof(g_stamps_fused)) == hipSuccess ? 0 : 3;
}
#endif
