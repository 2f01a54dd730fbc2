// push.hip — prototype push (nearest-patch projection) on gfx950.
//
// Reference: segmentation/push.py:24-158 (push_prototypes) and 162-280
// (update_prototypes_on_image, argmin core). The reference moves the distance map of every
// image to the host and runs (a) a 2M-iteration Python loop mapping pixels to patch sets,
// (b) a per-prototype gather + np.argmin. Here both stay on the device:
//   patch_mask_kernel   label map -> uint32 class bitmask per patch (push.py:184-186, 214-223)
//   push_argmin_wave_kernel  fused distance (bf16x6 products, C = 32 / 64) + masked per-prototype
//                       top-2 keys (push.py:249-263); push_argmin_kernel the same for C = 128 (f32)
//   push_top2_kernel    folds the pixel stripes' partial top-2
//   push_merge_kernel   strict-'<' fold in image order + winner gather (push.py:265-281)
//   push_top2_merge_kernel  the two above in one launch (protoseg_push_update, native path)
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "bf16_split.h"
#include "l2_bf16_common.h"
#include "protoseg_device.h"
#include "protoseg_host.h"
#include "l2_launch.h"

namespace protoseg {

namespace {

// Up to 512 threads x 4 columns: for a call of few images a Cityscapes patch row (2048 columns)
// in one pass, so the 129 workgroups of a 1-image call do not each walk the row twice (9.2 -> 7.3
// us); at 4+ images 256 threads (more workgroups resident: 14.5 vs 16.0 us at 8 images)
constexpr int kMaskThreads = 512;
template <typename TL>
__global__ __launch_bounds__(kMaskThreads) void patch_mask_kernel(const TL* __restrict__ label, int H, int W, int h, int w,
                                                         const int32_t* __restrict__ lut, int lut_size,
                                                         int base, uint32_t* __restrict__ mask) {
  // base: this mask word's first class (32 per word; classes base+1 .. base+32 -> bits 0 .. 31)
  extern __shared__ uint32_t smask[];  // [w]
  const int pi = blockIdx.x;
  const int img = blockIdx.y;
  // push.py:201-202: patch_height = img_height / model_output_height (float64)
  const double ph = static_cast<double>(H) / static_cast<double>(h);
  const double pw = static_cast<double>(W) / static_cast<double>(w);
  for (int q = threadIdx.x; q < w; q += blockDim.x) smask[q] = 0u;
  __syncthreads();
  // Rows of this patch row: push.py:217 patch_i = int(pixel_i / patch_height). int(i / ph) is
  // non-decreasing in i, so they are the contiguous run [r0, r1) found once (f64 divisions per
  // candidate row, not per row and column).
  int i0 = static_cast<int>(floor(pi * ph)) - 2;
  int i1 = static_cast<int>(ceil((pi + 1) * ph)) + 2;
  i0 = i0 < 0 ? 0 : i0;
  i1 = i1 > H ? H : i1;
  int r0 = i1, r1 = i1;
  for (int i = i0; i < i1; ++i) {
    const int q = static_cast<int>(static_cast<double>(i) / ph);
    if (q == pi && r0 == i1) r0 = i;
    if (q > pi) {
      r1 = i;
      break;
    }
  }
  const TL* L = label + static_cast<size_t>(img) * H * W;
  // 4 consecutive columns per thread (one 4-byte load per row for u8 labels); columns of one
  // patch are OR-ed in registers, so LDS atomics go once per (thread, patch), not per column
  const bool vec4 = sizeof(TL) == 1 && (W & 3) == 0 && (reinterpret_cast<uintptr_t>(label) & 3) == 0;
  auto cls_bit = [&](long long raw) -> uint32_t {
    long long c = raw;
    if (lut) {
      if (raw < 0 || raw >= lut_size) return 0u;
      c = lut[raw];
    }
    return (c > base && c <= base + 32) ? 1u << (c - 1 - base) : 0u;  // push.py:222-223: class c -> key c-1
  };
  for (int c0 = 4 * static_cast<int>(threadIdx.x); c0 < W; c0 += 4 * static_cast<int>(blockDim.x)) {
    uint32_t b4[4] = {0u, 0u, 0u, 0u};
    const int nc = W - c0 < 4 ? W - c0 : 4;
    if (vec4) {  // the patch row's label rows 8 at a time: 8 loads in flight, not one per round trip
      for (int i = r0; i < r1; i += 8) {
        uint32_t q[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)  // clamped rows, pinned (pin_batch); rows past r1 are not OR-ed
          q[u] = *reinterpret_cast<const uint32_t*>(L + static_cast<size_t>(i + u < r1 ? i + u : r1 - 1) * W + c0);
        pin_batch(q);
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (i + u < r1)
#pragma unroll
            for (int k = 0; k < 4; ++k) b4[k] |= cls_bit(static_cast<long long>((q[u] >> (8 * k)) & 0xffu));
      }
    }
    for (int i = vec4 ? r1 : r0; i < r1; ++i) {
      const TL* row = L + static_cast<size_t>(i) * W + c0;
      {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (k < nc) b4[k] |= cls_bit(static_cast<long long>(row[k]));
      }
    }
    int cur = -1;
    uint32_t acc = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k >= nc) break;
      const int pj = static_cast<int>(static_cast<double>(c0 + k) / pw);  // push.py:219
      if (pj != cur) {
        if (acc && cur >= 0 && cur < w) atomicOr(&smask[cur], acc);
        cur = pj;
        acc = 0u;
      }
      acc |= b4[k];
    }
    if (acc && cur >= 0 && cur < w) atomicOr(&smask[cur], acc);
  }
  __syncthreads();
  for (int q = threadIdx.x; q < w; q += blockDim.x)
    mask[static_cast<size_t>(img) * h * w + static_cast<size_t>(pi) * w + q] = smask[q];
}

// push_argmin_kernel: one workgroup per (pixel-block stripe, image, chunk of up to 8 prototype
// tiles of 32). The image's pixels are walked in blocks of kPushBlk 32-pixel tiles; each block's
// x ([C][128] of the NCHW map) is read from HBM ONCE, by LDS-DMA (buffer_load_dword ... lds,
// no registers) into one of two LDS buffers, so block b + 1 streams in while block b is
// computed. Wave w of the workgroup owns prototype tile w % nptc (its 32 prototypes' vectors in
// registers) and the pixel tiles tt = w / nptc, w / nptc + split, ... of every block, so all
// 4 SIMDs carry the same MFMA load (P = 190: 6 tiles x 2 = 12 waves).
// Layout B (pixel on the accumulator rows, prototype on the lane): A = x from LDS, lane (j, h)
// reads channels 32 ct + 16 h + r of pixel j (LDS rows of XS = 130 floats: the two half-waves
// land 32 banks apart, conflict-free); B = the same channels of prototype j; the products run
// on v_mfma_f32_32x32x2_f32, an exact f32 fma chain. ||x||^2 comes from the same A values
// (fma chain per half, then the two halves added), so every prototype tile sees the same value.
// Per lane, the smallest distance of its prototype over its rows with its patch, and the
// runner-up distance, are kept; as keys float_bits(d) << 32 | patch (d >= 0 after relu, so the
// bits order like d; equal distances resolve to the lower patch; the runner-up's patch bits are
// all ones) the half-waves merge and each (stripe, part) writes a partial top-2 that
// push_top2_kernel folds. The runner-up distance lets the host flag near-ties (SURVEY.md §7,
// hard part 2).
#ifndef PUSH_BLK
#define PUSH_BLK 4
#endif
constexpr int kPushBlk = PUSH_BLK;          // 32-pixel tiles per staged block
constexpr int kPushBlkPix = kPushBlk * 32;  // 128 pixels (at 4 tiles)
constexpr int kPushXS = kPushBlkPix + 2;    // LDS row stride (floats): 16 * XS = 32 (mod 64) banks
constexpr int kPushMaxTiles = 8;            // prototype tiles per chunk
#ifndef PUSH_SPLIT
#define PUSH_SPLIT 2
#endif
#ifndef PUSH_WG_TARGET
#define PUSH_WG_TARGET 256
#endif
constexpr int kPushSplit = PUSH_SPLIT;      // waves per prototype tile (pixel tiles split)

// LDS: 2 buffers of [C rows x XS] x + [128] patch class masks, then [waves][64] per-wave rows.
__host__ __device__ inline int push_buf_floats(int C) { return C * kPushXS + kPushBlkPix; }
__host__ __device__ inline size_t push_lds_bytes(int C, int waves) {
  return static_cast<size_t>(2) * push_buf_floats(C) * 4 + static_cast<size_t>(waves) * 128 * 4;
}

// (b1, s1) and (b2, s2), each b <= s: the two smallest of the four. A best key that becomes the
// runner-up drops its patch (bits all ones), like every runner-up key: only its distance counts.
__device__ __forceinline__ void top2_merge(unsigned long long& b, unsigned long long& s, unsigned long long b2,
                                           unsigned long long s2) {
  const unsigned long long lo = b < b2 ? b : b2, hi = (b < b2 ? b2 : b) | 0xffffffffull;
  const unsigned long long sm = s < s2 ? s : s2;
  b = lo;
  s = hi < sm ? hi : sm;
}

template <int NC>
__global__ __launch_bounds__(kPushMaxTiles * kPushSplit * 64) void push_argmin_kernel(
    const float* __restrict__ x, int HW, const float* __restrict__ protos, int P, int pt0, int nptc,
    const int32_t* __restrict__ proto_class, const uint32_t* __restrict__ mask,
    unsigned long long* __restrict__ part, int stripes) {
  using namespace bf16l;
  constexpr int C = NC * 32;
  extern __shared__ __attribute__((aligned(16))) float push_smem[];
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5, wave = wave_id();
  const int nw = blockDim.x >> 6;
  const int ptl = wave % nptc, sub = wave / nptc;  // prototype tile in the chunk, pixel-tile part
  const int stripe = blockIdx.x, img = blockIdx.y;
  // this wave's epilogue rows, two tiles: [32] ||x||^2, [32] class masks (as float bits) each
  float* xw = push_smem + 2 * push_buf_floats(C) + wave * 128;
  const int p = (pt0 + static_cast<int>(blockIdx.z) * nptc + ptl) * 32 + j;  // chunk z of nptc tiles
  const bool pvalid = p < P;
  // this lane's B fragments: prototype p, channels 32 ct + 16 h .. + 15 (four 16-B loads per
  // group; lanes past P read row P - 1 and are masked out below)
  float pv[NC][16];
  const float4* prow = reinterpret_cast<const float4*>(protos + static_cast<size_t>(pvalid ? p : P - 1) * C + 16 * h);
#pragma unroll
  for (int ct = 0; ct < NC; ++ct)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 v = prow[ct * 8 + q];
      pv[ct][4 * q] = v.x;
      pv[ct][4 * q + 1] = v.y;
      pv[ct][4 * q + 2] = v.z;
      pv[ct][4 * q + 3] = v.w;
    }
  // ||p||^2 from the same registers: an fma chain over this half's channels, then the two halves
  // added (the sum is the same in both halves). Also consumes the loads before the loop, so the
  // compiler's own vmcnt wait for them does not land at the first MFMA, where it would also wait
  // for the LDS-DMA prefetch of the next block (inline asm the wait-count pass cannot see).
  float p2 = 0.f;
#pragma unroll
  for (int ct = 0; ct < NC; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r) p2 = fmaf(pv[ct][r], pv[ct][r], p2);
  p2 += __shfl_xor(p2, 32);
  const int cls = pvalid ? proto_class[p] : -1;
  const bool active = cls >= 0 && cls < 32;
  const uint32_t wave_classes = wave_or(active ? (1u << cls) : 0u);
  const rsrc_t rx = make_rsrc(x + static_cast<size_t>(img) * C * HW, static_cast<unsigned>(C * HW * 4));
  const rsrc_t rm = make_rsrc(mask + static_cast<size_t>(img) * HW, static_cast<unsigned>(HW * 4));

  // block blk -> LDS buffer sb: row c = channel c, 128 pixels, then the 128 patch masks (2 DMA
  // wave-instructions per row; pixels past the map land as 0), spread over the workgroup's waves
  auto stage = [&](int blk, int sb) __attribute__((always_inline)) {
    float* X = push_smem + sb * push_buf_floats(C);
    const int n0 = blk * kPushBlkPix;
    for (int i = wave; i < 2 * C + 2; i += nw) {
      const int c = i >> 1, half = i & 1;
      const int n = n0 + 64 * half + lane;
      if (c < C)
        dma<float>(rx, X + c * kPushXS + 64 * half, n < HW ? static_cast<unsigned>((c * HW + n) * 4) : kOOB, 0u);
      else
        dma<float>(rm, X + C * kPushXS + 64 * half, n < HW ? static_cast<unsigned>(n * 4) : kOOB, 0u);
    }
  };

  // per lane: best distance and its patch, runner-up distance (candidates arrive in increasing
  // patch order, so a strict '<' keeps the lowest patch among equal distances)
  float bd = __builtin_inff(), sd = __builtin_inff();
  uint32_t bi = 0xffffffffu;
  const uint32_t clsbit = active ? (1u << cls) : 0u;
  // one tile's A fragments from LDS -> distances accumulator + ||x||^2 (fma chain per half,
  // halves added), staged with the tile's masks into this wave's rows for the epilogue
  auto mfma_tile = [&](const float* X, int tt, f32x16& acc, float* rows) __attribute__((always_inline)) {
    acc = zero16();
    float x2 = 0.f;
#pragma unroll
    for (int ct = 0; ct < NC; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float xa = X[(ct * 32 + 16 * h + r) * kPushXS + tt * 32 + j];
        x2 = fmaf(xa, xa, x2);
        acc = mfma32(xa, pv[ct][r], acc);
      }
    x2 += __shfl_xor(x2, 32);
    if (h == 0) rows[j] = x2;
  };
  auto epilogue = [&](const f32x16& acc, const float* rows, int nbase) __attribute__((always_inline)) {
    float x2r[16], mkr[16];
    load_rows16(rows + 4 * h, x2r);
    load_rows16(rows + 32 + 4 * h, mkr);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float d = l2_distance(x2r[r], p2, acc[r]);
      const float dm = (__float_as_uint(mkr[r]) & clsbit) ? d : __builtin_inff();  // outside the class: absent
      const bool c = dm < bd;
      sd = c ? bd : fminf(sd, dm);
      bi = c ? static_cast<uint32_t>(nbase + acc_row(r, h)) : bi;
      bd = c ? dm : bd;
    }
  };

  const int nblk = (HW + kPushBlkPix - 1) / kPushBlkPix;
  int sb = 0;
  if (stripe < nblk) stage(stripe, 0);
  for (int blk = stripe; blk < nblk; blk += stripes, sb ^= 1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of block blk
    __syncthreads();  // every wave's DMA of blk landed; block blk - stripes fully consumed
#ifndef PUSH_NO_DMA
    if (blk + stripes < nblk) stage(blk + stripes, sb ^ 1);
#endif
    if (wave_classes == 0u) continue;  // no prototype of this wave is pushed (wave-uniform)
    const float* X = push_smem + sb * push_buf_floats(C);
    const uint32_t* MK = reinterpret_cast<const uint32_t*>(X + C * kPushXS);
    const int n0 = blk * kPushBlkPix;
    // this wave's tiles in pairs: both tiles' MFMA chains are issued before the first tile's
    // epilogue, so the epilogue's VALU work overlaps the second chain in the MFMA pipe
#pragma unroll 1
    for (int ta = sub; ta < kPushBlk; ta += 2 * kPushSplit) {
      const int tb = ta + kPushSplit;
      const uint32_t mka = MK[ta * 32 + j];
      const uint32_t mkb = tb < kPushBlk ? MK[tb * 32 + j] : 0u;
      // tiles holding no patch of any class of this wave's prototypes are skipped
      const bool run_a = __ballot((mka & wave_classes) != 0u) != 0ull;
      const bool run_b = __ballot((mkb & wave_classes) != 0u) != 0ull;
      if (h == 0) {
        xw[32 + j] = __uint_as_float(mka);
        xw[96 + j] = __uint_as_float(mkb);
      }
      f32x16 acc_a, acc_b;
      if (run_a) mfma_tile(X, ta, acc_a, xw);
      if (run_b) mfma_tile(X, tb, acc_b, xw + 64);
      wave_lds_fence();
#ifndef PUSH_NO_EPI
      if (run_a) epilogue(acc_a, xw, n0 + ta * 32);
      if (run_b) epilogue(acc_b, xw + 64, n0 + tb * 32);
#endif
      wave_lds_fence();  // the row reads are done before the next pair rewrites them
    }
  }
  unsigned long long best = bd == __builtin_inff() ? ~0ull : (static_cast<unsigned long long>(__float_as_uint(bd)) << 32) | bi;
  unsigned long long second = sd == __builtin_inff() ? ~0ull : (static_cast<unsigned long long>(__float_as_uint(sd)) << 32) | 0xffffffffu;
  top2_merge(best, second, shfl_xor_u64(best, 32), shfl_xor_u64(second, 32));
  if (h == 0 && pvalid) {
    unsigned long long* o = part + ((static_cast<size_t>(img) * stripes * kPushSplit + stripe * kPushSplit + sub) * P + p) * 2;
    o[0] = best;
    o[1] = second;
  }
}

// ---- push distances on bf16 MFMA with exact three-term splits (bf16x6), C = 32 / 64 ---------
// Each f32 operand is split exactly into three bf16 terms (8 + 8 + 8 significant bits), and a
// product x.p is the sum of the six largest cross products (the three dropped ones are below
// 2^-24 relative): f32-class distances, as the f32 fma chain's, at 2.7x the v_mfma_f32_32x32x2_f32
// rate (6 v_mfma_f32_32x32x16_bf16 of 32 cycles per 16 channels, against 8 of 64). Layout B of
// the f32 kernel (rows = pixels, columns = prototypes); k-step s (16 channels) of lane half h
// holds channels push_chan(s, h, 0..7) = 32 (s >> 1) + 16 h + 8 (s & 1) + e, which are the
// channels a lane's x registers hold (xr[16 ct + r] = x[32 ct + 16 h + r]). push_dist_kernel forms
// the same products in the same order, so a tie is exactly a tie the argmin saw.
__device__ __forceinline__ constexpr int push_chan(int s, int h, int e) { return 32 * (s >> 1) + 16 * h + 8 * (s & 1) + e; }
// the x registers of a pixel tile -> the A fragments of the 2 NC k-steps (3 terms each)
template <int NC>
__device__ __forceinline__ void push_split_x(const float (&xr)[NC * 16], bf16x8 (&af)[2 * NC][3]) {
#pragma unroll
  for (int s = 0; s < 2 * NC; ++s) {
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = xr[16 * (s >> 1) + 8 * (s & 1) + e];
    split8<3>(v, af[s]);
  }
}
// (x || p)^T products of one prototype tile, k-steps in order, terms smallest first (mma_split<3>)
template <int NC>
__device__ __forceinline__ f32x16 push_xp(const bf16x8 (&af)[2 * NC][3], const bf16x8 (&bf)[2 * NC][3]) {
  f32x16 acc = zero16();
#pragma unroll
  for (int s = 0; s < 2 * NC; ++s) acc = mma_split<3>(af[s], bf[s], acc);
  return acc;
}
// ||p||^2 of prototype row pr (f32, C = 32 NC) in the lane half's fixed order, halves added: the
// value every push distance of the row uses
template <int NC>
__device__ __forceinline__ float push_p2(const float* __restrict__ pr, int h) {
  float s = 0.f;
#pragma unroll
  for (int ct = 0; ct < NC; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r) s = fmaf(pr[ct * 32 + 16 * h + r], pr[ct * 32 + 16 * h + r], s);
  return s + __shfl_xor(s, 32);
}

// Wave-streamed push argmin (C = 32 / 64): every wave owns whole 32-pixel tiles of one image and
// runs ALL of the launch chunk's prototype tiles on each, so the pixel loop has no workgroup
// barrier. The tile's x comes straight from HBM into registers (lane (j, h): x[ct * 32 + 16 h + r]
// [pixel j], one tile prefetched ahead) and is split once per tile into the bf16x6 A fragments;
// the chunk's prototype rows sit in LDS for the launch as three bf16 term images (one barrier
// after the prologue) and are read per prototype tile as the B fragments, two tiles' products
// interleaved on independent accumulators. Same arithmetic as push_dist_kernel (push_xp, the
// fma chains of ||x||^2 and push_p2), so ties are the ties protoseg_push_distances shows. The workgroup's waves merge their top-2
// keys in LDS at the end (order-free: min of keys), one partial per (workgroup, image).
#ifndef PW_WAVES
#define PW_WAVES 8
#endif
constexpr int kPwWaves = PW_WAVES;  // waves per workgroup (8: two per SIMD, the next tile's x prefetched; 12: three, no prefetch)
constexpr bool kPwPrefetch = kPwWaves <= 8;
constexpr int kPwMaxTiles = 8;  // prototype tiles per launch chunk (C = 32 / 64; C = 128 runs the block kernel)
__host__ __device__ inline int pw_max_tiles(int) { return kPwMaxTiles; }
// prototype rows in LDS as three bf16 term images [3][nptc * 32 rows][C], 16-B chunk ch of row r
// at chunk ch ^ swz<C / 8>(r) (the 16-lane groups of a ds_read_b128 of 16 rows land on distinct
// banks, bf16_split.h)
__host__ __device__ inline size_t pw_term_bytes(int C, int nptc) { return static_cast<size_t>(nptc) * 32 * C * 2; }
__host__ __device__ inline size_t pw_lds_bytes(int C, int nptc) {
  // term images + per prototype of the chunk: ||p||^2, the caller's bound, the class bit
  const size_t protos = 3 * pw_term_bytes(C, nptc) + static_cast<size_t>(3) * nptc * 32 * 4;
  const size_t merge = static_cast<size_t>(kPwWaves) * nptc * 32 * 16;
  return (protos > merge ? protos : merge) + static_cast<size_t>(kPwWaves) * 64 * 4;
}

// Launch plan of the wave-streamed kernel: the prototype tiles go in chunks of `per` (one
// launch's blockIdx.z; a remainder chunk is a second launch), each (image, chunk) over `wgs`
// workgroups of kPwWaves waves, one workgroup per CU resident (176 / 208 VGPRs: 2 waves per
// SIMD). A wave's work is ceil(ntile / (wgs waves)) pixel tiles x per prototype tiles, plus about
// one tile-pass of prologue (its rows into LDS, ||p||^2, the final merge), times the generations
// the launch needs. The plan minimises that over the launches with at most kPwMaxChunks chunks
// (each chunk reads x again); ties go to wider chunks. One Cityscapes image (1036 tiles, P = 190)
// thus runs 3 chunks of 2 tiles on 255 workgroups instead of 1 chunk of 6 on 130, which left
// half the CUs idle.
#ifndef PUSH_CHUNK_PLAN
#define PUSH_CHUNK_PLAN 1
#endif
#ifndef PUSH_MAX_CHUNKS
#define PUSH_MAX_CHUNKS 3  // (development A/B of the plan: tools/build_var.sh ... -DPUSH_MAX_CHUNKS=n)
#endif
constexpr int kPwMaxChunks = PUSH_MAX_CHUNKS;
struct PushPlan {
  int per;
  long long wgs;
};
inline PushPlan push_wave_plan(int npt, int maxt, int n_img, long long ntile, int cus) {
  const long long wmax = (ntile + kPwWaves - 1) / kPwWaves;
  const long long slots = static_cast<long long>(cus) * (kPwWaves < 8 ? 8 / kPwWaves : 1);  // 8 waves per CU
  auto fit_w = [&](int chunks) {  // workgroups per (image, chunk) for one generation
    long long w = slots / (static_cast<long long>(n_img) * chunks);
    return w < 1 ? 1 : w > wmax ? wmax : w;
  };
  auto cost = [&](int chunks, int per, long long w) {
    const long long rounds = (ntile + w * kPwWaves - 1) / (w * kPwWaves);
    const long long gens = (static_cast<long long>(n_img) * chunks * w + slots - 1) / slots;
    return gens * (rounds * per + 1);
  };
  PushPlan best{npt < maxt ? npt : maxt, 1};
  long long best_cost = -1;
  for (int per = maxt < npt ? maxt : npt; per >= 1; --per) {
    const int full = npt / per, rem = npt - full * per;
    if (per < npt && full + (rem ? 1 : 0) > kPwMaxChunks) continue;
    long long w = fit_w(full);
    if (rem) {
      const long long wr = fit_w(1);
      w = wr < w ? wr : w;  // one wgs for both launches (the partials' layout)
    }
    const long long c = cost(full, per, w) + (rem ? cost(1, rem, w) : 0);
    if (best_cost < 0 || c < best_cost) {
      best_cost = c;
      best = {per, w};
    }
  }
  return best;
}

template <int NC>
__global__ __launch_bounds__(kPwWaves * 64) void push_argmin_wave_kernel(
    const float* __restrict__ x, int HW, const float* __restrict__ protos, int P, int pt0, int nptc,
    const int32_t* __restrict__ proto_class, const uint32_t* __restrict__ mask,
    unsigned long long* __restrict__ part, int wgs, const float* __restrict__ sd0) {
  using namespace bf16l;
  constexpr int C = NC * 32;
  extern __shared__ __attribute__((aligned(16))) float pw_smem[];
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5, wave = wave_id();
  const int wgi = blockIdx.x, img = blockIdx.y;
  const int pbase = (pt0 + static_cast<int>(blockIdx.z) * nptc) * 32;  // chunk z of nptc tiles
  constexpr int kCpr = C / 8;  // 16-B chunks per bf16 row
  bf16* PL = reinterpret_cast<bf16*>(pw_smem);               // [3][nptc * 32][C] bf16 terms
  const int term_elems = nptc * 32 * C;
  const size_t region = pw_lds_bytes(C, nptc) / 4 - kPwWaves * 64;
  float* xw = pw_smem + region + wave * 64;  // this wave's rows: [32] ||x||^2, [32] class masks
  for (int i = static_cast<int>(threadIdx.x); i < nptc * 32 * kCpr; i += kPwWaves * 64) {
    const int row = i / kCpr, ch = i - row * kCpr;
    const bool ok = pbase + row < P;
    const float4* src = reinterpret_cast<const float4*>(protos + static_cast<size_t>(ok ? pbase + row : 0) * C + 8 * ch);
    const float4 u = src[0], w = src[1];
    float v[8] = {u.x, u.y, u.z, u.w, w.x, w.y, w.z, w.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = ok ? v[e] : 0.f;
    bf16x8 f[3];
    split8<3>(v, f);
    const int o = row * C + 8 * (ch ^ swz<kCpr>(row));
#pragma unroll
    for (int t = 0; t < 3; ++t) *reinterpret_cast<bf16x8*>(PL + t * term_elems + o) = f[t];
  }
  // per prototype of the chunk, in LDS (read per prototype tile in the epilogue, not held in
  // registers): ||p||^2 (push_p2: the fixed order of every push distance), the caller's bound
  // (see bd / sd below) and the class bit; the wave's OR of each tile's classes in scalar registers
  float* pv_p2 = reinterpret_cast<float*>(PL + 3 * term_elems);
  float* pv_bnd = pv_p2 + nptc * 32;
  uint32_t* pv_cls = reinterpret_cast<uint32_t*>(pv_bnd + nptc * 32);
  uint32_t tcls[kPwMaxTiles];
#pragma unroll
  for (int pt = 0; pt < kPwMaxTiles; ++pt) {
    tcls[pt] = 0u;
    if (pt < nptc) {
      const int p = pbase + pt * 32 + j;
      const float p2v = p < P ? push_p2<NC>(protos + static_cast<size_t>(p) * C, h) : 0.f;
      const int cls = p < P ? proto_class[p] : -1;
      const uint32_t cb = cls >= 0 && cls < 32 ? (1u << cls) : 0u;
      tcls[pt] = __builtin_amdgcn_readfirstlane(wave_or(cb));  // uniform: scalar registers
      if (wave == 0 && h == 0) {
        pv_p2[pt * 32 + j] = p2v;
        pv_bnd[pt * 32 + j] = sd0 && p < P ? sd0[p] : __builtin_inff();
        pv_cls[pt * 32 + j] = cb;
      }
    }
  }
  __syncthreads();
  const rsrc_t rx = make_rsrc(x + static_cast<size_t>(img) * C * HW, static_cast<unsigned>(C * HW * 4));
  const rsrc_t rm = make_rsrc(mask + static_cast<size_t>(img) * HW, static_cast<unsigned>(HW * 4));
  const int ntile = (HW + 31) / 32, nw = wgs * kPwWaves;
  // tile t's A operand: xr[ct * 16 + r] = x[ct * 32 + 16 h + r][32 t + j] (0 past the map)
  auto load_x = [&](int t, float (&xr)[NC * 16]) __attribute__((always_inline)) {
    const int n = t * 32 + j;
    const unsigned off = t < ntile && n < HW ? static_cast<unsigned>(((16 * h) * HW + n) * 4) : kOOB;
#pragma unroll
    for (int ct = 0; ct < NC; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        xr[ct * 16 + r] = BufIO<float>::load(rx, off, static_cast<unsigned>((ct * 32 + r) * HW * 4));
  };
  // bnd: the caller's bound (protoseg_push_update: the running runner-up distance before this
  // call, sd0[p]) or +inf. A candidate d >= min(sd, bnd) changes neither this lane's top-2 below
  // bnd nor the merged state (it cannot become the running best, best <= runner-up <= bnd, nor
  // lower the runner-up), so the epilogue skips a prototype tile whose candidates are all above
  // that threshold in every lane: two VALU per candidate instead of the ~12 of the masked update.
  // The per-image top-2 below bnd is then exact, above it partial (only the merge reads it).
  float bd[kPwMaxTiles], sd[kPwMaxTiles];
  uint32_t bi[kPwMaxTiles];
#pragma unroll
  for (int pt = 0; pt < kPwMaxTiles; ++pt) {
    bd[pt] = sd[pt] = __builtin_inff();
    bi[pt] = 0xffffffffu;
  }
  // one prototype tile's B fragments of k-step s (prototype j, channels push_chan(s, h, 0..7))
  auto load_pf = [&](int pt, int s, bf16x8 (&bf)[3]) __attribute__((always_inline)) {
    const int row = pt * 32 + j;
    const int o = row * C + 8 * ((push_chan(s, h, 0) >> 3) ^ swz<kCpr>(row));
#pragma unroll
    for (int t = 0; t < 3; ++t) bf[t] = *reinterpret_cast<const bf16x8*>(PL + t * term_elems + o);
  };
  // per lane (prototype j of tile pt): the tile's rows (pixels) in increasing order, strict '<'
  auto epilogue = [&](int pt, const f32x16& acc, int nbase) __attribute__((always_inline)) {
    float x2r[16], mkr[16];  // (re-read per prototype tile: not held across the MFMA chain)
    load_rows16(xw + 4 * h, x2r);
    float s[16];  // l2_distance before its relu: relu(s) < thr implies s < thr (thr >= 0)
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = l2_pre_relu(x2r[r], pv_p2[pt * 32 + j], acc[r]);
    float m4[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) m4[q] = fminf(fminf(s[4 * q], s[4 * q + 1]), fminf(s[4 * q + 2], s[4 * q + 3]));
    const float thr = fminf(sd[pt], pv_bnd[pt * 32 + j]);
    if (!__builtin_amdgcn_ballot_w64(fminf(fminf(m4[0], m4[1]), fminf(m4[2], m4[3])) < thr))
      return;  // no candidate below any lane's threshold: nothing changes (wave-uniform)
    load_rows16(xw + 32 + 4 * h, mkr);
    const uint32_t clsb = pv_cls[pt * 32 + j];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float d = __builtin_fmaxf(s[r], 0.f);  // = l2_distance(x2r[r], p2[pt], acc[r])
      const float dm = (__float_as_uint(mkr[r]) & clsb) ? d : __builtin_inff();
      const bool c = dm < bd[pt];
      sd[pt] = c ? bd[pt] : fminf(sd[pt], dm);
      bi[pt] = c ? static_cast<uint32_t>(nbase + acc_row(r, h)) : bi[pt];
      bd[pt] = c ? dm : bd[pt];
    }
  };
  // tile t's patch class mask of pixel j (0 past the map)
  auto load_mk = [&](int t) __attribute__((always_inline)) -> uint32_t {
    return __builtin_amdgcn_raw_buffer_load_b32(
        rm, t < ntile && t * 32 + j < HW ? static_cast<unsigned>((t * 32 + j) * 4) : kOOB, 0, 0);
  };
  int t = wave * wgs + wgi;
  float xr[NC * 16];
  uint32_t mkn = 0u;
  if constexpr (kPwPrefetch) {
    load_x(t, xr);
    mkn = load_mk(t);
  }
#pragma unroll 1
  for (; t < ntile; t += nw) {
    float cur[NC * 16];
    uint32_t mk;
    if constexpr (kPwPrefetch) {
#pragma unroll
      for (int i = 0; i < NC * 16; ++i) cur[i] = xr[i];
      mk = mkn;
      load_x(t + nw, xr);  // the next tile's loads, in flight under this tile's MFMAs
      mkn = load_mk(t + nw);
    } else {
      load_x(t, cur);
      mk = load_mk(t);
    }
    float x2 = 0.f;
#pragma unroll
    for (int i = 0; i < NC * 16; ++i) x2 = fmaf(cur[i], cur[i], x2);
    x2 += __shfl_xor(x2, 32);
    bf16x8 af[2 * NC][3];
    push_split_x<NC>(cur, af);
    wave_lds_fence();  // the previous tile's row reads are done
    if (h == 0) {
      xw[j] = x2;
      xw[32 + j] = __uint_as_float(mk);
    }
    wave_lds_fence();
    const int nbase = t * 32;
    // prototype tiles in pairs: two independent accumulator chains interleaved, each in
    // push_xp's order (k-steps, terms smallest first)
#pragma unroll
    for (int pa = 0; pa < kPwMaxTiles; pa += 2) {
      if (pa >= nptc) break;
      const int pb = pa + 1;
      const bool has_b = pb < nptc;
      // prototype tiles with no patch of their classes in this pixel tile are skipped
      const bool run_a = __ballot((mk & tcls[pa]) != 0u) != 0ull;
      const bool run_b = has_b && __ballot((mk & tcls[pb]) != 0u) != 0ull;
      if (!run_a && !run_b) continue;
      f32x16 acc_a = zero16(), acc_b = zero16();
#pragma unroll
      for (int s2 = 0; s2 < 2 * NC; ++s2) {
        bf16x8 fa[3], fb[3];
        load_pf(pa, s2, fa);
        load_pf(has_b ? pb : pa, s2, fb);
        acc_a = mma_split<3>(af[s2], fa, acc_a);
        acc_b = mma_split<3>(af[s2], fb, acc_b);
      }
      if (run_a) epilogue(pa, acc_a, nbase);
      if (run_b) epilogue(pb, acc_b, nbase);
    }
  }
  // halves, then the workgroup's waves (LDS, after every wave is done with the prototype rows)
  unsigned long long best[kPwMaxTiles], second[kPwMaxTiles];
#pragma unroll
  for (int pt = 0; pt < kPwMaxTiles; ++pt) {
    best[pt] = bd[pt] == __builtin_inff() ? ~0ull : (static_cast<unsigned long long>(__float_as_uint(bd[pt])) << 32) | bi[pt];
    second[pt] = sd[pt] == __builtin_inff() ? ~0ull
                                            : (static_cast<unsigned long long>(__float_as_uint(sd[pt])) << 32) | 0xffffffffu;
    top2_merge(best[pt], second[pt], shfl_xor_u64(best[pt], 32), shfl_xor_u64(second[pt], 32));
  }
  __syncthreads();
  unsigned long long* MK = reinterpret_cast<unsigned long long*>(pw_smem);  // [waves][nptc * 32][2]
  if (h == 0) {
#pragma unroll
    for (int pt = 0; pt < kPwMaxTiles; ++pt) {
      if (pt < nptc) {
        MK[(wave * nptc * 32 + pt * 32 + j) * 2] = best[pt];
        MK[(wave * nptc * 32 + pt * 32 + j) * 2 + 1] = second[pt];
      }
    }
  }
  __syncthreads();
  for (int q = static_cast<int>(threadIdx.x); q < nptc * 32; q += kPwWaves * 64) {
    const int p = pbase + q;
    if (p >= P) continue;
    unsigned long long b = MK[q * 2], s = MK[q * 2 + 1];
    for (int w = 1; w < kPwWaves; ++w) top2_merge(b, s, MK[(w * nptc * 32 + q) * 2], MK[(w * nptc * 32 + q) * 2 + 1]);
    unsigned long long* o = part + ((static_cast<size_t>(img) * wgs + wgi) * P + p) * 2;
    o[0] = b;
    o[1] = s;
  }
}

// Folds the stripes' partial top-2 of each (image, prototype): img_keys = the minimum key,
// img_second (optional) = the runner-up key (another patch), UINT64_MAX when absent.
__global__ __launch_bounds__(256) void push_top2_kernel(const unsigned long long* __restrict__ part, int n_img,
                                                        int stripes, int P, unsigned long long* __restrict__ keys,
                                                        unsigned long long* __restrict__ second) {
  const long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= static_cast<long long>(n_img) * P) return;
  const int img = static_cast<int>(i / P), p = static_cast<int>(i - static_cast<long long>(img) * P);
  unsigned long long b = ~0ull, s = ~0ull;
  const unsigned long long* o = part + (static_cast<size_t>(img) * stripes * P + p) * 2;
  const size_t step = static_cast<size_t>(P) * 2;
  int st = 0;
  for (; st + 8 <= stripes; st += 8) {  // 8 independent loads in flight, then the fold in order
    unsigned long long kb[8], ks[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      kb[u] = o[(st + u) * step];
      ks[u] = o[(st + u) * step + 1];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) top2_merge(b, s, kb[u], ks[u]);
  }
  for (; st < stripes; ++st) top2_merge(b, s, o[st * step], o[st * step + 1]);
  keys[i] = b;
  if (second) second[i] = s;
}

// One wave per prototype: fold the batch's keys in image order (strict '<', push.py:265),
// then copy the winning feature vector (push.py:276-280). With the runner-up keys, the
// running second-smallest distance over every patch seen so far is kept too (near-tie flag).
__global__ __launch_bounds__(256) void push_merge_kernel(const unsigned long long* __restrict__ keys,
                                                         const unsigned long long* __restrict__ keys2, int n_img,
                                                         long long first_img, const float* __restrict__ x, int C,
                                                         int hw, int P, float* __restrict__ gdist,
                                                         float* __restrict__ gsecond, long long* __restrict__ gimg,
                                                         int* __restrict__ gpatch, float* __restrict__ gfmap) {
  const int p = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (p >= P) return;
  float best = gdist[p];
  float sec = gsecond ? gsecond[p] : 0.f;
  int win = -1;
  uint32_t patch = 0;
  for (int img = 0; img < n_img; ++img) {
    const unsigned long long key = keys[static_cast<size_t>(img) * P + p];
    if (key == ~0ull) continue;  // no patch of the prototype's class (push.py:255-256)
    const float d = __uint_as_float(static_cast<uint32_t>(key >> 32));
    if (gsecond) {
      const unsigned long long k2 = keys2[static_cast<size_t>(img) * P + p];
      const float d2 = k2 == ~0ull ? __builtin_inff() : __uint_as_float(static_cast<uint32_t>(k2 >> 32));
      if (d < best)
        sec = best < d2 ? best : d2;
      else
        sec = d < sec ? d : sec;
    }
    if (d < best) {
      best = d;
      win = img;
      patch = static_cast<uint32_t>(key);
    }
  }
  if (lane == 0 && gsecond) gsecond[p] = sec;
  if (win < 0) return;
  if (lane == 0) {
    gdist[p] = best;
    gimg[p] = first_img + win;
    gpatch[p] = static_cast<int>(patch);
  }
  for (int c = lane; c < C; c += 64)
    gfmap[static_cast<size_t>(p) * C + c] = x[(static_cast<size_t>(win) * C + c) * hw + patch];
}

// push_top2_kernel + push_merge_kernel in one launch (protoseg_push_update): one wave per
// prototype folds each image's stripe partials across its lanes (a butterfly of top2_merge: the
// keys are unique per patch, so the fold's result does not depend on its order and equals
// push_top2_kernel's sequential one), then merges the images in order exactly as
// push_merge_kernel does. The images' partials are loaded 8 images at a time (all in flight).
__global__ __launch_bounds__(256) void push_top2_merge_kernel(const unsigned long long* __restrict__ part, int parts,
                                                              int n_img, long long first_img,
                                                              const float* __restrict__ x, int C, int hw, int P,
                                                              float* __restrict__ gdist, float* __restrict__ gsecond,
                                                              long long* __restrict__ gimg, int* __restrict__ gpatch,
                                                              float* __restrict__ gfmap) {
  const int p = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (p >= P) return;  // wave-uniform
  float best = gdist[p];
  float sec = gsecond ? gsecond[p] : 0.f;
  int win = -1;
  uint32_t patch = 0;
  for (int i0 = 0; i0 < n_img; i0 += 8) {
    unsigned long long kb[8], ks[8];
    {  // every image's first partial slot (pt = lane) in one batch: clamped, unconditional loads
       // pinned before the guards select (a guarded load waits on its own: 8 round trips)
      const int pt = lane < parts ? lane : 0;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int iu = i0 + u < n_img ? i0 + u : n_img - 1;
        const unsigned long long* o = part + ((static_cast<size_t>(iu) * parts + pt) * P + p) * 2;
        kb[u] = o[0];
        ks[u] = o[1];
      }
      pin_batch(kb);
      pin_batch(ks);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const bool ok = i0 + u < n_img && lane < parts;
        kb[u] = ok ? kb[u] : ~0ull;
        ks[u] = ok ? ks[u] : ~0ull;
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)  // more than 64 partials per image: the rest (top-2 of a set: order-free)
      if (i0 + u < n_img)
        for (int pt = lane + 64; pt < parts; pt += 64) {
          const unsigned long long* o = part + ((static_cast<size_t>(i0 + u) * parts + pt) * P + p) * 2;
          top2_merge(kb[u], ks[u], o[0], o[1]);
        }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) top2_merge(kb[u], ks[u], shfl_xor_u64(kb[u], m), shfl_xor_u64(ks[u], m));
      const unsigned long long key = kb[u];
      if (i0 + u >= n_img || key == ~0ull) continue;  // no patch of the prototype's class (push.py:255-256)
      const float d = __uint_as_float(static_cast<uint32_t>(key >> 32));
      if (gsecond) {
        const unsigned long long k2 = ks[u];
        const float d2 = k2 == ~0ull ? __builtin_inff() : __uint_as_float(static_cast<uint32_t>(k2 >> 32));
        if (d < best)
          sec = best < d2 ? best : d2;
        else
          sec = d < sec ? d : sec;
      }
      if (d < best) {
        best = d;
        win = i0 + u;
        patch = static_cast<uint32_t>(key);
      }
    }
  }
  if (lane == 0 && gsecond) gsecond[p] = sec;
  if (win < 0) return;
  if (lane == 0) {
    gdist[p] = best;
    gimg[p] = first_img + win;
    gpatch[p] = static_cast<int>(patch);
  }
  for (int c = lane; c < C; c += 64)
    gfmap[static_cast<size_t>(p) * C + c] = x[(static_cast<size_t>(win) * C + c) * hw + patch];
}

// push_dist_kernel: the distances of m (gathered) prototypes at every pixel of one image in
// push_argmin_kernel's arithmetic, operation for operation: the same layout-B MFMA chain
// (A = x channel 32 ct + 16 h + r of pixel j, B = the same channel of prototype j, in the same
// order), the same fma chains for ||x||^2 and ||p||^2 with the halves added, l2_distance. So two
// patches tie here exactly when they tie in the argmin kernel. One wave per (32-pixel tile,
// 32-prototype tile); x is read straight from HBM (a host-side tie resolution, not a hot path).
template <int NC>
__global__ __launch_bounds__(64) void push_dist_kernel(const float* __restrict__ x, int HW,
                                                       const float* __restrict__ protos, int m,
                                                       float* __restrict__ out) {
  constexpr int C = NC * 32;
  __shared__ float xs[32];
  const int lane = threadIdx.x, j = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.x * 32;
  const int p = blockIdx.y * 32 + j;
  const bool pvalid = p < m;
  float pv[NC][16];
  const float4* prow = reinterpret_cast<const float4*>(protos + static_cast<size_t>(pvalid ? p : m - 1) * C + 16 * h);
#pragma unroll
  for (int ct = 0; ct < NC; ++ct)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 v = prow[ct * 8 + q];
      pv[ct][4 * q] = v.x;
      pv[ct][4 * q + 1] = v.y;
      pv[ct][4 * q + 2] = v.z;
      pv[ct][4 * q + 3] = v.w;
    }
  float p2 = 0.f;
#pragma unroll
  for (int ct = 0; ct < NC; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r) p2 = fmaf(pv[ct][r], pv[ct][r], p2);
  p2 += __shfl_xor(p2, 32);
  const int n = n0 + j;
  f32x16 acc = zero16();
  float x2 = 0.f;
  if constexpr (NC <= 2) {  // the wave-streamed argmin's arithmetic (bf16x6 products, push_xp)
    float xr[NC * 16];
#pragma unroll
    for (int ct = 0; ct < NC; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) xr[ct * 16 + r] = n < HW ? x[static_cast<size_t>(ct * 32 + 16 * h + r) * HW + n] : 0.f;
#pragma unroll
    for (int i = 0; i < NC * 16; ++i) x2 = fmaf(xr[i], xr[i], x2);
    bf16x8 af[2 * NC][3], bf[2 * NC][3];
    push_split_x<NC>(xr, af);
#pragma unroll
    for (int s = 0; s < 2 * NC; ++s) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = pv[(s >> 1)][8 * (s & 1) + e];  // channel push_chan(s, h, e)
      split8<3>(v, bf[s]);
    }
    acc = push_xp<NC>(af, bf);
    p2 = push_p2<NC>(protos + static_cast<size_t>(pvalid ? p : m - 1) * C, h);
  } else {  // C = 128: the block kernel's exact f32 fma chain
#pragma unroll
    for (int ct = 0; ct < NC; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float xa = n < HW ? x[static_cast<size_t>(ct * 32 + 16 * h + r) * HW + n] : 0.f;
        x2 = fmaf(xa, xa, x2);
        acc = mfma32(xa, pv[ct][r], acc);
      }
  }
  x2 += __shfl_xor(x2, 32);
  if (h == 0) xs[j] = x2;
  __syncthreads();
  if (!pvalid) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = acc_row(r, h);
    if (n0 + row < HW) out[static_cast<size_t>(p) * HW + n0 + row] = l2_distance(xs[row], p2, acc[r]);
  }
}

int nc_of_push(int C) { return C == 32 ? 1 : C == 64 ? 2 : C == 128 ? 4 : 0; }

}  // namespace

}  // namespace protoseg

using namespace protoseg;

extern "C" int protoseg_patch_class_mask(const void* label, int label_dtype, int n_img, int H_img, int W_img, int h,
                                         int w, const int32_t* lut, int lut_size, uint32_t* mask,
                                         protoseg_stream_t stream) {
  return protoseg_patch_class_mask_words(label, label_dtype, n_img, H_img, W_img, h, w, lut, lut_size, 1, mask, stream);
}

extern "C" int protoseg_patch_class_mask_words(const void* label, int label_dtype, int n_img, int H_img, int W_img,
                                               int h, int w, const int32_t* lut, int lut_size, int words,
                                               uint32_t* mask, protoseg_stream_t stream) {
  if (words < 1 || words > 64) return fail(PROTOSEG_ERR_INVALID, "words=%d outside [1, 64]", words);
  if (!label || !mask) return fail(PROTOSEG_ERR_INVALID, "label and mask must be non-null");
  if (n_img <= 0 || H_img <= 0 || W_img <= 0 || h <= 0 || w <= 0)
    return fail(PROTOSEG_ERR_INVALID, "bad shape n_img=%d H=%d W=%d h=%d w=%d", n_img, H_img, W_img, h, w);
  if (lut && lut_size <= 0) return fail(PROTOSEG_ERR_INVALID, "lut_size must be > 0");
  if (static_cast<size_t>(w) * 4 > kMaxLds) return fail(PROTOSEG_ERR_UNSUPPORTED, "w=%d too wide", w);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid(h, n_img);
  const int mt = n_img >= 4 ? 256 : kMaskThreads;
  const size_t lds = static_cast<size_t>(w) * sizeof(uint32_t);
  for (int wd = 0; wd < words; ++wd) {  // word wd: classes 32 wd + 1 .. 32 wd + 32, plane [n_img][h*w]
    uint32_t* mw = mask + static_cast<size_t>(wd) * n_img * h * w;
    switch (label_dtype) {
      case PROTOSEG_I64:
        hipLaunchKernelGGL(patch_mask_kernel<int64_t>, grid, dim3(mt), lds, s, static_cast<const int64_t*>(label),
                           H_img, W_img, h, w, lut, lut_size, 32 * wd, mw);
        break;
      case PROTOSEG_I32:
        hipLaunchKernelGGL(patch_mask_kernel<int32_t>, grid, dim3(mt), lds, s, static_cast<const int32_t*>(label),
                           H_img, W_img, h, w, lut, lut_size, 32 * wd, mw);
        break;
      case PROTOSEG_U8:
        hipLaunchKernelGGL(patch_mask_kernel<uint8_t>, grid, dim3(mt), lds, s, static_cast<const uint8_t*>(label),
                           H_img, W_img, h, w, lut, lut_size, 32 * wd, mw);
        break;
      default:
        return fail(PROTOSEG_ERR_UNSUPPORTED, "label_dtype %d", label_dtype);
    }
  }
  return check_launch("patch_mask_kernel");
}

namespace {
// Partial top-2 scratch ([n_img][stripes x split][P][2] u64): one grow-only block per (device, stream),
// reused by later calls on that stream (kernels on one stream are ordered), so a call is only
// kernel launches and can be captured in a HIP graph once the block exists. A call that needs
// more takes a NEW block and retires the old one without freeing it: a graph that captured an
// earlier call still points there, and replaying it must not write into freed memory.
void* push_scratch(size_t need, hipStream_t s, int* status) {
  void* p = nullptr;
  *status = stream_scratch(ScratchKind::kPush, need, 1u << 20, s, &p);
  return p;
}
}  // namespace

extern "C" int protoseg_push_argmin(const float* x, int n_img, int C, int h, int w, const float* protos, int P,
                                    const int32_t* proto_class, const uint32_t* mask, uint64_t* img_keys,
                                    uint64_t* img_second, protoseg_stream_t stream) {
  return protoseg_push_argmin_words(x, n_img, C, h, w, protos, P, proto_class, mask, 1, img_keys, img_second, stream);
}

// The argmin of protoseg_push_argmin_words. With parts_out, the native path stops after the
// partial top-2 kernels and returns their scratch and count (the caller folds them:
// push_top2_merge_kernel); *parts_out = 0 when the wide path ran and wrote img_keys itself.
int push_argmin_impl(const float* x, int n_img, int C, int h, int w, const float* protos, int P,
                     const int32_t* proto_class, const uint32_t* mask, int words, uint64_t* img_keys,
                     uint64_t* img_second, hipStream_t s, const unsigned long long** part_out, int* parts_out,
                     const float* sd0) {
  if (words < 1 || words > 64) return fail(PROTOSEG_ERR_INVALID, "words=%d outside [1, 64]", words);
  if (!x || !protos || !proto_class || !mask || !img_keys)
    return fail(PROTOSEG_ERR_INVALID, "null pointer argument");
  if (parts_out) *parts_out = 0;
  if (n_img <= 0 || h <= 0 || w <= 0 || P <= 0) return fail(PROTOSEG_ERR_INVALID, "bad shape");
  const int nc = nc_of_push(C);
  if (n_img > 65535) return fail(PROTOSEG_ERR_UNSUPPORTED, "n_img=%d per call", n_img);
  if (!nc || words > 1) {  // other depths / more than 32 classes: the wide GEMM's distances + a masked argmin
    if (C <= 0 || C > 4096) return fail(PROTOSEG_ERR_UNSUPPORTED, "C=%d", C);
    const long long hwc = static_cast<long long>(h) * w;
    if (hwc * C * n_img >= (1LL << 31) || hwc * P >= (1LL << 31))
      return fail(PROTOSEG_ERR_UNSUPPORTED, "n_img*h*w*C or h*w*P >= 2^31");
    return wide_push_argmin(x, n_img, C, static_cast<int>(hwc), protos, P, proto_class, mask, words, img_keys,
                            img_second, s);
  }
  if (reinterpret_cast<uintptr_t>(protos) % 16 != 0) return fail(PROTOSEG_ERR_INVALID, "protos must be 16-B aligned");
  const long long HW = static_cast<long long>(h) * w;
  if (HW >= (1LL << 31) / 2) return fail(PROTOSEG_ERR_UNSUPPORTED, "h*w=%lld", HW);
  const int npt = static_cast<int>(ceil_div(P, 32));
  if (nc <= 2) {
    // wave-streamed kernel: prototype chunks of <= pw_max_tiles tiles, about one workgroup per
    // CU over the images (every wave at least one pixel tile)
    const int maxt = pw_max_tiles(nc);
    const long long ntile = ceil_div(HW, 32);
    int per = static_cast<int>(ceil_div(npt, ceil_div(npt, maxt)));
    long long wgs = ceil_div(256, static_cast<long long>(n_img));
    if (wgs > ceil_div(ntile, kPwWaves)) wgs = ceil_div(ntile, kPwWaves);
    if (wgs < 1) wgs = 1;
#if PUSH_CHUNK_PLAN
    {  // the chunk width and workgroups per (image, chunk) that minimise the busiest wave's work
      const PushPlan pl = push_wave_plan(npt, maxt, n_img, ntile, device_cus());
      per = pl.per;
      wgs = pl.wgs;
    }
#endif
    const int full = npt / per, rem = npt - full * per;
    const size_t need = static_cast<size_t>(n_img) * wgs * P * 2 * sizeof(unsigned long long);
    int st = PROTOSEG_OK;
    auto* part = static_cast<unsigned long long*>(push_scratch(need, s, &st));
    if (st) return st;
    auto launch = [&](auto kern, int chunks, int pt0, int nptc) {
      if (chunks <= 0) return;
      KernelTimer timer("push_argmin_wave_kernel", s);
      hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(wgs), n_img, chunks), dim3(kPwWaves * 64),
                         pw_lds_bytes(C, nptc), s, x, static_cast<int>(HW), protos, P, pt0, nptc, proto_class, mask,
                         part, static_cast<int>(wgs), sd0);
    };
    if (nc == 1) {
      if (int e = ensure_lds<push_argmin_wave_kernel<1>>()) return e;
      launch(push_argmin_wave_kernel<1>, full, 0, per);
      launch(push_argmin_wave_kernel<1>, rem ? 1 : 0, full * per, rem);
    } else {
      if (int e = ensure_lds<push_argmin_wave_kernel<2>>()) return e;
      launch(push_argmin_wave_kernel<2>, full, 0, per);
      launch(push_argmin_wave_kernel<2>, rem ? 1 : 0, full * per, rem);
    }
    if (int e = check_launch("push_argmin_wave_kernel")) return e;
    if (parts_out) {
      *part_out = part;
      *parts_out = static_cast<int>(wgs);
      return PROTOSEG_OK;
    }
    const long long n = static_cast<long long>(n_img) * P;
    hipLaunchKernelGGL(push_top2_kernel, dim3(static_cast<unsigned>(ceil_div(n, 256))), dim3(256), 0, s, part, n_img,
                       static_cast<int>(wgs), P, reinterpret_cast<unsigned long long*>(img_keys),
                       reinterpret_cast<unsigned long long*>(img_second));
    return check_launch("push_top2_kernel");
  }
  // prototype chunks of equal width (P = 361: 6 + 6 tiles, not 8 + 4, so both launches keep 3
  // waves per SIMD): `per` tiles in `full` chunks, then the remainder chunk
  const int per = static_cast<int>(ceil_div(npt, ceil_div(npt, kPushMaxTiles)));
  const int full = npt / per, rem = npt - full * per;
  const long long nblk = ceil_div(HW, kPushBlkPix);
  // One generation of workgroups per launch (one per CU: 12 waves at ~120 VGPRs fill a CU's
  // wave slots), each walking many 128-pixel blocks, so the prologue (prototype vectors, ||p||^2,
  // first DMA) and the tail are paid once: 2 generations of half-length workgroups measured
  // 22 % slower (P = 190, 8 images: 148 -> 115 us). Each prototype-chunk launch gets its own
  // generation (stripes do not shrink with the chunk count).
  long long stripes = ceil_div(PUSH_WG_TARGET, static_cast<long long>(n_img));
  if (stripes > nblk) stripes = nblk;
  if (stripes < 1) stripes = 1;
  const size_t need = static_cast<size_t>(n_img) * stripes * kPushSplit * P * 2 * sizeof(unsigned long long);
  int st = PROTOSEG_OK;
  auto* part = static_cast<unsigned long long*>(push_scratch(need, s, &st));
  if (st) return st;
  auto launch = [&](auto kern, int chunks, int pt0, int nptc) {
    if (chunks <= 0) return;
    const int waves = nptc * kPushSplit;
    KernelTimer timer("push_argmin_kernel", s);
    hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(stripes), n_img, chunks), dim3(waves * 64),
                       push_lds_bytes(C, waves), s, x, static_cast<int>(HW), protos, P, pt0, nptc, proto_class, mask,
                       part, static_cast<int>(stripes));
  };
  if (nc == 1) {
    launch(push_argmin_kernel<1>, full, 0, per);
    launch(push_argmin_kernel<1>, rem ? 1 : 0, full * per, rem);
  } else if (nc == 2) {
    if (int e = ensure_lds<push_argmin_kernel<2>>()) return e;
    launch(push_argmin_kernel<2>, full, 0, per);
    launch(push_argmin_kernel<2>, rem ? 1 : 0, full * per, rem);
  } else {
    if (push_lds_bytes(C, per * kPushSplit) > kMaxLds) return fail(PROTOSEG_ERR_UNSUPPORTED, "push LDS at C=%d", C);
    if (int e = ensure_lds<push_argmin_kernel<4>>()) return e;
    launch(push_argmin_kernel<4>, full, 0, per);
    launch(push_argmin_kernel<4>, rem ? 1 : 0, full * per, rem);
  }
  if (int e = check_launch("push_argmin_kernel")) return e;
  if (parts_out) {
    *part_out = part;
    *parts_out = static_cast<int>(stripes) * kPushSplit;
    return PROTOSEG_OK;
  }
  const long long n = static_cast<long long>(n_img) * P;
  hipLaunchKernelGGL(push_top2_kernel, dim3(static_cast<unsigned>(ceil_div(n, 256))), dim3(256), 0, s, part, n_img,
                     static_cast<int>(stripes) * kPushSplit, P, reinterpret_cast<unsigned long long*>(img_keys),
                     reinterpret_cast<unsigned long long*>(img_second));
  return check_launch("push_top2_kernel");
}

extern "C" int protoseg_push_argmin_words(const float* x, int n_img, int C, int h, int w, const float* protos, int P,
                                          const int32_t* proto_class, const uint32_t* mask, int words,
                                          uint64_t* img_keys, uint64_t* img_second, protoseg_stream_t stream) {
  return push_argmin_impl(x, n_img, C, h, w, protos, P, proto_class, mask, words, img_keys, img_second,
                          reinterpret_cast<hipStream_t>(stream), nullptr, nullptr, nullptr);
}

extern "C" int protoseg_push_distances(const float* x, int C, int h, int w, const float* protos, int m, float* dist,
                                       protoseg_stream_t stream) {
  return protoseg_push_distances_words(x, C, h, w, protos, m, 1, dist, stream);
}

extern "C" int protoseg_push_distances_words(const float* x, int C, int h, int w, const float* protos, int m, int words,
                                             float* dist, protoseg_stream_t stream) {
  if (words < 1 || words > 64) return fail(PROTOSEG_ERR_INVALID, "words=%d outside [1, 64]", words);
  if (!x || !protos || !dist) return fail(PROTOSEG_ERR_INVALID, "null pointer argument");
  if (h <= 0 || w <= 0 || m <= 0) return fail(PROTOSEG_ERR_INVALID, "bad shape h=%d w=%d m=%d", h, w, m);
  const int nc = nc_of_push(C);
  const long long HW = static_cast<long long>(h) * w;
  if (HW * C >= (1LL << 31) || HW * m >= (1LL << 31)) return fail(PROTOSEG_ERR_UNSUPPORTED, "h*w=%lld too large", HW);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!nc || words > 1) {  // the wide path's arithmetic, so ties here are the ties protoseg_push_argmin saw
    if (C <= 0 || C > 4096) return fail(PROTOSEG_ERR_UNSUPPORTED, "C=%d", C);
    return wide_push_distances_scratch(x, C, static_cast<int>(HW), protos, m, dist, s);
  }
  if (reinterpret_cast<uintptr_t>(protos) % 16 != 0) return fail(PROTOSEG_ERR_INVALID, "protos must be 16-B aligned");
  const dim3 grid(static_cast<unsigned>(ceil_div(HW, 32)), static_cast<unsigned>(ceil_div(m, 32)));
  const int n = static_cast<int>(HW);
  if (nc == 1)
    hipLaunchKernelGGL(push_dist_kernel<1>, grid, dim3(64), 0, s, x, n, protos, m, dist);
  else if (nc == 2)
    hipLaunchKernelGGL(push_dist_kernel<2>, grid, dim3(64), 0, s, x, n, protos, m, dist);
  else
    hipLaunchKernelGGL(push_dist_kernel<4>, grid, dim3(64), 0, s, x, n, protos, m, dist);
  return check_launch("push_dist_kernel");
}

extern "C" int protoseg_push_merge(const uint64_t* img_keys, const uint64_t* img_second, int n_img,
                                   int64_t first_img, const float* x, int C, int hw, int P, float* global_dist,
                                   float* global_second, int64_t* global_img, int32_t* global_patch,
                                   float* global_fmap, protoseg_stream_t stream) {
  if (!img_keys || !x || !global_dist || !global_img || !global_patch || !global_fmap)
    return fail(PROTOSEG_ERR_INVALID, "null pointer argument");
  if (!img_second != !global_second)
    return fail(PROTOSEG_ERR_INVALID, "img_second and global_second are given together or not at all");
  if (n_img <= 0 || C <= 0 || hw <= 0 || P <= 0) return fail(PROTOSEG_ERR_INVALID, "bad shape");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int waves_per_block = 4;
  hipLaunchKernelGGL(push_merge_kernel, dim3(static_cast<unsigned>(ceil_div(P, waves_per_block))),
                     dim3(waves_per_block * 64), 0, s, reinterpret_cast<const unsigned long long*>(img_keys),
                     reinterpret_cast<const unsigned long long*>(img_second), n_img,
                     static_cast<long long>(first_img), x, C, hw, P, global_dist, global_second,
                     reinterpret_cast<long long*>(global_img), global_patch, global_fmap);
  return check_launch("push_merge_kernel");
}

// push.py:184-281 for one batch of equal-geometry images in ONE host call: class masks, the
// masked top-2 argmin and the strict-'<' merge into the running state, with the mask and the
// per-image keys in this stream's scratch (kPushUpdate) instead of caller tensors. The result
// is the three-call sequence's (same kernels, same order).
extern "C" int protoseg_push_update(const void* label, int label_dtype, int n_img, int H_img, int W_img,
                                    const int32_t* lut, int lut_size, int words, const float* x, int C, int h, int w,
                                    const float* protos, int P, const int32_t* proto_class, int64_t first_img,
                                    float* global_dist, float* global_second, int64_t* global_img,
                                    int32_t* global_patch, float* global_fmap, protoseg_stream_t stream) {
  if (words < 1 || words > 64) return fail(PROTOSEG_ERR_INVALID, "words=%d outside [1, 64]", words);
  if (n_img <= 0 || h <= 0 || w <= 0 || P <= 0) return fail(PROTOSEG_ERR_INVALID, "bad shape");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const size_t hw = static_cast<size_t>(h) * w;
  const size_t mask_bytes = (static_cast<size_t>(words) * n_img * hw * 4 + 255) & ~static_cast<size_t>(255);
  const size_t key_bytes = static_cast<size_t>(n_img) * P * 8;
  void* sc = nullptr;
  if (int st = stream_scratch(ScratchKind::kPushUpdate, mask_bytes + 2 * key_bytes, 1u << 20, s, &sc)) return st;
  auto* mask = static_cast<uint32_t*>(sc);
  auto* keys = reinterpret_cast<uint64_t*>(static_cast<unsigned char*>(sc) + mask_bytes);
  uint64_t* second = global_second ? keys + static_cast<size_t>(n_img) * P : nullptr;
  if (int st = protoseg_patch_class_mask_words(label, label_dtype, n_img, H_img, W_img, h, w, lut, lut_size, words,
                                               mask, stream))
    return st;
  const unsigned long long* part = nullptr;
  int parts = 0;
  // the running runner-up (or, without one, the running best) bounds the candidates that can
  // still change the state: the argmin's per-image top-2 drops the rest (push_argmin_wave_kernel)
  const float* bound = global_second ? global_second : global_dist;
  if (int st = push_argmin_impl(x, n_img, C, h, w, protos, P, proto_class, mask, words, keys, second, s, &part, &parts,
                                bound))
    return st;
  if (parts == 0)  // the wide path wrote the per-image keys
    return protoseg_push_merge(keys, second, n_img, first_img, x, C, static_cast<int>(hw), P, global_dist,
                               global_second, global_img, global_patch, global_fmap, stream);
  if (!global_dist || !global_img || !global_patch || !global_fmap)
    return fail(PROTOSEG_ERR_INVALID, "null pointer argument");
  const int waves_per_block = 4;
  hipLaunchKernelGGL(push_top2_merge_kernel, dim3(static_cast<unsigned>(ceil_div(P, waves_per_block))),
                     dim3(waves_per_block * 64), 0, s, part, parts, n_img, static_cast<long long>(first_img), x, C,
                     static_cast<int>(hw), P, global_dist, global_second, reinterpret_cast<long long*>(global_img),
                     global_patch, global_fmap);
  return check_launch("push_top2_merge_kernel");
}
