// bbox.hip — high-activation bound boxes of the pushed prototypes on gfx950.
//
// Reference: segmentation/push.py:309-353 (inside update_prototypes_on_image) and
// helpers.py:48-82 (find_continuous_high_activation_crop). Per pushed prototype the reference
//   1. turns the winning image's distance map into activations (push.py:310-316),
//   2. cv2.resize(..., INTER_CUBIC) to the full image (push.py:318-319),
//   3. threshold = np.percentile(upsampled, 95) (push.py:322),
//   4. multiplies by the ground-truth mask of the prototype's class (push.py:325-326),
//   5. grows the receptive-field box greedily over pixels >= threshold, then adds a 5-px
//      margin (push.py:328-329, helpers.py:48-82).
// Here: act_kernel (1), cubic_upsample_kernel (2: one thread per output pixel, OpenCV's
// separable H-then-V INTER_CUBIC with A = -0.75, half-pixel centres, replicated border, every
// product and sum rounded separately as the scalar OpenCV code writes them), a radix select of
// the two order statistics numpy's 'linear' percentile interpolates between (3: three passes of
// select_hist_kernel, each map split over ~2048 / m workgroups, select_step_kernel between them),
// and bound_box_kernel (3-5: one 1024-thread workgroup per prototype map — the threshold in
// numpy's f32 arithmetic, then the greedy walk with every row/column probe a workgroup-wide OR).
#include <map>
#include <mutex>
#include <utility>

#include "protoseg_device.h"
#include "protoseg_host.h"

// The restated arithmetic rounds every product and sum separately: no FMA contraction in this
// file (the pragma, plus -ffp-contract=off for bbox.o in the Makefile; HIP's __fmul_rn et al.
// are header inlines that the default fast contraction would still fuse).
#pragma clang fp contract(off)

namespace protoseg {

namespace {

constexpr int kBoxThreads = 1024;
constexpr int kUpThreads = 256;
constexpr int kHistBins = 2048;

__device__ __forceinline__ float fmul(float a, float b) { return a * b; }
__device__ __forceinline__ float fadd(float a, float b) { return a + b; }
__device__ __forceinline__ float fsub(float a, float b) { return a - b; }

// OpenCV imgproc resize.cpp interpolateCubic, A = -0.75, f32.
__device__ __forceinline__ void cubic_coeffs(float x, float c[4]) {
  const float A = -0.75f;
  const float x1 = fadd(x, 1.0f);
  c[0] = fsub(fmul(fadd(fmul(fsub(fmul(A, x1), 5.0f * A), x1), 8.0f * A), x1), 4.0f * A);
  c[1] = fadd(fmul(fmul(fsub(fmul(A + 2.0f, x), A + 3.0f), x), x), 1.0f);
  const float omx = fsub(1.0f, x);
  c[2] = fadd(fmul(fmul(fsub(fmul(A + 2.0f, omx), A + 3.0f), omx), omx), 1.0f);
  c[3] = fsub(fsub(fsub(1.0f, c[0]), c[1]), c[2]);
}

// Source taps of output index d: fx = (float)((d + 0.5) * scale - 0.5) in f64 (scale =
// 1 / (dsize / ssize) as cv::resize forms it), sx = floor(fx), taps sx-1 .. sx+2 clamped.
__device__ __forceinline__ void cubic_taps(int d, double scale, int n_src, int idx[4], float c[4]) {
  const float f = static_cast<float>((static_cast<double>(d) + 0.5) * scale - 0.5);
  const float fl = floorf(f);
  const int s = static_cast<int>(fl);
  cubic_coeffs(fsub(f, fl), c);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    int t = s + k - 1;
    t = t < 0 ? 0 : t;
    idx[k] = t > n_src - 1 ? n_src - 1 : t;
  }
}

// push.py:312-316 on the f32 numpy map: log -> np.log((d + 1) / (d + eps)) (f32 ops; the log
// rounded from f64), linear -> max_dist - d, identity -> the caller passed activations.
__global__ __launch_bounds__(256) void act_kernel(const float* __restrict__ dist, size_t n, int kind, float eps,
                                                  float max_dist, float* __restrict__ act) {
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const float d = dist[i];
    float a;
    if (kind == PROTOSEG_ACT_LOG) {
      const float q = fadd(d, 1.0f) / fadd(d, eps);
      a = static_cast<float>(log(static_cast<double>(q)));
    } else if (kind == PROTOSEG_ACT_LINEAR) {
      a = fsub(max_dist, d);
    } else {
      a = d;
    }
    act[i] = a;
  }
}

// Output tile: kUpThreads columns x `rows` output rows of one map per workgroup (grid
// (ceil(W / 256), ceil(H / rows), m)). Phase 1: the horizontal pass for every source row the
// tile touches, one column per thread (its x taps computed once), into LDS. Phase 2: the
// vertical pass per output row from LDS, coalesced row stores. Each H-value is formed once per
// tile instead of once per output pixel; the arithmetic is the same sequence as OpenCV's.
constexpr int kUpMaxSrcRows = 72;
constexpr int kUpMaxRows = 64;

__global__ __launch_bounds__(kUpThreads) void cubic_upsample_kernel(const float* __restrict__ act, int h, int w,
                                                                    int H, int W, int rows, double scale_y,
                                                                    double scale_x, float* __restrict__ up) {
  __shared__ float hr[kUpMaxSrcRows][kUpThreads];
  __shared__ float ycoef[kUpMaxRows][4];
  __shared__ int yrow[kUpMaxRows][4];
  const int t = threadIdx.x;
  const int dx = blockIdx.x * kUpThreads + t;
  const int dy0 = blockIdx.y * rows;
  const int dy1 = dy0 + rows < H ? dy0 + rows : H;
  const int map = blockIdx.z;
  // Source row window [r0, r1] of this tile (taps are monotone in dy).
  int i0[4], i1[4];
  float c_unused[4];
  cubic_taps(dy0, scale_y, h, i0, c_unused);
  cubic_taps(dy1 - 1, scale_y, h, i1, c_unused);
  const int r0 = i0[0], r1 = i1[3];
  if (t < dy1 - dy0) {
    int yi[4];
    float b[4];
    cubic_taps(dy0 + t, scale_y, h, yi, b);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      ycoef[t][k] = b[k];
      yrow[t][k] = yi[k] - r0;
    }
  }
  const float* S = act + static_cast<size_t>(map) * h * w;
  if (dx < W) {
    int xi[4];
    float a[4];
    cubic_taps(dx, scale_x, w, xi, a);
    for (int r = r0; r <= r1; ++r) {  // HResizeCubic: S[x0]*a0 + S[x1]*a1 + S[x2]*a2 + S[x3]*a3
      const float* R = S + static_cast<size_t>(r) * w;
      hr[r - r0][t] = fadd(fadd(fadd(fmul(R[xi[0]], a[0]), fmul(R[xi[1]], a[1])), fmul(R[xi[2]], a[2])),
                           fmul(R[xi[3]], a[3]));
    }
  }
  __syncthreads();
  if (dx >= W) return;
  float* out = up + (static_cast<size_t>(map) * H + dy0) * W + dx;
  for (int j = 0; j < dy1 - dy0; ++j) {  // VResizeCubic: S0*b0 + S1*b1 + S2*b2 + S3*b3
    const float v = fadd(fadd(fadd(fmul(hr[yrow[j][0]][t], ycoef[j][0]), fmul(hr[yrow[j][1]][t], ycoef[j][1])),
                              fmul(hr[yrow[j][2]][t], ycoef[j][2])),
                         fmul(hr[yrow[j][3]][t], ycoef[j][3]));
    out[static_cast<size_t>(j) * W] = v;
  }
}

// The same resize with four adjacent output columns per thread (W % 4 == 0): 1024 columns per
// workgroup, the horizontal values of a source row stored and read as float4, and float4 row
// stores. Every output value is the same operation sequence as cubic_upsample_kernel's.
constexpr int kUp4Cols = 4 * kUpThreads;
constexpr int kUp4MaxSrcRows = 16;

__global__ __launch_bounds__(kUpThreads) void cubic_upsample4_kernel(const float* __restrict__ act, int h, int w,
                                                                     int H, int W, int rows, double scale_y,
                                                                     double scale_x, float* __restrict__ up) {
  __shared__ float4 hr[kUp4MaxSrcRows][kUpThreads];
  __shared__ float ycoef[kUpMaxRows][4];
  __shared__ int yrow[kUpMaxRows][4];
  const int t = threadIdx.x;
  const int dx0 = blockIdx.x * kUp4Cols + 4 * t;
  const int dy0 = blockIdx.y * rows;
  const int dy1 = dy0 + rows < H ? dy0 + rows : H;
  const int map = blockIdx.z;
  int i0[4], i1[4];
  float c_unused[4];
  cubic_taps(dy0, scale_y, h, i0, c_unused);
  cubic_taps(dy1 - 1, scale_y, h, i1, c_unused);
  const int r0 = i0[0], r1 = i1[3];
  if (t < dy1 - dy0) {
    int yi[4];
    float b[4];
    cubic_taps(dy0 + t, scale_y, h, yi, b);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      ycoef[t][k] = b[k];
      yrow[t][k] = yi[k] - r0;
    }
  }
  const float* S = act + static_cast<size_t>(map) * h * w;
  if (dx0 < W) {  // W % 4 == 0: the thread's four columns are all inside the row
    int xi[4][4];
    float a[4][4];
#pragma unroll
    for (int e = 0; e < 4; ++e) cubic_taps(dx0 + e, scale_x, w, xi[e], a[e]);
    for (int r = r0; r <= r1; ++r) {
      const float* R = S + static_cast<size_t>(r) * w;
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        o[e] = fadd(fadd(fadd(fmul(R[xi[e][0]], a[e][0]), fmul(R[xi[e][1]], a[e][1])), fmul(R[xi[e][2]], a[e][2])),
                    fmul(R[xi[e][3]], a[e][3]));
      hr[r - r0][t] = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
  __syncthreads();
  if (dx0 >= W) return;
  float4* out = reinterpret_cast<float4*>(up + (static_cast<size_t>(map) * H + dy0) * W + dx0);
  for (int j = 0; j < dy1 - dy0; ++j) {
    const float4 s0 = hr[yrow[j][0]][t], s1 = hr[yrow[j][1]][t], s2 = hr[yrow[j][2]][t], s3 = hr[yrow[j][3]][t];
    const float b0 = ycoef[j][0], b1 = ycoef[j][1], b2 = ycoef[j][2], b3 = ycoef[j][3];
    float4 v;
    v.x = fadd(fadd(fadd(fmul(s0.x, b0), fmul(s1.x, b1)), fmul(s2.x, b2)), fmul(s3.x, b3));
    v.y = fadd(fadd(fadd(fmul(s0.y, b0), fmul(s1.y, b1)), fmul(s2.y, b2)), fmul(s3.y, b3));
    v.z = fadd(fadd(fadd(fmul(s0.z, b0), fmul(s1.z, b1)), fmul(s2.z, b2)), fmul(s3.z, b3));
    v.w = fadd(fadd(fadd(fmul(s0.w, b0), fmul(s1.w, b1)), fmul(s2.w, b2)), fmul(s3.w, b3));
    out[static_cast<size_t>(j) * (W / 4)] = v;
  }
}

// Order-preserving f32 <-> u32 (NaN sorts last, as np.sort puts it).
__device__ __forceinline__ uint32_t fkey(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float fkey_inv(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// The percentile's order statistic is selected by a three-pass radix select over 11 + 11 + 10
// key bits, split across many workgroups per map: pass p histograms, in LDS (one sub-histogram
// per wave, so equal keys of different waves do not serialise on one LDS bin), the key bits
// (sh, width) of a chunk's elements whose higher bits match the prefix found so far, and adds the
// non-zero bins into the map's global histogram; a one-workgroup-per-map select then picks the
// bin holding the wanted rank, extends the prefix and clears the histogram for the next pass.
// Pass 2 also copies the elements of the chosen 11-bit bin into a per-map candidate list when
// they fit (`cap` per map), so pass 3 reads only those instead of the whole map. The smallest
// key above the final 22-bit prefix block (the next order statistic when no larger key shares
// the prefix) is taken on the way: above the 11-bit block in pass 2, inside it in pass 3.
constexpr int kHistThreads = 256;
constexpr int kHistWaves = kHistThreads / 64;
constexpr int kSelTarget = 4096;           // histogram workgroups per launch (all maps)
constexpr int kSelMinChunk = 1 << 15;      // elements per histogram workgroup, at least
constexpr int kPassShift[3] = {21, 10, 0};
constexpr int kPassWidth[3] = {11, 11, 10};

// Per-map select state in the scratch block: {prefix, pmask, rank, below, min_above, -,
// candidates written, candidate list in use}.
constexpr int kSelState = 8;

// numpy 'linear' percentile on f32 (push.py:322): q / 100 in f32, virtual index (n - 1) * q in
// f32, the two neighbouring ranks and the lerp weight.
__device__ __forceinline__ void percentile_ranks(size_t n, float percentile, uint32_t& lo, uint32_t& hi, float& g) {
  const float qq = percentile / 100.0f;
  const float vidx = fmul(static_cast<float>(n - 1), qq);
  if (vidx >= static_cast<float>(n - 1)) {
    lo = hi = static_cast<uint32_t>(n - 1);
  } else {
    const float fl = floorf(vidx < 0.f ? 0.f : vidx);
    lo = static_cast<uint32_t>(fl);
    hi = lo + 1u;
  }
  g = vidx < 0.f ? 0.f : fsub(vidx, floorf(vidx));
}

// grid (m), 256 threads: clear the map's histogram, seed its select state.
__global__ __launch_bounds__(256) void select_init_kernel(size_t n, float percentile, uint32_t* __restrict__ hist,
                                                          uint32_t* __restrict__ state) {
  uint32_t* h = hist + static_cast<size_t>(blockIdx.x) * kHistBins;
  for (int i = threadIdx.x; i < kHistBins; i += 256) h[i] = 0u;
  if (threadIdx.x < kSelState) {
    uint32_t lo, hi;
    float g;
    percentile_ranks(n, percentile, lo, hi, g);
    // prefix, pmask, rank still to find inside the prefix, elements below the prefix, smallest
    // key above the final prefix block, -, candidates written, candidate list in use
    const uint32_t init[kSelState] = {0u, 0u, lo, 0u, 0xffffffffu, 0u, 0u, 0u};
    state[static_cast<size_t>(blockIdx.x) * kSelState + threadIdx.x] = init[threadIdx.x];
  }
}

// grid (chunks, m), 256 threads: pass PASS histogram of one chunk of map blockIdx.y (of its
// candidate list in pass 3 when pass 2 filled one).
template <int PASS>
__global__ __launch_bounds__(kHistThreads) void select_hist_kernel(const float* __restrict__ up, size_t n,
                                                                   size_t chunk, float* __restrict__ cand,
                                                                   size_t cap, uint32_t* __restrict__ hist,
                                                                   uint32_t* __restrict__ chunk_hist,
                                                                   uint32_t* __restrict__ state) {
  // one sub-histogram per wave in pass 1 (every element lands in it); passes 2 and 3 add only
  // the few elements inside the prefix and keep the small footprint (more workgroups per CU)
  constexpr int kSub = PASS == 0 ? 2 : 1;
  __shared__ uint32_t h[kSub][kHistBins];
  __shared__ uint32_t s_min[kHistWaves];
  __shared__ uint32_t s_fill;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int map = blockIdx.y;
  uint32_t* st = state + static_cast<size_t>(map) * kSelState;
  const uint32_t prefix = st[0], pmask = st[1];
  const bool use_cand = PASS == 2 && st[7] != 0u;
  const bool fill_cand = PASS == 1 && st[7] != 0u;
  const float* src = use_cand ? cand + static_cast<size_t>(map) * cap : up + static_cast<size_t>(map) * n;
  const size_t total = use_cand ? st[6] : n;
  const size_t c0 = static_cast<size_t>(blockIdx.x) * chunk;
  if (c0 >= total) return;  // uniform (pass 3 on a short candidate list)
  const size_t len = (c0 + chunk < total ? c0 + chunk : total) - c0;
  const float* a = src + c0;
  float* cdst = cand + static_cast<size_t>(map) * cap;
  constexpr int sh = kPassShift[PASS];
  constexpr uint32_t bm = (1u << kPassWidth[PASS]) - 1u;
  // keys above the current prefix block: above the 11-bit block (pass 2), the 22-bit one (pass 3)
  const uint32_t above = prefix | (PASS == 1 ? 0x1fffffu : 0x3ffu);
  for (int i = t; i < kSub * kHistBins; i += kHistThreads) (&h[0][0])[i] = 0u;
  uint32_t* crow = chunk_hist + (static_cast<size_t>(map) * gridDim.x) * kHistBins;  // pass 1's per-chunk rows
  if (fill_cand && t == 0) {
    // this chunk's slots in the candidate list: after the earlier chunks' elements of the bin
    // (pass 1's per-chunk histogram rows)
    const uint32_t b0 = prefix >> 21;
    uint32_t base = 0u;
    for (unsigned c = 0; c < blockIdx.x; ++c) base += crow[static_cast<size_t>(c) * kHistBins + b0];
    s_fill = base;
  }
  __syncthreads();
  uint32_t mn = 0xffffffffu;
  uint32_t* hw = h[PASS == 0 ? (wave & 1) : 0];
  // Up to 16 values of this lane (bit u of `valid`): histogram, running min, candidate copy.
  // Called with wave-uniform control flow (the copy's wave scan needs every lane).
  auto process = [&](const float* v, int nv, uint32_t valid) {
    uint32_t match = 0u;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (u >= nv) break;
      const uint32_t k = fkey(v[u]);
      const bool ok = (valid >> u) & 1u;
      if (ok && (k & pmask) == prefix) {
        atomicAdd(&hw[(k >> sh) & bm], 1u);
        match |= 1u << u;
      }
      if (PASS > 0 && ok && k > above) mn = k < mn ? k : mn;
    }
    if (PASS == 1 && fill_cand) {
      // wave-wide slots, value-major: value u's matches of all lanes are one contiguous run
      // (ballot + mbcnt), so every store instruction writes consecutive addresses
      unsigned long long bal[16];
      uint32_t wtot = 0u;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        if (u >= nv) break;
        bal[u] = __ballot((match >> u) & 1u);
        wtot += __popcll(bal[u]);
      }
      if (wtot) {  // uniform
        uint32_t base = 0u;
        if (lane == 0) base = atomicAdd(&s_fill, wtot);
        base = __shfl(base, 0);
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          if (u >= nv) break;
          if ((match >> u) & 1u) {
            const uint32_t pos = base + __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(bal[u] >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(bal[u]), 0u));
            if (pos < cap) cdst[pos] = v[u];
          }
          base += __popcll(bal[u]);
        }
      }
    }
  };
  const bool aligned = (reinterpret_cast<uintptr_t>(a) & 15u) == 0;
  const size_t n4 = aligned ? len / 4 : 0;
  const float4* a4 = reinterpret_cast<const float4*>(a);
  size_t i0 = 0;
  for (; i0 + 8 * kHistThreads <= n4; i0 += 8 * kHistThreads) {  // eight float4 loads in flight
    float v[32];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float4 q = a4[i0 + u * kHistThreads + t];
      v[4 * u] = q.x; v[4 * u + 1] = q.y; v[4 * u + 2] = q.z; v[4 * u + 3] = q.w;
    }
    process(v, 16, 0xffffu);
    process(v + 16, 16, 0xffffu);
  }
  for (; i0 < n4; i0 += kHistThreads) {
    const bool ok = i0 + t < n4;
    const float4 q = ok ? a4[i0 + t] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float v[4] = {q.x, q.y, q.z, q.w};
    process(v, 4, ok ? 0xfu : 0u);
  }
  for (size_t j0 = n4 * 4; j0 < len; j0 += kHistThreads) {
    const bool ok = j0 + t < len;
    const float v[1] = {ok ? a[j0 + t] : 0.f};
    process(v, 1, ok ? 1u : 0u);
  }
  if (PASS > 0) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const uint32_t y = __shfl_xor(mn, o);
      mn = y < mn ? y : mn;
    }
    if (lane == 0) s_min[wave] = mn;
  }
  __syncthreads();
  uint32_t* gh = hist + static_cast<size_t>(map) * kHistBins;
  for (int b = t; b <= static_cast<int>(bm); b += kHistThreads) {
    uint32_t c = 0u;
#pragma unroll
    for (int w = 0; w < kSub; ++w) c += h[w][b];
    if (c) atomicAdd(&gh[b], c);
    if (PASS == 0) crow[static_cast<size_t>(blockIdx.x) * kHistBins + b] = c;
  }
  if (PASS > 0 && t == 0) {
    uint32_t m = s_min[0];
    for (int w = 1; w < kHistWaves; ++w) m = s_min[w] < m ? s_min[w] : m;
    if (m != 0xffffffffu) atomicMin(&st[4], m);
  }
}

// Whole-workgroup (1024 threads, 2 bins each) search of a map's global histogram for the bin
// holding `rank`: returns (bin, elements in lower bins, elements in the bin).
struct BinPick {
  uint32_t bin, excl, count;
};
__device__ BinPick pick_bin(const uint32_t* __restrict__ gh, uint32_t rank, uint32_t* scan, uint32_t* bcast) {
  const int t = threadIdx.x;
  const uint32_t h0 = gh[2 * t], h1 = gh[2 * t + 1];
  const uint32_t s = h0 + h1;
  scan[t] = s;
  __syncthreads();
  for (int off = 1; off < kBoxThreads; off <<= 1) {
    const uint32_t v = t >= off ? scan[t - off] : 0u;
    __syncthreads();
    scan[t] += v;
    __syncthreads();
  }
  const uint32_t incl = scan[t], excl = incl - s;
  if (excl <= rank && rank < incl) {
    const uint32_t r = rank - excl;
    if (r < h0) {
      bcast[0] = 2u * t; bcast[1] = excl; bcast[2] = h0;
    } else {
      bcast[0] = 2u * t + 1u; bcast[1] = excl + h0; bcast[2] = h1;
    }
  }
  __syncthreads();
  const BinPick p{bcast[0], bcast[1], bcast[2]};
  __syncthreads();
  return p;
}

// grid (m), 1024 threads: after pass `pass` (0 or 1), extend the prefix and clear the histogram;
// after pass 1, turn the candidate list on when the chosen bin's elements fit in it.
__global__ __launch_bounds__(kBoxThreads) void select_step_kernel(int pass, size_t cap, uint32_t* __restrict__ hist,
                                                                  uint32_t* __restrict__ state) {
  __shared__ uint32_t scan[kBoxThreads];
  __shared__ uint32_t bcast[4];
  uint32_t* gh = hist + static_cast<size_t>(blockIdx.x) * kHistBins;
  uint32_t* st = state + static_cast<size_t>(blockIdx.x) * kSelState;
  const BinPick p = pick_bin(gh, st[2], scan, bcast);  // all reads of gh are behind pick_bin's barriers
  gh[2 * threadIdx.x] = 0u;
  gh[2 * threadIdx.x + 1] = 0u;
  if (threadIdx.x == 0) {
    const int sh = kPassShift[pass];
    st[0] |= p.bin << sh;
    st[1] |= ((1u << kPassWidth[pass]) - 1u) << sh;
    st[2] -= p.excl;
    st[3] += p.excl;
    if (pass == 0) {  // pass 2 copies the bin's elements out when they fit
      st[6] = p.count;
      st[7] = p.count <= cap ? 1u : 0u;
    }
  }
}

template <typename TL>
__device__ __forceinline__ long long label_value(const TL* L, size_t i, const int32_t* lut, int lut_size) {
  const long long raw = static_cast<long long>(L[i]);
  if (!lut) return raw;
  if (raw < 0 || raw >= lut_size) return -1;
  return lut[raw];
}

// grid (m), 1024 threads, after the three select passes. rf [m, 4] = (start_h, end_h, start_w,
// end_w) of push.py:288-294; box [m, 4] = (start_h, end_h + 1, start_w, end_w + 1) of
// helpers.py:82; -1 rows for maps whose label index or rf box is out of range.
template <typename TL>
__global__ __launch_bounds__(kBoxThreads) void bound_box_kernel(
    const float* __restrict__ up, int H, int W, const TL* __restrict__ label, int n_label, const int32_t* label_index,
    const int32_t* __restrict__ lut, int lut_size, const int32_t* __restrict__ target_class,
    const int32_t* __restrict__ rf, float percentile, int margin, const uint32_t* __restrict__ hist,
    const uint32_t* __restrict__ state, float* __restrict__ thr_out, int32_t* __restrict__ box_out) {
  __shared__ uint32_t scan[kBoxThreads];
  __shared__ uint32_t bcast[4];
  __shared__ uint32_t s_next;
  const int map = blockIdx.x;
  const size_t n = static_cast<size_t>(H) * W;
  const float* U = up + static_cast<size_t>(map) * n;
  int sh = rf[4 * map + 0], eh = rf[4 * map + 1], sw = rf[4 * map + 2], ew = rf[4 * map + 3];
  const int li = label_index ? label_index[map] : 0;
  if (li < 0 || li >= n_label || sh < 0 || sh >= H || sw < 0 || sw >= W || eh < sh || ew < sw) {
    if (threadIdx.x < 4) box_out[4 * map + threadIdx.x] = -1;
    if (threadIdx.x == 0) thr_out[map] = __uint_as_float(0x7fc00000u);
    return;
  }

  // push.py:322 np.percentile(upsampled, q): numpy 'linear' on f32 — q / 100 in f32,
  // virtual index (n - 1) * q in f32, lerp between the two neighbouring order statistics with
  // numpy's _lerp (a + (b - a) * g, or b - (b - a) * (1 - g) when g >= 0.5), all f32.
  uint32_t lo, hi;
  float g;
  percentile_ranks(n, percentile, lo, hi, g);
  // The last pass's bin: the full key of rank lo, the elements below it and equal to it.
  const uint32_t* gh = hist + static_cast<size_t>(map) * kHistBins;
  const uint32_t* st = state + static_cast<size_t>(map) * kSelState;
  const uint32_t prefix = st[0], rank = st[2], below0 = st[3], min_above = st[4];
  if (threadIdx.x == 0) s_next = 0xffffffffu;
  const BinPick p = pick_bin(gh, rank, scan, bcast);
  const uint32_t key = prefix | p.bin;
  uint32_t key_hi = key;
  if (hi != lo && hi >= below0 + p.excl + p.count) {
    // the next order statistic: the next non-empty bin of the same 22-bit prefix, else the
    // smallest key above the prefix block
    const uint32_t b0 = 2u * threadIdx.x, b1 = b0 + 1u;
    uint32_t nb = 0xffffffffu;
    if (b1 > p.bin && gh[b1]) nb = b1;
    if (b0 > p.bin && gh[b0]) nb = b0;
    if (nb != 0xffffffffu) atomicMin(&s_next, nb);
    __syncthreads();
    key_hi = s_next != 0xffffffffu ? (prefix | s_next) : min_above;
  }
  const float A = fkey_inv(key), B = fkey_inv(key_hi);
  const float diff = fsub(B, A);
  const float thr = g >= 0.5f ? fsub(B, fmul(diff, fsub(1.0f, g))) : fadd(A, fmul(diff, g));

  // push.py:325-326 upsampled * (img_y == target_class + 1); helpers.py:51 mask = map >= thr.
  const TL* L = label + static_cast<size_t>(li) * n;
  const long long cls = static_cast<long long>(target_class[map]) + 1;
  auto hit = [&](int r, int c) -> bool {
    const size_t i = static_cast<size_t>(r) * W + c;
    const float u = U[i];
    const float v = label_value(L, i, lut, lut_size) == cls ? u : fmul(u, 0.0f);
    return v >= thr;
  };
  auto row_any = [&](int r, int c0, int c1) -> bool {  // np.amax(mask[r, c0:c1]) > 0.5
    c1 = c1 > W ? W : c1;
    bool f = false;
    for (int c = c0 + static_cast<int>(threadIdx.x); c < c1; c += kBoxThreads) f = f || hit(r, c);
    return __syncthreads_or(f) != 0;
  };
  auto col_any = [&](int c, int r0, int r1) -> bool {  // np.amax(mask[r0:r1, c]) > 0.5
    r1 = r1 > H ? H : r1;
    bool f = false;
    for (int r = r0 + static_cast<int>(threadIdx.x); r < r1; r += kBoxThreads) f = f || hit(r, c);
    return __syncthreads_or(f) != 0;
  };
  // helpers.py:53-75: the four sides in order, each re-tested until it fails once.
  bool st0 = false, st1 = false, st2 = false, st3 = false;
  while (!(st0 && st1 && st2 && st3)) {
    if (!st0 && sh > 0 && row_any(sh - 1, sw, ew + 1)) --sh; else st0 = true;
    if (!st1 && eh < H - 1 && row_any(eh + 1, sw, ew + 1)) ++eh; else st1 = true;
    if (!st2 && sw > 0 && col_any(sw - 1, sh, eh + 1)) --sw; else st2 = true;
    if (!st3 && ew < W - 1 && col_any(ew + 1, sh, eh + 1)) ++ew; else st3 = true;
  }
  // helpers.py:77-82
  sh = sh - margin > 0 ? sh - margin : 0;
  sw = sw - margin > 0 ? sw - margin : 0;
  eh = eh + margin < H - 1 ? eh + margin : H - 1;
  ew = ew + margin < W - 1 ? ew + margin : W - 1;
  if (threadIdx.x == 0) {
    thr_out[map] = thr;
    box_out[4 * map + 0] = sh;
    box_out[4 * map + 1] = eh + 1;
    box_out[4 * map + 2] = sw;
    box_out[4 * map + 3] = ew + 1;
  }
}

// Select histograms and state ([m][2048] u32 | [m][8] u32): one grow-only block per (device,
// stream), reused by later calls on that stream (kernels on one stream are ordered), so a call is
// only kernel launches and can be captured in a HIP graph once the block exists.
void* select_scratch(size_t need, hipStream_t s, int* status) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, std::pair<void*, size_t>> blocks;
  int dev = 0;
  *status = PROTOSEG_OK;
  if (hipGetDevice(&dev) != hipSuccess) {
    *status = check_launch("hipGetDevice");
    return nullptr;
  }
  std::lock_guard<std::mutex> lock(mu);
  auto& b = blocks[{dev, s}];
  if (b.second < need) {
    if (b.first && (hipStreamSynchronize(s) != hipSuccess || hipFree(b.first) != hipSuccess)) {
      *status = check_launch("bound-box scratch regrow");
      return nullptr;
    }
    b = {nullptr, 0};
    const size_t bytes = need < (1u << 20) ? (1u << 20) : need;
    const hipError_t e = hipMalloc(&b.first, bytes);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      b = {nullptr, 0};
      *status = fail(PROTOSEG_ERR_HIP, "hipMalloc (bound-box scratch, %zu B): %s", bytes, hipGetErrorString(e));
      return nullptr;
    }
    b.second = bytes;
  }
  return b.first;
}

}  // namespace

}  // namespace protoseg

using namespace protoseg;

extern "C" int protoseg_act_upsample(const float* dist, int m, int h, int w, int H, int W, int act_kind, float eps,
                                     float max_dist, float* act, float* up, protoseg_stream_t stream) {
  if (!dist || !act || !up) return fail(PROTOSEG_ERR_INVALID, "dist, act and up must be non-null");
  if (m <= 0 || h <= 0 || w <= 0 || H <= 0 || W <= 0)
    return fail(PROTOSEG_ERR_INVALID, "bad shape m=%d h=%d w=%d H=%d W=%d", m, h, w, H, W);
  if (m > 65535) return fail(PROTOSEG_ERR_UNSUPPORTED, "m=%d H=%d above the grid limit", m, H);
  if (act_kind < PROTOSEG_ACT_LOG || act_kind > PROTOSEG_ACT_IDENTITY)
    return fail(PROTOSEG_ERR_INVALID, "act_kind %d", act_kind);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const size_t n = static_cast<size_t>(m) * h * w;
  const int blocks = static_cast<int>(ceil_div(static_cast<long long>(n), 256) < 4096 ? ceil_div(n, 256) : 4096);
  hipLaunchKernelGGL(act_kernel, dim3(blocks), dim3(256), 0, s, dist, n, act_kind, eps, max_dist, act);
  int rc = check_launch("act_kernel");
  if (rc) return rc;
  // cv::resize: inv_scale = dsize / ssize, scale = 1 / inv_scale (both f64).
  const double scale_x = 1.0 / (static_cast<double>(W) / static_cast<double>(w));
  const double scale_y = 1.0 / (static_cast<double>(H) / static_cast<double>(h));
  // Output rows per tile: the source rows they touch (<= rows * h / H + 5) must fit the LDS window.
  long long rows = (static_cast<long long>(kUpMaxSrcRows - 6) * H) / h;
  rows = rows < 1 ? 1 : rows > kUpMaxRows ? kUpMaxRows : rows;
  if (W % 4 == 0 && (reinterpret_cast<uintptr_t>(up) & 15u) == 0) {
    // the float4 path: the source rows of a tile (<= rows4 * h / H + 5) fit its 16-row window
    long long rows4 = (static_cast<long long>(kUp4MaxSrcRows - 6) * H) / h;
    rows4 = rows4 < 1 ? 1 : rows4 > kUpMaxRows ? kUpMaxRows : rows4;
    const dim3 grid4(static_cast<unsigned>(ceil_div(W, kUp4Cols)), static_cast<unsigned>(ceil_div(H, rows4)), m);
    hipLaunchKernelGGL(cubic_upsample4_kernel, grid4, dim3(kUpThreads), 0, s, act, h, w, H, W, static_cast<int>(rows4),
                       scale_y, scale_x, up);
    return check_launch("cubic_upsample4_kernel");
  }
  const dim3 grid(static_cast<unsigned>(ceil_div(W, kUpThreads)), static_cast<unsigned>(ceil_div(H, rows)), m);
  hipLaunchKernelGGL(cubic_upsample_kernel, grid, dim3(kUpThreads), 0, s, act, h, w, H, W, static_cast<int>(rows),
                     scale_y, scale_x, up);
  return check_launch("cubic_upsample_kernel");
}

extern "C" int protoseg_bound_boxes(const float* up, int m, int H, int W, const void* label, int label_dtype,
                                    int n_label, const int32_t* label_index, const int32_t* lut, int lut_size,
                                    const int32_t* target_class, const int32_t* rf_box, float percentile, int margin,
                                    float* threshold, int32_t* box, protoseg_stream_t stream) {
  if (!up || !label || !target_class || !rf_box || !threshold || !box)
    return fail(PROTOSEG_ERR_INVALID, "up, label, target_class, rf_box, threshold and box must be non-null");
  if (m <= 0 || H <= 0 || W <= 0 || n_label <= 0)
    return fail(PROTOSEG_ERR_INVALID, "bad shape m=%d H=%d W=%d n_label=%d", m, H, W, n_label);
  if (static_cast<long long>(H) * W >= (1ll << 32)) return fail(PROTOSEG_ERR_UNSUPPORTED, "map too large");
  if (!(percentile >= 0.f && percentile <= 100.f)) return fail(PROTOSEG_ERR_INVALID, "percentile must be in [0, 100]");
  if (margin < 0) return fail(PROTOSEG_ERR_INVALID, "margin must be >= 0");
  if (lut && lut_size <= 0) return fail(PROTOSEG_ERR_INVALID, "lut_size must be > 0");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (label_dtype != PROTOSEG_I64 && label_dtype != PROTOSEG_I32 && label_dtype != PROTOSEG_U8)
    return fail(PROTOSEG_ERR_UNSUPPORTED, "label_dtype %d", label_dtype);
  if (m > 65535) return fail(PROTOSEG_ERR_UNSUPPORTED, "m=%d maps per call", m);
  const size_t n = static_cast<size_t>(H) * W;
  const size_t hist_bytes = static_cast<size_t>(m) * kHistBins * sizeof(uint32_t);
  const size_t state_bytes = static_cast<size_t>(m) * kSelState * sizeof(uint32_t);
  // candidate list: up to 1/8 of each map (the chosen 11-bit bin is a quarter-octave of values)
  const size_t cap = ceil_div(ceil_div(n, static_cast<size_t>(8)), static_cast<size_t>(4)) * 4;  // 16-B aligned lists
  int st = PROTOSEG_OK;
  // chunks per map: about kSelTarget histogram workgroups in all, each >= kSelMinChunk elements
  size_t chunks = ceil_div(static_cast<size_t>(kSelTarget), static_cast<size_t>(m));
  const size_t max_chunks = ceil_div(n, static_cast<size_t>(kSelMinChunk));
  chunks = chunks > max_chunks ? max_chunks : chunks;
  chunks = chunks < 1 ? 1 : chunks;
  const size_t chunk = ceil_div(ceil_div(n, chunks), static_cast<size_t>(4)) * 4;  // float4-aligned chunk starts
  chunks = ceil_div(n, chunk);
  const size_t cand_bytes = static_cast<size_t>(m) * cap * sizeof(float);
  const size_t rows_bytes = static_cast<size_t>(m) * chunks * kHistBins * sizeof(uint32_t);
  void* scratch = select_scratch(hist_bytes + state_bytes + cand_bytes + rows_bytes, s, &st);
  if (!scratch) return st;
  uint32_t* hist = static_cast<uint32_t*>(scratch);
  uint32_t* state = hist + static_cast<size_t>(m) * kHistBins;
  float* cand = reinterpret_cast<float*>(state + static_cast<size_t>(m) * kSelState);
  uint32_t* rows = reinterpret_cast<uint32_t*>(cand + static_cast<size_t>(m) * cap);
  const dim3 hgrid(static_cast<unsigned>(chunks), m);
  hipLaunchKernelGGL(select_init_kernel, dim3(m), dim3(256), 0, s, n, percentile, hist, state);
  if (int e = check_launch("select_init_kernel")) return e;
  hipLaunchKernelGGL(select_hist_kernel<0>, hgrid, dim3(kHistThreads), 0, s, up, n, chunk, cand, cap, hist, rows, state);
  if (int e = check_launch("select_hist_kernel<0>")) return e;
  hipLaunchKernelGGL(select_step_kernel, dim3(m), dim3(kBoxThreads), 0, s, 0, cap, hist, state);
  if (int e = check_launch("select_step_kernel")) return e;
  hipLaunchKernelGGL(select_hist_kernel<1>, hgrid, dim3(kHistThreads), 0, s, up, n, chunk, cand, cap, hist, rows, state);
  if (int e = check_launch("select_hist_kernel<1>")) return e;
  hipLaunchKernelGGL(select_step_kernel, dim3(m), dim3(kBoxThreads), 0, s, 1, cap, hist, state);
  if (int e = check_launch("select_step_kernel")) return e;
  hipLaunchKernelGGL(select_hist_kernel<2>, hgrid, dim3(kHistThreads), 0, s, up, n, chunk, cand, cap, hist, rows, state);
  if (int e = check_launch("select_hist_kernel<2>")) return e;
  switch (label_dtype) {
    case PROTOSEG_I64:
      hipLaunchKernelGGL(bound_box_kernel<int64_t>, dim3(m), dim3(kBoxThreads), 0, s, up, H, W,
                         static_cast<const int64_t*>(label), n_label, label_index, lut, lut_size, target_class, rf_box,
                         percentile, margin, hist, state, threshold, box);
      break;
    case PROTOSEG_I32:
      hipLaunchKernelGGL(bound_box_kernel<int32_t>, dim3(m), dim3(kBoxThreads), 0, s, up, H, W,
                         static_cast<const int32_t*>(label), n_label, label_index, lut, lut_size, target_class, rf_box,
                         percentile, margin, hist, state, threshold, box);
      break;
    default:
      hipLaunchKernelGGL(bound_box_kernel<uint8_t>, dim3(m), dim3(kBoxThreads), 0, s, up, H, W,
                         static_cast<const uint8_t*>(label), n_label, label_index, lut, lut_size, target_class, rf_box,
                         percentile, margin, hist, state, threshold, box);
      break;
  }
  return check_launch("bound_box_kernel");
}
