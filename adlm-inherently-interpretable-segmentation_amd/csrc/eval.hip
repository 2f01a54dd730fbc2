// eval.hip — segmentation evaluation counts of segmentation/eval_valid.py:159-197 on gfx950.
//
// The reference upsamples every image's logits [K, h, w] and distances [P, h, w] to the label
// resolution (F.interpolate, bilinear, align_corners=False: a [190, 1024, 2048] f32 tensor of
// 1.6 GB per Cityscapes image), takes argmax / argmin, copies both to the host and counts with
// numpy per class and per prototype. Here one kernel does it per output pixel, with the
// interpolation evaluated on the fly from the low-resolution maps (never materialised):
//   thread = output pixel; pred = argmax_k of the bilinear logits, nearest = argmin_p of the
//   bilinear distances; counts aggregated per wave (ballot by key) into LDS, then per workgroup
//   into the global int64 counters with atomics (integer adds: order-independent, exact).
#include <type_traits>

#include "protoseg_device.h"
#include "protoseg_host.h"

namespace protoseg {

namespace {

constexpr int kEvalThreads = 256;
constexpr int kEvalMaxK = 64;
constexpr int kEvalMaxP = 4096;

// torch area_pixel_compute_source_index (align_corners=False, linear): the source coordinate of
// output index dst for scale = in / out, clamped at 0; then the upsample_bilinear2d neighbours.
struct Lin {
  int i0, di;
  float l0, l1;
};
__device__ __forceinline__ Lin lin_of(float scale, int dst, int in) {
  float src = scale * (static_cast<float>(dst) + 0.5f) - 0.5f;
  src = src < 0.f ? 0.f : src;
  Lin r;
  r.i0 = static_cast<int>(src);
  r.di = r.i0 < in - 1 ? 1 : 0;
  r.l1 = src - static_cast<float>(r.i0);
  r.l0 = 1.f - r.l1;
  return r;
}

// Adds 1 to counter[key] for every lane with valid set, one LDS atomic per distinct key of the
// wave (labels and predictions are spatially coherent, so a wave holds few distinct keys).
__device__ __forceinline__ void wave_count(unsigned* counter, int key, bool valid) {
  unsigned long long pending = __ballot(valid);
  while (pending) {
    const int leader = __ffsll(static_cast<long long>(pending)) - 1;
    const int k = __shfl(key, leader);
    const unsigned long long m = __ballot(valid && key == k);
    if ((threadIdx.x & 63) == static_cast<unsigned>(leader)) atomicAdd(&counter[k], static_cast<unsigned>(__popcll(m)));
    pending &= ~m;
  }
}

// Adds the wave's sum of v to counter[key] (one LDS atomic per wave).
__device__ __forceinline__ void wave_sum_to(unsigned* counter, int key, unsigned v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  if ((threadIdx.x & 63) == 0 && v) atomicAdd(&counter[key], v);
}

// counts (int64): [0] correct, [1] total, [2, 2+K) I, [2+K, 2+2K) U, [2+2K, 2+2K+P) per-prototype.
template <typename TL>
__global__ __launch_bounds__(kEvalThreads) void eval_seg_kernel(const float* __restrict__ logits,
                                                                const float* __restrict__ dist, int h, int w, int K,
                                                                int P, const TL* __restrict__ ann, int H, int W,
                                                                const int32_t* __restrict__ lut, int lut_size,
                                                                const int32_t* __restrict__ proto_class,
                                                                unsigned long long* __restrict__ counts) {
  __shared__ unsigned s_cnt[2 + 2 * kEvalMaxK + kEvalMaxP];
  const int ncnt = 2 + 2 * K + (dist ? P : 0);
  for (int i = threadIdx.x; i < ncnt; i += kEvalThreads) s_cnt[i] = 0u;
  __syncthreads();
  const int b = blockIdx.z, y = blockIdx.y;
  const int x = blockIdx.x * kEvalThreads + threadIdx.x;
  const bool inside = x < W;
  // reference scale: (float)input_size / output_size (area_pixel_compute_scale)
  const Lin ly = lin_of(static_cast<float>(h) / static_cast<float>(H), y, h);
  const Lin lx = lin_of(static_cast<float>(w) / static_cast<float>(W), inside ? x : 0, w);
  // upsample_bilinear2d: h0l * (w0l * v00 + w1l * v01) + h1l * (w0l * v10 + w1l * v11)
  auto bilinear = [&](float v00, float v01, float v10, float v11) {
    return ly.l0 * (lx.l0 * v00 + lx.l1 * v01) + ly.l1 * (lx.l0 * v10 + lx.l1 * v11);
  };
  int pred = 0;
  {
    const float* lb = logits + static_cast<size_t>(b) * h * w * K;
    const float* r0 = lb + (static_cast<size_t>(ly.i0) * w) * K;
    const float* r1 = lb + (static_cast<size_t>(ly.i0 + ly.di) * w) * K;
    const int c0 = lx.i0 * K, c1 = (lx.i0 + lx.di) * K;
    float best = -INFINITY;
    for (int k = 0; k < K; ++k) {
      const float v = bilinear(r0[c0 + k], r0[c1 + k], r1[c0 + k], r1[c1 + k]);
      if (v > best || k == 0) {  // torch.argmax: first maximal index
        best = v;
        pred = k;
      }
    }
  }
  long long a = 0;
  if (inside) {
    a = static_cast<long long>(ann[(static_cast<size_t>(b) * H + y) * W + x]);
    if (lut) a = (a >= 0 && a < lut_size) ? lut[a] : 0;
  }
  const bool labelled = inside && a != 0;
  const bool hit = labelled && a - 1 == pred;
  wave_count(s_cnt, 0, hit);       // correct (eval_valid.py:178)
  wave_count(s_cnt, 1, labelled);  // total (180)
  // I[c] and U[c] (182-189): I[pred] for hits; U[pred] for labelled pixels; U[ann-1] when it
  // differs from pred.
  wave_count(s_cnt + 2, pred, hit);
  wave_count(s_cnt + 2 + K, pred, labelled);
  const int gt = static_cast<int>(a - 1);
  wave_count(s_cnt + 2 + K, gt, labelled && gt != pred && gt >= 0 && gt < K);
  if (dist) {  // nearest prototype (174) counted when its class equals pred (191-197)
    const float* db = dist + static_cast<size_t>(b) * P * h * w;
    const size_t o00 = static_cast<size_t>(ly.i0) * w + lx.i0, o01 = o00 + lx.di;
    const size_t o10 = static_cast<size_t>(ly.i0 + ly.di) * w + lx.i0, o11 = o10 + lx.di;
    const size_t plane = static_cast<size_t>(h) * w;
    float best = INFINITY;
    int near = 0;
    for (int p = 0; p < P; ++p) {
      const float* dp = db + p * plane;
      const float v = bilinear(dp[o00], dp[o01], dp[o10], dp[o11]);
      if (v < best || p == 0) {  // torch.argmin: first minimal index
        best = v;
        near = p;
      }
    }
    wave_count(s_cnt + 2 + 2 * K, near, inside && proto_class[near] == pred);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < ncnt; i += kEvalThreads)
    if (s_cnt[i]) atomicAdd(&counts[i], static_cast<unsigned long long>(s_cnt[i]));
}

// Row-group variant for upsampling (H >= h): every output row y with the same top source row
// i0 shares the two horizontally interpolated source rows, so a thread (one output column)
// computes a = w0 * v(i0, j0) + w1 * v(i0, j1) and b = (the same on row i0 + di) once per class
// / prototype and evaluates h0 * a + h1 * b — torch's expression, term for term — for up to
// kEvalRows output rows at once: 4 loads per class serve kEvalRows pixels instead of one.
// Grid: (column tiles, source rows h, images); a group with more rows runs in chunks.
constexpr int kEvalRows = 8;
constexpr int kEvalBatch = 4;  // classes / prototypes whose loads are in flight together

template <typename TL>
__global__ __launch_bounds__(kEvalThreads) void eval_rows_kernel(const float* __restrict__ logits,
                                                                 const float* __restrict__ dist, int h, int w, int K,
                                                                 int P, const TL* __restrict__ ann, int H, int W,
                                                                 const int32_t* __restrict__ lut, int lut_size,
                                                                 const int32_t* __restrict__ proto_class,
                                                                 unsigned long long* __restrict__ counts) {
  __shared__ unsigned s_cnt[2 + 2 * kEvalMaxK + kEvalMaxP];
  const int ncnt = 2 + 2 * K + (dist ? P : 0);
  for (int i = threadIdx.x; i < ncnt; i += kEvalThreads) s_cnt[i] = 0u;
  __syncthreads();
  const int b = blockIdx.z, i0 = blockIdx.y;
  const int x = blockIdx.x * kEvalThreads + threadIdx.x;
  const bool inside = x < W;
  const float sy = static_cast<float>(h) / static_cast<float>(H);
  // output rows whose top source row is i0 (monotone in y): a guess, then exact lin_of checks
  int y0 = static_cast<int>((static_cast<float>(i0) + 0.5f) / sy - 0.5f) - 2;
  y0 = y0 < 0 ? 0 : y0;
  while (y0 > 0 && lin_of(sy, y0, h).i0 >= i0) --y0;
  while (y0 < H && lin_of(sy, y0, h).i0 < i0) ++y0;
  int y1 = y0;
  while (y1 < H && lin_of(sy, y1, h).i0 == i0) ++y1;
  const int di = i0 < h - 1 ? 1 : 0;
  const Lin lx = lin_of(static_cast<float>(w) / static_cast<float>(W), inside ? x : 0, w);
  const int c0 = lx.i0, c1 = lx.i0 + lx.di;
  unsigned n_hit = 0, n_lab = 0;
  for (int ya = y0; ya < y1; ya += kEvalRows) {
    const int nr = y1 - ya < kEvalRows ? y1 - ya : kEvalRows;
    float l0[kEvalRows], l1[kEvalRows];
#pragma unroll
    for (int r = 0; r < kEvalRows; ++r) {
      const Lin ly = lin_of(sy, r < nr ? ya + r : ya, h);
      l0[r] = ly.l0;
      l1[r] = ly.l1;
    }
    int pred[kEvalRows];
    {
      // wave-uniform class base + 32-bit per-lane offsets; next class prefetched
      const float* lb = logits + static_cast<size_t>(b) * h * w * K;
      const unsigned q00 = static_cast<unsigned>((i0 * w + c0) * K), q01 = static_cast<unsigned>((i0 * w + c1) * K);
      const unsigned q10 = static_cast<unsigned>(((i0 + di) * w + c0) * K);
      const unsigned q11 = static_cast<unsigned>(((i0 + di) * w + c1) * K);
      float best[kEvalRows];
      float u00 = lb[q00], u01 = lb[q01], u10 = lb[q10], u11 = lb[q11];
      {
        const float a = lx.l0 * u00 + lx.l1 * u01;
        const float bb = lx.l0 * u10 + lx.l1 * u11;
#pragma unroll
        for (int r = 0; r < kEvalRows; ++r) {
          best[r] = l0[r] * a + l1[r] * bb;
          pred[r] = 0;
        }
      }
      // the other classes kEvalBatch at a time: the batch's loads (clamped, pinned) in flight
      // together, then evaluated in class order (one round trip per batch, not per class)
      for (int k0 = 1; k0 < K; k0 += kEvalBatch) {
        float uu[kEvalBatch][4];
#pragma unroll
        for (int j = 0; j < kEvalBatch; ++j) {
          const float* ln = lb + (k0 + j < K ? k0 + j : K - 1);
          uu[j][0] = ln[q00];
          uu[j][1] = ln[q01];
          uu[j][2] = ln[q10];
          uu[j][3] = ln[q11];
        }
#pragma unroll
        for (int j = 0; j < kEvalBatch; ++j) pin_batch(uu[j]);
#pragma unroll
        for (int j = 0; j < kEvalBatch; ++j) {
          if (k0 + j >= K) break;  // uniform
          const float a = lx.l0 * uu[j][0] + lx.l1 * uu[j][1];
          const float bb = lx.l0 * uu[j][2] + lx.l1 * uu[j][3];
#pragma unroll
          for (int r = 0; r < kEvalRows; ++r) {
            const float v = l0[r] * a + l1[r] * bb;
            if (v > best[r]) {  // torch.argmax: first maximal index
              best[r] = v;
              pred[r] = k0 + j;
            }
          }
        }
      }
    }
    int near[kEvalRows];
    if (dist) {
      // wave-uniform plane base + 32-bit per-lane offsets (saddr loads); the next prototype's
      // four values are loaded before the current one is evaluated
      const float* db = dist + static_cast<size_t>(b) * P * h * w;
      const unsigned o00 = static_cast<unsigned>(i0 * w + c0), o01 = static_cast<unsigned>(i0 * w + c1);
      const unsigned o10 = static_cast<unsigned>((i0 + di) * w + c0), o11 = static_cast<unsigned>((i0 + di) * w + c1);
      const size_t plane = static_cast<size_t>(h) * w;
      float best[kEvalRows];
      float v00 = db[o00], v01 = db[o01], v10 = db[o10], v11 = db[o11];
      {
        const float a = lx.l0 * v00 + lx.l1 * v01;
        const float bb = lx.l0 * v10 + lx.l1 * v11;
#pragma unroll
        for (int r = 0; r < kEvalRows; ++r) {
          best[r] = l0[r] * a + l1[r] * bb;
          near[r] = 0;
        }
      }
      for (int p0 = 1; p0 < P; p0 += kEvalBatch) {  // batched as the classes
        float vv[kEvalBatch][4];
#pragma unroll
        for (int j = 0; j < kEvalBatch; ++j) {
          const float* dn = db + static_cast<size_t>(p0 + j < P ? p0 + j : P - 1) * plane;
          vv[j][0] = dn[o00];
          vv[j][1] = dn[o01];
          vv[j][2] = dn[o10];
          vv[j][3] = dn[o11];
        }
#pragma unroll
        for (int j = 0; j < kEvalBatch; ++j) pin_batch(vv[j]);
#pragma unroll
        for (int j = 0; j < kEvalBatch; ++j) {
          if (p0 + j >= P) break;  // uniform
          const float a = lx.l0 * vv[j][0] + lx.l1 * vv[j][1];
          const float bb = lx.l0 * vv[j][2] + lx.l1 * vv[j][3];
#pragma unroll
          for (int r = 0; r < kEvalRows; ++r) {
            const float v = l0[r] * a + l1[r] * bb;
            if (v < best[r]) {  // torch.argmin: first minimal index
              best[r] = v;
              near[r] = p0 + j;
            }
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < kEvalRows; ++r) {
      if (r >= nr) break;  // nr is block-uniform
      const int y = ya + r;
      long long a = 0;
      if (inside) {
        a = static_cast<long long>(ann[(static_cast<size_t>(b) * H + y) * W + x]);
        if (lut) a = (a >= 0 && a < lut_size) ? lut[a] : 0;
      }
      const bool labelled = inside && a != 0;
      const bool hit = labelled && a - 1 == pred[r];
      n_hit += hit;
      n_lab += labelled;
      const int gt = static_cast<int>(a - 1);
      // keyed counts: one LDS atomic per lane (same-key lanes serialise in the LDS unit; measured
      // cheaper than a ballot loop over the wave's distinct keys and than per-thread key runs)
      if (hit) atomicAdd(&s_cnt[2 + pred[r]], 1u);
      if (labelled) atomicAdd(&s_cnt[2 + K + pred[r]], 1u);
      if (labelled && gt != pred[r] && gt >= 0 && gt < K) atomicAdd(&s_cnt[2 + K + gt], 1u);
      if (dist && inside && proto_class[near[r]] == pred[r]) atomicAdd(&s_cnt[2 + 2 * K + near[r]], 1u);
    }
  }
  wave_sum_to(s_cnt, 0, n_hit);
  wave_sum_to(s_cnt, 1, n_lab);
  __syncthreads();
  for (int i = threadIdx.x; i < ncnt; i += kEvalThreads)
    if (s_cnt[i]) atomicAdd(&counts[i], static_cast<unsigned long long>(s_cnt[i]));
}

}  // namespace

}  // namespace protoseg

using namespace protoseg;

extern "C" int protoseg_eval_counts(const float* logits, const float* dist, int B, int h, int w, int K, int P,
                                    const void* ann, int ann_dtype, int H, int W, const int32_t* lut, int lut_size,
                                    const int32_t* proto_class, int64_t* counts, protoseg_stream_t stream) {
  if (!logits || !ann || !counts) return fail(PROTOSEG_ERR_INVALID, "logits, ann and counts must be non-null");
  if (dist && !proto_class) return fail(PROTOSEG_ERR_INVALID, "dist needs proto_class");
  if (B <= 0 || h <= 0 || w <= 0 || K <= 0 || H <= 0 || W <= 0 || (dist && P <= 0))
    return fail(PROTOSEG_ERR_INVALID, "bad shape B=%d h=%d w=%d K=%d P=%d H=%d W=%d", B, h, w, K, P, H, W);
  if (K > kEvalMaxK) return fail(PROTOSEG_ERR_UNSUPPORTED, "K=%d > %d", K, kEvalMaxK);
  if (dist && P > kEvalMaxP) return fail(PROTOSEG_ERR_UNSUPPORTED, "P=%d > %d", P, kEvalMaxP);
  if (lut && lut_size <= 0) return fail(PROTOSEG_ERR_INVALID, "lut_size must be > 0");
  if (H > 65535 || B > 65535) return fail(PROTOSEG_ERR_UNSUPPORTED, "H=%d / B=%d per call", H, B);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  auto* c = reinterpret_cast<unsigned long long*>(counts);
  if (H >= h && h <= 65535) {  // upsampling: row-group kernel, one workgroup per (column tile, source row)
    const dim3 grid(static_cast<unsigned>(ceil_div(W, kEvalThreads)), h, B);
    switch (ann_dtype) {
      case PROTOSEG_I64:
        hipLaunchKernelGGL(eval_rows_kernel<int64_t>, grid, dim3(kEvalThreads), 0, s, logits, dist, h, w, K, P,
                           static_cast<const int64_t*>(ann), H, W, lut, lut_size, proto_class, c);
        break;
      case PROTOSEG_I32:
        hipLaunchKernelGGL(eval_rows_kernel<int32_t>, grid, dim3(kEvalThreads), 0, s, logits, dist, h, w, K, P,
                           static_cast<const int32_t*>(ann), H, W, lut, lut_size, proto_class, c);
        break;
      case PROTOSEG_U8:
        hipLaunchKernelGGL(eval_rows_kernel<uint8_t>, grid, dim3(kEvalThreads), 0, s, logits, dist, h, w, K, P,
                           static_cast<const uint8_t*>(ann), H, W, lut, lut_size, proto_class, c);
        break;
      default:
        return fail(PROTOSEG_ERR_UNSUPPORTED, "ann_dtype %d", ann_dtype);
    }
    return check_launch("eval_rows_kernel");
  }
  const dim3 grid(static_cast<unsigned>(ceil_div(W, kEvalThreads)), H, B);
  switch (ann_dtype) {
    case PROTOSEG_I64:
      hipLaunchKernelGGL(eval_seg_kernel<int64_t>, grid, dim3(kEvalThreads), 0, s, logits, dist, h, w, K, P,
                         static_cast<const int64_t*>(ann), H, W, lut, lut_size, proto_class, c);
      break;
    case PROTOSEG_I32:
      hipLaunchKernelGGL(eval_seg_kernel<int32_t>, grid, dim3(kEvalThreads), 0, s, logits, dist, h, w, K, P,
                         static_cast<const int32_t*>(ann), H, W, lut, lut_size, proto_class, c);
      break;
    case PROTOSEG_U8:
      hipLaunchKernelGGL(eval_seg_kernel<uint8_t>, grid, dim3(kEvalThreads), 0, s, logits, dist, h, w, K, P,
                         static_cast<const uint8_t*>(ann), H, W, lut, lut_size, proto_class, c);
      break;
    default:
      return fail(PROTOSEG_ERR_UNSUPPORTED, "ann_dtype %d", ann_dtype);
  }
  return check_launch("eval_seg_kernel");
}
