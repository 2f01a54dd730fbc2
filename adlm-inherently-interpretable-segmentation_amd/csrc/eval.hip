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
  const dim3 grid(static_cast<unsigned>(ceil_div(W, kEvalThreads)), H, B);
  auto* c = reinterpret_cast<unsigned long long*>(counts);
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
