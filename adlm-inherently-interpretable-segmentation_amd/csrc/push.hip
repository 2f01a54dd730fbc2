// push.hip — prototype push (nearest-patch projection) on gfx950.
//
// Reference: segmentation/push.py:24-158 (push_prototypes) and 162-280
// (update_prototypes_on_image, argmin core). The reference moves the distance map of every
// image to the host and runs (a) a 2M-iteration Python loop mapping pixels to patch sets,
// (b) a per-prototype gather + np.argmin. Here both stay on the device:
//   patch_mask_kernel   label map -> uint32 class bitmask per patch (push.py:184-186, 214-223)
//   push_argmin_kernel  fused distance + masked per-prototype min key (push.py:249-263)
//   push_merge_kernel   strict-'<' fold in image order + winner gather (push.py:265-281)
#include "protoseg_device.h"
#include "protoseg_host.h"

namespace protoseg {

namespace {

constexpr int kArgminWaves = 4;

template <typename TL>
__global__ __launch_bounds__(256) void patch_mask_kernel(const TL* __restrict__ label, int H, int W, int h, int w,
                                                         const int32_t* __restrict__ lut, int lut_size,
                                                         uint32_t* __restrict__ mask) {
  extern __shared__ uint32_t smask[];  // [w]
  const int pi = blockIdx.x;
  const int img = blockIdx.y;
  // push.py:201-202: patch_height = img_height / model_output_height (float64)
  const double ph = static_cast<double>(H) / static_cast<double>(h);
  const double pw = static_cast<double>(W) / static_cast<double>(w);
  for (int q = threadIdx.x; q < w; q += blockDim.x) smask[q] = 0u;
  __syncthreads();
  // Rows of this patch row: push.py:217 patch_i = int(pixel_i / patch_height).
  int i0 = static_cast<int>(floor(pi * ph)) - 2;
  int i1 = static_cast<int>(ceil((pi + 1) * ph)) + 2;
  i0 = i0 < 0 ? 0 : i0;
  i1 = i1 > H ? H : i1;
  const TL* L = label + static_cast<size_t>(img) * H * W;
  for (int col = threadIdx.x; col < W; col += blockDim.x) {
    const int pj = static_cast<int>(static_cast<double>(col) / pw);  // push.py:219
    uint32_t bits = 0u;
    for (int i = i0; i < i1; ++i) {
      if (static_cast<int>(static_cast<double>(i) / ph) != pi) continue;
      const long long raw = static_cast<long long>(L[static_cast<size_t>(i) * W + col]);
      long long c = raw;
      if (lut) {
        if (raw < 0 || raw >= lut_size) continue;
        c = lut[raw];
      }
      if (c > 0 && c <= 32) bits |= 1u << (c - 1);  // push.py:222-223: class c -> key c-1
    }
    if (bits && pj < w) atomicOr(&smask[pj], bits);
  }
  __syncthreads();
  for (int q = threadIdx.x; q < w; q += blockDim.x)
    mask[static_cast<size_t>(img) * h * w + static_cast<size_t>(pi) * w + q] = smask[q];
}

// Layout B tiles (pixel on the register rows, prototype on the lane): the per-prototype
// minimum over pixels is an in-register min plus one half-wave exchange.
// key = (float_bits(d) << 32) | patch — d >= 0 after relu, so the bit pattern orders like d
// and ties resolve to the lowest patch index.
template <int NC>
__global__ __launch_bounds__(kArgminWaves * 64) void push_argmin_kernel(
    const float* __restrict__ x, int HW, const float* __restrict__ protos, int P,
    const int32_t* __restrict__ proto_class, const uint32_t* __restrict__ mask,
    unsigned long long* __restrict__ keys) {
  constexpr int C = NC * 32;
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5, wave = threadIdx.x >> 6;
  const int pt = blockIdx.x;
  const int img = blockIdx.z;
  const int p = pt * 32 + j;
  const bool pvalid = p < P;
  float pv[NC][16];
#pragma unroll
  for (int ct = 0; ct < NC; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r)
      pv[ct][r] = pvalid ? protos[static_cast<size_t>(p) * C + ct * 32 + acc_row(r, h)] : 0.f;
  float p2 = 0.f;
  if (pvalid) {
#pragma clang fp contract(off)
    for (int c = 0; c < C; ++c) {
      const float v = protos[static_cast<size_t>(p) * C + c];
      p2 += v * v;
    }
  }
  const int cls = pvalid ? proto_class[p] : -1;
  const bool active = cls >= 0 && cls < 32;
  // classes of this wave's 32 prototypes: a tile without any of them is skipped
  const uint32_t wave_classes = wave_or(active ? (1u << cls) : 0u);
  const float* xi = x + static_cast<size_t>(img) * C * HW;
  const uint32_t* mi = mask + static_cast<size_t>(img) * HW;

  unsigned long long best = ~0ull;
  const int ntiles = (HW + 31) / 32;
  for (int t = blockIdx.y * kArgminWaves + wave; t < ntiles; t += gridDim.y * kArgminWaves) {
    const int n = t * 32 + j;
    const bool valid = n < HW;
    float xv[NC][16];
    float x2 = 0.f;
#pragma unroll
    for (int ct = 0; ct < NC; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = xi[static_cast<size_t>(ct * 32 + acc_row(r, h)) * HW + (valid ? n : 0)];
        xv[ct][r] = valid ? v : 0.f;
        x2 = fmaf(xv[ct][r], xv[ct][r], x2);
      }
    x2 += __shfl_xor(x2, 32);
    const uint32_t mk0 = mi[valid ? n : 0];
    const uint32_t mk = valid ? mk0 : 0u;
    // skip tiles holding no patch of any class of this wave's prototypes
    if ((wave_or(mk) & wave_classes) == 0u) continue;

    f32x16 acc = zero16();
#pragma unroll
    for (int ct = 0; ct < NC; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc = mfma32(xv[ct][r], pv[ct][r], acc);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int nr = acc_row(r, h);
      const float x2n = __shfl(x2, nr);
      const uint32_t mkn = __shfl(mk, nr);
      const float d = l2_distance(x2n, p2, acc[r]);
      if (active && ((mkn >> cls) & 1u)) {
        const unsigned long long key =
            (static_cast<unsigned long long>(__float_as_uint(d)) << 32) | static_cast<uint32_t>(t * 32 + nr);
        best = key < best ? key : best;
      }
    }
  }
  const unsigned long long other = shfl_xor_u64(best, 32);
  best = other < best ? other : best;
  if (h == 0 && pvalid && best != ~0ull) atomicMin(&keys[static_cast<size_t>(img) * P + p], best);
}

// One wave per prototype: fold the batch's keys in image order (strict '<', push.py:265),
// then copy the winning feature vector (push.py:276-280).
__global__ __launch_bounds__(256) void push_merge_kernel(const unsigned long long* __restrict__ keys, int n_img,
                                                         long long first_img, const float* __restrict__ x, int C,
                                                         int hw, int P, float* __restrict__ gdist,
                                                         long long* __restrict__ gimg, int* __restrict__ gpatch,
                                                         float* __restrict__ gfmap) {
  const int p = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (p >= P) return;
  float best = gdist[p];
  int win = -1;
  uint32_t patch = 0;
  for (int img = 0; img < n_img; ++img) {
    const unsigned long long key = keys[static_cast<size_t>(img) * P + p];
    if (key == ~0ull) continue;  // no patch of the prototype's class (push.py:255-256)
    const float d = __uint_as_float(static_cast<uint32_t>(key >> 32));
    if (d < best) {
      best = d;
      win = img;
      patch = static_cast<uint32_t>(key);
    }
  }
  if (win < 0) return;
  if (lane == 0) {
    gdist[p] = best;
    gimg[p] = first_img + win;
    gpatch[p] = static_cast<int>(patch);
  }
  for (int c = lane; c < C; c += 64)
    gfmap[static_cast<size_t>(p) * C + c] = x[(static_cast<size_t>(win) * C + c) * hw + patch];
}

int nc_of_push(int C) { return C == 32 ? 1 : C == 64 ? 2 : C == 128 ? 4 : 0; }

}  // namespace

}  // namespace protoseg

using namespace protoseg;

extern "C" int protoseg_patch_class_mask(const void* label, int label_dtype, int n_img, int H_img, int W_img, int h,
                                         int w, const int32_t* lut, int lut_size, uint32_t* mask,
                                         protoseg_stream_t stream) {
  if (!label || !mask) return fail(PROTOSEG_ERR_INVALID, "label and mask must be non-null");
  if (n_img <= 0 || H_img <= 0 || W_img <= 0 || h <= 0 || w <= 0)
    return fail(PROTOSEG_ERR_INVALID, "bad shape n_img=%d H=%d W=%d h=%d w=%d", n_img, H_img, W_img, h, w);
  if (lut && lut_size <= 0) return fail(PROTOSEG_ERR_INVALID, "lut_size must be > 0");
  if (static_cast<size_t>(w) * 4 > kMaxLds) return fail(PROTOSEG_ERR_UNSUPPORTED, "w=%d too wide", w);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid(h, n_img);
  const size_t lds = static_cast<size_t>(w) * sizeof(uint32_t);
  switch (label_dtype) {
    case PROTOSEG_I64:
      hipLaunchKernelGGL(patch_mask_kernel<int64_t>, grid, dim3(256), lds, s, static_cast<const int64_t*>(label),
                         H_img, W_img, h, w, lut, lut_size, mask);
      break;
    case PROTOSEG_I32:
      hipLaunchKernelGGL(patch_mask_kernel<int32_t>, grid, dim3(256), lds, s, static_cast<const int32_t*>(label),
                         H_img, W_img, h, w, lut, lut_size, mask);
      break;
    case PROTOSEG_U8:
      hipLaunchKernelGGL(patch_mask_kernel<uint8_t>, grid, dim3(256), lds, s, static_cast<const uint8_t*>(label),
                         H_img, W_img, h, w, lut, lut_size, mask);
      break;
    default:
      return fail(PROTOSEG_ERR_UNSUPPORTED, "label_dtype %d", label_dtype);
  }
  return check_launch("patch_mask_kernel");
}

extern "C" int protoseg_push_argmin(const float* x, int n_img, int C, int h, int w, const float* protos, int P,
                                    const int32_t* proto_class, const uint32_t* mask, uint64_t* img_keys,
                                    protoseg_stream_t stream) {
  if (!x || !protos || !proto_class || !mask || !img_keys)
    return fail(PROTOSEG_ERR_INVALID, "null pointer argument");
  if (n_img <= 0 || h <= 0 || w <= 0 || P <= 0) return fail(PROTOSEG_ERR_INVALID, "bad shape");
  const int nc = nc_of_push(C);
  if (!nc) return fail(PROTOSEG_ERR_UNSUPPORTED, "C=%d", C);
  if (n_img > 65535) return fail(PROTOSEG_ERR_UNSUPPORTED, "n_img=%d per call", n_img);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(img_keys, 0xff, static_cast<size_t>(n_img) * P * sizeof(uint64_t), s) != hipSuccess)
    return check_launch("memset img_keys");
  const int HW = h * w;
  const int npt = static_cast<int>(ceil_div(P, 32));
  const long long ntiles = ceil_div(HW, 32);
  long long splits = 1024 / (static_cast<long long>(npt) * n_img);
  if (splits < 1) splits = 1;
  const long long need = ceil_div(ntiles, kArgminWaves);
  if (splits > need) splits = need;
  const dim3 grid(npt, static_cast<unsigned>(splits), n_img);
  auto* keys = reinterpret_cast<unsigned long long*>(img_keys);
  if (nc == 1)
    hipLaunchKernelGGL(push_argmin_kernel<1>, grid, dim3(kArgminWaves * 64), 0, s, x, HW, protos, P, proto_class,
                       mask, keys);
  else if (nc == 2)
    hipLaunchKernelGGL(push_argmin_kernel<2>, grid, dim3(kArgminWaves * 64), 0, s, x, HW, protos, P, proto_class,
                       mask, keys);
  else
    hipLaunchKernelGGL(push_argmin_kernel<4>, grid, dim3(kArgminWaves * 64), 0, s, x, HW, protos, P, proto_class,
                       mask, keys);
  return check_launch("push_argmin_kernel");
}

extern "C" int protoseg_push_merge(const uint64_t* img_keys, int n_img, int64_t first_img, const float* x, int C,
                                   int hw, int P, float* global_dist, int64_t* global_img, int32_t* global_patch,
                                   float* global_fmap, protoseg_stream_t stream) {
  if (!img_keys || !x || !global_dist || !global_img || !global_patch || !global_fmap)
    return fail(PROTOSEG_ERR_INVALID, "null pointer argument");
  if (n_img <= 0 || C <= 0 || hw <= 0 || P <= 0) return fail(PROTOSEG_ERR_INVALID, "bad shape");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int waves_per_block = 4;
  hipLaunchKernelGGL(push_merge_kernel, dim3(static_cast<unsigned>(ceil_div(P, waves_per_block))),
                     dim3(waves_per_block * 64), 0, s, reinterpret_cast<const unsigned long long*>(img_keys), n_img,
                     static_cast<long long>(first_img), x, C, hw, P, global_dist,
                     reinterpret_cast<long long*>(global_img), global_patch, global_fmap);
  return check_launch("push_merge_kernel");
}
