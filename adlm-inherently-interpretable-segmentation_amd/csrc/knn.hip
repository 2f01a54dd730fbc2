// knn.hip — k-nearest-patch search and prototype pruning of find_nearest.py / prune.py on gfx950.
//
// Reference: find_nearest.py:66-342 (find_k_nearest_patches_to_prototypes, full_save=True as
// prune.py:20-30 calls it) and prune.py:33-43 (the pruning rule). Per image the reference copies
// the [P, h, w] distance map to the host, adds 10e6 to void patches (label map resized with
// PIL NEAREST, find_nearest.py:128-132), and runs a Python loop over prototypes: np.amin /
// np.argmin, a label vote over the patch's pixel box, and a heapq of the k closest images per
// prototype. Here:
//   resize_label_kernel   PIL NEAREST label resize (dataset.py:23-31), exact index sequence
//   knn_image_min_kernel  per (image, prototype): min / first argmin of d + 1e7 * void, in f64
//   knn_patch_label_kernel per (image, prototype): the box of the winning patch and its label
//   knn_heap_kernel       per prototype: heapq.heappush / heappushpop replayed in image order
//   knn_finalize_kernel   per prototype: heap.sort() + reverse, class-match count, prune flag
// Every step reproduces the reference's comparison sequence, so results are bit-exact for a
// given distance map (ties included).
#include <climits>
#include <cstdint>

#include "protoseg_device.h"
#include "protoseg_host.h"

namespace protoseg {

namespace {

constexpr int kKnnThreads = 256;
constexpr int kKnnMaxK = 64;
constexpr int kHeapThreads = 64;
constexpr int kLabelBins = 512;  // patch labels (converted - 1) in [-256, 255]
constexpr int kLabelBias = 256;
constexpr int kSkip = INT32_MIN;  // empty patch box: the image is not offered (find_nearest.py:179-180)

template <typename TL>
__device__ __forceinline__ long long converted(const TL* __restrict__ p, size_t i, const int32_t* __restrict__ lut,
                                               int lut_size) {
  const long long raw = static_cast<long long>(p[i]);
  if (!lut) return raw;
  return (raw >= 0 && raw < lut_size) ? lut[raw] : 0;
}

// PIL Image.resize(NEAREST) (ImagingScaleAffine): the source coordinate starts at scale / 2 and
// is advanced by repeated f64 additions of scale = in / out; index = (int) coordinate. The
// accumulated rounding is part of the result, so the additions are replayed, not multiplied.
__device__ __forceinline__ int pil_nearest(int dst, int n_in, int n_out) {
  const double a = static_cast<double>(n_in) / static_cast<double>(n_out);
  double xo = a * 0.5;
  for (int i = 0; i < dst; ++i) xo += a;
  const int s = static_cast<int>(xo);
  return s < n_in - 1 ? s : n_in - 1;
}

// labels [n, H, W] -> out [n, h, w] int32 (converted through lut when given).
template <typename TL>
__global__ __launch_bounds__(kKnnThreads) void resize_label_kernel(const TL* __restrict__ label, int H, int W, int h,
                                                                   int w, const int32_t* __restrict__ lut,
                                                                   int lut_size, int32_t* __restrict__ out) {
  const int x = blockIdx.x * kKnnThreads + threadIdx.x;
  const int y = blockIdx.y, img = blockIdx.z;
  if (x >= w) return;
  const int sy = pil_nearest(y, H, h), sx = pil_nearest(x, W, w);
  const long long v = converted(label + static_cast<size_t>(img) * H * W, static_cast<size_t>(sy) * W + sx, lut,
                                lut_size);
  out[(static_cast<size_t>(img) * h + y) * w + x] = static_cast<int32_t>(v);
}

struct MinIdx {
  double v;
  int i;
};

__device__ __forceinline__ MinIdx min_first(MinIdx a, MinIdx b) {
  return (b.v < a.v || (b.v == a.v && b.i < a.i)) ? b : a;
}

// One workgroup per (image, prototype): np.amin / np.argmin of proto_dist_ + 10e6 * (y == -1)
// (find_nearest.py:132, 140-145). The sum is formed in f64 like the reference's numpy
// broadcast (f32 map + f64 mask -> f64), so void patches of an all-void image keep their
// exact order and the +0.0 of non-void patches canonicalises -0.
__global__ __launch_bounds__(kKnnThreads) void knn_image_min_kernel(const float* __restrict__ dist, int P, int HW,
                                                                    const int32_t* __restrict__ small_label,
                                                                    double* __restrict__ min_dist,
                                                                    int32_t* __restrict__ min_idx) {
  __shared__ double s_v[kKnnThreads / 64];
  __shared__ int s_i[kKnnThreads / 64];
  const int p = blockIdx.x, img = blockIdx.y;
  const float* d = dist + (static_cast<size_t>(img) * P + p) * HW;
  const int32_t* y = small_label ? small_label + static_cast<size_t>(img) * HW : nullptr;
  MinIdx best{INFINITY, INT32_MAX};
  constexpr int kU = 4;
  int i = threadIdx.x;
  for (; i + (kU - 1) * kKnnThreads < HW; i += kU * kKnnThreads) {
    float dv[kU];
    bool vd[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      dv[u] = d[i + u * kKnnThreads];
      vd[u] = y && y[i + u * kKnnThreads] == 0;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u)
      best = min_first(best, MinIdx{static_cast<double>(dv[u]) + (vd[u] ? 10e6 : 0.0), i + u * kKnnThreads});
  }
  for (; i < HW; i += kKnnThreads) {
    const bool vd = y && y[i] == 0;
    best = min_first(best, MinIdx{static_cast<double>(d[i]) + (vd ? 10e6 : 0.0), i});
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    MinIdx o{__shfl_xor(best.v, off), __shfl_xor(best.i, off)};
    best = min_first(best, o);
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_v[wave] = best.v;
    s_i[wave] = best.i;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    MinIdx r{s_v[0], s_i[0]};
    for (int w = 1; w < kKnnThreads / 64; ++w) r = min_first(r, MinIdx{s_v[w], s_i[w]});
    min_dist[static_cast<size_t>(img) * P + p] = r.v;
    min_idx[static_cast<size_t>(img) * P + p] = r.i;
  }
}

// One wave per (image, prototype): the winning patch's pixel box (find_nearest.py:159-166) and
// its label (202-211): the prototype's class if any pixel of the box carries it, otherwise the
// most common value (np.unique + argmax: the smallest value among equally common ones).
// Labels are search_y = convert_targets(y) - 1 (find_nearest.py:113-116), void = -1.
template <typename TL>
__global__ __launch_bounds__(kKnnThreads) void knn_patch_label_kernel(
    const int32_t* __restrict__ min_idx, int n_img, int P, int h, int w, const TL* __restrict__ label, int H, int W,
    const int32_t* __restrict__ lut, int lut_size, const int32_t* __restrict__ proto_class,
    int32_t* __restrict__ patch_label, int32_t* __restrict__ status) {
  __shared__ unsigned s_hist[kKnnThreads / 64][kLabelBins];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const long long bp = static_cast<long long>(blockIdx.x) * (kKnnThreads / 64) + wave;
  if (bp >= static_cast<long long>(n_img) * P) return;
  const int img = static_cast<int>(bp / P), p = static_cast<int>(bp % P);
  const int idx = min_idx[bp];
  const int r = idx / w, c = idx % w;
  // find_nearest.py:119-120, 159-166: patch_height = img_height / model_output_height (f64),
  // bounds int(r * patch_height) .. int((r + 1) * patch_height); slicing clamps to the image.
  const double ph = static_cast<double>(H) / static_cast<double>(h);
  const double pw = static_cast<double>(W) / static_cast<double>(w);
  int r0 = static_cast<int>(r * ph), r1 = static_cast<int>((r + 1) * ph);
  int c0 = static_cast<int>(c * pw), c1 = static_cast<int>((c + 1) * pw);
  r1 = r1 < H ? r1 : H;
  c1 = c1 < W ? c1 : W;
  if (r1 <= r0 || c1 <= c0) {
    if (lane == 0) patch_label[bp] = kSkip;
    return;
  }
  const int bw = c1 - c0;
  const int nbox = (r1 - r0) * bw;
  const TL* L = label + static_cast<size_t>(img) * H * W;
  const long long target = proto_class[p];
  auto value_at = [&](int q) {
    const int rr = r0 + q / bw, cc = c0 + q % bw;
    return converted(L, static_cast<size_t>(rr) * W + cc, lut, lut_size) - 1;
  };
  bool has_target = false;
  for (int q0 = 0; q0 < nbox && !has_target; q0 += 64) {  // wave-uniform trip count
    const int q = q0 + lane;
    has_target = __ballot(q < nbox && value_at(q) == target) != 0;
  }
  if (has_target) {
    if (lane == 0) patch_label[bp] = static_cast<int32_t>(target);
    return;
  }
  unsigned* hist = s_hist[wave];
  for (int b = lane; b < kLabelBins; b += 64) hist[b] = 0u;
  __builtin_amdgcn_wave_barrier();
  bool bad = false;
  for (int q = lane; q < nbox; q += 64) {
    const long long v = value_at(q) + kLabelBias;
    if (v >= 0 && v < kLabelBins) atomicAdd(&hist[v], 1u);
    else bad = true;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  // lane scans bins [lane*8, lane*8+8) in increasing order: strict '>' keeps the smallest value
  unsigned best_n = 0;
  int best_b = kLabelBins;
  for (int b = lane * (kLabelBins / 64); b < (lane + 1) * (kLabelBins / 64); ++b)
    if (hist[b] > best_n) {
      best_n = hist[b];
      best_b = b;
    }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned on = __shfl_xor(best_n, off);
    const int ob = __shfl_xor(best_b, off);
    if (on > best_n || (on == best_n && ob < best_b)) {
      best_n = on;
      best_b = ob;
    }
  }
  if (__ballot(bad) && lane == 0) atomicOr(reinterpret_cast<unsigned*>(status), 1u);
  if (lane == 0) patch_label[bp] = best_b - kLabelBias;
}

struct HeapView {
  double* neg;
  int32_t* label;
  int32_t* patch;
  long long* img;
  int t;  // this thread's column in the [k][kHeapThreads] LDS arrays
  __device__ double key(int i) const { return neg[i * kHeapThreads + t]; }
  __device__ void move(int dst, int src) const {
    neg[dst * kHeapThreads + t] = neg[src * kHeapThreads + t];
    label[dst * kHeapThreads + t] = label[src * kHeapThreads + t];
    patch[dst * kHeapThreads + t] = patch[src * kHeapThreads + t];
    img[dst * kHeapThreads + t] = img[src * kHeapThreads + t];
  }
  __device__ void put(int i, double n, int l, int pa, long long im) const {
    neg[i * kHeapThreads + t] = n;
    label[i * kHeapThreads + t] = l;
    patch[i * kHeapThreads + t] = pa;
    img[i * kHeapThreads + t] = im;
  }
};

// CPython heapq._siftdown(heap, startpos, pos) with ImagePatch.__lt__ (negative distance).
__device__ void sift_down(const HeapView& h, int start, int pos) {
  const double nk = h.key(pos);
  const int nl = h.label[pos * kHeapThreads + h.t], np = h.patch[pos * kHeapThreads + h.t];
  const long long ni = h.img[pos * kHeapThreads + h.t];
  while (pos > start) {
    const int parent = (pos - 1) >> 1;
    if (nk < h.key(parent)) {
      h.move(pos, parent);
      pos = parent;
      continue;
    }
    break;
  }
  h.put(pos, nk, nl, np, ni);
}

// CPython heapq._siftup(heap, pos): the smaller child bubbles up to a leaf, then _siftdown.
__device__ void sift_up(const HeapView& h, int end, int pos) {
  const int start = pos;
  const double nk = h.key(pos);
  const int nl = h.label[pos * kHeapThreads + h.t], np = h.patch[pos * kHeapThreads + h.t];
  const long long ni = h.img[pos * kHeapThreads + h.t];
  int child = 2 * pos + 1;
  while (child < end) {
    const int right = child + 1;
    if (right < end && !(h.key(child) < h.key(right))) child = right;
    h.move(pos, child);
    pos = child;
    child = 2 * pos + 1;
  }
  h.put(pos, nk, nl, np, ni);
  sift_down(h, start, pos);
}

// One thread per prototype: the images of this batch offered in order (find_nearest.py:224-230):
// heappush while the heap holds fewer than k, else heappushpop (replace the root when
// root < item, i.e. the new distance is strictly smaller than the largest kept one).
// Heap state in global memory [P][k] (+ size [P]) is staged through LDS for the batch.
__global__ __launch_bounds__(kHeapThreads) void knn_heap_kernel(
    const double* __restrict__ min_dist, const int32_t* __restrict__ min_idx, const int32_t* __restrict__ patch_label,
    int n_img, long long first_img, int P, int k, double* __restrict__ heap_neg, int32_t* __restrict__ heap_label,
    int32_t* __restrict__ heap_patch, long long* __restrict__ heap_img, int32_t* __restrict__ heap_size) {
  extern __shared__ unsigned char s_raw[];
  HeapView h;
  h.neg = reinterpret_cast<double*>(s_raw);
  h.img = reinterpret_cast<long long*>(h.neg + k * kHeapThreads);
  h.label = reinterpret_cast<int32_t*>(h.img + k * kHeapThreads);
  h.patch = h.label + k * kHeapThreads;
  h.t = threadIdx.x;
  const int p = blockIdx.x * kHeapThreads + threadIdx.x;
  if (p >= P) return;
  int n = heap_size[p];
  for (int i = 0; i < n; ++i)
    h.put(i, heap_neg[static_cast<size_t>(p) * k + i], heap_label[static_cast<size_t>(p) * k + i],
          heap_patch[static_cast<size_t>(p) * k + i], heap_img[static_cast<size_t>(p) * k + i]);
  for (int b = 0; b < n_img; ++b) {
    const size_t bp = static_cast<size_t>(b) * P + p;
    const int lab = patch_label[bp];
    if (lab == kSkip) continue;
    const double item = -min_dist[bp];
    if (n < k) {  // heapq.heappush
      h.put(n, item, lab, min_idx[bp], first_img + b);
      sift_down(h, 0, n);
      ++n;
    } else if (h.key(0) < item) {  // heapq.heappushpop
      h.put(0, item, lab, min_idx[bp], first_img + b);
      sift_up(h, n, 0);
    }
  }
  heap_size[p] = n;
  for (int i = 0; i < n; ++i) {
    heap_neg[static_cast<size_t>(p) * k + i] = h.key(i);
    heap_label[static_cast<size_t>(p) * k + i] = h.label[i * kHeapThreads + h.t];
    heap_patch[static_cast<size_t>(p) * k + i] = h.patch[i * kHeapThreads + h.t];
    heap_img[static_cast<size_t>(p) * k + i] = h.img[i * kHeapThreads + h.t];
  }
}

// One thread per prototype: heaps[j].sort() (stable, by negative distance) then [::-1]
// (find_nearest.py:231-232) into [P][k] outputs, the count of nearest patches labelled with
// the prototype's class and the prune flag count < prune_threshold (prune.py:35-43).
// Slots past the heap size: distance inf, label kSkip, image -1, patch -1.
__global__ __launch_bounds__(kHeapThreads) void knn_finalize_kernel(
    const double* __restrict__ heap_neg, const int32_t* __restrict__ heap_label,
    const int32_t* __restrict__ heap_patch, const long long* __restrict__ heap_img,
    const int32_t* __restrict__ heap_size, int P, int k, const int32_t* __restrict__ proto_class,
    int prune_threshold, double* __restrict__ out_dist, int32_t* __restrict__ out_label,
    long long* __restrict__ out_img, int32_t* __restrict__ out_patch, int32_t* __restrict__ class_count,
    int32_t* __restrict__ prune) {
  const int p = blockIdx.x * kHeapThreads + threadIdx.x;
  if (p >= P) return;
  const int n = heap_size[p];
  int order[kKnnMaxK];
  const double* key = heap_neg + static_cast<size_t>(p) * k;
  // stable insertion sort ascending by key (list.sort with ImagePatch.__lt__)
  for (int i = 0; i < n; ++i) {
    int j = i;
    while (j > 0 && key[i] < key[order[j - 1]]) {
      order[j] = order[j - 1];
      --j;
    }
    order[j] = i;
  }
  int cnt = 0;
  const int cls = proto_class[p];
  for (int q = 0; q < k; ++q) {
    const size_t o = static_cast<size_t>(p) * k + q;
    if (q < n) {
      const int s = order[n - 1 - q];  // reversed: ascending distance
      const size_t si = static_cast<size_t>(p) * k + s;
      out_dist[o] = -key[s];
      out_label[o] = heap_label[si];
      out_img[o] = heap_img[si];
      out_patch[o] = heap_patch[si];
      cnt += heap_label[si] == cls;
    } else {
      out_dist[o] = INFINITY;
      out_label[o] = kSkip;
      out_img[o] = -1;
      out_patch[o] = -1;
    }
  }
  class_count[p] = cnt;
  prune[p] = cnt < prune_threshold ? 1 : 0;
}

template <template <typename> class F, typename... A>
int dispatch_label(int dtype, A&&... args) {
  switch (dtype) {
    case PROTOSEG_I64:
      return F<int64_t>::run(args...);
    case PROTOSEG_I32:
      return F<int32_t>::run(args...);
    case PROTOSEG_U8:
      return F<uint8_t>::run(args...);
    default:
      return fail(PROTOSEG_ERR_UNSUPPORTED, "label dtype %d", dtype);
  }
}

template <typename TL>
struct ResizeLaunch {
  static int run(const void* label, int n, int H, int W, int h, int w, const int32_t* lut, int lut_size,
                 int32_t* out, hipStream_t s) {
    const dim3 grid(static_cast<unsigned>(ceil_div(w, kKnnThreads)), h, n);
    hipLaunchKernelGGL(resize_label_kernel<TL>, grid, dim3(kKnnThreads), 0, s, static_cast<const TL*>(label), H, W,
                       h, w, lut, lut_size, out);
    return check_launch("resize_label_kernel");
  }
};

template <typename TL>
struct PatchLabelLaunch {
  static int run(const int32_t* min_idx, int n, int P, int h, int w, const void* label, int H, int W,
                 const int32_t* lut, int lut_size, const int32_t* proto_class, int32_t* patch_label, int32_t* status,
                 hipStream_t s) {
    const long long waves = static_cast<long long>(n) * P;
    const dim3 grid(static_cast<unsigned>(ceil_div(waves, kKnnThreads / 64)));
    hipLaunchKernelGGL(knn_patch_label_kernel<TL>, grid, dim3(kKnnThreads), 0, s, min_idx, n, P, h, w,
                       static_cast<const TL*>(label), H, W, lut, lut_size, proto_class, patch_label, status);
    return check_launch("knn_patch_label_kernel");
  }
};

size_t heap_lds(int k) { return static_cast<size_t>(k) * kHeapThreads * (8 + 8 + 4 + 4); }

}  // namespace

}  // namespace protoseg

using namespace protoseg;

extern "C" int protoseg_resize_label(const void* label, int label_dtype, int n_img, int H, int W, int h, int w,
                                     const int32_t* lut, int lut_size, int32_t* out, protoseg_stream_t stream) {
  if (!label || !out) return fail(PROTOSEG_ERR_INVALID, "label and out must be non-null");
  if (n_img <= 0 || H <= 0 || W <= 0 || h <= 0 || w <= 0)
    return fail(PROTOSEG_ERR_INVALID, "bad shape n_img=%d H=%d W=%d h=%d w=%d", n_img, H, W, h, w);
  if (lut && lut_size <= 0) return fail(PROTOSEG_ERR_INVALID, "lut_size must be > 0");
  if (h > 65535 || n_img > 65535) return fail(PROTOSEG_ERR_UNSUPPORTED, "h=%d / n_img=%d per call", h, n_img);
  return dispatch_label<ResizeLaunch>(label_dtype, label, n_img, H, W, h, w, lut, lut_size, out,
                                      reinterpret_cast<hipStream_t>(stream));
}

extern "C" int protoseg_knn_image_min(const float* dist, int n_img, int P, int h, int w, const int32_t* small_label,
                                      double* min_dist, int32_t* min_idx, protoseg_stream_t stream) {
  if (!dist || !min_dist || !min_idx) return fail(PROTOSEG_ERR_INVALID, "dist, min_dist and min_idx must be non-null");
  if (n_img <= 0 || P <= 0 || h <= 0 || w <= 0) return fail(PROTOSEG_ERR_INVALID, "bad shape");
  if (n_img > 65535) return fail(PROTOSEG_ERR_UNSUPPORTED, "n_img=%d per call", n_img);
  if (static_cast<long long>(h) * w >= (1LL << 31)) return fail(PROTOSEG_ERR_UNSUPPORTED, "h*w too large");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(knn_image_min_kernel, dim3(P, n_img), dim3(kKnnThreads), 0, s, dist, P, h * w, small_label,
                     min_dist, min_idx);
  return check_launch("knn_image_min_kernel");
}

extern "C" int protoseg_knn_patch_label(const int32_t* min_idx, int n_img, int P, int h, int w, const void* label,
                                        int label_dtype, int H, int W, const int32_t* lut, int lut_size,
                                        const int32_t* proto_class, int32_t* patch_label, int32_t* status,
                                        protoseg_stream_t stream) {
  if (!min_idx || !label || !proto_class || !patch_label || !status)
    return fail(PROTOSEG_ERR_INVALID, "null pointer argument");
  if (n_img <= 0 || P <= 0 || h <= 0 || w <= 0 || H <= 0 || W <= 0) return fail(PROTOSEG_ERR_INVALID, "bad shape");
  if (lut && lut_size <= 0) return fail(PROTOSEG_ERR_INVALID, "lut_size must be > 0");
  return dispatch_label<PatchLabelLaunch>(label_dtype, min_idx, n_img, P, h, w, label, H, W, lut, lut_size,
                                          proto_class, patch_label, status, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int protoseg_knn_heap_push(const double* min_dist, const int32_t* min_idx, const int32_t* patch_label,
                                      int n_img, int64_t first_img, int P, int k, double* heap_neg,
                                      int32_t* heap_label, int32_t* heap_patch, int64_t* heap_img,
                                      int32_t* heap_size, protoseg_stream_t stream) {
  if (!min_dist || !min_idx || !patch_label || !heap_neg || !heap_label || !heap_patch || !heap_img || !heap_size)
    return fail(PROTOSEG_ERR_INVALID, "null pointer argument");
  if (n_img <= 0 || P <= 0) return fail(PROTOSEG_ERR_INVALID, "bad shape n_img=%d P=%d", n_img, P);
  if (k <= 0 || k > kKnnMaxK) return fail(PROTOSEG_ERR_UNSUPPORTED, "k=%d outside [1, %d]", k, kKnnMaxK);
  const size_t lds = heap_lds(k);
  if (int st = ensure_lds<knn_heap_kernel, kKnnMaxK * kHeapThreads * 24>()) return st;
  hipLaunchKernelGGL(knn_heap_kernel, dim3(static_cast<unsigned>(ceil_div(P, kHeapThreads))), dim3(kHeapThreads), lds,
                     reinterpret_cast<hipStream_t>(stream), min_dist, min_idx, patch_label, n_img,
                     static_cast<long long>(first_img), P, k, heap_neg, heap_label, heap_patch,
                     reinterpret_cast<long long*>(heap_img), heap_size);
  return check_launch("knn_heap_kernel");
}

extern "C" int protoseg_knn_finalize(const double* heap_neg, const int32_t* heap_label, const int32_t* heap_patch,
                                     const int64_t* heap_img, const int32_t* heap_size, int P, int k,
                                     const int32_t* proto_class, int prune_threshold, double* out_dist,
                                     int32_t* out_label, int64_t* out_img, int32_t* out_patch, int32_t* class_count,
                                     int32_t* prune, protoseg_stream_t stream) {
  if (!heap_neg || !heap_label || !heap_patch || !heap_img || !heap_size || !proto_class || !out_dist || !out_label ||
      !out_img || !out_patch || !class_count || !prune)
    return fail(PROTOSEG_ERR_INVALID, "null pointer argument");
  if (P <= 0) return fail(PROTOSEG_ERR_INVALID, "bad shape P=%d", P);
  if (k <= 0 || k > kKnnMaxK) return fail(PROTOSEG_ERR_UNSUPPORTED, "k=%d outside [1, %d]", k, kKnnMaxK);
  hipLaunchKernelGGL(knn_finalize_kernel, dim3(static_cast<unsigned>(ceil_div(P, kHeapThreads))), dim3(kHeapThreads),
                     0, reinterpret_cast<hipStream_t>(stream), heap_neg, heap_label, heap_patch,
                     reinterpret_cast<const long long*>(heap_img), heap_size, P, k, proto_class, prune_threshold,
                     out_dist, out_label, reinterpret_cast<long long*>(out_img), out_patch, class_count, prune);
  return check_launch("knn_finalize_kernel");
}
