// kld.hip — the KLD similarity loss of segmentation/module.py:167-208 and its gradient, gfx950.
//
// The reference loops in Python over images x classes present x prototype pairs, with a
// masked_select, a log_softmax and two kl_div per pair and host syncs per class (module.py:170,
// 174). Here the same quantities come from four launches:
//   kld_lists_kernel     prototype -> class buckets (ascending prototype ids), module.py:173
//   kld_pairs_kernel     one workgroup per (class, image): masked max / log-sum-exp of each of the
//                        class's prototypes over the class's pixels (module.py:178-183), then the
//                        pair sums KL(p_i || p_j) (module.py:190-198) from chunks staged in LDS
//   kld_finalize_kernel  mean of exp(-(KL_ij + KL_ji) / 2) over all pairs (module.py:199-206)
//   kld_grad_kernel      d(g_loss * loss) / d distances, dense [B, P, HW]: what autograd of the
//                        reference ops produces; zero outside each prototype's class pixels
// Only the class's own prototype rows are read at the class's pixels, so the reads are about
// 1/K of the distance tensor; the dense gradient write is the dominant traffic.
//
// Reference semantics kept (oracle/kld_oracle.py): the label value c selects prototype column
// c (module.py:170-178: void = 0 pairs with class-0 prototypes, value K is skipped); a class
// with < 2 prototypes or < 2 pixels adds no pair (module.py:186); the loss is 0 without pairs.
#include <math.h>

#include <type_traits>

#include "protoseg_device.h"
#include "protoseg_host.h"

namespace protoseg {

namespace {

constexpr int kKldMaxPerClass = 32;  // prototypes of one class held per workgroup
constexpr int kKldMaxClasses = 63;   // K + 1 buckets handled by one wave
constexpr int kKldThreads = 256;     // = pixels per staged chunk
constexpr int kKldPair = kKldMaxPerClass * kKldMaxPerClass;
constexpr size_t kKldMaxDynLds = 2 * kKldMaxPerClass * kKldThreads * sizeof(float);  // p | log p chunks

size_t align256(size_t v) { return (v + 255) & ~static_cast<size_t>(255); }

// Workspace regions (bytes), written by the forward and read by the backward.
struct KldLayout {
  size_t off;    // int [K + 2]: bucket starts; bucket K = prototypes with no class in [0, K)
  size_t idx;    // int [P]: prototype ids grouped by bucket, ascending within a bucket
  size_t cnt;    // int [B * K]: pixels of label c in image b
  size_t mx;     // float [B * P]: max of d over the prototype's class pixels
  size_t lse;    // float [B * P]: log(sum exp(d - max)) over the same pixels
  size_t kl;     // float [B * K * 32 * 32]: KL(p_i || p_j) for class slots i, j
  size_t stat;   // int [4]: [0] pair count, [1] a class holds more than max_per_class prototypes
  size_t total;
};

KldLayout kld_layout(int B, int P, int K) {
  KldLayout l;
  size_t o = 0;
  l.off = o;
  o = align256(o + static_cast<size_t>(K + 2) * 4);
  l.idx = o;
  o = align256(o + static_cast<size_t>(P) * 4);
  l.cnt = o;
  o = align256(o + static_cast<size_t>(B) * K * 4);
  l.mx = o;
  o = align256(o + static_cast<size_t>(B) * P * 4);
  l.lse = o;
  o = align256(o + static_cast<size_t>(B) * P * 4);
  l.kl = o;
  o = align256(o + static_cast<size_t>(B) * K * kKldPair * 4);
  l.stat = o;
  o = align256(o + 16);
  l.total = o;
  return l;
}

struct KldPtrs {
  int *off, *idx, *cnt, *stat;
  float *mx, *lse, *kl;
};

KldPtrs kld_ptrs(void* ws, const KldLayout& l) {
  unsigned char* b = static_cast<unsigned char*>(ws);
  return {reinterpret_cast<int*>(b + l.off), reinterpret_cast<int*>(b + l.idx), reinterpret_cast<int*>(b + l.cnt),
          reinterpret_cast<int*>(b + l.stat), reinterpret_cast<float*>(b + l.mx), reinterpret_cast<float*>(b + l.lse),
          reinterpret_cast<float*>(b + l.kl)};
}

__device__ __forceinline__ int bucket_of(int pc, int K) { return (pc >= 0 && pc < K) ? pc : K; }

// One wave: lane c counts and lists the prototypes of bucket c (module.py:173, nonzero of the
// identity column = the prototypes whose class is c, ascending).
__global__ __launch_bounds__(64) void kld_lists_kernel(const int32_t* __restrict__ proto_class, int P, int K,
                                                       int max_per_class, int* __restrict__ off,
                                                       int* __restrict__ idx, int* __restrict__ stat) {
  const int c = threadIdx.x;
  const bool mine = c <= K;
  int n = 0;
  for (int p = 0; p < P; ++p) n += (mine && bucket_of(proto_class[p], K) == c) ? 1 : 0;
  int incl = n;
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    const int v = __shfl_up(incl, s);
    if (c >= s) incl += v;
  }
  const int start = incl - n;
  if (mine) off[c] = start;
  if (c == K) off[K + 1] = incl;
  int wpos = start;
  for (int p = 0; p < P; ++p)
    if (mine && bucket_of(proto_class[p], K) == c) idx[wpos++] = p;
  const bool over = mine && c < K && n > max_per_class;
  const unsigned long long any_over = __ballot(over);
  if (c == 0) {
    stat[0] = 0;
    stat[1] = any_over != 0ull ? 1 : 0;
  }
}

template <typename TL>
__device__ __forceinline__ long long label_at(const TL* lab, int n) {
  return static_cast<long long>(lab[n]);
}

// Merge of two (max, sum exp(. - max)) pairs; an empty side is (-inf, 0).
__device__ __forceinline__ void lse_merge(float& m, float& s, float mo, float so) {
  const float mm = fmaxf(m, mo);
  s = (mm == -INFINITY) ? 0.f : s * expf(m - mm) + so * expf(mo - mm);
  m = mm;
}

// One workgroup per (class c, image b). LDS: [mpc][256] p | [mpc][256] log p (dynamic).
template <typename TL>
__global__ __launch_bounds__(kKldThreads) void kld_pairs_kernel(const float* __restrict__ dist, int P, int HW,
                                                                const TL* __restrict__ label, int K, int mpc,
                                                                const int* __restrict__ off,
                                                                const int* __restrict__ idx, int* __restrict__ cnt_out,
                                                                float* __restrict__ mx_out, float* __restrict__ lse_out,
                                                                float* __restrict__ kl_out) {
  extern __shared__ __attribute__((aligned(16))) float kld_smem[];
  __shared__ int s_proto[kKldMaxPerClass];
  __shared__ float s_m[4][kKldMaxPerClass], s_s[4][kKldMaxPerClass];
  __shared__ float s_mx[kKldMaxPerClass], s_lse[kKldMaxPerClass];
  __shared__ int s_cnt[4];
  const int c = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int o0 = off[c];
  const int npc_all = off[c + 1] - o0;
  const int npc = npc_all < mpc ? npc_all : mpc;
  if (tid < npc) s_proto[tid] = idx[o0 + tid];
  __syncthreads();
  const TL* lab = label + static_cast<size_t>(b) * HW;
  const float* db = dist + static_cast<size_t>(b) * P * HW;

  // ---- pass 1: online max / sum-exp per prototype over the class's pixels (module.py:180-183)
  float m[kKldMaxPerClass], s[kKldMaxPerClass];
#pragma unroll
  for (int i = 0; i < kKldMaxPerClass; ++i) {
    m[i] = -INFINITY;
    s[i] = 0.f;
  }
  int cnt = 0;
  for (int n = tid; n < HW; n += kKldThreads) {
    if (label_at(lab, n) != c) continue;
    ++cnt;
#pragma unroll
    for (int i = 0; i < kKldMaxPerClass; ++i) {
      if (i < npc) {
        const float v = db[static_cast<size_t>(s_proto[i]) * HW + n];
        if (v > m[i]) {
          s[i] = s[i] * expf(m[i] - v) + 1.f;
          m[i] = v;
        } else {
          s[i] += expf(v - m[i]);
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < kKldMaxPerClass; ++i) {
    if (i < npc) {
      float mi = m[i], si = s[i];
#pragma unroll
      for (int sh = 32; sh >= 1; sh >>= 1) lse_merge(mi, si, __shfl_xor(mi, sh), __shfl_xor(si, sh));
      if (lane == 0) {
        s_m[wave][i] = mi;
        s_s[wave][i] = si;
      }
    }
  }
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) cnt += __shfl_xor(cnt, sh);
  if (lane == 0) s_cnt[wave] = cnt;
  __syncthreads();
  const int total = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
  if (tid < npc) {
    float mm = s_m[0][tid], ss = s_s[0][tid];
    for (int w = 1; w < 4; ++w) lse_merge(mm, ss, s_m[w][tid], s_s[w][tid]);
    const float l = logf(ss);
    s_mx[tid] = mm;
    s_lse[tid] = l;
    mx_out[static_cast<size_t>(b) * P + s_proto[tid]] = mm;
    lse_out[static_cast<size_t>(b) * P + s_proto[tid]] = l;
  }
  if (tid == 0) cnt_out[static_cast<size_t>(b) * K + c] = total;
  __syncthreads();
  if (npc < 2 || total < 2 || npc_all > mpc) return;  // module.py:186: no distribution / no pair

  // ---- pass 2: KL(p_i || p_j) = sum_n p_i (lp_i - lp_j) over the class's pixels (module.py:190-198)
  float* sp = kld_smem;                       // [npc][256]
  float* slp = kld_smem + npc * kKldThreads;  // [npc][256]
  const int E = npc * npc;
  int G = kKldThreads / E;  // pixel groups per (i, j) entry
  G = G < 1 ? 1 : (G > 16 ? 16 : G);
  const int ntask = E * G;  // <= 1024
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int base = 0; base < HW; base += kKldThreads) {
    const int n = base + tid;
    const bool in = n < HW && label_at(lab, n) == c;
    for (int i = 0; i < npc; ++i) {
      float lpv = 0.f, pv = 0.f;
      if (in) {
        const float v = db[static_cast<size_t>(s_proto[i]) * HW + n];
        lpv = (v - s_mx[i]) - s_lse[i];  // log_softmax: (x - max) - log(sum)
        pv = expf(lpv);
      }
      sp[i * kKldThreads + tid] = pv;
      slp[i * kKldThreads + tid] = lpv;
    }
    if (!__syncthreads_or(in)) continue;  // no pixel of the class in this chunk
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int task = tid + k * kKldThreads;
      if (task < ntask) {
        const int e = task / G, g = task - e * G;
        const int i = e / npc, j = e - i * npc;
        if (i != j) {
          const float* pi = sp + i * kKldThreads;
          const float* li = slp + i * kKldThreads;
          const float* lj = slp + j * kKldThreads;
          float a = acc[k];
          for (int q = g; q < kKldThreads; q += G) a = fmaf(pi[q], li[q] - lj[q], a);
          acc[k] = a;
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int task = tid + k * kKldThreads;
    if (task < ntask) kld_smem[task] = acc[k];
  }
  __syncthreads();
  float* klb = kl_out + (static_cast<size_t>(b) * K + c) * kKldPair;
  for (int e = tid; e < E; e += kKldThreads) {
    float v = 0.f;
    for (int g = 0; g < G; ++g) v += kld_smem[e * G + g];
    const int i = e / npc, j = e - i * npc;
    klb[i * kKldMaxPerClass + j] = v;
  }
}

// Mean over all pairs of exp(-kld), kld = (KL(p_j||p_i) + KL(p_i||p_j)) / 2 (module.py:195-206).
__global__ __launch_bounds__(256) void kld_finalize_kernel(int B, int K, int mpc, const int* __restrict__ off,
                                                           const int* __restrict__ cnt, const float* __restrict__ kl,
                                                           int* __restrict__ stat, float* __restrict__ loss_out,
                                                           int32_t* __restrict__ npairs_out) {
  __shared__ float s_sum[256];
  __shared__ int s_n[256];
  float sum = 0.f;
  int n = 0;
  for (int gi = threadIdx.x; gi < B * K; gi += 256) {
    const int c = gi % K;
    const int npc = off[c + 1] - off[c];
    if (npc < 2 || npc > mpc || cnt[gi] < 2) continue;
    const float* k = kl + static_cast<size_t>(gi) * kKldPair;
    for (int i = 0; i < npc; ++i)
      for (int j = i + 1; j < npc; ++j) {
        sum += expf(-((k[j * kKldMaxPerClass + i] + k[i * kKldMaxPerClass + j]) / 2.f));
        ++n;
      }
  }
  s_sum[threadIdx.x] = sum;
  s_n[threadIdx.x] = n;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (static_cast<int>(threadIdx.x) < w) {
      s_sum[threadIdx.x] += s_sum[threadIdx.x + w];
      s_n[threadIdx.x] += s_n[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const int np = s_n[0];
    float loss = np > 0 ? s_sum[0] / static_cast<float>(np) : 0.f;
    if (stat[1]) loss = __builtin_nanf("");
    stat[0] = np;
    loss_out[0] = loss;
    if (npairs_out) npairs_out[0] = np;
  }
}

// d(g_loss * loss)/d d for image b, bucket c, one 256-pixel chunk. Per class pixel n and class
// slot i (autograd of log_softmax + the two kl_div per pair, module.py:183-206):
//   g_i(n) = sum_{j != i} w_ij (p_i (lp_i - lp_j - KL_ij + 1) - p_j) / 2,
//   w_ij = -g_loss exp(-kld_ij) / n_pairs.
// Every row of bucket c is written for every pixel of the chunk (zero off the class), so the
// grid writes the whole [B, P, HW] tensor exactly once.
template <typename TL>
__global__ __launch_bounds__(kKldThreads) void kld_grad_kernel(
    const float* __restrict__ dist, int P, int HW, const TL* __restrict__ label, int K, int mpc,
    const int* __restrict__ off, const int* __restrict__ idx, const int* __restrict__ cnt,
    const float* __restrict__ mx, const float* __restrict__ lse, const float* __restrict__ kl,
    const int* __restrict__ stat, const float* __restrict__ g_loss, float* __restrict__ g_dist) {
  extern __shared__ __attribute__((aligned(16))) float kld_smem[];
  __shared__ int s_proto[kKldMaxPerClass];
  __shared__ float s_mx[kKldMaxPerClass], s_lse[kKldMaxPerClass];
  __shared__ float s_w[kKldPair], s_kl[kKldPair];
  const int c = blockIdx.y, b = blockIdx.z, tid = threadIdx.x;
  const int n = blockIdx.x * kKldThreads + tid;
  const int o0 = off[c];
  const int npc_all = off[c + 1] - o0;
  const int np = stat[0];
  const bool valid = c < K && npc_all >= 2 && npc_all <= mpc && np > 0 && cnt[static_cast<size_t>(b) * K + c] >= 2;
  float* gb = g_dist + static_cast<size_t>(b) * P * HW;
  if (!valid) {
    if (n < HW)
      for (int i = 0; i < npc_all; ++i) gb[static_cast<size_t>(idx[o0 + i]) * HW + n] = 0.f;
    return;
  }
  const int npc = npc_all;
  if (tid < npc) {
    const int p = idx[o0 + tid];
    s_proto[tid] = p;
    s_mx[tid] = mx[static_cast<size_t>(b) * P + p];
    s_lse[tid] = lse[static_cast<size_t>(b) * P + p];
  }
  const float gl = g_loss ? g_loss[0] : 1.f;
  const float* klb = kl + (static_cast<size_t>(b) * K + c) * kKldPair;
  for (int e = tid; e < npc * npc; e += kKldThreads) {
    const int i = e / npc, j = e - i * npc;
    const float kij = klb[i * kKldMaxPerClass + j], kji = klb[j * kKldMaxPerClass + i];
    s_kl[i * kKldMaxPerClass + j] = kij;
    s_w[i * kKldMaxPerClass + j] = i == j ? 0.f : -(gl / static_cast<float>(np)) * expf(-((kji + kij) / 2.f));
  }
  __syncthreads();
  const bool in = n < HW && label_at(label + static_cast<size_t>(b) * HW, n) == c;
  float* sp = kld_smem;  // [npc][256]: each thread uses only its own column
  float* slp = kld_smem + npc * kKldThreads;
  for (int i = 0; i < npc; ++i) {
    float lpv = 0.f, pv = 0.f;
    if (in) {
      const float v = dist[(static_cast<size_t>(b) * P + s_proto[i]) * HW + n];
      lpv = (v - s_mx[i]) - s_lse[i];
      pv = expf(lpv);
    }
    sp[i * kKldThreads + tid] = pv;
    slp[i * kKldThreads + tid] = lpv;
  }
  if (n >= HW) return;
  for (int i = 0; i < npc; ++i) {
    float g = 0.f;
    if (in) {
      const float pi = sp[i * kKldThreads + tid], li = slp[i * kKldThreads + tid];
      for (int j = 0; j < npc; ++j) {
        const float pj = sp[j * kKldThreads + tid], lj = slp[j * kKldThreads + tid];
        g = fmaf(s_w[i * kKldMaxPerClass + j], pi * (li - lj - s_kl[i * kKldMaxPerClass + j] + 1.f) - pj, g);
      }
      g *= 0.5f;
    }
    gb[static_cast<size_t>(s_proto[i]) * HW + n] = g;
  }
}

int kld_check(const float* dist, int B, int P, int HW, const void* label, int label_dtype, const int32_t* proto_class,
              int K, int max_per_class, const void* ws, size_t ws_bytes) {
  if (!dist || !label || !proto_class || !ws) return fail(PROTOSEG_ERR_INVALID, "null pointer argument");
  if (B <= 0 || P <= 0 || HW <= 0 || K <= 0)
    return fail(PROTOSEG_ERR_INVALID, "bad shape B=%d P=%d HW=%d K=%d", B, P, HW, K);
  if (K > kKldMaxClasses) return fail(PROTOSEG_ERR_UNSUPPORTED, "K=%d > %d classes", K, kKldMaxClasses);
  if (max_per_class < 1 || max_per_class > kKldMaxPerClass)
    return fail(PROTOSEG_ERR_UNSUPPORTED, "max_per_class=%d outside [1, %d]", max_per_class, kKldMaxPerClass);
  if (label_dtype != PROTOSEG_I64 && label_dtype != PROTOSEG_I32 && label_dtype != PROTOSEG_U8)
    return fail(PROTOSEG_ERR_UNSUPPORTED, "label_dtype %d", label_dtype);
  if (static_cast<unsigned long long>(B) * P * HW >= (1ull << 31))
    return fail(PROTOSEG_ERR_UNSUPPORTED, "B*P*HW >= 2^31");
  const size_t need = kld_layout(B, P, K).total;
  if (ws_bytes < need) return fail(PROTOSEG_ERR_INVALID, "workspace %zu B < %zu B", ws_bytes, need);
  return PROTOSEG_OK;
}

template <typename Fn>
int by_label(int label_dtype, Fn&& fn) {
  switch (label_dtype) {
    case PROTOSEG_I64:
      return fn(static_cast<int64_t*>(nullptr));
    case PROTOSEG_I32:
      return fn(static_cast<int32_t*>(nullptr));
    default:
      return fn(static_cast<uint8_t*>(nullptr));
  }
}

}  // namespace

}  // namespace protoseg

using namespace protoseg;

extern "C" size_t protoseg_kld_workspace_size(int B, int P, int K) {
  if (B <= 0 || P <= 0 || K <= 0) return 0;
  return kld_layout(B, P, K).total;
}

extern "C" int protoseg_kld_forward(const float* dist, int B, int P, int HW, const void* label, int label_dtype,
                                    const int32_t* proto_class, int K, int max_per_class, float* loss_out,
                                    int32_t* npairs_out, void* workspace, size_t workspace_bytes,
                                    protoseg_stream_t stream) {
  if (int st = kld_check(dist, B, P, HW, label, label_dtype, proto_class, K, max_per_class, workspace, workspace_bytes))
    return st;
  if (!loss_out) return fail(PROTOSEG_ERR_INVALID, "loss_out must be non-null");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const KldLayout l = kld_layout(B, P, K);
  const KldPtrs w = kld_ptrs(workspace, l);
  hipLaunchKernelGGL(kld_lists_kernel, dim3(1), dim3(64), 0, s, proto_class, P, K, max_per_class, w.off, w.idx, w.stat);
  if (int st = check_launch("kld_lists_kernel")) return st;
  const size_t lds = static_cast<size_t>(2) * max_per_class * kKldThreads * sizeof(float);
  const int st = by_label(label_dtype, [&](auto tl) {
    using TL = std::remove_pointer_t<decltype(tl)>;
    if (int e = ensure_lds<kld_pairs_kernel<TL>, kKldMaxDynLds>()) return e;
    hipLaunchKernelGGL(kld_pairs_kernel<TL>, dim3(K, B), dim3(kKldThreads), lds, s, dist, P, HW,
                       static_cast<const TL*>(label), K, max_per_class, w.off, w.idx, w.cnt, w.mx, w.lse, w.kl);
    return check_launch("kld_pairs_kernel");
  });
  if (st) return st;
  hipLaunchKernelGGL(kld_finalize_kernel, dim3(1), dim3(256), 0, s, B, K, max_per_class, w.off, w.cnt, w.kl, w.stat,
                     loss_out, npairs_out);
  return check_launch("kld_finalize_kernel");
}

extern "C" int protoseg_kld_backward(const float* dist, int B, int P, int HW, const void* label, int label_dtype,
                                     const int32_t* proto_class, int K, int max_per_class, const float* g_loss,
                                     const void* workspace, size_t workspace_bytes, float* g_dist,
                                     protoseg_stream_t stream) {
  if (int st = kld_check(dist, B, P, HW, label, label_dtype, proto_class, K, max_per_class, workspace, workspace_bytes))
    return st;
  if (!g_dist) return fail(PROTOSEG_ERR_INVALID, "g_dist must be non-null");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const KldLayout l = kld_layout(B, P, K);
  const KldPtrs w = kld_ptrs(const_cast<void*>(workspace), l);
  const size_t lds = static_cast<size_t>(2) * max_per_class * kKldThreads * sizeof(float);
  const dim3 grid(static_cast<unsigned>(ceil_div(HW, kKldThreads)), K + 1, B);
  return by_label(label_dtype, [&](auto tl) {
    using TL = std::remove_pointer_t<decltype(tl)>;
    if (int e = ensure_lds<kld_grad_kernel<TL>, kKldMaxDynLds>()) return e;
    hipLaunchKernelGGL(kld_grad_kernel<TL>, grid, dim3(kKldThreads), lds, s, dist, P, HW,
                       static_cast<const TL*>(label), K, max_per_class, w.off, w.idx, w.cnt, w.mx, w.lse, w.kl, w.stat,
                       g_loss, g_dist);
    return check_launch("kld_grad_kernel");
  });
}
