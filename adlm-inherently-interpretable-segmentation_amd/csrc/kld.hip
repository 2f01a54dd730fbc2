// kld.hip — the KLD similarity loss of segmentation/module.py:167-208 and its gradient, gfx950.
//
// The reference loops in Python over images x classes present x prototype pairs, with a
// masked_select, a log_softmax and two kl_div per pair and host syncs per class (module.py:170,
// 174). Here the same quantities come from these launches:
//   forward (protoseg_kld_forward):
//   kld_partial_kernel   one workgroup per (class c, image b, pixel range s): the class's prototype
//                        list (ascending ids, module.py:173; published once for the later
//                        kernels), the range's class pixels, one pass with a running max:
//                        the local max m_i and sum_n exp(z_i - m_i) of each class prototype
//                        (z = distance) and T_ij = sum_n exp(z_i - m_i) (z_i - z_j)
//   kld_merge_kernel     per (c, b): L_i = log-sum-exp over the ranges (module.py:183) and
//                        KL(p_i || p_j) = sum_s exp(m_i^s - L_i) T_ij^s - (L_i - L_j), which is
//                        sum_n p_i (lp_i - lp_j) regrouped (module.py:190-198)
//   kld_finalize_kernel  mean of exp(-(KL_ij + KL_ji) / 2) over all pairs (module.py:199-206)
//   backward, compact layout (protoseg_kld_backward_compact), ONE launch:
//   kld_grad_compact_kernel  per (c, b, s): proto_slot, pix_cls of the range's pixels, the
//                        group's coefficients and the gradient at its class pixels
//   backward, dense layout (protoseg_kld_backward): kld_coef_kernel + kld_grad_kernel, the
//                        [B, P, HW] gradient autograd of the reference ops produces
// Only the class's own prototype rows are read at the class's pixels (about 1/K of the distance
// tensor); the dense gradient write is the dominant traffic of the dense layout.
//
// Reference semantics kept (oracle/kld_oracle.py): the label value c selects prototype column
// c (module.py:170-178: void = 0 pairs with class-0 prototypes, value K is skipped); a class
// with < 2 prototypes or < 2 pixels adds no pair (module.py:186); the loss is 0 without pairs.
#include <math.h>

#include <algorithm>
#include <type_traits>

#include "protoseg_device.h"
#include "protoseg_host.h"

namespace protoseg {

namespace {

constexpr int kKldMaxPerClass = 32;  // prototypes of one class held per workgroup
constexpr int kKldMaxClasses = 63;   // K + 1 buckets handled by one wave
constexpr int kKldThreads = 256;     // = pixels per staged chunk
#ifndef KLD_RANGE
#define KLD_RANGE 1024
#endif
constexpr int kKldRange = KLD_RANGE;
  // pixels per kld_partial_kernel workgroup (a multiple of 256)
constexpr int kKldPair = kKldMaxPerClass * kKldMaxPerClass;
constexpr int kKldLdsStride = kKldThreads + 1;  // padded rows: conflict-free task reads
constexpr size_t kKldMaxDynLds = 2 * kKldMaxPerClass * kKldLdsStride * sizeof(float);
// one range partial: m[32] | s[32] | count | T[32][32]
constexpr int kKldPartFloats = 2 * kKldMaxPerClass + 1 + kKldPair;

// Per-wave phase stamps of the partial kernel (debug builds only: make stamps, tools/stamps_kld.py).
#ifdef PROTOSEG_STAMPS
__device__ unsigned long long g_stamps_kld[1 << 17];
#define KSTAMP(slot, clk)                                                                                 \
  do {                                                                                                  \
    const unsigned _g = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;                \
    const unsigned _i = (_g * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8 + (slot);                    \
    if ((threadIdx.x & 63) == 0 && _i < (1u << 17)) g_stamps_kld[_i] = clk;                           \
  } while (0)
#else
#define KSTAMP(slot, clk) \
  do {                    \
  } while (0)
#endif

size_t align256(size_t v) { return (v + 255) & ~static_cast<size_t>(255); }
int kld_ranges(int HW) { return static_cast<int>(ceil_div(HW, kKldRange)); }

// Workspace regions (bytes), written by the forward and read by the backward.
struct KldLayout {
  size_t off;    // int [K + 2]: bucket starts; bucket K = prototypes with no class in [0, K)
  size_t idx;    // int [P]: prototype ids grouped by bucket, ascending within a bucket
  size_t cnt;    // int [B * K]: pixels of label c in image b
  size_t lse;    // float [B * P]: log-sum-exp of d over the prototype's class pixels
  size_t kl;     // float [B * K * 32 * 32]: KL(p_i || p_j) for class slots i, j
  size_t part;   // float [B * K * S * kKldPartFloats]: per pixel-range partials
  size_t group;  // float [B * K * 2]: per (image, class) sum of exp(-kld) and pair count
  size_t stat;   // int [4]: [0] pair count, [1] a class holds more than max_per_class prototypes
  size_t slot;   // int [P]: bucket * 256 + position in the bucket (the compact gradient's column)
  size_t rcnt;   // int [B * K * S]: class pixels in each 1024-pixel range
  size_t plist;  // int [B * K * HW]: per (image, class) the class pixels of range s at s * 1024 + q
  size_t total;
};

KldLayout kld_layout(int B, int P, int HW, int K) {
  KldLayout l;
  size_t o = 0;
  l.off = o;
  o = align256(o + static_cast<size_t>(K + 2) * 4);
  l.idx = o;
  o = align256(o + static_cast<size_t>(P) * 4);
  l.cnt = o;
  o = align256(o + static_cast<size_t>(B) * K * 4);
  l.lse = o;
  o = align256(o + static_cast<size_t>(B) * P * 4);
  l.kl = o;
  o = align256(o + static_cast<size_t>(B) * K * kKldPair * 4);
  l.part = o;  // range partials (forward), then the backward's (w, KL) coefficient pairs
  const size_t per_bc = std::max(static_cast<size_t>(kld_ranges(HW)) * kKldPartFloats, static_cast<size_t>(2 * kKldPair));
  o = align256(o + static_cast<size_t>(B) * K * per_bc * 4);
  l.group = o;
  o = align256(o + static_cast<size_t>(B) * K * 2 * 4);
  l.stat = o;
  o = align256(o + 16);
  l.slot = o;
  o = align256(o + static_cast<size_t>(P) * 4);
  l.rcnt = o;
  o = align256(o + static_cast<size_t>(B) * K * kld_ranges(HW) * 4);
  l.plist = o;
  o = align256(o + static_cast<size_t>(B) * K * HW * 4);
  l.total = o;
  return l;
}

struct KldPtrs {
  int *off, *idx, *cnt, *stat;
  float *lse, *kl, *part, *group;
  int *slot, *rcnt, *plist;
};

KldPtrs kld_ptrs(void* ws, const KldLayout& l) {
  unsigned char* b = static_cast<unsigned char*>(ws);
  return {reinterpret_cast<int*>(b + l.off),    reinterpret_cast<int*>(b + l.idx),
          reinterpret_cast<int*>(b + l.cnt),    reinterpret_cast<int*>(b + l.stat),
          reinterpret_cast<float*>(b + l.lse),  reinterpret_cast<float*>(b + l.kl),
          reinterpret_cast<float*>(b + l.part), reinterpret_cast<float*>(b + l.group),
          reinterpret_cast<int*>(b + l.slot),   reinterpret_cast<int*>(b + l.rcnt),
          reinterpret_cast<int*>(b + l.plist)};
}

constexpr int kKldListMaxP = 1 << 20;

__device__ __forceinline__ int lane_rank(unsigned long long m) {  // set bits of m below this lane
  return __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(m >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(m), 0));
}

// One wave scans proto_class (64 prototypes per step) for bucket c (module.py:173: nonzero of the
// identity column = the prototypes whose class is c, ascending; bucket K: no class in [0, K)):
// its start in the bucket order and count, the first kKldMaxPerClass members into `first`, and
// with `publish` every member into idx / slot and the start into off[c] (the lists later
// kernels read: the owner workgroup of each bucket writes them in the forward's first launch).
__device__ __forceinline__ void class_list_scan(const int32_t* __restrict__ proto_class, int P, int K, int c,
                                                bool publish, int* first, int* start_out, int* cnt_out,
                                                int* __restrict__ off, int* __restrict__ idx, int* __restrict__ slot) {
  const int lane = threadIdx.x & 63;
  // one pass: the bucket start (prototypes of lower buckets) and the members in ascending order;
  // eight chunks' loads in flight at a time (the scan is on the workgroup's critical path)
  int start = 0, cnt = 0;
  for (int p0 = 0; p0 < P; p0 += 8 * 64) {
    int bk[8], pcv[8];
    // clamped, unconditional loads, pinned before any use: otherwise the compiler sinks each load
    // into its `p < P` branch with a wait of its own, eight round trips instead of one
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int p = p0 + 64 * u + lane;
      pcv[u] = proto_class[p < P ? p : P - 1];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) asm volatile("" : "+v"(pcv[u]));
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int p = p0 + 64 * u + lane, pc = pcv[u];
      bk[u] = p < P ? ((pc >= 0 && pc < K) ? pc : K) : K + 1;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int p = p0 + 64 * u + lane;
      start += __popcll(__ballot(bk[u] < c));
      const bool in = bk[u] == c;
      const unsigned long long m = __ballot(in);
      if (in && cnt + lane_rank(m) < kKldMaxPerClass) first[cnt + lane_rank(m)] = p;
      cnt += __popcll(m);
    }
  }
  if (publish) {  // the bucket's published list (a second pass: members past the first 32 too)
    int r0 = 0;
    for (int p0 = 0; p0 < P; p0 += 64) {
      const int p = p0 + lane;
      const int pc = p < P ? proto_class[p] : -1;
      const bool in = p < P && ((pc >= 0 && pc < K) ? pc : K) == c;
      const unsigned long long m = __ballot(in);
      if (in) {
        const int r = r0 + lane_rank(m);
        idx[start + r] = p;
        // the compact gradient's column: class * 256 + rank; a rank past 255 would wrap into the
        // next class's code, and such a class holds more prototypes than any max_per_class (its
        // groups add no pairs), so its prototypes get class -2, which no pixel carries
        slot[p] = r < 256 ? c * 256 + r : -2 * 256;
      }
      r0 += __popcll(m);
    }
    if (lane == 0) {
      off[c] = start;
      if (c == K) off[K + 1] = start + cnt;
    }
  }
  *start_out = start;
  *cnt_out = cnt;
}

template <typename TL>
__device__ __forceinline__ long long label_at(const TL* lab, int n) {
  return static_cast<long long>(lab[n]);
}


// n / d for 0 <= n < 2^23, d >= 1 with r = 1/d (v_rcp_f32, 1 ulp): the quotient estimate is
// within 1 of n / d, one correction step makes it exact; replaces the ~25-instruction integer
// division the compiler emits for a runtime divisor in the per-element task decompositions.
__device__ __forceinline__ int qdiv(int n, int d, float r) {
  int q = static_cast<int>(static_cast<float>(n) * r);
  const int rem = n - __mul24(q, d);
  q += rem >= d ? 1 : 0;
  q -= rem < 0 ? 1 : 0;
  return q;
}
__device__ __forceinline__ float qrcp(int d) { return __builtin_amdgcn_rcpf(static_cast<float>(d)); }

// Gathers rows[i][q] = d[s_proto[i]][list[q]] for i < npc, q < kq over the workgroup's threads
// (q fastest: consecutive lanes read consecutive class pixels of one prototype row), kG loads in
// flight per thread (pinned batches: the LDS address reads together, then the loads).
template <int kG>
__device__ __forceinline__ void gather_tasks(const float* __restrict__ db, int HW, const int* list, int kq,
                                             const int* s_proto, int npc, float* rows, int stride) {
  const int T = npc * kq;
  const float rk = qrcp(kq);
  // kG tasks per thread in flight: their LDS address reads, then their loads
  for (int t0 = threadIdx.x; t0 < T; t0 += kG * kKldThreads) {
    int pr[kG], lq[kG], ro[kG];
#pragma unroll
    for (int u = 0; u < kG; ++u) {
      const int t = t0 + u * kKldThreads;
      const int i = qdiv(t, kq, rk), q = t - i * kq;  // q < kq for every t: a valid list entry
      ro[u] = i * stride + q;
      pr[u] = s_proto[i < npc ? i : 0];
      lq[u] = list[q];
    }
    pin_batch(pr);
    pin_batch(lq);
    float v[kG];
#pragma unroll
    for (int u = 0; u < kG; ++u) v[u] = db[static_cast<size_t>(pr[u]) * HW + lq[u]];  // clamped: valid
    pin_batch(v);
#pragma unroll
    for (int u = 0; u < kG; ++u)
      if (t0 + u * kKldThreads < T) rows[ro[u]] = v[u];
  }
}

// Merge of two (max, sum exp(. - max)) pairs; an empty side is (-inf, 0).
__device__ __forceinline__ void lse_merge(float& m, float& s, float mo, float so) {
  const float mm = fmaxf(m, mo);
  s = (mm == -INFINITY) ? 0.f : s * expf(m - mm) + so * expf(mo - mm);
  m = mm;
}

// One workgroup per (class c, image b, pixel range s of 1024). The range's class pixels are
// compacted once (ballots, one prefix over the (row, wave) counts: pixel order kept) into an LDS
// list, which also goes to plist / rcnt for the backward. Then ONE pass over the list (online
// log-sum-exp): per chunk of 256 class pixels the distances are gathered into LDS, the chunk's
// max per prototype updates the running max m_i, the accumulators S_i = sum e_i and T_ij = sum
// e_i (z_i - z_j) (e_i = exp(z_i - m_i)) are rescaled by exp(m_old - m_new), and the chunk is
// added. The range partial (m_i, S_i, T_ij, count) is the one a separate max pass would give, up
// to rounding. LDS (dynamic): [mpc][257] e | [mpc][257] z, or with RC (recompute) [mpc][257] z
// only: e_i = exp(z_i - m_i) is recomputed where used (the same expression: same bits), half the
// LDS and more workgroups per CU for many prototypes per class, but more VGPRs (kld_recompute).
template <typename TL, bool RC>
__global__ __launch_bounds__(kKldThreads) __attribute__((amdgpu_waves_per_eu(5))) void kld_partial_kernel(const float* __restrict__ dist, int P, int HW,
                                                                  const TL* __restrict__ label, int K, int mpc,
                                                                  const int32_t* __restrict__ proto_class,
                                                                  int* __restrict__ off, int* __restrict__ idx,
                                                                  int* __restrict__ slot,
                                                                  float* __restrict__ part, int* __restrict__ rcnt,
                                                                  int* __restrict__ plist) {
  extern __shared__ __attribute__((aligned(16))) float kld_smem[];
  __shared__ int s_proto[kKldMaxPerClass];
  __shared__ float s_m[kKldMaxPerClass];
  __shared__ float s_scale[kKldMaxPerClass];
  __shared__ int s_wc[kKldRange / 64];
  __shared__ int s_list[kKldRange];
  __shared__ int s_cnt;
  constexpr int kRows = kKldRange / kKldThreads;
  const int c = blockIdx.x, b = blockIdx.y, rs = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  KSTAMP(7, __builtin_amdgcn_s_memrealtime());
  KSTAMP(0, __builtin_amdgcn_s_memtime());
  const TL* lab = label + static_cast<size_t>(b) * HW;
  const int n0 = rs * kKldRange, n1 = min(HW, n0 + kKldRange);
  bool in[kRows];
  int below[kRows];
#pragma unroll
  for (int r = 0; r < kRows; ++r) {  // all label loads in flight together (under the list scan);
    const int n = n0 + r * kKldThreads + tid;  // clamped, unconditional (see class_list_scan)
    const long long l = label_at(lab, n < n1 ? n : n0);
    in[r] = n < n1 && l == c;
  }
  // the class's prototype list (was a launch of its own): wave 0 of every workgroup scans
  // proto_class; the (image 0, range 0) workgroup of bucket c publishes it, the one of bucket
  // K - 1 also bucket K's (the prototypes without a class)
  const bool publish = b == 0 && rs == 0;
  if (wave == 0) {
    int st, cnt;
    class_list_scan(proto_class, P, K, c, publish, s_proto, &st, &cnt, off, idx, slot);
    if (lane == 0) s_cnt = cnt;
  } else if (wave == 1 && publish && c == K - 1) {  // bucket K: published only (its first
    int st, cnt;                                      // members land in s_list, rewritten below)
    class_list_scan(proto_class, P, K, K, true, s_list, &st, &cnt, off, idx, slot);
  }
#pragma unroll
  for (int r = 0; r < kRows; ++r) {
    const unsigned long long bal = __ballot(in[r]);
    below[r] = lane_rank(bal);
    if (lane == 0) s_wc[r * (kKldThreads / 64) + wave] = __popcll(bal);
  }
  if (tid < kKldMaxPerClass) s_m[tid] = -INFINITY;
  __syncthreads();
  KSTAMP(1, __builtin_amdgcn_s_memtime());
  const int npc_all = s_cnt;
  const int npc = npc_all < mpc ? npc_all : mpc;
  const size_t bc = static_cast<size_t>(b) * K + c;
  float* out = part + (bc * gridDim.z + rs) * kKldPartFloats;
  int* rc = rcnt + bc * gridDim.z + rs;
  if (npc < 1 || npc_all > mpc) {  // no prototype of the class, or the overflow case (loss is NaN)
    if (tid == 0) {
      out[2 * kKldMaxPerClass] = 0.f;
      *rc = 0;
    }
    return;
  }
  int total = 0;
  int* pl = plist + bc * HW + n0;
#pragma unroll
  for (int r = 0; r < kRows; ++r) {
    int pos = total + below[r];
    for (int w = 0; w < kKldThreads / 64; ++w) {
      const int v = s_wc[r * (kKldThreads / 64) + w];
      pos += w < wave ? v : 0;
      total += v;
    }
    if (in[r]) {
      const int n = n0 + r * kKldThreads + tid;
      s_list[pos] = n;
      pl[pos] = n;
    }
  }
  if (tid == 0) *rc = total;
  if (total == 0) {  // uniform
    if (tid == 0) out[2 * kKldMaxPerClass] = 0.f;
    KSTAMP(6, __builtin_amdgcn_s_memtime());
    return;
  }
  __syncthreads();
  KSTAMP(2, __builtin_amdgcn_s_memtime());
  const float* db = dist + static_cast<size_t>(b) * P * HW;

  float* se = kld_smem;                                      // [npc][257] (stored e)
  float* sz = RC ? kld_smem : kld_smem + npc * kKldLdsStride;  // [npc][257]
  const int E = npc * npc;
  // T_ij in 4 x 4 register blocks: thread = (block (bi, bj), pixel group g); per pixel it reads
  // e and z of its 4 rows and z of its 4 columns (12 LDS values for 16 fma, where one thread per
  // entry read 3 per fma: the LDS reads, not the fma, bounded the chunk) and the 4 rows' sum e_i.
  const int nbi = (npc + 3) >> 2, nblk = nbi * nbi;
  int G = kKldThreads / nblk;
  G = G > 64 ? 64 : G;
  const int blk = tid / G, g = tid - blk * G;  // G >= 4: the divisions are by small powers / ints once
  const bool worker = blk < nblk;
  const int bi = worker ? blk / nbi : 0, bj = worker ? blk - bi * nbi : 0;
  const int i0 = 4 * bi, j0 = 4 * bj;
  int ri[4], rj[4];  // LDS row offsets, clamped into the class's rows (rows past npc are discarded)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    ri[r] = min(i0 + r, npc - 1) * kKldLdsStride;
    rj[r] = min(j0 + r, npc - 1) * kKldLdsStride;
  }
  float acc[4][4], ssum[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    ssum[r] = 0.f;
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) acc[r][cc] = 0.f;
  }
  for (int base = 0; base < total; base += kKldThreads) {
    const int kq = min(kKldThreads, total - base);
    gather_tasks<4>(db, HW, s_list + base, kq, s_proto, npc, sz, kKldLdsStride);
    __syncthreads();
    if (base == 0) KSTAMP(3, __builtin_amdgcn_s_memtime());
    {  // chunk max per prototype (8 threads per row) -> running max and the rescale factor
      const int i = tid >> 3, l8 = tid & 7;
      float mx = -INFINITY;
      if (i < npc)
        for (int q = l8; q < kq; q += 32) {  // 4 LDS reads in flight (clamped: a repeat changes no max)
          float t[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) t[u] = sz[i * kKldLdsStride + (q + 8 * u < kq ? q + 8 * u : q)];
          pin_batch(t);
#pragma unroll
          for (int u = 0; u < 4; ++u) mx = fmaxf(mx, t[u]);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 1));
      mx = fmaxf(mx, __shfl_xor(mx, 2));
      mx = fmaxf(mx, __shfl_xor(mx, 4));
      if (i < npc && l8 == 0) {
        const float mo = s_m[i], mn = fmaxf(mo, mx);
        s_scale[i] = expf(mo - mn);  // mo = -inf (first chunk with pixels): 0, nothing to rescale
        s_m[i] = mn;
      }
    }
    __syncthreads();
    float mr[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float sc = s_scale[min(i0 + r, npc - 1)];
      mr[r] = s_m[min(i0 + r, npc - 1)];
      ssum[r] *= sc;
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) acc[r][cc] *= sc;
    }
    if constexpr (!RC) {
      const float rk = qrcp(kq);
      for (int t = tid; t < npc * kq; t += kKldThreads) {
        const int i = qdiv(t, kq, rk), q = t - i * kq;
        se[i * kKldLdsStride + q] = expf(sz[i * kKldLdsStride + q] - s_m[i]);
      }
      __syncthreads();
    }
    if (worker) {
      for (int q = g; q < kq; q += G) {
        float e[4], zi[4], zj[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          zi[r] = sz[ri[r] + q];
          zj[r] = sz[rj[r] + q];
          e[r] = RC ? expf(zi[r] - mr[r]) : se[ri[r] + q];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          ssum[r] += e[r];
#pragma unroll
          for (int cc = 0; cc < 4; ++cc) acc[r][cc] = fmaf(e[r], zi[r] - zj[cc], acc[r][cc]);
        }
      }
    }
    __syncthreads();
  }
  KSTAMP(4, __builtin_amdgcn_s_memtime());
  if (tid == 0) out[2 * kKldMaxPerClass] = static_cast<float>(total);
  // the pixel groups' blocks -> LDS [block][g][16], then a fixed-order sum over g per entry
  float* red = kld_smem;
  if (worker) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) red[(blk * G + g) * 16 + r * 4 + cc] = (bi == bj && r == cc) ? ssum[r] : acc[r][cc];
  }
  __syncthreads();
  for (int e = tid; e < E; e += kKldThreads) {
    const int i = e / npc, j = e - i * npc;
    const int b2 = (i >> 2) * nbi + (j >> 2), sl = (i & 3) * 4 + (j & 3);
    float v = 0.f;
    for (int g0 = 0; g0 < G; g0 += 8) {  // 8 LDS reads in flight (clamped, pinned), added in order
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = red[(b2 * G + (g0 + u < G ? g0 + u : G - 1)) * 16 + sl];
      pin_batch(t);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (g0 + u < G) v += t[u];
    }
    if (i == j) {
      out[i] = s_m[i];
      out[kKldMaxPerClass + i] = v;
    } else {
      out[2 * kKldMaxPerClass + 1 + i * kKldMaxPerClass + j] = v;
    }
  }
  KSTAMP(5, __builtin_amdgcn_s_memtime());
}

// One workgroup per (class c, image b): merges the range partials in range order. L_i per
// slot (thread i), the per-(range, slot) factors exp(m_i^s - L_i) once each (was once per entry
// and range), then KL_ij over the workgroup's 256 threads, and this group's sum of
// exp(-kld_ij) over its pairs i < j (per-thread partials added in a fixed order).
constexpr int kKldMergeMaxS = 64;  // ranges whose factors are staged in LDS (beyond: inline)
constexpr int kKldMergeRegS = 8;   // ranges held in registers by kld_merge_regs

// kld_merge_kernel for S <= kKldMergeRegS ranges: the range partials are read into registers
// first (counts, m_i^s and S_i^s with the group's scalars; then the workgroup's T_ij^s entries),
// so the merge waits on two global round trips instead of four; operations and order are the
// general path's (bit-identical results).
__device__ __forceinline__ void kld_merge_regs(const float* __restrict__ pb, int P, int K, int S, int npc, bool valid,
                                               int c, int b, const int* __restrict__ off,
                                               const int* __restrict__ idx, int* __restrict__ cnt_out,
                                               float* __restrict__ lse_out, float* __restrict__ kl_out,
                                               float* __restrict__ group_out, float* s_L, float* s_fac,
                                               float* s_kl, float* s_sum) {
  static_assert(kKldPair % 256 == 0 && kKldMergeRegS <= kKldMergeMaxS, "merge fast path layout");
  __shared__ int s_n[kKldMergeRegS];
  const int tid = threadIdx.x;
  float mi[kKldMergeRegS], si[kKldMergeRegS];
  int nr = 0;
  if (tid < kKldMergeRegS && tid < S && valid) nr = static_cast<int>(pb[tid * kKldPartFloats + 2 * kKldMaxPerClass]);
  {  // clamped loads, pinned before the guards select (pin_batch)
    const int sc = S - 1, tc = tid < kKldMaxPerClass ? tid : 0;
#pragma unroll
    for (int s = 0; s < kKldMergeRegS; ++s) {
      mi[s] = pb[(s < S ? s : sc) * kKldPartFloats + tc];
      si[s] = pb[(s < S ? s : sc) * kKldPartFloats + kKldMaxPerClass + tc];
    }
    pin_batch(mi);
    pin_batch(si);
#pragma unroll
    for (int s = 0; s < kKldMergeRegS; ++s) {
      const bool ld = s < S && tid < npc;
      mi[s] = ld ? mi[s] : 0.f;
      si[s] = ld ? si[s] : 0.f;
    }
  }
  // the entries this thread merges (e = tid + 256 u of the npc x npc grid), all ranges
  constexpr int kU = kKldPair / 256;
  float tv[kU][kKldMergeRegS];
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const int e = tid + 256 * u, i = e / (npc > 0 ? npc : 1), j = e - i * npc;
    const int ec = e < npc * npc ? i * kKldMaxPerClass + j : 0;  // clamped, pinned below
#pragma unroll
    for (int s = 0; s < kKldMergeRegS; ++s)
      tv[u][s] = pb[(s < S ? s : S - 1) * kKldPartFloats + 2 * kKldMaxPerClass + 1 + ec];
  }
#pragma unroll
  for (int u = 0; u < kU; ++u) pin_batch(tv[u]);
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const int e = tid + 256 * u;
#pragma unroll
    for (int s = 0; s < kKldMergeRegS; ++s) tv[u][s] = (e < npc * npc && s < S) ? tv[u][s] : 0.f;
  }
  if (tid < kKldMergeRegS) s_n[tid] = tid < S ? nr : 0;
  __syncthreads();
  int cnt = 0;
  for (int s = 0; s < S; ++s) cnt += s_n[s];
  float* gsum = group_out + (static_cast<size_t>(b) * K + c) * 2;  // (sum of exp(-kld), pairs)
  if (tid == 0) cnt_out[static_cast<size_t>(b) * K + c] = cnt;
  if (cnt == 0) {
    if (tid == 0) gsum[0] = gsum[1] = 0.f;
    return;
  }
  if (tid < npc) {  // L_i, then this slot's factors exp(m_i^s - L_i)
    float M = -INFINITY, Ssum = 0.f;
#pragma unroll
    for (int s = 0; s < kKldMergeRegS; ++s)
      if (s < S && s_n[s] > 0) lse_merge(M, Ssum, mi[s], si[s]);
    const float L = M + logf(Ssum);
    s_L[tid] = L;
    lse_out[static_cast<size_t>(b) * P + idx[off[c] + tid]] = L;
#pragma unroll
    for (int s = 0; s < kKldMergeRegS; ++s) s_fac[s * kKldMaxPerClass + tid] = expf(mi[s] - L);
  }
  __syncthreads();
  if (npc < 2 || cnt < 2) {
    if (tid == 0) gsum[0] = gsum[1] = 0.f;
    return;
  }
  float* klb = kl_out + (static_cast<size_t>(b) * K + c) * kKldPair;
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const int e = tid + 256 * u;
    if (e >= npc * npc) continue;
    const int i = e / npc, j = e - i * npc;
    if (i == j) continue;
    float t = 0.f;
#pragma unroll
    for (int s = 0; s < kKldMergeRegS; ++s)
      if (s < S && s_n[s] > 0) t = fmaf(s_fac[s * kKldMaxPerClass + i], tv[u][s], t);
    const float kl = t - (s_L[i] - s_L[j]);
    klb[i * kKldMaxPerClass + j] = kl;
    s_kl[i * kKldMaxPerClass + j] = kl;
  }
  __syncthreads();
  // this group's pairs i < j: kld = (KL(p_j||p_i) + KL(p_i||p_j)) / 2 (module.py:195-199)
  float sum = 0.f;
  for (int e = tid; e < npc * npc; e += 256) {
    const int i = e / npc, j = e - i * npc;
    if (i < j) sum += expf(-((s_kl[j * kKldMaxPerClass + i] + s_kl[i * kKldMaxPerClass + j]) / 2.f));
  }
  s_sum[tid] = sum;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (tid < w) s_sum[tid] += s_sum[tid + w];
    __syncthreads();
  }
  if (tid == 0) {
    gsum[0] = s_sum[0];
    gsum[1] = static_cast<float>(npc * (npc - 1) / 2);
  }
}
__global__ __launch_bounds__(256) void kld_merge_kernel(int P, int K, int S, int mpc, const int* __restrict__ off,
                                                        const int* __restrict__ idx, const float* __restrict__ part,
                                                        int* __restrict__ cnt_out, float* __restrict__ lse_out,
                                                        float* __restrict__ kl_out, float* __restrict__ group_out) {
  __shared__ float s_L[kKldMaxPerClass];
  __shared__ float s_sc[kKldMergeMaxS][kKldMaxPerClass];
  __shared__ int s_ok[kKldMergeMaxS];
  __shared__ float s_kl[kKldPair];
  __shared__ float s_sum[256];
  __shared__ int s_cnt;
  const int c = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int npc_all = off[c + 1] - off[c];
  const int npc = npc_all < mpc ? npc_all : mpc;
  const float* pb = part + (static_cast<size_t>(b) * K + c) * S * kKldPartFloats;
  const bool valid = npc >= 1 && npc_all <= mpc;
  if (S <= kKldMergeRegS) {  // the same sums with every global read in two round trips
    kld_merge_regs(pb, P, K, S, npc, valid, c, b, off, idx, cnt_out, lse_out, kl_out, group_out, s_L, &s_sc[0][0], s_kl,
                   s_sum);
    return;
  }
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  for (int s = tid; s < S && valid; s += 256) {
    const int n = static_cast<int>(pb[s * kKldPartFloats + 2 * kKldMaxPerClass]);
    if (s < kKldMergeMaxS) s_ok[s] = n > 0;
    atomicAdd(&s_cnt, n);  // integer sum: order-free
  }
  __syncthreads();
  const int cnt = s_cnt;
  float* gsum = group_out + (static_cast<size_t>(b) * K + c) * 2;  // (sum of exp(-kld), pairs)
  if (tid == 0) cnt_out[static_cast<size_t>(b) * K + c] = cnt;
  if (cnt == 0) {
    if (tid == 0) gsum[0] = gsum[1] = 0.f;
    return;
  }
  if (tid < npc) {  // L_i = log sum_s S_i^s exp(m_i^s)  (log-sum-exp of d over the class pixels)
    float M = -INFINITY, Ssum = 0.f;
    for (int s = 0; s < S; ++s) {
      const float* q = pb + s * kKldPartFloats;
      if (q[2 * kKldMaxPerClass] > 0.f) lse_merge(M, Ssum, q[tid], q[kKldMaxPerClass + tid]);
    }
    const float L = M + logf(Ssum);
    s_L[tid] = L;
    lse_out[static_cast<size_t>(b) * P + idx[off[c] + tid]] = L;
  }
  __syncthreads();
  if (npc < 2 || cnt < 2) {
    if (tid == 0) gsum[0] = gsum[1] = 0.f;
    return;
  }
  const int Ss = S < kKldMergeMaxS ? S : kKldMergeMaxS;
  for (int t = tid; t < Ss * npc; t += 256) {
    const int s = t / npc, i = t - s * npc;
    s_sc[s][i] = expf(pb[s * kKldPartFloats + i] - s_L[i]);
  }
  __syncthreads();
  float* klb = kl_out + (static_cast<size_t>(b) * K + c) * kKldPair;
  for (int e = tid; e < npc * npc; e += 256) {
    const int i = e / npc, j = e - i * npc;
    if (i == j) continue;
    float t = 0.f;
    for (int s = 0; s < S; ++s) {
      const float* q = pb + s * kKldPartFloats;
      const bool ok = s < kKldMergeMaxS ? s_ok[s] != 0 : q[2 * kKldMaxPerClass] > 0.f;
      if (ok) {
        const float sc = s < kKldMergeMaxS ? s_sc[s][i] : expf(q[i] - s_L[i]);
        t = fmaf(sc, q[2 * kKldMaxPerClass + 1 + i * kKldMaxPerClass + j], t);
      }
    }
    const float kl = t - (s_L[i] - s_L[j]);
    klb[i * kKldMaxPerClass + j] = kl;
    s_kl[i * kKldMaxPerClass + j] = kl;
  }
  __syncthreads();
  // this group's pairs i < j: kld = (KL(p_j||p_i) + KL(p_i||p_j)) / 2 (module.py:195-199)
  float sum = 0.f;
  for (int e = tid; e < npc * npc; e += 256) {
    const int i = e / npc, j = e - i * npc;
    if (i < j) sum += expf(-((s_kl[j * kKldMaxPerClass + i] + s_kl[i * kKldMaxPerClass + j]) / 2.f));
  }
  s_sum[tid] = sum;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (tid < w) s_sum[tid] += s_sum[tid + w];
    __syncthreads();
  }
  if (tid == 0) {
    gsum[0] = s_sum[0];
    gsum[1] = static_cast<float>(npc * (npc - 1) / 2);
  }
}

// Mean over all pairs of exp(-kld) (module.py:202-206): the per-(image, class) sums of
// kld_merge_kernel added in a fixed order.
__global__ __launch_bounds__(256) void kld_finalize_kernel(int groups, const float* __restrict__ group_sums,
                                                           const int* __restrict__ off, int K, int mpc,
                                                           int* __restrict__ stat, float* __restrict__ loss_out,
                                                           int32_t* __restrict__ npairs_out) {
  __shared__ float s_sum[256], s_n[256];
  float sum = 0.f, n = 0.f;
  for (int gi = threadIdx.x; gi < groups; gi += 256) {
    sum += group_sums[2 * gi];
    n += group_sums[2 * gi + 1];
  }
  // a class holding more than max_per_class prototypes: the loss is NaN (one class per thread,
  // loads in parallel rather than a chain of dependent ones)
  int over_c = 0;
  for (int c = threadIdx.x; c < K; c += 256) over_c |= off[c + 1] - off[c] > mpc;
  s_sum[threadIdx.x] = sum;
  s_n[threadIdx.x] = n;
  const bool over = __syncthreads_or(over_c) != 0;
  for (int w = 128; w >= 1; w >>= 1) {
    if (static_cast<int>(threadIdx.x) < w) {
      s_sum[threadIdx.x] += s_sum[threadIdx.x + w];
      s_n[threadIdx.x] += s_n[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const int np = static_cast<int>(s_n[0]);
    float loss = np > 0 ? s_sum[0] / static_cast<float>(np) : 0.f;
    if (over) loss = __builtin_nanf("");
    stat[0] = np;
    stat[1] = over ? 1 : 0;
    loss_out[0] = loss;
    if (npairs_out) npairs_out[0] = np;
  }
}

// Backward coefficients per (class c, image b): w_ij = -g_loss exp(-kld_ij) / n_pairs (mean,
// exp(-x) and the /2 of module.py:199-206 differentiated; w_ii = 0), and per slot i the group
// constants R_i = sum_j w_ij and WK_i = sum_j w_ij KL_ij of the regrouped gradient (kld_slot_grad).
// Layout per group (kKldCoefFloats): w [npc][npc] | (R_i, WK_i) [npc] at kKldPair.
constexpr int kKldCoefFloats = kKldPair + 2 * kKldMaxPerClass;
__global__ __launch_bounds__(64) void kld_coef_kernel(int K, int mpc, const int* __restrict__ off,
                                                      const int* __restrict__ cnt, const float* __restrict__ kl,
                                                      const int* __restrict__ stat, const float* __restrict__ g_loss,
                                                      float* __restrict__ coef) {
  __shared__ float s_w[kKldPair];
  const int c = blockIdx.x, b = blockIdx.y;
  const int npc = off[c + 1] - off[c];
  const int np = stat[0];
  if (npc < 2 || npc > mpc || np == 0 || cnt[static_cast<size_t>(b) * K + c] < 2) return;
  const float gl = g_loss ? g_loss[0] : 1.f;
  const float* klb = kl + (static_cast<size_t>(b) * K + c) * kKldPair;
  float* cb = coef + (static_cast<size_t>(b) * K + c) * kKldCoefFloats;
  for (int e = threadIdx.x; e < npc * npc; e += 64) {
    const int i = e / npc, j = e - i * npc;
    // the merge kernel leaves KL's diagonal unwritten (workspace garbage, possibly NaN): w_ii = 0
    // and KL_ii = 0 keep it out of every sum
    const float kij = i == j ? 0.f : klb[i * kKldMaxPerClass + j], kji = i == j ? 0.f : klb[j * kKldMaxPerClass + i];
    const float w = i == j ? 0.f : -(gl / static_cast<float>(np)) * expf(-((kji + kij) / 2.f));
    s_w[e] = w;
    cb[e] = w;
  }
  __syncthreads();
  const int i = threadIdx.x;
  if (i < npc) {
    float r = 0.f, wk = 0.f;
    for (int j = 0; j < npc; ++j) {
      const float w = s_w[i * npc + j];
      r += w;
      wk = fmaf(w, i == j ? 0.f : klb[i * kKldMaxPerClass + j], wk);
    }
    cb[kKldPair + 2 * i] = r;
    cb[kKldPair + 2 * i + 1] = wk;
  }
}

// d(g_loss * loss) / d z_i at one pixel of a contributing (image, class) group, regrouped from
// the autograd of log_softmax + the two kl_div per pair (module.py:183-206):
//   g_i = sum_j w_ij (p_i (lp_i - lp_j - KL_ij + 1) - p_j) / 2
//       = (p_i ((lp_i + 1) R_i - WK_i - sum_j w_ij lp_j) - sum_j w_ij p_j) / 2
// Two dot products per slot (four chains over j, fixed-order sum); `lp(j)` / `p(j)` read the
// pixel's log-probabilities / probabilities, `w(j)` row i of the group's w. Both gradient layouts
// (dense kld_grad_kernel, compact kld_grad_compact_kernel) call this: compact == dense bit for bit.
template <typename LP, typename PJ, typename WJ>
__device__ __forceinline__ float kld_slot_grad(int npc, float pi, float li, float ri, float wki, LP lp, PJ pj, WJ w) {
  float a[4] = {0.f, 0.f, 0.f, 0.f}, q[4] = {0.f, 0.f, 0.f, 0.f};
  int j = 0;
  for (; j + 3 < npc; j += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float wj = w(j + u);
      a[u] = fmaf(wj, lp(j + u), a[u]);
      q[u] = fmaf(wj, pj(j + u), q[u]);
    }
  }
  for (; j < npc; ++j) {
    const float wj = w(j);
    a[0] = fmaf(wj, lp(j), a[0]);
    q[0] = fmaf(wj, pj(j), q[0]);
  }
  const float A = (a[0] + a[1]) + (a[2] + a[3]), Q = (q[0] + q[1]) + (q[2] + q[3]);
  return 0.5f * (pi * ((li + 1.f) * ri - wki - A) - Q);
}

// kld_slot_grad for the four slots i0 .. i0 + 3 at once (the pixel's lp_j / p_j read once for
// the four): each slot's operations and order are kld_slot_grad's, so the results are its bits.
// Slots past npc repeat slot npc - 1 (their results are not stored).
template <typename LP, typename PJ, typename WIJ>
__device__ __forceinline__ void kld_block_grad(int npc, int i0, const float (&pi)[4], const float (&li)[4],
                                               const float (&ri)[4], const float (&wki)[4], LP lp, PJ pj, WIJ w,
                                               float (&g)[4]) {
  float a[4][4], q[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int u = 0; u < 4; ++u) a[r][u] = q[r][u] = 0.f;
  int ii[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) ii[r] = min(i0 + r, npc - 1);
  int j = 0;
  for (; j + 3 < npc; j += 4) {
    float lj[4], pjv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      lj[u] = lp(j + u);
      pjv[u] = pj(j + u);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float wj = w(ii[r], j + u);
        a[r][u] = fmaf(wj, lj[u], a[r][u]);
        q[r][u] = fmaf(wj, pjv[u], q[r][u]);
      }
  }
  for (; j < npc; ++j) {
    const float lj = lp(j), pjv = pj(j);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float wj = w(ii[r], j);
      a[r][0] = fmaf(wj, lj, a[r][0]);
      q[r][0] = fmaf(wj, pjv, q[r][0]);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float A = (a[r][0] + a[r][1]) + (a[r][2] + a[r][3]), Q = (q[r][0] + q[r][1]) + (q[r][2] + q[r][3]);
    g[r] = 0.5f * (pi[r] * ((li[r] + 1.f) * ri[r] - wki[r] - A) - Q);
  }
}

// d(g_loss * loss)/d d for one 256-pixel chunk of image b, thread = pixel. For a pixel of label
// c and class slot i (autograd of log_softmax + the two kl_div per pair, module.py:183-206):
//   g_i = sum_{j != i} w_ij (p_i (lp_i - lp_j - KL_ij + 1) - p_j) / 2.
// Every row of g_dist is written at the chunk's pixels (zero off each prototype's class), so the
// grid writes the whole [B, P, HW] tensor once, row segments coalesced across the threads.
// LDS (dynamic): [mpc][257] p | [mpc][257] log p | [mpc][257] g, this thread's column only.
template <typename TL>
__global__ __launch_bounds__(kKldThreads) void kld_grad_kernel(
    const float* __restrict__ dist, int P, int HW, const TL* __restrict__ label, int K, int mpc,
    const int* __restrict__ off, const int* __restrict__ idx, const int* __restrict__ cnt,
    const float* __restrict__ lse, const float* __restrict__ coef, const int* __restrict__ stat,
    float* __restrict__ g_dist) {
  extern __shared__ __attribute__((aligned(16))) float kld_smem[];
  const int b = blockIdx.y, tid = threadIdx.x;
  const int n = blockIdx.x * kKldThreads + tid;
  if (n >= HW) return;  // no barrier below
  float* sp = kld_smem;
  float* slp = sp + mpc * kKldLdsStride;
  float* sg = slp + mpc * kKldLdsStride;
  const long long lv = label_at(label + static_cast<size_t>(b) * HW, n);
  int c = (lv >= 0 && lv < K) ? static_cast<int>(lv) : -1;
  int npc = 0, o0 = 0;
  if (c >= 0) {
    o0 = off[c];
    npc = off[c + 1] - o0;
    if (npc < 2 || npc > mpc || stat[0] == 0 || cnt[static_cast<size_t>(b) * K + c] < 2) c = -1;
  }
  const float* db = dist + static_cast<size_t>(b) * P * HW;
  if (c >= 0) {
    for (int i = 0; i < npc; ++i) {
      const int pi = idx[o0 + i];
      const float lp = db[static_cast<size_t>(pi) * HW + n] - lse[static_cast<size_t>(b) * P + pi];
      slp[i * kKldLdsStride + tid] = lp;
      sp[i * kKldLdsStride + tid] = expf(lp);
    }
    const float* cb = coef + (static_cast<size_t>(b) * K + c) * kKldCoefFloats;
    for (int i = 0; i < npc; ++i) {
      sg[i * kKldLdsStride + tid] = kld_slot_grad(
          npc, sp[i * kKldLdsStride + tid], slp[i * kKldLdsStride + tid], cb[kKldPair + 2 * i], cb[kKldPair + 2 * i + 1],
          [&](int j) { return slp[j * kKldLdsStride + tid]; }, [&](int j) { return sp[j * kKldLdsStride + tid]; },
          [&](int j) { return cb[i * npc + j]; });
    }
  }
  float* gb = g_dist + static_cast<size_t>(b) * P * HW + n;
  for (int cc = 0; cc <= K; ++cc) {
    const int a0 = off[cc], a1 = off[cc + 1];
    for (int k = a0; k < a1; ++k) {
      const float v = (cc == c) ? sg[(k - a0) * kKldLdsStride + tid] : 0.f;
      gb[static_cast<size_t>(idx[k]) * HW] = v;
    }
  }
}

// The same gradient in the compact layout the layer backward expands (l2_bwd_fused /
// l2_bwd_onepass, protoseg_l2_bwd_kld): g_cls[g][slot] (g = b * HW + n, slot = the prototype's
// position in its class) at each pixel of a contributing (image, class) group, pix_cls[g] = that
// class. pix_cls is set to -1 everywhere first (one memset); one workgroup per (class c, image
// b, pixel range s) of a contributing group then walks the range's class-pixel list the forward
// left in plist. LDS (dynamic): [mpc][257] p | [mpc][257] log p | the group's coefficients; with
// RC the p rows are not stored: p = exp(lp) is recomputed where used (same bits, kld_recompute).
//
// The same launch also writes what used to take three more: proto_slot (workgroups (c, 0, 0)
// copy their bucket's columns; the one of bucket K - 1 also bucket K's), pix_cls for every pixel
// (the workgroup of the pixel's label, class 0's for labels outside [0, K), writes c or -1: each
// pixel exactly once, no memset), and the group's coefficients (kld_coef_kernel's arithmetic, in
// LDS).
template <typename TL, bool RC>
__global__ __launch_bounds__(kKldThreads) __attribute__((amdgpu_waves_per_eu(5))) void kld_grad_compact_kernel(
    const float* __restrict__ dist, int P, int HW, const TL* __restrict__ label, int K, int mpc,
    const int* __restrict__ off, const int* __restrict__ idx, const int* __restrict__ slot,
    const int* __restrict__ cnt, const float* __restrict__ lse, const float* __restrict__ kl,
    const int* __restrict__ stat, const float* __restrict__ g_loss, const int* __restrict__ rcnt,
    const int* __restrict__ plist, float* __restrict__ g_cls, int32_t* __restrict__ pix_cls,
    int32_t* __restrict__ proto_slot) {
  extern __shared__ __attribute__((aligned(16))) float kld_smem[];
  __shared__ int s_proto[kKldMaxPerClass];
  __shared__ float s_lse[kKldMaxPerClass];
  __shared__ int s_lq[kKldThreads];  // the chunk's class pixels (the gather's addresses from LDS)
  __shared__ float s_klg[kKldPair];  // the group's KL_ij (0 on the diagonal)
  constexpr int kRows = kKldRange / kKldThreads;
  const int c = blockIdx.x, b = blockIdx.y, rs = blockIdx.z, tid = threadIdx.x;
  const size_t bc = static_cast<size_t>(b) * K + c;
  // The prologue's global reads in three round trips: (1) the group's scalars and the range's
  // labels, (2) what depends on them (this thread's prototype id, its KL entries, the class-pixel
  // list), (3) the log-sum-exps and the first chunk's distances.
  const int o0 = off[c], o1 = off[c + 1];
  const int np = stat[0], ncls = cnt[bc], q1 = rcnt[bc * gridDim.z + rs];
  const TL* lab = label + static_cast<size_t>(b) * HW;
  const int n0 = rs * kKldRange, n1 = min(HW, n0 + kKldRange);
  long long lv[kRows];
#pragma unroll
  for (int r = 0; r < kRows; ++r) {
    const int n = n0 + r * kKldThreads + tid;
    const long long l = label_at(lab, n < n1 ? n : n0);  // clamped, unconditional
    lv[r] = n < n1 ? l : -1;
  }
  const int npc = o1 - o0;
  const bool contributes = npc >= 2 && npc <= mpc && np != 0 && ncls >= 2;
  {  // pix_cls: the pixels whose label is c (c = 0 also takes labels outside [0, K))
    int32_t* pcb = pix_cls + static_cast<size_t>(b) * HW;
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      const int n = n0 + r * kKldThreads + tid;
      const long long l = lv[r];
      const int owner = (l >= 0 && l < K) ? static_cast<int>(l) : 0;
      if (n < n1 && owner == c) pcb[n] = (l == c && contributes) ? c : -1;
    }
  }
  if (b == 0 && rs == 0) {
    for (int r = tid; r < npc; r += kKldThreads) proto_slot[idx[o0 + r]] = slot[idx[o0 + r]];
    if (c == K - 1)
      for (int r = off[K] + tid; r < off[K + 1]; r += kKldThreads) proto_slot[idx[r]] = slot[idx[r]];
  }
  if (!contributes || q1 == 0) return;  // uniform: the group adds no pair here
  const int* pl = plist + bc * HW + rs * kKldRange;
  float* sp = kld_smem;  // (stored p)
  float* slp = RC ? kld_smem : kld_smem + mpc * kKldLdsStride;
  float* scoef = slp + mpc * kKldLdsStride;  // w [npc][npc] | (R_i, WK_i) at kKldPair
  const float* klb = kl + bc * kKldPair;
  const int my_p = tid < npc ? idx[o0 + tid] : 0;
  {  // kld_coef_kernel's coefficients, same operations; KL_ij also into s_klg for the R / WK sums
    // (their guarded global reads compiled to a branch and a wait per j: a round trip each)
    const float gl = g_loss ? g_loss[0] : 1.f;
    for (int e = tid; e < npc * npc; e += kKldThreads) {
      const int i = e / npc, j = e - i * npc;
      float kk[2] = {klb[i * kKldMaxPerClass + j], klb[j * kKldMaxPerClass + i]};  // diagonal read, unused
      pin_batch(kk);
      const float kij = i == j ? 0.f : kk[0], kji = i == j ? 0.f : kk[1];
      s_klg[e] = kij;
      scoef[e] = i == j ? 0.f : -(gl / static_cast<float>(np)) * expf(-((kji + kij) / 2.f));
    }
  }
  if (tid < npc) {
    s_proto[tid] = my_p;
    s_lse[tid] = lse[static_cast<size_t>(b) * P + my_p];
  }
  if (tid < q1) s_lq[tid] = pl[tid];  // the first chunk's list, in the same round trip
  __syncthreads();
  if (tid < npc) {
    float r = 0.f, wk = 0.f;
    for (int j = 0; j < npc; ++j) {
      const float w = scoef[tid * npc + j];
      r += w;
      wk = fmaf(w, s_klg[tid * npc + j], wk);  // 0 on the diagonal
    }
    scoef[kKldPair + 2 * tid] = r;
    scoef[kKldPair + 2 * tid + 1] = wk;
  }
  const float* db = dist + static_cast<size_t>(b) * P * HW;
  for (int base = 0; base < q1; base += kKldThreads) {  // chunks of 256 class pixels
    const int kq = min(kKldThreads, q1 - base);
    const int* lq = s_lq;
    if (base > 0) {  // the previous chunk's loop-end barrier has passed: every s_lq read is done
      if (tid < kq) s_lq[tid] = pl[base + tid];
      __syncthreads();
    }
    gather_tasks<8>(db, HW, lq, kq, s_proto, npc, slp, kKldLdsStride);
    __syncthreads();
    const float rk = qrcp(kq);
    for (int t = tid; t < npc * kq; t += kKldThreads) {
      const int i = qdiv(t, kq, rk), q = t - i * kq;
      const float lp = slp[i * kKldLdsStride + q] - s_lse[i];
      slp[i * kKldLdsStride + q] = lp;
      if constexpr (!RC) sp[i * kKldLdsStride + q] = expf(lp);
    }
    __syncthreads();
    // one task per (pixel, block of 4 class slots), pixel fastest: a wave's lanes share the slot
    // block, so the w reads are broadcasts, and a pixel's lp_j / p_j are read once for its 4
    // slots; each slot is kld_slot_grad's sequence, so compact == dense bit for bit
    const int nib = (npc + 3) >> 2;
    for (int t = tid; t < nib * kq; t += kKldThreads) {
      const int ib = qdiv(t, kq, rk), q = t - ib * kq;
      float pi[4], li[4], ri[4], wki[4], g[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = min(4 * ib + r, npc - 1);
        li[r] = slp[i * kKldLdsStride + q];
        pi[r] = RC ? expf(li[r]) : sp[i * kKldLdsStride + q];
        ri[r] = scoef[kKldPair + 2 * i];
        wki[r] = scoef[kKldPair + 2 * i + 1];
      }
      kld_block_grad(
          npc, 4 * ib, pi, li, ri, wki, [&](int j) { return slp[j * kKldLdsStride + q]; },
          [&](int j) { return RC ? expf(slp[j * kKldLdsStride + q]) : sp[j * kKldLdsStride + q]; },
          [&](int i, int j) { return scoef[i * npc + j]; }, g);
      float* row = g_cls + (static_cast<size_t>(b) * HW + lq[q]) * mpc;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * ib + r < npc) row[4 * ib + r] = g[r];
    }
    __syncthreads();
  }
}

// Dense g_dist from the compact layout (protoseg_kld_expand): one thread per (image, prototype,
// pixel), row segments coalesced.
__global__ __launch_bounds__(256) void kld_expand_kernel(const float* __restrict__ g_cls,
                                                         const int32_t* __restrict__ pix_cls,
                                                         const int32_t* __restrict__ proto_slot, int P, int HW,
                                                         int mpc, int accumulate, float* __restrict__ g_dist) {
  const int n = blockIdx.x * 256 + threadIdx.x, p = blockIdx.y, b = blockIdx.z;
  if (n >= HW) return;
  const size_t g = static_cast<size_t>(b) * HW + n;
  const int sl = proto_slot[p];
  const float v = pix_cls[g] == (sl >> 8) ? g_cls[g * mpc + (sl & 255)] : 0.f;
  float* o = g_dist + (static_cast<size_t>(b) * P + p) * HW + n;
  *o = accumulate ? *o + v : v;
}

int kld_check(const float* dist, int B, int P, int HW, const void* label, int label_dtype, const int32_t* proto_class,
              int K, int max_per_class, const void* ws, size_t ws_bytes) {
  if (!dist || !label || !proto_class || !ws) return fail(PROTOSEG_ERR_INVALID, "null pointer argument");
  if (B <= 0 || P <= 0 || HW <= 0 || K <= 0)
    return fail(PROTOSEG_ERR_INVALID, "bad shape B=%d P=%d HW=%d K=%d", B, P, HW, K);
  if (K > kKldMaxClasses) return fail(PROTOSEG_ERR_UNSUPPORTED, "K=%d > %d classes", K, kKldMaxClasses);
  if (P > kKldListMaxP) return fail(PROTOSEG_ERR_UNSUPPORTED, "P=%d > %d prototypes", P, kKldListMaxP);
  if (max_per_class < 1 || max_per_class > kKldMaxPerClass)
    return fail(PROTOSEG_ERR_UNSUPPORTED, "max_per_class=%d outside [1, %d]", max_per_class, kKldMaxPerClass);
  if (label_dtype != PROTOSEG_I64 && label_dtype != PROTOSEG_I32 && label_dtype != PROTOSEG_U8)
    return fail(PROTOSEG_ERR_UNSUPPORTED, "label_dtype %d", label_dtype);
  if (static_cast<unsigned long long>(B) * P * HW >= (1ull << 31))
    return fail(PROTOSEG_ERR_UNSUPPORTED, "B*P*HW >= 2^31");
  const size_t need = kld_layout(B, P, HW, K).total;
  if (ws_bytes < need) return fail(PROTOSEG_ERR_INVALID, "workspace %zu B < %zu B", ws_bytes, need);
  return PROTOSEG_OK;
}

template <auto K>
struct KernelTag {
  static constexpr auto value = K;
};

// Recompute e / p instead of storing their rows (the RC kernels) when the stored rows would hold
// the partial / compact kernels to fewer workgroups per CU than their extra VGPRs do: measured
// (profiles/r04/r4t_ab_kld*.log) faster at 19 prototypes per class, slower at 10.
bool kld_recompute(int mpc) { return mpc > 12; }

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

extern "C" size_t protoseg_kld_workspace_size(int B, int P, int HW, int K) {
  if (B <= 0 || P <= 0 || HW <= 0 || K <= 0) return 0;
  return kld_layout(B, P, HW, K).total;
}

extern "C" int protoseg_kld_forward(const float* dist, int B, int P, int HW, const void* label, int label_dtype,
                                    const int32_t* proto_class, int K, int max_per_class, float* loss_out,
                                    int32_t* npairs_out, void* workspace, size_t workspace_bytes,
                                    protoseg_stream_t stream) {
  if (int st = kld_check(dist, B, P, HW, label, label_dtype, proto_class, K, max_per_class, workspace, workspace_bytes))
    return st;
  if (!loss_out) return fail(PROTOSEG_ERR_INVALID, "loss_out must be non-null");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const KldLayout l = kld_layout(B, P, HW, K);
  const KldPtrs w = kld_ptrs(workspace, l);
  const int S = kld_ranges(HW);
  const bool rc = kld_recompute(max_per_class);
  const size_t lds = std::max(static_cast<size_t>(rc ? 1 : 2) * max_per_class * kKldLdsStride * sizeof(float),
                              static_cast<size_t>(kKldThreads) * 16 * sizeof(float));
  const int st = by_label(label_dtype, [&](auto tl) {
    using TL = std::remove_pointer_t<decltype(tl)>;
    auto go = [&](auto kern) {
      if (int e = ensure_lds<decltype(kern)::value, kKldMaxDynLds>()) return e;
      hipLaunchKernelGGL(decltype(kern)::value, dim3(K, B, S), dim3(kKldThreads), lds, s, dist, P, HW,
                         static_cast<const TL*>(label), K, max_per_class, proto_class, w.off, w.idx, w.slot, w.part,
                         w.rcnt, w.plist);
      return check_launch("kld_partial_kernel");
    };
    return rc ? go(KernelTag<kld_partial_kernel<TL, true>>()) : go(KernelTag<kld_partial_kernel<TL, false>>());
  });
  if (st) return st;
  hipLaunchKernelGGL(kld_merge_kernel, dim3(K, B), dim3(256), 0, s, P, K, S, max_per_class, w.off, w.idx, w.part, w.cnt,
                     w.lse, w.kl, w.group);
  if (int e = check_launch("kld_merge_kernel")) return e;
  hipLaunchKernelGGL(kld_finalize_kernel, dim3(1), dim3(256), 0, s, B * K, w.group, w.off, K, max_per_class, w.stat,
                     loss_out, npairs_out);
  return check_launch("kld_finalize_kernel");
}

extern "C" size_t protoseg_kld_coef_bytes(int B, int K) {
  return B > 0 && K > 0 ? static_cast<size_t>(B) * K * kKldCoefFloats * sizeof(float) : 0;
}

extern "C" int protoseg_kld_backward(const float* dist, int B, int P, int HW, const void* label, int label_dtype,
                                     const int32_t* proto_class, int K, int max_per_class, const float* g_loss,
                                     void* workspace, size_t workspace_bytes, float* g_dist,
                                     protoseg_stream_t stream) {
  // the range partials are dead after the forward: their space holds the backward coefficients
  return protoseg_kld_backward_ex(dist, B, P, HW, label, label_dtype, proto_class, K, max_per_class, g_loss, workspace,
                                  workspace_bytes, nullptr, 0, g_dist, stream);
}

extern "C" int protoseg_kld_backward_ex(const float* dist, int B, int P, int HW, const void* label, int label_dtype,
                                        const int32_t* proto_class, int K, int max_per_class, const float* g_loss,
                                        const void* workspace, size_t workspace_bytes, float* coef_buf,
                                        size_t coef_bytes, float* g_dist, protoseg_stream_t stream) {
  if (int st = kld_check(dist, B, P, HW, label, label_dtype, proto_class, K, max_per_class, workspace, workspace_bytes))
    return st;
  if (!g_dist) return fail(PROTOSEG_ERR_INVALID, "g_dist must be non-null");
  if (coef_buf && coef_bytes < protoseg_kld_coef_bytes(B, K))
    return fail(PROTOSEG_ERR_INVALID, "coef_bytes %zu < protoseg_kld_coef_bytes %zu", coef_bytes,
                protoseg_kld_coef_bytes(B, K));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const KldLayout l = kld_layout(B, P, HW, K);
  const KldPtrs w = kld_ptrs(const_cast<void*>(workspace), l);
  float* coef = coef_buf ? coef_buf : w.part;
  hipLaunchKernelGGL(kld_coef_kernel, dim3(K, B), dim3(64), 0, s, K, max_per_class, w.off, w.cnt, w.kl, w.stat, g_loss,
                     coef);
  if (int st = check_launch("kld_coef_kernel")) return st;
  const size_t lds = static_cast<size_t>(3) * max_per_class * kKldLdsStride * sizeof(float);
  const dim3 grid(static_cast<unsigned>(ceil_div(HW, kKldThreads)), B);
  return by_label(label_dtype, [&](auto tl) {
    using TL = std::remove_pointer_t<decltype(tl)>;
    if (int e = ensure_lds<kld_grad_kernel<TL>, kKldMaxDynLds / 2 * 3>()) return e;
    hipLaunchKernelGGL(kld_grad_kernel<TL>, grid, dim3(kKldThreads), lds, s, dist, P, HW,
                       static_cast<const TL*>(label), K, max_per_class, w.off, w.idx, w.cnt, w.lse, coef, w.stat,
                       g_dist);
    return check_launch("kld_grad_kernel");
  });
}

extern "C" int protoseg_kld_backward_compact(const float* dist, int B, int P, int HW, const void* label,
                                             int label_dtype, const int32_t* proto_class, int K, int max_per_class,
                                             const float* g_loss, void* workspace, size_t workspace_bytes,
                                             float* g_cls, int32_t* pix_cls, int32_t* proto_slot,
                                             protoseg_stream_t stream) {
  if (int st = kld_check(dist, B, P, HW, label, label_dtype, proto_class, K, max_per_class, workspace, workspace_bytes))
    return st;
  if (!g_cls || !pix_cls || !proto_slot) return fail(PROTOSEG_ERR_INVALID, "g_cls, pix_cls and proto_slot must be non-null");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const KldLayout l = kld_layout(B, P, HW, K);
  const KldPtrs w = kld_ptrs(workspace, l);
  // one launch: proto_slot, pix_cls, the coefficients and the gradient (kld_grad_compact_kernel)
  const bool rc = kld_recompute(max_per_class);
  const size_t lds =
      (static_cast<size_t>(rc ? 1 : 2) * max_per_class * kKldLdsStride + kKldCoefFloats) * sizeof(float);
  return by_label(label_dtype, [&](auto tl) {
    using TL = std::remove_pointer_t<decltype(tl)>;
    auto go = [&](auto kern) {
      if (int e = ensure_lds<decltype(kern)::value, kKldMaxDynLds + kKldCoefFloats * sizeof(float)>()) return e;
      hipLaunchKernelGGL(decltype(kern)::value, dim3(K, B, kld_ranges(HW)), dim3(kKldThreads), lds, s, dist, P, HW,
                         static_cast<const TL*>(label), K, max_per_class, w.off, w.idx, w.slot, w.cnt, w.lse, w.kl,
                         w.stat, g_loss, w.rcnt, w.plist, g_cls, pix_cls, proto_slot);
      return check_launch("kld_grad_compact_kernel");
    };
    return rc ? go(KernelTag<kld_grad_compact_kernel<TL, true>>()) : go(KernelTag<kld_grad_compact_kernel<TL, false>>());
  });
}

extern "C" int protoseg_kld_expand(const float* g_cls, const int32_t* pix_cls, const int32_t* proto_slot, int B, int P,
                                   int HW, int max_per_class, int accumulate, float* g_dist, protoseg_stream_t stream) {
  if (!g_cls || !pix_cls || !proto_slot || !g_dist) return fail(PROTOSEG_ERR_INVALID, "null pointer argument");
  if (B <= 0 || P <= 0 || HW <= 0 || max_per_class < 1 || max_per_class > kKldMaxPerClass)
    return fail(PROTOSEG_ERR_INVALID, "bad shape B=%d P=%d HW=%d max_per_class=%d", B, P, HW, max_per_class);
  if (P > 65535) return fail(PROTOSEG_ERR_UNSUPPORTED, "P=%d > 65535", P);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(kld_expand_kernel, dim3(static_cast<unsigned>(ceil_div(HW, 256)), P, B), dim3(256), 0, s, g_cls,
                     pix_cls, proto_slot, P, HW, max_per_class, accumulate, g_dist);
  return check_launch("kld_expand_kernel");
}

#ifdef PROTOSEG_STAMPS
// Debug builds: copy (and with dst = null, clear) the KLD partial kernel's stamps.
extern "C" int protoseg_debug_stamps_kld(void* dst, size_t bytes) {
  using protoseg::g_stamps_kld;
  const size_t n = bytes < sizeof(g_stamps_kld) ? bytes : sizeof(g_stamps_kld);
  if (dst) return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_stamps_kld), n, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 3;
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_stamps_kld)) != hipSuccess) return 3;
  return hipMemset(p, 0, sizeof(g_stamps_kld)) == hipSuccess ? 0 : 3;
}
#endif
