// l2_wide.hip — the prototype layer for any prototype depth C and any class count K: the shapes
// the C in {32, 64, 128}, K <= 32 families do not hold in registers / LDS. That includes the
// reference's own construct_PPNet default, prototype_shape = (2000, 512, 1, 1) with 200 classes
// (model.py:394), and the DenseNet-161 add-on depths of BASELINE configs[4].
//
// Products in one of two modes, composed as strided GEMMs whose epilogues carry the layer's
// elementwise math: exact f32 (v_mfma_f32_32x32x2_f32: a k-ordered fma chain per output element;
// precision F32 / BF16X6, and push), or bf16x3 (precision BF16X3: each operand split into bf16
// hi + lo terms as it is staged, 3 v_mfma_f32_32x32x16_bf16 per 16-k step, f32 accumulation: the
// C = 64 family's arithmetic, 5.3x the f32 MFMA rate). Reference model.py:
//   forward   D[b]      = relu(x2 + p2 - 2 P X[b])                   M = P,  N = HW, K = C  (203-221)
//             logits[b] = act(D[b])^T W^T  (act applied on the load)  M = HW, N = K,  K = P  (231-237, 266-278)
//   backward (autograd of the same; D recomputed from x, never stored by the forward)
//             G_s[b]    = (W^T GL[b]^T) act'(D) + g_dist, masked by D > 0             M = P, N = HW, K = K
//             g_x[b]    = -2 P^T G_s[b] + 2 x sum_p G_s[b]                            M = C, N = HW, K = P
//             g_P       = -2 sum_b G_s[b] X[b]^T + 2 p sum_{b,n} G_s                   M = P, N = C,  K = B HW
//             g_W       = sum_b GL[b]^T act(D[b])^T                                    M = K, N = P,  K = B HW
// The two contractions over pixels (g_P, g_W) are split over workgroups (partial slabs summed in
// a fixed order: deterministic, no atomics). Every operand is addressed by (row, k, batch) strides,
// so no tensor is transposed or copied; NCHW rows give coalesced loads and stores along pixels.
#include "bf16_split.h"
#include "l2_bf16_common.h"
#include "protoseg_device.h"
#include "protoseg_host.h"
#include "l2_launch.h"

#include <map>
#include <type_traits>
#include <mutex>
#include <utility>
#include <vector>

namespace protoseg {

namespace {

constexpr int kWT = 64;        // workgroup output tile (rows and columns)
constexpr int kWKs = 32;       // contraction per LDS stage
constexpr int kWThreads = 256;

// the pre-split backward GEMMs' tile (wide_pre_gemm_kernel, below): 64 MI rows (MI = 3 or 4
// 32-row blocks per wave) x 128 columns x 32 k per stage, three stages
constexpr int kPreTN = 128, kPreTK = 32, kPreNS = 3;
constexpr int kColsumQ = 8;  // prototype chunks of the split g_x's column sums (wide_colsum_kernel)
constexpr int kPreBPlane = kPreTN * kPreTK * 2;                                  // 8 KiB
__host__ __device__ constexpr int pre_tm(int MI) { return 64 * MI; }
__host__ __device__ constexpr int pre_aplane(int MI) { return pre_tm(MI) * kPreTK * 2; }  // 12 / 16 KiB
__host__ __device__ constexpr int pre_stage(int MI) { return 2 * pre_aplane(MI) + 2 * kPreBPlane; }
__host__ __device__ constexpr int pre_lds(int MI) { return kPreNS * pre_stage(MI) + 16 * kPreTN * 4; }

enum WideEpi { kEpiStore = 0, kEpiDist = 1, kEpiGs = 2, kEpiGx = 3, kEpiGsSplit = 4 };

// bf16x3 stages: per operand, hi and lo terms as [row][k] bf16 rows of kWKs k, padded to kBRow
// elements (80-B rows: the 16-row groups of a ds_read_b128 fragment read land on distinct banks)
constexpr int kBRow = kWKs + 8;
constexpr int kBTile = kWT * kBRow;  // elements of one term of one 64-row operand stage

// Element (r, k) of batch b at p[b * sb + r * sr + k * sk]; r is the output row (A) or column (B).
// Every operand of the layer's GEMMs is a row- or column-major view of an NCHW / [P, C] / [K, P]
// tensor, so sr == 1 ("rows fast") or sk == 1 ("k fast"); element offsets are below 2^31
// (wide_family_fits), so addresses are 32-bit offsets from the operand's base.
struct Operand {
  const void* p;
  unsigned sr, sk, sb;
};

struct WideArgs {
  Operand A, B;
  int M, N, Kd, nb;  // per-batch contraction Kd; nb batches
  int bk;            // 1: the contraction runs over (batch, k) flattened, split over blockIdx.z
  int ksplit;        // workgroups along the contraction (bk: z = split; else z = b * ksplit + split)
  void* out;         // element (m, n) of output slab z at out[z * ob + m * om + n * on]
  long long om, on, ob;
  int accumulate;
  float eps;
  int act_kind;
  float* act;        // kEpiDist: optional activation output at act[b * ab + m * am + n * an]
  long long am, an, ab;
  const float* D;    // kEpiGs: the distance at the output's address
  const float* gd;   // kEpiGs: dense g_dist at the output's address, or null
  const void* xo;    // kEpiGx: x at the output's address
  int bf3;           // 1: bf16x3 products (precision BF16X3), 0: exact f32 MFMA
  void* out2;        // kEpiGsSplit: G_s as two bf16 planes, hi at out, lo at out2 (same offsets)
};

template <typename T>
__device__ __forceinline__ float load_elem(const void* p, long long i) {
  return XIO<T>::load(static_cast<const T*>(p), static_cast<size_t>(i));
}

// ACT < 0: the value as stored; else the activation of a distance (model.py:231-237).
template <int ACT>
__device__ __forceinline__ float on_load(float v, float eps) {
  if constexpr (ACT < 0) return v;
  else return activation(v, eps, ACT);
}

// One operand's share of a ROWS-row x 32-k stage (ROWS = 64 or 128): ROWS / 8 elements per thread.
//   MODE 0 (rows fast): row t % ROWS, k = (t / ROWS) ROWS / 8 + i — ROWS consecutive rows per k,
//                       coalesced, and each thread's k consecutive (one 16-B bf16 row piece);
//   MODE 1 (k fast):    k = t & 31, row (t >> 5) + 8i — 32 consecutive k per row, coalesced.
// The element's row (and, MODE 0, k) offset is fixed for the whole contraction; the stage moves
// a uniform base (non-bk) or, for a k-fast operand over the flattened (batch, pixel) contraction,
// one per-thread (batch, k) position advanced by 32 per stage (no division in the loop).
template <typename T, int ACT, int MODE, int ROWS>
struct Stager {
  static constexpr int kE = ROWS / 8;
  static constexpr int kLd = ROWS + 1;  // LDS row pitch (odd: k-fast stores spread over the banks)
  const T* p;
  unsigned fix[kE];
  unsigned rok;  // bit i: element i's row is inside the operand
  int kt;        // MODE 1: this thread's k in the stage
  int bb, kin;   // MODE 1, bk: batch and in-batch k of this thread's current contraction index
  unsigned sb;

  __device__ __forceinline__ static int row_of_e(int t, int i) { return MODE == 0 ? (t % ROWS) : (t >> 5) + 8 * i; }
  __device__ __forceinline__ static int k_of_e(int t, int i) { return MODE == 0 ? (t / ROWS) * kE + i : (t & 31); }

  __device__ __forceinline__ void init(const Operand& o, int R, int r0, int kbeg, int Kd, int bk) {
    p = static_cast<const T*>(o.p);
    const int t = threadIdx.x;
    rok = 0;
    sb = o.sb;
#pragma unroll
    for (int i = 0; i < kE; ++i) {
      const int r = row_of_e(t, i), k = k_of_e(t, i);
      const bool ok = r0 + r < R;
      rok |= ok ? (1u << i) : 0u;
      fix[i] = ok ? (MODE == 0 ? static_cast<unsigned>(r0 + r) + static_cast<unsigned>(k) * o.sk
                               : static_cast<unsigned>(r0 + r) * o.sr)
                  : 0u;
    }
    kt = t & 31;
    if (MODE == 1 && bk) {
      const int kk = kbeg + kt;  // flattened index of this thread's first element
      bb = kk / Kd;
      kin = kk - bb * Kd;
    }
  }
  // Stage at contraction base kb (flattened for bk); lim = kend - kb; base = the stage's uniform
  // offset. Raw values: the zeroing of elements outside the operand (okm) and the activation
  // happen in store(), after the MFMAs the loads are in flight under.
  __device__ __forceinline__ void load(unsigned base, int lim, int bk, float (&v)[kE], unsigned& okm) const {
    const unsigned kofs = MODE == 1 ? (bk ? static_cast<unsigned>(bb) * sb + static_cast<unsigned>(kin)
                                          : static_cast<unsigned>(kt))
                                    : 0u;
    okm = 0;
#pragma unroll
    for (int i = 0; i < kE; ++i) {
      const int k = k_of_e(static_cast<int>(threadIdx.x), i);
      const bool ok = ((rok >> i) & 1u) && k < lim;
      okm |= ok ? (1u << i) : 0u;
      // branch-free: an element outside the operand loads element 0 (zeroed in store())
      v[i] = XIO<T>::load(p, static_cast<size_t>(ok ? base + fix[i] + kofs : 0u));
    }
  }
  __device__ __forceinline__ void advance(int Kd) {  // MODE 1, bk: the next stage's (batch, k)
    kin += kWKs;
    while (kin >= Kd) {
      kin -= Kd;
      ++bb;
    }
  }
  // F32S: the f32 [k][row] stage (the f32 MFMAs' operand, and the epilogue sums' source);
  // Bh (bf16x3): hi / lo terms into the [row][k] stage at Bh, Bh + bt (bt: elements per term).
  template <bool F32S = true>
  __device__ __forceinline__ void store(float* S, const float (&v)[kE], unsigned okm, float eps, bf16* Bh = nullptr,
                                        int bt = kBTile) const {
    const int t = threadIdx.x;
    float xs[kE];
#pragma unroll
    for (int i = 0; i < kE; ++i) {
      xs[i] = ((okm >> i) & 1u) ? on_load<ACT>(v[i], eps) : 0.f;
      if constexpr (F32S) S[k_of_e(t, i) * kLd + row_of_e(t, i)] = xs[i];
    }
    if (!Bh) return;
    if constexpr (MODE == 0) {  // the thread's kE consecutive k of one row: 16-B writes of 8
#pragma unroll
      for (int g = 0; g < kE / 8; ++g) {
        float x8[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) x8[i] = xs[8 * g + i];
        bf16x8 f[2];
        split8<2>(x8, f);
        const int o = row_of_e(t, 0) * kBRow + k_of_e(t, 8 * g);
        *reinterpret_cast<bf16x8*>(Bh + o) = f[0];
        *reinterpret_cast<bf16x8*>(Bh + o + bt) = f[1];
      }
    } else {
#pragma unroll
      for (int i = 0; i < kE; ++i) {
        bf16 tm[2];
        split_terms<2>(xs[i], tm);
        const int o = row_of_e(t, i) * kBRow + k_of_e(t, i);
        Bh[o] = tm[0];
        Bh[o + bt] = tm[1];
      }
    }
  }
};

// Uniform offset of a stage at contraction base kb: batch b (non-bk) or flattened (bk, MODE 0:
// affine, sb == Kd * sk); MODE 1 bk carries its position per thread.
template <int MODE>
__device__ __forceinline__ unsigned stage_base(const Operand& o, int b, int kb, int bk) {
  if (bk) return MODE == 0 ? static_cast<unsigned>(kb) * o.sk : 0u;
  return static_cast<unsigned>(b) * o.sb + static_cast<unsigned>(kb) * (MODE == 0 ? o.sk : 1u);
}

// C[z] (TM x 64 tile, TM = 64 or 128 rows) = A (M x Kd) B^T (N x Kd) over 32-k stages,
// double-buffered in LDS (one barrier per stage, the next stage's global loads in flight under
// this stage's MFMAs), v_mfma_f32_32x32x2_f32: exact f32 fma chains in k order. TM = 64: each of
// the 4 waves one 32 x 32 block; TM = 128 (M >= 256): each wave a 32-row strip of two blocks,
// which halves the B-operand traffic per product and reads each A fragment once for two MFMAs.
// The epilogues' per-column / per-row sums come from the same LDS stages (a non-split workgroup
// contracts over the whole Kd of its batch): kEpiDist: x2[n] = sum_c X[c][n]^2 (B columns) and
// p2[m] = sum_c P[m][c]^2 (A rows); kEpiGx: cs[n] = sum_p G_s[p][n] (B columns). Thread t sums one
// column (row) over a fixed slice of the stage's k rows; the slices' partials are added in a fixed
// order: deterministic, the same bits in every workgroup of a column, no separate norms pass.
template <int EPI, typename TA, typename TB, int AACT, int BACT, typename TO, int MA, int MB, int TM, bool BF>
__global__ __launch_bounds__(kWThreads) void wide_gemm_kernel(WideArgs a) {
  constexpr int kLdA = TM + 1, kLdB = kWT + 1;
  constexpr int kNC = TM == 128 ? 2 : 1;  // 32-column blocks per wave
  constexpr int kQA = kWThreads / TM;     // k slices of the A-row sums
  constexpr bool kSumB = EPI == kEpiDist || EPI == kEpiGx, kSumA = EPI == kEpiDist, kSq = EPI == kEpiDist;
  static_assert(!BF || TM == 64, "bf16x3 stages: 64-row tiles");
  // f32 stages: the f32 MFMAs' operands; in bf16x3 mode only where the epilogue sums read them
  constexpr bool kFA = !BF || kSumA, kFB = !BF || kSumB;
  __shared__ float As[2][kFA ? kWKs * kLdA : 1];
  __shared__ float Bs[2][kFB ? kWKs * kLdB : 1];
  __shared__ __attribute__((aligned(16))) bf16 Bh[BF ? 2 : 1][2][BF ? 2 * kBTile : 8];  // [buffer][A | B][hi | lo rows]
  __shared__ float redB[kSumB ? 4 : 1][64];
  __shared__ float redA[kSumA ? kQA : 1][kSumA ? TM : 1];
  float sum_b = 0.f, sum_a = 0.f;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = lane & 31, h = lane >> 5;
  const int wm = TM == 128 ? wave : (wave & 1), wn0 = TM == 128 ? 0 : (wave >> 1);
  const int m0 = blockIdx.y * TM, n0 = blockIdx.x * kWT, z = blockIdx.z;
  // contraction range of this workgroup (flattened (batch, k) units for bk), whole stages
  const int split = a.bk ? z : z % a.ksplit, bsel = a.bk ? 0 : z / a.ksplit;
  const long long total = a.bk ? static_cast<long long>(a.nb) * a.Kd : a.Kd;
  const long long chunks = (total + kWKs - 1) / kWKs;
  const int kbeg = static_cast<int>((chunks * split / a.ksplit) * kWKs);
  int kend = static_cast<int>((chunks * (split + 1) / a.ksplit) * kWKs);
  if (kend > total) kend = static_cast<int>(total);
  Stager<TA, AACT, MA, TM> sa;
  Stager<TB, BACT, MB, kWT> sb;
  sa.init(a.A, a.M, m0, kbeg, a.Kd, a.bk);
  sb.init(a.B, a.N, n0, kbeg, a.Kd, a.bk);
  f32x16 acc[kNC];
#pragma unroll
  for (int c = 0; c < kNC; ++c) acc[c] = zero16();
  float va[TM / 8], vb[kWT / 8];
  unsigned oka = 0, okb = 0;
  const int nst = kend > kbeg ? (kend - kbeg + kWKs - 1) / kWKs : 0;
  if (nst > 0) {
    sa.load(stage_base<MA>(a.A, bsel, kbeg, a.bk), kend - kbeg, a.bk, va, oka);
    sb.load(stage_base<MB>(a.B, bsel, kbeg, a.bk), kend - kbeg, a.bk, vb, okb);
    sa.template store<kFA>(As[0], va, oka, a.eps, BF ? Bh[0][0] : nullptr);
    sb.template store<kFB>(Bs[0], vb, okb, a.eps, BF ? Bh[0][1] : nullptr);
    __syncthreads();
  }
  // (two stages of loads in flight measured 1-3 % slower at the 4-waves-per-SIMD register cap
  // they need: DESIGN 5.4)
  for (int st = 0; st < nst; ++st) {
    const int cur = st & 1;
    const bool more = st + 1 < nst;
    if (more) {  // the next stage's loads, in flight under this stage's MFMAs
      const int kb = kbeg + (st + 1) * kWKs;
      if (MA == 1 && a.bk) sa.advance(a.Kd);
      if (MB == 1 && a.bk) sb.advance(a.Kd);
      sa.load(stage_base<MA>(a.A, bsel, kb, a.bk), kend - kb, a.bk, va, oka);
      sb.load(stage_base<MB>(a.B, bsel, kb, a.bk), kend - kb, a.bk, vb, okb);
    }
    const float* Ac = As[cur];
    const float* Bc = Bs[cur];
    if constexpr (BF) {  // two 16-k steps: hi / lo fragments of row j, k 16 kk + 8 h .. + 7
      const bf16* Ab = Bh[cur][0] + (wm * 32 + j) * kBRow + 8 * h;
      const bf16* Bb = Bh[cur][1] + (wn0 * 32 + j) * kBRow + 8 * h;
#pragma unroll
      for (int kk = 0; kk < kWKs / 16; ++kk) {
        const bf16x8 af[2] = {*reinterpret_cast<const bf16x8*>(Ab + 16 * kk),
                              *reinterpret_cast<const bf16x8*>(Ab + 16 * kk + kBTile)};
        const bf16x8 bfr[2] = {*reinterpret_cast<const bf16x8*>(Bb + 16 * kk),
                               *reinterpret_cast<const bf16x8*>(Bb + 16 * kk + kBTile)};
        acc[0] = mma_split<2>(af, bfr, acc[0]);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < kWKs / 2; ++kk) {
        const float av = Ac[(2 * kk + h) * kLdA + wm * 32 + j];
#pragma unroll
        for (int c = 0; c < kNC; ++c) acc[c] = mfma32(av, Bc[(2 * kk + h) * kLdB + (wn0 + c) * 32 + j], acc[c]);
      }
    }
    if constexpr (kSumB) {
      const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float vbv = Bc[(8 * q + i) * kLdB + c];
        sum_b = kSq ? fmaf(vbv, vbv, sum_b) : sum_b + vbv;
      }
    }
    if constexpr (kSumA) {
      const int r = threadIdx.x % TM, q = threadIdx.x / TM;
#pragma unroll
      for (int i = 0; i < kWKs / kQA; ++i) {
        const float vav = Ac[((kWKs / kQA) * q + i) * kLdA + r];
        sum_a = fmaf(vav, vav, sum_a);
      }
    }
    if (more) {
      sa.template store<kFA>(As[cur ^ 1], va, oka, a.eps, BF ? Bh[cur ^ 1][0] : nullptr);
      sb.template store<kFB>(Bs[cur ^ 1], vb, okb, a.eps, BF ? Bh[cur ^ 1][1] : nullptr);
    }
    __syncthreads();
  }
  if constexpr (kSumB) redB[threadIdx.x >> 6][threadIdx.x & 63] = sum_b;
  if constexpr (kSumA) redA[threadIdx.x / TM][threadIdx.x % TM] = sum_a;
  if constexpr (kSumB) __syncthreads();

  // epilogue: lane column n, rows acc_row(r, h)
  const int bo = a.bk ? z : (a.ksplit > 1 ? z : bsel);  // output batch (or split slab) index
#pragma unroll
  for (int c = 0; c < kNC; ++c) {
    const int cn = (wn0 + c) * 32 + j;
    const int n = n0 + cn;
    if (n >= a.N) continue;
    float colsum = 0.f;
    if constexpr (kSumB) colsum = (redB[0][cn] + redB[1][cn]) + (redB[2][cn] + redB[3][cn]);
    // The element loads of the 16 rows (D, g_dist, x, the accumulated output) go out as one
    // batch before any store: through plain pointers the compiler must assume a store may alias
    // the next row's load, and interleaved they cost one round trip per row. Rows past M load
    // through row M - 1 (a valid address) and are not stored.
    constexpr bool kLd = EPI == kEpiGs || EPI == kEpiGsSplit || EPI == kEpiGx;
    float ld0[16], ld1[16], ldo[16];
    const bool acc_out = a.accumulate != 0;
    if constexpr (kLd) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mc = min(m0 + wm * 32 + acc_row(r, h), a.M - 1);
        const long long oc = bo * a.ob + mc * a.om + static_cast<long long>(n) * a.on;
        if constexpr (EPI == kEpiGx) {
          ld0[r] = load_elem<TO>(a.xo, oc);
        } else {
          ld0[r] = a.D[oc];
          ld1[r] = a.gd ? a.gd[oc] : 0.f;
        }
      }
      pin_batch(ld0);
      if constexpr (EPI != kEpiGx) pin_batch(ld1);
    }
    if (acc_out) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mc = min(m0 + wm * 32 + acc_row(r, h), a.M - 1);
        ldo[r] = XIO<TO>::load(static_cast<TO*>(a.out), static_cast<size_t>(bo * a.ob + mc * a.om + static_cast<long long>(n) * a.on));
      }
      pin_batch(ldo);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rm = wm * 32 + acc_row(r, h);
      const int m = m0 + rm;
      if (m >= a.M) continue;
      const long long o = bo * a.ob + m * a.om + static_cast<long long>(n) * a.on;
      float v = acc[c][r];
      if constexpr (EPI == kEpiDist) {
        float p2;
        if constexpr (kQA == 4) p2 = (redA[0][rm] + redA[1][rm]) + (redA[2][rm] + redA[3][rm]);
        else p2 = redA[0][rm] + redA[1][rm];
        const float d = l2_distance(colsum, p2, v);
        v = d;
        if (a.act) a.act[bo * a.ab + m * a.am + static_cast<long long>(n) * a.an] = activation(d, a.eps, a.act_kind);
      } else if constexpr (EPI == kEpiGs || EPI == kEpiGsSplit) {
        const float d = ld0[r];
        float g = v * activation_grad(d, a.eps, a.act_kind);
        if (a.gd) g += ld1[r];
        v = d > 0.f ? g : 0.f;  // relu backward
        if constexpr (EPI == kEpiGsSplit) {  // the pre-split GEMMs' operand: hi, lo planes
          const bf16 vh = static_cast<bf16>(v);
          static_cast<uint16_t*>(a.out)[o] = __builtin_bit_cast(uint16_t, vh);
          static_cast<uint16_t*>(a.out2)[o] = __builtin_bit_cast(uint16_t, static_cast<bf16>(v - static_cast<float>(vh)));
          continue;
        }
      } else if constexpr (EPI == kEpiGx) {
        // conv(x^2, ones) backward: 2x sum_p g_s; conv(x, P) backward: -2 P^T g_s
        v = -2.f * v + 2.f * ld0[r] * colsum;
      }
      TO* out = static_cast<TO*>(a.out);
      if (acc_out) v += ldo[r];
      XIO<TO>::store(out, static_cast<size_t>(o), v);
    }
  }
}

// rs[p] = sum_{b, n} G_s[b][p][n]: one workgroup per prototype, fixed-order tree.
__global__ __launch_bounds__(256) void wide_rowsum_kernel(const float* __restrict__ gs, int P, int HW, int B,
                                                          float* __restrict__ rs) {
  __shared__ float red[256];
  const int p = blockIdx.x;
  // thread t takes the (image, pixel) pairs t, t + 256, ... of the row's B * HW values, 8 loads
  // in flight (clamped addresses, pin_batch); small maps (7 x 7) keep every thread busy
  float s = 0.f;
  const int tot = B * HW;
  for (int i0 = static_cast<int>(threadIdx.x); i0 < tot; i0 += 8 * 256) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + 256 * u < tot ? i0 + 256 * u : tot - 1;
      const int b = i / HW;
      v[u] = gs[(static_cast<size_t>(b) * P + p) * HW + (i - b * HW)];
    }
    pin_batch(v);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (i0 + 256 * u < tot) s += v[u];
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (static_cast<int>(threadIdx.x) < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) rs[p] = red[0];
}

// Split-K partial slabs [nbatch][S][M][N] -> out[b * obatch + m * ldo + n] in slab order;
// kind 1 (g_P): -2 sum + 2 p rs[m].
__global__ __launch_bounds__(256) void wide_finish_kernel(const float* __restrict__ part, int S, int nbatch, int M,
                                                          int N, int kind, const float* __restrict__ protos,
                                                          const float* __restrict__ rs, float* __restrict__ out,
                                                          long long ldo, long long obatch) {
  const long long e = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  const long long mn = static_cast<long long>(M) * N;
  if (e >= mn * nbatch) return;
  const long long b = e / mn, r = e - b * mn;
  const int m = static_cast<int>(r / N), n = static_cast<int>(r - static_cast<long long>(m) * N);
  const float* pp = part + static_cast<size_t>(b) * S * mn + r;
  // slab order kept (the same sum bit for bit), 8 loads in flight (one at a time, a 64-slab
  // finish was a chain of L2 round trips)
  float s = 0.f;
  for (int i0 = 0; i0 < S; i0 += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = i0 + u < S ? pp[static_cast<size_t>(i0 + u) * mn] : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (i0 + u < S) s += v[u];
  }
  if (kind == 1) s = -2.f * s + 2.f * protos[r] * rs[m];
  out[b * obatch + m * ldo + n] = s;
}

// Stager mode of an operand: k fast (1) when a flattened contraction is not affine in its
// index (the (batch, pixel) runs of NCHW tensors), else rows fast (0) where sr == 1.
int stager_mode(const Operand& o, const WideArgs& a) {
  if (a.bk && a.nb > 1 && o.sb != static_cast<unsigned>(a.Kd) * o.sk) return o.sk == 1 ? 1 : -1;
  if (o.sr == 1) return 0;
  return o.sk == 1 ? 1 : -1;
}

#ifndef WIDE_TM128
#define WIDE_TM128 0  // 128-row tiles for M >= 256 (measured slower: DESIGN 5.4)
#endif
// bf16x3 GEMM on 128 x 128 output tiles (BF16X3 requests with M >= 128 and N >= 128): the
// 64 x 64 tile above is bound by its stages (loads, LDS writes, a barrier per 32 k) once bf16x3
// cuts the matrix-core cycles 5.3x, so here each of the 4 waves owns a 64 x 64 quarter (2 x 2
// blocks of 32 x 32): per 32-k stage 24 v_mfma_f32_32x32x16_bf16 per wave against 16 fragment
// reads, and every staged element feeds twice the products. Same stagers (128 rows: 16 elements
// per thread), contraction split, epilogues and operations per output element as
// wide_gemm_kernel; the epilogue sums come from f32 stages in two k slices (their own fixed order).
constexpr int kW2 = 128;
constexpr int kB2Tile = kW2 * kBRow;  // elements of one term of one 128-row operand stage
template <int EPI>
constexpr size_t bf3_lds_bytes() {
  constexpr bool kSumB = EPI == kEpiDist || EPI == kEpiGx, kSumA = EPI == kEpiDist;
  return static_cast<size_t>(2 * 2 * 2 * kB2Tile) * 2 + (kSumA ? 2 * kWKs * (kW2 + 1) * 4 : 0) +
         (kSumB ? 2 * kWKs * (kW2 + 1) * 4 : 0) + 2 * 2 * kW2 * 4;
}
template <int EPI, typename TA, typename TB, int AACT, int BACT, typename TO, int MA, int MB>
__global__ __launch_bounds__(kWThreads) void wide_bf3_kernel(WideArgs a) {
  constexpr int kLd = kW2 + 1;
  constexpr bool kSumB = EPI == kEpiDist || EPI == kEpiGx, kSumA = EPI == kEpiDist, kSq = EPI == kEpiDist;
  constexpr int kQ = kWThreads / kW2;  // 2 k slices of 16 per stage for the row / column sums
  extern __shared__ __attribute__((aligned(16))) unsigned char wsm[];
  bf16* Bh = reinterpret_cast<bf16*>(wsm);  // [buffer][A | B][hi | lo][128][kBRow]
  float* fb = reinterpret_cast<float*>(wsm + static_cast<size_t>(2 * 2 * 2 * kB2Tile) * 2);
  float* As = fb;                                          // [buffer][32][129] (kSumA)
  float* Bs = As + (kSumA ? 2 * kWKs * kLd : 0);           // [buffer][32][129] (kSumB)
  float* redA = Bs + (kSumB ? 2 * kWKs * kLd : 0);         // [kQ][128]
  float* redB = redA + kQ * kW2;                           // [kQ][128]
  auto bh = [&](int buf, int op) __attribute__((always_inline)) { return Bh + (buf * 2 + op) * 2 * kB2Tile; };
  float sum_b = 0.f, sum_a = 0.f;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = lane & 31, h = lane >> 5;
  const int wm = wave & 1, wn = wave >> 1;
  const int m0 = blockIdx.y * kW2, n0 = blockIdx.x * kW2, z = blockIdx.z;
  const int split = a.bk ? z : z % a.ksplit, bsel = a.bk ? 0 : z / a.ksplit;
  const long long total = a.bk ? static_cast<long long>(a.nb) * a.Kd : a.Kd;
  const long long chunks = (total + kWKs - 1) / kWKs;
  const int kbeg = static_cast<int>((chunks * split / a.ksplit) * kWKs);
  int kend = static_cast<int>((chunks * (split + 1) / a.ksplit) * kWKs);
  if (kend > total) kend = static_cast<int>(total);
  Stager<TA, AACT, MA, kW2> sa;
  Stager<TB, BACT, MB, kW2> sb;
  sa.init(a.A, a.M, m0, kbeg, a.Kd, a.bk);
  sb.init(a.B, a.N, n0, kbeg, a.Kd, a.bk);
  f32x16 acc[2][2];
#pragma unroll
  for (int bm = 0; bm < 2; ++bm)
#pragma unroll
    for (int bn = 0; bn < 2; ++bn) acc[bm][bn] = zero16();
  float va[kW2 / 8], vb[kW2 / 8];
  unsigned oka = 0, okb = 0;
  const int nst = kend > kbeg ? (kend - kbeg + kWKs - 1) / kWKs : 0;
  if (nst > 0) {
    sa.load(stage_base<MA>(a.A, bsel, kbeg, a.bk), kend - kbeg, a.bk, va, oka);
    sb.load(stage_base<MB>(a.B, bsel, kbeg, a.bk), kend - kbeg, a.bk, vb, okb);
    sa.template store<kSumA>(As, va, oka, a.eps, bh(0, 0), kB2Tile);
    sb.template store<kSumB>(Bs, vb, okb, a.eps, bh(0, 1), kB2Tile);
    __syncthreads();
  }
  for (int st = 0; st < nst; ++st) {
    const int cur = st & 1;
    const bool more = st + 1 < nst;
    if (more) {  // the next stage's loads, in flight under this stage's MFMAs
      const int kb = kbeg + (st + 1) * kWKs;
      if (MA == 1 && a.bk) sa.advance(a.Kd);
      if (MB == 1 && a.bk) sb.advance(a.Kd);
      sa.load(stage_base<MA>(a.A, bsel, kb, a.bk), kend - kb, a.bk, va, oka);
      sb.load(stage_base<MB>(a.B, bsel, kb, a.bk), kend - kb, a.bk, vb, okb);
    }
    const bf16* A0 = bh(cur, 0) + (wm * 64 + j) * kBRow + 8 * h;
    const bf16* B0 = bh(cur, 1) + (wn * 64 + j) * kBRow + 8 * h;
#pragma unroll
    for (int kk = 0; kk < kWKs / 16; ++kk) {
      bf16x8 af[2][2], bfr[2][2];  // [block][term]
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int tm = 0; tm < 2; ++tm) {
          af[q][tm] = *reinterpret_cast<const bf16x8*>(A0 + q * 32 * kBRow + 16 * kk + tm * kB2Tile);
          bfr[q][tm] = *reinterpret_cast<const bf16x8*>(B0 + q * 32 * kBRow + 16 * kk + tm * kB2Tile);
        }
#pragma unroll
      for (int bm = 0; bm < 2; ++bm)
#pragma unroll
        for (int bn = 0; bn < 2; ++bn) acc[bm][bn] = mma_split<2>(af[bm], bfr[bn], acc[bm][bn]);
    }
    if constexpr (kSumB) {
      const float* Bc = Bs + cur * kWKs * kLd;
      const int c = threadIdx.x % kW2, q = threadIdx.x / kW2;
#pragma unroll
      for (int i = 0; i < kWKs / kQ; ++i) {
        const float vbv = Bc[((kWKs / kQ) * q + i) * kLd + c];
        sum_b = kSq ? fmaf(vbv, vbv, sum_b) : sum_b + vbv;
      }
    }
    if constexpr (kSumA) {
      const float* Ac = As + cur * kWKs * kLd;
      const int r = threadIdx.x % kW2, q = threadIdx.x / kW2;
#pragma unroll
      for (int i = 0; i < kWKs / kQ; ++i) {
        const float vav = Ac[((kWKs / kQ) * q + i) * kLd + r];
        sum_a = fmaf(vav, vav, sum_a);
      }
    }
    if (more) {
      sa.template store<kSumA>(As + (cur ^ 1) * kWKs * kLd, va, oka, a.eps, bh(cur ^ 1, 0), kB2Tile);
      sb.template store<kSumB>(Bs + (cur ^ 1) * kWKs * kLd, vb, okb, a.eps, bh(cur ^ 1, 1), kB2Tile);
    }
    __syncthreads();
  }
  if constexpr (kSumB) redB[(threadIdx.x / kW2) * kW2 + threadIdx.x % kW2] = sum_b;
  if constexpr (kSumA) redA[(threadIdx.x / kW2) * kW2 + threadIdx.x % kW2] = sum_a;
  if constexpr (kSumA || kSumB) __syncthreads();

  const int bo = a.bk ? z : (a.ksplit > 1 ? z : bsel);  // output batch (or split slab) index
#pragma unroll
  for (int bn = 0; bn < 2; ++bn) {
    const int cn = wn * 64 + bn * 32 + j;
    const int n = n0 + cn;
    if (n >= a.N) continue;
    float colsum = 0.f;
    if constexpr (kSumB) colsum = redB[cn] + redB[kW2 + cn];
#pragma unroll
    for (int bm = 0; bm < 2; ++bm) {
      // the rows' element loads as one batch before the stores (wide_bf3 / wide_gemm bf16x3
      // epilogue: a load behind a possibly aliasing store waits a round trip)
      constexpr bool kLd = EPI == kEpiGs || EPI == kEpiGsSplit || EPI == kEpiGx;
      float ld0[16], ld1[16], ldo[16];
      const bool acc_out = a.accumulate != 0;
      if constexpr (kLd) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int mc = min(m0 + wm * 64 + bm * 32 + acc_row(r, h), a.M - 1);
          const long long oc = bo * a.ob + mc * a.om + static_cast<long long>(n) * a.on;
          if constexpr (EPI == kEpiGx) {
            ld0[r] = load_elem<TO>(a.xo, oc);
          } else {
            ld0[r] = a.D[oc];
            ld1[r] = a.gd ? a.gd[oc] : 0.f;
          }
        }
        pin_batch(ld0);
        if constexpr (EPI != kEpiGx) pin_batch(ld1);
      }
      if (acc_out) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int mc = min(m0 + wm * 64 + bm * 32 + acc_row(r, h), a.M - 1);
          ldo[r] = XIO<TO>::load(static_cast<TO*>(a.out),
                                 static_cast<size_t>(bo * a.ob + mc * a.om + static_cast<long long>(n) * a.on));
        }
        pin_batch(ldo);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rm = wm * 64 + bm * 32 + acc_row(r, h);
        const int m = m0 + rm;
        if (m >= a.M) continue;
        const long long o = bo * a.ob + m * a.om + static_cast<long long>(n) * a.on;
        float v = acc[bm][bn][r];
        if constexpr (EPI == kEpiDist) {
          const float p2 = redA[rm] + redA[kW2 + rm];
          const float d = l2_distance(colsum, p2, v);
          v = d;
          if (a.act) a.act[bo * a.ab + m * a.am + static_cast<long long>(n) * a.an] = activation(d, a.eps, a.act_kind);
        } else if constexpr (EPI == kEpiGs || EPI == kEpiGsSplit) {
          const float d = ld0[r];
          float g = v * activation_grad(d, a.eps, a.act_kind);
          if (a.gd) g += ld1[r];
          v = d > 0.f ? g : 0.f;  // relu backward
          if constexpr (EPI == kEpiGsSplit) {  // the pre-split GEMMs' operand: hi, lo planes
            const bf16 vh = static_cast<bf16>(v);
            static_cast<uint16_t*>(a.out)[o] = __builtin_bit_cast(uint16_t, vh);
            static_cast<uint16_t*>(a.out2)[o] = __builtin_bit_cast(uint16_t, static_cast<bf16>(v - static_cast<float>(vh)));
            continue;
          }
        } else if constexpr (EPI == kEpiGx) {
          v = -2.f * v + 2.f * ld0[r] * colsum;
        }
        TO* out = static_cast<TO*>(a.out);
        if (acc_out) v += ldo[r];
        XIO<TO>::store(out, static_cast<size_t>(o), v);
      }
    }
  }
}

template <int EPI, typename TA, typename TB, int AACT, int BACT, typename TO, int TM, bool BF>
int gemm_tm(const WideArgs& a, int grid_z, int ma, int mb, hipStream_t s) {
  const dim3 grid(static_cast<unsigned>(ceil_div(a.N, kWT)), static_cast<unsigned>(ceil_div(a.M, TM)),
                  static_cast<unsigned>(grid_z));
  if (ma == 0 && mb == 0)
    hipLaunchKernelGGL((wide_gemm_kernel<EPI, TA, TB, AACT, BACT, TO, 0, 0, TM, BF>), grid, dim3(kWThreads), 0, s, a);
  else if (ma == 0)
    hipLaunchKernelGGL((wide_gemm_kernel<EPI, TA, TB, AACT, BACT, TO, 0, 1, TM, BF>), grid, dim3(kWThreads), 0, s, a);
  else if (mb == 0)
    hipLaunchKernelGGL((wide_gemm_kernel<EPI, TA, TB, AACT, BACT, TO, 1, 0, TM, BF>), grid, dim3(kWThreads), 0, s, a);
  else
    hipLaunchKernelGGL((wide_gemm_kernel<EPI, TA, TB, AACT, BACT, TO, 1, 1, TM, BF>), grid, dim3(kWThreads), 0, s, a);
  return check_launch("wide_gemm_kernel");
}

#ifndef WIDE_BF3_128
#define WIDE_BF3_128 0  // 128 x 128 bf16x3 tiles where M, N >= 128 (measured slower at configs[4]: DESIGN 5.5)
#endif
template <int EPI, typename TA, typename TB, int AACT, int BACT, typename TO>
int gemm_bf3(const WideArgs& a, int grid_z, int ma, int mb, hipStream_t s) {
  const dim3 grid(static_cast<unsigned>(ceil_div(a.N, kW2)), static_cast<unsigned>(ceil_div(a.M, kW2)),
                  static_cast<unsigned>(grid_z));
  constexpr size_t lds = bf3_lds_bytes<EPI>();
  static_assert(lds <= kMaxLds, "bf16x3 128-tile LDS");
  auto go = [&](auto kern) {
    if (int e = ensure_lds<decltype(kern)::value, lds>()) return e;
    hipLaunchKernelGGL(decltype(kern)::value, grid, dim3(kWThreads), lds, s, a);
    return check_launch("wide_bf3_kernel");
  };
  if (ma == 0 && mb == 0) return go(std::integral_constant<decltype(&wide_bf3_kernel<EPI, TA, TB, AACT, BACT, TO, 0, 0>), &wide_bf3_kernel<EPI, TA, TB, AACT, BACT, TO, 0, 0>>());
  if (ma == 0) return go(std::integral_constant<decltype(&wide_bf3_kernel<EPI, TA, TB, AACT, BACT, TO, 0, 1>), &wide_bf3_kernel<EPI, TA, TB, AACT, BACT, TO, 0, 1>>());
  if (mb == 0) return go(std::integral_constant<decltype(&wide_bf3_kernel<EPI, TA, TB, AACT, BACT, TO, 1, 0>), &wide_bf3_kernel<EPI, TA, TB, AACT, BACT, TO, 1, 0>>());
  return go(std::integral_constant<decltype(&wide_bf3_kernel<EPI, TA, TB, AACT, BACT, TO, 1, 1>), &wide_bf3_kernel<EPI, TA, TB, AACT, BACT, TO, 1, 1>>());
}

// grid_z: batches x splits (or the bk splits); a.ksplit 0 means 1. a.bf3: bf16x3 products.
template <int EPI, typename TA, typename TB, int AACT, int BACT, typename TO>
int gemm(WideArgs a, int grid_z, hipStream_t s) {
  if (a.ksplit < 1) a.ksplit = 1;
  const int ma = stager_mode(a.A, a), mb = stager_mode(a.B, a);
  if (ma < 0 || mb < 0) return fail(PROTOSEG_ERR_UNSUPPORTED, "wide GEMM operand with no unit stride");
  if (a.bf3 && WIDE_BF3_128 && a.M >= kW2 && a.N >= kW2) return gemm_bf3<EPI, TA, TB, AACT, BACT, TO>(a, grid_z, ma, mb, s);
  if (a.bf3) return gemm_tm<EPI, TA, TB, AACT, BACT, TO, 64, true>(a, grid_z, ma, mb, s);
  if (WIDE_TM128 && a.M >= 256) return gemm_tm<EPI, TA, TB, AACT, BACT, TO, 128, false>(a, grid_z, ma, mb, s);
  return gemm_tm<EPI, TA, TB, AACT, BACT, TO, 64, false>(a, grid_z, ma, mb, s);
}

// Workgroups along a contraction of `total` for `groups` output tiles (x batches): about 1024
// workgroups in all (four per CU at the kernel's 35 KB of LDS), each at least 4 stages, at most 64.
int split_of(long long groups, long long total) {
  long long s = 1024 / (groups > 0 ? groups : 1);
  const long long cap = ceil_div(total, 4 * kWKs);
  if (s > cap) s = cap;
  if (s > 64) s = 64;
  return static_cast<int>(s < 1 ? 1 : s);
}
int tile_rows(int M) { return WIDE_TM128 && M >= 256 ? 128 : 64; }  // gemm()'s choice
int split_of(int M, int N, long long total) { return split_of(ceil_div(M, tile_rows(M)) * ceil_div(N, kWT), total); }
// The logits GEMM (M = HW, N = K per image): split over the prototypes when the images' tiles
// alone leave the CUs idle.
int logits_split(const Geometry& g) {
  const long long groups = ceil_div(g.HW, tile_rows(g.HW)) * ceil_div(g.K, kWT) * (g.npix / g.HW);
  return groups >= 512 ? 1 : split_of(groups, g.P);
}

// Pre-split backward (wide_pre_gemm_kernel): served for bf16x3 requests whose per-image pixel
// count keeps every 32-pixel k stage inside one image, and whose planes stay below 2^31 bytes.
bool wide_pre_fits(const Geometry& g) {
  const long long big = 1LL << 31;
  return g.HW % 32 == 0 && static_cast<long long>(g.npix) * g.C * 2 < big &&
         static_cast<long long>(g.npix) * g.P * 2 < big && static_cast<long long>(g.C) * (g.P + 32) * 2 < big;
}
// Row blocks per wave of a pre GEMM with M rows and `cols` output tiles along N (times `splits`):
// the one whose grid takes fewer rounds of 256 workgroups, then the one with fewer padded rows.
int pre_mi(long long M, long long cols) {
  const long long t3 = ceil_div(M, pre_tm(3)) * cols, t4 = ceil_div(M, pre_tm(4)) * cols;
  const long long r3 = ceil_div(t3, 256), r4 = ceil_div(t4, 256);
  if (r3 != r4) return r4 < r3 ? 4 : 3;
  return ceil_div(M, pre_tm(4)) * pre_tm(4) < ceil_div(M, pre_tm(3)) * pre_tm(3) ? 4 : 3;
}
int pre_split(const Geometry& g) {  // workgroups along the g_P contraction: at most 256 in all (one round), >= 4 stages each
  const long long tiles = ceil_div(g.P, pre_tm(3)) * ceil_div(g.C, kPreTN);
  long long s2 = 256 / tiles;
  const long long cap = ceil_div(static_cast<long long>(g.npix), 4 * kPreTK);
  if (s2 > cap) s2 = cap;
  return static_cast<int>(s2 < 1 ? 1 : s2 > 64 ? 64 : s2);
}
struct WideBwdLayout {
  size_t D, G, rs, part, xs, pt, cs, total;  // float offsets (G holds f32 G_s, or its two bf16 planes)
};
// Workgroups along the contraction (P) of the 64 x 64 tile's g_x GEMM: split when its output tiles
// alone leave the chip mostly idle (the construct_PPNet default: 7 x 7 maps, 256 tiles of 63
// stages each).
int gx_split(const Geometry& g) {
  const long long groups = ceil_div(g.C, tile_rows(g.C)) * ceil_div(g.HW, kWT) * (g.npix / g.HW);
  return groups >= 512 ? 1 : split_of(groups, g.P);
}
WideBwdLayout wide_bwd_layout(const Geometry& g) {
  WideBwdLayout l{};
  const size_t dp = static_cast<size_t>(g.npix) * g.P;
  size_t sp = static_cast<size_t>(split_of(g.P, g.C, g.npix)) * g.P * g.C;
  const size_t sw = static_cast<size_t>(split_of(g.K, g.P, g.npix)) * g.K * g.P;
  const bool pre = wide_pre_fits(g);
  if (pre) {
    const size_t sq = static_cast<size_t>(pre_split(g)) * g.P * g.C;
    sp = sp > sq ? sp : sq;
  }
  const int sxs = gx_split(g);
  const size_t sx = sxs > 1 ? static_cast<size_t>(sxs) * g.npix * g.C : 0;
  sp = sp > sx ? sp : sx;
  auto al = [](size_t v) { return (v + 63) & ~static_cast<size_t>(63); };
  l.D = 0;
  l.G = al(dp);
  l.rs = l.G + al(dp);
  l.part = l.rs + al(g.P);
  l.xs = l.part + al(sp > sw ? sp : sw);                                  // x as two bf16 planes
  l.pt = l.xs + (pre ? al(static_cast<size_t>(g.npix) * g.C) : 0);       // P^T as two bf16 planes
  l.cs = l.pt + (pre ? al(static_cast<size_t>(g.C) * (ceil_div(g.P, kPreTK) * kPreTK)) : 0);
  l.total = l.cs + (sxs > 1 ? al(static_cast<size_t>(kColsumQ) * g.npix) : 0);  // sum_p G_s partials (split g_x)
  return l;
}

Operand op(const void* p, long long sr, long long sk, long long sb) {
  return Operand{p, static_cast<unsigned>(sr), static_cast<unsigned>(sk), static_cast<unsigned>(sb)};
}

#ifndef WIDE_F16_MFMA
#define WIDE_F16_MFMA 1  // the fp16 distance GEMM below (0: the bf16x3 64 x 64 tile, for A/B)
#endif
// ---- fp16 feature maps (BASELINE configs[4]): the distance GEMM on v_mfma_f32_32x32x16_f16 ----
// x is exact in fp16. Each prototype row p is scaled by a power of two s_p (its largest |value|
// lands in [2^13, 2^14): no fp16 overflow, small values kept normal) and split into two fp16
// terms, p s_p = hi + lo (22 significant bits, |err| <= 2^-22 |p| s_p: finer than bf16x3's
// 3 x 2^-16). Then x.p = (x.hi + x.lo) / s_p: two f16 MFMAs per product instead of bf16x3's
// three, and no operand conversion in the GEMM (the split rows are built once per call by
// wide_f16_prep_kernel, x is read as stored). Epilogue as wide_gemm_kernel's kEpiDist: x2 from
// the staged x (fixed order), p2 exact in f32 from the prep, relu(x2 + p2 - 2 x.p).
// Workgroup: a 192-prototype x 128-pixel tile (4 waves, one per SIMD, each 3 x 2 blocks of
// 32 x 32), K in 32-channel stages, three LDS stages in flight by 16-B LDS-DMA (lane-linear
// pieces, swizzled through the source addresses), one barrier per stage.
constexpr int kF16TM = 192, kF16TN = 128, kF16TK = 32, kF16NS = 3;
constexpr int kF16ATerm = kF16TM * kF16TK * 2;             // one term's A stage [192 rows][64 B]
constexpr int kF16BTile = kF16TK * kF16TN * 2;             // the x stage [32 channels][256 B]
constexpr int kF16Stage = 2 * kF16ATerm + kF16BTile;       // 32 KiB
constexpr int kF16Lds = kF16NS * kF16Stage + 16 * kF16TN * 4 + 2 * kF16TM * 4;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short f16s4 __attribute__((ext_vector_type(4)));

struct F16DistArgs {
  const _Float16* x;      // [B][C][HW]
  unsigned x_bytes;
  const _Float16* ahi;    // [Mpad][Kpad]: scaled hi terms
  const _Float16* alo;    //               scaled lo terms
  unsigned a_bytes;       // bytes of one term
  const float* p2;        // [Mpad]: ||p||^2 (exact f32)
  const float* inv_s;     // [Mpad]: 1 / s_p (a power of two)
  int P, C, Kpad, HW, ntot;
  float* dist;            // [B][P][HW]
  unsigned d_bytes;
  float* act;             // optional [(b HW + n)][P]
  int act_kind;
  float eps;
};

// One wave per prototype row: s_p, the two fp16 terms of p s_p ([Mpad][Kpad], zero padding), ||p||^2.
__global__ __launch_bounds__(256) void wide_f16_prep_kernel(const float* __restrict__ protos, int P, int C, int Mpad,
                                                           int Kpad, _Float16* __restrict__ ahi,
                                                           _Float16* __restrict__ alo, float* __restrict__ p2,
                                                           float* __restrict__ inv_s) {
  const int lane = threadIdx.x & 63, row = static_cast<int>(blockIdx.x) * 4 + static_cast<int>(threadIdx.x >> 6);
  if (row >= Mpad) return;
  const bool valid = row < P;
  const float* pr = protos + static_cast<size_t>(valid ? row : 0) * C;
  float mx = 0.f, sq = 0.f;
  // 8 loads in flight per lane (a plain strided loop waits on each one); the same per-lane
  // summation order as one element at a time
  for (int c0 = 0; c0 < C; c0 += 8 * 64) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int c = c0 + 64 * u + lane;
      v[u] = valid && c < C ? pr[c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      mx = fmaxf(mx, fabsf(v[u]));
      sq = fmaf(v[u], v[u], sq);
    }
  }
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {  // butterfly: every lane ends with the same (fixed-order) sums
    mx = fmaxf(mx, __shfl_xor(mx, m));
    sq += __shfl_xor(sq, m);
  }
  int e = 0;
  (void)frexpf(mx, &e);  // mx < 2^e
  if (!(mx < 3.0e38f) || mx == 0.f) e = 14;  // zero / non-finite rows: s_p = 1
  e = e < -100 ? -100 : e;
  const float scale = ldexpf(1.f, 14 - e), inv = ldexpf(1.f, e - 14);
  _Float16* hr = ahi + static_cast<size_t>(row) * Kpad;
  _Float16* lr = alo + static_cast<size_t>(row) * Kpad;
  for (int k0 = 0; k0 < Kpad; k0 += 8 * 64) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = k0 + 64 * u + lane;
      v[u] = (valid && k < C ? pr[k] : 0.f) * scale;  // exact (power of two)
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = k0 + 64 * u + lane;
      if (k < Kpad) {
        const _Float16 hi = static_cast<_Float16>(v[u]);
        hr[k] = hi;
        lr[k] = static_cast<_Float16>(v[u] - static_cast<float>(hi));  // v - hi exact in f32
      }
    }
  }
  if (lane == 0) {
    p2[row] = valid ? sq : 0.f;
    inv_s[row] = inv;
  }
}

// 16-B LDS-DMA of one wave-instruction (1 KiB, lane-linear at lds + 16 lane); out-of-range
// lanes land as zeros. Inline asm so the compiler does not drain it before unrelated LDS reads
// (the dma<> note in l2_bf16_common.h); the kernel waits for it itself.
__device__ __forceinline__ void dma16(rsrc_t r, unsigned lds, unsigned voff, unsigned soff) {
  unsigned so = __builtin_amdgcn_readfirstlane(soff);
  asm volatile("" : "+s"(so));
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(__builtin_amdgcn_readfirstlane(lds)), "s"(r), "s"(so)
               : "memory");
}

// x stage image: 256-B rows (one channel, 128 pixels), 16-B chunk ch of row r at
// 256 r + 16 (ch ^ swz) (cdna_hip_programming.md T10 image (b): the transposed reads of the
// 32x32x16 B operand are conflict-free)
__device__ __forceinline__ constexpr int f16_bswz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
// A stage image: 64-B rows, 16-B chunk ch of row r at 64 r + 16 (ch ^ ((r >> 2) & 3)) (the
// ds_read_b128 row reads of 16 rows per lane group land on distinct banks)
__device__ __forceinline__ constexpr int f16_aswz(int r) { return (r >> 2) & 3; }

__global__ __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void wide_dist_f16_kernel(F16DistArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char fsm[];
  const unsigned S0 = static_cast<unsigned>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) void*)fsm));
  const int lane = threadIdx.x & 63, wave = bf16l::wave_id(), j = lane & 31, h = lane >> 5;
  const int n0 = static_cast<int>(blockIdx.x) * kF16TN, m0 = static_cast<int>(blockIdx.y) * kF16TM;
  const rsrc_t rx = make_rsrc(a.x, a.x_bytes), rah = make_rsrc(a.ahi, a.a_bytes), ral = make_rsrc(a.alo, a.a_bytes);
  float* red = reinterpret_cast<float*>(fsm + kF16NS * kF16Stage);     // [16][128] x2 partials
  float* rowv = red + 16 * kF16TN;                                     // [192] p2, [192] 1 / s_p
  for (int i = static_cast<int>(threadIdx.x); i < kF16TM; i += 256) {
    rowv[i] = a.p2[m0 + i];
    rowv[kF16TM + i] = a.inv_s[m0 + i];
  }

  // DMA pieces of a stage (1 KiB each): 12 per A term (16 rows each) and 8 of x (4 channel rows
  // each). Wave w issues A pieces 6 (w & 1) .. + 5 of term w >> 1 and x pieces 2 w, 2 w + 1: one
  // buffer resource per operand, no wave-dependent branches in the stage loop.
  const int pl = wave >> 1, half = wave & 1;
  const rsrc_t ra = pl ? ral : rah;
  unsigned voa[6], vox[2];
  int crow_of[2];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int r = 16 * (6 * half + i) + (lane >> 2), lc = (lane & 3) ^ f16_aswz(r);
    voa[i] = static_cast<unsigned>(((m0 + r) * a.Kpad + 8 * lc) * 2);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int crow = 4 * (2 * wave + i) + (lane >> 4), lc = (lane & 15) ^ f16_bswz(crow);
    const int col = n0 + 8 * lc;
    crow_of[i] = crow;
    if (col < a.ntot) {
      const int b = col / a.HW, n = col - b * a.HW;
      vox[i] = static_cast<unsigned>(((b * a.C + crow) * a.HW + n) * 2);
    } else {
      vox[i] = kOOB;
    }
  }
  const unsigned lda_off = static_cast<unsigned>(pl * kF16ATerm + 6 * half * 1024);
  const unsigned ldx_off = static_cast<unsigned>(2 * kF16ATerm + 2 * wave * 1024);
  auto issue = [&](int st) __attribute__((always_inline)) {
    const int k0 = st * kF16TK;
    const unsigned base = S0 + static_cast<unsigned>((st % kF16NS) * kF16Stage);
#pragma unroll
    for (int i = 0; i < 6; ++i)
      dma16(ra, base + lda_off + static_cast<unsigned>(i * 1024), voa[i], static_cast<unsigned>(k0 * 2));
#pragma unroll
    for (int i = 0; i < 2; ++i)
      dma16(rx, base + ldx_off + static_cast<unsigned>(i * 1024), k0 + crow_of[i] < a.C ? vox[i] : kOOB,
            static_cast<unsigned>(k0 * a.HW * 2));
  };

  // wave w: prototype rows 96 (w & 1) + 32 i (i < 3), pixel columns 64 (w >> 1) + 32 jj (jj < 2)
  const int rg = wave & 1, cp = wave >> 1;
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  f32x16 acc[3][2];
#pragma unroll
  for (int i = 0; i < 3; ++i) acc[i][0] = acc[i][1] = zero16();
  // x2: thread t sums columns 8 (t & 15) .. + 7 over channel rows 2 (t >> 4), + 1 of each stage
  float xs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int xcc = threadIdx.x & 15, xrg = threadIdx.x >> 4;

  const int nst = a.Kpad / kF16TK;
  issue(0);
  if (nst > 1) issue(1);
  for (int st = 0; st < nst; ++st) {
    if (st + 1 < nst) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    const unsigned sb = S0 + static_cast<unsigned>((st % kF16NS) * kF16Stage);
    // Schedule (one wave per SIMD: nothing else hides an LDS round trip): the first 16-k step's
    // fragments are read up front, the second step's and the x2 rows go out one per MFMA of the
    // first step, then the second step's MFMAs and the x2 arithmetic. Left alone the compiler
    // reloaded one fragment register per MFMA pair and waited on every read.
    f16x8 af[2][3][2], bfr[2][2];
    auto read_step = [&](int ks) __attribute__((always_inline)) {
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        // block (channel rows 16 ks + 8 h (+4), pixel columns 64 cp + 32 jj + 16 (g & 1) ..):
        // lane 4 q + p of the 16-lane group supplies row r0 + q, columns + 4 p .. + 3
        const int ch = 8 * cp + 4 * jj + 2 * (g & 1) + (p4 >> 1);
        f16s4 v[2];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          const int r = 16 * ks + 8 * h + 4 * hf + q4;
          const unsigned bo = static_cast<unsigned>(2 * kF16ATerm + 256 * r + 16 * (ch ^ f16_bswz(r)) + 8 * (p4 & 1));
          v[hf] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              reinterpret_cast<__attribute__((address_space(3))) f16s4*>(static_cast<uintptr_t>(sb + bo)));
        }
        bfr[ks][jj] = __builtin_bit_cast(f16x8, __builtin_shufflevector(v[0], v[1], 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int r = 96 * rg + 32 * i + j;
        const unsigned ao = static_cast<unsigned>(r * 64 + 16 * ((2 * ks + h) ^ f16_aswz(r)));
#pragma unroll
        for (int t = 0; t < 2; ++t)
          af[ks][i][t] = *reinterpret_cast<const __attribute__((address_space(3))) f16x8*>(
              static_cast<uintptr_t>(sb + static_cast<unsigned>(t * kF16ATerm) + ao));
      }
    };
    auto mfma_step = [&](int ks) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[ks][i][1], bfr[ks][jj], acc[i][jj], 0, 0, 0);
          acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[ks][i][0], bfr[ks][jj], acc[i][jj], 0, 0, 0);
        }
    };
    read_step(0);
    __builtin_amdgcn_sched_barrier(0);
    // x2 rows of the stage: this thread's 8 columns 8 xcc .. + 7 of channel rows 2 xrg, 2 xrg + 1
    // (zeros past C / past the pixels: the DMA filled them so)
    f16x8 xr[2];
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const int r = 2 * xrg + rr;
      xr[rr] = *reinterpret_cast<const __attribute__((address_space(3))) f16x8*>(
          static_cast<uintptr_t>(sb + static_cast<unsigned>(2 * kF16ATerm + 256 * r + 16 * (xcc ^ f16_bswz(r)))));
    }
    read_step(1);
    mfma_step(0);
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one LDS read
    }
    __builtin_amdgcn_sched_barrier(0);
    mfma_step(1);
#pragma unroll
    for (int rr = 0; rr < 2; ++rr)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = static_cast<float>(xr[rr][e]);
        xs[e] = fmaf(v, v, xs[e]);
      }
    // the stage after next goes out behind the MFMAs (their pipe is busy while the wave issues
    // it); its buffer was last read in stage st - 1, which every wave finished before this
    // stage's barrier
    __builtin_amdgcn_sched_barrier(0);
    if (st + 2 < nst) issue(st + 2);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[xrg * kF16TN + 8 * xcc + e] = xs[e];
  __syncthreads();

  const rsrc_t rd = make_rsrc(a.dist, a.d_bytes);
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int cn = 64 * cp + 32 * jj + j, col = n0 + cn;
    float x2 = red[cn];
#pragma unroll
    for (int q = 1; q < 16; ++q) x2 += red[q * kF16TN + cn];
    const int b = col < a.ntot ? col / a.HW : 0, n = col - b * a.HW;
    // the lane's part of the address (pixel, row 4h) in the voffset, the register's row in the
    // (uniform) soffset
    const unsigned cbase = col < a.ntot ? static_cast<unsigned>((b * a.P * a.HW + n + 4 * h * a.HW) * 4) : kOOB;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int rl = 96 * rg + 32 * i;
      float p2r[16], isr[16];
      bf16l::load_rows16(rowv + rl + 4 * h, p2r);
      bf16l::load_rows16(rowv + kF16TM + rl + 4 * h, isr);
      float d[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mu = m0 + rl + row_of(r);  // wave-uniform; this lane's row is mu + 4h
        d[r] = l2_distance(x2, p2r[r], acc[i][jj][r] * isr[r]);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(d[r]), rd, mu + 4 * h < a.P ? cbase : kOOB,
                                              static_cast<unsigned>(mu * a.HW * 4), 0);
      }
      if (a.act && col < a.ntot) {  // (return_activations: [pixel][P], uncoalesced; not the training path)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + rl + row_of(r) + 4 * h;
          if (m < a.P) a.act[static_cast<size_t>(col) * a.P + m] = activation(d[r], a.eps, a.act_kind);
        }
      }
    }
  }
}

int wide_distances_f16(const Geometry& g, const _Float16* x, const float* protos, float eps, int act_kind,
                       float* dist, float* act, hipStream_t s) {
  const int Mpad = static_cast<int>(ceil_div(g.P, kF16TM)) * kF16TM;
  const int Kpad = static_cast<int>(ceil_div(g.C, kF16TK)) * kF16TK;
  const size_t term = static_cast<size_t>(Mpad) * Kpad * 2;
  void* sc = nullptr;
  if (int st = stream_scratch(ScratchKind::kWideF16, 2 * term + static_cast<size_t>(Mpad) * 8, 1u << 20, s, &sc))
    return st;
  auto* ahi = static_cast<_Float16*>(sc);
  auto* alo = reinterpret_cast<_Float16*>(static_cast<unsigned char*>(sc) + term);
  auto* p2 = reinterpret_cast<float*>(static_cast<unsigned char*>(sc) + 2 * term);
  float* inv_s = p2 + Mpad;
  hipLaunchKernelGGL(wide_f16_prep_kernel, dim3(static_cast<unsigned>(Mpad / 4)), dim3(256), 0, s, protos, g.P, g.C,
                     Mpad, Kpad, ahi, alo, p2, inv_s);
  if (int st = check_launch("wide_f16_prep_kernel")) return st;
  if (int e = ensure_lds<wide_dist_f16_kernel, kF16Lds>()) return e;
  F16DistArgs a{};
  a.x = x;
  a.x_bytes = static_cast<unsigned>(static_cast<size_t>(g.npix) * g.C * 2);
  a.ahi = ahi, a.alo = alo, a.a_bytes = static_cast<unsigned>(term);
  a.p2 = p2, a.inv_s = inv_s;
  a.P = g.P, a.C = g.C, a.Kpad = Kpad, a.HW = g.HW, a.ntot = g.npix;
  a.dist = dist, a.d_bytes = static_cast<unsigned>(static_cast<size_t>(g.npix) * g.P * 4);
  a.act = act, a.act_kind = act_kind, a.eps = eps;
  KernelTimer timer("wide_dist_f16_kernel", s);
  hipLaunchKernelGGL(wide_dist_f16_kernel, dim3(static_cast<unsigned>(ceil_div(g.npix, kF16TN)),
                                                static_cast<unsigned>(Mpad / kF16TM)),
                     dim3(256), kF16Lds, s, a);
  return check_launch("wide_dist_f16_kernel");
}

// The fp16 path serves bf16x3 requests on fp16 maps whose 8-pixel runs stay inside one image
// and whose tensors stay below 2^31 bytes (buffer offsets).
bool wide_f16_fits(const Geometry& g, const void* x) {
  return g.HW % 8 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0 &&
         static_cast<long long>(g.npix) * g.C * 2 < (1LL << 31) && static_cast<long long>(g.npix) * g.P * 4 < (1LL << 31) &&
         static_cast<long long>(ceil_div(g.P, kF16TM)) * kF16TM * ceil_div(g.C, kF16TK) * kF16TK * 2 < (1LL << 31);
}

// ---- the wide backward's two large GEMMs on pre-split bf16 operands --------------------------
// g_x = -2 P^T G_s + 2 x sum_p G_s (M = C, N = pixels, K = P) and g_P = -2 G_s X^T + 2 p sum G_s
// (M = P, N = C, K = pixels, split over workgroups) with every operand stored as two bf16 planes
// (hi, lo) by its producer: the G_s GEMM's epilogue (kEpiGsSplit), wide_pt_split_kernel (P^T) and
// wide_x_split_kernel (x). The GEMM stages are then byte copies (16-B LDS-DMA, three stages in
// flight) and each 16-k step is 3 v_mfma_f32_32x32x16_bf16 (hi.lo + lo.hi + hi.hi): bf16x3
// products, the same split as the 64 x 64 tile's, without its per-stage conversion (which bound
// that kernel). Tile 192 x 128 x 32, 4 waves x (3 x 2) blocks, as wide_dist_f16_kernel.

struct PreArgs {
  const uint16_t *ahi, *alo;  // A planes: element (row, kg) at (kg / akb) sab + row lda + kg % akb
  unsigned a_bytes;
  long long sab;
  int lda, akb, arows;        // rows >= arows read 0
  const uint16_t *bhi, *blo;  // B planes. BT = 0: (col, kg) as A (ldb, bkb, sbb, bcols);
  unsigned b_bytes;           // BT = 1: (kg, col): col -> (cb, n) = (col / bnb, col % bnb),
  long long sbb;              //         cb sbb + kg ldb + n; kg >= bk read 0
  int ldb, bkb, bcols, bnb, bk;
  int M, N, K;                // K: the flattened contraction (a multiple of 32)
  int ksplit;
  float* slab;                // EPI 0: slab z: [M][N] f32 at z M N
  void* gx;                   // EPI 1: g_x (TO) at (b, c, n): (b C + c) HW + n, col = b HW + n
  const void* x;              //        x at the same offset
  unsigned o_bytes;
  int C, HW;
};

// Buffer-resource element IO of g_x / x in the feature map's dtype (out-of-range: load 0, store dropped).
// load_raw / from_raw: the element's bits (one 32-bit register) and their value, so a batch of
// loads can be pinned before any conversion (a conversion right behind its load makes the
// allocator reuse one destination register, i.e. one wait per load).
template <typename T> struct BufIO2 : BufIO<T> {};
template <> struct BufIO2<float> : BufIO<float> {
  static __device__ __forceinline__ uint32_t load_raw(rsrc_t r, unsigned voff, unsigned soff) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0);
  }
  static __device__ __forceinline__ float from_raw(uint32_t v) { return __uint_as_float(v); }
};
template <> struct BufIO2<uint16_t> : BufIO<uint16_t> {
  static __device__ __forceinline__ uint32_t load_raw(rsrc_t r, unsigned voff, unsigned soff) {
    return static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b16(r, voff, soff, 0));
  }
  static __device__ __forceinline__ float from_raw(uint32_t v) { return __uint_as_float(v << 16); }
};
template <> struct BufIO2<_Float16> {
  static __device__ __forceinline__ uint32_t load_raw(rsrc_t r, unsigned voff, unsigned soff) {
    return static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b16(r, voff, soff, 0));
  }
  static __device__ __forceinline__ float from_raw(uint32_t v) {
    return static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(v)));
  }
  static __device__ __forceinline__ float load(rsrc_t r, unsigned voff, unsigned soff) {
    return static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(__builtin_amdgcn_raw_buffer_load_b16(r, voff, soff, 0))));
  }
  static __device__ __forceinline__ void store(rsrc_t r, float v, unsigned voff, unsigned soff) {
    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, static_cast<_Float16>(v)), r, voff, soff, 0);
  }
};

template <int EPI, bool BT, typename TO, int MI>
__global__ __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void wide_pre_gemm_kernel(PreArgs a) {
  constexpr int kTM = pre_tm(MI), kAP = pre_aplane(MI), kStage = pre_stage(MI);
  constexpr int kAW = 2 * MI;  // A pieces per wave and stage (16 rows each)
  extern __shared__ __attribute__((aligned(16))) unsigned char psm[];
  const unsigned S0 = static_cast<unsigned>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) void*)psm));
  const int lane = threadIdx.x & 63, wave = bf16l::wave_id(), j = lane & 31, h = lane >> 5;
  const int n0 = static_cast<int>(blockIdx.x) * kPreTN, m0 = static_cast<int>(blockIdx.y) * kTM;
  const int z = static_cast<int>(blockIdx.z);
  const rsrc_t rah = make_rsrc(a.ahi, a.a_bytes), ral = make_rsrc(a.alo, a.a_bytes);
  const rsrc_t rbh = make_rsrc(a.bhi, a.b_bytes), rbl = make_rsrc(a.blo, a.b_bytes);
  const int nst_all = a.K / kPreTK;
  const int st0 = static_cast<int>((static_cast<long long>(nst_all) * z) / a.ksplit);
  const int st1 = static_cast<int>((static_cast<long long>(nst_all) * (z + 1)) / a.ksplit);
  const int nst = st1 - st0;

  // DMA pieces per stage (1 KiB each): A planes of 4 MI pieces (16 rows each), B planes of 8
  // (BT = 0: 16 columns each; BT = 1: 4 k rows each). Wave w issues plane w >> 1 of both
  // operands: A pieces 2 MI (w & 1) .. + 2 MI - 1, B pieces 4 (w & 1) .. + 3 — one buffer
  // resource per operand, no wave-dependent branches in the stage loop.
  const int pl = wave >> 1, half = wave & 1;
  const rsrc_t ra = pl ? ral : rah, rb = pl ? rbl : rbh;
  unsigned voa[kAW], vob[4];
  int krow[4];
#pragma unroll
  for (int i = 0; i < kAW; ++i) {
    const int r = 16 * (kAW * half + i) + (lane >> 2), lc = (lane & 3) ^ f16_aswz(r);
    voa[i] = m0 + r < a.arows ? static_cast<unsigned>((static_cast<long long>(m0 + r) * a.lda + 8 * lc) * 2) : kOOB;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int qb = 4 * half + i;
    krow[i] = 0;
    if constexpr (!BT) {
      const int r = 16 * qb + (lane >> 2), lc = (lane & 3) ^ f16_aswz(r);
      vob[i] = n0 + r < a.bcols ? static_cast<unsigned>((static_cast<long long>(n0 + r) * a.ldb + 8 * lc) * 2) : kOOB;
    } else {
      const int kr = 4 * qb + (lane >> 4), lc = (lane & 15) ^ f16_bswz(kr);
      const int col = n0 + 8 * lc;
      krow[i] = kr;
      if (col < a.bcols) {
        const int cb = col / a.bnb, n = col - cb * a.bnb;
        vob[i] = static_cast<unsigned>((cb * a.sbb + static_cast<long long>(kr) * a.ldb + n) * 2);
      } else {
        vob[i] = kOOB;
      }
    }
  }
  const unsigned lda_off = static_cast<unsigned>(pl * kAP + kAW * half * 1024);
  const unsigned ldb_off = static_cast<unsigned>(2 * kAP + pl * kPreBPlane + 4 * half * 1024);
  // stage soffsets advance by 32 k per issue (issue() runs for st = 0, 1, 2, ... in order): the
  // (block, rest) of kg in the A (and BT = 0 B) k-blocking, without a division per stage
  int kga = st0 * kPreTK, ka_b = kga / a.akb, ka_r = kga - ka_b * a.akb;
  int kb_b = BT ? 0 : kga / a.bkb, kb_r = BT ? 0 : kga - kb_b * a.bkb;
  auto issue = [&](int st) __attribute__((always_inline)) {  // global stage st0 + st into buffer st % 3
    const unsigned base = S0 + static_cast<unsigned>((st % kPreNS) * kStage);
    const unsigned sa = static_cast<unsigned>((ka_b * a.sab + ka_r) * 2);
#pragma unroll
    for (int i = 0; i < kAW; ++i) dma16(ra, base + lda_off + static_cast<unsigned>(i * 1024), voa[i], sa);
    if constexpr (!BT) {
      const unsigned sb = static_cast<unsigned>((kb_b * a.sbb + kb_r) * 2);
#pragma unroll
      for (int i = 0; i < 4; ++i) dma16(rb, base + ldb_off + static_cast<unsigned>(i * 1024), vob[i], sb);
      kb_r += kPreTK;
      if (kb_r == a.bkb) kb_r = 0, ++kb_b;
    } else {
      const int kg = kga;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        dma16(rb, base + ldb_off + static_cast<unsigned>(i * 1024), kg + krow[i] < a.bk ? vob[i] : kOOB,
              static_cast<unsigned>(static_cast<long long>(kg) * a.ldb * 2));
    }
    kga += kPreTK;
    ka_r += kPreTK;
    if (ka_r == a.akb) ka_r = 0, ++ka_b;
  };

  const int rg = wave & 1, cp = wave >> 1;
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  f32x16 acc[MI][2];
#pragma unroll
  for (int i = 0; i < MI; ++i) acc[i][0] = acc[i][1] = zero16();
  // EPI 1: column sums of B (sum_p G_s): thread t sums columns 8 (t & 15) .. + 7 over k rows
  // 2 (t >> 4), + 1 of each stage
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int xcc = threadIdx.x & 15, xrg = threadIdx.x >> 4;

  if (nst > 0) issue(0);
  if (nst > 1) issue(1);
  for (int st = 0; st < nst; ++st) {
    if (st + 1 < nst) {  // this stage's pieces landed; the next stage's (kAW + 4 per wave) may be in flight
      if constexpr (MI == 3) asm volatile("s_waitcnt vmcnt(10)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(12)\n\ts_barrier" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
    const unsigned sb = S0 + static_cast<unsigned>((st % kPreNS) * kStage);
    // schedule as in wide_dist_f16_kernel: step 0's fragments up front, step 1's (and the EPI 1
    // column-sum rows) one per MFMA of step 0, then step 1's MFMAs
    bf16x8 af[2][MI][2], bfr[2][2][2];
    auto read_step = [&](int ks) __attribute__((always_inline)) {
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const unsigned pb = sb + static_cast<unsigned>(2 * kAP + t * kPreBPlane);
          if constexpr (!BT) {
            const int c = 64 * cp + 32 * jj + j;
            bfr[ks][jj][t] = *reinterpret_cast<const __attribute__((address_space(3))) bf16x8*>(
                static_cast<uintptr_t>(pb + static_cast<unsigned>(c * 64 + 16 * ((2 * ks + h) ^ f16_aswz(c)))));
          } else {
            const int ch = 8 * cp + 4 * jj + 2 * (g & 1) + (p4 >> 1);
            f16s4 v[2];
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
              const int r = 16 * ks + 8 * h + 4 * hf + q4;
              v[hf] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(reinterpret_cast<__attribute__((address_space(3))) f16s4*>(
                  static_cast<uintptr_t>(pb + static_cast<unsigned>(256 * r + 16 * (ch ^ f16_bswz(r)) + 8 * (p4 & 1)))));
            }
            bfr[ks][jj][t] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v[0], v[1], 0, 1, 2, 3, 4, 5, 6, 7));
          }
        }
      }
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int r = 32 * MI * rg + 32 * i + j;
        const unsigned ao = static_cast<unsigned>(r * 64 + 16 * ((2 * ks + h) ^ f16_aswz(r)));
#pragma unroll
        for (int t = 0; t < 2; ++t)
          af[ks][i][t] = *reinterpret_cast<const __attribute__((address_space(3))) bf16x8*>(
              static_cast<uintptr_t>(sb + static_cast<unsigned>(t * kAP) + ao));
      }
    };
    read_step(0);
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 cr[2][2];  // EPI 1: B rows 2 xrg, 2 xrg + 1, columns 8 xcc .. + 7, hi and lo
    if constexpr (EPI == 1) {
#pragma unroll
      for (int rr = 0; rr < 2; ++rr)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int r = 2 * xrg + rr;
          cr[rr][t] = *reinterpret_cast<const __attribute__((address_space(3))) bf16x8*>(static_cast<uintptr_t>(
              sb + static_cast<unsigned>(2 * kAP + t * kPreBPlane + 256 * r + 16 * (xcc ^ f16_bswz(r)))));
        }
    }
    read_step(1);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) acc[i][jj] = mma_split<2>(af[0][i], bfr[0][jj], acc[i][jj]);
#pragma unroll
    for (int k = 0; k < 6 * MI; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one LDS read
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) acc[i][jj] = mma_split<2>(af[1][i], bfr[1][jj], acc[i][jj]);
    if constexpr (EPI == 1) {
#pragma unroll
      for (int rr = 0; rr < 2; ++rr)
#pragma unroll
        for (int e = 0; e < 8; ++e) cs[e] += static_cast<float>(cr[rr][0][e]) + static_cast<float>(cr[rr][1][e]);
    }
    // the stage after next goes out behind the MFMAs (wide_dist_f16_kernel)
    __builtin_amdgcn_sched_barrier(0);
    if (st + 2 < nst) issue(st + 2);
  }

  float* red = reinterpret_cast<float*>(psm + kPreNS * kStage);
  if constexpr (EPI == 1) {
#pragma unroll
    for (int e = 0; e < 8; ++e) red[xrg * kPreTN + 8 * xcc + e] = cs[e];
    __syncthreads();
  }

#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int cn = 64 * cp + 32 * jj + j, col = n0 + cn;
    if constexpr (EPI == 0) {  // slab z: [M][N] f32, lane = column
      const rsrc_t rs = make_rsrc(a.slab + static_cast<size_t>(z) * a.M * a.N, static_cast<unsigned>(static_cast<size_t>(a.M) * a.N * 4));
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int mu = m0 + 32 * MI * rg + 32 * i + row_of(r);  // wave-uniform; the lane's row is mu + 4h
          const bool ok = mu + 4 * h < a.M && col < a.N;
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[i][jj][r]), rs,
                                                ok ? static_cast<unsigned>(((4 * h) * a.N + col) * 4) : kOOB,
                                                static_cast<unsigned>(mu * a.N * 4), 0);
        }
    } else {  // g_x (TO) at (b C + c) HW + n: -2 acc + 2 x sum_p G_s
      float csum = red[cn];
#pragma unroll
      for (int q = 1; q < 16; ++q) csum += red[q * kPreTN + cn];
      const int b = col < a.N ? col / a.HW : 0, n = col - b * a.HW;
      const unsigned cbase = col < a.N ? static_cast<unsigned>((b * a.C * a.HW + n + 4 * h * a.HW) * sizeof(TO)) : kOOB;
      const rsrc_t ro = make_rsrc(a.gx, a.o_bytes), rxo = make_rsrc(a.x, a.o_bytes);
      // per 32-row block: the 16 x loads first (the stores to g_x may alias them as far as the
      // compiler knows, so a load after a store would wait a whole round trip each), then the
      // stores. A tile whose rows are all below M (the common case) keeps one voffset for every
      // row (the row in the uniform soffset): per-row guarded voffsets ran the 256-VGPR kernel
      // out of registers and the allocator put a wait behind every load.
      auto rows = [&](auto full_tag) __attribute__((always_inline)) {
        constexpr bool kFull = decltype(full_tag)::value;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          uint32_t xr[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int mu = m0 + 32 * MI * rg + 32 * i + row_of(r);
            xr[r] = BufIO2<TO>::load_raw(rxo, kFull || mu + 4 * h < a.M ? cbase : kOOB,
                                         static_cast<unsigned>(mu * a.HW * sizeof(TO)));
          }
          pin_batch(xr);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int mu = m0 + 32 * MI * rg + 32 * i + row_of(r);
            BufIO2<TO>::store(ro, -2.f * acc[i][jj][r] + 2.f * BufIO2<TO>::from_raw(xr[r]) * csum,
                              kFull || mu + 4 * h < a.M ? cbase : kOOB, static_cast<unsigned>(mu * a.HW * sizeof(TO)));
          }
        }
      };
      if (m0 + kTM <= a.M) rows(std::true_type());
      else rows(std::false_type());
    }
  }
}

// P^T as bf16 planes [C][kp] (k = p; zero past P): 64 x 64 tiles through LDS (coalesced both ways).
__global__ __launch_bounds__(256) void wide_pt_split_kernel(const float* __restrict__ protos, int P, int C, int kp,
                                                            uint16_t* __restrict__ hi, uint16_t* __restrict__ lo) {
  __shared__ float t[64][65];
  const int p0 = static_cast<int>(blockIdx.x) * 64, c0 = static_cast<int>(blockIdx.y) * 64;
  {  // the 16 loads of a thread in flight together (clamped addresses, pin_batch)
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int i = static_cast<int>(threadIdx.x) + 256 * k, pr = i >> 6, cc = i & 63;
      const int pp = p0 + pr < P ? p0 + pr : P - 1, c = c0 + cc < C ? c0 + cc : C - 1;
      v[k] = protos[static_cast<size_t>(pp) * C + c];
    }
    pin_batch(v);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int i = static_cast<int>(threadIdx.x) + 256 * k, pr = i >> 6, cc = i & 63;
      t[pr][cc] = p0 + pr < P && c0 + cc < C ? v[k] : 0.f;
    }
  }
  __syncthreads();
  for (int i = static_cast<int>(threadIdx.x); i < 64 * 64; i += 256) {
    const int cc = i >> 6, pr = i & 63;
    if (c0 + cc >= C || p0 + pr >= kp) continue;
    const float v = t[pr][cc];
    const bf16 vh = static_cast<bf16>(v);
    const size_t o = static_cast<size_t>(c0 + cc) * kp + p0 + pr;
    hi[o] = __builtin_bit_cast(uint16_t, vh);
    lo[o] = __builtin_bit_cast(uint16_t, static_cast<bf16>(v - static_cast<float>(vh)));
  }
}

// x (TX) -> bf16 planes of the same shape (hi = bf16(x), lo = bf16(x - hi); exact for fp16 / bf16 x).
template <typename TX>
__global__ __launch_bounds__(256) void wide_x_split_kernel(const TX* __restrict__ x, long long n, uint16_t* __restrict__ hi,
                                                           uint16_t* __restrict__ lo) {
  // 8 grid strides per step with their loads in flight (clamped addresses, pin_batch)
  const long long stride = static_cast<long long>(gridDim.x) * 256;
  for (long long i0 = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x; i0 < n; i0 += 8 * stride) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long long i = i0 + u * stride;
      v[u] = XIO<TX>::load(x, static_cast<size_t>(i < n ? i : n - 1));
    }
    pin_batch(v);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long long i = i0 + u * stride;
      if (i < n) {
        const bf16 vh = static_cast<bf16>(v[u]);
        hi[i] = __builtin_bit_cast(uint16_t, vh);
        lo[i] = __builtin_bit_cast(uint16_t, static_cast<bf16>(v[u] - static_cast<float>(vh)));
      }
    }
  }
}

// rs[p] = sum_{b, n} G_s[b][p][n] from the split planes (hi + lo per element), fixed-order tree.
__global__ __launch_bounds__(256) void wide_rowsum_split_kernel(const uint16_t* __restrict__ gh, const uint16_t* __restrict__ gl,
                                                                int P, int HW, int B, float* __restrict__ rs) {
  __shared__ float red[256];
  const int p = blockIdx.x;
  // per pixel n of the thread, the images in order (the summation order of one image at a time
  // when HW <= 256); 8 images' loads in flight through clamped addresses (pin_batch), not one
  // guarded load and its round trip per image
  float s = 0.f;
  for (int n = threadIdx.x; n < HW; n += 256) {
    for (int b0 = 0; b0 < B; b0 += 8) {
      uint32_t hv[8], lv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int bb = b0 + u < B ? b0 + u : B - 1;
        const size_t o = (static_cast<size_t>(bb) * P + p) * HW + n;
        hv[u] = gh[o];
        lv[u] = gl[o];
      }
      pin_batch(hv);
      pin_batch(lv);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (b0 + u < B) s += __uint_as_float(hv[u] << 16) + __uint_as_float(lv[u] << 16);
    }
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (static_cast<int>(threadIdx.x) < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) rs[p] = red[0];
}

// Partial column sums of G_s (f32): csq[q][b HW + n] = sum over prototype chunk q (of kColsumQ,
// blockIdx.y) of G_s[b][p][n]. Workgroup = 32 pixels x 8 prototype groups (group r sums p = r,
// r + 8, ... of the chunk in order, 4 loads in flight), the groups added in order; the finish adds
// the chunks in order.
__global__ __launch_bounds__(256) void wide_colsum_kernel(const float* __restrict__ gs, int P, int HW, int npix,
                                                          float* __restrict__ csq) {
  __shared__ float red[8][32];
  const int j = static_cast<int>(threadIdx.x) & 31, q = static_cast<int>(threadIdx.x) >> 5;
  const int g = static_cast<int>(blockIdx.x) * 32 + j;
  const int gc = g < npix ? g : npix - 1;
  const int b = gc / HW, n = gc - b * HW;
  const int ch = static_cast<int>(blockIdx.y);
  const int pb = static_cast<int>(static_cast<long long>(P) * ch / kColsumQ);
  const int pe = static_cast<int>(static_cast<long long>(P) * (ch + 1) / kColsumQ);
  const float* col = gs + static_cast<size_t>(b) * P * HW + n;
  float s = 0.f;
  for (int p0 = pb + q; p0 < pe; p0 += 32) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = p0 + 8 * u;
      v[u] = col[static_cast<size_t>(p < pe ? p : p0) * HW];
    }
    pin_batch(v);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (p0 + 8 * u < pe) s += v[u];
  }
  red[q][j] = s;
  __syncthreads();
  if (q == 0 && g < npix) {
    float t = red[0][j];
#pragma unroll
    for (int k = 1; k < 8; ++k) t += red[k][j];
    csq[static_cast<size_t>(ch) * npix + g] = t;
  }
}

// g_x from split-K slabs [B][S][C][HW]: -2 sum_z (slab order) + 2 x cs, stored in x's dtype.
template <typename TO>
__global__ __launch_bounds__(256) void wide_finish_gx_kernel(const float* __restrict__ part, int S, int B, int C, int HW,
                                                             const TO* __restrict__ x, const float* __restrict__ csq,
                                                             TO* __restrict__ gx) {
  const long long e = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  const long long mn = static_cast<long long>(C) * HW;
  if (e >= mn * B) return;
  const long long b = e / mn, r = e - b * mn;
  const int n = static_cast<int>(r % HW);
  const float* pp = part + static_cast<size_t>(b) * S * mn + r;
  float s = 0.f;
  for (int i0 = 0; i0 < S; i0 += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = pp[static_cast<size_t>(i0 + u < S ? i0 + u : 0) * mn];
    pin_batch(v);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (i0 + u < S) s += v[u];
  }
  const long long npix = static_cast<long long>(B) * HW;
  float cq[kColsumQ];
#pragma unroll
  for (int q = 0; q < kColsumQ; ++q) cq[q] = csq[q * npix + b * HW + n];
  float cs = cq[0];
#pragma unroll
  for (int q = 1; q < kColsumQ; ++q) cs += cq[q];
  const float xv = XIO<TO>::load(x, static_cast<size_t>(e));
  XIO<TO>::store(gx, static_cast<size_t>(e), -2.f * s + 2.f * xv * cs);
}

// D[b][p][n] into `dist` (ld P per image), optional act[g][p].
template <typename TX>
int wide_distances(const Geometry& g, const TX* x, const float* protos, float eps, int act_kind, float* dist,
                   float* act, hipStream_t s, int bf3 = 0) {
  const int B = g.npix / g.HW;
  WideArgs a{};
  a.A = op(protos, g.C, 1, 0);                                   // P[p][c]
  a.B = op(x, 1, g.HW, static_cast<long long>(g.C) * g.HW);      // X[b][c][n]: (n, c)
  a.M = g.P, a.N = g.HW, a.Kd = g.C, a.nb = B;
  a.out = dist, a.om = g.HW, a.on = 1, a.ob = static_cast<long long>(g.P) * g.HW;
  a.eps = eps, a.act_kind = act_kind;
  a.act = act, a.am = 1, a.an = g.P, a.ab = static_cast<long long>(g.HW) * g.P;  // act[(b HW + n) P + p]
  a.bf3 = bf3;
  if constexpr (std::is_same_v<TX, _Float16>) {
    if (bf3 && WIDE_F16_MFMA && wide_f16_fits(g, x)) return wide_distances_f16(g, x, protos, eps, act_kind, dist, act, s);
  }
  return gemm<kEpiDist, float, TX, -1, -1, float>(a, B, s);
}

}  // namespace

bool wide_family_fits(const Geometry& g) {
  const long long lim = 1LL << 31;
  return g.C >= 1 && g.P >= 1 && g.K >= 0 && static_cast<long long>(g.npix) * g.P < lim &&
         static_cast<long long>(g.npix) * g.C < lim && static_cast<long long>(g.npix) * g.K < lim &&
         static_cast<long long>(g.P) * g.C < lim && static_cast<long long>(g.P) * g.K < lim;
}

// The distances (when the caller wants logits only) and the logits' split-K slabs.
size_t wide_fwd_scratch_bytes(const Geometry& g, bool need_dist) {
  const size_t d = need_dist ? static_cast<size_t>(g.npix) * g.P : 0;
  const int S = logits_split(g);
  const size_t part = S > 1 ? static_cast<size_t>(S) * g.npix * g.K : 0;
  return (((d + 63) & ~static_cast<size_t>(63)) + part) * sizeof(float) + 256;
}

size_t wide_bwd_workspace_bytes(const Geometry& g) { return wide_bwd_layout(g).total * sizeof(float); }

namespace {
// D = distances of x in its stored dtype (F32 | BF16 | F16)
int distances_of(const Geometry& g, int x_dtype, const void* x, const float* protos, float eps, int act_kind, float* D,
                 float* act, hipStream_t s, int bf3) {
  if (x_dtype == PROTOSEG_BF16)
    return wide_distances(g, static_cast<const uint16_t*>(x), protos, eps, act_kind, D, act, s, bf3);
  if (x_dtype == PROTOSEG_F16)
    return wide_distances(g, static_cast<const _Float16*>(x), protos, eps, act_kind, D, act, s, bf3);
  return wide_distances(g, static_cast<const float*>(x), protos, eps, act_kind, D, act, s, bf3);
}
}  // namespace

int launch_fwd_wide(const Geometry& g, int x_dtype, const void* x, const float* protos, const float* w_last, float eps,
                    int act_kind, float* dist, float* act, float* logits, void* scratch, hipStream_t s, int bf3) {
  float* sc = static_cast<float*>(scratch);
  float* D = dist ? dist : sc;  // the logits read the distances back
  float* part = sc + (dist ? 0 : ((static_cast<size_t>(g.npix) * g.P + 63) & ~static_cast<size_t>(63)));
  int st = distances_of(g, x_dtype, x, protos, eps, act_kind, D, act, s, bf3);
  if (st || !logits) return st;
  // logits[b][n][k] = sum_p act(D[b][p][n]) W[k][p]; split over p into slabs [b][S][HW][K] when
  // the images' tiles are too few for the CUs
  const int S = logits_split(g), B = g.npix / g.HW;
  WideArgs a{};
  a.A = op(D, 1, g.HW, static_cast<long long>(g.P) * g.HW);   // (n, p) of D[b][p][n]
  a.B = op(w_last, g.ldw, 1, 0);                              // (k, p) of W[k][p]
  a.M = g.HW, a.N = g.K, a.Kd = g.P, a.nb = B, a.ksplit = S;
  a.out = S > 1 ? static_cast<void*>(part) : logits, a.om = g.K, a.on = 1, a.ob = static_cast<long long>(g.HW) * g.K;
  a.eps = eps, a.bf3 = bf3;
  st = act_kind == PROTOSEG_ACT_LOG ? gemm<kEpiStore, float, float, 0, -1, float>(a, B * S, s)
                                    : gemm<kEpiStore, float, float, 1, -1, float>(a, B * S, s);
  if (st || S == 1) return st;
  const long long e = static_cast<long long>(g.npix) * g.K;
  hipLaunchKernelGGL(wide_finish_kernel, dim3(static_cast<unsigned>(ceil_div(e, 256))), dim3(256), 0, s, part, S, B,
                     g.HW, g.K, 0, nullptr, nullptr, logits, static_cast<long long>(g.K),
                     static_cast<long long>(g.HW) * g.K);
  return check_launch("wide_finish_kernel");
}

namespace {
#ifndef WIDE_PRE
#define WIDE_PRE 1  // the pre-split backward GEMMs (0: the 64 x 64 bf16x3 tile, for A/B)
#endif
// grid: ceil(N / 128) column tiles x ceil(M / (64 MI)) row tiles x ksplit
template <int EPI, bool BT, typename TO, int MI>
int pre_gemm_mi(const PreArgs& a, hipStream_t s) {
  if (int e = ensure_lds<wide_pre_gemm_kernel<EPI, BT, TO, MI>, pre_lds(MI)>()) return e;
  KernelTimer timer(EPI == 0 ? "wide_pre_gp_kernel" : "wide_pre_gx_kernel", s);
  const dim3 grid(static_cast<unsigned>(ceil_div(a.N, kPreTN)), static_cast<unsigned>(ceil_div(a.M, pre_tm(MI))),
                  static_cast<unsigned>(a.ksplit));
  hipLaunchKernelGGL((wide_pre_gemm_kernel<EPI, BT, TO, MI>), grid, dim3(256), pre_lds(MI), s, a);
  return check_launch("wide_pre_gemm_kernel");
}
template <int EPI, bool BT, typename TO>
int pre_gemm(const PreArgs& a, int MI, hipStream_t s) {
  return MI == 4 ? pre_gemm_mi<EPI, BT, TO, 4>(a, s) : pre_gemm_mi<EPI, BT, TO, 3>(a, s);
}

// The wide backward on pre-split operands: G_s as bf16 planes (kEpiGsSplit), then g_x and g_P on
// wide_pre_gemm_kernel, g_W on the 64 x 64 tile (M = K classes is small).
int launch_bwd_wide_pre(const Geometry& g, int x_dtype, const void* x, const float* protos, const float* w_last,
                        float eps, int act_kind, const float* g_logits, const float* g_dist, void* g_x, float* g_protos,
                        float* g_w, float* ws, const WideBwdLayout& l, const float* D, hipStream_t s) {
  const int B = g.npix / g.HW;
  const long long img = static_cast<long long>(g.P) * g.HW;
  const size_t dp = static_cast<size_t>(g.npix) * g.P;
  uint16_t* gh = reinterpret_cast<uint16_t*>(ws + l.G);
  uint16_t* gl = gh + dp;
  int st = PROTOSEG_OK;
  {  // G_s as two bf16 planes [B][P][HW]
    WideArgs a{};
    a.A = op(w_last, 1, g.ldw, 0);
    a.B = op(g_logits, g.K, 1, static_cast<long long>(g.HW) * g.K);
    a.M = g.P, a.N = g.HW, a.Kd = g_logits ? g.K : 0, a.nb = B;
    a.out = gh, a.out2 = gl, a.om = g.HW, a.on = 1, a.ob = img;
    a.eps = eps, a.act_kind = act_kind, a.D = D, a.gd = g_dist, a.bf3 = 1;
    if ((st = gemm<kEpiGsSplit, float, float, -1, -1, float>(a, B, s))) return st;
  }
  if (g_x) {  // g_x[b][c][n] = -2 sum_p P[p][c] G_s[b][p][n] + 2 x sum_p G_s
    const int kp = static_cast<int>(ceil_div(g.P, kPreTK)) * kPreTK;
    uint16_t* ph = reinterpret_cast<uint16_t*>(ws + l.pt);
    uint16_t* pl = ph + static_cast<size_t>(g.C) * kp;
    hipLaunchKernelGGL(wide_pt_split_kernel, dim3(static_cast<unsigned>(ceil_div(kp, 64)), static_cast<unsigned>(ceil_div(g.C, 64))),
                       dim3(256), 0, s, protos, g.P, g.C, kp, ph, pl);
    if ((st = check_launch("wide_pt_split_kernel"))) return st;
    PreArgs a{};
    a.ahi = ph, a.alo = pl, a.a_bytes = static_cast<unsigned>(static_cast<size_t>(g.C) * kp * 2);
    a.sab = 0, a.lda = kp, a.akb = kp, a.arows = g.C;
    a.bhi = gh, a.blo = gl, a.b_bytes = static_cast<unsigned>(dp * 2);
    a.sbb = img, a.ldb = g.HW, a.bcols = g.npix, a.bnb = g.HW, a.bk = g.P;
    a.M = g.C, a.N = g.npix, a.K = kp, a.ksplit = 1;
    a.gx = g_x, a.x = x, a.C = g.C, a.HW = g.HW;
    const int mi = pre_mi(g.C, ceil_div(g.npix, kPreTN));
    if (x_dtype == PROTOSEG_BF16) {
      a.o_bytes = static_cast<unsigned>(static_cast<size_t>(g.npix) * g.C * 2);
      st = pre_gemm<1, true, uint16_t>(a, mi, s);
    } else if (x_dtype == PROTOSEG_F16) {
      a.o_bytes = static_cast<unsigned>(static_cast<size_t>(g.npix) * g.C * 2);
      st = pre_gemm<1, true, _Float16>(a, mi, s);
    } else {
      a.o_bytes = static_cast<unsigned>(static_cast<size_t>(g.npix) * g.C * 4);
      st = pre_gemm<1, true, float>(a, mi, s);
    }
    if (st) return st;
  }
  if (g_protos) {  // g_P[p][c] = -2 sum_{b,n} G_s[b][p][n] x[b][c][n] + 2 p rs[p]
    float* rs = ws + l.rs;
    hipLaunchKernelGGL(wide_rowsum_split_kernel, dim3(static_cast<unsigned>(g.P)), dim3(256), 0, s, gh, gl, g.P, g.HW, B, rs);
    if ((st = check_launch("wide_rowsum_split_kernel"))) return st;
    uint16_t* xh = reinterpret_cast<uint16_t*>(ws + l.xs);
    uint16_t* xl = xh + static_cast<size_t>(g.npix) * g.C;
    const long long nx = static_cast<long long>(g.npix) * g.C;
    const unsigned xg = static_cast<unsigned>(ceil_div(nx, 256) < 4096 ? ceil_div(nx, 256) : 4096);
    if (x_dtype == PROTOSEG_BF16)
      hipLaunchKernelGGL(wide_x_split_kernel<uint16_t>, dim3(xg), dim3(256), 0, s, static_cast<const uint16_t*>(x), nx, xh, xl);
    else if (x_dtype == PROTOSEG_F16)
      hipLaunchKernelGGL(wide_x_split_kernel<_Float16>, dim3(xg), dim3(256), 0, s, static_cast<const _Float16*>(x), nx, xh, xl);
    else
      hipLaunchKernelGGL(wide_x_split_kernel<float>, dim3(xg), dim3(256), 0, s, static_cast<const float*>(x), nx, xh, xl);
    if ((st = check_launch("wide_x_split_kernel"))) return st;
    const int S = pre_split(g);
    float* part = ws + l.part;
    PreArgs a{};
    a.ahi = gh, a.alo = gl, a.a_bytes = static_cast<unsigned>(dp * 2);
    a.sab = img, a.lda = g.HW, a.akb = g.HW, a.arows = g.P;
    a.bhi = xh, a.blo = xl, a.b_bytes = static_cast<unsigned>(nx * 2);
    a.sbb = static_cast<long long>(g.C) * g.HW, a.ldb = g.HW, a.bkb = g.HW, a.bcols = g.C;
    a.M = g.P, a.N = g.C, a.K = g.npix, a.ksplit = S;
    a.slab = part;
    if ((st = pre_gemm<0, false, float>(a, 3, s))) return st;  // 3: pre_split's tile count
    const long long e = static_cast<long long>(g.P) * g.C;
    hipLaunchKernelGGL(wide_finish_kernel, dim3(static_cast<unsigned>(ceil_div(e, 256))), dim3(256), 0, s, part, S, 1,
                       g.P, g.C, 1, protos, rs, g_protos, static_cast<long long>(g.C), 0LL);
    if ((st = check_launch("wide_finish_kernel"))) return st;
  }
  if (g_w && g_logits) {  // g_W[k][p] = sum_{b,n} GL[b][n][k] act(D[b][p][n]) (64 x 64 tile)
    const int S = split_of(g.K, g.P, g.npix);
    float* part = ws + l.part;
    WideArgs a{};
    a.A = op(g_logits, 1, g.K, static_cast<long long>(g.HW) * g.K);
    a.B = op(D, g.HW, 1, img);
    a.M = g.K, a.N = g.P, a.Kd = g.HW, a.nb = B, a.bk = 1, a.ksplit = S;
    a.out = part, a.om = g.P, a.on = 1, a.ob = static_cast<long long>(g.K) * g.P;
    a.eps = eps, a.bf3 = 1;
    st = act_kind == PROTOSEG_ACT_LOG ? gemm<kEpiStore, float, float, -1, 0, float>(a, S, s)
                                      : gemm<kEpiStore, float, float, -1, 1, float>(a, S, s);
    if (st) return st;
    const long long e = static_cast<long long>(g.K) * g.P;
    hipLaunchKernelGGL(wide_finish_kernel, dim3(static_cast<unsigned>(ceil_div(e, 256))), dim3(256), 0, s, part, S, 1,
                       g.K, g.P, 0, nullptr, nullptr, g_w, static_cast<long long>(g.ldw), 0LL);
    if ((st = check_launch("wide_finish_kernel"))) return st;
  }
  return PROTOSEG_OK;
}
}  // namespace

int launch_bwd_wide(const Geometry& g, int x_dtype, const void* x, const float* protos, const float* w_last, float eps,
                    int act_kind, const float* g_logits, const float* g_dist, void* g_x, float* g_protos, float* g_w,
                    void* workspace, hipStream_t s, int bf3, const float* dist_saved) {
  const WideBwdLayout l = wide_bwd_layout(g);
  float* ws = static_cast<float*>(workspace);
  float *D = ws + l.D, *G = ws + l.G, *rs = ws + l.rs;
  float* part = ws + l.part;
  const int B = g.npix / g.HW;
  const long long img = static_cast<long long>(g.P) * g.HW;
  int st = PROTOSEG_OK;
  if (dist_saved) D = const_cast<float*>(dist_saved);  // read-only below (G_s epilogue, g_W operand)
  else if ((st = distances_of(g, x_dtype, x, protos, eps, act_kind, D, nullptr, s, bf3))) return st;
  if (bf3 && WIDE_PRE && wide_pre_fits(g))
    return launch_bwd_wide_pre(g, x_dtype, x, protos, w_last, eps, act_kind, g_logits, g_dist, g_x, g_protos, g_w,
                               ws, l, D, s);
  {  // G_s[b][p][n] = (sum_k W[k][p] GL[b][n][k]) act'(D) + g_dist, relu mask (K = 0: g_dist alone)
    WideArgs a{};
    a.A = op(w_last, 1, g.ldw, 0);                               // (p, k) of W[k][p]
    a.B = op(g_logits, g.K, 1, static_cast<long long>(g.HW) * g.K);  // (n, k) of GL[b][n][k]
    a.M = g.P, a.N = g.HW, a.Kd = g_logits ? g.K : 0, a.nb = B;
    a.out = G, a.om = g.HW, a.on = 1, a.ob = img;
    a.eps = eps, a.act_kind = act_kind, a.D = D, a.gd = g_dist, a.bf3 = bf3;
    if ((st = gemm<kEpiGs, float, float, -1, -1, float>(a, B, s))) return st;
  }
  if (g_x) {  // g_x[b][c][n] = -2 sum_p P[p][c] G_s[b][p][n] + 2 x cs[b][n]
    WideArgs a{};
    a.A = op(protos, 1, g.C, 0);          // (c, p) of P[p][c]
    a.B = op(G, 1, g.HW, img);            // (n, p) of G_s[b][p][n]
    a.M = g.C, a.N = g.HW, a.Kd = g.P, a.nb = B;
    a.bf3 = bf3;
    const int Sx = gx_split(g);
    if (Sx > 1) {  // split over the prototypes: slabs [B][Sx][C][HW], then the epilogue in the finish
      float* cs = ws + l.cs;
      hipLaunchKernelGGL(wide_colsum_kernel, dim3(static_cast<unsigned>(ceil_div(g.npix, 32)), kColsumQ), dim3(256), 0, s, G,
                         g.P, g.HW, g.npix, cs);
      if ((st = check_launch("wide_colsum_kernel"))) return st;
      a.ksplit = Sx;
      a.out = part, a.om = g.HW, a.on = 1, a.ob = static_cast<long long>(g.C) * g.HW;
      if ((st = gemm<kEpiStore, float, float, -1, -1, float>(a, B * Sx, s))) return st;
      const unsigned fg = static_cast<unsigned>(ceil_div(static_cast<long long>(g.npix) * g.C, 256));
      if (x_dtype == PROTOSEG_BF16)
        hipLaunchKernelGGL(wide_finish_gx_kernel<uint16_t>, dim3(fg), dim3(256), 0, s, part, Sx, B, g.C, g.HW,
                           static_cast<const uint16_t*>(x), cs, static_cast<uint16_t*>(g_x));
      else if (x_dtype == PROTOSEG_F16)
        hipLaunchKernelGGL(wide_finish_gx_kernel<_Float16>, dim3(fg), dim3(256), 0, s, part, Sx, B, g.C, g.HW,
                           static_cast<const _Float16*>(x), cs, static_cast<_Float16*>(g_x));
      else
        hipLaunchKernelGGL(wide_finish_gx_kernel<float>, dim3(fg), dim3(256), 0, s, part, Sx, B, g.C, g.HW,
                           static_cast<const float*>(x), cs, static_cast<float*>(g_x));
      if ((st = check_launch("wide_finish_gx_kernel"))) return st;
    } else {
      a.out = g_x, a.om = g.HW, a.on = 1, a.ob = static_cast<long long>(g.C) * g.HW;
      a.xo = x;
      st = x_dtype == PROTOSEG_BF16  ? gemm<kEpiGx, float, float, -1, -1, uint16_t>(a, B, s)
           : x_dtype == PROTOSEG_F16 ? gemm<kEpiGx, float, float, -1, -1, _Float16>(a, B, s)
                                     : gemm<kEpiGx, float, float, -1, -1, float>(a, B, s);
      if (st) return st;
    }
  }
  if (g_protos) {  // g_P[p][c] = -2 sum_{b,n} G_s[b][p][n] x[b][c][n] + 2 p rs[p]
    hipLaunchKernelGGL(wide_rowsum_kernel, dim3(static_cast<unsigned>(g.P)), dim3(256), 0, s, G, g.P, g.HW, B, rs);
    if ((st = check_launch("wide_rowsum_kernel"))) return st;
    const int S = split_of(g.P, g.C, g.npix);
    WideArgs a{};
    a.A = op(G, g.HW, 1, img);                                        // (p, n) of G_s[b][p][n]
    a.B = op(x, g.HW, 1, static_cast<long long>(g.C) * g.HW);         // (c, n) of X[b][c][n]
    a.M = g.P, a.N = g.C, a.Kd = g.HW, a.nb = B, a.bk = 1, a.ksplit = S;
    a.out = part, a.om = g.C, a.on = 1, a.ob = static_cast<long long>(g.P) * g.C;
    a.bf3 = bf3;
    st = x_dtype == PROTOSEG_BF16  ? gemm<kEpiStore, float, uint16_t, -1, -1, float>(a, S, s)
         : x_dtype == PROTOSEG_F16 ? gemm<kEpiStore, float, _Float16, -1, -1, float>(a, S, s)
                                   : gemm<kEpiStore, float, float, -1, -1, float>(a, S, s);
    if (st) return st;
    const long long e = static_cast<long long>(g.P) * g.C;
    hipLaunchKernelGGL(wide_finish_kernel, dim3(static_cast<unsigned>(ceil_div(e, 256))), dim3(256), 0, s, part, S, 1,
                       g.P, g.C, 1, protos, rs, g_protos, static_cast<long long>(g.C), 0LL);
    if ((st = check_launch("wide_finish_kernel"))) return st;
  }
  if (g_w && g_logits) {  // g_W[k][p] = sum_{b,n} GL[b][n][k] act(D[b][p][n])
    const int S = split_of(g.K, g.P, g.npix);
    WideArgs a{};
    a.A = op(g_logits, 1, g.K, static_cast<long long>(g.HW) * g.K);  // (k, n) of GL[b][n][k]
    a.B = op(D, g.HW, 1, img);                                       // (p, n) of D[b][p][n], act on load
    a.M = g.K, a.N = g.P, a.Kd = g.HW, a.nb = B, a.bk = 1, a.ksplit = S;
    a.out = part, a.om = g.P, a.on = 1, a.ob = static_cast<long long>(g.K) * g.P;
    a.eps = eps, a.bf3 = bf3;
    st = act_kind == PROTOSEG_ACT_LOG ? gemm<kEpiStore, float, float, -1, 0, float>(a, S, s)
                                      : gemm<kEpiStore, float, float, -1, 1, float>(a, S, s);
    if (st) return st;
    const long long e = static_cast<long long>(g.K) * g.P;
    hipLaunchKernelGGL(wide_finish_kernel, dim3(static_cast<unsigned>(ceil_div(e, 256))), dim3(256), 0, s, part, S, 1,
                       g.K, g.P, 0, nullptr, nullptr, g_w, static_cast<long long>(g.ldw), 0LL);
    if ((st = check_launch("wide_finish_kernel"))) return st;
  }
  return PROTOSEG_OK;
}

namespace {

// Grow-only scratch per (device, stream) for the wide push path (stream_scratch).
void* wide_scratch(size_t need, hipStream_t s, int* st) {
  void* p = nullptr;
  *st = stream_scratch(ScratchKind::kWidePush, need, 0, s, &p);
  return p;
}

// One wave per (prototype, image): the masked minimum over the class patches as a key
// (float_bits(d) << 32 | patch: the lowest patch wins an exact tie) and the runner-up distance
// over the other class patches (protoseg_push_argmin's contract).
__global__ __launch_bounds__(256) void wide_push_argmin_kernel(const float* __restrict__ dist, int P, int hw,
                                                               const int32_t* __restrict__ proto_class,
                                                               const uint32_t* __restrict__ mask, size_t plane, int words,
                                                               unsigned long long* __restrict__ keys,
                                                               unsigned long long* __restrict__ second) {
  const int lane = threadIdx.x & 63;
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6), i = blockIdx.y;
  if (p >= P) return;
  const int pc = proto_class[p];
  const unsigned long long kNone = ~0ull;
  unsigned long long best = kNone;
  unsigned sec = 0xFFFFFFFFu;  // runner-up distance bits (d >= 0: bits order like values)
  if (pc >= 0 && (pc >> 5) < words) {
    const float* d = dist + (static_cast<size_t>(i) * P + p) * hw;
    const uint32_t* mk = mask + static_cast<size_t>(pc >> 5) * plane + static_cast<size_t>(i) * hw;  // word of the class
    for (int n = lane; n < hw; n += 64) {
      if (!((mk[n] >> (pc & 31)) & 1u)) continue;
      const unsigned long long k = (static_cast<unsigned long long>(__float_as_uint(d[n])) << 32) | static_cast<unsigned>(n);
      if (k < best) {
        const unsigned ob = static_cast<unsigned>(best >> 32);
        sec = best == kNone ? sec : (ob < sec ? ob : sec);
        best = k;
      } else {
        const unsigned kb = static_cast<unsigned>(k >> 32);
        sec = kb < sec ? kb : sec;
      }
    }
  }
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {  // merge (best, runner-up) pairs across lanes
    const unsigned long long ob = shfl_xor_u64(best, m);
    const unsigned os = __shfl_xor(sec, m);
    const unsigned long long lo = ob < best ? ob : best, hi = ob < best ? best : ob;
    const unsigned hb = hi == kNone ? 0xFFFFFFFFu : static_cast<unsigned>(hi >> 32);
    unsigned s2 = sec < os ? sec : os;
    s2 = hb < s2 ? hb : s2;
    best = lo;
    sec = s2;
  }
  if (lane == 0) {
    keys[static_cast<size_t>(i) * P + p] = best;
    if (second)
      second[static_cast<size_t>(i) * P + p] =
          sec == 0xFFFFFFFFu ? kNone : ((static_cast<unsigned long long>(sec) << 32) | 0xFFFFFFFFull);
  }
}

}  // namespace

// Distances of n_img images [n_img][P][hw] (the push's wide-C path).
int wide_push_distances(const float* x, int n_img, int C, int hw, const float* protos, int P, float* dist,
                        hipStream_t s) {
  Geometry g{};
  g.C = C, g.P = P, g.K = 0, g.HW = hw, g.npix = n_img * hw;
  return wide_distances(g, x, protos, 1e-4f, PROTOSEG_ACT_LOG, dist, nullptr, s);
}

int wide_push_distances_scratch(const float* x, int C, int hw, const float* protos, int m, float* dist, hipStream_t s) {
  return wide_push_distances(x, 1, C, hw, protos, m, dist, s);
}

int wide_push_argmin(const float* x, int n_img, int C, int hw, const float* protos, int P, const int32_t* proto_class,
                     const uint32_t* mask, int words, uint64_t* img_keys, uint64_t* img_second, hipStream_t s) {
  // images per pass: the pass's distances within ~1 GiB of scratch
  const size_t per_img = static_cast<size_t>(P) * hw;
  int nb = static_cast<int>((static_cast<size_t>(1) << 28) / (per_img ? per_img : 1));
  if (nb < 1) nb = 1;
  if (nb > n_img) nb = n_img;
  int st = PROTOSEG_OK;
  float* D = static_cast<float*>(wide_scratch((per_img * nb + 256) * sizeof(float), s, &st));
  if (st) return st;
  for (int i0 = 0; i0 < n_img; i0 += nb) {
    const int ni = n_img - i0 < nb ? n_img - i0 : nb;
    if ((st = wide_push_distances(x + static_cast<size_t>(i0) * C * hw, ni, C, hw, protos, P, D, s))) return st;
    // mask planes [words][n_img][hw]: class c in word c >> 5
    hipLaunchKernelGGL(wide_push_argmin_kernel, dim3(static_cast<unsigned>(ceil_div(P, 4)), ni), dim3(256), 0, s, D, P,
                       hw, proto_class, mask + static_cast<size_t>(i0) * hw, static_cast<size_t>(n_img) * hw, words,
                       reinterpret_cast<unsigned long long*>(img_keys) + static_cast<size_t>(i0) * P,
                       img_second ? reinterpret_cast<unsigned long long*>(img_second) + static_cast<size_t>(i0) * P
                                  : nullptr);
    if ((st = check_launch("wide_push_argmin_kernel"))) return st;
  }
  return PROTOSEG_OK;
}

}  // namespace protoseg
