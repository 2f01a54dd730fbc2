// adam.hip — the optimizer step of the layer's training step on gfx950: torch.optim.Adam
// (reference segmentation/module.py:391, `torch.optim.Adam(optimizer_specs)`: amsgrad off,
// maximize off, L2 weight decay per group) over up to kAdamMaxTensors f32 tensors in ONE launch.
//
//   g  = grad + wd * p                      (wd != 0)
//   m  = b1 m + (1 - b1) g                  v = b2 v + (1 - b2) g g
//   p -= (lr / (1 - b1^t)) m / (sqrt(v) / sqrt(1 - b2^t) + eps)
//
// the arithmetic of torch's fused Adam (f32, bias corrections from the step count t). Each tensor
// has its own step count on the device (state[k][0]; torch keeps state[p]['step'] per parameter),
// so the update can be captured in a HIP graph and replayed: every workgroup of tensor k reads
// t = state[k][0] + 1 at its start; the last of tensor k's workgroups to finish (ticket in
// state[k][1], a vector atomic) stores t and resets the ticket, after all of them have read it.
// A tensor with no elements gets one workgroup, which only advances its count.
#include "adam_update.h"
#include "protoseg_host.h"

namespace protoseg {

namespace {

constexpr int kAdamMaxTensors = 8;
constexpr int kAdamBlock = 256;
constexpr int kAdamPerThread = 4;

struct AdamTensors {
  float* p[kAdamMaxTensors];
  const float* g[kAdamMaxTensors];
  float* m[kAdamMaxTensors];
  float* v[kAdamMaxTensors];
  int* st[kAdamMaxTensors];
  long long n[kAdamMaxTensors];
  long long first_block[kAdamMaxTensors + 1];  // prefix sum of the tensors' workgroup counts
  int count;
};

__global__ __launch_bounds__(kAdamBlock) void adam_kernel(AdamTensors ts, float lr,
                                                          float beta1, float beta2, float eps, float wd) {
  __shared__ int last, t_sh;
  __shared__ float corr[2];
  const long long blk = blockIdx.x;
  int k = 0;
  while (k + 1 < ts.count && blk >= ts.first_block[k + 1]) ++k;
  const long long base = (blk - ts.first_block[k]) * (kAdamBlock * kAdamPerThread);
  float* __restrict__ p = ts.p[k];
  const float* __restrict__ g = ts.g[k];
  float* __restrict__ m = ts.m[k];
  float* __restrict__ v = ts.v[k];
  int* __restrict__ state = ts.st[k];
  const int nblk = static_cast<int>(ts.first_block[k + 1] - ts.first_block[k]);
  // the element loads go out with the step-count load (one memory round trip, not two)
  float gi[kAdamPerThread], pi[kAdamPerThread], mi[kAdamPerThread], vi[kAdamPerThread];
#pragma unroll
  for (int r = 0; r < kAdamPerThread; ++r) {
    const long long i = base + r * kAdamBlock + threadIdx.x;
    const bool ok = i < ts.n[k];
    gi[r] = ok ? g[i] : 0.f;
    pi[r] = ok ? p[i] : 0.f;
    mi[r] = ok ? m[i] : 0.f;
    vi[r] = ok ? v[i] : 0.f;
  }
  if (threadIdx.x == 0) {  // bias corrections once per workgroup (adam_update.h)
    const AdamCorr ac = adam_corr(state, lr, beta1, beta2);
    t_sh = ac.t;
    corr[0] = ac.step_size;
    corr[1] = ac.bc2_sqrt;
  }
  __syncthreads();
  const int t = t_sh;
  const float step_size = corr[0], bc2_sqrt = corr[1];
#pragma unroll
  for (int r = 0; r < kAdamPerThread; ++r) {
    const long long i = base + r * kAdamBlock + threadIdx.x;
    if (i < ts.n[k]) {
      adam_update(pi[r], mi[r], vi[r], gi[r], step_size, bc2_sqrt, beta1, beta2, eps, wd);
      m[i] = mi[r];
      v[i] = vi[r];
      p[i] = pi[r];
    }
  }
  // Step count: the last workgroup to arrive publishes t (all reads of state[0] are done by then:
  // each workgroup's read returned before its ticket, so no fence is needed — a device-scope
  // release here wrote back the XCD's L2 once per workgroup, ~30 ns each, serialised).
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(state + 1, 1) == nblk - 1;
  __syncthreads();
  if (last && threadIdx.x == 0) {
    atomicExch(state, t);
    atomicExch(state + 1, 0);
  }
}

}  // namespace

}  // namespace protoseg

using namespace protoseg;

extern "C" int protoseg_adam_step(int n_tensors, float* const* params, const float* const* grads,
                                  float* const* exp_avg, float* const* exp_avg_sq, const int64_t* numel,
                                  int32_t* const* state, float lr, float beta1, float beta2, float eps, float weight_decay,
                                  protoseg_stream_t stream) {
  if (n_tensors <= 0 || n_tensors > kAdamMaxTensors)
    return fail(PROTOSEG_ERR_INVALID, "n_tensors %d (1..%d)", n_tensors, kAdamMaxTensors);
  if (!params || !grads || !exp_avg || !exp_avg_sq || !numel || !state)
    return fail(PROTOSEG_ERR_INVALID, "pointer arrays and state must be non-null");
  if (!(beta1 >= 0.f && beta1 < 1.f && beta2 >= 0.f && beta2 < 1.f && eps >= 0.f))
    return fail(PROTOSEG_ERR_INVALID, "betas in [0, 1), eps >= 0");
  AdamTensors ts{};
  ts.count = n_tensors;
  long long blocks = 0;
  for (int k = 0; k < n_tensors; ++k) {
    if (numel[k] < 0 || !state[k] || (numel[k] > 0 && (!params[k] || !grads[k] || !exp_avg[k] || !exp_avg_sq[k])))
      return fail(PROTOSEG_ERR_INVALID, "tensor %d: null pointer or negative numel", k);
    ts.st[k] = state[k];
    ts.p[k] = params[k];
    ts.g[k] = grads[k];
    ts.m[k] = exp_avg[k];
    ts.v[k] = exp_avg_sq[k];
    ts.n[k] = numel[k];
    ts.first_block[k] = blocks;
    const long long nb = ceil_div(numel[k], kAdamBlock * kAdamPerThread);
    blocks += nb > 0 ? nb : 1;  // numel 0: one workgroup that advances the step count
  }
  ts.first_block[n_tensors] = blocks;
  if (blocks >= (1LL << 31)) return fail(PROTOSEG_ERR_UNSUPPORTED, "too many elements");
  hipLaunchKernelGGL(adam_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kAdamBlock), 0,
                     reinterpret_cast<hipStream_t>(stream), ts, lr, beta1, beta2, eps, weight_decay);
  return check_launch("adam_kernel");
}
