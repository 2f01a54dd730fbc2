// l2_launch.h — internal interface between the C ABI (l2_layer.hip) and the two kernel
// families of the prototype layer: exact f32-MFMA (l2_layer.hip) and bf16 split-MFMA
// (l2_bf16.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace protoseg {

// The KLD loss's distance gradient in its compact layout (kld.hip, protoseg_l2_bwd_kld): at
// global pixel g and prototype p, g_dist = val[g * mpc + (slot[p] & 255)] when pix[g] ==
// slot[p] >> 8, else 0. `slot` is indexed by the whole call's prototype (a chunk adds its p0).
struct CompactGd {
  const float* val = nullptr;  // [npix, mpc] f32
  const int* pix = nullptr;    // [npix] int32: class of the pixel's contributing group, or -1
  const int* slot = nullptr;   // [P] int32: class * 256 + position in the class
  int mpc = 0;
};

struct Geometry {
  int C, P, Pp, K, HW;
  int npix, ntiles;  // B*H*W pixels, 32-pixel tiles
  int ldw = 0;       // row stride of w_last / g_w (= P, or the full P for a prototype chunk)
  int ldd = 0, p0 = 0;  // g_dist: prototypes per image (= P, or the full P) and the chunk's first
  int xsig = 0;         // x is the add-on's pre-activation: sigmoid on load (bf16 fwd + fused bwd)
  CompactGd cgd;        // cgd.val != nullptr: the compact KLD gradient instead of a dense g_dist
  const float* protos = nullptr;  // wave backward: the chunk's prototype rows (2 p sum_n g_s in its slab)
};

// bf16 split family (C = 64). `terms` = 2 (3 products) or 3 (6 products).
bool bf16_fwd_fits(const Geometry& g, int terms);
// Every [npix, max(P, C)] f32 buffer below 2^31 bytes (buffer-resource offsets are 32-bit).
bool bf16_sizes_ok(const Geometry& g);
bool bf16_bwd_x_fits(const Geometry& g, int terms);
bool bf16_bwd_pw_fits(const Geometry& g, int terms);
size_t bf16_bwd_pw_workspace(const Geometry& g);

// Operand-image block (split P, P^T, W, W^T images and ||p||^2 in the kernels' LDS layout),
// built once per call by launch_prep_bf16 and shared by the kernels of that call.
size_t bf16_image_bytes(const Geometry& g, int terms);
// act_kind / eps select the constant factors folded into the W and W^T images (bf16_split.h).
// fwd_only: only the forward's images.
int launch_prep_bf16(const Geometry& g, int terms, const float* protos, const float* w_last, int act_kind, float eps,
                     void* img, hipStream_t stream, int fwd_only = 0);
// The images of nchunk prototype chunks of `per` rows (g.P rows in all, W columns at stride
// g.ldw) in one launch; chunk c's images at c * bf16_image_bytes(Pp(per)).
int launch_prep_bf16_chunks(const Geometry& g, int per, int nchunk, int terms, const float* protos,
                            const float* w_last, int act_kind, float eps, void* img, hipStream_t stream,
                            int fwd_only = 0);

// Adam step of the prototypes [P][64] and the last layer [K][P] (adam_update.h) fused with the
// operand prep of the updated values into `block` (launch_prep_bf16's bf16x3 block, fwd_only 0,
// one chunk); w and its state null iff K = 0. w_scale / wt_scale: act_unit / act_grad_unit.
struct AdamPrepArgs {
  float* p;
  const float* gp;
  float* mp;
  float* vp;
  int* stp;
  float* w;
  const float* gw;
  float* mw;
  float* vw;
  int* stw;
  int P, K;
  float lr_p, wd_p, lr_w, wd_w, beta1, beta2, eps;
  float w_scale, wt_scale;
  unsigned char* block;
};
int launch_adam_prep_bf16(const AdamPrepArgs& a, hipStream_t stream);

// accumulate != 0: logits += this call's (prototype chunks of one forward).
int launch_fwd_bf16(const Geometry& g, bool x_bf16, int terms, const void* x, const void* img, float eps, int act_kind,
                    float* dist, float* act, float* logits, hipStream_t stream,
                    int accumulate = 0);
// accumulate != 0: g_x += this call's gradient (prototype chunks of one backward).
int launch_bwd_x_bf16(const Geometry& g, bool x_bf16, int terms, const void* x, const void* img, float eps,
                      int act_kind, const float* g_logits, const float* g_dist, void* g_x, hipStream_t stream,
                      int accumulate = 0);
// One-kernel backward (l2_bwd_fused.hip): bf16x3 only, Pp <= 192 per launch; g_x (+= when
// accumulate), and the g_P / g_W slab in ws, summed by launch_bwd_reduce_bf16.
bool bf16_bwd_fused_fits(const Geometry& g, int terms);
// reduce = 0: the slab is left in ws for launch_bwd_reduce_bf16_chunks (one reduce per call).
int launch_bwd_fused_bf16(const Geometry& g, bool x_bf16, const void* x, const float* protos, const void* img,
                          float eps, int act_kind, const float* g_logits, const float* g_dist, void* g_x,
                          float* g_protos, float* g_w, float* ws, hipStream_t stream, int accumulate = 0,
                          int reduce = 1);
int bf16_bwd_fused_grid(const Geometry& g);
// Wave-owned backward (l2_bwd_wave.hip): bf16x3, P <= 384 per launch, 4 waves (one per SIMD)
// each owning a quarter of the prototypes for every product; reads the standard bf16 operand
// image block (launch_prep_bf16, bf16_image_bytes(P)); g_x (+= when accumulate) and a g_P / g_W
// slab per workgroup in the reduce kernel's layout with g_P transposed (gp_t = 1).
int bf16_wave_nb(int P);
bool bf16_bwd_wave_fits(const Geometry& g, int terms);
int bf16_bwd_wave_grid(const Geometry& g);
size_t bf16_bwd_wave_slab_elems(const Geometry& g);
int launch_bwd_wave_bf16(const Geometry& g, bool x_bf16, const void* x, const void* img, float eps, int act_kind,
                         const float* g_logits, const float* g_dist, void* g_x, float* ws, hipStream_t stream,
                         int accumulate = 0);
// Fixed-order sum of `slabs` partial slabs in ws (+ 2p sum g_s) into g_protos / g_w.
int launch_bwd_reduce_bf16(const Geometry& g, const float* ws, int slabs, const float* protos, int act_kind,
                           float* g_protos, float* g_w, hipStream_t stream);
// nchunk chunks of `per` prototypes (g.P in all, g_w columns at stride g.ldw); chunk c's slabs
// at ws + c * chunk_elems. gp_t: the slabs hold g_P transposed ([c][Pp], the wave kernel's).
int launch_bwd_reduce_bf16_chunks(const Geometry& g, int per, int nchunk, const float* ws, int slabs,
                                  size_t chunk_elems, const float* protos, int act_kind, float* g_protos, float* g_w,
                                  hipStream_t stream, int gp_t = 0);
int launch_bwd_pw_bf16(const Geometry& g, bool x_bf16, int terms, const void* x, const float* protos, const void* img,
                       float eps, int act_kind, const float* g_logits, const float* g_dist, float* g_protos,
                       float* g_w, float* ws, hipStream_t stream);

// Any C, any K (l2_wide.hip): exact f32 MFMA GEMMs with fused epilogues. Forward scratch: x2 / p2
// (+ the distances when dist is null and logits are wanted); backward workspace: D, G_s, sums and
// the split-K partial slabs.
bool wide_family_fits(const Geometry& g);
size_t wide_fwd_scratch_bytes(const Geometry& g, bool need_dist);
size_t wide_bwd_workspace_bytes(const Geometry& g);
int launch_fwd_wide(const Geometry& g, int x_dtype, const void* x, const float* protos, const float* w_last, float eps,
                    int act_kind, float* dist, float* act, float* logits, void* scratch, hipStream_t s,
                    int bf3);  // bf3: bf16x3 products (precision BF16X3), else exact f32
int launch_bwd_wide(const Geometry& g, int x_dtype, const void* x, const float* protos, const float* w_last, float eps,
                    int act_kind, const float* g_logits, const float* g_dist, void* g_x, float* g_protos, float* g_w,
                    void* workspace, hipStream_t s, int bf3,
                    const float* dist_saved = nullptr);  // the forward's distances: read, not recomputed
// The push's path for prototype depths push.hip does not hold (C outside {32, 64, 128}): the
// image's distances by the wide GEMM, then a masked argmin per (image, prototype) with
// protoseg_push_argmin's key contract; wide_push_distances_scratch = protoseg_push_distances.
int wide_push_argmin(const float* x, int n_img, int C, int hw, const float* protos, int P, const int32_t* proto_class,
                     const uint32_t* mask, int words, uint64_t* img_keys, uint64_t* img_second, hipStream_t s);
int wide_push_distances_scratch(const float* x, int C, int hw, const float* protos, int m, float* dist, hipStream_t s);

}  // namespace protoseg
