/*
 * protoseg_hip.h — C ABI of libprotoseg_hip.so, the MI355X (gfx950) hot path of ProtoSeg.
 *
 * The reference (tijaz17skane/ADLM-Inherently-Interpretable-Segmentation) has no native code:
 * every entry point below replaces a sequence of stock PyTorch ops or host Python loops.
 * The reference interface each one replaces is cited next to it (paths relative to the
 * reference root).
 *
 * Conventions (all entry points):
 *  - device pointers, plain integer shapes, a stream; no torch types;
 *  - tensors are dense, row-major, in the layouts stated per argument;
 *  - outputs are caller-allocated; temporary memory is the caller-owned workspace sized by the
 *    matching *_workspace_size() call, or the library's grow-only per-stream scratch (operand
 *    images, push masks / keys): allocated on a call's first use of a size and reused, never
 *    freed while the process runs, so once warm every call is kernel launches only (no sync,
 *    no allocation) and can be captured into a hipGraph;
 *  - return PROTOSEG_OK (0) or a protoseg_status code; protoseg_last_error() gives text;
 *  - reentrant: the only global state is a once-initialised per-kernel LDS attribute table.
 */
#ifndef PROTOSEG_HIP_H_
#define PROTOSEG_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same object as hipStream_t (struct ihipStream_t*); NULL = the legacy default stream. */
typedef struct ihipStream_t* protoseg_stream_t;

enum protoseg_status {
  PROTOSEG_OK = 0,
  PROTOSEG_ERR_INVALID = 1,      /* bad pointer / shape combination                      */
  PROTOSEG_ERR_UNSUPPORTED = 2,  /* valid request outside the compiled kernel family      */
  PROTOSEG_ERR_HIP = 3           /* a HIP runtime call or kernel launch failed            */
};

enum protoseg_dtype {
  PROTOSEG_F32 = 0,   /* float                                     */
  PROTOSEG_BF16 = 1,  /* bfloat16 bits in uint16_t                  */
  PROTOSEG_I64 = 2,   /* int64 labels (reference convert_targets)   */
  PROTOSEG_I32 = 3,
  PROTOSEG_U8 = 4,
  PROTOSEG_F16 = 5    /* IEEE half in uint16_t: feature maps of the wide family (fp16 add-on
                         output, BASELINE configs[4]); protoseg_l2_x_dtype_supported says where */
};

/* model.py:231-237 distance_2_similarity: 'log' -> log((d+1)/(d+eps)); 'linear' -> -d.
 * IDENTITY (protoseg_act_upsample only): the input already holds activations, e.g. from the
 * caller's prototype_activation_function_in_numpy (push.py:317-318). */
enum protoseg_act { PROTOSEG_ACT_LOG = 0, PROTOSEG_ACT_LINEAR = 1, PROTOSEG_ACT_IDENTITY = 2 };
/* Flag OR-ed into protoseg_l2_fwd / _bwd's act_kind: x is the add-on layers' pre-activation and
 * the kernels apply the add-on's final nn.Sigmoid on load (model.py:124-128, 164-175), so
 * sigmoid(x) is never materialised; the backward returns the gradient w.r.t. the pre-activation
 * (g_x * s (1 - s)). Served where protoseg_l2_x_sigmoid_supported() says so (BF16X3, C = 64),
 * PROTOSEG_ERR_UNSUPPORTED elsewhere. A backward with this flag always needs the workspace. */
enum { PROTOSEG_X_SIGMOID = 0x100 };
/* Flag OR-ed into protoseg_l2_fwd_ex's act_kind: `operands` already holds the images of these
 * protos / w_last (protoseg_l2_adam_prep wrote them with the step that produced the values, or an
 * earlier _ex forward on unchanged values), so the forward launches no prep. Needs a non-NULL
 * `operands` that protoseg_l2_train_operands_bytes sizes for the shape and protoseg_l2_adam_prep_supported;
 * PROTOSEG_ERR_INVALID otherwise. */
enum { PROTOSEG_OPERANDS_READY = 0x200 };

/* Arithmetic of the x.p / W.act / gradient products (always f32 accumulation):
 *  BF16X3  operands split in 2 bf16 terms, 3 bf16 MFMAs per product (|rel err| ~ 1e-5 on d)
 *  BF16X6  operands split in 3 bf16 terms, 6 bf16 MFMAs per product (f32-class)
 *  F32     v_mfma_f32_32x32x2_f32: an exact f32 fma chain
 * A request the bf16 family cannot serve (C != 64, LDS) runs on the F32 family. */
enum protoseg_precision { PROTOSEG_PREC_BF16X3 = 0, PROTOSEG_PREC_BF16X6 = 1, PROTOSEG_PREC_F32 = 2 };

int protoseg_version(void);                 /* MAJOR*10000 + MINOR*100 + PATCH */
const char* protoseg_last_error(void);      /* thread-local text of the last failure */

/* Measurement only (no reference counterpart): while set, every launch of the kernel named
 * `kernel` (e.g. "l2_bwd_pw_bf16_kernel") is bracketed by hipEventRecord(start_event) /
 * hipEventRecord(stop_event) on its launch stream, so a caller (bench.py) times that kernel
 * alone, as rocprofv3 does, instead of the whole call. The events are caller-owned
 * hipEvent_t handles; eager launches only (silent under graph capture). A null argument
 * clears the hook. */
int protoseg_timing_events(const char* kernel, void* start_event, void* stop_event);
/* `kernel` may also name a kernel family by prefix ("l2_fwd" matches l2_fwd_kernel and
 * l2_fwd_bf16_kernel); protoseg_timing_kernel() returns the full name of the last kernel the
 * hook bracketed ("" if none), i.e. which family served the call. */
const char* protoseg_timing_kernel(void);
/* Per-launch form: launch i (0 <= i < n) of the named kernel records start_events[i] /
 * stop_events[i], so a call that runs the kernel several times (prototype chunks) is timed
 * launch by launch, the durations rocprofv3 reports per dispatch (no span over the chunks'
 * prep / reduce launches). protoseg_timing_launches() returns how many pairs were recorded
 * since the hook was set or last queried, and resets that count. */
int protoseg_timing_events_n(const char* kernel, void* const* start_events, void* const* stop_events, int n);
int protoseg_timing_launches(void);

/*
 * Prototype layer forward. Replaces model.py:203-221 (_l2_convolution), 231-237
 * (distance_2_similarity) and 259-283 (forward_from_conv_features, patch-classification
 * branch: permute -> activation -> last_layer -> reshape), i.e. 2 conv2d + 9 elementwise
 * passes + 1 Linear, by one fused kernel.
 *
 *   x       [B, C, H, W]  x_dtype (PROTOSEG_F32 | PROTOSEG_BF16 | PROTOSEG_F16 where
 *                         protoseg_l2_x_dtype_supported), the add-on-layer output
 *   protos  [P, C]        f32 (prototype_vectors, 1x1 kernels flattened)
 *   w_last  [K, P]        f32 (last_layer.weight, no bias); may be NULL iff logits_out is NULL
 *   dist_out   [B, P, H, W]   f32 or NULL   distances (model.py:219, NCHW)
 *   act_out    [B*H*W, P]     f32 or NULL   prototype activations (model.py:273)
 *   logits_out [B, H, W, K]   f32 or NULL   logits NHWC (model.py:278)
 * Supported (protoseg_l2_supported() is authoritative):
 *   - K <= 32, P <= 4096, C = 64, BF16X3 / BF16X6: prototypes beyond one launch's LDS images run
 *     as prototype chunks inside the call (forward chunks of <= 384 rows at BF16X3, fewer at BF16X6);
 *   - K <= 32, P <= 4096, C in {32, 64, 128}, F32 (and the bf16 requests the bf16 family cannot
 *     serve, C != 64): the f32 family, over prototype chunks of what one launch's LDS holds;
 *   - any other C <= 4096, K <= 4096, P <= 65536 (e.g. the reference's default prototype_shape
 *     (2000, 512) with 200 classes, model.py:394), every precision request: the wide family
 *     (exact f32 MFMA GEMMs with fused epilogues, l2_wide.hip; scratch per stream, graph-safe);
 *   - every tensor addressed by the kernels (B*H*W*max(P, C)*4 bytes) below 2^31 bytes.
 */
int protoseg_l2_fwd(const void* x, int x_dtype, int B, int C, int H, int W,
                    const float* protos, int P, const float* w_last, int K,
                    float eps, int act_kind, int precision,
                    float* dist_out, float* act_out, float* logits_out,
                    protoseg_stream_t stream);

/*
 * Prototype layer backward: the autograd graph of model.py:203-221, 231-237, 266-278
 * (the reference has no custom backward). Distances are recomputed from x, never re-read.
 *
 *   g_logits [B, H, W, K] f32 or NULL   upstream grad of logits
 *   g_dist   [B, P, H, W] f32 or NULL   upstream grad of distances (KLD loss, module.py:167-208)
 *   g_x      [B, C, H, W] x_dtype or NULL
 *   g_protos [P, C] f32 or NULL   (overwritten, not accumulated)
 *   g_w      [K, P] f32 or NULL   (overwritten; requires g_logits)
 *   workspace: protoseg_l2_bwd_workspace_size(...) bytes, 256-B aligned.
 */
size_t protoseg_l2_bwd_workspace_size(int B, int C, int H, int W, int P, int K);
int protoseg_l2_bwd(const void* x, int x_dtype, int B, int C, int H, int W,
                    const float* protos, int P, const float* w_last, int K,
                    float eps, int act_kind, int precision,
                    const float* g_logits, const float* g_dist,
                    void* g_x, float* g_protos, float* g_w,
                    void* workspace, size_t workspace_bytes,
                    protoseg_stream_t stream);

/*
 * The same backward with the KLD loss's distance gradient in its compact layout
 * (protoseg_kld_backward_compact) instead of a dense [B, P, H, W] g_dist: the kernels expand
 * g_dist[b][p][n] = g_cls[g][proto_slot[p] & 255] where pix_cls[g] == proto_slot[p] >> 8
 * (g = b*H*W + n), 0 elsewhere, in registers. Same outputs as protoseg_l2_bwd given that dense
 * tensor (protoseg_kld_expand). Served by the bf16x3 training backward (g_x with g_protos /
 * g_w, C = 64, f32 x): protoseg_l2_bwd_kld_supported says whether a shape qualifies, otherwise
 * the call returns PROTOSEG_ERR_UNSUPPORTED before launching anything.
 *   g_cls      [B*H*W, max_per_class] f32
 *   pix_cls    [B*H*W] int32: class of the pixel's contributing (image, class) group, or -1
 *   proto_slot [P] int32: class * 256 + position of the prototype in its class
 */
int protoseg_l2_bwd_kld(const void* x, int x_dtype, int B, int C, int H, int W,
                        const float* protos, int P, const float* w_last, int K,
                        float eps, int act_kind, int precision,
                        const float* g_logits, const float* g_cls, const int32_t* pix_cls,
                        const int32_t* proto_slot, int max_per_class,
                        void* g_x, float* g_protos, float* g_w,
                        void* workspace, size_t workspace_bytes,
                        protoseg_stream_t stream);
int protoseg_l2_bwd_kld_supported(int B, int C, int H, int W, int P, int K, int x_dtype, int precision,
                                  int max_per_class);

/*
 * Backward kernel override of the bf16x3 training backward at C = 64 (measurement and tests):
 * "wave" (l2_bwd_wave.hip, 4 waves each owning a quarter of the prototypes), "fused"
 * (l2_bwd_fused.hip, P <= 192 per launch), or "" / NULL for the automatic choice (wave above 192
 * prototypes, fused below). The initial value is the PROTOSEG_BWD environment variable, read once.
 * Replaces nothing in the reference (its backward is autograd); process-wide.
 */
int protoseg_set_backward_kernel(const char* name);

/*
 * One operand prep per training step: the forward builds the backward's operand images (the
 * split P / W^T images and ||p||^2 in the backward kernel's layout) in the same prep launch as its
 * own, into a caller buffer the backward then reads instead of preparing them again.
 *   protoseg_l2_train_operands_bytes: the buffer size for (C, P, K, precision); 0 when the
 *     backward would not read one (it chunks prototypes, another family, not BF16X3): the _ex
 *     calls then ignore `operands` and behave as the plain calls.
 *   protoseg_l2_fwd_ex: protoseg_l2_fwd + fills `operands` (w_last non-NULL when K > 0; every
 *     output may be NULL to fill the operands only).
 *   protoseg_l2_bwd_ex / protoseg_l2_bwd_kld_ex: protoseg_l2_bwd / _kld reading `operands`
 *     (NULL: prepared inside the call). The caller guarantees that protos, w_last, P, K, C, eps,
 *     act_kind (X_SIGMOID aside) and precision are those of the forward that filled it, that its
 *     values are unchanged since, and that the backward kernel override (protoseg_set_backward_kernel)
 *     did not change.
 * Results are bit-identical to the plain calls (the same prep arithmetic, tests/test_gpu_operands.py).
 */
size_t protoseg_l2_train_operands_bytes(int C, int P, int K, int precision);
int protoseg_l2_fwd_ex(const void* x, int x_dtype, int B, int C, int H, int W,
                       const float* protos, int P, const float* w_last, int K,
                       float eps, int act_kind, int precision,
                       float* dist_out, float* act_out, float* logits_out,
                       void* operands, size_t operands_bytes, protoseg_stream_t stream);
int protoseg_l2_bwd_ex(const void* x, int x_dtype, int B, int C, int H, int W,
                       const float* protos, int P, const float* w_last, int K,
                       float eps, int act_kind, int precision,
                       const float* g_logits, const float* g_dist,
                       void* g_x, float* g_protos, float* g_w,
                       void* workspace, size_t workspace_bytes,
                       const void* operands, size_t operands_bytes, protoseg_stream_t stream);
/*
 * Backward reading the forward's distances instead of recomputing them, where that is cheaper:
 * the wide family (C outside {32, 64, 128}, K > 32 or P > 4096; e.g. BASELINE configs[4]'s
 * C = 1024), whose distance GEMM costs as much as the g_x one while the distances are a small
 * tensor. protoseg_l2_bwd_reads_dist says whether a shape reads `dist`; elsewhere the call is
 * protoseg_l2_bwd_ex (the C = 32 / 64 / 128 families recompute: at C = 64 reading the
 * [B, P, H, W] tensor costs more HBM time than the products). `dist` [B, P, H, W] f32 is the
 * dist_out of protoseg_l2_fwd on the same x, protos, eps, act_kind and precision (the backward's
 * own recompute gives the same bits, so the gradients are identical either way).
 */
int protoseg_l2_bwd_reads_dist(int C, int P, int K, int precision);
int protoseg_l2_bwd_saved(const void* x, int x_dtype, int B, int C, int H, int W,
                          const float* protos, int P, const float* w_last, int K,
                          float eps, int act_kind, int precision, const float* dist,
                          const float* g_logits, const float* g_dist,
                          void* g_x, float* g_protos, float* g_w,
                          void* workspace, size_t workspace_bytes, protoseg_stream_t stream);
int protoseg_l2_bwd_kld_ex(const void* x, int x_dtype, int B, int C, int H, int W,
                           const float* protos, int P, const float* w_last, int K,
                           float eps, int act_kind, int precision,
                           const float* g_logits, const float* g_cls, const int32_t* pix_cls,
                           const int32_t* proto_slot, int max_per_class,
                           void* g_x, float* g_protos, float* g_w,
                           void* workspace, size_t workspace_bytes,
                           const void* operands, size_t operands_bytes, protoseg_stream_t stream);


/* 1 if (C, P, K) is inside the compiled kernel family, else 0. */
int protoseg_l2_supported(int C, int P, int K);

/* 1 if protoseg_l2_fwd / _bwd read x (and write g_x) in x_dtype natively for (C, P, K), else 0:
 * F32 and BF16 everywhere protoseg_l2_supported; F16 in the wide family (no widening pass: the
 * GEMM stages convert on load, g_x is stored as fp16). */
int protoseg_l2_x_dtype_supported(int C, int P, int K, int x_dtype);

/* Largest P one protoseg_l2_fwd / _bwd call serves at (C, precision): 4096 (prototype chunks
 * inside the call, both families); 0 when C is outside the family or precision is unknown.
 * Callers holding more prototypes (push's bound-box distances) slice them into calls of at most
 * this many. */
int protoseg_l2_max_protos(int C, int precision);

/* 1 if protoseg_l2_fwd / _bwd accept PROTOSEG_X_SIGMOID for this shape and precision, else 0. */
int protoseg_l2_x_sigmoid_supported(int B, int C, int H, int W, int P, int K, int precision);

/*
 * Push, step 1: label map -> per-patch class bitmask. Replaces segmentation/push.py:184-186
 * (convert_targets via np.vectorize) and 214-223 (the per-pixel Python loop building
 * class_to_patch_index_dict). Pixel (i, j) of class c > 0 marks patch
 * (int(i / (H_img / h)), int(j / (W_img / w))) for class c-1, divisions in float64.
 *
 *   label  [n_img, H_img, W_img] label_dtype (PROTOSEG_I64 | PROTOSEG_I32 | PROTOSEG_U8)
 *   lut    [lut_size] int32 or NULL: label = lut[raw] (CITYSCAPES_19_EVAL_CATEGORIES etc.);
 *          raw values outside [0, lut_size) are ignored
 *   mask   [n_img, h, w] uint32: bit k set <=> a pixel of class k+1 falls in the patch
 * Classes above 32 are ignored (the reference would raise KeyError for class > num_classes).
 */
int protoseg_patch_class_mask(const void* label, int label_dtype, int n_img, int H_img, int W_img,
                              int h, int w, const int32_t* lut, int lut_size,
                              uint32_t* mask, protoseg_stream_t stream);
/* More than 32 classes (e.g. 200): `words` 32-bit mask planes, mask [words][n_img][h*w], plane wd
 * holding classes 32 wd + 1 .. 32 wd + 32 (bit k of plane wd <=> class 32 wd + k + 1).
 * words = 1 is protoseg_patch_class_mask. */
int protoseg_patch_class_mask_words(const void* label, int label_dtype, int n_img, int H_img, int W_img,
                                    int h, int w, const int32_t* lut, int lut_size, int words,
                                    uint32_t* mask, protoseg_stream_t stream);

/*
 * Push, step 2: for every image and prototype, the masked argmin of the distance over the
 * patches of the prototype's class. Replaces segmentation/push.py:193 + 209-263 (distances
 * for the whole image, D2H copy, per-prototype gather of class patches and np.argmin).
 * Distances are computed in-kernel (f32 MFMA, an exact f32 fma chain) with the reference's
 * rounding order for relu(||x||^2 + (||p||^2 - 2 x.p)), model.py:217-219.
 *
 *   x           [n_img, C, h, w] f32 (C in {32, 64, 128}: the fused kernel; other C: the wide path)
 *   proto_class [P] int32: argmax(prototype_class_identity[p]) (push.py:251); <0 = never pushed
 *   mask        [n_img, h*w] uint32 from protoseg_patch_class_mask
 *   img_keys    [n_img, P] uint64 out: (float_bits(d_min) << 32) | patch_index, or
 *               UINT64_MAX when the image holds no patch of the prototype's class.
 *   img_second  [n_img, P] uint64 out or NULL: the runner-up of the same image, as
 *               (float_bits(d_second) << 32) | 0xFFFFFFFF: the second-smallest distance over the
 *               class patches (another patch; equal to d_min on an exact tie), UINT64_MAX if
 *               the image holds fewer than two class patches.
 * Ties inside one image resolve to the lowest patch index here; the reference's order is the
 * iteration order of a Python set (push.py:214-230, 259-262), which the host restores for the
 * prototypes whose winning image holds an exact tie (img_second's distance == img_keys',
 * then protoseg_push_distances; protoseg_amd.push.resolve_exact_ties).
 * Scratch for the per-stripe partials is allocated once per (device, stream) and grows only by
 * a new block: blocks are never freed while the library is loaded, so a HIP graph that captured
 * an earlier call keeps valid pointers (an enlarged call must be captured again).
 */
int protoseg_push_argmin(const float* x, int n_img, int C, int h, int w,
                         const float* protos, int P, const int32_t* proto_class,
                         const uint32_t* mask, uint64_t* img_keys, uint64_t* img_second,
                         protoseg_stream_t stream);
/* The same with a protoseg_patch_class_mask_words mask of `words` planes (prototype class c reads
 * plane c >> 5). Prototype depths outside {32, 64, 128}, and every words > 1 call, take the wide
 * path: the image's distances by the exact-f32 GEMM of l2_wide.hip, then a masked top-2 per
 * (image, prototype), same key contract and tie rule (lowest patch index). */
int protoseg_push_argmin_words(const float* x, int n_img, int C, int h, int w,
                               const float* protos, int P, const int32_t* proto_class,
                               const uint32_t* mask, int words, uint64_t* img_keys, uint64_t* img_second,
                               protoseg_stream_t stream);

/*
 * Push, exact-tie resolution: distances of m prototypes at every patch of ONE image in
 * protoseg_push_argmin's arithmetic, operation for operation, so equal values here are exactly
 * the ties that kernel saw. The host then picks, among the class patches at the minimum, the
 * first in the reference's list(set) order (push.py:214-230 insertion order, np.argmin at
 * 259-262). Replaces the reference's proto_dist_[patch_i, patch_j, j] gather (push.py:259-260)
 * for those prototypes only.
 *   x      [C, h, w] f32 (one image); C outside {32, 64, 128}: the wide path's arithmetic
 *   protos [m, C] f32, 16-B aligned (the gathered prototypes)
 *   dist   [m, h*w] f32 out
 */
int protoseg_push_distances(const float* x, int C, int h, int w, const float* protos, int m, float* dist,
                            protoseg_stream_t stream);
/* protoseg_push_distances in protoseg_push_argmin_words' arithmetic for the same (C, words). */
int protoseg_push_distances_words(const float* x, int C, int h, int w, const float* protos, int m, int words,
                                  float* dist, protoseg_stream_t stream);

/*
 * Push, step 3: fold a batch of per-image keys into the running global minimum in image
 * order with a strict '<' (push.py:101, 265-281: earlier images win ties), and gather the
 * winning feature vector (push.py:276-280).
 *
 *   img_keys      [n_img, P] from protoseg_push_argmin on the same x
 *   img_second    [n_img, P] its runner-up keys, or NULL (then global_second must be NULL)
 *   first_img     dataset index of image 0 of this batch
 *   global_dist   [P] f32 in/out (init +inf)
 *   global_second [P] f32 in/out or NULL (init +inf): the second-smallest distance over every
 *                 class patch seen so far (any image), for near-tie flags
 *   global_img    [P] int64 in/out (init -1)
 *   global_patch  [P] int32 in/out (init -1)
 *   global_fmap   [P, C] f32 in/out
 */
int protoseg_push_merge(const uint64_t* img_keys, const uint64_t* img_second, int n_img, int64_t first_img,
                        const float* x, int C, int hw, int P,
                        float* global_dist, float* global_second, int64_t* global_img, int32_t* global_patch,
                        float* global_fmap, protoseg_stream_t stream);

/*
 * Steps 1-3 in one host call for one batch of equal-geometry images (push_prototypes' inner
 * step, push.py:184-281): protoseg_patch_class_mask_words -> protoseg_push_argmin_words ->
 * protoseg_push_merge, with the masks and per-image keys in library scratch on `stream`
 * (grow-only, one block per stream: capturable once it exists). Same results as the three calls;
 * global_second may be NULL (no runner-up tracking).
 */
int protoseg_push_update(const void* label, int label_dtype, int n_img, int H_img, int W_img,
                         const int32_t* lut, int lut_size, int words, const float* x, int C, int h, int w,
                         const float* protos, int P, const int32_t* proto_class, int64_t first_img,
                         float* global_dist, float* global_second, int64_t* global_img,
                         int32_t* global_patch, float* global_fmap, protoseg_stream_t stream);

/*
 * KLD similarity loss. Replaces segmentation/module.py:167-208 (the Python loop over images x
 * classes x prototype pairs: masked_select -> log_softmax -> two kl_div per pair -> mean of
 * exp(-kld)) and, in protoseg_kld_backward, its autograd. Semantics of the reference kept:
 * label value c selects the prototypes of class column c (void = 0 pairs with class 0, value
 * K is skipped, module.py:170-178); a class with < 2 prototypes or < 2 pixels adds no pair;
 * loss = 0 without pairs.
 *
 *   dist        [B, P, HW] f32: the distances of protoseg_l2_fwd (model.py:283, NCHW)
 *   label       [B, HW] label_dtype (PROTOSEG_I64 | I32 | U8): target_img of module.py:150
 *               (the resized label map before the void shift)
 *   proto_class [P] int32: class column of each prototype (argmax of prototype_class_identity;
 *               the identity is one-hot in the reference, model.py:66-71)
 *   K           num_classes (prototype_class_identity.shape[1]), K <= 63
 *   max_per_class  bound on prototypes per class, 1..32 (sizes LDS); a class holding more
 *               makes the loss NaN
 *   loss_out    [1] f32 device: mean over pairs of exp(-kld)
 *   npairs_out  [1] int32 device or NULL: number of pairs
 *   workspace   protoseg_kld_workspace_size(B, P, HW, K) bytes; the forward fills it and the
 *               backward of the same inputs reads it (and reuses its scratch part)
 * Backward:
 *   g_loss      [1] f32 device or NULL (= 1): upstream gradient of the loss
 *   g_dist      [B, P, HW] f32 out: d(g_loss * loss)/d dist (overwritten, dense; zero off each
 *               prototype's class pixels) — pass it to protoseg_l2_bwd as g_dist
 */
size_t protoseg_kld_workspace_size(int B, int P, int HW, int K);
int protoseg_kld_forward(const float* dist, int B, int P, int HW, const void* label, int label_dtype,
                         const int32_t* proto_class, int K, int max_per_class, float* loss_out,
                         int32_t* npairs_out, void* workspace, size_t workspace_bytes,
                         protoseg_stream_t stream);
int protoseg_kld_backward(const float* dist, int B, int P, int HW, const void* label, int label_dtype,
                          const int32_t* proto_class, int K, int max_per_class, const float* g_loss,
                          void* workspace, size_t workspace_bytes, float* g_dist,
                          protoseg_stream_t stream);
/*
 * protoseg_kld_backward with the per-pair coefficients in a caller buffer of
 * protoseg_kld_coef_bytes(B, K) bytes instead of the workspace's (dead) range-partial region, so
 * the workspace is only read: a caller that must not mutate it (an autograd op) needs no copy.
 */
size_t protoseg_kld_coef_bytes(int B, int K);
int protoseg_kld_backward_ex(const float* dist, int B, int P, int HW, const void* label, int label_dtype,
                             const int32_t* proto_class, int K, int max_per_class, const float* g_loss,
                             const void* workspace, size_t workspace_bytes, float* coef, size_t coef_bytes,
                             float* g_dist, protoseg_stream_t stream);
/*
 * The backward in the compact layout protoseg_l2_bwd_kld consumes (no [B, P, HW] tensor): the
 * gradient is non-zero only at the prototypes of each pixel's own class (module.py:173-178), so
 * it is stored per pixel and class slot. Same values as protoseg_kld_backward's g_dist:
 *   g_cls      [B*HW, max_per_class] f32 out: g_cls[g][i] = d loss / d dist[b][idx_c[i]][n] for
 *              the pixels of a contributing group (other entries are not written)
 *   pix_cls    [B*HW] int32 out: the pixel's class c when its (image, class) group adds pairs, else -1
 *   proto_slot [P] int32 out: class * 256 + position of the prototype among its class's prototypes
 *              (ascending prototype id); prototypes outside [0, K) get class K
 * protoseg_kld_expand writes (accumulate = 0) or adds (1) the dense g_dist these describe.
 */
int protoseg_kld_backward_compact(const float* dist, int B, int P, int HW, const void* label, int label_dtype,
                                  const int32_t* proto_class, int K, int max_per_class, const float* g_loss,
                                  void* workspace, size_t workspace_bytes,
                                  float* g_cls, int32_t* pix_cls, int32_t* proto_slot,
                                  protoseg_stream_t stream);
int protoseg_kld_expand(const float* g_cls, const int32_t* pix_cls, const int32_t* proto_slot,
                        int B, int P, int HW, int max_per_class, int accumulate, float* g_dist,
                        protoseg_stream_t stream);

/*
 * Segmentation evaluation counts. Replaces segmentation/eval_valid.py:159-197: bilinear upsample
 * (F.interpolate, align_corners=False) of logits and distances to the label resolution, argmax /
 * argmin, and the numpy counts per class and per prototype — without materialising the
 * upsampled tensors. Counts are ADDED to `counts` (zero it once per evaluation run, then call
 * per batch, as the reference accumulates its Counters).
 *
 *   logits      [B, h, w, K] f32 (PPNet.forward's logits, NHWC, model.py:278)
 *   dist        [B, P, h, w] f32 or NULL (distances, model.py:283): NULL skips the per-prototype counts
 *   ann         [B, H, W] ann_dtype (PROTOSEG_I64 | I32 | U8): labels after CLS_CONVERT (0 = void),
 *               or raw ids mapped through `lut` [lut_size] int32 (ids outside -> void)
 *   proto_class [P] int32 (argmax of prototype_class_identity), required with dist
 *   counts      [2 + 2K + P] int64 in/out: correct, total, I[K], U[K], per-prototype counts
 *               (pixels whose nearest prototype is p and whose prediction is p's class)
 * K <= 64, P <= 4096.
 */
int protoseg_eval_counts(const float* logits, const float* dist, int B, int h, int w, int K, int P,
                         const void* ann, int ann_dtype, int H, int W, const int32_t* lut, int lut_size,
                         const int32_t* proto_class, int64_t* counts, protoseg_stream_t stream);

/*
 * Label resize with PIL Image.resize(NEAREST) semantics. Replaces segmentation/dataset.py:23-31
 * (resize_label), used by find_nearest.py:128-130 (void mask of the k-NN search) and by
 * module.py:145 (KLD targets). out[y, x] = label[sy(y), sx(x)] where the source index follows
 * PIL's f64 accumulation (start scale/2, += scale per step, truncate): bit-exact to PIL.
 *   label [n_img, H, W] label_dtype (PROTOSEG_I64 | I32 | U8), mapped through `lut` when given
 *   out   [n_img, h, w] int32
 */
int protoseg_resize_label(const void* label, int label_dtype, int n_img, int H, int W, int h, int w,
                          const int32_t* lut, int lut_size, int32_t* out, protoseg_stream_t stream);

/*
 * k-nearest-patch search, step 1 of 3 per batch. Replaces find_nearest.py:132 and 140-145:
 * per image and prototype, np.amin / first np.argmin of dist + 10e6 * (label == void), the sum
 * formed in f64 as numpy broadcasts it.
 *   dist        [n_img, P, h, w] f32 (push_forward distances, find_nearest.py:103-104)
 *   small_label [n_img, h, w] int32 converted labels at map size (protoseg_resize_label), 0 = void;
 *               NULL = no void patches
 *   min_dist    [n_img, P] f64 out;  min_idx [n_img, P] int32 out (flat patch index r * w + c)
 */
int protoseg_knn_image_min(const float* dist, int n_img, int P, int h, int w, const int32_t* small_label,
                           double* min_dist, int32_t* min_idx, protoseg_stream_t stream);

/*
 * k-NN step 2: label of each winning patch. Replaces find_nearest.py:159-166 and 202-211: the
 * patch's pixel box int(r * H/h) .. int((r+1) * H/h) (f64) and the label of its pixels
 * (search_y = converted label - 1): the prototype's class when any pixel has it, else the most
 * common value (smallest on ties). An empty box yields INT32_MIN (the image is skipped,
 * find_nearest.py:179-180). Labels outside [-256, 255] after conversion set status bit 0.
 *   label  [n_img, H, W] label_dtype, raw ids mapped through `lut` when given
 *   proto_class [P] int32; patch_label [n_img, P] int32 out; status [1] int32 in/out
 */
int protoseg_knn_patch_label(const int32_t* min_idx, int n_img, int P, int h, int w, const void* label,
                             int label_dtype, int H, int W, const int32_t* lut, int lut_size,
                             const int32_t* proto_class, int32_t* patch_label, int32_t* status,
                             protoseg_stream_t stream);

/*
 * k-NN step 3: offers the batch's images, in order, to the per-prototype heaps. Replaces
 * find_nearest.py:224-230 (heapq.heappush while fewer than k, else heappushpop) with CPython
 * heapq's exact sift sequence, so ties resolve as the reference's do. Heap state persists across
 * calls: heap_neg [P, k] f64 (negative distances), heap_label / heap_patch [P, k] int32,
 * heap_img [P, k] int64 (first_img + image index), heap_size [P] int32 (zero it before the
 * first batch). k <= 64.
 */
int protoseg_knn_heap_push(const double* min_dist, const int32_t* min_idx, const int32_t* patch_label, int n_img,
                           int64_t first_img, int P, int k, double* heap_neg, int32_t* heap_label,
                           int32_t* heap_patch, int64_t* heap_img, int32_t* heap_size, protoseg_stream_t stream);

/*
 * k-NN finalisation and the pruning rule. Replaces find_nearest.py:227-232 (heaps[j].sort(),
 * [::-1]: ascending distance, stable) and prune.py:35-43: class_count[p] = number of the k
 * nearest patches labelled with p's class; prune[p] = class_count[p] < prune_threshold.
 * Outputs [P, k]: out_dist f64, out_label int32, out_img int64, out_patch int32; slots past a
 * heap's size hold inf / INT32_MIN / -1 / -1.
 */
int protoseg_knn_finalize(const double* heap_neg, const int32_t* heap_label, const int32_t* heap_patch,
                          const int64_t* heap_img, const int32_t* heap_size, int P, int k,
                          const int32_t* proto_class, int prune_threshold, double* out_dist, int32_t* out_label,
                          int64_t* out_img, int32_t* out_patch, int32_t* class_count, int32_t* prune,
                          protoseg_stream_t stream);

/*
 * Push outputs, high-activation bound boxes, step 1. Replaces segmentation/push.py:309-319:
 * the prototype's activation map on the winning image (log: np.log((d+1)/(d+eps)) in f32;
 * linear: max_dist - d, max_dist = C; identity: dist already holds activations) and
 * cv2.resize(act, (W, H), interpolation=cv2.INTER_CUBIC) (A = -0.75, half-pixel centres,
 * replicated border, horizontal then vertical pass, unfused f32).
 *   dist [m, h, w] f32   one distance map per pushed prototype (gathered by the caller)
 *   act  [m, h, w] f32 out;  up [m, H, W] f32 out
 */
int protoseg_act_upsample(const float* dist, int m, int h, int w, int H, int W, int act_kind, float eps,
                          float max_dist, float* act, float* up, protoseg_stream_t stream);

/*
 * Bound boxes, step 2. Replaces push.py:321-343 and helpers.py:48-82: threshold =
 * np.percentile(up, percentile) (numpy 'linear', f32), mask = up * (label == class + 1) >=
 * threshold, the receptive-field box grown greedily over the mask, a `margin`-pixel border
 * added (find_continuous_high_activation_crop, add_margin = 5).
 *   up [m, H, W] f32 from protoseg_act_upsample
 *   label [n_label, H, W] label_dtype (raw ids through `lut` when given); label_index [m] int32
 *         picks each map's image (NULL = image 0)
 *   target_class [m] int32 (push.py:251);  rf_box [m, 4] int32 (start_h, end_h, start_w, end_w)
 *         as push.py:288-294
 *   threshold [m] f32 out;  box [m, 4] int32 out = (start_h, end_h, start_w, end_w) as
 *         proto_bound_boxes[j, 1:5] (push.py:338-342); -1 (threshold NaN) when label_index or
 *         rf_box is out of range
 * m <= 65535. Scratch (per-map histograms and select state, a candidate list of up to 1/8 of
 * each map, per-chunk histogram rows: a little over m * H * W / 2 bytes) is a grow-only device block
 * per (device, stream), allocated on the first call that needs it; later calls on the stream
 * are kernel launches only (capturable in a HIP graph).
 */
int protoseg_bound_boxes(const float* up, int m, int H, int W, const void* label, int label_dtype, int n_label,
                         const int32_t* label_index, const int32_t* lut, int lut_size, const int32_t* target_class,
                         const int32_t* rf_box, float percentile, int margin, float* threshold, int32_t* box,
                         protoseg_stream_t stream);

/*
 * Optimizer step of the training step: torch.optim.Adam as the reference configures it
 * (segmentation/module.py:391: amsgrad off, L2 weight decay per group) over n_tensors (<= 8) f32
 * tensors in one launch, with torch's fused-Adam arithmetic:
 *   g = grad + weight_decay * p;  m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g^2;
 *   p -= lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
 *   params[k], grads[k], exp_avg[k], exp_avg_sq[k]: device f32 [numel[k]] (host pointer arrays)
 *   state[k]: device int32[2] per tensor = {its step count t of the previous call, 0}: tensor k
 *          uses t + 1 and stores it (torch keeps one step per parameter, state[p]['step']), so a
 *          HIP graph holding the call replays as successive steps; a tensor with numel 0 still
 *          advances its count.
 */
int protoseg_adam_step(int n_tensors, float* const* params, const float* const* grads,
                       float* const* exp_avg, float* const* exp_avg_sq, const int64_t* numel,
                       int32_t* const* state, float lr, float beta1, float beta2, float eps, float weight_decay,
                       protoseg_stream_t stream);

/*
 * The layer's optimizer step fused with the next forward's operand prep: protoseg_adam_step of
 * the prototype vectors [P, C] and the last layer [K, P] (each with its group's lr and
 * weight_decay, shared betas / eps; the same arithmetic, the same bits), then the operand images
 * protoseg_l2_fwd_ex would build from the updated values, written into `operands` (the same
 * bits), in ONE launch. The step's next protoseg_l2_fwd_ex then passes PROTOSEG_OPERANDS_READY
 * and launches no prep: the training step runs forward, backward (+ its slab reduce) and this
 * call. eps / act_kind / precision are the forward's. Served where
 * protoseg_l2_adam_prep_supported (BF16X3, C = 64, K <= 32, the shapes whose backward reads the
 * one-chunk image block); PROTOSEG_ERR_UNSUPPORTED elsewhere (nothing launched: run
 * protoseg_adam_step and a plain _ex forward). w_last and its state NULL iff K = 0.
 */
int protoseg_l2_adam_prep_supported(int C, int P, int K, int precision);
int protoseg_l2_adam_prep(int C, int P, int K, float eps, int act_kind, int precision,
                          float* protos, const float* g_protos, float* exp_avg_p, float* exp_avg_sq_p,
                          int32_t* state_p, float lr_p, float weight_decay_p,
                          float* w_last, const float* g_w, float* exp_avg_w, float* exp_avg_sq_w,
                          int32_t* state_w, float lr_w, float weight_decay_w,
                          float beta1, float beta2, float adam_eps,
                          void* operands, size_t operands_bytes, protoseg_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* PROTOSEG_HIP_H_ */
