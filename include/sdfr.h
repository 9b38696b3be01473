/*
 * sdfr.h -- C ABI of libsdfr.so, the MI355X (gfx950) SDF + hash-grid renderer.
 *
 * Plain pointers and sizes only; every pointer below is a DEVICE pointer
 * unless stated otherwise, `stream` is a hipStream_t passed as void*
 * (NULL = the legacy default stream).  All entry points are asynchronous
 * with respect to the host, enqueue on `stream`, return SDFR_OK (0) or a
 * negative status, and never allocate device memory.
 *
 * Reference interfaces replaced (paths relative to the reference root):
 *   sdfr_grid_encode_forward   <- grid_encode_forward
 *        im2scene/sdf/models/gridencoder/src/gridencoder.h:11,
 *        pybind export gridencoder/src/bindings.cpp:5, caller grid.py:54
 *   sdfr_grid_encode_backward  <- grid_encode_backward
 *        gridencoder.h:12, bindings.cpp:6, caller grid.py:84
 *   sdfr_sh_encode_forward     <- sh_encode_forward
 *        shencoder/src/shencoder.h:9, bindings.cpp:5, caller sphere_harmonics.py:32
 *   sdfr_sh_encode_backward    <- sh_encode_backward
 *        shencoder.h:10, bindings.cpp:6, caller sphere_harmonics.py:51
 *   sdfr_render_ngp_forward    <- VolumeFeatureRenderer.forward for
 *        rendering.type == "ngp" (sdf_model.py:411-423 -> render :363 ->
 *        render_rays :310 -> NGPSIRENGenerator.forward :1566 ->
 *        volume_integration :236).  The reference has no native op here;
 *        this one fuses the whole chain.
 *
 * Error behaviour mirrors the reference: the same argument combinations the
 * reference rejects with std::runtime_error / TORCH_CHECK return
 * SDFR_EINVAL here, with the reference's message in sdfr_last_error().
 */
#ifndef SDFR_H_
#define SDFR_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDFR_OK 0
#define SDFR_EINVAL (-1)       /* bad sizes / unsupported D, C, degree        */
#define SDFR_ELAUNCH (-2)      /* HIP launch or runtime error                 */
#define SDFR_EUNSUPPORTED (-3) /* valid for the reference, not implemented    */

#define SDFR_ABI_VERSION 13

int sdfr_abi_version(void);
/* Thread-local message for the last non-zero status of this thread. */
const char *sdfr_last_error(void);

/* ---------------------------------------------------------------------------
 * Multiresolution hash / tiled grid encoder (gridencoder.cu semantics).
 *   inputs      [B, D] fp32 in [0,1] (outside -> output 0)
 *   embeddings  [offsets[L], C] fp32
 *   offsets     [L+1] int32
 *   outputs     [L, B, C] fp32 (level-major, as the reference)
 *   dy_dx       [B, L*D*C] fp32 or NULL
 *   S = log2(per_level_scale) (fp32), H = base resolution
 *   gridtype 0 = hash, 1 = tiled; interp 0 = linear, 1 = smoothstep
 *   D in {2,3,4,5}, C in {1,2,4,8}; L <= 64.
 * ------------------------------------------------------------------------- */
int sdfr_grid_encode_forward(const float *inputs, const float *embeddings,
                             const int32_t *offsets, float *outputs,
                             uint32_t B, uint32_t D, uint32_t C, uint32_t L,
                             float S, uint32_t H, float *dy_dx,
                             uint32_t gridtype, int align_corners,
                             uint32_t interp, void *stream);

/*   grad            [L, B, C]
 *   grad_embeddings [offsets[L], C], must be zeroed by the caller (grid.py:75); may be
 *                   NULL when grad_inputs is given (input gradient only: the eikonal
 *                   term's pass, whose table gradient autograd.grad discards)
 *   dy_dx / grad_inputs: both NULL, or dy_dx [B, L*D*C] and grad_inputs [B, D]
 *   (grad_inputs is overwritten). */
int sdfr_grid_encode_backward(const float *grad, const float *inputs,
                              const float *embeddings, const int32_t *offsets,
                              float *grad_embeddings, uint32_t B, uint32_t D,
                              uint32_t C, uint32_t L, float S, uint32_t H,
                              const float *dy_dx, float *grad_inputs,
                              uint32_t gridtype, int align_corners,
                              uint32_t interp, void *stream);

/* The same with a caller-owned device workspace of at least
 * sdfr_grid_encode_backward_ws_bytes(...) bytes (0 = none needed: then ws may be
 * NULL).  With it, the table gradient of the fine levels is binned and summed in
 * LDS instead of scattered with global atomics (csrc/encoders.hip); with ws NULL
 * or too small, the workspace-free path runs (LDS windows for the coarse levels,
 * direct atomics for the hashed ones).  sdfr_grid_encode_backward is this function
 * with ws NULL: it allocates nothing (stream-ordered, HIP-graph-capture safe). */
size_t sdfr_grid_encode_backward_ws_bytes(uint32_t B, uint32_t D, uint32_t C, uint32_t L,
                                          float S, uint32_t H, int align_corners);
int sdfr_grid_encode_backward_ws(const float *grad, const float *inputs,
                                 const float *embeddings, const int32_t *offsets,
                                 float *grad_embeddings, uint32_t B, uint32_t D,
                                 uint32_t C, uint32_t L, float S, uint32_t H,
                                 const float *dy_dx, float *grad_inputs,
                                 uint32_t gridtype, int align_corners,
                                 uint32_t interp, void *ws, size_t ws_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * Real spherical harmonics (shencoder.cu semantics), C = degree.
 *   inputs [B, D], D must be 3; outputs [B, C*C]; dy_dx [B, D*C*C] or NULL.
 *   Degrees 1..8 are implemented (SDFace uses 4; 5..8 from the bands that
 *   csrc/sh_gen.py generates); other degrees -> SDFR_EUNSUPPORTED.
 * ------------------------------------------------------------------------- */
int sdfr_sh_encode_forward(const float *inputs, float *outputs, uint32_t B,
                           uint32_t D, uint32_t C, float *dy_dx, void *stream);

/* grad [B, C*C]; grad_inputs [B, D] accumulated into (caller zeroes it). */
int sdfr_sh_encode_backward(const float *grad, const float *inputs, uint32_t B,
                            uint32_t D, uint32_t C, const float *dy_dx,
                            float *grad_inputs, void *stream);

/* ---------------------------------------------------------------------------
 * Fused NGP renderer forward (inference / frozen renderer).
 *
 * Network: NGPSIRENGenerator(D=2, W=256, style_dim=256) with a
 * GridEncoder(L=16, C=2, H=16, 2^19 rows, desired 4096) and SHEncoder(4).
 * Parameter pointers are the PyTorch tensors of the reference state dict
 * (row-major [out, in] weights, sdf_model.py:1545-1564).
 * ------------------------------------------------------------------------- */
typedef struct sdfr_ngp_weights {
    const float *embeddings;      /* [offsets[L], 2]                              */
    const int32_t *offsets;       /* [L+1] (device)                               */
    uint32_t num_levels;          /* L (16)                                        */
    float log2_per_level_scale;   /* S                                            */
    uint32_t base_resolution;     /* H (16)                                        */
    float bound;                  /* NGPSIRENGenerator.bound (2)                   */
    const float *input_w, *input_b;     /* [256,32], [256]                        */
    const float *pts_w[3], *pts_b[3];   /* [256,256], [256]                       */
    const float *pts_gw[3], *pts_gb[3]; /* gamma LinearLayer [256,256], [256]     */
    const float *pts_bw[3], *pts_bb[3]; /* beta  LinearLayer [256,256], [256]     */
    const float *views_w, *views_b;     /* [256,272], [256]                       */
    const float *views_gw, *views_gb, *views_bw, *views_bb;
    const float *sigma_w, *sigma_b;     /* [1,256], [1]                           */
    const float *rgb_w, *rgb_b;         /* [3,256], [3]                           */
    const float *sigmoid_beta;          /* [1] (renderer.sigmoid_beta)            */
} sdfr_ngp_weights;

typedef struct sdfr_ngp_render_args {
    uint32_t B, H, W, N;          /* faces, image rows, cols, samples per ray      */
    const float *cam;             /* [B,3,4] c2w = [R^T | T]                       */
    const float *focal;           /* [B]                                           */
    const float *near_;           /* [B]                                           */
    const float *far_;            /* [B]                                           */
    const float *styles;          /* [B,256] renderer latent                       */
    const float *pix_x;           /* [W] renderer i-buffer row (x + 0.5)           */
    const float *pix_y;           /* [H] renderer j-buffer column                  */
    const float *t_vals;          /* [N]                                           */
    const float *t_rand;          /* NULL, [B,H,W] or [B,H,W,N]                    */
    const float *sigma_noise;     /* NULL or [B,H,W,N] (no_sdf mode only)          */
    int t_rand_per_sample;        /* 1 -> t_rand is [B,H,W,N] (stratified)         */
    int offset_sampling;          /* !opt.no_offset_sampling                       */
    int static_viewdirs;
    int z_normalize;              /* !opt.no_z_normalize                           */
    int force_background;
    int with_sdf;                 /* !opt.no_sdf                                   */
    float *rgb;                   /* [B,3,H,W]                     (required)      */
    float *features;              /* [B,256,H,W] or NULL                            */
    float *sdf;                   /* [B,H,W,N] or NULL                             */
    float *xyz;                   /* [B,3,H,W] or NULL                             */
    float *mask;                  /* [B,1,H,W] or NULL                             */
    void *workspace;              /* >= sdfr_render_ngp_workspace_bytes()          */
    size_t workspace_bytes;
    /* Optional hipEvent_t handles (NULL = skip), recorded on `stream`:
     * [0] at entry, [1] before the hash-grid kernel, [2] after it (ngp f16x3;
     * before the FiLM prep), [3] after the field (MLP + compositing) kernel. */
    void *stage_events[4];
    /* Field-stage GEMM arithmetic (both accumulate in fp32):
     * SDFR_FIELD_F16X3 (0, default) three v_mfma_f32_16x16x32_f16 per tile on a
     *   hi/lo fp16 split of row-scaled weights and activations (fp32-level
     *   accuracy);
     * SDFR_FIELD_FP32 (1) v_mfma_f32_16x16x4_f32 (exact fp32 fma chain). */
    int field_precision;
    /* NULL, or the split-fp16 weights packed beforehand by sdfr_render_ngp_pack /
     * sdfr_render_siren_pack from the SAME weights (f16x3 only): the per-call
     * row-scale and packing kernels are then skipped, only the per-face FiLM
     * vectors are formed. */
    const void *prepacked;
    /* Upper bound on the sample segments per ray of the f16x3 field stage (0 = the
     * default 4): batches too small to give every CU a workgroup split each ray's
     * samples over up to this many workgroups and chain the segments in a merge
     * kernel (sdf_model.py:273-289's cumprod re-associated: fp32-rounding-level
     * differences).  1 disables the split; 2 or 4 otherwise.  The workspace size
     * (sdfr_render_ngp_workspace_bytes) covers the default bound. */
    uint32_t max_field_segments;
    /* ABI 11.  styles_event: NULL, or a hipEvent_t that `stream` waits on before the
     * first use of `styles` (the FiLM prep; the ngp f16x3 path enqueues the sample
     * geometry and the hash-grid gather ahead of that wait, so a caller may still be
     * computing the styles on another stream).  field_event: NULL, or a hipEvent_t
     * recorded right before the field kernel (after the FiLM prep). */
    void *styles_event;
    void *field_event;
    /* ABI 12 (f16x3 ngp / FC only): NULL, or [B,H,W,32,2,8] fp16 -- the features
     * times features_mod[b,c] in the decoder's split-NHWC layout (hi / lo halves of
     * each 8-channel group, sdfr_modulate_to_nhwc_split's output, bit for bit), written
     * instead of the NCHW `features` (which must then be NULL). */
    void *features_split;
    const float *features_mod;    /* [B,256] with features_split                    */
} sdfr_ngp_render_args;

#define SDFR_FIELD_F16X3 0
#define SDFR_FIELD_FP32 1

size_t sdfr_render_ngp_workspace_bytes(uint32_t B, uint32_t H, uint32_t W,
                                       uint32_t N, uint32_t num_levels);

int sdfr_render_ngp_forward(const sdfr_ngp_weights *w,
                            const sdfr_ngp_render_args *a, void *stream);

/* ---------------------------------------------------------------------------
 * Fused SIREN renderer forward (rendering.type == "sdf", SirenGenerator,
 * sdf_model.py:101-139, BASELINE configs[4]): the same render chain as
 * sdfr_render_ngp_forward with the network's 8 FiLM layers fed by the
 * normalised sample points and the views layer by the unit view direction.
 * Replaces VolumeFeatureRenderer.forward for type "sdf" (sdf_model.py:411-423);
 * the reference has no native op here.  Takes the same render args
 * (field_precision must be SDFR_FIELD_F16X3); workspace from
 * sdfr_render_siren_workspace_bytes(B).  stage_events[1] == [2] (no encode stage).
 * ------------------------------------------------------------------------- */
typedef struct sdfr_siren_weights {
    uint32_t depth;                     /* D (8)                                    */
    uint32_t width;                     /* W (256)                                  */
    const float *pts_w[8], *pts_b[8];   /* [256,3] (layer 0) / [256,256], [256]     */
    const float *pts_gw[8], *pts_gb[8]; /* gamma LinearLayer [256,256], [256]       */
    const float *pts_bw[8], *pts_bb[8]; /* beta  LinearLayer [256,256], [256]       */
    const float *views_w, *views_b;     /* [256,259], [256]                         */
    const float *views_gw, *views_gb, *views_bw, *views_bb;
    const float *sigma_w, *sigma_b;     /* [1,256], [1]                             */
    const float *rgb_w, *rgb_b;         /* [3,256], [3]                             */
    const float *sigmoid_beta;          /* [1] (renderer.sigmoid_beta)              */
} sdfr_siren_weights;

size_t sdfr_render_siren_workspace_bytes(uint32_t B);

/* ---------------------------------------------------------------------------
 * Fused FCGenerator renderer forward (rendering.fc == 1, sdf_model.py:1599-1670:
 * the "plain Fourier MLP" of BASELINE configs[4]): positional encodings of the
 * normalised sample point (10 frequencies) -> x_in + style_in(styles) -> ReLU ->
 * 7 x (Linear 256, ReLU) -> sigma | [h, encodings of the view direction (4
 * frequencies)] -> views_linears (the colour features) -> rgb_linear, then the
 * same SDF -> density and compositing as the other networks
 * (sdf_model.py:231-301).  Replaces VolumeFeatureRenderer.forward for fc == 1
 * (sdf_model.py:411-423).  Same render args (field_precision must be
 * SDFR_FIELD_F16X3); workspace from sdfr_render_fc_workspace_bytes.
 * stage_events[1] == [2] (no encode stage).
 * ------------------------------------------------------------------------- */
typedef struct sdfr_fc_weights {
    uint32_t depth;                     /* D (8)                                    */
    uint32_t width;                     /* W (256)                                  */
    const float *x_in_w, *x_in_b;       /* [256,60], [256]                          */
    const float *style_w, *style_b;     /* style_in [256,256], [256]                */
    const float *pts_w[7], *pts_b[7];   /* [256,256], [256]                         */
    const float *views_w, *views_b;     /* [256,280], [256]                         */
    const float *sigma_w, *sigma_b;     /* [1,256], [1]                             */
    const float *rgb_w, *rgb_b;         /* [3,256], [3]                             */
    const float *sigmoid_beta;          /* [1] (renderer.sigmoid_beta)              */
} sdfr_fc_weights;

size_t sdfr_render_fc_workspace_bytes(uint32_t B, uint32_t H, uint32_t W, uint32_t N);

int sdfr_render_fc_forward(const sdfr_fc_weights *w,
                           const sdfr_ngp_render_args *a, void *stream);

/* Split-fp16 weight packing of the field kernel (row scales, scaled biases, MFMA
 * A-fragments), done once per weight version by the caller instead of per call:
 * `packed` holds sdfr_render_pack_bytes(net) bytes (net 0 ngp, 1 siren, 2 fc). */
size_t sdfr_render_pack_bytes(int net);
int sdfr_render_ngp_pack(const sdfr_ngp_weights *w, void *packed, void *stream);
int sdfr_render_siren_pack(const sdfr_siren_weights *w, void *packed, void *stream);
int sdfr_render_fc_pack(const sdfr_fc_weights *w, void *packed, void *stream);

int sdfr_render_siren_forward(const sdfr_siren_weights *w,
                              const sdfr_ngp_render_args *a, void *stream);

/* Profiling aid: enqueue only the hash-grid stage of the fused renderer
 * (writes the encoded samples into the workspace).  Same arguments. */
int sdfr_render_ngp_encode_only(const sdfr_ngp_weights *w,
                                const sdfr_ngp_render_args *a, void *stream);

#ifdef SDFR_ABLATION
/* Profiling hooks, exported only by `make ABLATION=1` builds (lib_abl/libsdfr.so,
 * process-global state; never in the product library):
 * sdfr_debug_set_field_variant selects an ablated field kernel for later calls
 * (0 = the product kernel; 1 no barrier, 2 no LDS A-operand reads, 4 no weight
 * staging, 8 no activations, 16 no compositing, 15/31 MFMA only -- wrong outputs,
 * to attribute kernel time); sdfr_debug_set_encode_mode the
 * hash-grid gather variant (default 289, or SDFR_ENC_MODE at load; 1, 2, 9, 33,
 * 257, 289, 290 -- all bit-identical, scripts/encode_time.py). */
int sdfr_debug_set_field_variant(int variant);
int sdfr_debug_set_encode_mode(int mode);
#endif

/* Accuracy probe for the two device sin implementations the field kernel can
 * use (software Cody-Waite + polynomial, hardware v_sin_f32 after reduction):
 * out_cw[i] = sin_cw(x[i]), out_hw[i] = sin_hw(x[i]), n elements. */
int sdfr_debug_sin_probe(const float *x, float *out_cw, float *out_hw, uint32_t n,
                         void *stream);

/* Accuracy probe for the split-fp16 field kernel's FiLM sin, whose argument is in
 * revolutions (1/(2 pi) folded into the FiLM vectors): out[i] = sin(2 pi u[i]) by
 * v_fract_f32 + v_sin_f32, n elements. */
int sdfr_debug_sin_rev_probe(const float *u, float *out, uint32_t n, void *stream);

/* Camera parameters from sampled angles (generate_camera_params, sdf_utils.py:97-159,
 * after its random draws; distance 1): viewpoint [B,2] = (azim, elev); ext [B,3,4] =
 * [R^T | T] with T = (cos e sin a, sin e, cos e cos a), R rows = normalize(up x z),
 * normalize(z x x), z = normalize(T), and the degenerate-x replacement of :151-154;
 * near / far [B] = 1 -/+ dist_radius; focal [B] = half_res / tan(fov_ang pi / 180).
 * azim, elev [B] on the device; fp32, one rounding per op. */
int sdfr_camera_extrinsics(const float *azim, const float *elev, uint32_t B, float dist_radius,
                           float fov_ang, float half_res, float *ext, float *focal, float *near_,
                           float *far_, float *viewpoint, void *stream);

/* ---------------------------------------------------------------------------
 * Renderer MLP linear layers for training (no reference native op: they replace
 * the rocBLAS fp32 GEMMs of F.linear in FiLMSiren / LinearLayer, sdf_model.py:23-69,
 * and of their autograd backward, on the op-by-op path stage-1 training takes,
 * training_utils.py:396-451).  Split-fp16 MFMA, fp32 accumulation, fp32-level
 * accuracy (rows / columns scaled by powers of two so no fp16 lo part goes
 * subnormal).  Row-major fp32 tensors; x, out, y_save 16-B aligned, and bias,
 * gamma, beta (read as 16-B vectors) 16-B aligned.
 *
 * sdfr_linear_pack: B [N,K] = w (transposed = 0; w is [N,K]) or w^T (transposed = 1;
 *   w is [K,N]) -> sdfr_linear_pack_bytes(N, K) bytes of split fragments + row scales.
 * sdfr_linear_f16x3: out [M,N] = x [M,K] . B^T (+ bias [N], NULL = none).  Forward
 *   (B = W [N,K]) and input gradient (B = W^T).  Shapes: (N, K) = (256, K <= 32 |
 *   <= 256 | <= 288) or (N <= 32 | <= 256 | <= 272, K <= 256), N and K multiples of 4.
 * sdfr_linear_wgrad_f16x3: gw [N,K] = dy[M,N]^T . x[M,K] (weight gradient), N = 256,
 *   K <= 288; ws >= sdfr_linear_wgrad_ws_bytes(M, N, K).  The sum over M is split
 *   over workgroups and their partials added in a fixed order (deterministic); each
 *   workgroup scales a column by the running maximum of the rows it has read, so
 *   dy and x are each read once (no separate column-maximum pass).
 * ------------------------------------------------------------------------- */
size_t sdfr_linear_pack_bytes(uint32_t N, uint32_t K);
int sdfr_linear_pack(const float *w, uint32_t N, uint32_t K, int transposed, void *packed,
                     void *stream);
int sdfr_linear_f16x3(float *out, const float *x, const void *packed, const float *bias,
                      uint32_t M, uint32_t N, uint32_t K, void *stream);
size_t sdfr_linear_wgrad_ws_bytes(uint32_t M, uint32_t N, uint32_t K);
int sdfr_linear_wgrad_f16x3(float *gw, const float *dy, const float *x, uint32_t M, uint32_t N,
                            uint32_t K, void *ws, size_t ws_bytes, void *stream);

/* FiLMSiren.forward / backward (sdf_model.py:62-67) around the same GEMM, F faces of
 * rows_per_face consecutive rows each (M = F rows_per_face), N = 256:
 * sdfr_film_linear_f16x3: y_save = x . W^T + bias; out = sin(gamma[f] * y + beta[f])
 *   (gamma, beta [F,N]; one rounding per op, as the reference's separate ops).
 * sdfr_film_backward: with u = gamma[f] y + beta[f] recomputed, du = ds cos(u):
 *   dy = du gamma[f] [M,N] (the input of the two GEMM gradients), dgamma[f] = sum du y,
 *   dbeta[f] = sum du, dbf[f] = sum dy (the bias gradient, per face) [F,N] each;
 *   every sum in a fixed order; ws >= sdfr_film_backward_ws_bytes(M, N, rows_per_face). */
int sdfr_film_linear_f16x3(float *out, float *y_save, const float *x, const void *packed,
                           const float *bias, const float *gamma, const float *beta, uint32_t M,
                           uint32_t N, uint32_t K, uint32_t rows_per_face, void *stream);
size_t sdfr_film_backward_ws_bytes(uint32_t M, uint32_t N, uint32_t rows_per_face);
int sdfr_film_backward(float *dy, float *dgamma, float *dbeta, float *dbf, const float *ds,
                       const float *y, const float *gamma, const float *beta, uint32_t M,
                       uint32_t N, uint32_t rows_per_face, void *ws, size_t ws_bytes,
                       void *stream);

/* sdfr_film_backward_grad: the derivative of sdfr_film_backward's (dy, dgamma, dbeta)
 * w.r.t. (ds, y, gamma, beta) -- the second-order step of a FiLM layer whose backward
 * was built with create_graph (the SIREN eikonal term, sdf_model.py:224-229, then
 * differentiated by the loss).  Given the upstream gradients g_dy [M,N], g_dgamma,
 * g_dbeta [F,N] (each may be NULL = 0), with u = gamma[f] y + beta[f] and
 * H = g_dy gamma[f] + g_dgamma[f] y + g_dbeta[f]:
 *   d_ds = H cos u, d_y = -H ds sin u gamma[f] + g_dgamma[f] ds cos u  [M,N],
 *   d_gamma[f] = sum (-H ds sin u y + g_dy ds cos u), d_beta[f] = sum -H ds sin u  [F,N];
 * sums in a fixed order; ws >= sdfr_film_backward_grad_ws_bytes(M, N, rows_per_face). */
size_t sdfr_film_backward_grad_ws_bytes(uint32_t M, uint32_t N, uint32_t rows_per_face);
int sdfr_film_backward_grad(float *d_ds, float *d_y, float *d_gamma, float *d_beta,
                            const float *ds, const float *y, const float *gamma,
                            const float *beta, const float *g_dy, const float *g_dgamma,
                            const float *g_dbeta, uint32_t M, uint32_t N, uint32_t rows_per_face,
                            void *ws, size_t ws_bytes, void *stream);

/* The MLP's narrow output heads for training (sigma_linear 256 -> 1, rgb_linear
 * 256 -> 3; LinearLayer, sdf_model.py:23-41, at :1586-1588), fp32 FMAs, J <= 4 outputs,
 * K <= 256 inputs (a multiple of 4), 16-B aligned x, w, gx:
 * sdfr_linear_head_forward: out [M,J] = x [M,K] . w [J,K]^T (+ bias [J], NULL = none).
 * sdfr_linear_head_backward: gx [M,K] = gy [M,J] . w; gw [J,K] = gy^T . x; gb [J] =
 *   column sums of gy -- each NULL to skip; gw / gb need ws >=
 *   sdfr_linear_head_ws_bytes(M, J, K) (per-workgroup partials added in a fixed order). */
int sdfr_linear_head_forward(float *out, const float *x, const float *w, const float *bias,
                             uint32_t M, uint32_t J, uint32_t K, void *stream);
size_t sdfr_linear_head_ws_bytes(uint32_t M, uint32_t J, uint32_t K);
int sdfr_linear_head_backward(float *gx, float *gw, float *gb, const float *gy, const float *x,
                              const float *w, uint32_t M, uint32_t J, uint32_t K, void *ws,
                              size_t ws_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * StyleGAN2 decoder ops (im2scene/sdf/models/sdf_op.py).
 *
 * sdfr_fused_bias_act <- fused_bias_act (fused_bias_act.cpp:11,
 *   fused_bias_act_kernel.cu:18; callers sdf_op.py:29, :49, :64):
 *   out[i] = f(x[i] + bias[(i / step_b) % size_b]) * scale over size_x floats,
 *   f by (act, grad): (1,*) identity, (3,0) x>0 ? x : alpha*x,
 *   (3,1) ref[i]>0 ? x : alpha*x, (*,2) 0.  bias NULL (size_b 0) = no bias;
 *   ref may be NULL unless (act, grad) == (3, 1).  out may alias x.
 * ------------------------------------------------------------------------- */
int sdfr_fused_bias_act(float *out, const float *x, const float *bias, const float *ref,
                        uint64_t size_x, uint32_t step_b, uint32_t size_b, int act,
                        int grad, float alpha, float scale, void *stream);

/* sdfr_mapping_linear: one mapping-network layer for inference (sdf_model.py:437-466
 * MappingLinear, EqualLinear + fused_leaky_relu, PixelNorm):
 *   x' = pixelnorm ? x * rsqrt(mean(x^2) + 1e-8) : x           (per sample)
 *   y  = x' . (W * wscale)^T + b * bscale                       (b NULL: no bias)
 *   out = act ? (y > 0 ? y : y * slope) * act_scale : y
 * x [B, K], W [O, K] (16-B aligned), b [O], out [B, O]; K = 256 or 512.
 * fp32 throughout; summation order differs from a GEMM's (fp32 rounding level). */
int sdfr_mapping_linear(float *out, const float *x, const float *w, const float *b, uint32_t B,
                        uint32_t K, uint32_t O, float wscale, float bscale, int act, float slope,
                        float act_scale, int pixelnorm, void *stream);

/* sdfr_decoder_styles: the fused decoder's per-call style prep (sdf_model.py:676-699):
 *   mods[off_k + b c_k + c] = latent[b, idx_k] . mod_w[k, c] + mod_b[k, c]
 *     (mod_w = EqualLinear weight * scale, mod_b = bias * lr_mul; rows zero-padded to cmax)
 *   demods[doff_j + b o_j + o] = rsqrt(dem_eps[j, o] + sum_c mods[layer_j][b, c]^2 dem_w[j, o, c])
 *     (dem_w = su^2 sum_{ky,kx} w^2 transposed to [Cout, Cin], dem_eps = su^2 1e-8).
 * K (style dim) and cmax are 256 or 512; L, J <= 16.  fp32, dot products summed in
 * a fixed order that is not a GEMM's (fp32 rounding level). */
typedef struct sdfr_style_args {
    uint32_t B, n_latent, K;
    const float *latent;              /* [B, n_latent, K]                        */
    uint32_t L, cmax;
    const float *mod_w;               /* [L, cmax, K]                            */
    const float *mod_b;               /* [L, cmax]                               */
    uint32_t mod_index[16], mod_c[16], mod_off[16];
    float *mods;                      /* per layer [B, c_k] at mod_off[k]        */
    uint32_t J, omax;
    const float *dem_w;               /* [J, omax, cmax]                         */
    const float *dem_eps;             /* [J, omax]                               */
    uint32_t dem_layer[16], dem_c[16], dem_off[16];
    float *demods;                    /* per layer [B, o_j] at dem_off[j]        */
} sdfr_style_args;

int sdfr_decoder_styles(const sdfr_style_args *a, void *stream);

/* sdfr_upfirdn2d <- upfirdn2d (upfirdn2d.cpp:12, upfirdn2d_kernel.cu; caller
 * sdf_op.py:230): input viewed as [major, in_h, in_w] (minor = 1), kernel
 * [kernel_h, kernel_w] (device), out [major, out_h, out_w] with
 *   out_h = (in_h*up_y + pad_y0 + pad_y1 - kernel_h) / down_y + 1  (same for w):
 * zero-insertion upsample, pad (negative = crop), true convolution with the
 * kernel, then keep every down-th sample (upfirdn2d_native, sdf_op.py:273). */
int sdfr_upfirdn2d(float *out, const float *input, const float *kernel, uint32_t major,
                   uint32_t in_h, uint32_t in_w, uint32_t kernel_h, uint32_t kernel_w,
                   int up_x, int up_y, int down_x, int down_y, int pad_x0, int pad_x1,
                   int pad_y0, int pad_y1, void *stream);

/* Fused StyledConv / ToRGB epilogue (no reference counterpart: replaces the
 * chain after each decoder convolution -- ModulatedConv2d demodulation and
 * upsample blur (sdf_model.py:676-699), NoiseInjection (:704), FusedLeakyReLU
 * (:818), ToRGB + skip Upsample (:821-843) -- with one pass over the
 * activations).  Activations are NHWC (channels_last):
 *   conv  [B,H,W,C], or [B,2H+1,2W+1,C] when blur_up (stride-2 transposed conv
 *         output; blurred with outer(fir,fir), pad (1,1), as ModulatedConv2d.blur)
 *   v     = lrelu((blur(conv) * demod[b,c] + noise_weight * noise[b,h,w])
 *                 + bias[c], negative_slope) * act_scale
 *   y     [B,H,W,C] = v * s_next[b,c] (the next conv's modulation; s_next NULL
 *         -> v), or y NULL (not stored)
 *   rgb   [B,3,H,W] (NCHW) = sum_c v * rgb_w[b,o,c] + rgb_b[o]
 *         + upfirdn2d(skip, outer(fir,fir), up 2, pad (2,1)) when skip != NULL;
 *         only when rgb_w != NULL, and not together with blur_up.
 * C must be a multiple of 4; with rgb_w, C/4 must be a power of two <= 64 or
 * a multiple of 64 (C <= 1024). */
typedef struct sdfr_styled_epilogue_args {
    uint32_t B, C, H, W;
    const float *conv;
    int blur_up;
    float fir[4];                 /* separable taps; outer(fir,fir) = the 2-D kernel */
    const float *demod;           /* [B,C] or NULL (no demodulation)               */
    const float *noise;           /* [B,H,W] or NULL                               */
    const float *noise_weight;    /* [1] NoiseInjection.weight (device)            */
    const float *bias;            /* [C] FusedLeakyReLU.bias                       */
    float negative_slope, act_scale;
    const float *s_next;          /* [B,C] or NULL                                 */
    float *y;                     /* [B,H,W,C] or NULL                             */
    const float *rgb_w;           /* [B,3,C] modulated ToRGB weight or NULL        */
    const float *rgb_b;           /* [3]                                           */
    const float *skip;            /* [B,3,H/2,W/2] or NULL                         */
    float *rgb;                   /* [B,3,H,W]                                     */
    /* instead of y: the round-to-nearest fp16 split y = hi + lo in the split-NHWC
     * layout below (the input format of sdfr_conv3x3_f16x3), or NULL */
    void *y_split;
} sdfr_styled_epilogue_args;

int sdfr_styled_epilogue(const sdfr_styled_epilogue_args *a, void *stream);

/* Decoder input staging: y[b,h,w,c] = x[b,c,h,w] * s[b,c] (NCHW -> NHWC with
 * the first ModulatedConv2d's modulation folded in).  C and H*W multiples of 4. */
int sdfr_modulate_to_nhwc(float *y, const float *x, const float *s, uint32_t B, uint32_t C,
                          uint32_t HW, void *stream);
/* The same with y written in the split-NHWC layout (C % 8 == 0).
 *
 * Split-NHWC: the round-to-nearest fp16 split x = hi + lo of an NHWC fp32 tensor,
 * fp16 [B,H,W,C/8,2,8]: per pixel and group of 8 channels, 8 hi then 8 lo
 * halves (32 channels of one pixel = one 128-B line). */
int sdfr_modulate_to_nhwc_split(void *y_split, const float *x, const float *s, uint32_t B,
                                uint32_t C, uint32_t HW, void *stream);

/* ---------------------------------------------------------------------------
 * Decoder 3x3 convolutions on split-fp16 MFMA (no reference counterpart: they
 * replace the MIOpen convolutions of ModulatedConv2d on the fused decoder path,
 * sdf_model.py:676-699, batched form conv(x * s, w) * demod).
 *
 * sdfr_conv_pack_weights: w [Cout][Cin][3][3] (ModulatedConv2d.weight[0]) times
 *   scale -> su [Cout] (per-row power-of-two scale, written) and the packed hi/lo
 *   fp16 fragments (sdfr_conv_pack_bytes(Cout, Cin) - 4*Cout bytes).
 * sdfr_conv3x3_f16x3: input in the split-NHWC layout ([B,H,W,Cin/8,2,8] fp16, as
 *   written by the *_split / y_split outputs above), NHWC fp32 out, result
 *   multiplied by su[o]
 *   (the caller folds 1/su into the demodulation -- exact, powers of two):
 *   transposed = 0: out [B,H,W,Cout] = conv2d(x, w, padding 1);
 *   transposed = 1: out [B,2H+1,2W+1,Cout] = conv_transpose2d(x, w^T, stride 2)
 *   (x [B,H,W,Cin]).  Cout % 128 == 0, Cin % 32 == 0.
 * ------------------------------------------------------------------------- */
size_t sdfr_conv_pack_bytes(uint32_t Cout, uint32_t Cin);
int sdfr_conv_pack_weights(const float *w, float scale, uint32_t Cout, uint32_t Cin,
                           void *packed, float *su, void *stream);
int sdfr_conv3x3_f16x3(float *out, const void *x_split, const void *packed,
                       uint32_t B, uint32_t H, uint32_t W, uint32_t Cin, uint32_t Cout,
                       int transposed, void *stream);
/* The same with a workspace: when the grid would leave CUs idle (small batches,
 * e.g. eval.py's one face) the K-steps of every tile are shared by 2-4 workgroups
 * whose fp32 partial tiles a second kernel sums in a fixed order (deterministic).
 * ws_bytes >= sdfr_conv_ws_bytes(B, H, W, Cout, transposed) enables it (0: no split
 * for this shape; a smaller or NULL workspace runs unsplit). */
int sdfr_conv3x3_f16x3_ws(float *out, const void *x_split, const void *packed,
                          uint32_t B, uint32_t H, uint32_t W, uint32_t Cin, uint32_t Cout,
                          int transposed, void *ws, size_t ws_bytes, void *stream);
size_t sdfr_conv_ws_bytes(uint32_t B, uint32_t H, uint32_t W, uint32_t Cout, int transposed);
/* Which kernel runs the transposed convolution (a process-wide setting, read by both
 * the launch and sdfr_conv_ws_bytes, so they always agree): 1 (default) conv_t_kernel
 * from 256 tiles of 64 channels x 16 x 16 positions, conv_x_kernel's split-K below;
 * 0 always conv_x_kernel; 2 conv_t_kernel at any tile count; 3 as 2 with each tile's
 * channel groups split 2 or 4 ways below 256 tiles (needs the workspace).  The
 * initial value is SDFR_CONV_T from the environment when the library loads (else 1);
 * mode -1 restores it.  Returns the previous mode, or SDFR_EINVAL for another value. */
int sdfr_set_conv_t_mode(int mode);

/* The regular (transposed = 0) convolution with the plain styled epilogue fused
 * into it (the conv output never goes to memory): per pixel and channel
 *   v = lrelu((conv * demod[b,c] + noise_weight * noise[b,h,w]) + bias[c],
 *             negative_slope) * act_scale         (demod already divided by su)
 *   y_split = v * s_next[b,c] in split-NHWC (s_next NULL -> v), when y_split
 *   rgb_partial[k,b,o,h,w] = sum_{c in [128k, 128k+128)} v * rgb_w[b,o,c], when
 *   rgb_w (k < Cout/128; sdfr_rgb_finish adds the parts, bias and skip); or, with
 *   rgb_base instead of rgb_w, rgb_w[b,o,c] = rgb_base[o,c] * rgb_s[b,c] (fp32 product
 *   formed in the kernel: ToRGB's scaled 1x1 weight times the face's style, the
 *   caller's [B,3,Cout] multiply saved).
 * Same operation order as sdfr_styled_epilogue for v and y.  H*W % 256 == 0. */
typedef struct sdfr_conv_act_args {
    const void *x_split;          /* [B,H,W,Cin/8,2,8] fp16                         */
    const void *packed;           /* sdfr_conv_pack_weights                         */
    uint32_t B, H, W, Cin, Cout;
    const float *demod;           /* [B,Cout]                                       */
    const float *noise;           /* [B,H,W] or NULL                                */
    const float *noise_weight;    /* [1] (device)                                   */
    const float *bias;            /* [Cout]                                         */
    float negative_slope, act_scale;
    const float *s_next;          /* [B,Cout] or NULL                               */
    void *y_split;                /* [B,H,W,Cout/8,2,8] fp16 or NULL                */
    const float *rgb_w;           /* [B,3,Cout] modulated ToRGB weight or NULL      */
    float *rgb_partial;           /* [Cout/128,B,3,H,W] fp32 (with rgb_w)           */
    void *ws;                     /* split-K partials or NULL                       */
    size_t ws_bytes;              /* >= sdfr_conv_act_ws_bytes(...) to split        */
    const float *rgb_base;        /* [3,Cout] (rgb_w NULL) or NULL         (ABI 10) */
    const float *rgb_s;           /* [B,Cout] with rgb_base                (ABI 10) */
} sdfr_conv_act_args;

int sdfr_conv3x3_f16x3_act(const sdfr_conv_act_args *a, void *stream);
/* Workspace that lets sdfr_conv3x3_f16x3_act split K when B*H*W/256 * Cout/128
 * workgroups would leave CUs idle (0: no split for this shape): the K-steps are
 * shared by 2 or 4 workgroups per tile, whose fp32 partial tiles a second kernel
 * sums in a fixed order before the epilogue. */
size_t sdfr_conv_act_ws_bytes(uint32_t B, uint32_t H, uint32_t W, uint32_t Cout);

/* The upsampling StyledConv in one call (ABI 13; sdf_model.py:660-701 + 704-818):
 * conv_transpose2d(x, w^T, stride 2) (the packed weights as sdfr_conv3x3_f16x3),
 * Blur(outer(fir, fir), pad (1, 1)) down to 2H x 2W, then per pixel and channel
 *   v = lrelu(blur * demod[b,o] + noise_weight * noise[b,y,x] + bias[o]) * act_scale
 * and y_split = split-NHWC fp16 of v * s_next[b,o] (sdfr_styled_epilogue's blur_up
 * arithmetic, in its order: the same bits as sdfr_conv3x3_f16x3 + that epilogue).
 * The blur and epilogue run inside the conv kernel for each block's interior pixels;
 * `raw` [B,2H+1,2W+1,Cout] fp32 is a workspace that receives only the conv values
 * of the blocks' band rows / columns, from which a second kernel finishes the block
 * border pixels.  Needs sdfr_conv_t_act_supported (H, W % 16 == 0 and at least 256
 * tiles of 64 channels x 16 x 16 positions; SDFR_EUNSUPPORTED otherwise). */
typedef struct sdfr_conv_t_act_args {
    const void *x_split;          /* [B,H,W,Cin/8,2,8] fp16                         */
    const void *packed;           /* sdfr_conv_pack_weights                         */
    uint32_t B, H, W, Cin, Cout;  /* input H x W; output 2H x 2W                    */
    float fir[4];                 /* the blur's 1-D taps                            */
    const float *demod;           /* [B,Cout] (x 1/su)                              */
    const float *noise;           /* [B,2H,2W] or NULL                              */
    const float *noise_weight;    /* [1] (device)                                   */
    const float *bias;            /* [Cout]                                         */
    float negative_slope, act_scale;
    const float *s_next;          /* [B,Cout] or NULL                               */
    void *y_split;                /* [B,2H,2W,Cout/8,2,8] fp16                      */
    float *raw;                   /* [B,2H+1,2W+1,Cout] fp32 workspace              */
} sdfr_conv_t_act_args;
int sdfr_conv_t_act(const sdfr_conv_t_act_args *a, void *stream);
int sdfr_conv_t_act_supported(uint32_t B, uint32_t H, uint32_t W, uint32_t Cin, uint32_t Cout);

/* ToRGB finish: rgb [B,3,H,W] = sum_k partial[k] + rgb_b[o]
 *   + upfirdn2d(skip, outer(fir,fir), up 2, pad (2,1)) when skip != NULL
 * (partial [nparts,B,3,H,W], skip [B,3,H/2,W/2], fir: 4 host floats). */
int sdfr_rgb_finish(float *rgb, const float *partial, uint32_t nparts, const float *rgb_b,
                    const float *skip, const float *fir, uint32_t B, uint32_t H, uint32_t W,
                    void *stream);

/* ---------------------------------------------------------------------------
 * Marching cubes (sdf_mesh.py's surface extraction: sdf_utils.py:188-205, which
 * calls scikit-image's marching_cubes(sdf_vol, 0) on the host; csrc/mesh.hip).
 *
 * Volume: n0 x n1 x n2 fp32 points (each >= 2, 4 n0 n1 n2 + 1 < 2^32) on the
 * device, point (i, j, k) at vol[i s0 + j s1 + k s2] (element strides, so the
 * reference's permute(1, 0, 2) is a stride swap).  A corner is inside when its
 * value < level; vertices lie on the sign-changing grid edges by linear
 * interpolation, in index coordinates (x = i + t ...).
 *
 *   sdfr_mc_count:  classify + scan into ws; writes counts[0] = vertices,
 *                   counts[1] = triangles to HOST memory (synchronises stream)
 *   sdfr_mc_emit:   same volume and ws (after sdfr_mc_count): verts [V,3] fp32,
 *                   faces [F,3] int32 (vertex ids), device
 * ------------------------------------------------------------------------- */
size_t sdfr_mc_workspace_bytes(uint32_t n0, uint32_t n1, uint32_t n2);
int sdfr_mc_count(const float *vol, uint32_t n0, uint32_t n1, uint32_t n2, int64_t s0,
                  int64_t s1, int64_t s2, float level, void *ws, size_t ws_bytes,
                  uint32_t *counts, void *stream);
int sdfr_mc_emit(const float *vol, uint32_t n0, uint32_t n1, uint32_t n2, int64_t s0,
                 int64_t s1, int64_t s2, float level, const void *ws, size_t ws_bytes,
                 float *verts, int32_t *faces, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* SDFR_H_ */
