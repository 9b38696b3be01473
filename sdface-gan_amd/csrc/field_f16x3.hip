// field_f16x3.hip -- the fused renderer's field stage on split-fp16 MFMA, for
// both SDFace networks:
//
//   NgpNet    NGPSIRENGenerator (sdf_model.py:1534-1592): hash-grid features (32)
//             -> input_linear -> 3 FiLM layers -> sigma | [h3, SH(16)] -> views
//             FiLM -> rgb.  Inputs come from the hash-grid encode kernel.
//   SirenNet  SirenGenerator (sdf_model.py:101-139): normalised points (3) -> 8
//             FiLM layers -> sigma | [h7, viewdir(3)] -> views FiLM -> rgb.
//             Points are formed in-kernel from the ray (bit-exact chain).
//
// followed by SDF->density and front-to-back alpha compositing
// (volume_integration, :236-301).  Every fp32 GEMM tile runs as three fp16 MFMAs
// (v_mfma_f32_32x32x16_f16 for ngp, v_mfma_f32_16x16x32_f16 for siren) on a hi/lo
// fp16 split of both operands:
//
//     W.x = W_hi.x_hi + W_hi.x_lo + W_lo.x_hi   (+ W_lo.x_lo, dropped: 2^-22 rel.)
//
// accumulated in fp32 by the matrix core: 5.3x the fp32 MFMA rate.  Accuracy
// (scripts/probe_split_f16.hip, measured on MI355X): a 256-deep dot product is as
// accurate as the fp32 fma chain PROVIDED the fp16 lo parts do not go subnormal --
// so every weight row is scaled by a power of two su (max |w| su in [0.5,1),
// xscale_kernel) and every sample's features by a power of two before the split.
// Power-of-two scaling commutes with rounding, so it is undone exactly: the FiLM
// gamma is divided by su (gamma' x_scaled == gamma x, bit for bit), the layer bias
// folds into the FiLM beta, and the feature scale is taken out in layer 0's FiLM.
//
// Work unit (field_r_kernel below): a workgroup of 4 waves, one per SIMD (512
// VGPRs), over 4 tiles of 16 rays; each wave computes ALL 256 output rows of every
// layer for 32 samples (16 rays x 2 consecutive samples), so a layer's accumulators,
// activated and split in place, are the next layer's B fragments (no LDS hand-off).
// The weight stream (0.8 MB per pass) is shared by the 4 waves through a 4-slot
// LDS-DMA ring of 16 KB slices (one per k-step of 16 K), with the packed weights' K
// permuted to match the accumulator layout (xprep_kernel).  The SIREN net runs on
// field_p_kernel (two waves per SIMD splitting each layer's rows, its own packing:
// 16 KB half-slices per k-step of 32 K), which is 6 % faster on its nine FiLM layers
// -- the one-wave kernel's 32x32 MFMAs hold a lower clock there (1.64 GHz, counters).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "f16x3.h"
#include "render_ngp.h"

namespace sdfr {

constexpr uint32_t kXSliceF4 = 1024;             // 16 KB: [8 tiles][hi,lo][64 lanes] x 16 B
// ----------------------------------------------------------------------------
// network policies.  Weight matrices ("layers") in order: layer 0, the dense
// 256x256 layers, the views layer.  One packed slice per k-step of 16 input features
// (8 output tiles of 32 rows): layer 0 has 2 (ngp, 32 features) or 1 (siren, xyz)
// k-steps, the dense layers 16, the views layer 17 (256 + 16 SH / 3 direction inputs).
// ----------------------------------------------------------------------------
struct NgpNet {
    static constexpr bool kSiren = false;
    static constexpr bool kGrid = true;        // layer-0 inputs from the hash-grid encode kernel
    static constexpr bool kPosEnc = false;     // layer-0 / views inputs: positional encodings
    static constexpr bool kSinAct = true;      // FiLM sin activations (else ReLU)
    static constexpr int kL0 = 2;              // layer-0 k-steps of 16 K
    static constexpr int kViewSteps = 17;      // views-layer k-steps (256 hidden + 16 SH)
    static constexpr bool kFieldR = true;      // field_r_kernel (else field_p_kernel)
    // input_linear (LinearLayer, affine: sdf_model.py:37-39) feeds pts_linears.0's
    // linear with no nonlinearity between them (:1574-1577), so the two are ONE affine
    // map W1 (W0 x + b0) + b1 = (W1 W0) x + (W1 b0 + b1), composed once per weight
    // version in fp64 (compose_kernel): layer 0 is that 32 -> 256 map with
    // pts_linears.0's FiLM, and the 256 x 256 GEMM of pts_linears.0 per sample is gone.
    static constexpr bool kCompose = true;
    static constexpr int kLayers = 4;          // composed 0, pts_linears.1-2, views
    static constexpr int kFilmN = 4;           // FiLM: pts_linears.0-2, views
    static constexpr int kHidden = 2;          // dense layers after layer 0
    static constexpr uint32_t kSlices = 2 + 16 * 2 + 17;     // k-steps of 16 K per pass
    __host__ __device__ static constexpr uint32_t K(int l) {
        return l == 0 ? kFeatIn : (l == 3 ? kViewsIn : kW);
    }
    __host__ __device__ static constexpr int film_layer(int f) { return f; }
};
struct SirenNet {
    static constexpr bool kSiren = true;
    static constexpr bool kGrid = false;
    static constexpr bool kPosEnc = false;
    static constexpr bool kSinAct = true;
    static constexpr int kL0 = 1;
    static constexpr int kViewSteps = 17;
    static constexpr bool kFieldR = false;
    static constexpr bool kCompose = false;
    static constexpr bool kSlice2 = false;
    static constexpr int kLayers = 9;          // pts_linears.0-7, views
    static constexpr int kFilmN = 9;
    static constexpr int kHidden = 7;
    static constexpr uint32_t kSlices = 2 + 16 * 7 + 18;     // field_p_kernel's half-slices
    __host__ __device__ static constexpr uint32_t K(int l) {
        return l == 0 ? 3u : (l == 8 ? kW + 3 : kW);
    }
    __host__ __device__ static constexpr int film_layer(int f) { return f; }
};
// FCGenerator (rendering.fc == 1, sdf_model.py:1599-1670): positional encodings of the
// normalised point (3 x 10 frequencies x sin, cos = 60) -> x_in (+ style_in(styles), a
// per-face bias) -> ReLU -> 7 x (256 -> 256, ReLU) -> sigma | [h7, posenc(view) (24)] ->
// views (no activation: the colour features) -> rgb.  Every layer is affine then ReLU,
// run as ReLU(fma(1/su, z, b)) on the row-scaled GEMM output z (1/su exact), i.e. the
// FiLM slot with gamma'' = 1/su and beta'' = the bias.
struct FcNet {
    static constexpr bool kSiren = false;
    static constexpr bool kGrid = false;
    static constexpr bool kPosEnc = true;
    static constexpr bool kSinAct = false;
    static constexpr int kL0 = 4;              // 60 encodings (+ 4 zero pad)
    static constexpr int kViewSteps = 18;      // 256 hidden + 24 view encodings (+ 8 pad)
    static constexpr bool kFieldR = true;
    static constexpr bool kCompose = false;
    static constexpr int kLayers = 9;          // x_in, pts_linears.0-6, views
    static constexpr int kFilmN = 9;           // (1/su, bias) per layer; layer 0 per face
    static constexpr int kHidden = 7;
    static constexpr uint32_t kSlices = 4 + 16 * 7 + 18;
    static constexpr uint32_t kPosIn = 60, kPosViews = 24;
    __host__ __device__ static constexpr uint32_t K(int l) {
        return l == 0 ? kPosIn : (l == 8 ? kW + kPosViews : kW);
    }
    __host__ __device__ static constexpr int film_layer(int f) { return f; }
};
constexpr int kMaxLayers = 9;

// field_p_kernel's packing (SirenNet): slices = 2 per k-step of 32 input features
// (8 output tiles of 16 rows each); layer 0 one k-step, dense layers 8, views 9.
template <class Net>
__host__ __device__ constexpr uint32_t xslice_base(int l) {
    return l == 0 ? 0u : (l == Net::kLayers - 1 ? 2u + 16u * Net::kHidden : 2u + 16u * (l - 1));
}

// K index of element j of lane group g in field_p_kernel's k-step q of layer l
// (-1 = zero pad).
template <class Net>
__device__ __forceinline__ int xperm_k(int l, uint32_t q, uint32_t g, uint32_t j) {
    if (l == 0) {
        if constexpr (Net::kSiren) return (g == 0 && j < 3) ? (int)j : -1;   // xyz
        return (int)(8 * g + j);                                           // 32 features
    }
    if (l == Net::kLayers - 1 && q == 8) {
        if constexpr (Net::kSiren) return (g == 0 && j < 3) ? (int)(kW + j) : -1;   // viewdir
        return g < 2 ? (int)(kW + 8 * g + j) : -1;                                // SH 0-15
    }
    return (int)(16 * (2 * q + (j >> 2)) + 4 * g + (j & 3));
}

constexpr int kRWaves = 4;
constexpr int kRThreads = kRWaves * 64;
constexpr uint32_t kRTiles = 4;          // 16-ray tiles per workgroup (one per wave)
constexpr uint32_t kRSamples = 2;        // samples of a ray per pass
constexpr uint32_t kRSliceF4 = 1024;     // 16 KB: one k-step's [8 tiles][hi, lo][64 lanes]

typedef float f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f16v mfma32(f4 a, f4 b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(as_h8(a), as_h8(b), c, 0, 0, 0);
}

template <class Net>
struct RNet {
    static constexpr int kL0 = Net::kL0;                           // layer-0 k-steps (K 3 / 32 / 60)
    static constexpr int kSteps = kL0 + 16 * Net::kHidden + Net::kViewSteps;   // (slices) per pass
    static constexpr int kViews = kL0 + 16 * Net::kHidden;         // first views k-step
    static_assert(!Net::kFieldR || kSteps == (int)Net::kSlices, "one packed slice per k-step");
};

template <class Net>
__host__ __device__ constexpr uint32_t rslice_base(int l) {
    return l == 0 ? 0u
                  : (uint32_t)RNet<Net>::kL0 + 16u * (l == Net::kLayers - 1 ? Net::kHidden : l - 1);
}

// K index (within layer l's input) of element j of lane half h in the layer's k-step s
// (-1 = zero pad)
template <class Net>
__device__ __forceinline__ int rperm_k(int l, uint32_t s, uint32_t h, uint32_t j) {
    const uint32_t e = 8 * h + j;
    if (l == 0) {
        if constexpr (Net::kSiren) return e < 3 ? (int)e : -1;   // xyz
        if constexpr (Net::kPosEnc) return 16 * s + e < Net::kPosIn ? (int)(16 * s + e) : -1;
        return (int)(16 * s + e);                               // 32 grid features
    }
    if (l == Net::kLayers - 1 && s >= 16) {
        if constexpr (Net::kSiren) return e < 3 ? (int)(kW + e) : -1;   // viewdir
        if constexpr (Net::kPosEnc)                                     // view encodings
            return 16 * (s - 16) + e < Net::kPosViews ? (int)(kW + 16 * (s - 16) + e) : -1;
        return (int)(kW + e);                                           // SH 0-15
    }
    return (int)(32 * (s >> 1) + 16 * (s & 1) + 8 * (j >> 2) + 4 * h + (j & 3));
}

__device__ __forceinline__ void xpin(f4 &x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void xpin(float &x) { asm volatile("" : "+v"(x)); }
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void xpin(f2v &x) { asm volatile("" : "+v"(x)); }

// field_r_kernel's colour tail (no MFMA beside it: the issue-bound stretch of a pass)
// on packed fp32 (v_pk_fma_f32 / v_pk_mul_f32: two lanes' worth of the same
// element-wise IEEE ops per instruction, results bit-identical); 0 = scalar
#ifndef SDFR_RTAILPK
#define SDFR_RTAILPK 1
#endif
constexpr bool kRTailPk = SDFR_RTAILPK != 0;

// ----------------------------------------------------------------------------
// prep 1: per-row power-of-two scales and scaled biases (one wave per row)
// ----------------------------------------------------------------------------
struct XScaleArgs {
    const float *w[kMaxLayers];
    const float *b[kMaxLayers];
    uint32_t K[kMaxLayers];
    float *su;       // [layers][256]
    float *bias_s;   // [layers][256]
    int raw_bias0;   // layer 0's bias stays unscaled (ngp: added after the GEMM)
};

__global__ void __launch_bounds__(256) xscale_kernel(const XScaleArgs a) {
    const uint32_t layer = blockIdx.x, lane = threadIdx.x & 63u;
    const uint32_t row = blockIdx.y * 4 + (threadIdx.x >> 6);
    const uint32_t K = a.K[layer];
    const float *wr = a.w[layer] + (size_t)row * K;
    float m = 0.0f;                        // max is order-independent: exact
    for (uint32_t k = lane; k < K; k += 64) m = fmaxf(m, fabsf(wr[k]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (lane != 0) return;
    float su = 1.0f;
    if (m > 0.0f && m < 3.0e38f) {
        int ex;
        (void)frexpf(m, &ex);              // m = f 2^ex, f in [0.5, 1)
        ex = ex < -100 ? -100 : (ex > 100 ? 100 : ex);
        su = ldexpf(1.0f, -ex);
    }
    a.su[layer * kW + row] = su;
    a.bias_s[layer * kW + row] =
        (layer == 0 && a.raw_bias0) ? a.b[0][row] : __fmul_rn(a.b[layer][row], su);
}

// prep 0 (ngp): layer 0 = pts_linears.0 o input_linear, one row per block, fp64 sums
// rounded once to fp32: wc = W1 W0 [256][32], bc = W1 b0 + b1 [256]
__global__ void __launch_bounds__(64) compose_kernel(const float *w0, const float *b0,
                                                     const float *w1, const float *b1,
                                                     float *wc, float *bc) {
    const uint32_t i = blockIdx.x, j = threadIdx.x;
    if (j > kFeatIn) return;
    const float *r1 = w1 + (size_t)i * kW;
    double acc = j < kFeatIn ? 0.0 : (double)b1[i];
    for (uint32_t k = 0; k < kW; ++k)
        acc = fma((double)r1[k], j < kFeatIn ? (double)w0[(size_t)k * kFeatIn + j] : (double)b0[k], acc);
    if (j < kFeatIn) wc[(size_t)i * kFeatIn + j] = (float)acc;
    else bc[i] = (float)acc;
}

// ----------------------------------------------------------------------------
// prep 2: FiLM vectors (gamma / su) + split-fp16 weight fragments
// ----------------------------------------------------------------------------
struct XPrepArgs {
    const float *styles;           // [B,256]
    const float *gw[kMaxLayers], *gb[kMaxLayers], *bw[kMaxLayers], *bb[kMaxLayers];
    const float *w[kMaxLayers];
    const float *lb[kMaxLayers];   // layer biases (unscaled)
    const float *su;               // [layers][256]
    float *film;                   // [B][films][2][256]
    f4 *packed;                    // [slices][8][2][64] fp16x8
    uint32_t B;
};

// field_r_kernel's packing (xprep_kernel): slice = one k-step of 16 K,
// [8 tiles of 32 rows][hi, lo][64 lanes], lane l holding W[32 T + (l & 31)][k] for
// k = rperm_k(layer, s, l >> 5, 0..7)
template <class Net>
__device__ __forceinline__ void r_pack(const XPrepArgs &a, uint32_t e) {
    const uint32_t slice = e / 512, rem = e % 512;
    if (slice >= (uint32_t)RNet<Net>::kSteps) return;
    const uint32_t t8 = rem >> 6, lane = rem & 63;
    int layer = 0;
    if (slice >= rslice_base<Net>(Net::kLayers - 1)) layer = Net::kLayers - 1;
    else if (slice >= (uint32_t)RNet<Net>::kL0) layer = 1 + (slice - RNet<Net>::kL0) / 16;
    const uint32_t s = slice - rslice_base<Net>(layer);
    const uint32_t row = 32 * t8 + (lane & 31), h = lane >> 5;
    const uint32_t K = Net::K(layer);
    const float sc = a.su[layer * kW + row];
    float v[8];
#pragma unroll
    for (uint32_t jj = 0; jj < 8; ++jj) {
        const int k = rperm_k<Net>(layer, s, h, jj);
        v[jj] = k < 0 ? 0.0f : __fmul_rn(a.w[layer][(size_t)row * K + k], sc);
    }
    f4 hi, lo;
    split8(v, hi, lo);
    f4 *dst = a.packed + (size_t)slice * kRSliceF4 + t8 * 128 + lane;
    dst[0] = hi;
    dst[64] = lo;
}

// blocks [0, B*films*2*256/4): FiLM rows, one wave per output row (lanes over K,
// butterfly sum); then packing, one (slice, t8, lane) per thread
template <class Net>
__global__ void __launch_bounds__(256) xprep_kernel(const XPrepArgs a) {
    constexpr int NF = Net::kFilmN;
    const uint32_t blk = blockIdx.x, j = threadIdx.x;
    const uint32_t nfilm = a.B * NF * 2 * kW / 4;
    if (blk < nfilm) {
        const uint32_t lane = j & 63u, row_id = blk * 4 + (j >> 6);
        const uint32_t jr = row_id % kW, rest = row_id / kW;
        const uint32_t b = rest / (NF * 2), rem = rest % (NF * 2);
        const uint32_t f = rem >> 1, which = rem & 1;
        const f4 s4 = reinterpret_cast<const f4 *>(a.styles + (size_t)b * kW)[lane];
        // one 256-long dot product per wave: lane l holds k = 4l .. 4l+3
        auto dot = [&](const float *W) {
            const f4 w4 = reinterpret_cast<const f4 *>(W + (size_t)jr * kW)[lane];
            float p = __fmaf_rn(s4.w, w4.w, __fmaf_rn(s4.z, w4.z, __fmaf_rn(s4.y, w4.y, __fmul_rn(s4.x, w4.x))));
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) p = __fadd_rn(p, __shfl_xor(p, o));
            return p;
        };
        if constexpr (Net::kPosEnc) {
            // FCGenerator: gamma'' = 1/su (exact), beta'' = the layer bias, + style_in(s)
            // for x_in (sdf_model.py:1654-1658: x_in(p) + style_in(styles), then ReLU)
            const int l = Net::film_layer(f);
            float v;
            if (which == 0) {
                v = __fdiv_rn(1.0f, a.su[l * kW + jr]);
            } else {
                v = a.lb[l][jr];
                if (f == 0) v = __fadd_rn(v, __fadd_rn(dot(a.gw[0]), a.gb[0][jr]));
            }
            if (lane == 0) a.film[(((size_t)b * NF + f) * 2 + which) * kW + jr] = v;
            return;
        }
        const float lin = __fadd_rn(dot(which ? a.bw[f] : a.gw[f]), (which ? a.bb[f] : a.gb[f])[jr]);
        // LinearLayer: std_init * linear + bias_init (sdf_model.py:39, 58-59).  The
        // activation sin(gamma (W x + b) + beta) of the modulated layer runs as
        // sin_rev(fma(gamma'', z, beta'')) on its bias-free, row-scaled GEMM output
        // z = su W x, in revolutions: gamma'' = gamma / (su 2pi) and
        // beta'' = (gamma b + beta) / 2pi, each one correctly rounded division (in
        // double) of the reference's fp32 gamma, beta and b.  Folding the bias into
        // beta'' leaves the accumulators starting from zero (no bias rows in LDS).
        constexpr double k2pi = 6.283185307179586476925;
        const int l = Net::film_layer(f);
        float v;
        if (which) {
            // gamma of the same row (its wave is another one)
            const float g = __fadd_rn(__fmul_rn(15.0f, __fadd_rn(dot(a.gw[f]), a.gb[f][jr])), 30.0f);
            const float bet = __fadd_rn(__fmul_rn(0.25f, lin), 0.0f);
            v = (float)(((double)g * (double)a.lb[l][jr] + (double)bet) / k2pi);
        } else {
            const float gam = __fadd_rn(__fmul_rn(15.0f, lin), 30.0f);
            v = (float)((double)gam / ((double)a.su[l * kW + jr] * k2pi));
        }
        if (lane == 0) a.film[(((size_t)b * NF + f) * 2 + which) * kW + jr] = v;
        return;
    }
    const uint32_t e = (blk - nfilm) * 256 + j;
    if (e >= Net::kSlices * 512) return;
    if constexpr (Net::kFieldR) {
        r_pack<Net>(a, e);
        return;
    }
    // field_p_kernel's half-slices
    const uint32_t slice = e / 512, rem = e % 512;
    const uint32_t t8 = rem >> 6, lane = rem & 63;
    int layer = 0;
    if (slice >= xslice_base<Net>(Net::kLayers - 1)) layer = Net::kLayers - 1;
    else if (slice >= 2) layer = 1 + (slice - 2) / 16;
    const uint32_t local = slice - xslice_base<Net>(layer);
    const uint32_t q = local >> 1, h = local & 1;
    const uint32_t row = 16 * (8 * h + t8) + (lane & 15), g = lane >> 4;
    const uint32_t K = Net::K(layer);
    const float s = a.su[layer * kW + row];
    float v[8];
#pragma unroll
    for (uint32_t jj = 0; jj < 8; ++jj) {
        const int k = xperm_k<Net>(layer, q, g, jj);
        v[jj] = k < 0 ? 0.0f : __fmul_rn(a.w[layer][(size_t)row * K + k], s);
    }
    f4 hi, lo;
    split8(v, hi, lo);
    f4 *dst = a.packed + (size_t)slice * kXSliceF4 + t8 * 128 + lane;
    dst[0] = hi;
    dst[64] = lo;
}

// ----------------------------------------------------------------------------
// field kernel
// ----------------------------------------------------------------------------
struct XFieldArgs {
    GeomArgs g;
    const float *enc;              // ngp: [L=16][S_total][2]; siren: unused
    const float2 *zd;              // ngp: [S_total] (z, segment length) from the encode kernel
    const f4 *packed;              // [slices][1024]
    const float *film;             // [B][films][2][256], gamma pre-divided by su
    const float *su;               // [layers][256]
    const float *bias_s;           // [layers][256]
    const float *sigma_w, *sigma_b, *rgb_w, *rgb_b, *sigmoid_beta;
    const float *sigma_noise;      // [B,H,W,N] or null (no_sdf only)
    int force_background, with_sdf;
    float *rgb, *features, *sdf, *xyz, *mask;
    _Float16 *feat_split;          // or the features x feat_mod in split-NHWC (ABI 12)
    const float *feat_mod;         // [B][256]
    uint32_t nseg;                 // sample segments per ray (1: whole rays, no merge)
    float *part;                   // nseg > 1: [nseg][kPartQ][rays] segment partials
};

// Small batches (eval.py renders one face per call) fill a fraction of the chip
// with one workgroup per 4 tiles: the 24 samples of a ray are then split into
// nseg segments marched by different workgroups, each compositing its samples
// front to back from T = 1, and field_merge_kernel chains the segments
// (acc = acc_1 + T_1 acc_2 + T_1 T_2 acc_3 ..., T = prod T_k), which is the
// same sum with the transmittance product re-associated (fp32-rounding-level
// differences; tests/test_gpu_render.py compares split and unsplit renders).
// Partials per (segment, ray): 256 features, rgb[3], xyz[3], T, w_last.
constexpr uint32_t kPartQ = kW + 8;

template <int B, int E, class F>
__device__ __forceinline__ void sfor(F &&f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        sfor<B + 1, E>(f);
    }
}

#ifndef SDFR_RVALU
#define SDFR_RVALU 5
#endif
constexpr int kRValuPerMfma = SDFR_RVALU;  // field_r_kernel: VALU slots after each MFMA
#ifndef SDFR_RDS
#define SDFR_RDS 2
#endif
constexpr int kRDsPerMfma = SDFR_RDS;      // field_r_kernel: LDS-read slots after each MFMA
// profiling-only ablations of field_r_kernel (wrong results by construction; bit flags:
// 1 no barrier, 2 no weight DMA after the prologue, 4 no FiLM/sin in the layer
// activations, 8 trivial colour tail, 16 no vmcnt wait before the barrier)
#ifndef SDFR_FABL
#define SDFR_FABL 0
#endif
constexpr int kFAbl = SDFR_FABL;

// ngp layer-0 inputs: the 32 hash-grid features of a sample span the 4 lane
// groups of its column.  They are scaled by the power of two 2^es that brings the
// sample's max |x| into [0.5, 1) before the hi/lo split, so neither fp16 part
// goes subnormal at any table scale (the reference initialises the table to
// U(-1e-4, 1e-4), grid.py:138-140, where unscaled features would lose their lo
// parts); the scaling is exact and undone exactly in act_pair<0>.
__device__ __forceinline__ int feat_scale(float (&v)[8]) {
    float m = 0.0f;
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[j]));
    m = fmaxf(m, __shfl_xor(m, 16));
    m = fmaxf(m, __shfl_xor(m, 32));
    if (!(m > 0.0f && m < 3.0e38f)) return 0;          // zeros (out of bounds) / non-finite
    int ex = __builtin_amdgcn_frexp_expf(m);          // m = f 2^ex, f in [0.5, 1)
    const int es = ex < -100 ? 100 : -ex;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = __builtin_ldexpf(v[j], es);
    return es;
}

constexpr int kRingSlots = 4;                        // weight ring: 4 half-slice slots (16 KB)
constexpr int kDmaPieces = 2;                        // 1 KB LDS-DMA pieces per wave per half-slice

__device__ __forceinline__ float ror8(float v) {   // lane n <- lane (n + 8) mod 16 of its row
    return __builtin_bit_cast(
        float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));
}

// ----------------------------------------------------------------------------
// field_p_kernel: wave pairs split the output rows.
//
// The previous field kernel (field_x2_kernel, git history) gave every wave the WHOLE
// weight matrix against its own 16-sample column, so each A fragment read from LDS fed
// 3 MFMAs and the eight waves of a CU read 8x the weight stream from LDS per pass.
// Here the two waves of a SIMD (w, w + 4) form a pair over 32 samples = 8 rays x 4
// consecutive samples (two MFMA blocks of N = 16: block c, lane n holds sample
// 4p + 2c + (n >= 8) of ray n & 7); wave h of the pair owns the 16-row output tiles
// 2t + h (t = 0..7), so each A fragment feeds 6 MFMAs and LDS A reads halve.  A
// layer's input k-step q (rows 32q .. 32q + 31 = tiles 2q, 2q+1 of the previous
// layer's output) is half in each wave: both activate their tile one k-step ahead
// (FiLM in the MFMA shadow) and write its (hi, lo) dword pairs to their 8-byte half of
// a double-buffered 4 KB exchange slot; after the k-step barrier both read the whole
// fragment back.  Per k-step and wave: 48 MFMAs, 16 A + 4 B ds_read_b128
// (field_x2_kernel: 32 A reads per 48 MFMAs), 4 pieces of the LDS-DMA weight ring.
// Balanced work matters: with one wave activating a whole k-step the other idled at
// the barrier (measured).  The sigma head and the colour head are per-wave half-sums
// over own rows, added in wave order (fp32-rounding-level differences to the previous
// kernel, <= 5e-7); alpha is computed once per sample block by one wave of the pair.
// Four samples of a ray per pass halve the per-ray feature accumulators (4 KB per wave
// in LDS).  Measured alternatives (in git history): issuing the two waves' LDS-DMA at
// different points (+-0), placing their activations after different groups (+5 %),
// the next k-step's B fragments read ahead of the last group (+-0), a packed-fp32
// colour head (raced: see below).
constexpr int kPWaves = 8;
constexpr int kPThreads = kPWaves * 64;
constexpr uint32_t kPTiles = 2;          // 16-ray tiles per workgroup (4 pairs x 8 rays)
constexpr uint32_t kPSamples = 4;        // samples of a ray per pass



template <class Net>
struct PNet {
    static constexpr int kSteps = 1 + 8 * Net::kHidden + 9;   // k-steps per pass
    static constexpr int kViews = 1 + 8 * Net::kHidden;        // first k-step of the views layer
    static_assert(2 * kSteps == (int)Net::kSlices && kSteps % 2 == 0, "ring parity per pass");
};

struct PRing {
    f4 *lds;          // weight ring: 4 half-slice slots of kXSliceF4
    uint2 *xch;       // this pair's exchange: [2 slots][2 blocks][hi, lo][wave h][64 lanes]
    v4i drsrc;
    uint32_t tid, wave, h;
    f4 na[4];         // the next k-step's group-0 A fragments (t0 hi, t0 lo, t1 hi, t1 lo)
};

// One LDS-DMA half-slice (this wave's pieces) with compile-time offsets as immediates
// (with the offsets as SGPR operands the unrolled pass spilled).  Straight-line asm
// only: a branch inside the asm would skip instructions the compiler counts as wait
// states of MFMA -> VALU hazards (measured: nondeterministic colour features).
template <uint32_t SLICE, uint32_t SLOT>
__device__ __forceinline__ void p_dma_i(const PRing &R) {
    const uint32_t sbase = R.wave * (kDmaPieces * 1024u);
    const uint32_t lbase = lds_addr(R.lds) + sbase;
    const uint32_t voff = (R.tid & 63u) * 16u;
#pragma unroll
    for (int k = 0; k < kDmaPieces; ++k) {
        uint32_t keep, so;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_add_u32 m0, %4, %6\n\ts_add_u32 %1, %5, %7\n\ts_nop 0\n\t"
            "buffer_load_dwordx4 %2, %3, %1 offen lds\n\ts_mov_b32 m0, %0"
            : "=&s"(keep), "=&s"(so)
            : "v"(voff), "s"(R.drsrc), "s"(lbase), "s"(sbase),
              "i"(SLOT * kXSliceF4 * 16u + k * 1024u), "i"(SLICE * kXSliceF4 * 16u + k * 1024u)
            : "memory", "scc");
    }
}

// B fragments of exchange chunk q (both blocks): (hi0, lo0, hi1, lo1).  Each 16-B
// fragment element is wave 0's 8 bytes then wave 1's, kept in two planes (one
// ds_write_b64 per wave writes 64 x 8 contiguous bytes: conflict-free; interleaved at a
// 16-B lane stride, as through round 4, the writes were 2-way bank conflicts), read back
// as two ds_read_b64 (conflict-free).
__device__ __forceinline__ void p_read_chunk(const PRing &R, int q, f4 (&b)[4]) {
    const uint2 *s = R.xch + (q & 1) * 512 + (R.tid & 63u);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint2 u0 = s[128 * k], u1 = s[128 * k + 64];
        const uint32_t w[4] = {u0.x, u0.y, u1.x, u1.y};
        b[k] = __builtin_bit_cast(f4, w);
    }
}

// One k-step of one wave: 8 own output tiles x 2 sample blocks x 3 split terms = 48
// MFMAs in 4 groups of 2 tiles (a group's 12 MFMAs term-major, so an accumulator is
// touched every 4th).  Own half-slice of k-step KS: ring slot 2 (KS & 1) + h.  The
// next k-step's half-slices are DMA'd at entry into the previous k-step's slots; the
// barrier (own DMA landed, own LDS traffic drained) sits ahead of group 3, behind it
// the next k-step's group-0 A fragments and B fragments (next_b) are read, so their
// latency hides under group 3.  side() runs after group 1.
template <class Net, int KS, bool ZC, class NextB, class Side>
__device__ __forceinline__ void pstep(PRing &R, f4 (&acc)[16], const f4 (&bf)[4], f4 (&bn)[4],
                                      NextB &&next_b, Side &&side) {
    constexpr f4 kZ = {0.0f, 0.0f, 0.0f, 0.0f};
    constexpr int KN = (KS + 1) % PNet<Net>::kSteps;
    const uint32_t lane = R.tid & 63u;
    // the next k-step's half-slices go into the slots of the previous k-step (closed by
    // its barrier)
    p_dma_i<2 * KN, 2 * (KN & 1)>(R);
    p_dma_i<2 * KN + 1, 2 * (KN & 1) + 1>(R);
    // local tile t = global tile 2t + h: half-slice t >> 2, position 2 (t & 3) + h
    const f4 *A = R.lds + 2 * (KS & 1) * kXSliceF4 + R.h * 128 + lane;
    const f4 *An = R.lds + 2 * (KN & 1) * kXSliceF4 + R.h * 128 + lane;
    auto aoff = [](int t, int hl) { return (t >> 2) * (int)kXSliceF4 + (t & 3) * 256 + hl * 64; };
    f4 a[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[0][i] = R.na[i];
#pragma unroll
    for (int grp = 0; grp < 4; ++grp) {
        if (grp == 3) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        }
        if (grp < 3) {
            const int tn = 2 * (grp + 1);
#pragma unroll
            for (int i = 0; i < 4; ++i) a[grp + 1][i] = A[aoff(tn + (i >> 1), i & 1)];
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) R.na[i] = An[aoff(i >> 1, i & 1)];
        }
        const int t0 = 2 * grp, t1 = t0 + 1;
        const f4 *ag = a[grp];
        // per accumulator: W_lo x_hi, W_hi x_lo, W_hi x_hi
        // ZC: the layer's first k-step starts its accumulators from zero
        acc[2 * t0] = mfma16(ag[1], bf[0], ZC ? kZ : acc[2 * t0]);
        acc[2 * t0 + 1] = mfma16(ag[1], bf[2], ZC ? kZ : acc[2 * t0 + 1]);
        acc[2 * t1] = mfma16(ag[3], bf[0], ZC ? kZ : acc[2 * t1]);
        acc[2 * t1 + 1] = mfma16(ag[3], bf[2], ZC ? kZ : acc[2 * t1 + 1]);
        acc[2 * t0] = mfma16(ag[0], bf[1], acc[2 * t0]);
        acc[2 * t0 + 1] = mfma16(ag[0], bf[3], acc[2 * t0 + 1]);
        acc[2 * t1] = mfma16(ag[2], bf[1], acc[2 * t1]);
        acc[2 * t1 + 1] = mfma16(ag[2], bf[3], acc[2 * t1 + 1]);
        acc[2 * t0] = mfma16(ag[0], bf[0], acc[2 * t0]);
        acc[2 * t0 + 1] = mfma16(ag[0], bf[2], acc[2 * t0 + 1]);
        acc[2 * t1] = mfma16(ag[2], bf[0], acc[2 * t1]);
        acc[2 * t1 + 1] = mfma16(ag[2], bf[2], acc[2 * t1 + 1]);
        // this group's A fragments stay allocated until its MFMAs have issued (pinning
        // the previous group's too measured 1.5 % slower)
        asm volatile("" ::"v"(ag[0]), "v"(ag[1]), "v"(ag[2]), "v"(ag[3]));
        __builtin_amdgcn_sched_barrier(0);
        if (grp == 1) side();
    }
    next_b(bn);
    __builtin_amdgcn_sched_barrier(0);
}

// This wave's half of exchange chunk q (k-step q of the next layer = global tiles
// 2q, 2q+1 of this layer's output; wave h holds tile 2q + h as local tile q):
// activate local tile q of both blocks, split it and write the (hi, lo) dword pairs
// to bytes 8h .. 8h + 7 of the chunk's 16-B B-fragment elements in slot q & 1.
//   MODE 0: ngp layer 0, FiLM of x 2^-es (the features were scaled by 2^es, feat_scale)
//   MODE 1: FiLM sin_rev(fma(gamma'', x, beta''))
//   MODE 2: FiLM + the sigma head's partial dot product (per lane over own tiles)
template <int MODE>
__device__ __forceinline__ void p_act(const PRing &R, f4 (&in)[16], int q, const float *gam,
                                      const float *bet, const float *sw, float (&sdfp)[2],
                                      uint32_t g, const int (&es)[2]) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const int f0 = 16 * (2 * q + (int)R.h) + 4 * (int)g;
    const f4 gm = *reinterpret_cast<const f4 *>(gam + f0);
    const f4 bt = *reinterpret_cast<const f4 *>(bet + f0);
    f4 w4;
    if constexpr (MODE == 2) w4 = *reinterpret_cast<const f4 *>(sw + f0);
    uint2 *dst = R.xch + (q & 1) * 512 + R.h * 64 + (R.tid & 63u);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const f4 z = in[2 * q + c];
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if constexpr (MODE == 0) v[r] = sin_rev(__fmaf_rn(gm[r], __builtin_ldexpf(z[r], -es[c]), bt[r]));
            else v[r] = sin_rev(__fmaf_rn(gm[r], z[r], bt[r]));
        }
        if constexpr (MODE == 2) {
#pragma unroll
            for (int r = 0; r < 4; ++r) sdfp[c] = __fmaf_rn(v[r], w4[r], sdfp[c]);
        }
        uint32_t hp[2], lp[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            h2 H;
            H[0] = (_Float16)v[2 * j];
            H[1] = (_Float16)v[2 * j + 1];
            hp[j] = __builtin_bit_cast(uint32_t, H);
            uint32_t l;
            asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(l) : "v"(hp[j]), "v"(v[2 * j]));
            asm("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
                : "+v"(l) : "v"(hp[j]), "v"(v[2 * j + 1]));
            lp[j] = l;
        }
        dst[256 * c] = make_uint2(hp[0], hp[1]);
        dst[256 * c + 128] = make_uint2(lp[0], lp[1]);
    }
}

template <class Net>
__global__ void __launch_bounds__(kPThreads, 2) field_p_kernel(const XFieldArgs a) {
    constexpr int NF = Net::kFilmN;
    constexpr int KV = PNet<Net>::kViews;
    constexpr int NL = Net::kLayers;
    __shared__ f4 ring_lds[kRingSlots * kXSliceF4];           // 64 KB weight ring
    __shared__ uint2 xch_lds[4][2 * 2 * 2 * 2 * 64];        // 32 KB: [pair][slot][block][hi,lo][h][lane]
    __shared__ f4 facc_lds[kPWaves][8 * 4 * 8];             // 32 KB: [wave][tile][g][ray] feature sums
    __shared__ float film_lds[NF * 2 * kW];                 // the workgroup's face
    __shared__ float cst[4 * kW];                           // sigma_w, rgb_w[3]
    __shared__ float sdfx_lds[4][2][2][64];                 // [pair][wave][block][lane] sigma half-sums
    __shared__ float pcol_lds[4][6][16];                    // wave 0's colour half-sums per column
    __shared__ float alx_lds[4][2][64];                     // [pair][block][lane] alpha
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t h = __builtin_amdgcn_readfirstlane(wave >> 2), pair = wave & 3u;
    const uint32_t n = lane & 15u, g = lane >> 4, r8 = n & 7u;
    const bool colB = n >= 8u;
    const GeomArgs &G = a.g;

    // workgroup = 2 tiles; pair k: tile k >> 1, rays 8 (k & 1) .. +7
    const uint32_t wg_per_face = (G.tiles_per_face + kPTiles - 1) / kPTiles;
    const uint32_t seg = blockIdx.x % a.nseg, blk = blockIdx.x / a.nseg;
    const uint32_t b = blk / wg_per_face;
    const float beta_s = a.with_sdf ? a.sigmoid_beta[0] : 1.0f;
    {
        const f4 *src = reinterpret_cast<const f4 *>(a.film + (size_t)b * NF * 2 * kW);
        f4 *dst = reinterpret_cast<f4 *>(film_lds);
        for (uint32_t i = tid; i < NF * 2 * kW / 4; i += kPThreads) dst[i] = src[i];
    }
    PRing R;
    R.lds = ring_lds;
    R.xch = xch_lds[pair];
    R.tid = tid;
    R.wave = __builtin_amdgcn_readfirstlane(wave);
    R.h = h;
    R.drsrc = make_rsrc(a.packed, Net::kSlices * kXSliceF4 * sizeof(f4));
    for (uint32_t i = tid; i < 4 * kW; i += kPThreads)
        cst[i] = i < kW ? a.sigma_w[i] : a.rgb_w[i - kW];
    // prologue: k-step 0's half-slices -> slots 0, 1 (each k-step issues the next)
    p_dma_i<0, 0>(R);
    p_dma_i<1, 1>(R);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    f4 *facc = facc_lds[wave];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) R.na[i] = R.lds[h * 128 + (i >> 1) * 256 + (i & 1) * 64 + lane];

    const float *sig_w = cst, *rgb_w = cst + kW;
    auto fg = [&](int f) { return (const float *)film_lds + f * 2 * kW; };
    auto fb = [&](int f) { return (const float *)film_lds + f * 2 * kW + kW; };
    const float sig_b = a.sigma_b[0];
    const float rgb_b0 = a.rgb_b[0], rgb_b1 = a.rgb_b[1], rgb_b2 = a.rgb_b[2];
    const float2 *enc2 = reinterpret_cast<const float2 *>(a.enc);
    const uint32_t npass = (G.N + kPSamples - 1) / kPSamples;
    const uint32_t pps = (npass + a.nseg - 1) / a.nseg;
    const uint32_t p_begin = seg * pps, p_end = min(npass, p_begin + pps);

    uint32_t tile_local = (blk % wg_per_face) * kPTiles + (pair >> 1);
    const bool tile_ok = tile_local < G.tiles_per_face;
    if (!tile_ok) tile_local = G.tiles_per_face - 1;
    const uint32_t tile = b * G.tiles_per_face + tile_local;
    const uint32_t ray_in_tile = 8u * (pair & 1u) + r8;
    uint32_t ray_local = tile_local * kTileRays + ray_in_tile;
    const bool ray_ok = tile_ok && ray_local < G.H * G.W;
    if (ray_local >= G.H * G.W) ray_local = G.H * G.W - 1;
    const uint32_t py = ray_local / G.W, px = ray_local % G.W;
    const uint32_t ray_index = (b * G.H + py) * G.W + px;

    Ray ray;
    make_ray(G.cam + (size_t)b * 12, G.focal[b], G.pix_x[px], G.pix_y[py], G.half_res, ray);
    const float nr = G.near_[b], fr = G.far_[b];
    const float span = __fsub_rn(fr, nr);
    const float dnorm = norm3_torch(ray.d[0], ray.d[1], ray.d[2]);
    f4 vx[4];                                               // the views layer's extra k-step
    {
        const float v0 = G.static_viewdirs ? ray.dir[0] : ray.d[0];
        const float v1 = G.static_viewdirs ? ray.dir[1] : ray.d[1];
        const float v2 = G.static_viewdirs ? ray.dir[2] : ray.d[2];
        const float vn = norm3_torch(v0, v1, v2);
        const float ux = __fdiv_rn(v0, vn), uy = __fdiv_rn(v1, vn), uz = __fdiv_rn(v2, vn);
        float v[8];
        if constexpr (Net::kSiren) {
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = 0.0f;
            if (g == 0) {
                v[0] = ux;
                v[1] = uy;
                v[2] = uz;
            }
        } else {
            const f4 qa = sh_quad(ux, uy, uz, (2 * g) & 3), qb = sh_quad(ux, uy, uz, (2 * g + 1) & 3);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = g < 2 ? qa[r] : 0.0f;
                v[4 + r] = g < 2 ? qb[r] : 0.0f;
            }
        }
        split8(v, vx[0], vx[1]);
        vx[2] = vx[0];                                       // both blocks: the same ray
        vx[3] = vx[1];
    }
    float T = 1.0f, wsum = 0.0f, racc0 = 0.0f, racc1 = 0.0f, racc2 = 0.0f;
    float xacc0 = 0.0f, xacc1 = 0.0f, xacc2 = 0.0f, w_last = 0.0f;
#pragma unroll
    for (int t = 0; t < 4; ++t) facc[t * 64 + lane] = f4{0.0f, 0.0f, 0.0f, 0.0f};
    const size_t tile_sid = (size_t)(tile * G.N) * kTileRays + ray_in_tile;
    float2 en[2][4];
    auto load_inputs = [&](uint32_t p) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            uint32_t s = kPSamples * p + 2 * c + (colB ? 1u : 0u);
            if (s >= G.N) s = G.N - 1;
            if constexpr (Net::kSiren) {
                const float z = sample_z(G.sc, nr, fr, ray_index, s);
                float np_[3];
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const float pp = __fadd_rn(ray.o[k], __fmul_rn(ray.d[k], z));
                    np_[k] = G.z_normalize ? __fdiv_rn(__fmul_rn(pp, 2.0f), span) : pp;
                }
                const bool g0 = g == 0;
                en[c][0] = make_float2(g0 ? np_[0] : 0.0f, g0 ? np_[1] : 0.0f);
                en[c][1] = make_float2(g0 ? np_[2] : 0.0f, 0.0f);
                en[c][2] = make_float2(0.0f, 0.0f);
                en[c][3] = make_float2(0.0f, 0.0f);
            } else {
                const size_t sid = tile_sid + (size_t)s * kTileRays;
#pragma unroll
                for (int k = 0; k < 4; ++k) en[c][k] = enc2[(4 * g + k) * (size_t)G.S_total + sid];
            }
        }
    };
    load_inputs(p_begin);

    for (uint32_t p = p_begin; p < p_end; ++p) {
        f4 X[16], Y[16];                                   // [2 local tile + block]
        f4 e[4];                                           // layer-0 B fragments
        int es[2] = {0, 0};
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            float v[8];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                v[2 * k] = en[c][k].x;
                v[2 * k + 1] = en[c][k].y;
            }
            if constexpr (!Net::kSiren) es[c] = feat_scale(v);
            split8(v, e[2 * c], e[2 * c + 1]);
        }
        float sdfp[2] = {0.0f, 0.0f};
        // activation of layer l's output, chunk q, by its owner (wave q >> 2)
        auto act_out = [&](auto L, f4 (&o)[16], int q) {
            constexpr int l = decltype(L)::value;
            constexpr int f = Net::film_layer(l) == l ? l : -1;   // layer l's FiLM
            static_assert(f >= 0, "one FiLM per layer");
            if constexpr (l == 0 && !Net::kSiren) p_act<0>(R, o, q, fg(f), fb(f), nullptr, sdfp, g, es);
            else if constexpr (l == NL - 2) p_act<2>(R, o, q, fg(f), fb(f), sig_w, sdfp, g, es);
            else p_act<1>(R, o, q, fg(f), fb(f), nullptr, sdfp, g, es);
        };
        auto chunk_b = [&](int q) { return [&, q](f4 (&bn)[4]) { p_read_chunk(R, q, bn); }; };
        f4 bn[4];
        // layer 0: one k-step on the encoded inputs; wave 0 activates chunk 0 of its output
        pstep<Net, 0, true>(R, X, e, bn, chunk_b(0), [&] {
            act_out(std::integral_constant<int, 0>{}, X, 0);
        });
        // hidden layers 1 .. kHidden (in -> out alternate between X and Y)
        auto dense = [&](auto L, f4 (&in)[16], f4 (&out)[16]) {
            constexpr int l = decltype(L)::value;
            sfor<0, 8>([&](auto J) {
                constexpr int j = decltype(J)::value;
                constexpr int KS = 1 + 8 * (l - 1) + j;
                f4 bc[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) bc[i] = bn[i];
                pstep<Net, KS, j == 0>(R, out, bc, bn, chunk_b((j + 1) & 7), [&] {
                    if constexpr (j < 7) act_out(std::integral_constant<int, l - 1>{}, in, j + 1);
                    else act_out(std::integral_constant<int, l>{}, out, 0);
                });
            });
        };
        sfor<1, Net::kHidden + 1>([&](auto L) {
            constexpr int l = decltype(L)::value;
            if constexpr (l & 1) dense(L, X, Y);
            else dense(L, Y, X);
        });
        // views layer: input chunks 0-7 (the last hidden layer's output, sigma head
        // chained: wave 0 chunks 0-3, wave 1 continues from its per-lane partial), then
        // the direction k-step; the compositing weights are formed at k-step 7
        constexpr bool kInX = (Net::kHidden & 1) == 0;     // last hidden output array
        f4 (&vin)[16] = kInX ? X : Y;
        f4 (&vout)[16] = kInX ? Y : X;
        const uint32_t s0 = kPSamples * p;
        float z[2] = {0.0f, 0.0f}, wj[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        float sdf_h = 0.0f, dist[2] = {0.0f, 0.0f};
        sfor<0, 9>([&](auto J) {
            constexpr int j = decltype(J)::value;
            constexpr int KS = KV + j;
            f4 bc[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) bc[i] = bn[i];
            if constexpr (j == 5 && !Net::kSiren) {
                // the compositing inputs that do not depend on the network (sample depth,
                // segment length) come from the encode kernel; waited at this barrier
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    uint32_t s = s0 + 2 * c + (colB ? 1u : 0u);
                    if (s >= G.N) s = G.N - 1;
                    const float2 v = a.zd[tile_sid + (size_t)s * kTileRays];
                    z[c] = v.x;
                    dist[c] = v.y;
                }
            }
            if constexpr (j == 7) {
                if (p + 1 < p_end) load_inputs(p + 1);
            }
            auto nb = [&](f4 (&o)[4]) {
                if constexpr (j < 7) {
                    p_read_chunk(R, j + 1, o);
                } else if constexpr (j == 7) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) o[i] = vx[i];
                }
            };
            pstep<Net, KS, j == 0>(R, vout, bc, bn, nb, [&] {
                if constexpr (j < 7) {
                    act_out(std::integral_constant<int, NL - 2>{}, vin, j + 1);
                    if constexpr (j == 6) {
                        // the pair's sigma half-sums, added in wave order after the barrier
                        sdfx_lds[pair][h][0][lane] = group_sum(sdfp[0]);
                        sdfx_lds[pair][h][1][lane] = group_sum(sdfp[1]);
                    }
                } else if constexpr (j == 7) {
                    // alpha of this wave's sample block h (the pair's waves split the
                    // blocks; exchanged through LDS across this k-step's barrier)
                    sdf_h = __fadd_rn(__fadd_rn(sdfx_lds[pair][0][h][lane], sdfx_lds[pair][1][h][lane]),
                                      sig_b);
                    const uint32_t s = s0 + 2 * h + (colB ? 1u : 0u);
                    const bool s_ok = s < G.N;
                    const uint32_t sc_ = s_ok ? s : G.N - 1;
                    if constexpr (Net::kSiren) {
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            const uint32_t sc = min(s0 + 2 * c + (colB ? 1u : 0u), G.N - 1);
                            z[c] = sample_z(G.sc, nr, fr, ray_index, sc);
                        }
                        const float zh = h ? z[1] : z[0];
                        dist[0] = dist[1] = (sc_ + 1 < G.N)
                                      ? __fmul_rn(__fsub_rn(sample_z(G.sc, nr, fr, ray_index, sc_ + 1), zh), dnorm)
                                      : __fmul_rn(1e10f, dnorm);
                    }
                    const float dh = h ? dist[1] : dist[0];
                    float alpha;
                    if (a.with_sdf) {
                        const float sig = __fdiv_rn(sigmoidf_(__fdiv_rn(-sdf_h, beta_s)), beta_s);
                        alpha = 1.0f - expf(-sig * dh);
                    } else {
                        float raw = sdf_h;
                        if (a.sigma_noise) raw += a.sigma_noise[(size_t)ray_index * G.N + sc_];
                        const float sp = raw > 20.0f ? raw : log1pf(expf(raw));
                        alpha = 1.0f - expf(-sp * dh);
                    }
                    alx_lds[pair][h][lane] = s_ok ? alpha : 0.0f;
                } else {
                    // compositing weights of the pass's 4 samples, identically in both
                    // lanes of a ray and both waves of the pair, front to back
                    const float al0 = alx_lds[pair][0][lane], al1 = alx_lds[pair][1][lane];
                    const float o0 = ror8(al0), o1 = ror8(al1);
                    const float aj[4] = {colB ? o0 : al0, colB ? al0 : o0, colB ? o1 : al1,
                                         colB ? al1 : o1};
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const uint32_t s = s0 + k;
                        if (s < G.N) {
                            float w = aj[k] * T;
                            if (a.force_background && s + 1 == G.N) w = 1.0f - wsum;
                            T = T * ((1.0f - aj[k]) + 1e-10f);
                            wsum += w;
                            wj[k] = w;
                        }
                    }
                }
            });
        });
        // colour features f = sin(gamma_v x + beta_v) of the own rows, rgb half-sums.
        // (Scalar fp32: a v_pk_fma_f32 form of this tail read some v_sin_f32 results
        // before they were written -- nondeterministic colour features -- so there is no
        // packed math in this kernel; tests/test_gpu_render.py::test_fused_render_deterministic.)
        const float *f3g = fg(NF - 1), *f3b = fb(NF - 1);
        float P[3][2] = {{0.0f, 0.0f}, {0.0f, 0.0f}, {0.0f, 0.0f}};   // [rgb][block] half-sums
        {
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int f0 = 16 * (2 * t + (int)h) + 4 * (int)g;
                const f4 gm = *reinterpret_cast<const f4 *>(f3g + f0);
                const f4 bt = *reinterpret_cast<const f4 *>(f3b + f0);
                const f4 w0 = *reinterpret_cast<const f4 *>(rgb_w + f0);
                const f4 w1 = *reinterpret_cast<const f4 *>(rgb_w + kW + f0);
                const f4 w2 = *reinterpret_cast<const f4 *>(rgb_w + 2 * kW + f0);
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    f4 fv;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        fv[r] = sin_rev(__fmaf_rn(gm[r], vout[2 * t + c][r], bt[r]));
                        P[0][c] = __fmaf_rn(fv[r], w0[r], P[0][c]);
                        P[1][c] = __fmaf_rn(fv[r], w1[r], P[1][c]);
                        P[2][c] = __fmaf_rn(fv[r], w2[r], P[2][c]);
                    }
                    vout[2 * t + c] = fv;
                }
            }
        }
        float pc[2][3];
#pragma unroll
        for (int o = 0; o < 3; ++o) {
            pc[0][o] = group_sum(P[o][0]);
            pc[1][o] = group_sum(P[o][1]);
        }
        if (h == 0 && g == 0) {
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int o = 0; o < 3; ++o) pcol_lds[pair][3 * c + o][n] = pc[c][o];
        }
        if (a.features) {
            // facc += w0 f0 + w1 f1 + w2 f2 + w3 f3 (in that order) by the lane of the
            // ray's samples 0 and 2 (block 0 / 1, n < 8)
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                f4 o0, o1;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    o0[r] = ror8(vout[2 * t][r]);
                    o1[r] = ror8(vout[2 * t + 1][r]);
                }
                if (!colB) {
                    f4 v = facc[(t * 4 + g) * 8 + r8];
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        v[r] = __fmaf_rn(wj[3], o1[r], __fmaf_rn(wj[2], vout[2 * t + 1][r],
                                         __fmaf_rn(wj[1], o0[r], __fmaf_rn(wj[0], vout[2 * t][r], v[r]))));
                    facc[(t * 4 + g) * 8 + r8] = v;
                }
            }
        }
        if (a.sdf && ray_ok && g == 0) {
            const uint32_t s = s0 + 2 * h + (colB ? 1u : 0u);   // this wave's block
            if (s < G.N) a.sdf[(size_t)ray_index * G.N + s] = sdf_h;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (h == 1) {
            float q[2][3];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                q[c][0] = sigmoidf_(__fadd_rn(__fadd_rn(pcol_lds[pair][3 * c][n], pc[c][0]), rgb_b0));
                q[c][1] = sigmoidf_(__fadd_rn(__fadd_rn(pcol_lds[pair][3 * c + 1][n], pc[c][1]), rgb_b1));
                q[c][2] = sigmoidf_(__fadd_rn(__fadd_rn(pcol_lds[pair][3 * c + 2][n], pc[c][2]), rgb_b2));
            }
            float racc[3] = {racc0, racc1, racc2};
#pragma unroll
            for (int o = 0; o < 3; ++o) {
                const float e0 = ror8(q[0][o]), e1 = ror8(q[1][o]);
                const float qj[4] = {colB ? e0 : q[0][o], colB ? q[0][o] : e0, colB ? e1 : q[1][o],
                                     colB ? q[1][o] : e1};
                float v = racc[o];
#pragma unroll
                for (int k = 0; k < 4; ++k) v = __fmaf_rn(wj[k], qj[k], v);
                racc[o] = v;
            }
            racc0 = racc[0];
            racc1 = racc[1];
            racc2 = racc[2];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (s0 + k < G.N) w_last = wj[k];
            if (a.xyz) {
                const float e0 = ror8(z[0]), e1 = ror8(z[1]);
                const float zj[4] = {colB ? e0 : z[0], colB ? z[0] : e0, colB ? e1 : z[1],
                                     colB ? z[1] : e1};
                float xa[3] = {xacc0, xacc1, xacc2};
#pragma unroll
                for (int k = 0; k < 4; ++k)
#pragma unroll
                    for (int d = 0; d < 3; ++d)
                        xa[d] = __fmaf_rn(wj[k], __fadd_rn(ray.o[d], __fmul_rn(ray.d[d], zj[k])), xa[d]);
                xacc0 = xa[0];
                xacc1 = xa[1];
                xacc2 = xa[2];
            }
        }
    }
    // the ring runs ahead across passes: no LDS-DMA may land after the workgroup ends
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!ray_ok || colB) return;
    if (a.nseg > 1) {
        const size_t Rr = (size_t)G.total_tiles * kTileRays;
        float *pp = a.part + (size_t)seg * kPartQ * Rr + (size_t)tile * kTileRays + ray_in_tile;
        if (a.features) {
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const uint32_t jf = 16 * (2 * t + h) + 4 * g;
                const f4 v = facc[(t * 4 + g) * 8 + r8];
                pp[(size_t)(jf + 0) * Rr] = v.x;
                pp[(size_t)(jf + 1) * Rr] = v.y;
                pp[(size_t)(jf + 2) * Rr] = v.z;
                pp[(size_t)(jf + 3) * Rr] = v.w;
            }
        }
        if (h == 1 && g == 0) {
            const float q[8] = {racc0, racc1, racc2, xacc0, xacc1, xacc2, T, w_last};
#pragma unroll
            for (int k = 0; k < 8; ++k) pp[(size_t)(kW + k) * Rr] = q[k];
        }
        return;
    }
    const size_t HW = (size_t)G.H * G.W;
    const size_t pix = (size_t)py * G.W + px;
    if (h == 1) {
        if (g < 3) {
            const float rc = g == 0 ? racc0 : (g == 1 ? racc1 : racc2);
            a.rgb[((size_t)b * 3 + g) * HW + pix] = __fadd_rn(-1.0f, __fmul_rn(2.0f, rc));
            if (a.xyz) {
                const float xc = g == 0 ? xacc0 : (g == 1 ? xacc1 : xacc2);
                a.xyz[((size_t)b * 3 + g) * HW + pix] = xc;
            }
        } else if (a.mask) {
            a.mask[(size_t)b * HW + pix] = w_last;
        }
    }
    if (a.features) {
        float *fbp = a.features + (size_t)b * kW * HW + pix;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const uint32_t jf = 16 * (2 * t + h) + 4 * g;
            const f4 v = facc[(t * 4 + g) * 8 + r8];
            fbp[(size_t)(jf + 0) * HW] = v.x;
            fbp[(size_t)(jf + 1) * HW] = v.y;
            fbp[(size_t)(jf + 2) * HW] = v.z;
            fbp[(size_t)(jf + 3) * HW] = v.w;
        }
    }
}

// ----------------------------------------------------------------------------
// field_r_kernel: one wave per SIMD on v_mfma_f32_32x32x16_f16.
//
// Design history (round 4, measured, git history): round 3's field_p_kernel put two waves
// on each SIMD (256 VGPRs each) that split every layer's rows and handed each layer's
// input across through LDS (exchange writes, B reads, 2-way bank conflicts); a one-wave
// 16x16x32 variant (field_q_kernel) removed the hand-off and ran at the same speed
// (55 % MFMA busy, 34 % of wave cycles waiting on issue: a 16-cycle MFMA leaves one wave
// two issue slots).  This kernel issues 32x32x16 MFMAs (32 cycles, the vector issue held
// for 8 of them): the same work per FLOP with three times the free issue slots.
// Opaque-register ablations (scripts/build_variants.sh; a plain "reuse the A registers"
// ablation lets hipcc merge identical MFMA chains and is invalid) priced the parts per
// SIMD: the A-fragment LDS reads ~1 % of cycles, the LDS-DMA issue ~8 %, a barrier per
// k-step ~9 % (now one per k-step pair), the colour tail ~13 % (now software pipelined).
//
// Work unit: a workgroup of 4 waves (one per SIMD, 512 VGPRs) over 4 tiles of 16 rays;
// wave w takes tile w, 2 samples of each of its 16 rays per pass: MFMA column
// c = lane & 31 is ray c & 15, sample 2p + (c >> 4); lane half h = lane >> 5.  Output
// tile T (32 rows of a 256-wide layer) is 16 accumulators per lane, register v holding
// row 32 T + (v & 3) + 8 (v >> 2) + 4 h.  Registers 8 s' .. 8 s' + 7 (s' = 0, 1) of a tile,
// activated and split, are the B fragment of k-step 2 T + s' of the next layer (element
// j = row 32 T + 16 s' + 8 (j >> 2) + 4 h + (j & 3)); the packed weights permute K to match
// (xprep_kernel, rperm_k).  Per k-step (16 K) and wave: 8 tiles x 3 split terms = 24
// MFMAs (768 cycles), 16 A ds_read_b128, 4 LDS-DMA pieces of the 16 KB weight slice.
struct RRing {
    f4 *lds;          // weight ring: 4 slots of kRSliceF4
    v4i drsrc;
    uint32_t tid, wave;
    uint32_t ubase;   // ring half of the pass's unit 0 (units per pass may be odd)
    f4 na[3][2];      // the next k-step's groups 0-2 A fragments (hi, lo)
};

// this wave's 4 pieces of slice SLICE -> ring slot `slot` (instruction offsets 0..3 KB
// move the global and the LDS address alike)
template <uint32_t SLICE>
__device__ __forceinline__ void r_dma(const RRing &R, uint32_t slot) {
    const uint32_t sbase = R.wave * 4096u;
    const uint32_t lbase = lds_addr(R.lds) + sbase + slot * (kRSliceF4 * 16u);
    const uint32_t voff = (R.tid & 63u) * 16u;
    uint32_t keep, so;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_add_u32 %1, %5, %6\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %2, %3, %1 offen lds\n\t"
        "buffer_load_dwordx4 %2, %3, %1 offen offset:1024 lds\n\t"
        "buffer_load_dwordx4 %2, %3, %1 offen offset:2048 lds\n\t"
        "buffer_load_dwordx4 %2, %3, %1 offen offset:3072 lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep), "=&s"(so)
        : "v"(voff), "s"(R.drsrc), "s"(lbase), "s"(sbase), "i"(SLICE * kRSliceF4 * 16u)
        : "memory", "scc");
}

// Ring units: k-steps (2u, 2u + 1) of a pass, the last k-step alone when a pass has an odd
// count; unit U (counted over all passes) holds the ring half U & 1 (slots 2 (U & 1) +
// 0, 1).  One barrier per unit, in its last k-step: behind it unit U + 2 is DMA'd into
// unit U's half.
template <class Net>
__device__ __forceinline__ uint32_t r_slot(const RRing &R, int ks) {
    return 2u * ((R.ubase + (uint32_t)(ks >> 1)) & 1u) + (uint32_t)(ks & 1);
}

// DMA of slice `piece` (0, 1) of in-pass unit V into ring half `half`
template <class Net, int V, int PIECE>
__device__ __forceinline__ void r_dma_unit(const RRing &R, uint32_t half) {
    constexpr int NS = RNet<Net>::kSteps;
    if constexpr (2 * V + PIECE < NS) r_dma<2 * V + PIECE>(R, 2u * half + PIECE);
}

// One LDS-DMA piece: this wave's 1 KB at offset K KB of its 4 KB share of slice SLICE
template <uint32_t SLICE, uint32_t K>
__device__ __forceinline__ void r_dma1(const RRing &R, uint32_t slot) {
    const uint32_t sbase = R.wave * 4096u;
    const uint32_t lbase = lds_addr(R.lds) + sbase + slot * (kRSliceF4 * 16u);
    const uint32_t voff = (R.tid & 63u) * 16u;
    uint32_t so;
    // (M0 is not restored: no compiler-generated code in field_r_kernel reads M0 --
    // checked in the ISA, as for the conv kernels' set_m0)
    asm volatile(
        "s_mov_b32 m0, %3\n\ts_add_u32 %0, %4, %5\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, %0 offen offset:%6 lds"
        : "=&s"(so)
        : "v"(voff), "s"(R.drsrc), "s"(lbase), "s"(sbase), "i"(SLICE * kRSliceF4 * 16u),
          "i"(K * 1024u)
        : "memory", "scc");
}

// Piece P (0..7: slice P >> 2, 1 KB part P & 3) of in-pass unit V (V >= units per pass:
// the next pass's unit V - UPP) into ring half `half`
template <class Net, int V, int P>
__device__ __forceinline__ void r_dma_piece(const RRing &R, uint32_t half) {
    constexpr int NS = RNet<Net>::kSteps, UPP = (NS + 1) / 2;
    constexpr int S = 2 * (V % UPP) + (P >> 2);
    if constexpr (S < NS) r_dma1<(uint32_t)S, (uint32_t)(P & 3)>(R, 2u * half + (uint32_t)(P >> 2));
}

// field_r_kernel's weight DMA placement: 1 = one piece per MFMA group, three behind the
// unit's barrier (groups 5-7) and five in the next k-step (groups 0-4); 0 = a whole
// slice at each of groups 5 and 6 (round 4)
#ifndef SDFR_RSPREAD
#define SDFR_RSPREAD 1
#endif
constexpr bool kRSpread = SDFR_RSPREAD != 0;

// One k-step of one wave: 8 output tiles x 3 split terms = 24 MFMAs in 8 groups of one
// tile.  Group gi's A fragments (hi, lo) were read during group gi - 3 (groups 0-2: by the
// previous k-step, R.na).  In a unit's last k-step the barrier (this wave's DMA of the next
// unit landed, its A reads of this unit done) sits ahead of group 5; behind it the unit
// after next is DMA'd (one slice at group 5, one at group 6) into this unit's half, and the
// next k-step's groups 0-2 A fragments are read.  side(gi) runs between group gi's MFMAs.
template <class Net, int KS, bool ZC, class Side>
__device__ __forceinline__ void rstep(RRing &R, f16v (&acc)[8], const f4 (&bf)[2], Side &&side) {
    constexpr int NS = RNet<Net>::kSteps;
    constexpr int UPP = (NS + 1) / 2;                       // units per pass
    constexpr bool kBar = (KS & 1) || KS == NS - 1;         // the unit's last k-step
    constexpr int U = KS >> 1;
    constexpr int VN = (U + 2) % UPP;                       // the unit DMA'd behind the barrier
    const uint32_t lane = R.tid & 63u;
    const f4 *A = R.lds + r_slot<Net>(R, KS) * kRSliceF4 + lane;
    const f4 *An = R.lds + r_slot<Net>(R, KS + 1) * kRSliceF4 + lane;
    const uint32_t half = (R.ubase + (uint32_t)U) & 1u;     // = the half of unit U + 2
    f4 a[8][2];
#pragma unroll
    for (int g = 0; g < 3; ++g) {
        a[g][0] = R.na[g][0];
        a[g][1] = R.na[g][1];
    }
    sfor<0, 8>([&](auto GI) {
        constexpr int gi = decltype(GI)::value;
        if constexpr (kBar && gi == 5) {
            if constexpr (!(kFAbl & 16)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if constexpr (!(kFAbl & 1)) __builtin_amdgcn_s_barrier();
        }
        if constexpr (kRSpread && !(kFAbl & 2)) {
            // the unit's barrier releases unit U + 2's pieces 0-2 here (groups 5-7) and
            // 3-7 in the first k-step of unit U + 1 (groups 0-4): at KS (a unit's first
            // k-step) those are unit U + 1's (behind the previous k-step's barrier; in a
            // workgroup's first pass they repeat the prologue's bytes)
            // (a pass with an odd k-step count ends in a one-k-step unit whose barrier
            // would wait on pieces issued just before it: the unit before it issues all
            // eight of unit U + 2's pieces behind its own barrier, 3 + 3 + 2)
            constexpr bool kOdd = (NS & 1) != 0;
            constexpr bool kLastSingle = kOdd && KS == NS - 1;
            constexpr bool kBeforeSingle = kOdd && KS == NS - 2;
            if constexpr (kBar && gi >= 5) {
                if constexpr (kBeforeSingle) {
                    sfor<3 * (gi - 5), (3 * (gi - 4) < 8 ? 3 * (gi - 4) : 8)>([&](auto PP) {
                        r_dma_piece<Net, U + 2, decltype(PP)::value>(R, half);
                    });
                } else {
                    r_dma_piece<Net, U + 2, gi - 5>(R, half);
                }
            }
            if constexpr ((KS & 1) == 0 && !kLastSingle && gi < 5)
                r_dma_piece<Net, U + 1, gi + 3>(R, (R.ubase + (uint32_t)U + 1u) & 1u);
        } else {
            if constexpr (kBar && gi == 5 && !(kFAbl & 2)) r_dma_unit<Net, VN, 0>(R, half);
            if constexpr (kBar && gi == 6 && !(kFAbl & 2)) r_dma_unit<Net, VN, 1>(R, half);
        }
        if constexpr (gi + 3 < 8) {
            a[gi + 3][0] = A[(gi + 3) * 128];
            a[gi + 3][1] = A[(gi + 3) * 128 + 64];
        } else if constexpr (KS + 1 < NS) {
            // (the next pass's first fragments are read after the pass tail, r_na)
            R.na[gi - 5][0] = An[(gi - 5) * 128];
            R.na[gi - 5][1] = An[(gi - 5) * 128 + 64];
        }
        side(GI);
        constexpr f16v kZ = {};
        // W_lo x_hi, W_hi x_lo, W_hi x_hi
        acc[gi] = mfma32(a[gi][1], bf[0], ZC ? kZ : acc[gi]);
        acc[gi] = mfma32(a[gi][0], bf[1], acc[gi]);
        acc[gi] = mfma32(a[gi][0], bf[0], acc[gi]);
        asm volatile("" ::"v"(a[gi][0]), "v"(a[gi][1]));
        sfor<0, 3>([&](auto I) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, kRDsPerMfma, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, kRValuPerMfma, 0);
        });
        __builtin_amdgcn_sched_barrier(0);
    });
}

// groups 0-2 A fragments of the k-step in ring slot `slot` (landed: behind its barrier)
__device__ __forceinline__ void r_na(RRing &R, uint32_t slot) {
    const f4 *A = R.lds + slot * kRSliceF4 + (R.tid & 63u);
#pragma unroll
    for (int g = 0; g < 3; ++g) {
        R.na[g][0] = A[g * 128];
        R.na[g][1] = A[g * 128 + 64];
    }
}

// FiLM activation of registers 8 s' .. 8 s' + 7 of output tile T into v[8] (element j =
// register 8 s' + j): film rows 32 T + 16 s' + 4 h + (0..3) (gm0, bt0, w0) and + 8 (gm1, ...);
// SIN false: ReLU(fma(1/su, z, b)) (FcNet)
template <int MODE, bool SIN = true>
__device__ __forceinline__ void r_act(const f16v &z, int sp, const f4 &gm0, const f4 &bt0,
                                      const f4 &w0, const f4 &gm1, const f4 &bt1, const f4 &w1,
                                      float &sdfp, int es, float (&v)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float zz = z[8 * sp + j];
        const float g = j < 4 ? gm0[j & 3] : gm1[j & 3], b = j < 4 ? bt0[j & 3] : bt1[j & 3];
        if constexpr (kFAbl & 4) v[j] = zz;
        else if constexpr (!SIN) v[j] = fmaxf(__fmaf_rn(g, zz, b), 0.0f);
        else if constexpr (MODE == 0) v[j] = sin_rev(__fmaf_rn(g, __builtin_ldexpf(zz, -es), b));
        else v[j] = sin_rev(__fmaf_rn(g, zz, b));
        if constexpr (MODE == 2) sdfp = __fmaf_rn(v[j], j < 4 ? w0[j & 3] : w1[j & 3], sdfp);
    }
}

// v_permlane16_swap of (pa, pb) between the two 16-lane rows of each pair: the even
// row gets pa(even) + pa(odd), the odd row pb(even) + pb(odd).  The results pass through
// an empty asm: on float values bit-cast to the builtin's operands, hipcc (ROCm 7.2)
// returned the first result twice (checked on a probe kernel's ISA).
__device__ __forceinline__ float row_pair_sum(float pa, float pb) {
    const auto sw = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(uint32_t, pa),
                                                     __builtin_bit_cast(uint32_t, pb), false, false);
    uint32_t r0 = sw[0], r1 = sw[1];
    asm volatile("" : "+v"(r0), "+v"(r1));
    return __fadd_rn(__builtin_bit_cast(float, r0), __builtin_bit_cast(float, r1));
}

// Round-to-nearest hi / lo fp16 split of channels c .. c + 3 of an 8-channel group held
// by lane half h (lanes l, l ^ 32 hold channels 0-3 and 4-7) into split-NHWC
// ([pixel][C / 8][hi 8, lo 8]; idx8 = NHWC element index of the group's channel 0): one
// v_permlane32_swap per dword gives lane h = 0 both hi halves and lane h = 1 both lo
// halves, so each lane issues one 16-B store.  Both lanes of a pair must execute it.
// (integer operands, results pinned as for row_pair_sum)
typedef _Float16 h4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store_split8_pair32(_Float16 *ys, size_t idx8, f4 v, uint32_t h) {
    // v pinned: hipcc otherwise folds the caller's fp32 product into the fp16 conversion
    // (v_fma_mixlo_f16: one rounding instead of modulate_nhwc_kernel's two -- a tie of
    // the fp32 product then rounds the other way)
    asm volatile("" : "+v"(v));
    h4f hi, lo;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        hi[r] = (_Float16)v[r];
        lo[r] = (_Float16)(v[r] - (float)hi[r]);
    }
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    const u2 hd = __builtin_bit_cast(u2, hi), ld = __builtin_bit_cast(u2, lo);
    uint32_t q[4];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const auto sw = __builtin_amdgcn_permlane32_swap(hd[k], ld[k], false, false);
        uint32_t r0 = sw[0], r1 = sw[1];
        asm volatile("" : "+v"(r0), "+v"(r1));
        q[k] = r0;          // h = 0: own hi / h = 1: partner's lo
        q[2 + k] = r1;      // h = 0: partner's hi / h = 1: own lo
    }
    *reinterpret_cast<f4 *>(ys + 2 * idx8 + (h ? 8 : 0)) = __builtin_bit_cast(f4, q);
}

// Element e of FCGenerator.transform_points (sdf_model.py:1628-1640) of ph = p / 2:
// e = 6 i + r, sin (r < 3) or cos (r >= 3) of (2^i pi) ph[r mod 3], with the reference's
// fp32 argument RN(RN32(2^i pi) ph) (a Python float times an fp32 tensor).  The sine of
// that fp32 argument: reduced to revolutions in fp64 (exact product, fraction to 2^-40),
// then v_sin_f32 (< 1e-6 absolute, tests/test_gpu_encoders.py).
__device__ __forceinline__ float posenc_val(const float (&ph)[3], uint32_t e) {
    const uint32_t i = e / 6u, r = e - 6u * i;
    const uint32_t c = r < 3u ? r : r - 3u;
    const float pc = c == 0u ? ph[0] : (c == 1u ? ph[1] : ph[2]);
    const float arg = __fmul_rn(__builtin_ldexpf(3.14159265358979323846f, (int)i), pc);
    double u = (double)arg * 0.15915494309189533577;     // 1 / (2 pi)
    if (r >= 3u) u += 0.25;                               // cos x = sin(x + pi / 2)
    u -= floor(u);
    return sin_rev((float)u);
}

template <class Net>
__global__ void __launch_bounds__(kRThreads, 1) field_r_kernel(const XFieldArgs a) {
    constexpr int NF = Net::kFilmN;
    constexpr int KV = RNet<Net>::kViews;
    constexpr int KL0 = RNet<Net>::kL0;
    constexpr int NS = RNet<Net>::kSteps;
    constexpr int NL = Net::kLayers;
    __shared__ f4 ring_lds[4 * kRSliceF4];                  // 64 KB weight ring
    __shared__ f4 facc_lds[kRWaves][16][64];                // 64 KB: [wave][f4 of 64 features][lane]
    __shared__ float film_lds[NF * 2 * kW];                 // the workgroup's face
    __shared__ float cst[4 * kW];                           // sigma_w, rgb_w[3]
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t c = lane & 31u, h = lane >> 5, r16 = c & 15u;
    const bool odd = c >= 16u;                              // sample 2p + 1 of the pass
    const GeomArgs &G = a.g;

    const uint32_t wg_per_face = (G.tiles_per_face + kRTiles - 1) / kRTiles;
    const uint32_t seg = blockIdx.x % a.nseg, blk = blockIdx.x / a.nseg;
    const uint32_t b = blk / wg_per_face;
    const float beta_s = a.with_sdf ? a.sigmoid_beta[0] : 1.0f;
    {
        const f4 *src = reinterpret_cast<const f4 *>(a.film + (size_t)b * NF * 2 * kW);
        f4 *dst = reinterpret_cast<f4 *>(film_lds);
        for (uint32_t i = tid; i < NF * 2 * kW / 4; i += kRThreads) dst[i] = src[i];
    }
    RRing R;
    R.lds = ring_lds;
    R.tid = tid;
    R.wave = wave;
    R.ubase = 0;
    R.drsrc = make_rsrc(a.packed, Net::kSlices * kXSliceF4 * sizeof(f4));
    for (uint32_t i = tid; i < 4 * kW; i += kRThreads)
        cst[i] = i < kW ? a.sigma_w[i] : a.rgb_w[i - kW];
    // prologue: units 0, 1 (slices 0-3) -> slots 0-3 (unit U's barrier issues unit U + 2)
    r_dma<0>(R, 0);
    r_dma<1>(R, 1);
    r_dma<2>(R, 2);
    r_dma<3>(R, 3);
    f4 *facc = &facc_lds[wave][0][lane];
#pragma unroll
    for (int t = 0; t < 16; ++t) facc[t * 64] = f4{0.0f, 0.0f, 0.0f, 0.0f};
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    const float *sig_w = cst, *rgb_w = cst + kW;
    auto fg = [&](int f) { return (const float *)film_lds + f * 2 * kW; };
    auto fb = [&](int f) { return (const float *)film_lds + f * 2 * kW + kW; };
    const float sig_b = a.sigma_b[0];
    const float rgb_b0 = a.rgb_b[0], rgb_b1 = a.rgb_b[1], rgb_b2 = a.rgb_b[2];
    const uint32_t npass = (G.N + kRSamples - 1) / kRSamples;
    const uint32_t pps = (npass + a.nseg - 1) / a.nseg;
    const uint32_t p_begin = seg * pps, p_end = min(npass, p_begin + pps);

    uint32_t tile_local = (blk % wg_per_face) * kRTiles + wave;
    const bool tile_ok = tile_local < G.tiles_per_face;
    if (!tile_ok) tile_local = G.tiles_per_face - 1;
    const uint32_t tile = b * G.tiles_per_face + tile_local;
    uint32_t ray_local = tile_local * kTileRays + r16;
    const bool ray_ok = tile_ok && ray_local < G.H * G.W;
    if (ray_local >= G.H * G.W) ray_local = G.H * G.W - 1;
    const uint32_t py = ray_local / G.W, px = ray_local % G.W;
    const uint32_t ray_index = (b * G.H + py) * G.W + px;

    Ray ray;
    make_ray(G.cam + (size_t)b * 12, G.focal[b], G.pix_x[px], G.pix_y[py], G.half_res, ray);
    const float nr = G.near_[b], fr = G.far_[b];
    const float span = __fsub_rn(fr, nr);
    const float dnorm = norm3_torch(ray.d[0], ray.d[1], ray.d[2]);
    constexpr int NVX = Net::kViewSteps - 16;
    f4 vx[NVX][2];                                          // the views layer's k-steps 16 (, 17)
    {
        const float v0 = G.static_viewdirs ? ray.dir[0] : ray.d[0];
        const float v1 = G.static_viewdirs ? ray.dir[1] : ray.d[1];
        const float v2 = G.static_viewdirs ? ray.dir[2] : ray.d[2];
        const float vn = norm3_torch(v0, v1, v2);
        const float ux = __fdiv_rn(v0, vn), uy = __fdiv_rn(v1, vn), uz = __fdiv_rn(v2, vn);
        float v[8];
        if constexpr (Net::kPosEnc) {
            // transform_points(views, True) (sdf_model.py:1628-1640): p / 2, 4 frequencies
            const float ph[3] = {__fmul_rn(ux, 0.5f), __fmul_rn(uy, 0.5f), __fmul_rn(uz, 0.5f)};
#pragma unroll
            for (int st = 1; st < NVX; ++st) {
                float w[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t e = 16 * st + 8 * h + j;
                    w[j] = e < Net::kPosViews ? posenc_val(ph, e) : 0.0f;
                }
                split8(w, vx[st][0], vx[st][1]);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = posenc_val(ph, 8 * h + j);
        } else if constexpr (Net::kSiren) {
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = 0.0f;
            if (h == 0) {
                v[0] = ux;
                v[1] = uy;
                v[2] = uz;
            }
        } else {
            const f4 qa = sh_quad(ux, uy, uz, 2 * h), qb = sh_quad(ux, uy, uz, 2 * h + 1);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = qa[r];
                v[4 + r] = qb[r];
            }
        }
        split8(v, vx[0][0], vx[0][1]);
    }
    float T = 1.0f, wsum = 0.0f, racc0 = 0.0f, racc1 = 0.0f, racc2 = 0.0f;
    float xacc0 = 0.0f, xacc1 = 0.0f, xacc2 = 0.0f, w_last = 0.0f;
    const size_t tile_sid = (size_t)(tile * G.N) * kTileRays + r16;
    const __amdgpu_buffer_rsrc_t enc_r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(a.enc), (short)0, Net::kGrid ? (int)(16u * G.S_total * 8u) : 0, 0x00020000);
    float2 en[2][4];                                        // [layer-0 k-step][level pair]
    float pin[3];                                           // FcNet: normalised point / 2
    auto load_inputs = [&](uint32_t p) {
        uint32_t s = kRSamples * p + (odd ? 1u : 0u);
        if (s >= G.N) s = G.N - 1;
        if constexpr (Net::kPosEnc) {
            const float z = sample_z(G.sc, nr, fr, ray_index, s);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const float pp = __fadd_rn(ray.o[k], __fmul_rn(ray.d[k], z));
                pin[k] = __fmul_rn(G.z_normalize ? __fdiv_rn(__fmul_rn(pp, 2.0f), span) : pp, 0.5f);
            }
        } else if constexpr (Net::kSiren) {
            const float z = sample_z(G.sc, nr, fr, ray_index, s);
            float np_[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const float pp = __fadd_rn(ray.o[k], __fmul_rn(ray.d[k], z));
                np_[k] = G.z_normalize ? __fdiv_rn(__fmul_rn(pp, 2.0f), span) : pp;
            }
            const bool h0 = h == 0;
            en[0][0] = make_float2(h0 ? np_[0] : 0.0f, h0 ? np_[1] : 0.0f);
            en[0][1] = make_float2(h0 ? np_[2] : 0.0f, 0.0f);
            en[0][2] = en[0][3] = make_float2(0.0f, 0.0f);
        } else {
            // buffer loads: one 32-bit lane offset (level 4 h, sample), the level step as a
            // wave-uniform offset (8 hoisted 64-bit addresses otherwise: VGPR pressure)
            const uint32_t voff = ((uint32_t)(tile_sid + (size_t)s * kTileRays) + 4 * h * G.S_total) * 8u;
#pragma unroll
            for (int st = 0; st < 2; ++st)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    // (index the builtin's vector directly: a bit_cast of it to another vector
                    // type made hipcc load one dword and use it twice, ROCm 7.2)
                    const auto v = __builtin_amdgcn_raw_buffer_load_b64(
                        enc_r, (int)voff, (int)((8 * st + k) * G.S_total * 8u), 0);
                    const uint32_t vx0 = v[0], vy0 = v[1];
                    en[st][k] = make_float2(__builtin_bit_cast(float, vx0), __builtin_bit_cast(float, vy0));
                }
        }
    };
    load_inputs(p_begin);

    for (uint32_t p = p_begin; p < p_end; ++p) {
        R.ubase = __builtin_amdgcn_readfirstlane(((p - p_begin) * (uint32_t)((NS + 1) / 2)) & 1u);
        r_na(R, r_slot<Net>(R, 0));
        f16v X[8], Y[8];
        f4 bf[2], E[KL0][2];                               // B fragments: current, layer 0's
        int es = 0;
        if constexpr (Net::kPosEnc) {
            // transform_points(p) (sdf_model.py:1628-1640): 10 frequencies x (sin, cos) of
            // the 3 coordinates; this lane half's 8 of each k-step's 16 (zero past 60)
#pragma unroll
            for (int st = 0; st < KL0; ++st) {
                float w[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t e = 16 * st + 8 * h + j;
                    w[j] = e < Net::kPosIn ? posenc_val(pin, e) : 0.0f;
                }
                split8(w, E[st][0], E[st][1]);
            }
        } else {
            float v[16];
#pragma unroll
            for (int st = 0; st < 2; ++st)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    v[8 * st + 2 * k] = en[st][k].x;
                    v[8 * st + 2 * k + 1] = en[st][k].y;
                }
            if constexpr (Net::kGrid) {
                // the sample's 32 features over both lane halves -> 2^es into [0.5, 1)
                float m = 0.0f;
#pragma unroll
                for (int j = 0; j < 16; ++j) m = fmaxf(m, fabsf(v[j]));
                m = fmaxf(m, __shfl_xor(m, 32));
                if (m > 0.0f && m < 3.0e38f) {
                    const int ex = __builtin_amdgcn_frexp_expf(m);
                    es = ex < -100 ? 100 : -ex;
#pragma unroll
                    for (int j = 0; j < 16; ++j) v[j] = __builtin_ldexpf(v[j], es);
                }
            }
            float u0[8], u1[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                u0[j] = v[j];
                u1[j] = v[8 + j];
            }
            split8(u0, E[0][0], E[0][1]);
            if constexpr (KL0 > 1) split8(u1, E[KL0 - 1][0], E[KL0 - 1][1]);
        }
        float sdfp = 0.0f;
        f4 bn[2];
        struct ActState {
            f4 gm0, bt0, w0, gm1, bt1, w1;
            float v[8];
        };
        ActState as;
        // activation of chunk q (registers 8 (q & 1) .. + 7 of tile q >> 1) of layer l's
        // output o into bn: film vectors read beside group G0, activated beside G0 + 1,
        // split beside G0 + 2
        auto act_side = [&](auto L, f16v (&o)[8], int q, auto GI, auto G0) {
            constexpr int l = decltype(L)::value;
            constexpr int gi = decltype(GI)::value, g0 = decltype(G0)::value;
            constexpr int MODE = (l == 0 && Net::kGrid) ? 0 : (l == NL - 2 ? 2 : 1);
            const int f = Net::film_layer(l);
            const int r0 = 32 * (q >> 1) + 16 * (q & 1) + 4 * (int)h;
            if constexpr (gi == g0) {
                as.gm0 = *reinterpret_cast<const f4 *>(fg(f) + r0);
                as.gm1 = *reinterpret_cast<const f4 *>(fg(f) + r0 + 8);
                as.bt0 = *reinterpret_cast<const f4 *>(fb(f) + r0);
                as.bt1 = *reinterpret_cast<const f4 *>(fb(f) + r0 + 8);
                if constexpr (MODE == 2) {
                    as.w0 = *reinterpret_cast<const f4 *>(sig_w + r0);
                    as.w1 = *reinterpret_cast<const f4 *>(sig_w + r0 + 8);
                }
            } else if constexpr (gi == g0 + 1) {
                r_act<MODE, Net::kSinAct>(o[q >> 1], q & 1, as.gm0, as.bt0, as.w0, as.gm1, as.bt1, as.w1, sdfp, es,
                            as.v);
            } else if constexpr (gi == g0 + 2) {
                split8(as.v, bn[0], bn[1]);
            }
        };
        // layer 0: K = 32 (ngp, 2 k-steps), 3 (siren, 1) or 60 (fc, 4); chunk 0 of its
        // output (tile 0 registers 0-7, final after group 0 of the last layer-0 k-step)
        // from group 1 on
        sfor<0, KL0>([&](auto J) {
            constexpr int j = decltype(J)::value;
            bf[0] = E[j][0];
            bf[1] = E[j][1];
            rstep<Net, j, j == 0>(R, X, bf, [&](auto GI) {
                if constexpr (j == KL0 - 1)
                    act_side(std::integral_constant<int, 0>{}, X, 0, GI, std::integral_constant<int, 2>{});
            });
        });
        // hidden layers 1 .. kHidden: 16 k-steps each (in -> out alternate X / Y)
        auto dense = [&](auto L, f16v (&in)[8], f16v (&out)[8]) {
            constexpr int l = decltype(L)::value;
            sfor<0, 16>([&](auto J) {
                constexpr int j = decltype(J)::value;
                constexpr int KS = KL0 + 16 * (l - 1) + j;
                bf[0] = bn[0];
                bf[1] = bn[1];
                rstep<Net, KS, j == 0>(R, out, bf, [&](auto GI) {
                    if constexpr (j < 15)
                        act_side(std::integral_constant<int, l - 1>{}, in, j + 1, GI,
                                 std::integral_constant<int, 0>{});
                    else
                        act_side(std::integral_constant<int, l>{}, out, 0, GI,
                                 std::integral_constant<int, 2>{});
                });
            });
        };
        sfor<1, Net::kHidden + 1>([&](auto L) {
            constexpr int l = decltype(L)::value;
            if constexpr (l & 1) dense(L, X, Y);
            else dense(L, Y, X);
        });
        constexpr bool kInX = (Net::kHidden & 1) == 0;
        f16v (&vin)[8] = kInX ? X : Y;
        f16v (&vout)[8] = kInX ? Y : X;
        const uint32_t s_own = kRSamples * p + (odd ? 1u : 0u);
        const bool s_ok = s_own < G.N;
        const uint32_t sc_ = s_ok ? s_own : G.N - 1;
        float z = 0.0f, dist = 0.0f, al = 0.0f, sdf_c = 0.0f, w_own = 0.0f;
        float wj[2] = {0.0f, 0.0f};
        sfor<0, Net::kViewSteps>([&](auto J) {
            constexpr int j = decltype(J)::value;
            constexpr int KS = KV + j;
            bf[0] = bn[0];
            bf[1] = bn[1];
            if constexpr (j == 14 && Net::kGrid) {
                const float2 v = a.zd[tile_sid + (size_t)sc_ * kTileRays];
                z = v.x;
                dist = v.y;
            }
            if constexpr (j == 16) {
                if (p + 1 < p_end) load_inputs(p + 1);
            }
            rstep<Net, KS, j == 0>(R, vout, bf, [&](auto GI) {
                constexpr int gi = decltype(GI)::value;
                if constexpr (j < 15) {
                    act_side(std::integral_constant<int, NL - 2>{}, vin, j + 1, GI,
                             std::integral_constant<int, 0>{});
                } else if constexpr (j == 15 && gi == 0) {
                    bn[0] = vx[0][0];                       // k-step 16's B: the direction
                    bn[1] = vx[0][1];
                    sdf_c = __fadd_rn(__fadd_rn(sdfp, __shfl_xor(sdfp, 32)), sig_b);
                } else if constexpr (j == 16 && gi == 0 && NVX > 1) {
                    bn[0] = vx[NVX - 1][0];                 // fc: k-step 17's B
                    bn[1] = vx[NVX - 1][1];
                } else if constexpr (j == 15 && gi == 1) {
                    if constexpr (!Net::kGrid) {
                        z = sample_z(G.sc, nr, fr, ray_index, sc_);
                        dist = (sc_ + 1 < G.N)
                                   ? __fmul_rn(__fsub_rn(sample_z(G.sc, nr, fr, ray_index, sc_ + 1), z), dnorm)
                                   : __fmul_rn(1e10f, dnorm);
                    }
                    float alpha;
                    if (a.with_sdf) {
                        const float sig = __fdiv_rn(sigmoidf_(__fdiv_rn(-sdf_c, beta_s)), beta_s);
                        alpha = 1.0f - expf(-sig * dist);
                    } else {
                        float raw = sdf_c;
                        if (a.sigma_noise) raw += a.sigma_noise[(size_t)ray_index * G.N + sc_];
                        const float sp = raw > 20.0f ? raw : log1pf(expf(raw));
                        alpha = 1.0f - expf(-sp * dist);
                    }
                    al = s_ok ? alpha : 0.0f;
                } else if constexpr (j == 16 && gi == 1) {
                    // the pass's two compositing weights, identically in both lanes of a ray
                    const float ao = __shfl_xor(al, 16);
                    const float aj[2] = {odd ? ao : al, odd ? al : ao};
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const uint32_t s = kRSamples * p + k;
                        if (s < G.N) {
                            float w = aj[k] * T;
                            if (a.force_background && s + 1 == G.N) w = 1.0f - wsum;
                            T = T * ((1.0f - aj[k]) + 1e-10f);
                            wsum += w;
                            wj[k] = w;
                        }
                    }
                    w_own = odd ? wj[1] : wj[0];
                }
            });
        });
        // colour features f = sin(gamma_v x + beta_v), rgb dot products, and the ray's
        // feature sums: w f of the two samples added across the lane rows by
        // v_permlane16_swap (a tile-0..3 value to the even row, its tile-4..7 partner to
        // the odd row), each row accumulating its half of the features
        const float *f3g = fg(NF - 1), *f3b = fb(NF - 1);
        // rgb dot products in 4 independent chains per channel (one per row r of a 4-row
        // group), added at the end: no 128-long serial fma chain for the scheduler to wait on
        float Pc[3][4] = {};
        f2v Pk[3][2] = {};                                 // (kRTailPk) the same sums, packed
        // 16 steps (tile t and its permlane partner t + 4, 4-row group bq), software
        // pipelined: the next step's film / rgb vectors and feature partials are read
        // (LDS) while this step's values are computed
        struct TailIn {
            f4 gm[2], bt[2], w0[2], w1[2], w2[2], fa;
        };
        auto tail_load = [&](int it, TailIn &T) {
            const int t = it >> 2, bq = it & 3;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int r0 = 32 * (t + 4 * u) + 8 * bq + 4 * (int)h;
                T.gm[u] = *reinterpret_cast<const f4 *>(f3g + r0);
                T.bt[u] = *reinterpret_cast<const f4 *>(f3b + r0);
                T.w0[u] = *reinterpret_cast<const f4 *>(rgb_w + r0);
                T.w1[u] = *reinterpret_cast<const f4 *>(rgb_w + kW + r0);
                T.w2[u] = *reinterpret_cast<const f4 *>(rgb_w + 2 * kW + r0);
            }
            T.fa = facc[(4 * t + bq) * 64];
        };
        TailIn tin[2];
        tail_load(0, tin[0]);
        sfor<0, 16>([&](auto IT) {
            constexpr int it = decltype(IT)::value, t = it >> 2, bq = it & 3;
            TailIn &T = tin[it & 1];
            if constexpr (it + 1 < 16) tail_load(it + 1, tin[(it + 1) & 1]);
            float fp[2][4];
            if constexpr (kRTailPk && !(kFAbl & 8)) {
                // packed: rows (2 rp, 2 rp + 1) of each tile as one f2v
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int rp = 0; rp < 2; ++rp) {
                        float fs[2];
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const int r = 2 * rp + h;
                            const float y = __fmaf_rn(T.gm[u][r], vout[t + 4 * u][4 * bq + r], T.bt[u][r]);
                            fs[h] = Net::kSinAct ? sin_rev(y) : y;
                        }
                        const f2v fv = {fs[0], fs[1]};
                        const f2v w0 = {T.w0[u][2 * rp], T.w0[u][2 * rp + 1]};
                        const f2v w1 = {T.w1[u][2 * rp], T.w1[u][2 * rp + 1]};
                        const f2v w2 = {T.w2[u][2 * rp], T.w2[u][2 * rp + 1]};
                        Pk[0][rp] = __builtin_elementwise_fma(fv, w0, Pk[0][rp]);
                        Pk[1][rp] = __builtin_elementwise_fma(fv, w1, Pk[1][rp]);
                        Pk[2][rp] = __builtin_elementwise_fma(fv, w2, Pk[2][rp]);
                        fp[u][2 * rp] = fv.x;
                        fp[u][2 * rp + 1] = fv.y;
                    }
                f4 acc4 = T.fa;
                const f2v wo = {w_own, w_own};
#pragma unroll
                for (int rp = 0; rp < 2; ++rp) {
                    const f2v pa = wo * f2v{fp[0][2 * rp], fp[0][2 * rp + 1]};
                    const f2v pb = wo * f2v{fp[1][2 * rp], fp[1][2 * rp + 1]};
                    acc4[2 * rp] = __fadd_rn(acc4[2 * rp], row_pair_sum(pa.x, pb.x));
                    acc4[2 * rp + 1] = __fadd_rn(acc4[2 * rp + 1], row_pair_sum(pa.y, pb.y));
                }
                facc[(4 * t + bq) * 64] = acc4;
#pragma unroll
                for (int o = 0; o < 3; ++o)
#pragma unroll
                    for (int rp = 0; rp < 2; ++rp) xpin(Pk[o][rp]);
                __builtin_amdgcn_sched_barrier(0);
                return;
            }
            if constexpr (kFAbl & 8) {
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int r = 0; r < 4; ++r) Pc[0][r] = __fadd_rn(Pc[0][r], vout[t + 4 * u][4 * bq + r]);
                __builtin_amdgcn_sched_barrier(0);
                return;
            }
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float y = __fmaf_rn(T.gm[u][r], vout[t + 4 * u][4 * bq + r], T.bt[u][r]);
                    const float f = Net::kSinAct ? sin_rev(y) : y;   // fc: views_linears output
                    Pc[0][r] = __fmaf_rn(f, T.w0[u][r], Pc[0][r]);
                    Pc[1][r] = __fmaf_rn(f, T.w1[u][r], Pc[1][r]);
                    Pc[2][r] = __fmaf_rn(f, T.w2[u][r], Pc[2][r]);
                    fp[u][r] = f;
                }
            // (accumulated whether or not the call wants features: no branch here)
            f4 acc4 = T.fa;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float pa = __fmul_rn(w_own, fp[0][r]);
                const float pb = __fmul_rn(w_own, fp[1][r]);
                acc4[r] = __fadd_rn(acc4[r], row_pair_sum(pa, pb));
            }
            facc[(4 * t + bq) * 64] = acc4;
            // the dot-product partials are materialised here (IR sinking otherwise defers
            // all 384 fmas past the loop and keeps every colour feature live: spills)
#pragma unroll
            for (int o = 0; o < 3; ++o)
#pragma unroll
                for (int r = 0; r < 4; ++r) xpin(Pc[o][r]);
            __builtin_amdgcn_sched_barrier(0);     // one step of look-ahead (VGPRs)
        });
        if constexpr (kRTailPk && !(kFAbl & 8)) {
#pragma unroll
            for (int o = 0; o < 3; ++o)
#pragma unroll
                for (int r = 0; r < 4; ++r) Pc[o][r] = Pk[o][r >> 1][r & 1];
        }
        float P0 = __fadd_rn(__fadd_rn(Pc[0][0], Pc[0][1]), __fadd_rn(Pc[0][2], Pc[0][3]));
        float P1 = __fadd_rn(__fadd_rn(Pc[1][0], Pc[1][1]), __fadd_rn(Pc[1][2], Pc[1][3]));
        float P2 = __fadd_rn(__fadd_rn(Pc[2][0], Pc[2][1]), __fadd_rn(Pc[2][2], Pc[2][3]));
        if (a.sdf && ray_ok && h == 0 && s_ok) a.sdf[(size_t)ray_index * G.N + s_own] = sdf_c;
        {
            P0 = __fadd_rn(P0, __shfl_xor(P0, 32));
            P1 = __fadd_rn(P1, __shfl_xor(P1, 32));
            P2 = __fadd_rn(P2, __shfl_xor(P2, 32));
            racc0 = __fmaf_rn(w_own, sigmoidf_(__fadd_rn(P0, rgb_b0)), racc0);
            racc1 = __fmaf_rn(w_own, sigmoidf_(__fadd_rn(P1, rgb_b1)), racc1);
            racc2 = __fmaf_rn(w_own, sigmoidf_(__fadd_rn(P2, rgb_b2)), racc2);
#pragma unroll
            for (int k = 0; k < 2; ++k)
                if (kRSamples * p + k < G.N) w_last = wj[k];
            if (a.xyz) {
                xacc0 = __fmaf_rn(w_own, __fadd_rn(ray.o[0], __fmul_rn(ray.d[0], z)), xacc0);
                xacc1 = __fmaf_rn(w_own, __fadd_rn(ray.o[1], __fmul_rn(ray.d[1], z)), xacc1);
                xacc2 = __fmaf_rn(w_own, __fadd_rn(ray.o[2], __fmul_rn(ray.d[2], z)), xacc2);
            }
        }
    }
    // the ring runs ahead across passes: no LDS-DMA may land after the workgroup ends
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // the two lanes of a ray (samples 2p, 2p + 1) add their partials
    racc0 = __fadd_rn(racc0, __shfl_xor(racc0, 16));
    racc1 = __fadd_rn(racc1, __shfl_xor(racc1, 16));
    racc2 = __fadd_rn(racc2, __shfl_xor(racc2, 16));
    xacc0 = __fadd_rn(xacc0, __shfl_xor(xacc0, 16));
    xacc1 = __fadd_rn(xacc1, __shfl_xor(xacc1, 16));
    xacc2 = __fadd_rn(xacc2, __shfl_xor(xacc2, 16));
    if (!ray_ok) return;
    // this lane's features: tiles 4 odd .. 4 odd + 3, register v = 4 bq + r of tile t at row
    // 32 t + 8 bq + 4 h + r
    const uint32_t tb = odd ? 4u : 0u;
    if (a.nseg > 1) {
        const size_t Rr = (size_t)G.total_tiles * kTileRays;
        float *pp = a.part + (size_t)seg * kPartQ * Rr + (size_t)tile * kTileRays + r16;
        if (a.features || a.feat_split) {
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int bq = 0; bq < 4; ++bq) {
                    const f4 v = facc[(4 * t + bq) * 64];
                    const uint32_t jf = 32 * (tb + t) + 8 * bq + 4 * h;
#pragma unroll
                    for (int r = 0; r < 4; ++r) pp[(size_t)(jf + r) * Rr] = v[r];
                }
        }
        if (!odd && h == 0) {
            const float q[8] = {racc0, racc1, racc2, xacc0, xacc1, xacc2, T, w_last};
#pragma unroll
            for (int k = 0; k < 8; ++k) pp[(size_t)(kW + k) * Rr] = q[k];
        }
        return;
    }
    const size_t HW = (size_t)G.H * G.W;
    const size_t pix = (size_t)py * G.W + px;
    if (!odd && h == 0) {
        a.rgb[((size_t)b * 3 + 0) * HW + pix] = __fadd_rn(-1.0f, __fmul_rn(2.0f, racc0));
        a.rgb[((size_t)b * 3 + 1) * HW + pix] = __fadd_rn(-1.0f, __fmul_rn(2.0f, racc1));
        a.rgb[((size_t)b * 3 + 2) * HW + pix] = __fadd_rn(-1.0f, __fmul_rn(2.0f, racc2));
        if (a.xyz) {
            a.xyz[((size_t)b * 3 + 0) * HW + pix] = xacc0;
            a.xyz[((size_t)b * 3 + 1) * HW + pix] = xacc1;
            a.xyz[((size_t)b * 3 + 2) * HW + pix] = xacc2;
        }
        if (a.mask) a.mask[(size_t)b * HW + pix] = w_last;
    }
    if (a.features) {
        float *fbp = a.features + (size_t)b * kW * HW + pix;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int bq = 0; bq < 4; ++bq) {
                const f4 v = facc[(4 * t + bq) * 64];
                const uint32_t jf = 32 * (tb + t) + 8 * bq + 4 * h;
#pragma unroll
                for (int r = 0; r < 4; ++r) fbp[(size_t)(jf + r) * HW] = v[r];
            }
    } else if (a.feat_split) {
        // the decoder's first input directly: v * mod[b, c] split hi / lo (fp32 product and
        // RN splits as modulate_nhwc_kernel); lanes h = 0, 1 (lane ^ 32) hold channels
        // 0-3 and 4-7 of an 8-channel group: one permlane32 swap per dword gives lane
        // h = 0 the group's 8 hi halves and lane h = 1 its 8 lo halves, one 16-B store each
        const float *fm = a.feat_mod + (size_t)b * kW;
        const size_t P = (size_t)b * HW + pix;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int bq = 0; bq < 4; ++bq) {
                const uint32_t jf = 32 * (tb + t) + 8 * bq + 4 * h;
                const f4 v = facc[(4 * t + bq) * 64] * *reinterpret_cast<const f4 *>(fm + jf);
                store_split8_pair32(a.feat_split, P * kW + (jf & ~7u), v, h);
            }
    }
}

// Chains the nseg segment partials of every ray (see kPartQ): one thread per
// (ray, quantity), quantities on grid.y.
__global__ void __launch_bounds__(256) field_merge_kernel(const XFieldArgs a) {
    const GeomArgs &G = a.g;
    const uint32_t rid = blockIdx.x * 256 + threadIdx.x, q = blockIdx.y;
    const size_t R = (size_t)G.total_tiles * kTileRays;
    if (rid >= R) return;
    const uint32_t tile = rid / kTileRays, b = tile / G.tiles_per_face;
    const uint32_t ray_local = (tile % G.tiles_per_face) * kTileRays + rid % kTileRays;
    const size_t HW = (size_t)G.H * G.W;
    if (ray_local >= HW) return;
    float *dst;
    float fsplit = 0.0f;                                 // (any non-null marker)
    if (q < kW) dst = a.features ? a.features + ((size_t)b * kW + q) * HW + ray_local
                                 : (a.feat_split ? &fsplit : nullptr);
    else if (q < kW + 3) dst = a.rgb + ((size_t)b * 3 + (q - kW)) * HW + ray_local;
    else if (q < kW + 6) dst = a.xyz ? a.xyz + ((size_t)b * 3 + (q - kW - 3)) * HW + ray_local
                                     : nullptr;
    else if (q == kW + 7) dst = a.mask ? a.mask + (size_t)b * HW + ray_local : nullptr;
    else dst = nullptr;                                  // T itself is not an output
    if (!dst) return;
    const float *pp = a.part + rid;
    const size_t segq = (size_t)kPartQ * R;
    float acc = pp[(size_t)q * R], Tp = pp[(size_t)(kW + 6) * R];
    for (uint32_t k = 1; k < a.nseg; ++k) {
        const float v = pp[k * segq + (size_t)q * R];
        acc = q == kW + 7 ? __fmul_rn(Tp, v) : __fmaf_rn(Tp, v, acc);   // w_last: last segment's
        Tp = __fmul_rn(Tp, pp[k * segq + (size_t)(kW + 6) * R]);
    }
    if (q >= kW && q < kW + 3) acc = __fadd_rn(-1.0f, __fmul_rn(2.0f, acc));
    if (dst == &fsplit) {                                // split-NHWC, times the modulation
        float v = __fmul_rn(acc, a.feat_mod[(size_t)b * kW + q]);
        asm volatile("" : "+v"(v));      // (no v_fma_mix fold of the product: see above)
        const _Float16 hv = (_Float16)v, lv = (_Float16)(v - (float)hv);
        const size_t o = 2 * (((size_t)b * HW + ray_local) * kW + (q & ~7u)) + (q & 7u);
        a.feat_split[o] = hv;
        a.feat_split[o + 8] = lv;
        return;
    }
    *dst = acc;
}

// ----------------------------------------------------------------------------
// host
// ----------------------------------------------------------------------------
// Sample segments per ray: enough workgroups for every CU (>= 256), at most max_seg
// (the call's max_field_segments, 0 = kFieldSplitMax), at least one pass (4 samples)
// in every segment, and never with force_background (its last weight needs the
// whole ray's sum).
uint32_t field_nseg(uint32_t B, uint32_t tiles_per_face, uint32_t N, int force_background,
                    uint32_t max_seg) {
    if (max_seg == 0 || max_seg > kFieldSplitMax) max_seg = kFieldSplitMax;
    const uint32_t wgs = B * ((tiles_per_face + kRTiles - 1) / kRTiles);
    const uint32_t npass = (N + kRSamples - 1) / kRSamples;
    uint32_t nseg = 1;
    while (!force_background && wgs * nseg < 256 && 2 * nseg <= max_seg) {
        const uint32_t c = 2 * nseg, pps = (npass + c - 1) / c;
        if ((c - 1) * pps >= npass) break;            // no empty last segment
        nseg = c;
    }
    return nseg;
}

size_t field_part_bytes(uint32_t B, uint32_t tiles_per_face, uint32_t N) {
    const uint32_t nseg = field_nseg(B, tiles_per_face, N, 0, kFieldSplitMax);
    return nseg > 1 ? (size_t)nseg * kPartQ * B * tiles_per_face * kTileRays * sizeof(float) : 0;
}

template <class Net>
static size_t xws_bytes() {
    return (size_t)Net::kSlices * kXSliceF4 * sizeof(f4) + 2 * Net::kLayers * kW * sizeof(float) +
           (Net::kCompose ? (size_t)(kFeatIn + 1) * kW * sizeof(float) : 0);
}

// the composed ngp layer 0 inside the region: W [256][32] | b [256]
template <class Net>
static float *xws_composed(char *xws) {
    return reinterpret_cast<float *>(xws + (size_t)Net::kSlices * kXSliceF4 * sizeof(f4)) +
           2 * Net::kLayers * kW;
}

// workspace region of this path: packed [slices][1024] f4 | su [L][256] | bias_s [L][256]
// (| composed layer 0, ngp)
size_t f16x3_ws_bytes(int net) {
    return net == 2 ? xws_bytes<FcNet>() : (net ? xws_bytes<SirenNet>() : xws_bytes<NgpNet>());
}

// The network's tensors in policy order (layer 0, dense layers, views; FiLM sets); for
// ngp also the two reference layers that make the composed layer 0 (xws_composed).
struct NetPtrs {
    const float *w[kMaxLayers], *b[kMaxLayers];
    const float *in_w, *in_b, *p0_w, *p0_b;
    const float *gw[kMaxLayers], *gb[kMaxLayers], *bw[kMaxLayers], *bb[kMaxLayers];
    const float *sigma_w, *sigma_b, *rgb_w, *rgb_b, *sigmoid_beta;
};

// Row scales, scaled biases and the packed MFMA A-fragments (xscale_kernel + the
// packing blocks of xprep_kernel) into `xws`; with styles/film the per-face FiLM
// blocks too.  pack_only: no FiLM (sdfr_render_*_pack).
template <class Net>
static int launch_xpack(const NetPtrs &P, uint32_t B, const float *styles, char *xws, float *film,
                        bool pack, hipStream_t st) {
    f4 *packed = reinterpret_cast<f4 *>(xws);
    float *su = reinterpret_cast<float *>(xws + (size_t)Net::kSlices * kXSliceF4 * sizeof(f4));
    float *bias_s = su + Net::kLayers * kW;
    NetPtrs Q = P;
    if constexpr (Net::kCompose) {
        float *wc = xws_composed<Net>(xws);
        Q.w[0] = wc;
        Q.b[0] = wc + kFeatIn * kW;
        if (pack) {
            hipLaunchKernelGGL(compose_kernel, dim3(kW), dim3(64), 0, st, P.in_w, P.in_b, P.p0_w,
                               P.p0_b, wc, wc + kFeatIn * kW);
            int rc = check_launch("render: compose layer 0");
            if (rc) return rc;
        }
    }
    if (pack) {
        XScaleArgs sa;
        for (int l = 0; l < Net::kLayers; ++l) {
            sa.w[l] = Q.w[l];
            sa.b[l] = Q.b[l];
            sa.K[l] = Net::K(l);
        }
        sa.su = su;
        sa.bias_s = bias_s;
        sa.raw_bias0 = 0;
        hipLaunchKernelGGL(xscale_kernel, dim3(Net::kLayers, kW / 4), dim3(256), 0, st, sa);
        int rc = check_launch("render: xscale");
        if (rc) return rc;
    }
    XPrepArgs p;
    p.styles = styles;
    for (int f = 0; f < Net::kFilmN; ++f) {
        p.gw[f] = P.gw[f];
        p.gb[f] = P.gb[f];
        p.bw[f] = P.bw[f];
        p.bb[f] = P.bb[f];
    }
    for (int l = 0; l < Net::kLayers; ++l) {
        p.w[l] = Q.w[l];
        p.lb[l] = Q.b[l];
    }
    p.su = su;
    p.film = film;
    p.packed = packed;
    p.B = film ? B : 0;
    // blocks [0, B films x 2 x 256 / 4): FiLM rows; then (pack) the fragment packing
    const uint32_t nfilm = p.B * Net::kFilmN * 2 * kW / 4;
    const uint32_t blocks = nfilm + (pack ? (Net::kSlices * 512 + 255) / 256 : 0);
    if (blocks == 0) return SDFR_OK;
    hipLaunchKernelGGL(xprep_kernel<Net>, dim3(blocks), dim3(256), 0, st, p);
    return check_launch("render: xprep");
}

// Per call: FiLM vectors of the batch, and the weight packing unless the caller
// passed weights packed beforehand (a->prepacked, f16x3 only).
template <class Net>
static int launch_xprep(const NetPtrs &P, const sdfr_ngp_render_args *a, char *xws, float *film,
                        hipStream_t st) {
    if (a->prepacked)
        return launch_xpack<Net>(P, a->B, a->styles, const_cast<char *>(
                                     reinterpret_cast<const char *>(a->prepacked)), film, false, st);
    return launch_xpack<Net>(P, a->B, a->styles, xws, film, true, st);
}

template <class Net>
static int launch_xfield(const NetPtrs &P, const sdfr_ngp_render_args *a, const GeomArgs &g,
                         const float *enc, char *xws, const float *film, hipStream_t st,
                         float *part = nullptr, const float2 *zd = nullptr) {
    XFieldArgs f;
    f.g = g;
    f.enc = enc;
    f.zd = zd;
    if (a->prepacked) xws = const_cast<char *>(reinterpret_cast<const char *>(a->prepacked));
    f.packed = reinterpret_cast<const f4 *>(xws);
    f.su = reinterpret_cast<const float *>(xws + (size_t)Net::kSlices * kXSliceF4 * sizeof(f4));
    f.bias_s = f.su + Net::kLayers * kW;
    f.film = film;
    f.sigma_w = P.sigma_w;
    f.sigma_b = P.sigma_b;
    f.rgb_w = P.rgb_w;
    f.rgb_b = P.rgb_b;
    f.sigmoid_beta = P.sigmoid_beta;
    f.sigma_noise = a->sigma_noise;
    f.force_background = a->force_background;
    f.with_sdf = a->with_sdf;
    f.rgb = a->rgb;
    f.features = a->features;
    f.feat_split = reinterpret_cast<_Float16 *>(a->features_split);
    f.feat_mod = a->features_mod;
    f.sdf = a->sdf;
    f.xyz = a->xyz;
    f.mask = a->mask;
    f.part = part;
    if (f.feat_split && (!f.feat_mod || f.features || !Net::kFieldR))
        return fail(SDFR_EUNSUPPORTED, "render: features_split needs features_mod, no NCHW "
                                       "features, and the ngp / FC field kernel");
    // field_r_kernel for ngp; the SIREN net (nine FiLM layers, no encode stage, no
    // sample-segment split) keeps field_p_kernel, 6 % faster on it (7.76 vs 8.25 ms per
    // 32 faces, interleaved A/B on one box; field_r_kernel is 3.5 % faster on ngp)
    if constexpr (Net::kFieldR) {
        f.nseg = part ? field_nseg(g.B, g.tiles_per_face, g.N, a->force_background,
                                   a->max_field_segments) : 1;
        const uint32_t blocks = g.B * ((g.tiles_per_face + kRTiles - 1) / kRTiles) * f.nseg;
        hipLaunchKernelGGL((field_r_kernel<Net>), dim3(blocks), dim3(kRThreads), 0, st, f);
    } else {
        if (part) return fail(SDFR_EUNSUPPORTED, "render: field_p_kernel has no segment split");
        f.nseg = 1;
        const uint32_t blocks = g.B * ((g.tiles_per_face + kPTiles - 1) / kPTiles);
        hipLaunchKernelGGL((field_p_kernel<Net>), dim3(blocks), dim3(kPThreads), 0, st, f);
    }
    int rc = check_launch("render: field (f16x3)");
    if (rc || f.nseg == 1) return rc;
    const uint32_t rays = g.total_tiles * kTileRays;
    hipLaunchKernelGGL(field_merge_kernel, dim3((rays + 255) / 256, kPartQ), dim3(256), 0, st, f);
    return check_launch("render: field segment merge");
}

static NetPtrs ngp_ptrs(const sdfr_ngp_weights *w) {
    NetPtrs P{};
    P.in_w = w->input_w;                       // composed into layer 0 (launch_xpack)
    P.in_b = w->input_b;
    P.p0_w = w->pts_w[0];
    P.p0_b = w->pts_b[0];
    for (int l = 1; l < 3; ++l) {
        P.w[l] = w->pts_w[l];
        P.b[l] = w->pts_b[l];
    }
    for (int f = 0; f < 3; ++f) {
        P.gw[f] = w->pts_gw[f];
        P.gb[f] = w->pts_gb[f];
        P.bw[f] = w->pts_bw[f];
        P.bb[f] = w->pts_bb[f];
    }
    P.w[3] = w->views_w;
    P.b[3] = w->views_b;
    P.gw[3] = w->views_gw;
    P.gb[3] = w->views_gb;
    P.bw[3] = w->views_bw;
    P.bb[3] = w->views_bb;
    P.sigma_w = w->sigma_w;
    P.sigma_b = w->sigma_b;
    P.rgb_w = w->rgb_w;
    P.rgb_b = w->rgb_b;
    P.sigmoid_beta = w->sigmoid_beta;
    return P;
}

int launch_xprep_ngp(const sdfr_ngp_weights *w, const sdfr_ngp_render_args *a, char *xws,
                     float *film, hipStream_t st) {
    return launch_xprep<NgpNet>(ngp_ptrs(w), a, xws, film, st);
}

int launch_xfield_ngp(const sdfr_ngp_weights *w, const sdfr_ngp_render_args *a,
                      const GeomArgs &g, const float *enc, char *xws, const float *film,
                      hipStream_t st, float *part, const float2 *zd) {
    return launch_xfield<NgpNet>(ngp_ptrs(w), a, g, enc, xws, film, st, part, zd);
}

// ----------------------------------------------------------------------------
// SIREN entry points
// ----------------------------------------------------------------------------
static size_t align256x(size_t v) { return (v + 255) & ~(size_t)255; }

// film [B][9][2][256] | split-fp16 region
static size_t siren_ws_layout(uint32_t B, size_t *o_x) {
    size_t off = align256x((size_t)B * SirenNet::kFilmN * 2 * kW * sizeof(float));
    if (o_x) *o_x = off;
    return off + align256x(xws_bytes<SirenNet>());
}

static NetPtrs siren_ptrs(const sdfr_siren_weights *w) {
    NetPtrs P{};
    for (int l = 0; l < 8; ++l) {
        P.w[l] = w->pts_w[l];
        P.b[l] = w->pts_b[l];
        P.gw[l] = w->pts_gw[l];
        P.gb[l] = w->pts_gb[l];
        P.bw[l] = w->pts_bw[l];
        P.bb[l] = w->pts_bb[l];
    }
    P.w[8] = w->views_w;
    P.b[8] = w->views_b;
    P.gw[8] = w->views_gw;
    P.gb[8] = w->views_gb;
    P.bw[8] = w->views_bw;
    P.bb[8] = w->views_bb;
    P.sigma_w = w->sigma_w;
    P.sigma_b = w->sigma_b;
    P.rgb_w = w->rgb_w;
    P.rgb_b = w->rgb_b;
    P.sigmoid_beta = w->sigmoid_beta;
    return P;
}

static int siren_validate(const sdfr_siren_weights *w, const sdfr_ngp_render_args *a) {
    if (!w || !a) return fail(SDFR_EINVAL, "render_siren: null args");
    if (w->depth != 8 || w->width != 256)
        return fail(SDFR_EUNSUPPORTED, "render_siren: fused path needs depth 8, width 256");
    if (a->field_precision != SDFR_FIELD_F16X3)
        return fail(SDFR_EUNSUPPORTED, "render_siren: only field_precision 0 (f16x3)");
    if (a->B == 0 || a->H == 0 || a->W == 0 || a->N == 0)
        return fail(SDFR_EINVAL, "render_siren: empty batch / image / sample count");
    if (a->max_field_segments > kFieldSplitMax || a->max_field_segments == 3)
        return fail(SDFR_EINVAL, "render_siren: max_field_segments must be 0, 1, 2 or 4");
    if (!a->cam || !a->focal || !a->near_ || !a->far_ || !a->styles || !a->pix_x ||
        !a->pix_y || !a->t_vals || !a->rgb || !a->workspace)
        return fail(SDFR_EINVAL, "render_siren: required pointer is null");
    for (int l = 0; l < 8; ++l)
        if (!w->pts_w[l] || !w->pts_b[l] || !w->pts_gw[l] || !w->pts_gb[l] || !w->pts_bw[l] ||
            !w->pts_bb[l])
            return fail(SDFR_EINVAL, "render_siren: FiLM weight pointer is null");
    const void *need[] = {w->views_w, w->views_b, w->views_gw, w->views_gb, w->views_bw,
                          w->views_bb, w->sigma_w, w->sigma_b, w->rgb_w, w->rgb_b};
    for (const void *p : need)
        if (!p) return fail(SDFR_EINVAL, "render_siren: weight pointer is null");
    if (a->with_sdf && !w->sigmoid_beta)
        return fail(SDFR_EINVAL, "render_siren: sigmoid_beta is required when with_sdf");
    if (a->workspace_bytes < siren_ws_layout(a->B, nullptr))
        return fail(SDFR_EINVAL, "render_siren: workspace too small");
    return SDFR_OK;
}

// ----------------------------------------------------------------------------
// FCGenerator entry points
// ----------------------------------------------------------------------------
// film [B][9][2][256] | split-fp16 region | sample-segment partials (small batches)
static size_t fc_ws_layout(uint32_t B, uint32_t H, uint32_t W, uint32_t N, size_t *o_x,
                           size_t *o_part) {
    size_t off = align256x((size_t)B * FcNet::kFilmN * 2 * kW * sizeof(float));
    if (o_x) *o_x = off;
    off += align256x(xws_bytes<FcNet>());
    if (o_part) *o_part = off;
    off += align256x(field_part_bytes(B, (H * W + kTileRays - 1) / kTileRays, N));
    return off;
}

static NetPtrs fc_ptrs(const sdfr_fc_weights *w) {
    NetPtrs P{};
    P.w[0] = w->x_in_w;
    P.b[0] = w->x_in_b;
    P.gw[0] = w->style_w;                      // style_in: layer 0's per-face bias
    P.gb[0] = w->style_b;
    for (int l = 0; l < 7; ++l) {
        P.w[1 + l] = w->pts_w[l];
        P.b[1 + l] = w->pts_b[l];
    }
    P.w[8] = w->views_w;
    P.b[8] = w->views_b;
    P.sigma_w = w->sigma_w;
    P.sigma_b = w->sigma_b;
    P.rgb_w = w->rgb_w;
    P.rgb_b = w->rgb_b;
    P.sigmoid_beta = w->sigmoid_beta;
    return P;
}

static int fc_validate(const sdfr_fc_weights *w, const sdfr_ngp_render_args *a) {
    if (!w || !a) return fail(SDFR_EINVAL, "render_fc: null args");
    if (w->depth != 8 || w->width != 256)
        return fail(SDFR_EUNSUPPORTED, "render_fc: fused path needs depth 8, width 256");
    if (a->field_precision != SDFR_FIELD_F16X3)
        return fail(SDFR_EUNSUPPORTED, "render_fc: only field_precision 0 (f16x3)");
    if (a->B == 0 || a->H == 0 || a->W == 0 || a->N == 0)
        return fail(SDFR_EINVAL, "render_fc: empty batch / image / sample count");
    if (a->max_field_segments > kFieldSplitMax || a->max_field_segments == 3)
        return fail(SDFR_EINVAL, "render_fc: max_field_segments must be 0, 1, 2 or 4");
    if (!a->cam || !a->focal || !a->near_ || !a->far_ || !a->styles || !a->pix_x ||
        !a->pix_y || !a->t_vals || !a->rgb || !a->workspace)
        return fail(SDFR_EINVAL, "render_fc: required pointer is null");
    for (int l = 0; l < 7; ++l)
        if (!w->pts_w[l] || !w->pts_b[l]) return fail(SDFR_EINVAL, "render_fc: weight pointer is null");
    const void *need[] = {w->x_in_w, w->x_in_b, w->style_w, w->style_b, w->views_w, w->views_b,
                          w->sigma_w, w->sigma_b, w->rgb_w, w->rgb_b};
    for (const void *p : need)
        if (!p) return fail(SDFR_EINVAL, "render_fc: weight pointer is null");
    if (a->with_sdf && !w->sigmoid_beta)
        return fail(SDFR_EINVAL, "render_fc: sigmoid_beta is required when with_sdf");
    if (a->workspace_bytes < fc_ws_layout(a->B, a->H, a->W, a->N, nullptr, nullptr))
        return fail(SDFR_EINVAL, "render_fc: workspace too small");
    return SDFR_OK;
}

}  // namespace sdfr

using namespace sdfr;

extern "C" {

size_t sdfr_render_fc_workspace_bytes(uint32_t B, uint32_t H, uint32_t W, uint32_t N) {
    return fc_ws_layout(B, H, W, N, nullptr, nullptr);
}

int sdfr_render_fc_pack(const sdfr_fc_weights *w, void *packed, void *stream) {
    if (!w || !packed) return fail(SDFR_EINVAL, "render_fc_pack: null pointer");
    return launch_xpack<FcNet>(fc_ptrs(w), 0, nullptr, reinterpret_cast<char *>(packed), nullptr,
                               true, (hipStream_t)stream);
}

int sdfr_render_fc_forward(const sdfr_fc_weights *w, const sdfr_ngp_render_args *a, void *stream) {
    int rc = fc_validate(w, a);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    size_t o_x, o_part;
    fc_ws_layout(a->B, a->H, a->W, a->N, &o_x, &o_part);
    char *ws = reinterpret_cast<char *>(a->workspace);
    float *film = reinterpret_cast<float *>(ws);
    const NetPtrs P = fc_ptrs(w);
    GeomArgs g;
    fill_geom_args(a, 1.0f, g);
    record_event(a->stage_events[0], st);
    wait_event(a->styles_event, st);
    if ((rc = launch_xprep<FcNet>(P, a, ws + o_x, film, st))) return rc;
    record_event(a->stage_events[1], st);
    record_event(a->stage_events[2], st);
    record_event(a->field_event, st);
    if ((rc = launch_xfield<FcNet>(P, a, g, nullptr, ws + o_x, film, st,
                                   reinterpret_cast<float *>(ws + o_part))))
        return rc;
    record_event(a->stage_events[3], st);
    return SDFR_OK;
}

size_t sdfr_render_siren_workspace_bytes(uint32_t B) { return siren_ws_layout(B, nullptr); }

size_t sdfr_render_pack_bytes(int net) { return f16x3_ws_bytes(net); }

int sdfr_render_ngp_pack(const sdfr_ngp_weights *w, void *packed, void *stream) {
    if (!w || !packed) return fail(SDFR_EINVAL, "render_ngp_pack: null pointer");
    return launch_xpack<NgpNet>(ngp_ptrs(w), 0, nullptr, reinterpret_cast<char *>(packed), nullptr,
                                true, (hipStream_t)stream);
}

int sdfr_render_siren_pack(const sdfr_siren_weights *w, void *packed, void *stream) {
    if (!w || !packed) return fail(SDFR_EINVAL, "render_siren_pack: null pointer");
    return launch_xpack<SirenNet>(siren_ptrs(w), 0, nullptr, reinterpret_cast<char *>(packed),
                                  nullptr, true, (hipStream_t)stream);
}

int sdfr_render_siren_forward(const sdfr_siren_weights *w, const sdfr_ngp_render_args *a,
                              void *stream) {
    int rc = siren_validate(w, a);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    size_t o_x;
    siren_ws_layout(a->B, &o_x);
    char *ws = reinterpret_cast<char *>(a->workspace);
    float *film = reinterpret_cast<float *>(ws);
    const NetPtrs P = siren_ptrs(w);
    GeomArgs g;
    fill_geom_args(a, 1.0f, g);
    record_event(a->stage_events[0], st);
    wait_event(a->styles_event, st);
    if ((rc = launch_xprep<SirenNet>(P, a, ws + o_x, film, st))) return rc;
    record_event(a->stage_events[1], st);
    record_event(a->stage_events[2], st);
    record_event(a->field_event, st);
    if ((rc = launch_xfield<SirenNet>(P, a, g, nullptr, ws + o_x, film, st))) return rc;
    record_event(a->stage_events[3], st);
    return SDFR_OK;
}

}  // extern "C"
