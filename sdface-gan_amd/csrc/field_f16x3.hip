// field_f16x3.hip -- the fused renderer's field stage on split-fp16 MFMA.
//
// Same job as ngp_field_kernel (render_ngp.hip): NGPSIRENGenerator's five
// dense layers (sdf_model.py:1566-1592) + SDF->density + front-to-back alpha
// compositing (volume_integration, :236-301) for 16 rays per wave, but every
// fp32 GEMM tile runs as three v_mfma_f32_16x16x32_f16 on a hi/lo fp16 split
// of both operands:
//
//     W.x = W_hi.x_hi + W_hi.x_lo + W_lo.x_hi   (+ W_lo.x_lo, dropped: 2^-22 rel.)
//
// accumulated in fp32 by the matrix core.  16x16x32 f16 issues 16x the FLOPs
// per cycle of 16x16x4 f32, so three of them are 5.3x the fp32 MFMA rate.
// Accuracy (scripts/probe_split_f16.hip, measured on MI355X): a 256-deep dot
// product is as accurate as the fp32 fma chain PROVIDED the fp16 lo parts do
// not go subnormal -- so every weight row is scaled by a power of two su
// (max |w| su in [0.5,1), ngp_xscale_kernel).  Power-of-two scaling commutes
// with rounding, so it is undone exactly: biases enter pre-scaled, the FiLM
// gamma is divided by su (gamma' x_scaled == gamma x, bit for bit), and the
// identity input layer multiplies by 1/su.
//
// Work unit: a wave owns 16 rays and evaluates TWO samples per pass (MFMA
// N = 2 x 16), so each A fragment read from LDS feeds 6 MFMAs and the weight
// stream (1.1 MB per pass, shared by the 4 waves of a workgroup through a
// 3-slot LDS ring) is amortised over 128 ray-samples.  The accumulator of
// layer l is the B operand of layer l+1 with no lane movement: after a pair of
// 16-row tiles (2q, 2q+1) is activated, its 8 values per lane are split in
// place into (hi, lo) fp16x8, which is exactly the k-step q fragment (the
// packed weights permute K to match, ngp_xprep_kernel).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "render_ngp.h"

namespace sdfr {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));

constexpr uint32_t kXSliceF4 = 1024;             // 16 KB: [8 t_out][hi,lo][64 lanes] x 16 B
constexpr uint32_t kXSlices = 2 + 16 * 3 + 18;   // half k-steps per pass
constexpr int kXStage = kXSliceF4 / kThreads;    // float4 staged per thread per slice
constexpr uint32_t kXCst = 10 * kW;              // bias_s[5], 1/su0, sigma_w, rgb_w[3]

// Schedule options (compile-time; DESIGN.md section 5 records the measured choice):
//   SDFR_X_PREFETCH  ring staged two slices ahead + next slice's first fragment
//                    read before the barrier (1) / one slice ahead (0)
//   SDFR_X_EPI       views layer output-group major with the compositing of tiles
//                    0-7 in the MFMA shadow of tiles 8-15 (1) / after the layer (0)
#ifndef SDFR_X_PREFETCH
#define SDFR_X_PREFETCH 1
#endif
#ifndef SDFR_X_EPI
#define SDFR_X_EPI 0
#endif
//   SDFR_X_BUFLOAD   ring staging loads as buffer_load (scalar slice offset, no
//                    per-load 64-bit address VALU) (1) / global_load (0)
#ifndef SDFR_X_BUFLOAD
#define SDFR_X_BUFLOAD 1
#endif

__host__ __device__ constexpr uint32_t xslice_base(uint32_t layer) {
    return layer == 0 ? 0u : (layer == 4 ? 50u : 2u + 16u * (layer - 1));
}
__host__ __device__ constexpr uint32_t layer_k(uint32_t layer) {
    return layer == 0 ? kFeatIn : (layer == 4 ? kViewsIn : kW);
}

__device__ __forceinline__ h8 as_h8(f4 v) { return __builtin_bit_cast(h8, v); }
__device__ __forceinline__ f4 mfma16(f4 a, f4 b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(as_h8(a), as_h8(b), c, 0, 0, 0);
}

// 8 fp32 -> (hi, lo) fp16x8, round-to-nearest both (v_cvt_pk_f16_f32)
__device__ __forceinline__ void split8(const float (&v)[8], f4 &hi, f4 &lo) {
    h8 H, L;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        H[j] = (_Float16)v[j];
        L[j] = (_Float16)__fsub_rn(v[j], (float)H[j]);
    }
    hi = __builtin_bit_cast(f4, H);
    lo = __builtin_bit_cast(f4, L);
}

// ----------------------------------------------------------------------------
// prep 1: per-row power-of-two scales and scaled biases
// ----------------------------------------------------------------------------
struct XScaleArgs {
    const float *w[5];
    const float *b[5];
    float *su;       // [5][256]
    float *bias_s;   // [5][256]
};

__global__ void __launch_bounds__(256) ngp_xscale_kernel(const XScaleArgs a) {
    const uint32_t layer = blockIdx.x, row = threadIdx.x;
    const uint32_t K = layer_k(layer);
    const float *wr = a.w[layer] + (size_t)row * K;
    float m = 0.0f;
    for (uint32_t k = 0; k < K; ++k) m = fmaxf(m, fabsf(wr[k]));
    float su = 1.0f;
    if (m > 0.0f && m < 3.0e38f) {
        int ex;
        (void)frexpf(m, &ex);              // m = f 2^ex, f in [0.5, 1)
        ex = ex < -100 ? -100 : (ex > 100 ? 100 : ex);
        su = ldexpf(1.0f, -ex);
    }
    a.su[layer * kW + row] = su;
    a.bias_s[layer * kW + row] = __fmul_rn(a.b[layer][row], su);
}

// ----------------------------------------------------------------------------
// prep 2: FiLM vectors (gamma / su) + split-fp16 weight fragments
// ----------------------------------------------------------------------------
struct XPrepArgs {
    const float *styles;           // [B,256]
    const float *gw[kFilm], *gb[kFilm], *bw[kFilm], *bb[kFilm];
    const float *w[5];
    const float *su;               // [5][256]
    float *film;                   // [B][4][2][256]
    f4 *packed;                    // [68][8][2][64] fp16x8
    uint32_t B;
};

// K index of element j of lane group g in k-step q of `layer` (-1 = zero pad).
__device__ __forceinline__ int xperm_k(uint32_t layer, uint32_t q, uint32_t g, uint32_t j) {
    if (layer == 0) return (int)(8 * g + j);
    if (layer == 4 && q == 8) return g < 2 ? (int)(kW + 8 * g + j) : -1;
    return (int)(16 * (2 * q + (j >> 2)) + 4 * g + (j & 3));
}

// blocks [0, B*8): FiLM rows; then packing, one (slice, t8, lane) per thread
__global__ void __launch_bounds__(256) ngp_xprep_kernel(const XPrepArgs a) {
    const uint32_t blk = blockIdx.x, j = threadIdx.x;
    const uint32_t nfilm = a.B * kFilm * 2;
    if (blk < nfilm) {
        const uint32_t b = blk / (kFilm * 2), rem = blk % (kFilm * 2);
        const uint32_t layer = rem >> 1, which = rem & 1;
        const float *W = which ? a.bw[layer] : a.gw[layer];
        const float *bias = which ? a.bb[layer] : a.gb[layer];
        const f4 *wr = reinterpret_cast<const f4 *>(W + (size_t)j * kW);
        const f4 *sr = reinterpret_cast<const f4 *>(a.styles + (size_t)b * kW);
        float acc = 0.0f;
#pragma unroll 8
        for (uint32_t k = 0; k < kW / 4; ++k) {
            const f4 w4 = wr[k], s4 = sr[k];
            acc = __fmaf_rn(s4.x, w4.x, acc);
            acc = __fmaf_rn(s4.y, w4.y, acc);
            acc = __fmaf_rn(s4.z, w4.z, acc);
            acc = __fmaf_rn(s4.w, w4.w, acc);
        }
        const float lin = __fadd_rn(acc, bias[j]);
        // LinearLayer: std_init * linear + bias_init (sdf_model.py:39, 58-59); the
        // gamma of network layer `layer+1` absorbs that layer's row scale exactly
        const float v = which ? __fadd_rn(__fmul_rn(0.25f, lin), 0.0f)
                              : __fdiv_rn(__fadd_rn(__fmul_rn(15.0f, lin), 30.0f),
                                          a.su[(layer + 1) * kW + j]);
        a.film[(((size_t)b * kFilm + layer) * 2 + which) * kW + j] = v;
        return;
    }
    const uint32_t e = (blk - nfilm) * 256 + j;
    if (e >= kXSlices * 512) return;
    const uint32_t slice = e / 512, rem = e % 512;
    const uint32_t t8 = rem >> 6, lane = rem & 63;
    uint32_t layer = 0;
    if (slice >= 50) layer = 4;
    else if (slice >= 2) layer = 1 + (slice - 2) / 16;
    const uint32_t local = slice - xslice_base(layer);
    // layers 0-3: k-step major (q, h); views layer: output-group major (h, q)
    const bool hmajor = SDFR_X_EPI && layer == 4;
    const uint32_t q = hmajor ? local % 9 : local >> 1;
    const uint32_t h = hmajor ? local / 9 : local & 1;
    const uint32_t row = 16 * (8 * h + t8) + (lane & 15), g = lane >> 4;
    const uint32_t K = layer_k(layer);
    const float s = a.su[layer * kW + row];
    float v[8];
#pragma unroll
    for (uint32_t jj = 0; jj < 8; ++jj) {
        const int k = xperm_k(layer, q, g, jj);
        v[jj] = k < 0 ? 0.0f : __fmul_rn(a.w[layer][(size_t)row * K + k], s);
    }
    f4 hi, lo;
    h8 H, L;
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
        H[jj] = (_Float16)v[jj];
        L[jj] = (_Float16)__fsub_rn(v[jj], (float)H[jj]);
    }
    hi = __builtin_bit_cast(f4, H);
    lo = __builtin_bit_cast(f4, L);
    f4 *dst = a.packed + (size_t)slice * kXSliceF4 + t8 * 128 + lane;
    dst[0] = hi;
    dst[64] = lo;
}

// ----------------------------------------------------------------------------
// field kernel
// ----------------------------------------------------------------------------
struct XFieldArgs {
    GeomArgs g;
    const float *enc;              // [L=16][S_total][2]
    const f4 *packed;              // [68][1024]
    const float *film;             // [B][4][2][256], gamma pre-divided by su
    const float *su;               // [5][256]
    const float *bias_s;           // [5][256]
    const float *sigma_w, *sigma_b, *rgb_w, *rgb_b, *sigmoid_beta;
    const float *sigma_noise;      // [B,H,W,N] or null (no_sdf only)
    int force_background, with_sdf;
    float *rgb, *features, *sdf, *xyz, *mask;
};

// Weight ring: 3 LDS slots; during slice `it` the wave computes from slot it%3,
// writes slice it+2 (held in registers since slice it-1) into slot (it+2)%3 --
// the slot of slice it-1, which every wave finished reading before the barrier
// that closed slice it-1 -- loads slice it+3 into registers, and reads the first
// fragment pair of slice it+1 (already visible: written during it-1), so the
// next slice's first MFMAs do not wait on LDS latency after the barrier.
struct XRing {
    f4 *lds;              // [3][kXSliceF4]
    const f4 *packed;
    f4 st[kXStage];       // slice it+2 (global -> regs -> LDS)
    f4 pre_h, pre_l;      // first (hi, lo) A fragment of the current slice
    __amdgpu_buffer_rsrc_t rsrc;   // the packed fragments (SDFR_X_BUFLOAD)
    uint32_t it;          // slice iteration (runs across passes)
    uint32_t tid;
};

__device__ __forceinline__ void xpin(f4 &x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void xpin(float &x) { asm volatile("" : "+v"(x)); }

// One half k-step: 8 output tiles (8H .. 8H+7) x 2 sample columns x 3 split
// terms = 48 MFMAs on one LDS ring slot, then `side` (register work issued in
// the MFMA shadow), the ring staging (XRing) and the slice barrier.
// Ablation variants (profiling builds only, sdfr_debug_set_field_variant; V = 0
// is the product): bit 0 drops the slice barrier, bit 1 the LDS A-fragment reads,
// bit 2 the ring staging, bit 3 the per-layer activations, bit 4 the per-pass
// compositing.  Any V != 0 computes wrong results by construction.
template <int V, int H, class Side>
__device__ __forceinline__ void xstep(XRing &R, f4 (&acc0)[16], f4 (&acc1)[16], const f4 b0h,
                                      const f4 b0l, const f4 b1h, const f4 b1l, Side &&side) {
    const uint32_t cur = R.it % 3u;
    const f4 *A = R.lds + cur * kXSliceF4 + (R.tid & 63u);
    f4 ah[8], al[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if constexpr ((V & 2) != 0) {
            ah[i] = b0h * (float)(i + 1);
            al[i] = b1l * (float)(i + 1);
        } else if (SDFR_X_PREFETCH && i == 0) {
            ah[0] = R.pre_h;
            al[0] = R.pre_l;
        } else {
            ah[i] = A[(2 * i) * 64];
            al[i] = A[(2 * i + 1) * 64];
        }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int t = 8 * H + i;
        acc0[t] = mfma16(al[i], b0h, acc0[t]);
        acc1[t] = mfma16(al[i], b1h, acc1[t]);
        acc0[t] = mfma16(ah[i], b0l, acc0[t]);
        acc1[t] = mfma16(ah[i], b1l, acc1[t]);
        acc0[t] = mfma16(ah[i], b0h, acc0[t]);
        acc1[t] = mfma16(ah[i], b1h, acc1[t]);
    }
    side();
    if constexpr ((V & 4) == 0) {
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t wslot = (R.it + 1u + SDFR_X_PREFETCH) % 3u;
#pragma unroll
        for (int i = 0; i < kXStage; ++i)
            R.lds[wslot * kXSliceF4 + R.tid + i * kThreads] = R.st[i];
        const uint32_t pf = (R.it + 2u + SDFR_X_PREFETCH) % kXSlices;
#pragma unroll
        for (int i = 0; i < kXStage; ++i) {
#if SDFR_X_BUFLOAD
            R.st[i] = __builtin_bit_cast(
                f4, __builtin_amdgcn_raw_buffer_load_b128(
                        R.rsrc, (int)((R.tid + i * kThreads) * sizeof(f4)),
                        (int)(pf * kXSliceF4 * sizeof(f4)), 0));
#else
            R.st[i] = R.packed[pf * kXSliceF4 + R.tid + i * kThreads];
#endif
        }
    }
    if constexpr ((V & 2) == 0 && SDFR_X_PREFETCH) {
        const f4 *An = R.lds + ((R.it + 1u) % 3u) * kXSliceF4 + (R.tid & 63u);
        R.pre_h = An[0];
        R.pre_l = An[64];
    }
    if constexpr ((V & 1) == 0) __syncthreads();
    ++R.it;
}

// Activate tile pair (2q, 2q+1) of one sample column in place and split it
// into the (hi, lo) B fragment of k-step q.
//   MODE 0: identity input layer, x * (1/su0)
//   MODE 1: FiLM sin(gamma' x + beta) (sdf_model.py:67, two roundings)
//   MODE 2: FiLM + partial sigma_linear dot product (the sdf head)
template <int MODE, int V>
__device__ __forceinline__ void act_pair(f4 &za, f4 &zb, int q, const float *gam,
                                         const float *bet, const float *sw, float &sdfp,
                                         uint32_t g) {
    if constexpr ((V & 8) != 0) {
        xpin(za);
        xpin(zb);
        return;
    }
    float v[8];
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        const f4 z = half ? zb : za;
        const int f0 = 16 * (2 * q + half) + 4 * (int)g;
        const f4 gm = *reinterpret_cast<const f4 *>(gam + f0);
        f4 bt = {0.0f, 0.0f, 0.0f, 0.0f};
        if constexpr (MODE != 0) bt = *reinterpret_cast<const f4 *>(bet + f0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float x;
            if constexpr (MODE == 0) x = __fmul_rn(z[r], gm[r]);
            else x = sin_hw(__fadd_rn(__fmul_rn(gm[r], z[r]), bt[r]));
            v[4 * half + r] = x;
        }
        if constexpr (MODE == 2) {
            const f4 w4 = *reinterpret_cast<const f4 *>(sw + f0);
#pragma unroll
            for (int r = 0; r < 4; ++r) sdfp = __fmaf_rn(v[4 * half + r], w4[r], sdfp);
        }
    }
    split8(v, za, zb);
    xpin(za);
    xpin(zb);
    if constexpr (MODE == 2) xpin(sdfp);
}

__device__ __forceinline__ void init_acc(f4 (&acc)[16], const float *bias, uint32_t g) {
#pragma unroll
    for (int t = 0; t < 16; ++t) acc[t] = *reinterpret_cast<const f4 *>(bias + 16 * t + 4 * g);
}

// A 256 -> 256 layer: out = W in + b over 8 k-steps.  In k-step q the next
// input pair (q+1) of each sample column is activated in the MFMA shadow; the
// last k-step activates the first pair of this layer's own output (its tiles
// 0-7 completed in the k-step's first half).
template <int V, class ActIn, class ActOut>
__device__ __forceinline__ void dense_layer(XRing &R, f4 (&in0)[16], f4 (&in1)[16],
                                            f4 (&out0)[16], f4 (&out1)[16], ActIn &&act_in,
                                            ActOut &&act_out) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int qn = q < 7 ? q + 1 : 7;
        xstep<V, 0>(R, out0, out1, in0[2 * q], in0[2 * q + 1], in1[2 * q], in1[2 * q + 1], [&] {
            if (q < 7) act_in(in0[2 * qn], in0[2 * qn + 1], qn, 0);
        });
        xstep<V, 1>(R, out0, out1, in0[2 * q], in0[2 * q + 1], in1[2 * q], in1[2 * q + 1], [&] {
            if (q < 7) {
                act_in(in1[2 * qn], in1[2 * qn + 1], qn, 1);
            } else {
                act_out(out0[0], out0[1], 0, 0);
                act_out(out1[0], out1[1], 0, 1);
            }
        });
    }
}

struct NoAct {
    __device__ __forceinline__ void operator()(f4 &, f4 &, int, int) const {}
};

template <int V>
__global__ void __launch_bounds__(kThreads, 1) ngp_field_x_kernel(const XFieldArgs a) {
    __shared__ f4 ring_lds[3 * kXSliceF4];                // 48 KB weight ring
    __shared__ float cst[kXCst];                           // 10 KB constants
    __shared__ float film_lds[kFilm * 2 * kW];             // 8 KB: the workgroup's face
    __shared__ f4 facc_lds[kWaves][16 * 64];               // 64 KB: feature accumulators
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t n = lane & 15u, g = lane >> 4;
    const GeomArgs &G = a.g;

    // a workgroup's 4 waves own 4 consecutive tiles of ONE face (grid = faces x
    // ceil(tiles_per_face / 4)), so the face's FiLM vectors are shared in LDS
    const uint32_t wg_per_face = (G.tiles_per_face + kWaves - 1) / kWaves;
    const uint32_t b = blockIdx.x / wg_per_face;
    uint32_t tile_local = (blockIdx.x % wg_per_face) * kWaves + wave;
    const bool tile_ok = tile_local < G.tiles_per_face;
    if (!tile_ok) tile_local = G.tiles_per_face - 1;
    const uint32_t tile = b * G.tiles_per_face + tile_local;
    uint32_t ray_local = (tile % G.tiles_per_face) * kTileRays + n;
    const bool ray_ok = tile_ok && ray_local < G.H * G.W;
    if (ray_local >= G.H * G.W) ray_local = G.H * G.W - 1;
    const uint32_t py = ray_local / G.W, px = ray_local % G.W;
    const uint32_t ray_index = (b * G.H + py) * G.W + px;

    Ray ray;
    make_ray(G.cam + (size_t)b * 12, G.focal[b], G.pix_x[px], G.pix_y[py], G.half_res, ray);
    const float nr = G.near_[b], fr = G.far_[b];
    const float dnorm = norm3_torch(ray.d[0], ray.d[1], ray.d[2]);
    // SH k-step fragment (identical for both sample columns): lanes g = 0, 1
    // hold SH 0-7 / 8-15, g = 2, 3 the zero padding of K = 272 -> 288
    f4 shh, shl;
    {
        const float v0 = G.static_viewdirs ? ray.dir[0] : ray.d[0];
        const float v1 = G.static_viewdirs ? ray.dir[1] : ray.d[1];
        const float v2 = G.static_viewdirs ? ray.dir[2] : ray.d[2];
        const float vn = norm3_torch(v0, v1, v2);
        const float ux = __fdiv_rn(v0, vn), uy = __fdiv_rn(v1, vn), uz = __fdiv_rn(v2, vn);
        const f4 qa = sh_quad(ux, uy, uz, (2 * g) & 3), qb = sh_quad(ux, uy, uz, (2 * g + 1) & 3);
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            v[r] = g < 2 ? qa[r] : 0.0f;
            v[4 + r] = g < 2 ? qb[r] : 0.0f;
        }
        split8(v, shh, shl);
    }
    const float beta_s = a.with_sdf ? a.sigmoid_beta[0] : 1.0f;
    {
        const f4 *src = reinterpret_cast<const f4 *>(a.film + (size_t)b * kFilm * 2 * kW);
        f4 *dst = reinterpret_cast<f4 *>(film_lds);
#pragma unroll
        for (uint32_t i = tid; i < kFilm * 2 * kW / 4; i += kThreads) dst[i] = src[i];
    }
    const float *film = film_lds;

    XRing R;
    R.lds = ring_lds;
    R.packed = a.packed;
    R.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<f4 *>(a.packed), 0,
                                               (int)(kXSlices * kXSliceF4 * sizeof(f4)),
                                               0x00020000);
    R.tid = tid;
    R.it = 0;
    // bias_s[5][256], 1/su of the input layer, sigma_linear row, rgb_linear rows
    for (uint32_t i = tid; i < kXCst; i += kThreads) {
        float v;
        if (i < 5 * kW) v = a.bias_s[i];
        else if (i < 6 * kW) v = __fdiv_rn(1.0f, a.su[i - 5 * kW]);
        else if (i < 7 * kW) v = a.sigma_w[i - 6 * kW];
        else v = a.rgb_w[i - 7 * kW];
        cst[i] = v;
    }
    // prologue: slices 0 (.. 1) -> slots; the next slice -> registers
    constexpr int kPro = 1 + SDFR_X_PREFETCH;
#pragma unroll
    for (int i = 0; i < kPro * kXStage; ++i) R.lds[tid + i * kThreads] = a.packed[tid + i * kThreads];
#pragma unroll
    for (int i = 0; i < kXStage; ++i) R.st[i] = a.packed[kPro * kXSliceF4 + tid + i * kThreads];
    __syncthreads();
    R.pre_h = R.lds[lane];
    R.pre_l = R.lds[64 + lane];

    f4 *facc = facc_lds[wave];
#pragma unroll
    for (int t = 0; t < 16; ++t) facc[t * 64 + lane] = f4{0.0f, 0.0f, 0.0f, 0.0f};
    float T = 1.0f, wsum = 0.0f, racc0 = 0.0f, racc1 = 0.0f, racc2 = 0.0f;
    float xacc0 = 0.0f, xacc1 = 0.0f, xacc2 = 0.0f, w_last = 0.0f;

    const float *bias_l = cst;                     // [5][256] (scaled)
    const float *inv_su0 = cst + 5 * kW;
    const float *sig_w = cst + 6 * kW, *rgb_w = cst + 7 * kW;
    const float *f0g = film, *f0b = film + kW, *f1g = film + 2 * kW, *f1b = film + 3 * kW;
    const float *f2g = film + 4 * kW, *f2b = film + 5 * kW, *f3g = film + 6 * kW,
                *f3b = film + 7 * kW;
    const float sig_b = a.sigma_b[0];
    const float rgb_b0 = a.rgb_b[0], rgb_b1 = a.rgb_b[1], rgb_b2 = a.rgb_b[2];

    // hash-grid features: lane group g holds levels 4g..4g+3 (K = 8g..8g+7)
    const float2 *enc2 = reinterpret_cast<const float2 *>(a.enc);
    const size_t tile_sid = (size_t)(tile * G.N) * kTileRays + n;
    float2 en[2][4];
    auto load_enc = [&](uint32_t s0) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            uint32_t s = s0 + j;
            if (s >= G.N) s = G.N - 1;
            const size_t sid = tile_sid + (size_t)s * kTileRays;
#pragma unroll
            for (int c = 0; c < 4; ++c) en[j][c] = enc2[(4 * g + c) * (size_t)G.S_total + sid];
        }
    };
    load_enc(0);

    const uint32_t npass = (G.N + 1) / 2;
    for (uint32_t p = 0; p < npass; ++p) {
        f4 X0[16], X1[16], Y0[16], Y1[16];
        f4 e0h, e0l, e1h, e1l;
        {
            float v0[8], v1[8];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                v0[2 * c] = en[0][c].x;
                v0[2 * c + 1] = en[0][c].y;
                v1[2 * c] = en[1][c].x;
                v1[2 * c + 1] = en[1][c].y;
            }
            split8(v0, e0h, e0l);
            split8(v1, e1h, e1l);
        }
        float sdfp0 = 0.0f, sdfp1 = 0.0f;
        auto act_id = [&](f4 &za, f4 &zb, int q, int) {
            float dummy = 0.0f;
            act_pair<0, V>(za, zb, q, inv_su0, nullptr, nullptr, dummy, g);
        };
        auto act_f0 = [&](f4 &za, f4 &zb, int q, int) {
            float dummy = 0.0f;
            act_pair<1, V>(za, zb, q, f0g, f0b, nullptr, dummy, g);
        };
        auto act_f1 = [&](f4 &za, f4 &zb, int q, int) {
            float dummy = 0.0f;
            act_pair<1, V>(za, zb, q, f1g, f1b, nullptr, dummy, g);
        };
        auto act_f2 = [&](f4 &za, f4 &zb, int q, int j) {
            if (j == 0) act_pair<2, V>(za, zb, q, f2g, f2b, sig_w, sdfp0, g);
            else act_pair<2, V>(za, zb, q, f2g, f2b, sig_w, sdfp1, g);
        };

        // layer 0: input_linear (32 -> 256) -> X
        init_acc(X0, bias_l, g);
        init_acc(X1, bias_l, g);
        xstep<V, 0>(R, X0, X1, e0h, e0l, e1h, e1l, [] {});
        xstep<V, 1>(R, X0, X1, e0h, e0l, e1h, e1l, [&] {
            act_id(X0[0], X0[1], 0, 0);
            act_id(X1[0], X1[1], 0, 1);
        });
        // layers 1-3: FiLM pts_linears.0..2
        init_acc(Y0, bias_l + kW, g);
        init_acc(Y1, bias_l + kW, g);
        dense_layer<V>(R, X0, X1, Y0, Y1, act_id, act_f0);
        init_acc(X0, bias_l + 2 * kW, g);
        init_acc(X1, bias_l + 2 * kW, g);
        dense_layer<V>(R, Y0, Y1, X0, X1, act_f0, act_f1);
        init_acc(Y0, bias_l + 3 * kW, g);
        init_acc(Y1, bias_l + 3 * kW, g);
        dense_layer<V>(R, X0, X1, Y0, Y1, act_f1, act_f2);
#if SDFR_X_EPI
        // layer 4: views FiLM ([h3, SH] 272 -> 256) -> X, output-group major (the
        // packing orders its 18 slices h-major): group 0 = tiles 0-7 over all 9
        // k-steps, activating h3 pair q+1 of both columns in k-step q's shadow;
        // group 1 = tiles 8-15, with the compositing of tiles 0-7 in its shadow.
        init_acc(X0, bias_l + 4 * kW, g);
        init_acc(X1, bias_l + 4 * kW, g);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int qn = q < 7 ? q + 1 : 7;
            xstep<V, 0>(R, X0, X1, Y0[2 * q], Y0[2 * q + 1], Y1[2 * q], Y1[2 * q + 1], [&] {
                if (q < 7) {
                    act_f2(Y0[2 * qn], Y0[2 * qn + 1], qn, 0);
                    act_f2(Y1[2 * qn], Y1[2 * qn + 1], qn, 1);
                }
            });
        }
#else
        // layer 4: views FiLM ([h3, SH] 272 -> 256) -> X; h3 pairs finish the sdf head
        init_acc(X0, bias_l + 4 * kW, g);
        init_acc(X1, bias_l + 4 * kW, g);
        dense_layer<V>(R, Y0, Y1, X0, X1, act_f2, NoAct{});
        xstep<V, 0>(R, X0, X1, shh, shl, shh, shl, [] {});
        xstep<V, 1>(R, X0, X1, shh, shl, shh, shl, [] {});
#endif
#if SDFR_X_EPI
        // volume_integration (sdf_model.py:236-301) weights of the pass's two
        // samples, front to back; a sample past N gets weight 0 (no branch, so
        // the compositing stays in the MFMA shadow)
        const uint32_t s0 = 2 * p, s1 = 2 * p + 1;
        const bool ok1 = s1 < G.N;
        float sdf0 = 0.0f, sdf1 = 0.0f, w0 = 0.0f, w1 = 0.0f;
        auto weights = [&] {
            sdf0 = __fadd_rn(group_sum(sdfp0), sig_b);
            sdf1 = __fadd_rn(group_sum(sdfp1), sig_b);
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
                const uint32_t s = jj ? s1 : s0;
                const uint32_t sc = s < G.N ? s : G.N - 1;
                const float sdf = jj ? sdf1 : sdf0;
                const float z = sample_z(G.sc, nr, fr, ray_index, sc);
                const float dist =
                    (sc + 1 < G.N)
                        ? __fmul_rn(__fsub_rn(sample_z(G.sc, nr, fr, ray_index, sc + 1), z), dnorm)
                        : __fmul_rn(1e10f, dnorm);
                float alpha;
                if (a.with_sdf) {
                    const float sig = __fdiv_rn(sigmoidf_(__fdiv_rn(-sdf, beta_s)), beta_s);
                    alpha = 1.0f - expf(-sig * dist);
                } else {
                    float raw = sdf;
                    if (a.sigma_noise) raw += a.sigma_noise[(size_t)ray_index * G.N + sc];
                    const float sp = raw > 20.0f ? raw : log1pf(expf(raw));
                    alpha = 1.0f - expf(-sp * dist);
                }
                float w = alpha * T;
                if (a.force_background && sc + 1 == G.N) w = 1.0f - wsum;
                const bool live = jj == 0 || ok1;
                if (live) {
                    T = T * ((1.0f - alpha) + 1e-10f);
                    wsum += w;
                }
                if (jj) w1 = live ? w : 0.0f;
                else w0 = w;
            }
            xpin(w0);
            xpin(w1);
        };
        // colour features f = sin(gamma_v' x + beta_v) of tile t, rgb_linear
        // partial dot products, feature compositing (sample s0 then s1)
        float q00 = 0.0f, q01 = 0.0f, q02 = 0.0f, q10 = 0.0f, q11 = 0.0f, q12 = 0.0f;
        auto epi_tile = [&](int t) {
            if constexpr ((V & 16) != 0) {
                racc0 += (X0[t][0] + X0[t][1]) + (X0[t][2] + X0[t][3]);
                racc1 += (X1[t][0] + X1[t][1]) + (X1[t][2] + X1[t][3]);
                return;
            }
            const int f0 = 16 * t + 4 * (int)g;
            const f4 gm = *reinterpret_cast<const f4 *>(f3g + f0);
            const f4 bt = *reinterpret_cast<const f4 *>(f3b + f0);
            const f4 wr0 = *reinterpret_cast<const f4 *>(rgb_w + f0);
            const f4 wr1 = *reinterpret_cast<const f4 *>(rgb_w + kW + f0);
            const f4 wr2 = *reinterpret_cast<const f4 *>(rgb_w + 2 * kW + f0);
            f4 fa, fb;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                fa[r] = sin_hw(__fadd_rn(__fmul_rn(gm[r], X0[t][r]), bt[r]));
                fb[r] = sin_hw(__fadd_rn(__fmul_rn(gm[r], X1[t][r]), bt[r]));
                q00 = __fmaf_rn(fa[r], wr0[r], q00);
                q01 = __fmaf_rn(fa[r], wr1[r], q01);
                q02 = __fmaf_rn(fa[r], wr2[r], q02);
                q10 = __fmaf_rn(fb[r], wr0[r], q10);
                q11 = __fmaf_rn(fb[r], wr1[r], q11);
                q12 = __fmaf_rn(fb[r], wr2[r], q12);
            }
            f4 v = facc[t * 64 + lane];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = __fmaf_rn(w0, fa[r], v[r]);
                v[r] = __fmaf_rn(w1, fb[r], v[r]);
            }
            facc[t * 64 + lane] = v;
            xpin(q00);
            xpin(q10);
        };
#if SDFR_X_EPI
        xstep<V, 0>(R, X0, X1, shh, shl, shh, shl, [&] { weights(); });
#pragma unroll
        for (int q = 0; q < 8; ++q)
            xstep<V, 1>(R, X0, X1, Y0[2 * q], Y0[2 * q + 1], Y1[2 * q], Y1[2 * q + 1],
                        [&] { epi_tile(q); });
        xstep<V, 1>(R, X0, X1, shh, shl, shh, shl, [] {});
        // next pass's hash-grid features, in flight behind the exposed compositing
        if (p + 1 < npass) load_enc(2 * p + 2);
#pragma unroll
        for (int t = 8; t < 16; ++t) epi_tile(t);
#endif

        // rgb head and the per-ray accumulators, sample s0 then s1
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
            if (jj && !ok1) break;
            const uint32_t s = jj ? s1 : s0;
            const float w = jj ? w1 : w0;
            const float r0 = __fadd_rn(group_sum(jj ? q10 : q00), rgb_b0);
            const float r1 = __fadd_rn(group_sum(jj ? q11 : q01), rgb_b1);
            const float r2 = __fadd_rn(group_sum(jj ? q12 : q02), rgb_b2);
            w_last = w;
            racc0 = __fmaf_rn(w, sigmoidf_(r0), racc0);
            racc1 = __fmaf_rn(w, sigmoidf_(r1), racc1);
            racc2 = __fmaf_rn(w, sigmoidf_(r2), racc2);
            if (a.xyz) {
                const float z = sample_z(G.sc, nr, fr, ray_index, s);
                xacc0 = __fmaf_rn(w, __fadd_rn(ray.o[0], __fmul_rn(ray.d[0], z)), xacc0);
                xacc1 = __fmaf_rn(w, __fadd_rn(ray.o[1], __fmul_rn(ray.d[1], z)), xacc1);
                xacc2 = __fmaf_rn(w, __fadd_rn(ray.o[2], __fmul_rn(ray.d[2], z)), xacc2);
            }
            if (a.sdf && ray_ok && g == 0) a.sdf[(size_t)ray_index * G.N + s] = jj ? sdf1 : sdf0;
        }
#else
        if (p + 1 < npass) load_enc(2 * p + 2);
        // compositing of the pass's two samples, front to back
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t s = 2 * p + j;
            if (s >= G.N) break;
            f4 (&Xj)[16] = j ? X1 : X0;
            const float sdf = __fadd_rn(group_sum(j ? sdfp1 : sdfp0), sig_b);
            const float z = sample_z(G.sc, nr, fr, ray_index, s);
            const float dist = (s + 1 < G.N)
                                   ? __fmul_rn(__fsub_rn(sample_z(G.sc, nr, fr, ray_index, s + 1), z),
                                               dnorm)
                                   : __fmul_rn(1e10f, dnorm);
            float alpha;
            if (a.with_sdf) {
                const float sig = __fdiv_rn(sigmoidf_(__fdiv_rn(-sdf, beta_s)), beta_s);
                alpha = 1.0f - expf(-sig * dist);
            } else {
                float raw = sdf;
                if (a.sigma_noise) raw += a.sigma_noise[(size_t)ray_index * G.N + s];
                const float sp = raw > 20.0f ? raw : log1pf(expf(raw));
                alpha = 1.0f - expf(-sp * dist);
            }
            float w = alpha * T;
            if (a.force_background && s + 1 == G.N) w = 1.0f - wsum;
            T = T * ((1.0f - alpha) + 1e-10f);
            wsum += w;
            // colour features f = sin(gamma_v' x + beta_v); rgb_linear; compositing
            float p0 = 0.0f, p1 = 0.0f, p2 = 0.0f;
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const int f0 = 16 * t + 4 * (int)g;
                const f4 gm = *reinterpret_cast<const f4 *>(f3g + f0);
                const f4 bt = *reinterpret_cast<const f4 *>(f3b + f0);
                const f4 w0 = *reinterpret_cast<const f4 *>(rgb_w + f0);
                const f4 w1 = *reinterpret_cast<const f4 *>(rgb_w + kW + f0);
                const f4 w2 = *reinterpret_cast<const f4 *>(rgb_w + 2 * kW + f0);
                f4 fv;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    fv[r] = sin_hw(__fadd_rn(__fmul_rn(gm[r], Xj[t][r]), bt[r]));
                    p0 = __fmaf_rn(fv[r], w0[r], p0);
                    p1 = __fmaf_rn(fv[r], w1[r], p1);
                    p2 = __fmaf_rn(fv[r], w2[r], p2);
                }
                Xj[t] = fv;
            }
            const float r0 = __fadd_rn(group_sum(p0), rgb_b0);
            const float r1 = __fadd_rn(group_sum(p1), rgb_b1);
            const float r2 = __fadd_rn(group_sum(p2), rgb_b2);
            w_last = w;
            racc0 = __fmaf_rn(w, sigmoidf_(r0), racc0);
            racc1 = __fmaf_rn(w, sigmoidf_(r1), racc1);
            racc2 = __fmaf_rn(w, sigmoidf_(r2), racc2);
            if (a.xyz) {
                xacc0 = __fmaf_rn(w, __fadd_rn(ray.o[0], __fmul_rn(ray.d[0], z)), xacc0);
                xacc1 = __fmaf_rn(w, __fadd_rn(ray.o[1], __fmul_rn(ray.d[1], z)), xacc1);
                xacc2 = __fmaf_rn(w, __fadd_rn(ray.o[2], __fmul_rn(ray.d[2], z)), xacc2);
            }
            if (a.features) {
#pragma unroll
                for (int t = 0; t < 16; ++t) {
                    f4 v = facc[t * 64 + lane];
                    v.x = __fmaf_rn(w, Xj[t].x, v.x);
                    v.y = __fmaf_rn(w, Xj[t].y, v.y);
                    v.z = __fmaf_rn(w, Xj[t].z, v.z);
                    v.w = __fmaf_rn(w, Xj[t].w, v.w);
                    facc[t * 64 + lane] = v;
                }
            }
            if (a.sdf && ray_ok && g == 0) a.sdf[(size_t)ray_index * G.N + s] = sdf;
        }
#endif
    }

    if (!ray_ok) return;
    const size_t HW = (size_t)G.H * G.W;
    const size_t pix = (size_t)py * G.W + px;
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
    if (a.features) {
        float *fb = a.features + (size_t)b * kW * HW + pix;
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const uint32_t jf = 16 * t + 4 * g;
            const f4 v = facc[t * 64 + lane];
            fb[(size_t)(jf + 0) * HW] = v.x;
            fb[(size_t)(jf + 1) * HW] = v.y;
            fb[(size_t)(jf + 2) * HW] = v.z;
            fb[(size_t)(jf + 3) * HW] = v.w;
        }
    }
}

// ----------------------------------------------------------------------------
// host
// ----------------------------------------------------------------------------
// workspace tail used by this path: packed [68][1024] f4 | su [5][256] | bias_s [5][256]
size_t f16x3_ws_bytes(uint32_t B) {
    (void)B;
    return (size_t)kXSlices * kXSliceF4 * sizeof(f4) + 2 * 5 * kW * sizeof(float);
}

static const float *xbias(const sdfr_ngp_weights *w, int l) {
    return l == 0 ? w->input_b : (l == 4 ? w->views_b : w->pts_b[l - 1]);
}
static const float *xweight(const sdfr_ngp_weights *w, int l) {
    return l == 0 ? w->input_w : (l == 4 ? w->views_w : w->pts_w[l - 1]);
}

int launch_xprep(const sdfr_ngp_weights *w, const sdfr_ngp_render_args *a, char *xws,
                 float *film, hipStream_t st) {
    f4 *packed = reinterpret_cast<f4 *>(xws);
    float *su = reinterpret_cast<float *>(xws + (size_t)kXSlices * kXSliceF4 * sizeof(f4));
    float *bias_s = su + 5 * kW;
    XScaleArgs sa;
    for (int l = 0; l < 5; ++l) {
        sa.w[l] = xweight(w, l);
        sa.b[l] = xbias(w, l);
    }
    sa.su = su;
    sa.bias_s = bias_s;
    hipLaunchKernelGGL(ngp_xscale_kernel, dim3(5), dim3(256), 0, st, sa);
    int rc = check_launch("render_ngp: xscale");
    if (rc) return rc;
    XPrepArgs p;
    p.styles = a->styles;
    for (int l = 0; l < 3; ++l) {
        p.gw[l] = w->pts_gw[l];
        p.gb[l] = w->pts_gb[l];
        p.bw[l] = w->pts_bw[l];
        p.bb[l] = w->pts_bb[l];
    }
    p.gw[3] = w->views_gw;
    p.gb[3] = w->views_gb;
    p.bw[3] = w->views_bw;
    p.bb[3] = w->views_bb;
    for (int l = 0; l < 5; ++l) p.w[l] = xweight(w, l);
    p.su = su;
    p.film = film;
    p.packed = packed;
    p.B = a->B;
    const uint32_t blocks = a->B * kFilm * 2 + (kXSlices * 512 + 255) / 256;
    hipLaunchKernelGGL(ngp_xprep_kernel, dim3(blocks), dim3(256), 0, st, p);
    return check_launch("render_ngp: xprep");
}

int launch_xfield(const sdfr_ngp_weights *w, const sdfr_ngp_render_args *a, const GeomArgs &g,
                  const float *enc, char *xws, const float *film, hipStream_t st) {
    XFieldArgs f;
    f.g = g;
    f.enc = enc;
    f.packed = reinterpret_cast<const f4 *>(xws);
    f.su = reinterpret_cast<const float *>(xws + (size_t)kXSlices * kXSliceF4 * sizeof(f4));
    f.bias_s = f.su + 5 * kW;
    f.film = film;
    f.sigma_w = w->sigma_w;
    f.sigma_b = w->sigma_b;
    f.rgb_w = w->rgb_w;
    f.rgb_b = w->rgb_b;
    f.sigmoid_beta = w->sigmoid_beta;
    f.sigma_noise = a->sigma_noise;
    f.force_background = a->force_background;
    f.with_sdf = a->with_sdf;
    f.rgb = a->rgb;
    f.features = a->features;
    f.sdf = a->sdf;
    f.xyz = a->xyz;
    f.mask = a->mask;
    const uint32_t blocks = g.B * ((g.tiles_per_face + kWaves - 1) / kWaves);
    switch (field_variant()) {
#ifdef SDFR_ABLATION
#define SDFR_XFIELD_CASE(V)                                                                  \
    case V:                                                                                  \
        hipLaunchKernelGGL(ngp_field_x_kernel<V>, dim3(blocks), dim3(kThreads), 0, st, f);   \
        break;
        SDFR_XFIELD_CASE(1)
        SDFR_XFIELD_CASE(2)
        SDFR_XFIELD_CASE(4)
        SDFR_XFIELD_CASE(8)
        SDFR_XFIELD_CASE(16)
        SDFR_XFIELD_CASE(31)
#undef SDFR_XFIELD_CASE
#endif
        default:
            hipLaunchKernelGGL(ngp_field_x_kernel<0>, dim3(blocks), dim3(kThreads), 0, st, f);
    }
    return check_launch("render_ngp: field (f16x3)");
}

}  // namespace sdfr
