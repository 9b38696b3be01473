// decoder.hip -- StyleGAN2 decoder ops for gfx950 (include/sdfr.h, "decoder ops").
//
// * sdfr_fused_bias_act / sdfr_upfirdn2d: drop-ins for the reference's two
//   native ops (fused_bias_act_kernel.cu:18-47, upfirdn2d_kernel.cu), same
//   argument meaning; element order of the arithmetic follows the reference
//   (x + bias, activation, * scale) so the bias/activation op is bit-exact.
// * sdfr_styled_epilogue: everything a StyledConv / ToRGB does after MIOpen's
//   convolution, in one streaming pass over NHWC activations:
//     [blur of the stride-2 transposed conv] -> demodulate -> + noise -> + bias
//     -> leaky ReLU * sqrt(2) -> (store, pre-multiplied by the NEXT conv's
//     modulation) and/or (1x1 ToRGB + upsampled skip).
//   The decoder thereby touches each activation tensor once for reading and
//   once for writing; the last layer's activations are never stored.
// * sdfr_modulate_to_nhwc: renderer features (NCHW) -> NHWC times the first
//   conv's modulation, an LDS-tiled transpose.
//
// All of these are HBM-streaming kernels: 16-B per lane accesses along the
// contiguous axis, >= 8 waves per CU, no LDS except the transpose tile.
#include <hip/hip_runtime.h>

#include <algorithm>

#include <string>

#include "sdfr_common.h"

namespace sdfr {

// ----------------------------------------------------------------------------
// fused_bias_act (fused_bias_act_kernel.cu:18-47)
// ----------------------------------------------------------------------------
__device__ __forceinline__ float fba(float x, float ref, int mode, float alpha) {
    switch (mode) {
        case 30: return x > 0.0f ? x : x * alpha;
        case 31: return ref > 0.0f ? x : x * alpha;
        case 12:
        case 32: return 0.0f;
        default: return x;
    }
}

__global__ __launch_bounds__(256) void fused_bias_act_kernel(
    float *__restrict__ out, const float *__restrict__ x, const float *__restrict__ bias,
    const float *__restrict__ ref, uint64_t n, uint32_t step_b, uint32_t size_b, int mode,
    float alpha, float scale) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        float v = x[i];
        if (bias) v = v + bias[(i / step_b) % size_b];
        const float r = ref ? ref[i] : 0.0f;
        out[i] = fba(v, r, mode, alpha) * scale;
    }
}

// 4 consecutive elements share a bias entry (step_b % 4 == 0, n % 4 == 0)
__global__ __launch_bounds__(256) void fused_bias_act_vec_kernel(
    float4 *__restrict__ out, const float4 *__restrict__ x, const float *__restrict__ bias,
    const float4 *__restrict__ ref, uint64_t n4, uint32_t step_b4, uint32_t size_b, int mode,
    float alpha, float scale) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        float4 v = x[i];
        if (bias) {
            const float b = bias[(i / step_b4) % size_b];
            v.x = v.x + b; v.y = v.y + b; v.z = v.z + b; v.w = v.w + b;
        }
        const float4 r = ref ? ref[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        float4 o;
        o.x = fba(v.x, r.x, mode, alpha) * scale;
        o.y = fba(v.y, r.y, mode, alpha) * scale;
        o.z = fba(v.z, r.z, mode, alpha) * scale;
        o.w = fba(v.w, r.w, mode, alpha) * scale;
        out[i] = o;
    }
}

// ----------------------------------------------------------------------------
// upfirdn2d (upfirdn2d_native semantics, sdf_op.py:273-316), one output / thread
// ----------------------------------------------------------------------------
struct UfdArgs {
    float *out;
    const float *in, *k;
    uint32_t major, in_h, in_w, kh, kw, out_h, out_w;
    int up_x, up_y, down_x, down_y, pad_x0, pad_y0;
};

__global__ __launch_bounds__(256) void upfirdn2d_kernel(UfdArgs a) {
    const uint64_t total = (uint64_t)a.major * a.out_h * a.out_w;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const int uh = (int)a.in_h * a.up_y, uw = (int)a.in_w * a.up_x;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
        const uint32_t ox = (uint32_t)(t % a.out_w);
        const uint32_t oy = (uint32_t)((t / a.out_w) % a.out_h);
        const uint64_t m = t / ((uint64_t)a.out_w * a.out_h);
        const float *src = a.in + m * a.in_h * a.in_w;
        float acc = 0.0f;
        for (uint32_t i = 0; i < a.kh; ++i) {
            const int r = (int)(oy * a.down_y + i) - a.pad_y0;   // row in the upsampled image
            if (r < 0 || r >= uh || r % a.up_y) continue;
            const float *row = src + (uint64_t)(r / a.up_y) * a.in_w;
            const float *krow = a.k + (uint64_t)(a.kh - 1 - i) * a.kw;
            for (uint32_t j = 0; j < a.kw; ++j) {
                const int c = (int)(ox * a.down_x + j) - a.pad_x0;
                if (c < 0 || c >= uw || c % a.up_x) continue;
                acc = fmaf(row[c / a.up_x], krow[a.kw - 1 - j], acc);
            }
        }
        a.out[t] = acc;
    }
}

// Tiled form for the 4x4 filters of the decoder and discriminator (Blur, Upsample and
// their gradients: up / down factors (1,1), (2,1), (1,2) on both axes).  A workgroup
// stages its output tile's input window (with the filter halo, zeros outside the
// image) in LDS with coalesced loads, then each lane computes TH/4 outputs of one
// column from LDS.  The taps are summed in upfirdn2d_kernel's order (i, then j,
// ascending; out-of-image taps add an exact zero), so results are the same bit for
// bit up to the sign of an all-zero sum.  The generic kernel above takes one output
// per thread with every input tap re-read through L1 and 64-bit index divisions:
// ~90 us per call on the discriminator's blurs, ~4-10x its HBM time.
__device__ __forceinline__ int floor_div(int n, int d) { return (n >= 0 ? n : n - d + 1) / d; }

template <int UP, int DOWN>
__global__ __launch_bounds__(256) void upfirdn2d_tile_kernel(UfdArgs a, uint32_t tiles_x,
                                                             uint32_t tiles_y) {
    constexpr int K = 4;
    constexpr int TW = 64, TH = 32 / DOWN, RPT = TH / 4;
    constexpr int IH = ((TH - 1) * DOWN + K - 1) / UP + 2;
    constexpr int IW = ((TW - 1) * DOWN + K - 1) / UP + 2;
    __shared__ float tile[IH * IW];
    const uint32_t bx = blockIdx.x;
    const uint32_t txi = bx % tiles_x, rest = bx / tiles_x;
    const uint32_t tyi = rest % tiles_y, m = rest / tiles_y;
    const int oy0 = (int)tyi * TH, ox0 = (int)txi * TW;
    const int ry0 = oy0 * DOWN - a.pad_y0, rx0 = ox0 * DOWN - a.pad_x0;   // upsampled coords
    const int iy0 = floor_div(ry0, UP), ix0 = floor_div(rx0, UP);
    const int in_h = (int)a.in_h, in_w = (int)a.in_w;
    const float *__restrict__ src = a.in + (uint64_t)m * a.in_h * a.in_w;
    for (int e = threadIdx.x; e < IH * IW; e += 256) {
        const int r = e / IW, c = e - r * IW;
        const int iy = iy0 + r, ix = ix0 + c;
        float v = 0.0f;
        if (iy >= 0 && iy < in_h && ix >= 0 && ix < in_w) v = src[(uint64_t)iy * a.in_w + ix];
        tile[e] = v;
    }
    float kf[K][K];                 // kf[i][j]: the tap upfirdn2d_kernel applies at (i, j)
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < K; ++j) kf[i][j] = a.k[(K - 1 - i) * K + (K - 1 - j)];
    __syncthreads();
    const int lx = threadIdx.x & 63, gy = threadIdx.x >> 6;
    const int ox = ox0 + lx;
    const int cx = lx * DOWN + (rx0 - ix0 * UP);      // tile column (upsampled) of tap j = 0
    float *__restrict__ dst = a.out + (uint64_t)m * a.out_h * a.out_w;
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
        const int oyl = gy * RPT + q;
        const int cy = oyl * DOWN + (ry0 - iy0 * UP);
        float acc = 0.0f;
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const int ry = cy + i;
            if (UP > 1 && (ry % UP)) continue;
            const float *row = tile + (ry / UP) * IW;
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const int rx = cx + j;
                if (UP > 1 && (rx % UP)) continue;
                acc = fmaf(row[rx / UP], kf[i][j], acc);
            }
        }
        const int oy = oy0 + oyl;
        if (oy < (int)a.out_h && ox < (int)a.out_w) dst[(uint64_t)oy * a.out_w + ox] = acc;
    }
}

template <int UP, int DOWN>
static void launch_ufd_tile(const UfdArgs &a, hipStream_t st) {
    constexpr int TW = 64, TH = 32 / DOWN;
    const uint32_t tx = (a.out_w + TW - 1) / TW, ty = (a.out_h + TH - 1) / TH;
    upfirdn2d_tile_kernel<UP, DOWN><<<(uint32_t)((uint64_t)tx * ty * a.major), 256, 0, st>>>(a, tx, ty);
}

// ----------------------------------------------------------------------------
// styled-conv epilogue
// ----------------------------------------------------------------------------
struct EpiArgs {
    uint32_t B, C, H, W;
    const float *conv;
    float fir[4];
    const float *demod, *noise, *noise_weight, *bias;
    float slope, act_scale;
    const float *s_next;
    float *y;
    const float *rgb_w, *rgb_b, *skip;
    float *rgb;
    _Float16 *ys;          // split-NHWC fp16 output (instead of y) or null
};

typedef _Float16 h4v __attribute__((ext_vector_type(4)));

// Round-to-nearest hi/lo fp16 split of 4 channels c .. c+3 (c % 4 == 0, C % 8 == 0)
// at NHWC element index idx = pix C + c, stored split-NHWC ([pix][C/8][hi 8, lo 8]):
// hi at 2 idx - (c & 7), lo 8 halves further.
__device__ __forceinline__ void store_split4(_Float16 *ys, size_t idx, float4 v) {
    h4v h, l;
    h[0] = (_Float16)v.x; h[1] = (_Float16)v.y; h[2] = (_Float16)v.z; h[3] = (_Float16)v.w;
    l[0] = (_Float16)(v.x - (float)h[0]);
    l[1] = (_Float16)(v.y - (float)h[1]);
    l[2] = (_Float16)(v.z - (float)h[2]);
    l[3] = (_Float16)(v.w - (float)h[3]);
    const size_t o = 2 * idx - (idx & 7u);
    *reinterpret_cast<h4v *>(ys + o) = h;
    *reinterpret_cast<h4v *>(ys + o + 8) = l;
}

// y (pre-multiplied by the next modulation) as fp32, or as the split-NHWC fp16
// the split-fp16 convolution consumes (conv_f16x3.hip)
__device__ __forceinline__ void store_y(const EpiArgs &a, size_t idx, float4 v) {
    if (a.ys) store_split4(a.ys, idx, v);
    else *reinterpret_cast<float4 *>(a.y + idx) = v;
}

// store_y for threads whose neighbour lane (lane ^ 1) holds channels c ^ 4 of the same
// pixel (epi_blur_kernel: channel quad fastest, C % 8 == 0): the split store goes out
// as ONE 16-B store per lane -- the even lane writes the 8 channels' hi halves, the
// odd lane their lo halves -- after one DPP quad_perm [1,0,3,2] exchange per dword
// instead of two 8-B stores per lane.  Both lanes of a pair must execute it.
__device__ __forceinline__ void store_y_pair(const EpiArgs &a, size_t idx, float4 v) {
    if (!a.ys) {
        *reinterpret_cast<float4 *>(a.y + idx) = v;
        return;
    }
    h4v h, l;
    h[0] = (_Float16)v.x; h[1] = (_Float16)v.y; h[2] = (_Float16)v.z; h[3] = (_Float16)v.w;
    l[0] = (_Float16)(v.x - (float)h[0]);
    l[1] = (_Float16)(v.y - (float)h[1]);
    l[2] = (_Float16)(v.z - (float)h[2]);
    l[3] = (_Float16)(v.w - (float)h[3]);
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    const u2 hd = __builtin_bit_cast(u2, h), ld = __builtin_bit_cast(u2, l);
    const bool odd = (idx & 4u) != 0;
    uint32_t q[4];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t send = odd ? hd[k] : ld[k];     // what the partner lane keeps
        const uint32_t recv = (uint32_t)__builtin_amdgcn_mov_dpp((int)send, 0xB1, 0xF, 0xF, false);
        q[k] = odd ? recv : hd[k];                     // even: own hi, partner hi
        q[2 + k] = odd ? ld[k] : recv;                 // odd: partner lo, own lo
    }
    const size_t i8 = idx & ~(size_t)7;
    *reinterpret_cast<uint4 *>(a.ys + 2 * i8 + (odd ? 8 : 0)) = __builtin_bit_cast(uint4, q);
}

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }

__device__ __forceinline__ float act1(float c, float dm, float nz, float b, float slope,
                                      float scale) {
    float v = c * dm;
    v = v + nz;          // image + weight * noise (sdf_model.py NoiseInjection)
    v = v + b;           // fused_bias_act: x + bias, lrelu, * scale
    v = v > 0.0f ? v : v * slope;
    return v * scale;
}

__device__ __forceinline__ float4 act4(float4 c, float4 dm, float nz, float4 b, float slope,
                                       float scale) {
    return make_float4(act1(c.x, dm.x, nz, b.x, slope, scale), act1(c.y, dm.y, nz, b.y, slope, scale),
                       act1(c.z, dm.z, nz, b.z, slope, scale), act1(c.w, dm.w, nz, b.w, slope, scale));
}

// skip image upsampled by upfirdn2d(up=2, pad=(2,1), outer(fir,fir)) at (y, x)
__device__ float skip_up(const float *__restrict__ img, uint32_t h2, uint32_t w2, int y, int x,
                         const float *fir) {
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = y + i - 2;
        if (r < 0 || (r & 1) || (r >> 1) >= (int)h2) continue;
        float row = 0.0f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = x + j - 2;
            if (c < 0 || (c & 1) || (c >> 1) >= (int)w2) continue;
            row = fmaf(img[(uint32_t)(r >> 1) * w2 + (uint32_t)(c >> 1)], fir[3 - j], row);
        }
        acc = fmaf(row, fir[3 - i], acc);
    }
    return acc;
}

constexpr uint32_t kEpiPixPerBlock = 64;

// Plain epilogue: TPP lanes per pixel (C/4 up to 16, 16 up to C = 256, 64 above),
// NQ = C/(4 TPP) float4 each,
// PPW = 64/TPP pixels per wave at a time; the 1x1 ToRGB is a TPP-lane reduction
// (log2 TPP shuffle steps).  Few channels per lane keep the per-channel constants
// small (high occupancy), and CH pixel rounds are loaded before any is used so
// ~8 float4 per lane are in flight (the pass is HBM-bound).
template <int NQ, bool RGB>
__global__ __launch_bounds__(256) void epi_plain_kernel(EpiArgs a, uint32_t tpp_log2) {
    constexpr int CH = NQ >= 8 ? 1 : 8 / NQ;
    const uint32_t TPP = 1u << tpp_log2;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t q = lane & (TPP - 1), g = lane >> tpp_log2;
    const uint32_t ppw = 64u >> tpp_log2;
    const uint32_t b = blockIdx.y;
    const uint32_t HW = a.H * a.W, C = a.C;

    float4 dm[NQ], bs[NQ], sn[NQ], rw[3][NQ];
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
        const uint32_t c = 4 * (q + k * TPP);
        dm[k] = a.demod ? ld4(a.demod + (size_t)b * C + c) : make_float4(1.f, 1.f, 1.f, 1.f);
        bs[k] = ld4(a.bias + c);
        sn[k] = a.s_next ? ld4(a.s_next + (size_t)b * C + c) : make_float4(1.f, 1.f, 1.f, 1.f);
        if (RGB) {
#pragma unroll
            for (int o = 0; o < 3; ++o) rw[o][k] = ld4(a.rgb_w + ((size_t)b * 3 + o) * C + c);
        }
    }
    const float nw = a.noise ? *a.noise_weight : 0.0f;
    const uint32_t p0 = blockIdx.x * kEpiPixPerBlock;
    const uint32_t step = 4 * ppw;                       // pixels between a lane's rounds
    for (uint32_t pp0 = wave * ppw + g; pp0 < kEpiPixPerBlock; pp0 += CH * step) {
        float4 cv[CH][NQ];
        float nz[CH];
#pragma unroll
        for (int r = 0; r < CH; ++r) {
            const uint32_t pp = pp0 + r * step, p = p0 + pp;
            const bool live = pp < kEpiPixPerBlock && p < HW;
            const size_t base = ((size_t)b * HW + (live ? p : 0)) * C;
            nz[r] = (a.noise && live) ? nw * a.noise[(size_t)b * HW + p] : 0.0f;
#pragma unroll
            for (int k = 0; k < NQ; ++k)
                cv[r][k] = live ? ld4(a.conv + base + 4 * (q + k * TPP)) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int r = 0; r < CH; ++r) {
            const uint32_t pp = pp0 + r * step, p = p0 + pp;
            const bool live = pp < kEpiPixPerBlock && p < HW;
            if (!RGB && !live) continue;
            const size_t base = ((size_t)b * HW + p) * C;
            float acc[3] = {0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < NQ; ++k) {
                const uint32_t c = 4 * (q + k * TPP);
                const float4 v = act4(cv[r][k], dm[k], nz[r], bs[k], a.slope, a.act_scale);
                if (live && (a.y || a.ys))
                    store_y(a, base + c,
                            make_float4(v.x * sn[k].x, v.y * sn[k].y, v.z * sn[k].z, v.w * sn[k].w));
                if (RGB) {
#pragma unroll
                    for (int o = 0; o < 3; ++o) {
                        acc[o] = fmaf(v.x, rw[o][k].x, acc[o]);
                        acc[o] = fmaf(v.y, rw[o][k].y, acc[o]);
                        acc[o] = fmaf(v.z, rw[o][k].z, acc[o]);
                        acc[o] = fmaf(v.w, rw[o][k].w, acc[o]);
                    }
                }
            }
            if (RGB) {
                for (uint32_t off = TPP >> 1; off; off >>= 1) {
#pragma unroll
                    for (int o = 0; o < 3; ++o) acc[o] += __shfl_xor(acc[o], off, 64);
                }
                // the butterfly left the sums in every lane: lane q < 3 finishes channel q
                if (live && q < 3) {
                    const int yy = (int)(p / a.W), xx = (int)(p % a.W);
                    float v = (q == 0 ? acc[0] : q == 1 ? acc[1] : acc[2]) + a.rgb_b[q];
                    if (a.skip)
                        v = v + skip_up(a.skip + ((size_t)b * 3 + q) * (HW / 4), a.H / 2, a.W / 2,
                                        yy, xx, a.fir);
                    a.rgb[((size_t)b * 3 + q) * HW + p] = v;
                }
            }
        }
    }
}

// Blur epilogue: thread = (face, row segment, column, channel quad); a sliding
// window of 4 horizontally filtered input rows gives the 4x4 separable blur
// with one new 16-B load per tap column per output row.
#ifndef BLUR_ROWS
#define BLUR_ROWS 16
#endif
#ifndef BLUR_GROUP
#define BLUR_GROUP 4
#endif
constexpr uint32_t kBlurRows = BLUR_ROWS;
constexpr int kBlurGroup = BLUR_GROUP;   // input rows loaded together (kBlurRows % it == 0)
#ifndef BLUR_COLS
#define BLUR_COLS 4
#endif
constexpr int kBlurCols = BLUR_COLS;     // adjacent output columns per thread
// XCD-aware block order: the dispatcher deals blocks round-robin over the 8 XCDs, so
// logically adjacent blocks (which share 3 input columns) would each fill the shared
// lines into a different L2; remapped, blocks p and p + 8 (same XCD, dispatched
// together) take adjacent column groups.  The grid is padded to a multiple of 8.
#ifndef BLUR_XCD
#define BLUR_XCD 1
#endif

// rps: output rows per segment (a multiple of kBlurGroup, at most kBlurRows): small
// batches use shorter segments so the grid still covers the chip
__global__ __launch_bounds__(256) void epi_blur_kernel(EpiArgs a, uint32_t nseg, uint32_t rps) {
    constexpr int NC = kBlurCols;                     // output columns per thread
    const uint32_t Q = a.C >> 2;
    const uint32_t WG = (a.W + NC - 1) / NC;           // column groups
    uint32_t bid = blockIdx.x;
    if (BLUR_XCD) bid = (bid & 7u) * (gridDim.x >> 3) + (bid >> 3);
    // (32-bit index arithmetic: the host keeps the thread count below 2^31)
    const uint32_t t = bid * blockDim.x + threadIdx.x;
    const uint32_t total = a.B * nseg * WG * Q;
    if (t >= total) return;
    const uint32_t q = t % Q;
    const uint32_t r1 = t / Q;
    const uint32_t ox0 = (r1 % WG) * NC;
    const uint32_t r2 = r1 / WG;
    const uint32_t seg = r2 % nseg;
    const uint32_t b = r2 / nseg;
    const uint32_t c = 4 * q;
    const uint32_t Hi = a.H + 1, Wi = a.W + 1, C = a.C;
    const float *src = a.conv + (size_t)b * Hi * Wi * C + c;
    const float f0 = a.fir[3], f1 = a.fir[2], f2 = a.fir[1], f3 = a.fir[0];   // flipped taps

    // input columns ox0 - 1 .. ox0 + NC + 1 of row r (shared by the NC outputs);
    // loads and filter split so that a group of rows is loaded before any is
    // filtered (4 rows x (NC + 3) loads in flight)
    auto hload = [&](int r, float4 (&v)[NC + 3]) {
        const bool rok = r >= 0 && r < (int)Hi;
        const float *row = src + (size_t)(rok ? r : 0) * Wi * C;
#pragma unroll
        for (int j = 0; j < NC + 3; ++j) {
            const int cc = (int)ox0 + j - 1;
            v[j] = (rok && cc >= 0 && cc < (int)Wi) ? ld4(row + (size_t)cc * C)
                                                    : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto hfilt = [&](const float4 (&v)[NC + 3], int k) -> float4 {   // output column ox0 + k
        const float fj[4] = {f0, f1, f2, f3};
        float4 h = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            h.x = fmaf(v[k + j].x, fj[j], h.x); h.y = fmaf(v[k + j].y, fj[j], h.y);
            h.z = fmaf(v[k + j].z, fj[j], h.z); h.w = fmaf(v[k + j].w, fj[j], h.w);
        }
        return h;
    };

    const float4 dm = a.demod ? ld4(a.demod + (size_t)b * C + c) : make_float4(1.f, 1.f, 1.f, 1.f);
    const float4 bs = ld4(a.bias + c);
    const float4 sn = a.s_next ? ld4(a.s_next + (size_t)b * C + c) : make_float4(1.f, 1.f, 1.f, 1.f);
    const float nw = a.noise ? *a.noise_weight : 0.0f;
    const uint32_t y0 = seg * rps;
    const uint32_t y1 = min(a.H, y0 + rps);
    float4 h0[NC], h1[NC], h2[NC];
    {
        float4 v0[NC + 3], v1[NC + 3], v2[NC + 3];
        hload((int)y0 - 1, v0);
        hload((int)y0, v1);
        hload((int)y0 + 1, v2);
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            h0[k] = hfilt(v0, k);
            h1[k] = hfilt(v1, k);
            h2[k] = hfilt(v2, k);
        }
    }
    for (uint32_t oy0 = y0; oy0 < y1; oy0 += kBlurGroup) {
        float4 v[kBlurGroup][NC + 3];
        float nz[kBlurGroup][NC];
#pragma unroll
        for (int g = 0; g < kBlurGroup; ++g) {
            hload((int)(oy0 + g) + 2, v[g]);
            const size_t prow = ((size_t)b * a.H + min(oy0 + g, a.H - 1)) * a.W;
#pragma unroll
            for (int k = 0; k < NC; ++k)
                nz[g][k] = a.noise ? nw * a.noise[prow + min(ox0 + k, a.W - 1)] : 0.0f;
        }
#pragma unroll
        for (int g = 0; g < kBlurGroup; ++g) {
            const uint32_t oy = oy0 + g;
#pragma unroll
            for (int k = 0; k < NC; ++k) {
                const float4 h3 = hfilt(v[g], k);
                if (oy < y1 && ox0 + k < a.W) {
                    float4 s;
                    s.x = fmaf(h3.x, f3, fmaf(h2[k].x, f2, fmaf(h1[k].x, f1, h0[k].x * f0)));
                    s.y = fmaf(h3.y, f3, fmaf(h2[k].y, f2, fmaf(h1[k].y, f1, h0[k].y * f0)));
                    s.z = fmaf(h3.z, f3, fmaf(h2[k].z, f2, fmaf(h1[k].z, f1, h0[k].z * f0)));
                    s.w = fmaf(h3.w, f3, fmaf(h2[k].w, f2, fmaf(h1[k].w, f1, h0[k].w * f0)));
                    const size_t pix = ((size_t)b * a.H + oy) * a.W + ox0 + k;
                    const float4 vv = act4(s, dm, nz[g][k], bs, a.slope, a.act_scale);
                    store_y_pair(a, pix * C + c,
                                 make_float4(vv.x * sn.x, vv.y * sn.y, vv.z * sn.z, vv.w * sn.w));
                }
                h0[k] = h1[k];
                h1[k] = h2[k];
                h2[k] = h3;
            }
        }
    }
}

// ToRGB finish after the conv-fused epilogue: one thread per 4 adjacent pixels of a
// row (float4), grid (W/4 / 64, H / 4, B * 3 planes).  The upsampled skip
// (upfirdn2d up 2, pad (2, 1), outer(fir, fir)) in closed form: a pixel of row / column
// parity p takes source rows / columns (y - 2 + p) / 2 + {0, 1} with taps fir[3 - p],
// fir[1 - p] -- the same products summed in the same order as skip_up's loop (which
// skips the odd taps), out-of-image sources as zeros (fma of 0 leaves the sum as is):
// bit-identical, without skip_up's 16-iteration branchy loop per pixel (the kernel was
// VALU-bound at 1.2 TB/s on the 256^2 layer).
__global__ __launch_bounds__(256) void rgb_finish_kernel(float *__restrict__ rgb,
                                                         const float *__restrict__ part,
                                                         uint32_t nparts, const float *rgb_b,
                                                         const float *__restrict__ skip,
                                                         float f0, float f1, float f2, float f3,
                                                         uint32_t B, uint32_t H, uint32_t W) {
    const uint32_t q = blockIdx.x * 64 + (threadIdx.x & 63u), y = blockIdx.y * 4 + (threadIdx.x >> 6);
    const uint32_t bo = blockIdx.z, o = bo % 3;
    if (4 * q >= W || y >= H) return;
    const size_t HW = (size_t)H * W, n = (size_t)B * 3 * HW;
    const size_t t = (size_t)bo * HW + (size_t)y * W + 4 * q;
    float4 v = ld4(part + t);
    for (uint32_t k = 1; k < nparts; ++k) {
        const float4 u = ld4(part + k * n + t);
        v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
    }
    const float bias = rgb_b[o];
    v.x = v.x + bias; v.y = v.y + bias; v.z = v.z + bias; v.w = v.w + bias;
    if (skip) {
        const float fir[4] = {f0, f1, f2, f3};
        const int h2 = (int)(H / 2), w2 = (int)(W / 2);
        const float *img = skip + (size_t)bo * (HW / 4);
        const int py = (int)(y & 1u), r0 = ((int)y - 2 + py) / 2;    // rows r0, r0 + 1
        const float wy0 = fir[3 - py], wy1 = fir[1 - py];
        // source columns 2q - 1 .. 2q + 2 of rows r0, r0 + 1
        float s[2][4];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int r = r0 + a, cc = 2 * (int)q - 1 + c;
                s[a][c] = (r >= 0 && r < h2 && cc >= 0 && cc < w2) ? img[r * w2 + cc] : 0.0f;
            }
        float out[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const int px = d & 1, c0 = (d >> 1) + px;      // column index into s: 2q-1+c0
            const float wx0 = fir[3 - px], wx1 = fir[1 - px];
            float row[2];
#pragma unroll
            for (int a = 0; a < 2; ++a) row[a] = fmaf(s[a][c0 + 1], wx1, fmaf(s[a][c0], wx0, 0.0f));
            out[d] = fmaf(row[1], wy1, fmaf(row[0], wy0, 0.0f));
        }
        v.x = v.x + out[0]; v.y = v.y + out[1]; v.z = v.z + out[2]; v.w = v.w + out[3];
    }
    *reinterpret_cast<float4 *>(rgb + t) = v;
}

// ----------------------------------------------------------------------------
// NCHW -> NHWC with modulation, 64 x 64 LDS tiles
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void modulate_nhwc_kernel(float *__restrict__ y,
                                                            _Float16 *__restrict__ ys,
                                                            const float *__restrict__ x,
                                                            const float *__restrict__ s,
                                                            uint32_t C, uint32_t HW) {
    __shared__ float tile[64][65];
    const uint32_t b = blockIdx.z, c0 = blockIdx.y * 64, p0 = blockIdx.x * 64;
    const uint32_t t = threadIdx.x;
    // load: 16 threads x float4 cover 64 pixels of one channel; 16 channels per pass
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t cl = (t >> 4) + 16 * k, pl = 4 * (t & 15);
        const uint32_t c = c0 + cl, p = p0 + pl;
        if (c < C && p < HW) {
            const float4 v = ld4(x + ((size_t)b * C + c) * HW + p);
            const float sc = s[(size_t)b * C + c];
            tile[cl][pl + 0] = v.x * sc; tile[cl][pl + 1] = v.y * sc;
            tile[cl][pl + 2] = v.z * sc; tile[cl][pl + 3] = v.w * sc;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t pl = (t >> 4) + 16 * k, cl = 4 * (t & 15);
        const uint32_t c = c0 + cl, p = p0 + pl;
        if (c < C && p < HW) {
            const float4 v =
                make_float4(tile[cl][pl], tile[cl + 1][pl], tile[cl + 2][pl], tile[cl + 3][pl]);
            const size_t idx = ((size_t)b * HW + p) * C + c;
            if (ys) store_split4(ys, idx, v);
            else *reinterpret_cast<float4 *>(y + idx) = v;
        }
    }
}

static uint32_t grid_for(uint64_t n, uint32_t per_block = 256) {
    const uint64_t blocks = (n + per_block - 1) / per_block;
    return (uint32_t)std::min<uint64_t>(blocks, 1u << 20);
}

static inline bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace sdfr

using namespace sdfr;

extern "C" {

// ----------------------------------------------------------------------------
// mapping-network layer for inference: out = act(x . (W wscale)^T + b bscale) act_scale,
// optionally PixelNorm on x first (sdf_model.py:437-466 MappingLinear, EqualLinear +
// fused_leaky_relu, PixelNorm; the whole layer in one launch -- at eval.py's batch of
// 1 the module path's 3-4 kernels per layer (scale multiply, GEMM, bias + act) cost
// more than their arithmetic).
// A workgroup owns 4 outputs, one wave each; lane l of a wave takes K-slice l
// (K/64 inputs, one contiguous piece of the weight row, so a wave reads the row as
// one coalesced run) for up to 16 samples, and the 64 slice partials of a sample
// are summed by a butterfly of lane exchanges (fixed order: deterministic; not
// the GEMM's order).  128 workgroups for a 512-wide layer at any batch.
// ----------------------------------------------------------------------------
constexpr uint32_t kMapOut = 4, kMapB = 16, kMapMaxK = 512;

struct MapArgs {
    const float *x, *w, *b;
    float *out;
    uint32_t B, K, O;
    float wscale, bscale, slope, act_scale;
    int act, pixelnorm;
};

__global__ __launch_bounds__(256) void mapping_linear_kernel(const MapArgs a) {
    __shared__ __attribute__((aligned(16))) float xs[kMapB * kMapMaxK];
    __shared__ float nrm[kMapB];
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    const uint32_t o = blockIdx.x * kMapOut + wv;
    const uint32_t kl = a.K / 64, k0 = lane * kl;
    // this lane's weight slice (K <= 512: at most 2 float4) is loaded before the
    // activations, so the two global-memory round trips of a layer overlap (a small
    // batch's launch is that latency)
    float4 wpre[kMapMaxK / 256];
#pragma unroll
    for (uint32_t k = 0; k < kMapMaxK / 256; ++k)
        wpre[k] = (o < a.O && 4 * k < kl) ? *reinterpret_cast<const float4 *>(a.w + (size_t)o * a.K + k0 + 4 * k)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
    for (uint32_t b0 = blockIdx.y * kMapB; b0 < a.B; b0 += gridDim.y * kMapB) {
        const uint32_t nb = min(kMapB, a.B - b0);
        if ((reinterpret_cast<uintptr_t>(a.x) & 15u) == 0) {
            // 16-B loads, up to 8 in flight per thread (a one-float-per-iteration loop
            // was a chain of up to 32 dependent L2 round trips at 16 samples)
            const float4 *x4 = reinterpret_cast<const float4 *>(a.x + (size_t)b0 * a.K);
            float4 *xs4 = reinterpret_cast<float4 *>(xs);
            const uint32_t n4 = nb * a.K / 4;
#pragma unroll 8
            for (uint32_t i = t; i < n4; i += 256) xs4[i] = x4[i];
        } else {
            for (uint32_t i = t; i < nb * a.K; i += 256) xs[i] = a.x[(size_t)b0 * a.K + i];
        }
        __syncthreads();
        if (a.pixelnorm) {                       // x * rsqrt(mean(x^2) + 1e-8)
            for (uint32_t b = wv; b < nb; b += 4) {
                float q = 0.0f;
                for (uint32_t k = lane; k < a.K; k += 64) q = __fmaf_rn(xs[b * a.K + k], xs[b * a.K + k], q);
#pragma unroll
                for (int m = 32; m >= 1; m >>= 1) q += __shfl_xor(q, m);
                if (lane == 0) nrm[b] = rsqrtf(__fadd_rn(__fdiv_rn(q, (float)a.K), 1e-8f));
            }
            __syncthreads();
            for (uint32_t i = t; i < nb * a.K; i += 256) xs[i] = __fmul_rn(xs[i], nrm[i / a.K]);
            __syncthreads();
        }
        float acc[kMapB];
#pragma unroll
        for (uint32_t b = 0; b < kMapB; ++b) acc[b] = 0.0f;
        if (o < a.O) {
#pragma unroll
            for (uint32_t kq = 0; kq < kMapMaxK / 256; ++kq) {
                const uint32_t k = 4 * kq;
                if (k >= kl) break;
                const float4 w4 = wpre[kq];
                const float wq[4] = {__fmul_rn(w4.x, a.wscale), __fmul_rn(w4.y, a.wscale),
                                     __fmul_rn(w4.z, a.wscale), __fmul_rn(w4.w, a.wscale)};
#pragma unroll
                for (uint32_t b = 0; b < kMapB; ++b) {
                    if (b < nb) {
                        const float4 x4 = *reinterpret_cast<const float4 *>(&xs[b * a.K + k0 + k]);
                        acc[b] = __fmaf_rn(x4.x, wq[0], acc[b]);
                        acc[b] = __fmaf_rn(x4.y, wq[1], acc[b]);
                        acc[b] = __fmaf_rn(x4.z, wq[2], acc[b]);
                        acc[b] = __fmaf_rn(x4.w, wq[3], acc[b]);
                    }
                }
            }
        }
#pragma unroll
        for (uint32_t b = 0; b < kMapB; ++b) {
            if (b < nb) {
#pragma unroll
                for (int m = 32; m >= 1; m >>= 1) acc[b] = __fadd_rn(acc[b], __shfl_xor(acc[b], m));
            }
        }
        if (o < a.O && lane < nb) {              // lane b stores sample b
            float y = 0.0f;
#pragma unroll
            for (uint32_t b = 0; b < kMapB; ++b)
                if (b == lane) y = acc[b];
            if (a.b) y = __fadd_rn(y, __fmul_rn(a.b[o], a.bscale));
            if (a.act) y = __fmul_rn(y > 0.0f ? y : __fmul_rn(y, a.slope), a.act_scale);
            a.out[(size_t)(b0 + lane) * a.O + o] = y;
        }
        __syncthreads();
    }
}

// ----------------------------------------------------------------------------
// Decoder style prep for inference (sdf_model.py:676-699): every layer's
// modulation s_k = latent[:, idx_k] . (W_k scale)^T + b_k lr_mul (conv and ToRGB
// EqualLinears) and every split-fp16 layer's demodulation / su,
// rsqrt(eps + s^2 . wsq) -- two launches instead of the batched GEMMs, gathers,
// copies and rsqrt of the module code.  Same structure as mapping_linear_kernel:
// a wave per output channel, lanes over the reduction, butterfly sum.
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void style_mod_kernel(const sdfr_style_args a) {
    __shared__ __attribute__((aligned(16))) float xs[kMapB * kMapMaxK];
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    const uint32_t k = blockIdx.y, c = blockIdx.x * kMapOut + wv;
    const uint32_t ck = a.mod_c[k], K = a.K, kl = K / 64, k0 = lane * kl;
    for (uint32_t b0 = blockIdx.z * kMapB; b0 < a.B; b0 += gridDim.z * kMapB) {
        const uint32_t nb = min(kMapB, a.B - b0);
        if ((reinterpret_cast<uintptr_t>(a.latent) & 15u) == 0) {
            // 16-B loads, several in flight per thread (see mapping_linear_kernel)
            const uint32_t K4 = K / 4;
#pragma unroll 8
            for (uint32_t i = t; i < nb * K4; i += 256) {
                const uint32_t b = i / K4, j = i - b * K4;
                reinterpret_cast<float4 *>(xs)[i] = *reinterpret_cast<const float4 *>(
                    a.latent + ((size_t)(b0 + b) * a.n_latent + a.mod_index[k]) * K + 4 * j);
            }
        } else {
            for (uint32_t i = t; i < nb * K; i += 256) {
                const uint32_t b = i / K, j = i - b * K;
                xs[i] = a.latent[((size_t)(b0 + b) * a.n_latent + a.mod_index[k]) * K + j];
            }
        }
        __syncthreads();
        float acc[kMapB];
#pragma unroll
        for (uint32_t b = 0; b < kMapB; ++b) acc[b] = 0.0f;
        if (c < ck) {
            const float *wr = a.mod_w + ((size_t)k * a.cmax + c) * K + k0;
            for (uint32_t j = 0; j < kl; j += 4) {
                const float4 w4 = *reinterpret_cast<const float4 *>(wr + j);
#pragma unroll
                for (uint32_t b = 0; b < kMapB; ++b) {
                    if (b < nb) {
                        const float4 x4 = *reinterpret_cast<const float4 *>(&xs[b * K + k0 + j]);
                        acc[b] = __fmaf_rn(x4.x, w4.x, acc[b]);
                        acc[b] = __fmaf_rn(x4.y, w4.y, acc[b]);
                        acc[b] = __fmaf_rn(x4.z, w4.z, acc[b]);
                        acc[b] = __fmaf_rn(x4.w, w4.w, acc[b]);
                    }
                }
            }
        }
#pragma unroll
        for (uint32_t b = 0; b < kMapB; ++b)
            if (b < nb)
#pragma unroll
                for (int m = 32; m >= 1; m >>= 1) acc[b] = __fadd_rn(acc[b], __shfl_xor(acc[b], m));
        if (c < ck && lane < nb) {
            float y = 0.0f;
#pragma unroll
            for (uint32_t b = 0; b < kMapB; ++b)
                if (b == lane) y = acc[b];
            a.mods[a.mod_off[k] + (size_t)(b0 + lane) * ck + c] =
                __fadd_rn(y, a.mod_b[(size_t)k * a.cmax + c]);
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void style_demod_kernel(const sdfr_style_args a) {
    __shared__ __attribute__((aligned(16))) float xs[kMapB * kMapMaxK];
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    const uint32_t j = blockIdx.y, o = blockIdx.x * kMapOut + wv;
    const uint32_t layer = a.dem_layer[j], cin = a.mod_c[layer], oj = a.dem_c[j];
    const uint32_t C = a.cmax, kl = C / 64, k0 = lane * kl;
    const float *mk = a.mods + a.mod_off[layer];
    for (uint32_t b0 = blockIdx.z * kMapB; b0 < a.B; b0 += gridDim.z * kMapB) {
        const uint32_t nb = min(kMapB, a.B - b0);
        if ((reinterpret_cast<uintptr_t>(mk) & 15u) == 0 && cin % 4 == 0) {
            const uint32_t C4 = C / 4;
#pragma unroll 8
            for (uint32_t i = t; i < nb * C4; i += 256) {
                const uint32_t b = i / C4, c4 = i - b * C4;
                float4 m = make_float4(0.f, 0.f, 0.f, 0.f);
                if (4 * c4 < cin) m = *reinterpret_cast<const float4 *>(mk + (size_t)(b0 + b) * cin + 4 * c4);
                reinterpret_cast<float4 *>(xs)[i] =
                    make_float4(__fmul_rn(m.x, m.x), __fmul_rn(m.y, m.y), __fmul_rn(m.z, m.z), __fmul_rn(m.w, m.w));
            }
        } else {
            for (uint32_t i = t; i < nb * C; i += 256) {
                const uint32_t b = i / C, cc = i - b * C;
                const float m = cc < cin ? mk[(size_t)(b0 + b) * cin + cc] : 0.0f;
                xs[i] = __fmul_rn(m, m);
            }
        }
        __syncthreads();
        float acc[kMapB];
#pragma unroll
        for (uint32_t b = 0; b < kMapB; ++b) acc[b] = 0.0f;
        if (o < oj) {
            const float *wr = a.dem_w + ((size_t)j * a.omax + o) * C + k0;
            for (uint32_t q = 0; q < kl; q += 4) {
                const float4 w4 = *reinterpret_cast<const float4 *>(wr + q);
#pragma unroll
                for (uint32_t b = 0; b < kMapB; ++b) {
                    if (b < nb) {
                        const float4 x4 = *reinterpret_cast<const float4 *>(&xs[b * C + k0 + q]);
                        acc[b] = __fmaf_rn(x4.x, w4.x, acc[b]);
                        acc[b] = __fmaf_rn(x4.y, w4.y, acc[b]);
                        acc[b] = __fmaf_rn(x4.z, w4.z, acc[b]);
                        acc[b] = __fmaf_rn(x4.w, w4.w, acc[b]);
                    }
                }
            }
        }
#pragma unroll
        for (uint32_t b = 0; b < kMapB; ++b)
            if (b < nb)
#pragma unroll
                for (int m = 32; m >= 1; m >>= 1) acc[b] = __fadd_rn(acc[b], __shfl_xor(acc[b], m));
        if (o < oj && lane < nb) {
            float y = 0.0f;
#pragma unroll
            for (uint32_t b = 0; b < kMapB; ++b)
                if (b == lane) y = acc[b];
            a.demods[a.dem_off[j] + (size_t)(b0 + lane) * oj + o] =
                rsqrtf(__fadd_rn(a.dem_eps[(size_t)j * a.omax + o], y));
        }
        __syncthreads();
    }
}

int sdfr_decoder_styles(const sdfr_style_args *p, void *stream) {
    if (!p) return fail(SDFR_EINVAL, "decoder_styles: null args");
    const sdfr_style_args &a = *p;
    if (a.B == 0) return SDFR_OK;
    if (a.L == 0 || a.L > 16 || a.J > 16)
        return fail(SDFR_EINVAL, "decoder_styles: 1 <= L <= 16 and J <= 16 layers");
    if (a.K % 256 != 0 || a.K > kMapMaxK || a.cmax % 256 != 0 || a.cmax > kMapMaxK)
        return fail(SDFR_EINVAL, "decoder_styles: style dim and widest layer must be 256 or 512");
    if (!a.latent || !a.mod_w || !a.mod_b || !a.mods || (a.J && (!a.dem_w || !a.dem_eps || !a.demods)))
        return fail(SDFR_EINVAL, "decoder_styles: null tensor pointer");
    for (uint32_t k = 0; k < a.L; ++k)
        if (a.mod_c[k] > a.cmax || a.mod_index[k] >= a.n_latent)
            return fail(SDFR_EINVAL, "decoder_styles: layer width / latent index out of range");
    for (uint32_t j = 0; j < a.J; ++j)
        if (a.dem_layer[j] >= a.L || a.dem_c[j] > a.omax)
            return fail(SDFR_EINVAL, "decoder_styles: demodulation layer out of range");
    hipStream_t st = (hipStream_t)stream;
    const uint32_t bz = std::min<uint32_t>((a.B + kMapB - 1) / kMapB, 64);
    style_mod_kernel<<<dim3(a.cmax / kMapOut, a.L, bz), 256, 0, st>>>(a);
    int rc = check_launch("decoder_styles: modulations");
    if (rc || a.J == 0) return rc;
    style_demod_kernel<<<dim3((a.omax + kMapOut - 1) / kMapOut, a.J, bz), 256, 0, st>>>(a);
    return check_launch("decoder_styles: demodulations");
}

int sdfr_mapping_linear(float *out, const float *x, const float *w, const float *b, uint32_t B,
                        uint32_t K, uint32_t O, float wscale, float bscale, int act, float slope,
                        float act_scale, int pixelnorm, void *stream) {
    if (B == 0) return SDFR_OK;
    if (!out || !x || !w) return fail(SDFR_EINVAL, "mapping_linear: null tensor pointer");
    if (K == 0 || K % 256 != 0 || K > kMapMaxK || O == 0)
        return fail(SDFR_EINVAL, "mapping_linear: K must be 256 or 512");
    if ((reinterpret_cast<uintptr_t>(w) & 15u) != 0)
        return fail(SDFR_EINVAL, "mapping_linear: W must be 16-byte aligned");
    MapArgs a{x, w, b, out, B, K, O, wscale, bscale, slope, act_scale, act, pixelnorm};
    const dim3 grid((O + kMapOut - 1) / kMapOut, std::min<uint32_t>((B + kMapB - 1) / kMapB, 64));
    mapping_linear_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(a);
    return check_launch("mapping_linear");
}

int sdfr_fused_bias_act(float *out, const float *x, const float *bias, const float *ref,
                        uint64_t size_x, uint32_t step_b, uint32_t size_b, int act, int grad,
                        float alpha, float scale, void *stream) {
    if (size_x == 0) return SDFR_OK;
    if (!out || !x) return fail(SDFR_EINVAL, "fused_bias_act: null tensor pointer");
    if (bias && (size_b == 0 || step_b == 0))
        return fail(SDFR_EINVAL, "fused_bias_act: bias needs size_b > 0 and step_b > 0");
    if (act == 3 && grad == 1 && !ref)
        return fail(SDFR_EINVAL, "fused_bias_act: grad mode 1 needs the reference output");
    const int mode = act * 10 + grad;
    if (!bias) size_b = 0;
    hipStream_t st = (hipStream_t)stream;
    const bool vec = size_x % 4 == 0 && (!bias || step_b % 4 == 0) && aligned16(out) &&
                     aligned16(x) && (!ref || aligned16(ref));
    if (vec) {
        const uint64_t n4 = size_x / 4;
        fused_bias_act_vec_kernel<<<grid_for(n4), 256, 0, st>>>(
            reinterpret_cast<float4 *>(out), reinterpret_cast<const float4 *>(x), bias,
            reinterpret_cast<const float4 *>(ref), n4, bias ? step_b / 4 : 1, size_b, mode, alpha,
            scale);
    } else {
        fused_bias_act_kernel<<<grid_for(size_x), 256, 0, st>>>(out, x, bias, ref, size_x,
                                                                 bias ? step_b : 1, size_b, mode,
                                                                 alpha, scale);
    }
    return check_launch("fused_bias_act");
}

int sdfr_upfirdn2d(float *out, const float *input, const float *kernel, uint32_t major,
                   uint32_t in_h, uint32_t in_w, uint32_t kernel_h, uint32_t kernel_w, int up_x,
                   int up_y, int down_x, int down_y, int pad_x0, int pad_x1, int pad_y0,
                   int pad_y1, void *stream) {
    if (up_x < 1 || up_y < 1 || down_x < 1 || down_y < 1)
        return fail(SDFR_EINVAL, "upfirdn2d: up and down factors must be >= 1");
    if (kernel_h == 0 || kernel_w == 0) return fail(SDFR_EINVAL, "upfirdn2d: empty kernel");
    const long oh = ((long)in_h * up_y + pad_y0 + pad_y1 - (long)kernel_h) / down_y + 1;
    const long ow = ((long)in_w * up_x + pad_x0 + pad_x1 - (long)kernel_w) / down_x + 1;
    if (oh <= 0 || ow <= 0) return fail(SDFR_EINVAL, "upfirdn2d: output size is not positive");
    if (major == 0 || in_h == 0 || in_w == 0) return SDFR_OK;
    if (!out || !input || !kernel) return fail(SDFR_EINVAL, "upfirdn2d: null tensor pointer");
    UfdArgs a{out, input, kernel, major, in_h, in_w, kernel_h, kernel_w, (uint32_t)oh,
              (uint32_t)ow, up_x, up_y, down_x, down_y, pad_x0, pad_y0};
    hipStream_t st = (hipStream_t)stream;
    // tiled form: 4x4 filter, the same factor on both axes, every size within int range
    // and the grid within 2^31 workgroups (64 x 16..32 outputs each)
    const bool tile = kernel_h == 4 && kernel_w == 4 && up_x == up_y && down_x == down_y &&
                      ((up_x == 1 && down_x == 1) || (up_x == 2 && down_x == 1) ||
                       (up_x == 1 && down_x == 2)) &&
                      in_h < (1u << 28) && in_w < (1u << 28) && oh < (1L << 28) && ow < (1L << 28) &&
                      (uint64_t)major * ((ow + 63) / 64) * ((oh + 15) / 16) < (1ull << 31) &&
                      std::abs(pad_x0) < (1 << 20) && std::abs(pad_y0) < (1 << 20);
    if (tile) {
        if (up_x == 2) launch_ufd_tile<2, 1>(a, st);
        else if (down_x == 2) launch_ufd_tile<1, 2>(a, st);
        else launch_ufd_tile<1, 1>(a, st);
    } else {
        upfirdn2d_kernel<<<grid_for((uint64_t)major * oh * ow), 256, 0, st>>>(a);
    }
    return check_launch("upfirdn2d");
}

int sdfr_styled_epilogue(const sdfr_styled_epilogue_args *p, void *stream) {
    if (!p) return fail(SDFR_EINVAL, "styled_epilogue: null args");
    const sdfr_styled_epilogue_args &s = *p;
    if (s.B == 0 || s.H == 0 || s.W == 0) return SDFR_OK;
    if (s.C == 0 || s.C % 4) return fail(SDFR_EINVAL, "styled_epilogue: C must be a multiple of 4");
    if (!s.conv || !s.bias || (s.noise && !s.noise_weight))
        return fail(SDFR_EINVAL, "styled_epilogue: null tensor pointer");
    const bool rgb = s.rgb_w != nullptr;
    if (rgb && (!s.rgb || !s.rgb_b)) return fail(SDFR_EINVAL, "styled_epilogue: rgb output missing");
    if (rgb && s.blur_up) return fail(SDFR_EINVAL, "styled_epilogue: ToRGB after a blur is not fused");
    if (!rgb && !s.y && !s.y_split) return fail(SDFR_EINVAL, "styled_epilogue: nothing to write");
    if (s.y && s.y_split) return fail(SDFR_EINVAL, "styled_epilogue: y and y_split are exclusive");
    if (s.y_split && s.C % 8) return fail(SDFR_EINVAL, "styled_epilogue: y_split needs C % 8 == 0");
    if (s.skip && (s.H % 2 || s.W % 2)) return fail(SDFR_EINVAL, "styled_epilogue: odd size with skip");
    for (const void *q : {(const void *)s.conv, (const void *)s.demod, (const void *)s.bias,
                          (const void *)s.s_next, (const void *)s.y, (const void *)s.rgb_w,
                          (const void *)s.y_split})
        if (q && !aligned16(q)) return fail(SDFR_EINVAL, "styled_epilogue: pointers must be 16-B aligned");
    EpiArgs a{s.B, s.C, s.H, s.W, s.conv, {s.fir[0], s.fir[1], s.fir[2], s.fir[3]},
              s.demod, s.noise, s.noise_weight, s.bias, s.negative_slope, s.act_scale,
              s.s_next, s.y, s.rgb_w, s.rgb_b, s.skip, s.rgb,
              reinterpret_cast<_Float16 *>(s.y_split)};
    hipStream_t st = (hipStream_t)stream;
    if (s.blur_up) {
        // row segments of kBlurRows (3 extra input rows each), halved while the grid
        // would leave CUs idle (eval.py's batch of 1: 64-128 blocks at 16 rows)
        uint32_t rps = kBlurRows, nseg = 0;
        uint64_t total = 0;
        for (;;) {
            nseg = (s.H + rps - 1) / rps;
            total = (uint64_t)s.B * nseg * ((s.W + kBlurCols - 1) / kBlurCols) * (s.C / 4);
            if (total >= 1024ull * 256 || rps <= (uint32_t)kBlurGroup) break;
            rps /= 2;
        }
        if (total >= (1ull << 31)) return fail(SDFR_EINVAL, "styled_epilogue(blur): too large");
        const uint32_t nb = (uint32_t)((total + 255) / 256);
        epi_blur_kernel<<<BLUR_XCD ? (nb + 7) & ~7u : nb, 256, 0, st>>>(a, nseg, rps);
        return check_launch("styled_epilogue(blur)");
    }
    const uint32_t Q = s.C / 4;
    const bool pow2 = (Q & (Q - 1)) == 0;
    if (Q <= 64 ? !pow2 : (Q % 64 != 0))
        return fail(SDFR_EUNSUPPORTED,
                    "styled_epilogue: C/4 must be a power of two <= 64 or a multiple of 64");
    // TPP lanes per pixel, NQ = Q / TPP float4 each: a 16-lane ToRGB reduction up to
    // C = 256 (NQ <= 4), whole waves above
    uint32_t tpp_log2 = 0, nq = 1;
    if (Q <= 16) {
        while ((1u << tpp_log2) < Q) ++tpp_log2;
    } else if (Q <= 64) {
        tpp_log2 = 4;
        nq = Q / 16;
    } else {
        tpp_log2 = 6;
        nq = Q / 64;
    }
    dim3 grid((s.H * s.W + kEpiPixPerBlock - 1) / kEpiPixPerBlock, s.B);
#define EPI(NQ)                                                                          \
    case NQ:                                                                             \
        if (rgb) epi_plain_kernel<NQ, true><<<grid, 256, 0, st>>>(a, tpp_log2);          \
        else epi_plain_kernel<NQ, false><<<grid, 256, 0, st>>>(a, tpp_log2);             \
        break;
    switch (nq) {
        EPI(1)
        EPI(2)
        EPI(3)
        EPI(4)
        EPI(8)
        default: return fail(SDFR_EUNSUPPORTED, "styled_epilogue: C > 1024");
    }
#undef EPI
    return check_launch("styled_epilogue");
}

static int modulate_common(float *y, void *ys, const float *x, const float *s, uint32_t B,
                           uint32_t C, uint32_t HW, void *stream) {
    if (B == 0 || C == 0 || HW == 0) return SDFR_OK;
    if ((!y && !ys) || !x || !s) return fail(SDFR_EINVAL, "modulate_to_nhwc: null tensor pointer");
    if (C % 4 || HW % 4) return fail(SDFR_EINVAL, "modulate_to_nhwc: C and H*W must be multiples of 4");
    if (ys && C % 8) return fail(SDFR_EINVAL, "modulate_to_nhwc_split: C must be a multiple of 8");
    if (!aligned16(x) || (y && !aligned16(y)) || (ys && !aligned16(ys)))
        return fail(SDFR_EINVAL, "modulate_to_nhwc: pointers must be 16-B aligned");
    dim3 grid((HW + 63) / 64, (C + 63) / 64, B);
    modulate_nhwc_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(
        y, reinterpret_cast<_Float16 *>(ys), x, s, C, HW);
    return check_launch("modulate_to_nhwc");
}

int sdfr_rgb_finish(float *rgb, const float *partial, uint32_t nparts, const float *rgb_b,
                    const float *skip, const float *fir, uint32_t B, uint32_t H, uint32_t W,
                    void *stream) {
    if (B == 0 || H == 0 || W == 0) return SDFR_OK;
    if (!rgb || !partial || !rgb_b || nparts == 0 || (skip && !fir))
        return fail(SDFR_EINVAL, "rgb_finish: null pointer");
    if (skip && (H % 2 || W % 2)) return fail(SDFR_EINVAL, "rgb_finish: odd size with skip");
    const uint64_t n = (uint64_t)B * 3 * H * W;
    const float f[4] = {skip ? fir[0] : 0.f, skip ? fir[1] : 0.f, skip ? fir[2] : 0.f,
                        skip ? fir[3] : 0.f};
    if (B * 3 > 65535 || (uint64_t)H * W >= (1ull << 31)) return fail(SDFR_EINVAL, "rgb_finish: too large");
    if (W % 4) return fail(SDFR_EINVAL, "rgb_finish: W must be a multiple of 4");
    (void)n;
    rgb_finish_kernel<<<dim3((W / 4 + 63) / 64, (H + 3) / 4, B * 3), 256, 0, (hipStream_t)stream>>>(
        rgb, partial, nparts, rgb_b, skip, f[0], f[1], f[2], f[3], B, H, W);
    return check_launch("rgb_finish");
}

int sdfr_modulate_to_nhwc(float *y, const float *x, const float *s, uint32_t B, uint32_t C,
                          uint32_t HW, void *stream) {
    if (!y && B && C && HW) return fail(SDFR_EINVAL, "modulate_to_nhwc: null tensor pointer");
    return modulate_common(y, nullptr, x, s, B, C, HW, stream);
}

int sdfr_modulate_to_nhwc_split(void *y_split, const float *x, const float *s, uint32_t B,
                                uint32_t C, uint32_t HW, void *stream) {
    if (!y_split && B && C && HW)
        return fail(SDFR_EINVAL, "modulate_to_nhwc_split: null tensor pointer");
    return modulate_common(nullptr, y_split, x, s, B, C, HW, stream);
}

}  // extern "C"
