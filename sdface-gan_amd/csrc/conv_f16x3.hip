// conv_f16x3.hip -- the StyleGAN2 decoder's 3x3 convolutions on split-fp16 MFMA.
//
// Replaces the two convolution forms of ModulatedConv2d on the fused decoder
// path (sdf_model.py:676-699, applied as conv(x * s, w) * demod -- the batched
// form of the reference's per-face modulated weights, see generator.py):
//   regular     out[b,y,x,o]   = sum_{i,ky,kx} x[b,y+ky-1,x+kx-1,i] w[o,i,ky,kx]   (pad 1)
//   transposed  out[b,2a+ky,2c+kx,o] += x[b,a,c,i] w[o,i,ky,kx]   (conv_transpose2d,
//               stride 2, output (2H+1) x (2W+1), before the upsampling blur)
// as implicit GEMMs over NHWC activations: M = output channels (A = weights),
// N = output pixels (B = activations), K = input channels x taps.  Every fp32
// tile product is W_hi.x_hi + W_hi.x_lo + W_lo.x_hi on v_mfma_f32_16x16x32_f16
// with fp32 accumulation (the field kernel's scheme):
// 5.3x the fp32 MFMA rate at fp32-level accuracy.  Weights are row-scaled by a
// power of two su[o] so their fp16 lo parts stay normal; the caller folds 1/su
// into the demodulation (exact).  A transposed conv is four implicit GEMMs, one
// per output parity class (oy & 1, ox & 1), each over its own tap subset.
//
// Workgroup: 128 output channels x 256 output pixels, 8 waves of 64 x 64 (two per
// SIMD), K in steps of 32 input channels at one tap.  Both operands arrive
// already split (weights pre-packed in fragment order; activations in the
// split-NHWC layout the previous epilogue writes, 32 channels of a pixel's hi and
// lo = one 128-B line) and are staged global -> LDS by LDS-DMA (buffer_load ...
// lds: no VGPRs, no VALU; the buffer range check zero-fills the padding taps)
// through a 3-stage ring of 48 KB stages: two K-steps stay in flight behind a
// counted vmcnt and a raw barrier, one workgroup per CU.  The workgroup order is
// XCD-aware, and the four parity classes of a transposed conv share one launch.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "sdfr_common.h"

namespace sdfr {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));

constexpr int kCT = 128;        // output channels per workgroup
constexpr int kPT = 256;        // output pixels per workgroup
constexpr int kStepF4 = 1024;   // f4 of weight fragments per K-step (16 KB)
constexpr int kStages = 3;   // LDS-DMA ring depth (kStages - 1 K-steps in flight)
constexpr uint32_t kCusPerXcd = 32;   // MI355X: 256 CUs in 8 XCDs (persistent grids)
// profiling-only ablations of conv_x_kernel (wrong results by construction): 1 = the
// raw-output epilogue stores only when a (never occurring) sentinel matches; 16 + c =
// only parity class c runs (the other classes' workgroups exit at once)
#ifndef SDFR_CABL
#define SDFR_CABL 0
#endif
constexpr int kCAbl = SDFR_CABL;
// conv_t_kernel ablations (profiling only): 1 no output stores (sentinel), 2 no barrier,
// 4 no weight DMA after the prologue, 8 no halo DMA after the prologue
#ifndef SDFR_TABL
#define SDFR_TABL 0
#endif
constexpr int kTAbl = SDFR_TABL;
// conv_h_kernel ablations (profiling only): 1 y stores only on a sentinel, 2 no epilogue
// (the accumulators stored on a sentinel), 4 no ToRGB partials
#ifndef SDFR_HABL
#define SDFR_HABL 0
#endif
constexpr int kHAbl = SDFR_HABL;
// conv_h_kernel's epilogue activation and ToRGB partials on packed fp32 (0: scalar)
#ifndef SDFR_HEPK
#define SDFR_HEPK 1
#endif
constexpr bool kHEpk = SDFR_HEPK != 0;
typedef float f2c __attribute__((ext_vector_type(2)));
// small batches: K-split conv_h_kernel + conv_h_finish_kernel (0: conv_x_kernel split-K)
#ifndef SDFR_HSPLIT
#define SDFR_HSPLIT 1
#endif
constexpr bool kHSplit = SDFR_HSPLIT != 0;


__device__ __forceinline__ f4 mfma16(f4 a, f4 b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a),
                                                  __builtin_bit_cast(h8, b), c, 0, 0, 0);
}

// ----------------------------------------------------------------------------
// weight packing: w [Cout][Cin][3][3] * scale -> su [Cout], fragments
// [tap 9][Cin/32][Cout/128][8 m-tiles][hi, lo][64 lanes] fp16x8, lane (m, g)
// holding w[o = 16 mt + m][i = 32 c + 8 g + j][tap], j = 0..7
// ----------------------------------------------------------------------------
__global__ void __launch_bounds__(256) conv_scale_kernel(const float *__restrict__ w, float scale,
                                                         uint32_t Cin, float *__restrict__ su) {
    const uint32_t o = blockIdx.x;
    float m = 0.0f;
    for (uint32_t k = threadIdx.x; k < Cin * 9; k += 256)
        m = fmaxf(m, fabsf(__fmul_rn(w[(size_t)o * Cin * 9 + k], scale)));
    __shared__ float red[256];
    red[threadIdx.x] = m;
    __syncthreads();
    for (uint32_t s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        float v = 1.0f;
        const float mx = red[0];
        if (mx > 0.0f && mx < 3.0e38f) {
            int ex;
            (void)frexpf(mx, &ex);
            ex = ex < -100 ? -100 : (ex > 100 ? 100 : ex);
            v = ldexpf(1.0f, -ex);
        }
        su[o] = v;
    }
}

__global__ void __launch_bounds__(256) conv_pack_kernel(const float *__restrict__ w, float scale,
                                                        uint32_t Cin, uint32_t Cout,
                                                        const float *__restrict__ su,
                                                        f4 *__restrict__ packed) {
    const uint32_t e = blockIdx.x * 256 + threadIdx.x;        // one (tap, c, cb, mt, lane)
    const uint32_t nC = Cin / 32, nB = Cout / kCT;
    const uint32_t total = 9 * nC * nB * 8 * 64;
    if (e >= total) return;
    const uint32_t lane = e & 63, mt = (e >> 6) & 7;
    uint32_t r = e >> 9;
    const uint32_t cb = r % nB;
    r /= nB;
    const uint32_t c = r % nC, tap = r / nC;
    const uint32_t o = cb * kCT + mt * 16 + (lane & 15), g = lane >> 4;
    const float s = su[o];
    h8 H, L;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t i = c * 32 + 8 * g + j;
        const float v = __fmul_rn(__fmul_rn(w[((size_t)o * Cin + i) * 9 + tap], scale), s);
        H[j] = (_Float16)v;
        L[j] = (_Float16)__fsub_rn(v, (float)H[j]);
    }
    f4 *dst = packed + ((size_t)(e >> 6) * 2) * 64 + lane;   // [.. mt][hi,lo][lane]
    dst[0] = __builtin_bit_cast(f4, H);
    dst[64] = __builtin_bit_cast(f4, L);
}

// ----------------------------------------------------------------------------
// implicit GEMM
// ----------------------------------------------------------------------------

// One output-pixel class: the plain convolution has one (every pixel, 9 taps); the
// stride-2 transposed one has four parity classes (4, 2, 2 and 1 taps) that share
// one launch, heaviest first, so their tails overlap.
struct ConvClass {
    uint32_t Hc, Wc;               // the class's output grid
    uint32_t py, px;               // output pixel (a, c) -> (sy (a + a0) + py, sy (c + c0) + px)
    uint32_t a0, c0;               // grid origin (0; conv_t_kernel's edge rows / columns)
    uint32_t ntaps, t0;            // its taps: dy/dx/tap[t0 .. t0 + ntaps)
    uint32_t tile0, ntiles;        // workgroups [tile0, tile0 + pad8(ntiles)) of the grid
    uint32_t td[3];                // tap descriptors, 8 bits per tap (tap | dy+1 << 4 | dx+1 << 6)
};

// Styled epilogue fused into a regular conv (sdfr_conv3x3_f16x3_act).
struct ActEpi {
    const float *demod, *noise, *noise_weight, *bias;   // [B,Cout], [B,H,W], [1], [Cout]
    float slope, scale;
    const float *s_next;           // [B,Cout] or null
    _Float16 *ys;                  // split-NHWC [B,H,W,Cout] or null
    const float *rgb_w;            // [B,3,Cout] or null
    float *rgbp;                   // [Cout/128, B, 3, H*W] ToRGB partial sums
    // or (rgb_w null) the ToRGB weight as base [3,Cout] x style [B,Cout], multiplied
    // here (the same fp32 product the caller would form: one launch less per layer)
    const float *rgb_base, *rgb_s;
};

struct ConvArgs {
    const _Float16 *xs;            // split-NHWC [B, Hin, Win, Cin/8, 2, 8]
    const f4 *wpk;                 // packed fragments (above)
    float *out;                    // [B, Hf, Wf, Cout]
    uint32_t B, Hin, Win, Cin, Cout;
    uint32_t Hf, Wf, sy;           // full output image, class stride
    uint32_t ncls;
    ConvClass cls[4];
    int dy[9], dx[9];              // input pixel = (a + dy, c + dx)
    uint32_t tap[9];               // packed weight tap (3 ky + kx)
    ActEpi e;                      // conv_x_kernel<true> only
    uint32_t ksplit;               // split-K factor (1: the epilogue runs in the conv kernel)
    uint32_t grid;                 // workgroup slots per split (padded class tiles)
    f4 *partial;                   // [ksplit][grid][16 (i, j)][512 threads] f4 when ksplit > 1
    uint32_t tiles_t;              // conv_t_kernel: 64-channel x 16 x 16-position tiles
    uint32_t ksplit_t;             // conv_t_kernel: channel-group split of a tile (1, 2, 4)
    float *ptl;                    // ksplit_t > 1: [ksplit_t][B, Hf, Wf, Cout] partial outputs
    float fir[4];                  // conv_t_kernel<true>: the blur's 1-D taps (outer(fir, fir))
};

typedef int v4i __attribute__((ext_vector_type(4)));

// Buffer resource over [base, base + bytes) (gfx950 raw buffer, range-checked).
__device__ __forceinline__ v4i make_rsrc(const void *base, uint32_t bytes) {
    const uint64_t b = reinterpret_cast<uint64_t>(base);
    v4i r;
    r.x = (int)(uint32_t)b;
    r.y = (int)(uint32_t)(b >> 32);
    r.z = (int)bytes;
    r.w = 0x00020000;
    return r;
}

// One LDS-DMA piece: 64 lanes x 16 B from rsrc at (voff + soff) to LDS byte
// address lds (wave-uniform base + 16 lane).  Inline asm, so hipcc neither
// tracks it in its own s_waitcnt bookkeeping (no vmcnt(0) drain in front of
// every ds_read of the ring) nor reserves M0 across it; completion is counted
// explicitly by the ring below.  Offsets past num_records read zeros.
// M0 = LDS destination base of the following DMAs (kernel code here never uses M0
// otherwise -- checked in the ISA; the register is reserved, so it cannot be
// declared clobbered).  A DMA's instruction offset moves both its global address
// and its LDS destination, so one M0 write serves several pieces.
__device__ __forceinline__ void set_m0(uint32_t lds) {
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0" : : "s"(lds) : "memory");
}
template <int IOFF>
__device__ __forceinline__ void dma16(v4i rsrc, uint32_t voff, uint32_t soff) {
    asm volatile("buffer_load_dwordx4 %0, %1, %2 offen offset:%3 lds"
                 :
                 : "v"(voff), "s"(rsrc), "s"(soff), "i"(IOFF)
                 : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)reinterpret_cast<uintptr_t>(p);
}

__device__ __forceinline__ float act1(float c, float dm, float nz, float b, float slope,
                                      float scale) {
    float v = c * dm;                  // same operation order as decoder.hip's epilogue
    v = v + nz;
    v = v + b;
    v = v > 0.0f ? v : v * slope;
    return v * scale;
}

// Round-to-nearest hi/lo split into split-NHWC (decoder.hip store_split4) for lane
// groups g = 2k, 2k+1 holding channels 4g..4g+3 of the same 8-channel group and
// pixel (lanes 16 g + n): one v_permlane16_swap per dword
// gives the even group both hi halves and the odd group both lo halves, so every
// lane issues ONE 16-B store (hi of the 8 channels at idx8, lo 16 B after it) instead
// of two 8-B stores.  idx8 = NHWC element index of the group's channel 0.  All lanes
// must execute it (cross-lane).
__device__ __forceinline__ void store_split8_pair(_Float16 *ys, size_t idx8, f4 v, uint32_t g) {
    h4 h, l;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        h[r] = (_Float16)v[r];
        l[r] = (_Float16)(v[r] - (float)h[r]);
    }
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    const u2 hd = __builtin_bit_cast(u2, h), ld = __builtin_bit_cast(u2, l);
    uint32_t q[4];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const auto r = __builtin_amdgcn_permlane16_swap(hd[k], ld[k], false, false);
        q[k] = r[0];          // even group: own hi / odd group: partner's lo
        q[2 + k] = r[1];      // even group: partner's hi / odd group: own lo
    }
    *reinterpret_cast<f4 *>(ys + 2 * idx8 + (g & 1u) * 8) = __builtin_bit_cast(f4, q);
}

// Epilogue of one workgroup tile: raw fp32 output (NHWC, class pixel placement) or,
// with ACT, the fused styled epilogue (sdfr_conv3x3_f16x3_act).
template <bool ACT>
__device__ __forceinline__ void conv_epilogue(const ConvArgs &a, f4 (&acc)[4][4], uint32_t lane,
                                              uint32_t wm, uint32_t wn, uint32_t cb, uint32_t pix0,
                                              uint32_t npix, uint32_t Hc, uint32_t Wc, uint32_t py,
                                              uint32_t px, uint32_t rs = 16, uint32_t a0 = 0,
                                              uint32_t c0 = 0) {
    // epilogue: lane (n, g) of tile (i, j) holds channels 16 mt + 4 g .. +3 of pixel 16 nt + n
    const uint32_t n = lane & 15u, g = lane >> 4;
    if constexpr (ACT) {
        // Styled epilogue on the accumulators (regular conv, H W % 256 == 0: one face
        // per workgroup): v = lrelu(acc demod + nw noise + bias) scale; y = v s_next
        // as split-NHWC; ToRGB partial over this workgroup's 128 channels -> rgbp.
        // n-tile row r = 4 wn + j holds pixels pix0 + r rs + n (rs = 16: a 256-pixel
        // strip; rs = W: a 16 x 16 block, conv_h_kernel).
        __shared__ float red[4][4][16][3];          // [wn][j][n][o] from the wm = 1 waves
        const ActEpi &e = a.e;
        const uint32_t HW = Hc * Wc, b = pix0 / HW;
        const float nw = e.noise ? *e.noise_weight : 0.0f;
        float part[4][3];
#pragma unroll
        for (int j = 0; j < 4; ++j) part[j][0] = part[j][1] = part[j][2] = 0.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t ch = cb * kCT + (4 * wm + i) * 16 + 4 * g;
            const f4 dm = *reinterpret_cast<const f4 *>(e.demod + (size_t)b * a.Cout + ch);
            const f4 bs = *reinterpret_cast<const f4 *>(e.bias + ch);
            const f4 sn = e.s_next ? *reinterpret_cast<const f4 *>(e.s_next + (size_t)b * a.Cout + ch)
                                   : f4{1.0f, 1.0f, 1.0f, 1.0f};
            f4 rw[3];
            const f4 rsty = e.rgb_base ? *reinterpret_cast<const f4 *>(e.rgb_s + (size_t)b * a.Cout + ch)
                                       : f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int o = 0; o < 3; ++o)
                rw[o] = e.rgb_w ? *reinterpret_cast<const f4 *>(e.rgb_w + ((size_t)b * 3 + o) * a.Cout + ch)
                      : e.rgb_base ? *reinterpret_cast<const f4 *>(e.rgb_base + (size_t)o * a.Cout + ch) * rsty
                                   : f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t P = pix0 + (4 * wn + j) * rs + n;
                const float nz = e.noise ? nw * e.noise[P] : 0.0f;
                f4 v;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = act1(acc[i][j][r], dm[r], nz, bs[r], e.slope, e.scale);
                if (e.ys) store_split8_pair(e.ys, (size_t)P * a.Cout + (ch & ~7u), v * sn, g);
#pragma unroll
                for (int o = 0; o < 3; ++o)
#pragma unroll
                    for (int r = 0; r < 4; ++r) part[j][o] = fmaf(v[r], rw[o][r], part[j][o]);
            }
        }
        if (e.rgb_w || e.rgb_base) {
            // sum over the 4 channel groups g (lanes n + 16 g), then over wm (LDS)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int o = 0; o < 3; ++o) {
                    part[j][o] += __shfl_xor(part[j][o], 16, 64);
                    part[j][o] += __shfl_xor(part[j][o], 32, 64);
                }
            if (wm == 1 && g == 0)
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int o = 0; o < 3; ++o) red[wn][j][n][o] = part[j][o];
            __syncthreads();
            if (wm == 0 && g < 3) {                 // lane (n, g = o) stores channel o
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t P = pix0 + (4 * wn + j) * rs + n;
                    const float s = (g == 0 ? part[j][0] : g == 1 ? part[j][1] : part[j][2]) +
                                    red[wn][j][n][g];
                    e.rgbp[(((size_t)cb * a.B + b) * 3 + g) * HW + (P - b * HW)] = s;
                }
            }
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t P = pix0 + (4 * wn + j) * 16 + n;
        if (P >= npix) continue;
        const uint32_t hw = Hc * Wc;
        const uint32_t b = P / hw, rem = P % hw;
        const uint32_t oy = a.sy * (rem / Wc + a0) + py, ox = a.sy * (rem % Wc + c0) + px;
        float *dst = a.out + (((size_t)b * a.Hf + oy) * a.Wf + ox) * a.Cout + cb * kCT + 4 * g;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if constexpr (kCAbl & 1) {
                if (acc[i][j][0] == 1.2345e-33f) *reinterpret_cast<f4 *>(dst + (4 * wm + i) * 16) = acc[i][j];
            } else {
                *reinterpret_cast<f4 *>(dst + (4 * wm + i) * 16) = acc[i][j];
            }
        }
    }
}

// Workgroup slot -> (class, tile); false for a padding slot.  Class ranges start at
// multiples of 8, so slot % 8 is the XCD.
__device__ __forceinline__ bool slot_tile(const ConvArgs &a, uint32_t slot, uint32_t &ci,
                                          uint32_t &tile) {
    ci = 0;
    for (uint32_t i = 1; i < a.ncls; ++i)
        if (slot >= a.cls[i].tile0) ci = i;
    const ConvClass &cl = a.cls[ci];
    const uint32_t loc = slot - cl.tile0;
    // XCD-aware tile order.  Workgroups are dealt round-robin to the 8 XCDs; give
    // each XCD one contiguous run of the class's tiles, with the Cout block fastest,
    // so the tiles that re-read an activation row (the other Cout blocks of the same
    // pixels, the rows above and below through the taps) run on the same XCD at
    // about the same time and hit its L2.  (The K splits of a slot, blockIdx.y, sit
    // on the same XCD: the grid's x extent is a multiple of 8.)
    tile = (loc & 7u) * ((cl.ntiles + 7) >> 3) + (loc >> 3);
    return tile < cl.ntiles;
}

template <bool ACT>
__global__ void __launch_bounds__(512, 1) conv_x_kernel(const ConvArgs a) {
    __shared__ f4 As[kStages][kStepF4];       // [mt 8][hi,lo][64]
    __shared__ f4 Bs[kStages][2 * kStepF4];   // [nt 16][hi,lo][64]
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR)
    const uint32_t wm = wave & 1u, wn = wave >> 1;
    uint32_t ci, tile;
    if (!slot_tile(a, blockIdx.x, ci, tile)) return;  // padding slot (whole workgroup)
    if constexpr (kCAbl >= 16) {
        if (ci != (uint32_t)(kCAbl - 16)) return;
    }
    const ConvClass &cl = a.cls[ci];
    const uint32_t Hc = cl.Hc, Wc = cl.Wc, py = cl.py, px = cl.px;
    const uint32_t ntaps = cl.ntaps;
    const uint32_t npix = a.B * Hc * Wc;
    const uint32_t nC = a.Cin / 32, nB = a.Cout / kCT;
    const uint32_t cb = tile % nB;
    const uint32_t pix0 = (tile / nB) * kPT;
    // split-K: blockIdx.y's share of the class's K-steps (channel group x tap)
    const uint32_t nk_all = nC * ntaps, split = blockIdx.y;
    const uint32_t k_begin = split * nk_all / a.ksplit, nk = (split + 1) * nk_all / a.ksplit - k_begin;

    // LDS-DMA sources (6 pieces of 1 KB per wave per K-step).  Weights: the K-step's
    // 16 KB block is contiguous; wave w moves pieces 2w, 2w+1.  Activations: the 32
    // channels of one pixel are one 128-B line of the split-NHWC input
    // ([g 4][hi 8, lo 8] halves); a piece is 8 pixels = 8 whole lines, region
    // (nt, half) of n-tile nt = pixels 16 nt + 8 half .. +7.  Lane l fetches pixel
    // l & 7, channel group g = (l >> 3) & 3, plane h = l >> 5 to LDS unit l, so a
    // region holds [h][g][pixel] and the fragment read below is conflict-free.
    // Wave w moves regions (2w, 0..1) and (2w+1, 0..1).
    const uint32_t xbytes = a.B * a.Hin * a.Win * a.Cin * 4;
    const v4i rw = make_rsrc(a.wpk, 9u * nC * nB * kStepF4 * 16u);
    const v4i rx = make_rsrc(a.xs, xbytes);
    const uint32_t loff = ((lane >> 3) & 3u) * 32u + (lane >> 5) * 16u;
    // per tap (8-bit descriptors, SGPRs): packed weight tap, dy, dx
    const uint32_t td0 = cl.td[0], td1 = cl.td[1], td2 = cl.td[2];
    auto tapdesc = [&](uint32_t t) -> uint32_t {
        const uint32_t w = t < 4 ? td0 : (t < 8 ? td1 : td2);
        return (w >> (8 * (t & 3u))) & 0xFFu;
    };
    // Per activation piece: the lane's own input offset (its output pixel at dy = dx
    // = 0, + channel group / plane) and a bit per tap telling whether the tap's
    // input pixel exists (zero padding otherwise): the K loop then needs one add
    // and one select per piece, all tap arithmetic being uniform (SALU).
    uint32_t xoff[4], tmask[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t P = pix0 + (2 * wave + (k >> 1)) * 16 + (k & 1) * 8 + (lane & 7u);
        const bool pv = P < npix;
        const uint32_t Pc = pv ? P : 0;
        const uint32_t hw = Hc * Wc;
        const uint32_t pb = Pc / hw, rem = Pc % hw, pa = rem / Wc + cl.a0, pc = rem % Wc + cl.c0;
        xoff[k] = ((pb * a.Hin + pa) * a.Win + pc) * a.Cin * 4u + loff;
        uint32_t m = 0;
        for (uint32_t t = 0; t < ntaps; ++t) {
            const uint32_t d = tapdesc(t);
            const int iy = (int)pa + (int)((d >> 4) & 3u) - 1, ix = (int)pc + (int)(d >> 6) - 1;
            if (pv && iy >= 0 && iy < (int)a.Hin && ix >= 0 && ix < (int)a.Win) m |= 1u << t;
        }
        tmask[k] = m;
    }

    // K-step issue order is sequential (0, 1, 2 in the prologue, then ks + 3 at
    // step ks): (channel group, tap) advance incrementally
    // The address work (SALU tap decode, VALU offsets) is done in prep_step, ahead
    // of the barrier and overlapped with MFMAs; fire_step after the barrier only
    // moves M0 and issues the six DMAs.
    uint32_t nx_c = k_begin / ntaps, nx_t = k_begin % ntaps;
    struct StepDma {
        uint32_t wsoff;           // weight pieces: global offset of this wave's first
        uint32_t offs[4];         // activation pieces: per-lane global offsets
    };
    auto prep_step = [&]() -> StepDma {
        StepDma r;
        const uint32_t c = nx_c, tl = nx_t;
        const bool wrap = nx_t + 1 == ntaps;
        nx_t = wrap ? 0u : nx_t + 1;
        nx_c = wrap ? nx_c + 1 : nx_c;
        const uint32_t d = tapdesc(tl);
        const uint32_t wbase = (((d & 15u) * nC + c) * nB + cb) * kStepF4 * 16u;
        r.wsoff = wbase + 2 * wave * 1024u;
        const int dy = (int)((d >> 4) & 3u) - 1, dx = (int)(d >> 6) - 1;
        const uint32_t toff = (uint32_t)((dy * (int)a.Win + dx) * (int)a.Cin * 4) + c * 128u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const bool ok = (tmask[k] >> tl) & 1u;
            r.offs[k] = ok ? xoff[k] + toff : 0x7FFFFFF0u;   // past num_records: zero fill
        }
        return r;
    };
    auto fire_step = [&](const StepDma &r, uint32_t buf) {
        set_m0(lds_addr(&As[buf][2 * wave * 64]));
        dma16<0>(rw, lane * 16u, r.wsoff);
        dma16<1024>(rw, lane * 16u, r.wsoff);
        // (one M0 per piece: an instruction offset would move the -- per-lane, possibly
        // small -- global offsets too)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            set_m0(lds_addr(&Bs[buf][(4 * wave + k) * 64]));
            dma16<0>(rx, r.offs[k], 0u);
        }
    };
    auto issue_step = [&](uint32_t ks, uint32_t buf) {
        (void)ks;
        fire_step(prep_step(), buf);
    };

    f4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.0f, 0.0f, 0.0f, 0.0f};

    // Fragments of one K-step: [0..3] A hi, [4..7] A lo, [8..11] B hi, [12..15] B lo.
    // B lane (g = lane >> 4, n = lane & 15): region (nt, n >> 3), unit h 32 + 8 g + (n & 7).
    const uint32_t boff = ((lane >> 3) & 1u) * 64u + (lane >> 4) * 8u + (lane & 7u);
    auto read_frags = [&](f4 (&R)[16], uint32_t st) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            R[i] = As[st][((4 * wm + i) * 2) * 64 + lane];
            R[4 + i] = As[st][((4 * wm + i) * 2 + 1) * 64 + lane];
            R[8 + i] = Bs[st][((4 * wn + i) * 2) * 64 + boff];
            R[12 + i] = Bs[st][((4 * wn + i) * 2) * 64 + boff + 32];
        }
    };
    // rows i0 .. i0+nr-1 of the wave's 4 x 4 tiles; per A fragment the three split
    // terms sweep the 4 B fragments (consecutive MFMAs never share an accumulator)
    auto mfma_rows = [&](const f4 (&R)[16], int i0, int nr) {
#pragma unroll
        for (int i = i0; i < i0 + nr; ++i) {
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(R[4 + i], R[8 + j], acc[i][j]);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(R[i], R[12 + j], acc[i][j]);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(R[i], R[8 + j], acc[i][j]);
        }
    };

    // Ring: step ks lives in stage ks % 3 and is read into registers half a step
    // early.  Half-way through step ks (rows 0-1 done) the wave waits for its pieces
    // of step ks+1 (ks+2's 6 may stay in flight), drains its LDS reads and meets the
    // others at a raw barrier: after it step ks+1 is in LDS everywhere and nobody
    // reads stage ks % 3 any more, so step ks+3 is issued into it and step ks+1's
    // fragments are read while rows 2-3 of step ks compute.
    uint32_t st_ks = 0;
    auto step = [&](uint32_t ks, const f4 (&R)[16], f4 (&Rn)[16]) {
        const bool fire = ks + kStages < nk;
        const bool more = kStages == 3 && ks + 2 < nk;
        StepDma pr = prep_step();                   // (counters advance past nk harmlessly)
        // materialise the DMA addresses here, in the MFMA shadow (the compiler would
        // otherwise sink them past the barrier into the issue block)
        asm volatile("" : "+s"(pr.wsoff));
#pragma unroll
        for (int k = 0; k < 4; ++k) asm volatile("" : "+v"(pr.offs[k]));
        mfma_rows(R, 0, 2);
        if (more) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        const uint32_t st = st_ks, st1 = st_ks == kStages - 1 ? 0u : st_ks + 1;
        st_ks = st1;                                   // ks % kStages, carried
        if (fire) fire_step(pr, st);
        if (ks + 1 < nk) read_frags(Rn, st1);
        mfma_rows(R, 2, 2);
    };
    issue_step(0, 0);
    if (nk > 1) issue_step(1, 1);
    if (kStages == 3 && nk > 2) issue_step(2, 2);
    if (kStages == 3 && nk > 2) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (nk > 1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    f4 R0[16], R1[16];
    read_frags(R0, 0);
    uint32_t ks = 0;
    for (; ks + 1 < nk; ks += 2) {
        step(ks, R0, R1);
        step(ks + 1, R1, R0);
    }
    if (ks < nk) step(ks, R0, R1);

    if (a.ksplit > 1) {      // partial sums; conv_splitk_kernel adds them and runs the epilogue
        f4 *pp = a.partial + ((size_t)split * a.grid + blockIdx.x) * 16 * 512 + tid;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) pp[(i * 4 + j) * 512] = acc[i][j];
        return;
    }
    conv_epilogue<ACT>(a, acc, lane, wm, wn, cb, pix0, npix, Hc, Wc, py, px, 16, cl.a0, cl.c0);
}

// Split-K finish: the ksplit partial tiles summed in split order (deterministic),
// then the tile's epilogue, with the conv kernel's slot -> tile mapping and lane
// roles.  Used when the unsplit grid would leave CUs idle (eval.py's batch of 1:
// 64 workgroups at 64^2, 128 at 128^2, for 256 CUs).
template <bool ACT>
__global__ void __launch_bounds__(512, 1) conv_splitk_kernel(const ConvArgs a) {
    uint32_t ci, tile;
    if (!slot_tile(a, blockIdx.x, ci, tile)) return;
    const ConvClass &cl = a.cls[ci];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t wm = wave & 1u, wn = wave >> 1;
    const uint32_t nB = a.Cout / kCT, cb = tile % nB, pix0 = (tile / nB) * kPT;
    // every split's 16 f4 loaded before the first add (all 64 loads in flight)
    f4 acc[4][4], t[3][16];
    const f4 *pp = a.partial + (size_t)blockIdx.x * 16 * 512 + tid;
    const size_t sstride = (size_t)a.grid * 16 * 512;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = pp[(i * 4 + j) * 512];
#pragma unroll
    for (uint32_t s = 1; s < 4; ++s)
        if (s < a.ksplit)
#pragma unroll
            for (int q = 0; q < 16; ++q) t[s - 1][q] = pp[s * sstride + q * 512];
#pragma unroll
    for (uint32_t s = 1; s < 4; ++s)
        if (s < a.ksplit)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] += t[s - 1][i * 4 + j];
    conv_epilogue<ACT>(a, acc, lane, wm, wn, cb, pix0, a.B * cl.Hc * cl.Wc, cl.Hc, cl.Wc, cl.py,
                       cl.px, 16, cl.a0, cl.c0);
}

// ----------------------------------------------------------------------------
// conv_h_kernel: the regular 3x3 convolution with the styled epilogue, on 16 x 16
// pixel blocks whose 18 x 18 input halo is staged ONCE per channel group and read
// at the nine tap offsets (conv_x_kernel stages every tap's 256 shifted pixels:
// 9 x 32 KB of activations per channel group against 41 KB here; with the 16 KB of
// weights per K-step the L2 -> LDS stream per K-step drops from 48 KB to ~21 KB).
//
// Halo image per channel group: [hy 18][hx 18] pixels of 128 B (the group's 32
// channels as split-NHWC quads q = 2 g + lo), quad q stored at slot q ^ swz(hx)
// with swz(hx) = (hx & 4) | (hx >> 1 & 1): the 16 lanes of every ds_read_b128
// lane group then hit 16 distinct bank quads whatever the tap's column shift
// (checked exhaustively for all shifts).  The LDS-DMA applies the swizzle through
// each lane's source address (a piece's destinations are fixed: 8 consecutive
// image pixels).  Zero padding: out-of-image lanes read past num_records.
// A fragment address is a per-lane base (one of 3 column shifts x hi/lo, plus the
// buffer) and a compile-time offset (row and column of the tap and n-tile), so the
// unrolled tap loop reads fragments without address VALU.  The weight ring and the
// mid-step barrier / next-step fragment schedule are conv_x_kernel's;
// the nine taps of a channel group are unrolled (stage = tap % 3), two groups per
// loop iteration so the register sets alternate.
//
// Persistent: one workgroup per CU (LDS 155 KB) walks a strided share of its XCD's
// contiguous tile run.  After the last K-step's barrier every LDS buffer is free, so
// the NEXT tile's prologue (halo of channel group 0, weights of its first three
// K-steps) is issued there and lands under the last MFMAs and this tile's epilogue,
// instead of behind a workgroup exit + dispatch + cold prologue.  The epilogue's
// per-channel operands (demod, bias, s_next, ToRGB weights) and the block's noise
// arrive in LDS by six more DMA pieces during the tile's second K-step, so the
// epilogue issues no global load that would have to wait (in-order vmcnt) behind the
// next tile's DMAs.
// ----------------------------------------------------------------------------
constexpr uint32_t kHaloW = 18;
constexpr uint32_t kHaloPx = kHaloW * kHaloW;          // 324
constexpr uint32_t kHaloPieces = 48;                  // 6 per wave; 41 carry pixels
constexpr uint32_t kHaloF4 = kHaloPieces * 64;        // 48 KB per buffer
// epilogue operand pieces (1 KB, one per wave 0..6): demod, bias, s_next (128
// channels in lanes 0-31 each), ToRGB weights o = 0 | 1, o = 2 (the face's rows of
// rgb_w, or rgb_base's), noise (16 rows x 16), the face's rgb_s row (rgb_base only)
constexpr uint32_t kEpPieces = 7;

__device__ __forceinline__ uint32_t halo_swz(uint32_t hx) { return (hx & 4u) | ((hx >> 1) & 1u); }

typedef __attribute__((address_space(3))) f4 lds_f4_t;
__device__ __forceinline__ f4 lds_f4(uint32_t byte_addr) {   // LDS byte address -> f4
    return *(const lds_f4_t *)(size_t)byte_addr;
}

// conv_epilogue<true> for a 16 x 16 block whose epilogue operands sit in LDS (Ep):
// same arithmetic in the same order; lane (n, g) of tile (i, j) holds channels
// 16 (4 wm + i) + 4 g .. +3 of block pixel (row 4 wn + j, column n).
__device__ __forceinline__ void conv_h_epilogue(const ConvArgs &a, f4 (&acc)[4][4], const f4 *Ep,
                                                uint32_t lane, uint32_t wm, uint32_t wn,
                                                uint32_t cb, uint32_t pix0, uint32_t b) {
    __shared__ float red[4][4][16][3];          // [wn][j][n][o] from the wm = 1 waves
    // opaque copies: nothing of the epilogue's address arithmetic is hoisted out of
    // conv_h_kernel's tile loop (it would stay live through the K loop and spill)
    asm volatile("" : "+v"(lane), "+s"(wm), "+s"(wn));
    uint32_t W = a.Win, HW = a.Hin * a.Win;
    asm volatile("" : "+s"(W), "+s"(HW));
    const uint32_t n = lane & 15u, g = lane >> 4;
    const ActEpi &e = a.e;
    const float nw = e.noise ? *e.noise_weight : 0.0f;
    const float *epn = reinterpret_cast<const float *>(Ep + 5 * 64);
    float part[4][3];
#pragma unroll
    for (int j = 0; j < 4; ++j) part[j][0] = part[j][1] = part[j][2] = 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t lq = (4 * wm + i) * 4 + g;     // f4 index of the channel quad
        const uint32_t ch = cb * kCT + 4 * lq;
        const f4 dm = Ep[lq], bs = Ep[64 + lq];
        const f4 sn = e.s_next ? Ep[128 + lq] : f4{1.0f, 1.0f, 1.0f, 1.0f};
        f4 rw[3] = {Ep[192 + lq], Ep[224 + lq], Ep[256 + lq]};
        if (e.rgb_base) {                               // base rows x the face's style
            const f4 rs = Ep[384 + lq];
#pragma unroll
            for (int o = 0; o < 3; ++o) rw[o] = rw[o] * rs;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t r = 4 * wn + j;
            const uint32_t P = pix0 + r * W + n;
            const float nz = e.noise ? nw * epn[r * 16 + n] : 0.0f;
            f4 v;
            if constexpr (kHEpk) {
                // packed fp32 (two channels per v_pk_* op, each the same IEEE operation
                // in the same order as act1: bit-identical; no MFMA runs beside the
                // epilogue, where packed fp32 would cost issue slots)
#pragma unroll
                for (int hp = 0; hp < 2; ++hp) {
                    const f2c c2 = {acc[i][j][2 * hp], acc[i][j][2 * hp + 1]};
                    f2c u = c2 * f2c{dm[2 * hp], dm[2 * hp + 1]};
                    u = u + f2c{nz, nz};
                    u = u + f2c{bs[2 * hp], bs[2 * hp + 1]};
                    const f2c neg = u * f2c{e.slope, e.slope};
                    u = f2c{u.x > 0.0f ? u.x : neg.x, u.y > 0.0f ? u.y : neg.y};
                    u = u * f2c{e.scale, e.scale};
                    v[2 * hp] = u.x;
                    v[2 * hp + 1] = u.y;
                }
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = act1(acc[i][j][q], dm[q], nz, bs[q], e.slope, e.scale);
            }
            if constexpr (kHAbl & 1) {
                if (e.ys && v[0] == 1.2345e-33f) store_split8_pair(e.ys, (size_t)P * a.Cout + (ch & ~7u), v * sn, g);
            } else {
                if (e.ys) store_split8_pair(e.ys, (size_t)P * a.Cout + (ch & ~7u), v * sn, g);
            }
            if constexpr (kHEpk) {
                // channels o = 0, 1 of the ToRGB partials as one packed chain (the same
                // fma per element, the same q order), o = 2 alone
                f2c p01 = {part[j][0], part[j][1]};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    p01 = __builtin_elementwise_fma(f2c{v[q], v[q]}, f2c{rw[0][q], rw[1][q]}, p01);
                    part[j][2] = fmaf(v[q], rw[2][q], part[j][2]);
                }
                part[j][0] = p01.x;
                part[j][1] = p01.y;
            } else {
#pragma unroll
                for (int o = 0; o < 3; ++o)
#pragma unroll
                    for (int q = 0; q < 4; ++q) part[j][o] = fmaf(v[q], rw[o][q], part[j][o]);
            }
        }
    }
    if (!(kHAbl & 4) && (e.rgb_w || e.rgb_base)) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int o = 0; o < 3; ++o) {
                part[j][o] += __shfl_xor(part[j][o], 16, 64);
                part[j][o] += __shfl_xor(part[j][o], 32, 64);
            }
        if (wm == 1 && g == 0)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int o = 0; o < 3; ++o) red[wn][j][n][o] = part[j][o];
        // raw barrier: the LDS writes above are all it orders (a __syncthreads fence
        // could add a vmcnt wait on the next tile's DMAs)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (wm == 0 && g < 3) {                 // lane (n, g = o) stores channel o
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t P = pix0 + (4 * wn + j) * W + n;
                const float s = (g == 0 ? part[j][0] : g == 1 ? part[j][1] : part[j][2]) +
                                red[wn][j][n][g];
                e.rgbp[(((size_t)cb * a.B + b) * 3 + g) * HW + (P - b * HW)] = s;
            }
        }
        // red is rewritten by the next tile's epilogue only after that tile's barriers
    }
}

template <bool SPLIT>
__global__ void __launch_bounds__(512, 1) conv_h_kernel(const ConvArgs a) {
    __shared__ f4 As[3][kStepF4];        // weight ring [mt 8][hi,lo][64]
    __shared__ f4 Hs[2][kHaloF4];        // halo images, by channel-group parity
    __shared__ f4 Ep[kEpPieces * 64];    // epilogue operands of the current tile
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t wm = wave & 1u, wn = wave >> 1;
    const uint32_t H = a.Hin, W = a.Win;
    const uint32_t nC = a.Cin / 32, nB = a.Cout / kCT;
    const uint32_t nbx = W / 16, nby = H / 16;
    const v4i rw = make_rsrc(a.wpk, 9u * nC * nB * kStepF4 * 16u);
    const v4i rx = make_rsrc(a.xs, a.B * H * W * a.Cin * 4);
    // tile -> Cout block cb, first pixel pix0 (image b, block origin y0, x0) and this
    // wave's halo pieces k = wave + 8 i (per-lane source offsets at channel group 0;
    // the group moves the buffer's soffset by 128 B)
    // K split (a.ksplit > 1, small batches): item = split * ntiles + tile takes channel
    // groups [cg0, cg1) of its tile and stores the raw partial accumulators;
    // conv_h_finish_kernel sums them and runs the epilogue
    const uint32_t ks = SPLIT ? a.ksplit : 1u, ntiles = a.cls[0].ntiles;
    uint32_t cb = 0, pix0 = 0, bimg = 0, y0 = 0, x0 = 0, hoff[6], cg0 = 0, cg1 = nC;
    auto setup = [&](uint32_t item) {
        uint32_t ln = lane, wv = wave;        // opaque: computed here, not hoisted
        asm volatile("" : "+v"(ln), "+s"(wv));
        uint32_t tile = item;
        if constexpr (SPLIT) {
            const uint32_t split = item / ntiles;
            tile = item - split * ntiles;
            cg0 = split * nC / ks;
            cg1 = (split + 1) * nC / ks;
        }
        cb = tile % nB;
        uint32_t blk = tile / nB;
        const uint32_t bx = blk % nbx;
        blk /= nbx;
        const uint32_t by = blk % nby, b = blk / nby;
        bimg = b;
        y0 = by * 16;
        x0 = bx * 16;
        pix0 = (b * H + y0) * W + x0;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const uint32_t h = 8u * (wv + 8u * i) + (ln >> 3);
            const uint32_t hy = h / kHaloW, hx = h - hy * kHaloW;
            const uint32_t q = (ln & 7u) ^ halo_swz(hx);
            const int y = (int)(y0 + hy) - 1, x = (int)(x0 + hx) - 1;
            const bool ok = h < kHaloPx && y >= 0 && y < (int)H && x >= 0 && x < (int)W;
            hoff[i] = ok ? (((b * H + (uint32_t)y) * W + (uint32_t)x) * a.Cin * 4u + q * 16u)
                         : 0x7FFFFFF0u;
        }
    };
    const uint32_t n = lane & 15u, g = lane >> 4;
    // fragment lane bases (bytes within a halo buffer): [column shift dx + 1][lo]
    uint32_t fb0[3][2];
#pragma unroll
    for (int d = 0; d < 3; ++d)
#pragma unroll
        for (int lo = 0; lo < 2; ++lo)
            fb0[d][lo] = (4u * wn * kHaloW + n) * 128u + (((2u * g + lo) ^ halo_swz(n + d)) << 4);
    const uint32_t hs0 = lds_addr(&Hs[0][0]), hs1 = lds_addr(&Hs[1][0]);

    auto uni = [](v4i r) {     // keep the resources in SGPRs (the inline asm needs them there)
        return v4i{__builtin_amdgcn_readfirstlane(r.x), __builtin_amdgcn_readfirstlane(r.y),
                   __builtin_amdgcn_readfirstlane(r.z), __builtin_amdgcn_readfirstlane(r.w)};
    };
    auto fire_w = [&](uint32_t c, uint32_t tap, uint32_t stage) {
        const uint32_t wsoff = __builtin_amdgcn_readfirstlane(
            ((tap * nC + c) * nB + cb) * kStepF4 * 16u + 2 * wave * 1024u);
        set_m0(lds_addr(&As[stage][2 * wave * 64]));
        dma16<0>(uni(rw), lane * 16u, wsoff);
        dma16<1024>(uni(rw), lane * 16u, wsoff);
    };
    uint32_t hsoff = 0;                   // soffset of the group being fetched (c * 128 B)
    auto fire_h = [&](int buf, int i) {
        set_m0(lds_addr(&Hs[buf][(wave + 8u * i) * 64]));
        dma16<0>(uni(rx), hoff[i], __builtin_amdgcn_readfirstlane(hsoff));
    };
    // the current tile's epilogue operands -> Ep (wave w moves piece w; null tensors
    // and the idle lanes read past num_records = zeros)
    auto fire_ep = [&] {
        if (wave >= kEpPieces) return;
        uint32_t lane = tid & 63u;            // opaque: computed here, not hoisted
        asm volatile("" : "+v"(lane));
        const ActEpi &e = a.e;
        const uint32_t OOB = 0x7FFFFFF0u;
        const uint32_t ch = cb * kCT + 4u * (lane & 31u), lo = lane < 32;
        const uint32_t bc = a.B * a.Cout * 4u;
        const float *base;
        uint32_t bytes, off;
        if (wave == 0) {
            base = e.demod; bytes = bc; off = lo ? (bimg * a.Cout + ch) * 4u : OOB;
        } else if (wave == 1) {
            base = e.bias; bytes = a.Cout * 4u; off = lo ? ch * 4u : OOB;
        } else if (wave == 2) {
            base = e.s_next; bytes = e.s_next ? bc : 0u; off = lo ? (bimg * a.Cout + ch) * 4u : OOB;
        } else if (wave == 3 || wave == 4) {
            const uint32_t o = wave == 3 ? (lane >> 5) : 2u;
            const bool ok = wave == 3 || lo;
            if (e.rgb_base) {
                base = e.rgb_base; bytes = 3u * a.Cout * 4u; off = ok ? (o * a.Cout + ch) * 4u : OOB;
            } else {
                base = e.rgb_w; bytes = e.rgb_w ? 3u * bc : 0u;
                off = ok ? ((bimg * 3u + o) * a.Cout + ch) * 4u : OOB;
            }
        } else if (wave == 5) {
            base = e.noise; bytes = e.noise ? a.B * H * W * 4u : 0u;
            off = ((bimg * H + y0 + (lane >> 2)) * W + x0 + 4u * (lane & 3u)) * 4u;
        } else {
            base = e.rgb_s; bytes = e.rgb_base ? bc : 0u; off = lo ? (bimg * a.Cout + ch) * 4u : OOB;
        }
        set_m0(lds_addr(&Ep[wave * 64]));
        dma16<0>(uni(make_rsrc(base, bytes)), off, 0u);
    };

    f4 acc[4][4];

    // fragments of tap T of a channel group whose halo lies at byte hs: A from stage
    // T % 3, B at the tap's offset (dy, dx) = (T / 3 - 1, T % 3 - 1)
    auto read_frags = [&](f4 (&R)[16], auto tapc, uint32_t hs) {
        constexpr int T = decltype(tapc)::value;
        constexpr uint32_t st = T % 3, dyp = T / 3, dxp = T % 3;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            R[i] = As[st][((4 * wm + i) * 2) * 64 + lane];
            R[4 + i] = As[st][((4 * wm + i) * 2 + 1) * 64 + lane];
        }
        const uint32_t bh = hs + fb0[dxp][0], bl = hs + fb0[dxp][1];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t imm = ((j + dyp) * kHaloW + dxp) * 128u;
            R[8 + j] = lds_f4(bh + imm);
            R[12 + j] = lds_f4(bl + imm);
        }
    };
    auto mfma_rows = [&](const f4 (&R)[16], int i0, int nr) {
#pragma unroll
        for (int i = i0; i < i0 + nr; ++i) {
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(R[4 + i], R[8 + j], acc[i][j]);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(R[i], R[12 + j], acc[i][j]);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(R[i], R[8 + j], acc[i][j]);
        }
    };

    // split term t (0: lo.hi, 1: hi.lo, 2: hi.hi; mfma_rows' order) of row i
    auto mfma_quad = [&](const f4 (&R)[16], int i, int t) {
        const f4 &ra = t == 0 ? R[4 + i] : R[i];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            acc[i][j] = mfma16(ra, t == 1 ? R[12 + j] : R[8 + j], acc[i][j]);
    };

    // prologue of a tile: halo of group 0, weights of steps 0-2 (every LDS buffer is
    // free once all waves passed the previous tile's last barrier)
    auto prologue = [&] {
        hsoff = cg0 * 128u;
#pragma unroll
        for (int i = 0; i < 6; ++i) fire_h(0, i);
        hsoff += 128u;                    // next: group cg0 + 1
        fire_w(cg0, 0, 0);
        fire_w(cg0, 1, 1);
        fire_w(cg0, 2, 2);
    };

    // persistent schedule: XCD x owns tiles [x per, (x + 1) per) (Cout block fastest,
    // as slot_tile); its workgroups take them with stride nwg, so the ones running
    // together share halos and weights in the XCD's L2
    const uint32_t nitems = ntiles * ks, per = (nitems + 7) >> 3;
    const uint32_t xcd = blockIdx.x & 7u, nwg = gridDim.x >> 3;
    const uint32_t tend = min(xcd * per + per, nitems);
    uint32_t tile = __builtin_amdgcn_readfirstlane(xcd * per + (blockIdx.x >> 3));
    if (tile >= tend) return;    // idle workgroup (whole)
    uint32_t next = tile + nwg;
    bool has_next = next < tend;

    // K-step (c, T): MFMAs of rows 0-1; wait for step (c, T)+1 (in flight may stay only
    // what step (c, T)-1 fired); barrier; fire step +3's weights (into stage T % 3) and,
    // at taps 0-5, halo piece T of group c + 1 (into the buffer group c - 1 used, whose
    // last fragment reads were before the barrier of (c - 1, 8)); read step +1's
    // fragments; MFMAs of rows 2-3.  The tile's second step also fires the epilogue
    // operands (older than everything step 3 waits for); the last one fires the next
    // tile's prologue.
    // P: parity of group c (its halo buffer), compile-time in the unrolled loop
    auto step = [&](uint32_t c, auto tapc, auto parc, const f4 (&R)[16], f4 (&Rn)[16]) {
        constexpr int T = decltype(tapc)::value;
        constexpr int P = decltype(parc)::value;
        const uint32_t s = (c - cg0) * 9 + T, nk = (cg1 - cg0) * 9;
        const bool prev_w = s + 2 < nk;                     // step s-1 fired weights
        const bool prev_h = T != 0 && T - 1 <= 5 && c + 1 < cg1;  // ... and a halo piece
        mfma_rows(R, 0, 2);
        if (prev_w && prev_h) asm volatile("s_waitcnt vmcnt(3) lgkmcnt(0)" ::: "memory");
        else if (prev_w) asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if constexpr (T == 1) {
            if (c == cg0 && !SPLIT) fire_ep();
        }
        // Issue order after the barrier, pinned by scheduling fences (left to itself
        // the compiler clumps all DMAs and reads in front of the MFMAs, and an LDS-DMA
        // issued in such a clump costs the wave several times its price between
        // MFMAs; measured -3.7 % conv time): the next step's 16 fragment reads one per
        // MFMA of row 2 (after the last step they read stale data nobody uses), then
        // the weight pair and the halo piece (and after the last step the next tile's
        // prologue) between the three MFMA quads of row 3.
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (T == 8) read_frags(Rn, std::integral_constant<int, 0>{}, P ? hs0 : hs1);
        else read_frags(Rn, std::integral_constant<int, T + 1>{}, P ? hs1 : hs0);
        mfma_rows(R, 2, 1);
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
        for (int k = 0; k < 12; ++k) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        mfma_quad(R, 3, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (s + 3 < nk) {
            constexpr uint32_t T3 = (T + 3) % 9;
            fire_w(c + (T + 3) / 9, T3, T % 3);
        }
        __builtin_amdgcn_sched_barrier(0);
        mfma_quad(R, 3, 1);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (T <= 5) {
            if (c + 1 < cg1) fire_h(1 - P, T);
        }
        if constexpr (T == 8) {
            if (s + 1 == nk && has_next) {
                setup(next);
                prologue();
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        mfma_quad(R, 3, 2);
        __builtin_amdgcn_sched_barrier(0);
    };

    setup(tile);
    prologue();
    bool first = true;
    for (;;) {
        const uint32_t ecb = cb, epix0 = pix0, eb = bimg;    // this tile (setup moves on)
        const uint32_t eitem = tile, c1 = cg1;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.0f, 0.0f, 0.0f, 0.0f};
        // everything but step 2's weights has landed (after the first tile: everything,
        // the previous epilogue's stores included); the previous epilogue's LDS reads
        // are done everywhere after the barrier
        if (first) asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        f4 R0[16], R1[16];
        read_frags(R0, std::integral_constant<int, 0>{}, hs0);
        // two channel groups per iteration: 18 steps alternate R0 / R1
        uint32_t c = cg0;
        for (; c + 1 < c1; c += 2) {
            step(c, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, R0, R1);
            step(c, std::integral_constant<int, 1>{}, std::integral_constant<int, 0>{}, R1, R0);
            step(c, std::integral_constant<int, 2>{}, std::integral_constant<int, 0>{}, R0, R1);
            step(c, std::integral_constant<int, 3>{}, std::integral_constant<int, 0>{}, R1, R0);
            step(c, std::integral_constant<int, 4>{}, std::integral_constant<int, 0>{}, R0, R1);
            step(c, std::integral_constant<int, 5>{}, std::integral_constant<int, 0>{}, R1, R0);
            hsoff += 128u;
            step(c, std::integral_constant<int, 6>{}, std::integral_constant<int, 0>{}, R0, R1);
            step(c, std::integral_constant<int, 7>{}, std::integral_constant<int, 0>{}, R1, R0);
            step(c, std::integral_constant<int, 8>{}, std::integral_constant<int, 0>{}, R0, R1);
            step(c + 1, std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{}, R1, R0);
            step(c + 1, std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{}, R0, R1);
            step(c + 1, std::integral_constant<int, 2>{}, std::integral_constant<int, 1>{}, R1, R0);
            step(c + 1, std::integral_constant<int, 3>{}, std::integral_constant<int, 1>{}, R0, R1);
            step(c + 1, std::integral_constant<int, 4>{}, std::integral_constant<int, 1>{}, R1, R0);
            step(c + 1, std::integral_constant<int, 5>{}, std::integral_constant<int, 1>{}, R0, R1);
            hsoff += 128u;
            step(c + 1, std::integral_constant<int, 6>{}, std::integral_constant<int, 1>{}, R1, R0);
            step(c + 1, std::integral_constant<int, 7>{}, std::integral_constant<int, 1>{}, R0, R1);
            step(c + 1, std::integral_constant<int, 8>{}, std::integral_constant<int, 1>{}, R1, R0);
        }
        if (c < c1) {
            step(c, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, R0, R1);
            step(c, std::integral_constant<int, 1>{}, std::integral_constant<int, 0>{}, R1, R0);
            step(c, std::integral_constant<int, 2>{}, std::integral_constant<int, 0>{}, R0, R1);
            step(c, std::integral_constant<int, 3>{}, std::integral_constant<int, 0>{}, R1, R0);
            step(c, std::integral_constant<int, 4>{}, std::integral_constant<int, 0>{}, R0, R1);
            step(c, std::integral_constant<int, 5>{}, std::integral_constant<int, 0>{}, R1, R0);
            step(c, std::integral_constant<int, 6>{}, std::integral_constant<int, 0>{}, R0, R1);
            step(c, std::integral_constant<int, 7>{}, std::integral_constant<int, 0>{}, R1, R0);
            step(c, std::integral_constant<int, 8>{}, std::integral_constant<int, 0>{}, R0, R1);
        }
        if (SPLIT) {    // raw partials of this split: [item][16 (i, j)][512 threads] f4
            f4 *pp = a.partial + (size_t)eitem * 16 * 512 + tid;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) pp[(i * 4 + j) * 512] = acc[i][j];
        } else if constexpr (kHAbl & 2) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (acc[i][j][0] == 1.2345e-33f)
                        *reinterpret_cast<f4 *>(a.e.ys + (size_t)(epix0 + lane) * 8u + 4u * (4u * i + j)) = acc[i][j];
        } else {
            conv_h_epilogue(a, acc, Ep, lane, wm, wn, ecb, epix0, eb);
        }
        if (!has_next) break;
        tile = next;
        next = tile + nwg;
        has_next = next < tend;
        first = false;
    }
}

// conv_h_kernel's grid: up to one workgroup per CU, a multiple of 8 (XCD count)
uint32_t conv_h_grid(uint32_t ntiles) {
    const uint32_t per = (ntiles + 7) >> 3;
    return 8u * (per < kCusPerXcd ? per : kCusPerXcd);
}

// conv_h_kernel's K-split finish: the ksplit partial tiles summed in split order
// (deterministic; the same K ranges and order as conv_x_kernel's split), then the
// fused epilogue.  A workgroup is a QUARTER tile: the two waves (wm = 0, 1) of one
// n-tile row group wn = blockIdx.y, so the finish of a batch-1 layer spreads over 4x the
// CUs of the conv (64 -> 256 workgroups at 64^2).
__global__ void __launch_bounds__(128) conv_h_finish_kernel(const ConvArgs a) {
    const uint32_t tile = blockIdx.x, wn = blockIdx.y;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wm = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t ntiles = a.cls[0].ntiles;
    const uint32_t tid = (wm + 2u * wn) * 64u + lane;       // conv_h_kernel's thread of it
    const uint32_t nB = a.Cout / kCT, nbx = a.Win / 16, nby = a.Hin / 16;
    const uint32_t cb = tile % nB, blk = tile / nB;
    const uint32_t bx = blk % nbx, by = (blk / nbx) % nby, b = blk / (nbx * nby);
    const uint32_t pix0 = (b * a.Hin + by * 16u) * a.Win + bx * 16u;
    f4 acc[4][4], t[3][16];
    const f4 *pp = a.partial + (size_t)tile * 16 * 512 + tid;
    const size_t sstride = (size_t)ntiles * 16 * 512;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = pp[(i * 4 + j) * 512];
#pragma unroll
    for (uint32_t s = 1; s < 4; ++s)
        if (s < a.ksplit)
#pragma unroll
            for (int q = 0; q < 16; ++q) t[s - 1][q] = pp[s * sstride + q * 512];
#pragma unroll
    for (uint32_t s = 1; s < 4; ++s)
        if (s < a.ksplit)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] += t[s - 1][i * 4 + j];
    conv_epilogue<true>(a, acc, lane, wm, wn, cb, pix0, a.B * a.Hin * a.Win, a.Hin, a.Win, 0, 0,
                        a.Win, 0, 0);
}

// ----------------------------------------------------------------------------
// conv_t_kernel: the stride-2 transposed convolution of an upsampling StyledConv
// (sdf_model.py:660-701, conv_transpose2d before the blur) for all four output parity
// classes of a 16 x 16 block of INPUT positions (a, c) in one workgroup, over one
// input halo per channel group (conv_h_kernel's 18 x 18 staging, anchored at
// (a - 1, c - 1)).  Class (py, px) of position (a, c) is output pixel
// (2 a + py, 2 c + px) and takes taps ky in {0, 2} (py = 0: inputs a, a - 1) or
// ky = 1 (py = 1: input a), likewise x: the four classes' 4 + 2 + 2 + 1 taps are nine
// K-steps per channel group over four input positions (dy, dx) in {0, -1}^2, ordered
// by position so a B fragment read from the halo serves every class-tap at it:
//     s    0     1     2     3  |  4     5  |  6     7  |  8
//   (ky,kx) (0,0) (0,1) (1,0) (1,1) | (2,0) (2,1) | (0,2) (1,2) | (2,2)
//   (dy,dx)        (0, 0)         |  (-1, 0)  |  (0, -1)  | (-1,-1)
// Every K-step is the same work for every wave (2 m-tiles x 4 n-tiles x 3 split terms
// into the step's class accumulators), so the nine taps of a channel group run like
// conv_h_kernel's nine: weight ring of 3 x 8 KB (64 channels x 32), halo of the next
// group fired over the first six steps, one barrier per step, persistent tiles.
// conv_x_kernel staged 256 shifted pixels per tap and ran each class as its own
// workgroups (a 1-tap class: 8-16 K-steps per 128 KB of fp32 stores).
// Output: the raw fp32 (2H + 1)^2 grid for rows / columns < 2H, 2W; the last row and
// column (even classes at a = H, c = W) are four thin classes of conv_x_kernel.
// ----------------------------------------------------------------------------
constexpr uint32_t kTCT = 64;          // output channels per conv_t workgroup
constexpr uint32_t kTStepF4 = 512;     // f4 of weight fragments per K-step (8 KB)

__host__ __device__ constexpr int t_ky(int s) {
    return (s == 2 || s == 3 || s == 7) ? 1 : ((s == 4 || s == 5 || s == 8) ? 2 : 0);
}
__host__ __device__ constexpr int t_kx(int s) { return s < 6 ? (s & 1) : 2; }
__host__ __device__ constexpr int t_pos(int s) { return s < 4 ? 0 : (s < 6 ? 1 : (s < 8 ? 2 : 3)); }

// ---- conv_t_kernel<true>: the upsampling StyledConv's blur and styled epilogue ----
// (sdf_model.py:674-683, 704-818: Blur(pad (1, 1), 4 x 4 = outer(fir, fir)) of the
// transposed conv's (2H + 1)^2 output, then demod, noise, bias, leaky ReLU x sqrt 2 and
// the next layer's modulation; epi_blur_kernel's arithmetic, in its order).  A block's
// 32 x 32 output pixels need its 35 x 35 conv outputs (one row / column before, two
// after): the interior 29 x 29 are finished here from the accumulators -- the 4-tap
// horizontal pass across lanes (DPP row shifts within the 16-lane rows that hold a
// position row's 16 columns), the vertical pass across a lane's rows, the rows at the
// 4-row wave boundaries exchanged through LDS -- and the border pixels (rows and
// columns 0, 30, 31 of a block) by conv_t_border_kernel, from the raw conv values of
// the band rows / columns (0-2, 29-31) that this kernel stores instead of the whole
// fp32 output.
__device__ __forceinline__ bool t_band(uint32_t r) { return r <= 2u || r >= 29u; }
__device__ __forceinline__ bool t_border(uint32_t r) { return r == 0u || r >= 30u; }

// value of lane n - 1 (PREV) or n + 1 of the lane's 16-lane row; 0 past the row's end.
// (The whole vector is bit-cast: hipcc (ROCm 7.2) reads element 0 for a bit_cast of one
// element v[k] of an ext-vector, whatever k -- DESIGN.md §5.2.)
template <bool PREV>
__device__ __forceinline__ f4 dpp_row_shift(f4 v) {
    typedef int i4 __attribute__((ext_vector_type(4)));
    constexpr int ctl = PREV ? 0x111 : 0x101;           // row_shr:1 / row_shl:1
    const i4 iv = __builtin_bit_cast(i4, v);
    i4 r;
    r.x = __builtin_amdgcn_update_dpp(0, iv.x, ctl, 0xF, 0xF, true);
    r.y = __builtin_amdgcn_update_dpp(0, iv.y, ctl, 0xF, 0xF, true);
    r.z = __builtin_amdgcn_update_dpp(0, iv.z, ctl, 0xF, 0xF, true);
    r.w = __builtin_amdgcn_update_dpp(0, iv.w, ctl, 0xF, 0xF, true);
    return __builtin_bit_cast(f4, r);
}

// store_split8_pair, the store only where `live` (both lanes of a pair agree on it)
__device__ __forceinline__ void store_split8_pair_if(_Float16 *ys, size_t idx8, f4 v, uint32_t g,
                                                     bool live) {
    asm volatile("" : "+v"(v));        // the fp32 product rounded first (not folded into the cvt)
    h4 h, l;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        h[r] = (_Float16)v[r];
        l[r] = (_Float16)(v[r] - (float)h[r]);
    }
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    const u2 hd = __builtin_bit_cast(u2, h), ld = __builtin_bit_cast(u2, l);
    uint32_t q[4];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const auto r = __builtin_amdgcn_permlane16_swap(hd[k], ld[k], false, false);
        uint32_t r0 = r[0], r1 = r[1];
        asm volatile("" : "+v"(r0), "+v"(r1));
        q[k] = r0;
        q[2 + k] = r1;
    }
#if defined(SDFR_TVAR) && SDFR_TVAR == 2
    if (live && q[0] == 0x12345u) *reinterpret_cast<f4 *>(ys + 2 * idx8 + (g & 1u) * 8) = __builtin_bit_cast(f4, q);
#else
    if (live) *reinterpret_cast<f4 *>(ys + 2 * idx8 + (g & 1u) * 8) = __builtin_bit_cast(f4, q);
#endif
}

// 4-tap filter in epi_blur_kernel's order: fma chain from 0 (horizontal, hfilt) ...
__device__ __forceinline__ f4 fir_h(const f4 &v0, const f4 &v1, const f4 &v2, const f4 &v3,
                                    float f0, float f1, float f2, float f3) {
    f4 h;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        h[k] = fmaf(v3[k], f3, fmaf(v2[k], f2, fmaf(v1[k], f1, fmaf(v0[k], f0, 0.0f))));
    return h;
}
// ... and from the first product (vertical)
__device__ __forceinline__ f4 fir_v(const f4 &h0, const f4 &h1, const f4 &h2, const f4 &h3,
                                    float f0, float f1, float f2, float f3) {
    f4 s;
#pragma unroll
    for (int k = 0; k < 4; ++k) s[k] = fmaf(h3[k], f3, fmaf(h2[k], f2, fmaf(h1[k], f1, h0[k] * f0)));
    return s;
}

// The epilogue of one conv_t_kernel<true> tile.  acc[2 py + px][i][j]: channels
// 16 (2 wm + i) + 4 g .. + 3 of the block's 64, input position (4 wn + j, n), output pixel
// (2 (4 wn + j) + py, 2 n + px) of the block.  Ep: the tile's demod, bias, s_next (64
// channels, f4 0-15 of pieces 0-2) and noise (32 x 32 floats from f4 192), staged at the
// tile's start (conv_t_kernel); Xs: 48 KB of LDS free during the epilogue (the halo
// buffer of odd channel groups).  No global load here: one issued behind the epilogue's
// stores would wait for them to drain (vmcnt retires in order).
__device__ __forceinline__ void conv_t_blur_epilogue(const ConvArgs &a0, f4 (&acc)[4][2][4],
                                                     const f4 *Ep, f4 *Xs, uint32_t lane,
                                                     uint32_t wave, uint32_t cb, uint32_t b,
                                                     uint32_t y0, uint32_t x0) {
    asm volatile("" : "+v"(lane), "+s"(wave));
    const ConvArgs &a = a0;
    const uint32_t wm = wave & 1u, wn = wave >> 1;
    const uint32_t n = lane & 15u, g = lane >> 4;
    const uint32_t C = a.Cout, Wf = a.Wf, H2 = 2u * a.Hin, W2 = 2u * a.Win;
    const ActEpi &e = a.e;
    const size_t pbase = (size_t)b * H2 + 2u * y0;
    const float nw = e.noise ? *e.noise_weight : 0.0f;   // (a scalar load)
    const float *epn = reinterpret_cast<const float *>(Ep + 192);
    // 1. the raw conv values of the band rows / columns (conv_t_border_kernel's input)
    {
        float *raw = a.out + (size_t)cb * kTCT + 2u * wm * 16u + 4u * g;
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t yr = 2u * (4u * wn + j) + (uint32_t)(q >> 1);
                const uint32_t xr = 2u * n + (uint32_t)(q & 1);
                if (t_band(yr) || t_band(xr)) {
                    float *dst = raw + ((size_t)(b * a.Hf + 2u * y0 + yr) * Wf + 2u * x0 + xr) * C;
#pragma unroll
                    for (int i = 0; i < 2; ++i) *reinterpret_cast<f4 *>(dst + i * 16) = acc[q][i][j];
                }
            }
    }
    const float f0 = a.fir[3], f1 = a.fir[2], f2 = a.fir[1], f3 = a.fir[0];   // flipped taps
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                       // the K loop's reads of Xs are done
#pragma unroll
    for (int i = 0; i < 2; ++i) {   // per 16-channel m-tile (register pressure)
        // (scheduling fences: left free, hipcc hoists m-tile 1's DPP reads above m-tile
        // 0's stores and spills them; a scratch reload behind the stores waits for them)
        __builtin_amdgcn_sched_barrier(0);
        // 2. horizontal pass in place: acc[2 py + px] <- conv row 2 a + py filtered at
        //    column 2 c + px (columns 2c-1 .. 2c+2: lane n - 1's px 1, own px 0 / 1, lane
        //    n + 1's px 0 / 1)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int py = 0; py < 2; ++py) {
                const f4 c0 = acc[2 * py][i][j], c1 = acc[2 * py + 1][i][j];
                const f4 l1 = dpp_row_shift<true>(c1);
                const f4 r0 = dpp_row_shift<false>(c0), r1 = dpp_row_shift<false>(c1);
                acc[2 * py][i][j] = fir_h(l1, c0, c1, r0, f0, f1, f2, f3);
                acc[2 * py + 1][i][j] = fir_h(c0, c1, r0, r1, f0, f1, f2, f3);
            }
        __builtin_amdgcn_sched_barrier(0);
        // 3. rows across the 4-row wave boundaries: wave (wm, wn) needs row 4 wn - 1's
        //    odd conv row (wave - 2's j = 3, py = 1) and row 4 wn + 4's two (wave + 2's
        //    j = 0).  (A barrier separates the previous m-tile's reads from these writes.)
        if (i) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        }
        f4 *mine = Xs + wave * 6u * 64u + lane;
#pragma unroll
        for (int q = 0; q < 4; ++q) mine[q * 64] = acc[q][i][0];
        mine[4 * 64] = acc[2][i][3];
        mine[5 * 64] = acc[3][i][3];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        // (read where used: wave - 2's rows for j = 0, wave + 2's for j = 3; the top and
        // bottom waves read a neighbour's slot of no use -- those pixels are borders)
        const f4 *above = Xs + ((wave - 2u) & 7u) * 6u * 64u + lane;
        const f4 *below = Xs + ((wave + 2u) & 7u) * 6u * 64u + lane;
        // 4. vertical pass, styled epilogue, split store (interior pixels)
        const uint32_t lq = (2u * wm + i) * 4u + g;         // f4 index of the channel quad
        const uint32_t ch = cb * kTCT + 4u * lq;
        const f4 dm = Ep[lq], bs = Ep[64 + lq], sn = Ep[128 + lq];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int px = 0; px < 2; ++px) {
                const f4 hm1 = j > 0 ? acc[2 + px][i][j - 1] : above[(4 + px) * 64];  // a - 1, py 1
                const f4 h00 = acc[px][i][j], h01 = acc[2 + px][i][j];                 // a, py 0 / 1
                const f4 hp0 = j < 3 ? acc[px][i][j + 1] : below[px * 64];            // a + 1, py 0
                const f4 hp1 = j < 3 ? acc[2 + px][i][j + 1] : below[(2 + px) * 64];  // a + 1, py 1
#pragma unroll
                for (int py = 0; py < 2; ++py) {
                    const f4 sv = py == 0 ? fir_v(hm1, h00, h01, hp0, f0, f1, f2, f3)
                                          : fir_v(h00, h01, hp0, hp1, f0, f1, f2, f3);
                    const uint32_t yr = 2u * (4u * wn + j) + py, xr = 2u * n + px;
                    const float nz = nw * epn[yr * 32u + xr];
                    f4 v;
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = act1(sv[r], dm[r], nz, bs[r], e.slope, e.scale);
                    const size_t P = (pbase + yr) * W2 + 2u * x0 + xr;
                    store_split8_pair_if(e.ys, P * C + (ch & ~7u), v * sn, g,
                                         !t_border(yr) && !t_border(xr));
                }
                __builtin_amdgcn_sched_barrier(0);
            }
    }
}

// The border pixels of conv_t_kernel<true>'s blocks (rows and columns 0, 30 and 31 of
// every 32 x 32 output block: their blur reaches a neighbouring block's conv outputs),
// from the raw band rows / columns and the edge classes' last row / column in a.out,
// with epi_blur_kernel's arithmetic.  The border pixels come in runs of three across
// each block boundary (rows / columns 32 k - 2 .. 32 k); a thread takes one channel
// quad of either a row run x 4 adjacent columns (6 x 7 raw values for 12 outputs) or a
// column run in one non-border row (4 x 6 raw values for 3 outputs).
__device__ __forceinline__ f4 border_ld(const float *src, int yy, int xx, uint32_t Hi, uint32_t Wi,
                                        uint32_t C) {
    return (yy >= 0 && yy < (int)Hi && xx >= 0 && xx < (int)Wi)
               ? *reinterpret_cast<const f4 *>(src + ((size_t)yy * Wi + xx) * C)
               : f4{0.0f, 0.0f, 0.0f, 0.0f};
}

__device__ __forceinline__ void border_out(const ConvArgs &a, uint32_t b, uint32_t Y, uint32_t X,
                                           uint32_t c, f4 s, const f4 &dm, const f4 &bs,
                                           const f4 &sn, float nw) {
    const ActEpi &e = a.e;
    const uint32_t C = a.Cout, H2 = 2u * a.Hin, W2 = 2u * a.Win;
    const size_t P = ((size_t)b * H2 + Y) * W2 + X;
    const float nz = e.noise ? nw * e.noise[P] : 0.0f;
    f4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = act1(s[r], dm[r], nz, bs[r], e.slope, e.scale);
    v = v * sn;
    asm volatile("" : "+v"(v));
    h4 hh, ll;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        hh[r] = (_Float16)v[r];
        ll[r] = (_Float16)(v[r] - (float)hh[r]);
    }
    const size_t idx = P * C + c, o = 2 * idx - (idx & 7u);
    *reinterpret_cast<h4 *>(e.ys + o) = hh;
    *reinterpret_cast<h4 *>(e.ys + o + 8) = ll;
}

template <bool ROWS>
__global__ void __launch_bounds__(256) conv_t_border_kernel(const ConvArgs a) {
    const uint32_t Q = a.Cout >> 2, H2 = 2u * a.Hin, W2 = 2u * a.Win;
    const uint32_t kb = H2 / 32u + 1u, mb = W2 / 32u + 1u;      // row / column boundaries
    const uint32_t items = ROWS ? kb * (W2 / 4u) : (H2 / 4u) * mb;
    const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (t >= (uint64_t)a.B * items * Q) return;
    const uint32_t q = (uint32_t)(t % Q);
    const uint64_t r1 = t / Q;
    const uint32_t item = (uint32_t)(r1 % items);
    const uint32_t b = (uint32_t)(r1 / items);
    const uint32_t c = 4u * q, C = a.Cout, Hi = a.Hf, Wi = a.Wf;
    const float *src = a.out + (size_t)b * Hi * Wi * C + c;
    const float f0 = a.fir[3], f1 = a.fir[2], f2 = a.fir[1], f3 = a.fir[0];
    const ActEpi &e = a.e;
    const f4 dm = *reinterpret_cast<const f4 *>(e.demod + (size_t)b * C + c);
    const f4 bs = *reinterpret_cast<const f4 *>(e.bias + c);
    const f4 sn = e.s_next ? *reinterpret_cast<const f4 *>(e.s_next + (size_t)b * C + c)
                           : f4{1.0f, 1.0f, 1.0f, 1.0f};
    const float nw = e.noise ? *e.noise_weight : 0.0f;
    if constexpr (ROWS) {
        // output rows 32 k - 2 .. 32 k (those inside the image) x columns X0 .. X0 + 3
        const uint32_t k = item / (W2 / 4u), X0 = 4u * (item % (W2 / 4u));
        const int Yb = 32 * (int)k - 2;
        // rows Yb - 1 .. Yb + 4 one at a time (a 4-row window of filtered rows: VGPRs)
        f4 h[4][4];
#pragma unroll
        for (int r = 0; r < 6; ++r) {
            f4 v[7];
#pragma unroll
            for (int j = 0; j < 7; ++j) v[j] = border_ld(src, Yb - 1 + r, (int)X0 - 1 + j, Hi, Wi, C);
#pragma unroll
            for (int x = 0; x < 4; ++x)
                h[r & 3][x] = fir_h(v[x], v[x + 1], v[x + 2], v[x + 3], f0, f1, f2, f3);
            if (r >= 3) {
                const int y = r - 3, Y = Yb + y;
                if (Y >= 0 && Y < (int)H2) {
#pragma unroll
                    for (int x = 0; x < 4; ++x)
                        border_out(a, b, (uint32_t)Y, X0 + x, c,
                                   fir_v(h[y & 3][x], h[(y + 1) & 3][x], h[(y + 2) & 3][x],
                                         h[(y + 3) & 3][x], f0, f1, f2, f3),
                                   dm, bs, sn, nw);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    } else {
        // rows 4 r .. 4 r + 3 (the non-border ones: 1 .. 29 of a block) x output columns
        // 32 m - 2 .. 32 m, rows one at a time through a 4-row window
        const uint32_t m = item % mb, Y0 = 4u * (item / mb);
        const int Xb = 32 * (int)m - 2;
        f4 h[4][3];
#pragma unroll
        for (int r = 0; r < 7; ++r) {
            f4 v[6];
#pragma unroll
            for (int j = 0; j < 6; ++j) v[j] = border_ld(src, (int)Y0 - 1 + r, Xb - 1 + j, Hi, Wi, C);
#pragma unroll
            for (int x = 0; x < 3; ++x)
                h[r & 3][x] = fir_h(v[x], v[x + 1], v[x + 2], v[x + 3], f0, f1, f2, f3);
            if (r >= 3) {
                const int y = r - 3;
                const uint32_t Y = Y0 + y, yb = Y & 31u;
                if (yb != 0u && yb < 30u) {
#pragma unroll
                    for (int x = 0; x < 3; ++x) {
                        const int X = Xb + x;
                        if (X < 0 || X >= (int)W2) continue;
                        border_out(a, b, Y, (uint32_t)X, c,
                                   fir_v(h[y & 3][x], h[(y + 1) & 3][x], h[(y + 2) & 3][x],
                                         h[(y + 3) & 3][x], f0, f1, f2, f3),
                                   dm, bs, sn, nw);
                    }
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

template <bool FUSE>
__global__ void __launch_bounds__(512, 1) conv_t_kernel(const ConvArgs a) {
    __shared__ f4 As[3][kTStepF4];       // weight ring [mt 4][hi,lo][64]
    __shared__ f4 Hs[2][kHaloF4];        // halo images, by channel-group parity
    __shared__ f4 Ep[FUSE ? 7 * 64 : 1]; // FUSE: the tile's epilogue operands
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t wm = wave & 1u, wn = wave >> 1;
    const uint32_t H = a.Hin, W = a.Win;
    const uint32_t nC = a.Cin / 32, nB = a.Cout / kCT, nT = a.Cout / kTCT;
    const uint32_t nbx = W / 16, nby = H / 16;
    const v4i rw = make_rsrc(a.wpk, 9u * nC * nB * kStepF4 * 16u);
    const v4i rx = make_rsrc(a.xs, a.B * H * W * a.Cin * 4);
    // tile -> 64-channel block cb, image b, block origin (y0, x0); this wave's halo
    // pieces k = wave + 8 i (per-lane source offsets at channel group 0)
    // work item = (tile, K split): the split's channel groups [cg0, cg1)
    const uint32_t ks = a.ksplit_t;
    uint32_t cb = 0, bimg = 0, y0 = 0, x0 = 0, split = 0, cg0 = 0, cg1 = 0, hoff[6];
    auto setup = [&](uint32_t item) {
        uint32_t ln = lane, wv = wave;        // opaque: computed here, not hoisted
        asm volatile("" : "+v"(ln), "+s"(wv));
        const uint32_t tile = item / ks;
        split = item - tile * ks;
        cg0 = split * nC / ks;
        cg1 = (split + 1) * nC / ks;
        cb = tile % nT;
        uint32_t blk = tile / nT;
        const uint32_t bx = blk % nbx;
        blk /= nbx;
        const uint32_t by = blk % nby, b = blk / nby;
        bimg = b;
        y0 = by * 16;
        x0 = bx * 16;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const uint32_t h = 8u * (wv + 8u * i) + (ln >> 3);
            const uint32_t hy = h / kHaloW, hx = h - hy * kHaloW;
            const uint32_t q = (ln & 7u) ^ halo_swz(hx);
            const int y = (int)(y0 + hy) - 1, x = (int)(x0 + hx) - 1;
            const bool ok = h < kHaloPx && y >= 0 && y < (int)H && x >= 0 && x < (int)W;
            hoff[i] = ok ? (((b * H + (uint32_t)y) * W + (uint32_t)x) * a.Cin * 4u + q * 16u)
                         : 0x7FFFFFF0u;
        }
    };
    uint32_t c0 = 0, c1 = 0;              // the running item's channel groups
    const uint32_t n = lane & 15u, g = lane >> 4;
    // B fragment lane bases (bytes within a halo buffer): [column offset dx + 1][lo]
    uint32_t fb0[2][2];
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
        for (int lo = 0; lo < 2; ++lo)
            fb0[d][lo] = (4u * wn * kHaloW + n) * 128u + (((2u * g + lo) ^ halo_swz(n + d)) << 4);
    const uint32_t hs0 = lds_addr(&Hs[0][0]), hs1 = lds_addr(&Hs[1][0]);

    auto uni = [](v4i r) {
        return v4i{__builtin_amdgcn_readfirstlane(r.x), __builtin_amdgcn_readfirstlane(r.y),
                   __builtin_amdgcn_readfirstlane(r.z), __builtin_amdgcn_readfirstlane(r.w)};
    };
    // weights of K-step S of group c (tap 3 ky + kx): this block's 4 m-tiles are 8 KB,
    // one 1 KB piece per wave
    auto fire_w = [&](uint32_t c, auto sc, uint32_t stage) {
        constexpr int S = decltype(sc)::value;
        constexpr uint32_t tap = 3 * t_ky(S) + t_kx(S);
        const uint32_t wsoff = __builtin_amdgcn_readfirstlane(
            ((tap * nC + c) * nB + (cb >> 1)) * kStepF4 * 16u + (cb & 1u) * kTStepF4 * 16u +
            wave * 1024u);
        set_m0(lds_addr(&As[stage][wave * 64]));
        dma16<0>(uni(rw), lane * 16u, wsoff);
    };
    uint32_t hsoff = 0;                   // soffset of the group being fetched (c * 128 B)
    auto fire_h = [&](int buf, int i) {
        set_m0(lds_addr(&Hs[buf][(wave + 8u * i) * 64]));
        dma16<0>(uni(rx), hoff[i], __builtin_amdgcn_readfirstlane(hsoff));
    };
    f4 acc[4][2][4];                      // [class 2 py + px][m-tile i][n-tile j]
    f4 Aset[2][4];                        // [hi i0, hi i1, lo i0, lo i1] by step parity
    f4 Bset[2][8];                        // [hi j0..3, lo j0..3] by position parity
    auto read_a = [&](f4 (&A)[4], uint32_t st) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            A[i] = As[st][((2 * wm + i) * 2) * 64 + lane];
            A[2 + i] = As[st][((2 * wm + i) * 2 + 1) * 64 + lane];
        }
    };
    auto read_b = [&](f4 (&Bf)[8], auto posc, uint32_t hs) {
        constexpr int pos = decltype(posc)::value;
        constexpr uint32_t dyp = (pos == 1 || pos == 3) ? 0 : 1, dxp = pos >= 2 ? 0 : 1;
        const uint32_t bh = hs + fb0[dxp][0], bl = hs + fb0[dxp][1];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t imm = ((j + dyp) * kHaloW + dxp) * 128u;
            Bf[j] = lds_f4(bh + imm);
            Bf[4 + j] = lds_f4(bl + imm);
        }
    };
    // split term t (0: lo.hi, 1: hi.lo, 2: hi.hi) of m-tile i into class cl
    auto mfma_quad = [&](auto clc, const f4 (&A)[4], const f4 (&Bf)[8], int i, int t) {
        constexpr int cl = decltype(clc)::value;
        const f4 &ra = t == 0 ? A[2 + i] : A[i];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            acc[cl][i][j] = mfma16(ra, t == 1 ? Bf[4 + j] : Bf[j], acc[cl][i][j]);
    };

    auto prologue = [&] {
        hsoff = cg0 * 128u;
#pragma unroll
        for (int i = 0; i < 6; ++i) fire_h(0, i);
        hsoff += 128u;
        fire_w(cg0, std::integral_constant<int, 0>{}, 0);
        fire_w(cg0, std::integral_constant<int, 1>{}, 1);
        fire_w(cg0, std::integral_constant<int, 2>{}, 2);
    };

    const uint32_t ntiles = a.tiles_t * ks, per = (ntiles + 7) >> 3;
    const uint32_t xcd = blockIdx.x & 7u, nwg = gridDim.x >> 3;
    const uint32_t tend = min(xcd * per + per, ntiles);
    uint32_t tile = __builtin_amdgcn_readfirstlane(xcd * per + (blockIdx.x >> 3));
    if (tile >= tend) return;
    uint32_t next = tile + nwg;
    bool has_next = next < tend;

    // K-step (c, S): MFMAs of m-tile 0; wait (in flight may stay only what step -1
    // fired: its weight piece and halo piece); barrier; read step +1's A fragments and,
    // at a position change, its B fragments; MFMAs of m-tile 1 with step +3's weight
    // piece and (S <= 5) a halo piece of group c + 1 between the split terms.  PAR:
    // parity of group c (its halo buffer and the fragment sets), compile-time.
    auto step = [&](uint32_t c, auto sc, auto parc) {
        constexpr int S = decltype(sc)::value, PAR = decltype(parc)::value;
        constexpr int cl = 2 * (t_ky(S) & 1) + (t_kx(S) & 1);
        constexpr int ka = (9 * PAR + S) & 1, kb = (4 * PAR + t_pos(S)) & 1;
        f4 (&A)[4] = Aset[ka];
        f4 (&An)[4] = Aset[ka ^ 1];
        f4 (&Bf)[8] = Bset[kb];
        f4 (&Bn)[8] = Bset[kb ^ 1];
        const auto CL = std::integral_constant<int, cl>{};
        const uint32_t k = (c - c0) * 9 + S, nk = (c1 - c0) * 9;
        const bool prev_w = k + 2 < nk;
        const bool prev_h = S != 0 && S - 1 <= 5 && c + 1 < c1;
        mfma_quad(CL, A, Bf, 0, 0);
        mfma_quad(CL, A, Bf, 0, 1);
        mfma_quad(CL, A, Bf, 0, 2);
        if (prev_w && prev_h) asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
        else if (prev_w || prev_h) asm volatile("s_waitcnt vmcnt(1) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        if constexpr (!(kTAbl & 2)) __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        read_a(An, (S + 1) % 3);
        if constexpr (S == 3 || S == 5 || S == 7)
            read_b(Bn, std::integral_constant<int, t_pos(S + 1)>{}, PAR ? hs1 : hs0);
        else if constexpr (S == 8)
            read_b(Bn, std::integral_constant<int, 0>{}, PAR ? hs0 : hs1);
        mfma_quad(CL, A, Bf, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (!(kTAbl & 4) && k + 3 < nk)
            fire_w(c + (S + 3) / 9, std::integral_constant<int, (S + 3) % 9>{}, S % 3);
        __builtin_amdgcn_sched_barrier(0);
        mfma_quad(CL, A, Bf, 1, 1);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (S <= 5 && !(kTAbl & 8)) {
            if (c + 1 < c1) fire_h(1 - PAR, S);
        }
        if constexpr (S == 8) {
            if (k + 1 == nk && has_next) {
                setup(next);
                prologue();
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        mfma_quad(CL, A, Bf, 1, 2);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto group = [&](uint32_t c, auto parc) {
        step(c, std::integral_constant<int, 0>{}, parc);
        step(c, std::integral_constant<int, 1>{}, parc);
        step(c, std::integral_constant<int, 2>{}, parc);
        step(c, std::integral_constant<int, 3>{}, parc);
        step(c, std::integral_constant<int, 4>{}, parc);
        step(c, std::integral_constant<int, 5>{}, parc);
        hsoff += 128u;
        step(c, std::integral_constant<int, 6>{}, parc);
        step(c, std::integral_constant<int, 7>{}, parc);
        step(c, std::integral_constant<int, 8>{}, parc);
    };

    setup(tile);
    prologue();
    bool first = true;
    for (;;) {
        const uint32_t ecb = cb, eb = bimg, ey0 = y0, ex0 = x0, esp = split;  // (setup moves on)
        c0 = cg0;
        c1 = cg1;
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[q][i][j] = f4{0.0f, 0.0f, 0.0f, 0.0f};
        // everything but step 2's weight piece (and, after the first tile, the previous
        // epilogue's 32 stores, younger than this tile's prologue) has landed; the
        // epilogue reads no LDS.  FUSE: its stores and loads vary per lane -- wait for
        // them all (as conv_h_kernel); its LDS exchange is done everywhere after the barrier.
        // FUSE: the tile's epilogue operands, one 1 KB piece per wave 0-6 -- demod, bias,
        // s_next (the block's 64 channels in lanes 0-15), the noise of its 32 x 32 output
        // pixels (8 rows per wave) -- loaded here, where the wait below drains the
        // previous epilogue's stores anyway, and written to Ep behind the barrier
        f4 epv = {0.0f, 0.0f, 0.0f, 0.0f};
        if constexpr (FUSE) {
            const ActEpi &e = a.e;
            const uint32_t ln = lane;
            const uint32_t ch = cb * kTCT + 4u * (ln & 15u);
            const bool lo = ln < 16u;
            const f4 *src = nullptr;
            if (wave == 0) src = lo ? reinterpret_cast<const f4 *>(e.demod + (size_t)bimg * a.Cout + ch) : nullptr;
            else if (wave == 1) src = lo ? reinterpret_cast<const f4 *>(e.bias + ch) : nullptr;
            else if (wave == 2) src = lo && e.s_next ? reinterpret_cast<const f4 *>(e.s_next + (size_t)bimg * a.Cout + ch) : nullptr;
            else if (wave < 7 && e.noise)
                src = reinterpret_cast<const f4 *>(
                    e.noise + ((size_t)bimg * 2u * H + 2u * y0 + 8u * (wave - 3u) + (ln >> 3)) * 2u * W +
                    2u * x0 + 4u * (ln & 7u));
            if (src) epv = *src;
            else if (wave == 2) epv = f4{1.0f, 1.0f, 1.0f, 1.0f};
        }
        if (first && !FUSE) asm volatile("s_waitcnt vmcnt(1) lgkmcnt(0)" ::: "memory");
#ifdef SDFR_TVAR
        else if (FUSE && SDFR_TVAR == 1 && !first) asm volatile("s_waitcnt vmcnt(40) lgkmcnt(0)" ::: "memory");
#endif
        else if (FUSE) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(33) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if constexpr (FUSE) {
            if (wave < 7) Ep[wave * 64 + lane] = epv;
        }
        read_a(Aset[0], 0);
        read_b(Bset[0], std::integral_constant<int, 0>{}, hs0);
        uint32_t c = c0;
        for (; c + 1 < c1; c += 2) {
            group(c, std::integral_constant<int, 0>{});
            group(c + 1, std::integral_constant<int, 1>{});
        }
        if (c < c1) group(c, std::integral_constant<int, 0>{});
        if constexpr (FUSE) {
            conv_t_blur_epilogue(a, acc, Ep, &Hs[1][0], lane, wave, ecb, eb, ey0, ex0);
        } else {   // raw fp32 outputs of the four classes
            uint32_t ln = lane, wmm = wm, wnn = wn;   // opaque: nothing hoisted into the K loop
            asm volatile("" : "+v"(ln), "+s"(wmm), "+s"(wnn));
            const uint32_t nn = ln & 15u, gg = ln >> 4;
            const uint32_t Wf = a.Wf, C = a.Cout;
            // (a K split writes its partial output; conv_t_finish_kernel sums them)
            float *base = (ks > 1 ? a.ptl + (size_t)esp * a.B * a.Hf * Wf * C : a.out) + ecb * kTCT +
                          4u * gg;
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t oy = 2u * (ey0 + 4u * wnn + j) + (uint32_t)(q >> 1);
                    const uint32_t ox = 2u * (ex0 + nn) + (uint32_t)(q & 1);
                    float *dst = base + ((size_t)(eb * a.Hf + oy) * Wf + ox) * C;
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        if constexpr (kTAbl & 1) {
                            if (acc[q][i][j][0] == 1.2345e-33f)
                                *reinterpret_cast<f4 *>(dst + (2u * wmm + i) * 16u) = acc[q][i][j];
                        } else {
                            *reinterpret_cast<f4 *>(dst + (2u * wmm + i) * 16u) = acc[q][i][j];
                        }
                    }
                }
        }
        if (!has_next) break;
        tile = next;
        next = tile + nwg;
        has_next = next < tend;
        first = false;
    }
}


}  // namespace
}  // namespace sdfr

using namespace sdfr;

extern "C" {

size_t sdfr_conv_pack_bytes(uint32_t Cout, uint32_t Cin) {
    return (size_t)9 * Cin * Cout * 2 * sizeof(_Float16) + (size_t)Cout * sizeof(float);
}

int sdfr_conv_pack_weights(const float *w, float scale, uint32_t Cout, uint32_t Cin,
                           void *packed, float *su, void *stream) {
    if (!w || !packed || !su) return fail(SDFR_EINVAL, "conv_pack_weights: null pointer");
    if (Cout == 0 || Cout % kCT || Cin == 0 || Cin % 32)
        return fail(SDFR_EINVAL, "conv_pack_weights: Cout % 128 and Cin % 32 must be 0");
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(conv_scale_kernel, dim3(Cout), dim3(256), 0, st, w, scale, Cin, su);
    int rc = check_launch("conv_pack_weights: scale");
    if (rc) return rc;
    const uint32_t total = 9 * (Cin / 32) * (Cout / kCT) * 8 * 64;
    hipLaunchKernelGGL(conv_pack_kernel, dim3((total + 255) / 256), dim3(256), 0, st, w, scale,
                       Cin, Cout, su, reinterpret_cast<f4 *>(packed));
    return check_launch("conv_pack_weights: pack");
}

}  // extern "C"

namespace {

// Shared setup of both entry points: shape checks, tap tables, classes; launches
// conv_x_kernel<ACT>.
// split-K factor: the largest of 4, 3, 2 that keeps the split grid within ~1.25 rounds
// of workgroups on the 256 CUs (one 512-thread workgroup per CU).  The 1.25: the
// batch-1 64 -> 128 transposed conv (136 workgroups, four unequal parity classes)
// measured 82 -> 66 us with a 2-way split over 272 (a one-round bound leaves it unsplit);
// 384 made the regular convs' 3-way splits slower.
#ifndef SDFR_KSPLIT_MAX
#define SDFR_KSPLIT_MAX 320
#endif
uint32_t conv_ksplit(uint32_t grid) {
    for (uint32_t k = 4; k > 1; --k)
        if (grid * k <= SDFR_KSPLIT_MAX) return k;
    return 1;
}

// conv_t_kernel's K-split finish: out = sum of the ksplit_t partials, in split order
// (deterministic), for every output row / column < 2H, 2W (the edge classes write theirs)
__global__ void __launch_bounds__(256) conv_t_finish_kernel(const ConvArgs a) {
    const uint32_t C4 = a.Cout / 4, W2 = 2 * a.Win, H2 = 2 * a.Hin;
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (uint64_t)a.B * H2 * W2 * C4) return;
    const uint32_t q = (uint32_t)(t % C4);
    uint64_t r = t / C4;
    const uint32_t ox = (uint32_t)(r % W2);
    r /= W2;
    const uint32_t oy = (uint32_t)(r % H2), b = (uint32_t)(r / H2);
    const size_t idx = (((size_t)b * a.Hf + oy) * a.Wf + ox) * a.Cout + 4 * q;
    const size_t stride = (size_t)a.B * a.Hf * a.Wf * a.Cout;
    f4 v = *reinterpret_cast<const f4 *>(a.ptl + idx);
    for (uint32_t k = 1; k < a.ksplit_t; ++k) v += *reinterpret_cast<const f4 *>(a.ptl + k * stride + idx);
    *reinterpret_cast<f4 *>(a.out + idx) = v;
}

// The transposed conv on conv_t_kernel (+ its edge classes): raw output, 16-aligned
// input, and at least one tile per CU (smaller batches keep conv_x_kernel's split-K).
// The mode (sdfr_set_conv_t_mode, SDFR_CONV_T): 0 selects conv_x_kernel (A/B measurements), 2 takes
// conv_t_kernel at any tile count (tests), 3 also splits each tile's channel groups 2 or 4
// ways below 256 tiles (*ks) when the caller's workspace holds the partial outputs
// (has_ws; sdfr_conv_ws_bytes sizes it).
// The mode (sdfr_set_conv_t_mode): SDFR_CONV_T read once when the library loads.
int conv_t_env_mode() {
    const char *e = getenv("SDFR_CONV_T");
    return e ? atoi(e) : 1;
}
int g_conv_t_mode = conv_t_env_mode();

bool use_conv_t(bool act, uint32_t B, uint32_t H, uint32_t W, uint32_t Cin, uint32_t Cout,
                bool has_ws, uint32_t *ks) {
    const int env = g_conv_t_mode;
    *ks = 1;
    if (env == 0 || act || H % 16 || W % 16 || Cout % kTCT) return false;
    const uint32_t tiles = B * (H / 16) * (W / 16) * (Cout / kTCT), nC = Cin / 32;
    if (tiles >= 256) return true;
    // (the K split -- env 3 -- measured slower than conv_x_kernel's split-K at one face:
    // its thin edge-class launch alone is a 29 us serial chain there)
    if (has_ws && env == 3)
        for (uint32_t k = 4; k > 1; k /= 2)
            if (tiles * k <= 256 && nC >= 2 * k) {
                *ks = k;
                return true;
            }
    return env >= 2;
}

// the partial outputs of conv_t_kernel's K split (for any Cin: an upper bound)
size_t conv_t_ws_bytes(uint32_t B, uint32_t H, uint32_t W, uint32_t Cout) {
    if (g_conv_t_mode != 3) return 0;
    uint32_t ks = 1;
    const uint32_t tiles = B * (H / 16) * (W / 16) * (Cout / kTCT);
    if (H % 16 || W % 16 || Cout % kTCT || tiles >= 256) return 0;
    for (uint32_t k = 4; k > 1 && ks == 1; k /= 2)
        if (tiles * k <= 256) ks = k;
    if (ks == 1) return 0;
    return (size_t)ks * B * (2 * H + 1) * (2 * W + 1) * Cout * sizeof(float);
}

// conv_t_kernel's four edge classes (row 2H: W + 1 and W pixels, column 2W: H and H
// pixels per face) as conv_x_kernel workgroup slots, and their split-K factor
// (SDFR_EDGE_SPLIT=1): ~70 thin tiles of a full-K loop at 32 faces leave most CUs
// idle, but the 4-way split measured 27 + 16 us per launch in the bench trace against
// 36 unsplit (the finish pass costs what the split saves), so it is off
#ifndef SDFR_EDGE_SPLIT
#define SDFR_EDGE_SPLIT 0
#endif
uint32_t conv_edge_grid(uint32_t B, uint32_t H, uint32_t W, uint32_t Cout) {
    uint32_t g = 0;
    for (uint32_t n : {W + 1, W, H, H}) g += ((B * n + kPT - 1) / kPT * (Cout / kCT) + 7) & ~7u;
    return g;
}
size_t conv_edge_ws_bytes(uint32_t B, uint32_t H, uint32_t W, uint32_t Cout) {
    if (!SDFR_EDGE_SPLIT || H % 16 || W % 16 || Cout % kCT) return 0;
    if (B * (H / 16) * (W / 16) * (Cout / kTCT) < 256) return 0;    // no conv_t_kernel (use_conv_t)
    const uint32_t g = conv_edge_grid(B, H, W, Cout), ks = conv_ksplit(g);
    return ks > 1 ? (size_t)ks * g * 16 * 512 * sizeof(f4) : 0;
}

uint32_t conv_grid(uint32_t B, uint32_t H, uint32_t W, uint32_t Cout) {   // regular conv
    return ((B * H * W + kPT - 1) / kPT * (Cout / kCT) + 7) & ~7u;
}

uint32_t conv_grid_t(uint32_t B, uint32_t H, uint32_t W, uint32_t Cout) {  // transposed (4 classes)
    uint32_t g = 0;
    for (uint32_t py = 0; py < 2; ++py)
        for (uint32_t px = 0; px < 2; ++px)
            g += ((B * (py ? H : H + 1) * (px ? W : W + 1) + kPT - 1) / kPT * (Cout / kCT) + 7) & ~7u;
    return g;
}

int conv_launch(ConvArgs &a, const void *x_split, const void *packed, uint32_t B, uint32_t H,
                uint32_t W, uint32_t Cin, uint32_t Cout, int transposed, bool act,
                hipStream_t st, const char *what, void *ws = nullptr, size_t ws_bytes = 0,
                bool fuse_t = false) {
    if (!x_split || !packed) return fail(SDFR_EINVAL, "conv3x3_f16x3: null pointer");
    if (B == 0 || H == 0 || W == 0 || Cout % kCT || Cin % 32 || Cin == 0 || Cout == 0)
        return fail(SDFR_EINVAL, "conv3x3_f16x3: bad shape (Cout % 128, Cin % 32)");
    if ((uint64_t)B * H * W * Cin * 4 >= (1ull << 31) || 9ull * Cin * Cout * 4 >= (1ull << 31) ||
        (uint64_t)B * H * W * Cout * 4 >= (1ull << 31))
        return fail(SDFR_EINVAL, "conv3x3_f16x3: tensor too large for 32-bit offsets (split B)");
    a.xs = reinterpret_cast<const _Float16 *>(x_split);
    a.wpk = reinterpret_cast<const f4 *>(packed);
    a.B = B;
    a.Hin = H;
    a.Win = W;
    a.Cin = Cin;
    a.Cout = Cout;
    // classes (heaviest first) -> contiguous workgroup ranges padded to multiples of 8
    uint32_t grid = 0, ntap = 0;
    auto add_class = [&](uint32_t Hc, uint32_t Wc, uint32_t py, uint32_t px, uint32_t nt,
                         uint32_t a0 = 0, uint32_t c0 = 0) {
        ConvClass &c = a.cls[a.ncls++];
        c.Hc = Hc;
        c.Wc = Wc;
        c.py = py;
        c.px = px;
        c.a0 = a0;
        c.c0 = c0;
        c.t0 = ntap - nt;
        c.ntaps = nt;
        c.tile0 = grid;
        c.ntiles = (B * Hc * Wc + kPT - 1) / kPT * (Cout / kCT);
        grid += (c.ntiles + 7) & ~7u;
        for (uint32_t t = 0; t < nt; ++t) {
            const uint32_t d = a.tap[c.t0 + t] | (uint32_t)(a.dy[c.t0 + t] + 1) << 4 |
                               (uint32_t)(a.dx[c.t0 + t] + 1) << 6;
            c.td[t >> 2] |= d << (8 * (t & 3u));
        }
    };
    if (!transposed) {
        a.Hf = H;
        a.Wf = W;
        a.sy = 1;
        for (int t = 0; t < 9; ++t) {
            a.dy[t] = t / 3 - 1;
            a.dx[t] = t % 3 - 1;
            a.tap[t] = t;
        }
        ntap = 9;
        add_class(H, W, 0, 0, 9);
    } else {
        // conv_transpose2d, stride 2: out (2a + ky, 2c + kx) <- x (a, c).  Parity class
        // (py, px): output (2a' + py, 2c' + px) takes ky in {0, 2} (py = 0, input row
        // a' - ky/2) or ky = 1 (py = 1, input row a'), likewise for x.
        a.Hf = 2 * H + 1;
        a.Wf = 2 * W + 1;
        a.sy = 2;
        uint32_t kst = 1;
        if (use_conv_t(act, B, H, W, Cin, Cout,
                       !fuse_t && ws != nullptr && ws_bytes >= conv_t_ws_bytes(B, H, W, Cout),
                       &kst)) {
            // conv_t_kernel: every output row / column < 2H, 2W; here the last row
            // (even classes at a = H: only the ky = 2 taps reach it) and column as four
            // thin classes of conv_x_kernel
            auto tap = [&](int ky, int kx) {
                a.dy[ntap] = -(ky >> 1);
                a.dx[ntap] = -(kx >> 1);
                a.tap[ntap] = (uint32_t)(ky * 3 + kx);
                ++ntap;
            };
            tap(2, 0), tap(2, 2);
            add_class(1, W + 1, 0, 0, 2, H, 0);       // row 2H, even columns
            tap(2, 1);
            add_class(1, W, 0, 1, 1, H, 0);           // row 2H, odd columns
            tap(0, 2), tap(2, 2);
            add_class(H, 1, 0, 0, 2, 0, W);           // column 2W, even rows < 2H
            tap(1, 2);
            add_class(H, 1, 1, 0, 1, 0, W);           // column 2W, odd rows
            a.grid = grid;
            a.ksplit = 1;
            a.partial = nullptr;
            a.tiles_t = B * (H / 16) * (W / 16) * (Cout / kTCT);
            a.ksplit_t = kst;
            a.ptl = kst > 1 ? reinterpret_cast<float *>(ws) : nullptr;
            if (fuse_t) hipLaunchKernelGGL(conv_t_kernel<true>, dim3(conv_h_grid(a.tiles_t)), dim3(512), 0, st, a);
            else hipLaunchKernelGGL(conv_t_kernel<false>, dim3(conv_h_grid(a.tiles_t * kst)), dim3(512), 0, st, a);
            int rc = check_launch(what);
            if (rc) return rc;
            if (kst > 1) {
                const uint64_t n4 = (uint64_t)B * 4 * H * W * (Cout / 4);
                hipLaunchKernelGGL(conv_t_finish_kernel, dim3((uint32_t)((n4 + 255) / 256)), dim3(256),
                                   0, st, a);
                if ((rc = check_launch(what))) return rc;
            }
            // the edge classes: ~70 thin tiles at B = 32, each a full-K loop, split-K
            // over up to 1.25 rounds of the chip when the workspace allows (the conv_t
            // K-split partials, if any, are consumed by the finish kernel above)
            a.grid = grid;
            const uint32_t eks = conv_ksplit(grid);
            if (SDFR_EDGE_SPLIT && ws && eks > 1 && kst == 1 &&
                ws_bytes >= (size_t)eks * grid * 16 * 512 * sizeof(f4)) {
                a.ksplit = eks;
                a.partial = reinterpret_cast<f4 *>(ws);
            }
            hipLaunchKernelGGL(conv_x_kernel<false>, dim3(grid, a.ksplit), dim3(512), 0, st, a);
            if (a.ksplit > 1) {
                if ((rc = check_launch(what))) return rc;
                hipLaunchKernelGGL(conv_splitk_kernel<false>, dim3(grid), dim3(512), 0, st, a);
            }
            if (fuse_t) {        // the blocks' border pixels, after the edge classes
                if ((rc = check_launch(what))) return rc;
                const uint32_t H2 = 2u * H, W2 = 2u * W;
                const uint64_t nr = (uint64_t)B * (H2 / 32u + 1u) * (W2 / 4u) * (Cout / 4u);
                const uint64_t nc = (uint64_t)B * (H2 / 4u) * (W2 / 32u + 1u) * (Cout / 4u);
                hipLaunchKernelGGL(conv_t_border_kernel<true>, dim3((uint32_t)((nr + 255) / 256)),
                                   dim3(256), 0, st, a);
                if ((rc = check_launch(what))) return rc;
                hipLaunchKernelGGL(conv_t_border_kernel<false>, dim3((uint32_t)((nc + 255) / 256)),
                                   dim3(256), 0, st, a);
            }
            return check_launch(what);
        }
        if (fuse_t) return fail(SDFR_EUNSUPPORTED, "conv_t_act: shape below conv_t_kernel's range");
        for (uint32_t py = 0; py < 2; ++py)
            for (uint32_t px = 0; px < 2; ++px) {
                uint32_t nt = 0;
                for (int ky = (int)py; ky < 3; ky += 2)
                    for (int kx = (int)px; kx < 3; kx += 2) {
                        a.dy[ntap] = -(ky >> 1);
                        a.dx[ntap] = -(kx >> 1);
                        a.tap[ntap] = (uint32_t)(ky * 3 + kx);
                        ++ntap;
                        ++nt;
                    }
                add_class(py ? H : H + 1, px ? W : W + 1, py, px, nt);
            }
    }
    a.grid = grid;
    a.ksplit = 1;
    a.partial = nullptr;
    const uint32_t ks = conv_ksplit(grid);
    if (ws && ks > 1 && ws_bytes >= (size_t)ks * grid * 16 * 512 * sizeof(f4)) {
        a.ksplit = ks;
        a.partial = reinterpret_cast<f4 *>(ws);
    }
    // the fused regular conv on conv_h_kernel; its K split (whole channel groups: the
    // same K ranges as conv_x_kernel's split-K when nC % ks == 0) at small batches
    if (act && !transposed && H % 16 == 0 && W % 16 == 0 &&
        (a.ksplit == 1 || kHSplit)) {
        // its split takes whole channel groups: the largest factor <= conv_ksplit's that
        // divides the group count
        while (a.ksplit > 1 && (Cin / 32) % a.ksplit) --a.ksplit;
        const uint32_t nt = a.cls[0].ntiles;
        if (a.ksplit > 1) {
            hipLaunchKernelGGL(conv_h_kernel<true>, dim3(conv_h_grid(nt * a.ksplit)), dim3(512), 0, st, a);
            int rc = check_launch(what);
            if (rc) return rc;
            hipLaunchKernelGGL(conv_h_finish_kernel, dim3(nt, 4), dim3(128), 0, st, a);
        } else {
            hipLaunchKernelGGL(conv_h_kernel<false>, dim3(conv_h_grid(nt)), dim3(512), 0, st, a);
        }
        return check_launch(what);
    }
    if (act) hipLaunchKernelGGL(conv_x_kernel<true>, dim3(grid, a.ksplit), dim3(512), 0, st, a);
    else hipLaunchKernelGGL(conv_x_kernel<false>, dim3(grid, a.ksplit), dim3(512), 0, st, a);
    if (a.ksplit > 1) {
        if (act) hipLaunchKernelGGL(conv_splitk_kernel<true>, dim3(grid), dim3(512), 0, st, a);
        else hipLaunchKernelGGL(conv_splitk_kernel<false>, dim3(grid), dim3(512), 0, st, a);
    }
    return check_launch(what);
}

}  // namespace

extern "C" {

int sdfr_conv3x3_f16x3_ws(float *out, const void *x_split, const void *packed,
                          uint32_t B, uint32_t H, uint32_t W, uint32_t Cin, uint32_t Cout,
                          int transposed, void *ws, size_t ws_bytes, void *stream) {
    if (!out) return fail(SDFR_EINVAL, "conv3x3_f16x3: null pointer");
    ConvArgs a{};
    a.out = out;
    return conv_launch(a, x_split, packed, B, H, W, Cin, Cout, transposed, false,
                       (hipStream_t)stream, "conv3x3_f16x3", ws, ws_bytes);
}

int sdfr_conv3x3_f16x3(float *out, const void *x_split, const void *packed,
                       uint32_t B, uint32_t H, uint32_t W, uint32_t Cin, uint32_t Cout,
                       int transposed, void *stream) {
    return sdfr_conv3x3_f16x3_ws(out, x_split, packed, B, H, W, Cin, Cout, transposed, nullptr, 0,
                                 stream);
}

int sdfr_set_conv_t_mode(int mode) {
    if (mode < -1 || mode > 3) return fail(SDFR_EINVAL, "set_conv_t_mode: mode must be -1..3");
    const int prev = g_conv_t_mode;
    g_conv_t_mode = mode == -1 ? conv_t_env_mode() : mode;
    return prev;
}

size_t sdfr_conv_ws_bytes(uint32_t B, uint32_t H, uint32_t W, uint32_t Cout, int transposed) {
    if (Cout % kCT || B == 0 || H == 0 || W == 0) return 0;
    const uint32_t grid = transposed ? conv_grid_t(B, H, W, Cout) : conv_grid(B, H, W, Cout);
    const uint32_t ks = conv_ksplit(grid);
    const size_t strip = ks > 1 ? (size_t)ks * grid * 16 * 512 * sizeof(f4) : 0;
    size_t tk = transposed ? conv_t_ws_bytes(B, H, W, Cout) : 0;
    if (transposed) {
        const size_t te = conv_edge_ws_bytes(B, H, W, Cout);
        tk = tk > te ? tk : te;
    }
    return strip > tk ? strip : tk;
}

int sdfr_conv3x3_f16x3_act(const sdfr_conv_act_args *p, void *stream) {
    if (!p) return fail(SDFR_EINVAL, "conv3x3_f16x3_act: null args");
    const sdfr_conv_act_args &s = *p;
    if (!s.demod || !s.bias || (s.noise && !s.noise_weight))
        return fail(SDFR_EINVAL, "conv3x3_f16x3_act: null tensor pointer");
    const bool rgb = s.rgb_w || s.rgb_base;
    if (s.rgb_w && s.rgb_base) return fail(SDFR_EINVAL, "conv3x3_f16x3_act: rgb_w and rgb_base are exclusive");
    if (s.rgb_base && !s.rgb_s) return fail(SDFR_EINVAL, "conv3x3_f16x3_act: rgb_base needs rgb_s");
    if (!s.y_split && !rgb) return fail(SDFR_EINVAL, "conv3x3_f16x3_act: nothing to write");
    if (rgb && !s.rgb_partial) return fail(SDFR_EINVAL, "conv3x3_f16x3_act: rgb_partial missing");
    if (((uint64_t)s.H * s.W) % kPT)
        return fail(SDFR_EUNSUPPORTED, "conv3x3_f16x3_act: H*W must be a multiple of 256");
    for (const void *q : {(const void *)s.demod, (const void *)s.bias, (const void *)s.s_next,
                          (const void *)s.rgb_w, (const void *)s.y_split, (const void *)s.rgb_base,
                          (const void *)s.rgb_s})
        if (q && reinterpret_cast<uintptr_t>(q) % 16)
            return fail(SDFR_EINVAL, "conv3x3_f16x3_act: pointers must be 16-B aligned");
    ConvArgs a{};
    a.e.demod = s.demod;
    a.e.noise = s.noise;
    a.e.noise_weight = s.noise_weight;
    a.e.bias = s.bias;
    a.e.slope = s.negative_slope;
    a.e.scale = s.act_scale;
    a.e.s_next = s.s_next;
    a.e.ys = reinterpret_cast<_Float16 *>(s.y_split);
    a.e.rgb_w = s.rgb_w;
    a.e.rgbp = s.rgb_partial;
    a.e.rgb_base = s.rgb_base;
    a.e.rgb_s = s.rgb_s;
    return conv_launch(a, s.x_split, s.packed, s.B, s.H, s.W, s.Cin, s.Cout, 0, true,
                       (hipStream_t)stream, "conv3x3_f16x3_act", s.ws, s.ws_bytes);
}

int sdfr_conv_t_act_supported(uint32_t B, uint32_t H, uint32_t W, uint32_t Cin, uint32_t Cout) {
    uint32_t ks = 1;
    return B && H && W && Cin && Cin % 32 == 0 && Cout % kCT == 0 &&
           use_conv_t(false, B, H, W, Cin, Cout, false, &ks) && ks == 1;
}

int sdfr_conv_t_act(const sdfr_conv_t_act_args *p, void *stream) {
    if (!p) return fail(SDFR_EINVAL, "conv_t_act: null args");
    const sdfr_conv_t_act_args &s = *p;
    if (!s.demod || !s.bias || !s.y_split || !s.raw || (s.noise && !s.noise_weight))
        return fail(SDFR_EINVAL, "conv_t_act: null tensor pointer");
    for (const void *q : {(const void *)s.demod, (const void *)s.bias, (const void *)s.s_next,
                          (const void *)s.y_split, (const void *)s.raw})
        if (q && reinterpret_cast<uintptr_t>(q) % 16)
            return fail(SDFR_EINVAL, "conv_t_act: pointers must be 16-B aligned");
    if (!sdfr_conv_t_act_supported(s.B, s.H, s.W, s.Cin, s.Cout))
        return fail(SDFR_EUNSUPPORTED, "conv_t_act: shape below conv_t_kernel's range "
                                       "(sdfr_conv_t_act_supported)");
    if ((uint64_t)s.B * (2 * s.H + 1) * (2 * s.W + 1) * s.Cout * 4 >= (1ull << 31))
        return fail(SDFR_EINVAL, "conv_t_act: tensor too large for 32-bit offsets (split B)");
    ConvArgs a{};
    a.out = s.raw;
    a.e.demod = s.demod;
    a.e.noise = s.noise;
    a.e.noise_weight = s.noise_weight;
    a.e.bias = s.bias;
    a.e.slope = s.negative_slope;
    a.e.scale = s.act_scale;
    a.e.s_next = s.s_next;
    a.e.ys = reinterpret_cast<_Float16 *>(s.y_split);
    for (int k = 0; k < 4; ++k) a.fir[k] = s.fir[k];
    return conv_launch(a, s.x_split, s.packed, s.B, s.H, s.W, s.Cin, s.Cout, 1, false,
                       (hipStream_t)stream, "conv_t_act", nullptr, 0, true);
}

size_t sdfr_conv_act_ws_bytes(uint32_t B, uint32_t H, uint32_t W, uint32_t Cout) {
    if (Cout % kCT || B == 0 || H == 0 || W == 0) return 0;
    const uint32_t grid = conv_grid(B, H, W, Cout), ks = conv_ksplit(grid);
    return ks > 1 ? (size_t)ks * grid * 16 * 512 * sizeof(f4) : 0;
}

}  // extern "C"
