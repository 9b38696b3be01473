// linear_f16x3.hip -- the renderer MLP's linear layers for TRAINING (stage 1,
// training_utils.py:396-451): when the renderer needs gradients the reference runs
// NGPSIRENGenerator / SirenGenerator op by op (sdf_model.py:1566-1592, 44-69, 23-41),
// i.e. F.linear over S = chunk x 64^2 x 24 = 196,608 samples at a time, and its
// backward.  Those three GEMM shapes run here on split-fp16 MFMA at fp32-level
// accuracy (f16x3.h), instead of rocBLAS's fp32 GEMMs:
//
//   sdfr_linear_f16x3        out[M,N] = x[M,K] . B[N,K]^T (+ bias[N])
//                            forward (B = W) and input gradient (B = W^T, no bias)
//   sdfr_linear_wgrad_f16x3  gw[N,K] = sum_m dy[m,n] x[m,k]   (weight gradient)
//
// Forward / input gradient: a workgroup is 8 waves over 128 rows of x (32 per wave:
// two MFMA N = 16 columns = rows m of x; two waves per row group, one half of the
// output tiles each); x tiles and the B fragments (pre-split, row-scaled by su[n],
// packed in MFMA A-fragment order by sdfr_linear_pack) stream through a 3-slot LDS
// ring by LDS-DMA; each row of x is scaled by a power of two from its running maximum
// (max |x_m| into [0.5, 1): the fp16 lo parts stay normal at any magnitude,
// activations and gradients alike; accumulators are rescaled exactly when a row's
// scale shrinks) and split per k-step.  Outputs accumulate in fp32 and are unscaled
// exactly.
//
// Weight gradient: the sum over m is split over workgroups (a contiguous range of
// rows each), each accumulating an [N,K] partial in fp32; a second kernel adds the
// partials in a fixed order (deterministic).  Every column of dy and of x is scaled
// by a power of two from its running maximum over the workgroup's rows (the
// accumulators are rescaled exactly when a scale shrinks), so the operands are read
// once.  Per m-step of 32 rows both operands are staged into LDS as split-fp16 MFMA
// fragments.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <type_traits>

#include "f16x3.h"
#include "render_ngp.h"
#include "sdfr_common.h"

namespace sdfr {
namespace {

// cos as sin_hw (render_ngp.h): 2 pi reduction by fma, then v_cos_f32 (revolutions)
__device__ __forceinline__ float cos_hw(float x) {
    constexpr float c_hi = 0.15915493667125702f;    // fl(1/(2pi))
    constexpr float c_lo = 6.4206382432985265e-09f;  // 1/(2pi) - c_hi
    const float k = __builtin_rintf(x * c_hi);
    float f = __fmaf_rn(x, c_hi, -k);
    f = __fmaf_rn(x, c_lo, f);
    return __builtin_amdgcn_cosf(f);
}

constexpr uint32_t kLinWaves = 8;
constexpr uint32_t kLinThreads = kLinWaves * 64;
constexpr uint32_t kLinRows = 256;                     // rows of x per forward block (32 per wave)
constexpr uint32_t kTileF4 = 128;                      // one 16-row tile: [hi,lo][64 lanes]

__host__ __device__ constexpr uint32_t ceil_div(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

// power of two s with max |.| * s in [0.5, 1) (1 for zero / non-finite maxima)
__device__ __forceinline__ float pow2_scale(float m) {
    if (!(m > 0.0f && m < 3.0e38f)) return 1.0f;
    int ex = __builtin_amdgcn_frexp_expf(m);
    ex = ex < -100 ? -100 : (ex > 100 ? 100 : ex);
    return __builtin_ldexpf(1.0f, -ex);
}

// ----------------------------------------------------------------------------
// packing: B [N,K] (or W [K,N] read transposed) -> su [N] and fragments
// [ks][nt][hi,lo][lane], lane (r = lane & 15, g = lane >> 4) holding
// B[16 nt + r][32 ks + 8 g + j] * su, j = 0..7 (zero past N / K)
// ----------------------------------------------------------------------------
__device__ __forceinline__ float bval(const float *w, uint32_t N, uint32_t K, int tr, uint32_t n,
                                      uint32_t k) {
    if (n >= N || k >= K) return 0.0f;
    return tr ? w[(size_t)k * N + n] : w[(size_t)n * K + k];
}

__global__ void __launch_bounds__(256) lin_scale_kernel(const float *__restrict__ w, uint32_t N,
                                                        uint32_t K, int tr, float *__restrict__ su) {
    const uint32_t n = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    float m = 0.0f;
    if (n < N)
        for (uint32_t k = lane; k < K; k += 64) m = fmaxf(m, fabsf(bval(w, N, K, tr, n, k)));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (lane == 0 && n < N) su[n] = pow2_scale(m);
}

__global__ void __launch_bounds__(256) lin_pack_kernel(const float *__restrict__ w, uint32_t N,
                                                       uint32_t K, int tr,
                                                       const float *__restrict__ su,
                                                       f4 *__restrict__ packed) {
    const uint32_t NT = ceil_div(N, 16), KS = ceil_div(K, 32);
    const uint32_t e = blockIdx.x * 256 + threadIdx.x;     // (ks, nt, lane)
    if (e >= KS * NT * 64) return;
    const uint32_t lane = e & 63u, nt = (e >> 6) % NT, ks = (e >> 6) / NT;
    const uint32_t n = 16 * nt + (lane & 15u), g = lane >> 4;
    const float s = n < N ? su[n] : 1.0f;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = __fmul_rn(bval(w, N, K, tr, n, 32 * ks + 8 * g + j), s);
    f4 hi, lo;
    split8(v, hi, lo);
    f4 *dst = packed + ((size_t)ks * NT + nt) * kTileF4 + lane;
    dst[0] = hi;
    dst[64] = lo;
}

// ----------------------------------------------------------------------------
// out = x . B^T (+ bias): NT output tiles of 16, KS k-steps of 32
// ----------------------------------------------------------------------------
struct LinArgs {
    const float *x;            // [M, K]
    const f4 *packed;          // [KS][NT][128]
    const float *su;           // [N]
    const float *bias;         // [N] or null
    float *out;                // [M, N]
    uint32_t M, N, K;
    // FiLM epilogue (FILM kernels): out = sin(gamma[f] * y + beta[f]), y = x B^T + bias
    // saved to y_save; f = m / rows_per_face
    const float *gamma, *beta; // [F, N]
    float *y_save;             // [M, N]
    uint32_t rows_per_face;
};

// a buffer resource over `bytes` bytes at `base`: loads past the end return zeros
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void *base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)bytes,
                                             0x00020000);
}
constexpr uint32_t kOob = 0x80000000u;                  // a buffer offset that reads zeros

__device__ __forceinline__ float ld1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}

// output tiles per workgroup (the weights of one split stay resident in LDS) and splits
template <int NT>
constexpr int fwd_ntw() { return NT > 9 ? (NT + 1) / 2 : NT; }
template <int NT>
constexpr int fwd_nsplit() { return (NT + fwd_ntw<NT>() - 1) / fwd_ntw<NT>(); }
// x prefetch depth in k-steps (divides KS, so every step's register slot is static;
// 3 for KS = 9 spills)
template <int KS>
constexpr int fwd_pf() { return KS % 2 == 0 ? 2 : 1; }

template <int NT, int KS, bool FILM>
__global__ void __launch_bounds__(kLinThreads) lin_fwd_kernel(const LinArgs a) {
    // Workgroup (split sp, row partition w): the split's NTW output tiles' B fragments
    // (weights, pre-split and packed; <= 144 KB) are loaded into LDS once by LDS-DMA and
    // stay resident; the workgroup then walks its blocks of 256 rows, each wave 32 rows
    // (two MFMA B columns of 16) x all NTW tiles, so every A fragment read from LDS feeds
    // 6 MFMAs.  No barriers in the main loop: a wave streams its rows' x through
    // registers PF k-steps ahead (branch-free buffer loads; rows past M and columns past
    // K read zeros), across block boundaries.  The two splits of a row range run on one
    // XCD (workgroup ids 8 apart) and share its x in L2.  Each row is scaled by a power
    // of two from its running maximum over the k-steps read so far (the fp16 lo parts
    // stay normal at any magnitude); when a row's scale shrinks its accumulators are
    // rescaled exactly.
    constexpr int NTW = fwd_ntw<NT>();
    constexpr int NSPLIT = fwd_nsplit<NT>();
    constexpr int PF = fwd_pf<KS>();
    __shared__ f4 wl[KS * NTW * kTileF4];                      // [ks][tile][hi 64 | lo 64]
    __shared__ float cst[4][NTW * 16];                          // 1/su, bias, gamma, beta
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t n = lane & 15u, g = lane >> 4;
    // workgroup id -> (split, row partition): ids 8 apart share an XCD
    const uint32_t id = blockIdx.x;
    const uint32_t sp = NSPLIT == 1 ? 0 : (id >> 3) & 1u;
    const uint32_t w = NSPLIT == 1 ? id : ((id >> 4) << 3) | (id & 7u);
    const uint32_t G = gridDim.x / NSPLIT;
    const uint32_t t0 = sp * NTW;                               // first output tile
    const uint32_t t_count = NT - t0 < (uint32_t)NTW ? NT - t0 : NTW;
    const uint32_t nblk = ceil_div(a.M, kLinRows);
    const uint32_t b0 = (uint32_t)((uint64_t)w * nblk / G);
    const uint32_t b1 = (uint32_t)((uint64_t)(w + 1) * nblk / G);

    {   // resident weights: pieces (ks, tile, hi/lo) of 1 KB, round-robin over the waves
        const v4i rs = make_rsrc(a.packed, KS * NT * kTileF4 * 16u);
        for (uint32_t p = wave; p < (uint32_t)(KS * NTW * 2); p += kLinWaves) {
            const uint32_t ks = p / (NTW * 2), tl = (p / 2) % NTW, h = p & 1u;
            if (tl >= t_count) continue;
            dma16(rs, lane * 16u, ((ks * NT + t0 + tl) * kTileF4 + h * 64) * 16u,
                  lds_addr(&wl[(ks * NTW + tl) * kTileF4 + h * 64]));
        }
        for (uint32_t c = tid; c < NTW * 16u; c += kLinThreads) {
            const uint32_t col = 16 * t0 + c;
            cst[0][c] = col < a.N ? 1.0f / a.su[col] : 0.0f;      // powers of two: exact
            cst[1][c] = (col < a.N && a.bias) ? a.bias[col] : 0.0f;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    if (b0 >= b1) return;

    // this lane's 8 K values (k = 32 q + 8 g + j) of its two rows in block blk
    // (rows = 0: an empty range, the loads read zeros -- branch-free past the last
    // block); only the last k-step can run past K (KS = ceil(K / 32)), the others take
    // compile-time offsets from the lane's row base
    uint32_t xbase[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) xbase[c] = ((wave * 32 + 16 * c + n) * a.K + 8 * g) * 4u;
    auto load_x = [&](uint32_t blk, int q, f4 (&v)[2][2]) {
        const uint32_t m0 = blk * kLinRows;
        const uint32_t rows = blk >= b1 ? 0u : (a.M - m0 < kLinRows ? a.M - m0 : kLinRows);
        const __amdgpu_buffer_rsrc_t xr = buf_rsrc(a.x + (size_t)m0 * a.K, rows * a.K * 4u);
        const uint32_t k0 = 32 * q + 8 * g;
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                // the constant part as the instruction's scalar offset
                const uint32_t voff = q + 1 < KS || k0 + 4 * h + 4 <= a.K ? xbase[c] : kOob;
                v[c][h] = __builtin_bit_cast(
                    f4, __builtin_amdgcn_raw_buffer_load_b128(xr, (int)voff, 128 * q + 16 * h, 0));
            }
    };
    f4 xb[PF][2][2];
#pragma unroll
    for (int p = 0; p < PF; ++p) load_x(b0, p, xb[p]);

    uint32_t face = 0xffffffffu;
    for (uint32_t blk = b0; blk < b1; ++blk) {
        const uint32_t m_blk = blk * kLinRows;
        const uint32_t rows = a.M - m_blk < kLinRows ? a.M - m_blk : kLinRows;
        bool straddle = false;
        if constexpr (FILM) {
            // the face's gamma / beta into LDS when it changes (every wave walks the same
            // blocks, so the barriers match; faces are ~98 K rows apart); a block that
            // straddles two faces reads them per row from global memory instead
            const uint32_t f0 = m_blk / a.rows_per_face, f1 = (m_blk + rows - 1) / a.rows_per_face;
            straddle = f0 != f1;
            if (!straddle && f0 != face) {
                __syncthreads();                                 // the last epilogue is done
                for (uint32_t c = tid; c < NTW * 16u; c += kLinThreads) {
                    const uint32_t col = 16 * t0 + c;
                    cst[2][c] = col < a.N ? a.gamma[(size_t)f0 * a.N + col] : 0.0f;
                    cst[3][c] = col < a.N ? a.beta[(size_t)f0 * a.N + col] : 0.0f;
                }
                __syncthreads();
                face = f0;
            }
        }
        float rmax[2] = {0.0f, 0.0f}, xs[2] = {1.0f, 1.0f};
        f4 acc[2][NTW];
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int t = 0; t < NTW; ++t) acc[c][t] = f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int q = 0; q < KS; ++q) {
            f4 xa[2][2];
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int h = 0; h < 2; ++h) xa[c][h] = xb[q % PF][c][h];
            // refill the slot with step q + PF (this block, or the next one's)
            if (q + PF < KS) load_x(blk, q + PF, xb[q % PF]);
            else load_x(blk + 1, q + PF - KS, xb[q % PF]);
            // running row maxima -> scales; rescale the rows whose scale shrank
            float ratio[2];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                float mx = 0.0f;
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int j = 0; j < 4; ++j) mx = fmaxf(mx, fabsf(xa[c][h][j]));
                mx = fmaxf(mx, __shfl_xor(mx, 16));
                mx = fmaxf(mx, __shfl_xor(mx, 32));
                rmax[c] = fmaxf(rmax[c], mx);
                const float sn = pow2_scale(rmax[c]);
                ratio[c] = __builtin_amdgcn_ldexpf(1.0f, __builtin_amdgcn_frexp_expf(sn) -
                                                             __builtin_amdgcn_frexp_expf(xs[c]));
                xs[c] = sn;
            }
            if (q > 0 && __any(ratio[0] != 1.0f || ratio[1] != 1.0f)) {
#pragma unroll
                for (int c = 0; c < 2; ++c)
#pragma unroll
                    for (int t = 0; t < NTW; ++t)
#pragma unroll
                        for (int r = 0; r < 4; ++r) acc[c][t][r] = __fmul_rn(acc[c][t][r], ratio[c]);
            }
            f4 bh[2], bl[2];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                float v[8];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    v[j] = __fmul_rn(xa[c][0][j], xs[c]);
                    v[4 + j] = __fmul_rn(xa[c][1][j], xs[c]);
                }
                split8(v, bh[c], bl[c]);
            }
            const f4 *A = wl + q * NTW * kTileF4 + lane;
#pragma unroll
            for (int t = 0; t < NTW; ++t) {
                if (t < (int)t_count) {
                    const f4 ah = A[t * kTileF4], al = A[t * kTileF4 + 64];
                    acc[0][t] = mfma16(al, bh[0], acc[0][t]);
                    acc[1][t] = mfma16(al, bh[1], acc[1][t]);
                    acc[0][t] = mfma16(ah, bl[0], acc[0][t]);
                    acc[1][t] = mfma16(ah, bl[1], acc[1][t]);
                    acc[0][t] = mfma16(ah, bh[0], acc[0][t]);
                    acc[1][t] = mfma16(ah, bh[1], acc[1][t]);
                }
            }
        }
        // lane (n, g) of tile t, column c holds output columns 16 (t0 + t) + 4 g + r of
        // row m_blk + 32 wave + 16 c + n (N % 16 == 0).  FiLM's gamma / beta from LDS, or
        // per row from global memory where the block straddles two faces (two copies of
        // the epilogue, so the common one carries no load waits)
        auto epilogue = [&](auto from_lds) {
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const uint32_t r_in = wave * 32 + 16 * c + n;
                if (r_in >= rows) continue;
                const uint32_t m = m_blk + r_in;
                const float inv_xs = 1.0f / xs[c];             // powers of two: exact
                float *orow = a.out + (size_t)m * a.N;
                const size_t frow = FILM ? (size_t)(m / a.rows_per_face) * a.N : 0;
#pragma unroll
                for (int t = 0; t < NTW; ++t) {
                    if (t >= (int)t_count) continue;
                    const uint32_t cl = 16 * t + 4 * g, c0 = 16 * t0 + cl;
                    const f4 is4 = *reinterpret_cast<const f4 *>(&cst[0][cl]);
                    const f4 b4 = *reinterpret_cast<const f4 *>(&cst[1][cl]);
                    f4 yv, v;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        float y = __fmul_rn(__fmul_rn(acc[c][t][r], inv_xs), is4[r]);
                        if (a.bias) y = __fadd_rn(y, b4[r]);
                        yv[r] = y;
                    }
                    if constexpr (FILM) {
                        // FiLMSiren.forward (sdf_model.py:62-67): sin(gamma * out + beta),
                        // one rounding per op as the reference's separate elementwise ops
                        f4 gm, bt;
                        if constexpr (decltype(from_lds)::value) {
                            gm = *reinterpret_cast<const f4 *>(&cst[2][cl]);
                            bt = *reinterpret_cast<const f4 *>(&cst[3][cl]);
                        } else {
                            gm = *reinterpret_cast<const f4 *>(a.gamma + frow + c0);
                            bt = *reinterpret_cast<const f4 *>(a.beta + frow + c0);
                        }
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            v[r] = sin_hw(__fadd_rn(__fmul_rn(gm[r], yv[r]), bt[r]));
                        *reinterpret_cast<f4 *>(a.y_save + (size_t)m * a.N + c0) = yv;
                    } else {
                        v = yv;
                    }
                    *reinterpret_cast<f4 *>(orow + c0) = v;
                }
            }
        };
        if (!FILM || !straddle) epilogue(std::true_type{});
        else epilogue(std::false_type{});
    }
}

// ----------------------------------------------------------------------------
// FiLM backward (elementwise part): with u = gamma[f] y + beta[f] (as the forward),
//   du = ds cos(u),  dy = du gamma[f]     (written: the GEMMs' input)
//   per-block column sums  du y (-> dgamma[f]),  du (-> dbeta[f]),  dy (-> db)
// Block (f, j) covers rows [f R + j rpb, ...) of face f; thread = column (N = 256).
// ----------------------------------------------------------------------------
// rows per thread whose loads are issued together (film_bwd / film_bwd2_kernel)
#ifndef SDFR_FILM_ROWS
#define SDFR_FILM_ROWS 4
#endif
constexpr int kFilmRows = SDFR_FILM_ROWS;

__global__ void __launch_bounds__(256) film_bwd_kernel(const float *__restrict__ ds,
                                                       const float *__restrict__ y,
                                                       const float *__restrict__ gamma,
                                                       const float *__restrict__ beta,
                                                       float *__restrict__ dy, uint32_t N,
                                                       uint32_t rows_per_face, uint32_t rpb,
                                                       float *__restrict__ part) {
    const uint32_t f = blockIdx.y, j = blockIdx.x, c = threadIdx.x;
    const uint32_t r0 = j * rpb, r1 = min(rows_per_face, r0 + rpb);
    const float gm = gamma[(size_t)f * N + c], bt = beta[(size_t)f * N + c];
    float sg = 0.0f, sb = 0.0f, sd = 0.0f;
    const size_t base = (size_t)f * rows_per_face;
    uint32_t r = r0;
    for (; r + kFilmRows <= r1; r += kFilmRows) {
        float dsv[kFilmRows], yv[kFilmRows];
#pragma unroll
        for (int k = 0; k < kFilmRows; ++k) {
            dsv[k] = ds[(base + r + k) * N + c];
            yv[k] = y[(base + r + k) * N + c];
        }
#pragma unroll
        for (int k = 0; k < kFilmRows; ++k) {
            const float u = __fadd_rn(__fmul_rn(gm, yv[k]), bt);
            const float du = __fmul_rn(dsv[k], cos_hw(u));
            const float d = __fmul_rn(du, gm);
            dy[(base + r + k) * N + c] = d;
            sg = __fadd_rn(sg, __fmul_rn(du, yv[k]));
            sb = __fadd_rn(sb, du);
            sd = __fadd_rn(sd, d);
        }
    }
    for (; r < r1; ++r) {
        const float yv = y[(base + r) * N + c];
        const float u = __fadd_rn(__fmul_rn(gm, yv), bt);
        const float du = __fmul_rn(ds[(base + r) * N + c], cos_hw(u));
        const float d = __fmul_rn(du, gm);
        dy[(base + r) * N + c] = d;
        sg = __fadd_rn(sg, __fmul_rn(du, yv));
        sb = __fadd_rn(sb, du);
        sd = __fadd_rn(sd, d);
    }
    float *p = part + ((size_t)f * gridDim.x + j) * 3 * N;
    p[c] = sg;
    p[N + c] = sb;
    p[2 * N + c] = sd;
}

// per face f: dgamma[f], dbeta[f], dbf[f] (the bias gradient's share of face f) =
// the face's block partials summed in a fixed order: block (32 columns, f), thread
// (column, group jg of the blocks j = jg mod 8), the 8 group sums added in order
__global__ void __launch_bounds__(256) film_bwd_reduce_kernel(const float *__restrict__ part,
                                                              uint32_t nb, uint32_t N,
                                                              float *__restrict__ dgamma,
                                                              float *__restrict__ dbeta,
                                                              float *__restrict__ dbf) {
    __shared__ float red[3][8][32];
    const uint32_t f = blockIdx.y, c = blockIdx.x * 32 + (threadIdx.x & 31u);
    const uint32_t jg = threadIdx.x >> 5;
    float sg = 0.0f, sb = 0.0f, sd = 0.0f;
    for (uint32_t j = jg; j < nb; j += 8) {
        const float *p = part + ((size_t)f * nb + j) * 3 * N;
        sg += p[c];
        sb += p[N + c];
        sd += p[2 * N + c];
    }
    red[0][jg][threadIdx.x & 31u] = sg;
    red[1][jg][threadIdx.x & 31u] = sb;
    red[2][jg][threadIdx.x & 31u] = sd;
    __syncthreads();
    if (jg == 0) {
        for (uint32_t k = 1; k < 8; ++k) {
            sg += red[0][k][threadIdx.x];
            sb += red[1][k][threadIdx.x];
            sd += red[2][k][threadIdx.x];
        }
        dgamma[(size_t)f * N + c] = sg;
        dbeta[(size_t)f * N + c] = sb;
        dbf[(size_t)f * N + c] = sd;
    }
}

// Second order (sdfr_film_backward_grad): the derivative of film_bwd_kernel's outputs
// (dy, dgamma, dbeta) w.r.t. its inputs, for a graph built with create_graph (the
// SIREN eikonal term, differentiated again by the loss).  Per element, with u = gm y +
// bt recomputed as film_bwd_kernel does and H = G_dy gm + G_dgamma y + G_dbeta:
//   d_ds = H cos u;  dU = -H ds sin u;  d_y = dU gm + G_dgamma ds cos u;
// per (face, column): d_gamma = sum (dU y + G_dy ds cos u), d_beta = sum dU.  One thread
// per column over a block of rows (film_bwd_kernel's layout); partials reduced by
// film_bwd_reduce_kernel (third sum unused).  The composite torch form (autograd of
// du = ds cos(gamma y + beta), dy = du gamma, the two row sums) launched ~18
// elementwise / reduction passes per layer.
__global__ void __launch_bounds__(256) film_bwd2_kernel(
    const float *__restrict__ ds, const float *__restrict__ y, const float *__restrict__ gamma,
    const float *__restrict__ beta, const float *__restrict__ gdy, const float *__restrict__ gdg,
    const float *__restrict__ gdb, float *__restrict__ d_ds, float *__restrict__ d_y, uint32_t N,
    uint32_t rows_per_face, uint32_t rpb, float *__restrict__ part) {
    const uint32_t f = blockIdx.y, j = blockIdx.x, c = threadIdx.x;
    const uint32_t r0 = j * rpb, r1 = min(rows_per_face, r0 + rpb);
    const size_t fc = (size_t)f * N + c;
    const float gm = gamma[fc], bt = beta[fc];
    const float gg = gdg ? gdg[fc] : 0.0f, gb = gdb ? gdb[fc] : 0.0f;
    float sg = 0.0f, sb = 0.0f;
    const size_t base = (size_t)f * rows_per_face;
    // one row's arithmetic; the column sums run over the rows in order
    auto row = [&](size_t e, float dsv, float yv, float gd) {
        const float u = __fadd_rn(__fmul_rn(gm, yv), bt);
        const float cu = cos_hw(u), su = sin_hw(u);
        const float h = __fadd_rn(__fadd_rn(__fmul_rn(gd, gm), __fmul_rn(gg, yv)), gb);
        const float dsc = __fmul_rn(dsv, cu);
        const float du_ = -__fmul_rn(__fmul_rn(h, dsv), su);
        d_ds[e] = __fmul_rn(h, cu);
        d_y[e] = __fadd_rn(__fmul_rn(du_, gm), __fmul_rn(gg, dsc));
        sg = __fadd_rn(sg, __fadd_rn(__fmul_rn(du_, yv), __fmul_rn(gd, dsc)));
        sb = __fadd_rn(sb, du_);
    };
    uint32_t r = r0;
    // kFilmRows rows' loads in flight per thread (two waves per SIMD run this kernel:
    // one row at a time left it at ~3.0 TB/s of its 1 GB per call)
    for (; r + kFilmRows <= r1; r += kFilmRows) {
        float dsv[kFilmRows], yv[kFilmRows], gd[kFilmRows];
#pragma unroll
        for (int k = 0; k < kFilmRows; ++k) {
            const size_t e = (base + r + k) * N + c;
            dsv[k] = ds[e];
            yv[k] = y[e];
            gd[k] = gdy ? gdy[e] : 0.0f;
        }
#pragma unroll
        for (int k = 0; k < kFilmRows; ++k) row((base + r + k) * N + c, dsv[k], yv[k], gd[k]);
    }
    for (; r < r1; ++r) {
        const size_t e = (base + r) * N + c;
        row(e, ds[e], y[e], gdy ? gdy[e] : 0.0f);
    }
    float *p = part + ((size_t)f * gridDim.x + j) * 3 * N;
    p[c] = sg;
    p[N + c] = sb;
    p[2 * N + c] = 0.0f;
}

// ----------------------------------------------------------------------------
// weight gradient partials: part[p][n][k] = sum over workgroup p's rows of
// dy[m, n] x[m, k] (N = 256; blockIdx.y = which 128 of the n).  16 waves in two roles
// per 32-row m-step, double-buffered in LDS with one barrier per step:
//   waves 8..15 (producers): one 16-column tile of dy or x per wave and task; a lane
//     loads 8 rows of one column (a step ahead; branch-free buffer loads, rows past the
//     workgroup's range and columns past K read zeros), which is exactly its MFMA
//     fragment; it scales the column by a power of two from the column's running
//     maximum over the rows seen so far, splits into hi/lo fp16 and stores the
//     fragments;
//   waves 0..7 (consumers): 2 n-tiles x one half of the k-tiles each, 3 MFMAs per
//     fragment pair, accumulated in fp32 over the workgroup's rows.
// The running maxima only grow, so a column's scale only shrinks (or leaves 1 when the
// column had been all zero): when a step changes scales the producers publish the
// ratios and the consumers rescale their accumulators exactly (powers of two, <= 1)
// before adding the step; the last scales are undone on the partial.  No pass over
// the operands beyond the one that feeds the MFMAs.
// The conversion VALU of the producers runs beside the consumers' MFMAs on every SIMD.
// ----------------------------------------------------------------------------
struct WgradArgs {
    const float *dy;           // [M, N]
    const float *x;            // [M, K]
    float *part;               // [P][N][K]
    uint32_t M, N, K, rows;    // rows per workgroup (multiple of 32)
};

constexpr uint32_t kWgWaves = 16, kWgThreads = kWgWaves * 64;

template <int KT>
__global__ void __launch_bounds__(kWgThreads) lin_wgrad_kernel(const WgradArgs a) {
    constexpr uint32_t NTn = 8;                             // n-tiles per workgroup
    constexpr uint32_t KH = (KT + 1) / 2;                   // k-tiles per consumer wave
    constexpr uint32_t kA = NTn * kTileF4, kB = KT * kTileF4;
    constexpr uint32_t kCols = (NTn + KT) * 16;             // dy columns, then x columns
    constexpr uint32_t kPer = ceil_div(NTn + KT, 8);        // tiles per producer wave
    __shared__ f4 As[2][kA];
    __shared__ f4 Bs[2][kB];
    __shared__ float ratio[2][kCols];                       // scale change of the step
    __shared__ float fin[kCols];                            // the last scales
    __shared__ uint32_t chg[2][8];                          // per producer wave: any change
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t n0 = blockIdx.y * NTn * 16;
    const uint32_t m_begin = blockIdx.x * a.rows;
    const uint32_t nrows = m_begin < a.M ? min(a.rows, a.M - m_begin) : 0;
    const uint32_t nsteps = ceil_div(nrows, 32);

    if (wave >= 8) {
        // ---- producer wave pw: tiles pw, pw + 8, ... (tile < 8: dy columns n0 + 16 tile
        // .., else x columns 16 (tile - 8) ..); lane = (column c = lane & 15, rows 8 g8 ..)
        const uint32_t pw = wave - 8, c = lane & 15u, g8 = lane >> 4;
        const __amdgpu_buffer_rsrc_t rdy = buf_rsrc(a.dy + (size_t)m_begin * a.N, nrows * a.N * 4u);
        const __amdgpu_buffer_rsrc_t rx = buf_rsrc(a.x + (size_t)m_begin * a.K, nrows * a.K * 4u);
        float stv[kPer][8];
        float rmax[kPer], scl[kPer];
#pragma unroll
        for (uint32_t i = 0; i < kPer; ++i) {
            rmax[i] = 0.0f;
            scl[i] = 1.0f;
        }
        auto load = [&](uint32_t step) {
#pragma unroll
            for (uint32_t i = 0; i < kPer; ++i) {
                const uint32_t tile = pw + 8 * i;
                const bool is_dy = tile < NTn;              // (i == 0)
                const uint32_t col = is_dy ? n0 + 16 * tile + c : 16 * (tile - NTn) + c;
                const uint32_t C = is_dy ? a.N : a.K;
                const bool ok = tile < NTn + KT && (is_dy || col < a.K);
                const uint32_t r0 = 32 * step + 8 * g8;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t off = ok ? ((r0 + j) * C + col) * 4u : kOob;
                    stv[i][j] = ld1(is_dy ? rdy : rx, off);
                }
            }
        };
        auto store = [&](uint32_t slot) {
            bool any = false;
#pragma unroll
            for (uint32_t i = 0; i < kPer; ++i) {
                const uint32_t tile = pw + 8 * i;
                if (tile >= NTn + KT) continue;             // wave-uniform
                float mx = 0.0f;
#pragma unroll
                for (int j = 0; j < 8; ++j) mx = fmaxf(mx, fabsf(stv[i][j]));
                mx = fmaxf(mx, __shfl_xor(mx, 16));
                mx = fmaxf(mx, __shfl_xor(mx, 32));
                rmax[i] = fmaxf(rmax[i], mx);
                const float sn = pow2_scale(rmax[i]);
                const float rt = sn / scl[i];               // powers of two: exact
                any |= rt != 1.0f;
                scl[i] = sn;
                if (g8 == 0) ratio[slot][16 * tile + c] = rt;
                float v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = __fmul_rn(stv[i][j], sn);
                f4 hi, lo;
                split8(v, hi, lo);
                f4 *dst = (tile < NTn ? As[slot] + tile * kTileF4
                                      : Bs[slot] + (tile - NTn) * kTileF4) + lane;
                dst[0] = hi;
                dst[64] = lo;
            }
            const uint32_t anyw = __builtin_amdgcn_readfirstlane(__any(any) ? 1u : 0u);
            if (lane == 0) chg[slot][pw] = anyw;
        };
        // (each role runs its own loop with the same barriers, one per step, so the
        // compiler never holds both roles' registers at once)
        if (nsteps > 0) {
            load(0);
            store(0);
            if (nsteps > 1) load(1);
        }
        __syncthreads();
        for (uint32_t s = 0; s < nsteps; ++s) {
            if (s + 1 < nsteps) {
                store((s & 1u) ^ 1u);                  // step s+1 (loaded a step ago)
                if (s + 2 < nsteps) load(s + 2);
            }
            __syncthreads();
        }
#pragma unroll
        for (uint32_t i = 0; i < kPer; ++i) {
            const uint32_t tile = pw + 8 * i;
            if (tile < NTn + KT && g8 == 0) fin[16 * tile + c] = scl[i];
        }
        __syncthreads();
        return;
    }

    // ---- consumer: n-tiles 2 (w & 3), +1; k-tiles [KH (w >> 2), ...)
    const uint32_t np = wave & 3u, kh = (wave >> 2) & 1u;
    const uint32_t k_begin = kh * KH;
    const uint32_t k_count = KT - k_begin < KH ? KT - k_begin : KH;
    const uint32_t kc = lane & 15u, g = lane >> 4;
    f4 acc[2][KH];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (uint32_t t = 0; t < KH; ++t) acc[i][t] = f4{0.0f, 0.0f, 0.0f, 0.0f};
    __syncthreads();
    for (uint32_t s = 0; s < nsteps; ++s) {
        const uint32_t slot = s & 1u;
        const uint4 c0 = *reinterpret_cast<const uint4 *>(&chg[slot][0]);
        const uint4 c1 = *reinterpret_cast<const uint4 *>(&chg[slot][4]);
        if (s > 0 && (c0.x | c0.y | c0.z | c0.w | c1.x | c1.y | c1.z | c1.w)) {
            // lane (kc, g) of (n-tile i, k-tile t) holds n = 16 (2 np + i) + 4 g + r,
            // k = 16 (k_begin + t) + kc
            f4 rn[2];
#pragma unroll
            for (int i = 0; i < 2; ++i)
                rn[i] = *reinterpret_cast<const f4 *>(&ratio[slot][16 * (2 * np + i) + 4 * g]);
#pragma unroll
            for (uint32_t t = 0; t < KH; ++t) {
                const float rk = t < k_count ? ratio[slot][NTn * 16 + 16 * (k_begin + t) + kc] : 1.0f;
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        acc[i][t][r] = __fmul_rn(__fmul_rn(acc[i][t][r], rn[i][r]), rk);
            }
        }
        const f4 *A = As[slot] + (2 * np) * kTileF4 + lane;
        const f4 a0h = A[0], a0l = A[64], a1h = A[kTileF4], a1l = A[kTileF4 + 64];
        const f4 *Bp = Bs[slot] + k_begin * kTileF4 + lane;
#pragma unroll
        for (uint32_t t = 0; t < KH; ++t) {
            if (t < k_count) {
                const f4 bh = Bp[t * kTileF4], bl = Bp[t * kTileF4 + 64];
                acc[0][t] = mfma16(a0l, bh, acc[0][t]);
                acc[1][t] = mfma16(a1l, bh, acc[1][t]);
                acc[0][t] = mfma16(a0h, bl, acc[0][t]);
                acc[1][t] = mfma16(a1h, bl, acc[1][t]);
                acc[0][t] = mfma16(a0h, bh, acc[0][t]);
                acc[1][t] = mfma16(a1h, bh, acc[1][t]);
            }
        }
        __syncthreads();
    }
    __syncthreads();                                   // fin[] written
    // unscale (exact; one power of two at a time) and store the partial
    float *pp = a.part + (size_t)blockIdx.x * a.N * a.K;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const uint32_t nb = 16 * (2 * np + i) + 4 * g;
        const f4 sn = *reinterpret_cast<const f4 *>(&fin[nb]);
#pragma unroll
        for (uint32_t t = 0; t < KH; ++t) {
            if (t >= k_count) continue;
            const uint32_t k = 16 * (k_begin + t) + kc;
            if (k >= a.K) continue;
            const float sk = fin[NTn * 16 + k];
#pragma unroll
            for (int r = 0; r < 4; ++r)
                pp[(size_t)(n0 + nb + r) * a.K + k] =
                    __fmul_rn(__fmul_rn(acc[i][t][r], 1.0f / sn[r]), 1.0f / sk);
        }
    }
}

__global__ void __launch_bounds__(256) lin_reduce_kernel(const float *__restrict__ part, uint32_t P,
                                                         uint32_t count, float *__restrict__ out) {
    const uint32_t e = blockIdx.x * 256 + threadIdx.x;
    if (e >= count) return;
    float s = 0.0f;
    uint32_t p = 0;
    for (; p + 8 <= P; p += 8) {                       // loads in flight, sums in order
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = part[(size_t)(p + j) * count + e];
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[j];
    }
    for (; p < P; ++p) s += part[(size_t)p * count + e];
    out[e] = s;
}

uint32_t wgrad_rows(uint32_t M) {
    // 128 row ranges x 2 n-halves = one round of 256 workgroups, whole m-steps
    const uint32_t r = ceil_div(ceil_div(M, 128), 32) * 32;
    return r < 32 ? 32 : r;
}

template <int NT, int KS, bool FILM = false>
int launch_fwd(const LinArgs &a, hipStream_t st) {
    // persistent: one workgroup per CU (resident weights take up to 146 KB of LDS),
    // NSPLIT of them per row partition; at most one partition per block of rows, and a
    // multiple of 8 partitions when split (the splits' ids are 8 apart)
    constexpr uint32_t ns = fwd_nsplit<NT>();
    const uint32_t nblk = ceil_div(a.M, kLinRows);
    uint32_t G = 256 / ns;
    if (nblk < G) G = ns > 1 ? std::max<uint32_t>(8, ceil_div(nblk, 8) * 8) : nblk;
    hipLaunchKernelGGL((lin_fwd_kernel<NT, KS, FILM>), dim3(G * ns), dim3(kLinThreads), 0, st, a);
    return check_launch("linear_f16x3");
}

uint32_t film_blocks_per_face(uint32_t F, uint32_t rows_per_face) {
    // ~512 blocks in all, at least 64 rows each
    uint32_t nb = ceil_div(512, F);
    const uint32_t maxb = ceil_div(rows_per_face, 64);
    return nb < 1 ? 1 : (nb > maxb ? maxb : nb);
}

template <int KT>
int launch_wgrad(const WgradArgs &a, uint32_t P, hipStream_t st) {
    hipLaunchKernelGGL((lin_wgrad_kernel<KT>), dim3(P, 2), dim3(kWgThreads), 0, st, a);
    return check_launch("linear_wgrad_f16x3");
}

}  // namespace
}  // namespace sdfr

using namespace sdfr;

extern "C" {

size_t sdfr_linear_pack_bytes(uint32_t N, uint32_t K) {
    return (size_t)ceil_div(K, 32) * ceil_div(N, 16) * kTileF4 * sizeof(f4) + (size_t)N * 4;
}

int sdfr_linear_pack(const float *w, uint32_t N, uint32_t K, int transposed, void *packed,
                     void *stream) {
    if (!w || !packed) return fail(SDFR_EINVAL, "linear_pack: null pointer");
    if (N == 0 || K == 0) return fail(SDFR_EINVAL, "linear_pack: empty matrix");
    hipStream_t st = (hipStream_t)stream;
    const size_t frag = (size_t)ceil_div(K, 32) * ceil_div(N, 16) * kTileF4 * sizeof(f4);
    float *su = reinterpret_cast<float *>(static_cast<char *>(packed) + frag);
    hipLaunchKernelGGL(lin_scale_kernel, dim3(ceil_div(N, 4)), dim3(256), 0, st, w, N, K,
                       transposed ? 1 : 0, su);
    int rc = check_launch("linear_pack: scale");
    if (rc) return rc;
    const uint32_t total = ceil_div(K, 32) * ceil_div(N, 16) * 64;
    hipLaunchKernelGGL(lin_pack_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, st, w, N, K,
                       transposed ? 1 : 0, su, reinterpret_cast<f4 *>(packed));
    return check_launch("linear_pack: pack");
}

int sdfr_film_linear_f16x3(float *out, float *y_save, const float *x, const void *packed,
                           const float *bias, const float *gamma, const float *beta, uint32_t M,
                           uint32_t N, uint32_t K, uint32_t rows_per_face, void *stream) {
    if (M == 0) return SDFR_OK;
    if (!out || !y_save || !x || !packed || !gamma || !beta)
        return fail(SDFR_EINVAL, "film_linear_f16x3: null pointer");
    if (rows_per_face == 0 || M % rows_per_face)
        return fail(SDFR_EINVAL, "film_linear_f16x3: M must be a multiple of rows_per_face");
    if (K % 4 || N != 256 ||
        (reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out) |
         reinterpret_cast<uintptr_t>(y_save) | reinterpret_cast<uintptr_t>(gamma) |
         reinterpret_cast<uintptr_t>(beta)) % 16)
        return fail(SDFR_EINVAL, "film_linear_f16x3: N = 256, K multiple of 4, 16-B aligned "
                                 "x, out, y_save, gamma, beta");
    LinArgs a;
    a.x = x;
    a.packed = static_cast<const f4 *>(packed);
    a.su = reinterpret_cast<const float *>(static_cast<const char *>(packed) +
                                           (size_t)ceil_div(K, 32) * 16 * kTileF4 * sizeof(f4));
    a.bias = bias;
    a.out = out;
    a.M = M;
    a.N = N;
    a.K = K;
    a.gamma = gamma;
    a.beta = beta;
    a.y_save = y_save;
    a.rows_per_face = rows_per_face;
    hipStream_t st = (hipStream_t)stream;
    const uint32_t KS = ceil_div(K, 32);
    if (KS == 8) return launch_fwd<16, 8, true>(a, st);
    if (KS == 9) return launch_fwd<16, 9, true>(a, st);
    return fail(SDFR_EUNSUPPORTED, "film_linear_f16x3: K must be <= 256 or 257..288");
}

size_t sdfr_film_backward_ws_bytes(uint32_t M, uint32_t N, uint32_t rows_per_face) {
    if (M == 0 || rows_per_face == 0) return 0;
    const uint32_t F = M / rows_per_face;
    return (size_t)F * film_blocks_per_face(F, rows_per_face) * 3 * N * 4;
}

int sdfr_film_backward(float *dy, float *dgamma, float *dbeta, float *dbf, const float *ds,
                       const float *y, const float *gamma, const float *beta, uint32_t M,
                       uint32_t N, uint32_t rows_per_face, void *ws, size_t ws_bytes,
                       void *stream) {
    if (M == 0) return SDFR_OK;
    if (!dy || !dgamma || !dbeta || !dbf || !ds || !y || !gamma || !beta)
        return fail(SDFR_EINVAL, "film_backward: null pointer");
    if (N != 256 || rows_per_face == 0 || M % rows_per_face)
        return fail(SDFR_EINVAL, "film_backward: N = 256, M a multiple of rows_per_face");
    if (!ws || ws_bytes < sdfr_film_backward_ws_bytes(M, N, rows_per_face))
        return fail(SDFR_EINVAL, "film_backward: workspace too small");
    const uint32_t F = M / rows_per_face, nb = film_blocks_per_face(F, rows_per_face);
    const uint32_t rpb = ceil_div(rows_per_face, nb);
    hipStream_t st = (hipStream_t)stream;
    float *part = static_cast<float *>(ws);
    hipLaunchKernelGGL(film_bwd_kernel, dim3(nb, F), dim3(256), 0, st, ds, y, gamma, beta, dy, N,
                       rows_per_face, rpb, part);
    int rc = check_launch("film_backward");
    if (rc) return rc;
    hipLaunchKernelGGL(film_bwd_reduce_kernel, dim3(N / 32, F), dim3(256), 0, st, part, nb, N,
                       dgamma, dbeta, dbf);
    return check_launch("film_backward: reduce");
}

int sdfr_film_backward_grad(float *d_ds, float *d_y, float *d_gamma, float *d_beta,
                            const float *ds, const float *y, const float *gamma,
                            const float *beta, const float *g_dy, const float *g_dgamma,
                            const float *g_dbeta, uint32_t M, uint32_t N, uint32_t rows_per_face,
                            void *ws, size_t ws_bytes, void *stream) {
    if (M == 0) return SDFR_OK;
    if (!d_ds || !d_y || !d_gamma || !d_beta || !ds || !y || !gamma || !beta)
        return fail(SDFR_EINVAL, "film_backward_grad: null pointer");
    if (N != 256 || rows_per_face == 0 || M % rows_per_face)
        return fail(SDFR_EINVAL, "film_backward_grad: N = 256, M a multiple of rows_per_face");
    if (!ws || ws_bytes < sdfr_film_backward_ws_bytes(M, N, rows_per_face) + (size_t)(M / rows_per_face) * N * 4)
        return fail(SDFR_EINVAL, "film_backward_grad: workspace too small");
    const uint32_t F = M / rows_per_face, nb = film_blocks_per_face(F, rows_per_face);
    const uint32_t rpb = ceil_div(rows_per_face, nb);
    hipStream_t st = (hipStream_t)stream;
    float *part = static_cast<float *>(ws);
    float *unused = part + (size_t)F * nb * 3 * N;          // the reduce's third sum
    hipLaunchKernelGGL(film_bwd2_kernel, dim3(nb, F), dim3(256), 0, st, ds, y, gamma, beta, g_dy,
                       g_dgamma, g_dbeta, d_ds, d_y, N, rows_per_face, rpb, part);
    int rc = check_launch("film_backward_grad");
    if (rc) return rc;
    hipLaunchKernelGGL(film_bwd_reduce_kernel, dim3(N / 32, F), dim3(256), 0, st, part, nb, N,
                       d_gamma, d_beta, unused);
    return check_launch("film_backward_grad: reduce");
}

size_t sdfr_film_backward_grad_ws_bytes(uint32_t M, uint32_t N, uint32_t rows_per_face) {
    if (M == 0 || rows_per_face == 0) return 0;
    return sdfr_film_backward_ws_bytes(M, N, rows_per_face) + (size_t)(M / rows_per_face) * N * 4;
}

int sdfr_linear_f16x3(float *out, const float *x, const void *packed, const float *bias,
                      uint32_t M, uint32_t N, uint32_t K, void *stream) {
    if (M == 0) return SDFR_OK;
    if (!out || !x || !packed) return fail(SDFR_EINVAL, "linear_f16x3: null pointer");
    if (K % 4 || N % 16 ||
        (reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out)) % 16)
        return fail(SDFR_EINVAL, "linear_f16x3: K a multiple of 4, N of 16, 16-B aligned x, out");
    LinArgs a;
    a.x = x;
    a.packed = static_cast<const f4 *>(packed);
    a.su = reinterpret_cast<const float *>(static_cast<const char *>(packed) +
                                           (size_t)ceil_div(K, 32) * ceil_div(N, 16) * kTileF4 *
                                               sizeof(f4));
    a.bias = bias;
    a.out = out;
    a.M = M;
    a.N = N;
    a.K = K;
    hipStream_t st = (hipStream_t)stream;
    const uint32_t NT = ceil_div(N, 16), KS = ceil_div(K, 32);
    // the renderer networks' shapes: K in {32, 64, 256, 288} -> N 256; N in {32, 64, 256,
    // 272, 288} <- K 256 (ngp / siren; the FCGenerator's x_in (60) and views (280) layers)
    if (NT == 16 && KS == 1) return launch_fwd<16, 1>(a, st);
    if (NT == 16 && KS == 2) return launch_fwd<16, 2>(a, st);
    if (NT == 16 && KS == 8) return launch_fwd<16, 8>(a, st);
    if (NT == 16 && KS == 9) return launch_fwd<16, 9>(a, st);
    if (NT == 2 && KS == 8) return launch_fwd<2, 8>(a, st);
    if (NT == 4 && KS == 8) return launch_fwd<4, 8>(a, st);
    if (NT == 17 && KS == 8) return launch_fwd<17, 8>(a, st);
    if (NT == 18 && KS == 8) return launch_fwd<18, 8>(a, st);
    return fail(SDFR_EUNSUPPORTED, "linear_f16x3: (N, K) must be (256, <=32 | <=64 | <=256 | <=288) "
                                   "or (<=32 | <=64 | <=288, <=256)");
}

size_t sdfr_linear_wgrad_ws_bytes(uint32_t M, uint32_t N, uint32_t K) {
    if (M == 0 || N == 0 || K == 0) return 0;
    const uint32_t P = ceil_div(M, wgrad_rows(M));
    return (size_t)P * N * K * 4;
}

int sdfr_linear_wgrad_f16x3(float *gw, const float *dy, const float *x, uint32_t M, uint32_t N,
                            uint32_t K, void *ws, size_t ws_bytes, void *stream) {
    if (!gw || (M && (!dy || !x))) return fail(SDFR_EINVAL, "linear_wgrad_f16x3: null pointer");
    if (N != 256 || K == 0 || K > 288 || K % 4)
        return fail(SDFR_EUNSUPPORTED,
                    "linear_wgrad_f16x3: N must be 256 and K <= 288 a multiple of 4");
    hipStream_t st = (hipStream_t)stream;
    if (M == 0) {
        if (hipMemsetAsync(gw, 0, (size_t)N * K * 4, st) != hipSuccess)
            return fail(SDFR_ELAUNCH, "linear_wgrad_f16x3: memset");
        return SDFR_OK;
    }
    if (!ws || ws_bytes < sdfr_linear_wgrad_ws_bytes(M, N, K))
        return fail(SDFR_EINVAL, "linear_wgrad_f16x3: workspace too small");
    WgradArgs a;
    a.dy = dy;
    a.x = x;
    a.part = static_cast<float *>(ws);
    a.M = M;
    a.N = N;
    a.K = K;
    a.rows = wgrad_rows(M);
    const uint32_t P = ceil_div(M, a.rows);
    const uint32_t KT = ceil_div(K, 16);
    int rc;
    if (KT <= 2) rc = launch_wgrad<2>(a, P, st);              // input_linear (K = 32)
    else if (KT <= 16) rc = launch_wgrad<16>(a, P, st);       // dense layers (K = 256)
    else if (KT <= 17) rc = launch_wgrad<17>(a, P, st);       // views (K = 272, 259)
    else rc = launch_wgrad<18>(a, P, st);
    if (rc) return rc;
    hipLaunchKernelGGL(lin_reduce_kernel, dim3(ceil_div(N * K, 256)), dim3(256), 0, st, a.part, P,
                       N * K, gw);
    return check_launch("linear_wgrad_f16x3: reduce");
}

}  // extern "C"
