// encoders.hip -- standalone hash-grid and SH encoder ops (drop-in for the
// reference's _gridencoder / _shencoder pybind modules), plus the library's
// error plumbing.  Semantics: gridencoder.cu:87-369, shencoder.cu:27-382.
//
// MI355X layout choices:
//  * forward grid = (ceil(B/256), L): blocks of one level run together, so the
//    level's table (<= 4 MiB at 2^19 x 2 fp32) sits in each XCD's 4 MiB L2
//    while it is gathered; C channels are fetched as one 8/16-byte load.
//  * all 2^D corner loads of a sample are issued before the first use.
//  * backward scatters with no-return fp32 global atomics (executed at the
//    memory side on gfx950); one thread owns all C channels of a (sample,level).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include <cstdio>
#include <string>

#include "sdfr_common.h"

namespace sdfr {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }

int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

int check_launch(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(SDFR_ELAUNCH, std::string(what) + ": " + hipGetErrorString(e));
    return SDFR_OK;
}

// ----------------------------------------------------------------------------
// grid encode forward
// ----------------------------------------------------------------------------
template <uint32_t D, uint32_t C>
__global__ void __launch_bounds__(256)
grid_fwd_kernel(const float *__restrict__ inputs, const float *__restrict__ emb,
                const int32_t *__restrict__ offsets, float *__restrict__ outputs,
                float *__restrict__ dy_dx, uint32_t B, uint32_t L, const LevelTable lt,
                uint32_t gridtype, int align_corners, uint32_t interp, int pair_ok) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const uint32_t level = blockIdx.y;
    LevelParam q = lt.p[level];
    finish_level(q, offsets, level, D, gridtype, align_corners);
    const float *grid = emb + (size_t)q.offset * C;
    float *out = outputs + ((size_t)level * B + b) * C;

    float x[D];
    bool oob = false;
#pragma unroll
    for (uint32_t d = 0; d < D; ++d) {
        x[d] = inputs[(size_t)b * D + d];
        if (x[d] < 0 || x[d] > 1) oob = true;
    }
    float *dd = dy_dx ? dy_dx + (size_t)b * D * L * C + (size_t)level * D * C : nullptr;
    if (oob) {
#pragma unroll
        for (uint32_t c = 0; c < C; ++c) out[c] = 0.0f;
        if (dd)
#pragma unroll
            for (uint32_t i = 0; i < D * C; ++i) dd[i] = 0.0f;
        return;
    }
    LevelCoord<D, C> lc;
    level_coord<D, C>(x, q, align_corners, interp, lc);
    // the 2^D corner rows, read once for the value AND every dy_dx term (which
    // are differences of the same corners, gridencoder.cu:201-244); paired
    // 16-B x-neighbour loads for D = 3, C = 2 on even-sized, even-based levels
    float v[1u << D][C];
    if constexpr (D == 3 && C == 2) {
        if (pair_ok && !((q.offset | q.hsize) & 1u))
            level_corners<D, C, true>(grid, q, align_corners, lc, v);
        else
            level_corners<D, C, false>(grid, q, align_corners, lc, v);
    } else {
        level_corners<D, C, false>(grid, q, align_corners, lc, v);
    }
    // value: corner weights and fma order of gridencoder.cu:160-192 (level_interp)
    float res[C];
#pragma unroll
    for (uint32_t c = 0; c < C; ++c) res[c] = 0.0f;
#pragma unroll
    for (uint32_t idx = 0; idx < (1u << D); ++idx) {
        float w = 1.0f;
#pragma unroll
        for (uint32_t d = 0; d < D; ++d)
            w = __fmul_rn(w, (idx & (1u << d)) ? lc.pos[d] : __fsub_rn(1.0f, lc.pos[d]));
#pragma unroll
        for (uint32_t c = 0; c < C; ++c) res[c] = __fmaf_rn(w, v[idx][c], res[c]);
    }
#pragma unroll
    for (uint32_t c = 0; c < C; ++c) out[c] = res[c];

    if (!dd) return;
#pragma unroll
    for (uint32_t gd = 0; gd < D; ++gd) {
        float rg[C];
#pragma unroll
        for (uint32_t c = 0; c < C; ++c) rg[c] = 0.0f;
#pragma unroll
        for (uint32_t idx = 0; idx < (1u << (D - 1)); ++idx) {
            float w = q.scale;
            uint32_t cl = 0;                       // corner with bit gd = 0
#pragma unroll
            for (uint32_t nd = 0; nd < D - 1; ++nd) {
                const uint32_t d = (nd >= gd) ? (nd + 1) : nd;
                if ((idx & (1u << nd)) == 0) {
                    w = __fmul_rn(w, __fsub_rn(1.0f, lc.pos[d]));
                } else {
                    w = __fmul_rn(w, lc.pos[d]);
                    cl |= 1u << d;
                }
            }
            const uint32_t cr = cl | (1u << gd);
#pragma unroll
            for (uint32_t c = 0; c < C; ++c)
                rg[c] = __fmaf_rn(__fmul_rn(w, __fsub_rn(v[cr][c], v[cl][c])), lc.pos_d[gd],
                                  rg[c]);
        }
#pragma unroll
        for (uint32_t c = 0; c < C; ++c) dd[gd * C + c] = rg[c];
    }
}

// ----------------------------------------------------------------------------
// grid encode backward: table scatter + input gradient
// ----------------------------------------------------------------------------
template <uint32_t D, uint32_t C>
__global__ void __launch_bounds__(256)
grid_bwd_kernel(const float *__restrict__ grad, const float *__restrict__ inputs,
                const int32_t *__restrict__ offsets, float *__restrict__ grad_emb, uint32_t B,
                const LevelTable lt, uint32_t gridtype, int align_corners, uint32_t interp,
                uint64_t lds_levels) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const uint32_t level = blockIdx.y;
    if ((lds_levels >> level) & 1u) return;   // grid_bwd_lds_kernel's levels
    LevelParam q = lt.p[level];
    finish_level(q, offsets, level, D, gridtype, align_corners);
    float x[D];
#pragma unroll
    for (uint32_t d = 0; d < D; ++d) {
        x[d] = inputs[(size_t)b * D + d];
        if (x[d] < 0 || x[d] > 1) return;   // grad stays 0 (gridencoder.cu:277-282)
    }
    LevelCoord<D, C> lc;
    level_coord<D, C>(x, q, align_corners, interp, lc);
    float g[C];
#pragma unroll
    for (uint32_t c = 0; c < C; ++c) g[c] = grad[((size_t)level * B + b) * C + c];
    float *gg = grad_emb + (size_t)q.offset * C;
#pragma unroll
    for (uint32_t idx = 0; idx < (1u << D); ++idx) {
        float w = 1.0f;
        uint32_t pl[D];
#pragma unroll
        for (uint32_t d = 0; d < D; ++d) {
            if ((idx & (1u << d)) == 0) {
                w = __fmul_rn(w, __fsub_rn(1.0f, lc.pos[d]));
                pl[d] = lc.pg[d];
            } else {
                w = __fmul_rn(w, lc.pos[d]);
                pl[d] = lc.pg[d] + 1;
            }
        }
        const uint32_t index = grid_index<D>(q, align_corners, pl) * C;
#pragma unroll
        for (uint32_t c = 0; c < C; ++c) atomicAdd(gg + index + c, __fmul_rn(w, g[c]));
    }
}

template <uint32_t D, uint32_t C>
__global__ void __launch_bounds__(256)
grid_input_bwd_kernel(const float *__restrict__ grad, const float *__restrict__ dy_dx,
                      float *__restrict__ grad_inputs, uint32_t B, uint32_t L) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B * D) return;
    const uint32_t b = t / D, d = t - b * D;
    const float *dd = dy_dx + (size_t)b * L * D * C;
    float r = 0.0f;
    for (uint32_t l = 0; l < L; ++l)
#pragma unroll
        for (uint32_t c = 0; c < C; ++c)
            r = __fmaf_rn(grad[((size_t)l * B + b) * C + c], dd[(size_t)l * D * C + d * C + c], r);
    grad_inputs[t] = r;
}

// Table gradient of the coarse (dense) levels: every sample of such a level
// lands on a few thousand rows, so direct global atomics serialise on the same
// addresses.  Here the level's gradient is cut into windows of kBwdWinRows rows
// and a workgroup owns one (level, window) pair and a contiguous run of samples:
// it accumulates the corners that fall in its window into LDS (ds_add_f32) and
// adds the rows it touched to global memory once.  Global atomics drop from one
// per (sample, corner) to one per (workgroup, touched row); every sample is
// re-read once per window of its level (20 B).  Same per-sample products as
// grid_bwd_kernel; the fp32 sums are re-associated, as atomics already are.
constexpr uint32_t kBwdLdsBytes = 128 * 1024;
constexpr uint32_t kBwdLevelWins = 24;        // levels needing more windows: direct atomics
struct BwdWindows {                           // level l owns windows [start[l], start[l+1])
    uint16_t start[kMaxLevels + 1];
    uint32_t nlevels;
};

template <uint32_t D, uint32_t C>
__global__ void __launch_bounds__(1024)
grid_bwd_lds_kernel(const float *__restrict__ grad, const float *__restrict__ inputs,
                    const int32_t *__restrict__ offsets, float *__restrict__ grad_emb,
                    uint32_t B, const LevelTable lt, uint32_t gridtype, int align_corners,
                    uint32_t interp, const BwdWindows wt, uint32_t per_block) {
    extern __shared__ float acc[];
    constexpr uint32_t kWin = kBwdLdsBytes / sizeof(float);        // floats per window
    uint32_t level = 0;
    while (level + 1 < wt.nlevels && wt.start[level + 1] <= blockIdx.y) ++level;
    const uint32_t win = blockIdx.y - wt.start[level];
    LevelParam q = lt.p[level];
    finish_level(q, offsets, level, D, gridtype, align_corners);
    const uint32_t n = q.hsize * C;
    const uint32_t lo = win * kWin;
    if (lo >= n) return;                                            // level smaller than planned
    const uint32_t hi = min(n, lo + kWin);
    // the last planned window of a level also takes any rows beyond the plan
    const bool last = blockIdx.y + 1 == wt.start[level + 1];
    float *gg = grad_emb + (size_t)q.offset * C;
    for (uint32_t i = threadIdx.x; i < hi - lo; i += blockDim.x) acc[i] = 0.0f;
    __syncthreads();
    const uint32_t b0 = blockIdx.x * per_block, b1 = min(B, b0 + per_block);
    for (uint32_t b = b0 + threadIdx.x; b < b1; b += blockDim.x) {
        float x[D];
        bool oob = false;
#pragma unroll
        for (uint32_t d = 0; d < D; ++d) {
            x[d] = inputs[(size_t)b * D + d];
            if (x[d] < 0 || x[d] > 1) oob = true;     // grad stays 0 (gridencoder.cu:277-282)
        }
        if (oob) continue;
        LevelCoord<D, C> lc;
        level_coord<D, C>(x, q, align_corners, interp, lc);
        float g[C];
#pragma unroll
        for (uint32_t c = 0; c < C; ++c) g[c] = grad[((size_t)level * B + b) * C + c];
#pragma unroll
        for (uint32_t idx = 0; idx < (1u << D); ++idx) {
            float w = 1.0f;
            uint32_t pl[D];
#pragma unroll
            for (uint32_t d = 0; d < D; ++d) {
                if ((idx & (1u << d)) == 0) {
                    w = __fmul_rn(w, __fsub_rn(1.0f, lc.pos[d]));
                    pl[d] = lc.pg[d];
                } else {
                    w = __fmul_rn(w, lc.pos[d]);
                    pl[d] = lc.pg[d] + 1;
                }
            }
            const uint32_t index = grid_index<D>(q, align_corners, pl) * C;
            if (index >= lo && index < hi) {
#pragma unroll
                for (uint32_t c = 0; c < C; ++c) atomicAdd(acc + (index - lo) + c, __fmul_rn(w, g[c]));
            } else if (last && index >= hi) {
#pragma unroll
                for (uint32_t c = 0; c < C; ++c) atomicAdd(gg + index + c, __fmul_rn(w, g[c]));
            }
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < hi - lo; i += blockDim.x) {
        const float v = acc[i];
        if (v != 0.0f) atomicAdd(gg + lo + i, v);
    }
}

template <uint32_t D, uint32_t C>
static int grid_fwd_launch(const float *in, const float *emb, const int32_t *off, float *out,
                           float *dydx, uint32_t B, uint32_t L, const LevelTable &lt,
                           uint32_t gt, int ac, uint32_t interp, hipStream_t st) {
    dim3 grid((B + 255) / 256, L);
    const int pair_ok = (reinterpret_cast<uintptr_t>(emb) & 7u) == 0;
    hipLaunchKernelGGL((grid_fwd_kernel<D, C>), grid, dim3(256), 0, st, in, emb, off, out, dydx,
                       B, L, lt, gt, ac, interp, pair_ok);
    return check_launch("grid_encode_forward");
}

template <uint32_t D, uint32_t C>
static int grid_bwd_launch(const float *grad, const float *in, const int32_t *off, float *gemb,
                           const float *dydx, float *gin, uint32_t B, uint32_t L,
                           const LevelTable &lt, uint32_t gt, int ac, uint32_t interp,
                           hipStream_t st) {
    // coarse levels go through LDS windows: a level holds at most (res+1)^D rows
    // rounded up to 8 (grid.py:117-128), so a level whose bound needs at most
    // kBwdLevelWins windows is planned that many (the device skips windows past
    // the level's real size, from `offsets`, and the last one adds any rows
    // beyond the plan directly).  The fine, hashed levels keep direct atomics:
    // their rows are spread over 4 MB tables (little same-address contention),
    // and re-reading every sample per window costs more than it saves
    // (measured: all 16 levels windowed 65 ms vs 39.5 ms at 3.1 M samples).
    // Below 4096 samples every level uses the direct atomics.
    const uint32_t win_rows = kBwdLdsBytes / sizeof(float) / C;
    BwdWindows wt;
    wt.nlevels = L;
    wt.start[0] = 0;
    uint64_t lds_levels = 0;
    for (uint32_t l = 0; l < L; ++l) {
        uint32_t nwin = 0;
        if (B >= 4096) {
            const double rows = std::pow((double)(ac ? lt.p[l].res : lt.p[l].res + 1),
                                         (double)D) + 8;
            const double need = std::ceil(rows / win_rows);
            if (need <= kBwdLevelWins) {
                nwin = (uint32_t)need;
                lds_levels |= 1ull << l;
            }
        }
        wt.start[l + 1] = (uint16_t)(wt.start[l] + nwin);
    }
    const uint32_t nwins = wt.start[L];
    if (nwins) {
        // ~256 workgroups over all windows, >= 4096 samples each
        const uint32_t nblk = std::max<uint32_t>(1, std::min<uint32_t>((B + 4095) / 4096,
                                                                     (256 + nwins - 1) / nwins));
        const uint32_t per_block = (B + nblk - 1) / nblk;
        static bool attr_set = false;   // > 64 KB of dynamic LDS must be opted into
        if (!attr_set) {
            if (hipFuncSetAttribute(reinterpret_cast<const void *>(&grid_bwd_lds_kernel<D, C>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)kBwdLdsBytes) != hipSuccess)
                return fail(SDFR_ELAUNCH, "grid_encode_backward: LDS attribute");
            attr_set = true;
        }
        hipLaunchKernelGGL((grid_bwd_lds_kernel<D, C>), dim3(nblk, nwins), dim3(1024),
                           kBwdLdsBytes, st, grad, in, off, gemb, B, lt, gt, ac, interp, wt,
                           per_block);
        int rc = check_launch("grid_encode_backward(lds windows)");
        if (rc) return rc;
    }
    int rc = SDFR_OK;
    if (lds_levels != (L == 64 ? ~0ull : (1ull << L) - 1ull)) {
        dim3 grid((B + 255) / 256, L);
        hipLaunchKernelGGL((grid_bwd_kernel<D, C>), grid, dim3(256), 0, st, grad, in, off, gemb,
                           B, lt, gt, ac, interp, lds_levels);
        rc = check_launch("grid_encode_backward");
    }
    if (rc || !dydx || !gin) return rc;
    hipLaunchKernelGGL((grid_input_bwd_kernel<D, C>), dim3((B * D + 255) / 256), dim3(256), 0,
                       st, grad, dydx, gin, B, L);
    return check_launch("grid_encode_backward(input)");
}

template <uint32_t D>
static int grid_fwd_dispatch_c(uint32_t C, const float *in, const float *emb, const int32_t *off,
                               float *out, float *dydx, uint32_t B, uint32_t L,
                               const LevelTable &lt, uint32_t gt, int ac, uint32_t interp,
                               hipStream_t st) {
    switch (C) {
        case 1: return grid_fwd_launch<D, 1>(in, emb, off, out, dydx, B, L, lt, gt, ac, interp, st);
        case 2: return grid_fwd_launch<D, 2>(in, emb, off, out, dydx, B, L, lt, gt, ac, interp, st);
        case 4: return grid_fwd_launch<D, 4>(in, emb, off, out, dydx, B, L, lt, gt, ac, interp, st);
        case 8: return grid_fwd_launch<D, 8>(in, emb, off, out, dydx, B, L, lt, gt, ac, interp, st);
    }
    return fail(SDFR_EINVAL, "GridEncoding: C must be 1, 2, 4, or 8.");
}

template <uint32_t D>
static int grid_bwd_dispatch_c(uint32_t C, const float *grad, const float *in, const int32_t *off,
                               float *gemb, const float *dydx, float *gin, uint32_t B, uint32_t L,
                               const LevelTable &lt, uint32_t gt, int ac, uint32_t interp,
                               hipStream_t st) {
    switch (C) {
        case 1: return grid_bwd_launch<D, 1>(grad, in, off, gemb, dydx, gin, B, L, lt, gt, ac, interp, st);
        case 2: return grid_bwd_launch<D, 2>(grad, in, off, gemb, dydx, gin, B, L, lt, gt, ac, interp, st);
        case 4: return grid_bwd_launch<D, 4>(grad, in, off, gemb, dydx, gin, B, L, lt, gt, ac, interp, st);
        case 8: return grid_bwd_launch<D, 8>(grad, in, off, gemb, dydx, gin, B, L, lt, gt, ac, interp, st);
    }
    return fail(SDFR_EINVAL, "GridEncoding: C must be 1, 2, 4, or 8.");
}

// ----------------------------------------------------------------------------
// SH encoder (degree <= 4), shencoder.cu:27-123
// ----------------------------------------------------------------------------
__device__ __forceinline__ void sh_eval(float x, float y, float z, uint32_t C, float *o) {
    const float xy = __fmul_rn(x, y), xz = __fmul_rn(x, z), yz = __fmul_rn(y, z);
    const float x2 = __fmul_rn(x, x), y2 = __fmul_rn(y, y), z2 = __fmul_rn(z, z);
    o[0] = 0.28209479177387814f;
    if (C <= 1) return;
    o[1] = __fmul_rn(-0.48860251190291987f, y);
    o[2] = __fmul_rn(0.48860251190291987f, z);
    o[3] = __fmul_rn(-0.48860251190291987f, x);
    if (C <= 2) return;
    o[4] = __fmul_rn(1.0925484305920792f, xy);
    o[5] = __fmul_rn(-1.0925484305920792f, yz);
    o[6] = __fmaf_rn(0.94617469575755997f, z2, -0.31539156525251999f);
    o[7] = __fmul_rn(-1.0925484305920792f, xz);
    o[8] = __fmaf_rn(0.54627421529603959f, x2, -__fmul_rn(0.54627421529603959f, y2));
    if (C <= 3) return;
    o[9] = __fmul_rn(__fmul_rn(0.59004358992664352f, y), __fmaf_rn(-3.0f, x2, y2));
    o[10] = __fmul_rn(__fmul_rn(2.8906114426405538f, xy), z);
    o[11] = __fmul_rn(__fmul_rn(0.45704579946446572f, y), __fmaf_rn(-5.0f, z2, 1.0f));
    o[12] = __fmul_rn(__fmul_rn(0.3731763325901154f, z), __fmaf_rn(5.0f, z2, -3.0f));
    o[13] = __fmul_rn(__fmul_rn(0.45704579946446572f, x), __fmaf_rn(-5.0f, z2, 1.0f));
    o[14] = __fmul_rn(__fmul_rn(1.4453057213202769f, z), __fsub_rn(x2, y2));
    o[15] = __fmul_rn(__fmul_rn(0.59004358992664352f, x), __fmaf_rn(3.0f, y2, -x2));
}

__device__ __forceinline__ void sh_eval_d(float x, float y, float z, uint32_t C, float *dx,
                                          float *dy, float *dz) {
    const float xy = __fmul_rn(x, y), xz = __fmul_rn(x, z), yz = __fmul_rn(y, z);
    const float x2 = __fmul_rn(x, x), y2 = __fmul_rn(y, y), z2 = __fmul_rn(z, z);
    dx[0] = 0.0f; dy[0] = 0.0f; dz[0] = 0.0f;
    if (C <= 1) return;
    dx[1] = 0.0f; dx[2] = 0.0f; dx[3] = -0.48860251190291992f;
    dy[1] = -0.48860251190291992f; dy[2] = 0.0f; dy[3] = 0.0f;
    dz[1] = 0.0f; dz[2] = 0.48860251190291992f; dz[3] = 0.0f;
    if (C <= 2) return;
    dx[4] = __fmul_rn(1.0925484305920792f, y); dx[5] = 0.0f; dx[6] = 0.0f;
    dx[7] = __fmul_rn(-1.0925484305920792f, z); dx[8] = __fmul_rn(1.0925484305920792f, x);
    dy[4] = __fmul_rn(1.0925484305920792f, x); dy[5] = __fmul_rn(-1.0925484305920792f, z);
    dy[6] = 0.0f; dy[7] = 0.0f; dy[8] = __fmul_rn(-1.0925484305920792f, y);
    dz[4] = 0.0f; dz[5] = __fmul_rn(-1.0925484305920792f, y);
    dz[6] = __fmul_rn(1.8923493915151202f, z); dz[7] = __fmul_rn(-1.0925484305920792f, x);
    dz[8] = 0.0f;
    if (C <= 3) return;
    dx[9] = __fmul_rn(-3.5402615395598609f, xy);
    dx[10] = __fmul_rn(2.8906114426405538f, yz);
    dx[11] = 0.0f;
    dx[12] = 0.0f;
    dx[13] = __fmaf_rn(-2.2852289973223288f, z2, 0.45704579946446572f);
    dx[14] = __fmul_rn(2.8906114426405538f, xz);
    dx[15] = __fmaf_rn(-1.7701307697799304f, x2, __fmul_rn(1.7701307697799304f, y2));
    dy[9] = __fmaf_rn(-1.7701307697799304f, x2, __fmul_rn(1.7701307697799304f, y2));
    dy[10] = __fmul_rn(2.8906114426405538f, xz);
    dy[11] = __fmaf_rn(-2.2852289973223288f, z2, 0.45704579946446572f);
    dy[12] = 0.0f;
    dy[13] = 0.0f;
    dy[14] = __fmul_rn(-2.8906114426405538f, yz);
    dy[15] = __fmul_rn(3.5402615395598609f, xy);
    dz[9] = 0.0f;
    dz[10] = __fmul_rn(2.8906114426405538f, xy);
    dz[11] = __fmul_rn(-4.5704579946446566f, yz);
    dz[12] = __fmaf_rn(5.597644988851731f, z2, -1.1195289977703462f);
    dz[13] = __fmul_rn(-4.5704579946446566f, xz);
    dz[14] = __fmaf_rn(1.4453057213202769f, x2, -__fmul_rn(1.4453057213202769f, y2));
    dz[15] = 0.0f;
}

__global__ void __launch_bounds__(256)
sh_fwd_kernel(const float *__restrict__ inputs, float *__restrict__ outputs,
              float *__restrict__ dy_dx, uint32_t B, uint32_t C) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const float x = inputs[(size_t)b * 3], y = inputs[(size_t)b * 3 + 1],
                z = inputs[(size_t)b * 3 + 2];
    const uint32_t C2 = C * C;
    float o[16];
    sh_eval(x, y, z, C, o);
    for (uint32_t i = 0; i < C2; ++i) outputs[(size_t)b * C2 + i] = o[i];
    if (dy_dx) {
        float dx[16], dy[16], dz[16];
        sh_eval_d(x, y, z, C, dx, dy, dz);
        float *p = dy_dx + (size_t)b * 3 * C2;
        for (uint32_t i = 0; i < C2; ++i) {
            p[i] = dx[i];
            p[C2 + i] = dy[i];
            p[2 * C2 + i] = dz[i];
        }
    }
}

__global__ void __launch_bounds__(256)
sh_bwd_kernel(const float *__restrict__ grad, const float *__restrict__ dy_dx,
              float *__restrict__ grad_inputs, uint32_t B, uint32_t C) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t b = t / 3;
    if (b >= B) return;
    const uint32_t d = t - b * 3, C2 = C * C;
    const float *g = grad + (size_t)b * C2;
    const float *dd = dy_dx + (size_t)b * 3 * C2 + d * C2;
    float acc = grad_inputs[t];
    for (uint32_t ch = 0; ch < C2; ++ch) acc = __fmaf_rn(g[ch], dd[ch], acc);
    grad_inputs[t] = acc;
}

}  // namespace sdfr

using namespace sdfr;

extern "C" {

int sdfr_abi_version(void) { return SDFR_ABI_VERSION; }

const char *sdfr_last_error(void) { return g_last_error.c_str(); }

int sdfr_grid_encode_forward(const float *inputs, const float *embeddings,
                             const int32_t *offsets, float *outputs, uint32_t B, uint32_t D,
                             uint32_t C, uint32_t L, float S, uint32_t H, float *dy_dx,
                             uint32_t gridtype, int align_corners, uint32_t interp,
                             void *stream) {
    if (D < 2 || D > 5) return fail(SDFR_EINVAL, "GridEncoding: D must be 2, 3, 4, or 5.");
    if (!(C == 1 || C == 2 || C == 4 || C == 8))
        return fail(SDFR_EINVAL, "GridEncoding: C must be 1, 2, 4, or 8.");
    if (L == 0 || L > (uint32_t)kMaxLevels)
        return fail(SDFR_EINVAL, "GridEncoding: 1 <= L <= 64 levels supported.");
    if (B == 0) return SDFR_OK;   // empty batch: nothing to launch (tensors may be NULL)
    if (!inputs || !embeddings || !offsets || !outputs)
        return fail(SDFR_EINVAL, "grid_encode_forward: null tensor pointer");
    hipStream_t st = (hipStream_t)stream;
    LevelTable lt;
    make_level_table(L, S, H, lt);
    switch (D) {
        case 2: return grid_fwd_dispatch_c<2>(C, inputs, embeddings, offsets, outputs, dy_dx, B, L, lt, gridtype, align_corners, interp, st);
        case 3: return grid_fwd_dispatch_c<3>(C, inputs, embeddings, offsets, outputs, dy_dx, B, L, lt, gridtype, align_corners, interp, st);
        case 4: return grid_fwd_dispatch_c<4>(C, inputs, embeddings, offsets, outputs, dy_dx, B, L, lt, gridtype, align_corners, interp, st);
        default: return grid_fwd_dispatch_c<5>(C, inputs, embeddings, offsets, outputs, dy_dx, B, L, lt, gridtype, align_corners, interp, st);
    }
}

int sdfr_grid_encode_backward(const float *grad, const float *inputs, const float *embeddings,
                              const int32_t *offsets, float *grad_embeddings, uint32_t B,
                              uint32_t D, uint32_t C, uint32_t L, float S, uint32_t H,
                              const float *dy_dx, float *grad_inputs, uint32_t gridtype,
                              int align_corners, uint32_t interp, void *stream) {
    (void)embeddings;
    if (D < 2 || D > 5) return fail(SDFR_EINVAL, "GridEncoding: D must be 2, 3, 4, or 5.");
    if (!(C == 1 || C == 2 || C == 4 || C == 8))
        return fail(SDFR_EINVAL, "GridEncoding: C must be 1, 2, 4, or 8.");
    if (L == 0 || L > (uint32_t)kMaxLevels)
        return fail(SDFR_EINVAL, "GridEncoding: 1 <= L <= 64 levels supported.");
    if (B == 0) return SDFR_OK;
    if (!grad || !inputs || !offsets || !grad_embeddings)
        return fail(SDFR_EINVAL, "grid_encode_backward: null tensor pointer");
    if ((dy_dx == nullptr) != (grad_inputs == nullptr))
        return fail(SDFR_EINVAL, "grid_encode_backward: dy_dx and grad_inputs go together");
    hipStream_t st = (hipStream_t)stream;
    LevelTable lt;
    make_level_table(L, S, H, lt);
    switch (D) {
        case 2: return grid_bwd_dispatch_c<2>(C, grad, inputs, offsets, grad_embeddings, dy_dx, grad_inputs, B, L, lt, gridtype, align_corners, interp, st);
        case 3: return grid_bwd_dispatch_c<3>(C, grad, inputs, offsets, grad_embeddings, dy_dx, grad_inputs, B, L, lt, gridtype, align_corners, interp, st);
        case 4: return grid_bwd_dispatch_c<4>(C, grad, inputs, offsets, grad_embeddings, dy_dx, grad_inputs, B, L, lt, gridtype, align_corners, interp, st);
        default: return grid_bwd_dispatch_c<5>(C, grad, inputs, offsets, grad_embeddings, dy_dx, grad_inputs, B, L, lt, gridtype, align_corners, interp, st);
    }
}

int sdfr_sh_encode_forward(const float *inputs, float *outputs, uint32_t B, uint32_t D,
                           uint32_t C, float *dy_dx, void *stream) {
    if (D != 3) return fail(SDFR_EINVAL, "SH encoder only support input dim == 3");
    if (C < 1 || C > 8) return fail(SDFR_EINVAL, "SH encoder only supports degree in [1, 8]");
    if (C > 4) return fail(SDFR_EUNSUPPORTED, "sdfr: SH degree > 4 not implemented");
    if (B == 0) return SDFR_OK;
    if (!inputs || !outputs) return fail(SDFR_EINVAL, "sh_encode_forward: null tensor pointer");
    hipLaunchKernelGGL(sh_fwd_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       inputs, outputs, dy_dx, B, C);
    return check_launch("sh_encode_forward");
}

int sdfr_sh_encode_backward(const float *grad, const float *inputs, uint32_t B, uint32_t D,
                            uint32_t C, const float *dy_dx, float *grad_inputs, void *stream) {
    (void)inputs;
    if (D != 3) return fail(SDFR_EINVAL, "SH encoder only support input dim == 3");
    if (C < 1 || C > 8) return fail(SDFR_EINVAL, "SH encoder only supports degree in [1, 8]");
    if (C > 4) return fail(SDFR_EUNSUPPORTED, "sdfr: SH degree > 4 not implemented");
    if (B == 0) return SDFR_OK;
    if (!grad || !dy_dx || !grad_inputs)
        return fail(SDFR_EINVAL, "sh_encode_backward: null tensor pointer");
    hipLaunchKernelGGL(sh_bwd_kernel, dim3((B * 3 + 255) / 256), dim3(256), 0,
                       (hipStream_t)stream, grad, dy_dx, grad_inputs, B, C);
    return check_launch("sh_encode_backward");
}

}  // extern "C"
