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
#include <utility>

#include "sdfr_common.h"
#include "sdfr_scan.h"

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

// Table gradient, binned (B >= 4096, D <= 3, with a workspace).  Direct fp32
// atomics ran at ~15 G adds/s on the hashed levels whatever the sample order
// (uniform random and the renderer's tile order alike: 39.7 / 35.5 ms for 3.1 M
// samples x 16 levels x 8 corners x 2 channels), i.e. the atomic path itself,
// not address contention, was the limit; and the coarse levels' LDS windows
// (grid_bwd_lds_kernel) re-evaluate every sample once per window.  Here every
// (sample, level, corner) contribution becomes one entry (row, w * grad[C]),
// counting-sorted into 32 bins of 2^sh rows per level (sh = log2 of the LDS
// window unless the level has more rows), and each bin is summed in LDS
// (ds_add_f32) and added to the table once.  Five launches:
//   grid_bin_count_kernel     per (block of samples, level): entries per bin
//   exclusive_scan_u32        counts, laid out [level][bin][block], -> offsets
//   grid_bin_scatter_kernel   recompute the entries, counting-sort them per
//                             block in LDS, write each bin's run contiguously
//   grid_bin_plan_kernel      cut every bin into work items (bin_chunk: a
//                             coarse level's single bin holds all of its B x 8
//                             entries; a hashed bin ~B x 8 / 32)
//   grid_bin_accum_kernel     per item: LDS window sums -> table, plain
//                             read-modify-write when the item is its whole bin
//                             (rows owned by one workgroup), else atomics on
//                             the touched rows only.  Bound by the LDS float
//                             atomics (4.6 ms at 3.1 M samples; 1.3 ms with
//                             plain, racy LDS adds = the streaming floor)
// HBM traffic per entry: 4 + 4C bytes written and read once (3.3 GB at 3.1 M
// samples x 11 hashed levels), plus the inputs twice and the gradient once.
// The per-entry products are grid_bwd_kernel's; the fp32 sums are
// re-associated, as the reference's atomics are.
constexpr uint32_t kBinCount = 32;
constexpr uint32_t kBinThreads = 256;
constexpr uint32_t kBinAccThreads = 1024;
constexpr uint32_t kBinLdsBytes = 128 * 1024;
template <uint32_t C>
constexpr uint32_t bin_rows() { return kBinLdsBytes / (4 * C); }   // LDS window (rows)
template <uint32_t C>
constexpr uint32_t bin_it() { return C <= 2 ? 2 : 1; }              // samples per thread
template <uint32_t C>
constexpr uint32_t bin_spb() { return kBinThreads * bin_it<C>(); }  // samples per block

struct BinLevels {
    uint8_t level[kMaxLevels];
    uint32_t n;
};

// the smallest sh >= log2(window) with hsize <= kBinCount << sh
template <uint32_t C>
__device__ __forceinline__ uint32_t bin_shift(uint32_t hsize) {
    uint32_t sh = 31u - __builtin_clz(bin_rows<C>());
    while (((uint64_t)kBinCount << sh) < hsize) ++sh;
    return sh;
}

// rows and interpolation weights of a sample's 2^D corners (grid_bwd_kernel's)
template <uint32_t D, uint32_t C>
__device__ __forceinline__ bool sample_corners(const float *__restrict__ inputs, uint32_t b,
                                               const LevelParam &q, int align_corners,
                                               uint32_t interp, uint32_t (&row)[1u << D],
                                               float (&w)[1u << D]) {
    float x[D];
#pragma unroll
    for (uint32_t d = 0; d < D; ++d) {
        x[d] = inputs[(size_t)b * D + d];
        if (x[d] < 0 || x[d] > 1) return false;     // grad stays 0 (gridencoder.cu:277-282)
    }
    LevelCoord<D, C> lc;
    level_coord<D, C>(x, q, align_corners, interp, lc);
#pragma unroll
    for (uint32_t idx = 0; idx < (1u << D); ++idx) {
        float wi = 1.0f;
        uint32_t pl[D];
#pragma unroll
        for (uint32_t d = 0; d < D; ++d) {
            if ((idx & (1u << d)) == 0) {
                wi = __fmul_rn(wi, __fsub_rn(1.0f, lc.pos[d]));
                pl[d] = lc.pg[d];
            } else {
                wi = __fmul_rn(wi, lc.pos[d]);
                pl[d] = lc.pg[d] + 1;
            }
        }
        w[idx] = wi;
        row[idx] = grid_index<D>(q, align_corners, pl);
    }
    return true;
}

template <uint32_t D, uint32_t C>
__global__ void __launch_bounds__(kBinThreads)
grid_bin_count_kernel(const float *__restrict__ inputs, const int32_t *__restrict__ offsets,
                      uint32_t B, const LevelTable lt, uint32_t gridtype, int align_corners,
                      uint32_t interp, const BinLevels bl, uint32_t *__restrict__ cnt) {
    __shared__ uint32_t hist[kBinCount];
    const uint32_t li = blockIdx.y, level = bl.level[li];
    LevelParam q = lt.p[level];
    finish_level(q, offsets, level, D, gridtype, align_corners);
    const uint32_t sh = bin_shift<C>(q.hsize);
    if (threadIdx.x < kBinCount) hist[threadIdx.x] = 0;
    __syncthreads();
#pragma unroll
    for (uint32_t it = 0; it < bin_it<C>(); ++it) {
        const uint32_t b = blockIdx.x * bin_spb<C>() + it * kBinThreads + threadIdx.x;
        uint32_t row[1u << D];
        float w[1u << D];
        if (b < B && sample_corners<D, C>(inputs, b, q, align_corners, interp, row, w))
#pragma unroll
            for (uint32_t idx = 0; idx < (1u << D); ++idx) atomicAdd(&hist[row[idx] >> sh], 1u);
    }
    __syncthreads();
    if (threadIdx.x < kBinCount)
        cnt[((size_t)li * kBinCount + threadIdx.x) * gridDim.x + blockIdx.x] = hist[threadIdx.x];
}

template <uint32_t D, uint32_t C>
__global__ void __launch_bounds__(kBinThreads)
grid_bin_scatter_kernel(const float *__restrict__ grad, const float *__restrict__ inputs,
                        const int32_t *__restrict__ offsets, uint32_t B, const LevelTable lt,
                        uint32_t gridtype, int align_corners, uint32_t interp, const BinLevels bl,
                        const uint32_t *__restrict__ ofs, uint32_t *__restrict__ e_row,
                        float *__restrict__ e_val) {
    constexpr uint32_t K = 1u << D, IT = bin_it<C>(), E = kBinThreads * IT * K;
    __shared__ uint32_t hist[kBinCount], lofs[kBinCount + 1];
    __shared__ uint32_t s_row[E];
    __shared__ float s_val[E * C];
    const uint32_t li = blockIdx.y, level = bl.level[li];
    LevelParam q = lt.p[level];
    finish_level(q, offsets, level, D, gridtype, align_corners);
    const uint32_t sh = bin_shift<C>(q.hsize);
    if (threadIdx.x < kBinCount) hist[threadIdx.x] = 0;
    __syncthreads();
    uint32_t row[IT][K], slot[IT][K];
    float w[IT][K], g[IT][C];
    bool ok[IT];
#pragma unroll
    for (uint32_t it = 0; it < IT; ++it) {
        const uint32_t b = blockIdx.x * bin_spb<C>() + it * kBinThreads + threadIdx.x;
        ok[it] = b < B && sample_corners<D, C>(inputs, b, q, align_corners, interp, row[it], w[it]);
        if (ok[it]) {
#pragma unroll
            for (uint32_t c = 0; c < C; ++c) g[it][c] = grad[((size_t)level * B + b) * C + c];
#pragma unroll
            for (uint32_t idx = 0; idx < K; ++idx)
                slot[it][idx] = atomicAdd(&hist[row[it][idx] >> sh], 1u);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (uint32_t k = 0; k < kBinCount; ++k) {
            lofs[k] = run;
            run += hist[k];
        }
        lofs[kBinCount] = run;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t it = 0; it < IT; ++it) {
        if (!ok[it]) continue;
#pragma unroll
        for (uint32_t idx = 0; idx < K; ++idx) {
            const uint32_t p = lofs[row[it][idx] >> sh] + slot[it][idx];
            s_row[p] = row[it][idx];
#pragma unroll
            for (uint32_t c = 0; c < C; ++c) s_val[p * C + c] = __fmul_rn(w[it][idx], g[it][c]);
        }
    }
    __syncthreads();
    const uint32_t total = lofs[kBinCount];
    for (uint32_t i = threadIdx.x; i < total; i += kBinThreads) {
        uint32_t lo = 0, hi = kBinCount;     // the last bin starting at or before i
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (lofs[mid] <= i) lo = mid;
            else hi = mid;
        }
        const size_t gp = ofs[((size_t)li * kBinCount + lo) * gridDim.x + blockIdx.x] + (i - lofs[lo]);
        e_row[gp] = s_row[i];
#pragma unroll
        for (uint32_t c = 0; c < C; ++c) e_val[gp * C + c] = s_val[i * C + c];
    }
}

// Entries per work item: bins are cut into pieces of ~2x the mean bin size, at
// least kBinChunkMin and at most kBinChunkMax entries.  A coarse level's single
// bin holds all of its B x 8 entries while a hashed bin holds ~B x 8 / 32, so at a
// training chunk (~196 K samples) a fixed 1 M cut left two items per coarse level
// -- a few CUs summing 1 M entries each while the rest idled.  Splitting costs one
// atomic write-back of the window per extra item, so hashed bins (near the mean)
// stay whole and keep the plain read-modify-write.
constexpr uint32_t kBinChunkMin = 1u << 16;
constexpr uint32_t kBinChunkMax = 1u << 20;
static uint32_t bin_chunk(uint64_t E, uint32_t npairs) {
    const uint64_t c = 2 * E / std::max<uint32_t>(npairs, 1u);
    return (uint32_t)std::min<uint64_t>(kBinChunkMax, std::max<uint64_t>(kBinChunkMin, c));
}

struct BinItem {
    uint32_t pair;     // level index * kBinCount + bin
    uint32_t start, end;
    uint32_t whole;    // the item is its bin's only one
};

// one workgroup: cut each (level, bin) entry run into items of <= chunk entries
__global__ void __launch_bounds__(kScanThreads)
grid_bin_plan_kernel(const uint32_t *__restrict__ ofs, uint32_t nblk, uint32_t npairs,
                     uint32_t chunk, BinItem *__restrict__ items, uint32_t *__restrict__ nitems) {
    uint32_t carry = 0;
    for (uint32_t p0 = 0; p0 < npairs; p0 += kScanThreads) {
        const uint32_t p = p0 + threadIdx.x;
        uint32_t s = 0, e = 0, n = 0;
        if (p < npairs) {
            s = ofs[(size_t)p * nblk];
            e = ofs[(size_t)(p + 1) * nblk];
            n = (e - s + chunk - 1) / chunk;
        }
        uint32_t ex;
        const uint32_t tot = block_exscan(n, ex);
        for (uint32_t k = 0; k < n; ++k) {
            const uint32_t a = s + k * chunk;
            items[carry + ex + k] = BinItem{p, a, min(e, a + chunk), n == 1 ? 1u : 0u};
        }
        carry += tot;
    }
    if (threadIdx.x == 0) *nitems = carry;
}

template <uint32_t C>
__global__ void __launch_bounds__(kBinAccThreads)
grid_bin_accum_kernel(const int32_t *__restrict__ offsets, const LevelTable lt, uint32_t D,
                      uint32_t gridtype, int align_corners, const BinLevels bl,
                      const BinItem *__restrict__ items, const uint32_t *__restrict__ nitems,
                      const uint32_t *__restrict__ e_row, const float *__restrict__ e_val,
                      float *__restrict__ grad_emb) {
    extern __shared__ float acc[];
    constexpr uint32_t R = bin_rows<C>();
    constexpr uint32_t U = 4;                    // entries in flight per thread
    if (blockIdx.x >= *nitems) return;
    const BinItem it = items[blockIdx.x];
    const uint32_t li = it.pair / kBinCount, bin = it.pair % kBinCount, level = bl.level[li];
    LevelParam q = lt.p[level];
    finish_level(q, offsets, level, D, gridtype, align_corners);
    const uint32_t sh = bin_shift<C>(q.hsize);
    const uint64_t base = (uint64_t)bin << sh;
    if (base >= q.hsize) return;
    const uint32_t end_row = (uint32_t)min((uint64_t)q.hsize, base + (1ull << sh));
    float *gg = grad_emb + (size_t)q.offset * C;
    // one sweep when the bin fits the LDS window (sh = log2 R), more for bigger tables
    for (uint32_t w0 = (uint32_t)base; w0 < end_row; w0 += R) {
        for (uint32_t i = threadIdx.x; i < R * C; i += kBinAccThreads) acc[i] = 0.0f;
        __syncthreads();
        for (uint32_t i0 = it.start + threadIdx.x; i0 < it.end; i0 += U * kBinAccThreads) {
            uint32_t r[U];
            float v[U][C];
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) {
                const uint32_t i = i0 + u * kBinAccThreads;
                r[u] = i < it.end ? e_row[i] - w0 : R;
#pragma unroll
                for (uint32_t c = 0; c < C; ++c) v[u][c] = i < it.end ? e_val[(size_t)i * C + c] : 0.0f;
            }
#pragma unroll
            for (uint32_t u = 0; u < U; ++u)
                if (r[u] < R)
#pragma unroll
                    for (uint32_t c = 0; c < C; ++c) atomicAdd(&acc[r[u] * C + c], v[u][c]);
        }
        __syncthreads();
        const uint32_t n = min(R, end_row - w0) * C;
        for (uint32_t i = threadIdx.x; i < n; i += kBinAccThreads) {
            const float v = acc[i];
            if (v == 0.0f) continue;
            if (it.whole) gg[(size_t)w0 * C + i] += v;     // rows owned by this workgroup
            else atomicAdd(gg + (size_t)w0 * C + i, v);
        }
        __syncthreads();
    }
}

// workspace of the binned path: counts [n_b][32][nblk] + 1, scan scratch,
// entries, work items
struct BinPlan {
    uint32_t nblk, n, max_items, chunk;
    uint64_t M, E;
    size_t cnt_off, bsum_off, row_off, val_off, item_off, nitem_off, bytes;
};

static size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

template <uint32_t C>
static BinPlan bin_plan(uint32_t B, uint32_t D, uint32_t n_b) {
    BinPlan p{};
    p.n = n_b;
    p.nblk = (B + bin_spb<C>() - 1) / bin_spb<C>();
    p.M = (uint64_t)n_b * kBinCount * p.nblk;
    p.E = (uint64_t)B * (1u << D) * n_b;
    p.cnt_off = 0;
    p.bsum_off = align256((p.M + 1) * sizeof(uint32_t));
    p.row_off = p.bsum_off + align256((size_t)scan_block_sums(p.M) * sizeof(uint32_t));
    p.val_off = p.row_off + align256(p.E * sizeof(uint32_t));
    p.chunk = bin_chunk(p.E, n_b * kBinCount);
    p.max_items = (uint32_t)(n_b * kBinCount + (p.E + p.chunk - 1) / p.chunk);
    p.item_off = p.val_off + align256(p.E * C * sizeof(float));
    p.nitem_off = p.item_off + align256((size_t)p.max_items * sizeof(BinItem));
    p.bytes = p.nitem_off + 256;
    return p;
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

// levels of the LDS-window path (bit mask) and the binned levels, as grid_bwd_launch plans them
template <uint32_t D, uint32_t C>
static uint64_t window_levels(uint32_t B, uint32_t L, const LevelTable &lt, int ac,
                              BwdWindows *wt) {
    const uint32_t win_rows = kBwdLdsBytes / sizeof(float) / C;
    uint64_t lds_levels = 0;
    if (wt) {
        wt->nlevels = L;
        wt->start[0] = 0;
    }
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
        if (wt) wt->start[l + 1] = (uint16_t)(wt->start[l] + nwin);
    }
    return lds_levels;
}

// binned path applies: D <= 3 (LDS staging of 2^D corners per sample), B >= 4096,
// and the entry count fits the uint32 scan; it then takes every level
template <uint32_t D, uint32_t C>
static bool bin_levels(uint32_t B, uint32_t L, BinLevels &bl) {
    bl.n = 0;
    if (D > 3 || B < 4096) return false;
    for (uint32_t l = 0; l < L; ++l) bl.level[bl.n++] = (uint8_t)l;
    return (uint64_t)B * (1u << D) * bl.n < (1ull << 32) - 1;
}

template <uint32_t D, uint32_t C>
static size_t grid_bwd_ws_bytes_t(uint32_t B, uint32_t L) {
    BinLevels bl;
    if (!bin_levels<D, C>(B, L, bl)) return 0;
    return bin_plan<C>(B, D, bl.n).bytes;
}

template <uint32_t D, uint32_t C>
static int grid_bin_launch(const float *grad, const float *in, const int32_t *off, float *gemb,
                           uint32_t B, const LevelTable &lt, uint32_t gt, int ac, uint32_t interp,
                           const BinLevels &bl, void *ws, hipStream_t st) {
    if constexpr (D <= 3) {
        const BinPlan p = bin_plan<C>(B, D, bl.n);
        char *w = (char *)ws;
        uint32_t *cnt = (uint32_t *)(w + p.cnt_off), *bsum = (uint32_t *)(w + p.bsum_off);
        uint32_t *e_row = (uint32_t *)(w + p.row_off);
        float *e_val = (float *)(w + p.val_off);
        const dim3 grid(p.nblk, bl.n);
        hipLaunchKernelGGL((grid_bin_count_kernel<D, C>), grid, dim3(kBinThreads), 0, st, in, off,
                           B, lt, gt, ac, interp, bl, cnt);
        exclusive_scan_u32(cnt, p.M, bsum, st);
        hipLaunchKernelGGL((grid_bin_scatter_kernel<D, C>), grid, dim3(kBinThreads), 0, st, grad,
                           in, off, B, lt, gt, ac, interp, bl, cnt, e_row, e_val);
        // > 64 KB of dynamic LDS must be opted into; the attribute is per device, so it
        // is set on every call (a host-side call, not a stream op, capture-safe)
        if (hipFuncSetAttribute(reinterpret_cast<const void *>(&grid_bin_accum_kernel<C>),
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)kBinLdsBytes) != hipSuccess)
            return fail(SDFR_ELAUNCH, "grid_encode_backward: LDS attribute (bins)");
        BinItem *items = (BinItem *)(w + p.item_off);
        uint32_t *nitems = (uint32_t *)(w + p.nitem_off);
        hipLaunchKernelGGL(grid_bin_plan_kernel, dim3(1), dim3(kScanThreads), 0, st, cnt, p.nblk,
                           bl.n * kBinCount, p.chunk, items, nitems);
        hipLaunchKernelGGL((grid_bin_accum_kernel<C>), dim3(p.max_items), dim3(kBinAccThreads),
                           kBinLdsBytes, st, off, lt, D, gt, ac, bl, items, nitems, e_row, e_val,
                           gemb);
        return check_launch("grid_encode_backward(bins)");
    } else {
        return fail(SDFR_EINVAL, "grid_encode_backward: binned path needs D <= 3");
    }
}

template <uint32_t D, uint32_t C>
static int grid_bwd_launch(const float *grad, const float *in, const int32_t *off, float *gemb,
                           const float *dydx, float *gin, uint32_t B, uint32_t L,
                           const LevelTable &lt, uint32_t gt, int ac, uint32_t interp,
                           void *ws, size_t ws_bytes, hipStream_t st) {
    int rc = SDFR_OK;
    BinLevels bl;
    if (!gemb) {
        // input gradient only (grad_embeddings NULL): the table gradient is skipped
    } else if (ws && bin_levels<D, C>(B, L, bl) && ws_bytes >= bin_plan<C>(B, D, bl.n).bytes) {
        // every level binned (the per-level table gradient above)
        rc = grid_bin_launch<D, C>(grad, in, off, gemb, B, lt, gt, ac, interp, bl, ws, st);
    } else {
        // without a workspace: coarse levels through LDS windows -- a level holds at
        // most (res+1)^D rows rounded up to 8 (grid.py:117-128), so a level whose
        // bound needs at most kBwdLevelWins windows is planned that many (the device
        // skips windows past the level's real size, from `offsets`, and the last one
        // adds any rows beyond the plan directly); the fine, hashed levels by direct
        // atomics.  Below 4096 samples every level uses the direct atomics.
        BwdWindows wt;
        const uint64_t lds_levels = window_levels<D, C>(B, L, lt, ac, &wt);
        const uint32_t nwins = wt.start[L];
        if (nwins) {
            // ~256 workgroups over all windows, >= 4096 samples each
            const uint32_t nblk = std::max<uint32_t>(
                1, std::min<uint32_t>((B + 4095) / 4096, (256 + nwins - 1) / nwins));
            const uint32_t per_block = (B + nblk - 1) / nblk;
            // > 64 KB of dynamic LDS: opted into per call (the attribute is per device)
            if (hipFuncSetAttribute(reinterpret_cast<const void *>(&grid_bwd_lds_kernel<D, C>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)kBwdLdsBytes) != hipSuccess)
                return fail(SDFR_ELAUNCH, "grid_encode_backward: LDS attribute");
            hipLaunchKernelGGL((grid_bwd_lds_kernel<D, C>), dim3(nblk, nwins), dim3(1024),
                               kBwdLdsBytes, st, grad, in, off, gemb, B, lt, gt, ac, interp, wt,
                               per_block);
            rc = check_launch("grid_encode_backward(lds windows)");
            if (rc) return rc;
        }
        if (lds_levels != (L == 64 ? ~0ull : (1ull << L) - 1ull)) {
            dim3 grid((B + 255) / 256, L);
            hipLaunchKernelGGL((grid_bwd_kernel<D, C>), grid, dim3(256), 0, st, grad, in, off,
                               gemb, B, lt, gt, ac, interp, lds_levels);
            rc = check_launch("grid_encode_backward");
        }
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
                               void *ws, size_t wsb, hipStream_t st) {
    switch (C) {
        case 1: return grid_bwd_launch<D, 1>(grad, in, off, gemb, dydx, gin, B, L, lt, gt, ac, interp, ws, wsb, st);
        case 2: return grid_bwd_launch<D, 2>(grad, in, off, gemb, dydx, gin, B, L, lt, gt, ac, interp, ws, wsb, st);
        case 4: return grid_bwd_launch<D, 4>(grad, in, off, gemb, dydx, gin, B, L, lt, gt, ac, interp, ws, wsb, st);
        case 8: return grid_bwd_launch<D, 8>(grad, in, off, gemb, dydx, gin, B, L, lt, gt, ac, interp, ws, wsb, st);
    }
    return fail(SDFR_EINVAL, "GridEncoding: C must be 1, 2, 4, or 8.");
}

template <uint32_t D>
static size_t grid_bwd_ws_dispatch_c(uint32_t C, uint32_t B, uint32_t L) {
    switch (C) {
        case 1: return grid_bwd_ws_bytes_t<D, 1>(B, L);
        case 2: return grid_bwd_ws_bytes_t<D, 2>(B, L);
        case 4: return grid_bwd_ws_bytes_t<D, 4>(B, L);
        case 8: return grid_bwd_ws_bytes_t<D, 8>(B, L);
    }
    return 0;
}

// ----------------------------------------------------------------------------
// SH encoder, shencoder.cu:27-355 (bands 0..3 term by term below, bands 4..7 from
// sh_bands.h)
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

// bands 4..7 (degrees 5..8): generated by csrc/sh_gen.py from the Legendre
// recurrence, same band convention as the terms above
#define SDFR_SH_FN static __device__ __forceinline__
#include "sh_bands.h"
#undef SDFR_SH_FN

// MAXC2 = 16 (degree <= 4, SDFace's) or 64 (degrees 5..8)
template <uint32_t MAXC2>
__global__ void __launch_bounds__(256)
sh_fwd_kernel(const float *__restrict__ inputs, float *__restrict__ outputs,
              float *__restrict__ dy_dx, uint32_t B, uint32_t C) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const float x = inputs[(size_t)b * 3], y = inputs[(size_t)b * 3 + 1],
                z = inputs[(size_t)b * 3 + 2];
    const uint32_t C2 = C * C;
    float o[MAXC2];
    sh_eval(x, y, z, C, o);
    if constexpr (MAXC2 > 16) sdfr_sh_bands_4_7(x, y, z, C, o, nullptr, nullptr, nullptr);
    for (uint32_t i = 0; i < C2; ++i) outputs[(size_t)b * C2 + i] = o[i];
    if (dy_dx) {
        float dx[MAXC2], dy[MAXC2], dz[MAXC2];
        sh_eval_d(x, y, z, C, dx, dy, dz);
        if constexpr (MAXC2 > 16) sdfr_sh_bands_4_7(x, y, z, C, o, dx, dy, dz);
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

size_t sdfr_grid_encode_backward_ws_bytes(uint32_t B, uint32_t D, uint32_t C, uint32_t L,
                                          float S, uint32_t H, int align_corners) {
    if (D < 2 || D > 3 || !(C == 1 || C == 2 || C == 4 || C == 8) || L == 0 ||
        L > (uint32_t)kMaxLevels)
        return 0;
    (void)S;
    (void)H;
    (void)align_corners;
    return D == 2 ? grid_bwd_ws_dispatch_c<2>(C, B, L) : grid_bwd_ws_dispatch_c<3>(C, B, L);
}

int sdfr_grid_encode_backward_ws(const float *grad, const float *inputs, const float *embeddings,
                                 const int32_t *offsets, float *grad_embeddings, uint32_t B,
                                 uint32_t D, uint32_t C, uint32_t L, float S, uint32_t H,
                                 const float *dy_dx, float *grad_inputs, uint32_t gridtype,
                                 int align_corners, uint32_t interp, void *ws, size_t ws_bytes,
                                 void *stream) {
    (void)embeddings;
    if (D < 2 || D > 5) return fail(SDFR_EINVAL, "GridEncoding: D must be 2, 3, 4, or 5.");
    if (!(C == 1 || C == 2 || C == 4 || C == 8))
        return fail(SDFR_EINVAL, "GridEncoding: C must be 1, 2, 4, or 8.");
    if (L == 0 || L > (uint32_t)kMaxLevels)
        return fail(SDFR_EINVAL, "GridEncoding: 1 <= L <= 64 levels supported.");
    if (B == 0) return SDFR_OK;
    if (!grad || !inputs || !offsets || (!grad_embeddings && !grad_inputs))
        return fail(SDFR_EINVAL, "grid_encode_backward: null tensor pointer");
    if ((dy_dx == nullptr) != (grad_inputs == nullptr))
        return fail(SDFR_EINVAL, "grid_encode_backward: dy_dx and grad_inputs go together");
    hipStream_t st = (hipStream_t)stream;
    LevelTable lt;
    make_level_table(L, S, H, lt);
    switch (D) {
        case 2: return grid_bwd_dispatch_c<2>(C, grad, inputs, offsets, grad_embeddings, dy_dx, grad_inputs, B, L, lt, gridtype, align_corners, interp, ws, ws_bytes, st);
        case 3: return grid_bwd_dispatch_c<3>(C, grad, inputs, offsets, grad_embeddings, dy_dx, grad_inputs, B, L, lt, gridtype, align_corners, interp, ws, ws_bytes, st);
        case 4: return grid_bwd_dispatch_c<4>(C, grad, inputs, offsets, grad_embeddings, dy_dx, grad_inputs, B, L, lt, gridtype, align_corners, interp, ws, ws_bytes, st);
        default: return grid_bwd_dispatch_c<5>(C, grad, inputs, offsets, grad_embeddings, dy_dx, grad_inputs, B, L, lt, gridtype, align_corners, interp, ws, ws_bytes, st);
    }
}

// The reference signature (gridencoder.h:12) has no workspace argument: it runs the
// workspace-free path (LDS windows for the coarse levels, direct atomics for the
// hashed ones).  Nothing is allocated, so it is stream-ordered and capture-safe;
// callers that can hand over scratch memory (the reference's own caller allocates
// every buffer, grid.py:75-82) use sdfr_grid_encode_backward_ws for the binned path.
int sdfr_grid_encode_backward(const float *grad, const float *inputs, const float *embeddings,
                              const int32_t *offsets, float *grad_embeddings, uint32_t B,
                              uint32_t D, uint32_t C, uint32_t L, float S, uint32_t H,
                              const float *dy_dx, float *grad_inputs, uint32_t gridtype,
                              int align_corners, uint32_t interp, void *stream) {
    return sdfr_grid_encode_backward_ws(grad, inputs, embeddings, offsets, grad_embeddings, B, D,
                                        C, L, S, H, dy_dx, grad_inputs, gridtype, align_corners,
                                        interp, nullptr, 0, stream);
}

int sdfr_sh_encode_forward(const float *inputs, float *outputs, uint32_t B, uint32_t D,
                           uint32_t C, float *dy_dx, void *stream) {
    if (D != 3) return fail(SDFR_EINVAL, "SH encoder only support input dim == 3");
    if (C < 1 || C > 8) return fail(SDFR_EINVAL, "SH encoder only supports degree in [1, 8]");
    if (B == 0) return SDFR_OK;
    if (!inputs || !outputs) return fail(SDFR_EINVAL, "sh_encode_forward: null tensor pointer");
    if (C <= 4)
        hipLaunchKernelGGL(sh_fwd_kernel<16>, dim3((B + 255) / 256), dim3(256), 0,
                           (hipStream_t)stream, inputs, outputs, dy_dx, B, C);
    else
        hipLaunchKernelGGL(sh_fwd_kernel<64>, dim3((B + 255) / 256), dim3(256), 0,
                           (hipStream_t)stream, inputs, outputs, dy_dx, B, C);
    return check_launch("sh_encode_forward");
}

int sdfr_sh_encode_backward(const float *grad, const float *inputs, uint32_t B, uint32_t D,
                            uint32_t C, const float *dy_dx, float *grad_inputs, void *stream) {
    (void)inputs;
    if (D != 3) return fail(SDFR_EINVAL, "SH encoder only support input dim == 3");
    if (C < 1 || C > 8) return fail(SDFR_EINVAL, "SH encoder only supports degree in [1, 8]");
    if (B == 0) return SDFR_OK;
    if (!grad || !dy_dx || !grad_inputs)
        return fail(SDFR_EINVAL, "sh_encode_backward: null tensor pointer");
    hipLaunchKernelGGL(sh_bwd_kernel, dim3((B * 3 + 255) / 256), dim3(256), 0,
                       (hipStream_t)stream, grad, dy_dx, grad_inputs, B, C);
    return check_launch("sh_encode_backward");
}

}  // extern "C"
