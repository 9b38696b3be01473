// sdfr_scan.h -- in-place exclusive prefix sum of a uint32 array on one stream
// (marching cubes' vertex / triangle numbering, the grid backward's bin offsets).
//
// Three launches: per-block totals of 2048-element tiles, one workgroup scanning
// the block totals, then each block scanning its tile from its total's offset.
// S[M] receives the grand total, so S must hold M + 1 elements; bsum holds
// scan_block_sums(M).  HBM-streaming: S is read twice and written once.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sdfr {
namespace {

constexpr int kScanThreads = 256;
constexpr int kScanPer = 8;                            // elements per thread
constexpr int kScanTile = kScanThreads * kScanPer;     // 2048 per block

// block-wide exclusive scan of one value per thread; returns the block total
__device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t &excl) {
    __shared__ uint32_t wsum[kScanThreads / 64];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o);
        if (lane >= (uint32_t)o) inc += t;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int q = 0; q < kScanThreads / 64; ++q) {
        before += (q < (int)w) ? wsum[q] : 0u;
        total += wsum[q];
    }
    __syncthreads();
    excl = before + inc - v;
    return total;
}

__device__ __forceinline__ void load_tile(const uint32_t *S, uint64_t M, uint64_t base,
                                          uint32_t (&x)[kScanPer]) {
#pragma unroll
    for (int q = 0; q < kScanPer; ++q) {
        const uint64_t e = base + q;
        x[q] = e < M ? S[e] : 0u;
    }
}

__global__ void __launch_bounds__(kScanThreads) scan_reduce(const uint32_t *S, uint64_t M,
                                                          uint32_t *bsum) {
    uint32_t x[kScanPer];
    load_tile(S, M, (uint64_t)blockIdx.x * kScanTile + threadIdx.x * kScanPer, x);
    uint32_t s = 0;
#pragma unroll
    for (int q = 0; q < kScanPer; ++q) s += x[q];
    uint32_t ex;
    const uint32_t tot = block_exscan(s, ex);
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// one block: exclusive scan of the nb block sums in place; S[M] = grand total
__global__ void __launch_bounds__(kScanThreads) scan_blocks(uint32_t *bsum, uint32_t nb,
                                                          uint32_t *S, uint64_t M) {
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < nb; b0 += kScanThreads) {
        const uint32_t b = b0 + threadIdx.x;
        const uint32_t v = b < nb ? bsum[b] : 0u;
        uint32_t ex;
        const uint32_t tot = block_exscan(v, ex);
        if (b < nb) bsum[b] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) S[M] = carry;
}

__global__ void __launch_bounds__(kScanThreads) scan_apply(uint32_t *S, uint64_t M,
                                                         const uint32_t *bsum) {
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * kScanPer;
    uint32_t x[kScanPer];
    load_tile(S, M, base, x);
    uint32_t s = 0;
#pragma unroll
    for (int q = 0; q < kScanPer; ++q) s += x[q];
    uint32_t ex;
    block_exscan(s, ex);
    uint32_t run = bsum[blockIdx.x] + ex;
#pragma unroll
    for (int q = 0; q < kScanPer; ++q) {
        if (base + q < M) S[base + q] = run;
        run += x[q];
    }
}

inline uint32_t scan_block_sums(uint64_t M) { return (uint32_t)((M + kScanTile - 1) / kScanTile); }

// S[0..M) := exclusive prefix sums, S[M] := total (M + 1 elements); bsum: scratch
inline void exclusive_scan_u32(uint32_t *S, uint64_t M, uint32_t *bsum, hipStream_t st) {
    const uint32_t nb = scan_block_sums(M);
    scan_reduce<<<nb, kScanThreads, 0, st>>>(S, M, bsum);
    scan_blocks<<<1, kScanThreads, 0, st>>>(bsum, nb, S, M);
    scan_apply<<<nb, kScanThreads, 0, st>>>(S, M, bsum);
}

}  // namespace
}  // namespace sdfr
