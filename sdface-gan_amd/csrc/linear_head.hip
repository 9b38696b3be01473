// linear_head.hip -- the renderer MLP's narrow output heads for TRAINING: sigma_linear
// (256 -> 1) and rgb_linear (256 -> 3) of NGPSIRENGenerator (LinearLayer,
// sdf_model.py:23-41, applied at :1586-1588) over the ~196 K samples of a stage-1 chunk.
// F.linear runs them as rocBLAS GEMMs with N = 1..3 (forward) and K = 1 (the input
// gradient is an outer product), ~0.5 ms each; they are HBM streams:
//
//   sdfr_linear_head_forward   out[M,J] = x[M,K] . w[J,K]^T (+ bias[J])      reads x
//   sdfr_linear_head_backward  gx[M,K] = gy[M,J] . w[J,K]                   writes gx
//                              gw[J,K] = sum_m gy[m,:]^T x[m,:],  gb = sum_m gy   reads x
//
// J <= 4, K <= 256 (multiple of 4), fp32 FMAs.  A row is 16 lanes (lane kq covers
// the 16-B quads kq, kq + 16, ...: every load is 256 contiguous bytes per row), a wave
// 4 rows at a time; the forward's dot products finish with a 16-lane butterfly.  The
// weight / bias gradients are per-workgroup partials (contiguous row ranges) added in
// a fixed order by a second kernel: deterministic.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "sdfr_common.h"

namespace sdfr {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kHeadThreads = 256;
constexpr uint32_t kHeadBlocks = 1024;          // backward partials (one round of 4 per CU)
constexpr uint32_t kQ = 4;                      // 16-B quads per lane (K <= 256)

__host__ __device__ constexpr uint32_t cdiv(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

__device__ __forceinline__ float row_sum16(float v) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o);
    return v;
}

template <int J>
__global__ void __launch_bounds__(kHeadThreads) head_fwd_kernel(const float *__restrict__ x,
                                                                const float *__restrict__ w,
                                                                const float *__restrict__ bias,
                                                                float *__restrict__ out,
                                                                uint32_t M, uint32_t K) {
    const uint32_t lane = threadIdx.x & 63u, kq = lane & 15u, rs = lane >> 4;
    const uint32_t KQ = K / 4;
    f4 wv[J][kQ];
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
        for (uint32_t i = 0; i < kQ; ++i) {
            const uint32_t q = kq + 16 * i;
            wv[j][i] = q < KQ ? *reinterpret_cast<const f4 *>(w + (size_t)j * K + 4 * q)
                              : f4{0.0f, 0.0f, 0.0f, 0.0f};
        }
    float bj[J];
#pragma unroll
    for (int j = 0; j < J; ++j) bj[j] = bias ? bias[j] : 0.0f;
    const uint32_t wave = (blockIdx.x * kHeadThreads + threadIdx.x) >> 6;
    const uint32_t nwaves = gridDim.x * (kHeadThreads / 64);
    for (uint32_t r0 = wave * 4; r0 < M; r0 += nwaves * 4) {
        const uint32_t m = r0 + rs;
        const bool ok = m < M;
        const f4 *xr = reinterpret_cast<const f4 *>(x + (size_t)(ok ? m : 0) * K);
        f4 xv[kQ];
#pragma unroll
        for (uint32_t i = 0; i < kQ; ++i) {
            const uint32_t q = kq + 16 * i;
            xv[i] = q < KQ ? xr[q] : f4{0.0f, 0.0f, 0.0f, 0.0f};
        }
#pragma unroll
        for (int j = 0; j < J; ++j) {
            float s = 0.0f;
#pragma unroll
            for (uint32_t i = 0; i < kQ; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) s = __fmaf_rn(xv[i][e], wv[j][i][e], s);
            s = row_sum16(s);
            if (ok && kq == 0) out[(size_t)m * J + j] = __fadd_rn(s, bj[j]);
        }
    }
}

// gx (if requested) and the workgroup's partial gw / gb (if requested) over a
// contiguous range of rows; part[blk] = [J][K] weight sums then [J] bias sums
template <int J>
__global__ void __launch_bounds__(kHeadThreads) head_bwd_kernel(const float *__restrict__ gy,
                                                                const float *__restrict__ x,
                                                                const float *__restrict__ w,
                                                                float *__restrict__ gx,
                                                                float *__restrict__ part,
                                                                uint32_t M, uint32_t K,
                                                                uint32_t rows_per_block) {
    __shared__ f4 red[kHeadThreads / 16][J][16 * kQ];           // [row slot][j][quad]
    __shared__ float redb[kHeadThreads / 16][J];
    const uint32_t lane = threadIdx.x & 63u, kq = lane & 15u;
    const uint32_t slot = threadIdx.x >> 4;                      // 16 row slots per block
    const uint32_t KQ = K / 4;
    const uint32_t m_begin = blockIdx.x * rows_per_block;
    const uint32_t m_end = min(M, m_begin + rows_per_block);
    f4 wv[J][kQ];
    if (gx) {
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (uint32_t i = 0; i < kQ; ++i) {
                const uint32_t q = kq + 16 * i;
                wv[j][i] = q < KQ ? *reinterpret_cast<const f4 *>(w + (size_t)j * K + 4 * q)
                                  : f4{0.0f, 0.0f, 0.0f, 0.0f};
            }
    }
    f4 acc[J][kQ];
    float accb[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        accb[j] = 0.0f;
#pragma unroll
        for (uint32_t i = 0; i < kQ; ++i) acc[j][i] = f4{0.0f, 0.0f, 0.0f, 0.0f};
    }
    for (uint32_t m = m_begin + slot; m < m_end; m += kHeadThreads / 16) {
        float g[J];
#pragma unroll
        for (int j = 0; j < J; ++j) g[j] = gy[(size_t)m * J + j];
        if (gx) {
            f4 *gr = reinterpret_cast<f4 *>(gx + (size_t)m * K);
#pragma unroll
            for (uint32_t i = 0; i < kQ; ++i) {
                const uint32_t q = kq + 16 * i;
                if (q >= KQ) continue;
                f4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float s = __fmul_rn(g[0], wv[0][i][e]);
#pragma unroll
                    for (int j = 1; j < J; ++j) s = __fmaf_rn(g[j], wv[j][i][e], s);
                    v[e] = s;
                }
                gr[q] = v;
            }
        }
        if (part) {
            const f4 *xr = reinterpret_cast<const f4 *>(x + (size_t)m * K);
#pragma unroll
            for (uint32_t i = 0; i < kQ; ++i) {
                const uint32_t q = kq + 16 * i;
                const f4 xv = q < KQ ? xr[q] : f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int j = 0; j < J; ++j)
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc[j][i][e] = __fmaf_rn(g[j], xv[e], acc[j][i][e]);
            }
#pragma unroll
            for (int j = 0; j < J; ++j) accb[j] = __fadd_rn(accb[j], g[j]);
        }
    }
    if (!part) return;
    // the 16 row slots' sums, added in slot order
#pragma unroll
    for (int j = 0; j < J; ++j) {
#pragma unroll
        for (uint32_t i = 0; i < kQ; ++i) red[slot][j][kq + 16 * i] = acc[j][i];
        if (kq == 0) redb[slot][j] = accb[j];
    }
    __syncthreads();
    float *pp = part + (size_t)blockIdx.x * ((J * K + J + 3) / 4 * 4);
    for (uint32_t e = threadIdx.x; e < J * KQ; e += kHeadThreads) {
        const uint32_t j = e / KQ, q = e % KQ;
        f4 s = red[0][j][q];
        for (uint32_t t = 1; t < kHeadThreads / 16; ++t) s += red[t][j][q];
        *reinterpret_cast<f4 *>(pp + (size_t)j * K + 4 * q) = s;
    }
    if (threadIdx.x < (uint32_t)J) {
        float s = redb[0][threadIdx.x];
        for (uint32_t t = 1; t < kHeadThreads / 16; ++t) s += redb[t][threadIdx.x];
        pp[J * K + threadIdx.x] = s;
    }
}

// gw / gb = the partials summed in a fixed order: thread (group gr, element e) sums
// partials gr, gr + 16, ... of element e; the 16 group sums are added in group order
__global__ void __launch_bounds__(256) head_reduce_kernel(const float *__restrict__ part,
                                                          uint32_t P, uint32_t count,
                                                          uint32_t stride, uint32_t nw,
                                                          float *__restrict__ gw,
                                                          float *__restrict__ gb) {
    __shared__ float red[16][16];
    const uint32_t el = threadIdx.x & 15u, gr = threadIdx.x >> 4;
    const uint32_t e = blockIdx.x * 16 + el;
    float s = 0.0f;
    if (e < count) {
        uint32_t p = gr;
        for (; p + 48 < P; p += 64) {                  // loads in flight, sums in order
            float v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = part[(size_t)(p + 16 * k) * stride + e];
#pragma unroll
            for (int k = 0; k < 4; ++k) s += v[k];
        }
        for (; p < P; p += 16) s += part[(size_t)p * stride + e];
    }
    red[gr][el] = s;
    __syncthreads();
    if (gr != 0 || e >= count) return;
    for (uint32_t k = 1; k < 16; ++k) s += red[k][el];
    if (e < nw) {
        if (gw) gw[e] = s;
    } else if (gb) {
        gb[e - nw] = s;
    }
}

template <int J>
int head_fwd_launch(const float *x, const float *w, const float *bias, float *out, uint32_t M,
                    uint32_t K, hipStream_t st) {
    const uint32_t blocks = std::min<uint32_t>(2048, cdiv(M, 16));
    hipLaunchKernelGGL((head_fwd_kernel<J>), dim3(blocks), dim3(kHeadThreads), 0, st, x, w, bias,
                       out, M, K);
    return check_launch("linear_head_forward");
}

template <int J>
int head_bwd_launch(const float *gy, const float *x, const float *w, float *gx, float *part,
                    uint32_t M, uint32_t K, uint32_t rpb, uint32_t P, hipStream_t st) {
    hipLaunchKernelGGL((head_bwd_kernel<J>), dim3(P), dim3(kHeadThreads), 0, st, gy, x, w, gx,
                       part, M, K, rpb);
    return check_launch("linear_head_backward");
}

uint32_t head_rows_per_block(uint32_t M) { return std::max<uint32_t>(16, cdiv(M, kHeadBlocks)); }
// floats per partial: [J][K] then [J], padded to 16 B
__host__ __device__ constexpr uint32_t head_part_stride(uint32_t J, uint32_t K) {
    return (J * K + J + 3) / 4 * 4;
}

}  // namespace
}  // namespace sdfr

using namespace sdfr;

extern "C" {

int sdfr_linear_head_forward(float *out, const float *x, const float *w, const float *bias,
                             uint32_t M, uint32_t J, uint32_t K, void *stream) {
    if (M == 0) return SDFR_OK;
    if (!out || !x || !w) return fail(SDFR_EINVAL, "linear_head_forward: null pointer");
    if (J == 0 || J > 4 || K == 0 || K > 256 || K % 4 ||
        (reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w)) % 16)
        return fail(SDFR_EINVAL, "linear_head_forward: J <= 4, K <= 256 a multiple of 4, "
                                 "16-B aligned x and w");
    hipStream_t st = (hipStream_t)stream;
    switch (J) {
        case 1: return head_fwd_launch<1>(x, w, bias, out, M, K, st);
        case 2: return head_fwd_launch<2>(x, w, bias, out, M, K, st);
        case 3: return head_fwd_launch<3>(x, w, bias, out, M, K, st);
        default: return head_fwd_launch<4>(x, w, bias, out, M, K, st);
    }
}

size_t sdfr_linear_head_ws_bytes(uint32_t M, uint32_t J, uint32_t K) {
    if (M == 0) return 0;
    return (size_t)cdiv(M, head_rows_per_block(M)) * head_part_stride(J, K) * 4;
}

int sdfr_linear_head_backward(float *gx, float *gw, float *gb, const float *gy, const float *x,
                              const float *w, uint32_t M, uint32_t J, uint32_t K, void *ws,
                              size_t ws_bytes, void *stream) {
    if (!gy || (gx && !w) || ((gw || gb) && !x))
        return fail(SDFR_EINVAL, "linear_head_backward: null pointer");
    if (J == 0 || J > 4 || K == 0 || K > 256 || K % 4 ||
        (reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w) |
         reinterpret_cast<uintptr_t>(gx)) % 16)
        return fail(SDFR_EINVAL, "linear_head_backward: J <= 4, K <= 256 a multiple of 4, "
                                 "16-B aligned x, w, gx");
    hipStream_t st = (hipStream_t)stream;
    const bool wgrad = gw || gb;
    if (M == 0) {
        if (gw && hipMemsetAsync(gw, 0, (size_t)J * K * 4, st) != hipSuccess)
            return fail(SDFR_ELAUNCH, "linear_head_backward: memset");
        if (gb && hipMemsetAsync(gb, 0, (size_t)J * 4, st) != hipSuccess)
            return fail(SDFR_ELAUNCH, "linear_head_backward: memset");
        return SDFR_OK;
    }
    if (!gx && !wgrad) return SDFR_OK;
    if (wgrad && (!ws || ws_bytes < sdfr_linear_head_ws_bytes(M, J, K)))
        return fail(SDFR_EINVAL, "linear_head_backward: workspace too small");
    const uint32_t rpb = head_rows_per_block(M), P = cdiv(M, rpb);
    float *part = wgrad ? static_cast<float *>(ws) : nullptr;
    int rc;
    switch (J) {
        case 1: rc = head_bwd_launch<1>(gy, x, w, gx, part, M, K, rpb, P, st); break;
        case 2: rc = head_bwd_launch<2>(gy, x, w, gx, part, M, K, rpb, P, st); break;
        case 3: rc = head_bwd_launch<3>(gy, x, w, gx, part, M, K, rpb, P, st); break;
        default: rc = head_bwd_launch<4>(gy, x, w, gx, part, M, K, rpb, P, st); break;
    }
    if (rc || !wgrad) return rc;
    const uint32_t count = J * K + J;
    hipLaunchKernelGGL(head_reduce_kernel, dim3(cdiv(count, 16)), dim3(256), 0, st, part, P,
                       count, head_part_stride(J, K), J * K, gw, gb);
    return check_launch("linear_head_backward: reduce");
}

}  // extern "C"
