// sdfr_common.h -- shared host/device helpers of libsdfr (gfx950 only).
//
// The grid-index and ray-sampling arithmetic below is the bit-exact part of
// the renderer: it is written with explicit round-to-nearest intrinsics
// (__fmul_rn / __fadd_rn / __fdiv_rn / __fmaf_rn) so that neither the
// compiler's contraction setting nor operator re-association can change it.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>
#include <string>

#include "../../include/sdfr.h"

namespace sdfr {

// ----------------------------------------------------------------------------
// error plumbing
// ----------------------------------------------------------------------------
void set_error(const std::string &msg);
int fail(int code, const std::string &msg);
int check_launch(const char *what);

// ----------------------------------------------------------------------------
// per-level grid parameters (gridencoder.cu:136-139, 66-84)
// ----------------------------------------------------------------------------
constexpr int kMaxLevels = 64;
enum : uint32_t {
    LVL_HASHED = 1u,   // index = fast_hash(pos) (stride > hashmap_size, gridtype 0)
    LVL_POW2 = 2u,     // hashmap_size is a power of two -> mask instead of %
    LVL_INRANGE = 4u,  // dense index provably < hashmap_size -> no modulo
};

struct LevelParam {
    float scale;        // exp2f(l*S)*H - 1
    uint32_t res;       // (uint32)ceil(scale) + 1
    uint32_t hsize;     // offsets[l+1] - offsets[l]
    uint32_t offset;    // offsets[l]
    uint32_t ndims;     // dims that entered the dense stride loop
    uint32_t flags;
};

struct LevelTable {
    LevelParam p[kMaxLevels];
};

// Host: the float part of the per-level parameters (needs only L, S, H, so
// no device->host copy of the offsets is ever required).  exp2f is evaluated
// correctly rounded (double, one rounding); see DESIGN.md "parity pinning".
inline void make_level_table(uint32_t L, float S, uint32_t H, LevelTable &t) {
    for (uint32_t l = 0; l < L; ++l) {
        LevelParam &q = t.p[l];
        float ls = (float)l * S;
        float e = (float)std::exp2((double)ls);
        q.scale = e * (float)H - 1.0f;
        q.res = (uint32_t)std::ceil(q.scale) + 1u;
        q.hsize = q.offset = q.ndims = q.flags = 0;
    }
}

// Device: the integer part, from the offsets buffer (wave-uniform, scalar).
// Mirrors the stride loop of get_grid_index (gridencoder.cu:66-84).
__device__ __forceinline__ void finish_level(LevelParam &q, const int32_t *__restrict__ offsets,
                                             uint32_t level, uint32_t D, uint32_t gridtype,
                                             int align_corners) {
    const uint32_t o0 = (uint32_t)offsets[level];
    q.offset = o0;
    q.hsize = (uint32_t)offsets[level + 1] - o0;
    uint32_t stride = 1, nd = 0;
    for (uint32_t d = 0; d < D && stride <= q.hsize; ++d) {
        stride *= align_corners ? q.res : (q.res + 1);
        ++nd;
    }
    q.ndims = nd;
    uint32_t f = 0;
    if (gridtype == 0 && stride > q.hsize) f |= LVL_HASHED;
    if ((q.hsize & (q.hsize - 1)) == 0) f |= LVL_POW2;
    if (!(f & LVL_HASHED) && nd == D && !align_corners && stride <= q.hsize) f |= LVL_INRANGE;
    q.flags = f;
}

// ----------------------------------------------------------------------------
// device: grid index (gridencoder.cu:50-84)
// ----------------------------------------------------------------------------
template <uint32_t D>
__device__ __forceinline__ uint32_t grid_index(const LevelParam &q, int align_corners,
                                               const uint32_t (&pg)[D]) {
    uint32_t index;
    if (q.flags & LVL_HASHED) {
        constexpr uint32_t primes[7] = {1u, 2654435761u, 805459861u, 3674653429u,
                                        2097192037u, 1434869437u, 2165219737u};
        index = 0;
#pragma unroll
        for (uint32_t i = 0; i < D; ++i) index ^= pg[i] * primes[i];
    } else {
        const uint32_t s = align_corners ? q.res : q.res + 1;
        uint32_t stride = 1;
        index = 0;
#pragma unroll
        for (uint32_t d = 0; d < D; ++d) {
            if (d < q.ndims) index += pg[d] * stride;
            stride *= s;
        }
        if (q.flags & LVL_INRANGE) return index;
    }
    return (q.flags & LVL_POW2) ? (index & (q.hsize - 1)) : (index % q.hsize);
}

__device__ __forceinline__ float smoothstep_f(float v) {
    return __fmul_rn(__fmul_rn(v, v), __fsub_rn(3.0f, __fmul_rn(2.0f, v)));
}
__device__ __forceinline__ float smoothstep_d(float v) {
    return __fmul_rn(__fmul_rn(6.0f, v), __fsub_rn(1.0f, v));
}

// Trilinear (multilinear) interpolation of one level; the corner order, the
// weight products and the fma accumulation follow gridencoder.cu:160-192.
template <uint32_t D, uint32_t C>
struct LevelCoord {
    float pos[D];
    float pos_d[D];
    uint32_t pg[D];
};

template <uint32_t D, uint32_t C>
__device__ __forceinline__ void level_coord(const float (&x)[D], const LevelParam &q,
                                            int align_corners, uint32_t interp,
                                            LevelCoord<D, C> &lc) {
#pragma unroll
    for (uint32_t d = 0; d < D; ++d) {
        float p = __fmaf_rn(x[d], q.scale, align_corners ? 0.0f : 0.5f);
        float f = floorf(p);
        lc.pg[d] = (uint32_t)f;
        p = __fsub_rn(p, (float)lc.pg[d]);
        if (interp == 1) {
            lc.pos_d[d] = smoothstep_d(p);
            p = smoothstep_f(p);
        } else {
            lc.pos_d[d] = 1.0f;
        }
        lc.pos[d] = p;
    }
}

template <uint32_t C>
struct VecC;
template <> struct VecC<1> { using T = float; };
template <> struct VecC<2> { using T = float2; };
template <> struct VecC<4> { using T = float4; };
template <> struct VecC<8> { using T = float4; };

template <uint32_t C>
__device__ __forceinline__ void load_row(const float *__restrict__ grid, uint32_t index,
                                         float (&v)[C]) {
    if constexpr (C == 1) {
        v[0] = grid[index];
    } else if constexpr (C == 2) {
        float2 t = *reinterpret_cast<const float2 *>(grid + index);
        v[0] = t.x; v[1] = t.y;
    } else {
#pragma unroll
        for (uint32_t c = 0; c < C; c += 4) {
            float4 t = *reinterpret_cast<const float4 *>(grid + index + c);
            v[c] = t.x; v[c + 1] = t.y; v[c + 2] = t.z; v[c + 3] = t.w;
        }
    }
}

template <uint32_t D, uint32_t C>
__device__ __forceinline__ void level_interp(const float *__restrict__ grid,
                                             const LevelParam &q, int align_corners,
                                             const LevelCoord<D, C> &lc, float (&out)[C]) {
#pragma unroll
    for (uint32_t c = 0; c < C; ++c) out[c] = 0.0f;
    // issue every corner load first (independent), then accumulate in order
    float v[1u << D][C];
    float wts[1u << D];
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
        wts[idx] = w;
        load_row<C>(grid, grid_index<D>(q, align_corners, pl) * C, v[idx]);
    }
#pragma unroll
    for (uint32_t idx = 0; idx < (1u << D); ++idx)
#pragma unroll
        for (uint32_t c = 0; c < C; ++c) out[c] = __fmaf_rn(wts[idx], v[idx][c], out[c]);
}

// 8-B-aligned 16-B row pair (global_load_dwordx4 at dword alignment)
typedef float f4_a8 __attribute__((ext_vector_type(4), aligned(8)));

// Rows i0 (x-corner g0) and i1 (g0+1) of a C = 2 level whose size is even:
// ONE 16-B load when the rows are consecutive, i1 = i0 +- 1 (every dense row;
// hashed rows -- prime 1 on x -- for 2/3 of the g0 parities), else the aligned
// pair holding i0 plus an 8-B load of i1 (for those lanes only).  Every row
// read lies inside the level.
__device__ __forceinline__ void load_xpair(const float *__restrict__ grid, uint32_t i0,
                                           uint32_t i1, float (&v0)[2], float (&v1)[2]) {
    const bool up = i1 == i0 + 1u, down = i1 + 1u == i0;
    const uint32_t base = up ? i0 : (down ? i1 : (i0 & ~1u));
    const f4_a8 t = *reinterpret_cast<const f4_a8 *>(grid + (size_t)base * 2);
    const bool lo0 = base == i0;
    v0[0] = lo0 ? t.x : t.z;
    v0[1] = lo0 ? t.y : t.w;
    if (up || down) {
        v1[0] = up ? t.z : t.x;
        v1[1] = up ? t.w : t.y;
    } else {
        const float2 u = *reinterpret_cast<const float2 *>(grid + (size_t)i1 * 2);
        v1[0] = u.x;
        v1[1] = u.y;
    }
}

// All 2^D corner rows of one level, corner idx bit d = (g_d or g_d + 1); with
// PAIR (D = 3, C = 2 only) the x-neighbours through load_xpair.
template <uint32_t D, uint32_t C, bool PAIR>
__device__ __forceinline__ void level_corners(const float *__restrict__ grid,
                                              const LevelParam &q, int align_corners,
                                              const LevelCoord<D, C> &lc,
                                              float (&v)[1u << D][C]) {
#pragma unroll
    for (uint32_t idx = 0; idx < (1u << D); idx += (PAIR ? 2u : 1u)) {
        uint32_t pl[D];
#pragma unroll
        for (uint32_t d = 0; d < D; ++d) pl[d] = (idx & (1u << d)) ? lc.pg[d] + 1 : lc.pg[d];
        const uint32_t i0 = grid_index<D>(q, align_corners, pl);
        if constexpr (PAIR) {
            static_assert(C == 2, "paired corner loads need C = 2");
            pl[0] = lc.pg[0] + 1;
            load_xpair(grid, i0, grid_index<D>(q, align_corners, pl), v[idx], v[idx + 1]);
        } else {
            load_row<C>(grid, i0 * C, v[idx]);
        }
    }
}

// ----------------------------------------------------------------------------
// device: ray generation + sampling (sdf_model.py:207-222, 310-351, 363-378)
// ----------------------------------------------------------------------------
struct Ray {
    float o[3];
    float d[3];      // rays_d (unnormalised)
    float dir[3];    // camera-frame direction (static_viewdirs)
};

__device__ __forceinline__ float norm3_torch(float x, float y, float z) {
    // torch.norm over a 3-wide dim on the reference's CPU path:
    // sqrt(fma(z,z,fma(y,y,x*x)))  (pinned by tests/golden)
    return __fsqrt_rn(__fmaf_rn(z, z, __fmaf_rn(y, y, __fmul_rn(x, x))));
}

__device__ __forceinline__ void make_ray(const float *__restrict__ cam12, float focal,
                                         float px, float py, float half_res, Ray &r) {
    r.dir[0] = __fdiv_rn(__fsub_rn(px, half_res), focal);
    r.dir[1] = -__fdiv_rn(__fsub_rn(py, half_res), focal);
    r.dir[2] = -1.0f;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float s = __fmul_rn(r.dir[0], cam12[k * 4 + 0]);
        s = __fadd_rn(s, __fmul_rn(r.dir[1], cam12[k * 4 + 1]));
        s = __fadd_rn(s, __fmul_rn(r.dir[2], cam12[k * 4 + 2]));
        r.d[k] = s;
        r.o[k] = cam12[k * 4 + 3];
    }
}

// z_vals[s] before perturbation: near*(1-t) + far*t
__device__ __forceinline__ float z_base(float nr, float fr, float t) {
    return __fadd_rn(__fmul_rn(nr, __fsub_rn(1.0f, t)), __fmul_rn(fr, t));
}

struct SampleCfg {
    const float *t_vals;
    const float *t_rand;
    int t_rand_per_sample;
    int offset_sampling;
    uint32_t N;
};

// Perturbed z of sample s of a ray (ray_index = flat [B,H,W] index).
__device__ __forceinline__ float sample_z(const SampleCfg &c, float nr, float fr,
                                          uint32_t ray_index, uint32_t s) {
    const float z = z_base(nr, fr, c.t_vals[s]);
    if (!c.t_rand) return z;
    if (c.offset_sampling) {
        const float up = (s + 1 < c.N) ? z_base(nr, fr, c.t_vals[s + 1]) : fr;
        const float tr = c.t_rand[ray_index];
        return __fadd_rn(z, __fmul_rn(__fsub_rn(up, z), tr));
    }
    const float tr = c.t_rand_per_sample ? c.t_rand[(size_t)ray_index * c.N + s]
                                         : c.t_rand[ray_index];
    const float lo = (s == 0) ? z
                              : __fmul_rn(0.5f, __fadd_rn(z, z_base(nr, fr, c.t_vals[s - 1])));
    const float up = (s + 1 < c.N)
                         ? __fmul_rn(0.5f, __fadd_rn(z_base(nr, fr, c.t_vals[s + 1]), z))
                         : z;
    return __fadd_rn(lo, __fmul_rn(__fsub_rn(up, lo), tr));
}

}  // namespace sdfr
