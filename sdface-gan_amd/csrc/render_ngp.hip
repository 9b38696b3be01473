// render_ngp.hip -- fused SDF + hash-grid volume renderer for MI355X (gfx950).
//
// Replaces VolumeFeatureRenderer.forward for rendering.type == "ngp"
// (sdf_model.py:411-423 -> render :363 -> render_rays :310 ->
// NGPSIRENGenerator.forward :1566 -> volume_integration :236) with three
// launches on one stream:
//
//  1. ngp_prep_kernel   per-face FiLM gamma/beta (4 layers x 256, from the
//                       renderer latent) and the MFMA-fragment packing of the
//                       five dense weight matrices (1.07 MB, read once per call).
//  2. ngp_encode_kernel ray generation + sampling (bit-exact vs. the reference
//                       float chain) and the 16-level hash-grid gather, one
//                       (sample, level) per thread, level-major grid so each
//                       level's <= 4 MiB table stays in every XCD's L2.
//                       Output [L][S][2] fp32 in "tile order" (16 rays of one
//                       sample contiguous), exactly what stage 3 reads.
//  3. ngp_field_kernel  the whole MLP on fp32 MFMA (v_mfma_f32_16x16x4_f32) +
//                       SDF->density + front-to-back alpha compositing.  A wave
//                       owns 16 rays and marches their samples in order; the
//                       MFMA N dimension is the ray, so every per-ray quantity
//                       (transmittance, colour/feature accumulators) is a
//                       per-lane register and compositing needs no cross-lane
//                       traffic.  Activations never leave registers: the
//                       accumulator tile of layer l is, element for element,
//                       the B operand of layer l+1 (K permuted consistently in
//                       the packed weights).  Weights stream through a 3-slot
//                       LDS ring (16 KB K-slices) shared by the 8 waves of the
//                       workgroup; the [S,260] raw tensor the reference
//                       materialises is never formed.
//
// Numerics: fp32 everywhere; MFMA f32 is an exact fmaf chain, so results
// differ from the reference only by summation order (tolerances in
// tests/test_gpu_render.py).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <string>

#include "render_ngp.h"

namespace sdfr {

constexpr uint32_t kSliceF4 = 1024;   // float4 per 16-wide K slice (16 t_out x 64 lanes)
constexpr uint32_t kSlices = 2 + 16 * 3 + 17;   // 67 slices per sample step

// slice index -> (layer, t_in)
__host__ __device__ constexpr uint32_t slice_base(uint32_t layer) {
    return layer == 0 ? 0u : (layer == 4 ? 50u : 2u + 16u * (layer - 1));
}

// ----------------------------------------------------------------------------
// 1. prep: FiLM vectors + packed weights
// ----------------------------------------------------------------------------
struct PrepArgs {
    const float *styles;           // [B,256]
    const float *gw[kFilm], *gb[kFilm], *bw[kFilm], *bb[kFilm];
    const float *w[5];             // layer weights, row-major [256, K]
    uint32_t K[5];
    float *film;                   // [B][4][2][256]
    f4 *packed;                    // [67][16][64]
    uint32_t B;
};

// blocks [0, B*4*2): film rows (256 threads = 256 outputs)
// blocks [B*8, B*8 + 67*4): packing, 256 float4 per block
__global__ void __launch_bounds__(256) ngp_prep_kernel(const PrepArgs a) {
    const uint32_t blk = blockIdx.x, j = threadIdx.x;
    const uint32_t nfilm = a.B * kFilm * 2;
    if (blk < nfilm) {
        const uint32_t b = blk / (kFilm * 2), rem = blk % (kFilm * 2);
        const uint32_t layer = rem >> 1, which = rem & 1;
        const float *W = which ? a.bw[layer] : a.gw[layer];
        const float *bias = which ? a.bb[layer] : a.gb[layer];
        const float *st = a.styles + (size_t)b * kW;
        const f4 *wr = reinterpret_cast<const f4 *>(W + (size_t)j * kW);
        const f4 *sr = reinterpret_cast<const f4 *>(st);
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
        // LinearLayer: std_init * linear + bias_init (sdf_model.py:39, 58-59)
        const float v = which ? __fadd_rn(__fmul_rn(0.25f, lin), 0.0f)
                              : __fadd_rn(__fmul_rn(15.0f, lin), 30.0f);
        a.film[(((size_t)b * kFilm + layer) * 2 + which) * kW + j] = v;
        return;
    }
    // packing: element (slice, t_out, lane) = W[16 t_out + (lane&15)][16 t_in + 4 (lane>>4) + r]
    const uint32_t e = (blk - nfilm) * 256 + j;
    if (e >= kSlices * kSliceF4) return;
    const uint32_t slice = e / kSliceF4, rem = e % kSliceF4;
    const uint32_t t_out = rem >> 6, lane = rem & 63;
    uint32_t layer = 0;
    if (slice >= 50) layer = 4;
    else if (slice >= 2) layer = 1 + (slice - 2) / 16;
    const uint32_t t_in = slice - slice_base(layer);
    const uint32_t row = 16 * t_out + (lane & 15);
    const uint32_t col = 16 * t_in + 4 * (lane >> 4);
    const float *src = a.w[layer] + (size_t)row * a.K[layer] + col;
    f4 v;
    v.x = src[0]; v.y = src[1]; v.z = src[2]; v.w = src[3];
    a.packed[e] = v;
}

// ----------------------------------------------------------------------------
// 2. encode: sampling + hash-grid gather
// ----------------------------------------------------------------------------
struct EncodeArgs {
    GeomArgs g;
    const float *emb;
    const int32_t *offsets;
    const f4 *gu;                  // [S_total] grid coordinate u (x, y, z) | inside [0,1]^3
    float *enc;                    // [L][S_total][2]
    LevelTable lt;
    int pair_ok;                   // table 16-B aligned (paired corner loads)
};

// Encode launch options (sdfr_debug_set_encode_mode / SDFR_ENC_MODE, ablations
// only; all bit-identical; times per 32 faces from scripts/encode_time.py):
//  +8 off   PAIR: the x-neighbour corners (g0, g0+1) from one aligned 16-B load
//           whenever their rows are {i, i^1} (hash prime 1 on x: always for
//           even g0; dense rows: for even i), an 8-B load of the second row
//           only for the other lanes.                      mode 9 0.94 -> 1 0.84 ms
//  +256     A8: the same with dword-aligned 16-B loads, so ANY consecutive rows
//           i, i+-1 come from one load (every dense row, 2/3 of the hashed
//           g0 parities).                                       -> 257 0.80 ms
//  low bits LPT levels per thread {y, y+16/LPT} (2: mode 2 0.83 ms; 4 was
//           slower, 1.17 ms, with four levels' tables live in each L2).
//  +32      SPT = 2 samples per thread, 256 apart: twice the corner loads in
//           flight per wave.                                    -> 289 0.77 ms
//           Since the per-sample coordinate comes precomputed (sample_geom_kernel)
//           one sample per thread is faster again: 257 0.787 vs 289 0.803 ms (and
//           258, two levels per thread, 0.824), interleaved on one box, geom
//           kernel included.
// The gather is bound by L1 tag lookups (one 128-B line per lane per load
// instruction, ~54 cycles per wave-load measured): the wins above all cut
// load instructions per sample-level (6 -> ~4.9).  Measured and dropped:
// XCD-owned levels (each XCD's blocks on two levels only: 1.22 vs 1.08 ms),
// sc1 (L2-dropping) output stores (+-1%), adjacent level pairs {2y, 2y+1}
// (1.09 ms), whole image rows per wave (0.86 ms), 4 samples per thread (0.78 ms),
// nontemporal table loads (2.1 ms: the table no longer stays in L2).
constexpr uint32_t kEncDefault = 256 | 1;

// level_interp<3,2> with paired x-corner loads: the same corner weights
// (x factor first, then y, z) and the same fma order over corners 0..7, so the
// result is bit-identical to level_interp.
__device__ __forceinline__ void level_interp_pair(const float *__restrict__ grid,
                                                  const LevelParam &q,
                                                  const LevelCoord<3, 2> &lc, float (&out)[2]) {
    float v[8][2];
    float wts[8];
#pragma unroll
    for (uint32_t idx = 0; idx < 8; idx += 2) {
        uint32_t pl[3];
        float w0 = __fsub_rn(1.0f, lc.pos[0]), w1 = lc.pos[0];
#pragma unroll
        for (uint32_t d = 1; d < 3; ++d) {
            const bool hi = idx & (1u << d);
            pl[d] = hi ? lc.pg[d] + 1 : lc.pg[d];
            const float f = hi ? lc.pos[d] : __fsub_rn(1.0f, lc.pos[d]);
            w0 = __fmul_rn(w0, f);
            w1 = __fmul_rn(w1, f);
        }
        wts[idx] = w0;
        wts[idx + 1] = w1;
        pl[0] = lc.pg[0];
        const uint32_t i0 = grid_index<3>(q, 0, pl);
        pl[0] = lc.pg[0] + 1;
        const uint32_t i1 = grid_index<3>(q, 0, pl);
        const float4 t = *reinterpret_cast<const float4 *>(grid + (size_t)(i0 & ~1u) * 2);
        const bool odd = i0 & 1u;
        v[idx][0] = odd ? t.z : t.x;
        v[idx][1] = odd ? t.w : t.y;
        if (i1 == (i0 ^ 1u)) {
            v[idx + 1][0] = odd ? t.x : t.z;
            v[idx + 1][1] = odd ? t.y : t.w;
        } else {
            const float2 u = *reinterpret_cast<const float2 *>(grid + (size_t)i1 * 2);
            v[idx + 1][0] = u.x;
            v[idx + 1][1] = u.y;
        }
    }
    out[0] = out[1] = 0.0f;
#pragma unroll
    for (uint32_t idx = 0; idx < 8; ++idx)
#pragma unroll
        for (uint32_t c = 0; c < 2; ++c) out[c] = __fmaf_rn(wts[idx], v[idx][c], out[c]);
}

// One thread: SPT samples (256 apart) x LPT levels ({y, y+16/LPT, ...}, or
// {LPT y, LPT y + 1, ...} with ADJ).  Branch-free: padding / out-of-box samples
// gather at u = 0.5 and store 0, so every corner load of the thread can be in
// flight at once.
// level_interp_pair with dword-aligned (not 16-B aligned) pair loads
// (load_xpair, sdfr_common.h): the two x-corners come from ONE 16-B load
// whenever their rows are consecutive.  Same weights and fma order as
// level_interp: bit-identical.
__device__ __forceinline__ void level_interp_adj(const float *__restrict__ grid,
                                                 const LevelParam &q,
                                                 const LevelCoord<3, 2> &lc, float (&out)[2]) {
    float v[8][2];
    float wts[8];
#pragma unroll
    for (uint32_t idx = 0; idx < 8; idx += 2) {
        uint32_t pl[3];
        float w0 = __fsub_rn(1.0f, lc.pos[0]), w1 = lc.pos[0];
#pragma unroll
        for (uint32_t d = 1; d < 3; ++d) {
            const bool hi = idx & (1u << d);
            pl[d] = hi ? lc.pg[d] + 1 : lc.pg[d];
            const float f = hi ? lc.pos[d] : __fsub_rn(1.0f, lc.pos[d]);
            w0 = __fmul_rn(w0, f);
            w1 = __fmul_rn(w1, f);
        }
        wts[idx] = w0;
        wts[idx + 1] = w1;
        pl[0] = lc.pg[0];
        const uint32_t i0 = grid_index<3>(q, 0, pl);
        pl[0] = lc.pg[0] + 1;
        const uint32_t i1 = grid_index<3>(q, 0, pl);
        load_xpair(grid, i0, i1, v[idx], v[idx + 1]);
    }
    out[0] = out[1] = 0.0f;
#pragma unroll
    for (uint32_t idx = 0; idx < 8; ++idx)
#pragma unroll
        for (uint32_t c = 0; c < 2; ++c) out[c] = __fmaf_rn(wts[idx], v[idx][c], out[c]);
}

// One thread: SPT samples (256 apart) x LPT levels {y, y + 16/LPT, ...}.
// Branch-free: padding / out-of-box samples gather at u = 0.5 and store 0, so
// every corner load of the thread can be in flight at once.
template <bool PAIR, bool A8, uint32_t LPT, uint32_t SPT>
__global__ void __launch_bounds__(256) ngp_encode_kernel(const EncodeArgs a) {
    float2 *out = reinterpret_cast<float2 *>(a.enc);
    uint32_t sid[SPT];
    bool live[SPT], in[SPT];
    float u[SPT][3];
#pragma unroll
    for (uint32_t k = 0; k < SPT; ++k) {
        sid[k] = (blockIdx.x * SPT + k) * 256 + threadIdx.x;
        live[k] = sid[k] < a.g.S_total;
        // the sample's grid coordinate, computed once per sample by sample_geom_kernel
        // (the per-level recomputation cost ~25 vector loads per wave on the texture
        // addresser that the gather is bound by)
        const f4 gv = a.gu[live[k] ? sid[k] : 0];
        in[k] = live[k] && gv.w != 0.0f;
        u[k][0] = in[k] ? gv.x : 0.5f;
        u[k][1] = in[k] ? gv.y : 0.5f;
        u[k][2] = in[k] ? gv.z : 0.5f;
    }
#pragma unroll
    for (uint32_t j = 0; j < LPT; ++j) {
        const uint32_t level = blockIdx.y + j * (16 / LPT);
        LevelParam q = a.lt.p[level];
        finish_level(q, a.offsets, level, 3, 0, 0);
        const float *grid = a.emb + (size_t)q.offset * 2;
        // pairs are 16-B aligned when the level base (offset) is even and the
        // table itself is 16-B aligned (host check, a.pair_ok); an even level
        // size keeps every aligned pair inside the level
        const bool pair = PAIR && a.pair_ok && !((q.offset | q.hsize) & 1u);
#pragma unroll
        for (uint32_t k = 0; k < SPT; ++k) {
            LevelCoord<3, 2> lc;
            level_coord<3, 2>(u[k], q, 0, 0, lc);
            float res[2];
            if (pair && A8)
                level_interp_adj(grid, q, lc, res);
            else if (pair)
                level_interp_pair(grid, q, lc, res);
            else
                level_interp<3, 2>(grid, q, 0, lc, res);
            if (live[k])
                out[(size_t)level * a.g.S_total + sid[k]] =
                    in[k] ? make_float2(res[0], res[1]) : make_float2(0.0f, 0.0f);
        }
    }
}

// Per-sample geometry, one thread per ray (each z computed once), in tile order:
//   gu [S]  the grid coordinate u = ((o + d z) (2 / (far - near)) + bound) / (2 bound)
//           (sdf_model.py:343-349, grid.py:149; the same rounded ops as sample_u), w = 1
//           when u lies in [0,1]^3 (the gather's zero-feature test, gridencoder.cu:104-111),
//           0 for that and for tile-padding rays;
//   zd [S]  depth z and segment length dist = (z_{s+1} - z_s) |d| (1e10 |d| for the last
//           sample), sdf_model.py:240-243 -- the compositing inputs field_r_kernel reads
//           (null: not wanted).
//   One thread per (ray, chunk of spt samples), ray fastest within a tile (coalesced
//   stores); spt = N at large batches, smaller when the rays alone would leave the chip
//   idle (eval.py's batch of 1: 4096 rays = 16 workgroups at one thread per ray).
__global__ void __launch_bounds__(256) sample_geom_kernel(const GeomArgs g, float2 *__restrict__ zd,
                                                          f4 *__restrict__ gu, uint32_t spt) {
    const uint32_t nchunk = (g.N + spt - 1) / spt;
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= g.total_tiles * nchunk * kTileRays) return;
    const uint32_t n = t % kTileRays, tc = t / kTileRays;
    const uint32_t tile = tc / nchunk, chunk = tc % nchunk;
    const uint32_t b = tile / g.tiles_per_face;
    uint32_t rl = (tile % g.tiles_per_face) * kTileRays + n;
    const bool ray_ok = rl < g.H * g.W;
    if (!ray_ok) rl = g.H * g.W - 1;                             // padding rays: any value
    const uint32_t y = rl / g.W, x = rl % g.W;
    const uint32_t ray_index = (b * g.H + y) * g.W + x;
    Ray ray;
    make_ray(g.cam + (size_t)b * 12, g.focal[b], g.pix_x[x], g.pix_y[y], g.half_res, ray);
    const float nr = g.near_[b], fr = g.far_[b];
    const float span = __fsub_rn(fr, nr);
    const float dnorm = norm3_torch(ray.d[0], ray.d[1], ray.d[2]);
    const size_t base = (size_t)tile * g.N * kTileRays + n;
    const uint32_t s_end = min(g.N, (chunk + 1) * spt);
    float z = sample_z(g.sc, nr, fr, ray_index, chunk * spt);
    for (uint32_t s = chunk * spt; s < s_end; ++s) {
        const float zn = s + 1 < g.N ? sample_z(g.sc, nr, fr, ray_index, s + 1) : 0.0f;
        if (zd) {
            const float dist = s + 1 < g.N ? __fmul_rn(__fsub_rn(zn, z), dnorm) : __fmul_rn(1e10f, dnorm);
            zd[base + (size_t)s * kTileRays] = make_float2(z, dist);
        }
        f4 u;
        bool in = ray_ok;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float p = __fadd_rn(ray.o[k], __fmul_rn(ray.d[k], z));            // :343
            const float np_ = g.z_normalize ? __fdiv_rn(__fmul_rn(p, 2.0f), span) : p;  // :349
            u[k] = __fdiv_rn(__fadd_rn(np_, g.bound), __fmul_rn(2.0f, g.bound));     // grid.py:149
            if (u[k] < 0 || u[k] > 1) in = false;
        }
        u[3] = in ? 1.0f : 0.0f;
        gu[base + (size_t)s * kTileRays] = u;
        z = zn;
    }
}

// ----------------------------------------------------------------------------
// 3. field: MLP on MFMA + compositing
// ----------------------------------------------------------------------------
constexpr int kStageF4 = kSliceF4 / kThreads;   // float4 staged per thread per slice

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Branch-free sinf for |x| < 2^12 (FiLM arguments are O(100)): Cody-Waite
// reduction by pi/2 with fma (3-part constant), minimax sin/cos on
// [-pi/4, pi/4] (Cephes coefficients), quadrant select.  Max error ~1e-7
// absolute; straight-line code so the compiler can interleave it with MFMA.
__device__ __forceinline__ float sin_cw(float x) {
    const float kf = __builtin_rintf(x * 0.636619772367581343f);
    const int q = (int)kf;
    float r = __fmaf_rn(-kf, 1.57079637050628662109375f, x);
    r = __fmaf_rn(-kf, -4.37113900018624283e-8f, r);
    r = __fmaf_rn(-kf, -1.71512451000597797e-15f, r);
    const float r2 = r * r;
    float ps = __fmaf_rn(r2, -1.9515295891e-4f, 8.3321608736e-3f);
    ps = __fmaf_rn(r2, ps, -1.6666654611e-1f);
    const float sn = __fmaf_rn(r * r2, ps, r);
    float pc = __fmaf_rn(r2, 2.443315711809948e-5f, -1.388731625493765e-3f);
    pc = __fmaf_rn(r2, pc, 4.166664568298827e-2f);
    const float cs = __fmaf_rn(r2 * r2, pc, __fmaf_rn(-0.5f, r2, 1.0f));
    const float v = (q & 1) ? cs : sn;
    return (q & 2) ? -v : v;
}

// The FiLM activation's sin: hardware v_sin_f32 after reduction (max |err|
// 3.7e-7 on |x| <= 200, measured; 1 transcendental + 6 VALU) instead of the
// polynomial (9e-8, ~17 VALU).  Both errors sit an order of magnitude below
// the fp32 summation-order differences of the MFMA GEMMs they feed.
__device__ __forceinline__ float kSin(float x) { return sin_hw(x); }

__global__ void sin_probe_kernel(const float *__restrict__ x, float *__restrict__ cw,
                                 float *__restrict__ hw, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    cw[i] = sin_cw(x[i]);
    hw[i] = sin_hw(x[i]);
}

__global__ void sin_rev_probe_kernel(const float *__restrict__ u, float *__restrict__ out,
                                     uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = sin_rev(u[i]);
}

// Camera extrinsics from sampled angles (sdf_utils.py:136-159, after the random
// draws), one thread per camera: the op chain of generate_camera_params in one
// launch instead of ~25 elementwise / reduction kernels.  Each op rounds once,
// as the tensor ops do; the library's sinf / cosf / sqrtf and the order of the
// 3-term norm may differ from torch's kernels by an ulp.
struct CamArgs {
    const float *azim, *elev;      // [B]
    float *ext, *vp;               // [B,3,4], [B,2]
    float *focal, *near_, *far_;   // [B] each
    float radius, fov_ang, half_res;
    uint32_t B;
};

__device__ __forceinline__ void cam_normalize(float (&v)[3]) {   // F.normalize(eps = 1e-5)
    const float n = fmaxf(__fsqrt_rn(__fadd_rn(__fadd_rn(__fmul_rn(v[0], v[0]), __fmul_rn(v[1], v[1])),
                                               __fmul_rn(v[2], v[2]))), 1e-5f);
    v[0] = __fdiv_rn(v[0], n);
    v[1] = __fdiv_rn(v[1], n);
    v[2] = __fdiv_rn(v[2], n);
}

__device__ __forceinline__ void cam_cross(const float (&a)[3], const float (&b)[3], float (&c)[3]) {
    c[0] = __fsub_rn(__fmul_rn(a[1], b[2]), __fmul_rn(a[2], b[1]));
    c[1] = __fsub_rn(__fmul_rn(a[2], b[0]), __fmul_rn(a[0], b[2]));
    c[2] = __fsub_rn(__fmul_rn(a[0], b[1]), __fmul_rn(a[1], b[0]));
}

__global__ void camera_kernel(const CamArgs c) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= c.B) return;
    const float az = c.azim[b], el = c.elev[b];
    c.vp[2 * b] = az;
    c.vp[2 * b + 1] = el;
    // dist = 1: near / far = dist -/+ radius; fov = fov_ang * pi / 180; focal = 0.5 res / tan(fov)
    c.near_[b] = __fsub_rn(1.0f, c.radius);
    c.far_[b] = __fadd_rn(1.0f, c.radius);
    const float fov = __fdiv_rn(__fmul_rn(c.fov_ang, (float)M_PI), 180.0f);
    c.focal[b] = __fdiv_rn(c.half_res, tanf(fov));
    const float ce = cosf(el);
    float dir[3] = {__fmul_rn(ce, sinf(az)), sinf(el), __fmul_rn(ce, cosf(az))};
    const float up[3] = {0.0f, 1.0f, 0.0f};
    float z[3] = {dir[0], dir[1], dir[2]}, x[3], y[3];
    cam_normalize(z);
    cam_cross(up, z, x);
    cam_normalize(x);
    cam_cross(z, x, y);
    cam_normalize(y);
    if (fabsf(x[0]) <= 5e-3f && fabsf(x[1]) <= 5e-3f && fabsf(x[2]) <= 5e-3f) {   // isclose(x, 0)
        cam_cross(y, z, x);
        cam_normalize(x);
    }
    float *e = c.ext + 12 * (size_t)b;       // [R^T | T], R rows = x, y, z; T = 1 * dir
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        e[4 * i + 0] = x[i];
        e[4 * i + 1] = y[i];
        e[4 * i + 2] = z[i];
        e[4 * i + 3] = dir[i];
    }
}

// Streaming state for the weight ring: slot s of `lds` holds one K-slice.
struct Ring {
    f4 *lds;              // [3][kSliceF4]
    const f4 *packed;
    f4 st[kStageF4];      // staged next slice (global -> regs -> LDS)
    uint32_t it;          // global slice iteration
    uint32_t tid;
};

struct NoSide {
    __device__ __forceinline__ void operator()() const {}
};

// One K-slice: stage slice it+1 into LDS, prefetch slice it+2, run the
// 16 t_out x 4 MFMAs of slice `it` against the B operand quad, barrier.
// A-operand quads are read four output tiles at a time, one group ahead,
// and the four accumulators of a group are interleaved so no MFMA waits on
// its predecessor (16x16x4 f32: 32-cycle issue, 40-cycle dependency).
// `side` is register work (the previous layer's activation of one tile, the
// compositing math...) placed in the same basic block as the MFMAs, so the
// scheduler issues it in the MFMA shadow instead of after the layer.
// Ablation variants (profiling builds only, selected by
// sdfr_debug_set_field_variant; V = 0 is the product): bit 0 drops the
// barrier, bit 1 the LDS A-operand reads, bit 2 the ring staging, bit 3 the
// activations.  Any V != 0 computes wrong results by construction.
enum : int { ABL_BARRIER = 1, ABL_LDSREAD = 2, ABL_STAGE = 4, ABL_ACT = 8 };

template <int V, class Side>
__device__ __forceinline__ void ring_step(Ring &R, f4 (&acc)[16], const f4 bq, Side &&side) {
    const uint32_t cur = R.it % 3u, nxt = (R.it + 1u) % 3u;
    // all 16 A-operand quads of this slice are read up front (one LDS latency
    // per slice, nothing queued ahead of them in the LDS pipe), then 4
    // accumulators are interleaved per MFMA group
    const f4 *A = R.lds + cur * kSliceF4 + (R.tid & 63u);
    f4 a[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = (V & ABL_LDSREAD) ? bq * (float)(i + 1) : A[i * 64];
#pragma unroll
    for (int grp = 0; grp < 4; ++grp) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            acc[4 * grp + i] = mfma4(a[4 * grp + i].x, bq.x, acc[4 * grp + i]);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            acc[4 * grp + i] = mfma4(a[4 * grp + i].y, bq.y, acc[4 * grp + i]);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            acc[4 * grp + i] = mfma4(a[4 * grp + i].z, bq.z, acc[4 * grp + i]);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            acc[4 * grp + i] = mfma4(a[4 * grp + i].w, bq.w, acc[4 * grp + i]);
    }
    side();
    if constexpr (!(V & ABL_STAGE)) {
        // slice it+1 (loaded at the end of the previous slice, so it had this
        // slice's whole MFMA body to land) -> LDS slot; then slice it+2 -> regs.
        // Writing at the END keeps the LDS writes out of the way of this
        // slice's A-operand reads.
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < kStageF4; ++i) R.lds[nxt * kSliceF4 + R.tid + i * kThreads] = R.st[i];
        const uint32_t pf = (R.it + 2u) % kSlices;
#pragma unroll
        for (int i = 0; i < kStageF4; ++i)
            R.st[i] = R.packed[pf * kSliceF4 + R.tid + i * kThreads];
    }
    if constexpr (!(V & ABL_BARRIER)) __syncthreads();
    ++R.it;
}

// Keep a register value's computation on this side of the next barrier: pure
// VALU work is otherwise free to float past s_barrier to its first use (the
// next slice), which would serialise it in front of that slice's MFMAs.
__device__ __forceinline__ void pin(f4 &x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(float &x) { asm volatile("" : "+v"(x)); }

// One tile of a FiLM activation, in place: x = sin(gamma*x + beta) with the
// reference's two roundings (sdf_model.py:67).
template <int V>
__device__ __forceinline__ void film_tile(f4 &x, const float *gam, const float *bet, int t,
                                          uint32_t g) {
    if constexpr ((V & ABL_ACT) != 0) return;
    const f4 gm = *reinterpret_cast<const f4 *>(gam + 16 * t + 4 * g);
    const f4 bt = *reinterpret_cast<const f4 *>(bet + 16 * t + 4 * g);
    x.x = kSin(__fadd_rn(__fmul_rn(gm.x, x.x), bt.x));
    x.y = kSin(__fadd_rn(__fmul_rn(gm.y, x.y), bt.y));
    x.z = kSin(__fadd_rn(__fmul_rn(gm.z, x.z), bt.z));
    x.w = kSin(__fadd_rn(__fmul_rn(gm.w, x.w), bt.w));
    pin(x);
}

__device__ __forceinline__ void init_bias(f4 (&acc)[16], const float *bias, uint32_t g) {
#pragma unroll
    for (int t = 0; t < 16; ++t) acc[t] = *reinterpret_cast<const f4 *>(bias + 16 * t + 4 * g);
}

// sin(gamma * out + beta) with the reference's two roundings (sdf_model.py:67)
__device__ __forceinline__ void film_act(f4 (&act)[16], const f4 (&acc)[16],
                                         const float *gam, const float *bet, uint32_t g) {
#pragma unroll
    for (int t = 0; t < 16; ++t) {
        const f4 gm = *reinterpret_cast<const f4 *>(gam + 16 * t + 4 * g);
        const f4 bt = *reinterpret_cast<const f4 *>(bet + 16 * t + 4 * g);
        f4 v;
        v.x = sin_cw(__fadd_rn(__fmul_rn(gm.x, acc[t].x), bt.x));
        v.y = sin_cw(__fadd_rn(__fmul_rn(gm.y, acc[t].y), bt.y));
        v.z = sin_cw(__fadd_rn(__fmul_rn(gm.z, acc[t].z), bt.z));
        v.w = sin_cw(__fadd_rn(__fmul_rn(gm.w, acc[t].w), bt.w));
        act[t] = v;
    }
}

__device__ __forceinline__ float dot_feat(const f4 (&act)[16], const float *w, uint32_t g) {
    float p = 0.0f;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
        const f4 wv = *reinterpret_cast<const f4 *>(w + 16 * t + 4 * g);
        p = __fmaf_rn(act[t].x, wv.x, p);
        p = __fmaf_rn(act[t].y, wv.y, p);
        p = __fmaf_rn(act[t].z, wv.z, p);
        p = __fmaf_rn(act[t].w, wv.w, p);
    }
    return group_sum(p);
}

template <int V>
__global__ void __launch_bounds__(kThreads, 1) ngp_field_kernel(const FieldArgs a) {
    __shared__ f4 ring_lds[3 * kSliceF4];   // 48 KB weight ring
    __shared__ float cst[kCst];              // 9 KB biases + sigma/rgb rows
    __shared__ float film_lds[kWaves][kFilm * 2 * kW];   // 32 KB: each wave's face
    __shared__ f4 facc_lds[kWaves][16 * 64];              // 64 KB: feature accumulators
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t n = lane & 15u, g = lane >> 4;
    const GeomArgs &G = a.g;

    uint32_t tile = blockIdx.x * kWaves + wave;
    const bool tile_ok = tile < G.total_tiles;
    if (!tile_ok) tile = G.total_tiles - 1;
    const uint32_t b = tile / G.tiles_per_face;
    uint32_t ray_local = (tile % G.tiles_per_face) * kTileRays + n;
    const bool ray_ok = tile_ok && ray_local < G.H * G.W;
    if (ray_local >= G.H * G.W) ray_local = G.H * G.W - 1;
    const uint32_t py = ray_local / G.W, px = ray_local % G.W;
    const uint32_t ray_index = (b * G.H + py) * G.W + px;

    Ray ray;
    make_ray(G.cam + (size_t)b * 12, G.focal[b], G.pix_x[px], G.pix_y[py], G.half_res, ray);
    const float nr = G.near_[b], fr = G.far_[b];
    const float dnorm = norm3_torch(ray.d[0], ray.d[1], ray.d[2]);
    f4 shq;
    {
        const float v0 = G.static_viewdirs ? ray.dir[0] : ray.d[0];
        const float v1 = G.static_viewdirs ? ray.dir[1] : ray.d[1];
        const float v2 = G.static_viewdirs ? ray.dir[2] : ray.d[2];
        const float vn = norm3_torch(v0, v1, v2);
        shq = sh_quad(__fdiv_rn(v0, vn), __fdiv_rn(v1, vn), __fdiv_rn(v2, vn), g);
    }
    const float beta_s = a.with_sdf ? a.sigmoid_beta[0] : 1.0f;
    {
        // this wave's face FiLM vectors (gamma/beta x 4 layers) -> LDS (own region,
        // read back only by this wave: no barrier needed beyond the prologue one)
        const f4 *src = reinterpret_cast<const f4 *>(a.film + (size_t)b * kFilm * 2 * kW);
        f4 *dst = reinterpret_cast<f4 *>(film_lds[wave]);
#pragma unroll
        for (uint32_t i = lane; i < kFilm * 2 * kW / 4; i += 64) dst[i] = src[i];
    }
    const float *film = film_lds[wave];

    Ring R;
    R.lds = ring_lds;
    R.packed = a.packed;
    R.tid = tid;
    R.it = 0;
    // per-network constants (5 biases, sigma_linear and rgb_linear rows) in LDS
    for (uint32_t i = tid; i < kCst; i += kThreads) {
        float v;
        if (i < 5 * kW) v = a.bias[i / kW][i % kW];
        else if (i < 6 * kW) v = a.sigma_w[i - 5 * kW];
        else v = a.rgb_w[i - 6 * kW];
        cst[i] = v;
    }
    // prologue: slice 0 -> slot 0, slice 1 -> regs
#pragma unroll
    for (int i = 0; i < kStageF4; ++i) R.lds[tid + i * kThreads] = a.packed[tid + i * kThreads];
#pragma unroll
    for (int i = 0; i < kStageF4; ++i) R.st[i] = a.packed[kSliceF4 + tid + i * kThreads];
    __syncthreads();

    // composited features sum_s w_s f_s live in this wave's LDS region (lane-
    // contiguous float4, conflict-free), not in 64 VGPRs per lane
    f4 *facc = facc_lds[wave];
#pragma unroll
    for (int t = 0; t < 16; ++t) facc[t * 64 + lane] = f4{0.0f, 0.0f, 0.0f, 0.0f};
    float T = 1.0f, wsum = 0.0f, racc0 = 0.0f, racc1 = 0.0f, racc2 = 0.0f;
    float xacc0 = 0.0f, xacc1 = 0.0f, xacc2 = 0.0f, w_last = 0.0f;

    const float2 *enc2 = reinterpret_cast<const float2 *>(a.enc);
    float z = sample_z(G.sc, nr, fr, ray_index, 0);
    const float *f0g = film, *f0b = film + kW, *f1g = film + 2 * kW, *f1b = film + 3 * kW;
    const float *f2g = film + 4 * kW, *f2b = film + 5 * kW, *f3g = film + 6 * kW,
                *f3b = film + 7 * kW;
    const float *bias_l = cst;                        // [5][256] in LDS
    const float *sig_w = cst + 5 * kW, *rgb_w = cst + 6 * kW;
    const float sig_b = a.sigma_b[0];
    const float rgb_b0 = a.rgb_b[0], rgb_b1 = a.rgb_b[1], rgb_b2 = a.rgb_b[2];

    // hash-grid features of sample 0 (levels 2g,2g+1 | 8+2g,9+2g of this lane group)
    size_t sid = (size_t)(tile * G.N) * kTileRays + n;
    float2 e0 = enc2[(2 * g) * (size_t)G.S_total + sid];
    float2 e1 = enc2[(2 * g + 1) * (size_t)G.S_total + sid];
    float2 e2 = enc2[(8 + 2 * g) * (size_t)G.S_total + sid];
    float2 e3 = enc2[(9 + 2 * g) * (size_t)G.S_total + sid];

    for (uint32_t s = 0; s < G.N; ++s) {
        const f4 in_lo = f4{e0.x, e0.y, e1.x, e1.y}, in_hi = f4{e2.x, e2.y, e3.x, e3.y};
        const float z_next = (s + 1 < G.N) ? sample_z(G.sc, nr, fr, ray_index, s + 1) : 0.0f;
        float sdf = 0.0f, w = 0.0f;
        f4 X[16], Y[16];
        // Software pipeline: layer l accumulates into one register set while
        // the previous layer's tiles are activated (sin) one slice ahead of
        // their use as B operands, inside the MFMA stream.
        // layer 0: input_linear (32 -> 256), identity LinearLayer -> X
        init_bias(X, bias_l, g);
        ring_step<V>(R, X, in_lo, [&] {
            if (s + 1 < G.N) {                        // prefetch the next sample's features
                sid += kTileRays;
                e0 = enc2[(2 * g) * (size_t)G.S_total + sid];
                e1 = enc2[(2 * g + 1) * (size_t)G.S_total + sid];
                e2 = enc2[(8 + 2 * g) * (size_t)G.S_total + sid];
                e3 = enc2[(9 + 2 * g) * (size_t)G.S_total + sid];
            }
        });
        ring_step<V>(R, X, in_hi, NoSide{});
        // layer 1: FiLM pts_linears.0 -> Y
        init_bias(Y, bias_l + kW, g);
#pragma unroll
        for (int t = 0; t < 16; ++t)
            ring_step<V>(R, Y, X[t], [&] {
                if (t == 15) film_tile<V>(Y[0], f0g, f0b, 0, g);
            });
        // layer 2: FiLM pts_linears.1 -> X
        init_bias(X, bias_l + 2 * kW, g);
#pragma unroll
        for (int t = 0; t < 16; ++t)
            ring_step<V>(R, X, Y[t], [&] {
                if (t < 15) film_tile<V>(Y[t + 1], f0g, f0b, t + 1, g);
                else film_tile<V>(X[0], f1g, f1b, 0, g);
            });
        // layer 3: FiLM pts_linears.2 -> Y
        init_bias(Y, bias_l + 3 * kW, g);
#pragma unroll
        for (int t = 0; t < 16; ++t)
            ring_step<V>(R, Y, X[t], [&] {
                if (t < 15) film_tile<V>(X[t + 1], f1g, f1b, t + 1, g);
                else film_tile<V>(Y[0], f2g, f2b, 0, g);
            });
        // layer 4: views FiLM ([h3, SH] 272 -> 256) -> X; sigma_linear and the
        // sample's compositing weight ride in the last h3 slice
        init_bias(X, bias_l + 4 * kW, g);
#pragma unroll
        for (int t = 0; t < 16; ++t)
            ring_step<V>(R, X, Y[t], [&] {
                if (t < 15) {
                    film_tile<V>(Y[t + 1], f2g, f2b, t + 1, g);
                } else {
                    sdf = __fadd_rn(dot_feat(Y, sig_w, g), sig_b);
                    // volume_integration (sdf_model.py:236-301), front to back
                    const float dist = (s + 1 < G.N) ? __fmul_rn(__fsub_rn(z_next, z), dnorm)
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
                    w = alpha * T;
                    if (a.force_background && s + 1 == G.N) w = 1.0f - wsum;
                    T = T * ((1.0f - alpha) + 1e-10f);
                    wsum += w;
                }
            });
        ring_step<V>(R, X, shq, NoSide{});
        // colour features f = sin(gamma_v * . + beta_v); rgb_linear; compositing
#pragma unroll
        for (int t = 0; t < 16; ++t) film_tile<V>(X[t], f3g, f3b, t, g);
        const float r0 = __fadd_rn(dot_feat(X, rgb_w, g), rgb_b0);
        const float r1 = __fadd_rn(dot_feat(X, rgb_w + kW, g), rgb_b1);
        const float r2 = __fadd_rn(dot_feat(X, rgb_w + 2 * kW, g), rgb_b2);
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
                v.x = __fmaf_rn(w, X[t].x, v.x);
                v.y = __fmaf_rn(w, X[t].y, v.y);
                v.z = __fmaf_rn(w, X[t].z, v.z);
                v.w = __fmaf_rn(w, X[t].w, v.w);
                facc[t * 64 + lane] = v;
            }
        }
        if (a.sdf && ray_ok && g == 0) a.sdf[(size_t)ray_index * G.N + s] = sdf;
        z = z_next;
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
            const uint32_t j = 16 * t + 4 * g;
            const f4 v = facc[t * 64 + lane];
            fb[(size_t)(j + 0) * HW] = v.x;
            fb[(size_t)(j + 1) * HW] = v.y;
            fb[(size_t)(j + 2) * HW] = v.z;
            fb[(size_t)(j + 3) * HW] = v.w;
        }
    }
}

// ----------------------------------------------------------------------------
// host side
// ----------------------------------------------------------------------------
struct Workspace {
    float *enc;
    f4 *packed;
    float *film;
};

static size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

// enc [L][S][2] | packed fp32 fragments | film | split-fp16 region (field_f16x3.hip) |
// segment partials | zd [S] (z, segment length) | gu [S] (grid coordinate, inside flag)
static size_t ws_layout(uint32_t B, uint32_t H, uint32_t W, uint32_t N, uint32_t L,
                        size_t *o_packed, size_t *o_film, size_t *o_x = nullptr,
                        size_t *o_part = nullptr, size_t *o_zd = nullptr,
                        size_t *o_gu = nullptr) {
    const size_t tiles = (size_t)B * ((H * W + kTileRays - 1) / kTileRays);
    const size_t S = tiles * N * kTileRays;
    size_t off = align256(S * L * 2 * sizeof(float));
    *o_packed = off;
    off += align256((size_t)kSlices * kSliceF4 * sizeof(f4));
    *o_film = off;
    off += align256((size_t)B * kFilm * 2 * kW * sizeof(float));
    if (o_x) *o_x = off;
    off += align256(f16x3_ws_bytes(0));
    if (o_part) *o_part = off;
    off += align256(field_part_bytes(B, (H * W + kTileRays - 1) / kTileRays, N));
    if (o_zd) *o_zd = off;
    off += align256(S * 2 * sizeof(float));
    if (o_gu) *o_gu = off;
    off += align256(S * 4 * sizeof(float));
    return off;
}

static int validate(const sdfr_ngp_weights *w, const sdfr_ngp_render_args *a) {
    if (!w || !a) return fail(SDFR_EINVAL, "render_ngp: null args");
    if (w->num_levels != 16)
        return fail(SDFR_EUNSUPPORTED, "render_ngp: fused path needs 16 levels x 2 features");
    if (a->B == 0 || a->H == 0 || a->W == 0 || a->N == 0)
        return fail(SDFR_EINVAL, "render_ngp: empty batch / image / sample count");
    if (a->field_precision != SDFR_FIELD_F16X3 && a->field_precision != SDFR_FIELD_FP32)
        return fail(SDFR_EINVAL, "render_ngp: field_precision must be 0 (f16x3) or 1 (fp32)");
    if (a->max_field_segments > kFieldSplitMax || a->max_field_segments == 3)
        return fail(SDFR_EINVAL, "render_ngp: max_field_segments must be 0, 1, 2 or 4");
    if (!a->cam || !a->focal || !a->near_ || !a->far_ || !a->styles || !a->pix_x ||
        !a->pix_y || !a->t_vals || !a->rgb || !a->workspace)
        return fail(SDFR_EINVAL, "render_ngp: required pointer is null");
    const void *need[] = {w->embeddings, w->offsets, w->input_w, w->input_b, w->views_w,
                          w->views_b, w->views_gw, w->views_gb, w->views_bw, w->views_bb,
                          w->sigma_w, w->sigma_b, w->rgb_w, w->rgb_b};
    for (const void *p : need)
        if (!p) return fail(SDFR_EINVAL, "render_ngp: weight pointer is null");
    if (a->with_sdf && !w->sigmoid_beta)
        return fail(SDFR_EINVAL, "render_ngp: sigmoid_beta is required when with_sdf");
    if (a->features_split) {
        if (a->field_precision != SDFR_FIELD_F16X3)
            return fail(SDFR_EUNSUPPORTED, "render_ngp: features_split needs the f16x3 field");
        if (a->features || !a->features_mod)
            return fail(SDFR_EINVAL, "render_ngp: features_split takes features_mod and no features");
    }
    for (int l = 0; l < 3; ++l)
        if (!w->pts_w[l] || !w->pts_b[l] || !w->pts_gw[l] || !w->pts_gb[l] || !w->pts_bw[l] ||
            !w->pts_bb[l])
            return fail(SDFR_EINVAL, "render_ngp: FiLM weight pointer is null");
    size_t op, of;
    if (a->workspace_bytes < ws_layout(a->B, a->H, a->W, a->N, 16, &op, &of))
        return fail(SDFR_EINVAL, "render_ngp: workspace too small");
    const uint64_t S = (uint64_t)a->B * ((a->H * a->W + 15) / 16) * a->N * 16;
    if (S * 16 >= (1ull << 32))
        return fail(SDFR_EINVAL, "render_ngp: too many samples per call (split the batch)");
    return SDFR_OK;
}

static void fill_geom(const sdfr_ngp_weights *w, const sdfr_ngp_render_args *a, GeomArgs &g) {
    fill_geom_args(a, w->bound, g);
}

void fill_geom_args(const sdfr_ngp_render_args *a, float bound, GeomArgs &g) {
    g.B = a->B;
    g.H = a->H;
    g.W = a->W;
    g.N = a->N;
    g.tiles_per_face = (a->H * a->W + kTileRays - 1) / kTileRays;
    g.total_tiles = a->B * g.tiles_per_face;
    g.S_total = g.total_tiles * a->N * kTileRays;
    g.half_res = (float)a->W * 0.5f;   // get_rays uses out_im_res * .5 for both axes
    g.cam = a->cam;
    g.focal = a->focal;
    g.near_ = a->near_;
    g.far_ = a->far_;
    g.pix_x = a->pix_x;
    g.pix_y = a->pix_y;
    g.sc.t_vals = a->t_vals;
    g.sc.t_rand = a->t_rand;
    g.sc.t_rand_per_sample = a->t_rand_per_sample;
    g.sc.offset_sampling = a->offset_sampling;
    g.sc.N = a->N;
    g.static_viewdirs = a->static_viewdirs;
    g.z_normalize = a->z_normalize;
    g.bound = bound;
}

void record_event(void *ev, hipStream_t st) {
    if (ev) (void)hipEventRecord(reinterpret_cast<hipEvent_t>(ev), st);
}

void wait_event(void *ev, hipStream_t st) {
    if (ev) (void)hipStreamWaitEvent(st, reinterpret_cast<hipEvent_t>(ev), 0);
}

#ifdef SDFR_ABLATION
static int g_field_variant = 0;   // profiling ablations only (see ABL_*)
int field_variant() { return g_field_variant; }
#else
int field_variant() { return 0; }
#endif

static void launch_field(int v, dim3 grid, hipStream_t st, const FieldArgs &f) {
    switch (v) {
#ifdef SDFR_ABLATION
#define SDFR_FIELD_CASE(V)                                                                   \
    case V:                                                                                  \
        hipLaunchKernelGGL(ngp_field_kernel<V>, grid, dim3(kThreads), 0, st, f);             \
        return;
        SDFR_FIELD_CASE(1)
        SDFR_FIELD_CASE(2)
        SDFR_FIELD_CASE(4)
        SDFR_FIELD_CASE(8)
        SDFR_FIELD_CASE(15)
        SDFR_FIELD_CASE(16)
        SDFR_FIELD_CASE(31)
#undef SDFR_FIELD_CASE
#endif
        default:
            hipLaunchKernelGGL(ngp_field_kernel<0>, grid, dim3(kThreads), 0, st, f);
    }
}


static int launch_prep(const sdfr_ngp_weights *w, const sdfr_ngp_render_args *a, f4 *packed,
                       float *film, hipStream_t st) {
    PrepArgs p;
    p.styles = a->styles;
    for (int l = 0; l < 3; ++l) {
        p.gw[l] = w->pts_gw[l];
        p.gb[l] = w->pts_gb[l];
        p.bw[l] = w->pts_bw[l];
        p.bb[l] = w->pts_bb[l];
        p.w[1 + l] = w->pts_w[l];
        p.K[1 + l] = kW;
    }
    p.gw[3] = w->views_gw;
    p.gb[3] = w->views_gb;
    p.bw[3] = w->views_bw;
    p.bb[3] = w->views_bb;
    p.w[0] = w->input_w;
    p.K[0] = kFeatIn;
    p.w[4] = w->views_w;
    p.K[4] = kViewsIn;
    p.film = film;
    p.packed = packed;
    p.B = a->B;
    const uint32_t blocks = a->B * kFilm * 2 + (kSlices * kSliceF4 + 255) / 256;
    hipLaunchKernelGGL(ngp_prep_kernel, dim3(blocks), dim3(256), 0, st, p);
    return check_launch("render_ngp: prep");
}

#ifdef SDFR_ABLATION
static uint32_t g_encode_mode = [] {
    const char *e = std::getenv("SDFR_ENC_MODE");   // ablations only
    return e ? (uint32_t)std::atoi(e) : kEncDefault;
}();
#endif

template <bool PAIR, bool A8, uint32_t LPT, uint32_t SPT>
static void launch_encode_mode(hipStream_t st, const EncodeArgs &e) {
    const uint32_t blocks = (e.g.S_total + 256 * SPT - 1) / (256 * SPT);
    hipLaunchKernelGGL((ngp_encode_kernel<PAIR, A8, LPT, SPT>), dim3(blocks, 16 / LPT),
                       dim3(256), 0, st, e);
}

// the per-sample geometry (sample_geom_kernel: gu always, zd when wanted)
static int launch_geom(const GeomArgs &g, float2 *zd, f4 *gu, hipStream_t st) {
    // samples per thread: all N, split while fewer than 64 k threads would run
    uint32_t spt = g.N;
    while (spt > 1 && (uint64_t)g.total_tiles * kTileRays * ((g.N + spt - 1) / spt) < 65536)
        spt = (spt + 1) / 2;
    const uint64_t threads = (uint64_t)g.total_tiles * kTileRays * ((g.N + spt - 1) / spt);
    hipLaunchKernelGGL(sample_geom_kernel, dim3((uint32_t)((threads + 255) / 256)), dim3(256),
                       0, st, g, zd, gu, spt);
    return check_launch("render_ngp: sample geometry");
}

static int launch_encode(const sdfr_ngp_weights *w, const sdfr_ngp_render_args *a,
                         const GeomArgs &g, float *enc, const f4 *gu, hipStream_t st) {
    EncodeArgs e;
    e.g = g;
    e.emb = w->embeddings;
    e.offsets = w->offsets;
    e.gu = gu;
    e.enc = enc;
    e.pair_ok = (reinterpret_cast<uintptr_t>(w->embeddings) & 15u) == 0;
    make_level_table(16, w->log2_per_level_scale, w->base_resolution, e.lt);
#ifdef SDFR_ABLATION
    switch (g_encode_mode) {
        case 8 | 1: launch_encode_mode<false, false, 1, 1>(st, e); break;
        case 1: launch_encode_mode<true, false, 1, 1>(st, e); break;
        case 2: launch_encode_mode<true, false, 2, 1>(st, e); break;
        case 32 | 1: launch_encode_mode<true, false, 1, 2>(st, e); break;
        case 256 | 1: launch_encode_mode<true, true, 1, 1>(st, e); break;
        case 256 | 2: launch_encode_mode<true, true, 2, 1>(st, e); break;
        case 256 | 32 | 2: launch_encode_mode<true, true, 2, 2>(st, e); break;
        case 256 | 32 | 1: launch_encode_mode<true, true, 1, 2>(st, e); break;
        default: launch_encode_mode<true, true, 1, 1>(st, e); break;   // 257
    }
#else
    static_assert(kEncDefault == (256 | 1), "product gather: A8, 1 level, 1 sample per thread");
    launch_encode_mode<true, true, 1, 1>(st, e);
#endif
    return check_launch("render_ngp: encode");
}

}  // namespace sdfr

using namespace sdfr;

extern "C" {

int sdfr_debug_sin_probe(const float *x, float *out_cw, float *out_hw, uint32_t n,
                         void *stream) {
    if (n == 0) return SDFR_OK;
    hipLaunchKernelGGL(sin_probe_kernel, dim3((n + 255) / 256), dim3(256), 0,
                       (hipStream_t)stream, x, out_cw, out_hw, n);
    return check_launch("sin_probe");
}

int sdfr_debug_sin_rev_probe(const float *u, float *out, uint32_t n, void *stream) {
    if (n == 0) return SDFR_OK;
    hipLaunchKernelGGL(sin_rev_probe_kernel, dim3((n + 255) / 256), dim3(256), 0,
                       (hipStream_t)stream, u, out, n);
    return check_launch("sin_rev_probe");
}

int sdfr_camera_extrinsics(const float *azim, const float *elev, uint32_t B, float dist_radius,
                           float fov_ang, float half_res, float *ext, float *focal, float *near_,
                           float *far_, float *viewpoint, void *stream) {
    if (B == 0) return SDFR_OK;
    if (!azim || !elev || !ext || !viewpoint || !focal || !near_ || !far_)
        return fail(SDFR_EINVAL, "camera_extrinsics: null tensor pointer");
    hipLaunchKernelGGL(camera_kernel, dim3((B + 63) / 64), dim3(64), 0, (hipStream_t)stream,
                       CamArgs{azim, elev, ext, viewpoint, focal, near_, far_, dist_radius,
                               fov_ang, half_res, B});
    return check_launch("camera_extrinsics");
}

#ifdef SDFR_ABLATION
// profiling hooks (make ABLATION=1 builds only; process-global)
int sdfr_debug_set_encode_mode(int mode) {
    const int ok[] = {1, 2, 9, 33, 257, 258, 289, 290};
    bool found = false;
    for (int m : ok) found |= m == mode;
    if (!found)
        return fail(SDFR_EINVAL,
                    "sdfr_debug_set_encode_mode: unknown mode");
    g_encode_mode = (uint32_t)mode;
    return SDFR_OK;
}

int sdfr_debug_set_field_variant(int variant) {
    const int ok[] = {0, 1, 2, 4, 8, 15, 16, 31};
    for (int v : ok)
        if (v == variant) {
            g_field_variant = variant;
            return SDFR_OK;
        }
    return fail(SDFR_EINVAL,
                "sdfr_debug_set_field_variant: variant must be 0,1,2,4,8,15,16,31");
}
#endif

size_t sdfr_render_ngp_workspace_bytes(uint32_t B, uint32_t H, uint32_t W, uint32_t N,
                                       uint32_t num_levels) {
    size_t op, of;
    return ws_layout(B, H, W, N, num_levels, &op, &of);
}

int sdfr_render_ngp_encode_only(const sdfr_ngp_weights *w, const sdfr_ngp_render_args *a,
                                void *stream) {
    int rc = validate(w, a);
    if (rc) return rc;
    GeomArgs g;
    fill_geom(w, a, g);
    size_t o_packed, o_film, o_x, o_part, o_zd, o_gu;
    ws_layout(a->B, a->H, a->W, a->N, 16, &o_packed, &o_film, &o_x, &o_part, &o_zd, &o_gu);
    char *ws = reinterpret_cast<char *>(a->workspace);
    f4 *gu = reinterpret_cast<f4 *>(ws + o_gu);
    hipStream_t st = (hipStream_t)stream;
    if ((rc = launch_geom(g, nullptr, gu, st))) return rc;
    return launch_encode(w, a, g, reinterpret_cast<float *>(ws), gu, st);
}

int sdfr_render_ngp_forward(const sdfr_ngp_weights *w, const sdfr_ngp_render_args *a,
                            void *stream) {
    int rc = validate(w, a);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    size_t o_packed, o_film, o_x, o_part, o_zd, o_gu;
    ws_layout(a->B, a->H, a->W, a->N, 16, &o_packed, &o_film, &o_x, &o_part, &o_zd, &o_gu);
    char *ws = reinterpret_cast<char *>(a->workspace);
    float *enc = reinterpret_cast<float *>(ws);
    f4 *packed = reinterpret_cast<f4 *>(ws + o_packed);
    float *film = reinterpret_cast<float *>(ws + o_film);
    f4 *gu = reinterpret_cast<f4 *>(ws + o_gu);

    GeomArgs g;
    fill_geom(w, a, g);
    record_event(a->stage_events[0], st);
    if (a->field_precision == SDFR_FIELD_F16X3) {
        // geometry and gather first (they do not read the styles), then the wait on
        // the caller's styles (ABI 11), the FiLM prep and the field kernel
        float2 *zd = reinterpret_cast<float2 *>(ws + o_zd);
        if ((rc = launch_geom(g, zd, gu, st))) return rc;
        record_event(a->stage_events[1], st);                  // the encode stage is the gather alone
        if ((rc = launch_encode(w, a, g, enc, gu, st))) return rc;
        record_event(a->stage_events[2], st);
        wait_event(a->styles_event, st);
        if ((rc = launch_xprep_ngp(w, a, ws + o_x, film, st))) return rc;
        record_event(a->field_event, st);
        float *part = reinterpret_cast<float *>(ws + o_part);
        if ((rc = launch_xfield_ngp(w, a, g, enc, ws + o_x, film, st, part, zd))) return rc;
        record_event(a->stage_events[3], st);
        return SDFR_OK;
    }
    wait_event(a->styles_event, st);
    if ((rc = launch_prep(w, a, packed, film, st))) return rc;
    if ((rc = launch_geom(g, nullptr, gu, st))) return rc;
    record_event(a->stage_events[1], st);
    if ((rc = launch_encode(w, a, g, enc, gu, st))) return rc;
    record_event(a->stage_events[2], st);
    record_event(a->field_event, st);

    FieldArgs f;
    f.g = g;
    f.enc = enc;
    f.packed = packed;
    f.film = film;
    f.bias[0] = w->input_b;
    for (int l = 0; l < 3; ++l) f.bias[1 + l] = w->pts_b[l];
    f.bias[4] = w->views_b;
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
    const uint32_t blocks = (g.total_tiles + kWaves - 1) / kWaves;
    launch_field(field_variant(), dim3(blocks), st, f);
    if ((rc = check_launch("render_ngp: field"))) return rc;
    record_event(a->stage_events[3], st);
    return SDFR_OK;
}

}  // extern "C"
