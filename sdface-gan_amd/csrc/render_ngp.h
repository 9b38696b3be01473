// render_ngp.h -- pieces shared by the fused ngp renderer's kernels
// (render_ngp.hip: prep, hash-grid encode, fp32-MFMA field kernel;
//  field_f16x3.hip: split-fp16 MFMA field kernel).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "sdfr_common.h"

namespace sdfr {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kW = 256;          // NGPSIRENGenerator width
constexpr uint32_t kFeatIn = 32;      // 16 levels x 2
constexpr uint32_t kViewsIn = 272;    // 256 + 16 SH
constexpr uint32_t kFilm = 4;         // FiLM layers: pts 0,1,2 + views
constexpr uint32_t kTileRays = 16;    // rays per wave (MFMA N)

// ----------------------------------------------------------------------------
// shared ray / sample geometry
// ----------------------------------------------------------------------------
struct GeomArgs {
    uint32_t B, H, W, N, tiles_per_face, total_tiles, S_total;
    float half_res;
    const float *cam, *focal, *near_, *far_, *pix_x, *pix_y;
    SampleCfg sc;
    int static_viewdirs, z_normalize;
    float bound;
};

// tile-order sample id -> (face, ray-in-face, sample)
struct SampleId {
    uint32_t b, ray_local, s, n, tile;
    bool valid;
};

__device__ __forceinline__ SampleId decode_sid(const GeomArgs &g, uint32_t sid) {
    SampleId r;
    r.n = sid & 15u;
    const uint32_t rest = sid >> 4;
    r.s = rest % g.N;
    r.tile = rest / g.N;
    r.b = r.tile / g.tiles_per_face;
    r.ray_local = (r.tile % g.tiles_per_face) * kTileRays + r.n;
    r.valid = r.tile < g.total_tiles && r.ray_local < g.H * g.W;
    return r;
}

struct FieldArgs {
    GeomArgs g;
    const float *enc;              // [L=16][S_total][2]
    const f4 *packed;              // [67][1024]
    const float *film;             // [B][4][2][256]
    const float *bias[5];          // input, pts0..2, views
    const float *sigma_w, *sigma_b, *rgb_w, *rgb_b, *sigmoid_beta;
    const float *sigma_noise;      // [B,H,W,N] or null (no_sdf only)
    int force_background, with_sdf;
    float *rgb, *features, *sdf, *xyz, *mask;
};

constexpr uint32_t kCst = 9 * kW;              // LDS constants: bias[5], sigma_w, rgb_w[3]
constexpr int kWaves = 4;                       // 1 wave per SIMD, 512 VGPR+AGPR
constexpr int kThreads = kWaves * 64;

// sin via the hardware v_sin_f32, whose argument is in revolutions: x/(2pi)
// = k + f with k = rint(x c_hi) and f = fma(x, c_hi, -k) + x c_lo (c_hi + c_lo =
// 1/(2pi) to ~2^-50; x c_hi is exact inside the fma, so f carries one rounding,
// |f| <= 0.5).  4 VALU + 1 transcendental; accuracy is measured against float64
// by tests/test_gpu_encoders.py::test_sin_accuracy (|x| <= 200).
__device__ __forceinline__ float sin_hw(float x) {
    constexpr float c_hi = 0.15915493667125702f;    // fl(1/(2pi))
    constexpr float c_lo = 6.4206382432985265e-09f;  // 1/(2pi) - c_hi
    const float k = __builtin_rintf(x * c_hi);
    float f = __fmaf_rn(x, c_hi, -k);
    f = __fmaf_rn(x, c_lo, f);
    return __builtin_amdgcn_sinf(f);
}

// sin of an argument given in REVOLUTIONS (u = x / 2pi): the hardware v_sin_f32
// alone.  The split-fp16 field kernel folds 1/(2pi) into its FiLM vectors
// (xprep_kernel), so a FiLM activation sin(gamma x + beta) is ONE fma and this one
// instruction (the radian sin_hw costs 4 more VALU per element).  v_sin_f32 reduces
// its argument itself: measured on MI355X over |u| <= 2048 revolutions
// (scripts/probe_sin_raw.hip, 4 M points per range) its max error against float64
// sin(2 pi u) equals that of v_sin_f32(v_fract_f32(u)) (1.25e-7), while ~6 % of the
// results differ from that form in the last bit -- so the exact v_fract_f32 in
// front of it (one VALU per activation) is dropped.  FiLM arguments stay within
// |u| <= 32 (|gamma x + beta| <= 200 rad).  The rounding of the folded argument,
// |u| 2^-24 revolutions, equals the reference's own rounding of gamma x + beta in
// radians; accuracy: tests/test_gpu_encoders.py::test_device_sin_rev_accuracy.
__device__ __forceinline__ float sin_rev(float u) { return __builtin_amdgcn_sinf(u); }

// SH degree 4 coefficients 4g..4g+3 of a unit direction (shencoder.cu:50-68)
__device__ __forceinline__ f4 sh_quad(float x, float y, float z, uint32_t g) {
    const float xy = __fmul_rn(x, y), xz = __fmul_rn(x, z), yz = __fmul_rn(y, z);
    const float x2 = __fmul_rn(x, x), y2 = __fmul_rn(y, y), z2 = __fmul_rn(z, z);
    f4 q0, q1, q2, q3;
    q0.x = 0.28209479177387814f;
    q0.y = __fmul_rn(-0.48860251190291987f, y);
    q0.z = __fmul_rn(0.48860251190291987f, z);
    q0.w = __fmul_rn(-0.48860251190291987f, x);
    q1.x = __fmul_rn(1.0925484305920792f, xy);
    q1.y = __fmul_rn(-1.0925484305920792f, yz);
    q1.z = __fmaf_rn(0.94617469575755997f, z2, -0.31539156525251999f);
    q1.w = __fmul_rn(-1.0925484305920792f, xz);
    q2.x = __fmaf_rn(0.54627421529603959f, x2, -__fmul_rn(0.54627421529603959f, y2));
    q2.y = __fmul_rn(__fmul_rn(0.59004358992664352f, y), __fmaf_rn(-3.0f, x2, y2));
    q2.z = __fmul_rn(__fmul_rn(2.8906114426405538f, xy), z);
    q2.w = __fmul_rn(__fmul_rn(0.45704579946446572f, y), __fmaf_rn(-5.0f, z2, 1.0f));
    q3.x = __fmul_rn(__fmul_rn(0.3731763325901154f, z), __fmaf_rn(5.0f, z2, -3.0f));
    q3.y = __fmul_rn(__fmul_rn(0.45704579946446572f, x), __fmaf_rn(-5.0f, z2, 1.0f));
    q3.z = __fmul_rn(__fmul_rn(1.4453057213202769f, z), __fsub_rn(x2, y2));
    q3.w = __fmul_rn(__fmul_rn(0.59004358992664352f, x), __fmaf_rn(3.0f, y2, -x2));
    return g == 0 ? q0 : (g == 1 ? q1 : (g == 2 ? q2 : q3));
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// sum over the 4 lane groups holding the same ray (lanes n, n+16, n+32, n+48)
__device__ __forceinline__ float group_sum(float v) {
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    return v;
}

// Split-fp16 field path (field_f16x3.hip).  Its workspace region (`xws`,
// f16x3_ws_bytes(net): 0 = ngp, 1 = siren) holds the packed fp16 fragments, row
// scales and scaled biases.
size_t f16x3_ws_bytes(int net);
int field_variant();   // profiling ablation selected by sdfr_debug_set_field_variant
int launch_xprep_ngp(const sdfr_ngp_weights *w, const sdfr_ngp_render_args *a, char *xws,
                     float *film, hipStream_t st);
int launch_xfield_ngp(const sdfr_ngp_weights *w, const sdfr_ngp_render_args *a,
                      const GeomArgs &g, const float *enc, char *xws, const float *film,
                      hipStream_t st, float *part, const float2 *zd);
// sample-segment split of the f16x3 field kernel for small batches
constexpr uint32_t kFieldSplitMax = 4;   // sample segments per ray at most
uint32_t field_nseg(uint32_t B, uint32_t tiles_per_face, uint32_t N, int force_background,
                    uint32_t max_seg);
size_t field_part_bytes(uint32_t B, uint32_t tiles_per_face, uint32_t N);
void fill_geom_args(const sdfr_ngp_render_args *a, float bound, GeomArgs &g);
void record_event(void *ev, hipStream_t st);
// stream waits on a caller's hipEvent_t (NULL: nothing)
void wait_event(void *ev, hipStream_t st);

// LDS-DMA: buffer resource over [base, base + bytes) (range-checked: offsets past
// it read zeros) and one 64-lane x 16-B piece from (voff + soff) to the LDS byte
// address lds (wave-uniform base + 16 lane).  Inline asm, so the compiler neither
// drains vmcnt in front of every LDS read nor holds M0; completion is counted by
// the caller (s_waitcnt vmcnt) and published to the other waves by a barrier.
typedef int v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4i make_rsrc(const void *base, uint32_t bytes) {
    const uint64_t b = reinterpret_cast<uint64_t>(base);
    v4i r;
    r.x = (int)(uint32_t)b;
    r.y = (int)(uint32_t)(b >> 32);
    r.z = (int)bytes;
    r.w = 0x00020000;
    return r;
}

__device__ __forceinline__ void dma16(v4i rsrc, uint32_t voff, uint32_t soff, uint32_t lds) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(rsrc), "s"(lds), "s"(soff)
        : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)reinterpret_cast<uintptr_t>(p);
}

}  // namespace sdfr
