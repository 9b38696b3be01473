/*
 * sdfr_oracle.c -- CPU ORACLE (test infrastructure only).
 *
 * Plain-C restatement of the reference SDFace-GAN hot-path arithmetic that
 * has to be reproduced bit-for-bit on the GPU (integer / index work and the
 * floating-point chain that feeds floorf()).  Only tests/, the smoke() check
 * in __graft_entry__.py and bench.py's cpu_baseline leg may load this
 * library.  Nothing in the product (sdface-gan_amd/) links or calls it.
 *
 * Reference files followed (paths relative to /root/reference):
 *   im2scene/sdf/models/gridencoder/src/gridencoder.cu
 *       fast_hash                 :50-63
 *       get_grid_index            :66-84
 *       kernel_grid (forward)     :87-245   (incl. OOB -> 0 :110-135, dy_dx :201-244)
 *       kernel_grid_backward      :248-340
 *       kernel_input_backward     :343-369
 *   im2scene/sdf/models/gridencoder/grid.py  offsets :117-128, bound map :149
 *   im2scene/sdf/models/shencoder/src/shencoder.cu
 *       kernel_sh degree<=4 values :50-68, dy_dx :130-200 (first 16 entries)
 *       kernel_sh_backward         :358-382
 *   im2scene/sdf/models/sdf_model.py
 *       get_rays                   :207-222
 *       render (viewdir norm)      :363-378
 *       render_rays sampling       :310-351
 *       volume_integration dists   :236-242
 *
 * Rounding conventions (pinned against the reference's own PyTorch CPU code
 * by tests/golden/make_golden.py; the CUDA kernels themselves cannot run in
 * this container and are "parity unpinned" against real nvcc output):
 *   - nvcc contracts `x*scale + 0.5f` and `acc += w*v` into fused multiply-add
 *     (default -fmad=true, no fast-math in gridencoder/backend.py:6-9); the
 *     oracle uses fmaf() at exactly those places.
 *   - PyTorch CPU elementwise ops round after every op (no contraction);
 *     torch.sum over a 3-wide last dim accumulates left to right;
 *     torch.norm over 3 values is sqrtf(fmaf(z,z,fmaf(y,y,x*x))).
 *   - per-level scale = exp2f(l*S)*H - 1 uses a correctly rounded exp2f
 *     (computed in double, rounded once).  CUDA's exp2f is documented at
 *     <=2 ulp; see DESIGN.md "parity pinning".
 */
#include <math.h>
#include <stdint.h>
#include <stddef.h>
#include <string.h>

#define ORC_OK 0
#define ORC_EINVAL -1

/* ------------------------------------------------------------------ */
/* per-level parameters (gridencoder.cu:137-139)                       */
/* ------------------------------------------------------------------ */
/* Sensitivity probe (tests only): exp2f's result moved by g_exp2_ulp[level]
 * ulps, standing in for a CUDA exp2f that is off by that much (<= 2 documented).
 * All zero by default: the correctly rounded value. */
static int32_t g_exp2_ulp[32];

void orc_set_exp2_ulp(const int32_t *off, uint32_t n) {
    for (uint32_t i = 0; i < 32; i++) g_exp2_ulp[i] = (off && i < n) ? off[i] : 0;
}

float orc_level_scale(uint32_t level, float S, uint32_t H) {
    float ls = (float)level * S;             /* level * S in fp32         */
    float e = (float)exp2((double)ls);       /* correctly rounded exp2f   */
    /* (an integer exponent is an exact power of two for any exp2f: not moved) */
    int32_t k = (level < 32 && ls != floorf(ls)) ? g_exp2_ulp[level] : 0;
    for (; k > 0; k--) e = nextafterf(e, INFINITY);
    for (; k < 0; k++) e = nextafterf(e, 0.0f);
    return e * (float)H - 1.0f;              /* *16 exact; one rounding   */
}

uint32_t orc_level_resolution(float scale) {
    return (uint32_t)ceilf(scale) + 1u;
}

/* fast_hash, gridencoder.cu:50-63 (uint32 wrap-around products). */
static uint32_t orc_fast_hash(const uint32_t *pg, uint32_t D) {
    static const uint32_t primes[7] = {1u, 2654435761u, 805459861u, 3674653429u,
                                       2097192037u, 1434869437u, 2165219737u};
    uint32_t r = 0;
    for (uint32_t i = 0; i < D; ++i) r ^= pg[i] * primes[i];
    return r;
}

/* get_grid_index, gridencoder.cu:66-84 */
uint32_t orc_grid_index(uint32_t gridtype, int align_corners, uint32_t ch,
                        uint32_t hashmap_size, uint32_t resolution,
                        const uint32_t *pg, uint32_t D, uint32_t C) {
    uint32_t stride = 1, index = 0;
    for (uint32_t d = 0; d < D && stride <= hashmap_size; d++) {
        index += pg[d] * stride;
        stride *= align_corners ? resolution : (resolution + 1);
    }
    if (gridtype == 0 && stride > hashmap_size) index = orc_fast_hash(pg, D);
    return (index % hashmap_size) * C + ch;
}

static float orc_smoothstep(float v) { return v * v * (3.0f - 2.0f * v); }
static float orc_smoothstep_d(float v) { return 6 * v * (1.0f - v); }

/* ------------------------------------------------------------------ */
/* kernel_grid, gridencoder.cu:87-245 (one sample, one level)          */
/* outputs: [L,B,C]; dy_dx: [B, L*D*C]                                 */
/* ------------------------------------------------------------------ */
static void orc_grid_one(const float *x, const float *grid, uint32_t hsize,
                         float scale, uint32_t res, uint32_t D, uint32_t C,
                         float *out, float *dydx, uint32_t gridtype,
                         int align_corners, uint32_t interp) {
    int oob = 0;
    for (uint32_t d = 0; d < D; d++)
        if (x[d] < 0 || x[d] > 1) oob = 1;
    if (oob) {
        for (uint32_t c = 0; c < C; c++) out[c] = 0;
        if (dydx)
            for (uint32_t i = 0; i < D * C; i++) dydx[i] = 0;
        return;
    }
    float pos[8], pos_d[8];
    uint32_t pg[8];
    for (uint32_t d = 0; d < D; d++) {
        pos[d] = fmaf(x[d], scale, align_corners ? 0.0f : 0.5f);
        pg[d] = (uint32_t)floorf(pos[d]);
        pos[d] -= (float)pg[d];
        if (interp == 1) {
            pos_d[d] = orc_smoothstep_d(pos[d]);
            pos[d] = orc_smoothstep(pos[d]);
        } else {
            pos_d[d] = 1.0f;
        }
    }
    float res_c[8] = {0};
    for (uint32_t idx = 0; idx < (1u << D); idx++) {
        float w = 1;
        uint32_t pl[8];
        for (uint32_t d = 0; d < D; d++) {
            if ((idx & (1u << d)) == 0) { w *= 1 - pos[d]; pl[d] = pg[d]; }
            else { w *= pos[d]; pl[d] = pg[d] + 1; }
        }
        uint32_t index = orc_grid_index(gridtype, align_corners, 0, hsize, res, pl, D, C);
        for (uint32_t c = 0; c < C; c++) res_c[c] = fmaf(w, grid[index + c], res_c[c]);
    }
    for (uint32_t c = 0; c < C; c++) out[c] = res_c[c];
    if (!dydx) return;
    for (uint32_t gd = 0; gd < D; gd++) {
        float rg[8] = {0};
        for (uint32_t idx = 0; idx < (1u << (D - 1)); idx++) {
            float w = scale;
            uint32_t pl[8];
            for (uint32_t nd = 0; nd < D - 1; nd++) {
                uint32_t d = (nd >= gd) ? (nd + 1) : nd;
                if ((idx & (1u << nd)) == 0) { w *= 1 - pos[d]; pl[d] = pg[d]; }
                else { w *= pos[d]; pl[d] = pg[d] + 1; }
            }
            pl[gd] = pg[gd];
            uint32_t il = orc_grid_index(gridtype, align_corners, 0, hsize, res, pl, D, C);
            pl[gd] = pg[gd] + 1;
            uint32_t ir = orc_grid_index(gridtype, align_corners, 0, hsize, res, pl, D, C);
            for (uint32_t c = 0; c < C; c++)
                rg[c] = fmaf(w * (grid[ir + c] - grid[il + c]), pos_d[gd], rg[c]);
        }
        for (uint32_t c = 0; c < C; c++) dydx[gd * C + c] = rg[c];
    }
}

static int orc_dims_ok(uint32_t D, uint32_t C) {
    if (D < 2 || D > 5) return 0;
    return C == 1 || C == 2 || C == 4 || C == 8;
}

int orc_grid_encode_forward(const float *inputs, const float *embeddings,
                            const int32_t *offsets, float *outputs, uint32_t B,
                            uint32_t D, uint32_t C, uint32_t L, float S,
                            uint32_t H, float *dy_dx, uint32_t gridtype,
                            int align_corners, uint32_t interp) {
    if (!orc_dims_ok(D, C)) return ORC_EINVAL;
    for (uint32_t l = 0; l < L; l++) {
        const float *grid = embeddings + (size_t)(uint32_t)offsets[l] * C;
        uint32_t hsize = (uint32_t)(offsets[l + 1] - offsets[l]);
        float scale = orc_level_scale(l, S, H);
        uint32_t res = orc_level_resolution(scale);
        for (uint32_t b = 0; b < B; b++) {
            float *dd = dy_dx ? dy_dx + (size_t)b * D * L * C + (size_t)l * D * C : NULL;
            orc_grid_one(inputs + (size_t)b * D, grid, hsize, scale, res, D, C,
                         outputs + ((size_t)l * B + b) * C, dd, gridtype,
                         align_corners, interp);
        }
    }
    return ORC_OK;
}

/* kernel_grid_backward + kernel_input_backward, gridencoder.cu:248-369.
 * grad: [L,B,C]; grad_embeddings must be zeroed by the caller (grid.py:75).
 * Sequential accumulation in (level, sample, corner) order. */
int orc_grid_encode_backward(const float *grad, const float *inputs,
                             const float *embeddings, const int32_t *offsets,
                             float *grad_embeddings, uint32_t B, uint32_t D,
                             uint32_t C, uint32_t L, float S, uint32_t H,
                             const float *dy_dx, float *grad_inputs,
                             uint32_t gridtype, int align_corners,
                             uint32_t interp) {
    (void)embeddings;
    if (!orc_dims_ok(D, C)) return ORC_EINVAL;
    for (uint32_t l = 0; l < L; l++) {
        float *gg = grad_embeddings + (size_t)(uint32_t)offsets[l] * C;
        uint32_t hsize = (uint32_t)(offsets[l + 1] - offsets[l]);
        float scale = orc_level_scale(l, S, H);
        uint32_t res = orc_level_resolution(scale);
        for (uint32_t b = 0; b < B; b++) {
            const float *x = inputs + (size_t)b * D;
            int oob = 0;
            for (uint32_t d = 0; d < D; d++)
                if (x[d] < 0 || x[d] > 1) oob = 1;
            if (oob) continue;
            float pos[8];
            uint32_t pg[8];
            for (uint32_t d = 0; d < D; d++) {
                pos[d] = fmaf(x[d], scale, align_corners ? 0.0f : 0.5f);
                pg[d] = (uint32_t)floorf(pos[d]);
                pos[d] -= (float)pg[d];
                if (interp == 1) pos[d] = orc_smoothstep(pos[d]);
            }
            const float *g = grad + ((size_t)l * B + b) * C;
            for (uint32_t idx = 0; idx < (1u << D); idx++) {
                float w = 1;
                uint32_t pl[8];
                for (uint32_t d = 0; d < D; d++) {
                    if ((idx & (1u << d)) == 0) { w *= 1 - pos[d]; pl[d] = pg[d]; }
                    else { w *= pos[d]; pl[d] = pg[d] + 1; }
                }
                uint32_t index = orc_grid_index(gridtype, align_corners, 0, hsize, res, pl, D, C);
                for (uint32_t c = 0; c < C; c++) gg[index + c] += w * g[c];
            }
        }
    }
    if (dy_dx && grad_inputs) {
        for (uint32_t b = 0; b < B; b++)
            for (uint32_t d = 0; d < D; d++) {
                float r = 0;
                for (uint32_t l = 0; l < L; l++)
                    for (uint32_t c = 0; c < C; c++)
                        r = fmaf(grad[((size_t)l * B + b) * C + c],
                                 dy_dx[(size_t)b * L * D * C + (size_t)l * D * C + d * C + c], r);
                grad_inputs[(size_t)b * D + d] = r;
            }
    }
    return ORC_OK;
}

/* ------------------------------------------------------------------ */
/* SH encoder, shencoder.cu:27-68 values, :130-200 dy_dx (degree<=4).  */
/* C is the degree; outputs [B, C*C]; dy_dx [B, D, C*C].              */
/* ------------------------------------------------------------------ */
static void orc_sh_one(const float *in, float *o, uint32_t C, float *dx,
                       float *dy, float *dz) {
    float x = in[0], y = in[1], z = in[2];
    float xy = x * y, xz = x * z, yz = y * z, x2 = x * x, y2 = y * y, z2 = z * z;
    o[0] = 0.28209479177387814f;
    if (C > 1) {
        o[1] = -0.48860251190291987f * y;
        o[2] = 0.48860251190291987f * z;
        o[3] = -0.48860251190291987f * x;
    }
    if (C > 2) {
        o[4] = 1.0925484305920792f * xy;
        o[5] = -1.0925484305920792f * yz;
        o[6] = fmaf(0.94617469575755997f, z2, -0.31539156525251999f);
        o[7] = -1.0925484305920792f * xz;
        o[8] = fmaf(0.54627421529603959f, x2, -(0.54627421529603959f * y2));
    }
    if (C > 3) {
        o[9] = (0.59004358992664352f * y) * fmaf(-3.0f, x2, y2);
        o[10] = (2.8906114426405538f * xy) * z;
        o[11] = (0.45704579946446572f * y) * fmaf(-5.0f, z2, 1.0f);
        o[12] = (0.3731763325901154f * z) * fmaf(5.0f, z2, -3.0f);
        o[13] = (0.45704579946446572f * x) * fmaf(-5.0f, z2, 1.0f);
        o[14] = (1.4453057213202769f * z) * (x2 - y2);
        o[15] = (0.59004358992664352f * x) * fmaf(3.0f, y2, -x2);
    }
    if (!dx) return;
    dx[0] = 0; dy[0] = 0; dz[0] = 0;
    if (C > 1) {
        dx[1] = 0.0f; dx[2] = 0.0f; dx[3] = -0.48860251190291992f;
        dy[1] = -0.48860251190291992f; dy[2] = 0.0f; dy[3] = 0.0f;
        dz[1] = 0.0f; dz[2] = 0.48860251190291992f; dz[3] = 0.0f;
    }
    if (C > 2) {
        dx[4] = 1.0925484305920792f * y; dx[5] = 0.0f; dx[6] = 0.0f;
        dx[7] = -1.0925484305920792f * z; dx[8] = 1.0925484305920792f * x;
        dy[4] = 1.0925484305920792f * x; dy[5] = -1.0925484305920792f * z;
        dy[6] = 0.0f; dy[7] = 0.0f; dy[8] = -1.0925484305920792f * y;
        dz[4] = 0.0f; dz[5] = -1.0925484305920792f * y;
        dz[6] = 1.8923493915151202f * z; dz[7] = -1.0925484305920792f * x;
        dz[8] = 0.0f;
    }
    if (C > 3) {
        dx[9] = -3.5402615395598609f * xy;
        dx[10] = 2.8906114426405538f * yz;
        dx[11] = 0.0f;
        dx[12] = 0.0f;
        dx[13] = fmaf(-2.2852289973223288f, z2, 0.45704579946446572f);
        dx[14] = 2.8906114426405538f * xz;
        dx[15] = fmaf(-1.7701307697799304f, x2, 1.7701307697799304f * y2);
        dy[9] = fmaf(-1.7701307697799304f, x2, 1.7701307697799304f * y2);
        dy[10] = 2.8906114426405538f * xz;
        dy[11] = fmaf(-2.2852289973223288f, z2, 0.45704579946446572f);
        dy[12] = 0.0f;
        dy[13] = 0.0f;
        dy[14] = -2.8906114426405538f * yz;
        dy[15] = 3.5402615395598609f * xy;
        dz[9] = 0.0f;
        dz[10] = 2.8906114426405538f * xy;
        dz[11] = -4.5704579946446566f * yz;
        dz[12] = fmaf(5.597644988851731f, z2, -1.1195289977703462f);
        dz[13] = -4.5704579946446566f * xz;
        dz[14] = fmaf(1.4453057213202769f, x2, -(1.4453057213202769f * y2));
        dz[15] = 0.0f;
    }
}

/* Bands 4..7 (degrees 5..8, shencoder.cu:74-123 and the matching dy_dx terms): the
 * Legendre-recurrence form that csrc/sh_gen.py generates for the HIP kernel (the same
 * header, so this C restatement and the kernel agree bit for bit); pinned against the
 * reference's own degree-8 formulas evaluated in fp32 (tests/golden/sh_deg8.npz) and
 * against scipy's spherical harmonics (tests/test_oracle.py). */
#include "../../sdface-gan_amd/csrc/sh_bands.h"

int orc_sh_encode_forward(const float *inputs, float *outputs, uint32_t B,
                          uint32_t D, uint32_t C, float *dy_dx) {
    if (D != 3 || C < 1 || C > 8) return ORC_EINVAL;
    uint32_t C2 = C * C;
    for (uint32_t b = 0; b < B; b++) {
        float o[64], dxs[3][64];
        float *dx = dy_dx ? dxs[0] : NULL;
        const float *in = inputs + (size_t)b * D;
        orc_sh_one(in, o, C < 4 ? C : 4, dx, dx ? dxs[1] : NULL, dx ? dxs[2] : NULL);
        if (C > 4) sdfr_sh_bands_4_7(in[0], in[1], in[2], C, o, dx, dx ? dxs[1] : NULL,
                                     dx ? dxs[2] : NULL);
        for (uint32_t i = 0; i < C2; i++) outputs[(size_t)b * C2 + i] = o[i];
        if (dy_dx)
            for (uint32_t d = 0; d < 3; d++)
                for (uint32_t i = 0; i < C2; i++)
                    dy_dx[(size_t)b * D * C2 + d * C2 + i] = dxs[d][i];
    }
    return ORC_OK;
}

/* kernel_sh_backward, shencoder.cu:358-382 (grad_inputs pre-zeroed). */
int orc_sh_encode_backward(const float *grad, const float *inputs, uint32_t B,
                           uint32_t D, uint32_t C, const float *dy_dx,
                           float *grad_inputs) {
    (void)inputs;
    if (D != 3 || C < 1 || C > 8) return ORC_EINVAL;
    uint32_t C2 = C * C;
    for (uint32_t b = 0; b < B; b++)
        for (uint32_t d = 0; d < D; d++) {
            float acc = grad_inputs[(size_t)b * D + d];
            for (uint32_t ch = 0; ch < C2; ch++)
                acc = fmaf(grad[(size_t)b * C2 + ch], dy_dx[(size_t)b * D * C2 + d * C2 + ch], acc);
            grad_inputs[(size_t)b * D + d] = acc;
        }
    return ORC_OK;
}

/* ------------------------------------------------------------------ */
/* Ray generation + sampling, sdf_model.py:207-222, 310-351, 363-378.  */
/* The bit-exact float chain that ends in the grid encoder's input     */
/* (x+bound)/(2*bound) (grid.py:149).                                  */
/*                                                                    */
/* cam [B,3,4] (c2w = [R^T | T]), focal/near/far [B], pix_x [W] (the  */
/* renderer's i buffer row), pix_y [H] (j buffer column), t_vals [N]. */
/* t_rand: NULL (perturb off), [B,H,W] (offset sampling) or           */
/* [B,H,W,N] (stratified, t_rand_per_sample=1).                       */
/* Outputs (any may be NULL): rays_d [B,H,W,3], viewdirs [B,H,W,3],   */
/* dnorm [B,H,W], z [B,H,W,N], pts [B,H,W,N,3], u [B,H,W,N,3].        */
/* ------------------------------------------------------------------ */
static float orc_norm3(const float *v) {
    return sqrtf(fmaf(v[2], v[2], fmaf(v[1], v[1], v[0] * v[0])));
}

int orc_sample_rays(const float *cam, const float *focal, const float *near,
                    const float *far, const float *pix_x, const float *pix_y,
                    const float *t_vals, const float *t_rand,
                    int t_rand_per_sample, int offset_sampling,
                    int static_viewdirs, int z_normalize, float half_res,
                    float bound, uint32_t B, uint32_t H, uint32_t W,
                    uint32_t N, float *rays_d, float *viewdirs, float *dnorm,
                    float *z_out, float *pts_out, float *u_out) {
    if (N > 4096) return ORC_EINVAL;
    float zb[4096];
    for (uint32_t b = 0; b < B; b++) {
        const float *c = cam + (size_t)b * 12;
        float f = focal[b], nr = near[b], fr = far[b];
        for (uint32_t r = 0; r < H; r++)
            for (uint32_t q = 0; q < W; q++) {
                size_t ray = ((size_t)b * H + r) * W + q;
                /* get_rays :208-210 */
                float dir[3];
                dir[0] = (pix_x[q] - half_res) / f;
                dir[1] = -((pix_y[r] - half_res) / f);
                dir[2] = -1.0f;
                /* :213 sum over last dim, left to right */
                float d[3], o[3];
                for (int k = 0; k < 3; k++) {
                    float s = dir[0] * c[k * 4 + 0];
                    s = s + dir[1] * c[k * 4 + 1];
                    s = s + dir[2] * c[k * 4 + 2];
                    d[k] = s;
                    o[k] = c[k * 4 + 3];
                }
                /* render :367 */
                const float *vsrc = static_viewdirs ? dir : d;
                float vn = orc_norm3(vsrc);
                if (rays_d) for (int k = 0; k < 3; k++) rays_d[ray * 3 + k] = d[k];
                if (viewdirs) for (int k = 0; k < 3; k++) viewdirs[ray * 3 + k] = vsrc[k] / vn;
                if (dnorm) dnorm[ray] = orc_norm3(d);
                /* render_rays :324 */
                for (uint32_t s = 0; s < N; s++) {
                    float a = nr * (1.0f - t_vals[s]);
                    float bb = fr * t_vals[s];
                    zb[s] = a + bb;
                }
                if (t_rand) {
                    if (offset_sampling) { /* :329-331,340 */
                        float tr = t_rand[ray];
                        float zt[4096];
                        for (uint32_t s = 0; s < N; s++) {
                            float up = (s + 1 < N) ? zb[s + 1] : fr;
                            zt[s] = zb[s] + (up - zb[s]) * tr;
                        }
                        memcpy(zb, zt, N * sizeof(float));
                    } else { /* :333-340 */
                        float zt[4096];
                        for (uint32_t s = 0; s < N; s++) {
                            float lo = (s == 0) ? zb[0] : 0.5f * (zb[s] + zb[s - 1]);
                            float up = (s + 1 < N) ? 0.5f * (zb[s + 1] + zb[s]) : zb[N - 1];
                            float tr = t_rand_per_sample ? t_rand[ray * N + s] : t_rand[ray];
                            zt[s] = lo + (up - lo) * tr;
                        }
                        memcpy(zb, zt, N * sizeof(float));
                    }
                }
                float span = fr - nr;
                for (uint32_t s = 0; s < N; s++) {
                    size_t si = ray * N + s;
                    if (z_out) z_out[si] = zb[s];
                    for (int k = 0; k < 3; k++) {
                        float p = o[k] + d[k] * zb[s];           /* :343 */
                        if (pts_out) pts_out[si * 3 + k] = p;
                        float np_ = z_normalize ? (p * 2.0f) / span : p; /* :349 */
                        if (u_out) u_out[si * 3 + k] = (np_ + bound) / (2.0f * bound); /* grid.py:149 */
                    }
                }
            }
    }
    return ORC_OK;
}
