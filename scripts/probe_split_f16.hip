// Accuracy probe: fp32 GEMM tile (16 x K) . (K x 16) on gfx950 computed
//   (a) with v_mfma_f32_16x16x4_f32 (exact fp32 fma chain, the current field kernel)
//   (b) with three v_mfma_f32_16x16x32_f16 per k-step on a hi/lo fp16 split of both
//       operands (A_hi B_hi + A_hi B_lo + A_lo B_hi, one fp32 accumulator)
// against a float64 host reference.  Also checks the 16x16x32 f16 operand maps with
// integer data.  Build: hipcc --offload-arch=gfx950 -O3 -o probe scripts/probe_split_f16.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

constexpr int K = 256;

__device__ inline void split(float x, _Float16 &hi, _Float16 &lo, int mode) {
    if (mode == 0) {  // round-to-nearest hi
        hi = (_Float16)x;
        lo = (_Float16)(x - (float)hi);
    } else {          // truncate mantissa to 11 bits (exact fp16 for normal range)
        const float h = __uint_as_float(__float_as_uint(x) & 0xFFFFE000u);
        hi = (_Float16)h;
        lo = (_Float16)(x - h);
    }
}

// A [16][K] row-major, B [K][16] row-major, out [16][16]
__global__ void gemm_f32(const float *A, const float *B, float *out) {
    const int lane = threadIdx.x;
    f4 acc = {0, 0, 0, 0};
    for (int k0 = 0; k0 < K; k0 += 4) {
        const float a = A[(lane & 15) * K + k0 + (lane >> 4)];
        const float b = B[(k0 + (lane >> 4)) * 16 + (lane & 15)];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
    }
    for (int r = 0; r < 4; ++r) out[((lane >> 4) * 4 + r) * 16 + (lane & 15)] = acc[r];
}

__global__ void gemm_split(const float *A, const float *B, float *out, int mode, int terms) {
    const int lane = threadIdx.x;
    f4 acc = {0, 0, 0, 0};
    for (int k0 = 0; k0 < K; k0 += 32) {
        h8 ah, al, bh, bl;
        for (int j = 0; j < 8; ++j) {
            const int k = k0 + 8 * (lane >> 4) + j;
            _Float16 h, l;
            split(A[(lane & 15) * K + k], h, l, mode);
            ah[j] = h; al[j] = l;
            split(B[k * 16 + (lane & 15)], h, l, mode);
            bh[j] = h; bl[j] = l;
        }
        if (terms >= 3) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc, 0, 0, 0);
        if (terms >= 2) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc, 0, 0, 0);
    }
    for (int r = 0; r < 4; ++r) out[((lane >> 4) * 4 + r) * 16 + (lane & 15)] = acc[r];
}

static void run(const char *name, float wamp, float tiny_frac, std::mt19937 &rng) {
    std::uniform_real_distribution<float> U(-1.f, 1.f);
    std::vector<float> A(16 * K), B(K * 16);
    for (auto &v : A) v = U(rng) * wamp * (U(rng) > 1 - 2 * tiny_frac ? 1e-4f : 1.f);
    for (auto &v : B) v = std::sin(30.f * U(rng) + 3.f);
    std::vector<double> ref(256);
    double mag = 0;
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            double s = 0, m = 0;
            for (int k = 0; k < K; ++k) {
                s += (double)A[i * K + k] * B[k * 16 + j];
                m += std::fabs((double)A[i * K + k] * B[k * 16 + j]);
            }
            ref[i * 16 + j] = s;
            mag = std::max(mag, m);
        }
    float *dA, *dB, *dO;
    hipMalloc(&dA, A.size() * 4);
    hipMalloc(&dB, B.size() * 4);
    hipMalloc(&dO, 256 * 4);
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    std::vector<float> o(256);
    auto report = [&](const char *tag) {
        hipMemcpy(o.data(), dO, 256 * 4, hipMemcpyDeviceToHost);
        double mx = 0, rms = 0;
        for (int i = 0; i < 256; ++i) {
            const double e = std::fabs(o[i] - ref[i]);
            mx = std::max(mx, e);
            rms += e * e;
        }
        printf("  %-28s max|err| %.3e  rms %.3e  (sum|ab| %.2f)\n", tag, mx, std::sqrt(rms / 256), mag);
    };
    printf("%s\n", name);
    gemm_f32<<<1, 64>>>(dA, dB, dO);
    report("fp32 mfma 16x16x4");
    for (int mode = 0; mode < 2; ++mode)
        for (int terms = 1; terms <= 3; ++terms) {
            gemm_split<<<1, 64>>>(dA, dB, dO, mode, terms);
            char tag[64];
            snprintf(tag, sizeof tag, "f16 split %s, %d term%s", mode ? "trunc" : "rn", terms,
                     terms > 1 ? "s" : "");
            report(tag);
        }
    hipFree(dA);
    hipFree(dB);
    hipFree(dO);
}

int main() {
    std::mt19937 rng(1234);
    run("SIREN hidden layer weights (|w| <= sqrt(6/256)/25)", std::sqrt(6.f / 256) / 25, 0, rng);
    run("unit weights (|w| <= 1)", 1.0f, 0, rng);
    run("weights with 10% tiny (1e-4x) entries", 0.1f, 0.1f, rng);
    run("small weights (|w| <= 1e-3)", 1e-3f, 0, rng);
    return 0;
}
