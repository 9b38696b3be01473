// Probe: back-to-back issue rate of v_mfma_f32_16x16x16_f16 vs v_mfma_f32_16x16x32_f16
// on one SIMD (one wave per SIMD, 4 independent accumulators, random operands), in
// s_memtime ticks per MFMA.  Profiling aid (decides whether the field kernel's
// half-empty SH k-step would gain from the K = 16 instruction).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int K32>
__global__ void __launch_bounds__(256) probe(const float *in, float *out, long long *ticks, int iters) {
    const int l = threadIdx.x;
    h8 a8, b8;
    for (int i = 0; i < 8; ++i) {
        a8[i] = (_Float16)in[(l * 8 + i) & 1023];
        b8[i] = (_Float16)in[(l * 8 + i + 7) & 1023];
    }
    h4 a4 = {a8[0], a8[1], a8[2], a8[3]}, b4 = {b8[0], b8[1], b8[2], b8[3]};
    f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if constexpr (K32) {
            c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, c3, 0, 0, 0);
        } else {
            c0 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c3, 0, 0, 0);
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 256 + l] = (c0 + c1 + c2 + c3)[l & 3];
    if (l == 0) ticks[blockIdx.x] = t1 - t0;
}

int main() {
    const int iters = 4096, blocks = 256;
    float *in, *out;
    long long *tk;
    hipMalloc(&in, 1024 * 4);
    hipMalloc(&out, blocks * 256 * 4);
    hipMalloc(&tk, blocks * 8);
    float h[1024];
    for (int i = 0; i < 1024; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 997.0f - 0.5f;
    hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    for (int rep = 0; rep < 2; ++rep) {
        for (int k32 = 0; k32 < 2; ++k32) {
            if (k32) probe<1><<<blocks, 256>>>(in, out, tk, iters);
            else probe<0><<<blocks, 256>>>(in, out, tk, iters);
            hipDeviceSynchronize();
            long long t[blocks];
            hipMemcpy(t, tk, sizeof(t), hipMemcpyDeviceToHost);
            double s = 0;
            for (int b = 0; b < blocks; ++b) s += (double)t[b];
            printf("%s: %.2f ticks per MFMA (mean over %d workgroups)\n",
                   k32 ? "16x16x32_f16" : "16x16x16_f16", s / blocks / (4.0 * iters), blocks);
        }
    }
    return 0;
}
