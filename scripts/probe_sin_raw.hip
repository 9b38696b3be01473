// Does v_sin_f32 need the v_fract_f32 in front of it?  For u over a range of
// revolutions, compare sin(fract(u)) with the raw hardware sin(u), bit for bit,
// and both against float64 sin(2 pi u).  Profiling aid (not a test):
//   hipcc --offload-arch=gfx950 -O3 scripts/probe_sin_raw.hip -o /tmp/probe_sin_raw
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

__global__ void k(const float *u, float *a, float *b, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    a[i] = __builtin_amdgcn_sinf(__builtin_amdgcn_fractf(u[i]));
    b[i] = __builtin_amdgcn_sinf(u[i]);
}

int main() {
    const int n = 1 << 22;
    const float spans[] = {1.0f, 8.0f, 64.0f, 256.0f, 512.0f, 4096.0f};
    std::vector<float> u(n), a(n), b(n);
    float *du, *da, *db;
    hipMalloc(&du, n * 4);
    hipMalloc(&da, n * 4);
    hipMalloc(&db, n * 4);
    unsigned s = 12345;
    for (float span : spans) {
        for (int i = 0; i < n; ++i) {
            s = s * 1664525u + 1013904223u;
            u[i] = ((s >> 8) * (1.0f / 16777216.0f) - 0.5f) * span;
        }
        hipMemcpy(du, u.data(), n * 4, hipMemcpyHostToDevice);
        k<<<(n + 255) / 256, 256>>>(du, da, db, n);
        hipMemcpy(a.data(), da, n * 4, hipMemcpyDeviceToHost);
        hipMemcpy(b.data(), db, n * 4, hipMemcpyDeviceToHost);
        long diff = 0;
        double ea = 0, eb = 0;
        for (int i = 0; i < n; ++i) {
            diff += a[i] != b[i];
            const double r = std::sin(2 * M_PI * (double)u[i]);
            ea = std::fmax(ea, std::fabs(a[i] - r));
            eb = std::fmax(eb, std::fabs(b[i] - r));
        }
        printf("span %7.0f: %ld / %d differ; max err fract+sin %.3e raw sin %.3e\n", span, diff, n,
               ea, eb);
    }
    return 0;
}
