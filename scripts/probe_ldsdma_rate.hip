// Probe: per-CU rate of the weight streams the MFMA kernels run on.  Every CU runs one
// 512-thread workgroup (8 waves, as conv_h_kernel) that only moves bytes:
//   mode 0  buffer_load_dwordx4 ... lds (1 KiB per wave-instruction, the conv / field
//           kernels' LDS-DMA), DEPTH pieces in flight per wave
//   mode 1  global_load_dwordx4 into registers (compiler-issued; not run by main)
//   mode 2  global_store_dwordx4 (1 KiB per wave-instruction, the conv epilogues' stores)
// from / to a buffer of SRC bytes (1 MiB: L2-resident, as a conv weight slice; 256 MiB:
// MALL / HBM).  Prints bytes per shader clock per CU (s_memtime ticks) and the chip rate.
// Profiling aid (both MFMA kernels stream ~13-15 B/clk/CU of weights).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/probe_ldsdma scripts/probe_ldsdma_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4i make_rsrc(const void *base, uint32_t bytes) {
    const uint64_t b = reinterpret_cast<uint64_t>(base);
    v4i r;
    r.x = (int)(uint32_t)b;
    r.y = (int)(uint32_t)(b >> 32);
    r.z = (int)bytes;
    r.w = 0x00020000;
    return r;
}

template <int MODE, int DEPTH>
__global__ void __launch_bounds__(512, 1) rate(const float *src, float *dst, uint32_t src_bytes,
                                               int iters, long long *ticks) {
    __shared__ f4 ring[8][16][64];                 // 8 waves x 16 pieces x 1 KiB
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const v4i rs = make_rsrc(src, src_bytes);
    const uint32_t mask = src_bytes / 1024u - 1u;  // pieces in the buffer (power of two)
    uint32_t piece = (blockIdx.x * 8u + wave) * 37u;
    f4 sink = {0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        piece = (piece + 1u) & mask;
        const uint32_t voff = piece * 1024u + lane * 16u;
        if constexpr (MODE == 0) {
            const uint32_t lds = (uint32_t)reinterpret_cast<uintptr_t>(&ring[wave][it & 15][0]);
            uint32_t keep;
            asm volatile(
                "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(voff), "s"(rs), "s"(lds)
                : "memory");
        } else if constexpr (MODE == 1) {
            // compiler-issued loads (it places the waits): a load issued from inline asm
            // leaves its destination registers free for the compiler to reuse while the
            // load is in flight -- a corrupted address and a memory fault
            f4 v = *reinterpret_cast<const f4 *>(reinterpret_cast<const char *>(src) + voff);
            sink += v;
        } else {
            f4 v = {(float)it, 1.f, 2.f, 3.f};
            *reinterpret_cast<f4 *>(reinterpret_cast<char *>(dst) + voff) = v;
        }
        __builtin_amdgcn_s_waitcnt((DEPTH & 0xF) | ((DEPTH >> 4) << 14) | 0x70 | 0xF00);
    }
    __builtin_amdgcn_s_waitcnt(0x70 | 0xF00);     // vmcnt(0)
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) ticks[blockIdx.x * 8 + wave] = t1 - t0;
    if (MODE == 1 && sink[0] == 1.2345e-33f) dst[tid] = sink[1];
}

template <int MODE, int DEPTH>
static void run(const char *name, const float *src, float *dst, uint32_t src_bytes, int ncu,
                long long *ticks) {
    const int iters = 4096;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int w = 0; w < 2; ++w) rate<MODE, DEPTH><<<ncu, 512>>>(src, dst, src_bytes, iters, ticks);
    hipEventRecord(e0);
    rate<MODE, DEPTH><<<ncu, 512>>>(src, dst, src_bytes, iters, ticks);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> t(ncu * 8);
    hipMemcpy(t.data(), ticks, t.size() * sizeof(long long), hipMemcpyDeviceToHost);
    std::sort(t.begin(), t.end());
    const double med = (double)t[t.size() / 2];
    const double bytes_cu = 8.0 * iters * 1024.0;
    const double total = bytes_cu * ncu;
    printf("%-34s src %6.1f MiB depth %2d: %6.2f B/clk/CU (median wave %.0f ticks), "
           "%6.2f TB/s chip, clock %.2f GHz\n",
           name, src_bytes / 1048576.0, DEPTH, bytes_cu / med, med, total / (ms * 1e-3) / 1e12,
           med / (ms * 1e-3) / 1e9);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int ncu = p.multiProcessorCount;
    printf("%s, %d CUs\n", p.gcnArchName, ncu);
    const uint32_t big = 256u << 20, small = 1u << 20;
    float *src, *dst;
    long long *ticks;
    hipMalloc(&src, big);
    hipMalloc(&dst, big);
    hipMalloc(&ticks, ncu * 8 * sizeof(long long));
    hipMemset(src, 0, big);
    hipMemset(dst, 0, big);
    for (uint32_t sz : {small, big}) {
        run<0, 2>("LDS-DMA buffer_load_dwordx4 lds", src, dst, sz, ncu, ticks);
        run<0, 4>("LDS-DMA buffer_load_dwordx4 lds", src, dst, sz, ncu, ticks);
        run<0, 8>("LDS-DMA buffer_load_dwordx4 lds", src, dst, sz, ncu, ticks);
        run<2, 4>("global_store_dwordx4", src, dst, sz, ncu, ticks);
        run<2, 8>("global_store_dwordx4", src, dst, sz, ncu, ticks);
    }
    hipError_t e = hipDeviceSynchronize();
    printf("status %s\n", hipGetErrorString(e));
    return e == hipSuccess ? 0 : 1;
}
