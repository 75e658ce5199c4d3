// LDS random-gather microbenchmark (not part of the product): cycles per
// wave-instruction per CU of data-dependent table lookups of the widths and
// layouts the sketch kernel can use.  Every workgroup fills a table in LDS and
// every lane then issues reads at random entries (register-resident random
// indices xor-ed with the loop counter: a bank permutation, so the conflict
// structure per instruction is that of uniform random indices).  LDS cycles
// per CU are derived from s_memtime / s_memrealtime (shader clock) and wall time.
//   hipcc --offload-arch=gfx950 -O3 -o tools/lds_microbench tools/lds_microbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int WG = 256;
constexpr int ITERS = 4096;
constexpr int NIDX = 8;   // independent reads in flight per iteration

// MODE: 0 b32 random over ENT entries; 1 b64 random; 2 b128 random;
// 3 b128 with REP lane replicas (entry e, replica c at unit e*REP + c, c = lane % REP)
// 4 b64 with REP lane replicas; 5 b32 with REP lane replicas; 6 b32 broadcast-free lane-linear (conflict-free reference)
template <int MODE, int ENT, int REP>
__global__ __launch_bounds__(WG) void k_lds(uint32_t seed, uint32_t *out, unsigned long long *clk) {
    extern __shared__ __align__(16) uint32_t T[];
    constexpr int UNITW = (MODE == 0 || MODE == 5 || MODE == 6) ? 1 : (MODE == 1 || MODE == 4) ? 2 : 4;
    constexpr int NU = ENT * ((MODE >= 3 && MODE <= 5) ? REP : 1);
    for (int i = threadIdx.x; i < NU * UNITW; i += WG) T[i] = i * 2654435761u;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    uint32_t r[NIDX];
    uint32_t x = seed ^ (blockIdx.x * 7919u + threadIdx.x * 104729u);
#pragma unroll
    for (int k = 0; k < NIDX; k++) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; r[k] = x % ENT; }
    uint32_t acc = 0;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; it++) {
        const uint32_t m = (uint32_t)it & (ENT - 1);
#pragma unroll
        for (int k = 0; k < NIDX; k++) {
            const uint32_t e = r[k] ^ m;
            if constexpr (MODE == 0) acc += T[e];
            else if constexpr (MODE == 1) { const uint2 v = ((const uint2 *)T)[e]; acc += v.x ^ v.y; }
            else if constexpr (MODE == 2) { const uint4 v = ((const uint4 *)T)[e]; acc += v.x ^ v.y ^ v.z ^ v.w; }
            else if constexpr (MODE == 3) { const uint4 v = ((const uint4 *)T)[e * REP + (lane % REP)]; acc += v.x ^ v.y ^ v.z ^ v.w; }
            else if constexpr (MODE == 4) { const uint2 v = ((const uint2 *)T)[e * REP + (lane % REP)]; acc += v.x ^ v.y; }
            else if constexpr (MODE == 5) acc += T[e * REP + (lane % REP)];
            else acc += T[(lane + k) & 63];
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
    if (acc == 0x12345678u) out[0] = acc;    // keep the reads
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = w1 - w0; }
}

template <int MODE, int ENT, int REP>
static int run(const char *name, int wgs_per_cu, uint32_t *d_out, unsigned long long *d_clk) {
    constexpr int UNITW = (MODE == 0 || MODE == 5 || MODE == 6) ? 1 : (MODE == 1 || MODE == 4) ? 2 : 4;
    constexpr int NU = ENT * ((MODE >= 3 && MODE <= 5) ? REP : 1);
    const size_t lds = (size_t)NU * UNITW * 4;
    CK(hipFuncSetAttribute((const void *)k_lds<MODE, ENT, REP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int nblk = 256 * wgs_per_cu * 4;        // 4 waves of workgroups per CU slot
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    hipLaunchKernelGGL((k_lds<MODE, ENT, REP>), dim3(nblk), dim3(WG), lds, 0, 1u, d_out, d_clk);   // warm
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((k_lds<MODE, ENT, REP>), dim3(nblk), dim3(WG), lds, 0, 2u, d_out, d_clk);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    unsigned long long clk[2];
    CK(hipMemcpy(clk, d_clk, 16, hipMemcpyDeviceToHost));
    const double ghz = clk[1] ? (double)clk[0] / clk[1] * 0.1 : 0.0;
    const double wave_inst_per_cu = (double)nblk / 256 * (WG / 64) * ITERS * NIDX;
    const double cyc = ms * 1e-3 * ghz * 1e9 / wave_inst_per_cu;
    printf("  {\"case\": \"%s\", \"lds_bytes\": %zu, \"ms\": %.3f, \"clock_ghz\": %.3f, \"cu_cycles_per_wave_inst\": %.3f, "
           "\"bytes_per_lane\": %d}%s\n", name, lds, ms, ghz, cyc, UNITW * 4, MODE == 6 && REP == 1 ? "" : ",");
    return 0;
}

int main() {
    uint32_t *d_out;
    unsigned long long *d_clk;
    CK(hipMalloc(&d_out, 4));
    CK(hipMalloc(&d_clk, 16));
    printf("{\"note\": \"random LDS gathers, 256-lane workgroups, 8 independent reads in flight per lane\", \"results\": [\n");
    run<0, 256, 1>("b32 random, 256 entries", 8, d_out, d_clk);
    run<1, 256, 1>("b64 random, 256 entries", 8, d_out, d_clk);
    run<1, 1024, 1>("b64 random, 1024 entries", 8, d_out, d_clk);
    run<2, 256, 1>("b128 random, 256 entries", 8, d_out, d_clk);
    run<3, 256, 2>("b128, 2 lane replicas", 8, d_out, d_clk);
    run<3, 256, 4>("b128, 4 lane replicas", 4, d_out, d_clk);
    run<3, 256, 8>("b128, 8 lane replicas", 2, d_out, d_clk);
    run<3, 256, 16>("b128, 16 lane replicas", 1, d_out, d_clk);
    run<4, 256, 4>("b64, 4 lane replicas", 8, d_out, d_clk);
    run<4, 256, 8>("b64, 8 lane replicas", 4, d_out, d_clk);
    run<4, 256, 16>("b64, 16 lane replicas", 2, d_out, d_clk);
    run<4, 256, 32>("b64, 32 lane replicas", 1, d_out, d_clk);
    run<5, 256, 16>("b32, 16 lane replicas", 4, d_out, d_clk);
    run<5, 256, 32>("b32, 32 lane replicas", 2, d_out, d_clk);
    run<6, 64, 1>("b32 conflict-free (lane-linear)", 8, d_out, d_clk);
    printf("]}\n");
    return 0;
}
