// valu_microbench.hip -- measured issue cost (cycles per wave64 instruction,
// per SIMD) of the integer VALU instructions the sketch kernel is made of, on
// gfx950.  Used to build the VALU roofline in DESIGN.md; not part of the
// product.  Each thread runs 8 independent dependency chains of one
// instruction; the grid fills every SIMD with 8 waves.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHAINS 8
template <int OP>
__global__ __launch_bounds__(256) void mb(uint32_t *out, int iters, uint32_t c) {
    uint32_t a[CHAINS];
    uint64_t b[CHAINS];
    for (int j = 0; j < CHAINS; j++) { a[j] = threadIdx.x * 7 + j; b[j] = ((uint64_t)a[j] << 32) | (a[j] * 3); }
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int j = 0; j < CHAINS; j++) {
            if constexpr (OP == 0) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 2) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 3) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(b[j]) : "v"(c), "v"(c) : "vcc");
            if constexpr (OP == 4) asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(b[j]));
            if constexpr (OP == 5) asm volatile("v_lshl_add_u64 %0, %0, 2, %0" : "+v"(b[j]));
            if constexpr (OP == 6) asm volatile("v_alignbit_b32 %0, %0, %1, 8" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 7) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 8) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 9) asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(b[j]));
            if constexpr (OP == 10) asm volatile("v_cmp_gt_u64 vcc, %0, %1" :: "v"(b[j]), "v"(b[(j + 1) % CHAINS]) : "vcc");
            if constexpr (OP == 11) asm volatile("v_mov_b32 %0, %1" : "=v"(a[j]) : "v"(a[(j + 1) % CHAINS]));
            if constexpr (OP == 12) asm volatile("v_perm_b32 %0, %1, %1, %0" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 13) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 14) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 15) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(a[j]) : "v"(c));
        }
    }
    uint32_t s = 0;
    for (int j = 0; j < CHAINS; j++) s += a[j] + (uint32_t)b[j] + (uint32_t)(b[j] >> 32);
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static const char *names[] = {"v_xor_b32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32", "v_lshlrev_b64",
                              "v_lshl_add_u64", "v_alignbit_b32", "v_add3_u32", "v_cndmask_b32", "v_lshrrev_b64",
                              "v_cmp_gt_u64", "v_mov_b32", "v_perm_b32", "v_mul_u32_u24", "v_mad_u32_u24",
                              "v_bitop3_b32"};

template <int OP>
static float run(uint32_t *d, int blocks, int iters, hipEvent_t e0, hipEvent_t e1) {
    hipLaunchKernelGGL(mb<OP>, dim3(blocks), dim3(256), 0, 0, d, 4, 12345u);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(mb<OP>, dim3(blocks), dim3(256), 0, 0, d, iters, 12345u);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const int blocks = cus * 8;          // 8 blocks x 4 waves = 32 waves / CU = 8 per SIMD
    const int iters = 20000;
    uint32_t *d;
    (void)hipMalloc(&d, (size_t)blocks * 256 * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float ms[16];
    ms[0] = run<0>(d, blocks, iters, e0, e1);   ms[1] = run<1>(d, blocks, iters, e0, e1);
    ms[2] = run<2>(d, blocks, iters, e0, e1);   ms[3] = run<3>(d, blocks, iters, e0, e1);
    ms[4] = run<4>(d, blocks, iters, e0, e1);   ms[5] = run<5>(d, blocks, iters, e0, e1);
    ms[6] = run<6>(d, blocks, iters, e0, e1);   ms[7] = run<7>(d, blocks, iters, e0, e1);
    ms[8] = run<8>(d, blocks, iters, e0, e1);   ms[9] = run<9>(d, blocks, iters, e0, e1);
    ms[10] = run<10>(d, blocks, iters, e0, e1); ms[11] = run<11>(d, blocks, iters, e0, e1);
    ms[12] = run<12>(d, blocks, iters, e0, e1); ms[13] = run<13>(d, blocks, iters, e0, e1);
    ms[14] = run<14>(d, blocks, iters, e0, e1); ms[15] = run<15>(d, blocks, iters, e0, e1);
    // wave-instructions per SIMD = waves per SIMD (8) * iters * CHAINS
    const double winst = 8.0 * iters * CHAINS;
    printf("{\"cus\": %d, \"clock_mhz\": %d, \"results\": [\n", cus, p.clockRate / 1000);
    for (int i = 0; i < 16; i++) {
        const double ns_per = ms[i] * 1e6 / winst;
        printf("  {\"inst\": \"%s\", \"ms\": %.3f, \"ns_per_wave_inst_per_simd\": %.4f, \"rel_to_xor\": %.2f}%s\n",
               names[i], ms[i], ns_per, ms[i] / ms[0], i < 15 ? "," : "");
    }
    printf("]}\n");
    return 0;
}
