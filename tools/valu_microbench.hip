// valu_microbench.hip -- measured issue cost (cycles per wave64 instruction,
// per SIMD) of the integer VALU instructions the sketch kernel is made of, on
// gfx950.  Used to build the VALU roofline in DESIGN.md; not part of the
// product.  Each thread runs 8 independent dependency chains of one
// instruction; the grid fills every SIMD with 8 waves.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CHAINS 8
#define REPS 8      // CHAINS*REPS instructions per loop iteration: loop overhead < 5 %
template <int OP>
__global__ __launch_bounds__(256) void mb(uint32_t *out, int iters, uint32_t c, unsigned long long *cyc) {
    unsigned long long t0;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0) :: "memory");
    uint32_t a[CHAINS];
    uint64_t b[CHAINS];
    uint32_t tmp;
    const uint64_t smask = 0x5555555555555555ull ^ c;
    for (int j = 0; j < CHAINS; j++) { a[j] = threadIdx.x * 7 + j; b[j] = ((uint64_t)a[j] << 32) | (a[j] * 3); }
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int jj = 0; jj < CHAINS * REPS; jj++) {
            const int j = jj % CHAINS;
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
            if constexpr (OP == 16) asm volatile("v_xor_b32_e64 %0, %1, %0" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 17) asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 18) asm volatile("v_add_u32_e64 %0, %1, %0" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 19) asm volatile("v_xor_b32_e32 %0, %1, %0\n\tv_xor_b32_e64 %0, %1, %0" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 20) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 21) asm volatile("v_add_f32_e32 %0, %1, %0" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 22) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(b[j]) : "v"(b[(j + 1) % CHAINS]));
            // the mask in an SGPR pair instead of VCC
            if constexpr (OP == 23) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[j]) : "v"(c), "s"(smask));
            // the canonical-k-mer select as the sketch kernel emits it: a 64-bit
            // compare into VCC and two selects reading it (3 instructions)
            if constexpr (OP == 24)
                asm volatile("v_cmp_lt_u64_e32 vcc, %0, %1\n\tv_cndmask_b32_e32 %2, %3, %2, vcc\n\tv_cndmask_b32_e32 %4, %5, %4, vcc"
                             : "+v"(b[j]), "+v"(b[(j + 1) % CHAINS]), "+v"(a[j]), "+v"(a[(j + 1) % CHAINS]),
                               "+v"(a[(j + 2) % CHAINS]), "+v"(a[(j + 3) % CHAINS]) :: "vcc");
            // the same select through the borrow of a 64-bit subtract and two
            // bitop3 (5 instructions, the mask in a VGPR)
            if constexpr (OP == 25)
                asm volatile("v_sub_co_u32 %4, vcc, %0, %1\n\tv_subb_co_u32 %4, vcc, %2, %3, vcc\n\t"
                             "v_subbrev_co_u32 %4, vcc, 0, 0, vcc\n\t"
                             "v_bitop3_b32 %0, %1, %0, %4 bitop3:0xca\n\tv_bitop3_b32 %2, %3, %2, %4 bitop3:0xca"
                             : "+v"(a[j]), "+v"(a[(j + 1) % CHAINS]), "+v"(a[(j + 2) % CHAINS]), "+v"(a[(j + 3) % CHAINS]),
                               "=&v"(tmp) :: "vcc");
        }
    }
    uint32_t s = 0;
    for (int j = 0; j < CHAINS; j++) s += a[j] + (uint32_t)b[j] + (uint32_t)(b[j] >> 32);
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    unsigned long long t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1) :: "memory");
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

static const char *names[] = {"v_xor_b32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32", "v_lshlrev_b64",
                              "v_lshl_add_u64", "v_alignbit_b32", "v_add3_u32", "v_cndmask_b32", "v_lshrrev_b64",
                              "v_cmp_gt_u64", "v_mov_b32", "v_perm_b32", "v_mul_u32_u24", "v_mad_u32_u24",
                              "v_bitop3_b32", "v_xor_b32_e64", "v_add_u32_e32", "v_add_u32_e64", "xor_e32+xor_e64 (2 instr)",
                              "v_fma_f32", "v_add_f32", "v_pk_fma_f32", "v_cndmask_b32_e64 (sgpr mask)",
                              "v_cmp_lt_u64 + 2 v_cndmask (3 instr)", "sub/subb/subbrev + 2 bitop3 (5 instr)"};

static unsigned long long *g_cyc;
static double g_med_cycles;
template <int OP>
static float run(uint32_t *d, int blocks, int iters, hipEvent_t e0, hipEvent_t e1) {
    hipLaunchKernelGGL(mb<OP>, dim3(blocks), dim3(256), 0, 0, d, 4, 12345u, g_cyc);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(mb<OP>, dim3(blocks), dim3(256), 0, 0, d, iters, 12345u, g_cyc);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h(blocks);
    (void)hipMemcpy(h.data(), g_cyc, blocks * 8, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    g_med_cycles = (double)h[blocks / 2];
    return ms;
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const int blocks = cus * 8;          // 8 blocks x 4 waves = 32 waves / CU = 8 per SIMD
    const int iters = 2500;
    uint32_t *d;
    (void)hipMalloc(&d, (size_t)blocks * 256 * 4);
    (void)hipMalloc(&g_cyc, (size_t)blocks * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float ms[26];
    double cy[26];
#define RUN(i) ms[i] = run<i>(d, blocks, iters, e0, e1); cy[i] = g_med_cycles;
    RUN(0) RUN(1) RUN(2) RUN(3) RUN(4) RUN(5) RUN(6) RUN(7)
    RUN(8) RUN(9) RUN(10) RUN(11) RUN(12) RUN(13) RUN(14) RUN(15)
    RUN(16) RUN(17) RUN(18) RUN(19) RUN(20) RUN(21) RUN(22) RUN(23) RUN(24) RUN(25)
    // wave-instructions per SIMD = waves per SIMD (8) * iters * CHAINS
    const double winst = 8.0 * iters * CHAINS * REPS;
    printf("{\"cus\": %d, \"clock_mhz\": %d, \"results\": [\n", cus, p.clockRate / 1000);
    for (int i = 0; i < 26; i++) {
        const double ns_per = ms[i] * 1e6 / winst;
        // a block's 4 waves sit on 4 SIMDs; 8 blocks per CU -> 8 waves per SIMD run together
        const double cyc_per = cy[i] / (8.0 * iters * CHAINS * REPS);
        printf("  {\"inst\": \"%s\", \"ms\": %.3f, \"ns_per_wave_inst_per_simd\": %.4f, \"cycles_per_wave_inst_per_simd\": %.3f, \"rel_to_xor\": %.2f}%s\n",
               names[i], ms[i], ns_per, cyc_per, ms[i] / ms[0], i < 25 ? "," : "");
    }
    printf("]}\n");
    return 0;
}
