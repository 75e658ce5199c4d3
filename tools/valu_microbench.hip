// valu_microbench.hip -- measured issue cost of every instruction class the
// sketch kernel's hot loop (k_sketch_hash21<64,2>, drep_amd/csrc/sketch.hip)
// is made of, on gfx950 at 8 waves per SIMD.  Not part of the product: its
// output (profiles/r06_valu_microbench.json) prices the hot loop's static
// instruction mix in tools/sketch_priced.py.
//
// Each thread runs CHAINS independent dependency chains of one instruction
// (or of one short sequence, priced per instruction of the sequence); the grid
// is 8 workgroups of 4 waves per CU, i.e. 8 waves on every SIMD.  The price is
// wall time per wave-instruction per SIMD (HIP events around the launch), and
// its cycles at the clock the chip held in the launch (s_memtime over
// s_memrealtime's 100 MHz, per workgroup, median).  LDS classes read random
// entries of a per-workgroup table laid out as the sketch kernel's tables are.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CHAINS 8
#define REPS 8      // CHAINS*REPS units per loop iteration: loop overhead < 5 %
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

struct Op { const char *name; int instrs; };   // instructions per unit
static const Op ops[] = {
    {"v_xor_b32_e32", 1},                     // 0
    {"v_mul_lo_u32", 1},                      // 1
    {"v_mul_hi_u32", 1},                      // 2
    {"v_mad_u64_u32", 1},                     // 3
    {"v_lshlrev_b64", 1},                     // 4
    {"v_lshl_add_u64", 1},                    // 5
    {"v_alignbit_b32", 1},                    // 6
    {"v_add3_u32", 1},                        // 7
    {"v_cndmask_b32_e32 (vcc)", 1},           // 8
    {"v_lshrrev_b64", 1},                     // 9
    {"v_cmp_lt_u64_e32 (vcc)", 1},            // 10
    {"v_mov_b32_e32", 1},                     // 11
    {"v_perm_b32", 1},                        // 12
    {"v_bitop3_b32", 1},                      // 13
    {"v_add_u32_e32", 1},                     // 14
    {"v_lshrrev_b32_e32", 1},                 // 15
    {"v_lshlrev_b32_e32", 1},                 // 16
    {"v_lshlrev_b32_sdwa (sgpr shift, byte select)", 1},  // 17
    {"v_and_b32_e32 (literal)", 1},           // 18
    {"v_min_u32_e32", 1},                     // 19
    {"v_cmp_ge_u32_e32 (vcc)", 1},            // 20
    {"v_bfi_b32", 1},                         // 21
    {"v_bfrev_b32_e32", 1},                   // 22
    {"v_not_b32_e32", 1},                     // 23
    {"v_or_b32_e32", 1},                      // 24
    {"v_mov_b64_e32", 1},                     // 25
    {"v_cndmask_b32_e64 (sgpr mask)", 1},     // 26
    // the canonical select as the kernel emits it: a 64-bit compare into VCC and two selects reading it
    {"select: v_cmp_lt_u64_e32 vcc + 2 v_cndmask_b32_e32", 3},              // 27
    // the same select through an SGPR-pair mask (e64 encodings)
    {"select: v_cmp_lt_u64_e64 s[2] + 2 v_cndmask_b32_e64", 3},             // 28
    // the same select through the borrow of a 64-bit subtract and two bitop3
    {"select: v_sub_co/v_subb_co/v_subbrev_co + 2 v_bitop3", 5},            // 29
    {"ds_read_b128, random 16-B entry of 256 (4 KiB)", 1},                  // 30
    {"ds_read_b64, random 8-B entry of 256 (2 KiB)", 1},                    // 31
    {"ds_read_b64, random 8-B entry of 1024 (8 KiB)", 1},                   // 32
    // 64 v_xor_b32 with 5 random-index LDS reads among them (2 b128 + 3 b64: the
    // kernel's 63 VALU : 5 LDS per k-mer); priced per VALU instruction
    {"mixed: 64 v_xor_b32 + 2 ds_read_b128 + 3 ds_read_b64 (per v_xor)", 1},  // 33
    // 64 v_xor_b32 with 4 s_mov_b32 among them (the loop's SALU constants); per v_xor
    {"mixed: 64 v_xor_b32 + 4 s_mov_b32 (per v_xor)", 1},                   // 34
    // 33's loop with the five reads replaced by empty statements defining the same
    // registers: 33 - 35 is what the five reads add to a VALU-bound stream
    {"control for 33: the same loop without the LDS reads (per v_xor)", 1},  // 35
};
constexpr int NOPS = sizeof(ops) / sizeof(ops[0]);

struct Tabs { u32x4 e[256]; u32x2 b[256]; uint64_t t[1024]; };
// LDS byte offset of a __shared__ object (the ds_read address operand)
__device__ __forceinline__ uint32_t lds_off(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

template <int OP>
__global__ __launch_bounds__(256) void mb(uint32_t *out, int iters, uint32_t c, unsigned long long *clk) {
    __shared__ Tabs tb;
    for (uint32_t i = threadIdx.x; i < 256; i += 256) {
        tb.e[i] = u32x4{i * 0x9E3779B9u, i * 0x85EBCA6Bu, i * 0xC2B2AE35u, i};
        tb.b[i] = u32x2{i * 0x27D4EB2Fu, i * 0x165667B1u};
    }
    for (uint32_t i = threadIdx.x; i < 1024; i += 256) tb.t[i] = (uint64_t)i * 0x9E3779B97F4A7C15ull;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t a[CHAINS];
    uint64_t b[CHAINS];
    u32x4 q[CHAINS];
    u32x2 w[CHAINS];
    uint32_t tmp = 0, ad[CHAINS];
    const uint64_t smask = 0x5555555555555555ull ^ c;
    for (int j = 0; j < CHAINS; j++) {
        a[j] = threadIdx.x * 7 + j;
        b[j] = ((uint64_t)a[j] << 32) | (a[j] * 3);
        ad[j] = (a[j] * 0x9E3779B9u) >> 24;
        q[j] = u32x4{0, 0, 0, 0};
        w[j] = u32x2{0, 0};
    }
    const uint32_t sh16 = 4, sh8 = 3;
    // LDS byte addresses: entry index (random per lane) << entry size + table base
    constexpr uint32_t kmask = OP == 32 ? 0x3ffu : 0xffu;
    constexpr uint32_t ksh = OP == 30 || OP == 33 || OP == 35 ? 4u : 3u;
    const uint32_t kbase = OP == 30 || OP == 33 || OP == 35 ? lds_off(&tb.e[0]) : OP == 31 ? lds_off(&tb.b[0]) : lds_off(&tb.t[0]);
    uint32_t ad2[CHAINS];
    for (int j = 0; j < CHAINS; j++) {
        ad[j] = kbase + ((ad[j] & kmask) << ksh);
        ad2[j] = lds_off(&tb.b[0]) + (((ad[j] >> 3) & 0xffu) << 3);
    }
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int jj = 0; jj < CHAINS * REPS; jj++) {
            const int j = jj % CHAINS;
            if constexpr (OP == 0) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 2) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 4) asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(b[j]));
            if constexpr (OP == 5) asm volatile("v_lshl_add_u64 %0, %0, 2, %0" : "+v"(b[j]));
            if constexpr (OP == 6) asm volatile("v_alignbit_b32 %0, %0, %1, 8" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 7) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 8) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 9) asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(b[j]));
            if constexpr (OP == 11) asm volatile("v_mov_b32 %0, %1" : "=v"(a[j]) : "v"(a[(j + 1) % CHAINS]));
            if constexpr (OP == 12) asm volatile("v_perm_b32 %0, %1, %1, %0" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 13) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 14) asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 15) asm volatile("v_lshrrev_b32_e32 %0, 1, %0" : "+v"(a[j]));
            if constexpr (OP == 16) asm volatile("v_lshlrev_b32_e32 %0, 18, %0" : "+v"(a[j]));
            if constexpr (OP == 17)
                asm volatile("v_lshlrev_b32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2"
                             : "+v"(a[j]) : "s"(sh16));
            if constexpr (OP == 18) asm volatile("v_and_b32_e32 %0, 0x1ff8, %0" : "+v"(a[j]));
            if constexpr (OP == 19) asm volatile("v_min_u32_e32 %0, %1, %0" : "+v"(a[j]) : "v"(a[(j + 1) % CHAINS]));
            if constexpr (OP == 21) asm volatile("v_bfi_b32 %0, %1, %0, %1" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 22) asm volatile("v_bfrev_b32_e32 %0, %0" : "+v"(a[j]));
            if constexpr (OP == 23) asm volatile("v_not_b32_e32 %0, %0" : "+v"(a[j]));
            if constexpr (OP == 24) asm volatile("v_or_b32_e32 %0, %1, %0" : "+v"(a[j]) : "v"(c));
            if constexpr (OP == 25) asm volatile("v_mov_b64_e32 %0, %1" : "=v"(b[j]) : "v"(b[(j + 1) % CHAINS]));
            if constexpr (OP == 26) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[j]) : "v"(c), "s"(smask));
            // (LDS classes: each chain's address is formed once per iteration, after the
            // reads land, so the loop body is the reads alone)
            // (sequences writing VCC or an SGPR pair, and the LDS reads: one asm
            // statement per 8 units, one per chain -- between separate statements the
            // compiler places an s_nop the kernel's own code does not have)
            if constexpr (OP == 3) if (j == 0) asm volatile("v_mad_u64_u32 %0, vcc, %8, %8, %0\n\tv_mad_u64_u32 %1, vcc, %8, %8, %1\n\tv_mad_u64_u32 %2, vcc, %8, %8, %2\n\tv_mad_u64_u32 %3, vcc, %8, %8, %3\n\tv_mad_u64_u32 %4, vcc, %8, %8, %4\n\tv_mad_u64_u32 %5, vcc, %8, %8, %5\n\tv_mad_u64_u32 %6, vcc, %8, %8, %6\n\tv_mad_u64_u32 %7, vcc, %8, %8, %7" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]), "+v"(b[6]), "+v"(b[7]) : "v"(c) : "vcc");
            if constexpr (OP == 10) if (j == 0) asm volatile("v_cmp_gt_u64 vcc, %0, %1\n\tv_cmp_gt_u64 vcc, %1, %2\n\tv_cmp_gt_u64 vcc, %2, %3\n\tv_cmp_gt_u64 vcc, %3, %4\n\tv_cmp_gt_u64 vcc, %4, %5\n\tv_cmp_gt_u64 vcc, %5, %6\n\tv_cmp_gt_u64 vcc, %6, %7\n\tv_cmp_gt_u64 vcc, %7, %0" :: "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]) : "vcc");
            if constexpr (OP == 20) if (j == 0) asm volatile("v_cmp_ge_u32_e32 vcc, %8, %0\n\tv_cmp_ge_u32_e32 vcc, %8, %1\n\tv_cmp_ge_u32_e32 vcc, %8, %2\n\tv_cmp_ge_u32_e32 vcc, %8, %3\n\tv_cmp_ge_u32_e32 vcc, %8, %4\n\tv_cmp_ge_u32_e32 vcc, %8, %5\n\tv_cmp_ge_u32_e32 vcc, %8, %6\n\tv_cmp_ge_u32_e32 vcc, %8, %7" :: "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "s"(c) : "vcc");
            if constexpr (OP == 27) if (j == 0) asm volatile("v_cmp_lt_u64_e32 vcc, %8, %9\n\tv_cndmask_b32_e32 %0, %1, %0, vcc\n\tv_cndmask_b32_e32 %2, %3, %2, vcc\n\tv_cmp_lt_u64_e32 vcc, %9, %10\n\tv_cndmask_b32_e32 %1, %2, %1, vcc\n\tv_cndmask_b32_e32 %3, %4, %3, vcc\n\tv_cmp_lt_u64_e32 vcc, %10, %11\n\tv_cndmask_b32_e32 %2, %3, %2, vcc\n\tv_cndmask_b32_e32 %4, %5, %4, vcc\n\tv_cmp_lt_u64_e32 vcc, %11, %12\n\tv_cndmask_b32_e32 %3, %4, %3, vcc\n\tv_cndmask_b32_e32 %5, %6, %5, vcc\n\tv_cmp_lt_u64_e32 vcc, %12, %13\n\tv_cndmask_b32_e32 %4, %5, %4, vcc\n\tv_cndmask_b32_e32 %6, %7, %6, vcc\n\tv_cmp_lt_u64_e32 vcc, %13, %14\n\tv_cndmask_b32_e32 %5, %6, %5, vcc\n\tv_cndmask_b32_e32 %7, %0, %7, vcc\n\tv_cmp_lt_u64_e32 vcc, %14, %15\n\tv_cndmask_b32_e32 %6, %7, %6, vcc\n\tv_cndmask_b32_e32 %0, %1, %0, vcc\n\tv_cmp_lt_u64_e32 vcc, %15, %8\n\tv_cndmask_b32_e32 %7, %0, %7, vcc\n\tv_cndmask_b32_e32 %1, %2, %1, vcc" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]), "+v"(b[6]), "+v"(b[7]) :: "vcc");
            if constexpr (OP == 28) if (j == 0) { uint64_t m; asm volatile("v_cmp_lt_u64_e64 %16, %8, %9\n\tv_cndmask_b32_e64 %0, %1, %0, %16\n\tv_cndmask_b32_e64 %2, %3, %2, %16\n\tv_cmp_lt_u64_e64 %16, %9, %10\n\tv_cndmask_b32_e64 %1, %2, %1, %16\n\tv_cndmask_b32_e64 %3, %4, %3, %16\n\tv_cmp_lt_u64_e64 %16, %10, %11\n\tv_cndmask_b32_e64 %2, %3, %2, %16\n\tv_cndmask_b32_e64 %4, %5, %4, %16\n\tv_cmp_lt_u64_e64 %16, %11, %12\n\tv_cndmask_b32_e64 %3, %4, %3, %16\n\tv_cndmask_b32_e64 %5, %6, %5, %16\n\tv_cmp_lt_u64_e64 %16, %12, %13\n\tv_cndmask_b32_e64 %4, %5, %4, %16\n\tv_cndmask_b32_e64 %6, %7, %6, %16\n\tv_cmp_lt_u64_e64 %16, %13, %14\n\tv_cndmask_b32_e64 %5, %6, %5, %16\n\tv_cndmask_b32_e64 %7, %0, %7, %16\n\tv_cmp_lt_u64_e64 %16, %14, %15\n\tv_cndmask_b32_e64 %6, %7, %6, %16\n\tv_cndmask_b32_e64 %0, %1, %0, %16\n\tv_cmp_lt_u64_e64 %16, %15, %8\n\tv_cndmask_b32_e64 %7, %0, %7, %16\n\tv_cndmask_b32_e64 %1, %2, %1, %16" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]), "+v"(b[6]), "+v"(b[7]), "=&s"(m)); }
            if constexpr (OP == 29) if (j == 0) asm volatile("v_sub_co_u32 %8, vcc, %0, %1\n\tv_subb_co_u32 %8, vcc, %2, %3, vcc\n\tv_subbrev_co_u32 %8, vcc, 0, 0, vcc\n\tv_bitop3_b32 %0, %1, %0, %8 bitop3:0xca\n\tv_bitop3_b32 %2, %3, %2, %8 bitop3:0xca\n\tv_sub_co_u32 %8, vcc, %1, %2\n\tv_subb_co_u32 %8, vcc, %3, %4, vcc\n\tv_subbrev_co_u32 %8, vcc, 0, 0, vcc\n\tv_bitop3_b32 %1, %2, %1, %8 bitop3:0xca\n\tv_bitop3_b32 %3, %4, %3, %8 bitop3:0xca\n\tv_sub_co_u32 %8, vcc, %2, %3\n\tv_subb_co_u32 %8, vcc, %4, %5, vcc\n\tv_subbrev_co_u32 %8, vcc, 0, 0, vcc\n\tv_bitop3_b32 %2, %3, %2, %8 bitop3:0xca\n\tv_bitop3_b32 %4, %5, %4, %8 bitop3:0xca\n\tv_sub_co_u32 %8, vcc, %3, %4\n\tv_subb_co_u32 %8, vcc, %5, %6, vcc\n\tv_subbrev_co_u32 %8, vcc, 0, 0, vcc\n\tv_bitop3_b32 %3, %4, %3, %8 bitop3:0xca\n\tv_bitop3_b32 %5, %6, %5, %8 bitop3:0xca\n\tv_sub_co_u32 %8, vcc, %4, %5\n\tv_subb_co_u32 %8, vcc, %6, %7, vcc\n\tv_subbrev_co_u32 %8, vcc, 0, 0, vcc\n\tv_bitop3_b32 %4, %5, %4, %8 bitop3:0xca\n\tv_bitop3_b32 %6, %7, %6, %8 bitop3:0xca\n\tv_sub_co_u32 %8, vcc, %5, %6\n\tv_subb_co_u32 %8, vcc, %7, %0, vcc\n\tv_subbrev_co_u32 %8, vcc, 0, 0, vcc\n\tv_bitop3_b32 %5, %6, %5, %8 bitop3:0xca\n\tv_bitop3_b32 %7, %0, %7, %8 bitop3:0xca\n\tv_sub_co_u32 %8, vcc, %6, %7\n\tv_subb_co_u32 %8, vcc, %0, %1, vcc\n\tv_subbrev_co_u32 %8, vcc, 0, 0, vcc\n\tv_bitop3_b32 %6, %7, %6, %8 bitop3:0xca\n\tv_bitop3_b32 %0, %1, %0, %8 bitop3:0xca\n\tv_sub_co_u32 %8, vcc, %7, %0\n\tv_subb_co_u32 %8, vcc, %1, %2, vcc\n\tv_subbrev_co_u32 %8, vcc, 0, 0, vcc\n\tv_bitop3_b32 %7, %0, %7, %8 bitop3:0xca\n\tv_bitop3_b32 %1, %2, %1, %8 bitop3:0xca" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), "=&v"(tmp) :: "vcc");
            if constexpr (OP == 30) if (j == 0) asm volatile("ds_read_b128 %0, %8\n\tds_read_b128 %1, %9\n\tds_read_b128 %2, %10\n\tds_read_b128 %3, %11\n\tds_read_b128 %4, %12\n\tds_read_b128 %5, %13\n\tds_read_b128 %6, %14\n\tds_read_b128 %7, %15" : "=&v"(q[0]), "=&v"(q[1]), "=&v"(q[2]), "=&v"(q[3]), "=&v"(q[4]), "=&v"(q[5]), "=&v"(q[6]), "=&v"(q[7]) : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3]), "v"(ad[4]), "v"(ad[5]), "v"(ad[6]), "v"(ad[7]));
            if constexpr (OP == 31 || OP == 32) if (j == 0) asm volatile("ds_read_b64 %0, %8\n\tds_read_b64 %1, %9\n\tds_read_b64 %2, %10\n\tds_read_b64 %3, %11\n\tds_read_b64 %4, %12\n\tds_read_b64 %5, %13\n\tds_read_b64 %6, %14\n\tds_read_b64 %7, %15" : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]), "=&v"(w[4]), "=&v"(w[5]), "=&v"(w[6]), "=&v"(w[7]) : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3]), "v"(ad[4]), "v"(ad[5]), "v"(ad[6]), "v"(ad[7]));
            if constexpr (OP == 33 || OP == 35) {
                asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a[j]) : "v"(c));
                if (jj == 5 || jj == 31) {
                    if constexpr (OP == 33) asm volatile("ds_read_b128 %0, %1" : "=&v"(q[j]) : "v"(ad[j]));
                    else asm volatile("" : "=&v"(q[j]) : "v"(ad[j]));
                }
                if (jj == 13 || jj == 40 || jj == 57) {
                    if constexpr (OP == 33) asm volatile("ds_read_b64 %0, %1" : "=&v"(w[j]) : "v"(ad2[j]));
                    else asm volatile("" : "=&v"(w[j]) : "v"(ad2[j]));
                }
            }
            if constexpr (OP == 34) {
                asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a[j]) : "v"(c));
                if ((jj & 15) == 7) {
                    uint32_t sv;
                    asm volatile("s_mov_b32 %0, 0x2745937f" : "=s"(sv));
                    asm volatile("" :: "s"(sv));
                }
            }
        }
        if constexpr ((OP >= 30 && OP <= 33) || OP == 35) {
            // the reads land before the next iteration's addresses are formed
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int j = 0; j < CHAINS; j++) {
                const uint32_t r = q[j].x ^ q[j].w ^ w[j].y ^ (ad[j] >> ksh);
                ad[j] = kbase + ((r & kmask) << ksh);
                ad2[j] = lds_off(&tb.b[0]) + (((r >> 8) & 0xffu) << 3);
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
    for (int j = 0; j < CHAINS; j++) s += a[j] + (uint32_t)b[j] + (uint32_t)(b[j] >> 32) + ad[j] + ad2[j] + tmp;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

static unsigned long long *g_clk;
template <int OP>
static void run(uint32_t *d, int blocks, int iters, hipEvent_t e0, hipEvent_t e1, float *ms, double *ghz) {
    hipLaunchKernelGGL(mb<OP>, dim3(blocks), dim3(256), 0, 0, d, iters, 12345u, g_clk);   // warm (clock up)
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(mb<OP>, dim3(blocks), dim3(256), 0, 0, d, iters, 12345u, g_clk);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(ms, e0, e1);
    std::vector<unsigned long long> h(2 * blocks);
    (void)hipMemcpy(h.data(), g_clk, 2 * blocks * 8, hipMemcpyDeviceToHost);
    std::vector<double> f;
    for (int k = 0; k < blocks; k++)
        if (h[2 * k + 1]) f.push_back((double)h[2 * k] / (double)h[2 * k + 1] * 0.1);   // GHz (realtime: 100 MHz)
    std::sort(f.begin(), f.end());
    *ghz = f.empty() ? 0.0 : f[f.size() / 2];
}

template <int OP>
static void run_all(uint32_t *d, int blocks, int iters, hipEvent_t e0, hipEvent_t e1, float *ms, double *ghz) {
    run<OP>(d, blocks, iters, e0, e1, ms + OP, ghz + OP);
    if constexpr (OP + 1 < NOPS) run_all<OP + 1>(d, blocks, iters, e0, e1, ms, ghz);
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const int blocks = cus * 8;          // 8 blocks x 4 waves = 32 waves / CU = 8 per SIMD
    const int iters = 4000;
    uint32_t *d;
    (void)hipMalloc(&d, (size_t)blocks * 256 * 4);
    (void)hipMalloc(&g_clk, (size_t)blocks * 16);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float ms[NOPS];
    double ghz[NOPS];
    run_all<0>(d, blocks, iters, e0, e1, ms, ghz);
    printf("{\"tool\": \"tools/valu_microbench.hip\", \"cus\": %d, \"simds\": %d, \"waves_per_simd\": 8, "
           "\"chains_per_thread\": %d, \"units_per_chain_iteration\": %d, \"iters\": %d, \"results\": [\n",
           cus, 4 * cus, CHAINS, REPS, iters);
    for (int i = 0; i < NOPS; i++) {
        // wave-instructions per SIMD: 8 waves x iters x CHAINS*REPS units x instrs per unit
        const double winst = 8.0 * iters * CHAINS * REPS * ops[i].instrs;
        const double ns = ms[i] * 1e6 / winst;
        printf("  {\"inst\": \"%s\", \"instrs_per_unit\": %d, \"ms\": %.4f, \"ns_per_wave_inst_per_simd\": %.4f, "
               "\"clock_ghz\": %.3f, \"cycles_per_wave_inst_per_simd\": %.3f}%s\n",
               ops[i].name, ops[i].instrs, ms[i], ns, ghz[i], ns * ghz[i], i + 1 < NOPS ? "," : "");
    }
    printf("]}\n");
    return 0;
}
