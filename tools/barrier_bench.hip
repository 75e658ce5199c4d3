// Grid-barrier latency on MI355X (development measurement, not the product):
// a cooperative launch of G workgroups runs K barrier rounds (agent-scope
// arrival counter + generation flag); every spin is bounded by a wall-clock
// timeout so a missing workgroup ends the kernel instead of hanging it.
// hipcc --offload-arch=gfx950 -O3 -o tools/barrier_bench tools/barrier_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ uint64_t wall() { return __builtin_amdgcn_s_memrealtime(); }   // 100 MHz

__global__ void k_barriers(uint32_t *count, uint32_t *gen, uint32_t rounds, uint32_t *timeout_flag) {
    __shared__ int abort_;
    for (uint32_t r = 0; r < rounds; r++) {
        __syncthreads();
        if (threadIdx.x == 0) {
            abort_ = 0;
            const uint32_t g = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t t = __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            if (t == gridDim.x - 1) {
                __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                const uint64_t t0 = wall();
                while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
                    __builtin_amdgcn_s_sleep(1);
                    if (wall() - t0 > 50000000ull) { atomicExch(timeout_flag, 1u); abort_ = 1; break; }   // 0.5 s
                }
            }
        }
        __syncthreads();
        if (abort_) return;
    }
}

int main(int argc, char **argv) {
    const uint32_t rounds = argc > 1 ? atoi(argv[1]) : 10000;
    uint32_t *count, *gen, *to;
    hipMalloc(&count, 4); hipMalloc(&gen, 4); hipMalloc(&to, 4);
    for (uint32_t G : {8u, 32u, 64u, 128u, 256u}) {
        hipMemset(count, 0, 4); hipMemset(gen, 0, 4); hipMemset(to, 0, 4);
        void *args[] = {&count, &gen, (void *)&rounds, &to};
        hipEvent_t a, b;
        hipEventCreate(&a); hipEventCreate(&b);
        hipEventRecord(a);
        hipError_t e = hipLaunchCooperativeKernel((const void *)k_barriers, dim3(G), dim3(256), args, 0, 0);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        uint32_t tflag = 0;
        hipMemcpy(&tflag, to, 4, hipMemcpyDeviceToHost);
        printf("{\"G\": %u, \"rounds\": %u, \"launch\": \"%s\", \"timeout\": %u, \"us_per_barrier\": %.3f}\n", G, rounds,
               hipGetErrorString(e), tflag, ms * 1e3 / rounds);
        if (e != hipSuccess || tflag) return 1;
    }
    return 0;
}
