// Does a kernel's instruction stream cost per launch (cold instruction cache
// after each dispatch)?  K dependent v_fma_f32 per launch, 2000 launches
// captured in a graph; time per launch against K.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)
template <int K>
__global__ void k_chain(float *out, float a, float b) {
    float x = threadIdx.x;
#pragma unroll
    for (int i = 0; i < K; i++) x = __builtin_fmaf(x, a, b + (float)i);   // distinct constants: no folding into a loop
    if (x == 12345.f) out[threadIdx.x] = x;
}
template <int K>
static int run(float *d, int grid) {
    hipStream_t s; CK(hipStreamCreate(&s));
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < 2000; i++) hipLaunchKernelGGL(k_chain<K>, dim3(grid), dim3(256), 0, s, d, 1.0001f, 0.5f);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s)); CK(hipStreamSynchronize(s));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < 3; r++) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s)); CK(hipStreamSynchronize(s));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"K\": %d, \"grid\": %d, \"us_per_launch\": %.3f}\n", K, grid, ms * 1e3 / 6000);
    CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g)); CK(hipStreamDestroy(s));
    return 0;
}
int main() {
    float *d; CK(hipMalloc(&d, 4096));
    for (int grid : {1, 200}) {
        if (run<16>(d, grid) || run<256>(d, grid) || run<1024>(d, grid) || run<4096>(d, grid)) return 1;
    }
    return 0;
}
