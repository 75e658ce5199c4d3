// Radix sort of the screen's (key, value) pairs, whole vs segmented -- a
// measurement tool, not product code.  Question: with the entries already cut
// into P value ranges (free for bottom-s sketches: every row is ascending), is
// a segmented sort of P ranges faster than one sort of all M entries?
// usage: sort_microbench [M] > json
#include <hip/hip_runtime.h>
#include <hipcub/device/device_radix_sort.hpp>
#include <hipcub/device/device_segmented_radix_sort.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

__global__ void k_fill(uint32_t *k, uint32_t *v, uint32_t M, uint32_t seed) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < M; i += gridDim.x * blockDim.x) {
        uint64_t x = (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
        x ^= x >> 31;
        x *= 0xBF58476D1CE4E5B9ull;
        x ^= x >> 29;
        k[i] = (uint32_t)x;
        v[i] = i;
    }
}
__global__ void k_offsets(uint32_t *b, uint32_t *e, uint32_t P, uint32_t M) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < P) {
        b[p] = (uint32_t)((uint64_t)M * p / P);
        e[p] = (uint32_t)((uint64_t)M * (p + 1) / P);
    }
}

int main(int argc, char **argv) {
    const uint32_t M = argc > 1 ? (uint32_t)atol(argv[1]) : 100000000u;
    uint32_t *ki, *ko, *vi, *vo, *ob, *oe;
    CK(hipMalloc(&ki, M * 4ull));
    CK(hipMalloc(&ko, M * 4ull));
    CK(hipMalloc(&vi, M * 4ull));
    CK(hipMalloc(&vo, M * 4ull));
    CK(hipMalloc(&ob, (1u << 20) * 4ull));
    CK(hipMalloc(&oe, (1u << 20) * 4ull));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, ki, vi, M, 1234u);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    printf("{\"M\": %u, \"results\": [\n", M);
    bool first = true;
    auto run = [&](const char *name, uint32_t P, int bits, auto &&fn) {
        size_t tb = 0;
        fn(nullptr, tb);
        void *tmp;
        CK(hipMalloc(&tmp, std::max<size_t>(tb, 16)));
        std::vector<float> ms;
        for (int r = 0; r < 6; r++) {
            CK(hipEventRecord(a, 0));
            fn(tmp, tb);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float t;
            CK(hipEventElapsedTime(&t, a, b));
            if (r) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        printf("%s {\"sort\": \"%s\", \"segments\": %u, \"bits\": %d, \"ms_median\": %.4f, \"ms_min\": %.4f}\n",
               first ? " " : ",", name, P, bits, ms[ms.size() / 2], ms[0]);
        fflush(stdout);
        first = false;
        CK(hipFree(tmp));
    };
    for (int bits : {32, 24})
        run("DeviceRadixSort", 1, bits, [&](void *t, size_t &tb) {
            CK(hipcub::DeviceRadixSort::SortPairs(t, tb, ki, ko, vi, vo, M, 0, bits, 0));
        });
    for (uint32_t P : {256u, 1024u, 4096u, 16384u, 65536u, 262144u}) {
        hipLaunchKernelGGL(k_offsets, dim3((P + 255) / 256), dim3(256), 0, 0, ob, oe, P, M);
        for (int bits : {32, 24, 16}) {
            if (bits < 32 && (uint64_t)M / P > (1ull << (bits - 6))) continue;     // keep a collision rate <= 1/64
            run("DeviceSegmentedRadixSort", P, bits, [&](void *t, size_t &tb) {
                CK(hipcub::DeviceSegmentedRadixSort::SortPairs(t, tb, ki, ko, vi, vo, M, P, ob, oe, 0, bits, 0));
            });
        }
    }
    printf("]}\n");
    return 0;
}
