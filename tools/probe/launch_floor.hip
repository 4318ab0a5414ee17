// launch_floor.hip -- MEASUREMENT ONLY: the floor under cfg1's launch-bound
// batch (1M IPv4 headers, 20 B each, 2-B results; k_small takes ~7 us).
// Kernels over the same 1M items with k_small's grid (one item per lane, two
// per lane-task: 4,096 blocks of 256 threads... see GRID): empty; results
// written only; 20 B read per item and the results written (no checksum work).
// Per-dispatch HIP event pairs (median of 200) and back-to-back (1,000
// launches between two events).  One JSON line per kernel.
//   hipcc -O3 --offload-arch=gfx950 tools/probe/launch_floor.hip -o pip_amd/lib/launch_floor
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                \
        }                                                                            \
    } while (0)

constexpr uint32_t kItems = 1u << 20, kStride = 20, kPerLane = 2;

__global__ __launch_bounds__(256) void k_empty(uint16_t* out) {
    if (threadIdx.x == 1023) out[0] = 1;  // never
}

__global__ __launch_bounds__(256) void k_write(uint16_t* out) {
    const uint32_t i0 = (blockIdx.x * 256u + threadIdx.x) * kPerLane;
#pragma unroll
    for (uint32_t k = 0; k < kPerLane; k++)
        if (i0 + k < kItems) __builtin_nontemporal_store((uint16_t)(i0 + k), out + i0 + k);
}

__global__ __launch_bounds__(256) void k_read_write(const uint8_t* __restrict__ a, uint16_t* out) {
    const uint32_t i0 = (blockIdx.x * 256u + threadIdx.x) * kPerLane;
    uint32_t w[kPerLane][5];
#pragma unroll
    for (uint32_t k = 0; k < kPerLane; k++) {
        const uint32_t* p = reinterpret_cast<const uint32_t*>(a + (uint64_t)(i0 + k) * kStride);
#pragma unroll
        for (int j = 0; j < 5; j++) w[k][j] = i0 + k < kItems ? __builtin_nontemporal_load(p + j) : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < kPerLane; k++) {
        const uint32_t s = w[k][0] ^ w[k][1] ^ w[k][2] ^ w[k][3] ^ w[k][4];
        if (i0 + k < kItems) __builtin_nontemporal_store((uint16_t)(s ^ (s >> 16)), out + i0 + k);
    }
}

int main() {
    uint8_t* a;
    uint16_t* out;
    CK(hipMalloc(&a, (size_t)kItems * kStride));
    CK(hipMalloc(&out, (size_t)kItems * 2));
    CK(hipMemset(a, 0x5a, (size_t)kItems * kStride));
    const dim3 grid((kItems / kPerLane + 255) / 256), block(256);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int kind = 0; kind < 3; kind++) {
        auto launch = [&]() {
            if (kind == 0) hipLaunchKernelGGL(k_empty, grid, block, 0, 0, out);
            else if (kind == 1) hipLaunchKernelGGL(k_write, grid, block, 0, 0, out);
            else hipLaunchKernelGGL(k_read_write, grid, block, 0, 0, a, out);
        };
        for (int i = 0; i < 200; i++) launch();
        CK(hipDeviceSynchronize());
        std::vector<float> d;
        for (int i = 0; i < 200; i++) {
            CK(hipEventRecord(e0, 0));
            launch();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            d.push_back(t * 1e3f);
        }
        std::sort(d.begin(), d.end());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < 1000; i++) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float b2b;
        CK(hipEventElapsedTime(&b2b, e0, e1));
        CK(hipGetLastError());
        static const char* names[] = {"empty", "write_results", "read_20B_write_results"};
        printf("{\"kernel\": \"%s\", \"grid\": %u, \"event_pair_median_us\": %.2f, \"event_pair_min_us\": %.2f, "
               "\"b2b_us\": %.2f}\n",
               names[kind], grid.x, d[d.size() / 2], d[0], b2b);
    }
    return 0;
}
