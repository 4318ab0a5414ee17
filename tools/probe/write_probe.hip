// write_probe.hip -- MEASUREMENT ONLY: what the checksum kernels' 2-byte
// result stores cost a read stream on MI355X (gfx950), by cache policy.
//
// k_flat's per-task result stores (44 x u16 per 64 KiB task on cfg2) cost
// 4.5 % of cfg2's time although they are 0.13 % of its bytes, while the same
// stores all aimed at ONE 128-B line cost nothing (profiles/r03_flat_end_probe
// .jsonl).  This probe streams 1 KiB rows exactly like k_flat's schedule (one
// T-row task per wave, a ring of U rows in flight, inline-asm loads) and ends
// every task with R u16 stores, varying the load and store cache policies:
//   store mode  none | spread (task t writes [t*R, t*R+R)) | sameline (every
//               task writes [0, R)) | block (the block's last wave writes its
//               4 tasks' results, whole lines when 4R is a multiple of 64)
//   load policy the aux bits of the row loads (nt, plain, sc1, sc0 sc1, sc1 nt)
//   store policy plain, nt, sc1, sc0 sc1 (for the spread stores)
// Prints one JSON line per arm: median per-launch ms and GB/s.
//   hipcc -O3 --offload-arch=gfx950 tools/probe/write_probe.hip -o pip_amd/lib/write_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t rfl(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

__device__ __forceinline__ i32x4 srsrc(const void* p, uint32_t bytes) {
    const uint64_t a = (uint64_t)p;
    return i32x4{(int)rfl((uint32_t)a), (int)rfl((uint32_t)(a >> 32)), (int)rfl(bytes), 0x00020000};
}
template <int LP>
__device__ __forceinline__ void ld(u32x4& v, const i32x4& r, uint32_t off) {
    if (LP == 0) asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen nt" : "=v"(v) : "v"(off), "s"(r));
    if (LP == 1) asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(r));
    if (LP == 2) asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen sc1" : "=v"(v) : "v"(off), "s"(r));
    if (LP == 3) asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen sc0 sc1" : "=v"(v) : "v"(off), "s"(r));
    if (LP == 4) asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen sc1 nt" : "=v"(v) : "v"(off), "s"(r));
}
template <int SP>
__device__ __forceinline__ void st(uint16_t* p, uint32_t v) {
    if (SP == 0) asm volatile("global_store_short %0, %1, off" ::"v"(p), "v"(v) : "memory");
    if (SP == 1) asm volatile("global_store_short %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
    if (SP == 2) asm volatile("global_store_short %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    if (SP == 3) asm volatile("global_store_short %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}

constexpr int U = 24;

// MODE: 0 none, 1 spread, 2 sameline, 3 block
template <int LP, int SP, int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void k_probe(
    const uint8_t* __restrict__ a, uint64_t rows, uint32_t T, uint32_t R, uint16_t* res) {
    __shared__ uint16_t s_res[4 * 64];
    __shared__ uint32_t s_cnt;
    const int lane = threadIdx.x & 63;
    const uint32_t w = rfl(threadIdx.x >> 6);
    if (MODE == 3) {
        if (threadIdx.x == 0) s_cnt = 0;
        __syncthreads();
    }
    const uint64_t n_tasks = (rows + T - 1) / T;
    const uint64_t task = (uint64_t)blockIdx.x * 4 + w;
    if (task >= n_tasks) return;
    const uint64_t r0 = task * T;
    const uint32_t nr = (uint32_t)min<uint64_t>(T, rows - r0);
    const i32x4 rs = srsrc(a + r0 * 1024, nr * 1024);
    uint32_t acc = 0;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) ld<LP>(v[u], rs, (u * 64 + lane) * 16);
    for (uint32_t j = 0; j < nr; j += U) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            asm volatile("s_waitcnt vmcnt(%1)" : "+v"(v[u]) : "n"(U - 1));
            acc += v[u].x + v[u].y + v[u].z + v[u].w;
            ld<LP>(v[u], rs, ((j + U + u) * 64 + lane) * 16);  // past the task: zeros, no request
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(v[0]));
#pragma unroll
    for (int u = 1; u < U; u++) asm volatile("" : "+v"(v[u]));
    const uint32_t r = (acc ^ (acc >> 16)) & 0xFFFFu;
    if (MODE == 1 && (uint32_t)lane < R) st<SP>(res + task * R + lane, r);
    if (MODE == 2 && (uint32_t)lane < R) st<SP>(res + lane, r);
    if (MODE == 3) {
        if ((uint32_t)lane < R) s_res[w * R + lane] = (uint16_t)r;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        uint32_t prev = 0;
        if (lane == 0) prev = atomicAdd(&s_cnt, 1u);
        prev = rfl(prev);
        const uint32_t active = (uint32_t)min<uint64_t>(4, n_tasks - (uint64_t)blockIdx.x * 4);
        if (prev + 1 == active) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            for (uint32_t i = lane; i < 4 * R; i += 64) st<SP>(res + (uint64_t)blockIdx.x * 4 * R + i, s_res[i]);
        }
    }
}

__global__ void k_fill(uint64_t* p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = (i * 0x9E3779B97F4A7C15ull) ^ (i >> 7);
}

typedef void (*kfn)(const uint8_t*, uint64_t, uint32_t, uint32_t, uint16_t*);
struct Arm {
    std::string name;
    kfn fn;
};

int main(int argc, char** argv) {
    const double gb = argc > 1 ? atof(argv[1]) : 6.216;
    const uint32_t T = argc > 2 ? (uint32_t)atoi(argv[2]) : 64, R = argc > 3 ? (uint32_t)atoi(argv[3]) : 44;
    const int rounds = 3, reps = 15;
    std::vector<Arm> arms = {
        {"nt_none", k_probe<0, 0, 0>},           {"nt_spread", k_probe<0, 0, 1>},
        {"nt_sameline", k_probe<0, 0, 2>},       {"nt_block", k_probe<0, 0, 3>},
        {"nt_spread_stnt", k_probe<0, 1, 1>},    {"nt_spread_stsc1", k_probe<0, 2, 1>},
        {"nt_spread_stsc01", k_probe<0, 3, 1>},  {"nt_block_stsc1", k_probe<0, 2, 3>},
        {"plain_none", k_probe<1, 0, 0>},        {"plain_spread", k_probe<1, 0, 1>},
        {"sc1_none", k_probe<2, 0, 0>},          {"sc1_spread", k_probe<2, 0, 1>},
        {"sc01_none", k_probe<3, 0, 0>},         {"sc01_spread", k_probe<3, 0, 1>},
        {"sc1nt_none", k_probe<4, 0, 0>},        {"sc1nt_spread", k_probe<4, 0, 1>},
    };
    if (getenv("PROBE_ARMS")) {
        std::string f = std::string(",") + getenv("PROBE_ARMS") + ",";
        std::vector<Arm> keep;
        for (const Arm& m : arms)
            if (f.find("," + m.name + ",") != std::string::npos) keep.push_back(m);
        arms = keep;
    }
    const uint64_t rows = (uint64_t)(gb * 1e9) / 1024;
    const uint64_t tasks = (rows + T - 1) / T;
    uint8_t* a;
    uint16_t* res;
    CK(hipMalloc(&a, rows * 1024));
    CK(hipMalloc(&res, (tasks + 8) * R * 2 + 4096));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t*)a, rows * 1024 / 8);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const dim3 grid((uint32_t)((tasks + 3) / 4));
    for (int rd = 0; rd < rounds; rd++) {
        for (const Arm& m : arms) {
            std::vector<float> ms;
            for (int i = 0; i < reps + 3; i++) {
                CK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL(m.fn, grid, dim3(256), 0, 0, a, rows, T, R, res);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float t;
                CK(hipEventElapsedTime(&t, e0, e1));
                if (i >= 3) ms.push_back(t);
            }
            CK(hipGetLastError());
            std::sort(ms.begin(), ms.end());
            const double med = ms[ms.size() / 2];
            printf("{\"probe\": \"write\", \"round\": %d, \"gbytes\": %.3f, \"T\": %u, \"R\": %u, \"arm\": \"%s\", "
                   "\"ms\": %.4f, \"GBps\": %.1f}\n",
                   rd, rows * 1024 / 1e9, T, R, m.name.c_str(), med, rows * 1024 / 1e6 / med);
            fflush(stdout);
        }
    }
    return 0;
}
