// stream_probe.hip -- MEASUREMENT ONLY: the HBM read rate of task schedules,
// stripped of all checksum work, on one batch-sized buffer (gfx950).
//
// Every variant streams the same bytes as consecutive 1 KiB rows (lane l of a
// row reads its 16-byte chunk, one coalesced buffer_load_dwordx4 nt per row, a
// ring of U rows in flight per wave, range-checked so loads past a task read
// zeros without a memory request) and differs only in who reads which rows:
//   disp    one task of T rows per wave, WPB waves per block, the hardware
//           dispatcher deals blocks in order (k_flat's schedule)
//   coop    one task of WPB*T rows per BLOCK, its waves interleaved row by row
//           (wave w reads rows w, w+WPB, ...), so a block's waves end together
//   persist a resident grid; each wave claims T-row tasks in global order from
//           one atomic counter, the next claim issued while the current task runs
// Prints one JSON line per (variant, size): median per-launch ms and GB/s.
//   hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-atomic-optimizer-strategy=None \
//         tools/probe/stream_probe.hip -o pip_amd/lib/stream_probe
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
__device__ __forceinline__ uint32_t rfl(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

template <int U>
constexpr int wpe() { return U >= 32 ? 2 : (U >= 24 ? 3 : 4); }

// The ring is written with inline asm: the compiler otherwise clusters a
// branch-free loop's reloads into batches (every row waited for before any
// reload), while k_flat's per-row branches keep its ring at vmcnt(U-1).
typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4 srsrc(const void* p, uint32_t bytes) {
    const uint64_t a = (uint64_t)p;
    return i32x4{(int)rfl((uint32_t)a), (int)rfl((uint32_t)(a >> 32)), (int)rfl(bytes), 0x00020000};
}
// POL: the load's cache-policy bits (1 = nt, 2 = sc0, 4 = sc1); the default
// arms use nt alone, the POL arms (kind 40 + POL) sweep the combinations
template <int POL = 1>
__device__ __forceinline__ void ld_asm(u32x4& v, const i32x4& r, uint32_t off) {
    if constexpr (POL == 0) asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(r));
    if constexpr (POL == 1) asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen nt" : "=v"(v) : "v"(off), "s"(r));
    if constexpr (POL == 2) asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen sc0" : "=v"(v) : "v"(off), "s"(r));
    if constexpr (POL == 3) asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen sc0 nt" : "=v"(v) : "v"(off), "s"(r));
    if constexpr (POL == 4) asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen sc1" : "=v"(v) : "v"(off), "s"(r));
    if constexpr (POL == 5) asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen sc1 nt" : "=v"(v) : "v"(off), "s"(r));
    if constexpr (POL == 6) asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen sc0 sc1" : "=v"(v) : "v"(off), "s"(r));
    if constexpr (POL == 7) asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen sc0 sc1 nt" : "=v"(v) : "v"(off), "s"(r));
}
template <int N>
__device__ __forceinline__ void wait_vm(u32x4& v) {
    asm volatile("s_waitcnt vmcnt(%1)" : "+v"(v) : "n"(N));
}

// rows [0, nr) of a resource, row j at byte (j * step + first) * 1 KiB
// OVH > 0: per row OVH dependent VALU ops and OVH/8 uniform branches on top of
// the add -- a stand-in for a real kernel's per-row bookkeeping
template <int U, int OVH = 0, int G = 1>
__device__ __forceinline__ uint32_t row_of(uint32_t j, uint32_t first, uint32_t step) {
    return ((j / G) * step + first) * G + j % G;
}
template <int U, int OVH = 0, int G = 1, int POL = 1>
__device__ __forceinline__ uint32_t stream_rows(i32x4 b, uint32_t first, uint32_t step, uint32_t nr, int lane) {
    uint32_t acc = 0;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) ld_asm<POL>(v[u], b, (row_of<U, OVH, G>(u, first, step) * 64 + lane) * 16);
    for (uint32_t j = 0; j < nr; j += U) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            wait_vm<U - 1>(v[u]);
            acc += v[u].x + v[u].y + v[u].z + v[u].w;
#pragma unroll
            for (int i = 0; i < OVH; i++) {
                acc = (acc ^ (uint32_t)(i * 0x9E37u)) + (acc >> 3);
                if (i % 8 == 7 && ((j + u + i) & 1)) acc ^= rfl(acc) >> 7;  // a uniform scalar branch
            }
            ld_asm<POL>(v[u], b, (row_of<U, OVH, G>(j + U + u, first, step) * 64 + lane) * 16);
        }
    }
    wait_vm<0>(v[0]);  // drain the dummies before their registers are reused:
#pragma unroll
    for (int u = 1; u < U; u++) asm volatile("" : "+v"(v[u]));  // every ring register live until here
    return acc;
}

// a wave task = tc chunks of 16 B (rows of 1 KiB counted from the task's start)
template <int U, int WPB>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(wpe<U>()))) void k_disp(
    const uint8_t* __restrict__ a, uint64_t chunks, uint32_t tc, uint32_t* out) {
    const int lane = threadIdx.x & 63;
    const uint64_t task = (uint64_t)blockIdx.x * WPB + rfl(threadIdx.x >> 6);
    const uint64_t c0 = task * tc;
    if (c0 >= chunks) return;
    const uint32_t nc = (uint32_t)min<uint64_t>(tc, chunks - c0);
    const uint32_t acc = stream_rows<U>(srsrc(a + c0 * 16, nc * 16), 0, 1, (nc + 63) / 64, lane);
    if (acc == 0x9E3779B9u) out[0] = acc;  // keeps the loads alive; never true on the fill
}

// a block task = tc chunks of 16 B
template <int U, int WPB, int OVH = 0, int G = 1, int POL = 1>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(wpe<U>()))) void k_coop(
    const uint8_t* __restrict__ a, uint64_t chunks, uint32_t tc, uint32_t* out) {
    const int lane = threadIdx.x & 63;
    const uint32_t w = rfl(threadIdx.x >> 6);
    const uint64_t c0 = (uint64_t)blockIdx.x * tc;
    if (c0 >= chunks) return;
    const uint32_t nc = (uint32_t)min<uint64_t>(tc, chunks - c0);
    const uint32_t nb = (nc + 63) / 64;
    // this wave's rows: groups of G rows, groups w, w+WPB, ... (rows past the task read zeros)
    const uint32_t ng = (nb + G - 1) / G, nr = ng > w ? (ng - w + WPB - 1) / WPB * G : 0;
    const uint32_t acc = stream_rows<U, OVH, G, POL>(srsrc(a + c0 * 16, nc * 16), w, WPB, nr, lane);
    if (acc == 0x9E3779B9u) out[0] = acc;
}

template <int U, int WPB>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(wpe<U>()))) void k_persist(
    const uint8_t* __restrict__ a, uint64_t rows, uint32_t T, uint32_t* out, uint32_t* ctr) {
    const int lane = threadIdx.x & 63;
    const uint64_t n_tasks = (rows + T - 1) / T;
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(ctr, 1u);
    t = rfl(t);
    uint32_t acc = 0;
    while (t < n_tasks) {
        uint32_t nxt = 0;
        if (lane == 0) nxt = atomicAdd(ctr, 1u);  // in flight while this task streams
        const uint64_t r0 = (uint64_t)t * T;
        const uint32_t nr = (uint32_t)min<uint64_t>(T, rows - r0);
        acc += stream_rows<U>(srsrc(a + r0 * 1024, nr * 1024), 0, 1, nr, lane);
        t = rfl(nxt);
    }
    if (acc == 0x9E3779B9u) out[0] = acc;
}

// persistent coop: a resident grid of G blocks; block b takes block tasks
// b, b+G, b+2G, ... (grid-stride, so the tasks in flight stay ~G wide) and each
// wave's ring runs straight across them (no drain between tasks)
__device__ __forceinline__ void gld_asm(u32x4& v, const uint8_t* p) {
    asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p));
}
template <int U>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(wpe<U>()))) void k_coop_persist(
    const uint8_t* __restrict__ a, uint64_t rows, uint32_t T, uint32_t* out) {
    const int lane = threadIdx.x & 63;
    const uint32_t w = rfl(threadIdx.x >> 6);
    const uint64_t bt = 4ull * T;                   // rows per block task
    const uint64_t n_tasks = rows / bt;             // whole tasks only (the probe's sizes)
    const uint64_t G = gridDim.x;
    const uint64_t my_tasks = n_tasks > blockIdx.x ? (n_tasks - blockIdx.x + G - 1) / G : 0;
    const uint64_t nr = my_tasks * T;               // this wave's rows over all its tasks
    const uint32_t sh = __builtin_ctz(T);  // T: a power of two
    auto addr = [&](uint64_t j) -> const uint8_t* {  // the wave's j-th row (past the end: row 0 again)
        if (j >= nr) j = 0;
        const uint64_t t = blockIdx.x + G * (j >> sh);
        return a + ((t * bt) + w + 4 * (j & (T - 1))) * 1024 + lane * 16;
    };
    uint32_t acc = 0;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) gld_asm(v[u], addr(u));
    for (uint64_t j = 0; j < nr; j += U) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            asm volatile("s_waitcnt vmcnt(%1)" : "+v"(v[u]) : "n"(U - 1));
            acc += v[u].x + v[u].y + v[u].z + v[u].w;
            gld_asm(v[u], addr(j + U + u));
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(v[0]));
#pragma unroll
    for (int u = 1; u < U; u++) asm volatile("" : "+v"(v[u]));
    if (acc == 0x9E3779B9u) out[0] = acc;
}

__global__ void k_fill(uint64_t* p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = (i * 0x9E3779B97F4A7C15ull) ^ (i >> 7);
}

struct Arm {
    std::string name;
    int U, WPB;
    uint32_t T;
    int kind;  // 0 disp, 1 coop, 2 persist, 3/4 coop with 24/48 ops of per-row overhead
};

// PROBE_TASK_SKEW=s (chunks): wave / block tasks s chunks shorter than T rows,
// so task starts drift off 1 KiB (and 128-B line) alignment, as packet tasks do
static uint32_t g_skew = 0;
template <int U, int WPB>
static void launch(const Arm& m, const uint8_t* a, uint64_t rows, uint32_t* out, uint32_t* ctr, int cus) {
    if (m.kind == 0) {
        const uint32_t tc = m.T * 64 - g_skew;
        const uint64_t tasks = (rows * 64 + tc - 1) / tc;
        hipLaunchKernelGGL((k_disp<U, WPB>), dim3((uint32_t)((tasks + WPB - 1) / WPB)), dim3(64 * WPB), 0, 0, a, rows * 64, tc, out);
    } else if (m.kind == 1) {
        const uint32_t tc = WPB * m.T * 64 - g_skew;
        hipLaunchKernelGGL((k_coop<U, WPB>), dim3((uint32_t)((rows * 64 + tc - 1) / tc)), dim3(64 * WPB), 0, 0, a, rows * 64, tc, out);
    } else if (m.kind == 5) {  // persistent coop: every wave slot the occupancy cap allows, 4-wave blocks
        hipLaunchKernelGGL((k_coop_persist<U>), dim3(cus * wpe<U>()), dim3(256), 0, 0, a, rows, m.T, out);
    } else if (m.kind >= 10 && m.kind < 40) {  // coop, rows in groups of G = kind - 10 (2, 4, 8, 16)
        const uint32_t tc = WPB * m.T * 64 - g_skew;
        const dim3 g((uint32_t)((rows * 64 + tc - 1) / tc));
        if (m.kind == 12) hipLaunchKernelGGL((k_coop<U, WPB, 0, 2>), g, dim3(64 * WPB), 0, 0, a, rows * 64, tc, out);
        if (m.kind == 14) hipLaunchKernelGGL((k_coop<U, WPB, 0, 4>), g, dim3(64 * WPB), 0, 0, a, rows * 64, tc, out);
        if (m.kind == 18) hipLaunchKernelGGL((k_coop<U, WPB, 0, 8>), g, dim3(64 * WPB), 0, 0, a, rows * 64, tc, out);
        if (m.kind == 26) hipLaunchKernelGGL((k_coop<U, WPB, 0, 16>), g, dim3(64 * WPB), 0, 0, a, rows * 64, tc, out);
    } else if (m.kind >= 40 && m.kind < 48) {  // coop, load cache policy kind - 40
        const uint32_t tc = WPB * m.T * 64 - g_skew;
        const dim3 g((uint32_t)((rows * 64 + tc - 1) / tc));
        const dim3 b(64 * WPB);
        switch (m.kind - 40) {
            case 0: hipLaunchKernelGGL((k_coop<U, WPB, 0, 1, 0>), g, b, 0, 0, a, rows * 64, tc, out); break;
            case 1: hipLaunchKernelGGL((k_coop<U, WPB, 0, 1, 1>), g, b, 0, 0, a, rows * 64, tc, out); break;
            case 2: hipLaunchKernelGGL((k_coop<U, WPB, 0, 1, 2>), g, b, 0, 0, a, rows * 64, tc, out); break;
            case 3: hipLaunchKernelGGL((k_coop<U, WPB, 0, 1, 3>), g, b, 0, 0, a, rows * 64, tc, out); break;
            case 4: hipLaunchKernelGGL((k_coop<U, WPB, 0, 1, 4>), g, b, 0, 0, a, rows * 64, tc, out); break;
            case 5: hipLaunchKernelGGL((k_coop<U, WPB, 0, 1, 5>), g, b, 0, 0, a, rows * 64, tc, out); break;
            case 6: hipLaunchKernelGGL((k_coop<U, WPB, 0, 1, 6>), g, b, 0, 0, a, rows * 64, tc, out); break;
            default: hipLaunchKernelGGL((k_coop<U, WPB, 0, 1, 7>), g, b, 0, 0, a, rows * 64, tc, out); break;
        }
    } else if (m.kind == 3 || m.kind == 4) {
        const uint32_t tc = WPB * m.T * 64 - g_skew;
        const dim3 g((uint32_t)((rows * 64 + tc - 1) / tc));
        if (m.kind == 3) hipLaunchKernelGGL((k_coop<U, WPB, 24>), g, dim3(64 * WPB), 0, 0, a, rows * 64, tc, out);
        else hipLaunchKernelGGL((k_coop<U, WPB, 48>), g, dim3(64 * WPB), 0, 0, a, rows * 64, tc, out);
    } else {
        const int blocks = cus * 4 * wpe<U>() / WPB;  // every wave slot the occupancy cap allows
        hipLaunchKernelGGL((k_persist<U, WPB>), dim3(blocks), dim3(64 * WPB), 0, 0, a, rows, m.T, out, ctr);
    }
}

static void run(const Arm& m, const uint8_t* a, uint64_t rows, uint32_t* out, uint32_t* ctr, int cus) {
#define PROBE_CASE(u, w) \
    if (m.U == u && m.WPB == w) return launch<u, w>(m, a, rows, out, ctr, cus);
    PROBE_CASE(16, 4) PROBE_CASE(24, 4) PROBE_CASE(32, 4) PROBE_CASE(24, 1) PROBE_CASE(24, 2) PROBE_CASE(24, 8)
    PROBE_CASE(16, 8) PROBE_CASE(16, 16) PROBE_CASE(24, 12) PROBE_CASE(32, 8) PROBE_CASE(32, 1) PROBE_CASE(16, 2)
    PROBE_CASE(2, 8) PROBE_CASE(3, 8) PROBE_CASE(4, 8) PROBE_CASE(4, 4) PROBE_CASE(6, 4) PROBE_CASE(8, 4)
    fprintf(stderr, "no instance U=%d WPB=%d\n", m.U, m.WPB);
    exit(2);
}

int main(int argc, char** argv) {
    // sizes in GB (1e9) of 1 KiB rows; default cfg2's 6.2 GB and cfg3's 9.4 GB
    std::vector<double> sizes = {6.216, 9.4};
    int reps = 15, rounds = 3, warm = 3;
    std::vector<Arm> arms = {
        {"disp_u24_w4_t64", 24, 4, 64, 0},   {"disp_u32_w4_t128", 32, 4, 128, 0}, {"coop_u24_w4_t64", 24, 4, 64, 1},
        {"coop_u24_w4_t32", 24, 4, 32, 1},   {"coop_u24_w4_t128", 24, 4, 128, 1}, {"coop_u16_w4_t64", 16, 4, 64, 1},
        {"coop_u16_w4_t32", 16, 4, 32, 1},   {"coop_u32_w4_t64", 32, 4, 64, 1},   {"coop_u32_w4_t128", 32, 4, 128, 1},
        {"coop_u24_w2_t64", 24, 2, 64, 1},   {"coop_u24_w2_t128", 24, 2, 128, 1}, {"coop_u24_w4_t64_ovh24", 24, 4, 64, 3},
        {"coop_u24_w4_t64_ovh48", 24, 4, 64, 4}, {"coop_u24_w4_t64_g2", 24, 4, 64, 12}, {"coop_u24_w4_t64_g4", 24, 4, 64, 14},
        {"coop_u24_w4_t64_g8", 24, 4, 64, 18}, {"coop_u24_w4_t64_g16", 24, 4, 64, 26},
        {"coop_persist_u24_t64", 24, 4, 64, 5}, {"coop_persist_u24_t16", 24, 4, 16, 5}, {"coop_persist_u16_t64", 16, 4, 64, 5}, {"coop_u16_w4_t64_ovh24", 16, 4, 64, 3}, {"coop_u16_w4_t64_ovh48", 16, 4, 64, 4},
        // wider blocks: 8 / 16 waves interleaved row by row over one block task
        {"coop_u24_w8_t64", 24, 8, 64, 1}, {"coop_u32_w8_t64", 32, 8, 64, 1}, {"coop_u16_w16_t64", 16, 16, 64, 1},
        {"coop_u16_w8_t64", 16, 8, 64, 1}, {"coop_u24_w8_t32", 24, 8, 32, 1},
        // k_flat_coop's jumbo schedule (ring 32, 64 rows per wave) under every load cache policy
        {"pol_plain", 32, 4, 64, 40}, {"pol_nt", 32, 4, 64, 41}, {"pol_sc0", 32, 4, 64, 42},
        {"pol_sc0_nt", 32, 4, 64, 43}, {"pol_sc1", 32, 4, 64, 44}, {"pol_sc1_nt", 32, 4, 64, 45},
        {"pol_sc0_sc1", 32, 4, 64, 46}, {"pol_sc0_sc1_nt", 32, 4, 64, 47},
        // k_packedb's schedule (cfg4): one ~64-row tile per one-wave block, a ring of 32 rows
        {"disp_u32_w1_t64", 32, 1, 64, 0}, {"disp_u32_w1_t128", 32, 1, 128, 0}, {"disp_u24_w1_t64", 24, 1, 64, 0},
        {"disp_u32_w1_t32", 32, 1, 32, 0}, {"disp_u32_w1_t16", 32, 1, 16, 0}, {"disp_u24_w4_t32", 24, 4, 32, 0},
        {"disp_u24_w4_t16", 24, 4, 16, 0}, {"disp_u16_w4_t16", 16, 4, 16, 0},
        // one ~64-row tile per 4-wave block, rows interleaved (a block-interleaved k_packedb)
        {"coop_u16_w4_t16", 16, 4, 16, 1}, {"coop_u24_w4_t16", 24, 4, 16, 1}, {"coop_u16_w4_t8", 16, 4, 8, 1},
        {"coop_u16_w2_t32", 16, 2, 32, 1}, {"coop_u24_w2_t32", 24, 2, 32, 1},
        // shallow rings (k_packedb's round-5 shape: 8 waves x 3 rows on a 64-row tile)
        {"coop_u3_w8_t8", 3, 8, 8, 1}, {"coop_u3_w8_t32", 3, 8, 32, 1}, {"coop_u3_w8_t64", 3, 8, 64, 1},
        {"coop_u2_w8_t64", 2, 8, 64, 1}, {"coop_u4_w8_t64", 4, 8, 64, 1}, {"coop_u4_w4_t64", 4, 4, 64, 1},
        {"coop_u6_w4_t64", 6, 4, 64, 1}, {"coop_u8_w4_t64", 8, 4, 64, 1}, {"coop_u8_w4_t16", 8, 4, 16, 1},
    };
    if (getenv("PROBE_ARMS")) {  // name filter: comma-separated list
        std::string f = std::string(",") + getenv("PROBE_ARMS") + ",";
        std::vector<Arm> keep;
        for (const Arm& m : arms)
            if (f.find("," + m.name + ",") != std::string::npos) keep.push_back(m);
        arms = keep;
    }
    if (argc > 1) {
        sizes.clear();
        for (char* s = argv[1]; *s;) {
            sizes.push_back(strtod(s, &s));
            if (*s == ',') s++;
        }
    }
    if (argc > 2) rounds = atoi(argv[2]);
    if (getenv("PROBE_WARM")) warm = atoi(getenv("PROBE_WARM"));  // launches before the timed ones (clock ramp: ~30)
    if (getenv("PROBE_TASK_SKEW")) g_skew = (uint32_t)atoi(getenv("PROBE_TASK_SKEW"));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const double gmax = *std::max_element(sizes.begin(), sizes.end());
    const uint64_t bytes_max = ((uint64_t)(gmax * 1e9) + 1023) / 1024 * 1024;
    uint8_t* a;
    uint32_t *out, *ctr;
    CK(hipMalloc(&a, bytes_max));
    CK(hipMalloc(&out, 4096));
    CK(hipMalloc(&ctr, 4096));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t*)a, bytes_max / 8);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int rd = 0; rd < rounds; rd++) {
        for (double g : sizes) {
            const uint64_t rows = (uint64_t)(g * 1e9) / 1024;
            for (const Arm& m : arms) {
                std::vector<float> ms;
                for (int i = 0; i < reps + warm; i++) {
                    CK(hipMemsetAsync(ctr, 0, 4, 0));
                    CK(hipEventRecord(e0, 0));
                    run(m, a, rows, out, ctr, cus);
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float t;
                    CK(hipEventElapsedTime(&t, e0, e1));
                    if (i >= warm) ms.push_back(t);
                }
                CK(hipGetLastError());
                std::sort(ms.begin(), ms.end());
                const double med = ms[ms.size() / 2];
                printf("{\"round\": %d, \"skew\": %u, \"gbytes\": %.3f, \"arm\": \"%s\", \"ms\": %.4f, \"min_ms\": %.4f, \"GBps\": %.1f}\n", rd, g_skew,
                       rows * 1024 / 1e9, m.name.c_str(), med, ms[0], rows * 1024 / 1e6 / med);
                fflush(stdout);
            }
        }
    }
    return 0;
}
