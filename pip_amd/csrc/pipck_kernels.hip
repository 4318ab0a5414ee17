// pipck_kernels.hip -- batch checksum kernels for MI355X (gfx950) + their C ABI.
//
// Hot path: plumk97/pip pip/pip_checksum.cpp:13-148 (pip_standard_checksum and
// its five wrappers) over batches of packets resident in HBM.  Integer
// reduction, HBM-read bound: no MFMA, no LDS tiling of the payload.  See
// pipck_device.hpp for why summing little-endian dwords in any order is exact.
//
// Kernels (launch choice in launch_fixed / launch_ragged below)
//   k_flat<U,PIPE>    fixed 16-B-multiple strides >= 1 KiB (cfg2/3/5): a wave
//                     task of consecutive packets streamed as coalesced 1 KiB
//                     rows, a ring of U rows in flight, <= 1 packet boundary
//                     per row, one wave reduce per packet; one task per wave.
//   k_flat_small<U>   fixed 16-B-multiple strides 64 B .. 1 KiB: the same row
//                     stream with many packets per row, reduced by packet with
//                     a DPP prefix scan into LDS partials.
//   k_flat_tiny<U>    8-B-multiple strides up to 64 B with pseudo-headers or
//                     RX verify: the row stream copied into an LDS stage that
//                     holds whole packets, then lane-per-packet sums from LDS.
//   k_small<NL,K>     packets <= 64 B incl. their first chunk's offset (cfg1's
//                     20-B headers): one lane per packet, every load of the
//                     wave task in flight before the first reduce.
//   k_fixed<G,NL>     the remaining fixed strides (unaligned medium packets):
//                     G lanes per packet, group reduce by cross-lane shuffles.
//   k_ragged<FIN,U,PIPE,NT,WPB>
//                     ragged batches and chain segments (cfg4): a wave owns a
//                     tile of 64 segments and streams its chunks as 1 KiB rows
//                     (a ring of U in flight); packed tiles locate segments by
//                     ballot + LDS marks + DPP max-scan, others by a search
//                     over the tile's chunk prefix; rows reduce by segment with
//                     a DPP prefix scan into LDS partials.  Tiles of <= 2-chunk
//                     segments are summed lane-per-segment instead.
//   k_chain_finish    per-packet fold of chain-segment partials + pseudo-header.
#include "pipck_common.hpp"
#include "pipck_device.hpp"

#include <cxxabi.h>
#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

namespace pipck {

static_assert(kErrRange == 1u << PIPCK_ERANGE, "pipck_device.hpp's error bit must match include/pipck.h");

// ---------------------------------------------------------------------------
// flows -> pseudo-header bases
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t addr_terms(uint32_t s_addr_mem) {
    uint32_t a = __builtin_bswap32(s_addr_mem);  // ntohl, pip_checksum.cpp:47
    return (a >> 16) + (a & 0xFFFFu);
}

__global__ void k_flows4(const pipck_flow4* __restrict__ f, uint32_t n, uint32_t* __restrict__ pseudo) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    pipck_flow4 x = f[i];
    pseudo[i] = addr_terms(x.src) + addr_terms(x.dst) + x.proto;
}

__global__ void k_flows6(const pipck_flow6* __restrict__ f, uint32_t n, uint32_t* __restrict__ pseudo) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&f[i]);  // src[4] dst[4] proto
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) s += addr_terms(w[k]);
    pseudo[i] = s + f[i].proto;
}

// tune flags bit 29 (same results): k_flat / k_packed store their results
// with plain write-back stores (the r02 policy) instead of the write-through
// sc1 stores (store_result16)
constexpr uint32_t kPlainResultStores = 1u << 29;

// ---------------------------------------------------------------------------
// fixed-stride kernel
// ---------------------------------------------------------------------------
template <int G, int NL, bool VERIFY, bool NT>
__global__ __launch_bounds__(256) void k_fixed(const uint8_t* __restrict__ arena, uint64_t stride, uint32_t len,
                                               uint64_t n, const uint32_t* __restrict__ pseudo, uint32_t n_flows,
                                               const uint32_t* __restrict__ flow_of, uint64_t flow_origin,
                                               uint16_t* __restrict__ out, uint8_t* __restrict__ ok,
                                               uint32_t* __restrict__ err) {
    constexpr int GPB = 256 / G;  // packets per block per iteration
    const int sub = threadIdx.x % G;
    uint64_t pkt = (uint64_t)blockIdx.x * GPB + threadIdx.x / G;
    const uint64_t step = (uint64_t)gridDim.x * GPB;
    const uint32_t lterm = len_term(len);
    const bool implicit_flow = pseudo != nullptr && flow_of == nullptr;
    uint32_t flow = 0, flow_step = 0;
    if (implicit_flow) {  // one 64-bit modulo per thread, then incremental
        flow = (uint32_t)((flow_origin + pkt) % n_flows);
        flow_step = (uint32_t)(step % n_flows);
    }
    for (; pkt < n; pkt += step) {
        const uintptr_t addr = (uintptr_t)arena + pkt * stride;
        const int head = (int)(addr & 15);
        const u32x4* base = reinterpret_cast<const u32x4*>(addr - head);
        const int end = head + (int)len;  // one past the last byte, relative to base
        const int nch = len ? (end + 15) >> 4 : 0;
        uint64_t acc = 0;
        for (int cb = 0; cb < nch; cb += G * NL) {  // one pass for packets <= G*NL*16 bytes
            u32x4 v[NL];
#pragma unroll
            for (int k = 0; k < NL; k++) {
                const int c = cb + k * G + sub;
                v[k] = c < nch ? (NT ? load_stream(base + c) : load_plain(base + c)) : u32x4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int k = 0; k < NL; k++) {
                const int c = cb + k * G + sub;
                const int lo = c == 0 ? head : 0;
                const int hi = end - 16 * c;
                u32x4 x = v[k];
                if (lo != 0) x = mask_chunk(x, lo, hi);  // a misaligned first chunk (rare)
                else if (hi < 16) x = mask_tail(x, hi);
                acc += sum4(x);
            }
        }
        uint32_t s = fold64(acc);
#pragma unroll
        for (int off = G / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, G);
        if (sub == 0) {
            const uint32_t F = be_fold(s, addr);
            uint32_t P = 0;
            bool fbad = false;  // a flow_of entry past the table (_n forms): result 0, ERANGE
            if (pseudo) P = (flow_of ? flow_pseudo(pseudo, flow_of[pkt], n_flows, fbad) : pseudo[flow]) + lterm;
            if (VERIFY)
                ok[pkt] = !fbad && fold16(P + F) == 0xFFFFu;
            else
                out[pkt] = fbad ? (uint16_t)0 : finish(P, F);
            if (fbad) flow_refused(err);
        }
        if (implicit_flow) {
            flow += flow_step;
            if (flow >= n_flows) flow -= n_flows;
        }
    }
}

// ---------------------------------------------------------------------------
// small-packet kernel: one lane per packet, K packets per lane in flight
// ---------------------------------------------------------------------------
// For packets of at most 64 bytes including their offset in the first 16-byte
// chunk (cfg1's 20-byte IPv4 headers at a 24-byte stride).  A wave owns 64*K
// consecutive packets; lane l takes packets base + 64k + l, so each of the K*NL
// load instructions reads 64 packets' chunks from one contiguous span.  Every
// data and flow-table load of the task is issued before the first reduce, and
// the 2-byte results are stored last (loads and stores share VM_CNT on gfx9):
// the k_fixed loop instead waits on each packet's loads, then on its flow
// entry, then stores, so it holds little in flight.  One task per wave (the
// dispatcher is the queue, as in k_flat).
template <int NL, int K, bool VERIFY, bool NT>
__global__ __launch_bounds__(256) void k_small(const uint8_t* __restrict__ arena, uint64_t stride, uint32_t len,
                                               uint64_t n, const uint32_t* __restrict__ pseudo, uint32_t n_flows,
                                               const uint32_t* __restrict__ flow_of, uint64_t flow_origin,
                                               uint16_t* __restrict__ out, uint8_t* __restrict__ ok, uint32_t kflags,
                                               uint32_t* __restrict__ err) {
    const int lane = threadIdx.x & 63;
    const uint64_t base = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * (64u * K);
    if (base >= n) return;  // wave-uniform
    u32x4 v[K][NL];
    uint32_t P[K];
    uint32_t fbad = 0;  // bit k: packet k's flow_of entry is past the table (_n forms): result 0, ERANGE
    uint32_t flow = 0;
    if (pseudo && !flow_of) flow = (uint32_t)((flow_origin + base + lane) % n_flows);
    const uint32_t fstep = pseudo && !flow_of ? 64u % n_flows : 0u;
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint64_t pkt = base + 64u * k + lane;
        const uintptr_t addr = (uintptr_t)arena + pkt * stride;
        const int head = (int)(addr & 15);
        const u32x4* b = reinterpret_cast<const u32x4*>(addr - head);
        const int nch = pkt < n && len ? (head + (int)len + 15) >> 4 : 0;
#pragma unroll
        for (int j = 0; j < NL; j++)
            v[k][j] = j < nch ? (NT ? load_stream(b + j) : load_plain(b + j)) : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint64_t pkt = base + 64u * k + lane;
        P[k] = 0;
        if (pseudo && pkt < n) {
            bool b = false;
            P[k] = flow_of ? flow_pseudo(pseudo, flow_of[pkt], n_flows, b) : pseudo[flow];
            fbad |= (uint32_t)b << k;
        }
        flow += fstep;
        if (flow >= n_flows) flow -= n_flows;
    }
    const uint32_t lterm = pseudo ? len_term(len) : 0u;
    uint32_t res[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint64_t pkt = base + 64u * k + lane;
        const uintptr_t addr = (uintptr_t)arena + pkt * stride;
        const int head = (int)(addr & 15);
        uint64_t acc = 0;
#pragma unroll
        for (int j = 0; j < NL; j++) {
            const int lo = j == 0 ? head : 0;
            const int hi = head + (int)len - 16 * j;
            u32x4 x = v[k][j];
            if (lo != 0 || hi < 16) x = mask_chunk(x, lo, hi);
            acc += sum4(x);
        }
        const uint32_t F = be_fold(fold64(acc), addr);
        res[k] = VERIFY ? (uint32_t)(fold16(P[k] + lterm + F) == 0xFFFFu) : (uint32_t)finish(P[k] + lterm, F);
        if ((fbad >> k) & 1u) res[k] = 0;
    }
    if (fbad) flow_refused(err);
    // Non-temporal result stores.  Results are 2 B per 20-B header here (10 %
    // of the bytes, unlike the streaming kernels' 0.1 %): the write-through sc1
    // policy that the streaming kernels use measured 0.5-1 % slower at 64M-256M
    // headers (profiles/r03_sc1_stores_scan.jsonl), so k_small keeps nt.
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint64_t pkt = base + 64u * k + lane;
        if (pkt < n) {
            if (VERIFY)
                __builtin_nontemporal_store((uint8_t)res[k], &ok[pkt]);
            else
                __builtin_nontemporal_store((uint16_t)res[k], &out[pkt]);
        }
    }
    (void)kflags;
}

// ---------------------------------------------------------------------------
// task split shared by the streaming kernels
// ---------------------------------------------------------------------------
// Static grid-stride over tasks; with the default grid (one task per wave,
// grid_for(.., 0)) the in-order block dispatcher then acts as the task queue
// and the tasks in flight form one contiguous window sliding through the arena.
// Optional XCD grouping (pipck_tune flags bit 3): the dispatcher deals blocks
// round-robin over the 8 XCDs, so blocks with equal blockIdx % 8 share an XCD
// and each such group can take one contiguous eighth of the tasks (8 windows).
// Measured: one window is as fast or faster from 38 to 151 GB
// (profiles/r01_size_scan3.jsonl), so grouping is off by default.  Speed only:
// any placement computes the same results.
struct TaskRange {
    uint64_t first, end, step;
};
constexpr uint32_t kXcdGroups = 8u;
constexpr uint32_t kNoPackedTiles = 16u;  // pipck_tune flags bit 4: ragged tiles always take the lookup path
constexpr uint32_t kWideBlocks = 32u;     // pipck_tune flags bit 5: 4-wave ragged blocks instead of 1-wave
template <uint32_t WPB = 4>  // waves per block
__device__ __forceinline__ TaskRange xcd_tasks(uint64_t n_tasks, bool grouped) {
    // wave-uniform as far as the compiler knows too: task addresses feed scalar
    // buffer resources, and a "divergent" one is wrapped in a readfirstlane loop
    const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (!grouped || gridDim.x < 8) return {(uint64_t)blockIdx.x * WPB + w, n_tasks, (uint64_t)gridDim.x * WPB};
    const uint32_t g = blockIdx.x & 7, gi = blockIdx.x >> 3;
    const uint32_t nb = (gridDim.x - g + 7) >> 3;  // blocks in group g
    const uint64_t b = n_tasks * g / 8, e = n_tasks * (g + 1) / 8;
    return {b + (uint64_t)gi * WPB + w, e, (uint64_t)nb * WPB};
}

// ---------------------------------------------------------------------------
// per-task timeline (internal measurement, pipck_trace_tasks in pipck_testing.h)
// ---------------------------------------------------------------------------
// With tune flags bit 20 the streaming kernels record, per wave task, the
// 100 MHz wall clock (s_memrealtime) when the task starts and when its results
// are stored, plus the wave's hardware slot, so tools/task_trace.py can see the
// launch ramp, the tail, per-XCD progress and the gap between consecutive tasks
// on one wave slot.  One 32-byte vector store per task; off by default.
constexpr uint32_t kTrace = 1u << 20;
struct TaskTrace {
    uint64_t task, t0, t1, hw;  // hw = XCC_ID << 32 | HW_ID
};
// XCD-weighted static deal (k_flat_xw; pipck_tune_xcd_weights in pipck_testing.h).
// The dispatcher deals block b to XCD b % 8, so every XCD gets an eighth of a
// launch's blocks whatever its HBM rate.  Here the grid is cut into periods of
// 8 M blocks, and in each period XCD x keeps only its first m_x blocks; the
// others exit at once.  The kept blocks take consecutive virtual block numbers
// in dispatch order, so the tasks in flight stay one contiguous window, and a
// faster XCD (larger m_x) takes a larger share of the tasks.
__device__ uint32_t g_xw[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // m_0 .. m_7, M
struct VBlock {
    uint64_t b, grid;  // virtual block number and virtual grid (kept blocks)
    bool live;
};
__device__ __forceinline__ VBlock xw_block() {
    const uint32_t M = g_xw[8];
    uint32_t A = 0;
#pragma unroll
    for (int x = 0; x < 8; x++) A += g_xw[x];
    const uint32_t P = 8u * M, j = blockIdx.x % P, x = j & 7u, i = j >> 3;
    uint32_t before = 0;  // kept blocks of this period dispatched before block j
#pragma unroll
    for (int y = 0; y < 8; y++) before += min(g_xw[y], i) + ((uint32_t)y < x && i < g_xw[y] ? 1u : 0u);
    const uint64_t periods = gridDim.x / P;
    return {(uint64_t)(blockIdx.x / P) * A + before, periods * A, i < g_xw[x]};
}

__device__ TaskTrace* g_trace = nullptr;
__device__ uint64_t g_trace_cap = 0;

__device__ __forceinline__ uint64_t trace_clock() { return __builtin_amdgcn_s_memrealtime(); }

// The buffer and its capacity, read once when a traced wave starts (a global
// load per task would add a vmcnt(0) wait -- for the task's result stores --
// to every task and perturb what it measures).
struct TraceBuf {
    TaskTrace* p;
    uint64_t cap;
};
__device__ __forceinline__ TraceBuf trace_buf(uint32_t kflags) {
    if (!(kflags & kTrace)) return TraceBuf{nullptr, 0};
    // consumed here (scalars): a load left pending on the untraced path would
    // stay in the compiler's wait model for the whole kernel and turn the
    // ring's vmcnt(U-1) waits into vmcnt(0)
    const uint64_t p = (uint64_t)g_trace, c = g_trace_cap;
    const uint64_t ps = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(p >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)p);
    const uint64_t cs = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(c >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)c);
    return TraceBuf{(TaskTrace*)ps, cs};
}
__device__ __forceinline__ void trace_task(uint32_t kflags, const TraceBuf& tb, uint64_t task, uint64_t t0, int lane) {
    if (!(kflags & kTrace)) return;
    TaskTrace* tr = tb.p;
    if (!tr || task >= tb.cap || lane != 0) return;
    const uint64_t t1 = trace_clock();
    const uint32_t hw = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
    const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID
    // a global (not FLAT) store: a FLAT access pending in a loop makes every
    // later vmcnt wait a vmcnt(0) (FLAT completes out of order)
    typedef __attribute__((address_space(1))) u32x4 global_v4;
    global_v4* d = (global_v4*)(tr + task);
    d[0] = u32x4{(uint32_t)task, (uint32_t)(task >> 32), (uint32_t)t0, (uint32_t)(t0 >> 32)};
    d[1] = u32x4{(uint32_t)t1, (uint32_t)(t1 >> 32), hw, xcc};
}

// ---------------------------------------------------------------------------
// flat-stream kernel: fixed strides of whole 16-byte chunks, >= 64 chunks each
// ---------------------------------------------------------------------------
// A wave owns a run of consecutive packets and streams their chunks as
// consecutive 1 KiB rows (lane l of row r reads chunk 64r + l): every load
// instruction is one fully coalesced 1 KiB read, U rows are in flight per
// wave, and since a packet spans >= 64 chunks a row holds at most one packet
// boundary.  Lanes keep a running u64 sum for the packet the row is in; at a
// boundary the finished packet's partials are folded and wave-reduced once.


// A finished packet is not reduced across the wave on the spot: every lane
// parks its folded partial (16 bits keep the residue and zero-ness) in the
// wave's LDS block, column-major (lane j's partial of packet i at j*pitch + i),
// and flat_write sums packet i's 64 partials in lane i at the task's end.  A
// per-packet DPP reduce cost ~27 issue slots (6 DPP adds with their wait
// states, readlane, the scalar fold); this costs a fold and one ds_write_b16.
// The pseudo-header loads and the global stores also wait for the task's end:
// on gfx9 both count in VM_CNT, so inside the row loop each one would make the
// next row's wait drain every load in flight.
constexpr uint32_t kFlatMaxRun = 64;  // packets per wave task
// tune flags bit 21 (MEASUREMENT ONLY, wrong results): the flat kernel's
// rows are waited for and consumed by one add each, with no per-packet
// work, so tools can time the access pattern alone.  (Bits 24..27 are the
// small kernel's packets per lane: this bit must not overlap them.)
constexpr uint32_t kLoadsOnly = 1u << 21;
// tune flags bit 22 (MEASUREMENT ONLY, no results): k_flat skips its task end
// (the per-packet LDS sums, pseudo-header add and result stores)
constexpr uint32_t kNoTaskEnd = 1u << 22;
// bit 23: k_flat's task end computes every result but stores none
// (MEASUREMENT ONLY, no results)
constexpr uint32_t kEndNoStore = 1u << 23;
// bit 28 (same results): the other fixed-stride schedule -- k_flat (one task
// per wave) instead of the block-cooperative k_flat_coop (pipck_coop.hip),
// the default for strides from 1 KiB to 64 KiB since round 4
constexpr uint32_t kFlatAltSchedule = 1u << 28;
// EXPERIMENTAL (same results): bit 30 = per-wave result stores (the r02 scheme) instead of one coalesced
// store of the whole block's results by its last wave; bit 31 = wave tasks of
// exactly the packet count the heuristic names, not rounded to a multiple of 16

constexpr uint32_t kFlatWaveStores = 1u << 30;
constexpr uint32_t kFlatFreeRun = 1u << 31;
// bit 30 in k_packed: tile rows on the r02 grid (from the tile's first chunk)
// instead of the 128-B line grid
constexpr uint32_t kPackedNoAlign = 1u << 30;
// u16 slots per lane row: >= run, and an odd number of dwords so the 64 lanes
// of one ds_write_b16 land in distinct banks (mod 32)
__host__ __device__ constexpr uint32_t flat_pitch(uint32_t run) {
    return ((run + 1) / 2 % 2 ? (run + 1) / 2 : (run + 1) / 2 + 1) * 2;
}
__device__ __forceinline__ void flat_stash(uint32_t acc, uint32_t i, uint16_t* part, uint32_t pitch, int lane) {
    part[lane * pitch + i] = (uint16_t)fold16(acc);
}

// Pseudo-header base of the task's packet `lane` (run <= 64), loaded when the
// task starts: at its end it is already in a register, so the wave's last act
// before exiting is a store, not a dependent table load.  (Issuing the task's
// first rows ahead of this load, so no round trip precedes them, measured
// 0.4-2.2 % SLOWER on cfg2-cfg5 in a separate-process A/B,
// profiles/r02_ab_rows_first.jsonl.)
__device__ __forceinline__ uint32_t flat_flow_of(uint64_t p0, uint32_t np, const uint32_t* pseudo,
                                                 const uint32_t* flow_of, int lane) {
    return pseudo && flow_of && (uint32_t)lane < np ? flow_of[p0 + lane] : 0u;
}
__device__ __forceinline__ uint32_t flat_pseudo(uint64_t p0, uint32_t np, const uint32_t* pseudo, uint32_t n_flows,
                                                const uint32_t* flow_of, uint32_t fo, uint64_t flow_origin, int lane,
                                                bool& fbad) {
    fbad = false;
    if (!pseudo || (uint32_t)lane >= np) return 0u;
    if (flow_of) return flow_pseudo(pseudo, fo, n_flows, fbad);  // n_flows bounds the entry (_n forms)
    const uint64_t f = flow_origin + p0 + (uint64_t)lane;
    // a 32-bit remainder where the index fits (wave-uniform test): the 64-bit one is ~100 instructions
    return pseudo[(flow_origin + p0 + 64u) >> 32 ? (uint32_t)(f % n_flows) : (uint32_t)f % n_flows];
}

template <bool VERIFY, bool TO_LDS = false>
__device__ __forceinline__ void flat_write(const uint16_t* part, uint32_t pitch, uint64_t p0, uint32_t np,
                                           uint32_t Pb, bool has_pseudo, uint32_t lterm, uint16_t* out, uint8_t* ok,
                                           int lane, uint32_t kflags, uint64_t magic, bool fbad, uint32_t* err) {
    if ((uint32_t)lane >= np) return;
    uint32_t s = 0;
#pragma unroll 16
    for (int j = 0; j < 64; j++) s += part[j * pitch + lane];
    const uint32_t F = bswap16(fold16(s));  // packets start 16-byte aligned: even address
    const uint32_t P = has_pseudo ? Pb + lterm : 0u;
    const uint64_t pkt = p0 + lane;
    uint32_t r = VERIFY ? (uint32_t)(fold16(P + F) == 0xFFFFu) : (uint32_t)finish(P, F);
    if (fbad) {  // a flow_of entry past the table: result 0, ERANGE
        r = 0;
        flow_refused(err);
    }
    if (!TO_LDS && (kflags & kEndNoStore) && (uint64_t)r != magic) return;  // measurement: never stores
    if (TO_LDS) {
        out[lane] = (uint16_t)r;  // `out` is this wave's row of the block's LDS results
    } else if (kflags & kPlainResultStores) {
        if (VERIFY)
            ok[pkt] = (uint8_t)r;
        else
            out[pkt] = (uint16_t)r;
    } else if (VERIFY) {
        store_result8(buf_rsrc(ok + p0, np), (uint32_t)(pkt - p0), r);
    } else {
        store_result16(buf_rsrc(out + p0, 2u * np), 2u * (uint32_t)(pkt - p0), r);
    }
}

// Row bookkeeping is incremental (cpp >= 64, so a row advances the packet by at
// most one): no divisions in the loop.  PIPE issues the next U rows' loads
// before reducing the current U, so a wave never drains its memory queue.
struct RowPos {
    uint32_t pkt, k;  // packet (within the task) and chunk-in-packet at lane 0 of the row
    __device__ __forceinline__ void advance(uint32_t cpp) {
        k += 64;
        if (k >= cpp) {
            k -= cpp;
            pkt++;
        }
    }
};

template <bool NT>
__device__ __forceinline__ void flat_load_row(u32x4& v, buf_t tb, uint32_t r, RowPos& lp, uint32_t cpp, uint32_t nch,
                                              int lane) {
    uint32_t c = r + lane;
    if (cpp != nch) {  // wave-uniform: strides with whole padding chunks
        // lanes on stride padding re-read their packet's last data chunk (a line
        // another lane fetches anyway; flat_reduce_row zeroes them)
        uint32_t k = lp.k + lane;
        if (k >= cpp) k -= cpp;
        if (k >= nch) c -= k - nch + 1;
    }
    // Unconditional, so the reduce can wait for one row at a time (vmcnt(N))
    // instead of all U; lanes past the task read zeros without a memory request.
    v = buf_load<NT>(tb, c * 16u);
    lp.advance(cpp);
}

template <int U, bool NT>
__device__ __forceinline__ void flat_load_rows(u32x4 (&v)[U], buf_t tb, uint32_t r0, RowPos& lp, uint32_t cpp,
                                               uint32_t nch, int lane) {
#pragma unroll
    for (int u = 0; u < U; u++) flat_load_row<NT>(v[u], tb, r0 + u * 64, lp, cpp, nch, lane);
}


// rs < tchunks (wave-uniform)
__device__ __forceinline__ void flat_reduce_row(const u32x4& v, uint32_t rs, uint32_t tchunks, const RowPos& pp,
                                                uint32_t& acc, uint32_t cpp, uint32_t nch, int tail, uint32_t np,
                                                uint16_t* part, uint32_t pitch, int lane, uint32_t kflags) {
    if (kflags & kLoadsOnly) {
        acc += v.x;
        return;
    }
    if (pp.k == 0 && rs > 0) {  // previous packet ended exactly at the last row's end
        flat_stash(acc, pp.pkt - 1, part, pitch, lane);
        acc = 0;
    }
    if (pp.k + 65 <= nch) {  // wave-uniform: 64 whole data chunks of one packet, none its last
        acc = dot4(v, acc);
        return;
    }
    uint32_t k = pp.k + lane;
    if (k >= cpp) k -= cpp;
    u32x4 x = v;
    if (k >= nch || rs + lane >= tchunks) x = u32x4{0u, 0u, 0u, 0u};
    else if (k == nch - 1 && tail < 16) x = mask_tail(x, tail);
    const uint32_t val = dot4(x, 0u);
    const uint32_t b = cpp - pp.k;  // first lane holding the next packet
    if (b >= 64 || pp.pkt + 1 >= np) {
        acc += val;
    } else {
        acc += lane < (int)b ? val : 0u;
        flat_stash(acc, pp.pkt, part, pitch, lane);
        acc = lane < (int)b ? 0u : val;
    }
}

template <int U>
__device__ __forceinline__ void flat_reduce_rows(const u32x4 (&v)[U], uint32_t r0, uint32_t tchunks, RowPos& pp,
                                                 uint32_t& acc, uint32_t cpp, uint32_t nch, int tail, uint32_t np,
                                                 uint16_t* part, uint32_t pitch, int lane, uint32_t kflags) {
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint32_t rs = r0 + u * 64;  // wave-uniform
        if (rs < tchunks) flat_reduce_row(v[u], rs, tchunks, pp, acc, cpp, nch, tail, np, part, pitch, lane, kflags);
        pp.advance(cpp);
    }
}

template <int U>
constexpr int flat_waves_per_simd() { return U >= 32 ? 2 : (U >= 24 ? 3 : (U >= 16 ? 4 : (U >= 8 ? 5 : 6))); }

// The kernel body; PROBE = false compiles the measurement-only bits (21-23)
// out of the production kernel k_flat (no per-row flag test), and k_flat_probe
// keeps them for the tools.
template <int U, bool PIPE, bool VERIFY, bool NT, int WPB, bool PROBE, bool XW = false>
__device__ __forceinline__ void flat_body(uint16_t* s_part, const uint8_t* __restrict__ arena, uint32_t cpp,
                                          uint32_t len, uint64_t n, uint32_t run, const uint32_t* __restrict__ pseudo,
                                          uint32_t n_flows, const uint32_t* __restrict__ flow_of, uint64_t flow_origin,
                                          uint16_t* __restrict__ out, uint8_t* __restrict__ ok, uint32_t kflags,
                                          uint32_t* __restrict__ err) {
    if (!PROBE) kflags &= ~(kLoadsOnly | kNoTaskEnd | kEndNoStore);
    // the block's place in the task order: its own number, or (XW) its number
    // among the blocks the XCD-weighted deal keeps
    uint64_t vb = blockIdx.x, vgrid = gridDim.x;
    if (XW) {
        const VBlock v = xw_block();
        if (!v.live) return;  // block-uniform, before any barrier
        vb = v.b;
        vgrid = v.grid;
        kflags &= ~kXcdGroups;
    }
    const int lane = threadIdx.x & 63;
    const uint32_t pitch = flat_pitch(run);
    uint16_t* part = s_part + (threadIdx.x >> 6) * 64u * pitch;
    const uint32_t nch = (len + 15) >> 4;                         // data chunks per packet (<= cpp)
    const int tail = nch ? (int)len - 16 * ((int)nch - 1) : 16;  // valid bytes of the last data chunk
    const uint32_t lterm = len_term(len);
    const uint64_t n_tasks = (n + run - 1) / run;
    const TaskRange tr = XW ? TaskRange{vb * WPB + (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)),
                                        n_tasks, vgrid * WPB}
                            : xcd_tasks<WPB>(n_tasks, (kflags & kXcdGroups) != 0);
    const TraceBuf trb = trace_buf(kflags);
    // Block-coalesced result stores (the default; needs one task per wave and
    // the block's waves on consecutive tasks): each wave parks its packets'
    // results in LDS and the block's LAST wave to finish writes all of them
    // with one coalesced store per 64 results.  Scattered per-wave stores of
    // 2 * run bytes hit partial 128-B lines that HBM3E (no write mask) must
    // read-modify-write between the read streams: they cost cfg2 4.5 % and
    // cfg5 1.5 % -- as much as the whole task end -- while the same stores all
    // aimed at one line cost nothing (profiles/r03_flat_end_probe.jsonl).  With
    // run a multiple of 16 (launch_fixed) a block's results are whole lines.
    const bool coalesce = !(kflags & (kFlatWaveStores | kXcdGroups)) && vgrid * WPB >= n_tasks;
    uint16_t* bres = s_part + WPB * 64u * pitch;                       // WPB * run u16
    uint32_t* bcnt = reinterpret_cast<uint32_t*>(bres + ((WPB * run + 1u) & ~1u));
    if (coalesce) {
        if (threadIdx.x == 0) *bcnt = 0;
        __syncthreads();
    }
    for (uint64_t task = tr.first; task < tr.end; task += tr.step) {
        const uint64_t t_start = (kflags & kTrace) ? trace_clock() : 0;
        const uint64_t p0 = task * run;
        const uint32_t np = (uint32_t)min<uint64_t>((uint64_t)run, n - p0);
        const uint32_t tchunks = np * cpp;
        // the task's chunks as a range-checked buffer (< 1 GiB: run <= 64, stride <= 16 MiB)
        const buf_t tb = buf_rsrc(reinterpret_cast<const u32x4*>(arena) + p0 * cpp, tchunks * 16u);
        uint32_t acc = 0;  // 16-bit folds (v_dot2_u32_u16): <= 65 chunks of a packet per lane
        RowPos lp{0, 0}, pp{0, 0};
        const uint32_t fo = flat_flow_of(p0, np, pseudo, flow_of, lane);
        bool fbad;
        const uint32_t Pb = flat_pseudo(p0, np, pseudo, n_flows, flow_of, fo, flow_origin, lane, fbad);
        u32x4 v[U];
        flat_load_rows<U, NT>(v, tb, 0, lp, cpp, nch, lane);
        if (PIPE && U >= 32) {  // deep ring: one loop, the last batch's reloads are clamped dummies
            for (uint32_t r0 = 0; r0 < tchunks; r0 += 64 * U) {
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const uint32_t rs = r0 + u * 64;  // wave-uniform
                    if (rs < tchunks) flat_reduce_row(v[u], rs, tchunks, pp, acc, cpp, nch, tail, np, part, pitch, lane, kflags);
                    pp.advance(cpp);
                    flat_load_row<NT>(v[u], tb, rs + 64 * U, lp, cpp, nch, lane);  // unconditional (past the end: zeros)
                }
            }
        } else if (PIPE) {
            // Ring: a reduced row's registers take the load U rows ahead at once.
            // While rows remain beyond the current batch every reload is issued
            // (clamped to the task's last chunk past its end, so the VM count
            // stays static and each reduce waits for its own row only); the
            // final batch is reduced without reloads -- cfg2 (ring 24) +0.6-2.1 %;
            // for the ring of 32 the second unrolled copy cost 0.6-1.2 %
            // (profiles/r01_ab_flat_tail_batch.jsonl), so it keeps one loop.
            uint32_t r0 = 0;
            for (; r0 + 64 * U < tchunks; r0 += 64 * U) {
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const uint32_t rs = r0 + u * 64;  // < tchunks here
                    flat_reduce_row(v[u], rs, tchunks, pp, acc, cpp, nch, tail, np, part, pitch, lane, kflags);
                    pp.advance(cpp);
                    flat_load_row<NT>(v[u], tb, rs + 64 * U, lp, cpp, nch, lane);
                }
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t rs = r0 + u * 64;  // wave-uniform
                if (rs < tchunks) flat_reduce_row(v[u], rs, tchunks, pp, acc, cpp, nch, tail, np, part, pitch, lane, kflags);
                pp.advance(cpp);
            }
        } else {
            for (uint32_t r0 = 0; r0 < tchunks; r0 += 64 * U) {
                flat_reduce_rows<U>(v, r0, tchunks, pp, acc, cpp, nch, tail, np, part, pitch, lane, kflags);
                if (r0 + 64 * U < tchunks) flat_load_rows<U, NT>(v, tb, r0 + 64 * U, lp, cpp, nch, lane);
            }
        }
        flat_stash(acc, np - 1, part, pitch, lane);
        wave_sync();
        if (coalesce && !(kflags & kNoTaskEnd)) {
            const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
            flat_write<VERIFY, true>(part, pitch, p0, np, Pb, pseudo != nullptr, lterm, bres + w * run, ok, lane,
                                     kflags, flow_origin | 0xFFFF000000000000ull, fbad, err);
            // release this wave's results, count it in; the last of the block's
            // active waves sees every other wave's results (LDS ops of a wave
            // complete in order; the fences order them against the count)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            uint32_t prev = 0;
            if (lane == 0) prev = atomicAdd(bcnt, 1u);
            prev = (uint32_t)__builtin_amdgcn_readfirstlane((int)prev);
            const uint64_t t0 = vb * WPB;
            const uint32_t active = (uint32_t)min<uint64_t>(WPB, n_tasks - t0);
            // measurement bit 23 (probe kernel only): the results are computed and
            // parked in LDS, and no wave stores them
            if (prev + 1 == active && !(PROBE && (kflags & kEndNoStore))) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                const uint64_t q0 = t0 * run;
                const uint32_t cnt = (uint32_t)min<uint64_t>((uint64_t)WPB * run, n - q0);
                if (kflags & kPlainResultStores) {
                    for (uint32_t i = lane; i < cnt; i += 64) {
                        if (VERIFY)
                            ok[q0 + i] = (uint8_t)bres[i];
                        else
                            out[q0 + i] = bres[i];
                    }
                } else if (VERIFY) {
                    const buf_t rb = buf_rsrc(ok + q0, cnt);
                    for (uint32_t i = lane; i < cnt; i += 64) store_result8(rb, i, bres[i]);
                } else {
                    const buf_t rb = buf_rsrc(out + q0, 2u * cnt);
                    for (uint32_t i = lane; i < cnt; i += 64) store_result16(rb, 2u * i, bres[i]);
                }
            }
        } else if (!(kflags & kNoTaskEnd)) {
            flat_write<VERIFY>(part, pitch, p0, np, Pb, pseudo != nullptr, lterm, out, ok, lane, kflags,
                               flow_origin | 0xFFFF000000000000ull, fbad, err);
        }
        trace_task(kflags, trb, task, t_start, lane);
        wave_sync();
    }
}

template <int U, bool PIPE, bool VERIFY, bool NT, int WPB = 4>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(flat_waves_per_simd<U>()))) void k_flat(
    const uint8_t* __restrict__ arena, uint32_t cpp, uint32_t len, uint64_t n, uint32_t run,
    const uint32_t* __restrict__ pseudo, uint32_t n_flows, const uint32_t* __restrict__ flow_of, uint64_t flow_origin,
    uint16_t* __restrict__ out, uint8_t* __restrict__ ok, uint32_t kflags, uint32_t* __restrict__ err) {
    extern __shared__ uint16_t s_part[];  // 4 waves x 64 lanes x pitch u16 (launch_fixed sizes it)
    flat_body<U, PIPE, VERIFY, NT, WPB, false>(s_part, arena, cpp, len, n, run, pseudo, n_flows, flow_of, flow_origin,
                                               out, ok, kflags, err);
}

// k_flat under the XCD-weighted static deal (xw_block; measurement arm, tools only)
template <int U, bool PIPE, bool VERIFY, bool NT, int WPB = 4>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(flat_waves_per_simd<U>()))) void k_flat_xw(
    const uint8_t* __restrict__ arena, uint32_t cpp, uint32_t len, uint64_t n, uint32_t run,
    const uint32_t* __restrict__ pseudo, uint32_t n_flows, const uint32_t* __restrict__ flow_of, uint64_t flow_origin,
    uint16_t* __restrict__ out, uint8_t* __restrict__ ok, uint32_t kflags, uint32_t* __restrict__ err) {
    extern __shared__ uint16_t s_part[];
    flat_body<U, PIPE, VERIFY, NT, WPB, false, true>(s_part, arena, cpp, len, n, run, pseudo, n_flows, flow_of,
                                                     flow_origin, out, ok, kflags, err);
}

// k_flat with the measurement bits 21-23 live (tools only)
template <int U, bool PIPE, bool VERIFY, bool NT, int WPB = 4>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(flat_waves_per_simd<U>()))) void k_flat_probe(
    const uint8_t* __restrict__ arena, uint32_t cpp, uint32_t len, uint64_t n, uint32_t run,
    const uint32_t* __restrict__ pseudo, uint32_t n_flows, const uint32_t* __restrict__ flow_of, uint64_t flow_origin,
    uint16_t* __restrict__ out, uint8_t* __restrict__ ok, uint32_t kflags, uint32_t* __restrict__ err) {
    extern __shared__ uint16_t s_part[];
    flat_body<U, PIPE, VERIFY, NT, WPB, true>(s_part, arena, cpp, len, n, run, pseudo, n_flows, flow_of, flow_origin,
                                              out, ok, kflags, err);
}

// ---------------------------------------------------------------------------
// flat-stream kernel for short fixed strides (16-byte multiples below 1 KiB)
// ---------------------------------------------------------------------------
// The k_flat stream (a wave task of consecutive packets read as 1 KiB rows, a
// ring of U rows in flight) for packets shorter than a row: a row now holds
// several packet boundaries.  Each lane tracks its chunk's packet and
// chunk-in-packet incrementally (64 chunks per row = q packets + rm chunks:
// no divisions), and a row reduces by packet with the head/tail prefix trick
// of the ragged kernel: the lane holding a packet's last chunk in the row adds
// its inclusive DPP prefix, the lane holding its first chunk (unless lane 0)
// subtracts its exclusive one, into the packet's LDS partial.
struct LanePos {
    uint32_t pkt, k;  // this lane's packet (within the task) and chunk-in-packet
    __device__ __forceinline__ void advance(uint32_t q, uint32_t rm, uint32_t cpp) {
        k += rm;
        pkt += q;
        if (k >= cpp) {
            k -= cpp;
            pkt++;
        }
    }
};

constexpr uint32_t kFlatSmallMaxRun = 1024;  // packets per wave task (LDS partials)

template <int U, bool VERIFY, bool NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(flat_waves_per_simd<U>()))) void k_flat_small(
    const uint8_t* __restrict__ arena, uint32_t cpp, uint32_t len, uint64_t n, uint32_t run,
    const uint32_t* __restrict__ pseudo, uint32_t n_flows, const uint32_t* __restrict__ flow_of, uint64_t flow_origin,
    uint16_t* __restrict__ out, uint8_t* __restrict__ ok, uint32_t kflags, uint32_t* __restrict__ err) {
    __shared__ uint32_t s_res[4][kFlatSmallMaxRun];
    const int lane = threadIdx.x & 63;
    uint32_t* res = s_res[threadIdx.x >> 6];
    const uint32_t nch = (len + 15) >> 4;                         // data chunks per packet (<= cpp)
    const int tail = nch ? (int)len - 16 * ((int)nch - 1) : 16;  // valid bytes of the last data chunk
    const uint32_t lterm = len_term(len);
    const uint32_t q = 64u / cpp, rm = 64u % cpp;
    const uint64_t n_tasks = (n + run - 1) / run;
    const TaskRange tr = xcd_tasks(n_tasks, (kflags & kXcdGroups) != 0);
    for (uint64_t task = tr.first; task < tr.end; task += tr.step) {
        const uint64_t p0 = task * run;
        const uint32_t np = (uint32_t)min<uint64_t>((uint64_t)run, n - p0);
        const uint32_t tchunks = np * cpp;
        const u32x4* tb = reinterpret_cast<const u32x4*>(arena) + p0 * cpp;
        for (uint32_t i = lane; i < np; i += 64) res[i] = 0;
        wave_sync();
        LanePos lp{(uint32_t)lane / cpp, (uint32_t)lane % cpp};
        LanePos pp = lp;
        u32x4 v[U];
        auto load_row = [&](u32x4& x, uint32_t rs) {
            uint32_t c = rs + lane;
            if (lp.k >= nch) c -= lp.k - nch + 1;  // padding: re-read the packet's last data chunk (masked)
            x = NT ? load_stream(tb + min(c, tchunks - 1)) : load_plain(tb + min(c, tchunks - 1));
            lp.advance(q, rm, cpp);
        };
#pragma unroll
        for (int u = 0; u < U; u++) load_row(v[u], u * 64);
        for (uint32_t r0 = 0; r0 < tchunks; r0 += 64 * U) {
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t rs = r0 + u * 64;
                if (rs < tchunks) {  // wave-uniform
                    const bool active = rs + lane < tchunks;
                    u32x4 x = v[u];
                    if (!active || pp.k >= nch) x = u32x4{0u, 0u, 0u, 0u};
                    else if (pp.k == nch - 1 && tail < 16) x = mask_tail(x, tail);
                    const uint32_t val = fold64(sum4(x));
                    const uint32_t inc = wave_incl_scan(val);
                    const bool t_ = active && (pp.k == cpp - 1 || lane == 63);
                    const bool h_ = active && pp.k == 0 && lane > 0;
                    if (t_ || h_) atomicAdd(&res[pp.pkt], (t_ ? inc : 0u) - (h_ ? inc - val : 0u));
                }
                pp.advance(q, rm, cpp);
                load_row(v[u], rs + 64 * U);  // ring: unconditional (clamped) reload
            }
        }
        wave_sync();
        uint32_t flow = 0;
        const uint32_t fstep = pseudo && !flow_of ? 64u % n_flows : 0u;
        if (pseudo && !flow_of) flow = (uint32_t)((flow_origin + p0 + lane) % n_flows);
        for (uint32_t i = lane; i < np; i += 64) {
            const uint64_t pkt = p0 + i;
            const uint32_t F = bswap16(fold16(res[i]));  // packets start 16-byte aligned: even address
            uint32_t P = 0;
            bool fbad = false;  // a flow_of entry past the table (_n forms): result 0, ERANGE
            if (pseudo) P = (flow_of ? flow_pseudo(pseudo, flow_of[pkt], n_flows, fbad) : pseudo[flow]) + lterm;
            if (VERIFY)
                ok[pkt] = !fbad && fold16(P + F) == 0xFFFFu;
            else
                out[pkt] = fbad ? (uint16_t)0 : finish(P, F);
            if (fbad) flow_refused(err);
            flow += fstep;
            if (flow >= n_flows) flow -= n_flows;
        }
        wave_sync();
    }
}

// ---------------------------------------------------------------------------
// flat-stream kernel for tiny fixed strides (8-byte multiples, 8 .. 64 B)
// ---------------------------------------------------------------------------
// cfg1's 20-byte IPv4 headers at a 24-byte stride.  A wave task of `run`
// consecutive packets is streamed as coalesced 1 KiB rows through a ring of U
// rows in flight, as in k_flat, and each arriving row is copied to an LDS
// stage (one ds_write_b128).  The stage holds a group of G rows that is a
// whole number P of packets (G x 1 KiB = P x stride, P = 64 or 128), so when
// a group is complete lane j sums packet j straight out of LDS: ceil(len/8)
// 8-byte reads from the packet's start, the last one masked to `len` -- the
// same mask for every packet, no per-lane offsets.  Each dword is folded by
// v_dot2_u32_u16 against (1,1): lo16 + hi16 (+ acc) in one instruction,
// residue- and zero-preserving (pipck_device.hpp).  Folded sums wait in LDS;
// pseudo-header lookups and the 2-byte stores run at the task's end (loads and
// stores share VM_CNT on gfx9: a store between row loads would make the next
// row's wait drain the ring).  The lane-per-packet kernels (k_small) spend
// ~60 VALU per 1 KiB row on per-lane offsets and masks and stall on issue at
// ~4.2 TB/s; this keeps the VALU work per row to the fold itself.
constexpr uint32_t kNoFlatTiny = 1u << 17;     // pipck_tune flags bit 17: never k_flat_tiny
constexpr uint32_t kForceFlatTiny = 1u << 18;  // bit 18: k_flat_tiny without pseudo-headers too
constexpr uint32_t kFlatTinyMaxHalves = 8;  // strides up to 64 B
constexpr uint32_t kFlatTinyMaxRun = 2048;  // packets per wave task

// Rows per LDS group for a stride of hpp 8-byte halves: the fewest whole rows
// holding a whole number of packets, doubled until that is >= 64 packets.
__host__ __device__ constexpr uint32_t tiny_group_rows(uint32_t hpp) {
    uint32_t odd = hpp, pow2 = 1;
    while (!(odd & 1u)) {
        odd >>= 1;
        pow2 <<= 1;
    }
    return odd * (pow2 > 1 ? pow2 / 2 : 1u);
}
// LDS per wave: the group stage plus one u16 per packet of the task
__host__ __device__ constexpr uint32_t tiny_wave_lds(uint32_t hpp, uint32_t run) {
    return tiny_group_rows(hpp) * 1024u + ((run * 2u + 15u) & ~15u);
}

template <int U, bool VERIFY, bool NT>
__global__ __launch_bounds__(256) void k_flat_tiny(const uint8_t* __restrict__ arena, uint32_t hpp, uint32_t len,
                                                   uint64_t n, uint32_t run, const uint32_t* __restrict__ pseudo,
                                                   uint32_t n_flows, const uint32_t* __restrict__ flow_of,
                                                   uint64_t flow_origin, uint16_t* __restrict__ out,
                                                   uint8_t* __restrict__ ok, uint32_t kflags,
                                                   uint32_t* __restrict__ err) {
    extern __shared__ uint32_t s_tiny[];  // 4 waves x tiny_wave_lds(hpp, run) bytes (launch_fixed sizes it)
    const int lane = threadIdx.x & 63;
    const uint32_t stride = 8u * hpp;
    const uint32_t G = tiny_group_rows(hpp), P = G * 128u / hpp;  // rows / packets per group
    uint8_t* stage = reinterpret_cast<uint8_t*>(s_tiny) + (threadIdx.x >> 6) * tiny_wave_lds(hpp, run);
    uint16_t* fs = reinterpret_cast<uint16_t*>(stage + G * 1024u);
    const uint32_t nq = (len + 7) >> 3;  // 8-byte reads per packet (len >= 1)
    const uint64_t mlast = low_bytes64((int)(len - 8 * (nq - 1)));
    const uint32_t lterm = len_term(len);
    const uint64_t n_tasks = (n + run - 1) / run;
    const TaskRange tr = xcd_tasks(n_tasks, (kflags & kXcdGroups) != 0);
    for (uint64_t task = tr.first; task < tr.end; task += tr.step) {
        const uint64_t p0 = task * run;
        const uint32_t np = (uint32_t)min<uint64_t>((uint64_t)run, n - p0);
        const uint32_t tchunks = (np * stride + 15) >> 4;
        // last chunk holding packet bytes: loads past it are clamped to it, so
        // the batch's trailing padding is never touched
        const uint32_t cmax = ((np - 1) * stride + len - 1) >> 4;
        const u32x4* tb = reinterpret_cast<const u32x4*>(arena + p0 * stride);
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t c = min((uint32_t)(u * 64 + lane), cmax);
            v[u] = NT ? load_stream(tb + c) : load_plain(tb + c);
        }
        uint32_t slot = 0, g0 = 0;  // row within the group; first packet of the group
        for (uint32_t r0 = 0; r0 < tchunks; r0 += 64 * U) {
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t rs = r0 + u * 64;
                if (rs < tchunks) {  // wave-uniform
                    *reinterpret_cast<u32x4*>(stage + slot * 1024u + lane * 16) = v[u];
                    if (++slot == G || rs + 64 >= tchunks) {  // group complete (or the task's last row)
                        wave_sync();
                        const uint32_t cnt = min(P, np - g0);
                        for (uint32_t j = lane; j < cnt; j += 64) {
                            const uint8_t* pk = stage + j * stride;
                            uint32_t acc = 0;
                            for (uint32_t q = 0; q + 1 < nq; q++) {
                                const uint2 x = *reinterpret_cast<const uint2*>(pk + 8 * q);
                                acc = dot_fold(x.x, dot_fold(x.y, acc));
                            }
                            const uint2 x = *reinterpret_cast<const uint2*>(pk + 8 * (nq - 1));
                            acc = dot_fold(x.x & (uint32_t)mlast, dot_fold(x.y & (uint32_t)(mlast >> 32), acc));
                            fs[g0 + j] = (uint16_t)bswap16(fold16(acc));  // packets start 8-byte aligned: even
                        }
                        wave_sync();
                        slot = 0;
                        g0 += P;
                    }
                }
                const uint32_t c = min(rs + 64 * U + lane, cmax);  // ring: unconditional (clamped) reload
                v[u] = NT ? load_stream(tb + c) : load_plain(tb + c);
            }
        }
        // results: 4 consecutive packets per lane and one 8-byte (4-byte for
        // RX verify) store where the output is aligned, the rest one by one
        auto result = [&](uint32_t i, uint32_t flow) -> uint32_t {
            const uint32_t F = fs[i];
            uint32_t P_ = 0;
            bool fbad = false;  // a flow_of entry past the table (_n forms): result 0, ERANGE
            if (pseudo) P_ = (flow_of ? flow_pseudo(pseudo, flow_of[p0 + i], n_flows, fbad) : pseudo[flow]) + lterm;
            if (fbad) {
                flow_refused(err);
                return 0u;
            }
            return VERIFY ? (uint32_t)(fold16(P_ + F) == 0xFFFFu) : (uint32_t)finish(P_, F);
        };
        const bool vec = ((VERIFY ? (uintptr_t)ok : (uintptr_t)out) & (VERIFY ? 3u : 7u)) == 0;  // p0 % 64 == 0
        const uint32_t nvec = vec ? np & ~3u : 0u;
        uint32_t flow = 0;
        const uint32_t fstep4 = pseudo && !flow_of ? 256u % n_flows : 0u;
        if (pseudo && !flow_of) flow = (uint32_t)((flow_origin + p0 + 4u * lane) % n_flows);
        for (uint32_t i = 4u * lane; i < nvec; i += 256) {
            uint32_t r[4], f = flow;
#pragma unroll
            for (int t = 0; t < 4; t++) {
                r[t] = result(i + t, f);
                if (++f == n_flows) f = 0;
            }
            if (VERIFY)
                __builtin_nontemporal_store(r[0] | r[1] << 8 | r[2] << 16 | r[3] << 24,
                                            reinterpret_cast<uint32_t*>(ok + p0 + i));
            else
                __builtin_nontemporal_store((uint64_t)(r[2] | r[3] << 16) << 32 | (r[0] | r[1] << 16),
                                            reinterpret_cast<uint64_t*>(out + p0 + i));
            flow += fstep4;
            if (flow >= n_flows) flow -= n_flows;
        }
        if (pseudo && !flow_of) flow = (uint32_t)((flow_origin + p0 + nvec + lane) % n_flows);
        for (uint32_t i = nvec + lane; i < np; i += 64) {
            const uint32_t x = result(i, flow);
            if (VERIFY)
                __builtin_nontemporal_store((uint8_t)x, &ok[p0 + i]);
            else
                __builtin_nontemporal_store((uint16_t)x, &out[p0 + i]);
            flow += pseudo && !flow_of ? 64u % n_flows : 0u;
            if (flow >= n_flows) flow -= n_flows;
        }
        wave_sync();
    }
}

// ---------------------------------------------------------------------------
// ragged / chain-segment kernel
// ---------------------------------------------------------------------------
struct RaggedTileLds {
    uint64_t base[64];  // 16-byte-aligned base address of each segment
    uint32_t pre[65];   // exclusive chunk prefix of the tile's segments; pre[64] = total
    uint32_t acc[64];   // LE residue partial per segment
    uint32_t span[64];  // (end << 4) | head, relative to the 16-byte-aligned base
    uint32_t mark[64];  // packed tiles: (row tag << 6) | segment starting at chunk row + i (max wins)
};

constexpr uint32_t kNoSeg = 0xFFFFFFFFu;
// k_ragged's per-segment record (len << 16 | F) of a refused chain segment:
// length 0 with a nonzero sum, which no real segment has
constexpr uint32_t kBadSeg = 0x0000FFFFu;
// A tile whose segments all span <= 2 chunks (20-B IPv4 headers) is summed
// lane-per-segment: 1.36 -> 1.69 TB/s on 20-B segments; at 3 chunks (40 B)
// the chunk stream is 3 % faster (profiles/r01_ragged_shapes6_tiny.jsonl).
constexpr uint32_t kTinyChunks = 2;
constexpr uint32_t kNoTinyTiles = 1u << 16;  // pipck_tune flags bit 16: tiny tiles take the chunk stream too


// Segment of chunk c: the last segment starting at or before c (which skips
// empty segments).  A lane's chunk advances by 64 per row, so it usually stays
// in the segment it held a row earlier (one LDS compare against that
// segment's end); only lanes that crossed a boundary binary-search the prefix.
__device__ __forceinline__ uint32_t ragged_seg_of(const RaggedTileLds& t, uint32_t c, uint32_t& scur) {
    uint32_t s = scur;
    if (c >= t.pre[s + 1]) {
        s = 0;
#pragma unroll
        for (int st = 32; st > 0; st >>= 1)
            if (t.pre[s + st] <= c) s += st;
    }
    scur = s;
    return s;
}

// Issue the 16-byte load of one row (chunks c0 .. c0+63) of the tile's chunk
// stream.  A packed tile (segments back to back at 16-byte granularity, see
// k_ragged) addresses chunk c directly at tbase + 16c, so its loads wait on
// nothing; otherwise each lane's segment is looked up first to find its base.
template <bool NT>
__device__ __forceinline__ void ragged_issue_row(const RaggedTileLds& t, uint32_t c0, uint32_t total, int lane,
                                                 u32x4& v, uint32_t& sx, uint32_t& scur, bool packed,
                                                 buf_t tbuf) {
    // The loads stay unconditional, so the reduce can wait for each row alone
    // (vmcnt(N)) instead of draining the whole batch at a branch join: on a
    // packed tile lanes past its last chunk read zeros from the range-checked
    // buffer (no memory request); elsewhere they re-read that chunk (same
    // cache line as a live lane; ragged_reduce ignores them).
    if (packed) {
        v = buf_load<NT>(tbuf, (c0 + lane) * 16u);
        __builtin_amdgcn_sched_barrier(0);  // keep row order (see flat_load_rows)
        return;
    }
    const uint32_t c = min(c0 + lane, total - 1);
    const u32x4* p;
    {
        const uint32_t s = ragged_seg_of(t, c, scur);
        sx = s;
        p = reinterpret_cast<const u32x4*>(t.base[s]) + (c - t.pre[s]);
    }
    v = NT ? load_stream(p) : load_plain(p);
    __builtin_amdgcn_sched_barrier(0);  // keep row order (see flat_load_rows)
}

template <int U, bool NT>
__device__ __forceinline__ void ragged_issue(const RaggedTileLds& t, uint32_t c0, uint32_t total, int lane,
                                             u32x4 (&v)[U], uint32_t (&sx)[U], uint32_t& scur, bool packed,
                                             buf_t tbuf) {
#pragma unroll
    for (int u = 0; u < U; u++) ragged_issue_row<NT>(t, c0 + u * 64, total, lane, v[u], sx[u], scur, packed, tbuf);
}

// Add a run of whole rows of one segment (per-lane u32 partials in racc) to the
// segment's LDS partial: one wave sum, one LDS add.
__device__ __forceinline__ void ragged_flush(RaggedTileLds& t, int lane, uint32_t& racc, uint32_t& rseg) {
    if (rseg == kNoSeg) return;  // wave-uniform
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(racc), 63);
    if (lane == 0) atomicAdd(&t.acc[rseg], tot);
    racc = 0;
    rseg = kNoSeg;
}

// Reduce one row by segment (the lookup path: tiles that are not packed).  A
// row lying wholly inside one segment only adds into the per-lane run partial
// racc.  Any other row takes a wave prefix scan: the lane holding a segment's
// last chunk in the row adds (its prefix - the prefix just before the
// segment's first chunk in the row) to the segment's LDS partial.
// row < total (wave-uniform).
__device__ __forceinline__ void ragged_reduce_row(RaggedTileLds& t, uint32_t row, uint32_t total, int lane,
                                                  const u32x4& v, uint32_t sx, uint32_t& racc, uint32_t& rseg) {
    const uint32_t c = row + lane;
    const bool active = c < total;
    const uint32_t s = sx;
    const uint32_t pre = t.pre[s];
    const uint32_t span = t.span[s];
    const int rel = (int)(c - pre);
    const int lo = rel == 0 ? (int)(span & 15) : 0;
    const int hi = (int)(span >> 4) - 16 * rel;
    u32x4 x = v;
    if (lo != 0) x = mask_chunk(x, lo, hi);  // a misaligned first chunk (rare)
    else if (hi < 16) x = mask_tail(x, hi);
    const uint32_t val = active ? dot4(x, 0u) : 0u;
    const uint32_t s0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)s);
    const uint32_t end0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)t.pre[s0 + 1]);
    rseg = (uint32_t)__builtin_amdgcn_readfirstlane((int)rseg);  // keep the run state scalar
    if (end0 >= row + 64) {  // the whole row is in segment s0 (pre[64] = total); wave-uniform
        if (s0 != rseg) {
            ragged_flush(t, lane, racc, rseg);
            rseg = s0;
        }
        racc += val;
        return;
    }
    ragged_flush(t, lane, racc, rseg);
    // Segment s's share of the row is inc[tail] - inc[head - 1]: the lane
    // holding its last chunk in the row adds its inclusive prefix, the lane
    // holding its first chunk (unless that is lane 0) subtracts its
    // exclusive one.  Both land in acc[s] mod 2^32, whose final value is
    // the true (non-wrapping) sum, so no cross-lane fetch is needed.
    const uint32_t inc = wave_incl_scan(val);
    const bool last_chunk = hi <= 16;  // this chunk ends its segment
    const bool tail = active && (lane == 63 || last_chunk);
    const bool head = active && rel == 0 && lane > 0;
    if (tail || head) atomicAdd(&t.acc[s], (tail ? inc : 0u) - (head ? inc - val : 0u));
}


// Segment ends a mixed row walks in scalar code; beyond this many the row
// finds its lanes' segments through LDS start marks instead.
constexpr uint32_t kRowEndsLoop = 4;
constexpr uint32_t kPackedMarksOnly = 1u << 19;  // pipck_tune flags bit 19: mixed rows always take the marks (k_packed: the end loop)

// Reduce one row of a packed tile (every segment starts 16-byte aligned where
// the previous one's chunks end).  Lane i of the wave holds segment i's start
// chunk pre_v and endt_v = end chunk | (len & 15) << 24.  The segment s0 of
// the row's first chunk is a ballot popcount (starts are non-decreasing),
// kept as scalars across rows.
//  * Interior row (s0 ends past the row): all 64 chunks are whole chunks of
//    s0 -- four dot2 ops into the lane's u32 run partial, nothing else.
//  * Mixed row: the segments ending inside the row are s0 .. s0+k-1 (a
//    ballot).  For k <= kRowEndsLoop a scalar loop reads each end E and tail
//    length (v_readlane) and every lane derives its segment (count of ends
//    <= its chunk), its head/tail flags and its tail mask with a few compares
//    -- no LDS round trip; more ends than that (rows of tiny segments) use LDS
//    start marks and a DPP max-scan.  Either way the row reduces by segment
//    with one DPP prefix scan and fire-and-forget LDS adds (head/tail trick),
//    and the run partial of the segment that ends here joins s0's tail lane.
__device__ __forceinline__ void ragged_reduce_row_packed(RaggedTileLds& t, uint32_t row, uint32_t total, int lane,
                                                         const u32x4& v, uint32_t pre_v, uint32_t endt_v,
                                                         uint32_t& s0, uint32_t& e0, uint32_t& racc, uint32_t& rseg,
                                                         uint32_t kflags, uint32_t lead) {
    if (row >= e0) {  // wave-uniform: the row starts past segment s0
        s0 = (uint32_t)__popcll(__ballot(pre_v <= row)) - 1u;
        e0 = (uint32_t)__builtin_amdgcn_readlane((int)endt_v, (int)s0) & 0xFFFFFFu;
    }
    s0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)s0);
    e0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)e0);
    rseg = (uint32_t)__builtin_amdgcn_readfirstlane((int)rseg);  // keep the run state scalar
    // interior row: all 64 chunks are whole chunks of s0 (and < total); the
    // first row of a tile with lead chunks (the previous tile's bytes before
    // the line-aligned start, see k_packed) takes the masked path
    if (e0 > row + 64 && (row != 0 || lead == 0)) {
        if (s0 != rseg) {
            ragged_flush(t, lane, racc, rseg);
            rseg = s0;
        }
        racc = dot4(v, racc);
        return;
    }
    // the run (whole rows of one segment) ends here: its wave total R joins
    // s0's tail contribution when it is s0's, else it is added on its own
    uint32_t R = 0;
    if (rseg != kNoSeg) {
        R = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(racc), 63);
        if (rseg != s0) {
            if (lane == 0) atomicAdd(&t.acc[rseg], R);
            R = 0;
        }
        racc = 0;
        rseg = kNoSeg;
    }
    const uint32_t c = row + lane;
    const bool active = c < total && c >= lead;
    const uint32_t end_v = endt_v & 0xFFFFFFu;
    const uint32_t k = (uint32_t)__popcll(__ballot(end_v > row && end_v <= row + 64));  // ends s0 .. s0+k-1
    uint32_t s;
    bool head, tail;
    u32x4 x = v;
    if (k <= kRowEndsLoop && !(kflags & kPackedMarksOnly)) {
        s = s0;
        head = false;
        tail = lane == 63;
        for (uint32_t j = 0; j < k; j++) {  // scalar loop over the row's segment ends
            const uint32_t et = (uint32_t)__builtin_amdgcn_readlane((int)endt_v, (int)(s0 + j));
            const uint32_t E = et & 0xFFFFFFu, tl = et >> 24;
            s += c >= E ? 1u : 0u;
            head = head || c == E;
            const bool last = c + 1 == E;
            tail = tail || last;
            if (tl && last) x = mask_tail(x, (int)tl);  // tl is wave-uniform: the mask is scalar
        }
    } else {
        // each segment starting inside the row marks its first chunk's slot (LDS
        // max, tagged by row so stale marks lose); a max-scan seeded with s0
        // carries the last start to every later lane
        const uint32_t tag = ((row >> 6) + 1u) << 6;
        if (pre_v > row && pre_v < row + 64) atomicMax(&t.mark[pre_v - row], tag | (uint32_t)lane);
        wave_sync();
        const uint32_t m = t.mark[lane];
        s = wave_incl_max(lane == 0 ? s0 : (m >= tag ? (m & 63u) : 0u));
        const int rel = (int)(c - t.pre[s]);
        const int hi = (int)(t.span[s] >> 4) - 16 * rel;  // packed: no head bytes
        if (hi < 16) x = mask_tail(x, hi);
        tail = lane == 63 || hi <= 16;
        head = rel == 0;
    }
    const uint32_t val = active ? dot4(x, 0u) : 0u;
    const uint32_t inc = wave_incl_scan(val);
    tail = tail && active;
    head = head && active && lane > 0;
    const uint32_t add = (tail ? inc + (s == s0 ? R : 0u) : 0u) - (head ? inc - val : 0u);
    if (tail || head) atomicAdd(&t.acc[s], add);
}

// Stream a tile's chunks U rows at a time and reduce them by segment.
// PIPE = a ring: as soon as row r is reduced, its registers take the load of
// row r + U, so U rows stay in flight throughout (the plain loop lets the
// queue run dry while it reduces a batch) at no extra VGPRs.
template <int U, bool PIPE, bool NT, bool PACKED>
__device__ __forceinline__ void ragged_stream(RaggedTileLds& t, uint32_t total, int lane, uintptr_t tbase,
                                              uint32_t pre_v, uint32_t endt_v, uint32_t& racc, uint32_t& rseg,
                                              uint32_t kflags, uint32_t lead) {
    u32x4 v[U];
    uint32_t sx[U];
    uint32_t scur = 0;
    uint32_t s0 = 0, e0 = 0;  // packed: segment of the row's first chunk and its end (scalars)
    if (!total) return;
    // packed: the tile's chunks as a range-checked buffer (<= 64 x 4,096 chunks)
    const buf_t tbuf = buf_rsrc(reinterpret_cast<const void*>(tbase), PACKED ? total * 16u : 0u);
    ragged_issue<U, NT>(t, 0, total, lane, v, sx, scur, PACKED, tbuf);
    for (uint32_t c0 = 0; c0 < total; c0 += 64 * U) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t row = c0 + u * 64;
            if (row < total) {  // wave-uniform
                if (PACKED)
                    ragged_reduce_row_packed(t, row, total, lane, v[u], pre_v, endt_v, s0, e0, racc, rseg, kflags,
                                             lead);
                else
                    ragged_reduce_row(t, row, total, lane, v[u], sx[u], racc, rseg);
            }
            if (PIPE) {
                // unconditional (clamped) reload: the VM count stays static, so each
                // reduce waits for its own row only (vmcnt(U-1))
                ragged_issue_row<NT>(t, row + 64 * U, total, lane, v[u], sx[u], scur, PACKED, tbuf);
            }
        }
        if (!PIPE && c0 + 64 * U < total) ragged_issue<U, NT>(t, c0 + 64 * U, total, lane, v, sx, scur, PACKED, tbuf);
    }
}

// The chunk stream of one tile of up to 64 segments (lane i = segment i, its
// bytes at addr, nch chunks counting its head offset, head = addr & 15) ->
// each lane's LE residue sum.  Tiles whose segments all fit kTinyChunks are
// summed lane-per-segment; packed tiles stream 16 B x 64 rows from the first
// segment's base; others map chunks to segments through the LDS prefix.
template <int U, bool PIPE, bool NT>
__device__ __forceinline__ uint32_t ragged_tile_sum(RaggedTileLds& t, int lane, uintptr_t addr, uint32_t head,
                                                    uint32_t len, uint32_t nch, bool packed_hint, uint32_t kflags,
                                                    uint32_t lead = 0) {
    if (__all(nch <= kTinyChunks) && !(kflags & kNoTinyTiles)) {
        // Tiny-segment tile (IPv4 headers, bare TCP/UDP headers): every lane
        // sums its own segment with its loads all in flight; no chunk stream.
        const u32x4* b = reinterpret_cast<const u32x4*>(addr - head);
        u32x4 v[kTinyChunks];
#pragma unroll
        for (uint32_t j = 0; j < kTinyChunks; j++)
            v[j] = j < nch ? (NT ? load_stream(b + j) : load_plain(b + j)) : u32x4{0u, 0u, 0u, 0u};
        uint32_t acc = 0;
#pragma unroll
        for (uint32_t j = 0; j < kTinyChunks; j++) {
            const int lo = j == 0 ? (int)head : 0;
            const int hi = (int)(head + len) - 16 * (int)j;
            u32x4 x = v[j];
            if (lo != 0 || hi < 16) x = mask_chunk(x, lo, hi);
            acc = dot4(x, acc);
        }
        return acc;
    }
    const uint32_t incl = wave_incl_scan(nch);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    t.pre[lane] = incl - nch;
    if (lane == 63) t.pre[64] = incl;
    t.span[lane] = ((head + len) << 4) | head;
    t.base[lane] = addr - head;
    t.acc[lane] = 0;
    t.mark[lane] = 0;
    const bool packed = (kflags & kNoPackedTiles) == 0 && packed_hint;
    const uintptr_t tbase = (uintptr_t)first_lane_u64(addr);
    wave_sync();
    uint32_t racc = 0;
    uint32_t rseg = kNoSeg;
    if (packed)
        ragged_stream<U, PIPE, NT, true>(t, total, lane, tbase, incl - nch, incl | (len & 15u) << 24, racc, rseg,
                                         kflags, lead);
    else  // fewer rows in flight: the lookup path needs a segment register per row
        ragged_stream<(U < 4 ? U : 4), PIPE, NT, false>(t, total, lane, tbase, incl - nch, incl, racc, rseg, kflags,
                                                        0u);
    ragged_flush(t, lane, racc, rseg);
    wave_sync();
    return t.acc[lane];
}

// One tile per wave, and by default one wave per block: tiles differ in size,
// and a block's slot (and LDS) is only released when its slowest wave ends, so
// 4-wave blocks idle ~a quarter of the wave slots on Zipf-sized traffic.
template <bool FINAL, int U, bool PIPE, bool NT, uint32_t WPB>
__global__ __launch_bounds__(256) void k_ragged(const uint8_t* __restrict__ arena, const pipck_desc* __restrict__ desc,
                                                uint64_t n, const uint32_t* __restrict__ pseudo,
                                                uint16_t* __restrict__ out, uint32_t* __restrict__ fseg,
                                                uint8_t* __restrict__ ok, uint32_t* __restrict__ err,
                                                uint32_t kflags, uint64_t arena_bytes, uint32_t n_flows) {
    __shared__ RaggedTileLds s_tile[WPB];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    RaggedTileLds& t = s_tile[w];
    const TaskRange tr = xcd_tasks<WPB>((n + 63) / 64, (kflags & kXcdGroups) != 0);
    uint64_t tile = tr.first;
    pipck_desc dn = pipck_desc{0, 0, 0};
    if (tile < tr.end && tile * 64 + lane < n) dn = desc[tile * 64 + lane];
    for (; tile < tr.end; tile += tr.step) {
        const uint64_t seg = tile * 64 + lane;
        const bool valid = seg < n;
        const pipck_desc d = dn;
        // prefetch the next tile's descriptors; they land while this tile streams
        const uint64_t nseg = (tile + tr.step) * 64 + lane;
        if (tile + tr.step < tr.end) dn = nseg < n ? desc[nseg] : pipck_desc{0, 0, 0};
        // out of domain: longer than 65535 B, bytes past the arena (overflow-safe),
        // or a flow past the table -- not read, result 0, PIPCK_ERANGE in err
        const bool bad = valid && (d.len > PIPCK_MAX_SEG_LEN || d.offset > arena_bytes ||
                                   (uint64_t)d.len > arena_bytes - d.offset || (FINAL && pseudo && d.flow >= n_flows));
        const uint32_t len = (valid && !bad) ? d.len : 0u;
        // the flow's pseudo-header base, loaded now so the tile's end waits on nothing
        const uint32_t Pbase = FINAL && pseudo && valid && !bad ? pseudo[d.flow] : 0u;
        const uintptr_t addr = (uintptr_t)arena + d.offset;
        const uint32_t head = (uint32_t)(addr & 15);
        const uint32_t nch = len ? (head + len + 15) >> 4 : 0u;
        // Packed tile: every segment starts 16-byte aligned right where the
        // previous one's chunks end (the layout of pip's TX batches and of the
        // synthetic arenas), so chunk c of the tile is at base[0] + 16c.
        const uint64_t next_off = (uint64_t)__shfl_down((long long)d.offset, 1, 64);
        const bool link = lane == 63 || seg + 1 >= n || d.offset + 16ull * nch == next_off;
        const bool packed = __all(head == 0 && link);
        const uint32_t le_sum = ragged_tile_sum<U, PIPE, NT>(t, lane, addr, head, len, nch, packed, kflags);
        if (valid) {
            const uint32_t F = bad ? 0u : be_fold(le_sum, addr);
            if (FINAL) {
                const uint32_t P = pseudo ? Pbase + len_term(len) : 0u;
                if (ok)  // RX verification: valid iff the sum incl. the checksum field folds to 0xFFFF
                    ok[seg] = !bad && fold16(P + F) == 0xFFFFu;
                else
                    out[seg] = bad ? (uint16_t)0 : finish(P, F);
            } else {
                // len <= 65535; a bad segment gets kBadSeg (length 0 with a nonzero
                // sum: no real segment) so k_chain_finish zeroes its packet
                fseg[seg] = bad ? kBadSeg : (len << 16) | F;
            }
            if (bad && err) atomicOr(err, 1u << PIPCK_ERANGE);
        }
        wave_sync();
    }
}

// ---------------------------------------------------------------------------
// packed ragged batches: lengths only, no per-packet descriptors
// ---------------------------------------------------------------------------
// Packet i starts at arena + 16 * c_i, c_i = the chunks (lengths rounded up to
// 16) of every earlier packet; tile_chunk[t] = c_{64t}.  The wave reads its 64
// u16 lengths (128 B) and one u64, derives every offset with a wave prefix
// scan of the chunk counts, and streams the tile as a packed tile of
// k_ragged.  Metadata per packet: 2 B + 1/8 B instead of a 16-byte
// descriptor.  One tile per wave, one wave per block.
template <bool VERIFY, int U, bool NT, bool MARKS>
__global__ __launch_bounds__(64) void k_packed(const uint8_t* __restrict__ arena, const uint16_t* __restrict__ lens,
                                               const uint64_t* __restrict__ tile_chunk, uint64_t n,
                                               const uint32_t* __restrict__ pseudo, uint32_t n_flows,
                                               const uint32_t* __restrict__ flow_of, uint64_t flow_origin,
                                               uint16_t* __restrict__ out, uint8_t* __restrict__ ok, uint32_t kflags,
                                               uint64_t arena_chunks, uint32_t* __restrict__ err) {
    __shared__ RaggedTileLds t;
    const int lane = threadIdx.x & 63;
    const uint64_t tile = blockIdx.x;
    const uint64_t t_start = (kflags & kTrace) ? trace_clock() : 0;
    const TraceBuf trb = trace_buf(kflags);
    const uint64_t seg = tile * 64 + lane;
    const bool valid = seg < n;
    const uint32_t len = valid ? lens[seg] : 0u;
    uint32_t Pbase = 0;
    bool fbad = false;  // a flow_of entry past the table (n_flows bounds it in the _n forms): result 0
    if (pseudo && valid) {  // loaded now so the tile's end waits on nothing
        const uint32_t f0 = (uint32_t)((flow_origin + tile * 64) % n_flows);  // one 64-bit modulo per tile
        const uint32_t f = flow_of ? flow_of[seg] : (f0 + (uint32_t)lane) % n_flows;
        fbad = f >= n_flows;
        Pbase = fbad ? 0u : pseudo[f];
    }
    // The tile's row grid starts on the 128-B line holding its first byte: the
    // `lead` chunks before it (the previous tile's last bytes) are loaded and
    // zeroed, and packet 0 of the tile is streamed as if it began there, so
    // every 1 KiB row is 8 whole lines and no line is fetched by two rows of a
    // tile (tune flags bit 30: the r02 grid from the tile's first chunk).
    const uint32_t nch = (len + 15) >> 4;
    const uint32_t nv = (uint32_t)min<uint64_t>(64, n - tile * 64);
    // The tile's chunks [tc0, tc0 + its chunk count) must lie in the arena
    // (scalar, overflow-safe): a tile reaching past it -- a stale or foreign
    // index -- reads nothing, sets PIPCK_ERANGE in err and yields 0 for each of
    // its packets.
    const uint64_t tc0 = tile_chunk[tile];
    const uint32_t tile_ch = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(nch), 63);
    if (!(tc0 <= arena_chunks && (uint64_t)tile_ch <= arena_chunks - tc0)) {
        if (lane == 0 && err) atomicOr(err, 1u << PIPCK_ERANGE);
        if (VERIFY)
            store_result8(buf_rsrc(ok + tile * 64, nv), (uint32_t)lane, 0u);
        else
            store_result16(buf_rsrc(out + tile * 64, 2u * nv), 2u * (uint32_t)lane, 0u);
        return;
    }
    const uintptr_t tbase = (uintptr_t)arena + 16ull * tc0;
    const uint32_t lead = (__all(nch <= kTinyChunks) || (kflags & kPackedNoAlign)) ? 0u : (uint32_t)(tbase >> 4) & 7u;
    const uint32_t nch_s = nch + (lane == 0 ? lead : 0u);
    const uint32_t excl = wave_incl_scan(nch_s) - nch_s;
    const uintptr_t addr = tbase - 16u * lead + 16ull * excl;
    // MARKS: the marks path compiled alone (the scalar end loop folded away)
    const uint32_t le_sum = ragged_tile_sum<U, true, NT>(t, lane, addr, 0u, len + (lane == 0 ? 16u * lead : 0u), nch_s,
                                                         true, MARKS ? kflags | kPackedMarksOnly : kflags, lead);
    const uint32_t F = bswap16(fold16(le_sum));  // 16-byte aligned: even address
    const uint32_t P = pseudo ? Pbase + len : 0u;
    uint32_t r = VERIFY ? (uint32_t)(fold16(P + F) == 0xFFFFu) : (uint32_t)finish(P, F);
    if (fbad) {
        r = 0;
        if (err) atomicOr(err, 1u << PIPCK_ERANGE);
    }
    if (kflags & kPlainResultStores) {
        if (valid) {
            if (VERIFY)
                ok[seg] = (uint8_t)r;
            else
                out[seg] = (uint16_t)r;
        }
    } else if (VERIFY) {  // write-through (sc1): see store_result16; lanes past the batch are range-checked off
        store_result8(buf_rsrc(ok + tile * 64, nv), (uint32_t)lane, r);
    } else {
        store_result16(buf_rsrc(out + tile * 64, 2u * nv), 2u * (uint32_t)lane, r);
    }
    trace_task(kflags, trb, tile, t_start, lane);
}

// Index of a packed batch: tile_chunk[t] for t = 0 .. ceil(n/64) (the last
// entry = the arena's chunks).  Pass 1 sums each tile's chunks into
// tile_chunk[t + 1]; pass 2, one block, turns them into a prefix in place.
__global__ __launch_bounds__(64) void k_packed_tile_sums(const uint16_t* __restrict__ lens, uint64_t n,
                                                         uint64_t* __restrict__ tile_chunk) {
    const uint64_t seg = (uint64_t)blockIdx.x * 64 + threadIdx.x;
    const uint32_t nch = seg < n ? (lens[seg] + 15u) >> 4 : 0u;
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(nch), 63);
    if (threadIdx.x == 0) tile_chunk[blockIdx.x + 1] = tot;
}

__global__ __launch_bounds__(1024) void k_packed_tile_scan(uint64_t* __restrict__ tile_chunk, uint64_t n_tiles) {
    __shared__ uint64_t part[1024];
    const uint32_t i = threadIdx.x;
    const uint64_t per = (n_tiles + 1023) / 1024, b = min<uint64_t>(n_tiles, i * per), e = min<uint64_t>(n_tiles, b + per);
    uint64_t s = 0;
    for (uint64_t k = b; k < e; k++) s += tile_chunk[k + 1];
    part[i] = s;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan of the 1024 partials
        const uint64_t x = i >= off ? part[i - off] : 0ull;
        __syncthreads();
        part[i] += x;
        __syncthreads();
    }
    // entries k+1 of this thread's range become inclusive prefixes (= the
    // exclusive prefix of tile k+1); each thread touches only its own entries
    uint64_t run = part[i] - s;
    for (uint64_t k = b; k < e; k++) {
        run += tile_chunk[k + 1];
        tile_chunk[k + 1] = run;
    }
    if (i == 0) tile_chunk[0] = 0;
}

// Per packet: the segments' folded sums and lengths, packed by k_ragged as
// (len << 16) | F, so no descriptor is read again.
// A packet whose segment range is not inside [0, n_segs], whose flow is past
// the table, or holding a segment k_ragged refused (kBadSeg) gets 0 and sets
// PIPCK_ERANGE in err.
__global__ void k_chain_finish(const uint64_t* __restrict__ seg_begin, const uint32_t* __restrict__ pkt_flow,
                               uint64_t n_pkts, const uint32_t* __restrict__ pseudo,
                               const uint32_t* __restrict__ fseg, uint16_t* __restrict__ out, uint64_t n_segs,
                               uint32_t n_flows, uint32_t* __restrict__ err) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_pkts) return;
    const uint64_t b = seg_begin[p], e = seg_begin[p + 1];
    const uint32_t flow = pkt_flow ? pkt_flow[p] : 0u;
    bool bad = b > e || e > n_segs || (pseudo && flow >= n_flows);
    uint32_t total_len = 0, F = 0;  // pip_buf::total_len is a u32 (pip/pip_buf.h:17)
    for (uint64_t s = b; !bad && s < e; s++) {
        const uint32_t x = fseg[s];
        if (x == kBadSeg) bad = true;  // (its error bit is set already)
        total_len += x >> 16;
        F += x & 0xFFFFu;
    }
    if (bad) {
        if (err) atomicOr(err, 1u << PIPCK_ERANGE);
        out[p] = 0;
        return;
    }
    const uint32_t P = pseudo ? pseudo[flow] + len_term(total_len) : 0u;
    out[p] = finish(P, F);
}

// ---------------------------------------------------------------------------
// launch-shape selection
// ---------------------------------------------------------------------------
struct Tune {
    std::atomic<uint32_t> lanes{0}, loads{0}, blocks{0}, flags{0};
};
static Tune g_tune;
bool wave_arm() { return g_tune.lanes.load() == kWaveArm; }
bool alt_schedule() { return (g_tune.flags.load() >> 28) & 1u; }
uint32_t g_tune_flags() { return g_tune.flags.load(); }
uint32_t g_tune_loads() { return g_tune.loads.load(); }
uint32_t g_tune_blocks() { return g_tune.blocks.load(); }
std::atomic<uint32_t> g_probes{0};  // pipck_tune_probes (pipck_testing.h)

// The batch kernel this thread launched last (pipck_common.hpp, PIPCK_LAUNCH).
thread_local const void* t_last_kernel = nullptr;

typedef void (*fixed_fn)(const uint8_t*, uint64_t, uint32_t, uint64_t, const uint32_t*, uint32_t, const uint32_t*,
                         uint64_t, uint16_t*, uint8_t*, uint32_t*);
struct Variant {
    int g, nl;
    fixed_fn fn[2][2];  // [verify][nt]
};
#define PIPCK_V(G, NL)                                                               \
    {                                                                                \
        G, NL, {                                                                     \
            {k_fixed<G, NL, false, false>, k_fixed<G, NL, false, true>},             \
            {k_fixed<G, NL, true, false>, k_fixed<G, NL, true, true>}                \
        }                                                                            \
    }
static const Variant kVariants[] = {
    PIPCK_V(1, 1),  PIPCK_V(1, 2),  PIPCK_V(2, 1),  PIPCK_V(2, 2),  PIPCK_V(4, 1),  PIPCK_V(4, 2),
    PIPCK_V(4, 4),  PIPCK_V(8, 2),  PIPCK_V(8, 4),  PIPCK_V(16, 2), PIPCK_V(16, 4), PIPCK_V(16, 6),
    PIPCK_V(32, 3), PIPCK_V(32, 4), PIPCK_V(64, 2), PIPCK_V(64, 4), PIPCK_V(64, 6), PIPCK_V(64, 9),
};
#undef PIPCK_V
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);

// A packet should be covered in ONE pass (all its loads in flight at once):
// among single-pass shapes take the one wasting the fewest 16-byte lane slots,
// then the most loads in flight per lane, then the widest group.  Packets too
// long for any single pass use the widest, deepest shape (fewest passes).
static const Variant& pick_variant(uint32_t nch) {
    const uint32_t fl = g_tune.lanes.load(), fn = g_tune.loads.load();
    const Variant* best = nullptr;
    double best_u = -1.0;
    for (const Variant& v : kVariants) {
        if ((fl && (uint32_t)v.g != fl) || (fn && (uint32_t)v.nl != fn)) continue;
        const uint32_t per = (uint32_t)(v.g * v.nl);
        if (nch > per) continue;
        const double u = nch ? (double)nch / (double)per : 1.0;
        const bool better = !best || u > best_u + 0.01 ||
                            (u > best_u - 0.01 && (v.nl > best->nl || (v.nl == best->nl && v.g > best->g)));
        if (better) {
            best = &v;
            best_u = u;
        }
    }
    if (best) return *best;
    for (int i = kNumVariants - 1; i >= 0; i--) {  // multi-pass: deepest matching shape
        const Variant& v = kVariants[i];
        if ((fl && (uint32_t)v.g != fl) || (fn && (uint32_t)v.nl != fn)) continue;
        if (!best || v.g * v.nl > best->g * best->nl) best = &v;
    }
    return best ? *best : kVariants[kNumVariants - 1];
}

constexpr uint32_t kNoSmall = 64u;  // pipck_tune flags bit 6: never the small-packet kernel
typedef void (*small_fn)(const uint8_t*, uint64_t, uint32_t, uint64_t, const uint32_t*, uint32_t, const uint32_t*,
                         uint64_t, uint16_t*, uint8_t*, uint32_t, uint32_t*);
struct SmallVariant {
    int k;              // packets per lane per wave task
    small_fn fn[4][2][2];  // [nl-1][verify][nt]
};
#define PIPCK_S1(NL, K)                                                                            \
    {                                                                                              \
        {k_small<NL, K, false, false>, k_small<NL, K, false, true>},                               \
            {k_small<NL, K, true, false>, k_small<NL, K, true, true>}                              \
    }
#define PIPCK_S(K) {K, {PIPCK_S1(1, K), PIPCK_S1(2, K), PIPCK_S1(3, K), PIPCK_S1(4, K)}}
// tune flags bits 24..27 select K (1 = 2, 2 = 4, 3 = 8, 4 = 16); default 2:
// deeper tasks measured slower (cfg1 at 64M-256M headers: K = 2 / 4 / 8 / 16
// -> 4.19 / 4.15 / 3.83 / 3.87 TB/s, plain loads beat nt by 10 %,
// profiles/r01_small_kernel_scan.jsonl)
static const SmallVariant kSmall[] = {PIPCK_S(2), PIPCK_S(4), PIPCK_S(8), PIPCK_S(16)};
#undef PIPCK_S
#undef PIPCK_S1
static const SmallVariant& small_variant() {
    const uint32_t k = (g_tune.flags.load() >> 24) & 0xFu;  // bits 24..27 (kLoadsOnly is bit 21)
    return kSmall[k >= 1 && k <= 4 ? k - 1 : 0];
}

constexpr uint32_t kNoFlatSmall = 128u;
constexpr uint64_t kHdrMinBatch = 8ull << 20;  // headers: k_hdr from here, k_small below  // pipck_tune flags bit 7: never the short-stride flat kernel

// host copies of the XCD-weighted deal's shape (pipck_tune_xcd_weights): kept
// blocks per period (0 = off) and blocks per XCD per period
static std::atomic<uint32_t> g_xw_kept{0}, g_xw_period{0};

static bool flat_allowed() { return (g_tune.flags.load() & 2u) == 0; }  // bit 1: never the flat kernel

typedef void (*flat_fn)(const uint8_t*, uint32_t, uint32_t, uint64_t, uint32_t, const uint32_t*, uint32_t,
                        const uint32_t*, uint64_t, uint16_t*, uint8_t*, uint32_t, uint32_t*);
struct FlatVariant {
    int u;
    bool pipe;
    flat_fn fn[2][2];  // [verify][nt]
    flat_fn probe;     // k_flat_probe (checksum, nt loads) for the default rings, else null
};
#define PIPCK_F(U, P)                                                                     \
    {                                                                                     \
        U, P, {                                                                           \
            {k_flat<U, P, false, false>, k_flat<U, P, false, true>},                      \
            {k_flat<U, P, true, false>, k_flat<U, P, true, true>}                         \
        }, (P && (U == 24 || U == 32)) ? k_flat_probe<U, P, false, true> : nullptr        \
    }
// loads_per_lane 2/4/8/16 = U rows in flight per wave; 3/5/9/13/17/25/33 = ring-pipelined U = 2/4/8/12/16/24/32
// (a ring of 40 or 48 -- 231 / 272 VGPRs -- ran cfg5 1 % / 28 % slower than 32,
// profiles/r01_flat_one_wave_scan.jsonl, r01_deep_ring_scan.jsonl)
static const FlatVariant kFlat[] = {PIPCK_F(2, false), PIPCK_F(4, false), PIPCK_F(8, false), PIPCK_F(16, false),
                                    PIPCK_F(2, true),  PIPCK_F(4, true),  PIPCK_F(8, true),  PIPCK_F(12, true),
                                    PIPCK_F(16, true), PIPCK_F(32, true), PIPCK_F(24, true)};
#undef PIPCK_F
static const flat_fn kFlatSmall[2][2] = {  // [verify][nt]
    {k_flat_small<16, false, false>, k_flat_small<16, false, true>},
    {k_flat_small<16, true, false>, k_flat_small<16, true, true>}};
#define PIPCK_T(R) \
    { {k_flat_tiny<R, false, false>, k_flat_tiny<R, false, true>}, {k_flat_tiny<R, true, false>, k_flat_tiny<R, true, true>} }
static const flat_fn kFlatTiny[3][2][2] = {PIPCK_T(4), PIPCK_T(8), PIPCK_T(16)};  // [ring 4/8/16][verify][nt]
#undef PIPCK_T

static const FlatVariant& flat_variant(uint32_t loads) {
    switch (loads) {
        case 2: return kFlat[0];
        case 4: return kFlat[1];
        case 8: return kFlat[2];
        case 3: return kFlat[4];
        case 5: return kFlat[5];
        case 9: return kFlat[6];
        case 16: return kFlat[3];
        case 13: return kFlat[7];
        case 17: return kFlat[8];
        case 33: return kFlat[9];
        case 25: return kFlat[10];

        default: return kFlat[2];
    }
}

// Default grid: blocks_per_cu 256-thread blocks per CU, or (0) one block per
// 4 work units -- every wave then takes exactly one task, and the in-order
// block dispatcher works as the task queue: the tasks in flight on the chip are
// always a contiguous window sliding through the arena (measured best; an
// explicit atomic queue or a resident-sized grid-stride grid lost 3-15 %,
// profiles/r01_grid_scan*.jsonl).
static uint32_t grid_for(uint64_t units_per_block_iter, uint64_t n, uint32_t blocks_per_cu = 8) {
    uint64_t need = (n + units_per_block_iter - 1) / units_per_block_iter;
    uint64_t cap = g_tune.blocks.load();
    if (!cap) cap = blocks_per_cu ? (uint64_t)device_cus() * blocks_per_cu : 0x7FFFFFFFull;
    if (need > cap) need = cap;
    return (uint32_t)(need ? need : 1);
}

// Load policy: tune flags bit 0 forces plain loads, bit 2 forces non-temporal
// ones; otherwise each kernel uses what measured faster on MI355X
// (profiles/README.md): nt for the streaming kernels, plain for small groups.
static bool nt_for(bool streaming) {
    const uint32_t f = g_tune.flags.load();
    if (f & 1u) return false;
    if (f & 4u) return true;
    return streaming;
}

// bounded: the _n forms (n_flows > 0 with d_pseudo; it bounds every d_flow_of
// entry on the device, d_err reports a refused one); the plain forms trust the
// entries and ignore n_flows when d_flow_of is given
static int launch_fixed(bool verify, const void* d_arena, uint64_t stride, uint32_t len, uint64_t n,
                        const uint32_t* d_pseudo, uint32_t n_flows, const uint32_t* d_flow_of, uint64_t flow_origin,
                        uint16_t* d_out, uint8_t* d_ok, uint32_t* d_err, void* stream, bool bounded) {
    if (n == 0) return PIPCK_OK;
    if (!d_arena || (verify ? !d_ok : !d_out)) {
        set_error("pipck_checksum_fixed: null arena/output");
        return PIPCK_EINVAL;
    }
    if (len > PIPCK_MAX_SEG_LEN) {
        set_error("pipck_checksum_fixed: len > 65535 is outside the batch domain");
        return PIPCK_ERANGE;
    }
    if (d_pseudo && (bounded || !d_flow_of) && n_flows == 0) {
        set_error("pipck_checksum_fixed: n_flows == 0");
        return PIPCK_EINVAL;
    }
    // the kernels' n_flows: the modulus without flow_of; with it, the bound of its entries
    const uint32_t nf = d_flow_of ? (bounded ? n_flows : UINT32_MAX) : (n_flows ? n_flows : 1u);
    if (stride < len && n > 1) {
        set_error("pipck_checksum_fixed: stride < len");
        return PIPCK_EINVAL;
    }
    if (g_tune.lanes.load() == kWaveArm)  // measurement arm: one packet per wave (pipck_wave.hip)
        return launch_wave(verify, false, d_arena, stride, len, nullptr, n, d_pseudo, nf, d_flow_of, flow_origin,
                           d_out, d_ok, d_err, as_stream(stream), (len + 30u) / 16u, g_tune.loads.load());
    const bool aligned = ((uintptr_t)d_arena % 16 == 0) && (stride % 16 == 0);
    if (aligned && flat_allowed() && !g_tune.lanes.load() && stride >= 64 * 16 && stride <= (1ull << 24) &&
        len <= stride) {
        const uint32_t cpp = (uint32_t)(stride / 16);
        // Every stride from 1 KiB to 64 KiB takes the block-cooperative stream
        // (a block's four waves on interleaved rows of one task, pipck_coop.hip).
        // Jumbo strides since round 3: cfg5 +0.6 % at 8M packets and +1.7 % at
        // 1M, cfg3 +0.9 % at 1M over k_flat (profiles/r03_flat_coop_scan.jsonl).
        // Shorter strides since round 4, with a ring of 32 rows: cfg2 -1.2 to
        // -1.5 % in time at 4M and 8M packets over three rounds, and -2.4 % /
        // -1.8 % / -1.5 % at 1,488 / 3,072 / 4,000-B strides, even at 1 / 2 KiB
        // (profiles/r04_cfg2_coop_scan.jsonl, r04_stride_scan.jsonl; one box,
        // one process, results equal).  At the 1 and 2 KiB strides k_flat
        // measured even to 1.3 % faster on the final build
        // (r04_schedule_ab.jsonl), so those two keep it.  The other schedule
        // is tune bit 28; strides past 64 KiB always take k_flat.
        const bool coop = (stride != 1024 && stride != 2048) != ((g_tune.flags.load() & kFlatAltSchedule) != 0);
        if (coop && stride <= 65536 &&
            launch_flat_coop(verify, d_arena, stride, len, n, d_pseudo, nf, d_flow_of, flow_origin, d_out, d_ok,
                             d_err, as_stream(stream), (g_tune.flags.load() >> 8) & 0xFFu, g_tune.loads.load(),
                             g_tune.flags.load()) == PIPCK_OK)
            return PIPCK_OK;
        // Rows in flight per wave and task size.  Jumbo packets (>= 4 KiB, cfg3
        // and cfg5): a ring of 32 rows (191 VGPRs, 2 waves/SIMD) over ~128-row
        // tasks, +1.9 % on cfg5 (7.12 TB/s) and +3.5 % on cfg3 over a ring of 16
        // with 64-row tasks (profiles/r01_flat_deep_ring_scan.jsonl).  Shorter
        // packets: a ring of 24 over ~64-row tasks (cfg2 +0.7-1.4 % over 16 in
        // three scans; a ring of 32 cost it 8-15 %).  One task per wave either way.
        const bool jumbo = cpp >= 256;
        const uint32_t flags = g_tune.flags.load();
        const uint32_t loads = g_tune.loads.load() ? g_tune.loads.load() : (jumbo ? 33u : 25u);
        const FlatVariant* fv = &flat_variant(loads);
        const uint32_t rows = (flags >> 8) & 0xFFu ? (flags >> 8) & 0xFFu : (jumbo ? 96u : 46u);
        uint32_t run = std::min(kFlatMaxRun, std::max<uint32_t>(1u, (64u * rows) / cpp));
        // Shorter packets: a multiple of 16 packets per wave task, so a block's
        // results (4 * run u16) are whole 128-B lines (written once, by the
        // block's last wave, see k_flat).  Measured with the sc1 result stores
        // (profiles/r03_flat_rows_scan.jsonl): cfg2 runs 0.884 ms at 32 packets
        // per task (46.5 rows) against 0.906 at 31 and 0.906 at 48; jumbo
        // packets are best at ~10 packets (96 rows), unrounded.
        if (!(flags & kFlatFreeRun) && !jumbo && run >= 12) run = std::min(kFlatMaxRun, (run + 8) / 16 * 16);
        const uint64_t tasks = (n + run - 1) / run;
        const uint32_t grid = grid_for(4, tasks, 0);
        // per-wave partials + the block's results + its completion counter
        const size_t lds = (4u * 64u * flat_pitch(run) + ((4u * run + 1u) & ~1u)) * sizeof(uint16_t) + 16u;
        // the measurement bits (21-23) run k_flat_probe; the production kernel has them compiled out
        const bool probe = (flags & (kLoadsOnly | kNoTaskEnd | kEndNoStore)) && fv->probe && !verify && nt_for(true);
        // the XCD-weighted deal (pipck_tune_xcd_weights): ring 24, checksum, nt loads
        const uint32_t xa = g_xw_kept.load();
        if (xa && !probe && !verify && nt_for(true) && fv->u == 24 && fv->pipe && grid >= 8) {
            const uint64_t P = 8ull * g_xw_period.load(), periods = (grid + xa - 1) / xa;
            PIPCK_LAUNCH((k_flat_xw<24, true, false, true>), dim3((uint32_t)(periods * P)), dim3(256), lds,
                         as_stream(stream), (const uint8_t*)d_arena, cpp, len, n, run, d_pseudo,
                         nf, d_flow_of, flow_origin, d_out, d_ok, flags, d_err);
            PIPCK_LAUNCHED("k_flat_xw");
            return PIPCK_OK;
        }
        PIPCK_LAUNCH(probe ? fv->probe : fv->fn[verify][nt_for(true)], dim3(grid), dim3(256), lds, as_stream(stream),
                           (const uint8_t*)d_arena, cpp, len, n, run, d_pseudo, nf, d_flow_of,
                           flow_origin, d_out, d_ok, flags, d_err);
        PIPCK_LAUNCHED("k_flat");
        return PIPCK_OK;
    }
    // Short aligned strides from 64 B: the row stream with several packets per
    // row (uniform 64/128/512-B packets: 6.0/5.8/6.1 TB/s vs 4.5/4.6/5.5 per
    // packet; below 64 B k_small's lane-per-packet is 3-8 % faster,
    // profiles/r01_ragged_shapes3.jsonl)
    if (aligned && !g_tune.lanes.load() && !(g_tune.flags.load() & kNoFlatSmall) && stride >= 64 && stride < 64 * 16 &&
        len <= stride) {
        const uint32_t cpp = (uint32_t)(stride / 16);
        const uint32_t flags = g_tune.flags.load();
        const uint32_t rows = (flags >> 8) & 0xFFu ? (flags >> 8) & 0xFFu : 64u;
        const uint32_t run = std::min(kFlatSmallMaxRun, std::max<uint32_t>(1u, (64u * rows) / cpp));
        const uint64_t tasks = (n + run - 1) / run;
        PIPCK_LAUNCH(kFlatSmall[verify][nt_for(true)], dim3(grid_for(4, tasks, 0)), dim3(256), 0,
                           as_stream(stream), (const uint8_t*)d_arena, cpp, len, n, run, d_pseudo,
                           nf, d_flow_of, flow_origin, d_out, d_ok, flags, d_err);
        PIPCK_LAUNCHED("k_flat_small");
        return PIPCK_OK;
    }
    // Packed 20/24-byte items with no pseudo-header (IPv4 headers, cfg1): rows
    // of whole headers streamed like the large-packet kernels (pipck_hdr.hip),
    // from 8M headers up: 8.6 % faster than k_small at 256M, 6-11 % at 16M-64M,
    // even at 8M, and slower below (1M: 15.3 vs 12.0 us) where k_small's many
    // tiny waves fill the chip sooner (profiles/r03_hdr_scan.jsonl).
    // pipck_tune loads_per_lane 8/16/24/32 = k_hdr with that ring at any size,
    // 1 = never k_hdr.
    {
        const uint32_t lq = g_tune.loads.load(), flags = g_tune.flags.load();
        // loads_per_lane 8/16/24/32 = one task per wave with that ring, 9/17/25/33 =
        // the block-cooperative row order with ring 8/16/24/32
        const bool force = lq == 8 || lq == 16 || lq == 24 || lq == 32;
        const bool force_coop = lq == 9 || lq == 17 || lq == 25 || lq == 33;
        if (!d_pseudo && (stride == 20 || stride == 24) && !g_tune.lanes.load() && lq != 1 &&
            (force || force_coop || n >= kHdrMinBatch) &&
            launch_hdr(verify, d_arena, stride, len, n, d_out, d_ok, as_stream(stream), (flags >> 8) & 0xFFu,
                       force ? lq : (force_coop ? lq - 1 : 0u), nt_for(true), flags, force_coop) == PIPCK_OK)
            return PIPCK_OK;
    }
    // Tiny 8-B-multiple strides with pseudo-headers (pure ACKs, small UDP) or
    // RX verify: the LDS-staged row stream.  cfg1 on 24-B strides, 256M
    // packets: with IPv4 pseudo-headers 1.29 vs 1.40 ms for k_small (+8.5 %),
    // verify 1.13 vs 1.15 ms; the bare IPv4-header checksum (no pseudo-header)
    // ran 1.24-1.34 vs 1.22 ms, so it stays on k_small
    // (profiles/r01_flat_tiny_scan.jsonl).
    if ((uintptr_t)d_arena % 16 == 0 && stride % 8 == 0 && stride >= 8 && stride <= 8 * kFlatTinyMaxHalves &&
        len >= 1 && len <= stride && (d_pseudo || verify || (g_tune.flags.load() & kForceFlatTiny)) &&
        !g_tune.lanes.load() && !(g_tune.flags.load() & kNoFlatTiny)) {
        const uint32_t hpp = (uint32_t)(stride / 8);
        const uint32_t flags = g_tune.flags.load();
        const uint32_t lq = g_tune.loads.load();
        const int ui = lq == 8 ? 1 : (lq == 16 ? 2 : 0);  // ring of 4 rows by default
        const uint32_t rows = (flags >> 8) & 0xFFu ? (flags >> 8) & 0xFFu : 12u;
        // whole LDS groups per task (so tasks start 1 KiB aligned), ~`rows` rows
        const uint32_t G = tiny_group_rows(hpp), P = G * 128u / hpp;
        const uint32_t run = std::max(1u, std::min(kFlatTinyMaxRun / P, rows / G)) * P;
        const uint64_t tasks = (n + run - 1) / run;
        const size_t lds = 4u * tiny_wave_lds(hpp, run);
        PIPCK_LAUNCH(kFlatTiny[ui][verify][nt_for(true)], dim3(grid_for(4, tasks, 0)), dim3(256), lds,
                           as_stream(stream), (const uint8_t*)d_arena, hpp, len, n, run, d_pseudo,
                           nf, d_flow_of, flow_origin, d_out, d_ok, flags, d_err);
        PIPCK_LAUNCHED("k_flat_tiny");
        return PIPCK_OK;
    }
    // Largest in-chunk offset any packet start can have: starts are
    // arena + i*stride, so their offsets mod 16 step by g = gcd(stride, 16).
    uint32_t g = 16;
    while (g > 1 && stride % g) g >>= 1;
    const uint32_t hmax = (uint32_t)((uintptr_t)d_arena % g) + 16u - g;
    const uint32_t small_nl = (hmax + len + 15u) / 16u;
    if (!g_tune.lanes.load() && !(g_tune.flags.load() & kNoSmall) && small_nl <= 4) {
        const SmallVariant& sv = small_variant();
        const uint64_t waves = (n + 64u * sv.k - 1) / (64u * sv.k);
        PIPCK_LAUNCH(sv.fn[small_nl ? small_nl - 1 : 0][verify][nt_for(false)], dim3((uint32_t)((waves + 3) / 4)), dim3(256), 0,
                           as_stream(stream), (const uint8_t*)d_arena, stride, len, n, d_pseudo,
                           nf, d_flow_of, flow_origin, d_out, d_ok, g_tune.flags.load(), d_err);
        PIPCK_LAUNCHED("k_small");
        return PIPCK_OK;
    }
    const uint32_t nch = (len + (aligned ? 0u : 15u) + 15u) / 16u;
    const Variant& v = pick_variant(nch);
    const uint32_t grid = grid_for(256 / v.g, n);
    PIPCK_LAUNCH(v.fn[verify][nt_for(false)], dim3(grid), dim3(256), 0, as_stream(stream), (const uint8_t*)d_arena,
                       stride, len, n, d_pseudo, nf, d_flow_of, flow_origin, d_out, d_ok, d_err);
    PIPCK_LAUNCHED("k_fixed");
    return PIPCK_OK;
}

template <bool FINAL, int U, bool PIPE, bool NT>
static void launch_ragged_k(bool wide, uint64_t tiles, hipStream_t s, const uint8_t* a, const pipck_desc* d,
                            uint64_t n, const uint32_t* ps, uint16_t* out, uint32_t* fseg, uint8_t* ok, uint32_t* err,
                            uint32_t f, uint64_t ab, uint32_t nf) {
    // one tile per wave: the in-order dispatcher hands out tiles as waves finish
    // (measured best, profiles/r01_size_scan*.jsonl)
    // (runs of 2-4 consecutive tiles per wave measured 2-5 % slower,
    // profiles/r01_ragged_tpw_scan.jsonl)
    if (wide)
        PIPCK_LAUNCH((k_ragged<FINAL, U, PIPE, NT, 4>), dim3(grid_for(4, tiles, 0)),
                           dim3(256), 0, s, a, d, n, ps, out, fseg, ok, err, f, ab, nf);
    else
        PIPCK_LAUNCH((k_ragged<FINAL, U, PIPE, NT, 1>), dim3(grid_for(1, tiles, 0)),
                           dim3(64), 0, s, a, d, n, ps, out, fseg, ok, err, f, ab, nf);
}

template <int U, bool PIPE>
static void launch_ragged_u(bool final_, bool nt, uint64_t tiles, hipStream_t s, const uint8_t* a,
                            const pipck_desc* d, uint64_t n, const uint32_t* ps, uint16_t* out, uint32_t* fseg,
                            uint8_t* ok, uint32_t* err, uint64_t ab, uint32_t nf) {
    const uint32_t f = g_tune.flags.load();
    const bool wide = (f & kWideBlocks) != 0;
    if (final_) {
        if (nt) launch_ragged_k<true, U, PIPE, true>(wide, tiles, s, a, d, n, ps, out, fseg, ok, err, f, ab, nf);
        else launch_ragged_k<true, U, PIPE, false>(wide, tiles, s, a, d, n, ps, out, fseg, ok, err, f, ab, nf);
    } else {
        if (nt) launch_ragged_k<false, U, PIPE, true>(wide, tiles, s, a, d, n, ps, out, fseg, ok, err, f, ab, nf);
        else launch_ragged_k<false, U, PIPE, false>(wide, tiles, s, a, d, n, ps, out, fseg, ok, err, f, ab, nf);
    }
}

// arena_bytes / n_flows bound every descriptor (UINT64_MAX / UINT32_MAX: trusted)
static int launch_ragged(bool final_, const void* d_arena, const pipck_desc* d_desc, uint64_t n,
                         const uint32_t* d_pseudo, uint16_t* d_out, uint32_t* d_fseg, uint8_t* d_ok, uint32_t* d_err,
                         hipStream_t s, uint64_t arena_bytes, uint32_t n_flows) {
    if (final_ && !d_fseg && g_tune.lanes.load() == kWaveArm)  // measurement arm: one packet per wave
        return launch_wave(d_ok != nullptr, true, d_arena, 0, 0, d_desc, n, d_pseudo, n_flows, nullptr, 0, d_out, d_ok,
                           d_err, s, 0, g_tune.loads.load() ? g_tune.loads.load() : 4u, arena_bytes);
    const uint64_t tiles = (n + 63) / 64;
    // loads_per_lane: 2/4/8/16 rows in flight on packed tiles (at most 4 on
    // others), 3/5/7/9/13/17/25/33 = ring-pipelined 2/4/6/8/12/16/24/32.
    // Default: ring of 24 (cfg4: ring 12 +2.5 % over plain 4,
    // profiles/r01_ragged_ring_scan.jsonl; ring 24 +1.4 % over 12/16 and ring
    // 32 -14 %, r01_deep_ring_scan.jsonl)
    const uint32_t u = g_tune.loads.load() ? g_tune.loads.load() : 25u;
    const bool nt = nt_for(true);
    const uint8_t* a = (const uint8_t*)d_arena;
    switch (u) {
        case 2: launch_ragged_u<2, false>(final_, nt, tiles, s, a, d_desc, n, d_pseudo, d_out, d_fseg, d_ok, d_err, arena_bytes, n_flows); break;
        case 4: launch_ragged_u<4, false>(final_, nt, tiles, s, a, d_desc, n, d_pseudo, d_out, d_fseg, d_ok, d_err, arena_bytes, n_flows); break;
        case 8: launch_ragged_u<8, false>(final_, nt, tiles, s, a, d_desc, n, d_pseudo, d_out, d_fseg, d_ok, d_err, arena_bytes, n_flows); break;
        case 16: launch_ragged_u<16, false>(final_, nt, tiles, s, a, d_desc, n, d_pseudo, d_out, d_fseg, d_ok, d_err, arena_bytes, n_flows); break;
        case 3: launch_ragged_u<2, true>(final_, nt, tiles, s, a, d_desc, n, d_pseudo, d_out, d_fseg, d_ok, d_err, arena_bytes, n_flows); break;
        case 9: launch_ragged_u<8, true>(final_, nt, tiles, s, a, d_desc, n, d_pseudo, d_out, d_fseg, d_ok, d_err, arena_bytes, n_flows); break;
        case 7: launch_ragged_u<6, true>(final_, nt, tiles, s, a, d_desc, n, d_pseudo, d_out, d_fseg, d_ok, d_err, arena_bytes, n_flows); break;
        case 13: launch_ragged_u<12, true>(final_, nt, tiles, s, a, d_desc, n, d_pseudo, d_out, d_fseg, d_ok, d_err, arena_bytes, n_flows); break;
        case 17: launch_ragged_u<16, true>(final_, nt, tiles, s, a, d_desc, n, d_pseudo, d_out, d_fseg, d_ok, d_err, arena_bytes, n_flows); break;
        case 25: launch_ragged_u<24, true>(final_, nt, tiles, s, a, d_desc, n, d_pseudo, d_out, d_fseg, d_ok, d_err, arena_bytes, n_flows); break;
        case 33: launch_ragged_u<32, true>(final_, nt, tiles, s, a, d_desc, n, d_pseudo, d_out, d_fseg, d_ok, d_err, arena_bytes, n_flows); break;
        default: launch_ragged_u<4, true>(final_, nt, tiles, s, a, d_desc, n, d_pseudo, d_out, d_fseg, d_ok, d_err, arena_bytes, n_flows); break;
    }
    PIPCK_LAUNCHED("k_ragged");
    return PIPCK_OK;
}

template <bool V, int U>
static void launch_packed_u(bool nt, uint64_t tiles, hipStream_t s, const uint8_t* a, const uint16_t* lens,
                            const uint64_t* tc, uint64_t n, const uint32_t* ps, uint32_t nf, const uint32_t* fo,
                            uint64_t origin, uint16_t* out, uint8_t* ok, uint32_t f, uint64_t ach, uint32_t* err) {
    const bool marks = (f & kPackedMarksOnly) != 0;
    if (nt && marks)
        PIPCK_LAUNCH((k_packed<V, U, true, true>), dim3((uint32_t)tiles), dim3(64), 0, s, a, lens, tc, n, ps, nf,
                           fo, origin, out, ok, f, ach, err);
    else if (nt)
        PIPCK_LAUNCH((k_packed<V, U, true, false>), dim3((uint32_t)tiles), dim3(64), 0, s, a, lens, tc, n, ps, nf,
                           fo, origin, out, ok, f, ach, err);
    else if (marks)
        PIPCK_LAUNCH((k_packed<V, U, false, true>), dim3((uint32_t)tiles), dim3(64), 0, s, a, lens, tc, n, ps, nf,
                           fo, origin, out, ok, f, ach, err);
    else
        PIPCK_LAUNCH((k_packed<V, U, false, false>), dim3((uint32_t)tiles), dim3(64), 0, s, a, lens, tc, n, ps, nf,
                           fo, origin, out, ok, f, ach, err);
}

// bounded: the _n forms (flow_of entries bounded by n_flows when it is given)
static int launch_packed(bool verify, const void* d_arena, uint64_t arena_bytes, const uint16_t* d_lens,
                         const uint64_t* d_tile_chunk, uint64_t n, const uint32_t* d_pseudo, uint32_t n_flows,
                         const uint32_t* d_flow_of, uint64_t flow_origin, uint16_t* d_out, uint8_t* d_ok,
                         uint32_t* d_err, hipStream_t s, bool bounded = true) {
    if (n == 0) return PIPCK_OK;
    if (!d_arena || !d_lens || !d_tile_chunk || (verify ? !d_ok : !d_out)) {
        set_error("pipck_checksum_packed: null pointer");
        return PIPCK_EINVAL;
    }
    if ((uintptr_t)d_arena % 16) {
        set_error("pipck_checksum_packed: the arena must be 16-byte aligned");
        return PIPCK_EINVAL;
    }
    if (d_pseudo && !d_flow_of && n_flows == 0) {
        set_error("pipck_checksum_packed: n_flows == 0");
        return PIPCK_EINVAL;
    }
    const uint64_t tiles = (n + 63) / 64;
    if (tiles > 0x7FFFFFFFull) {
        set_error("pipck_checksum_packed: more than 2^37 packets in one launch");
        return PIPCK_ERANGE;
    }
    // whole 16-byte chunks the kernel may read: the arena's bytes rounded up to 16
    const uint64_t ach = arena_bytes / 16 + (arena_bytes % 16 ? 1u : 0u);
    // Mixed rows take the LDS-marks path by default here (tune flags bit 19
    // selects the scalar end loop instead, the reverse of k_ragged), with a
    // ring of 32 rows (154 VGPRs, still 3 waves/SIMD): cfg4 1.2618 vs 1.2814 ms and, at 16M
    // packets, 2.448 vs 2.518 ms against the ring of 24 with the end loop, each
    // alone gaining less (profiles/r02_knob_scan_cfg4_packed.jsonl).
    const uint32_t f = g_tune.flags.load() ^ kPackedMarksOnly;
    const bool nt = nt_for(true);
    const uint8_t* a = (const uint8_t*)d_arena;
    // the kernel's n_flows: the modulus without flow_of; with it, the bound of its entries
    const uint32_t nf = d_flow_of ? (bounded && n_flows ? n_flows : UINT32_MAX) : (n_flows ? n_flows : 1u);
    // rows in flight per wave: 17/25/33 = rings of 16/24/32
    switch (g_tune.loads.load()) {
        case 17: verify ? launch_packed_u<true, 16>(nt, tiles, s, a, d_lens, d_tile_chunk, n, d_pseudo, nf, d_flow_of, flow_origin, d_out, d_ok, f, ach, d_err)
                        : launch_packed_u<false, 16>(nt, tiles, s, a, d_lens, d_tile_chunk, n, d_pseudo, nf, d_flow_of, flow_origin, d_out, d_ok, f, ach, d_err);
                 break;
        case 25: verify ? launch_packed_u<true, 24>(nt, tiles, s, a, d_lens, d_tile_chunk, n, d_pseudo, nf, d_flow_of, flow_origin, d_out, d_ok, f, ach, d_err)
                        : launch_packed_u<false, 24>(nt, tiles, s, a, d_lens, d_tile_chunk, n, d_pseudo, nf, d_flow_of, flow_origin, d_out, d_ok, f, ach, d_err);
                 break;
        default: verify ? launch_packed_u<true, 32>(nt, tiles, s, a, d_lens, d_tile_chunk, n, d_pseudo, nf, d_flow_of, flow_origin, d_out, d_ok, f, ach, d_err)
                        : launch_packed_u<false, 32>(nt, tiles, s, a, d_lens, d_tile_chunk, n, d_pseudo, nf, d_flow_of, flow_origin, d_out, d_ok, f, ach, d_err);
                 break;
    }
    PIPCK_LAUNCHED("k_packed");
    return PIPCK_OK;
}

int chains_unchecked(const void* d_arena, const pipck_desc* d_segs, uint64_t n_segs, const uint64_t* d_seg_begin,
                     const uint32_t* d_pkt_flow, uint64_t n_packets, const uint32_t* d_pseudo, uint32_t* d_scratch,
                     uint16_t* d_out, uint32_t* d_err, hipStream_t s, uint64_t arena_bytes, uint32_t n_flows) {
    if (n_segs) {
        int rc = launch_ragged(false, d_arena, d_segs, n_segs, nullptr, nullptr, d_scratch, nullptr, d_err, s,
                               arena_bytes, UINT32_MAX);
        if (rc) return rc;
    }
    const uint64_t blocks = (n_packets + 255) / 256;
    if (blocks > 0x7FFFFFFFull) {
        set_error("pipck_checksum_chains: too many packets for one launch");
        return PIPCK_ERANGE;
    }
    hipLaunchKernelGGL(k_chain_finish, dim3((uint32_t)blocks), dim3(256), 0, s, d_seg_begin, d_pkt_flow, n_packets,
                       d_pseudo, d_scratch, d_out, n_segs, n_flows, d_err);
    PIPCK_LAUNCHED("k_chain_finish");
    return PIPCK_OK;
}

}  // namespace pipck

using namespace pipck;

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

uint32_t pipck_version(void) { return ((uint32_t)PIPCK_VERSION_MAJOR << 16) | PIPCK_VERSION_MINOR; }

void pipck_tune(uint32_t lanes_per_packet, uint32_t loads_per_lane, uint32_t blocks, uint32_t flags) {
    g_tune.lanes.store(lanes_per_packet);
    g_tune.loads.store(loads_per_lane);
    g_tune.blocks.store(blocks);
    g_tune.flags.store(flags);
}

int pipck_last_launch(char* buf, size_t cap) {
    // the handle of a __global__ function is a symbol with the kernel's own
    // mangled name; demangled, it reads exactly as rocprofv3 names the kernel
    if (!buf || !cap) return PIPCK_EINVAL;
    buf[0] = 0;
    Dl_info info;
    if (!t_last_kernel || !dladdr(t_last_kernel, &info) || !info.dli_sname || info.dli_saddr != t_last_kernel) {
        set_error("pipck_last_launch: no batch launch on this thread, or its symbol is not exported");
        return PIPCK_EINVAL;
    }
    int st = 0;
    char* dem = abi::__cxa_demangle(info.dli_sname, nullptr, nullptr, &st);
    const char* name = st == 0 && dem ? dem : info.dli_sname;
    const size_t len = std::strlen(name);
    const int rc = len < cap ? PIPCK_OK : PIPCK_ERANGE;
    std::memcpy(buf, name, std::min(len, cap - 1));
    buf[std::min(len, cap - 1)] = 0;
    std::free(dem);
    if (rc) set_error("pipck_last_launch: buffer too small");
    return rc;
}

void pipck_tune_probes(uint32_t probes) { g_probes.store(probes); }

int pipck_tune_xcd_weights(const uint32_t* m, uint32_t period) {
    uint32_t w[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t kept = 0;
    if (m && period) {
        if (period > 4096) return PIPCK_EINVAL;
        for (int x = 0; x < 8; x++) {
            if (m[x] > period) return PIPCK_EINVAL;
            w[x] = m[x];
            kept += m[x];
        }
        if (!kept) return PIPCK_EINVAL;
        w[8] = period;
    }
    PIPCK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_xw), w, sizeof w));
    g_xw_period.store(w[8]);
    g_xw_kept.store(kept);
    return PIPCK_OK;
}

int pipck_trace_tasks(void* d_buf, uint64_t cap) {
    // d_buf: device memory for cap 32-byte records (null: off); the tasks of a
    // launch made with tune flags bit 20 land at their task index
    TaskTrace* p = (TaskTrace*)d_buf;
    const uint64_t c = d_buf ? cap : 0;
    PIPCK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &p, sizeof p));
    PIPCK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_trace_cap), &c, sizeof c));
    return PIPCK_OK;
}

int pipck_flows4_prepare(const pipck_flow4* d_flows, uint32_t n, uint32_t* d_pseudo, void* stream) {
    if (!n) return PIPCK_OK;
    if (!d_flows || !d_pseudo) {
        set_error("pipck_flows4_prepare: null pointer");
        return PIPCK_EINVAL;
    }
    hipLaunchKernelGGL(k_flows4, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream), d_flows, n, d_pseudo);
    PIPCK_LAUNCHED("k_flows4");
    return PIPCK_OK;
}

int pipck_flows6_prepare(const pipck_flow6* d_flows, uint32_t n, uint32_t* d_pseudo, void* stream) {
    if (!n) return PIPCK_OK;
    if (!d_flows || !d_pseudo) {
        set_error("pipck_flows6_prepare: null pointer");
        return PIPCK_EINVAL;
    }
    hipLaunchKernelGGL(k_flows6, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream), d_flows, n, d_pseudo);
    PIPCK_LAUNCHED("k_flows6");
    return PIPCK_OK;
}

int pipck_checksum_fixed_n(const void* d_arena, uint64_t stride, uint32_t len, uint64_t n, const uint32_t* d_pseudo,
                           uint32_t n_flows, const uint32_t* d_flow_of, uint64_t flow_origin, uint16_t* d_out,
                           uint32_t* d_err, void* stream) {
    return launch_fixed(false, d_arena, stride, len, n, d_pseudo, n_flows, d_flow_of, flow_origin, d_out, nullptr,
                        d_err, stream, true);
}

int pipck_verify_fixed_n(const void* d_arena, uint64_t stride, uint32_t len, uint64_t n, const uint32_t* d_pseudo,
                         uint32_t n_flows, const uint32_t* d_flow_of, uint64_t flow_origin, uint8_t* d_ok,
                         uint32_t* d_err, void* stream) {
    return launch_fixed(true, d_arena, stride, len, n, d_pseudo, n_flows, d_flow_of, flow_origin, nullptr, d_ok,
                        d_err, stream, true);
}

// the unbounded forms (flow_of entries trusted, n_flows unused with them)
int pipck_checksum_fixed(const void* d_arena, uint64_t stride, uint32_t len, uint64_t n, const uint32_t* d_pseudo,
                         uint32_t n_flows, const uint32_t* d_flow_of, uint64_t flow_origin, uint16_t* d_out,
                         void* stream) {
    return launch_fixed(false, d_arena, stride, len, n, d_pseudo, n_flows, d_flow_of, flow_origin, d_out, nullptr,
                        nullptr, stream, false);
}

int pipck_verify_fixed(const void* d_arena, uint64_t stride, uint32_t len, uint64_t n, const uint32_t* d_pseudo,
                       uint32_t n_flows, const uint32_t* d_flow_of, uint64_t flow_origin, uint8_t* d_ok,
                       void* stream) {
    return launch_fixed(true, d_arena, stride, len, n, d_pseudo, n_flows, d_flow_of, flow_origin, nullptr, d_ok,
                        nullptr, stream, false);
}

int pipck_checksum_ragged_n(const void* d_arena, uint64_t arena_bytes, const pipck_desc* d_desc, uint64_t n,
                            const uint32_t* d_pseudo, uint32_t n_flows, uint16_t* d_out, uint32_t* d_err,
                            void* stream) {
    if (n == 0) return PIPCK_OK;
    if (!d_arena || !d_desc || !d_out) {
        set_error("pipck_checksum_ragged: null pointer");
        return PIPCK_EINVAL;
    }
    if (d_pseudo && n_flows == 0) {
        set_error("pipck_checksum_ragged_n: n_flows == 0");
        return PIPCK_EINVAL;
    }
    return launch_ragged(true, d_arena, d_desc, n, d_pseudo, d_out, nullptr, nullptr, d_err, as_stream(stream),
                         arena_bytes, n_flows);
}

int pipck_verify_ragged_n(const void* d_arena, uint64_t arena_bytes, const pipck_desc* d_desc, uint64_t n,
                          const uint32_t* d_pseudo, uint32_t n_flows, uint8_t* d_ok, uint32_t* d_err, void* stream) {
    if (n == 0) return PIPCK_OK;
    if (!d_arena || !d_desc || !d_ok) {
        set_error("pipck_verify_ragged: null pointer");
        return PIPCK_EINVAL;
    }
    if (d_pseudo && n_flows == 0) {
        set_error("pipck_verify_ragged_n: n_flows == 0");
        return PIPCK_EINVAL;
    }
    return launch_ragged(true, d_arena, d_desc, n, d_pseudo, nullptr, nullptr, d_ok, d_err, as_stream(stream),
                         arena_bytes, n_flows);
}

// the unbounded forms (descriptors and flows trusted)
int pipck_checksum_ragged(const void* d_arena, const pipck_desc* d_desc, uint64_t n, const uint32_t* d_pseudo,
                          uint16_t* d_out, uint32_t* d_err, void* stream) {
    return pipck_checksum_ragged_n(d_arena, UINT64_MAX, d_desc, n, d_pseudo, UINT32_MAX, d_out, d_err, stream);
}

int pipck_verify_ragged(const void* d_arena, const pipck_desc* d_desc, uint64_t n, const uint32_t* d_pseudo,
                        uint8_t* d_ok, uint32_t* d_err, void* stream) {
    return pipck_verify_ragged_n(d_arena, UINT64_MAX, d_desc, n, d_pseudo, UINT32_MAX, d_ok, d_err, stream);
}

int pipck_checksum_packed_n(const void* d_arena, uint64_t arena_bytes, const uint16_t* d_lens,
                            const uint64_t* d_tile_chunk, uint64_t n, const uint32_t* d_pseudo, uint32_t n_flows,
                            const uint32_t* d_flow_of, uint64_t flow_origin, uint16_t* d_out, uint32_t* d_err,
                            void* stream) {
    return launch_packed(false, d_arena, arena_bytes, d_lens, d_tile_chunk, n, d_pseudo, n_flows, d_flow_of,
                         flow_origin, d_out, nullptr, d_err, as_stream(stream));
}

int pipck_verify_packed_n(const void* d_arena, uint64_t arena_bytes, const uint16_t* d_lens,
                          const uint64_t* d_tile_chunk, uint64_t n, const uint32_t* d_pseudo, uint32_t n_flows,
                          const uint32_t* d_flow_of, uint64_t flow_origin, uint8_t* d_ok, uint32_t* d_err,
                          void* stream) {
    return launch_packed(true, d_arena, arena_bytes, d_lens, d_tile_chunk, n, d_pseudo, n_flows, d_flow_of,
                         flow_origin, nullptr, d_ok, d_err, as_stream(stream));
}

// the unbounded forms (the index is trusted): every tile's chunks must lie in the arena
int pipck_checksum_packed(const void* d_arena, const uint16_t* d_lens, const uint64_t* d_tile_chunk, uint64_t n,
                          const uint32_t* d_pseudo, uint32_t n_flows, const uint32_t* d_flow_of, uint64_t flow_origin,
                          uint16_t* d_out, void* stream) {
    return launch_packed(false, d_arena, UINT64_MAX, d_lens, d_tile_chunk, n, d_pseudo, n_flows, d_flow_of,
                         flow_origin, d_out, nullptr, nullptr, as_stream(stream), false);
}

int pipck_verify_packed(const void* d_arena, const uint16_t* d_lens, const uint64_t* d_tile_chunk, uint64_t n,
                        const uint32_t* d_pseudo, uint32_t n_flows, const uint32_t* d_flow_of, uint64_t flow_origin,
                        uint8_t* d_ok, void* stream) {
    return launch_packed(true, d_arena, UINT64_MAX, d_lens, d_tile_chunk, n, d_pseudo, n_flows, d_flow_of,
                         flow_origin, nullptr, d_ok, nullptr, as_stream(stream), false);
}

int pipck_packed_index(const uint16_t* d_lens, uint64_t n, uint64_t* d_tile_chunk, void* stream) {
    if (!d_tile_chunk || (n && !d_lens)) {
        set_error("pipck_packed_index: null pointer");
        return PIPCK_EINVAL;
    }
    const uint64_t tiles = (n + 63) / 64;
    if (tiles > 0x7FFFFFFFull) {
        set_error("pipck_packed_index: more than 2^37 packets");
        return PIPCK_ERANGE;
    }
    hipStream_t s = as_stream(stream);
    if (tiles) {
        hipLaunchKernelGGL(k_packed_tile_sums, dim3((uint32_t)tiles), dim3(64), 0, s, d_lens, n, d_tile_chunk);
        PIPCK_LAUNCHED("k_packed_tile_sums");
    }
    hipLaunchKernelGGL(k_packed_tile_scan, dim3(1), dim3(1024), 0, s, d_tile_chunk, tiles);
    PIPCK_LAUNCHED("k_packed_tile_scan");
    return PIPCK_OK;
}

int pipck_checksum_chains_n(const void* d_arena, uint64_t arena_bytes, const pipck_desc* d_segs, uint64_t n_segs,
                            const uint64_t* d_seg_begin, const uint32_t* d_pkt_flow, uint64_t n_packets,
                            const uint32_t* d_pseudo, uint32_t n_flows, uint32_t* d_scratch, uint16_t* d_out,
                            uint32_t* d_err, void* stream) {
    if (n_packets == 0) return PIPCK_OK;
    if (!d_seg_begin || !d_out || (n_segs && (!d_arena || !d_segs || !d_scratch))) {
        set_error("pipck_checksum_chains: null pointer");
        return PIPCK_EINVAL;
    }
    if (d_pseudo && n_flows == 0) {
        set_error("pipck_checksum_chains_n: n_flows == 0");
        return PIPCK_EINVAL;
    }
    return chains_unchecked(d_arena, d_segs, n_segs, d_seg_begin, d_pkt_flow, n_packets, d_pseudo, d_scratch, d_out,
                            d_err, as_stream(stream), arena_bytes, n_flows);
}

// segments and flows trusted (segment ranges are still bounded by n_segs)
int pipck_checksum_chains(const void* d_arena, const pipck_desc* d_segs, uint64_t n_segs, const uint64_t* d_seg_begin,
                          const uint32_t* d_pkt_flow, uint64_t n_packets, const uint32_t* d_pseudo,
                          uint32_t* d_scratch, uint16_t* d_out, uint32_t* d_err, void* stream) {
    return pipck_checksum_chains_n(d_arena, UINT64_MAX, d_segs, n_segs, d_seg_begin, d_pkt_flow, n_packets, d_pseudo,
                                   UINT32_MAX, d_scratch, d_out, d_err, stream);
}

}  // extern "C"
