// pipck_rxdev.hip -- RX verification of received IP packets already in device
// memory (SURVEY.md section 8 f2 at HBM rate; pipck_rx_verify_device).
//
// pipck_rx_verify (pipck_rx.hip) takes packets in host memory: the host parses
// what each checksum covers and the GPU reads the bytes over PCIe (~50 GB/s).
// Packets that already sit in HBM -- a receive ring filled by a peer device,
// a capture replayed from device memory -- need no host at all.  They come in
// the byte-packed layout of pipck_checksum_packed_bytes (packets back to back,
// u16 lengths, a u64 byte offset per 64 packets) and are verified in ONE pass
// of k_packedb_rx, the cfg4 bench kernel's body (k_packedb) with RX = true:
//
//  1. the tile's stream, unchanged, leaves each packet's folded big-endian sum
//     S_all over its whole frame, relative to the packet's first byte;
//  2. while the rows stream by, the chunks of every packet's header window
//     (its first six aligned 16-byte chunks) are also copied to LDS; at the
//     tile's end each lane takes its packet's window from there (rx_from_window,
//     pipck_rxparse.hpp), realigns it to the packet start in registers, parses
//     the fields pipck_rx_verify's host parser reads (rx_parse: IHL, lengths,
//     fragment field, protocol, the IPv6 extension-header walk, addresses),
//     sums the IPv4 header exactly, and gets the L4 message's sum without
//     reading it again: S_l4 = S_all - S_pre - S_post (mod 0xFFFF), where
//     S_pre covers the bytes before the L4 message (IP header and extension
//     headers) and S_post the link padding after the IP length.
//
// Why the subtraction is exact: every sum here is taken
// relative to the packet's first byte, so sums of disjoint byte ranges add
// mod 0xFFFF; pip's verdict for a payload with its checksum field included is
// fold(fold(P + T)) == 0xFFFF with T the message's big-endian sum, which for
// P > 0 (TCP, UDP, ICMPv6: the protocol number is in P) depends only on
// (P + T) mod 0xFFFF.  ICMPv4 has no pseudo-header (P = 0): there "T = 0"
// (an all-zero message, whose correct checksum is 0xFFFF, not 0) must be told
// apart from T = k x 0xFFFF, so the kernel checks the message for a non-zero
// byte (its first 8 bytes from registers, the rest only if those are zero).
#include "pipck_common.hpp"
#include "pipck_rxparse.hpp"

#include <algorithm>
#include <atomic>
#include <mutex>
#include <vector>

namespace pipck {

// ---- frames in fixed-size slots (a receive ring: slot i at arena + i * stride,
// lens[i] bytes of frame in it, the rest of the slot unused) -----------------
// A slot length is written by whoever filled the ring (a peer device, a NIC, a
// tun reader: pip itself trusts the IP lengths of what recv() gave it,
// pip/pip_netif.cpp:45-77), so every ring kernel bounds it by the slot: a slot
// claiming more than slot_stride bytes is not read at all, gets verdict 0 and
// sets (1 << PIPCK_ERANGE) in err -- no load, and no parse read, leaves its slot.
//
// Three schedules (launch_ring_rx picks; all give the same verdicts):
//  * k_ring (the default, below k_ring_slots): slot groups, each wave choosing
//    per its own slots' lengths;
//  * k_ring_rx: a row stream over whole slots (tune flag bit 28);
//  * k_ring_slots: slot by slot, a wave per slot (the wave-per-packet arm).
//
// k_ring_rx (the row stream)
// streams the slots like k_flat_coop (pipck_coop.hip): a block task
// of K whole slots, its four waves on interleaved 1 KiB rows, a ring of U rows
// per wave, one LDS partial per lane per slot.  Unlike k_flat_coop each lane's
// load is predicated on the chunk lying inside its slot's frame (the slot's
// length from LDS), so the unused part of a slot is never read -- a sparse ring
// (short frames in jumbo slots) costs its frame bytes, not its slot bytes.  Each
// slot's first six chunks (its header window; slots are 16-byte aligned) are
// copied to LDS on the way, and at the task's end thread j judges slot j with
// rx_from_window (pipck_rxparse.hpp) from the frame's sum and that window.
constexpr int kRingU = 24;

__host__ __device__ constexpr uint32_t ring_pitch(uint32_t k) { return k | 1u; }

// ---- the schedule's feedback (jumbo slots: k_ring or the row stream) --------
// k_ring keeps 8 waves per SIMD, which sparse and short rings need; full jumbo
// slots stream 3 % faster through the row stream at 3 waves per SIMD
// (DESIGN.md section 9 f2), and a kernel's register budget is fixed at launch
// while a ring's fill is not.  A ring buffer is verified again and again, so
// each launch reports how full it was and the next launches of the same ring
// take the schedule that fits: a sample of the blocks evaluates ring_dense on
// its slots and adds it to a device counter (every-th block: ~64 reporters per
// launch, spread over the ring); the last to arrive writes
// {seq, dense, reporting blocks} into pinned host memory, where launch_ring_rx
// reads it for the following calls.  Speed only: both kernels give the same
// verdicts, and a report that two overlapping calls mixed only mixes the
// heuristic.
constexpr uint32_t kFbReports = 64;  // reporting blocks per launch (at most)
struct RingFb {
    unsigned long long* ctr;  // device: (dense << 32) | arrived; the last to arrive resets it
    uint32_t* host;           // pinned, coherent: {seq, dense, reported}
    uint32_t every;           // blocks with blockIdx % every == 0 report
    uint32_t parts;           // reporting blocks in this launch
    uint32_t seq;
};
static inline void fb_sample(RingFb& fb, uint64_t blocks) {
    fb.every = (uint32_t)std::max<uint64_t>(1, blocks / kFbReports);
    fb.parts = (uint32_t)((blocks + fb.every - 1) / fb.every);
}
// 64 slots are dense when the 1 KiB rows holding frame bytes (T) are at least
// 3/4 of the rows of their slots -- full jumbo slots
__device__ __forceinline__ bool ring_dense(uint32_t T, uint32_t nb, uint32_t stride) {
    return 4u * T >= 3u * nb * ((stride + 1023u) >> 10);
}
// lane 0 of one wave of a reporting block: count its verdict, and the last
// reporter publishes the launch's total (vector atomics and stores only)
__device__ __forceinline__ void ring_report(const RingFb& fb, bool dense, int lane) {
    if (lane != 0) return;
    const unsigned long long old = atomicAdd(fb.ctr, ((unsigned long long)(dense ? 1u : 0u) << 32) | 1ull);
    if ((uint32_t)old + 1u >= fb.parts) {  // the last reporter (or a count an overlapping call left)
        atomicExch(fb.ctr, 0ull);
        __hip_atomic_store(fb.host + 1, (uint32_t)(old >> 32) + (dense ? 1u : 0u), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(fb.host + 2, (uint32_t)old + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(fb.host, fb.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void k_ring_rx(
    const uint8_t* __restrict__ arena, uint32_t cpp, const uint16_t* __restrict__ lens, uint64_t n, uint32_t K,
    uint8_t* __restrict__ ok, uint32_t* __restrict__ err, RingFb fb) {
    extern __shared__ uint32_t s_ring[];  // part[64][pitch] | len[K] | hdr[6][K] (u32x4), launch_ring_rx sizes it
    const uint32_t pitch = ring_pitch(K);
    uint32_t* s_part = s_ring;
    uint32_t* s_len = s_part + 64u * pitch;
    u32x4* hdr = reinterpret_cast<u32x4*>(s_len + ((K + 3u) & ~3u));
    const int lane = threadIdx.x & 63;
    const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint64_t p0 = (uint64_t)blockIdx.x * K;
    const uint32_t np = (uint32_t)min<uint64_t>((uint64_t)K, n - p0);
    const uint32_t rows = (np * cpp + 63u) >> 6;
    for (uint32_t i = threadIdx.x; i < 64u * pitch; i += 256) s_part[i] = 0;
    for (uint32_t i = threadIdx.x; i < K; i += 256) {
        const uint32_t L = i < np ? (uint32_t)lens[p0 + i] : 0u;
        s_len[i] = L > 16u * cpp ? 0u : L;  // longer than its slot: not read (judged at the end)
    }
    __syncthreads();
    const buf_t tb = buf_rsrc(arena + p0 * cpp * 16u, np * cpp * 16u);
    uint32_t* part = s_part + lane * pitch;
    // this wave's rows w, w+4, ...: lane 0's slot and chunk-in-slot, advanced by
    // 256 chunks (q slots + rm chunks) per row, for the row consumed and for the
    // row loaded U rows ahead
    const uint32_t q = 256u / cpp, rm = 256u % cpp;
    uint32_t pkt = (64u * w) / cpp, k0 = (64u * w) % cpp;
    uint32_t lpkt = pkt, lk0 = k0;
    const uint32_t my_rows = rows > w ? (rows - w + 3) >> 2 : 0u;
    auto step = [&](uint32_t& pk, uint32_t& kk) {
        kk += rm;
        pk += q;
        if (kk >= cpp) {
            kk -= cpp;
            pk++;
        }
    };
    // the load of row j of this wave, only where the chunk lies in its frame
    auto load = [&](uint32_t j) -> u32x4 {
        uint32_t k = lk0 + (uint32_t)lane, pk = lpkt;
        if (k >= cpp) {
            k -= cpp;
            pk++;
        }
        const uint32_t L = pk < np ? s_len[pk] : 0u;
        // past the frame: an offset beyond the resource, which reads zeros with
        // no memory request (a predicated load would make every row wait vmcnt(0))
        // (skipping the load of a row past every frame, a wave-uniform branch,
        // turned every wait of the ring into vmcnt(0): the load always issues)
        return buf_load<true>(tb, 16u * k < L ? ((w + 4u * j) * 64u + (uint32_t)lane) * 16u : 0xFFFFFFF0u);
    };
    u32x4 v[kRingU];
#pragma unroll
    for (int u = 0; u < kRingU; u++) {
        v[u] = load((uint32_t)u);
        step(lpkt, lk0);
    }
    for (uint32_t j0 = 0; j0 < my_rows; j0 += kRingU) {
#pragma unroll
        for (int u = 0; u < kRingU; u++) {
            const uint32_t j = j0 + u;
            if (j < my_rows) {  // wave-uniform
                uint32_t k = k0 + (uint32_t)lane, pk = pkt;
                if (k >= cpp) {
                    k -= cpp;
                    pk++;
                }
                const uint32_t L = pk < np ? s_len[pk] : 0u;
                // only chunks inside a frame add anything: a row past every
                // lane's frame (most rows of a sparse ring) does no LDS work
                if (16u * k < L) {
                    u32x4 x = v[u];
                    if (16u * k + 16u > L) x = mask_tail(x, (int)(L - 16u * k));
                    atomicAdd(&part[pk], dot4(x, 0u));
                    if (k < 6u) hdr[k * K + pk] = x;  // the slot's header window
                }
                step(pkt, k0);
            }
            v[u] = load(j + kRingU);  // past the task: the resource's range check reads nothing
            step(lpkt, lk0);
        }
    }
    __syncthreads();
    const uint32_t i = threadIdx.x;
    if (i < np) {
        uint32_t s = 0;
#pragma unroll 16
        for (int l = 0; l < 64; l++) s += s_part[l * pitch + i];
        const uint32_t L = s_len[i];
        const uint32_t F = bswap16(fold16(s));  // slots start 16-byte aligned: even address
        uint32_t hw[24];
#pragma unroll
        for (int k = 0; k < 6; k++) {  // chunks past the frame were never captured: zero
            const u32x4 x = 16u * k < L ? hdr[k * K + i] : u32x4{0u, 0u, 0u, 0u};
            hw[4 * k] = x.x, hw[4 * k + 1] = x.y, hw[4 * k + 2] = x.z, hw[4 * k + 3] = x.w;
        }
        const uint8_t* pkp = arena + (p0 + i) * cpp * 16u;
        const bool bad = (uint32_t)lens[p0 + i] > 16u * cpp;
        if (bad && err) atomicOr(err, 1u << PIPCK_ERANGE);
        store_result8(buf_rsrc(ok + p0, np), i, bad ? 0u : rx_from_window(pkp, L, F, hw));
    }
    // the feedback (launch_ring_rx passes it for jumbo slots only, where K <= 64)
    if (fb.ctr && blockIdx.x % fb.every == 0 && w == 0) {
        const uint32_t Ls = (uint32_t)lane < np ? s_len[lane] : 0u;  // refused slots: 0
        ring_report(fb, ring_dense(wave_total((Ls + 1023u) >> 10), np, 16u * cpp), lane);
    }
}

// ---- the same ring, slot by slot (sparse rings: short frames in large slots) --
// k_ring_rx walks every row of every slot: a row past every lane's frame still
// issues its (range-checked, request-free) load and index math, so a ring of
// ~1 KB frames in 9,216-B slots costs the slot rows, not the frame bytes.
// k_ring_slots gives each wave kSlotG slots and touches only each frame's
// chunks: the first row (64 chunks = 1 KiB) of all kSlotG frames is in flight
// at once, a frame longer than 1 KiB then streams its further rows 4 at a time,
// and one wave reduce per slot gives its sum.  Lanes 0-5 of the first row are
// the header window; the block's 32 slots are judged by its first 32 threads.
// The round-4 default, now a measurement arm (the wave-per-packet tune arm).
constexpr int kSlotG = 8;

__global__ __launch_bounds__(256) void k_ring_slots(const uint8_t* __restrict__ arena, uint32_t cpp,
                                                    const uint16_t* __restrict__ lens, uint64_t n,
                                                    uint8_t* __restrict__ ok, uint32_t* __restrict__ err) {
    __shared__ u32x4 s_hdr[6][4 * kSlotG];
    __shared__ uint32_t s_sum[4 * kSlotG], s_len[4 * kSlotG];
    const int lane = threadIdx.x & 63;
    const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint64_t b0 = (uint64_t)blockIdx.x * (4u * kSlotG);
    const uint64_t p0 = b0 + w * kSlotG;  // this wave's first slot
    const uint32_t lmine = (lane < kSlotG && p0 + (uint32_t)lane < n) ? (uint32_t)lens[p0 + lane] : 0u;
    uint32_t L[kSlotG], Lc[kSlotG];
    buf_t r[kSlotG];
    u32x4 v[kSlotG];
#pragma unroll
    for (int g = 0; g < kSlotG; g++) {
        L[g] = (uint32_t)__builtin_amdgcn_readlane((int)lmine, g);
        Lc[g] = L[g] > 16u * cpp ? 0u : L[g];  // longer than its slot: not read (verdict 0 below)
        r[g] = buf_rsrc(arena + (p0 + g) * cpp * 16u, (Lc[g] + 15u) & ~15u);  // slots past n: L = 0
        v[g] = buf_load<true>(r[g], (uint32_t)lane * 16u);
    }
#pragma unroll
    for (int g = 0; g < kSlotG; g++) {
        const int hi = (int)Lc[g] - 16 * lane;
        const u32x4 x = hi < 16 ? mask_tail(v[g], hi) : v[g];  // past the frame: zeros
        uint32_t acc = dot4(x, 0u);
        if (lane < 6) s_hdr[lane][w * kSlotG + g] = x;
        const uint32_t nch = (Lc[g] + 15u) >> 4;
        for (uint32_t c0 = 64; c0 < nch; c0 += 256) {  // wave-uniform: frames over 1 KiB
            u32x4 e[4];
#pragma unroll
            for (int k = 0; k < 4; k++) e[k] = buf_load<true>(r[g], (c0 + 64u * k + (uint32_t)lane) * 16u);
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int h = (int)Lc[g] - 16 * (int)(c0 + 64u * k + (uint32_t)lane);
                acc = dot4(h < 16 ? mask_tail(e[k], h) : e[k], acc);
            }
        }
        const uint32_t s = wave_total(acc);
        if (lane == 0) {
            s_sum[w * kSlotG + g] = s;
            s_len[w * kSlotG + g] = L[g];
        }
    }
    __syncthreads();
    const uint32_t i = threadIdx.x;
    const uint32_t np = (uint32_t)min<uint64_t>(4u * kSlotG, n - b0);
    if (i < np) {
        const uint32_t Li = s_len[i];
        const uint32_t F = bswap16(fold16(s_sum[i]));  // slots start 16-byte aligned: even address
        uint32_t hw[24];
#pragma unroll
        for (int k = 0; k < 6; k++) {
            const u32x4 x = s_hdr[k][i];
            hw[4 * k] = x.x, hw[4 * k + 1] = x.y, hw[4 * k + 2] = x.z, hw[4 * k + 3] = x.w;
        }
        const uint8_t* pkp = arena + (b0 + i) * cpp * 16u;
        const bool bad = Li > 16u * cpp;
        if (bad && err) atomicOr(err, 1u << PIPCK_ERANGE);
        store_result8(buf_rsrc(ok + b0, np), i, bad ? 0u : rx_from_window(pkp, Li, F, hw));
    }
}

// ---- the default: slot groups of 64, the block choosing its schedule -------
// A block of four waves owns 64 consecutive slots; every wave reads their 64
// lengths (lane g: slot g) and the block picks its schedule from them before it
// reads a frame byte (block-uniform, so a ring may mix fills):
//  * every frame <= 512 B: S lanes per slot (S = 8 / 16 / 32, the least power
//    of two covering the longest frame in chunks), 64 / S slots per load
//    instruction, one segmented DPP reduce per instruction, the block's loads
//    dealt round-robin to its waves -- short frames in small slots cost a few
//    instructions per slot, not a wave reduce each (k_ring_slots: 0.62 ms for
//    8M ~130-B frames, all of it per-slot work);
//  * otherwise a stream of the block's (slot, 1 KiB row) items that hold frame
//    bytes: rows past a frame are never issued (a sparse ring costs its frame
//    bytes), U loads in flight per wave, a run partial per lane flushed with one
//    wave reduce when the slot changes.  Jumbo slots (>= kRingCoopRows rows
//    per slot on average) deal the items round-robin to the four waves, so the
//    block reads one contiguous window (k_flat_coop's lesson); shorter ones
//    give each wave the items of its own 16 slots.
// Each slot's header window (its first six chunks) goes to LDS on the way; after
// the block's barrier wave 0 judges the 64 slots (lane g: slot g) with
// rx_from_window, so one wave's parse is spread over 64 slots.
constexpr uint32_t kRingB = 64;        // slots per block
constexpr uint32_t kRingCoopRows = 2;  // mean rows per slot from which the waves interleave
// pipck_tune_ring (pipck_testing.h): k_ring's schedule switches, a word of their
// own (they once shared pipck_tune's flag bits 27 / 29 with the
// small kernel's depth and the result-store policy)
constexpr uint32_t kRingOwnSlots = 1u;  // the row stream never interleaves its waves
constexpr uint32_t kRingAllCoop = 2u;   // the row stream always interleaves them
constexpr uint32_t kRingNoAdapt = 4u;   // no feedback: k_ring at every fill (the round-5 default)
constexpr uint32_t kRingAdaptAll = 8u;  // the feedback at every slot stride (tests; default from 4 KiB)
constexpr uint64_t kAdaptMinStride = 4096;  // jumbo slots: below, k_ring wins at every fill
std::atomic<uint32_t> g_ring_mode{0};

struct RingLds {
    u32x4 hdr[6][kRingB];  // chunk k of slot g's header window
    uint32_t sum[kRingB];  // slot g's LE residue sum
};

// Sum of v over each aligned group of S lanes (S = 8, 16, 32), valid in lane
// S / 2 of the group: two quad swaps, a half-row mirror (8), a row mirror
// (16), then row_bcast:15 into rows 1 and 3 (32) -- DPP only, no LDS trips.
template <int S>
__device__ __forceinline__ uint32_t group_total(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, false);  // row_half_mirror
    if (S >= 16) v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xf, 0xf, false);  // row_mirror
    if (S >= 32) v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    return v;
}

// Short frames: group gi = lane / S of load j takes slot j * (64 / S) + gi,
// lane k = lane % S its chunk k; this wave takes loads first, first + step, ...
// Lc: lane g holds slot g's readable bytes, fetched per load for the group's
// slot (a ds_bpermute, again at the reduce rather than held: registers set the
// wave count, and a ring of U loads is reloaded as it is consumed).
template <int S, int U>
__device__ __forceinline__ void ring_short(RingLds& t, buf_t rb, uint32_t stride, uint32_t nb, uint32_t Lc,
                                           uint32_t first, uint32_t step, int lane) {
    constexpr uint32_t P = 64u / S;  // slots per load
    const uint32_t k = (uint32_t)lane % S, gi = (uint32_t)lane / S;
    const uint32_t loads = (nb + P - 1) / P;  // <= S
    auto issue = [&](uint32_t j) -> u32x4 {
        uint32_t off = 0xFFFFFFF0u;  // past the block's loads, or the frame: no request
        if (j < loads) {             // wave-uniform
            const uint32_t g = j * P + gi;
            const uint32_t Lg = (uint32_t)__shfl((int)Lc, (int)g, 64);
            if (16u * k < Lg) off = g * stride + 16u * k;
        }
        return buf_load<true>(rb, off);
    };
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = issue(first + step * u);
    for (uint32_t j0 = first; j0 < loads; j0 += step * U) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t j = j0 + step * u;
            if (j < loads) {  // wave-uniform
                const uint32_t g = j * P + gi;
                const int hi = (int)__shfl((int)Lc, (int)g, 64) - 16 * (int)k;
                const u32x4 x = hi < 16 ? mask_tail(v[u], hi) : v[u];
                const uint32_t tot = group_total<S>(dot4(x, 0u));
                if (k == S / 2) t.sum[g] = tot;
                if (k < 6) t.hdr[k][g] = x;
            }
            v[u] = issue(j + step * U);
        }
    }
}

// Longer frames: item i of the block's stream = row r of slot g, for the
// slots' row counts R (lane g: R_g = ceil(chunks_g / 64); incl their inclusive
// prefix).  Slot of item i: the number of slots whose rows all come before it
// (a ballot popcount); its row: i minus the rows before the slot.  This wave
// takes items first, first + step, ... below end; its run partial is flushed
// (one wave reduce, an LDS add: slots may be shared between waves) when the
// slot changes.
template <int U>
__device__ __forceinline__ void ring_rows(RingLds& t, buf_t rb, uint32_t stride, uint32_t Lc, uint32_t incl,
                                          uint32_t excl, uint32_t first, uint32_t end, uint32_t step, int lane) {
    u32x4 v[U];
    // per ring entry, one scalar: slot g (6 bits) | row r << 6 (6 bits: <= 64 rows
    // in a 64 KiB slot) | slot bytes L << 12 (17 bits) -- three scalars per entry
    // would take the kernel past 80 SGPRs, which costs a block per CU
    uint32_t se[U];
    auto issue = [&](uint32_t i, int u) {
        uint32_t g = 0, r = 0, L = 0;
        if (i < end) {  // wave-uniform
            g = (uint32_t)__popcll(__ballot(incl <= i));
            r = i - (uint32_t)__builtin_amdgcn_readlane((int)excl, (int)g);
            L = (uint32_t)__builtin_amdgcn_readlane((int)Lc, (int)g);
        }
        se[u] = g | r << 6 | L << 12;
        const uint32_t c = 64u * r + (uint32_t)lane;
        v[u] = buf_load<true>(rb, 16u * c < L ? g * stride + 16u * c : 0xFFFFFFF0u);
    };
    auto flush = [&](uint32_t g, uint32_t acc) {
        const uint32_t s = wave_total(acc);
        if (lane == 0) atomicAdd(&t.sum[g], s);
    };
#pragma unroll
    for (int u = 0; u < U; u++) issue(first + step * u, u);
    uint32_t cur = 0xFFFFFFFFu, acc = 0;
    for (uint32_t j0 = first; j0 < end; j0 += step * U) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = j0 + step * u;
            if (i < end) {  // wave-uniform
                const uint32_t g = se[u] & 63u, r = (se[u] >> 6) & 63u, L = se[u] >> 12;
                if (g != cur) {  // this wave's share of the previous slot is all in
                    if (cur != 0xFFFFFFFFu) flush(cur, acc);
                    cur = g;
                    acc = 0;
                }
                u32x4 x = v[u];
                if (L < 1024u * (r + 1u)) {  // wave-uniform: the frame ends in this row (else no mask)
                    const int hi = (int)L - 16 * (int)(64u * r + (uint32_t)lane);
                    if (hi < 16) x = mask_tail(x, hi);
                }
                acc = dot4(x, acc);
                if (r == 0 && lane < 6) t.hdr[lane][g] = x;
            }
            issue(i + step * U, u);  // past this wave's items: no request
        }
    }
    if (cur != 0xFFFFFFFFu) flush(cur, acc);
}

template <int U, int UD>
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_sgpr(80))) void k_ring(const uint8_t* __restrict__ arena, uint32_t stride,
                                              const uint16_t* __restrict__ lens, uint64_t n, uint32_t G,
                                              uint8_t* __restrict__ ok, uint32_t* __restrict__ err,
                                              uint32_t kflags, RingFb fb) {
    // (the block size is a compile-time constant: as a kernel argument it cost
    // the short-frame stream 40 %, profiles/r05_ring_schedule_ab.jsonl)
    constexpr uint32_t B = kRingB;
    __shared__ RingLds t;
    const int lane = threadIdx.x & 63;
    const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint64_t b0 = (uint64_t)blockIdx.x * B;  // the block's first slot
    const uint32_t nb = (uint32_t)min<uint64_t>(B, n - b0);
    const bool valid = (uint32_t)lane < nb;
    const uint32_t L = valid ? (uint32_t)lens[b0 + lane] : 0u;  // every wave: all 64 lengths
    const bool bad = L > stride;       // longer than its slot: not read, verdict 0
    const uint32_t Lc = bad ? 0u : L;  // the bytes this slot reads
    const uint32_t nch = (Lc + 15u) >> 4;
    const uint32_t cmax = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_max(nch), 63);
    if (w == 0) t.sum[lane] = 0;  // flushes add
    __syncthreads();
    const buf_t rb = buf_rsrc(arena + b0 * stride, nb * stride);  // the block's slots
    if (cmax <= 32) {
        if (cmax <= 8)
            ring_short<8, 8>(t, rb, stride, nb, Lc, w, 4u, lane);
        else if (cmax <= 16)
            ring_short<16, 8>(t, rb, stride, nb, Lc, w, 4u, lane);
        else
            ring_short<32, 8>(t, rb, stride, nb, Lc, w, 4u, lane);
    } else {
        const uint32_t R = (nch + 63u) >> 6;
        const uint32_t incl = wave_incl_scan(R);
        const uint32_t excl = incl - R;
        const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);  // the block's items
        const bool coop = (kflags & kRingAllCoop) || (!(kflags & kRingOwnSlots) && T >= kRingCoopRows * nb);
        if (coop) {
            // sub-groups of G slots, one after the other, the four waves on each
            for (uint32_t g0 = 0; g0 < nb; g0 += G) {
                const uint32_t ib = (uint32_t)__builtin_amdgcn_readlane((int)excl, (int)g0);
                const uint32_t ie = g0 + G < nb ? (uint32_t)__builtin_amdgcn_readlane((int)excl, (int)(g0 + G)) : T;
                ring_rows<UD>(t, rb, stride, Lc, incl, excl, ib + w, ie, 4u, lane);
            }
        } else {  // wave w: the items of its quarter of the slots
            const uint32_t q = B / 4u;
            const uint32_t ib = (uint32_t)__builtin_amdgcn_readlane((int)excl, (int)(q * w));
            const uint32_t ie = w < 3 ? (uint32_t)__builtin_amdgcn_readlane((int)excl, (int)(q * w + q)) : T;
            ring_rows<U>(t, rb, stride, Lc, incl, excl, ib, ie, 1u, lane);
        }
    }
    __syncthreads();
    if (w != 0) return;  // wave 0 judges the block's slots
    uint32_t r = 0;
    if (valid && !bad) {
        const uint32_t F = bswap16(fold16(t.sum[lane]));  // slots start 16-byte aligned: even address
        uint32_t hw[24];
#pragma unroll
        for (int k = 0; k < 6; k++) {  // chunks past the frame were never captured: zero
            const u32x4 x = 16u * k < L ? t.hdr[k][lane] : u32x4{0u, 0u, 0u, 0u};
            hw[4 * k] = x.x, hw[4 * k + 1] = x.y, hw[4 * k + 2] = x.z, hw[4 * k + 3] = x.w;
        }
        r = rx_from_window(arena + (b0 + (uint32_t)lane) * stride, L, F, hw);
    }
    if (bad && err) atomicOr(err, 1u << PIPCK_ERANGE);
    store_result8(buf_rsrc(ok + b0, nb), (uint32_t)lane, r);
    if (fb.ctr && blockIdx.x % fb.every == 0)  // the schedule's feedback (wave 0, after its stores)
        ring_report(fb, ring_dense(wave_total((nch + 63u) >> 6), nb, stride), lane);
}

// Per-ring feedback state (host side of RingFb), keyed by (device, ring
// address, slot stride); at most kFbRings rings, the least recently used one's
// buffers reused for a new ring (a launch of the old ring still in flight can
// then only mix the heuristic).  Never freed: 64 x (8 B device + 16 B pinned).
struct FbEntry {
    int dev = -1;
    const void* ring = nullptr;
    uint64_t stride = 0;
    unsigned long long* d_ctr = nullptr;
    uint32_t* h = nullptr;
    uint32_t seq = 0;
    uint64_t used = 0;
};
constexpr size_t kFbRings = 64;
static std::mutex g_fb_mu;
static std::vector<FbEntry> g_fb;
static uint64_t g_fb_clock = 0;

// The entry of this ring (created or recycled on first use, its counter zeroed
// on `s`), its next sequence number, and whether its last published report says
// the row stream fits: >= 90 % of the reporting blocks found their slots dense.
static int ring_feedback(const void* ring, uint64_t stride, hipStream_t s, RingFb* fb, bool* rows) {
    int dev = 0;
    PIPCK_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_fb_mu);
    FbEntry* e = nullptr;
    for (auto& x : g_fb)
        if (x.dev == dev && x.ring == ring && x.stride == stride) e = &x;
    fb->ctr = nullptr;  // no feedback unless an entry is found or made below (then k_ring)
    *rows = false;
    if (!e) {
        FbEntry x;
        x.dev = dev;
        bool made = false;
        if (g_fb.size() < kFbRings) {
            if (hipMalloc(reinterpret_cast<void**>(&x.d_ctr), sizeof(unsigned long long)) != hipSuccess) {
                (void)hipGetLastError();  // (our own failure) recycle an entry instead
            } else if (hipHostMalloc(reinterpret_cast<void**>(&x.h), 4 * sizeof(uint32_t), hipHostMallocCoherent) !=
                       hipSuccess) {
                (void)hipGetLastError();
                (void)hipFree(x.d_ctr);
            } else {
                made = true;
            }
        }
        if (made) {
            if (g_fb.empty()) g_fb.reserve(kFbRings);
            g_fb.push_back(x);
            e = &g_fb.back();
        } else {
            for (auto& y : g_fb)  // recycle this device's least recently used ring
                if (y.dev == dev && (!e || y.used < e->used)) e = &y;
            if (!e) return PIPCK_OK;  // every entry belongs to other devices
        }
        e->ring = ring;
        e->stride = stride;
        e->seq = 0;
        __atomic_store_n(&e->h[0], 0u, __ATOMIC_RELAXED);
        PIPCK_HIP(hipMemsetAsync(e->d_ctr, 0, sizeof(unsigned long long), s));
    }
    e->used = ++g_fb_clock;
    if (++e->seq == 0) e->seq = 1;
    const uint32_t seen = __atomic_load_n(&e->h[0], __ATOMIC_ACQUIRE);
    const uint32_t dense = __atomic_load_n(&e->h[1], __ATOMIC_RELAXED);
    const uint32_t parts = __atomic_load_n(&e->h[2], __ATOMIC_RELAXED);
    *rows = seen != 0 && parts != 0 && 10ull * dense >= 9ull * parts;
    fb->ctr = e->d_ctr;
    fb->host = e->h;
    fb->seq = e->seq;
    return PIPCK_OK;
}

int launch_ring_rx(const void* d_arena, uint64_t stride, const uint16_t* d_lens, uint64_t n, uint8_t* d_ok,
                   uint32_t* d_err, hipStream_t s) {
    if (n == 0) return PIPCK_OK;
    if (!d_arena || !d_lens || !d_ok) {
        set_error("pipck_rx_verify_ring: null pointer");
        return PIPCK_EINVAL;
    }
    if ((uintptr_t)d_arena % 16 || stride % 16 || stride < 1024 || stride > 65536) {
        set_error("pipck_rx_verify_ring: the arena must be 16-byte aligned and the slot stride a multiple of 16 "
                  "bytes from 1 KiB to 64 KiB");
        return PIPCK_EINVAL;
    }
    const uint32_t cpp = (uint32_t)(stride / 16);
    const uint32_t flags = g_ring_mode.load();
    // jumbo slots: k_ring or the row stream, by the feedback of this ring's
    // earlier launches (speed only, the verdicts are the same)
    RingFb fb{nullptr, nullptr, 1u, 0u, 0u};
    bool rows = false;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (!wave_arm() && !alt_schedule() && !(flags & kRingNoAdapt) &&
        (stride >= kAdaptMinStride || (flags & kRingAdaptAll)) &&
        hipStreamIsCapturing(s, &cap) == hipSuccess && cap == hipStreamCaptureStatusNone) {
        // (a stream being captured into a graph gets k_ring: the feedback's first
        // use allocates, and a replayed launch would keep reporting one sequence)
        const int rc = ring_feedback(d_arena, stride, s, &fb, &rows);
        if (rc) return rc;
    }
    if (wave_arm()) {  // measurement arm: slot by slot, a wave per slot
        const uint64_t blocks = (n + 4u * kSlotG - 1) / (4u * kSlotG);
        if (blocks > 0x7FFFFFFFull) {
            set_error("pipck_rx_verify_ring: too many slots for one launch");
            return PIPCK_ERANGE;
        }
        PIPCK_LAUNCH(k_ring_slots, dim3((uint32_t)blocks), dim3(256), 0, s, (const uint8_t*)d_arena, cpp, d_lens, n,
                     d_ok, d_err);
        PIPCK_LAUNCHED("k_ring_slots");
        return PIPCK_OK;
    }
    if (alt_schedule() || rows) {  // the row stream over whole slots (dense jumbo rings; tune bit 28: always)
        // K slots per block task: ~4 waves x 48 rows (x 64 for jumbo slots), a
        // multiple of 8, at most 256 (one slot per thread at the end) -- k_flat_coop's
        uint32_t K = (4u * (cpp >= 256 ? 64u : 48u) * 64u) / cpp;
        K = std::max<uint32_t>(8u, std::min<uint32_t>(256u, K / 8u * 8u));
        if ((uint64_t)K * stride >= (1ull << 31)) return PIPCK_EINVAL;
        const uint64_t blocks = (n + K - 1) / K;
        if (blocks > 0x7FFFFFFFull) {
            set_error("pipck_rx_verify_ring: too many slots for one launch");
            return PIPCK_ERANGE;
        }
        const size_t lds = 4u * (64u * ring_pitch(K) + ((K + 3u) & ~3u)) + 16u * 6u * K;
        if (fb.ctr) {
            if (K > 64) fb.ctr = nullptr;  // a report reads one wave's lengths: tasks of <= 64 slots only
            fb_sample(fb, blocks);
        }
        PIPCK_LAUNCH(k_ring_rx, dim3((uint32_t)blocks), dim3(256), lds, s, (const uint8_t*)d_arena, cpp, d_lens, n, K,
                     d_ok, d_err, fb);
        PIPCK_LAUNCHED("k_ring_rx");
        return PIPCK_OK;
    }
    // slot groups (k_ring): 64 slots per block; U = 8 loads in flight per wave in
    // the row stream (loads_per_lane 16 / 24 for more): the kernel's registers --
    // 48 VGPRs at 8, 79 at 16 -- set the waves per SIMD, which the short and
    // sparse rings need more than a deeper ring (short 1 KiB slots 0.27 against
    // 0.32 ms, sparse 9 KiB 1.32 against 1.46; full 1.5 KiB slots 0.846
    // against 0.858 of peak: profiles/r05_ring_schedule_ab.jsonl)
    const uint64_t blocks = (n + kRingB - 1) / kRingB;
    // the interleaved row stream covers all 64 slots at once, or G at a time (the
    // tune's blocks knob, 8 / 16 / 32): sub-groups helped jumbo slots only with a
    // ring of 24 (0.890 against 0.879 of peak) and drain a shallow ring between
    // groups of short slots (full 1.5 KiB slots 2.46 against 1.86 ms)
    const uint32_t gt = g_tune_blocks();
    const uint32_t G = (gt == 8 || gt == 16 || gt == 32) ? gt : 64u;
    if (blocks > 0x7FFFFFFFull) {
        set_error("pipck_rx_verify_ring: too many slots for one launch");
        return PIPCK_ERANGE;
    }
    const uint8_t* a = (const uint8_t*)d_arena;
    const uint32_t st = (uint32_t)stride;
    fb_sample(fb, blocks);
    // loads in flight per wave: U in the short and own-slot streams, UD in the
    // interleaved one (loads_per_lane 16 / 24: both; 17 / 25: UD only)
#define PIPCK_RING(UU, UUD)                                                                                     \
    PIPCK_LAUNCH((k_ring<UU, UUD>), dim3((uint32_t)blocks), dim3(256), 0, s, a, st, d_lens, n, G, d_ok, d_err,    \
                 flags, fb)
    switch (g_tune_loads()) {
        case 8: PIPCK_RING(8, 8); break;
        case 12: PIPCK_RING(12, 12); break;
        case 16: PIPCK_RING(16, 16); break;
        case 24: PIPCK_RING(24, 24); break;
        case 17: PIPCK_RING(8, 16); break;
        case 25: PIPCK_RING(8, 24); break;
        default: PIPCK_RING(8, 12); break;
    }
#undef PIPCK_RING
    PIPCK_LAUNCHED("k_ring");
    return PIPCK_OK;
}

}  // namespace pipck

extern "C" {

void pipck_tune_ring(uint32_t mode) { pipck::g_ring_mode.store(mode); }

int pipck_rx_verify_ring_n(const void* d_arena, uint64_t slot_stride, const uint16_t* d_lens, uint64_t n,
                           uint8_t* d_ok, uint32_t* d_err, void* stream) {
    return pipck::launch_ring_rx(d_arena, slot_stride, d_lens, n, d_ok, d_err, pipck::as_stream(stream));
}

// the same without the error word (every slot is still bounded on the device)
int pipck_rx_verify_ring(const void* d_arena, uint64_t slot_stride, const uint16_t* d_lens, uint64_t n,
                         uint8_t* d_ok, void* stream) {
    return pipck_rx_verify_ring_n(d_arena, slot_stride, d_lens, n, d_ok, nullptr, stream);
}

int pipck_rx_verify_device(const void* d_arena, uint64_t arena_bytes, const uint16_t* d_lens,
                           const uint64_t* d_tile_off, uint64_t n, uint8_t* d_ok, uint32_t* d_err, void* stream) {
    return pipck::launch_packedb_rx(d_arena, arena_bytes, d_lens, d_tile_off, n, d_ok, d_err,
                                    pipck::as_stream(stream));
}

}  // extern "C"
