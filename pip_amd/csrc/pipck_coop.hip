// pipck_coop.hip -- block-cooperative flat stream for fixed 16-B-multiple strides >= 1 KiB.
//
// Hot path: plumk97/pip pip/pip_checksum.cpp:42-87 (pip_inet{,6}_checksum) and
// :35-39 (pip_ip_checksum) over fixed-stride batches (cfg2, cfg3, cfg5).
//
// k_flat gives every wave its own task of consecutive packets (four separate
// 64 KiB streams per block).  The access-pattern probe (tools/probe/
// stream_probe.hip, profiles/r02_stream_probe.jsonl) streams the same bytes
// 4-5 % faster when a block's four waves read NEIGHBOURING line-aligned rows
// at the same time: one 1 KiB row each, wave w taking rows w, w+4, w+8, ... of
// the block's task, so the block moves as one contiguous window.  Round 2's
// kernels on that schedule lost their gain at the task end; round 3 found the
// end's cost to be the result stores (plain write-back stores evicted mid-
// stream; write-through sc1 stores cost nothing, pipck_device.hpp), so the
// schedule is tried again here.
//
// k_flat_coop: a block task is K whole packets (K * stride a multiple of 128
// bytes, so with a line-aligned arena every task and every row starts on a
// 128-B line).  Each lane of each row adds its chunk's sum (four dot2 folds)
// into an LDS partial of the packet that chunk belongs to -- part[lane][pkt],
// one u32 LDS add per lane per row, no cross-lane work in the stream -- and at
// the task's end thread j sums packet j's 64 partials, adds the pseudo-header
// loaded when the block started, and the block stores its K results once
// (write-through).  A ring of U rows per wave stays in flight.
#include "pipck_common.hpp"
#include "pipck_device.hpp"

#include <algorithm>

namespace pipck {

// pipck_tune flags bits 21 / 22 (MEASUREMENT ONLY, no results), as for k_flat:
// consume every row with one add and skip the per-row work / skip the task end
constexpr uint32_t kCoopLoadsOnly = 1u << 21;
constexpr uint32_t kCoopNoEnd = 1u << 22;

template <int U>
constexpr int coop_waves_per_simd() { return U >= 32 ? 2 : (U >= 24 ? 3 : (U >= 16 ? 4 : 5)); }

__host__ __device__ constexpr uint32_t coop_pitch(uint32_t k) { return k | 1u; }  // odd: lanes hit distinct banks

// The kernel body; PROBE = false compiles the measurement bits out of the
// production kernel k_flat_coop (no per-row flag test), k_flat_coop_probe keeps them.
template <int U, bool VERIFY, bool NT, bool PROBE>
__device__ __forceinline__ void coop_body(uint32_t* s_part, const uint8_t* __restrict__ arena, uint32_t cpp,
                                          uint32_t len, uint64_t n, uint32_t K, const uint32_t* __restrict__ pseudo,
                                          uint32_t n_flows, const uint32_t* __restrict__ flow_of, uint64_t flow_origin,
                                          uint16_t* __restrict__ out, uint8_t* __restrict__ ok, uint32_t kflags,
                                          uint32_t* __restrict__ err) {
    if (!PROBE) kflags &= ~(kCoopLoadsOnly | kCoopNoEnd);
    const int lane = threadIdx.x & 63;
    const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint32_t pitch = coop_pitch(K);
    const uint64_t p0 = (uint64_t)blockIdx.x * K;
    const uint32_t np = (uint32_t)min<uint64_t>((uint64_t)K, n - p0);
    const uint32_t tchunks = np * cpp;
    const uint32_t rows = (tchunks + 63) >> 6;
    const uint32_t nch = (len + 15) >> 4;                         // data chunks per packet (<= cpp)
    const int tail = nch ? (int)len - 16 * ((int)nch - 1) : 16;  // valid bytes of the last data chunk
    for (uint32_t i = threadIdx.x; i < 64u * pitch; i += 256) s_part[i] = 0;
    // pseudo-header base of packet threadIdx.x (K <= 256), loaded now so the
    // task's end waits on nothing.  With flow_of, n_flows bounds the entry (the
    // _n forms; UINT32_MAX: trusted): one past the table is refused at the end.
    uint32_t Pb = 0;
    bool fbad = false;
    if (pseudo && threadIdx.x < np) {
        const uint64_t pkt = p0 + threadIdx.x;
        Pb = flow_of ? flow_pseudo(pseudo, flow_of[pkt], n_flows, fbad)
                     : pseudo[(uint32_t)((flow_origin + pkt) % n_flows)];
    }
    __syncthreads();
    const buf_t tb = buf_rsrc(reinterpret_cast<const u32x4*>(arena) + p0 * cpp, tchunks * 16u);
    uint32_t* part = s_part + lane * pitch;
    // this wave's rows w, w+4, ...: lane 0's packet and chunk-in-packet, advanced
    // by 256 chunks (= q packets + rm chunks) per row without divisions
    const uint32_t q = 256u / cpp, rm = 256u % cpp;
    uint32_t pkt = (64u * w) / cpp, k0 = (64u * w) % cpp;
    const uint32_t my_rows = rows > w ? (rows - w + 3) >> 2 : 0u;
    u32x4 v[U];
    uint32_t probe = 0;
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = buf_load<NT>(tb, ((w + 4u * u) * 64u + lane) * 16u);  // past the task: zeros
    for (uint32_t j0 = 0; j0 < my_rows; j0 += U) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t j = j0 + u;
            if (j < my_rows && (kflags & kCoopLoadsOnly)) {  // measurement: consume the row, no per-row work
                probe += v[u].x;
            } else if (j < my_rows) {  // wave-uniform
                // lane's chunk: k0 + lane chunks into packet pkt (at most one boundary: cpp >= 64)
                uint32_t k = k0 + lane, pk = pkt;
                if (k >= cpp) {
                    k -= cpp;
                    pk++;
                }
                u32x4 x = v[u];
                if (k >= nch) x = u32x4{0u, 0u, 0u, 0u};  // stride padding
                else if (k == nch - 1 && tail < 16) x = mask_tail(x, tail);
                // chunks past the task read zeros and add nothing; keep their
                // (possibly out-of-task) packet index inside the LDS block
                if (pk < np) atomicAdd(&part[pk], dot4(x, 0u));
                k0 += rm;
                pkt += q;
                if (k0 >= cpp) {
                    k0 -= cpp;
                    pkt++;
                }
            }
            // ring: the row U ahead (unconditional: past the task it reads zeros, no request)
            v[u] = buf_load<NT>(tb, ((w + 4u * (j + U)) * 64u + lane) * 16u);
        }
    }
    __syncthreads();
    if (kflags & (kCoopLoadsOnly | kCoopNoEnd)) {  // measurement only: no results
        if (probe == 0x9E3779B9u) s_part[0] = probe;
        return;
    }
    const uint32_t i = threadIdx.x;
    if (i < np) {
        uint32_t s = 0;
#pragma unroll 16
        for (int l = 0; l < 64; l++) s += s_part[l * pitch + i];
        const uint32_t F = bswap16(fold16(s));  // packets start 16-byte aligned: even address
        const uint32_t P = pseudo ? Pb + len_term(len) : 0u;
        if (fbad) flow_refused(err);  // a flow_of entry past the table: result 0
        if (VERIFY)
            store_result8(buf_rsrc(ok + p0, np), i, fbad ? 0u : (uint32_t)(fold16(P + F) == 0xFFFFu));
        else
            store_result16(buf_rsrc(out + p0, 2u * np), 2u * i, fbad ? 0u : (uint32_t)finish(P, F));
    }
}

template <int U, bool VERIFY, bool NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(coop_waves_per_simd<U>()))) void k_flat_coop(
    const uint8_t* __restrict__ arena, uint32_t cpp, uint32_t len, uint64_t n, uint32_t K,
    const uint32_t* __restrict__ pseudo, uint32_t n_flows, const uint32_t* __restrict__ flow_of, uint64_t flow_origin,
    uint16_t* __restrict__ out, uint8_t* __restrict__ ok, uint32_t kflags, uint32_t* __restrict__ err) {
    extern __shared__ uint32_t s_part[];  // 64 lanes x pitch u32 (launch_coop sizes it)
    coop_body<U, VERIFY, NT, false>(s_part, arena, cpp, len, n, K, pseudo, n_flows, flow_of, flow_origin, out, ok,
                                    kflags, err);
}

// k_flat_coop with the measurement bits 21 / 22 live (tools only)
template <int U, bool VERIFY, bool NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(coop_waves_per_simd<U>()))) void
k_flat_coop_probe(const uint8_t* __restrict__ arena, uint32_t cpp, uint32_t len, uint64_t n, uint32_t K,
                  const uint32_t* __restrict__ pseudo, uint32_t n_flows, const uint32_t* __restrict__ flow_of,
                  uint64_t flow_origin, uint16_t* __restrict__ out, uint8_t* __restrict__ ok, uint32_t kflags,
                  uint32_t* __restrict__ err) {
    extern __shared__ uint32_t s_part[];
    coop_body<U, VERIFY, NT, true>(s_part, arena, cpp, len, n, K, pseudo, n_flows, flow_of, flow_origin, out, ok,
                                   kflags, err);
}

typedef void (*coop_fn)(const uint8_t*, uint32_t, uint32_t, uint64_t, uint32_t, const uint32_t*, uint32_t,
                        const uint32_t*, uint64_t, uint16_t*, uint8_t*, uint32_t, uint32_t*);

// Launch for an aligned arena, 16-B-multiple stride in [1 KiB, 64 KiB], len <=
// stride (checked by the caller); n_flows as launch_fixed hands it to every
// fixed kernel (the modulus, or with d_flow_of the entries' bound).
// rows_per_wave: task size target (0 = auto);
// ring: rows in flight per wave (0 = auto).  Returns PIPCK_OK, or PIPCK_EINVAL
// when the shape does not fit a block task (the caller then uses k_flat).
int launch_flat_coop(bool verify, const void* d_arena, uint64_t stride, uint32_t len, uint64_t n,
                     const uint32_t* d_pseudo, uint32_t n_flows, const uint32_t* d_flow_of, uint64_t flow_origin,
                     uint16_t* d_out, uint8_t* d_ok, uint32_t* d_err, hipStream_t s, uint32_t rows_per_wave,
                     uint32_t ring, uint32_t kflags) {
    const uint32_t cpp = (uint32_t)(stride / 16);
    const bool jumbo = cpp >= 256;
    // rows per wave: 64 for jumbo packets (cfg5: 24 packets per block task;
    // 48 rows lost 7 %, 80 rows 0.4 %), 48 for shorter ones (cfg2: 128 packets)
    const uint32_t rpw = rows_per_wave ? rows_per_wave : (jumbo ? 64u : 48u);
    // K packets per block task: ~4 * rpw rows, a multiple of 8 packets (8 * stride
    // is a multiple of 128 B), at most 256 (one packet per thread at the end)
    uint32_t K = (4u * rpw * 64u) / cpp;
    K = std::max<uint32_t>(8u, std::min<uint32_t>(256u, K / 8u * 8u));
    if ((uint64_t)K * cpp * 16u >= (1ull << 31)) return PIPCK_EINVAL;
    const uint64_t blocks = (n + K - 1) / K;
    if (blocks > 0x7FFFFFFFull) return PIPCK_EINVAL;
    const size_t lds = 64u * coop_pitch(K) * sizeof(uint32_t);
    const uint32_t nf = n_flows ? n_flows : 1u;
    // a ring of 32 rows at every stride (2 waves/SIMD): at 1,488-B strides
    // 0.887-0.891 ms against 0.894-0.897 for 24 (profiles/r04_cfg2_coop_scan.jsonl)
    const uint32_t u = ring ? ring : 32u;
    static const coop_fn kCoop[3][2] = {  // [ring 16 / 24 / 32][verify], non-temporal loads
        {k_flat_coop<16, false, true>, k_flat_coop<16, true, true>},
        {k_flat_coop<24, false, true>, k_flat_coop<24, true, true>},
        {k_flat_coop<32, false, true>, k_flat_coop<32, true, true>}};
    static const coop_fn kCoopProbe[3] = {k_flat_coop_probe<16, false, true>, k_flat_coop_probe<24, false, true>,
                                          k_flat_coop_probe<32, false, true>};
    const int ui = u >= 32 ? 2 : (u >= 24 ? 1 : 0);
    const bool probe = (kflags & (kCoopLoadsOnly | kCoopNoEnd)) && !verify;
    PIPCK_LAUNCH(probe ? kCoopProbe[ui] : kCoop[ui][verify], dim3((uint32_t)blocks), dim3(256), lds, s, (const uint8_t*)d_arena, cpp, len, n,
                 K, d_pseudo, nf, d_flow_of, flow_origin, d_out, d_ok, kflags, d_err);
    PIPCK_LAUNCHED("k_flat_coop");
    return PIPCK_OK;
}

}  // namespace pipck
