// pipck_packedb.hip -- byte-packed ragged batches (cfg4's bench layout) + their C ABI.
//
// Hot path: plumk97/pip pip/pip_checksum.cpp:42-87 (pip_inet{,6}_checksum)
// over a batch of variable-length segments laid back to back with NO padding:
// packet i starts at byte b_i = len_0 + ... + len_{i-1} of the arena.  The
// 16-byte-granular packed layout (pipck_checksum_packed, k_packed) rounds each
// segment up to 16 bytes; on cfg4's Zipf lengths that padding is 0.76 % of the
// bytes read, every one of them fetched from HBM.  Here nothing but packet
// bytes (and the 2-byte lengths) is read.
//
// k_packedb: one tile of 64 packets per block of W waves (8 by default).  Each
// wave reads the 64 u16 lengths and the tile's byte offset (one u64 per tile),
// derives every packet's offset with a wave prefix scan, and the block streams
// the tile as coalesced 1 KiB rows, wave w taking rows w, w + W, ..., from the
// 128-B line holding its first byte (rows are
// whole lines; the bytes before the tile's first packet belong to the
// previous tile and are summed into a discarded slot).  Since segments are no
// longer chunk-aligned, a 16-byte chunk may hold the end of one segment and
// the start of the next: each lane splits its chunk at that boundary into a
// low part (the segment holding the chunk's first byte, found by LDS start
// marks + a DPP max-scan) and a high part (the next segment), and the row
// reduces by segment with the head/tail prefix-scan trick over the low parts
// plus one LDS add per boundary lane for the high part.  A row wholly inside
// one segment is four dot2 ops into a per-lane run partial, nothing else.
// Segments are summed as little-endian dwords of aligned chunks and byte
// order is fixed once per segment from its start's parity (pipck_device.hpp).
//
// Tiles holding a segment shorter than 16 bytes (where one chunk could hold
// three segments) are summed lane-per-segment instead: correct for any
// lengths (0 included), slow, and absent from the BASELINE shapes (>= 64 B).
#include "pipck_common.hpp"
#include "pipck_device.hpp"
#include "pipck_rxparse.hpp"

namespace pipck {

// W = the waves that stream one tile together (rows dealt round-robin)
template <int W>
struct PackedbLdsT {
    // +1-encoded segment slots: 0 = the bytes before the tile's first packet,
    // s + 1 = packet s of the tile, nv + 1 .. 65 = bytes after its last packet
    uint32_t end[66];  // end[S] = byte (relative to the line-aligned base) where slot S ends
    uint32_t acc[66];  // LE residue partial per slot
    uint32_t mark[W][64];  // per wave: (row tag << 7) | S of the slot starting at chunk row + i (max wins)
};

// Add a run of whole rows of one slot (per-lane u32 partials in racc) to the
// slot's LDS partial: one wave sum, one LDS add.
template <int W>
__device__ __forceinline__ void packedb_flush(PackedbLdsT<W>& t, int lane, uint32_t& racc, uint32_t& rslot) {
    if (rslot == 0xFFFFFFFFu) return;  // wave-uniform
    const uint32_t tot = wave_total(racc);
    if (lane == 0) atomicAdd(&t.acc[rslot], tot);
    racc = 0;
    rslot = 0xFFFFFFFFu;
}

// One 1 KiB row (chunks row .. row+63 of the tile stream).  start_v / end_v:
// lane s holds packet s's first and one-past-last byte (relative); mfirst_v
// the first chunk whose first byte lies in packet s (start rounded up to 16);
// nv valid packets.  S0 / e0: the slot holding the row's first byte and its
// end byte (scalars, carried across rows).
//
// RX (k_packedb_rx): the row also hands every packet the chunks of its header
// window -- the six aligned chunks from the one holding its first byte, as far
// as the packet reaches -- into hdr[k * 64 + packet] in LDS, so the tile's end
// parses headers without reading them from memory again.  A chunk whose first
// byte lies in packet s is window chunk k = c - (start_s >> 4) of s when
// k < 6; a chunk holding a packet boundary is window chunk 0 of the packet
// that starts inside it.  (Tiles with a packet under 16 bytes take the
// lane-per-segment path and read their headers from memory.)
template <bool RX, int W>
__device__ __forceinline__ void packedb_reduce_row(PackedbLdsT<W>& t, uint32_t w, u32x4* hdr, uint32_t row,
                                                   uint32_t total, int lane,
                                                   const u32x4& v, uint32_t start_v, uint32_t end_v,
                                                   uint32_t mfirst_v, bool valid, uint32_t nv, uint32_t& S0,
                                                   uint32_t& e0, uint32_t& racc, uint32_t& rslot) {
    const uint32_t rb = 16u * row;  // the row's first byte
    if (rb >= e0) {                 // wave-uniform: the row starts past slot S0
        S0 = (uint32_t)__popcll(__ballot(valid && start_v <= rb));
        e0 = t.end[S0];
    }
    S0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)S0);
    e0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)e0);
    rslot = (uint32_t)__builtin_amdgcn_readfirstlane((int)rslot);
    if (e0 >= rb + 1024u) {  // interior row: every byte of the row in slot S0
        if (S0 != rslot) {
            packedb_flush(t, lane, racc, rslot);
            rslot = S0;
        }
        racc = dot4(v, racc);
        if (RX && S0 >= 1 && S0 <= nv) {  // the row may hold the last chunks of packet S0 - 1's window
            const uint32_t cs = (uint32_t)__builtin_amdgcn_readfirstlane((int)(t.end[S0 - 1] >> 4));
            if (row < cs + 6u) {  // wave-uniform
                const uint32_t k = row + (uint32_t)lane - cs;
                if (k < 6u) hdr[k * 64u + S0 - 1] = v;
            }
        }
        return;
    }
    // the run of whole rows ends here: its wave total joins S0's tail lane
    // when it is S0's, else it is added on its own
    uint32_t R = 0;
    if (rslot != 0xFFFFFFFFu) {
        R = wave_total(racc);
        if (rslot != S0) {
            if (lane == 0) atomicAdd(&t.acc[rslot], R);
            R = 0;
        }
        racc = 0;
        rslot = 0xFFFFFFFFu;
    }
    const uint32_t c = row + lane;
    const bool active = c < total;
    // slot of the chunk's first byte: marks of the packets whose first
    // byte-owned chunk falls in this row, max-scanned from S0 at lane 0
    const uint32_t tag = ((row >> 6) + 1u) << 7;
    if (valid && mfirst_v > row && mfirst_v < row + 64) atomicMax(&t.mark[w][mfirst_v - row], tag | (uint32_t)(lane + 1));
    wave_sync();
    const uint32_t m = t.mark[w][lane];
    const bool head = lane > 0 && m >= tag;
    const uint32_t S = wave_incl_max(lane == 0 ? S0 : (m >= tag ? (m & 127u) : 0u));
    // bytes of this chunk in slot S: [0, p); the rest [p, 16) opens slot S + 1
    const int p = (int)t.end[S] - 16 * (int)c;  // >= 1
    const uint32_t val = active ? dot4(v, 0u) : 0u;
    const uint32_t lo = (p >= 16 || !active) ? val : dot4(mask_tail(v, p), 0u);
    const uint32_t inc = wave_incl_scan(lo);
    const bool tail = active && (lane == 63 || p <= 16);
    const bool hd = active && head;
    const uint32_t add = (tail ? inc + (S == S0 ? R : 0u) : 0u) - (hd ? inc - lo : 0u);
    if (tail || hd) atomicAdd(&t.acc[S], add);
    if (active && p < 16) atomicAdd(&t.acc[S + 1], val - lo);
    if (RX && active) {
        if (S >= 1 && S <= nv) {  // the chunk's first byte is in packet S - 1
            const uint32_t k = c - (t.end[S - 1] >> 4);
            if (k < 6u) hdr[k * 64u + S - 1] = v;
        }
        if (p < 16 && S < nv) hdr[S] = v;  // packet S starts inside this chunk: its window chunk 0
    }
    (void)end_v;
    (void)nv;
}

// The tile's 1 KiB rows w, w + W, w + 2W, ... (W = 1: every row), a ring of
// U rows in flight.
template <int U, bool NT, bool RX, int W>
__device__ __forceinline__ void packedb_stream(PackedbLdsT<W>& t, uint32_t w, u32x4* hdr, uint32_t total, int lane,
                                               uintptr_t base, uint32_t start_v, uint32_t end_v, uint32_t mfirst_v,
                                               bool valid, uint32_t nv) {
    if (!total) return;
    // the tile's chunks as a range-checked buffer: reads end at the 16-byte
    // boundary after the tile's last byte
    const buf_t tb = buf_rsrc(reinterpret_cast<const void*>(base), total * 16u);
    u32x4 v[U];
    uint32_t S0 = 0, e0 = 0, racc = 0, rslot = 0xFFFFFFFFu;
#pragma unroll
    for (int u = 0; u < U; u++) {
        v[u] = buf_load<NT>(tb, ((w + W * u) * 64u + lane) * 16u);
        __builtin_amdgcn_sched_barrier(0);  // keep row order
    }
    for (uint32_t c0 = 64u * w; c0 < total; c0 += 64 * U * W) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t row = c0 + u * 64 * W;
            if (row < total)  // wave-uniform
                packedb_reduce_row<RX, W>(t, w, hdr, row, total, lane, v[u], start_v, end_v, mfirst_v, valid, nv, S0,
                                          e0, racc, rslot);
            // unconditional reload (past the tile: zeros, no request), so each
            // reduce waits for its own row only (vmcnt(U-1))
            v[u] = buf_load<NT>(tb, (row + 64u * U * W + lane) * 16u);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    packedb_flush(t, lane, racc, rslot);
}

// Lane-per-segment sum for tiles holding a segment shorter than 16 bytes.
__device__ __forceinline__ uint32_t packedb_lane_sum(uintptr_t base, uint32_t start, uint32_t len) {
    if (!len) return 0u;
    const u32x4* b = reinterpret_cast<const u32x4*>(base);
    const uint32_t c0 = start >> 4, c1 = (start + len - 1) >> 4;
    uint32_t acc = 0;
    for (uint32_t c = c0; c <= c1; c++) {
        const int lo = c == c0 ? (int)(start & 15u) : 0;
        const int hi = (int)(start + len) - 16 * (int)c;
        u32x4 x = load_plain(b + c);
        if (lo != 0 || hi < 16) x = mask_chunk(x, lo, hi);
        acc = dot4(x, acc);
    }
    return acc;
}

// The kernel body.  RX = true (k_packedb_rx: pipck_rx_verify_device,
// pipck_rxdev.hip): each frame's sum feeds rx_device_one (pipck_rxparse.hpp) at
// the tile's end and the ok byte carries the PIPCK_RX_* bits (VERIFY true, no
// pseudo-header).
template <bool VERIFY, int U, bool NT, bool RX, int W>
__device__ __forceinline__ void packedb_body(PackedbLdsT<W>& t, u32x4* hdr, const uint8_t* __restrict__ arena,
                                             const uint16_t* __restrict__ lens, const uint64_t* __restrict__ tile_off,
                                             uint64_t n, const uint32_t* __restrict__ pseudo, uint32_t n_flows,
                                             const uint32_t* __restrict__ flow_of, uint64_t flow_origin,
                                             uint16_t* __restrict__ out, uint8_t* __restrict__ ok,
                                             uint64_t arena_bytes, uint32_t* __restrict__ err) {
    const int lane = threadIdx.x & 63;
    const uint32_t w = W > 1 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0u;
    const uint64_t tile = blockIdx.x;
    const uint64_t seg = tile * 64 + lane;
    const bool valid = seg < n;
    const uint32_t len = valid ? lens[seg] : 0u;
    uint32_t Pbase = 0;
    bool fbad = false;  // a flow_of entry past the table (n_flows bounds it in the _n forms): result 0
    if (pseudo && valid) {  // loaded now so the tile's end waits on nothing
        const uint32_t f0 = (uint32_t)((flow_origin + tile * 64) % n_flows);
        const uint32_t f = flow_of ? flow_of[seg] : (f0 + (uint32_t)lane) % n_flows;
        fbad = f >= n_flows;
        Pbase = fbad ? 0u : pseudo[f];
    }
    const uint32_t nv = (uint32_t)min<uint64_t>(64, n - tile * 64);
    const uint32_t incl = wave_incl_scan(len);
    // The tile's bytes [toff, toff + its lengths) must lie in the arena (scalar,
    // overflow-safe): a tile reaching past arena_bytes -- a stale or foreign
    // index -- reads nothing, sets PIPCK_ERANGE in err and yields 0 for each of
    // its packets, so a wrong index can never take the loads outside the arena.
    const uint64_t toff = tile_off[tile];
    const uint32_t tile_len = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    const bool in_arena = toff <= arena_bytes && (uint64_t)tile_len <= arena_bytes - toff;
    if (!in_arena) {  // (block-uniform: every wave read the same index)
        if (w != 0) return;
        if (lane == 0 && err) atomicOr(err, 1u << PIPCK_ERANGE);
        if (VERIFY)
            store_result8(buf_rsrc(ok + tile * 64, nv), (uint32_t)lane, 0u);
        else
            store_result16(buf_rsrc(out + tile * 64, 2u * nv), 2u * (uint32_t)lane, 0u);
        return;
    }
    const uint64_t first = (uint64_t)(uintptr_t)arena + toff;
    const uintptr_t base = (uintptr_t)(first & ~127ull);  // the line holding the tile's first byte
    const uint32_t excl = incl - len;
    const uint32_t start = (uint32_t)(first - base) + excl;  // relative to base
    const uint32_t end = start + len;
    const uint32_t end_last = (uint32_t)__builtin_amdgcn_readlane((int)end, (int)(nv - 1));
    // slot ends: slot 0 (lead) ends where packet 0 starts; slot s + 1 at packet s's end
    if (w == 0) {  // (every wave holds the same values; one writes them)
        if (lane == 0) t.end[0] = (uint32_t)(first - base);
        t.end[lane + 1] = valid ? end : 0xFFFFFFFFu;  // past the last packet: never ends (trailing bytes)
        if (lane == 0) t.end[65] = 0xFFFFFFFFu;        // (end[64] is lane 63's: a full tile's last packet)
        t.acc[lane] = 0;
        if (lane < 2) t.acc[64 + lane] = 0;
    }
    t.mark[w][lane] = 0;
    if (W > 1)
        __syncthreads();
    else
        wave_sync();
    uint32_t le;
    const bool lane_path = __any(valid && len < 16);  // block-uniform
    if (lane_path) {
        if (w != 0) return;
        le = valid ? packedb_lane_sum(base, start, len) : 0u;
    } else {
        const uint32_t mfirst = (start + 15u) >> 4;  // first chunk whose first byte is in this packet
        const uint32_t total = (end_last + 15u) >> 4;
        packedb_stream<U, NT, RX, W>(t, w, hdr, total, lane, base, start, end, mfirst, valid, nv);
        if (W > 1) {
            __syncthreads();  // every wave's rows are in the slot partials
            if (w != 0) return;  // wave 0 finishes the tile
        } else {
            wave_sync();
        }
        le = t.acc[lane + 1];
    }
    const uint32_t f16 = fold16(le);
    const uint32_t F = (start & 1u) ? f16 : bswap16(f16);  // byte order from the packet's start parity
    const uint32_t P = pseudo ? Pbase + len : 0u;
    uint32_t r;
    if (RX) {  // the frame's header window: captured from the stream, or (lane path) read again
        const uint8_t* pk = reinterpret_cast<const uint8_t*>(base + start);
        uint32_t hw[24];
        if (lane_path) {
            rx_window_global(pk, len, hw);
        } else {
#pragma unroll
            for (int k = 0; k < 6; k++) {  // chunks past the packet's last one: zero (never captured)
                const u32x4 x = 16u * k < (start & 15u) + len ? hdr[k * 64 + lane] : u32x4{0u, 0u, 0u, 0u};
                hw[4 * k] = x.x, hw[4 * k + 1] = x.y, hw[4 * k + 2] = x.z, hw[4 * k + 3] = x.w;
            }
        }
        r = valid ? rx_from_window(pk, len, F, hw) : 0u;
    } else {
        r = VERIFY ? (uint32_t)(fold16(P + F) == 0xFFFFu) : (uint32_t)finish(P, F);
        if (fbad) {
            r = 0;
            if (err) atomicOr(err, 1u << PIPCK_ERANGE);
        }
    }
    if (VERIFY)  // write-through result stores (store_result16); lanes past the batch are range-checked off
        store_result8(buf_rsrc(ok + tile * 64, nv), (uint32_t)lane, r);
    else
        store_result16(buf_rsrc(out + tile * 64, 2u * nv), 2u * (uint32_t)lane, r);
}

// W waves stream one tile together, rows dealt round-robin (wave w: rows w,
// w + W, ...), so a block reads one contiguous window of its tile; slot
// partials meet in the block's LDS and wave 0 finishes the tile.  W = 8 with a
// ring of 3 rows is the default (cfg4: 1.151 ms = 0.900 of peak against 1.188
// ms = 0.873 for one wave per tile with a ring of 32 and 1.173 for 4 waves with
// a ring of 8, profiles/r05_packedb_waves_ab.jsonl), as fast as the loads-only
// block-interleaved stream over the same bytes (1.147 ms,
// profiles/r05_cfg4_ceiling_probe.jsonl).
template <bool VERIFY, int U, bool NT, int W>
__global__ __launch_bounds__(64 * W) void k_packedb(const uint8_t* __restrict__ arena, const uint16_t* __restrict__ lens,
                                                    const uint64_t* __restrict__ tile_off, uint64_t n,
                                                    const uint32_t* __restrict__ pseudo, uint32_t n_flows,
                                                    const uint32_t* __restrict__ flow_of, uint64_t flow_origin,
                                                    uint16_t* __restrict__ out, uint8_t* __restrict__ ok,
                                                    uint64_t arena_bytes, uint32_t* __restrict__ err) {
    __shared__ PackedbLdsT<W> t;
    packedb_body<VERIFY, U, NT, false, W>(t, nullptr, arena, lens, tile_off, n, pseudo, n_flows, flow_of,
                                          flow_origin, out, ok, arena_bytes, err);
}

// received IP frames: the stream, then each tile's headers parsed and judged
template <int U, bool NT, int W>
__global__ __launch_bounds__(64 * W) void k_packedb_rx(const uint8_t* __restrict__ arena,
                                                       const uint16_t* __restrict__ lens,
                                                       const uint64_t* __restrict__ tile_off, uint64_t n,
                                                       uint8_t* __restrict__ ok, uint64_t arena_bytes,
                                                       uint32_t* __restrict__ err) {
    __shared__ PackedbLdsT<W> t;
    __shared__ u32x4 hdr[6 * 64];  // header windows: chunk k of packet s at hdr[k * 64 + s]
    packedb_body<true, U, NT, true, W>(t, hdr, arena, lens, tile_off, n, nullptr, 1u, nullptr, 0, nullptr, ok,
                                       arena_bytes, err);
}

// The (W, U) a launch uses, as W * 100 + U.  Internal tune loads_per_lane 32 =
// one wave per tile with a ring of 32 (the round-4 schedule); 48 = 4 waves,
// ring 8; 72 / 74 = 8 waves, ring 2 / 4 (k_packedb); 28 = 2 waves, ring 16
// (k_packedb_rx).  Defaults, from same-box A/Bs
// (profiles/r05_packedb_waves_ab.jsonl): k_packedb 8 waves with a ring of 3
// (cfg4 1.147-1.150 ms against 1.188 for one wave); k_packedb_rx 4 waves with a
// ring of 8 (1.205-1.209 ms against 1.328-1.336 for one wave, 1.259 for 8
// waves: its tile ends with one wave judging 64 frames, which a narrower block
// overlaps better).
static int packedb_shape(bool rx) {
    switch (g_tune_loads()) {
        case 32: return 132;
        case 48: return 408;
        case 28: return rx ? 216 : 803;
        case 72: return rx ? 408 : 802;
        case 74: return rx ? 408 : 804;
        default: return rx ? 408 : 803;
    }
}

// tile_off[t] = bytes of every packet before packet 64 t (the last entry = the
// batch's bytes): pass 1 sums each tile's lengths into tile_off[t + 1], pass 2
// (one block) turns them into a prefix in place.
__global__ __launch_bounds__(64) void k_packedb_tile_sums(const uint16_t* __restrict__ lens, uint64_t n,
                                                          uint64_t* __restrict__ tile_off) {
    const uint64_t seg = (uint64_t)blockIdx.x * 64 + threadIdx.x;
    const uint32_t tot = wave_total(seg < n ? lens[seg] : 0u);
    if (threadIdx.x == 0) tile_off[blockIdx.x + 1] = tot;
}

__global__ __launch_bounds__(1024) void k_packedb_tile_scan(uint64_t* __restrict__ tile_off, uint64_t n_tiles) {
    __shared__ uint64_t part[1024];
    const uint32_t i = threadIdx.x;
    const uint64_t per = (n_tiles + 1023) / 1024, b = min<uint64_t>(n_tiles, i * per), e = min<uint64_t>(n_tiles, b + per);
    uint64_t s = 0;
    for (uint64_t k = b; k < e; k++) s += tile_off[k + 1];
    part[i] = s;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan of the 1024 partials
        const uint64_t x = i >= off ? part[i - off] : 0ull;
        __syncthreads();
        part[i] += x;
        __syncthreads();
    }
    uint64_t run = part[i] - s;
    for (uint64_t k = b; k < e; k++) {
        run += tile_off[k + 1];
        tile_off[k + 1] = run;
    }
    if (i == 0) tile_off[0] = 0;
}

// bounded: the _n forms (flow_of entries bounded by n_flows when it is given)
static int launch_packedb(bool verify, const void* d_arena, uint64_t arena_bytes, const uint16_t* d_lens,
                          const uint64_t* d_tile_off, uint64_t n, const uint32_t* d_pseudo, uint32_t n_flows,
                          const uint32_t* d_flow_of, uint64_t flow_origin, uint16_t* d_out, uint8_t* d_ok,
                          uint32_t* d_err, hipStream_t s, bool bounded = true) {
    if (n == 0) return PIPCK_OK;
    if (!d_arena || !d_lens || !d_tile_off || (verify ? !d_ok : !d_out)) {
        set_error("pipck_checksum_packed_bytes: null pointer");
        return PIPCK_EINVAL;
    }
    if ((uintptr_t)d_arena % 128) {
        set_error("pipck_checksum_packed_bytes: the arena must be 128-byte aligned");
        return PIPCK_EINVAL;
    }
    if (d_pseudo && !d_flow_of && n_flows == 0) {
        set_error("pipck_checksum_packed_bytes: n_flows == 0");
        return PIPCK_EINVAL;
    }
    const uint64_t tiles = (n + 63) / 64;
    if (tiles > 0x7FFFFFFFull) {
        set_error("pipck_checksum_packed_bytes: more than 2^37 packets in one launch");
        return PIPCK_ERANGE;
    }
    // the kernel's n_flows: the modulus without flow_of; with it, the bound of its entries
    const uint32_t nf = d_flow_of ? (bounded && n_flows ? n_flows : UINT32_MAX) : (n_flows ? n_flows : 1u);
    const uint8_t* a = (const uint8_t*)d_arena;
#define PIPCK_PB(WW, UU)                                                                                       \
    case WW * 100 + UU:                                                                                        \
        if (verify)                                                                                            \
            PIPCK_LAUNCH((k_packedb<true, UU, true, WW>), dim3((uint32_t)tiles), dim3(64 * WW), 0, s, a, d_lens, \
                         d_tile_off, n, d_pseudo, nf, d_flow_of, flow_origin, d_out, d_ok, arena_bytes, d_err);  \
        else                                                                                                   \
            PIPCK_LAUNCH((k_packedb<false, UU, true, WW>), dim3((uint32_t)tiles), dim3(64 * WW), 0, s, a,        \
                         d_lens, d_tile_off, n, d_pseudo, nf, d_flow_of, flow_origin, d_out, d_ok, arena_bytes,   \
                         d_err);                                                                               \
        break
    switch (packedb_shape(false)) {  // non-temporal loads throughout, as k_packed
        PIPCK_PB(1, 32);
        PIPCK_PB(4, 8);
        PIPCK_PB(8, 2);
        PIPCK_PB(8, 4);
        default:
        PIPCK_PB(8, 3);
    }
#undef PIPCK_PB
    PIPCK_LAUNCHED("k_packedb");
    return PIPCK_OK;
}

// pipck_rx_verify_device: the byte-packed stream with the RX verdicts at each
// tile's end (argument checks as pipck_checksum_packed_bytes)
int launch_packedb_rx(const void* d_arena, uint64_t arena_bytes, const uint16_t* d_lens, const uint64_t* d_tile_off,
                      uint64_t n, uint8_t* d_ok, uint32_t* d_err, hipStream_t s) {
    if (n == 0) return PIPCK_OK;
    if (!d_arena || !d_lens || !d_tile_off || !d_ok) {
        set_error("pipck_rx_verify_device: null pointer");
        return PIPCK_EINVAL;
    }
    if ((uintptr_t)d_arena % 128) {
        set_error("pipck_rx_verify_device: the arena must be 128-byte aligned");
        return PIPCK_EINVAL;
    }
    const uint64_t tiles = (n + 63) / 64;
    if (tiles > 0x7FFFFFFFull) {
        set_error("pipck_rx_verify_device: more than 2^37 packets in one launch");
        return PIPCK_ERANGE;
    }
    const uint8_t* a = (const uint8_t*)d_arena;
#define PIPCK_PBRX(WW, UU)                                                                                     \
    case WW * 100 + UU:                                                                                        \
        PIPCK_LAUNCH((k_packedb_rx<UU, true, WW>), dim3((uint32_t)tiles), dim3(64 * WW), 0, s, a, d_lens,       \
                     d_tile_off, n, d_ok, arena_bytes, d_err);                                                 \
        break
    switch (packedb_shape(true)) {
        PIPCK_PBRX(1, 32);
        PIPCK_PBRX(2, 16);
        default:
        PIPCK_PBRX(4, 8);
    }
#undef PIPCK_PBRX
    PIPCK_LAUNCHED("k_packedb_rx");
    return PIPCK_OK;
}

}  // namespace pipck

using namespace pipck;

extern "C" {

int pipck_checksum_packed_bytes_n(const void* d_arena, uint64_t arena_bytes, const uint16_t* d_lens,
                                  const uint64_t* d_tile_off, uint64_t n, const uint32_t* d_pseudo, uint32_t n_flows,
                                  const uint32_t* d_flow_of, uint64_t flow_origin, uint16_t* d_out, uint32_t* d_err,
                                  void* stream) {
    return launch_packedb(false, d_arena, arena_bytes, d_lens, d_tile_off, n, d_pseudo, n_flows, d_flow_of,
                          flow_origin, d_out, nullptr, d_err, as_stream(stream));
}

int pipck_verify_packed_bytes_n(const void* d_arena, uint64_t arena_bytes, const uint16_t* d_lens,
                                const uint64_t* d_tile_off, uint64_t n, const uint32_t* d_pseudo, uint32_t n_flows,
                                const uint32_t* d_flow_of, uint64_t flow_origin, uint8_t* d_ok, uint32_t* d_err,
                                void* stream) {
    return launch_packedb(true, d_arena, arena_bytes, d_lens, d_tile_off, n, d_pseudo, n_flows, d_flow_of,
                          flow_origin, nullptr, d_ok, d_err, as_stream(stream));
}

// the unbounded forms (the index is trusted): every tile's bytes must lie in the arena
int pipck_checksum_packed_bytes(const void* d_arena, const uint16_t* d_lens, const uint64_t* d_tile_off, uint64_t n,
                                const uint32_t* d_pseudo, uint32_t n_flows, const uint32_t* d_flow_of,
                                uint64_t flow_origin, uint16_t* d_out, void* stream) {
    return launch_packedb(false, d_arena, UINT64_MAX, d_lens, d_tile_off, n, d_pseudo, n_flows, d_flow_of,
                          flow_origin, d_out, nullptr, nullptr, as_stream(stream), false);
}

int pipck_verify_packed_bytes(const void* d_arena, const uint16_t* d_lens, const uint64_t* d_tile_off, uint64_t n,
                              const uint32_t* d_pseudo, uint32_t n_flows, const uint32_t* d_flow_of,
                              uint64_t flow_origin, uint8_t* d_ok, void* stream) {
    return launch_packedb(true, d_arena, UINT64_MAX, d_lens, d_tile_off, n, d_pseudo, n_flows, d_flow_of,
                          flow_origin, nullptr, d_ok, nullptr, as_stream(stream), false);
}

int pipck_packed_bytes_index(const uint16_t* d_lens, uint64_t n, uint64_t* d_tile_off, void* stream) {
    if (!d_tile_off || (n && !d_lens)) {
        set_error("pipck_packed_bytes_index: null pointer");
        return PIPCK_EINVAL;
    }
    const uint64_t tiles = (n + 63) / 64;
    if (tiles > 0x7FFFFFFFull) {
        set_error("pipck_packed_bytes_index: more than 2^37 packets");
        return PIPCK_ERANGE;
    }
    hipStream_t s = as_stream(stream);
    if (tiles) {
        hipLaunchKernelGGL(k_packedb_tile_sums, dim3((uint32_t)tiles), dim3(64), 0, s, d_lens, n, d_tile_off);
        PIPCK_LAUNCHED("k_packedb_tile_sums");
    }
    hipLaunchKernelGGL(k_packedb_tile_scan, dim3(1), dim3(1024), 0, s, d_tile_off, tiles);
    PIPCK_LAUNCHED("k_packedb_tile_scan");
    return PIPCK_OK;
}

}  // extern "C"
