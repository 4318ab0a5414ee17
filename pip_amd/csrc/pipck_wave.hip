// pipck_wave.hip -- the BASELINE north_star's literal kernel shape, kept as a
// measurement arm: ONE PACKET PER WAVEFRONT.
//
// Hot path: plumk97/pip pip/pip_checksum.cpp:42-87 (pip_inet{,6}_checksum),
// :35-39 (pip_ip_checksum) over fixed-stride and descriptor (ragged) batches.
//
// BASELINE.json's north_star sketches the kernel as "one packet per wavefront,
// coalesced HBM loads of the payload, ... partial sums with a wavefront reduce
// to the final 16-bit fold".  k_wave is exactly that: wave w of block b takes
// packet 4b + w, lane l loads chunks l, l + 64, ... of the packet (each load
// instruction one coalesced 1 KiB row of the packet), all of a packet's loads
// are issued before the first add (NL per lane per pass, range-checked: lanes
// past the packet send no request), each lane keeps a u32 partial, and one DPP
// wave reduce + two folds give the packet's sum; lane 0 adds the flow's
// pseudo-header (loaded before the payload) and stores the result.
//
// The shipped kernels are NOT this shape ("one packet per
// wavefront"): a packet is 1.5-9 KiB, so a wave holds at most one packet's
// bytes in flight and every packet pays a wave's dispatch, pseudo-header load,
// reduce and 2-byte store; the streaming kernels instead give a wave (or a
// block) many packets as one contiguous row stream.  Selected only through the
// internal tune hook (pipck_testing.h: lanes_per_packet = 256), for the GPU
// parity tests and tools/wave_ab.py.
#include "pipck_common.hpp"
#include "pipck_device.hpp"

namespace pipck {

template <int NL, bool VERIFY, bool DESC>
__global__ __launch_bounds__(256) void k_wave(const uint8_t* __restrict__ arena, uint64_t stride, uint32_t len,
                                              const pipck_desc* __restrict__ desc, uint64_t n,
                                              const uint32_t* __restrict__ pseudo, uint32_t n_flows,
                                              const uint32_t* __restrict__ flow_of, uint64_t flow_origin,
                                              uint16_t* __restrict__ out, uint8_t* __restrict__ ok,
                                              uint32_t* __restrict__ err, uint64_t arena_bytes) {
    const int lane = threadIdx.x & 63;
    const uint64_t pkt = (uint64_t)blockIdx.x * 4u + (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (pkt >= n) return;  // wave-uniform
    uint64_t off;
    uint32_t L, flow = 0;
    bool bad = false;
    if (DESC) {
        const pipck_desc d = desc[pkt];
        off = first_lane_u64(d.offset);
        L = (uint32_t)__builtin_amdgcn_readfirstlane((int)d.len);
        flow = (uint32_t)__builtin_amdgcn_readfirstlane((int)d.flow);
        // out of domain (as k_ragged): too long, past the arena, or a flow past the table
        bad = L > PIPCK_MAX_SEG_LEN || off > arena_bytes || (uint64_t)L > arena_bytes - off ||
              (pseudo && flow >= n_flows);
        if (bad) L = 0, flow = 0;
    } else {
        off = pkt * stride;
        L = len;
        if (pseudo) flow = flow_of ? flow_of[pkt] : (uint32_t)((flow_origin + pkt) % n_flows);
        // a flow_of entry past the table (n_flows bounds it in the _n forms): result 0
        bad = pseudo && flow_of && flow >= n_flows;
        if (bad) L = 0, flow = 0;
    }
    const uint32_t Pb = pseudo ? pseudo[flow] : 0u;  // issued before the payload: ready at the end
    const uintptr_t addr = (uintptr_t)arena + off;
    const int head = (int)(addr & 15u);
    const uint32_t nch = L ? ((uint32_t)head + L + 15u) >> 4 : 0u;
    const buf_t r = buf_rsrc(reinterpret_cast<const void*>(addr - (uintptr_t)head), nch * 16u);
    uint32_t acc = 0;
    for (uint32_t c0 = 0; c0 < nch; c0 += 64u * NL) {  // one pass for packets up to NL KiB
        u32x4 v[NL];
#pragma unroll
        for (int k = 0; k < NL; k++) v[k] = buf_load<true>(r, (c0 + 64u * k + (uint32_t)lane) * 16u);
#pragma unroll
        for (int k = 0; k < NL; k++) {
            const int rel = 16 * (int)(c0 + 64u * k + (uint32_t)lane) - head;  // packet byte at the chunk's byte 0
            acc = dot4(mask_chunk(v[k], max(0, -rel), (int)L - rel), acc);
        }
    }
    const uint32_t F = bad ? 0u : be_fold(wave_total(acc), addr);
    if (lane == 0) {
        const uint32_t P = pseudo ? Pb + len_term(L) : 0u;
        if (VERIFY)
            ok[pkt] = !bad && fold16(P + F) == 0xFFFFu;
        else
            out[pkt] = bad ? (uint16_t)0 : finish(P, F);
        if (bad && err) atomicOr(err, 1u << PIPCK_ERANGE);
    }
}

typedef void (*wave_fn)(const uint8_t*, uint64_t, uint32_t, const pipck_desc*, uint64_t, const uint32_t*, uint32_t,
                        const uint32_t*, uint64_t, uint16_t*, uint8_t*, uint32_t*, uint64_t);

// loads per lane per pass: 2 for packets up to 2 KiB, 4 above (cfg3 / cfg5 at
// 4: 0.85 / 0.84 of HBM peak against 0.71-0.73 / 0.69-0.71 at 8 and 16, which
// cover a jumbo packet in one pass; profiles/r04_wave_per_packet_ab.jsonl), or
// the caller's override
int launch_wave(bool verify, bool desc, const void* d_arena, uint64_t stride, uint32_t len, const pipck_desc* d_desc,
                uint64_t n, const uint32_t* d_pseudo, uint32_t n_flows, const uint32_t* d_flow_of,
                uint64_t flow_origin, uint16_t* d_out, uint8_t* d_ok, uint32_t* d_err, hipStream_t s,
                uint32_t max_chunks, uint32_t nl, uint64_t arena_bytes) {
    static const wave_fn kWave[4][2][2] = {  // [NL 2/4/8/16][verify][desc]
        {{k_wave<2, false, false>, k_wave<2, false, true>}, {k_wave<2, true, false>, k_wave<2, true, true>}},
        {{k_wave<4, false, false>, k_wave<4, false, true>}, {k_wave<4, true, false>, k_wave<4, true, true>}},
        {{k_wave<8, false, false>, k_wave<8, false, true>}, {k_wave<8, true, false>, k_wave<8, true, true>}},
        {{k_wave<16, false, false>, k_wave<16, false, true>}, {k_wave<16, true, false>, k_wave<16, true, true>}}};
    if (!nl) nl = max_chunks <= 128 ? 2u : 4u;
    const int ni = nl >= 16 ? 3 : (nl >= 8 ? 2 : (nl >= 4 ? 1 : 0));
    const uint64_t blocks = (n + 3) / 4;
    if (blocks > 0x7FFFFFFFull) {
        set_error("k_wave: batch too large for one launch");
        return PIPCK_ERANGE;
    }
    PIPCK_LAUNCH(kWave[ni][verify][desc], dim3((uint32_t)blocks), dim3(256), 0, s, (const uint8_t*)d_arena, stride,
                 len, d_desc, n, d_pseudo, n_flows ? n_flows : 1u, d_flow_of, flow_origin, d_out, d_ok, d_err, arena_bytes);
    PIPCK_LAUNCHED("k_wave");
    return PIPCK_OK;
}

}  // namespace pipck
