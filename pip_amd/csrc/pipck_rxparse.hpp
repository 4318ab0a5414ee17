// pipck_rxparse.hpp -- device-side parse + verdict of one received IP packet
// (pipck_rx_verify_device; see pipck_rxdev.hip for the design).  Included by
// pipck_packedb.hip, whose k_packedb_rx calls rx_from_window at each tile's end
// with the frame sum it has just streamed and the header window it captured
// (rx_device_one reads the window from memory: tiles with a frame under 16 B).
#pragma once
#include "pipck_device.hpp"

namespace pipck {

constexpr uint32_t kOkIp = 1, kOkL4 = 2, kL4Checked = 4;  // PIPCK_RX_* (include/pipck.h)
constexpr int kWinWords = 20;                             // 80 bytes realigned to the packet start

// Byte j (compile-time or run-time) of the realigned window; 0 past it.
__device__ __forceinline__ uint32_t win_byte(const uint32_t (&a)[kWinWords], uint32_t j) {
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < kWinWords; k++)
        if ((uint32_t)k == (j >> 2)) x = a[k];
    return (x >> (8u * (j & 3u))) & 0xFFu;
}
__device__ __forceinline__ uint32_t win_be16(const uint32_t (&a)[kWinWords], uint32_t j) {
    return win_byte(a, j) << 8 | win_byte(a, j + 1);
}

// Little-endian 16-bit word sum (dot2 partial) of bytes [lo, hi) of the window.
__device__ __forceinline__ uint32_t win_sum(const uint32_t (&a)[kWinWords], uint32_t lo, uint32_t hi) {
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kWinWords; k++) {
        const int b0 = 4 * k;
        const int l = max(0, (int)lo - b0), h = min(4, (int)hi - b0);  // bytes [l, h) of word k
        if (h <= l) continue;
        const uint32_t m = (h >= 4 ? 0xFFFFFFFFu : ((1u << (8 * h)) - 1u)) & ~((1u << (8 * l)) - 1u);
        s = dot_fold(a[k] & m, s);
    }
    return s;
}

// The same LE word sum of packet bytes [lo, hi) read from memory one byte at a
// time (ranges past the 80-byte window: long extension headers, long link
// padding -- rare).  Offsets are relative to the packet start p.
__device__ inline uint32_t mem_sum(const uint8_t* p, uint32_t lo, uint32_t hi) {
    uint32_t s = 0;
    for (uint32_t j = lo; j < hi; j++) s += (uint32_t)p[j] << (8u * (j & 1u));
    return fold16(s);
}
__device__ inline bool mem_any(const uint8_t* p, uint32_t lo, uint32_t hi) {
    for (uint32_t j = lo; j < hi; j++)
        if (p[j]) return true;
    return false;
}
__device__ __forceinline__ uint32_t mem_byte(const uint8_t* p, const uint32_t (&a)[kWinWords], uint32_t j) {
    return j < 4u * kWinWords ? win_byte(a, j) : (uint32_t)p[j];
}

// LE word sum of packet bytes [lo, hi), window first, memory past it.
__device__ __forceinline__ uint32_t range_sum(const uint8_t* p, const uint32_t (&a)[kWinWords], uint32_t lo,
                                              uint32_t hi) {
    uint32_t s = lo < 4u * kWinWords ? win_sum(a, lo, min(hi, 4u * kWinWords)) : 0u;
    if (hi > 4u * kWinWords) s += mem_sum(p, max(lo, 4u * kWinWords), hi);
    return s;
}

// One packet: p its first byte (any alignment), len its frame bytes, sall the
// folded big-endian sum of the whole frame from pass 1.  Returns the ok bits
// pipck_rx_verify gives the same bytes (rx_parse + k_rx_verify, pipck_rx.hip).
// The packet's first six aligned 16-byte chunks (from the one holding byte 0),
// none past the one holding its last byte.
__device__ __forceinline__ void rx_window_global(const uint8_t* p, uint32_t len, uint32_t (&w)[24]) {
    // (global loads with a per-lane guard: a buffer resource is scalar, and one
    // per lane made the compiler loop over the wave's 64 packet addresses)
    const uint32_t h = (uint32_t)((uintptr_t)p & 15u);
    const u32x4* base = reinterpret_cast<const u32x4*>(p - h);
#pragma unroll
    for (int c = 0; c < 6; c++) {
        const u32x4 v = 16u * c < h + len ? load_plain(base + c) : u32x4{0u, 0u, 0u, 0u};
        w[4 * c] = v.x, w[4 * c + 1] = v.y, w[4 * c + 2] = v.z, w[4 * c + 3] = v.w;
    }
}

// One packet whose window w (rx_window_global's chunks; chunks past the one
// holding the last byte zero) is already in registers.
__device__ inline uint32_t rx_from_window(const uint8_t* p, uint32_t len, uint32_t sall, const uint32_t (&w)[24]) {
    if (len < 20) return 0;
    const uint32_t h = (uint32_t)((uintptr_t)p & 15u);
    // (bytes after the frame in its last chunk belong to the next packet and
    // are never used: every range below ends <= len)
    // realign: a[k] = bytes [4k, 4k + 4) of the packet
    // (shifts by 2 and 1 words as masked blends: written as selects, the
    // compiler turned them into an indexed copy through scratch memory)
    const uint32_t q = h >> 2, r = h & 3u;
    const uint32_t m2 = 0u - ((q >> 1) & 1u), m1 = 0u - (q & 1u);
    uint32_t u[23], a[kWinWords];
#pragma unroll
    for (int k = 0; k < 22; k++) u[k] = w[k] ^ ((w[k] ^ w[k + 2]) & m2);
    u[22] = w[22] & ~m2;
#pragma unroll
    for (int k = 0; k < 21; k++) u[k] = u[k] ^ ((u[k] ^ u[k + 1]) & m1);
#pragma unroll
    for (int k = 0; k < kWinWords; k++) a[k] = __builtin_amdgcn_alignbyte(u[k + 1], u[k], r);

    const uint32_t b0 = a[0] & 0xFFu;
    uint32_t out = 0, ip_end, l4off, proto;
    uint32_t le_pre;  // LE sum of [0, l4off)
    uint32_t pseudo_addr;
    const bool v4 = (b0 >> 4) == 4;
    if (v4) {
        const uint32_t ihl = (b0 & 15u) * 4u, total = win_be16(a, 2);
        if (ihl < 20 || total < ihl || total > len) return 0;  // malformed
        uint32_t hs = 0;  // the whole header, exactly (<= 60 bytes: inside the window)
#pragma unroll
        for (int k = 0; k < 15; k++)
            if ((uint32_t)k < ihl / 4u) hs = dot_fold(a[k], hs);
        if (fold16(hs) == 0xFFFFu) out |= kOkIp;  // either byte order
        if (win_be16(a, 6) & 0x3FFFu) return out | kOkL4;  // a fragment: L4 unchecked
        proto = win_byte(a, 9);
        l4off = ihl;
        ip_end = total;
        le_pre = hs;
        pseudo_addr = bswap16(fold16(dot_fold(a[3], dot_fold(a[4], 0u))));  // [12, 20)
    } else if ((b0 >> 4) == 6 && len >= 40) {
        const uint32_t plen = win_be16(a, 4);
        if (40 + plen > len) return 0;
        out = kOkIp;  // no IPv6 header checksum
        ip_end = 40 + plen;
        // the upper-layer header (ipv6_upper in pipck_rx.hip): hop-by-hop 0,
        // destination options 60 and atomic fragments 44 are walked
        uint32_t nh = win_byte(a, 6), at = 40;
        int up = 0;
        for (int k = 0; k < 8; k++) {
            if (nh != 0 && nh != 60 && nh != 44) {
                up = nh == 43 ? 0 : 1;
                break;
            }
            if (at + 8 > ip_end) {
                up = -1;
                break;
            }
            const uint32_t next = mem_byte(p, a, at);
            if (nh == 44) {
                if (((mem_byte(p, a, at + 2) << 8) | mem_byte(p, a, at + 3)) & 0xFFF9u) break;  // up = 0
                at += 8;
            } else {
                at += 8u * (mem_byte(p, a, at + 1) + 1u);
            }
            if (at > ip_end) {
                up = -1;
                break;
            }
            nh = next;
        }
        if (up < 0) return out;             // an extension header past the payload
        if (up == 0) return out | kOkL4;    // fragment, routing header: unchecked
        proto = nh;
        l4off = at;
        if (l4off == 40) {  // no extension headers (the common case): the fixed header's ten words
            uint32_t f = 0;
#pragma unroll
            for (int k = 0; k < 10; k++) f = dot_fold(a[k], f);
            le_pre = f;
        } else {
            le_pre = range_sum(p, a, 0, l4off);
        }
        uint32_t s = 0;
#pragma unroll
        for (int k = 2; k < 10; k++) s = dot_fold(a[k], s);  // [8, 40)
        pseudo_addr = bswap16(fold16(s));
    } else {
        return 0;
    }
    const bool icmp = v4 ? proto == 1u : proto == 58u;
    if (proto != 6u && proto != 17u && !icmp) return out | kOkL4;  // no checksum this knows
    const uint32_t l4len = ip_end - l4off;
    if (l4len < (proto == 6u ? 20u : 8u)) return out;  // truncated: L4 bits clear
    if (proto == 17u && v4) {  // the UDP checksum field, bytes l4off + 6 and + 7 (static when IHL is 5)
        const uint32_t f = l4off == 20 ? (a[6] >> 16) : (win_byte(a, l4off + 6) | win_byte(a, l4off + 7));
        if (!f) return out | kOkL4;
    }
    // S_l4 = S_all - S_pre - S_post, all big-endian relative to the packet start
    const uint32_t pre = bswap16(fold16(le_pre));
    const uint32_t post = ip_end < len ? bswap16(fold16(range_sum(p, a, ip_end, len))) : 0u;
    const uint32_t x = sall + (0xFFFFu - pre) + (0xFFFFu - post);
    out |= kL4Checked;
    if (icmp && v4) {  // no pseudo-header: an all-zero message sums to 0, not 0xFFFF
        const bool nonzero = (win_sum(a, l4off, l4off + 8) != 0) || mem_any(p, l4off + 8, ip_end);
        if (nonzero && fold16(x) == 0xFFFFu) out |= kOkL4;
        return out;
    }
    const uint32_t P = proto + pseudo_addr + (l4len >> 16) + (l4len & 0xFFFFu);
    if (fold16(P + x) == 0xFFFFu) out |= kOkL4;
    return out;
}

__device__ inline uint32_t rx_device_one(const uint8_t* p, uint32_t len, uint32_t sall) {
    uint32_t w[24];
    rx_window_global(p, len, w);
    return rx_from_window(p, len, sall, w);
}

}  // namespace pipck
