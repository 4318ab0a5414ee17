// pipck_rx.hip -- RX verification of received IP packets in host memory.
//
// pip never checks a received checksum (pip/pip_netif.cpp:45-77 dispatches on
// the version nibble; pip/protocol/pip_tcp_input.cpp:11-73,
// pip/protocol/pip_udp.cpp:11-26 and pip/protocol/pip_icmp.cpp:11-20 use the
// headers as they come).  pipck_rx_verify checks a batch of packets as they
// come off the tun device, before pip_netif::input sees them: the IPv4 header
// checksum (pip_ip_checksum, pip/pip_checksum.cpp:35-39) and the TCP / UDP /
// ICMP checksum (pip_inet{,6}_checksum, :42-87, with the stored field included,
// so a packet that verifies sums to 0xFFFF before the final complement).
//
// Round 3-4 built this on the TX queue (two queue adds per packet and its
// chain kernels): ~22 ns of host work per packet, then the queue's kernels one
// after another -- 16K x 1,500-B packets from pinned memory in 0.78 ms, 29 GiB/s.
// Here the host only parses the few header fields that decide WHAT is summed
// (IHL, lengths, fragment field, protocol / extension headers, addresses into
// one pseudo-header partial) into a 24-byte record per packet, and one kernel
// per chunk of packets does the rest: a wave per packet reads the packet's
// bytes in place from pinned host memory (or from a pinned staging copy),
// sums the IPv4 header and the L4 message in one pass with byte masks, and
// writes the packet's ok bits.  Chunks are launched while the host parses the
// next one, so host parsing overlaps the PCIe reads.
#include "pipck_common.hpp"
#include "pipck_device.hpp"

#include <netinet/in.h>

#include <cstring>
#include <vector>

namespace pipck {

// ok bits (include/pipck.h PIPCK_RX_*; include/pip_checksum_amd.h PIP_RX_*)
constexpr uint8_t kRxIpOk = 1, kRxL4Ok = 2, kRxL4Checked = 4;
// record flags
constexpr uint8_t kRecIp = 1, kRecL4 = 2, kRecStaged = 4;

struct RxRec {
    uint64_t addr;    // packet start: a pinned host address, or (kRecStaged) an offset into the staging copy
    uint32_t pseudo;  // L4 pseudo-header partial: proto + address words + length (0 for ICMPv4)
    uint32_t span;    // bytes of the packet the sums cover, from its start
    uint16_t ihl;     // IPv4 header bytes [0, ihl) to verify (kRecIp)
    uint16_t l4off;   // L4 message [l4off, l4off + l4len) (kRecL4)
    uint16_t l4len;
    uint8_t base;     // ok bits the host already decided
    uint8_t flags;
};
static_assert(sizeof(RxRec) == 24, "RxRec layout");

// One wave per packet: lane l holds chunks l, l+64, ... of the packet's
// 16-byte-aligned span (range-checked buffer loads: nothing past the span is
// requested, and the aligned 16-byte blocks around the first and last byte lie
// in those bytes' pages).  Two masked dot2 sums per chunk -- the IPv4 header
// and the L4 message -- then two wave totals.  Byte order: the sums are of
// little-endian words at aligned addresses, fixed once per region from its
// start's parity (be_fold, pipck_device.hpp).
template <int U>
__global__ __launch_bounds__(256) void k_rx_verify(const RxRec* __restrict__ recs, uint32_t n,
                                                   const uint8_t* __restrict__ stage, uint8_t* __restrict__ res) {
    const int lane = threadIdx.x & 63;
    const uint32_t i = blockIdx.x * 4u + (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (i >= n) return;  // wave-uniform
    const RxRec r = recs[i];
    const uint32_t flags = (uint32_t)__builtin_amdgcn_readfirstlane((int)r.flags);
    uint32_t out = r.base;
    if (flags & (kRecIp | kRecL4)) {
        const uint64_t a64 = (flags & kRecStaged) ? (uint64_t)(uintptr_t)stage + r.addr : r.addr;
        const uintptr_t a = (uintptr_t)first_lane_u64(a64);
        const int head = (int)(a & 15u);
        const uint32_t span = (uint32_t)__builtin_amdgcn_readfirstlane((int)r.span);
        const uint32_t nch = ((uint32_t)head + span + 15u) >> 4;
        const buf_t rs = buf_rsrc(reinterpret_cast<const void*>(a - (uintptr_t)head), nch * 16u);
        const int ihl = (flags & kRecIp) ? (int)r.ihl : 0;
        const int lo4 = (int)r.l4off, hi4 = (flags & kRecL4) ? lo4 + (int)r.l4len : lo4;
        uint32_t hs = 0, ls = 0;
        for (uint32_t c0 = 0; c0 < nch; c0 += 64u * U) {  // wave-uniform
            u32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; u++) v[u] = buf_load<false>(rs, (c0 + 64u * u + (uint32_t)lane) * 16u);
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int rel = 16 * (int)(c0 + 64u * u + (uint32_t)lane) - head;  // packet byte at the chunk's byte 0
                hs = dot4(mask_chunk(v[u], max(0, -rel), ihl - rel), hs);
                ls = dot4(mask_chunk(v[u], max(0, lo4 - rel), hi4 - rel), ls);
            }
        }
        if (flags & kRecIp) {  // a header that verifies folds to 0xFFFF in either byte order
            if (fold16(wave_total(hs)) == 0xFFFFu) out |= kRxIpOk;
        }
        if (flags & kRecL4) {
            const uint32_t F = be_fold(wave_total(ls), a + (uintptr_t)lo4);
            out |= kRxL4Checked | (fold16(r.pseudo + F) == 0xFFFFu ? kRxL4Ok : 0u);
        }
    }
    store_result8(buf_rsrc(res + i, 1u), (uint32_t)lane, out);  // lane 0 only (range-checked)
}

static inline uint32_t rd16(const uint8_t* p) { return (uint32_t)p[0] << 8 | p[1]; }

// pip's pseudo-header words of an address (ntohl, hi + lo: pip_checksum.cpp:48-57, 66-84)
static inline uint32_t addr_words(const uint8_t* p, int bytes) {
    uint32_t s = 0;
    for (int k = 0; k < bytes; k += 2) s += rd16(p + k);
    return s;
}

// The upper-layer header of an IPv6 packet: walks the extension headers whose
// presence does not change the pseudo-header (hop-by-hop 0, destination
// options 60, an atomic fragment 44).  1: *proto / *off set; 0: the payload's
// checksum cannot be checked from this packet alone (a real fragment, a
// routing header 43 -- the pseudo-header takes the FINAL destination -- or more
// than 8 extension headers); -1: a header runs past the payload (malformed).
static int ipv6_upper(const uint8_t* b, uint32_t plen, uint8_t* proto, uint32_t* off) {
    const uint32_t end = 40 + plen;
    uint8_t nh = b[6];
    uint32_t at = 40;
    for (int k = 0; k < 8; k++) {
        if (nh != 0 && nh != 60 && nh != 44) {
            *proto = nh;
            *off = at;
            return nh == 43 ? 0 : 1;
        }
        if (at + 8 > end) return -1;
        const uint8_t* e = b + at;
        if (nh == 44) {
            if (rd16(e + 2) & 0xFFF9u) return 0;  // fragment offset (bits 15-3) or M (bit 0) set
            at += 8;
        } else {
            at += 8u * (e[1] + 1u);
        }
        if (at > end) return -1;
        nh = e[0];
    }
    return 0;
}

// What to sum for one received packet (b, len): fills r except addr.
static void rx_parse(const uint8_t* b, uint32_t len, RxRec& r) {
    r = RxRec{};
    if (!b || len < 20) return;  // 0: not an IP packet this can read
    uint8_t proto = 0;
    uint32_t l4off = 0, l4len = 0;
    const bool v4 = (b[0] >> 4) == 4;
    if (v4) {
        const uint32_t ihl = (b[0] & 15u) * 4u, total = rd16(b + 2);
        if (ihl < 20 || total < ihl || total > len) return;  // malformed: 0
        r.flags = kRecIp;
        r.ihl = (uint16_t)ihl;
        r.span = ihl;
        if (rd16(b + 6) & 0x3FFFu) {  // MF or an offset: the L4 checksum spans the reassembled datagram
            r.base |= kRxL4Ok;
            return;
        }
        proto = b[9], l4off = ihl, l4len = total - ihl;
    } else if ((b[0] >> 4) == 6 && len >= 40) {
        const uint32_t plen = rd16(b + 4);
        if (40 + plen > len) return;
        r.base |= kRxIpOk;  // IPv6 has no header checksum
        const int up = ipv6_upper(b, plen, &proto, &l4off);
        if (up < 0) return;  // an extension header past the payload: L4 bits stay clear
        if (up == 0) {
            r.base |= kRxL4Ok;  // not checkable from this packet (fragment, routing header)
            return;
        }
        l4len = 40 + plen - l4off;
    } else {
        return;
    }
    const bool icmp = v4 ? proto == IPPROTO_ICMP : proto == IPPROTO_ICMPV6;
    if (proto != IPPROTO_TCP && proto != IPPROTO_UDP && !icmp) {
        r.base |= kRxL4Ok;  // a protocol without a checksum this knows: unchecked
        return;
    }
    if (l4len < (proto == IPPROTO_TCP ? 20u : 8u)) return;  // truncated: L4 bits stay clear
    const uint8_t* l4 = b + l4off;
    if (proto == IPPROTO_UDP && v4 && !l4[6] && !l4[7]) {
        r.base |= kRxL4Ok;  // UDP over IPv4 without a checksum (RFC 768): unchecked
        return;
    }
    r.flags |= kRecL4;
    r.l4off = (uint16_t)l4off;
    r.l4len = (uint16_t)l4len;
    r.span = l4off + l4len;
    // ICMPv4: pip_ip_checksum over the message alone (RFC 792); TCP, UDP and
    // ICMPv6 (next header 58, RFC 4443 2.3) over their pseudo-headers
    if (!(icmp && v4))
        r.pseudo = proto + (v4 ? addr_words(b + 12, 8) : addr_words(b + 8, 32)) + (l4len >> 16) + (l4len & 0xFFFFu);
}

// A growable pinned, coherent host buffer the kernels read (and write) in place.
struct RxPinned {
    uint8_t* p = nullptr;
    size_t size = 0, cap = 0;
    int reserve(size_t need) {  // the caller makes sure no kernel still reads the old buffer
        if (need <= cap) return PIPCK_OK;
        size_t nc = cap ? cap : (1u << 16);
        while (nc < need) nc *= 2;
        uint8_t* np = nullptr;
        PIPCK_HIP(hipHostMalloc((void**)&np, nc, hipHostMallocCoherent));
        if (size) std::memcpy(np, p, size);
        if (p) (void)hipHostFree(p);
        p = np;
        cap = nc;
        return PIPCK_OK;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        size = cap = 0;
    }
};

// packets per kernel launch: a short first chunk so the GPU starts early, then
// longer ones; consecutive chunks alternate between two streams, so one
// chunk's last waves (waiting on PCIe) overlap the next chunk's first
constexpr uint32_t kRxFirstChunk = 1024, kRxChunk = 4096;

}  // namespace pipck

using namespace pipck;

struct pipck_rxq {
    int device = 0;
    hipStream_t stream[2] = {nullptr, nullptr};
    RxPinned recs, res, stage;         // records, ok bytes, copies of packets outside pinned memory
    std::vector<PinnedRef> held;       // pinned ranges this call reads in place
};

namespace {

// Can [p, p+len) be read in place?  Only inside a pinned range, which this call
// then holds until its kernels have finished (pipck_host_free refuses it meanwhile).
bool rx_hold(pipck_rxq* q, const void* p, uint32_t len) {
    const uintptr_t a = (uintptr_t)p;
    for (size_t i = q->held.size(), k = 0; i-- > 0 && k < 4; k++) {  // the latest few: O(1) per packet
        const PinnedRec& r = *q->held[i];
        if (a >= r.lo && a + len <= r.hi) return true;
    }
    PinnedRef r = pinned_lookup(p, len);
    if (!r || !pinned_acquire(*r)) return false;
    q->held.push_back(std::move(r));
    return true;
}

void rx_drop_holds(pipck_rxq* q) {
    for (PinnedRef& r : q->held) pinned_release(*r);
    q->held.clear();
}

int rx_sync(pipck_rxq* q) {
    for (hipStream_t s : q->stream) PIPCK_HIP(hipStreamSynchronize(s));
    return PIPCK_OK;
}

int rx_launch(pipck_rxq* q, uint32_t first, uint32_t count, uint32_t k) {
    if (!count) return PIPCK_OK;
    hipLaunchKernelGGL(k_rx_verify<4>, dim3((count + 3) / 4), dim3(256), 0, q->stream[k & 1],
                       reinterpret_cast<const RxRec*>(q->recs.p) + first, count, (const uint8_t*)q->stage.p,
                       q->res.p + first);
    PIPCK_LAUNCHED("k_rx_verify");
    return PIPCK_OK;
}

int rx_run(pipck_rxq* q, const void* const* pkts, const uint32_t* lens, uint64_t n, uint8_t* ok, uint64_t* n_verified) {
    int rc;
    if ((rc = q->recs.reserve(n * sizeof(RxRec))) || (rc = q->res.reserve(n)) || (rc = q->stage.reserve(16))) return rc;
    RxRec* recs = reinterpret_cast<RxRec*>(q->recs.p);
    q->stage.size = 0;
    uint32_t launched = 0, chunks = 0;  // records [0, launched) are on the streams
    for (uint64_t i = 0; i < n; i++) {
        RxRec& r = recs[i];
        const uint8_t* b = (const uint8_t*)pkts[i];
        rx_parse(b, lens[i], r);
        if (r.flags && rx_hold(q, b, r.span)) {
            r.addr = (uint64_t)(uintptr_t)b;  // read in place
        } else if (r.flags) {
            // not in pinned memory: a copy in the pinned staging, 16-byte aligned
            const size_t at = (q->stage.size + 15) & ~(size_t)15;
            if (at + r.span > q->stage.cap) {
                // growing frees the old buffer: every kernel that reads it must be done
                if ((rc = rx_sync(q))) return rc;
                if ((rc = q->stage.reserve(at + r.span + (at + r.span) / 2))) return rc;
            }
            std::memcpy(q->stage.p + at, b, r.span);
            q->stage.size = at + r.span;
            r.addr = at;
            r.flags |= kRecStaged;
        }
        if (i + 1 - launched >= (chunks ? kRxChunk : kRxFirstChunk)) {
            if ((rc = rx_launch(q, launched, (uint32_t)(i + 1 - launched), chunks++))) return rc;
            launched = (uint32_t)(i + 1);
        }
    }
    if ((rc = rx_launch(q, launched, (uint32_t)(n - launched), chunks))) return rc;
    if ((rc = rx_sync(q))) return rc;
    uint64_t good = 0;
    for (uint64_t i = 0; i < n; i++) {
        ok[i] = q->res.p[i];
        good += ok[i] == (kRxIpOk | kRxL4Ok | kRxL4Checked);
    }
    if (n_verified) *n_verified = good;
    return PIPCK_OK;
}

}  // namespace

extern "C" {

int pipck_rxq_create(pipck_ctx* ctx, pipck_rxq** out) {
    (void)ctx;
    if (!out) {
        set_error("pipck_rxq_create: null argument");
        return PIPCK_EINVAL;
    }
    *out = nullptr;
    pipck_rxq* q = new pipck_rxq();
    if (hipGetDevice(&q->device) != hipSuccess ||
        hipStreamCreateWithFlags(&q->stream[0], hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&q->stream[1], hipStreamNonBlocking) != hipSuccess) {
        set_error("pipck_rxq_create: no device / stream creation failed");
        if (q->stream[0]) (void)hipStreamDestroy(q->stream[0]);
        delete q;
        return PIPCK_EHIP;
    }
    *out = q;
    return PIPCK_OK;
}

int pipck_rxq_destroy(pipck_rxq* q) {
    if (!q) return PIPCK_OK;
    for (hipStream_t s : q->stream) {
        if (!s) continue;
        (void)hipStreamSynchronize(s);
        (void)hipStreamDestroy(s);
    }
    rx_drop_holds(q);
    q->recs.release();
    q->res.release();
    q->stage.release();
    delete q;
    return PIPCK_OK;
}

int pipck_rx_verify(pipck_rxq* q, const void* const* pkts, const uint32_t* lens, uint64_t n, uint8_t* ok,
                    uint64_t* n_verified) {
    if (n_verified) *n_verified = 0;
    if (!q || (n && (!pkts || !lens || !ok))) {
        set_error("pipck_rx_verify: null argument");
        return PIPCK_EINVAL;
    }
    if (n > 0xFFFFFFFFull) {
        set_error("pipck_rx_verify: more than 2^32 - 1 packets in one call");
        return PIPCK_ERANGE;
    }
    if (!n) return PIPCK_OK;
    int prev = 0;
    PIPCK_HIP(hipGetDevice(&prev));
    if (prev != q->device) PIPCK_HIP(hipSetDevice(q->device));
    int rc = rx_run(q, pkts, lens, n, ok, n_verified);
    if (rc) (void)rx_sync(q);  // nothing may still read what the holds protect
    rx_drop_holds(q);
    if (prev != q->device) (void)hipSetDevice(prev);
    return rc;
}

}  // extern "C"
