// pip_checksum_shim.cpp -- libpip_checksum_amd.so: pip's six checksum
// functions (pip/pip_checksum.h:17-34, plus pip_fold_uint32 at
// pip/pip_checksum.cpp:9) with identical signatures, computed on the MI355X.
//
// Each call marshals its pseudo-header terms (pip_checksum.cpp:45-55, 66-82,
// 92-107, 120-142) into the initial sum and hands the payload bytes -- one
// segment, or every segment of a pip_buf chain in order -- to
// pipck_host_sum(), which replays pip's per-segment loop on the device.
// Contexts are per thread (thread_local), so calls stay reentrant and
// lock-free across pip's TX threads, as pip's own functions are.
#include <netinet/in.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/pip_buf_layout.h"
#include "../../include/pip_checksum_amd.h"
#include "../../include/pipck.h"

namespace {

[[noreturn]] void die(const char* what, int rc) {
    std::fprintf(stderr, "libpip_checksum_amd: %s failed (status %d): %s\n", what, rc, pipck_last_error());
    std::abort();
}

struct ThreadCtx {
    pipck_ctx* ctx = nullptr;
    pipck_txq* txq = nullptr;
    pipck_rxq* rxq = nullptr;  // pip_checksum_amd_verify_packets: received packets, never pip's TX batch
    bool zero_copy = false;  // pip_checksum_amd_zero_copy(): pinned segments read in place at flush
    bool capture = false;    // pip_checksum_amd_capture(): pip's TX calls queue instead of computing
    // Chains whose pinned segments a batch reads in place stay referenced until
    // that batch completes (pip may drop its own references before the flush):
    // `keep` for the batch receiving adds, `keep_inflight` for the submitted one.
    std::vector<std::shared_ptr<pip_buf>> keep, keep_inflight;
    ~ThreadCtx() {
        if (rxq) pipck_rxq_destroy(rxq);
        if (txq) pipck_txq_destroy(txq);  // waits for the in-flight batch
        keep.clear();
        keep_inflight.clear();
        if (ctx) pipck_ctx_destroy(ctx);
    }
    pipck_ctx* get() {
        if (!ctx) {
            int rc = pipck_ctx_create(-1, &ctx);
            if (rc) die("pipck_ctx_create", rc);
        }
        return ctx;
    }
    pipck_txq* queue() {
        if (!txq) {
            int rc = pipck_txq_create(get(), &txq);
            if (rc) die("pipck_txq_create", rc);
        }
        return txq;
    }
};
thread_local ThreadCtx t_ctx;

uint32_t device_sum(const pipck_hseg* segs, uint32_t nseg, uint32_t init) {
    uint32_t out = 0;
    int rc = pipck_host_sum(t_ctx.get(), segs, nseg, init, &out);
    if (rc) die("pipck_host_sum", rc);
    return out;
}

// ntohl() of an address word as stored in memory
uint32_t be32(const void* p) {
    const uint8_t* b = (const uint8_t*)p;
    return (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3];
}
uint32_t split(uint32_t a) { return (a >> 16) + (a & 0xFFFFu); }
uint32_t v4_terms(const in_addr& a) { return split(be32(&a.s_addr)); }
uint32_t v6_terms(const in6_addr& a) {
    uint32_t s = 0;
    for (int i = 0; i < 4; i++) s += split(be32(a.s6_addr + 4 * i));
    return s;
}

// A chain's segments in order (pip_checksum.cpp:145), read through the layout view.
struct ChainSegs {
    pipck_hseg local[8];
    pipck_hseg* segs = local;
    uint32_t n = 0, cap = 8;
    uint32_t total_len = 0;
    explicit ChainSegs(const std::shared_ptr<pip_buf>& buf) {
        const pip_buf_layout* head = reinterpret_cast<const pip_buf_layout*>(buf.get());
        total_len = head->total_len;
        for (const pip_buf_layout* q = head; q; q = q->next) {
            if (n == cap) {
                pipck_hseg* bigger = (pipck_hseg*)std::malloc(sizeof(pipck_hseg) * cap * 2);
                if (!bigger) die("malloc", PIPCK_ENOMEM);
                std::memcpy(bigger, segs, sizeof(pipck_hseg) * n);
                if (segs != local) std::free(segs);
                segs = bigger;
                cap *= 2;
            }
            segs[n++] = pipck_hseg{q->payload, q->payload_len};
        }
    }
    ~ChainSegs() {
        if (segs != local) std::free(segs);
    }
    ChainSegs(const ChainSegs&) = delete;
    ChainSegs& operator=(const ChainSegs&) = delete;
};

void queue_chain(const std::shared_ptr<pip_buf>& buf, uint8_t proto, const void* src, const void* dst, int family,
                 void* csum_field);
uint8_t* capture_field(const std::shared_ptr<pip_buf>& buf, uint8_t proto);

uint16_t chain_checksum(const std::shared_ptr<pip_buf>& buf, uint32_t pseudo) {
    ChainSegs c(buf);
    // length term: the head's u32 total_len split hi + lo (pip_checksum.cpp:140-142)
    const uint32_t sum = device_sum(c.segs, c.n, pseudo + split(c.total_len));
    return (uint16_t)~(uint16_t)sum;
}

}  // namespace

uint32_t pip_fold_uint32(uint32_t num) { return (num & 0x0000FFFFu) + (num >> 16); }

uint32_t pip_standard_checksum(const void* payload, uint32_t len, uint32_t sum) {
    pipck_hseg s{payload, len};
    return device_sum(&s, 1, sum);
}

uint16_t pip_ip_checksum(const void* payload, uint32_t len) {
    if (t_ctx.capture && payload && len >= 20) {  // ip_sum at byte 10 (pip/pip_netif.cpp:94-97)
        pip_ip_checksum_deferred(payload, len, (uint8_t*)payload + 10);
        return 0;  // the caller stores htons(0); the flush stores the checksum over it
    }
    return (uint16_t)~(uint16_t)pip_standard_checksum(payload, len, 0);
}

uint16_t pip_inet_checksum(const void* payload, uint8_t proto, struct in_addr src, struct in_addr dst,
                           uint16_t len) {
    const uint32_t pseudo = v4_terms(src) + v4_terms(dst) + proto + len;
    return (uint16_t)~(uint16_t)pip_standard_checksum(payload, len, pseudo);
}

uint16_t pip_inet6_checksum(const void* payload, uint8_t proto, struct in6_addr src, struct in6_addr dst,
                            uint16_t len) {
    const uint32_t pseudo = v6_terms(src) + v6_terms(dst) + proto + len;
    return (uint16_t)~(uint16_t)pip_standard_checksum(payload, len, pseudo);
}

uint16_t pip_inet_checksum_buf(std::shared_ptr<pip_buf> buf, uint8_t proto, struct in_addr src, struct in_addr dst) {
    if (t_ctx.capture)
        if (uint8_t* field = capture_field(buf, proto)) {
            queue_chain(buf, proto, &src.s_addr, &dst.s_addr, 4, field);
            return 0;  // the caller stores htons(0); the flush stores the checksum over it
        }
    return chain_checksum(buf, v4_terms(src) + v4_terms(dst) + proto);
}

uint16_t pip_inet6_checksum_buf(std::shared_ptr<pip_buf> buf, uint8_t proto, struct in6_addr src,
                                struct in6_addr dst) {
    if (t_ctx.capture)
        if (uint8_t* field = capture_field(buf, proto)) {
            queue_chain(buf, proto, src.s6_addr, dst.s6_addr, 6, field);
            return 0;
        }
    return chain_checksum(buf, v6_terms(src) + v6_terms(dst) + proto);
}

// ---- deferred forms (batched TX path) -------------------------------------
// The queue computes the pseudo-header from the addresses itself and takes the
// length term from the queued bytes, which for a pip_buf chain equals the
// head's total_len (pip/pip_buf.h:81-97 keeps it as the sum of the segments).
namespace {

void queue_chain(const std::shared_ptr<pip_buf>& buf, uint8_t proto, const void* src, const void* dst, int family,
                 void* csum_field) {
    ChainSegs c(buf);
    pipck_txq* q = t_ctx.queue();
    int rc = family == 4 ? pipck_txq_add4(q, c.segs, c.n, proto, *(const uint32_t*)src, *(const uint32_t*)dst,
                                          csum_field)
                         : pipck_txq_add6(q, c.segs, c.n, proto, (const uint8_t*)src, (const uint8_t*)dst, csum_field);
    if (rc) die(family == 4 ? "pipck_txq_add4" : "pipck_txq_add6", rc);
    if (t_ctx.zero_copy) t_ctx.keep.push_back(buf);  // its pinned segments are read at flush time
}

// Where pip's TX callers store a chain's checksum: th_sum at byte 16 of the TCP
// header segment (pip/protocol/pip_tcp_packet.cpp:132-133), uh_sum at byte 6
// of the UDP header segment (pip/protocol/pip_udp.cpp:50-51, 60-61); null for
// anything else (computed synchronously even in capture mode).
uint8_t* capture_field(const std::shared_ptr<pip_buf>& buf, uint8_t proto) {
    const pip_buf_layout* head = reinterpret_cast<const pip_buf_layout*>(buf.get());
    if (!head || !head->payload) return nullptr;
    if (proto == IPPROTO_TCP && head->payload_len >= 20) return (uint8_t*)head->payload + 16;
    if (proto == IPPROTO_UDP && head->payload_len >= 8) return (uint8_t*)head->payload + 6;
    return nullptr;
}

}  // namespace

void pip_inet_checksum_buf_deferred(std::shared_ptr<pip_buf> buf, uint8_t proto, struct in_addr src,
                                    struct in_addr dst, void* csum_field) {
    queue_chain(buf, proto, &src.s_addr, &dst.s_addr, 4, csum_field);
}

void pip_inet6_checksum_buf_deferred(std::shared_ptr<pip_buf> buf, uint8_t proto, struct in6_addr src,
                                     struct in6_addr dst, void* csum_field) {
    queue_chain(buf, proto, src.s6_addr, dst.s6_addr, 6, csum_field);
}

void pip_ip_checksum_deferred(const void* hdr, uint32_t len, void* csum_field) {
    int rc = pipck_txq_add_ip(t_ctx.queue(), hdr, len, csum_field);
    if (rc) die("pipck_txq_add_ip", rc);
}

uint64_t pip_checksum_amd_pending() { return pipck_txq_pending(t_ctx.queue()); }

void pip_checksum_amd_submit() {
    int rc = pipck_txq_submit(t_ctx.queue());
    if (rc) die("pipck_txq_submit", rc);
    // the batch submitted before this one has completed; this one is in flight now
    t_ctx.keep_inflight.clear();
    t_ctx.keep_inflight.swap(t_ctx.keep);
}

void pip_checksum_amd_complete() {
    int rc = pipck_txq_complete(t_ctx.queue());
    if (rc) die("pipck_txq_complete", rc);
    t_ctx.keep_inflight.clear();
}

void pip_checksum_amd_flush() {
    pip_checksum_amd_submit();
    pip_checksum_amd_complete();
}

void pip_checksum_amd_zero_copy(bool on) {
    int rc = pipck_txq_auto_zero_copy(t_ctx.queue(), on ? 1 : 0);
    if (rc) die("pipck_txq_auto_zero_copy", rc);
    t_ctx.zero_copy = on;
}

void pip_checksum_amd_resident(bool on) {
    int rc = pipck_ctx_zero_copy(t_ctx.get(), on ? 3 : 2);
    if (rc) die("pipck_ctx_zero_copy", rc);
}

void pip_checksum_amd_capture(bool on) { t_ctx.capture = on; }

// ---- RX batch verification ------------------------
// pip never checks a received checksum (pip/pip_netif.cpp:45-77,
// pip/protocol/pip_tcp_input.cpp, pip/protocol/pip_udp.cpp:11-26).  Received
// packets go to this thread's RX queue (pipck_rx_verify, pip_amd/csrc/
// pipck_rx.hip): the host parses what each checksum covers, one kernel per
// chunk of packets sums and checks them, reading packets in pinned memory in
// place.  pip's deferred TX batch is not touched.
namespace {

pipck_rxq* rx_queue() {
    if (!t_ctx.rxq) {
        int rc = pipck_rxq_create(t_ctx.get(), &t_ctx.rxq);
        if (rc) die("pipck_rxq_create", rc);
    }
    return t_ctx.rxq;
}

}  // namespace

uint32_t pip_checksum_amd_rx_abi(void) { return PIP_CHECKSUM_AMD_RX_ABI; }

uint32_t pip_checksum_amd_verify_packets(const void* const* pkts, const uint32_t* lens, uint32_t n, uint8_t* ok) {
    if (!n) return 0;
    if (!pkts || !lens || !ok) die("pip_checksum_amd_verify_packets: null argument", PIPCK_EINVAL);
    static_assert(PIP_RX_IP_OK == PIPCK_RX_IP_OK && PIP_RX_L4_OK == PIPCK_RX_L4_OK &&
                      PIP_RX_L4_CHECKED == PIPCK_RX_L4_CHECKED && PIP_RX_VERIFIED == PIPCK_RX_VERIFIED,
                  "the drop-in's RX bits are pipck_rx_verify's");
    uint64_t good = 0;
    // Packets back to back in one buffer (a receive buffer read in order): one
    // DMA per chunk and the device verifier (pipck_host_rx_verify_packed: 2.2x
    // on 64-B frames, PCIe rate from pageable memory); same verdict bits.
    bool contiguous = pkts[0] != nullptr;
    for (uint32_t i = 0; contiguous && i < n; i++)
        contiguous = lens[i] <= 0xFFFFu && (i + 1 == n || (const uint8_t*)pkts[i + 1] == (const uint8_t*)pkts[i] + lens[i]);
    if (contiguous && n > 1) {
        std::vector<uint16_t> l16(lens, lens + n);
        int rc = pipck_host_rx_verify_packed(t_ctx.get(), pkts[0], l16.data(), n, ok, &good);
        if (rc) die("pipck_host_rx_verify_packed", rc);
        return (uint32_t)good;
    }
    int rc = pipck_rx_verify(rx_queue(), pkts, lens, n, ok, &good);
    if (rc) die("pipck_rx_verify", rc);
    return (uint32_t)good;
}

bool pip_checksum_amd_capturing() { return t_ctx.capture; }
