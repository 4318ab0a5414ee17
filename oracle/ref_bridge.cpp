// ref_bridge.cpp -- TEST INFRASTRUCTURE ONLY.
//
// extern "C" entry points over the REAL reference functions of
// /root/reference/pip/pip_checksum.cpp, so Python tests (ctypes) and the
// bench's cpu_baseline leg can call pip's own code.  Compiled against the
// reference's headers where they lie (oracle/Makefile, target `ref`); the
// output goes to oracle/_ref/ only.  Nothing from the reference is copied
// into this repository.
#include "pip_checksum.h"

#include <cstring>
#include <thread>
#include <vector>

// Exported by pip_checksum.cpp:9 but not declared in its header.
pip_uint32 pip_fold_uint32(pip_uint32 num);

extern "C" {

uint32_t ref_fold_uint32(uint32_t x) { return pip_fold_uint32(x); }

uint32_t ref_standard_checksum(const void* p, uint32_t len, uint32_t sum) {
    return pip_standard_checksum(p, len, sum);
}

uint16_t ref_ip_checksum(const void* p, uint32_t len) { return pip_ip_checksum(p, len); }

uint16_t ref_inet_checksum(const void* p, uint8_t proto, uint32_t src, uint32_t dst, uint16_t len) {
    pip_in_addr s, d;
    s.s_addr = src;
    d.s_addr = dst;
    return pip_inet_checksum(p, proto, s, d, len);
}

uint16_t ref_inet6_checksum(const void* p, uint8_t proto, const uint8_t* src, const uint8_t* dst,
                            uint16_t len) {
    pip_in6_addr s, d;
    std::memcpy(&s, src, 16);
    std::memcpy(&d, dst, 16);
    return pip_inet6_checksum(p, proto, s, d, len);
}

static std::shared_ptr<pip_buf> make_chain(const void* const* segs, const uint32_t* lens, uint32_t nseg) {
    std::shared_ptr<pip_buf> head, tail;
    std::vector<std::shared_ptr<pip_buf>> all;
    for (uint32_t i = 0; i < nseg; i++) all.push_back(std::make_shared<pip_buf>(segs[i], lens[i], 0));
    // link back to front so total_len propagates the way pip builds chains
    for (int i = (int)nseg - 2; i >= 0; i--) all[i]->set_next(all[i + 1]);
    return nseg ? all[0] : std::make_shared<pip_buf>(nullptr, 0, 0);
}

uint16_t ref_inet_checksum_chain(const void* const* segs, const uint32_t* lens, uint32_t nseg, uint8_t proto,
                                 uint32_t src, uint32_t dst) {
    pip_in_addr s, d;
    s.s_addr = src;
    d.s_addr = dst;
    return pip_inet_checksum_buf(make_chain(segs, lens, nseg), proto, s, d);
}

uint16_t ref_inet6_checksum_chain(const void* const* segs, const uint32_t* lens, uint32_t nseg, uint8_t proto,
                                  const uint8_t* src, const uint8_t* dst) {
    pip_in6_addr s, d;
    std::memcpy(&s, src, 16);
    std::memcpy(&d, dst, 16);
    return pip_inet6_checksum_buf(make_chain(segs, lens, nseg), proto, s, d);
}

// CPU baseline: pip's own pip_inet{,6}_checksum / pip_ip_checksum over a
// fixed-stride batch, on `threads` std::threads with contiguous shards.
// flows4: n_flows x {src s_addr, dst s_addr}; flows6: n_flows x 32 bytes.
void ref_batch_fixed(const uint8_t* arena, uint64_t stride, uint32_t len, uint64_t n, int family, uint8_t proto,
                     const uint32_t* flows4, const uint8_t* flows6, uint32_t n_flows, uint64_t flow_origin,
                     uint16_t* out, int threads) {
    if (threads < 1) threads = 1;
    auto work = [&](uint64_t b, uint64_t e) {
        for (uint64_t i = b; i < e; i++) {
            const uint8_t* p = arena + i * stride;
            uint32_t f = (uint32_t)((flow_origin + i) % n_flows);
            if (family == 4) {
                pip_in_addr s, d;
                s.s_addr = flows4[2 * f];
                d.s_addr = flows4[2 * f + 1];
                out[i] = pip_inet_checksum(p, proto, s, d, (pip_uint16)len);
            } else if (family == 6) {
                pip_in6_addr s, d;
                std::memcpy(&s, flows6 + 32 * f, 16);
                std::memcpy(&d, flows6 + 32 * f + 16, 16);
                out[i] = pip_inet6_checksum(p, proto, s, d, (pip_uint16)len);
            } else {
                out[i] = pip_ip_checksum(p, len);
            }
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < threads; t++) th.emplace_back(work, n * t / threads, n * (t + 1) / threads);
    work(0, n / threads);
    for (auto& x : th) x.join();
}

// The same over a ragged batch: packet i at arena + offsets[i], lens[i] bytes,
// through pip_inet_checksum (pip_checksum.cpp:42-61) / pip_inet6_checksum (:63-87).
void ref_batch_ragged(const uint8_t* arena, const uint64_t* offsets, const uint32_t* lens, uint64_t n, int family,
                      uint8_t proto, const uint32_t* flows4, const uint8_t* flows6, uint32_t n_flows,
                      uint64_t flow_origin, uint16_t* out, int threads) {
    if (threads < 1) threads = 1;
    auto work = [&](uint64_t b, uint64_t e) {
        for (uint64_t i = b; i < e; i++) {
            const uint8_t* p = arena + offsets[i];
            const uint32_t f = (uint32_t)((flow_origin + i) % n_flows);
            if (family == 4) {
                pip_in_addr s, d;
                s.s_addr = flows4[2 * f];
                d.s_addr = flows4[2 * f + 1];
                out[i] = pip_inet_checksum(p, proto, s, d, (pip_uint16)lens[i]);
            } else if (family == 6) {
                pip_in6_addr s, d;
                std::memcpy(&s, flows6 + 32 * f, 16);
                std::memcpy(&d, flows6 + 32 * f + 16, 16);
                out[i] = pip_inet6_checksum(p, proto, s, d, (pip_uint16)lens[i]);
            } else {
                out[i] = pip_ip_checksum(p, lens[i]);
            }
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < threads; t++) th.emplace_back(work, n * t / threads, n * (t + 1) / threads);
    work(0, n / threads);
    for (auto& x : th) x.join();
}

// CPU baseline of the call pip's TX path actually makes: pip_tcp_packet.cpp:28-37
// builds each TCP segment as a chain -- a 20-byte header pip_buf, then the
// payload pip_buf (pip_udp.cpp the same with an 8-byte UDP header) -- and
// :124-134 checksums it with pip_inet{,6}_checksum_buf (pip_checksum.cpp:90-148),
// which copies the shared_ptr and walks the chain, one pip_standard_checksum and
// fold per segment.  The chains are built once (pip builds them while
// constructing the packet) and point into the batch (pip_buf(p, len, 0): no
// copy); ref_chains_checksum times the checksum calls alone.
struct RefChains {
    std::vector<std::shared_ptr<pip_buf>> head;
};

void* ref_chains_build(const uint8_t* arena, const uint64_t* offsets, const uint32_t* lens, uint64_t n,
                       uint32_t hdr_len) {
    auto* c = new RefChains();
    c->head.reserve(n);
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t* p = arena + offsets[i];
        const uint32_t h = lens[i] < hdr_len ? lens[i] : hdr_len;
        auto head = std::make_shared<pip_buf>(p, h, 0);
        if (lens[i] > h) head->set_next(std::make_shared<pip_buf>(p + h, lens[i] - h, 0));
        c->head.push_back(std::move(head));
    }
    return c;
}

void ref_chains_free(void* h) { delete static_cast<RefChains*>(h); }

void ref_chains_checksum(void* h, int family, uint8_t proto, const uint32_t* flows4, const uint8_t* flows6,
                         uint32_t n_flows, uint64_t flow_origin, uint16_t* out, int threads) {
    auto* c = static_cast<RefChains*>(h);
    const uint64_t n = c->head.size();
    if (threads < 1) threads = 1;
    auto work = [&](uint64_t b, uint64_t e) {
        for (uint64_t i = b; i < e; i++) {
            const uint32_t f = (uint32_t)((flow_origin + i) % n_flows);
            if (family == 4) {
                pip_in_addr s, d;
                s.s_addr = flows4[2 * f];
                d.s_addr = flows4[2 * f + 1];
                out[i] = pip_inet_checksum_buf(c->head[i], proto, s, d);
            } else {
                pip_in6_addr s, d;
                std::memcpy(&s, flows6 + 32 * f, 16);
                std::memcpy(&d, flows6 + 32 * f + 16, 16);
                out[i] = pip_inet6_checksum_buf(c->head[i], proto, s, d);
            }
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < threads; t++) th.emplace_back(work, n * t / threads, n * (t + 1) / threads);
    work(0, n / threads);
    for (auto& x : th) x.join();
}

}  // extern "C"
