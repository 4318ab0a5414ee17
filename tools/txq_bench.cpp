// txq_bench.cpp -- throughput of the deferred TX queue (include/pipck.h, pipck_txq_*).
//
//   pip_amd/lib/txq_bench [packets] [payload] [rounds]
//
// Builds `packets` TCP/IPv4 segments in host memory the way pip's TX path
// does (a 20-byte header segment with th_sum = 0 chained to a payload
// segment, pip/protocol/pip_tcp_packet.cpp:28-37), queues all of them with
// their pseudo-header and th_sum address, and flushes: one H2D copy, one GPU
// batch, one D2H copy, htons(result) stored into every header.  Prints one
// JSON line: host-to-host rate of the whole add+flush cycle.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/pipck.h"

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 200000;
    const uint32_t payload = argc > 2 ? (uint32_t)atoi(argv[2]) : 1460;
    const int rounds = argc > 3 ? atoi(argv[3]) : 5;
    std::vector<uint8_t> hdr((size_t)n * 20), body((size_t)n * payload);
    for (size_t i = 0; i < body.size(); i++) body[i] = (uint8_t)(i * 2654435761u >> 24);
    for (size_t i = 0; i < hdr.size(); i++) hdr[i] = (uint8_t)(i * 40503u >> 8);
    pipck_ctx* ctx = nullptr;
    pipck_txq* q = nullptr;
    if (pipck_ctx_create(-1, &ctx) || pipck_txq_create(ctx, &q)) {
        fprintf(stderr, "txq_bench: %s\n", pipck_last_error());
        return 1;
    }
    double best = 1e30, add_s = 0, flush_s = 0;
    for (int r = 0; r < rounds; r++) {
        for (uint32_t i = 0; i < n; i++) hdr[(size_t)i * 20 + 16] = hdr[(size_t)i * 20 + 17] = 0;
        auto t0 = std::chrono::steady_clock::now();
        for (uint32_t i = 0; i < n; i++) {
            pipck_hseg segs[2] = {{&hdr[(size_t)i * 20], 20}, {&body[(size_t)i * payload], payload}};
            if (pipck_txq_add4(q, segs, 2, 6, 0x0100000Au + (i & 1023), 0x0200000Au, &hdr[(size_t)i * 20 + 16])) {
                fprintf(stderr, "txq_bench: add: %s\n", pipck_last_error());
                return 1;
            }
        }
        auto t1 = std::chrono::steady_clock::now();
        if (pipck_txq_flush(q)) {
            fprintf(stderr, "txq_bench: flush: %s\n", pipck_last_error());
            return 1;
        }
        auto t2 = std::chrono::steady_clock::now();
        const double a = std::chrono::duration<double>(t1 - t0).count();
        const double f = std::chrono::duration<double>(t2 - t1).count();
        if (a + f < best) {
            best = a + f;
            add_s = a;
            flush_s = f;
        }
    }
    const double bytes = (double)n * (20 + payload);
    printf("{\"tool\": \"txq_bench\", \"packets\": %u, \"l4_bytes\": %u, \"gib_per_s\": %.2f, \"mpkt_per_s\": %.3f, "
           "\"add_ms\": %.2f, \"flush_ms\": %.2f}\n",
           n, 20 + payload, bytes / best / (1u << 30), n / best / 1e6, add_s * 1e3, flush_s * 1e3);
    pipck_txq_destroy(q);
    pipck_ctx_destroy(ctx);
    return 0;
}
