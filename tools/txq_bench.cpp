// txq_bench.cpp -- throughput of the deferred TX queue (include/pipck.h, pipck_txq_*).
//
//   pip_amd/lib/txq_bench [packets] [payload] [rounds] [threads] [batch]
//
// Builds `packets` TCP/IPv4 segments in host memory the way pip's TX path
// does (a 20-byte header segment with th_sum = 0 chained to a payload
// segment, pip/protocol/pip_tcp_packet.cpp:28-37) and checksums them through
// TX queues, `threads` producer threads with one queue each over their share
// of the packets.  Three modes, each timed over `rounds` repetitions (best kept):
//   sync       add every packet, then pipck_txq_flush (one H2D, one GPU batch,
//              one D2H, htons(result) into every header);
//   pipelined  add `batch` packets, pipck_txq_submit, add the next `batch`
//              while the previous one is in flight; pipck_txq_complete at the end;
//   zero_copy  pipelined, with headers and payloads in pinned host memory
//              (pipck_host_alloc) added by pipck_txq_add4_zc: the GPU reads
//              them in place, nothing is copied at add time;
//   auto_zc    pipelined, plain pipck_txq_add4 on queues in automatic
//              zero-copy mode (pipck_txq_auto_zero_copy): the same in-place
//              reads, decided per segment by the pinned-range lookup.
// Every header's th_sum is checked against the first sync round.  Prints one
// JSON line per mode: host-to-host rate of the whole add+flush cycle.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../include/pipck.h"

namespace {

struct Shard {
    uint32_t first, n;
    pipck_txq* q = nullptr;
    int rc = 0;
};

int add_packet(pipck_txq* q, uint8_t* hdr, const uint8_t* body, uint32_t payload, uint32_t i, bool zc) {
    pipck_hseg segs[2] = {{&hdr[(size_t)i * 20], 20}, {&body[(size_t)i * payload], payload}};
    return (zc ? pipck_txq_add4_zc : pipck_txq_add4)(q, segs, 2, 6, 0x0100000Au + (i & 1023), 0x0200000Au,
                                                      &hdr[(size_t)i * 20 + 16]);
}

int run_shard(Shard& s, uint8_t* hdr, const uint8_t* body, uint32_t payload, bool pipelined, uint32_t batch, bool zc) {
    for (uint32_t i = s.first; i < s.first + s.n; i++) {
        int rc = add_packet(s.q, hdr, body, payload, i, zc);
        if (rc) return rc;
        if (pipelined && (i - s.first + 1) % batch == 0 && (rc = pipck_txq_submit(s.q))) return rc;
    }
    if (pipelined) {
        int rc = pipck_txq_submit(s.q);
        return rc ? rc : pipck_txq_complete(s.q);
    }
    return pipck_txq_flush(s.q);
}

}  // namespace

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 200000;
    const uint32_t payload = argc > 2 ? (uint32_t)atoi(argv[2]) : 1460;
    const int rounds = argc > 3 ? atoi(argv[3]) : 5;
    const uint32_t threads = std::max(1, argc > 4 ? atoi(argv[4]) : 1);
    const uint32_t batch = std::max(1, argc > 5 ? atoi(argv[5]) : 16384);
    // pinned, so the zero-copy mode can read them in place (the copying modes do not care)
    const size_t hdr_n = (size_t)n * 20, body_n = (size_t)n * payload;
    uint8_t* hdr = (uint8_t*)pipck_host_alloc(hdr_n);
    uint8_t* body = (uint8_t*)pipck_host_alloc(body_n ? body_n : 1);
    if (!hdr || !body) {
        fprintf(stderr, "txq_bench: pinned allocation failed\n");
        return 1;
    }
    for (size_t i = 0; i < body_n; i++) body[i] = (uint8_t)(i * 2654435761u >> 24);
    for (size_t i = 0; i < hdr_n; i++) hdr[i] = (uint8_t)(i * 40503u >> 8);
    pipck_ctx* ctx = nullptr;
    if (pipck_ctx_create(-1, &ctx)) {
        fprintf(stderr, "txq_bench: %s\n", pipck_last_error());
        return 1;
    }
    std::vector<Shard> shards(threads);
    for (uint32_t t = 0; t < threads; t++) {
        shards[t].first = (uint32_t)((uint64_t)n * t / threads);
        shards[t].n = (uint32_t)((uint64_t)n * (t + 1) / threads) - shards[t].first;
        if (pipck_txq_create(ctx, &shards[t].q)) {
            fprintf(stderr, "txq_bench: %s\n", pipck_last_error());
            return 1;
        }
    }
    std::vector<uint8_t> want;  // th_sum of every packet from the first sync round
    static const char* kModes[] = {"sync", "pipelined", "zero_copy", "auto_zc"};
    for (int mode = 0; mode < 4; mode++) {
        const bool pipelined = mode >= 1, zc = mode == 2;
        for (auto& s : shards) pipck_txq_auto_zero_copy(s.q, mode == 3);
        double best = 1e30;
        for (int r = 0; r < rounds; r++) {
            for (uint32_t i = 0; i < n; i++) hdr[(size_t)i * 20 + 16] = hdr[(size_t)i * 20 + 17] = 0;
            auto t0 = std::chrono::steady_clock::now();
            if (threads == 1) {  // inline: a thread spawn would dominate small batches
                shards[0].rc = run_shard(shards[0], hdr, body, payload, pipelined, batch, zc);
            } else {
                std::vector<std::thread> th;
                for (auto& s : shards)
                    th.emplace_back([&, pipelined, zc] { s.rc = run_shard(s, hdr, body, payload, pipelined, batch, zc); });
                for (auto& x : th) x.join();
            }
            auto t1 = std::chrono::steady_clock::now();
            for (auto& s : shards) {
                if (s.rc) {
                    fprintf(stderr, "txq_bench: %s\n", pipck_last_error());
                    return 1;
                }
            }
            best = std::min(best, std::chrono::duration<double>(t1 - t0).count());
            std::vector<uint8_t> got((size_t)n * 2);
            for (uint32_t i = 0; i < n; i++) std::memcpy(&got[(size_t)i * 2], &hdr[(size_t)i * 20 + 16], 2);
            if (want.empty()) {
                want = got;
            } else if (got != want) {
                fprintf(stderr, "txq_bench: %s round %d: checksums differ from the first round\n", kModes[mode], r);
                return 1;
            }
        }
        const double bytes = (double)n * (20 + payload);
        printf("{\"tool\": \"txq_bench\", \"mode\": \"%s\", \"threads\": %u, \"batch\": %u, \"packets\": %u, "
               "\"l4_bytes\": %u, \"gib_per_s\": %.2f, \"mpkt_per_s\": %.3f, \"ms\": %.2f}\n",
               kModes[mode], threads, pipelined ? batch : n, n, 20 + payload,
               bytes / best / (1u << 30), n / best / 1e6, best * 1e3);
        fflush(stdout);
    }
    for (auto& s : shards) pipck_txq_destroy(s.q);
    pipck_ctx_destroy(ctx);
    pipck_host_free(hdr);
    pipck_host_free(body);
    return 0;
}
