// percall_bench.cpp -- latency of pip's synchronous per-packet API through the
// drop-in (libpip_checksum_amd.so -> pipck_host_sum -> one GPU launch per call).
//
//   pip_amd/lib/percall_bench [calls]
//
// For 20-B IPv4 headers (pip_ip_checksum) and 1,480 / 8,980-B TCP segments
// (and a 65,535-B one) (pip_inet_checksum): median and p99 microseconds per call on one thread,
// for the staged path (H2D copy, kernel, D2H copy) and the zero-copy path
// (the kernel reads the pinned staging buffer and writes the result to
// pinned host memory directly) -- both through pipck_host_sum on a context of
// this tool's own (pipck_ctx_zero_copy 0 / 1), the call the drop-in makes --
// and the drop-in itself in its default mode, plus the resident service (mode
// 3: a block that stays on the GPU and polls a doorbell) through pipck_host_sum
// and through the drop-in (pip_checksum_amd_resident).  Results of all paths
// are checked equal.  One JSON line per (size, path).  Then the crossover with
// the deferred TX queue: N segments of 1,480 B added and flushed as one batch,
// microseconds per segment, for N = 1 .. 4,096.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/pip_checksum_amd.h"
#include "../include/pipck.h"

int main(int argc, char** argv) {
    const int calls = argc > 1 ? atoi(argv[1]) : 2000;
    std::vector<uint8_t> buf(65536);
    for (size_t i = 0; i < buf.size(); i++) buf[i] = (uint8_t)(i * 2654435761u >> 24);
    struct in_addr s, d;
    s.s_addr = 0x0100000Au;
    d.s_addr = 0x0200000Au;
    pipck_ctx* ctx = nullptr;
    if (pipck_ctx_create(-1, &ctx)) {
        fprintf(stderr, "percall_bench: %s\n", pipck_last_error());
        return 1;
    }
    static const char* kPath[] = {"staged", "zero_copy", "drop_in", "resident", "drop_in_resident"};
    for (uint32_t len : {20u, 1480u, 8980u, 65535u}) {
        uint32_t ref = 0;
        for (int path = 0; path < 5; path++) {
            if (path < 2) pipck_ctx_zero_copy(ctx, path);
            if (path == 3) pipck_ctx_zero_copy(ctx, 3);
            pip_checksum_amd_resident(path == 4);  // the drop-in's thread: auto mode, or resident for path 4
            if (path == 4) pipck_ctx_zero_copy(ctx, 2);  // release this context's resident block
            std::vector<double> us;
            uint32_t r = 0;
            for (int i = 0; i < calls + 50; i++) {
                auto t0 = std::chrono::steady_clock::now();
                if (path == 2 || path == 4) {
                    r = len == 20 ? pip_ip_checksum(buf.data(), len)
                                  : pip_inet_checksum(buf.data(), 6, s, d, (uint16_t)len);
                } else {  // what the drop-in computes: pip's folded sum, then ~ (pip_checksum.cpp:35-61)
                    const uint32_t pseudo = len == 20 ? 0u : 0x0A00u + 0x0001u + 0x0A00u + 0x0002u + 6u + len;  // 10.0.0.1 -> 10.0.0.2, TCP
                    pipck_hseg seg{buf.data(), len};
                    uint32_t sum = 0;
                    if (pipck_host_sum(ctx, &seg, 1, pseudo, &sum)) {
                        fprintf(stderr, "percall_bench: %s\n", pipck_last_error());
                        return 1;
                    }
                    r = (uint16_t)~(uint16_t)sum;
                }
                auto t1 = std::chrono::steady_clock::now();
                if (i >= 50) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
            }
            if (path == 0) ref = r;
            if (r != ref) {
                fprintf(stderr, "percall_bench: %s result %u != staged %u at len %u\n", kPath[path], r, ref, len);
                return 1;
            }
            std::sort(us.begin(), us.end());
            printf("{\"tool\": \"percall_bench\", \"len\": %u, \"path\": \"%s\", \"median_us\": %.2f, \"p99_us\": %.2f}\n",
                   len, kPath[path], us[us.size() / 2], us[us.size() * 99 / 100]);
            fflush(stdout);
        }
    }
    pip_checksum_amd_resident(false);
    // crossover: the deferred queue, N packets per flush
    pipck_txq* q = nullptr;
    if (pipck_txq_create(ctx, &q)) {
        fprintf(stderr, "percall_bench: %s\n", pipck_last_error());
        return 1;
    }
    std::vector<uint8_t> fields(2 * 4096);
    for (uint32_t npk : {1u, 2u, 4u, 8u, 16u, 32u, 64u, 128u, 256u, 1024u, 4096u}) {
        std::vector<double> us;
        const int reps = npk >= 1024 ? 200 : 1000;
        for (int i = 0; i < reps + 20; i++) {
            auto t0 = std::chrono::steady_clock::now();
            for (uint32_t k = 0; k < npk; k++) {
                pipck_hseg seg{buf.data() + (k % 16) * 64, 1480};
                if (pipck_txq_add4(q, &seg, 1, 6, s.s_addr, d.s_addr, &fields[2 * k])) {
                    fprintf(stderr, "percall_bench: %s\n", pipck_last_error());
                    return 1;
                }
            }
            if (pipck_txq_flush(q)) {
                fprintf(stderr, "percall_bench: %s\n", pipck_last_error());
                return 1;
            }
            auto t1 = std::chrono::steady_clock::now();
            if (i >= 20) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        }
        std::sort(us.begin(), us.end());
        printf("{\"tool\": \"percall_bench\", \"path\": \"deferred_queue\", \"packets_per_flush\": %u, \"len\": 1480, "
               "\"median_us_per_flush\": %.2f, \"median_us_per_packet\": %.3f}\n",
               npk, us[us.size() / 2], us[us.size() / 2] / npk);
        fflush(stdout);
    }
    pipck_txq_destroy(q);
    pipck_ctx_destroy(ctx);
    return 0;
}
