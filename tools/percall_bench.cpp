// percall_bench.cpp -- latency of pip's synchronous per-packet API through the
// drop-in (libpip_checksum_amd.so -> pipck_host_sum -> one GPU launch per call).
//
//   pip_amd/lib/percall_bench [calls]
//
// For 20-B IPv4 headers (pip_ip_checksum) and 1,480 / 8,980-B TCP segments
// (and a 65,535-B one) (pip_inet_checksum): median and p99 microseconds per call on one thread,
// for the staged path (H2D copy, kernel, D2H copy) and the zero-copy path
// (the kernel reads the pinned staging buffer and writes the result to
// pinned host memory directly; pipck_host_zero_copy(1)).  Results of both
// paths are checked equal.  One JSON line per (size, path).
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
    for (uint32_t len : {20u, 1480u, 8980u, 65535u}) {
        uint32_t ref = 0;
        for (int zc = 0; zc < 2; zc++) {
            pipck_host_zero_copy(zc);
            std::vector<double> us;
            uint32_t r = 0;
            for (int i = 0; i < calls + 50; i++) {
                auto t0 = std::chrono::steady_clock::now();
                r = len == 20 ? pip_ip_checksum(buf.data(), len)
                              : pip_inet_checksum(buf.data(), 6, s, d, (uint16_t)len);
                auto t1 = std::chrono::steady_clock::now();
                if (i >= 50) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
            }
            if (zc == 0) ref = r;
            if (r != ref) {
                fprintf(stderr, "percall_bench: zero-copy result %u != staged %u at len %u\n", r, ref, len);
                return 1;
            }
            std::sort(us.begin(), us.end());
            printf("{\"tool\": \"percall_bench\", \"len\": %u, \"path\": \"%s\", \"median_us\": %.2f, \"p99_us\": %.2f}\n",
                   len, zc ? "zero_copy" : "staged", us[us.size() / 2], us[us.size() * 99 / 100]);
            fflush(stdout);
        }
    }
    return 0;
}
