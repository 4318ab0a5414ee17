// stack_udp_bench.cpp -- MEASUREMENT / TEST INFRASTRUCTURE.
//
// pip's UDP transmit path at volume: pip_udp::output (pip/protocol/pip_udp.cpp:28-64)
// wraps the caller's buffer in a payload pip_buf behind an 8-byte UDP header pip_buf,
// takes the UDP checksum over that chain with pip_inet_checksum_buf /
// pip_inet6_checksum_buf (:50-51, :60-61) and hands it to pip_netif::output4 / output6,
// which adds the IP header (and, for IPv4, its checksum, pip/pip_netif.cpp:94-97).
// No connection state is involved, so every datagram is one call.
//
// Linked like stack_tx_bench.cpp by oracle/Makefile (pip's stack compiled from
// /root/reference):
//   _ref/stack_udp_ref : pip's own pip_checksum.cpp                       --mode ref
//   _ref/stack_udp_amd : the stack WITHOUT pip_checksum.o + libpip_checksum_amd.so
//        --mode sync        every checksum call runs on the GPU as it is made
//        --mode capture     pip's unchanged call sites queue their checksums; the output
//                           callback holds each datagram; every --batch datagrams one
//                           pip_checksum_amd_flush() fills every field, then they go out
//        --mode capture_zc  the same, the caller's buffers in pinned memory
//                           (pipck_host_alloc) read in place by the GPU
//   _ref/stack_udp_zero: every checksum returns 0 (oracle/ck_zero.cpp)     --mode zero
//        pip's UDP TX path with no checksum work: the ceiling of any offload
//
// --pipeline (capture modes): after every batch pip_checksum_amd_submit() starts it
// and completes the batch before, whose datagrams are then output while the GPU
// works (datagrams need no acknowledgement, so batches overlap on one socket).
//
// Output (one JSON line): payload GiB/s and datagrams/s through the whole TX path,
// and FNV-1a over every emitted IP + UDP header (both checksums, both lengths) --
// with --verify over every wire byte -- which must be equal across the builds and
// modes for the same arguments.
#include "pip_netif.h"
#include "pip_checksum.h"
#include "protocol/pip_udp.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unistd.h>
#include <vector>

#ifdef PIPCK_AMD
#include "pip_checksum_amd.h"
#include "pipck.h"
#endif

namespace {

enum Mode { REF, SYNC, CAPTURE, CAPTURE_ZC, ZERO };

Mode g_mode = REF;
bool g_hold = false;  // capture modes: datagrams wait for the flush
std::vector<std::vector<std::shared_ptr<pip_buf>>> g_pending;
uint64_t g_digest = 1469598103934665603ull;
uint64_t g_packets = 0, g_wire_bytes = 0;

bool g_verify = false;  // --verify: digest every wire byte; else the IP + UDP headers (both checksums, lengths)

// an emitted datagram: IP header segment -> UDP header segment -> payload segment
void emit(const std::vector<std::shared_ptr<pip_buf>>& segs) {
    uint64_t h = g_digest;
    for (size_t k = 0; k < segs.size(); k++) {
        const uint8_t* p = (const uint8_t*)segs[k]->payload();
        if (g_verify || k < 2)
            for (uint32_t i = 0; i < segs[k]->payload_len(); i++) h = (h ^ p[i]) * 1099511628211ull;
        g_wire_bytes += segs[k]->payload_len();
    }
    g_digest = h;
    g_packets++;
}

// pip_netif::output4/6 detach the IP header after the callback (pip_netif.cpp:107,
// :134), so a held datagram keeps a reference to every segment
void on_output(pip_netif&, std::shared_ptr<pip_buf> buf) {
    std::vector<std::shared_ptr<pip_buf>> segs;
    for (auto q = buf; q; q = q->next()) segs.push_back(q);
    if (g_hold)
        g_pending.push_back(std::move(segs));
    else
        emit(segs);
}

double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

int main(int argc, char** argv) {
    std::string mode = "ref";
    unsigned family = 6, len = 8952, batch = 256;
    size_t total = 1ull << 30;
    bool pipeline = false;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto val = [&]() -> const char* { return i + 1 < argc ? argv[++i] : ""; };
        if (a == "--mode") mode = val();
        else if (a == "--family") family = (unsigned)atoi(val());
        else if (a == "--len") len = (unsigned)atoi(val());
        else if (a == "--bytes") total = strtoull(val(), nullptr, 0);
        else if (a == "--batch") batch = (unsigned)atoi(val());
        else if (a == "--pipeline") pipeline = true;
        else if (a == "--verify") g_verify = true;
        else { fprintf(stderr, "unknown argument %s\n", a.c_str()); return 2; }
    }
    if (mode == "ref") g_mode = REF;
    else if (mode == "sync") g_mode = SYNC;
    else if (mode == "capture") g_mode = CAPTURE;
    else if (mode == "capture_zc") g_mode = CAPTURE_ZC;
    else if (mode == "zero") g_mode = ZERO;
    else { fprintf(stderr, "unknown mode %s\n", mode.c_str()); return 2; }
#if defined(PIPCK_ZERO)
    if (g_mode != ZERO) { fprintf(stderr, "this build links checksums that return 0: --mode zero only\n"); return 2; }
#elif !defined(PIPCK_AMD)
    if (g_mode != REF) { fprintf(stderr, "this build links pip's own pip_checksum.cpp: --mode ref only\n"); return 2; }
#else
    if (g_mode == REF) { fprintf(stderr, "this build links libpip_checksum_amd.so: sync/capture/capture_zc\n"); return 2; }
#endif
    if ((family != 4 && family != 6) || len < 1 || len > 65507 || batch < 1 || total < len) {
        fprintf(stderr, "bad --family / --len / --batch / --bytes\n");
        return 2;
    }
    if (pipeline && g_mode != CAPTURE && g_mode != CAPTURE_ZC) {
        fprintf(stderr, "--pipeline needs a capture mode\n");
        return 2;
    }
    const char* src = family == 4 ? "10.0.0.1" : "fd00::1";
    const char* dst = family == 4 ? "10.0.0.2" : "fd00::2";

    // the application's datagrams: a 64 MiB ring of distinct payloads, never
    // rewritten during the run (so in-place GPU reads of in-flight batches are safe)
    const size_t slots = std::max<size_t>(1, (64ull << 20) / len);
    const size_t ring_bytes = slots * len;
    uint8_t* ring = nullptr;
    std::vector<uint8_t> plain;
#ifdef PIPCK_AMD
    if (g_mode == CAPTURE_ZC) ring = (uint8_t*)pipck_host_alloc(ring_bytes);
#endif
    if (!ring) {
        plain.resize(ring_bytes);
        ring = plain.data();
    }
    for (size_t i = 0; i < ring_bytes; i++) ring[i] = (uint8_t)(i * 131 + (i >> 11) * 7 + 3);

    auto& nif = pip_netif::shared();
    nif.output_ip_data_callback = on_output;

    // one-time GPU initialisation (kernels, pinned staging) outside the timed
    // region: three warm-up datagrams in every mode, so pip's IP identification
    // counter (pip_netif.cpp:89) starts the timed datagrams at the same value
    double cold = now();
    pip_udp::output(ring, (pip_uint16)len, src, 5353, dst, 53);
#ifdef PIPCK_AMD
    if (g_mode == CAPTURE || g_mode == CAPTURE_ZC) {
        pip_checksum_amd_capture(true);
        if (g_mode == CAPTURE_ZC) pip_checksum_amd_zero_copy(true);
        g_hold = true;
    }
#endif
    for (int i = 0; i < 2; i++) {  // in capture modes: both double-buffered batches
        pip_udp::output(ring, (pip_uint16)len, src, 5353, dst, 53);
#ifdef PIPCK_AMD
        if (g_hold) {
            pip_checksum_amd_flush();
            for (auto& s : g_pending) emit(s);
            g_pending.clear();
        }
#endif
    }
    cold = now() - cold;
    g_digest = 1469598103934665603ull;  // the digest covers the timed datagrams only
    g_packets = g_wire_bytes = 0;

    const size_t count = total / len;
    std::vector<std::vector<std::shared_ptr<pip_buf>>> inflight;
    const double t0 = now();
    for (size_t i = 0; i < count; i++) {
        pip_udp::output(ring + (i % slots) * len, (pip_uint16)len, src, (pip_uint16)(5353 + (i & 7)), dst, 53);
#ifdef PIPCK_AMD
        if (g_hold && ((i + 1) % batch == 0 || i + 1 == count)) {
            if (pipeline) {
                pip_checksum_amd_submit();  // starts this batch, completes the one before
                for (auto& s : inflight) emit(s);
                inflight.clear();
                inflight.swap(g_pending);
            } else {
                pip_checksum_amd_flush();
                for (auto& s : g_pending) emit(s);
                g_pending.clear();
            }
        }
#endif
    }
#ifdef PIPCK_AMD
    if (pipeline) {
        pip_checksum_amd_complete();
        for (auto& s : inflight) emit(s);
        inflight.clear();
    }
#endif
    const double el = now() - t0;
#ifdef PIPCK_AMD
    if (g_hold) {
        pip_checksum_amd_zero_copy(false);
        pip_checksum_amd_capture(false);
    }
#endif
    printf("{\"tool\": \"stack_udp_bench\", \"mode\": \"%s\", \"family\": %u, \"len\": %u, \"batch\": %u, "
           "\"pipeline\": %s, \"datagrams\": %llu, \"payload_bytes\": %llu, \"seconds\": %.6f, "
           "\"payload_gib_per_s\": %.4f, \"mpkt_per_s\": %.4f, \"digest\": \"%016llx\", \"digest_of\": "
           "\"%s\", \"wire_bytes\": %llu, \"cold_ms\": %.3f}\n",
           mode.c_str(), family, len, batch, pipeline ? "true" : "false", (unsigned long long)g_packets,
           (unsigned long long)count * len, el, (double)count * len / el / (1u << 30), g_packets / el / 1e6,
           (unsigned long long)g_digest, g_verify ? "every wire byte" : "IP and UDP headers",
           (unsigned long long)g_wire_bytes, cold * 1e3);
    fflush(stdout);
    _exit(g_packets == count ? 0 : 4);  // pip's timer thread is detached and never stops
}
