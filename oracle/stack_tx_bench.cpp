// stack_tx_bench.cpp -- MEASUREMENT / TEST INFRASTRUCTURE.
//
// pip's TCP transmit path at volume: pip_tcp::write (pip/protocol/pip_tcp_public.cpp:43-48
// -> pip_tcp::_write, pip/protocol/pip_tcp_private.cpp:74-120) cuts the caller's buffer
// into MSS segments; every segment's TCP checksum is taken inside pip_tcp_packet's
// constructor (pip/protocol/pip_tcp_packet.cpp:124-134) and every IPv4 header's inside
// pip_netif::output4 (pip/pip_netif.cpp:94-97).  A scripted peer completes the handshake
// (MSS option + window scale 14, so pip's send window is 1 GiB) and ACKs every write(),
// which ends in a PUSH pip waits on (pip_tcp_private.cpp:99-107, 121-128, 211-226).
//
// Linked three ways by oracle/Makefile (pip's stack compiled from /root/reference):
//   _ref/stack_tx_ref : pip's own pip_checksum.cpp                      --mode ref
//   _ref/stack_tx_amd : the stack WITHOUT pip_checksum.o + libpip_checksum_amd.so
//        --mode sync        every checksum call runs on the GPU as it is made (unchanged pip)
//        --mode capture     the drop-in's capture mode: pip's unchanged call sites queue
//                           their checksums; the output callback holds each packet; one
//                           pip_checksum_amd_flush() per write() fills every field, then
//                           the packets go out
//        --mode capture_zc  the same, with the write() buffer in pinned memory
//                           (pipck_host_alloc) and pip_checksum_amd_zero_copy(true): the
//                           GPU reads the payload segments in place
//   _ref/stack_tx_zero: every checksum returns 0 (oracle/ck_zero.cpp)    --mode zero
//        pip's TX path with no checksum work: the ceiling of any offload (wrong wire bytes)
//
// --conns K opens K connections (client ports 40000+k) and writes to them in
// turn; --family 6 runs them over IPv6 (pip_tcp_packet.cpp:130 takes
// pip_inet6_checksum_buf, pip_netif::output6 adds no header checksum).  --pipeline (capture modes, K >= 2) overlaps the GPU with pip: after
// each write pip_checksum_amd_submit() starts that write's batch and completes
// the previous one, whose packets are then output and its connection ACKed
// while the GPU works on the next (pip waits for the ACK of a write's PUSH
// before that connection's next write, so overlap needs another connection).
//
// Output (one JSON line): payload GiB/s and packets/s through the whole TX path, and a
// digest of every emitted packet -- with --verify, FNV-1a over every wire byte; else over
// each packet's IPv4 and TCP checksum fields and length -- which must be equal across the
// three builds/modes for the same arguments.
#include "pip_netif.h"
#include "pip_checksum.h"
#include "protocol/pip_tcp.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

#ifdef PIPCK_AMD
#include "pip_checksum_amd.h"
#include "pipck.h"
#endif

namespace {

enum Mode { REF, SYNC, CAPTURE, CAPTURE_ZC, ZERO };

Mode g_mode = REF;
bool g_verify = false;
bool g_hold = false;  // capture modes: packets wait for the flush
struct Conn {
    uint16_t port;
    std::shared_ptr<pip_tcp> tcp;
    uint32_t cseq = 7000;
    uint32_t srv_next = 0;  // pip's next sequence number on this connection, from its emitted segments
    uint8_t* buf = nullptr;
    // segments pip sent and the peer has not ACKed yet (the ones pip's timer may
    // resend): sequence number and the time pip sent it, oldest first (g_sent_mu)
    std::deque<std::pair<uint32_t, double>> unacked;
};
std::vector<Conn> g_conns;
int g_connecting = -1;  // the connection whose SYN is being input
constexpr uint16_t kPortBase = 40000;
std::vector<std::vector<std::shared_ptr<pip_buf>>> g_pending;
uint64_t g_digest = 1469598103934665603ull;
uint64_t g_packets = 0, g_wire_bytes = 0;
FILE* g_dump = nullptr;   // --dump: one 12-byte record per packet (seq, ip_id, ip_sum, th_sum, length)

inline void fnv(const uint8_t* p, size_t n) {
    uint64_t h = g_digest;
    for (size_t i = 0; i < n; i++) h = (h ^ p[i]) * 1099511628211ull;
    g_digest = h;
}

// The same wire bytes with each IPv4 header's identification and checksum
// fields replaced by one byte "this header's checksum verifies" (an RFC 1071
// sum over the header, computed here on the host: test infrastructure).
// pip_netif::output4 numbers IPv4 headers from one unsynchronised counter
// (pip/pip_netif.cpp:90, `_identifer++`), so a resend by pip's timer thread --
// its stale-clock race, pip_tcp_check.cpp:45-56 -- shifts the ip_id, and so the
// ip_sum, of every later packet in pip's own build as much as in the drop-in's;
// this digest still compares every other byte and every header's validity.
uint64_t g_digest_noid = 1469598103934665603ull;
inline void fnv_noid(const uint8_t* p, size_t n) {
    uint64_t h = g_digest_noid;
    for (size_t i = 0; i < n; i++) h = (h ^ p[i]) * 1099511628211ull;
    g_digest_noid = h;
}
void digest_noid(const std::vector<std::shared_ptr<pip_buf>>& segs) {
    for (size_t s = 0; s < segs.size(); s++) {
        const uint8_t* b = (const uint8_t*)segs[s]->payload();
        const size_t n = segs[s]->payload_len();
        if (s == 0 && n >= 20 && (b[0] >> 4) == 4) {
            const size_t ihl = (size_t)(b[0] & 15) * 4;
            uint32_t sum = 0;
            for (size_t i = 0; i + 1 < ihl && i + 1 < n; i += 2) sum += (uint32_t)b[i] << 8 | b[i + 1];
            while (sum >> 16) sum = (sum & 0xFFFF) + (sum >> 16);
            std::vector<uint8_t> h(b, b + n);
            h[4] = h[5] = h[10] = 0;
            h[11] = sum == 0xFFFF;
            fnv_noid(h.data(), n);
        } else {
            fnv_noid(b, n);
        }
    }
}

// an emitted packet: IPv4 header segment -> TCP header segment -> payload segment(s)
void emit(const std::vector<std::shared_ptr<pip_buf>>& segs) {
    size_t len = 0;
    for (auto& s : segs) len += s->payload_len();
    if (g_verify) {
        for (auto& s : segs) fnv((const uint8_t*)s->payload(), s->payload_len());
        digest_noid(segs);
    } else {
        const uint8_t* ip = (const uint8_t*)segs[0]->payload();
        uint8_t rec[8] = {ip[10], ip[11], 0, 0, (uint8_t)len, (uint8_t)(len >> 8), 0, 0};
        if (segs.size() > 1 && segs[1]->payload_len() >= 18) {
            const uint8_t* th = (const uint8_t*)segs[1]->payload();
            rec[2] = th[16];
            rec[3] = th[17];
        }
        fnv(rec, sizeof rec);
    }
    if (segs.size() > 1 && segs[1]->payload_len() >= 8) {
        const uint8_t* th = (const uint8_t*)segs[1]->payload();
        const uint32_t seq = (uint32_t)th[4] << 24 | (uint32_t)th[5] << 16 | (uint32_t)th[6] << 8 | th[7];
        const unsigned k = (unsigned)(th[2] << 8 | th[3]) - kPortBase;  // pip's destination = the client port
        size_t data = 0;
        for (size_t i = 2; i < segs.size(); i++) data += segs[i]->payload_len();
        if (k < g_conns.size()) g_conns[k].srv_next = seq + (uint32_t)data + ((th[13] & (TH_SYN | TH_FIN)) ? 1 : 0);
    }
    if (g_dump) {
        const uint8_t* ip = (const uint8_t*)segs[0]->payload();
        uint8_t rec[12] = {0};
        if (segs.size() > 1 && segs[1]->payload_len() >= 18) memcpy(rec, (const uint8_t*)segs[1]->payload() + 4, 4);
        rec[4] = ip[4], rec[5] = ip[5], rec[6] = ip[10], rec[7] = ip[11];
        if (segs.size() > 1 && segs[1]->payload_len() >= 18)
            rec[8] = ((const uint8_t*)segs[1]->payload())[16], rec[9] = ((const uint8_t*)segs[1]->payload())[17];
        rec[10] = (uint8_t)(len >> 8), rec[11] = (uint8_t)len;
        fwrite(rec, 1, sizeof rec, g_dump);
    }
    g_packets++;
    g_wire_bytes += len;
}

std::thread::id g_main;
std::mutex g_sent_mu;                     // Conn::unacked: the main thread sends, pip's timer thread resends
uint64_t g_resends_stalled = 0;           // resent at >= 1 s of age: a real stall (the run fails)
uint64_t g_resends_stale_clock = 0;       // resent younger than 1 s: pip's timer race (below)
double g_max_resend_age = 0, g_max_unacked = 0;

double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

uint32_t rd32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

void on_output(pip_netif&, std::shared_ptr<pip_buf> buf) {
    auto q = buf->next();  // the TCP header segment
    const uint8_t* th = q && q->payload_len() >= 14 ? (const uint8_t*)q->payload() : nullptr;
    const unsigned k = th ? (unsigned)(th[2] << 8 | th[3]) - kPortBase : ~0u;  // pip's destination = the client port
    if (std::this_thread::get_id() != g_main) {
        // pip's timer thread resends the oldest unacknowledged segment once it is
        // 1 s old (pip/protocol/pip_tcp_check.cpp:25-39).  Its age here tells a
        // stall (>= 1 s: the run fails) from pip's own timer race: timer_tick
        // reads the clock BEFORE it takes the connection's mutex
        // (pip_tcp_check.cpp:45-56), so a segment sent while the timer waited on
        // that mutex is newer than the timer's `now`, and the unsigned
        // `now - send_time` (:30) wraps to a huge age.  pip's own build does
        // this too (profiles/r04_pip_timer_race.jsonl).  Either way the resent
        // copy is not digested: the wire digest covers the main thread's packets.
        double age = -1;
        const uint32_t seq = th ? rd32(th + 4) : 0;
        {
            std::lock_guard<std::mutex> g(g_sent_mu);
            if (k < g_conns.size())
                for (auto& u : g_conns[k].unacked)
                    if (u.first == seq) { age = now() - u.second; break; }
            if (age >= 0 && age < 1.0) g_resends_stale_clock++;
            else g_resends_stalled++;
            if (age > g_max_resend_age) g_max_resend_age = age;
        }
        if (th)
            fprintf(stderr, "resend by pip's timer: port %u seq %u flags 0x%02x at %.3f s, %s\n",
                    (unsigned)(th[2] << 8 | th[3]), seq, th[13], now(),
                    age < 0 ? "not an unacknowledged segment" :
                    age < 1.0 ? "younger than 1 s (pip's stale-clock race)" : "unacknowledged for >= 1 s (a stall)");
        return;
    }
    if (th && k < g_conns.size()) {
        size_t data = 0;
        for (auto p = q->next(); p; p = p->next()) data += p->payload_len();
        if (data || (th[13] & (TH_SYN | TH_FIN))) {  // queued for retransmission by pip
            std::lock_guard<std::mutex> g(g_sent_mu);
            g_conns[k].unacked.emplace_back(rd32(th + 4), now());
        }
    }
    std::vector<std::shared_ptr<pip_buf>> segs;
    for (auto q = buf; q; q = q->next()) segs.push_back(q);
    if (g_hold)
        g_pending.push_back(std::move(segs));
    else
        emit(segs);
}

// the peer's ACK of everything sent on connection k has been input: nothing is
// left for pip's timer; the oldest segment's age is the longest any waited
void acked(unsigned k) {
    std::lock_guard<std::mutex> g(g_sent_mu);
    auto& u = g_conns[k].unacked;
    if (!u.empty() && now() - u.front().second > g_max_unacked) g_max_unacked = now() - u.front().second;
    u.clear();
}

// the longest single stack action of the run (an input, a write, a flush)
struct ActionClock {
    double max = 0;
    const char* which = "none";
    double t = 0;
    void start() { t = now(); }
    void stop(const char* what) {
        const double d = now() - t;
        if (d > max) max = d, which = what;
    }
} g_act;

// after each stack action: capture modes store every queued field, then output the packets
void settle() {
#ifdef PIPCK_AMD
    if (!g_hold) return;
    pip_checksum_amd_flush();
    for (auto& s : g_pending) emit(s);
    g_pending.clear();
#endif
}

void on_connect(pip_netif&, std::shared_ptr<pip_tcp> tcp, const void* hs, pip_uint16) {
    if (g_connecting >= 0) g_conns[g_connecting].tcp = tcp;
    tcp->connected(hs);
}

void put16(uint8_t* p, uint16_t v) { p[0] = v >> 8; p[1] = (uint8_t)v; }
void put32(uint8_t* p, uint32_t v) { put16(p, v >> 16); put16(p + 2, (uint16_t)v); }

unsigned g_family = 4;  // --family 6: the connections run over IPv6 (fd00::2 -> fd00::1)

// a client segment to pip (10.0.0.2:port -> 10.0.0.1:80, or fd00::2 -> fd00::1);
// RX takes no checksum
std::vector<uint8_t> craft(uint16_t port, uint32_t seq, uint32_t ack, uint8_t flags, const std::vector<uint8_t>& opts) {
    const size_t thl = 20 + opts.size(), ihl = g_family == 6 ? 40 : 20;
    std::vector<uint8_t> p(ihl + thl, 0);
    if (g_family == 6) {
        p[0] = 0x60;
        put16(&p[4], (uint16_t)thl);  // payload length
        p[6] = IPPROTO_TCP;
        p[7] = 64;
        p[8] = 0xfd, p[23] = 2;   // source fd00::2
        p[24] = 0xfd, p[39] = 1;  // destination fd00::1
    } else {
        p[0] = 0x45;
        put16(&p[2], (uint16_t)p.size());
        p[8] = 64;
        p[9] = IPPROTO_TCP;
        const uint8_t cli[4] = {10, 0, 0, 2}, srv[4] = {10, 0, 0, 1};
        memcpy(&p[12], cli, 4);
        memcpy(&p[16], srv, 4);
    }
    uint8_t* t = &p[ihl];
    put16(t, port);
    put16(t + 2, 80);
    put32(t + 4, seq);
    put32(t + 8, ack);
    t[12] = (uint8_t)((thl / 4) << 4);
    t[13] = flags;
    put16(t + 14, 65535);  // << 14 (the SYN's window-scale option): a 1 GiB send window
    memcpy(t + 20, opts.data(), opts.size());
    return p;
}

}  // namespace

int main(int argc, char** argv) {
    std::string mode = "ref";
    unsigned mss = 1460;
    size_t total = 256ull << 20, per_write = 4ull << 20;
    unsigned conns = 1;
    bool pipeline = false;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto val = [&]() -> const char* { return i + 1 < argc ? argv[++i] : ""; };
        if (a == "--mode") mode = val();
        else if (a == "--mss") mss = (unsigned)atoi(val());
        else if (a == "--bytes") total = strtoull(val(), nullptr, 0);
        else if (a == "--write") per_write = strtoull(val(), nullptr, 0);
        else if (a == "--verify") g_verify = true;
        else if (a == "--conns") conns = (unsigned)atoi(val());
        else if (a == "--pipeline") pipeline = true;
        else if (a == "--dump") g_dump = fopen(val(), "wb");
        else if (a == "--family") g_family = (unsigned)atoi(val());
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
    if (mss < 1 || mss > 65495 || per_write < 1 || per_write > (1u << 30) || conns < 1 || conns > 64 ||
        (g_family != 4 && g_family != 6)) {
        fprintf(stderr, "bad --mss / --write / --conns / --family\n");
        return 2;
    }
    if (pipeline && (conns < 2 || (g_mode != CAPTURE && g_mode != CAPTURE_ZC))) {
        fprintf(stderr, "--pipeline needs a capture mode and --conns >= 2\n");
        return 2;
    }

    // each connection's send buffer: pip's pip_buf points into it (write(..., is_copy=false));
    // a buffer is rewritten only after its connection's previous write was ACKed
    g_conns.resize(conns);
    std::vector<std::vector<uint8_t>> plain(conns);
    for (unsigned k = 0; k < conns; k++) {
        g_conns[k].port = (uint16_t)(kPortBase + k);
        uint8_t* b = nullptr;
#ifdef PIPCK_AMD
        if (g_mode == CAPTURE_ZC) b = (uint8_t*)pipck_host_alloc(per_write);
#endif
        if (!b) {
            plain[k].resize(per_write);
            b = plain[k].data();
        }
        for (size_t i = 0; i < per_write; i++) b[i] = (uint8_t)(i * 131 + (i >> 11) * 7 + 1 + k);
        g_conns[k].buf = b;
    }
    uint8_t* buf = g_conns[0].buf;

    g_main = std::this_thread::get_id();
    // One-time GPU initialisation (device, streams, every kernel the calls below
    // reach, pinned staging) before pip's 1 s retransmit clock runs: a first flush
    // that loads its kernels during the handshake can outlast it.
    uint8_t z[20] = {0};
    struct in_addr a4;
    a4.s_addr = 0x0100000a;
    struct in6_addr a6;
    memset(&a6, 0, sizeof a6);
    auto warm = [&]() {
        auto head = std::make_shared<pip_buf>(20);
        head->set_next(std::make_shared<pip_buf>(buf, (pip_uint32)(per_write < 1460 ? per_write : 1460), 0));
        if (g_family == 6) {
            (void)pip_inet6_checksum_buf(head, IPPROTO_TCP, a6, a6);
        } else {
            (void)pip_ip_checksum(z, 20);
            (void)pip_inet_checksum_buf(head, IPPROTO_TCP, a4, a4);
        }
    };
    double cold[3] = {0, 0, 0};  // seconds: first synchronous calls, first and second capture flush
    double tw = now();
    warm();
    cold[0] = now() - tw;
#ifdef PIPCK_AMD
    if (g_mode == CAPTURE || g_mode == CAPTURE_ZC) {
        pip_checksum_amd_capture(true);
        if (g_mode == CAPTURE_ZC) pip_checksum_amd_zero_copy(true);
        g_hold = true;
        for (int i = 0; i < 2; i++) {  // warm this thread's TX queue (both double-buffered batches)
            tw = now();
            warm();
            pip_checksum_amd_flush();
            cold[1 + i] = now() - tw;
        }
    }
#endif
    auto& nif = pip_netif::shared();
    nif.output_ip_data_callback = on_output;
    nif.new_tcp_connect_callback = on_connect;

    const std::vector<uint8_t> opts = {2, 4, (uint8_t)(mss >> 8), (uint8_t)mss, 3, 3, 14, 1};
    for (unsigned k = 0; k < conns; k++) {
        Conn& c = g_conns[k];
        g_connecting = (int)k;
        auto syn = craft(c.port, c.cseq, 0, TH_SYN, opts);
        g_act.start();
        nif.input(syn.data());
        settle();
        g_act.stop("syn -> syn-ack");
        if (!c.tcp) { fprintf(stderr, "no connection %u\n", k); return 1; }
        c.cseq += 1;
        auto ack = craft(c.port, c.cseq, c.srv_next, TH_ACK, {});
        g_act.start();
        nif.input(ack.data());
        acked(k);
        settle();
        g_act.stop("handshake ack");
    }
    g_connecting = -1;
    auto ack_conn = [&](unsigned k) {  // the peer ACKs everything pip sent on connection k (and its PUSH)
        auto a = craft(g_conns[k].port, g_conns[k].cseq, g_conns[k].srv_next, TH_ACK, {});
        g_act.start();
        nif.input(a.data());
        acked(k);
        g_act.stop("ack input");
    };
    auto settle_timed = [&]() {
        g_act.start();
        settle();
        g_act.stop("flush");
    };

    const uint64_t pk0 = g_packets;
    size_t sent = 0;
    unsigned writes = 0;
    int prev = -1;  // --pipeline: the connection whose batch is in flight
    std::vector<std::vector<std::shared_ptr<pip_buf>>> inflight;
    const double t0 = now();
    fprintf(stderr, "timed region starts at %.3f s\n", t0);
    while (sent < total) {
        const unsigned k = writes % conns;
        const size_t want = total - sent < per_write ? total - sent : per_write;
        g_act.start();
        const uint32_t w = g_conns[k].tcp->write(g_conns[k].buf, (pip_uint32)want, false);
        g_act.stop("write");
        if (w == 0) { fprintf(stderr, "write stalled at %zu bytes\n", sent); return 1; }
        sent += w;
        writes++;
#ifdef PIPCK_AMD
        if (pipeline) {
            // start this write's batch; the previous one completes (fields stored)
            g_act.start();
            pip_checksum_amd_submit();
            g_act.stop("submit");
            for (auto& sg : inflight) emit(sg);
            inflight.clear();
            if (prev >= 0) ack_conn((unsigned)prev);
            inflight.swap(g_pending);  // this write's packets (and anything the ACK produced) wait for the next submit
            prev = (int)k;
            continue;
        }
#endif
        settle_timed();
        ack_conn(k);
        settle_timed();
    }
#ifdef PIPCK_AMD
    if (pipeline) {
        g_act.start();
        pip_checksum_amd_complete();
        g_act.stop("complete");
        for (auto& sg : inflight) emit(sg);
        inflight.clear();
        if (prev >= 0) ack_conn((unsigned)prev);
        settle_timed();
    }
#endif
    const double el = now() - t0;
    const uint64_t pk = g_packets - pk0;
#ifdef PIPCK_AMD
    if (g_hold) {
        pip_checksum_amd_zero_copy(false);
        pip_checksum_amd_capture(false);
    }
#endif
    uint64_t stalled, stale;
    double max_age, max_unacked;
    {
        std::lock_guard<std::mutex> g(g_sent_mu);
        stalled = g_resends_stalled, stale = g_resends_stale_clock;
        max_age = g_max_resend_age, max_unacked = g_max_unacked;
    }
    // retransmits: segments pip resent after waiting >= 1 s for their ACK (or not
    // found unacknowledged) -- a stall, and the run fails with exit 3;
    // stale_clock_resends: pip's timer race, younger segments (on_output above);
    // max_action_ms: the longest single input / write / flush of the run;
    // max_unacked_ms: the longest any segment waited for the peer's ACK (pip's
    // timer resends at 1,000)
    printf("{\"tool\": \"stack_tx_bench\", \"mode\": \"%s\", \"family\": %u, \"mss\": %u, \"write_bytes\": %zu, \"payload_bytes\": %zu, "
           "\"writes\": %u, \"conns\": %u, \"pipeline\": %s, \"packets\": %llu, \"seconds\": %.6f, \"payload_gib_per_s\": %.4f, \"mpkt_per_s\": %.4f, "
           "\"digest\": \"%016llx\", \"digest_of\": \"%s\", \"digest_noid\": \"%016llx\", \"wire_bytes\": %llu, \"retransmits\": %llu, "
           "\"stale_clock_resends\": %llu, \"max_resend_age_ms\": %.3f, \"max_action_ms\": %.3f, \"max_action\": \"%s\", "
           "\"max_unacked_ms\": %.3f, "
           "\"cold_ms\": {\"first_calls\": %.3f, \"first_flush\": %.3f, \"second_flush\": %.3f}}\n",
           mode.c_str(), g_family, mss, per_write, sent, writes, conns, pipeline ? "true" : "false", (unsigned long long)pk, el, sent / el / (1u << 30),
           pk / el / 1e6, (unsigned long long)g_digest, g_verify ? "every wire byte" : "ip_sum, th_sum, length",
           (unsigned long long)g_digest_noid, (unsigned long long)g_wire_bytes, (unsigned long long)stalled, (unsigned long long)stale, max_age * 1e3,
           g_act.max * 1e3, g_act.which, max_unacked * 1e3, cold[0] * 1e3, cold[1] * 1e3, cold[2] * 1e3);
    fflush(stdout);
    if (g_dump) fclose(g_dump);
    _exit(stalled ? 3 : 0);  // pip's timer thread is detached and never stops
}
