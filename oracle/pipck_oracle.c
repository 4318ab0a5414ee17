/*
 * pipck_oracle.c -- TEST INFRASTRUCTURE ONLY (see pipck_oracle.h).
 *
 * A clean-room CPU restatement of plumk97/pip's checksum, written from the
 * behaviour of /root/reference/pip/pip_checksum.cpp (cited per function), and
 * the CPU twin of the synthetic workload generator.  Scalar on purpose: this
 * is the parity oracle and the "pip's own CPU algorithm" baseline, so it keeps
 * the reference's big-endian 16-bit word loop and its u32 wrap-around.
 */
#include "pipck_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* pip/pip_checksum.cpp:9-11 -- one end-around fold of a 32-bit sum. */
uint32_t ock_fold_uint32(uint32_t x) { return (x & 0xFFFFu) + (x >> 16); }

/* pip/pip_checksum.cpp:13-33.  Big-endian byte pairs p[i]<<8|p[i+1] are added
 * to a u32 that may wrap mod 2^32; an odd trailing byte counts as p[n-1]<<8;
 * then two folds.  Result is in [0, 0xFFFF]. */
uint32_t ock_standard_checksum(const void* payload, uint32_t len, uint32_t sum) {
    const uint8_t* p = (const uint8_t*)payload;
    uint32_t i = 0;
    for (; i + 1 < len; i += 2) sum += ((uint32_t)p[i] << 8) | p[i + 1];
    if (i < len) sum += (uint32_t)p[i] << 8;
    return ock_fold_uint32(ock_fold_uint32(sum));
}

/* pip/pip_checksum.cpp:35-39 */
uint16_t ock_ip_checksum(const void* payload, uint32_t len) {
    return (uint16_t)~(uint16_t)ock_standard_checksum(payload, len, 0);
}

/* ntohl() of a network-order word as it sits in memory (pip_checksum.cpp:47,51) */
static uint32_t be32_at(const uint8_t* b) {
    return ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
}

static uint32_t addr4_terms(uint32_t s_addr) {
    uint8_t b[4];
    memcpy(b, &s_addr, 4);
    uint32_t a = be32_at(b);
    return (a >> 16) + (a & 0xFFFFu);
}

static uint32_t addr6_terms(const uint8_t* a16) {
    uint32_t s = 0;
    for (int i = 0; i < 4; i++) {
        uint32_t a = be32_at(a16 + 4 * i);
        s += (a >> 16) + (a & 0xFFFFu);
    }
    return s;
}

/* pip/pip_checksum.cpp:42-61.  Pseudo-header: src hi+lo, dst hi+lo, proto, u16 len. */
uint16_t ock_inet_checksum(const void* p, uint8_t proto, uint32_t src, uint32_t dst, uint16_t len) {
    uint32_t sum = addr4_terms(src) + addr4_terms(dst) + proto + len;
    return (uint16_t)~(uint16_t)ock_standard_checksum(p, len, sum);
}

/* pip/pip_checksum.cpp:63-87.  Same as above, with four big-endian words per address.
 * The reference interleaves src[i], dst[i]; addition order does not matter. */
uint16_t ock_inet6_checksum(const void* p, uint8_t proto, const uint8_t src[16], const uint8_t dst[16],
                            uint16_t len) {
    uint32_t sum = addr6_terms(src) + addr6_terms(dst) + proto + len;
    return (uint16_t)~(uint16_t)ock_standard_checksum(p, len, sum);
}

/* pip/pip_checksum.cpp:90-115.  Length term is the chain's u32 total_len split hi+lo
 * (:105-107); every segment is summed from its own start and folded (:110-112). */
uint16_t ock_inet_checksum_chain(const void* const* segs, const uint32_t* lens, uint32_t nseg,
                                 uint8_t proto, uint32_t src, uint32_t dst) {
    uint32_t total = 0;
    for (uint32_t s = 0; s < nseg; s++) total += lens[s];
    uint32_t sum = addr4_terms(src) + addr4_terms(dst) + proto + (total >> 16) + (total & 0xFFFFu);
    for (uint32_t s = 0; s < nseg; s++) sum = ock_standard_checksum(segs[s], lens[s], sum);
    /* pip's chain always holds at least one pip_buf, so its loop folds at least once;
     * zero segments are treated as one empty segment (as oracle/ref_bridge.cpp builds it). */
    if (nseg == 0) sum = ock_standard_checksum(NULL, 0, sum);
    return (uint16_t)~(uint16_t)sum;
}

/* pip/pip_checksum.cpp:118-148 */
uint16_t ock_inet6_checksum_chain(const void* const* segs, const uint32_t* lens, uint32_t nseg,
                                  uint8_t proto, const uint8_t src[16], const uint8_t dst[16]) {
    uint32_t total = 0;
    for (uint32_t s = 0; s < nseg; s++) total += lens[s];
    uint32_t sum = addr6_terms(src) + addr6_terms(dst) + proto + (total >> 16) + (total & 0xFFFFu);
    for (uint32_t s = 0; s < nseg; s++) sum = ock_standard_checksum(segs[s], lens[s], sum);
    if (nseg == 0) sum = ock_standard_checksum(NULL, 0, sum);
    return (uint16_t)~(uint16_t)sum;
}

/* ======================================================================
 * Synthetic workload generator.  The spec (shared with the device
 * generator in pip_amd/csrc/pipck_gen.hip, written independently):
 *   mix64      = SplitMix64 finalizer
 *   key(pkt)   = mix64(seed ^ mix64(pkt))
 *   class      = mix64(key ^ 0xA5A5A5A5A5A5A5A5) % 1000 : 0 all-zero, 1 all-0xFF, else random
 *   random     : byte b = byte (b%8) of mix64(key + b/8), little-endian
 *   headers    : TCP  -> th_off byte[12]=0x50 (random class), th_sum [16,17]=0
 *                UDP  -> uh_ulen [4,5]=len BE (random class), uh_sum [6,7]=0
 *                IPv4 -> byte[0]=0x45 (random class), ip_sum [10,11]=0
 *   flows      : fkey = mix64(seed ^ 0xF10F10F1 ^ mix64(flow)); v4 src=(u32)fkey,
 *                dst=(u32)(fkey>>32) as in-memory s_addr; v6 src = LE bytes of
 *                mix64(fkey+1), mix64(fkey+2); dst = mix64(fkey+3), mix64(fkey+4)
 *   zipf len   : w_k = floor(2^40/k), k=1..8937; u = mix64(key ^ 0x5A5A5A5A5A5A5A5A) % W;
 *                k = min{k : cum_k > u}; len = 63 + k
 * ====================================================================== */
uint64_t ock_mix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint64_t ock_cfg_seed(uint32_t cfg) { return 0x9E3779B97F4A7C15ull ^ (uint64_t)cfg; }

static uint64_t pkt_key(uint64_t seed, uint64_t pkt) { return ock_mix64(seed ^ ock_mix64(pkt)); }

void ock_gen_packet(uint64_t seed, uint64_t pkt, uint32_t len, uint32_t hdr_kind, uint8_t* dst,
                    uint64_t stride) {
    uint64_t key = pkt_key(seed, pkt);
    uint32_t cls = (uint32_t)(ock_mix64(key ^ 0xA5A5A5A5A5A5A5A5ull) % 1000u);
    if (cls == 0) {
        memset(dst, 0, len);
    } else if (cls == 1) {
        memset(dst, 0xFF, len);
    } else {
        for (uint32_t b = 0; b < len; b += 8) {
            uint64_t w = ock_mix64(key + b / 8);
            for (uint32_t i = 0; i < 8 && b + i < len; i++) dst[b + i] = (uint8_t)(w >> (8 * i));
        }
    }
    if (hdr_kind == OCK_HDR_TCP) {
        if (cls > 1 && len > 12) dst[12] = 0x50;
        if (len > 16) dst[16] = 0;
        if (len > 17) dst[17] = 0;
    } else if (hdr_kind == OCK_HDR_UDP) {
        if (cls > 1 && len > 5) { dst[4] = (uint8_t)(len >> 8); dst[5] = (uint8_t)len; }
        if (len > 6) dst[6] = 0;
        if (len > 7) dst[7] = 0;
    } else if (hdr_kind == OCK_HDR_IPV4) {
        if (cls > 1 && len > 0) dst[0] = 0x45;
        if (len > 10) dst[10] = 0;
        if (len > 11) dst[11] = 0;
    }
    if (stride > len) memset(dst + len, 0, stride - len);
}

static uint64_t flow_key(uint64_t seed, uint32_t flow) {
    return ock_mix64(seed ^ 0xF10F10F1ull ^ ock_mix64(flow));
}

void ock_gen_flow4(uint64_t seed, uint32_t flow, uint32_t* src, uint32_t* dst) {
    uint64_t f = flow_key(seed, flow);
    *src = (uint32_t)f;
    *dst = (uint32_t)(f >> 32);
}

static void put_le64(uint8_t* d, uint64_t v) {
    for (int i = 0; i < 8; i++) d[i] = (uint8_t)(v >> (8 * i));
}

void ock_gen_flow6(uint64_t seed, uint32_t flow, uint8_t src[16], uint8_t dst[16]) {
    uint64_t f = flow_key(seed, flow);
    put_le64(src, ock_mix64(f + 1));
    put_le64(src + 8, ock_mix64(f + 2));
    put_le64(dst, ock_mix64(f + 3));
    put_le64(dst + 8, ock_mix64(f + 4));
}

static uint64_t g_zipf_cum[OCK_ZIPF_K];
static pthread_once_t g_zipf_once = PTHREAD_ONCE_INIT;

static void zipf_init(void) {
    uint64_t c = 0;
    for (uint32_t k = 1; k <= OCK_ZIPF_K; k++) {
        c += (1ull << 40) / k;
        g_zipf_cum[k - 1] = c;
    }
}

uint32_t ock_zipf_len(uint64_t seed, uint64_t pkt) {
    pthread_once(&g_zipf_once, zipf_init);
    uint64_t u = ock_mix64(pkt_key(seed, pkt) ^ 0x5A5A5A5A5A5A5A5Aull) % g_zipf_cum[OCK_ZIPF_K - 1];
    uint32_t lo = 0, hi = OCK_ZIPF_K - 1; /* first index with cum > u */
    while (lo < hi) {
        uint32_t mid = (lo + hi) / 2;
        if (g_zipf_cum[mid] > u) hi = mid; else lo = mid + 1;
    }
    return 63u + (lo + 1u);
}

/* ---- threaded batch drivers ------------------------------------------- */
typedef struct {
    const uint8_t* arena;
    uint64_t stride;
    const uint64_t* offsets;
    const uint32_t* lens;
    uint32_t len;
    uint64_t begin, end;
    int family;
    uint8_t proto;
    uint64_t seed;
    uint32_t n_flows;
    uint64_t flow_origin;
    uint16_t* out;
    uint32_t hdr_kind;
    uint8_t* gen_arena;
} job_t;

static void* batch_worker(void* arg) {
    job_t* j = (job_t*)arg;
    for (uint64_t i = j->begin; i < j->end; i++) {
        const uint8_t* p = j->offsets ? j->arena + j->offsets[i] : j->arena + i * j->stride;
        uint32_t len = j->lens ? j->lens[i] : j->len;
        uint32_t flow = (uint32_t)((j->flow_origin + i) % j->n_flows);
        uint16_t r;
        if (j->family == 4) {
            uint32_t s, d;
            ock_gen_flow4(j->seed, flow, &s, &d);
            r = ock_inet_checksum(p, j->proto, s, d, (uint16_t)len);
        } else if (j->family == 6) {
            uint8_t s[16], d[16];
            ock_gen_flow6(j->seed, flow, s, d);
            r = ock_inet6_checksum(p, j->proto, s, d, (uint16_t)len);
        } else {
            r = ock_ip_checksum(p, len);
        }
        j->out[i] = r;
    }
    return NULL;
}

static void* gen_worker(void* arg) {
    job_t* j = (job_t*)arg;
    for (uint64_t i = j->begin; i < j->end; i++)
        ock_gen_packet(j->seed, j->flow_origin + i, j->len, j->hdr_kind, j->gen_arena + i * j->stride, j->stride);
    return NULL;
}

static void* gen_ragged_worker(void* arg) {
    job_t* j = (job_t*)arg;
    for (uint64_t i = j->begin; i < j->end; i++) {
        uint32_t len = j->lens[i];
        ock_gen_packet(j->seed, j->flow_origin + i, len, j->hdr_kind, j->gen_arena + j->offsets[i], (len + 15u) & ~15u);
    }
    return NULL;
}

static void run_jobs(job_t* proto_job, uint64_t n, int threads, void* (*fn)(void*)) {
    if (threads < 1) threads = 1;
    if ((uint64_t)threads > n) threads = n ? (int)n : 1;
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    job_t* jobs = (job_t*)calloc((size_t)threads, sizeof(job_t));
    for (int t = 0; t < threads; t++) {
        jobs[t] = *proto_job;
        jobs[t].begin = n * (uint64_t)t / (uint64_t)threads;
        jobs[t].end = n * (uint64_t)(t + 1) / (uint64_t)threads;
        if (t == 0) continue;
        pthread_create(&th[t], NULL, fn, &jobs[t]);
    }
    fn(&jobs[0]);
    for (int t = 1; t < threads; t++) pthread_join(th[t], NULL);
    free(jobs);
    free(th);
}

void ock_batch_fixed(const uint8_t* arena, uint64_t stride, uint32_t len, uint64_t n, int family,
                     uint8_t proto, uint64_t seed, uint32_t n_flows, uint64_t flow_origin, uint16_t* out,
                     int threads) {
    job_t j;
    memset(&j, 0, sizeof j);
    j.arena = arena; j.stride = stride; j.len = len; j.family = family; j.proto = proto;
    j.seed = seed; j.n_flows = n_flows ? n_flows : 1; j.flow_origin = flow_origin; j.out = out;
    run_jobs(&j, n, threads, batch_worker);
}

void ock_batch_ragged(const uint8_t* arena, const uint64_t* offsets, const uint32_t* lens, uint64_t n,
                      int family, uint8_t proto, uint64_t seed, uint32_t n_flows, uint64_t flow_origin,
                      uint16_t* out, int threads) {
    job_t j;
    memset(&j, 0, sizeof j);
    j.arena = arena; j.offsets = offsets; j.lens = lens; j.family = family; j.proto = proto;
    j.seed = seed; j.n_flows = n_flows ? n_flows : 1; j.flow_origin = flow_origin; j.out = out;
    run_jobs(&j, n, threads, batch_worker);
}

void ock_gen_fixed_batch(uint64_t seed, uint64_t first, uint64_t n, uint32_t len, uint32_t hdr_kind,
                         uint8_t* arena, uint64_t stride, int threads) {
    job_t j;
    memset(&j, 0, sizeof j);
    j.seed = seed; j.flow_origin = first; j.len = len; j.hdr_kind = hdr_kind;
    j.gen_arena = arena; j.stride = stride;
    run_jobs(&j, n, threads, gen_worker);
}

uint64_t ock_gen_ragged_layout(uint64_t seed, uint64_t first, uint64_t n, uint32_t* lens, uint64_t* offsets) {
    uint64_t off = 0;
    for (uint64_t i = 0; i < n; i++) {
        lens[i] = ock_zipf_len(seed, first + i);
        offsets[i] = off;
        off += (lens[i] + 15u) & ~15u;
    }
    return off;
}

void ock_gen_ragged_fill(uint64_t seed, uint64_t first, uint64_t n, uint32_t hdr_kind, const uint32_t* lens,
                         const uint64_t* offsets, uint8_t* arena, int threads) {
    job_t j;
    memset(&j, 0, sizeof j);
    j.seed = seed; j.flow_origin = first; j.hdr_kind = hdr_kind; j.lens = lens; j.offsets = offsets;
    j.gen_arena = arena;
    run_jobs(&j, n, threads, gen_ragged_worker);
}
