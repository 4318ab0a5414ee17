/*
 * pipck_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of pip's Internet checksum (plumk97/pip pip/pip_checksum.cpp)
 * plus the CPU twin of the synthetic packet generator.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the reported CPU baseline.  The product
 * (libpipck.so, libpip_checksum_amd.so) never links or calls it.
 *
 * Parity pin: every function here is checked against golden vectors produced
 * by the real pip_checksum.cpp compiled from /root/reference (oracle/Makefile
 * target `ref`, fixtures in tests/golden/, generator script
 * tests/golden/make_golden.py).
 */
#ifndef PIPCK_ORACLE_H
#define PIPCK_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- restatement of pip/pip_checksum.cpp ----------------------------- */
uint32_t ock_fold_uint32(uint32_t x);                                        /* :9-11  */
uint32_t ock_standard_checksum(const void* p, uint32_t len, uint32_t sum);   /* :13-33 */
uint16_t ock_ip_checksum(const void* p, uint32_t len);                       /* :35-39 */
uint16_t ock_inet_checksum(const void* p, uint8_t proto, uint32_t src_s_addr,
                           uint32_t dst_s_addr, uint16_t len);               /* :42-61 */
uint16_t ock_inet6_checksum(const void* p, uint8_t proto, const uint8_t src[16],
                            const uint8_t dst[16], uint16_t len);            /* :63-87 */
uint16_t ock_inet_checksum_chain(const void* const* segs, const uint32_t* lens, uint32_t nseg,
                                 uint8_t proto, uint32_t src_s_addr, uint32_t dst_s_addr); /* :90-115 */
uint16_t ock_inet6_checksum_chain(const void* const* segs, const uint32_t* lens, uint32_t nseg,
                                  uint8_t proto, const uint8_t src[16], const uint8_t dst[16]); /* :118-148 */

/* ---- synthetic workload generator (CPU twin of pipck_gen_* in libpipck) -- */
enum { OCK_HDR_NONE = 0, OCK_HDR_TCP = 1, OCK_HDR_UDP = 2, OCK_HDR_IPV4 = 3 };
enum { OCK_ZIPF_K = 8937 };

uint64_t ock_mix64(uint64_t x);
uint64_t ock_cfg_seed(uint32_t cfg);
/* fill `stride` bytes (stride >= len) of packet `pkt`; bytes [len, stride) are zero */
void ock_gen_packet(uint64_t seed, uint64_t pkt, uint32_t len, uint32_t hdr_kind,
                    uint8_t* dst, uint64_t stride);
void ock_gen_flow4(uint64_t seed, uint32_t flow, uint32_t* src_s_addr, uint32_t* dst_s_addr);
void ock_gen_flow6(uint64_t seed, uint32_t flow, uint8_t src[16], uint8_t dst[16]);
uint32_t ock_zipf_len(uint64_t seed, uint64_t pkt);   /* 64..9000, P(L=63+k) ~ 1/k */

/* ---- batch drivers (for fixtures and the CPU baseline) ----------------- */
/* family 4 or 6 selects the pseudo-header; family 0 = pip_ip_checksum (no pseudo).
 * Packet i lives at arena + i*stride with length lens ? lens[i] : len; flow = (flow_origin+i) % n_flows. */
void ock_batch_fixed(const uint8_t* arena, uint64_t stride, uint32_t len, uint64_t n,
                     int family, uint8_t proto, uint64_t seed, uint32_t n_flows,
                     uint64_t flow_origin, uint16_t* out, int threads);
void ock_batch_ragged(const uint8_t* arena, const uint64_t* offsets, const uint32_t* lens, uint64_t n,
                      int family, uint8_t proto, uint64_t seed, uint32_t n_flows,
                      uint64_t flow_origin, uint16_t* out, int threads);
/* generate a fixed-stride batch of packets [first, first+n) into arena */
void ock_gen_fixed_batch(uint64_t seed, uint64_t first, uint64_t n, uint32_t len, uint32_t hdr_kind,
                         uint8_t* arena, uint64_t stride, int threads);
/* Zipf lengths of packets [first, first+n) and their offsets in the device layout
 * (exclusive prefix of the lengths rounded up to 16); returns the arena size */
uint64_t ock_gen_ragged_layout(uint64_t seed, uint64_t first, uint64_t n, uint32_t* lens, uint64_t* offsets);
/* packets [first, first+n) at arena + offsets[i], lens[i] bytes each, padding to 16 zeroed */
void ock_gen_ragged_fill(uint64_t seed, uint64_t first, uint64_t n, uint32_t hdr_kind, const uint32_t* lens,
                         const uint64_t* offsets, uint8_t* arena, int threads);

#ifdef __cplusplus
}
#endif
#endif
