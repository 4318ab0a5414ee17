// pip_checksum_amd.h -- the C++ drop-in for plumk97/pip's checksum API,
// exported by libpip_checksum_amd.so with the reference's exact signatures and
// therefore its exact mangled names:
//
//   _Z15pip_fold_uint32j                                  pip/pip_checksum.cpp:9   (exported, undeclared)
//   _Z21pip_standard_checksumPKvjj                        pip/pip_checksum.h:17
//   _Z15pip_ip_checksumPKvj                               pip/pip_checksum.h:22
//   _Z17pip_inet_checksumPKvh7in_addrS1_t                 pip/pip_checksum.h:30
//   _Z18pip_inet6_checksumPKvh8in6_addrS1_t               pip/pip_checksum.h:31
//   _Z21pip_inet_checksum_bufSt10shared_ptrI7pip_bufEh7in_addrS2_   pip/pip_checksum.h:33
//   _Z22pip_inet6_checksum_bufSt10shared_ptrI7pip_bufEh8in6_addrS2_ pip/pip_checksum.h:34
//
// pip's callers (pip/pip_netif.cpp:97, pip/protocol/pip_udp.cpp:50,60,
// pip/protocol/pip_tcp_packet.cpp:128,130) keep including pip's own
// pip_checksum.h; a build links this library instead of pip_checksum.cpp
// (INTEGRATION.md).  This header exists for users outside pip's tree.
//
// Every call computes on the MI355X through the C ABI in pipck.h
// (pipck_host_sum); there is no CPU compute path.  A missing or failing GPU
// is fatal: the message is printed and the process aborts, because pip's API
// has no error channel (pip_checksum.h returns bare integers).
#ifndef PIP_CHECKSUM_AMD_H
#define PIP_CHECKSUM_AMD_H

#include <netinet/in.h>
#include <stdint.h>

#include <memory>

class pip_buf;  // pip/pip_buf.h:13 -- only read through its layout (pip_buf_layout.h)

uint32_t pip_fold_uint32(uint32_t num);
uint32_t pip_standard_checksum(const void* payload, uint32_t len, uint32_t sum);
uint16_t pip_ip_checksum(const void* payload, uint32_t len);
uint16_t pip_inet_checksum(const void* payload, uint8_t proto, struct in_addr src, struct in_addr dst, uint16_t len);
uint16_t pip_inet6_checksum(const void* payload, uint8_t proto, struct in6_addr src, struct in6_addr dst,
                            uint16_t len);
uint16_t pip_inet_checksum_buf(std::shared_ptr<pip_buf> buf, uint8_t proto, struct in_addr src, struct in_addr dst);
uint16_t pip_inet6_checksum_buf(std::shared_ptr<pip_buf> buf, uint8_t proto, struct in6_addr src,
                                struct in6_addr dst);

// ---- deferred forms for a batched TX path ----
// Queue a packet on this thread's TX queue instead of checksumming it now.
// The chain's bytes are copied at call time -- unless this thread turned
// zero-copy on (below): then segments in pinned memory are read at flush time.
// pip_checksum_amd_flush() checksums every queued packet on the GPU in one
// batch and stores htons(checksum) into each csum_field (what
// pip_tcp_packet.cpp:132-133 / pip_udp.cpp:51,61 / pip_netif.cpp:97 store), so
// it must run before those packets are output.
void pip_inet_checksum_buf_deferred(std::shared_ptr<pip_buf> buf, uint8_t proto, struct in_addr src,
                                    struct in_addr dst, void* csum_field);
void pip_inet6_checksum_buf_deferred(std::shared_ptr<pip_buf> buf, uint8_t proto, struct in6_addr src,
                                     struct in6_addr dst, void* csum_field);
void pip_ip_checksum_deferred(const void* hdr, uint32_t len, void* csum_field);
uint64_t pip_checksum_amd_pending();
void pip_checksum_amd_flush();
// Pipelined form of flush (pipck_txq_submit / pipck_txq_complete): submit
// starts the queued batch on the GPU and returns, so the thread can build the
// next batch meanwhile; the submitted packets' fields are stored by the next
// submit, complete or flush on this thread -- output them only after that.
void pip_checksum_amd_submit();
void pip_checksum_amd_complete();

// Zero-copy for this thread's queue -- an explicit opt-in, off by default and
// never switched on by the environment.  While on, every queued segment that
// lies in pinned memory (pipck_host_alloc / pipck_host_register, include/pipck.h)
// is NOT copied: the GPU reads it in place when its batch runs, so its bytes
// must stay unchanged until the flush (or the complete/submit after its
// submit) returns.  The queue keeps each such chain (shared_ptr) alive until
// then, and the pinned range cannot be freed meanwhile (PIPCK_EBUSY).
void pip_checksum_amd_zero_copy(bool on);

// Resident per-call service for this thread (pipck_ctx_zero_copy mode 3,
// include/pipck.h): pip's synchronous calls are answered by a GPU block that
// stays resident and polls a doorbell instead of a kernel launch per call.  The
// block exits after 10 ms without a call and restarts on the next one.  Off by
// default (auto mode); only this call turns it on (no environment variable).
// WORST CASE: while the block runs, every hipFree / hipHostFree /
// hipDeviceSynchronize anywhere in the process waits for it to exit, i.e. up
// to 10 ms after this thread's last checksum call; pip_checksum_amd_resident
// (false) ends it at once.  A latency path only: at ~7-9 us per call it cannot
// beat pip's own ~0.5 us loop on a 1,480-B segment.
void pip_checksum_amd_resident(bool on);

// Capture mode for this thread: pip's UNCHANGED TX call sites become queue
// entries.  While on, the three calls pip's TX path makes --
//   pip_ip_checksum(hdr, len >= 20)            ip_sum  at hdr + 10  (pip_netif.cpp:94-97)
//   pip_inet{,6}_checksum_buf(chain, TCP, ..)  th_sum  at head + 16 (pip_tcp_packet.cpp:128-133)
//   pip_inet{,6}_checksum_buf(chain, UDP, ..)  uh_sum  at head + 6  (pip_udp.cpp:50-51, 60-61)
// -- queue the packet with that field and return 0; pip then stores htons(0),
// which the next flush (or complete) overwrites with htons(checksum), the bytes
// pip's own build writes.  So the packets (their pip_buf chains, which
// pip_netif::output4 hands to output_ip_data_callback) must be held by the
// caller and output only after that flush.  Other calls compute at once.
void pip_checksum_amd_capture(bool on);
bool pip_checksum_amd_capturing();

// ---- RX batch verification (pip itself never verifies) ----
// Verify n received IP packets (as read from the tun device: IPv4 or IPv6,
// pkts[i] of lens[i] bytes) in one GPU batch on this thread.  ok[i] bits:
//   PIP_RX_IP_OK       the IPv4 header checksum verifies (always set for IPv6)
//   PIP_RX_L4_OK       no payload checksum failed: it verified, or there was
//                      none this call can check (see PIP_RX_L4_CHECKED)
//   PIP_RX_L4_CHECKED  the payload's checksum WAS computed: TCP or UDP over its
//                      pseudo-header, ICMPv4 over the message alone (RFC 792;
//                      pip_ip_checksum's arithmetic), ICMPv6 over the IPv6
//                      pseudo-header with next header 58 (RFC 4443 2.3)
// ok[i] == PIP_RX_VERIFIED (7): both checksums computed and verified.
// ok[i] == PIP_RX_IP_OK | PIP_RX_L4_OK (3): nothing failed but the payload was
// NOT checked -- an IPv4 fragment (MF or offset set: its L4 checksum spans the
// reassembled datagram), UDP over IPv4 with a zero checksum (RFC 768), an IPv6
// fragment or routing header, another protocol.  A caller that must not pass
// unchecked packets accepts 7 only.  A damaged checksum clears its OK bit (a
// checked-and-failed payload reads PIP_RX_L4_CHECKED without PIP_RX_L4_OK); a
// malformed packet (lengths that do not fit, a truncated TCP/UDP/ICMP header,
// not IPv4/IPv6) gets no L4 bits, or 0.  IPv6 hop-by-hop / destination-options
// headers and atomic fragments are walked to the upper layer.  Packets in
// pinned memory are read in place; packets that lie back to back in one buffer
// (pkts[i + 1] == pkts[i] + lens[i]) go to the GPU in one DMA per chunk
// (pipck_host_rx_verify_packed) -- same bits; the call returns when every
// result is known.  Returns the number of packets with ok == PIP_RX_VERIFIED.  Uses its
// own queue: pip's deferred TX batch is not touched.
//
// The meaning of ok[] changed once, in place (round 4): in RX ABI 1 a verified
// packet read ok == 3 and the return value counted those; since RX ABI 2 a
// verified packet reads 7 and 3 means NOT checked.  Code written for ABI 1
// would reject every verified packet and accept exactly the unchecked ones, so
// a caller checks the ABI it compiled against (PIP_CHECKSUM_AMD_RX_ABI) and the
// one the loaded library implements (pip_checksum_amd_rx_abi()) -- INTEGRATION.md
// "Migration notes".
#define PIP_CHECKSUM_AMD_RX_ABI 2
#define PIP_RX_IP_OK 1u
#define PIP_RX_L4_OK 2u
#define PIP_RX_L4_CHECKED 4u
#define PIP_RX_VERIFIED 7u
extern "C" uint32_t pip_checksum_amd_verify_packets(const void* const* pkts, const uint32_t* lens, uint32_t n,
                                                    uint8_t* ok);
extern "C" uint32_t pip_checksum_amd_rx_abi(void);  // PIP_CHECKSUM_AMD_RX_ABI of the loaded library

#endif
