/*
 * pipck.h -- C ABI of the MI355X Internet-checksum engine (libpipck.so).
 *
 * The engine computes plumk97/pip's one's-complement checksum
 * (pip/pip_checksum.cpp) on AMD MI355X (gfx950) with hand-written HIP kernels.
 * Everything here is plain C: pointers, sizes, int status codes; no torch or
 * C++ types.  Two layers:
 *
 *   1. Batch ABI (device-resident, the performance path).  Packets already in
 *      HBM, results (host-order u16, exactly what pip returns before the
 *      caller's htons) written to HBM.  Stream-ordered, asynchronous.
 *   2. Host ABI (context-owned buffers).  Host batches are pipelined
 *      H2D -> kernel -> D2H on two HIP streams; single packets / pip_buf chains
 *      go through an exact-semantics kernel.  libpip_checksum_amd.so (the C++
 *      drop-in for pip's six functions, include/pip_checksum_amd.h) is built on
 *      this layer.
 *
 * Reference interface each entry point replaces is cited per declaration.
 * Result semantics are bit-exact with pip_checksum.cpp, including 0x0000 being
 * returned as-is (never mapped to 0xFFFF) and per-segment odd-byte padding of
 * chains (pip_checksum.cpp:110-112, :145-147).
 *
 * Domain of the batch ABI: every segment is at most 65535 bytes (the IPv4/IPv6
 * payload-length field).  In that domain pip's u32 accumulator can never wrap,
 * which lets the kernels sum in any order.  The host ABI has no length limit
 * and reproduces pip's mod-2^32 wrap exactly (pip_checksum.cpp:16-23).
 */
#ifndef PIPCK_H
#define PIPCK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------ */
#define PIPCK_OK         0
#define PIPCK_EINVAL     1   /* bad argument (null pointer, zero flows, ...) */
#define PIPCK_ERANGE     2   /* a segment longer than 65535 bytes in a batch */
#define PIPCK_EHIP       3   /* a HIP runtime call failed; see pipck_last_error() */
#define PIPCK_ENODEV     4   /* no gfx950 device / HIP unavailable */
#define PIPCK_ENOMEM     5
#define PIPCK_EBUSY      6   /* a pinned range is still read in place by a queued TX batch */

#define PIPCK_MAX_SEG_LEN 65535u

/* Human-readable text of the last error on the calling thread. */
const char* pipck_last_error(void);
/* ABI version, (major << 16) | minor (PIPCK_VERSION_MAJOR / _MINOR of this
 * header; a minor step only adds entry points).  1.1: the RX verdicts are the
 * 3-bit PIPCK_RX_* values (7 = verified; 3 = nothing failed, payload NOT
 * checked) -- 1.0's single "ok == 3" meant verified.  1.2: the bounded _n forms
 * of the ragged, chain and ring calls.  1.3: the bounded _n forms of the
 * fixed-stride calls (pipck_checksum_fixed_n, pipck_verify_fixed_n,
 * pipck_update_fixed_n). */
#define PIPCK_VERSION_MAJOR 1
#define PIPCK_VERSION_MINOR 3
uint32_t pipck_version(void);

/* ---- flows / pseudo-headers ------------------------------------------ */
/* One flow = one (src, dst, proto) pseudo-header; packet i of a batch uses
 * flow  flow_of ? flow_of[i] : (flow_origin + i) % n_flows.
 * Addresses are in network order exactly as in struct in_addr / in6_addr.  */
typedef struct pipck_flow4 {
    uint32_t src;      /* in_addr.s_addr */
    uint32_t dst;
    uint8_t  proto;    /* IPPROTO_TCP / IPPROTO_UDP / ... */
    uint8_t  pad[3];
} pipck_flow4;

typedef struct pipck_flow6 {
    uint8_t src[16];   /* in6_addr */
    uint8_t dst[16];
    uint8_t proto;
    uint8_t pad[3];
} pipck_flow6;

/* Reduce a device flow table to one u32 pseudo-header base per flow:
 * src hi+lo + dst hi+lo + proto (pip_checksum.cpp:46-55 for v4, :70-82 for v6).
 * The per-packet length term is added by the checksum kernels. */
int pipck_flows4_prepare(const pipck_flow4* d_flows, uint32_t n_flows, uint32_t* d_pseudo, void* stream);
int pipck_flows6_prepare(const pipck_flow6* d_flows, uint32_t n_flows, uint32_t* d_pseudo, void* stream);

/* ---- batch ABI (device pointers, stream-ordered) ----------------------- */
/* d_pseudo == NULL selects pip_ip_checksum semantics (no pseudo-header,
 * pip_checksum.cpp:35-39).  Otherwise the result is
 *   ~fold(pseudo[flow] + hi16(len) + lo16(len) + sum16be(bytes))
 * which equals pip_inet_checksum / pip_inet6_checksum (pip_checksum.cpp:42-87)
 * and pip_inet{,6}_checksum_buf on a single-segment chain (:90-148).        */

/* Fixed stride: packet i = d_arena + i*stride, len bytes.  Any alignment.
 * The kernels load whole aligned 16-byte chunks, so the bytes from the 16-byte
 * boundary at or below d_arena to the one at or above the last packet's end
 * must be readable device memory (every hipMalloc / torch allocation is: they
 * are 256-byte granular); bytes outside the packets never affect a result. */
int pipck_checksum_fixed(const void* d_arena, uint64_t stride, uint32_t len, uint64_t n_packets,
                         const uint32_t* d_pseudo, uint32_t n_flows, const uint32_t* d_flow_of,
                         uint64_t flow_origin, uint16_t* d_out, void* stream);
/* Bounded form (replaces the same per-packet calls, pip_checksum.cpp:42-87,
 * where pip passes the addresses by value -- :42, :63 -- so no index of its
 * can go stale): with d_pseudo, n_flows must be > 0 (PIPCK_EINVAL otherwise),
 * and every d_flow_of entry is checked against it on the device.  A packet
 * whose entry is >= n_flows -- a stale or foreign flow index -- never reads
 * the pseudo-header table: its result is 0 and d_err (optional, device u32)
 * is OR-ed with (1 << PIPCK_ERANGE); every other packet's result is unchanged.
 * The plain name above trusts the entries (n_flows is then unused when
 * d_flow_of is given). */
int pipck_checksum_fixed_n(const void* d_arena, uint64_t stride, uint32_t len, uint64_t n_packets,
                           const uint32_t* d_pseudo, uint32_t n_flows, const uint32_t* d_flow_of,
                           uint64_t flow_origin, uint16_t* d_out, uint32_t* d_err, void* stream);

/* Ragged: one descriptor per packet. */
typedef struct pipck_desc {
    uint64_t offset;   /* byte offset of the packet (or segment) in the arena; any alignment */
    uint32_t len;      /* bytes, <= 65535 */
    uint32_t flow;     /* flow index (ignored when d_pseudo == NULL and for chain segments) */
} pipck_desc;

/* d_err (optional, device u32): OR-ed with (1 << PIPCK_ERANGE) when a
 * descriptor is out of domain; that packet's result is then 0.  This form
 * trusts the descriptors' offsets and flows (only len > 65535 is refused). */
int pipck_checksum_ragged(const void* d_arena, const pipck_desc* d_desc, uint64_t n_packets,
                          const uint32_t* d_pseudo, uint16_t* d_out, uint32_t* d_err, void* stream);
/* Bounded form: arena_bytes = the arena's size (readable from the 16-byte
 * boundary at or below d_arena to the one at or above d_arena + arena_bytes);
 * with d_pseudo, n_flows = its entries (> 0).  A descriptor whose bytes
 * [offset, offset + len) pass arena_bytes (overflow-safe), whose len exceeds
 * 65535 or whose flow is >= n_flows -- a stale or foreign descriptor -- is not
 * read: its result is 0 and d_err gets (1 << PIPCK_ERANGE).  The plain name
 * above is this with arena_bytes and n_flows unbounded. */
int pipck_checksum_ragged_n(const void* d_arena, uint64_t arena_bytes, const pipck_desc* d_desc, uint64_t n_packets,
                            const uint32_t* d_pseudo, uint32_t n_flows, uint16_t* d_out, uint32_t* d_err,
                            void* stream);

/* Packed ragged batch: per-packet lengths, no per-packet descriptors.
 * Packets lie back to back, each starting 16-byte aligned where the previous
 * one's bytes end rounded up to 16: packet i is at d_arena + 16 * c_i, with c_i
 * the sum of ceil(len_j / 16) over j < i (the layout of a TX staging arena and
 * of the synthetic cfg4 batches).  d_lens[i] = packet i's length (u16, so in
 * the batch domain by construction).  d_tile_chunk[t] = c_{64 t} for
 * t = 0 .. ceil(n/64) -- one u64 per 64 packets (pipck_packed_index builds it;
 * a producer that packs the arena knows it anyway) -- so the kernel reads 2 +
 * 1/8 bytes of metadata per packet instead of a 16-byte pipck_desc.  Flow of
 * packet i: d_flow_of ? d_flow_of[i] : (flow_origin + i) % n_flows; d_pseudo ==
 * NULL = pip_ip_checksum semantics.  Results as pipck_checksum_ragged
 * (pip_inet{,6}_checksum, pip_checksum.cpp:42-87).  d_arena 16-byte aligned;
 * a tile's loads start at the 128-byte line holding its first byte, so for an
 * arena that is not 128-byte aligned the bytes of its first line before
 * d_arena are loaded (same line, same page) and discarded. */
int pipck_checksum_packed(const void* d_arena, const uint16_t* d_lens, const uint64_t* d_tile_chunk,
                          uint64_t n_packets, const uint32_t* d_pseudo, uint32_t n_flows, const uint32_t* d_flow_of,
                          uint64_t flow_origin, uint16_t* d_out, void* stream);
/* RX verification of a packed batch (d_ok[i] = 1 iff packet i sums to 0xFFFF). */
int pipck_verify_packed(const void* d_arena, const uint16_t* d_lens, const uint64_t* d_tile_chunk,
                        uint64_t n_packets, const uint32_t* d_pseudo, uint32_t n_flows, const uint32_t* d_flow_of,
                        uint64_t flow_origin, uint8_t* d_ok, void* stream);
/* Bounded forms: arena_bytes = the arena's size (readable up to the 16-byte
 * boundary at or above it).  A tile of 64 packets whose chunks, as d_tile_chunk
 * and d_lens place them, reach past the arena -- a stale or foreign index --
 * is not read at all: each of its packets gets 0 (d_ok 0) and d_err (optional,
 * device u32) is OR-ed with (1 << PIPCK_ERANGE).  With d_flow_of and n_flows >
 * 0, an entry >= n_flows gives its packet 0 and sets the same bit (n_flows 0:
 * the entries are trusted).  The plain names above trust the index and the
 * flow entries (arena_bytes unbounded). */
int pipck_checksum_packed_n(const void* d_arena, uint64_t arena_bytes, const uint16_t* d_lens,
                            const uint64_t* d_tile_chunk, uint64_t n_packets, const uint32_t* d_pseudo,
                            uint32_t n_flows, const uint32_t* d_flow_of, uint64_t flow_origin, uint16_t* d_out,
                            uint32_t* d_err, void* stream);
int pipck_verify_packed_n(const void* d_arena, uint64_t arena_bytes, const uint16_t* d_lens,
                          const uint64_t* d_tile_chunk, uint64_t n_packets, const uint32_t* d_pseudo,
                          uint32_t n_flows, const uint32_t* d_flow_of, uint64_t flow_origin, uint8_t* d_ok,
                          uint32_t* d_err, void* stream);
/* Build d_tile_chunk (ceil(n/64) + 1 u64 entries; the last = the arena's 16-byte
 * chunks) from the lengths, on the stream. */
int pipck_packed_index(const uint16_t* d_lens, uint64_t n_packets, uint64_t* d_tile_chunk, void* stream);

/* Byte-packed ragged batch: packets back to back with NO padding -- packet i
 * at d_arena + b_i, b_i = len_0 + ... + len_{i-1} (a capture buffer, a
 * socket ring read in order, cfg4's bench layout).  d_tile_off[t] = b_{64 t}
 * for t = 0 .. ceil(n/64) (the last entry = the batch's bytes;
 * pipck_packed_bytes_index builds it), so the kernel reads 2 + 1/8 bytes of
 * metadata per packet and nothing but packet bytes otherwise (the 16-byte
 * granular layout above reads its padding too: 0.76 % of cfg4's bytes).
 * d_arena must be 128-byte aligned and readable up to the 16-byte boundary
 * after the last packet (any hipMalloc'd buffer of the batch's size is).
 * Flows and results as pipck_checksum_packed (pip_inet{,6}_checksum,
 * pip_checksum.cpp:42-87); any lengths 0..65535. */
int pipck_checksum_packed_bytes(const void* d_arena, const uint16_t* d_lens, const uint64_t* d_tile_off,
                                uint64_t n_packets, const uint32_t* d_pseudo, uint32_t n_flows,
                                const uint32_t* d_flow_of, uint64_t flow_origin, uint16_t* d_out, void* stream);
int pipck_verify_packed_bytes(const void* d_arena, const uint16_t* d_lens, const uint64_t* d_tile_off,
                              uint64_t n_packets, const uint32_t* d_pseudo, uint32_t n_flows,
                              const uint32_t* d_flow_of, uint64_t flow_origin, uint8_t* d_ok, void* stream);
/* Bounded forms, as pipck_checksum_packed_n: a tile whose bytes reach past
 * arena_bytes (readable to the 16-byte boundary at or above it) is not read;
 * its packets get 0 and d_err gets (1 << PIPCK_ERANGE); d_flow_of entries are
 * bounded by n_flows as there. */
int pipck_checksum_packed_bytes_n(const void* d_arena, uint64_t arena_bytes, const uint16_t* d_lens,
                                  const uint64_t* d_tile_off, uint64_t n_packets, const uint32_t* d_pseudo,
                                  uint32_t n_flows, const uint32_t* d_flow_of, uint64_t flow_origin, uint16_t* d_out,
                                  uint32_t* d_err, void* stream);
int pipck_verify_packed_bytes_n(const void* d_arena, uint64_t arena_bytes, const uint16_t* d_lens,
                                const uint64_t* d_tile_off, uint64_t n_packets, const uint32_t* d_pseudo,
                                uint32_t n_flows, const uint32_t* d_flow_of, uint64_t flow_origin, uint8_t* d_ok,
                                uint32_t* d_err, void* stream);
int pipck_packed_bytes_index(const uint16_t* d_lens, uint64_t n_packets, uint64_t* d_tile_off, void* stream);

/* Chains (pip_buf lists, pip_checksum.cpp:90-148): packet p owns segments
 * [d_seg_begin[p], d_seg_begin[p+1]); its pseudo-header length term is the
 * u32 sum of its segment lengths (pip_buf::total_len).  Every segment is
 * summed from its own start, exactly like pip's per-segment loop.
 * d_scratch: device u32[n_segs]. */
int pipck_checksum_chains(const void* d_arena, const pipck_desc* d_segs, uint64_t n_segs,
                          const uint64_t* d_seg_begin, const uint32_t* d_pkt_flow, uint64_t n_packets,
                          const uint32_t* d_pseudo, uint32_t* d_scratch, uint16_t* d_out, uint32_t* d_err,
                          void* stream);
/* Bounded form, as pipck_checksum_ragged_n for every segment (arena_bytes) and
 * every d_pkt_flow entry (n_flows, > 0 with d_pseudo): a packet holding a
 * refused segment, or with a flow past the table, gets 0 and d_err gets
 * (1 << PIPCK_ERANGE).  In both forms a packet whose [d_seg_begin[p],
 * d_seg_begin[p+1]) is not inside [0, n_segs] gets 0 and sets the same bit --
 * no segment record outside the scratch is read. */
int pipck_checksum_chains_n(const void* d_arena, uint64_t arena_bytes, const pipck_desc* d_segs, uint64_t n_segs,
                            const uint64_t* d_seg_begin, const uint32_t* d_pkt_flow, uint64_t n_packets,
                            const uint32_t* d_pseudo, uint32_t n_flows, uint32_t* d_scratch, uint16_t* d_out,
                            uint32_t* d_err, void* stream);

/* RX verification (a capability pip lacks): same
 * inputs as pipck_checksum_fixed but the packets carry their checksum field;
 * d_ok[i] = 1 when the one's-complement sum including the pseudo-header is
 * 0xFFFF (a valid packet), else 0. */
int pipck_verify_fixed(const void* d_arena, uint64_t stride, uint32_t len, uint64_t n_packets,
                       const uint32_t* d_pseudo, uint32_t n_flows, const uint32_t* d_flow_of,
                       uint64_t flow_origin, uint8_t* d_ok, void* stream);
/* Bounded form, as pipck_checksum_fixed_n: a refused packet verifies as 0. */
int pipck_verify_fixed_n(const void* d_arena, uint64_t stride, uint32_t len, uint64_t n_packets,
                         const uint32_t* d_pseudo, uint32_t n_flows, const uint32_t* d_flow_of,
                         uint64_t flow_origin, uint8_t* d_ok, uint32_t* d_err, void* stream);
/* The same for ragged batches (descriptors as for pipck_checksum_ragged);
 * out-of-domain descriptors verify as 0 and set d_err. */
int pipck_verify_ragged(const void* d_arena, const pipck_desc* d_desc, uint64_t n_packets,
                        const uint32_t* d_pseudo, uint8_t* d_ok, uint32_t* d_err, void* stream);
/* Bounded form, as pipck_checksum_ragged_n. */
int pipck_verify_ragged_n(const void* d_arena, uint64_t arena_bytes, const pipck_desc* d_desc, uint64_t n_packets,
                          const uint32_t* d_pseudo, uint32_t n_flows, uint8_t* d_ok, uint32_t* d_err, void* stream);

/* Incremental update for header rewrites (RFC 1624, SURVEY.md section 8 f4;
 * replaces a full re-run of pip_standard_checksum, pip_checksum.cpp:13-33,
 * after a field change).  Packet i at a = d_arena + i*stride carries pip's
 * checksum of the covered bytes a[cover_off, cover_off+cover_len) (an IPv4
 * header, or an L4 segment with flow pseudo-headers) as the big-endian u16 at
 * a + ck_off (htons(result), as pip's callers store it).  Bytes
 * a[edit_off, edit_off+edit_len) are replaced by d_new + i*new_stride, and
 * when d_pseudo_old / d_pseudo_new are given (prepared bases of the old and
 * new flow tables, e.g. a NAT address rewrite) the pseudo-header changes too;
 * the field is patched as  ~(~HC + ~m + m')  -- RFC 1624 eqn. 3.  The result
 * equals pip's full recomputation bit for bit (the 0x0000/0xFFFF corner eqn.
 * 3 cannot decide alone is settled by scanning that packet).
 * PIPCK_EINVAL unless: checksum field and edit lie in the cover at even
 * offsets from cover_off and do not overlap; edit_len is even or the edit
 * ends the cover; cover_off + cover_len <= stride; cover_len <= 65535. */
int pipck_update_fixed(void* d_arena, uint64_t stride, uint64_t n_packets, uint32_t cover_off, uint32_t cover_len,
                       uint32_t ck_off, uint32_t edit_off, uint32_t edit_len, const void* d_new,
                       uint64_t new_stride, const uint32_t* d_pseudo_old, const uint32_t* d_pseudo_new,
                       uint32_t n_flows, const uint32_t* d_flow_of, uint64_t flow_origin, void* stream);
/* Bounded form: with the pseudo-header tables, n_flows must be > 0 and bounds
 * every d_flow_of entry on the device.  A packet whose entry is >= n_flows is
 * left exactly as it was -- its edit bytes are not replaced and its checksum
 * field is not touched -- and d_err (optional, device u32) is OR-ed with
 * (1 << PIPCK_ERANGE).  The plain name above trusts the entries. */
int pipck_update_fixed_n(void* d_arena, uint64_t stride, uint64_t n_packets, uint32_t cover_off, uint32_t cover_len,
                         uint32_t ck_off, uint32_t edit_off, uint32_t edit_len, const void* d_new,
                         uint64_t new_stride, const uint32_t* d_pseudo_old, const uint32_t* d_pseudo_new,
                         uint32_t n_flows, const uint32_t* d_flow_of, uint64_t flow_origin, uint32_t* d_err,
                         void* stream);


/* ---- synthetic workloads (bench / tests; same spec as oracle/pipck_oracle.c) */
#define PIPCK_HDR_NONE 0
#define PIPCK_HDR_TCP  1
#define PIPCK_HDR_UDP  2
#define PIPCK_HDR_IPV4 3
uint64_t pipck_cfg_seed(uint32_t cfg);
/* packets [first_pkt, first_pkt+n) at d_arena + i*stride (any stride >= len); bytes [len,stride) zeroed */
int pipck_gen_fixed(void* d_arena, uint64_t stride, uint32_t len, uint64_t n, uint64_t first_pkt,
                    uint64_t seed, uint32_t hdr_kind, void* stream);
/* Zipf lengths 64..9000 for packets [first_pkt, first_pkt+n) -> d_len */
int pipck_gen_zipf_lengths(uint32_t* d_len, uint64_t n, uint64_t first_pkt, uint64_t seed, void* stream);
/* descriptors: offsets = exclusive prefix of roundup16(len); flow = (first_pkt+i) % n_flows.
 * *arena_bytes receives the arena size needed (synchronises the stream). */
int pipck_gen_ragged_layout(const uint32_t* d_len, uint64_t n, uint64_t first_pkt, uint32_t n_flows,
                            pipck_desc* d_desc, uint64_t* arena_bytes, void* stream);
int pipck_gen_ragged_fill(void* d_arena, const pipck_desc* d_desc, uint64_t n, uint64_t first_pkt,
                          uint64_t seed, uint32_t hdr_kind, void* stream);
/* byte-packed layout (pipck_checksum_packed_bytes): packets [first_pkt, first_pkt+n) with lengths d_lens */
int pipck_gen_packed_bytes(void* d_arena, const uint16_t* d_lens, const uint64_t* d_tile_off, uint64_t n,
                           uint64_t first_pkt, uint64_t seed, uint32_t hdr_kind, void* stream);
int pipck_gen_flows4(pipck_flow4* d_flows, uint32_t n_flows, uint64_t seed, uint8_t proto, void* stream);
int pipck_gen_flows6(pipck_flow6* d_flows, uint32_t n_flows, uint64_t seed, uint8_t proto, void* stream);

/* ---- host ABI ---------------------------------------------------------- */
typedef struct pipck_ctx pipck_ctx;

/* device < 0 selects the current HIP device. */
int pipck_ctx_create(int device, pipck_ctx** out);
int pipck_ctx_destroy(pipck_ctx* ctx);

/* One segment of a host-memory packet/chain. */
typedef struct pipck_hseg {
    const void* ptr;
    uint32_t len;
} pipck_hseg;

/* pip's exact sequential semantics over host bytes, computed on the device:
 *   sum = init; for each seg: sum = fold(fold((sum + sum16be(seg)) mod 2^32))
 * (pip_standard_checksum, pip_checksum.cpp:13-33, chained as at :110-112).
 * *out receives the final folded u32 in [0, 0xFFFF].  nseg == 0 behaves as one
 * empty segment (a pip_buf chain is never empty).  Synchronous. */
int pipck_host_sum(pipck_ctx* ctx, const pipck_hseg* segs, uint32_t nseg, uint32_t init, uint32_t* out);

/* Host-resident fixed-stride batch: H2D in chunks, kernel, D2H of results,
 * double-buffered over two streams.  h_arena may be pageable or pinned
 * (pinned: see pipck_host_alloc).  Flows are host tables (v4 or v6, by family). */
int pipck_host_checksum_fixed(pipck_ctx* ctx, const void* h_arena, uint64_t stride, uint32_t len,
                              uint64_t n_packets, int family, const void* h_flows, uint32_t n_flows,
                              uint64_t flow_origin, uint16_t* h_out);
/* Host-resident byte-packed ragged batch (a capture buffer or a socket ring read
 * in order: packet i's h_lens[i] bytes right after packet i-1's, no padding),
 * the layout of pipck_checksum_packed_bytes: chunks of whole packets (~64 MiB)
 * go H2D with their lengths, are indexed and checksummed on the device, and the
 * results come back, double-buffered over two streams.  Flows, family and
 * results as pipck_host_checksum_fixed (h_out[i] = pip_inet{,6}_checksum /
 * pip_ip_checksum of packet i, host order).  Synchronous. */
int pipck_host_checksum_packed_bytes(pipck_ctx* ctx, const void* h_arena, const uint16_t* h_lens, uint64_t n_packets,
                                     int family, const void* h_flows, uint32_t n_flows, uint64_t flow_origin,
                                     uint16_t* h_out);
/* This context's per-packet path (pipck_host_sum): 0 = staged (H2D copy,
 * kernel, D2H copy), 1 = zero-copy (the kernel reads the pinned, coherent
 * staging buffer and writes the result to pinned host memory), 2 = auto
 * (zero-copy up to 68 KiB of staged bytes -- any single IP datagram; the
 * mode of a new context), 3 = resident (up to 68 KiB: one 256-thread block of this context stays on
 * the GPU, polls a doorbell in pinned host memory and answers without a
 * launch; it exits after 10 ms without a call, or when the mode changes or
 * the context is destroyed, and relaunches on the next call; larger calls take
 * the staged copies), 4 = resident with the doorbell in fine-grained device
 * memory the host writes directly (large-BAR systems; falls back to mode 3's
 * pinned doorbell where that allocation fails).  Every path computes the same
 * result.  Nothing is read from the environment.
 * WORST CASE of modes 3/4: while the resident block runs it holds one CU slot,
 * and HIP makes every hipFree / hipHostFree / hipDeviceSynchronize in the
 * whole process wait for it to exit -- up to 10 ms after this context's last
 * call (the idle exit).  pipck_ctx_zero_copy(ctx, 2) ends it at once. */
int pipck_ctx_zero_copy(pipck_ctx* ctx, int mode);
void* pipck_host_alloc(size_t bytes);   /* pinned, coherent host memory (device-readable in place) */
/* Pin an existing host range (a utun / socket buffer ring) so the GPU can read
 * it in place at the same address; PIPCK_EINVAL if the runtime maps it to a
 * different device address. */
int pipck_host_register(void* p, size_t bytes);
/* Both refuse (PIPCK_EBUSY, nothing released) while a TX queue holds segments
 * of the range for an in-place read that has not completed; PIPCK_EINVAL for a
 * pointer that does not start such a range. */
int pipck_host_unregister(void* p);
int pipck_host_free(void* p);

/* ---- deferred TX queue -------------------------
 * pip checksums each segment synchronously while building it
 * (pip/protocol/pip_tcp_packet.cpp:124-134, pip/protocol/pip_udp.cpp:50-51,
 * 60-61, pip/pip_netif.cpp:97).  A TX queue defers that: packets are added with
 * their bytes (the payloads of a pip_buf chain, in order), their pseudo-header
 * and the address of their 16-bit checksum field; pipck_txq_flush copies the
 * batch to the device, checksums all of it in one pass and stores
 * htons(result) into every field -- exactly the bytes pip would have written.
 * Bytes are copied at add time, so buffers may be reused after add; the
 * checksum fields must stay valid until flush.  One queue per thread. */
typedef struct pipck_txq pipck_txq;
int pipck_txq_create(pipck_ctx* ctx, pipck_txq** out);
int pipck_txq_destroy(pipck_txq* q);
/* pip_inet_checksum_buf (pip_checksum.cpp:90-115): src/dst as in_addr.s_addr */
int pipck_txq_add4(pipck_txq* q, const pipck_hseg* segs, uint32_t nseg, uint8_t proto, uint32_t src, uint32_t dst,
                   void* csum_field);
/* pip_inet6_checksum_buf (pip_checksum.cpp:118-148): src/dst as in6_addr bytes */
int pipck_txq_add6(pipck_txq* q, const pipck_hseg* segs, uint32_t nseg, uint8_t proto, const uint8_t* src,
                   const uint8_t* dst, void* csum_field);
/* Zero-copy forms: the segments lie in pinned host memory (pipck_host_alloc or
 * pipck_host_register) and are read by the GPU in place when the batch runs --
 * nothing is copied at add time, so they must stay valid and unchanged until
 * the batch completes (flush, or the complete/submit after its submit).  A
 * segment outside every such range is refused (PIPCK_EINVAL): the GPU must
 * never touch an unpinned host page. */
int pipck_txq_add4_zc(pipck_txq* q, const pipck_hseg* segs, uint32_t nseg, uint8_t proto, uint32_t src,
                      uint32_t dst, void* csum_field);
int pipck_txq_add6_zc(pipck_txq* q, const pipck_hseg* segs, uint32_t nseg, uint8_t proto, const uint8_t* src,
                      const uint8_t* dst, void* csum_field);
/* Automatic zero-copy, an explicit per-queue opt-in (off at creation; no
 * environment variable turns it on): pipck_txq_add4/add6 then read every
 * segment that lies in a pinned range in place and copy the others, so pinned
 * segments follow the zero-copy contract above -- the GPU reads them at flush
 * time, so they must stay valid and UNCHANGED until their batch completes.
 * Lets callers that cannot choose the _zc forms -- pip's deferred drop-in,
 * through pip_checksum_amd_zero_copy() -- use pinned utun/socket buffers
 * without a copy.  Every in-place segment holds its pinned range until its
 * batch completes (see pipck_host_free). */
int pipck_txq_auto_zero_copy(pipck_txq* q, int on);
/* Largest flush (staged bytes + metadata) this queue runs in place: the
 * kernels read the coherent pinned staging directly and write the results into
 * it, with no copy command.  Larger flushes take one H2D and one D2H copy.
 * Default 32 MiB (the measured crossover); 0 = always copy.
 * Per queue; no environment variable changes it. */
int pipck_txq_inplace_max(pipck_txq* q, uint64_t bytes);
/* pip_ip_checksum (pip_checksum.cpp:35-39): an IPv4 header with ip_sum = 0 */
int pipck_txq_add_ip(pipck_txq* q, const void* hdr, uint32_t len, void* csum_field);
/* packets added since the last submit/flush */
uint64_t pipck_txq_pending(const pipck_txq* q);
/* Synchronous: returns once every queued field holds its checksum; the queue is then empty. */
int pipck_txq_flush(pipck_txq* q);
/* Asynchronous flush, double-buffered: submit starts the queued batch (H2D,
 * kernels, D2H on the queue's stream) and returns; new adds go to a second
 * batch meanwhile.  complete waits for the submitted batch and stores its
 * fields.  At most one batch is in flight: submit first completes the previous
 * one.  Fields of a submitted batch hold their checksums only after the next
 * complete, submit or flush returns. */
int pipck_txq_submit(pipck_txq* q);
int pipck_txq_complete(pipck_txq* q);
/* packets submitted and not yet completed */
uint64_t pipck_txq_inflight(const pipck_txq* q);

/* ---- RX verification of received packets --------
 * pip never checks a received checksum (pip/pip_netif.cpp:45-77 hands packets
 * to TCP / UDP / ICMP as they come).  pipck_rx_verify checks n IP packets as
 * read from the tun device (IPv4 or IPv6, pkts[i] of lens[i] bytes, link
 * padding after the IP length allowed) in one call and sets ok[i]:
 *   PIPCK_RX_IP_OK       the IPv4 header checksum verifies (always set for IPv6)
 *   PIPCK_RX_L4_OK       no payload checksum failed: it verified, or there was
 *                        none this can check (PIPCK_RX_L4_CHECKED clear)
 *   PIPCK_RX_L4_CHECKED  the payload's checksum was computed: TCP / UDP over
 *                        their pseudo-headers (pip_inet{,6}_checksum), ICMPv4
 *                        over the message (pip_ip_checksum, RFC 792), ICMPv6
 *                        over the IPv6 pseudo-header, next header 58
 * ok[i] == PIPCK_RX_VERIFIED (7): both checksums computed and verified; 3:
 * nothing failed but the payload was NOT checked (an IPv4 or IPv6 fragment, an
 * IPv6 routing header, UDP over IPv4 with a zero checksum, another protocol);
 * malformed lengths or a truncated TCP/UDP/ICMP header leave the L4 bits
 * clear; not IPv4/IPv6, 0.  IPv6 hop-by-hop / destination-options headers and
 * atomic fragments are walked to the upper layer.  Packets that lie in pinned
 * memory (pipck_host_alloc / pipck_host_register) are read in place by the GPU
 * and their ranges held until the call returns; others are copied.  Returns
 * when every ok[i] is set; *n_verified (optional) = packets with ok == 7.
 * One queue per thread (not thread-safe). */
#define PIPCK_RX_IP_OK 1u
#define PIPCK_RX_L4_OK 2u
#define PIPCK_RX_L4_CHECKED 4u
#define PIPCK_RX_VERIFIED 7u
typedef struct pipck_rxq pipck_rxq;
int pipck_rxq_create(pipck_ctx* ctx, pipck_rxq** out);
int pipck_rxq_destroy(pipck_rxq* q);
int pipck_rx_verify(pipck_rxq* q, const void* const* pkts, const uint32_t* lens, uint64_t n, uint8_t* ok,
                    uint64_t* n_verified);

/* The same verdicts for received IP packets already in DEVICE memory, in the
 * byte-packed layout of pipck_checksum_packed_bytes (frame i of d_lens[i]
 * bytes at d_arena + b_i, d_tile_off from pipck_packed_bytes_index; link
 * padding after the IP length allowed): d_ok[i] gets the PIPCK_RX_* bits
 * pipck_rx_verify gives the same bytes.  One kernel on `stream`, no host
 * work: the byte-packed stream sums every frame once, then a lane per packet
 * parses its headers and derives the IP-header and payload verdicts from that
 * sum.  The arena must be 128-byte aligned and readable to the 16-byte
 * boundary after the last frame.  Bounded as pipck_checksum_packed_bytes_n: a tile
 * reaching past arena_bytes is not read, its packets get 0 and d_err
 * (optional) gets (1 << PIPCK_ERANGE).  Asynchronous. */
int pipck_rx_verify_device(const void* d_arena, uint64_t arena_bytes, const uint16_t* d_lens,
                           const uint64_t* d_tile_off, uint64_t n_packets, uint8_t* d_ok, uint32_t* d_err,
                           void* stream);

/* The same verdicts for frames in the fixed-size slots of a receive ring in
 * DEVICE memory: frame i of d_lens[i] bytes at d_arena + i * slot_stride, the
 * rest of each slot unused and never read.  d_arena 16-byte aligned, readable
 * for n_slots * slot_stride bytes; slot_stride a multiple of 16 from 1,024 to
 * 65,536 (PIPCK_EINVAL otherwise).  The lengths are bounded on the device: a
 * slot with d_lens[i] > slot_stride (a corrupt or foreign length) is not read
 * at all -- no load and no header parse leaves its slot -- gets d_ok[i] = 0,
 * and d_err (optional, device u32) gets (1 << PIPCK_ERANGE).  One kernel on
 * `stream`, asynchronous; d_ok[i] as pipck_rx_verify_device.  For slot strides
 * from 4 KiB the kernel's schedule follows the fill this ring (d_arena,
 * slot_stride) reported in earlier calls -- a row stream for full slots,
 * slot groups otherwise; the verdicts are the same either way.  The first call
 * on a ring allocates 8 bytes of device and 16 of pinned host memory that stay
 * with the library (at most 64 rings remembered). */
int pipck_rx_verify_ring_n(const void* d_arena, uint64_t slot_stride, const uint16_t* d_lens, uint64_t n_slots,
                           uint8_t* d_ok, uint32_t* d_err, void* stream);
/* pipck_rx_verify_ring_n without the error word (slots are bounded the same way). */
int pipck_rx_verify_ring(const void* d_arena, uint64_t slot_stride, const uint16_t* d_lens, uint64_t n_slots,
                         uint8_t* d_ok, void* stream);

/* The same verdicts for received frames back to back in HOST memory (a receive
 * buffer read in order, a capture file's records): chunks of ~64 MiB go H2D by
 * DMA with their u16 lengths, pipck_rx_verify_device judges them, the verdicts
 * come back; double-buffered over the context's two streams, PCIe-bound at
 * every frame size (pipck_rx_verify reads each packet in place with a wave of
 * its own: better for scattered packets, slower for small ones).  h_frames
 * pinned (pipck_host_alloc) for full rate; pageable works.  Synchronous;
 * *n_verified (optional) = frames with ok == PIPCK_RX_VERIFIED. */
int pipck_host_rx_verify_packed(pipck_ctx* ctx, const void* h_frames, const uint16_t* h_lens, uint64_t n_frames,
                                uint8_t* h_ok, uint64_t* n_verified);

#ifdef __cplusplus
}
#endif
#endif /* PIPCK_H */
