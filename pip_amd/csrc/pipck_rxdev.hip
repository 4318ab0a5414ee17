// pipck_rxdev.hip -- RX verification of received IP packets already in device
// memory (SURVEY.md section 8 f2 at HBM rate; pipck_rx_verify_device).
//
// pipck_rx_verify (pipck_rx.hip) takes packets in host memory: the host parses
// what each checksum covers and the GPU reads the bytes over PCIe (~50 GB/s).
// Packets that already sit in HBM -- a receive ring filled by a peer device,
// a capture replayed from device memory -- need no host at all.  They come in
// the byte-packed layout of pipck_checksum_packed_bytes (packets back to back,
// u16 lengths, a u64 byte offset per 64 packets) and are verified in ONE pass
// of k_packedb_rx, the cfg4 bench kernel's body (k_packedb) with RX = true:
//
//  1. the tile's stream, unchanged, leaves each packet's folded big-endian sum
//     S_all over its whole frame, relative to the packet's first byte;
//  2. while the rows stream by, the chunks of every packet's header window
//     (its first six aligned 16-byte chunks) are also copied to LDS; at the
//     tile's end each lane takes its packet's window from there (rx_from_window,
//     pipck_rxparse.hpp), realigns it to the packet start in registers, parses
//     the fields pipck_rx_verify's host parser reads (rx_parse: IHL, lengths,
//     fragment field, protocol, the IPv6 extension-header walk, addresses),
//     sums the IPv4 header exactly, and gets the L4 message's sum without
//     reading it again: S_l4 = S_all - S_pre - S_post (mod 0xFFFF), where
//     S_pre covers the bytes before the L4 message (IP header and extension
//     headers) and S_post the link padding after the IP length.
//
// Why the subtraction is exact: every sum here is taken
// relative to the packet's first byte, so sums of disjoint byte ranges add
// mod 0xFFFF; pip's verdict for a payload with its checksum field included is
// fold(fold(P + T)) == 0xFFFF with T the message's big-endian sum, which for
// P > 0 (TCP, UDP, ICMPv6: the protocol number is in P) depends only on
// (P + T) mod 0xFFFF.  ICMPv4 has no pseudo-header (P = 0): there "T = 0"
// (an all-zero message, whose correct checksum is 0xFFFF, not 0) must be told
// apart from T = k x 0xFFFF, so the kernel checks the message for a non-zero
// byte (its first 8 bytes from registers, the rest only if those are zero).
#include "pipck_common.hpp"

extern "C" {

int pipck_rx_verify_device(const void* d_arena, uint64_t arena_bytes, const uint16_t* d_lens,
                           const uint64_t* d_tile_off, uint64_t n, uint8_t* d_ok, uint32_t* d_err, void* stream) {
    return pipck::launch_packedb_rx(d_arena, arena_bytes, d_lens, d_tile_off, n, d_ok, d_err,
                                    pipck::as_stream(stream));
}

}  // extern "C"
