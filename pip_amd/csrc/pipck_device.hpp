// pipck_device.hpp -- device-side arithmetic of the checksum engine (gfx950).
//
// Why order-free summation is exact.  pip (pip/pip_checksum.cpp:13-33) adds
// big-endian 16-bit words into a u32 and folds twice.  For a segment of at most
// 65535 bytes plus any pseudo-header, that u32 cannot wrap, and for a total T
// that did not wrap, fold(fold(T)) is
//     0                        if T == 0
//     1 + (T - 1) mod 0xFFFF   otherwise,
// i.e. it depends only on T mod 0xFFFF and on whether T == 0.  Both are
// preserved by every reduction used below:
//   * 2^16 == 1 (mod 0xFFFF), so a little-endian u32 word w contributes
//     w mod 0xFFFF == lo16(w) + hi16(w), and a u64 sum of LE u32 words has the
//     residue of the LE 16-bit word sum;
//   * the big-endian sum of a segment is 256 x its LE sum (mod 0xFFFF) when the
//     segment starts at an even address, and equal to it when it starts at an
//     odd one (pip restarts byte pairing at every chain segment,
//     pip_checksum.cpp:110-112) -- multiplying by 256 mod 0xFFFF is a 16-bit
//     byte swap;
//   * every fold used here maps 0 -> 0 and nonzero -> nonzero.
// So the kernels load 16-byte chunks at aligned addresses, sum LE dwords in any
// order, and only fix byte order once per segment.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pipck {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// residue- and zero-preserving folds
__device__ __forceinline__ uint32_t fold64(uint64_t x) {
    return (uint32_t)(x & 0xFFFFu) + (uint32_t)((x >> 16) & 0xFFFFu) + (uint32_t)((x >> 32) & 0xFFFFu) +
           (uint32_t)(x >> 48);
}
__device__ __forceinline__ uint32_t fold32(uint32_t x) { return (x & 0xFFFFu) + (x >> 16); }
// pip_fold_uint32 applied twice (pip_checksum.cpp:29-30); result in [0, 0xFFFF]
__device__ __forceinline__ uint32_t fold16(uint32_t x) { return fold32(fold32(x)); }
__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | (x >> 8); }

// Byte masks of a 16-byte chunk as two little-endian u64 halves.  The low n
// bytes (n clamped to [0, 16]) are ~0 >> (64 - 8k) per half -- one 64-bit
// shift each; k == 0 is selected explicitly because a shift by 64 wraps.
struct Mask128 {
    uint64_t m0, m1;
};
__device__ __forceinline__ uint64_t low_bytes64(int k) {  // k in [0, 8]
    return k > 0 ? (~0ull >> (64 - 8 * k)) : 0ull;
}
__device__ __forceinline__ Mask128 low_bytes(int n) {
    return {low_bytes64(min(max(n, 0), 8)), low_bytes64(min(max(n - 8, 0), 8))};
}
__device__ __forceinline__ u32x4 and_mask(u32x4 v, Mask128 m) {
    v.x &= (uint32_t)m.m0;
    v.y &= (uint32_t)(m.m0 >> 32);
    v.z &= (uint32_t)m.m1;
    v.w &= (uint32_t)(m.m1 >> 32);
    return v;
}
// Keep bytes [0, hi) of a chunk: a segment's last chunk.
__device__ __forceinline__ u32x4 mask_tail(u32x4 v, int hi) { return and_mask(v, low_bytes(hi)); }
// Keep bytes [lo, hi) of a chunk (0 <= lo; hi may lie outside [0, 16]).
__device__ __forceinline__ u32x4 mask_chunk(u32x4 v, int lo, int hi) {
    const Mask128 a = low_bytes(hi), b = low_bytes(lo);
    return and_mask(v, Mask128{a.m0 & ~b.m0, a.m1 & ~b.m1});
}

__device__ __forceinline__ uint64_t sum4(u32x4 v) {
    return (uint64_t)v.x + (uint64_t)v.y + (uint64_t)v.z + (uint64_t)v.w;
}

// lo16(w) + hi16(w) + acc in one v_dot2_u32_u16 against (1, 1): residue- and
// zero-preserving like the folds above, and a u32 cannot overflow before
// 2^32 / (2 * 0xFFFF) = 32768 dwords have been added.
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t dot_fold(uint32_t w, uint32_t acc) {
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, w), u16x2{1, 1}, acc, false);
}
// A 16-byte chunk added into a u32 partial with four dot2 ops (<= 2^19 per chunk)
__device__ __forceinline__ uint32_t dot4(const u32x4& v, uint32_t acc) {
    return dot_fold(v.w, dot_fold(v.z, dot_fold(v.y, dot_fold(v.x, acc))));
}

// LE residue sum of a segment -> pip's big-endian folded segment sum in [0,0xFFFF]
__device__ __forceinline__ uint32_t be_fold(uint32_t le_residue_sum, uintptr_t seg_addr) {
    uint32_t w = fold16(le_residue_sum);
    return (seg_addr & 1) ? w : bswap16(w);
}

// pseudo-header length term: pip adds total_len hi + lo (pip_checksum.cpp:140-142);
// identical to the flat variants' (u16)len (:91) inside the batch domain.
__device__ __forceinline__ uint32_t len_term(uint32_t len) { return (len >> 16) + (len & 0xFFFFu); }

// ~(u16)fold(fold(P + F)) -- the two folds of pip_standard_checksum
// (pip_checksum.cpp:29-30) and the final ~ of pip_inet_checksum (:60),
// pip_inet6_checksum (:86), pip_inet_checksum_buf (:114), pip_inet6_checksum_buf (:147)
__device__ __forceinline__ uint16_t finish(uint32_t pseudo_total, uint32_t be_sum) {
    return (uint16_t)~fold16(pseudo_total + be_sum);
}

// Pseudo-header base of a packet whose flow comes from a flow_of entry f.  The
// fixed-stride kernels get nf = the table's entries in the bounded _n forms
// (UINT32_MAX in the plain ones: trusted).  pip has no flow index to go stale --
// it passes the addresses by value on every call (pip_checksum.cpp:42,63) -- so
// an entry past the table is this engine's own failure mode and must never
// become a read outside the table: `bad` is set, the table is not read, and the
// caller stores 0 for that packet and reports it with flow_refused().
__device__ __forceinline__ uint32_t flow_pseudo(const uint32_t* pseudo, uint32_t f, uint32_t nf, bool& bad) {
    bad = f >= nf;
    return bad ? 0u : pseudo[f];
}
constexpr uint32_t kErrRange = 1u << 2;  // 1 << PIPCK_ERANGE (include/pipck.h)
__device__ __forceinline__ void flow_refused(uint32_t* err) {
    if (err) atomicOr(err, kErrRange);
}

// Arena loads are issued in the global address space explicitly.  A pointer
// rebuilt from an integer (the ragged kernel's LDS segment bases) is otherwise
// generic, and a FLAT load counts against LGKM_CNT as well as VM_CNT: every
// later s_waitcnt lgkmcnt(0) for an LDS read would then also wait for the
// outstanding HBM loads, serialising the rows in flight.
typedef __attribute__((address_space(1))) const u32x4 global_u32x4;
__device__ __forceinline__ const global_u32x4* as_global(const u32x4* p) { return (const global_u32x4*)p; }
// Non-temporal 16-byte load: the arena is streamed exactly once.
__device__ __forceinline__ u32x4 load_stream(const u32x4* p) { return __builtin_nontemporal_load(as_global(p)); }
__device__ __forceinline__ u32x4 load_plain(const u32x4* p) { return *as_global(p); }

// Range-checked 16-byte loads through a raw buffer resource (base, bytes): a
// lane whose offset reaches `bytes` gets zeros and sends NO memory request.
// The streaming kernels keep every row load unconditional (so each row waits
// for itself alone, vmcnt(U-1)); past a task's end those loads used to be
// clamped onto its last chunk, and with ~7 MB in flight per XCD against a 4 MB
// L2 that line was often gone again, so each clamped load could fetch 128 B
// once more.  Range checking covers the VGPR offset only (not soffset), so
// the row is part of the per-lane offset.
typedef __amdgpu_buffer_rsrc_t buf_t;
__device__ __forceinline__ buf_t buf_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
template <bool NT>
__device__ __forceinline__ u32x4 buf_load(buf_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, NT ? 2 : 0);  // aux bit 1 = nt (gfx94x/950)
}

// Result stores (2 B per packet, 1 B for RX verify) with the system-coherent
// policy (sc1): written through rather than left dirty in L2.  Plain stores of
// the results cost the flat kernel 2.7-4.5 % of cfg2's time -- dirty result
// lines evicted in the middle of the read stream -- and sc1 stores of the
// same results cost nothing measurable (tools/probe/write_probe.hip,
// profiles/r03_write_probe.jsonl).  Range-checked like the loads.
constexpr int kStoreSc1 = 16;  // gfx940+ cache-policy bit SC1
__device__ __forceinline__ void store_result16(buf_t r, uint32_t byte_off, uint32_t v) {
    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)v, r, (int)byte_off, 0, kStoreSc1);
}
__device__ __forceinline__ void store_result8(buf_t r, uint32_t byte_off, uint32_t v) {
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, r, (int)byte_off, 0, kStoreSc1);
}

// ---- wave-level helpers (wave64) shared by the streaming kernels
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// Inclusive wave-64 prefix sum on the DPP crossbar (GFX9 DPP: row_shr inside
// 16-lane rows, then row_bcast:15 / row_bcast:31 across rows) -- no LDS trips.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

// Wave total as a scalar: the DPP scan's last lane (six VALU steps and one
// v_readlane; a __shfl_xor butterfly would be six ds_bpermute round trips).
__device__ __forceinline__ uint32_t wave_total(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(v), 63);
}

// Lane 0's value of a 64-bit quantity, as a scalar (both halves zero-extended).
__device__ __forceinline__ uint64_t first_lane_u64(uint64_t x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// Inclusive wave-64 max-scan (same DPP pattern as wave_incl_scan).
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));  // row_shr:1
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));  // row_shr:2
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));  // row_shr:4
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));  // row_shr:8
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return v;
}

}  // namespace pipck
