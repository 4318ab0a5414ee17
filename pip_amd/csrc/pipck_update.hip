// pipck_update.hip -- incremental checksum update for header rewrites
// (RFC 1624).
//
// pip never rewrites a header in place: a resend re-sums the unchanged chain
// (pip/protocol/pip_tcp_private.cpp:168-178) and every field change means a
// full pass of pip_standard_checksum (pip/pip_checksum.cpp:13-33).  For a batch
// already carrying pip's checksums, a rewrite of a few bytes (sequence / ack
// numbers, ports, or the addresses behind the pseudo-header) only needs the
// old and new words:
//     HC' = ~(~HC + ~m + m')                           (RFC 1624, eqn. 3)
// Parity with pip's recomputation.  pip stores ~fold2(S) with fold2(S) in
// [0, 0xFFFF], 0 only for S == 0 (no u32 wrap below 65535 bytes).  So
//   * HC == 0xFFFF  <=>  S_old == 0: every covered byte and the pseudo-header
//     were zero, hence S_new is exactly the new words + the new pseudo base;
//   * otherwise ~HC >= 1, the one's-complement sum R of eqn. 3 is in
//     [1, 0xFFFF] with R == S_new (mod 0xFFFF): if R != 0xFFFF then
//     S_new != 0 and fold2(S_new) == R; if R == 0xFFFF pip gives 0x0000 for a
//     nonzero S_new and 0xFFFF for S_new == 0, which only a look at the whole
//     packet decides -- done here for that packet alone (rare).
#include "pipck_common.hpp"
#include "pipck_device.hpp"

namespace pipck {

// Big-endian word sum of bytes [0, n) of p, pairing from p[0]; an odd last
// byte is the high byte of a zero-padded word (pip_checksum.cpp:17-27).
__device__ __forceinline__ uint32_t be_words(const uint8_t* p, uint32_t n) {
    uint32_t s = 0;
    uint32_t i = 0;
    for (; i + 1 < n; i += 2) s += ((uint32_t)p[i] << 8) | p[i + 1];
    if (i < n) s += (uint32_t)p[i] << 8;
    return s;
}

__device__ __forceinline__ uint32_t ones_neg(uint32_t x) { return 0xFFFFu - fold16(x); }

__global__ __launch_bounds__(256) void k_update_fixed(uint8_t* __restrict__ arena, uint64_t stride, uint64_t n,
                                                      uint32_t cover_off, uint32_t cover_len, uint32_t ck_off,
                                                      uint32_t edit_off, uint32_t edit_len,
                                                      const uint8_t* __restrict__ nb, uint64_t new_stride,
                                                      const uint32_t* __restrict__ pseudo_old,
                                                      const uint32_t* __restrict__ pseudo_new, uint32_t n_flows,
                                                      const uint32_t* __restrict__ flow_of, uint64_t flow_origin,
                                                      uint32_t* __restrict__ err) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t* a = arena + i * stride;
    const uint8_t* e = nb + i * new_stride;
    uint32_t po = 0, pn = 0;
    if (pseudo_old) {
        const uint32_t f = flow_of ? flow_of[i] : (uint32_t)((flow_origin + i) % n_flows);
        // with flow_of, n_flows bounds the entry (pipck_update_fixed_n; UINT32_MAX:
        // trusted).  A stale entry must not turn into a checksum computed from
        // bytes outside the tables and written into the packet: the packet is
        // left exactly as it was -- edit bytes and checksum field -- and the
        // call reports PIPCK_ERANGE.
        if (flow_of && f >= n_flows) {
            flow_refused(err);
            return;
        }
        po = pseudo_old[f];
        pn = pseudo_new[f];
    }
    const uint32_t hc = ((uint32_t)a[ck_off] << 8) | a[ck_off + 1];
    const uint32_t m_old = be_words(a + edit_off, edit_len);
    const uint32_t m_new = be_words(e, edit_len);
    for (uint32_t k = 0; k < edit_len; k++) a[edit_off + k] = e[k];
    uint32_t r;
    if (hc == 0xFFFFu) {
        r = fold16(m_new + pn);  // S_old == 0: the rest of the packet is zero
    } else {
        r = fold16((hc ^ 0xFFFFu) + ones_neg(m_old) + fold16(m_new) + ones_neg(po) + fold16(pn));
        if (r == 0xFFFFu) {
            // S_new == 0 only with a zero pseudo-header, no length term and
            // zero bytes everywhere but the checksum field
            bool zero = pseudo_old ? (pn == 0 && cover_len == 0) : true;
            for (uint32_t k = 0; zero && k < cover_len; k++) {
                const uint32_t o = cover_off + k;
                if (o != ck_off && o != ck_off + 1 && a[o] != 0) zero = false;
            }
            if (zero) r = 0;
        }
    }
    const uint32_t ck = ~r & 0xFFFFu;
    a[ck_off] = (uint8_t)(ck >> 8);
    a[ck_off + 1] = (uint8_t)ck;
}

}  // namespace pipck

using namespace pipck;

static int update_fixed(void* d_arena, uint64_t stride, uint64_t n, uint32_t cover_off, uint32_t cover_len,
                        uint32_t ck_off, uint32_t edit_off, uint32_t edit_len, const void* d_new, uint64_t new_stride,
                        const uint32_t* d_pseudo_old, const uint32_t* d_pseudo_new, uint32_t n_flows,
                        const uint32_t* d_flow_of, uint64_t flow_origin, uint32_t* d_err, void* stream, bool bounded) {
    if (n == 0) return PIPCK_OK;
    const uint64_t cover_end = (uint64_t)cover_off + cover_len, edit_end = (uint64_t)edit_off + edit_len;
    const char* why = nullptr;
    if (!d_arena || (edit_len && !d_new)) why = "null arena/new bytes";
    else if ((d_pseudo_old == nullptr) != (d_pseudo_new == nullptr)) why = "pseudo_old and pseudo_new must both be set or both NULL";
    else if (d_pseudo_old && n_flows == 0 && (bounded || !d_flow_of)) why = "n_flows == 0";
    else if (cover_len > PIPCK_MAX_SEG_LEN) why = "cover_len > 65535 is outside the batch domain";
    else if (ck_off < cover_off || (uint64_t)ck_off + 2 > cover_end || ((ck_off - cover_off) & 1))
        why = "checksum field must be an even-offset word inside the cover";
    else if (edit_len && (edit_off < cover_off || edit_end > cover_end || ((edit_off - cover_off) & 1)))
        why = "edit must start at an even offset inside the cover";
    else if ((edit_len & 1) && edit_end != cover_end) why = "odd edit_len is only allowed at the end of the cover";
    else if (edit_len && edit_off < (uint64_t)ck_off + 2 && edit_end > ck_off) why = "edit overlaps the checksum field";
    else if (cover_end > stride) why = "cover exceeds the stride";
    if (why) {
        set_error(std::string("pipck_update_fixed: ") + why);
        return PIPCK_EINVAL;
    }
    if ((n + 255) / 256 > 0x7FFFFFFFull) {
        set_error("pipck_update_fixed: too many packets for one launch");
        return PIPCK_ERANGE;
    }
    // the kernel's n_flows: the modulus without flow_of; with it, the bound of its entries
    const uint32_t nf = d_flow_of ? (bounded ? n_flows : UINT32_MAX) : n_flows;
    hipLaunchKernelGGL(k_update_fixed, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, as_stream(stream),
                       (uint8_t*)d_arena, stride, n, cover_off, cover_len, ck_off, edit_off, edit_len,
                       (const uint8_t*)d_new, new_stride, d_pseudo_old, d_pseudo_new, nf, d_flow_of,
                       flow_origin, d_err);
    PIPCK_LAUNCHED("k_update_fixed");
    return PIPCK_OK;
}

extern "C" int pipck_update_fixed_n(void* d_arena, uint64_t stride, uint64_t n, uint32_t cover_off,
                                    uint32_t cover_len, uint32_t ck_off, uint32_t edit_off, uint32_t edit_len,
                                    const void* d_new, uint64_t new_stride, const uint32_t* d_pseudo_old,
                                    const uint32_t* d_pseudo_new, uint32_t n_flows, const uint32_t* d_flow_of,
                                    uint64_t flow_origin, uint32_t* d_err, void* stream) {
    return update_fixed(d_arena, stride, n, cover_off, cover_len, ck_off, edit_off, edit_len, d_new, new_stride,
                        d_pseudo_old, d_pseudo_new, n_flows, d_flow_of, flow_origin, d_err, stream, true);
}

// the unbounded form (flow_of entries trusted, n_flows unused with them)
extern "C" int pipck_update_fixed(void* d_arena, uint64_t stride, uint64_t n, uint32_t cover_off, uint32_t cover_len,
                                  uint32_t ck_off, uint32_t edit_off, uint32_t edit_len, const void* d_new,
                                  uint64_t new_stride, const uint32_t* d_pseudo_old, const uint32_t* d_pseudo_new,
                                  uint32_t n_flows, const uint32_t* d_flow_of, uint64_t flow_origin, void* stream) {
    return update_fixed(d_arena, stride, n, cover_off, cover_len, ck_off, edit_off, edit_len, d_new, new_stride,
                        d_pseudo_old, d_pseudo_new, n_flows, d_flow_of, flow_origin, nullptr, stream, false);
}
