// pipck_hdr.hip -- row-stream kernel for packed 20/24-byte items: IPv4 headers.
//
// Hot path: plumk97/pip pip/pip_checksum.cpp:35-39 (pip_ip_checksum) over a
// batch of 20-byte IPv4 headers (pip/pip_netif.cpp:94-97 calls it per packet)
// laid back to back at a 20-byte stride (cfg1) -- or 24 -- with no
// pseudo-header.  k_small gives each lane whole headers: every load instruction
// then covers 64 headers at a 20-byte stride (a 1,280-byte span read as 32
// bytes per lane, 1.6x the bytes through the cache), and one task is only 128
// headers.  Here a wave streams its task as coalesced rows of whole headers
// exactly like the large-packet kernels stream theirs:
//
//   * a row is C = 60 chunks (D = 5 dwords per header: 48 headers in 960 B) or
//     C = 63 (D = 6: 42 headers in 1,008 B); lane l < C loads chunk l of the
//     row (one coalesced buffer load), lanes >= C load nothing;
//   * since D >= 5 > 4, a 16-byte chunk holds the end of at most one header
//     that began in the lane before and the start of at most one new header,
//     and every header ends in the lane after the one it starts in.  The
//     header geometry repeats identically in every row, so each lane computes
//     once which of its dwords belong to a header started before it (H) and
//     which to the header starting in it (T), as byte masks that also drop a
//     header's bytes past `len`;
//   * per row: H = dot4(x & mH), T = dot4(x & mT), one DPP wave shift hands
//     T to the next lane, and the lane holding a header's last dword finishes
//     it: bswap16(fold(T_prev + H)) (headers start 4-byte aligned: even);
//   * results wait in LDS and the wave stores its task's results at the end
//     (a global store between the ring's loads would make each row's wait
//     drain the queue: stores count in VM_CNT on gfx9).
#include "pipck_common.hpp"
#include "pipck_device.hpp"

#include <algorithm>

namespace pipck {

// tune flags (same results): bit 29 = k_hdr's result stores plain write-back,
// bit 30 = non-temporal (default: write-through, sc1); bit 31 = one store per
// result instead of 16-byte pieces
constexpr uint32_t kHdrPlainStores = 1u << 29;
constexpr uint32_t kHdrNtStores = 1u << 30;
constexpr uint32_t kHdrNarrowStores = 1u << 31;
// measurement only (pipck_tune_probes, not a tune flag --
// the flags' settings all compute the same results): store each header's checksum
// INTO the header -- htons(result) at byte 10, its ip_sum, as pip_netif.cpp:97
// stores it -- instead of into the result array (which is left untouched): the
// "results inside the headers" layout, to weigh its write-back of whole dirty
// lines against the separate 2-byte result stream.
constexpr uint32_t kHdrInPlace = 1u << 28;  // the kernel's own flag word only (launch_hdr sets it)

template <int D>
struct HdrGeom {
    static constexpr uint32_t C = D == 5 ? 60u : 63u;  // chunks per row
    static constexpr uint32_t PR = C * 4u / D;          // headers per row
};

// lane l's dword masks for the header(s) its chunk touches: mH = bytes of a
// header begun in an earlier lane, mT = bytes of the header beginning in this
// lane; fin = row-local index of the header whose last dword this lane holds
// (or -1)
template <int D>
__device__ __forceinline__ void hdr_lane(int lane, uint32_t len, u32x4& mH, u32x4& mT, int& fin) {
    uint32_t h[4], t[4];
    int start = 4;
    fin = -1;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t d = 4u * lane + i, q = d % D;
        if (q == 0 && start == 4) start = i;
        if (q == D - 1) fin = (int)(d / D);
        const int vb = (int)len - 4 * (int)q;  // valid bytes of this dword
        const uint32_t m = vb >= 4 ? 0xFFFFFFFFu : (vb <= 0 ? 0u : (0xFFFFFFFFu >> (32 - 8 * vb)));
        h[i] = i < start ? m : 0u;
        t[i] = i < start ? 0u : m;
    }
    if ((uint32_t)lane >= HdrGeom<D>::C) {  // no chunk
#pragma unroll
        for (int i = 0; i < 4; i++) h[i] = t[i] = 0u;
        fin = -1;
    }
    mH = u32x4{h[0], h[1], h[2], h[3]};
    mT = u32x4{t[0], t[1], t[2], t[3]};
}

// COOP (round 4): the block's four waves share ONE task of 4 x rows rows and
// read interleaved rows (wave w: rows w, w+4, ...), so the block streams one
// contiguous window, as k_flat_coop does for large packets; rows carry no
// state across rows here (48 whole headers each), so nothing else changes but
// the row order, and the block stores its results together at the end.
template <int D, int U, bool VERIFY, bool NT, bool COOP = false>
__global__ __launch_bounds__(256) void k_hdr(const uint8_t* __restrict__ arena, uint32_t len, uint64_t n,
                                             uint32_t rows, uint16_t* __restrict__ out, uint8_t* __restrict__ ok,
                                             uint32_t kflags) {
    constexpr uint32_t C = HdrGeom<D>::C, PR = HdrGeom<D>::PR;
    extern __shared__ uint16_t s_res[];  // 4 waves x rows * PR results
    const int lane = threadIdx.x & 63;
    const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint64_t task = COOP ? (uint64_t)blockIdx.x : (uint64_t)blockIdx.x * 4 + w;
    const uint64_t per = (uint64_t)rows * PR * (COOP ? 4u : 1u);  // headers per task
    const uint64_t p0 = task * per;
    if (p0 >= n) return;  // wave-uniform (block-uniform for COOP)
    const uint32_t np = (uint32_t)min<uint64_t>(per, n - p0);
    const uint32_t nrows = (np + PR - 1) / PR;
    uint16_t* res = COOP ? s_res : s_res + w * rows * PR;
    // the task's bytes as a range-checked buffer, to the 16-byte boundary after its last header
    const uint64_t b0 = p0 * (4u * D);
    const buf_t tb = buf_rsrc(arena + b0, (uint32_t)(((uint64_t)np * (4u * D) + 15u) & ~15ull));
    u32x4 mH, mT;
    int fin;
    hdr_lane<D>(lane, len, mH, mT, fin);
    const uint32_t loff = (uint32_t)lane < C ? 16u * lane : 0x7FFFFFF0u;  // lanes >= C: out of range, no request
    // this wave's j-th row: j (one task per wave) or w + 4j (COOP)
    const uint32_t rstep = COOP ? 4u : 1u, rbase = COOP ? w : 0u;
    const uint32_t my_rows = COOP ? (nrows > w ? (nrows - w + 3u) / 4u : 0u) : nrows;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++)
        v[u] = buf_load<NT>(tb, (uint32_t)lane < C ? 16u * C * (rbase + rstep * u) + loff : loff);
    for (uint32_t j0 = 0; j0 < my_rows; j0 += U) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t j = j0 + u;
            const uint32_t r = rbase + rstep * j;
            if (j < my_rows) {  // wave-uniform
                const u32x4 x = v[u];
                const uint32_t H = dot4(x & mH, 0u), T = dot4(x & mT, 0u);
                // T of the lane before (wave_shr:1; lane 0 gets 0 and finishes nothing)
                const uint32_t Tp = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)T, 0x138, 0xf, 0xf, false);
                const uint32_t hi = r * PR + (uint32_t)fin;
                if (fin >= 0 && hi < np) {
                    const uint32_t F = bswap16(fold16(Tp + H));
                    res[hi] = VERIFY ? (uint16_t)(fold16(F) == 0xFFFFu) : (uint16_t)(~F & 0xFFFFu);
                }
            }
            // the row U ahead (unconditional: past the task it reads zeros, no request)
            v[u] = buf_load<NT>(tb, (uint32_t)lane < C ? 16u * C * (r + rstep * U) + loff : loff);
        }
    }
    if (COOP)
        __syncthreads();  // every wave's rows in res before the block stores them
    else
        wave_sync();
    if (!VERIFY && (kflags & kHdrInPlace)) {  // measurement: results into the headers' ip_sum
        const buf_t hb = buf_rsrc(arena + b0, (uint32_t)((uint64_t)np * (4u * D)));
        for (uint32_t i = COOP ? threadIdx.x : (uint32_t)lane; i < np; i += COOP ? 256u : 64u) {
            const uint32_t r = res[i];
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)((r >> 8) | (r << 8)), hb, (int)(i * 4u * D + 10u), 0, 0);
        }
        return;
    }
    // the task's results, contiguous from out + p0 (ok + p0): whole 16-byte
    // pieces as one b128 store per lane (a full task of 3,072 headers is 6 KiB
    // = 6 store instructions), the rest one result per lane
    const uint32_t policy = (kflags & kHdrPlainStores) ? 0 : ((kflags & kHdrNtStores) ? 2 : kStoreSc1);
    const uint32_t rbytes = VERIFY ? np : 2u * np;
    const buf_t rb = VERIFY ? buf_rsrc(ok + p0, np) : buf_rsrc(out + p0, 2u * np);
    uint32_t done = 0;
    // (16-byte pieces only where the caller's result array is 16-byte aligned there)
    if (!(kflags & kHdrNarrowStores) &&
        (VERIFY ? (uintptr_t)(ok + p0) : (uintptr_t)(out + p0)) % 16 == 0) {
        done = rbytes & ~15u;
        const uint32_t per_piece = VERIFY ? 16u : 8u;  // results per 16 bytes
        const uint32_t me = COOP ? threadIdx.x : (uint32_t)lane, nthr = COOP ? 256u : 64u;
        for (uint32_t o = 16u * me; o < done; o += 16u * nthr) {
            const uint16_t* r = res + (o / 16u) * per_piece;
            u32x4 x;
            if (VERIFY) {  // 16 one-byte flags
                uint32_t wv[4];
#pragma unroll
                for (int k = 0; k < 4; k++)
                    wv[k] = (uint32_t)r[4 * k] | ((uint32_t)r[4 * k + 1] << 8) | ((uint32_t)r[4 * k + 2] << 16) |
                            ((uint32_t)r[4 * k + 3] << 24);
                x = u32x4{wv[0], wv[1], wv[2], wv[3]};
            } else {
                x = *reinterpret_cast<const u32x4*>(r);  // 8 results, 16-byte aligned in LDS
            }
            if (policy == 0)
                __builtin_amdgcn_raw_buffer_store_b128(x, rb, (int)o, 0, 0);
            else if (policy == 2)
                __builtin_amdgcn_raw_buffer_store_b128(x, rb, (int)o, 0, 2);
            else
                __builtin_amdgcn_raw_buffer_store_b128(x, rb, (int)o, 0, kStoreSc1);
        }
        done /= VERIFY ? 1u : 2u;  // results stored
    }
    for (uint32_t i = done + (COOP ? threadIdx.x : (uint32_t)lane); i < np; i += COOP ? 256u : 64u) {
        if (VERIFY)
            store_result8(rb, i, res[i]);
        else
            store_result16(rb, 2u * i, res[i]);
    }
}

typedef void (*hdr_fn)(const uint8_t*, uint32_t, uint64_t, uint32_t, uint16_t*, uint8_t*, uint32_t);

// Launch for a 16-byte-aligned arena, stride 20 or 24, len <= stride, no
// pseudo-header.  rows: 1 KiB-ish rows per wave task (0 = auto); ring: rows in
// flight per wave (8 / 16 / 24 / 32, 0 = auto).  PIPCK_EINVAL when the shape does
// not fit (the caller then takes k_small).
int launch_hdr(bool verify, const void* d_arena, uint64_t stride, uint32_t len, uint64_t n, uint16_t* d_out,
               uint8_t* d_ok, hipStream_t s, uint32_t rows, uint32_t ring, bool nt, uint32_t kflags, bool coop) {
    if ((stride != 20 && stride != 24) || len > stride || (uintptr_t)d_arena % 16) return PIPCK_EINVAL;
    const uint32_t PR = stride == 20 ? HdrGeom<5>::PR : HdrGeom<6>::PR;
    // rows per wave task: 32 with a ring of 32 (the whole task in flight at
    // once) measured fastest at 128M-256M headers -- 0.979 ms at 256M vs
    // 0.99-1.08 for 24-48 rows or a ring of 24, and k_small's 1.089 -- and
    // shorter tasks were slower at every size down to 1M headers
    // (profiles/r03_hdr_scan.jsonl)
    const uint32_t R = rows ? std::min<uint32_t>(rows, 128u) : 32u;  // LDS: 4 x R x PR results
    const uint64_t per = (uint64_t)R * PR;
    const uint64_t tasks = (n + per - 1) / per;
    const uint64_t blocks = (tasks + 3) / 4;
    if (blocks > 0x7FFFFFFFull || per * stride >= (1ull << 31)) return PIPCK_EINVAL;
    const size_t lds = 4u * per * sizeof(uint16_t);
    const uint32_t u = ring ? ring : 32u;
    // bit 28 of the tune flags is the other fixed-stride schedule elsewhere (same
    // results); here it carries the in-place probe only when that probe is on
    kflags = (kflags & ~kHdrInPlace) | ((g_probes.load() & kProbeHdrInPlace) ? kHdrInPlace : 0u);
    const int ui = u >= 32 ? 3 : (u >= 24 ? 2 : (u >= 16 ? 1 : 0));
#define PIPCK_HD(D, U, CO) {{k_hdr<D, U, false, false, CO>, k_hdr<D, U, false, true, CO>}, \
                           {k_hdr<D, U, true, false, CO>, k_hdr<D, U, true, true, CO>}}
    static const hdr_fn kHdr[2][2][4][2][2] = {  // [coop][D][ring][verify][nt]
        {{PIPCK_HD(5, 8, false), PIPCK_HD(5, 16, false), PIPCK_HD(5, 24, false), PIPCK_HD(5, 32, false)},
         {PIPCK_HD(6, 8, false), PIPCK_HD(6, 16, false), PIPCK_HD(6, 24, false), PIPCK_HD(6, 32, false)}},
        {{PIPCK_HD(5, 8, true), PIPCK_HD(5, 16, true), PIPCK_HD(5, 24, true), PIPCK_HD(5, 32, true)},
         {PIPCK_HD(6, 8, true), PIPCK_HD(6, 16, true), PIPCK_HD(6, 24, true), PIPCK_HD(6, 32, true)}}};
#undef PIPCK_HD
    // a block covers 4 x R rows either way: four wave tasks, or one cooperative task
    PIPCK_LAUNCH(kHdr[coop][stride == 24][ui][verify][nt], dim3((uint32_t)blocks), dim3(256), lds, s,
                 (const uint8_t*)d_arena, len, n, R, d_out, d_ok, kflags);
    PIPCK_LAUNCHED("k_hdr");
    return PIPCK_OK;
}

}  // namespace pipck
