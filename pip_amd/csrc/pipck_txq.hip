// pipck_txq.hip -- deferred TX checksum queue.
//
// pip computes every TX checksum synchronously inside packet construction
// (pip/protocol/pip_tcp_packet.cpp:124-134, pip/protocol/pip_udp.cpp:50-51,
// 60-61, pip/pip_netif.cpp:97).  The queue collects those packets instead:
// segment bytes go into one pinned staging arena (16-byte aligned per
// segment), each packet's pseudo-header inputs into a record, and the address
// of its checksum field into a list.  A flush moves the batch to HBM with one
// H2D copy, runs the chain kernels (pipck_checksum_chains for TCP/UDP,
// pipck_checksum_ragged for IPv4 headers) plus a per-packet pseudo-header
// kernel, copies the u16 results back and stores htons(result) -- big-endian
// on the wire, as pip's callers do -- into each field.
#include "pipck_common.hpp"
#include "pipck_device.hpp"

#include <cstring>
#include <vector>

namespace pipck {

struct TxPseudo {  // one per TCP/UDP packet
    uint8_t family;  // 4 or 6
    uint8_t proto;
    uint8_t pad[2];
    uint8_t src[16];
    uint8_t dst[16];
};
static_assert(sizeof(TxPseudo) == 36, "TxPseudo layout");

__global__ void k_tx_pseudo(const TxPseudo* __restrict__ rec, uint32_t n, uint32_t* __restrict__ pseudo) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const TxPseudo r = rec[i];
    const int words = r.family == 6 ? 4 : 1;
    uint32_t s = r.proto;
    for (int k = 0; k < words; k++) {  // ntohl of each address word, hi + lo (pip_checksum.cpp:130-136, 161-170)
        const uint32_t a = (uint32_t)r.src[4 * k] << 24 | (uint32_t)r.src[4 * k + 1] << 16 |
                           (uint32_t)r.src[4 * k + 2] << 8 | r.src[4 * k + 3];
        const uint32_t b = (uint32_t)r.dst[4 * k] << 24 | (uint32_t)r.dst[4 * k + 1] << 16 |
                           (uint32_t)r.dst[4 * k + 2] << 8 | r.dst[4 * k + 3];
        s += (a >> 16) + (a & 0xFFFFu) + (b >> 16) + (b & 0xFFFFu);
    }
    pseudo[i] = s;
}

// A growable pinned host buffer.
struct PinnedBuf {
    uint8_t* p = nullptr;
    size_t size = 0, cap = 0;
    int reserve(size_t need) {
        if (need <= cap) return PIPCK_OK;
        size_t nc = cap ? cap : (1u << 20);
        while (nc < need) nc *= 2;
        uint8_t* np = nullptr;
        PIPCK_HIP(hipHostMalloc((void**)&np, nc, hipHostMallocDefault));
        if (size) std::memcpy(np, p, size);
        if (p) (void)hipHostFree(p);
        p = np;
        cap = nc;
        return PIPCK_OK;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        size = cap = 0;
    }
};

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    int reserve(size_t need) {
        if (need <= cap) return PIPCK_OK;
        if (p) PIPCK_HIP(hipFree(p));
        p = nullptr;
        cap = 0;
        const size_t nc = need + need / 2 + 256;
        PIPCK_HIP(hipMalloc(&p, nc));
        cap = nc;
        return PIPCK_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

}  // namespace pipck

using namespace pipck;

struct pipck_txq {
    pipck_ctx* ctx = nullptr;
    hipStream_t stream = nullptr;
    int device = 0;
    PinnedBuf bytes;                       // segment bytes, each segment 16-byte aligned
    std::vector<pipck_desc> inet_segs;     // offsets into `bytes`
    std::vector<uint64_t> inet_begin{0};   // CSR: packet p owns inet_segs[begin[p], begin[p+1])
    std::vector<TxPseudo> inet_pseudo;
    std::vector<uint8_t*> inet_field;
    std::vector<pipck_desc> ip_hdrs;
    std::vector<uint8_t*> ip_field;
    PinnedBuf meta;     // staging for descriptors/records and results
    DevBuf d_all;       // device copy of bytes + meta
    DevBuf d_work;      // pseudo bases, scratch, results
};

namespace {

int append_bytes(pipck_txq* q, const void* src, uint32_t len, uint64_t* off) {
    const size_t at = (q->bytes.size + 15) & ~(size_t)15;
    int rc = q->bytes.reserve(at + len);
    if (rc) return rc;
    if (at > q->bytes.size) std::memset(q->bytes.p + q->bytes.size, 0, at - q->bytes.size);
    if (len) std::memcpy(q->bytes.p + at, src, len);
    q->bytes.size = at + len;
    *off = at;
    return PIPCK_OK;
}

int add_inet(pipck_txq* q, const pipck_hseg* segs, uint32_t nseg, const TxPseudo& ps, void* field) {
    if (!q || !field || (nseg && !segs)) {
        set_error("pipck_txq_add: null argument");
        return PIPCK_EINVAL;
    }
    for (uint32_t i = 0; i < nseg; i++) {
        if (segs[i].len > PIPCK_MAX_SEG_LEN || (segs[i].len && !segs[i].ptr)) {
            set_error("pipck_txq_add: segment null or longer than 65535 bytes");
            return PIPCK_ERANGE;
        }
    }
    for (uint32_t i = 0; i < nseg; i++) {
        uint64_t off = 0;
        int rc = append_bytes(q, segs[i].ptr, segs[i].len, &off);
        if (rc) return rc;
        q->inet_segs.push_back(pipck_desc{off, segs[i].len, 0});
    }
    q->inet_begin.push_back(q->inet_segs.size());
    q->inet_pseudo.push_back(ps);
    q->inet_field.push_back((uint8_t*)field);
    return PIPCK_OK;
}

}  // namespace

extern "C" {

int pipck_txq_create(pipck_ctx* ctx, pipck_txq** out) {
    if (!out) return PIPCK_EINVAL;
    *out = nullptr;
    int dev = 0;
    PIPCK_HIP(hipGetDevice(&dev));
    pipck_txq* q = new pipck_txq();
    q->ctx = ctx;
    q->device = dev;
    PIPCK_HIP(hipStreamCreateWithFlags(&q->stream, hipStreamNonBlocking));
    *out = q;
    return PIPCK_OK;
}

int pipck_txq_destroy(pipck_txq* q) {
    if (!q) return PIPCK_OK;
    if (q->stream) {
        (void)hipStreamSynchronize(q->stream);
        (void)hipStreamDestroy(q->stream);
    }
    q->bytes.release();
    q->meta.release();
    q->d_all.release();
    q->d_work.release();
    delete q;
    return PIPCK_OK;
}

int pipck_txq_add4(pipck_txq* q, const pipck_hseg* segs, uint32_t nseg, uint8_t proto, uint32_t src, uint32_t dst,
                   void* csum_field) {
    TxPseudo ps{};
    ps.family = 4;
    ps.proto = proto;
    std::memcpy(ps.src, &src, 4);
    std::memcpy(ps.dst, &dst, 4);
    return add_inet(q, segs, nseg, ps, csum_field);
}

int pipck_txq_add6(pipck_txq* q, const pipck_hseg* segs, uint32_t nseg, uint8_t proto, const uint8_t* src,
                   const uint8_t* dst, void* csum_field) {
    if (!src || !dst) {
        set_error("pipck_txq_add6: null address");
        return PIPCK_EINVAL;
    }
    TxPseudo ps{};
    ps.family = 6;
    ps.proto = proto;
    std::memcpy(ps.src, src, 16);
    std::memcpy(ps.dst, dst, 16);
    return add_inet(q, segs, nseg, ps, csum_field);
}

int pipck_txq_add_ip(pipck_txq* q, const void* hdr, uint32_t len, void* csum_field) {
    if (!q || !csum_field || (len && !hdr)) {
        set_error("pipck_txq_add_ip: null argument");
        return PIPCK_EINVAL;
    }
    if (len > PIPCK_MAX_SEG_LEN) {
        set_error("pipck_txq_add_ip: header longer than 65535 bytes");
        return PIPCK_ERANGE;
    }
    uint64_t off = 0;
    int rc = append_bytes(q, hdr, len, &off);
    if (rc) return rc;
    q->ip_hdrs.push_back(pipck_desc{off, len, 0});
    q->ip_field.push_back((uint8_t*)csum_field);
    return PIPCK_OK;
}

uint64_t pipck_txq_pending(const pipck_txq* q) { return q ? q->inet_field.size() + q->ip_field.size() : 0; }

int pipck_txq_flush(pipck_txq* q) {
    if (!q) return PIPCK_EINVAL;
    const uint64_t n_in = q->inet_field.size(), n_ip = q->ip_field.size(), n_seg = q->inet_segs.size();
    if (n_in + n_ip == 0) return PIPCK_OK;
    int prev = 0;
    PIPCK_HIP(hipGetDevice(&prev));
    if (prev != q->device) PIPCK_HIP(hipSetDevice(q->device));
    // meta layout (each part 16-byte aligned): inet segs | inet begin | pseudo recs | flow ids | ip descs | results
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    const size_t o_segs = 0, o_begin = al(o_segs + n_seg * sizeof(pipck_desc));
    const size_t o_rec = al(o_begin + (n_in + 1) * sizeof(uint64_t));
    const size_t o_flow = al(o_rec + n_in * sizeof(TxPseudo));
    const size_t o_ip = al(o_flow + n_in * sizeof(uint32_t));
    const size_t o_res = al(o_ip + n_ip * sizeof(pipck_desc));
    const size_t meta_in = o_res, meta_all = al(o_res + (n_in + n_ip) * sizeof(uint16_t));
    int rc = q->meta.reserve(meta_all);
    if (rc) return rc;
    uint8_t* m = q->meta.p;
    if (n_seg) std::memcpy(m + o_segs, q->inet_segs.data(), n_seg * sizeof(pipck_desc));
    std::memcpy(m + o_begin, q->inet_begin.data(), (n_in + 1) * sizeof(uint64_t));
    if (n_in) std::memcpy(m + o_rec, q->inet_pseudo.data(), n_in * sizeof(TxPseudo));
    uint32_t* flow = reinterpret_cast<uint32_t*>(m + o_flow);
    for (uint64_t i = 0; i < n_in; i++) flow[i] = (uint32_t)i;  // packet i uses pseudo base i
    if (n_ip) std::memcpy(m + o_ip, q->ip_hdrs.data(), n_ip * sizeof(pipck_desc));

    const size_t nb = al(q->bytes.size);
    if ((rc = q->d_all.reserve(nb + meta_all))) return rc;
    if ((rc = q->d_work.reserve(al(n_in * 4) + al(std::max<uint64_t>(n_seg, 1) * 4) + 16))) return rc;
    uint8_t* d_bytes = (uint8_t*)q->d_all.p;
    uint8_t* d_meta = d_bytes + nb;
    uint32_t* d_pseudo = (uint32_t*)q->d_work.p;
    uint32_t* d_scratch = (uint32_t*)((uint8_t*)q->d_work.p + al(n_in * 4));
    hipStream_t s = q->stream;
    if (q->bytes.size) PIPCK_HIP(hipMemcpyAsync(d_bytes, q->bytes.p, q->bytes.size, hipMemcpyHostToDevice, s));
    PIPCK_HIP(hipMemcpyAsync(d_meta, m, meta_in, hipMemcpyHostToDevice, s));
    uint16_t* d_res = (uint16_t*)(d_meta + o_res);
    if (n_in) {
        hipLaunchKernelGGL(k_tx_pseudo, dim3((uint32_t)((n_in + 255) / 256)), dim3(256), 0, s,
                           (const TxPseudo*)(d_meta + o_rec), (uint32_t)n_in, d_pseudo);
        PIPCK_LAUNCHED("k_tx_pseudo");
        rc = pipck_checksum_chains(d_bytes, (const pipck_desc*)(d_meta + o_segs), n_seg,
                                   (const uint64_t*)(d_meta + o_begin), (const uint32_t*)(d_meta + o_flow), n_in,
                                   d_pseudo, d_scratch, d_res, nullptr, s);
        if (rc) return rc;
    }
    if (n_ip) {
        rc = pipck_checksum_ragged(d_bytes, (const pipck_desc*)(d_meta + o_ip), n_ip, nullptr, d_res + n_in, nullptr, s);
        if (rc) return rc;
    }
    PIPCK_HIP(hipMemcpyAsync(m + o_res, d_res, (n_in + n_ip) * sizeof(uint16_t), hipMemcpyDeviceToHost, s));
    PIPCK_HIP(hipStreamSynchronize(s));
    const uint16_t* res = reinterpret_cast<const uint16_t*>(m + o_res);
    for (uint64_t i = 0; i < n_in + n_ip; i++) {  // htons(result) into the field (pip_tcp_packet.cpp:132-133)
        uint8_t* f = i < n_in ? q->inet_field[i] : q->ip_field[i - n_in];
        f[0] = (uint8_t)(res[i] >> 8);
        f[1] = (uint8_t)res[i];
    }
    q->bytes.size = 0;
    q->inet_segs.clear();
    q->inet_begin.assign(1, 0);
    q->inet_pseudo.clear();
    q->inet_field.clear();
    q->ip_hdrs.clear();
    q->ip_field.clear();
    if (prev != q->device) PIPCK_HIP(hipSetDevice(prev));
    return PIPCK_OK;
}

}  // extern "C"
