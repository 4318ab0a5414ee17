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

// A growable pinned host buffer; coherent, so small flushes can let the kernels
// read it (and write results into it) in place.
struct PinnedBuf {
    uint8_t* p = nullptr;
    size_t size = 0, cap = 0;
    int reserve(size_t need) {
        if (need <= cap) return PIPCK_OK;
        size_t nc = cap ? cap : (1u << 20);
        while (nc < need) nc *= 2;
        uint8_t* np = nullptr;
        PIPCK_HIP(hipHostMalloc((void**)&np, nc, hipHostMallocCoherent));
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

// One batch of queued packets: host staging, bookkeeping and device buffers.
// A queue holds two, so one can be filled while the other is in flight.
struct TxBatch {
    PinnedBuf bytes;                       // segment bytes, each segment 16-byte aligned
    std::vector<pipck_desc> inet_segs;     // offsets into `bytes`, or (flow == 1) a zero-copy host address
    bool has_zc = false;                   // some inet segment is read in place from pinned host memory
    std::vector<uint64_t> inet_begin{0};   // CSR: packet p owns inet_segs[begin[p], begin[p+1])
    std::vector<TxPseudo> inet_pseudo;
    std::vector<uint8_t*> inet_field;
    std::vector<pipck_desc> ip_hdrs;
    std::vector<uint8_t*> ip_field;
    std::vector<PinnedRef> held;  // pinned ranges this batch reads in place (one hold each, released at complete)
    PinnedBuf meta;     // staging for descriptors/records and results
    DevBuf d_all;       // device copy of bytes + meta
    DevBuf d_work;      // pseudo bases, scratch, results
    size_t o_res = 0;   // offset of the results in `meta` (valid while in flight)
    uint64_t pending() const { return inet_field.size() + ip_field.size(); }
    void drop_holds() {
        for (PinnedRef& r : held) pinned_release(*r);
        held.clear();
    }
    void clear() {
        drop_holds();
        bytes.size = 0;
        inet_segs.clear();
        has_zc = false;
        inet_begin.assign(1, 0);
        inet_pseudo.clear();
        inet_field.clear();
        ip_hdrs.clear();
        ip_field.clear();
    }
    void release() {
        drop_holds();
        bytes.release();
        meta.release();
        d_all.release();
        d_work.release();
    }
};

}  // namespace pipck

using namespace pipck;

// A flush whose staged bytes + metadata fit 32 MiB runs without any copy
// command: the kernels read the coherent pinned staging in place and write the
// results into it.  Measured on one producer thread (tools/txq_bench.cpp,
// profiles/r01_txq_inplace_ab.jsonl): a 64-packet flush 40 vs 50 us, 1,024
// packets 0.10 vs 0.12 ms, pipelined 16K-packet batches +15 %.  Larger batches
// keep the H2D / D2H copies.  Per queue: pipck_txq_inplace_max.
constexpr uint64_t kInPlaceFlushMax = 32u << 20;

struct pipck_txq {
    pipck_ctx* ctx = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;  // recorded after the in-flight batch's D2H copy
    int device = 0;
    TxBatch batch[2];
    bool auto_zc = false;      // plain adds read pinned segments in place (pipck_txq_auto_zero_copy)
    uint64_t inplace_max = kInPlaceFlushMax;  // pipck_txq_inplace_max
    int cur = 0;         // batch receiving adds
    bool inflight = false;  // batch[cur ^ 1] has been submitted and not completed
};

namespace {

int append_bytes(TxBatch* b, const void* src, uint32_t len, uint64_t* off) {
    const size_t at = (b->bytes.size + 15) & ~(size_t)15;
    int rc = b->bytes.reserve(at + len);
    if (rc) return rc;
    if (at > b->bytes.size) std::memset(b->bytes.p + b->bytes.size, 0, at - b->bytes.size);
    if (len) std::memcpy(b->bytes.p + at, src, len);
    b->bytes.size = at + len;
    *off = at;
    return PIPCK_OK;
}

// Can [p, p+len) be read in place by batch b?  Only inside a pinned range
// (pipck_host_alloc / pipck_host_register), and the batch then holds that
// range until it completes, so the range cannot be freed or unregistered while
// the GPU may still read it.  Segments of one batch usually come from a few
// buffers (a header ring, a payload ring): the batch's held ranges answer most
// checks without the registry.
bool hold_pinned(TxBatch* b, const void* p, uint32_t len) {
    const uintptr_t a = (uintptr_t)p;
    // the most recently held ranges only, so a batch of many small buffers stays O(1)
    // per segment (a range found in the registry again is simply held twice)
    for (size_t i = b->held.size(), k = 0; i-- > 0 && k < 4; k++) {
        const PinnedRec& r = *b->held[i];
        if (a >= r.lo && a + len <= r.hi) return true;  // held: cannot have been removed
    }
    PinnedRef r = pinned_lookup(p, len);
    if (!r || !pinned_acquire(*r)) return false;  // unpinned, or being released right now
    b->held.push_back(std::move(r));
    return true;
}

// zc: every segment is read in place (refused unless pinned); otherwise, in a
// queue with auto_zc set, pinned segments are read in place and others copied.
int add_inet(pipck_txq* q, const pipck_hseg* segs, uint32_t nseg, const TxPseudo& ps, void* field, bool zc) {
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
    TxBatch* b = &q->batch[q->cur];
    const size_t seg0 = b->inet_segs.size(), bytes0 = b->bytes.size, held0 = b->held.size();
    // a refused packet leaves the batch as it was: its segments, bytes and the
    // pinned-range holds taken for it are all dropped
    auto rollback = [&] {
        b->inet_segs.resize(seg0);
        b->bytes.size = bytes0;
        for (size_t h = held0; h < b->held.size(); h++) pinned_release(*b->held[h]);
        b->held.resize(held0);
    };
    for (uint32_t i = 0; i < nseg; i++) {
        const bool in_place = (zc || q->auto_zc) && segs[i].len && hold_pinned(b, segs[i].ptr, segs[i].len);
        if (zc && segs[i].len && !in_place) {
            // the GPU would read it in place: it must be pinned; drop this packet's segments
            rollback();
            set_error("pipck_txq_add_zc: segment outside every range from pipck_host_alloc / "
                      "pipck_host_register");
            return PIPCK_EINVAL;
        }
        if (in_place) {
            // read in place at flush time (pinned host memory, device-accessible at the same address)
            b->inet_segs.push_back(pipck_desc{(uint64_t)(uintptr_t)segs[i].ptr, segs[i].len, 1u});
            b->has_zc = true;
            continue;
        }
        uint64_t off = 0;
        int rc = append_bytes(b, segs[i].ptr, segs[i].len, &off);
        if (rc) {
            rollback();
            return rc;
        }
        b->inet_segs.push_back(pipck_desc{off, segs[i].len, 0});
    }
    b->inet_begin.push_back(b->inet_segs.size());
    b->inet_pseudo.push_back(ps);
    b->inet_field.push_back((uint8_t*)field);
    return PIPCK_OK;
}

// Enqueue batch b on the queue's stream: H2D of bytes + metadata (or nothing,
// for a small batch), the pseudo-header and chain kernels, ragged IPv4
// headers, D2H of the results (or results written in place).
int enqueue(pipck_txq* q, TxBatch* b) {
    const uint64_t n_in = b->inet_field.size(), n_ip = b->ip_field.size(), n_seg = b->inet_segs.size();
    // meta layout (each part 16-byte aligned): inet segs | inet begin | pseudo recs | flow ids | ip descs | results
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    const size_t o_segs = 0, o_begin = al(o_segs + n_seg * sizeof(pipck_desc));
    const size_t o_rec = al(o_begin + (n_in + 1) * sizeof(uint64_t));
    const size_t o_flow = al(o_rec + n_in * sizeof(TxPseudo));
    const size_t o_ip = al(o_flow + n_in * sizeof(uint32_t));
    const size_t o_res = al(o_ip + n_ip * sizeof(pipck_desc));
    const size_t meta_in = o_res, meta_all = al(o_res + (n_in + n_ip) * sizeof(uint16_t));
    int rc = b->meta.reserve(meta_all);
    if (rc) return rc;
    const size_t nb = al(b->bytes.size);
    const bool in_place = nb + meta_all <= q->inplace_max;
    uint8_t* d_bytes = nullptr;
    if (in_place) {
        if ((rc = b->bytes.reserve(16))) return rc;  // a valid base even for an empty batch
        d_bytes = b->bytes.p;
    } else {
        if ((rc = b->d_all.reserve(nb + meta_all))) return rc;
        d_bytes = (uint8_t*)b->d_all.p;
    }
    uint8_t* m = b->meta.p;
    if (b->has_zc) {  // every descriptor becomes an absolute address (arena = null below)
        pipck_desc* d = reinterpret_cast<pipck_desc*>(m + o_segs);
        for (uint64_t i = 0; i < n_seg; i++) {
            const pipck_desc& x = b->inet_segs[i];
            d[i] = pipck_desc{x.flow ? x.offset : (uint64_t)(uintptr_t)(d_bytes + x.offset), x.len, 0u};
        }
    } else if (n_seg) {
        std::memcpy(m + o_segs, b->inet_segs.data(), n_seg * sizeof(pipck_desc));
    }
    std::memcpy(m + o_begin, b->inet_begin.data(), (n_in + 1) * sizeof(uint64_t));
    if (n_in) std::memcpy(m + o_rec, b->inet_pseudo.data(), n_in * sizeof(TxPseudo));
    uint32_t* flow = reinterpret_cast<uint32_t*>(m + o_flow);
    for (uint64_t i = 0; i < n_in; i++) flow[i] = (uint32_t)i;  // packet i uses pseudo base i
    if (n_ip) std::memcpy(m + o_ip, b->ip_hdrs.data(), n_ip * sizeof(pipck_desc));

    if ((rc = b->d_work.reserve(al(n_in * 4) + al(std::max<uint64_t>(n_seg, 1) * 4) + 16))) return rc;
    uint8_t* d_meta = in_place ? m : d_bytes + nb;
    uint32_t* d_pseudo = (uint32_t*)b->d_work.p;
    uint32_t* d_scratch = (uint32_t*)((uint8_t*)b->d_work.p + al(n_in * 4));
    hipStream_t s = q->stream;
    if (!in_place) {
        if (b->bytes.size) PIPCK_HIP(hipMemcpyAsync(d_bytes, b->bytes.p, b->bytes.size, hipMemcpyHostToDevice, s));
        PIPCK_HIP(hipMemcpyAsync(d_meta, m, meta_in, hipMemcpyHostToDevice, s));
    }
    uint16_t* d_res = (uint16_t*)(d_meta + o_res);
    if (n_in) {
        hipLaunchKernelGGL(k_tx_pseudo, dim3((uint32_t)((n_in + 255) / 256)), dim3(256), 0, s,
                           (const TxPseudo*)(d_meta + o_rec), (uint32_t)n_in, d_pseudo);
        PIPCK_LAUNCHED("k_tx_pseudo");
        rc = chains_unchecked(b->has_zc ? nullptr : d_bytes, (const pipck_desc*)(d_meta + o_segs), n_seg,
                              (const uint64_t*)(d_meta + o_begin), (const uint32_t*)(d_meta + o_flow), n_in, d_pseudo,
                              d_scratch, d_res, nullptr, s);
        if (rc) return rc;
    }
    if (n_ip) {
        rc = pipck_checksum_ragged(d_bytes, (const pipck_desc*)(d_meta + o_ip), n_ip, nullptr, d_res + n_in, nullptr, s);
        if (rc) return rc;
    }
    if (!in_place)
        PIPCK_HIP(hipMemcpyAsync(m + o_res, d_res, (n_in + n_ip) * sizeof(uint16_t), hipMemcpyDeviceToHost, s));
    PIPCK_HIP(hipEventRecord(q->done, s));
    b->o_res = o_res;
    return PIPCK_OK;
}

// Wait for the in-flight batch and store htons(result) into its fields.
int complete_inflight(pipck_txq* q) {
    if (!q->inflight) return PIPCK_OK;
    TxBatch* b = &q->batch[q->cur ^ 1];
    PIPCK_HIP(hipEventSynchronize(q->done));
    const uint64_t n_in = b->inet_field.size(), n = b->pending();
    const uint16_t* res = reinterpret_cast<const uint16_t*>(b->meta.p + b->o_res);
    for (uint64_t i = 0; i < n; i++) {  // htons(result) into the field (pip_tcp_packet.cpp:132-133)
        uint8_t* f = i < n_in ? b->inet_field[i] : b->ip_field[i - n_in];
        f[0] = (uint8_t)(res[i] >> 8);
        f[1] = (uint8_t)res[i];
    }
    b->clear();
    q->inflight = false;
    return PIPCK_OK;
}

// Runs `fn` with the queue's device current, restoring the caller's.
template <class F>
int on_device(pipck_txq* q, F fn) {
    int prev = 0;
    PIPCK_HIP(hipGetDevice(&prev));
    if (prev != q->device) PIPCK_HIP(hipSetDevice(q->device));
    const int rc = fn();
    if (prev != q->device) PIPCK_HIP(hipSetDevice(prev));
    return rc;
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
    if (hipStreamCreateWithFlags(&q->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&q->done, hipEventDisableTiming) != hipSuccess) {
        set_error("pipck_txq_create: stream/event creation failed");
        if (q->stream) (void)hipStreamDestroy(q->stream);
        delete q;
        return PIPCK_EHIP;
    }
    *out = q;
    return PIPCK_OK;
}

int pipck_txq_auto_zero_copy(pipck_txq* q, int on) {
    if (!q) {
        set_error("pipck_txq_auto_zero_copy: null queue");
        return PIPCK_EINVAL;
    }
    q->auto_zc = on != 0;
    return PIPCK_OK;
}

int pipck_txq_inplace_max(pipck_txq* q, uint64_t bytes) {
    if (!q) {
        set_error("pipck_txq_inplace_max: null queue");
        return PIPCK_EINVAL;
    }
    q->inplace_max = bytes;
    return PIPCK_OK;
}

int pipck_txq_destroy(pipck_txq* q) {
    if (!q) return PIPCK_OK;
    if (q->stream) {
        (void)hipStreamSynchronize(q->stream);
        (void)hipStreamDestroy(q->stream);
    }
    if (q->done) (void)hipEventDestroy(q->done);
    q->batch[0].release();
    q->batch[1].release();
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
    return add_inet(q, segs, nseg, ps, csum_field, false);
}

int pipck_txq_add4_zc(pipck_txq* q, const pipck_hseg* segs, uint32_t nseg, uint8_t proto, uint32_t src,
                      uint32_t dst, void* csum_field) {
    TxPseudo ps{};
    ps.family = 4;
    ps.proto = proto;
    std::memcpy(ps.src, &src, 4);
    std::memcpy(ps.dst, &dst, 4);
    return add_inet(q, segs, nseg, ps, csum_field, true);
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
    return add_inet(q, segs, nseg, ps, csum_field, false);
}

int pipck_txq_add6_zc(pipck_txq* q, const pipck_hseg* segs, uint32_t nseg, uint8_t proto, const uint8_t* src,
                      const uint8_t* dst, void* csum_field) {
    if (!src || !dst) {
        set_error("pipck_txq_add6_zc: null address");
        return PIPCK_EINVAL;
    }
    TxPseudo ps{};
    ps.family = 6;
    ps.proto = proto;
    std::memcpy(ps.src, src, 16);
    std::memcpy(ps.dst, dst, 16);
    return add_inet(q, segs, nseg, ps, csum_field, true);
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
    TxBatch* b = &q->batch[q->cur];
    uint64_t off = 0;
    int rc = append_bytes(b, hdr, len, &off);
    if (rc) return rc;
    b->ip_hdrs.push_back(pipck_desc{off, len, 0});
    b->ip_field.push_back((uint8_t*)csum_field);
    return PIPCK_OK;
}

uint64_t pipck_txq_pending(const pipck_txq* q) { return q ? q->batch[q->cur].pending() : 0; }

uint64_t pipck_txq_inflight(const pipck_txq* q) { return q && q->inflight ? q->batch[q->cur ^ 1].pending() : 0; }

int pipck_txq_submit(pipck_txq* q) {
    if (!q) return PIPCK_EINVAL;
    return on_device(q, [&] {
        int rc = complete_inflight(q);  // at most one batch in flight
        if (rc) return rc;
        TxBatch* b = &q->batch[q->cur];
        if (!b->pending()) {
            b->clear();  // nothing queued: nothing may stay held either
            return PIPCK_OK;
        }
        if ((rc = enqueue(q, b))) return rc;
        q->inflight = true;
        q->cur ^= 1;
        return PIPCK_OK;
    });
}

int pipck_txq_complete(pipck_txq* q) {
    if (!q) return PIPCK_EINVAL;
    return on_device(q, [&] { return complete_inflight(q); });
}

int pipck_txq_flush(pipck_txq* q) {
    int rc = pipck_txq_submit(q);
    return rc ? rc : pipck_txq_complete(q);
}

}  // extern "C"
