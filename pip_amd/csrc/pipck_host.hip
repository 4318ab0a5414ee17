// pipck_host.hip -- host ABI of the engine: contexts, host-memory batches and
// pip's exact per-packet semantics on the device.
//
// pipck_host_sum() is what the C++ drop-in (pip_checksum_shim.cpp) calls for
// each of pip's six functions.  Unlike the batch kernels it has no length
// limit, so it reproduces pip's u32 accumulator exactly, wrap included
// (pip/pip_checksum.cpp:16-23): the device computes, per segment, the exact
// sums A (bytes at even offsets) and B (bytes at odd offsets) in u64, and the
// big-endian word sum of the segment is 256*A + B; one thread then replays
// pip's chain loop  sum = fold(fold(sum + 256*A + B mod 2^32))  (:110-112).
#include "pipck_common.hpp"
#include "pipck_device.hpp"

#include <immintrin.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

namespace pipck {

static thread_local std::string t_err;
// pipck_host_sum path of a context: staged copies (0), zero-copy host access
// (1), auto (2: zero-copy up to kZeroCopyMax staged bytes, the default of a
// new context), or the resident service (3: doorbell in pinned host memory;
// 4: doorbell in fine-grained device memory).  Set per context only
// (pipck_ctx_zero_copy): nothing is read from the environment.
constexpr int kDefaultZeroCopy = 2;
// 68 KiB: the largest IP datagram (65,535 B) with its segment table and the
// 16-byte padding of up to 132 segments.  At 64 KiB the table pushed a 65,535-B
// call onto the staged path (26 us against 15 us zero-copy, r04_percall_latency).
constexpr size_t kZeroCopyMax = 68u << 10;
void set_error(const std::string& msg) { t_err = msg; }

static std::shared_mutex g_pinned_mu;
static std::map<uintptr_t, PinnedRef> g_pinned;  // lo -> range

void pinned_add(const void* p, size_t bytes) {
    auto r = std::make_shared<PinnedRec>();
    r->lo = (uintptr_t)p;
    r->hi = (uintptr_t)p + bytes;
    std::unique_lock<std::shared_mutex> g(g_pinned_mu);
    g_pinned[(uintptr_t)p] = std::move(r);
}

int pinned_remove(const void* p) {
    std::unique_lock<std::shared_mutex> g(g_pinned_mu);
    auto it = g_pinned.find((uintptr_t)p);
    if (it == g_pinned.end()) return PIPCK_EINVAL;
    uint64_t expect = 0;
    if (!it->second->state.compare_exchange_strong(expect, kPinnedRemoved, std::memory_order_acq_rel))
        return PIPCK_EBUSY;  // a queued batch will read it in place
    g_pinned.erase(it);
    return PIPCK_OK;
}

PinnedRef pinned_lookup(const void* p, size_t len) {
    const uintptr_t a = (uintptr_t)p;
    std::shared_lock<std::shared_mutex> g(g_pinned_mu);
    auto it = g_pinned.upper_bound(a);
    if (it == g_pinned.begin()) return nullptr;
    --it;
    if (a + len > it->second->hi) return nullptr;
    return it->second;
}

bool pinned_acquire(PinnedRec& r) {
    uint64_t s = r.state.load(std::memory_order_acquire);
    do {
        if (s & kPinnedRemoved) return false;
    } while (!r.state.compare_exchange_weak(s, s + 1, std::memory_order_acq_rel));
    return true;
}

void pinned_release(PinnedRec& r) { r.state.fetch_sub(1, std::memory_order_acq_rel); }

int device_cus() {
    static std::mutex mu;
    static std::vector<int> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    std::lock_guard<std::mutex> g(mu);
    if ((size_t)dev >= cache.size()) cache.resize(dev + 1, 0);
    if (!cache[dev]) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
        cache[dev] = cus;
    }
    return cache[dev];
}

// ---------------------------------------------------------------------------
// exact chain kernel: one 1024-thread block walks the segments in order
// ---------------------------------------------------------------------------
struct SegRef {
    uint64_t offset;  // 16-byte aligned offset in the staging buffer
    uint32_t len;
    uint32_t pad;
};

__global__ __launch_bounds__(1024) void k_exact_chain(const uint8_t* __restrict__ stage, const SegRef* __restrict__ segs,
                                                      uint32_t nseg, uint32_t init, uint32_t* __restrict__ out) {
    __shared__ uint64_t sa[16], sb[16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint32_t sum = init;  // meaningful in thread 0 only
    for (uint32_t s = 0; s < nseg; s++) {
        const SegRef r = segs[s];
        const u32x4* base = reinterpret_cast<const u32x4*>(stage + r.offset);
        const uint32_t nch = (r.len + 15) / 16;
        uint64_t A = 0, B = 0;
        for (uint32_t c = threadIdx.x; c < nch; c += blockDim.x) {
            u32x4 v = base[c];
            const int hi = (int)r.len - 16 * (int)c;
            if (hi < 16) v = mask_tail(v, hi);
#pragma unroll
            for (int k = 0; k < 4; k++) {  // offsets within the segment: 4k+0, 4k+2 even; 4k+1, 4k+3 odd
                const uint32_t x = v[k];
                A += (x & 0xFFu) + ((x >> 16) & 0xFFu);
                B += ((x >> 8) & 0xFFu) + (x >> 24);
            }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            A += __shfl_xor(A, off, 64);
            B += __shfl_xor(B, off, 64);
        }
        if (lane == 0) {
            sa[w] = A;
            sb[w] = B;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint64_t tA = 0, tB = 0;
            for (int i = 0; i < nw; i++) {
                tA += sa[i];
                tB += sb[i];
            }
            sum += (uint32_t)(256ull * tA + tB);  // u32 wrap exactly as pip's accumulator
            sum = fold16(sum);
        }
        __syncthreads();
    }
    // pip's chain always holds at least one pip_buf: zero segments == one empty segment
    // a system-scope release: the zero-copy caller spins on this word in host
    // memory instead of synchronising the stream (all reads of the staging
    // buffer are done by now)
    if (threadIdx.x == 0) __hip_atomic_store(out, nseg ? sum : fold16(sum), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------------------
// resident per-packet service (pipck_ctx_zero_copy mode 3)
// ---------------------------------------------------------------------------
// A launch per call costs ~10 us (percall_bench), 20x pip's scalar loop on a
// 1,480-B segment.  In mode 3 one 256-thread block stays resident and polls a
// doorbell word in coherent pinned host memory: the caller stages the request
// exactly as the zero-copy path does, writes its parameters, releases a new
// sequence number and spins on the completion word the block releases after
// storing the result -- no launch, no stream operation.  The block exits after
// kResidentIdleMs without a request (or when the context is destroyed), so it
// never outlives its caller's activity by more than that; the next call
// relaunches it.  All accesses to the mailbox are system-scope atomics
// (vector memory); the staged bytes are read after the acquiring load.
// The request lives in ONE 64-byte line (an x86 cache line, so the device's
// 64-byte read of it is a consistent snapshot, and the host writes `req`
// last): a poll is one vector load that returns the sequence number, the
// parameters and up to kResidentInlineSegs segment (offset, length) pairs, so
// a request costs two PCIe round trips (the poll, then the bytes) instead of
// one per dependent field.  Chains of more segments read their SegRef table
// from the staging buffer.
constexpr uint32_t kResidentInlineSegs = 5;
// The doorbell -- host-written, device-polled.  In fine-grained device memory
// when the host can write that directly (mode 4: large-BAR systems; the device
// then polls its own HBM), else in coherent pinned host memory (mode 3, and
// mode 4 where that allocation fails; each poll a PCIe read).
struct alignas(128) ResidentDoorbell {
    uint32_t req;    // host: sequence number of the posted request (written last)
    uint32_t nseg, init, pad0;
    uint64_t bytes;  // device-readable address of the staged segment bytes
    uint32_t seg[2 * kResidentInlineSegs];  // (offset from `bytes`, length) of the first segments
    uint32_t pad1[16];
    alignas(64) uint32_t stop;  // host: end the service
    uint32_t pad2[15];
};
static_assert(offsetof(ResidentDoorbell, pad1) == 64, "the request must fill one 64-byte line");
// The reply -- device-written, host-polled: always in coherent pinned host memory.
struct alignas(128) ResidentReply {
    uint32_t done;  // sequence number of the last completed request (release)
    uint32_t result;
    uint32_t alive;  // 1 while the service runs
    uint32_t pad[29];
};
// Idle exit.  While the block runs it holds a CU slot, and every hipFree /
// hipHostFree / device-wide synchronise in the process waits for it to exit:
// this bounds that stall (idle time + one poll, ~10 ms) -- the worst case
// pip_checksum_amd.h and pipck.h state.  A relaunch costs ~10 us, negligible
// against 10 ms of idleness.
constexpr uint32_t kResidentIdleMs = 10;

__global__ __launch_bounds__(256) void k_resident(const ResidentDoorbell* db, ResidentReply* rp, uint64_t idle_ticks) {
    __shared__ uint64_t sa[64], sb[64];  // per segment (up to 64 in flight at once), then folded in order
    __shared__ uint32_t s_line[16];
    __shared__ uint32_t s_go;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // the last request served: the same value in every thread (wave 0 polls against it)
    uint32_t last = (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)__hip_atomic_load(&rp->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    if (threadIdx.x == 0) __hip_atomic_store(&rp->alive, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t* line = reinterpret_cast<const uint32_t*>(db);
    for (;;) {
        if (w == 0) {
            // wave 0 polls: lanes 0..15 read the request line in one 64-byte load
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
            uint32_t go = 0;
            for (;;) {
                const uint32_t v = lane < 16 ? __hip_atomic_load(line + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
                const uint32_t r = (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
                if (r != last) {
                    if (lane < 16) s_line[lane] = v;
                    go = 1;
                    break;
                }
                if (__hip_atomic_load(&db->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) break;  // every wave exits
                __builtin_amdgcn_s_sleep(1);
            }
            // the staged bytes were written before `req`: order the reads below after it
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
            if (lane == 0) s_go = go;
        }
        __syncthreads();
        if (!s_go) break;
        const uint32_t req = s_line[0], nseg = s_line[1], init = s_line[2];
        const uint8_t* bytes = reinterpret_cast<const uint8_t*>((uint64_t)s_line[4] | (uint64_t)s_line[5] << 32);
        const SegRef* table = reinterpret_cast<const SegRef*>(bytes) - 0;  // SegRef table precedes the bytes
        uint32_t sum = init;  // thread 0
        if (nseg <= kResidentInlineSegs) {
            // every chunk of every segment in one pass over the block: each
            // thread issues up to 8 loads before summing any, so a request of
            // up to 32 KiB is one PCIe round trip
            uint32_t pre[kResidentInlineSegs + 1];
            pre[0] = 0;
#pragma unroll
            for (uint32_t k = 0; k < kResidentInlineSegs; k++)
                pre[k + 1] = pre[k] + (k < nseg ? (s_line[7 + 2 * k] + 15) / 16 : 0u);
            const uint32_t total = pre[kResidentInlineSegs];
            uint64_t A[kResidentInlineSegs] = {}, B[kResidentInlineSegs] = {};
            for (uint32_t c0 = threadIdx.x; c0 < total; c0 += 256 * 8) {
                u32x4 v[8];
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const uint32_t c = c0 + 256u * j;
                    uint32_t k = 0;
#pragma unroll
                    for (uint32_t q = 1; q < kResidentInlineSegs; q++) k += c >= pre[q] ? 1u : 0u;
                    v[j] = c < total ? *reinterpret_cast<const u32x4*>(bytes + s_line[6 + 2 * k] + 16u * (c - pre[k]))
                                     : u32x4{0u, 0u, 0u, 0u};
                }
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const uint32_t c = c0 + 256u * j;
                    if (c >= total) continue;
                    uint32_t k = 0;
#pragma unroll
                    for (uint32_t q = 1; q < kResidentInlineSegs; q++) k += c >= pre[q] ? 1u : 0u;
                    u32x4 x = v[j];
                    const int hi = (int)s_line[7 + 2 * k] - 16 * (int)(c - pre[k]);
                    if (hi < 16) x = mask_tail(x, hi);
                    uint64_t a = 0, b = 0;
#pragma unroll
                    for (int q = 0; q < 4; q++) {  // offsets 4q+0, 4q+2 even; 4q+1, 4q+3 odd
                        a += (x[q] & 0xFFu) + ((x[q] >> 16) & 0xFFu);
                        b += ((x[q] >> 8) & 0xFFu) + (x[q] >> 24);
                    }
#pragma unroll
                    for (uint32_t q = 0; q < kResidentInlineSegs; q++)
                        if (q == k) {
                            A[q] += a;
                            B[q] += b;
                        }
                }
            }
#pragma unroll
            for (uint32_t q = 0; q < kResidentInlineSegs; q++) {
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    A[q] += __shfl_xor(A[q], o, 64);
                    B[q] += __shfl_xor(B[q], o, 64);
                }
                if (lane == 0) {
                    sa[4 * q + w] = A[q];
                    sb[4 * q + w] = B[q];
                }
            }
            __syncthreads();
            if (threadIdx.x == 0)
                for (uint32_t q = 0; q < nseg; q++) {
                    const uint64_t a = sa[4 * q] + sa[4 * q + 1] + sa[4 * q + 2] + sa[4 * q + 3];
                    const uint64_t b = sb[4 * q] + sb[4 * q + 1] + sb[4 * q + 2] + sb[4 * q + 3];
                    sum += (uint32_t)(256ull * a + b);  // pip's u32 wrap, then two folds (pip_checksum.cpp:16-30)
                    sum = fold16(sum);
                }
            __syncthreads();
        }
        // longer chains: segments in groups of 64: wave w sums segments w, w+4, ... of the group
        // (all of one group's loads in flight together), thread 0 then replays
        // pip's sequential fold over them in order (pip_checksum.cpp:110-112)
        for (uint32_t g0 = 0; nseg > kResidentInlineSegs && g0 < nseg; g0 += 64) {
            const uint32_t gn = min(64u, nseg - g0);
            for (uint32_t k = (uint32_t)w; k < gn; k += 4) {
                const uint32_t sg = g0 + k;
                uint32_t off, len;
                if (sg < kResidentInlineSegs) {
                    off = s_line[6 + 2 * sg];
                    len = s_line[7 + 2 * sg];
                } else {
                    const SegRef r = *(reinterpret_cast<const SegRef*>(bytes) - (int64_t)(((nseg * sizeof(SegRef) + 15) & ~15ull) / sizeof(SegRef)) + sg);
                    off = (uint32_t)r.offset;
                    len = r.len;
                }
                const u32x4* base = reinterpret_cast<const u32x4*>(bytes + off);
                const uint32_t nch = (len + 15) / 16;
                uint64_t A = 0, B = 0;
                for (uint32_t c = (uint32_t)lane; c < nch; c += 64) {
                    u32x4 v = base[c];
                    const int hi = (int)len - 16 * (int)c;
                    if (hi < 16) v = mask_tail(v, hi);
#pragma unroll
                    for (int q = 0; q < 4; q++) {  // offsets 4q+0, 4q+2 even; 4q+1, 4q+3 odd
                        const uint32_t x = v[q];
                        A += (x & 0xFFu) + ((x >> 16) & 0xFFu);
                        B += ((x >> 8) & 0xFFu) + (x >> 24);
                    }
                }
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    A += __shfl_xor(A, o, 64);
                    B += __shfl_xor(B, o, 64);
                }
                if (lane == 0) {
                    sa[k] = A;
                    sb[k] = B;
                }
            }
            __syncthreads();
            if (threadIdx.x == 0)
                for (uint32_t k = 0; k < gn; k++) {
                    sum += (uint32_t)(256ull * sa[k] + sb[k]);  // pip's u32 wrap, then two folds
                    sum = fold16(sum);
                }
            __syncthreads();
        }
        (void)table;
        if (threadIdx.x == 0) {
            __hip_atomic_store(&rp->result, nseg ? sum : fold16(sum), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&rp->done, req, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        last = req;
        __syncthreads();
    }
    if (threadIdx.x == 0) __hip_atomic_store(&rp->alive, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace pipck

using namespace pipck;

struct pipck_ctx {
    int device = 0;
    hipStream_t stream[2] = {nullptr, nullptr};
    hipEvent_t done[2] = {nullptr, nullptr};
    // exact path staging
    uint8_t* h_stage = nullptr;  // pinned
    uint8_t* d_stage = nullptr;
    size_t stage_cap = 0;
    uint32_t* d_result = nullptr;
    uint32_t* h_result = nullptr;  // pinned
    // host batch pipeline
    uint8_t* d_chunk[2] = {nullptr, nullptr};
    uint16_t* d_out[2] = {nullptr, nullptr};
    size_t chunk_cap = 0;
    // byte-packed host batches (pipck_host_checksum_packed_bytes): per-chunk
    // lengths and tile index, beside d_chunk / d_out
    uint16_t* d_lens[2] = {nullptr, nullptr};
    uint64_t* d_tile_off[2] = {nullptr, nullptr};
    uint64_t packed_cap = 0;  // packets per chunk d_lens / d_tile_off hold
    uint64_t out_cap = 0;     // results per chunk d_out holds
    uint32_t* d_pseudo = nullptr;
    void* d_flows = nullptr;
    uint32_t flows_cap = 0;
    int zero_copy = kDefaultZeroCopy;  // pipck_host_sum path (pipck_ctx_zero_copy)
    // resident service (modes 3, 4): its own stream and mailbox
    hipStream_t res_stream = nullptr;
    ResidentDoorbell* db = nullptr;
    bool db_vram = false;
    ResidentReply* rp = nullptr;
    uint32_t res_seq = 0;
    bool res_launched = false;
    std::mutex mu;
};

namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// The host pipelines' double-buffered device chunks: d_chunk[i] of at least
// `bytes`, d_out[i] of at least `results` u16 (each grown on its own).
int reserve_chunks(pipck_ctx* c, size_t bytes, uint64_t results) {
    if (bytes > c->chunk_cap) {
        for (int i = 0; i < 2; i++) {
            if (c->d_chunk[i]) PIPCK_HIP(hipFree(c->d_chunk[i]));
            c->d_chunk[i] = nullptr;
        }
        c->chunk_cap = 0;
        for (int i = 0; i < 2; i++) PIPCK_HIP(hipMalloc((void**)&c->d_chunk[i], bytes));
        c->chunk_cap = bytes;
    }
    if (results > c->out_cap) {
        for (int i = 0; i < 2; i++) {
            if (c->d_out[i]) PIPCK_HIP(hipFree(c->d_out[i]));
            c->d_out[i] = nullptr;
        }
        c->out_cap = 0;
        for (int i = 0; i < 2; i++) PIPCK_HIP(hipMalloc((void**)&c->d_out[i], results * sizeof(uint16_t)));
        c->out_cap = results;
    }
    return PIPCK_OK;
}

// A host flow table to the device and its pseudo-header bases (stream 0; stream
// 1 waits for them).  family 0: none, *d_pseudo = null.
int upload_flows(pipck_ctx* c, int family, const void* h_flows, uint32_t n_flows, const uint32_t** d_pseudo) {
    *d_pseudo = nullptr;
    if (!family) return PIPCK_OK;
    const size_t fbytes = (size_t)n_flows * (family == 4 ? sizeof(pipck_flow4) : sizeof(pipck_flow6));
    if (n_flows > c->flows_cap) {
        if (c->d_flows) PIPCK_HIP(hipFree(c->d_flows));
        if (c->d_pseudo) PIPCK_HIP(hipFree(c->d_pseudo));
        c->d_flows = nullptr;
        c->d_pseudo = nullptr;
        c->flows_cap = 0;
        PIPCK_HIP(hipMalloc(&c->d_flows, (size_t)n_flows * sizeof(pipck_flow6)));
        PIPCK_HIP(hipMalloc((void**)&c->d_pseudo, (size_t)n_flows * sizeof(uint32_t)));
        c->flows_cap = n_flows;
    }
    PIPCK_HIP(hipMemcpyAsync(c->d_flows, h_flows, fbytes, hipMemcpyHostToDevice, c->stream[0]));
    int rc = family == 4 ? pipck_flows4_prepare((const pipck_flow4*)c->d_flows, n_flows, c->d_pseudo, c->stream[0])
                         : pipck_flows6_prepare((const pipck_flow6*)c->d_flows, n_flows, c->d_pseudo, c->stream[0]);
    if (rc) return rc;
    PIPCK_HIP(hipEventRecord(c->done[0], c->stream[0]));
    PIPCK_HIP(hipStreamWaitEvent(c->stream[1], c->done[0], 0));
    *d_pseudo = c->d_pseudo;
    return PIPCK_OK;
}

// Modes 3 and 4: make sure the resident block runs (launching it if it never
// ran or has exited after its idle timeout).
int resident_start(pipck_ctx* c) {
    if (!c->rp) {
        c->db_vram = c->zero_copy == 4 &&
                     hipExtMallocWithFlags((void**)&c->db, sizeof(ResidentDoorbell), hipDeviceMallocFinegrained) == hipSuccess;
        if (!c->db_vram) PIPCK_HIP(hipHostMalloc((void**)&c->db, sizeof(ResidentDoorbell), hipHostMallocCoherent));
        for (size_t i = 0; i < sizeof(ResidentDoorbell) / 4; i++) ((volatile uint32_t*)c->db)[i] = 0;
        PIPCK_HIP(hipHostMalloc((void**)&c->rp, sizeof(ResidentReply), hipHostMallocCoherent));
        std::memset((void*)c->rp, 0, sizeof(ResidentReply));
        PIPCK_HIP(hipStreamCreateWithFlags(&c->res_stream, hipStreamNonBlocking));
        c->res_seq = 0;
    }
    if (c->res_launched) {
        if (__atomic_load_n(&c->rp->alive, __ATOMIC_ACQUIRE)) return PIPCK_OK;
        const hipError_t q = hipStreamQuery(c->res_stream);
        if (q == hipErrorNotReady) return PIPCK_OK;  // launched, not started yet
        if (q != hipSuccess) PIPCK_HIP(q);
    }
    ((volatile uint32_t*)&c->db->stop)[0] = 0u;
    _mm_sfence();
    // the service may have finished requests up to res_seq; it resumes from `done`
    hipLaunchKernelGGL(k_resident, dim3(1), dim3(256), 0, c->res_stream, c->db, c->rp,
                       (uint64_t)kResidentIdleMs * 100000ull);
    PIPCK_LAUNCHED("k_resident");
    c->res_launched = true;
    return PIPCK_OK;
}

void resident_halt(pipck_ctx* c) {  // end the block (it restarts on the next call)
    if (!c->res_launched) return;
    ((volatile uint32_t*)&c->db->stop)[0] = 1u;
    _mm_sfence();
    (void)hipStreamSynchronize(c->res_stream);  // the block sees stop within one poll
    c->res_launched = false;
}

void resident_stop(pipck_ctx* c) {
    if (!c->rp) return;
    resident_halt(c);
    if (c->res_stream) (void)hipStreamDestroy(c->res_stream);
    if (c->db_vram) (void)hipFree(c->db);
    else (void)hipHostFree(c->db);
    (void)hipHostFree(c->rp);
    c->db = nullptr;
    c->rp = nullptr;
    c->res_stream = nullptr;
}

int grow_stage(pipck_ctx* c, size_t need) {
    if (need <= c->stage_cap) return PIPCK_OK;
    // hipHostFree / hipFree wait for the device: end the resident block first
    // (it restarts on its own on the next call)
    resident_halt(c);
    size_t cap = need < (1u << 20) ? (1u << 20) : need + need / 2;
    if (c->h_stage) PIPCK_HIP(hipHostFree(c->h_stage));
    if (c->d_stage) PIPCK_HIP(hipFree(c->d_stage));
    c->h_stage = nullptr;
    c->d_stage = nullptr;
    c->stage_cap = 0;
    // coherent (fine-grained): the zero-copy path's kernel reads it directly,
    // and no device cache may hold a previous call's bytes
    PIPCK_HIP(hipHostMalloc((void**)&c->h_stage, cap, hipHostMallocCoherent));
    PIPCK_HIP(hipMalloc((void**)&c->d_stage, cap));
    c->stage_cap = cap;
    return PIPCK_OK;
}

}  // namespace

extern "C" {

const char* pipck_last_error(void) { return pipck::t_err.c_str(); }

int pipck_ctx_create(int device, pipck_ctx** out) {
    if (!out) return PIPCK_EINVAL;
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0) {
        set_error(std::string("pipck_ctx_create: no HIP device: ") + hipGetErrorString(e));
        return PIPCK_ENODEV;
    }
    if (device < 0) PIPCK_HIP(hipGetDevice(&device));
    if (device >= n) {
        set_error("pipck_ctx_create: device index out of range");
        return PIPCK_EINVAL;
    }
    DeviceGuard g(device);
    hipDeviceProp_t prop;
    PIPCK_HIP(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_error(std::string("pipck_ctx_create: device is ") + prop.gcnArchName + ", libpipck is built for gfx950");
        return PIPCK_ENODEV;
    }
    pipck_ctx* c = new pipck_ctx();
    c->device = device;
    for (int i = 0; i < 2; i++) {
        PIPCK_HIP(hipStreamCreateWithFlags(&c->stream[i], hipStreamNonBlocking));
        PIPCK_HIP(hipEventCreateWithFlags(&c->done[i], hipEventDisableTiming));
    }
    PIPCK_HIP(hipMalloc((void**)&c->d_result, sizeof(uint32_t)));
    PIPCK_HIP(hipHostMalloc((void**)&c->h_result, sizeof(uint32_t), hipHostMallocCoherent));
    *out = c;
    return PIPCK_OK;
}

int pipck_ctx_destroy(pipck_ctx* c) {
    if (!c) return PIPCK_OK;
    DeviceGuard g(c->device);
    resident_stop(c);
    for (int i = 0; i < 2; i++) {
        if (c->stream[i]) (void)hipStreamSynchronize(c->stream[i]);
        if (c->d_chunk[i]) (void)hipFree(c->d_chunk[i]);
        if (c->d_out[i]) (void)hipFree(c->d_out[i]);
        if (c->d_lens[i]) (void)hipFree(c->d_lens[i]);
        if (c->d_tile_off[i]) (void)hipFree(c->d_tile_off[i]);
        if (c->done[i]) (void)hipEventDestroy(c->done[i]);
        if (c->stream[i]) (void)hipStreamDestroy(c->stream[i]);
    }
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    if (c->d_stage) (void)hipFree(c->d_stage);
    if (c->d_result) (void)hipFree(c->d_result);
    if (c->h_result) (void)hipHostFree(c->h_result);
    if (c->d_pseudo) (void)hipFree(c->d_pseudo);
    if (c->d_flows) (void)hipFree(c->d_flows);
    delete c;
    return PIPCK_OK;
}

int pipck_host_sum(pipck_ctx* c, const pipck_hseg* segs, uint32_t nseg, uint32_t init, uint32_t* out) {
    if (!c || !out || (nseg && !segs)) {
        set_error("pipck_host_sum: null argument");
        return PIPCK_EINVAL;
    }
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    // stage: [SegRef table][segment bytes, each 16-byte aligned]
    const size_t table = ((size_t)nseg * sizeof(SegRef) + 15) & ~(size_t)15;
    size_t need = table;
    for (uint32_t i = 0; i < nseg; i++) {
        if (segs[i].len && !segs[i].ptr) {
            set_error("pipck_host_sum: null segment with nonzero length");
            return PIPCK_EINVAL;
        }
        need += ((size_t)segs[i].len + 15) & ~(size_t)15;
    }
    int rc = grow_stage(c, need ? need : 16);
    if (rc) return rc;
    SegRef* refs = reinterpret_cast<SegRef*>(c->h_stage);
    size_t off = table;
    for (uint32_t i = 0; i < nseg; i++) {
        refs[i] = SegRef{off - table, segs[i].len, 0};
        if (segs[i].len) std::memcpy(c->h_stage + off, segs[i].ptr, segs[i].len);
        off += ((size_t)segs[i].len + 15) & ~(size_t)15;
    }
    hipStream_t s = c->stream[0];
    const int zc = c->zero_copy;
    if (zc >= 3 && need <= kZeroCopyMax) {
        // the resident block: post the request, spin on its completion word
        if ((rc = resident_start(c))) return rc;
        ResidentDoorbell* db = c->db;
        ResidentReply* rp = c->rp;
        const uint32_t seq = ++c->res_seq;
        volatile uint32_t* line = reinterpret_cast<volatile uint32_t*>(db);
        line[1] = nseg;
        line[2] = init;
        const uint64_t bytes = (uint64_t)(uintptr_t)(c->h_stage + table);
        line[4] = (uint32_t)bytes;
        line[5] = (uint32_t)(bytes >> 32);
        for (uint32_t i = 0; i < nseg && i < kResidentInlineSegs; i++) {
            line[6 + 2 * i] = (uint32_t)refs[i].offset;
            line[7 + 2 * i] = refs[i].len;
        }
        // the staged bytes and the parameters before the sequence number (the
        // doorbell may be write-combined device memory)
        _mm_sfence();
        line[0] = seq;
        _mm_sfence();
        auto t0 = std::chrono::steady_clock::now();
        while (__atomic_load_n(&rp->done, __ATOMIC_ACQUIRE) != seq) {
            const auto el = std::chrono::steady_clock::now() - t0;
            if (el > std::chrono::milliseconds(2)) {
                // the block may have hit its idle timeout just before the post:
                // relaunch it (it resumes from `done`, so it serves this request)
                if ((rc = resident_start(c))) return rc;
                if (el > std::chrono::seconds(2)) {
                    // end the block before returning: a block that starts late
                    // would otherwise serve this stale request while the next
                    // call rewrites the staging buffer and the doorbell
                    resident_halt(c);
                    set_error("pipck_host_sum: the resident service did not answer within 2 s");
                    return PIPCK_EHIP;
                }
            }
            __builtin_ia32_pause();
        }
        *out = __atomic_load_n(&rp->result, __ATOMIC_RELAXED);
        return PIPCK_OK;
    }
    if (zc == 1 || (zc >= 2 && need <= kZeroCopyMax)) {
        // The kernel reads the pinned staging buffer over PCIe and writes the
        // result into pinned host memory: no copy commands around the launch.
        // The result (<= 0xFFFF) replaces a sentinel no sum can take; the host
        // spins on it rather than synchronising the stream, and falls back to
        // a synchronise (which also reports a failed kernel) after 2 ms.
        __atomic_store_n(c->h_result, 0xFFFFFFFFu, __ATOMIC_RELAXED);
        hipLaunchKernelGGL(k_exact_chain, dim3(1), dim3(1024), 0, s, c->h_stage + table,
                           reinterpret_cast<const SegRef*>(c->h_stage), nseg, init, c->h_result);
        PIPCK_LAUNCHED("k_exact_chain");
        const auto t0 = std::chrono::steady_clock::now();
        uint32_t v;
        while ((v = __atomic_load_n(c->h_result, __ATOMIC_ACQUIRE)) == 0xFFFFFFFFu) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
                PIPCK_HIP(hipStreamSynchronize(s));
                v = __atomic_load_n(c->h_result, __ATOMIC_ACQUIRE);
                break;
            }
            __builtin_ia32_pause();
        }
        *out = v;
        return PIPCK_OK;
    } else {
        if (need) PIPCK_HIP(hipMemcpyAsync(c->d_stage, c->h_stage, need, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_exact_chain, dim3(1), dim3(1024), 0, s, c->d_stage + table,
                           reinterpret_cast<const SegRef*>(c->d_stage), nseg, init, c->d_result);
        PIPCK_LAUNCHED("k_exact_chain");
        PIPCK_HIP(hipMemcpyAsync(c->h_result, c->d_result, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    }
    PIPCK_HIP(hipStreamSynchronize(s));
    *out = *(volatile uint32_t*)c->h_result;
    return PIPCK_OK;
}

int pipck_ctx_zero_copy(pipck_ctx* c, int mode) {
    if (!c || mode < 0 || mode > 4) {
        set_error("pipck_ctx_zero_copy: null context or mode outside 0..4");
        return PIPCK_EINVAL;
    }
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    // any change releases the resident block's CU slot (3 <-> 4 also moves the doorbell)
    if (mode != c->zero_copy) resident_stop(c);
    c->zero_copy = mode;
    return PIPCK_OK;
}

int pipck_host_register(void* p, size_t bytes) {
    if (!p || !bytes) {
        set_error("pipck_host_register: null pointer or empty range");
        return PIPCK_EINVAL;
    }
    PIPCK_HIP(hipHostRegister(p, bytes, hipHostRegisterMapped));
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, p, 0) != hipSuccess || dp != p) {
        (void)hipHostUnregister(p);
        set_error("pipck_host_register: the device address of this range differs from the host address");
        return PIPCK_EINVAL;
    }
    pinned_add(p, bytes);
    return PIPCK_OK;
}

int pipck_host_unregister(void* p) {
    const int rc = pinned_remove(p);
    if (rc == PIPCK_EBUSY) {
        set_error("pipck_host_unregister: a queued TX batch still reads this range in place");
        return rc;
    }
    if (rc) {
        set_error("pipck_host_unregister: not a range made by pipck_host_register");
        return rc;
    }
    PIPCK_HIP(hipHostUnregister(p));
    return PIPCK_OK;
}

}  // extern "C"

namespace {

// Waits for both of the context's streams when a chunked host call leaves
// early: chunks already queued may still read the caller's input by DMA and
// write its result array, which the caller owns again once the call returns.
struct DrainOnError {
    pipck_ctx* c;
    bool armed = true;
    ~DrainOnError() {
        if (armed) {
            (void)hipStreamSynchronize(c->stream[0]);
            (void)hipStreamSynchronize(c->stream[1]);
        }
    }
    // The normal end: wait for BOTH streams whatever the first wait returns (a
    // chunk still queued on stream 1 must not read the caller's input or write
    // its results after the call has returned), then report the first error.
    int finish() {
        const hipError_t e0 = hipStreamSynchronize(c->stream[0]);
        const hipError_t e1 = hipStreamSynchronize(c->stream[1]);
        if (e0 != hipSuccess) return hip_fail(e0, "hipStreamSynchronize(stream 0)");
        if (e1 != hipSuccess) return hip_fail(e1, "hipStreamSynchronize(stream 1)");
        return PIPCK_OK;
    }
};

// Byte-packed host batches (packet i's h_lens[i] bytes right after packet
// i-1's): chunks of whole packets, ~64 MiB of bytes (at most 1M packets) each,
// double-buffered over the context's two streams -- H2D of the chunk's bytes
// and lengths, its tile index (pipck_packed_bytes_index), then work(b, first,
// m, stream) launches the chunk's kernel and its D2H.  Waits for both streams.
// The caller holds c->mu and the device.
template <typename Work>
int host_packed_chunks(pipck_ctx* c, const void* h_arena, const uint16_t* h_lens, uint64_t n, Work&& work) {
    constexpr uint64_t kTarget = 64ull << 20, kMaxPkts = 1ull << 20;
    int rc;
    if ((rc = reserve_chunks(c, (size_t)(kTarget + 65536 + 256), kMaxPkts))) return rc;  // overshoot < one packet
    if (kMaxPkts > c->packed_cap) {
        for (int i = 0; i < 2; i++) {
            if (c->d_lens[i]) PIPCK_HIP(hipFree(c->d_lens[i]));
            if (c->d_tile_off[i]) PIPCK_HIP(hipFree(c->d_tile_off[i]));
            c->d_lens[i] = nullptr;
            c->d_tile_off[i] = nullptr;
        }
        c->packed_cap = 0;
        for (int i = 0; i < 2; i++) {
            PIPCK_HIP(hipMalloc((void**)&c->d_lens[i], kMaxPkts * sizeof(uint16_t)));
            PIPCK_HIP(hipMalloc((void**)&c->d_tile_off[i], (kMaxPkts / 64 + 2) * sizeof(uint64_t)));
        }
        c->packed_cap = kMaxPkts;
    }
    const uint8_t* src = (const uint8_t*)h_arena;
    uint64_t first = 0, off = 0;
    DrainOnError drain{c};  // from the first enqueue on, every return waits for both streams
    for (uint64_t k = 0; first < n; k++) {
        uint64_t m = 0, bytes = 0;
        while (first + m < n && m < kMaxPkts && bytes < kTarget) bytes += h_lens[first + m++];
        const int b = (int)(k & 1);
        hipStream_t s = c->stream[b];
        if (bytes) PIPCK_HIP(hipMemcpyAsync(c->d_chunk[b], src + off, (size_t)bytes, hipMemcpyHostToDevice, s));
        PIPCK_HIP(hipMemcpyAsync(c->d_lens[b], h_lens + first, m * sizeof(uint16_t), hipMemcpyHostToDevice, s));
        if ((rc = pipck_packed_bytes_index(c->d_lens[b], m, c->d_tile_off[b], s))) return rc;
        if ((rc = work(b, first, m, s))) return rc;
        first += m;
        off += bytes;
    }
    drain.armed = false;
    return drain.finish();
}

}  // namespace

extern "C" {

void* pipck_host_alloc(size_t bytes) {
    // coherent (fine-grained): kernels may read it in place (zero-copy TX
    // segments), and no device cache may keep bytes the host rewrites later
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocCoherent) != hipSuccess) return nullptr;
    pinned_add(p, bytes);
    return p;
}

int pipck_host_free(void* p) {
    if (!p) return PIPCK_OK;
    const int rc = pinned_remove(p);
    if (rc == PIPCK_EBUSY) {
        set_error("pipck_host_free: a queued TX batch still reads this buffer in place");
        return rc;
    }
    if (rc) {
        set_error("pipck_host_free: not a buffer from pipck_host_alloc");
        return rc;
    }
    PIPCK_HIP(hipHostFree(p));
    return PIPCK_OK;
}

int pipck_host_checksum_packed_bytes(pipck_ctx* c, const void* h_arena, const uint16_t* h_lens, uint64_t n,
                                     int family, const void* h_flows, uint32_t n_flows, uint64_t flow_origin,
                                     uint16_t* h_out) {
    if (!c || (n && (!h_arena || !h_lens || !h_out)) || (family != 0 && family != 4 && family != 6) ||
        (family && (!h_flows || !n_flows))) {
        set_error("pipck_host_checksum_packed_bytes: bad argument");
        return PIPCK_EINVAL;
    }
    if (!n) return PIPCK_OK;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    const uint32_t* d_pseudo = nullptr;
    int rc = upload_flows(c, family, h_flows, n_flows, &d_pseudo);
    if (rc) return rc;
    return host_packed_chunks(c, h_arena, h_lens, n, [&](int b, uint64_t first, uint64_t m, hipStream_t s) {
        int r = pipck_checksum_packed_bytes_n(c->d_chunk[b], c->chunk_cap, c->d_lens[b], c->d_tile_off[b], m,
                                              d_pseudo, n_flows, nullptr, flow_origin + first, c->d_out[b], nullptr, s);
        if (r) return r;
        PIPCK_HIP(hipMemcpyAsync(h_out + first, c->d_out[b], m * sizeof(uint16_t), hipMemcpyDeviceToHost, s));
        return PIPCK_OK;
    });
}

int pipck_host_rx_verify_packed(pipck_ctx* c, const void* h_frames, const uint16_t* h_lens, uint64_t n, uint8_t* h_ok,
                                uint64_t* n_verified) {
    if (n_verified) *n_verified = 0;
    if (!c || (n && (!h_frames || !h_lens || !h_ok))) {
        set_error("pipck_host_rx_verify_packed: bad argument");
        return PIPCK_EINVAL;
    }
    if (!n) return PIPCK_OK;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    int rc = host_packed_chunks(c, h_frames, h_lens, n, [&](int b, uint64_t first, uint64_t m, hipStream_t s) {
        uint8_t* d_ok = reinterpret_cast<uint8_t*>(c->d_out[b]);  // u16 per packet: room for the u8 verdicts
        int r = pipck_rx_verify_device(c->d_chunk[b], c->chunk_cap, c->d_lens[b], c->d_tile_off[b], m, d_ok, nullptr, s);
        if (r) return r;
        PIPCK_HIP(hipMemcpyAsync(h_ok + first, d_ok, (size_t)m, hipMemcpyDeviceToHost, s));
        return PIPCK_OK;
    });
    if (rc) return rc;
    if (n_verified) {
        uint64_t good = 0;
        for (uint64_t i = 0; i < n; i++) good += h_ok[i] == PIPCK_RX_VERIFIED;
        *n_verified = good;
    }
    return PIPCK_OK;
}

int pipck_host_checksum_fixed(pipck_ctx* c, const void* h_arena, uint64_t stride, uint32_t len, uint64_t n,
                              int family, const void* h_flows, uint32_t n_flows, uint64_t flow_origin,
                              uint16_t* h_out) {
    if (!c || (n && (!h_arena || !h_out)) || (family != 0 && family != 4 && family != 6) ||
        (family && (!h_flows || !n_flows))) {
        set_error("pipck_host_checksum_fixed: bad argument");
        return PIPCK_EINVAL;
    }
    if (!n) return PIPCK_OK;
    if (stride < len) {
        set_error("pipck_host_checksum_fixed: stride < len");
        return PIPCK_EINVAL;
    }
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    const uint32_t* d_pseudo = nullptr;
    int rc = upload_flows(c, family, h_flows, n_flows, &d_pseudo);
    if (rc) return rc;
    // ~64 MiB chunks, double-buffered: chunk k uses stream k%2 (H2D -> kernel -> D2H)
    const uint64_t per_chunk = std::max<uint64_t>(1, (64ull << 20) / stride);
    const size_t chunk_bytes = (size_t)(per_chunk * stride);
    if ((rc = reserve_chunks(c, chunk_bytes, per_chunk))) return rc;
    DrainOnError drain{c};  // from the first enqueue on, every return waits for both streams
    for (uint64_t first = 0, k = 0; first < n; first += per_chunk, k++) {
        const uint64_t m = std::min<uint64_t>(per_chunk, n - first);
        const int b = (int)(k & 1);
        hipStream_t s = c->stream[b];
        const size_t bytes = (size_t)((m - 1) * stride + len);
        PIPCK_HIP(hipMemcpyAsync(c->d_chunk[b], (const uint8_t*)h_arena + first * stride, bytes,
                                 hipMemcpyHostToDevice, s));
        rc = pipck_checksum_fixed(c->d_chunk[b], stride, len, m, d_pseudo, n_flows, nullptr, flow_origin + first,
                                  c->d_out[b], s);
        if (rc) return rc;
        PIPCK_HIP(hipMemcpyAsync(h_out + first, c->d_out[b], m * sizeof(uint16_t), hipMemcpyDeviceToHost, s));
    }
    drain.armed = false;
    return drain.finish();
}

}  // extern "C"
