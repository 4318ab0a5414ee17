// pipck_gen.hip -- on-device synthetic workloads for the bench and the GPU tests.
//
// Packets are generated in HBM from global packet ids with a counter-based
// hash, so a batch never crosses PCIe, any packet can be regenerated on the
// CPU (oracle/pipck_oracle.c holds the independent CPU twin of this spec), and
// sharding over 1/2/4/8 GPUs does not change a single byte.
//
//   mix64      = SplitMix64 finalizer
//   key(pkt)   = mix64(seed ^ mix64(pkt))
//   class      = mix64(key ^ 0xA5A5A5A5A5A5A5A5) % 1000: 0 all-zero, 1 all-0xFF, else random
//   random     : byte b = byte (b % 8) of mix64(key + b / 8)
//   headers    : TCP th_off=0x50 (random class), th_sum=0; UDP uh_ulen=len (random class),
//                uh_sum=0; IPv4 ver/ihl=0x45 (random class), ip_sum=0
//   zipf len   : w_k = floor(2^40 / k), k = 1..8937, len = 63 + k by inverse CDF
#include "pipck_common.hpp"

#include <hipcub/hipcub.hpp>

#include <mutex>
#include <vector>

namespace pipck {

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t pkt_key(uint64_t seed, uint64_t pkt) { return mix64(seed ^ mix64(pkt)); }

// Bytes [8j, 8j+8) of a packet, header fields applied, bytes >= len zeroed.
__device__ __forceinline__ uint64_t packet_word(uint64_t key, uint32_t cls, uint32_t len, uint32_t hdr, uint32_t j) {
    uint64_t w = cls == 0 ? 0ull : cls == 1 ? ~0ull : mix64(key + j);
    const uint32_t b0 = 8 * j;
    auto set_byte = [&](uint32_t b, uint32_t v) {
        if (b >= b0 && b < b0 + 8) {
            const uint32_t sh = 8 * (b - b0);
            w = (w & ~(0xFFull << sh)) | ((uint64_t)(v & 0xFF) << sh);
        }
    };
    if (j < 3) {  // all header fields live in the first 24 bytes
        if (hdr == PIPCK_HDR_TCP) {
            if (cls > 1) set_byte(12, 0x50);
            set_byte(16, 0);
            set_byte(17, 0);
        } else if (hdr == PIPCK_HDR_UDP) {
            if (cls > 1) {
                set_byte(4, len >> 8);
                set_byte(5, len);
            }
            set_byte(6, 0);
            set_byte(7, 0);
        } else if (hdr == PIPCK_HDR_IPV4) {
            if (cls > 1) set_byte(0, 0x45);
            set_byte(10, 0);
            set_byte(11, 0);
        }
    }
    if (b0 + 8 > len) w = b0 >= len ? 0ull : (w & ((1ull << (8 * (len - b0))) - 1ull));
    return w;
}

__device__ __forceinline__ uint32_t packet_class(uint64_t key) {
    return (uint32_t)(mix64(key ^ 0xA5A5A5A5A5A5A5A5ull) % 1000ull);
}

// One wave per packet; lanes write 8-byte words of the packet's stride slot.
__global__ __launch_bounds__(256) void k_gen_fixed(uint64_t* __restrict__ arena, uint64_t stride_words, uint32_t len,
                                                   uint64_t n, uint64_t first, uint64_t seed, uint32_t hdr) {
    const int lane = threadIdx.x & 63;
    for (uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += (uint64_t)gridDim.x * 4) {
        const uint64_t key = pkt_key(seed, first + i);
        const uint32_t cls = packet_class(key);
        uint64_t* dst = arena + i * stride_words;
        for (uint32_t j = lane; j < stride_words; j += 64) dst[j] = packet_word(key, cls, len, hdr, j);
    }
}

// Byte strides (cfg1's packed 20-B headers): one lane per byte of the slot.
__global__ __launch_bounds__(256) void k_gen_fixed_bytes(uint8_t* __restrict__ arena, uint64_t stride, uint32_t len,
                                                         uint64_t n, uint64_t first, uint64_t seed, uint32_t hdr) {
    const uint64_t total = n * stride;
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < total;
         b += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = b / stride;
        const uint32_t k = (uint32_t)(b - i * stride);
        const uint64_t key = pkt_key(seed, first + i);
        arena[b] = (uint8_t)(packet_word(key, packet_class(key), len, hdr, k / 8) >> (8 * (k % 8)));
    }
}

__global__ void k_gen_zipf(uint32_t* __restrict__ out, uint64_t n, uint64_t first, uint64_t seed,
                           const uint64_t* __restrict__ cum, uint32_t K) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t u = mix64(pkt_key(seed, first + i) ^ 0x5A5A5A5A5A5A5A5Aull) % cum[K - 1];
    uint32_t lo = 0, hi = K - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (cum[mid] > u) hi = mid; else lo = mid + 1;
    }
    out[i] = 63u + lo + 1u;
}

__global__ void k_round16(const uint32_t* __restrict__ len, uint64_t* __restrict__ r, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) r[i] = (uint64_t)((len[i] + 15u) & ~15u);
}

__global__ void k_layout(const uint32_t* __restrict__ len, const uint64_t* __restrict__ off, uint64_t n,
                         uint64_t first, uint32_t n_flows, pipck_desc* __restrict__ d) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) d[i] = pipck_desc{off[i], len[i], (uint32_t)((first + i) % n_flows)};
}

__global__ __launch_bounds__(256) void k_gen_ragged(uint8_t* __restrict__ arena, const pipck_desc* __restrict__ d,
                                                    uint64_t n, uint64_t first, uint64_t seed, uint32_t hdr) {
    const int lane = threadIdx.x & 63;
    for (uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += (uint64_t)gridDim.x * 4) {
        const pipck_desc x = d[i];
        const uint64_t key = pkt_key(seed, first + i);
        const uint32_t cls = packet_class(key);
        uint64_t* dst = reinterpret_cast<uint64_t*>(arena + x.offset);
        const uint32_t words = ((x.len + 15u) & ~15u) / 8u;  // through the 16-byte padding
        for (uint32_t j = lane; j < words; j += 64) dst[j] = packet_word(key, cls, x.len, hdr, j);
    }
}

// Byte-packed batch (pipck_checksum_packed_bytes' layout): packet i (global id
// first + i) at tile_off[i / 64] + the lengths before it in its tile, no
// padding.  One wave per tile; lanes write a packet's bytes, packet by packet.
__global__ __launch_bounds__(64) void k_gen_packedb(uint8_t* __restrict__ arena, const uint16_t* __restrict__ lens,
                                                    const uint64_t* __restrict__ tile_off, uint64_t n, uint64_t first,
                                                    uint64_t seed, uint32_t hdr) {
    const int lane = threadIdx.x;
    const uint64_t t = blockIdx.x;
    uint64_t off = tile_off[t];
    for (uint32_t k = 0; k < 64 && t * 64 + k < n; k++) {
        const uint64_t i = t * 64 + k;
        const uint32_t len = lens[i];
        const uint64_t key = pkt_key(seed, first + i);
        const uint32_t cls = packet_class(key);
        for (uint32_t b = lane; b < len; b += 64)
            arena[off + b] = (uint8_t)(packet_word(key, cls, len, hdr, b / 8) >> (8 * (b % 8)));
        off += len;
    }
}

__global__ void k_gen_flows(uint8_t* __restrict__ out, uint32_t n, uint64_t seed, uint8_t proto, int v6) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t f = mix64(seed ^ 0xF10F10F1ull ^ mix64(i));
    if (!v6) {
        pipck_flow4* r = reinterpret_cast<pipck_flow4*>(out) + i;
        r->src = (uint32_t)f;
        r->dst = (uint32_t)(f >> 32);
        r->proto = proto;
        r->pad[0] = r->pad[1] = r->pad[2] = 0;
    } else {
        pipck_flow6* r = reinterpret_cast<pipck_flow6*>(out) + i;
        for (int h = 0; h < 4; h++) {
            const uint64_t v = mix64(f + 1 + h);
            uint8_t* dst = h < 2 ? r->src + 8 * h : r->dst + 8 * (h - 2);
            for (int b = 0; b < 8; b++) dst[b] = (uint8_t)(v >> (8 * b));
        }
        r->proto = proto;
        r->pad[0] = r->pad[1] = r->pad[2] = 0;
    }
}

// Zipf cumulative weights, one device copy per device.
constexpr uint32_t kZipfK = 8937;
static std::mutex g_zipf_mu;
static std::vector<uint64_t*> g_zipf_dev(64, nullptr);

static int zipf_table(const uint64_t** out) {
    int dev = 0;
    PIPCK_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> g(g_zipf_mu);
    if ((size_t)dev >= g_zipf_dev.size()) g_zipf_dev.resize(dev + 1, nullptr);
    if (!g_zipf_dev[dev]) {
        std::vector<uint64_t> cum(kZipfK);
        uint64_t c = 0;
        for (uint32_t k = 1; k <= kZipfK; k++) cum[k - 1] = (c += (1ull << 40) / k);
        uint64_t* d = nullptr;
        PIPCK_HIP(hipMalloc(&d, kZipfK * sizeof(uint64_t)));
        PIPCK_HIP(hipMemcpy(d, cum.data(), kZipfK * sizeof(uint64_t), hipMemcpyHostToDevice));
        g_zipf_dev[dev] = d;
    }
    *out = g_zipf_dev[dev];
    return PIPCK_OK;
}

static uint32_t gen_grid(uint64_t waves) {
    uint64_t blocks = (waves + 3) / 4, cap = (uint64_t)device_cus() * 16;
    return (uint32_t)(blocks < 1 ? 1 : blocks > cap ? cap : blocks);
}

}  // namespace pipck

using namespace pipck;

extern "C" {

uint64_t pipck_cfg_seed(uint32_t cfg) { return 0x9E3779B97F4A7C15ull ^ (uint64_t)cfg; }

int pipck_gen_fixed(void* d_arena, uint64_t stride, uint32_t len, uint64_t n, uint64_t first_pkt, uint64_t seed,
                    uint32_t hdr_kind, void* stream) {
    if (!n) return PIPCK_OK;
    if (!d_arena || stride < len || stride == 0) {
        set_error("pipck_gen_fixed: null arena or stride < len");
        return PIPCK_EINVAL;
    }
    if (stride % 8 || (uintptr_t)d_arena % 8) {
        hipLaunchKernelGGL(k_gen_fixed_bytes, dim3(gen_grid((n * stride + 63) / 64)), dim3(256), 0, as_stream(stream),
                           (uint8_t*)d_arena, stride, len, n, first_pkt, seed, hdr_kind);
        PIPCK_LAUNCHED("k_gen_fixed_bytes");
        return PIPCK_OK;
    }
    hipLaunchKernelGGL(k_gen_fixed, dim3(gen_grid(n)), dim3(256), 0, as_stream(stream), (uint64_t*)d_arena, stride / 8,
                       len, n, first_pkt, seed, hdr_kind);
    PIPCK_LAUNCHED("k_gen_fixed");
    return PIPCK_OK;
}

int pipck_gen_zipf_lengths(uint32_t* d_len, uint64_t n, uint64_t first_pkt, uint64_t seed, void* stream) {
    if (!n) return PIPCK_OK;
    const uint64_t* cum = nullptr;
    int rc = zipf_table(&cum);
    if (rc) return rc;
    hipLaunchKernelGGL(k_gen_zipf, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, as_stream(stream), d_len, n,
                       first_pkt, seed, cum, kZipfK);
    PIPCK_LAUNCHED("k_gen_zipf");
    return PIPCK_OK;
}

int pipck_gen_ragged_layout(const uint32_t* d_len, uint64_t n, uint64_t first_pkt, uint32_t n_flows,
                            pipck_desc* d_desc, uint64_t* arena_bytes, void* stream) {
    if (!n) {
        if (arena_bytes) *arena_bytes = 0;
        return PIPCK_OK;
    }
    if (!d_len || !d_desc || !n_flows) {
        set_error("pipck_gen_ragged_layout: bad argument");
        return PIPCK_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    uint64_t *rounded = nullptr, *off = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    PIPCK_HIP(hipMalloc(&rounded, n * sizeof(uint64_t)));
    PIPCK_HIP(hipMalloc(&off, n * sizeof(uint64_t)));
    const uint32_t g = (uint32_t)((n + 255) / 256);
    hipLaunchKernelGGL(k_round16, dim3(g), dim3(256), 0, s, d_len, rounded, n);
    PIPCK_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, rounded, off, (int64_t)n, s));
    PIPCK_HIP(hipMalloc(&tmp, tmp_bytes));
    PIPCK_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, rounded, off, (int64_t)n, s));
    hipLaunchKernelGGL(k_layout, dim3(g), dim3(256), 0, s, d_len, off, n, first_pkt, n_flows, d_desc);
    PIPCK_LAUNCHED("k_layout");
    uint64_t last_off = 0, last_len = 0;
    PIPCK_HIP(hipMemcpyAsync(&last_off, off + n - 1, 8, hipMemcpyDeviceToHost, s));
    PIPCK_HIP(hipMemcpyAsync(&last_len, rounded + n - 1, 8, hipMemcpyDeviceToHost, s));
    PIPCK_HIP(hipStreamSynchronize(s));
    PIPCK_HIP(hipFree(tmp));
    PIPCK_HIP(hipFree(off));
    PIPCK_HIP(hipFree(rounded));
    if (arena_bytes) *arena_bytes = last_off + last_len;
    return PIPCK_OK;
}

int pipck_gen_ragged_fill(void* d_arena, const pipck_desc* d_desc, uint64_t n, uint64_t first_pkt, uint64_t seed,
                          uint32_t hdr_kind, void* stream) {
    if (!n) return PIPCK_OK;
    if (!d_arena || !d_desc || (uintptr_t)d_arena % 16) {
        set_error("pipck_gen_ragged_fill: arena must be 16-byte aligned");
        return PIPCK_EINVAL;
    }
    hipLaunchKernelGGL(k_gen_ragged, dim3(gen_grid(n)), dim3(256), 0, as_stream(stream), (uint8_t*)d_arena, d_desc, n,
                       first_pkt, seed, hdr_kind);
    PIPCK_LAUNCHED("k_gen_ragged");
    return PIPCK_OK;
}

int pipck_gen_packed_bytes(void* d_arena, const uint16_t* d_lens, const uint64_t* d_tile_off, uint64_t n,
                           uint64_t first_pkt, uint64_t seed, uint32_t hdr_kind, void* stream) {
    if (!n) return PIPCK_OK;
    if (!d_arena || !d_lens || !d_tile_off) {
        set_error("pipck_gen_packed_bytes: null pointer");
        return PIPCK_EINVAL;
    }
    hipLaunchKernelGGL(k_gen_packedb, dim3((uint32_t)((n + 63) / 64)), dim3(64), 0, as_stream(stream),
                       (uint8_t*)d_arena, d_lens, d_tile_off, n, first_pkt, seed, hdr_kind);
    PIPCK_LAUNCHED("k_gen_packedb");
    return PIPCK_OK;
}

int pipck_gen_flows4(pipck_flow4* d_flows, uint32_t n, uint64_t seed, uint8_t proto, void* stream) {
    if (!n) return PIPCK_OK;
    hipLaunchKernelGGL(k_gen_flows, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream), (uint8_t*)d_flows, n, seed,
                       proto, 0);
    PIPCK_LAUNCHED("k_gen_flows");
    return PIPCK_OK;
}

int pipck_gen_flows6(pipck_flow6* d_flows, uint32_t n, uint64_t seed, uint8_t proto, void* stream) {
    if (!n) return PIPCK_OK;
    hipLaunchKernelGGL(k_gen_flows, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream), (uint8_t*)d_flows, n, seed,
                       proto, 1);
    PIPCK_LAUNCHED("k_gen_flows");
    return PIPCK_OK;
}

}  // extern "C"
