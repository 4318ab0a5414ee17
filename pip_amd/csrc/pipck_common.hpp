// pipck_common.hpp -- host-side plumbing shared by the libpipck.so sources.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <memory>
#include <string>

#include "../../include/pipck.h"
#include "pipck_testing.h"

namespace pipck {

void set_error(const std::string& msg);

// Map a HIP failure to PIPCK_EHIP with a message naming the call site.
inline int hip_fail(hipError_t e, const char* what) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return PIPCK_EHIP;
}

#define PIPCK_HIP(call)                                   \
    do {                                                  \
        hipError_t e_ = (call);                           \
        if (e_ != hipSuccess) return ::pipck::hip_fail(e_, #call); \
    } while (0)

// After a kernel launch: report launch-configuration errors synchronously.
#define PIPCK_LAUNCHED(name)                              \
    do {                                                  \
        hipError_t e_ = hipGetLastError();                \
        if (e_ != hipSuccess) return ::pipck::hip_fail(e_, name); \
    } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// The batch kernel this thread launched last (its host-side handle), so a
// measurement can name the exact template instantiation it timed
// (pipck_last_launch in pipck_testing.h: bench.py binds a PMC traffic file to
// that name).  One thread-local store per launch.
extern thread_local const void* t_last_kernel;
#define PIPCK_LAUNCH(K, ...)                                          \
    do {                                                              \
        ::pipck::t_last_kernel = reinterpret_cast<const void*>(K);    \
        hipLaunchKernelGGL(K, __VA_ARGS__);                           \
    } while (0)

// Number of CUs on the current device (cached per device).
int device_cus();

// Registry of the pinned host ranges the GPU may read in place (made by
// pipck_host_alloc / pipck_host_register).  Zero-copy TX segments are checked
// against it at add time: a kernel touching an unpinned host page would fault
// the GPU, so a bad pointer must fail as PIPCK_EINVAL instead.  A queue that
// records a segment for an in-place read also HOLDS the segment's range until
// that batch completes: pipck_host_free / pipck_host_unregister refuse a held
// range (PIPCK_EBUSY), so no range can be released while the GPU may read it.
struct PinnedRec {
    uintptr_t lo = 0, hi = 0;  // [lo, hi)
    // holders in the low bits, kPinnedRemoved once released: one atomic word,
    // so "acquire unless removed" and "remove unless held" cannot interleave
    std::atomic<uint64_t> state{0};
};
constexpr uint64_t kPinnedRemoved = 1ull << 63;
using PinnedRef = std::shared_ptr<PinnedRec>;
void pinned_add(const void* p, size_t bytes);
// PIPCK_OK, PIPCK_EINVAL (not a range start) or PIPCK_EBUSY (held by a queued batch)
int pinned_remove(const void* p);
// The range holding all of [p, p+len), or null.
PinnedRef pinned_lookup(const void* p, size_t len);
// Take / drop one hold; acquire fails once the range has been removed.
bool pinned_acquire(PinnedRec& r);
void pinned_release(PinnedRec& r);

// pipck_checksum_chains without argument checks, for callers whose segment
// descriptors hold absolute device-accessible addresses (d_arena == nullptr):
// the TX queue mixes its device staging copy with zero-copy pinned host segments.
int chains_unchecked(const void* d_arena, const pipck_desc* d_segs, uint64_t n_segs, const uint64_t* d_seg_begin,
                     const uint32_t* d_pkt_flow, uint64_t n_packets, const uint32_t* d_pseudo, uint32_t* d_scratch,
                     uint16_t* d_out, uint32_t* d_err, hipStream_t s, uint64_t arena_bytes = UINT64_MAX,
                     uint32_t n_flows = UINT32_MAX);

// The block-cooperative flat stream (pipck_coop.hip); PIPCK_EINVAL when the
// shape does not fit its block tasks (the caller then takes k_flat).
int launch_flat_coop(bool verify, const void* d_arena, uint64_t stride, uint32_t len, uint64_t n,
                     const uint32_t* d_pseudo, uint32_t n_flows, const uint32_t* d_flow_of, uint64_t flow_origin,
                     uint16_t* d_out, uint8_t* d_ok, uint32_t* d_err, hipStream_t s, uint32_t rows_per_wave,
                     uint32_t ring, uint32_t kflags);

// The header row stream (pipck_hdr.hip): 20/24-byte strides, no pseudo-header;
// PIPCK_EINVAL when the shape does not fit (the caller then takes k_small).
int launch_hdr(bool verify, const void* d_arena, uint64_t stride, uint32_t len, uint64_t n, uint16_t* d_out,
               uint8_t* d_ok, hipStream_t s, uint32_t rows, uint32_t ring, bool nt, uint32_t kflags, bool coop = false);

// pipck_rx_verify_device (pipck_packedb.hip): k_packedb with the RX verdicts.
int launch_ring_rx(const void* d_arena, uint64_t stride, const uint16_t* d_lens, uint64_t n, uint8_t* d_ok,
                   uint32_t* d_err, hipStream_t s);
int launch_packedb_rx(const void* d_arena, uint64_t arena_bytes, const uint16_t* d_lens, const uint64_t* d_tile_off,
                      uint64_t n, uint8_t* d_ok, uint32_t* d_err, hipStream_t s);

// The one-packet-per-wave measurement arm (pipck_wave.hip; pipck_tune
// lanes_per_packet == kWaveArm): fixed strides (desc == false) or descriptors.
constexpr uint32_t kWaveArm = 256;
bool wave_arm();  // pipck_tune(kWaveArm, ...) is in force (pipck_kernels.hip)
bool alt_schedule();  // pipck_tune flag bit 28 (the other schedule) is set
uint32_t g_tune_flags();  // pipck_tune's flags / loads_per_lane in force
uint32_t g_tune_loads();
uint32_t g_tune_blocks();
// measurement-only probes that change results (pipck_tune_probes, pipck_testing.h)
constexpr uint32_t kProbeHdrInPlace = 1u;
extern std::atomic<uint32_t> g_probes;
int launch_wave(bool verify, bool desc, const void* d_arena, uint64_t stride, uint32_t len, const pipck_desc* d_desc,
                uint64_t n, const uint32_t* d_pseudo, uint32_t n_flows, const uint32_t* d_flow_of,
                uint64_t flow_origin, uint16_t* d_out, uint8_t* d_ok, uint32_t* d_err, hipStream_t s,
                uint32_t max_chunks, uint32_t nl, uint64_t arena_bytes = UINT64_MAX);

}  // namespace pipck
