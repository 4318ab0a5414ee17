// Probe: can the host write fine-grained device memory directly (large-BAR mapping)?
// If so, a per-call mailbox could live in VRAM and the device would poll it locally.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>

__global__ void k_read(const volatile unsigned* p, unsigned* out) { out[0] = p[0] + p[1]; }

int main() {
    unsigned* p = nullptr;
    hipError_t e = hipExtMallocWithFlags((void**)&p, 4096, hipDeviceMallocFinegrained);
    printf("hipExtMallocWithFlags(finegrained): %s %p\n", hipGetErrorString(e), (void*)p);
    if (e != hipSuccess) return 1;
    hipPointerAttribute_t a;
    e = hipPointerGetAttributes(&a, p);
    printf("attributes: %s type=%d hostPointer=%p devicePointer=%p\n", hipGetErrorString(e), (int)a.type, a.hostPointer,
           a.devicePointer);
    fflush(stdout);
    // host write (segfaults if the device memory is not host-mapped)
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 1000; i++) ((volatile unsigned*)p)[i & 15] = 40 + (i & 1);
    auto t1 = std::chrono::steady_clock::now();
    ((volatile unsigned*)p)[0] = 40;
    ((volatile unsigned*)p)[1] = 2;
    printf("host wrote; 1000 stores %.2f us; host read back %u\n",
           std::chrono::duration<double, std::micro>(t1 - t0).count(), ((volatile unsigned*)p)[0]);
    unsigned* d = nullptr;
    hipHostMalloc((void**)&d, 64, hipHostMallocCoherent);
    hipLaunchKernelGGL(k_read, dim3(1), dim3(1), 0, 0, p, d);
    hipDeviceSynchronize();
    printf("device read sum %u (expect 42)\n", d[0]);
    return 0;
}
