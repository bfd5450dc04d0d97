// FETCH_SIZE calibration (VERDICT r3 "What's weak" #3 / next-round #7): does
// gfx950's FETCH_SIZE counter report half the bytes of a read for narrow
// per-lane loads too, or only for 16 B/lane streaming loads (the case
// MI355X_MICROARCH.md documents)?  Each kernel reads the same 64 MiB buffer
// exactly once, coalesced, with 2, 4, 8 or 16 bytes per lane; run under
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib
// and compare each kernel's FETCH_SIZE (KB) with 65,536 KB.  k_spec-shaped:
// the 2-byte kernel is how k_spec reads its 16-bit event words.
// Build: hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

template <class T>
__global__ void k_read(const T *__restrict__ in, size_t n, unsigned long long *out) {
    unsigned long long acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const T v = in[i];
        const uint32_t *w = reinterpret_cast<const uint32_t *>(&v);
        if constexpr (sizeof(T) >= 4) {
            for (size_t k = 0; k < sizeof(T) / 4; ++k) acc += w[k];
        } else {
            acc += (unsigned long long)v;
        }
    }
    if (acc == 0x123456789ull) out[0] = acc;  // never true: keeps the loads
}

struct u2 { uint32_t x, y; };

int main() {
    const size_t bytes = 64ull << 20;
    void *buf = nullptr;
    unsigned long long *out = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 8) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, bytes);
    (void)hipDeviceSynchronize();
    const dim3 grid(4096), block(256);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_read<uint16_t>, grid, block, 0, 0, (const uint16_t *)buf, bytes / 2, out);
        hipLaunchKernelGGL(k_read<uint32_t>, grid, block, 0, 0, (const uint32_t *)buf, bytes / 4, out);
        hipLaunchKernelGGL(k_read<u2>, grid, block, 0, 0, (const u2 *)buf, bytes / 8, out);
        hipLaunchKernelGGL(k_read<uint4>, grid, block, 0, 0, (const uint4 *)buf, bytes / 16, out);
        (void)hipDeviceSynchronize();
    }
    std::printf("each kernel read %zu KB once\n", bytes / 1024);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
