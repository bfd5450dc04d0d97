// Host-memory probe for lc_pack's output arrays (round 5): what a fresh
// page-locked block of a C3-sized event array costs -- hipHostMalloc, against
// malloc'd (2 MB-aligned, transparent-huge-page) memory first touched by 16
// threads and then registered with hipHostRegister -- and the H2D copy rate
// from each.  Usage: pin_probe [MB]
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

static void touch(char *p, size_t n, int nt) {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([=] { std::memset(p + n * t / nt, 1, n * (t + 1) / nt - n * t / nt); });
    for (auto &x : th) x.join();
}

int main(int argc, char **argv) {
    const size_t mb = argc > 1 ? (size_t)atol(argv[1]) : 660;
    const size_t n = mb << 20;
    void *d = nullptr;
    if (hipMalloc(&d, n) != hipSuccess) return 1;
    (void)hipFree(nullptr);
    auto h2d = [&](void *src) {
        (void)hipMemcpy(d, src, n, hipMemcpyHostToDevice);
        auto t = std::chrono::steady_clock::now();
        for (int i = 0; i < 3; ++i) (void)hipMemcpy(d, src, n, hipMemcpyHostToDevice);
        return 3.0 * n / (ms_since(t) * 1e-3) / 1e9;
    };
    auto t = std::chrono::steady_clock::now();
    void *a = nullptr;
    if (hipHostMalloc(&a, n, hipHostMallocDefault) != hipSuccess) return 2;
    const double t_hm = ms_since(t);
    t = std::chrono::steady_clock::now();
    touch((char *)a, n, 16);
    const double t_hm_touch = ms_since(t);
    const double r_hm = h2d(a);
    t = std::chrono::steady_clock::now();
    void *b = nullptr;
    if (posix_memalign(&b, 2u << 20, n)) return 3;
    madvise(b, n, MADV_HUGEPAGE);
    touch((char *)b, n, 16);
    const double t_touch = ms_since(t);
    t = std::chrono::steady_clock::now();
    const hipError_t e = hipHostRegister(b, n, hipHostRegisterDefault);
    const double t_reg = ms_since(t);
    const double r_reg = e == hipSuccess ? h2d(b) : 0.0;
    (void)hipHostUnregister(b);
    const double r_page = h2d(b);
    printf("{\"mb\": %zu, \"hipHostMalloc_ms\": %.1f, \"hipHostMalloc_touch16_ms\": %.1f, \"h2d_hostmalloc_gbs\": %.1f, "
           "\"thp_malloc_touch16_ms\": %.1f, \"hipHostRegister_ms\": %.1f, \"register_ok\": %d, \"h2d_registered_gbs\": %.1f, "
           "\"h2d_pageable_gbs\": %.1f}\n", mb, t_hm, t_hm_touch, r_hm, t_touch, t_reg, e == hipSuccess, r_reg, r_page);
    return 0;
}
