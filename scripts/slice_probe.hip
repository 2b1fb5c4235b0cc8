// slice_probe.hip — does a per-XCD column slice of the gathered table pay, and in which layout?
// Standalone: hipcc -O3 --offload-arch=gfx950 scripts/slice_probe.hip -o /tmp/slice_probe
// FB15K shape: 14,541 rows of 128 fp32 (7.4 MB), 310,116 uniformly random entries, summed 32 at
// a time.  A: whole 512-B rows, one wave per 32 entries (float2 lanes).  Sliced variants: 4 slices
// of 32 columns, a half-wave per 32 entries (4-B lanes, two 128-B rows per load instruction),
// slice = blockIdx % 4 (one slice per XCD pair under round-robin placement) or (blockIdx / 8) % 4
// (every XCD sees every slice); the slice read from the row-major table (stride 512 B) or from a
// slice-major copy (each slice contiguous, stride 128 B).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

constexpr int F = 128;
constexpr int U = 16;

__global__ __launch_bounds__(256) void whole_rows(const float* __restrict__ x, const int* __restrict__ idx, int E,
                                                  float* out) {
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int e0 = w * 32;
    if (e0 >= E) return;
    const int n = min(32, E - e0);
    const int my = idx[e0 + min(lane, n - 1)];
    float2 acc = make_float2(0.f, 0.f);
    for (int u0 = 0; u0 < n; u0 += U) {
        float2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int r = __builtin_amdgcn_readlane(my, min(u0 + u, n - 1));
            v[u] = *reinterpret_cast<const float2*>(x + (size_t)r * F + 2 * lane);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (u0 + u < n) { acc.x += v[u].x; acc.y += v[u].y; }
    }
    *reinterpret_cast<float2*>(out + (size_t)w * F + 2 * lane) = acc;
}

// MAJOR: slice-major table; XCDAFF: slice = blockIdx % 4, else (blockIdx / 8) % 4
template <bool MAJOR, bool XCDAFF>
__global__ __launch_bounds__(256) void sliced(const float* __restrict__ x, const int* __restrict__ idx, int E, int N,
                                              float* out) {
    const int lane = threadIdx.x & 63;
    const int hb = lane & 32, fl = lane & 31;
    const int q = XCDAFF ? (int)blockIdx.x % 4 : ((int)blockIdx.x / 8) % 4;
    const int grp = XCDAFF ? (int)blockIdx.x / 4 : ((int)blockIdx.x / 32) * 8 + (int)blockIdx.x % 8;
    const int c = grp * 8 + 2 * (threadIdx.x >> 6) + (hb ? 1 : 0);
    const int e0 = c * 32;
    const int nA = max(0, min(32, E - (e0 - (hb ? 32 : 0))));
    const int n = max(0, min(32, E - e0));
    const int nmax = max(nA, max(0, min(32, E - (e0 - (hb ? 32 : 0)) - 32)));
    if (nmax <= 0) return;
    const int my = idx[min(e0 + min(fl, max(n - 1, 0)), E - 1)];
    const float* base = MAJOR ? x + (size_t)q * N * 32 : x + q * 32;
    constexpr int RS = MAJOR ? 32 : F;
    float acc = 0.f;
    for (int u0 = 0; u0 < 32; u0 += U) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int r = __shfl(my, hb + min(u0 + u, max(n - 1, 0)));
            v[u] = base[(size_t)r * RS + fl];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (u0 + u < n) acc += v[u];
    }
    if (n > 0) out[(size_t)c * F + q * 32 + fl] = acc;
}

int main() {
    const int N = 14541, E = 310116;
    std::vector<int> idx(E);
    srand(1);
    for (auto& v : idx) v = rand() % N;
    std::vector<float> hx((size_t)N * F), hm((size_t)N * F);
    for (size_t i = 0; i < hx.size(); ++i) hx[i] = (float)(i % 97) * 0.01f;
    for (int r = 0; r < N; ++r)
        for (int f = 0; f < F; ++f) hm[(size_t)(f / 32) * N * 32 + (size_t)r * 32 + f % 32] = hx[(size_t)r * F + f];
    float *x, *xm, *out;
    int* di;
    const int nch = (E + 31) / 32;
    CHECK(hipMalloc(&x, hx.size() * 4));
    CHECK(hipMalloc(&xm, hm.size() * 4));
    CHECK(hipMalloc(&out, (size_t)(nch + 8) * F * 4));
    CHECK(hipMalloc(&di, E * 4));
    CHECK(hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(xm, hm.data(), hm.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(di, idx.data(), E * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        CHECK(hipDeviceSynchronize());
        const int reps = 50;
        CHECK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) launch();
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / reps;
        printf("{\"variant\": \"%s\", \"us\": %.2f, \"gathered_TBps\": %.2f}\n", name, us, (double)E * 512 / us / 1e6);
    };
    const int nb_whole = (nch + 3) / 4;
    const int ngrp = (nch + 7) / 8;
    timeit("whole 512B rows", [&] { hipLaunchKernelGGL(whole_rows, dim3(nb_whole), dim3(256), 0, 0, x, di, E, out); });
    timeit("col slice, xcd affinity", [&] { hipLaunchKernelGGL((sliced<false, true>), dim3(4 * ngrp), dim3(256), 0, 0, x, di, E, N, out); });
    timeit("col slice, no affinity", [&] { hipLaunchKernelGGL((sliced<false, false>), dim3(((ngrp + 7) / 8) * 32), dim3(256), 0, 0, x, di, E, N, out); });
    timeit("slice-major, xcd affinity", [&] { hipLaunchKernelGGL((sliced<true, true>), dim3(4 * ngrp), dim3(256), 0, 0, xm, di, E, N, out); });
    timeit("slice-major, no affinity", [&] { hipLaunchKernelGGL((sliced<true, false>), dim3(((ngrp + 7) / 8) * 32), dim3(256), 0, 0, xm, di, E, N, out); });
    CHECK(hipDeviceSynchronize());
    return 0;
}
