// gather_probe.hip — what a random 512-B row gather from a 7.4 MB table reaches on this chip.
// Standalone: hipcc -O3 --offload-arch=gfx950 scripts/gather_probe.hip -o /tmp/gather_probe
// Each wave sums C consecutive entries of a random row list (FB15K-237 shape: 14,541 rows of
// 128 fp32, 310,116 entries) and writes one row.  Variants: 8-B lanes (one row per load
// instruction) or 16-B lanes (two rows per instruction, half-waves), U loads in flight per
// lane, C entries per wave.  Prints one JSON line per variant: µs and gathered GB/s.
#include <hip/hip_runtime.h>

#include <algorithm>
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

// 8-byte lanes: lane l holds columns 2l, 2l+1 of the entry's row
template <int U>
__global__ __launch_bounds__(256) void gather8(const float* __restrict__ x, const int* __restrict__ idx, int E, int C,
                                               float* out) {
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int e0 = w * C;
    if (e0 >= E) return;
    const int e1 = min(E, e0 + C);
    float2 acc = make_float2(0.f, 0.f);
    for (int b = e0; b < e1; b += 64) {
        const int my = idx[min(b + lane, e1 - 1)];
        const int n = min(64, e1 - b);
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
                if (u0 + u < n) {
                    acc.x += v[u].x;
                    acc.y += v[u].y;
                }
        }
    }
    *reinterpret_cast<float2*>(out + (size_t)w * F + 2 * lane) = acc;
}

// 16-byte lanes: half-wave h takes entries e ≡ h (mod 2); lane holds 4 columns
template <int U>
__global__ __launch_bounds__(256) void gather16(const float* __restrict__ x, const int* __restrict__ idx, int E, int C,
                                                float* out) {
    const int lane = threadIdx.x & 63;
    const int h = lane >> 5;
    const int sl = lane & 31;
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int e0 = w * C;
    if (e0 >= E) return;
    const int e1 = min(E, e0 + C);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int b = e0; b < e1; b += 64) {
        const int my = idx[min(b + lane, e1 - 1)];
        const int n = min(64, e1 - b);
        for (int u0 = 0; u0 < n; u0 += 2 * U) {
            float4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int q = min(u0 + 2 * u + h, n - 1);
                const int r = __shfl(my, q);
                v[u] = *reinterpret_cast<const float4*>(x + (size_t)r * F + 4 * sl);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (u0 + 2 * u + h < n) {
                    acc.x += v[u].x;
                    acc.y += v[u].y;
                    acc.z += v[u].z;
                    acc.w += v[u].w;
                }
        }
    }
    acc.x += __shfl_xor(acc.x, 32);
    acc.y += __shfl_xor(acc.y, 32);
    acc.z += __shfl_xor(acc.z, 32);
    acc.w += __shfl_xor(acc.w, 32);
    if (h == 0) *reinterpret_cast<float4*>(out + (size_t)w * F + 4 * sl) = acc;
}


// Segmented flat gather over FB15K's real segment table: chunk c covers positions
// [cp[c], cp[c+1]) (<= 64, cut at segment ends unless a segment is longer than 64); a row
// complete inside the chunk is written as mean; a split row's partial goes to a carry slot.
template <int U>
__global__ __launch_bounds__(256) void seg_flat(const float* __restrict__ x, const int* __restrict__ e_col,
                                                const int* __restrict__ seg_of, const int* __restrict__ cp,
                                                const int* __restrict__ s_ptr, const int* __restrict__ s_cnt, int nch,
                                                float* out, float* carry) {
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= nch) return;
    const int p0 = cp[c], p1 = cp[c + 1];
    const int n = p1 - p0;
    const int pq = p0 + min(lane, n - 1);
    const int my = e_col[pq];
    const int myrow = seg_of[pq];
    const int nextrow = __shfl_down(myrow, 1);
    const bool last = lane == n - 1 || (lane < n - 1 && nextrow != myrow);
    const unsigned long long lastm = __ballot(last && lane < n);
    // per-row completeness: row starts at/after p0 and ends at/before p1
    const int rs = s_ptr[myrow], re = s_ptr[myrow + 1];
    const bool complete = rs >= p0 && re <= p1;
    const unsigned long long compm = __ballot(complete);
    const float cntf = (float)s_cnt[myrow];
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
        for (int u = 0; u < U; ++u) {
            const int q = u0 + u;
            if (q < n) {
                acc.x += v[u].x;
                acc.y += v[u].y;
                if ((lastm >> q) & 1ull) {
                    const int row = __builtin_amdgcn_readlane(myrow, q);
                    if ((compm >> q) & 1ull) {
                        const float d = __shfl(cntf, q);
                        *reinterpret_cast<float2*>(out + (size_t)row * F + 2 * lane) = make_float2(acc.x / d, acc.y / d);
                    } else {
                        *reinterpret_cast<float2*>(carry + ((size_t)2 * c + (q == n - 1 ? 1 : 0)) * F + 2 * lane) = acc;
                    }
                    acc = make_float2(0.f, 0.f);
                }
            }
        }
    }
}

// as seg_flat, without dependent metadata loads: a complete row's count is its entry span in
// the chunk; whether the chunk's first / last row is split comes with the chunk (flags)
template <int U>
__global__ __launch_bounds__(256) void seg_flat2(const float* __restrict__ x, const int* __restrict__ e_col,
                                                 const int* __restrict__ seg_of, const int* __restrict__ cp,
                                                 const int* __restrict__ cflags, const int* __restrict__ unused, int nch,
                                                 float* out, float* carry) {
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= nch) return;
    const int p0 = cp[c], p1 = cp[c + 1];
    const int fl = cflags[c];  // bit0: first row split, bit1: last row split
    const int mode = unused[0];   // probe bits: 1 no division, 2 no row stores
    const int n = p1 - p0;
    const int pq = p0 + min(lane, n - 1);
    const int my = e_col[pq];
    const int myrow = seg_of[pq];
    const int prevrow = __shfl_up(myrow, 1);
    const int nextrow = __shfl_down(myrow, 1);
    const bool first = lane == 0 || prevrow != myrow;
    const bool last = lane == n - 1 || (lane < n - 1 && nextrow != myrow);
    const unsigned long long lastm = __ballot(last && lane < n);
    const unsigned long long firstm = __ballot(first && lane < n);
    const int row0 = __builtin_amdgcn_readlane(myrow, 0);
    const int rowl = __builtin_amdgcn_readlane(myrow, n - 1);
    float2 acc = make_float2(0.f, 0.f);
    int qstart = 0;
    for (int u0 = 0; u0 < n; u0 += U) {
        float2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int r = __builtin_amdgcn_readlane(my, min(u0 + u, n - 1));
            v[u] = *reinterpret_cast<const float2*>(x + (size_t)r * F + 2 * lane);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int q = u0 + u;
            if (q < n) {
                if ((firstm >> q) & 1ull) qstart = q;
                acc.x += v[u].x;
                acc.y += v[u].y;
                if ((lastm >> q) & 1ull) {
                    const int row = __builtin_amdgcn_readlane(myrow, q);
                    const bool split = (row == row0 && (fl & 1)) || (row == rowl && (fl & 2));
                    if (!split) {
                        const float d = (float)(q - qstart + 1);
                        const float2 val = (mode & 1) ? acc : make_float2(acc.x / d, acc.y / d);
                        if (!(mode & 2) || val.x == 1234.5f)
                            *reinterpret_cast<float2*>(out + (size_t)row * F + 2 * lane) = val;
                    } else {
                        *reinterpret_cast<float2*>(carry + ((size_t)2 * c + (q == n - 1 ? 1 : 0)) * F + 2 * lane) = acc;
                    }
                    acc = make_float2(0.f, 0.f);
                }
            }
        }
    }
}

template <class K>
static void run(const char* name, K kern, int U, int C, const float* x, const int* idx, int E, float* out, int N) {
    const int waves = (E + C - 1) / C;
    const int blocks = (waves + 3) / 4;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, x, idx, E, C, out);
    CHECK(hipDeviceSynchronize());
    const int iters = 20;
    CHECK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, x, idx, E, C, out);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / iters;
    printf("{\"kernel\": \"%s\", \"U\": %d, \"C\": %d, \"waves\": %d, \"us\": %.2f, \"GBps\": %.0f}\n", name, U, C, waves,
           us, (double)E * F * 4 / (us * 1e-6) / 1e9);
    (void)N;
}

int main(int argc, char** argv) {
    const int N = 14541, E = 310116;
    const int sorted = argc > 1 ? atoi(argv[1]) : 0;
    std::vector<float> hx((size_t)N * F);
    std::vector<int> hi(E);
    srand(1);
    for (auto& v : hx) v = (float)rand() / RAND_MAX;
    for (auto& v : hi) v = rand() % N;
    if (sorted) {  // entries of a segment are unrelated rows anyway; sort within 64-entry blocks
        for (int b = 0; b < E; b += 64) {
            const int e = b + 64 < E ? b + 64 : E;
            std::vector<int> t(hi.begin() + b, hi.begin() + e);
            std::sort(t.begin(), t.end());
            std::copy(t.begin(), t.end(), hi.begin() + b);
        }
    }
    float *x, *out;
    int* idx;
    CHECK(hipMalloc(&x, hx.size() * 4));
    CHECK(hipMalloc(&idx, hi.size() * 4));
    CHECK(hipMalloc(&out, (size_t)E * F * 4));
    CHECK(hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(idx, hi.data(), hi.size() * 4, hipMemcpyHostToDevice));
    for (int C : {16, 32, 64, 128}) {
        run("gather8_U8", gather8<8>, 8, C, x, idx, E, out, N);
        run("gather8_U16", gather8<16>, 16, C, x, idx, E, out, N);
        run("gather8_U32", gather8<32>, 32, C, x, idx, E, out, N);
        run("gather16_U8", gather16<8>, 8, C, x, idx, E, out, N);
        run("gather16_U16", gather16<16>, 16, C, x, idx, E, out, N);
    }
    // ---- segmented variants on FB15K's real segment table (scripts/fb_seg.bin) ----
    FILE* f = fopen("scripts/fb_seg.bin", "rb");
    if (f) {
        int hdr[3];
        if (fread(hdr, 4, 3, f) != 3) return 1;
        const int S = hdr[0], E2 = hdr[1];
        std::vector<int> s_ptr(S + 1), e_col(E2), s_cnt(S);
        if (fread(s_ptr.data(), 4, S + 1, f) != (size_t)S + 1 || fread(e_col.data(), 4, E2, f) != (size_t)E2 ||
            fread(s_cnt.data(), 4, S, f) != (size_t)S)
            return 1;
        fclose(f);
        std::vector<int> seg_of(E2);
        for (int sgi = 0; sgi < S; ++sgi)
            for (int p = s_ptr[sgi]; p < s_ptr[sgi + 1]; ++p) seg_of[p] = sgi;
        for (int C : {32, 64}) {
            std::vector<int> cp{0};
            int p = 0;
            while (p < E2) {  // greedy: whole segments up to C positions; long segments cut
                int q = p;
                int sgi = seg_of[p];
                while (q < E2) {
                    const int end = s_ptr[seg_of[q] + 1];
                    if (end - p <= C) q = end;
                    else {
                        if (q == p) q = std::min(p + C, end);  // long segment: cut
                        break;
                    }
                }
                (void)sgi;
                cp.push_back(q);
                p = q;
            }
            const int nch = (int)cp.size() - 1;
            int *d_ecol, *d_seg, *d_cp, *d_sptr, *d_cnt;
            float* carry;
            CHECK(hipMalloc(&d_ecol, E2 * 4));
            CHECK(hipMalloc(&d_seg, E2 * 4));
            CHECK(hipMalloc(&d_cp, (nch + 1) * 4));
            CHECK(hipMalloc(&d_sptr, (std::max(S, nch) + 1) * 4));
            CHECK(hipMalloc(&d_cnt, S * 4));
            CHECK(hipMalloc(&carry, (size_t)2 * nch * F * 4));
            CHECK(hipMemcpy(d_ecol, e_col.data(), E2 * 4, hipMemcpyHostToDevice));
            CHECK(hipMemcpy(d_seg, seg_of.data(), E2 * 4, hipMemcpyHostToDevice));
            CHECK(hipMemcpy(d_cp, cp.data(), (nch + 1) * 4, hipMemcpyHostToDevice));
            CHECK(hipMemcpy(d_sptr, s_ptr.data(), (S + 1) * 4, hipMemcpyHostToDevice));
            CHECK(hipMemcpy(d_cnt, s_cnt.data(), S * 4, hipMemcpyHostToDevice));
            auto go = [&](auto kern, const char* name, int U) {
                const int blocks = (nch + 3) / 4;
                hipEvent_t a, b;
                CHECK(hipEventCreate(&a));
                CHECK(hipEventCreate(&b));
                for (int i = 0; i < 3; ++i)
                    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, x, d_ecol, d_seg, d_cp, d_sptr, d_cnt, nch, out, carry);
                CHECK(hipDeviceSynchronize());
                (void)0;
                CHECK(hipEventRecord(a));
                for (int i = 0; i < 20; ++i)
                    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, x, d_ecol, d_seg, d_cp, d_sptr, d_cnt, nch, out, carry);
                CHECK(hipEventRecord(b));
                CHECK(hipEventSynchronize(b));
                float ms = 0;
                CHECK(hipEventElapsedTime(&ms, a, b));
                const double us = ms * 1e3 / 20;
                printf("{\"kernel\": \"%s\", \"U\": %d, \"C\": %d, \"chunks\": %d, \"us\": %.2f, \"GBps\": %.0f}\n", name, U,
                       C, nch, us, (double)E2 * F * 4 / (us * 1e-6) / 1e9);
            };
            go(seg_flat<8>, "seg_flat_U8", 8);
            go(seg_flat<16>, "seg_flat_U16", 16);
            std::vector<int> fl(nch);
            for (int k = 0; k < nch; ++k) {
                const int a0 = cp[k], a1 = cp[k + 1];
                fl[k] = (s_ptr[seg_of[a0]] < a0 ? 1 : 0) | (s_ptr[seg_of[a1 - 1] + 1] > a1 ? 2 : 0);
            }
            CHECK(hipMemcpy(d_sptr, fl.data(), nch * 4, hipMemcpyHostToDevice));  // reuse as flags
            for (int mode : {0, 1, 2, 3}) {
                CHECK(hipMemcpy(d_cnt, &mode, 4, hipMemcpyHostToDevice));
                char nm[64];
                snprintf(nm, sizeof nm, "seg_flat2_U16_mode%d", mode);
                go(seg_flat2<16>, nm, 16);
            }
        }
    }
    return 0;
}
