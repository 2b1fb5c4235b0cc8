// mfma_probe.hip — cycles per v_mfma_f32_32x32x2_f32 in the tile GEMM's strip loop shape:
// one wave = 64 rows x 32 columns, K = 128 split across lane halves, A from LDS (ds_read_b128
// feeds four MFMAs), B per lane from global memory in chunks of 16 k (one chunk ahead).
// Variants: A_LDS (1: LDS reads, 0: constants), B_GLOBAL (1: loads, 0: constants), waves per
// SIMD (grid of 256 x WPS workgroups of 256 threads), repeated strips per wave.
// hipcc -O3 --offload-arch=gfx950 -ffp-contract=off scripts/mfma_probe.hip -o scripts/mfma_probe.bin
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

constexpr int K = 128, KH = 64, KC = 16, LDA = K + 4;

template <bool A_LDS, bool B_GLOBAL, bool ROLL>
__global__ __launch_bounds__(256) void strip(const float* __restrict__ W, int reps, float* out,
                                             unsigned long long* cyc) {
    __shared__ __attribute__((aligned(16))) float A[64 * LDA];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c = lane & 31, h = lane >> 5;
    for (int i = threadIdx.x; i < 64 * LDA; i += 256) A[i] = (float)(i % 7) * 0.1f;
    __syncthreads();
    const float* a0p = A + c * LDA + h * KH;
    const float* a1p = A + (32 + c) * LDA + h * KH;
    const int n = wave * 32 + c;
    const float* wp = W + n;  // B(k, n) = W[k * 128 + n]
    f32x16 acc0, acc1;
    for (int r = 0; r < 16; ++r) acc0[r] = acc1[r] = 0.f;
    auto load_chunk = [&](int k0, float (&o)[KC]) {
        if constexpr (B_GLOBAL) {
            const float* p = wp + (size_t)min(k0, K - KC) * 128;
#pragma unroll
            for (int j = 0; j < KC; ++j) o[j] = p[j * 128];
        } else {
#pragma unroll
            for (int j = 0; j < KC; ++j) o[j] = (float)(j + k0);
        }
    };
    float4 ca0 = *reinterpret_cast<const float4*>(a0p), ca1 = *reinterpret_cast<const float4*>(a1p);
    auto compute = [&](const float (&bc)[KC], int t) {
#pragma unroll
        for (int j = 0; j < KC; j += 4) {
            float4 x0, x1;
            if constexpr (!A_LDS) {
                x0 = make_float4(1.f, 2.f, 3.f, (float)t);
                x1 = x0;
            } else if constexpr (ROLL) {
                x0 = ca0;
                x1 = ca1;
                ca0 = *reinterpret_cast<const float4*>(a0p + t + j + 4);
                ca1 = *reinterpret_cast<const float4*>(a1p + t + j + 4);
                __builtin_amdgcn_sched_barrier(0);
            } else {
                x0 = *reinterpret_cast<const float4*>(a0p + t + j);
                x1 = *reinterpret_cast<const float4*>(a1p + t + j);
            }
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x0.x, bc[j], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(x1.x, bc[j], acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x0.y, bc[j + 1], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(x1.y, bc[j + 1], acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x0.z, bc[j + 2], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(x1.z, bc[j + 2], acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x0.w, bc[j + 3], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(x1.w, bc[j + 3], acc1, 0, 0, 0);
        }
    };
    unsigned long long t0 = 0;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    float b0[KC], b1[KC];
    const int kb = h * KH;
    load_chunk(kb, b0);
    for (int rep = 0; rep < reps; ++rep) {
        int t = 0;
#pragma unroll 1
        for (; t < KH - 2 * KC; t += 2 * KC) {
            load_chunk(kb + t + KC, b1);
            __builtin_amdgcn_sched_barrier(0);
            compute(b0, t);
            __builtin_amdgcn_sched_barrier(0);
            load_chunk(kb + t + 2 * KC, b0);
            __builtin_amdgcn_sched_barrier(0);
            compute(b1, t + KC);
            __builtin_amdgcn_sched_barrier(0);
        }
        load_chunk(kb + t + KC, b1);
        __builtin_amdgcn_sched_barrier(0);
        compute(b0, t);
        __builtin_amdgcn_sched_barrier(0);
        load_chunk(kb, b0);
        __builtin_amdgcn_sched_barrier(0);
        compute(b1, t + KC);
        __builtin_amdgcn_sched_barrier(0);
    }
    unsigned long long t1 = 0;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    float s = 0.f;
    for (int r = 0; r < 16; ++r) s += acc0[r] + acc1[r];
    if (s == 1234.5f) out[threadIdx.x] = s;
    if (lane == 0) cyc[blockIdx.x * 4 + wave] = t1 - t0;
}

template <bool A_LDS, bool B_GLOBAL, bool ROLL>
static void run(const char* name, int wps, const float* W, float* out, unsigned long long* cyc) {
    const int reps = 16;
    const int blocks = 256 * wps;
    hipLaunchKernelGGL((strip<A_LDS, B_GLOBAL, ROLL>), dim3(blocks), dim3(256), 0, 0, W, reps, out, cyc);
    CHECK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL((strip<A_LDS, B_GLOBAL, ROLL>), dim3(blocks), dim3(256), 0, 0, W, reps, out, cyc);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    unsigned long long* h = (unsigned long long*)malloc(blocks * 4 * 8);
    CHECK(hipMemcpy(h, cyc, blocks * 4 * 8, hipMemcpyDeviceToHost));
    double avg = 0;
    for (int i = 0; i < blocks * 4; ++i) avg += (double)h[i];
    avg /= blocks * 4;
    const double mfmas = 128.0 * reps;                       // per wave
    const double flops = 2.0 * 64 * 32 * K * reps * blocks * 4;  // all waves
    printf("{\"variant\": \"%s\", \"waves_per_simd\": %d, \"ticks_per_mfma\": %.1f, \"us\": %.1f, \"TFLOPs\": %.1f}\n",
           name, wps, avg / mfmas, ms * 1e3, flops / (ms * 1e-3) / 1e12);
    free(h);
}

int main() {
    float *W, *out;
    unsigned long long* cyc;
    CHECK(hipMalloc(&W, 128 * 128 * 4 * 237));
    CHECK(hipMemset(W, 0, 128 * 128 * 4 * 237));
    CHECK(hipMalloc(&out, 4096));
    CHECK(hipMalloc(&cyc, 256 * 4 * 4 * 8));
    for (int wps : {1, 2}) {
        run<false, false, false>("const A, const B", wps, W, out, cyc);
        run<true, false, false>("LDS A, const B", wps, W, out, cyc);
        run<true, false, true>("LDS A rolled, const B", wps, W, out, cyc);
        run<false, true, false>("const A, global B", wps, W, out, cyc);
        run<true, true, true>("LDS A rolled, global B", wps, W, out, cyc);
        run<true, true, false>("LDS A, global B", wps, W, out, cyc);
    }
    return 0;
}
