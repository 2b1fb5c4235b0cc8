// Probe: internal accumulation precision of v_mfma_f32_32x32x16_bf16 on gfx950.
// Decides whether a 3-way bf16 split of fp32 operands (6 partial products) reproduces fp32
// GEMM accuracy: each bf16 x bf16 product is exact in fp32; what matters is whether the 16
// products of one instruction (plus C) are summed with one rounding or with one per add.
// Case 1: C = 0, a0*b0 = 1, 15 products of 2^-25:   exact sum 1 + 15·2^-25 -> fp32 1 + 4·2^-23
//         (sequential fp32 adds from the big term: 1.0).
// Case 2: C = 1, 16 products of 2^-25:               exact 1 + 2^-21 (representable); sequential: 1.0
// Case 3: C = 0, the big term LAST (k = 15).
// Build: hipcc --offload-arch=gfx950 -O2 -o /tmp/mfma_bf16_probe scripts/mfma_bf16_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __bf16 to_bf16(float f) {  // exact for the powers of two used here
    unsigned u = __float_as_uint(f);
    unsigned short h = (unsigned short)(u >> 16);
    __bf16 r;
    __builtin_memcpy(&r, &h, 2);
    return r;
}

__global__ void probe(const float* A, const float* B, float c0, float* out) {
    // A [32][16] row-major, B [16][32] row-major; lane l: A row l%32, k = 8(l/32)..+8; B col l%32
    const int l = threadIdx.x;
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) {
        const int k = 8 * (l >> 5) + j;
        a[j] = to_bf16(A[(l & 31) * 16 + k]);
        b[j] = to_bf16(B[k * 32 + (l & 31)]);
    }
    f32x16 acc;
    for (int r = 0; r < 16; ++r) acc[r] = c0;
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
    for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
        out[row * 32 + (l & 31)] = acc[r];
    }
}

static void run(const char* name, int big_k, float c0, int nsmall) {
    float hA[32 * 16] = {0}, hB[16 * 32] = {0}, hO[32 * 32];
    for (int k = 0; k < 16; ++k) {
        if (k == big_k) {
            hA[k] = 1.0f;
            hB[k * 32] = 1.0f;
        } else if (nsmall-- > 0) {
            hA[k] = 1.0f / 8192.0f;     // 2^-13
            hB[k * 32] = 1.0f / 4096.0f;  // 2^-12
        }
    }
    float *dA, *dB, *dO;
    hipMalloc(&dA, sizeof hA);
    hipMalloc(&dB, sizeof hB);
    hipMalloc(&dO, sizeof hO);
    hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, c0, dO);
    hipMemcpy(hO, dO, sizeof hO, hipMemcpyDeviceToHost);
    const double v = hO[0];
    printf("%s: D[0][0] = %.10g = 1 + %.4f * 2^-23\n", name, v, (v - 1.0) * 8388608.0);
    hipFree(dA);
    hipFree(dB);
    hipFree(dO);
}

int main() {
    run("case1 C=0, big first, 15 x 2^-25 (exact: 1 + 4*2^-23, sequential: 1)", 0, 0.0f, 15);
    run("case2 C=1, 16 x 2^-25 (exact: 1 + 4*2^-23, sequential: 1)", -1, 1.0f, 16);
    run("case3 C=0, big last, 15 x 2^-25 (exact: 1 + 4*2^-23)", 15, 0.0f, 15);
    run("case4 C=0, big first, 3 x 2^-25 (exact 1 + 0.75*2^-23 -> 1 + 1*2^-23)", 0, 0.0f, 3);
    return 0;
}
