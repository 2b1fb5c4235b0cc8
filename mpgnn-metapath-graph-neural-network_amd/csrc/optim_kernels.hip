// The loops' optimizer step (main.py:1119 / main_rgcn.py:454: Adam(lr=0.01, weight_decay=5e-4))
// as one launch over every parameter tensor.
//
// torch.optim.Adam(fused=True) issues two multi-tensor launches per step: _foreach_add_ of the
// step counters and _fused_adam_, whose grid is one 512-thread block per 65,536-element chunk
// (C3's Net: 7.8 M floats -> ~120 blocks on a 256-CU chip, ~4 TB/s). Here the update is the
// same arithmetic — ATen's adam_math (ATen/native/hip/fused_adam_utils.cuh, the published
// header shipped with torch): L2 weight decay folded into the gradient, the moments in double
// rounded to float, the bias corrections from the incremented float step in double — over a
// grid of ~4 workgroups per CU with float4 accesses, and the step counters are incremented by
// the last workgroup to finish (each workgroup reads them first), so one launch replaces both.
// HBM-bound: 28 B read + 12 B written per parameter.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>

#include "mpgnn_rgcn.h"

namespace mpgnn {
namespace {

constexpr int kAdamThreads = 256;
constexpr int kAdamMax = 24;  // tensors per launch (kernel arguments by value, ~1.5 KB)

struct AdamList {
    int n;
    int64_t off4[kAdamMax + 1];  // tensor t owns float4 slots [off4[t], off4[t + 1])
    int64_t numel[kAdamMax];
    float* p[kAdamMax];
    const float* g[kAdamMax];
    float* m[kAdamMax];
    float* v[kAdamMax];
    float* step[kAdamMax];
};

// One element of ATen's adam_math<float, float, 4, ORIGINAL, false> (no grad scale, no
// maximize). CONTRACT = 1: the double-precision multiply-adds fused as clang's default HIP
// contraction (-ffp-contract=fast-honor-pragmas: the left product of a + b·c ... is the fma
// operand) forms them; 0: every product rounded. Which one torch's build matches is pinned by
// tests/test_gpu_parity.py::test_adam_step_bit_identical_to_torch (option MPGNN_OPT_ADAM_CONTRACT).
template <int CONTRACT>
__device__ __forceinline__ void adam_elem(float& param, float grad, float& ea, float& eas, double lr, double b1,
                                          double b2, double wd, double eps, float bc1, float bc2s) {
    if (wd != 0.0) {  // grad += param * weight_decay (float += double)
        grad = CONTRACT ? (float)__builtin_fma((double)param, wd, (double)grad)
                        : (float)((double)grad + (double)param * wd);
    }
    // exp_avg = beta1 * exp_avg + (1 - beta1) * grad
    ea = CONTRACT ? (float)__builtin_fma(b1, (double)ea, (1.0 - b1) * (double)grad)
                  : (float)(b1 * (double)ea + (1.0 - b1) * (double)grad);
    // exp_avg_sq = beta2 * exp_avg_sq + (1 - beta2) * grad * grad
    eas = CONTRACT ? (float)__builtin_fma(b2, (double)eas, ((1.0 - b2) * (double)grad) * (double)grad)
                   : (float)(b2 * (double)eas + ((1.0 - b2) * (double)grad) * (double)grad);
    const float step_size = (float)(lr / (double)bc1);
    const float denom = (float)((double)(sqrtf(eas) / bc2s) + eps);
    param = param - (step_size * ea) / denom;
}

constexpr int kAdamU = 4;  // float4 slots per thread in flight (their loads issued together)

template <int CONTRACT>
__global__ __launch_bounds__(kAdamThreads) void adam_step_kernel(AdamList L, double lr, double b1, double b2,
                                                                  double wd, double eps, int64_t per_block,
                                                                  int* arrive) {
    // the tensor table in LDS (a thread's slot -> tensor lookup and its pointers without a
    // dependent global load per slot), with each tensor's bias corrections
    __shared__ int64_t s_off[kAdamMax + 1], s_numel[kAdamMax];
    __shared__ float* s_ptr[4][kAdamMax];
    __shared__ float s_bc1[kAdamMax], s_bc2s[kAdamMax];
    const int tid = threadIdx.x;
    if (tid < L.n) {
        // the step this update uses: _foreach_add_(steps, 1) in float, then ATen's
        // 1 - pow(beta, step) in double, handed to adam_math as float
        const float st = *L.step[tid] + 1.0f;
        const double bc1 = 1.0 - ::pow(b1, (double)st);
        const double bc2 = 1.0 - ::pow(b2, (double)st);
        s_bc1[tid] = (float)bc1;
        s_bc2s[tid] = (float)::sqrt(bc2);
        s_numel[tid] = L.numel[tid];
        s_ptr[0][tid] = L.p[tid];
        s_ptr[1][tid] = const_cast<float*>(L.g[tid]);
        s_ptr[2][tid] = L.m[tid];
        s_ptr[3][tid] = L.v[tid];
    }
    if (tid <= L.n) s_off[tid] = L.off4[tid];
    __syncthreads();
    const int n = L.n;
    const int64_t beg = (int64_t)blockIdx.x * per_block;
    const int64_t end = min(beg + per_block, s_off[n]);
    int t = 0;
    for (int64_t s0 = beg + tid; s0 < end; s0 += kAdamThreads * kAdamU) {
        int tu[kAdamU];
        int64_t e0[kAdamU];
        bool full[kAdamU];
        float4 p[kAdamU], g[kAdamU], m[kAdamU], v[kAdamU];
#pragma unroll
        for (int u = 0; u < kAdamU; ++u) {
            const int64_t s = s0 + (int64_t)u * kAdamThreads;
            tu[u] = -1;
            full[u] = false;
            if (s < end) {
                while (s >= s_off[t + 1]) ++t;
                tu[u] = t;
                e0[u] = (s - s_off[t]) * 4;
                full[u] = s_numel[t] - e0[u] >= 4;
                if (full[u]) {
                    p[u] = *reinterpret_cast<const float4*>(s_ptr[0][t] + e0[u]);
                    g[u] = *reinterpret_cast<const float4*>(s_ptr[1][t] + e0[u]);
                    m[u] = *reinterpret_cast<const float4*>(s_ptr[2][t] + e0[u]);
                    v[u] = *reinterpret_cast<const float4*>(s_ptr[3][t] + e0[u]);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kAdamU; ++u) {
            const int k = tu[u];
            if (k < 0) continue;
            const float bc1 = s_bc1[k], bc2s = s_bc2s[k];
            if (full[u]) {
                adam_elem<CONTRACT>(p[u].x, g[u].x, m[u].x, v[u].x, lr, b1, b2, wd, eps, bc1, bc2s);
                adam_elem<CONTRACT>(p[u].y, g[u].y, m[u].y, v[u].y, lr, b1, b2, wd, eps, bc1, bc2s);
                adam_elem<CONTRACT>(p[u].z, g[u].z, m[u].z, v[u].z, lr, b1, b2, wd, eps, bc1, bc2s);
                adam_elem<CONTRACT>(p[u].w, g[u].w, m[u].w, v[u].w, lr, b1, b2, wd, eps, bc1, bc2s);
                *reinterpret_cast<float4*>(s_ptr[0][k] + e0[u]) = p[u];
                *reinterpret_cast<float4*>(s_ptr[2][k] + e0[u]) = m[u];
                *reinterpret_cast<float4*>(s_ptr[3][k] + e0[u]) = v[u];
            } else {  // a tensor's last 1-3 elements
                float* P = s_ptr[0][k];
                const float* G = s_ptr[1][k];
                float* M = s_ptr[2][k];
                float* Q = s_ptr[3][k];
                for (int64_t e = e0[u]; e < s_numel[k]; ++e) {
                    float pe = P[e], me = M[e], ve = Q[e];
                    adam_elem<CONTRACT>(pe, G[e], me, ve, lr, b1, b2, wd, eps, bc1, bc2s);
                    P[e] = pe;
                    M[e] = me;
                    Q[e] = ve;
                }
            }
        }
    }
    // the last workgroup to finish increments the step counters and re-arms the arrival counter.
    // Every workgroup's reads of the counters (above) returned before its arrival, so no fence is
    // needed (a release fence per workgroup would write back the XCD's L2 each time).
    if (tid == 0) {
        const int prev = (int)__hip_atomic_fetch_add(reinterpret_cast<unsigned*>(arrive), 1u, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
        if (prev == (int)gridDim.x - 1) {
            for (int k = 0; k < n; ++k) *L.step[k] = *L.step[k] + 1.0f;
            __hip_atomic_store(arrive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

int g_adam_contract = 1;

}  // namespace

int adam_contract_get() { return g_adam_contract; }
void adam_contract_set(int v) { g_adam_contract = v ? 1 : 0; }

}  // namespace mpgnn

extern "C" int32_t mpgnn_adam_step(const mpgnn_adam_tensor* tensors, int32_t n, double lr, double beta1, double beta2,
                                   double weight_decay, double eps, int32_t* arrive, void* stream) {
    using namespace mpgnn;
    if (n < 0 || (n > 0 && (tensors == nullptr || arrive == nullptr))) return MPGNN_ERR_ARG;
    if (n > kAdamMax) return MPGNN_ERR_UNSUPPORTED;
    if (n == 0) return MPGNN_OK;
    AdamList L{};
    L.n = n;
    int64_t slots = 0;
    for (int k = 0; k < n; ++k) {
        const mpgnn_adam_tensor& a = tensors[k];
        if (a.numel < 0 || (a.numel > 0 && (!a.param || !a.grad || !a.exp_avg || !a.exp_avg_sq)) || !a.step)
            return MPGNN_ERR_ARG;
        for (const void* q : {(const void*)a.param, (const void*)a.grad, (const void*)a.exp_avg,
                              (const void*)a.exp_avg_sq})
            if (reinterpret_cast<uintptr_t>(q) % 16) return MPGNN_ERR_UNSUPPORTED;
        L.off4[k] = slots;
        L.numel[k] = a.numel;
        L.p[k] = a.param;
        L.g[k] = a.grad;
        L.m[k] = a.exp_avg;
        L.v[k] = a.exp_avg_sq;
        L.step[k] = a.step;
        slots += (a.numel + 3) / 4;
    }
    L.off4[n] = slots;
    hipStream_t strm = static_cast<hipStream_t>(stream);
    // each workgroup a contiguous run of float4 slots, kAdamU per thread in flight
    const int64_t unit = (int64_t)kAdamThreads * kAdamU;
    // ~1024 workgroups (4 per CU): C3's Net (7.8 M floats) 43.3 µs = 5.0 TB/s of its 218 MB, against
    // 53.3 / 44.2 / 46.7 / 46.5 µs at 256 / 512 / 2048 / 4096 and 48.8 µs for torch's pair
    // (scripts/adam_probe.py, profiles/r06_adam_probe_c3.json)
    const int64_t per_block = std::max<int64_t>(unit, ((slots + 1023) / 1024 + unit - 1) / unit * unit);
    const int blocks = (int)std::max<int64_t>(1, (slots + per_block - 1) / per_block);
    if (g_adam_contract)
        hipLaunchKernelGGL(adam_step_kernel<1>, dim3(blocks), dim3(kAdamThreads), 0, strm, L, lr, beta1, beta2,
                           weight_decay, eps, per_block, reinterpret_cast<int*>(arrive));
    else
        hipLaunchKernelGGL(adam_step_kernel<0>, dim3(blocks), dim3(kAdamThreads), 0, strm, L, lr, beta1, beta2,
                           weight_decay, eps, per_block, reinterpret_cast<int*>(arrive));
    return hipGetLastError() == hipSuccess ? MPGNN_OK : MPGNN_ERR_HIP;
}
