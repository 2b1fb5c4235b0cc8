// score_kernels.hip — gfx950 kernels of the metapath score function.
//
// Reference: OutputLayer.forward, non-bag branch (model.py:74-89), driven by train()
// (main.py:641-673) inside score_relation_parallel (main.py:727-760), 100 epochs per candidate
// relation. For every source node of the edge dictionary (create_edge_dictionary,
// main.py:387-424: {source: [destinations of one relation]}) the reference runs a Python loop:
//     max_node = dsts[torch.argmax(weights[dsts])];  max_weights[source] = weights[max_node]
// and autograd sends d max_weights[source] back to weights[max_node], the contributions of the
// sources accumulated in REVERSE dictionary order (the CopySlices chain is unwound last source
// first). Here the dictionary is a CSR in dictionary order (keys, key_ptr, dst) and one wave
// scans one source's destinations; the backward walks, per destination node (one wave), a
// static list of the (source, edge) pairs that can select it, sorted by source rank descending,
// and adds the gradient of each pair that IS its source's argmax — the reference's order, no
// atomics.
//
// Both kernels move a few bytes per edge (index + weight gather) and are latency / HBM bound;
// they replace O(E) Python-level tensor ops per epoch.
#include <hip/hip_runtime.h>

#include <string>

#include "plan_internal.h"

namespace mpgnn {
namespace {

constexpr int kScoreThreads = 256;

int32_t hip_status(hipError_t e, const char* what) {
    if (e == hipSuccess) return MPGNN_OK;
    set_last_error(std::string(what) + ": " + hipGetErrorString(e));
    return MPGNN_ERR_HIP;
}

int32_t arg_fail(const char* msg) {
    set_last_error(msg);
    return MPGNN_ERR_ARG;
}

// torch.argmax over a float vector (ATen's reduction): the first index of the maximum, a NaN
// counting as larger than every number (the first NaN wins).
__device__ __forceinline__ bool takes_over(float best, float v) {
    return !__builtin_isnan(best) && (__builtin_isnan(v) || v > best);
}

constexpr int kScoreWaves = kScoreThreads / 64;

// One wave per dictionary key: lane l scans positions b + l, b + l + 64, ... keeping its first
// maximum, then the 64 candidates are combined by a butterfly whose operator — the candidate
// that takes over, else the smaller position — is associative, so the result is the first
// argmax of the whole row, as the sequential scan (a hub source no longer serialises a thread).
__global__ __launch_bounds__(kScoreThreads) void score_argmax_kernel(
        const float* __restrict__ w, const int32_t* __restrict__ keys, const int32_t* __restrict__ key_ptr,
        const int32_t* __restrict__ dst, int32_t K, float* __restrict__ max_w, int32_t* __restrict__ arg_pos,
        int32_t* __restrict__ max_node) {
    const int lane = threadIdx.x & 63;
    const int32_t k = (int32_t)(blockIdx.x * kScoreWaves + (threadIdx.x >> 6));
    if (k >= K) return;
    const int32_t b = key_ptr[k], e = key_ptr[k + 1];
    float bv = 0.0f;
    int32_t bp = INT32_MAX, bn = 0;  // bp == INT32_MAX: no candidate yet
    for (int32_t p = b + lane; p < e; p += 64) {
        const int32_t n = dst[p];
        const float v = w[n];
        if (bp == INT32_MAX || takes_over(bv, v)) {
            bv = v;
            bp = p;
            bn = n;
        }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const float ov = __shfl_xor(bv, m);
        const int32_t op = __shfl_xor(bp, m), on = __shfl_xor(bn, m);
        bool take;
        if (op == INT32_MAX) take = false;
        else if (bp == INT32_MAX) take = true;
        else if (takes_over(bv, ov)) take = true;
        else if (takes_over(ov, bv)) take = false;
        else take = op < bp;
        if (take) {
            bv = ov;
            bp = op;
            bn = on;
        }
    }
    if (lane == 0) {
        arg_pos[k] = bp;
        max_node[k] = bn;
        max_w[keys[k]] = bv;  // == weights[max_node], the same bits
    }
}

// One wave per destination node: lanes test 64 (source, edge) pairs of its list at a time
// (does the pair's edge hold its source's argmax?), then the matching gradients are added in
// list order from the ballot mask — the reference's accumulation order, no atomics.
__global__ __launch_bounds__(kScoreThreads) void score_scatter_kernel(
        const float* __restrict__ grad_max, const int32_t* __restrict__ keys, const int32_t* __restrict__ arg_pos,
        const int32_t* __restrict__ in_ptr, const int32_t* __restrict__ in_pos, const int32_t* __restrict__ in_key,
        int64_t N, float* __restrict__ grad_w) {
    const int lane = threadIdx.x & 63;
    const int64_t n = (int64_t)blockIdx.x * kScoreWaves + (threadIdx.x >> 6);
    if (n >= N) return;
    const int32_t b = in_ptr[n], e = in_ptr[n + 1];
    float acc = 0.0f;
    bool any = false;
    for (int32_t j0 = b; j0 < e; j0 += 64) {  // sources by rank, descending: the reference's order
        const int32_t j = j0 + lane;
        bool match = false;
        float g = 0.0f;
        if (j < e) {
            const int32_t k = in_key[j];
            match = arg_pos[k] == in_pos[j];
            if (match) g = grad_max[keys[k]];
        }
        unsigned long long mask = __ballot(match);
        while (mask) {
            const int l = __builtin_ctzll(mask);
            const float gv = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, g), l));
            acc = any ? acc + gv : gv;
            any = true;
            mask &= mask - 1;
        }
    }
    if (lane == 0) grad_w[n] = acc;
}

}  // namespace
}  // namespace mpgnn

using namespace mpgnn;

extern "C" int32_t mpgnn_score_argmax(const float* weights, int64_t num_nodes, const int32_t* keys,
                                      const int32_t* key_ptr, const int32_t* dst, int64_t num_keys,
                                      float* max_weights, int32_t* arg_pos, int32_t* max_node, void* stream) {
    if (num_nodes < 0 || num_keys < 0 || num_keys >= (int64_t)INT32_MAX) return arg_fail("mpgnn_score_argmax: bad sizes");
    if (num_nodes == 0) return MPGNN_OK;
    if (!weights || !max_weights) return arg_fail("mpgnn_score_argmax: NULL weights / max_weights");
    if (num_keys > 0 && (!keys || !key_ptr || !dst || !arg_pos || !max_node))
        return arg_fail("mpgnn_score_argmax: NULL dictionary / output");
    hipStream_t strm = static_cast<hipStream_t>(stream);
    int32_t st = hip_status(hipMemsetAsync(max_weights, 0, (size_t)num_nodes * sizeof(float), strm),
                            "memset max_weights");
    if (st != MPGNN_OK || num_keys == 0) return st;
    const unsigned grid = (unsigned)((num_keys + kScoreWaves - 1) / kScoreWaves);
    hipLaunchKernelGGL(score_argmax_kernel, dim3(grid), dim3(kScoreThreads), 0, strm, weights, keys, key_ptr, dst,
                       (int32_t)num_keys, max_weights, arg_pos, max_node);
    return hip_status(hipGetLastError(), "score_argmax_kernel launch");
}

extern "C" int32_t mpgnn_score_argmax_bwd(const float* grad_max, int64_t num_nodes, const int32_t* keys,
                                          const int32_t* arg_pos, const int32_t* in_ptr, const int32_t* in_pos,
                                          const int32_t* in_key, float* grad_weights, void* stream) {
    if (num_nodes < 0) return arg_fail("mpgnn_score_argmax_bwd: bad sizes");
    if (num_nodes == 0) return MPGNN_OK;
    if (!grad_max || !in_ptr || !grad_weights) return arg_fail("mpgnn_score_argmax_bwd: NULL argument");
    hipStream_t strm = static_cast<hipStream_t>(stream);
    const unsigned grid = (unsigned)((num_nodes + kScoreWaves - 1) / kScoreWaves);
    hipLaunchKernelGGL(score_scatter_kernel, dim3(grid), dim3(kScoreThreads), 0, strm, grad_max, keys, arg_pos,
                       in_ptr, in_pos, in_key, num_nodes, grad_weights);
    return hip_status(hipGetLastError(), "score_scatter_kernel launch");
}
