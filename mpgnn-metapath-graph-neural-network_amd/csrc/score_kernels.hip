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
constexpr int kMaxConfLists = 4;
constexpr int kMaxConfClasses = 4096;

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

// ---------------------------------------------------------------------------------------------
// Bag branch (model.py:45-72), trained by train(BAGS=True) inside score_relation_bags_parallel
// (main.py:641-673, 853-917). Bags are lists of source nodes; per bag, per member source in the
// dictionary (in bag order): s = LinearLayerAttri(feat[source]) (a dot over the F features),
// the FIRST argmax of weights[dst] * s over the source's destinations, v = weights[max] * s; the
// bag keeps the first member whose v is STRICTLY larger than the running maximum (-10 at the
// start), max_weights[bag] = v. One wave per bag walks its members in order; each member's
// argmax is the wave-parallel first-argmax of score_argmax_kernel over the products.
// ---------------------------------------------------------------------------------------------
// F.linear of one feature row, the same value in every lane of the wave. F <= 32: products added
// in feature order, no contraction into FMAs — the reference's CPU nn.Linear order at these sizes
// and exact for the one-hot colour features of its datasets (tests/test_score_bags.py pins the
// picks bit for bit). Wider rows (dense real features): lane l adds features l, l+64,
// ... in order, then a fixed xor butterfly — deterministic, one coalesced pass instead of every
// lane walking all F features; the reference's BLAS order is unknowable, so there the picks are
// held to the CPU nn.Linear path except at near-ties (tests/test_score_bags.py, dense case).
__device__ __forceinline__ float dot_row(const float* __restrict__ f, const float* __restrict__ wl, int F, int lane) {
    if (F <= 32) {
        float acc = 0.0f;
        for (int j = 0; j < F; ++j) acc = __fadd_rn(acc, __fmul_rn(f[j], wl[j]));
        return acc;
    }
    float acc = 0.0f;
    for (int j = lane; j < F; j += 64) acc = __fadd_rn(acc, __fmul_rn(f[j], wl[j]));
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) acc = __fadd_rn(acc, __shfl_xor(acc, sh));
    return acc;
}

__global__ __launch_bounds__(kScoreThreads) void score_bag_argmax_kernel(
        const float* __restrict__ w, const float* __restrict__ feat, int32_t F, const float* __restrict__ wlin,
        const int32_t* __restrict__ bag_ptr, const int32_t* __restrict__ mem_node, const int32_t* __restrict__ mem_key,
        const int32_t* __restrict__ key_ptr, const int32_t* __restrict__ dst, int32_t B, float* __restrict__ max_w,
        int32_t* __restrict__ bag_mem, float* __restrict__ bag_w, float* __restrict__ mem_s, float* __restrict__ mem_v,
        int32_t* __restrict__ mem_pos, int32_t* __restrict__ mem_max) {
    const int lane = threadIdx.x & 63;
    const int32_t i = (int32_t)(blockIdx.x * kScoreWaves + (threadIdx.x >> 6));
    if (i >= B) return;
    const int32_t mb = bag_ptr[i], me = bag_ptr[i + 1];
    float cur = -10.0f;   // max_weight_for_current_bag (model.py:57)
    float out_v = 0.0f, out_w = 0.0f;
    int32_t out_m = -1;
    for (int32_t m = mb; m < me; ++m) {
        const int32_t k = mem_key[m];
        if (k < 0) continue;  // `if source_node in node_dict` (model.py:59)
        const float s = dot_row(feat + (size_t)mem_node[m] * F, wlin, F, lane);
        const int32_t b = key_ptr[k], e = key_ptr[k + 1];
        float bv = 0.0f;
        int32_t bp = INT32_MAX, bn = 0;
        for (int32_t p = b + lane; p < e; p += 64) {
            const int32_t n = dst[p];
            const float v = __fmul_rn(w[n], s);  // weights_of_source *= lin(feat) (model.py:60-61)
            if (bp == INT32_MAX || takes_over(bv, v)) {
                bv = v;
                bp = p;
                bn = n;
            }
        }
#pragma unroll
        for (int sh = 32; sh >= 1; sh >>= 1) {
            const float ov = __shfl_xor(bv, sh);
            const int32_t op = __shfl_xor(bp, sh), on = __shfl_xor(bn, sh);
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
        // bv == weights[max_node] * lin(feat[source]) (model.py:64): the same product, the same bits
        if (lane == 0) {
            mem_s[m] = s;
            mem_v[m] = bv;
            mem_pos[m] = bp;
            mem_max[m] = bn;
        }
        if (bv > cur) {  // strict: the first member with the largest v keeps the bag (model.py:67-70)
            cur = bv;
            out_v = bv;
            out_m = m;
            out_w = w[bn];
        }
    }
    if (lane == 0) {
        max_w[i] = out_v;   // 0 when no member is in the dictionary (torch.zeros, model.py:48)
        bag_mem[i] = out_m;
        bag_w[i] = out_w;
    }
}

// d weights: one wave per destination node n walks its static candidate list — every (bag i,
// member m, edge position p) with dst[p] == n, bags DESCENDING — and adds g_i · s_m for the
// entries that are their bag's final pick (member m and m's argmax position p): autograd
// unwinds the reference's max_weights[i] = v CopySlices chain last bag first (overwritten picks
// of a bag contribute exact zeros).
__global__ __launch_bounds__(kScoreThreads) void score_bag_scatter_kernel(
        const float* __restrict__ g, const int32_t* __restrict__ bag_mem, const int32_t* __restrict__ mem_pos,
        const float* __restrict__ mem_s, const int32_t* __restrict__ in_ptr, const int32_t* __restrict__ in_bag,
        const int32_t* __restrict__ in_mem, const int32_t* __restrict__ in_pos, int64_t N, float* __restrict__ grad_w) {
    const int lane = threadIdx.x & 63;
    const int64_t n = (int64_t)blockIdx.x * kScoreWaves + (threadIdx.x >> 6);
    if (n >= N) return;
    const int32_t b = in_ptr[n], e = in_ptr[n + 1];
    float acc = 0.0f;
    bool any = false;
    for (int32_t j0 = b; j0 < e; j0 += 64) {
        const int32_t j = j0 + lane;
        bool match = false;
        float c = 0.0f;
        if (j < e) {
            const int32_t i = in_bag[j], m = in_mem[j];
            match = bag_mem[i] == m && mem_pos[m] == in_pos[j];
            if (match) c = __fmul_rn(g[i], mem_s[m]);
        }
        unsigned long long mask = __ballot(match);
        while (mask) {
            const int l = __builtin_ctzll(mask);
            const float cv = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, c), l));
            acc = any ? __fadd_rn(acc, cv) : cv;
            any = true;
            mask &= mask - 1;
        }
    }
    if (lane == 0) grad_w[n] = acc;
}

// d LinearLayerAttri.weight[j] = Σ_{bags i descending} feat[source_i][j] · (g_i · weights[max_i]):
// one wave per feature column; lanes form 64 bags' terms at once, lane order is then folded
// serially (the reference's accumulation order).
__global__ __launch_bounds__(64) void score_bag_lin_kernel(
        const float* __restrict__ g, const int32_t* __restrict__ bag_mem, const float* __restrict__ bag_w,
        const int32_t* __restrict__ mem_node, const float* __restrict__ feat, int32_t F, int32_t B,
        float* __restrict__ grad_lin) {
    const int lane = threadIdx.x;
    const int32_t j = blockIdx.x;
    float acc = 0.0f;
    bool any = false;
    for (int32_t i0 = B - 1; i0 >= 0; i0 -= 64) {
        const int32_t i = i0 - lane;  // lane 0 holds the highest bag of the chunk
        bool has = false;
        float c = 0.0f;
        if (i >= 0) {
            const int32_t m = bag_mem[i];
            has = m >= 0;
            if (has) c = __fmul_rn(feat[(size_t)mem_node[m] * F + j], __fmul_rn(g[i], bag_w[i]));
        }
        unsigned long long mask = __ballot(has);
        while (mask) {
            const int l = __builtin_ctzll(mask);
            const float cv = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, c), l));
            acc = any ? __fadd_rn(acc, cv) : cv;
            any = true;
            mask &= mask - 1;
        }
    }
    if (lane == 0) grad_lin[j] = acc;
}

// ---------------------------------------------------------------------------------------------
// All candidate relations of one scoring round at once (main.py:1309-1330 scores every relation
// with its own score_relation_parallel: 100 epochs each, split over MPI ranks). The dictionaries
// of every relation are ONE relation-major CSR (key k = a (relation, source) pair, destinations in
// edge order — the graph plan's segment order); relation r's weights are row r of a [R, N] matrix.
// Per key: the first argmax (score_argmax_kernel's), the prediction v = w[r][max], and the MSE
// gradient of the relation's mean loss as torch's mse_loss_backward forms it, alpha_r · (v − y)
// with alpha_r = fp32(2 / K_r), plus the squared error for the loss.
// ---------------------------------------------------------------------------------------------
// 8 lanes per key (dictionaries are short: ~1.5 destinations per key at C3; one wave per key left
// 63 of 64 lanes idle), a key's first argmax by an 8-lane butterfly with the associative first-max
// operator of score_argmax_kernel
constexpr int kMultiLanes = 8;
__global__ __launch_bounds__(kScoreThreads) void score_multi_argmax_kernel(
        const float* __restrict__ w, int64_t N, const int32_t* __restrict__ keys, const int32_t* __restrict__ key_ptr,
        const int32_t* __restrict__ dst, const int32_t* __restrict__ key_rel, int32_t K, const float* __restrict__ labels,
        const float* __restrict__ alpha, int32_t* __restrict__ arg_pos, int32_t* __restrict__ max_node,
        float* __restrict__ val, float* __restrict__ dval, float* __restrict__ sq) {
    const int sl = threadIdx.x & (kMultiLanes - 1);
    const int32_t k = (int32_t)(((size_t)blockIdx.x * kScoreThreads + threadIdx.x) / kMultiLanes);
    const bool live = k < K;  // every lane stays for the shuffles
    const int32_t kk = live ? k : K - 1;
    const int32_t b = key_ptr[kk], e = live ? key_ptr[kk + 1] : b;
    const int32_t r = key_rel[kk];
    const float* wr = w + (size_t)r * (size_t)N;
    float bv = 0.0f;
    int32_t bp = INT32_MAX, bn = 0;
    for (int32_t p = b + sl; p < e; p += kMultiLanes) {
        const int32_t n = dst[p];
        const float v = wr[n];
        if (bp == INT32_MAX || takes_over(bv, v)) {
            bv = v;
            bp = p;
            bn = n;
        }
    }
#pragma unroll
    for (int m = kMultiLanes / 2; m >= 1; m >>= 1) {
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
    if (live && sl == 0) {
        const float diff = __fsub_rn(bv, labels[keys[k]]);
        arg_pos[k] = bp;
        max_node[k] = bn;
        val[k] = bv;
        dval[k] = __fmul_rn(alpha[r], diff);  // alpha * (a - b) * grad_output(1)
        sq[k] = __fmul_rn(diff, diff);
    }
}

// loss[r] = Σ sq over relation r's keys / K_r (one wave per relation, a fixed lane-strided order)
__global__ __launch_bounds__(kScoreThreads) void score_multi_loss_kernel(const float* __restrict__ sq,
                                                                         const int32_t* __restrict__ rel_key_ptr,
                                                                         int32_t R, float* __restrict__ loss) {
    const int lane = threadIdx.x & 63;
    const int32_t r = (int32_t)(blockIdx.x * kScoreWaves + (threadIdx.x >> 6));
    if (r >= R) return;
    const int32_t b = rel_key_ptr[r], e = rel_key_ptr[r + 1];
    float acc = 0.0f;
    for (int32_t k = b + lane; k < e; k += 64) acc += sq[k];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m);
    if (lane == 0) loss[r] = e > b ? acc / (float)(e - b) : __builtin_nanf("");
}

// d weights of every relation: 8 lanes per (relation, destination) pair walk the pair's
// (edge position, key) candidates, keys DESCENDING, adding the gradients of the keys whose argmax
// is that edge in list order — score_scatter_kernel's order, per relation
__global__ __launch_bounds__(kScoreThreads) void score_multi_scatter_kernel(
        const float* __restrict__ dval, const int32_t* __restrict__ arg_pos, const int32_t* __restrict__ pair_ptr,
        const int64_t* __restrict__ pair_target, const int32_t* __restrict__ in_pos, const int32_t* __restrict__ in_key,
        int32_t T, float* __restrict__ grad_w) {
    const int lane = threadIdx.x & 63;
    const int sl = lane & (kMultiLanes - 1);
    const int sub0 = lane & ~(kMultiLanes - 1);  // first lane of this pair's group
    const int32_t pi = (int32_t)(((size_t)blockIdx.x * kScoreThreads + threadIdx.x) / kMultiLanes);
    const bool live = pi < T;
    const int32_t b = live ? pair_ptr[pi] : 0, e = live ? pair_ptr[pi + 1] : 0;
    // rounds: the group's longest list decides (wave-uniform loop over the maximum)
    int32_t n_rounds = (e - b + kMultiLanes - 1) / kMultiLanes;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) n_rounds = max(n_rounds, __shfl_xor(n_rounds, m));
    float acc = 0.0f;
    bool any = false;
    for (int32_t rd = 0; rd < n_rounds; ++rd) {
        const int32_t j = b + rd * kMultiLanes + sl;
        bool match = false;
        float g = 0.0f;
        if (j < e) {
            const int32_t k = in_key[j];
            match = arg_pos[k] == in_pos[j];
            if (match) g = dval[k];
        }
        unsigned long long mask = (__ballot(match) >> sub0) & ((1ull << kMultiLanes) - 1);
        while (mask) {  // per group; the groups of a wave iterate together (uniform trip count below)
            const int l = __builtin_ctzll(mask);
            const float gv = __shfl(g, sub0 + l);
            acc = any ? __fadd_rn(acc, gv) : gv;
            any = true;
            mask &= mask - 1;
        }
    }
    if (live && sl == 0) grad_w[pair_target[pi]] = acc;
}


// ---------------------------------------------------------------------------------------
// Per-epoch scoring of the training loop (main.py:1084-1099 mpgnn_validation, main.py:1101-1115
// mpgnn_test): for each (row index, label) pair list, the argmax of the class scores of every
// listed row (torch.argmax(pred[idx], 1): first maximum, NaN wins) and the [3, C] confusion
// counts the macro F1 is finished from (metrics.py): predictions per class, labels per class,
// agreeing positions per class. Labels outside [0, C) count in no class. One workgroup per list,
// LDS histograms, integer adds: exact and order-free — one launch instead of the ~45 small
// torch ops (index, argmax, compare, where, scatter_add, stack) the counts took per epoch.
// ---------------------------------------------------------------------------------------
constexpr int kConfThreads = 1024;

struct ConfArgs {
    const float* scores;
    int64_t rows;
    int32_t C;
    int32_t n_lists;
    const int64_t* idx[kMaxConfLists];     // nullptr: rows 0..n-1
    const int64_t* labels[kMaxConfLists];
    int64_t n[kMaxConfLists];
    int64_t* out;                          // [n_lists][3][C]
};

// the predicted class of score row `row` (first maximum, a NaN wins: torch.argmax); C: none
__device__ __forceinline__ int conf_pred(const ConfArgs& a, int64_t row) {
    const int C = a.C;
    if (row < 0 || row >= a.rows) return C;  // a row outside the score matrix predicts no class
    const float* s = a.scores + row * (int64_t)C;
    float bv = s[0];
    int pc = 0;
    for (int c = 1; c < C; ++c) {
        const float v = s[c];
        if (takes_over(bv, v)) {
            bv = v;
            pc = c;
        }
    }
    return pc;
}

// One workgroup per list. C <= kConfRegC (the loops' 2 classes): each thread counts in registers,
// the counts are summed by wave butterflies and one LDS add per wave and counter (integer sums:
// any order, the same counts); wider C: LDS atomics per pair. Pairs in batches of kConfBatch per
// thread (their list loads, then their score rows: two round trips per batch, not per pair).
constexpr int kConfRegC = 8, kConfBatch = 8;  // 8192 pairs per pass: the loops' lists in one pass
__global__ __launch_bounds__(kConfThreads) void confusion_counts_kernel(ConfArgs a) {
    extern __shared__ int conf_lds[];  // [3][C + 1]
    const int C = a.C, L = (int)blockIdx.x;
    for (int k = threadIdx.x; k < 3 * (C + 1); k += kConfThreads) conf_lds[k] = 0;
    __syncthreads();
    const int64_t* idx = a.idx[L];
    const int64_t* lab = a.labels[L];
    const int64_t n = a.n[L];
    const bool reg = C <= kConfRegC;
    int cp[kConfRegC], cy[kConfRegC], cm[kConfRegC];
#pragma unroll
    for (int c = 0; c < kConfRegC; ++c) cp[c] = cy[c] = cm[c] = 0;
    for (int64_t j0 = threadIdx.x; j0 < n; j0 += (int64_t)kConfBatch * kConfThreads) {
        int64_t row[kConfBatch], y[kConfBatch];
#pragma unroll
        for (int u = 0; u < kConfBatch; ++u) {
            const int64_t j = j0 + (int64_t)u * kConfThreads;
            row[u] = j < n ? (idx ? idx[j] : j) : -1;
            y[u] = j < n ? lab[j] : -1;
        }
#pragma unroll
        for (int u = 0; u < kConfBatch; ++u) {
            if (j0 + (int64_t)u * kConfThreads >= n) break;
            const int pc = conf_pred(a, row[u]);
            const int yc = (y[u] >= 0 && y[u] < C) ? (int)y[u] : C;
            if (reg) {
#pragma unroll
                for (int c = 0; c < kConfRegC; ++c) {
                    cp[c] += pc == c;
                    cy[c] += yc == c;
                    cm[c] += (pc == yc && yc == c);
                }
            } else {
                atomicAdd(&conf_lds[pc], 1);
                atomicAdd(&conf_lds[(C + 1) + yc], 1);
                atomicAdd(&conf_lds[2 * (C + 1) + (pc == yc ? yc : C)], 1);
            }
        }
    }
    if (reg) {
#pragma unroll
        for (int c = 0; c < kConfRegC; ++c) {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                cp[c] += __shfl_xor(cp[c], o);
                cy[c] += __shfl_xor(cy[c], o);
                cm[c] += __shfl_xor(cm[c], o);
            }
        }
        if ((threadIdx.x & 63) == 0) {
            for (int c = 0; c < C; ++c) {
                atomicAdd(&conf_lds[c], cp[c]);
                atomicAdd(&conf_lds[(C + 1) + c], cy[c]);
                atomicAdd(&conf_lds[2 * (C + 1) + c], cm[c]);
            }
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < 3 * C; k += kConfThreads)
        a.out[(int64_t)L * 3 * C + k] = (int64_t)conf_lds[(k / C) * (C + 1) + k % C];
}

// ---------------------------------------------------------------------------------------
// The training loss of the loops (main.py:1065, main_rgcn.py:402, 422; ``F.nll_loss(out[train_idx], train_y)``):
// the mean negative log-probability of each listed (row, target) pair, targets equal to
// ignore_index skipped. Forward: one workgroup sums the picked entries and counts the kept
// pairs (total_weight, an exact integer count in float as in torch's kernel); loss = -(sum /
// total_weight). Backward: grad[row, target] += -(grad_loss / total_weight) — torch's
// nll_loss backward value, placed where index_select's backward would add it (the caller
// zeroes grad). Three torch ops and seven launches per epoch become one launch forward and two
// backward. A pair outside the matrix makes the loss NaN and is skipped by the backward (the
// host validates the lists once, metrics.nll_loss_rows).
// ---------------------------------------------------------------------------------------
constexpr int kNllThreads = 1024;
constexpr int kNllWClasses = 1024;

__global__ __launch_bounds__(kNllThreads) void nll_rows_fwd_kernel(const float* __restrict__ logp, int64_t rows, int C,
                                                                   const int64_t* __restrict__ idx,
                                                                   const int64_t* __restrict__ tgt, int64_t n,
                                                                   int64_t ignore, const float* __restrict__ cw,
                                                                   float* __restrict__ loss,
                                                                   float* __restrict__ total_weight) {
    __shared__ float s_sum[kNllThreads / 64], s_w[kNllThreads / 64];
    __shared__ float s_cw[kNllWClasses];  // the class weights (C <= kNllWClasses), read once
    const bool lds_w = cw != nullptr && C <= kNllWClasses;
    if (lds_w)
        for (int k = threadIdx.x; k < C; k += kNllThreads) s_cw[k] = cw[k];
    __syncthreads();
    // kNllBatch pairs per thread in flight: the list loads of a batch, then its matrix loads
    // (two memory round trips per batch instead of two per pair)
    constexpr int kNllBatch = 8;
    float sum = 0.f, w = 0.f;
    for (int64_t j0 = 0; j0 < n; j0 += (int64_t)kNllBatch * kNllThreads) {
        int64_t r[kNllBatch], t[kNllBatch];
#pragma unroll
        for (int u = 0; u < kNllBatch; ++u) {
            const int64_t j = j0 + (int64_t)u * kNllThreads + threadIdx.x;
            t[u] = j < n ? tgt[j] : ignore;
            r[u] = j < n ? idx[j] : 0;
        }
        float v[kNllBatch];
#pragma unroll
        for (int u = 0; u < kNllBatch; ++u) {
            const bool ok = r[u] >= 0 && r[u] < rows && t[u] >= 0 && t[u] < C;
            v[u] = ok ? logp[r[u] * C + t[u]] : __builtin_nanf("");
        }
#pragma unroll
        for (int u = 0; u < kNllBatch; ++u)
            if (t[u] != ignore) {
                // class weight of the pair (F.nll_loss(weight=...)); 1 without weights (1·v = v)
                const float wt = (cw != nullptr && t[u] >= 0 && t[u] < C) ? (lds_w ? s_cw[t[u]] : cw[t[u]]) : 1.f;
                sum += wt * v[u];
                w += wt;
            }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        sum += __shfl_xor(sum, o);
        w += __shfl_xor(w, o);
    }
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_sum[wv] = sum;
        s_w[wv] = w;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float S = 0.f, W = 0.f;
        for (int k = 0; k < kNllThreads / 64; ++k) {
            S += s_sum[k];
            W += s_w[k];
        }
        loss[0] = -(S / W);
        total_weight[0] = W;
    }
}

__global__ __launch_bounds__(kScoreThreads) void nll_rows_bwd_kernel(const float* __restrict__ grad_loss,
                                                                     const float* __restrict__ total_weight,
                                                                     int64_t rows, int C, const int64_t* __restrict__ idx,
                                                                     const int64_t* __restrict__ tgt, int64_t n,
                                                                     int64_t ignore, const float* __restrict__ cw,
                                                                     float* __restrict__ grad) {
    const int64_t j = (int64_t)blockIdx.x * kScoreThreads + threadIdx.x;
    if (j >= n) return;
    const int64_t t = tgt[j];
    const int64_t r = idx[j];
    if (t == ignore || r < 0 || r >= rows || t < 0 || t >= C) return;
    // equal addends per (row, class): order-free
    atomicAdd(grad + r * C + t, -((cw != nullptr ? cw[t] : 1.f) * (grad_loss[0] / total_weight[0])));
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

extern "C" int32_t mpgnn_score_bag_argmax(const float* weights, const float* feat, int32_t feat_dim, const float* lin_weight,
                                          const int32_t* bag_ptr, const int32_t* mem_node, const int32_t* mem_key,
                                          int64_t num_bags, const int32_t* key_ptr, const int32_t* dst, float* max_weights,
                                          int32_t* bag_mem, float* bag_w, float* mem_s, float* mem_v, int32_t* mem_pos,
                                          int32_t* mem_max, void* stream) {
    if (num_bags < 0 || num_bags >= (int64_t)INT32_MAX || feat_dim < 0) return arg_fail("mpgnn_score_bag_argmax: bad sizes");
    if (num_bags == 0) return MPGNN_OK;
    if (!weights || !bag_ptr || !mem_node || !mem_key || !max_weights || !bag_mem || !bag_w || !mem_s || !mem_v ||
        !mem_pos || !mem_max || (feat_dim > 0 && (!feat || !lin_weight)))
        return arg_fail("mpgnn_score_bag_argmax: NULL argument");
    hipStream_t strm = static_cast<hipStream_t>(stream);
    const unsigned grid = (unsigned)((num_bags + kScoreWaves - 1) / kScoreWaves);
    hipLaunchKernelGGL(score_bag_argmax_kernel, dim3(grid), dim3(kScoreThreads), 0, strm, weights, feat, feat_dim,
                       lin_weight, bag_ptr, mem_node, mem_key, key_ptr, dst, (int32_t)num_bags, max_weights, bag_mem,
                       bag_w, mem_s, mem_v, mem_pos, mem_max);
    return hip_status(hipGetLastError(), "score_bag_argmax_kernel launch");
}

extern "C" int32_t mpgnn_score_bag_argmax_bwd(const float* grad_max, int64_t num_bags, const int32_t* bag_mem,
                                              const float* bag_w, const int32_t* mem_node, const float* mem_s,
                                              const int32_t* mem_pos, const float* feat, int32_t feat_dim,
                                              int64_t num_nodes, const int32_t* in_ptr, const int32_t* in_bag,
                                              const int32_t* in_mem, const int32_t* in_pos, float* grad_weights,
                                              float* grad_lin, void* stream) {
    if (num_bags < 0 || num_bags >= (int64_t)INT32_MAX || num_nodes < 0 || feat_dim < 0)
        return arg_fail("mpgnn_score_bag_argmax_bwd: bad sizes");
    hipStream_t strm = static_cast<hipStream_t>(stream);
    if (num_nodes > 0) {
        if (!in_ptr || !grad_weights) return arg_fail("mpgnn_score_bag_argmax_bwd: NULL candidate list / output");
        const unsigned grid = (unsigned)((num_nodes + kScoreWaves - 1) / kScoreWaves);
        hipLaunchKernelGGL(score_bag_scatter_kernel, dim3(grid), dim3(kScoreThreads), 0, strm, grad_max, bag_mem,
                           mem_pos, mem_s, in_ptr, in_bag, in_mem, in_pos, num_nodes, grad_weights);
        int32_t st = hip_status(hipGetLastError(), "score_bag_scatter_kernel launch");
        if (st != MPGNN_OK) return st;
    }
    if (feat_dim > 0 && grad_lin) {
        if (num_bags == 0) return hip_status(hipMemsetAsync(grad_lin, 0, (size_t)feat_dim * sizeof(float), strm),
                                             "memset grad_lin");
        hipLaunchKernelGGL(score_bag_lin_kernel, dim3((unsigned)feat_dim), dim3(64), 0, strm, grad_max, bag_mem, bag_w,
                           mem_node, feat, feat_dim, (int32_t)num_bags, grad_lin);
        return hip_status(hipGetLastError(), "score_bag_lin_kernel launch");
    }
    return MPGNN_OK;
}

extern "C" int32_t mpgnn_score_argmax_multi(const float* weights, int64_t num_nodes, const int32_t* keys,
                                            const int32_t* key_ptr, const int32_t* dst, const int32_t* key_rel,
                                            int64_t num_keys, const float* labels, const float* alpha, int32_t* arg_pos,
                                            int32_t* max_node, float* values, float* grad_values, float* sq_err,
                                            void* stream) {
    if (num_nodes < 0 || num_keys < 0 || num_keys >= (int64_t)INT32_MAX)
        return arg_fail("mpgnn_score_argmax_multi: bad sizes");
    if (num_keys == 0) return MPGNN_OK;
    if (!weights || !keys || !key_ptr || !dst || !key_rel || !labels || !alpha || !arg_pos || !max_node || !values ||
        !grad_values || !sq_err)
        return arg_fail("mpgnn_score_argmax_multi: NULL argument");
    hipStream_t strm = static_cast<hipStream_t>(stream);
    const int64_t per_block = kScoreThreads / kMultiLanes;
    const unsigned grid = (unsigned)((num_keys + per_block - 1) / per_block);
    hipLaunchKernelGGL(score_multi_argmax_kernel, dim3(grid), dim3(kScoreThreads), 0, strm, weights, num_nodes, keys,
                       key_ptr, dst, key_rel, (int32_t)num_keys, labels, alpha, arg_pos, max_node, values, grad_values,
                       sq_err);
    return hip_status(hipGetLastError(), "score_multi_argmax_kernel launch");
}

extern "C" int32_t mpgnn_score_loss_multi(const float* sq_err, const int32_t* rel_key_ptr, int64_t num_rel, float* loss,
                                          void* stream) {
    if (num_rel < 0 || num_rel >= (int64_t)INT32_MAX) return arg_fail("mpgnn_score_loss_multi: bad sizes");
    if (num_rel == 0) return MPGNN_OK;
    if (!rel_key_ptr || !loss) return arg_fail("mpgnn_score_loss_multi: NULL argument");
    hipStream_t strm = static_cast<hipStream_t>(stream);
    const unsigned grid = (unsigned)((num_rel + kScoreWaves - 1) / kScoreWaves);
    hipLaunchKernelGGL(score_multi_loss_kernel, dim3(grid), dim3(kScoreThreads), 0, strm, sq_err, rel_key_ptr,
                       (int32_t)num_rel, loss);
    return hip_status(hipGetLastError(), "score_multi_loss_kernel launch");
}

extern "C" int32_t mpgnn_score_argmax_multi_bwd(const float* grad_values, const int32_t* arg_pos,
                                                const int32_t* pair_ptr, const int64_t* pair_target,
                                                const int32_t* in_pos, const int32_t* in_key, int64_t num_pairs,
                                                int64_t grad_size, float* grad_weights, void* stream) {
    if (num_pairs < 0 || num_pairs >= (int64_t)INT32_MAX || grad_size < 0)
        return arg_fail("mpgnn_score_argmax_multi_bwd: bad sizes");
    if (grad_size == 0) return MPGNN_OK;
    if (!grad_weights || (num_pairs > 0 && (!grad_values || !arg_pos || !pair_ptr || !pair_target || !in_pos || !in_key)))
        return arg_fail("mpgnn_score_argmax_multi_bwd: NULL argument");
    hipStream_t strm = static_cast<hipStream_t>(stream);
    int32_t st = hip_status(hipMemsetAsync(grad_weights, 0, (size_t)grad_size * sizeof(float), strm), "memset grad");
    if (st != MPGNN_OK || num_pairs == 0) return st;
    const int64_t per_block = kScoreThreads / kMultiLanes;
    const unsigned grid = (unsigned)((num_pairs + per_block - 1) / per_block);
    hipLaunchKernelGGL(score_multi_scatter_kernel, dim3(grid), dim3(kScoreThreads), 0, strm, grad_values, arg_pos,
                       pair_ptr, pair_target, in_pos, in_key, (int32_t)num_pairs, grad_weights);
    return hip_status(hipGetLastError(), "score_multi_scatter_kernel launch");
}

extern "C" int32_t mpgnn_confusion_counts(const float* scores, int64_t rows, int32_t num_classes, int32_t n_lists,
                                          const int64_t* const* row_idx, const int64_t* const* labels,
                                          const int64_t* n, int64_t* counts, void* stream) {
    // 3·(C + 1) int32 LDS histograms: C <= 4096 keeps them under the 64 KB a launch gets without
    // an opt-in attribute
    if (rows < 0 || num_classes <= 0 || num_classes > kMaxConfClasses || n_lists < 0 || n_lists > kMaxConfLists)
        return arg_fail("mpgnn_confusion_counts: bad sizes (1 <= num_classes <= 4096, 0 <= n_lists <= 4)");
    if (n_lists == 0) return MPGNN_OK;
    if (!counts || !labels || !n) return arg_fail("mpgnn_confusion_counts: NULL argument");
    ConfArgs a{};
    a.scores = scores;
    a.rows = rows;
    a.C = num_classes;
    a.n_lists = n_lists;
    a.out = counts;
    for (int l = 0; l < n_lists; ++l) {
        if (n[l] < 0 || n[l] >= (int64_t)INT32_MAX) return arg_fail("mpgnn_confusion_counts: bad list length");
        a.idx[l] = row_idx ? row_idx[l] : nullptr;
        if (n[l] > 0 && (!labels[l] || !scores || (!a.idx[l] && n[l] > rows)))
            return arg_fail("mpgnn_confusion_counts: NULL labels / scores, or an index-free list longer than rows");
        a.labels[l] = labels[l];
        a.n[l] = n[l];
    }
    hipStream_t strm = static_cast<hipStream_t>(stream);
    const size_t lds = (size_t)3 * (num_classes + 1) * sizeof(int);
    hipLaunchKernelGGL(confusion_counts_kernel, dim3(n_lists), dim3(kConfThreads), lds, strm, a);
    return hip_status(hipGetLastError(), "confusion_counts_kernel launch");
}

extern "C" int32_t mpgnn_nll_rows_fwd_weighted(const float* logp, int64_t rows, int32_t num_classes,
                                               const int64_t* row_idx, const int64_t* target, int64_t n,
                                               int64_t ignore_index, const float* class_weight, float* loss,
                                               float* total_weight, void* stream) {
    if (rows < 0 || num_classes <= 0 || n < 0) return arg_fail("mpgnn_nll_rows_fwd_weighted: bad sizes");
    if (!loss || !total_weight || (n > 0 && (!logp || !row_idx || !target)))
        return arg_fail("mpgnn_nll_rows_fwd_weighted: NULL argument");
    hipStream_t strm = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(nll_rows_fwd_kernel, dim3(1), dim3(kNllThreads), 0, strm, logp, rows, (int)num_classes, row_idx,
                       target, n, ignore_index, class_weight, loss, total_weight);
    return hip_status(hipGetLastError(), "nll_rows_fwd_kernel launch");
}

extern "C" int32_t mpgnn_nll_rows_fwd(const float* logp, int64_t rows, int32_t num_classes, const int64_t* row_idx,
                                      const int64_t* target, int64_t n, int64_t ignore_index, float* loss,
                                      float* total_weight, void* stream) {
    return mpgnn_nll_rows_fwd_weighted(logp, rows, num_classes, row_idx, target, n, ignore_index, nullptr, loss,
                                       total_weight, stream);
}

// The same gradient written whole (no zero fill before it): one thread per (row, class), the
// row's positions j in row_idx from a CSR over the rows (row_ptr / row_perm, j ascending), its
// kept pairs of this class added in sequence from 0 — the scatter's value bit for bit (equal
// addends: every sequential order gives the same sum).
__global__ __launch_bounds__(kScoreThreads) void nll_rows_bwd_dense_kernel(
    const float* __restrict__ grad_loss, const float* __restrict__ total_weight, int64_t rows, int C,
    const int* __restrict__ row_ptr, const int* __restrict__ row_perm, const int64_t* __restrict__ tgt,
    int64_t ignore, const float* __restrict__ cw, float* __restrict__ grad) {
    const int64_t e = (int64_t)blockIdx.x * kScoreThreads + threadIdx.x;
    if (e >= rows * C) return;
    const int64_t i = e / C;
    const int c = (int)(e - i * C);
    float v = 0.0f;
    const int p1 = row_ptr[i + 1];
    for (int p = row_ptr[i]; p < p1; ++p) {
        const int64_t t = tgt[row_perm[p]];
        if (t != ignore && t == c) v += -((cw != nullptr ? cw[c] : 1.f) * (grad_loss[0] / total_weight[0]));
    }
    grad[e] = v;
}

extern "C" int32_t mpgnn_nll_rows_bwd_dense(const float* grad_loss, const float* total_weight, int64_t rows,
                                            int32_t num_classes, const int32_t* row_ptr, const int32_t* row_perm,
                                            const int64_t* target, int64_t ignore_index, const float* class_weight,
                                            float* grad_logp, void* stream) {
    if (rows < 0 || num_classes <= 0 || rows * num_classes / kScoreThreads >= (int64_t)INT32_MAX)
        return arg_fail("mpgnn_nll_rows_bwd_dense: bad sizes");
    if (rows == 0) return MPGNN_OK;
    if (!grad_loss || !total_weight || !row_ptr || !row_perm || !target || !grad_logp)
        return arg_fail("mpgnn_nll_rows_bwd_dense: NULL argument");
    hipStream_t strm = static_cast<hipStream_t>(stream);
    const int64_t total = rows * num_classes;
    hipLaunchKernelGGL(nll_rows_bwd_dense_kernel, dim3((unsigned)((total + kScoreThreads - 1) / kScoreThreads)),
                       dim3(kScoreThreads), 0, strm, grad_loss, total_weight, rows, (int)num_classes, row_ptr, row_perm,
                       target, ignore_index, class_weight, grad_logp);
    return hip_status(hipGetLastError(), "nll_rows_bwd_dense_kernel launch");
}

extern "C" int32_t mpgnn_nll_rows_bwd_weighted(const float* grad_loss, const float* total_weight, int64_t rows,
                                               int32_t num_classes, const int64_t* row_idx, const int64_t* target,
                                               int64_t n, int64_t ignore_index, const float* class_weight,
                                               float* grad_logp, void* stream) {
    if (rows < 0 || num_classes <= 0 || n < 0 || n / kScoreThreads >= (int64_t)INT32_MAX)
        return arg_fail("mpgnn_nll_rows_bwd_weighted: bad sizes");
    if (n == 0) return MPGNN_OK;
    if (!grad_loss || !total_weight || !row_idx || !target || !grad_logp)
        return arg_fail("mpgnn_nll_rows_bwd_weighted: NULL argument");
    hipStream_t strm = static_cast<hipStream_t>(stream);
    const unsigned grid = (unsigned)((n + kScoreThreads - 1) / kScoreThreads);
    hipLaunchKernelGGL(nll_rows_bwd_kernel, dim3(grid), dim3(kScoreThreads), 0, strm, grad_loss, total_weight, rows,
                       (int)num_classes, row_idx, target, n, ignore_index, class_weight, grad_logp);
    return hip_status(hipGetLastError(), "nll_rows_bwd_kernel launch");
}

extern "C" int32_t mpgnn_nll_rows_bwd(const float* grad_loss, const float* total_weight, int64_t rows,
                                      int32_t num_classes, const int64_t* row_idx, const int64_t* target, int64_t n,
                                      int64_t ignore_index, float* grad_logp, void* stream) {
    return mpgnn_nll_rows_bwd_weighted(grad_loss, total_weight, rows, num_classes, row_idx, target, n, ignore_index,
                                       nullptr, grad_logp, stream);
}
