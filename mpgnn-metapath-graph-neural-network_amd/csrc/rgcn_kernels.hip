// rgcn_kernels.hip — gfx950 (CDNA4) kernels for the relation-typed mean aggregation and the
// per-relation dense transform of MPGNN / RGCN layers, plus their backward.
//
// Reference semantics (all fp32):
//   h_r[i]  = (Σ_{e: node_1(e)=i, rel(e)=r} x[node_2(e)]) / max(1, deg_r(i))
//             PyG 2.3.1 propagate(flow='target_to_source', aggr='mean'), mp_rgcn_layer.py:236
//   out     = Σ_r h_r @ W_r + x @ root + bias      mp_rgcn_layer.py:245,265,268 (mode SINGLE,
//             one r, 2-D W) / RGCNConv loop ≙ mp_rgcn_layer.py:249-258 (mode ALL, W[R,F,F])
//
// Kernel map:
//   piece_sum_kernel   ordered partial sums of runs longer than kPieceEntries (one wave/piece)
//   seg_tile_kernel    one workgroup = one 64-row tile. Relation tiles: 64 segments (node_1, r)
//                      of one relation — wavefront segmented gather-sum of x rows into LDS
//                      (edge order, bit-exact mean), then v_mfma_f32_32x32x2_f32 against W_r.
//                      Root tiles: 64 consecutive nodes — x rows into LDS, MFMA against root.
//                      Forward writes Y[seg] = h_seg @ W_r, Y_root[i] = x_i @ root; backward
//                      ("dgrad") writes G[seg] = (dout[node_1] @ W_rᵀ) / cnt, G_root = dout @ rootᵀ.
//   row_sum_kernel     out[i] = (Σ_{entries of row i, in order} src) + extra[i] + bias: the
//                      forward combine Σ_r Y + Y_root + bias (reference add order) and the
//                      transposed grad_x gather Σ G + G_root.
//   outer_accum_kernel dW_r / droot / dbias partial slabs  P_c = A_cᵀ B_c over a chunk of rows.
//   reduce_slabs_kernel ordered sum of the partial slabs of each group (deterministic).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <mutex>
#include <string>
#include <vector>

#include "plan_internal.h"

namespace mpgnn {

int adam_contract_get();  // optim_kernels.hip (MPGNN_OPT_ADAM_CONTRACT)
void adam_contract_set(int v);

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kThreads = 256;  // 4 waves of 64
constexpr int kWaves = 4;
constexpr int kRowsPerWave = kTileRows / kWaves;  // 16 (seg_tile_kernel)
constexpr int kSumRowsPerWave = 8;               // row_sum_kernel: 32 rows per workgroup
constexpr int kColTile = 128;                    // output columns per workgroup (4 × 32-col strips)
constexpr int kSlice = 32;                       // rows per K-slice in outer_accum_kernel
constexpr int kMaxF = 256;

__host__ __device__ constexpr int round_up(int a, int b) { return (a + b - 1) / b * b; }

// ----------------------------------------------------------------------------------------
// small vector helpers
// ----------------------------------------------------------------------------------------
template <int V>
__device__ __forceinline__ void vload(const float* __restrict__ p, float (&v)[V]) {
    if constexpr (V == 4) {
        const float4 t = *reinterpret_cast<const float4*>(p);
        v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    } else if constexpr (V == 2) {
        const float2 t = *reinterpret_cast<const float2*>(p);
        v[0] = t.x; v[1] = t.y;
    } else {
        v[0] = *p;
    }
}

template <int V>
__device__ __forceinline__ void vstore(float* p, const float (&v)[V]) {
    if constexpr (V == 4) {
        *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    } else if constexpr (V == 2) {
        *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
    } else {
        *p = v[0];
    }
}

// vstore through a buffer resource over a wave-uniform base with the sc1 cache policy (aux bit
// 4) — the row outputs of the gather-sum kernels (segment means: 17.4 -> 16.8 µs at C3) and of
// the bf16 GEMMs leave this way
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <int V>
__device__ __forceinline__ void vstore_sc1(float* base, int off, const float (&v)[V]) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
    if constexpr (V == 4) {
        __builtin_amdgcn_raw_buffer_store_b128(
            u32x4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])}, r, off * 4,
            0, 16);
    } else if constexpr (V == 2) {
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(v[0]), __float_as_uint(v[1])}, r, off * 4, 0, 16);
    } else {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[0]), r, off * 4, 0, 16);
    }
}

// vload through a buffer resource with the sc1 cache policy (bypasses this CU's L1: the partials
// other workgroups stored sc1 in the same launch, flat_split_arrive)
template <int V>
__device__ __forceinline__ void vload_sc1(const float* base, int off, float (&v)[V]) {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7fffffff, 0x00020000);
    if constexpr (V == 4) {
        const u32x4 t = __builtin_amdgcn_raw_buffer_load_b128(r, off * 4, 0, 16);
        v[0] = __uint_as_float(t.x); v[1] = __uint_as_float(t.y); v[2] = __uint_as_float(t.z); v[3] = __uint_as_float(t.w);
    } else if constexpr (V == 2) {
        const u32x2 t = __builtin_amdgcn_raw_buffer_load_b64(r, off * 4, 0, 16);
        v[0] = __uint_as_float(t.x); v[1] = __uint_as_float(t.y);
    } else {
        v[0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off * 4, 0, 16));
    }
}

// ReLU with torch's semantics (clamp_min(x, 0)): x < 0 → 0, NaN and -0.0 pass through, so a
// diverging run still shows NaN (fmaxf(NaN, 0) would return 0).
__device__ __forceinline__ float relu_f(float v) { return v < 0.0f ? 0.0f : v; }
// threshold_backward(grad, result, 0): result <= 0 → 0, else grad (NaN results pass grad)
__device__ __forceinline__ float relu_bwd_f(float g, float y) { return y <= 0.0f ? 0.0f : g; }

__device__ __forceinline__ int readlane(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }

// Uniform read of a plan table through the constant address space: an SMEM load (lgkmcnt), so
// waiting for it does not also drain the wave's outstanding vector loads and stores (vmcnt is
// in order).  Only for tables the kernels never write.
__device__ __forceinline__ int ld_uniform(const int* p, int i) {
    return ((const __attribute__((address_space(4))) int*)(p))[i];
}

// ----------------------------------------------------------------------------------------
// Wavefront segmented gather-sum.
//
// The wave owns `nrows` (≤ RPW) consecutive rows.  Lane j (j ≤ nrows) holds in `bnd` the
// position where row j's entries start (row j covers entries [bnd_j, bnd_{j+1})); the entries
// of consecutive rows are contiguous.  Entry q is a position p = (ent ? ent[q] : q) or, when
// ent[q] < 0, the ordered partial sum P[-ent[q]-1 - piece_off] of a piece of a long run
// (piece_sum_kernel).  Position p contributes source row
//     src_row(p) = (idx ? idx[p] : p) - idx_off
// unless the filter rejects it (idx[p] outside [flo, fhi)).  Lanes span the feature dimension
// (V floats per lane, T chunks of 64·V columns); every lane adds its columns in entry order
// starting from 0.0f, which is exactly ATen's sequential scatter_add_ into a zeroed output —
// for runs without pieces the sums are bit-identical to the reference.  Loads are issued
// unconditionally (clamped addresses) and software-pipelined one group of UNR entries ahead:
// a load behind a per-entry branch makes hipcc wait for each entry separately
// (cdna_hip_programming.md §5 trap (c)).  Each finished row is handed to flush(row, live, acc).
// ----------------------------------------------------------------------------------------
struct GatherSrc {
    const float* src;  // [*, F]
    int F;
    const int* idx;    // nullable
    int idx_off;
    int filter;        // keep a position only when idx[p] lies in [flo, fhi)
    int flo, fhi;
    const int* dummy;  // any valid int table: the target of loads whose result is discarded
    const int* ent;    // nullable: two-level entries (position >= 0 | -(piece+1))
    const float* P;    // piece partial sums [*, F] (rows k - piece_off)
    int piece_off;
};

template <int V, int T, int UNR, int RPW, class Flush>
__device__ __forceinline__ void wave_gather(const GatherSrc& g, int bnd, int nrows, int lane, Flush&& flush) {
    float acc[T][V];
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int q = 0; q < V; ++q) acc[t][q] = 0.0f;

    const int p_begin = readlane(bnd, 0);
    const int p_end = readlane(bnd, nrows);
    int r = 0;
    int r_end = nrows > 0 ? readlane(bnd, 1) : p_end;
    int colc[T];
#pragma unroll
    for (int t = 0; t < T; ++t) colc[t] = min((t * 64 + lane) * V, g.F - V);

    for (int pb = p_begin; pb < p_end; pb += 64) {
        const int np = min(64, p_end - pb);
        // branch-free index resolution: every load is issued (clamped or from the dummy
        // table) and its result selected — a branch around a load makes hipcc wait for it at
        // the join, and the join here comes before the row loads
        const int qq = min(pb + lane, p_end - 1);
        const bool has_ent = g.ent != nullptr;
        const bool has_idx = g.idx != nullptr;
        const int e_raw = (has_ent ? g.ent : g.dummy)[has_ent ? qq : 0];
        const int e = has_ent ? e_raw : qq;
        const bool my_piece = e < 0;
        const int ix_raw = (has_idx ? g.idx : g.dummy)[has_idx ? max(e, 0) : 0];
        const int ix = has_idx ? ix_raw : e;
        bool my_keep = lane < np;
        if (g.filter) my_keep = my_keep && (my_piece || (ix >= g.flo && ix < g.fhi));
        int my_src = my_piece ? -e - 1 - g.piece_off : ix - g.idx_off;
        my_src = my_keep ? my_src : 0;  // rejected entry: a valid row is loaded, never added
        const unsigned long long keep = __ballot(my_keep);
        const unsigned long long from_piece = __ballot(my_piece);
        float v[2][UNR][T][V];
        auto issue = [&](float (&dst)[UNR][T][V], int u) {
#pragma unroll
            for (int uu = 0; uu < UNR; ++uu) {
                const int q = min(u + uu, np - 1);
                const int row = readlane(my_src, q);
                const float* base = (((from_piece >> q) & 1ull) ? g.P : g.src) + (size_t)row * g.F;
#pragma unroll
                for (int t = 0; t < T; ++t) vload<V>(base + colc[t], dst[uu][t]);
            }
        };
        auto consume = [&](const float (&src)[UNR][T][V], int u) {
#pragma unroll
            for (int uu = 0; uu < UNR; ++uu) {
                const int q = u + uu;
                if (q < np) {
                    const int p = pb + q;
                    while (p >= r_end) {
                        flush(r, true, acc);
                        ++r;
                        r_end = readlane(bnd, r + 1);
                    }
                    if ((keep >> q) & 1ull) {
#pragma unroll
                        for (int t = 0; t < T; ++t)
#pragma unroll
                            for (int c = 0; c < V; ++c) acc[t][c] += src[uu][t][c];
                    }
                }
            }
        };
        // Two groups of UNR row loads are issued together, then consumed in order.  No buffer
        // is carried across iterations: a loop-carried buffer is copied at the back edge, and
        // the copy waits for the loads just issued into it (one round trip per group).
        // sched_barrier(0) keeps the loads ahead of the adds.
        for (int u = 0; u < np; u += 2 * UNR) {
            issue(v[0], u);
            issue(v[1], u + UNR);  // entries past np are clamped loads, never added
            __builtin_amdgcn_sched_barrier(0);
            consume(v[0], u);
            consume(v[1], u + UNR);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    for (; r < RPW; ++r) flush(r, r < nrows, acc);
}

template <int V, int T>
__device__ __forceinline__ void zero_acc(float (&acc)[T][V]) {
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int q = 0; q < V; ++q) acc[t][q] = 0.0f;
}

// ----------------------------------------------------------------------------------------
// piece_sum_kernel: P[k - k_lo] = Σ_{p in [pb[k], pe[k]), kept} src[idx(p) - idx_off]   (one
// wave per piece, positions summed in order from 0.0f; a piece has <= kPieceEntries entries)
// ----------------------------------------------------------------------------------------
struct PieceArgs {
    const int* pb;
    const int* pe;
    int k_lo, k_hi;
    const float* src;
    int F;
    const int* idx;
    int idx_off;
    int filter;
    int flo, fhi;
    const int* dummy;
    float* P;
};

template <int V, int T>
__global__ __launch_bounds__(kThreads) void piece_sum_kernel(PieceArgs a) {
    const int lane = threadIdx.x & 63;
    const int k = a.k_lo + blockIdx.x * kWaves + (threadIdx.x >> 6);
    if (k >= a.k_hi) return;
    GatherSrc g{};
    g.src = a.src;
    g.F = a.F;
    g.idx = a.idx;
    g.idx_off = a.idx_off;
    g.filter = a.filter;
    g.dummy = a.dummy;
    g.flo = a.flo;
    g.fhi = a.fhi;
    const int bnd = lane == 0 ? a.pb[k] : a.pe[k];
    float* out = a.P + (size_t)(k - a.k_lo) * a.F;
    wave_gather<V, T, 8, 1>(g, bnd, 1, lane, [&](int, bool live, float (&acc)[T][V]) {
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const int col = (t * 64 + lane) * V;
            if (live && col < a.F) vstore<V>(out + col, acc[t]);
        }
        zero_acc<V, T>(acc);
    });
}

// ----------------------------------------------------------------------------------------
// MFMA tile:  acc(64 × 128-column tile) = A_lds[64 × Kp] · B[K × N]
// v_mfma_f32_32x32x2_f32: lane l holds A[i = l&31][kk = l>>5] and B[kk][j = l&31];
// C/D: col = l&31, row = (r&3) + 8(r>>2) + 4(l>>5).  The K dimension is split in two halves
// so that lane-half h walks k ∈ [h·Kp/2, (h+1)·Kp/2) contiguously (one ds_read_b128 feeds
// four MFMAs); the MFMA sums over both halves, so every k is covered exactly once.
// Wave w owns column strip w (32 columns) of the tile and BOTH 32-row halves, so its two
// accumulators share every B value; waves whose strip starts past N idle.
// ----------------------------------------------------------------------------------------
struct BSrc {
    const float* W;  // element (k, n) = trans ? W[n*ldw + k] : W[k*ldw + n]
    int ldw;
    int K, N;
    int trans;
};

struct MfmaTile {
    f32x16 acc0, acc1;  // rows 0..31 / 32..63 of strip `nb`
    int nb;
    bool active;
};

// B(k, n) of the tile: TRANS = false reads W[k*ldw + n] (rows k, 32 consecutive columns per
// half-wave); TRANS = true reads W[n*ldw + k] (row n, four consecutive k per float4 load).
// CLAMP = true handles K < Kp (zero-padded A columns): addresses are clamped to row K-1 and the
// value is replaced by 0 when consumed.  Both are template parameters so the K loop is
// straight-line code: a runtime branch there makes hipcc wait for every prefetch.  K is
// padded to a multiple of 64 in LDS (zeros), so K < Kp needs CLAMP.
template <bool TRANS, bool CLAMP>
struct BLoader {
    const float* W;  // uniform base (SGPRs); lanes add 32-bit element offsets (K·N ≤ 2^16)
    int n, ldw, K;
    __device__ __forceinline__ BLoader(const BSrc& b, int n_) {
        W = b.W;
        n = n_;
        ldw = b.ldw;
        K = b.K;
    }
    // KC consecutive k starting at k0.  The chunk base is clamped (whole chunk inside W) and
    // the addresses are uniform base + 32-bit lane offset: no per-k 64-bit address survives in
    // VGPRs (with per-k 64-bit products the persistent loop's LICM hoisted 64 of them: spills).
    template <int KC>
    __device__ __forceinline__ void load_chunk(int k0, float (&o)[KC]) const {
        if constexpr (!CLAMP) {
            const int kc = min(k0, K - KC);
            if constexpr (!TRANS) {
                const float* p = W + (size_t)kc * ldw;
#pragma unroll
                for (int j = 0; j < KC; ++j) o[j] = p[j * ldw + n];
            } else {
                const float* p = W + kc;
#pragma unroll
                for (int j = 0; j < KC; j += 4) {
                    const float4 tv = *reinterpret_cast<const float4*>(p + n * ldw + j);
                    o[j] = tv.x;
                    o[j + 1] = tv.y;
                    o[j + 2] = tv.z;
                    o[j + 3] = tv.w;
                }
            }
        } else {
#pragma unroll
            for (int j = 0; j < KC; ++j) {
                const int k = min(k0 + j, K - 1);
                o[j] = TRANS ? W[n * ldw + k] : W[k * ldw + n];
            }
        }
    }
};

// K loop of one strip: B is staged in registers in chunks of KC k-values per lane, one chunk
// ahead (a chunk feeds 2·KC MFMAs ≈ 2k SIMD cycles, more than an L2/Infinity-Cache round
// trip); A comes from LDS (ds_read_b128 feeds four MFMAs).  sched_barrier(0) pins each chunk's
// loads where they are written — left alone, the scheduler sinks them below the MFMAs and the
// next chunk then waits for them.  KH % (2·KC) == 0 (Kp % 64 == 0).
constexpr int kKC = 16;

template <bool TRANS, bool CLAMP>
__device__ __forceinline__ void mfma_loop(f32x16& acc0, f32x16& acc1, const float* a0p, const float* a1p, int KH,
                                          int kb, const BSrc& b, int n) {
    const BLoader<TRANS, CLAMP> ld(b, n);
    auto load_chunk = [&](int k0, float (&o)[kKC]) { ld.template load_chunk<kKC>(k0, o); };
    auto compute_chunk = [&](const float (&bc)[kKC], int t, int k0) {
#pragma unroll
        for (int j = 0; j < kKC; j += 4) {
            const float4 a0 = *reinterpret_cast<const float4*>(a0p + t + j);
            const float4 a1 = *reinterpret_cast<const float4*>(a1p + t + j);
            float bq[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) bq[q] = (!CLAMP || k0 + j + q < b.K) ? bc[j + q] : 0.0f;
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.x, bq[0], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.x, bq[0], acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.y, bq[1], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.y, bq[1], acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.z, bq[2], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.z, bq[2], acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.w, bq[3], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.w, bq[3], acc1, 0, 0, 0);
        }
    };
    float b0[kKC], b1[kKC];
    load_chunk(kb, b0);
    // the last pair is peeled so no chunk is loaded past KH (an unconsumed load would be
    // waited for — with every store before it — where its registers are next written)
    int t = 0;
#pragma unroll 1
    for (; t < KH - 2 * kKC; t += 2 * kKC) {
        load_chunk(kb + t + kKC, b1);
        __builtin_amdgcn_sched_barrier(0);
        compute_chunk(b0, t, kb + t);
        __builtin_amdgcn_sched_barrier(0);
        load_chunk(kb + t + 2 * kKC, b0);
        __builtin_amdgcn_sched_barrier(0);
        compute_chunk(b1, t + kKC, kb + t + kKC);
        __builtin_amdgcn_sched_barrier(0);
    }
    load_chunk(kb + t + kKC, b1);
    __builtin_amdgcn_sched_barrier(0);
    compute_chunk(b0, t, kb + t);
    __builtin_amdgcn_sched_barrier(0);
    compute_chunk(b1, t + kKC, kb + t + kKC);
}

__device__ __forceinline__ void mfma_tile(MfmaTile& mt, const float* A_lds, int lda, int Kp,
                                          const BSrc& b, int n_base, int wave, int lane) {
    const int c = lane & 31;
    const int h = lane >> 5;
    f32x16 acc0, acc1;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        acc0[r] = 0.0f;
        acc1[r] = 0.0f;
    }
    mt.nb = wave;
    mt.active = n_base + wave * 32 < b.N;
    if (mt.active) {
        const int KH = Kp / 2;
        const int n = min(n_base + wave * 32 + c, b.N - 1);  // clamped: columns >= N are never stored
        const float* a0p = A_lds + c * lda + h * KH;
        const float* a1p = A_lds + (32 + c) * lda + h * KH;
        const int kb = h * KH;
        const bool exact_k = b.K == Kp;                        // no padded k: clamp-free loop
        const bool vec_ok = (b.ldw & 3) == 0 && b.K >= kKC;
        if (!b.trans) {
            if (exact_k && b.K >= kKC) mfma_loop<false, false>(acc0, acc1, a0p, a1p, KH, kb, b, n);
            else mfma_loop<false, true>(acc0, acc1, a0p, a1p, KH, kb, b, n);
        } else {
            if (exact_k && vec_ok) mfma_loop<true, false>(acc0, acc1, a0p, a1p, KH, kb, b, n);
            else mfma_loop<true, true>(acc0, acc1, a0p, a1p, KH, kb, b, n);
        }
    }
    mt.acc0 = acc0;
    mt.acc1 = acc1;
}

// Dense tile loader: rows [0, nrows) of A[*, K] (contiguous, row stride K) into
// lds[64][lda] with zeros past K (up to width) and past nrows.  Every load of a batch is
// issued before any LDS store (float4 when K % 4 == 0).
__device__ void load_dense_tile(const float* __restrict__ A, int K, int nrows, float* lds, int lda, int width) {
    if ((K & 3) == 0 && (width & 3) == 0) {
        const int w4 = width >> 2;
        const int total = kTileRows * w4;
        constexpr int kBatch = 8;
        for (int i0 = threadIdx.x; i0 < total; i0 += kBatch * kThreads) {
            float4 v[kBatch];
#pragma unroll
            for (int it = 0; it < kBatch; ++it) {
                const int i = min(i0 + it * kThreads, total - 1);
                const int r = min(i / w4, max(nrows - 1, 0));
                const int c = min((i % w4) * 4, K - 4);
                v[it] = *reinterpret_cast<const float4*>(A + (size_t)r * K + c);
            }
#pragma unroll
            for (int it = 0; it < kBatch; ++it) {
                const int i = i0 + it * kThreads;
                if (i < total) {
                    const int r = i / w4;
                    const int c = (i % w4) * 4;
                    const bool ok = r < nrows && c < K;
                    *reinterpret_cast<float4*>(lds + r * lda + c) = ok ? v[it] : make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
        }
        return;
    }
    const int total = kTileRows * width;
    for (int i0 = threadIdx.x; i0 < total; i0 += 8 * kThreads) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = min(i0 + u * kThreads, total - 1);
            const int r = min(i / width, max(nrows - 1, 0));
            const int c = min(i % width, K - 1);
            v[u] = A[(size_t)r * K + c];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * kThreads;
            if (i < total) {
                const int r = i / width;
                const int c = i % width;
                lds[r * lda + c] = (r < nrows && c < K) ? v[u] : 0.0f;
            }
        }
    }
}

// ----------------------------------------------------------------------------------------
// seg_tile_kernel
//   blocks [0, n_rel_tiles): relation tiles (plan tiles t_off + blockIdx.x), rows = segments
//   blocks [n_rel_tiles, ...): root tiles, rows = nodes row_lo + 64·(blockIdx.x - n_rel_tiles)
// ----------------------------------------------------------------------------------------
struct SegTileArgs {
    const int* tile_begin;
    const int* tile_end;
    int tile_off;
    int n_rel_tiles;
    int gather_kind;     // 0: mean of src[e_col[e]] over the segment's edges; 1: src[s_row[s]];
                         // 2: dense rows src[s - sel_b] (precomputed segment means H)
    const float* src;    // x (forward) or dout (dgrad); also the root-tile rows
    int F;               // gather width = K of the MFMA
    const int* s_ptr;    // segment boundaries over edges (exact order) or over ragged entries
    const int* e_col;
    const int* s_row;
    const int* s_cnt;
    const int* s_rel;
    const int* ent;      // nullable: ragged entries (s_ptr then indexes entries)
    const float* P;      // piece partials of long segments
    int piece_off;
    const float* W;      // nullable: no transform (segment means only)
    int w_per_rel;       // W_r = W + s_rel[s] * K * N
    const float* Wroot;  // root-tile B (same orientation as W)
    int trans;
    int N;               // output width
    float* Y;            // relation-tile output rows s - sel_b
    float* Yroot;        // root-tile output rows i - row_lo
    int row_lo, row_hi;
    int y_div;           // divide the relation-tile MFMA result by cnt (dgrad)
    int sel_b;
    float* H;            // nullable: copy of the gathered relation-tile rows, row = s - sel_b, width F
    const float* Hsrc;   // gather_kind 2: precomputed relation-tile rows, row = s - sel_b
};

template <int V, int T>
__global__ __launch_bounds__(kThreads) void seg_tile_kernel(SegTileArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int Kp = round_up(a.F, 64);
    const int lda = Kp + 4;
    float* s_scale = smem;                  // [64] cnt as float (dgrad)
    float* A_lds = smem + kTileRows;        // [64][lda]

    const bool root_tile = (int)blockIdx.x >= a.n_rel_tiles;
    int s0, nrows;
    if (!root_tile) {
        const int tile = blockIdx.x + a.tile_off;
        s0 = a.tile_begin[tile];
        nrows = a.tile_end[tile] - s0;
    } else {
        s0 = a.row_lo + ((int)blockIdx.x - a.n_rel_tiles) * kTileRows;
        nrows = min(kTileRows, a.row_hi - s0);
    }
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const bool div_rows = !root_tile && a.y_div;
    if (div_rows && threadIdx.x < kTileRows)
        s_scale[threadIdx.x] = threadIdx.x < nrows ? (float)a.s_cnt[s0 + threadIdx.x] : 1.0f;

    // ---- gather phase: each wave builds 16 tile rows ---------------------------------
    const int wr0 = wave * kRowsPerWave;
    int wn = nrows - wr0;
    wn = wn < 0 ? 0 : (wn > kRowsPerWave ? kRowsPerWave : wn);
    const int sw = s0 + wr0;
    GatherSrc g{};
    g.src = a.src;
    g.F = a.F;
    g.dummy = a.s_ptr;
    int bnd = 0;
    const int* cnt_rows = nullptr;
    if (root_tile) {
        bnd = sw + (lane <= wn ? lane : wn);  // positions = node ids, source row = position
    } else if (a.gather_kind == 0) {
        if (lane <= wn) bnd = a.s_ptr[sw + lane];
        g.idx = a.e_col;
        g.ent = a.ent;
        g.P = a.P;
        g.piece_off = a.piece_off;
        cnt_rows = a.s_cnt + sw;
    } else {
        bnd = sw + (lane <= wn ? lane : wn);
        g.idx = a.s_row;
    }
    // saved segment means (backward): rows s - sel_b of H, consecutive for the wave's rows
    float* hrow0 = (a.H != nullptr && !root_tile && blockIdx.y == 0) ? a.H + (size_t)(sw - a.sel_b) * a.F : nullptr;
    float* lds_w = A_lds + wr0 * lda;
    if (root_tile || a.gather_kind == 2) {
        // contiguous rows: one coalesced float4 sweep of the whole 64-row tile
        const float* base = root_tile ? a.src + (size_t)s0 * a.F : a.Hsrc + (size_t)(s0 - a.sel_b) * a.F;
        load_dense_tile(base, a.F, nrows, A_lds, lda, Kp);
    } else {
        wave_gather<V, T, (V * T <= 2 ? 8 : 4), kRowsPerWave>(
            g, bnd, wn, lane, [&](int r, bool live, float (&acc)[T][V]) {
                const bool do_div = live && cnt_rows != nullptr;
                const float cnt = do_div ? (float)cnt_rows[r] : 1.0f;
#pragma unroll
                for (int t = 0; t < T; ++t) {
                    const int col = (t * 64 + lane) * V;
                    float v[V];
#pragma unroll
                    for (int q = 0; q < V; ++q) v[q] = live ? (do_div ? acc[t][q] / cnt : acc[t][q]) : 0.0f;
                    if (col < Kp) vstore<V>(lds_w + r * lda + col, v);
                    if (hrow0 != nullptr && live && col < a.F) vstore<V>(hrow0 + (size_t)r * a.F + col, v);
                }
                zero_acc<V, T>(acc);
            });
    }
    __syncthreads();
    if (a.W == nullptr) return;

    // ---- MFMA phase --------------------------------------------------------------------
    const float* W = root_tile ? a.Wroot : a.W;
    if (!root_tile && a.w_per_rel) W += (size_t)a.s_rel[s0] * a.F * a.N;
    BSrc b;
    b.W = W;
    b.K = a.F;
    b.N = a.N;
    b.trans = a.trans;
    b.ldw = a.trans ? a.F : a.N;
    const int n_base = blockIdx.y * kColTile;
    float* Yt = root_tile ? a.Yroot + (size_t)(s0 - a.row_lo) * a.N : a.Y + (size_t)(s0 - a.sel_b) * a.N;
    MfmaTile mt;
    mfma_tile(mt, A_lds, lda, Kp, b, n_base, wave, lane);
    const int c = lane & 31;
    const int h = lane >> 5;
    const int col = n_base + mt.nb * 32 + c;
    if (mt.active && col < a.N) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
            if (row < nrows) {
                float v = mt.acc0[r];
                if (div_rows) v = v / s_scale[row];
                Yt[(size_t)row * a.N + col] = v;
            }
            if (row + 32 < nrows) {
                float v = mt.acc1[r];
                if (div_rows) v = v / s_scale[row + 32];
                Yt[(size_t)(row + 32) * a.N + col] = v;
            }
        }
    }
}

// ----------------------------------------------------------------------------------------
// tile_gemm_kernel — persistent, software-pipelined tile GEMM (forward transform and dgrad)
//
// Work item = (64-row tile, 128-column block).  Tiles [0, n_rel): relation-pure segment tiles
// (plan tiles tile_off + i); tiles [n_rel, n_rel + n_root): node tiles row_lo + 64·j for the
// root weight.  Each workgroup (2 per CU) walks work items blockIdx.x, +gridDim.x, … and keeps
// the next item's A rows in flight in registers while the current item runs on the MFMA pipe;
// the A tile is double-buffered in LDS (one barrier per item) and the epilogue stores drain
// behind the next item's MFMAs.  (A straight launch of one tile per workgroup runs load → MFMA
// → store in lockstep on every CU: memory and the matrix pipe never overlap.)
//   a_kind 2: relation rows = s_src[s] >= 0 ? src[s_src[s]] : Hsrc[-s_src[s] - 1 - m_lo]
//             (segment means: x row of a single-edge segment / compact multi-edge mean),
//             root rows = src[i]   (forward)
//   a_kind 1: relation rows = src[s_row[s]],    root rows = src[i]   (dgrad; / cnt on output)
// ----------------------------------------------------------------------------------------
struct TileGemmArgs {
    const int* tile_begin;
    const int* tile_end;
    int tile_off;
    int n_rel, n_root, ncol;
    int a_kind;
    const float* src;
    const float* Hsrc;
    const int* s_src;
    int m_lo;
    const int* s_row;
    const int* s_cnt;
    const int* s_rel;
    int K;
    const float* W;
    int w_per_rel;
    const float* Wroot;
    int trans;
    int N;
    float* Y;
    float* Yroot;
    int row_lo, row_hi;
    int y_div;
    int sel_b;
};

struct TileItem {
    int s0, nrows, n_base;
    int root;  // int, not bool: a padded struct copy is not scalarised (scratch round trip)
};

__device__ __forceinline__ TileItem tile_item(const TileGemmArgs& a, int w) {
    TileItem it;
    const int tile = w / a.ncol;
    it.n_base = (w - tile * a.ncol) * kColTile;
    it.root = tile >= a.n_rel;
    if (!it.root) {
        const int tt = tile + a.tile_off;
        it.s0 = ld_uniform(a.tile_begin, tt);
        it.nrows = ld_uniform(a.tile_end, tt) - it.s0;
    } else {
        it.s0 = a.row_lo + (tile - a.n_rel) * kTileRows;
        it.nrows = min(kTileRows, a.row_hi - it.s0);
    }
    return it;
}

// Issue the loads of an item's A rows (float4 slot j of this thread = tile element
// threadIdx.x + j·256) into registers; addresses are clamped so every load is valid.
template <int KB, int WPT>
__device__ __forceinline__ void tile_issue(const TileGemmArgs& a, const TileItem& it, int tid, float4 (&v)[WPT], int& cnt_raw) {
    constexpr int W4 = 16 * KB;
    // relation rows are gathered: through s_row (dgrad) or s_src (forward); root rows contiguous
    const bool gathered = !it.root;
    cnt_raw = 1;
    int row[WPT];
#pragma unroll
    for (int j = 0; j < WPT; ++j) row[j] = it.s0 + min((tid + j * kThreads) / W4, it.nrows - 1);
    // uniform branch around the whole index batch (and the dgrad counts): the loads issue back
    // to back and are waited for once (a per-element select compiles to a branch + vmcnt(0)
    // around each load)
    if (gathered) {
        if (a.y_div) cnt_raw = a.s_cnt[it.s0 + min(tid & (kTileRows - 1), it.nrows - 1)];
        const int* idx = a.a_kind == 1 ? a.s_row : a.s_src;
#pragma unroll
        for (int j = 0; j < WPT; ++j) row[j] = idx[row[j]];
    }
#pragma unroll
    for (int j = 0; j < WPT; ++j) {
        const int c = min(((tid + j * kThreads) % W4) * 4, a.K - 4);
        const float* base = row[j] >= 0 ? a.src + (size_t)row[j] * a.K : a.Hsrc + (size_t)(-row[j] - 1 - a.m_lo) * a.K;
        v[j] = *reinterpret_cast<const float4*>(base + c);
    }
}

template <int KB, int WPT>
__device__ __forceinline__ void tile_commit(const TileGemmArgs& a, const TileItem& it, int tid, const float4 (&v)[WPT],
                                            int cnt_raw, float* A, float* scale) {
    constexpr int W4 = 16 * KB;
    constexpr int lda = 64 * KB + 4;
#pragma unroll
    for (int j = 0; j < WPT; ++j) {
        const int i = tid + j * kThreads;
        const int r = i / W4;
        const int c = (i % W4) * 4;
        const bool ok = r < it.nrows && c < a.K;
        *reinterpret_cast<float4*>(A + r * lda + c) = ok ? v[j] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (tid < kTileRows) scale[tid] = (float)cnt_raw;
}

// One strip (64 rows × 32 columns, this wave) of a persistent item: b0 arrives holding the
// item's first B chunk; once its last chunk is in registers the NEXT item's first chunk is
// loaded into b0, so it is in flight across the epilogue and the item boundary (a cold start
// would expose a full L2/MALL miss per item).
template <bool TRANS, bool CLAMP>
__device__ __forceinline__ void mfma_strip(f32x16& acc0, f32x16& acc1, const float* a0p, const float* a1p, int KH,
                                           int kb, const BLoader<TRANS, CLAMP>& ld, float (&b0)[kKC],
                                           const BLoader<TRANS, CLAMP>& ld_next, int kb_next) {
    // A fragments roll one 4-k step ahead: the ds_read_b128 pair for step j+1 is issued before
    // step j's eight MFMAs, so LDS latency hides behind them (read just in time it was exposed
    // every 8 MFMAs: ~10 µs of a 37 µs launch).  The read after the last step lands in the
    // 4-float row pad (lda = Kp + 4) and is never used.
    float4 ca0 = *reinterpret_cast<const float4*>(a0p);
    float4 ca1 = *reinterpret_cast<const float4*>(a1p);
    auto compute_chunk = [&](const float (&bc)[kKC], int t, int k0) {
#pragma unroll
        for (int j = 0; j < kKC; j += 4) {
            const float4 a0 = ca0, a1 = ca1;
            ca0 = *reinterpret_cast<const float4*>(a0p + t + j + 4);
            ca1 = *reinterpret_cast<const float4*>(a1p + t + j + 4);
            __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of this step's MFMAs
            float bq[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) bq[q] = (!CLAMP || k0 + j + q < ld.K) ? bc[j + q] : 0.0f;
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.x, bq[0], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.x, bq[0], acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.y, bq[1], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.y, bq[1], acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.z, bq[2], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.z, bq[2], acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.w, bq[3], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.w, bq[3], acc1, 0, 0, 0);
        }
    };
    auto ldc = [&](const BLoader<TRANS, CLAMP>& l, int k0, float (&o)[kKC]) { l.template load_chunk<kKC>(k0, o); };
    float b1[kKC];
    int t = 0;
#pragma unroll 1
    for (; t < KH - 2 * kKC; t += 2 * kKC) {
        ldc(ld, kb + t + kKC, b1);
        __builtin_amdgcn_sched_barrier(0);
        compute_chunk(b0, t, kb + t);
        __builtin_amdgcn_sched_barrier(0);
        ldc(ld, kb + t + 2 * kKC, b0);
        __builtin_amdgcn_sched_barrier(0);
        compute_chunk(b1, t + kKC, kb + t + kKC);
        __builtin_amdgcn_sched_barrier(0);
    }
    ldc(ld, kb + t + kKC, b1);
    __builtin_amdgcn_sched_barrier(0);
    compute_chunk(b0, t, kb + t);
    __builtin_amdgcn_sched_barrier(0);
    ldc(ld_next, kb_next, b0);
    __builtin_amdgcn_sched_barrier(0);
    compute_chunk(b1, t + kKC, kb + t + kKC);
}

// Output rows of an item from an LDS staging tile [64][kColTile + 4] to Y / Y_root (float4
// rows when N % 4 == 0), divided by the item's row scales for the dgrad.  256 threads (mt).
__device__ __forceinline__ void tile_store(const TileGemmArgs& a, const TileItem& it, int mt, const float* S,
                                           const float* sc) {
    constexpr int ldo = kColTile + 4;
    float* Yt = it.root ? a.Yroot + (size_t)(it.s0 - a.row_lo) * a.N : a.Y + (size_t)(it.s0 - a.sel_b) * a.N;
    const bool div_rows = !it.root && a.y_div;
    const int ncols = min(kColTile, a.N - it.n_base);
    if ((a.N & 3) == 0) {
        const int c4n = ncols >> 2;
#pragma unroll
        for (int j = 0; j < kTileRows * (kColTile / 4) / 256; ++j) {
            const int i = mt + j * 256;
            const int row = i >> 5;
            const int c4 = i & 31;
            if (row < it.nrows && c4 < c4n) {
                float4 val = *reinterpret_cast<const float4*>(S + row * ldo + c4 * 4);
                if (div_rows) {
                    const float d = sc[row];
                    val.x = val.x / d;
                    val.y = val.y / d;
                    val.z = val.z / d;
                    val.w = val.w / d;
                }
                *reinterpret_cast<float4*>(Yt + (size_t)row * a.N + it.n_base + c4 * 4) = val;
            }
        }
    } else {
        for (int i = mt; i < kTileRows * kColTile; i += 256) {
            const int row = i >> 7;
            const int cc = i & 127;
            if (row < it.nrows && cc < ncols) {
                float val = S[row * ldo + cc];
                if (div_rows) val = val / sc[row];
                Yt[(size_t)row * a.N + it.n_base + cc] = val;
            }
        }
    }
}

__device__ __forceinline__ int opaque(int x) {
    asm volatile("" : "+v"(x));
    return x;
}

__device__ __forceinline__ BSrc item_bsrc(const TileGemmArgs& a, const TileItem& it) {
    BSrc b;
    b.W = it.root ? a.Wroot : a.W;
    if (!it.root && a.w_per_rel) b.W += (size_t)ld_uniform(a.s_rel, it.s0) * a.K * a.N;
    b.K = a.K;
    b.N = a.N;
    b.trans = a.trans;
    b.ldw = a.trans ? a.K : a.N;
    return b;
}

// Item order: the 8 workgroup groups g = blockIdx % 8 (the blocks one XCD receives under
// round-robin placement — a speed-only assumption) each own a contiguous eighth of the item
// list, so the relation weights an XCD's L2 pulls in are one eighth of them; within a group
// the workgroups stride through their eighth.  Bijective for any grid (every item is visited
// exactly once whatever the placement).
struct ItemOrder {
    int base, stride, end;
    __device__ __forceinline__ ItemOrder(int n_items) {
        const int g = blockIdx.x & 7;
        const int per = (n_items + 7) >> 3;
        base = g * per + (blockIdx.x >> 3);
        stride = ((int)gridDim.x - g + 7) >> 3;  // workgroups in group g
        end = min(n_items, (g + 1) * per);
    }
};

template <int KB, bool TRANS, bool CLAMP>
__device__ __forceinline__ void tile_gemm_body(const TileGemmArgs& a, float* smem) {
    constexpr int Kp = 64 * KB;
    constexpr int KH = Kp / 2;
    constexpr int lda = Kp + 4;
    constexpr int ldo = kColTile + 4;                   // staged output tile row stride
    constexpr int bstride = kTileRows * (lda > ldo ? lda : ldo);
    constexpr int WPT = 4 * KB;                         // float4 per thread per tile
    float* bufs = smem;                                 // [2][64][max(lda, ldo)]
    float* scales = smem + 2 * bstride;                 // [2][64]
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int n_items = (a.n_rel + a.n_root) * a.ncol;
    const ItemOrder ord(n_items);
    int w = ord.base;
    if (w >= ord.end) return;

    float4 v[WPT];
    int cnt_raw;
    TileItem cur = tile_item(a, w);
    tile_issue<KB, WPT>(a, cur, threadIdx.x, v, cnt_raw);
    float b0[kKC];
    {
        const int lane = threadIdx.x & 63;
        const BLoader<TRANS, CLAMP> ld0(item_bsrc(a, cur), min(cur.n_base + wave * 32 + (lane & 31), a.N - 1));
        ld0.template load_chunk<kKC>((lane >> 5) * KH, b0);
    }
    tile_commit<KB, WPT>(a, cur, threadIdx.x, v, cnt_raw, bufs, scales);
    __syncthreads();
    for (int buf = 0; w < ord.end; buf ^= 1) {
        // Laundered per item: otherwise LICM hoists every thread-invariant LDS/global offset
        // of the loop body (dozens of them) and holds them live across the loop (spills).
        const int tid = opaque(threadIdx.x);
        const int lane = tid & 63;
        const int c = lane & 31;
        const int h = lane >> 5;
        const int wn = w + ord.stride;
        const bool has_next = wn < ord.end;
        const TileItem nxt = has_next ? tile_item(a, wn) : cur;
        if (has_next) tile_issue<KB, WPT>(a, nxt, tid, v, cnt_raw);  // in flight during this item's MFMAs
        float* A = bufs + buf * bstride;
        const bool active = cur.n_base + wave * 32 < a.N;
        const BLoader<TRANS, CLAMP> ld_next(item_bsrc(a, nxt), min(nxt.n_base + wave * 32 + c, a.N - 1));
        f32x16 acc0, acc1;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            acc0[r] = 0.0f;
            acc1[r] = 0.0f;
        }
        {   // unconditional (a wave past N computes clamped columns and stores nothing): a branch
            // here would join b0 through register copies that wait for the preloaded chunk
            const BLoader<TRANS, CLAMP> ld(item_bsrc(a, cur), min(cur.n_base + wave * 32 + c, a.N - 1));
            const float* a0p = A + c * lda + h * KH;
            const float* a1p = A + (32 + c) * lda + h * KH;
            if constexpr (KB == 2) {  // (KB 3, 4: no registers left)
                // two accumulation chains over the halves of this lane's K range, added before
                // the epilogue: half the fma rounding chain (accuracy vs the float64 truth)
                constexpr int KH2 = KH / 2;
                f32x16 acc2, acc3;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    acc2[r] = 0.0f;
                    acc3[r] = 0.0f;
                }
                mfma_strip<TRANS, CLAMP>(acc0, acc1, a0p, a1p, KH2, h * KH, ld, b0, ld, h * KH + KH2);
                mfma_strip<TRANS, CLAMP>(acc2, acc3, a0p + KH2, a1p + KH2, KH2, h * KH + KH2, ld, b0, ld_next, h * KH);
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    acc0[r] = acc0[r] + acc2[r];
                    acc1[r] = acc1[r] + acc3[r];
                }
            } else {
                mfma_strip<TRANS, CLAMP>(acc0, acc1, a0p, a1p, KH, h * KH, ld, b0, ld_next, h * KH);
            }
        }
        // epilogue: accumulators -> LDS (the consumed A buffer) -> whole-row coalesced stores
        __syncthreads();
        if (active) {
            float* o = A + (4 * h) * ldo + wave * 32 + c;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2);
                o[row * ldo] = acc0[r];
                o[(row + 32) * ldo] = acc1[r];
            }
        }
        __syncthreads();
        // next item's A tile first: its vmcnt wait then does not also wait for this item's stores
        if (has_next) tile_commit<KB, WPT>(a, nxt, tid, v, cnt_raw, bufs + (buf ^ 1) * bstride, scales + (buf ^ 1) * kTileRows);
        {
            float* Yt = cur.root ? a.Yroot + (size_t)(cur.s0 - a.row_lo) * a.N : a.Y + (size_t)(cur.s0 - a.sel_b) * a.N;
            const bool div_rows = !cur.root && a.y_div;
            const float* sc = scales + buf * kTileRows;
            const int ncols = min(kColTile, a.N - cur.n_base);
            if ((a.N & 3) == 0) {
                const int c4n = ncols >> 2;  // float4 columns of this block
#pragma unroll
                for (int j = 0; j < kTileRows * (kColTile / 4) / kThreads; ++j) {
                    const int i = tid + j * kThreads;
                    const int row = i >> 5;
                    const int c4 = i & 31;
                    if (row < cur.nrows && c4 < c4n) {
                        float4 val = *reinterpret_cast<const float4*>(A + row * ldo + c4 * 4);
                        if (div_rows) {
                            const float d = sc[row];
                            val.x = val.x / d;
                            val.y = val.y / d;
                            val.z = val.z / d;
                            val.w = val.w / d;
                        }
                        *reinterpret_cast<float4*>(Yt + (size_t)row * a.N + cur.n_base + c4 * 4) = val;
                    }
                }
            } else {
                for (int i = tid; i < kTileRows * kColTile; i += kThreads) {
                    const int row = i >> 7;
                    const int cc = i & 127;
                    if (row < cur.nrows && cc < ncols) {
                        float val = A[row * ldo + cc];
                        if (div_rows) val = val / sc[row];
                        Yt[(size_t)row * a.N + cur.n_base + cc] = val;
                    }
                }
            }
        }
        __syncthreads();
        cur = nxt;
        w = wn;
    }
}


// ----------------------------------------------------------------------------------------
// rel_gemm_kernel — B-stationary persistent GEMM for the forward transform and the dgrad
// (K = 64·KB ∈ {64, 128}, N = 128 output columns).
//
//   forward: Y[s] = H[s] @ W_rel(s)              Y_root[i] = x[i] @ root
//   dgrad:   G[s] = (dout[s_row[s]] @ W_relᵀ) / cnt[s]   G_root[i] = dout[i] @ rootᵀ
//
// Work items are 32-row relation-pure tiles (plan t32 tables) followed by 32-node root tiles;
// workgroup b owns the contiguous item range [b·n/G, (b+1)·n/G), so consecutive items mostly
// share a relation.  Wave w owns output columns [32w, 32w + 32) and holds its K × 32 slice of
// the current relation's weight IN REGISTERS (KH = K/2 VGPRs: lane-half h carries
// k ∈ [h·KH, (h+1)·KH), column 32w + (lane & 31)), so the weight is read once per relation
// run instead of once per tile; the next run's slice is fetched into a second register set
// during the last tile of the current run.  A tiles (32 rows × K) are double-buffered in LDS:
// item i+1's rows are loaded into registers before item i's MFMAs and written to the other
// buffer after them (one barrier per item).  v_mfma_f32_32x32x2_f32 (exact f32 fma chain):
// each wave issues KH MFMAs per item from ds_read_b128 A fragments (one per four MFMAs).
// Output rows leave straight from the accumulators: each accumulator register is two 128-B
// row segments (C/D layout: col = lane & 31, row = (r & 3) + 8(r >> 2) + 4(lane >> 5)).
// ----------------------------------------------------------------------------------------
constexpr int kFirstRec = 8 + 6 * 32;  // ints per item range of RelGemmArgs::first

struct RelGemmArgs {
    const int* t_begin;   // 32-row relation tiles (segments)
    const int* t_end;
    int t_lo;             // first tile of the selection
    int n_rel, n_root;    // items [0, n_rel) tiles t_lo + i; [n_rel, n_rel + n_root) node rows
    const float* Arel;    // forward: compact multi-edge means Hm (row m - m_lo); dgrad: unused
    const float* Aroot;   // forward: x; dgrad: dout  (row i)
    const int* s_src;     // forward: A row of segment s = s_src[s] >= 0 ? x[s_src[s]] : Hm[-s_src[s] - 1 - m_lo]
    int m_lo;
    const int* s_row;
    const int* s_cnt;
    const int* s_rel;
    const float* W;       // [R][K][N] (w_per_rel) or [K][N]; dgrad: [R][N][K] / [N][K] (transposed use)
    int w_per_rel;
    const float* Wroot;   // [K][N]; dgrad [N][K]
    float* Y;             // rows s - sel_b
    float* Yroot;         // rows i - row_lo
    int sel_b, row_lo, row_hi;
    // fused mode-SINGLE layer (CAT): node rows i read [x_i | mean_i] against [root; W] (K = 2·F_in);
    // node_map[i] = 0 (no segment of the relation), s_src + 1 (x row), or s_src (< 0: Hm row).
    // Forward, not CAT (mode-SINGLE root epilogue): root rows i with node_map[i] == 0 are final —
    // act((0 + x_i @ root) + bias); the others stay x_i @ root for single_fix_kernel
    const int* node_map;
    int m_rows;           // CAT: rows of Hm (indices are clamped to the tables: a bad map cannot fault)
    const float* bias;    // nullable, CAT epilogue
    int relu;             // CAT epilogue: fused ReLU
    const int* wg_items;  // nullable (rel_gemm_bf3_kernel): [G + 1] first item of each range
    int wg_cus;           // > 0 with wg_items: G = 2·wg_cus, ranges 2c and 2c+1 belong to one CU (below)
    unsigned* zero;       // nullable (rel_gemm_bf3_kernel): zero_words words zeroed by the launch — the
    int zero_words;       // next gather-sum's piece counters (dgrad -> grad_x), instead of a memset launch
    // nullable (rel_gemm_bf3_kernel, K = 128, MPGNN_OPT_GEMM_FIRST): per item range (kFirstRec ints)
    // {i_beg, i_end, weight index of item i_beg (-1 root), its r0, its nrows, 0, 0, 0, then the
    // gathered row numbers of items i_beg .. i_beg + 2 (clamped to the range) [3][32] and their
    // dgrad counts [3][32]}: the prologue reads them in one round instead of range -> tiles ->
    // s_src / s_row hops
    const int* first;
#ifdef MPGNN_STAMPS
    unsigned long long* stamps;
#endif
};

#ifdef MPGNN_STAMPS
// Debug build only (csrc/Makefile `stamps`): per wave and item, shader-clock stamps of the
// phases of rel_gemm_kernel, written by lane 0 with vector stores (scripts/stamps_gemm.py).
constexpr int kStampItems = 32, kStampPhases = 8;  // row 0: HW_ID, XCC_ID, start, 3 prologue, rt start, rt end
static unsigned long long* g_stamps_host = nullptr;  // set by mpgnn_debug_stamps_set, passed as an argument
#define MPGNN_STAMP_PTR a.stamps
#define stamp(k, ph) stamp_at(a.stamps, k, ph)
#define stamp_id() stamp_id_at(a.stamps)
#define stamp_pro(k) stamp_pro_at(a.stamps, k)
#define stamp_end() stamp_end_at(a.stamps)
__device__ __forceinline__ void stamp_at(unsigned long long* g_stamps, int k, int ph) {
    if (g_stamps != nullptr && (threadIdx.x & 63) == 0 && k < kStampItems) {
        const size_t w = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        g_stamps[(w * (kStampItems + 1) + 1 + k) * kStampPhases + ph] = __builtin_readcyclecounter();
    }
}
__device__ __forceinline__ void stamp_id_at(unsigned long long* g_stamps) {
    if (g_stamps != nullptr && (threadIdx.x & 63) == 0) {
        const size_t w = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        unsigned long long* o = g_stamps + w * (kStampItems + 1) * kStampPhases;
        o[0] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
        o[1] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
        o[2] = __builtin_readcyclecounter();
        o[6] = __builtin_amdgcn_s_memrealtime();
    }
}
__device__ __forceinline__ void stamp_end_at(unsigned long long* g_stamps) {
    if (g_stamps != nullptr && (threadIdx.x & 63) == 0) {
        const size_t w = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        g_stamps[w * (kStampItems + 1) * kStampPhases + 7] = __builtin_amdgcn_s_memrealtime();
    }
}
// prologue stamps: row 0 slots 3..5 of the wave
__device__ __forceinline__ void stamp_pro_at(unsigned long long* g_stamps, int k) {
    if (g_stamps != nullptr && (threadIdx.x & 63) == 0) {
        const size_t w = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        g_stamps[w * (kStampItems + 1) * kStampPhases + k] = __builtin_readcyclecounter();
    }
}
#else
#define stamp(k, ph) ((void)0)
#define stamp_id() ((void)0)
#define stamp_pro(k) ((void)0)
#define stamp_end() ((void)0)
#endif

// REPI: the mode-SINGLE root epilogue (RelGemmArgs::node_map, forward only) — its own
// instantiation over ROOT items only (n_rel == 0: no gathered rows, no weight changes), launched
// after the relation items' normal kernel; the mode-ALL kernels carry none of its registers
template <int KB, bool DGRAD, int NB = 1, int OCC = 2, bool CAT = false, bool PIPE = true, bool REPI = false>
struct RelGemm {
    static constexpr int K = 64 * KB;
    static constexpr int KH = K / 2;
    static constexpr int N = 128 * NB;  // output / weight row stride; a workgroup covers 128 columns
    // first output column of this workgroup (grid.y = NB column blocks)
    __device__ static __forceinline__ int col0() { return NB > 1 ? (int)blockIdx.y * 128 : 0; }
    // the next relation run's weight slice prefetched into a second register set (K = 256: two
    // slices would not fit; three workgroups per CU: neither)
    // pipelined dgrad (the forward's cross-item loop) keeps the previous item's outputs in 16 more
    // registers: its weight slice is reloaded after the chain on a relation change instead
    static constexpr bool kPrefetchB = KB <= 2 && OCC <= 2 && !(DGRAD && PIPE);
    static constexpr int lda = K + 4;
    static constexpr int WPT = 32 * (K / 4) / kThreads;  // float4 of an A tile per thread

    struct Item {
        int r0, nrows, root;
        const float* w;   // weight matrix of the item (uniform)
    };

    __device__ static __forceinline__ Item item(const RelGemmArgs& a, int i) {
        Item it;
        if constexpr (REPI) {  // root items only
            it.root = 1;
            it.r0 = a.row_lo + i * 32;
            it.nrows = min(32, a.row_hi - it.r0);
            it.w = a.Wroot;
            return it;
        }
        it.root = i >= a.n_rel;
        if (!it.root) {
            it.r0 = ld_uniform(a.t_begin, a.t_lo + i);
            it.nrows = ld_uniform(a.t_end, a.t_lo + i) - it.r0;
            it.w = a.W + (a.w_per_rel ? (size_t)ld_uniform(a.s_rel, it.r0) * K * N : 0);
        } else {
            it.r0 = a.row_lo + (i - a.n_rel) * 32;
            it.nrows = min(32, a.row_hi - it.r0);
            it.w = a.Wroot;
        }
        return it;
    }

    // Descriptors of the workgroup's items i_beg + lane (lanes < 64), fetched once with vector
    // loads; per item they are read back with readlane (no dependent scalar loads in the loop).
    struct ItemTable {
        int r0, nrows, wrel;  // wrel: weight index (relation id), -1 = root weight
    };
    __device__ static __forceinline__ ItemTable item_table(const RelGemmArgs& a, int i_beg, int i_end, int lane) {
        ItemTable t;
        const int i = min(i_beg + lane, i_end - 1);
        if (i < a.n_rel) {
            t.r0 = a.t_begin[a.t_lo + i];
            t.nrows = a.t_end[a.t_lo + i] - t.r0;
            t.wrel = a.w_per_rel ? a.s_rel[t.r0] : 0;
        } else {
            t.r0 = a.row_lo + (i - a.n_rel) * 32;
            t.nrows = min(32, a.row_hi - t.r0);
            t.wrel = -1;
        }
        return t;
    }
    __device__ static __forceinline__ Item item_at(const RelGemmArgs& a, const ItemTable& t, int k) {
        Item it;
        it.r0 = readlane(t.r0, k);
        it.nrows = readlane(t.nrows, k);
        const int wr = readlane(t.wrel, k);
        it.root = wr < 0;
        it.w = it.root ? a.Wroot : a.W + (size_t)wr * K * N;
        return it;
    }

    // The A rows of a relation item are gathered: forward, segment s reads x[s_src[s]] (a
    // single-edge segment: its mean is that x row) or its compact mean Hm[-s_src[s] - 1 - m_lo];
    // dgrad reads dout[s_row[s]] (scaled by 1/cnt at the output). The row numbers (and dgrad
    // scale) of an item are loaded one item earlier than its rows, so issuing the rows costs
    // one round trip, not two. Root items read rows r0.. of Aroot directly.
    __device__ static __forceinline__ void gather_idx(const RelGemmArgs& a, const Item& it, int tid, int (&row)[WPT],
                                                      int& cnt) {
        constexpr int W4 = K / 4;
#pragma unroll
        for (int j = 0; j < WPT; ++j) row[j] = it.r0 + min((tid + j * kThreads) / W4, it.nrows - 1);
        cnt = 1;
        if constexpr (REPI) {  // root epilogue: this lane's row of the item has a segment?
            if (it.root) cnt = a.node_map[it.r0 + min(tid & 31, it.nrows - 1)];
        }
        if constexpr (CAT) {  // a thread's float4 column is fixed (256 % W4 == 0): x half or mean half
            const bool mh = (tid % W4) >= W4 / 2;
#pragma unroll
            for (int j = 0; j < WPT; ++j) row[j] = mh ? a.node_map[row[j]] : row[j] + 1;
            return;
        }
        if (!it.root) {
            if constexpr (DGRAD) {
                cnt = a.s_cnt[it.r0 + min(tid & 31, it.nrows - 1)];
#pragma unroll
                for (int j = 0; j < WPT; ++j) row[j] = a.s_row[row[j]];
            } else {
#pragma unroll
                for (int j = 0; j < WPT; ++j) row[j] = a.s_src[row[j]];
            }
        }
    }
    __device__ static __forceinline__ void issue_rows(const RelGemmArgs& a, int tid, const int (&row)[WPT],
                                                      float4 (&v)[WPT], int& zm) {
        constexpr int W4 = K / 4;
        if constexpr (CAT) {  // rows of F = K/2 floats: x[v - 1] (v > 0), Hm[-v - 1 - m_lo] (v < 0), 0 (v == 0)
            constexpr int F = K / 2;
            const int c4 = ((tid % W4) % (W4 / 2)) * 4;
            zm = 0;
#pragma unroll
            for (int j = 0; j < WPT; ++j) {
                const int r = row[j];
                const float* base = r >= 0 ? a.Aroot + (size_t)min(max(r - 1, 0), a.row_hi - 1) * F
                                           : a.Arel + (size_t)min(max(-r - 1 - a.m_lo, 0), a.m_rows - 1) * F;
                zm |= (r == 0 ? 1 : 0) << j;
                v[j] = *reinterpret_cast<const float4*>(base + c4);
            }
            return;
        }
        zm = 0;
#pragma unroll
        for (int j = 0; j < WPT; ++j) {
            const int c4 = ((tid + j * kThreads) % W4) * 4;
            const float* base;
            if constexpr (DGRAD) {
                base = a.Aroot + (size_t)row[j] * K;
            } else {
                base = row[j] >= 0 ? a.Aroot + (size_t)row[j] * K : a.Arel + (size_t)(-row[j] - 1 - a.m_lo) * K;
            }
            v[j] = *reinterpret_cast<const float4*>(base + c4);
        }
    }

    __device__ static __forceinline__ void commit(const Item& it, int tid, const float4 (&v)[WPT], int cnt, float* A,
                                                  float* sc, int zm = 0) {
        constexpr int W4 = K / 4;
#pragma unroll
        for (int j = 0; j < WPT; ++j) {
            const int e = tid + j * kThreads;
            const int r = e / W4;
            *reinterpret_cast<float4*>(A + r * lda + (e % W4) * 4) =
                (r < it.nrows && !((zm >> j) & 1)) ? v[j] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        // the dgrad row scale as a reciprocal (one IEEE division per row and item here, a multiply
        // per output in the epilogue instead of a 10-instruction division: ≤ 1.5 ulp apart);
        // REPI: one word, bit k = row k of the item has a segment of the relation (wave 0's lanes k
        // loaded row k's flag); read back as a wave-uniform value, so the epilogue's 16 flags cost
        // no vector registers
        if constexpr (REPI) {
            const unsigned long long bm = __ballot(cnt != 0);
            if (tid == 0) reinterpret_cast<unsigned*>(sc)[0] = (unsigned)bm;
        } else {
            if (tid < 32) sc[tid] = 1.0f / (float)cnt;
        }
    }

    // CAT: B = [root; W] — lane half 0 takes root's K/2 rows, half 1 W's
    __device__ static __forceinline__ void load_b_cat(const RelGemmArgs& a, int wave, int lane, float (&b)[KH]) {
        const int c = lane & 31, h = lane >> 5;
        const float* p = (h ? a.W : a.Wroot) + col0() + wave * 32 + c;
#pragma unroll
        for (int j = 0; j < KH; ++j) b[j] = p[j * N];
    }

    // this wave's K × 32 weight slice: lane-half h holds k = h·KH + j, column 32·wave + c
    __device__ static __forceinline__ void load_b(const float* w, int wave, int lane, float (&b)[KH]) {
        const int c = lane & 31, h = lane >> 5;
        if constexpr (!DGRAD) {
            const float* p = w + (size_t)(h * KH) * N + col0() + wave * 32 + c;
#pragma unroll
            for (int j = 0; j < KH; ++j) b[j] = p[j * N];
        } else {  // B(k, n) = W[n][k]: K consecutive floats of row n = 32·wave + c
            const float* p = w + (size_t)(col0() + wave * 32 + c) * K + h * KH;
#pragma unroll
            for (int j = 0; j < KH; j += 4) {
                const float4 t = *reinterpret_cast<const float4*>(p + j);
                b[j] = t.x;
                b[j + 1] = t.y;
                b[j + 2] = t.z;
                b[j + 3] = t.w;
            }
        }
    }

    // Forward loop, software-pipelined across items so the MFMA pipe sees one barrier per item
    // and nothing else: item i's 16 output stores go out one per MFMA group of item i+1's
    // chain (bounds-checked buffer stores: rows past a partial item's end are dropped by the
    // descriptor, no exec branches), and item i+1's A tile is committed to the other LDS
    // buffer three quarters into item i's chain (its rows were issued at the top of item i).
    __device__ static void run_fwd(const RelGemmArgs& a, float* smem) {
        float* As = smem;                 // [2][32][lda]
        float* Sc = smem + 2 * 32 * lda;  // [2][32] dgrad row scales (forward: unused)
        const int tid = threadIdx.x;
        const int lane = tid & 63, c = lane & 31, h = lane >> 5;
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        const int n_items = a.n_rel + a.n_root;
        const int G = (int)gridDim.x;
        const int g = (int)blockIdx.x & 7, q = G >> 3, rem = G & 7;
        const int rng = g * q + min(g, rem) + ((int)blockIdx.x >> 3);
        const int i_beg = (int)((long long)rng * n_items / G);
        const int i_end = (int)((long long)(rng + 1) * n_items / G);
        if (i_beg >= i_end) return;

        stamp_id();
        float4 v[WPT];
        int cnt;
        const ItemTable tab = REPI ? ItemTable{} : item_table(a, i_beg, i_end, lane);
        auto get_item = [&](int i) {
            if constexpr (REPI) return item(a, i);
            return i - i_beg < 64 ? item_at(a, tab, i - i_beg) : item(a, i);
        };
        Item cur = get_item(i_beg);
        int zm = 0;
        {
            int crow[WPT];
            gather_idx(a, cur, tid, crow, cnt);
            issue_rows(a, tid, crow, v, zm);
        }
        int nrow[WPT];
        int ncnt = 1;
        if (i_beg + 1 < i_end) gather_idx(a, get_item(i_beg + 1), tid, nrow, ncnt);
        float b[KH];
        if constexpr (CAT) load_b_cat(a, wave, lane, b);
        else load_b(cur.w, wave, lane, b);
        commit(cur, tid, v, cnt, As, Sc, zm);
#pragma unroll
        for (int j = 0; j < KH; ++j) asm volatile("" ::"v"(b[j]));
        __syncthreads();

        constexpr int NG = KH / 4;                 // MFMA groups (one A fragment each) per chain
        constexpr int SPG = (16 + NG - 1) / NG;    // previous item's stores per group
        constexpr int kCommitAt = (3 * NG) / 4;    // group after which the next tile is committed
        constexpr bool kSplit = KB <= 2 || CAT;    // two accumulation chains (accuracy)
        // CAT epilogue: + bias (this lane's column), fused ReLU
        float bias_c = 0.0f;
        if constexpr (CAT || REPI) bias_c = a.bias != nullptr ? a.bias[col0() + wave * 32 + c] : 0.0f;
        // this lane's byte offset of output row `row` inside an item's first row (col block + strip)
        const int col_b = (col0() + wave * 32 + c) * 4;
        // the first chain stores through an empty descriptor (every store dropped): the stores
        // are unconditional, so the wait-count pass never merges a store-free path into the loop
        // (that would make the next item's index wait also wait for this item's stores)
        float prev[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) prev[r] = 0.0f;
        __amdgpu_buffer_rsrc_t prev_rsrc = __builtin_amdgcn_make_buffer_rsrc(a.Y, (short)0, 0, 0x00020000);
        auto store_prev = [&](int r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(prev[r]), prev_rsrc, row * (N * 4) + col_b, 0, 0);
        };
        int buf = 0;
        for (int i = i_beg; i < i_end; ++i) {
            stamp(i - i_beg, 0);
            const bool has_next = i + 1 < i_end;
            const Item nxt = has_next ? get_item(i + 1) : cur;
            if (has_next) {
                issue_rows(a, tid, nrow, v, zm);
                cnt = ncnt;
                if (i + 2 < i_end) gather_idx(a, get_item(i + 2), tid, nrow, ncnt);
            }
            const bool new_w = !CAT && !REPI && nxt.w != cur.w;
            float bn[kPrefetchB ? KH : 1];
            if constexpr (kPrefetchB) {
                if (new_w) load_b(nxt.w, wave, lane, bn);
            }
            const float* Ab = As + buf * 32 * lda + c * lda + h * KH;
            f32x16 acc, acc2;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                acc[r] = 0.0f;
                acc2[r] = 0.0f;
            }
            float4 af = *reinterpret_cast<const float4*>(Ab);
#pragma unroll
            for (int gi = 0; gi < NG; ++gi) {
                const int j = 4 * gi;
                const float4 cf = af;
                if (j + 4 < KH) af = *reinterpret_cast<const float4*>(Ab + j + 4);
                f32x16& ac = (kSplit && j >= KH / 2) ? acc2 : acc;
                ac = __builtin_amdgcn_mfma_f32_32x32x2f32(cf.x, b[j], ac, 0, 0, 0);
                ac = __builtin_amdgcn_mfma_f32_32x32x2f32(cf.y, b[j + 1], ac, 0, 0, 0);
                ac = __builtin_amdgcn_mfma_f32_32x32x2f32(cf.z, b[j + 2], ac, 0, 0, 0);
                ac = __builtin_amdgcn_mfma_f32_32x32x2f32(cf.w, b[j + 3], ac, 0, 0, 0);
#pragma unroll
                for (int u = 0; u < SPG; ++u)
                    if (gi * SPG + u < 16) store_prev(gi * SPG + u);
                if (gi == kCommitAt - 1 && has_next) {
                    commit(nxt, tid, v, cnt, As + (buf ^ 1) * 32 * lda, Sc + (buf ^ 1) * 32, zm);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            stamp(i - i_beg, 1);
            // this item's outputs become the next chain's stores
            unsigned emask = 0;
            if constexpr (REPI) emask = __builtin_amdgcn_readfirstlane(reinterpret_cast<const unsigned*>(Sc)[buf * 32]);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                prev[r] = kSplit ? acc[r] + acc2[r] : acc[r];
                if constexpr (DGRAD) {  // row scale 1/cnt of relation rows (reciprocal, see commit)
                    if (!cur.root) prev[r] = prev[r] * Sc[buf * 32 + (r & 3) + 8 * (r >> 2) + 4 * h];
                }
                if constexpr (CAT) {
                    prev[r] = prev[r] + bias_c;
                    if (a.relu) prev[r] = relu_f(prev[r]);
                }
                if constexpr (REPI) {  // a row without a segment: (0 + x_i @ root) + bias, act
                    if (cur.root && !((emask >> ((r & 3) + 8 * (r >> 2) + 4 * h)) & 1u)) {
                        const float e = (0.0f + prev[r]) + bias_c;
                        prev[r] = a.relu ? relu_f(e) : e;
                    }
                }
            }
            {
                float* Yt = cur.root ? a.Yroot + (size_t)(cur.r0 - a.row_lo) * N : a.Y + (size_t)(cur.r0 - a.sel_b) * N;
                const int bytes = __builtin_amdgcn_readfirstlane(cur.nrows) * N * 4;
                prev_rsrc = __builtin_amdgcn_make_buffer_rsrc(Yt, (short)0, bytes, 0x00020000);
            }
            if (new_w) {
                if constexpr (kPrefetchB) {
#pragma unroll
                    for (int j = 0; j < KH; ++j) b[j] = bn[j];
                } else {
                    load_b(nxt.w, wave, lane, b);
                }
            }
            stamp(i - i_beg, 3);
            __syncthreads();
            stamp(i - i_beg, 4);
            cur = nxt;
            buf ^= 1;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) store_prev(r);
    }

    __device__ static void run(const RelGemmArgs& a, float* smem) {
        if constexpr (!DGRAD || PIPE) {
            run_fwd(a, smem);
            return;
        }
        float* As = smem;                 // [2][32][lda]
        float* Sc = smem + 2 * 32 * lda;  // [2][32] dgrad row scales
        float* Pt = Sc + 64 + 4;          // dgrad, K <= 128: [4 waves][16][64] first-half partials
        const int tid = threadIdx.x;
        const int lane = tid & 63, c = lane & 31, h = lane >> 5;
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        const int n_items = a.n_rel + a.n_root;
        // range index: workgroups b, b + 8, b + 16, … (one XCD under round-robin placement, a
        // speed-only assumption) take consecutive item ranges, so a relation run split over
        // several workgroups has its weight slice served from one XCD's L2
        const int G = (int)gridDim.x;
        const int g = (int)blockIdx.x & 7, q = G >> 3, rem = G & 7;
        const int rng = g * q + min(g, rem) + ((int)blockIdx.x >> 3);
        const int i_beg = (int)((long long)rng * n_items / G);
        const int i_end = (int)((long long)(rng + 1) * n_items / G);
        if (i_beg >= i_end) return;

        stamp_id();
        float4 v[WPT];
        int cnt;
        // up to 64 items per workgroup through the register table, the rest by scalar loads
        const ItemTable tab = item_table(a, i_beg, i_end, lane);
        auto get_item = [&](int i) { return i - i_beg < 64 ? item_at(a, tab, i - i_beg) : item(a, i); };
        Item cur = get_item(i_beg);
        {
            int crow[WPT], zm_unused;
            gather_idx(a, cur, tid, crow, cnt);
            issue_rows(a, tid, crow, v, zm_unused);
        }
        int nrow[WPT];  // gathered rows (+ dgrad scale) of the item after the current one
        int ncnt = 1;
        if (i_beg + 1 < i_end) gather_idx(a, get_item(i_beg + 1), tid, nrow, ncnt);
        float b[KH];
        load_b(cur.w, wave, lane, b);
        commit(cur, tid, v, cnt, As, Sc);
        // Consume the prologue's weight loads here. Otherwise the wait-count pass merges their
        // pending state into the loop header and, in EVERY iteration, makes the MFMAs wait on
        // vmcnt values that only the in-flight prefetches (next A tile, next weight slice)
        // can satisfy — serialising the prefetch latency with the MFMA chain.
#pragma unroll
        for (int j = 0; j < KH; ++j) asm volatile("" ::"v"(b[j]));
        __syncthreads();
        int buf = 0;
        for (int i = i_beg; i < i_end; ++i) {
            stamp(i - i_beg, 0);
            const bool has_next = i + 1 < i_end;
            const Item nxt = has_next ? get_item(i + 1) : cur;
            if (has_next) {  // in flight during this item's MFMAs: rows of the next item, row
                             // numbers of the one after
                int zm_unused;
                issue_rows(a, tid, nrow, v, zm_unused);
                cnt = ncnt;
                if (i + 2 < i_end) gather_idx(a, get_item(i + 2), tid, nrow, ncnt);
            }
            const bool new_w = nxt.w != cur.w;
            float bn[kPrefetchB ? KH : 1];
            if constexpr (kPrefetchB) {
                if (new_w) load_b(nxt.w, wave, lane, bn);  // the next relation run's slice
            }
            const float* Ab = As + buf * 32 * lda + c * lda + h * KH;
            // K <= 128: two accumulation chains (k-steps j < KH/2 and j >= KH/2) added in the
            // epilogue, half the rounding chain of one K-long fma chain (accuracy vs the float64
            // truth). Forward: the second chain in registers; dgrad (no registers left): the first
            // half's sums parked in LDS (this lane's own 16 floats, no barrier). K = 256: one chain.
            constexpr bool kSplit = KB <= 2 && !DGRAD;
            constexpr bool kSplitLds = KB <= 2 && DGRAD;
            float* pt = Pt + (wave * 16) * 64 + lane;
            f32x16 acc, acc2;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                acc[r] = 0.0f;
                acc2[r] = 0.0f;
            }
            float4 af = *reinterpret_cast<const float4*>(Ab);
#pragma unroll
            for (int j = 0; j < KH; j += 4) {
                const float4 cf = af;
                if (j + 4 < KH) af = *reinterpret_cast<const float4*>(Ab + j + 4);
                if (kSplitLds && j == KH / 2) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        pt[r * 64] = acc[r];
                        acc[r] = 0.0f;
                    }
                }
                f32x16& ac = (kSplit && j >= KH / 2) ? acc2 : acc;
                ac = __builtin_amdgcn_mfma_f32_32x32x2f32(cf.x, b[j], ac, 0, 0, 0);
                ac = __builtin_amdgcn_mfma_f32_32x32x2f32(cf.y, b[j + 1], ac, 0, 0, 0);
                ac = __builtin_amdgcn_mfma_f32_32x32x2f32(cf.z, b[j + 2], ac, 0, 0, 0);
                ac = __builtin_amdgcn_mfma_f32_32x32x2f32(cf.w, b[j + 3], ac, 0, 0, 0);
            }
            stamp(i - i_beg, 1);
            // next item's A tile into the other LDS buffer BEFORE this item's output stores: its
            // wait (vmcnt, in order) then covers only the row loads issued at the top of the
            // item, not 16 stores issued just before it (each would cost a write round trip)
            if (has_next) commit(nxt, tid, v, cnt, As + (buf ^ 1) * 32 * lda, Sc + (buf ^ 1) * 32);
            stamp(i - i_beg, 2);
            // epilogue: each accumulator register = rows (r&3) + 8(r>>2) + 4h, column 32·wave + c
            const float* sc = Sc + buf * 32;
            float* Yt = cur.root ? a.Yroot + (size_t)(cur.r0 - a.row_lo) * N : a.Y + (size_t)(cur.r0 - a.sel_b) * N;
            auto out_val = [&](int r, int row) {
                float o = kSplit ? acc[r] + acc2[r] : (kSplitLds ? pt[r * 64] + acc[r] : acc[r]);
                if constexpr (DGRAD) {
                    if (!cur.root) o = o * sc[row];
                }
                return o;
            };
            float* Yc = Yt + col0() + wave * 32 + c;
            if (cur.nrows == 32) {  // uniform: a full item stores straight, no per-row exec branches
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
                    Yc[(size_t)row * N] = out_val(r, row);
                }
            } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
                    if (row < cur.nrows) Yc[(size_t)row * N] = out_val(r, row);
                }
            }
            if (new_w) {
                if constexpr (kPrefetchB) {
#pragma unroll
                    for (int j = 0; j < KH; ++j) b[j] = bn[j];
                } else {
                    load_b(nxt.w, wave, lane, b);  // after this item's chain: b is free
                }
            }
            stamp(i - i_beg, 3);
            __syncthreads();
            stamp(i - i_beg, 4);
            cur = nxt;
            buf ^= 1;
        }
    }
};

template <int KB, bool DGRAD, int NB = 1, int OCC = 2, bool CAT = false, bool PIPE = true, bool REPI = false>
__global__ __launch_bounds__(kThreads, OCC) void rel_gemm_kernel(RelGemmArgs a) {
    extern __shared__ float smem[];
    RelGemm<KB, DGRAD, NB, OCC, CAT, PIPE, REPI>::run(a, smem);
}

// ----------------------------------------------------------------------------------------
// rel_gemm_bf3_kernel — rel_gemm_kernel's B-stationary persistent GEMM (same items, gathers,
// cross-item pipeline, outputs) on the bf16 matrix cores: v_mfma_f32_32x32x16_bf16 runs 16× the
// FLOP/clk of v_mfma_f32_32x32x2_f32 (MI355X_MICROARCH.md §Matrix cores). Every fp32 operand is
// split EXACTLY into three bf16 pieces, a = a0 + a1 + a2 (round-to-nearest: |a1| ≤ 2^-9|a|,
// |a2| ≤ 2^-18|a|; each bf16 × bf16 product is exact in fp32) and the six products down to
// 2^-18 relative are accumulated:
//     hi += a0·b0        lo += a2·b0 + a1·b1 + a0·b2 + a1·b0 + a0·b1        out = hi + lo
// (dropped: a1·b2, a2·b1 ≤ 2^-27, a2·b2). 6 MFMAs of 32 cycles per 16 k instead of 8 of 64:
// 2.67× the fp32-MFMA rate. Accuracy: the hardware adds each instruction's 16 products before
// rounding into the accumulator (scripts/mfma_bf16_probe.hip), and the small terms sum in their
// own accumulator, so the result is at least as close to the float64 truth as the fp32 fmaf
// chain of rel_gemm_kernel (tests/test_gpu_parity.py holds it to the same bars).
//
// Registers: the wave's K × 32 weight slice as 3 × K/16 bf16x8 fragments (K = 128: 96 VGPRs,
// lane-half h holds k ∈ [16s + 8h, 16s + 8h + 8) of k-step s, column 32·wave + (lane & 31)).
// LDS: the A tile as three bf16 planes [32][K + 8] (double-buffered; the 16-B pad makes the
// fragment reads ds_read_b128-conflict-free), split once by the committing thread.
// ----------------------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// Workgroup → item range when the host balanced the ranges per CU (gemm_ranges, G = 2·C
// workgroups on C CUs): blocks b and b + C run on one CU (the dispatcher fills every CU's first
// slot before any second one — observed on MI355X, speed only, never correctness); the CU's two
// workgroups take the two halves 2c, 2c + 1 of CU range c, and CU ranges are consecutive on an XCD
// (blocks b ≡ x mod 8 share XCD x).
__device__ __forceinline__ int wg_pair_range(int b, int C) {
    const int cu = b % C, half = b / C;
    return 2 * ((cu & 7) * (C >> 3) + (cu >> 3)) + half;
}

__device__ __forceinline__ void split3_bf16(float a, __bf16& h0, __bf16& h1, __bf16& h2) {
#ifdef MPGNN_PROBE_NOSPLIT  // probe build only (scripts/r05_probe_nosplit.sh): the split's VALU cost
    h0 = (__bf16)a;
    h1 = (__bf16)0.0f;
    h2 = (__bf16)0.0f;
    return;
#endif
    h0 = (__bf16)a;               // v_cvt_pk_bf16_f32: round to nearest even
    const float r1 = a - (float)h0;  // exact
    h1 = (__bf16)r1;
    const float r2 = r1 - (float)h1;  // exact, ≤ 8 significant bits: h2 == r2
    h2 = (__bf16)r2;
}

template <int KB, bool DGRAD>
struct RelGemmBf3 {
    using Base = RelGemm<KB, DGRAD>;
    static constexpr int K = 64 * KB;
    static constexpr int N = 128;
    static constexpr int NS = K / 16;              // k-steps of 16
    static constexpr int LDAB = K + 8;             // bf16 row stride of an A plane
    static constexpr int PLANE = 32 * LDAB;        // bf16 per plane
    static constexpr int WPT = Base::WPT;          // float4 of an A tile per thread
    using Item = typename Base::Item;
    using ItemTable = typename Base::ItemTable;

    static constexpr size_t lds_bytes() { return (size_t)2 * 3 * PLANE * 2 + 2 * 32 * sizeof(float) + 64; }

    __device__ static __forceinline__ void commit(const Item& it, int tid, const float4 (&v)[WPT], int cnt,
                                                  __bf16* A, float* sc) {
        constexpr int W4 = K / 4;
#pragma unroll
        for (int j = 0; j < WPT; ++j) {
            const int e = tid + j * kThreads;
            const int r = e / W4;
            const float4 x = r < it.nrows ? v[j] : make_float4(0.f, 0.f, 0.f, 0.f);
            __bf16 p0[4], p1[4], p2[4];
            split3_bf16(x.x, p0[0], p1[0], p2[0]);
            split3_bf16(x.y, p0[1], p1[1], p2[1]);
            split3_bf16(x.z, p0[2], p1[2], p2[2]);
            split3_bf16(x.w, p0[3], p1[3], p2[3]);
            __bf16* d = A + r * LDAB + (e % W4) * 4;
            typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
            *reinterpret_cast<bf16x4*>(d) = bf16x4{p0[0], p0[1], p0[2], p0[3]};
            *reinterpret_cast<bf16x4*>(d + PLANE) = bf16x4{p1[0], p1[1], p1[2], p1[3]};
            *reinterpret_cast<bf16x4*>(d + 2 * PLANE) = bf16x4{p2[0], p2[1], p2[2], p2[3]};
        }
        if (tid < 32) sc[tid] = 1.0f / (float)cnt;
    }

    // the wave's weight slice as bf16 pieces: b[s][p][j] = piece p of B(16s + 8h + j, 32·wave + c)
    __device__ static __forceinline__ void load_b_raw(const float* w, int wave, int lane, float (&f)[NS][8]) {
        const int c = lane & 31, h = lane >> 5;
        if constexpr (!DGRAD) {
            const float* p = w + (size_t)(8 * h) * N + wave * 32 + c;
#pragma unroll
            for (int s = 0; s < NS; ++s)
#pragma unroll
                for (int j = 0; j < 8; ++j) f[s][j] = p[(16 * s + j) * N];
        } else {  // B(k, n) = W[n][k]: 8 consecutive floats of row n = 32·wave + c
            const float* p = w + (size_t)(wave * 32 + c) * K + 8 * h;
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const float4 t0 = *reinterpret_cast<const float4*>(p + 16 * s);
                const float4 t1 = *reinterpret_cast<const float4*>(p + 16 * s + 4);
                f[s][0] = t0.x; f[s][1] = t0.y; f[s][2] = t0.z; f[s][3] = t0.w;
                f[s][4] = t1.x; f[s][5] = t1.y; f[s][6] = t1.z; f[s][7] = t1.w;
            }
        }
    }
    __device__ static __forceinline__ void split_b(const float (&f)[NS][8], bf16x8 (&b)[NS][3]) {
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                __bf16 h0, h1, h2;
                split3_bf16(f[s][j], h0, h1, h2);
                b[s][0][j] = h0;
                b[s][1][j] = h1;
                b[s][2][j] = h2;
            }
    }
    __device__ static __forceinline__ void load_b(const float* w, int wave, int lane, bf16x8 (&b)[NS][3]) {
        float f[NS][8];
        load_b_raw(w, wave, lane, f);
        split_b(f, b);
    }

    // one float4 of the next item's A tile (thread part j) split into the LDS planes; rows past
    // nrows are zeros. No branch: the k-step that carries it stays one scheduling region.
    __device__ static __forceinline__ void commit_part(int j, int tid, int nrows, const float4& v, __bf16* A) {
        constexpr int W4 = K / 4;
        const int e = tid + j * kThreads;
        const int r = e / W4;
        const float4 x = r < nrows ? v : make_float4(0.f, 0.f, 0.f, 0.f);
        __bf16 p0[4], p1[4], p2[4];
        split3_bf16(x.x, p0[0], p1[0], p2[0]);
        split3_bf16(x.y, p0[1], p1[1], p2[1]);
        split3_bf16(x.z, p0[2], p1[2], p2[2]);
        split3_bf16(x.w, p0[3], p1[3], p2[3]);
        __bf16* d = A + r * LDAB + (e % W4) * 4;
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        *reinterpret_cast<bf16x4*>(d) = bf16x4{p0[0], p0[1], p0[2], p0[3]};
        *reinterpret_cast<bf16x4*>(d + PLANE) = bf16x4{p1[0], p1[1], p1[2], p1[3]};
        *reinterpret_cast<bf16x4*>(d + 2 * PLANE) = bf16x4{p2[0], p2[1], p2[2], p2[3]};
    }

    // Interleaved item skeleton (round 5): the same items, gathers, products and stores as run(),
    // bit-identical outputs, but the next item's tile commit is cut into its WPT float4 parts and
    // each part is scheduled INSIDE one k-step among that k-step's six MFMAs (sched_group_barrier:
    // the next k-step's three fragment reads first, then MFMA / VALU / LDS-write / store groups),
    // and the k-steps carry no branch. run() committed the whole tile in one k-step as ~150 VALU
    // instructions in a row (waiting on its rows), during which the wave issued no MFMA.
    __device__ static void run_il(const RelGemmArgs& a, __bf16* smem) {
        __bf16* As = smem;                                            // [2][3 planes][32][LDAB]
        float* Sc = reinterpret_cast<float*>(smem + 2 * 3 * PLANE);  // [2][32] dgrad row scales
        const int tid = threadIdx.x;
        const int lane = tid & 63, c = lane & 31, h = lane >> 5;
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        const int n_items = a.n_rel + a.n_root;
        const int G = (int)gridDim.x;
        const int g = (int)blockIdx.x & 7, q = G >> 3, rem = G & 7;
        const int rng = a.wg_cus > 0 ? wg_pair_range((int)blockIdx.x, a.wg_cus) : g * q + min(g, rem) + ((int)blockIdx.x >> 3);
        const int* rec = a.first != nullptr ? a.first + (size_t)rng * kFirstRec : nullptr;
        const int i_beg = rec ? ld_uniform(rec, 0) : a.wg_items ? ld_uniform(a.wg_items, rng) : (int)((long long)rng * n_items / G);
        const int i_end = rec ? ld_uniform(rec, 1) : a.wg_items ? ld_uniform(a.wg_items, rng + 1) : (int)((long long)(rng + 1) * n_items / G);
        if (i_beg >= i_end) return;
        stamp_id();

        // Prologue (round 5): the stamps showed ~10k cycles from the launch to the first item —
        // six dependent round trips (range, tile rows, s_rel, s_src, rows, then the weight slice).
        // Now: the item table reads each item's weight index from the range table (no s_rel
        // hop), the row numbers of the first three items are requested together, the weight
        // slice is requested beside them and split while the first rows are in flight.
        ItemTable tab;
        {
            const int i = min(i_beg + lane, i_end - 1);
            if (i < a.n_rel) {
                tab.r0 = a.t_begin[a.t_lo + i];
                tab.nrows = a.t_end[a.t_lo + i] - tab.r0;
                tab.wrel = a.w_per_rel ? (a.wg_items ? a.wg_items[G + 1 + i] : a.s_rel[tab.r0]) : 0;
            } else {
                tab.r0 = a.row_lo + (i - a.n_rel) * 32;
                tab.nrows = min(32, a.row_hi - tab.r0);
                tab.wrel = -1;
            }
        }
        auto get_item = [&](int i) { return i - i_beg < 64 ? Base::item_at(a, tab, i - i_beg) : Base::item(a, i); };
        Item cur;
        float4 va[WPT], vb[WPT];
        int cnta = 1, cntb = 1, zm = 0;
        int nrow[WPT];
        int ncnt = 1;
        int crow[WPT], c0;
        int r1[WPT];
        if (rec != nullptr) {  // the first three items' row numbers from the range's record (one round)
            const int wr = ld_uniform(rec, 2);
            cur.r0 = ld_uniform(rec, 3);
            cur.nrows = ld_uniform(rec, 4);
            cur.root = wr < 0;
            cur.w = cur.root ? a.Wroot : a.W + (size_t)wr * K * N;
            constexpr int W4 = K / 4;
#pragma unroll
            for (int j = 0; j < WPT; ++j) {
                const int q = (tid + j * kThreads) / W4;
                crow[j] = rec[8 + q];
                r1[j] = rec[8 + 32 + q];
                nrow[j] = rec[8 + 64 + q];
            }
            c0 = DGRAD ? rec[8 + 96 + (tid & 31)] : 1;
            cnta = DGRAD ? rec[8 + 128 + (tid & 31)] : 1;
            ncnt = DGRAD ? rec[8 + 160 + (tid & 31)] : 1;
        } else {
            cur = get_item(i_beg);
            Base::gather_idx(a, cur, tid, crow, c0);
            Base::gather_idx(a, get_item(min(i_beg + 1, i_end - 1)), tid, r1, cnta);
            Base::gather_idx(a, get_item(min(i_beg + 2, i_end - 1)), tid, nrow, ncnt);
        }
        float wf[NS][8];
        load_b_raw(cur.w, wave, lane, wf);
        Base::issue_rows(a, tid, crow, vb, zm);
        stamp_pro(3);
        Base::issue_rows(a, tid, r1, va, zm);
        bf16x8 b[NS][3];
        split_b(wf, b);
        stamp_pro(4);
        commit(cur, tid, vb, c0, As, Sc);
        stamp_pro(5);
        __syncthreads();

        constexpr int SPG = (16 + NS - 1) / NS;  // previous item's stores per k-step
        // store offsets: lane part (column, lane half) in a VGPR, row part (r) a constant soffset
        const int col_b = (wave * 32 + c) * 4 + h * (4 * N * 4);
        float prev[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) prev[r] = 0.0f;
        __amdgpu_buffer_rsrc_t prev_rsrc = __builtin_amdgcn_make_buffer_rsrc(a.Y, (short)0, 0, 0x00020000);
        int buf = 0;
        auto step = [&](int i, float4 (&vc)[WPT], int& cntc, float4 (&vn)[WPT], int& cntn) {
            stamp(i - i_beg, 0);
            const bool has_next = i + 1 < i_end;
            const Item nxt = has_next ? get_item(i + 1) : cur;
            {  // unconditional (past the range: the last item's rows again), so no register
               // shuffle waits on these loads at the top of the item
                int zn;
                Base::issue_rows(a, tid, nrow, vn, zn);
                cntn = ncnt;
                Base::gather_idx(a, get_item(min(i + 3, i_end - 1)), tid, nrow, ncnt);
            }
            const bool new_w = nxt.w != cur.w;
            const int nr = has_next ? nxt.nrows : 0;  // last item: the commit writes zeros nobody reads
            const __bf16* Ab = As + buf * 3 * PLANE + c * LDAB + 8 * h;
            __bf16* An = As + (buf ^ 1) * 3 * PLANE;
            if constexpr (DGRAD) Sc[(buf ^ 1) * 32 + (tid & 31)] = 1.0f / (float)cntc;  // same value per tid & 31
            f32x16 hi, lo;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                hi[r] = 0.0f;
                lo[r] = 0.0f;
            }
            bf16x8 f0 = *reinterpret_cast<const bf16x8*>(Ab);
            bf16x8 f1 = *reinterpret_cast<const bf16x8*>(Ab + PLANE);
            bf16x8 f2 = *reinterpret_cast<const bf16x8*>(Ab + 2 * PLANE);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const bf16x8 a0 = f0, a1 = f1, a2 = f2;
                if (s + 1 < NS) {
                    f0 = *reinterpret_cast<const bf16x8*>(Ab + 16 * (s + 1));
                    f1 = *reinterpret_cast<const bf16x8*>(Ab + PLANE + 16 * (s + 1));
                    f2 = *reinterpret_cast<const bf16x8*>(Ab + 2 * PLANE + 16 * (s + 1));
                }
                lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b[s][0], lo, 0, 0, 0);
                lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[s][1], lo, 0, 0, 0);
                lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[s][2], lo, 0, 0, 0);
                lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[s][0], lo, 0, 0, 0);
                lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[s][1], lo, 0, 0, 0);
                hi = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[s][0], hi, 0, 0, 0);
#pragma unroll
                for (int u = 0; u < SPG; ++u) {
                    const int r = s * SPG + u;
                    if (r < 16)
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(prev[r]), prev_rsrc, col_b,
                                                              ((r & 3) + 8 * (r >> 2)) * (N * 4), 16);
                }
                // parts of the next tile: part j in k-step 1 + j·NS / WPT
#pragma unroll
                for (int j = 0; j < WPT; ++j)
                    if (s == 1 + (j * NS) / WPT) commit_part(j, tid, nr, vc[j], An);
                if (s + 1 < NS) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);  // next fragments
#pragma unroll
                for (int m = 0; m < 6; ++m) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
                    __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);  // VALU
                    if (m < 3) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // LDS write
                    if (m < SPG) __builtin_amdgcn_sched_group_barrier(0x040, 1, 0);  // store
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            stamp(i - i_beg, 1);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                prev[r] = hi[r] + lo[r];
                if constexpr (DGRAD) {
                    if (!cur.root) prev[r] = prev[r] * Sc[buf * 32 + (r & 3) + 8 * (r >> 2) + 4 * h];
                }
            }
            {
                float* Yt = cur.root ? a.Yroot + (size_t)(cur.r0 - a.row_lo) * N : a.Y + (size_t)(cur.r0 - a.sel_b) * N;
                const int bytes = __builtin_amdgcn_readfirstlane(cur.nrows) * N * 4;
                prev_rsrc = __builtin_amdgcn_make_buffer_rsrc(Yt, (short)0, bytes, 0x00020000);
            }
            if (new_w) {
                stamp(i - i_beg, 2);
                load_b(nxt.w, wave, lane, b);
            }
            stamp(i - i_beg, 3);
            __syncthreads();
            stamp(i - i_beg, 4);
            cur = nxt;
            buf ^= 1;
        };
        for (int i = i_beg; i < i_end; i += 2) {
            step(i, va, cnta, vb, cntb);
            if (i + 1 < i_end) step(i + 1, vb, cntb, va, cnta);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(prev[r]), prev_rsrc, col_b, ((r & 3) + 8 * (r >> 2)) * (N * 4), 16);
        stamp_end();
    }

    __device__ static void run(const RelGemmArgs& a, __bf16* smem) {
        __bf16* As = smem;                                            // [2][3 planes][32][LDAB]
        float* Sc = reinterpret_cast<float*>(smem + 2 * 3 * PLANE);  // [2][32] dgrad row scales
        const int tid = threadIdx.x;
        const int lane = tid & 63, c = lane & 31, h = lane >> 5;
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        const int n_items = a.n_rel + a.n_root;
        const int G = (int)gridDim.x;
        const int g = (int)blockIdx.x & 7, q = G >> 3, rem = G & 7;
        const int rng = a.wg_cus > 0 ? wg_pair_range((int)blockIdx.x, a.wg_cus) : g * q + min(g, rem) + ((int)blockIdx.x >> 3);
        // equal item counts, or the host's cost-balanced ranges (a weight switch costs an exposed
        // slice load: MPGNN_OPT_GEMM_SWITCH_COST)
        const int i_beg = a.wg_items ? ld_uniform(a.wg_items, rng) : (int)((long long)rng * n_items / G);
        const int i_end = a.wg_items ? ld_uniform(a.wg_items, rng + 1) : (int)((long long)(rng + 1) * n_items / G);
        if (i_beg >= i_end) return;

        // A rows are gathered TWO items ahead (the bf16 chain of an item is 2.67x shorter than the
        // fp32 one: one item of lead left the commit waiting on the gathers): rows of item i+1
        // sit in one register set (committed three quarters into item i's chain), rows of item
        // i+2 are issued into the other at the top of item i, and the row numbers of item i+3
        // are loaded then. The two sets swap roles every item (the loop body is instantiated
        // twice), so no register copy waits on loads in flight.
        const ItemTable tab = Base::item_table(a, i_beg, i_end, lane);
        auto get_item = [&](int i) { return i - i_beg < 64 ? Base::item_at(a, tab, i - i_beg) : Base::item(a, i); };
        Item cur = get_item(i_beg);
        float4 va[WPT], vb[WPT];
        int cnta = 1, cntb = 1, zm = 0;
        {
            int crow[WPT], c0;
            Base::gather_idx(a, cur, tid, crow, c0);
            Base::issue_rows(a, tid, crow, va, zm);
            commit(cur, tid, va, c0, As, Sc);
        }
        int nrow[WPT];
        int ncnt = 1;
        if (i_beg + 1 < i_end) {
            int r1[WPT];
            Base::gather_idx(a, get_item(i_beg + 1), tid, r1, cnta);
            Base::issue_rows(a, tid, r1, va, zm);
        }
        if (i_beg + 2 < i_end) Base::gather_idx(a, get_item(i_beg + 2), tid, nrow, ncnt);
        bf16x8 b[NS][3];
        load_b(cur.w, wave, lane, b);
        __syncthreads();

        constexpr int SPG = (16 + NS - 1) / NS;  // previous item's stores per k-step
        constexpr int kCommitAt = (3 * NS) / 4;  // k-step after which the next tile is committed
        const int col_b = (wave * 32 + c) * 4;
        float prev[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) prev[r] = 0.0f;
        __amdgpu_buffer_rsrc_t prev_rsrc = __builtin_amdgcn_make_buffer_rsrc(a.Y, (short)0, 0, 0x00020000);
        auto store_prev = [&](int r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
            // cache policy sc1 (aux bit 4): measured 49.8 -> 48.7 us at C3, the combine unchanged
            // (nt, aux bit 1, cost the combine 22.8 -> 28.3 us: Y left the MALL)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(prev[r]), prev_rsrc, row * (N * 4) + col_b, 0, 16);
        };
        int buf = 0;
        // item i: vc = rows of item i+1 (committed in this item), vn = receives rows of item i+2
        auto step = [&](int i, float4 (&vc)[WPT], int& cntc, float4 (&vn)[WPT], int& cntn) {
            const bool has_next = i + 1 < i_end;
            const Item nxt = has_next ? get_item(i + 1) : cur;
            if (i + 2 < i_end) {
                int zn;
                Base::issue_rows(a, tid, nrow, vn, zn);
                cntn = ncnt;
                if (i + 3 < i_end) Base::gather_idx(a, get_item(i + 3), tid, nrow, ncnt);
            }
            const bool new_w = nxt.w != cur.w;
            const __bf16* Ab = As + buf * 3 * PLANE + c * LDAB + 8 * h;
            f32x16 hi, lo;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                hi[r] = 0.0f;
                lo[r] = 0.0f;
            }
            bf16x8 f0 = *reinterpret_cast<const bf16x8*>(Ab);
            bf16x8 f1 = *reinterpret_cast<const bf16x8*>(Ab + PLANE);
            bf16x8 f2 = *reinterpret_cast<const bf16x8*>(Ab + 2 * PLANE);
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const bf16x8 a0 = f0, a1 = f1, a2 = f2;
                if (s + 1 < NS) {
                    f0 = *reinterpret_cast<const bf16x8*>(Ab + 16 * (s + 1));
                    f1 = *reinterpret_cast<const bf16x8*>(Ab + PLANE + 16 * (s + 1));
                    f2 = *reinterpret_cast<const bf16x8*>(Ab + 2 * PLANE + 16 * (s + 1));
                }
                lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b[s][0], lo, 0, 0, 0);
                lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[s][1], lo, 0, 0, 0);
                lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[s][2], lo, 0, 0, 0);
                lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[s][0], lo, 0, 0, 0);
                lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[s][1], lo, 0, 0, 0);
                hi = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[s][0], hi, 0, 0, 0);
#pragma unroll
                for (int u = 0; u < SPG; ++u)
                    if (s * SPG + u < 16) store_prev(s * SPG + u);
                if (s == kCommitAt - 1 && has_next) commit(nxt, tid, vc, cntc, As + (buf ^ 1) * 3 * PLANE, Sc + (buf ^ 1) * 32);
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                prev[r] = hi[r] + lo[r];
                if constexpr (DGRAD) {  // row scale 1/cnt of relation rows
                    if (!cur.root) prev[r] = prev[r] * Sc[buf * 32 + (r & 3) + 8 * (r >> 2) + 4 * h];
                }
            }
            {
                float* Yt = cur.root ? a.Yroot + (size_t)(cur.r0 - a.row_lo) * N : a.Y + (size_t)(cur.r0 - a.sel_b) * N;
                const int bytes = __builtin_amdgcn_readfirstlane(cur.nrows) * N * 4;
                prev_rsrc = __builtin_amdgcn_make_buffer_rsrc(Yt, (short)0, bytes, 0x00020000);
            }
            if (new_w) load_b(nxt.w, wave, lane, b);  // after the chain: the slice registers are free
            __syncthreads();
            cur = nxt;
            buf ^= 1;
        };
        for (int i = i_beg; i < i_end; i += 2) {
            step(i, va, cnta, vb, cntb);
            if (i + 1 < i_end) step(i + 1, vb, cntb, va, cnta);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) store_prev(r);
    }
};

template <int KB, bool DGRAD, bool IL = false>
__global__ __launch_bounds__(kThreads, 2) void rel_gemm_bf3_kernel(RelGemmArgs a) {
    extern __shared__ __bf16 smem_bf[];
    if (a.zero != nullptr)  // a few words, one store per thread at most (read by a later launch only)
        for (int i = (int)(blockIdx.x * kThreads + threadIdx.x); i < a.zero_words; i += (int)(gridDim.x * kThreads))
            a.zero[i] = 0u;
    if constexpr (IL) RelGemmBf3<KB, DGRAD>::run_il(a, smem_bf);
    else RelGemmBf3<KB, DGRAD>::run(a, smem_bf);
}

// ----------------------------------------------------------------------------------------
// rel_gemm_w1_kernel — the bf16-split GEMM of rel_gemm_bf3_kernel (K = N = 128: the same
// items' products, the same MFMA instruction, k-step order and six-product order, so the same
// bits) with ONE workgroup per CU: one wave per SIMD owning the whole 512-entry register file.
// What that buys over two workgroups of 32-row items:
//   * 64-row items (two 32-row sub-tiles of one relation, or 64 node rows): one barrier, one
//     epilogue hand-off and one item-table step per 64 rows, 96 MFMAs per wave per item;
//   * the next relation's weight slice loaded into a second register set at the top of the item
//     before the switch (its latency hidden by that item's chain) and split after the chain —
//     rel_gemm_bf3_kernel's registers held one slice, so each switch exposed a slice load
//     (stamped: ~85 % of an item);
//   * half the launch's load storm (256 workgroups fetch their first slice and rows, not 512).
// Item table (gemm_w1_items, host-built per plan): [G + 1] first item of each workgroup's
// range (XCD-contiguous ranges, balanced by sub-tiles), then per item {r0, nrows, weight index
// (-1: root)}. Rows are gathered two items ahead, the next item's tile is committed to the other
// LDS buffer inside the k-steps (one float4 part per k-step), the previous item's outputs are
// stored inside the next item's chain — rel_gemm_bf3_kernel's pipeline at twice the rows.
// ----------------------------------------------------------------------------------------
template <bool DGRAD>
struct RelGemmW1 {
    static constexpr int K = 128;
    static constexpr int N = 128;
    static constexpr int NS = K / 16;              // k-steps
    static constexpr int LDAB = K + 8;             // bf16 row stride of an A plane (conflict-free b128 reads)
    static constexpr int ROWS = 64;                // rows per item
    static constexpr int PLANE = ROWS * LDAB;      // bf16 per plane
    static constexpr int WPT = ROWS * (K / 4) / kThreads;  // 8 float4 of an A tile per thread
    static constexpr int W4 = K / 4;

    static constexpr size_t lds_bytes() { return (size_t)2 * 3 * PLANE * 2 + 2 * ROWS * sizeof(float); }

    struct Item {
        int r0, nrows, root;
        const float* w;
    };
    __device__ static __forceinline__ Item item(const RelGemmArgs& a, int i, int G) {
        const int* t = a.wg_items + G + 1 + 3 * i;
        Item it;
        it.r0 = ld_uniform(t, 0);
        it.nrows = ld_uniform(t, 1);
        const int wr = ld_uniform(t, 2);
        it.root = wr < 0;
        it.w = it.root ? a.Wroot : a.W + (size_t)wr * K * N;
        return it;
    }
    // row of thread part j: (tid >> 5) + 8 j; forward A row = s_src (x row, or compact mean row
    // -(v+1)), dgrad = dout row s_row (scaled 1 / cnt at the output); root items: the node row
    __device__ static __forceinline__ void gather_idx(const RelGemmArgs& a, const Item& it, int tid, int (&row)[WPT],
                                                      int& cnt) {
#pragma unroll
        for (int j = 0; j < WPT; ++j) row[j] = it.r0 + min((tid >> 5) + 8 * j, it.nrows - 1);
        cnt = 1;
        if (!it.root) {
            if constexpr (DGRAD) {
                cnt = a.s_cnt[it.r0 + min(tid & 63, it.nrows - 1)];
#pragma unroll
                for (int j = 0; j < WPT; ++j) row[j] = a.s_row[row[j]];
            } else {
#pragma unroll
                for (int j = 0; j < WPT; ++j) row[j] = a.s_src[row[j]];
            }
        }
    }
    __device__ static __forceinline__ void issue_rows(const RelGemmArgs& a, int tid, const int (&row)[WPT],
                                                      float4 (&v)[WPT]) {
        const int c4 = (tid & 31) * 4;
#pragma unroll
        for (int j = 0; j < WPT; ++j) {
            const float* base;
            if constexpr (DGRAD) base = a.Aroot + (size_t)row[j] * K;
            else base = row[j] >= 0 ? a.Aroot + (size_t)row[j] * K : a.Arel + (size_t)(-row[j] - 1 - a.m_lo) * K;
            v[j] = *reinterpret_cast<const float4*>(base + c4);
        }
    }
    __device__ static __forceinline__ void commit_part(int j, int tid, int nrows, const float4& v, __bf16* A) {
        const int r = (tid >> 5) + 8 * j;
        const float4 x = r < nrows ? v : make_float4(0.f, 0.f, 0.f, 0.f);
        __bf16 p0[4], p1[4], p2[4];
        split3_bf16(x.x, p0[0], p1[0], p2[0]);
        split3_bf16(x.y, p0[1], p1[1], p2[1]);
        split3_bf16(x.z, p0[2], p1[2], p2[2]);
        split3_bf16(x.w, p0[3], p1[3], p2[3]);
        __bf16* d = A + r * LDAB + (tid & 31) * 4;
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        *reinterpret_cast<bf16x4*>(d) = bf16x4{p0[0], p0[1], p0[2], p0[3]};
        *reinterpret_cast<bf16x4*>(d + PLANE) = bf16x4{p1[0], p1[1], p1[2], p1[3]};
        *reinterpret_cast<bf16x4*>(d + 2 * PLANE) = bf16x4{p2[0], p2[1], p2[2], p2[3]};
    }
    __device__ static __forceinline__ void commit(int tid, int nrows, const float4 (&v)[WPT], __bf16* A) {
#pragma unroll
        for (int j = 0; j < WPT; ++j) commit_part(j, tid, nrows, v[j], A);
    }
    // the wave's weight slice (raw fp32): f[s][j] = B(16s + 8h + j, 32·wave + c)
    __device__ static __forceinline__ void load_b_raw(const float* w, int wave, int lane, float (&f)[NS][8]) {
        RelGemmBf3<2, DGRAD>::load_b_raw(w, wave, lane, f);
    }
    __device__ static __forceinline__ void split_b(const float (&f)[NS][8], bf16x8 (&b)[NS][3]) {
        RelGemmBf3<2, DGRAD>::split_b(f, b);
    }

    __device__ static void run(const RelGemmArgs& a, __bf16* smem) {
        __bf16* As = smem;                                            // [2][3 planes][64][LDAB]
        float* Sc = reinterpret_cast<float*>(smem + 2 * 3 * PLANE);  // [2][64] dgrad row scales
        const int tid = threadIdx.x;
        const int lane = tid & 63, c = lane & 31, h = lane >> 5;
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        const int G = (int)gridDim.x;
        const int rng = ((int)blockIdx.x & 7) * (G >> 3) + ((int)blockIdx.x >> 3);  // XCD-contiguous ranges
        const int i_beg = ld_uniform(a.wg_items, rng);
        const int i_end = ld_uniform(a.wg_items, rng + 1);
        if (i_beg >= i_end) return;
        stamp_id();

        Item cur = item(a, i_beg, G);
        float4 va[WPT], vb[WPT];
        int cnta = 1, cntb = 1;
        int nrow[WPT];
        int ncnt = 1;
        {
            int crow[WPT], c0, r1[WPT];
            gather_idx(a, cur, tid, crow, c0);
            gather_idx(a, item(a, min(i_beg + 1, i_end - 1), G), tid, r1, cnta);
            gather_idx(a, item(a, min(i_beg + 2, i_end - 1), G), tid, nrow, ncnt);
            float wf[NS][8];
            load_b_raw(cur.w, wave, lane, wf);
            issue_rows(a, tid, crow, vb);
            issue_rows(a, tid, r1, va);
            stamp_pro(3);
            bf16x8 b0[NS][3];
            split_b(wf, b0);
            stamp_pro(4);
            commit(tid, cur.nrows, vb, As);
            stamp_pro(5);
            if constexpr (DGRAD) {
                if (tid < ROWS) Sc[tid] = 1.0f / (float)c0;
            }
            __syncthreads();
            run_items(a, As, Sc, tid, lane, c, h, wave, G, i_beg, i_end, cur, va, vb, cnta, cntb, nrow, ncnt, b0);
        }
    }

    __device__ static __forceinline__ void run_items(const RelGemmArgs& a, __bf16* As, float* Sc, int tid, int lane,
                                                     int c, int h, int wave, int G, int i_beg, int i_end, Item cur,
                                                     float4 (&va)[WPT], float4 (&vb)[WPT], int& cnta, int& cntb,
                                                     int (&nrow)[WPT], int& ncnt, bf16x8 (&b)[NS][3]) {
        constexpr int SPG = (32 + NS - 1) / NS;  // previous item's stores per k-step (2 sub-tiles × 16)
        const int col_b = (wave * 32 + c) * 4 + h * (4 * N * 4);
        float prev[2][16];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int r = 0; r < 16; ++r) prev[u][r] = 0.0f;
        __amdgpu_buffer_rsrc_t prev_rsrc = __builtin_amdgcn_make_buffer_rsrc(a.Y, (short)0, 0, 0x00020000);
        float wf[NS][8];  // the next relation's slice, raw (loaded one item ahead of its first use)
        int buf = 0;
        auto step = [&](int i, float4 (&vc)[WPT], int& cntc, float4 (&vn)[WPT], int& cntn) {
            stamp(i - i_beg, 0);
            const bool has_next = i + 1 < i_end;
            const Item nxt = has_next ? item(a, i + 1, G) : cur;
            {  // unconditional (past the range: the last item's rows again)
                issue_rows(a, tid, nrow, vn);
                cntn = ncnt;
                gather_idx(a, item(a, min(i + 3, i_end - 1), G), tid, nrow, ncnt);
            }
            const bool new_w = nxt.w != cur.w;
            if (new_w) load_b_raw(nxt.w, wave, lane, wf);
            const int nr = has_next ? nxt.nrows : 0;
            const __bf16* Ab = As + buf * 3 * PLANE + c * LDAB + 8 * h;
            __bf16* An = As + (buf ^ 1) * 3 * PLANE;
            if constexpr (DGRAD) {
                if (tid < ROWS) Sc[(buf ^ 1) * ROWS + tid] = 1.0f / (float)cntc;
            }
            f32x16 hi0, lo0, hi1, lo1;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                hi0[r] = 0.0f;
                lo0[r] = 0.0f;
                hi1[r] = 0.0f;
                lo1[r] = 0.0f;
            }
            bf16x8 f0 = *reinterpret_cast<const bf16x8*>(Ab);
            bf16x8 f1 = *reinterpret_cast<const bf16x8*>(Ab + PLANE);
            bf16x8 f2 = *reinterpret_cast<const bf16x8*>(Ab + 2 * PLANE);
            bf16x8 g0 = *reinterpret_cast<const bf16x8*>(Ab + 32 * LDAB);
            bf16x8 g1 = *reinterpret_cast<const bf16x8*>(Ab + PLANE + 32 * LDAB);
            bf16x8 g2 = *reinterpret_cast<const bf16x8*>(Ab + 2 * PLANE + 32 * LDAB);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const bf16x8 a0 = f0, a1 = f1, a2 = f2, e0 = g0, e1 = g1, e2 = g2;
                if (s + 1 < NS) {
                    f0 = *reinterpret_cast<const bf16x8*>(Ab + 16 * (s + 1));
                    f1 = *reinterpret_cast<const bf16x8*>(Ab + PLANE + 16 * (s + 1));
                    f2 = *reinterpret_cast<const bf16x8*>(Ab + 2 * PLANE + 16 * (s + 1));
                    g0 = *reinterpret_cast<const bf16x8*>(Ab + 32 * LDAB + 16 * (s + 1));
                    g1 = *reinterpret_cast<const bf16x8*>(Ab + PLANE + 32 * LDAB + 16 * (s + 1));
                    g2 = *reinterpret_cast<const bf16x8*>(Ab + 2 * PLANE + 32 * LDAB + 16 * (s + 1));
                }
                lo0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b[s][0], lo0, 0, 0, 0);
                lo1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(e2, b[s][0], lo1, 0, 0, 0);
                lo0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[s][1], lo0, 0, 0, 0);
                lo1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(e1, b[s][1], lo1, 0, 0, 0);
                lo0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[s][2], lo0, 0, 0, 0);
                lo1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(e0, b[s][2], lo1, 0, 0, 0);
                lo0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[s][0], lo0, 0, 0, 0);
                lo1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(e1, b[s][0], lo1, 0, 0, 0);
                lo0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[s][1], lo0, 0, 0, 0);
                lo1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(e0, b[s][1], lo1, 0, 0, 0);
                hi0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[s][0], hi0, 0, 0, 0);
                hi1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(e0, b[s][0], hi1, 0, 0, 0);
#pragma unroll
                for (int v = 0; v < SPG; ++v) {
                    const int q = s * SPG + v;  // 0..31: sub-tile q >> 4, register q & 15
                    if (q < 32) {
                        const int u = q >> 4, r = q & 15;
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(prev[u][r]), prev_rsrc, col_b,
                                                              (32 * u + (r & 3) + 8 * (r >> 2)) * (N * 4), 16);
                    }
                }
                // part j of the next tile in k-step j (WPT == NS)
                commit_part(s, tid, nr, vc[s], An);
                if (s + 1 < NS) __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);  // next fragments
#pragma unroll
                for (int m = 0; m < 12; ++m) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);             // one MFMA
                    __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);             // VALU
                    if (m < 3) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // LDS write
                    if (m < SPG) __builtin_amdgcn_sched_group_barrier(0x040, 1, 0);  // store
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            stamp(i - i_beg, 1);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                prev[0][r] = hi0[r] + lo0[r];
                prev[1][r] = hi1[r] + lo1[r];
                if constexpr (DGRAD) {
                    if (!cur.root) {
                        prev[0][r] = prev[0][r] * Sc[buf * ROWS + (r & 3) + 8 * (r >> 2) + 4 * h];
                        prev[1][r] = prev[1][r] * Sc[buf * ROWS + 32 + (r & 3) + 8 * (r >> 2) + 4 * h];
                    }
                }
            }
            {
                float* Yt = cur.root ? a.Yroot + (size_t)(cur.r0 - a.row_lo) * N : a.Y + (size_t)(cur.r0 - a.sel_b) * N;
                const int bytes = __builtin_amdgcn_readfirstlane(cur.nrows) * N * 4;
                prev_rsrc = __builtin_amdgcn_make_buffer_rsrc(Yt, (short)0, bytes, 0x00020000);
            }
            if (new_w) {
                stamp(i - i_beg, 2);
                split_b(wf, b);
            }
            stamp(i - i_beg, 3);
            __syncthreads();
            stamp(i - i_beg, 4);
            cur = nxt;
            buf ^= 1;
        };
        for (int i = i_beg; i < i_end; i += 2) {
            step(i, va, cnta, vb, cntb);
            if (i + 1 < i_end) step(i + 1, vb, cntb, va, cnta);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(prev[u][r]), prev_rsrc, col_b,
                                                      (32 * u + (r & 3) + 8 * (r >> 2)) * (N * 4), 16);
        stamp_end();
    }
};

template <bool DGRAD>
__global__ __launch_bounds__(kThreads, 1) void rel_gemm_w1_kernel(RelGemmArgs a) {
    extern __shared__ __bf16 smem_bf[];
    RelGemmW1<DGRAD>::run(a, smem_bf);
}

// ----------------------------------------------------------------------------------------
// single_bf3_kernel — the whole unsharded mode-SINGLE layer (CustomRGCNConv over one relation,
// mp_rgcn_layer.py:231-268, + the model's ReLU) in one launch on the bf16 matrix cores:
//     out[i] = act((mean_i @ W + x_i @ root) + bias)      mean_i = 0 without a segment
// in the reference's association (out = h @ W; out += x @ root; out += bias). A node has at
// most one segment of the relation, so a 32-row item of node rows needs no combine. The
// workgroup's eight waves split K: waves 0-3 hold the root slice and multiply the item's x
// rows, waves 4-7 hold the W slice and multiply its mean rows (node_map: x row, compact mean
// Hm row, or none), each over 32 columns with rel_gemm_bf3_kernel's exact three-piece split
// (six products, fp32 accumulation); the mean half hands its tile to the x half through LDS,
// which adds, finishes and stores. Persistent over items; the rows of item i+1 are gathered
// during item i, their node_map entries one item earlier still.
//   C3 (455 items of 32 rows): one item per workgroup is latency, not MFMA, bound — the split
//   halves each wave's chain and the bf16 pieces cut it 2.67x against the fp32 K = 256 chain.
// ----------------------------------------------------------------------------------------
struct SingleBf3Args {
    const float* x;       // [N][K]
    const float* H;       // compact means, row m - m_lo
    const int* node_map;  // [N]: s_src + 1 (x row), s_src (< 0: Hm row), 0 (no segment)
    int m_lo, m_rows, N;
    // non-null (round 6, MPGNN_OPT_SINGLE_FOLD): the mean half computes a multi-edge segment's
    // mean itself from the compact lists — Σ over 32-edge pieces (each summed in edge order from
    // 0.0f) in piece order, / cnt: the means kernel's exact arithmetic — instead of reading H;
    // H_out (nullable, training) receives those rows for the backward
    const int* m_ptr;
    const int* em_col;
    const int* m_cnt;
    float* H_out;
    const float* W;       // [K][128]
    const float* root;    // [K][128]
    const float* bias;    // nullable [128]
    int relu;
    float* out;           // [N][128]
};

constexpr int kSingleThreads = 512;

template <int KB>
struct SingleBf3 {
    using Gemm = RelGemmBf3<KB, false>;
    static constexpr int K = 64 * KB, N = 128, NS = K / 16, LDAB = K + 8, PLANE = 32 * LDAB;
    static constexpr int W4 = K / 4;              // float4 per row
    static constexpr int WPT = 32 * W4 / 256;     // float4 per thread of a half
    static constexpr int LDO = N + 4;             // fp32 row stride of the exchanged tile
    static constexpr size_t lds_bytes() { return (size_t)6 * PLANE * 2 + (size_t)32 * LDO * sizeof(float); }

    // per-thread state of one item: thread t of a half holds float4 (t + 256 j) of its 32 x K tile
    struct Rows {
        int mp[WPT];
        float4 v[WPT];
    };
    // the mean half's node_map entries of item it
    __device__ static __forceinline__ void load_map(const SingleBf3Args& a, int it, bool mh, int t, Rows& q) {
        if (mh) {
#pragma unroll
            for (int j = 0; j < WPT; ++j) q.mp[j] = a.node_map[min(it * 32 + (t + j * 256) / W4, a.N - 1)];
        }
    }
    // x rows (x half) or mean rows (mean half: x row, compact mean row, or zeros) of item it;
    // indices are clamped into the tables: a bad map cannot fault
    // the fold of one multi-edge segment (global compact index mg) at float4 column c4: the
    // segment means kernel's sums (32-edge pieces, each from 0.0f in edge order, added in piece
    // order from 0.0f), then / cnt (IEEE); four edges' rows in flight
    __device__ static __forceinline__ float4 fold_mean(const SingleBf3Args& a, int mg, int c4) {
        const int e0 = a.m_ptr[mg], e1 = a.m_ptr[mg + 1];
        const float d = (float)a.m_cnt[mg];
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int ps = e0; ps < e1; ps += 32) {
            const int pe = min(ps + 32, e1);
            float4 pc = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int e = ps; e < pe; e += 4) {
                int src[4];
                float4 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) src[u] = a.em_col[min(e + u, pe - 1)];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    v[u] = *reinterpret_cast<const float4*>(a.x + (size_t)min(max(src[u], 0), a.N - 1) * K + c4);
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (e + u < pe) {
                        pc.x += v[u].x;
                        pc.y += v[u].y;
                        pc.z += v[u].z;
                        pc.w += v[u].w;
                    }
            }
            acc.x += pc.x;
            acc.y += pc.y;
            acc.z += pc.z;
            acc.w += pc.w;
        }
        return make_float4(acc.x / d, acc.y / d, acc.z / d, acc.w / d);
    }
    __device__ static __forceinline__ void issue(const SingleBf3Args& a, int it, bool mh, int t, Rows& q) {
#pragma unroll
        for (int j = 0; j < WPT; ++j) {
            const int e = t + j * 256;
            const int row = min(it * 32 + e / W4, a.N - 1);
            const int c4 = (e % W4) * 4;
            const float* base;
            bool zero = false;
            if (!mh) {
                base = a.x + (size_t)row * K;
            } else {
                const int m = q.mp[j];
                zero = m == 0;
                if (m < 0 && a.m_ptr != nullptr) {  // fold the multi-edge segment's mean here
                    const int mg = -m - 1;
                    q.v[j] = fold_mean(a, mg, c4);
                    if (a.H_out != nullptr && it * 32 + e / W4 < a.N)
                        *reinterpret_cast<float4*>(a.H_out + (size_t)(mg - a.m_lo) * K + c4) = q.v[j];
                    continue;
                }
                base = m > 0 ? a.x + (size_t)min(m - 1, a.N - 1) * K
                             : a.H + (size_t)min(max(-m - 1 - a.m_lo, 0), max(a.m_rows - 1, 0)) * K;
                if (zero) base = a.x;
            }
            q.v[j] = *reinterpret_cast<const float4*>(base + c4);
            if (zero) q.v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    // the half's tile as three bf16 planes (rows past N: zeros)
    __device__ static __forceinline__ void commit(const SingleBf3Args& a, int it, bool mh, int t, const Rows& q,
                                                  __bf16* smem) {
        __bf16* P = smem + (mh ? 3 * PLANE : 0);
#pragma unroll
        for (int j = 0; j < WPT; ++j) {
            const int e = t + j * 256;
            const int r = e / W4;
            const float4 xv = it * 32 + r < a.N ? q.v[j] : make_float4(0.f, 0.f, 0.f, 0.f);
            __bf16 p0[4], p1[4], p2[4];
            split3_bf16(xv.x, p0[0], p1[0], p2[0]);
            split3_bf16(xv.y, p0[1], p1[1], p2[1]);
            split3_bf16(xv.z, p0[2], p1[2], p2[2]);
            split3_bf16(xv.w, p0[3], p1[3], p2[3]);
            __bf16* d = P + r * LDAB + (e % W4) * 4;
            typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
            *reinterpret_cast<bf16x4*>(d) = bf16x4{p0[0], p0[1], p0[2], p0[3]};
            *reinterpret_cast<bf16x4*>(d + PLANE) = bf16x4{p1[0], p1[1], p1[2], p1[3]};
            *reinterpret_cast<bf16x4*>(d + 2 * PLANE) = bf16x4{p2[0], p2[1], p2[2], p2[3]};
        }
    }
    // the wave's 32 x 32 product of its half's tile (committed, barrier passed) with its slice
    __device__ static __forceinline__ f32x16 chain(bool mh, int c, int h, const __bf16* smem, const bf16x8 (&b)[NS][3]) {
        const __bf16* Ab = smem + (mh ? 3 * PLANE : 0) + c * LDAB + 8 * h;
        f32x16 hi, lo;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            hi[r] = 0.0f;
            lo[r] = 0.0f;
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(Ab + 16 * s);
            const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(Ab + PLANE + 16 * s);
            const bf16x8 a2 = *reinterpret_cast<const bf16x8*>(Ab + 2 * PLANE + 16 * s);
            lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b[s][0], lo, 0, 0, 0);
            lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[s][1], lo, 0, 0, 0);
            lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[s][2], lo, 0, 0, 0);
            lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[s][0], lo, 0, 0, 0);
            lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[s][1], lo, 0, 0, 0);
            hi = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[s][0], hi, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) hi[r] = hi[r] + lo[r];
        return hi;
    }
    // mean half: its tile into LDS (before a barrier); x half (after it): (mean@W + x@root) + bias, act, store
    __device__ static __forceinline__ void put_mean(int col, int h, const f32x16& acc, __bf16* smem) {
        float* Ot = reinterpret_cast<float*>(smem + 6 * PLANE);
#pragma unroll
        for (int r = 0; r < 16; ++r) Ot[((r & 3) + 8 * (r >> 2) + 4 * h) * LDO + col] = acc[r];
    }
    __device__ static __forceinline__ void finish(const SingleBf3Args& a, int it, int col, int h, float bcol,
                                                  const f32x16& acc, const __bf16* smem) {
        const float* Ot = reinterpret_cast<const float*>(smem + 6 * PLANE);
        const int r0 = it * 32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
            float o = (Ot[row * LDO + col] + acc[r]) + bcol;
            if (a.relu) o = relu_f(o);
            if (r0 + row < a.N) a.out[(size_t)(r0 + row) * N + col] = o;
        }
    }
};

template <int KB>
__global__ __launch_bounds__(kSingleThreads, 1) void single_bf3_kernel(SingleBf3Args a) {
    using S = SingleBf3<KB>;
    extern __shared__ __bf16 smem_bf[];
    const int tid = threadIdx.x, lane = tid & 63, c = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool mh = wave >= 4;  // wave-uniform: the mean half
    const int t = tid & 255;    // thread within its half
    const int wq = wave & 3;    // column block of the wave
    const int n_items = (a.N + 31) / 32;
    const int G = (int)gridDim.x;
    const int g = (int)blockIdx.x & 7, q = G >> 3, rem = G & 7;
    const int rng = g * q + min(g, rem) + ((int)blockIdx.x >> 3);  // consecutive items on one XCD
    const int i_beg = (int)((long long)rng * n_items / G);
    const int i_end = (int)((long long)(rng + 1) * n_items / G);
    if (i_beg >= i_end) return;

    typename S::Rows rows;
    S::load_map(a, i_beg, mh, t, rows);
    S::issue(a, i_beg, mh, t, rows);
    if (i_beg + 1 < i_end) S::load_map(a, i_beg + 1, mh, t, rows);
    bf16x8 b[S::NS][3];
    S::Gemm::load_b(mh ? a.W : a.root, wq, lane, b);
    S::commit(a, i_beg, mh, t, rows, smem_bf);
    if (i_beg + 1 < i_end) S::issue(a, i_beg + 1, mh, t, rows);
    if (i_beg + 2 < i_end) S::load_map(a, i_beg + 2, mh, t, rows);
    const int col = wq * 32 + c;
    const float bcol = a.bias != nullptr ? a.bias[col] : 0.0f;
    __syncthreads();

    for (int i = i_beg; i < i_end; ++i) {
        const f32x16 acc = S::chain(mh, c, h, smem_bf, b);
        if (mh) S::put_mean(col, h, acc, smem_bf);
        __syncthreads();  // the mean tile is in LDS; both A tiles are free
        if (!mh) S::finish(a, i, col, h, bcol, acc, smem_bf);
        if (i + 1 < i_end) S::commit(a, i + 1, mh, t, rows, smem_bf);
        if (i + 2 < i_end) S::issue(a, i + 2, mh, t, rows);
        if (i + 3 < i_end) S::load_map(a, i + 3, mh, t, rows);
        __syncthreads();  // the next item's A tiles are in LDS; the mean tile is free
    }
}

// ----------------------------------------------------------------------------------------
// rel_gemm_bf3w_kernel — the K = 256, N = 256 transform (C5: F_in = F_out = 256) and its dgrad
// on the bf16 matrix cores with the exact three-piece split of the fp32 operands. A wave's
// K × 32 weight slice in bf16 pieces would take 192 VGPRs at K = 256, so the workgroup's eight
// waves SPLIT K: waves 0-3 multiply k ∈ [0, 128), waves 4-7 k ∈ [128, 256), each over one
// 32-column strip of the workgroup's 128 columns (96 VGPRs of slice, as at K = 128). The six
// products of a k-step go into ONE fp32 accumulator (each MFMA adds its 16 exact products and
// rounds once: six roundings per 16 k against the fp32 chain's sixteen). The upper half hands its
// 32 × 128 partial tile to the lower half through LDS (double-buffered), which adds
// (lower + upper), applies the dgrad row scale, and stores the tile DURING the next item's chain
// (bounds-checked buffer stores, two per k-step); the next item's A tile is committed to the other
// LDS buffer three quarters into the chain and the rows of the item after it are issued right
// then: one barrier per item. The two 128-column blocks of an item are two workgroups eight block
// ids apart — one XCD, same item range — so the second gather of the A rows hits that XCD's L2.
// Items, row gathers and outputs as rel_gemm_kernel (RelGemmArgs: relation tiles of segments,
// then node rows; forward A = x row / compact mean row, dgrad A = dout[node_1] scaled by 1/cnt).
// ----------------------------------------------------------------------------------------
__device__ int g_one_i32 = 1;  // RelGemmBf3W::row_val_load's stand-in (never written)

template <bool DGRAD>
struct RelGemmBf3W {
    static constexpr int K = 256, N = 256, KH = 128, NS = KH / 16, LDAB = KH + 8, PLANE = 32 * LDAB;
    static constexpr int WPT = 4;                 // float4 per thread: 32 rows × 32 float4 of a K half / 256
    static constexpr int LDO = 128 + 4;           // fp32 row stride of the exchanged partial tile
    // [2 buffers][2 halves][3 planes] bf16 + [2][32][LDO] exchange tiles + [3][32] row scales
    static constexpr size_t lds_bytes() {
        return (size_t)12 * PLANE * 2 + (size_t)2 * 32 * LDO * sizeof(float) + 3 * 32 * sizeof(float);
    }
    struct Item {
        int r0, nrows, root;
        const float* w;
    };
    // Item descriptors of a 64-item window, lane l holding item base + l (vector loads, read back
    // with readlane: no dependent scalar loads on the item loop's critical path)
    struct Tab {
        int r0, nrows, wrel;  // wrel: weight index, -1 = root
    };
    __device__ static __forceinline__ Tab load_tab(const RelGemmArgs& a, int base, int i_end, int lane) {
        Tab tb;
        const int i = min(base + lane, i_end - 1);
        if (i < a.n_rel) {
            tb.r0 = a.t_begin[a.t_lo + i];
            tb.nrows = a.t_end[a.t_lo + i] - tb.r0;
            tb.wrel = a.w_per_rel ? a.s_rel[tb.r0] : 0;
        } else {
            tb.r0 = a.row_lo + (i - a.n_rel) * 32;
            tb.nrows = min(32, a.row_hi - tb.r0);
            tb.wrel = -1;
        }
        return tb;
    }
    __device__ static __forceinline__ Item item_at(const RelGemmArgs& a, const Tab& tb, int k) {
        Item it;
        it.r0 = readlane(tb.r0, k);
        it.nrows = readlane(tb.nrows, k);
        const int wr = readlane(tb.wrel, k);
        it.root = wr < 0;
        it.w = it.root ? a.Wroot : a.W + (size_t)wr * K * N;
        return it;
    }
    // source row of each of the thread's WPT tile rows (row t/32 + 8j of the item)
    __device__ static __forceinline__ void gather_idx(const RelGemmArgs& a, const Item& it, int t, int (&row)[WPT]) {
#pragma unroll
        for (int j = 0; j < WPT; ++j) row[j] = it.r0 + min(t / 32 + 8 * j, it.nrows - 1);
        if (!it.root) {
            if constexpr (DGRAD) {
#pragma unroll
                for (int j = 0; j < WPT; ++j) row[j] = a.s_row[row[j]];
            } else {
#pragma unroll
                for (int j = 0; j < WPT; ++j) row[j] = a.s_src[row[j]];
            }
        }
    }
    __device__ static __forceinline__ void issue(const RelGemmArgs& a, int kh, int t, const int (&row)[WPT],
                                                 float4 (&v)[WPT]) {
        const int c4 = kh * KH + (t & 31) * 4;
#pragma unroll
        for (int j = 0; j < WPT; ++j) {
            const float* base;
            if constexpr (DGRAD) {
                base = a.Aroot + (size_t)row[j] * K;
            } else {
                base = row[j] >= 0 ? a.Aroot + (size_t)row[j] * K : a.Arel + (size_t)(-row[j] - 1 - a.m_lo) * K;
            }
            v[j] = *reinterpret_cast<const float4*>(base + c4);
        }
    }
    // the epilogue's per-row value of tile row t (< 32): dgrad 1 / count of a relation row;
    // forward with the mode-SINGLE root epilogue: 1 when the node has a segment of the relation,
    // 0 when its root row is final; 1 otherwise. Issued when the item starts, read before the
    // item's barrier (a chain later), so the load's latency is off the critical path
    // (always a load — of g_one_i32 when the item has no such value — so no branch or select
    // after it makes the compiler wait for the load where it is issued)
    __device__ static __forceinline__ int row_val_load(const RelGemmArgs& a, const Item& it, int t) {
        const int r = it.r0 + min(t, it.nrows - 1);
        const int* p;
        if constexpr (DGRAD) p = it.root ? &g_one_i32 : a.s_cnt + r;
        else p = (it.root && a.node_map != nullptr) ? a.node_map + r : &g_one_i32;
        return *p;
    }
    __device__ static __forceinline__ float row_val(int v) {
        if constexpr (DGRAD) return 1.0f / (float)v;
        else return v != 0 ? 1.0f : 0.0f;
    }
    __device__ static __forceinline__ void commit(const Item& it, int kh, int t, const float4 (&v)[WPT],
                                                  __bf16* planes) {
        __bf16* P = planes + kh * 3 * PLANE;
#pragma unroll
        for (int j = 0; j < WPT; ++j) {
            const int r = t / 32 + 8 * j;
            const float4 x = r < it.nrows ? v[j] : make_float4(0.f, 0.f, 0.f, 0.f);
            __bf16 p0[4], p1[4], p2[4];
            split3_bf16(x.x, p0[0], p1[0], p2[0]);
            split3_bf16(x.y, p0[1], p1[1], p2[1]);
            split3_bf16(x.z, p0[2], p1[2], p2[2]);
            split3_bf16(x.w, p0[3], p1[3], p2[3]);
            __bf16* d = P + r * LDAB + (t & 31) * 4;
            typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
            *reinterpret_cast<bf16x4*>(d) = bf16x4{p0[0], p0[1], p0[2], p0[3]};
            *reinterpret_cast<bf16x4*>(d + PLANE) = bf16x4{p1[0], p1[1], p1[2], p1[3]};
            *reinterpret_cast<bf16x4*>(d + 2 * PLANE) = bf16x4{p2[0], p2[1], p2[2], p2[3]};
        }
    }
    // IL: one float4 part of the commit (rows past nrows: zeros) / of the row issue
    __device__ static __forceinline__ void commit_part(int j, int kh, int t, int nrows, const float4& v, __bf16* planes) {
        __bf16* P = planes + kh * 3 * PLANE;
        const int r = t / 32 + 8 * j;
        const float4 x = r < nrows ? v : make_float4(0.f, 0.f, 0.f, 0.f);
        __bf16 p0[4], p1[4], p2[4];
        split3_bf16(x.x, p0[0], p1[0], p2[0]);
        split3_bf16(x.y, p0[1], p1[1], p2[1]);
        split3_bf16(x.z, p0[2], p1[2], p2[2]);
        split3_bf16(x.w, p0[3], p1[3], p2[3]);
        __bf16* d = P + r * LDAB + (t & 31) * 4;
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        *reinterpret_cast<bf16x4*>(d) = bf16x4{p0[0], p0[1], p0[2], p0[3]};
        *reinterpret_cast<bf16x4*>(d + PLANE) = bf16x4{p1[0], p1[1], p1[2], p1[3]};
        *reinterpret_cast<bf16x4*>(d + 2 * PLANE) = bf16x4{p2[0], p2[1], p2[2], p2[3]};
    }
    __device__ static __forceinline__ void issue_part(const RelGemmArgs& a, int j, int kh, int t, int row, float4& v) {
        const int c4 = kh * KH + (t & 31) * 4;
        (void)j;
        const float* base;
        if constexpr (DGRAD) {
            base = a.Aroot + (size_t)row * K;
        } else {
            base = row >= 0 ? a.Aroot + (size_t)row * K : a.Arel + (size_t)(-row - 1 - a.m_lo) * K;
        }
        v = *reinterpret_cast<const float4*>(base + c4);
    }
    // the wave's slice: B(kh·128 + 16s + 8h + j, col) in bf16 pieces
    __device__ static __forceinline__ void load_b(const float* w, int kh, int col, int h, bf16x8 (&b)[NS][3]) {
        float f[NS][8];
        if constexpr (!DGRAD) {
            const float* p = w + (size_t)(kh * KH + 8 * h) * N + col;
#pragma unroll
            for (int s = 0; s < NS; ++s)
#pragma unroll
                for (int j = 0; j < 8; ++j) f[s][j] = p[(size_t)(16 * s + j) * N];
        } else {  // B(k, n) = W[n][k]
            const float* p = w + (size_t)col * K + kh * KH + 8 * h;
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const float4 t0 = *reinterpret_cast<const float4*>(p + 16 * s);
                const float4 t1 = *reinterpret_cast<const float4*>(p + 16 * s + 4);
                f[s][0] = t0.x; f[s][1] = t0.y; f[s][2] = t0.z; f[s][3] = t0.w;
                f[s][4] = t1.x; f[s][5] = t1.y; f[s][6] = t1.z; f[s][7] = t1.w;
            }
        }
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                __bf16 h0, h1, h2;
                split3_bf16(f[s][j], h0, h1, h2);
                b[s][0][j] = h0;
                b[s][1][j] = h1;
                b[s][2][j] = h2;
            }
    }
};

// IL (round 5, MPGNN_OPT_GEMM_W_IL; GEMM_IL's skeleton at K = 128): the next item's commit and the row loads of the
// item after it cut into their four float4 parts, part j committed and re-issued in k-step
// 2j + 1 among that k-step's MFMAs (sched_group_barrier), the stores of the previous item
// unconditional (the upper K half's target has no bytes: dropped by the bounds check), so the
// k-steps carry no branch. Same products, same order: bit-identical outputs.
template <bool DGRAD, bool IL = false>
__global__ __launch_bounds__(512, 1) void rel_gemm_bf3w_kernel(RelGemmArgs a) {
    using G = RelGemmBf3W<DGRAD>;
    extern __shared__ __bf16 smem_bf[];
    __bf16* As = smem_bf;                                                   // [2][2 halves][3][PLANE]
    float* Ot = reinterpret_cast<float*>(smem_bf + 12 * G::PLANE);         // [2][32][LDO]
    float* Sc = Ot + 2 * 32 * G::LDO;                                      // [2][32]
    const int tid = threadIdx.x, lane = tid & 63, c = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int kh = wave >> 2;   // K half of the wave (uniform)
    const int wq = wave & 3;    // 32-column strip
    const int t = tid & 255;    // thread within its half
    // block b: XCD b & 7; within an XCD, consecutive pairs (cb = 0, 1) share an item range
    const int Gx = (int)gridDim.x;
    const int xcd = (int)blockIdx.x & 7, slot = (int)blockIdx.x >> 3;
    const int per_xcd = Gx >> 3;                 // launched as a multiple of 16
    const int cb = slot & 1;
    const int n_ranges = Gx >> 1;
    const int rng = xcd * (per_xcd >> 1) + (slot >> 1);
    const int n_items = a.n_rel + a.n_root;
    const int i_beg = (int)((long long)rng * n_items / n_ranges);
    const int i_end = (int)((long long)(rng + 1) * n_items / n_ranges);
    if (i_beg >= i_end) return;
    stamp_id();
    const int col = cb * 128 + wq * 32 + c;
    const bool root_epi = !DGRAD && a.node_map != nullptr;
    const float bias_c = (root_epi && a.bias != nullptr) ? a.bias[col] : 0.0f;

    // item windows: tab_a covers [wb, wb + 64), tab_b the next 64 items (loaded one window ahead)
    int wb = i_beg;
    typename G::Tab tab_a = G::load_tab(a, wb, i_end, lane), tab_b = G::load_tab(a, wb + 64, i_end, lane);
    auto get_item = [&](int i) {
        return i - wb < 64 ? G::item_at(a, tab_a, i - wb) : G::item_at(a, tab_b, i - wb - 64);
    };
    // prologue: item i_beg committed, rows of i_beg+1 in flight, sources of i_beg+2 loaded
    typename G::Item cur = get_item(i_beg);
    int row[G::WPT];
    float4 v[G::WPT];
    G::gather_idx(a, cur, t, row);
    G::issue(a, kh, t, row, v);
    bf16x8 b[G::NS][3];
    G::load_b(cur.w, kh, col, h, b);
    G::commit(cur, kh, t, v, As);
    typename G::Item nxt = cur, nn = cur;
    if (i_beg + 1 < i_end) {
        nxt = get_item(i_beg + 1);
        G::gather_idx(a, nxt, t, row);
        G::issue(a, kh, t, row, v);
    }
    if (i_beg + 2 < i_end) {
        nn = get_item(i_beg + 2);
        G::gather_idx(a, nn, t, row);
    }
    __syncthreads();

    float prev[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) prev[r] = 0.0f;
    // the lower half's store target: item i-1's rows (bounds: its nrows; none before the first)
    __amdgpu_buffer_rsrc_t prev_rsrc = __builtin_amdgcn_make_buffer_rsrc(a.Y, (short)0, 0, 0x00020000);
    auto store_prev = [&](int r) {
        const int rr = (r & 3) + 8 * (r >> 2) + 4 * h;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(prev[r]), prev_rsrc, rr * (G::N * 4) + col * 4, 0, 0);
    };
    int buf = 0;
    for (int i = i_beg; i < i_end; ++i) {
        stamp(i - i_beg, 0);
        const bool has_next = i + 1 < i_end;
        const bool val_lane = kh == 0 && t < 32;
        const int rv = G::row_val_load(a, cur, t & 31);  // row t & 31's epilogue value, to Sc before the barrier
        const __bf16* Ab = As + (buf * 2 + kh) * 3 * G::PLANE + c * G::LDAB + 8 * h;
        // the small products in their own accumulator (as rel_gemm_bf3_kernel): the a0·b0 chain
        // rounds once per k-step at the sum's magnitude instead of six times (round 5: C5's
        // grad_x was 2.2x the fp32 reference path's error off the float64 truth with one)
        f32x16 acc, hi;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            acc[r] = 0.0f;
            hi[r] = 0.0f;
        }
        bf16x8 f0 = *reinterpret_cast<const bf16x8*>(Ab);
        bf16x8 f1 = *reinterpret_cast<const bf16x8*>(Ab + G::PLANE);
        bf16x8 f2 = *reinterpret_cast<const bf16x8*>(Ab + 2 * G::PLANE);
#pragma unroll
        for (int s = 0; s < G::NS; ++s) {
            const bf16x8 a0 = f0, a1 = f1, a2 = f2;
            if (s + 1 < G::NS) {
                f0 = *reinterpret_cast<const bf16x8*>(Ab + 16 * (s + 1));
                f1 = *reinterpret_cast<const bf16x8*>(Ab + G::PLANE + 16 * (s + 1));
                f2 = *reinterpret_cast<const bf16x8*>(Ab + 2 * G::PLANE + 16 * (s + 1));
            }
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b[s][0], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[s][1], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[s][2], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[s][0], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[s][1], acc, 0, 0, 0);
            hi = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[s][0], hi, 0, 0, 0);
            if constexpr (!IL) {
                if (kh == 0) {  // item i-1's tile leaves two rows per k-step
                    store_prev(2 * s);
                    store_prev(2 * s + 1);
                }
                if (s == (3 * G::NS) / 4 - 1 && has_next) {
                    G::commit(nxt, kh, t, v, As + (buf ^ 1) * 6 * G::PLANE);
                    if (i + 2 < i_end) G::issue(a, kh, t, row, v);  // item i+2's rows, in flight for a chain
                }
            } else {
                store_prev(2 * s);  // upper half: zero-byte target, dropped
                store_prev(2 * s + 1);
                if ((s & 1) == 1) {  // part j = s / 2 of item i+1's tile, then item i+2's rows of part j
                    const int j = s >> 1;
                    G::commit_part(j, kh, t, has_next ? nxt.nrows : 0, v[j], As + (buf ^ 1) * 6 * G::PLANE);
                    G::issue_part(a, j, kh, t, row[j], v[j]);
                }
                __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);  // next fragments
#pragma unroll
                for (int m = 0; m < 6; ++m) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
                    if (m < 3) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
                    if (m < 2) __builtin_amdgcn_sched_group_barrier(0x040, 1, 0);
                    if (m == 2) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        stamp(i - i_beg, 1);
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = hi[r] + acc[r];
        float* Oe = Ot + buf * 32 * G::LDO;
        if (kh == 1) {
#pragma unroll
            for (int r = 0; r < 16; ++r) Oe[((r & 3) + 8 * (r >> 2) + 4 * h) * G::LDO + wq * 32 + c] = acc[r];
        }
        if (has_next && nxt.w != cur.w) G::load_b(nxt.w, kh, col, h, b);  // after the chain: registers free
        const typename G::Item next_item = nxt;
        if (i + 3 < i_end) {  // sources of item i+3 (row was consumed by the issue above)
            if (i + 3 - wb >= 64) {  // item i+3 opens the next window: shift, prefetch the one after
                wb += 64;
                tab_a = tab_b;
                tab_b = G::load_tab(a, wb + 64, i_end, lane);
            }
            typename G::Item it3 = get_item(i + 3);
            G::gather_idx(a, it3, t, row);
            nxt = nn;
            nn = it3;
        } else {
            nxt = nn;
        }
        if (val_lane) Sc[(i & 1) * 32 + t] = G::row_val(rv);
        stamp(i - i_beg, 3);
        __syncthreads();  // upper partial tile of item i in LDS; item i+1's tiles committed
        stamp(i - i_beg, 4);
        if (kh == 0) {
            // straight-line epilogue: the tile, then the uniform per-item case on all 16 values
            // (a per-row branch made the compiler wait on each LDS read in turn)
            const float* sc = Sc + (i & 1) * 32;
            float o[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) o[r] = acc[r] + Oe[((r & 3) + 8 * (r >> 2) + 4 * h) * G::LDO + wq * 32 + c];
            if constexpr (DGRAD) {
                if (!cur.root) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) o[r] = o[r] * sc[(r & 3) + 8 * (r >> 2) + 4 * h];
                }
            } else if (root_epi && cur.root) {
                // mode-SINGLE root epilogue (RelGemmArgs::node_map): a row without a segment of
                // the relation is final, act((0 + x_i @ root) + bias); single_fix_kernel finishes
                // the others from x_i @ root
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    float f = (0.0f + o[r]) + bias_c;
                    f = a.relu ? relu_f(f) : f;
                    o[r] = sc[(r & 3) + 8 * (r >> 2) + 4 * h] == 0.0f ? f : o[r];
                }
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) prev[r] = o[r];
            float* Yt = cur.root ? a.Yroot + (size_t)(cur.r0 - a.row_lo) * G::N : a.Y + (size_t)(cur.r0 - a.sel_b) * G::N;
            const int bytes = __builtin_amdgcn_readfirstlane(cur.nrows) * G::N * 4;
            prev_rsrc = __builtin_amdgcn_make_buffer_rsrc(Yt, (short)0, bytes, 0x00020000);
        }  // (the upper half's rsrc keeps 0 bytes: its IL stores are dropped)
        cur = next_item;
        buf ^= 1;
    }
    if (kh == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) store_prev(r);
    }
    stamp_end();
}

template <int KB>  // Kp = 64·KB
__global__ __launch_bounds__(kThreads, 2) void tile_gemm_kernel(TileGemmArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    // the B-load variant is fixed for the launch: dispatched once, outside the item loop
    const bool exact_k = a.K == 64 * KB && a.K >= kKC;
    const int ldw = a.trans ? a.K : a.N;
    if (!a.trans) {
        if (exact_k) tile_gemm_body<KB, false, false>(a, smem);
        else tile_gemm_body<KB, false, true>(a, smem);
    } else {
        if (exact_k && (ldw & 3) == 0) tile_gemm_body<KB, true, false>(a, smem);
        else tile_gemm_body<KB, true, true>(a, smem);
    }
}

// ----------------------------------------------------------------------------------------
// row_sum_kernel:  out[i] = (Σ_{entries of row i, in order} src) + extra[i - lo] + bias
//   (extra and bias only for rows i in [lo, hi)); the forward combine Σ_r Y + Y_root + bias
//   and the transposed grad_x gather Σ G + G_root.  No LDS, 4 rows per wave.
// ----------------------------------------------------------------------------------------
struct RowSumArgs {
    int N;              // one past the last row
    int r_begin;        // first row (rows [r_begin, N))
    int list_kind;      // 0: ptr[row] array; 1: lower_bound in keys[kb, ke)
    const int* ptr;
    const int* keys;
    int kb, ke;
    GatherSrc g;
    const float* extra; // nullable [hi - lo, F]
    const float* bias;  // nullable [F]
    int lo, hi;
    const int* cnt;     // nullable: divide row i by cnt[i] (segment means)
    int out_off;        // out row = i - out_off
    float* out;         // [*, F]
    const int* res;     // resolved entries of the ragged list g.ent (gather_rows_kernel)
};

__device__ __forceinline__ int lower_bound_i32(const int* keys, int lo, int hi, int v) {
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (keys[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// Calls f(std::integral_constant<int, r>) for a wave-uniform runtime r in [0, N).
template <int N, class F>
__device__ __forceinline__ void dispatch_row(int r, F&& f) {
    if constexpr (N > 1) {
        if (r == N - 1) f(std::integral_constant<int, N - 1>{});
        else dispatch_row<N - 1>(r, f);
    } else {
        f(std::integral_constant<int, 0>{});
    }
}

// EXTRA: the launch adds extra rows and/or bias (combine, grad_x); the means launch does not
// and keeps those registers free (occupancy).
template <int V, int T, bool EXTRA>
__global__ __launch_bounds__(kThreads) void row_sum_kernel(RowSumArgs a) {
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int row0 = a.r_begin + (blockIdx.x * kWaves + wave) * kSumRowsPerWave;
    if (row0 >= a.N) return;
    const int wn = min(kSumRowsPerWave, a.N - row0);
    int bnd = 0;
    if (lane <= kSumRowsPerWave) {
        const int i = row0 + (lane <= wn ? lane : wn);
        bnd = a.list_kind == 0 ? a.ptr[i] : lower_bound_i32(a.keys, a.kb, a.ke, i);
    }
    const int F = a.g.F;
    // per-row operands of the flush, loaded up front with the row bounds: a load inside the
    // flush waits (vmcnt is in order) for every row load already in flight
    // (unconditional: absent operands read a valid dummy row and are discarded by selects)
    const bool has_cnt = a.cnt != nullptr;
    const int cnt_raw = (has_cnt ? a.cnt : a.g.dummy)[has_cnt ? min(row0 + min(lane, kSumRowsPerWave - 1), a.N - 1) : 0];
    const int cnt_l = has_cnt ? cnt_raw : 1;
    constexpr int NX = EXTRA ? kSumRowsPerWave : 1;
    float ex[NX][T][V], bb[T][V];
    int colc[T];
#pragma unroll
    for (int t = 0; t < T; ++t) colc[t] = min((t * 64 + lane) * V, F - V);
    const bool has_ex = EXTRA && a.extra != nullptr && a.hi > a.lo;
    const bool has_b = EXTRA && a.bias != nullptr;
#pragma unroll
    for (int r = 0; r < NX; ++r) {
        const int i = min(max(row0 + r, a.lo), a.hi - 1);  // clamped into the own range
        const float* eb = has_ex ? a.extra + (size_t)(i - a.lo) * F : a.g.src;
#pragma unroll
        for (int t = 0; t < T; ++t) {
            vload<V>(eb + (has_ex ? colc[t] : 0), ex[r][t]);
#pragma unroll
            for (int q = 0; q < V; ++q) ex[r][t][q] = has_ex ? ex[r][t][q] : 0.0f;
        }
    }
#pragma unroll
    for (int t = 0; t < T; ++t) {
        vload<V>((has_b ? a.bias : a.g.src) + (has_b ? colc[t] : 0), bb[t]);
#pragma unroll
        for (int q = 0; q < V; ++q) bb[t][q] = has_b ? bb[t][q] : 0.0f;
    }
    // flush of row r: r is wave-uniform, so it is dispatched to a copy with a compile-time row
    // (indexing ex[r] with a runtime r turned the array into LDS traffic)
    auto flush_row = [&](auto RI, bool live, float (&acc)[T][V]) {
        constexpr int r = decltype(RI)::value;
        const int i = row0 + r;
        if (live) {
            const bool own = i >= a.lo && i < a.hi;
            const float div = (float)readlane(cnt_l, r);
#pragma unroll
            for (int t = 0; t < T; ++t) {
                const int col = (t * 64 + lane) * V;
                if (col < F) {
                    float v[V];
#pragma unroll
                    for (int q = 0; q < V; ++q) {
                        v[q] = has_cnt ? acc[t][q] / div : acc[t][q];
                        if constexpr (EXTRA)
                            if (own) v[q] = (v[q] + ex[r][t][q]) + bb[t][q];  // zeros when absent
                    }
                    vstore<V>(a.out + (size_t)(i - a.out_off) * F + col, v);
                }
            }
        }
        zero_acc<V, T>(acc);
    };
    wave_gather<V, T, (V * T <= 2 ? 8 : 4), kSumRowsPerWave>(
        a.g, bnd, wn, lane, [&](int r, bool live, float (&acc)[T][V]) {
            dispatch_row<kSumRowsPerWave>(r, [&](auto RI) { flush_row(RI, live, acc); });
        });
}


// ----------------------------------------------------------------------------------------
// flat_rows_kernel — the fast-path row sums (segment means, grad_x, forward combine).
//
// One wave per plan chunk: at most kFlatChunk consecutive positions of the list, cut at row
// ends except inside rows longer than a chunk (FlatHost, plan_internal.h).  Every wave does the
// same bounded work whatever the degree skew, and does it like a plain gather: one coalesced
// load of the chunk's values and row ids, then its source rows in flight 16 at a time, summed
// in position order.  A row that starts and ends in the chunk is written (divided by its entry
// count for means); the chunk's first / last row, when split with a neighbouring chunk, goes to
// a carry slot and finalize_rows_kernel adds the slots in chunk order.  Rows held in one chunk
// are therefore summed exactly in the reference order; split rows (longer than a chunk, or
// crossing one) are summed as ordered partials (tolerance 1e-4, like the ragged pieces).
// ----------------------------------------------------------------------------------------
struct FlatArgs {
    const int* chunk_ptr;
    const int* chunk_info;  // bit0 first row split, bit1 last row split, >>2 carry slot (long group: piece)
    const int* group_ptr;   // chunk range of each workgroup
    const int* group_long;  // 1: the pieces of one long row, summed in LDS in piece order
    int g_lo, g_hi;         // groups of this launch
    const int* table;       // value per position: source row + idx_off
    const int* row_of;      // output row per position
    const float* src;       // [*, F]
    int F;
    int idx_off;
    int filter, flo, fhi;   // keep a value only when flo <= value < fhi
    const int* cnt;         // nullable: divide complete rows by cnt[row] (global counts in shards)
    int row_off;            // out row = row - row_off
    float* out;
    float* carry;           // [slots][F]
    const int* dummy;       // any valid int table
    const float* extra;     // nullable: a value v < 0 is extra row -(v+1) (augmented lists)
    const float* bias;      // nullable: added to complete rows in [lo, hi) after their sum
    int lo, hi;
    int relu;               // fused activation on complete rows (unsharded combine only)
    // nullable: rows split over > kFlatLongPieces chunks are finished inside the launch — each
    // piece's partial is stored write-through (sc1), its wave drains and adds 1 to arrive[k]
    // (agent scope); the wave whose add completes the row sums the row's slots in chunk order
    // (sc1 loads) and finishes it (finalize_rows_kernel's mode-0 arithmetic, without its launch)
    unsigned* arrive;       // [nsplit], zero at launch
    const int* row_split;   // split index per row
    const int* split_ptr;
    const int* split_slot;
    // nullable (round 6, MPGNN_OPT_FLAT_PAD): the list's chunks re-laid per workgroup slot
    // (4·group + wave): pad_desc[slot] = {n, info, long group, 0}, pad_val / pad_row[32·slot + q]
    // = table / row_of of the chunk's position q — all at addresses the wave knows from its
    // group and wave number, fetched by one round of vector loads instead of two dependent
    // scalar hops (group → chunk range) and a vector hop (chunk → its positions)
    const int4* pad_desc;
    const int* pad_val;
    const int* pad_row;
    // nullable (grad_x, round 6): the ReLU backward of the layer that produced this layer's input
    // fused into the row finish — out = mask > 0 ? v : 0 with mask = that input (relu_bwd_f)
    const float* mask;
};

// The finishing step of a complete row: / cnt (IEEE), + bias on own rows, fused ReLU.
template <int V, int T>
__device__ __forceinline__ void flat_finish_store(const FlatArgs& a, int rr, float d, bool div, const float (&bb)[T][V],
                                                  const float (&acc)[T][V], int lane) {
    const bool addb = a.bias != nullptr && rr >= a.lo && rr < a.hi;
    float* dst = a.out + (size_t)(rr - a.row_off) * a.F;
    const bool msk = a.mask != nullptr;
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const int col = (t * 64 + lane) * V;
        if (col < a.F) {
            float o[V], mv[V];
            if (msk) vload<V>(a.mask + (size_t)(rr - a.row_off) * a.F + col, mv);
#pragma unroll
            for (int k = 0; k < V; ++k) {
                o[k] = div ? acc[t][k] / d : acc[t][k];
                if (addb) o[k] = o[k] + bb[t][k];
                if (a.relu) o[k] = relu_f(o[k]);
                if (msk) o[k] = relu_bwd_f(o[k], mv[k]);
            }
            vstore_sc1<V>(dst, col, o);
        }
    }
}

template <int V, int T>
__device__ __forceinline__ void flat_finish_store(const FlatArgs& a, int rr, float d, bool div, const float (&bb)[T][V],
                                                  const float (&acc)[T][V], int lane);

// A piece of a row split over more than kFlatLongPieces chunks: store the partial write-through,
// count it; the last piece's wave adds the row's slots in chunk order (from 0.0f, as
// finalize_rows_kernel) and finishes the row.  Hand-off: sc1 stores -> this wave's vmcnt(0) ->
// one lane's agent-scope atomic add; the adder that completes the count reads the slots with
// sc1 loads only after its add has returned (MI355X_MICROARCH.md § visibility, first row).
template <int V, int T>
__device__ __forceinline__ void flat_split_arrive(const FlatArgs& a, int rr, float d, bool div,
                                                  const float (&bb)[T][V], int lane) {
    const int F = a.F;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the piece's sc1 partial has left the wave
    const int k = ld_uniform(a.row_split, rr);
    const int s0 = ld_uniform(a.split_ptr, k), s1 = ld_uniform(a.split_ptr, k + 1);
    unsigned old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(a.arrive + k, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = (unsigned)readlane((int)old, 0);
    if (old + 1 != (unsigned)(s1 - s0)) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the loads below the add
    int colc[T];
#pragma unroll
    for (int t = 0; t < T; ++t) colc[t] = min((t * 64 + lane) * V, F - V);
    float sum[T][V];
    zero_acc<V, T>(sum);
    constexpr int SB = 8;  // slots in flight (rare path: kept small, the chunk loop's registers bound the kernel)
    for (int sb = s0; sb < s1; sb += SB) {
        const int my_sl = a.split_slot[min(sb + (lane & (SB - 1)), s1 - 1)];
        float v[SB][T][V];
#pragma unroll
        for (int u = 0; u < SB; ++u) {
            const float* base = a.carry + (size_t)readlane(my_sl, u) * F;
#pragma unroll
            for (int t = 0; t < T; ++t) vload_sc1<V>(base, colc[t], v[u][t]);
        }
#pragma unroll
        for (int u = 0; u < SB; ++u)
            if (sb + u < s1)
#pragma unroll
                for (int t = 0; t < T; ++t)
#pragma unroll
                    for (int q = 0; q < V; ++q) sum[t][q] += v[u][t][q];
    }
    flat_finish_store<V, T>(a, rr, d, div, bb, sum, lane);
}

// One wave sums one chunk (<= 32 positions): complete rows are finished and stored; the
// partial of a split row goes to carry slot `info >> 2` of `carry` (global slots, or the LDS
// piece slots of a long group).  With a.arrive, a piece of a > kFlatLongPieces row is counted
// after the loop (one piece per chunk) and its row finished by the wave that completes it.
template <int V, int T, int U, bool GLOBAL>
__device__ __forceinline__ void flat_chunk_body(const FlatArgs& a, int n, int info, int val, int row, int lane,
                                                float* carry, const float (&bb)[T][V]);

template <int V, int T, int U, bool GLOBAL>
__device__ __forceinline__ void flat_chunk(const FlatArgs& a, int c, int lane, float* carry, const float (&bb)[T][V]) {
    const int p0 = ld_uniform(a.chunk_ptr, c);
    const int n = ld_uniform(a.chunk_ptr, c + 1) - p0;  // 1 .. kFlatChunk
    const int info = ld_uniform(a.chunk_info, c);
    const int pq = p0 + min(lane, n - 1);
    flat_chunk_body<V, T, U, GLOBAL>(a, n, info, a.table[pq], a.row_of[pq], lane, carry, bb);
}

// n positions (1 .. kFlatChunk), lane q < n holding position q's table value and output row
template <int V, int T, int U, bool GLOBAL>
__device__ __forceinline__ void flat_chunk_body(const FlatArgs& a, int n, int info, int val, int row, int lane,
                                                float* carry, const float (&bb)[T][V]) {
    const int F = a.F;
    bool keep = lane < n;
    const bool isx = val < 0;  // augmented lists: the row's trailing extra entry
    if (a.filter) keep = keep && (isx || (val >= a.flo && val < a.fhi));
    const int srow = keep ? (isx ? -val - 1 : val - a.idx_off) : 0;
    const unsigned long long xm = __ballot(keep && isx);
    const bool has_cnt = a.cnt != nullptr;
    const int cnt_l = (has_cnt ? a.cnt : a.dummy)[has_cnt ? row : 0];
    const int next = __shfl_down(row, 1);
    const unsigned long long lastm = __ballot(lane < n && (lane == n - 1 || next != row));
    const unsigned long long keepm = __ballot(keep);
    const int rf = readlane(row, 0);
    const int rl = readlane(row, n - 1);
    const bool fs = info & 1, ls = info & 2;
    const int slot0 = info >> 2;
    int colc[T];
#pragma unroll
    for (int t = 0; t < T; ++t) colc[t] = min((t * 64 + lane) * V, F - V);

    float acc[T][V];
    zero_acc<V, T>(acc);
    const bool fuse = GLOBAL && a.arrive != nullptr;  // GLOBAL: carry is a.carry (not LDS piece slots)
    int arr_row = -1;  // the split row this chunk holds a piece of (fuse)
    for (int u0 = 0; u0 < n; u0 += U) {
        float v[U][T][V];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int q = min(u0 + u, n - 1);
            const int r = readlane(srow, q);
            const float* base = (((xm >> q) & 1ull) ? a.extra : a.src) + (size_t)r * F;
#pragma unroll
            for (int t = 0; t < T; ++t) vload<V>(base + colc[t], v[u][t]);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int q = u0 + u;
            if (q < n) {
                if ((keepm >> q) & 1ull) {
#pragma unroll
                    for (int t = 0; t < T; ++t)
#pragma unroll
                        for (int k = 0; k < V; ++k) acc[t][k] += v[u][t][k];
                }
                if ((lastm >> q) & 1ull) {
                    const int rr = readlane(row, q);
                    const bool split = (rr == rf && fs) || (rr == rl && ls);
                    if (!split) {
                        flat_finish_store<V, T>(a, rr, (float)readlane(cnt_l, q), has_cnt, bb, acc, lane);
                    } else {  // a split chunk holds one row: its partial
                        float* dst = carry + (size_t)slot0 * F;
                        if (fuse) {  // write-through: another wave may sum it in this launch
#pragma unroll
                            for (int t = 0; t < T; ++t) {
                                const int col = (t * 64 + lane) * V;
                                if (col < F) vstore_sc1<V>(dst, col, acc[t]);
                            }
                            arr_row = rr;
                        } else {
#pragma unroll
                            for (int t = 0; t < T; ++t) {
                                const int col = (t * 64 + lane) * V;
                                if (col < F) vstore<V>(dst + col, acc[t]);
                            }
                        }
                    }
                    zero_acc<V, T>(acc);
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    if (arr_row >= 0)
        flat_split_arrive<V, T>(a, arr_row, has_cnt ? (float)a.cnt[arr_row] : 1.0f, has_cnt, bb, lane);
}

// flat_rows_kernel — one workgroup per group: a normal group's waves take one chunk each; a
// long group's waves sum the pieces w, w + 4, … into LDS slots, then wave 0 adds the slots in
// piece order and finishes the row (one launch, no finalize for rows of <= 16 pieces).
template <int V, int T, int U = 16>
__global__ __launch_bounds__(kThreads) void flat_rows_kernel(FlatArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds_pieces[];  // [max_pieces][F] (long groups)
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int F = a.F;
    int colc[T];
#pragma unroll
    for (int t = 0; t < T; ++t) colc[t] = min((t * 64 + lane) * V, F - V);
    const bool has_b = a.bias != nullptr;
    float bb[T][V];
#pragma unroll
    for (int t = 0; t < T; ++t) {
        vload<V>(has_b ? a.bias + colc[t] : a.src, bb[t]);
#pragma unroll
        for (int k = 0; k < V; ++k) bb[t][k] = has_b ? bb[t][k] : 0.0f;
    }
    // persistent over groups (grid-stride): the waves stay resident instead of a short-lived
    // workgroup per group; every wave of a workgroup walks the same groups, so the long groups'
    // barriers line up
    for (int g = a.g_lo + (int)blockIdx.x; g < a.g_hi; g += (int)gridDim.x) {
        if (a.pad_desc != nullptr) {  // one round of loads: the slot's descriptor and positions
            const int slot = 4 * g + wave;
            const int4 d = a.pad_desc[slot];
            const int q = 32 * slot + (lane & 31);
            const int val = a.pad_val[q], row = a.pad_row[q];
            const int n = __builtin_amdgcn_readfirstlane(d.x);
            if (__builtin_amdgcn_readfirstlane(d.z) == 0) {  // a normal group (uniform over the workgroup)
                if (n > 0) flat_chunk_body<V, T, U, true>(a, n, __builtin_amdgcn_readfirstlane(d.y), val, row, lane,
                                                          a.carry, bb);
                continue;
            }
        }
        const int c0 = ld_uniform(a.group_ptr, g), c1 = ld_uniform(a.group_ptr, g + 1);
        const bool lng = ld_uniform(a.group_long, g) != 0;
        if (!lng) {
            const int c = c0 + wave;
            if (c < c1) flat_chunk<V, T, U, true>(a, c, lane, a.carry, bb);
            continue;
        }
        // a long row's pieces (the same 16 loads in flight as a normal chunk: more would raise
        // the kernel's register count and cost every group occupancy)
        for (int c = c0 + wave; c < c1; c += kWaves) flat_chunk<V, T, U, false>(a, c, lane, lds_pieces, bb);
        __syncthreads();
        if (wave == 0) {
            const int rr = a.row_of[ld_uniform(a.chunk_ptr, c0)];
            float acc[T][V];
            zero_acc<V, T>(acc);
            for (int k = 0; k < c1 - c0; ++k) {  // pieces in order
#pragma unroll
                for (int t = 0; t < T; ++t) {
                    float v[V];
                    vload<V>(lds_pieces + (size_t)k * F + colc[t], v);
#pragma unroll
                    for (int q = 0; q < V; ++q) acc[t][q] += v[q];
                }
            }
            const bool has_cnt = a.cnt != nullptr;
            flat_finish_store<V, T>(a, rr, has_cnt ? (float)a.cnt[rr] : 1.0f, has_cnt, bb, acc, lane);
        }
        __syncthreads();  // the LDS piece slots are free for the next long group
    }
}

// finalize_rows_kernel — one wave per row.
//   mode 0 (segment means): split rows k in [k0, k1): out[row] = (Σ carry slots in order) / cnt
//   mode 1 (combine, grad_x): every row in [r_lo, r_hi):
//       v = split ? Σ slots : (no entries ? 0 : out[row]);  own rows: v = (v + extra) + bias
struct FinalArgs {
    int mode;
    const int* split_row;
    const int* split_ptr;
    const int* split_slot;
    int k0, k1;
    const int* row_split;  // mode 1
    const int* row_ptr;    // mode 1: no entries when row_ptr[r] == row_ptr[r + 1]
    int r_lo, r_hi;
    const float* carry;
    int F;
    const int* cnt;        // nullable (mode 0)
    const float* extra;    // nullable [hi - lo, F]
    const float* bias;     // nullable [F]
    int lo, hi;
    int row_off;
    float* out;
    const float* dummy;    // any valid float row
    int relu;              // fused activation after the bias
    const float* mask;     // nullable: FlatArgs::mask
};

// one wave, work index w (mode 0: split row k0 + w; mode 1: row r_lo + w)
template <int V, int T>
__device__ __forceinline__ void finalize_row(const FinalArgs& a, int w, int lane) {
    const int F = a.F;
    int row, k;
    if (a.mode == 0) {
        k = a.k0 + w;
        if (k >= a.k1) return;
        row = ld_uniform(a.split_row, k);
    } else {
        row = a.r_lo + w;
        if (row >= a.r_hi) return;
        k = ld_uniform(a.row_split, row);
    }
    int colc[T];
#pragma unroll
    for (int t = 0; t < T; ++t) colc[t] = min((t * 64 + lane) * V, F - V);
    const bool own = row >= a.lo && row < a.hi;
    const bool has_ex = a.extra != nullptr && own;
    const bool has_b = a.bias != nullptr && own;
    // operands first (independent loads in flight together)
    float ex[T][V], bb[T][V];
#pragma unroll
    for (int t = 0; t < T; ++t) {
        vload<V>(has_ex ? a.extra + (size_t)(row - a.lo) * F + colc[t] : a.dummy, ex[t]);
        vload<V>(has_b ? a.bias + colc[t] : a.dummy, bb[t]);
    }
    float acc[T][V];
    zero_acc<V, T>(acc);
    if (k >= 0) {
        // slots of one row: 32 in flight per round trip (a hub in-list has up to ~190)
        constexpr int SB = (V * T <= 2) ? 32 : 16;
        const int s0 = ld_uniform(a.split_ptr, k), s1 = ld_uniform(a.split_ptr, k + 1);
        for (int sb = s0; sb < s1; sb += SB) {
            const int my_sl = a.split_slot[min(sb + (lane & (SB - 1)), s1 - 1)];
            float v[SB][T][V];
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const int sl = readlane(my_sl, u);
#pragma unroll
                for (int t = 0; t < T; ++t) vload<V>(a.carry + (size_t)sl * F + colc[t], v[u][t]);
            }
#pragma unroll
            for (int u = 0; u < SB; ++u)
                if (sb + u < s1)
#pragma unroll
                    for (int t = 0; t < T; ++t)
#pragma unroll
                        for (int q = 0; q < V; ++q) acc[t][q] += v[u][t][q];
        }
        if (a.cnt != nullptr) {
            const float d = (float)ld_uniform(a.cnt, row);
#pragma unroll
            for (int t = 0; t < T; ++t)
#pragma unroll
                for (int q = 0; q < V; ++q) acc[t][q] = acc[t][q] / d;
        }
    } else if (a.mode == 1 && ld_uniform(a.row_ptr, row) != ld_uniform(a.row_ptr, row + 1)) {
#pragma unroll
        for (int t = 0; t < T; ++t) vload<V>(a.out + (size_t)(row - a.row_off) * F + colc[t], acc[t]);
    }
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const int col = (t * 64 + lane) * V;
        if (col < F) {
            float o[V];
#pragma unroll
            for (int q = 0; q < V; ++q) {
                o[q] = acc[t][q];
                if (has_ex) o[q] = o[q] + ex[t][q];
                if (has_b) o[q] = o[q] + bb[t][q];
                if (a.relu) o[q] = relu_f(o[q]);
            }
            if (a.mask != nullptr) {
                float mv[V];
                vload<V>(a.mask + (size_t)(row - a.row_off) * F + col, mv);
#pragma unroll
                for (int q = 0; q < V; ++q) o[q] = relu_bwd_f(o[q], mv[q]);
            }
            vstore<V>(a.out + (size_t)(row - a.row_off) * F + col, o);
        }
    }
}

template <int V, int T>
__global__ __launch_bounds__(kThreads) void finalize_rows_kernel(FinalArgs a) {
    finalize_row<V, T>(a, (int)blockIdx.x * kWaves + (int)(threadIdx.x >> 6), (int)(threadIdx.x & 63));
}


// ----------------------------------------------------------------------------------------
// gather_rows_kernel — the row-sum / segment-mean gather for F % 4 == 0 (any summation
// order: it reproduces row_sum_kernel bit for bit).
//
// A wave owns RPW = 4·G consecutive rows, split between G = 64 / S sub-waves of S lanes; each
// lane carries 4 consecutive columns (16-byte loads), so one load instruction moves G rows of
// F ≤ 4·S floats.  Sub-wave g sums its rows g, g + G, g + 2G, g + 3G one after the other, each
// in entry order from 0.0f — the same sequential sums as the reference's scatter_add_.
// Entry values (a source row, or -(piece+1) for the partial sum of a piece of a long run) are
// fetched S per lane-slice in one load and handed to the sub-wave by ds_bpermute; each lane
// forms its own address (no scalar readlane chain per row), and U rows per lane are in flight
// before any is added.  Row operands (counts, extra rows, bias) are loaded in the prologue, so
// the flush of a finished row is stores only.
// ----------------------------------------------------------------------------------------
struct GatherRowsArgs {
    int N;              // one past the last row
    int r_begin;        // first row
    int row_kind;       // 0: entries [ptr[i], ptr[i+1]); 1: [lower_bound(keys, i), lower_bound(keys, i+1));
                        // 2: [ptr[i], pe[i]) (pieces)
    const int* ptr;
    const int* pe;
    const int* keys;
    int kb, ke;
    const int* table;   // entry values
    const float* src;   // [*, F]
    int F;
    int idx_off;        // source row = value - idx_off
    int filter, flo, fhi;  // keep a value v >= 0 only when flo <= v < fhi
    const float* P;     // piece partial sums, row = -(v+1) - piece_off
    int piece_off;
    const float* extra; // nullable [hi - lo, F] added to own rows
    const float* bias;  // nullable [F] added to own rows
    int lo, hi;
    const int* cnt;     // nullable: divide row i by cnt[i]
    int out_off;
    float* out;
    const int* dummy;   // any valid int table
};

__device__ __forceinline__ float4 f4_add(float4 a, float4 b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

template <int S, bool EXTRA, int KR = 4>  // KR: rows per sub-wave (1 for the 32-entry pieces)
__global__ __launch_bounds__(kThreads) void gather_rows_kernel(GatherRowsArgs a) {
    constexpr int G = 64 / S;    // rows per load instruction
    constexpr int RPW = KR * G;  // rows per wave
    constexpr int U = KR == 1 ? S : 16;  // row loads in flight per lane (a whole piece when KR = 1)
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int sub = lane / S;
    const int sl = lane % S;
    const int row0 = a.r_begin + (blockIdx.x * kWaves + wave) * RPW;
    if (row0 >= a.N) return;
    const int F = a.F;
    const int col = min(4 * sl, F - 4);
    const bool col_live = 4 * sl < F;

    // ---- prologue: row bounds (lane j < RPW: row row0 + j), counts, extra rows, bias -----
    int my_beg = 0, my_end = 0;
    if (a.row_kind == 1) {
        // sorted keys[kb, ke): the wave finds lower_bound(row0) by a 64-ary search (one probe per
        // lane per round: ~3 dependent loads instead of a 17-deep binary search per row), then
        // the bounds of its RPW rows by ballots over the following keys, 64 at a time
        int l = a.kb, hgh = a.ke;  // wave-uniform; the answer lies in [l, hgh]
        while (hgh - l > 64) {
            const int step = (hgh - l + 63) >> 6;
            const int pj = l + lane * step;
            const bool pv = pj < hgh;
            const unsigned long long ge = __ballot(pv && a.keys[min(pj, hgh - 1)] >= row0);
            const unsigned long long vm = __ballot(pv);
            if (ge == 0) {
                l = l + (63 - __builtin_clzll(vm)) * step + 1;  // past the last valid probe
            } else {
                const int js = __builtin_ctzll(ge);
                hgh = l + js * step;
                if (js > 0) l = l + (js - 1) * step + 1;
            }
        }
        int cntv = 0;  // lane j <= RPW: lower_bound(row0 + j) - base
        const int base = l;
        for (int q0 = base; q0 < a.ke; q0 += 64) {
            const int q = q0 + lane;
            const int kv = q < a.ke ? a.keys[q] : INT_MAX;
#pragma unroll
            for (int j = 0; j <= RPW; ++j) {
                const int cj = __popcll(__ballot(kv < row0 + j));
                if (lane == j) cntv += cj;
            }
            // done once a key of this chunk reaches past the wave's last row (keys are sorted)
            if (__ballot(kv >= row0 + RPW) != 0) break;
        }
        const int b = base + cntv, e = base + __shfl(cntv, min(lane + 1, 63));
        const bool valid = lane < RPW && row0 + lane < a.N;
        my_beg = valid ? b : 0;
        my_end = valid ? e : 0;
    } else {
        const int i = min(row0 + min(lane, RPW - 1), a.N - 1);
        const int b = a.ptr[i];
        const int e = (a.row_kind == 2 ? a.pe : a.ptr + 1)[i];
        const bool valid = lane < RPW && row0 + lane < a.N;
        my_beg = valid ? b : 0;
        my_end = valid ? e : 0;
    }
    // (every array below is indexed only by unrolled compile-time indices: a runtime index
    // turns it into LDS / scratch traffic)
    int beg[KR], off[KR + 1];
    off[0] = 0;
#pragma unroll
    for (int k = 0; k < KR; ++k) {
        const int j = sub + G * k;
        beg[k] = __shfl(my_beg, j);
        off[k + 1] = off[k] + (__shfl(my_end, j) - beg[k]);
    }
    const int total = off[KR];
    int steps = total;  // wave maximum over the sub-waves
#pragma unroll
    for (int m = S; m < 64; m <<= 1) steps = max(steps, __shfl_xor(steps, m));
    steps = __builtin_amdgcn_readfirstlane(steps);
    const int row_s = row0 + sub;  // row of ordinal k: row_s + G·k

    const bool has_cnt = a.cnt != nullptr;
    float cntf[KR];
#pragma unroll
    for (int k = 0; k < KR; ++k) {
        const int c = (has_cnt ? a.cnt : a.dummy)[has_cnt ? min(row_s + G * k, a.N - 1) : 0];
        cntf[k] = has_cnt ? (float)c : 1.0f;
    }
    float4 ex[KR], bb = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < KR; ++k) ex[k] = bb;
    if constexpr (EXTRA) {
        const bool has_ex = a.extra != nullptr && a.hi > a.lo;
        const bool has_b = a.bias != nullptr;
        const unsigned me = has_ex ? ~0u : 0u, mb = has_b ? ~0u : 0u;
        auto msk = [](float4 v, unsigned m) {
            return make_float4(__uint_as_float(__float_as_uint(v.x) & m), __uint_as_float(__float_as_uint(v.y) & m),
                               __uint_as_float(__float_as_uint(v.z) & m), __uint_as_float(__float_as_uint(v.w) & m));
        };
#pragma unroll
        for (int k = 0; k < KR; ++k) {
            const int i = min(max(row_s + G * k, a.lo), a.hi - 1);
            const float* eb = has_ex ? a.extra + (size_t)(i - a.lo) * F + col : a.src;
            ex[k] = msk(*reinterpret_cast<const float4*>(eb), me);
        }
        bb = msk(*reinterpret_cast<const float4*>(has_b ? a.bias + col : a.src), mb);
    }

    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int kcur = 0;  // row (of this sub-wave) being summed
    auto flush_to = [&](int kstop) {  // rows kcur .. kstop-1 are complete
        while (kcur < kstop) {
            const int i = row_s + G * kcur;
            if (i < a.N && col_live) {
                const float c = cntf[0];  // slot 0 always holds row kcur's operands
                float4 v = acc;
                if (has_cnt) v = make_float4(v.x / c, v.y / c, v.z / c, v.w / c);
                if constexpr (EXTRA) {
                    if (i >= a.lo && i < a.hi) v = f4_add(f4_add(v, ex[0]), bb);
                }
                *reinterpret_cast<float4*>(a.out + (size_t)(i - a.out_off) * F + col) = v;
            }
            // rows finish in order: shift the per-row operands down one slot (constant indices;
            // selecting slot kcur was folded into an indexed LDS load)
#pragma unroll
            for (int k = 0; k + 1 < KR; ++k) {
                cntf[k] = cntf[k + 1];
                if constexpr (EXTRA) ex[k] = ex[k + 1];
            }
            acc = make_float4(0.f, 0.f, 0.f, 0.f);
            ++kcur;
        }
    };

    for (int vb = 0; vb < steps; vb += S) {
        // entry value of this lane's slot v = vb + sl of its sub-wave (one load per lane)
        const int v = vb + sl;
        int k = 0, q = beg[0] + v;
#pragma unroll
        for (int kk = 1; kk < KR; ++kk) {
            const bool ge = v >= off[kk];
            k = ge ? kk : k;
            q = ge ? beg[kk] + (v - off[kk]) : q;
        }
        const bool in = v < total;
        const bool has_table = a.table != nullptr;  // no table: the entry position is the value
        const int val_raw = (in && has_table ? a.table : a.dummy)[in && has_table ? q : 0];
        const int my_val = in ? (has_table ? val_raw : q) : 0;
        const int my_k = in ? k : KR;
        const int nst = min(S, steps - vb);  // wave-uniform
        for (int u0 = 0; u0 < nst; u0 += U) {
            float4 buf[U];
            int bk[U];
            bool keep[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int srcl = sub * S + min(u0 + u, S - 1);
                const int val = __shfl(my_val, srcl);
                const int kr = (u0 + u < nst) ? __shfl(my_k, srcl) : KR;
                const bool piece = val < 0;
                bool kp = kr < KR;
                if (a.filter) kp = kp && (piece || (val >= a.flo && val < a.fhi));
                int row = piece ? -val - 1 - a.piece_off : val - a.idx_off;
                row = kp ? row : 0;
                const float* base = piece ? a.P : a.src;
                buf[u] = *reinterpret_cast<const float4*>(base + (size_t)row * F + col);
                bk[u] = kr;
                keep[u] = kp;
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (bk[u] < KR && bk[u] != kcur) flush_to(bk[u]);
                if (keep[u]) acc = f4_add(acc, buf[u]);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    flush_to(KR);
}

// ----------------------------------------------------------------------------------------
// outer_accum_kernel:  D[c] = Σ_{p in chunk c} A[a_row(p)]ᵀ ⊗ B[b_row(p)]   (M × Nn, one
// 128 × 128 block per workgroup: grid (chunks, M/128, Nn/128))
//   dW_r = Σ_{seg of r} h_segᵀ dout[node_1(seg)]   (A = H rows, B = dout rows via b_idx)
//   droot = Σ_i x_iᵀ dout_i, dbias = Σ_i dout_i     (A = x, B = dout, contiguous rows)
// A chunk's rows stream through LDS in slices of 32: the index loads run two slices ahead,
// the row loads one slice ahead (registers), so each slice costs one barrier and its MFMAs
// hide the next slice's memory.  The MFMA k-step pairs rows (2t, 2t+1) across the lane halves,
// so a slice of nr rows takes ceil(nr/2) steps — a 3-segment relation runs 2 steps, not 16.
// LDS rows are stored in pairs padded so that rows 2t and 2t+1 fall 32 banks apart (the two
// lane halves of a ds_read_b32 are conflict-free).  D goes to a partial slab P[c] — or, when
// the chunk is its group's only chunk (`dst_idx` ≥ 0), straight into dst[dst_idx]; the ordered
// slab sum (reduce_slabs_kernel) then skips that group.
// ----------------------------------------------------------------------------------------
struct OuterArgs {
    const int* chunk_begin;  // nullable: row chunks [row_lo + c*chunk, ...)
    const int* chunk_end;
    const int* chunk_dst;    // nullable: weight index of a relation's single chunk, else -1
    int chunk_off;
    int dst_mode;            // 0 slabs only; 1 chunk_dst indexes dst (mode ALL); 2 chunk_dst >= 0
                             // means "write dst itself" (one weight); 3 single root chunk -> dst
    int row_lo, row_hi, chunk_rows;
    const float* A;
    int M;
    int a_off;
    const int* a_idx;        // nullable: A row of position p = a_idx[p] >= 0 ? A[a_idx[p]] : A2[-a_idx[p] - 1 - a2_off]
    const float* A2;
    int a2_off;
    const float* B;
    int Nn;
    const int* b_idx;        // nullable
    float* P;                // [nchunks][M][Nn]
    float* dst;              // direct destination (see dst_mode)
    float* Pb;               // nullable: [nchunks][Nn] column sums of B (bias grad)
    float* dst_b;            // direct bias destination when dst_mode == 3
    int bias_of_a;           // outer_bf3_kernel root chunks: Pb = column sums of A instead (M == 128)
    // outer_bf3_kernel on one 128 × 128 quadrant of wider matrices (0 = the 128-wide defaults):
    // A / B row strides and first columns, D / P row stride, the quadrant's element offset in a
    // D / P matrix, elements per P slab, per Pb row
    int lda, ldb, a_col0, b_col0, ldd, d_off, pb_stride;
    int64_t p_stride;
    // outer_bf3v_kernel_t (round 5): nullable [G + 1] first chunk of each workgroup's contiguous
    // chunk range, balanced by slices (outer_ranges); wg_cus > 0: ranges 2c, 2c + 1 on one CU
    const int* wg_chunks;
    int wg_cus;
#ifdef MPGNN_STAMPS
    unsigned long long* stamps;  // debug build: per-slice phase stamps (scripts/stamps_outer.py)
#endif
};

constexpr int kOuterLd = 288;                        // one row pair: 128 + 32 pad + 128
__device__ __forceinline__ int outer_row(int k) { return (k >> 1) * kOuterLd + (k & 1) * 160; }
constexpr int kOuterBuf = (kSlice / 2) * kOuterLd;   // floats per 32-row matrix image
constexpr int kOuterBlock = 32;                      // rows per accumulation block (a multiple of SL)

// SL: rows per slice (32, or 16 = half the LDS, three workgroups per CU: MPGNN_OPT_OUTER_SLICE)
template <bool VEC, int SL = kSlice>
__device__ __forceinline__ void outer_accum_body(const OuterArgs& a, const int cidx) {
    constexpr int OB = (SL / 2) * kOuterLd;  // floats per SL-row matrix image
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* bufs = smem;  // [2 buffers][A, B][OB]
    int p0, p1;
    if (a.chunk_begin != nullptr) {
        p0 = ld_uniform(a.chunk_begin, cidx + a.chunk_off);
        p1 = ld_uniform(a.chunk_end, cidx + a.chunk_off);
    } else {
        p0 = a.row_lo + cidx * a.chunk_rows;
        p1 = min(a.row_hi, p0 + a.chunk_rows);
    }
    const int m_base = blockIdx.y * kColTile;
    const int n_base = blockIdx.z * kColTile;
    const int mcols = min(kColTile, a.M - m_base);
    const int ncols = min(kColTile, a.Nn - n_base);
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int c = lane & 31;
    const int h = lane >> 5;
    const int nslices = (p1 - p0 + SL - 1) / SL;

    // staging: thread t owns float4 slots i = t + j·256 (j < 4) of each 32 × 128 slice:
    // row i >> 5, columns 4·(i & 31) .. +3 (scalar path: 16 floats, row i >> 7, column i & 127)
    constexpr int NS = VEC ? SL * 128 / (4 * kThreads) : SL * 128 / kThreads;
    float4 va[VEC ? NS : 1], vb[VEC ? NS : 1];
    float sa[VEC ? 1 : NS], sb[VEC ? 1 : NS];
    // A and B row index of each staged slot (next slice), loaded one slice earlier
    int ai[NS], bi[NS];
    int ai_next[NS], bi_next[NS];
    auto slot_row = [&](int j) { return VEC ? ((tid + j * kThreads) >> 5) : ((tid + j * kThreads) >> 7); };
    auto slot_col = [&](int j) { return VEC ? 4 * ((tid + j * kThreads) & 31) : ((tid + j * kThreads) & 127); };
    auto load_idx = [&](int slice, int (&oa)[NS], int (&ob)[NS]) {
        const int ps = p0 + slice * SL;
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            const int p = min(ps + slot_row(j), p1 - 1);
            ob[j] = a.b_idx != nullptr ? a.b_idx[p] : p;
            oa[j] = a.a_idx != nullptr ? a.a_idx[p] : p - a.a_off;
        }
    };
    auto arow = [&](int r) {
        return r >= 0 ? a.A + (size_t)r * a.M : a.A2 + (size_t)(-r - 1 - a.a2_off) * a.M;
    };
    auto issue = [&](int slice) {
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            if constexpr (VEC) {
                const int ca = min(m_base + slot_col(j), a.M - 4);
                const int cb = min(n_base + slot_col(j), a.Nn - 4);
                va[j] = *reinterpret_cast<const float4*>(arow(ai[j]) + ca);
                vb[j] = *reinterpret_cast<const float4*>(a.B + (size_t)bi[j] * a.Nn + cb);
            } else {
                const int ca = min(m_base + slot_col(j), a.M - 1);
                const int cb = min(n_base + slot_col(j), a.Nn - 1);
                sa[j] = arow(ai[j])[ca];
                sb[j] = a.B[(size_t)bi[j] * a.Nn + cb];
            }
        }
    };
    auto commit = [&](int slice, float* buf) {
        const int nr = min(SL, p1 - p0 - slice * SL);
        float* Al = buf;
        float* Bl = buf + OB;
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            const int r = slot_row(j);
            const int col = slot_col(j);
            const bool live = r < nr;
            if constexpr (VEC) {
                // bit mask, not a select of the array element (that one went through scratch)
                const unsigned ka = (live && col < mcols) ? ~0u : 0u;
                const unsigned kb = (live && col < ncols) ? ~0u : 0u;
                auto msk = [](float4 v, unsigned k) {
                    return make_float4(__uint_as_float(__float_as_uint(v.x) & k), __uint_as_float(__float_as_uint(v.y) & k),
                                       __uint_as_float(__float_as_uint(v.z) & k), __uint_as_float(__float_as_uint(v.w) & k));
                };
                *reinterpret_cast<float4*>(Al + outer_row(r) + col) = msk(va[j], ka);
                *reinterpret_cast<float4*>(Bl + outer_row(r) + col) = msk(vb[j], kb);
            } else {
                Al[outer_row(r) + col] = (live && col < mcols) ? sa[j] : 0.0f;
                Bl[outer_row(r) + col] = (live && col < ncols) ? sb[j] : 0.0f;
            }
        }
    };

    // acc sums one block of kOuterBlock rows (an fma chain of kOuterBlock products), tot the
    // blocks in row order: the rounding chain of a chunk of n rows is kOuterBlock + n/kOuterBlock
    // instead of n (same for the bias column sums: bblk per block, bsum over blocks)
    f32x16 acc[4], tot[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            acc[q][r] = 0.0f;
            tot[q][r] = 0.0f;
        }
    float bsum = 0.0f, bblk = 0.0f;
    const bool do_bsum = a.Pb != nullptr && blockIdx.y == 0 && tid < kColTile;

    if (nslices > 0) {
        load_idx(0, ai, bi);
        if (nslices > 1) load_idx(1, ai_next, bi_next);
        issue(0);
        commit(0, bufs);
    }
    __syncthreads();
    for (int sl = 0; sl < nslices; ++sl) {
        float* cur = bufs + (sl & 1) * 2 * OB;
        const bool more = sl + 1 < nslices;  // uniform
        if (more) {
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                ai[j] = ai_next[j];
                bi[j] = bi_next[j];
            }
            if (sl + 2 < nslices) load_idx(sl + 2, ai_next, bi_next);
            issue(sl + 1);
        }
        const int nr = min(SL, p1 - p0 - sl * SL);
        if (do_bsum) {
            // rows >= nr were committed as zeros, so all 32 are added (x + 0 = x: same sum as
            // stopping at nr); the loads are independent, only the adds chain, in row order
            const float* Bl = cur + OB;
            float bl[SL];
#pragma unroll
            for (int r = 0; r < SL; ++r) bl[r] = Bl[outer_row(r) + tid];
#pragma unroll
            for (int r = 0; r < SL; ++r) bblk += bl[r];
        }
        // k-step t covers rows 2t (lanes h = 0) and 2t + 1 (h = 1); rows >= nr are zero
        const float* Ar = cur + outer_row(h) + c;
        const float* Br = cur + OB + outer_row(h) + wave * 32 + c;
        const int steps = (nr + 1) >> 1;
        float av[4], bv;
#pragma unroll
        for (int q = 0; q < 4; ++q) av[q] = Ar[q * 32];
        bv = Br[0];
        for (int t = 0; t < steps; ++t) {
            float an[4], bn;
            const int o = (t + 1 < steps ? t + 1 : t) * kOuterLd;  // next pair (rolled one step ahead)
#pragma unroll
            for (int q = 0; q < 4; ++q) an[q] = Ar[o + q * 32];
            bn = Br[o];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q], bv, acc[q], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 4; ++q) av[q] = an[q];
            bv = bn;
        }
        if (((sl + 1) * SL) % kOuterBlock == 0 || !more) {  // block boundary (uniform)
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    tot[q][r] += acc[q][r];
                    acc[q][r] = 0.0f;
                }
            bsum += bblk;
            bblk = 0.0f;
        }
        if (more) commit(sl + 1, bufs + ((sl + 1) & 1) * 2 * OB);
        __syncthreads();
    }

    // destination: the group's only chunk writes the result itself, others a partial slab
    float* D = a.P + (size_t)cidx * a.M * a.Nn;
    float* Db = a.Pb != nullptr ? a.Pb + (size_t)cidx * a.Nn : nullptr;
    if (a.dst_mode == 1 || a.dst_mode == 2) {
        const int di = ld_uniform(a.chunk_dst, cidx + a.chunk_off);
        if (di >= 0) D = a.dst + (size_t)(a.dst_mode == 1 ? di : 0) * a.M * a.Nn;
    } else if (a.dst_mode == 3) {
        D = a.dst;
        Db = a.dst_b;
    }
    const int col = n_base + wave * 32 + c;
    if (D != nullptr && wave * 32 < ncols && col < a.Nn) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m_base + q * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (m < a.M) D[(size_t)m * a.Nn + col] = tot[q][r];
            }
        }
    }
    if (do_bsum && Db != nullptr && tid < ncols) Db[n_base + tid] = bsum;
}

template <bool VEC>
__global__ __launch_bounds__(kThreads, 2) void outer_accum_kernel(OuterArgs a) {
    outer_accum_body<VEC>(a, (int)blockIdx.x);
}

// Persistent form of the two-part outer-product launch: workgroup w walks the chunks w, w + G, …
// of [root chunks (`ra`, ra_n of them) | weight chunks (`wa`)] as ONE stream of 16-row slices —
// the next slice's rows (and the row indices of the one after) are in flight during the current
// slice's MFMAs ACROSS chunk boundaries, so no chunk pays a cold prologue; a finished chunk's
// partial goes out after the next slice is committed (its stores never hold up a commit).
// Same arithmetic per chunk as outer_accum_body (32-row blocks, block totals in row order).
struct OuterCursor {
    int pos;        // position in the workgroup's chunk sequence (outer_bf3v_kernel_t; else = chunk)
    int chunk;      // global chunk id: [0, ra_n) root chunks, then weight chunks
    int sl, ns;     // slice within the chunk, slices of the chunk
    int p0, p1;     // the chunk's row range
};

template <bool VEC, int SL>
__global__ __launch_bounds__(kThreads, 2) void outer_persist_kernel(OuterArgs ra, OuterArgs wa, int ra_n, int n_all) {
    constexpr int OB = (SL / 2) * kOuterLd;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* bufs = smem;  // [2 buffers][A, B][OB]
    const int G = (int)gridDim.x;
    if ((int)blockIdx.x >= n_all) return;
    const int m_base = blockIdx.y * kColTile;
    const int n_base = blockIdx.z * kColTile;
    const int M = wa.M, Nn = wa.Nn;  // same widths in both parts
    const int mcols = min(kColTile, M - m_base);
    const int ncols = min(kColTile, Nn - n_base);
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int c = lane & 31;
    const int h = lane >> 5;

    // the two parts' fields selected BY VALUE (wave-uniform ternaries stay in SGPRs; a reference
    // to a kernel-argument struct picked at run time would put both structs in scratch)
    struct Src {
        const float *A, *A2, *B;
        const int *a_idx, *b_idx;
        int a_off, a2_off;
    };
    auto src_of = [&](int chunk) {
        const bool r = chunk < ra_n;
        Src x;
        x.A = r ? ra.A : wa.A;
        x.A2 = r ? ra.A2 : wa.A2;
        x.B = r ? ra.B : wa.B;
        x.a_idx = r ? ra.a_idx : wa.a_idx;
        x.b_idx = r ? ra.b_idx : wa.b_idx;
        x.a_off = r ? ra.a_off : wa.a_off;
        x.a2_off = r ? ra.a2_off : wa.a2_off;
        return x;
    };
    // every chunk holds >= 1 row (relation chunks by construction, root chunks by their count)
    auto open_chunk = [&](int chunk) {
        OuterCursor k;
        k.chunk = chunk;
        k.sl = 0;
        int p0 = 0, p1 = 0;
        if (chunk < ra_n) {  // root chunks: fixed-length row ranges
            p0 = ra.row_lo + chunk * ra.chunk_rows;
            p1 = min(ra.row_hi, p0 + ra.chunk_rows);
        } else if (chunk < n_all) {  // relation-pure weight chunks
            p0 = ld_uniform(wa.chunk_begin, chunk - ra_n + wa.chunk_off);
            p1 = ld_uniform(wa.chunk_end, chunk - ra_n + wa.chunk_off);
        }
        k.p0 = p0;
        k.p1 = p1;
        k.ns = (p1 - p0 + SL - 1) / SL;
        return k;
    };
    auto advance = [&](const OuterCursor& k) {
        if (k.sl + 1 < k.ns) {
            OuterCursor n = k;
            n.sl = k.sl + 1;
            return n;
        }
        return open_chunk(k.chunk + G);
    };
    auto valid = [&](const OuterCursor& k) { return k.chunk < n_all && k.ns > 0; };

    constexpr int NS = VEC ? SL * 128 / (4 * kThreads) : SL * 128 / kThreads;
    float4 va[VEC ? NS : 1], vb[VEC ? NS : 1];
    float sa[VEC ? 1 : NS], sb[VEC ? 1 : NS];
    int ai[NS], bi[NS], ai_next[NS], bi_next[NS];
    auto slot_row = [&](int j) { return VEC ? ((tid + j * kThreads) >> 5) : ((tid + j * kThreads) >> 7); };
    auto slot_col = [&](int j) { return VEC ? 4 * ((tid + j * kThreads) & 31) : ((tid + j * kThreads) & 127); };
    auto load_idx = [&](const OuterCursor& k, int (&oa)[NS], int (&ob)[NS]) {
        const Src a = src_of(k.chunk);
        const int ps = k.p0 + k.sl * SL;
        const int last = max(k.p1 - 1, k.p0);
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            const int p = min(ps + slot_row(j), last);
            ob[j] = a.b_idx != nullptr ? a.b_idx[p] : p;
            oa[j] = a.a_idx != nullptr ? a.a_idx[p] : p - a.a_off;
        }
    };
    auto issue = [&](const OuterCursor& k) {
        const Src a = src_of(k.chunk);
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            const float* ar = ai[j] >= 0 ? a.A + (size_t)ai[j] * M : a.A2 + (size_t)(-ai[j] - 1 - a.a2_off) * M;
            if constexpr (VEC) {
                const int ca = min(m_base + slot_col(j), M - 4);
                const int cb = min(n_base + slot_col(j), Nn - 4);
                va[j] = *reinterpret_cast<const float4*>(ar + ca);
                vb[j] = *reinterpret_cast<const float4*>(a.B + (size_t)bi[j] * Nn + cb);
            } else {
                const int ca = min(m_base + slot_col(j), M - 1);
                const int cb = min(n_base + slot_col(j), Nn - 1);
                sa[j] = ar[ca];
                sb[j] = a.B[(size_t)bi[j] * Nn + cb];
            }
        }
    };
    auto commit = [&](const OuterCursor& k, float* buf) {
        const int nr = min(SL, k.p1 - k.p0 - k.sl * SL);
        float* Al = buf;
        float* Bl = buf + OB;
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            const int r = slot_row(j);
            const int col = slot_col(j);
            const bool live = r < nr;
            if constexpr (VEC) {
                const unsigned ka = (live && col < mcols) ? ~0u : 0u;
                const unsigned kb = (live && col < ncols) ? ~0u : 0u;
                auto msk = [](float4 v, unsigned m) {
                    return make_float4(__uint_as_float(__float_as_uint(v.x) & m), __uint_as_float(__float_as_uint(v.y) & m),
                                       __uint_as_float(__float_as_uint(v.z) & m), __uint_as_float(__float_as_uint(v.w) & m));
                };
                *reinterpret_cast<float4*>(Al + outer_row(r) + col) = msk(va[j], ka);
                *reinterpret_cast<float4*>(Bl + outer_row(r) + col) = msk(vb[j], kb);
            } else {
                Al[outer_row(r) + col] = (live && col < mcols) ? sa[j] : 0.0f;
                Bl[outer_row(r) + col] = (live && col < ncols) ? sb[j] : 0.0f;
            }
        }
    };

    f32x16 acc[4], tot[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            acc[q][r] = 0.0f;
            tot[q][r] = 0.0f;
        }
    float bsum = 0.0f, bblk = 0.0f;

    OuterCursor cur = open_chunk((int)blockIdx.x);
    if (!valid(cur)) return;
    OuterCursor nx = advance(cur);   // rows in flight during cur
    OuterCursor nn = valid(nx) ? advance(nx) : nx;  // row indices in flight during cur
    load_idx(cur, ai, bi);
    if (valid(nx)) load_idx(nx, ai_next, bi_next);
    issue(cur);
    commit(cur, bufs);
    __syncthreads();
    int buf = 0;
    while (true) {
        float* cbuf = bufs + buf * 2 * OB;
        const bool more = valid(nx);
        if (more) {
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                ai[j] = ai_next[j];
                bi[j] = bi_next[j];
            }
            if (valid(nn)) load_idx(nn, ai_next, bi_next);
            issue(nx);
        }
        const bool is_root = cur.chunk < ra_n;
        const bool do_bsum = is_root && ra.Pb != nullptr && blockIdx.y == 0 && tid < kColTile;
        const int nr = min(SL, cur.p1 - cur.p0 - cur.sl * SL);
        if (do_bsum) {
            const float* Bl = cbuf + OB;
            float bl[SL];
#pragma unroll
            for (int r = 0; r < SL; ++r) bl[r] = Bl[outer_row(r) + tid];
#pragma unroll
            for (int r = 0; r < SL; ++r) bblk += bl[r];
        }
        const float* Ar = cbuf + outer_row(h) + c;
        const float* Br = cbuf + OB + outer_row(h) + wave * 32 + c;
        const int steps = (nr + 1) >> 1;
        float av[4], bv;
#pragma unroll
        for (int q = 0; q < 4; ++q) av[q] = Ar[q * 32];
        bv = Br[0];
        // one k-step as a lambda, no scheduling barriers: the code the compiler makes of this form
        // interleaves the next step's LDS reads with the MFMAs best (C3 103.4 -> 99.9 us, C2
        // 407 -> 396 us per layer vs the grouped, barrier-fenced plain loop; same arithmetic)
        auto kstep = [&](int t) {
            float an[4], bn;
            const int o = (t + 1 < steps ? t + 1 : t) * kOuterLd;
#pragma unroll
            for (int q = 0; q < 4; ++q) an[q] = Ar[o + q * 32];
            bn = Br[o];
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q], bv, acc[q], 0, 0, 0);
#pragma unroll
            for (int q = 0; q < 4; ++q) av[q] = an[q];
            bv = bn;
        };
        for (int t = 0; t < steps; ++t) kstep(t);
        const bool chunk_end = cur.sl + 1 == cur.ns;
        if (((cur.sl + 1) * SL) % kOuterBlock == 0 || chunk_end) {  // block boundary (uniform)
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    tot[q][r] += acc[q][r];
                    acc[q][r] = 0.0f;
                }
            bsum += bblk;
            bblk = 0.0f;
        }
        if (more) commit(nx, bufs + (buf ^ 1) * 2 * OB);  // before the chunk's stores (in-order vmcnt)
        if (chunk_end) {
            float* D;
            float* Db = nullptr;
            if (is_root) {
                const int cidx = cur.chunk;
                D = ra.P + (size_t)cidx * M * Nn;
                Db = ra.Pb != nullptr ? ra.Pb + (size_t)cidx * Nn : nullptr;
                if (ra.dst_mode == 3) {
                    D = ra.dst;
                    Db = ra.dst_b;
                }
            } else {
                const int cidx = cur.chunk - ra_n;
                D = wa.P + (size_t)cidx * M * Nn;
                if (wa.dst_mode == 1 || wa.dst_mode == 2) {
                    const int di = ld_uniform(wa.chunk_dst, cidx + wa.chunk_off);
                    if (di >= 0) D = wa.dst + (size_t)(wa.dst_mode == 1 ? di : 0) * M * Nn;
                }
            }
            // laundered lane offsets: otherwise LICM hoists the 64 store offsets out of the chunk
            // loop and holds them live across it (spills)
            const int ln = opaque(lane);
            const int col = n_base + wave * 32 + (ln & 31);
            const int h4 = 4 * (ln >> 5);
            if (D != nullptr && wave * 32 < ncols && col < Nn) {
                float* Dc = D + col;
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int m = m_base + q * 32 + (r & 3) + 8 * (r >> 2) + h4;
                        if (m < M) Dc[(size_t)m * Nn] = tot[q][r];
                    }
            }
            if (do_bsum && Db != nullptr && tid < ncols) Db[n_base + tid] = bsum;
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int r = 0; r < 16; ++r) tot[q][r] = 0.0f;
            bsum = 0.0f;
        }
        __syncthreads();
        if (!more) break;
        cur = nx;
        nx = nn;
        nn = valid(nn) ? advance(nn) : nn;
        buf ^= 1;
    }
}

// ----------------------------------------------------------------------------------------
// outer_bf3_kernel — outer_persist_kernel's persistent chunk stream (same chunks, cursors,
// destinations, bias column sums) for M = Nn = 128 on the bf16 matrix cores with the exact
// three-way operand split of rel_gemm_bf3_kernel:  D[m][n] += Σ_p A[p][m] · B[p][n].
// The K dimension of v_mfma_f32_32x32x16_bf16 runs over the chunk's ROWS, so both operands are
// read "down a column": a slice of 16 rows is staged TRANSPOSED in LDS as three bf16 planes per
// matrix, [128 columns][16 rows + 8 pad] (48-B column stride: the 16-B fragment reads and the
// 16-B plane writes are bank-conflict-free). Thread t stages column t & 127 of rows
// 8·(t >> 7) .. +8 of both matrices: the rows of a wave are uniform, so their bases come from
// readlane (SGPRs) and every load is a coalesced 256-B row piece. Rows are fetched two slices
// ahead (two register sets alternating roles), row indices three. Wave w owns output columns
// [32w, 32w + 32) and all 128 m: 4 blocks × (hi, lo) accumulators; per 16 rows 24 MFMAs.
// ----------------------------------------------------------------------------------------
constexpr int kOb3Ld = 24;                  // bf16 per plane column: 16 rows + 8 pad
constexpr int kOb3Plane = 128 * kOb3Ld;     // bf16 per plane
constexpr size_t kOb3Lds = (size_t)2 * 6 * kOb3Plane * 2 + 256 * sizeof(float);  // 2 buffers × 6 planes + bias exchange

__global__ __launch_bounds__(kThreads, 2) void outer_bf3_kernel(OuterArgs ra, OuterArgs wa, int ra_n, int n_all) {
    constexpr int SL = 16;
    extern __shared__ __attribute__((aligned(16))) __bf16 ob3_smem[];
    __bf16* planes = ob3_smem;                                          // [2][A0 A1 A2 B0 B1 B2][128][24]
    float* bx = reinterpret_cast<float*>(ob3_smem + 2 * 6 * kOb3Plane);  // [256] bias exchange
    const int G = (int)gridDim.x;
    if ((int)blockIdx.x >= n_all) return;
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int c = lane & 31;
    const int h = lane >> 5;
    const int col = tid & 127;                                         // staged column
    const int half = __builtin_amdgcn_readfirstlane(tid >> 7);         // staged rows 8·half .. +8 (uniform)

    struct Src {
        const float *A, *A2, *B;
        const int *a_idx, *b_idx;
        int a_off, a2_off;
    };
    // quadrant geometry (the same for both chunk streams; 0 = the 128-wide defaults)
    const int lda = ra.lda ? ra.lda : 128, ldb = ra.ldb ? ra.ldb : 128, ldd = ra.ldd ? ra.ldd : 128;
    const int pb_stride = ra.pb_stride ? ra.pb_stride : 128;
    const int64_t p_stride = ra.p_stride ? ra.p_stride : 128 * 128;
    auto src_of = [&](int chunk) {
        const bool r = chunk < ra_n;
        Src x;
        x.A = (r ? ra.A : wa.A) + ra.a_col0;
        x.A2 = (r ? ra.A2 : wa.A2) + ra.a_col0;
        x.B = (r ? ra.B : wa.B) + ra.b_col0;
        x.a_idx = r ? ra.a_idx : wa.a_idx;
        x.b_idx = r ? ra.b_idx : wa.b_idx;
        x.a_off = r ? ra.a_off : wa.a_off;
        x.a2_off = r ? ra.a2_off : wa.a2_off;
        return x;
    };
    auto open_chunk = [&](int chunk) {
        OuterCursor k;
        k.chunk = chunk;
        k.sl = 0;
        int p0 = 0, p1 = 0;
        if (chunk < ra_n) {
            p0 = ra.row_lo + chunk * ra.chunk_rows;
            p1 = min(ra.row_hi, p0 + ra.chunk_rows);
        } else if (chunk < n_all) {
            p0 = ld_uniform(wa.chunk_begin, chunk - ra_n + wa.chunk_off);
            p1 = ld_uniform(wa.chunk_end, chunk - ra_n + wa.chunk_off);
        }
        k.p0 = p0;
        k.p1 = p1;
        k.ns = (p1 - p0 + SL - 1) / SL;
        return k;
    };
    auto advance = [&](const OuterCursor& k) {
        if (k.sl + 1 < k.ns) {
            OuterCursor n = k;
            n.sl = k.sl + 1;
            return n;
        }
        return open_chunk(k.chunk + G);
    };
    auto valid = [&](const OuterCursor& k) { return k.chunk < n_all && k.ns > 0; };

    // row indices of a slice: lanes 0..7 of the wave hold those of its 8 staged rows
    auto load_idx = [&](const OuterCursor& k, int& ia, int& ib) {
        const Src a = src_of(k.chunk);
        const int p = min(k.p0 + k.sl * SL + 8 * half + (lane & 7), max(k.p1 - 1, k.p0));
        ib = a.b_idx != nullptr ? a.b_idx[p] : p;
        ia = a.a_idx != nullptr ? a.a_idx[p] : p - a.a_off;
    };
    // rows of a slice into registers (row bases uniform: readlane of the index lanes)
    auto issue = [&](const OuterCursor& k, int ia, int ib, float (&va)[8], float (&vb)[8]) {
        const Src a = src_of(k.chunk);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int ra_ = __builtin_amdgcn_readlane(ia, j);
            const int rb_ = __builtin_amdgcn_readlane(ib, j);
            const float* arow = ra_ >= 0 ? a.A + (size_t)ra_ * lda : a.A2 + (size_t)(-ra_ - 1 - a.a2_off) * lda;
            va[j] = arow[col];
            vb[j] = a.B[(size_t)rb_ * ldb + col];
        }
    };
    // split + transposed store of one staged slice; rows past the chunk's end are zeros
    auto commit = [&](const OuterCursor& k, const float (&va)[8], const float (&vb)[8], __bf16* buf) {
        const int nr = min(SL, k.p1 - k.p0 - k.sl * SL) - 8 * half;  // live rows of this half (uniform)
        bf16x8 pa[3], pb[3];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float xa = j < nr ? va[j] : 0.0f;
            const float xb = j < nr ? vb[j] : 0.0f;
            __bf16 a0, a1, a2, b0, b1, b2;
            split3_bf16(xa, a0, a1, a2);
            split3_bf16(xb, b0, b1, b2);
            pa[0][j] = a0; pa[1][j] = a1; pa[2][j] = a2;
            pb[0][j] = b0; pb[1][j] = b1; pb[2][j] = b2;
        }
        __bf16* d = buf + col * kOb3Ld + 8 * half;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            *reinterpret_cast<bf16x8*>(d + q * kOb3Plane) = pa[q];
            *reinterpret_cast<bf16x8*>(d + (3 + q) * kOb3Plane) = pb[q];
        }
    };

    f32x16 hi[4], lo[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            hi[q][r] = 0.0f;
            lo[q][r] = 0.0f;
        }
    float bpart = 0.0f;  // this thread's share of its column's bias sum (root chunks)

    OuterCursor cur = open_chunk((int)blockIdx.x);
    if (!valid(cur)) return;
    OuterCursor c1 = advance(cur);                 // rows in set X during cur
    OuterCursor c2 = valid(c1) ? advance(c1) : c1;  // rows issued into set Y during cur
    OuterCursor c3 = valid(c2) ? advance(c2) : c2;  // indices loaded during cur
    float xa[8], xb[8], ya[8], yb[8];
    int ia, ib, ja = 0, jb = 0;
    load_idx(cur, ia, ib);
    issue(cur, ia, ib, xa, xb);
    commit(cur, xa, xb, planes);
    if (valid(c1)) {
        load_idx(c1, ia, ib);
        issue(c1, ia, ib, xa, xb);
    }
    if (valid(c2)) load_idx(c2, ja, jb);
    __syncthreads();
    int buf = 0;
    // one slice: vn receives the rows of c2, vc (rows of c1) is committed after the MFMAs
    auto step = [&](float (&vca)[8], float (&vcb)[8], float (&vna)[8], float (&vnb)[8]) -> bool {
        const bool more = valid(c1);
        if (valid(c2)) {
            issue(c2, ja, jb, vna, vnb);
            if (valid(c3)) load_idx(c3, ja, jb);
        }
        const bool is_root = cur.chunk < ra_n;
        const __bf16* cb = planes + buf * 6 * kOb3Plane;
        // B fragment (this wave's 32 columns) and per m-block A fragments, 6 products each
        const __bf16* Bf = cb + 3 * kOb3Plane + (wave * 32 + c) * kOb3Ld + 8 * h;
        const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(Bf);
        const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(Bf + kOb3Plane);
        const bf16x8 b2 = *reinterpret_cast<const bf16x8*>(Bf + 2 * kOb3Plane);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const __bf16* Af = cb + (q * 32 + c) * kOb3Ld + 8 * h;
            const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(Af);
            const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(Af + kOb3Plane);
            const bf16x8 a2 = *reinterpret_cast<const bf16x8*>(Af + 2 * kOb3Plane);
            lo[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, lo[q], 0, 0, 0);
            lo[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, lo[q], 0, 0, 0);
            lo[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, lo[q], 0, 0, 0);
            lo[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, lo[q], 0, 0, 0);
            lo[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, lo[q], 0, 0, 0);
            hi[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, hi[q], 0, 0, 0);
        }
        if (is_root && ra.Pb != nullptr) {  // bias: the column sum of dout over the chunk's rows
            const int nr = min(SL, cur.p1 - cur.p0 - cur.sl * SL) - 8 * half;
            // this thread's column over its 8 rows of cur's slice, rebuilt exactly from the three
            // pieces in LDS ((b0 + b1) + b2 == b: the partial sums of the split are representable)
            const __bf16* bc = cb + (ra.bias_of_a ? 0 : 3 * kOb3Plane) + col * kOb3Ld + 8 * half;
            const bf16x8 q0 = *reinterpret_cast<const bf16x8*>(bc);
            const bf16x8 q1 = *reinterpret_cast<const bf16x8*>(bc + kOb3Plane);
            const bf16x8 q2 = *reinterpret_cast<const bf16x8*>(bc + 2 * kOb3Plane);
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (j < nr) bpart += ((float)q0[j] + (float)q1[j]) + (float)q2[j];
        }
        const bool chunk_end = cur.sl + 1 == cur.ns;
        if (more) commit(c1, vca, vcb, planes + (buf ^ 1) * 6 * kOb3Plane);
        if (chunk_end) {
            float* D;
            float* Db = nullptr;
            if (is_root) {
                const int cidx = cur.chunk;
                D = ra.P + (size_t)cidx * p_stride + ra.d_off;
                Db = ra.Pb != nullptr ? ra.Pb + (size_t)cidx * pb_stride + ra.b_col0 : nullptr;
                if (ra.dst_mode == 3) {
                    D = ra.dst != nullptr ? ra.dst + ra.d_off : nullptr;
                    Db = ra.dst_b != nullptr ? ra.dst_b + ra.b_col0 : nullptr;
                }
            } else {
                const int cidx = cur.chunk - ra_n;
                D = wa.P + (size_t)cidx * p_stride + ra.d_off;
                if (wa.dst_mode == 1 || wa.dst_mode == 2) {
                    const int di = ld_uniform(wa.chunk_dst, cidx + wa.chunk_off);
                    if (di >= 0) D = wa.dst + (size_t)(wa.dst_mode == 1 ? di : 0) * p_stride + ra.d_off;
                }
            }
            const int ln = opaque(lane);
            const int ocol = wave * 32 + (ln & 31);
            const int h4 = 4 * (ln >> 5);
            if (D != nullptr) {  // (a bias-only root part has no weight destination)
                float* Dc = D + ocol;
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int m = q * 32 + (r & 3) + 8 * (r >> 2) + h4;
                        Dc[(size_t)m * ldd] = hi[q][r] + lo[q][r];
                    }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    hi[q][r] = 0.0f;
                    lo[q][r] = 0.0f;
                }
            if (is_root && ra.Pb != nullptr) {  // the two row-halves of each column, in order
                bx[tid] = bpart;
                bpart = 0.0f;
                __syncthreads();
                if (tid < 128 && Db != nullptr) Db[tid] = bx[tid] + bx[tid + 128];
            }
        }
        __syncthreads();
        if (!more) return false;
        cur = c1;
        c1 = c2;
        c2 = c3;
        c3 = valid(c3) ? advance(c3) : c3;
        buf ^= 1;
        return true;
    };
    while (step(xa, xb, ya, yb) && step(ya, yb, xa, xb)) {
    }
}

// ----------------------------------------------------------------------------------------
// outer_bf3v_kernel — outer_bf3_kernel (same chunk streams, cursors, destinations, pipeline,
// six-product split, accumulators, epilogue) with 16-byte row gathers: a slice's 16 rows are
// staged ROW-major, thread t holding columns 4·(t & 31) .. +3 of rows (t >> 5) and (t >> 5) + 8
// of both matrices (4 float4 loads per slice instead of 16 dword loads: outer_bf3_kernel issued
// 2.4x the forward GEMM's vector-memory instructions), and the MFMA fragments, which run down
// the columns (K = the slice's rows), are read with ds_read_b64_tr_b16 (gfx950's transposed LDS
// read: a 16-lane group reads 4 rows × 16 columns, lane i receives column i).  Planes
// [16 rows][160] bf16: the 320-B row stride puts the four rows of a transposed read on disjoint
// bank quarters (conflict-free).  The bias column sums (root chunks) are taken per thread over
// its own 4 columns × 2 rows, exact from the three pieces as in outer_bf3_kernel, and the 8
// row-group partials of each column are added in order at the chunk's end.
// ----------------------------------------------------------------------------------------
constexpr int kOvLd = 160;                       // bf16 per staged row: 128 + 32 pad (320 B)
constexpr int kOvPlane = 16 * kOvLd;             // bf16 per plane (16 rows)
constexpr size_t kOvLds = (size_t)2 * 6 * kOvPlane * 2 + 8 * 128 * sizeof(float);  // 2 buffers × 6 planes + bias partials
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// 8 consecutive k (rows k0 .. k0 + 8 of a plane) of column `col0 + (lane & 15)` for the lane's
// 16-lane group: two transposed reads of 4 rows each (lane 4q + p addresses row k0 + q,
// columns col0 + 4p .. +3)
__device__ __forceinline__ bf16x8 ov_frag(const __bf16* plane, int k0, int col0, int lane) {
    const int i = lane & 15;
    const __bf16* base = plane + (k0 + (i >> 2)) * kOvLd + col0 + 4 * (i & 3);
    typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(base));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(base + 4 * kOvLd));
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// SQ (round 5, MPGNN_OPT_OUTER_SQ): each wave owns a 64 × 64 quarter of the 128 × 128 slab (2 × 2
// blocks of 32 × 32: twelve fragments per k-step, 24 transposed reads for 24 MFMAs, against 15
// fragments / 30 reads for a 128 × 32 strip), and the next slice's commit is scheduled among the
// MFMAs (branch-free; past the last slice it writes zeros nobody reads). Same products, same
// per-block accumulators: bit-identical slabs.
// VAR (round 6, MPGNN_OPT_OUTER_VARIANT; same rows, same products: bit-identical slabs):
//   1 (SIDX) a slice's four row indices per wave (wave-uniform values) are fetched with scalar loads
//     instead of lane-0..3 vector loads read back by readlane: counted by lgkmcnt, so an index wait
//     no longer covers the row loads and slab stores issued before it (measured slower: 64 -> 69 µs,
//     each scalar wait drains the wave's LDS operations too);
//   2 (LATE) the rows of the slice two ahead are issued AFTER this slice's fragment reads and MFMAs,
//     not before them: the vector-memory wait that the index of that slice implies (it covers the
//     rows of the next slice, issued one slice earlier) then falls behind the MFMAs already queued
//     instead of in front of them (the stamps put ~1 k of a slice's ~4.5 k cycles there).
template <bool SQ, int VAR = 0>
__global__ __launch_bounds__(kThreads, 2) void outer_bf3v_kernel_t(OuterArgs ra, OuterArgs wa, int ra_n, int n_all) {
    constexpr int SL = 16;
    extern __shared__ __attribute__((aligned(16))) __bf16 ov_smem[];
    __bf16* planes = ov_smem;                                         // [2][A0 A1 A2 B0 B1 B2][16][160]
    float* bx = reinterpret_cast<float*>(ov_smem + 2 * 6 * kOvPlane);  // [8 row groups][128] bias partials
    const int G = (int)gridDim.x;
    // the workgroup's chunks: its list of the host's window-balanced deal (outer_ranges), or every
    // G-th chunk. Cursors walk list positions; chunk id = list[position]
    int c_beg = (int)blockIdx.x, c_end = n_all, c_step = G;
    const int* clist = nullptr;
    if (ra.wg_chunks != nullptr) {
        c_beg = ld_uniform(ra.wg_chunks, (int)blockIdx.x);
        c_end = ld_uniform(ra.wg_chunks, (int)blockIdx.x + 1);
        c_step = 1;
        clist = ra.wg_chunks + G + 1;
    }
    if (c_beg >= c_end) return;
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int c = lane & 31;
    const int h = lane >> 5;
    const int srow = tid >> 5;         // staged rows srow, srow + 8 (0 .. 7: two per wave)
    const int scol = (tid & 31) * 4;   // staged columns scol .. +3

    struct Src {
        const float *A, *A2, *B;
        const int *a_idx, *b_idx;
        int a_off, a2_off;
    };
    const int lda = ra.lda ? ra.lda : 128, ldb = ra.ldb ? ra.ldb : 128, ldd = ra.ldd ? ra.ldd : 128;
    const int pb_stride = ra.pb_stride ? ra.pb_stride : 128;
    const int64_t p_stride = ra.p_stride ? ra.p_stride : 128 * 128;
    auto src_of = [&](int chunk) {
        const bool r = chunk < ra_n;
        Src x;
        x.A = (r ? ra.A : wa.A) + ra.a_col0;
        x.A2 = (r ? ra.A2 : wa.A2) + ra.a_col0;
        x.B = (r ? ra.B : wa.B) + ra.b_col0;
        x.a_idx = r ? ra.a_idx : wa.a_idx;
        x.b_idx = r ? ra.b_idx : wa.b_idx;
        x.a_off = r ? ra.a_off : wa.a_off;
        x.a2_off = r ? ra.a2_off : wa.a2_off;
        return x;
    };
    auto open_chunk = [&](int pos) {
        OuterCursor k;
        k.pos = pos;
        const int chunk = pos < c_end ? (clist != nullptr ? ld_uniform(clist, pos) : pos) : n_all;
        k.chunk = chunk;
        k.sl = 0;
        int p0 = 0, p1 = 0;
        if (chunk < ra_n) {
            p0 = ra.row_lo + chunk * ra.chunk_rows;
            p1 = min(ra.row_hi, p0 + ra.chunk_rows);
        } else if (chunk < n_all) {
            p0 = ld_uniform(wa.chunk_begin, chunk - ra_n + wa.chunk_off);
            p1 = ld_uniform(wa.chunk_end, chunk - ra_n + wa.chunk_off);
        }
        k.p0 = p0;
        k.p1 = p1;
        k.ns = (p1 - p0 + SL - 1) / SL;
        return k;
    };
    auto advance = [&](const OuterCursor& k) {
        if (k.sl + 1 < k.ns) {
            OuterCursor n = k;
            n.sl = k.sl + 1;
            return n;
        }
        return open_chunk(k.pos + c_step);
    };
    auto valid = [&](const OuterCursor& k) { return k.pos < c_end && k.ns > 0; };

    // row indices of a slice: lanes 0..3 of the wave hold those of its staged rows
    // 2·wave, 2·wave + 1, 2·wave + 8, 2·wave + 9
    constexpr bool SIDX = VAR == 1;
    struct Idx {  // SIDX: the four rows' indices (uniform); else lanes 0..3 of .a[0] / .b[0]
        int a[4], b[4];
    };
    auto load_idx = [&](const OuterCursor& k, Idx& x) {
        const Src a = src_of(k.chunk);
        if constexpr (SIDX) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int r = 2 * wave + (q & 1) + 8 * (q >> 1);
                const int p = min(k.p0 + k.sl * SL + r, max(k.p1 - 1, k.p0));
                x.b[q] = a.b_idx != nullptr ? ld_uniform(a.b_idx, p) : p;
                x.a[q] = a.a_idx != nullptr ? ld_uniform(a.a_idx, p) : p - a.a_off;
            }
        } else {
            const int r = 2 * wave + (lane & 1) + 8 * ((lane >> 1) & 1);
            const int p = min(k.p0 + k.sl * SL + r, max(k.p1 - 1, k.p0));
            x.b[0] = a.b_idx != nullptr ? a.b_idx[p] : p;
            x.a[0] = a.a_idx != nullptr ? a.a_idx[p] : p - a.a_off;
        }
    };
    // this lane's two rows (srow: index lane 0 | 1 by half; srow + 8: lane 2 | 3) as float4
    auto issue = [&](const OuterCursor& k, const Idx& x, float4 (&va)[2], float4 (&vb)[2]) {
        const Src a = src_of(k.chunk);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            int a0, a1, b0, b1;
            if constexpr (SIDX) {
                a0 = x.a[2 * j]; a1 = x.a[2 * j + 1];
                b0 = x.b[2 * j]; b1 = x.b[2 * j + 1];
            } else {
                a0 = __builtin_amdgcn_readlane(x.a[0], 2 * j); a1 = __builtin_amdgcn_readlane(x.a[0], 2 * j + 1);
                b0 = __builtin_amdgcn_readlane(x.b[0], 2 * j); b1 = __builtin_amdgcn_readlane(x.b[0], 2 * j + 1);
            }
            const int ra_ = h ? a1 : a0, rb_ = h ? b1 : b0;
            const float* arow = ra_ >= 0 ? a.A + (size_t)ra_ * lda : a.A2 + (size_t)(-ra_ - 1 - a.a2_off) * lda;
            va[j] = *reinterpret_cast<const float4*>(arow + scol);
            vb[j] = *reinterpret_cast<const float4*>(a.B + (size_t)rb_ * ldb + scol);
        }
    };
    // split + row-major store of one staged slice; rows past the chunk's end are zeros
    auto commit = [&](const OuterCursor& k, const float4 (&va)[2], const float4 (&vb)[2], __bf16* buf) {
        const int nr = min(SL, k.p1 - k.p0 - k.sl * SL);  // live rows of the slice
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const bool live = srow + 8 * j < nr;
            const float4 xa = live ? va[j] : make_float4(0.f, 0.f, 0.f, 0.f);
            const float4 xb = live ? vb[j] : make_float4(0.f, 0.f, 0.f, 0.f);
            const float fa[4] = {xa.x, xa.y, xa.z, xa.w}, fb[4] = {xb.x, xb.y, xb.z, xb.w};
            bf16x4 pa[3], pb[3];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                __bf16 a0, a1, a2, b0, b1, b2;
                split3_bf16(fa[e], a0, a1, a2);
                split3_bf16(fb[e], b0, b1, b2);
                pa[0][e] = a0; pa[1][e] = a1; pa[2][e] = a2;
                pb[0][e] = b0; pb[1][e] = b1; pb[2][e] = b2;
            }
            __bf16* d = buf + (srow + 8 * j) * kOvLd + scol;
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                *reinterpret_cast<bf16x4*>(d + q * kOvPlane) = pa[q];
                *reinterpret_cast<bf16x4*>(d + (3 + q) * kOvPlane) = pb[q];
            }
        }
    };

    f32x16 hi[4], lo[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            hi[q][r] = 0.0f;
            lo[q][r] = 0.0f;
        }
    float bpart[4] = {0.0f, 0.0f, 0.0f, 0.0f};  // this thread's columns over its rows (root chunks)

    OuterCursor cur = open_chunk(c_beg);
    if (!valid(cur)) return;
#ifdef MPGNN_STAMPS
    stamp_id_at(ra.stamps);
    int nsl = 0;  // slices done (stamped while < kStampItems)
#endif
    OuterCursor c1 = advance(cur);
    OuterCursor c2 = valid(c1) ? advance(c1) : c1;
    OuterCursor c3 = valid(c2) ? advance(c2) : c2;
    float4 xa[2], xb[2], ya[2], yb[2];
    Idx ii, jj;
#pragma unroll
    for (int q = 0; q < 4; ++q) jj.a[q] = jj.b[q] = 0;
    load_idx(cur, ii);
    issue(cur, ii, xa, xb);
    commit(cur, xa, xb, planes);
    if (valid(c1)) {
        load_idx(c1, ii);
        issue(c1, ii, xa, xb);
    }
    if (valid(c2)) load_idx(c2, jj);
    __syncthreads();
    int buf = 0;
    const int g = lane >> 4;          // 16-lane group of the transposed reads
    const int kq = 8 * (g >> 1);      // the group's k rows: kq .. kq + 8 (= 8·h)
    const int mq = 16 * (g & 1);      // the group's 16 columns within a 32-column block
    auto step = [&](float4 (&vca)[2], float4 (&vcb)[2], float4 (&vna)[2], float4 (&vnb)[2]) -> bool {
#ifdef MPGNN_STAMPS
        stamp_at(ra.stamps, nsl, 0);
#endif
        const bool more = valid(c1);
        if (VAR != 2 && valid(c2)) {
            issue(c2, jj, vna, vnb);
            if (valid(c3)) load_idx(c3, jj);
        }
#ifdef MPGNN_STAMPS
        stamp_at(ra.stamps, nsl, 6);
#endif
        const bool is_root = cur.chunk < ra_n;
        const __bf16* cb = planes + buf * 6 * kOvPlane;
        if constexpr (!SQ) {
            const int ncol = wave * 32 + mq;
            const bf16x8 b0 = ov_frag(cb + 3 * kOvPlane, kq, ncol, lane);
            const bf16x8 b1 = ov_frag(cb + 4 * kOvPlane, kq, ncol, lane);
            const bf16x8 b2 = ov_frag(cb + 5 * kOvPlane, kq, ncol, lane);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bf16x8 a0 = ov_frag(cb, kq, q * 32 + mq, lane);
                const bf16x8 a1 = ov_frag(cb + kOvPlane, kq, q * 32 + mq, lane);
                const bf16x8 a2 = ov_frag(cb + 2 * kOvPlane, kq, q * 32 + mq, lane);
                lo[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, lo[q], 0, 0, 0);
                lo[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, lo[q], 0, 0, 0);
                lo[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, lo[q], 0, 0, 0);
                lo[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, lo[q], 0, 0, 0);
                lo[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, lo[q], 0, 0, 0);
                hi[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, hi[q], 0, 0, 0);
            }
        } else {
            // wave quarter (mh, nh): blocks q = 2·qm + qn at rows 64·mh + 32·qm, cols 64·nh + 32·qn
            const int mh = wave >> 1, nh = wave & 1;
            bf16x8 bq[2][3];
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int p = 0; p < 3; ++p) bq[j][p] = ov_frag(cb + (3 + p) * kOvPlane, kq, 64 * nh + 32 * j + mq, lane);
            commit(c1, vca, vcb, planes + (buf ^ 1) * 6 * kOvPlane);  // unconditional: zeros past the end
            __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);  // the B fragments first
#pragma unroll
            for (int qm = 0; qm < 2; ++qm) {
                bf16x8 a[3];
#pragma unroll
                for (int p = 0; p < 3; ++p) a[p] = ov_frag(cb + p * kOvPlane, kq, 64 * mh + 32 * qm + mq, lane);
#pragma unroll
                for (int qn = 0; qn < 2; ++qn) {
                    const int q = 2 * qm + qn;
                    const bf16x8* b = bq[qn];
                    lo[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], lo[q], 0, 0, 0);
                    lo[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], lo[q], 0, 0, 0);
                    lo[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], lo[q], 0, 0, 0);
                    lo[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], lo[q], 0, 0, 0);
                    lo[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], lo[q], 0, 0, 0);
                    hi[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], hi[q], 0, 0, 0);
                }
                // this half's A fragments, then its MFMAs with the commit's VALU and LDS writes
                __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
#pragma unroll
                for (int m = 0; m < 12; ++m) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
                    if (m < 6) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (is_root && ra.Pb != nullptr) {  // bias: column sums over the chunk's rows, exact from the pieces
            const int nr = min(SL, cur.p1 - cur.p0 - cur.sl * SL);
            const __bf16* bc = cb + (ra.bias_of_a ? 0 : 3 * kOvPlane) + srow * kOvLd + scol;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const bf16x4 q0 = *reinterpret_cast<const bf16x4*>(bc + 8 * j * kOvLd);
                const bf16x4 q1 = *reinterpret_cast<const bf16x4*>(bc + 8 * j * kOvLd + kOvPlane);
                const bf16x4 q2 = *reinterpret_cast<const bf16x4*>(bc + 8 * j * kOvLd + 2 * kOvPlane);
                if (srow + 8 * j < nr)
#pragma unroll
                    for (int e = 0; e < 4; ++e) bpart[e] += ((float)q0[e] + (float)q1[e]) + (float)q2[e];
            }
        }
        const bool chunk_end = cur.sl + 1 == cur.ns;
#ifdef MPGNN_STAMPS
        stamp_at(ra.stamps, nsl, 1);
#endif
        if (VAR == 2 && valid(c2)) {
            issue(c2, jj, vna, vnb);
            if (valid(c3)) load_idx(c3, jj);
        }
        if (!SQ && more) commit(c1, vca, vcb, planes + (buf ^ 1) * 6 * kOvPlane);
#ifdef MPGNN_STAMPS
        stamp_at(ra.stamps, nsl, 2);
#endif
        if (chunk_end) {
            float* D;
            float* Db = nullptr;
            if (is_root) {
                const int cidx = cur.chunk;
                D = ra.P + (size_t)cidx * p_stride + ra.d_off;
                Db = ra.Pb != nullptr ? ra.Pb + (size_t)cidx * pb_stride + ra.b_col0 : nullptr;
                if (ra.dst_mode == 3) {
                    D = ra.dst != nullptr ? ra.dst + ra.d_off : nullptr;
                    Db = ra.dst_b != nullptr ? ra.dst_b + ra.b_col0 : nullptr;
                }
            } else {
                const int cidx = cur.chunk - ra_n;
                D = wa.P + (size_t)cidx * p_stride + ra.d_off;
                if (wa.dst_mode == 1 || wa.dst_mode == 2) {
                    const int di = ld_uniform(wa.chunk_dst, cidx + wa.chunk_off);
                    if (di >= 0) D = wa.dst + (size_t)(wa.dst_mode == 1 ? di : 0) * p_stride + ra.d_off;
                }
            }
            const int ln = opaque(lane);
            const int h4 = 4 * (ln >> 5);
            if (D != nullptr) {
                if constexpr (!SQ) {
                    float* Dc = D + wave * 32 + (ln & 31);
#pragma unroll
                    for (int q = 0; q < 4; ++q)
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const int m = q * 32 + (r & 3) + 8 * (r >> 2) + h4;
                            Dc[(size_t)m * ldd] = hi[q][r] + lo[q][r];
                        }
                } else {
                    const int mh = wave >> 1, nh = wave & 1;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        float* Dc = D + 64 * nh + 32 * (q & 1) + (ln & 31);
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const int m = 64 * mh + 32 * (q >> 1) + (r & 3) + 8 * (r >> 2) + h4;
                            Dc[(size_t)m * ldd] = hi[q][r] + lo[q][r];
                        }
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    hi[q][r] = 0.0f;
                    lo[q][r] = 0.0f;
                }
            if (is_root && ra.Pb != nullptr) {  // the 8 row groups of each column, in order
                *reinterpret_cast<float4*>(bx + srow * 128 + scol) = make_float4(bpart[0], bpart[1], bpart[2], bpart[3]);
#pragma unroll
                for (int e = 0; e < 4; ++e) bpart[e] = 0.0f;
                __syncthreads();
                if (tid < 128 && Db != nullptr) {
                    float t = bx[tid];
#pragma unroll
                    for (int r = 1; r < 8; ++r) t += bx[r * 128 + tid];
                    Db[tid] = t;
                }
            }
        }
#ifdef MPGNN_STAMPS
        stamp_at(ra.stamps, nsl, 3);
        if (chunk_end) stamp_at(ra.stamps, nsl, 5);
#endif
        __syncthreads();
#ifdef MPGNN_STAMPS
        stamp_at(ra.stamps, nsl, 4);
        ++nsl;
        if (!more) stamp_end_at(ra.stamps);
#endif
        if (!more) return false;
        cur = c1;
        c1 = c2;
        c2 = c3;
        c3 = valid(c3) ? advance(c3) : c3;
        buf ^= 1;
        return true;
    };
    while (step(xa, xb, ya, yb) && step(ya, yb, xa, xb)) {
    }
}

// ----------------------------------------------------------------------------------------
// bwd_bf3_kernel — the GEMM work of a layer's backward at F_in = F_out = 128 in ONE persistent
// launch over rel_gemm's items (32-row relation tiles, then 32-node root items), both products
// that read dout on the bf16 matrix cores with the exact three-way split:
//   dgrad   G[seg] = (dout[node_1] @ W_rᵀ) / cnt,  G_root = dout @ rootᵀ      (waves 0-3)
//   dW      dW_r += Σ_rows A_rowᵀ dout_row, droot += x_iᵀ dout_i, dbias += Σ dout_i   (waves 4-7)
// The item's dout rows are gathered ONCE (waves 0-3) and committed both row-major (dgrad's A
// operand) and transposed (dW's B operand: K = the item's rows); waves 4-7 gather its A rows
// (x row or compact mean through s_src; x rows for root items) into transposed planes. dW
// accumulates in registers over a workgroup's run of items of one weight and leaves as one
// slab per run; the host knows every workgroup's item range, so the slabs of one weight are
// contiguous and reduce_slabs3_kernel sums them in order (deterministic). Replaces the dgrad
// launch, outer_bf3_kernel's second gather of dout + its 256-row chunk slabs.
// Waves 0-3 and 4-7 run separate loops (disjoint register sets) with the same two barriers
// per item; the rows of item i+1 are in flight during item i, their indices one item earlier.
// ----------------------------------------------------------------------------------------
constexpr int kBwThreads = 512;
constexpr int kBwLdt = 40;                     // transposed plane column: 32 rows + 8 pad (bf16, 80 B)
constexpr int kBwTPlane = 128 * kBwLdt;        // bf16 per transposed plane
constexpr int kBwLdab = 136;                   // row-major plane row: K + 8 (bf16)
constexpr int kBwRPlane = 32 * kBwLdab;        // bf16 per row-major plane
constexpr size_t kBwLds = (size_t)(3 * kBwRPlane + 6 * kBwTPlane) * 2 + (32 + 256) * sizeof(float);

struct BwdArgs {
    RelGemmArgs g;         // items + dgrad operands (DGRAD use: Aroot = dout, W / Wroot transposed);
                           // g.Y == nullptr: no grad_x wanted (no dgrad chain)
    const float* x;        // [N][128] layer input: A rows of dW
    const float* Hm;       // saved compact means (row m - g.m_lo)
    float* slabs;          // [n_slabs][128][128]
    float* bslabs;         // [n_slabs][128] bias partials (root runs)
    const int* wg_slab0;   // [G] first slab of each workgroup
};

__device__ __forceinline__ void bw_range(int n_items, int& i_beg, int& i_end) {
    const int G = (int)gridDim.x;
    const int g = (int)blockIdx.x & 7, q = G >> 3, rem = G & 7;
    const int rng = g * q + min(g, rem) + ((int)blockIdx.x >> 3);  // consecutive items on one XCD
    i_beg = (int)((long long)rng * n_items / G);
    i_end = (int)((long long)(rng + 1) * n_items / G);
}

// waves 0-3: dout rows of every item (both layouts) and, with g.Y, the dgrad products. Rows
// are gathered two items ahead (two register sets alternating roles), row indices three; the
// next item's weight slice is loaded after the chain (the registers are free then).
__device__ __forceinline__ void bw_dgrad_half(const BwdArgs& A, int i_beg, int i_end, __bf16* Rp, __bf16* Dt,
                                              float* Sc) {
    using Bs = RelGemm<2, true>;
    using Ds = RelGemmBf3<2, true>;
    using Item = Bs::Item;
    constexpr int N = 128, NS = 8, WPT = Bs::WPT, W4 = 32;
    const RelGemmArgs& a = A.g;
    const int t = threadIdx.x;  // 0..255
    const int lane = t & 63, c = lane & 31, h = lane >> 5;
    const int wq = __builtin_amdgcn_readfirstlane(t >> 6);
    const bool want_dx = a.Y != nullptr;
    const int col_b = (wq * 32 + c) * 4;
    Item cur = Bs::item(a, i_beg);
    float4 va[WPT], vb[WPT];
    int cnta = 1, cntb = 1, nrow[WPT], ncnt = 1, zm;
    {
        int r0[WPT];
        Bs::gather_idx(a, cur, t, r0, cnta);
        Bs::issue_rows(a, t, r0, va, zm);
    }
    if (i_beg + 1 < i_end) {
        int r1[WPT];
        Bs::gather_idx(a, Bs::item(a, i_beg + 1), t, r1, cntb);
        Bs::issue_rows(a, t, r1, vb, zm);
    }
    if (i_beg + 2 < i_end) Bs::gather_idx(a, Bs::item(a, i_beg + 2), t, nrow, ncnt);
    bf16x8 b[NS][3];
    if (want_dx) Ds::load_b(cur.w, wq, lane, b);
    // item i: vc / cntc hold its rows; after the commit they receive item i+2's
    auto step = [&](int i, float4 (&vc)[WPT], int& cntc) {
#pragma unroll
        for (int j = 0; j < WPT; ++j) {  // commit: split once, row-major (dgrad A) + transposed (dW B)
            const int e = t + j * 256;
            const int r = e / W4, c4 = (e % W4) * 4;
            const float4 xv = r < cur.nrows ? vc[j] : make_float4(0.f, 0.f, 0.f, 0.f);
            __bf16 p0[4], p1[4], p2[4];
            split3_bf16(xv.x, p0[0], p1[0], p2[0]);
            split3_bf16(xv.y, p0[1], p1[1], p2[1]);
            split3_bf16(xv.z, p0[2], p1[2], p2[2]);
            split3_bf16(xv.w, p0[3], p1[3], p2[3]);
            typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
            __bf16* d = Rp + r * kBwLdab + c4;
            *reinterpret_cast<bf16x4*>(d) = bf16x4{p0[0], p0[1], p0[2], p0[3]};
            *reinterpret_cast<bf16x4*>(d + kBwRPlane) = bf16x4{p1[0], p1[1], p1[2], p1[3]};
            *reinterpret_cast<bf16x4*>(d + 2 * kBwRPlane) = bf16x4{p2[0], p2[1], p2[2], p2[3]};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                __bf16* dt = Dt + (c4 + q) * kBwLdt + r;
                dt[0] = p0[q];
                dt[kBwTPlane] = p1[q];
                dt[2 * kBwTPlane] = p2[q];
            }
        }
        if (t < 32) Sc[t] = 1.0f / (float)cntc;
        if (i + 2 < i_end) {
            int zn;
            Bs::issue_rows(a, t, nrow, vc, zn);
            cntc = ncnt;
            if (i + 3 < i_end) Bs::gather_idx(a, Bs::item(a, i + 3), t, nrow, ncnt);
        }
        const bool has_next = i + 1 < i_end;
        const Item nxt = has_next ? Bs::item(a, i + 1) : cur;
        __syncthreads();  // (1) the item's planes are in LDS
        if (want_dx) {
            const __bf16* Ab = Rp + c * kBwLdab + 8 * h;
            f32x16 hi, lo;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                hi[r] = 0.0f;
                lo[r] = 0.0f;
            }
#pragma unroll
            for (int s2 = 0; s2 < NS; ++s2) {
                const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(Ab + 16 * s2);
                const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(Ab + kBwRPlane + 16 * s2);
                const bf16x8 a2 = *reinterpret_cast<const bf16x8*>(Ab + 2 * kBwRPlane + 16 * s2);
                lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b[s2][0], lo, 0, 0, 0);
                lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[s2][1], lo, 0, 0, 0);
                lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[s2][2], lo, 0, 0, 0);
                lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[s2][0], lo, 0, 0, 0);
                lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[s2][1], lo, 0, 0, 0);
                hi = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[s2][0], hi, 0, 0, 0);
            }
            float* Yt = cur.root ? a.Yroot + (size_t)(cur.r0 - a.row_lo) * N : a.Y + (size_t)(cur.r0 - a.sel_b) * N;
            const int bytes = __builtin_amdgcn_readfirstlane(cur.nrows) * N * 4;
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(Yt, (short)0, bytes, 0x00020000);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int rr = (r & 3) + 8 * (r >> 2) + 4 * h;
                float o = hi[r] + lo[r];
                if (!cur.root) o = o * Sc[rr];
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o), rs, rr * (N * 4) + col_b, 0, 16);
            }
            if (has_next && nxt.w != cur.w) Ds::load_b(nxt.w, wq, lane, b);  // after the chain
        }
        __syncthreads();  // (2) planes free for the next commit
        cur = nxt;
    };
    for (int i = i_beg; i < i_end; i += 2) {
        step(i, va, cnta);
        if (i + 1 < i_end) step(i + 1, vb, cntb);
    }
}

// waves 4-7: A rows of every item (transposed) and the dW / droot / dbias products; rows two
// items ahead like the other half
__device__ __forceinline__ void bw_dw_half(const BwdArgs& A, int i_beg, int i_end, const __bf16* Dt, __bf16* Xt,
                                           float* bx) {
    using Bs = RelGemm<2, true>;
    using Item = Bs::Item;
    const RelGemmArgs& a = A.g;
    const int t = threadIdx.x - 256;  // 0..255
    const int lane = t & 63, c = lane & 31, h = lane >> 5;
    const int wq = __builtin_amdgcn_readfirstlane(t >> 6);
    const int col = t & 127;
    const int hf = __builtin_amdgcn_readfirstlane(t >> 7);  // staged rows 8·hf + 16u .. +8 (u = 0, 1)
    // lanes 0..7 of the wave: A-row index of staged row 8·hf + 16u + lane (x row >= 0, else Hm row)
    auto load_idx = [&](const Item& it, int (&ia)[2]) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int k = min(8 * hf + 16 * u + (lane & 7), it.nrows - 1);
            ia[u] = it.root ? it.r0 + k : a.s_src[it.r0 + k];
        }
    };
    auto issue = [&](const int (&ia)[2], float (&xv)[2][8]) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int rw = __builtin_amdgcn_readlane(ia[u], j);
                const float* base = rw >= 0 ? A.x + (size_t)rw * 128 : A.Hm + (size_t)(-rw - 1 - a.m_lo) * 128;
                xv[u][j] = base[col];
            }
    };
    Item cur = Bs::item(a, i_beg);
    int nia[2] = {0, 0};
    float xa[2][8], xb[2][8];
    {
        int ia[2];
        load_idx(cur, ia);
        issue(ia, xa);
    }
    if (i_beg + 1 < i_end) {
        int ia[2];
        load_idx(Bs::item(a, i_beg + 1), ia);
        issue(ia, xb);
    }
    if (i_beg + 2 < i_end) load_idx(Bs::item(a, i_beg + 2), nia);
    f32x16 hi[4], lo[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            hi[q][r] = 0.0f;
            lo[q][r] = 0.0f;
        }
    float bpart = 0.0f;
    int slab = A.wg_slab0[blockIdx.x];
    int pending_b = -1;  // bias slab whose two halves wait in bx for the barrier
    auto step = [&](int i, float (&xv)[2][8]) {
        if (pending_b >= 0) {  // after barrier (2) of the previous item
            if (t < 128) A.bslabs[(size_t)pending_b * 128 + col] = bx[t] + bx[t + 128];
            pending_b = -1;
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int nr = min(8, cur.nrows - (8 * hf + 16 * u));  // live rows of this group (uniform)
            bf16x8 pa[3];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                __bf16 a0, a1, a2;
                split3_bf16(j < nr ? xv[u][j] : 0.0f, a0, a1, a2);
                pa[0][j] = a0;
                pa[1][j] = a1;
                pa[2][j] = a2;
            }
            __bf16* d = Xt + col * kBwLdt + 8 * hf + 16 * u;
#pragma unroll
            for (int p = 0; p < 3; ++p) *reinterpret_cast<bf16x8*>(d + p * kBwTPlane) = pa[p];
        }
        if (i + 2 < i_end) {
            issue(nia, xv);
            if (i + 3 < i_end) load_idx(Bs::item(a, i + 3), nia);
        }
        const bool has_next = i + 1 < i_end;
        const Item nxt = has_next ? Bs::item(a, i + 1) : cur;
        __syncthreads();  // (1)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            const __bf16* Bf = Dt + (wq * 32 + c) * kBwLdt + 16 * s2 + 8 * h;
            const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(Bf);
            const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(Bf + kBwTPlane);
            const bf16x8 b2 = *reinterpret_cast<const bf16x8*>(Bf + 2 * kBwTPlane);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const __bf16* Af = Xt + (q * 32 + c) * kBwLdt + 16 * s2 + 8 * h;
                const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(Af);
                const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(Af + kBwTPlane);
                const bf16x8 a2 = *reinterpret_cast<const bf16x8*>(Af + 2 * kBwTPlane);
                lo[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, lo[q], 0, 0, 0);
                lo[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, lo[q], 0, 0, 0);
                lo[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, lo[q], 0, 0, 0);
                lo[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, lo[q], 0, 0, 0);
                lo[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, lo[q], 0, 0, 0);
                hi[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, hi[q], 0, 0, 0);
            }
        }
        if (cur.root) {  // dbias: this thread's column of dout over its staged rows, rebuilt exactly
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const __bf16* bc = Dt + col * kBwLdt + 8 * hf + 16 * u;
                const bf16x8 q0 = *reinterpret_cast<const bf16x8*>(bc);
                const bf16x8 q1 = *reinterpret_cast<const bf16x8*>(bc + kBwTPlane);
                const bf16x8 q2 = *reinterpret_cast<const bf16x8*>(bc + 2 * kBwTPlane);
#pragma unroll
                for (int j = 0; j < 8; ++j) bpart += ((float)q0[j] + (float)q1[j]) + (float)q2[j];
            }
        }
        if (!has_next || nxt.w != cur.w) {  // the run ends: its slab
            float* D = A.slabs + (size_t)slab * 128 * 128;
            const int ocol = wq * 32 + c;
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = q * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    D[(size_t)m * 128 + ocol] = hi[q][r] + lo[q][r];
                    hi[q][r] = 0.0f;
                    lo[q][r] = 0.0f;
                }
            if (cur.root) {
                bx[t] = bpart;
                bpart = 0.0f;
                pending_b = slab;
            }
            ++slab;
        }
        __syncthreads();  // (2)
        cur = nxt;
    };
    for (int i = i_beg; i < i_end; i += 2) {
        step(i, xa);
        if (i + 1 < i_end) step(i + 1, xb);
    }
    if (pending_b >= 0 && t < 128) A.bslabs[(size_t)pending_b * 128 + col] = bx[t] + bx[t + 128];
}

__global__ __launch_bounds__(kBwThreads, 1) void bwd_bf3_kernel(BwdArgs A) {
    extern __shared__ __attribute__((aligned(16))) __bf16 bw_smem[];
    __bf16* Rp = bw_smem;
    __bf16* Dt = Rp + 3 * kBwRPlane;
    __bf16* Xt = Dt + 3 * kBwTPlane;
    float* Sc = reinterpret_cast<float*>(Xt + 3 * kBwTPlane);
    float* bx = Sc + 32;
    int i_beg, i_end;
    bw_range(A.g.n_rel + A.g.n_root, i_beg, i_end);
    if (i_beg >= i_end) return;
    if (threadIdx.x < 256) bw_dgrad_half(A, i_beg, i_end, Rp, Dt, Sc);
    else bw_dw_half(A, i_beg, i_end, Dt, Xt, bx);
}

// dst[group g] (elems floats) = Σ_{c in chunks of g, ascending} P[c]
struct ReduceArgs {
    const float* P;
    int elems;
    const int* gptr;     // nullable: single group [0, nchunks)
    int g_off;           // chunk index base subtracted from gptr values
    int nchunks;
    const int* gdst;     // nullable: destination index of each group (else blockIdx.x)
    int g_base;          // group index offset into gptr / gdst
    float* dst;
    int skip_single;     // groups of exactly one chunk were written directly: skip them
    int acc;             // dst = dst + Σ (mpgnn_rgcn_bwd_accumulate)
};

__device__ __forceinline__ void reduce_slabs_body(const ReduceArgs& a, const int g) {
    const int e = blockIdx.y * kThreads + threadIdx.x;
    if (e >= a.elems) return;
    int c0 = 0, c1 = a.nchunks;
    if (a.gptr != nullptr) {
        c0 = a.gptr[a.g_base + g] - a.g_off;
        c1 = a.gptr[a.g_base + g + 1] - a.g_off;
    }
    if (c1 - c0 == 1 && a.skip_single) return;  // written directly by outer_accum_kernel
    // slabs are read 32 at a time (independent loads in flight: a chained loop paid one L2
    // round trip per chunk); each block of 32 is summed as a pairwise tree (slabs past the end
    // enter as 0), the blocks in chunk order: fixed order (deterministic), rounding chain
    // 5 + blocks instead of one add per chunk
    constexpr int kB = 32;
    float s = 0.0f;
    const float* P = a.P + e;
    for (int cb = c0; cb < c1; cb += kB) {
        float v[kB];
#pragma unroll
        for (int u = 0; u < kB; ++u) v[u] = cb + u < c1 ? P[(size_t)(cb + u) * a.elems] : 0.0f;
#pragma unroll
        for (int w = kB / 2; w >= 1; w >>= 1)
#pragma unroll
            for (int u = 0; u < w; ++u) v[u] = v[u] + v[u + w];
        s += v[0];
    }
    const int d = a.gdst != nullptr ? a.gdst[a.g_base + g] : g;
    float* dp = a.dst + (size_t)d * a.elems + e;
    *dp = a.acc ? *dp + s : s;
}


// Up to three reductions (dW groups, droot, dbias) in one launch: blocks [0, n0) → r0,
// [n0, n0 + n1) → r1, the rest → r2; grid.y covers the widest.
// Weight indices without a segment (relations absent from the graph) get zeros from the
// same launch instead of a memset of the whole gradient.
constexpr int kMaxZeroIds = 32;
struct ZeroList {
    float* dst;
    int elems;
    int n;
    int ids[kMaxZeroIds];
};

__global__ __launch_bounds__(kThreads) void reduce_slabs3_kernel(ReduceArgs r0, ReduceArgs r1, ReduceArgs r2, int n0,
                                                                 int n1, int n2, ZeroList z) {
    const int b = (int)blockIdx.x;
    if (b < n0) reduce_slabs_body(r0, b);
    else if (b < n0 + n1) reduce_slabs_body(r1, b - n0);
    else if (b < n0 + n1 + n2) reduce_slabs_body(r2, b - n0 - n1);
    else {
        const int e = blockIdx.y * kThreads + threadIdx.x;
        if (e < z.elems) z.dst[(size_t)z.ids[b - n0 - n1 - n2] * z.elems + e] = 0.0f;
    }
}

// dst = act_out > 0 ? grad_out : 0 (ReLU backward, threshold_backward semantics: a NaN or inf
// gradient where the output was clamped gives 0, as torch's does); float4 when all three
// pointers are 16-byte aligned, the last n % 4 elements scalar.
__global__ __launch_bounds__(kThreads) void relu_bwd_kernel(const float* g, const float* y, int64_t n, float* d, int vec) {
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (vec) {
        const int64_t n4 = n / 4;
        for (int64_t k = i; k < n4; k += stride) {
            const float4 gv = reinterpret_cast<const float4*>(g)[k];
            const float4 yv = reinterpret_cast<const float4*>(y)[k];
            reinterpret_cast<float4*>(d)[k] = make_float4(relu_bwd_f(gv.x, yv.x), relu_bwd_f(gv.y, yv.y),
                                                          relu_bwd_f(gv.z, yv.z), relu_bwd_f(gv.w, yv.w));
        }
        i += n4 * 4;
        if (i >= n) return;
        // tail: at most 3 elements, thread i handles element n4 * 4 + (its global id)
    }
    for (int64_t k = i; k < n; k += stride) d[k] = relu_bwd_f(g[k], y[k]);
}

// Dropout's backward (torch's masked_scale: grad · mask · scale) and the ReLU backward of the
// layer whose output the dropout took (MPNetm: F.relu(conv) then Dropout(0.6), model.py:211-215)
// in one pass: dst = relu_bwd(g · (float)mask · scale, act) — masked_scale's arithmetic, then
// threshold_backward's rule.
__global__ __launch_bounds__(kThreads) void dropout_relu_bwd_kernel(const float* __restrict__ g,
                                                                    const unsigned char* __restrict__ mask,
                                                                    const float* __restrict__ act, float scale,
                                                                    int64_t n, float* __restrict__ d) {
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    for (int64_t k = (int64_t)blockIdx.x * kThreads + threadIdx.x; k < n; k += stride) {
        const float v = (g[k] * (float)mask[k]) * scale;
        d[k] = act != nullptr ? relu_bwd_f(v, act[k]) : v;
    }
}

// The wrappers' Linear heads with few outputs (model.py:147 Net.lin, :226 MPNetm.fc2):
// out[i][o] = act(Σ_f x[i][f]·W[o][f] + b[o]) for O <= 8, F <= 256 (F % 4 == 0). Four rows per
// wave, 16 lanes per row: lane s of a row holds columns 4s + 64k (k < F/64, rounded up). The
// products are exact in float64 and summed there (the lane's, then a fixed 16-lane butterfly,
// then + b), one rounding to fp32 at the end: the logits are the correctly rounded dot to within
// float64's error — closer to the exact value than any fp32 summation order (the library GEMM's
// included), so the heads' whole-model gradient checks keep their bars. Deterministic. W (<= 8
// KB) is re-read per row group from L1.
constexpr int kLinSmallO = 8;
__global__ __launch_bounds__(kThreads) void linear_small_fwd_kernel(const float* __restrict__ x, int N, int F,
                                                                    const float* __restrict__ W, int O,
                                                                    const float* __restrict__ bias, int act,
                                                                    float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int sub = lane & 15, q = lane >> 4;
    const int groups = (int)gridDim.x * (kThreads / 64);  // 4 rows each
    const double b = (bias != nullptr && sub < O) ? (double)bias[sub] : 0.0;
    for (int i0 = ((int)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6)) * 4; i0 < N; i0 += groups * 4) {
        const int i = i0 + q;
        float4 xv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int f = 4 * sub + 64 * k;
            xv[k] = (i < N && f < F) ? *reinterpret_cast<const float4*>(x + (size_t)i * F + f)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        double v = 0.0;
        for (int o = 0; o < O; ++o) {  // wave-uniform
            double t = 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int f = 4 * sub + 64 * k;
                if (f < F) {
                    const float4 wv = *reinterpret_cast<const float4*>(W + (size_t)o * F + f);
                    t += (double)xv[k].x * (double)wv.x;
                    t += (double)xv[k].y * (double)wv.y;
                    t += (double)xv[k].z * (double)wv.z;
                    t += (double)xv[k].w * (double)wv.w;
                }
            }
#pragma unroll
            for (int m = 8; m >= 1; m >>= 1) t += __shfl_xor(t, m);  // within the row's 16 lanes
            v = sub == o ? t : v;
        }
        float r = (float)(v + b);
        if (act == MPGNN_ACT_LOG_SOFTMAX) {  // over the row's O logits (its 16 lanes; wave-uniform branch)
            float mx = sub < O ? r : -INFINITY;
#pragma unroll
            for (int m = 8; m >= 1; m >>= 1) mx = fmaxf(mx, __shfl_xor(mx, m));
            float se = sub < O ? expf(r - mx) : 0.0f;
#pragma unroll
            for (int m = 8; m >= 1; m >>= 1) se += __shfl_xor(se, m);
            r = (r - mx) - logf(se);
        }
        if (i < N && sub < O) out[(size_t)i * O + sub] = act == MPGNN_ACT_RELU ? relu_f(r) : r;
    }
}

// Backward of a narrow head followed by log_softmax (Net.lin + F.log_softmax, model.py:147-148):
// per row i, dl = g_i - exp(logp_i) · Σ_o g_i[o] (log_softmax's backward), then in the same pass
// grad_x[i] = dl @ W (ReLU mask of the head's input fused when given) and this workgroup's
// partial of dW = dlᵀ x, db = Σ dl over its row slice (rows i ≡ grp mod G of the slice summed
// in order per thread, the G groups in order through LDS): P[part][o][0..F]. The ordered sum of
// the partials is linear_wgrad_sum_kernel's. One launch replaces log_softmax's backward, the
// dgrad and the partial weight gradient.
constexpr int kLsmO = 8;
// OM: compiled bound on O (2: Net's two classes; 8). Thread layout: 4 consecutive columns per
// thread (float4), F/4 threads per row, G = 256·4/F row groups per workgroup; rows i ≡ grp (mod G)
// of the slice per thread, RB of them in flight together.
template <int OM, int RB>
__global__ __launch_bounds__(kThreads) void linear_lsm_bwd_kernel(const float* __restrict__ g,
                                                                  const float* __restrict__ logp,
                                                                  const float* __restrict__ x,
                                                                  const float* __restrict__ mask, int N, int F, int O,
                                                                  const float* __restrict__ W, float* __restrict__ gx,
                                                                  int rows, float* __restrict__ P) {
    __shared__ float red[(4 * kThreads + kThreads) * OM];  // [G][O][F + 1]: G·(F + 1) <= 1024 + 256 per output
    const int tid = threadIdx.x;
    const int F4 = F / 4;
    const int G = kThreads / F4;
    const int f = (tid % F4) * 4, grp = tid / F4;
    const bool live = grp < G;
    float4 w[OM], acc[OM];
    float bacc[OM];
#pragma unroll
    for (int o = 0; o < OM; ++o) {
        w[o] = (live && o < O) ? *reinterpret_cast<const float4*>(W + (size_t)o * F + f) : make_float4(0.f, 0.f, 0.f, 0.f);
        acc[o] = make_float4(0.f, 0.f, 0.f, 0.f);
        bacc[o] = 0.0f;
    }
    const int r0 = (int)blockIdx.x * rows, r1 = min(N, r0 + rows);
    if (live) {
        for (int i0 = r0 + grp; i0 < r1; i0 += G * RB) {
            // the batch's operands first (one round trip per batch), rows past r1 clamped (unused)
            float gi[RB][OM], lp[RB][OM];
            float4 xv[RB], mv[RB];
#pragma unroll
            for (int u = 0; u < RB; ++u) {
                const int i = min(i0 + u * G, r1 - 1);
#pragma unroll
                for (int o = 0; o < OM; ++o) {
                    gi[u][o] = o < O ? g[(size_t)i * O + o] : 0.0f;
                    lp[u][o] = o < O ? logp[(size_t)i * O + o] : 0.0f;
                }
                xv[u] = *reinterpret_cast<const float4*>(x + (size_t)i * F + f);
                mv[u] = mask != nullptr ? *reinterpret_cast<const float4*>(mask + (size_t)i * F + f)
                                        : make_float4(1.f, 1.f, 1.f, 1.f);
            }
#pragma unroll
            for (int u = 0; u < RB; ++u) {
                const int i = i0 + u * G;
                if (i >= r1) break;
                float S = 0.0f, dl[OM];
#pragma unroll
                for (int o = 0; o < OM; ++o)
                    if (o < O) S += gi[u][o];
#pragma unroll
                for (int o = 0; o < OM; ++o) dl[o] = o < O ? gi[u][o] - expf(lp[u][o]) * S : 0.0f;
                if (gx != nullptr) {
                    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                    for (int o = 0; o < OM; ++o)
                        if (o < O) {
                            v.x = fmaf(dl[o], w[o].x, v.x);
                            v.y = fmaf(dl[o], w[o].y, v.y);
                            v.z = fmaf(dl[o], w[o].z, v.z);
                            v.w = fmaf(dl[o], w[o].w, v.w);
                        }
                    if (mask != nullptr)
                        v = make_float4(relu_bwd_f(v.x, mv[u].x), relu_bwd_f(v.y, mv[u].y), relu_bwd_f(v.z, mv[u].z),
                                        relu_bwd_f(v.w, mv[u].w));
                    *reinterpret_cast<float4*>(gx + (size_t)i * F + f) = v;
                }
#pragma unroll
                for (int o = 0; o < OM; ++o)
                    if (o < O) {
                        acc[o].x = fmaf(dl[o], xv[u].x, acc[o].x);
                        acc[o].y = fmaf(dl[o], xv[u].y, acc[o].y);
                        acc[o].z = fmaf(dl[o], xv[u].z, acc[o].z);
                        acc[o].w = fmaf(dl[o], xv[u].w, acc[o].w);
                        bacc[o] += dl[o];
                    }
            }
        }
    }
    const int E = O * (F + 1);
    if (live) {
#pragma unroll
        for (int o = 0; o < OM; ++o)
            if (o < O) {
                float* rp = red + grp * E + o * (F + 1) + f;
                rp[0] = acc[o].x;
                rp[1] = acc[o].y;
                rp[2] = acc[o].z;
                rp[3] = acc[o].w;
                if (f == 0) red[grp * E + o * (F + 1) + F] = bacc[o];
            }
    }
    __syncthreads();
    float* Pp = P + (size_t)blockIdx.x * E;
    for (int e = tid; e < E; e += kThreads) {
        float t = red[e];
        for (int q = 1; q < G; ++q) t += red[q * E + e];
        Pp[e] = t;
    }
}

// grad of a Linear head's input: gx[i][f] = Σ_o g[i][o]·W[o][f] for O <= 8 (g @ W), float4 columns
__global__ __launch_bounds__(kThreads) void linear_small_dgrad_kernel(const float* __restrict__ g, int N, int O,
                                                                      const float* __restrict__ W, int F,
                                                                      float* __restrict__ gx,
                                                                      const float* __restrict__ mask) {
    const int F4 = F / 4;
    const int64_t total = (int64_t)N * F4;
    for (int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x; e < total; e += (int64_t)gridDim.x * kThreads) {
        const int i = (int)(e / F4), f = (int)(e % F4) * 4;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int o = 0; o < O; ++o) {
            const float gv = g[(size_t)i * O + o];
            const float4 wv = *reinterpret_cast<const float4*>(W + (size_t)o * F + f);
            acc.x = fmaf(gv, wv.x, acc.x);
            acc.y = fmaf(gv, wv.y, acc.y);
            acc.z = fmaf(gv, wv.z, acc.z);
            acc.w = fmaf(gv, wv.w, acc.w);
        }
        if (mask != nullptr) {  // the ReLU backward of the layer that produced the head's input, fused
            const float4 m = *reinterpret_cast<const float4*>(mask + (size_t)i * F + f);
            acc = make_float4(relu_bwd_f(acc.x, m.x), relu_bwd_f(acc.y, m.y), relu_bwd_f(acc.z, m.z),
                              relu_bwd_f(acc.w, m.w));
        }
        *reinterpret_cast<float4*>(gx + (size_t)i * F + f) = acc;
    }
}

// y[i][f] = act(y[i][f] + b[f]) in place (the bias / ReLU of a Linear head computed by the GEMM)
__global__ __launch_bounds__(kThreads) void bias_act_kernel(float* __restrict__ y, int64_t n4, int F4,
                                                            const float* __restrict__ bias, int act) {
    for (int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x; e < n4; e += (int64_t)gridDim.x * kThreads) {
        float4 v = reinterpret_cast<float4*>(y)[e];
        if (bias != nullptr) {
            const float4 b = reinterpret_cast<const float4*>(bias)[e % F4];
            v = make_float4(v.x + b.x, v.y + b.y, v.z + b.z, v.w + b.w);
        }
        if (act == MPGNN_ACT_RELU) v = make_float4(relu_f(v.x), relu_f(v.y), relu_f(v.z), relu_f(v.w));
        reinterpret_cast<float4*>(y)[e] = v;
    }
}

// Linear-layer weight / bias gradient with K = N rows (the wrappers' heads: model.py:147,
// :224-226): gw[o][f] = Σ_i g[i][o]·x[i][f], gb[o] = Σ_i g[i][o]. Stage 1: workgroup p sums
// its row slice into partial P[p][o][0..F] (column F = the bias); thread t owns column
// f = t % F and outputs o ≡ t / F (mod 256 / F) — the g loads are wave-uniform. Stage 2 sums
// the partials in a fixed order (deterministic, no atomics). Heads with more outputs than one
// pass holds (O > 32·256/F, e.g. MPNetm.fc1 128 -> 128) run in output blocks [o_lo, o_lo + O).
constexpr int kLinAcc = 32;  // outputs per thread (O ≤ kLinAcc · 256 / F)
constexpr int kLinRows = 8;  // rows per load batch
constexpr int kLinRowsPerPart = 64;
__global__ __launch_bounds__(kThreads) void linear_wgrad_part_kernel(const float* __restrict__ x,
                                                                     const float* __restrict__ g, int ldg, int N, int F,
                                                                     int O, int rows, float* __restrict__ P) {
    const int tid = threadIdx.x;
    const int G = kThreads / F;
    const int f = tid % F, grp = tid / F;
    if (grp >= G) return;
    const int r0 = (int)blockIdx.x * rows, r1 = min(N, r0 + rows);
    float acc[kLinAcc], bacc[kLinAcc];
#pragma unroll
    for (int k = 0; k < kLinAcc; ++k) acc[k] = bacc[k] = 0.0f;
    // rows in batches of kLinRows: the batch's loads are issued together (one round trip per
    // batch, not per row), then added in row order
    for (int i0 = r0; i0 < r1; i0 += kLinRows) {
        float xv[kLinRows];
#pragma unroll
        for (int u = 0; u < kLinRows; ++u) xv[u] = x[(size_t)min(i0 + u, r1 - 1) * F + f];
#pragma unroll
        for (int k = 0; k < kLinAcc; ++k) {
            const int o = grp + k * G;
            if (o < O) {
                float gv[kLinRows];
#pragma unroll
                for (int u = 0; u < kLinRows; ++u) gv[u] = i0 + u < r1 ? g[(size_t)(i0 + u) * ldg + o] : 0.0f;
#pragma unroll
                for (int u = 0; u < kLinRows; ++u) {
                    acc[k] = __builtin_fmaf(gv[u], xv[u], acc[k]);
                    bacc[k] += gv[u];
                }
            }
        }
    }
    float* Pp = P + (size_t)blockIdx.x * O * (F + 1);
#pragma unroll
    for (int k = 0; k < kLinAcc; ++k) {
        const int o = grp + k * G;
        if (o < O) {
            Pp[(size_t)o * (F + 1) + f] = acc[k];
            if (f == 0) Pp[(size_t)o * (F + 1) + F] = bacc[k];
        }
    }
}

__global__ __launch_bounds__(kThreads) void linear_wgrad_sum_kernel(const float* __restrict__ P, int parts, int F, int O,
                                                                    float* __restrict__ gw, float* __restrict__ gb) {
    // one wave per element: lane l sums the partials p ≡ l (mod 64) in order, then the 64 lane
    // sums are combined by a fixed butterfly (deterministic: the same order every launch)
    const int e = (int)blockIdx.x * kWaves + (int)(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int elems = O * (F + 1);
    if (e >= elems) return;
    const int o = e / (F + 1), f = e % (F + 1);
    if (f == F && gb == nullptr) return;
    float s = 0.0f;
    for (int p = lane; p < parts; p += 64) s += P[(size_t)p * elems + e];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
    if (lane == 0) {
        if (f == F) gb[o] = s;
        else gw[(size_t)o * F + f] = s;
    }
}

// G[s] = dh[s] / cnt[sel_b + s] for the segment rows of a selection (segment-means backward)
__global__ __launch_bounds__(kThreads) void scale_rows_kernel(const float* dh, const int* cnt, int sel_b, int rows,
                                                              int F, float* G) {
    const size_t n = (size_t)rows * F;
    for (size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (size_t)gridDim.x * kThreads) {
        const int r = (int)(i / F);
        G[i] = dh[i] / (float)cnt[sel_b + r];
    }
}

// ----------------------------------------------------------------------------------------
// kernel timing: hipEvent pairs on the launch stream (mpgnn_timing_*)
// ----------------------------------------------------------------------------------------
struct TimingRecord {
    int kind;
    hipEvent_t start, stop;
};
static std::mutex g_timing_mu;
static bool g_timing_on = false;
static std::vector<TimingRecord> g_timing;
static std::vector<hipEvent_t> g_event_pool;  // events of reset records, reused (no create per launch)

static bool pooled_event(hipEvent_t* e) {  // g_timing_mu held
    if (!g_event_pool.empty()) {
        *e = g_event_pool.back();
        g_event_pool.pop_back();
        return true;
    }
    // timing-only events: no system-scope fence (no cache writeback / invalidate between the
    // kernels being timed)
    return hipEventCreateWithFlags(e, hipEventDisableSystemFence) == hipSuccess;
}
static int64_t g_timing_mask = ~int64_t(0);  // MPGNN_OPT_TIMING_MASK: kinds timed (bit = kind)

struct TimedLaunch {
    int kind;
    hipStream_t stream;
    hipEvent_t start = nullptr, stop = nullptr;
    bool on;
    TimedLaunch(int k, hipStream_t s) : kind(k), stream(s) {
        std::lock_guard<std::mutex> lk(g_timing_mu);
        on = g_timing_on && ((g_timing_mask >> k) & 1) && pooled_event(&start) && pooled_event(&stop);
        if (on) (void)hipEventRecord(start, stream);
    }
    ~TimedLaunch() {
        if (!on) return;
        (void)hipEventRecord(stop, stream);
        std::lock_guard<std::mutex> lk(g_timing_mu);
        g_timing.push_back({kind, start, stop});
    }
};

// ----------------------------------------------------------------------------------------
// host-side dispatch
// ----------------------------------------------------------------------------------------
static int32_t hip_check(hipError_t e, const char* what) {
    if (e == hipSuccess) return MPGNN_OK;
    set_last_error(std::string(what) + ": " + hipGetErrorString(e));
    return MPGNN_ERR_HIP;
}

static int32_t arg_error(const std::string& msg) {
    set_last_error(msg);
    return MPGNN_ERR_ARG;
}

// (V, T) variant for a gather of width F; returns false when F > kMaxF.
static bool pick_vt(int F, int* V, int* T) {
    if (F <= 64) { *V = 1; *T = 1; return true; }
    if (F <= 128 && F % 2 == 0) { *V = 2; *T = 1; return true; }
    if (F <= 256 && F % 4 == 0) { *V = 4; *T = 1; return true; }
    if (F <= 256 && F % 2 == 0) { *V = 2; *T = 2; return true; }
    if (F <= 256) { *V = 1; *T = 4; return true; }
    return false;
}

#define MPGNN_VT_DISPATCH(V, T, KERNEL, ...)                                          \
    do {                                                                              \
        if (V == 1 && T == 1) KERNEL<1, 1>(__VA_ARGS__);                              \
        else if (V == 2 && T == 1) KERNEL<2, 1>(__VA_ARGS__);                         \
        else if (V == 4 && T == 1) KERNEL<4, 1>(__VA_ARGS__);                         \
        else if (V == 2 && T == 2) KERNEL<2, 2>(__VA_ARGS__);                         \
        else KERNEL<1, 4>(__VA_ARGS__);                                               \
    } while (0)

template <int V, int T>
static void launch_seg(const SegTileArgs& a, int nblocks, int ncoltiles, hipStream_t st) {
    const int Kp = round_up(a.F, 64);
    const size_t lds = (size_t)(kTileRows + kTileRows * (Kp + 4)) * sizeof(float);
    hipLaunchKernelGGL((seg_tile_kernel<V, T>), dim3(nblocks, ncoltiles), dim3(kThreads), lds, st, a);
}

static int cu_count() {
    static int n = 0;
    if (n == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}

template <int KB>
static void launch_tile_gemm_kb(const TileGemmArgs& a, hipStream_t st) {
    constexpr int lda = 64 * KB + 4;
    constexpr int ldo = kColTile + 4;
    const size_t lds = (size_t)(2 * kTileRows * (lda > ldo ? lda : ldo) + 2 * kTileRows) * sizeof(float);
    const int per_cu = (2 * lds <= 160 * 1024) ? 2 : 1;
    const int n_items = (a.n_rel + a.n_root) * a.ncol;
    const int grid = std::min(n_items, cu_count() * per_cu);
    hipLaunchKernelGGL((tile_gemm_kernel<KB>), dim3(grid), dim3(kThreads), lds, st, a);
}



template <int KB, bool DGRAD, int NB>
static void launch_rel_gemm_wide(const RelGemmArgs& a, hipStream_t st) {
    constexpr int lda = 64 * KB + 4;
    const size_t lds = (size_t)(2 * 32 * lda + 64 + 4) * sizeof(float);
    const int n_items = a.n_rel + a.n_root;
    const int grid = std::min(n_items, std::max(1, cu_count() * 2 / NB));
    // K = 256 dgrad: the pipelined loop's extra registers would spill (128 for the B slice)
    if (!DGRAD && a.node_map != nullptr) {  // relation items, then root items with the root epilogue
        RelGemmArgs rel = a, rt = a;
        rel.n_root = 0;
        rel.node_map = nullptr;
        rt.n_rel = 0;
        if (rel.n_rel > 0)
            hipLaunchKernelGGL((rel_gemm_kernel<KB, false, NB, 2, false, true>),
                               dim3(std::min(rel.n_rel, std::max(1, cu_count() * 2 / NB)), NB), dim3(kThreads), lds, st, rel);
        if (rt.n_root > 0)
            hipLaunchKernelGGL((rel_gemm_kernel<KB, false, NB, 2, false, true, true>),
                               dim3(std::min(rt.n_root, std::max(1, cu_count() * 2 / NB)), NB), dim3(kThreads), lds, st, rt);
        return;
    }
    hipLaunchKernelGGL((rel_gemm_kernel<KB, DGRAD, NB, 2, false, !DGRAD>), dim3(grid, NB), dim3(kThreads), lds, st, a);
}

template <int KB, bool DGRAD>
static void launch_rel_gemm_t(const RelGemmArgs& a, hipStream_t st) {
    constexpr int lda = 64 * KB + 4;
    const size_t lds = (size_t)(2 * 32 * lda + 64 + 4 + (DGRAD ? 4 * 16 * 64 : 0)) * sizeof(float);
    const int n_items = a.n_rel + a.n_root;
    const int grid = std::min(n_items, cu_count() * 2);  // two workgroups per CU
    if (!DGRAD && a.node_map != nullptr) {  // relation items, then root items with the root epilogue
        RelGemmArgs rel = a, rt = a;
        rel.n_root = 0;
        rel.node_map = nullptr;
        rt.n_rel = 0;
        if (rel.n_rel > 0)
            hipLaunchKernelGGL((rel_gemm_kernel<KB, false>), dim3(std::min(rel.n_rel, cu_count() * 2)), dim3(kThreads), lds, st,
                               rel);
        if (rt.n_root > 0)
            hipLaunchKernelGGL((rel_gemm_kernel<KB, false, 1, 2, false, true, true>), dim3(std::min(rt.n_root, cu_count() * 2)),
                               dim3(kThreads), lds, st, rt);
        return;
    }
    hipLaunchKernelGGL((rel_gemm_kernel<KB, DGRAD>), dim3(grid), dim3(kThreads), lds, st, a);
}

// process defaults of the per-plan switches (mpgnn_set_option; plans copy them when created)
static std::mutex g_opt_mu;
static Options g_defaults;
Options default_options() {
    std::lock_guard<std::mutex> lk(g_opt_mu);
    return g_defaults;
}


template <int KB, bool DGRAD>
static void launch_rel_gemm_bf3(const RelGemmArgs& a, bool il, hipStream_t st) {
    const size_t lds = RelGemmBf3<KB, DGRAD>::lds_bytes();
    const int grid = std::min(a.n_rel + a.n_root, cu_count() * 2);  // two workgroups per CU
    if (il) hipLaunchKernelGGL((rel_gemm_bf3_kernel<KB, DGRAD, true>), dim3(grid), dim3(kThreads), lds, st, a);
    else hipLaunchKernelGGL((rel_gemm_bf3_kernel<KB, DGRAD>), dim3(grid), dim3(kThreads), lds, st, a);
}

// K = N = 256: one 512-thread workgroup per CU; column-block pairs on one XCD (grid a multiple of
// 16: 8 XCDs × pairs), item ranges split over the pairs
template <bool DGRAD>
static void launch_rel_gemm_bf3w(const RelGemmArgs& a, bool il, hipStream_t st) {
    const size_t lds = RelGemmBf3W<DGRAD>::lds_bytes();
    const int n_items = a.n_rel + a.n_root;
    int pairs = std::min(n_items, cu_count() / 2);
    pairs = std::max(8, (pairs + 7) / 8 * 8);
    if (il) hipLaunchKernelGGL((rel_gemm_bf3w_kernel<DGRAD, true>), dim3(2 * pairs), dim3(512), lds, st, a);
    else hipLaunchKernelGGL((rel_gemm_bf3w_kernel<DGRAD, false>), dim3(2 * pairs), dim3(512), lds, st, a);
}


// rel_gemm_bf3_kernel's item ranges balanced by cost = items + c · weight runs (each range pays
// one exposed weight-slice load per run it holds), followed by every item's weight index (the
// relation value of its tiles, -1 for root items) so that the kernel's item table needs no
// dependent s_rel load. Cached per plan; made outside captures (nullptr: the kernel's equal split
// and s_rel lookups). Uploaded on the caller's stream from a pinned buffer the plan keeps and
// published in the cache only after that stream has drained the copy (once per key).
// RelGemmArgs::first from the item ranges: one workgroup per range, thread t < 96 the row number
// of item k = t / 32 (clamped to the range), position q = t % 32 — gather_idx's values — thread
// 96 + t its dgrad count
__global__ __launch_bounds__(kThreads) void gemm_first_kernel(const int* __restrict__ ranges, int G, int n_rel,
                                                              int t_lo, const int* __restrict__ t_begin,
                                                              const int* __restrict__ t_end,
                                                              const int* __restrict__ map, const int* __restrict__ cnt,
                                                              int row_lo, int row_hi, int* __restrict__ rec) {
    const int rng = (int)blockIdx.x, t = threadIdx.x;
    const int i_beg = ranges[rng], i_end = ranges[rng + 1];
    int* r = rec + (size_t)rng * kFirstRec;
    if (i_beg >= i_end) {
        if (t == 0) r[0] = r[1] = i_beg;
        return;
    }
    auto tile = [&](int i, int& r0, int& nrows) {
        if (i < n_rel) {
            r0 = t_begin[t_lo + i];
            nrows = t_end[t_lo + i] - r0;
        } else {
            r0 = row_lo + (i - n_rel) * 32;
            nrows = min(32, row_hi - r0);
        }
    };
    if (t == 0) {
        int r0, nrows;
        tile(i_beg, r0, nrows);
        r[0] = i_beg;
        r[1] = i_end;
        r[2] = i_beg < n_rel ? ranges[G + 1 + i_beg] : -1;
        r[3] = r0;
        r[4] = nrows;
        r[5] = r[6] = r[7] = 0;
    }
    if (t < 192) {
        const int k = (t % 96) / 32, q = t % 32;
        const int i = min(i_beg + k, i_end - 1);
        int r0, nrows;
        tile(i, r0, nrows);
        const int row = r0 + min(q, nrows - 1);
        if (t < 96) r[8 + t] = i < n_rel ? map[row] : row;
        else r[8 + t] = (i < n_rel && cnt != nullptr) ? cnt[row] : 1;
    }
}

static const int* gemm_ranges(const mpgnn_plan* p, int t_lo, int n_rel, int n_root, int G, bool pairs,
                              hipStream_t st);

// Cached per plan, ranges table and direction (made outside captures; nullptr: the kernel's hops)
static const int* gemm_first(const mpgnn_plan* p, const int* ranges, int G, const RelGemmArgs& r, bool dgrad,
                             hipStream_t st) {
    if (ranges == nullptr || G <= 0) return nullptr;
    const std::array<int64_t, 5> key{(int64_t)(intptr_t)ranges, G, dgrad ? 1 : 0, r.row_lo, r.row_hi};
    std::lock_guard<std::mutex> lk(p->bw_mu);
    auto it = p->gemm_first.find(key);
    if (it != p->gemm_first.end()) return it->second.dev;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    mpgnn_plan::GemmRanges e;
    if (hipMalloc(reinterpret_cast<void**>(&e.dev), (size_t)G * kFirstRec * sizeof(int)) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    hipLaunchKernelGGL(gemm_first_kernel, dim3(G), dim3(kThreads), 0, st, ranges, G, r.n_rel, r.t_lo, r.t_begin,
                       r.t_end, dgrad ? r.s_row : r.s_src, dgrad ? r.s_cnt : nullptr, r.row_lo, r.row_hi, e.dev);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {  // published once complete
        (void)hipGetLastError();
        (void)hipFree(e.dev);
        return nullptr;
    }
    p->gemm_first[key] = e;
    return e.dev;
}

static const int* gemm_ranges(const mpgnn_plan* p, int t_lo, int n_rel, int n_root, int G, bool pairs,
                              hipStream_t st) {
    const int cost = p->opt.gemm_switch_cost;
    if (cost <= 0 || G <= 1) return nullptr;
    const std::array<int64_t, 5> key{t_lo, n_rel, n_root, G * 2 + (pairs ? 1 : 0), cost};
    std::lock_guard<std::mutex> lk(p->bw_mu);
    auto it = p->gemm_ranges.find(key);
    if (it != p->gemm_ranges.end()) return it->second.dev;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    const int n = n_rel + n_root;
    const double c = cost / 100.0;
    std::vector<double> cum(n + 1, 0.0);
    std::vector<int> wrel(n, -1);
    int prev_w = -2;
    for (int i = 0; i < n; ++i) {
        int w = -1;  // root items
        if (i < n_rel) {
            const int d = (int)(std::upper_bound(p->rel_t32_ptr.begin(), p->rel_t32_ptr.end(), t_lo + i) -
                                p->rel_t32_ptr.begin()) - 1;
            w = d;
            wrel[i] = (d >= 0 && d < (int)p->rel_val32.size()) ? p->rel_val32[d] : 0;
        }
        cum[i + 1] = cum[i] + 1.0 + (w != prev_w ? c : 0.0);
        prev_w = w;
    }
    const size_t words = (size_t)G + 1 + (size_t)n;
    mpgnn_plan::GemmRanges e;
    if (hipHostMalloc(reinterpret_cast<void**>(&e.host), words * sizeof(int), hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    int* tab = e.host;
    // boundaries of `parts` ranges of [lo, hi) with equal cost (first item whose cost prefix
    // reaches the target)
    auto split = [&](int lo, int hi, int parts, int* out) {
        int i = lo;
        for (int k = 1; k < parts; ++k) {
            const double target = cum[lo] + (cum[hi] - cum[lo]) * k / parts;
            while (i < hi && cum[i] < target) ++i;
            out[k] = std::max(out[k - 1], std::min(i, hi));
        }
    };
    tab[0] = 0;
    tab[G] = n;
    if (pairs) {  // CU ranges first, then each CU range in two halves (its two workgroups)
        std::vector<int> cu(G / 2 + 1, n);
        cu[0] = 0;
        split(0, n, G / 2, cu.data());
        for (int c = 0; c < G / 2; ++c) {
            tab[2 * c] = cu[c];
            int two[2] = {cu[c], cu[c]};
            split(cu[c], cu[c + 1], 2, two);
            tab[2 * c + 1] = two[1];
        }
    } else {
        split(0, n, G, tab);
    }
    std::copy(wrel.begin(), wrel.end(), tab + G + 1);
    if (hipMalloc(reinterpret_cast<void**>(&e.dev), words * sizeof(int)) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipHostFree(e.host);
        return nullptr;
    }
    // published only once complete: a later launch on another stream that hits the cache must not
    // read the table before the copy lands (once per plan and key, outside captures)
    if (hipMemcpyAsync(e.dev, e.host, words * sizeof(int), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipFree(e.dev);
        (void)hipHostFree(e.host);
        return nullptr;
    }
    p->gemm_ranges[key] = e;
    return e.dev;
}

// rel_gemm_w1_kernel's item table: the selection's 32-row tiles paired into 64-row items (two
// consecutive tiles of one relation; a relation's odd last tile alone), then the node rows
// [row_lo, row_hi) in 64-row root items; G contiguous ranges balanced by cost = sub-tiles + c per
// weight switch. Layout: [G + 1] first item per range, then {r0, nrows, weight index | -1} per
// item. Cached per plan like gemm_ranges (made outside captures; nullptr: no table).
static const int* gemm_w1_items(const mpgnn_plan* p, int t_lo, int n_rel, int row_lo, int row_hi, bool root, int G,
                                hipStream_t st) {
    if (G <= 0) return nullptr;
    const int cost = std::max(p->opt.gemm_switch_cost, 0);
    const std::array<int64_t, 5> key{t_lo, n_rel, (int64_t)row_lo * 2 + (root ? 1 : 0), -(int64_t)G - 1, (int64_t)row_hi * 1024 + cost};
    std::lock_guard<std::mutex> lk(p->bw_mu);
    auto it = p->gemm_ranges.find(key);
    if (it != p->gemm_ranges.end()) return it->second.dev;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    if ((int64_t)p->t32_begin.size() < (int64_t)t_lo + n_rel) return nullptr;
    std::vector<int> items;  // r0, nrows, w triplets
    int d = (int)(std::upper_bound(p->rel_t32_ptr.begin(), p->rel_t32_ptr.end(), t_lo) - p->rel_t32_ptr.begin()) - 1;
    for (int t = t_lo; t < t_lo + n_rel;) {
        while (d + 1 < (int)p->rel_t32_ptr.size() && p->rel_t32_ptr[d + 1] <= t) ++d;
        const int w = (d >= 0 && d < (int)p->rel_val32.size()) ? p->rel_val32[d] : 0;
        const bool pair = t + 1 < t_lo + n_rel && d + 1 < (int)p->rel_t32_ptr.size() && t + 1 < p->rel_t32_ptr[d + 1];
        const int r0 = p->t32_begin[t];
        const int r1 = pair ? p->t32_end[t + 1] : p->t32_end[t];
        items.push_back(r0);
        items.push_back(r1 - r0);
        items.push_back(w);
        t += pair ? 2 : 1;
    }
    if (root)
        for (int r0 = row_lo; r0 < row_hi; r0 += 64) {
            items.push_back(r0);
            items.push_back(std::min(64, row_hi - r0));
            items.push_back(-1);
        }
    const int n = (int)items.size() / 3;
    std::vector<double> cum(n + 1, 0.0);
    for (int i = 0; i < n; ++i) {
        const bool sw = i == 0 || items[3 * i + 2] != items[3 * i - 1];
        cum[i + 1] = cum[i] + (items[3 * i + 1] > 32 ? 2.0 : 1.0) + (sw ? cost / 100.0 : 0.0);
    }
    const size_t words = (size_t)G + 1 + (size_t)n * 3;
    mpgnn_plan::GemmRanges e;
    if (hipHostMalloc(reinterpret_cast<void**>(&e.host), words * sizeof(int), hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    int* tab = e.host;
    tab[0] = 0;
    int i = 0;
    for (int k = 1; k < G; ++k) {
        const double target = cum[n] * k / G;
        while (i < n && cum[i] < target) ++i;
        tab[k] = std::max(tab[k - 1], i);
    }
    tab[G] = n;
    std::copy(items.begin(), items.end(), tab + G + 1);
    if (hipMalloc(reinterpret_cast<void**>(&e.dev), words * sizeof(int)) != hipSuccess ||
        hipMemcpyAsync(e.dev, e.host, words * sizeof(int), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {  // published only once complete
        (void)hipGetLastError();
        if (e.dev) (void)hipFree(e.dev);
        (void)hipHostFree(e.host);
        return nullptr;
    }
    p->gemm_ranges[key] = e;
    return e.dev;
}

// outer_bf3v_kernel_t's chunk lists per workgroup. The chunks are dealt in windows of G
// consecutive chunks (as round robin: every workgroup works in the same window at a time, so the
// rows gathered concurrently stay a narrow slice of the relation-major order — contiguous ranges
// per workgroup measured 10 µs slower at C3: 67.5 -> 77.5), but inside a window the chunks go,
// largest first, to the workgroups with the least cost so far (cost = 16-row slices + 1 for the
// chunk-end slab store). Chunks [0, n_root): root chunks (rows row_lo.. in chunk_rows pieces),
// then the plan's weight chunks [c_lo, c_lo + nch). Table: [G + 1] list offsets, then the lists.
// Cached per plan, made outside captures (nullptr: the kernel's round robin).
static const int* outer_ranges(const mpgnn_plan* p, int c_lo, int nch, int row_lo, int row_hi, int chunk_rows,
                               int n_root, int G, hipStream_t st) {
    if (G <= 1) return nullptr;
    const std::array<int64_t, 5> key{c_lo, nch, (int64_t)row_lo * 4096 + chunk_rows, row_hi, G};
    std::lock_guard<std::mutex> lk(p->bw_mu);
    auto it = p->outer_ranges.find(key);
    if (it != p->outer_ranges.end()) return it->second.dev;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    if ((int64_t)p->chunk_begin.size() < (int64_t)c_lo + nch || (int64_t)p->chunk_end.size() < (int64_t)c_lo + nch)
        return nullptr;
    const int n = n_root + nch;
    std::vector<int> cost(n);
    for (int k = 0; k < n; ++k) {
        int rows;
        if (k < n_root) rows = std::min(chunk_rows, row_hi - (row_lo + k * chunk_rows));
        else rows = p->chunk_end[c_lo + k - n_root] - p->chunk_begin[c_lo + k - n_root];
        cost[k] = (std::max(rows, 0) + 15) / 16 + 1;
    }
    std::vector<std::vector<int>> lists(G);
    std::vector<int64_t> load(G, 0);
    std::vector<int> order, wgs(G);
    for (int w0 = 0; w0 < n; w0 += G) {
        const int w1 = std::min(n, w0 + G);
        order.resize(w1 - w0);
        for (int k = w0; k < w1; ++k) order[k - w0] = k;
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return cost[a] > cost[b]; });
        for (int g = 0; g < G; ++g) wgs[g] = g;
        std::stable_sort(wgs.begin(), wgs.end(), [&](int a, int b) { return load[a] < load[b]; });
        for (size_t j = 0; j < order.size(); ++j) {
            const int g = wgs[j];
            lists[g].push_back(order[j]);
            load[g] += cost[order[j]];
        }
    }
    for (auto& l : lists) std::sort(l.begin(), l.end());  // each workgroup walks its chunks in order
    const size_t words = (size_t)G + 1 + (size_t)n;
    mpgnn_plan::GemmRanges e;
    if (hipHostMalloc(reinterpret_cast<void**>(&e.host), words * sizeof(int), hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    int* tab = e.host;
    int pos = 0;
    for (int g = 0; g < G; ++g) {
        tab[g] = pos;
        for (int k : lists[g]) tab[G + 1 + pos++] = k;
    }
    tab[G] = pos;
    if (hipMalloc(reinterpret_cast<void**>(&e.dev), words * sizeof(int)) != hipSuccess ||
        hipMemcpyAsync(e.dev, e.host, words * sizeof(int), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {  // published only once complete (as gemm_ranges)
        (void)hipGetLastError();
        if (e.dev) (void)hipFree(e.dev);
        (void)hipHostFree(e.host);
        return nullptr;
    }
    p->outer_ranges[key] = e;
    return e.dev;
}

static void launch_rel_gemm(const RelGemmArgs& a, int K, bool dgrad, const Options& o, hipStream_t st) {
    if (o.gemm_bf3 && (K == 64 || K == 128) && a.node_map == nullptr) {
        if (K == 64) {
            if (dgrad) launch_rel_gemm_bf3<1, true>(a, o.gemm_il, st);
            else launch_rel_gemm_bf3<1, false>(a, o.gemm_il, st);
        } else {
            if (dgrad) launch_rel_gemm_bf3<2, true>(a, o.gemm_il, st);
            else launch_rel_gemm_bf3<2, false>(a, o.gemm_il, st);
        }
        return;
    }
    // C5: split-K bf16 kernel, two column blocks; forward with node_map: the mode-SINGLE root
    // epilogue in the same launch (relation items write Y, root items finish the rows without a
    // segment, single_fix_kernel the others)
    if (o.gemm_bf3 && K == 256 && (a.node_map == nullptr || !dgrad)) {
        if (dgrad) launch_rel_gemm_bf3w<true>(a, o.gemm_w_il, st);
        else launch_rel_gemm_bf3w<false>(a, o.gemm_w_il, st);
        return;
    }
    if (K == 256) {  // F_in = F_out = 256 (C5): two 128-column blocks, K = 256
        if (dgrad) launch_rel_gemm_wide<4, true, 2>(a, st);
        else launch_rel_gemm_wide<4, false, 2>(a, st);
        return;
    }
    if (K == 64) {
        if (dgrad) launch_rel_gemm_t<1, true>(a, st);
        else launch_rel_gemm_t<1, false>(a, st);
    } else {
        if (dgrad) launch_rel_gemm_t<2, true>(a, st);
        else launch_rel_gemm_t<2, false>(a, st);
    }
}

static void launch_tile_gemm(const TileGemmArgs& a, hipStream_t st) {
    const int kb = (round_up(a.K, 64)) / 64;
    if (kb <= 1) launch_tile_gemm_kb<1>(a, st);
    else if (kb == 2) launch_tile_gemm_kb<2>(a, st);
    else if (kb == 3) launch_tile_gemm_kb<3>(a, st);
    else launch_tile_gemm_kb<4>(a, st);
}

template <int V, int T>
static void launch_rowsum(const RowSumArgs& a, hipStream_t st) {
    const int rows_per_block = kWaves * kSumRowsPerWave;
    const int rows = a.N - a.r_begin;
    const dim3 grid((rows + rows_per_block - 1) / rows_per_block);
    if (a.extra != nullptr || a.bias != nullptr)
        hipLaunchKernelGGL((row_sum_kernel<V, T, true>), grid, dim3(kThreads), 0, st, a);
    else
        hipLaunchKernelGGL((row_sum_kernel<V, T, false>), grid, dim3(kThreads), 0, st, a);
}

template <int V, int T>
static void launch_piece(const PieceArgs& a, hipStream_t st) {
    const int n = a.k_hi - a.k_lo;
    hipLaunchKernelGGL((piece_sum_kernel<V, T>), dim3((n + kWaves - 1) / kWaves), dim3(kThreads), 0, st, a);
}


struct Selection {
    int64_t d_lo = 0, d_hi = 0;
    int sel_b = 0, sel_e = 0;
    int t_lo = 0, t_hi = 0;
    int t32_lo = 0, t32_hi = 0;   // 32-row tiles (rel_gemm_kernel)
    int c_lo = 0, c_hi = 0;
    int sp_lo = 0, sp_hi = 0;     // seg-list pieces of the selection
    int tap_lo = 0, tap_hi = 0;   // ta-list pieces (mode SINGLE)
    int ta_e_lo = 0, ta_e_hi = 0; // ta entry range (mode SINGLE)
    int m_lo = 0, m_hi = 0;       // multi-edge segments (rows of the compact means Hm)
    bool all_segments = false;    // selection covers every local segment
};

static void fill_selection(const mpgnn_plan* p, Selection* s);

static int32_t make_selection(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R, Selection* s) {
    int32_t st = select_relations(p, mode, relation, R, &s->d_lo, &s->d_hi);
    if (st != MPGNN_OK) return st;
    if (p->nrel == 0) return MPGNN_OK;
    fill_selection(p, s);
    return MPGNN_OK;
}

// Sub-selection of the dense relation range [d_lo, d_hi) (overlapped forward groups).
static Selection range_selection(const mpgnn_plan* p, int64_t d_lo, int64_t d_hi) {
    Selection s;
    s.d_lo = d_lo;
    s.d_hi = d_hi;
    if (p->nrel > 0) fill_selection(p, &s);
    return s;
}

static void fill_selection(const mpgnn_plan* p, Selection* s) {
    s->sel_b = p->rel_seg_ptr[s->d_lo];
    s->sel_e = p->rel_seg_ptr[s->d_hi];
    s->t_lo = p->rel_tile_ptr[s->d_lo];
    s->t_hi = p->rel_tile_ptr[s->d_hi];
    s->t32_lo = p->rel_t32_ptr[s->d_lo];
    s->t32_hi = p->rel_t32_ptr[s->d_hi];
    s->c_lo = p->rel_chunk_ptr[s->d_lo];
    s->c_hi = p->rel_chunk_ptr[s->d_hi];
    s->sp_lo = p->rel_seg_piece_ptr[s->d_lo];
    s->sp_hi = p->rel_seg_piece_ptr[s->d_hi];
    s->tap_lo = p->rel_ta_piece_ptr[s->d_lo];
    s->tap_hi = p->rel_ta_piece_ptr[s->d_hi];
    s->ta_e_lo = p->rel_ta_ent_ptr[s->d_lo];
    s->ta_e_hi = p->rel_ta_ent_ptr[s->d_hi];
    s->m_lo = p->rel_m_ptr[s->d_lo];
    s->m_hi = p->rel_m_ptr[s->d_hi];
    s->all_segments = (s->sel_b == 0 && s->sel_e == p->S);
}

static size_t align256(size_t b) { return (b + 255) / 256 * 256; }
static size_t align16(size_t b) { return (b + 15) / 16 * 16; }
// the grad_x list's split-row counters, whole 16-byte words (run_grad_x zeroes them per call)
static size_t split_counter_bytes(const mpgnn_plan* p) { return align16((size_t)p->tx_f.nsplit * sizeof(unsigned)); }

struct RootChunks {
    int rows_lo = 0, rows_hi = 0, chunk = 256, n = 0;
};

static RootChunks root_chunks(int64_t lo, int64_t hi) {
    RootChunks r;
    r.rows_lo = (int)lo;
    r.rows_hi = (int)hi;
    const int rows = (int)(hi - lo);
    int ch = std::max(g_chunk_rows, round_up((rows + 1023) / 1024, kSlice));
    r.chunk = ch;
    r.n = rows > 0 ? (rows + ch - 1) / ch : 0;
    return r;
}

// Workspace: forward and backward regions are used by different calls, so they overlap.
struct WsLayout {
    size_t y = 0, yroot = 0, hf = 0, pseg = 0, prw = 0, nmap = 0;  // forward
    size_t g = 0, groot = 0, h = 0, pdx = 0, p = 0, proot = 0, pb = 0;  // backward
    size_t bw = 0, bwb = 0;  // bwd_bf3_kernel slabs (F_in = F_out = 128)
    size_t total = 0;      // max(forward, backward): what mpgnn_rgcn_bwd needs
    size_t fwd_total = 0;  // forward part only (mpgnn_rgcn_fwd / _fwd_act)
};

static WsLayout ws_layout(const mpgnn_plan* p, int32_t mode, const Selection& s, int F_in, int F_out,
                          int64_t row_lo, int64_t row_hi, const RootChunks& rc) {
    WsLayout w;
    const size_t S_sel = (size_t)(s.sel_e - s.sel_b);
    const size_t rows = (size_t)(row_hi - row_lo);
    const size_t fmax = (size_t)std::max(F_in, F_out);
    size_t off = 0;
    w.y = off; off += align256(S_sel * F_out * sizeof(float));
    w.yroot = off; off += align256(rows * F_out * sizeof(float));
    const size_t Sm_sel = (size_t)(s.m_hi - s.m_lo);
    w.hf = off; off += align256(Sm_sel * F_in * sizeof(float));  // compact multi-edge means
    // piece partials (exact-order / mode SINGLE lists) or flat-list carry slots
    const size_t seg_slots = std::max({(size_t)(s.sp_hi - s.sp_lo), (size_t)p->seg_f.nslots, (size_t)p->segm_f.nslots});
    w.pseg = off; off += align256(seg_slots * fmax * sizeof(float));
    w.prw = off; off += align256((mode == MPGNN_MODE_ALL ? std::max({(size_t)p->rw_l.npieces, (size_t)p->rw_f.nslots,
                                                                     (size_t)p->rwx_f.nslots})
                                                         : 0) * F_out * sizeof(float));
    w.nmap = off; off += align256((mode == MPGNN_MODE_SINGLE ? (size_t)p->N : 0) * sizeof(int32_t));
    const size_t fwd = off;
    w.fwd_total = std::max<size_t>(fwd, 256);
    off = 0;
    const size_t dx_pieces = (mode == MPGNN_MODE_ALL)
                                 ? std::max({(size_t)p->t_l.npieces, (size_t)p->t_f.nslots, (size_t)p->tx_f.nslots})
                                 : (size_t)(s.tap_hi - s.tap_lo);
    w.g = off; off += align256(S_sel * F_in * sizeof(float));
    w.groot = off; off += align256(rows * F_in * sizeof(float));
    w.h = off; off += align256(Sm_sel * F_in * sizeof(float));
    // + the grad_x list's split-row counters behind its carry slots (run_grad_x)
    w.pdx = off;
    off += align256(align16(std::max(dx_pieces, seg_slots) * F_in * sizeof(float)) +
                    (mode == MPGNN_MODE_ALL ? split_counter_bytes(p) : 0));
    w.p = off; off += align256((size_t)(s.c_hi - s.c_lo) * F_in * F_out * sizeof(float));
    w.proot = off; off += align256((size_t)rc.n * F_in * F_out * sizeof(float));
    w.pb = off; off += align256((size_t)rc.n * F_out * sizeof(float));
    if (F_in == 128 && F_out == 128) {  // bwd_bf3_kernel: one slab per (workgroup, weight run)
        const size_t ns = (size_t)cu_count() + (size_t)std::max<int64_t>(s.d_hi - s.d_lo, 0) + 2;
        w.bw = off; off += align256(ns * F_in * F_out * sizeof(float));
        w.bwb = off; off += align256(ns * F_out * sizeof(float));
    }
    w.total = std::max<size_t>(std::max(fwd, off), 256);
    return w;
}

static int32_t check_common(const mpgnn_plan* p, int F_in, int F_out) {
    if (!p) return arg_error("NULL plan");
    if (!p->d.block && !p->device_built) {
        set_last_error("plan is not on a device: call mpgnn_plan_upload first");
        return MPGNN_ERR_NOT_ON_DEVICE;
    }
    if (F_in < 1 || F_out < 1) return arg_error("feature widths must be >= 1");
    if (F_in > kMaxF || F_out > kMaxF) {
        set_last_error("feature width > 256 is not compiled in");
        return MPGNN_ERR_UNSUPPORTED;
    }
    return MPGNN_OK;
}

static void clamp_rows(const mpgnn_plan* p, int64_t* lo, int64_t* hi) {
    *lo = std::max<int64_t>(0, std::min<int64_t>(*lo, p->N));
    *hi = std::max<int64_t>(*lo, std::min<int64_t>(*hi, p->N));
}

// One seg_tile_kernel launch: relation tiles of the selection (+ root tiles when Wroot).
//   forward (gather_kind 0): Y[s - sel_b] = mean(src over s) @ W_rel(s), H = the means,
//                            Yroot[i - row_lo] = src[i] @ Wroot
//   dgrad   (gather_kind 1): Y[s - sel_b] = (src[node_1(s)] @ W_relᵀ) / cnt, Yroot = src @ Wrootᵀ
static int32_t run_seg(const mpgnn_plan* p, int32_t mode, const Selection& s, int gather_kind, const float* src,
                       int K, const float* W, const float* Wroot, int trans, int N, float* Y, float* Yroot,
                       int64_t row_lo, int64_t row_hi, float* H, float* Pseg, bool exact, int kind,
                       hipStream_t strm, const float* Hsrc = nullptr, const int* root_map = nullptr,
                       const float* root_bias = nullptr, int root_relu = 0, unsigned* zero = nullptr,
                       int zero_words = 0, bool* zeroed = nullptr) {
    if (zeroed != nullptr) *zeroed = false;
    const int m_lo = s.m_lo;
    const int n_rel = s.t_hi - s.t_lo;
    const int n_root = (Wroot != nullptr) ? (int)((row_hi - row_lo + kTileRows - 1) / kTileRows) : 0;
    if (n_rel + n_root == 0) return MPGNN_OK;
    int V, T;
    pick_vt(K, &V, &T);
    const bool ragged = gather_kind == 0 && !exact && s.sp_hi > s.sp_lo;
    if (ragged) {
        PieceArgs pa{};
        pa.pb = p->d.seg_pb;
        pa.pe = p->d.seg_pe;
        pa.k_lo = s.sp_lo;
        pa.k_hi = s.sp_hi;
        pa.src = src;
        pa.F = K;
        pa.idx = p->d.e_col;
        pa.P = Pseg;
        TimedLaunch tl(MPGNN_K_PIECE, strm);
        MPGNN_VT_DISPATCH(V, T, launch_piece, pa, strm);
        int32_t st = hip_check(hipGetLastError(), "piece_sum_kernel(seg) launch");
        if (st != MPGNN_OK) return st;
    }
    // B-stationary GEMM (weights in registers per relation run) for the bench shapes
    if (gather_kind != 0 && W != nullptr && p->opt.rel_gemm && (((K == 64 || K == 128) && N == 128) || (K == 256 && N == 256 && p->opt.rel_wide)) &&
        trans == (gather_kind == 1 ? 1 : 0)) {
        RelGemmArgs r{};
        r.t_begin = p->d.t32_begin;
        r.t_end = p->d.t32_end;
        r.t_lo = s.t32_lo;
        r.n_rel = s.t32_hi - s.t32_lo;
        r.n_root = (Wroot != nullptr) ? (int)((row_hi - row_lo + 31) / 32) : 0;
        if (r.n_rel + r.n_root == 0) return MPGNN_OK;
        r.Arel = Hsrc;
        r.Aroot = src;
        r.s_src = p->d.s_src;
        r.m_lo = m_lo;
        r.s_row = p->d.s_row;
        r.s_cnt = p->d.s_cnt;
        r.s_rel = p->d.s_rel;
        r.W = W;
        r.w_per_rel = (mode == MPGNN_MODE_ALL);
        r.Wroot = Wroot;
        r.Y = Y;
        r.Yroot = Yroot;
        r.sel_b = s.sel_b;
        r.row_lo = (int)row_lo;
        r.row_hi = (int)row_hi;
        if (gather_kind != 1 && root_map != nullptr) {  // mode-SINGLE root epilogue (see RelGemmArgs)
            r.node_map = root_map;
            r.bias = root_bias;
            r.relu = root_relu;
        }
#ifdef MPGNN_STAMPS
        r.stamps = gather_kind == 1 ? nullptr : g_stamps_host;
#endif
        if (p->opt.gemm_bf3 && p->opt.gemm_w1 && K == 128 && r.node_map == nullptr && cu_count() % 8 == 0) {
            // one workgroup per CU, 64-row items (rel_gemm_w1_kernel)
            const int G = cu_count();
            r.wg_items = gemm_w1_items(p, r.t_lo, r.n_rel, r.row_lo, r.row_hi, Wroot != nullptr, G, strm);
            if (r.wg_items != nullptr) {
                TimedLaunch tl(kind, strm);
                if (gather_kind == 1)
                    hipLaunchKernelGGL(rel_gemm_w1_kernel<true>, dim3(G), dim3(kThreads), RelGemmW1<true>::lds_bytes(), strm, r);
                else
                    hipLaunchKernelGGL(rel_gemm_w1_kernel<false>, dim3(G), dim3(kThreads), RelGemmW1<false>::lds_bytes(), strm, r);
                return hip_check(hipGetLastError(), "rel_gemm_w1_kernel launch");
            }
        }
        if (p->opt.gemm_bf3 && (K == 64 || K == 128) && r.node_map == nullptr) {
            const int G = std::min(r.n_rel + r.n_root, cu_count() * 2);
            const bool pairs = p->opt.gemm_cu_pairs && G == cu_count() * 2 && cu_count() % 8 == 0;
            r.wg_items = gemm_ranges(p, r.t_lo, r.n_rel, r.n_root, G, pairs, strm);
            r.wg_cus = (pairs && r.wg_items != nullptr) ? cu_count() : 0;
            if (p->opt.gemm_first && K == 128 && p->opt.gemm_il && r.wg_items != nullptr && r.w_per_rel)
                r.first = gemm_first(p, r.wg_items, G, r, gather_kind == 1, strm);
        }
        if (zero != nullptr && zero_words > 0 && p->opt.gemm_bf3 && (K == 64 || K == 128) && r.node_map == nullptr) {
            r.zero = zero;  // launch_rel_gemm takes rel_gemm_bf3_kernel for these shapes
            r.zero_words = zero_words;
            if (zeroed != nullptr) *zeroed = true;
        }
        TimedLaunch tl(kind, strm);
        launch_rel_gemm(r, K, gather_kind == 1, p->opt, strm);
        return hip_check(hipGetLastError(), "rel_gemm_kernel launch");
    }
    // tile_gemm stages A rows as float4 (K % 4 == 0); other widths take seg_tile_kernel
    if (gather_kind != 0 && W != nullptr && (K & 3) == 0) {
        TileGemmArgs t{};
        t.tile_begin = p->d.tile_begin;
        t.tile_end = p->d.tile_end;
        t.tile_off = s.t_lo;
        t.n_rel = n_rel;
        t.n_root = n_root;
        t.ncol = (N + kColTile - 1) / kColTile;
        t.a_kind = gather_kind;
        t.src = src;
        t.Hsrc = Hsrc;
        t.s_src = p->d.s_src;
        t.m_lo = m_lo;
        t.s_row = p->d.s_row;
        t.s_cnt = p->d.s_cnt;
        t.s_rel = p->d.s_rel;
        t.K = K;
        t.W = W;
        t.w_per_rel = (mode == MPGNN_MODE_ALL);
        t.Wroot = Wroot;
        t.trans = trans;
        t.N = N;
        t.Y = Y;
        t.Yroot = Yroot;
        t.row_lo = (int)row_lo;
        t.row_hi = (int)row_hi;
        t.y_div = gather_kind == 1;
        t.sel_b = s.sel_b;
        TimedLaunch tl(kind, strm);
        launch_tile_gemm(t, strm);
        return hip_check(hipGetLastError(), "tile_gemm_kernel launch");
    }
    // odd widths (F % 4 != 0): seg_tile_kernel recomputes the means of its tiles from x
    // (gather kind 0) instead of reading the compact ones
    if (gather_kind == 2) gather_kind = 0;
    const bool ragged_t = gather_kind == 0 && !exact && s.sp_hi > s.sp_lo;
    if (ragged_t && !ragged) {
        PieceArgs pa{};
        pa.pb = p->d.seg_pb;
        pa.pe = p->d.seg_pe;
        pa.k_lo = s.sp_lo;
        pa.k_hi = s.sp_hi;
        pa.src = src;
        pa.F = K;
        pa.idx = p->d.e_col;
        pa.P = Pseg;
        TimedLaunch tl(MPGNN_K_PIECE, strm);
        MPGNN_VT_DISPATCH(V, T, launch_piece, pa, strm);
        int32_t st = hip_check(hipGetLastError(), "piece_sum_kernel(seg) launch");
        if (st != MPGNN_OK) return st;
    }
    SegTileArgs a{};
    a.tile_begin = p->d.tile_begin;
    a.tile_end = p->d.tile_end;
    a.tile_off = s.t_lo;
    a.n_rel_tiles = n_rel;
    a.gather_kind = gather_kind;
    a.src = src;
    a.F = K;
    a.s_ptr = ragged_t ? p->d.seg_ent_ptr : p->d.s_ptr;
    a.e_col = p->d.e_col;
    a.s_row = p->d.s_row;
    a.s_cnt = p->d.s_cnt;
    a.s_rel = p->d.s_rel;
    a.ent = ragged_t ? p->d.seg_ent : nullptr;
    a.P = Pseg;
    a.piece_off = s.sp_lo;
    a.W = W;
    a.w_per_rel = (mode == MPGNN_MODE_ALL);
    a.Wroot = Wroot;
    a.trans = trans;
    a.N = W ? N : 1;
    a.Y = Y;
    a.Yroot = Yroot;
    a.row_lo = (int)row_lo;
    a.row_hi = (int)row_hi;
    a.y_div = gather_kind == 1;
    a.sel_b = s.sel_b;
    a.H = H;
    a.Hsrc = Hsrc;
    const int ncol = W ? (N + kColTile - 1) / kColTile : 1;
    TimedLaunch tl(kind, strm);
    MPGNN_VT_DISPATCH(V, T, launch_seg, a, n_rel + n_root, ncol, strm);
    return hip_check(hipGetLastError(), "seg_tile_kernel launch");
}

template <int S, int KR>
static void launch_gather_rows_k(const GatherRowsArgs& a, hipStream_t st) {
    constexpr int rows_per_block = kWaves * KR * (64 / S);
    const int rows = a.N - a.r_begin;
    const dim3 grid((rows + rows_per_block - 1) / rows_per_block);
    if (a.extra != nullptr || a.bias != nullptr)
        hipLaunchKernelGGL((gather_rows_kernel<S, true, KR>), grid, dim3(kThreads), 0, st, a);
    else
        hipLaunchKernelGGL((gather_rows_kernel<S, false, KR>), grid, dim3(kThreads), 0, st, a);
}

// pieces (<= kPieceEntries entries each): one per sub-wave, all its entries in flight at once
// (C3 mode-SINGLE grad_x, 70 pieces: four pieces chained per sub-wave took 26 us); rows: four
// per sub-wave, their entries concatenated (rows average a few entries)
template <int S>
static void launch_gather_rows_s(const GatherRowsArgs& a, hipStream_t st, bool pieces) {
    if (pieces) launch_gather_rows_k<S, 1>(a, st);
    else launch_gather_rows_k<S, 4>(a, st);
}

static void launch_gather_rows(const GatherRowsArgs& a, hipStream_t st, bool pieces = false) {
    if (a.F <= 32) launch_gather_rows_s<8>(a, st, pieces);
    else if (a.F <= 64) launch_gather_rows_s<16>(a, st, pieces);
    else if (a.F <= 128) launch_gather_rows_s<32>(a, st, pieces);
    else launch_gather_rows_s<64>(a, st, pieces);
}

// Ordered row sums out[i] = Σ list(i) + extra + bias, with the pieces of long rows first.
// F % 4 == 0 runs gather_rows_kernel (16-byte lanes, several rows per load instruction);
// other widths the scalar row_sum_kernel.  Both sum every row in entry order.
static int32_t run_rowsum(const mpgnn_plan* p, RowSumArgs a, const int* pb, const int* pe, int k_lo, int k_hi,
                          float* P, hipStream_t strm) {
    a.g.dummy = p->d.s_ptr;  // S + 1 >= 1 entries: always a valid target
    const bool vec = (a.g.F & 3) == 0 && a.g.F <= kMaxF;
    int V, T;
    pick_vt(a.g.F, &V, &T);
    if (k_hi > k_lo) {
        if (vec) {
            GatherRowsArgs ga{};
            ga.N = k_hi;
            ga.r_begin = k_lo;
            ga.row_kind = 2;
            ga.ptr = pb;
            ga.pe = pe;
            ga.table = a.g.idx;
            ga.src = a.g.src;
            ga.F = a.g.F;
            ga.idx_off = a.g.idx_off;
            ga.filter = a.g.filter;
            ga.flo = a.g.flo;
            ga.fhi = a.g.fhi;
            ga.out = P;
            ga.out_off = k_lo;
            ga.dummy = a.g.dummy;
            TimedLaunch tl(MPGNN_K_PIECE, strm);
            launch_gather_rows(ga, strm, true);
        } else {
            PieceArgs pa{};
            pa.pb = pb;
            pa.pe = pe;
            pa.k_lo = k_lo;
            pa.k_hi = k_hi;
            pa.src = a.g.src;
            pa.F = a.g.F;
            pa.idx = a.g.idx;
            pa.idx_off = a.g.idx_off;
            pa.filter = a.g.filter;
            pa.dummy = a.g.dummy;
            pa.flo = a.g.flo;
            pa.fhi = a.g.fhi;
            pa.P = P;
            TimedLaunch tl(MPGNN_K_PIECE, strm);
            MPGNN_VT_DISPATCH(V, T, launch_piece, pa, strm);
        }
        int32_t st = hip_check(hipGetLastError(), "piece sum launch");
        if (st != MPGNN_OK) return st;
        a.g.P = P;
        a.g.piece_off = k_lo;
    }
    if (a.N <= a.r_begin) return MPGNN_OK;
    if (vec) {
        GatherRowsArgs ga{};
        ga.N = a.N;
        ga.r_begin = a.r_begin;
        ga.row_kind = a.list_kind;
        ga.ptr = a.ptr;
        ga.keys = a.keys;
        ga.kb = a.kb;
        ga.ke = a.ke;
        ga.table = a.g.ent != nullptr ? a.res : a.g.idx;
        ga.src = a.g.src;
        ga.F = a.g.F;
        ga.idx_off = a.g.idx_off;
        ga.filter = a.g.filter;
        ga.flo = a.g.flo;
        ga.fhi = a.g.fhi;
        ga.P = a.g.P;
        ga.piece_off = a.g.piece_off;
        ga.extra = a.extra;
        ga.bias = a.bias;
        ga.lo = a.lo;
        ga.hi = a.hi;
        ga.cnt = a.cnt;
        ga.out_off = a.out_off;
        ga.out = a.out;
        ga.dummy = a.g.dummy;
        launch_gather_rows(ga, strm);
        return hip_check(hipGetLastError(), "gather_rows_kernel launch");
    }
    MPGNN_VT_DISPATCH(V, T, launch_rowsum, a, strm);
    return hip_check(hipGetLastError(), "row_sum_kernel launch");
}

static void launch_outer_bf3(dim3 grid, const OuterArgs& r_in, const OuterArgs& w, int ra_n, int n_all, bool vec,
                             bool sq, hipStream_t st, int var = 0) {
    OuterArgs r = r_in;
#ifdef MPGNN_STAMPS
    r.stamps = g_stamps_host;
#endif
    if (vec)
        if (sq) hipLaunchKernelGGL(outer_bf3v_kernel_t<true>, grid, dim3(kThreads), kOvLds, st, r, w, ra_n, n_all);
        else if (var == 1) hipLaunchKernelGGL((outer_bf3v_kernel_t<false, 1>), grid, dim3(kThreads), kOvLds, st, r, w, ra_n, n_all);
        else if (var == 2) hipLaunchKernelGGL((outer_bf3v_kernel_t<false, 2>), grid, dim3(kThreads), kOvLds, st, r, w, ra_n, n_all);
        else hipLaunchKernelGGL(outer_bf3v_kernel_t<false>, grid, dim3(kThreads), kOvLds, st, r, w, ra_n, n_all);
    else
        hipLaunchKernelGGL(outer_bf3_kernel, grid, dim3(kThreads), kOb3Lds, st, r, w, ra_n, n_all);
}
template <int V, int T>
static void launch_flat(const FlatArgs& a, int max_pieces, int wg_per_cu, int u, hipStream_t st) {
    const int n_groups = a.g_hi - a.g_lo;
    const int n = wg_per_cu > 0 ? std::min(n_groups, cu_count() * wg_per_cu) : n_groups;
    const size_t lds = (size_t)max_pieces * a.F * sizeof(float);  // 0 when the list has no long row
    if (u == 32) hipLaunchKernelGGL((flat_rows_kernel<V, T, 32>), dim3(n), dim3(kThreads), lds, st, a);
    else if (u == 8) hipLaunchKernelGGL((flat_rows_kernel<V, T, 8>), dim3(n), dim3(kThreads), lds, st, a);
    else hipLaunchKernelGGL((flat_rows_kernel<V, T>), dim3(n), dim3(kThreads), lds, st, a);
}

template <int V, int T>
static void launch_final(const FinalArgs& a, int nrows, hipStream_t st) {
    hipLaunchKernelGGL((finalize_rows_kernel<V, T>), dim3((nrows + kWaves - 1) / kWaves), dim3(kThreads), 0, st, a);
}

// In-place ReLU for the paths whose combine has no fused activation (exact order, mode SINGLE).
__global__ __launch_bounds__(kThreads) void relu_kernel(float* __restrict__ p, size_t n) {
    for (size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (size_t)gridDim.x * kThreads)
        p[i] = relu_f(p[i]);
}

// Node map of one relation's segments for the fused mode-SINGLE layer: map[s_row[s]] =
// s_src[s] + 1 (x row) or s_src[s] (< 0: compact mean row); nodes without a segment keep 0.
__global__ __launch_bounds__(kThreads) void node_map_kernel(const int* __restrict__ s_row, const int* __restrict__ s_src,
                                                            int sel_b, int sel_e, int* __restrict__ map) {
    const int s = sel_b + (int)(blockIdx.x * kThreads + threadIdx.x);
    if (s >= sel_e) return;
    const int v = s_src[s];
    map[s_row[s]] = v >= 0 ? v + 1 : v;
}

// Mode-SINGLE combine for the widths the fused layer does not take (F % 4 == 0): a node has at
// most one segment of the relation, so out[i] = act((0 + Y[seg(i)] + Yroot[i]) + bias) streams
// row by row through a per-call node -> segment map (seg_map_kernel) — the same sums, in the same
// order, as the gather_rows path it replaces (a binary search of s_row per row, then a separate
// ReLU pass over the output): C5 single, F = 256, 2 M rows.
__global__ __launch_bounds__(kThreads) void seg_map_kernel(const int* __restrict__ s_row, int sel_b, int sel_e,
                                                           int* __restrict__ map) {
    const int s = sel_b + (int)(blockIdx.x * kThreads + threadIdx.x);
    if (s < sel_e) map[s_row[s]] = s - sel_b;
}

__global__ __launch_bounds__(kThreads) void single_combine_kernel(const float* __restrict__ Y, const float* __restrict__ Yroot,
                                                                  const float* __restrict__ bias,
                                                                  const int* __restrict__ map, int N, int F, int lo,
                                                                  int hi, int relu, float* __restrict__ out) {
    // one wave per row, lanes over its float4 columns (no index division)
    const int F4 = F >> 2;
    const int lane = threadIdx.x & 63;
    const bool own_terms = Yroot != nullptr || bias != nullptr;
    for (int i = (int)blockIdx.x * kWaves + (int)(threadIdx.x >> 6); i < N; i += (int)gridDim.x * kWaves) {
        const int m = map[i];
        const bool own = own_terms && i >= lo && i < hi;
        for (int c4 = lane; c4 < F4; c4 += 64) {
            const int c = 4 * c4;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (m >= 0) v = f4_add(v, *reinterpret_cast<const float4*>(Y + (size_t)m * F + c));
            if (own) {
                const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
                const float4 ex = Yroot ? *reinterpret_cast<const float4*>(Yroot + (size_t)(i - lo) * F + c) : z;
                const float4 bb = bias ? *reinterpret_cast<const float4*>(bias + c) : z;
                v = f4_add(f4_add(v, ex), bb);
            }
            if (relu) v = make_float4(relu_f(v.x), relu_f(v.y), relu_f(v.z), relu_f(v.w));
            *reinterpret_cast<float4*>(out + (size_t)i * F + c) = v;
        }
    }
}

// After the root epilogue (RelGemmArgs::node_map, not CAT): the rows WITH a segment of the
// relation, out[s_row[s]] = act(((0 + Y[s]) + x_i @ root) + bias) — the combine's order. One wave
// per segment row.
__global__ __launch_bounds__(kThreads) void single_fix_kernel(const float* __restrict__ Y, const int* __restrict__ s_row,
                                                              int sel_b, int sel_e, const float* __restrict__ bias,
                                                              int F, int relu, float* __restrict__ out) {
    const int F4 = F >> 2;
    const int lane = threadIdx.x & 63;
    const int n = sel_e - sel_b;
    for (int k = (int)blockIdx.x * kWaves + (int)(threadIdx.x >> 6); k < n; k += (int)gridDim.x * kWaves) {
        const int i = s_row[sel_b + k];
        for (int c4 = lane; c4 < F4; c4 += 64) {
            const int c = 4 * c4;
            float4* o = reinterpret_cast<float4*>(out + (size_t)i * F + c);
            const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
            float4 v = f4_add(f4_add(z, *reinterpret_cast<const float4*>(Y + (size_t)k * F + c)), *o);
            v = f4_add(v, bias ? *reinterpret_cast<const float4*>(bias + c) : z);
            if (relu) v = make_float4(relu_f(v.x), relu_f(v.y), relu_f(v.z), relu_f(v.w));
            *o = v;
        }
    }
}

// Every relation's node map at once (plan upload): segment s of dense relation d (binary search
// of s in rel_seg_ptr) sets map[d·N + s_row[s]].
__global__ __launch_bounds__(kThreads) void rel_node_map_kernel(const int* __restrict__ rel_seg_ptr, int nrel,
                                                                const int* __restrict__ s_row,
                                                                const int* __restrict__ s_src, int S, int64_t N,
                                                                int* __restrict__ map) {
    const int s = (int)(blockIdx.x * kThreads + threadIdx.x);
    if (s >= S) return;
    int lo = 0, hi = nrel;  // largest d with rel_seg_ptr[d] <= s
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (rel_seg_ptr[mid] <= s) lo = mid;
        else hi = mid;
    }
    const int v = s_src[s];
    map[(int64_t)lo * N + s_row[s]] = v >= 0 ? v + 1 : v;
}

int32_t build_rel_node_maps(mpgnn_plan* p, void* stream) {
    const size_t rows = (size_t)p->nrel + 1;  // + the all-zero row of an absent relation
    const size_t bytes = rows * (size_t)p->N * sizeof(int32_t);
    if (p->N == 0 || bytes > ((size_t)1 << 30)) return MPGNN_OK;  // per-call maps instead
    hipStream_t strm = static_cast<hipStream_t>(stream);
    void* m = nullptr;
    if (hipMalloc(&m, bytes) != hipSuccess) {
        (void)hipGetLastError();
        return MPGNN_OK;  // not fatal: per-call maps
    }
    int32_t st = hip_check(hipMemsetAsync(m, 0, bytes, strm), "memset node maps");
    if (st == MPGNN_OK && p->S > 0) {
        hipLaunchKernelGGL(rel_node_map_kernel, dim3((unsigned)((p->S + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                           strm, p->d.rel_seg_ptr, (int)p->nrel, p->d.s_row, p->d.s_src, (int)p->S, p->N,
                           static_cast<int*>(m));
        st = hip_check(hipGetLastError(), "rel_node_map_kernel launch");
    }
    // published only once complete: calls on other streams may read it right after
    if (st == MPGNN_OK) st = hip_check(hipStreamSynchronize(strm), "node maps");
    if (st != MPGNN_OK) {
        (void)hipFree(m);
        return st;
    }
    p->d.rel_node_map = static_cast<int32_t*>(m);
    return MPGNN_OK;
}

template <int KB>
static void launch_rel_gemm_cat(const RelGemmArgs& a, hipStream_t st) {
    constexpr int lda = 64 * KB + 4;
    const size_t lds = (size_t)(2 * 32 * lda + 64 + 4) * sizeof(float);
    const int grid = std::min(a.n_root, cu_count() * 2);
    hipLaunchKernelGGL((rel_gemm_kernel<KB, false, 1, 2, true>), dim3(grid), dim3(kThreads), lds, st, a);
}

// Fast-path row sums over a flat chunked list: flat_rows_kernel over groups [g_lo, g_hi), then
// finalize_rows_kernel — mode 0 over split rows [k_lo, k_hi) (means: no empty rows, no extra),
// mode 1 over every row [r_lo, r_hi) (split and empty rows, extra + bias on own rows).
struct FlatRun {
    const FlatDev* fd;
    int max_pieces;       // the list's largest long group (LDS slots)
    int g_lo, g_hi, k_lo, k_hi;
    const int* table;
    int idx_off, filter, flo, fhi;
    const float* src;
    int F;
    int row_off;
    float* out;
    float* carry;
    int final_mode;
    const int* row_ptr;   // mode 1
    int r_lo, r_hi;       // mode 1
    const int* cnt;       // mode 0
    const float* extra;
    const float* bias;
    int lo, hi;
    int relu;             // fused activation (unsharded forward combine)
    unsigned* arrive;     // mode 0: [nsplit] zeroed piece counters — split rows finished in the launch
    int wg_per_cu;        // the plan's MPGNN_OPT_FLAT_WG_PER_CU
    int u = 16;           // the plan's MPGNN_OPT_FLAT_U: rows in flight per wave (8, 16, 32)
    int ngroups = 0;      // groups of the whole list (the padded slot tables cover them all)
    const mpgnn_plan* plan = nullptr;  // non-null with MPGNN_OPT_FLAT_PAD: padded slot tables
    const float* mask = nullptr;       // FlatArgs::mask
};

// flat_rows_kernel's padded slot tables of one (list, value table) pair (FlatArgs::pad_desc):
// one thread per (slot, position); a slot past its group's chunks, or of a long group, has n = 0
__global__ __launch_bounds__(kThreads) void flat_pad_kernel(int64_t nslots, const int* __restrict__ group_ptr,
                                                            const int* __restrict__ group_long,
                                                            const int* __restrict__ chunk_ptr,
                                                            const int* __restrict__ chunk_info,
                                                            const int* __restrict__ table, const int* __restrict__ row_of,
                                                            int4* desc, int* pval, int* prow) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t slot = t >> 5;
    const int q = (int)(t & 31);
    if (slot >= nslots) return;
    const int g = (int)(slot >> 2), w = (int)(slot & 3);
    const int lng = group_long[g] != 0;
    const int c = group_ptr[g] + w;
    int n = 0, info = 0, p0 = 0;
    if (!lng && c < group_ptr[g + 1]) {
        p0 = chunk_ptr[c];
        n = chunk_ptr[c + 1] - p0;
        info = chunk_info[c];
    }
    if (q == 0) desc[slot] = make_int4(n, info, lng, 0);
    const int pq = p0 + min(q, max(n - 1, 0));  // flat_chunk's lane clamp
    pval[t] = n > 0 ? table[pq] : 0;
    prow[t] = n > 0 ? row_of[pq] : 0;
}

// Cached per plan and (list, table); made outside captures (false: the kernel's scalar path)
static bool flat_pad_tables(const mpgnn_plan* p, const FlatDev* fd, int ngroups, const int* table, hipStream_t st,
                            FlatArgs* a) {
    if (ngroups <= 0 || table == nullptr) return false;
    const std::array<int64_t, 5> key{(int64_t)(intptr_t)fd, (int64_t)(intptr_t)table, ngroups, 0, 0};
    std::lock_guard<std::mutex> lk(p->bw_mu);
    auto it = p->flat_pads.find(key);
    const int64_t nslots = 4 * (int64_t)ngroups;
    auto set = [&](char* base) {
        a->pad_desc = reinterpret_cast<const int4*>(base);
        a->pad_val = reinterpret_cast<const int*>(base + nslots * 16);
        a->pad_row = reinterpret_cast<const int*>(base + nslots * 16 + nslots * 32 * 4);
    };
    if (it != p->flat_pads.end()) {
        set(reinterpret_cast<char*>(it->second.dev));
        return true;
    }
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return false;
    mpgnn_plan::GemmRanges e;
    const size_t bytes = (size_t)nslots * (16 + 2 * 32 * 4);
    if (hipMalloc(reinterpret_cast<void**>(&e.dev), bytes) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    char* base = reinterpret_cast<char*>(e.dev);
    const int64_t nthr = nslots * 32;
    hipLaunchKernelGGL(flat_pad_kernel, dim3((unsigned)((nthr + kThreads - 1) / kThreads)), dim3(kThreads), 0, st,
                       nslots, fd->group_ptr, fd->group_long, fd->chunk_ptr, fd->chunk_info, table, fd->row_of,
                       reinterpret_cast<int4*>(base), reinterpret_cast<int*>(base + nslots * 16),
                       reinterpret_cast<int*>(base + nslots * 16 + nslots * 32 * 4));
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {  // published once complete
        (void)hipGetLastError();
        (void)hipFree(e.dev);
        return false;
    }
    p->flat_pads[key] = e;
    set(base);
    return true;
}

static int32_t run_flat(const FlatRun& f, hipStream_t strm) {
    int V, T;
    pick_vt(f.F, &V, &T);
    if (f.g_hi > f.g_lo) {
        FlatArgs a{};
        a.chunk_ptr = f.fd->chunk_ptr;
        a.chunk_info = f.fd->chunk_info;
        a.group_ptr = f.fd->group_ptr;
        a.group_long = f.fd->group_long;
        a.g_lo = f.g_lo;
        a.g_hi = f.g_hi;
        a.table = f.table;
        a.row_of = f.fd->row_of;
        a.src = f.src;
        a.F = f.F;
        a.idx_off = f.idx_off;
        a.filter = f.filter;
        a.flo = f.flo;
        a.fhi = f.fhi;
        a.cnt = f.cnt;
        a.dummy = f.fd->chunk_ptr;
        a.row_off = f.row_off;
        if (f.final_mode == 0) {  // augmented lists carry the extra rows; bias at the flush
            a.extra = f.extra;
            a.bias = f.bias;
            a.lo = f.lo;
            a.hi = f.hi;
        }
        a.out = f.out;
        a.carry = f.carry;
        a.relu = f.final_mode == 0 ? f.relu : 0;
        // mode 0 finishes rows here; mode 1 leaves them to the finalize (which adds extra rows)
        a.mask = f.final_mode == 0 ? f.mask : nullptr;
        if (f.final_mode == 0 && f.arrive != nullptr) {
            a.arrive = f.arrive;
            a.row_split = f.fd->row_split;
            a.split_ptr = f.fd->split_ptr;
            a.split_slot = f.fd->split_slot;
        }  // mode 1: the finalize adds extra + bias first
        if (f.plan != nullptr && f.plan->opt.flat_pad && f.wg_per_cu == 0)
            (void)flat_pad_tables(f.plan, f.fd, f.ngroups, f.table, strm, &a);
        MPGNN_VT_DISPATCH(V, T, launch_flat, a, f.max_pieces, f.wg_per_cu, f.u, strm);
        int32_t st = hip_check(hipGetLastError(), "flat_rows_kernel launch");
        if (st != MPGNN_OK) return st;
    }
    FinalArgs b{};
    b.mode = f.final_mode;
    b.split_row = f.fd->split_row;
    b.split_ptr = f.fd->split_ptr;
    b.split_slot = f.fd->split_slot;
    b.k0 = f.k_lo;
    b.k1 = f.k_hi;
    b.row_split = f.fd->row_split;
    b.row_ptr = f.row_ptr;
    b.r_lo = f.r_lo;
    b.r_hi = f.r_hi;
    b.carry = f.carry;
    b.F = f.F;
    b.cnt = f.cnt;
    b.extra = f.final_mode == 0 ? nullptr : f.extra;  // mode 0: extra rows are inside the slots
    b.bias = f.bias;
    b.lo = f.lo;
    b.hi = f.hi;
    b.row_off = f.row_off;
    b.out = f.out;
    b.dummy = f.out;
    b.relu = f.relu;
    b.mask = f.mask;
    const int nrows = f.final_mode == 0 ? f.k_hi - f.k_lo : f.r_hi - f.r_lo;
    if (nrows <= 0 || (f.final_mode == 0 && f.arrive != nullptr && f.g_hi > f.g_lo)) return MPGNN_OK;
    TimedLaunch tl(MPGNN_K_FINAL, strm);
    MPGNN_VT_DISPATCH(V, T, launch_final, b, nrows, strm);
    return hip_check(hipGetLastError(), "finalize_rows_kernel launch");
}

// Segment means H[s - sel_b] = (Σ_{e in s} x[node_2(e)]) / cnt(s) for the selection, through
// the ragged row-sum (pieces of segments > kPieceEntries first) or in exact edge order.
static int32_t run_means(const mpgnn_plan* p, const Selection& s, const float* x, int F, float* H, float* Pseg,
                         bool exact, hipStream_t strm) {
    if (s.sel_e == s.sel_b) return MPGNN_OK;
    if (!exact) {
        // flat chunked list; chunks and splits of the relation range [d_lo, d_hi)
        FlatRun f{};
        f.wg_per_cu = p->opt.flat_wg_per_cu;
        f.u = p->opt.flat_u;
        f.plan = p;
        f.fd = &p->d.seg_f;
        f.max_pieces = p->seg_f.max_pieces;
        f.ngroups = p->seg_f.ngroups;
        f.g_lo = p->seg_f.cut_group_ptr[s.d_lo];
        f.g_hi = p->seg_f.cut_group_ptr[s.d_hi];
        f.k_lo = p->seg_f.cut_split_ptr[s.d_lo];
        f.k_hi = p->seg_f.cut_split_ptr[s.d_hi];
        f.table = p->d.e_col;
        f.src = x;
        f.F = F;
        f.row_off = s.sel_b;
        f.out = H;
        f.carry = Pseg;
        f.final_mode = 0;
        f.cnt = p->d.s_cnt;
        return run_flat(f, strm);
    }
    const bool ragged = !exact && s.sp_hi > s.sp_lo;
    RowSumArgs a{};
    a.r_begin = s.sel_b;
    a.N = s.sel_e;
    a.list_kind = 0;
    a.ptr = ragged ? p->d.seg_ent_ptr : p->d.s_ptr;
    a.g.src = x;
    a.g.F = F;
    a.g.idx = p->d.e_col;
    a.g.ent = ragged ? p->d.seg_ent : nullptr;
    a.res = p->d.seg_res;
    a.cnt = p->d.s_cnt;
    a.out = H;
    a.out_off = s.sel_b;
    return run_rowsum(p, a, p->d.seg_pb, p->d.seg_pe, ragged ? s.sp_lo : 0, ragged ? s.sp_hi : 0, Pseg, strm);
}

// Compact means of the selection's multi-edge segments: Hm[m - m_lo] = (Σ x[em_col]) / m_cnt[m]
// for m in [m_lo, m_hi) — the flat chunked list (rows inside one chunk in reference order), or
// the sequential row sum in exact mode. The single-edge segments' means are x rows (s_src).
static int32_t run_means_multi(const mpgnn_plan* p, const Selection& s, const float* x, int F, float* Hm,
                               float* carry, bool exact, hipStream_t strm) {
    if (s.m_hi == s.m_lo) return MPGNN_OK;
    if (!exact) {
        FlatRun f{};
        f.wg_per_cu = p->opt.flat_wg_per_cu;
        f.u = p->opt.flat_u;
        f.plan = p;
        f.fd = &p->d.segm_f;
        f.max_pieces = p->segm_f.max_pieces;
        f.ngroups = p->segm_f.ngroups;
        f.g_lo = p->segm_f.cut_group_ptr[s.d_lo];
        f.g_hi = p->segm_f.cut_group_ptr[s.d_hi];
        f.k_lo = p->segm_f.cut_split_ptr[s.d_lo];
        f.k_hi = p->segm_f.cut_split_ptr[s.d_hi];
        f.table = p->d.em_col;
        f.src = x;
        f.F = F;
        f.row_off = s.m_lo;
        f.out = Hm;
        f.carry = carry;
        f.final_mode = 0;
        f.cnt = p->d.m_cnt;
        return run_flat(f, strm);
    }
    RowSumArgs a{};
    a.r_begin = s.m_lo;
    a.N = s.m_hi;
    a.list_kind = 0;
    a.ptr = p->d.m_ptr;
    a.g.src = x;
    a.g.F = F;
    a.g.idx = p->d.em_col;
    a.cnt = p->d.m_cnt;
    a.out = Hm;
    a.out_off = s.m_lo;
    return run_rowsum(p, a, nullptr, nullptr, 0, 0, carry, strm);
}

}  // namespace mpgnn

using namespace mpgnn;

extern "C" {

int32_t mpgnn_relu_bwd(const float* grad_out, const float* act_out, int64_t n, float* dst, void* stream) {
    if (n < 0) return arg_error("negative n");
    if (n == 0) return MPGNN_OK;
    if (!grad_out || !act_out || !dst) return arg_error("NULL grad_out, act_out or dst");
    hipStream_t strm = static_cast<hipStream_t>(stream);
    const bool vec = ((reinterpret_cast<uintptr_t>(grad_out) | reinterpret_cast<uintptr_t>(act_out) |
                       reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
    const int64_t units = vec ? (n + 3) / 4 : n;
    const int blocks = (int)std::min<int64_t>((units + kThreads - 1) / kThreads, 8192);
    hipLaunchKernelGGL(relu_bwd_kernel, dim3(blocks), dim3(kThreads), 0, strm, grad_out, act_out, n, dst, vec ? 1 : 0);
    return hip_check(hipGetLastError(), "relu_bwd_kernel launch");
}

static int linear_parts(int64_t N) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(4096, (N + kLinRowsPerPart - 1) / kLinRowsPerPart));
}

static int linear_block(int F) { return kLinAcc * (kThreads / F); }  // outputs per pass

// F = O = 128 (MPNetm.fc1 of one 128-wide metapath, model.py:224): gw = gᵀ x is a 128 × 128
// outer-product sum over N rows — outer_bf3_kernel's root-chunk stream with A = grad_out,
// B = x and the bias column sums taken from A (bias_of_a), row chunks of >= 64 rows (about two
// per CU), then the ordered slab sum (reduce_slabs3_kernel). The scalar pair below needs 2 × ~50 µs
// for this width at C3 (two output blocks), the library's sliced GEMM ~45-60 µs.
static bool linear_bf3(int64_t N, int32_t F, int32_t O) { return default_options().gemm_bf3 && F == 128 && O == 128 && N > 0; }
static int linear_bf3_chunk(int64_t N) {
    const int64_t per = (N + 2 * (int64_t)cu_count() - 1) / (2 * (int64_t)cu_count());
    return (int)std::max<int64_t>(64, (per + 15) / 16 * 16);
}

int32_t mpgnn_linear_wgrad_workspace_bytes(int64_t N, int32_t F, int32_t O, int64_t* bytes) {
    if (!bytes) return arg_error("NULL bytes");
    if (N < 0 || F <= 0 || O <= 0) return arg_error("bad N, F or O");
    if (F > kThreads) return arg_error("mpgnn_linear_wgrad: needs F <= 256");
    *bytes = (int64_t)linear_parts(N) * std::min(O, linear_block(F)) * (F + 1) * (int64_t)sizeof(float);
    if (linear_bf3(N, F, O)) {
        const int64_t nch = (N + linear_bf3_chunk(N) - 1) / linear_bf3_chunk(N);
        *bytes = std::max<int64_t>(*bytes, nch * (128 * 128 + 128) * (int64_t)sizeof(float));
    }
    return MPGNN_OK;
}

// Linear head forward / input gradient (model.py:147, 224-226): F = O = 128 on the bf16-split GEMM
// (rel_gemm_bf3_kernel over node rows only: forward with W read transposed as the dgrad does,
// the input gradient as a plain forward), O <= 8 with a wave per row; others: unsupported.
static int linear_grid(int64_t work) { return (int)std::max<int64_t>(1, std::min<int64_t>(8 * (int64_t)cu_count(), (work + kThreads - 1) / kThreads)); }

static int32_t linear_gemm128(const float* A, int64_t N, const float* W, bool transposed, float* out, hipStream_t strm) {
    RelGemmArgs a{};
    a.n_rel = 0;
    a.n_root = (int)((N + 31) / 32);
    a.Aroot = A;
    a.W = W;
    a.Wroot = W;
    a.Yroot = out;
    a.Y = out;
    a.row_lo = 0;
    a.row_hi = (int)N;
    launch_rel_gemm(a, 128, transposed, default_options(), strm);
    return hip_check(hipGetLastError(), "rel_gemm_bf3_kernel launch (linear)");
}

int32_t mpgnn_linear_fwd(const float* x, int64_t N, int32_t F, const float* weight, int32_t O, const float* bias,
                         int32_t act, float* out, void* stream) {
    if (N < 0 || N > INT32_MAX || F <= 0 || O <= 0) return arg_error("mpgnn_linear_fwd: bad N, F or O");
    if (act != MPGNN_ACT_NONE && act != MPGNN_ACT_RELU && act != MPGNN_ACT_LOG_SOFTMAX)
        return arg_error("mpgnn_linear_fwd: bad act");
    const bool gemm = F == 128 && O == 128 && default_options().gemm_bf3 && act != MPGNN_ACT_LOG_SOFTMAX;
    const bool small = O <= kLinSmallO && F <= 256 && F % 4 == 0;
    if (!gemm && !small) return MPGNN_ERR_UNSUPPORTED;
    if (N == 0) return MPGNN_OK;
    if (!x || !weight || !out) return arg_error("mpgnn_linear_fwd: NULL pointer");
    if (((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(weight) | reinterpret_cast<uintptr_t>(out) |
          reinterpret_cast<uintptr_t>(bias)) & 15) != 0)
        return arg_error("mpgnn_linear_fwd: pointers must be 16-byte aligned");
    hipStream_t strm = static_cast<hipStream_t>(stream);
    if (gemm) {
        int32_t st = linear_gemm128(x, N, weight, true, out, strm);
        if (st != MPGNN_OK || (bias == nullptr && act == MPGNN_ACT_NONE)) return st;
        const int64_t n4 = N * 128 / 4;
        hipLaunchKernelGGL(bias_act_kernel, dim3(linear_grid(n4)), dim3(kThreads), 0, strm, out, n4, 32, bias, act);
        return hip_check(hipGetLastError(), "bias_act_kernel launch");
    }
    const int grid = (int)std::min<int64_t>(8 * (int64_t)cu_count(), (N + 15) / 16);  // 16 rows per workgroup
    hipLaunchKernelGGL(linear_small_fwd_kernel, dim3(grid), dim3(kThreads), 0, strm, x, (int)N, F, weight, O, bias, act, out);
    return hip_check(hipGetLastError(), "linear_small_fwd_kernel launch");
}

static int32_t linear_dgrad_impl(const float* grad_out, int64_t N, int32_t O, const float* weight, int32_t F,
                                 float* grad_x, const float* mask, void* stream) {
    if (N < 0 || N > INT32_MAX || F <= 0 || O <= 0) return arg_error("mpgnn_linear_dgrad: bad N, F or O");
    const bool gemm = F == 128 && O == 128 && default_options().gemm_bf3;
    const bool small = O <= kLinSmallO && F % 4 == 0;
    if (!gemm && !small) return MPGNN_ERR_UNSUPPORTED;
    if (N == 0) return MPGNN_OK;
    if (!grad_out || !weight || !grad_x) return arg_error("mpgnn_linear_dgrad: NULL pointer");
    if (((reinterpret_cast<uintptr_t>(grad_out) | reinterpret_cast<uintptr_t>(weight) | reinterpret_cast<uintptr_t>(grad_x) |
          reinterpret_cast<uintptr_t>(mask)) & 15) != 0)
        return arg_error("mpgnn_linear_dgrad: pointers must be 16-byte aligned");
    hipStream_t strm = static_cast<hipStream_t>(stream);
    if (gemm) {
        int32_t st = linear_gemm128(grad_out, N, weight, false, grad_x, strm);
        if (st != MPGNN_OK || mask == nullptr) return st;
        const int64_t n = N * F;
        hipLaunchKernelGGL(relu_bwd_kernel, dim3((unsigned)std::min<int64_t>((n + kThreads - 1) / kThreads, 4096)),
                           dim3(kThreads), 0, strm, grad_x, mask, n, grad_x, 1);
        return hip_check(hipGetLastError(), "relu_bwd_kernel (linear dgrad mask) launch");
    }
    hipLaunchKernelGGL(linear_small_dgrad_kernel, dim3(linear_grid(N * (F / 4))), dim3(kThreads), 0, strm, grad_out, (int)N, O,
                       weight, F, grad_x, mask);
    return hip_check(hipGetLastError(), "linear_small_dgrad_kernel launch");
}

int32_t mpgnn_dropout_relu_bwd(const float* grad_out, const uint8_t* mask, const float* act_out, float scale, int64_t n,
                               float* dst, void* stream) {
    if (n < 0) return arg_error("mpgnn_dropout_relu_bwd: bad n");
    if (n == 0) return MPGNN_OK;
    if (!grad_out || !mask || !dst) return arg_error("mpgnn_dropout_relu_bwd: NULL pointer");
    hipStream_t strm = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(dropout_relu_bwd_kernel, dim3((unsigned)std::min<int64_t>((n + kThreads - 1) / kThreads, 8192)),
                       dim3(kThreads), 0, strm, grad_out, mask, act_out, scale, n, dst);
    return hip_check(hipGetLastError(), "dropout_relu_bwd_kernel launch");
}

int32_t mpgnn_linear_dgrad(const float* grad_out, int64_t N, int32_t O, const float* weight, int32_t F, float* grad_x,
                           void* stream) {
    return linear_dgrad_impl(grad_out, N, O, weight, F, grad_x, nullptr, stream);
}

int32_t mpgnn_linear_dgrad_relu_in(const float* grad_out, int64_t N, int32_t O, const float* weight, int32_t F,
                                   const float* x, float* grad_x, void* stream) {
    if (N > 0 && x == nullptr) return arg_error("mpgnn_linear_dgrad_relu_in: NULL x");
    return linear_dgrad_impl(grad_out, N, O, weight, F, grad_x, x, stream);
}

static int lsm_parts(int64_t N) { return (int)std::max<int64_t>(1, std::min<int64_t>(1024, (N + 31) / 32)); }

int32_t mpgnn_linear_logsoftmax_bwd_workspace_bytes(int64_t N, int32_t F, int32_t O, int64_t* bytes) {
    if (!bytes) return arg_error("NULL bytes");
    if (N < 0 || N > INT32_MAX || F <= 0 || O <= 0) return arg_error("bad N, F or O");
    if (F > kThreads || F % 4 != 0 || O > kLsmO) return MPGNN_ERR_UNSUPPORTED;
    *bytes = (int64_t)lsm_parts(N) * O * (F + 1) * (int64_t)sizeof(float);
    return MPGNN_OK;
}

int32_t mpgnn_linear_logsoftmax_bwd(const float* grad_logp, const float* logp, const float* x, int64_t N, int32_t F,
                                    int32_t O, const float* weight, const float* relu_in, float* grad_x,
                                    float* grad_weight, float* grad_bias, void* workspace, void* stream) {
    if (N < 0 || N > INT32_MAX || F <= 0 || O <= 0) return arg_error("bad N, F or O");
    if (F > kThreads || F % 4 != 0 || O > kLsmO) return MPGNN_ERR_UNSUPPORTED;
    if (((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(weight) | reinterpret_cast<uintptr_t>(relu_in) |
          reinterpret_cast<uintptr_t>(grad_x)) & 15) != 0)
        return arg_error("mpgnn_linear_logsoftmax_bwd: x, weight, relu_in, grad_x must be 16-byte aligned");
    if (!grad_weight || !workspace || !weight || (N > 0 && (!x || !grad_logp || !logp)))
        return arg_error("mpgnn_linear_logsoftmax_bwd: NULL pointer");
    hipStream_t strm = static_cast<hipStream_t>(stream);
    if (N == 0) {
        int32_t st = hip_check(hipMemsetAsync(grad_weight, 0, (size_t)O * F * sizeof(float), strm), "memset");
        if (st == MPGNN_OK && grad_bias) st = hip_check(hipMemsetAsync(grad_bias, 0, (size_t)O * sizeof(float), strm), "memset");
        return st;
    }
    const int parts = lsm_parts(N);
    const int rows = (int)((N + parts - 1) / parts);
    float* P = static_cast<float*>(workspace);
    if (O <= 2)
        hipLaunchKernelGGL((linear_lsm_bwd_kernel<2, 4>), dim3(parts), dim3(kThreads), 0, strm, grad_logp, logp, x,
                           relu_in, (int)N, F, O, weight, grad_x, rows, P);
    else
        hipLaunchKernelGGL((linear_lsm_bwd_kernel<kLsmO, 4>), dim3(parts), dim3(kThreads), 0, strm, grad_logp, logp, x,
                           relu_in, (int)N, F, O, weight, grad_x, rows, P);
    int32_t st = hip_check(hipGetLastError(), "linear_lsm_bwd_kernel launch");
    if (st != MPGNN_OK) return st;
    const int elems = O * (F + 1);
    hipLaunchKernelGGL(linear_wgrad_sum_kernel, dim3((elems + kWaves - 1) / kWaves), dim3(kThreads), 0, strm, P, parts, F,
                       O, grad_weight, grad_bias);
    return hip_check(hipGetLastError(), "linear_wgrad_sum_kernel launch");
}

int32_t mpgnn_linear_wgrad(const float* x, const float* grad_out, int64_t N, int32_t F, int32_t O, float* grad_weight,
                           float* grad_bias, void* workspace, void* stream) {
    if (N < 0 || F <= 0 || O <= 0) return arg_error("bad N, F or O");
    if (F > kThreads) return arg_error("mpgnn_linear_wgrad: needs F <= 256");
    if (N > INT32_MAX) return arg_error("N too large");
    if (!grad_weight || !workspace || (N > 0 && (!x || !grad_out))) return arg_error("NULL pointer");
    hipStream_t strm = static_cast<hipStream_t>(stream);
    const int parts = linear_parts(N);
    const int rows = (int)((N + parts - 1) / parts);
    float* P = static_cast<float*>(workspace);
    if (N == 0) {
        int32_t st = hip_check(hipMemsetAsync(grad_weight, 0, (size_t)O * F * sizeof(float), strm), "memset");
        if (st == MPGNN_OK && grad_bias) st = hip_check(hipMemsetAsync(grad_bias, 0, (size_t)O * sizeof(float), strm), "memset");
        return st;
    }
    if (linear_bf3(N, F, O)) {
        const int chunk = linear_bf3_chunk(N);
        const int nch = (int)((N + chunk - 1) / chunk);
        float* Pb = P + (size_t)nch * 128 * 128;
        OuterArgs orr{};
        orr.row_lo = 0;
        orr.row_hi = (int)N;
        orr.chunk_rows = chunk;
        orr.dst_mode = nch == 1 ? 3 : 0;
        orr.A = grad_out;  // D[o][f] = Σ_i g[i][o] · x[i][f]
        orr.M = 128;
        orr.B = x;
        orr.Nn = 128;
        orr.P = P;
        orr.dst = grad_weight;
        orr.Pb = grad_bias ? Pb : nullptr;
        orr.dst_b = grad_bias;
        orr.bias_of_a = 1;
        OuterArgs none{};
        launch_outer_bf3(dim3(std::min(nch, cu_count() * 2)), orr, none, nch, nch, default_options().outer_vec, default_options().outer_sq, strm);
        int32_t st = hip_check(hipGetLastError(), "outer_bf3_kernel (linear) launch");
        if (st != MPGNN_OK || nch == 1) return st;
        ReduceArgs rw{}, rb{};
        rw.P = P;
        rw.elems = 128 * 128;
        rw.nchunks = nch;
        rw.dst = grad_weight;
        rb.P = Pb;
        rb.elems = 128;
        rb.nchunks = nch;
        rb.dst = grad_bias;
        const int nb = grad_bias ? 1 : 0;
        hipLaunchKernelGGL(reduce_slabs3_kernel, dim3(1 + nb, (128 * 128 + kThreads - 1) / kThreads), dim3(kThreads), 0,
                           strm, rw, rb, ReduceArgs{}, 1, nb, 0, ZeroList{});
        return hip_check(hipGetLastError(), "reduce_slabs3_kernel (linear) launch");
    }
    // output blocks in order; the partials buffer is reused (stream order)
    for (int o_lo = 0; o_lo < O; o_lo += linear_block(F)) {
        const int Ob = std::min(O - o_lo, linear_block(F));
        hipLaunchKernelGGL(linear_wgrad_part_kernel, dim3(parts), dim3(kThreads), 0, strm, x, grad_out + o_lo, O, (int)N,
                           F, Ob, rows, P);
        int32_t st = hip_check(hipGetLastError(), "linear_wgrad_part_kernel launch");
        if (st != MPGNN_OK) return st;
        const int elems = Ob * (F + 1);
        hipLaunchKernelGGL(linear_wgrad_sum_kernel, dim3((elems + kWaves - 1) / kWaves), dim3(kThreads), 0, strm, P,
                           parts, F, Ob, grad_weight + (size_t)o_lo * F, grad_bias ? grad_bias + o_lo : nullptr);
        if ((st = hip_check(hipGetLastError(), "linear_wgrad_sum_kernel launch")) != MPGNN_OK) return st;
    }
    return MPGNN_OK;
}

// The per-plan switches of enum mpgnn_option: set / read one in `o`. MPGNN_ERR_UNSUPPORTED
// (nothing set) when `option` is not one of them.
static int32_t set_switch(Options& o, int32_t option, int64_t value) {
    switch (option) {
        case MPGNN_OPT_EXACT_ORDER: o.exact_order = value != 0; return MPGNN_OK;
        case MPGNN_OPT_REL_GEMM: o.rel_gemm = value != 0; return MPGNN_OK;
        case MPGNN_OPT_REL_WIDE: o.rel_wide = value != 0; return MPGNN_OK;
        case MPGNN_OPT_GEMM_BF3: o.gemm_bf3 = value != 0; return MPGNN_OK;
        case MPGNN_OPT_GEMM_IL: o.gemm_il = value != 0; return MPGNN_OK;
        case MPGNN_OPT_GEMM_CU_PAIRS: o.gemm_cu_pairs = value != 0; return MPGNN_OK;
        case MPGNN_OPT_BWD_FUSED: o.bwd_fused = value != 0; return MPGNN_OK;
        case MPGNN_OPT_FLAT_FUSE_SPLIT: o.flat_fuse_split = value != 0; return MPGNN_OK;
        case MPGNN_OPT_OUTER_VEC: o.outer_vec = value != 0; return MPGNN_OK;
        case MPGNN_OPT_OUTER_SQ: o.outer_sq = value != 0; return MPGNN_OK;
        case MPGNN_OPT_OUTER_RANGES: o.outer_ranges = value != 0; return MPGNN_OK;
        case MPGNN_OPT_GEMM_W_IL: o.gemm_w_il = value != 0; return MPGNN_OK;
        case MPGNN_OPT_GEMM_W1: o.gemm_w1 = value != 0; return MPGNN_OK;
        case MPGNN_OPT_FLAT_PAD: o.flat_pad = value != 0; return MPGNN_OK;
        case MPGNN_OPT_SINGLE_FOLD: o.single_fold = value != 0; return MPGNN_OK;
        case MPGNN_OPT_BWD_SIDE_REDUCE: o.side_reduce = value != 0; return MPGNN_OK;
        case MPGNN_OPT_GEMM_FIRST: o.gemm_first = value != 0; return MPGNN_OK;
        case MPGNN_OPT_FLAT_U:
            if (value != 8 && value != 16 && value != 32) return arg_error("MPGNN_OPT_FLAT_U must be 8, 16 or 32");
            o.flat_u = (int)value;
            return MPGNN_OK;
        case MPGNN_OPT_OUTER_VARIANT:
            if (value < 0 || value > 2) return arg_error("MPGNN_OPT_OUTER_VARIANT must be 0, 1 or 2");
            o.outer_variant = (int)value;
            return MPGNN_OK;
        case MPGNN_OPT_GEMM_SWITCH_COST:
            if (value < 0 || value > 10000) return arg_error("MPGNN_OPT_GEMM_SWITCH_COST must be 0..10000 (percent of an item)");
            o.gemm_switch_cost = (int)value;
            return MPGNN_OK;
        case MPGNN_OPT_FLAT_WG_PER_CU:
            if (value < 0 || value > 64) return arg_error("MPGNN_OPT_FLAT_WG_PER_CU must be 0..64");
            o.flat_wg_per_cu = (int)value;
            return MPGNN_OK;
        default: return MPGNN_ERR_UNSUPPORTED;
    }
}
static bool get_switch(const Options& o, int32_t option, int64_t* value) {
    switch (option) {
        case MPGNN_OPT_EXACT_ORDER: *value = o.exact_order; return true;
        case MPGNN_OPT_REL_GEMM: *value = o.rel_gemm; return true;
        case MPGNN_OPT_REL_WIDE: *value = o.rel_wide; return true;
        case MPGNN_OPT_GEMM_BF3: *value = o.gemm_bf3; return true;
        case MPGNN_OPT_GEMM_IL: *value = o.gemm_il; return true;
        case MPGNN_OPT_GEMM_CU_PAIRS: *value = o.gemm_cu_pairs; return true;
        case MPGNN_OPT_BWD_FUSED: *value = o.bwd_fused; return true;
        case MPGNN_OPT_FLAT_FUSE_SPLIT: *value = o.flat_fuse_split; return true;
        case MPGNN_OPT_OUTER_VEC: *value = o.outer_vec; return true;
        case MPGNN_OPT_OUTER_SQ: *value = o.outer_sq; return true;
        case MPGNN_OPT_OUTER_RANGES: *value = o.outer_ranges; return true;
        case MPGNN_OPT_GEMM_W_IL: *value = o.gemm_w_il; return true;
        case MPGNN_OPT_GEMM_W1: *value = o.gemm_w1; return true;
        case MPGNN_OPT_OUTER_VARIANT: *value = o.outer_variant; return true;
        case MPGNN_OPT_FLAT_U: *value = o.flat_u; return true;
        case MPGNN_OPT_FLAT_PAD: *value = o.flat_pad; return true;
        case MPGNN_OPT_SINGLE_FOLD: *value = o.single_fold; return true;
        case MPGNN_OPT_BWD_SIDE_REDUCE: *value = o.side_reduce; return true;
        case MPGNN_OPT_GEMM_FIRST: *value = o.gemm_first; return true;
        case MPGNN_OPT_GEMM_SWITCH_COST: *value = o.gemm_switch_cost; return true;
        case MPGNN_OPT_FLAT_WG_PER_CU: *value = o.flat_wg_per_cu; return true;
        default: return false;
    }
}

int32_t mpgnn_set_option(int32_t option, int64_t value) {
    {
        std::lock_guard<std::mutex> lk(g_opt_mu);
        const int32_t st = set_switch(g_defaults, option, value);
        if (st != MPGNN_ERR_UNSUPPORTED) return st;
    }
    switch (option) {
        case MPGNN_OPT_TIMING_MASK: {
            std::lock_guard<std::mutex> lk(g_timing_mu);
            g_timing_mask = value;
            return MPGNN_OK;
        }
        case MPGNN_OPT_PLAN_THREADS:
            if (value < 0 || value > 256) return arg_error("MPGNN_OPT_PLAN_THREADS must be 0..256");
            g_plan_threads = (int)value;
            return MPGNN_OK;
        case MPGNN_OPT_CHUNK_ROWS:
            if (value < 32 || value > 1024 || value % 32 != 0)
                return arg_error("MPGNN_OPT_CHUNK_ROWS must be 32..1024, a multiple of 32");
            g_chunk_rows = (int)value;
            return MPGNN_OK;
        case MPGNN_OPT_ADAM_CONTRACT:
            if (value != 0 && value != 1) return arg_error("MPGNN_OPT_ADAM_CONTRACT must be 0 or 1");
            adam_contract_set((int)value);
            return MPGNN_OK;
        default:
            return arg_error("unknown option " + std::to_string(option) +
                             " (measured-slower variants of round 1 were withdrawn: DESIGN.md §4)");
    }
}

int32_t mpgnn_get_option(int32_t option, int64_t* value) {
    if (!value) return arg_error("NULL value");
    {
        std::lock_guard<std::mutex> lk(g_opt_mu);
        if (get_switch(g_defaults, option, value)) return MPGNN_OK;
    }
    switch (option) {
        case MPGNN_OPT_TIMING_MASK: {
            std::lock_guard<std::mutex> lk(g_timing_mu);
            *value = g_timing_mask;
            return MPGNN_OK;
        }
        case MPGNN_OPT_PLAN_THREADS: *value = g_plan_threads; return MPGNN_OK;
        case MPGNN_OPT_CHUNK_ROWS: *value = g_chunk_rows; return MPGNN_OK;
        case MPGNN_OPT_ADAM_CONTRACT: *value = adam_contract_get(); return MPGNN_OK;
        default: return arg_error("unknown option " + std::to_string(option));
    }
}

int32_t mpgnn_plan_set_option(mpgnn_plan* p, int32_t option, int64_t value) {
    if (!p) return arg_error("NULL plan");
    const int32_t st = set_switch(p->opt, option, value);
    if (st == MPGNN_ERR_UNSUPPORTED)
        return arg_error("option " + std::to_string(option) + " is not a per-plan switch (process-wide or build-time: mpgnn_set_option)");
    return st;
}

int32_t mpgnn_plan_get_option(const mpgnn_plan* p, int32_t option, int64_t* value) {
    if (!p || !value) return arg_error("NULL plan or value");
    if (!get_switch(p->opt, option, value))
        return arg_error("option " + std::to_string(option) + " is not a per-plan switch");
    return MPGNN_OK;
}

int32_t mpgnn_rel_mean_fwd(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R,
                           const float* x, int32_t F, float* h, void* stream) {
    int32_t st = check_common(p, F, 1);
    if (st != MPGNN_OK) return st;
    Selection s;
    if ((st = make_selection(p, mode, relation, R, &s)) != MPGNN_OK) return st;
    if (s.t_hi == s.t_lo) return MPGNN_OK;
    if (!x || !h) return arg_error("NULL x or h");
    // always in exact edge order: bit-identical to PyG's scatter_add_ mean
    hipStream_t strm = static_cast<hipStream_t>(stream);
    TimedLaunch tl(MPGNN_K_MEAN, strm);
    return run_means(p, s, x, F, h, nullptr, true, strm);
}

int32_t mpgnn_rgcn_workspace_bytes(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R,
                                   int32_t F_in, int32_t F_out, int64_t row_lo, int64_t row_hi,
                                   int64_t* bytes) {
    if (!p || !bytes) return arg_error("NULL argument");
    Selection s;
    int32_t st = make_selection(p, mode, relation, R, &s);
    if (st != MPGNN_OK) return st;
    clamp_rows(p, &row_lo, &row_hi);
    WsLayout w = ws_layout(p, mode, s, std::max(F_in, 1), std::max(F_out, 1), row_lo, row_hi,
                           root_chunks(row_lo, row_hi));
    *bytes = (int64_t)w.total;
    return MPGNN_OK;
}

int32_t mpgnn_rgcn_hsave_rows(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R, int64_t* rows) {
    if (!p || !rows) return arg_error("NULL argument");
    Selection s;
    int32_t st = make_selection(p, mode, relation, R, &s);
    if (st != MPGNN_OK) return st;
    *rows = (int64_t)(s.m_hi - s.m_lo);
    return MPGNN_OK;
}

int32_t mpgnn_rgcn_fwd_workspace_bytes(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R,
                                       int32_t F_in, int32_t F_out, int64_t row_lo, int64_t row_hi,
                                       int64_t* bytes) {
    if (!p || !bytes) return arg_error("NULL argument");
    Selection s;
    int32_t st = make_selection(p, mode, relation, R, &s);
    if (st != MPGNN_OK) return st;
    clamp_rows(p, &row_lo, &row_hi);
    WsLayout w = ws_layout(p, mode, s, std::max(F_in, 1), std::max(F_out, 1), row_lo, row_hi,
                           root_chunks(row_lo, row_hi));
    *bytes = (int64_t)w.fwd_total;
    return MPGNN_OK;
}

static int32_t rgcn_fwd_impl(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R, const float* x,
                             int32_t F_in, const float* weight, const float* root, const float* bias,
                             int32_t F_out, int64_t row_lo, int64_t row_hi, float* out, float* h_save,
                             void* workspace, int32_t act, void* stream);

int32_t mpgnn_rgcn_fwd(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R, const float* x,
                       int32_t F_in, const float* weight, const float* root, const float* bias,
                       int32_t F_out, int64_t row_lo, int64_t row_hi, float* out, float* h_save,
                       void* workspace, void* stream) {
    return rgcn_fwd_impl(p, mode, relation, R, x, F_in, weight, root, bias, F_out, row_lo, row_hi, out, h_save,
                         workspace, MPGNN_ACT_NONE, stream);
}

int32_t mpgnn_rgcn_fwd_act(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R, const float* x,
                           int32_t F_in, const float* weight, const float* root, const float* bias,
                           int32_t F_out, float* out, float* h_save, void* workspace, int32_t act,
                           void* stream) {
    if (act != MPGNN_ACT_NONE && act != MPGNN_ACT_RELU) return arg_error("unknown activation");
    if (p && (p->shard_lo != 0 || p->shard_hi != p->N))
        return arg_error("fused activation needs an unsharded plan (sharded outputs are partial sums)");
    return rgcn_fwd_impl(p, mode, relation, R, x, F_in, weight, root, bias, F_out, 0, p ? p->N : 0, out, h_save,
                         workspace, act, stream);
}

}  // extern "C"

static int32_t rgcn_fwd_impl(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R, const float* x,
                             int32_t F_in, const float* weight, const float* root, const float* bias,
                             int32_t F_out, int64_t row_lo, int64_t row_hi, float* out, float* h_save,
                             void* workspace, int32_t act, void* stream) {
    int32_t st = check_common(p, F_in, F_out);
    if (st != MPGNN_OK) return st;
    Selection s;
    if ((st = make_selection(p, mode, relation, R, &s)) != MPGNN_OK) return st;
    if (p->N == 0) return MPGNN_OK;
    if (!x || !weight || !out) return arg_error("NULL x, weight or out");
    if (!workspace) return arg_error("NULL workspace");
    clamp_rows(p, &row_lo, &row_hi);
    hipStream_t strm = static_cast<hipStream_t>(stream);
    const RootChunks rc = root_chunks(row_lo, row_hi);
    const WsLayout w = ws_layout(p, mode, s, F_in, F_out, row_lo, row_hi, rc);
    char* ws = static_cast<char*>(workspace);
    float* Y = reinterpret_cast<float*>(ws + w.y);
    float* Yroot = root ? reinterpret_cast<float*>(ws + w.yroot) : nullptr;
    const Options& o = p->opt;
    const bool exact = o.exact_order;
    const bool own_range = row_lo == p->shard_lo && row_hi == p->shard_hi;
    // Mode SINGLE, unsharded, F_in ∈ {64, 128}, F_out = 128: ONE fused GEMM per layer,
    //   out[i] = act([x_i | mean_i] @ [root; W] + bias)   (K = 2·F_in; mean_i = 0 without a segment)
    // — a node has at most one segment of the relation, so the transform, the root term, the
    // combine and the activation of mp_rgcn_layer.py:245-268 (+ model.py:211,214) need no Y,
    // Y_root or combine pass.
    const bool cat = mode == MPGNN_MODE_SINGLE && !exact && o.rel_gemm && root != nullptr &&
                     (F_in == 64 || F_in == 128) && F_out == 128 && row_lo == 0 && row_hi == p->N &&
                     p->shard_lo == 0 && p->shard_hi == p->N && p->N <= INT32_MAX - 1;
    // the relation's node map: the plan's (absent relation: its zero row), else built per call
    auto relation_node_map = [&](const int** nmap) -> int32_t {
        if (!p->node_maps_tried) {  // first unsharded fused mode-SINGLE call: every relation's map
            hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
            if (hipStreamIsCapturing(strm, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone) {
                std::lock_guard<std::mutex> lk(p->node_map_mu);
                if (!p->node_maps_tried) {
                    const int32_t e = build_rel_node_maps(const_cast<mpgnn_plan*>(p), strm);
                    p->node_maps_tried = true;
                    if (e != MPGNN_OK) return e;
                }
            }
        }
        if (p->d.rel_node_map != nullptr) {
            *nmap = p->d.rel_node_map + (size_t)(s.d_hi > s.d_lo ? s.d_lo : p->nrel) * (size_t)p->N;
            return MPGNN_OK;
        }
        int* m = reinterpret_cast<int*>(ws + w.nmap);
        TimedLaunch tl(MPGNN_K_ROW_FWD, strm);
        int32_t e = hip_check(hipMemsetAsync(m, 0, (size_t)p->N * sizeof(int), strm), "memset node map");
        if (e != MPGNN_OK) return e;
        if (s.sel_e > s.sel_b) {
            hipLaunchKernelGGL(node_map_kernel, dim3((s.sel_e - s.sel_b + kThreads - 1) / kThreads), dim3(kThreads), 0,
                               strm, p->d.s_row, p->d.s_src, s.sel_b, s.sel_e, m);
            if ((e = hip_check(hipGetLastError(), "node_map_kernel launch")) != MPGNN_OK) return e;
        }
        *nmap = m;
        return MPGNN_OK;
    };
    // Mode SINGLE, F_in = F_out = 256 (the wide B-stationary GEMM; K = 512 of the fused layer would
    // not fit the weight slice in registers), unsharded: the root items' epilogue finishes every
    // row without a segment of the relation — act((0 + x_i @ root) + bias) straight into out (87 %
    // of C5's rows) — and single_fix_kernel adds Y to the rows with one: no Y_root buffer, no
    // combine pass over all N rows.
    const bool root_epi = mode == MPGNN_MODE_SINGLE && !exact && o.rel_gemm && o.rel_wide && root != nullptr &&
                          F_in == 256 && F_out == 256 && row_lo == 0 && row_hi == p->N && p->shard_lo == 0 &&
                          p->shard_hi == p->N && p->N <= INT32_MAX - 1;
    if (root_epi) {
        float* H = h_save ? h_save : reinterpret_cast<float*>(ws + w.hf);
        {
            TimedLaunch tl(MPGNN_K_MEAN, strm);
            st = run_means_multi(p, s, x, F_in, H, reinterpret_cast<float*>(ws + w.pseg), exact, strm);
            if (st != MPGNN_OK) return st;
        }
        const int* nmap = nullptr;
        if ((st = relation_node_map(&nmap)) != MPGNN_OK) return st;
        st = run_seg(p, mode, s, 2, x, F_in, weight, root, 0, F_out, Y, out, row_lo, row_hi, nullptr, nullptr, true,
                     MPGNN_K_SEG_FWD, strm, H, nmap, bias, act == MPGNN_ACT_RELU ? 1 : 0);
        if (st != MPGNN_OK || s.sel_e <= s.sel_b) return st;
        TimedLaunch tl(MPGNN_K_ROW_FWD, strm);
        hipLaunchKernelGGL(single_fix_kernel, dim3((unsigned)std::min<int64_t>((s.sel_e - s.sel_b + kWaves - 1) / kWaves, 1 << 20)),
                           dim3(kThreads), 0, strm, Y, p->d.s_row, (int)s.sel_b, (int)s.sel_e, bias, F_out,
                           act == MPGNN_ACT_RELU ? 1 : 0, out);
        return hip_check(hipGetLastError(), "single_fix_kernel launch");
    }
    if (cat) {
        float* H = h_save ? h_save : reinterpret_cast<float*>(ws + w.hf);
        const int* nmap = nullptr;
        if ((st = relation_node_map(&nmap)) != MPGNN_OK) return st;
        if (o.gemm_bf3) {  // split-K layer on the bf16 matrix cores
            SingleBf3Args sa{};
            sa.x = x;
            sa.H = H;
            sa.node_map = nmap;
            sa.m_lo = s.m_lo;
            sa.m_rows = std::max(s.m_hi - s.m_lo, 1);
            sa.N = (int)p->N;
            sa.W = weight;
            sa.root = root;
            sa.bias = bias;
            sa.relu = act == MPGNN_ACT_RELU;
            sa.out = out;
            const int n_gi = (int)((p->N + 31) / 32);
            if (o.single_fold) {  // the means inside the layer's GEMM launch (no means launch)
                sa.m_ptr = p->d.m_ptr;
                sa.em_col = p->d.em_col;
                sa.m_cnt = p->d.m_cnt;
                sa.H_out = h_save;
            } else {
                TimedLaunch tl(MPGNN_K_MEAN, strm);
                st = run_means_multi(p, s, x, F_in, H, reinterpret_cast<float*>(ws + w.pseg), exact, strm);
                if (st != MPGNN_OK) return st;
            }
            const int grid = (int)std::min<int64_t>(n_gi, cu_count());
            TimedLaunch tl(MPGNN_K_SEG_FWD, strm);
            if (F_in == 64)
                hipLaunchKernelGGL(single_bf3_kernel<1>, dim3(grid), dim3(kSingleThreads), SingleBf3<1>::lds_bytes(), strm, sa);
            else
                hipLaunchKernelGGL(single_bf3_kernel<2>, dim3(grid), dim3(kSingleThreads), SingleBf3<2>::lds_bytes(), strm, sa);
            return hip_check(hipGetLastError(), "single_bf3_kernel launch");
        }
        {
            TimedLaunch tl(MPGNN_K_MEAN, strm);
            st = run_means_multi(p, s, x, F_in, H, reinterpret_cast<float*>(ws + w.pseg), exact, strm);
            if (st != MPGNN_OK) return st;
        }
        RelGemmArgs r{};
        r.n_rel = 0;
        r.n_root = (int)((p->N + 31) / 32);
        r.Arel = H;
        r.Aroot = x;
        r.m_lo = s.m_lo;
        r.m_rows = std::max(s.m_hi - s.m_lo, 1);
        r.node_map = nmap;
        r.W = weight;
        r.Wroot = root;
        r.Yroot = out;
        r.row_lo = 0;
        r.row_hi = (int)p->N;
        r.bias = bias;
        r.relu = act == MPGNN_ACT_RELU;
        TimedLaunch tl(MPGNN_K_SEG_FWD, strm);
        if (F_in == 64) launch_rel_gemm_cat<2>(r, strm);
        else launch_rel_gemm_cat<4>(r, strm);
        return hip_check(hipGetLastError(), "rel_gemm_kernel (fused mode SINGLE) launch");
    }
    {
        // 1) Hm[m] = mean(x over multi-edge segment m)  (the saved means when training); a
        //    single-edge segment's mean is its x row, read by the GEMM through s_src
        float* H = h_save ? h_save : reinterpret_cast<float*>(ws + w.hf);
#ifdef MPGNN_PROBE_OVERLAP
        // PROBE BUILD ONLY (scripts/r06_probe_overlap.sh; never the product library): the means on a
        // side stream CONCURRENT with the whole transform GEMM, which then reads stale Hm rows — WRONG
        // results. Bounds what running the means beside the GEMM's Hm-free items could save
        // (VERDICT r5 item 1). MPGNN_PROBE_OVERLAP = 1: means launched first; 2: the GEMM first.
        {
            static hipStream_t side = nullptr;
            static hipEvent_t e0 = nullptr, e1 = nullptr;
            if (side == nullptr) {
                (void)hipStreamCreateWithFlags(&side, hipStreamNonBlocking);
                (void)hipEventCreateWithFlags(&e0, hipEventDisableTiming);
                (void)hipEventCreateWithFlags(&e1, hipEventDisableTiming);
            }
            (void)hipEventRecord(e0, strm);
            (void)hipStreamWaitEvent(side, e0, 0);
            if (MPGNN_PROBE_OVERLAP == 1)
                st = run_means_multi(p, s, x, F_in, H, reinterpret_cast<float*>(ws + w.pseg), exact, side);
            if (st != MPGNN_OK) return st;
            st = run_seg(p, mode, s, 2, x, F_in, weight, root, 0, F_out, Y, Yroot, row_lo, row_hi, nullptr, nullptr,
                         true, MPGNN_K_SEG_FWD, strm, H);
            if (st != MPGNN_OK) return st;
            if (MPGNN_PROBE_OVERLAP == 2)
                st = run_means_multi(p, s, x, F_in, H, reinterpret_cast<float*>(ws + w.pseg), exact, side);
            if (st != MPGNN_OK) return st;
            (void)hipEventRecord(e1, side);
            (void)hipStreamWaitEvent(strm, e1, 0);
        }
#else
        {
            TimedLaunch tl(MPGNN_K_MEAN, strm);
            st = run_means_multi(p, s, x, F_in, H, reinterpret_cast<float*>(ws + w.pseg), exact, strm);
            if (st != MPGNN_OK) return st;
        }
        // 2) Y[seg] = mean(seg) @ W_rel(seg); Yroot[i] = x[i] @ root   (MFMA tiles)
        st = run_seg(p, mode, s, 2, x, F_in, weight, root, 0, F_out, Y, Yroot, row_lo, row_hi, nullptr, nullptr, true,
                     MPGNN_K_SEG_FWD, strm, H);
        if (st != MPGNN_OK) return st;
#endif
    }

    // 2) out[i] = (Σ_{seg of row i, relation order} Y[seg] + Yroot[i]) + bias
    RowSumArgs a{};
    a.N = (int)p->N;
    a.g.src = Y;
    a.g.F = F_out;
    a.extra = Yroot;
    a.bias = bias;
    a.lo = (int)row_lo;
    a.hi = (int)row_hi;
    a.out = out;
    int k_lo = 0, k_hi = 0;
    if (mode == MPGNN_MODE_ALL && !exact && Yroot != nullptr && own_range) {
        // augmented row-major list: Σ_r Y + Y_root per own row, + bias at the flush
        if (row_lo != 0 || row_hi != p->N) {  // rows outside the shard may have no entry
            st = hip_check(hipMemsetAsync(out, 0, (size_t)p->N * F_out * sizeof(float), strm), "memset out");
            if (st != MPGNN_OK) return st;
        }
        FlatRun f{};
        f.wg_per_cu = p->opt.flat_wg_per_cu;
        f.u = p->opt.flat_u;
        f.plan = p;
        f.fd = &p->d.rwx_f;
        f.max_pieces = p->rwx_f.max_pieces;
        f.ngroups = p->rwx_f.ngroups;
        f.g_lo = 0;
        f.g_hi = p->rwx_f.ngroups;
        f.k_lo = 0;
        f.k_hi = p->rwx_f.nsplit;
        f.table = p->d.rwx_val;
        f.idx_off = s.sel_b;
        f.filter = !s.all_segments;
        f.flo = s.sel_b;
        f.fhi = s.sel_e;
        f.src = Y;
        f.F = F_out;
        f.row_off = 0;
        f.out = out;
        f.carry = reinterpret_cast<float*>(ws + w.prw);
        f.final_mode = 0;
        f.extra = Yroot;
        f.bias = bias;
        f.lo = (int)row_lo;
        f.hi = (int)row_hi;
        f.relu = act == MPGNN_ACT_RELU;
        TimedLaunch tl(MPGNN_K_ROW_FWD, strm);
        return run_flat(f, strm);
    }
    if (mode == MPGNN_MODE_ALL && !exact) {
        FlatRun f{};
        f.wg_per_cu = p->opt.flat_wg_per_cu;
        f.u = p->opt.flat_u;
        f.plan = p;
        f.fd = &p->d.rw_f;
        f.max_pieces = p->rw_f.max_pieces;
        f.ngroups = p->rw_f.ngroups;
        f.g_lo = 0;
        f.g_hi = p->rw_f.ngroups;
        f.table = p->d.rw_seg;
        f.idx_off = s.sel_b;
        f.filter = !s.all_segments;
        f.flo = s.sel_b;
        f.fhi = s.sel_e;
        f.src = Y;
        f.F = F_out;
        f.row_off = 0;
        f.out = out;
        f.carry = reinterpret_cast<float*>(ws + w.prw);
        f.final_mode = 1;
        f.row_ptr = p->d.rw_ptr;
        f.r_lo = 0;
        f.r_hi = (int)p->N;
        f.extra = Yroot;
        f.bias = bias;
        f.lo = (int)row_lo;
        f.hi = (int)row_hi;
        f.relu = act == MPGNN_ACT_RELU;
        TimedLaunch tl(MPGNN_K_ROW_FWD, strm);
        return run_flat(f, strm);
    }
    if (mode == MPGNN_MODE_ALL) {
        const bool ragged = !exact && p->rw_l.npieces > 0;
        a.list_kind = 0;
        a.ptr = ragged ? p->d.rw_ent_ptr : p->d.rw_ptr;
        a.g.ent = ragged ? p->d.rw_ent : nullptr;
        a.res = p->d.rw_res;
        a.g.idx = p->d.rw_seg;
        a.g.idx_off = s.sel_b;
        a.g.filter = !s.all_segments;
        a.g.flo = s.sel_b;
        a.g.fhi = s.sel_e;
        if (ragged) k_hi = (int)(size_t)p->rw_l.npieces;
    } else if (!exact && F_out % 4 == 0 && p->N > 0) {
        int* m = reinterpret_cast<int*>(ws + w.nmap);
        TimedLaunch tl(MPGNN_K_ROW_FWD, strm);
        if ((st = hip_check(hipMemsetAsync(m, 0xFF, (size_t)p->N * sizeof(int), strm), "memset segment map"))) return st;
        if (s.sel_e > s.sel_b)
            hipLaunchKernelGGL(seg_map_kernel, dim3((s.sel_e - s.sel_b + kThreads - 1) / kThreads), dim3(kThreads), 0, strm,
                               p->d.s_row, (int)s.sel_b, (int)s.sel_e, m);
        hipLaunchKernelGGL(single_combine_kernel, dim3((unsigned)std::min<int64_t>((p->N + kWaves - 1) / kWaves, 1 << 20)),
                           dim3(kThreads), 0, strm, Y, Yroot, bias, m, (int)p->N, F_out, (int)row_lo, (int)row_hi,
                           act == MPGNN_ACT_RELU ? 1 : 0, out);
        return hip_check(hipGetLastError(), "single_combine_kernel launch");
    } else {
        a.list_kind = 1;  // at most one segment per row: no pieces
        a.keys = p->d.s_row;
        a.kb = s.sel_b;
        a.ke = s.sel_e;
        a.g.idx_off = s.sel_b;
    }
    {
        TimedLaunch tl(MPGNN_K_ROW_FWD, strm);
        st = run_rowsum(p, a, p->d.rw_pb, p->d.rw_pe, k_lo, k_hi, reinterpret_cast<float*>(ws + w.prw), strm);
        if (st != MPGNN_OK) return st;
    }
    if (act == MPGNN_ACT_RELU) {
        const size_t n = (size_t)p->N * F_out;
        hipLaunchKernelGGL(relu_kernel, dim3((unsigned)std::min<size_t>((n + kThreads - 1) / kThreads, 4096)),
                           dim3(kThreads), 0, strm, out, n);
        return hip_check(hipGetLastError(), "relu_kernel launch");
    }
    return MPGNN_OK;
}

// grad_x-style transposed gather: dx[j] = Σ_{edges (i, r, j) of the selection} G[seg] (+ Groot[j]
// for own rows), over the flat / ragged / mode-SINGLE lists (used by mpgnn_rgcn_bwd and
// mpgnn_rel_mean_bwd).
// Where the piece counters of the augmented transposed list live in the carry region Pdx (F_in
// floats per slot), 16-byte aligned; split_counter_bytes(p) of them.
static unsigned* split_counters(const mpgnn_plan* p, float* Pdx, int F_in) {
    return reinterpret_cast<unsigned*>(reinterpret_cast<char*>(Pdx) + align16((size_t)p->tx_f.nslots * F_in * sizeof(float)));
}

static int32_t run_grad_x(const mpgnn_plan* p, int32_t mode, const Selection& s, const float* G, const float* Groot,
                          int F_in, int64_t row_lo, int64_t row_hi, float* grad_x, float* Pdx, bool exact,
                          hipStream_t strm, bool counters_zeroed = false, const float* mask = nullptr) {
    int32_t st = MPGNN_OK;
    bool masked = mask == nullptr;  // the mask applied (fused into the flat list's row finish)
    RowSumArgs a{};
    a.N = (int)p->N;
    a.g.src = G;
    a.g.F = F_in;
    a.g.idx_off = s.sel_b;
    a.extra = Groot;
    a.bias = nullptr;
    a.lo = (int)row_lo;
    a.hi = (int)row_hi;
    a.out = grad_x;
    int k_lo = 0, k_hi = 0;
    const int *pb = nullptr, *pe = nullptr;
    const bool own_range = row_lo == p->shard_lo && row_hi == p->shard_hi;
    if (mode == MPGNN_MODE_ALL && !exact && Groot != nullptr && own_range) {
        // augmented transposed list: Σ G + G_root per own row
        if (row_lo != 0 || row_hi != p->N) {
            st = hip_check(hipMemsetAsync(grad_x, 0, (size_t)p->N * F_in * sizeof(float), strm), "memset grad_x");
            if (st != MPGNN_OK) return st;
        }
        FlatRun f{};
        f.wg_per_cu = p->opt.flat_wg_per_cu;
        f.u = p->opt.flat_u;
        // no padded slot tables here: the transposed lists are mostly long groups (measured +0.5 µs)
        f.fd = &p->d.tx_f;
        f.max_pieces = p->tx_f.max_pieces;
        f.ngroups = p->tx_f.ngroups;
        f.g_lo = 0;
        f.g_hi = p->tx_f.ngroups;
        f.k_lo = 0;
        f.k_hi = p->tx_f.nsplit;
        f.table = p->d.tx_val;
        f.idx_off = s.sel_b;
        f.filter = !s.all_segments;
        f.flo = s.sel_b;
        f.fhi = s.sel_e;
        f.src = G;
        f.F = F_in;
        f.row_off = 0;
        f.out = grad_x;
        f.carry = Pdx;
        f.final_mode = 0;
        f.extra = Groot;
        f.lo = (int)row_lo;
        f.hi = (int)row_hi;
        f.mask = mask;
        masked = true;
        TimedLaunch tl(MPGNN_K_ROW_DX, strm);
        if (p->opt.flat_fuse_split && p->tx_f.nsplit > 0) {
            // piece counters behind the carry slots (ws_layout reserves them in the pdx region)
            // 16-byte aligned start and length: one fill launch (a ragged memset is two)
            f.arrive = split_counters(p, Pdx, F_in);
            if (!counters_zeroed) {  // else zeroed by the dgrad launch before this one (grad_x_part)
                st = hip_check(hipMemsetAsync(f.arrive, 0, split_counter_bytes(p), strm), "memset split counters");
                if (st != MPGNN_OK) return st;
            }
        }
        st = run_flat(f, strm);
        if (st != MPGNN_OK) return st;
    } else if (mode == MPGNN_MODE_ALL && !exact) {
        FlatRun f{};
        f.wg_per_cu = p->opt.flat_wg_per_cu;
        f.u = p->opt.flat_u;
        // no padded slot tables here: the transposed lists are mostly long groups (measured +0.5 µs)
        f.fd = &p->d.t_f;
        f.max_pieces = p->t_f.max_pieces;
        f.ngroups = p->t_f.ngroups;
        f.g_lo = 0;
        f.g_hi = p->t_f.ngroups;
        f.table = p->d.t_seg;
        f.idx_off = s.sel_b;
        f.filter = !s.all_segments;
        f.flo = s.sel_b;
        f.fhi = s.sel_e;
        f.src = G;
        f.F = F_in;
        f.row_off = 0;
        f.out = grad_x;
        f.carry = Pdx;
        f.final_mode = 1;
        f.row_ptr = p->d.t_ptr;
        f.r_lo = 0;
        f.r_hi = (int)p->N;
        f.extra = Groot;
        f.lo = (int)row_lo;
        f.hi = (int)row_hi;
        TimedLaunch tl(MPGNN_K_ROW_DX, strm);
        st = run_flat(f, strm);
        if (st != MPGNN_OK) return st;
    } else if (mode == MPGNN_MODE_ALL) {
        const bool ragged = !exact && p->t_l.npieces > 0 && s.sel_e > s.sel_b;
        a.list_kind = 0;
        a.ptr = ragged ? p->d.t_ent_ptr : p->d.t_ptr;
        a.g.ent = ragged ? p->d.t_ent : nullptr;
        a.res = p->d.t_res;
        a.g.idx = p->d.t_seg;
        a.g.filter = !s.all_segments;
        a.g.flo = s.sel_b;
        a.g.fhi = s.sel_e;
        if (ragged) {
            pb = p->d.t_pb;
            pe = p->d.t_pe;
            k_hi = (int)(size_t)p->t_l.npieces;
        }
    } else {
        a.list_kind = 1;
        a.g.idx = p->d.ta_seg;
        if (!exact) {
            a.keys = p->d.ta_key;
            a.kb = s.ta_e_lo;
            a.ke = s.ta_e_hi;
            a.g.ent = p->d.ta_ent;
            a.res = p->d.ta_res;
            pb = p->d.ta_pb;
            pe = p->d.ta_pe;
            k_lo = s.tap_lo;
            k_hi = s.tap_hi;
        } else {
            a.keys = p->d.ta_col;
            a.kb = (s.d_hi > s.d_lo) ? p->rel_edge_ptr[s.d_lo] : 0;
            a.ke = (s.d_hi > s.d_lo) ? p->rel_edge_ptr[s.d_hi] : 0;
        }
    }
    if (!(mode == MPGNN_MODE_ALL && !exact)) {
        TimedLaunch tl(MPGNN_K_ROW_DX, strm);
        st = run_rowsum(p, a, pb, pe, k_lo, k_hi, Pdx, strm);
        if (st != MPGNN_OK) return st;
    }
    if (!masked) {  // the other lists: the ReLU backward as one in-place pass after them
        const int64_t n = (int64_t)p->N * F_in;
        const int vec = ((reinterpret_cast<uintptr_t>(grad_x) | reinterpret_cast<uintptr_t>(mask)) & 15) == 0;
        hipLaunchKernelGGL(relu_bwd_kernel, dim3((unsigned)std::min<int64_t>((n + kThreads - 1) / kThreads, 4096)),
                           dim3(kThreads), 0, strm, grad_x, mask, n, grad_x, vec);
        return hip_check(hipGetLastError(), "relu_bwd_kernel (grad_x mask) launch");
    }
    return MPGNN_OK;
}

// Workspace of mpgnn_rel_mean_bwd: G = dh / cnt (S_sel × F), then the gather's carry slots.
static void mean_bwd_layout(const mpgnn_plan* p, int32_t mode, const Selection& s, int F, size_t* off_pdx,
                            size_t* total) {
    const size_t S_sel = (size_t)(s.sel_e - s.sel_b);
    const size_t seg_slots = std::max((size_t)(s.sp_hi - s.sp_lo), (size_t)p->seg_f.nslots);
    const size_t dx_pieces = (mode == MPGNN_MODE_ALL)
                                 ? std::max({(size_t)p->t_l.npieces, (size_t)p->t_f.nslots, (size_t)p->tx_f.nslots})
                                 : (size_t)(s.tap_hi - s.tap_lo);
    *off_pdx = align256(S_sel * F * sizeof(float));
    *total = std::max<size_t>(*off_pdx + align256(std::max(dx_pieces, seg_slots) * F * sizeof(float)), 256);
}

extern "C" {

int32_t mpgnn_rel_mean_bwd_workspace_bytes(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R, int32_t F,
                                           int64_t* bytes) {
    if (!p || !bytes) return arg_error("NULL argument");
    Selection s;
    int32_t st = make_selection(p, mode, relation, R, &s);
    if (st != MPGNN_OK) return st;
    size_t off, total;
    mean_bwd_layout(p, mode, s, std::max(F, 1), &off, &total);
    *bytes = (int64_t)total;
    return MPGNN_OK;
}

int32_t mpgnn_rel_mean_bwd(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R, const float* dh, int32_t F,
                           float* dx, void* workspace, void* stream) {
    int32_t st = check_common(p, F, F);
    if (st != MPGNN_OK) return st;
    Selection s;
    if ((st = make_selection(p, mode, relation, R, &s)) != MPGNN_OK) return st;
    if (p->N == 0) return MPGNN_OK;
    if (!dx || !workspace || (s.sel_e > s.sel_b && !dh)) return arg_error("NULL dh, dx or workspace");
    hipStream_t strm = static_cast<hipStream_t>(stream);
    if (s.sel_e == s.sel_b)
        return hip_check(hipMemsetAsync(dx, 0, (size_t)p->N * F * sizeof(float), strm), "memset dx");
    size_t off_pdx, total;
    mean_bwd_layout(p, mode, s, F, &off_pdx, &total);
    char* ws = static_cast<char*>(workspace);
    float* G = reinterpret_cast<float*>(ws);
    const int rows = s.sel_e - s.sel_b;
    const size_t n = (size_t)rows * F;
    hipLaunchKernelGGL(scale_rows_kernel, dim3((unsigned)std::min<size_t>((n + kThreads - 1) / kThreads, 8192)),
                       dim3(kThreads), 0, strm, dh, p->d.s_cnt, s.sel_b, rows, F, G);
    if ((st = hip_check(hipGetLastError(), "scale_rows_kernel launch")) != MPGNN_OK) return st;
    TimedLaunch tl(MPGNN_K_ROW_DX, strm);
    return run_grad_x(p, mode, s, G, nullptr, F, p->shard_lo, p->shard_hi, dx,
                      reinterpret_cast<float*>(ws + off_pdx), p->opt.exact_order, strm);
}


static int32_t bwd_params(const mpgnn_plan* p, int32_t mode, int32_t R, const float* x, int32_t F_in, int32_t F_out,
                          const float* h_save, const float* grad_out, float* grad_weight, float* grad_root,
                          float* grad_bias, const Selection& s, const WsLayout& w, const RootChunks& rc, char* ws,
                          hipStream_t strm, bool acc, hipStream_t side = nullptr, hipEvent_t ev_fork = nullptr,
                          hipEvent_t ev_join = nullptr, bool* forked = nullptr);


// The backward at F_in = F_out = 128 through bwd_bf3_kernel (dgrad + dW / droot / dbias in one
// launch) + reduce_slabs3_kernel + grad_x. Returns MPGNN_ERR_UNSUPPORTED (nothing launched) when
// its slab layout is not cached and cannot be made now (graph capture): the caller falls back.
static int32_t bwd_fused(const mpgnn_plan* p, int32_t mode, int32_t R, const float* x, const float* weight,
                         const float* root, const float* h_save, const float* grad_out, int64_t row_lo, int64_t row_hi,
                         float* grad_x, float* grad_weight, float* grad_root, float* grad_bias, const Selection& s,
                         const WsLayout& w, char* ws, hipStream_t strm, const float* gx_mask) {
    const int n_rel = s.t32_hi - s.t32_lo;
    const int n_root = (int)((row_hi - row_lo + 31) / 32);
    const int n_items = n_rel + n_root;
    if (n_root == 0) return MPGNN_ERR_UNSUPPORTED;
    const int G = std::min(n_items, cu_count());
    // one workgroup per CU walks its items with the next item's rows in flight: few items per
    // workgroup (C3 mode SINGLE: 3) it saves the second launch and gather (epoch 0.74 -> 0.69 ms);
    // at C3 mode ALL (29 items per workgroup) the two launches at two workgroups per CU are
    // faster (epoch 1.17 vs 1.30 ms) — measured, the split point is conservative
    if (n_items > 4 * cu_count()) return MPGNN_ERR_UNSUPPORTED;
    const int64_t nd = s.d_hi - s.d_lo;
    // ---- slab layout (host: every workgroup's item range, runs of one weight) ----
    const std::array<int64_t, 8> key{mode, s.t32_lo, s.t32_hi, s.d_lo, s.d_hi, row_lo, row_hi, G};
    mpgnn_plan::BwSlabs lay;
    {
        std::lock_guard<std::mutex> lk(p->bw_mu);
        auto it = p->bw_slabs.find(key);
        if (it != p->bw_slabs.end()) {
            lay = it->second;
        } else {
            hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
            if (hipStreamIsCapturing(strm, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone)
                return MPGNN_ERR_UNSUPPORTED;
            std::vector<int> wkey(n_items);
            for (int i = 0; i < n_items; ++i) {
                if (i >= n_rel) {
                    wkey[i] = -1;  // root
                } else if (mode != MPGNN_MODE_ALL) {
                    wkey[i] = 0;   // one weight
                } else {
                    const int t = s.t32_lo + i;
                    wkey[i] = (int)(std::upper_bound(p->rel_t32_ptr.begin(), p->rel_t32_ptr.end(), t) -
                                    p->rel_t32_ptr.begin()) - 1;
                }
            }
            // workgroup blockIdx g holds the rng(g)-th consecutive item range (bw_range); slabs are
            // numbered in item order, so each weight's slabs are contiguous (relations, then root)
            std::vector<int> tab((size_t)G + (size_t)p->nrel + 1, 0), skey, perm(G);
            for (int g = 0; g < G; ++g) {
                const int gx = g & 7, q = G >> 3, rem = G & 7;
                perm[gx * q + std::min(gx, rem) + (g >> 3)] = g;
            }
            int ns = 0;
            for (int rg = 0; rg < G; ++rg) {
                const int ib = (int)((long long)rg * n_items / G), ie = (int)((long long)(rg + 1) * n_items / G);
                tab[perm[rg]] = ns;
                for (int i = ib; i < ie; ++i)
                    if (i == ib || wkey[i] != wkey[i - 1]) {
                        skey.push_back(wkey[i]);
                        ++ns;
                    }
            }
            int root_lo = ns;
            for (int k = 0; k < ns; ++k)
                if (skey[k] < 0) {
                    root_lo = k;
                    break;
                }
            // relation slab ranges, indexed by absolute dense relation (reduce_slabs_body's gptr)
            int* rp = tab.data() + G;
            int k = 0;
            for (int64_t d = 0; d <= p->nrel; ++d) {
                while (k < root_lo && skey[k] < d) ++k;
                rp[d] = k;
            }
            int* dev = nullptr;
            if (hipMalloc(&dev, tab.size() * sizeof(int)) != hipSuccess) {
                (void)hipGetLastError();
                return MPGNN_ERR_UNSUPPORTED;
            }
            if (hipMemcpy(dev, tab.data(), tab.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) {
                (void)hipGetLastError();
                (void)hipFree(dev);
                return MPGNN_ERR_UNSUPPORTED;
            }
            lay.dev = dev;
            lay.n_slabs = ns;
            lay.root_lo = root_lo;
            p->bw_slabs[key] = lay;
        }
    }
    if ((size_t)lay.n_slabs * 128 * 128 * sizeof(float) > w.bwb - w.bw) return MPGNN_ERR_UNSUPPORTED;
    float* slabs = reinterpret_cast<float*>(ws + w.bw);
    float* bslabs = reinterpret_cast<float*>(ws + w.bwb);
    int32_t st = MPGNN_OK;
    if (mode == MPGNN_MODE_ALL && nd != (int64_t)R) {  // weight ids without a relation of the plan: zeros
        if ((st = hip_check(hipMemsetAsync(grad_weight, 0, (size_t)std::max(R, 0) * 128 * 128 * sizeof(float), strm),
                            "memset grad_weight")) != MPGNN_OK)
            return st;
    }
    BwdArgs A{};
    RelGemmArgs& r = A.g;
    r.t_begin = p->d.t32_begin;
    r.t_end = p->d.t32_end;
    r.t_lo = s.t32_lo;
    r.n_rel = n_rel;
    r.n_root = n_root;
    r.Aroot = grad_out;
    r.s_src = p->d.s_src;
    r.m_lo = s.m_lo;
    r.s_row = p->d.s_row;
    r.s_cnt = p->d.s_cnt;
    r.s_rel = p->d.s_rel;
    r.W = weight;
    r.w_per_rel = (mode == MPGNN_MODE_ALL);
    r.Wroot = root;
    r.Y = grad_x != nullptr ? reinterpret_cast<float*>(ws + w.g) : nullptr;
    r.Yroot = grad_x != nullptr ? reinterpret_cast<float*>(ws + w.groot) : nullptr;
    r.sel_b = s.sel_b;
    r.row_lo = (int)row_lo;
    r.row_hi = (int)row_hi;
    A.x = x;
    A.Hm = h_save;
    A.slabs = slabs;
    A.bslabs = bslabs;
    A.wg_slab0 = lay.dev;
    {
        TimedLaunch tl(MPGNN_K_OUTER, strm);
        hipLaunchKernelGGL(bwd_bf3_kernel, dim3(G), dim3(kBwThreads), kBwLds, strm, A);
        if ((st = hip_check(hipGetLastError(), "bwd_bf3_kernel launch")) != MPGNN_OK) return st;
    }
    {
        ReduceArgs r3[3] = {};
        int gx[3] = {0, 0, 0};
        // weights: mode ALL one group per selected dense relation (its contiguous slab range),
        // mode SINGLE one group (every relation slab)
        r3[0].P = slabs;
        r3[0].elems = 128 * 128;
        r3[0].dst = grad_weight;
        if (mode == MPGNN_MODE_ALL) {
            r3[0].gptr = lay.dev + G;
            r3[0].g_base = (int)s.d_lo;
            r3[0].gdst = p->d.rel_val32;
            gx[0] = (int)nd;
        } else {
            r3[0].nchunks = lay.root_lo;
            gx[0] = 1;
        }
        r3[1].P = slabs + (size_t)lay.root_lo * 128 * 128;
        r3[1].elems = 128 * 128;
        r3[1].nchunks = lay.n_slabs - lay.root_lo;
        r3[1].dst = grad_root;
        gx[1] = grad_root != nullptr ? 1 : 0;
        r3[2].P = bslabs + (size_t)lay.root_lo * 128;
        r3[2].elems = 128;
        r3[2].nchunks = lay.n_slabs - lay.root_lo;
        r3[2].dst = grad_bias;
        gx[2] = grad_bias != nullptr ? 1 : 0;
        ZeroList zl{};
        TimedLaunch tl(MPGNN_K_REDUCE, strm);
        hipLaunchKernelGGL(reduce_slabs3_kernel, dim3(gx[0] + gx[1] + gx[2], (128 * 128 + kThreads - 1) / kThreads),
                           dim3(kThreads), 0, strm, r3[0], r3[1], r3[2], gx[0], gx[1], gx[2], zl);
        if ((st = hip_check(hipGetLastError(), "reduce_slabs3_kernel launch")) != MPGNN_OK) return st;
    }
    if (grad_x != nullptr)
        st = run_grad_x(p, mode, s, reinterpret_cast<float*>(ws + w.g), reinterpret_cast<float*>(ws + w.groot), 128,
                        row_lo, row_hi, grad_x, reinterpret_cast<float*>(ws + w.pdx), false, strm, false, gx_mask);
    return st;
}

// A side stream of the current device for this host thread, with a fork / join event pair, made
// once (outside captures: false there until made). Per thread, so concurrent callers never share
// events.
static bool side_stream(hipStream_t* side, hipEvent_t* ev_fork, hipEvent_t* ev_join, hipStream_t strm) {
    struct Side {
        hipStream_t s = nullptr;
        hipEvent_t a = nullptr, b = nullptr;
    };
    thread_local std::array<Side, 64> sides{};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
        (void)hipGetLastError();
        return false;
    }
    Side& e = sides[dev];
    if (e.s == nullptr) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(strm, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
            (void)hipGetLastError();
            return false;
        }
        if (hipStreamCreateWithFlags(&e.s, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&e.a, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e.b, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            e = Side{};
            return false;
        }
    }
    *side = e.s;
    *ev_fork = e.a;
    *ev_join = e.b;
    return true;
}

static int32_t rgcn_bwd_impl(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R, const float* x,
                             int32_t F_in, const float* weight, const float* root, int32_t F_out,
                             const float* h_save, const float* grad_out, int64_t row_lo, int64_t row_hi,
                             float* grad_x, float* grad_weight, float* grad_root, float* grad_bias,
                             void* workspace, void* stream, bool acc, const float* gx_mask = nullptr) {
    int32_t st = check_common(p, F_in, F_out);
    if (st != MPGNN_OK) return st;
    Selection s;
    if ((st = make_selection(p, mode, relation, R, &s)) != MPGNN_OK) return st;
    if (!grad_out || !weight) return arg_error("NULL grad_out or weight");
    clamp_rows(p, &row_lo, &row_hi);
    hipStream_t strm = static_cast<hipStream_t>(stream);
    const RootChunks rc = root_chunks(row_lo, row_hi);
    const WsLayout w = ws_layout(p, mode, s, F_in, F_out, row_lo, row_hi, rc);
    char* ws = static_cast<char*>(workspace);
    if (!ws) return arg_error("NULL workspace");
    const Options& o = p->opt;
    const bool exact = o.exact_order;

    const bool want_x = grad_x != nullptr && p->N > 0;
    const bool want_p = grad_weight != nullptr || grad_root != nullptr || grad_bias != nullptr;
    if (acc) {
        // accumulating parameter gradients: the mode-ALL F = 128 path (outer_bf3_kernel + the
        // ordered slab sum) only, decided before anything is launched
        const int nch = s.c_hi - s.c_lo;
        if (mode != MPGNN_MODE_ALL || !o.gemm_bf3 || F_in != 128 || F_out != 128 || !grad_weight || !grad_root ||
            !grad_bias || nch <= 0 || rc.n <= 0 || !x)
            return MPGNN_ERR_UNSUPPORTED;
        // where mpgnn_rgcn_bwd takes the one-launch bwd_fused path (few items per CU) its
        // gradients are summed in another order: refused, so that the caller's fallback (fresh
        // gradients + one add) stays bit-identical to autograd's accumulation of that path
        const int64_t items = (int64_t)(s.t32_hi - s.t32_lo) + (row_hi - row_lo + 31) / 32;
        if (o.bwd_fused && o.rel_gemm && !exact && root && (h_save != nullptr || s.m_hi == s.m_lo) &&
            p->N <= INT32_MAX - 1 && row_hi > row_lo && items <= 4 * (int64_t)cu_count())
            return MPGNN_ERR_UNSUPPORTED;
    }
    if (!acc && o.bwd_fused && o.gemm_bf3 && o.rel_gemm && !exact && F_in == 128 && F_out == 128 && p->N > 0 && x != nullptr &&
        root != nullptr && grad_weight != nullptr && grad_root != nullptr && (h_save != nullptr || s.m_hi == s.m_lo) &&
        p->N <= INT32_MAX - 1) {
        st = bwd_fused(p, mode, R, x, weight, root, h_save, grad_out, row_lo, row_hi, want_x ? grad_x : nullptr,
                       grad_weight, grad_root, grad_bias, s, w, ws, strm, gx_mask);
        if (st != MPGNN_ERR_UNSUPPORTED) return st;
        st = MPGNN_OK;
    }
    // ---- grad_x = Σ_r A_rᵀ ((dout @ W_rᵀ) / cnt) + dout @ rootᵀ ----------------------
    auto grad_x_part = [&](hipStream_t strm) -> int32_t {
        float* G = reinterpret_cast<float*>(ws + w.g);
        float* Groot = root ? reinterpret_cast<float*>(ws + w.groot) : nullptr;
        float* Pdx = reinterpret_cast<float*>(ws + w.pdx);
        // the augmented transposed list's piece counters (run_grad_x's first branch) are zeroed by
        // the dgrad GEMM launch itself where it is rel_gemm_bf3_kernel: one memset launch less
        const bool aug = mode == MPGNN_MODE_ALL && !exact && Groot != nullptr && row_lo == p->shard_lo &&
                         row_hi == p->shard_hi && o.flat_fuse_split && p->tx_f.nsplit > 0;
        bool zeroed = false;
        int32_t e = run_seg(p, mode, s, 1, grad_out, F_out, weight, root, 1, F_in, G, Groot, row_lo, row_hi, nullptr,
                            nullptr, true, MPGNN_K_SEG_DGRAD, strm, nullptr, nullptr, nullptr, 0,
                            aug ? split_counters(p, Pdx, F_in) : nullptr,
                            aug ? (int)(split_counter_bytes(p) / sizeof(unsigned)) : 0, &zeroed);
        if (e != MPGNN_OK) return e;
        return run_grad_x(p, mode, s, G, Groot, F_in, row_lo, row_hi, grad_x, Pdx, exact, strm, zeroed, gx_mask);
    };
    // (the two halves on two streams — parameter gradients on a side stream forked from and
    // joined into the caller's — measured slower: C3 epoch 1.163 -> 1.207 ms; not kept)
    // MPGNN_OPT_BWD_SIDE_REDUCE: the weight gradient's outer products first, then its ordered
    // slab sum (HBM-bound, ~40 VGPRs) on a side stream beside the dgrad GEMM (MFMA-bound, 464 of a
    // SIMD's 512 VGPRs) and grad_x, joined before this call returns
    if (o.side_reduce && want_x && want_p && !acc) {
        hipStream_t side = nullptr;
        hipEvent_t ev_fork = nullptr, ev_join = nullptr;
        if (side_stream(&side, &ev_fork, &ev_join, strm)) {
            bool forked = false;
            st = bwd_params(p, mode, R, x, F_in, F_out, h_save, grad_out, grad_weight, grad_root, grad_bias, s, w, rc, ws,
                            strm, acc, side, ev_fork, ev_join, &forked);
            if (st != MPGNN_OK) return st;
            st = grad_x_part(strm);
            if (forked) {
                const int32_t sj = hip_check(hipStreamWaitEvent(strm, ev_join, 0), "join side reduce");
                if (st == MPGNN_OK) st = sj;
            }
            return st;
        }
    }
    if (want_x && (st = grad_x_part(strm)) != MPGNN_OK) return st;
    if (want_p) st = bwd_params(p, mode, R, x, F_in, F_out, h_save, grad_out, grad_weight, grad_root, grad_bias, s, w,
                                rc, ws, strm, acc);
    return st;
}

int32_t mpgnn_rgcn_bwd(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R, const float* x,
                       int32_t F_in, const float* weight, const float* root, int32_t F_out,
                       const float* h_save, const float* grad_out, int64_t row_lo, int64_t row_hi,
                       float* grad_x, float* grad_weight, float* grad_root, float* grad_bias,
                       void* workspace, void* stream) {
    return rgcn_bwd_impl(p, mode, relation, R, x, F_in, weight, root, F_out, h_save, grad_out, row_lo, row_hi, grad_x,
                         grad_weight, grad_root, grad_bias, workspace, stream, false);
}

int32_t mpgnn_rgcn_bwd_accumulate(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R, const float* x,
                                  int32_t F_in, const float* weight, const float* root, int32_t F_out,
                                  const float* h_save, const float* grad_out, int64_t row_lo, int64_t row_hi,
                                  float* grad_x, float* grad_weight, float* grad_root, float* grad_bias,
                                  void* workspace, void* stream) {
    return rgcn_bwd_impl(p, mode, relation, R, x, F_in, weight, root, F_out, h_save, grad_out, row_lo, row_hi, grad_x,
                         grad_weight, grad_root, grad_bias, workspace, stream, true);
}

int32_t mpgnn_rgcn_bwd_relu_in(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R, const float* x,
                               int32_t F_in, const float* weight, const float* root, int32_t F_out,
                               const float* h_save, const float* grad_out, int64_t row_lo, int64_t row_hi,
                               float* grad_x, float* grad_weight, float* grad_root, float* grad_bias,
                               void* workspace, void* stream, int32_t accumulate) {
    if (grad_x != nullptr && x == nullptr) return arg_error("NULL x (the grad_x mask)");
    return rgcn_bwd_impl(p, mode, relation, R, x, F_in, weight, root, F_out, h_save, grad_out, row_lo, row_hi, grad_x,
                         grad_weight, grad_root, grad_bias, workspace, stream, accumulate != 0, x);
}

// the parameter gradients of mpgnn_rgcn_bwd (dW / droot / dbias outer products + slab reduce)
static int32_t bwd_params(const mpgnn_plan* p, int32_t mode, int32_t R, const float* x, int32_t F_in, int32_t F_out,
                          const float* h_save, const float* grad_out, float* grad_weight, float* grad_root,
                          float* grad_bias, const Selection& s, const WsLayout& w, const RootChunks& rc, char* ws,
                          hipStream_t strm, bool acc, hipStream_t side, hipEvent_t ev_fork, hipEvent_t ev_join,
                          bool* forked) {
    int32_t st = MPGNN_OK;
    if (forked != nullptr) *forked = false;
    const size_t wsize = (size_t)F_in * F_out;
    const bool exact = p->opt.exact_order;
    const int mt = (F_in + kColTile - 1) / kColTile;
    const int nt = (F_out + kColTile - 1) / kColTile;
    const size_t outer_lds = (size_t)(4 * kOuterBuf) * sizeof(float);
    const bool outer_vec = (F_in & 3) == 0 && (F_out & 3) == 0;
    auto launch_outer = [&](dim3 grid, const OuterArgs& o) {
        if (outer_vec) hipLaunchKernelGGL(outer_accum_kernel<true>, grid, dim3(kThreads), outer_lds, strm, o);
        else hipLaunchKernelGGL(outer_accum_kernel<false>, grid, dim3(kThreads), outer_lds, strm, o);
    };

    // ---- grad_weight[r] = Σ_{seg of r} h_segᵀ dout[node_1(seg)] -------------------------
    // ---- grad_root = xᵀ dout, grad_bias = Σ dout  (rows [row_lo, row_hi)) ---------------
    // Both outer-product accumulations go out as ONE launch when their grids match, and the
    // slab reductions (dW groups, droot, dbias) as one more.
    struct Part {
        ReduceArgs r;
        int gx, ey;
    };
    std::vector<Part> reduces;
    ZeroList zl{};
    bool have_w = false, have_root = false;
    OuterArgs ow{}, orr{};
    int nch = 0;
    if (grad_weight != nullptr) {
        const size_t wbytes = (mode == MPGNN_MODE_ALL ? (size_t)std::max(R, 0) : 1) * wsize * sizeof(float);
        // every weight index with a segment range is written (directly or by the slab reduce,
        // zeros for an empty range); only indices absent from the plan need the memset
        // (accumulating: absent relation ids keep their gradient)
        const bool all_written = acc || ((mode == MPGNN_MODE_ALL) ? (s.d_hi - s.d_lo) == (int64_t)R : (s.c_hi > s.c_lo));
        if (!all_written && mode == MPGNN_MODE_ALL && (int64_t)R - (s.d_hi - s.d_lo) <= kMaxZeroIds) {
            // the few absent relation ids are zeroed by the reduce launch
            zl.dst = grad_weight;
            zl.elems = (int)wsize;
            int64_t d = s.d_lo;
            for (int32_t id = 0; id < R; ++id) {
                while (d < s.d_hi && p->rel_values[d] < id) ++d;
                if (d < s.d_hi && p->rel_values[d] == id) continue;
                zl.ids[zl.n++] = id;
            }
        } else if (!all_written) {
            if ((st = hip_check(hipMemsetAsync(grad_weight, 0, wbytes, strm), "memset grad_weight")) != MPGNN_OK)
                return st;
        }
        nch = s.c_hi - s.c_lo;
        if (nch > 0) {
            if (!x) return arg_error("NULL x (grad_weight reads the single-edge segment means from x)");
            const float* H = h_save;
            if (H == nullptr) {
                float* Hw = reinterpret_cast<float*>(ws + w.h);
                st = run_means_multi(p, s, x, F_in, Hw, reinterpret_cast<float*>(ws + w.pdx), exact, strm);
                if (st != MPGNN_OK) return st;
                H = Hw;
            }
            float* P = reinterpret_cast<float*>(ws + w.p);
            ow.chunk_begin = p->d.chunk_begin;
            ow.chunk_end = p->d.chunk_end;
            ow.chunk_dst = p->d.chunk_dst;
            ow.chunk_off = s.c_lo;
            // accumulating: every chunk to a slab, the reduce adds dst + Σ (the MFMA kernel's
            // epilogue stays store-only: a read-modify-write there cost 9 us per launch)
            ow.dst_mode = acc ? 0 : (mode == MPGNN_MODE_ALL ? 1 : 2);
            ow.A = x;  // segment s: x[s_src[s]] or Hm[-s_src[s] - 1 - m_lo]
            ow.a_idx = p->d.s_src;
            ow.A2 = H;
            ow.a2_off = s.m_lo;
            ow.M = F_in;
            ow.a_off = 0;
            ow.B = grad_out;
            ow.Nn = F_out;
            ow.b_idx = p->d.s_row;
            ow.P = P;
            ow.dst = grad_weight;
            ow.Pb = nullptr;
            have_w = true;
            ReduceArgs r{};
            r.P = P;
            r.elems = (int)wsize;
            r.dst = grad_weight;
            r.skip_single = acc ? 0 : 1;
            r.acc = acc ? 1 : 0;
            const int ey = (int)((wsize + kThreads - 1) / kThreads);
            if (mode == MPGNN_MODE_ALL) {
                r.gptr = p->d.rel_chunk_ptr;
                r.g_off = s.c_lo;
                r.gdst = p->d.rel_val32;
                r.g_base = (int)s.d_lo;
                reduces.push_back({r, (int)(s.d_hi - s.d_lo), ey});
            } else if (nch > 1) {  // one chunk: written directly
                r.gptr = nullptr;
                r.nchunks = nch;
                r.gdst = nullptr;
                reduces.push_back({r, 1, ey});
            }
        }
    }
    if (grad_root != nullptr || grad_bias != nullptr) {
        if (rc.n == 0) {
            if (grad_root && (st = hip_check(hipMemsetAsync(grad_root, 0, wsize * sizeof(float), strm), "memset")))
                return st;
            if (grad_bias && (st = hip_check(hipMemsetAsync(grad_bias, 0, F_out * sizeof(float), strm), "memset")))
                return st;
        } else {
            if (!x) return arg_error("NULL x");
            float* P = reinterpret_cast<float*>(ws + w.proot);
            float* Pb = reinterpret_cast<float*>(ws + w.pb);
            orr.chunk_begin = nullptr;
            orr.row_lo = rc.rows_lo;
            orr.row_hi = rc.rows_hi;
            orr.chunk_rows = rc.chunk;
            orr.dst_mode = (rc.n == 1 && !acc) ? 3 : 0;
            orr.A = x;
            orr.M = F_in;
            orr.a_off = 0;
            orr.B = grad_out;
            orr.Nn = F_out;
            orr.b_idx = nullptr;
            orr.P = P;
            orr.dst = grad_root;
            orr.Pb = grad_bias ? Pb : nullptr;
            orr.dst_b = grad_bias;
            have_root = true;
            if ((rc.n > 1 || acc) && grad_root) {
                ReduceArgs r{};
                r.P = P;
                r.elems = (int)wsize;
                r.nchunks = rc.n;
                r.dst = grad_root;
                r.acc = acc ? 1 : 0;
                reduces.push_back({r, 1, (int)((wsize + kThreads - 1) / kThreads)});
            }
            if ((rc.n > 1 || acc) && grad_bias) {
                ReduceArgs r{};
                r.P = Pb;
                r.elems = F_out;
                r.nchunks = rc.n;
                r.dst = grad_bias;
                r.acc = acc ? 1 : 0;
                reduces.push_back({r, 1, (F_out + kThreads - 1) / kThreads});
            }
        }
    }
    const int root_y = grad_root ? mt : 1;
    const bool bf3 = have_w && have_root && root_y == mt && p->opt.gemm_bf3 && F_in == 128 && F_out == 128;
    // F_in = F_out = 256 (C5): the same kernel over the four 128 × 128 quadrants of every dW_r /
    // droot slab (the bias column sums taken by the two quadrants of the first A half)
    const bool bf3q = have_w && have_root && root_y == mt && p->opt.gemm_bf3 && F_in == 256 && F_out == 256 && !acc;
    if (acc && !bf3) return MPGNN_ERR_UNSUPPORTED;  // (excluded by rgcn_bwd_impl's check)
    // balanced contiguous chunk ranges per workgroup (outer_bf3v_kernel_t only)
    auto with_ranges = [&](OuterArgs& o, int n_all, int gx) {
        o.wg_chunks = nullptr;
        o.wg_cus = 0;
        if (!p->opt.outer_vec || !p->opt.outer_ranges) return;
        o.wg_chunks = outer_ranges(p, s.c_lo, nch, rc.rows_lo, rc.rows_hi, rc.chunk, rc.n, gx, strm);
        (void)n_all;
    };
    if (bf3q) {
        TimedLaunch tl(MPGNN_K_OUTER, strm);
        const int n_all = nch + rc.n;
        const int gx = std::max(1, std::min(n_all, cu_count() * 2));
        with_ranges(orr, n_all, gx);
        for (int qa = 0; qa < 2; ++qa)
            for (int qb = 0; qb < 2; ++qb) {
                OuterArgs rq = orr, wq = ow;
                for (OuterArgs* o : {&rq, &wq}) {
                    o->lda = F_in;
                    o->ldb = F_out;
                    o->a_col0 = qa * 128;
                    o->b_col0 = qb * 128;
                    o->ldd = F_out;
                    o->d_off = qa * 128 * F_out + qb * 128;
                    o->p_stride = (int64_t)F_in * F_out;
                    o->pb_stride = F_out;
                }
                if (qa != 0) {  // the bias column sums once per B half
                    rq.Pb = nullptr;
                    rq.dst_b = nullptr;
                }
                launch_outer_bf3(dim3(gx), rq, wq, rc.n, n_all, p->opt.outer_vec, p->opt.outer_sq, strm, p->opt.outer_variant);
                if ((st = hip_check(hipGetLastError(), "outer_bf3_kernel (quadrant) launch")) != MPGNN_OK) return st;
            }
    } else if (bf3) {
        // F_in = F_out = 128: the bf16-split persistent kernel (outer_bf3_kernel)
        TimedLaunch tl(MPGNN_K_OUTER, strm);
        const int n_all = nch + rc.n;
        const int gx = std::max(1, std::min(n_all, cu_count() * 2));
        with_ranges(orr, n_all, gx);
        launch_outer_bf3(dim3(gx), orr, ow, rc.n, n_all, p->opt.outer_vec, p->opt.outer_sq, strm, p->opt.outer_variant);
        if ((st = hip_check(hipGetLastError(), "outer_bf3_kernel launch")) != MPGNN_OK) return st;
    } else if (have_w && have_root && root_y == mt) {
        TimedLaunch tl(MPGNN_K_OUTER, strm);
        // one launch: root chunks (all full length; the relation chunks of small relations are
        // short) dispatched first so they are not the launch's tail, 16-row LDS slices
        const size_t lds16 = (size_t)(4 * (16 / 2) * kOuterLd) * sizeof(float);
        {
            // persistent: two workgroups per CU per column tile pair, root chunks first
            const int n_all = nch + rc.n;
            const int gx = std::max(1, std::min(n_all, cu_count() * 2 / std::max(1, mt * nt)));
            const dim3 gridp(gx, mt, nt);
            // 32-row slices (F % 4 == 0): half the barriers per MFMA of 16-row ones, two workgroups per
            // CU in 72 KB of LDS each (C3: 111.8 -> 108.4 us)
            if (outer_vec)
                hipLaunchKernelGGL((outer_persist_kernel<true, 32>), gridp, dim3(kThreads), 2 * lds16, strm, orr, ow, rc.n,
                                   n_all);
            else
                hipLaunchKernelGGL((outer_persist_kernel<false, 16>), gridp, dim3(kThreads), lds16, strm, orr, ow, rc.n, n_all);
        }
        if ((st = hip_check(hipGetLastError(), "outer_persist_kernel launch")) != MPGNN_OK) return st;
    } else {
        if (have_w) {
            TimedLaunch tl(MPGNN_K_OUTER, strm);
            launch_outer(dim3(nch, mt, nt), ow);
            if ((st = hip_check(hipGetLastError(), "outer_accum_kernel(dW) launch")) != MPGNN_OK) return st;
        }
        if (have_root) {
            TimedLaunch tl(MPGNN_K_OUTER, strm);
            launch_outer(dim3(rc.n, root_y, nt), orr);
            if ((st = hip_check(hipGetLastError(), "outer_accum_kernel(root) launch")) != MPGNN_OK) return st;
        }
    }
    if (reduces.empty() && zl.n == 0) return MPGNN_OK;
    {
        ReduceArgs r3[3] = {};
        int gx[3] = {0, 0, 0}, ey = zl.n > 0 ? (zl.elems + kThreads - 1) / kThreads : 0;
        for (size_t k = 0; k < reduces.size(); ++k) {
            r3[k] = reduces[k].r;
            gx[k] = reduces[k].gx;
            ey = std::max(ey, reduces[k].ey);
        }
        // MPGNN_OPT_BWD_SIDE_REDUCE: the ordered slab sum on a side stream forked here (the caller
        // runs grad_x's launches meanwhile and joins on ev_join)
        hipStream_t rs = strm;
        if (side != nullptr && ev_fork != nullptr && ev_join != nullptr &&
            hipEventRecord(ev_fork, strm) == hipSuccess && hipStreamWaitEvent(side, ev_fork, 0) == hipSuccess)
            rs = side;
        (void)hipGetLastError();
        {
            TimedLaunch tl(MPGNN_K_REDUCE, rs);
            hipLaunchKernelGGL(reduce_slabs3_kernel, dim3(gx[0] + gx[1] + gx[2] + zl.n, ey), dim3(kThreads), 0, rs,
                               r3[0], r3[1], r3[2], gx[0], gx[1], gx[2], zl);
            if ((st = hip_check(hipGetLastError(), "reduce_slabs3_kernel launch")) != MPGNN_OK) return st;
        }
        if (rs != strm) {
            if ((st = hip_check(hipEventRecord(ev_join, rs), "side reduce event")) != MPGNN_OK) return st;
            if (forked != nullptr) *forked = true;
        }
        return MPGNN_OK;
    }
}

// Debug: workgroups per CU the runtime admits for the forward tile kernel at gather width F.
int32_t mpgnn_debug_occupancy(int32_t F, int32_t* seg_tile_blocks_per_cu, int32_t* tile_gemm_blocks_per_cu,
                              int32_t* tile_gemm_grid) {
    if (!seg_tile_blocks_per_cu || !tile_gemm_blocks_per_cu || !tile_gemm_grid) return arg_error("NULL argument");
    int V, T;
    if (!pick_vt(F, &V, &T)) return MPGNN_ERR_UNSUPPORTED;
    const int Kp = round_up(F, 64);
    const size_t lds = (size_t)(kTileRows + kTileRows * (Kp + 4)) * sizeof(float);
    int nb = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, seg_tile_kernel<2, 1>, kThreads, lds);
    *seg_tile_blocks_per_cu = nb;
    if (e != hipSuccess) return hip_check(e, "hipOccupancyMaxActiveBlocksPerMultiprocessor");
    const int kb = Kp / 64;
    int nt = 0;
    size_t lds_t = 0;
    auto occ = [&](auto kern, int KB) {
        const int lda = 64 * KB + 4, ldo = kColTile + 4;
        lds_t = (size_t)(2 * kTileRows * (lda > ldo ? lda : ldo) + 2 * kTileRows) * sizeof(float);
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&nt, kern, kThreads, lds_t);
    };
    if (kb <= 1) e = occ(tile_gemm_kernel<1>, 1);
    else if (kb == 2) e = occ(tile_gemm_kernel<2>, 2);
    else if (kb == 3) e = occ(tile_gemm_kernel<3>, 3);
    else e = occ(tile_gemm_kernel<4>, 4);
    *tile_gemm_blocks_per_cu = nt;
    *tile_gemm_grid = cu_count() * ((2 * lds_t <= 160 * 1024) ? 2 : 1);
    return hip_check(e, "hipOccupancyMaxActiveBlocksPerMultiprocessor");
}

#ifdef MPGNN_STAMPS
int32_t mpgnn_debug_stamps_set(void* dev_ptr) {
    g_stamps_host = static_cast<unsigned long long*>(dev_ptr);
    return MPGNN_OK;
}
#endif

int32_t mpgnn_timing_enable(int32_t on) {
    std::lock_guard<std::mutex> lk(g_timing_mu);
    g_timing_on = on != 0;
    return MPGNN_OK;
}

int32_t mpgnn_timing_reset(void) {
    std::lock_guard<std::mutex> lk(g_timing_mu);
    for (auto& r : g_timing) {
        g_event_pool.push_back(r.start);
        g_event_pool.push_back(r.stop);
    }
    g_timing.clear();
    return MPGNN_OK;
}

int32_t mpgnn_timing_query(int32_t kind, double* total_ms, int64_t* launches) {
    if (!total_ms || !launches) return arg_error("NULL argument");
    std::lock_guard<std::mutex> lk(g_timing_mu);
    double tot = 0.0;
    int64_t n = 0;
    for (auto& r : g_timing) {
        if (r.kind != kind) continue;
        int32_t st = hip_check(hipEventSynchronize(r.stop), "hipEventSynchronize");
        if (st != MPGNN_OK) return st;
        float ms = 0.0f;
        if ((st = hip_check(hipEventElapsedTime(&ms, r.start, r.stop), "hipEventElapsedTime")) != MPGNN_OK) return st;
        tot += ms;
        ++n;
    }
    *total_ms = tot;
    *launches = n;
    return MPGNN_OK;
}

}  // extern "C"
