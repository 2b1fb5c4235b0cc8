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
//   seg_tile_kernel    one workgroup = one relation-pure tile of 64 segments (node_1, r):
//                      wavefront segmented gather-sum of x rows into an LDS tile (edge order,
//                      bit-exact mean), then v_mfma_f32_32x32x2_f32 against W_r.  Forward
//                      writes Y[seg] = h_seg @ W_r (+ h_seg itself for backward); backward
//                      ("dgrad") writes G[seg] = (dout[node_1] @ W_rᵀ) / cnt.
//   row_tile_kernel    one workgroup = 64 output rows: ordered sum of the rows' Y (or G)
//                      entries into LDS + MFMA of the dense tile (x @ root, dout @ rootᵀ),
//                      epilogue (Σ + root-term) + bias.
//   outer_accum_kernel dW_r / droot partial slabs  P_c = A_cᵀ B_c over a chunk of rows (MFMA).
//   reduce_slabs_kernel ordered sum of the partial slabs of each group (deterministic).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "plan_internal.h"

namespace mpgnn {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kThreads = 256;  // 4 waves of 64
constexpr int kWaves = 4;
constexpr int kRowsPerWave = kTileRows / kWaves;  // 16
constexpr int kColTile = 128;                    // output columns per workgroup (4 × 32-col strips)
constexpr int kSlice = 32;                       // rows per K-slice in outer_accum_kernel
constexpr int kMaxF = 256;  // LDS budget: row_tile_kernel holds 64×(G + K + 4) floats

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

__device__ __forceinline__ int readlane(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }

// ----------------------------------------------------------------------------------------
// Wavefront segmented gather-sum into an LDS tile.
//
// The wave owns `nrows` (≤ 16) consecutive tile rows.  Lane j (j ≤ nrows) holds in `bnd` the
// position where row j's entries start (so row j covers positions [bnd_j, bnd_{j+1})), and the
// positions of consecutive rows are contiguous.  Position p contributes source row
//     src_row(p) = (idx ? idx[p] : p) - idx_off
// unless a filter rejects it (fidx[p] outside [flo, fhi)).  With a two-level list (g.ent) the
// wave walks entries instead: an entry >= 0 is a position as above, an entry -(k+1) adds the
// partial sum P[k - piece_off] of an ordered piece of a long run (piece_sum_kernel).  Lanes span the feature dimension
// (V floats per lane, T chunks of 64·V columns); every lane adds its columns in position
// order starting from 0.0f, which is exactly ATen's sequential scatter_add_ into a zeroed
// output — the sums are bit-identical to the reference.  Each finished row is optionally
// divided by cnt[row] (IEEE division = `out / count` of PyG's mean), written to LDS with
// zeros in [F, width), and optionally copied to global memory.
// ----------------------------------------------------------------------------------------
struct GatherSrc {
    const float* src;  // [*, F]
    int F;
    const int* idx;    // nullable
    int idx_off;
    const int* fidx;   // nullable filter index
    int flo, fhi;
    const int* ent;    // nullable: two-level entries (position >= 0 | -(piece+1))
    const float* P;    // piece partial sums [*, F] (rows k - piece_off)
    int piece_off;
};

template <int V, int T>
__device__ __forceinline__ void flush_row(float (&acc)[T][V], bool live, const int* cnt_rows, int r,
                                          float* lds_row, int width, int F, float* grow, int lane) {
    float scale_div = 1.0f;
    const bool do_div = live && cnt_rows != nullptr;
    if (do_div) scale_div = (float)cnt_rows[r];
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const int col = (t * 64 + lane) * V;
        float v[V];
#pragma unroll
        for (int q = 0; q < V; ++q) v[q] = live ? (do_div ? acc[t][q] / scale_div : acc[t][q]) : 0.0f;
        if (col < width) vstore<V>(lds_row + col, v);
        if (grow != nullptr && live && col < F) vstore<V>(grow + col, v);
#pragma unroll
        for (int q = 0; q < V; ++q) acc[t][q] = 0.0f;
    }
}

template <int V, int T, int UNR>
__device__ void wave_gather(const GatherSrc& g, int bnd, int nrows, const int* cnt_rows,
                            float* lds, int lda, int width, float* gout, int gout_ld, int lane) {
    float acc[T][V];
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int q = 0; q < V; ++q) acc[t][q] = 0.0f;

    const int p_begin = readlane(bnd, 0);
    const int p_end = readlane(bnd, nrows);
    int r = 0;
    int r_end = nrows > 0 ? readlane(bnd, 1) : p_end;

    auto flush = [&](int row) {
        const bool live = row < nrows;
        float* grow = (gout != nullptr && live) ? gout + (size_t)row * gout_ld : nullptr;
        flush_row<V, T>(acc, live, cnt_rows, row, lds + row * lda, width, g.F, grow, lane);
    };

    // column offsets of this lane, clamped so that every load is unconditional (the value of
    // a lane past F is never stored); a load behind a per-entry branch makes hipcc wait for
    // each entry separately (cdna_hip_programming.md §5 trap (c))
    int colc[T];
#pragma unroll
    for (int t = 0; t < T; ++t) colc[t] = min((t * 64 + lane) * V, g.F - V);

    for (int pb = p_begin; pb < p_end; pb += 64) {
        const int np = min(64, p_end - pb);
        int my_src = 0;
        bool my_keep = false;
        bool my_piece = false;
        if (lane < np) {
            const int e = g.ent != nullptr ? g.ent[pb + lane] : pb + lane;
            if (e >= 0) {
                my_keep = true;
                if (g.fidx != nullptr) {
                    const int f = g.fidx[e];
                    my_keep = (f >= g.flo) && (f < g.fhi);
                }
                my_src = (g.idx != nullptr ? g.idx[e] : e) - g.idx_off;
            } else {
                my_keep = true;
                my_piece = true;
                my_src = -e - 1 - g.piece_off;
            }
            if (!my_keep) my_src = 0;  // rejected entry: load a valid row, never added
        }
        const unsigned long long keep = __ballot(my_keep);
        const unsigned long long from_piece = __ballot(my_piece);
        for (int u = 0; u < np; u += UNR) {
            float v[UNR][T][V];
#pragma unroll
            for (int uu = 0; uu < UNR; ++uu) {
                const int q = min(u + uu, np - 1);
                const int row = readlane(my_src, q);
                const float* base = (((from_piece >> q) & 1ull) ? g.P : g.src) + (size_t)row * g.F;
#pragma unroll
                for (int t = 0; t < T; ++t) vload<V>(base + colc[t], v[uu][t]);
            }
#pragma unroll
            for (int uu = 0; uu < UNR; ++uu) {
                const int q = u + uu;
                if (q < np) {
                    const int p = pb + q;
                    while (p >= r_end) {
                        flush(r);
                        ++r;
                        r_end = readlane(bnd, r + 1);
                    }
                    if ((keep >> q) & 1ull) {
#pragma unroll
                        for (int t = 0; t < T; ++t)
#pragma unroll
                            for (int c = 0; c < V; ++c) acc[t][c] += v[uu][t][c];
                    }
                }
            }
        }
    }
    for (; r < kRowsPerWave; ++r) flush(r);
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
    const int* fidx;
    int flo, fhi;
    float* P;
};

template <int V, int T>
__global__ __launch_bounds__(kThreads) void piece_sum_kernel(PieceArgs a) {
    const int lane = threadIdx.x & 63;
    const int k = a.k_lo + blockIdx.x * kWaves + (threadIdx.x >> 6);
    if (k >= a.k_hi) return;
    const int p0 = a.pb[k], p1 = a.pe[k];
    const int np = p1 - p0;  // <= 32 <= 64
    int my_src = 0;
    bool my_keep = false;
    if (lane < np) {
        const int p = p0 + lane;
        my_keep = true;
        if (a.fidx != nullptr) {
            const int f = a.fidx[p];
            my_keep = (f >= a.flo) && (f < a.fhi);
        }
        my_src = (a.idx != nullptr ? a.idx[p] : p) - a.idx_off;
    }
    if (!my_keep) my_src = 0;
    const unsigned long long keep = __ballot(my_keep);
    float acc[T][V];
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int c = 0; c < V; ++c) acc[t][c] = 0.0f;
    int colc[T];
#pragma unroll
    for (int t = 0; t < T; ++t) colc[t] = min((t * 64 + lane) * V, a.F - V);
    constexpr int UNR = (V * T <= 2 ? 8 : 4);
    for (int u = 0; u < np; u += UNR) {
        float v[UNR][T][V];
#pragma unroll
        for (int uu = 0; uu < UNR; ++uu) {
            const float* base = a.src + (size_t)readlane(my_src, min(u + uu, np - 1)) * a.F;
#pragma unroll
            for (int t = 0; t < T; ++t) vload<V>(base + colc[t], v[uu][t]);
        }
#pragma unroll
        for (int uu = 0; uu < UNR; ++uu)
            if (u + uu < np && ((keep >> (u + uu)) & 1ull)) {
#pragma unroll
                for (int t = 0; t < T; ++t)
#pragma unroll
                    for (int c = 0; c < V; ++c) acc[t][c] += v[uu][t][c];
            }
    }
    float* out = a.P + (size_t)(k - a.k_lo) * a.F;
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const int col = (t * 64 + lane) * V;
        if (col < a.F) vstore<V>(out + col, acc[t]);
    }
}

// Dense tile loader: rows [row0, row0+64) of A[*, K] into lds[64][lda] with zeros past
// K (up to width) and past nrows.  All of a thread's loads are issued before any LDS store
// (float4 when the row stride allows), so the tile costs one memory latency, not 32.
__device__ void load_dense_tile(const float* __restrict__ A, int K, int row0, int nrows, float* lds,
                                int lda, int width) {
    if ((K & 3) == 0 && (width & 3) == 0) {
        const int w4 = width >> 2;
        const int total = kTileRows * w4;  // float4 slots
        constexpr int kBatch = 8;
        for (int i0 = threadIdx.x; i0 < total; i0 += kBatch * kThreads) {
            float4 v[kBatch];
#pragma unroll
            for (int it = 0; it < kBatch; ++it) {
                const int i = min(i0 + it * kThreads, total - 1);
                const int r = i / w4;
                const int c = (i - r * w4) * 4;
                const int rr = min(r, max(nrows - 1, 0));
                const int cc = min(c, K - 4);
                v[it] = *reinterpret_cast<const float4*>(A + (size_t)(row0 + rr) * K + cc);
            }
#pragma unroll
            for (int it = 0; it < kBatch; ++it) {
                const int i = i0 + it * kThreads;
                if (i < total) {
                    const int r = i / w4;
                    const int c = (i - r * w4) * 4;
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
            const int i = i0 + u * kThreads;
            v[u] = 0.0f;
            if (i < total) {
                const int r = i / width;
                const int c = i - r * width;
                if (r < nrows && c < K) v[u] = A[(size_t)(row0 + r) * K + c];
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * kThreads;
            if (i < total) {
                const int r = i / width;
                lds[r * lda + (i - r * width)] = v[u];
            }
        }
    }
}

// ----------------------------------------------------------------------------------------
// MFMA tile:  acc(64 × 128-column tile) = A_lds[64 × Kp] · B[K × N]
// v_mfma_f32_32x32x2_f32: lane l holds A[i = l&31][kk = l>>5] and B[kk][j = l&31];
// C/D: col = l&31, row = (r&3) + 8(r>>2) + 4(l>>5).  The K dimension is split in two halves
// so that lane-half h walks k ∈ [h·Kp/2, (h+1)·Kp/2) contiguously (one ds_read_b128 feeds
// four MFMAs); the MFMA sums over both halves, so every k is covered exactly once.
// Wave w owns blocks b ∈ {w, w+4} of the (2 row-halves × NS strips) grid, b = mb·NS + nb.
// ----------------------------------------------------------------------------------------
struct BSrc {
    const float* W;  // element (k, n) = trans ? W[n*ldw + k] : W[k*ldw + n]
    int ldw;
    int K, N;
    int trans;
};

// Wave w owns column strip w (32 columns) of the 128-column tile and BOTH 32-row halves, so
// its two accumulators share every B value; waves whose strip starts past N idle.
struct MfmaTile {
    f32x16 acc0, acc1;  // rows 0..31 / 32..63 of strip `nb`
    int nb;
    bool active;
};

__device__ __forceinline__ void mfma_tile(MfmaTile& mt, const float* A_lds, int lda, int Kp,
                                          const BSrc& b, int n_base, int wave, int lane) {
    const int c = lane & 31;
    const int h = lane >> 5;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        mt.acc0[r] = 0.0f;
        mt.acc1[r] = 0.0f;
    }
    mt.nb = wave;
    mt.active = n_base + wave * 32 < b.N;
    if (!mt.active) return;
    const int KH = Kp / 2;
    const int n = min(n_base + wave * 32 + c, b.N - 1);  // clamped: columns >= N are never stored
    const float* a0p = A_lds + c * lda + h * KH;
    const float* a1p = A_lds + (32 + c) * lda + h * KH;
    const int kb = h * KH;
    f32x16 acc0 = mt.acc0, acc1 = mt.acc1;
    // B values are loaded one group of 4 k ahead with clamped addresses; the k < K select is
    // applied when the group is consumed, so the prefetch is never waited for early.
    auto mfma8 = [&](const float (&braw)[4], int k0, int t) {
        const float4 a0 = *reinterpret_cast<const float4*>(a0p + t);
        const float4 a1 = *reinterpret_cast<const float4*>(a1p + t);
        float bq[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) bq[j] = (k0 + j < b.K) ? braw[j] : 0.0f;
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.x, bq[0], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.x, bq[0], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.y, bq[1], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.y, bq[1], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.z, bq[2], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.z, bq[2], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.w, bq[3], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.w, bq[3], acc1, 0, 0, 0);
    };
    if (!b.trans) {
        // B(k, n) = W[k*ldw + n]: rows k of W, 32 consecutive columns per half-wave
        const float* wp = b.W + n;
        auto ld4 = [&](int k0, float (&o)[4]) {
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = wp[(size_t)min(k0 + j, b.K - 1) * b.ldw];
        };
        float b0[4], b1[4];
        ld4(kb, b0);
        for (int t = 0; t < KH; t += 8) {  // KH % 8 == 0 (Kp % 16 == 0): ping-pong, no copies
            ld4(kb + t + 4, b1);
            mfma8(b0, kb + t, t);
            ld4(kb + t + 8, b0);
            mfma8(b1, kb + t + 4, t + 4);
        }
    } else {
        // B(k, n) = W[n*ldw + k]: row n of W, four consecutive k per load
        const float* wp = b.W + (size_t)n * b.ldw;
        const bool vec = (b.K & 3) == 0 && (b.ldw & 3) == 0;
        auto ld4 = [&](int k0, float (&o)[4]) {
            if (vec) {
                const float4 tv = *reinterpret_cast<const float4*>(wp + min(k0, b.K - 4));
                o[0] = tv.x;
                o[1] = tv.y;
                o[2] = tv.z;
                o[3] = tv.w;
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) o[j] = wp[min(k0 + j, b.K - 1)];
            }
        };
        float b0[4], b1[4];
        ld4(kb, b0);
        for (int t = 0; t < KH; t += 8) {
            ld4(kb + t + 4, b1);
            mfma8(b0, kb + t, t);
            ld4(kb + t + 8, b0);
            mfma8(b1, kb + t + 4, t + 4);
        }
    }
    mt.acc0 = acc0;
    mt.acc1 = acc1;
}

// ----------------------------------------------------------------------------------------
// seg_tile_kernel
// ----------------------------------------------------------------------------------------
struct SegTileArgs {
    const int* tile_begin;
    const int* tile_end;
    int tile_off;
    int gather_kind;     // 0: mean of src[e_col[e]] over the segment's edges; 1: src[s_row[s]]
    const float* src;
    int F;               // gather width = K of the MFMA
    const int* s_ptr;    // segment boundaries over edges (exact order) or over ragged entries
    const int* e_col;
    const int* s_row;
    const int* s_cnt;
    const int* s_rel;
    const int* s_pos;
    const int* ent;      // nullable: ragged entries (s_ptr then indexes entries)
    const float* P;      // piece partials of long segments
    int piece_off;
    const float* W;      // nullable: no transform (segment means only)
    int w_per_rel;       // W_r = W + s_rel[s] * K * N
    int trans;
    int N;               // output width
    float* Y;            // output rows
    int y_use_pos;       // row = s_pos[s] (row-major position) else s - sel_b
    int y_div;           // divide the MFMA result by cnt (dgrad)
    int sel_b;
    float* H;            // nullable: copy of the gathered tile rows, row = s - sel_b, width F
    int ablate;          // debug (MPGNN_OPT_ABLATE): 1 = skip gather, 2 = skip MFMA; wrong results
};

template <int V, int T>
__global__ __launch_bounds__(kThreads) void seg_tile_kernel(SegTileArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int Kp = round_up(a.F, 16);
    const int lda = Kp + 4;
    int* s_dst = reinterpret_cast<int*>(smem);            // [64] destination row of each tile row
    float* s_scale = smem + kTileRows;                    // [64] cnt as float (dgrad)
    float* A_lds = smem + 2 * kTileRows;                  // [64][lda]

    const int tile = blockIdx.x + a.tile_off;
    const int s0 = a.tile_begin[tile];
    const int nrows = a.tile_end[tile] - s0;
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;

    if (threadIdx.x < kTileRows) {
        const int r = threadIdx.x;
        const int s = s0 + r;
        s_dst[r] = r < nrows ? (a.y_use_pos ? a.s_pos[s] : s - a.sel_b) : -1;
        s_scale[r] = r < nrows ? (float)a.s_cnt[s] : 1.0f;
    }

    // ---- gather phase: each wave builds 16 tile rows ---------------------------------
    const int wr0 = wave * kRowsPerWave;
    int wn = nrows - wr0;
    wn = wn < 0 ? 0 : (wn > kRowsPerWave ? kRowsPerWave : wn);
    const int sw = s0 + wr0;
    GatherSrc g;
    g.src = a.src;
    g.F = a.F;
    g.fidx = nullptr;
    g.flo = g.fhi = 0;
    g.idx_off = 0;
    int bnd = 0;
    const int* cnt_rows = nullptr;
    g.ent = nullptr;
    g.P = nullptr;
    g.piece_off = 0;
    if (a.gather_kind == 0) {
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
    // saved segment means (backward): row s - sel_b of H, consecutive for the wave's rows
    float* gout = (a.H != nullptr && blockIdx.y == 0) ? a.H + (size_t)(sw - a.sel_b) * a.F : nullptr;
    if (!(a.ablate & 1))
        wave_gather<V, T, (V * T <= 2 ? 8 : 4)>(g, bnd, wn, cnt_rows, A_lds + wr0 * lda, lda, Kp, gout, a.F,
                                                lane);
    __syncthreads();
    if (a.W == nullptr) return;
    if (a.ablate & 2) {  // keep the gathered tile observable, skip the contraction
        if (threadIdx.x < kTileRows && threadIdx.x < nrows)
            a.Y[(size_t)s_dst[threadIdx.x] * a.N] = A_lds[threadIdx.x * lda];
        return;
    }

    // ---- MFMA phase --------------------------------------------------------------------
    const float* W = a.W;
    if (a.w_per_rel) W += (size_t)a.s_rel[s0] * a.F * a.N;
    BSrc b;
    b.W = W;
    b.K = a.F;
    b.N = a.N;
    b.trans = a.trans;
    b.ldw = a.trans ? a.F : a.N;
    const int n_base = blockIdx.y * kColTile;
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
                if (a.y_div) v = v / s_scale[row];
                a.Y[(size_t)s_dst[row] * a.N + col] = v;
            }
            if (row + 32 < nrows) {
                float v = mt.acc1[r];
                if (a.y_div) v = v / s_scale[row + 32];
                a.Y[(size_t)s_dst[row + 32] * a.N + col] = v;
            }
        }
    }
}

// ----------------------------------------------------------------------------------------
// row_tile_kernel
// ----------------------------------------------------------------------------------------
struct RowTileArgs {
    int N;              // rows of the output
    int list_kind;      // 0: ptr[N+1] array; 1: lower_bound in keys[kb, ke)
    const int* ptr;
    const int* keys;
    int kb, ke;
    const int* idx;
    int idx_off;
    const int* fidx;
    int flo, fhi;
    const int* ent;     // nullable: ragged entries (ptr / keys then index entries)
    const float* P;     // piece partials
    int piece_off;
    const float* gsrc;  // gathered rows, width G
    int G;              // output width
    const float* A;     // dense rows [N, K] (nullable: no root term)
    int K;
    const float* W;     // root (K×G, trans=0) or root viewed transposed (trans=1, W[n*K + k])
    int trans;
    const float* bias;  // nullable
    int row_lo, row_hi;
    float* out;         // [N, G]
};

__device__ __forceinline__ int lower_bound_i32(const int* keys, int lo, int hi, int v) {
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (keys[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
}

template <int V, int T>
__global__ __launch_bounds__(kThreads) void row_tile_kernel(RowTileArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int Gp = round_up(a.G, 4);
    const int ldg = Gp;
    const int Kp = round_up(a.K > 0 ? a.K : 1, 16);
    const int lda = Kp + 4;
    float* S_lds = smem;                         // [64][ldg]
    float* A_lds = smem + kTileRows * ldg;       // [64][lda]

    const int row0 = blockIdx.x * kTileRows;
    int nrows = a.N - row0;
    nrows = nrows > kTileRows ? kTileRows : nrows;
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int wr0 = wave * kRowsPerWave;
    int wn = nrows - wr0;
    wn = wn < 0 ? 0 : (wn > kRowsPerWave ? kRowsPerWave : wn);

    int bnd = 0;
    if (lane <= kRowsPerWave) {
        int i = row0 + wr0 + (lane <= wn ? lane : wn);
        if (a.list_kind == 0) bnd = a.ptr[i];
        else bnd = lower_bound_i32(a.keys, a.kb, a.ke, i);
    }
    GatherSrc g;
    g.src = a.gsrc;
    g.F = a.G;
    g.idx = a.idx;
    g.idx_off = a.idx_off;
    g.fidx = a.fidx;
    g.flo = a.flo;
    g.fhi = a.fhi;
    g.ent = a.ent;
    g.P = a.P;
    g.piece_off = a.piece_off;
    wave_gather<V, T, (V * T <= 2 ? 8 : 4)>(g, bnd, wn, nullptr, S_lds + wr0 * ldg, ldg, Gp, nullptr, 0,
                                            lane);
    const bool has_root = a.A != nullptr && a.W != nullptr;
    if (has_root) load_dense_tile(a.A, a.K, row0, nrows, A_lds, lda, Kp);
    __syncthreads();

    const int n_base = blockIdx.y * kColTile;
    const int c = lane & 31;
    const int h = lane >> 5;
    if (has_root) {
        BSrc b;
        b.W = a.W;
        b.K = a.K;
        b.N = a.G;
        b.trans = a.trans;
        b.ldw = a.trans ? a.K : a.G;
        MfmaTile mt;
        mfma_tile(mt, A_lds, lda, Kp, b, n_base, wave, lane);
        const int col = n_base + mt.nb * 32 + c;
        if (mt.active && col < a.G) {
            const float bv = a.bias != nullptr ? a.bias[col] : 0.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
#pragma unroll
                for (int half = 0; half < 2; ++half) {
                    const int row = (r & 3) + 8 * (r >> 2) + 4 * h + 32 * half;
                    if (row < nrows) {
                        const int i = row0 + row;
                        float v = S_lds[row * ldg + col];
                        if (i >= a.row_lo && i < a.row_hi) {
                            v = v + (half ? mt.acc1[r] : mt.acc0[r]);
                            if (a.bias != nullptr) v = v + bv;
                        }
                        a.out[(size_t)i * a.G + col] = v;
                    }
                }
            }
        }
    } else {
        // no root weight: out = Σ (+ bias on own rows)
        const int cols = min(kColTile, a.G - n_base);
        for (int e = threadIdx.x; e < nrows * cols; e += kThreads) {
            const int row = e / cols;
            const int col = n_base + (e - row * cols);
            const int i = row0 + row;
            float v = S_lds[row * ldg + col];
            if (a.bias != nullptr && i >= a.row_lo && i < a.row_hi) v = v + a.bias[col];
            a.out[(size_t)i * a.G + col] = v;
        }
    }
}

// ----------------------------------------------------------------------------------------
// outer_accum_kernel:  P[c] = Σ_{p in chunk c} A[a_row(p)]ᵀ ⊗ B[b_row(p)]   (M × Nn slab)
//   segment chunks: p = segment id, a_row = p - a_off (H), b_row = s_row[p] (dout)
//   row chunks:     p = node id,    a_row = p (x),          b_row = p (dout)
// ----------------------------------------------------------------------------------------
struct OuterArgs {
    const int* chunk_begin;  // nullable: row chunks [row_lo + c*chunk, ...)
    const int* chunk_end;
    int chunk_off;
    int row_lo, row_hi, chunk_rows;
    const float* A;
    int M;
    int a_off;
    const float* B;
    int Nn;
    const int* b_idx;        // nullable
    float* P;                // [nchunks][M][Nn]
    float* Pb;               // nullable: [nchunks][Nn] column sums of B (bias grad)
};

__global__ __launch_bounds__(kThreads) void outer_accum_kernel(OuterArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int ld = kColTile + 4;
    float* A_lds = smem;                 // [kSlice][ld]
    float* B_lds = smem + kSlice * ld;   // [kSlice][ld]
    int* s_brow = reinterpret_cast<int*>(smem + 2 * kSlice * ld);  // [kSlice]

    const int cidx = blockIdx.x;
    int p0, p1;
    if (a.chunk_begin != nullptr) {
        p0 = a.chunk_begin[cidx + a.chunk_off];
        p1 = a.chunk_end[cidx + a.chunk_off];
    } else {
        p0 = a.row_lo + cidx * a.chunk_rows;
        p1 = min(a.row_hi, p0 + a.chunk_rows);
    }
    const int m_base = blockIdx.y * kColTile;
    const int n_base = blockIdx.z * kColTile;
    const int mcols = min(kColTile, a.M - m_base);
    const int ncols = min(kColTile, a.Nn - n_base);
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int c = lane & 31;
    const int h = lane >> 5;
    // wave w owns blocks b = w + 4q (q < 4) of the 4 × 4 grid, b = mb*4 + nb
    f32x16 acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[q][r] = 0.0f;
    const int nb = wave;  // every q of this wave shares column strip `wave`
    float bsum = 0.0f;

    for (int ps = p0; ps < p1; ps += kSlice) {
        const int nr = min(kSlice, p1 - ps);
        if (threadIdx.x < kSlice) {
            const int p = ps + threadIdx.x;
            s_brow[threadIdx.x] = threadIdx.x < nr ? (a.b_idx ? a.b_idx[p] : p) : 0;
        }
        __syncthreads();
        for (int e = threadIdx.x; e < kSlice * kColTile; e += kThreads) {
            const int r = e / kColTile;
            const int col = e - r * kColTile;
            float av = 0.0f, bv = 0.0f;
            if (r < nr) {
                if (col < mcols) av = a.A[(size_t)(ps + r - a.a_off) * a.M + m_base + col];
                if (col < ncols) bv = a.B[(size_t)s_brow[r] * a.Nn + n_base + col];
            }
            A_lds[r * ld + col] = av;
            B_lds[r * ld + col] = bv;
        }
        __syncthreads();
        if (a.Pb != nullptr && blockIdx.y == 0 && threadIdx.x < kColTile) {
            for (int r = 0; r < nr; ++r) bsum += B_lds[r * ld + threadIdx.x];
        }
#pragma unroll 4
        for (int t = 0; t < kSlice / 2; ++t) {
            const int k = h * (kSlice / 2) + t;
            const float bv = B_lds[k * ld + nb * 32 + c];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float av = A_lds[k * ld + q * 32 + c];
                acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[q], 0, 0, 0);
            }
        }
        __syncthreads();
    }
    float* P = a.P + (size_t)cidx * a.M * a.Nn;
    const int col = n_base + nb * 32 + c;
    if (col < a.Nn) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m_base + q * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (m < a.M) P[(size_t)m * a.Nn + col] = acc[q][r];
            }
        }
    }
    if (a.Pb != nullptr && blockIdx.y == 0 && threadIdx.x < ncols)
        a.Pb[(size_t)cidx * a.Nn + n_base + threadIdx.x] = bsum;
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
};

__global__ __launch_bounds__(kThreads) void reduce_slabs_kernel(ReduceArgs a) {
    const int g = blockIdx.x;
    const int e = blockIdx.y * kThreads + threadIdx.x;
    if (e >= a.elems) return;
    int c0 = 0, c1 = a.nchunks;
    if (a.gptr != nullptr) {
        c0 = a.gptr[a.g_base + g] - a.g_off;
        c1 = a.gptr[a.g_base + g + 1] - a.g_off;
    }
    float s = 0.0f;
    for (int c = c0; c < c1; ++c) s += a.P[(size_t)c * a.elems + e];
    const int d = a.gdst != nullptr ? a.gdst[a.g_base + g] : g;
    a.dst[(size_t)d * a.elems + e] = s;
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

struct TimedLaunch {
    int kind;
    hipStream_t stream;
    hipEvent_t start = nullptr, stop = nullptr;
    bool on;
    TimedLaunch(int k, hipStream_t s) : kind(k), stream(s) {
        std::lock_guard<std::mutex> lk(g_timing_mu);
        on = g_timing_on;
        if (on && hipEventCreate(&start) == hipSuccess && hipEventCreate(&stop) == hipSuccess)
            (void)hipEventRecord(start, stream);
        else
            on = false;
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
static void launch_seg(const SegTileArgs& a, int ntiles, int ncoltiles, hipStream_t st) {
    const int Kp = round_up(a.F, 16);
    const size_t lds = (size_t)(2 * kTileRows + kTileRows * (Kp + 4)) * sizeof(float);
    hipLaunchKernelGGL((seg_tile_kernel<V, T>), dim3(ntiles, ncoltiles), dim3(kThreads), lds, st, a);
}

template <int V, int T>
static void launch_row(const RowTileArgs& a, int nrowtiles, int ncoltiles, hipStream_t st) {
    const int Gp = round_up(a.G, 4);
    const int Kp = round_up(a.K > 0 ? a.K : 1, 16);
    const bool has_root = a.A != nullptr && a.W != nullptr;
    const size_t lds = (size_t)(kTileRows * Gp + (has_root ? kTileRows * (Kp + 4) : 0)) * sizeof(float);
    hipLaunchKernelGGL((row_tile_kernel<V, T>), dim3(nrowtiles, ncoltiles), dim3(kThreads), lds, st, a);
}

template <int V, int T>
static void launch_piece(const PieceArgs& a, hipStream_t st) {
    const int n = a.k_hi - a.k_lo;
    hipLaunchKernelGGL((piece_sum_kernel<V, T>), dim3((n + kWaves - 1) / kWaves), dim3(kThreads), 0, st, a);
}

static bool g_exact_order = false;  // MPGNN_OPT_EXACT_ORDER: no ragged pieces anywhere
static int g_ablate = 0;            // MPGNN_OPT_ABLATE (debug/profiling only)

struct Selection {
    int64_t d_lo = 0, d_hi = 0;
    int sel_b = 0, sel_e = 0;
    int t_lo = 0, t_hi = 0;
    int c_lo = 0, c_hi = 0;
    int sp_lo = 0, sp_hi = 0;   // seg-list pieces of the selection
    int tap_lo = 0, tap_hi = 0; // ta-list pieces (mode SINGLE)
    int ta_e_lo = 0, ta_e_hi = 0; // ta entry range (mode SINGLE)
    bool all_segments = false;  // selection covers every local segment
};

static int32_t make_selection(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R, Selection* s) {
    int32_t st = select_relations(p, mode, relation, R, &s->d_lo, &s->d_hi);
    if (st != MPGNN_OK) return st;
    if (p->nrel == 0) return MPGNN_OK;
    s->sel_b = p->rel_seg_ptr[s->d_lo];
    s->sel_e = p->rel_seg_ptr[s->d_hi];
    s->t_lo = p->rel_tile_ptr[s->d_lo];
    s->t_hi = p->rel_tile_ptr[s->d_hi];
    s->c_lo = p->rel_chunk_ptr[s->d_lo];
    s->c_hi = p->rel_chunk_ptr[s->d_hi];
    s->sp_lo = p->rel_seg_piece_ptr[s->d_lo];
    s->sp_hi = p->rel_seg_piece_ptr[s->d_hi];
    s->tap_lo = p->rel_ta_piece_ptr[s->d_lo];
    s->tap_hi = p->rel_ta_piece_ptr[s->d_hi];
    s->ta_e_lo = p->rel_ta_ent_ptr[s->d_lo];
    s->ta_e_hi = p->rel_ta_ent_ptr[s->d_hi];
    s->all_segments = (s->sel_b == 0 && s->sel_e == p->S);
    return MPGNN_OK;
}

static size_t align256(size_t b) { return (b + 255) / 256 * 256; }

struct RootChunks {
    int rows_lo = 0, rows_hi = 0, chunk = 256, n = 0;
};

static RootChunks root_chunks(int64_t lo, int64_t hi) {
    RootChunks r;
    r.rows_lo = (int)lo;
    r.rows_hi = (int)hi;
    const int rows = (int)(hi - lo);
    int ch = std::max(kChunkRows, round_up((rows + 1023) / 1024, kSlice));
    r.chunk = ch;
    r.n = rows > 0 ? (rows + ch - 1) / ch : 0;
    return r;
}

// Workspace: forward and backward regions are used by different calls, so they overlap.
struct WsLayout {
    size_t y = 0, pseg = 0, prw = 0;                       // forward
    size_t g = 0, h = 0, pdx = 0, p = 0, proot = 0, pb = 0; // backward
    size_t total = 0;
};

static WsLayout ws_layout(const mpgnn_plan* p, int32_t mode, const Selection& s, int F_in, int F_out,
                          const RootChunks& rc) {
    WsLayout w;
    const size_t S_sel = (size_t)(s.sel_e - s.sel_b);
    const size_t y_rows = (mode == MPGNN_MODE_ALL) ? (size_t)p->S : S_sel;
    size_t off = 0;
    w.y = off; off += align256(y_rows * F_out * sizeof(float));
    w.pseg = off; off += align256((size_t)(s.sp_hi - s.sp_lo) * F_in * sizeof(float));
    w.prw = off; off += align256((mode == MPGNN_MODE_ALL ? p->rw_l.piece_b.size() : 0) * F_out * sizeof(float));
    const size_t fwd = off;
    off = 0;
    const size_t dx_pieces = (mode == MPGNN_MODE_ALL) ? p->t_l.piece_b.size() : (size_t)(s.tap_hi - s.tap_lo);
    w.g = off; off += align256(S_sel * F_in * sizeof(float));
    w.h = off; off += align256(S_sel * F_in * sizeof(float));
    w.pdx = off; off += align256(dx_pieces * F_in * sizeof(float));
    w.p = off; off += align256((size_t)(s.c_hi - s.c_lo) * F_in * F_out * sizeof(float));
    w.proot = off; off += align256((size_t)rc.n * F_in * F_out * sizeof(float));
    w.pb = off; off += align256((size_t)rc.n * F_out * sizeof(float));
    w.total = std::max<size_t>(std::max(fwd, off), 256);
    return w;
}

static int32_t check_common(const mpgnn_plan* p, int F_in, int F_out) {
    if (!p) return arg_error("NULL plan");
    if (!p->d.block) {
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

// Forward segment tiles: Y[seg] = mean(src over seg) @ W_rel(seg)   (W == nullptr: H only)
static int32_t run_seg_forward(const mpgnn_plan* p, int32_t mode, const Selection& s, const float* x, int F_in,
                               const float* W, int F_out, float* Y, float* H, float* Pseg, bool exact,
                               int kind, hipStream_t strm) {
    const int ntiles = s.t_hi - s.t_lo;
    if (ntiles == 0) return MPGNN_OK;
    int V, T;
    pick_vt(F_in, &V, &T);
    const bool ragged = !exact && s.sp_hi > s.sp_lo;
    if (ragged) {
        PieceArgs pa{};
        pa.pb = p->d.seg_pb;
        pa.pe = p->d.seg_pe;
        pa.k_lo = s.sp_lo;
        pa.k_hi = s.sp_hi;
        pa.src = x;
        pa.F = F_in;
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
    a.gather_kind = 0;
    a.src = x;
    a.F = F_in;
    a.s_ptr = ragged ? p->d.seg_ent_ptr : p->d.s_ptr;
    a.e_col = p->d.e_col;
    a.s_row = p->d.s_row;
    a.s_cnt = p->d.s_cnt;
    a.s_rel = p->d.s_rel;
    a.s_pos = p->d.s_pos;
    a.ent = ragged ? p->d.seg_ent : nullptr;
    a.P = Pseg;
    a.piece_off = s.sp_lo;
    a.W = W;
    a.w_per_rel = (mode == MPGNN_MODE_ALL);
    a.trans = 0;
    a.N = W ? F_out : 1;
    a.Y = Y;
    a.y_use_pos = (mode == MPGNN_MODE_ALL);
    a.y_div = 0;
    a.sel_b = s.sel_b;
    a.H = H;
    a.ablate = g_ablate;
    const int ncol = W ? (F_out + kColTile - 1) / kColTile : 1;
    TimedLaunch tl(kind, strm);
    MPGNN_VT_DISPATCH(V, T, launch_seg, a, ntiles, ncol, strm);
    return hip_check(hipGetLastError(), "seg_tile_kernel launch");
}

}  // namespace mpgnn

using namespace mpgnn;

extern "C" {

int32_t mpgnn_set_option(int32_t option, int64_t value) {
    if (option == MPGNN_OPT_EXACT_ORDER) {
        g_exact_order = value != 0;
        return MPGNN_OK;
    }
    if (option == MPGNN_OPT_ABLATE) {
        g_ablate = (int)value;
        return MPGNN_OK;
    }
    return arg_error("unknown option " + std::to_string(option));
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
    return run_seg_forward(p, mode, s, x, F, nullptr, 1, nullptr, h, nullptr, true, MPGNN_K_MEAN,
                           static_cast<hipStream_t>(stream));
}

int32_t mpgnn_rgcn_workspace_bytes(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R,
                                   int32_t F_in, int32_t F_out, int64_t row_lo, int64_t row_hi,
                                   int64_t* bytes) {
    if (!p || !bytes) return arg_error("NULL argument");
    Selection s;
    int32_t st = make_selection(p, mode, relation, R, &s);
    if (st != MPGNN_OK) return st;
    clamp_rows(p, &row_lo, &row_hi);
    WsLayout w = ws_layout(p, mode, s, std::max(F_in, 1), std::max(F_out, 1), root_chunks(row_lo, row_hi));
    *bytes = (int64_t)w.total;
    return MPGNN_OK;
}

int32_t mpgnn_rgcn_fwd(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R, const float* x,
                       int32_t F_in, const float* weight, const float* root, const float* bias,
                       int32_t F_out, int64_t row_lo, int64_t row_hi, float* out, float* h_save,
                       void* workspace, void* stream) {
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
    const WsLayout w = ws_layout(p, mode, s, F_in, F_out, rc);
    char* ws = static_cast<char*>(workspace);
    float* Y = reinterpret_cast<float*>(ws + w.y);
    const bool exact = g_exact_order;
    const int ncol = (F_out + kColTile - 1) / kColTile;

    // 1) Y[seg] = mean(x over seg) @ W_rel(seg)     (+ h_save = the means)
    st = run_seg_forward(p, mode, s, x, F_in, weight, F_out, Y, h_save, reinterpret_cast<float*>(ws + w.pseg),
                         exact, MPGNN_K_SEG_FWD, strm);
    if (st != MPGNN_OK) return st;

    // 2) out[i] = Σ_{seg of row i, relation order} Y[seg] + x[i] @ root + bias
    int V, T;
    pick_vt(F_out, &V, &T);
    RowTileArgs a{};
    a.N = (int)p->N;
    a.P = reinterpret_cast<float*>(ws + w.prw);
    if (mode == MPGNN_MODE_ALL) {
        const bool ragged = !exact && !p->rw_l.piece_b.empty();
        const int* fidx = s.all_segments ? nullptr : p->d.rw_seg;
        if (ragged) {
            PieceArgs pa{};
            pa.pb = p->d.rw_pb;
            pa.pe = p->d.rw_pe;
            pa.k_lo = 0;
            pa.k_hi = (int)p->rw_l.piece_b.size();
            pa.src = Y;
            pa.F = F_out;
            pa.fidx = fidx;
            pa.flo = s.sel_b;
            pa.fhi = s.sel_e;
            pa.P = reinterpret_cast<float*>(ws + w.prw);
            TimedLaunch tl(MPGNN_K_PIECE, strm);
            MPGNN_VT_DISPATCH(V, T, launch_piece, pa, strm);
            if ((st = hip_check(hipGetLastError(), "piece_sum_kernel(rw) launch")) != MPGNN_OK) return st;
        }
        a.list_kind = 0;
        a.ptr = ragged ? p->d.rw_ent_ptr : p->d.rw_ptr;
        a.ent = ragged ? p->d.rw_ent : nullptr;
        a.idx = nullptr;
        a.idx_off = 0;
        a.fidx = fidx;
        a.flo = s.sel_b;
        a.fhi = s.sel_e;
    } else {
        a.list_kind = 1;  // at most one segment per row: no pieces
        a.keys = p->d.s_row;
        a.kb = s.sel_b;
        a.ke = s.sel_e;
        a.idx = nullptr;
        a.idx_off = s.sel_b;
        a.fidx = nullptr;
        a.ent = nullptr;
    }
    a.gsrc = Y;
    a.G = F_out;
    a.A = root ? x : nullptr;
    a.K = F_in;
    a.W = root;
    a.trans = 0;
    a.bias = bias;
    a.row_lo = (int)row_lo;
    a.row_hi = (int)row_hi;
    a.out = out;
    const int nrt = (int)((p->N + kTileRows - 1) / kTileRows);
    TimedLaunch tl(MPGNN_K_ROW_FWD, strm);
    MPGNN_VT_DISPATCH(V, T, launch_row, a, nrt, ncol, strm);
    return hip_check(hipGetLastError(), "row_tile_kernel launch");
}

int32_t mpgnn_rgcn_bwd(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R, const float* x,
                       int32_t F_in, const float* weight, const float* root, int32_t F_out,
                       const float* h_save, const float* grad_out, int64_t row_lo, int64_t row_hi,
                       float* grad_x, float* grad_weight, float* grad_root, float* grad_bias,
                       void* workspace, void* stream) {
    int32_t st = check_common(p, F_in, F_out);
    if (st != MPGNN_OK) return st;
    Selection s;
    if ((st = make_selection(p, mode, relation, R, &s)) != MPGNN_OK) return st;
    if (!grad_out || !weight) return arg_error("NULL grad_out or weight");
    clamp_rows(p, &row_lo, &row_hi);
    hipStream_t strm = static_cast<hipStream_t>(stream);
    const RootChunks rc = root_chunks(row_lo, row_hi);
    const WsLayout w = ws_layout(p, mode, s, F_in, F_out, rc);
    char* ws = static_cast<char*>(workspace);
    if (!ws) return arg_error("NULL workspace");
    const int ntiles = s.t_hi - s.t_lo;
    const size_t wsize = (size_t)F_in * F_out;
    const bool exact = g_exact_order;

    // ---- grad_x = Σ_r A_rᵀ ((dout @ W_rᵀ) / cnt) + dout @ rootᵀ ----------------------
    if (grad_x != nullptr && p->N > 0) {
        float* G = reinterpret_cast<float*>(ws + w.g);
        if (ntiles > 0) {
            int V, T;
            pick_vt(F_out, &V, &T);
            SegTileArgs a{};
            a.tile_begin = p->d.tile_begin;
            a.tile_end = p->d.tile_end;
            a.tile_off = s.t_lo;
            a.gather_kind = 1;
            a.src = grad_out;
            a.F = F_out;
            a.s_ptr = p->d.s_ptr;
            a.e_col = p->d.e_col;
            a.s_row = p->d.s_row;
            a.s_cnt = p->d.s_cnt;
            a.s_rel = p->d.s_rel;
            a.s_pos = p->d.s_pos;
            a.W = weight;
            a.w_per_rel = (mode == MPGNN_MODE_ALL);
            a.trans = 1;
            a.N = F_in;
            a.Y = G;
            a.y_use_pos = 0;
            a.y_div = 1;
            a.sel_b = s.sel_b;
            a.H = nullptr;
            const int ncol = (F_in + kColTile - 1) / kColTile;
            TimedLaunch tl(MPGNN_K_SEG_DGRAD, strm);
            MPGNN_VT_DISPATCH(V, T, launch_seg, a, ntiles, ncol, strm);
            if ((st = hip_check(hipGetLastError(), "seg_tile_kernel(dgrad) launch")) != MPGNN_OK) return st;
        }
        int V, T;
        pick_vt(F_in, &V, &T);
        RowTileArgs a{};
        a.N = (int)p->N;
        a.P = reinterpret_cast<float*>(ws + w.pdx);
        PieceArgs pa{};
        pa.src = G;
        pa.F = F_in;
        pa.idx_off = s.sel_b;
        pa.P = reinterpret_cast<float*>(ws + w.pdx);
        if (mode == MPGNN_MODE_ALL) {
            const bool ragged = !exact && !p->t_l.piece_b.empty();
            const int* fidx = s.all_segments ? nullptr : p->d.t_seg;
            if (ragged && ntiles > 0) {
                pa.pb = p->d.t_pb;
                pa.pe = p->d.t_pe;
                pa.k_lo = 0;
                pa.k_hi = (int)p->t_l.piece_b.size();
                pa.idx = p->d.t_seg;
                pa.fidx = fidx;
                pa.flo = s.sel_b;
                pa.fhi = s.sel_e;
                TimedLaunch tl(MPGNN_K_PIECE, strm);
                MPGNN_VT_DISPATCH(V, T, launch_piece, pa, strm);
                if ((st = hip_check(hipGetLastError(), "piece_sum_kernel(t) launch")) != MPGNN_OK) return st;
            }
            a.list_kind = 0;
            a.ptr = ragged ? p->d.t_ent_ptr : p->d.t_ptr;
            a.ent = ragged ? p->d.t_ent : nullptr;
            a.idx = p->d.t_seg;
            a.idx_off = s.sel_b;
            a.fidx = fidx;
            a.flo = s.sel_b;
            a.fhi = s.sel_e;
            a.piece_off = 0;
        } else {
            const bool ragged = !exact;
            if (ragged && s.tap_hi > s.tap_lo) {
                pa.pb = p->d.ta_pb;
                pa.pe = p->d.ta_pe;
                pa.k_lo = s.tap_lo;
                pa.k_hi = s.tap_hi;
                pa.idx = p->d.ta_seg;
                TimedLaunch tl(MPGNN_K_PIECE, strm);
                MPGNN_VT_DISPATCH(V, T, launch_piece, pa, strm);
                if ((st = hip_check(hipGetLastError(), "piece_sum_kernel(ta) launch")) != MPGNN_OK) return st;
            }
            a.list_kind = 1;
            if (ragged) {
                a.keys = p->d.ta_key;
                a.kb = s.ta_e_lo;
                a.ke = s.ta_e_hi;
                a.ent = p->d.ta_ent;
                a.piece_off = s.tap_lo;
            } else {
                a.keys = p->d.ta_col;
                a.kb = (s.d_hi > s.d_lo) ? p->rel_edge_ptr[s.d_lo] : 0;
                a.ke = (s.d_hi > s.d_lo) ? p->rel_edge_ptr[s.d_hi] : 0;
                a.ent = nullptr;
            }
            a.idx = p->d.ta_seg;
            a.idx_off = s.sel_b;
            a.fidx = nullptr;
        }
        a.gsrc = G;
        a.G = F_in;
        a.A = root ? grad_out : nullptr;
        a.K = F_out;
        a.W = root;
        a.trans = 1;
        a.bias = nullptr;
        a.row_lo = (int)row_lo;
        a.row_hi = (int)row_hi;
        a.out = grad_x;
        const int nrt = (int)((p->N + kTileRows - 1) / kTileRows);
        const int ncol = (F_in + kColTile - 1) / kColTile;
        {
            TimedLaunch tl(MPGNN_K_ROW_DX, strm);
            MPGNN_VT_DISPATCH(V, T, launch_row, a, nrt, ncol, strm);
        }
        if ((st = hip_check(hipGetLastError(), "row_tile_kernel(dx) launch")) != MPGNN_OK) return st;
    }

    const int mt = (F_in + kColTile - 1) / kColTile;
    const int nt = (F_out + kColTile - 1) / kColTile;
    const size_t outer_lds = (size_t)(2 * kSlice * (kColTile + 4) + kSlice) * sizeof(float);

    // ---- grad_weight[r] = Σ_{seg of r} h_segᵀ dout[node_1(seg)] -------------------------
    if (grad_weight != nullptr) {
        const size_t wbytes = (mode == MPGNN_MODE_ALL ? (size_t)std::max(R, 0) : 1) * wsize * sizeof(float);
        if ((st = hip_check(hipMemsetAsync(grad_weight, 0, wbytes, strm), "memset grad_weight")) != MPGNN_OK)
            return st;
        const int nch = s.c_hi - s.c_lo;
        if (nch > 0) {
            const float* H = h_save;
            if (H == nullptr) {
                float* Hw = reinterpret_cast<float*>(ws + w.h);
                st = run_seg_forward(p, mode, s, x, F_in, nullptr, 1, nullptr, Hw, reinterpret_cast<float*>(ws + w.pdx),
                                     true, MPGNN_K_MEAN, strm);
                if (st != MPGNN_OK) return st;
                H = Hw;
            }
            float* P = reinterpret_cast<float*>(ws + w.p);
            OuterArgs o{};
            o.chunk_begin = p->d.chunk_begin;
            o.chunk_end = p->d.chunk_end;
            o.chunk_off = s.c_lo;
            o.A = H;
            o.M = F_in;
            o.a_off = s.sel_b;
            o.B = grad_out;
            o.Nn = F_out;
            o.b_idx = p->d.s_row;
            o.P = P;
            o.Pb = nullptr;
            {
                TimedLaunch tl(MPGNN_K_OUTER, strm);
                hipLaunchKernelGGL(outer_accum_kernel, dim3(nch, mt, nt), dim3(kThreads), outer_lds, strm, o);
            }
            if ((st = hip_check(hipGetLastError(), "outer_accum_kernel(dW) launch")) != MPGNN_OK) return st;
            ReduceArgs r{};
            r.P = P;
            r.elems = (int)wsize;
            r.dst = grad_weight;
            const int ey = (int)((wsize + kThreads - 1) / kThreads);
            TimedLaunch tl(MPGNN_K_REDUCE, strm);
            if (mode == MPGNN_MODE_ALL) {
                r.gptr = p->d.rel_chunk_ptr;
                r.g_off = s.c_lo;
                r.gdst = p->d.rel_val32;
                r.g_base = (int)s.d_lo;
                hipLaunchKernelGGL(reduce_slabs_kernel, dim3((int)(s.d_hi - s.d_lo), ey), dim3(kThreads), 0, strm, r);
            } else {
                r.gptr = nullptr;
                r.nchunks = nch;
                r.gdst = nullptr;
                hipLaunchKernelGGL(reduce_slabs_kernel, dim3(1, ey), dim3(kThreads), 0, strm, r);
            }
            if ((st = hip_check(hipGetLastError(), "reduce_slabs_kernel(dW) launch")) != MPGNN_OK) return st;
        }
    }

    // ---- grad_root = xᵀ dout, grad_bias = Σ dout  (rows [row_lo, row_hi)) -------------
    if (grad_root != nullptr || grad_bias != nullptr) {
        if (rc.n == 0) {
            if (grad_root && (st = hip_check(hipMemsetAsync(grad_root, 0, wsize * sizeof(float), strm), "memset")))
                return st;
            if (grad_bias && (st = hip_check(hipMemsetAsync(grad_bias, 0, F_out * sizeof(float), strm), "memset")))
                return st;
            return MPGNN_OK;
        }
        if (!x) return arg_error("NULL x");
        float* P = reinterpret_cast<float*>(ws + w.proot);
        float* Pb = reinterpret_cast<float*>(ws + w.pb);
        OuterArgs o{};
        o.chunk_begin = nullptr;
        o.row_lo = rc.rows_lo;
        o.row_hi = rc.rows_hi;
        o.chunk_rows = rc.chunk;
        o.A = x;
        o.M = F_in;
        o.a_off = 0;
        o.B = grad_out;
        o.Nn = F_out;
        o.b_idx = nullptr;
        o.P = P;
        o.Pb = grad_bias ? Pb : nullptr;
        {
            TimedLaunch tl(MPGNN_K_OUTER, strm);
            hipLaunchKernelGGL(outer_accum_kernel, dim3(rc.n, grad_root ? mt : 1, nt), dim3(kThreads), outer_lds, strm, o);
        }
        if ((st = hip_check(hipGetLastError(), "outer_accum_kernel(root) launch")) != MPGNN_OK) return st;
        if (grad_root) {
            ReduceArgs r{};
            r.P = P;
            r.elems = (int)wsize;
            r.nchunks = rc.n;
            r.dst = grad_root;
            TimedLaunch tl(MPGNN_K_REDUCE, strm);
            hipLaunchKernelGGL(reduce_slabs_kernel, dim3(1, (int)((wsize + kThreads - 1) / kThreads)), dim3(kThreads),
                               0, strm, r);
            if ((st = hip_check(hipGetLastError(), "reduce_slabs_kernel(root) launch")) != MPGNN_OK) return st;
        }
        if (grad_bias) {
            ReduceArgs r{};
            r.P = Pb;
            r.elems = F_out;
            r.nchunks = rc.n;
            r.dst = grad_bias;
            TimedLaunch tl(MPGNN_K_REDUCE, strm);
            hipLaunchKernelGGL(reduce_slabs_kernel, dim3(1, (F_out + kThreads - 1) / kThreads), dim3(kThreads), 0,
                               strm, r);
            if ((st = hip_check(hipGetLastError(), "reduce_slabs_kernel(bias) launch")) != MPGNN_OK) return st;
        }
    }
    return MPGNN_OK;
}

int32_t mpgnn_timing_enable(int32_t on) {
    std::lock_guard<std::mutex> lk(g_timing_mu);
    g_timing_on = on != 0;
    return MPGNN_OK;
}

int32_t mpgnn_timing_reset(void) {
    std::lock_guard<std::mutex> lk(g_timing_mu);
    for (auto& r : g_timing) {
        (void)hipEventDestroy(r.start);
        (void)hipEventDestroy(r.stop);
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
