// plan_device.hip — the graph plan built on the GPU from device-resident edge arrays
// (mpgnn_plan_create_device, include/mpgnn_rgcn.h).
//
// Same tables, bit for bit, as the host builder (plan.cpp) and its numpy restatement
// (oracle/plan_oracle.py); tests/test_plan_device.py compares all three. The reference re-derives
// this bookkeeping on every call (`edge_index[:, edge_type == r]`, mp_rgcn_layer.py:29-35, :231,
// and per relation in the RGCNConv loop ≙ :250-251); here it is built once per graph, on the card
// the graph already lives on:
//
//   - every stable counting sort of plan.cpp is a stable LSD radix sort (rocPRIM) of a packed key
//     whose value payload is the position in the previous order, so ties keep that order;
//   - every prefix sum is a device scan; run starts come from adjacent-key comparisons;
//   - the greedy chunking of the flat lists (plan.cpp build_flat), a sequential scan on the host,
//     is a pointer walk over runs: the next chunk start of every run is found by binary search,
//     then the first chunk start of each 256-run block is iterated to its fixed point (block b's
//     walk from its entry gives block b+1's entry; entry 0 is exact, so iteration i makes entries
//     0..i exact and a pass without change is the answer — in practice 2-3 passes), and chunk and
//     workgroup-group tables follow from prefix sums over runs and list elements.
//
// Only the per-relation tables (O(R)), the tile/chunk lists of the weight-gradient passes
// (O(S/32)) and the table sizes come back to the host; the big tables stay on the device and are
// copied into the plan's host vectors only when a table is exported (tests, mpgnn_plan_export).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <limits>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "plan_internal.h"

namespace mpgnn {
namespace {

struct BuildError : std::runtime_error {
    int32_t code;
    BuildError(int32_t c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define DCHECK(x)                                                                                      \
    do {                                                                                               \
        hipError_t e_ = (x);                                                                           \
        if (e_ != hipSuccess)                                                                          \
            throw BuildError(e_ == hipErrorOutOfMemory ? MPGNN_ERR_ALLOC : MPGNN_ERR_HIP,              \
                             std::string(#x) + ": " + hipGetErrorString(e_));                          \
    } while (0)

constexpr int kT = 256;
constexpr int kWalkBlock = 256;  // runs per block of the chunk-start walk

inline dim3 grid_for(int64_t n) {
    int64_t b = (n + kT - 1) / kT;
    return dim3((unsigned)std::min<int64_t>(std::max<int64_t>(b, 1), 1 << 20));
}

#define FOR_EACH(i, n) \
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)(n); i += (int64_t)gridDim.x * blockDim.x)

// first index i in [lo, hi) with a[i] > v (hi if none); a ascending
template <class T, class V>
__device__ inline int64_t upper_bound_dev(const T* a, int64_t lo, int64_t hi, V v) {
    while (lo < hi) {
        const int64_t m = (lo + hi) >> 1;
        if (a[m] > v) hi = m; else lo = m + 1;
    }
    return lo;
}
// first index i in [lo, hi) with a[i] >= v
template <class T, class V>
__device__ inline int64_t lower_bound_dev(const T* a, int64_t lo, int64_t hi, V v) {
    while (lo < hi) {
        const int64_t m = (lo + hi) >> 1;
        if (a[m] < v) lo = m + 1; else hi = m;
    }
    return lo;
}

// ---- kernels: relations, valid edges, segments ---------------------------------------------
__global__ void k_rel_dense(const int64_t* n1, const int64_t* n2, const int64_t* et, int64_t E, int64_t N,
                            const int64_t* rel_vals, int64_t R, int32_t* rel_d, int32_t* valid, uint8_t* invalid) {
    FOR_EACH(e, E) {
        const int32_t d = (int32_t)lower_bound_dev(rel_vals, 0, R, et[e]);
        rel_d[e] = d;
        const int64_t a = n1[e], b = n2[e];
        const bool ok = a >= 0 && a < N && b >= 0 && b < N;
        valid[e] = ok ? 1 : 0;
        if (!ok) invalid[d] = 1;
    }
}

template <class K>
__global__ void k_row_keys(const int32_t* ids, int64_t V, const int32_t* rel_d, const int64_t* n1, int64_t N, K* keys) {
    FOR_EACH(a, V) {
        const int32_t e = ids[a];
        keys[a] = (K)rel_d[e] * (K)N + (K)n1[e];
    }
}

template <class K>
__global__ void k_seg_heads(const K* keys, const int32_t* ids, int64_t V, const int64_t* n1, const int64_t* n2,
                            int64_t lo, int64_t hi, int32_t side, int32_t* head, int32_t* loc) {
    FOR_EACH(a, V) {
        head[a] = (a == 0 || keys[a] != keys[a - 1]) ? 1 : 0;
        const int32_t e = ids[a];
        const int64_t k = side == MPGNN_SHARD_ROWS ? n1[e] : n2[e];
        loc[a] = (k >= lo && k < hi) ? 1 : 0;
    }
}

__global__ void k_gstart(int64_t V, const int32_t* head, const int32_t* hx, int32_t* gstart, int64_t G) {
    FOR_EACH(a, V) if (head[a]) gstart[hx[a]] = (int32_t)a;
    if (blockIdx.x == 0 && threadIdx.x == 0) gstart[G] = (int32_t)V;
}

__global__ void k_kept(int64_t G, const int32_t* gstart, const int32_t* lx, int32_t* kept) {
    FOR_EACH(g, G) kept[g] = lx[gstart[g + 1]] > lx[gstart[g]] ? 1 : 0;
}

__global__ void k_fill_edges(int64_t V, const int32_t* ids, const int32_t* head, const int32_t* hx, const int32_t* loc,
                             const int32_t* lx, const int32_t* sidx, const int64_t* n2, int32_t* e_col, int32_t* e_id,
                             int32_t* seg_of_edge) {
    FOR_EACH(a, V) {
        if (!loc[a]) continue;
        const int32_t g = hx[a] + head[a] - 1;
        const int32_t w = lx[a], e = ids[a];
        e_col[w] = (int32_t)n2[e];
        e_id[w] = e;
        seg_of_edge[w] = sidx[g];
    }
}

__global__ void k_fill_segs(int64_t G, const int32_t* gstart, const int32_t* kept, const int32_t* sidx, const int32_t* lx,
                            const int32_t* ids, const int64_t* n1, const int32_t* rel_d, const int32_t* rel_val32,
                            int32_t* s_row, int32_t* seg_d, int32_t* s_rel, int32_t* s_cnt, int32_t* s_ptr) {
    FOR_EACH(g, G) {
        if (!kept[g]) continue;
        const int32_t s = sidx[g], a0 = gstart[g];
        const int32_t e0 = ids[a0];
        s_row[s] = (int32_t)n1[e0];
        seg_d[s] = rel_d[e0];
        s_rel[s] = rel_val32[rel_d[e0]];
        s_cnt[s] = gstart[g + 1] - a0;  // GLOBAL count of (row, relation)
        s_ptr[s] = lx[a0];
    }
}

// out[i] = lower_bound(sorted[0, n), i) for i in [0, m)
__global__ void k_lower_bound_iota(const int32_t* sorted, int64_t n, int32_t* out, int64_t m) {
    FOR_EACH(i, m) out[i] = (int32_t)lower_bound_dev(sorted, 0, n, (int32_t)i);
}

__global__ void k_gather(const int32_t* src, const int32_t* idx, int64_t n, int32_t* out) {
    FOR_EACH(i, n) out[i] = src[idx[i]];
}

__global__ void k_set(int32_t* p, int64_t i, int32_t v) {
    if (blockIdx.x == 0 && threadIdx.x == 0) p[i] = v;
}

__global__ void k_iota(int32_t* p, int64_t n) {
    FOR_EACH(i, n) p[i] = (int32_t)i;
}

// out[n] = out[n-1] + in[n-1] after an exclusive scan of n elements (the total)
__global__ void k_scan_total(const int32_t* in, int32_t* out, int64_t n) {
    if (blockIdx.x == 0 && threadIdx.x == 0) out[n] = n > 0 ? out[n - 1] + in[n - 1] : 0;
}

// ---- multi-edge segments ---------------------------------------------------------------------
__global__ void k_multi_flags(int64_t S, const int32_t* s_ptr, const int32_t* s_cnt, int32_t* mflag, int32_t* mlen) {
    FOR_EACH(s, S) {
        const int32_t loc = s_ptr[s + 1] - s_ptr[s];
        const bool multi = !(loc == 1 && s_cnt[s] == 1);
        mflag[s] = multi ? 1 : 0;
        mlen[s] = multi ? loc : 0;
    }
}

__global__ void k_multi_segs(int64_t S, const int32_t* s_ptr, const int32_t* s_cnt, const int32_t* e_col, const int32_t* mflag,
                             const int32_t* m_id, const int32_t* m_off, int32_t* s_src, int32_t* m_cnt, int32_t* m_ptr) {
    FOR_EACH(s, S) {
        if (!mflag[s]) {
            s_src[s] = e_col[s_ptr[s]];
            continue;
        }
        const int32_t m = m_id[s];
        s_src[s] = -m - 1;
        m_cnt[m] = s_cnt[s];
        m_ptr[m] = m_off[s];
    }
}

__global__ void k_multi_edges(int64_t E, const int32_t* seg_of_edge, const int32_t* s_ptr, const int32_t* mflag,
                              const int32_t* m_off, const int32_t* e_col, int32_t* em_col) {
    FOR_EACH(w, E) {
        const int32_t s = seg_of_edge[w];
        if (mflag[s]) em_col[m_off[s] + (int32_t)w - s_ptr[s]] = e_col[w];
    }
}

__global__ void k_rel_m_ptr(int64_t R, const int32_t* rel_seg_ptr, int64_t S, const int32_t* m_id, int32_t Sm, int32_t* out) {
    FOR_EACH(d, R + 1) out[d] = (d < R && rel_seg_ptr[d] < S) ? m_id[rel_seg_ptr[d]] : Sm;
}

__global__ void k_scatter_pos(const int32_t* perm, int64_t n, int32_t* pos) {
    FOR_EACH(q, n) pos[perm[q]] = (int32_t)q;
}

// ---- transposed orders -------------------------------------------------------------------------
__global__ void k_tseg_keys(int64_t E, const int32_t* by_col, const int32_t* seg_of_edge, const int32_t* seg_d, int32_t* t_seg,
                            int32_t* key_d) {
    FOR_EACH(q, E) {
        const int32_t s = seg_of_edge[by_col[q]];
        t_seg[q] = s;
        key_d[q] = seg_d[s];
    }
}

__global__ void k_ta(int64_t E, const int32_t* by_rel_col, const int32_t* e_col, const int32_t* seg_of_edge, int32_t* ta_col,
                     int32_t* ta_seg) {
    FOR_EACH(q, E) {
        const int32_t v = by_rel_col[q];
        ta_col[q] = e_col[v];
        ta_seg[q] = seg_of_edge[v];
    }
}

__global__ void k_ta_heads(int64_t E, const int32_t* td, const int32_t* ta_col, int32_t* head) {
    FOR_EACH(q, E) head[q] = (q == 0 || td[q] != td[q - 1] || ta_col[q] != ta_col[q - 1]) ? 1 : 0;
}

__global__ void k_run_starts(int64_t n, const int32_t* head, const int32_t* hx, int32_t* starts, int64_t nruns) {
    FOR_EACH(q, n) if (head[q]) starts[hx[q]] = (int32_t)q;
    if (blockIdx.x == 0 && threadIdx.x == 0) starts[nruns] = (int32_t)n;
}

// ---- ragged lists ----------------------------------------------------------------------------
__global__ void k_ragged_count(int64_t runs, const int32_t* run_ptr, int32_t* cnt_ent, int32_t* cnt_pc) {
    FOR_EACH(r, runs) {
        const int32_t len = run_ptr[r + 1] - run_ptr[r];
        const int32_t np = len <= kPieceEntries ? 0 : (len + kPieceEntries - 1) / kPieceEntries;
        cnt_ent[r] = np == 0 ? len : np;
        cnt_pc[r] = np;
    }
}

__global__ void k_ragged_fill(int64_t n_ent, int64_t runs, const int32_t* run_ptr, const int32_t* ent_ptr, const int32_t* rpp,
                              int32_t* ent, int32_t* pb, int32_t* pe) {
    FOR_EACH(j, n_ent) {
        const int64_t r = upper_bound_dev(ent_ptr, 0, runs + 1, (int32_t)j) - 1;
        const int32_t k = (int32_t)j - ent_ptr[r];
        if (rpp[r + 1] == rpp[r]) {
            ent[j] = run_ptr[r] + k;
        } else {
            const int32_t pc = rpp[r] + k;
            ent[j] = -pc - 1;
            pb[pc] = run_ptr[r] + k * kPieceEntries;
            pe[pc] = min(run_ptr[r] + (k + 1) * kPieceEntries, run_ptr[r + 1]);
        }
    }
}

__global__ void k_resolve(int64_t n, const int32_t* ent, const int32_t* idx, int32_t* res) {
    FOR_EACH(j, n) res[j] = ent[j] >= 0 ? idx[ent[j]] : ent[j];
}

__global__ void k_ta_key(int64_t n_ent, int64_t runs, const int32_t* ent_ptr, const int32_t* run_key, int32_t* ta_key) {
    FOR_EACH(j, n_ent) ta_key[j] = run_key[upper_bound_dev(ent_ptr, 0, runs + 1, (int32_t)j) - 1];
}

// per-relation entry / piece offsets of the (relation, node_2) runs: first run of relation >= d
__global__ void k_rel_ta(int64_t R, const int32_t* run_rel, int64_t runs, const int32_t* ent_ptr, const int32_t* rpp,
                         int32_t* rel_ent, int32_t* rel_pc) {
    FOR_EACH(d, R + 1) {
        const int64_t r = lower_bound_dev(run_rel, 0, runs, (int32_t)d);
        rel_ent[d] = ent_ptr[r];
        rel_pc[d] = rpp[r];
    }
}

// ---- flat chunked lists (plan.cpp build_flat) ------------------------------------------------
__global__ void k_flat_cutstart(const int32_t* cuts, int64_t ncuts, int32_t* es) {
    FOR_EACH(i, ncuts) if (cuts[i] < cuts[i + 1]) es[cuts[i]] = 1;
}

// element starts: a forced cut, a long run, or the first short run after a long one
__global__ void k_flat_elems(int64_t runs, const int32_t* run_ptr, int32_t C, int32_t* es) {
    FOR_EACH(r, runs) {
        const bool lng = run_ptr[r + 1] - run_ptr[r] > C;
        const bool prev_lng = r > 0 && run_ptr[r] - run_ptr[r - 1] > C;
        if (lng || prev_lng) es[r] = 1;
    }
}

__global__ void k_flat_elem_first(int64_t runs, const int32_t* es, const int32_t* eid, int32_t* elem_first, int64_t NE) {
    FOR_EACH(r, runs) if (es[r]) elem_first[eid[r]] = (int32_t)r;
    if (blockIdx.x == 0 && threadIdx.x == 0) elem_first[NE] = (int32_t)runs;
}

// next chunk start after run r: a long run is followed by the next run; a short run r opening a
// chunk at run_ptr[r] is followed by the first run whose end overflows the chunk, or the end of
// its stretch (plan.cpp: "run r does not fit the open chunk: close it before r")
__global__ void k_flat_step(int64_t runs, const int32_t* run_ptr, int32_t C, const int32_t* es, const int32_t* eid,
                            const int32_t* elem_first, int32_t* step) {
    FOR_EACH(r, runs) {
        const int32_t q = run_ptr[r];
        if (run_ptr[r + 1] - q > C) {
            step[r] = (int32_t)r + 1;
            continue;
        }
        const int32_t se = elem_first[eid[r] + es[r]];  // next element start
        // first r' in (r, se) with run_ptr[r'+1] > q + C  ==  (first i in (r+1, se] with run_ptr[i] > q + C) - 1
        const int64_t i = upper_bound_dev(run_ptr, r + 2, (int64_t)se + 1, q + C);
        step[r] = (int32_t)(i - 1);
    }
}

__global__ void k_flat_walk(int64_t nb, int64_t runs, const int32_t* step, const int32_t* ein, int32_t* eout, int32_t* changed) {
    FOR_EACH(b, nb) {
        int32_t v = ein[b];
        const int64_t end = std::min<int64_t>((b + 1) * kWalkBlock, runs);
        while (v < end) v = step[v];
        if (b == 0) eout[0] = 0;
        if (b + 1 < nb) {
            eout[b + 1] = v;
            if (v != ein[b + 1]) *changed = 1;
        }
    }
}

__global__ void k_flat_mark(int64_t nb, int64_t runs, const int32_t* step, const int32_t* entry, int32_t* onchain) {
    FOR_EACH(b, nb) {
        int32_t v = entry[b];
        const int64_t end = std::min<int64_t>((b + 1) * kWalkBlock, runs);
        while (v < end) {
            onchain[v] = 1;
            v = step[v];
        }
    }
}

// chunks ending in run r (chunk ends are pushed in run order), split pieces, local long pieces
__global__ void k_flat_count(int64_t runs, const int32_t* run_ptr, int32_t C, const int32_t* es, const int32_t* eid,
                             const int32_t* elem_first, const int32_t* onchain, int32_t* cnt, int32_t* sp, int32_t* spk,
                             int32_t* lk) {
    FOR_EACH(r, runs) {
        const int32_t q = run_ptr[r], e = run_ptr[r + 1];
        if (e - q > C) {
            const int32_t k = (e - q + C - 1) / C;
            cnt[r] = k;
            const bool split = k > kFlatLongPieces;
            sp[r] = split ? 1 : 0;
            spk[r] = split ? k : 0;
            lk[r] = split ? 0 : k;
            continue;
        }
        const int32_t ei = eid[r] + es[r] - 1;
        const int32_t f = elem_first[ei], se = elem_first[ei + 1];
        const int32_t inner = (onchain[r] && !es[r]) ? 1 : 0;
        const int32_t fin = ((int32_t)r == se - 1 && run_ptr[se] > run_ptr[f]) ? 1 : 0;
        cnt[r] = inner + fin;
        sp[r] = 0;
        spk[r] = 0;
        lk[r] = 0;
    }
}

__global__ void k_flat_fill(int64_t runs, const int32_t* run_ptr, int32_t C, const int32_t* es, const int32_t* eid,
                            const int32_t* elem_first, const int32_t* onchain, const int32_t* coff, const int32_t* soff,
                            const int32_t* slotoff, int32_t* chunk_ptr, int32_t* chunk_info, int32_t* split_row,
                            int32_t* split_ptr, int32_t* row_split) {
    FOR_EACH(r, runs) {
        const int32_t q = run_ptr[r], e = run_ptr[r + 1];
        int32_t j = coff[r];
        if (e - q > C) {
            const int32_t k = (e - q + C - 1) / C;
            const bool local = k <= kFlatLongPieces;
            for (int32_t i = 0; i < k; ++i, ++j) {
                chunk_ptr[j + 1] = min(q + (i + 1) * C, e);
                const int32_t flags = (i > 0 ? 1 : 0) | (i + 1 < k ? 2 : 0);
                chunk_info[j] = flags | ((local ? i : slotoff[r] + i) << 2);
            }
            if (!local) {
                split_row[soff[r]] = (int32_t)r;
                split_ptr[soff[r]] = slotoff[r];
            }
            row_split[r] = local ? -1 : soff[r];
            continue;
        }
        row_split[r] = -1;
        if (onchain[r] && !es[r]) {
            chunk_ptr[j + 1] = q;
            chunk_info[j] = 0;
            ++j;
        }
        const int32_t ei = eid[r] + es[r] - 1;
        const int32_t f = elem_first[ei], se = elem_first[ei + 1];
        if ((int32_t)r == se - 1 && run_ptr[se] > run_ptr[f]) {
            chunk_ptr[j + 1] = run_ptr[se];
            chunk_info[j] = 0;
        }
    }
}

__global__ void k_flat_gcount(int64_t NE, const int32_t* elem_first, const int32_t* run_ptr, int32_t C, const int32_t* coff,
                              int32_t* gcnt) {
    FOR_EACH(x, NE) {
        const int32_t f = elem_first[x], fn = elem_first[x + 1];
        const int32_t nc = coff[fn] - coff[f];
        const int32_t len = run_ptr[f + 1] - run_ptr[f];
        const bool local_long = len > C && (len + C - 1) / C <= kFlatLongPieces;
        gcnt[x] = local_long ? 1 : (nc + kFlatGroup - 1) / kFlatGroup;
    }
}

__global__ void k_flat_gfill(int64_t NE, const int32_t* elem_first, const int32_t* run_ptr, int32_t C, const int32_t* coff,
                             const int32_t* goff, int32_t* group_ptr, int32_t* group_long) {
    FOR_EACH(x, NE) {
        const int32_t f = elem_first[x];
        const int32_t len = run_ptr[f + 1] - run_ptr[f];
        const bool local_long = len > C && (len + C - 1) / C <= kFlatLongPieces;
        for (int32_t g = goff[x], i = 0; g < goff[x + 1]; ++g, ++i) {
            group_ptr[g] = coff[f] + i * kFlatGroup;
            group_long[g] = local_long ? 1 : 0;
        }
    }
}

__global__ void k_flat_row_of(int64_t P, const int32_t* run_ptr, int64_t runs, int32_t* row_of) {
    FOR_EACH(q, P) row_of[q] = (int32_t)(upper_bound_dev(run_ptr, 0, runs + 1, (int32_t)q) - 1);
}

__global__ void k_flat_cuts(const int32_t* cuts, int64_t n, int64_t runs, const int32_t* eid, const int32_t* goff,
                            const int32_t* soff, int32_t* cgp, int32_t* csp) {
    FOR_EACH(i, n) {
        const int32_t r = cuts[i];
        // a cut below `runs` starts a non-empty section, hence a list element
        cgp[i] = goff[r < runs ? eid[r] : eid[runs]];
        csp[i] = soff[r < runs ? r : runs];
    }
}

// ---- augmented lists (own rows get a trailing extra-row entry) ---------------------------------
__global__ void k_aug_ptr(int64_t N, const int32_t* ptr, int64_t lo, int64_t hi, int32_t* xptr) {
    FOR_EACH(i, N + 1) xptr[i] = ptr[i] + (int32_t)(std::min(std::max(i, lo), hi) - lo);
}

__global__ void k_aug_vals(int64_t P, const int32_t* ptr, int64_t N, const int32_t* val, const int32_t* xptr, int32_t* out) {
    FOR_EACH(q, P) {
        const int64_t i = upper_bound_dev(ptr, 0, N + 1, (int32_t)q) - 1;
        out[xptr[i] + (int32_t)q - ptr[i]] = val[q];
    }
}

__global__ void k_aug_extra(int64_t lo, int64_t hi, const int32_t* xptr, int32_t* out) {
    FOR_EACH(k, hi - lo) out[xptr[lo + k + 1] - 1] = -(int32_t)k - 1;
}

// ---- tiles --------------------------------------------------------------------------------------
__global__ void k_t32_cost(int64_t T, const int32_t* tb, const int32_t* te, const int32_t* s_ptr, int32_t* cost) {
    FOR_EACH(t, T) {
        const int64_t e = s_ptr[te[t]] - s_ptr[tb[t]];
        const int64_t g = (23 * e + 1000) / 64;  // plan_internal.h item_cost()
        cost[t] = (int32_t)(g > 64 ? g : 64);
    }
}

// ---- the builder --------------------------------------------------------------------------------
class Builder {
public:
    Builder(mpgnn_plan* p, hipStream_t s) : p_(p), s_(s) {}
    ~Builder() {
        for (void* t : temps_) (void)hipFree(t);
    }

    template <class T>
    T* temp(int64_t n) {
        void* ptr = nullptr;
        DCHECK(hipMalloc(&ptr, (size_t)std::max<int64_t>(n, 1) * sizeof(T)));
        temps_.push_back(ptr);
        return static_cast<T*>(ptr);
    }
    void release(void* ptr) {
        auto it = std::find(temps_.begin(), temps_.end(), ptr);
        if (it != temps_.end()) {
            (void)hipFree(ptr);
            temps_.erase(it);
        }
    }
    // a plan table: owned by the plan, copied into `host` on export
    int32_t* table(std::vector<int32_t>* host, int64_t n) {
        void* ptr = nullptr;
        DCHECK(hipMalloc(&ptr, (size_t)std::max<int64_t>(n, 1) * sizeof(int32_t)));
        p_->dev_allocs.push_back(ptr);
        if (host) p_->dev_tables.push_back({host, static_cast<int32_t*>(ptr), n});
        return static_cast<int32_t*>(ptr);
    }
    // a small table computed on the device and needed on the host as well
    void download(std::vector<int32_t>& h, const int32_t* d, int64_t n) {
        h.resize(n);
        if (n > 0) DCHECK(hipMemcpyAsync(h.data(), d, n * sizeof(int32_t), hipMemcpyDeviceToHost, s_));
        DCHECK(hipStreamSynchronize(s_));
    }
    int32_t* upload(std::vector<int32_t>* host_table, const std::vector<int32_t>& h) {
        int32_t* d = table(nullptr, (int64_t)h.size());
        if (!h.empty()) DCHECK(hipMemcpyAsync(d, h.data(), h.size() * sizeof(int32_t), hipMemcpyHostToDevice, s_));
        DCHECK(hipStreamSynchronize(s_));  // h may be temporary
        (void)host_table;
        return d;
    }
    int32_t read(const int32_t* d, int64_t i) {
        int32_t v = 0;
        DCHECK(hipMemcpyAsync(&v, d + i, sizeof(v), hipMemcpyDeviceToHost, s_));
        DCHECK(hipStreamSynchronize(s_));
        return v;
    }
    void check_launch() { DCHECK(hipGetLastError()); }

    // out[0..n) = exclusive prefix of in, out[n] = total; returns the total
    int64_t scan(const int32_t* in, int32_t* out, int64_t n) {
        if (n > 0) {
            size_t bytes = 0;
            DCHECK(rocprim::exclusive_scan(nullptr, bytes, in, out, 0, (size_t)n, rocprim::plus<int32_t>(), s_));
            void* t = temp<char>((int64_t)bytes);
            DCHECK(rocprim::exclusive_scan(t, bytes, in, out, 0, (size_t)n, rocprim::plus<int32_t>(), s_));
            release(t);
        }
        hipLaunchKernelGGL(k_scan_total, dim3(1), dim3(1), 0, s_, in, out, n);
        check_launch();
        return read(out, n);
    }
    int32_t max_of(const int32_t* in, int64_t n) {
        if (n <= 0) return 0;
        int32_t* d = temp<int32_t>(1);
        size_t bytes = 0;
        DCHECK(rocprim::reduce(nullptr, bytes, in, d, 0, (size_t)n, rocprim::maximum<int32_t>(), s_));
        void* t = temp<char>((int64_t)bytes);
        DCHECK(rocprim::reduce(t, bytes, in, d, 0, (size_t)n, rocprim::maximum<int32_t>(), s_));
        const int32_t v = read(d, 0);
        release(t);
        release(d);
        return v;
    }
    template <class K, class V>
    void sort_pairs(const K* kin, K* kout, const V* vin, V* vout, int64_t n, unsigned bits) {
        if (n <= 0) return;
        bits = std::max(1u, std::min<unsigned>(bits, 8 * sizeof(K)));
        size_t bytes = 0;
        DCHECK(rocprim::radix_sort_pairs(nullptr, bytes, kin, kout, vin, vout, (size_t)n, 0, bits, s_));
        void* t = temp<char>((int64_t)bytes);
        DCHECK(rocprim::radix_sort_pairs(t, bytes, kin, kout, vin, vout, (size_t)n, 0, bits, s_));
        release(t);
    }
    // run starts of a head-flag array: starts[0..nruns) + starts[nruns] = n; returns nruns
    int64_t run_starts(const int32_t* head, int64_t n, int32_t*& starts) {
        int32_t* hx = temp<int32_t>(n + 1);
        const int64_t nr = scan(head, hx, n);
        starts = temp<int32_t>(nr + 1);
        hipLaunchKernelGGL(k_run_starts, grid_for(n), dim3(kT), 0, s_, n, head, hx, starts, nr);
        check_launch();
        release(hx);
        return nr;
    }

    void ragged(const int32_t* run_ptr, int64_t runs, RaggedHost& H, int32_t** d_ent, int32_t** d_ent_ptr, int32_t** d_pb,
                int32_t** d_pe, int32_t** d_rpp);
    void flat(const int32_t* run_ptr, int64_t runs, int64_t P, const std::vector<int32_t>& cuts, int32_t C, FlatHost& H,
              FlatDev& D);
    template <class K>
    void build(const int64_t* ei, const int64_t* et, int64_t E, int64_t N, int64_t lo, int64_t hi, int32_t side);
    void build_all(const int64_t* ei, const int64_t* et, int64_t E, int64_t N, int64_t lo, int64_t hi, int32_t side);

    hipStream_t stream() const { return s_; }

private:
    mpgnn_plan* p_;
    hipStream_t s_;
    std::vector<void*> temps_;
};

static unsigned bits_for(uint64_t n) {  // bits of the largest key below n
    unsigned b = 0;
    while (b < 64 && (n - 1) >> b) ++b;
    return std::max(1u, b);
}

void Builder::ragged(const int32_t* run_ptr, int64_t runs, RaggedHost& H, int32_t** d_ent, int32_t** d_ent_ptr,
                     int32_t** d_pb, int32_t** d_pe, int32_t** d_rpp) {
    int32_t* ce = temp<int32_t>(runs);
    int32_t* cp = temp<int32_t>(runs);
    hipLaunchKernelGGL(k_ragged_count, grid_for(runs), dim3(kT), 0, s_, runs, run_ptr, ce, cp);
    check_launch();
    int32_t* ent_ptr = table(&H.ent_ptr, runs + 1);
    int32_t* rpp = table(&H.run_piece_ptr, runs + 1);
    const int64_t n_ent = scan(ce, ent_ptr, runs);
    const int64_t n_pc = scan(cp, rpp, runs);
    release(ce);
    release(cp);
    int32_t* ent = table(&H.ent, n_ent);
    int32_t* pb = table(&H.piece_b, n_pc);
    int32_t* pe = table(&H.piece_e, n_pc);
    hipLaunchKernelGGL(k_ragged_fill, grid_for(n_ent), dim3(kT), 0, s_, n_ent, runs, run_ptr, ent_ptr, rpp, ent, pb, pe);
    check_launch();
    H.npieces = n_pc;
    H.nent = n_ent;
    *d_ent = ent;
    if (d_ent_ptr) *d_ent_ptr = ent_ptr;
    *d_pb = pb;
    *d_pe = pe;
    if (d_rpp) *d_rpp = rpp;
}

void Builder::flat(const int32_t* run_ptr, int64_t runs, int64_t P, const std::vector<int32_t>& cuts, int32_t C, FlatHost& H,
                   FlatDev& D) {
    H = FlatHost{};
    const int64_t ncut = (int64_t)cuts.size() - 1;
    int32_t* d_cuts = temp<int32_t>((int64_t)cuts.size());
    DCHECK(hipMemcpyAsync(d_cuts, cuts.data(), cuts.size() * sizeof(int32_t), hipMemcpyHostToDevice, s_));
    // list elements: stretches of short runs (greedy chunks) and long runs (pieces)
    int32_t* es = temp<int32_t>(runs + 1);
    DCHECK(hipMemsetAsync(es, 0, (runs + 1) * sizeof(int32_t), s_));
    hipLaunchKernelGGL(k_flat_cutstart, grid_for(ncut), dim3(kT), 0, s_, d_cuts, ncut, es);
    hipLaunchKernelGGL(k_flat_elems, grid_for(runs), dim3(kT), 0, s_, runs, run_ptr, C, es);
    check_launch();
    int32_t* eid = temp<int32_t>(runs + 1);
    const int64_t NE = scan(es, eid, runs);
    int32_t* elem_first = temp<int32_t>(NE + 1);
    hipLaunchKernelGGL(k_flat_elem_first, grid_for(runs), dim3(kT), 0, s_, runs, es, eid, elem_first, NE);
    check_launch();
    // chunk starts: step per run, block entries to their fixed point, then mark the chain
    int32_t* step = temp<int32_t>(runs);
    hipLaunchKernelGGL(k_flat_step, grid_for(runs), dim3(kT), 0, s_, runs, run_ptr, C, es, eid, elem_first, step);
    check_launch();
    const int64_t nb = (runs + kWalkBlock - 1) / kWalkBlock;
    int32_t* ea = temp<int32_t>(nb);
    int32_t* eb = temp<int32_t>(nb);
    int32_t* changed = temp<int32_t>(1);
    {
        std::vector<int32_t> init(nb);
        for (int64_t b = 0; b < nb; ++b) init[b] = (int32_t)(b * kWalkBlock);
        if (nb) DCHECK(hipMemcpyAsync(ea, init.data(), nb * sizeof(int32_t), hipMemcpyHostToDevice, s_));
        for (int64_t it = 0; it <= nb && nb > 0; ++it) {
            DCHECK(hipMemsetAsync(changed, 0, sizeof(int32_t), s_));
            hipLaunchKernelGGL(k_flat_walk, grid_for(nb), dim3(kT), 0, s_, nb, runs, step, ea, eb, changed);
            check_launch();
            std::swap(ea, eb);
            if (read(changed, 0) == 0) break;
        }
    }
    int32_t* onchain = temp<int32_t>(runs);
    DCHECK(hipMemsetAsync(onchain, 0, std::max<int64_t>(runs, 1) * sizeof(int32_t), s_));
    hipLaunchKernelGGL(k_flat_mark, grid_for(nb), dim3(kT), 0, s_, nb, runs, step, ea, onchain);
    check_launch();
    release(step);
    // chunk / split / slot offsets over runs
    int32_t* cnt = temp<int32_t>(runs);
    int32_t* sp = temp<int32_t>(runs);
    int32_t* spk = temp<int32_t>(runs);
    int32_t* lk = temp<int32_t>(runs);
    hipLaunchKernelGGL(k_flat_count, grid_for(runs), dim3(kT), 0, s_, runs, run_ptr, C, es, eid, elem_first, onchain, cnt, sp,
                       spk, lk);
    check_launch();
    int32_t* coff = temp<int32_t>(runs + 1);
    int32_t* soff = temp<int32_t>(runs + 1);
    int32_t* slotoff = temp<int32_t>(runs + 1);
    const int64_t nch = scan(cnt, coff, runs);
    const int64_t nsplit = scan(sp, soff, runs);
    const int64_t nslots = scan(spk, slotoff, runs);
    H.max_pieces = max_of(lk, runs);
    D.chunk_ptr = table(&H.chunk_ptr, nch + 1);
    D.chunk_info = table(&H.chunk_info, nch);
    D.split_row = table(&H.split_row, nsplit);
    D.split_ptr = table(&H.split_ptr, nsplit + 1);
    D.split_slot = table(&H.split_slot, nslots);
    D.row_split = table(&H.row_split, runs);
    hipLaunchKernelGGL(k_set, dim3(1), dim3(1), 0, s_, D.chunk_ptr, (int64_t)0, 0);
    hipLaunchKernelGGL(k_set, dim3(1), dim3(1), 0, s_, D.split_ptr, nsplit, (int32_t)nslots);
    hipLaunchKernelGGL(k_iota, grid_for(nslots), dim3(kT), 0, s_, D.split_slot, nslots);
    hipLaunchKernelGGL(k_flat_fill, grid_for(runs), dim3(kT), 0, s_, runs, run_ptr, C, es, eid, elem_first, onchain, coff, soff,
                       slotoff, D.chunk_ptr, D.chunk_info, D.split_row, D.split_ptr, D.row_split);
    check_launch();
    // workgroup groups over list elements
    int32_t* gcnt = temp<int32_t>(NE);
    hipLaunchKernelGGL(k_flat_gcount, grid_for(NE), dim3(kT), 0, s_, NE, elem_first, run_ptr, C, coff, gcnt);
    check_launch();
    int32_t* goff = temp<int32_t>(NE + 1);
    const int64_t ngroups = scan(gcnt, goff, NE);
    D.group_ptr = table(&H.group_ptr, ngroups + 1);
    D.group_long = table(&H.group_long, ngroups);
    hipLaunchKernelGGL(k_flat_gfill, grid_for(NE), dim3(kT), 0, s_, NE, elem_first, run_ptr, C, coff, goff, D.group_ptr,
                       D.group_long);
    hipLaunchKernelGGL(k_set, dim3(1), dim3(1), 0, s_, D.group_ptr, ngroups, (int32_t)nch);
    D.row_of = table(&H.row_of, P);
    hipLaunchKernelGGL(k_flat_row_of, grid_for(P), dim3(kT), 0, s_, P, run_ptr, runs, D.row_of);
    check_launch();
    // section boundaries (forced cuts)
    int32_t* cgp = temp<int32_t>(ncut + 1);
    int32_t* csp = temp<int32_t>(ncut + 1);
    hipLaunchKernelGGL(k_flat_cuts, grid_for(ncut + 1), dim3(kT), 0, s_, d_cuts, ncut + 1, runs, eid, goff, soff, cgp, csp);
    check_launch();
    download(H.cut_group_ptr, cgp, ncut + 1);
    download(H.cut_split_ptr, csp, ncut + 1);
    H.nslots = (int32_t)nslots;
    H.ngroups = (int32_t)ngroups;
    H.nsplit = (int32_t)nsplit;
    for (void* t : {(void*)d_cuts, (void*)es, (void*)eid, (void*)elem_first, (void*)ea, (void*)eb, (void*)changed,
                    (void*)onchain, (void*)cnt, (void*)sp, (void*)spk, (void*)lk, (void*)coff, (void*)soff, (void*)slotoff,
                    (void*)gcnt, (void*)goff, (void*)cgp, (void*)csp})
        release(t);
}

template <class K>
void Builder::build(const int64_t* ei, const int64_t* et, int64_t E, int64_t N, int64_t lo, int64_t hi, int32_t side) {
    mpgnn_plan* p = p_;
    const int64_t* n1 = ei;
    const int64_t* n2 = ei + E;
    const int64_t R = p->nrel;
    DeviceTables& d = p->d;

    // ---- dense relation ids, valid edges, invalid relations ----------------------------------
    int64_t* rel_vals = temp<int64_t>(R);
    if (R) DCHECK(hipMemcpyAsync(rel_vals, p->rel_values.data(), R * sizeof(int64_t), hipMemcpyHostToDevice, s_));
    int32_t* rel_d = temp<int32_t>(E);
    int32_t* valid = temp<int32_t>(E);
    uint8_t* invalid = temp<uint8_t>(R);
    if (R) DCHECK(hipMemsetAsync(invalid, 0, R, s_));
    hipLaunchKernelGGL(k_rel_dense, grid_for(E), dim3(kT), 0, s_, n1, n2, et, E, N, rel_vals, R, rel_d, valid, invalid);
    check_launch();
    p->rel_invalid.assign(R, 0);
    if (R) DCHECK(hipMemcpyAsync(p->rel_invalid.data(), invalid, R, hipMemcpyDeviceToHost, s_));
    d.rel_val32 = table(nullptr, R);
    if (R) DCHECK(hipMemcpyAsync(d.rel_val32, p->rel_val32.data(), R * sizeof(int32_t), hipMemcpyHostToDevice, s_));
    // valid edge ids in edge order
    int32_t* vx = temp<int32_t>(E + 1);
    const int64_t V = scan(valid, vx, E);
    int32_t* ids = temp<int32_t>(V);
    {
        int32_t* cnt = temp<int32_t>(1);
        size_t bytes = 0;
        rocprim::counting_iterator<int32_t> it(0);
        if (E > 0) {
            DCHECK(rocprim::select(nullptr, bytes, it, valid, ids, cnt, (size_t)E, s_));
            void* t = temp<char>((int64_t)bytes);
            DCHECK(rocprim::select(t, bytes, it, valid, ids, cnt, (size_t)E, s_));
            release(t);
        }
        release(cnt);
    }
    release(vx);
    release(valid);

    // ---- (relation, node_1, edge) order: radix sort of rel·N + node_1 over edge order --------
    K* keys = temp<K>(V);
    K* keys_s = temp<K>(V);
    int32_t* ids_s = temp<int32_t>(V);
    hipLaunchKernelGGL(k_row_keys<K>, grid_for(V), dim3(kT), 0, s_, ids, V, rel_d, n1, N, keys);
    check_launch();
    sort_pairs(keys, keys_s, ids, ids_s, V, bits_for((uint64_t)std::max<int64_t>(R, 1) * (uint64_t)std::max<int64_t>(N, 1)));
    release(keys);
    release(ids);

    // ---- segments -----------------------------------------------------------------------------
    int32_t* head = temp<int32_t>(V);
    int32_t* loc = temp<int32_t>(V);
    hipLaunchKernelGGL(k_seg_heads<K>, grid_for(V), dim3(kT), 0, s_, keys_s, ids_s, V, n1, n2, lo, hi, side, head, loc);
    check_launch();
    release(keys_s);
    int32_t* hx = temp<int32_t>(V + 1);
    const int64_t G = scan(head, hx, V);
    int32_t* lx = temp<int32_t>(V + 1);
    const int64_t E_loc = scan(loc, lx, V);
    int32_t* gstart = temp<int32_t>(G + 1);
    hipLaunchKernelGGL(k_gstart, grid_for(V), dim3(kT), 0, s_, V, head, hx, gstart, G);
    int32_t* kept = temp<int32_t>(G);
    hipLaunchKernelGGL(k_kept, grid_for(G), dim3(kT), 0, s_, G, gstart, lx, kept);
    check_launch();
    int32_t* sidx = temp<int32_t>(G + 1);
    const int64_t S = scan(kept, sidx, G);
    p->E = E_loc;
    p->S = S;
    d.e_col = table(&p->e_col, E_loc);
    int32_t* e_id = table(&p->e_id, E_loc);
    int32_t* seg_of_edge = temp<int32_t>(E_loc);
    hipLaunchKernelGGL(k_fill_edges, grid_for(V), dim3(kT), 0, s_, V, ids_s, head, hx, loc, lx, sidx, n2, d.e_col, e_id,
                       seg_of_edge);
    d.s_row = table(&p->s_row, S);
    d.s_rel = table(&p->s_rel, S);
    d.s_cnt = table(&p->s_cnt, S);
    d.s_ptr = table(&p->s_ptr, S + 1);
    int32_t* seg_d = temp<int32_t>(S);
    hipLaunchKernelGGL(k_fill_segs, grid_for(G), dim3(kT), 0, s_, G, gstart, kept, sidx, lx, ids_s, n1, rel_d, d.rel_val32,
                       d.s_row, seg_d, d.s_rel, d.s_cnt, d.s_ptr);
    hipLaunchKernelGGL(k_set, dim3(1), dim3(1), 0, s_, d.s_ptr, S, (int32_t)E_loc);
    check_launch();
    for (void* t : {(void*)head, (void*)loc, (void*)hx, (void*)lx, (void*)gstart, (void*)kept, (void*)sidx, (void*)ids_s,
                    (void*)rel_d, (void*)rel_vals, (void*)invalid})
        release(t);
    // per-relation segment / edge ranges
    d.rel_seg_ptr = table(&p->rel_seg_ptr, R + 1);
    hipLaunchKernelGGL(k_lower_bound_iota, grid_for(R + 1), dim3(kT), 0, s_, seg_d, S, d.rel_seg_ptr, R + 1);
    int32_t* rel_edge_ptr = temp<int32_t>(R + 1);
    hipLaunchKernelGGL(k_gather, grid_for(R + 1), dim3(kT), 0, s_, d.s_ptr, d.rel_seg_ptr, R + 1, rel_edge_ptr);
    check_launch();
    download(p->rel_seg_ptr, d.rel_seg_ptr, R + 1);
    download(p->rel_edge_ptr, rel_edge_ptr, R + 1);
    release(rel_edge_ptr);

    // ---- multi-edge segments --------------------------------------------------------------------
    {
        int32_t* mflag = temp<int32_t>(S);
        int32_t* mlen = temp<int32_t>(S);
        hipLaunchKernelGGL(k_multi_flags, grid_for(S), dim3(kT), 0, s_, S, d.s_ptr, d.s_cnt, mflag, mlen);
        check_launch();
        int32_t* m_id = temp<int32_t>(S + 1);
        int32_t* m_off = temp<int32_t>(S + 1);
        const int64_t Sm = scan(mflag, m_id, S);
        const int64_t Em = scan(mlen, m_off, S);
        d.s_src = table(&p->s_src, S);
        d.m_cnt = table(&p->m_cnt, Sm);
        d.m_ptr = table(&p->m_ptr, Sm + 1);
        d.em_col = table(&p->em_col, Em);
        hipLaunchKernelGGL(k_multi_segs, grid_for(S), dim3(kT), 0, s_, S, d.s_ptr, d.s_cnt, d.e_col, mflag, m_id, m_off, d.s_src,
                           d.m_cnt, d.m_ptr);
        hipLaunchKernelGGL(k_set, dim3(1), dim3(1), 0, s_, d.m_ptr, Sm, (int32_t)Em);
        hipLaunchKernelGGL(k_multi_edges, grid_for(E_loc), dim3(kT), 0, s_, E_loc, seg_of_edge, d.s_ptr, mflag, m_off, d.e_col,
                           d.em_col);
        int32_t* rel_m_ptr = temp<int32_t>(R + 1);
        hipLaunchKernelGGL(k_rel_m_ptr, grid_for(R + 1), dim3(kT), 0, s_, R, d.rel_seg_ptr, S, m_id, (int32_t)Sm, rel_m_ptr);
        check_launch();
        download(p->rel_m_ptr, rel_m_ptr, R + 1);
        for (void* t : {(void*)mflag, (void*)mlen, (void*)m_id, (void*)m_off, (void*)rel_m_ptr}) release(t);
    }

    // ---- row-major segment order (node_1, relation) -------------------------------------------
    {
        int32_t* iota = temp<int32_t>(S);
        hipLaunchKernelGGL(k_iota, grid_for(S), dim3(kT), 0, s_, iota, S);
        int32_t* rows_s = temp<int32_t>(S);
        d.rw_seg = table(&p->rw_seg, S);
        sort_pairs(d.s_row, rows_s, iota, d.rw_seg, S, bits_for((uint64_t)std::max<int64_t>(N, 1)));
        d.rw_ptr = table(&p->rw_ptr, N + 1);
        hipLaunchKernelGGL(k_lower_bound_iota, grid_for(N + 1), dim3(kT), 0, s_, rows_s, S, d.rw_ptr, N + 1);
        d.s_pos = table(&p->s_pos, S);
        hipLaunchKernelGGL(k_scatter_pos, grid_for(S), dim3(kT), 0, s_, d.rw_seg, S, d.s_pos);
        check_launch();
        release(iota);
        release(rows_s);
    }

    // ---- transposed orders for grad_x ------------------------------------------------------------
    int32_t* ta_runs = nullptr;
    int64_t nruns = 0;
    int32_t* run_rel = nullptr;
    int32_t* run_key = nullptr;
    {
        int32_t* iota = temp<int32_t>(E_loc);
        hipLaunchKernelGGL(k_iota, grid_for(E_loc), dim3(kT), 0, s_, iota, E_loc);
        int32_t* cols_s = temp<int32_t>(E_loc);
        int32_t* by_col = temp<int32_t>(E_loc);
        sort_pairs(d.e_col, cols_s, iota, by_col, E_loc, bits_for((uint64_t)std::max<int64_t>(N, 1)));
        d.t_ptr = table(&p->t_ptr, N + 1);
        hipLaunchKernelGGL(k_lower_bound_iota, grid_for(N + 1), dim3(kT), 0, s_, cols_s, E_loc, d.t_ptr, N + 1);
        d.t_seg = table(&p->t_seg, E_loc);
        int32_t* key_d = temp<int32_t>(E_loc);
        hipLaunchKernelGGL(k_tseg_keys, grid_for(E_loc), dim3(kT), 0, s_, E_loc, by_col, seg_of_edge, seg_d, d.t_seg, key_d);
        check_launch();
        release(iota);
        release(cols_s);
        // (relation, node_2, node_1, edge): stable radix sort of the relation over col-major order
        int32_t* td = temp<int32_t>(E_loc);
        int32_t* by_rel_col = temp<int32_t>(E_loc);
        sort_pairs(key_d, td, by_col, by_rel_col, E_loc, bits_for((uint64_t)std::max<int64_t>(R, 1)));
        release(key_d);
        release(by_col);
        d.ta_col = table(&p->ta_col, E_loc);
        d.ta_seg = table(&p->ta_seg, E_loc);
        hipLaunchKernelGGL(k_ta, grid_for(E_loc), dim3(kT), 0, s_, E_loc, by_rel_col, d.e_col, seg_of_edge, d.ta_col, d.ta_seg);
        check_launch();
        release(by_rel_col);
        int32_t* h2 = temp<int32_t>(E_loc);
        hipLaunchKernelGGL(k_ta_heads, grid_for(E_loc), dim3(kT), 0, s_, E_loc, td, d.ta_col, h2);
        check_launch();
        nruns = run_starts(h2, E_loc, ta_runs);
        run_rel = temp<int32_t>(nruns);
        run_key = temp<int32_t>(nruns);
        hipLaunchKernelGGL(k_gather, grid_for(nruns), dim3(kT), 0, s_, td, ta_runs, nruns, run_rel);
        hipLaunchKernelGGL(k_gather, grid_for(nruns), dim3(kT), 0, s_, d.ta_col, ta_runs, nruns, run_key);
        check_launch();
        release(h2);
        release(td);
    }
    release(seg_d);
    release(seg_of_edge);

    // ---- ragged lists ----------------------------------------------------------------------------
    int32_t* seg_rpp = nullptr;
    ragged(d.s_ptr, S, p->seg_l, &d.seg_ent, &d.seg_ent_ptr, &d.seg_pb, &d.seg_pe, &seg_rpp);
    ragged(d.rw_ptr, N, p->rw_l, &d.rw_ent, &d.rw_ent_ptr, &d.rw_pb, &d.rw_pe, nullptr);
    ragged(d.t_ptr, N, p->t_l, &d.t_ent, &d.t_ent_ptr, &d.t_pb, &d.t_pe, nullptr);
    int32_t* ta_ent_ptr = nullptr;
    int32_t* ta_rpp = nullptr;
    ragged(ta_runs, nruns, p->ta_l, &d.ta_ent, &ta_ent_ptr, &d.ta_pb, &d.ta_pe, &ta_rpp);
    auto resolve = [&](RaggedHost& H, const int32_t* ent, const int32_t* idx, int32_t** res) {
        *res = table(&H.res, H.nent);
        hipLaunchKernelGGL(k_resolve, grid_for(H.nent), dim3(kT), 0, s_, H.nent, ent, idx, *res);
        check_launch();
    };
    resolve(p->seg_l, d.seg_ent, d.e_col, &d.seg_res);
    resolve(p->rw_l, d.rw_ent, d.rw_seg, &d.rw_res);
    resolve(p->t_l, d.t_ent, d.t_seg, &d.t_res);
    resolve(p->ta_l, d.ta_ent, d.ta_seg, &d.ta_res);
    d.ta_key = table(&p->ta_key, p->ta_l.nent);
    hipLaunchKernelGGL(k_ta_key, grid_for(p->ta_l.nent), dim3(kT), 0, s_, p->ta_l.nent, nruns, ta_ent_ptr, run_key, d.ta_key);
    {
        int32_t* re = temp<int32_t>(R + 1);
        int32_t* rp = temp<int32_t>(R + 1);
        hipLaunchKernelGGL(k_rel_ta, grid_for(R + 1), dim3(kT), 0, s_, R, run_rel, nruns, ta_ent_ptr, ta_rpp, re, rp);
        int32_t* sp = temp<int32_t>(R + 1);
        hipLaunchKernelGGL(k_gather, grid_for(R + 1), dim3(kT), 0, s_, seg_rpp, d.rel_seg_ptr, R + 1, sp);
        check_launch();
        download(p->rel_ta_ent_ptr, re, R + 1);
        download(p->rel_ta_piece_ptr, rp, R + 1);
        download(p->rel_seg_piece_ptr, sp, R + 1);
        release(re);
        release(rp);
        release(sp);
    }
    release(run_rel);
    release(run_key);

    // ---- flat lists --------------------------------------------------------------------------
    const std::vector<int32_t> node_cuts{0, (int32_t)N};
    flat(d.s_ptr, S, E_loc, p->rel_seg_ptr, kFlatChunk, p->seg_f, d.seg_f);
    {
        const int64_t nm = (int64_t)p->rel_m_ptr.back();  // Sm (rel_m_ptr[R] = Sm)
        const int32_t em = read(d.m_ptr, nm);
        flat(d.m_ptr, nm, em, p->rel_m_ptr, kFlatChunk, p->segm_f, d.segm_f);
    }
    flat(d.rw_ptr, N, S, node_cuts, kFlatChunkRowMajor, p->rw_f, d.rw_f);
    flat(d.t_ptr, N, E_loc, node_cuts, kFlatChunk, p->t_f, d.t_f);
    auto augment = [&](const int32_t* ptr, int64_t P, const int32_t* val, FlatHost& F, FlatDev& FD, std::vector<int32_t>* hval,
                       int32_t** dval, int32_t C) {
        int32_t* xptr = temp<int32_t>(N + 1);
        hipLaunchKernelGGL(k_aug_ptr, grid_for(N + 1), dim3(kT), 0, s_, N, ptr, lo, hi, xptr);
        const int64_t XP = P + (hi - lo);
        *dval = table(hval, XP);
        hipLaunchKernelGGL(k_aug_vals, grid_for(P), dim3(kT), 0, s_, P, ptr, N, val, xptr, *dval);
        hipLaunchKernelGGL(k_aug_extra, grid_for(hi - lo), dim3(kT), 0, s_, lo, hi, xptr, *dval);
        check_launch();
        flat(xptr, N, XP, node_cuts, C, F, FD);
        release(xptr);
    };
    augment(d.t_ptr, E_loc, d.t_seg, p->tx_f, d.tx_f, &p->tx_val, &d.tx_val, kFlatChunk);
    augment(d.rw_ptr, S, d.rw_seg, p->rwx_f, d.rwx_f, &p->rwx_val, &d.rwx_val, kFlatChunkRowMajor);
    release(ta_runs);

    // ---- relation-pure tiles and reduction chunks (host, O(S/32); plan.cpp build) ------------
    p->rel_tile_ptr.assign(R + 1, 0);
    p->rel_t32_ptr.assign(R + 1, 0);
    p->rel_chunk_ptr.assign(R + 1, 0);
    const int64_t s_all = p->rel_seg_ptr[R];
    const int32_t chunk_cap =
        (int32_t)std::max<int64_t>(g_chunk_rows, (s_all + kChunkTarget - 1) / kChunkTarget + 31) / 32 * 32;
    for (int64_t r = 0; r < R; ++r) {
        for (int32_t s = p->rel_seg_ptr[r]; s < p->rel_seg_ptr[r + 1]; s += kTile32) {
            p->t32_begin.push_back(s);
            p->t32_end.push_back(std::min<int32_t>(s + kTile32, p->rel_seg_ptr[r + 1]));
        }
        p->rel_t32_ptr[r + 1] = (int32_t)p->t32_begin.size();
        for (int32_t s = p->rel_seg_ptr[r]; s < p->rel_seg_ptr[r + 1]; s += kTileRows) {
            p->tile_begin.push_back(s);
            p->tile_end.push_back(std::min<int32_t>(s + kTileRows, p->rel_seg_ptr[r + 1]));
        }
        p->rel_tile_ptr[r + 1] = (int32_t)p->tile_begin.size();
        const int32_t sb = p->rel_seg_ptr[r], se = p->rel_seg_ptr[r + 1];
        const int32_t nch = (se - sb + chunk_cap - 1) / chunk_cap;
        const int32_t per = nch > 0 ? ((se - sb + nch - 1) / nch + 31) / 32 * 32 : 0;
        for (int32_t s = sb; s < se; s += per) {
            p->chunk_begin.push_back(s);
            p->chunk_end.push_back(std::min<int32_t>(s + per, se));
            p->chunk_dst.push_back(nch == 1 ? p->rel_val32[r] : -1);
        }
        p->rel_chunk_ptr[r + 1] = (int32_t)p->chunk_begin.size();
    }
    d.tile_begin = upload(nullptr, p->tile_begin);
    d.tile_end = upload(nullptr, p->tile_end);
    d.t32_begin = upload(nullptr, p->t32_begin);
    d.t32_end = upload(nullptr, p->t32_end);
    d.chunk_begin = upload(nullptr, p->chunk_begin);
    d.chunk_end = upload(nullptr, p->chunk_end);
    d.chunk_dst = upload(nullptr, p->chunk_dst);
    d.rel_chunk_ptr = upload(nullptr, p->rel_chunk_ptr);
    {
        const int64_t T = (int64_t)p->t32_begin.size();
        int32_t* cost = temp<int32_t>(T);
        hipLaunchKernelGGL(k_t32_cost, grid_for(T), dim3(kT), 0, s_, T, d.t32_begin, d.t32_end, d.s_ptr, cost);
        check_launch();
        d.t32_cost = table(&p->t32_cost, T + 1);
        scan(cost, d.t32_cost, T);  // t32_cost[t] = Σ_{u<t} cost[u], t32_cost[T] = total
        release(cost);
    }
    DCHECK(hipStreamSynchronize(s_));
}

void Builder::build_all(const int64_t* ei, const int64_t* et, int64_t E, int64_t N, int64_t lo, int64_t hi, int32_t side) {
    mpgnn_plan* p = p_;
    p->N = N;
    p->E_in = E;
    p->shard_lo = lo;
    p->shard_hi = hi;
    // sorted distinct relation values (sort + unique of a copy of edge_type)
    if (E > 0) {
        int64_t* a = temp<int64_t>(E);
        int64_t* b = temp<int64_t>(E);
        DCHECK(hipMemcpyAsync(a, et, E * sizeof(int64_t), hipMemcpyDeviceToDevice, s_));
        size_t bytes = 0;
        DCHECK(rocprim::radix_sort_keys(nullptr, bytes, a, b, (size_t)E, 0, 64, s_));
        void* t = temp<char>((int64_t)bytes);
        DCHECK(rocprim::radix_sort_keys(t, bytes, a, b, (size_t)E, 0, 64, s_));
        release(t);
        size_t* cnt = temp<size_t>(1);
        bytes = 0;
        DCHECK(rocprim::unique(nullptr, bytes, b, a, cnt, (size_t)E, rocprim::equal_to<int64_t>(), s_));
        t = temp<char>((int64_t)bytes);
        DCHECK(rocprim::unique(t, bytes, b, a, cnt, (size_t)E, rocprim::equal_to<int64_t>(), s_));
        size_t R = 0;
        DCHECK(hipMemcpyAsync(&R, cnt, sizeof(R), hipMemcpyDeviceToHost, s_));
        DCHECK(hipStreamSynchronize(s_));
        p->rel_values.resize(R);
        DCHECK(hipMemcpyAsync(p->rel_values.data(), a, R * sizeof(int64_t), hipMemcpyDeviceToHost, s_));
        DCHECK(hipStreamSynchronize(s_));
        release(t);
        release(cnt);
        release(a);
        release(b);
    }
    const int64_t R = (int64_t)p->rel_values.size();
    p->nrel = R;
    p->rel_val32.resize(R);
    for (int64_t r = 0; r < R; ++r) {
        const int64_t v = p->rel_values[r];
        p->rel_val32[r] = (v >= 0 && v <= std::numeric_limits<int32_t>::max()) ? (int32_t)v : -1;
    }
    if ((uint64_t)std::max<int64_t>(R, 1) * (uint64_t)std::max<int64_t>(N, 1) <= (uint64_t)std::numeric_limits<uint32_t>::max())
        build<uint32_t>(ei, et, E, N, lo, hi, side);
    else
        build<uint64_t>(ei, et, E, N, lo, hi, side);
}

}  // namespace

// Copies every device-only table into its host vector (once): mpgnn_plan_export / table_size of a
// device-built plan.
int32_t sync_host_tables(mpgnn_plan* p) {
    if (!p->device_built) return MPGNN_OK;
    std::call_once(p->host_once, [&] {
        int32_t st = MPGNN_OK;
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(p->device);
        for (auto& t : p->dev_tables) {
            t.host->resize((size_t)t.n);
            if (t.n > 0 && hipMemcpy(t.host->data(), t.dev, (size_t)t.n * sizeof(int32_t), hipMemcpyDeviceToHost) != hipSuccess) {
                st = MPGNN_ERR_HIP;
                set_last_error("hipMemcpy of a device-built plan table failed");
                break;
            }
        }
        (void)hipSetDevice(prev);
        p->host_sync_status = st;  // every later call reports the same outcome (no half-filled OK)
    });
    if (p->host_sync_status != MPGNN_OK) set_last_error("a device-built plan's tables could not be copied to the host");
    return p->host_sync_status;
}

void free_device_plan(mpgnn_plan* p) {
    for (void* ptr : p->dev_allocs) (void)hipFree(ptr);
    p->dev_allocs.clear();
}

}  // namespace mpgnn

using namespace mpgnn;

extern "C" int32_t mpgnn_plan_create_device(const int64_t* edge_index, const int64_t* edge_type, int64_t num_edges,
                                            int64_t num_nodes, int64_t shard_lo, int64_t shard_hi, int32_t side,
                                            int32_t device, void* stream, mpgnn_plan** out) {
    if (!out) {
        set_last_error("out is NULL");
        return MPGNN_ERR_ARG;
    }
    *out = nullptr;
    if (side != MPGNN_SHARD_GATHERED && side != MPGNN_SHARD_ROWS) {
        set_last_error("unknown shard side");
        return MPGNN_ERR_ARG;
    }
    if (num_edges < 0 || num_nodes < 0) {
        set_last_error("negative size");
        return MPGNN_ERR_ARG;
    }
    if (num_edges > 0 && (!edge_index || !edge_type)) {
        set_last_error("edge arrays are NULL");
        return MPGNN_ERR_ARG;
    }
    if (num_edges >= (int64_t)std::numeric_limits<int32_t>::max() || num_nodes >= (int64_t)std::numeric_limits<int32_t>::max()) {
        set_last_error("graph exceeds int32 index range");
        return MPGNN_ERR_UNSUPPORTED;
    }
    shard_lo = std::max<int64_t>(0, shard_lo);
    shard_hi = std::min<int64_t>(num_nodes, shard_hi);
    if (shard_hi < shard_lo) shard_hi = shard_lo;
    mpgnn_plan* p = new (std::nothrow) mpgnn_plan();
    if (!p) {
        set_last_error("plan allocation failed");
        return MPGNN_ERR_ALLOC;
    }
    p->opt = mpgnn::default_options();
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) {
        delete p;
        set_last_error("hipSetDevice failed");
        return MPGNN_ERR_HIP;
    }
    p->device = device;
    p->device_built = true;
    int32_t st = MPGNN_OK;
    try {
        Builder b(p, static_cast<hipStream_t>(stream));
        b.build_all(edge_index, edge_type, num_edges, num_nodes, shard_lo, shard_hi, side);
    } catch (const BuildError& e) {
        st = e.code;
        set_last_error(std::string("device plan build: ") + e.what());
    } catch (const std::bad_alloc&) {
        st = MPGNN_ERR_ALLOC;
        set_last_error("host allocation failed while building the plan");
    } catch (const std::exception& e) {  // e.g. length_error from a vector resize: never cross the C ABI
        st = MPGNN_ERR_ALLOC;
        set_last_error(std::string("device plan build: ") + e.what());
    }
    (void)hipSetDevice(prev);
    if (st != MPGNN_OK) {
        free_device_plan(p);
        delete p;
        return st;
    }
    *out = p;
    return MPGNN_OK;
}
