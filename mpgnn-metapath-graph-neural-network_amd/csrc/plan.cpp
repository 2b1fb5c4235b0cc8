// plan.cpp — host-side graph plan builder (segment tables) for the relation-typed SpMM.
//
// The reference recomputes, on every call and for every relation, the boolean compaction
// `edge_index[:, edge_type == r]` (mp_rgcn_layer.py:29-35, called at :231 for one relation
// and once per relation in the RGCNConv loop ≙ :250-251), then lets PyG gather
// x[edge_index[1]] and scatter-add into edge_index[0] (flow='target_to_source',
// model.py:137,190). Here the graph is sorted ONCE into tables that make every later pass a
// contiguous, order-preserving walk:
//
//   relation-major edges   stable sort by (relation, node_1)    -> segments (node_1, relation)
//   row-major segments     stable sort of segments by node_1    -> combine pass (sum over r)
//   col-major edges        stable sort by (node_2, relation)    -> grad_x (transposed SpMM)
//   relation/col edges     stable sort by (relation, node_2)    -> grad_x for one relation
//
// All sorts are stable counting sorts, O(E + N + R). Within a segment the edges keep their
// original order, which is what makes the GPU segment sums bit-identical to ATen's
// sequential scatter_add_ (SURVEY §8c "Determinism facts").
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <limits>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "plan_internal.h"

namespace mpgnn {

static thread_local std::string g_last_error;

void set_last_error(const std::string& msg) { g_last_error = msg; }

static int32_t fail(int32_t code, const std::string& msg) {
    set_last_error(msg);
    return code;
}

int32_t select_relations(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R,
                         int64_t* d_lo, int64_t* d_hi) {
    const auto& rv = p->rel_values;
    if (mode == MPGNN_MODE_SINGLE) {
        auto it = std::lower_bound(rv.begin(), rv.end(), relation);
        int64_t d = it - rv.begin();
        if (it == rv.end() || *it != relation) {  // relation absent: empty mask (no error)
            *d_lo = *d_hi = d;
            return MPGNN_OK;
        }
        if (p->rel_invalid[d])
            return fail(MPGNN_ERR_INDEX, "edge of relation " + std::to_string(relation) +
                                             " has a node index out of range [0, N)");
        *d_lo = d;
        *d_hi = d + 1;
        return MPGNN_OK;
    }
    if (mode == MPGNN_MODE_ALL) {
        if (R < 0) return fail(MPGNN_ERR_ARG, "num_relations must be >= 0");
        int64_t lo = std::lower_bound(rv.begin(), rv.end(), (int64_t)0) - rv.begin();
        int64_t hi = std::lower_bound(rv.begin(), rv.end(), (int64_t)R) - rv.begin();
        for (int64_t d = lo; d < hi; ++d)
            if (p->rel_invalid[d])
                return fail(MPGNN_ERR_INDEX, "edge of relation " + std::to_string(rv[d]) +
                                                 " has a node index out of range [0, N)");
        *d_lo = lo;
        *d_hi = hi;
        return MPGNN_OK;
    }
    return fail(MPGNN_ERR_ARG, "unknown mode " + std::to_string(mode));
}

// ---- host parallelism ------------------------------------------------------------------
// The build is a chain of O(E) passes with scattered accesses (32 M edges at C5). Passes over
// independent elements split into contiguous thread ranges; the counting sorts keep their
// stability by giving thread t the t-th contiguous slice of the input and the t-th slot of
// every bucket. Results do not depend on the thread count (tests/test_plan.py).
int g_chunk_rows = kChunkRows;
int g_plan_threads = 0;  // MPGNN_OPT_PLAN_THREADS: 0 = hardware concurrency, capped at 16
static constexpr int64_t kParMin = 1 << 16;  // fewer elements: one thread

static int plan_threads(int64_t n) {
    if (n < kParMin) return 1;
    int t = g_plan_threads > 0 ? g_plan_threads : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    return (int)std::max<int64_t>(1, std::min<int64_t>(t, n / (kParMin / 4)));
}

// fn(t, begin, end) over T contiguous ranges of [0, n)
template <class Fn>
static void parallel_ranges(int64_t n, int T, Fn fn) {
    if (T <= 1) {
        fn(0, (int64_t)0, n);
        return;
    }
    std::vector<std::thread> pool;
    pool.reserve(T - 1);
    for (int t = 1; t < T; ++t) pool.emplace_back([&, t] { fn(t, n * t / T, n * (t + 1) / T); });
    fn(0, (int64_t)0, n / T);
    for (auto& th : pool) th.join();
}

template <class Fn>
static void parallel_for(int64_t n, Fn fn) {
    parallel_ranges(n, plan_threads(n), [&](int, int64_t b, int64_t e) {
        for (int64_t i = b; i < e; ++i) fn(i);
    });
}

// Exclusive prefix sum in place; returns the total.
static int64_t exclusive_scan(std::vector<int32_t>& v) {
    int64_t acc = 0;
    for (auto& x : v) {
        const int64_t c = x;
        x = (int32_t)acc;
        acc += c;
    }
    return acc;
}

// Starts of the runs of [0, n) where same(a - 1, a) is false (a = 0 always starts), then n.
template <class SameFn>
static std::vector<int32_t> run_starts(int64_t n, SameFn same) {
    std::vector<uint8_t> head(n);
    parallel_for(n, [&](int64_t a) { head[a] = a == 0 || !same(a - 1, a); });
    const int T = plan_threads(n);
    std::vector<int64_t> part(T + 1, 0);
    parallel_ranges(n, T, [&](int t, int64_t b, int64_t e) {
        int64_t c = 0;
        for (int64_t a = b; a < e; ++a) c += head[a];
        part[t + 1] = c;
    });
    for (int t = 0; t < T; ++t) part[t + 1] += part[t];
    std::vector<int32_t> starts(part[T] + 1, (int32_t)n);
    parallel_ranges(n, T, [&](int t, int64_t b, int64_t e) {
        int64_t w = part[t];
        for (int64_t a = b; a < e; ++a)
            if (head[a]) starts[w++] = (int32_t)a;
    });
    return starts;
}

// Stable counting sort of `items` by key(item) in [0, nkeys). Returns the bucket pointers.
template <class KeyFn>
static void counting_sort(const std::vector<int32_t>& items, int64_t nkeys, KeyFn key,
                          std::vector<int32_t>& out, std::vector<int32_t>* ptr_out) {
    const int64_t n = (int64_t)items.size();
    // per-thread histograms cost T·nkeys: use threads only when the input dominates
    const int T = (nkeys <= 4 * n) ? plan_threads(n) : 1;
    std::vector<int32_t> ptr(nkeys + 1, 0);
    out.assign(items.size(), 0);
    if (T == 1) {
        for (int32_t it : items) ptr[key(it) + 1]++;
        for (int64_t k = 0; k < nkeys; ++k) ptr[k + 1] += ptr[k];
        std::vector<int32_t> cur(ptr.begin(), ptr.end() - 1);
        for (int32_t it : items) out[cur[key(it)]++] = it;
    } else {
        std::vector<std::vector<int32_t>> hist(T);
        parallel_ranges(n, T, [&](int t, int64_t b, int64_t e) {
            hist[t].assign(nkeys, 0);
            int32_t* h = hist[t].data();
            for (int64_t i = b; i < e; ++i) h[key(items[i])]++;
        });
        // bucket k starts at ptr[k]; thread t writes after threads < t: hist[t][k] becomes its cursor
        parallel_ranges(nkeys, T, [&](int, int64_t kb, int64_t ke) {
            for (int64_t k = kb; k < ke; ++k) {
                int32_t c = 0;
                for (int t = 0; t < T; ++t) c += hist[t][k];
                ptr[k + 1] = c;
            }
        });
        for (int64_t k = 0; k < nkeys; ++k) ptr[k + 1] += ptr[k];
        parallel_ranges(nkeys, T, [&](int, int64_t kb, int64_t ke) {
            for (int64_t k = kb; k < ke; ++k) {
                int32_t c = ptr[k];
                for (int t = 0; t < T; ++t) {
                    const int32_t h = hist[t][k];
                    hist[t][k] = c;
                    c += h;
                }
            }
        });
        parallel_ranges(n, T, [&](int t, int64_t b, int64_t e) {
            int32_t* cur = hist[t].data();
            for (int64_t i = b; i < e; ++i) out[cur[key(items[i])]++] = items[i];
        });
    }
    if (ptr_out) ptr_out->swap(ptr);
}

// Two-level list (see RaggedHost) over runs given by run_ptr: counts per run, prefix sums,
// then every run fills its own entries and pieces.
static void build_ragged(const std::vector<int32_t>& run_ptr, RaggedHost& L) {
    const int64_t runs = run_ptr.empty() ? 0 : (int64_t)run_ptr.size() - 1;
    L.ent_ptr.assign(runs + 1, 0);
    L.run_piece_ptr.assign(runs + 1, 0);
    parallel_for(runs, [&](int64_t r) {
        const int32_t len = run_ptr[r + 1] - run_ptr[r];
        const int32_t np = len <= kPieceEntries ? 0 : (len + kPieceEntries - 1) / kPieceEntries;
        L.ent_ptr[r] = np == 0 ? len : np;
        L.run_piece_ptr[r] = np;
    });
    const int64_t n_ent = exclusive_scan(L.ent_ptr);
    const int64_t n_pc = exclusive_scan(L.run_piece_ptr);
    L.ent_ptr[runs] = (int32_t)n_ent;
    L.run_piece_ptr[runs] = (int32_t)n_pc;
    L.nent = n_ent;
    L.npieces = n_pc;
    L.ent.assign(n_ent, 0);
    L.piece_b.assign(n_pc, 0);
    L.piece_e.assign(n_pc, 0);
    parallel_for(runs, [&](int64_t r) {
        const int32_t a = run_ptr[r], b = run_ptr[r + 1];
        int32_t w = L.ent_ptr[r];
        if (L.run_piece_ptr[r + 1] == L.run_piece_ptr[r]) {
            for (int32_t q = a; q < b; ++q) L.ent[w++] = q;
        } else {
            int32_t k = L.run_piece_ptr[r];
            for (int32_t q = a; q < b; q += kPieceEntries, ++k) {
                L.ent[w++] = -k - 1;
                L.piece_b[k] = q;
                L.piece_e[k] = std::min<int32_t>(q + kPieceEntries, b);
            }
        }
    });
}

// Flat chunked list over runs r (positions [run_ptr[r], run_ptr[r+1]), output row r) with
// forced cuts at run indices `cuts` (ascending, first 0, last = runs); see FlatHost.
static void build_flat(const std::vector<int32_t>& run_ptr, const std::vector<int32_t>& cuts, FlatHost& L,
                       int32_t chunk = kFlatChunk) {
    const int32_t runs = run_ptr.empty() ? 0 : (int32_t)run_ptr.size() - 1;
    const int32_t P = runs > 0 ? run_ptr[runs] : 0;
    L = FlatHost{};
    L.row_of.resize(P);
    parallel_for(runs, [&](int64_t r) {
        for (int32_t q = run_ptr[r]; q < run_ptr[r + 1]; ++q) L.row_of[q] = (int32_t)r;
    });
    L.row_split.assign(runs, -1);
    L.chunk_ptr.push_back(0);
    L.group_ptr.push_back(0);
    L.cut_group_ptr.push_back(0);
    L.split_ptr.push_back(0);
    L.cut_split_ptr.push_back(0);
    int32_t slot = 0;
    auto nch = [&] { return (int32_t)L.chunk_ptr.size() - 1; };
    auto close_group = [&](int32_t is_long) {
        if (nch() > L.group_ptr.back()) {
            L.group_ptr.push_back(nch());
            L.group_long.push_back(is_long);
        }
    };
    for (size_t ci = 0; ci + 1 < cuts.size(); ++ci) {
        int32_t cs = run_ptr[cuts[ci]];  // start of the open chunk
        for (int32_t r = cuts[ci]; r < cuts[ci + 1]; ++r) {
            const int32_t q = run_ptr[r], e = run_ptr[r + 1];
            if (e - q <= chunk) {
                if (e - cs > chunk) {  // run r does not fit the open chunk: close it before r
                    L.chunk_ptr.push_back(q);
                    L.chunk_info.push_back(0);
                    cs = q;
                    if (nch() - L.group_ptr.back() == kFlatGroup) close_group(0);
                }
                continue;
            }
            // long run: close the open chunk and group, then the run's pieces
            if (q > cs) {
                L.chunk_ptr.push_back(q);
                L.chunk_info.push_back(0);
            }
            close_group(0);
            const int32_t k = (e - q + chunk - 1) / chunk;
            const bool local = k <= kFlatLongPieces;
            if (!local) {
                L.row_split[r] = (int32_t)L.split_row.size();
                L.split_row.push_back(r);
                L.split_ptr.push_back(L.split_ptr.back());
            }
            for (int32_t i = 0; i < k; ++i) {
                L.chunk_ptr.push_back(std::min(q + (i + 1) * chunk, e));
                const int32_t flags = (i > 0 ? 1 : 0) | (i + 1 < k ? 2 : 0);
                if (local) {
                    L.chunk_info.push_back(flags | (i << 2));
                } else {
                    L.chunk_info.push_back(flags | (slot << 2));
                    L.split_slot.push_back(slot++);
                    ++L.split_ptr.back();
                    if (nch() - L.group_ptr.back() == kFlatGroup) close_group(0);
                }
            }
            close_group(local ? 1 : 0);
            if (local) L.max_pieces = std::max(L.max_pieces, k);
            cs = e;
        }
        const int32_t pe = run_ptr[cuts[ci + 1]];
        if (pe > cs) {
            L.chunk_ptr.push_back(pe);
            L.chunk_info.push_back(0);
        }
        close_group(0);
        L.cut_group_ptr.push_back((int32_t)L.group_ptr.size() - 1);
        L.cut_split_ptr.push_back((int32_t)L.split_row.size());
    }
    L.nslots = slot;
    L.ngroups = (int32_t)L.group_ptr.size() - 1;
    L.nsplit = (int32_t)L.split_row.size();
}

// Resolved entries: a position p becomes idx[p] (what the gather loads), a piece reference
// stays negative — the gather then needs one index load per entry instead of two.
static void resolve_ragged(RaggedHost& L, const std::vector<int32_t>& idx) {
    L.res.resize(L.ent.size());
    parallel_for((int64_t)L.ent.size(), [&](int64_t q) { L.res[q] = L.ent[q] >= 0 ? idx[L.ent[q]] : L.ent[q]; });
}

struct PhaseTimer {
    bool on = std::getenv("MPGNN_PLAN_TIMING") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void mark(const char* what) {
        if (!on) return;
        auto n = std::chrono::steady_clock::now();
        fprintf(stderr, "[plan] %-28s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(n - t).count());
        t = n;
    }
};

static int32_t build(const int64_t* ei, const int64_t* et, int64_t E, int64_t N, int64_t lo,
                     int64_t hi, int32_t side, mpgnn_plan* p) {
    PhaseTimer tm;
    const int64_t* n1 = ei;
    const int64_t* n2 = ei + E;
    p->N = N;
    p->E_in = E;
    p->shard_lo = lo;
    p->shard_hi = hi;

    // ---- dense relation ids (sorted distinct values of edge_type) ----------------------
    std::vector<int32_t> rel_d(E);
    if (E > 0) {
        int64_t mn = et[0], mx = et[0];
        for (int64_t e = 1; e < E; ++e) {
            mn = std::min(mn, et[e]);
            mx = std::max(mx, et[e]);
        }
        const unsigned long long span = (unsigned long long)mx - (unsigned long long)mn;
        if (span < (unsigned long long)(4 * E + 4096)) {
            std::vector<int32_t> map(span + 1, -1);
            for (int64_t e = 0; e < E; ++e) map[et[e] - mn] = 0;
            int32_t nd = 0;
            for (size_t v = 0; v <= span; ++v)
                if (map[v] == 0) {
                    map[v] = nd++;
                    p->rel_values.push_back(mn + (int64_t)v);
                }
            parallel_for(E, [&](int64_t e) { rel_d[e] = map[et[e] - mn]; });
        } else {
            std::vector<int64_t> vals(et, et + E);
            std::sort(vals.begin(), vals.end());
            vals.erase(std::unique(vals.begin(), vals.end()), vals.end());
            p->rel_values = vals;
            for (int64_t e = 0; e < E; ++e)
                rel_d[e] = (int32_t)(std::lower_bound(vals.begin(), vals.end(), et[e]) - vals.begin());
        }
    }
    const int64_t R = (int64_t)p->rel_values.size();
    p->nrel = R;
    p->rel_invalid.assign(R, 0);
    p->rel_val32.resize(R);
    for (int64_t d = 0; d < R; ++d) {
        int64_t v = p->rel_values[d];
        p->rel_val32[d] = (v >= 0 && v <= std::numeric_limits<int32_t>::max()) ? (int32_t)v : -1;
    }

    tm.mark("dense relation ids");
    // ---- valid edges, global (relation, node_1, edge) order ------------------------------
    std::vector<int32_t> valid;
    valid.reserve(E);
    for (int64_t e = 0; e < E; ++e) {
        if (n1[e] < 0 || n1[e] >= N || n2[e] < 0 || n2[e] >= N) {
            p->rel_invalid[rel_d[e]] = 1;
            continue;
        }
        valid.push_back((int32_t)e);
    }
    std::vector<int32_t> by_row, by_rel_row;
    counting_sort(valid, N, [&](int32_t e) { return (int64_t)n1[e]; }, by_row, nullptr);
    counting_sort(by_row, R, [&](int32_t e) { return (int64_t)rel_d[e]; }, by_rel_row, nullptr);

    tm.mark("valid + 2 counting sorts");
    // ---- segments: runs of equal (relation, node_1); keep those with a local edge --------
    // pass 1: run starts (global segments); pass 2: local edge count of each; prefix sums
    // give segment ids and edge offsets; pass 3: every kept segment fills its own entries.
    p->rel_seg_ptr.assign(R + 1, 0);
    p->rel_edge_ptr.assign(R + 1, 0);
    const int64_t V = (int64_t)by_rel_row.size();
    const std::vector<int32_t> gstart = run_starts(V, [&](int64_t a, int64_t b) {  // global segments, + V
        const int32_t ea = by_rel_row[a], eb = by_rel_row[b];
        return rel_d[ea] == rel_d[eb] && n1[ea] == n1[eb];
    });
    const int64_t G = (int64_t)gstart.size() - 1;
    tm.mark("  segment run starts");
    std::vector<int32_t> seg_id(G), edge_off(G);  // kept: local edge count, then offsets
    parallel_for(G, [&](int64_t g) {
        int32_t c = 0;
        for (int32_t a = gstart[g]; a < gstart[g + 1]; ++a) {
            const int32_t e = by_rel_row[a];
            const int64_t k = side == MPGNN_SHARD_ROWS ? n1[e] : n2[e];
            c += (k >= lo && k < hi) ? 1 : 0;
        }
        edge_off[g] = c;
        seg_id[g] = c > 0 ? 1 : 0;
    });
    tm.mark("  segment local counts");
    const int64_t S_loc = exclusive_scan(seg_id);
    const int64_t E_loc = exclusive_scan(edge_off);
    p->e_col.assign(E_loc, 0);
    p->e_id.assign(E_loc, 0);
    p->s_row.assign(S_loc, 0);
    p->s_rel.assign(S_loc, 0);
    p->s_cnt.assign(S_loc, 0);
    p->s_ptr.assign(S_loc + 1, (int32_t)E_loc);
    std::vector<int32_t> seg_of_edge(E_loc);  // segment id of each local edge (relation-major order)
    std::vector<int32_t> seg_d(S_loc);        // dense relation of each kept segment (ascending)
    parallel_for(G, [&](int64_t g) {
        const int32_t a0 = gstart[g], a1 = gstart[g + 1];
        const int32_t next_off = g + 1 < G ? edge_off[g + 1] : (int32_t)E_loc;
        if (next_off == edge_off[g]) return;  // no local edge: segment not kept
        const int32_t sid = seg_id[g];
        const int32_t e0 = by_rel_row[a0];
        int32_t w = edge_off[g];
        for (int32_t a = a0; a < a1; ++a) {
            const int32_t e = by_rel_row[a];
            const int64_t k = side == MPGNN_SHARD_ROWS ? n1[e] : n2[e];
            if (k >= lo && k < hi) {
                p->e_col[w] = (int32_t)n2[e];
                p->e_id[w] = e;
                seg_of_edge[w] = sid;
                ++w;
            }
        }
        p->s_row[sid] = (int32_t)n1[e0];
        seg_d[sid] = rel_d[e0];
        p->s_rel[sid] = p->rel_val32[rel_d[e0]];
        p->s_cnt[sid] = a1 - a0;  // GLOBAL count of (row, relation)
        p->s_ptr[sid] = edge_off[g];
    });
    tm.mark("  segment fill");
    p->E = E_loc;
    p->S = S_loc;
    // kept segments per dense relation: segments are relation-major, so the range of relation d
    // starts at the first segment whose dense relation is >= d
    for (int64_t d = 0; d <= R; ++d)
        p->rel_seg_ptr[d] = (int32_t)(std::lower_bound(seg_d.begin(), seg_d.end(), (int32_t)d) - seg_d.begin());
    for (int64_t d = 0; d < R; ++d)
        p->rel_edge_ptr[d + 1] = p->s_ptr[p->rel_seg_ptr[d + 1]];
    tm.mark("segments");

    // ---- multi-edge segments: the only means the forward materialises ------------------
    // A segment with one local edge and global count 1 has mean == x[node_2] bit for bit (x / 1),
    // so the transform GEMMs read that x row directly (s_src[s] = node_2 >= 0). Every other
    // segment (78 % of the C3 segments are single-edge, 87 % at C5) gets a compact row m of Hm
    // (s_src[s] = -(m + 1)), summed over the compacted edge list em_col / m_ptr.
    {
        const int64_t S = p->S;
        std::vector<int32_t> m_id(S), m_off(S);
        parallel_for(S, [&](int64_t s) {
            const int32_t loc = p->s_ptr[s + 1] - p->s_ptr[s];
            const bool multi = !(loc == 1 && p->s_cnt[s] == 1);
            m_id[s] = multi ? 1 : 0;
            m_off[s] = multi ? loc : 0;
        });
        const int64_t Sm = exclusive_scan(m_id);
        const int64_t Em = exclusive_scan(m_off);
        p->s_src.assign(S, 0);
        p->m_cnt.assign(Sm, 0);
        p->m_ptr.assign(Sm + 1, (int32_t)Em);
        p->em_col.assign(Em, 0);
        parallel_for(S, [&](int64_t s) {
            const int32_t b = p->s_ptr[s], e = p->s_ptr[s + 1];
            const bool multi = !(e - b == 1 && p->s_cnt[s] == 1);
            if (!multi) {
                p->s_src[s] = p->e_col[b];
                return;
            }
            const int32_t m = m_id[s];
            p->s_src[s] = -m - 1;
            p->m_cnt[m] = p->s_cnt[s];
            p->m_ptr[m] = m_off[s];
            std::copy(p->e_col.begin() + b, p->e_col.begin() + e, p->em_col.begin() + m_off[s]);
        });
        p->rel_m_ptr.assign(R + 1, (int32_t)Sm);
        for (int64_t d = 0; d < R; ++d)
            p->rel_m_ptr[d] = p->rel_seg_ptr[d] < S ? m_id[p->rel_seg_ptr[d]] : (int32_t)Sm;
    }
    tm.mark("multi-edge segments");


    // ---- row-major segment order (node_1, relation) -------------------------------------
    {
        std::vector<int32_t> segs(p->S);
        parallel_for(p->S, [&](int64_t s) { segs[s] = (int32_t)s; });
        counting_sort(segs, N, [&](int32_t s) { return (int64_t)p->s_row[s]; }, p->rw_seg, &p->rw_ptr);
        p->s_pos.assign(p->S, 0);
        parallel_for(p->S, [&](int64_t q) { p->s_pos[p->rw_seg[q]] = (int32_t)q; });
    }

    tm.mark("row-major order");
    const std::vector<int32_t> node_cuts{0, (int32_t)N};
    // augmented lists: own rows [lo, hi) get a trailing extra-row entry
    auto augment = [&](const std::vector<int32_t>& ptr, const std::vector<int32_t>& val, FlatHost& F,
                       std::vector<int32_t>& out_val, int32_t chunk) {
        std::vector<int32_t> xptr(N + 1, 0);
        parallel_for(N, [&](int64_t i) { xptr[i] = ptr[i] + (int32_t)std::clamp<int64_t>(i, lo, hi) - (int32_t)lo; });
        xptr[N] = ptr[N] + (int32_t)(hi - lo);
        out_val.assign(xptr[N], 0);
        parallel_for(N, [&](int64_t i) {
            int32_t w = xptr[i];
            for (int32_t q = ptr[i]; q < ptr[i + 1]; ++q) out_val[w++] = val[q];
            if (i >= lo && i < hi) out_val[w] = -(int32_t)(i - lo) - 1;
        });
        build_flat(xptr, node_cuts, F, chunk);
    };
    // The backward-only tables (transposed orders, grad_x lists) are independent of the forward
    // ones from here on: built on a second host thread beside them (C5: ~2x shorter plan build).
    std::exception_ptr bwd_error;
    std::thread bwd_thread([&] {
        try {
            // ---- transposed orders for grad_x -------------------------------------------
            std::vector<int32_t> edges(p->E);
            parallel_for(p->E, [&](int64_t k) { edges[k] = (int32_t)k; });
            std::vector<int32_t> by_col;  // (node_2, relation, node_1, edge)
            counting_sort(edges, N, [&](int32_t k) { return (int64_t)p->e_col[k]; }, by_col, &p->t_ptr);
            p->t_seg.resize(p->E);
            parallel_for(p->E, [&](int64_t q) { p->t_seg[q] = seg_of_edge[by_col[q]]; });
            // edges are relation-major, so an edge's dense relation follows from its position
            std::vector<int32_t> edge_d(p->E);
            parallel_for(R, [&](int64_t d) {
                for (int32_t k = p->rel_edge_ptr[d]; k < p->rel_edge_ptr[d + 1]; ++k) edge_d[k] = (int32_t)d;
            });
            std::vector<int32_t> by_rel_col;  // (relation, node_2, node_1, edge)
            counting_sort(by_col, R, [&](int32_t k) { return (int64_t)edge_d[k]; }, by_rel_col, nullptr);
            p->ta_col.resize(p->E);
            p->ta_seg.resize(p->E);
            parallel_for(p->E, [&](int64_t q) {
                p->ta_col[q] = p->e_col[by_rel_col[q]];
                p->ta_seg[q] = seg_of_edge[by_rel_col[q]];
            });
            // ragged + flat grad_x lists
            build_ragged(p->t_ptr, p->t_l);
            resolve_ragged(p->t_l, p->t_seg);
            build_flat(p->t_ptr, node_cuts, p->t_f);
            augment(p->t_ptr, p->t_seg, p->tx_f, p->tx_val, kFlatChunk);
            // runs of equal (relation, node_2) in ta order (mode SINGLE grad_x)
            const std::vector<int32_t> run_ptr = run_starts(p->E, [&](int64_t a, int64_t b) {
                return edge_d[a] == edge_d[b] && p->ta_col[a] == p->ta_col[b];
            });
            const int64_t nruns = (int64_t)run_ptr.size() - 1;
            std::vector<int32_t> run_key(nruns), run_rel(nruns);
            parallel_for(nruns, [&](int64_t r) {
                run_key[r] = p->ta_col[run_ptr[r]];
                run_rel[r] = edge_d[run_ptr[r]];
            });
            build_ragged(run_ptr, p->ta_l);
            resolve_ragged(p->ta_l, p->ta_seg);
            const size_t runs = run_key.size();
            p->ta_key.resize(p->ta_l.ent.size());
            parallel_for((int64_t)runs, [&](int64_t r) {
                for (int32_t q = p->ta_l.ent_ptr[r]; q < p->ta_l.ent_ptr[r + 1]; ++q) p->ta_key[q] = run_key[r];
            });
            p->rel_ta_ent_ptr.assign(R + 1, 0);
            p->rel_ta_piece_ptr.assign(R + 1, 0);
            size_t r = 0;
            for (int64_t d = 0; d < R; ++d) {
                p->rel_ta_ent_ptr[d] = p->ta_l.ent_ptr[r];
                p->rel_ta_piece_ptr[d] = p->ta_l.run_piece_ptr[r];
                while (r < runs && run_rel[r] == d) ++r;
            }
            p->rel_ta_ent_ptr[R] = p->ta_l.ent_ptr[runs];
            p->rel_ta_piece_ptr[R] = p->ta_l.run_piece_ptr[runs];
        } catch (...) {
            bwd_error = std::current_exception();
        }
    });
    try {
        // ---- forward lists: ragged (exact order) + flat (segments, multi-edge, combine) ----
        build_ragged(p->s_ptr, p->seg_l);
        build_ragged(p->rw_ptr, p->rw_l);
        resolve_ragged(p->seg_l, p->e_col);
        resolve_ragged(p->rw_l, p->rw_seg);
        // segments over edges, cut at relation boundaries (mode SINGLE selects one relation)
        std::vector<int32_t> seg_cuts(p->rel_seg_ptr.begin(), p->rel_seg_ptr.end());
        build_flat(p->s_ptr, seg_cuts, p->seg_f);
        build_flat(p->m_ptr, p->rel_m_ptr, p->segm_f);  // multi-edge segments, cut at relations
        build_flat(p->rw_ptr, node_cuts, p->rw_f, kFlatChunkRowMajor);
        augment(p->rw_ptr, p->rw_seg, p->rwx_f, p->rwx_val, kFlatChunkRowMajor);
    } catch (...) {
        bwd_thread.join();
        throw;
    }
    tm.mark("forward lists");
    bwd_thread.join();
    if (bwd_error) std::rethrow_exception(bwd_error);
    tm.mark("backward tables (joined)");
    p->rel_seg_piece_ptr.assign(R + 1, 0);
    for (int64_t d = 0; d <= R; ++d) p->rel_seg_piece_ptr[d] = p->seg_l.run_piece_ptr[p->rel_seg_ptr[d]];

    // ---- relation-pure tiles and reduction chunks --------------------------------------
    p->rel_tile_ptr.assign(R + 1, 0);
    p->rel_t32_ptr.assign(R + 1, 0);
    p->t32_cost.assign(1, 0);
    p->rel_chunk_ptr.assign(R + 1, 0);
    // Reduction chunk length: kChunkRows, grown with the graph so that there are about
    // kChunkTarget chunks in all. Every chunk writes an F_in × F_out partial slab that the
    // reduce kernel reads back, so at C5 (S = 27.5 M, F = 256) 128-row chunks would write as
    // many slab bytes as the whole input of dW (56 GB); 4096 chunks keep the slabs at ~1 GB
    // and still give > 16 workgroups per CU.
    const int64_t s_all = p->rel_seg_ptr[R];
    const int32_t chunk_cap = (int32_t)std::max<int64_t>(g_chunk_rows, (s_all + kChunkTarget - 1) / kChunkTarget + 31) / 32 * 32;
    for (int64_t d = 0; d < R; ++d) {
        for (int32_t s = p->rel_seg_ptr[d]; s < p->rel_seg_ptr[d + 1]; s += kTile32) {
            p->t32_begin.push_back(s);
            p->t32_end.push_back(std::min<int32_t>(s + kTile32, p->rel_seg_ptr[d + 1]));
        }
        p->rel_t32_ptr[d + 1] = (int32_t)p->t32_begin.size();
        for (size_t t = p->t32_cost.size() - 1; t < p->t32_begin.size(); ++t) {
            const int64_t e = p->s_ptr[p->t32_end[t]] - p->s_ptr[p->t32_begin[t]];
            p->t32_cost.push_back(p->t32_cost.back() + item_cost(e));
        }
        for (int32_t s = p->rel_seg_ptr[d]; s < p->rel_seg_ptr[d + 1]; s += kTileRows) {
            p->tile_begin.push_back(s);
            p->tile_end.push_back(std::min<int32_t>(s + kTileRows, p->rel_seg_ptr[d + 1]));
        }
        p->rel_tile_ptr[d + 1] = (int32_t)p->tile_begin.size();
        // balanced chunks of at most chunk_cap segments (multiples of 32 rows but the last)
        const int32_t sb = p->rel_seg_ptr[d], se = p->rel_seg_ptr[d + 1];
        const int32_t nch = (se - sb + chunk_cap - 1) / chunk_cap;
        const int32_t per = nch > 0 ? ((se - sb + nch - 1) / nch + 31) / 32 * 32 : 0;
        for (int32_t s = sb; s < se; s += per) {
            p->chunk_begin.push_back(s);
            p->chunk_end.push_back(std::min<int32_t>(s + per, se));
            p->chunk_dst.push_back(nch == 1 ? p->rel_val32[d] : -1);
        }
        p->rel_chunk_ptr[d + 1] = (int32_t)p->chunk_begin.size();
    }
    tm.mark("tiles + chunks");
    return MPGNN_OK;
}

}  // namespace mpgnn

using namespace mpgnn;

extern "C" {

int32_t mpgnn_abi_version(void) { return 1; }

const char* mpgnn_last_error(void) { return g_last_error.c_str(); }

const char* mpgnn_status_string(int32_t s) {
    switch (s) {
        case MPGNN_OK: return "ok";
        case MPGNN_ERR_ARG: return "invalid argument";
        case MPGNN_ERR_INDEX: return "index out of range";
        case MPGNN_ERR_HIP: return "HIP runtime error";
        case MPGNN_ERR_NOT_ON_DEVICE: return "plan not uploaded to a device";
        case MPGNN_ERR_ALLOC: return "allocation failed";
        case MPGNN_ERR_UNSUPPORTED: return "unsupported feature width";
        default: return "unknown status";
    }
}

int32_t mpgnn_plan_create(const int64_t* edge_index, const int64_t* edge_type, int64_t num_edges,
                          int64_t num_nodes, int64_t shard_lo, int64_t shard_hi, mpgnn_plan** out) {
    return mpgnn_plan_create_sharded(edge_index, edge_type, num_edges, num_nodes, shard_lo, shard_hi,
                                     MPGNN_SHARD_GATHERED, out);
}

int32_t mpgnn_plan_create_sharded(const int64_t* edge_index, const int64_t* edge_type, int64_t num_edges,
                                  int64_t num_nodes, int64_t shard_lo, int64_t shard_hi, int32_t side,
                                  mpgnn_plan** out) {
    if (!out) return fail(MPGNN_ERR_ARG, "out is NULL");
    if (side != MPGNN_SHARD_GATHERED && side != MPGNN_SHARD_ROWS) return fail(MPGNN_ERR_ARG, "unknown shard side");
    *out = nullptr;
    if (num_edges < 0 || num_nodes < 0) return fail(MPGNN_ERR_ARG, "negative size");
    if (num_edges > 0 && (!edge_index || !edge_type)) return fail(MPGNN_ERR_ARG, "edge arrays are NULL");
    if (num_edges >= (int64_t)std::numeric_limits<int32_t>::max() ||
        num_nodes >= (int64_t)std::numeric_limits<int32_t>::max())
        return fail(MPGNN_ERR_UNSUPPORTED, "graph exceeds int32 index range");
    shard_lo = std::max<int64_t>(0, shard_lo);
    shard_hi = std::min<int64_t>(num_nodes, shard_hi);
    if (shard_hi < shard_lo) shard_hi = shard_lo;
    mpgnn_plan* p = new (std::nothrow) mpgnn_plan();
    if (!p) return fail(MPGNN_ERR_ALLOC, "plan allocation failed");
    p->opt = mpgnn::default_options();
    try {
        int32_t st = build(edge_index, edge_type, num_edges, num_nodes, shard_lo, shard_hi, side, p);
        if (st != MPGNN_OK) {
            delete p;
            return st;
        }
    } catch (const std::bad_alloc&) {
        delete p;
        return fail(MPGNN_ERR_ALLOC, "host allocation failed while building the plan");
    }
    *out = p;
    return MPGNN_OK;
}

int32_t mpgnn_plan_destroy(mpgnn_plan* p) {
    if (!p) return MPGNN_OK;
    if (p->d.block || p->device_built) {
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(p->device);
        if (p->d.block) (void)hipFree(p->d.block);
        free_device_plan(p);
        if (p->d.rel_node_map) (void)hipFree(p->d.rel_node_map);
        for (auto& kv : p->bw_slabs) (void)hipFree(kv.second.dev);
        for (auto* m : {&p->gemm_ranges, &p->outer_ranges, &p->flat_pads, &p->gemm_first})
            for (auto& kv : *m) {
                (void)hipFree(kv.second.dev);
                (void)hipHostFree(kv.second.host);
            }
        (void)hipSetDevice(prev);
    }
    delete p;
    return MPGNN_OK;
}

int32_t mpgnn_plan_get_info(const mpgnn_plan* p, mpgnn_plan_info* info) {
    if (!p || !info) return fail(MPGNN_ERR_ARG, "NULL argument");
    std::memset(info, 0, sizeof(*info));
    info->num_nodes = p->N;
    info->num_edges_in = p->E_in;
    info->num_edges = p->E;
    info->num_segments = p->S;
    info->num_relations = p->nrel;
    info->num_tiles = (int64_t)p->tile_begin.size();
    info->num_chunks = (int64_t)p->chunk_begin.size();
    info->shard_lo = p->shard_lo;
    info->shard_hi = p->shard_hi;
    info->device = p->device;
    return MPGNN_OK;
}

static const void* table_ptr(const mpgnn_plan* p, int32_t t, int64_t* n, int32_t* eb) {
    *eb = 4;
    switch (t) {
        case MPGNN_T_REL_VALUES: *eb = 8; *n = (int64_t)p->rel_values.size(); return p->rel_values.data();
        case MPGNN_T_REL_SEG_PTR: *n = (int64_t)p->rel_seg_ptr.size(); return p->rel_seg_ptr.data();
        case MPGNN_T_REL_EDGE_PTR: *n = (int64_t)p->rel_edge_ptr.size(); return p->rel_edge_ptr.data();
        case MPGNN_T_E_COL: *n = (int64_t)p->e_col.size(); return p->e_col.data();
        case MPGNN_T_E_ID: *n = (int64_t)p->e_id.size(); return p->e_id.data();
        case MPGNN_T_S_PTR: *n = (int64_t)p->s_ptr.size(); return p->s_ptr.data();
        case MPGNN_T_S_ROW: *n = (int64_t)p->s_row.size(); return p->s_row.data();
        case MPGNN_T_S_REL: *n = (int64_t)p->s_rel.size(); return p->s_rel.data();
        case MPGNN_T_S_CNT: *n = (int64_t)p->s_cnt.size(); return p->s_cnt.data();
        case MPGNN_T_S_POS: *n = (int64_t)p->s_pos.size(); return p->s_pos.data();
        case MPGNN_T_RW_PTR: *n = (int64_t)p->rw_ptr.size(); return p->rw_ptr.data();
        case MPGNN_T_RW_SEG: *n = (int64_t)p->rw_seg.size(); return p->rw_seg.data();
        case MPGNN_T_T_PTR: *n = (int64_t)p->t_ptr.size(); return p->t_ptr.data();
        case MPGNN_T_T_SEG: *n = (int64_t)p->t_seg.size(); return p->t_seg.data();
        case MPGNN_T_TA_COL: *n = (int64_t)p->ta_col.size(); return p->ta_col.data();
        case MPGNN_T_TA_SEG: *n = (int64_t)p->ta_seg.size(); return p->ta_seg.data();
        case MPGNN_T_REL_INVALID: *eb = 1; *n = (int64_t)p->rel_invalid.size(); return p->rel_invalid.data();
        case MPGNN_T_S_SRC: *n = (int64_t)p->s_src.size(); return p->s_src.data();
        case MPGNN_T_M_PTR: *n = (int64_t)p->m_ptr.size(); return p->m_ptr.data();
        case MPGNN_T_EM_COL: *n = (int64_t)p->em_col.size(); return p->em_col.data();
        case MPGNN_T_M_CNT: *n = (int64_t)p->m_cnt.size(); return p->m_cnt.data();
        case MPGNN_T_REL_M_PTR: *n = (int64_t)p->rel_m_ptr.size(); return p->rel_m_ptr.data();
        default: break;
    }
    if (t >= MPGNN_T_SEG_F_GROUP_PTR && t < MPGNN_T_COUNT) {
        const int k = t - MPGNN_T_SEG_F_GROUP_PTR;
        const FlatHost* lists[4] = {&p->seg_f, &p->t_f, &p->rw_f, &p->segm_f};
        const std::vector<int32_t>* v = (k & 1) ? &lists[k >> 1]->group_long : &lists[k >> 1]->group_ptr;
        *n = (int64_t)v->size();
        return v->data();
    }
    const bool seg_lists = t >= MPGNN_T_SEG_F_CHUNK_PTR && t <= MPGNN_T_RW_F_SPLIT_SLOT;
    if (seg_lists || (t >= MPGNN_T_SEGM_F_CHUNK_PTR && t <= MPGNN_T_SEGM_F_SPLIT_SLOT)) {
        const int k = seg_lists ? t - MPGNN_T_SEG_F_CHUNK_PTR : t - MPGNN_T_SEGM_F_CHUNK_PTR;
        const FlatHost& L = !seg_lists ? p->segm_f : (k < 6 ? p->seg_f : (k < 12 ? p->t_f : p->rw_f));
        const std::vector<int32_t>* v = nullptr;
        switch (k % 6) {
            case 0: v = &L.chunk_ptr; break;
            case 1: v = &L.chunk_info; break;
            case 2: v = &L.row_of; break;
            case 3: v = &L.split_row; break;
            case 4: v = &L.split_ptr; break;
            default: v = &L.split_slot; break;
        }
        *n = (int64_t)v->size();
        return v->data();
    }
    switch (t) {
        default: *n = -1; return nullptr;
    }
}

int32_t mpgnn_plan_table_size(const mpgnn_plan* p, int32_t table, int64_t* elems, int32_t* elem_bytes) {
    if (!p || !elems || !elem_bytes) return fail(MPGNN_ERR_ARG, "NULL argument");
    if (int32_t st = sync_host_tables(const_cast<mpgnn_plan*>(p)); st != MPGNN_OK) return st;
    table_ptr(p, table, elems, elem_bytes);
    if (*elems < 0) return fail(MPGNN_ERR_ARG, "unknown table id " + std::to_string(table));
    return MPGNN_OK;
}

int32_t mpgnn_plan_export(const mpgnn_plan* p, int32_t table, void* dst, int64_t capacity) {
    if (!p) return fail(MPGNN_ERR_ARG, "NULL plan");
    if (int32_t st = sync_host_tables(const_cast<mpgnn_plan*>(p)); st != MPGNN_OK) return st;
    int64_t n = 0;
    int32_t eb = 0;
    const void* src = table_ptr(p, table, &n, &eb);
    if (n < 0) return fail(MPGNN_ERR_ARG, "unknown table id " + std::to_string(table));
    if (n * eb > capacity) return fail(MPGNN_ERR_ARG, "destination too small");
    if (n > 0) {
        if (!dst) return fail(MPGNN_ERR_ARG, "NULL destination");
        std::memcpy(dst, src, (size_t)(n * eb));
    }
    return MPGNN_OK;
}

int32_t mpgnn_plan_digest(const mpgnn_plan* cp, uint64_t* out) {
    if (!cp || !out) return fail(MPGNN_ERR_ARG, "NULL argument");
    mpgnn_plan* p = const_cast<mpgnn_plan*>(cp);
    if (int32_t st = sync_host_tables(p); st != MPGNN_OK) return st;
    uint64_t h = 1469598103934665603ull;  // FNV-1a over 32-bit words, sizes included
    auto word = [&](uint64_t w) { h = (h ^ w) * 1099511628211ull; };
    auto vec = [&](const std::vector<int32_t>& v) {
        word(v.size());
        for (int32_t x : v) word((uint32_t)x);
    };
    for (int64_t v : {p->N, p->E_in, p->E, p->S, p->nrel, p->shard_lo, p->shard_hi}) word((uint64_t)v);
    for (int64_t v : p->rel_values) word((uint64_t)v);
    for (uint8_t v : p->rel_invalid) word(v);
    for (const std::vector<int32_t>* v :
         {&p->rel_seg_ptr, &p->rel_edge_ptr, &p->rel_tile_ptr, &p->rel_t32_ptr, &p->rel_chunk_ptr, &p->e_col, &p->e_id,
          &p->s_ptr, &p->s_row, &p->s_rel, &p->s_cnt, &p->s_pos, &p->rw_ptr, &p->rw_seg, &p->t_ptr, &p->t_seg, &p->ta_col,
          &p->ta_seg, &p->tile_begin, &p->tile_end, &p->t32_begin, &p->t32_end, &p->t32_cost, &p->chunk_begin,
          &p->chunk_end, &p->rel_val32, &p->chunk_dst, &p->s_src, &p->m_ptr, &p->em_col, &p->m_cnt, &p->rel_m_ptr,
          &p->tx_val, &p->rwx_val, &p->ta_key, &p->rel_ta_ent_ptr, &p->rel_seg_piece_ptr, &p->rel_ta_piece_ptr})
        vec(*v);
    for (const RaggedHost* L : {&p->seg_l, &p->t_l, &p->ta_l, &p->rw_l}) {
        for (const std::vector<int32_t>* v : {&L->ent, &L->ent_ptr, &L->piece_b, &L->piece_e, &L->res, &L->run_piece_ptr})
            vec(*v);
        word((uint64_t)L->nent);
        word((uint64_t)L->npieces);
    }
    for (const FlatHost* L : {&p->seg_f, &p->t_f, &p->rw_f, &p->tx_f, &p->rwx_f, &p->segm_f}) {
        for (const std::vector<int32_t>* v : {&L->chunk_ptr, &L->chunk_info, &L->row_of, &L->group_ptr, &L->group_long,
                                              &L->split_row, &L->split_ptr, &L->split_slot, &L->row_split,
                                              &L->cut_group_ptr, &L->cut_split_ptr})
            vec(*v);
        for (int32_t v : {L->nslots, L->max_pieces, L->ngroups, L->nsplit}) word((uint32_t)v);
    }
    *out = h;
    return MPGNN_OK;
}

int32_t mpgnn_plan_select(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R,
                          int64_t* seg_begin, int64_t* seg_end) {
    if (!p || !seg_begin || !seg_end) return fail(MPGNN_ERR_ARG, "NULL argument");
    int64_t lo = 0, hi = 0;
    int32_t st = select_relations(p, mode, relation, R, &lo, &hi);
    if (st != MPGNN_OK) return st;
    *seg_begin = p->rel_seg_ptr.empty() ? 0 : p->rel_seg_ptr[lo];
    *seg_end = p->rel_seg_ptr.empty() ? 0 : p->rel_seg_ptr[hi];
    return MPGNN_OK;
}

int32_t mpgnn_plan_upload(mpgnn_plan* p, int32_t device) {
    if (!p) return fail(MPGNN_ERR_ARG, "NULL plan");
    if (p->d.block || p->device_built) {
        if (p->device == device) return MPGNN_OK;
        return fail(MPGNN_ERR_ARG, "plan already uploaded to another device");
    }
    struct Item {
        int32_t** dst;
        const std::vector<int32_t>* src;
    };
    Item items[] = {
        {&p->d.e_col, &p->e_col},       {&p->d.s_ptr, &p->s_ptr},
        {&p->d.s_row, &p->s_row},       {&p->d.s_rel, &p->s_rel},
        {&p->d.s_cnt, &p->s_cnt},       {&p->d.s_pos, &p->s_pos},
        {&p->d.rw_ptr, &p->rw_ptr},     {&p->d.rw_seg, &p->rw_seg},
        {&p->d.t_ptr, &p->t_ptr},       {&p->d.t_seg, &p->t_seg},
        {&p->d.ta_col, &p->ta_col},     {&p->d.ta_seg, &p->ta_seg},
        {&p->d.tile_begin, &p->tile_begin}, {&p->d.tile_end, &p->tile_end},
        {&p->d.t32_begin, &p->t32_begin}, {&p->d.t32_end, &p->t32_end},
        {&p->d.t32_cost, &p->t32_cost},
        {&p->d.chunk_begin, &p->chunk_begin}, {&p->d.chunk_end, &p->chunk_end},
        {&p->d.rel_chunk_ptr, &p->rel_chunk_ptr}, {&p->d.rel_val32, &p->rel_val32},
        {&p->d.chunk_dst, &p->chunk_dst},
        {&p->d.seg_ent, &p->seg_l.ent}, {&p->d.seg_ent_ptr, &p->seg_l.ent_ptr},
        {&p->d.seg_pb, &p->seg_l.piece_b}, {&p->d.seg_pe, &p->seg_l.piece_e},
        {&p->d.t_ent, &p->t_l.ent}, {&p->d.t_ent_ptr, &p->t_l.ent_ptr},
        {&p->d.t_pb, &p->t_l.piece_b}, {&p->d.t_pe, &p->t_l.piece_e},
        {&p->d.ta_ent, &p->ta_l.ent}, {&p->d.ta_key, &p->ta_key},
        {&p->d.ta_pb, &p->ta_l.piece_b}, {&p->d.ta_pe, &p->ta_l.piece_e},
        {&p->d.rw_ent, &p->rw_l.ent}, {&p->d.rw_ent_ptr, &p->rw_l.ent_ptr},
        {&p->d.rw_pb, &p->rw_l.piece_b}, {&p->d.rw_pe, &p->rw_l.piece_e},
        {&p->d.seg_res, &p->seg_l.res}, {&p->d.t_res, &p->t_l.res},
        {&p->d.ta_res, &p->ta_l.res}, {&p->d.rw_res, &p->rw_l.res},
        {&p->d.seg_f.chunk_ptr, &p->seg_f.chunk_ptr}, {&p->d.seg_f.chunk_info, &p->seg_f.chunk_info},
        {&p->d.seg_f.row_of, &p->seg_f.row_of}, {&p->d.seg_f.split_row, &p->seg_f.split_row},
        {&p->d.seg_f.split_ptr, &p->seg_f.split_ptr}, {&p->d.seg_f.split_slot, &p->seg_f.split_slot},
        {&p->d.seg_f.row_split, &p->seg_f.row_split}, {&p->d.seg_f.group_ptr, &p->seg_f.group_ptr}, {&p->d.seg_f.group_long, &p->seg_f.group_long},
        {&p->d.t_f.chunk_ptr, &p->t_f.chunk_ptr}, {&p->d.t_f.chunk_info, &p->t_f.chunk_info},
        {&p->d.t_f.row_of, &p->t_f.row_of}, {&p->d.t_f.split_row, &p->t_f.split_row},
        {&p->d.t_f.split_ptr, &p->t_f.split_ptr}, {&p->d.t_f.split_slot, &p->t_f.split_slot},
        {&p->d.t_f.row_split, &p->t_f.row_split}, {&p->d.t_f.group_ptr, &p->t_f.group_ptr}, {&p->d.t_f.group_long, &p->t_f.group_long},
        {&p->d.rw_f.chunk_ptr, &p->rw_f.chunk_ptr}, {&p->d.rw_f.chunk_info, &p->rw_f.chunk_info},
        {&p->d.rw_f.row_of, &p->rw_f.row_of}, {&p->d.rw_f.split_row, &p->rw_f.split_row},
        {&p->d.rw_f.split_ptr, &p->rw_f.split_ptr}, {&p->d.rw_f.split_slot, &p->rw_f.split_slot},
        {&p->d.rw_f.row_split, &p->rw_f.row_split}, {&p->d.rw_f.group_ptr, &p->rw_f.group_ptr}, {&p->d.rw_f.group_long, &p->rw_f.group_long},
        {&p->d.tx_f.chunk_ptr, &p->tx_f.chunk_ptr}, {&p->d.tx_f.chunk_info, &p->tx_f.chunk_info},
        {&p->d.tx_f.row_of, &p->tx_f.row_of}, {&p->d.tx_f.split_row, &p->tx_f.split_row},
        {&p->d.tx_f.split_ptr, &p->tx_f.split_ptr}, {&p->d.tx_f.split_slot, &p->tx_f.split_slot},
        {&p->d.tx_f.row_split, &p->tx_f.row_split}, {&p->d.tx_f.group_ptr, &p->tx_f.group_ptr}, {&p->d.tx_f.group_long, &p->tx_f.group_long}, {&p->d.tx_val, &p->tx_val},
        {&p->d.rwx_f.chunk_ptr, &p->rwx_f.chunk_ptr}, {&p->d.rwx_f.chunk_info, &p->rwx_f.chunk_info},
        {&p->d.rwx_f.row_of, &p->rwx_f.row_of}, {&p->d.rwx_f.split_row, &p->rwx_f.split_row},
        {&p->d.rwx_f.split_ptr, &p->rwx_f.split_ptr}, {&p->d.rwx_f.split_slot, &p->rwx_f.split_slot},
        {&p->d.rwx_f.row_split, &p->rwx_f.row_split}, {&p->d.rwx_f.group_ptr, &p->rwx_f.group_ptr}, {&p->d.rwx_f.group_long, &p->rwx_f.group_long}, {&p->d.rwx_val, &p->rwx_val},
        {&p->d.rel_seg_ptr, &p->rel_seg_ptr}, {&p->d.s_src, &p->s_src}, {&p->d.m_ptr, &p->m_ptr}, {&p->d.em_col, &p->em_col}, {&p->d.m_cnt, &p->m_cnt},
        {&p->d.segm_f.chunk_ptr, &p->segm_f.chunk_ptr}, {&p->d.segm_f.chunk_info, &p->segm_f.chunk_info},
        {&p->d.segm_f.row_of, &p->segm_f.row_of}, {&p->d.segm_f.split_row, &p->segm_f.split_row},
        {&p->d.segm_f.split_ptr, &p->segm_f.split_ptr}, {&p->d.segm_f.split_slot, &p->segm_f.split_slot},
        {&p->d.segm_f.row_split, &p->segm_f.row_split}, {&p->d.segm_f.group_ptr, &p->segm_f.group_ptr}, {&p->d.segm_f.group_long, &p->segm_f.group_long},
    };
    size_t total = 0;
    std::vector<size_t> offs;
    for (auto& it : items) {
        offs.push_back(total);
        total += ((it.src->size() * sizeof(int32_t) + 255) / 256) * 256;
    }
    total = std::max<size_t>(total, 256);
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess) return fail(MPGNN_ERR_HIP, "hipGetDevice failed");
    if (hipSetDevice(device) != hipSuccess) return fail(MPGNN_ERR_HIP, "hipSetDevice failed");
    void* block = nullptr;
    hipError_t err = hipMalloc(&block, total);
    if (err != hipSuccess) {
        (void)hipSetDevice(prev);
        return fail(MPGNN_ERR_ALLOC, std::string("hipMalloc: ") + hipGetErrorString(err));
    }
    std::vector<char> staging(total, 0);
    for (size_t i = 0; i < sizeof(items) / sizeof(items[0]); ++i) {
        if (!items[i].src->empty())
            std::memcpy(staging.data() + offs[i], items[i].src->data(), items[i].src->size() * sizeof(int32_t));
        *items[i].dst = reinterpret_cast<int32_t*>(static_cast<char*>(block) + offs[i]);
    }
    err = hipMemcpy(block, staging.data(), total, hipMemcpyHostToDevice);
    (void)hipSetDevice(prev);
    if (err != hipSuccess) {
        (void)hipFree(block);
        return fail(MPGNN_ERR_HIP, std::string("hipMemcpy: ") + hipGetErrorString(err));
    }
    p->d.block = block;
    p->d.block_bytes = total;
    p->device = device;
    return MPGNN_OK;  // the mode-SINGLE node maps are built on first use (build_rel_node_maps)
}

}  // extern "C"
