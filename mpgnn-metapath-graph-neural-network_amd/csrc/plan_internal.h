// plan_internal.h — the graph plan shared by the host builder (plan.cpp) and the HIP
// launchers (rgcn_kernels.hip). Not part of the public ABI (include/mpgnn_rgcn.h).
#pragma once

#include <atomic>
#include <array>
#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "mpgnn_rgcn.h"

namespace mpgnn {

// Kernel-path switches of ONE plan (header enum mpgnn_option). A plan copies the process
// defaults (mpgnn_set_option) when it is created; mpgnn_plan_set_option changes that plan only,
// so every launch is decided by the plan it runs on (no process-wide switch is read on the
// compute path).
struct Options {
    bool exact_order = false;     // MPGNN_OPT_EXACT_ORDER: no ragged pieces anywhere
    bool rel_gemm = true;         // MPGNN_OPT_REL_GEMM: B-stationary GEMM for K ∈ {64, 128}, N = 128
    bool rel_wide = true;         // MPGNN_OPT_REL_WIDE: ... also for F_in = F_out = 256 (C5)
    bool gemm_bf3 = true;         // MPGNN_OPT_GEMM_BF3: the GEMMs on the bf16 matrix cores (3-way split)
    bool bwd_fused = true;        // MPGNN_OPT_BWD_FUSED: see bwd_bf3_kernel
    bool flat_fuse_split = true;  // MPGNN_OPT_FLAT_FUSE_SPLIT: hub rows of grad_x finished in the gather launch
    bool outer_vec = true;        // MPGNN_OPT_OUTER_VEC: outer_bf3v_kernel (16-B gathers, transposed LDS reads)
    bool outer_sq = false;        // MPGNN_OPT_OUTER_SQ: its 64 x 64 wave quarters + interleaved commit (measured slower)
    bool gemm_w_il = true;        // MPGNN_OPT_GEMM_W_IL: the K = 256 GEMM's interleaved commit
    bool outer_ranges = true;     // MPGNN_OPT_OUTER_RANGES: its chunks in balanced contiguous ranges per workgroup
    bool gemm_il = true;          // MPGNN_OPT_GEMM_IL: the interleaved GEMM item skeleton
    bool gemm_w1 = false;         // MPGNN_OPT_GEMM_W1: one workgroup per CU, 64-row items (K = N = 128)
    int outer_variant = 0;        // MPGNN_OPT_OUTER_VARIANT: weight-gradient slice pipeline order (0, 1, 2)
    int flat_u = 16;              // MPGNN_OPT_FLAT_U: gather-sum rows in flight per wave
    bool flat_pad = true;         // MPGNN_OPT_FLAT_PAD: forward gather-sum chunks from padded slot tables
    bool single_fold = false;     // MPGNN_OPT_SINGLE_FOLD: mode-SINGLE means folded into single_bf3_kernel
    bool side_reduce = false;     // MPGNN_OPT_BWD_SIDE_REDUCE: the weight gradient's slab sum on a side stream
    bool gemm_first = true;       // MPGNN_OPT_GEMM_FIRST: the bf16-split GEMM's prologue from per-range records
    bool gemm_cu_pairs = true;    // MPGNN_OPT_GEMM_CU_PAIRS: GEMM item ranges balanced per CU
    int gemm_switch_cost = 150;  // MPGNN_OPT_GEMM_SWITCH_COST: range balance, items + c/100 per weight run (round 6 re-sweep)
    int flat_wg_per_cu = 0;       // MPGNN_OPT_FLAT_WG_PER_CU: persistent grid of flat_rows_kernel (0: off)
};
// a copy of the process defaults (rgcn_kernels.hip)
Options default_options();

// Segments are packed into relation-pure tiles of this many rows: one workgroup of the
// segment-transform kernel owns one tile (rgcn_kernels.hip, seg_tile_kernel).
constexpr int kTileRows = 64;
// 32-row relation-pure tiles of the B-stationary GEMM (rel_gemm_kernel): the work unit one
// wave-quad turns into 32 output rows while W_r stays in registers.
constexpr int kTile32 = 32;
// Cost model of one item of the fused mean + transform kernel, in units of 64 shader cycles:
// the MFMA strip takes 64 units; gathering an edge's 512-B row costs ≈ 23 cycles per CU.  Items
// are split over workgroups by prefix cost (fused_mean_gemm_kernel).
constexpr int kRootItemCost = 64;
inline int32_t item_cost(int64_t edges) {
    const int64_t g = (23 * edges + 1000) / 64;
    return (int32_t)(g > 64 ? g : 64);
}
// Relation-pure reduction chunks for the weight gradient (outer_accum_kernel): at most this
// many segments, balanced within a relation (bounds the longest workgroup's MFMA chain).
// 256 with the persistent 32-row-slice kernel (outer_persist_kernel): survey-recipe C3 outer +
// slab reduce 128.4 -> 120 us per layer (224: 135, 288: 129, 320: 137, 384: 135; 128: 136);
// scripts/layer_ab.py --chunk-rows, profiles/r02_chunk_rows_ab.jsonl
constexpr int kChunkRows = 256;
constexpr int64_t kChunkTarget = 4096;  // reduction chunks per graph (chunk length grows past kChunkRows)
// Ragged lists: a run (segment / gathered row) longer than this many entries is cut into
// ordered pieces of at most kPieceEntries, summed by piece_sum_kernel; consumers then add the
// piece partials in order.  Bounds the serial work of every wave (hub skew).
constexpr int kPieceEntries = 32;

// Two-level list over a position array: runs r cover positions [run_ptr[r], run_ptr[r+1]).
// ent[] lists, run by run, either a position p (>= 0) or a piece reference -(k+1); a piece k
// covers positions [piece_b[k], piece_e[k]).  ent_ptr[r] is the first entry of run r.
struct RaggedHost {
    std::vector<int32_t> ent, ent_ptr, piece_b, piece_e;
    std::vector<int32_t> res;            // [entries] idx[position] | -(piece+1)
    std::vector<int32_t> run_piece_ptr;  // [runs+1] first piece of each run
    int64_t nent = 0, npieces = 0;       // sizes (a device-built plan keeps the vectors on the device)
};

// Flat chunked list (flat_rows_kernel): the positions of a list whose consecutive runs are
// output rows, cut into chunks of at most kFlatChunk positions at run ends (and at forced cuts:
// relation boundaries of the segment lists). A run longer than a chunk is cut into pieces of
// kFlatChunk positions that hold only that run. Chunks are dealt to workgroups in GROUPS:
//   - a normal group: up to kFlatGroup chunks of complete runs (one wave each);
//   - a long group: the 2..kFlatLongPieces pieces of ONE run; the workgroup's waves sum the
//     pieces into LDS and one wave adds them in piece order (no second launch);
//   - pieces of a run longer than kFlatLongPieces chunks (grad_x hubs) go to normal groups as
//     split chunks: their partials go to global carry slots that finalize_rows_kernel adds in
//     chunk order.
constexpr int kFlatChunk = 32;
// The row-major (combine) lists: measured on the C3 survey graph (S + N = 222 k positions,
// ~15 per row) with the bf16-split GEMM, 16 / 32 / 48 / 64 positions per chunk: combine
// 26.7 / 22.7 / 23.2 / 24.5 µs (round 2 chose 16 on the 63 k-position graph of round 1)
constexpr int kFlatChunkRowMajor = 32;
constexpr int kFlatGroup = 4;         // chunks per normal group (= waves per workgroup)
constexpr int kFlatLongPieces = 16;   // pieces a long group sums in LDS (<= 16 · F floats); more
                                      // pieces serialise too much in one workgroup (C3 grad_x hubs:
                                      // 32 -> 49 vs 62 us)

struct FlatHost {
    std::vector<int32_t> chunk_ptr;   // [nch+1] positions
    std::vector<int32_t> chunk_info;  // [nch] bit0: first run split, bit1: last run split, >>2: carry slot
                                      // (long-group pieces: the piece index, an LDS slot)
    std::vector<int32_t> row_of;      // [positions] output row of each position
    std::vector<int32_t> group_ptr;   // [ngroups+1] chunk range of each workgroup
    std::vector<int32_t> group_long;  // [ngroups] 1: long group (pieces of one run)
    std::vector<int32_t> split_row;   // [nsplit] rows split across workgroups
    std::vector<int32_t> split_ptr;   // [nsplit+1] into split_slot
    std::vector<int32_t> split_slot;  // partial slots of each split row, in chunk order
    std::vector<int32_t> row_split;   // [nrows] split index of each row, -1 if not split
    std::vector<int32_t> cut_group_ptr;  // [ncuts+1] group range of each forced-cut section
    std::vector<int32_t> cut_split_ptr;  // [ncuts+1] split-row range of each section
    int32_t nslots = 0;
    int32_t max_pieces = 0;           // largest long group (its LDS slots: max_pieces · F floats)
    int32_t ngroups = 0, nsplit = 0;  // sizes (a device-built plan keeps the vectors on the device)
};

struct FlatDev {
    int32_t *chunk_ptr = nullptr, *chunk_info = nullptr, *row_of = nullptr;
    int32_t *group_ptr = nullptr, *group_long = nullptr;
    int32_t *split_row = nullptr, *split_ptr = nullptr, *split_slot = nullptr, *row_split = nullptr;
};

struct DeviceTables {
    int32_t* e_col = nullptr;
    int32_t* s_ptr = nullptr;
    int32_t* s_row = nullptr;
    int32_t* s_rel = nullptr;
    int32_t* s_cnt = nullptr;
    int32_t* s_pos = nullptr;
    int32_t* rw_ptr = nullptr;
    int32_t* rw_seg = nullptr;
    int32_t* t_ptr = nullptr;
    int32_t* t_seg = nullptr;
    int32_t* ta_col = nullptr;
    int32_t* ta_seg = nullptr;
    int32_t* tile_begin = nullptr;  // [num_tiles] first segment of the tile
    int32_t* tile_end = nullptr;    // [num_tiles] one past the last segment
    int32_t* t32_begin = nullptr;   // [num_tiles32] first segment of a 32-row tile
    int32_t* t32_end = nullptr;     // [num_tiles32] one past its last segment
    int32_t* t32_cost = nullptr;    // [num_tiles32 + 1] prefix of fused-kernel item costs
    int32_t* chunk_begin = nullptr; // [num_chunks]
    int32_t* chunk_end = nullptr;   // [num_chunks]
    int32_t* rel_chunk_ptr = nullptr; // [nrel+1]
    int32_t* chunk_dst = nullptr;   // [num_chunks] weight index when the relation has ONE chunk, else -1
    int32_t* rel_val32 = nullptr;   // [nrel] relation id clamped to int32 (-1 when it does not fit)
    // ragged lists (see RaggedHost)
    int32_t *seg_ent = nullptr, *seg_ent_ptr = nullptr, *seg_pb = nullptr, *seg_pe = nullptr;
    int32_t *t_ent = nullptr, *t_ent_ptr = nullptr, *t_pb = nullptr, *t_pe = nullptr;
    int32_t *ta_ent = nullptr, *ta_key = nullptr, *ta_pb = nullptr, *ta_pe = nullptr;
    int32_t *rw_ent = nullptr, *rw_ent_ptr = nullptr, *rw_pb = nullptr, *rw_pe = nullptr;
    int32_t *seg_res = nullptr, *t_res = nullptr, *ta_res = nullptr, *rw_res = nullptr;  // resolved entries
    FlatDev seg_f, t_f, rw_f;       // flat chunked lists (segment means, grad_x, combine)
    FlatDev tx_f, rwx_f;            // grad_x / combine lists with a trailing extra-row entry per own row
    // multi-edge segments (see mpgnn_plan::s_src)
    int32_t *s_src = nullptr, *m_ptr = nullptr, *em_col = nullptr, *m_cnt = nullptr;
    FlatDev segm_f;                 // flat chunked list of the multi-edge segments over em_col
    int32_t *tx_val = nullptr, *rwx_val = nullptr;  // their entry values (segment id | -(own row + 1))
    int32_t* rel_seg_ptr = nullptr; // [nrel+1] segment range of each dense relation
    // mode-SINGLE node maps, one row of N per dense relation + an all-zero row (absent relation):
    // map[d·N + i] = s_src + 1 (x row) or s_src (< 0: compact mean) of node i's relation-d
    // segment, 0 without one; built on the device at the first unsharded mode-SINGLE call when
    // (R+1)·N·4 <= 1 GiB (else, and inside a graph capture, the layer builds the relation's map
    // per call). Mode-ALL and sharded plans never allocate them.
    int32_t* rel_node_map = nullptr;
    void* block = nullptr;          // single hipMalloc holding every table above (but the maps)
    size_t block_bytes = 0;
};

}  // namespace mpgnn

struct mpgnn_plan {
    mpgnn::Options opt;  // this plan's kernel switches (copied from the process defaults at creation)
    int64_t N = 0;
    int64_t E_in = 0;
    int64_t E = 0;  // local edges kept
    int64_t S = 0;
    int64_t nrel = 0;
    int64_t shard_lo = 0, shard_hi = 0;

    std::vector<int64_t> rel_values;   // [nrel]
    std::vector<uint8_t> rel_invalid;  // [nrel]
    std::vector<int32_t> rel_seg_ptr;  // [nrel+1]
    std::vector<int32_t> rel_edge_ptr; // [nrel+1]
    std::vector<int32_t> rel_tile_ptr; // [nrel+1]
    std::vector<int32_t> rel_t32_ptr;  // [nrel+1] 32-row tiles of each relation
    std::vector<int32_t> rel_chunk_ptr;// [nrel+1]

    std::vector<int32_t> e_col, e_id;          // [E]
    std::vector<int32_t> s_ptr;                // [S+1]
    std::vector<int32_t> s_row, s_rel, s_cnt, s_pos;  // [S]
    std::vector<int32_t> rw_ptr;               // [N+1]
    std::vector<int32_t> rw_seg;               // [S]
    std::vector<int32_t> t_ptr;                // [N+1]
    std::vector<int32_t> t_seg;                // [E]
    std::vector<int32_t> ta_col, ta_seg;       // [E]
    std::vector<int32_t> tile_begin, tile_end; // [num_tiles]
    std::vector<int32_t> t32_begin, t32_end;   // [num_tiles32]
    std::vector<int32_t> t32_cost;             // [num_tiles32 + 1] prefix sum of item_cost()
    std::vector<int32_t> chunk_begin, chunk_end; // [num_chunks]
    std::vector<int32_t> rel_val32;            // [nrel]
    std::vector<int32_t> chunk_dst;            // [num_chunks] see DeviceTables::chunk_dst
    // A segment whose mean is one x row (one local edge, global count 1): s_src = its node_2;
    // otherwise s_src = -(m + 1), m = its multi-edge segment index (row m of the compact Hm)
    std::vector<int32_t> s_src;                // [S]
    std::vector<int32_t> m_ptr, em_col, m_cnt; // [Sm+1] / [Em] / [Sm]
    std::vector<int32_t> rel_m_ptr;            // [nrel+1]

    // ragged lists: segments over edges (forward gather), node_2 over col-major edges (grad_x,
    // all relations), (relation, node_2) runs over ta order (grad_x, one relation), node_1
    // over row-major segments (forward combine)
    mpgnn::RaggedHost seg_l, t_l, ta_l, rw_l;
    mpgnn::FlatHost segm_f;               // multi-edge segments over em_col (cut at relations)
    mpgnn::FlatHost seg_f, t_f, rw_f;     // flat chunked lists: segments over edges (cut at
                                          // relations), node_2 over col-major edges, node_1 over segments
    // grad_x / combine lists over [shard_lo, shard_hi) rows with one trailing entry per own row
    // (value -(row - shard_lo + 1): the G_root / Y_root row), so the flat kernel sums
    // (Σ entries) + extra in the reference order and no finalize pass is needed
    mpgnn::FlatHost tx_f, rwx_f;
    std::vector<int32_t> tx_val, rwx_val;
    std::vector<int32_t> ta_key;               // [ta entries] node_2 of each ta entry
    std::vector<int32_t> rel_ta_ent_ptr;       // [nrel+1] ta entry range of each relation
    std::vector<int32_t> rel_seg_piece_ptr;    // [nrel+1] seg pieces of each relation
    std::vector<int32_t> rel_ta_piece_ptr;     // [nrel+1] ta pieces of each relation

    int device = -1;
    mpgnn::DeviceTables d;

    // plans built on the device (plan_device.hip): every table is its own allocation and the big
    // ones reach their host vector only when exported (sync_host_tables)
    bool device_built = false;
    struct DevTable {
        std::vector<int32_t>* host;
        const int32_t* dev;
        int64_t n;
    };
    std::vector<DevTable> dev_tables;
    std::vector<void*> dev_allocs;
    std::once_flag host_once;
    int32_t host_sync_status = MPGNN_OK;  // outcome of the once-only host copy (sync_host_tables)
    // mode-SINGLE node maps (DeviceTables::rel_node_map): built lazily by the first unsharded
    // fused mode-SINGLE call that is not being graph-captured; tried once per plan
    mutable std::mutex node_map_mu;
    mutable std::atomic<bool> node_maps_tried{false};
    // bwd_bf3_kernel's slab layout per (selection, row range, grid): the first slab of every
    // workgroup and the slab range of every dense relation, on the device (made outside graph
    // captures by the first backward call of that shape; freed with the plan)
    struct BwSlabs {
        int* dev = nullptr;  // [G] first slab per workgroup, then [nrel + 1] relation slab ranges
        int n_slabs = 0, root_lo = 0;
    };
    mutable std::mutex bw_mu;
    mutable std::map<std::array<int64_t, 8>, BwSlabs> bw_slabs;
    // rel_gemm_bf3_kernel's cost-balanced item ranges per (tile range, root items, grid, cost):
    // [G + 1] first item of each range, then [items] weight index of each item, on the device
    // (made outside graph captures, uploaded from the pinned copy; both freed with the plan)
    struct GemmRanges {
        int* dev = nullptr;
        int* host = nullptr;  // pinned
    };
    mutable std::map<std::array<int64_t, 5>, GemmRanges> gemm_ranges;
    // rel_gemm_bf3_kernel's per-range prologue records (RelGemmArgs::first; device only)
    mutable std::map<std::array<int64_t, 5>, GemmRanges> gemm_first;
    // outer_bf3v_kernel_t's per-workgroup chunk ranges (same ownership as gemm_ranges)
    mutable std::map<std::array<int64_t, 5>, GemmRanges> outer_ranges;
    // flat_rows_kernel's padded slot tables per (list, value table) (rgcn_kernels.hip
    // flat_pad_tables): one device block {desc, val, row}; host unused
    mutable std::map<std::array<int64_t, 5>, GemmRanges> flat_pads;
};

namespace mpgnn {

void set_last_error(const std::string& msg);
// rgcn_kernels.hip: allocate + fill DeviceTables::rel_node_map on `stream` (synchronised before
// return; first unsharded mode-SINGLE use of the plan, never during a graph capture)
int32_t build_rel_node_maps(mpgnn_plan* p, void* stream);
// plan_device.hip: copy a device-built plan's tables into its host vectors (once); free its tables
int32_t sync_host_tables(mpgnn_plan* p);
void free_device_plan(mpgnn_plan* p);
extern int g_chunk_rows;     // MPGNN_OPT_CHUNK_ROWS: reduction chunk base length (default kChunkRows)
extern int g_plan_threads;  // host threads of mpgnn_plan_create (0 = hardware concurrency, ≤ 16)

// Resolve (mode, relation, R) to a contiguous dense-relation range [d_lo, d_hi).
// Returns MPGNN_ERR_INDEX if a selected relation is flagged invalid.
int32_t select_relations(const mpgnn_plan* p, int32_t mode, int64_t relation, int32_t R,
                         int64_t* d_lo, int64_t* d_hi);

}  // namespace mpgnn
