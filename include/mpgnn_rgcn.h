/*
 * mpgnn_rgcn.h — C ABI of the MI355X (gfx950) relation-typed aggregation library.
 *
 * This is the drop-in boundary for the hot path of the reference
 * (francescoferrini/MPGNN-Metapath-Graph-Neural-Network): the relation-masked
 * mean aggregation + per-relation dense transform of
 *   - CustomRGCNConv.forward      mp_rgcn_layer.py:158-271  ("mode SINGLE": one
 *     relation per call, 2-D weight [F_in, F_out], used by MPNetm model.py:190,192)
 *   - PyG RGCNConv.forward loop   ≙ mp_rgcn_layer.py:249-258 with weight [R, F_in, F_out]
 *     ("mode ALL": relations 0..R-1, used by Net model.py:137-138)
 * plus their autograd backward (implicit at main.py:1078 / main_rgcn.py:392).
 *
 * Conventions
 *   - Every function returns int32_t status: 0 = ok, < 0 = mpgnn_status. No exception
 *     crosses the ABI; mpgnn_last_error() returns a thread-local message.
 *   - Graph tensors follow the reference loader (main.py:366-372):
 *     edge_index int64 [2, E] row-major (row 0 = node_1, row 1 = node_2), edge_type int64 [E].
 *     The plan is always built for flow='target_to_source' (model.py:137,190): rows of the
 *     output are edge_index[0]; the gathered side is edge_index[1]. A caller that wants PyG's
 *     default 'source_to_target' passes the two rows swapped.
 *   - Feature/weight buffers are fp32, row-major, contiguous, 16-byte aligned DEVICE pointers
 *     owned by the caller (PyTorch caching allocator). All kernels are enqueued on `stream`
 *     (a hipStream_t passed as void*); no call synchronises the device except
 *     mpgnn_plan_upload().
 *   - Multi-GPU (dst-range sharding): a plan built with [shard_lo, shard_hi)
 *     keeps only edges whose node_2 lies in the range, while per-(node_1, relation) counts
 *     stay GLOBAL, so forward outputs of all shards sum (all-reduce) to the unsharded result.
 *     The root/bias term is added only for output rows in [row_lo, row_hi).
 */
#ifndef MPGNN_RGCN_H
#define MPGNN_RGCN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mpgnn_plan mpgnn_plan; /* opaque graph plan (segment tables) */

enum mpgnn_status {
    MPGNN_OK = 0,
    MPGNN_ERR_ARG = -1,         /* bad shape / null pointer / bad mode */
    MPGNN_ERR_INDEX = -2,       /* node index out of range (reference: index_select raises) */
    MPGNN_ERR_HIP = -3,         /* HIP runtime error */
    MPGNN_ERR_NOT_ON_DEVICE = -4, /* kernel called before mpgnn_plan_upload */
    MPGNN_ERR_ALLOC = -5,       /* host or device allocation failed */
    MPGNN_ERR_UNSUPPORTED = -6  /* feature width outside the compiled kernel range (1..256) */
};

enum mpgnn_mode {
    MPGNN_MODE_SINGLE = 0, /* CustomRGCNConv: edges with edge_type == relation; weight [F_in, F_out] */
    MPGNN_MODE_ALL = 1     /* RGCNConv: relations 0..num_relations-1; weight [R, F_in, F_out] */
};

/* Host tables exported by mpgnn_plan_export (tests compare them bit-exactly with the oracle). */
enum mpgnn_table {
    MPGNN_T_REL_VALUES = 0,  /* int64 [nrel]   sorted distinct relation ids                        */
    MPGNN_T_REL_SEG_PTR = 1, /* int32 [nrel+1] segment range of each relation                      */
    MPGNN_T_REL_EDGE_PTR = 2,/* int32 [nrel+1] edge range of each relation                         */
    MPGNN_T_E_COL = 3,       /* int32 [E]      node_2 of each edge, relation-major order            */
    MPGNN_T_E_ID = 4,        /* int32 [E]      original edge id of each edge, relation-major order  */
    MPGNN_T_S_PTR = 5,       /* int32 [S+1]    edge range of each segment                           */
    MPGNN_T_S_ROW = 6,       /* int32 [S]      node_1 of each segment                               */
    MPGNN_T_S_REL = 7,       /* int32 [S]      relation id of each segment                          */
    MPGNN_T_S_CNT = 8,       /* int32 [S]      GLOBAL edge count of (node_1, relation)              */
    MPGNN_T_S_POS = 9,       /* int32 [S]      position of the segment in (node_1, relation) order  */
    MPGNN_T_RW_PTR = 10,     /* int32 [N+1]    row-major segment range of each node_1               */
    MPGNN_T_RW_SEG = 11,     /* int32 [S]      segment id at each row-major position                */
    MPGNN_T_T_PTR = 12,      /* int32 [N+1]    edge range of each node_2 in (node_2, rel) order     */
    MPGNN_T_T_SEG = 13,      /* int32 [E]      segment id of each edge in (node_2, rel) order       */
    MPGNN_T_TA_COL = 14,     /* int32 [E]      node_2 of each edge in (rel, node_2) order           */
    MPGNN_T_TA_SEG = 15,     /* int32 [E]      segment id of each edge in (rel, node_2) order       */
    MPGNN_T_REL_INVALID = 16,/* uint8 [nrel]   1 if an edge of this relation had a bad node index   */
    /* flat chunked lists (fast-path row sums): for list L in {SEG = segments over edges (cut at
     * relations), T = node_2 over col-major edges, RW = node_1 over row-major segments}:
     * CHUNK_PTR [nch+1] positions (<= 32 each, cut at row ends; a longer row is cut into pieces
     * that hold only that row), CHUNK_INFO [nch] (bit0 first row split, bit1 last row split, >>2
     * carry slot — a long group's piece index), ROW_OF [positions], SPLIT_ROW [nsplit] (rows of
     * more than 16 pieces: summed across workgroups by the finalize kernel), SPLIT_PTR [nsplit+1],
     * SPLIT_SLOT [slots]                                                                         */
    MPGNN_T_SEG_F_CHUNK_PTR = 17, MPGNN_T_SEG_F_CHUNK_INFO = 18, MPGNN_T_SEG_F_ROW_OF = 19,
    MPGNN_T_SEG_F_SPLIT_ROW = 20, MPGNN_T_SEG_F_SPLIT_PTR = 21, MPGNN_T_SEG_F_SPLIT_SLOT = 22,
    MPGNN_T_T_F_CHUNK_PTR = 23, MPGNN_T_T_F_CHUNK_INFO = 24, MPGNN_T_T_F_ROW_OF = 25,
    MPGNN_T_T_F_SPLIT_ROW = 26, MPGNN_T_T_F_SPLIT_PTR = 27, MPGNN_T_T_F_SPLIT_SLOT = 28,
    MPGNN_T_RW_F_CHUNK_PTR = 29, MPGNN_T_RW_F_CHUNK_INFO = 30, MPGNN_T_RW_F_ROW_OF = 31,
    MPGNN_T_RW_F_SPLIT_ROW = 32, MPGNN_T_RW_F_SPLIT_PTR = 33, MPGNN_T_RW_F_SPLIT_SLOT = 34,
    /* multi-edge segments (the only segment means the layers materialise): a segment with one
     * local edge and global count 1 has mean == x[node_2] and is read from x directly */
    MPGNN_T_S_SRC = 35,      /* int32 [S]      node_2 of a single-edge segment (>= 0), else -(m+1)  */
    MPGNN_T_M_PTR = 36,      /* int32 [Sm+1]   edge range of multi-edge segment m in EM_COL         */
    MPGNN_T_EM_COL = 37,     /* int32 [Em]     node_2 of the edges of multi-edge segments, in order */
    MPGNN_T_M_CNT = 38,      /* int32 [Sm]     GLOBAL edge count of multi-edge segment m            */
    MPGNN_T_REL_M_PTR = 39,  /* int32 [nrel+1] multi-edge segment range of each relation            */
    /* SEGM = the flat chunked list of the multi-edge segments over EM_COL (cut at relations) */
    MPGNN_T_SEGM_F_CHUNK_PTR = 40, MPGNN_T_SEGM_F_CHUNK_INFO = 41, MPGNN_T_SEGM_F_ROW_OF = 42,
    MPGNN_T_SEGM_F_SPLIT_ROW = 43, MPGNN_T_SEGM_F_SPLIT_PTR = 44, MPGNN_T_SEGM_F_SPLIT_SLOT = 45,
    /* workgroup groups of the flat lists (SEG, T, RW, SEGM): GROUP_PTR [ngroups+1] chunk range of
     * each workgroup (<= 4 chunks of complete rows, or the 2..16 pieces of one long row),
     * GROUP_LONG [ngroups] 1 for a long row's group (pieces summed in LDS, in order)         */
    MPGNN_T_SEG_F_GROUP_PTR = 46, MPGNN_T_SEG_F_GROUP_LONG = 47, MPGNN_T_T_F_GROUP_PTR = 48,
    MPGNN_T_T_F_GROUP_LONG = 49, MPGNN_T_RW_F_GROUP_PTR = 50, MPGNN_T_RW_F_GROUP_LONG = 51,
    MPGNN_T_SEGM_F_GROUP_PTR = 52, MPGNN_T_SEGM_F_GROUP_LONG = 53,
    MPGNN_T_COUNT = 54
};

typedef struct mpgnn_plan_info {
    int64_t num_nodes;      /* N                                         */
    int64_t num_edges_in;   /* E given to plan_create                    */
    int64_t num_edges;      /* local (shard) edges kept                  */
    int64_t num_segments;   /* S = distinct local (node_1, relation)     */
    int64_t num_relations;  /* distinct relation ids in edge_type        */
    int64_t num_tiles;      /* 64-segment relation-pure tiles            */
    int64_t num_chunks;     /* relation-pure reduction chunks (dW)       */
    int64_t shard_lo, shard_hi;
    int32_t device;         /* -1 until mpgnn_plan_upload                */
    int32_t reserved;
} mpgnn_plan_info;

/* Build the segment tables on the host (O(E + N + R) counting sorts).
 * Replaces the per-call `edge_type == r` compaction mp_rgcn_layer.py:29-35,231,251 and
 * the index bookkeeping of PyG propagate (mp_rgcn_layer.py:236 / RGCNConv loop).
 * edge_index/edge_type are HOST pointers. Edges whose node ids fall outside [0, N) are
 * dropped and their relation is flagged invalid; kernels touching a flagged relation return
 * MPGNN_ERR_INDEX (mirrors IndexError of x.index_select). */
int32_t mpgnn_plan_create(const int64_t* edge_index, const int64_t* edge_type,
                          int64_t num_edges, int64_t num_nodes,
                          int64_t shard_lo, int64_t shard_hi, mpgnn_plan** out);
/* Shard by either side of the edges: MPGNN_SHARD_GATHERED keeps the edges whose
 * node_2 (the gathered row) is in [shard_lo, shard_hi) — every output row gets a partial sum
 * (global per-(node_1, relation) counts), summed across ranks by an all-reduce /
 * reduce-scatter; MPGNN_SHARD_ROWS keeps the edges whose node_1 (the aggregating row) is in
 * the range — the rank computes complete output rows for its range only (zeros elsewhere),
 * assembled across ranks by an all-gather (or an all-reduce of the disjoint rows).
 * In both, x @ root + bias is added for the rows in [shard_lo, shard_hi) only. */
enum mpgnn_shard_side { MPGNN_SHARD_GATHERED = 0, MPGNN_SHARD_ROWS = 1 };
int32_t mpgnn_plan_create_sharded(const int64_t* edge_index, const int64_t* edge_type, int64_t num_edges,
                                  int64_t num_nodes, int64_t shard_lo, int64_t shard_hi, int32_t side,
                                  mpgnn_plan** out);
/* The same plan built on the GPU from DEVICE-resident edge arrays (edge_index [2, E] and
 * edge_type [E], int64, on device `device`), enqueued on `stream` (a hipStream_t; NULL = the
 * null stream) and synchronised before return: stable radix sorts and prefix sums instead of the
 * host counting sorts, tables bit-identical to mpgnn_plan_create_sharded's. The tables stay on
 * the device (the plan counts as uploaded to `device`); mpgnn_plan_export copies them back on
 * first use. Replaces the per-call boolean compaction of mp_rgcn_layer.py:29-35 (called at :231)
 * like mpgnn_plan_create, for a graph that already lives on the GPU. */
int32_t mpgnn_plan_create_device(const int64_t* edge_index, const int64_t* edge_type, int64_t num_edges,
                                 int64_t num_nodes, int64_t shard_lo, int64_t shard_hi, int32_t side,
                                 int32_t device, void* stream, mpgnn_plan** out);
int32_t mpgnn_plan_destroy(mpgnn_plan* plan);
/* 64-bit fingerprint (FNV-1a) of every table of the plan, exported or internal: equal for plans
 * built from the same graph by either builder (tests/test_plan_device.py). */
int32_t mpgnn_plan_digest(const mpgnn_plan* plan, uint64_t* out);
int32_t mpgnn_plan_get_info(const mpgnn_plan* plan, mpgnn_plan_info* info);
/* Element count of an exported table, and a copy of it into host memory. */
int32_t mpgnn_plan_table_size(const mpgnn_plan* plan, int32_t table, int64_t* elems, int32_t* elem_bytes);
int32_t mpgnn_plan_export(const mpgnn_plan* plan, int32_t table, void* dst, int64_t capacity_bytes);
/* Copy the tables to device `device` (synchronous; call once per graph). */
int32_t mpgnn_plan_upload(mpgnn_plan* plan, int32_t device);

/* Rows (segments) a mode/relation selects: [seg_begin, seg_end) in relation-major order. */
int32_t mpgnn_plan_select(const mpgnn_plan* plan, int32_t mode, int64_t relation,
                          int32_t num_relations, int64_t* seg_begin, int64_t* seg_end);

const char* mpgnn_last_error(void);
const char* mpgnn_status_string(int32_t status);
int32_t mpgnn_abi_version(void);

/* --- device entry points ------------------------------------------------------------ */

/* Segment means h[s - seg_begin, :] = (Σ_{e in s} x[node_2(e), :]) / count(s), summed in
 * original edge order from 0.0f: bit-identical to PyG 2.3.1 scatter(reduce='mean') as
 * called by propagate at mp_rgcn_layer.py:236. h is [seg_end - seg_begin, F]. */
int32_t mpgnn_rel_mean_fwd(const mpgnn_plan* plan, int32_t mode, int64_t relation,
                           int32_t num_relations, const float* x, int32_t F, float* h,
                           void* stream);

/* Backward of mpgnn_rel_mean_fwd (autograd of PyG propagate's mean, mp_rgcn_layer.py:236):
 * dx[j] = Σ_{edges (i, r, j) of the selection} dh[seg(i, r)] / count(seg), dh [seg_end - seg_begin, F]
 * in the plan's segment order, dx [N, F] (every row written; rows without an edge are 0).
 * Scratch: mpgnn_rel_mean_bwd_workspace_bytes. */
int32_t mpgnn_rel_mean_bwd_workspace_bytes(const mpgnn_plan* plan, int32_t mode, int64_t relation,
                                           int32_t num_relations, int32_t F, int64_t* bytes);
int32_t mpgnn_rel_mean_bwd(const mpgnn_plan* plan, int32_t mode, int64_t relation, int32_t num_relations,
                           const float* dh, int32_t F, float* dx, void* workspace, void* stream);

/* ReLU backward of a layer whose ReLU was fused into the forward (mpgnn_rgcn_fwd_act):
 * dst[i] = act_out[i] > 0 ? grad_out[i] : 0 for n floats, one pass (dst may alias grad_out).
 * Replaces autograd's threshold_backward of F.relu(conv(...)) (model.py:144,146; main_rgcn
 * Net) and of the ReLU after each metapath layer (model.py:213-215). */
int32_t mpgnn_relu_bwd(const float* grad_out, const float* act_out, int64_t n, float* dst, void* stream);

/* Dropout's backward with the ReLU backward of the layer before it fused (MPNetm: F.relu(conv)
 * then Dropout(0.6), model.py:211-215): dst[i] = act_out[i] <= 0 ? 0 : grad_out[i] · mask[i] · scale
 * (torch's native_dropout_backward arithmetic, then threshold_backward's rule; act_out NULL: the
 * dropout backward alone). mask: the forward's keep mask (bool bytes), scale = 1 / (1 - p). */
int32_t mpgnn_dropout_relu_bwd(const float* grad_out, const uint8_t* mask, const float* act_out, float scale, int64_t n,
                               float* dst, void* stream);

/* Weight / bias gradient of the wrappers' Linear heads over all N node rows (Net.lin,
 * model.py:147; MPNetm.fc1/fc2, model.py:224-226): grad_weight[o][f] = Σ_i grad_out[i][o]·x[i][f],
 * grad_bias[o] = Σ_i grad_out[i][o] (nullable), row-sliced partials summed in a fixed order
 * (deterministic). x [N,F], grad_out [N,O], grad_weight [O,F] row-major fp32; F <= 256, any O
 * (blocks of 32·(256/F) outputs per pass). Scratch: mpgnn_linear_wgrad_workspace_bytes. Replaces autograd's
 * grad_outᵀ @ x of F.linear (a serial-K library GEMM at K = N). */
int32_t mpgnn_linear_wgrad_workspace_bytes(int64_t N, int32_t F, int32_t O, int64_t* bytes);
int32_t mpgnn_linear_wgrad(const float* x, const float* grad_out, int64_t N, int32_t F, int32_t O, float* grad_weight,
                           float* grad_bias, void* workspace, void* stream);

/* Per-epoch scoring of the training loop: replaces mpgnn_validation / mpgnn_test's
 * torch.argmax(pred[idx], 1) + the per-class counts behind f1_score(..., average='macro')
 * (main.py:1084-1115; the reference's scikit-learn call on host lists). For each of n_lists
 * (<= 4) lists l: p_j = argmax over the num_classes scores of row row_idx[l][j] of scores
 * [rows, num_classes] (first maximum, a NaN wins: torch.argmax), y_j = labels[l][j];
 * counts[l][0][c] = #{p_j = c}, counts[l][1][c] = #{y_j = c}, counts[l][2][c] = #{p_j = y_j = c}
 * (int64, [n_lists][3][num_classes]; labels outside [0, num_classes) and rows outside
 * [0, rows) count in no class). row_idx NULL (or row_idx[l] NULL): rows 0..n[l]-1. Host arrays
 * of device pointers; one launch. */
int32_t mpgnn_confusion_counts(const float* scores, int64_t rows, int32_t num_classes, int32_t n_lists,
                               const int64_t* const* row_idx, const int64_t* const* labels, const int64_t* n,
                               int64_t* counts, void* stream);

/* The loops' training loss F.nll_loss(out[train_idx], train_y) (main.py:1065, mean
 * reduction, no class weights) over log-probabilities logp [rows, num_classes]: pairs j with
 * target[j] == ignore_index are skipped; *total_weight = the kept pairs' count (float);
 * *loss = -(Σ_j logp[row_idx[j], target[j]] / *total_weight) (NaN when nothing is kept, or when
 * a kept pair lies outside the matrix). One launch (one workgroup). */
int32_t mpgnn_nll_rows_fwd(const float* logp, int64_t rows, int32_t num_classes, const int64_t* row_idx,
                           const int64_t* target, int64_t n, int64_t ignore_index, float* loss, float* total_weight,
                           void* stream);
/* Its input gradient: grad_logp[row_idx[j], target[j]] += -(*grad_loss / *total_weight) for every
 * kept pair inside the matrix (torch's nll_loss backward value, index_select's backward
 * placement; device scalars). grad_logp [rows, num_classes] must be zeroed by the caller. */
int32_t mpgnn_nll_rows_bwd(const float* grad_loss, const float* total_weight, int64_t rows, int32_t num_classes,
                           const int64_t* row_idx, const int64_t* target, int64_t n, int64_t ignore_index,
                           float* grad_logp, void* stream);
/* The same input gradient written WHOLE (zeros included: no fill launch before it), from the
 * pairs grouped by row — row_perm[row_ptr[i] .. row_ptr[i+1]) = the positions j with
 * row_idx[j] == i, ascending (int32 CSR over the rows, built once per list by the caller) —
 * bit-identical to the zero fill + mpgnn_nll_rows_bwd. */
int32_t mpgnn_nll_rows_bwd_dense(const float* grad_loss, const float* total_weight, int64_t rows, int32_t num_classes,
                                 const int32_t* row_ptr, const int32_t* row_perm, const int64_t* target,
                                 int64_t ignore_index, const float* class_weight, float* grad_logp, void* stream);
/* The class-weighted loss of main_rgcn.py's training step (F.nll_loss(out[train_idx], train_y,
 * weight=class_weight), main_rgcn.py:376-380): each kept pair weighted by class_weight[target]
 * (float [num_classes], device; NULL: 1 — exactly the unweighted calls above), *total_weight =
 * the sum of the kept pairs' weights, *loss = -(Σ w·logp) / *total_weight; the gradient
 * -(w · (*grad_loss / *total_weight)) per pair. mpgnn_nll_rows_bwd_dense takes class_weight too. */
int32_t mpgnn_nll_rows_fwd_weighted(const float* logp, int64_t rows, int32_t num_classes, const int64_t* row_idx,
                                    const int64_t* target, int64_t n, int64_t ignore_index, const float* class_weight,
                                    float* loss, float* total_weight, void* stream);
int32_t mpgnn_nll_rows_bwd_weighted(const float* grad_loss, const float* total_weight, int64_t rows,
                                    int32_t num_classes, const int64_t* row_idx, const int64_t* target, int64_t n,
                                    int64_t ignore_index, const float* class_weight, float* grad_logp, void* stream);

/* Forward and input gradient of the wrappers' Linear heads (Net.lin model.py:147; MPNetm.fc1 /
 * fc2 model.py:224-226), replacing F.linear / grad_out @ weight (host-cheap single launches on the
 * eager epoch's path): out = act(x @ weightᵀ + bias) with x [N,F], weight [O,F], bias [O]
 * (nullable), act MPGNN_ACT_NONE / _RELU; grad_x = grad_out @ weight ([N,O] @ [O,F]).
 * Supported: F = O = 128 (bf16-split matrix-core GEMM, fp32-level accuracy) and O <= 8 (F <= 256
 * for the forward, F % 4 == 0; the forward's dots summed in float64, rounded once); other shapes return MPGNN_ERR_UNSUPPORTED (the caller keeps the
 * library GEMM). Pointers 16-byte aligned. */
int32_t mpgnn_linear_fwd(const float* x, int64_t N, int32_t F, const float* weight, int32_t O, const float* bias,
                         int32_t act, float* out, void* stream);
int32_t mpgnn_linear_dgrad(const float* grad_out, int64_t N, int32_t O, const float* weight, int32_t F, float* grad_x,
                           void* stream);
/* Backward of out = log_softmax(x @ weightᵀ + bias) (mpgnn_linear_fwd with MPGNN_ACT_LOG_SOFTMAX;
 * Net.lin + F.log_softmax, model.py:147-148) from grad_logp and the forward's logp [N,O]:
 * dl = grad_logp - exp(logp) · Σ_o grad_logp[o] per row (log_softmax's backward), grad_x = dl @
 * weight (nullable; relu_in [N,F] nullable: the ReLU backward of the layer that produced x fused,
 * as mpgnn_linear_dgrad_relu_in), grad_weight = dlᵀ x, grad_bias = Σ_i dl (nullable): one pass
 * over the rows + the ordered sum of its per-slice partials (deterministic). O <= 8, F <= 256
 * (else MPGNN_ERR_UNSUPPORTED, nothing launched). Scratch: _workspace_bytes. */
int32_t mpgnn_linear_logsoftmax_bwd_workspace_bytes(int64_t N, int32_t F, int32_t O, int64_t* bytes);
int32_t mpgnn_linear_logsoftmax_bwd(const float* grad_logp, const float* logp, const float* x, int64_t N, int32_t F,
                                    int32_t O, const float* weight, const float* relu_in, float* grad_x,
                                    float* grad_weight, float* grad_bias, void* workspace, void* stream);

/* mpgnn_linear_dgrad with the ReLU backward of the layer that produced the head's input x [N,F]
 * fused (grad_x = x <= 0 ? 0 : grad_out @ weight): Net.lin over the last conv's ReLU output. */
int32_t mpgnn_linear_dgrad_relu_in(const float* grad_out, int64_t N, int32_t O, const float* weight, int32_t F,
                                   const float* x, float* grad_x, void* stream);

/* The loops' optimizer step (Adam(lr=0.01, weight_decay=5e-4), main.py:1119 / main_rgcn.py:454)
 * over n <= 24 fp32 parameter tensors in ONE launch, replacing torch.optim.Adam(fused=True)'s
 * _foreach_add_(steps, 1) + _fused_adam_ pair: for each tensor, step += 1 (float, device
 * scalar), then ATen's fused update (L2 decay folded into the gradient, moments in double rounded
 * to float, bias corrections 1 - beta^step in double; no amsgrad / maximize / grad scaling).
 * Pointers 16-byte aligned (else MPGNN_ERR_UNSUPPORTED, nothing launched); `arrive`: a device
 * int32 the caller zeroes once and keeps for the optimizer (the launch leaves it zero). */
typedef struct mpgnn_adam_tensor {
    float* param;
    const float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    float* step;
    int64_t numel;
} mpgnn_adam_tensor;
int32_t mpgnn_adam_step(const mpgnn_adam_tensor* tensors, int32_t n, double lr, double beta1, double beta2,
                        double weight_decay, double eps, int32_t* arrive, void* stream);

/* Bytes of scratch the fwd/bwd calls need (caller allocates, e.g. torch.empty(uint8)). */
int32_t mpgnn_rgcn_workspace_bytes(const mpgnn_plan* plan, int32_t mode, int64_t relation,
                                   int32_t num_relations, int32_t F_in, int32_t F_out,
                                   int64_t row_lo, int64_t row_hi, int64_t* bytes);
/* Forward-only part of it (enough for mpgnn_rgcn_fwd / mpgnn_rgcn_fwd_act; the backward's
 * gradient partials are not reserved) — inference / no-grad callers at C5 scale save ~50 GB. */
int32_t mpgnn_rgcn_fwd_workspace_bytes(const mpgnn_plan* plan, int32_t mode, int64_t relation,
                                       int32_t num_relations, int32_t F_in, int32_t F_out,
                                       int64_t row_lo, int64_t row_hi, int64_t* bytes);

/* Rows of the h_save buffer of mpgnn_rgcn_fwd / _fwd_act / _bwd for a selection: the
 * MULTI-EDGE segments of the selection (mpgnn_table MPGNN_T_REL_M_PTR range). The means of the
 * single-edge segments are x rows themselves and are not stored (mpgnn_table MPGNN_T_S_SRC). */
int32_t mpgnn_rgcn_hsave_rows(const mpgnn_plan* plan, int32_t mode, int64_t relation,
                              int32_t num_relations, int64_t* rows);

/* Layer forward:  out = Σ_{r} mean_r(x) @ W_r  + x @ root + bias
 *   (mode SINGLE: the single relation `relation`, W = weight [F_in, F_out];
 *    mode ALL: r = 0..num_relations-1, W_r = weight[r] of [R, F_in, F_out]).
 * root / bias may be NULL (root_weight=False / bias=False). out is [N, F_out].
 * h_save (nullable) receives the multi-edge segment means [mpgnn_rgcn_hsave_rows, F_in] for
 * backward (bit-identical to PyG's mean, as mpgnn_rel_mean_fwd); the backward reads the
 * single-edge segments' means from x. */
int32_t mpgnn_rgcn_fwd(const mpgnn_plan* plan, int32_t mode, int64_t relation,
                       int32_t num_relations, const float* x, int32_t F_in,
                       const float* weight, const float* root, const float* bias,
                       int32_t F_out, int64_t row_lo, int64_t row_hi, float* out,
                       float* h_save, void* workspace, void* stream);

enum mpgnn_activation {
    MPGNN_ACT_NONE = 0,
    MPGNN_ACT_RELU = 1,
    MPGNN_ACT_LOG_SOFTMAX = 2 /* mpgnn_linear_fwd with O <= 8 only: log_softmax over each row's O outputs
                                 (Net's lin + F.log_softmax, model.py:147-148, in the head's launch) */
};

/* Layer forward with the caller's activation fused into the combine epilogue:
 *   out = act(Σ_r mean_r(x) @ W_r + x @ root + bias)
 * i.e. `F.relu(conv(x, edge_index, edge_type))` of model.py:144-146 (Net) and the ReLU after
 * each metapath layer of MPNetm (model.py:211,214) in one call. Unsharded plans only (a
 * sharded layer's out is a partial sum: activate after the all-reduce); rows [0, N). */
int32_t mpgnn_rgcn_fwd_act(const mpgnn_plan* plan, int32_t mode, int64_t relation,
                           int32_t num_relations, const float* x, int32_t F_in,
                           const float* weight, const float* root, const float* bias,
                           int32_t F_out, float* out, float* h_save, void* workspace,
                           int32_t act, void* stream);

/* Layer backward given grad_out [N, F_out] and the h_save of the forward (NULL: recomputed).
 * x (the forward's input) is needed for grad_weight (single-edge segment means) and grad_root.
 * Any grad_* pointer may be NULL to skip that gradient.
 *   grad_x      [N, F_in]           (= Σ_r A_rᵀ (grad_out W_rᵀ) + grad_out rootᵀ)
 *   grad_weight [F_in, F_out] or [R, F_in, F_out]
 *   grad_root   [F_in, F_out], grad_bias [F_out]  (rows [row_lo, row_hi) only) */
int32_t mpgnn_rgcn_bwd(const mpgnn_plan* plan, int32_t mode, int64_t relation,
                       int32_t num_relations, const float* x, int32_t F_in,
                       const float* weight, const float* root, int32_t F_out,
                       const float* h_save, const float* grad_out,
                       int64_t row_lo, int64_t row_hi,
                       float* grad_x, float* grad_weight, float* grad_root, float* grad_bias,
                       void* workspace, void* stream);

/* mpgnn_rgcn_bwd with the parameter gradients ACCUMULATED: grad_weight / grad_root / grad_bias
 * (all three required) receive dst + this call's gradient, computed exactly as mpgnn_rgcn_bwd's
 * and added once per element (the value autograd's gradient accumulation of a parameter used
 * twice produces: Net applies the same conv2 for layers 1..L-1, model.py:144-146). grad_x is
 * written as by mpgnn_rgcn_bwd. Mode ALL, F_in = F_out = 128 on the bf16-split path only;
 * MPGNN_ERR_UNSUPPORTED otherwise, with nothing launched. */
int32_t mpgnn_rgcn_bwd_accumulate(const mpgnn_plan* plan, int32_t mode, int64_t relation,
                                  int32_t num_relations, const float* x, int32_t F_in,
                                  const float* weight, const float* root, int32_t F_out,
                                  const float* h_save, const float* grad_out,
                                  int64_t row_lo, int64_t row_hi,
                                  float* grad_x, float* grad_weight, float* grad_root, float* grad_bias,
                                  void* workspace, void* stream);

/* mpgnn_rgcn_bwd (accumulate = 0) / mpgnn_rgcn_bwd_accumulate (1) for a layer whose input x is
 * the ReLU output of the previous layer (Net, model.py:144-146: F.relu(conv(...)) feeding the
 * next conv): grad_x is written with that ReLU's backward fused — grad_x[i] = x[i] <= 0 ? 0 :
 * (the gradient w.r.t. x)[i] (threshold_backward's rule) — i.e. the gradient w.r.t. the previous
 * layer's pre-activation output, so that layer's own ReLU backward launch is skipped. Used by
 * Net's forward for its internal activations only (no caller sees the masked gradient). */
int32_t mpgnn_rgcn_bwd_relu_in(const mpgnn_plan* plan, int32_t mode, int64_t relation,
                               int32_t num_relations, const float* x, int32_t F_in,
                               const float* weight, const float* root, int32_t F_out,
                               const float* h_save, const float* grad_out,
                               int64_t row_lo, int64_t row_hi,
                               float* grad_x, float* grad_weight, float* grad_root, float* grad_bias,
                               void* workspace, void* stream, int32_t accumulate);

/* --- score function --------------------------------------------------------
 * The metapath-candidate score of the reference, OutputLayer.forward non-bag branch
 * (model.py:74-89) as trained by train() / score_relation_parallel (main.py:641-673, 727-760).
 * The edge dictionary of one relation (create_edge_dictionary, main.py:387-424) is a CSR in
 * dictionary order: source keys[k] (int32 node ids, k = 0..num_keys-1, mask order), its
 * destinations dst[key_ptr[k] .. key_ptr[k+1]) in edge-file order (every key has >= 1).
 * All pointers are DEVICE pointers; weights / max_weights / grad_* are fp32 [num_nodes].
 *
 * mpgnn_score_argmax: max_weights = 0, then for every key k: arg_pos[k] = the position p of the
 * FIRST maximum of weights[dst[p]] (torch.argmax: NaN counts as the maximum), max_node[k] =
 * dst[arg_pos[k]], max_weights[keys[k]] = weights[max_node[k]] (bit-identical to model.py:85-87).
 * Replaces the per-source Python loop of model.py:82-87. */
int32_t mpgnn_score_argmax(const float* weights, int64_t num_nodes, const int32_t* keys, const int32_t* key_ptr,
                           const int32_t* dst, int64_t num_keys, float* max_weights, int32_t* arg_pos,
                           int32_t* max_node, void* stream);
/* Backward of mpgnn_score_argmax (autograd of model.py:87 `max_weights[source] = weights[max_node]`):
 * grad_weights[n] = Σ grad_max[keys[k]] over the keys whose argmax edge points at n, added in
 * DESCENDING k (the order autograd unwinds the reference's CopySlices chain), 0 where none.
 * (in_ptr [num_nodes+1], in_pos, in_key) list, per destination node n, every (edge position p,
 * key k) of the dictionary with dst[p] == n, sorted by k descending — built once per dictionary. */
int32_t mpgnn_score_argmax_bwd(const float* grad_max, int64_t num_nodes, const int32_t* keys, const int32_t* arg_pos,
                               const int32_t* in_ptr, const int32_t* in_pos, const int32_t* in_key,
                               float* grad_weights, void* stream);

/* Bag branch of the score (OutputLayer.forward with BAGS=True, model.py:45-72; trained by
 * train(BAGS=True) / score_relation_bags_parallel, main.py:641-673, 853-917; replaces the
 * per-bag, per-source Python loop). Bags are a CSR over their member source nodes: bag i holds
 * mem_node[bag_ptr[i] .. bag_ptr[i+1]) in bag order, mem_key[m] = the dictionary key index of
 * member m (-1 if it is no key: skipped, model.py:59). feat is fp32 [num_nodes, feat_dim]
 * (data.x), lin_weight fp32 [feat_dim] (LinearLayerAttri.weight[0]).
 * mpgnn_score_bag_argmax, per bag in member order: s_m = Σ_j feat[node][j]·lin[j] (feature
 * order, no FMA contraction), mem_pos[m] = the position p of the FIRST maximum of
 * weights[dst[p]]·s_m (torch.argmax), mem_max[m] = dst[p], mem_v[m] = weights[mem_max[m]]·s_m;
 * the bag's pick is the first member whose v is strictly larger than the running maximum
 * (starting at -10): bag_mem[i] = that member (-1: none), max_weights[i] = its v (0: none),
 * bag_w[i] = weights[its max node]. Members that are no key leave their mem_* entries unwritten. */
int32_t mpgnn_score_bag_argmax(const float* weights, const float* feat, int32_t feat_dim, const float* lin_weight,
                               const int32_t* bag_ptr, const int32_t* mem_node, const int32_t* mem_key,
                               int64_t num_bags, const int32_t* key_ptr, const int32_t* dst, float* max_weights,
                               int32_t* bag_mem, float* bag_w, float* mem_s, float* mem_v, int32_t* mem_pos,
                               int32_t* mem_max, void* stream);
/* Backward of mpgnn_score_bag_argmax (autograd of model.py:64,70): grad_weights[n] = Σ
 * grad_max[i]·s_{pick(i)} over the bags whose pick points at n, added in DESCENDING bag order
 * (0 where none); grad_lin[j] = Σ_{bags i with a pick, descending} feat[node_i][j]·(grad_max[i]·
 * bag_w[i]). (in_ptr [num_nodes+1], in_bag, in_mem, in_pos): per destination node n, every (bag,
 * member, edge position) candidate with dst[position] == n, bags descending — built once per
 * (bags, dictionary). grad_lin may be NULL (not wanted). */
int32_t mpgnn_score_bag_argmax_bwd(const float* grad_max, int64_t num_bags, const int32_t* bag_mem,
                                   const float* bag_w, const int32_t* mem_node, const float* mem_s,
                                   const int32_t* mem_pos, const float* feat, int32_t feat_dim,
                                   int64_t num_nodes, const int32_t* in_ptr, const int32_t* in_bag,
                                   const int32_t* in_mem, const int32_t* in_pos, float* grad_weights,
                                   float* grad_lin, void* stream);

/* Every candidate relation of one scoring round at once (main.py:1309-1330 runs
 * score_relation_parallel per relation, 100 epochs each, split over MPI ranks). The relations'
 * dictionaries form ONE relation-major CSR: key k = (relation key_rel[k] in [0, R), source keys[k]),
 * destinations dst[key_ptr[k] .. key_ptr[k+1]) in edge order; weights are row-major [R, num_nodes].
 * mpgnn_score_argmax_multi, per key: arg_pos / max_node as mpgnn_score_argmax over row key_rel[k],
 * values[k] = weights[key_rel[k]][max_node[k]] (the prediction of source keys[k]),
 * grad_values[k] = alpha[key_rel[k]] · (values[k] − labels[keys[k]]) — torch's mse_loss_backward
 * with alpha_r = fp32(2 / K_r) and grad_output 1 — and sq_err[k] = (values[k] − labels[keys[k]])².
 * mpgnn_score_loss_multi: loss[r] = Σ sq_err over r's keys rel_key_ptr[r] .. rel_key_ptr[r+1] / K_r
 * (fixed lane-strided order: torch's mean to fp32 rounding). mpgnn_score_argmax_multi_bwd:
 * grad_weights[0 .. grad_size) = 0, then for every (relation, destination) pair i the ordered sum
 * (keys DESCENDING) of grad_values of the keys whose argmax edge is one of the pair's candidates
 * (in_pos / in_key over pair_ptr[i] .. pair_ptr[i+1]) goes to grad_weights[pair_target[i]]. */
int32_t mpgnn_score_argmax_multi(const float* weights, int64_t num_nodes, const int32_t* keys, const int32_t* key_ptr,
                                 const int32_t* dst, const int32_t* key_rel, int64_t num_keys, const float* labels,
                                 const float* alpha, int32_t* arg_pos, int32_t* max_node, float* values,
                                 float* grad_values, float* sq_err, void* stream);
int32_t mpgnn_score_loss_multi(const float* sq_err, const int32_t* rel_key_ptr, int64_t num_rel, float* loss,
                               void* stream);
int32_t mpgnn_score_argmax_multi_bwd(const float* grad_values, const int32_t* arg_pos, const int32_t* pair_ptr,
                                     const int64_t* pair_target, const int32_t* in_pos, const int32_t* in_key,
                                     int64_t num_pairs, int64_t grad_size, float* grad_weights, void* stream);

/* --- options ----------------------------------------------------------------------------
 * MPGNN_OPT_EXACT_ORDER = 1: every gather-sum adds its entries strictly in the reference's
 * sequential order (no ordered-piece split of long runs). Default 0: runs longer than 32
 * entries are summed as ordered 32-entry partial sums (deterministic, bounded serial work per
 * wave); runs of <= 32 entries — the forward segment means of almost every segment — are
 * bit-identical to the reference either way. mpgnn_rel_mean_fwd is always exact. */
enum mpgnn_option {
    MPGNN_OPT_EXACT_ORDER = 0,
    MPGNN_OPT_TIMING_MASK = 3,   /* kernel kinds timed while timing is enabled (bit k = kind k); default all */
    MPGNN_OPT_REL_GEMM = 5,      /* 1 (default): B-stationary GEMM (weights in registers) for F_in, F_out in
                                    {64,128} x {128}; 0: the tile GEMM (the width fallback) */
    MPGNN_OPT_PLAN_THREADS = 11, /* host threads of mpgnn_plan_create: 0 (default) = hardware concurrency capped
                                    at 16; the tables do not depend on it */
    MPGNN_OPT_REL_WIDE = 19,     /* 1 (default): the B-stationary GEMM also takes F_in = F_out = 256 (two 128-column
                                    blocks); 0: tile_gemm_kernel there */
    MPGNN_OPT_CHUNK_ROWS = 20,   /* backward weight-gradient reduction chunks: base length in rows (multiple of 32,
                                    32..1024, default 256) of the root chunks and of the relation chunks of plans
                                    created afterwards; same results up to fp32 summation order of the slabs */
    MPGNN_OPT_GEMM_BF3 = 24,     /* 1 (default): the transform / dgrad GEMMs (K in {64,128}, N = 128) on the bf16
                                    matrix cores with each fp32 operand split exactly into three bf16 pieces (six
                                    products, fp32 accumulation: fp32-level accuracy at 2.67x the fp32-MFMA rate);
                                    0: the fp32-MFMA kernel (v_mfma_f32_32x32x2_f32) */
    MPGNN_OPT_BWD_FUSED = 25,    /* 1 (default): mpgnn_rgcn_bwd at F_in = F_out = 128 (bf16-split GEMMs) runs
                                    dgrad and dW / droot / dbias in one launch that gathers dout once;
                                    0: the dgrad launch + the chunked dW launch */
    MPGNN_OPT_FLAT_WG_PER_CU = 26, /* gather-sum lists (means, combine, grad_x): 0 = one workgroup per list group;
                                    k > 0 = a persistent grid of k workgroups per CU walking the groups */
    MPGNN_OPT_FLAT_FUSE_SPLIT = 27, /* 1 (default): grad_x rows split over more than 16 chunks (hub nodes) are
                                    finished inside the gather-sum launch by the wave adding their last
                                    piece (same sums, same order); 0: finalize_rows_kernel after it */
    MPGNN_OPT_OUTER_VEC = 28,    /* 1 (default): the bf16-split weight-gradient kernel gathers rows 16 B per lane
                                    and reads its column fragments with transposed LDS reads
                                    (outer_bf3v_kernel); 0: 4-B column gathers (outer_bf3_kernel) */
    MPGNN_OPT_GEMM_SWITCH_COST = 29 /* the bf16-split GEMM's workgroup item ranges (K = 64, 128): 0 = equal item
                                    counts; c > 0 = ranges balanced by items + (c / 100) per weight run, each
                                    run paying an exposed weight-slice load (default 150: the round-6 re-sweep
                                    with the prologue records, C3 forward 43.1-43.3 us at 120-150 against
                                    44.0-44.4 at 250, 45.7 at 400; round 5 chose 250; outputs bit-identical) */,
    MPGNN_OPT_GEMM_IL = 30       /* 1 (default): the bf16-split GEMM (K = 64, 128) commits the next item's tile in
                                    parts scheduled among the MFMAs of the current item's k-steps; 0: the
                                    round-4 skeleton (whole tile in one k-step); outputs bit-identical */,
    MPGNN_OPT_GEMM_CU_PAIRS = 31 /* 1 (default): the bf16-split GEMM's item ranges are balanced per CU (the two
                                    workgroups a CU runs take the halves of one CU range); 0: per workgroup;
                                    outputs bit-identical */,
    MPGNN_OPT_OUTER_SQ = 32      /* 1: the bf16-split weight gradient (F = 128, and the quadrants at 256) gives each
                                    wave a 64 x 64 quarter of the slab and schedules the next slice's commit among
                                    the MFMAs; 0 (default, measured faster at C3: 65.7 vs 68.0 us): 128 x 32
                                    strips; slabs bit-identical */,
    MPGNN_OPT_OUTER_RANGES = 33  /* 1 (default): that kernel's workgroups take contiguous chunk ranges balanced by
                                    16-row slices (per CU); 0: every G-th chunk; slabs bit-identical */,
    MPGNN_OPT_GEMM_W_IL = 34     /* the K = 256 bf16-split GEMM (F_in = F_out = 256, C5): 1 (default) commits the
                                    next item's tile in four parts among the k-steps' MFMAs (as GEMM_IL at
                                    K = 128; round-5 A/B at C5: forward 26.2 -> 23.9 ms, dgrad 25.6 -> 23.2 ms,
                                    mode SINGLE 2.31 -> 1.87 ms per layer); 0: the whole tile in one k-step;
                                    outputs bit-identical */,
    MPGNN_OPT_GEMM_W1 = 35       /* the bf16-split GEMM at K = N = 128 (transform and dgrad): 1 runs
                                    rel_gemm_w1_kernel (one workgroup per CU, one wave per SIMD, 64-row items,
                                    the next relation's weight slice prefetched into a second register set);
                                    0 rel_gemm_bf3_kernel (two workgroups per CU, 32-row items); outputs
                                    bit-identical */,
    MPGNN_OPT_OUTER_VARIANT = 36 /* the bf16-split weight gradient (outer_bf3v_kernel_t) slice pipeline: 0 (default)
                                    the next-next slice's rows issued before this slice's MFMAs; 1 its row
                                    indices by scalar loads; 2 its rows issued after this slice's MFMAs; slabs
                                    bit-identical */,
    MPGNN_OPT_FLAT_U = 37,       /* gather-sum lists (means, combine, grad_x): rows in flight per wave, 16
                                    (default), 8 or 32; sums bit-identical */
    MPGNN_OPT_FLAT_PAD = 38      /* forward gather-sum lists (means, combine): 1 (default) fetches a normal
                                    group's chunk (descriptor, positions' values and rows) from per-slot padded
                                    tables built once per plan and list, in one round of vector loads (C3:
                                    means 18.5 -> 17.6 µs, combine 24.9 -> 24.2 µs); 0 the scalar chunk-range
                                    hops; sums bit-identical */,
    MPGNN_OPT_SINGLE_FOLD = 39   /* the fused mode-SINGLE layer (single_bf3_kernel, F_in in {64, 128}, F_out =
                                    128): 1 computes the relation's multi-edge segment means inside the GEMM
                                    launch (the means kernel's arithmetic: 32-edge pieces in order) instead of a
                                    separate means launch; 0 the two launches; outputs and saved means
                                    bit-identical */,
    MPGNN_OPT_BWD_SIDE_REDUCE = 41 /* mpgnn_rgcn_bwd (not accumulating): 1 runs the weight gradient's outer
                                    products first, then its ordered slab sum on a library side stream beside the
                                    dgrad GEMM and grad_x, joined before the call returns; 0 (default) all in
                                    stream order; gradients bit-identical */,
    MPGNN_OPT_GEMM_FIRST = 42    /* the bf16-split GEMM at K = 128, mode ALL: 1 (default) reads each workgroup's
                                    range and its first three items' gathered row numbers from a per-range record
                                    built once per plan (one round trip, not range -> tiles -> row-index hops; C3
                                    forward GEMM 45.1-45.2 -> 44.75-44.9 us, alternated 3x); 0 the hops; outputs
                                    bit-identical */,
    MPGNN_OPT_ADAM_CONTRACT = 40 /* process-wide: mpgnn_adam_step's double multiply-adds fused (1, default: the
                                    contraction clang's default HIP flags give ATen's kernel) or each product
                                    rounded (0); pinned bit-for-bit against torch by the GPU tests */
    /* ids 1, 2, 4, 6-10, 12-18, 21-23: round-1 profiling switches and measured-slower kernel variants,
       withdrawn in round 2; mpgnn_set_option refuses them with MPGNN_ERR_ARG */
};
/* Process defaults. The kernel switches (every option except TIMING_MASK, PLAN_THREADS,
 * CHUNK_ROWS and ADAM_CONTRACT) are PER PLAN: a plan copies the defaults when it is created and is changed only by
 * mpgnn_plan_set_option, so no launch reads process-wide state; mpgnn_set_option of a switch
 * therefore affects plans created afterwards. TIMING_MASK (profiling) and PLAN_THREADS /
 * CHUNK_ROWS (plan build parameters, read when a plan is built) stay process-wide. */
int32_t mpgnn_set_option(int32_t option, int64_t value);
/* Current default value of an option (tests save and restore the shipped defaults around overrides). */
int32_t mpgnn_get_option(int32_t option, int64_t* value);
/* One plan's kernel switch (MPGNN_ERR_ARG for the process-wide options). Not synchronised with
 * launches on other threads that use the same plan: set switches before using the plan. */
int32_t mpgnn_plan_set_option(mpgnn_plan* plan, int32_t option, int64_t value);
int32_t mpgnn_plan_get_option(const mpgnn_plan* plan, int32_t option, int64_t* value);

/* --- graph file reader --------------------------------------------------------------
 * link.dat (`node_1 \t relation \t node_2`, one edge per line) → the tensors of
 * get_edge_index_and_type_no_reverse (main.py:366-372 ≡ main_rgcn.py:357-363), replacing the
 * pandas.read_csv + Python-list conversion of main.py:150-151,369-371. Host only (no GPU).
 * mpgnn_links_count: number of non-blank lines. mpgnn_links_parse: fills edge_index
 * (int64 [2, rows], row 0 = node_1, row 1 = node_2) and edge_type (int64 [rows]) in file
 * order; MPGNN_ERR_ARG if the file does not hold exactly `rows` three-integer lines. */
int32_t mpgnn_links_count(const char* path, int64_t* rows);
int32_t mpgnn_links_parse(const char* path, int64_t* edge_index, int64_t* edge_type, int64_t rows);
/* node.dat / label.dat (`id \t value …` numeric rows; the reference reads them with
 * pandas.read_csv(sep='\t', header=None), main.py:140-147,176-182): mpgnn_tsv_shape returns the
 * non-blank line count and the widest row's field count; mpgnn_tsv_parse_f64 fills a row-major
 * float64 [rows, cols] matrix in file order, shorter rows padded with NaN (read_csv's fill);
 * MPGNN_ERR_ARG on a non-numeric field, a row wider than cols or a row-count mismatch. */
int32_t mpgnn_tsv_shape(const char* path, int64_t* rows, int64_t* cols);
int32_t mpgnn_tsv_parse_f64(const char* path, double* out, int64_t rows, int64_t cols);

/* --- kernel timing (bench / profiling) ----------------------------------------------
 * When enabled, every kernel launch of the entry points above is bracketed by a pair of
 * hipEvents recorded on the launch stream; mpgnn_timing_query synchronises those events and
 * returns the summed duration and the launch count of one kernel kind. */
enum mpgnn_kernel_kind {
    MPGNN_K_SEG_FWD = 0,   /* tile_gemm_kernel: Y = H @ W_r, Y_root = x @ root (forward)   */
    MPGNN_K_ROW_FWD = 1,   /* combine Σ_r Y + Y_root + bias (flat_rows / row_sum kernels)  */
    MPGNN_K_SEG_DGRAD = 2, /* tile_gemm_kernel: (dout @ W_rᵀ) / cnt, dout @ rootᵀ          */
    MPGNN_K_ROW_DX = 3,    /* grad_x transposed gather-sum + G_root (flat_rows / row_sum)  */
    MPGNN_K_OUTER = 4,     /* outer_accum_kernel: dW / droot / dbias                      */
    MPGNN_K_REDUCE = 5,    /* reduce_slabs_kernel                                         */
    MPGNN_K_MEAN = 6,      /* segment means H (flat_rows / row_sum kernels)               */
    MPGNN_K_PIECE = 7,     /* ordered partial sums of long runs (exact-order lists)       */
    MPGNN_K_FINAL = 8,     /* finalize_rows_kernel: split / empty rows, extra + bias      */
    MPGNN_K_COUNT = 9
};
int32_t mpgnn_timing_enable(int32_t on);
/* Debug: workgroups per CU the runtime admits at width F for the gather-tile kernel
 * (seg_tile_kernel) and the persistent tile GEMM (tile_gemm_kernel), and the grid the
 * latter is launched with. */
int32_t mpgnn_debug_occupancy(int32_t F, int32_t* seg_tile_blocks_per_cu, int32_t* tile_gemm_blocks_per_cu,
                              int32_t* tile_gemm_grid);
int32_t mpgnn_timing_reset(void);
int32_t mpgnn_timing_query(int32_t kernel_kind, double* total_ms, int64_t* launches);

#ifdef __cplusplus
}
#endif

#endif /* MPGNN_RGCN_H */
