/*
 * admm_tomo.h -- C-ABI of the MI355X-native decentralized-ADMM tomography hot path.
 *
 * The reference (prsinha1/Distributed-Inverse-Problem-Admm) is pure Python and
 * has no FFI.  Its hot-path boundary is two duck-typed Python functions:
 *
 *   build_node_problem(Ai, bi, rho, neighbor_terms, N, lam_tv, Qij_terms)
 *       -> /root/reference/block_5_node_problem.py:6-32
 *   decentralized_admm(A_dense_list, sinograms, G, Wi_list, Qij_diag_fn, N, ...)
 *       -> /root/reference/block_6_admm_loop_ver2.py:15-326
 *          (kwarg surface also of block_6_admm_loop.py:72-84)
 *
 * plus the operator they consume, the ODL ray transform materialised as a dense
 * matrix (block_2_load_odl_data.py:16-96), used only through `A @ x`,
 * `A.T @ r` and column norms (block_6_admm_loop_ver2.py:145,193;
 * block_3_graph_and_precisions.py:20-23).  The Python drop-ins in
 * distributed-inverse-problem-admm_amd/ call the entry points below through
 * ctypes.  Each entry point names the reference code it replaces.
 *
 * Conventions
 *   - All array arguments are DEVICE pointers owned by the caller (PyTorch
 *     tensors).  The context owns only geometry tables and scratch.
 *   - Image layout: node-major, C-order pixels, x[v*N*N + i*N + j] <-> pixel
 *     (x_i, y_j) of ODL's uniform_discr([-1,-1],[1,1],[N,N]) (axis 0 = x).
 *   - Sinogram layout: node-major, angle-major: b[v*A*D + t*D + k]
 *     (block_6_admm_loop_ver2.py:46 flattens the (angles, det) sinogram in C order).
 *   - "sample" arrays (images given to the projector, sinograms) have the
 *     context dtype (ADMM_DTYPE_F32 or ADMM_DTYPE_F64); solver state
 *     (x, d, e, y, z, q, A^T b, sum q) is always float64.
 *   - Every call is stream-ordered and asynchronous on `stream` (a hipStream_t;
 *     NULL = default stream); nothing synchronises the host except
 *     admm_ctx_create / admm_ctx_destroy / admm_batch_bind.
 *   - Return 0 on success; a negative code on failure, with a message
 *     available from admm_last_error() (thread-local).
 *   - One context per device, used from one host thread.
 */
#ifndef ADMM_TOMO_H
#define ADMM_TOMO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ADMM_ABI_VERSION 9

#define ADMM_OK 0
#define ADMM_E_INVALID (-1)
#define ADMM_E_HIP (-2)
#define ADMM_E_STATE (-3)

#define ADMM_DTYPE_F32 0
#define ADMM_DTYPE_F64 1

#define ADMM_TV_ISO 0
#define ADMM_TV_ANISO 1

/* edge fusion (admm_batch.fusion) */
#define ADMM_FUSE_MIDPOINT 0 /* z = (a_i + a_j)/2   (block_6_admm_loop_ver2.py:220-223, as run) */
#define ADMM_FUSE_WEIGHTED 1 /* z = (W_i a_i + W_j a_j)/(W_i + W_j)  (commented at _ver2:221-222;
                                ADMM_Algo.pdf eq.(2)); keeps both endpoint duals */

/* admm_batch.flags: x_ext's local rows are written only by admm_node_update (the caller
 * never changes x between updates), so an update may start from the previous update's
 * diagnostics instead of projecting x again. */
#define ADMM_BATCH_KEEP_X 1

/* per-node statistics written by admm_node_update (float64) */
#define ADMM_NODE_STAT_MSE_SINO 0 /* ||A x - b||^2           (block_6_admm_loop_ver2.py:190-194) */
#define ADMM_NODE_STAT_G2 1       /* ||g||^2 stationarity    (block_6_admm_loop_ver2.py:145-149) */
#define ADMM_NODE_STAT_TV 2       /* TV(x)                   (block_4_tv_helpers.py:5-14) */
#define ADMM_NODE_STAT_QUAD 3     /* sum_j rho/2 ||x-v_ij||^2_Q (block_5_node_problem.py:26-29) */
#define ADMM_NODE_STAT_IMG 4      /* ||x - phantom||^2       (block_6_admm_loop_ver2.py:199-204) */
#define ADMM_NODE_STAT_SBRES2 5   /* ||A^T(Ax-b) + rho(D x - c) + mu K^T e||^2: stationarity of eq.(1)
                                     with the split-Bregman dual p = mu e / lam (ABI 3) */
#define ADMM_NODE_STATS 6

/* per-edge statistics written by admm_consensus (float64) */
#define ADMM_EDGE_STAT_RA2 0 /* ||x_a - z||^2 */
#define ADMM_EDGE_STAT_RB2 1 /* ||x_b - z||^2 */
#define ADMM_EDGE_STAT_DZ2 2 /* ||z_new - z_old||^2 */
#define ADMM_EDGE_STATS 3

/* Parallel-beam geometry of one graph node.  Replaces the ODL construction of
 * block_2_load_odl_data.py:16-65: space [-1,1]^2 (N x N), angles
 * uniform_partition(angle_min, angle_max, n_angles) midpoints, detector
 * uniform_partition(det_min, det_max, n_det) midpoints.  All nodes share it. */
typedef struct admm_geom {
    int32_t N;
    int32_t n_angles;
    int32_t n_det;
    int32_t reserved;
    double angle_min, angle_max;
    double det_min, det_max;
} admm_geom;

typedef struct admm_ctx admm_ctx;

/* The batch of graph nodes this device updates, their incident edges and the
 * solver parameters.  All pointers are device pointers. */
typedef struct admm_batch {
    int32_t V;        /* local graph nodes (rows 0..V-1 of x_ext) */
    int32_t n_xext;   /* rows of x_ext: local nodes + halo (neighbour) nodes */
    int32_t n_edges;  /* edge slots stored on this device */
    int32_t tv_iters; /* split-Bregman rounds per x-update (T_tv) */
    int32_t cg_iters; /* CG steps per round (K_cg) */
    int32_t tv_kind;  /* ADMM_TV_ISO / ADMM_TV_ANISO */
    double rho, lam, mu;

    double* x_ext;        /* [n_xext][n]  node images; rows < V updated in place   */
    double* d;            /* [V][2][n]    split variable d ~ Kx (warm state)        */
    double* e;            /* [V][2][n]    Bregman variable (warm state)             */
    const double* atb;    /* [V][n]       A^T b                                     */
    const double* dsum;   /* [V][n]       D_i = sum_j q_ij (setup data: also packed into the
                           * CG operator's sample layout at admm_batch_bind -- rebind
                           * after changing it)                                     */
    const void* b;        /* [V][m]       sinograms (context dtype)                 */
    const double* phantom;/* [n] or NULL  for ||x - phantom||^2                     */

    double* y;            /* [E][n] dual of the lower-numbered endpoint (y_ij,min)  */
    double* z;            /* [E][n] consensus z_ij; NULL (ABI 7, midpoint fusion): derived
                           * from x_prev below instead of stored                       */
    const double* q;      /* [Qslots][n] precision vectors                         */
    const int32_t* edge_a;    /* [E] x_ext row of the lower endpoint               */
    const int32_t* edge_b;    /* [E] x_ext row of the higher endpoint              */
    const int32_t* inc_off;   /* [V+1] CSR over local nodes of incident edge-ends  */
    const int32_t* inc_edge;  /* [nnz] edge slot                                   */
    const int32_t* inc_qslot; /* [nnz] q slot of q_ij seen from this node           */
    const int32_t* inc_sign;  /* [nnz] +1 if this node is the lower endpoint, else -1 */

    double* node_stats;   /* [V][ADMM_NODE_STATS] */
    double* edge_stats;   /* [E][ADMM_EDGE_STATS] */

    /* ABI 2: edge fusion.  MIDPOINT keeps the single-y form (y_ij,max = -y);
     * WEIGHTED needs y_b and w (both NULL for MIDPOINT). */
    int32_t fusion;       /* ADMM_FUSE_* */
    int32_t flags;        /* ADMM_BATCH_* (0 in ABI-2 callers that predate it: was reserved) */
    double* y_b;          /* [E][n] dual of the higher-numbered endpoint (y_ij,max)   */
    const double* w;      /* [n_xext][n] W of the node in each x_ext row (W_i, make_precisions) */

    /* ABI 7: derived consensus (midpoint fusion, z == NULL).  z_ij is never stored: by the
     * single-y invariant it is the midpoint of the two endpoint images of the last consensus
     * (block_6_admm_loop_ver2.py:210-223 with y_ij,i + y_ij,j = 0), so the library keeps
     * those images instead -- one row per x_ext row, not one per edge -- and forms
     * z_ij = (x_prev[a] + x_prev[b]) / 2 wherever z is read (neighbour gather, diagnostics,
     * the dual residual); admm_consensus sets x_prev = x_ext after its edge updates.
     * Zero-filled by the caller before the first iteration (z = 0, block_6_..._ver2.py:42). */
    double* x_prev;       /* [n_xext][n] or NULL (stored z)                            */
} admm_batch;

int admm_abi_version(void);
const char* admm_last_error(void);

/* Context: geometry tables + scratch.  dtype = ADMM_DTYPE_*.  max_images bounds
 * the batch size of the operator entry points below. */
int admm_ctx_create(admm_ctx** out, const admm_geom* geom, int dtype, int max_images, int device);
/* ABI 4: a context for an operator given as an explicit matrix instead of a geometry:
 * the reference's A_dense_list entries (block_2_load_odl_data.py:68-96 `_to_dense_matrix`,
 * loaded back at block_7_main.py:16-22 / block_3_graph_and_precisions.py:283-287).
 * HOST arrays: A (m x N*N, rows = sinogram entries in the layout above, columns = C-order
 * pixels) as CSR -- indptr[m + 1] (int64), indices[nnz] (int32), values[nnz] (float64,
 * rounded to the context dtype).  The library keeps A and A^T as device CSR; every entry
 * point below (operator, batch, consensus) works unchanged, with the projector replaced
 * by CSR products.  nnz < 2^31. */
int admm_ctx_create_matrix(admm_ctx** out, int N, int m, long long nnz, const long long* indptr,
                           const int* indices, const double* values, int dtype, int max_images, int device);
int admm_ctx_destroy(admm_ctx* ctx);

/* --- operator entry points (replace ODL RayTransform / dense A) ---------- */

/* sino[v] = A img[v] for v < nimg.  Replaces `Ai @ x`
 * (block_5_node_problem.py:21, block_6_admm_loop_ver2.py:193). */
int admm_project_fwd(admm_ctx* ctx, const void* img, void* sino, int nimg, void* stream);
/* img[v] = A^T sino[v].  Replaces `Ai.T @ r` (block_6_admm_loop_ver2.py:145). */
int admm_project_adj(admm_ctx* ctx, const void* sino, void* img, int nimg, void* stream);
/* W[p] = max(sum_r A[r,p]^2, 1e-12) (float64).  Replaces make_precisions'
 * column sums (block_3_graph_and_precisions.py:20-23, block_1_env_and_imports.py:16-18). */
int admm_column_norms_sq(admm_ctx* ctx, double* W, void* stream);
/* (gx, gy) = K x, forward differences (block_4_tv_helpers.py:17-23), float64. */
int admm_tv_grad(admm_ctx* ctx, const double* x, double* gx, double* gy, int nimg, void* stream);
/* out = K^T (px, py), exact adjoint of admm_tv_grad (block_4_tv_helpers.py:25-35). */
int admm_tv_div(admm_ctx* ctx, const double* px, const double* py, double* out, int nimg,
                void* stream);

/* --- node batch (replaces the node loop + CVXPY/SCS solve and the edge updates) --- */

/* Bind a batch (pointers are captured; the contents may change between calls).
 * Allocates scratch and records the update sequence as a hipGraph.  Synchronous. */
int admm_batch_bind(admm_ctx* ctx, const admm_batch* batch);
/* A^T b for the bound batch (setup; writes batch->atb, which is then const). */
int admm_batch_atb(admm_ctx* ctx, double* atb_out, void* stream);
/* One x-update of every bound node: neighbour gather v_ij = z_ij - y_ij,i
 * (y_ij,i = y for the lower endpoint, -y or y_b for the higher one),
 * fixed-count split-Bregman/CG solve of eq.(1), diagnostics into node_stats.
 * Replaces block_6_admm_loop_ver2.py:81-197 (build_node_problem + SCS + g check). */
int admm_node_update(admm_ctx* ctx, void* stream);
/* admm_node_update with `tv_iters` split-Bregman rounds instead of the bound count
 * (warm-started from the current x, d, e: k calls of r rounds continue one solve of
 * k*r rounds up to rounding).  The chunked solves of block_6_admm_loop.py:14-69
 * (_scs_solve_in_chunks) use it between snapshots.  ABI 3. */
int admm_node_update_rounds(admm_ctx* ctx, int tv_iters, void* stream);
/* Edge updates z = (a_i + a_j)/2 (or the W-weighted mean, ADMM_FUSE_WEIGHTED),
 * y += x - z at both ends, and the residual partial sums
 * into edge_stats.  Replaces block_6_admm_loop_ver2.py:210-253.  Every edge
 * slot of the batch is processed; x_ext halo rows must be current. */
int admm_consensus(admm_ctx* ctx, void* stream);
/* Average duration (ms) of a launch of the forward projector's tap kernel (k_fwdg,
 * which makes every sample tap; its segment partial sums are not combined) on the
 * bound batch, timed with HIP events on `stream`.
 * in_solve = 0: `reps` back-to-back launches on the batch's current x (the image
 *   rows stay in L2 from one launch to the next).
 * in_solve = 1 (ABI 5): one x-update of the bound batch is enqueued directly (the
 *   launch sequence its graph replays) with events around each CG step's forward
 *   tap launch -- right after the CG / TV update that wrote p and p^T, as in every
 *   solve; the batch's state advances by that x-update.  `reps` is ignored.
 * Measurement helper for bench.py; synchronises. */
int admm_time_forward(admm_ctx* ctx, int reps, int in_solve, void* stream, double* ms_out);
/* ABI 6: the grouped forward projector's plan `plan` (0: 64-ray chunks, 1: chunks aligned
 * per (row segment, angle) at the detector centre, 2: chunks aligned per (row segment,
 * chunk); 3-5: plans 0-2 with each block's rays clipped to those crossing its row segment
 * inside the image) for this context's geometry: angle groups, blocks per node chunk, touched row
 * pixels staged per node chunk (the host planner's model), and active = 1 if it is the plan
 * the bound batch (or, before a bind, the context) uses.  groups = 0: no such plan.
 * No device work.  (Tests and tuning; the plans give bitwise-identical projections.) */
int admm_fwd_plan_info(admm_ctx* ctx, int plan, int* groups, int* blocks, double* staged, int* active);
/* ABI 8: how the bound batch projects: vb = node-interleave width of its sample buffers;
 * mirror = 1 if the projectors run in mirror mode (angles (t + 1/2) pi / a over [0, pi), a even,
 * symmetric detector: angle a-1-t projects I as angle t projects flipud(I), so each batch
 * projects virtual images -- its nodes at (i, j) and at (N-1-i, j) -- over the first a/2 angles,
 * full-width sample vectors even for narrow batches; admm_fwd_plan_info then reports the half
 * geometry's plans).  No device work. */
int admm_batch_info(admm_ctx* ctx, int* vb, int* mirror);
/* ABI 9: admm_consensus for the edge slots [e0, e1) only (stored z, midpoint fusion), whose
 * endpoints must all lie in x_ext rows [0, rows) -- the caller's promise; only those rows are
 * read.  With the rank-internal edges (both endpoints local, rows < V) first in slot order
 * (admm_hip/plan.py), a rank runs them while the halo exchange is still writing rows >= V, then
 * the rest: the same per-edge arithmetic and statistics as one admm_consensus, bitwise.
 * Replaces block_6_admm_loop_ver2.py:210-253 for those edges.  Enqueued directly (no graph). */
int admm_consensus_range(admm_ctx* ctx, int e0, int e1, int rows, void* stream);
/* ABI 9: average duration (ms) of the bound batch's back projector launch inside the CG solve
 * (the adjoint `Ai.T @ r` of block_6_admm_loop_ver2.py:145 fused with the CG operator
 * H p = A^T A p + rho D p + mu K^T K p and its dot products): one x-update is enqueued directly
 * with HIP events around each CG step's back projection (right after its forward combine, as in
 * every solve); the batch's state advances by that x-update.  Measurement helper for bench.py's
 * roofline of the dominant kernel; synchronises. */
int admm_time_back(admm_ctx* ctx, void* stream, double* ms_out);

/* --- per-pixel edge masks for masked precisions (setup) --- */

#define ADMM_MASK_KNN 0   /* top-k per node, symmetrised, + max spanning tree if disconnected */
#define ADMM_MASK_MST 1   /* maximum spanning tree of the complete graph at the pixel        */
#define ADMM_MASK_CHAIN 2 /* random permutation chain (orders from admm_chain_orders)         */
#define ADMM_Q_ARITHMETIC 0 /* q_ij = max((W_i + W_j)/2, 1e-12)        (block_3:33-39) */
#define ADMM_Q_HARMONIC 1   /* q_ij = max(W_i W_j / (W_i + W_j), 1e-12) (block_3:26-32) */
#define ADMM_MASK_MAX_NODES 64

/* keep[(i*V + j)*n + p] = 1 if edge (i, j) is active at pixel p, for all ordered pairs
 * (symmetric, zero diagonal).  Replaces _build_all_pixel_masks and its per-pixel helpers
 * (block_3_graph_and_precisions.py:62-187: _pixel_mask_knn_then_connect :62-110,
 * _pixel_mask_mst :113-131, _pixel_mask_chain :134-151).  W: [V][n] float64 device
 * (make_precisions' W_i), orders: [n][V] int32 device (ADMM_MASK_CHAIN only, else NULL),
 * keep: [V][V][n] uint8 device.  2 <= V <= ADMM_MASK_MAX_NODES.  kNN ties (equal q) go to
 * the higher node index; the reference's tie order is numpy argpartition's (unspecified).
 * Asynchronous on `stream` (current device). */
int admm_pixel_masks(const double* W, int V, int64_t n, int strategy, int k, int q_mode,
                     const int32_t* orders, uint8_t* keep, void* stream);
/* Host: the node orders of `_pixel_mask_chain` (block_3:134-151) for n pixels --
 * numpy Generator(PCG64).permutation(V) called n times in pixel order, replayed from
 * the bit generator state {state, inc} (pcg[0..3] = state_hi, state_lo, inc_hi, inc_lo;
 * has_uint32 / uinteger as numpy reports them).  orders: [n][V] int32 host memory.
 * pcg_out (may be NULL) receives the state afterwards (same layout + has_uint32, uinteger). */
int admm_chain_orders(const uint64_t pcg[4], int has_uint32, uint32_t uinteger, int V, int64_t n,
                      int32_t* orders, uint64_t pcg_out[6]);

#ifdef __cplusplus
}
#endif
#endif /* ADMM_TOMO_H */
