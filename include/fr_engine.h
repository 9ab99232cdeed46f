/*
 * fr_engine.h — C-ABI of the MI355X-native BPR training hot path.
 *
 * Drop-in boundary for sdu-zyx/Multi-modal-Food-Recommendation (FoodRec).  The reference is
 * pure Python on PyTorch; its "FFI" for this path is the set of ATen calls the plugin models
 * make.  Each export below replaces one of those call sites (file:line in /root/reference):
 *
 *   fr_spmm_csr          torch.sparse.mm(norm_adj, X) + torch.stack(..).mean(1)
 *                        models/cikm_model.py:187-190,199-202  models/pricai_modelx.py:183-226
 *                        models/lightgcn.py:136-144
 *   fr_bpr_fwd/_bwd      gather + mul().sum(1) + BPRLoss + EmbLoss
 *                        models/cikm_model.py:255-279  models/pricai_modelx.py:252-274
 *                        models/lightgcn.py:158-177  common/loss.py:32-34,45-50
 *   fr_dcor_fwd/_bwd     PRICAI_ModelX.correlation_distance x3 (models/pricai_modelx.py:263,409-437)
 *   fr_infonce_fwd/_bwd  PRICAI_ModelX.CL_loss (models/pricai_modelx.py:354-378)
 *   fr_adam_step         torch.optim.Adam.step (common/trainer.py:143-144,224)
 *   fr_sampler_*         TrainDataLoader.get_random_neg / init_neg_list (utils/dataloader.py:40-48,145-151)
 *
 * Conventions:
 *   - every function returns int: 0 = FR_OK, otherwise an fr_status code; it never throws
 *     across the ABI.  fr_last_error() returns a thread-local message for the last failure.
 *   - every pointer named d_* (or documented "device") is caller-owned device memory; the
 *     library never allocates or frees caller memory.  Scratch comes from a caller workspace
 *     whose size is returned by the matching *_workspace() query.
 *   - work is stream-ordered on the caller's hipStream_t (passed as void*), with no implicit
 *     host synchronisation, so calls may be captured into a hipGraph.
 *   - thread-safe for distinct streams.
 */
#ifndef FR_ENGINE_H
#define FR_ENGINE_H

#include <stdint.h>
#include <stdbool.h>

#ifdef __cplusplus
extern "C" {
#endif

enum fr_status {
  FR_OK = 0,
  FR_EINVAL = 1,   /* bad argument (null pointer, size, unsupported d)            */
  FR_EHIP = 2,     /* a HIP runtime call failed (message in fr_last_error)       */
  FR_ENOTSUP = 3,  /* combination not supported by this build                    */
  FR_ERANGE = 4,   /* an index/id outside its table                               */
  FR_EIO = 5,      /* a file could not be opened / mapped (message in fr_last_error) */
  FR_EPARSE = 6    /* a malformed field in a text file (line in fr_last_error)   */
};

enum fr_dtype { FR_F32 = 0, FR_BF16 = 1 };

int fr_version(void);
const char* fr_last_error(void);
/* number of HIP devices visible (0 when the runtime has no GPU) */
int fr_device_count(void);

/* ------------------------------------------------------------------------------------------
 * CSR SpMM with fused layer epilogue (LightGCN propagation, SURVEY 8(a) a6-a8,a12,a15).
 *
 *   acc[r]  = sum_{e in [rowptr[r], rowptr[r+1])} val[e] * X[col[e], 0:d]
 *   Y1[r]   = acc                                      (if d_Y1 != NULL)
 *   Y2[r]   = alpha*acc + beta1*A1[r] + beta2*A2[r]     (if d_Y2 != NULL; A1/A2 may be NULL)
 *
 * Rows are processed as work units of at most `chunk` edges (nnz balance for heavy rows).
 * The plan (built once per adjacency by fr_spmm_plan_host) lists units as int32 pairs
 * {row, chunk_index}: first the n_plain units of rows with <= chunk edges, then the units of
 * split rows grouped by row.  split_rows lists {row, first_partial, n_chunks} int32 triples;
 * partial sums of split rows go to the workspace and are combined in chunk order, so the
 * result is deterministic run to run.
 *
 * Y1/Y2 must not alias X.  A1/A2 may alias Y2 (same-row read-before-write).
 * Leading dimensions are in elements.  d must be a multiple of 4 and <= 1024.
 * ------------------------------------------------------------------------------------------ */
typedef struct fr_spmm_plan {
  const int32_t* d_units;       /* [n_units][2]  {row, chunk}                           */
  const int32_t* d_split_rows;  /* [n_split][3]  {row, first_partial, n_chunks}         */
  int64_t n_units;
  int64_t n_plain;
  int64_t n_split;
  int32_t chunk;                /* edges per unit                                        */
} fr_spmm_plan;

/* workspace bytes needed by fr_spmm_csr for this plan and feature width */
int64_t fr_spmm_workspace(const fr_spmm_plan* plan, int d);

/* Host-side planner: fills units (capacity n_rows + nnz/chunk + 1 pairs) and split_rows
 * (capacity n_rows triples) from a host copy of rowptr.  Returns FR_OK and writes counts. */
int fr_spmm_plan_host(const int64_t* rowptr, int64_t n_rows, int32_t chunk,
                      int32_t* units, int64_t* n_units, int64_t* n_plain,
                      int32_t* split_rows, int64_t* n_split);

int fr_spmm_csr(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val,
                int64_t n_rows, const fr_spmm_plan* plan,
                const float* d_X, int64_t ldx, int d,
                float* d_Y1, int64_t ldy1,
                float* d_Y2, int64_t ldy2, float alpha,
                const float* d_A1, int64_t lda1, float beta1,
                const float* d_A2, int64_t lda2, float beta2,
                void* d_workspace, int64_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * Fused gather-dot-BPR + EmbLoss.
 *   s+_b = <U[u_b], I[p_b]>,  s-_b = <U[u_b], I[n_b]>
 *   out[0] = -mean_b log(gamma + sigmoid(s+_b - s-_b))                  (BPRLoss)
 *   out[1..3] = ||Ue[u]||_F, ||Ie[p]||_F, ||Ie[n]||_F over the gathered [B,d] blocks
 *   out[4] = (out[1]+out[2]+out[3]) / B                                 (EmbLoss, unweighted)
 * Ue/Ie may be NULL (then out[1..4] = 0).  Index arrays are int64 device arrays.
 * workspace: fr_bpr_workspace(B) bytes; it keeps the per-triple scores and the norms that
 * fr_bpr_bwd reuses, so pass the same workspace to the matching backward call.
 * ------------------------------------------------------------------------------------------ */
int64_t fr_bpr_workspace(int64_t B);

int fr_bpr_fwd(const float* d_U, int64_t ldu, const float* d_I, int64_t ldi,
               const float* d_Ue, int64_t ldue, const float* d_Ie, int64_t ldie,
               const int64_t* d_u, const int64_t* d_p, const int64_t* d_n,
               int64_t B, int d, float gamma, float* d_out,
               void* d_workspace, int64_t workspace_bytes, void* stream);
/* fr_bpr_fwd that also writes the gathered item rows [I[p] ; I[n]] to d_rows ([2B, d], row stride
 * ld_rows; NULL: not written) -- the torch.cat([item_all[pos], item_all[neg]]) HealthRec's KD
 * term reads (cikm_model.py:256-257, 263) without a separate index_select launch. */
int fr_bpr_fwd_rows(const float* d_U, int64_t ldu, const float* d_I, int64_t ldi,
                    const float* d_Ue, int64_t ldue, const float* d_Ie, int64_t ldie,
                    const int64_t* d_u, const int64_t* d_p, const int64_t* d_n,
                    int64_t B, int d, float gamma, float* d_out, float* d_rows, int64_t ld_rows,
                    void* d_workspace, int64_t workspace_bytes, void* stream);
/* fr_bpr_fwd_rows with out[4] = w_emb * EmbLoss in fp32 (the models' reg_weight * reg term,
 * e.g. pricai_modelx.py:267, without a multiply launch; w_emb 1 is the EmbLoss itself). */
int fr_bpr_fwd_ex(const float* d_U, int64_t ldu, const float* d_I, int64_t ldi,
                  const float* d_Ue, int64_t ldue, const float* d_Ie, int64_t ldie,
                  const int64_t* d_u, const int64_t* d_p, const int64_t* d_n,
                  int64_t B, int d, float gamma, float w_emb, float* d_out, float* d_rows, int64_t ld_rows,
                  void* d_workspace, int64_t workspace_bytes, void* stream);

/* Backward.  g_mf scales d(out[0]); g_reg scales d(out[4]) (i.e. reg_weight * upstream grad).
 * d_gscale (optional, device float[2]) multiplies g_mf / g_reg on the device so no host
 * read of the upstream gradient is needed (d_gscale[1] is read only when dUe or dIe is given, so
 * a BPR-only backward may pass a single device float).  Gradients are ACCUMULATED (+=) into dU/dI/dUe/dIe
 * (any may be NULL); each uses the leading dimension of its forward table (ldu/ldi/ldue/ldie).  deterministic != 0 selects the ordered (atomic-free) scatter. */
int fr_bpr_bwd(const float* d_U, int64_t ldu, const float* d_I, int64_t ldi,
               const float* d_Ue, int64_t ldue, const float* d_Ie, int64_t ldie,
               const int64_t* d_u, const int64_t* d_p, const int64_t* d_n,
               int64_t B, int d, float gamma, float g_mf, float g_reg, const float* d_gscale,
               float* d_dU, float* d_dI, float* d_dUe, float* d_dIe,
               int deterministic, void* d_workspace, int64_t workspace_bytes, void* stream);
/* fr_bpr_bwd (non-deterministic scatter) plus d_extra_i [2B, d] (row stride ld_extra): the gradient of
 * the gathered item rows [I[pos]; I[neg]] from another consumer (HealthRec's KD term reads exactly
 * those rows, cikm_model.py:256-263), added to the pos / neg rows inside the same scatter. */
int fr_bpr_bwd_ex(const float* d_U, int64_t ldu, const float* d_I, int64_t ldi,
                  const float* d_Ue, int64_t ldue, const float* d_Ie, int64_t ldie,
                  const int64_t* d_u, const int64_t* d_p, const int64_t* d_n,
                  int64_t B, int d, float gamma, float g_mf, float g_reg, const float* d_gscale,
                  float* d_dU, float* d_dI, float* d_dUe, float* d_dIe, const float* d_extra_i, int64_t ld_extra,
                  void* d_workspace, int64_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * Fused multi-view distance correlation (CLUSSL SSL loss).
 * views: HOST array of V (<= 4) device pointers to [n, d] fp32 row-major (ld = d) matrices.
 * pairs: P (a,b) view-index pairs (host int32 [P][2]); out[k] = dcor(view a_k, view b_k)
 * exactly as PRICAI_ModelX.correlation_distance, and out[P] = sum_k out[k].
 * The backward takes d(out[P]) (the summed loss) scaled by g (or device d_gscale[0]) and
 * ACCUMULATES into dviews[v] (any may be NULL).
 * ------------------------------------------------------------------------------------------ */
/* SSL kernel choice: mfma = 1 (default) runs the dCor / InfoNCE Gram tiles on v_mfma_f32_16x16x4_f32,
 * 2 the same with the round-4 InfoNCE kernels (row-layout logits, W staged in LDS), 0 the VALU 4x4-per-thread tiles (A/B
 * measurements), -1 keeps it; returns the previous choice. */
/* Measurement: fr_stamp launches one single-lane kernel that writes the device's constant-rate wall
 * clock (fr_stamp_hz ticks per second, 0 without a device) to *d_slot: two stamps on a stream bracket
 * the kernels issued between them, also inside a captured HIP graph (no timing events there). */
int fr_stamp(int64_t* d_slot, void* stream);
int64_t fr_stamp_hz(void);
int fr_ssl_kernels(int mfma);
int64_t fr_dcor_workspace(int64_t n, int n_views);

int fr_dcor_fwd(const float* const* d_views, int n_views, int64_t n, int d,
                const int32_t* pairs, int n_pairs, float* d_out,
                void* d_workspace, int64_t workspace_bytes, void* stream);

int fr_dcor_bwd(const float* const* d_views, int n_views, int64_t n, int d,
                const int32_t* pairs, int n_pairs, float g, const float* d_gscale,
                float* const* d_dviews,
                void* d_workspace, int64_t workspace_bytes, void* stream);
/* _ex forms: out[P] = weight * sum_k out[k] in fp32 (CLUSSL's loss_cl * SSL term, pricai_modelx.py:263-
 * 267, without a separate multiply launch; weight 1 is the plain sum); the backward with overwrite != 0
 * WRITES dviews (no zero-filled buffers needed) instead of accumulating. */
int fr_dcor_fwd_ex(const float* const* d_views, int n_views, int64_t n, int d,
                   const int32_t* pairs, int n_pairs, float weight, float* d_out,
                   void* d_workspace, int64_t workspace_bytes, void* stream);
int fr_dcor_bwd_ex(const float* const* d_views, int n_views, int64_t n, int d,
                   const int32_t* pairs, int n_pairs, float g, const float* d_gscale,
                   float* const* d_dviews, int overwrite,
                   void* d_workspace, int64_t workspace_bytes, void* stream);

/* CLUSSL's view sum and SSL gathers (PRICAI_ModelX.forward + calculate_loss,
 * models/pricai_modelx.py:227-263: item_emb = ingre + image + text, then each view at the batch
 * items): d_total = ((views[0] + views[1]) + ...) [n, d] in that order, d_gathered[k] [m, d] =
 * views[k][ids] (ids outside [0, n) gather zeros).  1 <= n_views <= 4, d % 4 == 0, 16-byte aligned. */
int fr_views_sum_gather(const float* const* d_views, int n_views, int64_t n, int d,
                        const int64_t* d_ids, int64_t m, float* d_total, float* const* d_gathered,
                        void* stream);
/* Its backward: d_dviews[k] = d_gsum (NULL: zeros) + sum over j with ids[j] = r of d_grows[k][j], written in
 * full.  Default: a broadcast, then float atomics (one wave-instruction per row and view; duplicate ids
 * add in hardware order, as torch's index_add_).  deterministic != 0: the (id, j) pairs are sorted (one
 * workgroup, workspace m * 8 bytes) and the head of each id's run adds that row's terms in increasing j
 * (no atomics; m <= 8192). */
int64_t fr_views_sum_gather_bwd_workspace(int64_t m);
int fr_views_sum_gather_bwd(const float* d_gsum, const float* const* d_grows, int n_views, int64_t n, int d,
                            const int64_t* d_ids, int64_t m, float* const* d_dviews, int deterministic,
                            void* d_workspace, int64_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * Fused InfoNCE / NT-Xent (PRICAI_ModelX.CL_loss, hidden_norm=True): H is [2b, d];
 * out[0] = (CE([h1 h2^T | h1 h1^T - 1e9 I]/tau) + CE([h2 h1^T | h2 h2^T - 1e9 I]/tau)) / b.
 * ------------------------------------------------------------------------------------------ */
int64_t fr_infonce_workspace(int64_t b);

int fr_infonce_fwd(const float* d_H, int64_t b, int d, float tau, float* d_out,
                   void* d_workspace, int64_t workspace_bytes, void* stream);

int fr_infonce_bwd(const float* d_H, int64_t b, int d, float tau, float g, const float* d_gscale,
                   float* d_dH, void* d_workspace, int64_t workspace_bytes, void* stream);

/* InfoNCE over several view pairs in the same launches (CLUSSL's ssl_mode infonce:
 * sum over pairs (a, b) of CL_loss(cat([views[a], views[b]])), pricai_modelx.py:263 / :354-378):
 * views are n_views (<= 4) tables [b, d]; pairs[2k], pairs[2k+1] index them (n_pairs <= 16).  No
 * concatenated copies; every view is normalised once; the backward sums each view's upstream over
 * the pairs that hold it and writes d_dviews[v] (entries may be NULL).
 * out[0] = the fp32 sum of the pair losses in pair order, out[1 + k] = pair k's loss.
 * fr_infonce_fwd/_bwd are this with the two halves of H as views 0, 1 and one pair (d_dH written). */
int64_t fr_infonce_multi_workspace(int n_views, int64_t b, int d, int n_pairs);
int fr_infonce_multi_fwd(const float* const* d_views, int n_views, int64_t b, int d, const int32_t* pairs,
                         int n_pairs, float tau, float* d_out, void* d_workspace, int64_t workspace_bytes,
                         void* stream);
int fr_infonce_multi_bwd(const float* const* d_views, int n_views, int64_t b, int d, const int32_t* pairs,
                         int n_pairs, float tau, float g, const float* d_gscale, float* const* d_dviews,
                         void* d_workspace, int64_t workspace_bytes, void* stream);
/* out[0] = weight * (the fp32 pair sum) (CLUSSL's loss_cl * CL term without a multiply launch). */
int fr_infonce_multi_fwd_ex(const float* const* d_views, int n_views, int64_t b, int d, const int32_t* pairs,
                            int n_pairs, float tau, float weight, float* d_out, void* d_workspace,
                            int64_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * Multi-tensor Adam, following torch.optim.Adam (amsgrad=False, maximize=False) element order:
 *   g += wd*p;  m = m + (1-b1)(g-m);  v = v*b2 + ((1-b2)g)g;
 *   p += (-lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps),   bc_k = 1 - b_k^step (host, double)
 * The pointer arrays and numel are HOST arrays of device pointers (they travel in the kernel
 * argument block, 24 tensors per launch).  step is 1-based (after increment).
 * d_skip (optional device int32): when *d_skip != 0 the update is a no-op (NaN guard).
 * ------------------------------------------------------------------------------------------ */
int fr_adam_step(float* const* params, const float* const* grads,
                 float* const* exp_avg, float* const* exp_avg_sq,
                 const int64_t* numel, int n_tensors, int64_t max_numel,
                 double lr, double beta1, double beta2, double eps, double weight_decay,
                 int64_t step, const int32_t* d_skip, void* stream);

/* Device-scalar variant (graph-capturable optimiser step): each tensor's step counter lives in
 * device memory (int64, incremented by the call before use) and the learning rate is read from
 * d_lr (device double; NULL -> lr), so a captured step replays with the current step and lr.
 * d_steps is a HOST array of device pointers, one per tensor.  The launch's last workgroup bumps
 * the counters; it finds out that it is last through d_ticket, FR_ADAM_TICKET_WORDS device uint32
 * words owned by the caller (16-byte aligned, zero before first use; every launch leaves them zero).
 * Launches that share ticket words must not overlap: give each optimiser its own. */
#define FR_ADAM_TICKET_WORDS 32
int fr_adam_step_dev(float* const* params, const float* const* grads,
                     float* const* exp_avg, float* const* exp_avg_sq,
                     int64_t* const* d_steps, const int64_t* numel, int n_tensors,
                     const double* d_lr, double lr, double beta1, double beta2, double eps,
                     double weight_decay, const int32_t* d_skip, uint32_t* d_ticket, void* stream);

/* ------------------------------------------------------------------------------------------
 * Negative sampler (host code): numpy legacy MT19937 stream, masked-rejection bounded ints,
 * exactly the draws np.random.randint(num_items) makes in TrainDataLoader.get_random_neg.
 * state: 624 uint32 key + pos (as numpy.random.get_state()[1:3]); updated in place.
 * Exclusion sets are per-user sorted int64 lists in CSR form (train items, valid+test items):
 * excl_ptr / excl2_ptr hold n_users + 1 entries, start at 0 and never decrease.  Every user id
 * must lie in [0, n_users) (FR_ERANGE otherwise, checked before any lookup); a user whose two
 * lists together contain every item of [0, num_items) returns FR_ERANGE (the reference's
 * rejection loop would not end).  Unsorted lists give wrong draws, never an out-of-bounds read.
 * ------------------------------------------------------------------------------------------ */
int fr_sampler_negatives(uint32_t* mt_key, int32_t* mt_pos, int64_t num_items,
                         const int64_t* users, int64_t n, int64_t n_users,
                         const int64_t* excl_ptr, const int64_t* excl_items,
                         const int64_t* excl2_ptr, const int64_t* excl2_items,
                         int64_t* out_neg);
/* the same draws for users[perm[k]], k < n (the epoch's permutation order: no permuted copy of the
 * users); users holds n_pairs ids and every perm value must index it (FR_ERANGE otherwise) */
int fr_sampler_negatives_perm(uint32_t* mt_key, int32_t* mt_pos, int64_t num_items,
                              const int64_t* users, int64_t n_pairs, const int64_t* perm, int64_t n,
                              int64_t n_users, const int64_t* excl_ptr, const int64_t* excl_items,
                              const int64_t* excl2_ptr, const int64_t* excl2_items,
                              int64_t* out_neg);

/* raw masked-rejection draws (test hook): out[i] = np.random.randint(high) for i < n */
int fr_sampler_randint(uint32_t* mt_key, int32_t* mt_pos, int64_t high, int64_t n, int64_t* out);

/* ---- embedding-table backward (row scatter-add) -------------------------------------------
 * dW[r,:] = sum of G[i,:] over positions i with idx[i] == r, r != padding_idx (-1: none); every
 * row of dW is written (zeros where untouched).  Replaces the backward of the reference's row
 * gathers: ingr_all[ingredients] (FoodRec/models/cikm_model.py:230), ingre_embedding(...) with
 * padding_idx (cikm_model.py:67-68, 270-271), image_/text_embedding (cikm_model.py:83-87).
 * Deterministic (position-ordered sums inside fixed chunks, chunk partials in chunk order); no
 * launch shape depends on device data (graph capturable).  n <= 2^18, d % 4 == 0. */
int64_t fr_embedding_bwd_workspace(int64_t n, int64_t num_rows, int d);
int fr_embedding_bwd(const int64_t* d_idx, int64_t n, const float* d_grad, int64_t ldg, int d,
                     int64_t num_rows, int64_t padding_idx, float* d_out, int64_t ldo,
                     void* d_workspace, int64_t workspace_bytes, void* stream);

/* The same scatter with float atomics (run-to-run summation order not fixed; fr_embedding_bwd is
 * the deterministic form): d_out += scatter, d = 64; rows equal to hot_row (e.g. an ingredient
 * padding id that fills half the positions) are pre-summed per workgroup (one atomic row update per
 * workgroup).  The caller zero-fills d_out for a plain embedding gradient.  2 launches (fill + this)
 * instead of the sort path's 8. */
int fr_embedding_bwd_atomic(const int64_t* d_idx, int64_t n, const float* d_grad, int64_t ldg, int d,
                            int64_t num_rows, int64_t padding_idx, int64_t hot_row, float* d_out, int64_t ldo,
                            void* stream);

/* Row-gradient form of the same scatter: rmap[r] = the first position i with idx[i] == r (else -1;
 * padding_idx rows get -1) and rows[i, :] = sum over positions j with idx[j] == r of grad[j, :]
 * (the same sums in the same order as fr_embedding_bwd, deterministic); rows of non-owner
 * positions are left unwritten.  rmap: [num_rows] int32; rows: [n, d] fp32 (ld = d).  No dense
 * table is touched.  Workspace: fr_embedding_rowgrad_workspace(n, num_rows, d) bytes. */
int64_t fr_embedding_rowgrad_workspace(int64_t n, int64_t num_rows, int d);
int fr_embedding_rowgrad(const int64_t* d_idx, int64_t n, const float* d_grad, int64_t ldg, int d,
                         int64_t num_rows, int64_t padding_idx, int32_t* d_rmap, float* d_rows,
                         void* d_workspace, int64_t workspace_bytes, void* stream);
/* byte offset, inside the workspace, of the int32 status word of the last fr_embedding_bwd on it:
 * 0 = consistent; non-zero bits name the step that met an out-of-range index on the device and
 * skipped that access instead of faulting (1 scan, 2 place, 4/8 bucket order, 16 segsum, 32 fix-up) */
int64_t fr_embedding_bwd_status_offset(int64_t num_rows);

/* ---- Linear weight/bias gradient over many rows ---------------------------------------------
 * dW[n,k] = sum_m dY[m,n] X[m,k] (written with row stride ldw), db[n] = sum_m dY[m,n] (d_db may
 * be null).  Replaces the weight-gradient GEMMs of the Linear layers of the reference's ingredient
 * Transformer (FoodRec/models/cikm_model.py:33-35, nn.TransformerEncoderLayer over 2B x 20 tokens)
 * and of image_trs / text_trs (cikm_model.py:240-241).  Split over row slabs, slab partials summed
 * in fixed order (deterministic).  N, K multiples of 4; dY, X 16-byte aligned. */
int64_t fr_linear_wgrad_workspace(int64_t M, int N, int K);
int fr_linear_wgrad(const float* d_dy, int64_t ldy, const float* d_x, int64_t ldx, int64_t M, int N, int K,
                    float* d_dw, int64_t ldw, float* d_db, void* d_workspace, int64_t workspace_bytes,
                    void* stream);

/* ---- LayerNorm over the last dimension ---------------------------------------------------------
 * Forward writes y and per-row mean / rstd (fp32); backward writes dx and, when requested, dgamma /
 * dbeta (deterministic block partials + ordered reduce; workspace from fr_layernorm_bwd_workspace).
 * Replaces nn.LayerNorm in the reference's ingredient Transformer (FoodRec/models/cikm_model.py:33-35)
 * and target_attention_layer's shared Q/K LayerNorm (cikm_model.py:326-327, 349-350).
 * d = 4 * 2^k <= 256; gamma/beta may be null (no affine). */
int fr_layernorm_fwd(const float* d_x, int64_t ldx, int64_t rows, int d, const float* d_gamma,
                     const float* d_beta, float eps, float* d_y, int64_t ldy, float* d_mean, float* d_rstd,
                     void* stream);
int64_t fr_layernorm_bwd_workspace(int d);
int fr_layernorm_bwd(const float* d_dy, int64_t lddy, const float* d_x, int64_t ldx, int64_t rows, int d,
                     const float* d_mean, const float* d_rstd, const float* d_gamma, float* d_dx, int64_t lddx,
                     float* d_dgamma, float* d_dbeta, void* d_workspace, int64_t workspace_bytes, void* stream);

/* ---- device negative sampling over a CSR interaction graph --------------------------------------
 * out[b] = item id uniform in [0, n_items), redrawn (counter-based RNG: seed, b, attempt) while
 * item_base + id is in user d_users[b]'s CSR row (sorted columns); at most max_tries draws.  The
 * reference's get_random_neg (FoodRec/utils/dataloader.py:145-151) for graphs whose exclusion lists
 * do not fit the host sampler (BASELINE config 4, 200M interactions). */
int fr_sample_negatives_csr(const int64_t* d_rowptr, const int32_t* d_col, int64_t n_users, const int64_t* d_users,
                            int64_t B, int64_t n_items, int64_t item_base, uint64_t seed, int max_tries,
                            int64_t* d_out, void* stream);

/* ==========================================================================================
 * bf16 tables (BASELINE config 5: d=256 bf16 embeddings, fp32 arithmetic, fp32 Adam state).
 * Tables are uint16_t bit patterns of bfloat16 (torch.bfloat16 storage), row-major, 16-B aligned
 * rows (ld % 8 == 0).  Same semantics as the fp32 entry points; results are rounded to bf16 once
 * per output element (round to nearest even).
 * ========================================================================================== */

/* fr_spmm_csr over bf16 X/Y1/Y2/A1/A2 (fp32 edge values and accumulation); d % 8 == 0.
 * Replaces torch.sparse.mm(norm_adj, X) + the layer mean (models/lightgcn.py:136-144) at d=256. */
int64_t fr_spmm_bf16_workspace(const fr_spmm_plan* plan, int d);
int fr_spmm_csr_bf16(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val,
                     int64_t n_rows, const fr_spmm_plan* plan,
                     const uint16_t* d_X, int64_t ldx, int d,
                     uint16_t* d_Y1, int64_t ldy1,
                     uint16_t* d_Y2, int64_t ldy2, float alpha,
                     const uint16_t* d_A1, int64_t lda1, float beta1,
                     const uint16_t* d_A2, int64_t lda2, float beta2,
                     void* d_workspace, int64_t workspace_bytes, void* stream);

/* fr_bpr_fwd / fr_bpr_bwd over bf16 tables (models/lightgcn.py:158-177, common/loss.py:32-50).
 * Workspace: fr_bpr_workspace(B).  The backward is the deterministic owner-slot scatter; each
 * destination row's fp32 sum is added to the bf16 gradient row once. */
int fr_bpr_fwd_bf16(const uint16_t* d_U, int64_t ldu, const uint16_t* d_I, int64_t ldi,
                    const uint16_t* d_Ue, int64_t ldue, const uint16_t* d_Ie, int64_t ldie,
                    const int64_t* d_u, const int64_t* d_p, const int64_t* d_n,
                    int64_t B, int d, float gamma, float* d_out,
                    void* d_workspace, int64_t workspace_bytes, void* stream);
int fr_bpr_bwd_bf16(const uint16_t* d_U, int64_t ldu, const uint16_t* d_I, int64_t ldi,
                    const uint16_t* d_Ue, int64_t ldue, const uint16_t* d_Ie, int64_t ldie,
                    const int64_t* d_u, const int64_t* d_p, const int64_t* d_n,
                    int64_t B, int d, float gamma, float g_mf, float g_reg, const float* d_gscale,
                    uint16_t* d_dU, uint16_t* d_dI, uint16_t* d_dUe, uint16_t* d_dIe,
                    void* d_workspace, int64_t workspace_bytes, void* stream);

/* Row-gradient Adam: tensors whose gradient is g[r] = rmap[r] >= 0 ? rows[rmap[r]] : 0 (a [R, d]
 * table gathered by rows on the step, d a power of two >= 4; rows/rmap from fr_embedding_rowgrad).
 * Same per-element arithmetic as fr_adam_step_dev (bit-identical to the dense update with the dense
 * zero-padded gradient) at 24 B instead of 28 B (+ the dense zero fill) per parameter.  Replaces
 * torch.optim.Adam.step for HealthRec's image/text feature tables (cikm_model.py:83-87). */
int fr_adam_step_rows(float* const* params, const float* const* grads, float* const* exp_avg,
                      float* const* exp_avg_sq, int64_t* const* d_steps, const int64_t* numel,
                      const int32_t* const* d_rmaps, const int32_t* row_dims, int n_tensors, const double* d_lr,
                      double lr, double beta1, double beta2, double eps, double weight_decay,
                      const int32_t* d_skip, uint32_t* d_ticket, void* stream);

/* Row-gradient Adam with deferred zero-gradient steps (exact "lazy rows").  Same contract as
 * fr_adam_step_rows (torch.optim.Adam.step, common/trainer.py:224, over cikm_model.py:83-87's
 * image/text tables), but a row with no gradient this step is not touched: the step's
 * (-lr/bc1, sqrt(bc2), and as a double in floats 2-3 RN64(1 / sqrt(bc2)_f32)) go to
 * d_hist[t][(step % hist_cap)] and d_last[t][r] holds the step row r is
 * current through.  A row with a gradient first replays its skipped steps with g = 0 (the dense
 * kernel's float operations), then applies this step.  fr_adam_flush_rows brings every row up to
 * the current step; after a flush p, exp_avg and exp_avg_sq equal fr_adam_step_rows' bit for bit.
 * The caller flushes before any full-table read and at least every hist_cap - 1 steps.
 * d_ids[t][0..n_ids[t]): the ids whose gradient rows d_rmaps[t] maps (duplicates allowed; the
 * kernel works per id, not per table row).  d_last: int32 [R] per tensor (zero at step 0); d_hist:
 * float32 [hist_cap, 4] per tensor (16-byte aligned); n_tensors <= 16.  Deferred zero-gradient steps
 * are replayed with the division by sqrt(bc2) as RN32(double(s) * that reciprocal): bit-identical to
 * the dense step (a quotient of two fp32 numbers is never within 2^-49 of an fp32 rounding
 * boundary; the double product is within 2^-52). */
int fr_adam_step_rows_lazy(float* const* params, const float* const* grads, float* const* exp_avg,
                           float* const* exp_avg_sq, int64_t* const* d_steps, const int64_t* numel,
                           const int32_t* const* d_rmaps, const int64_t* const* d_ids, const int64_t* n_ids,
                           const int32_t* row_dims, int32_t* const* d_last,
                           float* const* d_hist, int32_t hist_cap, int n_tensors, const double* d_lr,
                           double lr, double beta1, double beta2, double eps, double weight_decay,
                           const int32_t* d_skip, void* stream);
int fr_adam_flush_rows(float* const* params, float* const* exp_avg, float* const* exp_avg_sq,
                       int64_t* const* d_steps, const int64_t* numel, const int32_t* row_dims,
                       int32_t* const* d_last, float* const* d_hist, int32_t hist_cap, int n_tensors,
                       double beta1, double beta2, double eps, double weight_decay, void* stream);

/* Catch-up for a lazily updated table before a row gather (the forward of cikm_model.py:240-241's
 * image_trs/text_trs over embImage/embText rows): rows d_ids[0..n) (duplicates allowed) replay their
 * deferred zero-gradient steps through the current step, so the gather reads the dense-Adam values. */
int fr_adam_catch_up_rows(float* param, float* exp_avg, float* exp_avg_sq, const int64_t* d_step,
                          const int64_t* d_ids, int64_t n, int64_t rows, int32_t row_dim, int32_t* d_last,
                          const float* d_hist, int32_t hist_cap, double beta1, double beta2, double eps,
                          double weight_decay, void* stream);

/* fr_adam_catch_up_rows for up to 4 tables gathered at the same ids (HealthRec's image and text
 * tables at the batch's items), one launch (grid.y = table). */
int fr_adam_catch_up_rows_multi(int n_tables, float* const* params, float* const* exp_avg,
                                float* const* exp_avg_sq, const int64_t* const* d_steps, const int64_t* rows,
                                const int32_t* row_dims, int32_t* const* d_last, const float* const* d_hist,
                                const int64_t* d_ids, int64_t n, int32_t hist_cap, double beta1, double beta2,
                                double eps, double weight_decay, void* stream);
/* Diagnostic: n random operand sets through the replay kernels' rounding shortcuts, on the device,
 * against the compiler's IEEE fp32 division and sqrt.  d_bad (3 device counters, accumulated):
 * in-range division mismatches, in-range sqrt mismatches, full-range sqrt_rn mismatches. */
int fr_adam_rounding_selftest(int64_t n, uint64_t seed, unsigned long long* d_bad, void* stream);

/* Background slice of a flush (no reference counterpart: the reference's torch.optim.Adam updates
 * every row every step, common/trainer.py:143-144,224).  At device step counter st, rows
 * [R s / K, R (s + 1) / K), s = st % n_slices, of every table replay their deferred zero-gradient
 * steps through st; rows already current skip.  One launch per step bounds every row's backlog by
 * n_slices steps; bit-identical to the dense update like every lazy-row replay. */
int fr_adam_catch_up_slice(int n_tables, float* const* params, float* const* exp_avg, float* const* exp_avg_sq,
                           const int64_t* const* d_steps, const int64_t* rows, const int32_t* row_dims,
                           int32_t* const* d_last, const float* const* d_hist, int32_t n_slices, int32_t hist_cap,
                           double beta1, double beta2, double eps, double weight_decay, void* stream);
/* A/B switch (library state): the background slice on at most max_blocks workgroups in total, each
 * striding over its rows (0, the default: one wave per row). */
int fr_adam_slice_blocks(int64_t max_blocks);
/* the same slice in n_parts launches: part p replays the p-th of n_parts even row ranges of the step's
 * slice (a step issues every part, at points of its choosing, before the optimiser's lazy kernels) */
int fr_adam_catch_up_slice_part(int n_tables, float* const* params, float* const* exp_avg,
                                float* const* exp_avg_sq, const int64_t* const* d_steps, const int64_t* rows,
                                const int32_t* row_dims, int32_t* const* d_last, const float* const* d_hist,
                                int32_t n_slices, int32_t part, int32_t n_parts, int32_t hist_cap, double beta1,
                                double beta2, double eps, double weight_decay, void* stream);

/* Mixed-precision Adam for one bf16 parameter (torch.optim.Adam.step, common/trainer.py:224):
 * the update runs on the fp32 master copy with fp32 exp_avg / exp_avg_sq (same element order as
 * fr_adam_step) and the bf16 parameter is re-rounded from the master.  d_step: device int64
 * counter incremented by the call; d_lr: device double (NULL -> lr).  numel % 8 == 0. */
int fr_adam_step_bf16(uint16_t* d_param, float* d_master, const uint16_t* d_grad,
                      float* d_exp_avg, float* d_exp_avg_sq, int64_t* d_step, int64_t numel,
                      const double* d_lr, double lr, double beta1, double beta2, double eps,
                      double weight_decay, const int32_t* d_skip, void* stream);

/* ------------------------------------------------------------------------------------------
 * Full-sort top-k (BASELINE config 5's MFMA user x item GEMM).
 * For each of n_users query rows U[u] (dtype FR_BF16: d in {64,128,256}; FR_F32: d in {64,128}):
 *   score(u, i) = <U[u], I[i]> for i < n_items         (full_sort_predict, the dense MMRec form:
 *                                                         common/abstract_recommender.py:39-50)
 *   items (item_base + i) present in the exclusion CSR row of user id uid[u] are skipped
 *   (history masking; d_ex_ptr NULL = no masking, the reference trainer's evaluate())
 *   out_items[u, 0:k] / out_scores[u, 0:k] = the k best by (score desc, item id asc)
 *                                            (torch.topk in Trainer.evaluate, trainer.py:476-503)
 *   hits[u, j] = out_items[u, j] is in held-out CSR row uid[u] (TopKEvaluator.evaluate's
 *                `i in pos_items`, utils/topk_evaluator.py:104-107); d_hits may be NULL.
 * uid: device int64 [n_users] global user ids (NULL = row index).  CSR rows: int64 rowptr,
 * int32 sorted columns; test_base / ex_base offset item ids into the CSR column space.
 * k <= 32.  Missing entries (fewer than k admissible items) are item -1, score -inf.
 * Never materialises the n_users x n_items score matrix.  Workspace: fr_topk_workspace.
 * ------------------------------------------------------------------------------------------ */
int64_t fr_topk_workspace(int64_t n_users, int64_t n_items, int k);
int fr_topk_scores(const void* d_U, int64_t ldu, int64_t n_users, const void* d_I, int64_t ldi,
                   int64_t n_items, int d, int dtype, int k, const int64_t* d_uid,
                   const int64_t* d_ex_ptr, const int32_t* d_ex_col, int64_t ex_base,
                   const int64_t* d_test_ptr, const int32_t* d_test_col, int64_t test_base,
                   float* d_out_scores, int64_t* d_out_items, uint8_t* d_hits,
                   void* d_workspace, int64_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * Fused post-norm Transformer encoder layer, training forward + backward.
 * Replaces nn.TransformerEncoderLayer(d_model=64, nhead=2, dim_feedforward=256, dropout=p,
 * activation=gelu|relu) of HealthRec's ingredient encoder (FoodRec/models/cikm_model.py:33-35,
 * called at :232-238 over 2B sequences of L ingredient tokens):
 *   x1 = LN1(x + dropout1(MHA(x, key_padding_mask)))   x2 = LN2(x1 + dropout2(FF(x1)))
 * x / out: [n_seq, L, 64] fp32 batch-first; d_mask: [n_seq, L] additive key mask (0 / -inf,
 * torch's canonical float form) or NULL.  L in {4, 5, 8, 10, 16, 20}.
 * d_params (12 device pointers, torch parameter order): in_proj_weight [192,64], in_proj_bias,
 *   out_proj.weight [64,64], out_proj.bias, norm1.weight, norm1.bias, linear1.weight [256,64],
 *   linear1.bias, linear2.weight [64,256], linear2.bias, norm2.weight, norm2.bias.
 * eps[2]: norm1/norm2 eps.  drop[4]: p of attention-prob dropout, dropout1, dropout (FF act),
 * dropout2.  Masks come from a counter-based hash of (seed, *d_counter, site, element); the
 * forward stores the counter value it used in *d_seed_out and the backward reads it back (the
 * caller advances the counter; graph replays draw fresh masks).
 * Forward saves qkv [T,192], ctx [T,64], y1 [T,64] (LN1 input), fact [T,256] (dropout(act(FF1))),
 * y2 [T,64] (LN2 input), st1/st2 [T,2] (mean, rstd), T = n_seq * L, and dact (keep/(1-p) *
 * act'(FF1)) as fr_encoder_dact_numel(n_seq, L) floats in the kernels' MFMA fragment layout
 * (opaque to the caller; only fr_encoder_bwd reads it).  (Recomputing the FF activation in the
 * backward instead -- one more GEMM and the GELU / GELU' epilogue -- measured 175k vs 147k cycles
 * per backward launch: the VALU epilogue, not the 42 MB of saved activations, is the cost.)
 * Backward writes dx and its per-workgroup weight-gradient partials d_partials
 * [fr_encoder_partials(n_seq, L)]; with d_grad non-NULL it also sums them in workgroup order
 * (deterministic) into the flat parameter gradient d_grad [fr_encoder_grad_numel()] (the 12
 * gradients concatenated in d_params order), with d_grad NULL it leaves them for a later
 * fr_encoder_reduce or for the next backward call: d_prev_partials / d_prev_grad (both or neither)
 * name another call's partials (same n_seq and L) that this launch reduces into d_prev_grad -- a
 * stacked encoder's layer-(k+1) reduction folded into layer k's launch.
 * ------------------------------------------------------------------------------------------ */
int64_t fr_encoder_partials(int64_t n_seq, int L);
int64_t fr_encoder_grad_numel(void);
int64_t fr_encoder_dact_numel(int64_t n_seq, int L);
/* Diagnostics: enable (1) / disable (0) / keep (-1) per-phase s_memtime stamps of workgroup 0 and
 * copy the stamp table (uint64 [2][32]: forward, backward; shader clock) to host_marks if non-NULL. */
int fr_encoder_profile(int enable, uint64_t* host_marks);
int fr_encoder_fwd(const float* d_x, const float* d_mask, int64_t n_seq, int L, const float* const* d_params,
                   const float* eps, const float* drop, uint64_t seed, int gelu, const int64_t* d_counter,
                   int64_t* d_seed_out, float* d_out, float* d_qkv, float* d_ctx, float* d_y1, float* d_fact,
                   float* d_dact, float* d_y2, float* d_st1, float* d_st2, void* stream);
int fr_encoder_bwd(const float* d_dout, const float* d_x, const float* d_mask, int64_t n_seq, int L,
                   const float* const* d_params, const float* eps, const float* drop, uint64_t seed, int gelu,
                   const int64_t* d_seed_in, const float* d_qkv, const float* d_ctx, const float* d_y1,
                   const float* d_fact, const float* d_dact, const float* d_y2, const float* d_st1,
                   const float* d_st2, float* d_dx, float* d_grad, float* d_partials, int64_t partial_floats,
                   const float* d_prev_partials, float* d_prev_grad, void* stream);
int fr_encoder_reduce(const float* d_partials, int64_t n_seq, int L, float* d_grad, void* stream);
/* A/B switches (host-side library state): reduce_mode 0 = the column-slice ordered partial reduction
 * (default), 1 = the form streaming whole 1 KiB pieces of each workgroup's partial row;
 * -1 leaves the setting.  Both are deterministic. */
int fr_encoder_options(int reduce_mode);

/* ------------------------------------------------------------------------------------------
 * HealthRec's loss head after the encoder as one op (models/cikm_model.py:245-264, 304-308,
 * 311-369): fr_modal_fusion's know / hin per item (see below) feeding fr_health_kd's terms,
 *   d_out[0] = w_health * sum(BCE(sigmoid(mlp(hin)), labels)),
 *   d_out[1] = w_kd * max(0, 1 - mean_i cos(know_i, rows_i) - kd_threshold),  d_out[2] = the gate,
 * with know / hin and their gradients kept in registers.  Forward: 1 launch when d_ticket (a zero-
 * initialised int32, reset to 0 by the launch) is given -- the last block to arrive runs the fixed-
 * order finalize -- else 2 (per-item kernel + finalize kernel).  Backward: 1 launch writing d_denc [n, L, 64], d_dquery [n, 2, 64], d_drows
 * [n, 64] and one partial row per block; fr_modal_head_reduce sums them in block order into d_grad
 * [fr_modal_head_grad_numel()] = dW1 [64x64] | db1 [64] | dW2 [16x64, rows >= H zero] | db2 [16] |
 * d ln_a.weight [32] | d ln_a.bias | d ln_b.weight | d ln_b.bias.  d_ln / d_mlp as in
 * fr_modal_fusion_* / fr_health_kd_*.  Replaces 7 launches of the separate ops.
 * ------------------------------------------------------------------------------------------ */
int64_t fr_modal_head_partials(int64_t n_items, int backward);
int64_t fr_modal_head_grad_numel(void);
int fr_modal_head_fwd(const float* d_enc, const float* d_query, const int64_t* d_ids, const int64_t* d_num,
                      int64_t pad_id, int64_t n_items, int L, const float* const* d_ln, float eps, const float* d_rows,
                      const float* d_labels, int H, const float* const* d_mlp, float kd_threshold, float w_health,
                      float w_kd, float* d_out, float* d_partials, int64_t partial_floats, int32_t* d_ticket,
                      void* stream);
/* The forward's per-item kernel alone (block partials only; d_out untouched), and HealthRec's loss
 * finalize as one launch: the head's finalize (d_out[0..2] as fr_modal_head_fwd writes them), the EmbLoss
 * ingredient norms from fr_gather_norms_fwd's partials (d_nrm, as fr_reg_combine_norms_fwd), d_reg =
 * w_reg * (d_emb3[0] + (nrm[0] + nrm[1]) / B), and, when d_acc is given, the step's bookkeeping over
 * the parts [d_mf, d_out[0], d_out[1], d_reg] exactly as fr_step_book (counters advanced, fp32 sum to
 * d_loss, NaN flag).  The loss chain after the encoder is then 4 launches: items, finalize, backward,
 * reduce (models/cikm_model.py:245-279 + trainer.py:183-193).  d_head_partials NULL: no head finalize;
 * d_norm_partials NULL: no norms / reg; the bookkeeping needs both. */
int fr_modal_head_fwd_items(const float* d_enc, const float* d_query, const int64_t* d_ids, const int64_t* d_num,
                            int64_t pad_id, int64_t n_items, int L, const float* const* d_ln, float eps,
                            const float* d_rows, const float* d_labels, int H, const float* const* d_mlp,
                            float kd_threshold, float w_health, float w_kd, float* d_partials, int64_t partial_floats,
                            void* stream);
int fr_healthrec_loss_finalize(const float* d_head_partials, int64_t n_items, float kd_threshold, float w_health,
                               float w_kd, float* d_out, const float* d_norm_partials, int64_t n_norm_rows,
                               const float* d_emb3, float B, float w_reg, float* d_nrm, float* d_reg,
                               const float* d_mf, double* d_acc, int accumulate, int32_t* d_nan,
                               int64_t* const* d_counters, int n_counters, float* d_loss, void* stream);
int fr_modal_head_bwd(const float* d_enc, const float* d_query, const int64_t* d_ids, const int64_t* d_num,
                      int64_t pad_id, int64_t n_items, int L, const float* const* d_ln, float eps, const float* d_rows,
                      const float* d_labels, int H, const float* const* d_mlp, float kd_threshold, float w_health,
                      float w_kd, const float* d_out, const float* d_gh, const float* d_gk, float* d_denc,
                      float* d_dquery, float* d_drows, float* d_partials, int64_t partial_floats, void* stream);
int fr_modal_head_reduce(const float* d_partials, int64_t n_items, float* d_grad, void* stream);

/* ------------------------------------------------------------------------------------------
 * Fused modal fusion of HealthRec (models/cikm_model.py:245-249 with target_attention_layer,
 * :311-369), per item i of the 2B batch items:
 *   item_health = target_attention(Q_i, E_i, E_i, key mask ids_i == pad_id)   (mm_target_atten)
 *   item_mm     = target_attention(E_i, Q_i, Q_i)                            (ingre_target_atten)
 *   know[i]     = F.normalize(item_mm, dim=1).sum(1) / num[i]
 *   hin[i]      = F.normalize(item_health, dim=1).mean(1)        (input of the health MLP)
 * target_attention: 2 heads of 32 (chunk/cat), LayerNorm(32, eps) on the q and k heads, scores
 * q k^T / sqrt(32), padded keys -> -(2^32 - 1), softmax, @ v.  d_enc [n, L, 64] (encoder output),
 * d_query [n, 2, 64] (image / text projections), d_ids [n, L] int64, d_num [n] int64;
 * d_ln: 4 device pointers {mm_target_atten.ln.weight, .bias, ingre_target_atten.ln.weight, .bias}
 * (both with the same eps).  L in {4, 5, 8, 10, 16, 20}.
 * Backward recomputes the forward and writes d_denc, d_dquery and d_dln (float [4][32]: the four
 * LayerNorm parameter gradients, block partials in d_partials summed in block order).
 * ------------------------------------------------------------------------------------------ */
int64_t fr_modal_fusion_partials(int64_t n_items);
int fr_modal_fusion_fwd(const float* d_enc, const float* d_query, const int64_t* d_ids, const int64_t* d_num,
                        int64_t pad_id, int64_t n_items, int L, const float* const* d_ln, float eps, float* d_know,
                        float* d_hin, void* stream);
int fr_modal_fusion_bwd(const float* d_enc, const float* d_query, const int64_t* d_ids, const int64_t* d_num,
                        int64_t pad_id, int64_t n_items, int L, const float* const* d_ln, float eps,
                        const float* d_dknow, const float* d_dhin, float* d_denc, float* d_dquery, float* d_dln,
                        float* d_partials, int64_t partial_floats, void* stream);

/* ------------------------------------------------------------------------------------------
 * Fused health / KD loss head of HealthRec (models/cikm_model.py:249-264,304-308), over n items:
 *   out[0] = w_health * sum BCE(sigmoid(W2 relu(W1 hin + b1) + b2), labels)      (health_mlp, BCELoss)
 *   out[1] = w_kd * max(0, 1 - mean_i cos(know_i, rows_i) - kd_threshold)          (norm_loss of KD)
 *   out[2] = 1 - mean cos - kd_threshold (saved for the backward's gate)
 * d_hin/d_know/d_rows [n, 64] (rows = item_all[pos; neg]), d_labels [n, H] float, H <= 16,
 * d_mlp = {W1 [64,64], b1 [64], W2 [H,64], b2 [H]} (nn.Linear layout).  The forward writes d_out
 * from block partials summed in block order by the last block (d_partials from
 * fr_health_kd_partials(n, 0), zero-filled once before first use; the kernel re-zeroes its ticket).
 * The ticket is word 0 of d_partials.  The backward takes the upstream gradients of out[0] / out[1] as device scalars and writes
 * d_dhin, d_dknow, d_drows and d_dmlp = {dW1, db1, dW2, db2} (block partials, block order).
 * ------------------------------------------------------------------------------------------ */
int64_t fr_health_kd_partials(int64_t n_items, int backward);
int fr_health_kd_fwd(const float* d_hin, const float* d_know, const float* d_rows, const float* d_labels,
                     int64_t n_items, int H, const float* const* d_mlp, float kd_threshold, float w_health,
                     float w_kd, float* d_out, float* d_partials, int64_t partial_floats, void* stream);
int fr_health_kd_bwd(const float* d_hin, const float* d_know, const float* d_rows, const float* d_labels,
                     int64_t n_items, int H, const float* const* d_mlp, float kd_threshold, float w_health,
                     float w_kd, const float* d_out, const float* d_gh, const float* d_gk, float* d_dhin,
                     float* d_dknow, float* d_drows, float* const* d_dmlp, float* d_partials,
                     int64_t partial_floats, void* stream);

/* ------------------------------------------------------------------------------------------
 * Modal projections over gathered feature rows (image_trs / text_trs of HealthRec,
 * models/cikm_model.py:240-241: Linear(K -> 64) applied to embImage / embText rows of the batch items).
 * fr_gather_linear_fwd: Y[i, 0:64] = X[ids[i], 0:K] W^T + b  (W [64, K] nn.Linear layout, b may be
 *   NULL, Y rows at stride ldy: the two modalities write one [n, 2, 64] query tensor).  K a multiple of
 *   16, X rows / W 16-byte aligned.  Deterministic.
 * fr_rows_matmul: out[i, 0:K] = S[i, 0:64] W  -- the table gradient of a gathered Linear input as
 *   (per-id sum of dY rows) x W (the compact rows of fr_embedding_rowgrad on dY), instead of scattering
 *   dX = dY W (replaces the index backward of embImage[ids] feeding image_trs).
 * fr_linear_wgrad_gather: fr_linear_wgrad with X row m read from X[ids[m]] (dW = dY^T X[ids]).
 * ------------------------------------------------------------------------------------------ */
int fr_gather_linear_fwd(const int64_t* d_ids, int64_t n, const float* d_x, int64_t ldx, int K, const float* d_w,
                         const float* d_b, float* d_y, int64_t ldy, void* stream);
int fr_rows_matmul(const float* d_s, int64_t lds, int64_t n, const float* d_w, int K, float* d_out, int64_t ldo,
                   void* stream);
int fr_linear_wgrad_gather(const float* d_dy, int64_t ldy, const int64_t* d_ids, const float* d_x, int64_t ldx,
                           int64_t M, int N, int K, float* d_dw, int64_t ldw, float* d_db, void* d_workspace,
                           int64_t workspace_bytes, void* stream);
/* The same three for several tables (<= 4) at the same ids in one launch each (blockIdx.z = table):
 * HealthRec's image and text projections share the batch's item ids.
 *   fr_gather_linear_fwd_multi: table t writes Y[i, 64 t .. 64 t + 64) (ldy >= 64 n_tab); d_b may be NULL
 *     (or hold NULL entries);
 *   fr_rows_matmul_multi: out_t[i, 0:K_t] = S[i, 64 t .. 64 t + 64) W_t (lds >= 64 n_tab);
 *   fr_linear_wgrad_gather_multi: dW_t = dY_t^T X_t[ids], db_t = colsum dY_t, dY_t = columns
 *     [N t, N t + N) of dY; workspace fr_linear_wgrad_gather_multi_workspace(M, N, n_tab, K).
 * Host arrays of per-table pointers / sizes; results bit-identical to the per-table calls. */
int fr_gather_linear_fwd_multi(const int64_t* d_ids, int64_t n, int n_tab, const float* const* d_x, const int64_t* ldx,
                               const int* K, const float* const* d_w, const float* const* d_b, float* d_y, int64_t ldy,
                               void* stream);
int fr_rows_matmul_multi(const float* d_s, int64_t lds, int64_t n, int n_tab, const float* const* d_w, const int* K,
                         float* const* d_out, const int64_t* ldo, void* stream);
int64_t fr_linear_wgrad_gather_multi_workspace(int64_t M, int N, int n_tab, const int* K);
int fr_linear_wgrad_gather_multi(const float* d_dy, int64_t ldy, const int64_t* d_ids, int64_t M, int N, int n_tab,
                                 const float* const* d_x, const int64_t* ldx, const int* K, float* const* d_dw,
                                 const int64_t* ldw, float* const* d_db, void* d_workspace, int64_t workspace_bytes,
                                 void* stream);

/* ------------------------------------------------------------------------------------------
 * Ingredient gather + EmbLoss norms of its two halves (models/cikm_model.py:230, 270-279).
 * fr_gather_norms_fwd: E[i] = W[ids[i]] (64-wide fp32 rows) and nrm[0] = ||E[:half]||_F,
 *   nrm[1] = ||E[half:]||_F (block partials from fr_gather_norms_partials, fixed-order sums).
 * fr_norms_bwd_coef: out[i] = G[i] + [ids[i] != pad] * (gn[h] / nrm[h]) * E[i], h = (i >= half),
 *   gn[1] read at d_gn + gn_stride (0 for a broadcast gradient); zero where a norm is zero.
 * fr_gather_norms_fwd with d_nrm NULL leaves the norms' finalize to fr_reg_combine_norms_fwd: the same
 *   fixed-order sums (bit-identical nrm) plus, when d_out is given, HealthRec's EmbLoss assembly
 *   d_out[0] = w * (d_a[0] + (nrm[0] + nrm[1]) / B) (fr_reg_combine_fwd's arithmetic) in one launch,
 *   issued where the loss needs it instead of before the encoder.  n = the gather's row count.
 * ------------------------------------------------------------------------------------------ */
int64_t fr_gather_norms_partials(int64_t n);
int fr_gather_norms_fwd(const int64_t* d_ids, int64_t n, int64_t half, const float* d_w, int64_t ldw, float* d_e,
                        float* d_partials, int64_t partial_floats, float* d_nrm, void* stream);
int fr_norms_bwd_coef(const int64_t* d_ids, int64_t n, int64_t half, int64_t pad, const float* d_g, const float* d_e,
                      const float* d_gn, int64_t gn_stride, const float* d_nrm, float* d_out, void* stream);
int fr_reg_combine_norms_fwd(const float* d_a, const float* d_partials, int64_t n, float B, float w, float* d_nrm,
                             float* d_out, void* stream);
/* fr_norms_bwd_coef's rows scattered with fr_embedding_bwd_atomic's float atomics in one launch:
 * d_out[ids[i]] += G[i] + [ids[i] != pad] (gn[h] / nrm[h]) E[i] for ids in [0, num_rows), the
 * hot_row's positions pre-summed per workgroup (HealthRec's deferred ingredient rows, added into the
 * RI backward's d ingre: cikm_model.py:230 + 270-279).  G, E: [n, 64] dense fp32. */
int fr_norms_bwd_scatter(const int64_t* d_ids, int64_t n, int64_t half, int64_t pad, const float* d_g,
                         const float* d_e, const float* d_gn, int64_t gn_stride, const float* d_nrm, int64_t num_rows,
                         int64_t hot_row, float* d_out, int64_t ldo, void* stream);

/* ------------------------------------------------------------------------------------------
 * Host-side readers of the reference's on-disk interaction formats (no GPU).
 *   FR_IO_NEGATIVE  data.{valid,test}.negative: "(u,i)\tn1\tn2..." per line; the first field is
 *                   dropped, the rest are int() ids -> ragged rows (values, offsets[rows+1]).
 *                   Replaces InteractionData.load_negative_file (utils/dataset.py:245-256).
 *   FR_IO_RATING    data.{train,valid,test}.rating: "u\ti\trating..." -> values[rows][2] = (u, i),
 *                   aux[rows] = float(rating) (NaN when the line has no third field; aux may be
 *                   NULL).  Replaces the int(arr[0]), int(arr[1]), float(arr[2]) parses of
 *                   utils/dataset.py:93-176.
 * fr_io_open maps the file and counts rows / values in parallel byte ranges cut at line starts;
 * the caller allocates; fr_io_fill parses into its arrays (FR_EPARSE + the 1-based line of the
 * first malformed field, as the reference's int()/float() would raise); fr_io_close unmaps.
 * threads <= 0: min(hardware threads, 16), and at least 4 MB of text per thread.
 * ------------------------------------------------------------------------------------------ */
enum fr_io_mode { FR_IO_NEGATIVE = 0, FR_IO_RATING = 1 };
typedef struct fr_io_table fr_io_table;
int fr_io_open(const char* path, int mode, int threads, fr_io_table** table, int64_t* rows, int64_t* values);
int fr_io_fill(fr_io_table* table, int64_t* values, int64_t* offsets, double* aux, int64_t* bad_line);
void fr_io_close(fr_io_table* table);

/* Evaluation candidates of EvalByUserDataloader (utils/dataloader.py:228-302), host arrays:
 * fr_io_remove_positives: for each user u and each positive p of pos[pos_off[u]:pos_off[u+1]] in
 *   order, clears alive[] of the first still-alive occurrence of p in neg[neg_off[u]:neg_off[u+1]]
 *   (list.remove in place; the mask persists, so repeated evaluations see the reference's mutated
 *   lists); lens[u] = |pos_u| + alive negatives of u, *total = sum(lens).
 * fr_io_candidates: out_items[cand_off[u]:] = pos_u followed by the alive negatives of u in file
 *   order, out_users[...] = users[u]  (items = pos + neg).  cand_off = exclusive prefix of lens. */
int fr_io_remove_positives(const int64_t* neg, const int64_t* neg_off, uint8_t* alive, const int64_t* pos,
                           const int64_t* pos_off, int64_t n_users, int64_t* lens, int64_t* total, int threads);
int fr_io_candidates(const int64_t* neg, const int64_t* neg_off, const uint8_t* alive, const int64_t* pos,
                     const int64_t* pos_off, const int64_t* users, int64_t n_users, const int64_t* cand_off,
                     int64_t* out_users, int64_t* out_items, int threads);

/* ------------------------------------------------------------------------------------------
 * fr_spmm_csr_ex: fr_spmm_csr over split row tables, a column mask and a row list.
 *   fr_tab      rows [0, split) at lo (stride ld_lo), rows [split, n) at hi (stride ld_hi, row r at
 *               hi + (r - split) * ld_hi); hi == NULL: every row at lo.  X, Y1, Y2, A1, A2 may each
 *               be split (one split row for the call).  HealthRec's propagation reads its ego table
 *               as [user_embedding ; item_ir] / [item_embedding ; ingre_embedding[:-1]] and writes
 *               its gradient into the tables' own buffers: the torch.cat / split / slice glue of
 *               cikm_model.py:185-199 (and of their backward) disappears.
 *   d_col_mask  optional uint8 per X row: edges to a row with mask 0 are skipped (X known zero
 *               there: the backward of a propagation evaluated at a few rows).
 *   rows        optional fr_rowlist: only the listed rows (ids[k][i] + off[k]) are computed, one
 *               workgroup per listed row (d = 64; deterministic, equal to the full launch's row to
 *               fp32 rounding); the other rows of Y are not written.  The training step needs the UI propagation only
 *               at the batch's users and items (cikm_model.py:255-261): 3B rows instead of U + I.
 *   d_a1_gate   optional uint8 per output row: A1's row r is read only where a1_gate[r] != 0 and
 *               counts as zero elsewhere (A1 = the upstream gradient itself, valid only at the
 *               marked rows: no zero fill of the rest of it is needed).
 * fr_rows_mark: mask[ids[k][i] + off[k]] = value (sets / clears a column mask from a row list).
 * fr_rows_mark_zero: the same, and rows ids[k][i] + off[k] of Z ([*, d], stride ldz) set to 0
 *               (the batch rows of an upstream gradient about to be accumulated into); with
 *               d_bits, also bit (row & 31) of d_bits[row >> 5] set (value != 0) or cleared.
 * fr_spmm_sparse_upstream: Y2 = alpha * A X + beta1 * gate(X), d = 64, for an X that is non-zero
 *               only at the rows whose bit is set in d_bits (ceil(n_rows / 32) words): X is read
 *               only there, gate(X) = X at marked rows and 0 elsewhere.  One workgroup per 64 rows
 *               scans its edge range against the bitmask (staged in LDS up to 32,768 rows, read
 *               from L2 beyond) and gathers only the marked columns; every row of Y2 (split at
 *               `split`) is written.
 *               The summation order of a row's hits is run-to-run variable (LDS float atomics):
 *               the deterministic mode uses fr_spmm_csr_ex with d_col_mask / d_a1_gate instead.
 * ------------------------------------------------------------------------------------------ */
typedef struct fr_tab {
  const float* lo;
  int64_t ld_lo;
  const float* hi;
  int64_t ld_hi;
} fr_tab;
typedef struct fr_rowlist {
  const int64_t* ids[3];
  int64_t n[3];
  int64_t off[3];
} fr_rowlist;
int fr_spmm_csr_ex(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val, int64_t n_rows,
                   const fr_spmm_plan* plan, int64_t split, const fr_tab* X, int d, const fr_tab* Y1,
                   const fr_tab* Y2, float alpha, const fr_tab* A1, float beta1, const fr_tab* A2,
                   float beta2, const uint8_t* d_col_mask, const fr_rowlist* rows, const uint8_t* d_a1_gate,
                   void* d_workspace, int64_t workspace_bytes, void* stream);
/* fr_spmm_csr_range: fr_spmm_csr_ex (no mask, no row list) over output rows [row_lo, row_hi) only;
 * the other rows of Y1 / Y2 are not written.  For a bipartite graph whose rows [0, s) connect only
 * to [s, n) (HealthRec's RI graph, cikm_model.py:136-180 at :185-208): the last propagation layer
 * is needed at the item rows only and the first backward layer of an item-only upstream gradient
 * is non-zero at the ingredient rows only. */
int fr_spmm_csr_range(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val, int64_t n_rows,
                      const fr_spmm_plan* plan, int64_t split, const fr_tab* X, int d, const fr_tab* Y1,
                      const fr_tab* Y2, float alpha, const fr_tab* A1, float beta1, const fr_tab* A2, float beta2,
                      int64_t row_lo, int64_t row_hi, void* d_workspace, int64_t workspace_bytes, void* stream);
/* Device-built row lists (HealthRec's RI forward evaluated at the item rows its UI layer reads):
 * fr_rows_frontier marks, in d_mark [I] (4-B aligned; zero on entry, left zero), the item columns (U + i) of the
 *   batch users' rows of a [users | items] CSR and the batch items p, n, then writes them to d_list and
 *   their number to d_count (order arbitrary).  Two launches.
 * fr_spmm_csr_list: fr_spmm_csr_ex's epilogue (split tables, Y1 / Y2 / A1 / A2) for the rows
 *   d_list[0 .. *d_count) only (the count read on the device; max_rows bounds it for the grid), d = 64,
 *   rows bit-identical to the full launch's. */
int fr_rows_frontier(const int64_t* d_rowptr, const int32_t* d_col, int64_t U, int64_t I, const int64_t* d_u,
                     const int64_t* d_p, const int64_t* d_n, int64_t B, uint8_t* d_mark, int32_t* d_list,
                     int32_t* d_count, void* stream);
int fr_spmm_csr_list(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val, int64_t n_rows, int64_t split,
                     const fr_tab* X, const fr_tab* Y1, const fr_tab* Y2, float alpha, const fr_tab* A1, float beta1,
                     const fr_tab* A2, float beta2, const int32_t* d_list, const int32_t* d_count, int64_t max_rows,
                     void* stream);
/* fr_spmm_list_scatter: Y[c - split] += alpha * A[r][c] * X[r] over the listed rows r (d_list[0 ..
 *   *d_count), max_rows bounds it) and their columns c >= split; zero_first: Y's n_rows - split rows
 *   set to 0 first (same stream).  For a SYMMETRIC adjacency and an X zero outside the list this is
 *   Y = alpha * (A X)[split:], the side rows of a transpose product at cost proportional to the listed
 *   rows' degrees (HealthRec's RI backward, first launch of the bipartite two-layer form,
 *   cikm_model.py:185-208).  Float atomics: summation order unspecified.  X: fp32 [*, 64] (ldx),
 *   Y: fp32 [n_rows - split, 64] (ldy), not aliasing X. */
int fr_spmm_list_scatter(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val, int64_t n_rows,
                         int64_t split, const int32_t* d_list, const int32_t* d_count, int64_t max_rows,
                         const float* d_X, int64_t ldx, float* d_Y, int64_t ldy, float alpha, int zero_first,
                         void* stream);
int fr_rows_mark(uint8_t* d_mask, const fr_rowlist* rows, uint8_t value, void* stream);
int fr_rows_mark_zero(uint8_t* d_mask, const fr_rowlist* rows, uint8_t value, float* d_Z, int64_t ldz, int d,
                      uint32_t* d_bits, void* stream);
/* fr_spmm_scatter_upstream: fr_spmm_sparse_upstream's result for a SYMMETRIC adjacency (HealthRec's UI
 * graph, cikm_model.py:136-180) by scattering from the listed rows' own CSR rows: Y2 = alpha A X +
 * beta1 gate(X), X non-zero only at the rows of `rows` (mask[r] != 0 and bit r set in d_bits).
 * Work proportional to the listed rows' degrees; the first occurrence of each row claims it by
 * clearing its bit (d_bits is clear for the listed rows on return).  Float-atomic summation order. */
int fr_spmm_scatter_upstream(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val, int64_t n_rows,
                             const uint8_t* d_mask, uint32_t* d_bits, const fr_rowlist* rows, const float* d_X,
                             int64_t ldx, int64_t split, const fr_tab* Y2, float alpha, float beta1, void* stream);
/* fr_spmm_sparse_upstream over a rectangular slice [n_rows x n_cols] (the row-sharded config-4
 * step's A_ui / A_iu, engine/sharded.py): the bitmask (ceil(n_cols / 32) words, read from L2) marks
 * the non-zero rows of X (the slice's columns); A1 is read at every output row (no gate). */
int fr_spmm_sparse_upstream_rect(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val, int64_t n_rows,
                                 int64_t n_cols, const uint32_t* d_bits, const float* d_X, int64_t ldx,
                                 const fr_tab* Y2, float alpha, const fr_tab* A1, float beta1, void* stream);
int fr_spmm_sparse_upstream(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val, int64_t n_rows,
                            const uint32_t* d_bits, const float* d_X, int64_t ldx, int64_t split, const fr_tab* Y2,
                            float alpha, const fr_tab* A1, float beta1, void* stream);
/* Either of the two above over an edge-balanced row-block plan (engine ops._sparse_plan, built once
 * per adjacency): block b = (row_lo, row_hi, edge_lo, edge_hi) in d_blocks[4b .. 4b+3], at most 64
 * rows of a bounded edge count, or one chunk of a heavy row (a Zipf item row of config 4's 10M x 1M
 * graph has up to 434k edges; with uniform 64-row blocks its workgroup scans them alone).  Chunks add
 * into their row atomically after the rows in d_split_rows got their own term (beta1 * gate(A1)).
 * ungated = 1: the rectangular form (bitmask over n_cols, A1 at every row); 0: the square gated form
 * (split tables at `split`).  The sparse-upstream backward of lightgcn.py:134-147's propagation
 * (ops.propagate_rows) and of the row-sharded step (engine/sharded.py). */
int fr_spmm_sparse_upstream_blocks(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val, int64_t n_rows,
                                   int64_t n_cols, int ungated, const uint32_t* d_bits, const float* d_X, int64_t ldx,
                                   int64_t split, const fr_tab* Y2, float alpha, const fr_tab* A1, float beta1,
                                   const int64_t* d_blocks, int64_t n_blocks, const int64_t* d_split_rows,
                                   int64_t n_split_rows, void* stream);
/* fr_spmm_sparse_upstream / fr_spmm_sparse_upstream_blocks with a side job: the launch also zeroes
 * d_zero[0 .. zero_floats) (16-B aligned, a multiple of 4 floats) -- the region the next kernel on the
 * stream accumulates into (HealthRec's d ingre rows before the RI backward's list scatter), folded
 * into this launch instead of a memset node of its own. */
int fr_spmm_sparse_upstream_zero(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val, int64_t n_rows,
                                 const uint32_t* d_bits, const float* d_X, int64_t ldx, int64_t split,
                                 const fr_tab* Y2, float alpha, const fr_tab* A1, float beta1, float* d_zero,
                                 int64_t zero_floats, void* stream);
int fr_spmm_sparse_upstream_blocks_zero(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val,
                                        int64_t n_rows, int64_t n_cols, int ungated, const uint32_t* d_bits,
                                        const float* d_X, int64_t ldx, int64_t split, const fr_tab* Y2, float alpha,
                                        const fr_tab* A1, float beta1, const int64_t* d_blocks, int64_t n_blocks,
                                        const int64_t* d_split_rows, int64_t n_split_rows, float* d_zero,
                                        int64_t zero_floats, void* stream);
/* Rows per block of the sparse-upstream kernel (its LDS row accumulator): a plan block of more rows,
 * rows outside [0, n_rows) or an edge range outside its rows is refused by the kernel (the block
 * computes nothing) and flagged in the library's plan status. */
int fr_spmm_sparse_block_rows(void);
/* The plan status the sparse-upstream kernel sets (0: every block was valid; bit 0: a block of more
 * than fr_spmm_sparse_block_rows() rows or outside the adjacency; bit 1: a block whose edge range
 * leaves its rows), cleared when clear != 0.  Synchronous (a device symbol read): not inside graph
 * capture. */
int fr_spmm_plan_status(int clear);

/* fr_graph_bpr_finish: the tail of HealthRec's fused propagation + BPR backward (engine
 * ops.graph_bpr), after both propagation backwards have written dUe (user_embedding's gradient)
 * and dIe (item_embedding's):
 *   mask[u_b] = mask[U + p_b] = mask[U + n_b] = 0   (clears the column mask; d_mask may be NULL;
 *     with d_bits, the same rows' bits of that bitmask cleared too),
 *   dUe[u_b] += r_u Ue[u_b], dIe[p_b] += r_p Ie[p_b], dIe[n_b] += r_n Ie[n_b]   (float atomics)
 *     with r_x = g_reg * d_greg[0] / B / ||.||_F of block x (the norms fr_bpr_fwd left in the
 *     workspace): EmbLoss(u_ego, pos_ego, neg_ego)'s gradient, cikm_model.py:273-279;
 *   d_zero[0 .. zero_n) = 0   (ingre_embedding's padding row, not a graph node).
 * d_dUe / d_dIe may be NULL (that table's rows skipped: CLUSSL adds the item rows later, into the
 * item views' gradient, with a second call that has d_dUe and d_mask NULL).
 * One launch instead of three (unmark, EmbLoss scatter, padding-row fill). */
int fr_graph_bpr_finish(uint8_t* d_mask, int64_t U, const float* d_Ue, int64_t ldue, const float* d_Ie,
                        int64_t ldie, const int64_t* d_u, const int64_t* d_p, const int64_t* d_n, int64_t B,
                        int d, float g_reg, const float* d_greg, float* d_dUe, float* d_dIe,
                        float* d_zero, int zero_n, uint32_t* d_bits, void* d_workspace, int64_t workspace_bytes,
                        void* stream);

/* ------------------------------------------------------------------------------------------
 * fr_feed_batch: one step's batch in one launch.  Replaces TrainDataLoader.__getitem__ x B +
 * default_collate (utils/dataloader.py:50-115) as the engine stages them on the device.
 *   feed mode (d_perm != NULL): triple i of batch *d_cursor (device) of the staged epoch:
 *     k = perm[cursor * B + i];  u[i] = users[k];  p[i] = items[k];  n[i] = negs[cursor * B + i]
 *     (the cursor is not advanced here);
 *   plain mode: p, n are inputs.
 *   Both: rows j of [p ; n]: pn[j], out_codes[j] = codes[pn[j]] ([L] int64), out_nums[j],
 *   out_health[j] = health[pn[j]] ([H] float, optional: H = 0 and NULLs), out_kpm[j][c] =
 *   -inf where out_codes[j][c] == pad, else 0 (optional: HealthRec's key-padding mask,
 *   cikm_model.py:231-232, in the additive float form the encoder layer consumes).
 *   An item id outside [0, n_items) is replaced by 0 in every output (p / n included) and sets the
 *   sticky device flag *d_err = 1 (optional: NULL) that the trainer checks at epoch end.
 * ------------------------------------------------------------------------------------------ */
int fr_feed_batch(const int64_t* d_perm, const int64_t* d_users, const int64_t* d_items, const int64_t* d_negs,
                  const int64_t* d_cursor, int64_t B, int64_t* d_u, int64_t* d_p, int64_t* d_n,
                  const int64_t* d_codes, int L, const int64_t* d_nums, const float* d_health, int H,
                  int64_t n_items, int64_t pad, int64_t* d_pn, int64_t* d_out_codes, int64_t* d_out_nums,
                  float* d_out_health, float* d_out_kpm, int32_t* d_err, void* stream);

/* fr_step_book: the training loop's per-step loss bookkeeping (common/trainer.py:183-193) on the
 * device: acc[i] (+)= (double)*parts[i] for the n (<= 8) scalar loss components,
 * *nan |= isnan(sum of the parts in fp32, left to right), and each of the n_counters (<= 8) device
 * int64 step counters += 1 (dropout-hash step counters, the device feed's batch cursor), and, when
 * d_loss_out is not NULL, *d_loss_out = that fp32 sum (the loss the step returns,
 * common/trainer.py:225).  One launch, no host sync. */
int fr_step_book(const float* const* d_parts, int n, double* d_acc, int accumulate, int32_t* d_nan,
                 int64_t* const* d_counters, int n_counters, float* d_loss_out, void* stream);

/* ------------------------------------------------------------------------------------------
 * fr_rank_metrics: the per-user ranking of Trainer._valid_by_user_epoch (common/trainer.py:231-282;
 * metrics_by_user / get_auc_fast :49-69) over EvalByUserDataloader's candidate lists
 * (utils/dataloader.py:228-302).  User u's candidate scores are d_scores[d_offsets[u] ..
 * d_offsets[u+1]), its first d_npos[u] candidates the positives.  Outputs per user:
 *   d_hits[u]  bit t (t < k) = rank t of np.argsort(scores)[::-1] is a positive;
 *   d_auc[u]   sum over positives p of #{negatives j: score[j] < score[p]} (strict);
 *   d_flags[u] 0 = exact, 1 = the k+1 largest scores tie or a score is NaN (numpy's tie order
 *              decides: rank on the host), 2 = more than fr_rank_capacity() candidates.
 * k <= 31.  One launch, one wave per user, no host sync. */
/* fr_score_segments: the evaluation's candidate scores without materialised gathers --
 * d_out[e] = dot(d_user[d_uid[s]], d_item[d_items[e]]) for e in [d_offsets[s], d_offsets[s + 1]),
 * s < n_seg (HealthRec / CLUSSL / LightGCN inference_fast, cikm_model.py:294-302, over
 * EvalByUserDataloader's per-user lists, dataloader.py:228-302).  d = 64; row strides in floats. */
int fr_score_segments(const float* d_user, int64_t ld_user, const float* d_item, int64_t ld_item,
                      const int64_t* d_uid, const int64_t* d_offsets, int64_t n_seg, const int64_t* d_items, int d,
                      float* d_out, void* stream);
int fr_rank_metrics(const float* d_scores, const int64_t* d_offsets, const int32_t* d_npos, int64_t n_users,
                    int k, uint32_t* d_hits, int64_t* d_auc, uint8_t* d_flags, void* stream);
int fr_rank_capacity(void);

/* fr_reg_combine_fwd / _bwd: HealthRec's weighted EmbLoss from its two fused pieces,
 * out = w * (a[0] + (b[0] + ... + b[nb-1]) / B)  (cikm_model.py:267-279); backward da = g w,
 * db[i] = g w / B.  One launch each. */
int fr_reg_combine_fwd(const float* d_a, const float* d_b, int nb, float B, float w, float* d_out, void* stream);
int fr_reg_combine_bwd(const float* d_g, int nb, float B, float w, float* d_da, float* d_db, void* stream);

/* ------------------------------------------------------------------------------------------
 * RCCL communicator (SURVEY 8(b) fr_comm_init / fr_allreduce_f32; new work: the reference is
 * single-process, utils/configurator.py:110-114).  One communicator per process and GPU (the
 * calling thread's current HIP device); collectives are stream-ordered on the caller's stream.
 * Replaces, for a host that binds only this ABI, the torch.distributed (backend "nccl" = RCCL)
 * calls of engine/sharded.py (per-layer item all-reduce, _all_reduce) and engine/dist.py (dense
 * gradient all-reduce, GradAllReduce.communicate_dense; row all-gather, RowExchange.exchange).
 *   fr_comm_available      1 if an RCCL library could be resolved (the process's own copy first)
 *   fr_comm_unique_id      rank 0 draws the 128-byte id (fr_comm_unique_id_bytes) and ships it to
 *                          the other ranks out of band (a TCP store, a file, MPI ...)
 *   fr_comm_init           ncclCommInitRank (collective over the world's ranks)
 *   fr_allreduce_f32       in-place float sum of n elements
 *   fr_allgather_f32       recv[world * n] = every rank's send[n], in rank order
 *   fr_comm_destroy        frees the communicator (NULL is a no-op)
 * FR_ENOTSUP when no RCCL library is present; RCCL failures -> FR_EHIP + fr_last_error.
 * ------------------------------------------------------------------------------------------ */
int fr_comm_available(void);
int64_t fr_comm_unique_id_bytes(void);
int fr_comm_unique_id(void* out, int64_t out_bytes);
int fr_comm_init(int rank, int world, const void* unique_id, void** comm);
int fr_allreduce_f32(void* comm, float* buf, int64_t n, void* stream);
int fr_allgather_f32(void* comm, const float* send, float* recv, int64_t n, void* stream);
int fr_comm_destroy(void* comm);

#ifdef __cplusplus
}
#endif
#endif /* FR_ENGINE_H */
