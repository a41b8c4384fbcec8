/* mlpgpu.h -- C ABI of libmlpgpu, the MI355X (gfx950) pairwise-posterior and
 * consistency engine that replaces the hot path of kuangmeng/MLProbs'
 * baseMSA/C_P_NP_Aln.
 *
 * The reference has no library boundary on this path: its pair loop calls
 * C++ member functions of a shared ProbabilisticModel from OpenMP threads and
 * keeps heap-allocated SparseMatrix objects.  Each entry
 * point below names the reference code it replaces.  Plain pointers and sizes
 * only; no C++ or torch types cross this boundary.
 *
 * Conventions
 *  - A family is n sequences of uppercase letters 'A'..'Z' (gaps stripped,
 *    as after MultiSequence::LoadMFA(..., true), CPNP/MSA.cpp:136).
 *  - Pair index p enumerates (a, b), a < b, row-major: the order of the
 *    reference's seqsPairs table (CPNP/MSA.cpp:907-919).
 *  - The posterior of pair p is the sparse matrix sparseMatrices[a][b]
 *    (CPNP/MSA.cpp:1023-1025): rows = residues 1..L_a of a, 1-based columns
 *    of b, entries >= 0.01 (CPNP/SparseMatrix.h:14), columns ascending.
 *  - Sparse set layout ("canonical CSR"): for pair p, row_ptr has L_a + 2
 *    int32 entries at row offset R(p) = sum_{q<p} (L_{a_q} + 2); row i
 *    (1..L_a) spans pair-local entries [row_ptr[i], row_ptr[i+1]);
 *    row_ptr[0] = row_ptr[1] = 0.  Entries of all pairs are concatenated
 *    in pair order; ent_off[p] is the first entry of pair p, ent_off[P]
 *    the total.  Columns are uint16 (L <= 65535), values float.
 *  - Every call returns MLP_OK (0) or an error code; never exit().
 *    mlp_last_error() gives a message.  One context per host thread.
 */
#ifndef MLPGPU_H
#define MLPGPU_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MLP_OK 0
#define MLP_ERR_ARG 1       /* bad argument */
#define MLP_ERR_HIP 2       /* HIP runtime / device error */
#define MLP_ERR_OVERFLOW 3  /* partition function overflow (reference: exit(1), CPNP/MSAPartProbs.cpp:547-589) */
#define MLP_ERR_STATE 4     /* call sequence error (e.g. no family loaded) */
#define MLP_ERR_COMM 5      /* RCCL error */
#define MLP_ERR_MEMORY 6    /* device allocation failed */

typedef struct mlp_ctx mlp_ctx;

/* Create a context bound to HIP device `device`. */
int mlp_ctx_create(int device, mlp_ctx **out);
/* A context that runs every stage below on the host CPU instead (host
 * threads, MLP_HOST_THREADS, at most 16) and never initialises the HIP
 * runtime: for families too small to pay for a device (runtime start-up and
 * teardown alone cost 0.2-0.4 s per process).  Same results, bit for bit:
 * the reference's own operation order, the partition function in x87 long
 * double like the reference.  Covers the C_P_NP_Aln entry points
 * (mlp_viterbi / mlp_model_adjustment / mlp_family_features, mlp_posteriors
 * with pid 0-4 and MLP_PID_NPDO, mlp_relax, the CSR calls) and QuickProbs'
 * posterior and consistency stages (mlp_posteriors with MLP_PID_QP,
 * mlp_relax_qp / mlp_relax_qp_selective, QuickProbs' plain double partition
 * function); the profile-posterior calls return MLP_ERR_STATE (callers fall
 * back to their host restatement). */
int mlp_ctx_create_host(mlp_ctx **out);
/* 1 for a host context. */
int mlp_ctx_is_host(const mlp_ctx *ctx);
/* A context that drives every GPU of `device_mask` (bit k = HIP device k;
 * devices that do not exist are ignored) from this one host thread (SURVEY.md
 * section 8b: "a ctx drives all GPUs in its mask").  For families of at least
 * 1e9 pair-cells mlp_posteriors over all pairs and the relaxation rounds are
 * split into contiguous pair ranges, one shard (child context) per device:
 * posteriors balanced by DP cells (mlp_shard_plan), consistency rounds by
 * estimated multiply-adds (mlp_relax_shard_plan); the shards' sparse sets are
 * all-gathered over xGMI (every shard pulls every other shard's new block on
 * its own copy streams, peer copies), so every shard holds the whole store
 * after each stage and round; the whole store is sent to the shards only
 * when it came another way (an unsharded stage, mlp_csr_import).  With 2-8
 * virtual shards on one GPU the results are bit-identical to one device
 * (tests/test_gpu_shards.py); runs over several physical GPUs are untested
 * (no multi-GPU box here).  Everything else runs on the first device. */
int mlp_ctx_create_mask(uint64_t device_mask, mlp_ctx **out);
/* Number of shards (0: one per device of the mask when the family is large
 * enough; k > 0: always k, spread round-robin over the mask's devices --
 * several "virtual" shards may share a GPU). */
int mlp_set_shards(mlp_ctx *ctx, int nshards);
/* Shards the next whole-family call would use (1 = single device). */
int mlp_shard_count(mlp_ctx *ctx);
void mlp_ctx_destroy(mlp_ctx *ctx);
const char *mlp_last_error(const mlp_ctx *ctx);
/* Device bytes the posterior stage may hold as batch scratch (default: the
 * device's free HBM less a reserve of max(16 GiB, 7%) for the store and the
 * relaxation, ~224 GiB on MI355X; larger batches shorten the per-batch
 * kernel tails).  A
 * one-shot process (the c_p_np_aln drop-in) asks for less: a fresh process's
 * large allocation waits while the driver clears memory another process just
 * released.  No reference counterpart (the reference allocates per pair). */
int mlp_set_scratch(mlp_ctx *ctx, uint64_t bytes);

/* Upload a family (replaces the sequence side of MultiSequence, CPNP/MultiSequence.h:267-315).
 * residues: concatenated uppercase letters; offsets[n+1] delimit sequence k. */
int mlp_family_load(mlp_ctx *ctx, int n, const char *residues, const int64_t *offsets);
int64_t mlp_family_npairs(const mlp_ctx *ctx);

/* Posterior stage for pairs [p_begin, p_end) in pair order.  Replaces the
 * body of the pdoAlign pair loop (CPNP/MSA.cpp:927-1032): per pid, the
 * 5-state + partition function + local posteriors merged by RMS (pid 0/1),
 * local only (pid 2) or partition function only (pid >= 3); the MEA distance
 * 1 - score / min(L_a, L_b); and the sparse matrix (>= 0.01).
 * pid | MLP_PID_NPDO replaces npdoAlign's ArrangePosteriorProbs loop
 * (CPNP/MSA.cpp:1636-1765) instead: the same models, the RMS terms summed in
 * its order (global, local, 5-state) and the distance score / #B, #B = the
 * match columns of the MEA path (CPNP/MSA.cpp:1744-1753).
 * delta = initDistrib[2] after ModelAdjustmentTest (CPNP/MSA.cpp:861-870).
 * pid = MLP_PID_QP runs QuickProbs' posterior stage instead (the realigner
 * MLProbs calls, PosteriorStage::computePairwise + combineMatrices,
 * QP/Alignment/Multiple/PosteriorStage.cpp:123-196): the same 5-state pair-HMM
 * and QuickProbs' double-precision VTML200 partition function, merged as
 * sqrt((a^2 + b^2) / 2), MEA distance, entries >= 0.01 stored as QuickProbs'
 * 16-bit fixed point q read back as q / 65535 (delta is ignored).
 * Results stay in device memory in the context's canonical CSR store. */
#define MLP_PID_QP 16
#define MLP_PID_NPDO 32
int mlp_posteriors(mlp_ctx *ctx, int pid, float delta, int64_t p_begin, int64_t p_end);

/* Per-pair scalars of pairs [p_begin, p_end) (host arrays, may be NULL):
 * distance, MEA score, nnz. */
int mlp_pair_results(mlp_ctx *ctx, int64_t p_begin, int64_t p_end, float *dist, float *mea,
                     int64_t *nnz);

/* Family test (replaces ModelAdjustmentTest / Alter_ModelAdjustmentTest,
 * CPNP/MSA.cpp:646-882): the Viterbi alignment of every pair
 * (CPNP/ProbabilisticModel.h:1043-1170).  mlp_viterbi runs pairs
 * [p_begin, p_end); keep_paths keeps every path on the host (needed by
 * mlp_family_features). */
int mlp_viterbi(mlp_ctx *ctx, int64_t p_begin, int64_t p_end, int keep_paths);
/* Per pair: identical residues in match columns and path length. */
int mlp_viterbi_results(mlp_ctx *ctx, int64_t p_begin, int64_t p_end, float *match, int32_t *len);
/* Path of pair p, forward order: 0 = 'B' (both), 1 = 'X', 2 = 'Y'. */
int mlp_viterbi_path(mlp_ctx *ctx, int64_t p, uint8_t *codes, int32_t *len);
/* ModelAdjustmentTest: average identity, its standard deviation, the
 * initDistrib[2] it selects and the returned code (variance_mean + class),
 * the per-pair identities summed in pair order. */
int mlp_model_adjustment(mlp_ctx *ctx, float *identity, float *variance, float *delta, int32_t *code);
/* Alter_ModelAdjustmentTest (the `-G` line): f = {identity, variance,
 * tmp_sp, peak_ratio, factor}, ints = {N, avg_len}, serial in pair order. */
int mlp_family_features(mlp_ctx *ctx, float theta, float *f, int32_t *ints);

/* Total entries of the canonical CSR store (all pairs currently held). */
int mlp_csr_total(mlp_ctx *ctx, int64_t *total);
/* Host copy of the full canonical CSR store (see layout above):
 * row_ptr: sum_p (L_a + 2) int32; ent_off: P + 1 int64; cols/vals: total. */
int mlp_csr_export(mlp_ctx *ctx, int32_t *row_ptr, int64_t *ent_off, uint16_t *cols, float *vals);
/* Replace the store with host data in the same layout (e.g. to relax a
 * sparse set computed elsewhere). */
int mlp_csr_import(mlp_ctx *ctx, const int32_t *row_ptr, const int64_t *ent_off,
                   const uint16_t *cols, const float *vals);

/* `iters` rounds of the consistency transformation over the whole store.
 * Replaces MSA::DoRelaxation x numConsistencyReps (CPNP/MSA.cpp:1041-1051,
 * 1119-1129, 1172-1360).  With a communicator (or in-process shards), each
 * rank relaxes the output pairs of its range from mlp_relax_shard_plan
 * (balanced by estimated multiply-adds) and the new store is all-gathered
 * after every round. */
int mlp_relax(mlp_ctx *ctx, int iters);
/* QuickProbs' consistency stage instead (ConsistencyStage::run / doRelaxation,
 * QP/Alignment/Multiple/ConsistencyStage.cpp:90-258), on a sparse set from
 * mlp_posteriors(MLP_PID_QP): default configuration (every z accepted by the
 * deterministic selectivity filter, self-weight 3), z weighted by
 * seq_weights[z] / W_xy, normalised by the weight sum; rounds re-sparsify at
 * 0.01 except the last (1e-5) into 16-bit fixed point.  iters < 0: QuickProbs'
 * default (2 rounds up to 50 sequences, else 1). */
int mlp_relax_qp(mlp_ctx *ctx, int iters, const float *seq_weights);
/* The same with QuickProbs' selectivity (ConsistencyStage.cpp:35-47, 171-205;
 * ExtendedMSA::doAlign, QP/Alignment/Multiple/ExtendedMSA.cpp:96-176): z is
 * accepted for (x, y) iff max(sel_dist[x][z], sel_dist[y][z]) <= selectivity
 * (the Deterministic filter), W_xy counts the accepted z only
 * (1 + (s - 1) A_xy / selectivity).  sel_dist: N x N host matrix, row-major
 * (QuickProbs passes the guide tree's subtree sizes with selectivity 200);
 * NULL accepts every z (= mlp_relax_qp). */
int mlp_relax_qp_selective(mlp_ctx *ctx, int iters, const float *seq_weights, const float *sel_dist,
                           float selectivity);

/* The weighted profile-profile posterior of QuickProbs' progressive
 * construction and refinement (ParallelProbabilisticModel::buildPosterior,
 * QP/Alignment/Multiple/ParallelProbabilisticModel.cpp:301-430) from the
 * device-resident sparse set (every pair; after mlp_relax_qp*): profile A
 * holds sequences labels1[0..n1) over L1 columns, B labels2[0..n2) over L2.
 * map1 / map2: per sequence of the profile, in order, its Sequence::getMapping
 * array (len + 1 entries: 0, then the column of each residue).  out receives
 * the dense (L1 + 1) x (L2 + 1) matrix, bit-identical to the reference's
 * (weights w_i w_j / sum in double, cast to float; terms in the reference's
 * order).  MLP_ERR_STATE when a row of L2 + 1 floats does not fit in LDS. */
int mlp_profile_posterior(mlp_ctx *ctx, const float *seq_weights, int n1, const int32_t *labels1, int L1,
                          const int32_t *map1, int n2, const int32_t *labels2, int L2, const int32_t *map2,
                          float *out);
/* C_P_NP_Aln's profile-profile posterior instead (ProbabilisticModel::
 * BuildPosterior, CPNP/ProbabilisticModel.h:1197-1379), cutoff 0: with
 * seq_weights (int, the guide tree's getSeqsWeights) the weighted form of
 * the progressive merges, w = (float)(w1 w2) / (float sum of w1 w2); NULL:
 * the unweighted form of refinement (terms += v).  Same layout, same
 * bit-identical term order. */
int mlp_profile_posterior_cpnp(mlp_ctx *ctx, const int32_t *seq_weights, int n1, const int32_t *labels1, int L1,
                               const int32_t *map1, int n2, const int32_t *labels2, int L2, const int32_t *map2,
                               float *out);
/* out = NULL: the matrix stays in a pinned host buffer of the context,
 * returned here and valid until the next mlp_profile_posterior* call. */
const float *mlp_profile_result(const mlp_ctx *ctx);

/* The profile posterior left on the device: with mlp_profile_defer(ctx, 1)
 * the mlp_profile_posterior* calls (out = NULL) skip the copy back (and
 * mlp_profile_result returns NULL); then
 *   mlp_profile_mea: the MEA alignment of that matrix (ComputeAlignment,
 *     ProbabilisticModel.h:804-864, ChooseBestOfThree ScoreType.h:347-366;
 *     QuickProbs' computeAlignment is the same recurrence), bit-identical
 *     score and path, computed on the device; path = 'B'/'X'/'Y' in forward
 *     order, capacity L1 + L2 bytes;
 *   mlp_profile_gather: vals[k] = matrix[cells[k]] (row-major (L2 + 1)).
 * mlp_profile_mea returns MLP_ERR_STATE (nothing written) when a strip of
 * the device pipeline gave up waiting for the one above (bounded spins);
 * the matrix is still on the device and the caller computes the MEA on the
 * host instead. */
int mlp_profile_defer(mlp_ctx *ctx, int on);
int mlp_profile_mea(mlp_ctx *ctx, char *path, int32_t *path_len, float *score);
int mlp_profile_gather(mlp_ctx *ctx, int64_t n, const int64_t *cells, float *vals);
/* A dense (L1 + 1) x (L2 + 1) posterior from the host (row-major, row 0 and
 * column 0 unused) made the context's device-resident matrix, as if a
 * deferred mlp_profile_posterior* had computed it: for callers that build
 * the profile posterior elsewhere, and for testing mlp_profile_mea on any
 * matrix.  Every entry must be finite and >= +0 (a posterior's range; the
 * device MEA's hand-off and choices rely on it): MLP_ERR_ARG otherwise.
 * MLP_ERR_STATE on a host context. */
int mlp_profile_set(mlp_ctx *ctx, int L1, int L2, const float *post);

/* Evaluation only (not a drop-in path): the consistency transform of the
 * output pairs (x, y), x in xs, y in ys, x < y, as dense 16x16 block
 * products on the fp32 matrix cores (v_mfma_f32_16x16x4_f32), from the
 * current store.  Fused products: held to the 1e-4 relative rule, not to bit
 * identity.  res[7] = {kernel seconds, dense MACs issued, outputs, max
 * relative error vs a double-precision sum on sampled cells, cells checked,
 * output tiles, operand blocks}. */
int mlp_relax_blockmfma_eval(mlp_ctx *ctx, int nx, const int32_t *xs, int ny, const int32_t *ys, double *res);

/* Multi-GPU (one process per GPU): RCCL over xGMI. */
int mlp_comm_unique_id(unsigned char id[128]);
int mlp_comm_init(mlp_ctx *ctx, const unsigned char id[128], int nranks, int rank);
/* This rank's contiguous pair range (cost-balanced split). */
int mlp_shard_range(mlp_ctx *ctx, int nranks, int rank, int64_t *p_begin, int64_t *p_end);
/* Host-only planning (no device needed; what mlp_shard_range and
 * mlp_allgather use).  mlp_shard_plan: contiguous pair range of `rank` for a
 * family with lengths lens[n], balanced by DP cells (L_a + 1)(L_b + 1).
 * mlp_gather_layout: info[3r..3r+2] = (p_begin, p_end, entries) of rank r;
 * checks that the ranges tile [0, npairs) in rank order and writes the
 * first global entry of every rank's block to ebase[nranks + 1]. */
int mlp_shard_plan(int n, const int32_t *lens, int nranks, int rank, int64_t *p_begin, int64_t *p_end);
int mlp_gather_layout(int nranks, int64_t npairs, const int64_t *info, int64_t *ebase);
/* Consistency-round sharding (host only): contiguous output-pair ranges
 * bounds[r] .. bounds[r + 1] of equal estimated work, sum_z nnz(x, z)
 * nnz(z, y) / L_z + (n - 2) nnz(x, y) per output pair (x, y), from the
 * current per-pair entry counts.  bounds: nranks + 1. */
int mlp_relax_shard_plan(int n, const int32_t *lens, const int64_t *pair_nnz, int nranks, int64_t *bounds);
/* After every rank ran mlp_posteriors on its shard (or mlp_relax_range on
 * its output range): all-gather the CSR store and the per-pair scalars so
 * every rank holds the whole family (RCCL grouped broadcasts of each rank's
 * block into its global place).  Without a communicator, or at one rank, a
 * no-op; MLP_TEST_ALLGATHER_FORCE=1 runs the grouped body at one rank too (the
 * test hook that exercises it on a one-GPU box). */
int mlp_allgather(mlp_ctx *ctx);
/* One C_P_NP_Aln consistency round (as mlp_relax, CPNP/MSA.cpp:1172-1360)
 * over the output pairs [r0, r1) only, from the whole store: the range one
 * rank computes when the caller does its own exchange (device or host
 * context).  Afterwards the context holds that range's block, entries from 0
 * (store range [r0, r1)), ready for mlp_allgather or the caller's exchange
 * plus mlp_csr_import. */
int mlp_relax_range(mlp_ctx *ctx, int64_t r0, int64_t r1);

/* The process's device memory pool (per device): contexts take their
 * large buffers (batch scratch, CSR store, relaxation and gather buffers)
 * from blocks the process keeps, and a destroyed context's buffers go back
 * to the pool, not to the driver -- a fresh allocation right after a large
 * release can wait seconds while the driver clears it, so a context created
 * after another (a new family, the shards of a mask) reuses its memory.
 * mlp_pool_info: bytes held in blocks and the part of them free;
 * mlp_pool_trim: blocks with nothing in use back to the driver (also done
 * automatically when an allocation fails). */
int mlp_pool_info(int device, uint64_t *held, uint64_t *free_bytes);
int mlp_pool_trim(int device);

/* Wait for all device work of the context. */
int mlp_synchronize(mlp_ctx *ctx);

/* Per-kernel device time accumulated since the last reset (HIP events on
 * the context stream), enabled by mlp_profile(ctx, 1).  One launch per
 * group and posterior batch; a group whose kernels run in parts (the local
 * totals: the forward chains beside the backward sweeps, the backward chains
 * after them) sums its parts' device time into that launch.  Kernel ids:
 * 0 forward, 1 backward, 2 local totals, 3 merge/MEA/sparsify, 4 compact,
 * 5 relax, 6 transpose, 7 filter, 8 allgather, 9 viterbi. */
#define MLP_NKERNELS 10
int mlp_profile(mlp_ctx *ctx, int enable);
int mlp_kernel_times(mlp_ctx *ctx, double *ms, int64_t *launches, int64_t *cells);
int mlp_profile_reset(mlp_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif
