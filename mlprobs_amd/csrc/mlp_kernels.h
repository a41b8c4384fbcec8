// mlp_kernels.h -- shared host/device declarations for the posterior and
// relaxation kernels (internal to libmlpgpu; not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "mlp_knobs.h"

namespace mlp {

constexpr int kWave = 64;        // CDNA wavefront
constexpr int kWavesPerBlock = 4;  // independent chains (waves) per workgroup
constexpr int kEll = 64;         // sparse slots per posterior row before overflow

// Chains.  One wave sweeps a chain of pairs whose rows are stacked: global
// row g of the chain is row i = g - row0[q] of member q.  Lane r owns rows
// g = r (mod 64) and walks them one after another, W steps per row (W >= every
// member's L2 + 1; the extra columns are idle), so lane r works on column
// j = (tau - r) mod W of row 64 * floor((tau - r) / W) + r at step tau: an
// anti-diagonal wavefront that wraps from one 64-row strip into the next and
// from one pair into the next without draining.
constexpr int kChainMax = 32;    // pairs per chain
// residue bytes per chain (LDS) when stacking pairs: 4 regions + the PF
// tables stay under 160 KB / 6 workgroups, so LDS never binds the sweeps'
// occupancy before their VGPR budget does
constexpr int kChainSeqSoft = 4800;
constexpr int kChainSeqMax = 50000;   // residue bytes of a single-pair chain (one wave per block)
constexpr int kMinWidth = 192;   // W floor: boundary chunks are loaded 64 columns ahead
// W for a chain whose widest member has L2 columns (+1): multiple of 8 so the
// unrolled step loops never straddle a boundary-chunk switch
// chain widths are multiples of this: every wavefront segment (64 steps, or
// W mod 64 at a row's end) is a whole number of the sweeps' and the merge's
// load-queue groups (static_asserts in posterior.hip)
constexpr int kWidthQuantum = 8;
__host__ __device__ constexpr int chain_width(int maxL2) {
  return ((maxL2 + 1 < kMinWidth ? kMinWidth : maxL2 + 1) + kWidthQuantum - 1) & ~(kWidthQuantum - 1);
}
// LDS residue bytes of a chain of `n` members with sum of L1 = `sum_l1`:
// a zero area of W + 2, then per member the padded row (L1 + 2) and column
// (W + 1) sequences
__host__ __device__ constexpr int chain_seq_bytes(int W, int sum_l1, int n) {
  return W + 2 + sum_l1 + n * (W + 3);
}
// A chain launch's LDS layout is one int: the largest member count (bits
// 24+) and residue bytes (bits 0-23) over its chains.
__host__ __device__ constexpr int chain_lds_pack(int seq_bytes, int max_members) {
  return (max_members << 24) | seq_bytes;
}
// strips of a chain with `rows` stacked rows
__host__ __device__ constexpr int chain_strips(int rows) { return (rows + 63) >> 6; }
// step slots of a chain: steps tau = -1 .. S*W + 63, rounded up to 8
__host__ __device__ constexpr int64_t chain_steps(int rows, int W) {
  return ((int64_t)chain_strips(rows) * W + 65 + 7) & ~(int64_t)7;
}

// Model constants (CPNP/ProbabilisticModel.h:42-47 plus the PF factors of
// CPNP/MSAPartProbs.cpp:698-709).  Letter-indexed tables (26 uppercase
// letters) live in a device buffer `Tables` and are staged into LDS.
struct ModelScalars {
  float init[5];      // initialDistribution
  float t[5][5];      // transProb
  float lt[3][3];     // local_transProb
  float rt1;          // random_transProb[1]
  double pf_open, pf_ext;  // exp(beta*gap_open), exp(beta*gap_ext)
  float vit_init[3];       // Viterbi start/end scores (CPNP/ProbabilisticModel.h:1068-1070)
};

struct Tables {
  float match[26 * 26];   // matchProb['A'+r]['A'+c]
  float ins[26];          // insProb['A'+r][*]
  double sub[26 * 26];    // PF score factor, [seq2 letter][seq1 letter]
  double rsub[26 * 26];   // 1 / sub (correctly rounded; the PF backward's posterior quotient)
};

// Per-pair bookkeeping of one batch (device arrays indexed by slot; slots
// are ordered chain by chain).
struct PairMeta {
  const int32_t* pa;       // seq index of row sequence (seq1)
  const int32_t* pb;       // seq index of column sequence (seq2)
  const int32_t* row0;     // first stacked row of the pair in its chain
  const int32_t* chain;    // chain of the pair
  const int64_t* rm_off;   // base of the pair's chunk maxima (L1 x ceil(L2 / 64) floats)
  const int64_t* ell_row;  // first ELL row of the pair (rows 1..L1)
};

// Per-chain bookkeeping (device arrays indexed by chain = wave).
struct ChainMeta {
  const int32_t* first;    // first slot
  const int32_t* count;    // members (<= kChainMax)
  const int32_t* width;    // W
  const int32_t* rows;     // stacked rows (sum of L1 + 1)
  const int32_t* seq_bytes;// residues of all members (LDS staging)
  const int64_t* cell_off; // base of the chain's step-diagonal region (chain_steps * 64 slots)
  const int64_t* bnd_off;  // base of the chain's boundary row (W entries)
};

struct PairRec {           // per-pair scalars produced along the pipeline
  float tf5;               // 5-state forward total (last cell)
  float b5[5];             // 5-state backward at (1,1)M,(1,0)X1,X2,(0,1)Y1,Y2
  float tfl, tbl;          // local-model chain totals
  double zmant;            // PF total Z, scaled mantissa
  int32_t zexp;            // PF total Z frame
  int32_t flags;           // bit0: PF overflow, bit1: ELL overflow
  float mea;               // MEA score
  float dist;              // 1 - mea / min(L1, L2); npdoAlign: mea / #B
  int64_t nnz;             // sparse entries of the pair
};

struct SeqSet {
  const uint8_t* res;      // residue letters, 'A'..'Z' as 0..25
  const int64_t* off;
  const int32_t* len;
};

struct Scratch {
  float* f5;               // step-diagonal: 5-state fwd M, then f+b (in place)
  float* fl;               // local fwd M (the merge adds fl + bl)
  double* zm;              // PF forward Zm (packed with frame)
  float* pg;               // PF posterior, element idx at pg[idx * pg_stride]
  int32_t pg_stride;       // 2: in the low half of the slot's consumed PF forward Zm (zm)
  float* bl;               // step-diagonal: local bwd M (the merge adds fl + bl)
  // local-model chain totals (k_local_totals): per pair (rows 1..L1, chunks
  // of 64 columns, row-major from rm_off) the largest chain element of each
  // chunk, forward (f_M) and backward (b_M + emission), written by the sweeps
  float* cmf;
  float* cmb;
  // k_local_totals' per-wave candidate lists (64 rows x clist_row floats per
  // resident wave) and its pair counter (work queue)
  float* clist;
  int32_t clist_row;
  int32_t* tot_next;
  // lane-per-pair forward chain fold (k_local_bounds / k_local_list /
  // k_local_fold): per ELL row, the chain's lower bound at the row's start
  // (the exact fold of the chunk maxima of the rows before); the per-row
  // candidate counts go to ell_cnt until the merge overwrites it; pairs
  // whose bound failed the fold's check are listed in rep ([0] = count) for
  // k_local_totals to redo
  float* crb;
  int32_t* rep;
  int32_t force_repair;    // test hook (MLP_TOT_FORCE_REPAIR): every pair goes to the repair list
  float* bnd5;             // chain boundary row, HMMs (and the Viterbi sweep): a 32-byte record per column (5-state, local)
  double* bndz;            // partition function: a 32-byte record per column (3 doubles, frame)
  float* bndm;             // MEA boundary: 1 float per column
  int32_t* bndc;           // MEA boundary #B counts (npdoAlign distance): 1 int per column
  uint16_t* ell_col;       // [ell row][kEll]
  float* ell_val;
  int32_t* ell_cnt;        // [ell row]
  int32_t* lf_cnt;         // [ell row] the lane fold's candidate counts: ell_cnt (dead until the merge),
                           // or a per-batch array when a deferred finish still compacts the last batch
  uint8_t* vt;             // step-diagonal Viterbi traceback bits
};

// Viterbi family test outputs (per slot).
struct VitOut {
  uint8_t* path;           // traceback order: 0 = B (match), 1 = X, 2 = Y
  const int64_t* path_off; // per slot, capacity L1 + L2
  int32_t* path_len;
  float* match;            // identical residue pairs in B columns
  int32_t* state;          // best terminating state (k_viterbi -> k_vit_trace)
};

// kQP: QuickProbs' posterior stage (QP/Alignment/Multiple/PosteriorStage.cpp:
// 123-196): its partition function runs in the transposed orientation of
// C_P_NP_Aln's (so the three-term sums add in the other order) and keeps only
// posteriors in [0.001, 1]; the merge is the RMS of two models.
enum ModelSet : int { kHmm5 = 1, kLocal = 2, kPF = 4, kQP = 8 };
constexpr int kPidQP = 16;  // pid code of the QuickProbs posterior stage (include/mlpgpu.h MLP_PID_QP)
constexpr int kPidNpdo = 32;  // flag: npdoAlign's pair body (include/mlpgpu.h MLP_PID_NPDO)

inline int model_set_for_pid(int pid) {
  pid &= ~kPidNpdo;
  if (pid == kPidQP) return kHmm5 | kPF | kQP;
  if (pid == 2) return kLocal;
  if (pid >= 3) return kPF;
  return kHmm5 | kLocal | kPF;
}

// A second stream for the sweeps of one batch: when a model set runs as
// two kernels (fp32 HMMs, fp64 partition function) they touch disjoint
// scratch and run concurrently, so the one's tail of partly filled CUs
// overlaps the other's body.  fork / join: events (timing disabled).
struct SideStream {
  hipStream_t st;
  hipEvent_t fork, join;
  // join_mode 0: each sweep joins the side stream before it returns.  1: the
  // backward sweep records the join but does not wait (the caller waits
  // before the merge), so the local totals, which need only the fp32 sweep,
  // run beside the fp64 backward.  2: per-model chains -- neither sweep forks
  // or joins after the forward's fork; the caller joins before the merge.
  int join_mode;
};
// launchers (posterior.hip).  lds_seq: chain_lds_pack(max seq_bytes, max members).
hipError_t launch_forward(int models, const ModelScalars& ms, const Tables* tab, SeqSet seqs,
                          PairMeta pm, ChainMeta cm, PairRec* rec, Scratch sc, int64_t nchains,
                          int lds_seq, hipStream_t st, const SideStream* side);
hipError_t launch_backward(int models, const ModelScalars& ms, const Tables* tab, SeqSet seqs,
                           PairMeta pm, ChainMeta cm, PairRec* rec, Scratch sc, int64_t nchains,
                           int lds_seq, int64_t npairs, hipStream_t st, const SideStream* side);
// parts: kTotFwd (the forward chains, one persistent wave per pair; reads
// only what the forward sweep wrote, so it may run beside the backward sweep),
// kTotBwd (the backward chains, one wave per pair), or both in one kernel
constexpr int kTotFwd = 1, kTotBwd = 2;
hipError_t launch_local_totals(const ModelScalars& ms, const Tables* tab, SeqSet seqs, PairMeta pm, ChainMeta cm,
                               PairRec* rec, Scratch sc, int64_t npairs, int nwaves, hipStream_t st,
                               int parts = kTotFwd | kTotBwd);
// The same totals with the forward chain folded one pair per lane: its half
// between the forward and the backward sweeps (bounds, listing into the
// still-dead local backward array, fold), the rest after the backward sweep
// (backward chains, repair of failed bounds).
hipError_t launch_local_fwd_lanefold(SeqSet seqs, PairMeta pm, ChainMeta cm, PairRec* rec, Scratch sc, int64_t npairs,
                                     int nwaves, hipStream_t st);
hipError_t launch_local_bwd_lanefold(const ModelScalars& ms, const Tables* tab, SeqSet seqs, PairMeta pm, ChainMeta cm,
                                     PairRec* rec, Scratch sc, int64_t npairs, int nwaves, hipStream_t st);
// bytes after the local backward array the lane fold's unconditional
// read-ahead may touch past a batch's last pair (24 floats, rounded up)
constexpr size_t kLaneFoldPad = 256;
// resident waves of k_local_totals (persistent: each takes pairs off a counter)
constexpr int kTotalsWaves = 8192;
// chunk maxima per pair row (columns 1..L2 in chunks of 64)
__host__ __device__ constexpr int local_chunks(int L2) { return (L2 + 63) >> 6; }
hipError_t launch_fold_totals(const ModelScalars& ms, const Tables* tab, SeqSet seqs, PairMeta pm,
                              PairRec* rec, int64_t npairs, hipStream_t st);
hipError_t launch_merge(int models, int pid, const ModelScalars& ms, SeqSet seqs, PairMeta pm,
                        ChainMeta cm, PairRec* rec, Scratch sc, int64_t nchains, int lds_seq,
                        hipStream_t st);
// the pairs' sparse entry counts (PairRec::nnz) from the merge's row counts
hipError_t launch_pair_nnz(SeqSet seqs, PairMeta pm, PairRec* rec, Scratch sc, int64_t npairs, hipStream_t st);
hipError_t launch_viterbi(const ModelScalars& ms, const Tables* tab, SeqSet seqs, PairMeta pm,
                          ChainMeta cm, Scratch sc, VitOut vo, int64_t nchains, int lds_seq,
                          int64_t npairs, hipStream_t st);
hipError_t launch_compact(SeqSet seqs, PairMeta pm, PairRec* rec, Scratch sc,
                          const int64_t* ent_base, int32_t* out_rowptr, const int64_t* rowptr_base,
                          uint16_t* out_cols, float* out_vals, int64_t npairs, hipStream_t st);

// relaxation (relax.hip)
// QuickProbs' consistency round (ConsistencyStage::doRelaxation, QP/Alignment/
// Multiple/ConsistencyStage.cpp:133-258) instead of C_P_NP_Aln's: an accepted
// z is weighted by w_z / W_xy, W_xy = (1 + (s - 1) A_xy / a)(w_x + w_y) with
// A_xy the number of accepted z, the sum starts from P_xy (not 2 P_xy) and is
// divided by 1 + sum_z w_z / W_xy.  Selectivity (the Deterministic filter,
// ConsistencyStage.cpp:35-47, 171-186): z is accepted for (x, y) iff
// max(D[x][z], D[y][z]) <= a; without D every z is.
struct QpRelax {
  int on;                    // 0: C_P_NP_Aln's round
  const float* weights;      // per sequence (device)
  float selfweight;
  const float* seldist;      // N x N selectivity distances (device) or null
  float selectivity;         // a (the filter threshold and the A_xy divisor)
};
__device__ __forceinline__ bool qp_accept(const QpRelax& q, int n, int x, int y, int z) {
  if (!q.seldist) return true;
  const float dx = q.seldist[(int64_t)x * n + z], dy = q.seldist[(int64_t)y * n + z];
  return (dx > dy ? dx : dy) <= q.selectivity;  // std::max(x, y), then x <= a
}
struct RelaxArgs {
  int n;                     // sequences in the family
  const int32_t* lens;
  const int64_t* rp_off;     // per pair (a < b): row_ptr offset (L_a + 2 entries)
  const int32_t* rowptr;
  const int64_t* ent_off;
  const uint16_t* cols;
  const float* vals;
  const int64_t* trp_off;    // transposed blocks: row_ptr offset (L_b + 2 entries)
  const int32_t* trowptr;
  const uint16_t* tcols;
  const float* tvals;        // entries at ent_off (same count as the block)
  const int64_t* task_pair;  // tasks: (output pair, first row of 64)
  const int32_t* task_row0;
  int64_t ntasks;
  float* out;                // raw relaxed values at the input entry slots
  QpRelax qp;
};
struct TransposeArgs {
  int n;
  const int32_t* lens;
  const int64_t* rp_off;
  const int32_t* rowptr;
  const int64_t* ent_off;
  const uint16_t* cols;
  const float* vals;
  const int64_t* trp_off;
  int32_t* trowptr;
  uint16_t* tcols;
  float* tvals;
  const int64_t* pairs;      // blocks to transpose
  int64_t npairs;
  int max_len;               // LDS cursor capacity (max L_b)
};
struct FilterArgs {
  int n;
  const int32_t* lens;
  const int64_t* rp_off;
  const int32_t* rowptr;     // old pattern
  const int64_t* ent_off;    // old entry base
  const uint16_t* cols;
  const float* raw;          // relaxed values at old slots
  int64_t* pair_nnz;         // out (count pass)
  const int64_t* new_ent_off;// in (write pass)
  int32_t* new_rowptr;       // same offsets as rp_off
  uint16_t* new_cols;
  float* new_vals;
  const int64_t* pairs;      // output pairs handled
  int64_t npairs;
  int write;
  float cutoff;              // keep values >= cutoff (0.01; QuickProbs' last round 1e-5)
  int fixed16;               // QuickProbs: store (uint16)(v * 65535) / 65535
};
// Row-bitmap images for the relaxation (relax.hip).  Every block P(a, b)
// and its transpose is packed once per round as one 16-byte aligned record:
//   vals  f32[nnz]
//   hdr   u32[R + 1]
//   words {u32 bits, u32 base}[NW]
// R = rows of that orientation.  Row r's bitmap covers only the 32-column
// words between its first and last entry: hdr[r] = woff | c0w << 16 | nw << 24
// (first word index in `words`, first word's column / 32, word count; hdr[0]
// is an empty row), words[woff + w] covers columns 32 (c0w + w) .. + 31 and
// base is the entry index of its first set bit.  Divergent posteriors spread
// ~10 entries of a row over ~100 columns, so this is ~3.5 words per row
// instead of C / 32 + 1.  Image 2p is P(a, b) of pair p (rows a), image
// 2p + 1 its transpose (rows b).  Needs C <= 8000 (c0w, nw fit 8 bits) and
// nnz, NW < 65536.
struct ImgLayout {
  int64_t hdr, words, end;  // byte offsets (vals at 0)
};
__host__ __device__ inline int64_t mlp_align16(int64_t v) { return (v + 15) & ~(int64_t)15; }
__host__ __device__ inline ImgLayout img_layout(int rows, int64_t nnz, int64_t nwords) {
  ImgLayout l;
  l.hdr = mlp_align16(4 * nnz);
  l.words = l.hdr + mlp_align16(4 * (int64_t)(rows + 1));
  l.end = mlp_align16(l.words + 8 * nwords);
  return l;
}
struct PackArgs {
  int n;
  const int32_t* lens;
  const int64_t* rp_off;
  const int32_t* rowptr;
  const int64_t* ent_off;
  const uint16_t* cols;
  const float* vals;
  const int64_t* trp_off;
  const int32_t* trowptr;
  const uint16_t* tcols;
  const float* tvals;
  const int64_t* img_off;    // 2P + 1 byte offsets (write pass)
  int32_t* nwords;           // 2P bitmap word counts (count pass: out, write pass: in)
  uint8_t* img;
  int64_t nimg;              // 2P
  int count;                 // 1 = count pass, 0 = write pass
};
constexpr int kTileMax = 4;  // output pairs (x_t, y) sharing y per workgroup
struct TileRelaxArgs {
  int n;
  const int32_t* lens;
  const int64_t* rp_off;     // the output pairs' own patterns (masks) and values
  const int32_t* rowptr;
  const int64_t* ent_off;
  const uint16_t* cols;
  const float* vals;
  const int64_t* img_off;
  const int32_t* nwords;
  const uint8_t* img;
  int64_t img_chunks;        // image buffer size / 16
  const int32_t* tiles;      // per tile: kTileMax pair indices (-1 = none), kTileMax x's, y
  int64_t ntiles;
  float* out;                // raw relaxed values at the input entry slots
  int cap;                   // LDS bytes for one staged tile (multiple of 16)
  QpRelax qp;
};
constexpr int kTileInts = 2 * kTileMax + 1;
#ifndef MLP_RELAX_THREADS
#define MLP_RELAX_THREADS 1024
#endif
// workgroup of the tiled relaxation: 1024 threads (16 waves, 128 VGPRs, one
// per CU), or 512 with two workgroups sharing a CU's LDS and SIMDs
constexpr int kRelaxThreads = MLP_RELAX_THREADS;
constexpr int kRelaxGroupsPerCU = 1024 / kRelaxThreads;
size_t tile_relax_lds(int cap);
int tile_relax_prefetch(int cap);              // 16-byte chunks per thread, 0 = too large
int tile_relax_slots(int64_t cells);           // cells per thread, 0 = too many
int tile_relax_max_cap();                      // largest tile the prefetch registers hold
hipError_t launch_pack(const PackArgs& a, hipStream_t st);
// one_per_cu: the one-workgroup class (KP = 9 whatever its cap: the KP = 5
// instance is bounded to 64 VGPRs for two workgroups per CU)
hipError_t launch_relax_tiles(const TileRelaxArgs& a, int slots, bool one_per_cu, hipStream_t st);
// dense-block MFMA evaluation of the consistency transform (relax_mfma.hip):
// res = {kernel s, dense MACs, outputs, max rel err, cells checked, tiles, blocks}
int relax_blockmfma_eval(int n, const int32_t* lens, const int64_t* rp_off, const int32_t* rowptr,
                         const int64_t* ent_off, const uint16_t* cols, const float* vals, int nx, const int32_t* xs,
                         int ny, const int32_t* ys, double* res, std::string& err);
// profile posterior (profile.hip)
struct ProfileArgs {
  int n;                     // family size
  const int32_t* rowptr;     // the sparse set (pairs a < b) and its transposes
  const uint16_t* cols;
  const float* vals;
  const int32_t* trowptr;
  const uint16_t* tcols;
  const float* tvals;
  int n1, n2, L1, L2;        // profile sizes (sequences, columns)
  const int64_t* rpb;        // n1 x n2: row_ptr base of block (i, j); ~base: transposed block
  const int64_t* eb;         // n1 x n2: entry base of block (i, j)
  int32_t* inv1;             // n1 x (L1 + 1): residue of sequence i in column r, 0 = gap
                             // (zeroed by the caller, filled by launch_profile_posterior)
  const int32_t* map1;       // per sequence i of A: column of its residue k (k = 1..len)
  const int64_t* map1_off;   // per i: offset of its map (k = 0 at map1_off[i])
  int64_t map1_len;          // entries of map1
  const int32_t* map2;       // per sequence j of B: column of its residue k (k = 1..len)
  const int64_t* map2_off;   // per j: offset of its map (k = 0 at map2_off[j])
  const float* w;            // n1 x n2: (float)(w_i w_j / sum)
  float* out;                // (L1 + 1) x (L2 + 1); rows 1..L1 written
  int stage;                 // staged entries per run (<= the LDS stage; set by launch_profile_posterior)
};
size_t profile_lds(int L2);
// Device MEA of the dense profile posterior (k_profile_mea): one workgroup
// per 64-row strip, strips pipelined across CUs through HBM.  Workspace
// layout (mea_layout): the choices (2 bits a cell -- bit 0: D the largest,
// bit 1: L >= U -- per strip, 16-step block and lane a uint32), each
// strip's last row (NaN until written: the next strip polls the values), the
// score and an error word (a strip that waited too long for the one above).
constexpr int kMeaBlk = 16;  // steps per block (one uint32 of choices per lane)
struct MeaLayout {
  int nstrips, nblk, rowpitch;
  size_t o_tb, o_row, o_score, o_err, bytes;
};
MeaLayout mea_layout(int L1, int L2);
static_assert(kMeaBlk % 4 == 0 && 2 * kMeaBlk <= 32, "a block's choices fill one uint32 per lane; windows load 4 at a time");
constexpr size_t kMeaGuard = 512;              // readable bytes before and after a dense profile posterior (MEA windows)
struct MeaArgs {
  const float* post;         // (L1 + 1) x (L2 + 1)
  int L1, L2;
  uint8_t* work;             // mea_layout(L1, L2).bytes
  int spin_limit;            // polls a strip waits before giving up (1 << 22; MLP_MEA_SPINS: test hook)
};
hipError_t launch_profile_mea(const MeaArgs& a, hipStream_t st);
hipError_t launch_profile_gather(const float* post, const int64_t* cells, int64_t n, float* out, hipStream_t st);
hipError_t launch_profile_posterior(const ProfileArgs& a, hipStream_t st);
hipError_t launch_transpose(const TransposeArgs& a, hipStream_t st);
hipError_t launch_relax_tasks(const RelaxArgs& a, hipStream_t st);
hipError_t launch_filter(const FilterArgs& a, hipStream_t st);

}  // namespace mlp
