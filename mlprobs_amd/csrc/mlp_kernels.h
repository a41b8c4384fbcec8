// mlp_kernels.h -- shared host/device declarations for the posterior and
// relaxation kernels (internal to libmlpgpu; not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mlp {

constexpr int kWave = 64;        // CDNA wavefront
constexpr int kWavesPerBlock = 4;  // independent pairs per workgroup
constexpr int kEll = 64;         // sparse slots per posterior row before overflow
constexpr int kSeqLds = 2048;    // column residues staged in LDS per wave (longer: LONG kernels)

// Steps of one 64-row strip: columns 0..L2 plus the 63-step skew, padded to
// a multiple of 8 so the step loops unroll without remainders.
__host__ __device__ constexpr int strip_steps(int L2) { return (L2 + 64 + 7) & ~7; }

// Model constants (CPNP/ProbabilisticModel.h:42-47 plus the PF factors of
// CPNP/MSAPartProbs.cpp:698-709).  Letter-indexed tables (26 uppercase
// letters) live in a device buffer `Tables` and are staged into LDS.
struct ModelScalars {
  float init[5];      // initialDistribution
  float t[5][5];      // transProb
  float lt[3][3];     // local_transProb
  float rt1;          // random_transProb[1]
  double pf_open, pf_ext;  // exp(beta*gap_open), exp(beta*gap_ext)
};

struct Tables {
  float match[26 * 26];   // matchProb['A'+r]['A'+c]
  float ins[26];          // insProb['A'+r][*]
  double sub[26 * 26];    // PF score factor, [seq2 letter][seq1 letter]
};

// Per-pair bookkeeping of one batch (device arrays, length npairs).
struct PairMeta {
  const int32_t* pa;       // seq index of row sequence (seq1)
  const int32_t* pb;       // seq index of column sequence (seq2)
  const int64_t* cell_off; // base of the pair's strip-diagonal region
  const int64_t* rm_off;   // base of the pair's row-major chain region
  const int64_t* bnd_off;  // base of the pair's boundary columns
  const int64_t* ell_row;  // first ELL row of the pair (rows 1..L1)
};

struct PairRec {           // per-pair scalars produced along the pipeline
  float tf5;               // 5-state forward total (last cell)
  float b5[5];             // 5-state backward at (1,1)M,(1,0)X1,X2,(0,1)Y1,Y2
  float tfl, tbl;          // local-model chain totals
  double zmant;            // PF total Z, scaled mantissa
  int32_t zexp;            // PF total Z frame
  int32_t flags;           // bit0: PF overflow, bit1: ELL overflow
  float mea;               // MEA score
  float dist;              // 1 - mea / min(L1, L2)
  int64_t nnz;             // sparse entries of the pair
};

struct SeqSet {
  const uint8_t* res;      // residue letters, 'A'..'Z' as 0..25
  const int64_t* off;
  const int32_t* len;
};

struct Scratch {
  float* f5;               // strip-diagonal: 5-state fwd M, then f+b (in place)
  float* fl;               // local fwd M, then f+b
  double* zm;              // PF forward Zm (packed with frame)
  float* pg;               // PF posterior
  float* chf;              // row-major local fwd M   (chain for total)
  float* chb;              // row-major local bwd M + emission
  float* bnd5;             // boundary columns: 5 floats per column
  float* bndl;             // 3 floats per column
  double* bndz;            // 3 doubles per column
  int32_t* bnde;           // 1 int per column
  float* bndm;             // MEA boundary: 1 float per column
  uint16_t* ell_col;       // [ell row][kEll]
  float* ell_val;
  int32_t* ell_cnt;        // [ell row]
};

enum ModelSet : int { kHmm5 = 1, kLocal = 2, kPF = 4 };

inline int model_set_for_pid(int pid) {
  if (pid == 2) return kLocal;
  if (pid >= 3) return kPF;
  return kHmm5 | kLocal | kPF;
}

// launchers (posterior.hip)
hipError_t launch_forward(int models, const ModelScalars& ms, const Tables* tab, SeqSet seqs,
                          PairMeta pm, PairRec* rec, Scratch sc, int64_t npairs, int max_len2,
                          hipStream_t st);
hipError_t launch_backward(int models, const ModelScalars& ms, const Tables* tab, SeqSet seqs,
                           PairMeta pm, PairRec* rec, Scratch sc, int64_t npairs, int max_len2,
                           hipStream_t st);
hipError_t launch_local_totals(SeqSet seqs, PairMeta pm, PairRec* rec, Scratch sc, int64_t npairs,
                               hipStream_t st);
hipError_t launch_merge(int models, int pid, const ModelScalars& ms, SeqSet seqs, PairMeta pm,
                        PairRec* rec, Scratch sc, int64_t npairs, hipStream_t st);
hipError_t launch_compact(SeqSet seqs, PairMeta pm, PairRec* rec, Scratch sc,
                          const int64_t* ent_base, int32_t* out_rowptr, const int64_t* rowptr_base,
                          uint16_t* out_cols, float* out_vals, int64_t npairs, hipStream_t st);

// relaxation (relax.hip)
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
};
hipError_t launch_transpose(const TransposeArgs& a, hipStream_t st);
hipError_t launch_relax_tasks(const RelaxArgs& a, hipStream_t st);
hipError_t launch_filter(const FilterArgs& a, hipStream_t st);

}  // namespace mlp
