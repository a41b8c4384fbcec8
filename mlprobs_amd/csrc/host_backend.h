// host_backend.h -- the C ABI's host (CPU) implementation of the C_P_NP_Aln
// stages, for families too small to pay for a device (HIP runtime start-up
// and teardown alone cost 0.2-0.4 s per process, more than the reference
// needs for a small family; SURVEY.md section 7, hard part 7).  Internal to
// libmlpgpu: a context created by mlp_ctx_create_host() runs every entry
// point here and never calls the HIP runtime.
//
// Each function restates the reference code it names with the same float /
// double / long double operation sequence, so its results are the
// reference's bit for bit (the partition function included: it runs in
// x87 long double like CPNP/MSAPartProbs.cpp).  Pairs are spread over host
// threads; every pair is computed by one thread in the reference's order.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "mlp_kernels.h"

namespace mlph {

struct FamilyView {
  int n;
  const int32_t* lens;
  const int64_t* offs;
  const uint8_t* res;     // letters 'A'..'Z'
  const int32_t* pa;      // per pair (row-major order): first sequence
  const int32_t* pb;      //                             second sequence
};

// Canonical CSR store (include/mlpgpu.h layout) on the host.
struct Store {
  std::vector<int32_t> rowptr;   // rp_off[P] entries
  std::vector<int64_t> ent_off;  // P + 1
  std::vector<uint16_t> cols;
  std::vector<float> vals;
};

int threads_for(int64_t work_units);

// ComputeViterbiAlignment + the ModelAdjustmentTest counting loop
// (CPNP/ProbabilisticModel.h:1043-1170, CPNP/MSA.cpp:818-841): per pair the
// path length, the identical residues in 'B' columns and (when `paths`) the
// path in forward order (0 = B, 1 = X, 2 = Y) at vit_off[p].
void viterbi(const mlp::Tables& T, const mlp::ModelScalars& ms, const FamilyView& f, int64_t p0, int64_t p1,
             int32_t* len, float* match, const int64_t* vit_off, uint8_t* paths);

// The pdoAlign / ArrangePosteriorProbs pair body (CPNP/MSA.cpp:939-1025,
// 1665-1760) for pairs [p0, p1): posteriors of the models `pid` selects,
// RMS merge, MEA (score and, for npdo, #B), distance, sparse matrix.  The
// store's entries for these pairs are appended in pair order (store must
// hold pairs [.., p0)).  Returns 0, or 3 (MLP_ERR_OVERFLOW) when the
// partition function reaches long double infinity (the reference exits).
int posteriors(const mlp::Tables& T, const mlp::ModelScalars& ms, const FamilyView& f, int pid, bool npdo,
               int64_t p0, int64_t p1, const std::vector<int64_t>& rp_off, Store& st, float* dist, float* mea,
               int64_t* nnz, std::string& err);

// QuickProbs' posterior stage (PosteriorStage::computePairwise +
// combineMatrices, QP/Alignment/Multiple/PosteriorStage.cpp:123-196) for pairs
// [p0, p1): the 5-state posterior above, QuickProbs' double partition
// function (PartitionFunction.cpp:71-291; T.sub / ms.pf_* from the QuickProbs
// tables), RMS of the two fused with the MEA score, distance
// 1 - score / min(L1, L2), entries >= `cutoff` as 16-bit fixed point read back
// as q / 65535 (PackedSparseMatrix, SparseEntry.h:31-32).
void qp_posteriors(const mlp::Tables& T, const mlp::ModelScalars& ms, const FamilyView& f, int64_t p0, int64_t p1,
                   float cutoff, const std::vector<int64_t>& rp_off, Store& st, float* dist, float* mea,
                   int64_t* nnz);

// QuickProbs' consistency round instead of C_P_NP_Aln's (ConsistencyStage::
// doRelaxation, QP/Alignment/Multiple/ConsistencyStage.cpp:133-266): z
// accepted iff max(seldist[x][z], seldist[y][z]) <= selectivity (NULL: all),
// P' = (P + sum_z w_z P_xz P_zy) / (1 + sum_z w_z), w_z = weights[z] / W_xy,
// W_xy = (1 + (selfweight - 1) A_xy / selectivity)(w_x + w_y); entries >=
// cutoff kept as 16-bit fixed point.
struct QpRelaxHost {
  const float* weights;
  const float* seldist;
  float selectivity, selfweight, cutoff;
};

// One MSA::DoRelaxation round (CPNP/MSA.cpp:1172-1360) over every pair, or
// QuickProbs' round when qp is given.  With an output range [r0, r1) only
// those pairs are computed: the store then holds their block, entries from 0
// (ent_off[r0] = 0 .. ent_off[r1]), rows of other pairs cleared.
void relax(const FamilyView& f, const std::vector<int64_t>& rp_off, Store& st, int64_t* nnz,
           const QpRelaxHost* qp = nullptr, int64_t r0 = 0, int64_t r1 = -1);

}  // namespace mlph
