// msa_host.h -- host side of the c_p_np_aln drop-in: sequence I/O, the guide
// tree, profile-profile posteriors from the sparse set, MEA alignment of two
// profiles and iterative refinement.  These stages run once per family (the
// all-pairs stages they consume run on the GPU through libmlpgpu); each
// function cites the reference code whose behaviour it reproduces
// (kuangmeng/MLProbs baseMSA/C_P_NP_Aln).
#pragma once
#include <stdint.h>

#include <functional>
#include <memory>
#include <set>
#include <string>
#include <utility>
#include <vector>

namespace cpnp {

// One (possibly gapped) row of an alignment: data[0] is unused ('@'),
// residues / '-' at 1..length (Sequence.h:24-125).
struct Row {
  std::string header;
  std::string data;   // data[0] = '@'
  int label = 0;      // input position (GetLabel)
  int sort_label = 0; // GetSortLabel
  int length() const { return (int)data.size() - 1; }
};

using Profile = std::vector<Row>;

// FASTA in the reference's MultiSequence::LoadMFA(..., stripGaps = true)
// semantics (Sequence.h:56-119, MultiSequence.h:267-312).  Returns false
// and sets `err` on the conditions where the reference exits with status 1.
bool load_fasta(const std::string& path, std::vector<Row>& out, std::string& err);

// MultiSequence::WriteMFA, 60 columns (Sequence.h:281-303).
void write_mfa(std::string& out, const Profile& p, int columns = 60);

// std::allocator whose resize leaves the elements uninitialised: buffers
// that a copy fills right after (C3's row pointers are 210 MB)
template <class T>
struct NoInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = NoInitAlloc<U>;
  };
  NoInitAlloc() = default;
  template <class U>
  NoInitAlloc(const NoInitAlloc<U>&) {}
  template <class U>
  void construct(U* p) noexcept {
    ::new ((void*)p) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new ((void*)p) U(std::forward<A>(a)...);
  }
};

// Canonical sparse set of libmlpgpu (include/mlpgpu.h): pair (a < b) has
// row_ptr[rp_off[p] .. + L_a + 2) and entries from ent_off[p].
struct SparseSet {
  int n = 0;
  std::vector<int> lens;
  std::vector<int64_t> rp_off, ent_off;
  std::vector<int32_t, NoInitAlloc<int32_t>> row_ptr;  // (filled by mlp_csr_export)
  std::vector<uint16_t> cols;
  std::vector<float> vals;
  int64_t pair(int a, int b) const {  // a < b, row-major (CPNP/MSA.cpp:907-919)
    return (int64_t)a * n - (int64_t)a * (a + 1) / 2 + (b - a - 1);
  }
};

// UPGMA-style cluster tree over the distance matrix (MSAClusterTree.cpp:
// generateClusterTree(varianceid)) and the sequence weights derived from it
// (MSAGuideTree.cpp getSeqsWeights).
struct GuideTree {
  struct Node {
    int left = -1, right = -1, parent = -1;
    float dist = 0;
    bool leaf = false;
    int order = 0;
  };
  std::vector<Node> nodes;
  int root = -1;
  std::vector<int> weights;
};
GuideTree build_tree(std::vector<std::vector<float>> dist, int varianceid);

// Profile-profile posterior (ProbabilisticModel.h:1197-1376): weighted when
// `weights` is non-null.  Returns the dense (len1 + 1) x (len2 + 1) matrix.
std::vector<float> build_posterior(const Profile& a, const Profile& b, const SparseSet& sp,
                                   const int* weights, float cutoff);
void build_posterior_into(const Profile& a, const Profile& b, const SparseSet& sp, const int* weights,
                          float cutoff, std::vector<float>& post, std::vector<size_t>* dirty = nullptr);

// A device implementation of build_posterior (the GPU's BuildPosterior):
// returns the dense matrix, valid until its next call, or nullptr to fall
// back to the host.  Used by the progressive merges and both refinements
// when set and the cutoff is 0.
using ProfileBackend = std::function<const float*(const Profile& a, const Profile& b, const int* weights)>;
void set_profile_backend(ProfileBackend fn);
// build_posterior through the backend when possible, else into a reused
// host buffer; the result is valid until the next call
const float* profile_posterior(const Profile& a, const Profile& b, const SparseSet& sp, const int* weights,
                               float cutoff);

// The profile posterior and its MEA both on the device (the matrix never
// comes back): fills `path` and `score` and, when `cells` is given, `vals`
// with the matrix at those row-major indices; false = use the host path.
using MeaBackend = std::function<bool(const Profile& a, const Profile& b, const int* weights,
                                      const std::vector<int64_t>* cells, std::vector<float>* vals,
                                      std::string& path, float* score)>;
void set_mea_backend(MeaBackend fn);
// device_mea through the backend when set and the cutoff is 0 (timed with the MEA)
bool device_mea(const Profile& a, const Profile& b, const int* weights, float cutoff,
                const std::vector<int64_t>* cells, std::vector<float>* vals, std::string& path, float* score);

// MEA alignment of two profiles (ProbabilisticModel.h:804-864): the path
// ('B', 'X', 'Y') and its score.
std::string mea_path(int len1, int len2, const std::vector<float>& post, float* score);
std::string mea_path(int len1, int len2, const float* post, float* score);  // (len1 + 1) x (len2 + 1) row-major
// the two evaluations mea_path chooses between (wave: threads pipelined
// over 64-row bands, for large matrices); identical results
std::string mea_path_serial(int len1, int len2, const float* post, float* score);
std::string mea_path_dispatch(int len1, int len2, const float* post, float* score);  // untimed
std::string mea_path_wave(int len1, int len2, const float* post, float* score);  // threads over 64-row bands
// SIMD lanes over rows (8: AVX2, 16: AVX-512; 0: none), MLP_MEA_SIMD overrides
int mea_simd_lanes();
std::string mea_path_simd(int len1, int len2, const float* post, float* score, int lanes);
// accumulated seconds of profile posteriors and MEA, calls (MLP_CLI_TIMES)
void profile_times(double* post, double* mea, int64_t* calls, int64_t* device_calls);

// Profile merge along a path (Sequence.h AddGaps) and helpers.
Profile merge(const Profile& a, const Profile& b, const std::string& path, bool sort_by_label);

// MultiSequence::Project (MultiSequence.h:662-734): the rows of `idx`, in
// index order, without the columns that are gaps in all of them.
Profile project(const Profile& p, const std::set<int>& idx);

// The C library's rand() / srand() sequence (glibc TYPE_3), reproduced.
void libc_srand(uint32_t seed);
int libc_rand_next();

struct Options {
  int consistency = 2;          // -c
  int refinement = 100;         // -ir
  float cutoff = 0;             // -co
  bool align_order = false;     // -a
  bool verbose = false;         // -v
};

// Progressive alignment over the guide tree followed by iterative
// refinement (MSA.cpp:1369-1635, ComputeFinalAlignment).
Profile progressive_alignment(const std::vector<Row>& seqs, const SparseSet& sp, const GuideTree& tree,
                              int pid, Options& opt);

// Non-progressive strategy (c_p_np_aln -p 1, MSA::npdoAlign,
// CPNP/MSA.cpp:1084-1140) after posteriors and consistency:
// the alignment graph of every sparse entry (ComputeGraph + AlignGraph,
// CPNP/MSA.cpp:1776-1844, AlignGraph.h:894-1160), rows in input order ...
Profile graph_alignment(const std::vector<Row>& seqs, const SparseSet& sp);
// ... and its refinement (DoRefinement + FindSimilar, CPNP/MSA.cpp:1852-2082)
// over the npdoAlign distances (score / #B).  Seeds rand() from time(0) per
// pass like the reference; MLP_SRAND_TIME fixes that clock (tests).
Profile np_refinement(Profile aln, const SparseSet& sp, const std::vector<std::vector<float>>& dist,
                      const Options& opt);

}  // namespace cpnp
