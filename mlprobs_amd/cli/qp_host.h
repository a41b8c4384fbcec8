// qp_host.h -- host side of the `quickprobs` drop-in (the QuickProbs 2
// realigner MLProbs calls, realign/QuickProbs): sequence I/O, the UPGMA guide
// tree with its sequence weights and subtree distances, the weighted
// profile-profile posterior, progressive construction and column
// refinement.  The all-pairs posterior and consistency stages run on the GPU
// (libmlpgpu: mlp_posteriors(MLP_PID_QP), mlp_relax_qp_selective).  Each
// function cites the QuickProbs code (under realign/QuickProbs/src) whose
// behaviour it reproduces; `QP/` below stands for that directory.
#pragma once
#include <stdint.h>

#include <functional>
#include <random>
#include <string>
#include <utility>
#include <vector>

namespace qph {

// One (possibly gapped) row: data[0] = '@', residues / '-' at 1..length
// (QP/Alignment/DataStructures/Sequence.h).
struct Seq {
  std::string header;
  std::string data;
  int sort_label = 0;   // sequenceLabel (GetSortLabel)
  int label = 0;        // inputLabel (GetLabel)
  int length() const { return (int)data.size() - 1; }
};
using Profile = std::vector<Seq>;

// SequenceIO::load(FASTA) + checkAndCorrect (QP/Alignment/DataStructures/
// SequenceIO.cpp:18-135).  On failure returns false with `out_msg` (printed
// on stdout by the reference, one line per illegal character) and `err`
// (the exception text).
bool load_fasta(const std::string& path, std::vector<Seq>& seqs, std::string& out_msg, std::string& err);
// the same on the file's bytes
bool load_fasta_text(const std::string& text, std::vector<Seq>& seqs, std::string& out_msg, std::string& err);

// SequenceIO::saveFasta (SequenceIO.cpp:176-199): 60 columns.
void write_fasta(std::string& out, const Profile& p);

// The all-pairs sparse set (pairs a < b from libmlpgpu, rows = a) plus the
// transposes QuickProbs keeps as sparseMatrices[b][a]
// (FilteredSparseMatrix::computeTranspose; the 16-bit values round-trip).
struct Sparse {
  int n = 0;
  std::vector<int> lens;
  // per ordered pair (a, b), a != b: CSR rows 1..L_a (row_ptr has L_a + 2)
  struct Block {
    const int32_t* rp = nullptr;
    const uint16_t* cols = nullptr;
    const float* vals = nullptr;
  };
  std::vector<Block> blocks;  // n * n
  std::vector<int32_t> row_ptr, trow_ptr;
  std::vector<int64_t> rp_off, ent_off;
  std::vector<uint16_t> cols, tcols;
  std::vector<float> vals, tvals;
  const Block& at(int a, int b) const { return blocks[(size_t)a * n + b]; }
  void build_views();  // transposes + the n x n view table
};

// GuideTree + ClusterTree (QP/Alignment/Multiple/GuideTree.cpp,
// ClusterTree.cpp): UPGMA over the posterior distances.
struct Tree {
  struct Node {
    int left = -1, right = -1, parent = -1;
    float dist = 0;
    bool leaf = false;
    int order = 0, depth = 0;
  };
  int n = 0, root = -1;
  std::vector<Node> nodes;
  std::vector<float> weights;           // calculateSeqsWeights
  std::vector<float> subtree_distances() const;  // calculateSubtreeDistances, n x n
};
Tree build_tree(std::vector<float> dist, int n);  // dist: n x n (copied: the build overwrites it)

struct Options {
  int consistency = -1;  // -c (QuickProbs: < 0 -> 2 rounds up to 50 sequences, else 1)
  int refinement = -1;   // -r (<= 0 -> 30 passes up to 200 sequences, else 200)
};

// Where the weighted profile posteriors come from: `device` (libmlpgpu's
// mlp_profile_posterior over the device-resident sparse set) when set and it
// succeeds, else the host restatement over `host_sparse()` (built on first
// use).
struct PosteriorBackend {
  // returns the dense (L1 + 1) x (L2 + 1) matrix (valid until the next call)
  // or nullptr to use the host path
  std::function<const float*(const std::vector<float>& w, const Profile& A, const Profile& B)> device;
  // the posterior and its MEA on the device: path and score, or false
  std::function<bool(const std::vector<float>& w, const Profile& A, const Profile& B, std::string& path,
                     float* score)>
      device_mea;
  std::function<const Sparse&()> host_sparse;
};

// ConstructionStage::processTree + ColumnRefinement (QP/Alignment/Multiple/
// ConstructionStage.cpp, RefinementBase.cpp, ColumnRefinement.cpp).
Profile construct_and_refine(const std::vector<Seq>& seqs, const PosteriorBackend& be, const Tree& tree,
                             const Options& opt, int threads);

// Sequence::getMapping arrays of a profile, concatenated (len + 1 per row).
std::vector<int32_t> profile_maps(const Profile& p, int threads = 1);

}  // namespace qph
