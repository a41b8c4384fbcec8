// pipeline.h -- the MLProbs pipeline (kuangmeng/MLProbs MLProbs.py and
// utils/*.py) as one native driver, `mlprobs`:
//
//   features (c_p_np_aln -G) -> classifier 1 (branch forest) -> base MSA
//   (c_p_np_aln -p 0|1) -> BLOSUM62 column scores -> classifier 3 (regions
//   forest) [-> classifier 2 (seq_lens forest)] -> split into column regions
//   -> quickprobs on each region, kept if its average column score is not
//   worse -> combine -> whole-family quickprobs fallbacks.
//
// Every Python stage is restated here with the reference's own semantics
// (its dict-of-headers parsing, sorted keys, slice bounds, file naming and
// error fallbacks; the file:line cited at each function).  The region files
// of ./tmp/seperate_regions live in memory (Dir).  The two aligners run
// in-process (runners.h: host context for small families, one shared device
// context otherwise) or, for the baseline, as external commands exactly as
// MLProbs.py spawns them (ExternalTools).
#pragma once
#include <stdint.h>

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "runners.h"

namespace mlpp {

// ---------------------------------------------------------------- forests
// A RandomForestClassifier exported by tools/export_forests.py (`.forest`)
// and evaluated as scikit-learn 0.21.3's predict does for one sample:
// features cast to float32, each tree walked with x <= threshold -> left,
// the leaf's class weights normalised per tree, summed over the trees in
// order, divided by the tree count, first maximum (sklearn/ensemble/
// forest.py predict / predict_proba, sklearn/tree/tree.py predict_proba).
struct Forest {
  int n_features = 0, n_classes = 0;
  std::vector<double> classes;
  struct Tree {
    std::vector<int32_t> left, right, feature;
    std::vector<double> threshold, value;  // value: node_count x n_classes
  };
  std::vector<Tree> trees;
  bool load(const std::string& path, std::string& err);
  std::vector<double> predict_proba(const std::vector<double>& x) const;
  double predict(const std::vector<double>& x) const;
};
// para.txt: one float per line (max, min pairs per feature)
bool read_para(const std::string& path, std::vector<double>& para, std::string& err);

// ---------------------------------------------------------------- MSA text
// The header-keyed parse every utils module repeats (e.g.
// calculate_column_scores.py:41-58): lines starting with '>' are keys (the
// whole line), the other lines after a key are concatenated without '\r';
// a repeated key keeps its last value; the final assignment always happens
// (an input without headers gives {"": ""}).  `last_len` = len(value) of the
// last record (the reference's `lens`).
struct Dic {
  std::map<std::string, std::string> rows;  // sorted keys, as sorted(dic.keys())
  size_t last_len = 0;
};
Dic parse_dic(const std::vector<std::string>& lines);
std::vector<std::string> split_newline(const std::string& text);  // str.split("\n")
std::vector<std::string> splitlines(const std::string& text);     // str.splitlines()

// calculateColScore (calculate_column_scores.py:37-82): per column the
// BLOSUM62 sum of pairs over the sorted keys / (N (N - 1) / 2), their mean
// (un_sp), standard deviation and the fraction of columns >= 1.
struct ColScores {
  std::vector<double> col;
  double un_sp = 0, sd = 0, peak = 0;
  int64_t lens = 0;   // alignment length (the last record's)
  int64_t nkeys = 0;  // distinct headers
  bool error = false; // the reference raises (ZeroDivisionError / IndexError)
  std::string error_msg;
};
ColScores column_scores(const Dic& d);
// getAvgColScore (calculate_column_scores.py:84-121): -1 when there is no
// pair or no column
double avg_col_score(const std::string& file_text, bool* error = nullptr);

// Region detection (unreliable_regions.py:9-44, reliable_regions.py:10-53):
// [head, item] pairs as the reference builds them (head 1-based, item the
// 0-based index of the first column past the run, or the last column).
std::vector<std::pair<int64_t, int64_t>> unreliable_regions(const std::vector<double>& col, double sigma, double beta,
                                                            int class_lens);
std::vector<std::pair<int64_t, int64_t>> reliable_regions(const std::vector<double>& col, double threshold,
                                                          int class_lens_max, int class_lens_min);

// ./tmp/seperate_regions: file name -> content
using Dir = std::map<std::string, std::string>;
// seperateUnreliableRegions / seperateReliableRegions (unreliable_regions.py:
// 46-101, reliable_regions.py:55-110; identical bodies)
void separate_regions(const std::vector<std::pair<int64_t, int64_t>>& regions, const std::string& real_output,
                      Dir& dir);

// ---------------------------------------------------------------- tools
// The two aligners as MLProbs.py calls them.
struct Tools {
  virtual ~Tools() = default;
  // subprocess.getstatusoutput("c_p_np_aln -G|-p N file"): exit status and
  // stdout + stderr with one trailing newline removed
  virtual int cpnp(const std::string& seq_file, bool features, int program, std::string& text) = 0;
  // os.system("quickprobs file > out"): the bytes quickprobs writes on
  // stdout for an input with this content / for the input file
  virtual std::string quickprobs_text(const std::string& fasta) = 0;
  virtual std::string quickprobs_file(const std::string& seq_file) = 0;
  virtual const char* name() const = 0;
};
// in-process (runners.h), one Session for the whole pipeline run
std::unique_ptr<Tools> in_process_tools(mlpr::Session* session);
// external commands (e.g. the reference CLIs built from source), run through
// /bin/sh like MLProbs.py; tmpdir holds the per-region input files
std::unique_ptr<Tools> external_tools(const std::string& cpnp_cmd, const std::string& qp_cmd,
                                      const std::string& tmpdir);

// ---------------------------------------------------------------- driver
struct Models {
  Forest branch, regions, seq_lens;
  std::vector<double> branch_para, regions_para, seq_lens_para;
  bool load(const std::string& dir, std::string& err);
};

// What one run did (for the bench and the tests): the stage outputs the
// fixtures pin, and the time of each stage.
struct Trace {
  std::string features_line;        // -G text
  std::vector<double> features1;    // classifier 1 input (normalised)
  int class1 = -1;                  // 0 progressive, 1 non-progressive
  int killed_stage = 0;
  ColScores cs;
  int class_region = -1, class_lens = -1;
  std::vector<std::pair<int64_t, int64_t>> regions;
  std::vector<std::string> realigned;  // region files handed to quickprobs, in order
  std::vector<int> kept_original;      // per realigned region: 1 = the original block was kept
  std::string path;                    // "RIR" / "RCR" / "fallback ..."
  std::map<std::string, double> times; // seconds per stage
  int quickprobs_calls = 0;
};

// MLProbs.py main (MLProbs.py:36-99): the final MSA text as written to the
// output file; false (err set) where the reference pipeline itself would
// raise (a Python exception) and leave no output.
bool run_pipeline(const std::string& seq_file, Tools& tools, const Models& models, std::string& result, Trace& tr,
                  std::string& err, bool verbose);

}  // namespace mlpp
