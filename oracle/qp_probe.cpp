// qp_probe.cpp -- TEST INFRASTRUCTURE ONLY (oracle side).
//
// A harness that links the *reference's own* QuickProbs sources
// (realign/QuickProbs/src, compiled in place by `make -C oracle qp` into
// oracle/_ref/qpobj/) and calls its posterior stage on given inputs, dumping
// the outputs as the tagged binary records of ref_probe.cpp.  It is used to
//   (1) dump QuickProbs' constant tables (pair-HMM logs, the exp-space
//       partition function parameters from VTML200) for the GPU build
//       (tools/gen_params.py --qp),
//   (2) generate golden vectors of PosteriorStage::computePairwise
//       (QP/Alignment/Multiple/PosteriorStage.cpp:123-196) under tests/golden/
//       (tests/golden/gen_golden.py).
// Nothing in the product (mlprobs_amd/, include/) links or calls this.
//
//   qp_probe params            -> tables
//   qp_probe pair SEQ1 SEQ2    -> posteriors, distance, sparse matrix
//   qp_probe bench FILE PAIRS THREADS -> reference CPU posterior-stage timing
//   qp_probe relax FILE ITERS [SEL] -> posterior stage + ITERS consistency
//                                 rounds (FILE: lines "weight sequence"; SEL: the
//                                 selectivity threshold over posterior distances)
// (records written to $REF_PROBE_OUT)

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

// Compiled with -fno-access-control: the model tables are protected members.
#include "Alignment/DataStructures/Sequence.h"
#include "Alignment/DataStructures/SparseMatrixType.h"
#include "Alignment/Multiple/BufferSet.h"
#include "Alignment/Multiple/Configuration.h"
#include "Alignment/Multiple/ExpPartitionFunctionParams.h"
#include "Alignment/Multiple/ParallelProbabilisticModel.h"
#include "Alignment/Multiple/PartitionFunction.h"
#include "Alignment/Multiple/PosteriorStage.h"
#include "Alignment/Multiple/ConsistencyStage.h"
#include "Alignment/DataStructures/MultiSequence.h"

#include <algorithm>
#include <fstream>
#include <omp.h>
#include <sstream>

using namespace quickprobs;

static FILE *g_out = nullptr;

static void rec(const char *name, char dtype, const void *data, uint64_t count) {
  uint32_t n = (uint32_t)strlen(name);
  fwrite(&n, 4, 1, g_out);
  fwrite(name, 1, n, g_out);
  fwrite(&dtype, 1, 1, g_out);
  fwrite(&count, 8, 1, g_out);
  size_t es = (dtype == 'f' || dtype == 'i') ? 4 : (dtype == 'd' || dtype == 'q') ? 8 : (dtype == 'h') ? 2 : 1;
  fwrite(data, es, count, g_out);
}

// The protein configuration QuickProbs runs MLProbs' families with
// (Configuration::setType, QP/Alignment/Multiple/Configuration.cpp:306-330).
static std::shared_ptr<Configuration> protein_config() {
  auto cfg = std::make_shared<Configuration>();
  cfg->hardware.numThreads = 1;
  cfg->setType(AlignmentType::PROTEIN);
  return cfg;
}

static Sequence *make_seq(const std::string &s, int label) {
  auto *v = new std::vector<char>();
  v->push_back('@');
  for (char c : s) v->push_back(c);
  return new Sequence(v, "s", (int)s.size(), label, label);
}

static int cmd_params() {
  auto cfg = protein_config();
  PosteriorStage stage(cfg);
  const ProbabilisticModel &m = *stage.getModel();
  rec("initial", 'f', m.initialDistribution, 5);
  rec("trans", 'f', &m.transProb[0][0], 25);
  rec("match", 'f', &m.matchProb[0][0], 256 * 256);
  rec("ins", 'f', &m.insProb[0][0], 256 * 5);
  const auto &raw = dynamic_cast<const ExpPartitionFunctionParams<double> &>(*stage.function->params).raw;
  rec("pf_term_open", 'd', &raw.termGapOpen, 1);
  rec("pf_term_extend", 'd', &raw.termGapExtend, 1);
  rec("pf_open", 'd', &raw.gapOpen, 1);
  rec("pf_extend", 'd', &raw.gapExt, 1);
  rec("pf_sub", 'd', raw.subMatrix, 26 * 26);
  const float cutoff = cfg->algorithm.posteriorCutoff;
  rec("cutoff", 'f', &cutoff, 1);
  return 0;
}

static int cmd_pair(const char *a, const char *b) {
  auto cfg = protein_config();
  PosteriorStage stage(cfg);
  std::unique_ptr<Sequence> s1(make_seq(a, 0)), s2(make_seq(b, 1));
  const int L1 = s1->GetLength(), L2 = s2->GetLength();
  const size_t layer = (size_t)(L1 + 1) * (L2 + 1);
  BufferSet buf(layer);
  float dist = 0;
  // computePairwise leaves: f2 = partition-function posterior, f1 = pair-HMM
  // posterior, f0 = their combination (PosteriorStage.cpp:123-158)
  stage.computePairwise(*s1, *s2, buf, dist);
  rec("dist", 'f', &dist, 1);
  rec("post_hmm", 'f', buf.f1(), layer);
  rec("post_pf", 'f', buf.f2(), layer);
  rec("post", 'f', buf.f0(), layer);
  // the sparse form the posterior stage keeps (PosteriorStage.cpp:104-106)
  SparseMatrixType sm(L1, L2, buf.f0(), cfg->algorithm.posteriorCutoff);
  std::vector<int32_t> rp(L1 + 2, 0);
  std::vector<uint16_t> cols, q;
  for (int i = 1; i <= L1; i++) {
    const auto *row = sm.getRowPtr(i);
    for (int k = 0; k < sm.getRowSize(i); k++) {
      cols.push_back((uint16_t)row[k].getColumn());
      q.push_back(row[k].second);  // the stored fixed-point value (SparseEntry.h:31-32)
    }
    rp[i + 1] = (int32_t)cols.size();
  }
  rec("row_ptr", 'i', rp.data(), rp.size());
  rec("cols", 'h', cols.data(), cols.size());
  rec("qvals", 'h', q.data(), q.size());
  return 0;
}

// Sparse set of all pairs (a < b) as one CSR: row_ptr per pair (L_a + 2,
// relative), 16-bit values.
static void dump_set(const char *tag, int n, Array<SparseMatrixType *> &mats) {
  std::vector<int32_t> rp;
  std::vector<uint16_t> cols, q;
  std::vector<int64_t> eo(1, 0);
  for (int a = 0; a < n; a++)
    for (int b = a + 1; b < n; b++) {
      SparseMatrixType *m = mats[a][b];
      const int L1 = m->getSeq1Length();
      const size_t base = cols.size();
      rp.push_back(0);
      rp.push_back(0);
      for (int i = 1; i <= L1; i++) {
        const auto *row = m->getRowPtr(i);
        for (int k = 0; k < m->getRowSize(i); k++) {
          cols.push_back((uint16_t)row[k].getColumn());
          q.push_back(row[k].second);
        }
        rp.push_back((int32_t)(cols.size() - base));
      }
      eo.push_back((int64_t)cols.size());
    }
  std::string t(tag);
  rec((t + ".row_ptr").c_str(), 'i', rp.data(), rp.size());
  rec((t + ".ent_off").c_str(), 'q', eo.data(), eo.size());
  rec((t + ".cols").c_str(), 'h', cols.data(), cols.size());
  rec((t + ".qvals").c_str(), 'h', q.data(), q.size());
}

// PosteriorStage::run's pair loop, then ConsistencyStage::run with the
// default configuration (QP/Alignment/Multiple/ConsistencyStage.cpp:90-128):
// the last round keeps entries >= 1e-5 instead of the 0.01 cutoff.
static int cmd_relax(const char *path, int iters, float selectivity) {
  auto cfg = protein_config();
  // selectivity > 0: the Deterministic filter's threshold (default 200, which
  // accepts every z for posterior distances <= 1); the stage reads it at
  // construction (ConsistencyStage.cpp:44-47)
  if (selectivity > 0) cfg->algorithm.consistency.selectivity = selectivity;
  std::ifstream in(path);
  std::vector<float> w;
  MultiSequence set;
  std::string line;
  while (std::getline(in, line)) {
    std::istringstream ls(line);
    float wt;
    std::string s;
    if (!(ls >> wt >> s)) continue;
    set.AddSequence(make_seq(s, (int)w.size()));
    w.push_back(wt);
  }
  const int n = (int)w.size();
  Array<float> dist(n);
  Array<SparseMatrixType *> mats(n);
  PosteriorStage post(cfg);
  post(set, dist, mats);
  std::vector<float> d;
  for (int a = 0; a < n; a++)
    for (int b = a + 1; b < n; b++) d.push_back(dist[a][b]);
  rec("dist", 'f', d.data(), d.size());
  std::vector<float> full((size_t)n * n);  // the N x N matrix the stage's filter reads
  for (int a = 0; a < n; a++)
    for (int b = 0; b < n; b++) full[(size_t)a * n + b] = dist[a][b];
  rec("seldist", 'f', full.data(), full.size());
  const float sel = cfg->algorithm.consistency.selectivity;
  rec("selectivity", 'f', &sel, 1);
  dump_set("it0", n, mats);
  ConsistencyStage cons(cfg);
  cons.selfweight = n > cfg->algorithm.consistency.selfweightThreshold ? cfg->algorithm.consistency.largeSelfweight
                                                                       : cfg->algorithm.consistency.smallSelfweight;
  for (int it = 0; it < iters; it++) {
    const bool filter = it != iters - 1;  // numFilterings < 0 (Configuration.cpp:105)
    Array<SparseMatrixType *> nm = cons.doRelaxation(w.data(), &set, dist, mats, filter);
    for (int a = 0; a < n; a++)
      for (int b = 0; b < n; b++)
        if (a != b) {
          delete mats[a][b];
          mats[a][b] = nm[a][b];
        }
    dump_set(("it" + std::to_string(it + 1)).c_str(), n, mats);
  }
  return 0;
}

// Reference CPU baseline for the QuickProbs posterior stage: PosteriorStage::
// computePairwise over the first `pairs` pairs of a family file (one sequence
// per line), OpenMP over pairs like PosteriorStage::run; prints one JSON line.
static int cmd_bench(const char *path, int pairs, int threads) {
  auto cfg = protein_config();
  std::ifstream in(path);
  std::vector<std::string> seqs;
  std::string line;
  while (std::getline(in, line))
    if (!line.empty()) seqs.push_back(line);
  const int n = (int)seqs.size();
  std::vector<std::pair<int, int>> pl;
  for (int a = 0; a < n && (int)pl.size() < pairs; a++)
    for (int b = a + 1; b < n && (int)pl.size() < pairs; b++) pl.push_back({a, b});
  std::vector<std::unique_ptr<Sequence>> sq;
  size_t maxL = 0;
  for (int k = 0; k < n; k++) {
    sq.emplace_back(make_seq(seqs[k], k));
    maxL = std::max(maxL, seqs[k].size());
  }
  PosteriorStage stage(cfg);
  omp_set_num_threads(threads);
  double cells = 0;
  for (auto &p : pl) cells += (double)(seqs[p.first].size() + 1) * (seqs[p.second].size() + 1);
  const double t0 = omp_get_wtime();
#pragma omp parallel
  {
    BufferSet buf((maxL + 1) * (maxL + 1));
#pragma omp for schedule(dynamic)
    for (int k = 0; k < (int)pl.size(); k++) {
      float d;
      stage.computePairwise(*sq[pl[k].first], *sq[pl[k].second], buf, d);
    }
  }
  const double dt = omp_get_wtime() - t0;
  printf("{\"pairs\": %d, \"seconds\": %.3f, \"pair_cells_per_s\": %.1f, \"threads\": %d}\n", (int)pl.size(), dt,
         cells / dt, threads);
  return 0;
}

int main(int argc, char **argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: qp_probe params | pair SEQ1 SEQ2\n");
    return 2;
  }
  if (std::string(argv[1]) == "bench" && argc == 5) return cmd_bench(argv[2], atoi(argv[3]), atoi(argv[4]));
  const char *outp = getenv("REF_PROBE_OUT");
  if (!outp) {
    fprintf(stderr, "set REF_PROBE_OUT\n");
    return 2;
  }
  g_out = fopen(outp, "wb");
  if (!g_out) return 3;
  const std::string cmd = argv[1];
  int rc = 2;
  if (cmd == "params") rc = cmd_params();
  else if (cmd == "pair" && argc == 4) rc = cmd_pair(argv[2], argv[3]);
  else if (cmd == "relax" && (argc == 4 || argc == 5)) rc = cmd_relax(argv[2], atoi(argv[3]), argc == 5 ? atof(argv[4]) : 0);
  fclose(g_out);
  return rc;
}
