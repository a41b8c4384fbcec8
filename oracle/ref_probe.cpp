// ref_probe.cpp -- TEST INFRASTRUCTURE ONLY (oracle side).
//
// A harness that links the *reference's own* C_P_NP_Aln objects (compiled in
// place from /root/reference/baseMSA/C_P_NP_Aln by oracle/Makefile into
// oracle/_ref/) and calls the reference functions on given inputs, dumping
// their outputs as tagged binary records.  It is used to
//   (1) generate golden vectors under tests/golden/ (tools/gen_golden.py),
//   (2) dump the reference's constant parameter tables (tools/gen_params.py),
//   (3) time the reference's own posterior pair loop as the CPU baseline
//       ("cpu_baseline.kind = reference" in bench.py).
// Nothing in the product (mlprobs_amd/, include/) links or calls this.
//
// The per-pair call sequence in cmd_family()/pair_posterior() follows
// CPNP/MSA.cpp:939-1025 (pdoAlign pair body); relaxation calls the
// reference's MSA::DoRelaxation (CPNP/MSA.cpp:1172) directly.

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <cmath>
#include <vector>
#include <string>
#include <iostream>
#include <fstream>
#include <sstream>
#include <set>
#include <list>
#include <map>
#include <algorithm>
#include <chrono>
#include <omp.h>

// Compiled with -fno-access-control so private MSA members can be called.
#include "MSA.h"

extern VF initDistrib;
extern VF gapOpen;
extern VF gapExtend;
extern VVF emitPairs;
extern VF emitSingle;
extern double sub_matrix[26][26];
extern int subst_index[26];
extern void init_arguments();
extern VF *ComputePostProbs(int a, int b, string seq1, string seq2);
// Raw constant tables, read by symbol (layout mirrors CPNP/MSAReadMatrix.h:11-14
// and CPNP/Defaults.h); only dumped, never modified.
struct RawScoreMatrix { char monomers[26]; float matrix[676]; };
extern RawScoreMatrix gonnet_160;
extern float BLOSUM62[20][20];
extern float emitPairsDefault[20][20];
extern float emitSingleDefault[20];
extern string alphabetDefault;

// Mirror of ProbabilisticModel's private data layout (CPNP/ProbabilisticModel.h:42-47).
struct ModelTables {
  float initialDistribution[5];
  float transProb[5][5];
  float matchProb[256][256];
  float insProb[256][5];
  float local_transProb[3][3];
  float random_transProb[2];
};

static FILE *g_out = nullptr;

static void rec(const char *name, char dtype, const void *data, uint64_t count) {
  uint32_t n = (uint32_t)strlen(name);
  fwrite(&n, 4, 1, g_out);
  fwrite(name, 1, n, g_out);
  fwrite(&dtype, 1, 1, g_out);
  fwrite(&count, 8, 1, g_out);
  size_t es = (dtype == 'f' || dtype == 'i') ? 4 : (dtype == 'd' || dtype == 'q') ? 8 : 1;
  fwrite(data, es, count, g_out);
}
template <class V> static void recf(const char *name, const V &v) { rec(name, 'f', v.data(), v.size()); }
static void recf1(const char *name, float x) { rec(name, 'f', &x, 1); }
static void reci1(const char *name, int x) { rec(name, 'i', &x, 1); }

static MSA *fake_msa() {
  MSA *m = (MSA *)calloc(1, sizeof(MSA));
  return m;
}

static void setup_params(MSA *m) {
  init_arguments();
  m->ReadParameters();
}

static void dump_sparse(const char *prefix, SparseMatrix *s) {
  int L1 = s->GetSeq1Length();
  std::vector<int> rs(L1 + 1, 0), cols;
  std::vector<float> vals;
  for (int i = 1; i <= L1; i++) {
    rs[i] = s->GetRowSize(i);
    auto p = s->GetRowPtr(i);
    for (int k = 0; k < rs[i]; k++) {
      cols.push_back(p[k].first);
      vals.push_back(p[k].second);
    }
  }
  std::string n = prefix;
  rec((n + ".rowsize").c_str(), 'i', rs.data(), rs.size());
  rec((n + ".cols").c_str(), 'i', cols.data(), cols.size());
  rec((n + ".vals").c_str(), 'f', vals.data(), vals.size());
}

// One pair exactly as CPNP/MSA.cpp:946-1010; returns posterior (caller deletes).
static VF *pair_posterior(ProbabilisticModel &model, Sequence *seq1, Sequence *seq2,
                          int a, int b, int pid) {
  VF *posterior;
  if (pid == 2) {
    VF *forward = model.ComputeForwardMatrix(seq1, seq2, false);
    VF *backward = model.ComputeBackwardMatrix(seq1, seq2, false);
    posterior = model.ComputePosteriorMatrix(seq1, seq2, *forward, *backward, false);
    delete forward;
    delete backward;
  } else if (pid >= 3) {
    posterior = ::ComputePostProbs(a, b, seq1->GetString(), seq2->GetString());
  } else {
    VF *forward = model.ComputeForwardMatrix(seq1, seq2);
    VF *backward = model.ComputeBackwardMatrix(seq1, seq2);
    VF *double_posterior = model.ComputePosteriorMatrix(seq1, seq2, *forward, *backward);
    delete forward;
    delete backward;
    VF *global_posterior = ::ComputePostProbs(a, b, seq1->GetString(), seq2->GetString());
    forward = model.ComputeForwardMatrix(seq1, seq2, false);
    backward = model.ComputeBackwardMatrix(seq1, seq2, false);
    posterior = model.ComputePosteriorMatrix(seq1, seq2, *forward, *backward, false);
    delete forward;
    delete backward;
    VF::iterator ptr1 = double_posterior->begin();
    VF::iterator ptr2 = global_posterior->begin();
    VF::iterator ptr = posterior->begin();
    for (int i = 0; i <= seq1->GetLength(); i++) {
      for (int j = 0; j <= seq2->GetLength(); j++) {
        float v1 = *ptr1;
        float v2 = *ptr2;
        float v3 = *ptr;
        *ptr = sqrt((v1 * v1 + v2 * v2 + v3 * v3) / 3);
        ptr1++;
        ptr2++;
        ptr++;
      }
    }
    delete double_posterior;
    delete global_posterior;
  }
  return posterior;
}

static MultiSequence *load(const char *fasta) {
  MultiSequence *s = new MultiSequence();
  s->LoadMFA(std::string(fasta), true);
  return s;
}

// params [delta]
static int cmd_params(int argc, char **argv) {
  MSA *m = fake_msa();
  setup_params(m);
  if (argc > 0) initDistrib[2] = (float)atof(argv[0]);
  ProbabilisticModel model(initDistrib, gapOpen, gapExtend, emitPairs, emitSingle);
  ModelTables t;
  static_assert(sizeof(ModelTables) == sizeof(ProbabilisticModel), "layout");
  memcpy(&t, &model, sizeof(t));
  rec("initDistrib", 'f', initDistrib.data(), initDistrib.size());
  rec("gapOpen", 'f', gapOpen.data(), gapOpen.size());
  rec("gapExtend", 'f', gapExtend.data(), gapExtend.size());
  std::vector<float> ep(256 * 256);
  for (int i = 0; i < 256; i++)
    for (int j = 0; j < 256; j++) ep[i * 256 + j] = emitPairs[i][j];
  rec("emitPairs", 'f', ep.data(), ep.size());
  rec("emitSingle", 'f', emitSingle.data(), emitSingle.size());
  rec("initialDistribution", 'f', t.initialDistribution, 5);
  rec("transProb", 'f', t.transProb, 25);
  rec("matchProb", 'f', t.matchProb, 65536);
  rec("insProb", 'f', t.insProb, 256 * 5);
  rec("local_transProb", 'f', t.local_transProb, 9);
  rec("random_transProb", 'f', t.random_transProb, 2);
  rec("sub_matrix", 'd', sub_matrix, 26 * 26);
  rec("subst_index", 'i', subst_index, 26);
  rec("gonnet.monomers", 'c', gonnet_160.monomers, 26);
  rec("gonnet.matrix", 'f', gonnet_160.matrix, 676);
  rec("blosum62", 'f', BLOSUM62, 400);
  rec("emitPairsDefault", 'f', emitPairsDefault, 400);
  rec("emitSingleDefault", 'f', emitSingleDefault, 20);
  rec("alphabet", 'c', alphabetDefault.data(), alphabetDefault.size());
  return 0;
}

// pair <fasta> <a> <b> <delta>
static int cmd_pair(int argc, char **argv) {
  if (argc < 4) return 2;
  MultiSequence *seqs = load(argv[0]);
  int a = atoi(argv[1]), b = atoi(argv[2]);
  MSA *m = fake_msa();
  setup_params(m);
  initDistrib[2] = (float)atof(argv[3]);
  ProbabilisticModel model(initDistrib, gapOpen, gapExtend, emitPairs, emitSingle);
  Sequence *s1 = seqs->GetSequence(a), *s2 = seqs->GetSequence(b);
  reci1("L1", s1->GetLength());
  reci1("L2", s2->GetLength());
  {
    VF *f = model.ComputeForwardMatrix(s1, s2, true);
    VF *bk = model.ComputeBackwardMatrix(s1, s2, true);
    VF *p = model.ComputePosteriorMatrix(s1, s2, *f, *bk, true);
    recf("hmm5.fwd", *f);
    recf("hmm5.bwd", *bk);
    recf("hmm5.post", *p);
    recf1("hmm5.total", model.ComputeTotalProbability(s1, s2, *f, *bk, true));
    auto al = model.ComputeAlignment(s1->GetLength(), s2->GetLength(), *p);
    recf1("hmm5.mea", al.second);
    delete al.first;
    delete f; delete bk; delete p;
  }
  {
    VF *f = model.ComputeForwardMatrix(s1, s2, false);
    VF *bk = model.ComputeBackwardMatrix(s1, s2, false);
    VF *p = model.ComputePosteriorMatrix(s1, s2, *f, *bk, false);
    recf("local.fwd", *f);
    recf("local.bwd", *bk);
    recf("local.post", *p);
    recf1("local.total", model.ComputeTotalProbability(s1, s2, *f, *bk, false));
    delete f; delete bk; delete p;
  }
  {
    VF *p = ::ComputePostProbs(a, b, s1->GetString(), s2->GetString());
    recf("pf.post", *p);
    delete p;
  }
  for (int pid = 0; pid <= 3; pid++) {
    if (pid == 1) continue;
    VF *p = pair_posterior(model, s1, s2, a, b, pid);
    char nm[64];
    snprintf(nm, sizeof nm, "pid%d.post", pid);
    recf(nm, *p);
    auto al = model.ComputeAlignment(s1->GetLength(), s2->GetLength(), *p);
    snprintf(nm, sizeof nm, "pid%d.mea", pid);
    recf1(nm, al.second);
    std::string path(al.first->begin(), al.first->end());
    snprintf(nm, sizeof nm, "pid%d.path", pid);
    rec(nm, 'c', path.data(), path.size());
    delete al.first;
    SparseMatrix sm(s1->GetLength(), s2->GetLength(), *p);
    snprintf(nm, sizeof nm, "pid%d.csr", pid);
    dump_sparse(nm, &sm);
    delete p;
  }
  {
    auto v = model.ComputeViterbiAlignment(s1, s2);
    std::string path(v.first->begin(), v.first->end());
    rec("viterbi.path", 'c', path.data(), path.size());
    recf1("viterbi.score", v.second);
    delete v.first;
  }
  return 0;
}

// family <fasta> <reps> [pid_override|-1] [threads]
// Runs ModelAdjustmentTest (single thread: the reference's identity sum is an
// unsynchronised OpenMP reduction, CPNP/MSA.cpp:840), the pdoAlign pair loop,
// then `reps` x MSA::DoRelaxation, dumping distances and every CSR.
static int cmd_family(int argc, char **argv) {
  if (argc < 2) return 2;
  MultiSequence *seqs = load(argv[0]);
  int reps = atoi(argv[1]);
  int pid_override = argc > 2 ? atoi(argv[2]) : -1;
  int threads = argc > 3 ? atoi(argv[3]) : 1;
  omp_set_num_threads(1);
  MSA *m = fake_msa();
  setup_params(m);
  float delta0 = initDistrib[2];
  int vm = m->ModelAdjustmentTest(seqs);
  omp_set_num_threads(threads);
  int pid = vm % 10;
  reci1("variance_mean", vm);
  recf1("delta_default", delta0);
  recf1("delta", initDistrib[2]);
  if (pid_override >= 0) pid = pid_override;
  reci1("pid", pid);
  const int n = seqs->GetNumSequences();
  reci1("N", n);
  std::vector<int> lens(n);
  for (int i = 0; i < n; i++) lens[i] = seqs->GetSequence(i)->GetLength();
  rec("lens", 'i', lens.data(), n);
  ProbabilisticModel model(initDistrib, gapOpen, gapExtend, emitPairs, emitSingle);
  SafeVector<SafeVector<SparseMatrix *> > sparse(n, SafeVector<SparseMatrix *>(n, NULL));
  std::vector<float> dist(n * n, 0.f), mea(n * n, 0.f);
  int np = n * (n - 1) / 2;
  std::vector<std::pair<int, int> > pairs;
  for (int a = 0; a < n; a++)
    for (int b = a + 1; b < n; b++) pairs.push_back({a, b});
#pragma omp parallel for schedule(dynamic)
  for (int p = 0; p < np; p++) {
    int a = pairs[p].first, b = pairs[p].second;
    Sequence *s1 = seqs->GetSequence(a), *s2 = seqs->GetSequence(b);
    VF *post = pair_posterior(model, s1, s2, a, b, pid);
    auto al = model.ComputeAlignment(s1->GetLength(), s2->GetLength(), *post);
    dist[a * n + b] = dist[b * n + a] =
        1.0f - al.second / min(s1->GetLength(), s2->GetLength());
    mea[a * n + b] = al.second;
    sparse[a][b] = new SparseMatrix(s1->GetLength(), s2->GetLength(), *post);
    delete al.first;
    delete post;
  }
  recf("distances", dist);
  recf("mea", mea);
  char nm[64];
  for (int p = 0; p < np; p++) {
    snprintf(nm, sizeof nm, "it0.p%d", p);
    dump_sparse(nm, sparse[pairs[p].first][pairs[p].second]);
  }
  m->numPairs = np;
  m->seqsPairs = new MSA::SeqsPair[np];
  for (int p = 0; p < np; p++) {
    m->seqsPairs[p].seq1 = pairs[p].first;
    m->seqsPairs[p].seq2 = pairs[p].second;
  }
  for (int r = 0; r < reps; r++) {
    SafeVector<SafeVector<SparseMatrix *> > ns = m->DoRelaxation(seqs, sparse);
    for (int i = 0; i < n; i++)
      for (int j = 0; j < n; j++) {
        delete sparse[i][j];
        sparse[i][j] = ns[i][j];
      }
    for (int p = 0; p < np; p++) {
      snprintf(nm, sizeof nm, "it%d.p%d", r + 1, p);
      dump_sparse(nm, sparse[pairs[p].first][pairs[p].second]);
    }
  }
  return 0;
}

// Per-pair sparse dump (bench and relaxbench): int64 count, then per pair
// int32 a, int32 b, int32 L1, float dist, float mea, int64 nnz,
// int32 rowptr[L1 + 2] (pair-local), int32 cols[nnz], float vals[nnz].
static void dump_pairs(const char *path, const std::vector<std::pair<int, int> > &pairs,
                       const std::vector<SparseMatrix *> &sm, const std::vector<float> &dist,
                       const std::vector<float> &mea) {
  FILE *f = fopen(path, "wb");
  if (!f) { fprintf(stderr, "cannot write %s\n", path); exit(3); }
  int64_t np = pairs.size();
  fwrite(&np, 8, 1, f);
  std::vector<int32_t> rp, cols;
  std::vector<float> vals;
  for (int64_t p = 0; p < np; p++) {
    SparseMatrix *m = sm[p];
    int32_t hdr[3] = {pairs[p].first, pairs[p].second, m->GetSeq1Length()};
    fwrite(hdr, 4, 3, f);
    float dm[2] = {dist.empty() ? 0.f : dist[p], mea.empty() ? 0.f : mea[p]};
    fwrite(dm, 4, 2, f);
    const int L1 = m->GetSeq1Length();
    rp.assign(L1 + 2, 0);
    cols.clear();
    vals.clear();
    for (int i = 1; i <= L1; i++) {
      auto r = m->GetRowPtr(i);
      for (int k = 0; k < m->GetRowSize(i); k++) {
        cols.push_back(r[k].first);
        vals.push_back(r[k].second);
      }
      rp[i + 1] = (int32_t)cols.size();
    }
    int64_t nnz = cols.size();
    fwrite(&nnz, 8, 1, f);
    fwrite(rp.data(), 4, rp.size(), f);
    fwrite(cols.data(), 4, cols.size(), f);
    fwrite(vals.data(), 4, vals.size(), f);
  }
  fclose(f);
}

// bench <fasta> <pid> <maxpairs> <threads> [dump]  -> JSON on stdout
// Times the reference's pdoAlign pair body (posterior + MEA + sparsify,
// CPNP/MSA.cpp:939-1025) over the first `maxpairs` pairs in reference order;
// with `dump`, writes their sparse matrices, distances and MEA scores there
// afterwards (same-run parity readouts in bench.py).
static int cmd_bench(int argc, char **argv) {
  if (argc < 4) return 2;
  MultiSequence *seqs = load(argv[0]);
  int pid = atoi(argv[1]);
  long maxpairs = atol(argv[2]);
  int threads = atoi(argv[3]);
  const char *dump = argc > 4 ? argv[4] : nullptr;
  MSA *m = fake_msa();
  setup_params(m);
  if (getenv("REF_PROBE_DELTA")) initDistrib[2] = (float)atof(getenv("REF_PROBE_DELTA"));
  ProbabilisticModel model(initDistrib, gapOpen, gapExtend, emitPairs, emitSingle);
  const int n = seqs->GetNumSequences();
  std::vector<std::pair<int, int> > pairs;
  for (int a = 0; a < n && (long)pairs.size() < maxpairs; a++)
    for (int b = a + 1; b < n && (long)pairs.size() < maxpairs; b++) pairs.push_back({a, b});
  long np = pairs.size();
  double cells = 0;
  for (auto &pr : pairs)
    cells += (double)(seqs->GetSequence(pr.first)->GetLength() + 1) *
             (seqs->GetSequence(pr.second)->GetLength() + 1);
  omp_set_num_threads(threads);
  std::vector<float> dist(np), mea(np);
  std::vector<SparseMatrix *> sm(np, nullptr);
  auto t0 = std::chrono::steady_clock::now();
#pragma omp parallel for schedule(dynamic)
  for (long p = 0; p < np; p++) {
    int a = pairs[p].first, b = pairs[p].second;
    Sequence *s1 = seqs->GetSequence(a), *s2 = seqs->GetSequence(b);
    VF *post = pair_posterior(model, s1, s2, a, b, pid);
    auto al = model.ComputeAlignment(s1->GetLength(), s2->GetLength(), *post);
    dist[p] = 1.0f - al.second / min(s1->GetLength(), s2->GetLength());
    mea[p] = al.second;
    sm[p] = new SparseMatrix(s1->GetLength(), s2->GetLength(), *post);
    delete al.first;
    delete post;
  }
  auto t1 = std::chrono::steady_clock::now();
  double sec = std::chrono::duration<double>(t1 - t0).count();
  if (dump) dump_pairs(dump, pairs, sm, dist, mea);
  for (auto *x : sm) delete x;
  printf("{\"pairs\": %ld, \"pair_cells\": %.0f, \"seconds\": %.6f, \"threads\": %d, "
         "\"pair_cells_per_s\": %.6e}\n",
         np, cells, sec, threads, cells / sec);
  return 0;
}

// npdo <fasta> <pid> <delta> <dump>
// The reference's own ArrangePosteriorProbs (CPNP/MSA.cpp:1636-1765, the
// npdoAlign pair loop) over every pair: sparse matrices and the distances
// score / #B, in the dump_pairs format (mea field unused).
static int cmd_npdo(int argc, char **argv) {
  if (argc < 4) return 2;
  MultiSequence *seqs = load(argv[0]);
  const int pid = atoi(argv[1]);
  MSA *m = fake_msa();
  setup_params(m);
  initDistrib[2] = (float)atof(argv[2]);
  ProbabilisticModel model(initDistrib, gapOpen, gapExtend, emitPairs, emitSingle);
  const int n = seqs->GetNumSequences();
  std::vector<std::pair<int, int> > pairs;
  for (int a = 0; a < n; a++)
    for (int b = a + 1; b < n; b++) pairs.push_back({a, b});
  m->numPairs = (int)pairs.size();
  m->seqsPairs = new MSA::SeqsPair[pairs.size()];
  for (size_t k = 0; k < pairs.size(); k++) {
    m->seqsPairs[k].seq1 = pairs[k].first;
    m->seqsPairs[k].seq2 = pairs[k].second;
  }
  SafeVector<SafeVector<SparseMatrix *> > sparse(n, SafeVector<SparseMatrix *>(n, NULL));
  VVF distances(n, VF(n, 0));
  m->ArrangePosteriorProbs(seqs, model, sparse, distances, pid);
  std::vector<SparseMatrix *> sm;
  std::vector<float> dist;
  for (auto &pr : pairs) {
    sm.push_back(sparse[pr.first][pr.second]);
    dist.push_back(distances[pr.first][pr.second]);
  }
  dump_pairs(argv[3], pairs, sm, dist, {});
  return 0;
}

// relaxbench <fasta> <store> <sample> <threads> <dump>  -> JSON on stdout
// Times the reference's MSA::DoRelaxation (CPNP/MSA.cpp:1172-1281, its own
// pair loop over seqsPairs) on a strided sample of `sample` output pairs,
// with every input block present.  The input is a sparse set in the
// canonical layout of include/mlpgpu.h written by bench.py (int64 P, int64
// total, int32 row_ptr, int64 ent_off[P + 1], uint16 cols, float vals),
// loaded into the reference's own SparseMatrix objects.  The sample's output
// matrices go to `dump` (dump_pairs format).
static int cmd_relaxbench(int argc, char **argv) {
  if (argc < 5) return 2;
  MultiSequence *seqs = load(argv[0]);
  const long sample = atol(argv[2]);
  const int threads = atoi(argv[3]);
  const int n = seqs->GetNumSequences();
  FILE *f = fopen(argv[1], "rb");
  if (!f) return 3;
  int64_t P = 0, total = 0;
  if (fread(&P, 8, 1, f) != 1 || fread(&total, 8, 1, f) != 1 || P != (int64_t)n * (n - 1) / 2) return 4;
  std::vector<int> lens(n);
  for (int i = 0; i < n; i++) lens[i] = seqs->GetSequence(i)->GetLength();
  std::vector<std::pair<int, int> > pairs;
  std::vector<int64_t> roff(P + 1, 0);
  for (int a = 0; a < n; a++)
    for (int b = a + 1; b < n; b++) {
      roff[pairs.size() + 1] = roff[pairs.size()] + lens[a] + 2;
      pairs.push_back({a, b});
    }
  std::vector<int32_t> rp(roff[P]);
  std::vector<int64_t> eo(P + 1);
  std::vector<uint16_t> cols(std::max<int64_t>(total, 1));
  std::vector<float> vals(std::max<int64_t>(total, 1));
  if (fread(rp.data(), 4, rp.size(), f) != rp.size() || fread(eo.data(), 8, P + 1, f) != (size_t)(P + 1) ||
      fread(cols.data(), 2, total, f) != (size_t)total || fread(vals.data(), 4, total, f) != (size_t)total)
    return 5;
  fclose(f);
  omp_set_num_threads(threads);
  MSA *m = fake_msa();
  SafeVector<SafeVector<SparseMatrix *> > sparse(n, SafeVector<SparseMatrix *>(n, NULL));
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t p = 0; p < P; p++) {
    const int a = pairs[p].first, b = pairs[p].second, L1 = lens[a];
    const int32_t *r = rp.data() + roff[p];
    SparseMatrix *s = new SparseMatrix();  // the reference's own layout (SparseMatrix.h:28-33)
    s->seq1Length = L1;
    s->seq2Length = lens[b];
    const int64_t nnz = r[L1 + 1];
    s->data.resize(nnz);
    for (int64_t k = 0; k < nnz; k++) {
      s->data[k].first = cols[eo[p] + k];
      s->data[k].second = vals[eo[p] + k];
    }
    s->rowSize.resize(L1 + 1);
    s->rowSize[0] = -1;
    s->rowPtrs.resize(L1 + 1);
    s->rowPtrs[0] = s->data.end();
    for (int i = 1; i <= L1; i++) {
      s->rowPtrs[i] = s->data.begin() + r[i];
      s->rowSize[i] = r[i + 1] - r[i];
    }
    sparse[a][b] = s;
  }
  std::vector<std::pair<int, int> > pick;
  const int64_t stride = std::max<int64_t>(1, P / std::max<long>(sample, 1));
  for (int64_t p = 0; p < P && (long)pick.size() < sample; p += stride) pick.push_back(pairs[p]);
  m->numPairs = (int)pick.size();
  m->seqsPairs = new MSA::SeqsPair[pick.size()];
  for (size_t k = 0; k < pick.size(); k++) {
    m->seqsPairs[k].seq1 = pick[k].first;
    m->seqsPairs[k].seq2 = pick[k].second;
  }
  auto t0 = std::chrono::steady_clock::now();
  SafeVector<SafeVector<SparseMatrix *> > ns = m->DoRelaxation(seqs, sparse);
  auto t1 = std::chrono::steady_clock::now();
  double sec = std::chrono::duration<double>(t1 - t0).count();
  std::vector<SparseMatrix *> out;
  for (auto &pr : pick) out.push_back(ns[pr.first][pr.second]);
  dump_pairs(argv[4], pick, out, {}, {});
  printf("{\"pairs\": %zu, \"stride\": %ld, \"seconds\": %.6f, \"threads\": %d}\n", pick.size(), (long)stride, sec,
         threads);
  return 0;
}

int main(int argc, char **argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: ref_probe params|pair|family|bench|relaxbench ...\n");
    return 2;
  }
  std::string cmd = argv[1];
  if (cmd == "bench") return cmd_bench(argc - 2, argv + 2);
  if (cmd == "relaxbench") return cmd_relaxbench(argc - 2, argv + 2);
  if (cmd == "npdo") return cmd_npdo(argc - 2, argv + 2);
  const char *outp = getenv("REF_PROBE_OUT");
  if (!outp) {
    fprintf(stderr, "set REF_PROBE_OUT\n");
    return 2;
  }
  g_out = fopen(outp, "wb");
  if (!g_out) return 3;
  int rc = 2;
  if (cmd == "params") rc = cmd_params(argc - 2, argv + 2);
  else if (cmd == "pair") rc = cmd_pair(argc - 2, argv + 2);
  else if (cmd == "family") rc = cmd_family(argc - 2, argv + 2);
  fclose(g_out);
  return rc;
}
