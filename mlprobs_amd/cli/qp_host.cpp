// qp_host.cpp -- see qp_host.h.
#include "qp_host.h"

#include <math.h>
#include <chrono>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cctype>
#include <limits>
#include <numeric>
#include <set>
#include <stdexcept>

#include "msa_host.h"  // cpnp::mea_path: QuickProbs' computeAlignment is the same MEA recurrence
#include "pool.h"

namespace qph {

// ------------------------------------------------------------------ FASTA
bool load_fasta(const std::string& path, std::vector<Seq>& seqs, std::string& out_msg, std::string& err) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) {
    err = "SequenceIO::load(): unable to open input file.";
    return false;
  }
  std::string buf;
  char tmp[1 << 16];
  size_t got;
  while ((got = fread(tmp, 1, sizeof tmp, f)) > 0) buf.append(tmp, got);
  fclose(f);
  return load_fasta_text(buf, seqs, out_msg, err);
}

bool load_fasta_text(const std::string& buf, std::vector<Seq>& seqs, std::string& out_msg, std::string& err) {
  // std::istream::getline(buffer, MAX_LINE_LENGTH = 10000) semantics
  // (SequenceIO.h:64): a line of 10000+ characters stores its first 9999 and
  // fails the stream, which ends the read; a final unterminated line counts.
  size_t pos = 0;
  bool good = true;
  auto getline = [&](std::string& s) {
    s.clear();
    if (pos >= buf.size()) {
      good = false;
      return;
    }
    const size_t e = buf.find('\n', pos);
    const size_t end = e == std::string::npos ? buf.size() : e;
    if (end - pos >= 10000) {
      s.assign(buf, pos, 9999);
      good = false;
      return;
    }
    s.assign(buf, pos, end - pos);
    pos = e == std::string::npos ? buf.size() : e + 1;
    if (pos >= buf.size()) good = false;  // eofbit once the last line is read
  };
  auto peek_is_header = [&]() { return pos < buf.size() && buf[pos] == '>'; };
  seqs.clear();
  std::string line;
  // SequenceIO::loadFasta (SequenceIO.cpp:84-135)
  while (good) {
    getline(line);
    if (line.empty() || line[0] != '>') continue;
    std::string header = line.substr(1);
    while (!header.empty() && isspace((unsigned char)header[0])) header.erase(0, 1);
    while (!header.empty() && isspace((unsigned char)header.back())) header.pop_back();
    Seq s;
    s.header = header;
    s.data = "@";
    while (good) {
      if (peek_is_header()) break;
      getline(line);
      if (line.empty()) continue;
      if (line.back() == '\r') line.pop_back();
      s.data += line;
    }
    s.sort_label = s.label = (int)seqs.size();
    seqs.push_back(std::move(s));
  }
  if (seqs.empty()) {
    err = "SequenceIO::loadFasta(): no sequences read.";
    return false;
  }
  // SequenceIO::checkAndCorrect (SequenceIO.cpp:60-80)
  bool ok = true;
  for (Seq& s : seqs)
    for (size_t i = 1; i < s.data.size(); i++) {
      char& c = s.data[i];
      if (c == '.') c = '-';
      else if (isalpha((unsigned char)c)) c = (char)toupper((unsigned char)c);
      else {
        out_msg += std::string("illegal sequence character:") + c + "\n";
        ok = false;
      }
    }
  if (!ok) {
    err = "Illegal characters in sequence set!";
    return false;
  }
  return true;
}

void write_fasta(std::string& out, const Profile& p) {
  // 60-column lines, appended a line at a time
  size_t total = out.size();
  for (const Seq& s : p) total += s.header.size() + 2 + (size_t)s.length() + s.length() / 60 + 1;
  out.reserve(total);
  for (const Seq& s : p) {
    out += '>';
    out += s.header;
    out += '\n';
    const int L = s.length();
    for (int c0 = 1; c0 <= L; c0 += 60) {
      out.append(s.data, (size_t)c0, (size_t)std::min(60, L - c0 + 1));
      out += '\n';
    }
  }
}

// ------------------------------------------------------------------ sparse set
void Sparse::build_views() {
  const int64_t P = (int64_t)n * (n - 1) / 2;
  blocks.assign((size_t)n * n, Block{});
  // transposed blocks: L_b + 2 row pointers per pair, entries at the same offsets
  std::vector<int64_t> trp_off(P + 1, 0);
  for (int a = 0, p = 0; a < n; a++)
    for (int b = a + 1; b < n; b++, p++) trp_off[p + 1] = trp_off[p] + lens[b] + 2;
  trow_ptr.assign(P > 0 ? trp_off[P] : 1, 0);
  tcols.resize(cols.size());
  tvals.resize(vals.size());
  mlpr::parallel_for_dynamic(P, mlpr::host_threads(), [&](int64_t p) {
    int a = 0;
    int64_t q = p;
    while (q >= n - 1 - a) { q -= n - 1 - a; ++a; }
    const int b = a + 1 + (int)q;
    const int32_t* rp = row_ptr.data() + rp_off[p];
    const uint16_t* c = cols.data() + ent_off[p];
    const float* v = vals.data() + ent_off[p];
    int32_t* trp = trow_ptr.data() + trp_off[p];
    uint16_t* tc = tcols.data() + ent_off[p];
    float* tv = tvals.data() + ent_off[p];
    const int La = lens[a], Lb = lens[b];
    // rows of the transpose: columns of P(a, b), entries in ascending i
    // (PackedSparseMatrix::fillTransposed, QP/Alignment/DataStructures/PackedSparseMatrix.cpp:101-140)
    std::vector<int32_t> cnt(Lb + 2, 0);
    for (int e = rp[1]; e < rp[La + 1]; e++) cnt[c[e]]++;
    trp[0] = 0;
    trp[1] = 0;
    for (int j = 1; j <= Lb; j++) trp[j + 1] = trp[j] + cnt[j];
    std::vector<int32_t> cur(trp, trp + Lb + 2);
    for (int i = 1; i <= La; i++)
      for (int e = rp[i]; e < rp[i + 1]; e++) {
        const int k = cur[c[e]]++;
        tc[k] = (uint16_t)i;
        tv[k] = v[e];
      }
  });
  for (int a = 0, p = 0; a < n; a++)
    for (int b = a + 1; b < n; b++, p++) {
      blocks[(size_t)a * n + b] = Block{row_ptr.data() + rp_off[p], cols.data() + ent_off[p], vals.data() + ent_off[p]};
      blocks[(size_t)b * n + a] =
          Block{trow_ptr.data() + trp_off[p], tcols.data() + ent_off[p], tvals.data() + ent_off[p]};
    }
}

// ------------------------------------------------------------------ guide tree
// ClusterTree::build (QP/Alignment/Multiple/ClusterTree.cpp:22-140): closest
// pair first in (i ascending, j < i ascending) order with a strict '<' from
// 2.0; the merged cluster keeps row i; average linkage in float.
Tree build_tree(std::vector<float> D, int n) {
  Tree T;
  T.n = n;
  T.nodes.assign(2 * (size_t)n + 1, Tree::Node{});
  for (int i = 0; i < n; i++) T.nodes[i].leaf = true;
  std::vector<unsigned> cluster_leafs(T.nodes.size() + 1, 0);
  for (int i = 0; i < n; i++) cluster_leafs[i] = 1;
  std::vector<int> rows(n), node(n);  // the valid list, rows ascending
  for (int i = 0; i < n; i++) rows[i] = node[i] = i;
  std::vector<float> joins(n + 1);
  for (int nodeIdx = n; nodeIdx < 2 * n - 1; nodeIdx++) {
    float minDist = 2.0f;
    int bi = -1, bj = -1;
    const int len = (int)rows.size();
    for (int a = 0; a < len; a++) {
      const int mini = rows[a];
      for (int b = 0; b < len && rows[b] < mini; b++) {
        const float d = D[(size_t)mini * n + rows[b]];
        if (d < 0) throw std::runtime_error("ERROR: It is impossible to have distance value less than zero");
        if (d < minDist) {
          minDist = d;
          bi = a;
          bj = b;
        }
      }
    }
    if (bi < 0) throw std::runtime_error("OOPS: Error occurred while constructing the cluster tree\n");
    const float branch = minDist * 0.5f;
    const int li = node[bi], rj = node[bj];
    T.nodes[li].parent = nodeIdx;
    T.nodes[li].dist = branch;
    T.nodes[rj].parent = nodeIdx;
    T.nodes[rj].dist = branch;
    T.nodes[nodeIdx].left = li;
    T.nodes[nodeIdx].right = rj;
    cluster_leafs[nodeIdx] = cluster_leafs[li] + cluster_leafs[rj];
    const int mi = rows[bi], mj = rows[bj];
    rows.erase(rows.begin() + bj);
    node.erase(node.begin() + bj);
    const int bi2 = bi - 1;  // bj < bi
    const unsigned isize = cluster_leafs[li], jsize = cluster_leafs[rj];
    for (int c = 0; c < (int)rows.size(); c++) {
      const int idx = rows[c];
      const float idist = D[(size_t)mi * n + idx], jdist = D[(size_t)mj * n + idx];
      joins[idx] = (idist * isize + jdist * jsize) / (isize + jsize);
    }
    node[bi2] = nodeIdx;
    for (int c = 0; c < (int)rows.size(); c++) {
      const int mn = rows[c];
      D[(size_t)mi * n + mn] = joins[mn];
      D[(size_t)mn * n + mi] = joins[mn];
    }
  }
  T.root = n >= 1 ? 2 * n - 2 : -1;
  // GuideTree::calculateSeqsWeights (GuideTree.cpp:117-160)
  for (int i = 0; i < n; i++)
    for (int cur = i; cur != -1; cur = T.nodes[cur].parent) {
      ++T.nodes[cur].order;
      ++T.nodes[i].depth;
    }
  T.weights.assign(n, 0.f);
  for (int i = 0; i < n; i++) {
    float w = 0;
    for (int cur = i; T.nodes[cur].parent != -1; cur = T.nodes[cur].parent) w += T.nodes[cur].dist / T.nodes[cur].order;
    T.weights[i] = w;
  }
  float wsum = std::accumulate(T.weights.begin(), T.weights.end(), 0.0f);
  if (wsum == 0) {
    std::fill(T.weights.begin(), T.weights.end(), 1.0f);
    wsum = (float)n;
  }
  for (float& w : T.weights) w = w / wsum;
  return T;
}

// GuideTree::calculateSubtreeDistances (GuideTree.cpp:195-224): for i != j,
// the sizes of the two subtrees just below their lowest common ancestor.
std::vector<float> Tree::subtree_distances() const {
  std::vector<float> d((size_t)n * n, 0.f);
  std::vector<std::vector<int>> paths(n);
  for (int i = 0; i < n; i++)
    for (int cur = i; cur != -1; cur = nodes[cur].parent) paths[i].push_back(cur);
  for (int i = 0; i < n; i++)
    for (int j = i + 1; j < n; j++) {
      const std::vector<int>& p1 = paths[i].size() > paths[j].size() ? paths[i] : paths[j];
      const std::vector<int>& p2 = paths[i].size() > paths[j].size() ? paths[j] : paths[i];
      size_t k = 0;  // common suffix (the root side)
      while (p1[p1.size() - 1 - k] == p2[p2.size() - 1 - k]) k++;
      const int id1 = p1[p1.size() - 1 - k], id2 = p2[p2.size() - 1 - k];
      const float v = (float)(size_t)(nodes[id1].order + nodes[id2].order);
      d[(size_t)i * n + j] = d[(size_t)j * n + i] = v;
    }
  return d;
}

// ------------------------------------------------------------------ construction
namespace {

// Sequence::getMapping (QP/Alignment/DataStructures/Sequence.cpp:112-121)
void mapping(const Seq& s, std::vector<int>& m) {
  m.assign(s.length() + 1, 0);
  for (int i = 1, j = 1; i <= s.length(); i++)
    if (s.data[i] != '-') m[j++] = i;
}

// ParallelProbabilisticModel::buildPosterior (QP/Alignment/Multiple/
// ParallelProbabilisticModel.cpp:301-430), construction selectivity FLT_MAX
// (every pair): weights w1 w2 / sum(w1 w2) in double, cast to float; each
// cell accumulates in (i, j, row, entry) order.  Threads own disjoint ranges
// of dense rows, which keeps that order per cell.
void build_posterior(const std::vector<float>& w, const Profile& A, const Profile& B, const Sparse& sp,
                     std::vector<float>& post, int threads) {
  const int L1 = A[0].length(), L2 = B[0].length(), W2 = L2 + 1;
  if (post.size() < (size_t)(L1 + 1) * W2) post.resize((size_t)(L1 + 1) * W2);
  std::fill(post.begin(), post.begin() + W2, 0.f);  // row 0 (the threads zero rows 1..L1)
  double total = 0;
  for (const Seq& a : A) {
    const double w1 = w[a.label];
    for (const Seq& b : B) total += w1 * (double)w[b.label];
  }
  std::vector<std::vector<int>> m1(A.size()), m2(B.size());
  for (size_t i = 0; i < A.size(); i++) mapping(A[i], m1[i]);
  for (size_t j = 0; j < B.size(); j++) mapping(B[j], m2[j]);
  const int nt = std::max(1, std::min(threads, L1 / 16));
  mlpr::parallel(nt, [&](int t, int T) {
    const int r0 = 1 + (int)((int64_t)L1 * t / T), r1 = 1 + (int)((int64_t)L1 * (t + 1) / T);  // dense rows [r0, r1)
    std::fill(post.begin() + (size_t)r0 * W2, post.begin() + (size_t)r1 * W2, 0.f);
    for (size_t i = 0; i < A.size(); i++) {
      const int first = A[i].label;
      const std::vector<int>& map1 = m1[i];
      const double w1 = w[first];
      const int La = sp.lens[first];
      // rows ii whose dense row falls in [r0, r1): map1 is increasing
      const int ii0 = (int)(std::lower_bound(map1.begin() + 1, map1.begin() + La + 1, r0) - map1.begin());
      const int ii1 = (int)(std::lower_bound(map1.begin() + 1, map1.begin() + La + 1, r1) - map1.begin());
      if (ii0 >= ii1) continue;
      for (size_t j = 0; j < B.size(); j++) {
        const int second = B[j].label;
        const int* map2 = m2[j].data();
        const double w2 = w[second];
        const float wf = (float)((w1 * w2) / total);
        const Sparse::Block& blk = sp.at(first, second);
        for (int ii = ii0; ii < ii1; ii++) {
          float* base = post.data() + (size_t)map1[ii] * W2;
          for (int e = blk.rp[ii]; e < blk.rp[ii + 1]; e++) base[map2[blk.cols[e]]] += wf * blk.vals[e];
        }
      }
    }
  });
}

// Sequence::AddGaps (Sequence.cpp:67-92)
Seq add_gaps(const Seq& s, const std::string& path, char id) {
  Seq r;
  r.header = s.header;
  r.sort_label = s.sort_label;
  r.label = s.label;
  r.data.assign(path.size() + 1, '-');
  r.data[0] = '@';
  const char* src = s.data.data() + 1;
  char* dst = &r.data[1];
  for (size_t c = 0; c < path.size(); c++)
    if (path[c] == 'B' || path[c] == id) dst[c] = *src++;
  return r;
}

// time split of the host stages (MLP_CLI_TIMES)
double g_t_post = 0, g_t_mea = 0, g_t_merge = 0, g_t_update = 0, g_t_split = 0;
int64_t g_n_terms = 0;
double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

// ConstructionStage::alignAlignments (ConstructionStage.cpp:86-126)
Profile align_alignments(const std::vector<float>& w, const Profile& A, const Profile& B, const PosteriorBackend& be,
                         std::vector<float>& post, int threads) {
  const double t0 = now();
  float score;
  std::string path;
  if (be.device_mea && be.device_mea(w, A, B, path, &score)) {
    g_t_mea += now() - t0;
  } else {
    const float* P = be.device ? be.device(w, A, B) : nullptr;
    if (!P) {
      build_posterior(w, A, B, be.host_sparse(), post, threads);
      P = post.data();
    }
    const double t1 = now();
    path = cpnp::mea_path(A[0].length(), B[0].length(), P, &score);
    g_t_post += t1 - t0;
    g_t_mea += now() - t1;
  }
  g_n_terms += (int64_t)A.size() * (int64_t)B.size();
  const double t2 = now();
  Profile r(A.size() + B.size());
  const int na = (int)A.size(), nr = (int)r.size();
  const int nt = (int64_t)nr * (int64_t)path.size() > 200000 ? std::max(1, threads) : 1;
  mlpr::parallel_for(nr, nt, [&](int64_t k) { r[k] = k < na ? add_gaps(A[k], path, 'X') : add_gaps(B[k - na], path, 'Y'); });
  // MultiSequence::SortByLabel (the labels are distinct)
  std::sort(r.begin(), r.end(), [](const Seq& a, const Seq& b) { return a.sort_label < b.sort_label; });
  g_t_merge += now() - t2;
  return r;
}

// ConstructionStage::processTree (ConstructionStage.cpp:52-84)
Profile process_tree(const Tree& T, int node, const std::vector<Seq>& seqs, const std::vector<float>& w,
                     const PosteriorBackend& be, std::vector<float>& post, int threads) {
  const Tree::Node& nd = T.nodes[node];
  if (nd.leaf) return Profile{seqs[node]};
  const Profile l = process_tree(T, nd.left, seqs, w, be, post, threads);
  const Profile r = process_tree(T, nd.right, seqs, w, be, post, threads);
  return align_alignments(w, l, r, be, post, threads);
}

// MultiSequence::extractSubset (QP/Alignment/DataStructures/MultiSequence.cpp:407-464)
Profile extract_subset(const Profile& aln, const std::set<int>& idx, int threads) {
  const int L = aln[*idx.begin()].length();
  const std::vector<int> rows(idx.begin(), idx.end());
  const int nt = (int64_t)rows.size() * L > 200000 ? std::max(1, threads) : 1;
  std::vector<char> keep(L + 1, 0);
  // columns not gapped in every selected row (column blocks in parallel)
  mlpr::parallel_for((L + 255) / 256, nt, [&](int64_t blk) {
    const int c0 = 1 + 256 * (int)blk, c1 = std::min(L, c0 + 255);
    for (int i : rows) {
      const char* d = aln[i].data.data();
      for (int c = c0; c <= c1; c++) keep[c] |= d[c] != '-';
    }
  });
  std::vector<int> cols;
  for (int c = 1; c <= L; c++)
    if (keep[c]) cols.push_back(c);
  Profile r(rows.size());
  mlpr::parallel_for((int64_t)rows.size(), nt, [&](int64_t k) {
    const Seq& src = aln[rows[k]];
    Seq& s = r[k];
    s.header = src.header;
    s.sort_label = src.sort_label;
    s.label = src.label;
    s.data.resize(cols.size() + 1);
    s.data[0] = '@';
    const char* d = src.data.data();
    for (size_t q = 0; q < cols.size(); q++) s.data[q + 1] = d[cols[q]];
  });
  return r;
}

// det_uniform_int_distribution<int>(lo, hi) over std::mt19937
// (QP/Common/deterministic_random.h): rejection of the biased tail, then mod.
int det_uniform(std::mt19937& g, int lo, int hi) {
  const unsigned diff = (unsigned)hi - (unsigned)lo + 1u;
  if (diff == 0) return (int)g();
  const unsigned bad = std::numeric_limits<unsigned>::max() / diff;
  for (;;) {
    const unsigned r = (unsigned)g();
    if (r / diff < bad) return (int)(r % diff + (unsigned)lo);
  }
}

// ColumnRefinement (QP/Alignment/Multiple/ColumnRefinement.cpp) with its
// defaults: column fraction 1, no recursion (maxDepth 0), length acceptance.
struct ColumnRefiner {
  std::vector<std::pair<int, float>> scores;  // persists between calls, like the member columnScores
  std::mt19937 engine;                        // default seed (ref-seed 0)
  int cfg_iterations;                         // config refinement.iterations (-1 unless -r)

  // updateColumnScores (ColumnRefinement.cpp:120-174): resize keeps the
  // previous call's (sorted, filtered) entries at the front, and the gap
  // counts are added onto them.
  void update(const Profile& aln, int threads) {
    const int n = (int)aln.size(), L = aln[0].length();
    scores.resize(L, std::pair<int, float>(0, 0));
    // gap counts per column; adding them at once equals adding 1.0f per gap
    // (integers below 2^24 are exact in float); column blocks in parallel
    std::vector<int> gaps(L, 0);
    const int nt = (int64_t)n * L > 200000 ? std::max(1, threads) : 1;
    mlpr::parallel_for((L + 255) / 256, nt, [&](int64_t blk) {
      const int c0 = 256 * (int)blk, c1 = std::min(L, c0 + 256);
      for (int i = 0; i < n; i++) {
        const char* d = aln[i].data.data() + 1;
        for (int c = c0; c < c1; c++) gaps[c] += d[c] == '-';
      }
    });
    for (int c = 0; c < (int)scores.size(); c++) {
      scores[c].first = c;
      scores[c].second += (float)gaps[c];
    }
    std::stable_sort(scores.begin(), scores.end(), [n](const std::pair<int, float>& a, const std::pair<int, float>& b) {
      return fabsf((float)n / 2 - a.second) > fabsf((float)n / 2 - b.second);
    });
    scores.erase(std::remove_if(scores.begin(), scores.end(),
                                [](const std::pair<int, float>& e) { return e.second == 0; }),
                 scores.end());
  }
  int hi() const {
    const int used = (int)((float)scores.size() * 1.0f);
    return std::min(std::max(used, cfg_iterations), (int)scores.size());
  }
};

}  // namespace

std::vector<int32_t> profile_maps(const Profile& p, int threads) {
  // Sequence::getMapping of every row, appended: row k's map has one entry
  // per residue plus the leading 0, so every row's offset is known up front
  // and the rows are filled independently (a refinement pass maps all n
  // rows, ~2e5 entries at 512 x 400: on the host threads when that large)
  std::vector<int64_t> off(p.size() + 1, 0);
  const int64_t cells = (int64_t)p.size() * (p.empty() ? 0 : p[0].length());
  const int nt = cells > 200000 ? std::max(1, threads) : 1;
  mlpr::parallel_for((int64_t)p.size(), nt, [&](int64_t k) {
    const char* d = p[k].data.data();
    int64_t res = 0;
    for (int i = 1, L = p[k].length(); i <= L; i++) res += d[i] != '-';
    off[k + 1] = res + 1;
  });
  for (size_t k = 0; k < p.size(); k++) off[k + 1] += off[k];
  std::vector<int32_t> out((size_t)off[p.size()]);
  mlpr::parallel_for((int64_t)p.size(), nt, [&](int64_t k) {
    int32_t* o = out.data() + off[k];
    *o++ = 0;
    const char* d = p[k].data.data();
    for (int i = 1, L = p[k].length(); i <= L; i++)
      if (d[i] != '-') *o++ = i;
  });
  return out;
}

Profile construct_and_refine(const std::vector<Seq>& seqs, const PosteriorBackend& be, const Tree& tree,
                             const Options& opt, int threads) {
  const int n = (int)seqs.size();
  // ExtendedMSA::doAlign (ExtendedMSA.cpp:178-186): weights saturated at 1e-6
  std::vector<float> w = tree.weights;
  for (float& x : w) x = std::max(x, 1e-6f);
  std::vector<float> post;
  Profile aln = process_tree(tree, tree.root, seqs, w, be, post, threads);
  // RefinementBase::operator() (RefinementBase.cpp:13-49)
  const int iters = opt.refinement > 0 ? opt.refinement : (n > 200 ? 200 : 30);
  ColumnRefiner cr;
  cr.cfg_iterations = opt.refinement;
  cr.update(aln, threads);  // initialise (ColumnRefinement.cpp:64-80)
  const bool prepared = cr.hi() > 0;
  for (int it = 0; it < iters && prepared; it++) {
    // split (ColumnRefinement.cpp:94-118)
    double tu = now();
    cr.update(aln, threads);
    g_t_update += now() - tu;
    tu = now();
    const int hi = cr.hi();
    if (hi <= 0) continue;
    const int rnd = det_uniform(cr.engine, 0, hi - 1);
    const int col = std::min(cr.scores[rnd].first, aln[0].length() - 1);
    std::set<int> g1, g2;
    for (int i = 0; i < n; i++) (aln[i].data[col + 1] == '-' ? g1 : g2).insert(i);
    if (g1.empty() || g2.empty()) continue;
    const Profile p1 = extract_subset(aln, g1, threads), p2 = extract_subset(aln, g2, threads);
    g_t_split += now() - tu;
    Profile cand = align_alignments(w, p1, p2, be, post, threads);
    if (aln[0].length() >= cand[0].length()) aln = std::move(cand);  // checkAcceptance (length)
  }
  if (getenv("MLP_CLI_TIMES"))
    fprintf(stderr,
            "[host] profile posteriors %.3f s (%lld sequence pairs), MEA %.3f s, merges %.3f s, column scores "
            "%.3f s, splits %.3f s, %d refinement passes (MEA SIMD lanes %d)\n",
            g_t_post, (long long)g_n_terms, g_t_mea, g_t_merge, g_t_update, g_t_split, iters, cpnp::mea_simd_lanes());
  return aln;
}

}  // namespace qph
