// msa_host.cpp -- see msa_host.h.
#include "msa_host.h"

#include <stdexcept>

#include <chrono>
#include <atomic>
#include <thread>
#include "pool.h"

#include <immintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <cctype>
#include <set>

namespace cpnp {

// ------------------------------------------------------------------ FASTA
// Byte reader with the reference FileBuffer's Get / UnGet / GetLine
// (FileBuffer.h): a line ends at '\n' only, so '\r' stays in the line.
namespace {
struct Reader {
  std::string buf;
  size_t pos = 0;
  bool eof() const { return pos >= buf.size(); }
  bool get(char& ch) {
    if (pos >= buf.size()) return false;
    ch = buf[pos++];
    return true;
  }
  void unget() { --pos; }
  void line(std::string& s) {
    s.clear();
    char ch;
    while (get(ch) && ch != '\n') s += ch;
  }
};
}  // namespace

bool load_fasta(const std::string& path, std::vector<Row>& out, std::string& err) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) {
    err = "ERROR: Could not open file '" + path + "' for reading.";
    return false;
  }
  Reader in;
  char tmp[1 << 16];
  size_t got;
  while ((got = fread(tmp, 1, sizeof tmp, f)) > 0) in.buf.append(tmp, got);
  fclose(f);
  out.clear();
  // MultiSequence::LoadMFA: sequences until the first record that fails
  while (true) {
    std::string header;
    while (!in.eof()) {
      in.line(header);
      if (!header.empty()) break;
    }
    if (header.empty() || header[0] != '>') {
      if (out.empty() && !header.empty()) {
        err = "ERROR: MSF input is not supported by this build";
        return false;
      }
      break;
    }
    header = header.substr(1);
    while (!header.empty() && isspace((unsigned char)header[0])) header = header.substr(1);
    while (!header.empty() && isspace((unsigned char)header.back())) header.pop_back();
    Row r;
    r.header = header;
    r.data = "@";
    char ch;
    while (in.get(ch)) {
      if (ch == '>') {
        in.unget();
        break;
      }
      if (isspace((unsigned char)ch)) continue;
      if (ch == '.') ch = '-';
      if (ch == '-') continue;   // stripGaps
      if (!((ch >= 'A' && ch <= 'Z') || (ch >= 'a' && ch <= 'z'))) {
        err = std::string("ERROR: Unknown character encountered: ") + ch;
        return false;
      }
      if (ch >= 'a' && ch <= 'z') ch = ch - 'a' + 'A';
      r.data += ch;
    }
    if (r.length() == 0) break;   // an empty record ends the input (Sequence::Fail)
    r.label = r.sort_label = (int)out.size();
    out.push_back(std::move(r));
  }
  if (out.empty()) {
    err = "ERROR: No sequences read.";
    return false;
  }
  return true;
}

void write_mfa(std::string& out, const Profile& p, int columns) {
  // whole lines at a time (a -p 1 alignment of 512 rows is ~10 MB: per
  // character appends took 0.2 s)
  size_t total = out.size();
  for (const Row& r : p) total += r.header.size() + 2 + (size_t)r.length() + r.length() / columns + 1;
  out.reserve(total);
  for (const Row& r : p) {
    out += '>';
    out += r.header;
    out += '\n';
    const int L = r.length();
    for (int c0 = 1; c0 <= L; c0 += columns) {
      out.append(r.data, (size_t)c0, (size_t)std::min(columns, L - c0 + 1));
      out += '\n';
    }
  }
}

// ------------------------------------------------------------------ tree
GuideTree build_tree(std::vector<std::vector<float>> dist, int varianceid) {
  const int n = (int)dist.size();
  GuideTree t;
  t.nodes.assign(2 * n + 1, GuideTree::Node());
  for (int i = 0; i < n; i++) t.nodes[i].leaf = true;
  // active clusters in a list ordered by their matrix index; each cluster
  // keeps the node it currently stands for (MSAClusterTree.cpp:164-295)
  std::vector<int> active(n), node_of(n), size_of(2 * n + 1, 0);
  for (int i = 0; i < n; i++) {
    active[i] = i;
    node_of[i] = i;
    size_of[i] = 1;
  }
  std::vector<float> joins(n + 1, 0.f);
  const int first = n, last = 2 * n - 1;
  for (int node = first; node < last; node++) {
    float best = 1.1f;
    int bi = -1, bj = -1;   // positions in `active`
    for (size_t x = 0; x < active.size(); x++) {
      const int mi = active[x];
      for (size_t y = 0; y < active.size() && active[y] < mi; y++) {
        float d = dist[mi][active[y]];
        if (d < 0) {
          fprintf(stderr, "ERROR: It is impossible to have distance value less than zero\n");
          d = 0;
        }
        if (d < best) {
          best = d;
          bi = (int)x;
          bj = (int)y;
        }
      }
    }
    if (bi < 0)   // the reference prints this and exits with -1 (the CLI does, from the exception)
      throw std::runtime_error("OOPS: Error occurred while constructing the cluster tree\n");
    const int mi = active[bi], mj = active[bj];
    const float half = best * 0.5f;
    GuideTree::Node& par = t.nodes[node];
    par.left = node_of[mi];
    par.right = node_of[mj];
    t.nodes[node_of[mi]].parent = node;
    t.nodes[node_of[mi]].dist = half;
    t.nodes[node_of[mj]].parent = node;
    t.nodes[node_of[mj]].dist = half;
    size_of[node] = size_of[node_of[mi]] + size_of[node_of[mj]];
    active.erase(active.begin() + bj);
    const unsigned isize = size_of[node_of[mi]], jsize = size_of[node_of[mj]];
    for (int idx : active) {
      const float idist = dist[mi][idx], jdist = dist[mj][idx];
      if (varianceid == 0) joins[idx] = (idist + jdist) / 2;
      else joins[idx] = (idist * isize + jdist * jsize) / (isize + jsize);
    }
    node_of[mi] = node;
    for (int idx : active) {
      dist[mi][idx] = joins[idx];
      dist[idx][mi] = joins[idx];
    }
  }
  t.root = n >= 1 ? (n == 1 ? 0 : last - 1) : -1;
  // sequence weights (MSAGuideTree.cpp getSeqsWeights)
  for (int i = 0; i < n; i++)
    for (int cur = i; cur >= 0; cur = t.nodes[cur].parent) t.nodes[cur].order++;
  t.weights.assign(n, 0);
  for (int i = 0; i < n; i++) {
    float w = 0;
    for (int cur = i; t.nodes[cur].parent >= 0; cur = t.nodes[cur].parent)
      w += t.nodes[cur].dist / t.nodes[cur].order;
    t.weights[i] = (int)(100 * w);
  }
  int wsum = 0;
  for (int i = 0; i < n; i++) wsum += t.weights[i];
  if (wsum == 0) {
    for (int i = 0; i < n; i++) t.weights[i] = 1;
    wsum = n;
  }
  for (int i = 0; i < n; i++) {
    t.weights[i] = (t.weights[i] * 1000) / wsum;   // INT_MULTIPLY (MSADef.h)
    if (t.weights[i] < 1) t.weights[i] = 1;
  }
  return t;
}

// ------------------------------------------------------------------ profiles
static void mapping(const Row& r, std::vector<int>& m) {   // Sequence::GetMapping
  m.clear();
  m.reserve(r.length() + 1);
  m.push_back(0);
  for (int i = 1; i <= r.length(); i++)
    if (r.data[i] != '-') m.push_back(i);
}

std::vector<float> build_posterior(const Profile& A, const Profile& B, const SparseSet& sp,
                                   const int* weights, float cutoff) {
  std::vector<float> post;
  build_posterior_into(A, B, sp, weights, cutoff, post);
  return post;
}

void build_posterior_into(const Profile& A, const Profile& B, const SparseSet& sp, const int* weights,
                          float cutoff, std::vector<float>& post, std::vector<size_t>* dirty) {
  const int len1 = A[0].length(), len2 = B[0].length();
  const int64_t W2 = len2 + 1;
  const size_t cells = (size_t)(len1 + 1) * W2;
  // with `dirty` the buffer is all zero on entry (only the cells it lists were
  // written since) and the written cells are listed: the long profiles of the
  // -p 1 alignment graph make the dense fill cost more than the adds
  if (dirty && cutoff == 0.f) {
    if (post.size() < cells) post.resize(cells, 0.f);
  } else {
    dirty = nullptr;
    post.assign(cells, 0.f);
  }
  float total = 0;
  if (weights)
    for (const Row& x : A)
      for (const Row& y : B) total += weights[x.label] * weights[y.label];
  static thread_local std::vector<std::vector<int>> m2s;
  static thread_local std::vector<int> m1;
  if (m2s.size() < B.size()) m2s.resize(B.size());
  for (size_t yb = 0; yb < B.size(); yb++) mapping(B[yb], m2s[yb]);
  for (const Row& x : A) {
    mapping(x, m1);
    for (size_t yb = 0; yb < B.size(); yb++) {
      const Row& y = B[yb];
      const std::vector<int>& m2 = m2s[yb];
      const int first = x.label, second = y.label;
      const float w = weights ? (float)(weights[first] * weights[second]) / total : 1.f;
      const int lo = std::min(first, second), hi = std::max(first, second);
      const int64_t p = sp.pair(lo, hi);
      const int32_t* rp = sp.row_ptr.data() + sp.rp_off[p];
      const uint16_t* cols = sp.cols.data() + sp.ent_off[p];
      const float* vals = sp.vals.data() + sp.ent_off[p];
      const int rows = sp.lens[lo], ncols = sp.lens[hi];
      // the reference subtracts the cutoff from every cell of the pair
      // (ProbabilisticModel.h:1229-1283); x - 0.0f == x for every value the
      // sums take (no -0.0: they start at +0 and add non-negative terms), so
      // with the default cutoff 0 that O(L1 L2) sweep is skipped exactly,
      // and so is a pair without entries (consistency empties most of a
      // divergent family's pairs)
      const float sub = weights ? w * cutoff : cutoff;
      const bool do_sub = sub != 0.f;
      const int32_t nnz = (int32_t)(sp.ent_off[p + 1] - sp.ent_off[p]);
      if (!do_sub && nnz == 0) continue;
      // without the cutoff sweep only rows first .. last with entries matter
      int r0 = 1, r1 = rows;
      if (!do_sub) {
        r0 = (int)(std::upper_bound(rp + 1, rp + rows + 2, 0) - rp) - 1;   // first row with rp[r + 1] > 0
        r1 = (int)(std::lower_bound(rp + 1, rp + rows + 2, nnz) - rp) - 1;  // last row with rp[r] < nnz
      }
      // next row to visit: every row with the cutoff sweep, else the next
      // one holding entries (consistency leaves few, scattered rows)
      auto next_row = [&](int r) {
        return do_sub ? r + 1 : (int)(std::upper_bound(rp + r + 2, rp + rows + 2, rp[r + 1]) - rp) - 1;
      };
      if (first < second) {
        for (int ii = r0; ii <= r1; ii = next_row(ii)) {
          const int64_t base = (int64_t)m1[ii] * W2;
          for (int32_t e = rp[ii]; e < rp[ii + 1]; e++) {
            post[base + m2[cols[e]]] += weights ? w * vals[e] : vals[e];
            if (dirty) dirty->push_back(base + m2[cols[e]]);
          }
          if (do_sub)
            for (int jj = 0; jj < ncols; jj++) post[base + m2[jj]] -= sub;
        }
      } else {
        for (int jj = r0; jj <= r1; jj = next_row(jj)) {
          const int64_t base = m2[jj];
          for (int32_t e = rp[jj]; e < rp[jj + 1]; e++) {
            post[base + (int64_t)m1[cols[e]] * W2] += weights ? w * vals[e] : vals[e];
            if (dirty) dirty->push_back(base + (int64_t)m1[cols[e]] * W2);
          }
          if (do_sub)
            for (int ii = 0; ii < ncols; ii++) post[base + (int64_t)m1[ii] * W2] -= sub;
        }
      }
    }
  }
}

static ProfileBackend& profile_backend() {
  static ProfileBackend fn;
  return fn;
}
void set_profile_backend(ProfileBackend fn) { profile_backend() = std::move(fn); }

// time split of the profile stages (MLP_CLI_TIMES)
static double g_t_post = 0, g_t_mea = 0;
static int64_t g_n_post = 0, g_n_dev = 0;
static double wall() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
void profile_times(double* post, double* mea, int64_t* calls, int64_t* device_calls) {
  *post = g_t_post;
  *mea = g_t_mea;
  *calls = g_n_post;
  *device_calls = g_n_dev;
}

static MeaBackend& mea_backend() {
  static MeaBackend fn;
  return fn;
}
void set_mea_backend(MeaBackend fn) { mea_backend() = std::move(fn); }

bool device_mea(const Profile& a, const Profile& b, const int* weights, float cutoff,
                const std::vector<int64_t>* cells, std::vector<float>* vals, std::string& path, float* score) {
  if (!mea_backend() || cutoff != 0.f) return false;
  const double t0 = wall();
  const bool ok = mea_backend()(a, b, weights, cells, vals, path, score);
  if (ok) {
    g_t_mea += wall() - t0;
    g_n_post++;
    g_n_dev++;
  }
  return ok;
}

static const float* profile_posterior_impl(const Profile& a, const Profile& b, const SparseSet& sp,
                                           const int* weights, float cutoff);
const float* profile_posterior(const Profile& a, const Profile& b, const SparseSet& sp, const int* weights,
                               float cutoff) {
  const double t0 = wall();
  const float* p = profile_posterior_impl(a, b, sp, weights, cutoff);
  g_t_post += wall() - t0;
  g_n_post++;
  return p;
}

static const float* profile_posterior_impl(const Profile& a, const Profile& b, const SparseSet& sp,
                                           const int* weights, float cutoff) {
  if (profile_backend() && cutoff == 0.f)
    if (const float* p = profile_backend()(a, b, weights)) {
      g_n_dev++;
      return p;
    }
  // reused, kept all zero between calls: only the cells the previous call
  // wrote are cleared (fresh pages, or a full fill, cost more than the adds)
  static thread_local std::vector<float> buf;
  static thread_local std::vector<size_t> dirty;
  for (size_t k : dirty) buf[k] = 0.f;
  dirty.clear();
  build_posterior_into(a, b, sp, weights, cutoff, buf, &dirty);
  if (cutoff != 0.f) {   // a full fill: the whole used range is dirty
    const size_t cells = (size_t)(a[0].length() + 1) * (b[0].length() + 1);
    dirty.resize(cells);
    for (size_t k = 0; k < cells; k++) dirty[k] = k;
  }
  return buf.data();
}

std::string mea_path(int len1, int len2, const std::vector<float>& post, float* score) {
  return mea_path(len1, len2, post.data(), score);
}

std::string mea_path(int len1, int len2, const float* post, float* score) {
  const double t0 = wall();
  std::string r = mea_path_dispatch(len1, len2, post, score);
  g_t_mea += wall() - t0;
  return r;
}

// ---- MEA on host SIMD lanes: N rows per strip, lane r at column t - r at
// step t (the GPU sweeps' skewed wavefront, on one core).  Up and up-left
// come from lane r - 1's values one and two steps earlier (a lane shift, the
// row above the strip entering lane 0), left from the lane's own previous
// value; every cell runs the serial recurrence's add and its three compares
// in ChooseBestOfThree's order, so values, ties and the path are the serial
// result bit for bit.  The dependency chain per step is shared by N cells.
namespace {
// Traceback of a strip: per step one byte of lanes taking 'D' and one of
// lanes taking 'L' (else 'U').
std::string mea_trace(int len1, int len2, int N, int T, const uint8_t* tbm) {
  std::string path;
  int r = len1, c = len2;
  while (r != 0 || c != 0) {
    char ch;
    if (r == 0) {
      ch = 'L';
    } else if (c == 0) {
      ch = 'U';
    } else {
      const int sr = (r - 1) / N, lr = (r - 1) % N;
      const size_t at = ((size_t)sr * T + c + lr) * (N / 4);  // N/8 bytes of D bits, then N/8 of L bits
      const uint32_t dm = N == 8 ? tbm[at] : tbm[at] | (uint32_t)tbm[at + 1] << 8;
      const uint32_t lm = N == 8 ? tbm[at + 1] : tbm[at + 2] | (uint32_t)tbm[at + 3] << 8;
      ch = (dm >> lr) & 1 ? 'D' : (lm >> lr) & 1 ? 'L' : 'U';
    }
    switch (ch) {
      case 'L': c--; path += 'Y'; break;
      case 'U': r--; path += 'X'; break;
      default: c--; r--; path += 'B'; break;
    }
  }
  std::reverse(path.begin(), path.end());
  return path;
}

__attribute__((target("avx2"))) std::string mea_simd8(int len1, int len2, const float* post, float* score) {
  constexpr int N = 8;
  const int W2 = len2 + 1;
  const int ns = (len1 + N - 1) / N;
  const int T = len2 + N;  // steps of a strip: t = 1 .. len2 + N - 1
  std::vector<float> rowA(W2, 0.f), rowB(W2, 0.f);  // V of the row above the strip / of its last row
  float* above = rowA.data();
  float* below = rowB.data();
  std::vector<uint8_t> tbm((size_t)ns * T * (N / 4));
  const __m256i shl = _mm256_setr_epi32(0, 0, 1, 2, 3, 4, 5, 6);  // lane r <- lane r - 1
  const __m256i lane = _mm256_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7);
  const __m256 zero = _mm256_setzero_ps();
  alignas(32) float vout[N];
  for (int s = 0; s < ns; s++) {
    const int i0 = 1 + s * N;
    const int nr = std::min(N, len1 - i0 + 1);
    // post[idx[r] + t]: row i0 + r (the last row for lanes past len1), column t - r
    alignas(32) int32_t ix[N];
    for (int r = 0; r < N; r++) ix[r] = (i0 + std::min(r, nr - 1)) * W2 - r;
    const __m256i idx = _mm256_load_si256((const __m256i*)ix);
    __m256 p1 = zero, p2 = zero;  // the lanes' values one and two steps back
    uint8_t* tbs = tbm.data() + (size_t)s * T * (N / 4);
    for (int t = 1; t < T; t++) {
      const __m256 up = _mm256_blend_ps(_mm256_permutevar8x32_ps(p1, shl), _mm256_set1_ps(above[std::min(t, len2)]), 1);
      const __m256 ul =
          _mm256_blend_ps(_mm256_permutevar8x32_ps(p2, shl), _mm256_set1_ps(above[std::min(t - 1, len2)]), 1);
      __m256 pr;
      __m256 live;  // columns 1 .. len2
      if (t >= N && t <= len2) {
        pr = _mm256_i32gather_ps(post + t, idx, 4);
        live = _mm256_castsi256_ps(_mm256_set1_epi32(-1));
      } else {
        const __m256i j = _mm256_sub_epi32(_mm256_set1_epi32(t), lane);
        live = _mm256_castsi256_ps(_mm256_and_si256(_mm256_cmpgt_epi32(j, _mm256_setzero_si256()),
                                                    _mm256_cmpgt_epi32(_mm256_set1_epi32(len2 + 1), j)));
        pr = _mm256_mask_i32gather_ps(zero, post + t, idx, live, 4);
      }
      const __m256 x1 = _mm256_add_ps(pr, ul), x2 = p1, x3 = up;
      const __m256 m12 = _mm256_cmp_ps(x1, x2, _CMP_GE_OQ), m13 = _mm256_cmp_ps(x1, x3, _CMP_GE_OQ),
                   m23 = _mm256_cmp_ps(x2, x3, _CMP_GE_OQ);
      const __m256 d = _mm256_and_ps(m12, m13), l = _mm256_andnot_ps(m12, m23);
      __m256 v = _mm256_blendv_ps(_mm256_blendv_ps(x3, x2, l), x1, d);
      if (t < N) v = _mm256_and_ps(v, _mm256_castsi256_ps(_mm256_cmpgt_epi32(_mm256_set1_epi32(t), lane)));  // column <= 0: 0
      tbs[(size_t)t * 2] = (uint8_t)_mm256_movemask_ps(d);
      tbs[(size_t)t * 2 + 1] = (uint8_t)_mm256_movemask_ps(l);
      const int jl = t - (nr - 1);
      if (jl >= 1 && jl <= len2) {
        _mm256_store_ps(vout, v);
        below[jl] = vout[nr - 1];
      }
      p2 = p1;
      p1 = v;
      (void)live;
    }
    below[0] = 0.f;
    std::swap(above, below);
  }
  if (score) *score = len1 ? above[len2] : 0.f;
  return mea_trace(len1, len2, N, T, tbm.data());
}

// 16 lanes (AVX-512), strips pipelined over host threads: strip s goes to
// thread s mod T and runs in chunks of steps, each chunk started once strip
// s - 1 has finished the columns its lane 0 reads (a per-strip count of
// finished columns, spun on).  Every cell sees its neighbours' final values:
// the serial result bit for bit, for any T.
struct Mea16 {
  int len1, len2, W2, ns, TS;
  const float* post;
  float* rows;
  uint8_t* tbm;
  std::atomic<int>* done;
};

__attribute__((target("avx512f,avx512bw,avx512vl"))) void mea16_strips(const Mea16& m, int th, int nth) {
  constexpr int N = 16, CHUNK = 256;
  const int len1 = m.len1, len2 = m.len2, W2 = m.W2, TS = m.TS;
  const float* post = m.post;
  const __m512i shl = _mm512_setr_epi32(0, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14);
  const __m512i lane = _mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
  const __m512 zero = _mm512_setzero_ps();
  alignas(64) float vout[N];
  for (int s = th; s < m.ns; s += nth) {
    const int i0 = 1 + s * N;
    const int nr = std::min(N, len1 - i0 + 1);
    alignas(64) int32_t ix[N];
    for (int r = 0; r < N; r++) ix[r] = (i0 + std::min(r, nr - 1)) * W2 - r;
    const __m512i idx = _mm512_load_si512((const void*)ix);
    const float* above = m.rows + (size_t)s * W2;
    float* below = m.rows + (size_t)(s + 1) * W2;
    below[0] = 0.f;
    __m512 p1 = zero, p2 = zero;
    uint8_t* tbs = m.tbm + (size_t)s * TS * (N / 4);
    for (int c0 = 1; c0 < TS; c0 += CHUNK) {
      const int c1 = std::min(TS, c0 + CHUNK);
      // lane 0 reads the row above through column min(c1 - 1, len2)
      const int need = std::min(c1 - 1, len2) + 1;
      for (int spins = 0; m.done[s].load(std::memory_order_acquire) < need; spins++) {
        if (spins < 4000) {
          _mm_pause();
        } else {
          std::this_thread::yield();
        }
      }
      for (int t = c0; t < c1; t++) {
        const __m512 up =
            _mm512_mask_blend_ps(1, _mm512_permutexvar_ps(shl, p1), _mm512_set1_ps(above[std::min(t, len2)]));
        const __m512 ul =
            _mm512_mask_blend_ps(1, _mm512_permutexvar_ps(shl, p2), _mm512_set1_ps(above[std::min(t - 1, len2)]));
        __m512 pr;
        if (t >= N && t <= len2) {
          pr = _mm512_i32gather_ps(idx, post + t, 4);
        } else {
          const __m512i j = _mm512_sub_epi32(_mm512_set1_epi32(t), lane);
          const __mmask16 live = _mm512_cmpgt_epi32_mask(j, _mm512_setzero_si512()) &
                                 _mm512_cmpgt_epi32_mask(_mm512_set1_epi32(len2 + 1), j);
          pr = _mm512_mask_i32gather_ps(zero, live, idx, post + t, 4);
        }
        const __m512 x1 = _mm512_add_ps(pr, ul), x2 = p1, x3 = up;
        const __mmask16 m12 = _mm512_cmp_ps_mask(x1, x2, _CMP_GE_OQ), m13 = _mm512_cmp_ps_mask(x1, x3, _CMP_GE_OQ),
                        m23 = _mm512_cmp_ps_mask(x2, x3, _CMP_GE_OQ);
        const __mmask16 d = m12 & m13, l = (__mmask16)(~m12 & m23);
        __m512 v = _mm512_mask_blend_ps(d, _mm512_mask_blend_ps(l, x3, x2), x1);
        if (t < N) v = _mm512_maskz_mov_ps(_mm512_cmpgt_epi32_mask(_mm512_set1_epi32(t), lane), v);
        tbs[(size_t)t * 4] = (uint8_t)d;
        tbs[(size_t)t * 4 + 1] = (uint8_t)(d >> 8);
        tbs[(size_t)t * 4 + 2] = (uint8_t)l;
        tbs[(size_t)t * 4 + 3] = (uint8_t)(l >> 8);
        const int jl = t - (nr - 1);
        if (jl >= 1 && jl <= len2) {
          _mm512_store_ps(vout, v);
          below[jl] = vout[nr - 1];
        }
        p2 = p1;
        p1 = v;
      }
      // the last row is final through column c1 - 1 - (nr - 1)
      m.done[s + 1].store(std::min(len2, c1 - nr) + 1, std::memory_order_release);
    }
    m.done[s + 1].store(W2, std::memory_order_release);
  }
}

// 16 lanes (AVX-512), strips pipelined over host threads: strip s goes to
// thread s mod T and runs in chunks of steps, each chunk started once strip
// s - 1 has finished the columns its lane 0 reads (a per-strip count of
// finished columns, spun on).  Every cell sees its neighbours' final values:
// the serial result bit for bit, for any T.
std::string mea_simd16(int len1, int len2, const float* post, float* score, int T) {
  constexpr int N = 16;
  Mea16 m;
  m.len1 = len1;
  m.len2 = len2;
  m.W2 = len2 + 1;
  m.ns = (len1 + N - 1) / N;
  m.TS = len2 + N;  // steps of a strip: t = 1 .. len2 + N - 1
  m.post = post;
  // rows[(s + 1) W2 ..]: the last row of strip s; rows[0 ..]: row 0 (zeros)
  std::vector<float> rows((size_t)(m.ns + 1) * m.W2, 0.f);
  std::vector<uint8_t> tbm((size_t)m.ns * m.TS * (N / 4));
  std::vector<std::atomic<int>> done(m.ns + 1);  // done[s + 1]: leading columns of strip s's last row finished
  for (auto& d : done) d.store(0, std::memory_order_relaxed);
  done[0].store(m.W2, std::memory_order_relaxed);
  m.rows = rows.data();
  m.tbm = tbm.data();
  m.done = done.data();
  T = std::max(1, std::min(T, m.ns));
  if (T > 1) {
    mlpr::parallel(T, [&](int th, int nth) { mea16_strips(m, th, nth); });
  } else {
    mea16_strips(m, 0, 1);
  }
  if (score) *score = len1 ? rows[(size_t)m.ns * m.W2 + len2] : 0.f;
  return mea_trace(len1, len2, N, m.TS, tbm.data());
}
}  // namespace

int mea_simd_lanes() {
  static const int lanes = getenv("MLP_MEA_SIMD") ? atoi(getenv("MLP_MEA_SIMD"))  // 0: serial; 8, 16
                           : __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
                                   __builtin_cpu_supports("avx512vl")
                               ? 16
                           : __builtin_cpu_supports("avx2") ? 8
                                                            : 0;
  return lanes;
}

std::string mea_path_simd(int len1, int len2, const float* post, float* score, int lanes) {
  if ((int64_t)(len1 + 1) * (len2 + 1) >= (1LL << 31)) return mea_path_serial(len1, len2, post, score);  // 32-bit gathers
  if (lanes == 16 && __builtin_cpu_supports("avx512f")) {
    // strips over threads only on request (MLP_MEA_THREAD_MIN cells): on the
    // GPU box (16-core quota) QuickProbs C3's ~4e6-cell refinement MEAs ran
    // 0.95-1.4 s single-threaded against 1.0-1.8 s threaded (tools/qp_mea_ab.sh)
    static const int64_t tmin = getenv("MLP_MEA_THREAD_MIN") ? atoll(getenv("MLP_MEA_THREAD_MIN")) : INT64_MAX;
    const int T = (int64_t)len1 * len2 >= tmin ? std::min(16, mlpr::host_threads()) : 1;
    return mea_simd16(len1, len2, post, score, T);
  }
  if (lanes == 8 && __builtin_cpu_supports("avx2")) return mea_simd8(len1, len2, post, score);
  return mea_path_serial(len1, len2, post, score);
}

std::string mea_path_dispatch(int len1, int len2, const float* post, float* score) {
  // one parallel region per call, threads pipelined over 64-row bands, for
  // matrices large enough to pay for the thread wake-up (MLP_MEA_WAVE_MIN
  // cells; 0 = always serial).  Measured on the GPU box (16 cores): C2 -p 1
  // refinement MEA 0.66 -> 0.38 s (profiles of several thousand columns),
  // but ~1000 x 1000 (QuickProbs C3 refinement) 0.62 -> 0.86 s with every
  // call threaded, hence the 2.5e6-cell floor.
  static const int64_t wave_min = getenv("MLP_MEA_WAVE_MIN") ? atoll(getenv("MLP_MEA_WAVE_MIN")) : 2500000;
  // SIMD lanes first: one core at 0.5-0.6 ns a cell with 16 lanes (1.1 with
  // 8) against ~7 ns serial, faster than the threaded bands at every size
  if (const int lanes = mea_simd_lanes()) return mea_path_simd(len1, len2, post, score, lanes);
  if (wave_min > 0 && (int64_t)len1 * len2 >= wave_min && len1 >= 128 && mlpr::host_threads() > 1)
    return mea_path_wave(len1, len2, post, score);
  return mea_path_serial(len1, len2, post, score);
}

// The same recurrence with threads pipelined over bands of 64 rows: band b
// goes to thread b mod T, which walks it in 256-column tiles, each tile
// started once the band above has finished that tile's columns (an atomic
// count of finished columns per band, spun on).  Every cell still sees its
// three neighbours' final values: the serial result bit for bit.
std::string mea_path_wave(int len1, int len2, const float* post, float* score) {
  const int W2 = len2 + 1;
  constexpr int RB = 64, CB = 256;
  static thread_local std::vector<float> V;
  static thread_local std::vector<char> tb;
  if (V.size() < (size_t)(len1 + 1) * W2) {
    V.resize((size_t)(len1 + 1) * W2);
    tb.resize((size_t)(len1 + 1) * W2);
  }
  float* Vp = V.data();
  char* tbp = tb.data();
  for (int j = 0; j <= len2; j++) {
    Vp[j] = 0;
    tbp[j] = 'L';
  }
  const int nb = (len1 + RB - 1) / RB;
  std::vector<std::atomic<int>> done(nb + 1);
  for (auto& d : done) d.store(0, std::memory_order_relaxed);
  done[0].store(len2 + 1, std::memory_order_relaxed);  // row 0: complete
  const int T = std::max(1, std::min({mlpr::host_threads(), 16, nb}));
  mlpr::parallel(T, [&](int t, int nt) {
    for (int b = t; b < nb; b += nt) {
      const int i0 = 1 + b * RB, i1 = std::min(len1, i0 + RB - 1);
      for (int i = i0; i <= i1; i++) {
        Vp[(size_t)i * W2] = 0;
        tbp[(size_t)i * W2] = 'U';
      }
      for (int j0 = 1; j0 <= len2; j0 += CB) {
        const int j1 = std::min(len2, j0 + CB - 1);
        // the band above must have finished columns .. j1
        // spin briefly, then yield: the CPU may be shared (parallel test runs)
        for (int spins = 0; done[b].load(std::memory_order_acquire) < j1 + 1; spins++) {
          if (spins < 2000) {
#if defined(__x86_64__)
            __builtin_ia32_pause();
#endif
          } else {
            std::this_thread::yield();
          }
        }
        for (int i = i0; i <= i1; i++) {
          const float* pr = post + (size_t)i * W2;
          float* cur = Vp + (size_t)i * W2;
          const float* up = cur - W2;
          char* tr = tbp + (size_t)i * W2;
          for (int j = j0; j <= j1; j++) {
            const float x1 = pr[j] + up[j - 1], x2 = cur[j - 1], x3 = up[j];
            float v;
            char c;
            if (x1 >= x2) {
              if (x1 >= x3) { v = x1; c = 'D'; } else { v = x3; c = 'U'; }
            } else if (x2 >= x3) {
              v = x2; c = 'L';
            } else {
              v = x3; c = 'U';
            }
            cur[j] = v;
            tr[j] = c;
          }
        }
        done[b + 1].store(j1 + 1, std::memory_order_release);
      }
    }
  });
  if (score) *score = Vp[(size_t)len1 * W2 + len2];
  std::string path;
  int r = len1, c = len2;
  while (r != 0 || c != 0) {
    switch (tbp[(size_t)r * W2 + c]) {
      case 'L': c--; path += 'Y'; break;
      case 'U': r--; path += 'X'; break;
      default: c--; r--; path += 'B'; break;
    }
  }
  std::reverse(path.begin(), path.end());
  return path;
}

std::string mea_path_serial(int len1, int len2, const float* post, float* score) {
  const int W2 = len2 + 1;
  std::vector<float> rows(2 * (size_t)W2);
  float* oldr = rows.data();
  float* newr = rows.data() + W2;
  std::vector<char> tb((size_t)(len1 + 1) * W2);
  for (int j = 0; j <= len2; j++) {
    oldr[j] = 0;
    tb[j] = 'L';
  }
  for (int i = 1; i <= len1; i++) {
    newr[0] = 0;
    tb[(size_t)i * W2] = 'U';
    const float* pr = post + (size_t)i * W2;
    for (int j = 1; j <= len2; j++) {
      // ChooseBestOfThree (ScoreType.h:347-366): D, L, U
      const float x1 = pr[j] + oldr[j - 1], x2 = newr[j - 1], x3 = oldr[j];
      float v;
      char b;
      if (x1 >= x2) {
        if (x1 >= x3) { v = x1; b = 'D'; } else { v = x3; b = 'U'; }
      } else if (x2 >= x3) {
        v = x2; b = 'L';
      } else {
        v = x3; b = 'U';
      }
      newr[j] = v;
      tb[(size_t)i * W2 + j] = b;
    }
    std::swap(oldr, newr);
  }
  if (score) *score = oldr[len2];
  std::string path;
  int r = len1, c = len2;
  while (r != 0 || c != 0) {
    switch (tb[(size_t)r * W2 + c]) {
      case 'L': c--; path += 'Y'; break;
      case 'U': r--; path += 'X'; break;
      default: c--; r--; path += 'B'; break;
    }
  }
  std::reverse(path.begin(), path.end());
  return path;
}

static Row add_gaps(const Row& r, const std::string& path, char id) {   // Sequence::AddGaps
  Row o;
  o.header = r.header;
  o.label = r.label;
  o.sort_label = r.sort_label;
  o.data.assign(path.size() + 1, '-');
  o.data[0] = '@';
  const char* src = r.data.data() + 1;
  char* dst = &o.data[1];
  for (size_t c = 0; c < path.size(); c++)
    if (path[c] == 'B' || path[c] == id) dst[c] = *src++;
  return o;
}

// threads for a profile of n rows x L columns (data movement only; small
// profiles stay serial)
static int row_threads(size_t n, size_t L) { return n * L > 200000 ? mlpr::host_threads() : 1; }

Profile merge(const Profile& a, const Profile& b, const std::string& path, bool sort_by_label) {
  const int na = (int)a.size(), nr = (int)(a.size() + b.size());
  Profile out(nr);
  mlpr::parallel_for(nr, row_threads(nr, path.size()),
                     [&](int64_t k) { out[k] = k < na ? add_gaps(a[k], path, 'X') : add_gaps(b[k - na], path, 'Y'); });
  // MultiSequence::SortByLabel (a swap sort; the labels are distinct, so any
  // sort gives its order)
  if (sort_by_label)
    std::sort(out.begin(), out.end(), [](const Row& x, const Row& y) { return x.sort_label < y.sort_label; });
  return out;
}
Profile project(const Profile& p, const std::set<int>& idx) {
  const std::vector<int> rows(idx.begin(), idx.end());
  const int L = p[rows[0]].length();
  const int nt = row_threads(rows.size(), (size_t)L);
  std::vector<char> has(L + 1, 0);
  mlpr::parallel_for((L + 255) / 256, nt, [&](int64_t blk) {
    const int c0 = 1 + 256 * (int)blk, c1 = std::min(L, c0 + 255);
    for (int k : rows) {
      const char* d = p[k].data.data();
      for (int i = c0; i <= c1; i++) has[i] |= d[i] != '-';
    }
  });
  std::vector<int> keep;
  for (int i = 1; i <= L; i++)
    if (has[i]) keep.push_back(i);
  Profile out(rows.size());
  mlpr::parallel_for((int64_t)rows.size(), nt, [&](int64_t q) {
    const Row& src = p[rows[q]];
    Row& r = out[q];
    r.header = src.header;
    r.label = src.label;
    r.sort_label = src.sort_label;
    r.data.resize(keep.size() + 1);
    r.data[0] = '@';
    for (size_t c = 0; c < keep.size(); c++) r.data[c + 1] = src.data[keep[c]];
  });
  return out;
}

static Profile process_tree(const GuideTree& t, int node, const std::vector<Row>& seqs,
                            const SparseSet& sp, const Options& opt) {
  const GuideTree::Node& nd = t.nodes[node];
  if (nd.leaf) return Profile{seqs[node]};
  Profile left = process_tree(t, nd.left, seqs, sp, opt);
  Profile right = process_tree(t, nd.right, seqs, sp, opt);
  // AlignAlignments (MSA.cpp:1410-1474) with the tree weights
  std::string path;
  float sc;
  if (!device_mea(left, right, t.weights.data(), opt.cutoff, nullptr, nullptr, path, &sc)) {
    const float* post = profile_posterior(left, right, sp, t.weights.data(), opt.cutoff);
    path = mea_path(left[0].length(), right[0].length(), post, &sc);
  }
  return merge(left, right, path, !opt.align_order);
}

// The refinement splits come from the C library's rand(): at its default
// seed in the -p 0 path (which never seeds it, CPNP/MSA.cpp:1545), seeded with
// srand(time(0)) in the -p 1 refinement (CPNP/MSA.cpp:1896).  The GPU runtime
// libraries of this build may draw from the shared libc generator during
// initialisation, so the generator is reproduced here instead: glibc's
// TYPE_3 additive feedback generator (r[i] = r[i-3] + r[i-31]) seeded as
// srandom_r does (Park-Miller by Schrage's method, first 310 outputs
// discarded).
namespace {
struct LibcRand {
  uint32_t r[34];
  int k = 0;
  explicit LibcRand(uint32_t seed = 1) {
    int32_t s[34];
    s[0] = (int32_t)(seed ? seed : 1);
    int32_t word = s[0];
    for (int i = 1; i < 31; i++) {
      const long hi = word / 127773, lo = word % 127773;
      long w = 16807 * lo - 2836 * hi;
      if (w < 0) w += 2147483647;
      s[i] = word = (int32_t)w;
    }
    for (int i = 31; i < 34; i++) s[i] = s[i - 31];
    for (int i = 0; i < 34; i++) r[i] = (uint32_t)s[i];
    k = 34;
    for (int i = 34; i < 344; i++) next_raw();
  }
  uint32_t next_raw() {
    // ring of the last 34 values: r[k % 34]
    const uint32_t v = r[(k - 31) % 34] + r[(k - 3) % 34];
    r[k % 34] = v;
    ++k;
    return v;
  }
  int next() { return (int)(next_raw() >> 1); }
};
LibcRand& libc_rand() {
  static LibcRand g;
  return g;
}
}  // namespace

void libc_srand(uint32_t seed) { libc_rand() = LibcRand(seed); }
int libc_rand_next() { return libc_rand().next(); }

// DoIterativeRefinement (MSA.cpp:1537-1625): 2 = no split, 1 = unchanged score
static int refine_once(Profile& aln, const SparseSet& sp, const Options& opt) {
  std::set<int> one, two;
  const int n = (int)aln.size();
  for (int i = 0; i < n; i++) {
    if (libc_rand().next() % 2) one.insert(i);
    else two.insert(i);
  }
  if (one.empty() || two.empty()) return 2;
  const Profile g1 = project(aln, one), g2 = project(aln, two);
  // accuracy of the current alignment: the posterior at the columns both
  // groups occupy, summed in column order
  const int L = aln[0].length();
  const int W2 = g2[0].length() + 1;
  std::vector<int64_t> cells;
  int i1 = 0, i2 = 0;
  for (int i = 1; i <= L; i++) {
    bool f1 = false, f2 = false;
    for (int k : one)
      if (aln[k].data[i] != '-') { f1 = true; break; }
    if (f1) i1++;
    for (int k : two)
      if (aln[k].data[i] != '-') { f2 = true; break; }
    if (f2) i2++;
    if (f1 && f2) cells.push_back((int64_t)i1 * W2 + i2);
  }
  std::vector<float> vals(cells.size());
  float after;
  std::string path;
  if (!device_mea(g1, g2, nullptr, opt.cutoff, &cells, &vals, path, &after)) {
    const float* post = profile_posterior(g1, g2, sp, nullptr, opt.cutoff);
    for (size_t k = 0; k < cells.size(); k++) vals[k] = post[cells[k]];
    path = mea_path(g1[0].length(), g2[0].length(), post, &after);
  }
  float before = 0;
  for (float v : vals) before += v;
  aln = merge(g1, g2, path, false);
  return before == after ? 1 : 0;
}

Profile progressive_alignment(const std::vector<Row>& seqs, const SparseSet& sp, const GuideTree& tree,
                              int pid, Options& opt) {
  Profile aln = process_tree(tree, tree.root, seqs, sp, opt);
  const int n = (int)aln.size();
  if (opt.align_order) {   // ComputeFinalAlignment: SaveOrdering, then sorted merges stay off
    for (int i = 0; i < n; i++) aln[i].sort_label = i;
    opt.align_order = false;
  }
  int reps = opt.refinement;
  if (pid > 3 || n > 150) reps = 0;
  if (n <= 50) reps = 2 * reps;
  int ineffective = 0;
  const int warmup = 100;
  for (int i = 0; i < reps; i++) {
    const int flag = refine_once(aln, sp, opt);
    if (n > 20) {
      if (n < 200) {
        if (flag > 0) {
          if (reps < 4 * n) reps++;
          if (flag == 1) ineffective++;
        }
        if (ineffective > 2 * n && i > warmup) break;
      } else if (n > 200) {
        reps = 10;
      }
    }
  }
  return aln;
}

}  // namespace cpnp
