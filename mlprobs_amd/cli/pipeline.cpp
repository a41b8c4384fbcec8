// pipeline.cpp -- see pipeline.h.  Reference files (kuangmeng/MLProbs):
//   MLProbs.py:36-99                          main: stages, killed_stage fallbacks
//   utils/prepare_features_4_classifier_1.py  -G features, normalisation (16-42)
//   utils/classifier_c_p_np_aln.py            classifier 1, base MSA (17-51)
//   utils/calculate_column_scores.py          BLOSUM62 column scores (15-141)
//   utils/classifier_realign_strategy.py      classifier 3 (13-29)
//   utils/classifier_region_min_length.py     classifier 2 (13-29)
//   utils/unreliable_regions.py, reliable_regions.py, seperate_regions.py
//   utils/do_realign.py                       per-region realignment, combine (12-204)
#include "pipeline.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <fstream>
#include <iostream>
#include <sstream>

namespace mlpp {

namespace {

double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

bool read_file(const std::string& path, std::string& out) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  out.clear();
  char buf[1 << 16];
  size_t got;
  while ((got = fread(buf, 1, sizeof buf, f)) > 0) out.append(buf, got);
  fclose(f);
  return true;
}

bool write_file(const std::string& path, const std::string& data) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) return false;
  const bool ok = fwrite(data.data(), 1, data.size(), f) == data.size();
  return fclose(f) == 0 && ok;
}

// Python float(str) for the numeric strings the pipeline reads (a C "%f"
// field or a para.txt line): strtod after stripping whitespace, as float()
// accepts surrounding whitespace.
bool py_float(const std::string& s, double* v) {
  size_t a = 0, b = s.size();
  while (a < b && isspace((unsigned char)s[a])) a++;
  while (b > a && isspace((unsigned char)s[b - 1])) b--;
  if (a == b) return false;
  const std::string t = s.substr(a, b - a);
  char* end;
  *v = strtod(t.c_str(), &end);
  return *end == 0;
}

std::string py_strip(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && isspace((unsigned char)s[a])) a++;
  while (b > a && isspace((unsigned char)s[b - 1])) b--;
  return s.substr(a, b - a);
}

// "ARNDCQEGHILKMFPSTWYV" and BLOSUM62 as calculate_column_scores.py:11-35
// holds them (its getIdx / matrix)
const char kAlpha[] = "ARNDCQEGHILKMFPSTWYV";
const int kBlosum62[20][20] = {
    {4, -1, -2, -2, 0, -1, -1, 0, -2, -1, -1, -1, -1, -2, -1, 1, 0, -3, -2, 0},
    {-1, 5, 0, -2, -3, 1, 0, -2, 0, -3, -2, 2, -1, -3, -2, -1, -1, -3, -2, -3},
    {-2, 0, 6, 1, -3, 0, 0, 0, 1, -3, -3, 0, -2, -3, -2, 1, 0, -4, -2, -3},
    {-2, -2, 1, 6, -3, 0, 2, -1, -1, -3, -4, -1, -3, -3, -1, 0, -1, -4, -3, -3},
    {0, -3, -3, -3, 9, -3, -4, -3, -3, -1, -1, -3, -1, -2, -3, -1, -1, -2, -2, -1},
    {-1, 1, 0, 0, -3, 5, 2, -2, 0, -3, -2, 1, 0, -3, -1, 0, -1, -2, -1, -2},
    {-1, 0, 0, 2, -4, 2, 5, -2, 0, -3, -3, 1, -2, -3, -1, 0, -1, -3, -2, -2},
    {0, -2, 0, -1, -3, -2, -2, 6, -2, -4, -4, -2, -3, -3, -2, 0, -2, -2, -3, -3},
    {-2, 0, 1, -1, -3, 0, 0, -2, 8, -3, -3, -1, -2, -1, -2, -1, -2, -2, 2, -3},
    {-1, -3, -3, -3, -1, -3, -3, -4, -3, 4, 2, -3, 1, 0, -3, -2, -1, -3, -1, 3},
    {-1, -2, -3, -4, -1, -2, -3, -4, -3, 2, 4, -2, 2, 0, -3, -2, -1, -2, -1, 1},
    {-1, 2, 0, -1, -3, 1, 1, -2, -1, -3, -2, 5, -1, -3, -1, 0, -1, -3, -2, -2},
    {-1, -1, -2, -3, -1, 0, -2, -3, -2, 1, 2, -1, 5, 0, -2, -1, -1, -1, -1, 1},
    {-2, -3, -3, -3, -2, -3, -3, -3, -1, 0, 0, -3, 0, 6, -4, -2, -2, 1, 3, -1},
    {-1, -2, -2, -1, -3, -1, -1, -2, -2, -3, -3, -1, -2, -4, 7, -1, -1, -4, -3, -2},
    {1, -1, 1, 0, -1, 0, 0, 0, -1, -2, -2, 0, -1, -2, -1, 4, 1, -3, -2, -2},
    {0, -1, 0, -1, -1, -1, -1, -2, -2, -1, -1, -1, -1, -2, -1, 1, 5, -2, -2, 0},
    {-3, -3, -4, -4, -2, -2, -3, -2, -2, -3, -2, -3, -1, 1, -4, -3, -2, 11, 2, -3},
    {-2, -2, -2, -3, -2, -1, -2, -3, 2, -1, -1, -2, -1, 3, -3, -2, -2, 2, 7, -1},
    {0, -3, -3, -3, -1, -2, -2, -3, -3, 3, 1, -2, 1, -1, -2, -2, 0, -3, -1, 4}};

int blosum_index(unsigned char c) {
  static int idx[256];
  static bool init = [] {
    for (int& v : idx) v = -1;
    for (int k = 0; k < 20; k++) idx[(unsigned char)kAlpha[k]] = k;
    return true;
  }();
  (void)init;
  return idx[c];
}

}  // namespace

// ------------------------------------------------------------------ forests
bool Forest::load(const std::string& path, std::string& err) {
  std::string buf;
  if (!read_file(path, buf)) {
    err = "cannot read " + path;
    return false;
  }
  size_t pos = 0;
  auto take = [&](void* dst, size_t bytes) {
    if (pos + bytes > buf.size()) return false;
    memcpy(dst, buf.data() + pos, bytes);
    pos += bytes;
    return true;
  };
  char magic[4];
  uint32_t hdr[4];
  if (!take(magic, 4) || memcmp(magic, "MLPF", 4) || !take(hdr, sizeof hdr) || hdr[0] != 1) {
    err = path + ": not a forest file (tools/export_forests.py)";
    return false;
  }
  const uint32_t nt = hdr[1];
  n_features = (int)hdr[2];
  n_classes = (int)hdr[3];
  classes.resize(n_classes);
  bool ok = take(classes.data(), sizeof(double) * n_classes);
  trees.resize(nt);
  for (uint32_t t = 0; t < nt && ok; t++) {
    uint32_t nc = 0;
    ok = take(&nc, 4);
    Tree& T = trees[t];
    T.left.resize(nc);
    T.right.resize(nc);
    T.feature.resize(nc);
    T.threshold.resize(nc);
    T.value.resize((size_t)nc * n_classes);
    ok = ok && take(T.left.data(), 4ull * nc) && take(T.right.data(), 4ull * nc) && take(T.feature.data(), 4ull * nc) &&
         take(T.threshold.data(), 8ull * nc) && take(T.value.data(), 8ull * nc * n_classes);
    for (uint32_t k = 0; ok && k < nc; k++)
      if (T.left[k] >= 0 && (T.left[k] >= (int)nc || T.right[k] < 0 || T.right[k] >= (int)nc || T.feature[k] < 0 ||
                             T.feature[k] >= n_features))
        ok = false;
  }
  if (!ok || pos != buf.size()) {
    err = path + ": truncated or malformed forest";
    return false;
  }
  return true;
}

std::vector<double> Forest::predict_proba(const std::vector<double>& x) const {
  std::vector<float> xf(n_features);   // check_array(X, dtype=np.float32)
  for (int k = 0; k < n_features; k++) xf[k] = (float)x[k];
  std::vector<double> all(n_classes, 0.0), p(n_classes);
  for (const Tree& T : trees) {
    int node = 0;
    while (T.left[node] != -1) node = (double)xf[T.feature[node]] <= T.threshold[node] ? T.left[node] : T.right[node];
    double norm = 0.0;
    for (int c = 0; c < n_classes; c++) norm += (p[c] = T.value[(size_t)node * n_classes + c]);
    if (norm == 0.0) norm = 1.0;
    for (int c = 0; c < n_classes; c++) all[c] += p[c] / norm;
  }
  for (double& v : all) v /= (double)trees.size();
  return all;
}

double Forest::predict(const std::vector<double>& x) const {
  const std::vector<double> pr = predict_proba(x);
  int best = 0;
  for (int c = 1; c < n_classes; c++)
    if (pr[c] > pr[best]) best = c;   // np.argmax: the first maximum
  return classes[best];
}

bool read_para(const std::string& path, std::vector<double>& para, std::string& err) {
  std::string text;
  if (!read_file(path, text)) {
    err = "cannot read " + path;
    return false;
  }
  para.clear();
  for (const std::string& line : splitlines(text)) {
    double v;
    if (!py_float(line, &v)) {
      err = path + ": bad line '" + line + "'";
      return false;
    }
    para.push_back(v);
  }
  return true;
}

bool Models::load(const std::string& dir, std::string& err) {
  return branch.load(dir + "/branch.forest", err) && regions.load(dir + "/regions.forest", err) &&
         seq_lens.load(dir + "/seq_lens.forest", err) && read_para(dir + "/branch.para", branch_para, err) &&
         read_para(dir + "/regions.para", regions_para, err) && read_para(dir + "/seq_lens.para", seq_lens_para, err);
}

// (float(t) - para[2i + 1]) / (para[2i] - para[2i + 1]) for each feature
// (prepare_features_4_classifier_1.py:39-40 and the classifiers' own copies)
static bool normalise(const std::vector<double>& raw, const std::vector<double>& para, std::vector<double>& out) {
  if (para.size() < 2 * raw.size()) return false;
  out.resize(raw.size());
  for (size_t i = 0; i < raw.size(); i++) out[i] = (raw[i] - para[i * 2 + 1]) / (para[i * 2] - para[i * 2 + 1]);
  return true;
}

// ------------------------------------------------------------------ text
std::vector<std::string> split_newline(const std::string& text) {
  std::vector<std::string> out;
  size_t a = 0;
  while (true) {
    const size_t e = text.find('\n', a);
    if (e == std::string::npos) {
      out.push_back(text.substr(a));
      return out;
    }
    out.push_back(text.substr(a, e - a));
    a = e + 1;
  }
}

std::vector<std::string> splitlines(const std::string& text) {
  // str.splitlines(): \n, \r, \r\n and the other ASCII line boundaries
  // \v \f \x1c \x1d \x1e; no trailing empty line
  std::vector<std::string> out;
  size_t a = 0, i = 0;
  const size_t n = text.size();
  while (i < n) {
    const char c = text[i];
    if (c == '\n' || c == '\r' || c == '\v' || c == '\f' || c == '\x1c' || c == '\x1d' || c == '\x1e') {
      out.push_back(text.substr(a, i - a));
      i += (c == '\r' && i + 1 < n && text[i + 1] == '\n') ? 2 : 1;
      a = i;
    } else {
      i++;
    }
  }
  if (a < n) out.push_back(text.substr(a));
  return out;
}

static std::string drop_cr(const std::string& s) {
  std::string r;
  r.reserve(s.size());
  for (char c : s)
    if (c != '\r') r += c;
  return r;
}

Dic parse_dic(const std::vector<std::string>& lines) {
  Dic d;
  bool has_key = false;
  std::string key, value;
  for (const std::string& line : lines) {
    if (!line.empty() && line[0] == '>') {
      if (has_key) {
        d.rows[key] = value;
        value.clear();
        key.clear();
      }
      has_key = true;
      key = line;
    } else if (has_key) {
      value = drop_cr(value) + drop_cr(line);
    }
  }
  d.rows[key] = value;
  d.last_len = value.size();
  return d;
}

// ------------------------------------------------------------------ column scores
ColScores column_scores(const Dic& d) {
  ColScores cs;
  const int64_t N = (int64_t)d.rows.size();
  cs.nkeys = N;
  cs.lens = (int64_t)d.last_len;
  const double lens_ = (double)(N * (N - 1)) / 2;   // (len * (len - 1)) / 2, a float
  std::vector<const std::string*> rows;
  for (const auto& kv : d.rows) rows.push_back(&kv.second);
  // The reference sums matrix[a][b] over the pairs k1 < k2 of sorted keys in
  // doubles; every partial sum is an integer well below 2^53, so the sum is
  // exact in any order: per column, letter counts give the same integer.
  cs.col.resize(cs.lens);
  int64_t cnt[20];
  for (int64_t i = 0; i < cs.lens; i++) {
    std::fill(cnt, cnt + 20, 0);
    for (const std::string* r : rows) {
      if ((int64_t)r->size() <= i) {
        cs.error = true;
        cs.error_msg = "IndexError: string index out of range (calculate_column_scores.py:66)";
        return cs;
      }
      const int k = blosum_index((unsigned char)(*r)[i]);
      if (k >= 0) cnt[k]++;
    }
    int64_t s = 0;
    for (int a = 0; a < 20; a++) {
      if (!cnt[a]) continue;
      s += cnt[a] * (cnt[a] - 1) / 2 * kBlosum62[a][a];
      for (int b = a + 1; b < 20; b++) s += cnt[a] * cnt[b] * kBlosum62[a][b];
    }
    if (lens_ == 0) {
      cs.error = true;
      cs.error_msg = "ZeroDivisionError: float division by zero (calculate_column_scores.py:70)";
      return cs;
    }
    cs.col[i] = (double)s / lens_;
  }
  double un = 0.0;
  for (double v : cs.col) un += v;
  if (cs.lens != 0) {
    un /= (double)cs.lens;
    double sd = 0.0;   // getSD (calculate_column_scores.py:123-128)
    for (double v : cs.col) sd += (v - un) * (v - un);
    sd /= (double)cs.lens;
    cs.sd = sqrt(sd);
    double ratio = 0.0;   // getPeakLengthRatio (:130-135)
    for (double v : cs.col)
      if (v >= 1.0) ratio += 1;
    cs.peak = ratio / (double)cs.lens;
  } else {
    un = 0;
  }
  cs.un_sp = un;
  return cs;
}

double avg_col_score(const std::string& file_text, bool* error) {
  const Dic d = parse_dic(splitlines(file_text));
  const int64_t N = (int64_t)d.rows.size();
  const double lens_ = (double)(N * (N - 1)) / 2;
  if (lens_ * (double)d.last_len == 0) return -1;
  const ColScores cs = column_scores(d);
  if (cs.error) {
    if (error) *error = true;
    return -1;
  }
  double s = 0;
  for (double v : cs.col) s += v;
  return s / (double)cs.lens;
}

// ------------------------------------------------------------------ regions
std::vector<std::pair<int64_t, int64_t>> unreliable_regions(const std::vector<double>& col, double sigma, double beta,
                                                            int class_lens) {
  int64_t div = 30;   // lens_seq_4_devide
  if (class_lens == 2) div = 20;
  if (class_lens == 1) div = 10;
  else if (class_lens == 0) div = 1;
  const int64_t last_col = (int64_t)col.size() - 1;
  std::vector<std::pair<int64_t, int64_t>> out;
  int t1 = 0, t2 = 0;
  int64_t head = 0;
  for (int64_t item = 0; item < (int64_t)col.size(); item++) {
    const double v = col[item];
    const bool in = v <= sigma && v >= beta;
    if (in && t1 == 0) {
      head = item + 1;
      t1 = 1;
    } else if (in && t1 == 1 && t2 == 0) {
      t2 = 1;
    } else if (in && t1 == 1 && t2 == 1) {
      if (item == last_col && item - head > div) out.push_back({head, item});
    } else if ((v > sigma || v < beta) && t1 == 1 && t2 == 1) {
      if (item - head > div) out.push_back({head, item});
      t1 = t2 = 0;
      head = 0;
    } else {
      t1 = t2 = 0;
      head = 0;
    }
  }
  return out;
}

std::vector<std::pair<int64_t, int64_t>> reliable_regions(const std::vector<double>& col, double threshold,
                                                          int class_lens_max, int class_lens_min) {
  const bool set_max = class_lens_max > 0;
  const int64_t last_col = (int64_t)col.size() - 1;
  std::vector<std::pair<int64_t, int64_t>> out;
  int64_t head = 0;
  int t1 = 0, t2 = 0;
  // the reference's `while class_lens_max < item - head` shrink loop, with
  // its int(col_score[tmp_head]) truncation (reliable_regions.py:28-33)
  auto shrink = [&](int64_t& item) {
    if (!set_max) return;
    while (class_lens_max < item - head) {
      if (col[item] > (double)(int64_t)col[head] && head > 1) head += 1;
      else item -= 1;
    }
  };
  for (int64_t item0 = 0; item0 < (int64_t)col.size(); item0++) {
    int64_t item = item0;
    const double v = col[item];
    if (v > threshold && t1 == 0) {
      head = item + 1;
      t1 = 1;
    } else if (v > threshold && t1 == 1 && t2 == 0) {
      t2 = 1;
    } else if (v > threshold && t1 == 1 && t2 == 1) {
      if (item == last_col && item - head > class_lens_min && item - head >= 3) {
        shrink(item);
        out.push_back({head, item});
      }
    } else if (v <= threshold && t1 == 1 && t2 == 1) {
      if (item - head > class_lens_min && item - head >= 3) {
        shrink(item);
        out.push_back({head, item});
      }
      t1 = t2 = 0;
      head = 0;
    } else {
      t1 = t2 = 0;
      head = 0;
    }
  }
  return out;
}

// Python's s[a:b] for 0 <= a (the only slices these files take)
static std::string py_slice(const std::string& s, int64_t a, int64_t b) {
  const int64_t n = (int64_t)s.size();
  if (b < 0) b = std::max<int64_t>(0, n + b);
  a = std::min(a, n);
  b = std::min(b, n);
  return b > a ? s.substr(a, b - a) : std::string();
}

void separate_regions(const std::vector<std::pair<int64_t, int64_t>>& R, const std::string& real_output, Dir& dir) {
  const std::vector<std::string> lines = split_newline(real_output);
  const Dic d = parse_dic(lines);
  const int64_t lens = (int64_t)d.last_len;
  auto block = [&](int64_t a, int64_t b) {
    std::string s;
    for (const auto& kv : d.rows) s += kv.first + "\n" + py_slice(kv.second, a, b) + "\n";
    return s;
  };
  if (R.empty()) {
    std::string s;
    for (const std::string& l : lines) s += l + "\n";
    dir["0-" + std::to_string(lens - 1) + ".reliable"] = s;
    return;
  }
  if (R[0].first > 1) dir["0-" + std::to_string(R[0].first - 2) + ".reliable"] = block(0, R[0].first - 1);
  for (const auto& it : R)
    dir[std::to_string(it.first - 1) + "-" + std::to_string(it.second - 1) + ".unreliable"] =
        block(it.first - 1, it.second);
  if (R.size() == 1 && lens > R[0].second) {
    dir[std::to_string(R[0].second) + "-" + std::to_string(lens - 1) + ".reliable"] = block(R[0].second, lens);
  } else if (R.size() > 1) {
    for (size_t i = 0; i + 1 < R.size(); i++)
      dir[std::to_string(R[i].second) + "-" + std::to_string(R[i + 1].first - 2) + ".reliable"] =
          block(R[i].second, R[i + 1].first - 1);
    if (R.back().second < lens)
      dir[std::to_string(R.back().second) + "-" + std::to_string(lens - 1) + ".reliable"] = block(R.back().second, lens);
  }
}

// ------------------------------------------------------------------ tools
namespace {

// getstatusoutput's text: one trailing newline removed
std::string strip_one_newline(std::string s) {
  if (!s.empty() && s.back() == '\n') s.pop_back();
  return s;
}

struct InProcess : Tools {
  mlpr::Session* s;
  explicit InProcess(mlpr::Session* s_) : s(s_) {}
  const char* name() const override { return "in-process"; }
  int cpnp(const std::string& seq_file, bool features, int program, std::string& text) override {
    std::vector<cpnp::Row> seqs;
    std::string out, err;
    int status = 0;
    if (!cpnp::load_fasta(seq_file, seqs, err)) {
      status = 1;
    } else {
      for (size_t k = 0; k < seqs.size(); k++) seqs[k].label = seqs[k].sort_label = (int)k;
      status = mlpr::run_cpnp(std::move(seqs), features, program == 0, cpnp::Options(), s, out, err);
    }
    text = strip_one_newline(status ? out + err + "\n" : out);
    return status;
  }
  std::string quickprobs_on(std::vector<qph::Seq>& seqs, bool loaded, const std::string& msg) {
    if (!loaded) return msg;   // the reference prints the illegal characters on stdout
    for (const qph::Seq& q : seqs)
      if (q.data.find('-') != std::string::npos) return std::string();
    std::string out, err;
    const int status = mlpr::run_qp(std::move(seqs), qph::Options(), 0, s, out, err);
    return status ? std::string() : out;
  }
  std::string quickprobs_text(const std::string& fasta) override {
    std::vector<qph::Seq> seqs;
    std::string msg, err;
    const bool ok = qph::load_fasta_text(fasta, seqs, msg, err);
    return quickprobs_on(seqs, ok, msg);
  }
  std::string quickprobs_file(const std::string& seq_file) override {
    std::vector<qph::Seq> seqs;
    std::string msg, err;
    const bool ok = qph::load_fasta(seq_file, seqs, msg, err);
    return quickprobs_on(seqs, ok, msg);
  }
};

// One shell word: the path in single quotes, embedded quotes as '\''.  The
// tool commands themselves (--cpnp / --quickprobs) stay shell text, as
// MLProbs.py's os.system strings are; only the file paths are quoted.
std::string shell_quote(const std::string& a) {
  std::string r = "'";
  for (char ch : a) {
    if (ch == '\'') r += "'\\''";
    else r += ch;
  }
  return r + "'";
}

struct External : Tools {
  std::string cp, qp, tmp;
  int count = 0;
  External(const std::string& c, const std::string& q, const std::string& t) : cp(c), qp(q), tmp(t) {}
  const char* name() const override { return "external"; }
  int cpnp(const std::string& seq_file, bool features, int program, std::string& text) override {
    const std::string cmd =
        cp + (features ? " -G " : " -p " + std::to_string(program) + " ") + shell_quote(seq_file) + " 2>&1";
    FILE* p = popen(cmd.c_str(), "r");
    text.clear();
    if (!p) return 127;
    char buf[1 << 16];
    size_t got;
    while ((got = fread(buf, 1, sizeof buf, p)) > 0) text.append(buf, got);
    const int st = pclose(p);
    text = strip_one_newline(text);
    return WIFEXITED(st) ? WEXITSTATUS(st) : 1;
  }
  std::string run_qp(const std::string& in) {
    const std::string out = tmp + "/mlprobs_" + std::to_string(getpid()) + "_qp_out_" + std::to_string(count++);
    const std::string cmd = qp + " " + shell_quote(in) + " > " + shell_quote(out);
    if (system(cmd.c_str()) == -1) return std::string();
    std::string res;
    read_file(out, res);
    remove(out.c_str());
    return res;
  }
  std::string quickprobs_text(const std::string& fasta) override {
    const std::string in =
        tmp + "/mlprobs_" + std::to_string(getpid()) + "_qp_in_" + std::to_string(count++) + ".unreliable";
    write_file(in, fasta);
    std::string r = run_qp(in);
    remove(in.c_str());
    return r;
  }
  std::string quickprobs_file(const std::string& seq_file) override { return run_qp(seq_file); }
};

}  // namespace

std::unique_ptr<Tools> in_process_tools(mlpr::Session* s) { return std::unique_ptr<Tools>(new InProcess(s)); }
std::unique_ptr<Tools> external_tools(const std::string& c, const std::string& q, const std::string& t) {
  return std::unique_ptr<Tools>(new External(c, q, t));
}

// ------------------------------------------------------------------ realign + combine
namespace {

std::string base_name(const std::string& f) {   // os.path.splitext(name)[0]
  const size_t d = f.rfind('.');
  return d == std::string::npos || d == 0 ? f : f.substr(0, d);
}
std::string ext_of(const std::string& f) {   // os.path.splitext(name)[-1][1:]
  const size_t d = f.rfind('.');
  return d == std::string::npos || d == 0 ? std::string() : f.substr(d + 1);
}

int header_count(const std::string& text) {   // getFileLen (do_realign.py:112-119)
  int n = 0;
  for (const std::string& l : splitlines(text)) {
    const std::string s = py_strip(l);
    if (!s.empty() && s[0] == '>') n++;
  }
  return n;
}

bool has_upper(const std::string& s) {
  for (char c : s)
    if (c >= 'A' && c <= 'Z') return true;
  return false;
}

// doRealign (do_realign.py:49-71) + perProcess (:20-47) + addPerProcess (:73-101).
// false (err set) where the reference raises: getAvgColScore indexes every
// row at every column of the last row (calculate_column_scores.py:106-112),
// so a ragged MSA raises IndexError and MLProbs.py ends without output.
bool realign_region(Tools& tools, Dir& dir, const std::string& name, Trace& tr, std::string& err) {
  const std::string ret = base_name(name) + ".reliable";
  const std::string region = dir[name];
  // perProcess: rows with a letter, gaps removed; all-gap rows set aside
  const Dic d = parse_dic(splitlines(region));
  std::string tmp_file;
  std::vector<std::string> tmp_array;
  for (const auto& kv : d.rows) {
    if (has_upper(kv.second)) {
      std::string r;
      for (char c : kv.second)
        if (c != '-' && c != '.') r += c;
      tmp_file += kv.first + "\n" + r + "\n";
    } else {
      tmp_array.push_back(kv.first);
    }
  }
  std::string out = tools.quickprobs_text(tmp_file);
  tr.quickprobs_calls++;
  bool kept = false;
  bool ragged = false;
  // os.path.getsize / getAvgColScore, left operand first like Python
  if (out.empty() || avg_col_score(region, &ragged) > (ragged ? 0.0 : avg_col_score(out, &ragged)) || ragged) {
    if (ragged) {
      err = "IndexError: string index out of range (calculate_column_scores.py:110, getAvgColScore on " + name + ")";
      return false;
    }
    out = region;
    kept = true;
  }
  tr.realigned.push_back(name);
  tr.kept_original.push_back(kept);
  // addPerProcess: sorted rows, then the all-gap rows as '-' * len
  const Dic r = parse_dic(splitlines(out));
  const size_t lens = r.rows.empty() ? 0 : r.rows.begin()->second.size();
  std::string s;
  for (const auto& kv : r.rows) s += kv.first + "\n" + kv.second + "\n";
  for (const std::string& h : tmp_array) s += h + "\n" + std::string(lens, '-') + "\n";
  dir[ret] = s;
  return true;
}

// combineFiles (do_realign.py:121-199); false where the reference raises
bool combine(const std::string& input_text, Dir& dir, std::string& output, bool& written, std::string& err) {
  const int seq_file_lens = header_count(input_text);
  std::vector<std::string> need;
  for (const auto& kv : dir)
    if (ext_of(kv.first) == "reliable" && kv.first[0] != '.') need.push_back(kv.first);
  written = false;
  if (need.size() == 1) {   // mv
    output = dir[need[0]];
    written = true;
    return true;
  }
  if (need.empty()) {   // need_combination_files[0]: IndexError
    err = "IndexError: list index out of range (do_realign.py:147)";
    return false;
  }
  std::vector<int64_t> nums;
  for (const std::string& f : need) nums.push_back(atoll(f.substr(0, f.find('-')).c_str()));
  std::sort(nums.begin(), nums.end());
  std::vector<std::string> files;
  for (int64_t num : nums)
    for (const std::string& f : need)
      if (std::to_string(num) == f.substr(0, f.find('-'))) files.push_back(f);
  if (files.size() != need.size()) {   // prints "ERROR: file length" and returns: no output file
    printf("ERROR: file length\n");
    return true;
  }
  // a block without the family's sequences falls back to its .unreliable original
  auto pick = [&](const std::string& f, std::string& text) -> bool {
    const std::string& t = dir[f];
    if (t.empty() || header_count(t) != seq_file_lens) {
      const std::string alt = base_name(f) + ".unreliable";
      printf("[ERROR] Fixed: No sequences read Error !\n");
      auto it = dir.find(alt);
      if (it == dir.end()) {
        err = "FileNotFoundError: " + alt + " (do_realign.py:153)";
        return false;
      }
      text = it->second;
      return true;
    }
    text = t;
    return true;
  };
  std::string text;
  if (!pick(files[0], text)) return false;
  std::map<std::string, std::string> dic;
  {
    bool has_key = false;
    std::string key, value;
    for (const std::string& line : splitlines(text)) {
      if (!line.empty() && line[0] == '>') {
        if (has_key) {
          dic[key] = value;
          value.clear();
          key.clear();
        }
        has_key = true;
        key = line;
      } else if (has_key) {
        value = drop_cr(value) + drop_cr(line);
      }
    }
    dic[key] = value;
  }
  for (size_t fi = 1; fi < files.size(); fi++) {
    if (!pick(files[fi], text)) return false;
    bool has_key = false;
    std::string key, value;
    for (const std::string& line : splitlines(text)) {
      if (!line.empty() && line[0] == '>') {
        if (has_key) {
          auto it = dic.find(key);
          if (it == dic.end()) {
            err = "KeyError: " + key + " (do_realign.py:185)";
            return false;
          }
          it->second += value;
          value.clear();
          key.clear();
        }
        has_key = true;
        key = line;
      } else if (has_key) {
        value = drop_cr(value) + drop_cr(line);
      }
    }
    auto it = dic.find(key);
    if (it == dic.end()) {
      err = "KeyError: " + key + " (do_realign.py:193)";
      return false;
    }
    it->second += value;
  }
  output.clear();
  for (const auto& kv : dic) output += kv.first + "\n" + kv.second + "\n";
  written = true;
  return true;
}

}  // namespace

// ------------------------------------------------------------------ driver
bool run_pipeline(const std::string& seq_file, Tools& tools, const Models& M, std::string& result, Trace& tr,
                  std::string& err, bool verbose) {
  const double sigma = 1.2, beta = 0.0, threshold = 2.0;   // MLProbs.py:24-26
  auto say = [&](const char* fmt, double v) {
    if (verbose) {
      printf(fmt, v);
      fflush(stdout);
    }
  };
  const double t_start = now();
  double t = t_start;
  auto lap = [&](const char* stage) {
    const double t1 = now();
    tr.times[stage] += t1 - t;
    t = t1;
    return tr.times[stage];
  };
  std::string input_text;
  if (!read_file(seq_file, input_text)) {
    err = "FileNotFoundError: " + seq_file;
    return false;
  }
  bool have_output = false;
  // ---- getFeatures4Classifier1 (prepare_features_4_classifier_1.py:23-42)
  tools.cpnp(seq_file, true, 0, tr.features_line);
  std::vector<std::string> fc;
  {
    size_t a = 0;
    while (true) {
      const size_t e = tr.features_line.find('\t', a);
      fc.push_back(tr.features_line.substr(a, e == std::string::npos ? std::string::npos : e - a));
      if (e == std::string::npos) break;
      a = e + 1;
    }
  }
  std::vector<double> raw1(5, 0.0);
  double avg_pid = 0, sd_pid = 0, factor = 0;
  if (fc.size() >= 7) {
    const int fields[5] = {0, 2, 3, 4, 5};   // identity, N, avg_len, avg_sp, peak ratio
    for (int k = 0; k < 5; k++)
      if (!py_float(fc[fields[k]], &raw1[k])) {
        err = "ValueError: could not convert string to float: '" + fc[fields[k]] + "'";
        return false;
      }
    avg_pid = raw1[0];
    if (!py_float(fc[1], &sd_pid) || !py_float(fc[6], &factor)) {
      err = "ValueError: could not convert string to float";
      return false;
    }
  }
  if (!normalise(raw1, M.branch_para, tr.features1)) {
    err = "IndexError: branch para.txt too short";
    return false;
  }
  say("[ELAPSED TIME] Preparing data for \"Classifier 1\" takes %.3f sec.\n", lap("features"));
  // ---- AlteredPnp (classifier_c_p_np_aln.py:17-51)
  {
    const double c = M.branch.predict(tr.features1);
    tr.class1 = (int)c >= 2 || (int)c < 0 ? 0 : (int)c;
  }
  lap("classifier 1");
  std::string real_output;
  if (tools.cpnp(seq_file, false, tr.class1, real_output) != 0) tr.killed_stage = 2;
  say("[ELAPSED TIME] Get base MSA spends %.3f sec.\n", lap("base MSA"));
  // ---- calculateColScore
  tr.cs = column_scores(parse_dic(split_newline(real_output)));
  if (tr.cs.error) {
    err = tr.cs.error_msg;
    return false;
  }
  lap("column scores");
  // ---- classifier 3 (classifier_realign_strategy.py:13-29)
  std::vector<double> f3;
  if (!normalise({tr.cs.peak, avg_pid, tr.cs.sd, tr.cs.un_sp}, M.regions_para, f3)) {
    err = "IndexError: regions para.txt too short";
    return false;
  }
  double cr = M.regions.predict(f3);
  if (cr > 1 || cr < 0) cr = 1;
  tr.class_region = (int)cr;
  lap("classifier 3");
  Dir dir;
  if (tr.class_region == 1) {
    // classifier 2 (classifier_region_min_length.py:13-29)
    std::vector<double> f2;
    if (!normalise({(double)tr.cs.lens, (double)tr.cs.nkeys, avg_pid, sd_pid, tr.cs.un_sp}, M.seq_lens_para, f2)) {
      err = "IndexError: seq_lens para.txt too short";
      return false;
    }
    double cl = M.seq_lens.predict(f2);
    if (cl > 3 || cl < 0) cl = 3;
    tr.class_lens = (int)cl;
    lap("classifier 2");
    // seperateCategory1Regions (seperate_regions.py:11-24)
    if (tr.killed_stage != 2) {
      tr.regions = unreliable_regions(tr.cs.col, sigma, beta, tr.class_lens);
      separate_regions(tr.regions, real_output, dir);
    } else {
      tr.killed_stage = 4;
      result = tools.quickprobs_file(seq_file);
      tr.quickprobs_calls++;
      have_output = true;
    }
    tr.path = "RIR";
  } else {
    // seperateCategory2Regions (seperate_regions.py:26-39)
    if (tr.killed_stage != 2) {
      tr.regions = reliable_regions(tr.cs.col, threshold, 0, 0);
      separate_regions(tr.regions, real_output, dir);
    } else {
      tr.killed_stage = 4;
      result = tools.quickprobs_file(seq_file);
      tr.quickprobs_calls++;
      have_output = true;
    }
    tr.path = "RCR";
  }
  say("[ELAPSED TIME] Region separation takes %.3f sec.\n", lap("regions"));
  if (tr.killed_stage != 4) {
    // doRealignDir (do_realign.py:103-110)
    if ((factor > 0 && tr.class_region == 0) || tr.class_region == 1) {
      std::vector<std::string> names;
      for (const auto& kv : dir)
        if (ext_of(kv.first) == "unreliable" && kv.first[0] != '.') names.push_back(kv.first);
      for (const std::string& f : names)
        if (!realign_region(tools, dir, f, tr, err)) return false;
    } else {   // ExceptionHandling (:201-204): quickprobs on the whole family
      dir.clear();
      dir["0-0.reliable"] = tools.quickprobs_file(seq_file);
      tr.quickprobs_calls++;
      tr.path += " whole-family";
    }
    say("[ELAPSED TIME] Realigments spend %.3f sec.\n", lap("realign"));
    bool written = false;
    if (!combine(input_text, dir, result, written, err)) return false;
    have_output = written;
    lap("combine");
  } else if (!have_output || result.empty()) {
    result = tools.quickprobs_file(seq_file);
    tr.quickprobs_calls++;
    have_output = true;
  }
  if (!have_output) {   // os.path.getsize on a missing file
    err = "FileNotFoundError: the output file was never written";
    return false;
  }
  if (result.empty()) {   // MLProbs.py:95-99
    if (verbose) printf("[ERROR] Result is Empty ?\n");
    result = tools.quickprobs_file(seq_file);
    tr.quickprobs_calls++;
    tr.path += " fallback";
  }
  lap("fallback");
  say("[ELAPSED TIME] Total Running time: %.3f sec.\n", now() - t_start);
  return true;
}

}  // namespace mlpp
