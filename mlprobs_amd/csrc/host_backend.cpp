// host_backend.cpp -- see host_backend.h.  Reference code restated here:
//   ScoreType.h:36-68, 198-216, 251-285    EXP, LOOKUP, LOG_PLUS_EQUALS / LOG_ADD
//   ProbabilisticModel.h:153-493           forward, backward, totals, posterior (5-state and local)
//   ProbabilisticModel.h:804-864           ComputeAlignment (MEA)
//   ProbabilisticModel.h:1043-1170         ComputeViterbiAlignment
//   MSAPartProbs.cpp:78-394, 400-660       reverse / forward partition function (long double)
//   SparseMatrix.h:55-98, 205-248          sparse matrix, stable transpose
//   MSA.cpp:946-1025, 1670-1753            pid branches, RMS merge orders, distances
//   MSA.cpp:1172-1360                      DoRelaxation / Relax / Relax1
//   QP/Alignment/Multiple/PosteriorStage.cpp:123-196, PartitionFunction.cpp:71-291,
//   ConsistencyStage.cpp:133-300           QuickProbs' posterior and consistency stages
// All of it is plain host C++ (no HIP call), compiled without FMA
// contraction like the reference's scalar SSE build.
#include "host_backend.h"
#include "mlp_knobs.h"

#include <math.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <thread>

namespace mlph {

namespace {

constexpr float kLogZero = -2e20f;
constexpr float kLogOne = 0.0f;
constexpr float kUnderflow = 7.5f;   // LOG_UNDERFLOW_THRESHOLD
constexpr float kCutoff = 0.01f;     // POSTERIOR_CUTOFF

inline float lookup(float x) {
  if (x <= 1.00f) return ((-0.009350833524763f * x + 0.130659527668286f) * x + 0.498799810682272f) * x + 0.693203116424741f;
  if (x <= 2.50f) return ((-0.014532321752540f * x + 0.139942324101744f) * x + 0.495635523139337f) * x + 0.692140569840976f;
  if (x <= 4.50f) return ((-0.004605031767994f * x + 0.063427417320019f) * x + 0.695956496475118f) * x + 0.514272634594009f;
  return ((-0.000458661602210f * x + 0.009695946122598f) * x + 0.930734667215156f) * x + 0.168037164329057f;
}

inline float log_add(float x, float y) {
  if (x < y) return (x == kLogZero || y - x >= kUnderflow) ? y : lookup(y - x) + x;
  return (y == kLogZero || x - y >= kUnderflow) ? x : lookup(x - y) + y;
}

inline float exp_ref(float xf) {   // the double polynomial on the float argument
  const double x = xf;
  double r;
  if (x > -2) {
    if (x > -0.5) {
      if (x > 0) return (float)exp(x);
      r = (((0.03254409303190190000 * x + 0.16280432765779600000) * x + 0.49929760485974900000) * x +
           0.99995149601363700000) * x + 0.99999925508501600000;
    } else if (x > -1) {
      r = (((0.01973899026052090000 * x + 0.13822379685007000000) * x + 0.48056651562365000000) * x +
           0.99326940370383500000) * x + 0.99906756856399500000;
    } else {
      r = (((0.00940528203591384000 * x + 0.09414963667859410000) * x + 0.40825793595877300000) * x +
           0.93933625499130400000) * x + 0.98369508190545300000;
    }
  } else if (x > -8) {
    if (x > -4)
      r = (((0.00217245711583303000 * x + 0.03484829428350620000) * x + 0.22118199801337800000) * x +
           0.67049462206469500000) * x + 0.83556950223398500000;
    else
      r = (((0.00012398771025456900 * x + 0.00349155785951272000) * x + 0.03727721426017900000) * x +
           0.17974997741536900000) * x + 0.33249299994217400000;
  } else if (x > -16) {
    r = (((0.00000051741713416603 * x + 0.00002721456879608080) * x + 0.00053418601865636800) * x +
         0.00464101989351936000) * x + 0.01507447981459420000;
  } else {
    return 0;
  }
  return (float)r;
}

// host threads over a work counter (OpenMP-free: the CLIs bring libgomp)
template <class F>
void parallel_for(int64_t n, int threads, F body) {
  if (threads <= 1 || n <= 1) {
    for (int64_t k = 0; k < n; k++) body(k);
    return;
  }
  std::atomic<int64_t> next(0);
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; t++)
    pool.emplace_back([&]() {
      for (int64_t k; (k = next.fetch_add(1)) < n;) body(k);
    });
  for (auto& th : pool) th.join();
}

struct PairSeqs {
  const char* s1;   // 0-based letters of the first sequence
  const char* s2;
  int L1, L2;
};

inline int lc(char c) { return c - 'A'; }

// 5-state forward (flag = true): F[5 * (i * W + j) + k]
void forward5(const mlp::Tables& T, const mlp::ModelScalars& ms, const PairSeqs& q, std::vector<float>& F) {
  const int L1 = q.L1, L2 = q.L2, W = L2 + 1;
  F.assign((size_t)5 * (L1 + 1) * W, kLogZero);
  auto at = [&](int i, int j) { return F.data() + (size_t)5 * ((size_t)i * W + j); };
  at(1, 1)[0] = ms.init[0] + T.match[lc(q.s1[0]) * 26 + lc(q.s2[0])];
  for (int k = 0; k < 2; k++) {
    at(1, 0)[2 * k + 1] = ms.init[2 * k + 1] + T.ins[lc(q.s1[0])];
    at(0, 1)[2 * k + 2] = ms.init[2 * k + 2] + T.ins[lc(q.s2[0])];
  }
  for (int i = 0; i <= L1; i++)
    for (int j = 0; j <= L2; j++) {
      if (!(i > 1 || j > 1)) continue;
      float* c = at(i, j);
      if (i > 0 && j > 0) {
        const float* d = at(i - 1, j - 1);
        float v = d[0] + ms.t[0][0];
        for (int k = 1; k < 5; k++) v = log_add(v, d[k] + ms.t[k][0]);
        c[0] = v + T.match[lc(q.s1[i - 1]) * 26 + lc(q.s2[j - 1])];
      }
      if (i > 0) {
        const float* u = at(i - 1, j);
        const float ins = T.ins[lc(q.s1[i - 1])];
        for (int k = 0; k < 2; k++)
          c[2 * k + 1] = ins + log_add(u[0] + ms.t[0][2 * k + 1], u[2 * k + 1] + ms.t[2 * k + 1][2 * k + 1]);
      }
      if (j > 0) {
        const float* l = at(i, j - 1);
        const float ins = T.ins[lc(q.s2[j - 1])];
        for (int k = 0; k < 2; k++)
          c[2 * k + 2] = ins + log_add(l[0] + ms.t[0][2 * k + 2], l[2 * k + 2] + ms.t[2 * k + 2][2 * k + 2]);
      }
    }
}

void backward5(const mlp::Tables& T, const mlp::ModelScalars& ms, const PairSeqs& q, std::vector<float>& B) {
  const int L1 = q.L1, L2 = q.L2, W = L2 + 1;
  B.assign((size_t)5 * (L1 + 1) * W, kLogZero);
  auto at = [&](int i, int j) { return B.data() + (size_t)5 * ((size_t)i * W + j); };
  for (int k = 0; k < 5; k++) at(L1, L2)[k] = ms.init[k];
  for (int i = L1; i >= 0; i--)
    for (int j = L2; j >= 0; j--) {
      float* c = at(i, j);
      if (i < L1 && j < L2) {
        const float pxy = at(i + 1, j + 1)[0] + T.match[lc(q.s1[i]) * 26 + lc(q.s2[j])];
        for (int k = 0; k < 5; k++) c[k] = log_add(c[k], pxy + ms.t[k][0]);
      }
      if (i < L1) {
        const float* dn = at(i + 1, j);
        const float ins = T.ins[lc(q.s1[i])];
        for (int k = 0; k < 2; k++) {
          c[0] = log_add(c[0], dn[2 * k + 1] + ins + ms.t[0][2 * k + 1]);
          c[2 * k + 1] = log_add(c[2 * k + 1], dn[2 * k + 1] + ins + ms.t[2 * k + 1][2 * k + 1]);
        }
      }
      if (j < L2) {
        const float* r = at(i, j + 1);
        const float ins = T.ins[lc(q.s2[j])];
        for (int k = 0; k < 2; k++) {
          c[0] = log_add(c[0], r[2 * k + 2] + ins + ms.t[0][2 * k + 2]);
          c[2 * k + 2] = log_add(c[2 * k + 2], r[2 * k + 2] + ins + ms.t[2 * k + 2][2 * k + 2]);
        }
      }
    }
}

// 3-state local model (flag = false)
void forward_local(const mlp::Tables& T, const mlp::ModelScalars& ms, const PairSeqs& q, std::vector<float>& F) {
  const int L1 = q.L1, L2 = q.L2, W = L2 + 1;
  F.assign((size_t)3 * (L1 + 1) * W, kLogZero);
  auto at = [&](int i, int j) { return F.data() + (size_t)3 * ((size_t)i * W + j); };
  const float two_rt1 = 2 * ms.rt1;
  for (int i = 0; i <= L1; i++)
    for (int j = 0; j <= L2; j++) {
      float* c = at(i, j);
      const int c1 = i ? lc(q.s1[i - 1]) : 0, c2 = j ? lc(q.s2[j - 1]) : 0;
      if (i == 1 && j == 1) c[0] = T.match[c1 * 26 + c2] - T.ins[c1] - T.ins[c2] - two_rt1;
      if (!(i > 1 || j > 1)) continue;
      if (i > 0 && j > 0) {
        const float* d = at(i - 1, j - 1);
        const float m = T.match[c1 * 26 + c2], i1 = T.ins[c1], i2 = T.ins[c2];
        float v = m - i1 - i2 - two_rt1;
        for (int k = 0; k < 3; k++) v = log_add(v, m - i1 - i2 + d[k] + ms.lt[k][0] - two_rt1);
        c[0] = v;
      }
      if (i > 0) {
        const float* u = at(i - 1, j);
        c[1] = log_add(u[0] + ms.lt[0][1] - ms.rt1, u[1] + ms.lt[1][1] - ms.rt1);
      }
      if (j > 0) {
        const float* l = at(i, j - 1);
        c[2] = log_add(l[0] + ms.lt[0][2] - ms.rt1, l[2] + ms.lt[2][2] - ms.rt1);
      }
    }
}

void backward_local(const mlp::Tables& T, const mlp::ModelScalars& ms, const PairSeqs& q, std::vector<float>& B) {
  const int L1 = q.L1, L2 = q.L2, W = L2 + 1;
  B.assign((size_t)3 * (L1 + 1) * W, kLogZero);
  auto at = [&](int i, int j) { return B.data() + (size_t)3 * ((size_t)i * W + j); };
  const float two_rt1 = 2 * ms.rt1;
  for (int i = L1; i >= 0; i--)
    for (int j = L2; j >= 0; j--) {
      float* c = at(i, j);
      c[0] = kLogOne;
      if (i < L1 && j < L2) {
        const int c1 = lc(q.s1[i]), c2 = lc(q.s2[j]);
        const float pxy = at(i + 1, j + 1)[0] + T.match[c1 * 26 + c2] - T.ins[c1] - T.ins[c2];
        for (int k = 0; k < 3; k++) c[k] = log_add(c[k], pxy + ms.lt[k][0] - two_rt1);
      }
      if (i < L1) {
        const float* dn = at(i + 1, j);
        c[0] = log_add(c[0], dn[1] + ms.lt[0][1] - ms.rt1);
        c[1] = log_add(c[1], dn[1] + ms.lt[1][1] - ms.rt1);
      }
      if (j < L2) {
        const float* r = at(i, j + 1);
        c[0] = log_add(c[0], r[2] + ms.lt[0][2] - ms.rt1);
        c[2] = log_add(c[2], r[2] + ms.lt[2][2] - ms.rt1);
      }
    }
}

// ComputeTotalProbability + ComputePosteriorMatrix (ProbabilisticModel.h:405-493)
void posterior_hmm(const mlp::Tables& T, const mlp::ModelScalars& ms, const PairSeqs& q, bool five,
                   const std::vector<float>& F, const std::vector<float>& B, std::vector<float>& P) {
  const int L1 = q.L1, L2 = q.L2, W = L2 + 1;
  const int S = five ? 5 : 3;
  float tf = kLogZero, tb = kLogZero;
  if (five) {
    const size_t last = (size_t)5 * ((size_t)(L1 + 1) * W - 1);
    for (int k = 0; k < 5; k++) tf = log_add(tf, F[last + k] + B[last + k]);
    const size_t c11 = (size_t)5 * (W + 1), c10 = (size_t)5 * W, c01 = 5;
    tb = F[c11] + B[c11];
    for (int k = 0; k < 2; k++) {
      tb = log_add(tb, F[c10 + 2 * k + 1] + B[c10 + 2 * k + 1]);
      tb = log_add(tb, F[c01 + 2 * k + 2] + B[c01 + 2 * k + 2]);
    }
  } else {
    const float two_rt1 = 2 * ms.rt1;
    for (int i = 1; i <= L1; i++)
      for (int j = 1; j <= L2; j++) {
        const size_t ij = (size_t)3 * ((size_t)i * W + j);
        const int c1 = lc(q.s1[i - 1]), c2 = lc(q.s2[j - 1]);
        tf = log_add(tf, F[ij]);
        tb = log_add(tb, B[ij] + T.match[c1 * 26 + c2] - T.ins[c1] - T.ins[c2] - two_rt1);
      }
  }
  const float total = (tf + tb) / 2;
  P.resize((size_t)(L1 + 1) * W);
  for (size_t c = 0; c < P.size(); c++) P[c] = exp_ref(std::min(kLogOne, F[c * S] + B[c * S] - total));
  P[0] = 0;
}

// ComputePostProbs: partf + revers_partf (MSAPartProbs.cpp:400-660, 78-394),
// in long double; seq0 = the pair's first sequence, seq1 the second.
// Returns false on the reference's "huge val" stop.
bool posterior_pf(const mlp::Tables& T, const mlp::ModelScalars& ms, const PairSeqs& q, std::vector<float>& P) {
  const int len0 = q.L1, len1 = q.L2;
  const double d = ms.pf_open, e = ms.pf_ext, endopen = 1.0, endext = 1.0;
  auto score = [&](char b, char a) { return T.sub[lc(b) * 26 + lc(a)]; };  // sub_matrix[S(seq1 i)][T(seq0 j)]
  const long double inf = HUGE_VALL;
  // ---- forward: Zm full (len1 + 1) x (len0 + 1), Ze / Zf two rows
  // per-thread buffers, reused across pairs (fresh large allocations fault
  // in new pages every time and serialise the threads in the kernel)
  static thread_local std::vector<long double> Zm, Ze, Zf, Rm, Re, Rf;
  Zm.assign((size_t)(len1 + 1) * (len0 + 1), 0.0L);
  Ze.assign(2 * (size_t)(len0 + 1), 0.0L);
  Zf.assign(2 * (size_t)(len0 + 1), 0.0L);
  auto zm = [&](int i, int j) -> long double& { return Zm[(size_t)i * (len0 + 1) + j]; };
  long double* Ze0 = Ze.data();
  long double* Ze1 = Ze.data() + len0 + 1;
  long double* Zf0 = Zf.data();
  long double* Zf1 = Zf.data() + len0 + 1;
  long double zz = 0;
  zm(0, 0) = 1.00;
  Zf0[0] = Ze0[0] = 0;
  Zf1[0] = zm(0, 0) * endopen;
  Ze0[1] = zm(0, 0) * endopen;
  for (int j = 2; j <= len0; j++) Ze0[j] = Ze0[j - 1] * endext;
  for (int i = 1; i <= len1; i++) {
    for (int j = 1; j <= len0; j++) {
      const double sc = score(q.s2[i - 1], q.s1[j - 1]);
      double open0 = d, open1 = d, extend0 = e, extend1 = e;
      if (i == len1) { open0 = endopen; extend0 = endext; }
      if (j == len0) { open1 = endopen; extend1 = endext; }
      Ze1[j] = zm(i, j - 1) * open0 + Ze1[j - 1] * extend0;
      if (Ze1[j] >= inf) return false;
      Zf1[j] = zm(i - 1, j) * open1 + Zf0[j] * extend1;
      if (Zf1[j] >= inf) return false;
      zm(i, j) = (zm(i - 1, j - 1) + Ze0[j - 1] + Zf0[j - 1]) * sc;
      if (zm(i, j) >= inf) return false;
      zz = zm(i, j) + Ze1[j] + Zf1[j];
    }
    for (int t = 0; t <= len0; t++) {
      Ze0[t] = Ze1[t];
      Ze1[t] = 0;
      Zf0[t] = Zf1[t];
      Zf1[t] = 0;
    }
    Zf1[0] = 1;
  }
  zm(0, 0) = zz;
  // ---- reverse: two rows of Zm / Ze / Zf; P(i, j) from Zfm
  Rm.assign(2 * (size_t)(len0 + 1), 0.0L);
  Re.assign(2 * (size_t)(len0 + 1), 0.0L);
  Rf.assign(2 * (size_t)(len0 + 1), 0.0L);
  long double* Rm0 = Rm.data();
  long double* Rm1 = Rm.data() + len0 + 1;
  long double* Re0 = Re.data();
  long double* Re1 = Re.data() + len0 + 1;
  long double* Rf0 = Rf.data();
  long double* Rf1 = Rf.data() + len0 + 1;
  P.assign((size_t)(len0 + 1) * (len1 + 1), 0.0f);
  Rm1[len0] = 1;
  Re0[len0] = Rf0[len0] = 0;
  Rf1[len0] = Rm1[len0] * endopen;
  Re0[len0 - 1] = Rm1[len0] * endopen;
  for (int j = len0 - 2; j >= 0; j--) Re0[j] = Re0[j + 1] * endext;
  for (int i = len1 - 1; i >= 0; i--) {
    for (int j = len0 - 1; j >= 0; j--) {
      const double sc = score(q.s2[i], q.s1[j]);
      double open0 = d, open1 = d, extend0 = e, extend1 = e;
      if (i == 0) { open0 = endopen; extend0 = endext; }
      if (j == 0) { open1 = endopen; extend1 = endext; }
      Rf1[j] = Rm1[j] * open1 + Rf0[j] * extend1;
      Re1[j] = Rm0[j + 1] * open0 + Re1[j + 1] * extend0;
      Rm0[j] = (Rm1[j + 1] + Rf0[j + 1] + Re0[j + 1]) * sc;
      long double tv = zm(i + 1, j + 1) * Rm0[j];
      tv /= (sc * zm(0, 0));
      P[(size_t)(j + 1) * (len1 + 1) + (i + 1)] = (float)tv;
    }
    for (int t = 0; t <= len0; t++) {
      Re0[t] = Re1[t];
      Re1[t] = 0;
      Rf0[t] = Rf1[t];
      Rf1[t] = 0;
      Rm1[t] = Rm0[t];
      Rm0[t] = 0;
    }
    Rf0[len0] = 1;
  }
  P[0] = 0;
  return true;
}

// ComputeAlignment's value recurrence and the #B of its traced path
// (ProbabilisticModel.h:804-864; ChooseBestOfThree, ScoreType.h:347-366)
float mea_score(int L1, int L2, const std::vector<float>& P, int* nb) {
  const int W = L2 + 1;
  std::vector<float> o(W, 0.f), n(W, 0.f);
  std::vector<int> oc(W, 0), ncnt(W, 0);
  for (int i = 1; i <= L1; i++) {
    n[0] = 0;
    ncnt[0] = 0;
    const float* pr = P.data() + (size_t)i * W;
    for (int j = 1; j <= L2; j++) {
      const float x1 = pr[j] + o[j - 1], x2 = n[j - 1], x3 = o[j];
      if (x1 >= x2) {
        if (x1 >= x3) { n[j] = x1; ncnt[j] = oc[j - 1] + 1; }
        else { n[j] = x3; ncnt[j] = oc[j]; }
      } else if (x2 >= x3) {
        n[j] = x2; ncnt[j] = ncnt[j - 1];
      } else {
        n[j] = x3; ncnt[j] = oc[j];
      }
    }
    std::swap(o, n);
    std::swap(oc, ncnt);
  }
  if (nb) *nb = oc[L2];
  return o[L2];
}

// QuickProbs' PartitionFunction::computeForward / computeReverse
// (QP/Alignment/Multiple/PartitionFunction.cpp:71-156, 185-289): plain double,
// Zm over (L1 + 1) x (L2 + 1) rows of seq1, two-row Ze / Zf buffers; the
// posterior keeps values in [0.001, 1] (PartitionFunction.cpp:262-266).
void posterior_pf_qp(const mlp::Tables& T, const mlp::ModelScalars& ms, const PairSeqs& q, std::vector<float>& P) {
  const int L1 = q.L1, L2 = q.L2, lda = L2 + 1;
  const double go = ms.pf_open, ge = ms.pf_ext, tgo = 1.0, tge = 1.0;  // terminal gaps: exp(beta * 0)
  // T.sub is [seq2 letter][seq1 letter]
  auto score = [&](char c1, char c2) { return T.sub[lc(c2) * 26 + lc(c1)]; };
  static thread_local std::vector<double> Zm, buf;
  Zm.assign((size_t)(L1 + 1) * lda, 0.0);
  buf.assign(10 * (size_t)lda, 0.0);
  double* Ze = buf.data();            // rows 0 / 1 at Ze, Ze + lda
  double* Zf = buf.data() + 2 * lda;
  double zz = 0;
  Zm[0] = 1.0;
  Zf[0] = Ze[0] = 0;
  Zf[lda] = Zm[0] * tgo;
  Ze[1] = Zm[0] * tgo;
  for (int j = 2; j <= L2; j++) Ze[j] = Ze[j - 1] * tge;
  for (int i = 1; i <= L1; i++) {
    for (int j = 1; j <= L2; j++) {
      const double sc = score(q.s1[i - 1], q.s2[j - 1]);
      double open0 = go, extend0 = ge, open1 = go, extend1 = ge;
      if (i == L1) { open0 = tgo; extend0 = tge; }
      if (j == L2) { open1 = tgo; extend1 = tge; }
      Ze[lda + j] = Zm[(size_t)i * lda + j - 1] * open0 + Ze[lda + j - 1] * extend0;
      Zf[lda + j] = Zm[(size_t)(i - 1) * lda + j] * open1 + Zf[j] * extend1;
      Zm[(size_t)i * lda + j] = (Zm[(size_t)(i - 1) * lda + j - 1] + Ze[j - 1] + Zf[j - 1]) * sc;
      zz = Zm[(size_t)i * lda + j] + Ze[lda + j] + Zf[lda + j];
    }
    for (int t = 0; t <= L2; t++) {
      Ze[t] = Ze[lda + t];
      Ze[lda + t] = 0;
      Zf[t] = Zf[lda + t];
      Zf[lda + t] = 0;
    }
    Zf[lda] = 1;
  }
  Zm[0] = zz;
  double* Rm = buf.data() + 4 * lda;
  double* Re = buf.data() + 6 * lda;
  double* Rf = buf.data() + 8 * lda;
  P.assign((size_t)(L1 + 1) * lda, 0.0f);
  Rm[lda + L2] = 1;
  Re[L2] = Rf[L2] = 0;
  Rf[lda + L2] = Rm[lda + L2] * tgo;
  Re[L2 - 1] = Rm[lda + L2] * tgo;
  for (int j = L2 - 2; j >= 0; j--) Re[j] = Re[j + 1] * tge;
  for (int i = L1 - 1; i >= 0; i--) {
    for (int j = L2 - 1; j >= 0; j--) {
      const double sc = score(q.s1[i], q.s2[j]);
      double open0 = go, extend0 = ge, open1 = go, extend1 = ge;
      if (i == 0) { open0 = tgo; extend0 = tge; }
      if (j == 0) { open1 = tgo; extend1 = tge; }
      Rf[lda + j] = Rm[lda + j] * open1 + Rf[j] * extend1;
      Re[lda + j] = Rm[j + 1] * open0 + Re[lda + j + 1] * extend0;
      Rm[j] = (Rm[lda + j + 1] + Rf[j + 1] + Re[j + 1]) * sc;
      double tv = Zm[(size_t)(i + 1) * lda + j + 1] * Rm[j];
      tv /= (sc * Zm[0]);
      const float prob = (float)tv;
      if (prob <= 1 && prob >= 0.001) P[(size_t)(i + 1) * lda + j + 1] = prob;
    }
    for (int t = 0; t <= L2; t++) {
      Re[t] = Re[lda + t];
      Re[lda + t] = 0;
      Rf[t] = Rf[lda + t];
      Rf[lda + t] = 0;
      Rm[lda + t] = Rm[t];
      Rm[t] = 0;
    }
    Rf[L2] = 1;
  }
  P[0] = 0;
}

inline float fixed16(float v) { return (float)(uint32_t)(uint16_t)(v * 65535.0f) / 65535.0f; }

}  // namespace

int threads_for(int64_t units) {
  static const int hw = [] {
    const int t = (int)mlp::knob("MLP_HOST_THREADS", (double)std::thread::hardware_concurrency());
    return std::max(1, std::min(t, 16));
  }();
  return (int)std::max<int64_t>(1, std::min<int64_t>(hw, units));
}

void viterbi(const mlp::Tables& T, const mlp::ModelScalars& ms, const FamilyView& f, int64_t p0, int64_t p1,
             int32_t* len_out, float* match_out, const int64_t* vit_off, uint8_t* paths) {
  parallel_for(p1 - p0, threads_for(p1 - p0), [&](int64_t k) {
    const int64_t p = p0 + k;
    const int a = f.pa[p], b = f.pb[p];
    const char* s1 = (const char*)f.res + f.offs[a];
    const char* s2 = (const char*)f.res + f.offs[b];
    const int L1 = f.lens[a], L2 = f.lens[b], W = L2 + 1;
    static thread_local std::vector<float> V;
    static thread_local std::vector<int8_t> tb;
    V.assign((size_t)3 * (L1 + 1) * W, kLogZero);
    tb.assign((size_t)3 * (L1 + 1) * W, -1);
    V[0] = ms.vit_init[0];
    V[1] = ms.vit_init[1];
    V[2] = ms.vit_init[2];
    for (int i = 0; i <= L1; i++)
      for (int j = 0; j <= L2; j++) {
        const size_t ij = (size_t)3 * ((size_t)i * W + j);
        const int c1 = i ? lc(s1[i - 1]) : 0, c2 = j ? lc(s2[j - 1]) : 0;
        if (i > 0 && j > 0) {
          const size_t d = ij - (size_t)3 * (W + 1);
          for (int k = 0; k < 3; k++) {
            const float nv = V[k + d] + ms.lt[k][0] + T.match[c1 * 26 + c2];
            if (V[ij] < nv) { V[ij] = nv; tb[ij] = (int8_t)k; }
          }
        }
        if (i > 0) {
          const size_t u = ij - (size_t)3 * W;
          const float fm = T.ins[c1] + V[u] + ms.lt[0][1], fi = T.ins[c1] + V[1 + u] + ms.lt[1][1];
          if (fm >= fi) { V[1 + ij] = fm; tb[1 + ij] = 0; } else { V[1 + ij] = fi; tb[1 + ij] = 1; }
        }
        if (j > 0) {
          const size_t l = ij - 3;
          const float fm = T.ins[c2] + V[l] + ms.lt[0][2], fi = T.ins[c2] + V[2 + l] + ms.lt[2][2];
          if (fm >= fi) { V[2 + ij] = fm; tb[2 + ij] = 0; } else { V[2 + ij] = fi; tb[2 + ij] = 2; }
        }
      }
    float best = kLogZero;
    int state = -1;
    const size_t last = (size_t)3 * ((size_t)(L1 + 1) * W - 1);
    for (int k = 0; k < 3; k++) {
      const float v = V[k + last] + ms.vit_init[k];
      if (best < v) { best = v; state = k; }
    }
    // traceback (reverse order), then the identity count in forward order
    std::vector<uint8_t> rev;
    rev.reserve(L1 + L2);
    int r = L1, c = L2;
    while (r != 0 || c != 0) {
      const int ns = tb[(size_t)state + (size_t)3 * ((size_t)r * W + c)];
      if (state == 0) { c--; r--; rev.push_back(0); }
      else if (state % 2 == 1) { r--; rev.push_back(1); }
      else { c--; rev.push_back(2); }
      state = ns;
    }
    const int n = (int)rev.size();
    float nm = 0;
    int i = 0, j = 0;
    for (int t = n - 1; t >= 0; t--) {
      if (rev[t] == 0) {
        if (s1[i] == s2[j]) nm += 1;
        i++;
        j++;
      } else if (rev[t] == 1) {
        i++;
      } else {
        j++;
      }
    }
    len_out[p] = n;
    match_out[p] = nm;
    if (paths)
      for (int t = 0; t < n; t++) paths[vit_off[p] + t] = rev[n - 1 - t];
  });
}

int posteriors(const mlp::Tables& T, const mlp::ModelScalars& ms, const FamilyView& f, int pid, bool npdo,
               int64_t p0, int64_t p1, const std::vector<int64_t>& rp_off, Store& st, float* dist, float* mea,
               int64_t* nnz, std::string& err) {
  const int64_t np = p1 - p0;
  std::vector<std::vector<uint16_t>> pc(np);
  std::vector<std::vector<float>> pv(np);
  std::atomic<int64_t> bad(-1);
  parallel_for(np, threads_for(np), [&](int64_t k) {
    const int64_t p = p0 + k;
    const int a = f.pa[p], b = f.pb[p];
    PairSeqs q{(const char*)f.res + f.offs[a], (const char*)f.res + f.offs[b], f.lens[a], f.lens[b]};
    const int W = q.L2 + 1;
    static thread_local std::vector<float> F, B, post, p5, pg;
    if (pid == 2 || pid < 2) {   // local model (CPNP/MSA.cpp:946-957, 979-989)
      forward_local(T, ms, q, F);
      backward_local(T, ms, q, B);
      posterior_hmm(T, ms, q, false, F, B, post);
    }
    if (pid != 2) {
      if (!posterior_pf(T, ms, q, pg)) {
        int64_t none = -1;
        bad.compare_exchange_strong(none, p);
        return;
      }
      if (pid >= 3) post.swap(pg);
    }
    if (pid < 2) {   // 5-state and the RMS merge (CPNP/MSA.cpp:992-1001; npdo: 1699-1708)
      forward5(T, ms, q, F);
      backward5(T, ms, q, B);
      posterior_hmm(T, ms, q, true, F, B, p5);
      for (size_t c = 0; c < post.size(); c++) {
        const float v1 = p5[c], v2 = pg[c], v3 = post[c];
        post[c] = npdo ? sqrtf((v2 * v2 + v3 * v3 + v1 * v1) / 3) : sqrtf((v1 * v1 + v2 * v2 + v3 * v3) / 3);
      }
    }
    int nb = 0;
    const float sc = mea_score(q.L1, q.L2, post, &nb);
    mea[p] = sc;
    dist[p] = npdo ? sc / (float)nb : 1.0f - sc / (float)std::min(q.L1, q.L2);
    // SparseMatrix (SparseMatrix.h:55-98), canonical row pointers
    int32_t* rp = st.rowptr.data() + rp_off[p];
    rp[0] = rp[1] = 0;
    std::vector<uint16_t>& cc = pc[k];
    std::vector<float>& vv = pv[k];
    for (int i = 1; i <= q.L1; i++) {
      const float* row = post.data() + (size_t)i * W;
      for (int j = 1; j <= q.L2; j++)
        if (row[j] >= kCutoff) {
          cc.push_back((uint16_t)j);
          vv.push_back(row[j]);
        }
      rp[i + 1] = (int32_t)cc.size();
    }
  });
  if (bad.load() >= 0) {
    err = "partition function overflow (pair " + std::to_string(bad.load()) + "): huge val, as the reference";
    return 3;
  }
  int64_t run = st.ent_off[p0];
  for (int64_t k = 0; k < np; k++) {
    st.ent_off[p0 + k] = run;
    nnz[p0 + k] = (int64_t)pc[k].size();
    run += (int64_t)pc[k].size();
  }
  st.ent_off[p1] = run;
  st.cols.resize(run);
  st.vals.resize(run);
  for (int64_t k = 0; k < np; k++) {
    std::copy(pc[k].begin(), pc[k].end(), st.cols.begin() + st.ent_off[p0 + k]);
    std::copy(pv[k].begin(), pv[k].end(), st.vals.begin() + st.ent_off[p0 + k]);
  }
  return 0;
}

void qp_posteriors(const mlp::Tables& T, const mlp::ModelScalars& ms, const FamilyView& f, int64_t p0, int64_t p1,
                   float cutoff, const std::vector<int64_t>& rp_off, Store& st, float* dist, float* mea,
                   int64_t* nnz) {
  const int64_t np = p1 - p0;
  std::vector<std::vector<uint16_t>> pc(np);
  std::vector<std::vector<float>> pv(np);
  parallel_for(np, threads_for(np), [&](int64_t k) {
    const int64_t p = p0 + k;
    const int a = f.pa[p], b = f.pb[p];
    PairSeqs q{(const char*)f.res + f.offs[a], (const char*)f.res + f.offs[b], f.lens[a], f.lens[b]};
    const int W = q.L2 + 1;
    static thread_local std::vector<float> F, B, ph, pf, oldr, newr;
    posterior_pf_qp(T, ms, q, pf);
    forward5(T, ms, q, F);
    backward5(T, ms, q, B);
    posterior_hmm(T, ms, q, true, F, B, ph);
    // combineMatrices (PosteriorStage.cpp:160-196): the RMS in place of ph,
    // the MEA value recurrence over two rows
    oldr.assign(W, 0.f);
    newr.assign(W, 0.f);
    for (int i = 0; i <= q.L1; i++) {
      for (int j = 0; j <= q.L2; j++) {
        const size_t c = (size_t)i * W + j;
        if (i == 0 || j == 0) {
          ph[c] = 0;
          newr[j] = 0;
        } else {
          const float v1 = ph[c], v2 = pf[c];
          ph[c] = sqrtf((v1 * v1 + v2 * v2) * 0.5f);
          const float x = ph[c] + oldr[j - 1], y = newr[j - 1], z = oldr[j];
          newr[j] = x >= y ? (x >= z ? x : z) : (y >= z ? y : z);
        }
      }
      std::swap(oldr, newr);
    }
    const float total = oldr[q.L2];
    mea[p] = total;
    dist[p] = 1.0f - total / (float)std::min(q.L1, q.L2);
    int32_t* rp = st.rowptr.data() + rp_off[p];
    rp[0] = rp[1] = 0;
    std::vector<uint16_t>& cc = pc[k];
    std::vector<float>& vv = pv[k];
    cc.clear();
    vv.clear();
    for (int i = 1; i <= q.L1; i++) {
      const float* row = ph.data() + (size_t)i * W;
      for (int j = 1; j <= q.L2; j++)
        if (row[j] >= cutoff) {
          cc.push_back((uint16_t)j);
          vv.push_back(fixed16(row[j]));
        }
      rp[i + 1] = (int32_t)cc.size();
    }
  });
  int64_t run = st.ent_off[p0];
  for (int64_t k = 0; k < np; k++) {
    st.ent_off[p0 + k] = run;
    nnz[p0 + k] = (int64_t)pc[k].size();
    run += (int64_t)pc[k].size();
  }
  st.ent_off[p1] = run;
  st.cols.resize(run);
  st.vals.resize(run);
  for (int64_t k = 0; k < np; k++) {
    std::copy(pc[k].begin(), pc[k].end(), st.cols.begin() + st.ent_off[p0 + k]);
    std::copy(pv[k].begin(), pv[k].end(), st.vals.begin() + st.ent_off[p0 + k]);
  }
}

void relax(const FamilyView& f, const std::vector<int64_t>& rp_off, Store& st, int64_t* nnz, const QpRelaxHost* qp,
           int64_t r0, int64_t r1) {
  const int n = f.n;
  const int64_t P = (int64_t)n * (n - 1) / 2;
  if (r1 < 0) r1 = P;
  const int64_t nout = r1 - r0;
  auto pidx = [&](int a, int b) { return (int64_t)a * n - (int64_t)a * (a + 1) / 2 + (b - a - 1); };
  // stable transposes of every block (SparseMatrix::ComputeTranspose): rows
  // = the second sequence's residues, entries in the first sequence's order
  std::vector<int64_t> trp_off(P + 1, 0);
  for (int64_t p = 0; p < P; p++) trp_off[p + 1] = trp_off[p] + f.lens[f.pb[p]] + 2;
  std::vector<int32_t> trp(trp_off[P]);
  std::vector<uint16_t> tcols(st.cols.size());
  std::vector<float> tvals(st.vals.size());
  parallel_for(P, threads_for(P), [&](int64_t p) {
    const int La = f.lens[f.pa[p]], Lb = f.lens[f.pb[p]];
    const int32_t* rp = st.rowptr.data() + rp_off[p];
    const int64_t e0 = st.ent_off[p];
    int32_t* t = trp.data() + trp_off[p];
    std::fill(t, t + Lb + 2, 0);
    for (int32_t e = 0; e < rp[La + 1]; e++) t[st.cols[e0 + e] + 1]++;
    for (int r = 1; r <= Lb + 1; r++) t[r] += t[r - 1];   // t[r] = start of row r (r >= 1)
    std::vector<int32_t> cur(t, t + Lb + 1);
    for (int i = 1; i <= La; i++)
      for (int32_t e = rp[i]; e < rp[i + 1]; e++) {
        const int c = st.cols[e0 + e];
        const int32_t pos = cur[c]++;
        tcols[e0 + pos] = (uint16_t)i;
        tvals[e0 + pos] = st.vals[e0 + e];
      }
  });
  // row r of P(x, z) as (cols, vals, begin, end)
  struct Row { const uint16_t* c; const float* v; int32_t b, e; };
  auto row_of = [&](int x, int z, int r) -> Row {
    if (x < z) {
      const int64_t p = pidx(x, z);
      const int32_t* rp = st.rowptr.data() + rp_off[p];
      return {st.cols.data() + st.ent_off[p], st.vals.data() + st.ent_off[p], rp[r], rp[r + 1]};
    }
    const int64_t p = pidx(z, x);
    const int32_t* rp = trp.data() + trp_off[p];
    return {tcols.data() + st.ent_off[p], tvals.data() + st.ent_off[p], rp[r], rp[r + 1]};
  };
  std::vector<std::vector<uint16_t>> nc(P);
  std::vector<std::vector<float>> nv(P);
  std::vector<int32_t> nrp(st.rowptr.size());
  parallel_for(nout, threads_for(nout), [&](int64_t k) {
    const int64_t p = r0 + k;
    const int x = f.pa[p], y = f.pb[p];
    const int Lx = f.lens[x], Ly = f.lens[y], W = Ly + 1;
    const int32_t* rp = st.rowptr.data() + rp_off[p];
    const uint16_t* cx = st.cols.data() + st.ent_off[p];
    const float* vx = st.vals.data() + st.ent_off[p];
    // GetPosterior (dense), z = x and z = y: posterior += posterior
    static thread_local std::vector<float> post;
    post.assign((size_t)(Lx + 1) * W, 0.f);
    for (int i = 1; i <= Lx; i++)
      for (int32_t e = rp[i]; e < rp[i + 1]; e++) post[(size_t)i * W + cx[e]] = vx[e];
    // QuickProbs: z accepted by the selectivity filter (ConsistencyStage.cpp:
    // 180-203), its weight w_z / W_xy, the weight sum in z order
    auto accept = [&](int z) {
      if (!qp->seldist) return true;
      const float dx = qp->seldist[(size_t)x * n + z], dy = qp->seldist[(size_t)y * n + z];
      return (dx > dy ? dx : dy) <= qp->selectivity;
    };
    float wxy = 0.f, sumw = 1.0f;
    if (qp) {
      int accepted = 0;
      for (int z = 0; z < n; z++) accepted += z != x && z != y && accept(z);
      wxy = 1.0f + (qp->selfweight - 1.0f) * (float)accepted / qp->selectivity;
      wxy *= qp->weights[x] + qp->weights[y];
    } else {
      for (float& v : post) v += v;   // z = x and z = y (CPNP/MSA.cpp:1211-1213)
    }
    // z ascending; Relax / Relax1 / transposed Relax all add, per cell, the
    // terms of z's k in ascending order
    for (int z = 0; z < n; z++) {
      if (z == x || z == y) continue;
      float wz = 1.0f;
      if (qp) {
        if (!accept(z)) continue;
        wz = qp->weights[z] / wxy;
        sumw += wz;
      }
      for (int i = 1; i <= Lx; i++) {
        const Row A = row_of(x, z, i);
        float* base = post.data() + (size_t)i * W;
        for (int32_t u = A.b; u < A.e; u++) {
          const Row Bk = row_of(z, y, A.c[u]);
          const float a = qp ? wz * A.v[u] : A.v[u];   // weight * XZ * ZY (ConsistencyStage.cpp:294)
          for (int32_t w = Bk.b; w < Bk.e; w++) base[Bk.c[w]] += a * Bk.v[w];
        }
      }
    }
    const float div = qp ? sumw : (float)n;
    for (float& v : post) v /= div;
    // mask to the old pattern, then SparseMatrix at the cutoff
    const float cut = qp ? qp->cutoff : kCutoff;
    int32_t* out = nrp.data() + rp_off[p];
    out[0] = out[1] = 0;
    for (int i = 1; i <= Lx; i++) {
      for (int32_t e = rp[i]; e < rp[i + 1]; e++) {
        const float v = post[(size_t)i * W + cx[e]];
        if (v >= cut) {
          nc[p].push_back(cx[e]);
          nv[p].push_back(qp ? fixed16(v) : v);
        }
      }
      out[i + 1] = (int32_t)nc[p].size();
    }
  });
  int64_t run = 0;
  for (int64_t p = 0; p < P; p++) {
    st.ent_off[p] = run;
    if (p >= r0 && p < r1) nnz[p] = (int64_t)nc[p].size();
    run += (int64_t)nc[p].size();
  }
  st.ent_off[P] = run;
  st.cols.resize(run);
  st.vals.resize(run);
  for (int64_t p = r0; p < r1; p++) {
    std::copy(nc[p].begin(), nc[p].end(), st.cols.begin() + st.ent_off[p]);
    std::copy(nv[p].begin(), nv[p].end(), st.vals.begin() + st.ent_off[p]);
  }
  st.rowptr.swap(nrp);
}

}  // namespace mlph
