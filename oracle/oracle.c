/* oracle.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CPU restatement of the reference hot path in plain C.  Each function cites
 * the reference lines it follows.  Compiled with -ffp-contract=off and no
 * fast-math so every float operation rounds exactly like the reference's
 * x86-64 SSE build (CPNP/Makefile:1-16, no -march => no FMA).
 */
#include "oracle.h"

#include <ctype.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../mlprobs_amd/csrc/mlp_params_default.inc"
#include "../mlprobs_amd/csrc/mlp_params_qp.inc"

#define LOG_ZERO (-2e20f)
#define LOG_ONE (0.0f)
#define LOG_UNDERFLOW_THRESHOLD (7.5f)
#define POSTERIOR_CUTOFF (0.01f)

/* CPNP/ScoreType.h:26-28.  The reference's float LOG resolves to the float
 * overload of std::log (pinned by tests/test_oracle_golden.py::test_tables). */
static float LOG(float x) { return logf(x); }

/* CPNP/ScoreType.h:36-68: piecewise quartic with double coefficients. */
static float EXP(float xf) {
  double x = xf;
  if (x > -2) {
    if (x > -0.5) {
      if (x > 0) return (float)exp(x);
      return (float)((((0.03254409303190190000 * x + 0.16280432765779600000) * x +
                       0.49929760485974900000) * x + 0.99995149601363700000) * x +
                     0.99999925508501600000);
    }
    if (x > -1)
      return (float)((((0.01973899026052090000 * x + 0.13822379685007000000) * x +
                       0.48056651562365000000) * x + 0.99326940370383500000) * x +
                     0.99906756856399500000);
    return (float)((((0.00940528203591384000 * x + 0.09414963667859410000) * x +
                     0.40825793595877300000) * x + 0.93933625499130400000) * x +
                   0.98369508190545300000);
  }
  if (x > -8) {
    if (x > -4)
      return (float)((((0.00217245711583303000 * x + 0.03484829428350620000) * x +
                       0.22118199801337800000) * x + 0.67049462206469500000) * x +
                     0.83556950223398500000);
    return (float)((((0.00012398771025456900 * x + 0.00349155785951272000) * x +
                     0.03727721426017900000) * x + 0.17974997741536900000) * x +
                   0.33249299994217400000);
  }
  if (x > -16)
    return (float)((((0.00000051741713416603 * x + 0.00002721456879608080) * x +
                     0.00053418601865636800) * x + 0.00464101989351936000) * x +
                   0.01507447981459420000);
  return 0;
}

/* CPNP/ScoreType.h:196-216: log(1+e^x) on [0, 7.5], piecewise cubic. */
static float LOOKUP(float x) {
  if (x <= 1.00f)
    return ((-0.009350833524763f * x + 0.130659527668286f) * x + 0.498799810682272f) * x +
           0.693203116424741f;
  if (x <= 2.50f)
    return ((-0.014532321752540f * x + 0.139942324101744f) * x + 0.495635523139337f) * x +
           0.692140569840976f;
  if (x <= 4.50f)
    return ((-0.004605031767994f * x + 0.063427417320019f) * x + 0.695956496475118f) * x +
           0.514272634594009f;
  return ((-0.000458661602210f * x + 0.009695946122598f) * x + 0.930734667215156f) * x +
         0.168037164329057f;
}

/* CPNP/ScoreType.h:251-258 and 279-285. */
static float LOG_ADD(float x, float y) {
  if (x < y) return (x == LOG_ZERO || y - x >= LOG_UNDERFLOW_THRESHOLD) ? y : LOOKUP(y - x) + x;
  return (y == LOG_ZERO || x - y >= LOG_UNDERFLOW_THRESHOLD) ? x : LOOKUP(x - y) + y;
}
#define LOG_PLUS_EQUALS(x, y) ((x) = LOG_ADD((x), (y)))

/* ---------------------------------------------------------------- tables */

void orc_model_init(orc_model *m, float delta) {
  /* CPNP/MSA.cpp:444-500: defaults, unknown residues 1e-10 / 1e-5. */
  static float emitPairs[256][256];
  static float emitSingle[256];
  float initDistrib[5], gapOpen[4], gapExtend[4];
  for (int i = 0; i < 256; i++) {
    emitSingle[i] = (float)1e-5;
    for (int j = 0; j < 256; j++) emitPairs[i][j] = (float)1e-10;
  }
  memcpy(initDistrib, mlp_init_distrib, sizeof initDistrib);
  memcpy(gapOpen, mlp_gap_open, sizeof gapOpen);
  memcpy(gapExtend, mlp_gap_extend, sizeof gapExtend);
  if (delta >= 0) initDistrib[2] = delta;
  const char *alpha = MLP_ALPHABET;
  int tri = 0;
  for (int i = 0; i < 20; i++) {
    unsigned char ui = (unsigned char)toupper(alpha[i]), li = (unsigned char)tolower(alpha[i]);
    emitSingle[li] = emitSingle[ui] = mlp_emit_single[i];
    for (int j = 0; j <= i; j++, tri++) {
      unsigned char uj = (unsigned char)toupper(alpha[j]), lj = (unsigned char)tolower(alpha[j]);
      float v = mlp_emit_pairs_lower[tri];
      emitPairs[li][lj] = emitPairs[li][uj] = emitPairs[ui][lj] = emitPairs[ui][uj] = v;
      emitPairs[lj][li] = emitPairs[lj][ui] = emitPairs[uj][li] = emitPairs[uj][ui] = v;
    }
  }
  /* CPNP/ProbabilisticModel.h:75-99 */
  float tm[5][5];
  memset(tm, 0, sizeof tm);
  tm[0][0] = 1;
  for (int i = 0; i < 2; i++) {
    tm[0][2 * i + 1] = gapOpen[2 * i];
    tm[0][2 * i + 2] = gapOpen[2 * i];
    tm[0][0] -= (gapOpen[2 * i] + gapOpen[2 * i]);
    tm[2 * i + 1][2 * i + 1] = gapExtend[2 * i];
    tm[2 * i + 2][2 * i + 2] = gapExtend[2 * i];
    tm[2 * i + 1][2 * i + 2] = 0;
    tm[2 * i + 2][2 * i + 1] = 0;
    tm[2 * i + 1][0] = 1 - gapExtend[2 * i];
    tm[2 * i + 2][0] = 1 - gapExtend[2 * i];
  }
  for (int i = 0; i < 5; i++) {
    m->initialDistribution[i] = LOG(initDistrib[i]);
    for (int j = 0; j < 5; j++) m->transProb[i][j] = LOG(tm[i][j]);
  }
  m->initialDistribution[2] = LOG(initDistrib[1]);
  /* CPNP/ProbabilisticModel.h:102-107 */
  for (int i = 0; i < 256; i++) {
    for (int j = 0; j < 5; j++) m->insProb[i][j] = LOG(emitSingle[i]);
    for (int j = 0; j < 256; j++) m->matchProb[i][j] = LOG(emitPairs[i][j]);
  }
  /* CPNP/ProbabilisticModel.h:111-133 */
  float lt[3][3];
  memset(lt, 0, sizeof lt);
  lt[0][0] = 1;
  lt[0][1] = gapOpen[1];
  lt[0][2] = gapOpen[1];
  lt[0][0] -= (gapOpen[1] + gapOpen[1]);
  lt[1][1] = gapExtend[1];
  lt[2][2] = gapExtend[1];
  lt[1][2] = 0;
  lt[2][1] = 0;
  lt[1][0] = 1 - gapExtend[1];
  lt[2][0] = 1 - gapExtend[1];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) m->local_transProb[i][j] = LOG(lt[i][j]);
  m->random_transProb[0] = LOG(initDistrib[2]);
  m->random_transProb[1] = LOG(1 - initDistrib[2]);
}

void orc_pf_tables(double sub_matrix[26][26], int subst_index[26]) {
  /* CPNP/MSAReadMatrix.cpp:85-116 with beta = 1/T, T = 5 (CPNP/MSA.cpp:78,
   * MSAReadMatrix.cpp:171).  The reference evaluates exp() on a float
   * argument through the float overload. */
  const char *bases = MLP_GONNET_MONOMERS;
  int n = (int)strlen(bases), pos = 0;
  float beta = (float)(1.0 / 5.0f);
  memset(sub_matrix, 0, sizeof(double) * 26 * 26);
  for (int i = 0; i < n; i++) subst_index[i] = -1;
  for (int i = 0; i < n; i++) subst_index[bases[i] - 'A'] = i;
  for (int i = 0; i < n; i++)
    for (int j = 0; j <= i; j++) {
      double v = expf(beta * mlp_gonnet160_lower[pos++]);
      sub_matrix[i][j] = v;
      sub_matrix[j][i] = v;
    }
}

float orc_delta_for_identity(float identity, float d) {
  if (identity <= 0.125) return 0.108854f;
  if (identity <= 0.15) return 0.132548f;
  if (identity <= 0.175) return 0.165248f;
  if (identity <= 0.2) return 0.168284f;
  if (identity <= 0.25) return 0.170705f;
  if (identity <= 0.3) return 0.100675f;
  if (identity <= 0.35) return 0.090755f;
  if (identity <= 0.4) return 0.146188f;
  if (identity <= 0.45) return 0.167858f;
  if (identity <= 0.5) return 0.250769f;
  return d;
}

/* ------------------------------------------------------------- pair HMMs */

void orc_forward(const orc_model *m, const char *s1, int L1, const char *s2, int L2, int flag,
                 float *F) {
  const int S = flag ? 5 : 3;
  const int W = L2 + 1;
  const size_t n = (size_t)S * (L1 + 1) * W;
  for (size_t k = 0; k < n; k++) F[k] = LOG_ZERO;
  const float rt1 = m->random_transProb[1];
  /* CPNP/ProbabilisticModel.h:173-183 */
  if (flag) {
    F[0 + S * (1 * W + 1)] =
        m->initialDistribution[0] + m->matchProb[(unsigned char)s1[1]][(unsigned char)s2[1]];
    for (int k = 0; k < 2; k++) {
      F[2 * k + 1 + S * (1 * W + 0)] =
          m->initialDistribution[2 * k + 1] + m->insProb[(unsigned char)s1[1]][k];
      F[2 * k + 2 + S * (0 * W + 1)] =
          m->initialDistribution[2 * k + 2] + m->insProb[(unsigned char)s2[1]][k];
    }
  }
  /* CPNP/ProbabilisticModel.h:205-271 */
  for (int i = 0; i <= L1; i++) {
    unsigned char c1 = (i == 0) ? '~' : (unsigned char)s1[i];
    for (int j = 0; j <= L2; j++) {
      unsigned char c2 = (j == 0) ? '~' : (unsigned char)s2[j];
      float *ij = F + (size_t)S * ((size_t)i * W + j);
      if (i == 1 && j == 1 && !flag)
        ij[0] = m->matchProb[c1][c2] - m->insProb[c1][0] - m->insProb[c2][0] - 2 * rt1;
      if (i > 1 || j > 1) {
        if (i > 0 && j > 0) {
          const float *i1j1 = ij - S * (W + 1);
          if (flag) {
            ij[0] = i1j1[0] + m->transProb[0][0];
            for (int k = 1; k < 5; k++) LOG_PLUS_EQUALS(ij[0], i1j1[k] + m->transProb[k][0]);
            ij[0] += m->matchProb[c1][c2];
          } else {
            ij[0] = m->matchProb[c1][c2] - m->insProb[c1][0] - m->insProb[c2][0] - 2 * rt1;
            for (int k = 0; k < 3; k++)
              LOG_PLUS_EQUALS(ij[0], m->matchProb[c1][c2] - m->insProb[c1][0] -
                                         m->insProb[c2][0] + i1j1[k] +
                                         m->local_transProb[k][0] - 2 * rt1);
          }
        }
        if (i > 0) {
          const float *i1j = ij - S * W;
          if (flag) {
            for (int k = 0; k < 2; k++)
              ij[2 * k + 1] = m->insProb[c1][k] +
                              LOG_ADD(i1j[0] + m->transProb[0][2 * k + 1],
                                      i1j[2 * k + 1] + m->transProb[2 * k + 1][2 * k + 1]);
          } else {
            ij[1] = LOG_ADD(i1j[0] + m->local_transProb[0][1] - rt1,
                            i1j[1] + m->local_transProb[1][1] - rt1);
          }
        }
        if (j > 0) {
          const float *ij1 = ij - S;
          if (flag) {
            for (int k = 0; k < 2; k++)
              ij[2 * k + 2] = m->insProb[c2][k] +
                              LOG_ADD(ij1[0] + m->transProb[0][2 * k + 2],
                                      ij1[2 * k + 2] + m->transProb[2 * k + 2][2 * k + 2]);
          } else {
            ij[2] = LOG_ADD(ij1[0] + m->local_transProb[0][2] - rt1,
                            ij1[2] + m->local_transProb[2][2] - rt1);
          }
        }
      }
    }
  }
}

void orc_backward(const orc_model *m, const char *s1, int L1, const char *s2, int L2, int flag,
                  float *B) {
  const int S = flag ? 5 : 3;
  const int W = L2 + 1;
  const size_t n = (size_t)S * (L1 + 1) * W;
  for (size_t k = 0; k < n; k++) B[k] = LOG_ZERO;
  const float rt1 = m->random_transProb[1];
  /* CPNP/ProbabilisticModel.h:310-313 */
  if (flag)
    for (int k = 0; k < 5; k++) B[(size_t)5 * ((size_t)(L1 + 1) * W - 1) + k] = m->initialDistribution[k];
  /* CPNP/ProbabilisticModel.h:334-392 */
  for (int i = L1; i >= 0; i--) {
    unsigned char c1 = (i == L1) ? '~' : (unsigned char)s1[i + 1];
    for (int j = L2; j >= 0; j--) {
      unsigned char c2 = (j == L2) ? '~' : (unsigned char)s2[j + 1];
      float *ij = B + (size_t)S * ((size_t)i * W + j);
      if (!flag) ij[0] = LOG_ONE;
      if (i < L1 && j < L2) {
        const float *i1j1 = ij + S * (W + 1);
        if (flag) {
          const float ProbXY = i1j1[0] + m->matchProb[c1][c2];
          for (int k = 0; k < 5; k++) LOG_PLUS_EQUALS(ij[k], ProbXY + m->transProb[k][0]);
        } else {
          const float ProbXY =
              i1j1[0] + m->matchProb[c1][c2] - m->insProb[c1][0] - m->insProb[c2][0];
          for (int k = 0; k < 3; k++)
            LOG_PLUS_EQUALS(ij[k], ProbXY + m->local_transProb[k][0] - 2 * rt1);
        }
      }
      if (i < L1) {
        const float *i1j = ij + S * W;
        if (flag) {
          for (int k = 0; k < 2; k++) {
            LOG_PLUS_EQUALS(ij[0], i1j[2 * k + 1] + m->insProb[c1][k] + m->transProb[0][2 * k + 1]);
            LOG_PLUS_EQUALS(ij[2 * k + 1],
                            i1j[2 * k + 1] + m->insProb[c1][k] + m->transProb[2 * k + 1][2 * k + 1]);
          }
        } else {
          LOG_PLUS_EQUALS(ij[0], i1j[1] + m->local_transProb[0][1] - rt1);
          LOG_PLUS_EQUALS(ij[1], i1j[1] + m->local_transProb[1][1] - rt1);
        }
      }
      if (j < L2) {
        const float *ij1 = ij + S;
        if (flag) {
          for (int k = 0; k < 2; k++) {
            LOG_PLUS_EQUALS(ij[0], ij1[2 * k + 2] + m->insProb[c2][k] + m->transProb[0][2 * k + 2]);
            LOG_PLUS_EQUALS(ij[2 * k + 2],
                            ij1[2 * k + 2] + m->insProb[c2][k] + m->transProb[2 * k + 2][2 * k + 2]);
          }
        } else {
          LOG_PLUS_EQUALS(ij[0], ij1[2] + m->local_transProb[0][2] - rt1);
          LOG_PLUS_EQUALS(ij[2], ij1[2] + m->local_transProb[2][2] - rt1);
        }
      }
    }
  }
}

/* CPNP/ProbabilisticModel.h:405-454 */
float orc_total(const orc_model *m, const char *s1, int L1, const char *s2, int L2,
                const float *F, const float *B, int flag) {
  float tf = LOG_ZERO, tb = LOG_ZERO;
  const int W = L2 + 1;
  if (flag) {
    size_t last = (size_t)5 * ((size_t)(L1 + 1) * W - 1);
    for (int k = 0; k < 5; k++) LOG_PLUS_EQUALS(tf, F[last + k] + B[last + k]);
    size_t c11 = (size_t)5 * (W + 1), c10 = (size_t)5 * W, c01 = 5;
    tb = F[c11] + B[c11];
    for (int k = 0; k < 2; k++) {
      LOG_PLUS_EQUALS(tb, F[c10 + 2 * k + 1] + B[c10 + 2 * k + 1]);
      LOG_PLUS_EQUALS(tb, F[c01 + 2 * k + 2] + B[c01 + 2 * k + 2]);
    }
  } else {
    const float rt1 = m->random_transProb[1];
    size_t ij = 0;
    for (int i = 0; i <= L1; i++) {
      unsigned char c1 = (i == 0) ? '~' : (unsigned char)s1[i];
      for (int j = 0; j <= L2; j++) {
        unsigned char c2 = (j == 0) ? '~' : (unsigned char)s2[j];
        if (i > 0 && j > 0) {
          LOG_PLUS_EQUALS(tf, F[ij]);
          LOG_PLUS_EQUALS(tb, B[ij] + m->matchProb[c1][c2] - m->insProb[c1][0] -
                                  m->insProb[c2][0] - 2 * rt1);
        }
        ij += 3;
      }
    }
  }
  return (tf + tb) / 2;
}

/* CPNP/ProbabilisticModel.h:464-493 */
void orc_posterior(const orc_model *m, const char *s1, int L1, const char *s2, int L2,
                   const float *F, const float *B, int flag, float *P) {
  const int S = flag ? 5 : 3;
  float T = orc_total(m, s1, L1, s2, L2, F, B, flag);
  size_t n = (size_t)(L1 + 1) * (L2 + 1), ij = 0;
  for (size_t c = 0; c < n; c++, ij += S) {
    float v = F[ij] + B[ij] - T;
    P[c] = EXP(v < LOG_ONE ? v : LOG_ONE); /* std::min(LOG_ONE, v) */
  }
  P[0] = 0;
}

/* ------------------------------------------------------ partition function */

/* partf (CPNP/MSAPartProbs.cpp:400-660), low-memory branch, endgaps = 1.
 * seqA = sequences[0] (len0), seqB = sequences[1] (len1), 0-based strings.
 * Returns Zm[(len1+1)*(len0+1)] with Zm[0] = total. NULL on overflow. */
static long double *pf_forward(const char *seqA, int len0, const char *seqB, int len1,
                               const double sm[26][26], const int si[26], double d, double e,
                               double endgapopen, double endgapextend) {
  const int W = len0 + 1;
  long double *Zm = calloc((size_t)(len1 + 1) * W, sizeof(long double));
  long double *Ze0 = calloc(W, sizeof(long double)), *Ze1 = calloc(W, sizeof(long double));
  long double *Zf0 = calloc(W, sizeof(long double)), *Zf1 = calloc(W, sizeof(long double));
  long double zz = 0;
  int bad = 0;
  Zm[0] = 1.00;
  Zf0[0] = Ze0[0] = 0;
  Zf1[0] = Zm[0] * endgapopen;
  Ze0[1] = Zm[0] * endgapopen;
  for (int j = 2; j <= len0; j++) Ze0[j] = Ze0[j - 1] * endgapextend;
  for (int i = 1; i <= len1 && !bad; i++) {
    for (int j = 1; j <= len0; j++) {
      int Si = si[seqB[i - 1] - 'A'];
      int Tj = si[seqA[j - 1] - 'A'];
      double score = sm[Si][Tj];
      double open0 = d, extend0 = e, open1 = d, extend1 = e;
      if (i == len1) { open0 = endgapopen; extend0 = endgapextend; }
      if (j == len0) { open1 = endgapopen; extend1 = endgapextend; }
      Ze1[j] = Zm[(size_t)i * W + j - 1] * open0 + Ze1[j - 1] * extend0;
      if (Ze1[j] >= HUGE_VALL) { bad = 1; break; }
      Zf1[j] = Zm[(size_t)(i - 1) * W + j] * open1 + Zf0[j] * extend1;
      if (Zf1[j] >= HUGE_VALL) { bad = 1; break; }
      Zm[(size_t)i * W + j] = (Zm[(size_t)(i - 1) * W + j - 1] + Ze0[j - 1] + Zf0[j - 1]) * score;
      if (Zm[(size_t)i * W + j] >= HUGE_VALL) { bad = 1; break; }
      zz = Zm[(size_t)i * W + j] + Ze1[j] + Zf1[j];
    }
    for (int t = 0; t <= len0; t++) {
      Ze0[t] = Ze1[t]; Ze1[t] = 0;
      Zf0[t] = Zf1[t]; Zf1[t] = 0;
    }
    Zf1[0] = 1;
  }
  Zm[0] = zz;
  free(Ze0); free(Ze1); free(Zf0); free(Zf1);
  if (bad) { free(Zm); return NULL; }
  return Zm;
}

/* revers_partf (CPNP/MSAPartProbs.cpp:78-394), low-memory branch, endgaps = 1.
 * Writes post[(j+1)*(len1+1)+(i+1)]. */
static void pf_reverse(const char *seqA, int len0, const char *seqB, int len1,
                       const double sm[26][26], const int si[26], const long double *Zfm,
                       double d, double e, double endgapopen, double endgapextend, float *post) {
  const int W = len0 + 1;
  long double *Zm0 = calloc(W, sizeof(long double)), *Zm1 = calloc(W, sizeof(long double));
  long double *Ze0 = calloc(W, sizeof(long double)), *Ze1 = calloc(W, sizeof(long double));
  long double *Zf0 = calloc(W, sizeof(long double)), *Zf1 = calloc(W, sizeof(long double));
  for (size_t k = 0; k < (size_t)(len0 + 1) * (len1 + 1); k++) post[k] = 0;
  Zm1[len0] = 1;
  Ze0[len0] = Zf0[len0] = 0;
  Zf1[len0] = Zm1[len0] * endgapopen;
  if (len0 >= 1) Ze0[len0 - 1] = Zm1[len0] * endgapopen;
  for (int j = len0 - 2; j >= 0; j--) Ze0[j] = Ze0[j + 1] * endgapextend;
  for (int i = len1 - 1; i >= 0; i--) {
    for (int j = len0 - 1; j >= 0; j--) {
      int Si = si[seqB[i] - 'A'];
      int Tj = si[seqA[j] - 'A'];
      double scorez = sm[Si][Tj];
      double open0 = d, extend0 = e, open1 = d, extend1 = e;
      if (i == 0) { open0 = endgapopen; extend0 = endgapextend; }
      if (j == 0) { open1 = endgapopen; extend1 = endgapextend; }
      Zf1[j] = Zm1[j] * open1 + Zf0[j] * extend1;
      Ze1[j] = Zm0[j + 1] * open0 + Ze1[j + 1] * extend0;
      Zm0[j] = (Zm1[j + 1] + Zf0[j + 1] + Ze0[j + 1]) * scorez;
      long double tempvar = Zfm[(size_t)(i + 1) * W + (j + 1)] * Zm0[j];
      tempvar /= (scorez * Zfm[0]);
      post[(size_t)(j + 1) * (len1 + 1) + (i + 1)] = (float)tempvar;
    }
    for (int t = 0; t <= len0; t++) {
      Ze0[t] = Ze1[t]; Ze1[t] = 0;
      Zf0[t] = Zf1[t]; Zf1[t] = 0;
      Zm1[t] = Zm0[t]; Zm0[t] = 0;
    }
    Zf0[len0] = 1;
  }
  post[0] = 0;
  free(Zm0); free(Zm1); free(Ze0); free(Ze1); free(Zf0); free(Zf1);
}

/* ComputePostProbs (CPNP/MSAPartProbs.cpp:665-727): sequences[0] = seq1. */
int orc_pf_posterior(const char *s1, int L1, const char *s2, int L2, float *post) {
  static double sm[26][26];
  static int si[26];
  static int init = 0;
  if (!init) {
#pragma omp critical(orc_pf_init)
    {
      if (!init) { orc_pf_tables(sm, si); init = 1; }
    }
  }
  double beta = (float)(1.0 / 5.0f);
  double gap_open = -22, gap_ext = -1;
  double termgapopen = exp(beta * 0.0), termgapextend = exp(beta * 0.0);
  gap_open = exp(beta * gap_open);
  gap_ext = exp(beta * gap_ext);
  const char *A = s1 + 1, *B = s2 + 1; /* 0-based GetString() */
  long double *Zfm = pf_forward(A, L1, B, L2, sm, si, gap_open, gap_ext, termgapopen, termgapextend);
  if (!Zfm) return 1;
  pf_reverse(A, L1, B, L2, sm, si, Zfm, gap_open, gap_ext, termgapopen, termgapextend, post);
  free(Zfm);
  return 0;
}

/* ----------------------------------------------------- merge / MEA / CSR */

int orc_pair_posterior(const orc_model *m, const char *s1, int L1, const char *s2, int L2,
                       int pid, float *post) {
  const int npdo = pid & ORC_NPDO;  /* ArrangePosteriorProbs' merge order (CPNP/MSA.cpp:1699-1708) */
  pid &= ~ORC_NPDO;
  size_t cells = (size_t)(L1 + 1) * (L2 + 1);
  if (pid >= 3) return orc_pf_posterior(s1, L1, s2, L2, post);
  float *F = malloc(sizeof(float) * 5 * cells), *B = malloc(sizeof(float) * 5 * cells);
  if (pid == 2) {
    orc_forward(m, s1, L1, s2, L2, 0, F);
    orc_backward(m, s1, L1, s2, L2, 0, B);
    orc_posterior(m, s1, L1, s2, L2, F, B, 0, post);
    free(F); free(B);
    return 0;
  }
  float *p5 = malloc(sizeof(float) * cells), *pg = malloc(sizeof(float) * cells);
  orc_forward(m, s1, L1, s2, L2, 1, F);
  orc_backward(m, s1, L1, s2, L2, 1, B);
  orc_posterior(m, s1, L1, s2, L2, F, B, 1, p5);
  int rc = orc_pf_posterior(s1, L1, s2, L2, pg);
  orc_forward(m, s1, L1, s2, L2, 0, F);
  orc_backward(m, s1, L1, s2, L2, 0, B);
  orc_posterior(m, s1, L1, s2, L2, F, B, 0, post);
  /* CPNP/MSA.cpp:992-1007 (pdoAlign: double affine, global, local);
   * CPNP/MSA.cpp:1699-1708 (ArrangePosteriorProbs: global, local, double affine) */
  for (size_t c = 0; c < cells; c++) {
    float v1 = p5[c], v2 = pg[c], v3 = post[c];
    post[c] = npdo ? sqrtf((v2 * v2 + v3 * v3 + v1 * v1) / 3) : sqrtf((v1 * v1 + v2 * v2 + v3 * v3) / 3);
  }
  free(F); free(B); free(p5); free(pg);
  return rc;
}

float orc_mea(int L1, int L2, const float *post, char *path, int *pathlen) {
  /* CPNP/ProbabilisticModel.h:804-864; ChooseBestOfThree ScoreType.h:347-366 */
  const int W = L2 + 1;
  float *oldRow = malloc(sizeof(float) * W), *newRow = malloc(sizeof(float) * W);
  char *tb = path ? malloc((size_t)(L1 + 1) * W) : NULL;
  for (int j = 0; j <= L2; j++) {
    oldRow[j] = 0;
    if (tb) tb[j] = 'L';
  }
  const float *pp = post + W;
  for (int i = 1; i <= L1; i++) {
    newRow[0] = 0;
    pp++;
    if (tb) tb[(size_t)i * W] = 'U';
    for (int j = 1; j <= L2; j++) {
      float x1 = *(pp++) + oldRow[j - 1], x2 = newRow[j - 1], x3 = oldRow[j];
      char b;
      float x;
      if (x1 >= x2) {
        if (x1 >= x3) { x = x1; b = 'D'; } else { x = x3; b = 'U'; }
      } else if (x2 >= x3) { x = x2; b = 'L'; } else { x = x3; b = 'U'; }
      newRow[j] = x;
      if (tb) tb[(size_t)i * W + j] = b;
    }
    float *t = oldRow; oldRow = newRow; newRow = t;
  }
  float total = oldRow[L2];
  if (tb) {
    int r = L1, c = L2, n = 0;
    while (r != 0 || c != 0) {
      char ch = tb[(size_t)r * W + c];
      if (ch == 'L') { c--; path[n++] = 'Y'; }
      else if (ch == 'U') { r--; path[n++] = 'X'; }
      else { c--; r--; path[n++] = 'B'; }
    }
    for (int a = 0, z = n - 1; a < z; a++, z--) { char t = path[a]; path[a] = path[z]; path[z] = t; }
    if (pathlen) *pathlen = n;
    free(tb);
  }
  free(oldRow); free(newRow);
  return total;
}

int64_t orc_sparsify(int L1, int L2, const float *post, int32_t *rowptr, int32_t *cols,
                     float *vals) {
  const int W = L2 + 1;
  int64_t n = 0;
  rowptr[0] = 0;
  rowptr[1] = 0;
  for (int i = 1; i <= L1; i++) {
    const float *row = post + (size_t)i * W;
    for (int j = 1; j <= L2; j++) {
      if (row[j] >= POSTERIOR_CUTOFF) {
        if (cols) { cols[n] = j; vals[n] = row[j]; }
        n++;
      }
    }
    rowptr[i + 1] = (int32_t)n;
  }
  return n;
}

/* ------------------------------------------------------------ relaxation */

typedef struct {
  int L1, L2;
  const int32_t *rp; /* L1+2 entries */
  const int32_t *cols;
  const float *vals;
} csr_view;

/* MSA::Relax (CPNP/MSA.cpp:1290-1322): XZ rows x, ZY rows z. */
/* w: QuickProbs' weight (ConsistencyStage::relax, QP/.../ConsistencyStage.cpp:
 * 264-292: weight * XZ * ZY); 1 for C_P_NP_Aln, where (1 * a) * b == a * b. */
static void relax_xz_zy(csr_view xz, csr_view zy, float *post, int Wy, float w) {
  for (int i = 1; i <= xz.L1; i++) {
    float *base = post + (size_t)i * Wy;
    for (int a = xz.rp[i]; a < xz.rp[i + 1]; a++) {
      int z = xz.cols[a];
      float v = w * xz.vals[a];
      for (int b = zy.rp[z]; b < zy.rp[z + 1]; b++) base[zy.cols[b]] += v * zy.vals[b];
    }
  }
}

/* MSA::Relax1 (CPNP/MSA.cpp:1331-1360): ZX rows z, ZY rows z. */
static void relax_zx_zy(csr_view zx, csr_view zy, float *post, int Wy, float w) {
  for (int k = 1; k <= zx.L1; k++) {
    for (int a = zx.rp[k]; a < zx.rp[k + 1]; a++) {
      float v = w * zx.vals[a];
      float *base = post + (size_t)zx.cols[a] * Wy;
      for (int b = zy.rp[k]; b < zy.rp[k + 1]; b++) base[zy.cols[b]] += v * zy.vals[b];
    }
  }
}

/* SparseMatrix::ComputeTranspose (CPNP/SparseMatrix.h:205-248): rows of the
 * result are the columns of s; entries within a row keep ascending source row. */
static void transpose(csr_view s, int32_t *rp, int32_t *cur, int32_t *cols, float *vals) {
  const int R = s.L2;
  for (int r = 0; r <= R + 1; r++) rp[r] = 0;
  const int nnz = s.rp[s.L1 + 1];
  for (int a = 0; a < nnz; a++) rp[s.cols[a] + 1]++;
  for (int r = 1; r <= R + 1; r++) rp[r] += rp[r - 1];
  for (int r = 0; r <= R; r++) cur[r] = rp[r];
  for (int i = 1; i <= s.L1; i++)
    for (int a = s.rp[i]; a < s.rp[i + 1]; a++) {
      int p = cur[s.cols[a]]++;
      cols[p] = i;
      vals[p] = s.vals[a];
    }
}

static int pair_index(int N, int a, int b) { /* a < b, row-major */
  return a * N - a * (a + 1) / 2 + (b - a - 1);
}

/* qp: QuickProbs' ConsistencyStage::doRelaxation (QP/Alignment/Multiple/
 * ConsistencyStage.cpp:133-258) with the Deterministic selectivity filter
 * (qp_accept below; without seldist every z is accepted): P' = (P + sum_z
 * w_z / W_xy P_xz P_zy) / (1 + sum_z w_z / W_xy) over the accepted z,
 * W_xy = (1 + (s - 1) A_xy / a)(w_x + w_y), re-sparsified at `cutoff` into
 * 16-bit fixed point (values out as q / 65535). */
static int qp_accept(const float *seldist, float a, int N, int i, int j, int k);
static int64_t relax_impl(int qp, const float *weights, float selfweight, float cutoff,
                          const float *seldist, float selectivity,
                          int N, const int32_t *lens, const int64_t *row_off, const int64_t *ent_off,
                          const int32_t *in_rp, const int32_t *in_cols, const float *in_vals,
                          int32_t *out_rp, int64_t *out_ent_off, int32_t *out_cols, float *out_vals,
                          int64_t max_out, const uint8_t *select);

int64_t orc_relax(int N, const int32_t *lens, const int64_t *row_off, const int64_t *ent_off,
                  const int32_t *in_rp, const int32_t *in_cols, const float *in_vals,
                  int32_t *out_rp, int64_t *out_ent_off, int32_t *out_cols, float *out_vals,
                  int64_t max_out) {
  return relax_impl(0, NULL, 0, 0, NULL, 200.0f, N, lens, row_off, ent_off, in_rp, in_cols, in_vals, out_rp, out_ent_off,
                    out_cols, out_vals, max_out, NULL);
}

int64_t orc_relax_subset(int N, const int32_t *lens, const int64_t *row_off, const int64_t *ent_off,
                         const int32_t *in_rp, const int32_t *in_cols, const float *in_vals,
                         int32_t *out_rp, int64_t *out_ent_off, int32_t *out_cols, float *out_vals,
                         int64_t max_out, const uint8_t *select) {
  return relax_impl(0, NULL, 0, 0, NULL, 200.0f, N, lens, row_off, ent_off, in_rp, in_cols, in_vals, out_rp, out_ent_off,
                    out_cols, out_vals, max_out, select);
}

int64_t orc_qp_relax(const float *weights, float selfweight, float cutoff,
                     int N, const int32_t *lens, const int64_t *row_off, const int64_t *ent_off,
                     const int32_t *in_rp, const int32_t *in_cols, const float *in_vals,
                     int32_t *out_rp, int64_t *out_ent_off, int32_t *out_cols, float *out_vals,
                     int64_t max_out) {
  return relax_impl(1, weights, selfweight, cutoff, NULL, 200.0f, N, lens, row_off, ent_off, in_rp, in_cols, in_vals,
                    out_rp, out_ent_off, out_cols, out_vals, max_out, NULL);
}

int64_t orc_qp_relax_sel(const float *weights, float selfweight, float cutoff, const float *seldist,
                         float selectivity, int N, const int32_t *lens, const int64_t *row_off,
                         const int64_t *ent_off, const int32_t *in_rp, const int32_t *in_cols,
                         const float *in_vals, int32_t *out_rp, int64_t *out_ent_off, int32_t *out_cols,
                         float *out_vals, int64_t max_out) {
  return relax_impl(1, weights, selfweight, cutoff, seldist, selectivity, N, lens, row_off, ent_off, in_rp, in_cols,
                    in_vals, out_rp, out_ent_off, out_cols, out_vals, max_out, NULL);
}

/* The Deterministic selectivity filter (ConsistencyStage.cpp:35-47, 171-186):
 * x = max(D[i][k], D[j][k]); filter = x <= a ? 2 : 0; the Park-Miller draw
 * seed * RND_MAX_INV lies in [0, 1.0026], so z is accepted iff x <= a (a draw
 * of exactly 0 with filter 0 gives w = 0, not < 0: rejected as well). */
static int qp_accept(const float *seldist, float a, int N, int i, int j, int k) {
  if (!seldist) return 1;
  const float di = seldist[(size_t)i * N + k], dj = seldist[(size_t)j * N + k];
  return (di > dj ? di : dj) <= a;
}

static int64_t qp_sparsify_vals(int L1, int L2, const float *post, float cutoff, int32_t *rowptr, int32_t *cols,
                                float *vals) {
  const int W = L2 + 1;
  int64_t n = 0;
  rowptr[0] = rowptr[1] = 0;
  for (int i = 1; i <= L1; i++) {
    for (int j = 1; j <= L2; j++) {
      const float v = post[(size_t)i * W + j];
      if (v >= cutoff) {
        if (cols) cols[n] = j;
        if (vals) vals[n] = (float)(uint16_t)(v * 65535.0f) / 65535.0f;
        n++;
      }
    }
    rowptr[i + 1] = (int32_t)n;
  }
  return n;
}

static int64_t relax_impl(int qp, const float *weights, float selfweight, float cutoff,
                          const float *seldist, float selectivity,
                          int N, const int32_t *lens, const int64_t *row_off, const int64_t *ent_off,
                          const int32_t *in_rp, const int32_t *in_cols, const float *in_vals,
                          int32_t *out_rp, int64_t *out_ent_off, int32_t *out_cols, float *out_vals,
                          int64_t max_out, const uint8_t *select) {
  const int P = N * (N - 1) / 2;
  int64_t *cnt = calloc(P > 0 ? P : 1, sizeof(int64_t));
  float **dense = calloc(P > 0 ? P : 1, sizeof(float *));
#define VIEW(a, b) ((csr_view){lens[a], lens[b], in_rp + row_off[pair_index(N, a, b)], \
                               in_cols + ent_off[pair_index(N, a, b)],                  \
                               in_vals + ent_off[pair_index(N, a, b)]})
#pragma omp parallel for schedule(dynamic)
  for (int p = 0; p < P; p++) {
    int i = 0, q = p;
    while (q >= N - 1 - i) { q -= N - 1 - i; i++; }
    int j = i + 1 + q;
    const int L1 = lens[i], L2 = lens[j], W = L2 + 1;
    if (select && !select[p]) {  /* not requested: empty output rows */
      int32_t *rp = out_rp + row_off[p];
      for (int r = 0; r <= L1 + 1; r++) rp[r] = 0;
      cnt[p] = 0;
      dense[p] = NULL;
      continue;
    }
    float *post = calloc((size_t)(L1 + 1) * W, sizeof(float));
    csr_view xy = VIEW(i, j);
    for (int x = 1; x <= L1; x++)
      for (int a = xy.rp[x]; a < xy.rp[x + 1]; a++) post[(size_t)x * W + xy.cols[a]] = xy.vals[a];
    if (!qp)  /* z = x and z = y (CPNP/MSA.cpp:1211-1213) */
      for (size_t k = 0; k < (size_t)(L1 + 1) * W; k++) post[k] += post[k];
    float wxy = 0, sumW = 1.0f;
    if (qp) {  /* ConsistencyStage.cpp:165-203 */
      int accepted = 0;
      for (int k = 0; k < N; k++)
        if (k != i && k != j && qp_accept(seldist, selectivity, N, i, j, k)) accepted++;
      wxy = 1.0f + (selfweight - 1.0f) * (float)accepted / selectivity;
      wxy *= weights[i] + weights[j];
    }
    int maxL = 0;
    for (int k = 0; k < N; k++) if (lens[k] > maxL) maxL = lens[k];
    int32_t *trp = malloc(sizeof(int32_t) * (maxL + 2));
    int32_t *tcur = malloc(sizeof(int32_t) * (maxL + 2));
    int32_t *tcols = NULL;
    float *tvals = NULL;
    int64_t tcap = 0;
    for (int k = 0; k < N; k++) {
      if (k == i || k == j) continue;
      if (qp && !qp_accept(seldist, selectivity, N, i, j, k)) continue;
      float w = 1.0f;
      if (qp) {
        w = weights[k] / wxy;
        sumW += w;
      }
      if (k < i) {
        relax_zx_zy(VIEW(k, i), VIEW(k, j), post, W, w);
      } else if (k < j) {
        relax_xz_zy(VIEW(i, k), VIEW(k, j), post, W, w);
      } else {
        csr_view jk = VIEW(j, k);
        int64_t nnz = jk.rp[jk.L1 + 1];
        if (nnz > tcap) {
          tcap = nnz;
          tcols = realloc(tcols, sizeof(int32_t) * (tcap ? tcap : 1));
          tvals = realloc(tvals, sizeof(float) * (tcap ? tcap : 1));
        }
        transpose(jk, trp, tcur, tcols, tvals);
        csr_view t = {jk.L2, jk.L1, trp, tcols, tvals};
        relax_xz_zy(VIEW(i, k), t, post, W, w);
      }
    }
    free(trp); free(tcur); free(tcols); free(tvals);
    for (size_t k = 0; k < (size_t)(L1 + 1) * W; k++) post[k] /= qp ? sumW : (float)N;
    /* mask (CPNP/MSA.cpp:1237-1261) */
    for (int y = 0; y <= L2; y++) post[y] = 0;
    for (int x = 1; x <= L1; x++) {
      float *base = post + (size_t)x * W;
      int curr = 0;
      for (int a = xy.rp[x]; a < xy.rp[x + 1]; a++) {
        while (curr < xy.cols[a]) base[curr++] = 0;
        curr++;
      }
      while (curr <= L2) base[curr++] = 0;
    }
    int32_t *rp = out_rp + row_off[p];
    cnt[p] = qp ? qp_sparsify_vals(L1, L2, post, cutoff, rp, NULL, NULL) : orc_sparsify(L1, L2, post, rp, NULL, NULL);
    dense[p] = post;
  }
#undef VIEW
  int64_t total = 0;
  for (int p = 0; p < P; p++) { out_ent_off[p] = total; total += cnt[p]; }
  if (total > max_out) {
    for (int p = 0; p < P; p++) free(dense[p]);
    free(dense); free(cnt);
    return -1;
  }
#pragma omp parallel for schedule(dynamic)
  for (int p = 0; p < P; p++) {
    int i = 0, q = p;
    while (q >= N - 1 - i) { q -= N - 1 - i; i++; }
    int j = i + 1 + q;
    if (!dense[p]) continue;
    if (qp)
      qp_sparsify_vals(lens[i], lens[j], dense[p], cutoff, out_rp + row_off[p], out_cols + out_ent_off[p],
                       out_vals + out_ent_off[p]);
    else
      orc_sparsify(lens[i], lens[j], dense[p], out_rp + row_off[p], out_cols + out_ent_off[p],
                   out_vals + out_ent_off[p]);
    free(dense[p]);
  }
  free(dense); free(cnt);
  return total;
}

/* ----------------------------------------------------- Viterbi + family */

float orc_viterbi(const orc_model *m, const char *s1, int L1, const char *s2, int L2,
                  char *path, int *pathlen) {
  /* CPNP/ProbabilisticModel.h:1043-1170 */
  const int W = L2 + 1;
  size_t n = (size_t)3 * (L1 + 1) * W;
  float *V = malloc(sizeof(float) * n);
  int *T = malloc(sizeof(int) * n);
  for (size_t k = 0; k < n; k++) { V[k] = LOG_ZERO; T[k] = -1; }
  V[0] = LOG(0.6080327034f);
  V[1] = LOG(0.1959836632f);
  V[2] = LOG(0.1959836632f);
  for (int i = 0; i <= L1; i++) {
    unsigned char c1 = (i == 0) ? '~' : (unsigned char)s1[i];
    for (int j = 0; j <= L2; j++) {
      unsigned char c2 = (j == 0) ? '~' : (unsigned char)s2[j];
      size_t ij = (size_t)3 * ((size_t)i * W + j);
      if (i > 0 && j > 0) {
        size_t i1j1 = ij - 3 * (W + 1);
        for (int k = 0; k < 3; k++) {
          float nv = V[k + i1j1] + m->local_transProb[k][0] + m->matchProb[c1][c2];
          if (V[ij] < nv) { V[ij] = nv; T[ij] = k; }
        }
      }
      if (i > 0) {
        size_t i1j = ij - 3 * W;
        float fm = m->insProb[c1][0] + V[i1j] + m->local_transProb[0][1];
        float fi = m->insProb[c1][0] + V[1 + i1j] + m->local_transProb[1][1];
        if (fm >= fi) { V[1 + ij] = fm; T[1 + ij] = 0; } else { V[1 + ij] = fi; T[1 + ij] = 1; }
      }
      if (j > 0) {
        size_t ij1 = ij - 3;
        float fm = m->insProb[c2][0] + V[ij1] + m->local_transProb[0][2];
        float fi = m->insProb[c2][0] + V[2 + ij1] + m->local_transProb[2][2];
        if (fm >= fi) { V[2 + ij] = fm; T[2 + ij] = 0; } else { V[2 + ij] = fi; T[2 + ij] = 2; }
      }
    }
  }
  float best = LOG_ZERO;
  int state = -1;
  V[0] = LOG(0.6080327034f);
  V[1] = LOG(0.1959836632f);
  V[2] = LOG(0.1959836632f);
  size_t last = (size_t)3 * ((size_t)(L1 + 1) * W - 1);
  for (int k = 0; k < 3; k++) {
    float tp = V[k + last] + V[k];
    if (best < tp) { best = tp; state = k; }
  }
  int r = L1, c = L2, len = 0;
  while (r != 0 || c != 0) {
    int ns = T[state + (size_t)3 * ((size_t)r * W + c)];
    if (state == 0) { c--; r--; if (path) path[len] = 'B'; }
    else if (state % 2 == 1) { r--; if (path) path[len] = 'X'; }
    else { c--; if (path) path[len] = 'Y'; }
    len++;
    state = ns;
  }
  if (path)
    for (int a = 0, z = len - 1; a < z; a++, z--) { char t = path[a]; path[a] = path[z]; path[z] = t; }
  if (pathlen) *pathlen = len;
  free(V); free(T);
  return best;
}

int orc_model_adjustment(const orc_model *m, int N, const char *const *seqs,
                         const int32_t *lens, float *identity_out, float *delta_out) {
  /* CPNP/MSA.cpp:775-882, with the per-pair identities summed serially in
   * pair order (the reference's OpenMP `identity +=` is unsynchronised). */
  const int P = N * (N - 1) / 2;
  float *pids = malloc(sizeof(float) * (P > 0 ? P : 1));
#pragma omp parallel for schedule(dynamic)
  for (int p = 0; p < P; p++) {
    int a = 0, q = p;
    while (q >= N - 1 - a) { q -= N - 1 - a; a++; }
    int b = a + 1 + q;
    char *path = malloc(lens[a] + lens[b] + 2);
    int len = 0;
    orc_viterbi(m, seqs[a], lens[a], seqs[b], lens[b], path, &len);
    float match = 0;
    int i = 1, j = 1;
    for (int k = 0; k < len; k++) {
      if (path[k] == 'B') {
        if (seqs[a][i++] == seqs[b][j++]) match += 1;
      } else if (path[k] == 'X') i++;
      else j++;
    }
    pids[p] = match / len;
    free(path);
  }
  float identity = 0;
  for (int p = 0; p < P; p++) identity += pids[p];
  identity /= P;
  float variance = 0;
  for (int k = 0; k < P; k++) variance += (pids[k] - identity) * (pids[k] - identity);
  variance /= P;
  variance = sqrtf(variance);
  free(pids);
  if (identity_out) *identity_out = identity;
  if (delta_out) *delta_out = orc_delta_for_identity(identity, mlp_init_distrib[2]);
  int vm = (variance > 0.115) ? 10 : 0;
  if (identity <= 0.18) return vm + 0;
  if (identity <= 0.25) return vm + 1;
  if (identity <= 0.4) return vm + 2;
  if (identity <= 0.7) return vm + 3;
  return vm + 4;
}

int64_t orc_pair_loop(const orc_model *m, int N, const char *const *seqs, const int32_t *lens,
                      int pid, int64_t max_pairs, int threads, float *dist_out,
                      int64_t *nnz_out) {
  int64_t P = (int64_t)N * (N - 1) / 2;
  if (max_pairs >= 0 && max_pairs < P) P = max_pairs;
  int64_t total = 0;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel for schedule(dynamic) reduction(+ : total)
  for (int64_t p = 0; p < P; p++) {
    int a = 0;
    int64_t q = p;
    while (q >= N - 1 - a) { q -= N - 1 - a; a++; }
    int b = a + 1 + (int)q;
    int L1 = lens[a], L2 = lens[b];
    float *post = malloc(sizeof(float) * (size_t)(L1 + 1) * (L2 + 1));
    orc_pair_posterior(m, seqs[a], L1, seqs[b], L2, pid, post);
    float score = orc_mea(L1, L2, post, NULL, NULL);
    if (dist_out) dist_out[p] = 1.0f - score / (L1 < L2 ? L1 : L2);
    int32_t *rp = malloc(sizeof(int32_t) * (L1 + 2));
    int64_t nnz = orc_sparsify(L1, L2, post, rp, NULL, NULL);
    if (nnz_out) nnz_out[p] = nnz;
    total += nnz;
    free(rp);
    free(post);
  }
  return total;
}

/* ------------------------------------------------------------ QuickProbs
 * QuickProbs' posterior stage (QP/Alignment/Multiple/PosteriorStage.cpp:
 * 123-196): the 5-state pair-HMM above with the default tables (QuickProbs'
 * ProteinHmm5 tables are the same; tools/gen_params.py --qp checks it) and
 * its own partition function in double over exp(beta * VTML200)
 * (mlp_params_qp.inc, QP/Alignment/Multiple/PartitionFunction.cpp:71-291,
 * restated below with its two-row buffers).  s1, s2 are '@'-prefixed. */
static double qp_sub(char a, char b) { return mlp_qp_pf_sub[(a - 'A') * 26 + (b - 'A')]; }

void orc_qp_pf_posterior(const char *s1, int L1, const char *s2, int L2, float *post) {
  const int lda = L2 + 1;
  const size_t cells = (size_t)(L1 + 1) * lda;
  const double go = mlp_qp_pf_open, ge = mlp_qp_pf_extend, tgo = 1.0, tge = 1.0;  /* exp(beta * 0) */
  double *Zm = calloc(cells, sizeof(double));
  double *buf = calloc(4 * (size_t)lda, sizeof(double));
  double *Ze = buf, *Zf = buf + 2 * lda, zz = 0;
  /* forward, PartitionFunction.cpp:85-156 */
  Zm[0] = 1.0;
  Zf[0] = Ze[0] = 0;
  Zf[lda + 0] = Zm[0] * tgo;
  Ze[1] = Zm[0] * tgo;
  for (int j = 2; j <= L2; j++) Ze[j] = Ze[j - 1] * tge;
  for (int i = 1; i <= L1; i++) {
    for (int j = 1; j <= L2; j++) {
      const double score = qp_sub(s1[i], s2[j]);
      double open0 = go, extend0 = ge, open1 = go, extend1 = ge;
      if (i == L1) { open0 = tgo; extend0 = tge; }
      if (j == L2) { open1 = tgo; extend1 = tge; }
      Ze[lda + j] = Zm[(size_t)i * lda + j - 1] * open0 + Ze[lda + j - 1] * extend0;
      Zf[lda + j] = Zm[(size_t)(i - 1) * lda + j] * open1 + Zf[j] * extend1;
      Zm[(size_t)i * lda + j] = (Zm[(size_t)(i - 1) * lda + j - 1] + Ze[j - 1] + Zf[j - 1]) * score;
      zz = Zm[(size_t)i * lda + j] + Ze[lda + j] + Zf[lda + j];
    }
    for (int t = 0; t <= L2; t++) {
      Ze[t] = Ze[lda + t]; Ze[lda + t] = 0;
      Zf[t] = Zf[lda + t]; Zf[lda + t] = 0;
    }
    Zf[lda + 0] = 1;
  }
  Zm[0] = zz;
  /* reverse, PartitionFunction.cpp:185-289 */
  double *rb = calloc(6 * (size_t)lda, sizeof(double));
  double *Rm = rb, *Re = rb + 2 * lda, *Rf = rb + 4 * lda;
  for (size_t c = 0; c < cells; c++) post[c] = 0.0f;
  Rm[lda + L2] = 1;
  Re[L2] = Rf[L2] = 0;
  Rf[lda + L2] = Rm[lda + L2] * tgo;
  Re[L2 - 1] = Rm[lda + L2] * tgo;
  for (int j = L2 - 2; j >= 0; j--) Re[j] = Re[j + 1] * tge;
  for (int i = L1 - 1; i >= 0; i--) {
    for (int j = L2 - 1; j >= 0; j--) {
      const double scorez = qp_sub(s1[i + 1], s2[j + 1]);
      double open0 = go, extend0 = ge, open1 = go, extend1 = ge;
      if (i == 0) { open0 = tgo; extend0 = tge; }
      if (j == 0) { open1 = tgo; extend1 = tge; }
      Rf[lda + j] = Rm[lda + j] * open1 + Rf[j] * extend1;
      Re[lda + j] = Rm[j + 1] * open0 + Re[lda + j + 1] * extend0;
      Rm[j] = (Rm[lda + j + 1] + Rf[j + 1] + Re[j + 1]) * scorez;
      double tempvar = Zm[(size_t)(i + 1) * lda + j + 1] * Rm[j];
      tempvar /= (scorez * Zm[0]);
      const float probability = (float)tempvar;
      if (probability <= 1 && probability >= 0.001) post[(size_t)(i + 1) * lda + j + 1] = probability;
    }
    for (int t = 0; t <= L2; t++) {
      Re[t] = Re[lda + t]; Re[lda + t] = 0;
      Rf[t] = Rf[lda + t]; Rf[lda + t] = 0;
      Rm[lda + t] = Rm[t]; Rm[t] = 0;
    }
    Rf[L2] = 1;
  }
  post[0] = 0;
  free(Zm); free(buf); free(rb);
}

/* PosteriorStage::computePairwise + combineMatrices: HMM posterior (post_hmm),
 * partition-function posterior (post_pf), their RMS (post); returns the
 * distance 1 - MEA / min(L1, L2). */
float orc_qp_pair(const orc_model *m, const char *s1, int L1, const char *s2, int L2,
                  float *post_hmm, float *post_pf, float *post) {
  const size_t cells = (size_t)(L1 + 1) * (L2 + 1);
  orc_qp_pf_posterior(s1, L1, s2, L2, post_pf);
  float *F = malloc(sizeof(float) * 5 * cells), *B = malloc(sizeof(float) * 5 * cells);
  orc_forward(m, s1, L1, s2, L2, 1, F);
  orc_backward(m, s1, L1, s2, L2, 1, B);
  orc_posterior(m, s1, L1, s2, L2, F, B, 1, post_hmm);
  free(F); free(B);
  /* combineMatrices, PosteriorStage.cpp:160-196 */
  const int W = L2 + 1;
  float *oldRow = calloc(W, sizeof(float)), *newRow = calloc(W, sizeof(float));
  for (int i = 0; i <= L1; i++) {
    for (int j = 0; j <= L2; j++) {
      const size_t c = (size_t)i * W + j;
      if (i == 0 || j == 0) {
        post[c] = 0;
        newRow[j] = 0;
      } else {
        const float v1 = post_hmm[c], v2 = post_pf[c];
        post[c] = sqrtf((v1 * v1 + v2 * v2) * 0.5f);
        float a = post[c] + oldRow[j - 1], b = newRow[j - 1], d = oldRow[j];
        newRow[j] = a >= b ? (a >= d ? a : d) : (b >= d ? b : d);
      }
    }
    float *t = oldRow; oldRow = newRow; newRow = t;
  }
  const float total = oldRow[L2];
  free(oldRow); free(newRow);
  return 1.0f - total / (float)(L1 < L2 ? L1 : L2);
}

/* FilteredSparseMatrix(L1, L2, post, cutoff) with 16-bit fixed-point values
 * (QP/DataStructures/PackedSparseMatrix.cpp:40-80, SparseEntry.h:31-32).
 * Returns the entry count; cols / q may be NULL to count. */
int64_t orc_qp_sparsify(int L1, int L2, const float *post, int32_t *rowptr, int32_t *cols, uint16_t *q) {
  const int W = L2 + 1;
  int64_t n = 0;
  rowptr[0] = rowptr[1] = 0;
  for (int i = 1; i <= L1; i++) {
    for (int j = 1; j <= L2; j++) {
      const float v = post[(size_t)i * W + j];
      if (v >= mlp_qp_cutoff) {
        if (cols) cols[n] = j;
        if (q) q[n] = (uint16_t)(v * 65535.0f);
        n++;
      }
    }
    rowptr[i + 1] = (int32_t)n;
  }
  return n;
}

/* ------------------------------------------------------------ bulk checkers
 * The pdoAlign pair body (CPNP/MSA.cpp:939-1025: posterior by pid, MEA
 * distance 1 - score/min(L), SparseMatrix at 0.01) for a list of pairs, with
 * the sparse rows returned: rowptr (L_a + 2 per listed pair, pair-local
 * values), ent_off[np + 1], cols/vals with room for max_out entries.
 * Returns the total entries, or -1 when max_out is too small. */
int64_t orc_pairs_csr(const orc_model *m, int N, const char *const *seqs, const int32_t *lens, int pid,
                      const int64_t *pairs, int64_t np, int threads, float *dist_out, float *mea_out,
                      int32_t *rowptr, int64_t *ent_off, int32_t *cols, float *vals, int64_t max_out) {
  (void)N;
  int32_t **pc = calloc(np > 0 ? np : 1, sizeof(int32_t *));
  float **pv = calloc(np > 0 ? np : 1, sizeof(float *));
  int64_t *cnt = calloc(np > 0 ? np : 1, sizeof(int64_t));
  int64_t *roff = calloc(np + 1, sizeof(int64_t));
  for (int64_t k = 0; k < np; k++) {
    int a = 0;
    int64_t q = pairs[k];
    while (q >= N - 1 - a) { q -= N - 1 - a; a++; }
    roff[k + 1] = roff[k] + lens[a] + 2;
  }
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel for schedule(dynamic)
  for (int64_t k = 0; k < np; k++) {
    int a = 0;
    int64_t q = pairs[k];
    while (q >= N - 1 - a) { q -= N - 1 - a; a++; }
    int b = a + 1 + (int)q;
    int L1 = lens[a], L2 = lens[b];
    float *post = malloc(sizeof(float) * (size_t)(L1 + 1) * (L2 + 1));
    orc_pair_posterior(m, seqs[a], L1, seqs[b], L2, pid, post);
    float score;
    if (pid & ORC_NPDO) {  /* distance = score / #B (CPNP/MSA.cpp:1744-1753) */
      char *path = malloc((size_t)L1 + L2 + 1);
      int plen = 0, nb = 0;
      score = orc_mea(L1, L2, post, path, &plen);
      for (int t = 0; t < plen; t++) nb += path[t] == 'B';
      free(path);
      if (dist_out) dist_out[k] = score / nb;
    } else {
      score = orc_mea(L1, L2, post, NULL, NULL);
      if (dist_out) dist_out[k] = 1.0f - score / (L1 < L2 ? L1 : L2);
    }
    if (mea_out) mea_out[k] = score;
    int32_t *rp = rowptr + roff[k];
    int64_t nnz = orc_sparsify(L1, L2, post, rp, NULL, NULL);
    pc[k] = malloc(sizeof(int32_t) * (nnz ? nnz : 1));
    pv[k] = malloc(sizeof(float) * (nnz ? nnz : 1));
    orc_sparsify(L1, L2, post, rp, pc[k], pv[k]);
    cnt[k] = nnz;
    free(post);
  }
  int64_t total = 0;
  for (int64_t k = 0; k < np; k++) { ent_off[k] = total; total += cnt[k]; }
  ent_off[np] = total;
  if (total <= max_out)
    for (int64_t k = 0; k < np; k++) {
      memcpy(cols + ent_off[k], pc[k], sizeof(int32_t) * cnt[k]);
      memcpy(vals + ent_off[k], pv[k], sizeof(float) * cnt[k]);
    }
  for (int64_t k = 0; k < np; k++) { free(pc[k]); free(pv[k]); }
  free(pc); free(pv); free(cnt); free(roff);
  return total <= max_out ? total : -1;
}

/* Compare two sparse sets pair by pair under the parity rule of SURVEY.md
 * section 8c: entries on both sides within rtol * max(|ref|, 1e-6); an entry
 * on one side only is allowed iff its value lies within 10 * rtol of the
 * cutoff; `exact` additionally counts every bit difference.  Pair k has L1[k]
 * rows; its row pointers start at *_roff[k] and its entries at *_eoff[k].
 * stats: {pairs, ref entries, our entries, common, max rel err, flips at the
 * cutoff, violations, exact mismatches (value bits or presence)}. */
void orc_csr_compare(int64_t np, const int32_t *L1, float rtol, float cutoff,
                     const int64_t *r_roff, const int64_t *r_eoff, const int32_t *r_rp,
                     const int32_t *r_cols, const float *r_vals,
                     const int64_t *o_roff, const int64_t *o_eoff, const int32_t *o_rp,
                     const uint16_t *o_cols, const float *o_vals, double *stats) {
  double nref = 0, nours = 0, both = 0, worst = 0, flips = 0, bad = 0, inexact = 0;
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : nref, nours, both, flips, bad, inexact) reduction(max : worst)
  for (int64_t k = 0; k < np; k++) {
    const int32_t *rr = r_rp + r_roff[k], *orow = o_rp + o_roff[k];
    const int32_t *rc = r_cols + r_eoff[k];
    const float *rv = r_vals + r_eoff[k];
    const uint16_t *oc = o_cols + o_eoff[k];
    const float *ov = o_vals + o_eoff[k];
    for (int i = 1; i <= L1[k]; i++) {
      int a = rr[i], ae = rr[i + 1], b = orow[i], be = orow[i + 1];
      nref += ae - a;
      nours += be - b;
      while (a < ae || b < be) {
        const int ca = a < ae ? rc[a] : 1 << 30, cb = b < be ? (int)oc[b] : 1 << 30;
        if (ca == cb) {
          const double r = rv[a], o = ov[b];
          const double den = fabs(r) > 1e-6 ? fabs(r) : 1e-6;
          const double e = fabs(o - r) / den;
          if (e > worst) worst = e;
          if (e > rtol) bad += 1;
          if (rv[a] != ov[b]) inexact += 1;
          both += 1;
          a++, b++;
        } else {
          const double v = ca < cb ? rv[a] : ov[b];
          if (ca < cb) a++; else b++;
          flips += 1;
          inexact += 1;
          if (fabs(v - cutoff) > 10.0 * rtol * cutoff) bad += 1;
        }
      }
    }
  }
  stats[0] = (double)np; stats[1] = nref; stats[2] = nours; stats[3] = both;
  stats[4] = worst; stats[5] = flips; stats[6] = bad; stats[7] = inexact;
}
