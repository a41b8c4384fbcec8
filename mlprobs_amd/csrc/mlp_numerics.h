// mlp_numerics.h -- device-side log-space arithmetic for gfx950.
//
// Bit-faithful to the reference's scalar float sequence (CPNP/ScoreType.h):
// every function below performs exactly the IEEE operations of its reference
// counterpart, in the same order.  The translation unit MUST be compiled with
// -ffp-contract=off (no FMA contraction) and without fast-math; fp32 division
// and sqrt stay correctly rounded (hipcc default).  Branches of the reference
// are expressed as selects so a wave never diverges inside the DP inner loop.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MLP_LOG_ZERO (-2e20f)
#define MLP_LOG_ONE (0.0f)

// LOOKUP: log(1 + e^x) on [0, 7.5], piecewise cubic (CPNP/ScoreType.h:196-216).
// Coefficients are selected, then the cubic is evaluated in the reference's
// Horner order; d outside [0, 7.5) only occurs on lanes whose result is
// discarded by mlp_log_add.
__device__ __forceinline__ float mlp_lookup(float x) {
  const bool p1 = x <= 1.00f, p2 = x <= 2.50f, p3 = x <= 4.50f;
  const float a = p1 ? -0.009350833524763f : p2 ? -0.014532321752540f : p3 ? -0.004605031767994f : -0.000458661602210f;
  const float b = p1 ? 0.130659527668286f : p2 ? 0.139942324101744f : p3 ? 0.063427417320019f : 0.009695946122598f;
  const float c = p1 ? 0.498799810682272f : p2 ? 0.495635523139337f : p3 ? 0.695956496475118f : 0.930734667215156f;
  const float d = p1 ? 0.693203116424741f : p2 ? 0.692140569840976f : p3 ? 0.514272634594009f : 0.168037164329057f;
  return ((a * x + b) * x + c) * x + d;
}

// LOG_ADD (CPNP/ScoreType.h:279-285): exact LOG_ZERO sentinel test and the
// 7.5 underflow cutoff; the result adds LOOKUP(hi - lo) to lo.
__device__ __forceinline__ float mlp_log_add(float x, float y) {
  const bool lt = x < y;
  const float hi = lt ? y : x;
  const float lo = lt ? x : y;
  const float d = hi - lo;
  const float r = mlp_lookup(d) + lo;
  return (lo == MLP_LOG_ZERO || d >= 7.5f) ? hi : r;
}

// max / min of two non-NaN floats as one v_max_f32 / v_min_f32 (fmaxf /
// fminf canonicalise inputs the compiler cannot prove canonical first).
// Only where the operands come from loads or DPP moves: inside LOG_ADD the
// opaque asm costs the scheduler more than the canonicalisation it saves
__device__ __forceinline__ float mlp_max(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float mlp_min(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// LDS-table form of LOOKUP.  The interval is found from
// q = floor(min(d * (2 - 2^-23), 15)): q <= 1 <=> d <= 1, q <= 4 <=> d <= 2.5,
// q <= 8 <=> d <= 4.5 for every float d >= 0 (checked exhaustively on [0, 8);
// the product rounds below the even integer exactly at the three breakpoints),
// so lk[q] (16 float4 rows, filled by mlp_lookup_table) holds the reference's
// coefficients of d's interval.  Three VALU ops (mul, convert, and) instead
// of compare/select chains.
__device__ __forceinline__ void mlp_lookup_table(float4* lk) {
  const float4 k0 = make_float4(-0.009350833524763f, 0.130659527668286f, 0.498799810682272f, 0.693203116424741f);
  const float4 k1 = make_float4(-0.014532321752540f, 0.139942324101744f, 0.495635523139337f, 0.692140569840976f);
  const float4 k2 = make_float4(-0.004605031767994f, 0.063427417320019f, 0.695956496475118f, 0.514272634594009f);
  const float4 k3 = make_float4(-0.000458661602210f, 0.009695946122598f, 0.930734667215156f, 0.168037164329057f);
  for (int q = 0; q < 16; ++q) lk[q] = q < 2 ? k0 : q < 5 ? k1 : q < 9 ? k2 : k3;
}
constexpr int kLookupRows = 16;

// LOG_ADD with LDS coefficients.  max/min replace the reference's compare
// (identical results for non-NaN inputs; for x == y both operands are equal).
// The reference's `lo == LOG_ZERO` test is implied by `d >= 7.5`: if lo is
// LOG_ZERO and d < 7.5 then hi == LOG_ZERO too (float spacing at 2e20 is
// 1.6e13) and LOOKUP(0) + LOG_ZERO rounds back to LOG_ZERO == hi.
__device__ __forceinline__ float mlp_log_add_t(float x, float y, const float4* __restrict__ lk) {
  const float hi = fmaxf(x, y), lo = fminf(x, y);
  const float d = hi - lo;
  // the row's byte offset 16 q directly: fl(d * 16 M) = 16 fl(d * M) (a power
  // of two scales exactly), so floor(.) & 0xf0 = 16 floor(fl(d * M)) for
  // d < 7.5, the row above; for d >= 7.5 any row (the result is hi).  The
  // hardware conversion saturates, so no clamp (the min and the shift of the
  // table index were two half-rate instructions per LOG_ADD: C3 forward
  // 184 -> 180.5, backward 243.7 -> 237, local totals 97-100 -> 83-92 ms a
  // step, profiles/r05o_ab_lookup_byteoff.txt)
  // Round 6: the integer floor(fl(d * 16M)) without the half-rate convert:
  // fma(d, 16M, -0.5) + 1.5 * 2^23 rounds to it in the float's low mantissa
  // bits (a tie, fl(d * 16M) an integer, goes to the even one, which keeps
  // every multiple of 16 in its row), two full-rate instructions for a
  // full-rate multiply and a half-rate convert; the same row on every float
  // d in [0, 7.5) (tools/check_lookup_rows.py, exhaustive; sampled in
  // tests/test_numerics_lookup_rows.py)
  // (asm: the compiler's v_fma_f32 takes 16M from an SGPR, a half-rate
  // operand; v_fmamk_f32 carries it as a literal, -0.5 in a VGPR)
  float t;
  asm("v_fmamk_f32 %0, %1, 0x41ffffff, %2" : "=v"(t) : "v"(d), "v"(-0.5f));
  const float u = t + 12582912.0f;
  const float4 c = *(const float4*)((const char*)lk + (__float_as_int(u) & 0xf0));
  const float r = (((c.x * d + c.y) * d + c.z) * d + c.w) + lo;
  return (d >= 7.5f) ? hi : r;
}

// LOG_ADD(LOG_ZERO, y) == max(LOG_ZERO, y) exactly: above LOG_ZERO the sentinel
// returns y; below it the gap to LOG_ZERO exceeds the float spacing at 2e20
// (1.6e13) and thus the 7.5 cutoff.
__device__ __forceinline__ float mlp_log_add_from_zero(float y) { return fmaxf(MLP_LOG_ZERO, y); }

// EXP (CPNP/ScoreType.h:36-68) for x <= 0 (the only domain the posterior
// uses: min(LOG_ONE, .) clamps, CPNP/ProbabilisticModel.h:484).  The quartic
// runs in double on the float argument, like the reference.
__device__ __forceinline__ float mlp_exp_nonpos(float xf) {
  const double x = (double)xf;
  double c4, c3, c2, c1, c0;
  if (x > -2) {
    if (x > -0.5) {
      c4 = 0.03254409303190190000; c3 = 0.16280432765779600000; c2 = 0.49929760485974900000;
      c1 = 0.99995149601363700000; c0 = 0.99999925508501600000;
    } else if (x > -1) {
      c4 = 0.01973899026052090000; c3 = 0.13822379685007000000; c2 = 0.48056651562365000000;
      c1 = 0.99326940370383500000; c0 = 0.99906756856399500000;
    } else {
      c4 = 0.00940528203591384000; c3 = 0.09414963667859410000; c2 = 0.40825793595877300000;
      c1 = 0.93933625499130400000; c0 = 0.98369508190545300000;
    }
  } else if (x > -8) {
    if (x > -4) {
      c4 = 0.00217245711583303000; c3 = 0.03484829428350620000; c2 = 0.22118199801337800000;
      c1 = 0.67049462206469500000; c0 = 0.83556950223398500000;
    } else {
      c4 = 0.00012398771025456900; c3 = 0.00349155785951272000; c2 = 0.03727721426017900000;
      c1 = 0.17974997741536900000; c0 = 0.33249299994217400000;
    }
  } else {
    c4 = 0.00000051741713416603; c3 = 0.00002721456879608080; c2 = 0.00053418601865636800;
    c1 = 0.00464101989351936000; c0 = 0.01507447981459420000;
  }
  const float r = (float)((((c4 * x + c3) * x + c2) * x + c1) * x + c0);
  return (x > -16) ? r : 0.0f;
}

// LDS-table form of EXP for x <= 0: row k of `ex` (6 doubles, 5 used) holds
// the coefficients of interval k; row 6 is all zero (x <= -16 -> 0).
__device__ __forceinline__ void mlp_exp_table(double* ex) {
  const double c[7][5] = {
      {0.03254409303190190000, 0.16280432765779600000, 0.49929760485974900000, 0.99995149601363700000, 0.99999925508501600000},
      {0.01973899026052090000, 0.13822379685007000000, 0.48056651562365000000, 0.99326940370383500000, 0.99906756856399500000},
      {0.00940528203591384000, 0.09414963667859410000, 0.40825793595877300000, 0.93933625499130400000, 0.98369508190545300000},
      {0.00217245711583303000, 0.03484829428350620000, 0.22118199801337800000, 0.67049462206469500000, 0.83556950223398500000},
      {0.00012398771025456900, 0.00349155785951272000, 0.03727721426017900000, 0.17974997741536900000, 0.33249299994217400000},
      {0.00000051741713416603, 0.00002721456879608080, 0.00053418601865636800, 0.00464101989351936000, 0.01507447981459420000},
      {0, 0, 0, 0, 0}};
  for (int k = 0; k < 7; ++k) {
    for (int q = 0; q < 5; ++q) ex[k * 6 + q] = c[k][q];
    ex[k * 6 + 5] = 0;
  }
}
// The breakpoints -0.5 .. -16 are powers of two, so for x <= 0 the interval
// follows from the biased exponent E of x: k = clamp(E - 125, 0, 6); e.g.
// x = -0.5 has E = 126 -> k = 1, as `x > -0.5` fails in the reference chain
// (checked exhaustively over all non-positive floats).
__device__ __forceinline__ float mlp_exp_nonpos_t(float xf, const double* __restrict__ ex) {
  const double x = (double)xf;
  const int e = (int)((__float_as_uint(xf) >> 23) & 0xFF) - 125;
  const int k = min(max(e, 0), 6);
  const double* c = ex + k * 6;
  return (float)((((c[0] * x + c[1]) * x + c[2]) * x + c[3]) * x + c[4]);
}
__device__ __forceinline__ float mlp_post_from_sum_t(float s, float T, const double* __restrict__ ex) {
  const float v = s - T;
  return mlp_exp_nonpos_t(v < MLP_LOG_ONE ? v : MLP_LOG_ONE, ex);
}

// Posterior from (f + b) and the pair total (CPNP/ProbabilisticModel.h:484):
// EXP(min(LOG_ONE, (f + b) - T)); `s` is the stored float sum f + b.
__device__ __forceinline__ float mlp_post_from_sum(float s, float T) {
  const float v = s - T;
  return mlp_exp_nonpos(v < MLP_LOG_ONE ? v : MLP_LOG_ONE);
}

// x / 3 correctly rounded for 0 <= x <= 3 (the RMS merge's sum of three
// squared posteriors) in three instructions instead of the IEEE division
// sequence (v_div_scale x2, v_rcp, 5 FMAs, v_div_fmas, v_div_fixup): the
// product with RN(1/3), its exact residual by FMA, one corrected FMA.
// Checked against RN(x / 3) on every float in [0, 3], denormals included
// (tests/test_numerics_div3.py; tools/check_div3.py runs the whole range).
__device__ __forceinline__ float mlp_div3(float x) {
  const float r = 0x1.555556p-2f;  // RN(1/3)
  const float q = x * r;
  const float e = __builtin_fmaf(-q, 3.0f, x);
  return __builtin_fmaf(e, r, q);
}

// ---- wave-level neighbour exchange (DPP wave shifts, gfx9 family) --------
// lane l receives lane l-1's value; lane 0 keeps `old`.
__device__ __forceinline__ float mlp_shr1(float v, float old) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ int mlp_shr1i(int v, int old) {
  return __builtin_amdgcn_update_dpp(old, v, 0x138, 0xf, 0xf, false);
}
// lane l receives lane l+1's value; lane 63 keeps `old`.
__device__ __forceinline__ float mlp_shl1(float v, float old) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), 0x130, 0xf, 0xf, false));
}
__device__ __forceinline__ int mlp_shl1i(int v, int old) {
  return __builtin_amdgcn_update_dpp(old, v, 0x130, 0xf, 0xf, false);
}
// Shifts whose vacated lane (0 for shr, 63 for shl) reads 0 (DPP bound_ctrl):
// no old-value copy; for when that lane's result is overwritten or unused.
__device__ __forceinline__ float mlp_shr1z(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float mlp_shl1z(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xf, 0xf, true));
}
__device__ __forceinline__ int mlp_shr1zi(int v) { return __builtin_amdgcn_mov_dpp(v, 0x138, 0xf, 0xf, true); }
__device__ __forceinline__ int mlp_shl1zi(int v) { return __builtin_amdgcn_mov_dpp(v, 0x130, 0xf, 0xf, true); }
__device__ __forceinline__ double mlp_shr1zd(double v) {
  const int2 vv = *reinterpret_cast<const int2*>(&v);
  int2 r;
  r.x = __builtin_amdgcn_mov_dpp(vv.x, 0x138, 0xf, 0xf, true);
  r.y = __builtin_amdgcn_mov_dpp(vv.y, 0x138, 0xf, 0xf, true);
  return *reinterpret_cast<double*>(&r);
}
__device__ __forceinline__ double mlp_shl1zd(double v) {
  const int2 vv = *reinterpret_cast<const int2*>(&v);
  int2 r;
  r.x = __builtin_amdgcn_mov_dpp(vv.x, 0x130, 0xf, 0xf, true);
  r.y = __builtin_amdgcn_mov_dpp(vv.y, 0x130, 0xf, 0xf, true);
  return *reinterpret_cast<double*>(&r);
}
__device__ __forceinline__ double mlp_shr1d(double v, double old) {
  const int2 vv = *reinterpret_cast<const int2*>(&v), oo = *reinterpret_cast<const int2*>(&old);
  int2 r;
  r.x = __builtin_amdgcn_update_dpp(oo.x, vv.x, 0x138, 0xf, 0xf, false);
  r.y = __builtin_amdgcn_update_dpp(oo.y, vv.y, 0x138, 0xf, 0xf, false);
  return *reinterpret_cast<double*>(&r);
}
__device__ __forceinline__ double mlp_shl1d(double v, double old) {
  const int2 vv = *reinterpret_cast<const int2*>(&v), oo = *reinterpret_cast<const int2*>(&old);
  int2 r;
  r.x = __builtin_amdgcn_update_dpp(oo.x, vv.x, 0x130, 0xf, 0xf, false);
  r.y = __builtin_amdgcn_update_dpp(oo.y, vv.y, 0x130, 0xf, 0xf, false);
  return *reinterpret_cast<double*>(&r);
}

// ---- scaled fp64 for the partition function ------------------------------
// The reference runs the partition function in x87 long double
// (CPNP/MSAPartProbs.cpp).  We run it in fp64 with a per-lane power-of-two
// frame: stored value = true value * 2^(-MLP_PF_STEP * e).  Power-of-two
// rescaling is exact, so every product/sum rounds like unscaled fp64.
#define MLP_PF_STEP 200
#define MLP_PF_HUGE 0x1p200
// The reference stops with "ERROR: huge val error" once a forward value
// reaches long double infinity, 2^16384 (CPNP/MSAPartProbs.cpp:547-589,
// OS_HUGE_VALL = HUGE_VALL): the cell's largest value x 2^(200 e) >= 2^16384.
__device__ __forceinline__ bool mlp_pf_ldbl_overflow(double m, double e, double f, int E) {
  return E > 81 || (E == 81 && fmax(fmax(m, e), f) >= 0x1p184);
}
// Packed storage of (value, e): e in the 8 low mantissa bits (2^-44 rel.).
__device__ __forceinline__ double mlp_pf_pack(double v, int e) {
  unsigned long long b = (unsigned long long)__double_as_longlong(v);
  b = (b & ~0xFFull) | (unsigned long long)(e & 0xFF);
  return __longlong_as_double((long long)b);
}
__device__ __forceinline__ double mlp_pf_unpack(double p, int* e) {
  unsigned long long b = (unsigned long long)__double_as_longlong(p);
  *e = (int)(b & 0xFF);
  return __longlong_as_double((long long)(b & ~0xFFull));
}
