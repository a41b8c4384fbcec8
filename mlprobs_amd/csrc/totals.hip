// totals.hip -- per-pair kernels of the posterior stage that follow the
// sweeps: the exact local-model chain totals, the 5-state backward total fold
// and the ELL -> canonical CSR compaction (one wave per pair / 8 pairs per
// wave; no wavefront).
#include "mlp_kernels.h"
#include "mlp_numerics.h"

namespace mlp {

#define LZ MLP_LOG_ZERO

__device__ __forceinline__ float readlane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ int64_t wave_index() {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  return (int64_t)blockIdx.x * (blockDim.x >> 6) + w;
}
static inline dim3 wave_grid(int64_t n) {
  return dim3((unsigned)((n + kWavesPerBlock - 1) / kWavesPerBlock));
}

// =====================================================================
// Local-model totals: the reference sums LOG_PLUS_EQUALS over all interior
// cells in row-major order (CPNP/ProbabilisticModel.h:435-450), a single
// non-associative chain, for the forward and the backward half.
//
// Rows are padded to a multiple of 4 with LOG_ZERO, a no-op element.  An
// element x changes the running value acc only if acc - x < 7.5: otherwise
// LOG_ADD returns acc unchanged (CPNP/ScoreType.h:279-285), so skipping it is
// exact; acc never decreases, so a skipped element stays skippable.
// =====================================================================
// Variant (default): 8 pairs per wave, 8 lanes per pair.  Chunks of 64
// elements per chain (8 per lane, two float4 loads); candidates of each
// chain (elements with acc - x < 7.5, acc = chain value at the chunk start)
// are compacted in order into LDS, then lanes 0..15 fold the 16 chains of the
// wave in parallel.  The candidate list is a superset of the elements that
// change acc: LOG_ADD(acc, x) for acc - x >= 7.5 returns acc exactly, so
// folding every listed element reproduces the reference's serial chain.
#ifndef MLP_TOT_PAIRS
#define MLP_TOT_PAIRS 8
#endif
constexpr int kTotPairs = MLP_TOT_PAIRS;   // pairs per wave
constexpr int kTotLP = 64 / kTotPairs;      // lanes per pair
constexpr int kTotEL = 64 / kTotLP;         // elements per lane per 64-element chunk (float4 pieces: >= 4)
static_assert(kTotEL >= 4 && kTotEL % 4 == 0, "MLP_TOT_PAIRS must be 4, 8 or 16");
__global__ __launch_bounds__(256) void k_local_totals_multi(SeqSet sq, PairMeta pm, PairRec* __restrict__ rec,
                                                            Scratch sc, int64_t npairs) {
  __shared__ float4 lk[kLookupRows];
  __shared__ float list[kWavesPerBlock][2 * kTotPairs][64];
  if (threadIdx.x == 0) mlp_lookup_table(lk);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int g = lane / kTotLP, sub = lane % kTotLP;
  const int64_t p = ((int64_t)blockIdx.x * kWavesPerBlock + w) * kTotPairs + g;
  int64_t ne = 0, base = 0;
  if (p < npairs) {
    const int L1 = sq.len[pm.pa[p]], L2 = sq.len[pm.pb[p]];
    ne = (int64_t)L1 * ((L2 + 3) & ~3);
    base = pm.rm_off[p];
  }
  int64_t emax = ne;
  for (int off = 32; off >= kTotLP; off >>= 1) emax = max(emax, (int64_t)__shfl_xor(emax, off));
  const float* __restrict__ cf = sc.chf + base;
  const float* __restrict__ cb = sc.chb + base;
  // chain c = 2g (forward) / 2g+1 (backward) is folded on lane c
  float acc = LZ;
  float nf[kTotEL], nb[kTotEL];
  auto load = [&](int64_t e0, float* f, float* b) {
    const int64_t e = e0 + sub * kTotEL;   // ne is a multiple of 4: float4 pieces are all-in or all-out
#pragma unroll
    for (int h = 0; h < kTotEL / 4; ++h) {
      float4 vf = make_float4(LZ, LZ, LZ, LZ), vb = vf;
      if (e + 4 * h < ne) {
        vf = *reinterpret_cast<const float4*>(cf + e + 4 * h);
        vb = *reinterpret_cast<const float4*>(cb + e + 4 * h);
      }
      f[4 * h + 0] = vf.x; f[4 * h + 1] = vf.y; f[4 * h + 2] = vf.z; f[4 * h + 3] = vf.w;
      b[4 * h + 0] = vb.x; b[4 * h + 1] = vb.y; b[4 * h + 2] = vb.z; b[4 * h + 3] = vb.w;
    }
  };
  // two chunks in flight: HBM latency exceeds one chunk's fold
  float nf2[kTotEL], nb2[kTotEL];
  load(0, nf, nb);
  load(64, nf2, nb2);
  // exclusive prefix of a per-lane count over the kTotLP lanes of its group
  auto group_scan = [&](int c) {
    int x = c;
#pragma unroll
    for (int d = 1; d < kTotLP; d <<= 1) {
      const int y = __shfl_up(x, d, kTotLP);
      x += (sub >= d) ? y : 0;
    }
    return x - c;
  };
  auto chunk = [&](int64_t e0, float* xf, float* xb) {
    const float af = __shfl(acc, 2 * g), ab = __shfl(acc, 2 * g + 1);
    const int64_t e = e0 + sub * kTotEL;
    unsigned ff = 0, fb = 0;
#pragma unroll
    for (int k = 0; k < kTotEL; ++k) {
      const bool in = e + k < ne;
      ff |= (in && !(af - xf[k] >= 7.5f)) ? (1u << k) : 0u;
      fb |= (in && !(ab - xb[k] >= 7.5f)) ? (1u << k) : 0u;
    }
    const int cf_n = __popc(ff), cb_n = __popc(fb);
    int pf = group_scan(cf_n), pb = group_scan(cb_n);
    float* lf = list[w][2 * g];
    float* lb = list[w][2 * g + 1];
#pragma unroll
    for (int k = 0; k < kTotEL; ++k) {
      if (ff & (1u << k)) lf[pf++] = xf[k];
      if (fb & (1u << k)) lb[pb++] = xb[k];
    }
    // totals per chain: last lane of the group holds the inclusive sums
    const int tot_f = __shfl(pf, g * kTotLP + kTotLP - 1), tot_b = __shfl(pb, g * kTotLP + kTotLP - 1);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // chain `lane` (< 16) folds its list; count from its group's last lane
    const int cnt_f = __shfl(tot_f, (lane >> 1) * kTotLP), cnt_b = __shfl(tot_b, (lane >> 1) * kTotLP);
    const int cnt = lane < 2 * kTotPairs ? ((lane & 1) ? cnt_b : cnt_f) : 0;
    const float* my = list[w][lane & (2 * kTotPairs - 1)];
    for (int k = 0; __any(k < cnt); ++k) {
      if (k < cnt) acc = mlp_log_add_t(acc, my[k], lk);
    }
    __builtin_amdgcn_wave_barrier();
  };
  for (int64_t e0 = 0; e0 < emax; e0 += 128) {
    float xf[kTotEL], xb[kTotEL];
#pragma unroll
    for (int k = 0; k < kTotEL; ++k) { xf[k] = nf[k]; xb[k] = nb[k]; }
    if (e0 + 128 < emax) load(e0 + 128, nf, nb);
    chunk(e0, xf, xb);
    if (e0 + 64 >= emax) break;
#pragma unroll
    for (int k = 0; k < kTotEL; ++k) { xf[k] = nf2[k]; xb[k] = nb2[k]; }
    if (e0 + 192 < emax) load(e0 + 192, nf2, nb2);
    chunk(e0 + 64, xf, xb);
  }
  const float tf = __shfl(acc, 2 * g), tb = __shfl(acc, 2 * g + 1);
  if (p < npairs && sub == 0) {
    rec[p].tfl = tf;
    rec[p].tbl = tb;
  }
}

// Variant: one wave per pair, candidates folded serially (see above).
__global__ __launch_bounds__(256) void k_local_totals_wave(SeqSet sq, PairMeta pm, PairRec* __restrict__ rec,
                                                           Scratch sc, int64_t npairs) {
  __shared__ float4 lk[kLookupRows];
  if (threadIdx.x == 0) mlp_lookup_table(lk);
  __syncthreads();
  const int64_t p = wave_index();
  if (p >= npairs) return;
  const int lane = threadIdx.x & 63;
  const int L1 = sq.len[pm.pa[p]], L2 = sq.len[pm.pb[p]];
  const int64_t ne = (int64_t)L1 * ((L2 + 3) & ~3);
  const float* __restrict__ cf = sc.chf + pm.rm_off[p];
  const float* __restrict__ cbk = sc.chb + pm.rm_off[p];
  // lane 0 carries the forward chain, lane 1 the backward chain: one LOG_ADD
  // sequence advances both (LOG_ADD(acc, LOG_ZERO) == acc keeps an idle
  // chain unchanged)
  float acc = LZ;
  float tf = LZ, tb = LZ;   // wave-uniform copies
  float xf = LZ, xb = LZ;
  if (lane < ne) { xf = cf[lane]; xb = cbk[lane]; }
  for (int64_t c0 = 0; c0 < ne; c0 += 64) {
    const float cxf = xf, cxb = xb;
    const int64_t nx = c0 + 64 + lane;
    xf = LZ; xb = LZ;
    if (nx < ne) { xf = cf[nx]; xb = cbk[nx]; }   // prefetch next chunk
    uint64_t mf = __ballot(!(tf - cxf >= 7.5f));
    uint64_t mb = __ballot(!(tb - cxb >= 7.5f));
    while (mf | mb) {
      const float vf = mf ? readlane_f(cxf, __builtin_ctzll(mf)) : LZ;
      const float vb = mb ? readlane_f(cxb, __builtin_ctzll(mb)) : LZ;
      acc = mlp_log_add_t(acc, lane == 0 ? vf : vb, lk);
      tf = readlane_f(acc, 0);
      tb = readlane_f(acc, 1);
      if (mf) mf = (mf & (mf - 1)) & __ballot(!(tf - cxf >= 7.5f));
      if (mb) mb = (mb & (mb - 1)) & __ballot(!(tb - cxb >= 7.5f));
    }
  }
  if (lane == 0) {
    rec[p].tfl = tf;
    rec[p].tbl = tb;
  }
}

// =====================================================================
// ELL -> CSR compaction: one wave per pair.
// =====================================================================
__global__ __launch_bounds__(256) void k_compact(SeqSet sq, PairMeta pm, Scratch sc,
                                                 const int64_t* __restrict__ ent_base,
                                                 int32_t* __restrict__ out_rowptr,
                                                 const int64_t* __restrict__ rowptr_base,
                                                 uint16_t* __restrict__ out_cols,
                                                 float* __restrict__ out_vals, int64_t npairs) {
  const int64_t p = wave_index();
  if (p >= npairs) return;
  const int lane = threadIdx.x & 63;
  const int L1 = sq.len[pm.pa[p]];
  const int64_t er0 = pm.ell_row[p];
  const int64_t eb = ent_base[p];
  int32_t* rp = out_rowptr + rowptr_base[p];
  if (lane == 0) { rp[0] = 0; rp[1] = 0; }
  int run = 0;
  for (int r0 = 1; r0 <= L1; r0 += 64) {
    const int i = r0 + lane;
    const int c = (i <= L1) ? min(sc.ell_cnt[er0 + i - 1], kEll) : 0;
    // inclusive wave scan
    int x = c;
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(x, off);
      if (lane >= off) x += y;
    }
    const int start = run + x - c;
    if (i <= L1) {
      rp[i + 1] = start + c;
      for (int k = 0; k < c; ++k) {
        out_cols[eb + start + k] = sc.ell_col[(er0 + i - 1) * kEll + k];
        out_vals[eb + start + k] = sc.ell_val[(er0 + i - 1) * kEll + k];
      }
    }
    run += __shfl(x, 63);
  }
}

// =====================================================================
// 5-state backward total fold: T_bwd over the initial cells (run on device
// by the first lane of the merge kernel's caller via this tiny kernel).
// =====================================================================
__global__ void k_fold_totals(ModelScalars ms, SeqSet sq, PairMeta pm, PairRec* __restrict__ rec,
                              const Tables* __restrict__ tab, int64_t npairs) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npairs) return;
  const uint8_t* s1 = sq.res + sq.off[pm.pa[p]];
  const uint8_t* s2 = sq.res + sq.off[pm.pb[p]];
  const int c1 = s1[0], c2 = s2[0];
  const float f0 = ms.init[0] + tab->match[c1 * 26 + c2];
  const float fx1 = ms.init[1] + tab->ins[c1], fx2 = ms.init[3] + tab->ins[c1];
  const float fy1 = ms.init[2] + tab->ins[c2], fy2 = ms.init[4] + tab->ins[c2];
  PairRec& r = rec[p];
  // CPNP/ProbabilisticModel.h:421-432
  float tb = f0 + r.b5[0];
  tb = mlp_log_add(tb, fx1 + r.b5[1]);
  tb = mlp_log_add(tb, fy1 + r.b5[2]);
  tb = mlp_log_add(tb, fx2 + r.b5[3]);
  tb = mlp_log_add(tb, fy2 + r.b5[4]);
  r.b5[0] = tb;  // merge kernel reads the folded backward total here
}

// ------------------------------------------------------------ launchers
hipError_t launch_local_totals(SeqSet seqs, PairMeta pm, PairRec* rec, Scratch sc, int64_t npairs,
                               hipStream_t st) {
  if (npairs <= 0) return hipSuccess;
  const char* v = getenv("MLP_TOTALS");
  if (v && v[0] == 'w')
    hipLaunchKernelGGL(k_local_totals_wave, wave_grid(npairs), dim3(64 * kWavesPerBlock), 0, st, seqs, pm, rec, sc, npairs);
  else
    hipLaunchKernelGGL(k_local_totals_multi, dim3((unsigned)((npairs + kTotPairs * kWavesPerBlock - 1) / (kTotPairs * kWavesPerBlock))),
                       dim3(64 * kWavesPerBlock), 0, st, seqs, pm, rec, sc, npairs);
  return hipGetLastError();
}

hipError_t launch_fold_totals(const ModelScalars& ms, const Tables* tab, SeqSet seqs, PairMeta pm,
                              PairRec* rec, int64_t npairs, hipStream_t st) {
  if (npairs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_fold_totals, dim3((unsigned)((npairs + 255) / 256)), dim3(256), 0, st, ms, seqs, pm, rec, tab, npairs);
  return hipGetLastError();
}

hipError_t launch_compact(SeqSet seqs, PairMeta pm, PairRec* rec, Scratch sc,
                          const int64_t* ent_base, int32_t* out_rowptr, const int64_t* rowptr_base,
                          uint16_t* out_cols, float* out_vals, int64_t npairs, hipStream_t st) {
  if (npairs <= 0) return hipSuccess;
  (void)rec;
  hipLaunchKernelGGL(k_compact, wave_grid(npairs), dim3(64 * kWavesPerBlock), 0, st, seqs, pm, sc,
                     ent_base, out_rowptr, rowptr_base, out_cols, out_vals, npairs);
  return hipGetLastError();
}

}  // namespace mlp
