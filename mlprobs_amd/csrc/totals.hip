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
// non-associative chain, for the forward half (f_M) and the backward half
// (b_M + emission).
//
// An element x changes the running value acc only if acc - x < 7.5:
// otherwise LOG_ADD returns acc unchanged (CPNP/ScoreType.h:279-285), so
// skipping it is exact; acc never decreases, so a skipped element stays
// skippable.  The sweeps leave, per pair row and 64-column chunk, the
// largest chain element of the chunk (Scratch::cmf / cmb); a chunk with
// acc - max >= 7.5 holds no element that can change acc (fl(acc - x) >=
// fl(acc - max) for x <= max) and is skipped whole.  At C3 about 0.5% of the
// forward chunks and 0.07% of the backward ones are not skippable; only
// those are read, 64 elements gathered from the step-diagonal f_M / b_M
// (their addresses from the chain layout), and folded exactly in order.
// One wave per pair; acc is wave-uniform.
// =====================================================================
template <bool BWD>
__device__ __forceinline__ float local_chain_fold(const float* __restrict__ cmx, const float* __restrict__ vals,
                                                  int L1, int L2, int row0, int W, int64_t cell_off,
                                                  const uint8_t* s1, const uint8_t* s2, const float* match,
                                                  const float* ins, float two_rt1, const float4* lk, int lane) {
  const int nch = local_chunks(L2);
  const int64_t n = (int64_t)L1 * nch;
  float acc = LZ;
  for (int64_t k0 = 0; k0 < n; k0 += 64) {
    const int64_t kk = k0 + lane;
    const float mx = kk < n ? cmx[kk] : LZ;
    uint64_t live = __ballot(kk < n && !(acc - mx >= 7.5f));
    while (live) {
      const int64_t ck = k0 + __builtin_ctzll(live);
      const int i = (int)(ck / nch) + 1, cidx = (int)(ck % nch);
      const int j = 64 * cidx + 1 + lane;   // this lane's column of the chunk
      float x = LZ;
      const bool in = j <= L2;
      if (in) {
        const int g = row0 + i, r = g & 63;
        const int64_t tau = (int64_t)W * (g >> 6) + r + j;
        const float v = vals[cell_off + (tau + 1) * 64 + r];
        if constexpr (BWD) {
          // CPNP/ProbabilisticModel.h:444-445, the backward sweep's expression
          const int c1 = s1[i - 1], c2 = s2[j - 1];
          x = v + match[c1 * 26 + c2] - ins[c1] - ins[c2] - two_rt1;
        } else {
          x = v;
        }
      }
      // the chunk's elements in column order; candidates only (exact)
      uint64_t m = __ballot(in && !(acc - x >= 7.5f));
      while (m) {
        const float v = readlane_f(x, __builtin_ctzll(m));
        acc = mlp_log_add_t(acc, v, lk);
        m &= m - 1;
        m &= __ballot(!(acc - x >= 7.5f));
      }
      live &= live - 1;
      live &= __ballot(!(acc - mx >= 7.5f));
    }
  }
  return acc;
}

__global__ __launch_bounds__(256) void k_local_totals(ModelScalars ms, const Tables* __restrict__ tab, SeqSet sq,
                                                      PairMeta pm, ChainMeta cm, PairRec* __restrict__ rec,
                                                      Scratch sc, int64_t npairs) {
  __shared__ float4 lk[kLookupRows];
  __shared__ float match[26 * 26], ins[26];
  if (threadIdx.x == 0) mlp_lookup_table(lk);
  for (int k = threadIdx.x; k < 26 * 26; k += blockDim.x) match[k] = tab->match[k];
  if (threadIdx.x < 26) ins[threadIdx.x] = tab->ins[threadIdx.x];
  __syncthreads();
  const int64_t p = wave_index();
  if (p >= npairs) return;
  const int lane = threadIdx.x & 63;
  const int L1 = sq.len[pm.pa[p]], L2 = sq.len[pm.pb[p]];
  const int h = pm.chain[p];
  const int W = cm.width[h], row0 = pm.row0[p];
  const int64_t cell_off = cm.cell_off[h];
  const uint8_t* s1 = sq.res + sq.off[pm.pa[p]];
  const uint8_t* s2 = sq.res + sq.off[pm.pb[p]];
  const int64_t rm = pm.rm_off[p];
  const float tf = local_chain_fold<false>(sc.cmf + rm, sc.fl, L1, L2, row0, W, cell_off, s1, s2, match, ins,
                                           2 * ms.rt1, lk, lane);
  const float tb = local_chain_fold<true>(sc.cmb + rm, sc.bl, L1, L2, row0, W, cell_off, s1, s2, match, ins,
                                          2 * ms.rt1, lk, lane);
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
hipError_t launch_local_totals(const ModelScalars& ms, const Tables* tab, SeqSet seqs, PairMeta pm, ChainMeta cm,
                               PairRec* rec, Scratch sc, int64_t npairs, hipStream_t st) {
  if (npairs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_local_totals, wave_grid(npairs), dim3(64 * kWavesPerBlock), 0, st, ms, tab, seqs, pm, cm, rec,
                     sc, npairs);
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
