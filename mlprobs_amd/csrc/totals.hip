// totals.hip -- per-pair kernels of the posterior stage that follow the
// sweeps: the exact local-model chain totals, the 5-state backward total fold
// and the ELL -> canonical CSR compaction (one wave per pair / 8 pairs per
// wave; no wavefront).
#include <stdio.h>

#include <algorithm>

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
// skipping it is exact.  LOG_ADD(acc, x) >= max(acc, x) (the LOOKUP cubic
// lies >= 4.4e-4 above d on every float d in [0, 7.5), checked exhaustively),
// so acc is at least every element before it in the chain: an element with
// bound - x >= 7.5, bound = the largest element before it, is skipped exactly
// (fl(acc - x) >= fl(bound - x) for acc >= bound).
//
// Forward: the bound is the largest element of the rows before (prefix
// maximum of the sweeps' per-chunk maxima, Scratch::cmf) and of the row so
// far.  At C3 (pid 0, the family's delta) the forward chain's values rise
// along the rows: ~18k of the 160k terms of a pair change acc, ~55k pass the
// bound (local_fwd_fold).
// Backward (0.1% of the chunks hold a candidate): chunks whose maximum
// (Scratch::cmb) passes the test against acc are gathered and folded.
// =====================================================================
#define TOT_STAT(k, v)

// Fold chunks [kb, ke) of a chain (row-major chunk index (i - 1) * nch + c)
// whose maximum passes the test against acc, elements gathered from the
// step-diagonal array.
template <bool BWD>
__device__ __forceinline__ float fold_chunks(float acc, int64_t kb, int64_t ke, const float* __restrict__ cmx,
                                             const float* __restrict__ vals, int L2, int row0, int W,
                                             int64_t cell_off, const uint8_t* s1, const uint8_t* s2,
                                             const float* match, const float* ins, float two_rt1,
                                             const float4* lk, int lane) {
  const int nch = local_chunks(L2);
  for (int64_t k0 = kb; k0 < ke; k0 += 64) {
    const int64_t kk = k0 + lane;
    const float mx = kk < ke ? cmx[kk] : LZ;
    uint64_t live = __ballot(kk < ke && !(acc - mx >= 7.5f));
    while (live) {
      TOT_STAT(BWD ? 4 : 3, 1);
      const int64_t ck = k0 + __builtin_ctzll(live);
      const int i = (int)(ck / nch) + 1, cidx = (int)(ck % nch);
      const int j = 64 * cidx + 1 + lane;  // this lane's column of the chunk
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

// Forward chain: stream the pair's f_M strip by strip in its step-diagonal
// layout (one coalesced 256-B slab per step; lane r holds row 64 S + r in
// column order), list every element that passes the bound test in the
// lane's row list (this wave's region of Scratch::clist, one row of
// clist_row floats per lane: every element fits), then fold the strip's
// rows in order: per 64 listed elements, a ballot of those that pass the
// test against acc, the lowest folded, the ballot renewed (the rest of the
// list stays in order; an element that stopped passing is skipped, exactly).
//
// The row lists are written a whole 64-byte line at a time: each lane keeps
// the latest listed elements of its row in LDS (`lbuf`, this wave's
// kLbufSlots x 64 floats, lane-interleaved: conflict-free, a ring per lane)
// and, checked once per 8 steps (so the divergent flush runs at most once per
// 8 steps, not every step some lane fills up), stores its oldest 16 with
// four 16-byte stores once 16 have gathered (the strip's remainder at its
// end).
// Single 4-byte stores to 64 rows' lists left partly written lines that the
// caches evicted long before they filled (the lists of all resident waves
// exceed L2 and MALL): at C3 the listing took 104 ms a step with the stores,
// 19 ms without them (profiles/r04e_ab_totals_nostore.txt).
constexpr int kLbufSlots = 24;  // 16 to flush + up to 8 listed since the last check
static_assert(kLbufSlots % 4 == 0 && kLbufSlots >= 16 + 8, "flush groups of 4 never wrap; 16 to flush + 8 listed");
// the 16 elements from ring slot s0 (a multiple of 16 in list order) to dst
__device__ __forceinline__ void lbuf_flush16(float* __restrict__ dst, const float* lbuf, int s0, int lane) {
  float4* d = reinterpret_cast<float4*>(dst);
  // s0 is 0, 8 or 16: the 16 slots are two contiguous runs of 8 at most
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    int slot = s0 + 4 * q;
    slot = slot >= kLbufSlots ? slot - kLbufSlots : slot;  // 4 | kLbufSlots: a group never wraps
    const float* b = lbuf + slot * 64 + lane;
    d[q] = make_float4(b[0], b[64], b[128], b[192]);
  }
}
template <bool FOLD = true>
__device__ __forceinline__ float local_fwd_fold(const float* __restrict__ cmf, const float* __restrict__ fl, int L1,
                                                int L2, int row0, int W, int64_t cell_off, const float4* lk,
                                                float* __restrict__ region, int row_cap, int lane,
                                                float* __restrict__ lbuf, const float* __restrict__ rbp, bool* bad) {
  const int nch = local_chunks(L2);
  float acc = LZ, carry = LZ;  // carry: the largest element of the pair's rows before strip S
  const int S0 = (row0 + 1) >> 6, S1 = (row0 + L1) >> 6;
  const int tend = L2 + 63;  // steps of a strip: lane r holds column t - r at step t
  float* mine = region + (int64_t)lane * row_cap;
  for (int S = S0; S <= S1; ++S) {
    const int i = 64 * S + lane - row0;  // this lane's pair row
    const bool row_in = i >= 1 && i <= L1;
    float rmx = LZ;
    if (row_in)
      for (int c = 0; c < nch; ++c) {
        rmx = fmaxf(rmx, cmf[(int64_t)(i - 1) * nch + c]);
      }
    float incl = rmx;  // inclusive prefix maximum over the strip's rows
    for (int off = 1; off < 64; off <<= 1) {
      const float y = __shfl_up(incl, off);
      if (lane >= off) incl = fmaxf(incl, y);
    }
    float before = __shfl_up(incl, 1);
    if (lane == 0) before = LZ;
    // rbp (k_local_bounds): the fold of the chunk maxima of the rows before,
    // a tighter bound than their maximum, checked where the fold reaches the row
    const float rb = (rbp && row_in) ? rbp[i - 1] : LZ;
    float run = fmaxf(fmaxf(carry, before), rb);
    carry = fmaxf(carry, readlane_f(incl, 63));
    int cnt = 0;
    int done = 0;  // list elements already stored (a multiple of 16)
    const float* slab = fl + cell_off + ((int64_t)W * S + 1) * 64 + lane;  // + t * 64: step W S + t
    for (int t0 = 1; t0 <= tend; t0 += 8) {
      float x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        x[u] = (t0 + u <= tend) ? slab[(int64_t)(t0 + u) * 64] : LZ;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int j = t0 + u - lane;
        if (row_in && j >= 1 && j <= L2) {
          if (!(run - x[u] >= 7.5f)) {
            lbuf[(cnt % kLbufSlots) * 64 + lane] = x[u];
            ++cnt;
          }
          run = fmaxf(run, x[u]);
        }
      }
      if (cnt - done >= 16) {  // at most 8 listed since the last check: <= 24 in the ring
        lbuf_flush16(mine + done, lbuf, done % kLbufSlots, lane);
        done += 16;
      }
    }
    for (int k = done; k < cnt; ++k) mine[k] = lbuf[(k % kLbufSlots) * 64 + lane];  // the strip's remainder
    TOT_STAT(1, cnt);
    if constexpr (!FOLD) {  // timing experiment: streaming only
      acc = fmaxf(acc, (float)__builtin_amdgcn_readlane(cnt, 5));
      continue;
    }
    // the lists were written by this wave: same-CU visibility
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // the strip's rows in order
    for (int r = 0; r < 64; ++r) {
      if (rbp && readlane_f(rb, r) > acc) {  // the row's bound exceeds the chain: the caller redoes the pair
        *bad = true;
        return acc;
      }
      const int n = __builtin_amdgcn_readlane(cnt, r);
      const float* lst = region + (int64_t)r * row_cap;
      for (int k0 = 0; k0 < n; k0 += 64) {
        const bool in = k0 + lane < n;
        const float x = in ? lst[k0 + lane] : LZ;
        uint64_t live = __ballot(in && !(acc - x >= 7.5f));
        while (live) {
          const float v = readlane_f(x, __builtin_ctzll(live));
          acc = mlp_log_add_t(acc, v, lk);
          TOT_STAT(5, 1);
          live &= live - 1;
          live &= __ballot(!(acc - x >= 7.5f));
        }
      }
    }
    // the next strip's stores must not overtake this strip's list reads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  }
  return acc;
}

// Persistent: gridDim.x * 4 waves, each taking pairs off Scratch::tot_next
// until none is left (every wave reaches the exit).  With `only` (the
// lane-fold path's repair list: [0] = count, then slots) just those pairs.
__global__ __launch_bounds__(256) void k_local_totals(ModelScalars ms, const Tables* __restrict__ tab, SeqSet sq,
                                                      PairMeta pm, ChainMeta cm, PairRec* __restrict__ rec,
                                                      Scratch sc, int64_t npairs, const int32_t* __restrict__ only,
                                                      int parts) {
  __shared__ float4 lk[kLookupRows];
  __shared__ float match[26 * 26], ins[26];
  __shared__ float lbuf_all[kWavesPerBlock * kLbufSlots * 64];  // per wave: a ring per lane
  // beside the backward sweeps (MLP_TOT_BESIDE) the serial chains are the
  // batch's critical path and issue little: the SIMDs serve them first
  __builtin_amdgcn_s_setprio(3);
  if (threadIdx.x == 0) mlp_lookup_table(lk);
  for (int k = threadIdx.x; k < 26 * 26; k += blockDim.x) match[k] = tab->match[k];
  if (threadIdx.x < 26) ins[threadIdx.x] = tab->ins[threadIdx.x];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  float* region = sc.clist + wave_index() * 64 * (int64_t)sc.clist_row;
  float* lbuf = lbuf_all + (threadIdx.x >> 6) * kLbufSlots * 64;

  // one counter increment per wave, every lane taking part (no divergent
  // branch around the atomic): lane 0 receives the pair number
  auto take = [&]() -> int64_t {
    const int got = atomicAdd(sc.tot_next, lane == 0 ? 1 : 0);
    return __builtin_amdgcn_readfirstlane(got);
  };
  const int64_t ntask = only ? (int64_t)only[0] : npairs;
  for (int64_t task = take(); task < ntask; task = take()) {
    const int64_t p = only ? (int64_t)only[1 + task] : task;
    const int L1 = sq.len[pm.pa[p]], L2 = sq.len[pm.pb[p]];
    const int h = pm.chain[p];
    const int W = cm.width[h], row0 = pm.row0[p];
    const int64_t cell_off = cm.cell_off[h];
    const uint8_t* s1 = sq.res + sq.off[pm.pa[p]];
    const uint8_t* s2 = sq.res + sq.off[pm.pb[p]];
    const int64_t rm = pm.rm_off[p];
    bool bad = false;
    // with the folded bound (sc.crb) when k_local_bounds ran; a pair whose
    // bound failed is redone with the running maximum (exact either way)
    const float* rbp = sc.crb ? sc.crb + pm.ell_row[p] : nullptr;
    float tf = local_fwd_fold(sc.cmf + rm, sc.fl, L1, L2, row0, W, cell_off, lk, region, sc.clist_row, lane, lbuf, rbp,
                              &bad);
    if (bad) {
      bad = false;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      tf = local_fwd_fold(sc.cmf + rm, sc.fl, L1, L2, row0, W, cell_off, lk, region, sc.clist_row, lane, lbuf, nullptr,
                          &bad);
    }
    if (parts & kTotBwd) {
      const float tb = fold_chunks<true>(LZ, 0, (int64_t)L1 * local_chunks(L2), sc.cmb + rm, sc.bl, L2, row0, W,
                                         cell_off, s1, s2, match, ins, 2 * ms.rt1, lk, lane);
      if (lane == 0) rec[p].tbl = tb;
    }
    if (lane == 0) rec[p].tfl = tf;
  }
}

// =====================================================================
// Lane-per-pair forward chain.  The chain itself is serial, so one wave
// folding one pair issues ~20 wave instructions per folded element with one
// useful lane; here 64 pairs share a wave, one per lane, after a listing pass
// has put each pair's candidates in chain order into its region of the local
// backward array, dead between the two sweeps.
//
// The listing uses a tighter exact skip bound than the running maximum: the
// chain value at the start of row i is at least the exact LOG_ADD fold of the
// chunk maxima of the rows before (a subsequence of the chain, in order:
// folding fewer terms cannot give more, up to LOG_ADD's non-monotonic step
// at the 7.5 cutoff, ~5.5e-4).  That is checked where it is used: the fold
// compares each row's bound with the chain value at the row's start, and a
// pair whose bound exceeded it is redone by k_local_totals (repair list).
// At C3 the bound lists ~19% of the elements against ~35% for the running
// maximum (the elements that change the value: ~11%).
// =====================================================================

// Lane per pair: crb[ell + i - 1] = fold of the chunk maxima of rows 1..i-1.
__global__ __launch_bounds__(256) void k_local_bounds(SeqSet sq, PairMeta pm, Scratch sc, int64_t npairs) {
  __shared__ float4 lk[kLookupRows];
  __builtin_amdgcn_s_setprio(3);  // (as k_local_totals)
  if (threadIdx.x == 0) mlp_lookup_table(lk);
  __syncthreads();
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npairs) return;
  const int L1 = sq.len[pm.pa[p]], L2 = sq.len[pm.pb[p]];
  const int nch = local_chunks(L2);
  const float* __restrict__ cmx = sc.cmf + pm.rm_off[p];
  float* __restrict__ rb = sc.crb + pm.ell_row[p];
  float acc = LZ;
  constexpr int kRow = 8;  // a row's chunk maxima loaded together (L2 <= 512), then folded
  if (nch <= kRow) {
    // rows kAhead ahead in a register ring: each lane's loads are its own
    // pair's (uncoalesced), so a row loaded just before its fold waits the
    // whole memory latency once per row
    constexpr int kAhead = 4;
    float v[kAhead][kRow];
#pragma unroll
    for (int a = 0; a < kAhead; ++a)
#pragma unroll
      for (int u = 0; u < kRow; ++u) v[a][u] = (a < L1 && u < nch) ? cmx[(int64_t)a * nch + u] : LZ;
    for (int i = 0; i < L1; i += kAhead) {
#pragma unroll
      for (int a = 0; a < kAhead; ++a) {
        if (i + a < L1) {
          rb[i + a] = acc;
#pragma unroll
          for (int u = 0; u < kRow; ++u) acc = mlp_log_add_t(acc, v[a][u], lk);  // LOG_ADD(acc, LZ) == acc
        }
        const int nx = i + a + kAhead;
#pragma unroll
        for (int u = 0; u < kRow; ++u) v[a][u] = (nx < L1 && u < nch) ? cmx[(int64_t)nx * nch + u] : LZ;
      }
    }
    return;
  }
  for (int i = 0; i < L1; ++i) {
    rb[i] = acc;
    for (int c0 = 0; c0 < nch; c0 += kRow) {
      float v[kRow];
#pragma unroll
      for (int u = 0; u < kRow; ++u) v[u] = c0 + u < nch ? cmx[(int64_t)i * nch + c0 + u] : LZ;
#pragma unroll
      for (int u = 0; u < kRow; ++u) acc = mlp_log_add_t(acc, v[u], lk);  // LOG_ADD(acc, LZ) == acc
    }
  }
}

// Candidate k of pair row i (1-based): the lists go to the local backward
// array (Scratch::bl), dead until the backward sweep: the forward chain is
// folded between the forward and the backward sweeps, on the HMM stream,
// while the partition function's sweeps run on the side stream.  The pair's
// region is bl's slots cell_off + row0 W .. + (L1 + 1) W (the chain's rows
// partition its slots among the members); row i's candidates are contiguous
// at rows + (i - 1) * RS, RS = L2 rounded up to 4 floats, from the first
// 16-byte boundary: (L1 + 1) W >= L1 RS + 3 + W floats, W >= RS, W >= 8.
__device__ __forceinline__ float* lanefold_rows(const Scratch& sc, int64_t cell_off, int row0, int W) {
  // (pointer arithmetic from the slot, not an integer round trip: the
  // compiler keeps the global address space -- global, not flat, loads)
  float* const b = sc.bl + cell_off + (int64_t)row0 * W;
  const int mis = (int)((reinterpret_cast<uintptr_t>(b) >> 2) & 3);
  return b + ((4 - mis) & 3);
}
__device__ __forceinline__ int lanefold_rs(int L2) { return (L2 + 3) & ~3; }

// Wave per pair (persistent, as k_local_totals): the forward chain's
// candidates listed row by row (element x of row i is listed unless
// max(crb[i], max of the row so far) - x >= 7.5), each row contiguous,
// written 64 bytes at a time through the lane's LDS ring.
__global__ __launch_bounds__(256) void k_local_list(SeqSet sq, PairMeta pm, ChainMeta cm, Scratch sc,
                                                    int64_t npairs) {
  __shared__ float lbuf_all[kWavesPerBlock * kLbufSlots * 64];  // contiguous rows: per wave a ring per lane
  const int lane = threadIdx.x & 63;
  float* lbuf = lbuf_all + (threadIdx.x >> 6) * kLbufSlots * 64;
  auto take = [&]() -> int64_t {
    const int got = atomicAdd(sc.tot_next, lane == 0 ? 1 : 0);
    return __builtin_amdgcn_readfirstlane(got);
  };
  for (int64_t p = take(); p < npairs; p = take()) {
    const int L1 = sq.len[pm.pa[p]], L2 = sq.len[pm.pb[p]];
    const int h = pm.chain[p];
    const int W = cm.width[h], row0 = pm.row0[p];
    const int64_t cell_off = cm.cell_off[h];
    const int64_t ell = pm.ell_row[p];
    float* __restrict__ rows = lanefold_rows(sc, cell_off, row0, W);
    const int RS = lanefold_rs(L2);
    const int S0 = (row0 + 1) >> 6, S1 = (row0 + L1) >> 6;
    const int tend = L2 + 63;
    for (int S = S0; S <= S1; ++S) {
      const int i = 64 * S + lane - row0;
      const bool row_in = i >= 1 && i <= L1;
      float run = row_in ? sc.crb[ell + i - 1] : LZ;
      int cnt = 0;
      const float* slab = sc.fl + cell_off + ((int64_t)W * S + 1) * 64 + lane;
      float* __restrict__ mine = rows + (int64_t)(row_in ? i - 1 : 0) * RS;
      int done = 0;
      for (int t0 = 1; t0 <= tend; t0 += 8) {
        float x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = (t0 + u <= tend) ? slab[(int64_t)(t0 + u) * 64] : LZ;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int j = t0 + u - lane;
          if (row_in && j >= 1 && j <= L2) {
            if (!(run - x[u] >= 7.5f)) {
              lbuf[(cnt % kLbufSlots) * 64 + lane] = x[u];
              ++cnt;
            }
            run = fmaxf(run, x[u]);
          }
        }
        if (cnt - done >= 16) {  // at most 8 listed since the last check: <= 24 in the ring
          lbuf_flush16(mine + done, lbuf, done % kLbufSlots, lane);
          done += 16;
        }
      }
      for (int k = done; k < cnt; ++k) mine[k] = lbuf[(k % kLbufSlots) * 64 + lane];
      if (row_in) sc.lf_cnt[ell + i - 1] = cnt;
    }
  }
}

// Lane per pair: the forward chain over the listed candidates, rows in
// lockstep across the wave (row i of every lane's pair in the same outer
// iteration).  LOG_ADD(acc, x) == acc whenever acc - x >= 7.5, and
// LOG_ADD(acc, LOG_ZERO) == acc: every listed element and the padding fold
// unconditionally.  16-byte loads: the fold runs one lane's chain per pair,
// so the kernel lasts as long as the longest chain and every load the chain
// waits for adds to it.  Within a row, eight elements per step with the next
// 16 in flight; the next row's first 16 (its count read two rows ahead)
// loaded at the row's start.  The loads are unconditional (elements past a
// row's count are masked where they are folded; the reads stay inside the
// pair's region or, past its last row, inside the batch scratch's padding
// after bl, kLaneFoldPad): predicated loads made every wait a vmcnt(0).
__global__ __launch_bounds__(256) void k_local_fold(SeqSet sq, PairMeta pm, ChainMeta cm, PairRec* __restrict__ rec,
                                                    Scratch sc, int64_t npairs) {
  __shared__ float4 lk[kLookupRows];
  if (threadIdx.x == 0) mlp_lookup_table(lk);
  __syncthreads();
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npairs) return;
  const int L1 = sq.len[pm.pa[p]], L2 = sq.len[pm.pb[p]];
  const int h = pm.chain[p];
  const int64_t ell = pm.ell_row[p];
  float acc = LZ;
  bool bad = false;
  int n = sc.lf_cnt[ell];
  float rb = sc.crb[ell];
  const float4* __restrict__ rows4 = reinterpret_cast<const float4*>(lanefold_rows(sc, cm.cell_off[h], pm.row0[p], cm.width[h]));
  const int RS4 = lanefold_rs(L2) >> 2;
  int n1 = sc.lf_cnt[ell + min(1, L1 - 1)];
  float4 a0 = rows4[0], a1 = rows4[1], b0 = rows4[2], b1 = rows4[3];
  auto fold4 = [&](const float4 v, int k) {
    acc = mlp_log_add_t(acc, k < n ? v.x : LZ, lk);
    acc = mlp_log_add_t(acc, k + 1 < n ? v.y : LZ, lk);
    acc = mlp_log_add_t(acc, k + 2 < n ? v.z : LZ, lk);
    acc = mlp_log_add_t(acc, k + 3 < n ? v.w : LZ, lk);
  };
  for (int i = 1; i <= L1; ++i) {
    const float4* __restrict__ src = rows4 + (int64_t)(i - 1) * RS4;
    const float4* __restrict__ nxt = src + RS4;
    const int n2 = sc.lf_cnt[ell + min(i + 1, L1 - 1)];  // (past the last row: unused)
    const float rb_next = sc.crb[ell + min(i, L1 - 1)];
    const float4 na0 = nxt[0], na1 = nxt[1], nb0 = nxt[2], nb1 = nxt[3];
    bad |= rb > acc;  // the listing's bound must not exceed the chain at the row's start
    for (int k = 0; k < n; k += 8) {
      const float4 c0 = src[(k >> 2) + 4], c1 = src[(k >> 2) + 5];
      fold4(a0, k);
      if (k + 4 < n) fold4(a1, k + 4);
      a0 = b0;
      a1 = b1;
      b0 = c0;
      b1 = c1;
    }
    a0 = na0;
    a1 = na1;
    b0 = nb0;
    b1 = nb1;
    n = n1;
    n1 = n2;
    rb = rb_next;
  }
  rec[p].tfl = acc;
  if (bad || sc.force_repair) {
    const int k = atomicAdd(&sc.rep[0], 1);
    sc.rep[1 + k] = (int32_t)p;
  }
}

// Wave per pair, after the backward sweep: the backward chain over the chunks
// whose maximum passes the test (k_local_totals' second half).
__global__ __launch_bounds__(256) void k_local_btot(ModelScalars ms, const Tables* __restrict__ tab, SeqSet sq,
                                                    PairMeta pm, ChainMeta cm, PairRec* __restrict__ rec, Scratch sc,
                                                    int64_t npairs) {
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
  const uint8_t* s1 = sq.res + sq.off[pm.pa[p]];
  const uint8_t* s2 = sq.res + sq.off[pm.pb[p]];
  const float tb = fold_chunks<true>(LZ, 0, (int64_t)L1 * local_chunks(L2), sc.cmb + pm.rm_off[p], sc.bl, L2,
                                     pm.row0[p], cm.width[h], cm.cell_off[h], s1, s2, match, ins, 2 * ms.rt1, lk, lane);
  if (lane == 0) rec[p].tbl = tb;
}

// =====================================================================
// Sparse entries per pair: the sum of its rows' counts (k_merge's ell_cnt,
// overflowing rows included, as the per-row atomics it replaces summed):
// one wave per pair, after the merge.
// =====================================================================
__global__ __launch_bounds__(256) void k_pair_nnz(SeqSet sq, PairMeta pm, PairRec* __restrict__ rec, Scratch sc,
                                                  int64_t npairs) {
  const int64_t p = wave_index();
  if (p >= npairs) return;
  const int lane = threadIdx.x & 63;
  const int L1 = sq.len[pm.pa[p]];
  const int32_t* __restrict__ cn = sc.ell_cnt + pm.ell_row[p];
  long long s = 0;
  for (int i = lane; i < L1; i += 64) s += cn[i];
  for (int o = 32; o; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) rec[p].nnz = s;
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
  // per wave: the row (lane) of each entry of the current 64-row chunk, and
  // the rows' first entries, so the chunk's entries are copied 64 consecutive
  // ones at a time (coalesced stores) instead of one row per lane
  __shared__ uint8_t rowid_all[kWavesPerBlock][64 * kEll];
  __shared__ int32_t rstart_all[kWavesPerBlock][64];
  const int64_t p = wave_index();
  if (p >= npairs) return;
  const int lane = threadIdx.x & 63;
  uint8_t* rowid = rowid_all[threadIdx.x >> 6];
  int32_t* rstart = rstart_all[threadIdx.x >> 6];
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
    const int first = x - c;  // within the chunk
    if (i <= L1) rp[i + 1] = run + x;
    rstart[lane] = first;
    for (int k = 0; k < c; ++k) rowid[first + k] = (uint8_t)lane;
    const int tot = __shfl(x, 63);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int64_t src0 = (er0 + r0 - 1) * kEll;
    for (int e = lane; e < tot; e += 64) {
      const int r = rowid[e];
      const int64_t s = src0 + (int64_t)r * kEll + (e - rstart[r]);
      out_cols[eb + run + e] = sc.ell_col[s];
      out_vals[eb + run + e] = sc.ell_val[s];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    run += tot;
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
                               PairRec* rec, Scratch sc, int64_t npairs, int nwaves, hipStream_t st, int parts) {
  if (npairs <= 0) return hipSuccess;
  if (!(parts & kTotFwd)) {  // the backward chains alone
    hipLaunchKernelGGL(k_local_btot, wave_grid(npairs), dim3(64 * kWavesPerBlock), 0, st, ms, tab, seqs, pm, cm, rec,
                       sc, npairs);
    return hipGetLastError();
  }
  if (sc.crb)  // the folded row bounds (lane per pair)
    hipLaunchKernelGGL(k_local_bounds, dim3((unsigned)((npairs + 255) / 256)), dim3(256), 0, st, seqs, pm, sc, npairs);
  hipError_t e = hipMemsetAsync(sc.tot_next, 0, sizeof(int32_t), st);
  if (e != hipSuccess) return e;
  if (nwaves % kWavesPerBlock) return hipErrorInvalidValue;  // every wave owns a list region
  hipLaunchKernelGGL(k_local_totals, wave_grid(nwaves), dim3(64 * kWavesPerBlock), 0, st, ms, tab, seqs, pm, cm, rec,
                     sc, npairs, (const int32_t*)nullptr, parts);
  return hipGetLastError();
}

// The lane fold, forward half: between the forward and the backward sweeps
// (the lists live in bl until the backward sweep writes it).
hipError_t launch_local_fwd_lanefold(SeqSet seqs, PairMeta pm, ChainMeta cm, PairRec* rec, Scratch sc, int64_t npairs,
                                     int nwaves, hipStream_t st) {
  if (npairs <= 0) return hipSuccess;
  if (nwaves % kWavesPerBlock) return hipErrorInvalidValue;
  hipError_t e;
  if ((e = hipMemsetAsync(sc.rep, 0, sizeof(int32_t), st)) != hipSuccess) return e;
  const dim3 lanes((unsigned)((npairs + 255) / 256));
  hipLaunchKernelGGL(k_local_bounds, lanes, dim3(256), 0, st, seqs, pm, sc, npairs);
  if ((e = hipMemsetAsync(sc.tot_next, 0, sizeof(int32_t), st)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_local_list, wave_grid(nwaves), dim3(64 * kWavesPerBlock), 0, st, seqs, pm, cm, sc, npairs);
  hipLaunchKernelGGL(k_local_fold, lanes, dim3(256), 0, st, seqs, pm, cm, rec, sc, npairs);
  return hipGetLastError();
}

// ... and after the backward sweep: the backward chains, then the pairs whose
// bound failed (normally none: the waves find an empty list and exit) redone
// with the running-maximum bound, both chains.
hipError_t launch_local_bwd_lanefold(const ModelScalars& ms, const Tables* tab, SeqSet seqs, PairMeta pm, ChainMeta cm,
                                     PairRec* rec, Scratch sc, int64_t npairs, int nwaves, hipStream_t st) {
  if (npairs <= 0) return hipSuccess;
  if (nwaves % kWavesPerBlock) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_local_btot, wave_grid(npairs), dim3(64 * kWavesPerBlock), 0, st, ms, tab, seqs, pm, cm, rec, sc,
                     npairs);
  hipError_t e;
  if ((e = hipMemsetAsync(sc.tot_next, 0, sizeof(int32_t), st)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_local_totals, wave_grid(std::min(nwaves, 1024)), dim3(64 * kWavesPerBlock), 0, st, ms, tab, seqs,
                     pm, cm, rec, sc, npairs, (const int32_t*)sc.rep, kTotFwd | kTotBwd);
  return hipGetLastError();
}

hipError_t launch_pair_nnz(SeqSet seqs, PairMeta pm, PairRec* rec, Scratch sc, int64_t npairs, hipStream_t st) {
  if (npairs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pair_nnz, wave_grid(npairs), dim3(64 * kWavesPerBlock), 0, st, seqs, pm, rec, sc, npairs);
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
