// profile.hip -- the weighted profile-profile posterior of QuickProbs'
// progressive construction and refinement (ParallelProbabilisticModel::
// buildPosterior, QP/Alignment/Multiple/ParallelProbabilisticModel.cpp:301-430)
// from the device-resident sparse set.
//
// posterior[r][c] accumulates w_ij * P_ij(ii, jj) over the sequence pairs
// (i in profile A, j in profile B) where sequence i has residue ii in column r
// and j has jj in column c, in the reference's order: i, then j, then the row
// ii of block (i, j), then its entries.  One wave owns one dense row r and
// keeps it in LDS; for a run of up to 64 consecutive pairs (i, j) it loads
// the rows' extents (one lane per pair, so a small profile B still fills the
// wave), computes the products of all their entries in parallel into an LDS
// stage, and then adds the stage into the row one pair after another.  The
// entries of one row hit distinct columns, so each pair's adds are one
// parallel step, and a wave's LDS operations retire in order: every cell
// sees its terms in the reference's sequence, with the reference's float
// operations
// (w * v, then +=).
//
// Sequences i with a gap in column r contribute nothing; each wave compacts
// them away 64 at a time before forming its runs (most of a long alignment's
// cells are gaps).  A short profile A leaves most of the chip idle (a wave
// per column), so gridDim.y waves can then share a row: wave k owns the
// column range [c0, c1) of row r, walks the same entries and adds only the
// ones landing in its range.  Each cell still has one owner and its terms in
// the same order, so the split changes no bit of the result.
#include <stdlib.h>

#include <algorithm>

#include "mlp_kernels.h"
#include "mlp_numerics.h"

namespace mlp {

constexpr int kProfStage = 1024;  // staged entries per run of pairs

// LDS writes of some lanes made visible to the other lanes of the wave
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// acc += v as one ds_add_f32 (IEEE round-to-nearest add, like acc + v)
__device__ __forceinline__ void lds_add(float* a, float v) {
  __hip_atomic_fetch_add(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

static __host__ __device__ inline size_t prof_acc_bytes(int cols) { return ((size_t)cols * 4 + 15) & ~(size_t)15; }
static size_t profile_lds_cols(int cols) { return prof_acc_bytes(cols) + (size_t)kProfStage * 9 + 7 * 65 * 8; }
size_t profile_lds(int L2) { return profile_lds_cols(L2 + 1); }

__global__ __launch_bounds__(64) void k_profile_post(ProfileArgs A) {
  const int lane = threadIdx.x;
  const int r = blockIdx.x + 1;
  const int W2 = A.L2 + 1;
  const int cw = (W2 + gridDim.y - 1) / gridDim.y;
  const int c0 = blockIdx.y * cw, c1 = min(W2, c0 + cw);
  extern __shared__ __align__(16) uint8_t lds[];
  float* acc = (float*)lds;                                     // columns c0 .. c1 - 1
  int32_t* st_c = (int32_t*)(lds + prof_acc_bytes(cw));         // staged dense columns
  float* st_p = (float*)(st_c + kProfStage);                    // staged products
  int64_t* l_e = (int64_t*)(st_p + kProfStage);                 // per lane: first entry (absolute)
  int32_t* l_st = (int32_t*)(l_e + 65);                         // per lane: stage start (prefix), [64] = total
  int32_t* l_tr = l_st + 65;                                    // per lane: transposed block
  int32_t* l_j = l_tr + 65;                                     // per lane: sequence j of profile B
  float* l_w = (float*)(l_j + 65);                              // per lane: pair weight
  int32_t* l_i = (int32_t*)(l_w + 65);                          // sequences i with a residue in column r
  int32_t* l_ii = l_i + 65;                                     // ... and that residue
  uint8_t* st_l = (uint8_t*)(l_ii + 65);                        // staged entry -> its lane
  for (int c = c0 + lane; c < c1; c += 64) acc[c - c0] = 0.f;
  for (int i0 = 0; i0 < A.n1; i0 += 64) {
    // the next (up to) 64 sequences i, compacted to those with a residue in
    // column r (the others contribute nothing)
    {
      const int i = i0 + lane;
      const int ii = i < A.n1 ? A.inv1[(int64_t)i * (A.L1 + 1) + r] : 0;
      const unsigned long long m = __ballot(ii != 0);
      if (ii != 0) {
        const int pos = __popcll(m & ((1ull << lane) - 1));
        l_i[pos] = i;
        l_ii[pos] = ii;
      }
      if (lane == 0) l_i[64] = __popcll(m);
    }
    wave_sync();
    const int64_t Q = (int64_t)l_i[64] * A.n2;
    // runs of 64 consecutive pairs (i, j) of the compacted list, i-major:
    // the reference's order
    for (int64_t q0 = 0; q0 < Q;) {
      // ---- extents of the rows ii of blocks (i, j), one lane per pair
      const int64_t q = q0 + lane;
      int cnt = 0, jl = 0, tr = 0;
      int64_t e = 0;
      float wv = 0.f;
      if (q < Q) {
        const int k = (int)(q / A.n2);
        jl = (int)(q - (int64_t)k * A.n2);
        const int ii = l_ii[k];
        const int64_t pair = (int64_t)l_i[k] * A.n2 + jl;
        const int64_t rb = A.rpb[pair];
        tr = rb < 0;
        const int32_t* rp = tr ? A.trowptr + (~rb) : A.rowptr + rb;
        const int b = rp[ii];
        cnt = rp[ii + 1] - b;
        e = A.eb[pair] + b;
        wv = A.w[pair];
      }
      // inclusive prefix of cnt over the lanes
      int x = cnt;
      for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d);
        if (lane >= d) x += y;
      }
      const int start = x - cnt;
      // lanes whose rows fit the stage (a prefix of the run; the first lane
      // always takes part, a longer row is added in pieces below)
      const bool fits = x <= A.stage || lane == 0;
      const unsigned long long fitm = __ballot(fits && q < Q);
      const int nl = __popcll(~fitm) ? __builtin_ctzll(~fitm) : 64;
      l_e[lane] = e;
      l_st[lane] = start;
      l_tr[lane] = tr;
      l_j[lane] = jl;
      l_w[lane] = wv;
      if (lane == 63) l_st[64] = x;
      wave_sync();
      const int total_staged = l_st[nl];  // entries of lanes 0 .. nl-1
      const bool big = nl == 1 && total_staged > A.stage;
      if (!big) {
        // ---- which pair each staged entry belongs to (lane-serial fill)
        if (lane < nl)
          for (int k = 0; k < cnt; ++k) st_l[start + k] = (uint8_t)lane;
        wave_sync();
        // ---- products of every staged entry, in parallel, four entries a
        // lane at a time: their column / value loads (first touches of the
        // blocks, HBM) issue together, then the column maps, then the stores
        for (int t0 = lane; t0 < total_staged; t0 += 4 * 64) {
          int col[4], moff[4];
          float v[4], wq[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int t = t0 + 64 * u;
            col[u] = 0;
            v[u] = 0.f;
            moff[u] = 0;
            wq[u] = 0.f;
            if (t < total_staged) {
              const int lo = st_l[t];
              const int64_t ent = l_e[lo] + (t - l_st[lo]);
              col[u] = l_tr[lo] ? A.tcols[ent] : A.cols[ent];
              v[u] = l_tr[lo] ? A.tvals[ent] : A.vals[ent];
              moff[u] = (int)A.map2_off[l_j[lo]];
              wq[u] = l_w[lo];
            }
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int t = t0 + 64 * u;
            if (t < total_staged) {
              const int c = A.map2[moff[u] + col[u]];
              st_c[t] = c;
              if (c >= c0 && c < c1) st_p[t] = wq[u] * v[u];  // posterior[id] += w * v
            }
          }
        }
        wave_sync();
        // ---- add them pair by pair: LDS float adds without return, which a
        // wave's LDS pipe applies in issue order (one pair's entries hit
        // distinct columns; a later pair's add to the same cell lands after)
        for (int l = 0; l < nl; ++l) {
          const int s0 = l_st[l], s1 = l_st[l + 1];
          for (int t = s0 + lane; t < s1; t += 64) {
            const int c = st_c[t];
            if (c >= c0 && c < c1) lds_add(&acc[c - c0], st_p[t]);
          }
        }
      } else {
        // ---- one row longer than the stage: add it piecewise, in order
        const int64_t e0 = l_e[0];
        const int n = total_staged, tr0 = l_tr[0];
        const float w = l_w[0];
        const int32_t* m2 = A.map2 + A.map2_off[l_j[0]];
        for (int t = lane; t < n; t += 64) {
          const int col = tr0 ? A.tcols[e0 + t] : A.cols[e0 + t];
          const float v = tr0 ? A.tvals[e0 + t] : A.vals[e0 + t];
          const int c = m2[col];
          if (c >= c0 && c < c1) acc[c - c0] = acc[c - c0] + w * v;
        }
      }
      wave_sync();
      q0 += nl;
    }
  }
  wave_sync();
  float* o = A.out + (int64_t)r * W2;
  for (int c = c0 + lane; c < c1; c += 64) o[c] = acc[c - c0];
}

// MEA of a dense (L1 + 1) x (L2 + 1) posterior (ProbabilisticModel.h:804-864,
// ChooseBestOfThree ScoreType.h:347-366; QuickProbs' computeAlignment is the
// same recurrence).  One workgroup (one wave) per strip of 64 rows: lane r
// holds row 64 s + r + 1 and is at column j = t - r at step t (a skewed
// wavefront).  up = the upper lane's value of the previous step (DPP wave
// shift; lane 0 takes the strip above's last row), diagonal = the previous
// step's up, left = the lane's own previous value: every cell adds and
// compares exactly as the serial loop does, so scores and choices are the
// reference's bit for bit.  The strips run on different CUs at once: strip
// s's last lane writes its row and, after every 16-step block, publishes
// how many columns of it are final; strip s + 1 waits for the columns its
// next block reads -- a pipeline with ~100 steps of lag per strip instead of
// one CU doing every strip.  The hand-off is the guide's sc1 form
// (MI355X_MICROARCH.md, "Valid forms"): the row is stored and loaded only
// with sc1 (relaxed agent-scope) accesses, the storing wave waits for its
// stores (vmcnt(0)) before the sc1 flag store, the reader polls the flag with
// sc1 loads -- no L2 write-back per block (an agent release) and no L1
// invalidate per poll (an acquire).
// Choices: 2 bits per cell (0 D, 1 L, 2 U), one uint32 per lane and block;
// the host traces back.  A strip that waits implausibly long sets the error
// word and returns (every wave reaches an exit; the host falls back).
__device__ __forceinline__ float mea_readlane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

MeaLayout mea_layout(int L1, int L2) {
  MeaLayout m;
  m.nstrips = (L1 + 63) / 64;
  m.nblk = (L2 + 63 + kMeaBlk - 1) / kMeaBlk;  // steps 1 .. L2 + 63
  m.rowpitch = (L2 + 1 + 63) & ~63;
  size_t o = 0;
  auto take = [&](size_t n) {
    const size_t at = o;
    o += (n + 255) & ~(size_t)255;
    return at;
  };
  m.o_tb = take((size_t)m.nstrips * m.nblk * 64 * 4);
  m.o_row = take((size_t)m.nstrips * m.rowpitch * 4);
  m.o_prog = take((size_t)m.nstrips * 4);
  m.o_score = take(4);
  m.o_err = take(4);
  m.bytes = o;
  return m;
}

__global__ __launch_bounds__(64) void k_profile_mea(MeaArgs A, MeaLayout M) {
  const int s = blockIdx.x, lane = threadIdx.x;
  const int L1 = A.L1, L2 = A.L2, W2 = L2 + 1;
  const int i = 64 * s + 1 + lane;
  const int nr = min(64, L1 - 64 * s);
  const float* prow = A.post + (int64_t)min(i, L1) * W2;
  float* rows = reinterpret_cast<float*>(A.work + M.o_row);
  const float* above = rows + (int64_t)(s > 0 ? s - 1 : 0) * M.rowpitch;
  float* below = rows + (int64_t)s * M.rowpitch;
  int* prog = reinterpret_cast<int*>(A.work + M.o_prog);
  int* err = reinterpret_cast<int*>(A.work + M.o_err);
  uint32_t* tbw = reinterpret_cast<uint32_t*>(A.work + M.o_tb) + (int64_t)s * M.nblk * 64;
  if (lane == 0) __hip_atomic_store(below, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  float v = 0.f, upp = 0.f;  // own value and up of the previous step
  float pv[kMeaBlk], pn[kMeaBlk];
#pragma unroll
  for (int u = 0; u < kMeaBlk; ++u) pv[u] = prow[min(max(1 + u - lane, 0), L2)];
  for (int b = 0; b < M.nblk; ++b) {
    const int t0 = kMeaBlk * b + 1;
    // the row above through column min(t0 + 15, L2)
    float ab = 0.f;
    if (s > 0) {
      const int need = min(t0 + kMeaBlk - 1, L2);
      int spins = 0;
      for (;;) {
        const int have = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(prog + s - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (have >= need) break;
        if (++spins > A.spin_limit) {  // ~seconds: give up (the host falls back)
          if (lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          return;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      // the poll matched: an agent-scope acquire orders the row loads below
      // after it (once per 16-step block, not per poll; the writer's release
      // is its s_waitcnt vmcnt(0) before the flag store)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      // lanes 0..15: above[t0 + u]; an sc1 load (L2), like every load of the handed-off row
      ab = __hip_atomic_load(above + min(t0 + lane, L2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the next block's posterior
#pragma unroll
    for (int u = 0; u < kMeaBlk; ++u) pn[u] = prow[min(max(t0 + kMeaBlk + u - lane, 0), L2)];
    uint32_t bits = 0;
#pragma unroll
    for (int u = 0; u < kMeaBlk; ++u) {
      const int j = t0 + u - lane;
      const float up = mlp_shr1(v, mea_readlane(ab, u));
      const float x1 = ((j >= 1 && j <= L2) ? pv[u] : 0.f) + upp, x2 = v, x3 = up;
      // ChooseBestOfThree's value is the largest of the three whichever it
      // picks (the values are non-negative sums: no NaN, no -0), so the step's
      // dependency chain is one max3; its pick (D, else L, else U) is off it
      float nv = fmaxf(fmaxf(x1, x2), x3);
      const uint32_t c = (x1 >= x2 && x1 >= x3) ? 0u : (x2 >= x3 ? 1u : 2u);
      nv = j >= 1 ? nv : 0.f;  // column 0 (and the lanes not started yet)
      bits |= c << (2 * u);
      if (lane == nr - 1 && j >= 1 && j <= L2) {
        __hip_atomic_store(below + j, nv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1 store
        if (s == M.nstrips - 1 && j == L2) *reinterpret_cast<float*>(A.work + M.o_score) = nv;
      }
      upp = up;
      v = nv;
    }
    tbw[(int64_t)b * 64 + lane] = bits;
#pragma unroll
    for (int u = 0; u < kMeaBlk; ++u) pv[u] = pn[u];
    // the last row is final through column t0 + 15 - (nr - 1): every store
    // of this wave has completed (in L2) before the sc1 flag store
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0)
      __hip_atomic_store(prog + s, min(L2, t0 + kMeaBlk - 1 - (nr - 1)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ __launch_bounds__(256) void k_profile_gather(const float* post, const int64_t* cells, int64_t n,
                                                       float* out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) out[k] = post[cells[k]];
}
hipError_t launch_profile_gather(const float* post, const int64_t* cells, int64_t n, float* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_profile_gather, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, post, cells, n, out);
  return hipGetLastError();
}

hipError_t launch_profile_mea(const MeaArgs& a, hipStream_t st) {
  if (a.L1 <= 0 || a.L2 <= 0) return hipSuccess;
  const MeaLayout m = mea_layout(a.L1, a.L2);
  hipError_t e = hipMemsetAsync(a.work + m.o_prog, 0, m.o_err + 4 - m.o_prog, st);  // progress, score, error
  if (e != hipSuccess) return e;
  // the handed-off rows start as NaN every launch: a read that ever got
  // ahead of its hand-off would poison the path's scores and show up in the
  // byte-identical tests instead of silently reusing the previous call's row
  e = hipMemsetAsync(a.work + m.o_row, 0xff, (size_t)m.nstrips * m.rowpitch * 4, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_profile_mea, dim3((unsigned)m.nstrips), dim3(64), 0, st, a, m);
  return hipGetLastError();
}

// inv1[i][map1_i[k]] = k: the column -> residue map of profile A, one
// thread per map entry (k = 0 entries skipped)
__global__ __launch_bounds__(256) void k_profile_inv(ProfileArgs A) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= A.map1_len) return;
  int lo = 0, hi = A.n1 - 1;  // the sequence whose map holds entry t
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (A.map1_off[mid] <= t) lo = mid; else hi = mid - 1;
  }
  const int k = (int)(t - A.map1_off[lo]);
  if (k > 0) A.inv1[(int64_t)lo * (A.L1 + 1) + A.map1[t]] = k;
}

hipError_t launch_profile_posterior(const ProfileArgs& a_in, hipStream_t st) {
  if (a_in.L1 <= 0) return hipSuccess;
  ProfileArgs a = a_in;
  // test hook: a smaller stage reaches the partial-run and long-row branches
  // with small profiles (MLP_PROFILE_STAGE, 1..kProfStage)
  a.stage = kProfStage;
  if (const char* e = getenv("MLP_PROFILE_STAGE")) a.stage = std::max(1, std::min(kProfStage, atoi(e)));
  hipLaunchKernelGGL(k_profile_inv, dim3((unsigned)((a.map1_len + 255) / 256)), dim3(256), 0, st, a);
  // column ranges per row: only rows too few to give every CU a wave are
  // split (at C3 refinement, one range per row measured fastest: 376 ms of
  // profile kernels against 393 / 466 ms for 2 / 4 ranges); ranges of at
  // least 64 columns (MLP_PROFILE_SPLIT overrides, for measurement)
  int k = (256 + a.L1 - 1) / a.L1;
  if (const char* e = getenv("MLP_PROFILE_SPLIT")) k = atoi(e);
  k = std::max(1, std::min(k, std::min(16, (a.L2 + 1 + 63) / 64)));
  const size_t lds = profile_lds_cols((a.L2 + 1 + k - 1) / k);
  (void)hipFuncSetAttribute((const void*)k_profile_post, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k_profile_post, dim3((unsigned)a.L1, (unsigned)k), dim3(64), lds, st, a);
  return hipGetLastError();
}

}  // namespace mlp
