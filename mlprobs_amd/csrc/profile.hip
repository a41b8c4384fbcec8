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
        // distinct columns; a later pair's add to the same cell lands after).
        // Eight pairs at a time: their entries' column / product reads issue
        // together, then the eight adds in pair order (the reads touch other
        // arrays than the adds), one LDS round trip per eight pairs instead of
        // three per pair; a pair of more than 64 entries (a transposed row)
        // takes the group through the entry loop
        for (int l0 = 0; l0 < nl; l0 += 8) {
          int n8 = 0;
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (l0 + u < nl) n8 = max(n8, __builtin_amdgcn_readlane(cnt, l0 + u));
          if (n8 <= 64) {
            int cc[8];
            float pp[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              cc[u] = -1;
              pp[u] = 0.f;
              if (l0 + u < nl && lane < __builtin_amdgcn_readlane(cnt, l0 + u)) {
                const int t = __builtin_amdgcn_readlane(start, l0 + u) + lane;
                cc[u] = st_c[t];
                pp[u] = st_p[t];
              }
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
              if (cc[u] >= c0 && cc[u] < c1) lds_add(&acc[cc[u] - c0], pp[u]);
          } else {
            for (int l = l0; l < min(nl, l0 + 8); ++l) {
              const int s0 = l_st[l], s1 = l_st[l + 1];
              for (int t = s0 + lane; t < s1; t += 64) {
                const int c = st_c[t];
                if (c >= c0 && c < c1) lds_add(&acc[c - c0], st_p[t]);
              }
            }
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
// reference's bit for bit.  The strips run on different CUs at once, a
// pipeline: strip s's last lane stores each value of its row as it is final
// (relaxed agent-scope stores, sc1); strip s + 1 polls the columns it needs
// next with relaxed agent-scope loads of the values themselves, 64 at a time.
// The rows are NaN-filled before every launch and a value is never NaN
// (non-negative sums), so a column is final once it reads as a number: no
// progress flag, no release wait on the writer, no acquire on the reader,
// and one poll serves up to four 16-step blocks.  (Round 4's form -- a flag
// per block behind a vmcnt(0) store drain and an acquire -- spent ~2 us a
// block in those waits: 0.30 ms for a one-strip L2 = 2000 MEA.)
// Choices: 2 bits per cell (bit 0: D is the largest; bit 1: L >= U), one
// uint32 per lane and block; the host decodes D, else L, else U and traces
// back.  A strip that waits implausibly long sets the error
// word and returns (every wave reaches an exit; the host falls back).

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
  m.o_score = take(4);
  m.o_err = take(4);
  m.bytes = o;
  return m;
}

// a lane's 16 posterior values of a block: row-contiguous columns c0 ..
// c0 + 15, four 16-byte loads (dword-aligned).  The dense posterior has
// kMeaGuard readable bytes before and after it, so a window that reaches past
// the row (a strip's first and last blocks, rows of fewer than 63 columns)
// still reads inside the buffer; mea_mask then zeroes the columns outside
// 1 .. L2 (the recurrence starts at column 1, ProbabilisticModel.h:821-823).
typedef float mea_f4 __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ void mea_window(float (&p)[kMeaBlk], const float* prow, int c0) {
#pragma unroll
  for (int q = 0; q < kMeaBlk / 4; ++q) {
    const mea_f4 x = *(const mea_f4*)(prow + c0 + 4 * q);
    p[4 * q] = x.x;
    p[4 * q + 1] = x.y;
    p[4 * q + 2] = x.z;
    p[4 * q + 3] = x.w;
  }
}
__device__ __forceinline__ void mea_mask(float (&p)[kMeaBlk], int c0, int L2) {
#pragma unroll
  for (int u = 0; u < kMeaBlk; ++u) p[u] = (c0 + u >= 1 && c0 + u <= L2) ? p[u] : 0.f;
}

// One 16-step block of strip s (see above); false: the strip gave up waiting.
struct MeaStrip {
  const float* prow;
  const float* above;
  float* below;
  uint32_t* tbw;
  int* err;
  float* score;  // the last strip's, else null
  int L2, nr, lane, spin_limit;
  float v, upp, ch;  // own value and up of the previous step; the row above: lane k of ch holds column t0 + k
  int have;          // columns .. have of the row above are final
};
__device__ __forceinline__ bool mea_block(MeaStrip& S, float (&p)[kMeaBlk], int b) {
  const int lane = S.lane, L2 = S.L2;
  const int t0 = kMeaBlk * b + 1;
  // (wave-uniform: edge blocks) the block's columns run from t0 - 63 (lane 63,
  // first step) to t0 + kMeaBlk - 1 (lane 0, last step)
  if (t0 - 63 < 1 || t0 + kMeaBlk - 1 > L2) mea_mask(p, t0 - lane, L2);
  const int need = min(t0 + kMeaBlk - 1, L2);
  if (need > S.have) {  // (wave-uniform) poll the next 64 columns of the row above
    int spins = 0;
    for (;;) {
      const float x = __hip_atomic_load(S.above + min(t0 + lane, L2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long nan = __ballot(x != x);
      const int ready = nan ? __builtin_ctzll(nan) : 64;  // a prefix of the lanes (the row fills in order)
      S.have = min(t0 + ready - 1, L2);
      if (S.have >= need) {
        S.ch = x;
        break;
      }
      if (++spins > S.spin_limit) {  // ~seconds: give up (the host falls back)
        if (lane == 0) __hip_atomic_store(S.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  // the block's 16 steps: a dependency chain of one wave shift and one max3
  // per step (ChooseBestOfThree's value is the largest of the three
  // whichever it picks: the values are non-negative sums, no NaN, no -0; its
  // pick, D else L else U, is off the chain).  A lane whose column is 0 or
  // less (not started) gets 0 without a select: its inputs are all 0 (the
  // posterior window reads 0 there, and the row above at column <= 0 is 0
  // by the same argument; lane 0 is always at a column >= 1).
  uint32_t bits = 0;
  float rv[kMeaBlk];
  // The row above enters lane 0 through the wave shift's `old` operand from
  // ch, which shifts one lane down a step (off the chain; no readlane).
  float v = S.v, upp = S.upp, ch = S.ch;
#pragma unroll
  for (int u = 0; u < kMeaBlk; ++u) {
    const float up = mlp_shr1(v, ch);
    ch = mlp_shl1z(ch);
    const float x1 = p[u] + upp;
    const float nv = fmaxf(fmaxf(x1, v), up);
    // the pick as two flags, x1 the largest (D) and v >= up (L over U); the
    // host decodes D, else L, else U
    bits |= (x1 == nv ? 1u : 0u) << (2 * u) | (v >= up ? 2u : 0u) << (2 * u);
    rv[u] = nv;
    upp = up;
    v = nv;
  }
  S.v = v;
  S.upp = upp;
  S.ch = ch;
  // the last row, columns t0 - (nr - 1) .. + 15: sc1 stores the next strip
  // polls directly (no flag, no wait: a column is final once it is not NaN)
  // (columns outside 1 .. L2 go to column 0, which no strip reads: one
  // branch for the 16 stores instead of one per store)
  const int j0 = t0 - (S.nr - 1);
  if (lane == S.nr - 1) {
    if (j0 >= 1 && j0 + kMeaBlk - 1 <= L2) {  // (wave-uniform) inside the row: immediate offsets
#pragma unroll
      for (int u = 0; u < kMeaBlk; ++u)
        __hip_atomic_store(S.below + j0 + u, rv[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
#pragma unroll
      for (int u = 0; u < kMeaBlk; ++u) {
        const int j = j0 + u;
        __hip_atomic_store(S.below + ((j >= 1 && j <= L2) ? j : 0), rv[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (S.score && j0 <= L2 && L2 < j0 + kMeaBlk) {  // the score: cell (L1, L2)
      float sc = 0.f;
#pragma unroll
      for (int u = 0; u < kMeaBlk; ++u) sc = j0 + u == L2 ? rv[u] : sc;
      *S.score = sc;
    }
  }
  S.tbw[(int64_t)b * 64 + lane] = bits;
  return true;
}

// The posterior windows are loaded four blocks (64 steps) ahead into two
// register sets in turn, so a load has a whole 64-step super-block to land
// (one block ahead exposed its ~1 us L2 latency every 16 steps); the window
// of a block past the strip's end re-reads the last block (no branch around
// the loads, whose waits the compiler then counts exactly).
__global__ __launch_bounds__(64) void k_profile_mea(MeaArgs A, MeaLayout M) {
  const int s = blockIdx.x, lane = threadIdx.x;
  const int L1 = A.L1, L2 = A.L2, W2 = L2 + 1;
  const int i = 64 * s + 1 + lane;
  float* rows = reinterpret_cast<float*>(A.work + M.o_row);
  MeaStrip S;
  S.prow = A.post + (int64_t)min(i, L1) * W2;
  S.above = rows + (int64_t)(s > 0 ? s - 1 : 0) * M.rowpitch;
  S.below = rows + (int64_t)s * M.rowpitch;
  S.tbw = reinterpret_cast<uint32_t*>(A.work + M.o_tb) + (int64_t)s * M.nblk * 64;
  S.err = reinterpret_cast<int*>(A.work + M.o_err);
  S.score = s == M.nstrips - 1 ? reinterpret_cast<float*>(A.work + M.o_score) : nullptr;
  S.L2 = L2;
  S.nr = min(64, L1 - 64 * s);
  S.lane = lane;
  S.spin_limit = A.spin_limit;
  S.v = S.upp = S.ch = 0.f;
  S.have = s > 0 ? 0 : L2;
  const int nb = M.nblk;
  float PA[4][kMeaBlk], PB[4][kMeaBlk];
#pragma unroll
  for (int q = 0; q < 4; ++q) mea_window(PA[q], S.prow, kMeaBlk * min(q, nb - 1) + 1 - lane);
  for (int b0 = 0; b0 < nb; b0 += 8) {
#pragma unroll
    for (int q = 0; q < 4; ++q) mea_window(PB[q], S.prow, kMeaBlk * min(b0 + 4 + q, nb - 1) + 1 - lane);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (b0 + q < nb && !mea_block(S, PA[q], b0 + q)) return;
#pragma unroll
    for (int q = 0; q < 4; ++q) mea_window(PA[q], S.prow, kMeaBlk * min(b0 + 8 + q, nb - 1) + 1 - lane);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (b0 + 4 + q < nb && !mea_block(S, PB[q], b0 + 4 + q)) return;
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
  hipError_t e = hipMemsetAsync(a.work + m.o_score, 0, m.o_err + 4 - m.o_score, st);  // score, error
  if (e != hipSuccess) return e;
  // the handed-off rows start as NaN every launch: a column is final once it
  // reads as a number (the next strip polls the values themselves)
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
  // with small profiles (MLP_TEST_PROFILE_STAGE, 1..kProfStage)
  a.stage = std::max(1, std::min(kProfStage, (int)knob("MLP_TEST_PROFILE_STAGE", kProfStage)));
  hipLaunchKernelGGL(k_profile_inv, dim3((unsigned)((a.map1_len + 255) / 256)), dim3(256), 0, st, a);
  // column ranges per row: only rows too few to give every CU a wave are
  // split (at C3 refinement, one range per row measured fastest: 376 ms of
  // profile kernels against 393 / 466 ms for 2 / 4 ranges); ranges of at
  // least 64 columns (MLP_TEST_PROFILE_SPLIT overrides, for measurement)
  int k = (int)knob("MLP_TEST_PROFILE_SPLIT", (256 + a.L1 - 1) / a.L1);
  k = std::max(1, std::min(k, std::min(16, (a.L2 + 1 + 63) / 64)));
  const size_t lds = profile_lds_cols((a.L2 + 1 + k - 1) / k);
  (void)hipFuncSetAttribute((const void*)k_profile_post, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k_profile_post, dim3((unsigned)a.L1, (unsigned)k), dim3(64), lds, st, a);
  return hipGetLastError();
}

}  // namespace mlp
