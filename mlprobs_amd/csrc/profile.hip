// profile.hip -- the weighted profile-profile posterior of QuickProbs'
// progressive construction and refinement (ParallelProbabilisticModel::
// buildPosterior, QP/Alignment/Multiple/ParallelProbabilisticModel.cpp:301-430)
// from the device-resident sparse set.
//
// posterior[r][c] accumulates w_ij * P_ij(ii, jj) over the sequence pairs
// (i in profile A, j in profile B) where sequence i has residue ii in column r
// and j has jj in column c, in the reference's order: i, then j, then the row
// ii of block (i, j), then its entries.  One wave owns one dense row r and
// keeps it in LDS; for a run of up to 64 j's it loads the rows' extents (one
// lane per j), computes the products of all their entries in parallel into an
// LDS stage, and then adds the stage into the row one j after another.  The
// entries of one row hit distinct columns, so each j's adds are one parallel
// step, and a wave's LDS operations retire in order: every cell sees its
// terms in the reference's sequence, with the reference's float operations
// (w * v, then +=).
#include "mlp_kernels.h"

namespace mlp {

constexpr int kProfStage = 2048;  // staged entries per run of j's

// LDS writes of some lanes made visible to the other lanes of the wave
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

static __host__ __device__ inline size_t prof_acc_bytes(int L2) { return ((size_t)(L2 + 1) * 4 + 15) & ~(size_t)15; }
size_t profile_lds(int L2) { return prof_acc_bytes(L2) + (size_t)kProfStage * 8 + 3 * 65 * 8; }

__global__ __launch_bounds__(64) void k_profile_post(ProfileArgs A) {
  extern __shared__ __align__(16) uint8_t lds[];
  float* acc = (float*)lds;                                     // L2 + 1
  int32_t* st_c = (int32_t*)(lds + prof_acc_bytes(A.L2));      // staged dense columns
  float* st_p = (float*)(st_c + kProfStage);                    // staged products
  int64_t* l_e = (int64_t*)(st_p + kProfStage);                 // per lane: first entry (absolute)
  int32_t* l_st = (int32_t*)(l_e + 65);                         // per lane: stage start (prefix), [64] = total
  int32_t* l_tr = l_st + 65;                                    // per lane: transposed block
  const int lane = threadIdx.x;
  const int r = blockIdx.x + 1;
  const int W2 = A.L2 + 1;
  for (int c = lane; c < W2; c += 64) acc[c] = 0.f;
  for (int i = 0; i < A.n1; ++i) {
    const int ii = __builtin_amdgcn_readfirstlane(A.inv1[(int64_t)i * (A.L1 + 1) + r]);
    if (ii == 0) continue;  // sequence i has a gap in column r
    for (int j0 = 0; j0 < A.n2;) {
      // ---- extents of the rows ii of blocks (i, j0 + lane)
      const int j = j0 + lane;
      int cnt = 0;
      int64_t e = 0;
      int tr = 0;
      if (j < A.n2) {
        const int64_t q = (int64_t)i * A.n2 + j;
        const int64_t rb = A.rpb[q];
        tr = rb < 0;
        const int32_t* rp = tr ? A.trowptr + (~rb) : A.rowptr + rb;
        const int b = rp[ii];
        cnt = rp[ii + 1] - b;
        e = A.eb[q] + b;
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
      const bool fits = x <= kProfStage || lane == 0;
      const unsigned long long fitm = __ballot(fits && j < A.n2);
      const int nl = __popcll(~fitm) ? __builtin_ctzll(~fitm) : 64;
      l_e[lane] = e;
      l_st[lane] = start;
      l_tr[lane] = tr;
      if (lane == 63) l_st[64] = x;
      wave_sync();
      const int total_staged = l_st[nl];  // entries of lanes 0 .. nl-1
      const bool big = nl == 1 && total_staged > kProfStage;
      if (!big) {
        // ---- products of every staged entry, in parallel
        for (int t = lane; t < total_staged; t += 64) {
          int lo = 0, hi = nl - 1;  // last lane l with l_st[l] <= t
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (l_st[mid] <= t) lo = mid; else hi = mid - 1;
          }
          const int64_t ent = l_e[lo] + (t - l_st[lo]);
          const int col = l_tr[lo] ? A.tcols[ent] : A.cols[ent];
          const float v = l_tr[lo] ? A.tvals[ent] : A.vals[ent];
          const int jj = j0 + lo;
          st_c[t] = A.map2[A.map2_off[jj] + col];
          st_p[t] = A.w[(int64_t)i * A.n2 + jj] * v;  // posterior[id] += w * v
        }
        wave_sync();
        // ---- add them j by j (a wave's LDS operations retire in order)
        for (int l = 0; l < nl; ++l) {
          const int s0 = l_st[l], s1 = l_st[l + 1];
          for (int t = s0 + lane; t < s1; t += 64) {
            const int c = st_c[t];
            acc[c] = acc[c] + st_p[t];
          }
        }
      } else {
        // ---- one row longer than the stage: add it piecewise, in order
        const int64_t e0 = l_e[0];
        const int n = total_staged, tr0 = l_tr[0];
        const float w = A.w[(int64_t)i * A.n2 + j0];
        const int32_t* m2 = A.map2 + A.map2_off[j0];
        for (int t = lane; t < n; t += 64) {
          const int col = tr0 ? A.tcols[e0 + t] : A.cols[e0 + t];
          const float v = tr0 ? A.tvals[e0 + t] : A.vals[e0 + t];
          const int c = m2[col];
          acc[c] = acc[c] + w * v;
        }
      }
      wave_sync();
      j0 += nl;
    }
  }
  wave_sync();
  float* o = A.out + (int64_t)r * W2;
  for (int c = lane; c < W2; c += 64) o[c] = acc[c];
}

hipError_t launch_profile_posterior(const ProfileArgs& a, hipStream_t st) {
  if (a.L1 <= 0) return hipSuccess;
  const size_t lds = profile_lds(a.L2);
  hipFuncSetAttribute((const void*)k_profile_post, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k_profile_post, dim3((unsigned)a.L1), dim3(64), lds, st, a);
  return hipGetLastError();
}

}  // namespace mlp
