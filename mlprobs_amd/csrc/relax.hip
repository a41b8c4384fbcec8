// relax.hip -- probabilistic-consistency relaxation for gfx950.
//
// Replaces MSA::DoRelaxation / Relax / Relax1 (CPNP/MSA.cpp:1172-1360):
//   P'_xy(i,j) = mask_xy( (2 P_xy(i,j) + sum_z sum_k P_xz(i,k) P_zy(k,j)) / N ),
// re-sparsified at 0.01 (CPNP/SparseMatrix.h:55-98).
//
// Bit-exactness: for one output cell the reference accumulates in the order
// z ascending, then k ascending (that is what Relax, Relax1 and the transpose
// branch all reduce to, CPNP/MSA.cpp:1219-1231), each term a rounded float
// product added to the running float sum.  Here one lane owns one output row
// i of one output pair and walks exactly that order, so every cell's sum is
// bit-identical; only the cells of the old sparsity pattern of P_xy are
// accumulated (all others are masked to zero by the reference anyway).
//
// Orientation: A_z = P(x, z) and B_z = P(z, y).  Blocks are stored for a < b
// only, so A_z for z < x and B_z for z > y come from the transposed blocks,
// built stably (row order preserved, like SparseMatrix::ComputeTranspose,
// CPNP/SparseMatrix.h:205-248) by k_transpose.
#include "mlp_kernels.h"
#include "mlp_numerics.h"

namespace mlp {

__device__ __forceinline__ int64_t pair_index(int n, int a, int b) {  // a < b
  return (int64_t)a * n - (int64_t)a * (a + 1) / 2 + (b - a - 1);
}


// One lane per output row.  Accumulators live in `out` at the positions of
// the row's input entries (their column list is the output mask).
__global__ __launch_bounds__(256) void k_relax(RelaxArgs A) {
  const int64_t task = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (task >= A.ntasks) return;
  const int lane = threadIdx.x & 63;
  const int64_t p = A.task_pair[task];
  // recover (x, y) from p
  const int n = A.n;
  int x = 0;
  int64_t q = p;
  while (q >= n - 1 - x) { q -= n - 1 - x; ++x; }
  const int y = x + 1 + (int)q;
  const int Lx = A.lens[x];
  const int i = A.task_row0[task] + lane;
  if (i > Lx) return;
  const int32_t* rpxy = A.rowptr + A.rp_off[p];
  const int64_t exy = A.ent_off[p];
  const int mb = rpxy[i], me = rpxy[i + 1];
  if (mb == me) return;
  const uint16_t* mcol = A.cols + exy;
  float* acc = A.out + exy;
  for (int e = mb; e < me; ++e) {
    const float v = A.vals[exy + e];
    acc[e] = v + v;  // contribution of z = x and z = y (CPNP/MSA.cpp:1211-1213)
  }
  for (int z = 0; z < n; ++z) {
    if (z == x || z == y) continue;
    // A_z row i
    const uint16_t* acol;
    const float* aval;
    int ab, ae;
    if (z > x) {
      const int64_t pz = pair_index(n, x, z);
      const int32_t* rp = A.rowptr + A.rp_off[pz];
      ab = rp[i]; ae = rp[i + 1];
      acol = A.cols + A.ent_off[pz];
      aval = A.vals + A.ent_off[pz];
    } else {
      const int64_t pz = pair_index(n, z, x);
      const int32_t* rp = A.trowptr + A.trp_off[pz];
      ab = rp[i]; ae = rp[i + 1];
      acol = A.tcols + A.ent_off[pz];
      aval = A.tvals + A.ent_off[pz];
    }
    if (ab == ae) continue;
    // B_z rows
    const int32_t* brp;
    const uint16_t* bcol;
    const float* bval;
    if (z < y) {
      const int64_t pz = pair_index(n, z, y);
      brp = A.rowptr + A.rp_off[pz];
      bcol = A.cols + A.ent_off[pz];
      bval = A.vals + A.ent_off[pz];
    } else {
      const int64_t pz = pair_index(n, y, z);
      brp = A.trowptr + A.trp_off[pz];
      bcol = A.tcols + A.ent_off[pz];
      bval = A.tvals + A.ent_off[pz];
    }
    for (int u = ab; u < ae; ++u) {
      const int k = acol[u];
      const float av = aval[u];
      int bb = brp[k];
      const int be = brp[k + 1];
      int s = mb;
      int ms = mcol[s];
      // merge-join the sorted B row with the sorted mask row
      for (; bb < be; ++bb) {
        const int jc = bcol[bb];
        while (ms < jc) {
          if (++s == me) break;
          ms = mcol[s];
        }
        if (s == me) break;
        if (ms == jc) acc[s] += av * bval[bb];
      }
    }
  }
  const float fn = (float)n;
  for (int e = mb; e < me; ++e) acc[e] = acc[e] / fn;  // CPNP/MSA.cpp:1233-1235
}

// Stable CSR transpose of one block per wave (rows processed in order, the
// entries of one row have distinct columns, so LDS cursors never collide).

__global__ __launch_bounds__(64) void k_transpose(TransposeArgs A) {
  extern __shared__ int32_t cur[];
  if ((int64_t)blockIdx.x >= A.npairs) return;
  const int64_t p = A.pairs[blockIdx.x];
  const int lane = threadIdx.x;
  const int n = A.n;
  int a = 0;
  int64_t q = p;
  while (q >= n - 1 - a) { q -= n - 1 - a; ++a; }
  const int b = a + 1 + (int)q;
  const int La = A.lens[a], Lb = A.lens[b];
  const int32_t* rp = A.rowptr + A.rp_off[p];
  const uint16_t* cols = A.cols + A.ent_off[p];
  const float* vals = A.vals + A.ent_off[p];
  int32_t* trp = A.trowptr + A.trp_off[p];
  uint16_t* tc = A.tcols + A.ent_off[p];
  float* tv = A.tvals + A.ent_off[p];
  for (int r = lane; r <= Lb + 1; r += 64) cur[r] = 0;
  __syncthreads();
  const int nnz = rp[La + 1];
  for (int e = lane; e < nnz; e += 64) atomicAdd(&cur[cols[e] + 1], 1);
  __syncthreads();
  // exclusive scan over rows 0..Lb+1 -> trp[r] = start of transposed row r
  int run = 0;
  for (int r0 = 0; r0 <= Lb + 1; r0 += 64) {
    const int r = r0 + lane;
    const int c = (r <= Lb + 1) ? cur[r] : 0;
    int xs = c;
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(xs, off);
      if (lane >= off) xs += y;
    }
    if (r <= Lb + 1) {  // inclusive over shifted counts = start of row r
      trp[r] = run + xs;
      cur[r] = run + xs;
    }
    run += __shfl(xs, 63);
  }
  __syncthreads();
  // scatter rows in order; entries within a row have distinct columns
  for (int i = 1; i <= La; ++i) {
    const int rb = rp[i], re = rp[i + 1];
    for (int e = rb + lane; e < re; e += 64) {
      const int c = cols[e];
      const int pos = cur[c];
      cur[c] = pos + 1;
      tc[pos] = (uint16_t)i;
      tv[pos] = vals[e];
    }
    __syncthreads();
  }
}

// Threshold + compaction of relaxed values (CPNP/SparseMatrix.h:55-98 with
// the mask of CPNP/MSA.cpp:1237-1261 already applied by construction).

__global__ __launch_bounds__(256) void k_filter(FilterArgs A) {
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= A.npairs) return;
  const int64_t p = A.pairs[w];
  const int lane = threadIdx.x & 63;
  const int n = A.n;
  int a = 0;
  int64_t q = p;
  while (q >= n - 1 - a) { q -= n - 1 - a; ++a; }
  const int La = A.lens[a];
  const int32_t* rp = A.rowptr + A.rp_off[p];
  const int64_t eo = A.ent_off[p];
  int32_t* nrp = A.new_rowptr + A.rp_off[p];
  const int64_t neo = A.write ? A.new_ent_off[p] : 0;
  int64_t run = 0;
  if (A.write && lane == 0) { nrp[0] = 0; nrp[1] = 0; }
  for (int r0 = 1; r0 <= La; r0 += 64) {
    const int i = r0 + lane;
    int c = 0;
    int rb = 0, re = 0;
    if (i <= La) {
      rb = rp[i]; re = rp[i + 1];
      for (int e = rb; e < re; ++e) c += (A.raw[eo + e] >= 0.01f) ? 1 : 0;
    }
    int xs = c;
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(xs, off);
      if (lane >= off) xs += y;
    }
    if (A.write && i <= La) {
      int pos = (int)run + xs - c;
      nrp[i + 1] = pos + c;
      for (int e = rb; e < re; ++e) {
        const float v = A.raw[eo + e];
        if (v >= 0.01f) {
          A.new_cols[neo + pos] = A.cols[eo + e];
          A.new_vals[neo + pos] = v;
          ++pos;
        }
      }
    }
    run += __shfl(xs, 63);
  }
  if (!A.write && lane == 0) A.pair_nnz[p] = run;
}

hipError_t launch_transpose(const TransposeArgs& a, hipStream_t st) {
  if (a.npairs <= 0) return hipSuccess;
  const size_t lds = sizeof(int32_t) * (size_t)(a.max_len + 2);
  hipLaunchKernelGGL(k_transpose, dim3((unsigned)a.npairs), dim3(64), lds, st, a);
  return hipGetLastError();
}
hipError_t launch_relax_tasks(const RelaxArgs& a, hipStream_t st) {
  if (a.ntasks <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_relax, dim3((unsigned)((a.ntasks + 3) / 4)), dim3(256), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_filter(const FilterArgs& a, hipStream_t st) {
  if (a.npairs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_filter, dim3((unsigned)((a.npairs + 3) / 4)), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace mlp
