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

// ------------------------------------------------------------ block images
// One wave per image: copy the block (or its transpose) into the packed
// layout of mlp_kernels.h (img_ent_off / img_bytes).
__global__ __launch_bounds__(256) void k_pack(PackArgs A) {
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= A.nimg) return;
  const int lane = threadIdx.x & 63;
  const int64_t p = q >> 1;
  const bool tr = q & 1;
  const int n = A.n;
  int a = 0;
  int64_t r = p;
  while (r >= n - 1 - a) { r -= n - 1 - a; ++a; }
  const int b = a + 1 + (int)r;
  const int rows = tr ? A.lens[b] : A.lens[a];
  const int64_t e0 = A.ent_off[p];
  const int64_t nnz = A.ent_off[p + 1] - e0;
  const int32_t* rp = tr ? A.trowptr + A.trp_off[p] : A.rowptr + A.rp_off[p];
  const uint16_t* cols = (tr ? A.tcols : A.cols) + e0;
  const float* vals = (tr ? A.tvals : A.vals) + e0;
  uint8_t* dst = A.img + A.img_off[q];
  uint16_t* drp = (uint16_t*)dst;
  uint2* dent = (uint2*)(dst + img_ent_off(rows));
  const uint32_t wstride = (uint32_t)A.threads * 8;
  for (int k = lane; k < rows + 2; k += 64) drp[k] = (uint16_t)rp[k];
  for (int64_t e = lane; e < nnz; e += 64) {
    const uint32_t c = cols[e];
    dent[e] = make_uint2(c | (((c >> 5) * wstride) << 10), __float_as_uint(vals[e]));
  }
}

// ------------------------------------------------- pair-resident relaxation
// One workgroup per output pair (x, y), one thread per row i of x.  For each
// z (ascending) the workgroup stages A_z = P(x, z) and B_z = P(z, y) as block
// images in LDS (the next z's images are prefetched into registers while the
// current z is computed), and thread i walks A_z row i (k ascending) and each
// B_z row k, adding a * b into the accumulator of output cell (i, j) when
// (i, j) is in the mask (the pattern of P_xy, CPNP/MSA.cpp:1237-1261).  The
// per-cell order is therefore z ascending, then k ascending -- the order of
// Relax / Relax1 (CPNP/MSA.cpp:1276-1350) -- and every sum is bit-identical
// (the adds are ds_add_f32, IEEE round-to-nearest like the host's float +=;
// one lane's LDS operations complete in issue order).
//
// The mask of row i is a bitmap over j, one 64-bit element per 32 columns:
// low half the bits, high half the accumulator slot of the word's first set
// bit; word-major (word w of thread t at w * threads + t), so a wave's mask
// reads never share a bank.  A hit's slot is that base plus the popcount of
// the lower bits.  Accumulators are the pair's entry slots, in LDS.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // plain vector: stays in VGPRs

size_t pair_relax_lds(int threads, int img_cap, int mask_words, int acc_cap) {
  return 2 * (size_t)img_cap + (size_t)mask_words * threads * 8 + 4 * (size_t)acc_cap;
}

int pair_relax_prefetch(int threads, int img_cap) {
  const int chunks = (img_cap / 16 + threads - 1) / threads;
  for (int kp : {1, 2, 4, 8, 16})
    if (chunks <= kp) return kp;
  return 0;
}

template <int KP>
__global__ __launch_bounds__(1024) void k_relax_pair(PairRelaxArgs A) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int nt = blockDim.x;
  const int tid = threadIdx.x;
  const int64_t p = A.pairs[blockIdx.x];
  const int n = A.n;
  const int64_t exy = A.ent_off[p];
  const int64_t nxy = A.ent_off[p + 1] - exy;
  if (nxy == 0) return;  // empty mask: nothing survives
  int x = 0;
  int64_t q = p;
  while (q >= n - 1 - x) { q -= n - 1 - x; ++x; }
  const int y = x + 1 + (int)q;
  const int Lx = A.lens[x];
  const int mw = A.mask_words;
  uint8_t* sA = lds;
  uint8_t* sB = lds + A.img_cap;
  uint2* mask = (uint2*)(lds + 2 * A.img_cap);
  float* acc = (float*)(mask + (size_t)mw * nt);

  // mask bitmap, slot bases and the z = x, z = y term (CPNP/MSA.cpp:1211-1213)
  const int i = tid + 1;
  const int32_t* rpxy = A.rowptr + A.rp_off[p];
  int mb = 0, me = 0;
  if (i <= Lx) { mb = rpxy[i]; me = rpxy[i + 1]; }
  for (int w = 0; w < mw; ++w) mask[w * nt + tid].x = 0;
  for (int e = mb; e < me; ++e) {
    const int j = A.cols[exy + e];
    mask[(j >> 5) * nt + tid].x |= 1u << (j & 31);
    const float v = A.vals[exy + e];
    acc[e] = v + v;
  }
  {
    int run = mb;
    for (int w = 0; w < mw; ++w) {
      mask[w * nt + tid].y = (uint32_t)run;
      run += __popc(mask[w * nt + tid].x);
    }
  }
  const bool active = me > mb;
  const uint8_t* mbase = (const uint8_t*)mask + tid * 8;

  // images of A_z = P(x, z) and B_z = P(z, y); false when either is empty
  auto images = [&](int z, int64_t& qa, int64_t& qb) -> bool {
    int64_t pa, pb;
    if (z > x) { pa = pair_index(n, x, z); qa = 2 * pa; } else { pa = pair_index(n, z, x); qa = 2 * pa + 1; }
    if (z < y) { pb = pair_index(n, z, y); qb = 2 * pb; } else { pb = pair_index(n, y, z); qb = 2 * pb + 1; }
    return A.ent_off[pa + 1] > A.ent_off[pa] && A.ent_off[pb + 1] > A.ent_off[pb];
  };
  auto next_z = [&](int z, int64_t& qa, int64_t& qb) -> int {
    for (++z; z < n; ++z)
      if (z != x && z != y && images(z, qa, qb)) return z;
    return n;
  };
  // register prefetch of the next z's images (written out, not in lambdas:
  // arrays captured by reference end up in scratch)
  u32x4 ra[KP], rb[KP];
  int na = 0, nb = 0;  // 16-byte chunks of the prefetched images
  int64_t qa, qb;
  int z = next_z(-1, qa, qb);
  int Lz_next = z < n ? A.lens[z] : 0;
#define MLP_ISSUE()                                                          \
  {                                                                          \
    const u32x4* ga = (const u32x4*)(A.img + A.img_off[qa]);                 \
    const u32x4* gb = (const u32x4*)(A.img + A.img_off[qb]);                 \
    na = (int)((A.img_off[qa + 1] - A.img_off[qa]) >> 4);                    \
    nb = (int)((A.img_off[qb + 1] - A.img_off[qb]) >> 4);                    \
    _Pragma("unroll") for (int m = 0; m < KP; ++m) {                         \
      const int c = tid + m * nt;                                            \
      ra[m] = ga[min(c, na - 1)];                                            \
      rb[m] = gb[min(c, nb - 1)];                                            \
    }                                                                        \
  }
  if (z < n) MLP_ISSUE();
  while (z < n) {
#pragma unroll
    for (int m = 0; m < KP; ++m) {
      const int c = tid + m * nt;
      if (c < na) ((u32x4*)sA)[c] = ra[m];
      if (c < nb) ((u32x4*)sB)[c] = rb[m];
    }
    __syncthreads();
    const int Lz = Lz_next;
    z = next_z(z, qa, qb);
    Lz_next = z < n ? A.lens[z] : 0;
    if (z < n) MLP_ISSUE();
#ifdef MLP_RELAX_NOCOMPUTE
    if (false) {
#else
    if (active) {
#endif
      const uint16_t* Arp = (const uint16_t*)sA;
      const uint2* Aent = (const uint2*)(sA + img_ent_off(Lx));
      const uint16_t* Brp = (const uint16_t*)sB;
      const uint2* Bent = (const uint2*)(sB + img_ent_off(Lz));
      const int a0 = Arp[i], a1 = Arp[i + 1];
      for (int t = a0; t < a1; ++t) {
        const uint2 ea = Aent[t];
        const int k = ea.x & 1023;
        const float av = __uint_as_float(ea.y);
        const int b0 = Brp[k], b1 = Brp[k + 1];
        // four entries of B_z row k at a time: distinct columns, so their
        // updates are independent; the groups stay in k order
        for (int u = b0; u < b1; u += 4) {
          uint2 eb[4], mk[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) eb[g] = Bent[min(u + g, b1 - 1)];
#pragma unroll
          for (int g = 0; g < 4; ++g) mk[g] = *(const uint2*)(mbase + (eb[g].x >> 10));
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const uint32_t sh = eb[g].x & 31;
            if (u + g < b1 && ((mk[g].x >> sh) & 1u)) {
              const uint32_t slot = mk[g].y + __popc(mk[g].x & ((1u << sh) - 1u));
              __hip_atomic_fetch_add(acc + slot, av * __uint_as_float(eb[g].y), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_WORKGROUP);
            }
          }
        }
      }
    }
    __syncthreads();
  }
#undef MLP_ISSUE
  const float fn = (float)n;
  for (int e = mb; e < me; ++e) A.out[exy + e] = acc[e] / fn;  // CPNP/MSA.cpp:1233-1235
}

hipError_t launch_pack(const PackArgs& a, hipStream_t st) {
  if (a.nimg <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pack, dim3((unsigned)((a.nimg + 3) / 4)), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_relax_pairs(const PairRelaxArgs& a, int threads, hipStream_t st) {
  if (a.npairs <= 0) return hipSuccess;
  const size_t lds = pair_relax_lds(threads, a.img_cap, a.mask_words, a.acc_cap);
  const int kp = pair_relax_prefetch(threads, a.img_cap);
  const dim3 grid((unsigned)a.npairs), block((unsigned)threads);
  switch (kp) {
#define MLP_RELAX_CASE(K)                                                                    \
  case K:                                                                                    \
    hipFuncSetAttribute((const void*)k_relax_pair<K>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                        (int)lds);                                                           \
    hipLaunchKernelGGL(k_relax_pair<K>, grid, block, lds, st, a);                            \
    break;
    MLP_RELAX_CASE(1)
    MLP_RELAX_CASE(2)
    MLP_RELAX_CASE(4)
    MLP_RELAX_CASE(8)
    MLP_RELAX_CASE(16)
#undef MLP_RELAX_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
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
