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

#include <algorithm>

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
// One wave per image: the block (or its transpose) in the layout of
// mlp_kernels.h (img_layout): CSR for the left-factor role, row bitmaps with
// per-word entry bases for the right-factor role.
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
  const int ncol = tr ? A.lens[a] : A.lens[b];
  const int W = (ncol >> 5) + 1;
  const int64_t e0 = A.ent_off[p];
  const int64_t nnz = A.ent_off[p + 1] - e0;
  const int32_t* rp = tr ? A.trowptr + A.trp_off[p] : A.rowptr + A.rp_off[p];
  const uint16_t* cols = (tr ? A.tcols : A.cols) + e0;
  const float* vals = (tr ? A.tvals : A.vals) + e0;
  const ImgLayout L = img_layout(rows, ncol, nnz);
  uint8_t* dst = A.img + A.img_off[q];
  uint16_t* dcols = (uint16_t*)dst;
  uint16_t* drp = (uint16_t*)(dst + L.rp);
  float* dvals = (float*)(dst + L.vals);
  uint2* dbits = (uint2*)(dst + L.bits);
  for (int k = lane; k < rows + 2; k += 64) drp[k] = (uint16_t)rp[k];
  for (int64_t e = lane; e < nnz; e += 64) {
    dcols[e] = cols[e];
    dvals[e] = vals[e];
  }
  // row bitmaps: lane per row, words in column order
  for (int k = lane + 1; k <= rows; k += 64) {
    int e = rp[k];
    const int re = rp[k + 1];
    for (int w = 0; w < W; ++w) {
      uint32_t bits = 0;
      const int base = e;
      while (e < re && (cols[e] >> 5) == w) {
        bits |= 1u << (cols[e] & 31);
        ++e;
      }
      dbits[(int64_t)(k - 1) * W + w] = make_uint2(bits, (uint32_t)base);
    }
  }
}

// ------------------------------------------------- pair-resident relaxation
// One workgroup per output pair (x, y).  The output cells (the mask: the
// pattern of P_xy, CPNP/MSA.cpp:1237-1261) are cut into tasks of up to four
// cells of one row i; a thread owns a few tasks, their accumulators live in
// registers.  For each z (ascending) the workgroup stages A_z = P(x, z) (CSR)
// and B_z = P(z, y) (row bitmaps) in LDS -- the next z's ranges are
// prefetched into registers while the current z is computed -- and a task
// walks A_z row i (k ascending), looking its cells' columns j up in the
// bitmap of B_z row k.  Each cell's sum therefore runs z ascending, then k
// ascending: the order of Relax / Relax1 (CPNP/MSA.cpp:1276-1350), so every
// float sum is bit-identical to the reference's.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // plain vector: stays in VGPRs
constexpr int kRelaxZChunk = 256;  // z schedule entries per LDS fill
static __host__ __device__ inline size_t relax_tp_bytes(int max_len) {
  return (4 * (size_t)(max_len + 2) + 15) & ~(size_t)15;
}

size_t pair_relax_lds(int cap_a, int cap_b, int max_len) {
  return (size_t)cap_a + (size_t)cap_b + relax_tp_bytes(max_len) + 16 * kRelaxZChunk;
}

int pair_relax_prefetch(int cap) {
  const int chunks = (cap / 16 + kRelaxThreads - 1) / kRelaxThreads;
  for (int kp : {1, 2, 4, 8, 16})
    if (chunks <= kp) return kp;
  return 0;
}

int pair_relax_slots(int64_t tasks) {
  const int64_t per = (tasks + kRelaxThreads - 1) / kRelaxThreads;
  for (int sl : {1, 2, 4, 8})
    if (per <= sl) return sl;
  return 0;
}

template <int KP, int SL>
__global__ __launch_bounds__(kRelaxThreads) void k_relax_pair(PairRelaxArgs A) {
  extern __shared__ __align__(16) uint8_t lds[];
  constexpr int nt = kRelaxThreads;
  constexpr int NC = kRelaxCells;
  const int tid = threadIdx.x;
  const int64_t p = A.pairs[blockIdx.x];
  const int n = A.n;
  const int64_t exy = A.ent_off[p];
  if (A.ent_off[p + 1] == exy) return;  // empty mask: nothing survives
  int x = 0;
  int64_t q = p;
  while (q >= n - 1 - x) { q -= n - 1 - x; ++x; }
  const int y = x + 1 + (int)q;
  const int Lx = A.lens[x], Ly = A.lens[y];
  const int W = (Ly >> 5) + 1;
  uint8_t* sA = lds;
  uint8_t* sB = lds + A.cap_a;
  int32_t* tp = (int32_t*)(lds + A.cap_a + A.cap_b);  // tasks before row i

  // tasks: row i contributes ceil(m_i / NC); prefix by wave 0
  const int32_t* rpxy = A.rowptr + A.rp_off[p];
  if (tid < 64) {
    int run = 0;
    if (tid == 0) tp[1] = 0;
    for (int r0 = 1; r0 <= Lx; r0 += 64) {
      const int i = r0 + tid;
      const int c = i <= Lx ? (rpxy[i + 1] - rpxy[i] + NC - 1) / NC : 0;
      int xs = c;
      for (int off = 1; off < 64; off <<= 1) {
        const int v = __shfl_up(xs, off);
        if (tid >= off) xs += v;
      }
      if (i <= Lx) tp[i + 1] = run + xs;
      run += __shfl(xs, 63);
    }
  }
  __syncthreads();
  const int ntask = tp[Lx + 1];
  int ti[SL];           // row of each task (0 = no task)
  uint32_t wo[SL][NC];  // byte offset of the cell's word in a bitmap row
  uint32_t bm[SL][NC];  // the cell's bit (0 = no cell: never hits)
  float acc[SL][NC];
#pragma unroll
  for (int s = 0; s < SL; ++s) {
    const int g = tid + s * nt;
    ti[s] = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) { wo[s][c] = 0; bm[s][c] = 0; acc[s][c] = 0.f; }
    if (g < ntask) {
      int lo = 1, hi = Lx;  // last row with tp[row] <= g
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (tp[mid] <= g) lo = mid; else hi = mid - 1;
      }
      ti[s] = lo;
      const int e0 = rpxy[lo] + NC * (g - tp[lo]), e1 = rpxy[lo + 1];
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (e0 + c < e1) {
          const uint32_t j = A.cols[exy + e0 + c];
          wo[s][c] = (j >> 5) * 8;
          bm[s][c] = 1u << (j & 31);
          const float v = A.vals[exy + e0 + c];
          acc[s][c] = v + v;  // z = x and z = y (CPNP/MSA.cpp:1211-1213)
        }
    }
  }
  if (tid == 0) tp[0] = 0;  // tp[0] (unused by the scan) doubles as a 0.0f for misses
  const float* zero = (const float*)tp;

  // The z schedule, ZC values of z at a time, in LDS: per z the 16-byte
  // offsets of the A_z range (P(x, z)) and the B_z range (P(z, y)), both
  // blocks' entry counts and L_z; nnz 0 marks a z to skip (z = x, z = y or
  // an empty block).  Filling it costs one memory round trip per ZC values
  // of z instead of one per z.
  uint4* ztab = (uint4*)(lds + A.cap_a + A.cap_b + relax_tp_bytes(A.max_len));
  int zbase = 0, zpos = -1;
  auto fill = [&]() {
    __syncthreads();  // every wave is done reading the previous chunk
    if (tid < kRelaxZChunk) {
      const int z = zbase + tid;
      uint4 e = make_uint4(0, 0, 0, 0);
      if (z < n && z != x && z != y) {
        int64_t pa, pb, qa, qb;
        if (z > x) { pa = pair_index(n, x, z); qa = 2 * pa; } else { pa = pair_index(n, z, x); qa = 2 * pa + 1; }
        if (z < y) { pb = pair_index(n, z, y); qb = 2 * pb; } else { pb = pair_index(n, y, z); qb = 2 * pb + 1; }
        const int na = (int)(A.ent_off[pa + 1] - A.ent_off[pa]);
        const int nb = (int)(A.ent_off[pb + 1] - A.ent_off[pb]);
        if (na > 0 && nb > 0) {
          const int Lz = A.lens[z];
          const ImgLayout lb = img_layout(Lz, Ly, nb);
          e = make_uint4((uint32_t)(A.img_off[qa] >> 4), (uint32_t)((A.img_off[qb] + lb.vals) >> 4),
                         (uint32_t)na | ((uint32_t)nb << 16), (uint32_t)Lz);
        }
      }
      ztab[tid] = e;
    }
    __syncthreads();
  };
  // next scheduled z (uniform across the workgroup); .z == 0 when done
  auto next = [&]() -> uint4 {
    for (;;) {
      if (++zpos == kRelaxZChunk) {
        zbase += kRelaxZChunk;
        if (zbase >= n) return make_uint4(0, 0, 0, 0);
        zpos = 0;
        fill();
      }
      if (zbase + zpos >= n) return make_uint4(0, 0, 0, 0);
      const uint4 e = ztab[zpos];
      if (e.z) return e;
    }
  };
  // register prefetch of the next z's ranges (written out: arrays captured
  // by reference in a lambda end up in scratch)
  u32x4 ra[KP], rb[KP];
  int ca = 0, cb = 0;  // 16-byte chunks of the prefetched ranges
  fill();
  uint4 en = next();
#define MLP_ISSUE()                                                                    \
  {                                                                                    \
    const int Lz_ = (int)en.w, na_ = (int)(en.z & 0xffff), nb_ = (int)(en.z >> 16);   \
    const ImgLayout la = img_layout(Lx, Lz_, na_), lb = img_layout(Lz_, Ly, nb_);      \
    const u32x4* ga = (const u32x4*)(A.img + ((int64_t)en.x << 4));                    \
    const u32x4* gb = (const u32x4*)(A.img + ((int64_t)en.y << 4));                    \
    ca = (int)(la.bits >> 4);                                                          \
    cb = (int)((lb.end - lb.vals + 15) >> 4);                                          \
    _Pragma("unroll") for (int m = 0; m < KP; ++m) {                                   \
      const int c = tid + m * nt;                                                      \
      ra[m] = ga[min(c, ca - 1)];                                                      \
      rb[m] = gb[min(c, cb - 1)];                                                      \
    }                                                                                  \
  }
  if (en.z) MLP_ISSUE();
#ifdef MLP_RELAX_NOSTAGE
  const uint4 e0 = en;
#endif
  while (en.z) {
#pragma unroll
    for (int m = 0; m < KP; ++m) {
      const int c = tid + m * nt;
      if (c < ca) ((u32x4*)sA)[c] = ra[m];
      if (c < cb) ((u32x4*)sB)[c] = rb[m];
    }
    __syncthreads();
#ifdef MLP_RELAX_NOSTAGE  // timing experiment: every z computes on the first z's images
    const int Lz = (int)e0.w, nzA = (int)(e0.z & 0xffff), nzB = (int)(e0.z >> 16);
    en = next();
    ca = cb = 0;
#else
    const int Lz = (int)en.w, nzA = (int)(en.z & 0xffff), nzB = (int)(en.z >> 16);
    en = next();
    if (en.z) MLP_ISSUE();
#endif
    {
      const ImgLayout la = img_layout(Lx, Lz, nzA), lb = img_layout(Lz, Ly, nzB);
      const uint16_t* Acols = (const uint16_t*)sA;
      const uint16_t* Arp = (const uint16_t*)(sA + la.rp);
      const float* Avals = (const float*)(sA + la.vals);
      const float* Bvals = (const float*)sB;
      const uint8_t* Bbits = sB + (lb.bits - lb.vals) - 8 * W;  // row k at k * W words
      const uint32_t W8 = 8 * W;
#pragma unroll
      for (int s = 0; s < SL; ++s) {
#ifdef MLP_RELAX_NOCOMPUTE
        continue;
#endif
        if (ti[s] == 0) continue;
        const int a0 = Arp[ti[s]], a1 = Arp[ti[s] + 1];
        // two A entries per iteration (the second a zero-weight copy of the
        // first past the row end: + 0.0f leaves a positive sum unchanged)
        for (int t = a0; t < a1; t += 2) {
          const bool two = t + 1 < a1;
          const int k0 = Acols[t], k1 = Acols[two ? t + 1 : t];
          const float av0 = Avals[t];
          const float av1 = two ? Avals[t + 1] : 0.f;
          const uint8_t* r0 = Bbits + __umul24(k0, W8);
          const uint8_t* r1 = Bbits + __umul24(k1, W8);
          uint2 w0[NC], w1[NC];
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            w0[c] = *(const uint2*)(r0 + wo[s][c]);
            w1[c] = *(const uint2*)(r1 + wo[s][c]);
          }
          float b0[NC], b1[NC];
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            const uint32_t below = bm[s][c] - 1u;
            const uint32_t i0 = w0[c].y + __popc(w0[c].x & below);
            const uint32_t i1 = w1[c].y + __popc(w1[c].x & below);
            b0[c] = *((w0[c].x & bm[s][c]) ? Bvals + i0 : zero);
            b1[c] = *((w1[c].x & bm[s][c]) ? Bvals + i1 : zero);
          }
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            acc[s][c] += av0 * b0[c];  // a miss adds av * 0 = +0: no change
            acc[s][c] += av1 * b1[c];
          }
        }
      }
    }
    __syncthreads();
  }
#undef MLP_ISSUE
  const float fn = (float)n;  // CPNP/MSA.cpp:1233-1235
#pragma unroll
  for (int s = 0; s < SL; ++s) {
    const int g = tid + s * nt;
    if (ti[s] == 0) continue;
    const int e0 = rpxy[ti[s]] + NC * (g - tp[ti[s]]);
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (bm[s][c]) A.out[exy + e0 + c] = acc[s][c] / fn;
  }
}

hipError_t launch_pack(const PackArgs& a, hipStream_t st) {
  if (a.nimg <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pack, dim3((unsigned)((a.nimg + 3) / 4)), dim3(256), 0, st, a);
  return hipGetLastError();
}

template <int KP>
static hipError_t launch_relax_kp(const PairRelaxArgs& a, int slots, size_t lds, hipStream_t st) {
  const dim3 grid((unsigned)a.npairs), block(kRelaxThreads);
  switch (slots) {
#define MLP_RELAX_CASE(SL)                                                                  \
  case SL:                                                                                  \
    hipFuncSetAttribute((const void*)k_relax_pair<KP, SL>,                                  \
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);              \
    hipLaunchKernelGGL((k_relax_pair<KP, SL>), grid, block, lds, st, a);                    \
    break;
    MLP_RELAX_CASE(1)
    MLP_RELAX_CASE(2)
    MLP_RELAX_CASE(4)
    MLP_RELAX_CASE(8)
#undef MLP_RELAX_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_relax_pairs(const PairRelaxArgs& a, int slots, hipStream_t st) {
  if (a.npairs <= 0) return hipSuccess;
  const size_t lds = pair_relax_lds(a.cap_a, a.cap_b, a.max_len);
  switch (pair_relax_prefetch(std::max(a.cap_a, a.cap_b))) {
    case 1: return launch_relax_kp<1>(a, slots, lds, st);
    case 2: return launch_relax_kp<2>(a, slots, lds, st);
    case 4: return launch_relax_kp<4>(a, slots, lds, st);
    case 8: return launch_relax_kp<8>(a, slots, lds, st);
    case 16: return launch_relax_kp<16>(a, slots, lds, st);
    default: return hipErrorInvalidValue;
  }
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
