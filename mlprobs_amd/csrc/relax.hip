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
    // z = x and z = y (CPNP/MSA.cpp:1211-1213); QuickProbs starts from P_xy
    acc[e] = A.qp.on ? v : v + v;
  }
  float wxy = 0.f, sumw = 1.0f;  // QuickProbs' weights (ConsistencyStage.cpp:199-203)
  if (A.qp.on) {
    int accepted = 0;
    for (int z = 0; z < n; ++z) accepted += z != x && z != y && qp_accept(A.qp, n, x, y, z);
    wxy = 1.0f + (A.qp.selfweight - 1.0f) * (float)accepted / A.qp.selectivity;
    wxy *= A.qp.weights[x] + A.qp.weights[y];
  }
  for (int z = 0; z < n; ++z) {
    if (z == x || z == y) continue;
    if (A.qp.on && !qp_accept(A.qp, n, x, y, z)) continue;
    float wk = 1.0f;  // (1 * a) * b == a * b: C_P_NP_Aln's unweighted terms
    if (A.qp.on) {
      wk = A.qp.weights[z] / wxy;
      sumw += wk;
    }
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
      const float av = wk * aval[u];
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
  const float fn = A.qp.on ? sumw : (float)n;
  for (int e = mb; e < me; ++e) acc[e] = acc[e] / fn;  // CPNP/MSA.cpp:1233-1235; ConsistencyStage.cpp:224-226
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
      for (int e = rb; e < re; ++e) c += (A.raw[eo + e] >= A.cutoff) ? 1 : 0;
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
        if (v >= A.cutoff) {
          A.new_cols[neo + pos] = A.cols[eo + e];
          // QuickProbs' 16-bit entries (SparseEntry.h:31-32)
          A.new_vals[neo + pos] = A.fixed16 ? (float)(uint32_t)(uint16_t)(v * 65535.0f) / 65535.0f : v;
          ++pos;
        }
      }
    }
    run += __shfl(xs, 63);
  }
  if (!A.write && lane == 0) A.pair_nnz[p] = run;
}

// ------------------------------------------------------------ block images
// One wave per image.  Count pass: bitmap words of the image (host sizes the
// records from them); write pass: the record of mlp_kernels.h (img_layout).
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
  // words spanned by row k: first .. last entry's 32-column word
  auto row_words = [&](int k) -> int {
    const int rb = rp[k], re = rp[k + 1];
    return rb < re ? (cols[re - 1] >> 5) - (cols[rb] >> 5) + 1 : 0;
  };
  if (A.count) {
    int s = 0;
    for (int k = lane + 1; k <= rows; k += 64) s += row_words(k);
    for (int off = 32; off; off >>= 1) s += __shfl_xor(s, off);
    if (lane == 0) A.nwords[q] = s;
    return;
  }
  const ImgLayout L = img_layout(rows, nnz, A.nwords[q]);
  uint8_t* dst = A.img + A.img_off[q];
  float* dvals = (float*)dst;
  uint32_t* dhdr = (uint32_t*)(dst + L.hdr);
  uint2* dwords = (uint2*)(dst + L.words);
  for (int64_t e = lane; e < nnz; e += 64) dvals[e] = vals[e];
  if (lane == 0) dhdr[0] = 0;
  int run = 0;  // words before this 64-row chunk
  for (int k0 = 1; k0 <= rows; k0 += 64) {
    const int k = k0 + lane;
    const int nw = k <= rows ? row_words(k) : 0;
    int xs = nw;
    for (int off = 1; off < 64; off <<= 1) {
      const int v = __shfl_up(xs, off);
      if (lane >= off) xs += v;
    }
    if (k <= rows) {
      const int woff = run + xs - nw;
      int e = rp[k];
      const int re = rp[k + 1];
      const int c0w = nw ? cols[e] >> 5 : 0;
      dhdr[k] = (uint32_t)woff | (uint32_t)c0w << 16 | (uint32_t)nw << 24;
      for (int w = 0; w < nw; ++w) {
        uint32_t bits = 0;
        const int base = e;
        while (e < re && (cols[e] >> 5) == c0w + w) {
          bits |= 1u << (cols[e] & 31);
          ++e;
        }
        dwords[woff + w] = make_uint2(bits, (uint32_t)base);
      }
    }
    run += __shfl(xs, 63);
  }
}

// ------------------------------------------------------------ tiled relaxation
// One workgroup per tile of up to kTileMax output pairs (x_t, y) sharing y;
// one thread slot per output cell (i, j) of the masks (the patterns of
// P_{x_t y}, CPNP/MSA.cpp:1237-1261), its accumulator in a register.  For
// each z (ascending) the workgroup stages the row bitmaps of A_t = P(x_t, z)
// (rows i) and of the one shared C = P(y, z) (rows j, i.e. P(z, y)
// transposed) in LDS -- the next z's images are prefetched into registers
// while the current z is computed -- and a cell intersects A_t row i with
// C row j word by word: each common column k contributes
// P_{x_t z}(i, k) * P_{z y}(k, j).  Set bits are taken lowest first, so each
// cell's sum runs z ascending, then k ascending: the order of Relax / Relax1
// (CPNP/MSA.cpp:1276-1350), and every float sum is bit-identical to the
// reference's.  A divergent C3 cell meets ~1.2 common columns per z over
// ~1.8 overlapping words, where a lookup per A entry costs ~11 probes.
// Sharing C across the tile divides its traffic per output pair by T; the
// XCD-aware tile order lets tiles of one x group run on one XCD, so their A
// blocks meet in that XCD's L2.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // plain vector: stays in VGPRs
#define MLP_PF_LOAD(dst, src) (dst) = (src)
#ifndef MLP_RELAX_ZCHUNK
#define MLP_RELAX_ZCHUNK 32
#endif
constexpr int kRelaxZChunk = MLP_RELAX_ZCHUNK;  // z schedule entries per LDS fill (64 B each); 32 leaves the staging area 7.7 KB more than 128 (C3 round 1 1.258 -> 1.205 s)
constexpr int kZEntBytes = 64;
static_assert(kRelaxZChunk <= kRelaxThreads, "one thread fills each z entry of a chunk");
static_assert(kTileMax == 4, "a z entry packs the tile's outputs as uint4 / float4 lanes");
// LDS: [z schedule][QuickProbs z weights][per-output A bases, weights, weight sums][tile]
static __host__ __device__ inline size_t relax_tile_off() {
  return (size_t)kZEntBytes * kRelaxZChunk + 16 * kRelaxZChunk + 16 * kTileMax + 16 + 16 + 16 + 8 * kTileMax;
}
size_t tile_relax_lds(int cap) { return relax_tile_off() + (size_t)cap + 16; }  // + a word pair read past the last row

int tile_relax_prefetch(int cap) {
  const int chunks = (cap / 16 + kRelaxThreads - 1) / kRelaxThreads;
  for (int kp : {5, 9})
    if (chunks <= kp) return kp;
  return 0;
}

int tile_relax_max_cap() { return 9 * kRelaxThreads * 16; }

int tile_relax_slots(int64_t cells) {
  const int64_t per = (cells + kRelaxThreads - 1) / kRelaxThreads;
  for (int sl : {4, 6, 8, 12})
    if (per <= sl) return sl;
  if (kRelaxThreads < 1024 && per <= 16) return 16;
  return 0;
}

// workgroup-uniform values read from LDS: keep them in SGPRs
__device__ __forceinline__ uint4 rfl(uint4 v) {
  return make_uint4(__builtin_amdgcn_readfirstlane(v.x), __builtin_amdgcn_readfirstlane(v.y),
                    __builtin_amdgcn_readfirstlane(v.z), __builtin_amdgcn_readfirstlane(v.w));
}

#ifdef MLP_RELAX_STATS  // measurement variant: trips of the word walk and the hit loop, lane sums vs wave maxima
__device__ unsigned long long g_rstat[4];
#define RSTAT_INC(v) ++(v)
#else
#define RSTAT_INC(v)
#endif
template <int KP, int SL, bool QP>
// KP = 5 (tiles within half the LDS): two workgroups per CU, so 8 waves per
// SIMD and at most 64 VGPRs; KP = 9: one workgroup, 4 waves per SIMD
__global__ __launch_bounds__(kRelaxThreads, KP == 5 && kRelaxThreads == 1024 ? 8 : 4) void k_relax_tile(TileRelaxArgs A) {
  extern __shared__ __align__(16) uint8_t lds[];
  constexpr int nt = kRelaxThreads;
  constexpr int TM = kTileMax;
  const int tid = threadIdx.x;
  // blocks b, b + 8, ... share an XCD: give each XCD a contiguous run of tiles
  const int64_t nb = gridDim.x, bid = blockIdx.x;
  const int64_t xcd = bid & 7, per = nb >> 3, rem = nb & 7;
  const int64_t tile = xcd * per + (xcd < rem ? xcd : rem) + (bid >> 3);
  const int32_t* td = A.tiles + tile * kTileInts;
  const int n = A.n;
  int pt[TM], xt[TM], Lxt[TM];
  int64_t eo[TM];
  int T = 0;
#pragma unroll
  for (int t = 0; t < TM; ++t) {
    pt[t] = td[t];
    xt[t] = td[TM + t];
    T = pt[t] >= 0 ? t + 1 : T;
    Lxt[t] = pt[t] >= 0 ? A.lens[xt[t]] : 0;
    eo[t] = pt[t] >= 0 ? A.ent_off[pt[t]] : 0;
  }
  const int y = td[2 * TM];
  const int Ly = A.lens[y];
  uint4* ztab = (uint4*)lds;
  float4* wtab = (float4*)(lds + kZEntBytes * kRelaxZChunk);  // QuickProbs: w_z / W_{x_t y} per z of the chunk
  int4* zb = (int4*)(lds + kZEntBytes * kRelaxZChunk + 16 * kRelaxZChunk);  // per output: A_t image bases this z
  float* zw = (float*)(zb + TM);  // per output: this z's weight
  float* zsum = zw + 4;           // per output: 1 + sum of the weights so far (z ascending)
  float* wxy = zsum + 4;          // per output: QuickProbs' W_{x_t y} (ConsistencyStage.cpp:199-203)
  const uint8_t** gptr = (const uint8_t**)(wxy + 4);  // per output: its image in HBM (read in place this z)
  uint8_t* tileb = lds + relax_tile_off();
  if constexpr (QP) {  // accepted z per output (A_xy)
    int* nacc = (int*)wxy;
    if (tid < TM) nacc[tid] = 0;
    __syncthreads();
    if (A.qp.seldist) {
      int c[TM];
#pragma unroll
      for (int t = 0; t < TM; ++t) c[t] = 0;
      for (int z = tid; z < n; z += nt)
#pragma unroll
        for (int t = 0; t < TM; ++t)
          c[t] += td[t] >= 0 && z != y && z != td[TM + t] && qp_accept(A.qp, n, td[TM + t], y, z);
#pragma unroll
      for (int t = 0; t < TM; ++t)
        if (c[t]) atomicAdd(&nacc[t], c[t]);
    }
    __syncthreads();
  }
  if (tid < TM) {
    zsum[tid] = 1.0f;
    float w = 1.0f;
    if constexpr (QP) {
      const int xx = td[TM + tid];
      if (td[tid] >= 0) {
        const int accepted = A.qp.seldist ? ((const int*)wxy)[tid] : n - 2;
        w = 1.0f + (A.qp.selfweight - 1.0f) * (float)accepted / A.qp.selectivity;
        w *= A.qp.weights[xx] + A.qp.weights[y];
      }
    }
    wxy[tid] = w;
  }
  // cells before output t (the masks' entries, in CSR order)
  int cb[TM + 1];
  cb[0] = 0;
#pragma unroll
  for (int t = 0; t < TM; ++t) cb[t + 1] = cb[t] + (t < T ? (int)(A.ent_off[pt[t] + 1] - eo[t]) : 0);

  // slot s of this thread: cell g = tid + s * nt: i | j << 13 | t << 26 (0 = none)
  uint32_t cel[SL];
  float acc[SL];
#pragma unroll
  for (int s = 0; s < SL; ++s) {
    const int g = tid + s * nt;
    cel[s] = 0;
    acc[s] = 0.f;
    if (g < cb[TM]) {
      int t = 0;
#pragma unroll
      for (int u = 1; u < TM; ++u) t += g >= cb[u] ? 1 : 0;
      int e = g, Lx = Lxt[0], p = pt[0];
      int64_t ex = eo[0];
#pragma unroll
      for (int u = 1; u < TM; ++u)
        if (t == u) { e = g - cb[u]; Lx = Lxt[u]; p = pt[u]; ex = eo[u]; }
      const int32_t* rp = A.rowptr + A.rp_off[p];
      int lo = 1, hi = Lx;  // row i: last row with rp[i] <= e
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (rp[mid] <= e) lo = mid; else hi = mid - 1;
      }
      const uint32_t j = A.cols[ex + e];
      cel[s] = (uint32_t)lo | j << 13 | (uint32_t)t << 26;
      const float v = A.vals[ex + e];
      acc[s] = QP ? v : v + v;  // z = x and z = y (CPNP/MSA.cpp:1211-1213); QuickProbs starts from P_xy
    }
  }

  // The z schedule, kRelaxZChunk values of z at a time, in LDS (4 uint4 per
  // z): {C start / 16, nnz(C) (0: skip z), C chunks, L_z}, {A_t start / 16},
  // {nnz(A_t) (0: output t skips z)}, {A_t chunks}.  z = y, an empty C or no
  // live A_t skip the whole z.
  int zbase = 0, zpos = -1;
  auto fill = [&]() {
    __syncthreads();  // every wave is done reading the previous chunk
    if (tid < kRelaxZChunk) {
      const int z = zbase + tid;
      uint4 e0 = make_uint4(0, 0, 0, 0), e1 = e0, e2 = e0, e3 = e0;
      if (z < n && z != y) {
        int64_t pc, qc;
        if (y < z) { pc = pair_index(n, y, z); qc = 2 * pc; } else { pc = pair_index(n, z, y); qc = 2 * pc + 1; }
        const int nzc = (int)(A.ent_off[pc + 1] - A.ent_off[pc]);
        if (nzc > 0) {
          uint32_t ao[TM], na[TM], ac[TM];
          bool any = false;
#pragma unroll
          for (int t = 0; t < TM; ++t) {
            ao[t] = na[t] = ac[t] = 0;
            const int xx = td[TM + t];  // (not xt[]: arrays captured by a lambda end up in scratch)
            if (td[t] >= 0 && z != xx && (!QP || qp_accept(A.qp, n, xx, y, z))) {
              int64_t pa, qa;
              if (xx < z) { pa = pair_index(n, xx, z); qa = 2 * pa; } else { pa = pair_index(n, z, xx); qa = 2 * pa + 1; }
              const int nza = (int)(A.ent_off[pa + 1] - A.ent_off[pa]);
              if (nza > 0) {
                ao[t] = (uint32_t)(A.img_off[qa] >> 4);
                na[t] = (uint32_t)nza;
                ac[t] = (uint32_t)((A.img_off[qa + 1] - A.img_off[qa]) >> 4);
                any = true;
              }
            }
          }
          if (any) {
            // outputs in passes over this z when their images and C exceed
            // the staging area (greedy in output order): pass of output t in
            // bits 2t, 2t+1, passes - 1 in bits 8-9 of e0.w; an output whose
            // image does not fit beside C even alone is not staged (bit 12 + t:
            // its cells read the image from HBM; small-class tiles only)
            const uint32_t cC = (uint32_t)((A.img_off[qc + 1] - A.img_off[qc]) >> 4);
            const uint32_t capc = (uint32_t)A.cap >> 4;
            uint32_t used = cC, grp = 0, gsel = 0, gmask = 0;
#pragma unroll
            for (int t = 0; t < TM; ++t) {
              if (na[t] == 0) continue;
              if (cC + ac[t] > capc) {  // not staged: its cells read the image in HBM (pass 0)
                gmask |= 1u << t;
                ac[t] = 0;
                continue;
              }
              if (used + ac[t] > capc && used > cC) {
                ++grp;
                used = cC;
              }
              used += ac[t];
              gsel |= grp << (2 * t);
            }
            e0 = make_uint4((uint32_t)(A.img_off[qc] >> 4), (uint32_t)nzc, cC, gsel | grp << 8 | gmask << 12);
            e1 = make_uint4(ao[0], ao[1], ao[2], ao[3]);
            e2 = make_uint4(na[0], na[1], na[2], na[3]);
            e3 = make_uint4(ac[0], ac[1], ac[2], ac[3]);
          }
        }
      }
      ztab[4 * tid] = e0;
      ztab[4 * tid + 1] = e1;
      ztab[4 * tid + 2] = e2;
      ztab[4 * tid + 3] = e3;
      if constexpr (QP) {  // every accepted z != x_t, y counts in the weight sum, scheduled or not
        float wz[TM];
#pragma unroll
        for (int t = 0; t < TM; ++t)
          wz[t] = (z < n && z != y && td[t] >= 0 && z != td[TM + t] && qp_accept(A.qp, n, td[TM + t], y, z))
                      ? A.qp.weights[z] / wxy[t]
                      : 0.f;
        wtab[tid] = make_float4(wz[0], wz[1], wz[2], wz[3]);
      }
    }
    __syncthreads();
    if constexpr (QP) {  // weight sums in z order (ConsistencyStage.cpp:205-217); + 0 leaves them unchanged
      if (tid < TM) {
        float sw = zsum[tid];
        for (int k = 0; k < kRelaxZChunk && zbase + k < n; ++k) {
          const float4 w4 = wtab[k];
          sw += tid == 0 ? w4.x : tid == 1 ? w4.y : tid == 2 ? w4.z : w4.w;
        }
        zsum[tid] = sw;
      }
    }
  };
  // next scheduled z (uniform across the workgroup); returns false when done
  uint4 nC, nAo, nNa, nAc;  // the staged-next z's entry
  float4 nW = make_float4(1.f, 1.f, 1.f, 1.f);  // its QuickProbs weights
  int zpass = 0;  // pass of the current z (several when its images exceed the staging area)
  auto next = [&]() -> bool {
    for (;;) {
      if (zpos >= 0 && zpass < (int)((nC.w >> 8) & 3) && nC.y) {
        ++zpass;  // the same z again, the next subset of outputs
      } else {
        zpass = 0;
        if (++zpos == kRelaxZChunk) {
          zbase += kRelaxZChunk;
          if (zbase >= n) return false;
          zpos = 0;
          fill();
        }
        if (zbase + zpos >= n) return false;
        nC = rfl(ztab[4 * zpos]);
      }
      if (nC.y) {
        nAo = rfl(ztab[4 * zpos + 1]);
        nNa = rfl(ztab[4 * zpos + 2]);
        nAc = rfl(ztab[4 * zpos + 3]);
        if ((nC.w >> 8) & 3) {  // keep this pass's outputs only
          const uint32_t g = nC.w;
          const uint32_t p = (uint32_t)zpass;
          if (((g >> 0) & 3) != p) { nNa.x = 0; nAc.x = 0; }
          if (((g >> 2) & 3) != p) { nNa.y = 0; nAc.y = 0; }
          if (((g >> 4) & 3) != p) { nNa.z = 0; nAc.z = 0; }
          if (((g >> 6) & 3) != p) { nNa.w = 0; nAc.w = 0; }
        }
        if constexpr (QP) {
          const float4 w4 = wtab[zpos];
          const uint4 u = rfl(make_uint4(__float_as_uint(w4.x), __float_as_uint(w4.y), __float_as_uint(w4.z),
                                         __float_as_uint(w4.w)));  // (readfirstlane is an int builtin)
          nW = make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
        }
        return true;
      }
    }
  };
  // register prefetch of the next z's tile: segments A_0 .. A_{TM-1}, C,
  // contiguous in LDS (written out: arrays captured by a lambda end up in scratch)
  u32x4 pf[KP];
  int sg[TM + 1];  // segment starts (16-byte chunks) of the prefetched tile
  const u32x4* g16 = (const u32x4*)A.img;
#define MLP_ISSUE()                                                                      \
  {                                                                                      \
    const uint32_t ao_[TM] = {nAo.x, nAo.y, nAo.z, nAo.w};                               \
    const uint32_t ac_[TM] = {nAc.x, nAc.y, nAc.z, nAc.w};                               \
    int dl_[TM];                                                                         \
    sg[0] = 0;                                                                           \
    _Pragma("unroll") for (int t = 0; t < TM; ++t) {                                     \
      dl_[t] = (int)ao_[t] - sg[t];                                                      \
      sg[t + 1] = sg[t] + (int)ac_[t];                                                   \
    }                                                                                    \
    const int tot_ = sg[TM] + (int)nC.z;                                                 \
    const int dC_ = (int)nC.x - sg[TM];                                                  \
    /* unconditional loads (past the tile: its first chunk again), so the */            \
    /* KP loads issue back to back with no wait between them */                          \
    _Pragma("unroll") for (int m = 0; m < KP; ++m) {                                     \
      const int c = tid + m * nt < tot_ ? tid + m * nt : 0;                              \
      int d = dC_;                                                                       \
      _Pragma("unroll") for (int t = TM - 1; t >= 0; --t) d = c < sg[t + 1] ? dl_[t] : d; \
      MLP_PF_LOAD(pf[m], g16[(uint32_t)(c + d)]);                                        \
    }                                                                                    \
  }
  // KP = 9: the next z's tile is loaded into registers while this z computes;
  // KP = 5 (two workgroups per CU): loaded at the stage, the other
  // workgroup's compute covers the wait and the registers stay free
  constexpr bool kRegPrefetch = KP == 9;
  fill();
  bool more = next();
  if (kRegPrefetch && more) MLP_ISSUE();
#ifdef MLP_RELAX_STATS
  // per (slot, z): lanes' word steps and hits summed, and 64 x the wave's
  // maximum (the trips the wave issues); lane 0 keeps the wave's totals
  uint32_t st_w = 0, st_h = 0;
  unsigned long long sw_sum = 0, sw_max = 0, sh_sum = 0, sh_max = 0;
#define RSTAT_SLOT()                                                                  \
  {                                                                                   \
    uint32_t a_ = st_w, b_ = st_h, ma_ = st_w, mb_ = st_h;                            \
    for (int o_ = 32; o_; o_ >>= 1) {                                                 \
      a_ += __shfl_xor(a_, o_); b_ += __shfl_xor(b_, o_);                             \
      ma_ = max(ma_, (uint32_t)__shfl_xor(ma_, o_)); mb_ = max(mb_, (uint32_t)__shfl_xor(mb_, o_)); \
    }                                                                                 \
    sw_sum += a_; sh_sum += b_; sw_max += 64ull * ma_; sh_max += 64ull * mb_;         \
    st_w = st_h = 0;                                                                  \
  }
#else
#define RSTAT_SLOT()
#endif
  while (more) {
    if constexpr (!kRegPrefetch) MLP_ISSUE();
    // stage the prefetched tile; outputs' A bases (+ validity) into zb
    const int tot = sg[TM] + (int)nC.z;
#pragma unroll
    for (int m = 0; m < KP; ++m) {
      const int c = tid + m * nt;
      if (c < tot) ((u32x4*)tileb)[c] = pf[m];
    }
    const uint32_t cbase = (uint32_t)(relax_tile_off() + 16 * (size_t)sg[TM]);
    const int nzC = (int)nC.y;
    const uint32_t gmz = (nC.w >> 12) & 15;  // this z's outputs read in HBM
    if (tid == 0) {
      zw[0] = nW.x; zw[1] = nW.y; zw[2] = nW.z; zw[3] = nW.w;
      const uint32_t na_[TM] = {nNa.x, nNa.y, nNa.z, nNa.w};
      const uint32_t ao_[TM] = {nAo.x, nAo.y, nAo.z, nAo.w};
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        // in HBM (bit 12 + t): offsets from the image's own start
        const bool g = (nC.w >> (12 + t)) & 1;
        const uint32_t ab = g ? 0u : (uint32_t)(relax_tile_off() + 16 * (size_t)sg[t]);
        const uint32_t ho = ab + (uint32_t)mlp_align16(4 * (int64_t)na_[t]);
        zb[t] = make_int4((int)ab, (int)ho, (int)(ho + (uint32_t)mlp_align16(4 * (int64_t)(Lxt[t] + 1))),
                          (int)na_[t]);
        gptr[t] = A.img + 16 * (uint64_t)ao_[t];
      }
    }
    __syncthreads();
    more = next();
    if (kRegPrefetch && more) MLP_ISSUE();
    // the lowest hit of m: `below` = the bits under it, m loses it; the
    // compiler folds `below & bits` into one v_bitop3 per side (11 VALU a
    // hit instead of 14 with 1 << ctz(m): C3 round 1 1206 -> 1155 ms)
#define MLP_HIT_BITS(m, below)      \
  const uint32_t t_ = (m) - 1u;     \
  const uint32_t below = t_ & ~(m); \
  (m) &= t_;
#define MLP_HITS(m, xa, xc)                                                        \
      while (m) { /* common columns k, ascending */                                \
        RSTAT_INC(st_h);                                                           \
        MLP_HIT_BITS(m, below);                                                    \
        const float va = QP ? wk * Avals[xa.y + __popc(xa.x & below)]              \
                            : Avals[xa.y + __popc(xa.x & below)];                  \
        const float vc = Cvals[xc.y + __popc(xc.x & below)];                       \
        ac += va * vc;                                                             \
      }
    // per word pair: the load, then the common columns of each word (a single
    // loop over loads and hits, MLP_RELAX_FLAT in round 4, ran 1.69 s against
    // 1.21 s: the wave issues both bodies every iteration)
#define MLP_WALK(pa, pc, we, a0, c0)                                                                  \
    for (int w = max(a0, c0); w < we; w += 2) {                                                       \
      RSTAT_INC(st_w);                                                                                \
      const uint2 xa0 = pa[w], xa1 = pa[w + 1], xc0 = pc[w], xc1 = pc[w + 1];                         \
      uint32_t m0 = xa0.x & xc0.x;                                                                    \
      uint32_t m1 = w + 1 < we ? xa1.x & xc1.x : 0u;                                                  \
      MLP_HITS(m0, xa0, xc0)                                                                          \
      MLP_HITS(m1, xa1, xc1)                                                                          \
    }
    // the cell loop, twice: with every image in LDS, and (GA) for a z where
    // some output image is read in place from HBM (generic loads)
#define MLP_CELLS(GA, ONE) \
    {                                                                                                            \
      const float* Cvals = (const float*)(lds + cbase);                                                          \
      const uint32_t* Chdr = (const uint32_t*)(lds + cbase + (uint32_t)mlp_align16(4 * (int64_t)nzC));           \
      const uint2* Cwords = (const uint2*)((const uint8_t*)Chdr + (uint32_t)mlp_align16(4 * (int64_t)(Ly + 1))); \
      /* row headers of slot s + 1 are read while slot s intersects */                                           \
      /* GA: outputs of this z may be read in HBM (generic pointers); ONE: the */                                \
      /* tile has one output, its bases are workgroup-uniform (SGPRs) */                                         \
      auto headers = [&](uint32_t cl, int4& z4, uint32_t& ha, uint32_t& hc, const uint8_t*& ab) {                \
        z4 = (ONE) ? z4u : zb[cl >> 26];                                                                         \
        ab = (GA) && ((ONE) ? (gmz & 1) != 0 : ((gmz >> (cl >> 26)) & 1) != 0) ? ((ONE) ? gp0 : gptr[cl >> 26])  \
                                                                             : (const uint8_t*)lds;              \
        ha = z4.w ? ((const uint32_t*)(ab + z4.y))[cl & 0x1fff] : 0u;  /* nw 0: no words */                      \
        hc = Chdr[(cl >> 13) & 0x1fff];                                                                          \
      };                                                                                                         \
      uint32_t cl = cel[0];                                                                                      \
      asm volatile("" : "+v"(cl));                                                                               \
      int4 z4;                                                                                                   \
      uint32_t ha, hc;                                                                                           \
      const uint8_t* ab;                                                                                         \
      headers(cl, z4, ha, hc, ab);                                                                               \
_Pragma("unroll")                                                                                         \
      for (int s = 0; s < SL; ++s) {                                                                             \
        uint32_t cl1 = 0, ha1 = 0, hc1 = 0;                                                                      \
        int4 z41 = make_int4(0, 0, 0, 0);                                                                        \
        const uint8_t* ab1 = lds;                                                                                \
        if (s + 1 < SL) {                                                                                        \
          cl1 = cel[s + 1];                                                                                      \
          /* re-derive the cells' offsets every z: hoisting them out of the z */                                 \
          /* loop would hold ~4 more registers per slot */                                                       \
          asm volatile("" : "+v"(cl1));                                                                          \
          headers(cl1, z41, ha1, hc1, ab1);                                                                      \
        }                                                                                                        \
        if (cl != 0) {                                                                                           \
          const int a0 = (int)((ha >> 16) & 0xff), c0 = (int)((hc >> 16) & 0xff);                                \
          const int we = min(a0 + (int)(ha >> 24), c0 + (int)(hc >> 24));                                        \
          const uint2* pa = (const uint2*)(ab + z4.z) + ((int)(ha & 0xffff) - a0);                               \
          const uint2* pc = Cwords + ((int)(hc & 0xffff) - c0);                                                  \
          const float* Avals = (const float*)(ab + z4.x);                                                        \
          const float wk = QP ? ((ONE) ? w0 : zw[cl >> 26]) : 1.0f;  /* weight * XZ * ZY (ConsistencyStage.cpp:284) */ \
          float ac = acc[s];                                                                                     \
          MLP_WALK(pa, pc, we, a0, c0)                                                                           \
          acc[s] = ac;                                                                                           \
        }                                                                                                        \
        RSTAT_SLOT();                                                                                            \
        cl = cl1;                                                                                                \
        z4 = z41;                                                                                                \
        ha = ha1;                                                                                                \
        hc = hc1;                                                                                                \
        ab = ab1;                                                                                                \
      }                                                                                                          \
    }
    // one-output tiles (most at C3: one output of up to 6144 cells): the
    // image bases are workgroup-uniform, read once per z into SGPRs instead
    // of an LDS read per slot (C3 round 1 1154 -> 1118 ms)
    if (T == 1) {
      const uint4 zu = rfl(*(const uint4*)zb);
      const int4 z4u = make_int4((int)zu.x, (int)zu.y, (int)zu.z, (int)zu.w);
      const uint8_t* gp0 = (const uint8_t*)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)gptr[0] >> 32)) << 32) |
                                            (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uint64_t)gptr[0]));
      const float w0 = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(zw[0])));
      if (gmz) MLP_CELLS(true, true) else MLP_CELLS(false, true)
    } else {
      const int4 z4u = make_int4(0, 0, 0, 0);
      const uint8_t* gp0 = nullptr;
      const float w0 = 0.f;
      if (gmz) MLP_CELLS(true, false) else MLP_CELLS(false, false)
    }
#undef MLP_CELLS
#undef MLP_WALK
#undef MLP_HITS
    __syncthreads();
  }
#undef MLP_ISSUE
#undef RSTAT_SLOT
#ifdef MLP_RELAX_STATS
  if ((tid & 63) == 0) {
    atomicAdd(&g_rstat[0], sw_sum);
    atomicAdd(&g_rstat[1], sw_max);
    atomicAdd(&g_rstat[2], sh_sum);
    atomicAdd(&g_rstat[3], sh_max);
  }
#endif
  __syncthreads();  // the weight sums of the last chunk
  const float fn = (float)n;  // CPNP/MSA.cpp:1233-1235; QuickProbs: / the weight sum
#pragma unroll
  for (int s = 0; s < SL; ++s) {
    if (cel[s] == 0) continue;
    const int g = tid + s * nt;
    const int t = (int)(cel[s] >> 26);
    int e = g;
    int64_t ex = eo[0];
#pragma unroll
    for (int u = 1; u < TM; ++u)
      if (t == u) { e = g - cb[u]; ex = eo[u]; }
    A.out[ex + e] = acc[s] / (QP ? zsum[t] : fn);
  }
}

hipError_t launch_pack(const PackArgs& a, hipStream_t st) {
  if (a.nimg <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pack, dim3((unsigned)((a.nimg + 3) / 4)), dim3(256), 0, st, a);
  return hipGetLastError();
}

template <int KP, bool QP>
static hipError_t launch_tiles_kp(const TileRelaxArgs& a, int slots, size_t lds, hipStream_t st) {
  const dim3 grid((unsigned)a.ntiles), block(kRelaxThreads);
  switch (slots) {
#define MLP_RELAX_CASE(SL)                                                                  \
  case SL:                                                                                  \
    hipFuncSetAttribute((const void*)k_relax_tile<KP, SL, QP>,                              \
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);              \
    hipLaunchKernelGGL((k_relax_tile<KP, SL, QP>), grid, block, lds, st, a);                \
    break;
    MLP_RELAX_CASE(4)
    MLP_RELAX_CASE(6)
    MLP_RELAX_CASE(8)
    MLP_RELAX_CASE(12)
#if MLP_RELAX_THREADS < 1024
    MLP_RELAX_CASE(16)
#endif
#undef MLP_RELAX_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_relax_tiles(const TileRelaxArgs& a, int slots, bool one_per_cu, hipStream_t st) {
  if (a.ntiles <= 0) return hipSuccess;
  const size_t lds = tile_relax_lds(a.cap);
  hipError_t e;
  const int kpv = tile_relax_prefetch(a.cap);
  // MLP_TEST_RELAX_KP: force the large-prefetch variant
  switch ((int)knob("MLP_TEST_RELAX_KP", one_per_cu && kpv ? 9 : kpv)) {
    case 5: e = a.qp.on ? launch_tiles_kp<5, true>(a, slots, lds, st) : launch_tiles_kp<5, false>(a, slots, lds, st); break;
    case 9: e = a.qp.on ? launch_tiles_kp<9, true>(a, slots, lds, st) : launch_tiles_kp<9, false>(a, slots, lds, st); break;
    default: return hipErrorInvalidValue;
  }
#ifdef MLP_RELAX_STATS
  {
    unsigned long long h[4];
    hipStreamSynchronize(st);
    hipMemcpyFromSymbol(h, HIP_SYMBOL(g_rstat), sizeof h);
    fprintf(stderr, "relax stats: slots %d word steps lane-sum %llu wave-issued %llu (efficiency %.3f) | hits lane-sum %llu "
            "wave-issued %llu (efficiency %.3f)\n", slots, h[0], h[1], h[1] ? (double)h[0] / h[1] : 0.0, h[2], h[3],
            h[3] ? (double)h[2] / h[3] : 0.0);
    for (auto& v : h) v = 0;
    hipMemcpyToSymbol(HIP_SYMBOL(g_rstat), h, sizeof h);
  }
#endif
  return e;
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
