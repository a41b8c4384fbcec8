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
  uint16_t* dcols = (uint16_t*)dst;
  uint16_t* drp = (uint16_t*)(dst + L.rp);
  float* dvals = (float*)(dst + L.vals);
  uint32_t* dhdr = (uint32_t*)(dst + L.hdr);
  uint2* dwords = (uint2*)(dst + L.words);
  for (int k = lane; k < rows + 2; k += 64) drp[k] = (uint16_t)rp[k];
  for (int64_t e = lane; e < nnz; e += 64) {
    dcols[e] = cols[e];
    dvals[e] = vals[e];
  }
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
// One workgroup per tile of up to kTileMax output pairs (x_t, y) sharing y.
// The output cells (the mask: the pattern of P_{x_t y}, CPNP/MSA.cpp:1237-1261)
// are cut into tasks of up to four cells of one row i; a thread owns a few
// tasks, their accumulators live in registers.  For each z (ascending) the
// workgroup stages the A_t = P(x_t, z) blocks (CSR) and the one shared
// B = P(z, y) block (row bitmaps over each row's column span) in LDS -- the
// next z's ranges are prefetched into registers while the current z is
// computed -- and a task walks A_t row i (k ascending), looking its cells'
// columns j up in the bitmap of B row k.  Each cell's sum therefore runs
// z ascending, then k ascending: the order of Relax / Relax1
// (CPNP/MSA.cpp:1276-1350), so every float sum is bit-identical to the
// reference's.  Sharing B across the tile halves (T = 2) to quarters (T = 4)
// the B traffic per output pair; the XCD-aware tile order lets tiles with the
// same x group run on one XCD, so their A blocks meet in that XCD's L2.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // plain vector: stays in VGPRs
#ifdef MLP_RELAX_NOLOAD  // timing experiment: no global loads for the staging
#define MLP_PF_LOAD(dst, src) (dst) = u32x4{(uint32_t)c, 0u, 0u, 0u}
#else
#define MLP_PF_LOAD(dst, src) (dst) = (src)
#endif
#ifdef MLP_RELAX_SEQADDR  // timing experiment: each workgroup streams consecutive memory over z
#define MLP_PF_SRC ((uint32_t)((((uint64_t)tile * 7919 + (uint64_t)zcount) * (uint64_t)tot_) % (uint64_t)(A.img_chunks - tot_)) + (uint32_t)c)
#else
#define MLP_PF_SRC ((uint32_t)(c + d))
#endif
constexpr int kRelaxZChunk = 128;  // z schedule entries per LDS fill (48 B each)
constexpr int kRelaxGuard = 2048;  // LDS bytes after the tile: unchecked bitmap-word reads stay inside
static __host__ __device__ inline size_t relax_tp_bytes(int max_len) {
  return (4 * (size_t)kTileMax * (max_len + 2) + 15) & ~(size_t)15;
}
// LDS: [z schedule][task prefixes][per-output A bases][zero][tile][guard];
// the schedule (6 KB) in front keeps unchecked reads below the tile inside too
static __host__ __device__ inline size_t relax_tile_off(int max_len) {
  return 48 * (size_t)kRelaxZChunk + relax_tp_bytes(max_len) + 32 * kTileMax + 16;
}
size_t tile_relax_lds(int cap, int max_len) { return relax_tile_off(max_len) + (size_t)cap + kRelaxGuard; }

int tile_relax_prefetch(int cap) {
  const int chunks = (cap / 16 + kRelaxThreads - 1) / kRelaxThreads;
  for (int kp : {6, 12})
    if (chunks <= kp) return kp;
  return 0;
}

int tile_relax_max_cap() { return 12 * kRelaxThreads * 16; }

int tile_relax_slots(int64_t tasks) {
  const int64_t per = (tasks + kRelaxThreads - 1) / kRelaxThreads;
  for (int sl : {2, 4})
    if (per <= sl) return sl;
  return 0;
}


// workgroup-uniform values read from LDS: keep them in SGPRs
__device__ __forceinline__ uint4 rfl(uint4 v) {
  return make_uint4(__builtin_amdgcn_readfirstlane(v.x), __builtin_amdgcn_readfirstlane(v.y),
                    __builtin_amdgcn_readfirstlane(v.z), __builtin_amdgcn_readfirstlane(v.w));
}

template <int KP, int SL>
__global__ __launch_bounds__(kRelaxThreads) void k_relax_tile(TileRelaxArgs A) {
  extern __shared__ __align__(16) uint8_t lds[];
  constexpr int nt = kRelaxThreads;
  constexpr int NC = kRelaxCells;
  constexpr int TM = kTileMax;
  const int tid = threadIdx.x;
  // blocks b, b + 8, ... share an XCD: give each XCD a contiguous run of tiles
  const int64_t nb = gridDim.x, bid = blockIdx.x;
  const int64_t xcd = bid & 7, per = nb >> 3, rem = nb & 7;
  const int64_t tile = xcd * per + (xcd < rem ? xcd : rem) + (bid >> 3);
  const int32_t* td = A.tiles + tile * kTileInts;
  const int n = A.n;
  int pt[TM], xt[TM], Lxt[TM];
  int T = 0;
#pragma unroll
  for (int t = 0; t < TM; ++t) {
    pt[t] = td[t];
    xt[t] = td[TM + t];
    T = pt[t] >= 0 ? t + 1 : T;
    Lxt[t] = pt[t] >= 0 ? A.lens[xt[t]] : 0;
  }
  const int y = td[2 * TM];
  const int tps = A.max_len + 2;
  uint4* ztab = (uint4*)lds;
  int32_t* tp = (int32_t*)(lds + 48 * kRelaxZChunk);  // per output: tasks before row i
  int4* zb = (int4*)(lds + 48 * kRelaxZChunk + relax_tp_bytes(A.max_len));  // per output: A bases this z
  int4* oinf = zb + TM;  // per output: {pair, L_x, tasks before it, -} (per-lane lookups by output)
  float* zero = (float*)(oinf + TM);
  uint8_t* tileb = lds + relax_tile_off(A.max_len);

  // task prefixes: wave t scans output t (row i contributes ceil(m_i / NC))
  {
    const int wv = tid >> 6, ln = tid & 63;
    if (wv < T) {
      const int64_t p = td[wv];
      const int Lx = A.lens[td[TM + wv]];
      const int32_t* rpxy = A.rowptr + A.rp_off[p];
      int32_t* tw = tp + wv * tps;
      int run = 0;
      if (ln == 0) tw[1] = 0;
      for (int r0 = 1; r0 <= Lx; r0 += 64) {
        const int i = r0 + ln;
        const int c = i <= Lx ? (rpxy[i + 1] - rpxy[i] + NC - 1) / NC : 0;
        int xs = c;
        for (int off = 1; off < 64; off <<= 1) {
          const int v = __shfl_up(xs, off);
          if (ln >= off) xs += v;
        }
        if (i <= Lx) tw[i + 1] = run + xs;
        run += __shfl(xs, 63);
      }
    }
    if (tid == 0) *zero = 0.f;
  }
  __syncthreads();
  int tb[TM + 1];
  tb[0] = 0;
#pragma unroll
  for (int t = 0; t < TM; ++t)
    tb[t + 1] = tb[t] + (t < T ? __builtin_amdgcn_readfirstlane(tp[t * tps + Lxt[t] + 1]) : 0);
  if (tid < TM) {
    int4 o = make_int4(-1, 0, 0, 0);
#pragma unroll
    for (int t = 0; t < TM; ++t)
      if (tid == t) o = make_int4(pt[t], Lxt[t], tb[t], 0);
    oinf[tid] = o;
  }
  __syncthreads();

  uint32_t tio[SL];     // row i (0 = no task) | output t << 16 of each task
  uint32_t jw[SL][NC];  // the cell's 32-column word index j >> 5
  uint32_t bm[SL][NC];  // the cell's bit (0 = no cell: never hits)
  float acc[SL][NC];
#pragma unroll
  for (int s = 0; s < SL; ++s) {
    const int g = tid + s * nt;
    tio[s] = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) { jw[s][c] = 0; bm[s][c] = 0; acc[s][c] = 0.f; }
    if (g < tb[TM]) {
      int t = 0;
#pragma unroll
      for (int u = 1; u < TM; ++u) t += g >= tb[u] ? 1 : 0;
      const int4 o = oinf[t];
      const int gl = g - o.z;
      const int32_t* tt = tp + t * tps;
      int lo = 1, hi = o.y;  // last row with tt[row] <= gl
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (tt[mid] <= gl) lo = mid; else hi = mid - 1;
      }
      const int64_t p = o.x;
      const int64_t exy = A.ent_off[p];
      const int32_t* rpxy = A.rowptr + A.rp_off[p];
      tio[s] = (uint32_t)lo | (uint32_t)t << 16;
      const int e0 = rpxy[lo] + NC * (gl - tt[lo]), e1 = rpxy[lo + 1];
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (e0 + c < e1) {
          const uint32_t j = A.cols[exy + e0 + c];
          jw[s][c] = j >> 5;
          bm[s][c] = 1u << (j & 31);
          const float v = A.vals[exy + e0 + c];
          acc[s][c] = v + v;  // z = x and z = y (CPNP/MSA.cpp:1211-1213)
        }
    }
  }

  // The z schedule, kRelaxZChunk values of z at a time, in LDS (3 uint4 per
  // z): {B range start / 16, nnz(B) | L_z << 16 (0: skip z), B chunks, -},
  // {A_t range start / 16}, {nnz(A_t) (0: output t skips z)}.  z = y, an
  // empty B or no live A_t skip the whole z.
  int zbase = 0, zpos = -1;
  auto fill = [&]() {
    __syncthreads();  // every wave is done reading the previous chunk
    if (tid < kRelaxZChunk) {
      const int z = zbase + tid;
      uint4 e0 = make_uint4(0, 0, 0, 0), e1 = e0, e2 = e0;
      if (z < n && z != y) {
        int64_t pb, qb;
        if (z < y) { pb = pair_index(n, z, y); qb = 2 * pb; } else { pb = pair_index(n, y, z); qb = 2 * pb + 1; }
        const int nbz = (int)(A.ent_off[pb + 1] - A.ent_off[pb]);
        if (nbz > 0) {
          uint32_t ao[TM], na[TM];
          bool any = false;
#pragma unroll
          for (int t = 0; t < TM; ++t) {
            ao[t] = 0;
            na[t] = 0;
            const int xx = td[TM + t];  // (not xt[]: arrays captured by a lambda end up in scratch)
            if (td[t] >= 0 && z != xx) {
              int64_t pa, qa;
              if (xx < z) { pa = pair_index(n, xx, z); qa = 2 * pa; } else { pa = pair_index(n, z, xx); qa = 2 * pa + 1; }
              const int nza = (int)(A.ent_off[pa + 1] - A.ent_off[pa]);
              if (nza > 0) {
                ao[t] = (uint32_t)(A.img_off[qa] >> 4);
                na[t] = (uint32_t)nza;
                any = true;
              }
            }
          }
          if (any) {
            const int Lz = A.lens[z];
            const int nw = A.nwords[qb];
            const ImgLayout lb = img_layout(Lz, nbz, nw);
            e0 = make_uint4((uint32_t)((A.img_off[qb] + lb.vals) >> 4), (uint32_t)nbz | ((uint32_t)Lz << 16),
                            (uint32_t)(img_b_bytes(Lz, nbz, nw) >> 4), 0);
            e1 = make_uint4(ao[0], ao[1], ao[2], ao[3]);
            e2 = make_uint4(na[0], na[1], na[2], na[3]);
          }
        }
      }
      ztab[3 * tid] = e0;
      ztab[3 * tid + 1] = e1;
      ztab[3 * tid + 2] = e2;
    }
    __syncthreads();
  };
  // next scheduled z (uniform across the workgroup); returns false when done
  uint4 nB, nAo, nNa;  // the staged-next z's entry
  auto next = [&]() -> bool {
    for (;;) {
      if (++zpos == kRelaxZChunk) {
        zbase += kRelaxZChunk;
        if (zbase >= n) return false;
        zpos = 0;
        fill();
      }
      if (zbase + zpos >= n) return false;
      nB = rfl(ztab[3 * zpos]);
      if (nB.y) {
        nAo = rfl(ztab[3 * zpos + 1]);
        nNa = rfl(ztab[3 * zpos + 2]);
        return true;
      }
    }
  };
  // register prefetch of the next z's tile: segments A_0 .. A_{TM-1}, B,
  // contiguous in LDS (written out: arrays captured by a lambda end up in scratch)
  u32x4 pf[KP];
  int sg[TM + 1];  // segment starts (16-byte chunks) of the prefetched tile
  const u32x4* g16 = (const u32x4*)A.img;
#define MLP_ISSUE()                                                                      \
  {                                                                                      \
    const uint32_t ao_[TM] = {nAo.x, nAo.y, nAo.z, nAo.w};                               \
    const uint32_t na_[TM] = {nNa.x, nNa.y, nNa.z, nNa.w};                               \
    int dl_[TM];                                                                         \
    sg[0] = 0;                                                                           \
    _Pragma("unroll") for (int t = 0; t < TM; ++t) {                                     \
      const int ca_ = na_[t] ? (int)(img_a_bytes(Lxt[t], na_[t]) >> 4) : 0;              \
      dl_[t] = (int)ao_[t] - sg[t];                                                      \
      sg[t + 1] = sg[t] + ca_;                                                           \
    }                                                                                    \
    const int tot_ = sg[TM] + (int)nB.z;                                                 \
    const int dB_ = (int)nB.x - sg[TM];                                                  \
    _Pragma("unroll") for (int m = 0; m < KP; ++m) {                                     \
      const int c = tid + m * nt;                                                        \
      if (c < tot_) {                                                                    \
        int d = dB_;                                                                     \
        _Pragma("unroll") for (int t = TM - 1; t >= 0; --t) d = c < sg[t + 1] ? dl_[t] : d; \
        MLP_PF_LOAD(pf[m], g16[MLP_PF_SRC]);                                             \
      }                                                                                  \
    }                                                                                    \
  }
  fill();
  int zcount = 0;
  (void)zcount;
  bool more = next();
  if (more) MLP_ISSUE();
#ifdef MLP_RELAX_SAMEADDR  // timing experiment: every z loads the first z's tile again
  const uint4 fB = nB, fAo = nAo, fNa = nNa;
#endif
#ifdef MLP_RELAX_NOSTAGE  // timing experiment: every z computes on the first z's tile
  const uint4 fB = nB, fAo = nAo, fNa = nNa;
#endif
  while (more) {
    // stage the prefetched tile; outputs' A bases (+ validity) into zb
    const int tot = sg[TM] + (int)nB.z;
#pragma unroll
    for (int m = 0; m < KP; ++m) {
      const int c = tid + m * nt;
      if (c < tot) ((u32x4*)tileb)[c] = pf[m];
    }
    const int Lz = (int)(nB.y >> 16), nzB = (int)(nB.y & 0xffff);
    const uint32_t boff = (uint32_t)(relax_tile_off(A.max_len) + 16 * (size_t)sg[TM]);
    if (tid == 0) {
      const uint32_t na_[TM] = {nNa.x, nNa.y, nNa.z, nNa.w};
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        const uint32_t ab = (uint32_t)(relax_tile_off(A.max_len) + 16 * (size_t)sg[t]);
        const uint32_t rpo = ab + (uint32_t)mlp_align16(2 * (int64_t)na_[t]);
        zb[t] = make_int4((int)ab, (int)rpo, (int)(rpo + (uint32_t)mlp_align16(2 * (int64_t)(Lxt[t] + 2))),
                          (int)na_[t]);
      }
    }
    __syncthreads();
    more = next();
    ++zcount;
#ifdef MLP_RELAX_NOSTAGE
    nB = fB; nAo = fAo; nNa = fNa;
#else
#ifdef MLP_RELAX_SAMEADDR
    nB = fB; nAo = fAo; nNa = fNa;
#endif
    if (more) MLP_ISSUE();
#endif
    {
      const float* Bvals = (const float*)(lds + boff);
      const uint32_t* Bhdr = (const uint32_t*)(lds + boff + (uint32_t)mlp_align16(4 * (int64_t)nzB));
      const uint2* Bwords = (const uint2*)((const uint8_t*)Bhdr + (uint32_t)mlp_align16(4 * (int64_t)(Lz + 1)));
#pragma unroll
      for (int s = 0; s < SL; ++s) {
        const int ti = (int)(tio[s] & 0xffff);
#ifdef MLP_RELAX_NOCOMPUTE  // timing experiment: staging only
        continue;
#endif
        if (ti == 0) continue;
        const int4 z4 = zb[tio[s] >> 16];
        if (z4.w == 0) continue;
        const uint16_t* Acols = (const uint16_t*)(lds + z4.x);
        const uint16_t* Arp = (const uint16_t*)(lds + z4.y);
        const float* Avals = (const float*)(lds + z4.z);
        const int a0 = Arp[ti], a1 = Arp[ti + 1];
        // two A entries per iteration (the second a zero-weight copy of the
        // first past the row end: + 0.0f leaves a positive sum unchanged)
        for (int t = a0; t < a1; t += 2) {
          const bool two = t + 1 < a1;
          const int k0 = Acols[t], k1 = Acols[two ? t + 1 : t];
          const float av0 = Avals[t];
          const float av1 = two ? Avals[t + 1] : 0.f;
          const uint32_t h0 = Bhdr[k0], h1 = Bhdr[k1];
          // word of column word jw in row k: woff + (jw - c0w), valid iff jw - c0w < nw
          const int o0 = (int)(h0 & 0xffff) - (int)((h0 >> 16) & 0xff);
          const int o1 = (int)(h1 & 0xffff) - (int)((h1 >> 16) & 0xff);
          const uint32_t c00 = (h0 >> 16) & 0xff, c01 = (h1 >> 16) & 0xff;
          const uint32_t nw0 = h0 >> 24, nw1 = h1 >> 24;
          uint2 w0[NC], w1[NC];
#pragma unroll
          for (int c = 0; c < NC; ++c) {  // unchecked: |jw - c0w| < 256 words stays in LDS
            w0[c] = Bwords[o0 + (int)jw[s][c]];
            w1[c] = Bwords[o1 + (int)jw[s][c]];
          }
          float b0[NC], b1[NC];
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            const uint32_t below = bm[s][c] - 1u;
            const bool h0c = (jw[s][c] - c00 < nw0) && (w0[c].x & bm[s][c]);
            const bool h1c = (jw[s][c] - c01 < nw1) && (w1[c].x & bm[s][c]);
            const uint32_t i0 = w0[c].y + __popc(w0[c].x & below);
            const uint32_t i1 = w1[c].y + __popc(w1[c].x & below);
            b0[c] = *(h0c ? Bvals + i0 : zero);
            b1[c] = *(h1c ? Bvals + i1 : zero);
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
    const int ti = (int)(tio[s] & 0xffff);
    if (ti == 0) continue;
    const int g = tid + s * nt;
    const int t = (int)(tio[s] >> 16);
    const int4 o = oinf[t];
    const int64_t exy = A.ent_off[o.x];
    const int e0 = A.rowptr[A.rp_off[o.x] + ti] + NC * (g - o.z - tp[t * tps + ti]);
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
static hipError_t launch_tiles_kp(const TileRelaxArgs& a, int slots, size_t lds, hipStream_t st) {
  const dim3 grid((unsigned)a.ntiles), block(kRelaxThreads);
  switch (slots) {
#define MLP_RELAX_CASE(SL)                                                                  \
  case SL:                                                                                  \
    hipFuncSetAttribute((const void*)k_relax_tile<KP, SL>,                                  \
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);              \
    hipLaunchKernelGGL((k_relax_tile<KP, SL>), grid, block, lds, st, a);                    \
    break;
    MLP_RELAX_CASE(2)
    MLP_RELAX_CASE(4)
#undef MLP_RELAX_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_relax_tiles(const TileRelaxArgs& a, int slots, hipStream_t st) {
  if (a.ntiles <= 0) return hipSuccess;
  const size_t lds = tile_relax_lds(a.cap, a.max_len);
  const char* kp = getenv("MLP_RELAX_KP");  // test hook: force the large-prefetch variant
  switch (kp ? atoi(kp) : tile_relax_prefetch(a.cap)) {
    case 6: return launch_tiles_kp<6>(a, slots, lds, st);
    case 12: return launch_tiles_kp<12>(a, slots, lds, st);
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
