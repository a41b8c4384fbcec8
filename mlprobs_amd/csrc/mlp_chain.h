// mlp_chain.h -- device-side machinery shared by the chained-wavefront
// sweeps (posterior.hip, viterbi.hip): LDS tables, chain staging, the per-lane
// cursor over stacked rows and the double-buffered strip boundary.  See
// mlp_kernels.h ("Chains") for the schedule.
#pragma once
#include "mlp_kernels.h"
#include "mlp_numerics.h"

namespace mlp {

#define LZ MLP_LOG_ZERO

// LDS-resident tables of one workgroup: letter-indexed emissions, the PF
// score factors and the LOOKUP coefficient rows (one ds_read_b128 per
// LOG_ADD instead of compare/select chains).  Only the parts a kernel's
// model set reads are staged: LDS bounds the sweeps' occupancy (the HMM
// tables are 3 KB, the PF factors 5.4 KB).
template <bool H> struct LdsHmmPart {
  float4 lk[kLookupRows];
  float match[26 * 26];
};
template <> struct LdsHmmPart<false> {};
template <bool P> struct LdsPfPart { double sub[26 * 26]; };
template <> struct LdsPfPart<false> {};
template <bool R> struct LdsPfRecip { double rsub[26 * 26]; };   // the PF backward's quotient only
template <> struct LdsPfRecip<false> {};
template <bool H, bool P, bool R = false>
struct LdsTablesT : LdsHmmPart<H>, LdsPfPart<P>, LdsPfRecip<R> {
  float ins[26];   // row insert emissions (every cursor)
};
// RECIP: the PF backward sweep, which also reads the reciprocals
template <int M, bool RECIP = false>
using LdsTablesFor = LdsTablesT<(M & (kHmm5 | kLocal)) != 0, (M & kPF) != 0, RECIP && (M & kPF) != 0>;

template <bool H, bool P, bool R>
__device__ __forceinline__ void stage_tables(LdsTablesT<H, P, R>& L, const Tables* __restrict__ tab) {
  for (int k = threadIdx.x; k < 26 * 26; k += blockDim.x) {
    if constexpr (H) L.match[k] = tab->match[k];
    if constexpr (P) L.sub[k] = tab->sub[k];
    if constexpr (R) L.rsub[k] = tab->rsub[k];
  }
  if (threadIdx.x < 26) L.ins[threadIdx.x] = tab->ins[threadIdx.x];
  if constexpr (H) {
    if (threadIdx.x == 0) mlp_lookup_table(L.lk);
  }
  __syncthreads();
}
template <bool H, bool P, bool R>
__device__ __forceinline__ const float4* lookup_of(const LdsTablesT<H, P, R>& L) {
  if constexpr (H) return L.lk;
  else return nullptr;
}

__device__ __forceinline__ int64_t wave_index() {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  return (int64_t)blockIdx.x * (blockDim.x >> 6) + w;
}

__device__ __forceinline__ float readlane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  const int2 w = *reinterpret_cast<const int2*>(&v);
  int2 r;
  r.x = __builtin_amdgcn_readlane(w.x, l);
  r.y = __builtin_amdgcn_readlane(w.y, l);
  return *reinterpret_cast<double*>(&r);
}

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------- chains
// LDS copy of one chain member's bookkeeping (80 bytes).
struct ChainPair {
  int L1, L2, row0, roff, coff, slot;
  float T5, TL;      // merge: pair totals
  int64_t rm, ell;   // local-chain base, first ELL row
  double zmant;      // backward: PF total
  int zexp, pad;
  double rzmant;     // backward: 1 / zmant
  double pad2;
};
// each wave's LDS region: the members' bookkeeping (count + 1 entries),
// then the residues (chain_lds_pack)
__host__ __device__ constexpr int chain_lds_meta(int lds) {
  return (int)sizeof(ChainPair) * ((lds >> 24) + 1);
}
__host__ __device__ constexpr int chain_lds_stride(int lds) {
  return chain_lds_meta(lds) + (((lds & 0xffffff) + 15) & ~15);
}

struct ChainView {
  const ChainPair* P;   // K + 1 entries, P[K].row0 = rows
  const uint8_t* seq;   // residues of all members
  int K, W, rows, S;
  int64_t ell0;         // the first member's first ELL row (members' rows follow in slot order)
};

enum StageKind { kStageFwd = 0, kStageBwd = 1, kStageMerge = 2 };

// Stage the chain's members (bookkeeping + both residue strings) into this
// wave's LDS region.
template <int KIND>
__device__ ChainView stage_chain(uint8_t* dyn, int lds_seq, int64_t ch, SeqSet sq, PairMeta pm,
                                 ChainMeta cm, const PairRec* __restrict__ rec) {
  const int lane = threadIdx.x & 63;
  uint8_t* region = dyn + (threadIdx.x >> 6) * chain_lds_stride(lds_seq);
  ChainPair* P = reinterpret_cast<ChainPair*>(region);
  uint8_t* seq = region + chain_lds_meta(lds_seq);
  const int K = cm.count[ch], first = cm.first[ch];
  int L1 = 0, L2 = 0, a = 0, b = 0;
  if (lane < K) {
    a = pm.pa[first + lane];
    b = pm.pb[first + lane];
    L1 = sq.len[a];
    L2 = sq.len[b];
  }
  const int W = cm.width[ch];
  // residue layout: [W + 2 zeros: idle lanes] then per member
  //   row seq padded  0, s1[0..L1-1], 0          (L1 + 2 bytes; c1 = [i], c1n = [i+1])
  //   col seq padded  0, s2[0..L2-1], 0 .. 0     (W + 1 bytes; c2 = [j], c2n = [j+1])
  int x = lane < K ? L1 + W + 3 : 0;
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  const int roff = W + 2 + x - (lane < K ? L1 + W + 3 : 0);
  if (lane < K) {
    const int slot = first + lane;
    ChainPair c;
    c.L1 = L1; c.L2 = L2; c.row0 = pm.row0[slot]; c.roff = roff; c.coff = roff + L1 + 2; c.slot = slot;
    c.T5 = 0.f; c.TL = 0.f; c.rm = pm.rm_off[slot]; c.ell = pm.ell_row[slot];
    c.zmant = 1.0; c.zexp = 0; c.pad = 0; c.rzmant = 1.0; c.pad2 = 0.0;
    if constexpr (KIND == kStageBwd) {
      c.zmant = rec[slot].zmant;
      c.zexp = rec[slot].zexp;
      c.rzmant = 1.0 / c.zmant;
    }
    if constexpr (KIND == kStageMerge) {
      // CPNP/ProbabilisticModel.h:405-454: T = (T_fwd + T_bwd) / 2; the
      // 5-state backward total was folded into b5[0] by k_fold_totals
      const PairRec& r = rec[slot];
      c.T5 = (r.tf5 + r.b5[0]) / 2;
      c.TL = (r.tfl + r.tbl) / 2;
    }
    P[lane] = c;
  }
  if (lane == 0) P[K].row0 = cm.rows[ch];
  const int total = __shfl(x, 63) + W + 2;
  for (int k = lane * 4; k < total; k += 256) *reinterpret_cast<uint32_t*>(seq + k) = 0u;
  wave_sync_lds();
  for (int q = 0; q < K; ++q) {
    const int aq = __shfl(a, q), bq = __shfl(b, q);
    const int l1 = __shfl(L1, q), l2 = __shfl(L2, q), ro = __shfl(roff, q);
    const uint8_t* s1 = sq.res + sq.off[aq];
    const uint8_t* s2 = sq.res + sq.off[bq];
    for (int k = lane; k < l1; k += 64) seq[ro + 1 + k] = s1[k];
    for (int k = lane; k < l2; k += 64) seq[ro + l1 + 2 + 1 + k] = s2[k];
  }
  wave_sync_lds();
  ChainView v;
  v.P = P;
  v.seq = seq;
  v.K = K;
  v.W = W;
  v.rows = cm.rows[ch];
  v.S = chain_strips(v.rows);
  v.ell0 = pm.ell_row[first];
  return v;
}

// Where one lane is in the chain: stacked row g (idle outside [0, rows)),
// column j, member q and its row i, plus the member's values the sweeps need.
// The per-row thresholds turn the sweeps' per-step edge and end tests into
// one compare of j each (set when the lane enters a row, i.e. once per W
// steps): a forward cell takes every recurrence (i >= 1, j >= 1, not (1, 1))
// iff j >= jlo; a backward cell is inside its pair (not the last row or
// column) iff j < jhi; the pair's last cell is j == jend; the backward's
// first-cell records (rows 0 and 1, columns 0 and 1) need j <= jfirst.
struct Cursor {
  int g, j, q, i, L1, L2;
  int ca;          // LDS offset of column residue j (padded column seq + j)
  int c1, c1n;     // residues i and i + 1 of the row sequence (0 outside)
  int c1x, c1nx;   // 26 c1, 26 c1n: the rows of the match table
  float ins1, ins1n;
  int slot;
  int64_t rm, ell;
  float T5, TL;
  double zmant, rzmant;
  int zexp;
  int jlo, jhi, jend, jfirst, jact;   // jact: L2 (an active row) or -1 (idle)
  int jpf;   // PF backward: the cell is off rows 1, L1 and columns 1, L2 iff 2 <= j < jpf
  int jm;    // merge: a cell of the pair (i >= 1, 1 <= j <= L2) iff (unsigned)(j - 1) < jm
  uint32_t ellr;  // merge: the row's first ELL slot from the chain's first, (ell - ell0 + i - 1) * kEll
};

__device__ __forceinline__ void locate(Cursor& c, const ChainView& C, const float* __restrict__ ins) {
  if (c.g < 0 || c.g >= C.rows) {
    c.q = -1; c.i = -1; c.L1 = -1; c.L2 = -1; c.c1 = 0; c.c1n = 0; c.c1x = 0; c.c1nx = 0;
    c.ca = c.j;   // the zero area
    c.ins1 = ins[0]; c.ins1n = ins[0];
    c.jlo = 1 << 30; c.jhi = 0; c.jend = -1; c.jfirst = -1; c.jact = -1; c.jpf = 2; c.jm = 0; c.ellr = 0;
    return;
  }
  int q = c.q < 0 ? 0 : c.q;
  while (C.P[q + 1].row0 <= c.g) ++q;
  while (C.P[q].row0 > c.g) --q;
  const ChainPair& m = C.P[q];
  c.q = q;
  c.i = c.g - m.row0;
  c.L1 = m.L1;
  c.L2 = m.L2;
  c.ca = m.coff + c.j;
  c.slot = m.slot;
  c.rm = m.rm;
  c.ell = m.ell;
  c.T5 = m.T5;
  c.TL = m.TL;
  c.zmant = m.zmant;
  c.rzmant = m.rzmant;
  c.zexp = m.zexp;
  c.c1 = C.seq[m.roff + c.i];
  c.c1n = C.seq[m.roff + c.i + 1];
  c.c1x = 26 * c.c1;
  c.c1nx = 26 * c.c1n;
  c.ins1 = ins[c.c1];
  c.ins1n = ins[c.c1n];
  c.jlo = c.i >= 2 ? 1 : c.i == 1 ? 2 : 1 << 30;
  c.jhi = c.i < c.L1 ? c.L2 : 0;
  c.jend = c.i == c.L1 ? c.L2 : -1;
  c.jfirst = c.i <= 1 ? 1 : -1;
  c.jact = c.L2;
  c.jpf = c.i >= 2 && c.i < c.L1 && c.L2 > 2 ? c.L2 : 2;
  c.jm = c.i >= 1 ? c.L2 : 0;
  c.ellr = (uint32_t)(c.ell - C.ell0 + c.i - 1) * (uint32_t)kEll;
}

// forward-order cursor at step 0: lane r at u = -r
__device__ __forceinline__ void cursor_start_fwd(Cursor& c, const ChainView& C, const float* ins, int lane) {
  c.q = -1;
  c.g = lane == 0 ? 0 : lane - 64;
  c.j = lane == 0 ? 0 : C.W - lane;
  locate(c, C, ins);
}
// on_row(): the sweep's own per-row state, after the lane entered its next row
struct NoRowState {
  __device__ void operator()() const {}
};
template <class F = NoRowState>
__device__ __forceinline__ void cursor_next(Cursor& c, const ChainView& C, const float* ins, F on_row = F()) {
  ++c.ca;
  if (++c.j == C.W) {
    c.j = 0;
    c.g += 64;
    locate(c, C, ins);
    on_row();
  }
}
// reverse-order cursor at step tau (u = tau - lane >= 0)
__device__ __forceinline__ void cursor_start_bwd(Cursor& c, const ChainView& C, const float* ins, int lane, int tau) {
  const int u = tau - lane;
  c.q = -1;
  c.g = 64 * (u / C.W) + lane;
  c.j = u % C.W;
  locate(c, C, ins);
}
template <class F = NoRowState>
__device__ __forceinline__ void cursor_prev(Cursor& c, const ChainView& C, const float* ins, F on_row = F()) {
  --c.ca;
  if (--c.j < 0) {
    c.j = C.W - 1;
    c.g -= 64;
    locate(c, C, ins);
    on_row();
  }
}

// ---- scalar-addressed buffer access: a wave-uniform base built on the
// scalar unit (a raw buffer resource; word 3 = 0x00020000, the gfx9
// family's 32-bit data format) plus a loop-invariant per-lane byte offset,
// so the sweeps' per-step loads and stores cost no VALU address arithmetic
// (global stores took one or two 64-bit adds each)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
typedef unsigned mlp_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void bstore(const float* base, uint32_t boff, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), wave_rsrc(base), boff, 0, 0);
}
__device__ __forceinline__ void bstore(const int32_t* base, uint32_t boff, int32_t v) {
  __builtin_amdgcn_raw_buffer_store_b32((unsigned)v, wave_rsrc(base), boff, 0, 0);
}
__device__ __forceinline__ void bstore(const double* base, uint32_t boff, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(mlp_u32x2, v), wave_rsrc(base), boff, 0, 0);
}
__device__ __forceinline__ void bstore(const uint16_t* base, uint32_t boff, uint16_t v) {
  __builtin_amdgcn_raw_buffer_store_b16(v, wave_rsrc(base), boff, 0, 0);
}
typedef unsigned mlp_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void bstore4(const float* base, uint32_t boff, float4 v) {
  const mlp_u32x4 u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(u, wave_rsrc(base), boff, 0, 0);
}
__device__ __forceinline__ void bstore4(const uint16_t* base, uint32_t boff, uint4 v) {
  const mlp_u32x4 u = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(u, wave_rsrc(base), boff, 0, 0);
}
__device__ __forceinline__ void bstore2(const uint16_t* base, uint32_t boff, uint2 v) {
  const mlp_u32x2 u = {v.x, v.y};
  __builtin_amdgcn_raw_buffer_store_b64(u, wave_rsrc(base), boff, 0, 0);
}
__device__ __forceinline__ float bload(const float* base, uint32_t boff) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(wave_rsrc(base), boff, 0, 0));
}
__device__ __forceinline__ double bload(const double* base, uint32_t boff) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(wave_rsrc(base), boff, 0, 0));
}

// A chain's boundary rows are stored column-major, one 32-byte record per
// column: the HMMs' (bnd5) the 5-state values then the local model's three,
// the partition function's (bndz) its three doubles then the frame.  The one
// lane that crosses the strip stores its column's record: the column of that
// lane at a step is wave-uniform (a scalar counter), so the stores' whole
// address is scalar, two 16-byte stores a step where one store per component
// took eight, and consecutive steps fill a line in four steps instead of each
// component's line in 32 (the component-major rows before left L2 lines
// partly written).  A chunk's load is two 16-byte loads a lane, contiguous
// across the lanes.
template <class T>
__device__ __forceinline__ void bnd_put(const T* comp, int j_uniform, T v) { bstore(comp + j_uniform, 0, v); }
__device__ __forceinline__ void bnd_put_hmm(const float* recs, int j_uniform, float4 a, float4 b) {
  bstore4(recs + 8 * j_uniform, 0, a);
  bstore4(recs + 8 * j_uniform + 4, 0, b);
}
__device__ __forceinline__ void bnd_put_pf(const double* recs, int j_uniform, double m, double e, double f, int E) {
  const uint64_t um = (uint64_t)__double_as_longlong(m), ue = (uint64_t)__double_as_longlong(e);
  const uint64_t uf = (uint64_t)__double_as_longlong(f);
  const mlp_u32x4 a = {(uint32_t)um, (uint32_t)(um >> 32), (uint32_t)ue, (uint32_t)(ue >> 32)};
  const mlp_u32x4 b = {(uint32_t)uf, (uint32_t)(uf >> 32), (uint32_t)E, 0u};
  __builtin_amdgcn_raw_buffer_store_b128(a, wave_rsrc(recs + 4 * j_uniform), 0, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b128(b, wave_rsrc(recs + 4 * j_uniform + 2), 0, 0, 0);
}
// a column's records into the loader's registers
__device__ __forceinline__ void bnd_get_hmm(const Scratch& sc, int64_t bo, uint32_t col, float* n5, float* nl) {
  const float4* r = reinterpret_cast<const float4*>(sc.bnd5 + bo * 8) + 2 * (int64_t)col;
  const float4 a = r[0], b = r[1];
  n5[0] = a.x; n5[1] = a.y; n5[2] = a.z; n5[3] = a.w; n5[4] = b.x;
  nl[0] = b.y; nl[1] = b.z; nl[2] = b.w;
}
__device__ __forceinline__ void bnd_get_pf(const Scratch& sc, int64_t bo, uint32_t col, double* nz, int& ne) {
  const uint4* r = reinterpret_cast<const uint4*>(sc.bndz + bo * 4) + 2 * (int64_t)col;
  const uint4 a = r[0], b = r[1];
  nz[0] = __longlong_as_double((long long)(((uint64_t)a.y << 32) | a.x));
  nz[1] = __longlong_as_double((long long)(((uint64_t)a.w << 32) | a.z));
  nz[2] = __longlong_as_double((long long)(((uint64_t)b.y << 32) | b.x));
  ne = (int)b.z;
}

// Boundary row of the neighbouring strip, read 64 columns at a time (one per
// lane) and double-buffered: the sweeps switch buffers between 64-step
// segments, so the chunk in use is loop-invariant in the step loop and was
// loaded a whole segment earlier -- reading it never waits on the loads and
// stores issued since (vmcnt is in order on gfx9).  Column indices are
// clamped to the chain's W columns; columns a lane must not use are never
// consumed by an active cell.
template <int M>
struct BoundaryChunks {
  float c5[5], n5[5], cl[3], nl[3];
  double cz[3], nz[3];
  int ce, ne;
  // back: lanes the chunk is loaded shifted up by, so that lane 63 holds the
  // segment's first column (the backward sweep's partial segments)
  __device__ __forceinline__ void load_next(const Scratch& sc, int64_t bo, int W, int col0, int lane, int back = 0) {
    const uint32_t col = (uint32_t)min(max(col0 + lane - back, 0), W - 1);
    if constexpr ((M & (kHmm5 | kLocal)) != 0) bnd_get_hmm(sc, bo, col, n5, nl);
    if constexpr ((M & kPF) != 0) bnd_get_pf(sc, bo, col, nz, ne);
  }
  uint8_t* area = nullptr;   // (interface of LdsBoundaryChunks; unused)
  __device__ __forceinline__ void advance(int) { advance(); }
  __device__ __forceinline__ void advance() {
#pragma unroll
    for (int k = 0; k < 5; ++k) c5[k] = n5[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) { cl[k] = nl[k]; cz[k] = nz[k]; }
    ce = ne;
  }
  // Neighbour shift of one step: X = src shifted by one lane toward higher
  // lanes (SHR, forward) or lower lanes (backward); the vacated lane (0 / 63)
  // takes the current chunk's column for this step when TAKE, else 0 (unused
  // there).  The chunk rotates one lane per step (toward lane 0 forward,
  // toward lane 63 backward), so that column is always in the vacated lane
  // and enters through the DPP shift's `old` operand: no readlane per value.
  // TAKE steps of a segment run consecutively from its first column.
  // (Round 3 read the column with readlane instead.)
  template <bool SHR, bool TAKE>
  __device__ __forceinline__ void shift(int q, const float* S5, float* X5, const float* SL, float* XL,
                                        double sZm, double sZe, double sZf, int se,
                                        double& Zm, double& Ze, double& Zf, int& e) {
    (void)q;
    if constexpr ((M & kHmm5) != 0) {
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        X5[k] = TAKE ? (SHR ? mlp_shr1(S5[k], c5[k]) : mlp_shl1(S5[k], c5[k]))
                     : (SHR ? mlp_shr1z(S5[k]) : mlp_shl1z(S5[k]));
        if (TAKE) c5[k] = SHR ? mlp_shl1z(c5[k]) : mlp_shr1z(c5[k]);
      }
    }
    if constexpr ((M & kLocal) != 0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        XL[k] = TAKE ? (SHR ? mlp_shr1(SL[k], cl[k]) : mlp_shl1(SL[k], cl[k]))
                     : (SHR ? mlp_shr1z(SL[k]) : mlp_shl1z(SL[k]));
        if (TAKE) cl[k] = SHR ? mlp_shl1z(cl[k]) : mlp_shr1z(cl[k]);
      }
    }
    if constexpr ((M & kPF) != 0) {
      if constexpr (TAKE) {
        Zm = SHR ? mlp_shr1d(sZm, cz[0]) : mlp_shl1d(sZm, cz[0]);
        Ze = SHR ? mlp_shr1d(sZe, cz[1]) : mlp_shl1d(sZe, cz[1]);
        Zf = SHR ? mlp_shr1d(sZf, cz[2]) : mlp_shl1d(sZf, cz[2]);
        e = SHR ? mlp_shr1i(se, ce) : mlp_shl1i(se, ce);
#pragma unroll
        for (int k = 0; k < 3; ++k) cz[k] = SHR ? mlp_shl1zd(cz[k]) : mlp_shr1zd(cz[k]);
        ce = SHR ? mlp_shl1zi(ce) : mlp_shr1zi(ce);
      } else {
        Zm = SHR ? mlp_shr1zd(sZm) : mlp_shl1zd(sZm);
        Ze = SHR ? mlp_shr1zd(sZe) : mlp_shl1zd(sZe);
        Zf = SHR ? mlp_shr1zd(sZf) : mlp_shl1zd(sZf);
        e = SHR ? mlp_shr1zi(se) : mlp_shl1zi(se);
      }
    }
  }
};

// The same boundary chunk staged in LDS (the posterior sweeps): at a
// segment's start every lane writes its column of the chunk loaded a segment
// earlier into this wave's 64-column area, and each step all lanes read the
// step's column (one address: a broadcast) into the register the DPP shift
// keeps in the vacated lane.  Against the rotating chunk registers this
// drops one DPP move per component and step (8 per step in the 5-state +
// local sweeps, 7 in the partition function's) for two LDS reads.
template <int M>
struct LdsChunkLayout {
  static constexpr int raw = ((M & kHmm5) ? 20 : 0) + ((M & kLocal) ? 12 : 0) + ((M & kPF) ? 28 : 0);
  static constexpr int bytes = (raw + 15) & ~15;   // per column
  static constexpr int o5 = 0, ol = (M & kHmm5) ? 20 : 0, oz = ol + ((M & kLocal) ? 12 : 0), oe = oz + 24;
};
template <int M>
struct LdsBoundaryChunks {
  using Lay = LdsChunkLayout<M>;
  float n5[5] = {}, nl[3] = {};   // (the first segment's chunk is never read by an active cell)
  double nz[3] = {};
  int ne = 0;
  uint8_t* area;   // this wave's 64 x Lay::bytes
  __device__ __forceinline__ void load_next(const Scratch& sc, int64_t bo, int W, int col0, int lane, int back = 0) {
    const uint32_t col = (uint32_t)min(max(col0 + lane - back, 0), W - 1);
    if constexpr ((M & (kHmm5 | kLocal)) != 0) bnd_get_hmm(sc, bo, col, n5, nl);
    if constexpr ((M & kPF) != 0) bnd_get_pf(sc, bo, col, nz, ne);
  }
  // the loaded chunk becomes the current one: this lane's column into LDS
  // (the wave's reads of the previous chunk precede it in LDS order)
  __device__ __forceinline__ void advance(int lane) {
    uint32_t w[Lay::bytes / 4] = {};
    if constexpr ((M & kHmm5) != 0) {
#pragma unroll
      for (int k = 0; k < 5; ++k) w[Lay::o5 / 4 + k] = __float_as_uint(n5[k]);
    }
    if constexpr ((M & kLocal) != 0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) w[Lay::ol / 4 + k] = __float_as_uint(nl[k]);
    }
    if constexpr ((M & kPF) != 0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const uint64_t b = (uint64_t)__double_as_longlong(nz[k]);
        w[Lay::oz / 4 + 2 * k] = (uint32_t)b;
        w[Lay::oz / 4 + 2 * k + 1] = (uint32_t)(b >> 32);
      }
      w[Lay::oe / 4] = (uint32_t)ne;
    }
    uint4* dst = reinterpret_cast<uint4*>(area + lane * Lay::bytes);
#pragma unroll
    for (int k = 0; k < Lay::bytes / 16; ++k) dst[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
  }
  // as BoundaryChunks::shift; col: the LDS address of the chunk column this
  // step takes (the caller forms it once per group of unrolled steps, the
  // steps' offsets then fold into the reads)
  template <bool SHR>
  __device__ __forceinline__ void shift_at(const uint8_t* col, const float* S5, float* X5, const float* SL,
                                           float* XL, double sZm, double sZe, double sZf, int se, double& Zm,
                                           double& Ze, double& Zf, int& e) {
    uint32_t w[Lay::bytes / 4];
    const uint4* src = reinterpret_cast<const uint4*>(col);
#pragma unroll
    for (int k = 0; k < Lay::bytes / 16; ++k) {
      const uint4 v = src[k];
      w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
    }
    if constexpr ((M & kHmm5) != 0) {
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const float o = __uint_as_float(w[Lay::o5 / 4 + k]);
        X5[k] = SHR ? mlp_shr1(S5[k], o) : mlp_shl1(S5[k], o);
      }
    }
    if constexpr ((M & kLocal) != 0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float o = __uint_as_float(w[Lay::ol / 4 + k]);
        XL[k] = SHR ? mlp_shr1(SL[k], o) : mlp_shl1(SL[k], o);
      }
    }
    if constexpr ((M & kPF) != 0) {
      double o[3];
#pragma unroll
      for (int k = 0; k < 3; ++k)
        o[k] = __longlong_as_double((long long)(((uint64_t)w[Lay::oz / 4 + 2 * k + 1] << 32) | w[Lay::oz / 4 + 2 * k]));
      Zm = SHR ? mlp_shr1d(sZm, o[0]) : mlp_shl1d(sZm, o[0]);
      Ze = SHR ? mlp_shr1d(sZe, o[1]) : mlp_shl1d(sZe, o[1]);
      Zf = SHR ? mlp_shr1d(sZf, o[2]) : mlp_shl1d(sZf, o[2]);
      e = SHR ? mlp_shr1i(se, (int)w[Lay::oe / 4]) : mlp_shl1i(se, (int)w[Lay::oe / 4]);
    }
  }
};

// Stores of the boundary row before a segment's chunk load must be visible
// to it (same wave, other lanes): order them once per 64-step segment.
__device__ __forceinline__ void boundary_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}


struct ChainLaunch {
  dim3 grid, block;
  size_t lds;
};
// 4 waves (chains) per workgroup; 1 when a chain's residues need a large
// LDS region.
static inline ChainLaunch chain_launch(int64_t nchains, int lds_seq) {
  const int stride = chain_lds_stride(lds_seq);
  const int wpb = stride * kWavesPerBlock <= 40 * 1024 ? kWavesPerBlock : 1;
  ChainLaunch l;
  l.grid = dim3((unsigned)((nchains + wpb - 1) / wpb));
  l.block = dim3(64 * wpb);
  l.lds = (size_t)stride * wpb;
  return l;
}


}  // namespace mlp
