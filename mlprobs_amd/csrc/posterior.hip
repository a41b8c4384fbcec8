// posterior.hip -- all-pairs pairwise posterior kernels for gfx950 (CDNA4).
//
// Replaces the per-pair body of the pdoAlign pair loop (CPNP/MSA.cpp:939-1025):
//   5-state double-affine pair-HMM forward/backward (CPNP/ProbabilisticModel.h:153-395),
//   3-state local pair-HMM forward/backward (same functions, flag = false),
//   global partition function (CPNP/MSAPartProbs.cpp:78-727),
//   totals + posteriors (CPNP/ProbabilisticModel.h:405-493),
//   RMS merge (CPNP/MSA.cpp:992-1007), MEA (CPNP/ProbabilisticModel.h:804-864),
//   distance (CPNP/MSA.cpp:1019-1020) and sparsification (CPNP/SparseMatrix.h:55-98).
//
// Execution model: one 64-lane wave per pair.  The pair's DP matrix (rows
// 0..L1 = seq1 prefix, columns 0..L2 = seq2 prefix) is cut into strips of 64
// rows; lane r owns row 64*s + r and visits column j = t - r at step t (an
// anti-diagonal wavefront).  The up / down neighbour arrives through a DPP
// wave shift (v_mov_b32_dpp wave_shr:1 / wave_shl:1), the diagonal is the
// previous step's neighbour value, the left / right value stays in the lane.
// Strip-to-strip rows go through a small per-pair boundary column buffer.
// Cell values are stored in a strip-diagonal layout
//     idx = cell_off + ((s * strip_steps(L2)) + t) * 64 + lane
// so every store / load of a step is one coalesced 256-byte wave access.
//
// All float arithmetic reproduces the reference's operation order exactly
// (see mlp_numerics.h); the partition function runs in scaled fp64 instead
// of x87 long double.
#include "mlp_kernels.h"
#include "mlp_numerics.h"

#include <type_traits>

namespace mlp {

#define LZ MLP_LOG_ZERO

// LDS-resident tables of one workgroup: letter-indexed emissions, the PF
// score factors and the LOOKUP coefficient sets (one ds_read_b128 per
// LOG_ADD instead of twelve selects).
// Residue supply: the residue a lane needs at step t is the residue its
// upper neighbour needed one step earlier, so residues flow down the wave by
// DPP; only lane 0 / 63 takes a new one, read with v_readlane out of a
// 64-residue chunk loaded once per 64 steps.
struct ResidueChunk {
  int chunk;
  int base;
  __device__ __forceinline__ void init() { base = -(1 << 30); chunk = 0; }
  // residue code at position q (0-based) of seq, 0 outside [0, len).
  __device__ __forceinline__ int get(const uint8_t* seq, int len, int q) {
    const int cb = q & ~63;
    if (cb != base) {
      base = cb;
      const int pos = cb + (int)(threadIdx.x & 63);
      chunk = (pos >= 0 && pos < len) ? (int)seq[pos] : 0;
    }
    const int v = __builtin_amdgcn_readlane(chunk, q & 63);
    return (q >= 0 && q < len) ? v : 0;
  }
};

struct LdsTables {
  float4 lk[kLookupRows];
  float match[26 * 26];
  float ins[26];
  double sub[26 * 26];
  uint8_t seq[kWavesPerBlock][kSeqLds];
};

// Column residues of this wave's pair: staged in LDS (no VMEM wait in the
// step loop); LONG kernels (L2 > kSeqLds) use the chunked global path.
template <bool LONG>
struct ColumnResidues {
  const uint8_t* lds;
  const uint8_t* glob;
  int len;
  ResidueChunk rc;
  __device__ __forceinline__ void init(uint8_t* buf, const uint8_t* g, int L) {
    lds = buf; glob = g; len = L; rc.init();
    if constexpr (!LONG) {
      for (int k = threadIdx.x & 63; k < L; k += 64) buf[k] = g[k];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  __device__ __forceinline__ int get(int q) {
    if constexpr (!LONG) return (q >= 0 && q < len) ? (int)lds[q] : 0;
    else return rc.get(glob, len, q);
  }
};

__device__ __forceinline__ void stage_tables(LdsTables& L, const Tables* __restrict__ tab) {
  for (int k = threadIdx.x; k < 26 * 26; k += blockDim.x) {
    L.match[k] = tab->match[k];
    L.sub[k] = tab->sub[k];
  }
  if (threadIdx.x < 26) L.ins[threadIdx.x] = tab->ins[threadIdx.x];
  if (threadIdx.x == 0) mlp_lookup_table(L.lk);
  __syncthreads();
}

__device__ __forceinline__ int64_t wave_pair_index() {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  return (int64_t)blockIdx.x * kWavesPerBlock + w;
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

// Boundary row of the neighbouring strip, read 64 columns at a time (one per
// lane) and double-buffered: the sweeps run their steps in chunks of 64 and
// switch buffers between chunks, so the chunk in use is loop-invariant in the
// step loop and was loaded a whole chunk earlier -- reading it never waits on
// the loads and stores issued since (vmcnt is in order on gfx9).  Loads use
// clamped addresses; out-of-range columns are masked at take().
template <int M>
struct BoundaryChunks {
  float c5[5], n5[5], cl[3], nl[3];
  double cz[3], nz[3];
  int ce, ne;
  __device__ __forceinline__ void load_next(const Scratch& sc, int64_t bo, int L2, int col0, int lane) {
    const int col = col0 + lane;
    const int64_t bi = bo + min(max(col, 0), L2);
    if constexpr ((M & kHmm5) != 0) {
#pragma unroll
      for (int k = 0; k < 5; ++k) n5[k] = sc.bnd5[bi * 5 + k];
    }
    if constexpr ((M & kLocal) != 0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) nl[k] = sc.bndl[bi * 3 + k];
    }
    if constexpr ((M & kPF) != 0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) nz[k] = sc.bndz[bi * 3 + k];
      ne = sc.bnde[bi];
    }
  }
  __device__ __forceinline__ void advance() {
#pragma unroll
    for (int k = 0; k < 5; ++k) c5[k] = n5[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) { cl[k] = nl[k]; cz[k] = nz[k]; }
    ce = ne;
  }
  // the value of column q of the current chunk into lane `who`'s neighbour
  // state; `ok` (wave-uniform) = the column lies inside 0..L2
  __device__ __forceinline__ void take(int q, bool ok, bool who, float* X5, float* XL,
                                       double& Zm, double& Ze, double& Zf, int& e) const {
    if constexpr ((M & kHmm5) != 0) {
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const float v = ok ? readlane_f(c5[k], q) : LZ;
        X5[k] = who ? v : X5[k];
      }
    }
    if constexpr ((M & kLocal) != 0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float v = ok ? readlane_f(cl[k], q) : LZ;
        XL[k] = who ? v : XL[k];
      }
    }
    if constexpr ((M & kPF) != 0) {
      const double z0 = ok ? readlane_d(cz[0], q) : 0.0, z1 = ok ? readlane_d(cz[1], q) : 0.0;
      const double z2 = ok ? readlane_d(cz[2], q) : 0.0;
      const int ee = ok ? __builtin_amdgcn_readlane(ce, q) : 0;
      Zm = who ? z0 : Zm; Ze = who ? z1 : Ze; Zf = who ? z2 : Zf; e = who ? ee : e;
    }
  }
};

// Depth of the software-pipelined loads of the backward step loop.
constexpr int kPrefetch = 4;

// Bring three scaled-fp64 frames to their common maximum (exact: powers of two).
__device__ __forceinline__ int pf_align(double& a0, double& a1, double& a2, int ea,
                                        double& b0, double& b1, double& b2, int eb,
                                        double& c0, double& c1, double& c2, int ec) {
  const int E = max(max(ea, eb), ec);
  if (ea != E) { const int k = -MLP_PF_STEP * (E - ea); a0 = ldexp(a0, k); a1 = ldexp(a1, k); a2 = ldexp(a2, k); }
  if (eb != E) { const int k = -MLP_PF_STEP * (E - eb); b0 = ldexp(b0, k); b1 = ldexp(b1, k); b2 = ldexp(b2, k); }
  if (ec != E) { const int k = -MLP_PF_STEP * (E - ec); c0 = ldexp(c0, k); c1 = ldexp(c1, k); c2 = ldexp(c2, k); }
  return E;
}
__device__ __forceinline__ void pf_rescale(double& zm, double& ze, double& zf, int& E) {
  if (fmax(fmax(zm, ze), zf) > MLP_PF_HUGE) {
    zm *= 0x1p-200; ze *= 0x1p-200; zf *= 0x1p-200;
    E += 1;
  }
}

// =====================================================================
// Forward: 5-state, local and partition-function forward in one sweep.
// Steps where every lane is an interior cell (rows 2..L1-1, columns
// 2..L2-1) take a branch-free path; the others evaluate the reference's
// boundary conditions per lane.
// =====================================================================
template <int M, bool LONG>
__global__ __launch_bounds__(256) void k_forward(ModelScalars ms, const Tables* __restrict__ tab,
                                                 SeqSet sq, PairMeta pm, PairRec* __restrict__ rec,
                                                 Scratch sc, int64_t npairs) {
  __shared__ LdsTables T_;
  stage_tables(T_, tab);
  const int64_t p = wave_pair_index();
  if (p >= npairs) return;
  const float4* __restrict__ lk = T_.lk;
  const int lane = threadIdx.x & 63;
  const int a = pm.pa[p], b = pm.pb[p];
  const int L1 = sq.len[a], L2 = sq.len[b];
  const uint8_t* __restrict__ s1 = sq.res + sq.off[a];
  const uint8_t* __restrict__ s2 = sq.res + sq.off[b];
  const int S = (L1 + 64) >> 6;
  const int T = strip_steps(L2);
  const int64_t cbase = pm.cell_off[p];
  const int64_t rmb = pm.rm_off[p];
  const int Wp = (L2 + 3) & ~3;
  const int64_t bo = pm.bnd_off[p];
  const float rt1 = ms.rt1, two_rt1 = 2 * ms.rt1;
  const double pfo = ms.pf_open, pfe = ms.pf_ext;
  int pf_over = 0;
  ColumnResidues<LONG> cres;
  cres.init(T_.seq[(threadIdx.x >> 6)], s2, L2);

  for (int s = 0; s < S; ++s) {
    const int i = (s << 6) + lane;
    const bool row_ok = i <= L1;
    const int c1 = (i >= 1 && i <= L1) ? (int)s1[i - 1] : 0;
    const float ins1 = T_.ins[c1];
    const bool strip_interior = s >= 1 && (s << 6) + 63 <= L1 - 1;
    // per-lane state: Lx = own cell at j-1, Ux = cell (i-1, j), Dx = (i-1, j-1)
    float L5[5], U5[5], D5[5];
    float LL[3], UL[3], DL[3];
    double LZm = 0, LZe = 0, LZf = 0, UZm = 0, UZe = 0, UZf = 0, DZm = 0, DZe = 0, DZf = 0;
    int Le = 0, Ue = 0, De = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k) L5[k] = U5[k] = D5[k] = LZ;
#pragma unroll
    for (int k = 0; k < 3; ++k) LL[k] = UL[k] = DL[k] = LZ;
    // row-major chain staging; unused slots stay LOG_ZERO, a no-op in the chain
    float cb0 = LZ, cb1 = LZ, cb2 = LZ, cb3 = LZ;
    int c2 = 0;
    BoundaryChunks<M> bc;
    if (s > 0) {
      bc.load_next(sc, bo, L2, 0, lane);
      bc.advance();
      bc.load_next(sc, bo, L2, 64, lane);
    }

    for (int c = 0; (c << 6) < T; ++c) {
    if (s > 0 && c > 0) {
      bc.advance();
      bc.load_next(sc, bo, L2, (c + 1) << 6, lane);
    }
    const int tend = min(T, (c << 6) + 64);
    for (int t = c << 6; t < tend; ++t) {
      const int j = t - lane;
      const int c2new = cres.get(t - 1);   // residue j: s2[j-1]
      c2 = mlp_shr1i(c2, c2new);
      if constexpr ((M & kHmm5) != 0) {
#pragma unroll
        for (int k = 0; k < 5; ++k) { D5[k] = U5[k]; U5[k] = mlp_shr1(L5[k], LZ); }
      }
      if constexpr ((M & kLocal) != 0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) { DL[k] = UL[k]; UL[k] = mlp_shr1(LL[k], LZ); }
      }
      if constexpr ((M & kPF) != 0) {
        DZm = UZm; DZe = UZe; DZf = UZf; De = Ue;
        UZm = mlp_shr1d(LZm, 0.0); UZe = mlp_shr1d(LZe, 0.0); UZf = mlp_shr1d(LZf, 0.0);
        Ue = mlp_shr1i(Le, 0);
      }
      if (s > 0) {
        // lane 0 takes row 64*s-1, column t, from the boundary buffer
        bc.take(t & 63, t <= L2, lane == 0, U5, UL, UZm, UZe, UZf, Ue);
      }

      const int64_t idx = cbase + ((int64_t)s * T + t) * 64 + lane;
      auto cell = [&](auto int_tag) {
        constexpr bool INT = decltype(int_tag)::value;
        const bool act = INT || (row_ok && j >= 0 && j <= L2);
        const bool gen = INT || (i > 1 || j > 1);
        // ------------------------------------------------ 5-state forward
        if constexpr ((M & kHmm5) != 0) {
          const float m = T_.match[c1 * 26 + c2];
          const float ins2 = T_.ins[c2];
          // CPNP/ProbabilisticModel.h:213-256
          float vm = D5[0] + ms.t[0][0];
          vm = mlp_log_add_t(vm, D5[1] + ms.t[1][0], lk);
          vm = mlp_log_add_t(vm, D5[2] + ms.t[2][0], lk);
          vm = mlp_log_add_t(vm, D5[3] + ms.t[3][0], lk);
          vm = mlp_log_add_t(vm, D5[4] + ms.t[4][0], lk);
          vm = vm + m;
          const float vx1 = ins1 + mlp_log_add_t(U5[0] + ms.t[0][1], U5[1] + ms.t[1][1], lk);
          const float vx2 = ins1 + mlp_log_add_t(U5[0] + ms.t[0][3], U5[3] + ms.t[3][3], lk);
          const float vy1 = ins2 + mlp_log_add_t(L5[0] + ms.t[0][2], L5[2] + ms.t[2][2], lk);
          const float vy2 = ins2 + mlp_log_add_t(L5[0] + ms.t[0][4], L5[4] + ms.t[4][4], lk);
          float C[5];
          if constexpr (INT) {
            C[0] = vm; C[1] = vx1; C[2] = vy1; C[3] = vx2; C[4] = vy2;
          } else {
#pragma unroll
            for (int k = 0; k < 5; ++k) C[k] = LZ;
            // CPNP/ProbabilisticModel.h:173-183 initial cells
            if (i == 1 && j == 1) C[0] = ms.init[0] + m;
            if (i == 1 && j == 0) { C[1] = ms.init[1] + ins1; C[3] = ms.init[3] + ins1; }
            if (i == 0 && j == 1) { C[2] = ms.init[2] + ins2; C[4] = ms.init[4] + ins2; }
            if (gen) {
              if (i > 0 && j > 0) C[0] = vm;
              if (i > 0) { C[1] = vx1; C[3] = vx2; }
              if (j > 0) { C[2] = vy1; C[4] = vy2; }
            }
          }
          sc.f5[idx] = C[0];   // every lane: inactive slots of the strip are never read
          if (act) {
            if (!INT && i == L1 && j == L2) {  // CPNP/ProbabilisticModel.h:415-419 (forward half)
              float tf = LZ;
#pragma unroll
              for (int k = 0; k < 5; ++k) tf = mlp_log_add_t(tf, C[k] + ms.init[k], lk);
              rec[p].tf5 = tf;
            }
            if (lane == 63) {
#pragma unroll
              for (int k = 0; k < 5; ++k) sc.bnd5[(bo + j) * 5 + k] = C[k];
            }
          }
#pragma unroll
          for (int k = 0; k < 5; ++k) L5[k] = C[k];
        }
        // ------------------------------------------------ local forward
        if constexpr ((M & kLocal) != 0) {
          const float m = T_.match[c1 * 26 + c2];
          const float ins2 = T_.ins[c2];
          const float base = m - ins1 - ins2;
          float vm = base - two_rt1;
          vm = mlp_log_add_t(vm, base + DL[0] + ms.lt[0][0] - two_rt1, lk);
          vm = mlp_log_add_t(vm, base + DL[1] + ms.lt[1][0] - two_rt1, lk);
          vm = mlp_log_add_t(vm, base + DL[2] + ms.lt[2][0] - two_rt1, lk);
          const float vx = mlp_log_add_t(UL[0] + ms.lt[0][1] - rt1, UL[1] + ms.lt[1][1] - rt1, lk);
          const float vy = mlp_log_add_t(LL[0] + ms.lt[0][2] - rt1, LL[2] + ms.lt[2][2] - rt1, lk);
          float Cm = vm, Cx = vx, Cy = vy;
          if constexpr (!INT) {
            Cm = LZ; Cx = LZ; Cy = LZ;
            if (i == 1 && j == 1) Cm = base - two_rt1;
            if (gen) {
              if (i > 0 && j > 0) Cm = vm;
              if (i > 0) Cx = vx;
              if (j > 0) Cy = vy;
            }
          }
          sc.fl[idx] = Cm;
          if (act) {
            if (lane == 63) {
              sc.bndl[(bo + j) * 3 + 0] = Cm;
              sc.bndl[(bo + j) * 3 + 1] = Cx;
              sc.bndl[(bo + j) * 3 + 2] = Cy;
            }
          }
          // row-major chain copy of interior M values (CPNP/ProbabilisticModel.h:438-447)
          if (act && (INT || (i >= 1 && j >= 1))) {
            const int q = (j - 1) & 3;
            cb0 = q == 0 ? Cm : cb0;
            cb1 = q == 1 ? Cm : cb1;
            cb2 = q == 2 ? Cm : cb2;
            cb3 = q == 3 ? Cm : cb3;
            if (q == 3 || (!INT && j == L2)) {
              *reinterpret_cast<float4*>(sc.chf + rmb + (int64_t)(i - 1) * Wp + ((j - 1) & ~3)) =
                  make_float4(cb0, cb1, cb2, cb3);
              cb0 = cb1 = cb2 = cb3 = LZ;
            }
          }
          LL[0] = Cm; LL[1] = Cx; LL[2] = Cy;
        }
        // ------------------------------------------------ partition function forward
        if constexpr ((M & kPF) != 0) {
          // cell (i, j) <-> reference Zm[ip = j][jp = i] (CPNP/MSAPartProbs.cpp:510-609)
          double Zm, Ze, Zf;
          int E;
          const double score = T_.sub[c2 * 26 + c1];
          if constexpr (INT) {
            E = pf_align(UZm, UZe, UZf, Ue, DZm, DZe, DZf, De, LZm, LZe, LZf, Le);
            Ze = UZm * pfo + UZe * pfe;
            Zf = LZm * pfo + LZf * pfe;
            Zm = (DZm + DZe + DZf) * score;
            pf_rescale(Zm, Ze, Zf, E);
          } else if (i == 0) {
            Zm = (j == 0) ? 1.0 : 0.0; Ze = 0.0; Zf = (j >= 1) ? 1.0 : 0.0; E = 0;
          } else if (j == 0) {
            Zm = 0.0; Ze = 1.0; Zf = 0.0; E = 0;
          } else {
            E = pf_align(UZm, UZe, UZf, Ue, DZm, DZe, DZf, De, LZm, LZe, LZf, Le);
            const double o0 = (j == L2) ? 1.0 : pfo, e0 = (j == L2) ? 1.0 : pfe;
            const double o1 = (i == L1) ? 1.0 : pfo, e1 = (i == L1) ? 1.0 : pfe;
            Ze = UZm * o0 + UZe * e0;
            Zf = LZm * o1 + LZf * e1;
            Zm = (DZm + DZe + DZf) * score;
            pf_rescale(Zm, Ze, Zf, E);
          }
          sc.zm[idx] = mlp_pf_pack(Zm, E);
          if (act) {
            pf_over |= (E > 250);
            if (!INT && i == L1 && j == L2) {  // CPNP/MSAPartProbs.cpp:591,612
              rec[p].zmant = (Zm + Ze) + Zf;
              rec[p].zexp = E;
            }
            if (lane == 63) {
              sc.bndz[(bo + j) * 3 + 0] = Zm;
              sc.bndz[(bo + j) * 3 + 1] = Ze;
              sc.bndz[(bo + j) * 3 + 2] = Zf;
              sc.bnde[bo + j] = E;
            }
          }
          LZm = Zm; LZe = Ze; LZf = Zf; Le = E;
        }
      };
      if (strip_interior && t >= 65 && t <= L2 - 1) cell(std::true_type{});
      else cell(std::false_type{});
    }
    }
    // the next strip's lane 0 reads what lane 63 wrote
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  }
  if constexpr ((M & kPF) != 0) {
    if (__any(pf_over)) {
      if (lane == 0) atomicOr(&rec[p].flags, 1);
    }
  }
}

// =====================================================================
// Backward: reverse sweep; emits f+b (in place), PF posterior, chains.
// Interior steps: rows 2..L1-1, columns 2..L2-1 on every lane.
// =====================================================================
template <int M, bool LONG>
__global__ __launch_bounds__(256) void k_backward(ModelScalars ms, const Tables* __restrict__ tab,
                                                  SeqSet sq, PairMeta pm, PairRec* __restrict__ rec,
                                                  Scratch sc, int64_t npairs) {
  __shared__ LdsTables T_;
  stage_tables(T_, tab);
  const int64_t p = wave_pair_index();
  if (p >= npairs) return;
  const float4* __restrict__ lk = T_.lk;
  const int lane = threadIdx.x & 63;
  const int a = pm.pa[p], b = pm.pb[p];
  const int L1 = sq.len[a], L2 = sq.len[b];
  const uint8_t* __restrict__ s1 = sq.res + sq.off[a];
  const uint8_t* __restrict__ s2 = sq.res + sq.off[b];
  const int S = (L1 + 64) >> 6;
  const int T = strip_steps(L2);
  const int64_t cbase = pm.cell_off[p];
  const int64_t rmb = pm.rm_off[p];
  const int Wp = (L2 + 3) & ~3;
  const int64_t bo = pm.bnd_off[p];
  const float rt1 = ms.rt1, two_rt1 = 2 * ms.rt1;
  const double pfo = ms.pf_open, pfe = ms.pf_ext;
  const double zmant = (M & kPF) ? rec[p].zmant : 1.0;
  const int zexp = (M & kPF) ? rec[p].zexp : 0;
  ColumnResidues<LONG> cres;
  cres.init(T_.seq[(threadIdx.x >> 6)], s2, L2);

  for (int s = S - 1; s >= 0; --s) {
    const int i = (s << 6) + lane;
    const bool row_ok = i <= L1;
    const int c1 = (i >= 1 && i <= L1) ? (int)s1[i - 1] : 0;   // residue i
    const int c1n = (i < L1) ? (int)s1[i] : 0;                  // residue i+1
    const float ins1 = T_.ins[c1], ins1n = T_.ins[c1n];
    const bool strip_interior = s >= 1 && (s << 6) + 63 <= L1 - 1;
    // Rx = own cell (i, j+1), Nx = (i+1, j), Gx = (i+1, j+1)
    float R5[5], N5[5], G5[5];
    float RL[3], NL[3], GL[3];
    double RZm = 0, RZe = 0, RZf = 0, NZm = 0, NZe = 0, NZf = 0, GZm = 0, GZe = 0, GZf = 0;
    int Re = 0, Ne = 0, Ge = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k) R5[k] = N5[k] = G5[k] = LZ;
#pragma unroll
    for (int k = 0; k < 3; ++k) RL[k] = NL[k] = GL[k] = LZ;
    float cb0 = LZ, cb1 = LZ, cb2 = LZ, cb3 = LZ;
    int c2n = 0;  // residue j+1
    BoundaryChunks<M> bc;
    const int c_top = (T - 1) >> 6;
    if (s < S - 1) {
      bc.load_next(sc, bo, L2, (c_top << 6) - 63, lane);
      bc.advance();
      bc.load_next(sc, bo, L2, ((c_top - 1) << 6) - 63, lane);
    }
    // the step-t loads of f5 / fl / zm are issued kPrefetch steps earlier;
    // every slot of the strip was written by the forward sweep, values of
    // inactive cells are never used
    const int64_t sbase = cbase + (int64_t)s * T * 64 + lane;
    // queue slot u always serves steps t0 - u: the loop is unrolled by
    // kPrefetch (T is a multiple of 8) so every slot is a fixed register
    float q5[kPrefetch] = {}, ql[kPrefetch] = {};
    double qz[kPrefetch] = {};
#pragma unroll
    for (int k = 0; k < kPrefetch; ++k) {
      const int tt = T - 1 - k;
      if constexpr ((M & kHmm5) != 0) q5[k] = sc.f5[sbase + (int64_t)tt * 64];
      if constexpr ((M & kLocal) != 0) ql[k] = sc.fl[sbase + (int64_t)tt * 64];
      if constexpr ((M & kPF) != 0) qz[k] = sc.zm[sbase + (int64_t)tt * 64];
    }

    for (int c = c_top; c >= 0; --c) {
    if (s < S - 1 && c < c_top) {
      bc.advance();
      bc.load_next(sc, bo, L2, ((c - 1) << 6) - 63, lane);
    }
    // T - 1 = 7 (mod 8): every chunk holds a whole number of unrolled groups
    for (int t0 = min(T - 1, (c << 6) + 63); t0 >= (c << 6); t0 -= kPrefetch)
#pragma unroll
    for (int u = 0; u < kPrefetch; ++u) {
      const int t = t0 - u;
      const int j = t - lane;
      const float f5v = q5[u], flv = ql[u];
      const double zmv = qz[u];
      // residues: lane 63 takes s2[j] for its column j = t - 63
      c2n = mlp_shl1i(c2n, cres.get(t - 63));
      // residue j (current column) = c2n of lane+1 at this step
      const int c2 = mlp_shl1i(c2n, cres.get(t - 64));
      if constexpr ((M & kHmm5) != 0) {
#pragma unroll
        for (int k = 0; k < 5; ++k) { G5[k] = N5[k]; N5[k] = mlp_shl1(R5[k], LZ); }
      }
      if constexpr ((M & kLocal) != 0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) { GL[k] = NL[k]; NL[k] = mlp_shl1(RL[k], LZ); }
      }
      if constexpr ((M & kPF) != 0) {
        GZm = NZm; GZe = NZe; GZf = NZf; Ge = Ne;
        NZm = mlp_shl1d(RZm, 0.0); NZe = mlp_shl1d(RZe, 0.0); NZf = mlp_shl1d(RZf, 0.0);
        Ne = mlp_shl1i(Re, 0);
      }
      if (s < S - 1) {
        // lane 63 takes row 64*(s+1), column t-63, from the boundary buffer
        const int col = t - 63;
        bc.take(t & 63, col >= 0 && col <= L2, lane == 63, N5, NL, NZm, NZe, NZf, Ne);
      }

      const int64_t idx = cbase + ((int64_t)s * T + t) * 64 + lane;
      auto cell = [&](auto int_tag) {
        constexpr bool INT = decltype(int_tag)::value;
        const bool act = INT || (row_ok && j >= 0 && j <= L2);
        const bool in_i = INT || i < L1;
        const bool in_j = INT || j < L2;
        // ------------------------------------------------ 5-state backward
        if constexpr ((M & kHmm5) != 0) {
          const float ins2n = T_.ins[c2n];
          const float mn = T_.match[c1n * 26 + c2n];
          float B[5];
          // CPNP/ProbabilisticModel.h:310-313, 340-378
          const float pxy = G5[0] + mn;
          if constexpr (INT) {
#pragma unroll
            for (int k = 0; k < 5; ++k) B[k] = mlp_log_add_from_zero(pxy + ms.t[k][0]);
          } else {
            const bool last = (i == L1 && j == L2);
#pragma unroll
            for (int k = 0; k < 5; ++k)
              B[k] = last ? ms.init[k] : ((in_i && in_j) ? mlp_log_add_from_zero(pxy + ms.t[k][0]) : LZ);
          }
          if (in_i) {
            B[0] = mlp_log_add_t(B[0], N5[1] + ins1n + ms.t[0][1], lk);
            B[1] = mlp_log_add_t(B[1], N5[1] + ins1n + ms.t[1][1], lk);
            B[0] = mlp_log_add_t(B[0], N5[3] + ins1n + ms.t[0][3], lk);
            B[3] = mlp_log_add_t(B[3], N5[3] + ins1n + ms.t[3][3], lk);
          }
          if (in_j) {
            B[0] = mlp_log_add_t(B[0], R5[2] + ins2n + ms.t[0][2], lk);
            B[2] = mlp_log_add_t(B[2], R5[2] + ins2n + ms.t[2][2], lk);
            B[0] = mlp_log_add_t(B[0], R5[4] + ins2n + ms.t[0][4], lk);
            B[4] = mlp_log_add_t(B[4], R5[4] + ins2n + ms.t[4][4], lk);
          }
          sc.f5[idx] = f5v + B[0];   // f + b (CPNP/ProbabilisticModel.h:484)
          if (act) {
            if (!INT) {
              if (i == 1 && j == 1) rec[p].b5[0] = B[0];
              if (i == 1 && j == 0) { rec[p].b5[1] = B[1]; rec[p].b5[3] = B[3]; }
              if (i == 0 && j == 1) { rec[p].b5[2] = B[2]; rec[p].b5[4] = B[4]; }
            }
            if (lane == 0) {
#pragma unroll
              for (int k = 0; k < 5; ++k) sc.bnd5[(bo + j) * 5 + k] = B[k];
            }
          }
#pragma unroll
          for (int k = 0; k < 5; ++k) R5[k] = B[k];
        }
        // ------------------------------------------------ local backward
        if constexpr ((M & kLocal) != 0) {
          const float ins2n = T_.ins[c2n];
          const float mn = T_.match[c1n * 26 + c2n];
          float Bm = MLP_LOG_ONE, Bx = LZ, By = LZ;
          if (in_i && in_j) {
            const float pxy = GL[0] + mn - ins1n - ins2n;
            Bm = mlp_log_add_t(Bm, pxy + ms.lt[0][0] - two_rt1, lk);
            Bx = mlp_log_add_from_zero(pxy + ms.lt[1][0] - two_rt1);
            By = mlp_log_add_from_zero(pxy + ms.lt[2][0] - two_rt1);
          }
          if (in_i) {
            Bm = mlp_log_add_t(Bm, NL[1] + ms.lt[0][1] - rt1, lk);
            Bx = mlp_log_add_t(Bx, NL[1] + ms.lt[1][1] - rt1, lk);
          }
          if (in_j) {
            Bm = mlp_log_add_t(Bm, RL[2] + ms.lt[0][2] - rt1, lk);
            By = mlp_log_add_t(By, RL[2] + ms.lt[2][2] - rt1, lk);
          }
          sc.fl[idx] = flv + Bm;
          if (act) {
            if (lane == 0) {
              sc.bndl[(bo + j) * 3 + 0] = Bm;
              sc.bndl[(bo + j) * 3 + 1] = Bx;
              sc.bndl[(bo + j) * 3 + 2] = By;
            }
          }
          // chain element (CPNP/ProbabilisticModel.h:444-445)
          if (act && (INT || (i >= 1 && j >= 1))) {
            const float e = Bm + T_.match[c1 * 26 + c2] - ins1 - T_.ins[c2] - two_rt1;
            const int q = (j - 1) & 3;
            cb0 = q == 0 ? e : cb0;
            cb1 = q == 1 ? e : cb1;
            cb2 = q == 2 ? e : cb2;
            cb3 = q == 3 ? e : cb3;
            if (q == 0) {
              *reinterpret_cast<float4*>(sc.chb + rmb + (int64_t)(i - 1) * Wp + (j - 1)) =
                  make_float4(cb0, cb1, cb2, cb3);
              cb0 = cb1 = cb2 = cb3 = LZ;
            }
          }
          RL[0] = Bm; RL[1] = Bx; RL[2] = By;
        }
        // ------------------------------------------------ partition function reverse
        if constexpr ((M & kPF) != 0) {
          // cell (i, j) <-> reverse Zm[ip = j-1][jp = i-1] (CPNP/MSAPartProbs.cpp:233-321)
          double Zm = 0, Ze = 0, Zf = 0;
          int E = 0;
          float post = 0.0f;
          const double score = T_.sub[c2 * 26 + c1];
          if (INT || (i >= 1 && j >= 1)) {
            double nZm = NZm, nZe = NZe, nZf = NZf, rZm = RZm, rZe = RZe, rZf = RZf;
            double gZm = GZm, gZe = GZe, gZf = GZf;
            int ne = Ne, re = Re, ge = Ge;
            double o0 = pfo, e0 = pfe, o1 = pfo, e1 = pfe;
            if constexpr (!INT) {
              // boundary row L1+1 / column L2+1 (init of CPNP/MSAPartProbs.cpp:217-226)
              if (i == L1) { nZm = 0.0; nZf = 1.0; nZe = 0.0; ne = 0; }
              if (j == L2) { rZm = 0.0; rZf = 0.0; rZe = 1.0; re = 0; }
              if (j == L2) {
                const bool corner = (i == L1);
                gZm = corner ? 1.0 : 0.0; gZf = 0.0; gZe = corner ? 0.0 : 1.0; ge = 0;
              } else if (i == L1) {
                gZm = 0.0; gZf = 1.0; gZe = 0.0; ge = 0;
              }
              if (j == 1) { o0 = 1.0; e0 = 1.0; }
              if (i == 1) { o1 = 1.0; e1 = 1.0; }
            }
            E = pf_align(nZm, nZe, nZf, ne, rZm, rZe, rZf, re, gZm, gZe, gZf, ge);
            Zf = rZm * o1 + rZf * e1;
            Ze = nZm * o0 + nZe * e0;
            Zm = (gZm + gZf + gZe) * score;
            pf_rescale(Zm, Ze, Zf, E);
            if (act) {
              int ef;
              const double zf = mlp_pf_unpack(zmv, &ef);
              const double q = (zf * Zm) / (score * zmant);
              post = (float)ldexp(q, MLP_PF_STEP * (ef + E - zexp));
            }
          }
          sc.pg[idx] = post;
          if (act) {
            if (lane == 0) {
              sc.bndz[(bo + j) * 3 + 0] = Zm;
              sc.bndz[(bo + j) * 3 + 1] = Ze;
              sc.bndz[(bo + j) * 3 + 2] = Zf;
              sc.bnde[bo + j] = E;
            }
          }
          RZm = Zm; RZe = Ze; RZf = Zf; Re = E;
        }
      };
      if (strip_interior && t >= 65 && t <= L2 - 1) cell(std::true_type{});
      else cell(std::false_type{});
      // refill slot u after its value is dead, so the load reuses the register
      // (a loop-carried copy of a pending load would drain vmcnt)
      const int tt = max(t - kPrefetch, 0);
      if constexpr ((M & kHmm5) != 0) q5[u] = sc.f5[sbase + (int64_t)tt * 64];
      if constexpr ((M & kLocal) != 0) ql[u] = sc.fl[sbase + (int64_t)tt * 64];
      if constexpr ((M & kPF) != 0) qz[u] = sc.zm[sbase + (int64_t)tt * 64];
    }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  }
}

// =====================================================================
// Local-model totals: the reference sums LOG_PLUS_EQUALS over all interior
// cells in row-major order (CPNP/ProbabilisticModel.h:435-450), a single
// non-associative chain, for the forward and the backward half.
//
// One lane per pair walks its two chains serially (the exact reference
// order; rows are padded to a multiple of 4 with LOG_ZERO, a no-op element).
// A wave owns 64 pairs and stages 16-element tiles of all 64 chains through
// LDS with coalesced loads.  Inside a tile an element x is folded with the
// exact LOG_ADD unless acc - x >= 7.5, where LOG_ADD returns acc unchanged
// (CPNP/ScoreType.h:279-285), so the skip is exact.
// =====================================================================
constexpr int kTile = 32;
__global__ __launch_bounds__(64) void k_local_totals_lane(SeqSet sq, PairMeta pm, PairRec* __restrict__ rec,
                                                          Scratch sc, int64_t npairs) {
  __shared__ float tf_t[64][kTile + 1];
  __shared__ float tb_t[64][kTile + 1];
  const int lane = threadIdx.x;
  const int64_t g0 = (int64_t)blockIdx.x * 64;
  const int64_t p = g0 + lane;
  int64_t ne = 0, base = 0;
  if (p < npairs) {
    const int L1 = sq.len[pm.pa[p]], L2 = sq.len[pm.pb[p]];
    ne = (int64_t)L1 * ((L2 + 3) & ~3);
    base = pm.rm_off[p];
  }
  int64_t emax = ne;
  for (int off = 32; off >= 1; off >>= 1) emax = max(emax, (int64_t)__shfl_xor(emax, off));
  // loader geometry: 8 lanes x float4 cover one pair's 32-element tile;
  // 8 rounds cover the 64 pairs
  const int part = lane & 7;
  int64_t nq[8], bq[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int q = k * 8 + (lane >> 3);
    nq[k] = __shfl(ne, q);
    bq[k] = __shfl(base, q);
  }
  float4 pf[8], pb[8];
  auto load = [&](int64_t e0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t e = e0 + part * 4;
      pf[k] = make_float4(LZ, LZ, LZ, LZ);
      pb[k] = pf[k];
      if (e < nq[k]) {
        pf[k] = *reinterpret_cast<const float4*>(sc.chf + bq[k] + e);
        pb[k] = *reinterpret_cast<const float4*>(sc.chb + bq[k] + e);
      }
    }
  };
  float tf = LZ, tb = LZ;
  load(0);
  for (int64_t e0 = 0; e0 < emax; e0 += kTile) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int q = k * 8 + (lane >> 3);
      tf_t[q][part * 4 + 0] = pf[k].x; tf_t[q][part * 4 + 1] = pf[k].y;
      tf_t[q][part * 4 + 2] = pf[k].z; tf_t[q][part * 4 + 3] = pf[k].w;
      tb_t[q][part * 4 + 0] = pb[k].x; tb_t[q][part * 4 + 1] = pb[k].y;
      tb_t[q][part * 4 + 2] = pb[k].z; tb_t[q][part * 4 + 3] = pb[k].w;
    }
    __syncthreads();
    if (e0 + kTile < emax) load(e0 + kTile);  // prefetch the next tile meanwhile
#pragma unroll 8
    for (int u = 0; u < kTile; ++u) {
      const float xf = tf_t[lane][u], xb = tb_t[lane][u];
      tf = mlp_log_add(tf, xf);
      tb = mlp_log_add(tb, xb);
    }
    __syncthreads();
  }
  if (p < npairs) {
    rec[p].tfl = tf;
    rec[p].tbl = tb;
  }
}

// Variant: 8 lanes per pair, 8 pairs per wave.  Each group streams 8
// consecutive elements of its pair; every lane evaluates the exact LOG_ADD of
// the group's running total with its own element and the group adopts the
// result of its first pending candidate (a shuffle), so one wave instruction
// stream folds eight chains at once.
__device__ __forceinline__ float fold_group(float acc, float x, int sub, int gbase) {
  bool cand = !(acc - x >= 7.5f);
  while (true) {
    const uint64_t m = __ballot(cand);
    if (m == 0) break;
    const uint32_t gm = (uint32_t)(m >> gbase) & 0xFFu;
    const int first = gm ? __builtin_ctz(gm) : 8;
    const float v = mlp_log_add(acc, x);
    const float nv = __shfl(v, gbase + (first & 7));
    if (gm) acc = nv;
    cand = cand && (sub > first) && !(acc - x >= 7.5f);
  }
  return acc;
}

__global__ __launch_bounds__(256) void k_local_totals_grp(SeqSet sq, PairMeta pm, PairRec* __restrict__ rec,
                                                          Scratch sc, int64_t npairs) {
  const int lane = threadIdx.x & 63;
  const int sub = lane & 7, gbase = lane & ~7;
  const int64_t wave = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const int64_t p = wave * 8 + (lane >> 3);
  int64_t ne = 0, base = 0;
  if (p < npairs) {
    const int L1 = sq.len[pm.pa[p]], L2 = sq.len[pm.pb[p]];
    ne = (int64_t)L1 * ((L2 + 3) & ~3);
    base = pm.rm_off[p];
  }
  int64_t emax = ne;
  for (int off = 32; off >= 8; off >>= 1) emax = max(emax, (int64_t)__shfl_xor(emax, off));
  const float* __restrict__ cf = sc.chf + base;
  const float* __restrict__ cbk = sc.chb + base;
  float tf = LZ, tb = LZ;
  float xf = (sub < ne) ? cf[sub] : LZ, xb = (sub < ne) ? cbk[sub] : LZ;
  for (int64_t e0 = 0; e0 < emax; e0 += 8) {
    const float cxf = xf, cxb = xb;
    const int64_t en = e0 + 8 + sub;
    xf = LZ; xb = LZ;
    if (en < ne) { xf = cf[en]; xb = cbk[en]; }  // prefetch the next chunk
    tf = fold_group(tf, cxf, sub, gbase);
    tb = fold_group(tb, cxb, sub, gbase);
  }
  if (p < npairs && sub == 0) {
    rec[p].tfl = tf;
    rec[p].tbl = tb;
  }
}

// Variant: one wave per pair, candidates folded serially (see above).
__global__ __launch_bounds__(256) void k_local_totals_wave(SeqSet sq, PairMeta pm, PairRec* __restrict__ rec,
                                                           Scratch sc, int64_t npairs) {
  __shared__ float4 lk[kLookupRows];
  if (threadIdx.x == 0) mlp_lookup_table(lk);
  __syncthreads();
  const int64_t p = wave_pair_index();
  if (p >= npairs) return;
  const int lane = threadIdx.x & 63;
  const int L1 = sq.len[pm.pa[p]], L2 = sq.len[pm.pb[p]];
  const int64_t ne = (int64_t)L1 * ((L2 + 3) & ~3);
  const float* __restrict__ cf = sc.chf + pm.rm_off[p];
  const float* __restrict__ cbk = sc.chb + pm.rm_off[p];
  // lane 0 carries the forward chain, lane 1 the backward chain: one LOG_ADD
  // sequence advances both (LOG_ADD(acc, LOG_ZERO) == acc keeps an idle
  // chain unchanged)
  float acc = LZ;
  float tf = LZ, tb = LZ;   // wave-uniform copies
  float xf = LZ, xb = LZ;
  if (lane < ne) { xf = cf[lane]; xb = cbk[lane]; }
  for (int64_t c0 = 0; c0 < ne; c0 += 64) {
    const float cxf = xf, cxb = xb;
    const int64_t nx = c0 + 64 + lane;
    xf = LZ; xb = LZ;
    if (nx < ne) { xf = cf[nx]; xb = cbk[nx]; }   // prefetch next chunk
    uint64_t mf = __ballot(!(tf - cxf >= 7.5f));
    uint64_t mb = __ballot(!(tb - cxb >= 7.5f));
    while (mf | mb) {
      const float vf = mf ? readlane_f(cxf, __builtin_ctzll(mf)) : LZ;
      const float vb = mb ? readlane_f(cxb, __builtin_ctzll(mb)) : LZ;
      acc = mlp_log_add_t(acc, lane == 0 ? vf : vb, lk);
      tf = readlane_f(acc, 0);
      tb = readlane_f(acc, 1);
      if (mf) mf = (mf & (mf - 1)) & __ballot(!(tf - cxf >= 7.5f));
      if (mb) mb = (mb & (mb - 1)) & __ballot(!(tb - cxb >= 7.5f));
    }
  }
  if (lane == 0) {
    rec[p].tfl = tf;
    rec[p].tbl = tb;
  }
}

// Variant (default): 8 pairs per wave, 8 lanes per pair.  Chunks of 64
// elements per chain (8 per lane, two float4 loads); candidates of each
// chain (elements with acc - x < 7.5, acc = chain value at the chunk start)
// are compacted in order into LDS, then lanes 0..15 fold the 16 chains of the
// wave in parallel.  The candidate list is a superset of the elements that
// change acc: LOG_ADD(acc, x) for acc - x >= 7.5 returns acc exactly, so
// folding every listed element reproduces the reference's serial chain.
constexpr int kTotPairs = 8;   // pairs per wave
__global__ __launch_bounds__(256) void k_local_totals_multi(SeqSet sq, PairMeta pm, PairRec* __restrict__ rec,
                                                            Scratch sc, int64_t npairs) {
  __shared__ float4 lk[kLookupRows];
  __shared__ float list[kWavesPerBlock][2 * kTotPairs][64];
  if (threadIdx.x == 0) mlp_lookup_table(lk);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int g = lane >> 3, sub = lane & 7;
  const int64_t p = ((int64_t)blockIdx.x * kWavesPerBlock + w) * kTotPairs + g;
  int64_t ne = 0, base = 0;
  if (p < npairs) {
    const int L1 = sq.len[pm.pa[p]], L2 = sq.len[pm.pb[p]];
    ne = (int64_t)L1 * ((L2 + 3) & ~3);
    base = pm.rm_off[p];
  }
  int64_t emax = ne;
  for (int off = 32; off >= 8; off >>= 1) emax = max(emax, (int64_t)__shfl_xor(emax, off));
  const float* __restrict__ cf = sc.chf + base;
  const float* __restrict__ cb = sc.chb + base;
  // chain c = 2g (forward) / 2g+1 (backward) is folded on lane c
  float acc = LZ;
  float nf[8], nb[8];
  auto load = [&](int64_t e0, float* f, float* b) {
    const int64_t e = e0 + sub * 8;   // ne is a multiple of 4: float4 pieces are all-in or all-out
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float4 vf = make_float4(LZ, LZ, LZ, LZ), vb = vf;
      if (e + 4 * h < ne) {
        vf = *reinterpret_cast<const float4*>(cf + e + 4 * h);
        vb = *reinterpret_cast<const float4*>(cb + e + 4 * h);
      }
      f[4 * h + 0] = vf.x; f[4 * h + 1] = vf.y; f[4 * h + 2] = vf.z; f[4 * h + 3] = vf.w;
      b[4 * h + 0] = vb.x; b[4 * h + 1] = vb.y; b[4 * h + 2] = vb.z; b[4 * h + 3] = vb.w;
    }
  };
  // two chunks in flight: HBM latency exceeds one chunk's fold
  float nf2[8], nb2[8];
  load(0, nf, nb);
  load(64, nf2, nb2);
  // exclusive prefix of a per-lane count over the 8 lanes of its group
  auto group_scan = [&](int c) {
    int x = c;
#pragma unroll
    for (int d = 1; d < 8; d <<= 1) {
      const int y = __shfl_up(x, d, 8);
      x += (sub >= d) ? y : 0;
    }
    return x - c;
  };
  auto chunk = [&](int64_t e0, float* xf, float* xb) {
    const float af = __shfl(acc, 2 * g), ab = __shfl(acc, 2 * g + 1);
    const int64_t e = e0 + sub * 8;
    unsigned ff = 0, fb = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const bool in = e + k < ne;
      ff |= (in && !(af - xf[k] >= 7.5f)) ? (1u << k) : 0u;
      fb |= (in && !(ab - xb[k] >= 7.5f)) ? (1u << k) : 0u;
    }
    const int cf_n = __popc(ff), cb_n = __popc(fb);
    int pf = group_scan(cf_n), pb = group_scan(cb_n);
    float* lf = list[w][2 * g];
    float* lb = list[w][2 * g + 1];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (ff & (1u << k)) lf[pf++] = xf[k];
      if (fb & (1u << k)) lb[pb++] = xb[k];
    }
    // totals per chain: last lane of the group holds the inclusive sums
    const int tot_f = __shfl(pf, g * 8 + 7), tot_b = __shfl(pb, g * 8 + 7);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // chain `lane` (< 16) folds its list; count from its group's last lane
    const int cnt_f = __shfl(tot_f, (lane >> 1) * 8), cnt_b = __shfl(tot_b, (lane >> 1) * 8);
    const int cnt = lane < 2 * kTotPairs ? ((lane & 1) ? cnt_b : cnt_f) : 0;
    const float* my = list[w][lane & (2 * kTotPairs - 1)];
    for (int k = 0; __any(k < cnt); ++k) {
      if (k < cnt) acc = mlp_log_add_t(acc, my[k], lk);
    }
    __builtin_amdgcn_wave_barrier();
  };
  for (int64_t e0 = 0; e0 < emax; e0 += 128) {
    float xf[8], xb[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { xf[k] = nf[k]; xb[k] = nb[k]; }
    if (e0 + 128 < emax) load(e0 + 128, nf, nb);
    chunk(e0, xf, xb);
    if (e0 + 64 >= emax) break;
#pragma unroll
    for (int k = 0; k < 8; ++k) { xf[k] = nf2[k]; xb[k] = nb2[k]; }
    if (e0 + 192 < emax) load(e0 + 192, nf2, nb2);
    chunk(e0 + 64, xf, xb);
  }
  const float tf = __shfl(acc, 2 * g), tb = __shfl(acc, 2 * g + 1);
  if (p < npairs && sub == 0) {
    rec[p].tfl = tf;
    rec[p].tbl = tb;
  }
}

// =====================================================================
// Merge + MEA + sparsify: forward wavefront over the merged posterior.
// =====================================================================
template <int M, int PID>
__global__ __launch_bounds__(256) void k_merge(ModelScalars ms, SeqSet sq, PairMeta pm,
                                               PairRec* __restrict__ rec, Scratch sc, int64_t npairs) {
  __shared__ double ex[7 * 6];
  if (threadIdx.x == 0) mlp_exp_table(ex);
  __syncthreads();
  const int64_t p = wave_pair_index();
  if (p >= npairs) return;
  const int lane = threadIdx.x & 63;
  const int L1 = sq.len[pm.pa[p]], L2 = sq.len[pm.pb[p]];
  const int S = (L1 + 64) >> 6;
  const int T = strip_steps(L2);
  const int64_t cbase = pm.cell_off[p];
  const int64_t bo = pm.bnd_off[p];
  const int64_t er0 = pm.ell_row[p];
  // pair totals
  float T5 = 0.f, TL = 0.f;
  if constexpr ((M & kHmm5) != 0) {
    // CPNP/ProbabilisticModel.h:421-432 with the forward values of the
    // initial cells (CPNP/ProbabilisticModel.h:173-183)
    const PairRec& r = rec[p];
    const uint8_t* s1 = sq.res + sq.off[pm.pa[p]];
    const uint8_t* s2 = sq.res + sq.off[pm.pb[p]];
    (void)s1; (void)s2;
    float tb = r.b5[0];  // caller pre-adds forward parts (see fold_totals)
    T5 = (r.tf5 + tb) / 2;
  }
  if constexpr ((M & kLocal) != 0) TL = (rec[p].tfl + rec[p].tbl) / 2;
  int64_t my_nnz = 0;
  int ell_over = 0;
  float score = 0.f;
  for (int s = 0; s < S; ++s) {
    const int i = (s << 6) + lane;
    const bool row_ok = i >= 1 && i <= L1;
    float Lv = 0.f, Uv = 0.f, Dv = 0.f;
    int cnt = 0;
    const int64_t erow = er0 + (i - 1);
    // boundary row 64s-1 (MEA values), double-buffered as in BoundaryChunks
    float bch = 0.f, bnx = 0.f;
    if (s > 0) {
      bch = sc.bndm[bo + min(lane, L2)];
      bnx = sc.bndm[bo + min(64 + lane, L2)];
    }
    // slots of the strip written by the backward sweep; values of inactive
    // cells are never used
    const int64_t sbase = cbase + (int64_t)s * T * 64 + lane;
    constexpr int QD = 8;
    // fixed-register load queue: slot u serves steps t0 + u (T % QD == 0)
    float q5[QD] = {}, ql[QD] = {}, qg[QD] = {};
#pragma unroll
    for (int k = 0; k < QD; ++k) {
      if constexpr ((M & kHmm5) != 0) q5[k] = sc.f5[sbase + (int64_t)k * 64];
      if constexpr ((M & kLocal) != 0) ql[k] = sc.fl[sbase + (int64_t)k * 64];
      if constexpr ((M & kPF) != 0) qg[k] = sc.pg[sbase + (int64_t)k * 64];
    }
    for (int c = 0; (c << 6) < T; ++c) {
    if (s > 0 && c > 0) {
      bch = bnx;
      bnx = sc.bndm[bo + min(((c + 1) << 6) + lane, L2)];
    }
    const int tend = min(T, (c << 6) + 64);
    for (int t0 = c << 6; t0 < tend; t0 += QD)
#pragma unroll
    for (int u = 0; u < QD; ++u) {
      const int t = t0 + u;
      const int j = t - lane;
      const float f5v = q5[u], flv = ql[u], pgv = qg[u];
      Dv = Uv;
      Uv = mlp_shr1(Lv, 0.f);
      if (s > 0) {
        const float v = (t <= L2) ? readlane_f(bch, t & 63) : 0.f;
        if (lane == 0) Uv = v;
      }
      const bool act = row_ok && j >= 1 && j <= L2;
      const int64_t idx = cbase + ((int64_t)s * T + t) * 64 + lane;
      float P = 0.f;
      if (act) {
        if constexpr (PID == 2) {
          P = mlp_post_from_sum_t(flv, TL, ex);
        } else if constexpr (PID >= 3) {
          P = pgv;
        } else {
          const float v1 = mlp_post_from_sum_t(f5v, T5, ex);
          const float v2 = pgv;
          const float v3 = mlp_post_from_sum_t(flv, TL, ex);
          P = sqrtf((v1 * v1 + v2 * v2 + v3 * v3) / 3);
        }
      }
      // MEA (CPNP/ProbabilisticModel.h:831-834): value of ChooseBestOfThree
      float Cv = 0.f;
      if (act) {
        const float x1 = P + Dv, x2 = Lv, x3 = Uv;
        Cv = fmaxf(fmaxf(x1, x2), x3);
        if (P >= 0.01f) {  // POSTERIOR_CUTOFF (CPNP/SparseMatrix.h:14)
          if (cnt < kEll) {
            sc.ell_col[erow * kEll + cnt] = (uint16_t)j;
            sc.ell_val[erow * kEll + cnt] = P;
          } else {
            ell_over = 1;
          }
          ++cnt;
        }
        if (i == L1 && j == L2) score = Cv;
      }
      if (lane == 63 && i <= L1 && j >= 0 && j <= L2) sc.bndm[bo + j] = Cv;
      Lv = Cv;
      // refill slot u once its value is dead (see k_backward)
      const int tt = min(t + QD, T - 1);
      if constexpr ((M & kHmm5) != 0) q5[u] = sc.f5[sbase + (int64_t)tt * 64];
      if constexpr ((M & kLocal) != 0) ql[u] = sc.fl[sbase + (int64_t)tt * 64];
      if constexpr ((M & kPF) != 0) qg[u] = sc.pg[sbase + (int64_t)tt * 64];
    }
    }
    if (row_ok) {
      sc.ell_cnt[erow] = cnt;
      my_nnz += cnt;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  }
  // wave reductions
  for (int off = 32; off >= 1; off >>= 1) my_nnz += __shfl_xor(my_nnz, off);
  const int over = __any(ell_over) ? 1 : 0;
  const int owner = L1 & 63;
  const float sc_ = __shfl(score, owner);
  if (lane == 0) {
    rec[p].nnz = my_nnz;
    rec[p].mea = sc_;
    rec[p].dist = 1.0f - sc_ / (float)min(L1, L2);
    if (over) atomicOr(&rec[p].flags, 2);
  }
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
  const int64_t p = wave_pair_index();
  if (p >= npairs) return;
  const int lane = threadIdx.x & 63;
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
    const int start = run + x - c;
    if (i <= L1) {
      rp[i + 1] = start + c;
      for (int k = 0; k < c; ++k) {
        out_cols[eb + start + k] = sc.ell_col[(er0 + i - 1) * kEll + k];
        out_vals[eb + start + k] = sc.ell_val[(er0 + i - 1) * kEll + k];
      }
    }
    run += __shfl(x, 63);
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
// MLP_FUSE=1 runs all three models in one sweep (default: two sweeps).
static bool fuse_models() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("MLP_FUSE");
    v = (e && e[0] == '1') ? 1 : 0;
  }
  return v == 1;
}

static inline dim3 wave_grid(int64_t npairs) {
  return dim3((unsigned)((npairs + kWavesPerBlock - 1) / kWavesPerBlock));
}

// One sweep kernel K<M, LONG> per model set; LONG when a column sequence of
// the batch does not fit the per-wave LDS residue buffer.
template <template <int, bool> class K>
static hipError_t launch_sweep(int models, bool long_seq, const ModelScalars& ms, const Tables* tab,
                               SeqSet seqs, PairMeta pm, PairRec* rec, Scratch sc, int64_t npairs,
                               hipStream_t st) {
  const dim3 g = wave_grid(npairs), b(64 * kWavesPerBlock);
  auto go = [&](auto m_tag) {
    constexpr int Mv = decltype(m_tag)::value;
    if (long_seq) hipLaunchKernelGGL((K<Mv, true>::fn), g, b, 0, st, ms, tab, seqs, pm, rec, sc, npairs);
    else hipLaunchKernelGGL((K<Mv, false>::fn), g, b, 0, st, ms, tab, seqs, pm, rec, sc, npairs);
  };
  switch (models) {
    case kHmm5 | kLocal | kPF:
      if (fuse_models()) {
        go(std::integral_constant<int, kHmm5 | kLocal | kPF>{});
      } else {  // fp32 HMMs and the fp64 partition function as two sweeps: fewer VGPRs each
        go(std::integral_constant<int, kHmm5 | kLocal>{});
        go(std::integral_constant<int, kPF>{});
      }
      break;
    case kLocal: go(std::integral_constant<int, kLocal>{}); break;
    case kPF: go(std::integral_constant<int, kPF>{}); break;
    case kHmm5: go(std::integral_constant<int, kHmm5>{}); break;
    default: return hipErrorInvalidValue;
  }
  return hipSuccess;
}
template <int M, bool LONG> struct ForwardK { static constexpr auto fn = k_forward<M, LONG>; };
template <int M, bool LONG> struct BackwardK { static constexpr auto fn = k_backward<M, LONG>; };

hipError_t launch_forward(int models, const ModelScalars& ms, const Tables* tab, SeqSet seqs,
                          PairMeta pm, PairRec* rec, Scratch sc, int64_t npairs, int max_len2,
                          hipStream_t st) {
  if (npairs <= 0) return hipSuccess;
  const hipError_t e = launch_sweep<ForwardK>(models, max_len2 > kSeqLds, ms, tab, seqs, pm, rec, sc, npairs, st);
  if (e != hipSuccess) return e;
  return hipGetLastError();
}

hipError_t launch_backward(int models, const ModelScalars& ms, const Tables* tab, SeqSet seqs,
                           PairMeta pm, PairRec* rec, Scratch sc, int64_t npairs, int max_len2,
                           hipStream_t st) {
  if (npairs <= 0) return hipSuccess;
  const hipError_t e = launch_sweep<BackwardK>(models, max_len2 > kSeqLds, ms, tab, seqs, pm, rec, sc, npairs, st);
  if (e != hipSuccess) return e;
  if (models & kHmm5) {
    // fold the 5-state backward total (needs Tables for the initial cells)
    hipLaunchKernelGGL(k_fold_totals, dim3((unsigned)((npairs + 255) / 256)), dim3(256), 0, st, ms, seqs, pm, rec, tab, npairs);
  }
  return hipGetLastError();
}

hipError_t launch_local_totals(SeqSet seqs, PairMeta pm, PairRec* rec, Scratch sc, int64_t npairs,
                               hipStream_t st) {
  if (npairs <= 0) return hipSuccess;
  const char* v = getenv("MLP_TOTALS");
  if (v && v[0] == 'g')
    hipLaunchKernelGGL(k_local_totals_grp, dim3((unsigned)((npairs + 8 * kWavesPerBlock - 1) / (8 * kWavesPerBlock))), dim3(64 * kWavesPerBlock), 0, st, seqs, pm, rec, sc, npairs);
  else if (!v || v[0] == 'm')
    hipLaunchKernelGGL(k_local_totals_multi, dim3((unsigned)((npairs + kTotPairs * kWavesPerBlock - 1) / (kTotPairs * kWavesPerBlock))),
                       dim3(64 * kWavesPerBlock), 0, st, seqs, pm, rec, sc, npairs);
  else if (v[0] == 'w')
    hipLaunchKernelGGL(k_local_totals_wave, wave_grid(npairs), dim3(64 * kWavesPerBlock), 0, st, seqs, pm, rec, sc, npairs);
  else
    hipLaunchKernelGGL(k_local_totals_lane, dim3((unsigned)((npairs + 63) / 64)), dim3(64), 0, st, seqs, pm, rec, sc, npairs);
  return hipGetLastError();
}

hipError_t launch_merge(int models, int pid, const ModelScalars& ms, SeqSet seqs, PairMeta pm,
                        PairRec* rec, Scratch sc, int64_t npairs, hipStream_t st) {
  if (npairs <= 0) return hipSuccess;
  const dim3 g = wave_grid(npairs), b(64 * kWavesPerBlock);
  if (pid == 2) hipLaunchKernelGGL((k_merge<kLocal, 2>), g, b, 0, st, ms, seqs, pm, rec, sc, npairs);
  else if (pid >= 3) hipLaunchKernelGGL((k_merge<kPF, 3>), g, b, 0, st, ms, seqs, pm, rec, sc, npairs);
  else hipLaunchKernelGGL((k_merge<kHmm5 | kLocal | kPF, 0>), g, b, 0, st, ms, seqs, pm, rec, sc, npairs);
  (void)models;
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
