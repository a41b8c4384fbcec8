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
//     idx = cell_off + ((s * (L2 + 64)) + t) * 64 + lane
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
struct LdsTables {
  float4 lk[4];
  float match[26 * 26];
  float ins[26];
  double sub[26 * 26];
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
template <int M>
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
  const int T = L2 + 64;
  const int64_t cbase = pm.cell_off[p];
  const int64_t rmb = pm.rm_off[p];
  const int Wp = (L2 + 3) & ~3;
  const int64_t bo = pm.bnd_off[p];
  const float rt1 = ms.rt1, two_rt1 = 2 * ms.rt1;
  const double pfo = ms.pf_open, pfe = ms.pf_ext;
  int pf_over = 0;

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
    float cb0 = 0, cb1 = 0, cb2 = 0, cb3 = 0;  // row-major chain staging
    int c2 = 0;
    ResidueChunk rc2;
    rc2.init();
    float bch5[5], bchl[3];
    double bchz[3];
    int bche = 0;
    int bbase = -(1 << 30);

    for (int t = 0; t < T; ++t) {
      const int j = t - lane;
      const int c2new = rc2.get(s2, L2, t - 1);   // residue j: s2[j-1]
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
        const int cbk = t & ~63;
        if (cbk != bbase) {
          bbase = cbk;
          const int col = cbk + lane;
          const bool ok = col <= L2;
          const int64_t bi = bo + col;
          if constexpr ((M & kHmm5) != 0) {
#pragma unroll
            for (int k = 0; k < 5; ++k) bch5[k] = ok ? sc.bnd5[bi * 5 + k] : LZ;
          }
          if constexpr ((M & kLocal) != 0) {
#pragma unroll
            for (int k = 0; k < 3; ++k) bchl[k] = ok ? sc.bndl[bi * 3 + k] : LZ;
          }
          if constexpr ((M & kPF) != 0) {
#pragma unroll
            for (int k = 0; k < 3; ++k) bchz[k] = ok ? sc.bndz[bi * 3 + k] : 0.0;
            bche = ok ? sc.bnde[bi] : 0;
          }
        }
        const int q = t & 63;
        if (lane == 0) {
          if constexpr ((M & kHmm5) != 0) {
#pragma unroll
            for (int k = 0; k < 5; ++k) U5[k] = readlane_f(bch5[k], q);
          }
          if constexpr ((M & kLocal) != 0) {
#pragma unroll
            for (int k = 0; k < 3; ++k) UL[k] = readlane_f(bchl[k], q);
          }
          if constexpr ((M & kPF) != 0) {
            UZm = readlane_d(bchz[0], q); UZe = readlane_d(bchz[1], q); UZf = readlane_d(bchz[2], q);
            Ue = __builtin_amdgcn_readlane(bche, q);
          }
        }
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
          if (act) {
            sc.f5[idx] = C[0];
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
          if (act) {
            sc.fl[idx] = Cm;
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
          if (act) {
            pf_over |= (E > 250);
            sc.zm[idx] = mlp_pf_pack(Zm, E);
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
template <int M>
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
  const int T = L2 + 64;
  const int64_t cbase = pm.cell_off[p];
  const int64_t rmb = pm.rm_off[p];
  const int Wp = (L2 + 3) & ~3;
  const int64_t bo = pm.bnd_off[p];
  const float rt1 = ms.rt1, two_rt1 = 2 * ms.rt1;
  const double pfo = ms.pf_open, pfe = ms.pf_ext;
  const double zmant = (M & kPF) ? rec[p].zmant : 1.0;
  const int zexp = (M & kPF) ? rec[p].zexp : 0;

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
    float cb0 = 0, cb1 = 0, cb2 = 0, cb3 = 0;
    int c2n = 0;  // residue j+1
    ResidueChunk rcn, rcc;
    rcn.init();
    rcc.init();
    float bch5[5], bchl[3];
    double bchz[3];
    int bche = 0;
    int bbase = -(1 << 30);

    for (int t = T - 1; t >= 0; --t) {
      const int j = t - lane;
      // residues: lane 63 takes s2[j] for its column j = t - 63
      c2n = mlp_shl1i(c2n, rcn.get(s2, L2, t - 63));
      // residue j (current column) = c2n of lane+1 at this step
      const int c2 = mlp_shl1i(c2n, rcc.get(s2, L2, t - 64));
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
        const int cbk = col & ~63;
        if (cbk != bbase) {
          bbase = cbk;
          const int cc = cbk + lane;
          const bool ok = cc >= 0 && cc <= L2;
          const int64_t bi = bo + cc;
          if constexpr ((M & kHmm5) != 0) {
#pragma unroll
            for (int k = 0; k < 5; ++k) bch5[k] = ok ? sc.bnd5[bi * 5 + k] : LZ;
          }
          if constexpr ((M & kLocal) != 0) {
#pragma unroll
            for (int k = 0; k < 3; ++k) bchl[k] = ok ? sc.bndl[bi * 3 + k] : LZ;
          }
          if constexpr ((M & kPF) != 0) {
#pragma unroll
            for (int k = 0; k < 3; ++k) bchz[k] = ok ? sc.bndz[bi * 3 + k] : 0.0;
            bche = ok ? sc.bnde[bi] : 0;
          }
        }
        const int q = col & 63;
        if (lane == 63) {
          if constexpr ((M & kHmm5) != 0) {
#pragma unroll
            for (int k = 0; k < 5; ++k) N5[k] = readlane_f(bch5[k], q);
          }
          if constexpr ((M & kLocal) != 0) {
#pragma unroll
            for (int k = 0; k < 3; ++k) NL[k] = readlane_f(bchl[k], q);
          }
          if constexpr ((M & kPF) != 0) {
            NZm = readlane_d(bchz[0], q); NZe = readlane_d(bchz[1], q); NZf = readlane_d(bchz[2], q);
            Ne = __builtin_amdgcn_readlane(bche, q);
          }
        }
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
          if (act) {
            sc.f5[idx] = sc.f5[idx] + B[0];   // f + b (CPNP/ProbabilisticModel.h:484)
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
          if (act) {
            sc.fl[idx] = sc.fl[idx] + Bm;
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
              const double zf = mlp_pf_unpack(sc.zm[idx], &ef);
              const double q = (zf * Zm) / (score * zmant);
              post = (float)ldexp(q, MLP_PF_STEP * (ef + E - zexp));
            }
          }
          if (act) {
            sc.pg[idx] = post;
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
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  }
}

// =====================================================================
// Local-model totals: the reference sums LOG_PLUS_EQUALS over all interior
// cells in row-major order (CPNP/ProbabilisticModel.h:435-450), a single
// non-associative chain, for the forward and the backward half.
//
// One wave per pair streams 64 consecutive row-major elements at a time.  An
// element x leaves the running sum acc unchanged iff acc - x >= 7.5 (the
// LOG_ADD cutoff), and acc never decreases (LOOKUP(d) - d >= 4.46e-4 for
// every float d in [0, 7.5), checked exhaustively), so an element that is
// skippable against the current acc is skippable at its turn too.  Only the
// remaining candidates are folded in, serially and in order, with the exact
// LOG_ADD: the result is bit-identical to the reference's chain.
// =====================================================================
__global__ __launch_bounds__(256) void k_local_totals(SeqSet sq, PairMeta pm, PairRec* __restrict__ rec,
                                                      Scratch sc, int64_t npairs) {
  const int64_t p = wave_pair_index();
  if (p >= npairs) return;
  const int lane = threadIdx.x & 63;
  const int L1 = sq.len[pm.pa[p]], L2 = sq.len[pm.pb[p]];
  const int Wp = (L2 + 3) & ~3;
  const float* __restrict__ cf = sc.chf + pm.rm_off[p];
  const float* __restrict__ cbk = sc.chb + pm.rm_off[p];
  float tf = LZ, tb = LZ;
  for (int i = 0; i < L1; ++i) {
    const float* rf = cf + (int64_t)i * Wp;
    const float* rb = cbk + (int64_t)i * Wp;
    for (int c0 = 0; c0 < L2; c0 += 64) {
      const int j = c0 + lane;
      const bool ok = j < L2;
      const float xf = ok ? rf[j] : LZ;
      const float xb = ok ? rb[j] : LZ;
      uint64_t mf = __ballot(ok && !(tf - xf >= 7.5f));
      uint64_t mb = __ballot(ok && !(tb - xb >= 7.5f));
      while (mf | mb) {
        if (mf) {
          const int l = __builtin_ctzll(mf);
          const float v = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xf), l));
          tf = mlp_log_add(tf, v);
          mf &= mf - 1;
          mf &= __ballot(!(tf - xf >= 7.5f));
        }
        if (mb) {
          const int l = __builtin_ctzll(mb);
          const float v = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xb), l));
          tb = mlp_log_add(tb, v);
          mb &= mb - 1;
          mb &= __ballot(!(tb - xb >= 7.5f));
        }
      }
    }
  }
  if (lane == 0) {
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
  const int T = L2 + 64;
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
    float bch = 0.f;
    int bbase = -(1 << 30);
    for (int t = 0; t < T; ++t) {
      const int j = t - lane;
      Dv = Uv;
      Uv = mlp_shr1(Lv, 0.f);
      if (s > 0) {
        const int cbk = t & ~63;
        if (cbk != bbase) {
          bbase = cbk;
          const int col = cbk + lane;
          bch = (col <= L2) ? sc.bndm[bo + col] : 0.f;
        }
        const float v = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bch), t & 63));
        if (lane == 0) Uv = v;
      }
      const bool act = row_ok && j >= 1 && j <= L2;
      const int64_t idx = cbase + ((int64_t)s * T + t) * 64 + lane;
      float P = 0.f;
      if (act) {
        if constexpr (PID == 2) {
          P = mlp_post_from_sum_t(sc.fl[idx], TL, ex);
        } else if constexpr (PID >= 3) {
          P = sc.pg[idx];
        } else {
          const float v1 = mlp_post_from_sum_t(sc.f5[idx], T5, ex);
          const float v2 = sc.pg[idx];
          const float v3 = mlp_post_from_sum_t(sc.fl[idx], TL, ex);
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
static inline dim3 wave_grid(int64_t npairs) {
  return dim3((unsigned)((npairs + kWavesPerBlock - 1) / kWavesPerBlock));
}

hipError_t launch_forward(int models, const ModelScalars& ms, const Tables* tab, SeqSet seqs,
                          PairMeta pm, PairRec* rec, Scratch sc, int64_t npairs, hipStream_t st) {
  if (npairs <= 0) return hipSuccess;
  const dim3 g = wave_grid(npairs), b(64 * kWavesPerBlock);
  switch (models) {
    case kHmm5 | kLocal | kPF: hipLaunchKernelGGL(k_forward<kHmm5 | kLocal | kPF>, g, b, 0, st, ms, tab, seqs, pm, rec, sc, npairs); break;
    case kLocal: hipLaunchKernelGGL(k_forward<kLocal>, g, b, 0, st, ms, tab, seqs, pm, rec, sc, npairs); break;
    case kPF: hipLaunchKernelGGL(k_forward<kPF>, g, b, 0, st, ms, tab, seqs, pm, rec, sc, npairs); break;
    case kHmm5: hipLaunchKernelGGL(k_forward<kHmm5>, g, b, 0, st, ms, tab, seqs, pm, rec, sc, npairs); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_backward(int models, const ModelScalars& ms, const Tables* tab, SeqSet seqs,
                           PairMeta pm, PairRec* rec, Scratch sc, int64_t npairs, hipStream_t st) {
  if (npairs <= 0) return hipSuccess;
  const dim3 g = wave_grid(npairs), b(64 * kWavesPerBlock);
  switch (models) {
    case kHmm5 | kLocal | kPF: hipLaunchKernelGGL(k_backward<kHmm5 | kLocal | kPF>, g, b, 0, st, ms, tab, seqs, pm, rec, sc, npairs); break;
    case kLocal: hipLaunchKernelGGL(k_backward<kLocal>, g, b, 0, st, ms, tab, seqs, pm, rec, sc, npairs); break;
    case kPF: hipLaunchKernelGGL(k_backward<kPF>, g, b, 0, st, ms, tab, seqs, pm, rec, sc, npairs); break;
    case kHmm5: hipLaunchKernelGGL(k_backward<kHmm5>, g, b, 0, st, ms, tab, seqs, pm, rec, sc, npairs); break;
    default: return hipErrorInvalidValue;
  }
  if (models & kHmm5) {
    // fold the 5-state backward total (needs Tables for the initial cells)
    hipLaunchKernelGGL(k_fold_totals, dim3((unsigned)((npairs + 255) / 256)), dim3(256), 0, st, ms, seqs, pm, rec, tab, npairs);
  }
  return hipGetLastError();
}

hipError_t launch_local_totals(SeqSet seqs, PairMeta pm, PairRec* rec, Scratch sc, int64_t npairs,
                               hipStream_t st) {
  if (npairs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_local_totals, wave_grid(npairs), dim3(64 * kWavesPerBlock), 0, st, seqs, pm, rec, sc, npairs);
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
