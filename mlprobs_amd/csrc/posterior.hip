// posterior.hip -- all-pairs pairwise posterior sweeps for gfx950 (CDNA4).
//
// Replaces the per-pair body of the pdoAlign pair loop (CPNP/MSA.cpp:939-1025):
//   5-state double-affine pair-HMM forward/backward (CPNP/ProbabilisticModel.h:153-395),
//   3-state local pair-HMM forward/backward (same functions, flag = false),
//   global partition function (CPNP/MSAPartProbs.cpp:78-727),
//   posteriors (CPNP/ProbabilisticModel.h:464-493), RMS merge (CPNP/MSA.cpp:992-1007),
//   MEA (CPNP/ProbabilisticModel.h:804-864), distance (CPNP/MSA.cpp:1019-1020)
//   and sparsification (CPNP/SparseMatrix.h:55-98).
// The totals, the compaction and the local-model chain live in totals.hip.
//
// Execution model (see mlp_kernels.h, "Chains"): one 64-lane wave sweeps a
// chain of pairs whose DP rows are stacked.  Lane r owns stacked rows
// g = r (mod 64) and spends W steps on each (columns 0..W-1, the ones past
// the pair's L2 idle), so at step tau it works on column j = (tau - r) mod W
// of row g = 64 floor((tau - r) / W) + r.  The up/down neighbour arrives by a
// DPP wave shift (wave_shr:1 / wave_shl:1), the diagonal is the previous
// step's neighbour value, the left/right value stays in the lane.  Rows
// 64k - 1 -> 64k cross from lane 63 to lane 0 through a per-chain boundary
// row in HBM (written W - 63 steps before it is read).  A lane that finishes
// a row continues with its next row at once, across strips and across pairs,
// so the wave only idles for the 63-step skew at the chain's two ends.
// Cell values live in a step-diagonal layout
//     idx = cell_off + (tau + 1) * 64 + lane
// so every per-step load / store of a wave is one coalesced 256-byte access.
//
// All float arithmetic reproduces the reference's operation order exactly
// (see mlp_numerics.h); the partition function runs in scaled fp64 instead
// of x87 long double.
#include "mlp_chain.h"

#include <type_traits>

namespace mlp {

// Depth of the software-pipelined loads of the backward step loop.
constexpr int kPrefetch = 4;
static_assert(kWidthQuantum % kPrefetch == 0 && 64 % kPrefetch == 0,
              "the backward's prefetch groups must divide every segment (64 steps or W mod 64)");

// Waves per SIMD the sweeps are compiled for (launch bounds: 6 waves <=> at
// most 80 VGPRs, 5 <=> 96): the chains of a batch keep ~8 waves per SIMD
// queued, and the extra resident waves hide the DP's dependency stalls.  The
// PF backward holds more fp64 state and runs at MLP_PF_BWD_WAVES (5: 94
// VGPRs; at 6 it now fits 80 VGPRs without spilling); the all-in-one M = 7
// build keeps the compiler's choice.  The forward sweeps run at 5 waves
// (MLP_FWD_WAVES) since round 4: at 94 VGPRs the compiler keeps what it
// rematerialised at 80, and the forward group took 202-203 ms a C3 step
// against 215-217 at 6 waves (the backward group 219 against 224 beside it;
// profiles/r04k_ab_fwd_waves.txt).
#ifndef MLP_SWEEP_WAVES
#define MLP_SWEEP_WAVES 6
#endif
#ifndef MLP_PF_BWD_WAVES
#define MLP_PF_BWD_WAVES 5
#endif
#ifndef MLP_FWD_WAVES
#define MLP_FWD_WAVES 5
#endif
#ifndef MLP_BWD_WAVES
#define MLP_BWD_WAVES MLP_SWEEP_WAVES
#endif
template <int M>
struct SweepWaves {
  static constexpr int fwd = M == 7 ? 1 : MLP_FWD_WAVES;
  static constexpr int bwd = M == 7 ? 1 : ((M & 4) != 0 && MLP_BWD_WAVES > MLP_PF_BWD_WAVES ? MLP_PF_BWD_WAVES : MLP_BWD_WAVES);
};

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
// Move a cell's three values to the next frame when the largest exceeds 2^200.
__device__ __forceinline__ void pf_rescale(double& m, double& e, double& f, int& E) {
  const double mx = fmax(fmax(m, e), f);
  if (mx > MLP_PF_HUGE) {
    m = ldexp(m, -MLP_PF_STEP); e = ldexp(e, -MLP_PF_STEP); f = ldexp(f, -MLP_PF_STEP);
    ++E;
  }
}
// Frame changes are rare (a pair's values cross 2^200 a few times at most),
// so both frame steps run as wave-uniform branches around the common case:
// with all three neighbour frames equal pf_align does nothing (E = ea), and
// pf_rescale acts only past 2^200.  The per-lane code inside is unchanged,
// so every value rounds as before; the compiler no longer if-converts the
// ldexp blocks into always-executed selects.
__device__ __forceinline__ bool wave_none(bool p) { return __ballot(p) == 0; }
__device__ __forceinline__ int pf_align_fast(double& a0, double& a1, double& a2, int ea,
                                             double& b0, double& b1, double& b2, int eb,
                                             double& c0, double& c1, double& c2, int ec) {
  if (wave_none(ea != eb || eb != ec)) return ea;
  return pf_align(a0, a1, a2, ea, b0, b1, b2, eb, c0, c1, c2, ec);
}
__device__ __forceinline__ void pf_rescale_fast(double& m, double& e, double& f, int& E) {
  const double mx = fmax(fmax(m, e), f);
  if (wave_none(mx > MLP_PF_HUGE)) return;
  if (mx > MLP_PF_HUGE) {
    m = ldexp(m, -MLP_PF_STEP); e = ldexp(e, -MLP_PF_STEP); f = ldexp(f, -MLP_PF_STEP);
    ++E;
  }
}

// =====================================================================
// Forward sweep: 5-state forward, local forward, PF forward Zm.
// =====================================================================
template <int M>
__global__ __launch_bounds__(256, SweepWaves<M>::fwd) void k_forward(ModelScalars ms, const Tables* __restrict__ tab,
                                                 SeqSet sq, PairMeta pm, ChainMeta cm,
                                                 PairRec* __restrict__ rec, Scratch sc,
                                                 int64_t nchains, int lds_seq) {
  __shared__ LdsTablesFor<M> T_;
  extern __shared__ __align__(16) uint8_t dyn[];
  stage_tables(T_, tab);
  const int64_t ch = wave_index();
  if (ch >= nchains) return;
  const float4* __restrict__ lk = lookup_of(T_);
  const int lane = threadIdx.x & 63;
  const ChainView C = stage_chain<kStageFwd>(dyn, lds_seq, ch, sq, pm, cm, rec);
  const int W = C.W, S = C.S;
  // slot of step tau, lane l: cell0 + tau * 64 + l (a wave-uniform row
  // pointer per step plus the lane: scalar-addressed stores, no per-step
  // 64-bit lane arithmetic)
  const int64_t cell0 = cm.cell_off[ch] + 64;
  const uint32_t ul4 = (uint32_t)lane * 4;   // the lane's byte offset in a step's fp32 slots
  const int64_t bo = cm.bnd_off[ch];
  // lane 63's column (the strip's last row, stored into the boundary row):
  // W - 63 at step 0 (idle until step 63), one column per step, wrapping at W
  int j63 = W - 63;
  float* const bh = sc.bnd5 + bo * 8;    // boundary records (mlp_chain.h)
  double* const bz = sc.bndz + bo * 4;
  const float rt1 = ms.rt1, two_rt1 = 2 * ms.rt1;
  const double pfo = ms.pf_open, pfe = ms.pf_ext;
  Cursor c;
  // the local chain's chunk maxima (CPNP/ProbabilisticModel.h:438-447, for
  // k_local_totals' exact skip test): per lane the column that ends its
  // current 64-column chunk (a multiple of 64, or L2; -1 on rows without
  // chunks) and that chunk's element of cmf; set when the lane enters a row
  int jst = -1;
  uint32_t cmo4 = 0;       // byte offset of that element (cmf < 2 GB: cells / 16 bytes of a batch)
  float cmx = -INFINITY;   // the chunk's running maximum (row 0 / column 0 hold LZ: no effect)
  auto local_row = [&]() {
    if constexpr ((M & kLocal) != 0) {
      jst = c.q >= 0 && c.i >= 1 ? min(64, c.L2) : -1;
      cmo4 = (uint32_t)(c.rm + (int64_t)(c.i - 1) * local_chunks(c.L2)) * 4u;
      cmx = -INFINITY;
    }
  };
  cursor_start_fwd(c, C, T_.ins, lane);
  local_row();
  // per-lane state: Lx = own cell at j-1, Ux = cell (i-1, j), Dx = (i-1, j-1)
  float L5[5], U5[5], D5[5];
  float LL[3], UL[3], DL[3];
  double LZm = 0, LZe = 0, LZf = 0, UZm = 0, UZe = 0, UZf = 0, DZm = 0, DZe = 0, DZf = 0;
  int Le = 0, Ue = 0, De = 0;
#pragma unroll
  for (int k = 0; k < 5; ++k) L5[k] = U5[k] = D5[k] = LZ;
#pragma unroll
  for (int k = 0; k < 3; ++k) LL[k] = UL[k] = DL[k] = LZ;
  __shared__ __align__(16) uint8_t chunk_lds[kWavesPerBlock * 64 * LdsChunkLayout<M>::bytes];
  LdsBoundaryChunks<M> bc;
  bc.area = chunk_lds + (threadIdx.x >> 6) * 64 * LdsChunkLayout<M>::bytes;
  const int nseg = (W + 63) >> 6;

  // segments: lane 0's 64-column chunks of strip k; k == S: the skew tail
  for (int k = 0; k <= S; ++k) {
    const int segs = k < S ? nseg : 1;
    for (int m = 0; m < segs; ++m) {
      const int t_lo = k * W + 64 * m;
      const int t_hi = k < S ? min(t_lo + 64, (k + 1) * W) : t_lo + 64;
      if (k < S) {
        boundary_fence();
        bc.advance(lane);
        bc.load_next(sc, bo, W, m + 1 < nseg ? 64 * (m + 1) : 0, lane);
      }
      // unrolled by 4 (segments hold multiples of 8 steps) so the rotating
      // left/up/diagonal roles stay in fixed registers
      for (int t0 = t_lo; t0 < t_hi; t0 += 4) {
      // the chunk column of step t0 + u: bc.area + (t0 + u - t_lo) * bytes
      const uint8_t* const colp = bc.area + (t0 - t_lo) * LdsChunkLayout<M>::bytes;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = t0 + u;
        const int i = c.i, j = c.j, L1 = c.L1, L2 = c.L2;
        // wave-uniform: no lane on an initial cell, row 0 or column 0 (the
        // common case away from the pairs' edges), so the recurrences' values
        // are taken as they are, without the per-lane selects of the edges
        const bool interior = wave_none(j < c.jlo);
        const int c1 = c.c1;
        const int c2 = C.seq[c.ca];          // residue j (0 at j = 0 and past L2)
        const float ins1 = c.ins1;
        // diagonal = previous up; up = upper lane's left.  Lane 0's up value is
        // the boundary row (stacked row 64k - 1, column t - t_lo + 64m) in
        // strips >= 1, unused otherwise (row 0 of the chain, idle tail)
        if constexpr ((M & kHmm5) != 0) {
#pragma unroll
          for (int k5 = 0; k5 < 5; ++k5) D5[k5] = U5[k5];
        }
        if constexpr ((M & kLocal) != 0) {
#pragma unroll
          for (int k3 = 0; k3 < 3; ++k3) DL[k3] = UL[k3];
        }
        if constexpr ((M & kPF) != 0) { DZm = UZm; DZe = UZe; DZf = UZf; De = Ue; }
        // every step takes lane 0's value from the chunk (in strip 0 and the
        // skew tail lane 0's up value is unused -- row 0 of the chain, the
        // idle tail -- so whatever the chunk holds is harmless): one form of
        // the shift, no branch joining two register assignments
        bc.template shift_at<true>(colp + u * LdsChunkLayout<M>::bytes, L5, U5, LL, UL, LZm, LZe, LZf, Le, UZm, UZe,
                                   UZf, Ue);
        const int64_t tcell = cell0 + (int64_t)t * 64;   // wave-uniform
        // the HMMs' boundary record of lane 63's column (bnd_put_hmm)
        float4 bha = make_float4(0.f, 0.f, 0.f, 0.f), bhb = make_float4(0.f, 0.f, 0.f, 0.f);
        // ------------------------------------------------ 5-state forward
        if constexpr ((M & kHmm5) != 0) {
          const float mt = T_.match[c.c1x + c2];
          const float ins2 = T_.ins[c2];
          // CPNP/ProbabilisticModel.h:213-256
          float vm = D5[0] + ms.t[0][0];
          vm = mlp_log_add_t(vm, D5[1] + ms.t[1][0], lk);
          vm = mlp_log_add_t(vm, D5[2] + ms.t[2][0], lk);
          vm = mlp_log_add_t(vm, D5[3] + ms.t[3][0], lk);
          vm = mlp_log_add_t(vm, D5[4] + ms.t[4][0], lk);
          vm = vm + mt;
          const float vx1 = ins1 + mlp_log_add_t(U5[0] + ms.t[0][1], U5[1] + ms.t[1][1], lk);
          const float vx2 = ins1 + mlp_log_add_t(U5[0] + ms.t[0][3], U5[3] + ms.t[3][3], lk);
          const float vy1 = ins2 + mlp_log_add_t(L5[0] + ms.t[0][2], L5[2] + ms.t[2][2], lk);
          const float vy2 = ins2 + mlp_log_add_t(L5[0] + ms.t[0][4], L5[4] + ms.t[4][4], lk);
          float Cc[5];
          if (interior) {  // every lane's cell takes all five recurrences
            Cc[0] = vm; Cc[1] = vx1; Cc[2] = vy1; Cc[3] = vx2; Cc[4] = vy2;
          } else {
            // (the edge tests only here: kept from being hoisted into the interior path)
            int ie = i, je = j;
            asm volatile("" : "+v"(ie), "+v"(je));
#pragma unroll
            for (int k5 = 0; k5 < 5; ++k5) Cc[k5] = LZ;
            // CPNP/ProbabilisticModel.h:173-183 initial cells
            if (ie == 1 && je == 1) Cc[0] = ms.init[0] + mt;
            if (ie == 1 && je == 0) { Cc[1] = ms.init[1] + ins1; Cc[3] = ms.init[3] + ins1; }
            if (ie == 0 && je == 1) { Cc[2] = ms.init[2] + ins2; Cc[4] = ms.init[4] + ins2; }
            if (ie > 1 || je > 1) {
              if (ie > 0 && je > 0) Cc[0] = vm;
              if (ie > 0) { Cc[1] = vx1; Cc[3] = vx2; }
              if (je > 0) { Cc[2] = vy1; Cc[4] = vy2; }
            }
          }
          bstore(sc.f5 + tcell, ul4, Cc[0]);   // every lane: values of idle cells are never used
          if (j == c.jend) {  // CPNP/ProbabilisticModel.h:415-419 (forward half)
            float tf = LZ;
#pragma unroll
            for (int k5 = 0; k5 < 5; ++k5) tf = mlp_log_add_t(tf, Cc[k5] + ms.init[k5], lk);
            rec[c.slot].tf5 = tf;
          }
          bha = make_float4(Cc[0], Cc[1], Cc[2], Cc[3]);
          bhb.x = Cc[4];
#pragma unroll
          for (int k5 = 0; k5 < 5; ++k5) L5[k5] = Cc[k5];
        }
        // ------------------------------------------------ local forward
        if constexpr ((M & kLocal) != 0) {
          const float mt = T_.match[c.c1x + c2];
          const float ins2 = T_.ins[c2];
          const float bs = mt - ins1 - ins2;
          float vm = bs - two_rt1;
          vm = mlp_log_add_t(vm, bs + DL[0] + ms.lt[0][0] - two_rt1, lk);
          vm = mlp_log_add_t(vm, bs + DL[1] + ms.lt[1][0] - two_rt1, lk);
          vm = mlp_log_add_t(vm, bs + DL[2] + ms.lt[2][0] - two_rt1, lk);
          const float vx = mlp_log_add_t(UL[0] + ms.lt[0][1] - rt1, UL[1] + ms.lt[1][1] - rt1, lk);
          const float vy = mlp_log_add_t(LL[0] + ms.lt[0][2] - rt1, LL[2] + ms.lt[2][2] - rt1, lk);
          float Cm = LZ, Cx = LZ, Cy = LZ;
          if (interior) {
            Cm = vm; Cx = vx; Cy = vy;
          } else {
            int ie = i, je = j;
            asm volatile("" : "+v"(ie), "+v"(je));
            if (ie == 1 && je == 1) Cm = bs - two_rt1;
            if (ie > 1 || je > 1) {
              if (ie > 0 && je > 0) Cm = vm;
              if (ie > 0) Cx = vx;
              if (je > 0) Cy = vy;
            }
          }
          bstore(sc.fl + tcell, ul4, Cm);
          bhb.y = Cm; bhb.z = Cx; bhb.w = Cy;
          // the chain total's input: the largest f_M of each 64-column chunk
          // of the row (from column 0, whose LZ never exceeds a real value)
          cmx = mlp_max(cmx, Cm);
          if (j == jst) {
            bstore(sc.cmf, cmo4, cmx);
            cmo4 += 4;
            jst = min(jst + 64, L2);
            cmx = -INFINITY;
          }
          LL[0] = Cm; LL[1] = Cx; LL[2] = Cy;
        }
        if constexpr ((M & (kHmm5 | kLocal)) != 0) {
          if (lane == 63) bnd_put_hmm(bh, j63, bha, bhb);
        }
        // ------------------------------------------------ partition function forward
        if constexpr ((M & kPF) != 0) {
          // cell (i, j) <-> reference Zm[ip = j][jp = i] (CPNP/MSAPartProbs.cpp:510-609)
          double Zm, Ze, Zf;
          int E;
          const double score = T_.sub[c2 * 26 + c1];
          if (i == 0) {
            Zm = (j == 0) ? 1.0 : 0.0; Ze = 0.0; Zf = (j >= 1) ? 1.0 : 0.0; E = 0;
          } else if (j == 0) {
            Zm = 0.0; Ze = 1.0; Zf = 0.0; E = 0;
          } else {
            // align copies: U becomes the next column's D with its own frame
            double uZm = UZm, uZe = UZe, uZf = UZf, dZm = DZm, dZe = DZe, dZf = DZf;
            double lZm = LZm, lZe = LZe, lZf = LZf;
            E = pf_align_fast(uZm, uZe, uZf, Ue, dZm, dZe, dZf, De, lZm, lZe, lZf, Le);
            // the last column / row use factors 1.0 (x * 1.0 + y * 1.0 ==
            // x + y exactly): both forms computed, one selected -- no
            // per-lane selects of the factors themselves
            const double ze_g = uZm * pfo + uZe * pfe, ze_1 = uZm + uZe;
            const double zf_g = lZm * pfo + lZf * pfe, zf_1 = lZm + lZf;
            Ze = (j == L2) ? ze_1 : ze_g;
            Zf = (i == L1) ? zf_1 : zf_g;
            // QuickProbs' Ze/Zf are ours transposed (QP/PartitionFunction.cpp:128-130)
            Zm = ((M & kQP) != 0 ? (dZm + dZf) + dZe : (dZm + dZe) + dZf) * score;
            pf_rescale_fast(Zm, Ze, Zf, E);
          }
          bstore(sc.zm + tcell, 2 * ul4, mlp_pf_pack(Zm, E));
          // QuickProbs' plain double has no such stop; frames past 2^50000 are
          // ours.  Frames reach 81 (2^16200) only near overflow: the
          // three-way maximum runs only when some active lane's frame got there
          if (!wave_none(E > ((M & kQP) != 0 ? 250 : 80) && j <= c.jact))
            if (j <= c.jact && ((M & kQP) != 0 ? E > 250 : mlp_pf_ldbl_overflow(Zm, Ze, Zf, E)))
              atomicOr(&rec[c.slot].flags, 1);
          if (j == c.jend) {  // CPNP/MSAPartProbs.cpp:591,612; QP/PartitionFunction.cpp:132,155
            rec[c.slot].zmant = (M & kQP) != 0 ? (Zm + Zf) + Ze : (Zm + Ze) + Zf;
            rec[c.slot].zexp = E;
          }
          if (lane == 63) bnd_put_pf(bz, j63, Zm, Ze, Zf, E);
          LZm = Zm; LZe = Ze; LZf = Zf; Le = E;
        }
        cursor_next(c, C, T_.ins, local_row);
        j63 = j63 + 1 == W ? 0 : j63 + 1;
      }
      }
    }
  }
}

// =====================================================================
// Backward sweep (reverse step order): 5-state f+b (in place), local b
// and the chunk maxima of its chain, PF posterior.
// =====================================================================
template <int M>
__global__ __launch_bounds__(256, SweepWaves<M>::bwd) void k_backward(ModelScalars ms, const Tables* __restrict__ tab,
                                                  SeqSet sq, PairMeta pm, ChainMeta cm,
                                                  PairRec* __restrict__ rec, Scratch sc,
                                                  int64_t nchains, int lds_seq) {
  __shared__ LdsTablesFor<M, true> T_;
  extern __shared__ __align__(16) uint8_t dyn[];
  stage_tables(T_, tab);
  const int64_t ch = wave_index();
  if (ch >= nchains) return;
  const float4* __restrict__ lk = lookup_of(T_);
  const int lane = threadIdx.x & 63;
  const ChainView C = stage_chain<kStageBwd>(dyn, lds_seq, ch, sq, pm, cm, rec);
  const int W = C.W, S = C.S;
  const int64_t cell0 = cm.cell_off[ch] + 64;   // slot of step tau, lane l: cell0 + tau * 64 + l
  const uint32_t ul4 = (uint32_t)lane * 4;     // the lane's byte offset in a step's fp32 slots
  const int64_t bo = cm.bnd_off[ch];
  float* const bh = sc.bnd5 + bo * 8;    // boundary records (mlp_chain.h)
  double* const bz = sc.bndz + bo * 4;
  const float rt1 = ms.rt1, two_rt1 = 2 * ms.rt1;
  const double pfo = ms.pf_open, pfe = ms.pf_ext;
  const int top = S * W + 62;   // last step with an active lane (lane 63, column W-1)
  // lane 0's column (the strip's first row, stored into the boundary row):
  // top mod W at the first step, one column less per step, wrapping to W - 1
  int j0 = top % W;
  Cursor c;
  // the local chain's chunk maxima, columns descending: a chunk starts at
  // its top column (L2 or a multiple of 64) and ends at 64 c + 1, where its
  // element of cmb is stored; per lane the next such column (-1 on rows
  // without chunks) and its element, set when the lane enters a row (every
  // active lane enters at column W - 1)
  int jsb = -1;
  uint32_t cmob4 = 0;   // byte offset of that element in cmb
  float cmx = -INFINITY;
  auto local_row = [&]() {
    if constexpr ((M & kLocal) != 0) {
      jsb = c.q >= 0 && c.i >= 1 ? ((c.L2 - 1) & ~63) + 1 : -1;
      cmob4 = (uint32_t)(c.rm + (int64_t)(c.i - 1) * local_chunks(c.L2) + ((c.L2 - 1) >> 6)) * 4u;
    }
  };
  cursor_start_bwd(c, C, T_.ins, lane, top);
  local_row();
  // Rx = own cell (i, j+1), Nx = (i+1, j), Gx = (i+1, j+1)
  float R5[5], N5[5], G5[5];
  float RL[3], NL[3], GL[3];
  double RZm = 0, RZe = 0, RZf = 0, NZm = 0, NZe = 0, NZf = 0, GZm = 0, GZe = 0, GZf = 0;
  int Re = 0, Ne = 0, Ge = 0;
#pragma unroll
  for (int k = 0; k < 5; ++k) R5[k] = N5[k] = G5[k] = LZ;
#pragma unroll
  for (int k = 0; k < 3; ++k) RL[k] = NL[k] = GL[k] = LZ;
  __shared__ __align__(16) uint8_t chunk_lds[kWavesPerBlock * 64 * LdsChunkLayout<M>::bytes];
  LdsBoundaryChunks<M> bc;
  bc.area = chunk_lds + (threadIdx.x >> 6) * 64 * LdsChunkLayout<M>::bytes;
  const int nseg = (W + 63) >> 6;
  // the step-t loads of f5 / zm are issued kPrefetch steps earlier into
  // fixed registers: slot u serves steps t0 - u (segments hold whole groups
  // of kPrefetch steps); every slot was written by the forward sweep, values
  // of idle cells are never used
  float q5[kPrefetch] = {};
  double qz[kPrefetch] = {};
#pragma unroll
  for (int k = 0; k < kPrefetch; ++k) {
    const int64_t at = cell0 + (int64_t)(top - k) * 64;
    if constexpr ((M & kHmm5) != 0) q5[k] = bload(sc.f5 + at, ul4);
    if constexpr ((M & kPF) != 0) qz[k] = bload(sc.zm + at, 2 * ul4);
  }

  // segments, in processing order: lane 63's 64-column chunks of strip k
  // (steps kW + 63 + 64m .. ), k = S-1 .. 0, m descending; then steps -1..62
  for (int k = S - 1; k >= -1; --k) {
    const int segs = k >= 0 ? nseg : 1;
    for (int m = segs - 1; m >= 0; --m) {
      int t_lo, t_hi;   // inclusive
      if (k >= 0) {
        t_lo = k * W + 63 + 64 * m;
        t_hi = k * W + 63 + min(64 * m + 63, W - 1);
        boundary_fence();
        bc.advance(lane);
        // chunk before (k, m): (k, m-1) or (k-1, last); holds stacked row 64k+64
        {
          const int col0 = m > 0 ? 64 * (m - 1) : 64 * (nseg - 1);
          // that segment's first step is its column min(63, W - 1 - col0): lane 63 holds it
          bc.load_next(sc, bo, W, col0, lane, 63 - min(63, W - 1 - col0));
        }
      } else {
        t_lo = -1;
        t_hi = 62;
      }
      for (int t0 = t_hi; t0 >= t_lo; t0 -= kPrefetch) {
      // the chunk column of step t0 - u is 63 - (t_hi - t0 + u): the group's
      // lowest (u = kPrefetch - 1) plus kPrefetch - 1 - u columns
      const uint8_t* const colp = bc.area + (63 - (t_hi - t0) - (kPrefetch - 1)) * LdsChunkLayout<M>::bytes;
#pragma unroll
      for (int u = 0; u < kPrefetch; ++u) {
        const int t = t0 - u;
        const int i = c.i, j = c.j, L1 = c.L1, L2 = c.L2;
        // wave-uniform: every lane inside its pair (not the last row, column
        // or cell), so the recurrences run without the edge selects
        const bool interior = wave_none(j >= c.jhi);
        // the edge tests, for the edge paths only (kept from being hoisted
        // into the interior path)
        auto edges = [&](bool& in_i, bool& in_j, bool& last) {
          int ie = i, je = j;
          asm volatile("" : "+v"(ie), "+v"(je));
          in_i = ie < L1;
          in_j = je < L2;
          last = ie == L1 && je == L2;
        };
        const float f5v = q5[u];
        const double zmv = qz[u];
        const int c1 = c.c1, c1n = c.c1n;
        const int c2 = C.seq[c.ca];        // residue j   (0 at j = 0 and past L2)
        const int c2n = C.seq[c.ca + 1];   // residue j+1 (0 past L2)
        const float ins1 = c.ins1, ins1n = c.ins1n;
        // diagonal = previous down; down = lower lane's right.  Lane 63's down
        // value is the boundary row (stacked row 64k + 64, column t - 63 - kW)
        // in strips < S-1, unused otherwise
        if constexpr ((M & kHmm5) != 0) {
#pragma unroll
          for (int k5 = 0; k5 < 5; ++k5) G5[k5] = N5[k5];
        }
        if constexpr ((M & kLocal) != 0) {
#pragma unroll
          for (int k3 = 0; k3 < 3; ++k3) GL[k3] = NL[k3];
        }
        if constexpr ((M & kPF) != 0) { GZm = NZm; GZe = NZe; GZf = NZf; Ge = Ne; }
        // (one form of the shift: lane 63's down value is unused in the last
        // strip -- the chain's last row, in_i false -- and in the skew head)
        // the chunk's column for this step: lane 63 held the segment's first
        // (the load's shift), each step one lane below
        bc.template shift_at<false>(colp + (kPrefetch - 1 - u) * LdsChunkLayout<M>::bytes, R5, N5, RL, NL, RZm, RZe,
                                    RZf, Re, NZm, NZe, NZf, Ne);
        const int64_t tcell = cell0 + (int64_t)t * 64;   // wave-uniform
        // the HMMs' boundary record of lane 0's column (bnd_put_hmm)
        float4 bha = make_float4(0.f, 0.f, 0.f, 0.f), bhb = make_float4(0.f, 0.f, 0.f, 0.f);
        // ------------------------------------------------ 5-state backward
        if constexpr ((M & kHmm5) != 0) {
          const float ins2n = T_.ins[c2n];
          const float mn = T_.match[c.c1nx + c2n];
          float B[5];
          // CPNP/ProbabilisticModel.h:310-313, 340-378
          const float pxy = G5[0] + mn;
          if (interior) {  // every lane: in_i, in_j, not the last cell -- no per-lane selects
#pragma unroll
            for (int k5 = 0; k5 < 5; ++k5) B[k5] = mlp_log_add_from_zero(pxy + ms.t[k5][0]);
            B[0] = mlp_log_add_t(B[0], N5[1] + ins1n + ms.t[0][1], lk);
            B[1] = mlp_log_add_t(B[1], N5[1] + ins1n + ms.t[1][1], lk);
            B[0] = mlp_log_add_t(B[0], N5[3] + ins1n + ms.t[0][3], lk);
            B[3] = mlp_log_add_t(B[3], N5[3] + ins1n + ms.t[3][3], lk);
            B[0] = mlp_log_add_t(B[0], R5[2] + ins2n + ms.t[0][2], lk);
            B[2] = mlp_log_add_t(B[2], R5[2] + ins2n + ms.t[2][2], lk);
            B[0] = mlp_log_add_t(B[0], R5[4] + ins2n + ms.t[0][4], lk);
            B[4] = mlp_log_add_t(B[4], R5[4] + ins2n + ms.t[4][4], lk);
          } else {
          bool in_i, in_j, last;
          edges(in_i, in_j, last);
#pragma unroll
          for (int k5 = 0; k5 < 5; ++k5)
            B[k5] = last ? ms.init[k5] : ((in_i && in_j) ? mlp_log_add_from_zero(pxy + ms.t[k5][0]) : LZ);
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
          }  // !interior
          bstore(sc.f5 + tcell, ul4, f5v + B[0]);   // f + b (CPNP/ProbabilisticModel.h:484)
          if (j <= c.jfirst) {   // rows 0 and 1, columns 0 and 1 of an active pair
            if (i == 1 && j == 1) rec[c.slot].b5[0] = B[0];
            if (i == 1 && j == 0) { rec[c.slot].b5[1] = B[1]; rec[c.slot].b5[3] = B[3]; }
            if (i == 0 && j == 1) { rec[c.slot].b5[2] = B[2]; rec[c.slot].b5[4] = B[4]; }
          }
          bha = make_float4(B[0], B[1], B[2], B[3]);
          bhb.x = B[4];
#pragma unroll
          for (int k5 = 0; k5 < 5; ++k5) R5[k5] = B[k5];
        }
        // ------------------------------------------------ local backward
        if constexpr ((M & kLocal) != 0) {
          const float ins2n = T_.ins[c2n];
          const float mn = T_.match[c.c1nx + c2n];
          float Bm = MLP_LOG_ONE, Bx = LZ, By = LZ;
          if (interior) {
            const float pxy = GL[0] + mn - ins1n - ins2n;
            Bm = mlp_log_add_t(Bm, pxy + ms.lt[0][0] - two_rt1, lk);
            Bx = mlp_log_add_from_zero(pxy + ms.lt[1][0] - two_rt1);
            By = mlp_log_add_from_zero(pxy + ms.lt[2][0] - two_rt1);
            Bm = mlp_log_add_t(Bm, NL[1] + ms.lt[0][1] - rt1, lk);
            Bx = mlp_log_add_t(Bx, NL[1] + ms.lt[1][1] - rt1, lk);
            Bm = mlp_log_add_t(Bm, RL[2] + ms.lt[0][2] - rt1, lk);
            By = mlp_log_add_t(By, RL[2] + ms.lt[2][2] - rt1, lk);
          } else {
          bool in_i, in_j, last;
          edges(in_i, in_j, last);
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
          }  // !interior
          bstore(sc.bl + tcell, ul4, Bm);   // f + b is formed by the merge (the same float add)
          bhb.y = Bm; bhb.z = Bx; bhb.w = By;
          // chain element (CPNP/ProbabilisticModel.h:444-445); columns descend,
          // so a chunk starts at its top column (L2: idle columns above it are
          // dropped there; or a multiple of 64: reset by the store before it)
          // and ends at 64c + 1
          {
            const float e = Bm + T_.match[c.c1x + c2] - ins1 - T_.ins[c2] - two_rt1;
            cmx = j == L2 ? e : mlp_max(cmx, e);
            if (j == jsb) {
              bstore(sc.cmb, cmob4, cmx);
              cmob4 -= 4;
              jsb -= 64;
              cmx = -INFINITY;
            }
          }
          RL[0] = Bm; RL[1] = Bx; RL[2] = By;
        }
        if constexpr ((M & (kHmm5 | kLocal)) != 0) {
          if (lane == 0) bnd_put_hmm(bh, j0, bha, bhb);
        }
        // ------------------------------------------------ partition function reverse
        if constexpr ((M & kPF) != 0) {
          // cell (i, j) <-> reverse Zm[ip = j-1][jp = i-1] (CPNP/MSAPartProbs.cpp:233-321)
          double Zm = 0, Ze = 0, Zf = 0;
          int E = 0;
          float post = 0.0f;
          const double score = T_.sub[c2 * 26 + c1];
          // wave-uniform: every lane strictly inside rows 2..L1-1, columns 2..L2-1
          const bool pf_inner = wave_none((uint32_t)(j - 2) >= (uint32_t)(c.jpf - 2));
          if (i >= 1 && j >= 1) {
            double nZm = NZm, nZe = NZe, nZf = NZf, rZm = RZm, rZe = RZe, rZf = RZf;
            double gZm = GZm, gZe = GZe, gZf = GZf;
            int ne = Ne, re = Re, ge = Ge;
            const double o0 = pfo, e0 = pfe, o1 = pfo, e1 = pfe;
            if (pf_inner) {  // no lane on row 1, L1 or column 1, L2: no boundary values, general factors
              E = pf_align_fast(nZm, nZe, nZf, ne, rZm, rZe, rZf, re, gZm, gZe, gZf, ge);
              Zf = rZm * o1 + rZf * e1;
              Ze = nZm * o0 + nZe * e0;
            } else {
            // boundary row L1+1 / column L2+1 (init of CPNP/MSAPartProbs.cpp:217-226)
            if (i == L1) { nZm = 0.0; nZf = 1.0; nZe = 0.0; ne = 0; }
            if (j == L2) { rZm = 0.0; rZf = 0.0; rZe = 1.0; re = 0; }
            if (j == L2) {
              const bool corner = (i == L1);
              gZm = corner ? 1.0 : 0.0; gZf = 0.0; gZe = corner ? 0.0 : 1.0; ge = 0;
            } else if (i == L1) {
              gZm = 0.0; gZf = 1.0; gZe = 0.0; ge = 0;
            }
            E = pf_align_fast(nZm, nZe, nZf, ne, rZm, rZe, rZf, re, gZm, gZe, gZf, ge);
            // first row / column: factors 1.0 (x * 1.0 + y * 1.0 == x + y)
            const double zf_g = rZm * o1 + rZf * e1, zf_1 = rZm + rZf;
            const double ze_g = nZm * o0 + nZe * e0, ze_1 = nZm + nZe;
            Zf = (i == 1) ? zf_1 : zf_g;
            Ze = (j == 1) ? ze_1 : ze_g;
            }
            Zm = ((M & kQP) != 0 ? (gZm + gZe) + gZf : (gZm + gZf) + gZe) * score;  // QP/PartitionFunction.cpp:260
            pf_rescale_fast(Zm, Ze, Zf, E);
            if (j <= c.jact) {
              int ef;
              const double zf = mlp_pf_unpack(zmv, &ef);
              // C_P_NP_Aln (long double in the reference, parity within 1e-4):
              // the quotient as products with the factor's and the total's
              // reciprocals (a few fp64 ulps from the division); QuickProbs
              // (plain double, bit-exact) divides like the reference
              double qv;
#ifdef MLP_PF_DIVIDE  // A/B build (tools/pf_quotient_ab.py): the division for C_P_NP_Aln too
              if constexpr (true)
#else
              if constexpr ((M & kQP) != 0)
#endif
                qv = (zf * Zm) / (score * c.zmant);
              else
                qv = (zf * Zm) * (T_.rsub[c2 * 26 + c1] * c.rzmant);
              post = (float)ldexp(qv, MLP_PF_STEP * (ef + E - c.zexp));
              // QuickProbs stores only probabilities in [0.001, 1] (QP/PartitionFunction.cpp:266-272)
              if constexpr ((M & kQP) != 0) post = (post <= 1.0f && post >= 0.001f) ? post : 0.0f;
            }
          }
          bstore(sc.pg + tcell * sc.pg_stride, ul4 * sc.pg_stride, post);   // after this cell's zm was read (prefetch)
          if (lane == 0) bnd_put_pf(bz, j0, Zm, Ze, Zf, E);
          RZm = Zm; RZe = Ze; RZf = Zf; Re = E;
        }
        // refill slot u after its value is dead, so the load reuses the register
        // (a loop-carried copy of a pending load would drain vmcnt)
        const int64_t at = cell0 + (int64_t)max(t - kPrefetch, -1) * 64;
        if constexpr ((M & kHmm5) != 0) q5[u] = bload(sc.f5 + at, ul4);
        if constexpr ((M & kPF) != 0) qz[u] = bload(sc.zm + at, 2 * ul4);
        cursor_prev(c, C, T_.ins, local_row);
        j0 = j0 == 0 ? W - 1 : j0 - 1;
      }
      }
    }
  }
}

// =====================================================================
// Merge + MEA + sparsify: forward-order sweep over the merged posterior.
// =====================================================================
// NP: the ArrangePosteriorProbs pair body of npdoAlign (CPNP/MSA.cpp:1670-1753):
// pid 0/1 merge the squares in its order (global, local, 5-state), and the
// distance is score / #B of the MEA path.  #B rides along the value
// recurrence: every cell carries the B count of the path its ChooseBestOfThree
// choice extends (the traceback follows exactly those choices), so the last
// cell holds the count of the traced path without a traceback matrix.
#ifndef MLP_ELL_CHUNK
#define MLP_ELL_CHUNK 8
#endif
constexpr int kEllChunk = MLP_ELL_CHUNK;   // staged ELL entries a lane writes at once (4, 8 or 16)
static_assert(kEllChunk == 4 || kEllChunk == 8 || kEllChunk == 16 || kEllChunk == 32, "ELL chunk: 4, 8, 16 or 32 entries");
template <int M, int PID, bool NP = false>
#ifndef MLP_MERGE_WAVES
#define MLP_MERGE_WAVES 6
#endif
// (NP with all three models carries the #B counts beside their values: at 6
// waves its 80 VGPRs spilled 56 bytes a lane; 5 waves give it 96)
__global__ __launch_bounds__(256, NP && M == (kHmm5 | kLocal | kPF) ? 5 : MLP_MERGE_WAVES) void k_merge(ModelScalars ms, SeqSet sq, PairMeta pm, ChainMeta cm,
                                               PairRec* __restrict__ rec, Scratch sc, int64_t nchains,
                                               int lds_seq) {
  __shared__ double ex[7 * 6];
  __shared__ float noins[26];   // the merge needs no emissions; cursor fills ins from here
  extern __shared__ __align__(16) uint8_t dyn[];
  if (threadIdx.x < 26) noins[threadIdx.x] = 0.f;
  if (threadIdx.x == 0) mlp_exp_table(ex);
  __syncthreads();
  const int64_t ch = wave_index();
  if (ch >= nchains) return;
  const int lane = threadIdx.x & 63;
  const ChainView C = stage_chain<kStageMerge>(dyn, lds_seq, ch, sq, pm, cm, rec);
  const int W = C.W, S = C.S;
  const int64_t cell0 = cm.cell_off[ch] + 64;   // slot of step tau, lane l: cell0 + tau * 64 + l
  const uint32_t ul4 = (uint32_t)lane * 4;
  const int64_t bo = cm.bnd_off[ch];
  int j63 = W - 63;   // lane 63's column (scalar; see k_forward)
  const int last = S * W + 63;   // last step with an active lane
  Cursor c;
  cursor_start_fwd(c, C, noins, lane);
  float Lv = 0.f, Uv = 0.f, Dv = 0.f;
  int Lc = 0, Uc = 0, Dc = 0;   // NP: #B of the path into the left / up / diagonal cell
  int cnt = 0;
  // MEA boundary row (stacked row 64k - 1), double-buffered as in BoundaryChunks
  float bch = 0.f, bnx = 0.f;
  int cch = 0, cnx = 0;
  constexpr int QD = 8;  // divides every segment (chain widths are multiples of 8): 12 or 16 break the queue
  static_assert(kWidthQuantum % QD == 0 && 64 % QD == 0, "the merge's load queue must divide every segment");
  // fixed-register load queue: slot u serves steps t0 + u (segments hold
  // whole groups of QD steps); values of idle cells are never used
  float q5[QD] = {}, ql[QD] = {}, qb[QD] = {}, qg[QD] = {};
#pragma unroll
  for (int k = 0; k < QD; ++k) {
    const int64_t at = cell0 + (int64_t)k * 64;
    if constexpr ((M & kHmm5) != 0) q5[k] = bload(sc.f5 + at, ul4);
    if constexpr ((M & kLocal) != 0) { ql[k] = bload(sc.fl + at, ul4); qb[k] = bload(sc.bl + at, ul4); }
    if constexpr ((M & kPF) != 0) qg[k] = bload(sc.pg + at * sc.pg_stride, ul4 * sc.pg_stride);
  }
  const uint16_t* const ecol = sc.ell_col + C.ell0 * kEll;   // the chain's ELL rows (wave-uniform)
  const float* const evals = sc.ell_val + C.ell0 * kEll;
  // the lane's staged ELL entries (see the cutoff below), kEllChunk of them
  constexpr int KS = kEllChunk;
  __shared__ __align__(16) float ell_stv[kWavesPerBlock * 64 * KS];
  __shared__ __align__(16) uint16_t ell_stc[kWavesPerBlock * 64 * KS];
  float* const stv = ell_stv + ((threadIdx.x >> 6) * 64 + lane) * KS;
  uint16_t* const stc = ell_stc + ((threadIdx.x >> 6) * 64 + lane) * KS;
  // entries k0 .. k0 + KS - 1 of the lane's row (k0 a multiple of KS:
  // aligned slots of the row's kEll)
  auto ell_flush = [&](int k0) {
    const uint32_t e = c.ellr + (uint32_t)k0;
#pragma unroll
    for (int q = 0; q < KS / 4; ++q) bstore4(evals, 4u * e + 16u * q, reinterpret_cast<const float4*>(stv)[q]);
    if constexpr (KS == 4) {
      bstore2(ecol, 2u * e, *reinterpret_cast<const uint2*>(stc));
    } else {
#pragma unroll
      for (int q = 0; q < KS / 8; ++q) bstore4(ecol, 2u * e + 16u * q, reinterpret_cast<const uint4*>(stc)[q]);
    }
  };
  const int nseg = (W + 63) >> 6;
  for (int k = 0; k <= S; ++k) {
    const int segs = k < S ? nseg : 1;
    for (int m = 0; m < segs; ++m) {
      const int t_lo = k * W + 64 * m;
      const int t_hi = k < S ? min(t_lo + 64, (k + 1) * W) : t_lo + 64;
      if (k < S) {
        boundary_fence();
        bch = bnx;
        bnx = sc.bndm[bo + min((m + 1 < nseg ? 64 * (m + 1) : 0) + lane, W - 1)];
        if constexpr (NP) {
          cch = cnx;
          cnx = sc.bndc[bo + min((m + 1 < nseg ? 64 * (m + 1) : 0) + lane, W - 1)];
        }
      }
      const bool take_bnd = k >= 1 && k < S;
      for (int t0 = t_lo; t0 < t_hi; t0 += QD)
#pragma unroll
      for (int u = 0; u < QD; ++u) {
        const int t = t0 + u;
        const int i = c.i, j = c.j, L1 = c.L1, L2 = c.L2;
        // local f + b (CPNP/ProbabilisticModel.h:484): the same float add the
        // backward sweep used to do in place
        const float f5v = q5[u], flv = ql[u] + qb[u], pgv = qg[u];
        Dv = Uv;
        // boundary column t - t_lo in lane 0 of the rotating chunk (BoundaryChunks::shift)
        Uv = take_bnd ? mlp_shr1(Lv, bch) : mlp_shr1z(Lv);
        if (take_bnd) bch = mlp_shl1z(bch);
        if constexpr (NP) {
          Dc = Uc;
          Uc = take_bnd ? mlp_shr1i(Lc, cch) : mlp_shr1zi(Lc);
          if (take_bnd) cch = mlp_shl1zi(cch);
        }
        const bool act = (uint32_t)(j - 1) < (uint32_t)c.jm;   // q >= 0, i >= 1, 1 <= j <= L2
        float P = 0.f;
        if (act) {
          if constexpr (PID == 2) {
            P = mlp_post_from_sum_t(flv, c.TL, ex);
          } else if constexpr (PID == kPidQP) {
            // QP/ParallelProbabilisticModel.cpp:246-248 (a zero total reads as 1) and
            // PosteriorStage::combineMatrices (QP/PosteriorStage.cpp:176-178)
            const float v1 = mlp_post_from_sum_t(f5v, c.T5 == 0.f ? 1.0f : c.T5, ex);
            const float v2 = pgv;
            P = sqrtf((v1 * v1 + v2 * v2) * 0.5f);
          } else if constexpr (PID >= 3) {
            P = pgv;
          } else {
            const float v1 = mlp_post_from_sum_t(f5v, c.T5, ex);
            const float v2 = pgv;
            const float v3 = mlp_post_from_sum_t(flv, c.TL, ex);
            if constexpr (NP)
              P = sqrtf(mlp_div3(v2 * v2 + v3 * v3 + v1 * v1));  // CPNP/MSA.cpp:1699-1708
            else
              P = sqrtf(mlp_div3(v1 * v1 + v2 * v2 + v3 * v3));  // CPNP/MSA.cpp:992-1001
          }
        }
        // MEA (CPNP/ProbabilisticModel.h:831-834): value of ChooseBestOfThree
        float Cv = 0.f;
        int Cc = 0;
        if (act) {
          const float x1 = P + Dv, x2 = Lv, x3 = Uv;
          Cv = mlp_max(mlp_max(x1, x2), x3);
          if constexpr (NP)  // ChooseBestOfThree's pick (ScoreType.h:347-366): D, else L, else U
            Cc = (x1 >= x2 && x1 >= x3) ? Dc + 1 : (x1 < x2 && x2 >= x3) ? Lc : Uc;
          // POSTERIOR_CUTOFF (CPNP/SparseMatrix.h:14).  A row's entries arrive
          // one per step over ~10-30 steps; stored one by one (2 + 4 bytes) the
          // rows' lines left L2 partly written several times (1.6 B/cell written
          // against 0.16, the stores ~20% of the merge).  Staged per lane in
          // LDS, they go out kEllChunk at a time (aligned 16-byte pieces), the row's
          // last chunk when it completes (slots past cnt carry stale values
          // k_compact never reads).  A row past kEll entries keeps counting,
          // stores nothing more and is flagged when it completes.
          const bool keep = P >= 0.01f;
          if (keep && cnt < kEll) {
            stv[cnt & (KS - 1)] = PID == kPidQP ? (float)(uint32_t)(uint16_t)(P * 65535.0f) / 65535.0f : P;
            stc[cnt & (KS - 1)] = (uint16_t)j;
            if ((cnt & (KS - 1)) == KS - 1) ell_flush(cnt - (KS - 1));
          }
          cnt += keep ? 1 : 0;
          if (j == L2) {   // row complete
            if ((cnt & (KS - 1)) != 0 && cnt < kEll) ell_flush(cnt & ~(KS - 1));
            if (cnt > kEll) atomicOr(&rec[c.slot].flags, 2);
            sc.ell_cnt[c.ell + (i - 1)] = cnt;
            // (the pair's nnz: k_pair_nnz sums these counts after the merge)
            cnt = 0;
            if (i == L1) {
              rec[c.slot].mea = Cv;
              if constexpr (NP)
                rec[c.slot].dist = Cv / (float)Cc;  // CPNP/MSA.cpp:1744-1753
              else
                rec[c.slot].dist = 1.0f - Cv / (float)min(L1, L2);
            }
          }
        }
        if (lane == 63) bnd_put(sc.bndm + bo, j63, Cv);
        Lv = Cv;
        if constexpr (NP) {
          if (lane == 63) bnd_put(sc.bndc + bo, j63, Cc);
          Lc = Cc;
        }
        // refill slot u once its value is dead (see k_backward)
        const int64_t at = cell0 + (int64_t)min(t + QD, last) * 64;
        if constexpr ((M & kHmm5) != 0) q5[u] = bload(sc.f5 + at, ul4);
        if constexpr ((M & kLocal) != 0) { ql[u] = bload(sc.fl + at, ul4); qb[u] = bload(sc.bl + at, ul4); }
        if constexpr ((M & kPF) != 0) qg[u] = bload(sc.pg + at * sc.pg_stride, ul4 * sc.pg_stride);
        cursor_next(c, C, noins);
        j63 = j63 + 1 == W ? 0 : j63 + 1;
      }
    }
  }
}

// ------------------------------------------------------------ launchers
template <template <int> class K, bool kFwd>
static hipError_t launch_sweep(int models, const ModelScalars& ms, const Tables* tab, SeqSet seqs,
                               PairMeta pm, ChainMeta cm, PairRec* rec, Scratch sc, int64_t nchains,
                               int lds_seq, hipStream_t st, const SideStream* side) {
  const ChainLaunch l = chain_launch(nchains, lds_seq);
  auto go = [&](auto m_tag, hipStream_t s) {
    constexpr int Mv = decltype(m_tag)::value;
    hipLaunchKernelGGL((K<Mv>::fn), l.grid, l.block, l.lds, s, ms, tab, seqs, pm, cm, rec, sc, nchains, lds_seq);
  };
  // two kernels: the second on the side stream, joined back before returning
  auto pair = [&](auto a_tag, auto... b_tags) -> hipError_t {
    if (!side) {
      go(a_tag, st);
      (go(b_tags, st), ...);
      return hipSuccess;
    }
    hipError_t e;
    // per-model chains: the backward follows the forward on each stream
    const bool fork = !(side->join_mode == 2 && !kFwd);
    const bool record = !(side->join_mode == 2 && kFwd);
    const bool wait = side->join_mode == 0 || (side->join_mode == 1 && kFwd);
    if (fork) {
      if ((e = hipEventRecord(side->fork, st)) != hipSuccess) return e;
      if ((e = hipStreamWaitEvent(side->st, side->fork, 0)) != hipSuccess) return e;
    }
    go(a_tag, st);
    (go(b_tags, side->st), ...);
    if (record && (e = hipEventRecord(side->join, side->st)) != hipSuccess) return e;
    return wait ? hipStreamWaitEvent(st, side->join, 0) : hipSuccess;
  };
  switch (models) {
    case kHmm5 | kLocal | kPF:
      // fp32 HMMs and the fp64 partition function as two sweeps: fewer VGPRs each
      return pair(std::integral_constant<int, kHmm5 | kLocal>{}, std::integral_constant<int, kPF>{});
    case kLocal: go(std::integral_constant<int, kLocal>{}, st); break;
    case kPF: go(std::integral_constant<int, kPF>{}, st); break;
    case kHmm5: go(std::integral_constant<int, kHmm5>{}, st); break;
    case kHmm5 | kPF | kQP:  // QuickProbs: the same fp32 pair-HMM sweep, its own partition function
      return pair(std::integral_constant<int, kHmm5>{}, std::integral_constant<int, kPF | kQP>{});
    default: return hipErrorInvalidValue;
  }
  return hipSuccess;
}
template <int M> struct ForwardK { static constexpr auto fn = k_forward<M>; };
template <int M> struct BackwardK { static constexpr auto fn = k_backward<M>; };

hipError_t launch_forward(int models, const ModelScalars& ms, const Tables* tab, SeqSet seqs,
                          PairMeta pm, ChainMeta cm, PairRec* rec, Scratch sc, int64_t nchains,
                          int lds_seq, hipStream_t st, const SideStream* side) {
  if (nchains <= 0) return hipSuccess;
  const hipError_t e = launch_sweep<ForwardK, true>(models, ms, tab, seqs, pm, cm, rec, sc, nchains, lds_seq, st, side);
  if (e != hipSuccess) return e;
  return hipGetLastError();
}

hipError_t launch_backward(int models, const ModelScalars& ms, const Tables* tab, SeqSet seqs,
                           PairMeta pm, ChainMeta cm, PairRec* rec, Scratch sc, int64_t nchains,
                           int lds_seq, int64_t npairs, hipStream_t st, const SideStream* side) {
  if (nchains <= 0) return hipSuccess;
  const hipError_t e = launch_sweep<BackwardK, false>(models, ms, tab, seqs, pm, cm, rec, sc, nchains, lds_seq, st, side);
  if (e != hipSuccess) return e;
  // fold the 5-state backward total (needs Tables for the initial cells)
  if (models & kHmm5) return launch_fold_totals(ms, tab, seqs, pm, rec, npairs, st);
  return hipGetLastError();
}

hipError_t launch_merge(int models, int pid, const ModelScalars& ms, SeqSet seqs, PairMeta pm,
                        ChainMeta cm, PairRec* rec, Scratch sc, int64_t nchains, int lds_seq,
                        hipStream_t st) {
  if (nchains <= 0) return hipSuccess;
  const ChainLaunch l = chain_launch(nchains, lds_seq);
  if (pid & kPidNpdo) {
    pid &= ~kPidNpdo;
    if (pid == 2)
      hipLaunchKernelGGL((k_merge<kLocal, 2, true>), l.grid, l.block, l.lds, st, ms, seqs, pm, cm, rec, sc, nchains, lds_seq);
    else if (pid >= 3)
      hipLaunchKernelGGL((k_merge<kPF, 3, true>), l.grid, l.block, l.lds, st, ms, seqs, pm, cm, rec, sc, nchains, lds_seq);
    else
      hipLaunchKernelGGL((k_merge<kHmm5 | kLocal | kPF, 0, true>), l.grid, l.block, l.lds, st, ms, seqs, pm, cm, rec, sc, nchains, lds_seq);
  } else if (pid == kPidQP)
    hipLaunchKernelGGL((k_merge<kHmm5 | kPF | kQP, kPidQP>), l.grid, l.block, l.lds, st, ms, seqs, pm, cm, rec, sc, nchains, lds_seq);
  else if (pid == 2)
    hipLaunchKernelGGL((k_merge<kLocal, 2>), l.grid, l.block, l.lds, st, ms, seqs, pm, cm, rec, sc, nchains, lds_seq);
  else if (pid >= 3)
    hipLaunchKernelGGL((k_merge<kPF, 3>), l.grid, l.block, l.lds, st, ms, seqs, pm, cm, rec, sc, nchains, lds_seq);
  else
    hipLaunchKernelGGL((k_merge<kHmm5 | kLocal | kPF, 0>), l.grid, l.block, l.lds, st, ms, seqs, pm, cm, rec, sc, nchains, lds_seq);
  (void)models;
  return hipGetLastError();
}

}  // namespace mlp
