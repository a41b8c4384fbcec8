// viterbi.hip -- all-pairs Viterbi alignment of the family test
// (CPNP/MSA.cpp:646-882 ModelAdjustmentTest / Alter_ModelAdjustmentTest, each
// pair through ProbabilisticModel::ComputeViterbiAlignment,
// CPNP/ProbabilisticModel.h:1043-1170).
//
// k_viterbi sweeps the chains with the same wrapped wavefront as the
// posterior forward sweep (mlp_chain.h): 3-state max-plus recurrence, one
// traceback byte per cell in the step-diagonal layout (bits 0-1: match
// predecessor 0..2 or 3 = none; bit 2: X from X; bit 3: Y from Y).
// k_vit_trace walks every pair back from its best terminating state, one lane
// per pair, and emits the path plus the identical-residue count.
#include "mlp_chain.h"

namespace mlp {

__global__ __launch_bounds__(256) void k_viterbi(ModelScalars ms, const Tables* __restrict__ tab,
                                                 SeqSet sq, PairMeta pm, ChainMeta cm, Scratch sc,
                                                 VitOut vo, int64_t nchains, int lds_seq) {
  __shared__ LdsTablesT<true, false> T_;
  extern __shared__ __align__(16) uint8_t dyn[];
  stage_tables(T_, tab);
  const int64_t ch = wave_index();
  if (ch >= nchains) return;
  const int lane = threadIdx.x & 63;
  const ChainView C = stage_chain<kStageFwd>(dyn, lds_seq, ch, sq, pm, cm, nullptr);
  const int W = C.W, S = C.S;
  const int64_t base = cm.cell_off[ch] + 64 + lane;
  const int64_t bo = cm.bnd_off[ch];
  Cursor c;
  cursor_start_fwd(c, C, T_.ins, lane);
  // Lx = own cell (i, j-1), Ux = (i-1, j), Dx = (i-1, j-1); states M, X, Y
  float LV[3], UV[3], DV[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) LV[k] = UV[k] = DV[k] = LZ;
  float n5[5] = {}, m5[5] = {};
  double z0 = 0, z1 = 0, z2 = 0;
  int ze = 0;
  BoundaryChunks<kLocal> bc;
  const int nseg = (W + 63) >> 6;
  for (int k = 0; k <= S; ++k) {
    const int segs = k < S ? nseg : 1;
    for (int m = 0; m < segs; ++m) {
      const int t_lo = k * W + 64 * m;
      const int t_hi = k < S ? min(t_lo + 64, (k + 1) * W) : t_lo + 64;
      if (k < S) {
        boundary_fence();
        bc.advance();
        bc.load_next(sc, bo, W, m + 1 < nseg ? 64 * (m + 1) : 0, lane);
      }
      const bool take_bnd = k >= 1 && k < S;
      for (int t0 = t_lo; t0 < t_hi; t0 += 4)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = t0 + u;
        const int i = c.i, j = c.j;
        const int c1 = c.c1;
        const int c2 = C.seq[c.ca];
        const float ins1 = c.ins1, ins2 = T_.ins[c2];
#pragma unroll
        for (int k3 = 0; k3 < 3; ++k3) DV[k3] = UV[k3];
        if (take_bnd)
          bc.template shift<true, true>(t - t_lo, n5, m5, LV, UV, z0, z1, z2, ze, z0, z1, z2, ze);
        else
          bc.template shift<true, false>(0, n5, m5, LV, UV, z0, z1, z2, ze, z0, z1, z2, ze);
        // CPNP/ProbabilisticModel.h:1086-1124
        float V0 = LZ, V1 = LZ, V2 = LZ;
        int b0 = 3, b1 = 0, b2 = 0;
        if (i == 0 && j == 0) { V0 = ms.vit_init[0]; V1 = ms.vit_init[1]; V2 = ms.vit_init[2]; }
        if (i > 0 && j > 0) {
          const float mt = T_.match[c1 * 26 + c2];
#pragma unroll
          for (int k3 = 0; k3 < 3; ++k3) {
            const float nv = DV[k3] + ms.lt[k3][0] + mt;
            if (V0 < nv) { V0 = nv; b0 = k3; }
          }
        }
        if (i > 0) {
          const float fm = ins1 + UV[0] + ms.lt[0][1];
          const float fi = ins1 + UV[1] + ms.lt[1][1];
          V1 = fm >= fi ? fm : fi;
          b1 = fm >= fi ? 0 : 1;
        }
        if (j > 0) {
          const float fm = ins2 + LV[0] + ms.lt[0][2];
          const float fi = ins2 + LV[2] + ms.lt[2][2];
          V2 = fm >= fi ? fm : fi;
          b2 = fm >= fi ? 0 : 1;
        }
        sc.vt[base + (int64_t)t * 64] = (uint8_t)(b0 | (b1 << 2) | (b2 << 3));
        if (c.q >= 0 && i == c.L1 && j == c.L2) {
          // best terminating state (CPNP/ProbabilisticModel.h:1128-1139)
          float best = LZ;
          int st = -1;
          const float tv[3] = {V0 + ms.vit_init[0], V1 + ms.vit_init[1], V2 + ms.vit_init[2]};
#pragma unroll
          for (int k3 = 0; k3 < 3; ++k3)
            if (best < tv[k3]) { best = tv[k3]; st = k3; }
          vo.state[c.slot] = st;
        }
        if (lane == 63) {   // the boundary record of the column (mlp_chain.h: the local model's three)
          float4* const r = reinterpret_cast<float4*>(sc.bnd5 + bo * 8) + 2 * (int64_t)(uint32_t)j;
          r[1] = make_float4(0.f, V0, V1, V2);
        }
        LV[0] = V0; LV[1] = V1; LV[2] = V2;
        cursor_next(c, C, T_.ins);
      }
    }
  }
}

// Traceback (CPNP/ProbabilisticModel.h:1143-1165), one lane per pair; the
// path is written in traceback order.  A match cell without a predecessor
// better than LOG_ZERO (the reference leaves -1 there and then reads out of
// the state block) is followed as a match; it does not occur on real input.
__global__ __launch_bounds__(256) void k_vit_trace(SeqSet sq, PairMeta pm, ChainMeta cm, Scratch sc,
                                                   VitOut vo, int64_t npairs) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npairs) return;
  const int a = pm.pa[p], b = pm.pb[p];
  const int L1 = sq.len[a], L2 = sq.len[b];
  const uint8_t* s1 = sq.res + sq.off[a];
  const uint8_t* s2 = sq.res + sq.off[b];
  const int ch = pm.chain[p];
  const int W = cm.width[ch];
  const int64_t cb = cm.cell_off[ch] + 64;
  const int row0 = pm.row0[p];
  uint8_t* out = vo.path + vo.path_off[p];
  int state = vo.state[p];
  int r = L1, c = L2, n = 0;
  float match = 0;
  while (r != 0 || c != 0) {
    const int g = row0 + r;
    const int ln = g & 63;
    const int64_t tau = (int64_t)(g >> 6) * W + ln + c;
    const int bits = sc.vt[cb + tau * 64 + ln];
    int ns = state == 0 ? (bits & 3) : state == 1 ? ((bits >> 2) & 1) : ((bits >> 3) & 1) * 2;
    if (ns == 3) ns = 0;
    if (state == 0) {
      if (s1[r - 1] == s2[c - 1]) match += 1;
      --r; --c;
      out[n++] = 0;
    } else if (state == 1) {
      --r;
      out[n++] = 1;
    } else {
      --c;
      out[n++] = 2;
    }
    state = ns;
  }
  vo.path_len[p] = n;
  vo.match[p] = match;
}

hipError_t launch_viterbi(const ModelScalars& ms, const Tables* tab, SeqSet seqs, PairMeta pm,
                          ChainMeta cm, Scratch sc, VitOut vo, int64_t nchains, int lds_seq,
                          int64_t npairs, hipStream_t st) {
  if (nchains <= 0) return hipSuccess;
  const ChainLaunch l = chain_launch(nchains, lds_seq);
  hipLaunchKernelGGL(k_viterbi, l.grid, l.block, l.lds, st, ms, tab, seqs, pm, cm, sc, vo, nchains, lds_seq);
  hipLaunchKernelGGL(k_vit_trace, dim3((unsigned)((npairs + 255) / 256)), dim3(256), 0, st, seqs, pm, cm, sc, vo, npairs);
  return hipGetLastError();
}

}  // namespace mlp
