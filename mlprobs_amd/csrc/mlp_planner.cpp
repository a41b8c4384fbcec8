// mlp_planner.cpp -- batch planning of the posterior stage and the Viterbi
// family test: chains of pairs (mlp_kernels.h, "Chains"), the batch scratch's
// sub-buffers and the plan's upload.
#include "mlp_runtime.h"

// Chains of one batch (mlp_kernels.h, "Chains"): pairs sorted by column
// count, stacked greedily; slots ordered chain by chain, chains longest first.

void plan_chains(const mlp_ctx* c, int64_t p, int64_t q, ChainPlan& P) {
  const int64_t np = q - p;
  std::vector<int64_t> byw(np);
  std::iota(byw.begin(), byw.end(), p);
  std::stable_sort(byw.begin(), byw.end(), [&](int64_t x, int64_t y) {
    const int ax = c->lens[c->pb[x]], ay = c->lens[c->pb[y]];
    if (ax != ay) return ax > ay;
    return c->lens[c->pa[x]] > c->lens[c->pa[y]];
  });
  // Chains are built greedily up to a row target.  The sweeps are
  // throughput-bound at their occupancy (6 waves per SIMD): per-SIMD step
  // rate measured at C3 (MI355X) 1.44 / 1.50 / 1.74 wave-steps per us at
  // 4.3 / 5.1 / 6 resident waves, so what matters is keeping every slot
  // busy -- at least ~2 waves per resident slot -- while the strip and
  // skew waste stays small; with the two model kernels overlapped
  // (SideStream) 640- to 4096-row chains run within 1 % of each other in
  // the sweeps, and the merge (one kernel, its own tail) prefers ~1024.
  int64_t total_rows = 0;
  for (int64_t k = p; k < q; k++) total_rows += c->lens[c->pa[k]] + 1;
  int64_t target_rows = std::max<int64_t>(512, std::min<int64_t>(1024, total_rows / (2 * 6 * 4 * (int64_t)c->cus)));
  struct ChainH { int64_t begin, end; int W, rows, seq; int64_t cost; };
  std::vector<ChainH> chains;
  ChainH cur{0, 0, 0, 0, 0, 0};
  for (int64_t k = 0; k < np; k++) {
    const int64_t x = byw[k];
    const int L1 = c->lens[c->pa[x]], L2 = c->lens[c->pb[x]];
    const int w = chain_width(L2);
    const int n_in = (int)(cur.end - cur.begin);
    const bool fits = n_in > 0 && n_in < kChainMax && cur.rows + L1 + 1 <= target_rows &&
                      chain_seq_bytes(cur.W, cur.rows - n_in + L1, n_in + 1) <= kChainSeqSoft &&
                      cur.W - w <= std::max(8, cur.W / 16);
    if (!fits) {
      if (cur.end > cur.begin) chains.push_back(cur);
      cur = ChainH{k, k, w, 0, 0, 0};
    }
    cur.end = k + 1;
    cur.rows += L1 + 1;
    cur.seq = chain_seq_bytes(cur.W, cur.rows - (int)(cur.end - cur.begin), (int)(cur.end - cur.begin));
  }
  if (cur.end > cur.begin) chains.push_back(cur);
  for (auto& h : chains) h.cost = (int64_t)chain_strips(h.rows) * h.W;
  std::stable_sort(chains.begin(), chains.end(), [](const ChainH& x, const ChainH& y) { return x.cost > y.cost; });
  P = ChainPlan();
  P.np = np;
  P.nch = (int64_t)chains.size();
  P.order.resize(np); P.pa.resize(np); P.pb.resize(np); P.row0.resize(np); P.chain.resize(np);
  P.rm.resize(np); P.ell.resize(np);
  P.first.resize(P.nch); P.count.resize(P.nch); P.width.resize(P.nch); P.rows.resize(P.nch);
  P.seqb.resize(P.nch); P.cell.resize(P.nch); P.bndo.resize(P.nch);
  int64_t s = 0;
  for (int64_t h = 0; h < P.nch; h++) {
    const ChainH& ch = chains[h];
    P.first[h] = (int32_t)s;
    P.count[h] = (int32_t)(ch.end - ch.begin);
    P.width[h] = ch.W;
    P.rows[h] = ch.rows;
    P.seqb[h] = ch.seq;
    P.cell[h] = P.cells;
    P.bndo[h] = P.bnd;
    P.cells += chain_steps(ch.rows, ch.W) * 64;
    P.bnd += ch.W;
    P.lds_seq = std::max(P.lds_seq, ch.seq);
    int row0 = 0;
    for (int64_t k = ch.begin; k < ch.end; k++, s++) {
      const int64_t x = byw[k];
      const int L1 = c->lens[c->pa[x]], L2 = c->lens[c->pb[x]];
      P.order[s] = x;
      P.pa[s] = c->pa[x];
      P.pb[s] = c->pb[x];
      P.row0[s] = row0;
      P.chain[s] = (int32_t)h;
      P.rm[s] = P.rm_total;
      P.ell[s] = P.ell_rows;
      row0 += L1 + 1;
      P.rm_total += (int64_t)L1 * local_chunks(L2);
      P.ell_rows += L1;
    }
  }
  int kmax = 0;
  for (int64_t h = 0; h < P.nch; h++) kmax = std::max(kmax, P.count[h]);
  P.lds_seq = chain_lds_pack(P.lds_seq, kmax);
}

// Upload the plan's per-slot / per-chain metadata; returns device views.

PlanDev carve_plan(Carver& cv, const ChainPlan& P) {
  PlanDev d;
  d.o_pa = cv.take(P.np * 4); d.o_pb = cv.take(P.np * 4); d.o_r0 = cv.take(P.np * 4);
  d.o_ch = cv.take(P.np * 4); d.o_rm = cv.take(P.np * 8); d.o_ell = cv.take(P.np * 8);
  d.o_cf = cv.take(P.nch * 4); d.o_cc = cv.take(P.nch * 4); d.o_cw = cv.take(P.nch * 4);
  d.o_cr = cv.take(P.nch * 4); d.o_cs = cv.take(P.nch * 4); d.o_cco = cv.take(P.nch * 8);
  d.o_cbo = cv.take(P.nch * 8);
  return d;
}
int upload_plan(mlp_ctx* c, char* base, const PlanDev& d, const ChainPlan& P, PairMeta& pm,
                       ChainMeta& cm, hipStream_t st, uint8_t* stage) {
  if (!st) st = c->stream;
  // with `stage` (pinned, >= the plan region's bytes) the arrays are gathered
  // there and go up in one asynchronous copy; else one pageable copy each
  const size_t span = d.o_cbo + P.nch * 8 - d.o_pa;
  auto up = [&](size_t o, const void* h, size_t n) {
    if (stage) {
      memcpy(stage + (o - d.o_pa), h, n);
      return hipSuccess;
    }
    return hipMemcpyAsync(base + o, h, n, hipMemcpyHostToDevice, st);
  };
  HIPCHK(c, up(d.o_pa, P.pa.data(), P.np * 4));
  HIPCHK(c, up(d.o_pb, P.pb.data(), P.np * 4));
  HIPCHK(c, up(d.o_r0, P.row0.data(), P.np * 4));
  HIPCHK(c, up(d.o_ch, P.chain.data(), P.np * 4));
  HIPCHK(c, up(d.o_rm, P.rm.data(), P.np * 8));
  HIPCHK(c, up(d.o_ell, P.ell.data(), P.np * 8));
  HIPCHK(c, up(d.o_cf, P.first.data(), P.nch * 4));
  HIPCHK(c, up(d.o_cc, P.count.data(), P.nch * 4));
  HIPCHK(c, up(d.o_cw, P.width.data(), P.nch * 4));
  HIPCHK(c, up(d.o_cr, P.rows.data(), P.nch * 4));
  HIPCHK(c, up(d.o_cs, P.seqb.data(), P.nch * 4));
  HIPCHK(c, up(d.o_cco, P.cell.data(), P.nch * 8));
  HIPCHK(c, up(d.o_cbo, P.bndo.data(), P.nch * 8));
  if (stage) HIPCHK(c, hipMemcpyAsync(base + d.o_pa, stage, span, hipMemcpyHostToDevice, st));
  pm.pa = (const int32_t*)(base + d.o_pa);
  pm.pb = (const int32_t*)(base + d.o_pb);
  pm.row0 = (const int32_t*)(base + d.o_r0);
  pm.chain = (const int32_t*)(base + d.o_ch);
  pm.rm_off = (const int64_t*)(base + d.o_rm);
  pm.ell_row = (const int64_t*)(base + d.o_ell);
  cm.first = (const int32_t*)(base + d.o_cf);
  cm.count = (const int32_t*)(base + d.o_cc);
  cm.width = (const int32_t*)(base + d.o_cw);
  cm.rows = (const int32_t*)(base + d.o_cr);
  cm.seq_bytes = (const int32_t*)(base + d.o_cs);
  cm.cell_off = (const int64_t*)(base + d.o_cco);
  cm.bnd_off = (const int64_t*)(base + d.o_cbo);
  return MLP_OK;
}

// upper bound of one pair's step-diagonal slots (as if alone in a chain whose
// width may exceed its own by the stacking slack)
int64_t pair_slots_bound(const mlp_ctx* c, int64_t q) {
  const int L1 = c->lens[c->pa[q]], L2 = c->lens[c->pb[q]];
  const int64_t Wb = chain_width(L2) + chain_width(L2) / 8 + 8;
  return (int64_t)(L1 + 1 + 64) * Wb + 80 * 64;
}
int64_t pair_width_bound(const mlp_ctx* c, int64_t q) {
  const int L2 = c->lens[c->pb[q]];
  return chain_width(L2) + chain_width(L2) / 8 + 8;
}
