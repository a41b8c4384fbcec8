// mlp_posteriors.cpp -- the all-pairs posterior stage (mlp_posteriors):
// per batch k_forward -> k_backward -> local totals -> k_merge -> k_compact
// (posterior.hip, totals.hip), batches planned by mlp_planner.cpp under the
// scratch budget; the host context's and the sharded variants.  Reference:
// CPNP/MSA.cpp:907-1034 (pdoAlign / npdoAlign pair loops).
#include "mlp_runtime.h"

static int host_posteriors(mlp_ctx* c, int pid, float delta, int64_t p0, int64_t p1) {
  const bool npdo = (pid & kPidNpdo) != 0;
  pid &= ~kPidNpdo;
  if (c->store_p0 == c->store_p1 || p0 != c->store_p1) {  // as the device store: append or restart
    c->store_p0 = c->store_p1 = p0;
    c->store_total = 0; ++c->store_ver;
    c->hs.ent_off[p0] = 0;
    c->hs.cols.clear();
    c->hs.vals.clear();
  }
  Tables T;
  ModelScalars ms;
  if (pid == kPidQP) {  // QuickProbs' posterior stage (its HMM tables are these; its own PF)
    build_tables(T, ms, -1.f, true);
    mlph::qp_posteriors(T, ms, host_view(c), p0, p1, mlp_qp_cutoff, c->rp_off, c->hs, c->dist.data(),
                        c->mea.data(), c->nnz.data());
  } else {
    build_tables(T, ms, delta);
    const int rc = mlph::posteriors(T, ms, host_view(c), pid, npdo, p0, p1, c->rp_off, c->hs, c->dist.data(),
                                    c->mea.data(), c->nnz.data(), c->err);
    if (rc) return rc == 3 ? MLP_ERR_OVERFLOW : MLP_ERR_STATE;
  }
  for (int64_t p = p0; p <= p1; p++) c->ent_off[p] = c->hs.ent_off[p];
  c->store_p1 = p1;
  c->store_total = c->hs.ent_off[p1];
  ++c->store_ver;
  return MLP_OK;
}

static int sharded_posteriors(mlp_ctx* c, int pid, float delta, int S) {
  int rc;
  if ((rc = ensure_shards(c, S))) return rc;
  std::vector<int64_t> b(S), e(S);
  for (int s = 0; s < S; s++) mlp_shard_plan(c->n, c->lens.data(), S, s, &b[s], &e[s]);
  if ((rc = run_shards(c, [&](mlp_ctx* ch, int s) { return mlp_posteriors(ch, pid, delta, b[s], e[s]); })))
    return rc;
  return allgather_shards(c);
}

extern "C" {

int mlp_posteriors(mlp_ctx* c, int pid, float delta, int64_t p0, int64_t p1) {
  if (!c) return MLP_ERR_ARG;
  if (c->n < 2) { c->err = "family needs >= 2 sequences"; return MLP_ERR_STATE; }
  if (p0 < 0 || p1 > c->P || p0 > p1) { c->err = "bad pair range"; return MLP_ERR_ARG; }
  if (c->host) return host_posteriors(c, pid, delta, p0, p1);
  if (p0 == 0 && p1 == c->P && !c->comm) {
    const int S = shard_count(c);
    if (S > 1) return sharded_posteriors(c, pid, delta, S);
  }
  hipSetDevice(c->device);
  // a range that continues the held one is appended; anything else restarts
  if (c->store_p0 == c->store_p1 || p0 != c->store_p1) {
    c->store_p0 = c->store_p1 = p0;
    c->store_total = 0; ++c->store_ver;
  }
  ModelScalars ms;
  build_tables(c->h_tables, ms, delta, pid == kPidQP);
  HIPCHK(c, hipMemcpyAsync(c->d_tables, &c->h_tables, sizeof(Tables), hipMemcpyHostToDevice, c->stream));
  const int models = model_set_for_pid(pid);
  SeqSet seqs{c->d_res, c->d_off, c->d_len};
  hipStream_t st = c->stream;

  // step-diagonal bytes per slot of the models this pid runs: f5 (5-state),
  // fl + bl (local), zm + pg (partition function)
  // Under a small scratch budget the PF posterior goes into the low half of
  // the PF forward Zm slot of its own cell (read kPrefetch steps before the
  // backward writes it): 4 B per cell less scratch, 20% bigger batches, at
  // the price of a strided read in the merge.  C3 at the CLIs' 16 GB:
  // posteriors 0.94 s against 1.01 s; at the bench's ~140 GB the batches are
  // large anyway and the merge's extra bytes cost 17 ms a step (690 vs
  // 679 ms; profiles/r03d_ab_tottr_pg.txt).  MLP_TEST_PG_SEPARATE=0 / 1 forces it.
  const double pg_knob = knob("MLP_TEST_PG_SEPARATE", -1);
  const bool pg_in_zm = pg_knob >= 0 ? pg_knob == 0 : c->scratch_budget <= (48ull << 30);
  const int slot_bytes =
      ((models & kHmm5) ? 4 : 0) + ((models & kLocal) ? 8 : 0) + ((models & kPF) ? (pg_in_zm ? 8 : 12) : 0);
  auto pair_bytes = [&](int64_t q) {
    const int L1 = c->lens[c->pa[q]], L2 = c->lens[c->pb[q]];
    const int64_t rmc = (models & kLocal) ? (int64_t)L1 * local_chunks(L2) : 0;
    return (size_t)(pair_slots_bound(c, q) * slot_bytes + rmc * 8) +
           (size_t)pair_width_bound(c, q) * (32 + 32 + 4 + 4) +
           (size_t)L1 * (kEll * 6 + 4 + 4) + 4 + kPerSlotMeta;  // + the lane fold's row bounds, repair slot
  };
  // Batches run one after another on the context stream (two batches
  // alternating over two streams with half the scratch each measured slower
  // at C3: 0.81 s vs 0.75 s, the smaller batches lose more to their tails
  // than the overlap wins); the host plans batch b + 1 while batch b's
  // kernels run, and finishes batch b (entry offsets from its pair records,
  // compaction into the store) while batch b + 1's sweeps run.
  const SideStream* side = &c->side;
  // model sets whose sweeps run as two kernels: the partition function's on the side stream
  const bool side_used = (models & kPF) && models != kPF;
  // k_local_totals: persistent waves, each with 64 candidate rows as wide as
  // the family's widest chain row (<= 1 GB of lists), sized once per call so
  // every batch carves the same bytes (no reallocation between batches) and
  // counted inside the scratch budget
  const int tot_row = (chain_width(c->max_len) + 15) & ~15;
  int tot_waves = (int)std::max<int64_t>(64, std::min<int64_t>(kTotalsWaves, (int64_t)(1LL << 30) / (64LL * tot_row * 4)));
  tot_waves = (tot_waves + kWavesPerBlock - 1) / kWavesPerBlock * kWavesPerBlock;  // whole workgroups
  const size_t clist_bytes = (models & kLocal) ? (size_t)tot_waves * 64 * tot_row * 4 : 0;
  // the forward local chain folded one pair per lane (k_local_list +
  // k_local_fold) between the forward and the backward sweeps, its
  // candidates listed into the local backward array (dead until the backward
  // sweep writes it), on the HMM stream while the partition function's
  // sweeps run on the side stream; the backward chains after the backward
  // sweep.  The fold lasts as long as its longest chain (~5 ms a batch), on
  // the HMM stream's critical path: under the CLIs' small budgets (PF
  // posterior in the Zm slots, ~38 batches at C3) the one-wave-per-pair
  // k_local_totals after both sweeps runs shorter (C3 drop-in posteriors
  // 0.92 against 1.03 s, profiles/r05b_cli_lanefold.txt).
  // MLP_TEST_TOT_LANEFOLD=0 / 1 forces either
  const double lf_knob = knob("MLP_TEST_TOT_LANEFOLD", -1);
  const bool lanefold = (models & kLocal) && (lf_knob >= 0 ? lf_knob != 0 : !pg_in_zm);
  // the side stream joins before the merge (the partition function's sweeps
  // run on without a join between them: the lane fold does not wait for them)
  SideStream side_lf;
  if (lanefold && side_used) {
    side_lf = *side;
    side_lf.join_mode = 2;
    side = &side_lf;
  }
  // the one-wave fold's listing bound: the folded chunk maxima of the rows
  // before (k_local_bounds) instead of their maximum (MLP_TEST_TOT_FOLDBOUND=0 / 1)
  const bool foldbound = (models & kLocal) && !lanefold && knob("MLP_TEST_TOT_FOLDBOUND", 1) != 0;
  // the one-wave fold's forward chains on stream2 beside the backward sweeps
  // (they read only what the forward sweep wrote), the backward chains after
  // them on the context stream (MLP_TEST_TOT_BESIDE=0 / 1 / 2, 2 the default:
  // the partition function's sweeps joined before the merge only, so the HMM
  // backward starts right after the HMM forward).  C3 drop-in posteriors at
  // 16 GB: 0.90 s after the sweeps, 0.83 beside, 0.82 with the late join, 0.77
  // with the totals kernels at wave priority 3 (profiles/r05z_cli_totals_beside.txt)
  const int tb_mode = (int)knob("MLP_TEST_TOT_BESIDE", 2);
  const bool tot_beside = (models & kLocal) && !lanefold && tb_mode != 0;
  if (tot_beside && side_used && tb_mode == 2) {
    side_lf = *side;
    side_lf.join_mode = 2;
    side = &side_lf;
  }
  auto budget_for = [&](size_t b) { return std::max<size_t>(b > clist_bytes ? b - clist_bytes : 0, 32u << 20); };
  size_t batch_target = batch_target_for(c, p0, p1, pair_bytes, budget_for(c->scratch_budget));
  int64_t all_cells = 0, done_cells = 0;
  for (int64_t k = p0; k < p1; k++) all_cells += pair_cost_cells(c, k);
  const int64_t base_total = c->store_total;
  // a launched batch whose host part and compaction are still to come
  struct Pending {
    bool live = false;
    int64_t p = 0, q = 0, np = 0, bcells = 0;
    std::vector<int64_t> order;
    const PairRec* rec = nullptr;  // the records' host copy (pinned, c->h_rec[parity])
    int par = 0;
    char* base = nullptr;
    size_t o_entb = 0, o_rpb = 0;
    PairMeta pm;
    Scratch sc;
    PairRec* d_rec = nullptr;
  } B;
  // Deferred finish: batch b + 1's sweeps are launched before the host
  // finishes batch b (entry offsets, store growth, its compaction), so that
  // host work overlaps the sweeps instead of idling the device between
  // batches; batch b + 1's merge follows b's compaction in stream order.  What
  // b's compaction reads (plan, records, entry bases, ELL rows) lives in a
  // front region the sweeps never write: plan and records twice (batch
  // parity), ELL rows once (written only by the merges).
  // MLP_TEST_DEFER_FINISH=0 finishes each batch before the next is launched.
  const bool defer = knob("MLP_TEST_DEFER_FINISH", 1) != 0;
  struct Front {
    bool set = false;
    int64_t np = 0, nch = 0, ell = 0;  // capacities
  } front;
  // the front a batch of plan P is carved with: the current one, or (first
  // batch, or one that needs more) the widened one, 5% slack
  auto front_for = [&](const ChainPlan& P) {
    Front f = front;
    if (!f.set || P.np > f.np || P.nch > f.nch || P.ell_rows > f.ell) {
      f.set = true;
      f.np = std::max<int64_t>(f.np, P.np + P.np / 20 + 64);
      f.nch = std::max<int64_t>(f.nch, P.nch + P.nch / 20 + 64);
      f.ell = std::max<int64_t>(f.ell, P.ell_rows + P.ell_rows / 20 + 1024);
    }
    return f;
  };
  int par = 0;
  // host part + compaction of the launched batch
  auto finish = [&]() -> int {
    if (!B.live) return MLP_OK;
    B.live = false;
    HIPCHK(c, hipEventSynchronize(c->ev_done[B.par]));
    const int64_t np = B.np;
    for (int64_t s = 0; s < np; s++) {
      if (B.rec[s].flags & 1) {
        c->err = "partition function overflow (pair " + std::to_string(B.order[s]) + ")";
        return MLP_ERR_OVERFLOW;
      }
      if (B.rec[s].flags & 2) {
        c->err = "posterior row exceeds " + std::to_string(kEll) + " entries >= 0.01 (pair " +
                 std::to_string(B.order[s]) + "); unsupported input";
        return MLP_ERR_STATE;
      }
    }
    // ---- canonical entry offsets (pair order) and compaction
    // entry bases through pinned staging of the batch's parity: its last
    // copy (two batches back) ran before the merge finish() waited for last
    std::vector<int64_t> slot_of(np);
    if (c->h_ent_n[B.par] < (size_t)np * 2) {
      if (c->h_ent[B.par]) hipHostFree(c->h_ent[B.par]);
      c->h_ent[B.par] = nullptr;
      c->h_ent_n[B.par] = 0;
      const size_t n = (size_t)np * 2 + (size_t)np / 4 + 128;
      HIPCHK(c, hipHostMalloc((void**)&c->h_ent[B.par], n * 8, hipHostMallocDefault));
      c->h_ent_n[B.par] = n;
    }
    int64_t* h_entb = c->h_ent[B.par];
    int64_t* h_rpb = h_entb + np;
    for (int64_t s = 0; s < np; s++) slot_of[B.order[s] - B.p] = s;
    int64_t run = c->store_total;
    for (int64_t k = 0; k < np; k++) {
      const int64_t s = slot_of[k];
      const int64_t pp = B.p + k;
      c->ent_off[pp] = run;
      c->nnz[pp] = B.rec[s].nnz;
      c->dist[pp] = B.rec[s].dist;
      c->mea[pp] = B.rec[s].mea;
      h_entb[s] = run;
      h_rpb[s] = c->rp_off[pp];
      run += B.rec[s].nnz;
    }
    c->ent_off[B.q] = run;
    int rc;
    done_cells += B.bcells;
    // the set's final size, extrapolated from the pairs done so far (+10%)
    const int64_t want = run + (int64_t)((double)(run - base_total) / (double)done_cells *
                                         (double)(all_cells - done_cells) * 1.1);
    if ((rc = grow_store(c, run, c->store_total, want, false))) return rc;
    HIPCHK(c, hipMemcpyAsync(B.base + B.o_entb, h_entb, np * 8, hipMemcpyHostToDevice, st));
    HIPCHK(c, hipMemcpyAsync(B.base + B.o_rpb, h_rpb, np * 8, hipMemcpyHostToDevice, st));
    {
      Timer t(c, KCOMPACT, B.bcells, st);
      HIPCHK(c, launch_compact(seqs, B.pm, B.d_rec, B.sc, (const int64_t*)(B.base + B.o_entb), c->d_rowptr,
                               (const int64_t*)(B.base + B.o_rpb), c->d_cols, c->d_vals, np, st));
    }
    c->store_total = run; ++c->store_ver;
    c->store_p1 = B.q;
    return MLP_OK;
  };
  int64_t p = p0;
  ChainPlan P;
  // a batch's scratch layout (256-byte aligned sub-buffers) under front `fr`
  // (its region first, this batch's parity); returns the bytes
  struct BatchOffs {
    size_t f5, fl, bl, pg, zm, cmf, cmb, tn, cl, crb, rep, lfc, b5, bz, bm, bc, ec, ev, en, entb, rpb, rec;
    PlanDev pd;
  };
  auto carve = [&](const ChainPlan& P, const Front& fr, BatchOffs& o) -> size_t {
    Carver cv;
    const int64_t np = P.np;
    const bool h5 = models & kHmm5, lo = models & kLocal, pf = models & kPF;
    if (defer) {
      ChainPlan cap;
      cap.np = fr.np;
      cap.nch = fr.nch;
      const PlanDev pd0 = carve_plan(cv, cap), pd1 = carve_plan(cv, cap);
      const size_t r0 = cv.take(fr.np * sizeof(PairRec)), r1 = cv.take(fr.np * sizeof(PairRec));
      o.pd = par ? pd1 : pd0;
      o.rec = par ? r1 : r0;
      o.entb = cv.take(fr.np * 8);
      o.rpb = cv.take(fr.np * 8);
      o.ec = cv.take(fr.ell * kEll * 2);
      o.ev = cv.take(fr.ell * kEll * 4);
      o.en = cv.take(fr.ell * 4);
    }
    o.f5 = cv.take(h5 ? P.cells * 4 : 0);
    o.fl = cv.take(lo ? P.cells * 4 : 0);
    o.bl = cv.take(lo ? P.cells * 4 + (lanefold ? kLaneFoldPad : 0) : 0);
    o.pg = cv.take(pf && !pg_in_zm ? P.cells * 4 : 0);
    o.zm = cv.take(pf ? P.cells * 8 : 0);
    o.cmf = cv.take(lo ? P.rm_total * 4 : 0);
    o.cmb = cv.take(lo ? P.rm_total * 4 : 0);
    o.tn = cv.take(lo ? 256 : 0);
    o.cl = cv.take(clist_bytes);
    o.crb = cv.take(lanefold || foldbound ? P.ell_rows * 4 : 0);
    o.rep = cv.take(lanefold ? (np + 1) * 4 : 0);
    o.lfc = cv.take(lanefold && defer ? P.ell_rows * 4 : 0);  // (else the lane fold counts in ell_cnt)
    o.b5 = cv.take(P.bnd * 32);   // the HMMs' boundary records (mlp_chain.h, bnd_put_hmm)
    o.bz = cv.take(P.bnd * 32);   // the partition function's
    o.bm = cv.take(P.bnd * 4);
    o.bc = cv.take(P.bnd * 4);
    if (!defer) {
      o.ec = cv.take(P.ell_rows * kEll * 2);
      o.ev = cv.take(P.ell_rows * kEll * 4);
      o.en = cv.take(P.ell_rows * 4);
      o.entb = cv.take(np * 8);
      o.rpb = cv.take(np * 8);
      o.rec = cv.take(np * sizeof(PairRec));
      o.pd = carve_plan(cv, P);
    }
    return cv.off;
  };
  bool calibrated = false;
  while (p < p1) {
    int64_t q;
    int rc;
    if ((rc = next_batch(c, p, p1, batch_target, pair_bytes, &q))) return rc;
    plan_chains(c, p, q, P);          // host planning overlaps the previous batch's kernels
    if (!calibrated) {
      // pair_bytes bounds each pair as if alone in a chain of a wider member;
      // the planned chains need less (C3: ~14%).  Once, from the first batch:
      // re-plan the batches to the budget at the measured ratio, then take
      // the first batch again (each batch is checked against the budget below)
      calibrated = true;
      BatchOffs o;
      size_t bound = 0;
      for (int64_t k = p; k < q; k++) bound += pair_bytes(k);
      const size_t got = carve(P, front_for(P), o);
      const double r = (double)(got > clist_bytes ? got - clist_bytes : 0) / (double)std::max<size_t>(bound, 1);
      if (q < p1 && r > 0.1 && r < 0.97) {
        batch_target = batch_target_for(
            c, p, p1, pair_bytes, std::max<size_t>((size_t)((double)budget_for(c->scratch_budget) / r * 0.99), 32u << 20));
        if ((rc = next_batch(c, p, p1, batch_target, pair_bytes, &q))) return rc;
        plan_chains(c, p, q, P);
      }
    }
    {  // a batch over the budget (the ratio varies with the pairs), carved as it will be, or
       // whose chunk maxima pass the sweeps' 32-bit buffer offsets: fewer pairs
      BatchOffs o;
      while (q - p > 1 && (carve(P, front_for(P), o) > c->scratch_budget || P.rm_total * 4 >= (1ll << 31))) {
        q = p + std::max<int64_t>(1, (q - p) * 97 / 100);
        plan_chains(c, p, q, P);
      }
    }
    if (defer) {
      // a batch that needs a wider front finishes the pending one first
      // (nothing then reads the old front) and widens it
      const Front f = front_for(P);
      if (!front.set || f.np != front.np || f.nch != front.nch || f.ell != front.ell) {
        if ((rc = finish())) return rc;
        front = f;
      }
    } else if ((rc = finish())) {  // the previous batch
      return rc;
    }
    const int64_t np = P.np, nch = P.nch;
    // ---- carve scratch
    BatchOffs o;
    const size_t need = carve(P, front, o);
    const PlanDev& pd = o.pd;
    // with more batches to come, 3% headroom (capped at the budget): they are
    // planned to the same bytes, and one that needs a little more would
    // otherwise reallocate the scratch
    const size_t want =
        q < p1 && c->scratch.bytes < need ? std::max(need, std::min(c->scratch_budget, need + need / 32)) : need;
    if (c->scratch.bytes < want && (rc = finish())) return rc;  // a reallocation: nothing may still read the old one
    if ((rc = ensure(c, c->scratch, want))) {
      if (rc != MLP_ERR_MEMORY || c->scratch_budget < (64u << 20)) return rc;
      c->scratch_budget /= 2;  // the device is shared: plan smaller batches and retry
      batch_target = batch_target_for(c, p, p1, pair_bytes, budget_for(c->scratch_budget));
      calibrated = false;
      front = Front();
      continue;
    }
    char* base = (char*)c->scratch.p;
    Scratch sc{};
    sc.f5 = (float*)(base + o.f5);
    sc.fl = (float*)(base + o.fl);
    sc.pg = pg_in_zm ? (float*)(base + o.zm) : (float*)(base + o.pg);
    sc.pg_stride = pg_in_zm ? 2 : 1;
    sc.zm = (double*)(base + o.zm);
    sc.bl = (float*)(base + o.bl);
    sc.cmf = (float*)(base + o.cmf);
    sc.cmb = (float*)(base + o.cmb);
    sc.clist = (float*)(base + o.cl);
    sc.clist_row = tot_row;
    sc.tot_next = (int32_t*)(base + o.tn);
    sc.crb = lanefold || foldbound ? (float*)(base + o.crb) : nullptr;
    sc.rep = (int32_t*)(base + o.rep);
    static const bool force_repair = knob_set("MLP_TEST_TOT_FORCE_REPAIR");
    sc.force_repair = force_repair ? 1 : 0;
    sc.bnd5 = (float*)(base + o.b5);
    sc.bndz = (double*)(base + o.bz);
    sc.bndm = (float*)(base + o.bm);
    sc.bndc = (int32_t*)(base + o.bc);
    sc.ell_col = (uint16_t*)(base + o.ec);
    sc.ell_val = (float*)(base + o.ev);
    sc.ell_cnt = (int32_t*)(base + o.en);
    sc.lf_cnt = lanefold && defer ? (int32_t*)(base + o.lfc) : sc.ell_cnt;
    PairRec* d_rec = (PairRec*)(base + o.rec);
    PairMeta pm;
    ChainMeta cm;
    {  // the plan through this parity's pinned staging (its last batch is finished)
      const size_t up_need = pd.o_cbo + P.nch * 8 - pd.o_pa;
      if (c->h_up_n[par] < up_need) {
        if (c->h_up[par]) hipHostFree(c->h_up[par]);
        c->h_up[par] = nullptr;
        c->h_up_n[par] = 0;
        const size_t n = up_need + up_need / 8 + 4096;
        HIPCHK(c, hipHostMalloc((void**)&c->h_up[par], n, hipHostMallocDefault));
        c->h_up_n[par] = n;
      }
    }
    if ((rc = upload_plan(c, base, pd, P, pm, cm, st, c->h_up[par]))) return rc;
    const int lds_seq = P.lds_seq;
    HIPCHK(c, hipMemsetAsync(d_rec, 0, np * sizeof(PairRec), st));
    int64_t bcells = 0;
    for (int64_t k = p; k < q; k++) bcells += pair_cost_cells(c, k);
    hipEvent_t fwd_ref = nullptr;
    {
      Timer t(c, KFWD, bcells, st);
      if (side_used) t.span(side->st, false, nullptr);
      fwd_ref = t.e0;
      HIPCHK(c, launch_forward(models, ms, c->d_tables, seqs, pm, cm, d_rec, sc, nch, lds_seq, st, side));
    }
    // the local totals group times once per batch: its kernels' device time,
    // the parts after the first (another stream, or after the backward sweep)
    // adding to the batch's one launch
    if (lanefold) {  // the forward chains, beside the partition function's sweeps
      Timer t(c, KTOT, bcells, st);
      HIPCHK(c, launch_local_fwd_lanefold(seqs, pm, cm, d_rec, sc, np, tot_waves, st));
    }
    if (tot_beside) {  // the forward chains on stream2, beside the backward sweeps
      HIPCHK(c, hipEventRecord(c->ev_fork, st));
      HIPCHK(c, hipStreamWaitEvent(c->stream2, c->ev_fork, 0));
      Timer t(c, KTOT, bcells, c->stream2);
      HIPCHK(c, launch_local_totals(ms, c->d_tables, seqs, pm, cm, d_rec, sc, np, tot_waves, c->stream2, kTotFwd));
      HIPCHK(c, hipEventRecord(c->ev_tot, c->stream2));
    }
    {
      Timer t(c, KBWD, bcells, st);
      if (side_used) t.span(side->st, true, fwd_ref);
      HIPCHK(c, launch_backward(models, ms, c->d_tables, seqs, pm, cm, d_rec, sc, nch, lds_seq, np, st, side));
    }
    if (models & kLocal) {
      Timer t(c, KTOT, bcells, st);
      if (lanefold) {
        t.cont = true;
        HIPCHK(c, launch_local_bwd_lanefold(ms, c->d_tables, seqs, pm, cm, d_rec, sc, np, tot_waves, st));
      } else if (tot_beside) {
        t.cont = true;
        HIPCHK(c, launch_local_totals(ms, c->d_tables, seqs, pm, cm, d_rec, sc, np, tot_waves, st, kTotBwd));
        HIPCHK(c, hipStreamWaitEvent(st, c->ev_tot, 0));
      } else {
        HIPCHK(c, launch_local_totals(ms, c->d_tables, seqs, pm, cm, d_rec, sc, np, tot_waves, st));
      }
    }
    // the previous batch: its host part while this batch's sweeps run, its
    // compaction before this batch's merge overwrites the ELL rows
    if (defer && (rc = finish())) return rc;
    if (side->join_mode != 0) HIPCHK(c, hipStreamWaitEvent(st, side->join, 0));  // deferred join
    {
      Timer t(c, KMERGE, bcells, st);
      HIPCHK(c, launch_merge(models, pid, ms, seqs, pm, cm, d_rec, sc, nch, lds_seq, st));
      HIPCHK(c, launch_pair_nnz(seqs, pm, d_rec, sc, np, st));
    }
    B.live = true;
    B.p = p;
    B.q = q;
    B.np = np;
    B.bcells = bcells;
    B.order = P.order;
    // the records come back into pinned memory: a pageable copy would hold
    // the host until the merge has run, and the next batch's planning and
    // launches with it (the buffer's last batch was finished before this one)
    if (c->h_rec_n[par] < (size_t)np) {
      if (c->h_rec[par]) hipHostFree(c->h_rec[par]);
      c->h_rec[par] = nullptr;
      c->h_rec_n[par] = 0;
      const size_t n = (size_t)np + (size_t)np / 8 + 64;
      HIPCHK(c, hipHostMalloc((void**)&c->h_rec[par], n * sizeof(PairRec), hipHostMallocDefault));
      c->h_rec_n[par] = n;
    }
    B.rec = c->h_rec[par];
    B.par = par;
    B.base = base;
    B.o_entb = o.entb;
    B.o_rpb = o.rpb;
    B.pm = pm;
    B.sc = sc;
    B.d_rec = d_rec;
    HIPCHK(c, hipMemcpyAsync(c->h_rec[par], d_rec, np * sizeof(PairRec), hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipEventRecord(c->ev_done[par], st));  // (its last waiter, finish(), has run)
    par ^= 1;
    p = q;
  }
  int rc;
  if ((rc = finish())) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream2));
  HIPCHK(c, hipMemcpyAsync(c->d_ent_off, c->ent_off.data(), sizeof(int64_t) * (c->P + 1),
                           hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MLP_OK;
}

}  // extern "C"
