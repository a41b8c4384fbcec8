// mlp_relax_rt.cpp -- probabilistic-consistency rounds (mlp_relax,
// mlp_relax_range, mlp_relax_qp_selective): transposes, packed images, the
// tile plan for k_relax_tile, the row-task fallback and the re-sparsifying
// filter (relax.hip).  Reference: CPNP/MSA.cpp:1172-1360 and QuickProbs'
// ConsistencyStage.cpp:35-300.
#include "mlp_runtime.h"

extern "C" {

// ------------------------------------------------------------------ relax
static int relax_rounds(mlp_ctx* c, int iters, const QpRelax& qp, const float* h_w, const float* h_sel);
static int relax_one(mlp_ctx* c, const QpRelax& qp, bool last);

int mlp_relax(mlp_ctx* c, int iters) {
  if (!c || iters < 0) return MLP_ERR_ARG;
  if (c->host) {
    if (c->n < 2) return MLP_ERR_STATE;
    if (c->store_p0 != 0 || c->store_p1 != c->P) {
      c->err = "relaxation needs every pair";
      return MLP_ERR_STATE;
    }
    for (int it = 0; it < iters; it++) mlph::relax(host_view(c), c->rp_off, c->hs, c->nnz.data());
    c->ent_off = c->hs.ent_off;
    c->store_total = c->hs.ent_off[c->P];
    ++c->store_ver;
    return MLP_OK;
  }
  return relax_rounds(c, iters, QpRelax{0, nullptr, 0.f, nullptr, 200.f}, nullptr, nullptr);
}

int mlp_relax_range(mlp_ctx* c, int64_t r0, int64_t r1) {
  if (!c || r0 < 0 || r1 < r0 || r1 > c->P) return MLP_ERR_ARG;
  if (c->n < 2) return MLP_ERR_STATE;
  if (c->store_p0 != 0 || c->store_p1 != c->P) {
    c->err = "relaxation needs every pair";
    return MLP_ERR_STATE;
  }
  if (c->host) {
    mlph::relax(host_view(c), c->rp_off, c->hs, c->nnz.data(), nullptr, r0, r1);
    c->ent_off = c->hs.ent_off;
    c->store_p0 = r0;
    c->store_p1 = r1;
    c->store_total = c->hs.ent_off[r1];
    ++c->store_ver;
    return MLP_OK;
  }
  if (c->comm && c->nranks > 1) {
    c->err = "mlp_relax_range with a communicator: mlp_relax shards the rounds itself";
    return MLP_ERR_STATE;
  }
  c->rel_r0 = r0;
  c->rel_r1 = r1;
  const int rc = relax_one(c, QpRelax{0, nullptr, 0.f, nullptr, 200.f}, true);
  c->rel_r0 = c->rel_r1 = -1;
  return rc;
}

// QuickProbs' consistency stage (ConsistencyStage::operator() / run,
// QP/Alignment/Multiple/ConsistencyStage.cpp:62-128) with its default
// configuration: 2 rounds up to 50 sequences, 1 above (iters < 0), self-weight
// 3, every round but the last re-sparsified at 0.01, the last at 1e-5.
int mlp_relax_qp(mlp_ctx* c, int iters, const float* seq_weights) {
  return mlp_relax_qp_selective(c, iters, seq_weights, nullptr, 200.f);
}

int mlp_relax_qp_selective(mlp_ctx* c, int iters, const float* seq_weights, const float* sel_dist,
                           float selectivity) {
  if (!c || !seq_weights || !(selectivity > 0)) return MLP_ERR_ARG;
  if (c->n < 2) return MLP_ERR_STATE;
  if (iters < 0) iters = c->n > 50 ? 1 : 2;
  if (c->host) {
    if (c->store_p0 != 0 || c->store_p1 != c->P) {
      c->err = "relaxation needs every pair";
      return MLP_ERR_STATE;
    }
    for (int it = 0; it < iters; it++) {
      const mlph::QpRelaxHost q{seq_weights, sel_dist, selectivity, 3.0f, it == iters - 1 ? 1e-5f : 0.01f};
      mlph::relax(host_view(c), c->rp_off, c->hs, c->nnz.data(), &q);
    }
    c->ent_off = c->hs.ent_off;
    c->store_total = c->hs.ent_off[c->P];
    ++c->store_ver;
    return MLP_OK;
  }
  int rc;
  if ((rc = ensure(c, c->r_weights, sizeof(float) * c->n))) return rc;
  HIPCHK(c, hipMemcpyAsync(c->r_weights.p, seq_weights, sizeof(float) * c->n, hipMemcpyHostToDevice, c->stream));
  const float* dsel = nullptr;
  if (sel_dist) {
    const size_t bytes = sizeof(float) * (size_t)c->n * c->n;
    if ((rc = ensure(c, c->r_seldist, bytes))) return rc;
    HIPCHK(c, hipMemcpyAsync(c->r_seldist.p, sel_dist, bytes, hipMemcpyHostToDevice, c->stream));
    dsel = (const float*)c->r_seldist.p;
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));  // the caller's buffers may go away
  return relax_rounds(c, iters, QpRelax{1, (const float*)c->r_weights.p, 3.0f, dsel, selectivity}, seq_weights,
                      sel_dist);
}

// Output-pair ranges of one round for S shards / ranks, balanced by the
// estimated work (mlp_relax_shard_plan).
static void relax_bounds(const mlp_ctx* c, int S, std::vector<int64_t>& bounds) {
  bounds.assign(S + 1, 0);
  mlp_relax_shard_plan(c->n, c->lens.data(), c->nnz.data(), S, bounds.data());
}

static int relax_one(mlp_ctx* c, const QpRelax& qp, bool last);

static int sharded_relax(mlp_ctx* c, int iters, const QpRelax& qp, const float* h_w, const float* h_sel, int S) {
  int rc;
  if ((rc = ensure_shards(c, S))) return rc;
  std::vector<QpRelax> q(S, qp);
  if (qp.on) {  // QuickProbs' weights and selectivity matrix on every shard
    if ((rc = run_shards(c, [&](mlp_ctx* ch, int s) -> int {
          int r;
          if ((r = ensure(ch, ch->r_weights, sizeof(float) * c->n))) return r;
          HIPCHK(ch, hipMemcpy(ch->r_weights.p, h_w, sizeof(float) * c->n, hipMemcpyHostToDevice));
          q[s].weights = (const float*)ch->r_weights.p;
          if (h_sel) {
            const size_t bytes = sizeof(float) * (size_t)c->n * c->n;
            if ((r = ensure(ch, ch->r_seldist, bytes))) return r;
            HIPCHK(ch, hipMemcpy(ch->r_seldist.p, h_sel, bytes, hipMemcpyHostToDevice));
            q[s].seldist = (const float*)ch->r_seldist.p;
          }
          return MLP_OK;
        })))
      return rc;
  }
  for (int it = 0; it < iters; it++) {
    std::vector<int64_t> bounds;
    relax_bounds(c, S, bounds);
    // the shards hold the parent's store from the last all-gather; a store
    // that came another way (an unsharded stage, mlp_csr_import) is sent out
    const bool send = c->shards_full_ver != c->store_ver;
    if ((rc = run_shards(c, [&](mlp_ctx* ch, int s) -> int {
          int r;
          if (send && (r = broadcast_store(c, ch))) return r;
          ch->rel_r0 = bounds[s];
          ch->rel_r1 = bounds[s + 1];
          r = relax_one(ch, q[s], it == iters - 1);
          ch->rel_r0 = ch->rel_r1 = -1;
          return r;
        })))
      return rc;
    if ((rc = allgather_shards(c))) return rc;
  }
  return MLP_OK;
}

static int relax_rounds(mlp_ctx* c, int iters, const QpRelax& qp, const float* h_w, const float* h_sel) {
  if (c->n < 2) return MLP_ERR_STATE;
  if (c->store_p0 != 0 || c->store_p1 != c->P) {
    c->err = "relaxation needs every pair (all-gather first)";
    return MLP_ERR_STATE;
  }
  const int S = c->comm ? 1 : shard_count(c);
  if (S > 1) return sharded_relax(c, iters, qp, h_w, h_sel, S);
  int rc;
  for (int it = 0; it < iters; it++) {
    if ((rc = relax_one(c, qp, it == iters - 1))) return rc;
    if (c->comm && c->nranks > 1) {
      if ((rc = mlp_allgather(c))) return rc;
    }
  }
  return MLP_OK;
}

// One consistency round over output pairs [r0, r1) (all pairs; a shard's
// range; or this rank's MAC-balanced range with a communicator).
static int relax_one(mlp_ctx* c, const QpRelax& qp, bool last) {
  if (c->store_p0 != 0 || c->store_p1 != c->P) {
    c->err = "relaxation needs every pair (all-gather first)";
    return MLP_ERR_STATE;
  }
  hipSetDevice(c->device);
  HIPCHK(c, hipStreamSynchronize(c->stream2));  // the batch scratch is idle: its temporaries come from there
  c->arena_on = true;
  c->arena_off = 0;
  struct ArenaOff {
    mlp_ctx* c;
    ~ArenaOff() {
      c->arena_on = false;
      c->tr_ver = ~0ull;  // the lent transposes are gone after the round
    }
  } arena_guard{c};
  int64_t r0 = 0, r1 = c->P;
  if (c->rel_r0 >= 0) {
    r0 = c->rel_r0;
    r1 = c->rel_r1;
  } else if (c->comm && c->nranks > 1) {
    std::vector<int64_t> bounds;
    relax_bounds(c, c->nranks, bounds);
    r0 = bounds[c->rank];
    r1 = bounds[c->rank + 1];
  }
  const int64_t nout = r1 - r0;
  int rc;
  // MLP_LOG_RELAX=1: wall time of the round's phases on stderr (each mark
  // drains the stream first, so the phases do not overlap while logging)
  static const bool rlog = knob_set("MLP_LOG_RELAX");
  auto rl_t = std::chrono::steady_clock::now();
  auto mark = [&](const char* what) {
    if (!rlog) return;
    hipStreamSynchronize(c->stream);
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "[relax] %-22s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(t - rl_t).count());
    rl_t = t;
  };
  {
    const int64_t total = c->store_total;
    if ((rc = ensure_tmp(c, c->r_trowptr, sizeof(int32_t) * c->trp_off[c->P]))) return rc;
    if ((rc = ensure_tmp(c, c->r_tcols, sizeof(uint16_t) * std::max<int64_t>(total, 1)))) return rc;
    if ((rc = ensure_tmp(c, c->r_tvals, sizeof(float) * std::max<int64_t>(total, 1)))) return rc;
    if ((rc = ensure_tmp(c, c->r_raw, sizeof(float) * std::max<int64_t>(total, 1)))) return rc;
    if ((rc = ensure_tmp(c, c->r_pairs, sizeof(int64_t) * std::max<int64_t>(c->P, 1)))) return rc;
    if ((rc = ensure_tmp(c, c->r_nnz, sizeof(int64_t) * std::max<int64_t>(c->P, 1)))) return rc;
    if ((rc = ensure_tmp(c, c->r_newoff, sizeof(int64_t) * (c->P + 1)))) return rc;
    if ((rc = ensure(c, c->r_newrp, sizeof(int32_t) * c->rp_off[c->P]))) return rc;
    // all pairs are transposed (every rank reads every block)
    std::vector<int64_t> allp(c->P);
    std::iota(allp.begin(), allp.end(), 0);
    HIPCHK(c, hipMemcpyAsync(c->r_pairs.p, allp.data(), sizeof(int64_t) * c->P, hipMemcpyHostToDevice, c->stream));
    mark("buffers");
    TransposeArgs ta;
    ta.n = c->n;
    ta.lens = c->d_len;
    ta.rp_off = c->d_rp_off;
    ta.rowptr = c->d_rowptr;
    ta.ent_off = c->d_ent_off;
    ta.cols = c->d_cols;
    ta.vals = c->d_vals;
    ta.trp_off = c->d_trp_off;
    ta.trowptr = (int32_t*)c->r_trowptr.p;
    ta.tcols = (uint16_t*)c->r_tcols.p;
    ta.tvals = (float*)c->r_tvals.p;
    ta.pairs = (const int64_t*)c->r_pairs.p;
    ta.npairs = c->P;
    ta.max_len = c->max_len;
    {
      Timer t(c, KTRANS, total);
      HIPCHK(c, launch_transpose(ta, c->stream));
    }
    mark("transpose");
    // Tiled path (k_relax_tile) for every output pair whose blocks fit the
    // LDS tile; the row-task kernel for the rest (MLP_TEST_RELAX_PATH=tasks: all).
    int64_t LDS_MAX = 160 * 1024 / kRelaxGroupsPerCU;
    if (knob_set("MLP_TEST_RELAX_LDS_KB"))
      LDS_MAX = std::max(32, std::min(160, (int)knob("MLP_TEST_RELAX_LDS_KB", 0))) * 1024;
    const char* mode = knob_str("MLP_TEST_RELAX_PATH");
    const int tmax = std::max(1, std::min(kTileMax, (int)knob("MLP_TEST_RELAX_TILE", kTileMax)));
    bool tasks_only = (mode && !strcmp(mode, "tasks")) || c->max_len > 8000 || c->P >= (1LL << 31);
    std::vector<int32_t> nwords(2 * c->P, 0);
    if ((rc = ensure_tmp(c, c->r_nwords, sizeof(int32_t) * std::max<int64_t>(2 * c->P, 1)))) return rc;
    PackArgs pk;
    pk.n = c->n;
    pk.lens = c->d_len;
    pk.rp_off = c->d_rp_off;
    pk.rowptr = c->d_rowptr;
    pk.ent_off = c->d_ent_off;
    pk.cols = c->d_cols;
    pk.vals = c->d_vals;
    pk.trp_off = c->d_trp_off;
    pk.trowptr = (const int32_t*)c->r_trowptr.p;
    pk.tcols = (const uint16_t*)c->r_tcols.p;
    pk.tvals = (const float*)c->r_tvals.p;
    pk.img_off = nullptr;
    pk.nwords = (int32_t*)c->r_nwords.p;
    pk.img = nullptr;
    pk.nimg = 2 * c->P;
    pk.count = 1;
    if (!tasks_only) {
      {
        Timer t(c, KTRANS, total);
        HIPCHK(c, launch_pack(pk, c->stream));
      }
      HIPCHK(c, hipMemcpyAsync(nwords.data(), c->r_nwords.p, sizeof(int32_t) * 2 * c->P, hipMemcpyDeviceToHost,
                               c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    mark("pack count");
    // record offsets; per sequence the largest image with its residues as
    // rows (the A_t = P(x, .) and C = P(y, .) roles)
    std::vector<int64_t> img_off(2 * c->P + 1, 0), maxI(c->n, 0);
    std::vector<char> big(c->n, 0);
    for (int64_t p = 0; p < c->P && !tasks_only; p++) {
      const int64_t nz = c->ent_off[p + 1] - c->ent_off[p];
      const int a = c->pa[p], b = c->pb[p];
      for (int o = 0; o < 2; o++) {
        const int64_t q = 2 * p + o;
        const int xr = o ? b : a;
        const int64_t bytes = img_layout(c->lens[xr], nz, nwords[q]).end;
        img_off[q + 1] = img_off[q] + bytes;
        if (nz >= 65536 || nwords[q] >= 65536) big[a] = big[b] = 1;
        maxI[xr] = std::max(maxI[xr], bytes);
      }
    }
    if (img_off[2 * c->P] >= (1LL << 36)) tasks_only = true;  // z schedule holds offsets / 16 in 32 bits
    // Tiles: per y, consecutive x's (ascending) while the staged images fit
    // and the cell slots allow.  A tile's LDS need is the largest, over z,
    // of its images P(x_t, z) + P(y, z) (exact per z up to n = 2048; the
    // per-sequence maxima beyond).  Two classes: tiles within half the LDS
    // run two workgroups per CU (8 waves per SIMD, the kernel's latency
    // hiding); the rest one.
    const int64_t zs = (int64_t)tile_relax_lds(0);
    const int64_t budget = std::min<int64_t>(LDS_MAX - zs, tile_relax_max_cap()) & ~(int64_t)15;
    int64_t small_budget = std::min<int64_t>(budget, (80 * 1024 - zs) & ~(int64_t)15);
    if (LDS_MAX < 160 * 1024) small_budget = 0;
    if (knob_set("MLP_TEST_RELAX_SMALL_KB"))  // a small staging area for the small class
      small_budget =
          std::min(budget, std::max<int64_t>(64, (int64_t)knob("MLP_TEST_RELAX_SMALL_KB", 0) * 1024 - zs)) & ~(int64_t)15;
    const int n = c->n;
    const bool exact = !tasks_only && n <= 2048;
    const int64_t kSmallCells = 8 * (int64_t)kRelaxThreads;  // 8 slots: the 64-VGPR budget of 8 waves per SIMD
    // z's per tile whose images may exceed the staging area (staged in passes)
    const int max_over = (int)knob("MLP_TEST_RELAX_SPLIT_Z", n / 16);
    // z's on which a small-class output's image may not fit beside C even
    // alone (the kernel reads that image in place from HBM on those z's);
    // 0: such outputs go to the one-workgroup class.  No limit by default: at
    // C3 round 1 every output has such z's, and the small class with images
    // read in place runs 1.32 s against 1.60 s for the one-workgroup class
    // (limits of 8 / 32 z's: 1.60 / 1.55 s)
    const int max_glob = (int)knob("MLP_TEST_RELAX_GLOBAL_Z", n);
    std::vector<int32_t> isz;  // image bytes of P(s, z), s's residues as rows: isz[s * n + z]
    if (exact) {
      isz.assign((size_t)n * n, 0);
      for (int64_t p = 0; p < c->P; p++) {
        const int a = c->pa[p], b = c->pb[p];
        isz[(size_t)a * n + b] = (int32_t)(img_off[2 * p + 1] - img_off[2 * p]);
        isz[(size_t)b * n + a] = (int32_t)(img_off[2 * p + 2] - img_off[2 * p + 1]);
      }
    }
    struct TileRec { int x0, y, cls; int64_t first, need, cells; };
    struct YPlan {
      std::vector<int32_t> ints;
      std::vector<TileRec> recs;
      std::vector<int64_t> tp;
      std::vector<int32_t> tr;
    };
    std::vector<YPlan> yplans(n);
    std::atomic<int64_t> n_hbm_outputs{0};  // small-class outputs whose image is read from HBM on some z
    auto plan_y = [&](int yy) {
      YPlan& Y = yplans[yy];
      struct Cur {
        int cnt = 0;
        int32_t p[kTileMax], x[kTileMax];
        int64_t bound = 0, cells = 0, peak = 0;
        std::vector<int64_t> sum;
      } cur[2];
      const int64_t lim[2] = {small_budget, budget};
      const int32_t* iy = exact ? &isz[(size_t)yy * n] : nullptr;
      auto flush = [&](int k) {
        Cur& t = cur[k];
        if (!t.cnt) return;
        Y.recs.push_back({t.x[0], yy, k, (int64_t)Y.ints.size(), exact ? t.peak : t.bound + maxI[yy], t.cells});
        for (int u = 0; u < kTileMax; u++) Y.ints.push_back(u < t.cnt ? t.p[u] : -1);
        for (int u = 0; u < kTileMax; u++) Y.ints.push_back(u < t.cnt ? t.x[u] : 0);
        Y.ints.push_back(yy);
        t.cnt = 0;
        t.bound = t.cells = t.peak = 0;
      };
      // LDS need of tile t with output x added
      // LDS need of tile t with output x added, and the z's where it exceeds `lim`
      auto need_with = [&](const Cur& t, int x, int64_t lim, int* over) -> int64_t {
        *over = 0;
        if (!exact) return t.bound + maxI[x] + maxI[yy];
        const int32_t* ix = &isz[(size_t)x * n];
        int64_t m = 0;
        int o = 0;
        for (int z = 0; z < n; z++) {
          const int64_t v = (t.cnt ? t.sum[z] : (int64_t)iy[z]) + ix[z];
          m = std::max(m, v);
          o += v > lim;
        }
        *over = o;
        return m;
      };
      for (int x = 0; x < yy; x++) {
        const int64_t p = pair_index_host(n, x, yy);
        if (p < r0 || p >= r1) continue;
        const int64_t nz = c->ent_off[p + 1] - c->ent_off[p];
        if (nz == 0) continue;  // empty mask: the filter writes an empty block
        int k = -1;
        int64_t alone = 0;
        int alone_over = 0;  // small class: z's where the output alone exceeds the staging area
        if (!tasks_only && !big[x] && !big[yy] && tile_relax_slots(nz)) {
          const Cur empty{};
          int unused;
          alone = need_with(empty, x, budget, &unused);
          k = alone <= small_budget && nz <= kSmallCells ? 0 : alone <= budget ? 1 : -1;
          if (k == 1 && exact && max_glob > 0 && small_budget > 0 && nz <= kSmallCells) {
            // the small class (two workgroups per CU) if C fits on every z and
            // the output's own image fits beside it on all but a few
            const int32_t* ix = &isz[(size_t)x * n];
            int ov = 0;
            bool cfits = true;
            for (int z = 0; z < n && cfits; z++) {
              cfits = iy[z] <= small_budget;
              ov += (int64_t)iy[z] + ix[z] > small_budget;
            }
            if (cfits && ov <= max_glob) {
              k = 0;
              alone_over = ov;
              if (ov) n_hbm_outputs.fetch_add(1, std::memory_order_relaxed);
            }
          }
        }
        if (k < 0) {
          for (int g = 1; g <= c->lens[x]; g += 64) {
            Y.tp.push_back(p);
            Y.tr.push_back(g);
          }
          continue;
        }
        Cur& t = cur[k];
        // a tile may exceed its staging area on a few z's (outliers: the
        // kernel stages those z's outputs in passes), never on one output
        int over = alone_over;
        int64_t nd = t.cnt ? need_with(t, x, lim[k], &over) : alone;
        if (t.cnt && (t.cnt == tmax || (exact ? over > max_over : nd > lim[k]) ||
                      !tile_relax_slots(t.cells + nz) || (k == 0 && t.cells + nz > kSmallCells))) {
          flush(k);
          nd = alone;
          over = alone_over;
        }
        if (exact) {
          const int32_t* ix = &isz[(size_t)x * n];
          if (!t.cnt) t.sum.assign(iy, iy + n);
          for (int z = 0; z < n; z++) t.sum[z] += ix[z];
        }
        t.p[t.cnt] = (int32_t)p;
        t.x[t.cnt] = x;
        t.cnt++;
        t.bound += maxI[x];
        t.cells += nz;
        t.peak = over ? lim[k] : nd;   // split z's: the staging area is the class bound
      }
      flush(0);
      flush(1);
    };
    {
      const int nth = tasks_only ? 1 : mlph::threads_for((int64_t)n * n / 4096 + 1);
      std::vector<std::thread> th;
      std::atomic<int> next_y{1};
      for (int w = 0; w < nth; w++)
        th.emplace_back([&]() {
          for (int yy; (yy = next_y.fetch_add(1)) < n;) plan_y(yy);
        });
      for (auto& t : th) t.join();
    }
    mark("plan");
    // per class: tiles ordered by (first x, y) for the XCD-aware grid order
    std::vector<int32_t> tiles;
    std::vector<int64_t> tp;
    std::vector<int32_t> tr;
    int64_t cls_tiles[2] = {0, 0}, cls_cap[2] = {0, 0}, cls_cells[2] = {0, 0};
    // the small class in one launch per slot count (cells per thread): fewer
    // registers and idle slots than one launch sized for its largest tile
    std::vector<std::pair<int, int64_t>> small_groups;  // (slots, tiles), in launch order
    for (int k = 0; k < 2; k++) {
      std::vector<std::pair<int, const TileRec*>> order;  // (y, record)
      for (int yy = 1; yy < n; yy++)
        for (const TileRec& r : yplans[yy].recs)
          if (r.cls == k) order.push_back({yy, &r});
      std::stable_sort(order.begin(), order.end(), [&](const auto& u, const auto& v) {
        if (k == 0) {
          const int su = tile_relax_slots(u.second->cells), sv = tile_relax_slots(v.second->cells);
          if (su != sv) return su < sv;
        }
        return u.second->x0 != v.second->x0 ? u.second->x0 < v.second->x0 : u.first < v.first;
      });
      if (k == 0)
        for (const auto& o : order) {
          const int sl = tile_relax_slots(o.second->cells);
          if (small_groups.empty() || small_groups.back().first != sl) small_groups.push_back({sl, 0});
          small_groups.back().second++;
        }
      for (const auto& o : order) {
        const std::vector<int32_t>& src = yplans[o.first].ints;
        tiles.insert(tiles.end(), src.begin() + o.second->first, src.begin() + o.second->first + kTileInts);
        cls_cap[k] = std::max(cls_cap[k], o.second->need);
        cls_cells[k] = std::max(cls_cells[k], o.second->cells);
      }
      cls_tiles[k] = (int64_t)order.size();
    }
    for (int yy = 1; yy < n; yy++) {
      tp.insert(tp.end(), yplans[yy].tp.begin(), yplans[yy].tp.end());
      tr.insert(tr.end(), yplans[yy].tr.begin(), yplans[yy].tr.end());
    }
    const int64_t ntiles = cls_tiles[0] + cls_tiles[1];
    if (ntiles) {
      if ((rc = ensure_tmp(c, c->r_img, std::max<int64_t>(img_off[2 * c->P], 16)))) return rc;
      if ((rc = ensure_tmp(c, c->r_imgoff, sizeof(int64_t) * (2 * c->P + 1)))) return rc;
      if ((rc = ensure_tmp(c, c->r_tiles, sizeof(int32_t) * tiles.size()))) return rc;
      HIPCHK(c, hipMemcpyAsync(c->r_imgoff.p, img_off.data(), sizeof(int64_t) * (2 * c->P + 1),
                               hipMemcpyHostToDevice, c->stream));
      HIPCHK(c, hipMemcpyAsync(c->r_tiles.p, tiles.data(), sizeof(int32_t) * tiles.size(), hipMemcpyHostToDevice,
                               c->stream));
      pk.img_off = (const int64_t*)c->r_imgoff.p;
      pk.img = (uint8_t*)c->r_img.p;
      pk.count = 0;
      Timer t(c, KTRANS, total);
      HIPCHK(c, launch_pack(pk, c->stream));
    }
    mark("order, images");
    const int64_t nt = (int64_t)tp.size();
    if (knob_set("MLP_LOG_PLAN")) {
      int64_t mx = 0;
      for (int i = 0; i < c->n; i++) mx = std::max(mx, maxI[i]);
      fprintf(stderr,
              "relax plan: tiles %lld (cap %lld, cells %lld) + %lld (cap %lld, cells %lld) row tasks %lld budget %lld/%lld "
              "max image %lld hbm-image outputs %lld\n",
              (long long)cls_tiles[0], (long long)cls_cap[0], (long long)cls_cells[0], (long long)cls_tiles[1],
              (long long)cls_cap[1], (long long)cls_cells[1], (long long)nt, (long long)small_budget, (long long)budget,
              (long long)mx, (long long)n_hbm_outputs.load());
    }
    if (mode && !strcmp(mode, "pairs") && nt) {  // test hook: the pair-resident path must cover all
      c->err = "MLP_TEST_RELAX_PATH=pairs: " + std::to_string(nt) + " row tasks fell back";
      return MLP_ERR_STATE;
    }
    if ((rc = ensure_tmp(c, c->r_tasks_p, sizeof(int64_t) * std::max<int64_t>(nt, 1)))) return rc;
    if ((rc = ensure_tmp(c, c->r_tasks_r, sizeof(int32_t) * std::max<int64_t>(nt, 1)))) return rc;
    if (nt) {
      HIPCHK(c, hipMemcpyAsync(c->r_tasks_p.p, tp.data(), sizeof(int64_t) * nt, hipMemcpyHostToDevice, c->stream));
      HIPCHK(c, hipMemcpyAsync(c->r_tasks_r.p, tr.data(), sizeof(int32_t) * nt, hipMemcpyHostToDevice, c->stream));
    }
    RelaxArgs ra;
    ra.n = c->n;
    ra.lens = c->d_len;
    ra.rp_off = c->d_rp_off;
    ra.rowptr = c->d_rowptr;
    ra.ent_off = c->d_ent_off;
    ra.cols = c->d_cols;
    ra.vals = c->d_vals;
    ra.trp_off = c->d_trp_off;
    ra.trowptr = (const int32_t*)c->r_trowptr.p;
    ra.tcols = (const uint16_t*)c->r_tcols.p;
    ra.tvals = (const float*)c->r_tvals.p;
    ra.task_pair = (const int64_t*)c->r_tasks_p.p;
    ra.task_row0 = (const int32_t*)c->r_tasks_r.p;
    ra.ntasks = nt;
    ra.out = (float*)c->r_raw.p;
    ra.qp = qp;
    TileRelaxArgs pr;
    pr.n = c->n;
    pr.lens = c->d_len;
    pr.rp_off = c->d_rp_off;
    pr.rowptr = c->d_rowptr;
    pr.ent_off = c->d_ent_off;
    pr.cols = c->d_cols;
    pr.vals = c->d_vals;
    pr.img_off = (const int64_t*)c->r_imgoff.p;
    pr.nwords = (const int32_t*)c->r_nwords.p;
    pr.img = (const uint8_t*)c->r_img.p;
    pr.img_chunks = img_off[2 * c->P] / 16;
    pr.out = (float*)c->r_raw.p;
    pr.qp = qp;
    TileRelaxArgs pc[2] = {pr, pr};
    for (int k = 0; k < 2; k++) {
      pc[k].tiles = (const int32_t*)c->r_tiles.p + (k ? cls_tiles[0] * kTileInts : 0);
      pc[k].ntiles = cls_tiles[k];
      pc[k].cap = (int)mlp_align16(cls_cap[k]);
    }
    {
      Timer t(c, KRELAX, c->ent_off[r1] - c->ent_off[r0]);
      // the one-workgroup-per-CU class on the side stream, concurrently
      const bool fork = cls_tiles[0] && cls_tiles[1];
      if (fork) {
        HIPCHK(c, hipEventRecord(c->side.fork, c->stream));
        HIPCHK(c, hipStreamWaitEvent(c->side.st, c->side.fork, 0));
      }
      if (cls_tiles[1])
        HIPCHK(c, launch_relax_tiles(pc[1], tile_relax_slots(cls_cells[1]), true, fork ? c->side.st : c->stream));
      int64_t first = 0;
      for (const auto& g : small_groups) {
        TileRelaxArgs a = pc[0];
        a.tiles += first * kTileInts;
        a.ntiles = g.second;
        HIPCHK(c, launch_relax_tiles(a, g.first, false, c->stream));
        first += g.second;
      }
      HIPCHK(c, launch_relax_tasks(ra, c->stream));
      if (fork) {
        HIPCHK(c, hipEventRecord(c->side.join, c->side.st));
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->side.join, 0));
      }
    }
    mark("relax kernels");
    // filter: count, host scan, write
    std::vector<int64_t> outp(nout);
    std::iota(outp.begin(), outp.end(), r0);
    HIPCHK(c, hipMemcpyAsync(c->r_pairs.p, outp.data(), sizeof(int64_t) * nout, hipMemcpyHostToDevice, c->stream));
    FilterArgs fa;
    fa.n = c->n;
    fa.lens = c->d_len;
    fa.rp_off = c->d_rp_off;
    fa.rowptr = c->d_rowptr;
    fa.ent_off = c->d_ent_off;
    fa.cols = c->d_cols;
    fa.raw = (const float*)c->r_raw.p;
    fa.pair_nnz = (int64_t*)c->r_nnz.p;
    fa.new_ent_off = (const int64_t*)c->r_newoff.p;
    fa.new_rowptr = (int32_t*)c->r_newrp.p;
    fa.new_cols = nullptr;
    fa.new_vals = nullptr;
    fa.pairs = (const int64_t*)c->r_pairs.p;
    fa.npairs = nout;
    fa.write = 0;
    fa.cutoff = qp.on && last ? 1e-5f : 0.01f;
    fa.fixed16 = qp.on;
    {
      Timer t(c, KFILTER, 0);
      HIPCHK(c, launch_filter(fa, c->stream));
    }
    std::vector<int64_t> pn(nout);
    // k_filter writes pair_nnz at the global pair index
    HIPCHK(c, hipMemcpyAsync(pn.data(), (const int64_t*)c->r_nnz.p + r0, sizeof(int64_t) * nout, hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    // new canonical offsets of my pairs, starting at 0 (gathered below)
    std::vector<int64_t> noff(c->P + 1, 0);
    int64_t run = 0;
    for (int64_t k = 0; k < nout; k++) {
      noff[r0 + k] = run;
      run += pn[k];
    }
    if ((rc = ensure_tmp(c, c->r_newcols, sizeof(uint16_t) * std::max<int64_t>(run, 1)))) return rc;
    if ((rc = ensure_tmp(c, c->r_newvals, sizeof(float) * std::max<int64_t>(run, 1)))) return rc;
    HIPCHK(c, hipMemcpyAsync(c->r_newoff.p, noff.data(), sizeof(int64_t) * (c->P + 1), hipMemcpyHostToDevice, c->stream));
    mark("filter count, scan");
    fa.new_cols = (uint16_t*)c->r_newcols.p;
    fa.new_vals = (float*)c->r_newvals.p;
    fa.write = 1;
    {
      Timer t(c, KFILTER, 0);
      HIPCHK(c, launch_filter(fa, c->stream));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    // swap in the new store (my shard), keep row_ptr canonical
    std::swap(c->d_rowptr, *(int32_t**)&c->r_newrp.p);
    {
      // sizes of the swapped buffers: both are rp_off[P] ints
      size_t bsz = c->r_newrp.bytes;
      (void)bsz;
    }
    if ((rc = grow_store(c, run, 0))) return rc;
    HIPCHK(c, hipMemcpyAsync(c->d_cols, c->r_newcols.p, sizeof(uint16_t) * run, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_vals, c->r_newvals.p, sizeof(float) * run, hipMemcpyDeviceToDevice, c->stream));
    for (int64_t k = 0; k < nout; k++) c->nnz[r0 + k] = pn[k];
    for (int64_t p = r0; p <= r1; p++) c->ent_off[p] = noff[p];
    c->ent_off[r1] = run;
    // outside the range: empty blocks, as the host context lays them out
    // (0 before r0, the range's total after r1)
    for (int64_t p = 0; p < r0; p++) c->ent_off[p] = 0;
    for (int64_t p = r1 + 1; p <= c->P; p++) c->ent_off[p] = run;
    c->store_p0 = r0;
    c->store_p1 = r1;
    c->store_total = run; ++c->store_ver;
    HIPCHK(c, hipMemcpyAsync(c->d_ent_off, c->ent_off.data(), sizeof(int64_t) * (c->P + 1), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    mark("filter write, swap");
  }
  return MLP_OK;
}

}  // extern "C"
