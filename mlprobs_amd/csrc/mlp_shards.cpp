// mlp_shards.cpp -- the multi-GPU paths of libmlpgpu:
// in-process shards over a device mask (child contexts, peer-copy all-gather),
// the pair and relaxation shard plans, and the RCCL communicator with its
// all-gather of the sparse posteriors (one process per GPU).
#include "mlp_runtime.h"

// ------------------------------------------------------------ in-process shards
// One context can spread the posterior stage and the consistency rounds over
// several GPUs of one process ("a ctx drives all GPUs
// in its mask"): child contexts, one per device, each compute a contiguous
// pair range; the parent gathers their sparse sets over xGMI (peer copies)
// into its canonical store and, before every relaxation round, copies the
// whole store back to every child.  Virtual shards (more shards than
// devices, mlp_set_shards) exercise the same path on one GPU.
static const double kShardMinCells = 1e9;  // smaller families stay on one device

std::vector<int> mask_devices(uint64_t mask) {
  int cnt = 0;
  if (hipGetDeviceCount(&cnt) != hipSuccess) cnt = 0;
  std::vector<int> d;
  for (int k = 0; k < cnt && k < 64; k++)
    if (mask >> k & 1) d.push_back(k);
  return d;
}

int shard_count(mlp_ctx* c) {
  if (c->shards_req > 0) return c->shards_req;
  if (c->n < 2) return 1;
  const std::vector<int> devs = mask_devices(c->dev_mask);
  if (devs.size() < 2) return 1;
  double cells = 0;
  for (int64_t p = 0; p < c->P; p++) cells += pair_cost_cells(c, p);
  return cells >= kShardMinCells ? (int)devs.size() : 1;
}

// MLP_TEST_FORCE_PEER=1 (test hook): peer copies even between contexts on one
// device, so virtual shards exercise the xGMI branch
static bool force_peer() {
  return knob("MLP_TEST_FORCE_PEER", 0) > 0;
}

static hipError_t copy_on(hipStream_t st, mlp_ctx* dst, void* d, const mlp_ctx* src, const void* s, size_t bytes) {
  if (!bytes) return hipSuccess;
  if (dst->device == src->device && !force_peer()) return hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, st);
  return hipMemcpyPeerAsync(d, dst->device, s, src->device, bytes, st);
}

static hipError_t copy_from(mlp_ctx* dst, void* d, const mlp_ctx* src, const void* s, size_t bytes) {
  return copy_on(dst->stream, dst, d, src, s, bytes);
}

int ensure_shards(mlp_ctx* c, int S) {
  if ((int)c->shards.size() == S) return MLP_OK;
  for (mlp_ctx* ch : c->shards) mlp_ctx_destroy(ch);
  c->shards.clear();
  c->shards_full_ver = ~0ull;  // new shards hold no store yet
  std::vector<int> devs = mask_devices(c->dev_mask);
  if (devs.empty()) devs.push_back(c->device);
  std::vector<int> per(devs.size(), 0);
  for (int s = 0; s < S; s++) per[s % devs.size()]++;
  for (int s = 0; s < S; s++) {
    const size_t di = s % devs.size();
    mlp_ctx* ch = nullptr;
    int rc = mlp_ctx_create(devs[di], &ch);
    if (rc) {
      c->err = "shard context on device " + std::to_string(devs[di]) + " failed";
      return rc;
    }
    // shards sharing a device share its scratch budget (and the parent's
    // cap), less what each of them and the parent keep beside it: a gathered
    // copy of the whole store and the all-gather's staging buffers (~0.16 B
    // per pair-cell at C3 pid 0; 0.5 B planned)
    double cells = 0;
    for (int64_t p = 0; p < c->P; p++) cells += pair_cost_cells(c, p);
    const size_t keep = (size_t)(0.5 * cells) + (256ull << 20);
    size_t b = std::min(ch->scratch_budget, c->scratch_budget);
    const size_t copies = keep * (size_t)(per[di] + 1);
    b = b > 2 * copies ? b - copies : b / 2;
    ch->scratch_budget = b / per[di];
    ch->profile = c->profile;
    c->shards.push_back(ch);
    if ((rc = mlp_family_load(ch, c->n, (const char*)c->h_res.data(), c->offs.data()))) {
      c->err = "shard family load: " + ch->err;
      return rc;
    }
  }
  for (int d : devs)
    if (d != c->device) {  // xGMI peer access both ways (errors: already enabled / no peer path)
      hipSetDevice(c->device);
      hipDeviceEnablePeerAccess(d, 0);
      hipSetDevice(d);
      hipDeviceEnablePeerAccess(c->device, 0);
    }
  hipGetLastError();
  hipSetDevice(c->device);
  return MLP_OK;
}

// The parent's whole store onto one shard (before a relaxation round).
int broadcast_store(mlp_ctx* c, mlp_ctx* ch) {
  int rc;
  if ((rc = grow_store(ch, c->store_total, 0))) return rc;
  HIPCHK(ch, copy_from(ch, ch->d_rowptr, c, c->d_rowptr, sizeof(int32_t) * c->rp_off[c->P]));
  HIPCHK(ch, copy_from(ch, ch->d_cols, c, c->d_cols, sizeof(uint16_t) * c->store_total));
  HIPCHK(ch, copy_from(ch, ch->d_vals, c, c->d_vals, sizeof(float) * c->store_total));
  ch->ent_off = c->ent_off;
  ch->nnz = c->nnz;
  ch->dist = c->dist;
  ch->mea = c->mea;
  HIPCHK(ch, hipMemcpyAsync(ch->d_ent_off, ch->ent_off.data(), sizeof(int64_t) * (c->P + 1), hipMemcpyHostToDevice,
                            ch->stream));
  HIPCHK(ch, hipStreamSynchronize(ch->stream));
  ch->store_p0 = 0;
  ch->store_p1 = c->P;
  ch->store_total = c->store_total;
  ++ch->store_ver;
  return MLP_OK;
}

// All-gather of the shards' blocks: after the
// posteriors or a relaxation round every shard holds the entries of its own
// contiguous pair range; each shard then pulls every other shard's block
// into place concurrently, one copy stream per source (xGMI peer copies
// between GPUs: all of a device's links at once, instead of the parent's
// serial gather followed by a whole-store broadcast), and the parent takes
// the full store from the shard on its own device.  Per-pair scalars and
// entry offsets are assembled on the host.
int allgather_shards(mlp_ctx* c) {
  const int S = (int)c->shards.size();
  std::vector<int64_t> ebase(S + 1, 0);
  for (int s = 0; s < S; s++) {
    const mlp_ctx* ch = c->shards[s];
    if (ch->store_p0 != (s ? c->shards[s - 1]->store_p1 : 0)) {
      c->err = "shard ranges do not tile the pair range";
      return MLP_ERR_STATE;
    }
    ebase[s + 1] = ebase[s] + ch->store_total;
  }
  if (c->shards[S - 1]->store_p1 != c->P) {
    c->err = "shard ranges do not tile the pair range";
    return MLP_ERR_STATE;
  }
  const int64_t total = ebase[S];
  const auto t0 = std::chrono::steady_clock::now();
  // global offsets and scalars (host)
  for (int s = 0; s < S; s++) {
    const mlp_ctx* ch = c->shards[s];
    for (int64_t p = ch->store_p0; p < ch->store_p1; p++) {
      c->dist[p] = ch->dist[p];
      c->mea[p] = ch->mea[p];
      c->nnz[p] = ch->nnz[p];
      c->ent_off[p] = ebase[s] + ch->ent_off[p] - ch->ent_off[ch->store_p0];
    }
  }
  c->ent_off[c->P] = total;
  struct Src { const mlp_ctx* ch; const uint16_t* cols; const float* vals; const int32_t* rp; int64_t p0, p1, n; };
  std::vector<Src> src(S);
  for (int s = 0; s < S; s++) {
    const mlp_ctx* ch = c->shards[s];
    src[s] = {ch, ch->d_cols, ch->d_vals, ch->d_rowptr, ch->store_p0, ch->store_p1, ch->store_total};
  }
  // phase 1: every destination pulls every block (sources stay untouched)
  int rc = run_shards(c, [&](mlp_ctx* ch, int s) -> int {
    int r;
    if ((r = ensure(ch, ch->ag_cols, sizeof(uint16_t) * std::max<int64_t>(total, 1)))) return r;
    if ((r = ensure(ch, ch->ag_vals, sizeof(float) * std::max<int64_t>(total, 1)))) return r;
    while ((int)ch->cst.size() < S) {
      hipStream_t st;
      HIPCHK(ch, hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
      ch->cst.push_back(st);
    }
    for (int q = 0; q < S; q++) {
      const Src& b = src[q];
      hipStream_t st = ch->cst[q];
      HIPCHK(ch, copy_on(st, ch, (uint16_t*)ch->ag_cols.p + ebase[q], b.ch, b.cols, sizeof(uint16_t) * b.n));
      HIPCHK(ch, copy_on(st, ch, (float*)ch->ag_vals.p + ebase[q], b.ch, b.vals, sizeof(float) * b.n));
      if (q != s)  // row pointers of the block, in place (disjoint pair ranges)
        HIPCHK(ch, copy_on(st, ch, ch->d_rowptr + c->rp_off[b.p0], b.ch, b.rp + c->rp_off[b.p0],
                           sizeof(int32_t) * (c->rp_off[b.p1] - c->rp_off[b.p0])));
    }
    for (int q = 0; q < S; q++) HIPCHK(ch, hipStreamSynchronize(ch->cst[q]));
    return MLP_OK;
  });
  if (rc) return rc;
  // phase 2: swap the gathered store in
  rc = run_shards(c, [&](mlp_ctx* ch, int) -> int {
    uint16_t* oc = ch->d_cols;
    float* ov = ch->d_vals;
    const int64_t ocap = ch->ent_cap;
    ch->d_cols = (uint16_t*)ch->ag_cols.p;
    ch->d_vals = (float*)ch->ag_vals.p;
    ch->ent_cap = (int64_t)std::min(ch->ag_cols.bytes / sizeof(uint16_t), ch->ag_vals.bytes / sizeof(float));
    ch->ag_cols.p = oc;
    ch->ag_cols.bytes = sizeof(uint16_t) * (size_t)ocap;
    ch->ag_vals.p = ov;
    ch->ag_vals.bytes = sizeof(float) * (size_t)ocap;
    ch->ent_off = c->ent_off;
    ch->nnz = c->nnz;
    ch->dist = c->dist;
    ch->mea = c->mea;
    HIPCHK(ch, hipMemcpyAsync(ch->d_ent_off, ch->ent_off.data(), sizeof(int64_t) * (c->P + 1), hipMemcpyHostToDevice,
                              ch->stream));
    HIPCHK(ch, hipStreamSynchronize(ch->stream));
    ch->store_p0 = 0;
    ch->store_p1 = c->P;
    ch->store_total = total;
    ++ch->store_ver;
    return MLP_OK;
  });
  if (rc) return rc;
  // the parent: one copy of the full store from the shard on its device
  int home = 0;
  for (int s = 0; s < S; s++)
    if (c->shards[s]->device == c->device) { home = s; break; }
  const mlp_ctx* h = c->shards[home];
  hipSetDevice(c->device);
  if ((rc = grow_store(c, total, 0))) return rc;
  HIPCHK(c, copy_from(c, c->d_cols, h, h->d_cols, sizeof(uint16_t) * total));
  HIPCHK(c, copy_from(c, c->d_vals, h, h->d_vals, sizeof(float) * total));
  HIPCHK(c, copy_from(c, c->d_rowptr, h, h->d_rowptr, sizeof(int32_t) * c->rp_off[c->P]));
  HIPCHK(c, hipMemcpyAsync(c->d_ent_off, c->ent_off.data(), sizeof(int64_t) * (c->P + 1), hipMemcpyHostToDevice,
                           c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->store_p0 = 0;
  c->store_p1 = c->P;
  c->store_total = total;
  ++c->store_ver;
  c->shards_full_ver = c->store_ver;
  if (c->profile) {
    c->kms[KGATHER] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    c->klaunch[KGATHER] += 1;
    c->kcells[KGATHER] += total;
  }
  return MLP_OK;
}

extern "C" {

// ------------------------------------------------------------------ shards
int mlp_shard_plan(int n, const int32_t* lens, int nranks, int rank, int64_t* b, int64_t* e) {
  if (n < 0 || (n > 0 && !lens) || nranks < 1 || rank < 0 || rank >= nranks || !b || !e) return MLP_ERR_ARG;
  // contiguous ranges of the row-major pair order, balanced by DP cells
  const int64_t P = (int64_t)n * (n - 1) / 2;
  auto cost = [&](int a, int bb) { return (double)(lens[a] + 1) * (double)(lens[bb] + 1); };
  double total = 0;
  for (int a = 0; a < n; a++)
    for (int bb = a + 1; bb < n; bb++) total += cost(a, bb);
  auto cut = [&](int r) -> int64_t {
    if (r <= 0) return 0;
    if (r >= nranks) return P;
    const double target = total * r / nranks;
    double acc = 0;
    int64_t p = 0;
    for (int a = 0; a < n; a++)
      for (int bb = a + 1; bb < n; bb++, p++) {
        if (acc >= target) return p;
        acc += cost(a, bb);
      }
    return P;
  };
  *b = cut(rank);
  *e = cut(rank + 1);
  return MLP_OK;
}

int mlp_shard_range(mlp_ctx* c, int nranks, int rank, int64_t* b, int64_t* e) {
  if (!c) return MLP_ERR_ARG;
  return mlp_shard_plan(c->n, c->lens.data(), nranks, rank, b, e);
}

// Estimated work of output pair (x, y) in one consistency round: the
// reference's multiply-adds if every block's entries spread evenly over the
// residues of z, sum_z nnz(x, z) nnz(z, y) / L_z, plus (n - 2) nnz(x, y) for
// the per-z visit of every mask cell.  Contiguous ranges of equal estimated
// work (shard output pairs by MACs).
int mlp_relax_shard_plan(int n, const int32_t* lens, const int64_t* pair_nnz, int nranks, int64_t* bounds) {
  if (n < 0 || nranks < 1 || !bounds || (n > 0 && (!lens || !pair_nnz))) return MLP_ERR_ARG;
  const int64_t P = (int64_t)n * (n - 1) / 2;
  std::vector<double> cost(std::max<int64_t>(P, 1), 0.0);
  if (n <= 1024) {
    // O(n^3 / 2) multiply-adds (1.5e8 at n = 1024, ~0.1 s serial): rows x
    // spread over host threads (the split only balances; any x order gives
    // the same costs)
    std::vector<float> M((size_t)n * n, 0.f);
    for (int a = 0, p = 0; a < n; a++)
      for (int b = a + 1; b < n; b++, p++) M[(size_t)a * n + b] = M[(size_t)b * n + a] = (float)pair_nnz[p];
    std::atomic<int> next(0);
    auto work = [&]() {
      std::vector<double> acc(n);
      for (int x; (x = next.fetch_add(1)) < n;) {
        std::fill(acc.begin(), acc.end(), 0.0);
        for (int z = 0; z < n; z++) {
          const double w = M[(size_t)x * n + z] / std::max(1, lens[z]);
          if (w == 0) continue;
          const float* mz = &M[(size_t)z * n];
          for (int y = x + 1; y < n; y++) acc[y] += w * mz[y];
        }
        const int64_t base = pair_index_host(n, x, x + 1);
        for (int y = x + 1; y < n; y++) cost[base + (y - x - 1)] = acc[y];
      }
    };
    const int nt = n >= 256 ? std::max(1, std::min(16, (int)std::thread::hardware_concurrency())) : 1;
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; t++) pool.emplace_back(work);
    work();
    for (std::thread& th : pool) th.join();
  } else {  // large families: per-sequence totals only
    std::vector<double> T(n, 0.0);
    for (int a = 0, p = 0; a < n; a++)
      for (int b = a + 1; b < n; b++, p++) T[a] += pair_nnz[p], T[b] += pair_nnz[p];
    double Lm = 0;
    for (int k = 0; k < n; k++) Lm += lens[k];
    Lm = std::max(1.0, Lm / n);
    for (int a = 0, p = 0; a < n; a++)
      for (int b = a + 1; b < n; b++, p++) cost[p] = (double)pair_nnz[p] * (T[a] + T[b]) / (2 * Lm);
  }
  double total = 0;
  for (int64_t p = 0; p < P; p++) total += cost[p] += (double)(n - 2) * pair_nnz[p];
  bounds[0] = 0;
  int64_t p = 0;
  double run = 0;
  for (int r = 1; r < nranks; r++) {
    const double target = total * r / nranks;
    while (p < P && run < target) run += cost[p++];
    bounds[r] = p;
  }
  bounds[nranks] = P;
  return MLP_OK;
}

int mlp_gather_layout(int nranks, int64_t npairs, const int64_t* info, int64_t* ebase) {
  if (nranks < 1 || !info || !ebase) return MLP_ERR_ARG;
  ebase[0] = 0;
  for (int r = 0; r < nranks; r++) {
    if (info[3 * r] != (r == 0 ? 0 : info[3 * (r - 1) + 1]) || info[3 * r + 1] < info[3 * r] ||
        info[3 * r + 2] < 0)
      return MLP_ERR_STATE;
    ebase[r + 1] = ebase[r] + info[3 * r + 2];
  }
  return info[3 * (nranks - 1) + 1] == npairs ? MLP_OK : MLP_ERR_STATE;
}

// ------------------------------------------------------------------ comm
int mlp_comm_unique_id(unsigned char id[128]) {
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return MLP_ERR_COMM;
  static_assert(sizeof(u) == 128, "nccl id size");
  memcpy(id, &u, 128);
  return MLP_OK;
}

int mlp_comm_init(mlp_ctx* c, const unsigned char id[128], int nranks, int rank) {
  if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return MLP_ERR_ARG;
  if (c->host) return MLP_ERR_STATE;
  hipSetDevice(c->device);
  ncclUniqueId u;
  memcpy(&u, id, 128);
  NCCLCHK(c, ncclCommInitRank(&c->comm, nranks, u, rank));
  c->nranks = nranks;
  c->rank = rank;
  return MLP_OK;
}

// Every rank holds pairs [store_p0, store_p1) with entries from 0; after the
// gather every rank holds [0, P) in canonical layout.
int mlp_allgather(mlp_ctx* c) {
  if (!c) return MLP_ERR_ARG;
  // MLP_TEST_ALLGATHER_FORCE=1: the grouped body at one rank as well (test hook)
  static const bool force = knob("MLP_TEST_ALLGATHER_FORCE", 0) > 0;
  if (!c->comm || (c->nranks == 1 && !force)) return MLP_OK;
  hipSetDevice(c->device);
  const int R = c->nranks;
  Timer tm(c, KGATHER, 0);
  // 1. exchange ranges and entry counts (tiny; through device memory)
  std::vector<int64_t> mine = {c->store_p0, c->store_p1, c->store_total, 0};
  int64_t* d_info = nullptr;
  HIPCHK(c, hipMalloc((void**)&d_info, sizeof(int64_t) * 4 * R));
  HIPCHK(c, hipMemcpyAsync(d_info + 4 * c->rank, mine.data(), 32, hipMemcpyHostToDevice, c->stream));
  NCCLCHK(c, ncclAllGather(d_info + 4 * c->rank, d_info, 4, ncclInt64, c->comm, c->stream));
  std::vector<int64_t> info(4 * R);
  HIPCHK(c, hipMemcpyAsync(info.data(), d_info, sizeof(int64_t) * 4 * R, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  hipFree(d_info);
  // ranges must tile [0, P) in rank order
  std::vector<int64_t> ebase(R + 1, 0), tri(3 * R);
  for (int r = 0; r < R; r++)
    for (int k = 0; k < 3; k++) tri[3 * r + k] = info[4 * r + k];
  if (mlp_gather_layout(R, c->P, tri.data(), ebase.data()) != MLP_OK) {
    c->err = "shards must tile the pair range [0, P) in rank order";
    return MLP_ERR_STATE;
  }
  const int64_t total = ebase[R];
  // 2. new entry arrays; my block moves to its global place
  uint16_t* nc = (uint16_t*)pool_alloc(c->device, sizeof(uint16_t) * std::max<int64_t>(total, 1));
  float* nv = nc ? (float*)pool_alloc(c->device, sizeof(float) * std::max<int64_t>(total, 1)) : nullptr;
  if (!nv) {
    pool_free(c->device, nc);
    c->err = "device allocation (gather) failed";
    return MLP_ERR_MEMORY;
  }
  // per-pair scalars through device memory
  float* d_sc = nullptr;
  int64_t* d_nz = nullptr;
  HIPCHK(c, hipMalloc((void**)&d_sc, sizeof(float) * 2 * std::max<int64_t>(c->P, 1)));
  HIPCHK(c, hipMalloc((void**)&d_nz, sizeof(int64_t) * std::max<int64_t>(c->P, 1)));
  const int64_t mp0 = c->store_p0, mp1 = c->store_p1;
  HIPCHK(c, hipMemcpyAsync(d_sc + mp0, c->dist.data() + mp0, sizeof(float) * (mp1 - mp0), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(d_sc + c->P + mp0, c->mea.data() + mp0, sizeof(float) * (mp1 - mp0), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(d_nz + mp0, c->nnz.data() + mp0, sizeof(int64_t) * (mp1 - mp0), hipMemcpyHostToDevice, c->stream));
  NCCLCHK(c, ncclGroupStart());
  for (int r = 0; r < R; r++) {
    const int64_t rp0 = info[4 * r], rp1 = info[4 * r + 1], cnt = info[4 * r + 2];
    const bool me = r == c->rank;
    if (cnt > 0) {
      NCCLCHK(c, ncclBroadcast(me ? (const void*)c->d_cols : nullptr, nc + ebase[r], cnt * 2, ncclUint8, r, c->comm, c->stream));
      NCCLCHK(c, ncclBroadcast(me ? (const void*)c->d_vals : nullptr, nv + ebase[r], cnt, ncclFloat32, r, c->comm, c->stream));
    }
    const int64_t rb = c->rp_off[rp0], re = c->rp_off[rp1];
    if (re > rb) NCCLCHK(c, ncclBroadcast(c->d_rowptr + rb, c->d_rowptr + rb, re - rb, ncclInt32, r, c->comm, c->stream));
    if (rp1 > rp0) {
      NCCLCHK(c, ncclBroadcast(d_sc + rp0, d_sc + rp0, rp1 - rp0, ncclFloat32, r, c->comm, c->stream));
      NCCLCHK(c, ncclBroadcast(d_sc + c->P + rp0, d_sc + c->P + rp0, rp1 - rp0, ncclFloat32, r, c->comm, c->stream));
      NCCLCHK(c, ncclBroadcast(d_nz + rp0, d_nz + rp0, rp1 - rp0, ncclInt64, r, c->comm, c->stream));
    }
  }
  NCCLCHK(c, ncclGroupEnd());
  HIPCHK(c, hipMemcpyAsync(c->dist.data(), d_sc, sizeof(float) * c->P, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->mea.data(), d_sc + c->P, sizeof(float) * c->P, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->nnz.data(), d_nz, sizeof(int64_t) * c->P, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  hipFree(d_sc);
  hipFree(d_nz);
  pool_free(c->device, c->d_cols);
  pool_free(c->device, c->d_vals);
  c->d_cols = nc;
  c->d_vals = nv;
  c->ent_cap = std::max<int64_t>(total, 1);
  c->ent_off[0] = 0;
  for (int64_t p = 0; p < c->P; p++) c->ent_off[p + 1] = c->ent_off[p] + c->nnz[p];
  HIPCHK(c, hipMemcpyAsync(c->d_ent_off, c->ent_off.data(), sizeof(int64_t) * (c->P + 1), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->store_p0 = 0;
  c->store_p1 = c->P;
  c->store_total = total; ++c->store_ver;
  return MLP_OK;
}

}  // extern "C"
