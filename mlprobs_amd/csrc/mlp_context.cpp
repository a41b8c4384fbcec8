// mlp_context.cpp -- contexts, parameter tables, the family, the canonical CSR
// store and the kernel-group timers of libmlpgpu (C ABI: include/mlpgpu.h).
// Parameter tables are built on the host exactly as the reference builds them
// (CPNP/MSA.cpp:444-500, ProbabilisticModel.h:58-135, MSAReadMatrix.cpp:85-116)
// and are bit-identical to the reference's (tests/test_oracle_golden.py).
#include "mlp_runtime.h"

// ------------------------------------------------------------------ device pool
namespace {

// One device's blocks.  A block is one hipMalloc; its free ranges are kept
// by offset (coalesced on release); live allocations map base -> (block,
// bytes).  First fit over the blocks in allocation order.
struct PoolBlock {
  char* base;
  size_t bytes;
  std::map<size_t, size_t> free;   // offset -> length
};
struct DevicePool {
  std::mutex mu;
  int contexts = 0;   // live device contexts on the device
  std::vector<PoolBlock> blocks;
  std::map<char*, std::pair<size_t, size_t>> live;   // ptr -> (block index, bytes); kOwn: a small allocation
};
constexpr size_t kPoolAlign = 2u << 20;
// below this a buffer is a plain allocation of its own (a small release does
// not stall the next allocation, and small buffers would fragment the blocks)
constexpr size_t kPoolMin = 64u << 20;
constexpr size_t kOwn = SIZE_MAX;
thread_local hipError_t pool_last_error = hipSuccess;

DevicePool& pool_of(int device) {
  static std::mutex mu;
  static std::map<int, std::unique_ptr<DevicePool>> pools;
  std::lock_guard<std::mutex> g(mu);
  std::unique_ptr<DevicePool>& p = pools[device];
  if (!p) p.reset(new DevicePool());
  return *p;
}

// the blocks with nothing live in them back to the driver (caller holds mu)
size_t pool_trim_locked(DevicePool& P) {
  size_t freed = 0;
  std::vector<PoolBlock> keep;
  std::vector<size_t> remap(P.blocks.size(), SIZE_MAX);
  for (size_t b = 0; b < P.blocks.size(); b++) {
    PoolBlock& B = P.blocks[b];
    if (B.free.size() == 1 && B.free.begin()->first == 0 && B.free.begin()->second == B.bytes) {
      hipFree(B.base);
      freed += B.bytes;
    } else {
      remap[b] = keep.size();
      keep.push_back(std::move(B));
    }
  }
  for (auto& kv : P.live)
    if (kv.second.first != kOwn) kv.second.first = remap[kv.second.first];
  P.blocks = std::move(keep);
  return freed;
}

// empty blocks back to the driver, largest first, until the pool holds at
// most `keep` bytes (caller holds mu)
void pool_shrink_locked(DevicePool& P, size_t keep) {
  size_t held = 0;
  for (const PoolBlock& B : P.blocks) held += B.bytes;
  while (held > keep) {
    size_t best = SIZE_MAX;
    for (size_t b = 0; b < P.blocks.size(); b++) {
      const PoolBlock& B = P.blocks[b];
      const bool empty = B.free.size() == 1 && B.free.begin()->first == 0 && B.free.begin()->second == B.bytes;
      if (empty && (best == SIZE_MAX || B.bytes > P.blocks[best].bytes)) best = b;
    }
    if (best == SIZE_MAX) return;
    hipFree(P.blocks[best].base);
    held -= P.blocks[best].bytes;
    P.blocks.erase(P.blocks.begin() + best);
    for (auto& kv : P.live)
      if (kv.second.first != kOwn && kv.second.first > best) kv.second.first--;
  }
}

}  // namespace

// A process without live contexts on a device keeps at most MLP_POOL_KEEP_GB
// (default 32 GiB) of blocks there: the next context (a new family, the next
// mask of shards) reuses them, while other processes on the device -- the
// drop-in CLIs a pipeline starts beside a library user -- get the rest back.
void pool_ctx_opened(int device) {
  DevicePool& P = pool_of(device);
  std::lock_guard<std::mutex> g(P.mu);
  P.contexts++;
}

void pool_ctx_closed(int device) {
  DevicePool& P = pool_of(device);
  std::lock_guard<std::mutex> g(P.mu);
  if (--P.contexts > 0) return;
  P.contexts = 0;
  int cur = device;
  hipGetDevice(&cur);
  if (cur != device) hipSetDevice(device);
  pool_shrink_locked(P, (size_t)(knob("MLP_POOL_KEEP_GB", 32.0) * double(1ull << 30)));
  if (cur != device) hipSetDevice(cur);
}

void* pool_alloc(int device, size_t bytes) {
  DevicePool& P = pool_of(device);
  const bool own = bytes < kPoolMin;
  const size_t need = own ? std::max<size_t>(bytes, 256) : (bytes + kPoolAlign - 1) & ~(kPoolAlign - 1);
  std::lock_guard<std::mutex> g(P.mu);
  if (!own) {   // best fit over the blocks' free ranges
    size_t bb = SIZE_MAX, boff = 0, blen = SIZE_MAX;
    for (size_t b = 0; b < P.blocks.size(); b++)
      for (const auto& kv : P.blocks[b].free)
        if (kv.second >= need && kv.second < blen) {
          bb = b;
          boff = kv.first;
          blen = kv.second;
        }
    if (bb != SIZE_MAX) {
      PoolBlock& B = P.blocks[bb];
      B.free.erase(boff);
      if (blen > need) B.free[boff + need] = blen - need;
      P.live[B.base + boff] = {bb, need};
      return B.base + boff;
    }
  }
  void* p = nullptr;
  int cur = device;
  hipGetDevice(&cur);
  if (cur != device) hipSetDevice(device);
  hipError_t e = hipMalloc(&p, need);
  if (e != hipSuccess) {
    hipGetLastError();
    if (pool_trim_locked(P)) e = hipMalloc(&p, need);
    if (e != hipSuccess) hipGetLastError();
  }
  if (cur != device) hipSetDevice(cur);
  pool_last_error = e;
  if (e != hipSuccess) return nullptr;
  if (own) {
    P.live[(char*)p] = {kOwn, need};
    return p;
  }
  P.blocks.push_back(PoolBlock{(char*)p, need, {}});
  P.live[(char*)p] = {P.blocks.size() - 1, need};
  return p;
}

void pool_free(int device, void* p) {
  if (!p) return;
  DevicePool& P = pool_of(device);
  std::lock_guard<std::mutex> g(P.mu);
  auto lv = P.live.find((char*)p);
  if (lv == P.live.end()) return;
  if (lv->second.first == kOwn) {
    P.live.erase(lv);
    hipFree(p);
    return;
  }
  PoolBlock& B = P.blocks[lv->second.first];
  size_t off = (size_t)((char*)p - B.base), len = lv->second.second;
  P.live.erase(lv);
  auto next = B.free.lower_bound(off);
  if (next != B.free.end() && next->first == off + len) {   // coalesce with the range after
    len += next->second;
    next = B.free.erase(next);
  }
  if (next != B.free.begin()) {   // and the one before
    auto prev = std::prev(next);
    if (prev->first + prev->second == off) {
      off = prev->first;
      len += prev->second;
      B.free.erase(prev);
    }
  }
  B.free[off] = len;
}

extern "C" int mlp_pool_info(int device, uint64_t* held, uint64_t* free_bytes) {
  DevicePool& P = pool_of(device);
  std::lock_guard<std::mutex> g(P.mu);
  uint64_t h = 0, f = 0;
  for (const PoolBlock& B : P.blocks) {
    h += B.bytes;
    for (const auto& kv : B.free) f += kv.second;
  }
  if (held) *held = h;
  if (free_bytes) *free_bytes = f;
  return MLP_OK;
}

extern "C" int mlp_pool_trim(int device) {
  DevicePool& P = pool_of(device);
  std::lock_guard<std::mutex> g(P.mu);
  pool_trim_locked(P);
  return MLP_OK;
}

size_t pool_free_bytes(int device) {
  DevicePool& P = pool_of(device);
  std::lock_guard<std::mutex> g(P.mu);
  size_t n = 0;
  for (const PoolBlock& B : P.blocks)
    for (const auto& kv : B.free) n += kv.second;
  return n;
}

std::string pool_failure(int device, size_t bytes) {
  uint64_t held = 0, pfree = 0;
  mlp_pool_info(device, &held, &pfree);
  size_t freeb = 0, total = 0;
  int cur = device;
  hipGetDevice(&cur);
  if (cur != device) hipSetDevice(device);
  if (hipMemGetInfo(&freeb, &total) != hipSuccess) hipGetLastError();
  if (cur != device) hipSetDevice(cur);
  const auto mb = [](uint64_t b) { return std::to_string(b >> 20); };
  return "device allocation failed (" + std::to_string(bytes) + " bytes: " + hipGetErrorName(pool_last_error) +
         "; device " + std::to_string(device) + " free " + mb(freeb) + " of " + mb(total) + " MB, pool holds " +
         mb(held) + " MB, " + mb(pfree) + " MB of it free)";
}

// ------------------------------------------------------------------ helpers

int ensure(mlp_ctx* c, DevBuf& b, size_t bytes) {
  if (b.lent) {  // a lent buffer is only valid inside the round that carved it
    b.p = nullptr;
    b.bytes = 0;
    b.lent = false;
  }
  if (b.bytes >= bytes) return MLP_OK;
  if (b.p) {   // as hipFree would: nothing in flight may still use it when it is handed out again
    hipDeviceSynchronize();
    pool_free(c->device, b.p);
  }
  b.p = nullptr;
  b.bytes = 0;
  const size_t want = std::max<size_t>(bytes, 256);
  if (!(b.p = pool_alloc(c->device, want))) {
    c->err = pool_failure(c->device, want);
    return MLP_ERR_MEMORY;
  }
  b.bytes = want;
  return MLP_OK;
}

// A relaxation round's temporaries (transposes, images, tiles, raw values,
// the filtered entries) carved from the posterior stage's batch scratch,
// idle between posterior stages: at C3 ~10 GB fewer bytes per process (a
// fresh process's allocations wait while the driver clears what earlier
// processes released).  Valid until the round ends; without scratch room
// the buffer is an owned allocation as before.
int ensure_tmp(mlp_ctx* c, DevBuf& b, size_t bytes) {
  const size_t need = (std::max<size_t>(bytes, 256) + 255) & ~(size_t)255;
  if (c->arena_on && c->scratch.p && c->arena_off + need <= c->scratch.bytes) {
    if (b.p && !b.lent) pool_free(c->device, b.p);
    b.p = (char*)c->scratch.p + c->arena_off;
    b.bytes = need;
    b.lent = true;
    c->arena_off += need;
    return MLP_OK;
  }
  return ensure(c, b, bytes);
}

hipEvent_t pool_event(mlp_ctx* c) {
  if (c->evused == c->evpool.size()) {
    hipEvent_t e;
    hipEventCreate(&e);
    c->evpool.push_back(e);
  }
  return c->evpool[c->evused++];
}

void flush_timers(mlp_ctx* c) {
  for (const mlp_ctx::TimerRec& r : c->tpend) {
    hipEventSynchronize(r.e1);
    float ms = 0;
    if (r.e1b) {
      hipEventSynchronize(r.e1b);
      auto at = [&](hipEvent_t e) {
        float t = 0;
        hipEventElapsedTime(&t, r.eref, e);
        return t;
      };
      const float t0 = r.e0b ? std::min(at(r.e0), at(r.e0b)) : at(r.e0);
      ms = std::max(at(r.e1), at(r.e1b)) - t0;
    } else {
      hipEventElapsedTime(&ms, r.e0, r.e1);
    }
    c->kms[r.id] += ms;
    if (!r.cont) {
      c->klaunch[r.id] += 1;
      c->kcells[r.id] += r.cells;
    }
  }
  c->tpend.clear();
  c->evused = 0;
}

// Parameter tables exactly as the reference builds them.
void build_tables(Tables& T, ModelScalars& ms, float delta, bool qp) {
  static thread_local float emitPairs[256][256];  // shards build their tables concurrently
  static thread_local float emitSingle[256];
  for (int i = 0; i < 256; i++) {
    emitSingle[i] = (float)1e-5;
    for (int j = 0; j < 256; j++) emitPairs[i][j] = (float)1e-10;
  }
  float initDistrib[5], gapOpen[4], gapExtend[4];
  memcpy(initDistrib, mlp_init_distrib, sizeof initDistrib);
  memcpy(gapOpen, mlp_gap_open, sizeof gapOpen);
  memcpy(gapExtend, mlp_gap_extend, sizeof gapExtend);
  if (delta >= 0) initDistrib[2] = delta;
  const char* alpha = MLP_ALPHABET;
  int tri = 0;
  for (int i = 0; i < 20; i++) {
    unsigned char ui = (unsigned char)toupper(alpha[i]);
    emitSingle[ui] = mlp_emit_single[i];
    for (int j = 0; j <= i; j++, tri++) {
      unsigned char uj = (unsigned char)toupper(alpha[j]);
      emitPairs[ui][uj] = emitPairs[uj][ui] = mlp_emit_pairs_lower[tri];
    }
  }
  // CPNP/ProbabilisticModel.h:75-99
  float tm[5][5] = {{0}};
  tm[0][0] = 1;
  for (int i = 0; i < 2; i++) {
    tm[0][2 * i + 1] = gapOpen[2 * i];
    tm[0][2 * i + 2] = gapOpen[2 * i];
    tm[0][0] -= (gapOpen[2 * i] + gapOpen[2 * i]);
    tm[2 * i + 1][2 * i + 1] = gapExtend[2 * i];
    tm[2 * i + 2][2 * i + 2] = gapExtend[2 * i];
    tm[2 * i + 1][0] = 1 - gapExtend[2 * i];
    tm[2 * i + 2][0] = 1 - gapExtend[2 * i];
  }
  for (int i = 0; i < 5; i++) {
    ms.init[i] = logf(initDistrib[i]);
    for (int j = 0; j < 5; j++) ms.t[i][j] = logf(tm[i][j]);
  }
  ms.init[2] = logf(initDistrib[1]);
  float lt[3][3] = {{0}};
  lt[0][0] = 1;
  lt[0][1] = gapOpen[1];
  lt[0][2] = gapOpen[1];
  lt[0][0] -= (gapOpen[1] + gapOpen[1]);
  lt[1][1] = gapExtend[1];
  lt[2][2] = gapExtend[1];
  lt[1][0] = 1 - gapExtend[1];
  lt[2][0] = 1 - gapExtend[1];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) ms.lt[i][j] = logf(lt[i][j]);
  ms.rt1 = logf(1 - initDistrib[2]);
  for (int r = 0; r < 26; r++) {
    T.ins[r] = logf(emitSingle['A' + r]);
    for (int c = 0; c < 26; c++) T.match[r * 26 + c] = logf(emitPairs['A' + r]['A' + c]);
  }
  // Partition function (CPNP/MSAReadMatrix.cpp:85-116, MSAPartProbs.cpp:698-709)
  const char* bases = MLP_GONNET_MONOMERS;
  const int nb = (int)strlen(bases);
  static thread_local double sm[26][26];
  int si[26];
  for (int i = 0; i < 26; i++) si[i] = -1;
  for (int i = 0; i < nb; i++) si[bases[i] - 'A'] = i;
  const float beta = (float)(1.0 / 5.0f);
  int pos = 0;
  for (int i = 0; i < nb; i++)
    for (int j = 0; j <= i; j++) {
      const double v = expf(beta * mlp_gonnet160_lower[pos++]);
      sm[i][j] = sm[j][i] = v;
    }
  // J, O, U have subst_index -1 in the reference (an out-of-bounds read);
  // they are scored as X here.
  const int xi = si['X' - 'A'];
  for (int r = 0; r < 26; r++)
    for (int c = 0; c < 26; c++) {
      const int a = si[r] >= 0 ? si[r] : xi, b = si[c] >= 0 ? si[c] : xi;
      T.sub[r * 26 + c] = sm[a][b];
    }
  const double beta_d = beta;
  ms.pf_open = exp(beta_d * -22.0);
  ms.pf_ext = exp(beta_d * -1.0);
  if (qp) {  // QuickProbs' partition function: VTML200 (mlp_params_qp.inc); its pair-HMM is this one
    for (int r = 0; r < 26; r++)
      for (int c = 0; c < 26; c++) T.sub[r * 26 + c] = mlp_qp_pf_sub[c * 26 + r];  // [seq2][seq1]
    ms.pf_open = mlp_qp_pf_open;
    ms.pf_ext = mlp_qp_pf_extend;
  }
  for (int k = 0; k < 26 * 26; k++) T.rsub[k] = 1.0 / T.sub[k];
  // CPNP/ProbabilisticModel.h:1068-1070: LOG(0.6080327034), LOG(0.1959836632) x 2
  ms.vit_init[0] = logf(0.6080327034f);
  ms.vit_init[1] = logf(0.1959836632f);
  ms.vit_init[2] = logf(0.1959836632f);
}

// ------------------------------------------------------------------ C ABI
extern "C" {

int mlp_ctx_create(int device, mlp_ctx** out) {
  if (!out) return MLP_ERR_ARG;
  *out = nullptr;
  mlp_ctx* c = new mlp_ctx();
  c->device = device;
  if (hipSetDevice(device) != hipSuccess) {
    delete c;
    return MLP_ERR_HIP;
  }
  hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, device);
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return MLP_ERR_HIP;
  }
  if (hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return MLP_ERR_HIP;
  }
  if (hipStreamCreateWithFlags(&c->side.st, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->side.fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->side.join, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_done[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_done[1], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_tot, hipEventDisableTiming) != hipSuccess) {
    delete c;
    return MLP_ERR_HIP;
  }
  c->side.join_mode = 0;
  if (hipMalloc((void**)&c->d_tables, sizeof(Tables)) != hipSuccess) {
    delete c;
    return MLP_ERR_MEMORY;
  }
  size_t freeb = 0, total = 0;
  hipMemGetInfo(&freeb, &total);
  // per-batch scratch: the free HBM less a reserve for the CSR store and the
  // relaxation's own buffers (its temporaries are carved from this scratch
  // when it is idle): larger batches keep every SIMD busy through the serial
  // local-total chains and shorten the per-batch tails -- on MI355X ~224 GiB,
  // the C3 posterior stage in three batches instead of five (step 576 -> 545-557
  // ms, totals 61 -> 48.5 ms; round 4 measured half the free HBM until then).
  // The budget is a cap: a batch allocates only what its pairs need, so a
  // family smaller than the device takes no more than it uses.  Planned from
  // the free HBM as the driver reports it (a device shared with another
  // process gets smaller batches, never an oversubscription); an allocation
  // that still fails halves the budget and retries.
  {
    const size_t usable = freeb + pool_free_bytes(device);   // the pool's free ranges serve it too
    const size_t reserve = std::max<size_t>(16ull << 30, total / 100 * 7);
    c->scratch_budget = usable > 2 * reserve ? usable - reserve : usable / 2;
  }
  if (knob_set("MLP_SCRATCH_GB")) c->scratch_budget = (size_t)(knob("MLP_SCRATCH_GB", 0) * (1ull << 30));
  pool_ctx_opened(device);
  *out = c;
  return MLP_OK;
}

int mlp_ctx_create_host(mlp_ctx** out) {
  if (!out) return MLP_ERR_ARG;
  *out = new mlp_ctx();
  (*out)->host = true;
  return MLP_OK;
}

int mlp_ctx_is_host(const mlp_ctx* c) { return c && c->host ? 1 : 0; }

int mlp_ctx_create_mask(uint64_t device_mask, mlp_ctx** out) {
  if (!out) return MLP_ERR_ARG;
  *out = nullptr;
  const std::vector<int> devs = mask_devices(device_mask);
  if (devs.empty()) return MLP_ERR_ARG;
  int rc = mlp_ctx_create(devs[0], out);
  if (rc) return rc;
  uint64_t m = 0;
  for (int d : devs) m |= 1ull << d;
  (*out)->dev_mask = m;
  return MLP_OK;
}

int mlp_set_shards(mlp_ctx* c, int nshards) {
  if (!c || nshards < 0) return MLP_ERR_ARG;
  c->shards_req = nshards;
  return MLP_OK;
}

int mlp_shard_count(mlp_ctx* c) { return c ? (c->host ? 1 : shard_count(c)) : 0; }

void mlp_ctx_destroy(mlp_ctx* c) {
  if (!c) return;
  if (c->host) {
    delete c;
    return;
  }
  for (mlp_ctx* ch : c->shards) mlp_ctx_destroy(ch);
  c->shards.clear();
  hipSetDevice(c->device);
  hipStreamSynchronize(c->stream);
  hipStreamSynchronize(c->stream2);
  if (c->side.st) hipStreamSynchronize(c->side.st);
  if (c->d_tables) hipFree(c->d_tables);
  // the family's arrays and the store: back to the pool
  void* ptrs[] = {c->d_res, c->d_off, c->d_len, c->d_rp_off, c->d_trp_off, c->d_rowptr, c->d_ent_off,
                  c->d_cols, c->d_vals};
  for (void* p : ptrs) pool_free(c->device, p);
  DevBuf* bufs[] = {&c->scratch, &c->r_trowptr, &c->r_tcols, &c->r_tvals, &c->r_raw, &c->r_newrp,
                    &c->r_newcols, &c->r_newvals, &c->r_tasks_p, &c->r_tasks_r, &c->r_pairs,
                    &c->r_nnz, &c->r_newoff, &c->r_img, &c->r_imgoff, &c->r_tiles, &c->r_nwords, &c->r_weights,
                    &c->r_seldist, &c->r_profile, &c->r_mea, &c->ag_cols, &c->ag_vals};
  for (DevBuf* b : bufs)
    if (b->p && !b->lent) pool_free(c->device, b->p);
  if (c->comm) ncclCommDestroy(c->comm);
  for (hipEvent_t e : c->evpool) hipEventDestroy(e);
  if (knob_set("MLP_LOG_PROFILE") && (c->prof_t[0] > 0 || c->prof_t[1] > 0))
    fprintf(stderr, "[profile posterior] host preparation %.3f s, device round trips %.3f s\n", c->prof_t[0],
            c->prof_t[1]);
  if (c->h_prof_in) hipHostFree(c->h_prof_in);
  if (c->h_prof_out) hipHostFree(c->h_prof_out);
  if (c->h_mea) hipHostFree(c->h_mea);
  for (PairRec* r : c->h_rec)
    if (r) hipHostFree(r);
  for (uint8_t* u : c->h_up)
    if (u) hipHostFree(u);
  for (int64_t* u : c->h_ent)
    if (u) hipHostFree(u);
  for (hipStream_t st : c->cst) hipStreamDestroy(st);
  hipStreamDestroy(c->stream);
  hipStreamDestroy(c->stream2);
  if (c->side.st) {
    hipStreamDestroy(c->side.st);
    hipEventDestroy(c->side.fork);
    hipEventDestroy(c->side.join);
  }
  for (hipEvent_t e : {c->ev_done[0], c->ev_done[1], c->ev_fork, c->ev_tot}) {
    if (e) hipEventDestroy(e);
  }
  const int device = c->device;
  delete c;
  pool_ctx_closed(device);
}

const char* mlp_last_error(const mlp_ctx* c) { return c ? c->err.c_str() : "null context"; }

int mlp_set_scratch(mlp_ctx* c, uint64_t bytes) {
  if (!c || bytes < (64u << 20)) return MLP_ERR_ARG;
  c->scratch_budget = (size_t)bytes;
  return MLP_OK;
}

int mlp_family_load(mlp_ctx* c, int n, const char* residues, const int64_t* offsets) {
  if (!c || n < 1 || !residues || !offsets) return MLP_ERR_ARG;
  for (mlp_ctx* ch : c->shards) mlp_ctx_destroy(ch);  // re-created for the new family when needed
  c->shards.clear();
  c->shards_full_ver = ~0ull;
  if (!c->host) hipSetDevice(c->device);
  c->n = n;
  c->lens.assign(n, 0);
  c->offs.assign(offsets, offsets + n + 1);
  c->max_len = 0;
  const int64_t tot = offsets[n];
  std::vector<uint8_t> codes(std::max<int64_t>(tot, 1));
  for (int k = 0; k < n; k++) {
    const int64_t L = offsets[k + 1] - offsets[k];
    if (L < 1 || L > 65535) {
      c->err = "sequence length must be in [1, 65535]";
      return MLP_ERR_ARG;
    }
    c->lens[k] = (int32_t)L;
    c->max_len = std::max(c->max_len, (int)L);
    for (int64_t q = offsets[k]; q < offsets[k + 1]; q++) {
      const unsigned char ch = (unsigned char)residues[q];
      if (ch < 'A' || ch > 'Z') {
        c->err = "residues must be uppercase letters A-Z";
        return MLP_ERR_ARG;
      }
      codes[q] = (uint8_t)(ch - 'A');
    }
  }
  c->h_res.assign(residues, residues + tot);
  c->P = (int64_t)n * (n - 1) / 2;
  c->pa.resize(c->P);
  c->pb.resize(c->P);
  c->rp_off.assign(c->P + 1, 0);
  c->trp_off.assign(c->P + 1, 0);
  int64_t p = 0;
  for (int a = 0; a < n; a++)
    for (int b = a + 1; b < n; b++, p++) {
      c->pa[p] = a;
      c->pb[p] = b;
      c->rp_off[p + 1] = c->rp_off[p] + c->lens[a] + 2;
      c->trp_off[p + 1] = c->trp_off[p] + c->lens[b] + 2;
    }
  int rc;
  c->ent_off.assign(c->P + 1, 0);
  c->dist.assign(c->P, 0.f);
  c->mea.assign(c->P, 0.f);
  c->nnz.assign(c->P, 0);
  c->store_p0 = c->store_p1 = 0;
  c->store_total = 0; ++c->store_ver;
  c->vit_len.assign(c->P, 0);
  c->vit_match.assign(c->P, 0.f);
  c->vit_off.assign(c->P + 1, 0);
  for (int64_t q = 0; q < c->P; q++) c->vit_off[q + 1] = c->vit_off[q] + c->lens[c->pa[q]] + c->lens[c->pb[q]];
  c->vit_path.clear();
  c->vit_done = c->vit_paths = false;
  if (c->host) {
    c->hs.rowptr.assign(c->rp_off[c->P], 0);
    c->hs.ent_off.assign(c->P + 1, 0);
    c->hs.cols.clear();
    c->hs.vals.clear();
    return MLP_OK;
  }
  if ((rc = dalloc(c, &c->d_res, codes.size()))) return rc;
  if ((rc = dalloc(c, &c->d_off, n + 1))) return rc;
  if ((rc = dalloc(c, &c->d_len, n))) return rc;
  if ((rc = dalloc(c, &c->d_rp_off, c->P + 1))) return rc;
  if ((rc = dalloc(c, &c->d_trp_off, c->P + 1))) return rc;
  if ((rc = dalloc(c, &c->d_rowptr, c->rp_off[c->P]))) return rc;
  if ((rc = dalloc(c, &c->d_ent_off, c->P + 1))) return rc;
  HIPCHK(c, hipMemcpy(c->d_res, codes.data(), codes.size(), hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->d_off, offsets, sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->d_len, c->lens.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->d_rp_off, c->rp_off.data(), sizeof(int64_t) * (c->P + 1), hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->d_trp_off, c->trp_off.data(), sizeof(int64_t) * (c->P + 1), hipMemcpyHostToDevice));
  return MLP_OK;
}

int64_t mlp_family_npairs(const mlp_ctx* c) { return c ? c->P : 0; }

}  // extern "C"

// grow the entry store to hold `need` entries, keeping `keep` existing ones
int grow_store(mlp_ctx* c, int64_t need, int64_t keep, int64_t want, bool sync2) {
  if (need <= c->ent_cap) return MLP_OK;
  // a compaction may still be writing the old store on stream2 (two-slot
  // batches); the caller passes false when its compactions use the context stream
  if (sync2) HIPCHK(c, hipStreamSynchronize(c->stream2));
  // `want`: the caller's estimate of the final size, so a growing store is
  // reallocated (and copied) once rather than every 1.5x
  int64_t cap = std::max<int64_t>(std::max<int64_t>(need, want), c->ent_cap + c->ent_cap / 2);
  uint16_t* nc = (uint16_t*)pool_alloc(c->device, sizeof(uint16_t) * cap);
  float* nv = nc ? (float*)pool_alloc(c->device, sizeof(float) * cap) : nullptr;
  if (!nv) {
    pool_free(c->device, nc);
    c->err = "device allocation (CSR store) failed";
    return MLP_ERR_MEMORY;
  }
  if (keep > 0) {
    HIPCHK(c, hipMemcpyAsync(nc, c->d_cols, sizeof(uint16_t) * keep, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(nv, c->d_vals, sizeof(float) * keep, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  pool_free(c->device, c->d_cols);
  pool_free(c->device, c->d_vals);
  c->d_cols = nc;
  c->d_vals = nv;
  c->ent_cap = cap;
  return MLP_OK;
}

extern "C" {

int mlp_pair_results(mlp_ctx* c, int64_t p0, int64_t p1, float* dist, float* mea, int64_t* nnz) {
  if (!c || p0 < 0 || p1 > c->P || p0 > p1) return MLP_ERR_ARG;
  for (int64_t p = p0; p < p1; p++) {
    if (dist) dist[p - p0] = c->dist[p];
    if (mea) mea[p - p0] = c->mea[p];
    if (nnz) nnz[p - p0] = c->nnz[p];
  }
  return MLP_OK;
}

int mlp_csr_total(mlp_ctx* c, int64_t* total) {
  if (!c || !total) return MLP_ERR_ARG;
  *total = c->store_total;
  return MLP_OK;
}

int mlp_csr_export(mlp_ctx* c, int32_t* row_ptr, int64_t* ent_off, uint16_t* cols, float* vals) {
  if (!c) return MLP_ERR_ARG;
  if (c->host) {
    if (row_ptr) memcpy(row_ptr, c->hs.rowptr.data(), sizeof(int32_t) * c->rp_off[c->P]);
    if (ent_off) memcpy(ent_off, c->ent_off.data(), sizeof(int64_t) * (c->P + 1));
    if (cols && c->store_total) memcpy(cols, c->hs.cols.data(), sizeof(uint16_t) * c->store_total);
    if (vals && c->store_total) memcpy(vals, c->hs.vals.data(), sizeof(float) * c->store_total);
    return MLP_OK;
  }
  hipSetDevice(c->device);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (row_ptr) HIPCHK(c, hipMemcpy(row_ptr, c->d_rowptr, sizeof(int32_t) * c->rp_off[c->P], hipMemcpyDeviceToHost));
  if (ent_off) memcpy(ent_off, c->ent_off.data(), sizeof(int64_t) * (c->P + 1));
  if (cols && c->store_total) HIPCHK(c, hipMemcpy(cols, c->d_cols, sizeof(uint16_t) * c->store_total, hipMemcpyDeviceToHost));
  if (vals && c->store_total) HIPCHK(c, hipMemcpy(vals, c->d_vals, sizeof(float) * c->store_total, hipMemcpyDeviceToHost));
  return MLP_OK;
}

int mlp_relax_blockmfma_eval(mlp_ctx* c, int nx, const int32_t* xs, int ny, const int32_t* ys, double* res) {
  if (!c || !xs || !ys || !res || nx <= 0 || ny <= 0) return MLP_ERR_ARG;
  if (c->host) return MLP_ERR_STATE;
  if (c->store_p0 != 0 || c->store_p1 != c->P) {
    c->err = "blockmfma eval needs every pair";
    return MLP_ERR_STATE;
  }
  for (int k = 0; k < nx; k++)
    if (xs[k] < 0 || xs[k] >= c->n) return MLP_ERR_ARG;
  for (int k = 0; k < ny; k++)
    if (ys[k] < 0 || ys[k] >= c->n) return MLP_ERR_ARG;
  std::vector<int32_t> rp(c->rp_off[c->P]);
  std::vector<uint16_t> cols(std::max<int64_t>(c->store_total, 1));
  std::vector<float> vals(std::max<int64_t>(c->store_total, 1));
  int rc;
  if ((rc = mlp_csr_export(c, rp.data(), nullptr, cols.data(), vals.data()))) return rc;
  hipSetDevice(c->device);
  return mlp::relax_blockmfma_eval(c->n, c->lens.data(), c->rp_off.data(), rp.data(), c->ent_off.data(), cols.data(),
                                   vals.data(), nx, xs, ny, ys, res, c->err);
}

int mlp_csr_import(mlp_ctx* c, const int32_t* row_ptr, const int64_t* ent_off, const uint16_t* cols,
                   const float* vals) {
  if (!c || !row_ptr || !ent_off) return MLP_ERR_ARG;
  if (c->n < 2) return MLP_ERR_STATE;
  const int64_t total = ent_off[c->P];
  if (c->host) {
    c->hs.rowptr.assign(row_ptr, row_ptr + c->rp_off[c->P]);
    c->hs.ent_off.assign(ent_off, ent_off + c->P + 1);
    c->hs.cols.assign(cols, cols + total);
    c->hs.vals.assign(vals, vals + total);
    c->ent_off.assign(ent_off, ent_off + c->P + 1);
    for (int64_t p = 0; p < c->P; p++) c->nnz[p] = ent_off[p + 1] - ent_off[p];
    c->store_p0 = 0;
    c->store_p1 = c->P;
    c->store_total = total; ++c->store_ver;
    return MLP_OK;
  }
  hipSetDevice(c->device);
  int rc;
  if ((rc = grow_store(c, total, 0))) return rc;
  HIPCHK(c, hipMemcpy(c->d_rowptr, row_ptr, sizeof(int32_t) * c->rp_off[c->P], hipMemcpyHostToDevice));
  if (total) {
    HIPCHK(c, hipMemcpy(c->d_cols, cols, sizeof(uint16_t) * total, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_vals, vals, sizeof(float) * total, hipMemcpyHostToDevice));
  }
  c->ent_off.assign(ent_off, ent_off + c->P + 1);
  HIPCHK(c, hipMemcpy(c->d_ent_off, ent_off, sizeof(int64_t) * (c->P + 1), hipMemcpyHostToDevice));
  for (int64_t p = 0; p < c->P; p++) c->nnz[p] = ent_off[p + 1] - ent_off[p];
  c->store_p0 = 0;
  c->store_p1 = c->P;
  c->store_total = total; ++c->store_ver;
  return MLP_OK;
}

int mlp_synchronize(mlp_ctx* c) {
  if (!c) return MLP_ERR_ARG;
  if (c->host) return MLP_OK;
  for (mlp_ctx* ch : c->shards) {
    hipSetDevice(ch->device);
    HIPCHK(c, hipStreamSynchronize(ch->stream));
  }
  hipSetDevice(c->device);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MLP_OK;
}

int mlp_profile(mlp_ctx* c, int enable) {
  if (!c) return MLP_ERR_ARG;
  c->profile = enable != 0;
  for (mlp_ctx* ch : c->shards) ch->profile = c->profile;
  return MLP_OK;
}

int mlp_profile_reset(mlp_ctx* c) {
  if (!c) return MLP_ERR_ARG;
  if (c->host) return MLP_OK;
  for (mlp_ctx* ch : c->shards) mlp_profile_reset(ch);
  flush_timers(c);
  for (int k = 0; k < MLP_NKERNELS; k++) {
    c->kms[k] = 0;
    c->klaunch[k] = 0;
    c->kcells[k] = 0;
  }
  return MLP_OK;
}

int mlp_kernel_times(mlp_ctx* c, double* ms, int64_t* launches, int64_t* cells) {
  if (!c) return MLP_ERR_ARG;
  if (c->host) {
    for (int k = 0; k < MLP_NKERNELS; k++) {
      if (ms) ms[k] = 0;
      if (launches) launches[k] = 0;
      if (cells) cells[k] = 0;
    }
    return MLP_OK;
  }
  flush_timers(c);
  for (mlp_ctx* ch : c->shards) {
    hipSetDevice(ch->device);
    flush_timers(ch);
  }
  hipSetDevice(c->device);
  for (int k = 0; k < MLP_NKERNELS; k++) {  // shards: device time summed over the shards
    double m = c->kms[k];
    int64_t l = c->klaunch[k], e = c->kcells[k];
    for (const mlp_ctx* ch : c->shards) {
      m += ch->kms[k];
      l += ch->klaunch[k];
      e += ch->kcells[k];
    }
    if (ms) ms[k] = m;
    if (launches) launches[k] = l;
    if (cells) cells[k] = e;
  }
  return MLP_OK;
}

}  // extern "C"
