// mlp_runtime.h -- internal header of the libmlpgpu host runtime (not part of
// the C ABI, include/mlpgpu.h).  The context (mlp_ctx), device buffers,
// kernel-group timers and the helpers the runtime's translation units share:
//   mlp_context.cpp    contexts, model tables, family, CSR store, timers
//   mlp_planner.cpp    batch planning: chains, scratch carving, plan upload
//   mlp_posteriors.cpp the posterior stage (mlp_posteriors)
//   mlp_profile_rt.cpp profile posterior + device MEA, Viterbi family test
//   mlp_shards.cpp     in-process shards, shard plans, RCCL all-gather
//   mlp_relax_rt.cpp   consistency rounds (mlp_relax*)
#pragma once
#include "../../include/mlpgpu.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "host_backend.h"
#include "mlp_kernels.h"
#include "mlp_params_default.inc"
#include "mlp_params_qp.inc"

using namespace mlp;

// runtime helpers shared by the translation units, not exported from the library
#define MLP_HIDDEN __attribute__((visibility("hidden")))

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  bool lent = false;  // carved from the idle batch scratch (ensure_tmp), not owned
};

enum KernelId { KFWD = 0, KBWD, KTOT, KMERGE, KCOMPACT, KRELAX, KTRANS, KFILTER, KGATHER, KVITERBI };

struct mlp_ctx {
  int device = 0;
  int cus = 256;                      // compute units (chain planning)
  bool host = false;                  // mlp_ctx_create_host: every stage on the CPU, no HIP call
  mlph::Store hs;                     // the host context's canonical CSR store
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;      // the local totals' forward chains beside the backward sweeps
  SideStream side{};                  // concurrent second sweep kernel of a batch (mlp_kernels.h)
  std::string err;
  // parameter tables
  Tables* d_tables = nullptr;
  Tables h_tables;
  // family
  int n = 0;
  int max_len = 0;
  int64_t P = 0;
  std::vector<int32_t> lens;
  std::vector<int64_t> offs;
  std::vector<uint8_t> h_res;         // residue letters of the family (host)
  std::vector<int32_t> pa, pb;        // per pair
  std::vector<int64_t> rp_off;        // canonical row_ptr offsets (P + 1)
  std::vector<int64_t> trp_off;       // transposed row_ptr offsets (P + 1)
  uint8_t* d_res = nullptr;
  int64_t* d_off = nullptr;
  int32_t* d_len = nullptr;
  int64_t* d_rp_off = nullptr;
  int64_t* d_trp_off = nullptr;
  // canonical CSR store
  int32_t* d_rowptr = nullptr;        // rp_off[P] ints
  int64_t* d_ent_off = nullptr;       // P + 1
  uint16_t* d_cols = nullptr;
  float* d_vals = nullptr;
  int64_t ent_cap = 0;
  std::vector<int64_t> ent_off;       // host mirror (P + 1)
  int64_t store_p0 = 0, store_p1 = 0; // pairs currently held (contiguous)
  int64_t store_total = 0;
  uint64_t store_ver = 0, tr_ver = ~0ull;
  // pinned host staging of the profile posterior (uploads; result)
  void* h_prof_in = nullptr;
  size_t h_prof_in_bytes = 0;
  float* h_prof_out = nullptr;
  size_t h_prof_out_bytes = 0;
  double prof_t[2] = {0, 0};  // host preparation, device round trip (MLP_PROFILE_TIMES)
  // the last profile posterior's matrix on the device (mlp_profile_defer / _mea / _gather)
  bool prof_defer = false;
  float* prof_dout = nullptr;
  int prof_L1 = 0, prof_L2 = 0;
  uint8_t* h_mea = nullptr;           // pinned: MEA choices + score
  PairRec* h_rec[2] = {nullptr, nullptr};  // pinned: a posterior batch's pair records (batch parity)
  size_t h_rec_n[2] = {0, 0};
  uint8_t* h_up[2] = {nullptr, nullptr};   // pinned: a batch's plan on its way up (batch parity)
  size_t h_up_n[2] = {0, 0};
  int64_t* h_ent[2] = {nullptr, nullptr};  // pinned: a batch's entry bases (parity; written when it is finished)
  size_t h_ent_n[2] = {0, 0};
  size_t h_mea_bytes = 0;
  std::vector<float> dist, mea;
  std::vector<int64_t> nnz;
  // Viterbi family test (per pair, pair order)
  std::vector<int32_t> vit_len;
  std::vector<float> vit_match;
  std::vector<int64_t> vit_off;       // path offsets (P + 1), capacity L_a + L_b
  std::vector<uint8_t> vit_path;      // forward order, 0 = B, 1 = X, 2 = Y (when kept)
  bool vit_done = false, vit_paths = false;
  // batch scratch
  DevBuf scratch;                     // batch scratch of the posterior stage
  // the posterior stage's synchronisation events, created once: a batch's
  // records on the host (by batch parity), the fork to stream2 and its join
  hipEvent_t ev_done[2] = {nullptr, nullptr}, ev_fork = nullptr, ev_tot = nullptr;
  size_t scratch_budget = 0;
  // relaxation buffers
  bool arena_on = false;               // relax_one: temporaries come from the batch scratch
  size_t arena_off = 0;
  DevBuf r_trowptr, r_tcols, r_tvals, r_raw, r_newrp, r_newcols, r_newvals, r_tasks_p, r_tasks_r,
      r_pairs, r_nnz, r_newoff, r_img, r_imgoff, r_tiles, r_nwords, r_weights, r_seldist, r_profile, r_mea;
  // comm
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  // in-process shards: child contexts, one per device of the mask (or
  // virtual shards sharing devices); empty = the single-device path
  uint64_t dev_mask = 0;
  int shards_req = 0;                // 0: one per device when the family is large enough
  std::vector<mlp_ctx*> shards;
  int64_t rel_r0 = -1, rel_r1 = -1;  // a shard's output-pair range for one relaxation round
  // all-gather (allgather_shards): the incoming store, copy streams (one per
  // source shard) and the parent store version every shard holds in full
  DevBuf ag_cols, ag_vals;
  std::vector<hipStream_t> cst;
  uint64_t shards_full_ver = ~0ull;
  // profiling
  bool profile = false;
  double kms[MLP_NKERNELS] = {0};
  int64_t klaunch[MLP_NKERNELS] = {0};
  int64_t kcells[MLP_NKERNELS] = {0};
  // deferred kernel timers: event pairs resolved by flush_timers()
  // e0 / e1 on the timed stream; e0b / e1b (optional) on the side stream, the
  // group's span then runs from the earlier start to the later end, measured
  // from eref (recorded on the context stream before both)
  // cont: a later part of the group's launch (time added, launch and cells counted once)
  struct TimerRec { int id; int64_t cells; bool cont; hipEvent_t e0, e1, e0b, e1b, eref; };
  std::vector<TimerRec> tpend;
  std::vector<hipEvent_t> evpool;
  size_t evused = 0;
};

#define HIPCHK(ctx, expr)                                                          \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) {                                                        \
      (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e_);              \
      return MLP_ERR_HIP;                                                          \
    }                                                                              \
  } while (0)

#define NCCLCHK(ctx, expr)                                                         \
  do {                                                                             \
    ncclResult_t r_ = (expr);                                                      \
    if (r_ != ncclSuccess) {                                                       \
      (ctx)->err = std::string(#expr) + ": " + ncclGetErrorString(r_);             \
      return MLP_ERR_COMM;                                                         \
    }                                                                              \
  } while (0)

// ---- the process's device memory pool (mlp_context.cpp): large buffers
// (batch scratch, CSR stores, relaxation and gather buffers) are carved from
// blocks the process keeps; a released buffer goes back to its block, not to
// the driver.  A fresh allocation right after a large release can wait
// seconds while the driver clears what was released,
// so contexts created one after another (the shards of a mask, a new family's
// context) reuse what the last one held.  Blocks go back to the driver only
// when an allocation fails or on mlp_pool_trim.
MLP_HIDDEN void* pool_alloc(int device, size_t bytes);   // nullptr on failure
MLP_HIDDEN void pool_free(int device, void* p);
MLP_HIDDEN size_t pool_free_bytes(int device);           // reusable bytes held
MLP_HIDDEN void pool_ctx_opened(int device);             // a device context's lifetime:
MLP_HIDDEN void pool_ctx_closed(int device);             // the last close shrinks the pool
// the error text for a failed pool_alloc: the request, the driver's error
// and what the device and the pool held at the time
MLP_HIDDEN std::string pool_failure(int device, size_t bytes);

// ---- device buffers, timers (mlp_context.cpp)
MLP_HIDDEN int ensure(mlp_ctx* c, DevBuf& b, size_t bytes);
MLP_HIDDEN int ensure_tmp(mlp_ctx* c, DevBuf& b, size_t bytes);
// the family's arrays, from the pool as well (a relaxation round swaps the
// row pointers with a pooled buffer)
template <class T>
inline int dalloc(mlp_ctx* c, T** p, size_t count) {
  pool_free(c->device, *p);
  *p = (T*)pool_alloc(c->device, std::max<size_t>(count, 1) * sizeof(T));
  if (!*p) {
    c->err = pool_failure(c->device, std::max<size_t>(count, 1) * sizeof(T));
    return MLP_ERR_MEMORY;
  }
  return MLP_OK;
}

MLP_HIDDEN hipEvent_t pool_event(mlp_ctx* c);
// Kernel-group timer: HIP events around the launches on `st`, resolved later
// (flush_timers), so timing never serialises the host with the device.  With
// a side stream (span()), the group's kernels on both streams: from the
// earlier start to the later end.
struct Timer {
  mlp_ctx* c;
  int id;
  int64_t cells;
  hipStream_t st;
  hipEvent_t e0 = nullptr;
  bool cont = false;  // continues the group's previous launch (TimerRec::cont)
  hipStream_t sb = nullptr;
  hipEvent_t e0b = nullptr, eref = nullptr;
  Timer(mlp_ctx* c_, int id_, int64_t cells_, hipStream_t st_ = nullptr)
      : c(c_), id(id_), cells(cells_), st(st_ ? st_ : c_->stream) {
    if (c->profile) {
      e0 = pool_event(c);
      hipEventRecord(e0, st);
    }
  }
  // the group also has kernels on stream b; start_b: they start after this
  // point in b's order (else they start after e0); ref: an event on the timed
  // stream before anything of the group on either stream
  void span(hipStream_t b, bool start_b, hipEvent_t ref) {
    if (!c->profile || !b) return;
    sb = b;
    eref = ref ? ref : e0;
    if (start_b) {
      e0b = pool_event(c);
      hipEventRecord(e0b, b);
    }
  }
  ~Timer() {
    if (!c->profile || !e0) return;
    hipEvent_t e1 = pool_event(c), e1b = nullptr;
    hipEventRecord(e1, st);
    if (sb) {
      e1b = pool_event(c);
      hipEventRecord(e1b, sb);
    }
    c->tpend.push_back({id, cells, cont, e0, e1, e0b, e1b, eref});
  }
};
MLP_HIDDEN void flush_timers(mlp_ctx* c);

// parameter tables exactly as the reference builds them
MLP_HIDDEN void build_tables(Tables& T, ModelScalars& ms, float delta, bool qp = false);

static inline int64_t pair_index_host(int n, int a, int b) {  // a < b, row-major
  return (int64_t)a * n - (int64_t)a * (a + 1) / 2 + (b - a - 1);
}

static int pair_cost_cells(const mlp_ctx* c, int64_t p) {
  return (c->lens[c->pa[p]] + 1) * (c->lens[c->pb[p]] + 1);
}

// grow the entry store to hold `need` entries, keeping `keep` existing ones
MLP_HIDDEN int grow_store(mlp_ctx* c, int64_t need, int64_t keep, int64_t want = 0, bool sync2 = true);

// ---- batch planning (mlp_planner.cpp)
// Equal-sized batches of a pair range under the scratch budget, given an
// upper bound of one pair's scratch bytes.
template <class F>
inline size_t batch_target_for(mlp_ctx* c, int64_t p0, int64_t p1, F pair_bytes, size_t budget = 0) {
  if (!budget) budget = c->scratch_budget;
  size_t all = 0, biggest = 0;
  for (int64_t q = p0; q < p1; q++) {
    const size_t b = pair_bytes(q);
    all += b;
    biggest = std::max(biggest, b);
  }
  const size_t nb = (all + budget - 1) / std::max<size_t>(budget, 1);
  // a batch stops before the pair that would pass the target, so each holds
  // more than all / nb - biggest: nb batches of near-equal bytes
  if (nb > 1) return std::min(budget, all / nb + biggest);
  return budget;
}
template <class F>
inline int next_batch(mlp_ctx* c, int64_t p, int64_t p1, size_t target, F pair_bytes, int64_t* q_out) {
  int64_t q = p;
  size_t bytes = 0;
  while (q < p1) {
    const size_t add = pair_bytes(q);
    if (q > p && bytes + add > target) break;
    if (chain_seq_bytes(chain_width(c->lens[c->pb[q]]), c->lens[c->pa[q]], 1) > kChainSeqMax) {
      c->err = "pair " + std::to_string(q) + ": sequences too long for the LDS residue staging";
      return MLP_ERR_ARG;
    }
    bytes += add;
    ++q;
  }
  *q_out = q;
  return MLP_OK;
}

// Chains of one batch (mlp_kernels.h, "Chains"): pairs sorted by column
// count, stacked greedily; slots ordered chain by chain, chains longest first.
struct ChainPlan {
  int64_t np = 0, nch = 0;
  std::vector<int64_t> order;                       // slot -> pair
  std::vector<int32_t> pa, pb, row0, chain;         // per slot
  std::vector<int64_t> rm, ell;                     // per slot
  std::vector<int32_t> first, count, width, rows, seqb;  // per chain
  std::vector<int64_t> cell, bndo;                  // per chain
  int64_t cells = 0, rm_total = 0, bnd = 0, ell_rows = 0;
  int lds_seq = 0;   // chain_lds_pack(max residue bytes, max members)
};
MLP_HIDDEN void plan_chains(const mlp_ctx* c, int64_t p, int64_t q, ChainPlan& P);

// Scratch carving: 256-byte aligned sub-buffers of one device allocation.
struct Carver {
  size_t off = 0;
  size_t take(size_t b) {
    const size_t o = off;
    off += (b + 255) & ~(size_t)255;
    return o;
  }
};

// Upload the plan's per-slot / per-chain metadata; returns device views.
struct PlanDev {
  size_t o_pa, o_pb, o_r0, o_ch, o_rm, o_ell, o_cf, o_cc, o_cw, o_cr, o_cs, o_cco, o_cbo;
};
MLP_HIDDEN PlanDev carve_plan(Carver& cv, const ChainPlan& P);
MLP_HIDDEN int upload_plan(mlp_ctx* c, char* base, const PlanDev& d, const ChainPlan& P, PairMeta& pm, ChainMeta& cm,
                hipStream_t st = nullptr, uint8_t* stage = nullptr);
// upper bounds of one pair's step-diagonal slots / chain width (as if alone in a chain whose
// width may exceed its own by the stacking slack)
MLP_HIDDEN int64_t pair_slots_bound(const mlp_ctx* c, int64_t q);
MLP_HIDDEN int64_t pair_width_bound(const mlp_ctx* c, int64_t q);
constexpr size_t kPerSlotMeta = 4 * sizeof(int64_t) + 4 * sizeof(int32_t) + sizeof(PairRec) + 7 * 8 + 16;

// ---- in-process shards (mlp_shards.cpp)
MLP_HIDDEN std::vector<int> mask_devices(uint64_t mask);
MLP_HIDDEN int shard_count(mlp_ctx* c);
MLP_HIDDEN int ensure_shards(mlp_ctx* c, int S);
// run fn(shard, index) on every shard, one host thread each
template <class F>
inline int run_shards(mlp_ctx* c, F fn) {
  const int S = (int)c->shards.size();
  std::vector<int> rcs(S, MLP_OK);
  std::vector<std::thread> th;
  for (int s = 0; s < S; s++)
    th.emplace_back([&, s]() {
      hipSetDevice(c->shards[s]->device);
      rcs[s] = fn(c->shards[s], s);
    });
  for (auto& t : th) t.join();
  hipSetDevice(c->device);
  for (int s = 0; s < S; s++)
    if (rcs[s] != MLP_OK) {
      c->err = "shard " + std::to_string(s) + ": " + c->shards[s]->err;
      return rcs[s];
    }
  return MLP_OK;
}
MLP_HIDDEN int broadcast_store(mlp_ctx* c, mlp_ctx* ch);
MLP_HIDDEN int allgather_shards(mlp_ctx* c);

// ---- the host context (mlp_ctx_create_host): host_backend.cpp
static mlph::FamilyView host_view(const mlp_ctx* c) {
  return mlph::FamilyView{c->n, c->lens.data(), c->offs.data(), c->h_res.data(), c->pa.data(), c->pb.data()};
}
