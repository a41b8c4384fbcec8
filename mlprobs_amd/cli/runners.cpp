// runners.cpp -- see runners.h.  The bodies of the two drop-in CLIs after
// argument parsing and input reading, moved here from c_p_np_aln.cpp and
// quickprobs.cpp so the pipeline driver can call them in-process.
#include "runners.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <iostream>
#include <memory>
#include <stdexcept>
#include <thread>

namespace mlpr {

namespace {

struct RunError : std::runtime_error {
  int status;
  RunError(int s, const std::string& m) : std::runtime_error(m), status(s) {}
};

void check(mlp_ctx* ctx, int rc, const char* what, int status) {
  if (rc != MLP_OK) throw RunError(status, std::string("ERROR: ") + what + ": " + (ctx ? mlp_last_error(ctx) : "no context"));
}

// Device 0 by default.  MLP_DEVICES=<mask> (bit k = HIP device k, e.g. 0xff)
// opts in to one context over several GPUs, which shards families of >= 1e9
// pair-cells over them (mlp_ctx_create_mask); that path is verified with
// virtual shards on one GPU only, so it is not the default.
int open_device(mlp_ctx** ctx) {
  if (const char* m = getenv("MLP_DEVICES")) {
    const unsigned long long mask = strtoull(m, nullptr, 0);
    if (mask) return mlp_ctx_create_mask(mask, ctx);
  }
  return mlp_ctx_create(0, ctx);
}

// the batch scratch of the drop-ins' device contexts (one family per process)
constexpr size_t kDefaultScratch = 16ull << 30;

// The context one run uses: a fresh host context for a small family, else
// the session's device context (or a fresh one without a session).
struct Ctx {
  mlp_ctx* c = nullptr;
  bool owned = false;
  ~Ctx() {
    if (owned && c) mlp_ctx_destroy(c);
  }
  void open(Session* s, double cells, size_t default_scratch, int status) {
    const double host_max = s ? s->host_max() : Session().host_max();
    if (cells <= host_max) {
      if (s) s->host_runs++;
      check(nullptr, mlp_ctx_create_host(&c), "host context", status);
      owned = true;
      stage("host context");
      return;
    }
    if (s) s->device_runs++;
    if (s) s->ready();
    if (s && s->dev) {
      c = s->dev;
      return;
    }
    check(nullptr, open_device(&c), "device", status);
    stage("device init");
    // one family per process: a moderate batch scratch.  Right after a
    // process that held a lot of device memory exits, a fresh process can
    // take ~40 GB at once; the allocation that goes past that stalls ~5.7 s
    // (once, whatever its size or chunking: tools/probe/alloc_seq.sh,
    // tools/ab_r03.sh chunks; profiles/r03d_*)
    const size_t scratch = s && s->scratch_bytes ? s->scratch_bytes : default_scratch;
    if (!getenv("MLP_SCRATCH_GB")) check(c, mlp_set_scratch(c, scratch), "device", status);
    if (s) s->dev = c;
    else owned = true;
  }
};

}  // namespace

Session::~Session() {
  ready();
  if (dev) mlp_ctx_destroy(dev);
}

void Session::prewarm() {
  if (dev || warm.joinable()) return;
  const size_t scratch = scratch_bytes ? scratch_bytes : kDefaultScratch;
  warm = std::thread([this, scratch]() {
    mlp_ctx* c = nullptr;
    if (open_device(&c) != MLP_OK) {
      if (c) mlp_ctx_destroy(c);
      return;   // the first device run opens (and reports) it again
    }
    if (!getenv("MLP_SCRATCH_GB")) mlp_set_scratch(c, scratch);
    dev = c;
  });
}

void Session::ready() {
  if (warm.joinable()) {
    warm.join();
    stage("device init (prewarmed)");
  }
}

double Session::host_max() const {
  if (host_max_cells >= 0) return host_max_cells;
  return getenv("MLP_HOST_MAX_CELLS") ? atof(getenv("MLP_HOST_MAX_CELLS")) : 4e6;
}

double pair_cells(const std::vector<int>& lens) {
  double c = 0;
  for (size_t a = 0; a < lens.size(); a++)
    for (size_t b = a + 1; b < lens.size(); b++) c += (double)(lens[a] + 1) * (double)(lens[b] + 1);
  return c;
}

void stage(const char* name) {
  static const bool on = getenv("MLP_CLI_TIMES") != nullptr;
  static auto t0 = std::chrono::steady_clock::now();
  if (!on) return;
  if (!name) {  // first call, from main: time since the process started (loader, static init)
    double up = 0, start = 0;
    if (FILE* f = fopen("/proc/uptime", "r")) { if (fscanf(f, "%lf", &up) != 1) up = 0; fclose(f); }
    if (FILE* f = fopen("/proc/self/stat", "r")) {
      char buf[1024];
      const size_t n = fread(buf, 1, sizeof buf - 1, f);
      fclose(f);
      buf[n] = 0;
      const char* q = strrchr(buf, ')');  // fields after the command name; starttime is field 22
      for (int k = 2; q && k < 22; k++) q = strchr(q + 1, ' ');
      if (q) start = strtod(q + 1, nullptr) / (double)sysconf(_SC_CLK_TCK);
    }
    std::cerr << "[stage] process start to main " << (up - start) << " s" << std::endl;
    t0 = std::chrono::steady_clock::now();
    return;
  }
  const auto t1 = std::chrono::steady_clock::now();
  std::cerr << "[stage] " << name << " " << std::chrono::duration<double>(t1 - t0).count() << " s" << std::endl;
  t0 = t1;
}

// ---------------------------------------------------------------- c_p_np_aln
// Profile MEAs of at least this many cells run on the device (both
// drop-ins), smaller ones on the host's SIMD lanes, where a device round trip
// costs more than the recurrence.  Floors 0 / 1e5 / 2.5e5 / 5e5 / never:
// C2 -p 0 progressive 0.37 / 0.39 / 0.13 / 0.13 / 0.13 s, C2 -p 1 refinement
// 0.62 / 0.58 / 0.55 / 0.58 / 0.80 s, QuickProbs C3 construction +
// refinement 1.62 / 1.62 / 1.63 / 1.70 / 2.04 s, every output identical
// (tools/ab_r03.sh meamin, profiles/r03f_ab_meamin.txt).  MLP_MEA_GPU_MIN
// overrides.  Round 5 (device MEA rebuilt, deferred matrices no longer
// pinned on the host), floors 2.5e5 / 5e4 / 0: C2 -p 0 progressive 0.14-0.30
// / 0.28-0.32 / 0.28-0.33 s, C2 -p 1 refinement 0.22-0.25 / 0.24-0.25 /
// 0.25-0.26 s, every output the reference's (profiles/r05x_cpnp_mea_floor.txt).
// QuickProbs' floor is lower: its device path keeps the posterior on the
// device and returns only the path, and since round 5's device MEA (about
// twice as fast) QuickProbs C3 construction + refinement runs 0.90-0.97 s at
// 2.5e5, 0.84-0.87 at 1e5, 0.81-0.84 at 5e4 and 0 (C2: 0.063-0.068 / 0.062
// / 0.057 / 0.058), outputs identical (profiles/r05v_qp_mea_floor.txt).
static int64_t mea_gpu_min(int64_t dflt = 250000) {
  static const char* e = getenv("MLP_MEA_GPU_MIN");
  return e ? atoll(e) : dflt;
}
constexpr int64_t kQpMeaGpuMin = 50000;

using cpnp::Row;

int run_cpnp(std::vector<Row> seqs, bool just_features, bool progressive, cpnp::Options opt, Session* session,
             std::string& out, std::string& err) {
  out.clear();
  err.clear();
  if (seqs.empty()) {
    err = "ERROR: No sequences read.";
    return 1;
  }
  const int n = (int)seqs.size();
  // a fresh process's rand() state (glibc seed 1): refinement of -p 0 draws
  // from it without seeding (CPNP/MSA.cpp:1545)
  cpnp::libc_srand(1);
  try {
    Ctx cx;
    stage("parse");
    // Small families run on the host (mlp_ctx_create_host: the same stages,
    // bit for bit, without initialising the GPU runtime, whose start-up and
    // teardown alone cost 0.2-0.4 s per process); at ~2e7 pair-cells/s on the
    // host threads, families up to MLP_HOST_MAX_CELLS pair-cells (default 4e6,
    // 0: always the GPU) finish there before a device would be ready.
    std::vector<int> lens;
    for (const Row& r : seqs) lens.push_back(r.length());
    // one family per process: a 16 GB batch scratch, like quickprobs (C3
    // -p 0 back to back after a large process: 3.1-3.3 s every run at 16 GB;
    // at 24 / 32 GB 3 of 4 and 2 of 4 runs stalled 4-6 s; profiles/r03d_*)
    cx.open(session, pair_cells(lens), kDefaultScratch, 1);
    mlp_ctx* ctx = cx.c;
    std::string res;
    std::vector<int64_t> off(1, 0);
    for (const Row& r : seqs) {
      res.append(r.data, 1, std::string::npos);
      off.push_back((int64_t)res.size());
    }
    check(ctx, mlp_family_load(ctx, n, res.data(), off.data()), "family", 1);
    stage("load");

    if (just_features) {   // CPNP/MSA.cpp:153-166 (theta = 1.0)
      float f[5];
      int32_t ints[2];
      check(ctx, mlp_family_features(ctx, 1.0f, f, ints), "family test", 1);
      char line[512];
      snprintf(line, sizeof line, "%f\t%f\t%d\t%d\t%f\t%f\t%f\n", f[0], f[1], ints[0], ints[1], f[2], f[3], f[4]);
      out = line;
      return 0;
    }
    cpnp::Profile aln;
    if (n == 1) {
      aln.push_back(seqs[0]);
    } else {
      // ModelAdjustmentTest (CPNP/MSA.cpp:775-882) -> pid, delta
      float identity, variance, delta;
      int32_t code;
      check(ctx, mlp_model_adjustment(ctx, &identity, &variance, &delta, &code), "family test", 1);
      stage("family test (Viterbi)");
      const int pid = code % 10, vpid = code / 10;
      // pdoAlign (CPNP/MSA.cpp:895-1081): posteriors, distances, tree, consistency;
      // npdoAlign (CPNP/MSA.cpp:1084-1140): ArrangePosteriorProbs' pair body,
      // consistency, alignment graph, refinement
      const int64_t P = mlp_family_npairs(ctx);
      check(ctx, mlp_posteriors(ctx, progressive ? pid : pid | MLP_PID_NPDO, delta, 0, P), "posteriors", 1);
      std::vector<float> dist(P);
      check(ctx, mlp_pair_results(ctx, 0, P, dist.data(), nullptr, nullptr), "results", 1);
      std::vector<std::vector<float>> D(n, std::vector<float>(n, 0.f));
      for (int a = 0, p = 0; a < n; a++)
        for (int b = a + 1; b < n; b++, p++) D[a][b] = D[b][a] = dist[p];
      stage("posteriors");
      cpnp::GuideTree tree;
      if (progressive) {
        tree = cpnp::build_tree(D, vpid);
        stage("guide tree");
      }
      if (opt.consistency > 0) check(ctx, mlp_relax(ctx, opt.consistency), "consistency", 1);
      check(ctx, mlp_synchronize(ctx), "consistency", 1);
      stage("consistency");
      cpnp::SparseSet sp;
      sp.n = n;
      sp.lens.resize(n);
      for (int k = 0; k < n; k++) sp.lens[k] = seqs[k].length();
      sp.rp_off.assign(P + 1, 0);
      for (int a = 0, p = 0; a < n; a++)
        for (int b = a + 1; b < n; b++, p++) sp.rp_off[p + 1] = sp.rp_off[p] + sp.lens[a] + 2;
      int64_t total = 0;
      check(ctx, mlp_csr_total(ctx, &total), "sparse set", 1);
      sp.row_ptr.resize(sp.rp_off[P]);
      sp.ent_off.resize(P + 1);
      sp.cols.resize(std::max<int64_t>(total, 1));
      sp.vals.resize(std::max<int64_t>(total, 1));
      check(ctx, mlp_csr_export(ctx, sp.row_ptr.data(), sp.ent_off.data(), sp.cols.data(), sp.vals.data()),
            "sparse set", 1);
      stage("sparse set to host");
      // BuildPosterior of the merges and refinement passes on the GPU
      // (mlp_profile_posterior_cpnp) once the profile pair holds enough sparse
      // entries to pay for a device round trip (~0.1-0.2 ms; the host adds
      // ~5e4 entries in that time); the sparse set stays resident.  After
      // consistency a divergent family's set is nearly empty (C2: 5e4 entries
      // over 8128 pairs), a similar family's is not.
      static const int64_t gpu_min = getenv("MLP_PROFILE_GPU_MIN") ? atoll(getenv("MLP_PROFILE_GPU_MIN")) : 100000;
      std::vector<int32_t> lab1, lab2, map1, map2;
      auto fill = [](const cpnp::Profile& p, std::vector<int32_t>& lab, std::vector<int32_t>& map) {
        lab.clear();
        map.clear();
        for (const Row& r : p) {   // Sequence::GetMapping: 0, then the column of each residue
          lab.push_back(r.label);
          map.push_back(0);
          for (int c = 1; c <= r.length(); c++)
            if (r.data[c] != '-') map.push_back(c);
        }
      };
      cpnp::set_profile_backend([&](const cpnp::Profile& a, const cpnp::Profile& b, const int* w) -> const float* {
        if (mlp_ctx_is_host(ctx)) return nullptr;
        int64_t entries = 0;
        for (const Row& x : a)
          for (const Row& y : b) {
            const int64_t p = sp.pair(std::min(x.label, y.label), std::max(x.label, y.label));
            entries += sp.ent_off[p + 1] - sp.ent_off[p];
          }
        if (entries < gpu_min) return nullptr;
        fill(a, lab1, map1);
        fill(b, lab2, map2);
        const int rc = mlp_profile_posterior_cpnp(ctx, w, (int)a.size(), lab1.data(), a[0].length(), map1.data(),
                                                  (int)b.size(), lab2.data(), b[0].length(), map2.data(), nullptr);
        if (rc == MLP_ERR_STATE) return nullptr;   // a profile wider than an LDS row: the host computes it
        check(ctx, rc, "profile posterior", 1);
        return mlp_profile_result(ctx);
      });
      // Profile posterior and MEA both on the device (mlp_profile_mea): only
      // the path (and the few cells a refinement scores) come back.  By
      // default every MEA of a device context runs there (C2 -p 1 refinement
      // 0.66 s against 0.93 s with the host MEA, outputs identical;
      // tools/ab_r03.sh cpnpmea); MLP_MEA_GPU_MIN sets a cell floor below
      // which the host computes it.
      const int64_t mea_min = mea_gpu_min();
      cpnp::set_mea_backend([&](const cpnp::Profile& a, const cpnp::Profile& b, const int* w,
                                const std::vector<int64_t>* cells, std::vector<float>* vals, std::string& path,
                                float* score) -> bool {
        if (mlp_ctx_is_host(ctx) || mea_min == INT64_MAX) return false;
        const int L1 = a[0].length(), L2 = b[0].length();
        if ((int64_t)L1 * L2 < mea_min) return false;
        fill(a, lab1, map1);
        fill(b, lab2, map2);
        check(ctx, mlp_profile_defer(ctx, 1), "profile posterior", 1);
        const int rc = mlp_profile_posterior_cpnp(ctx, w, (int)a.size(), lab1.data(), L1, map1.data(), (int)b.size(),
                                                  lab2.data(), L2, map2.data(), nullptr);
        if (rc == MLP_ERR_STATE) {   // a profile wider than an LDS row: the host computes it
          check(ctx, mlp_profile_defer(ctx, 0), "profile posterior", 1);
          return false;
        }
        check(ctx, rc, "profile posterior", 1);
        if (cells && !cells->empty())
          check(ctx, mlp_profile_gather(ctx, (int64_t)cells->size(), cells->data(), vals->data()),
                "profile posterior", 1);
        path.resize((size_t)L1 + L2);
        int32_t np = 0;
        const int mrc = mlp_profile_mea(ctx, &path[0], &np, score);
        if (mrc == MLP_ERR_STATE) {   // the device pipeline gave up: the host MEA
          check(ctx, mlp_profile_defer(ctx, 0), "profile posterior", 1);
          return false;
        }
        check(ctx, mrc, "MEA", 1);
        path.resize(np);
        check(ctx, mlp_profile_defer(ctx, 0), "profile posterior", 1);
        return true;
      });
      struct Unset {  // the backends capture this frame: clear them on every exit
        ~Unset() {
          cpnp::set_profile_backend(nullptr);
          cpnp::set_mea_backend(nullptr);
        }
      } unset;
      if (progressive) {
        aln = cpnp::progressive_alignment(seqs, sp, tree, pid, opt);
        stage("progressive + refinement");
      } else {
        aln = cpnp::graph_alignment(seqs, sp);
        stage("alignment graph");
        aln = cpnp::np_refinement(std::move(aln), sp, D, opt);
        stage("refinement");
      }
    }
    if (getenv("MLP_CLI_TIMES")) {
      double tp, tm;
      int64_t nc, nd;
      cpnp::profile_times(&tp, &tm, &nc, &nd);
      fprintf(stderr, "[host] profile posteriors %.3f s (%lld calls, %lld on the GPU), MEA %.3f s\n", tp,
              (long long)nc, (long long)nd, tm);
    }
    cpnp::write_mfa(out, aln);
    stage("alignment");
  } catch (const RunError& e) {
    err = e.what();
    return e.status;
  } catch (const std::exception& e) {   // the reference's own abort paths (e.g. the cluster tree's OOPS)
    err = e.what();
    return 255;
  }
  stage("context teardown");
  return 0;
}

// ---------------------------------------------------------------- quickprobs
int run_qp(std::vector<qph::Seq> seqs, const qph::Options& opt, int threads, Session* session, std::string& out,
           std::string& err) {
  out.clear();
  err.clear();
  if (threads <= 0) threads = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  const int n = (int)seqs.size();
  qph::Profile aln;
  try {
    if (n == 1) {
      aln.push_back(seqs[0]);
    } else {
      Ctx cx;
      stage("parse");
      // Small families (MLProbs realigns one column region per call) run on
      // the host context: the same stages bit for bit on host threads, no
      // HIP runtime start-up (0.14-0.22 s per process); above
      // MLP_HOST_MAX_CELLS pair-cells (default 4e6, 0: always the GPU) the GPU.
      std::vector<int> lens;
      for (const qph::Seq& s : seqs) lens.push_back(s.length());
      // one family per process: a 16 GB batch scratch (C3 posteriors 0.82 s
      // at 16 GB vs 6.9-7.2 s at 64 GB in a fresh process, 1.16 s at 8 GB)
      cx.open(session, pair_cells(lens), kDefaultScratch, 255);
      mlp_ctx* ctx = cx.c;
      std::string res;
      std::vector<int64_t> off(1, 0);
      for (const qph::Seq& s : seqs) {
        res.append(s.data, 1, std::string::npos);
        off.push_back((int64_t)res.size());
      }
      check(ctx, mlp_family_load(ctx, n, res.data(), off.data()), "family", 255);
      // PosteriorStage::run (QP/Alignment/Multiple/PosteriorStage.cpp:58-117)
      const int64_t P = mlp_family_npairs(ctx);
      check(ctx, mlp_posteriors(ctx, MLP_PID_QP, 0.f, 0, P), "posteriors", 255);
      std::vector<float> dist(P);
      check(ctx, mlp_pair_results(ctx, 0, P, dist.data(), nullptr, nullptr), "results", 255);
      std::vector<float> D((size_t)n * n, 0.f);
      for (int a = 0, p = 0; a < n; a++)
        for (int b = a + 1; b < n; b++, p++) D[(size_t)a * n + b] = D[(size_t)b * n + a] = dist[p];
      stage("posteriors");
      // ClusterTree (UPGMA) and its weights; subtree sizes for the selectivity
      // (ExtendedMSA.cpp:86-100, 176)
      const qph::Tree tree = qph::build_tree(D, n);
      const std::vector<float> seld = tree.subtree_distances();
      std::vector<float> wc = tree.weights;
      for (float& w : wc) w = std::max(w, 1e-6f);  // consistency.saturation
      stage("guide tree");
      if (opt.consistency != 0)
        check(ctx, mlp_relax_qp_selective(ctx, opt.consistency, wc.data(), seld.data(), 200.f), "consistency", 255);
      check(ctx, mlp_synchronize(ctx), "consistency", 255);
      stage("consistency");
      // construction + refinement: profile posteriors on the GPU from the
      // device-resident sparse set; the host copy of the set is fetched only
      // if a profile is too wide for the kernel's LDS row (or on a host context)
      std::unique_ptr<qph::Sparse> host_sp;
      qph::PosteriorBackend be;
      be.device = [&](const std::vector<float>& w, const qph::Profile& A, const qph::Profile& B) -> const float* {
        if (mlp_ctx_is_host(ctx)) return nullptr;
        const int L1 = A[0].length(), L2 = B[0].length();
        std::vector<int32_t> l1, l2;
        for (const qph::Seq& q : A) l1.push_back(q.label);
        for (const qph::Seq& q : B) l2.push_back(q.label);
        const std::vector<int32_t> m1 = qph::profile_maps(A, threads), m2 = qph::profile_maps(B, threads);
        // out = NULL: the matrix stays in the library's pinned buffer
        const int rc = mlp_profile_posterior(ctx, w.data(), (int)A.size(), l1.data(), L1, m1.data(), (int)B.size(),
                                             l2.data(), L2, m2.data(), nullptr);
        if (rc == MLP_ERR_STATE) return nullptr;  // too wide: the host restatement
        check(ctx, rc, "profile posterior", 255);
        return mlp_profile_result(ctx);
      };
      // posterior and MEA both on the device, only the path comes back
      // (k_profile_mea, strips pipelined across CUs): at C3 construction +
      // refinement 1.72 s against 2.18-2.22 s with the host MEA, outputs
      // identical (tools/ab_r03.sh mea); MLP_MEA_DEVICE=0 keeps the MEA on
      // the host
      double t_maps = 0;
      const char* mea_dev = getenv("MLP_MEA_DEVICE");
      if ((!mea_dev || atoi(mea_dev) > 0) && !mlp_ctx_is_host(ctx)) {
        be.device_mea = [&](const std::vector<float>& w, const qph::Profile& A, const qph::Profile& B,
                            std::string& path, float* score) -> bool {
          const int L1 = A[0].length(), L2 = B[0].length();
          if ((int64_t)L1 * L2 < mea_gpu_min(kQpMeaGpuMin)) return false;
          const auto tm0 = std::chrono::steady_clock::now();
          std::vector<int32_t> l1, l2;
          for (const qph::Seq& q : A) l1.push_back(q.label);
          for (const qph::Seq& q : B) l2.push_back(q.label);
          const std::vector<int32_t> m1 = qph::profile_maps(A, threads), m2 = qph::profile_maps(B, threads);
          t_maps += std::chrono::duration<double>(std::chrono::steady_clock::now() - tm0).count();
          check(ctx, mlp_profile_defer(ctx, 1), "profile posterior", 255);
          const int rc = mlp_profile_posterior(ctx, w.data(), (int)A.size(), l1.data(), L1, m1.data(), (int)B.size(),
                                               l2.data(), L2, m2.data(), nullptr);
          if (rc == MLP_ERR_STATE) {  // too wide: the host restatement
            check(ctx, mlp_profile_defer(ctx, 0), "profile posterior", 255);
            return false;
          }
          check(ctx, rc, "profile posterior", 255);
          path.resize((size_t)L1 + L2);
          int32_t np = 0;
          const int mrc = mlp_profile_mea(ctx, &path[0], &np, score);
          if (mrc == MLP_ERR_STATE) {  // the device pipeline gave up: the host MEA
            check(ctx, mlp_profile_defer(ctx, 0), "profile posterior", 255);
            return false;
          }
          check(ctx, mrc, "MEA", 255);
          path.resize(np);
          check(ctx, mlp_profile_defer(ctx, 0), "profile posterior", 255);
          return true;
        };
      }
      be.host_sparse = [&]() -> const qph::Sparse& {
        if (!host_sp) {
          host_sp.reset(new qph::Sparse());
          qph::Sparse& sp = *host_sp;
          sp.n = n;
          sp.lens.resize(n);
          for (int k = 0; k < n; k++) sp.lens[k] = seqs[k].length();
          sp.rp_off.assign(P + 1, 0);
          for (int a = 0, p = 0; a < n; a++)
            for (int b = a + 1; b < n; b++, p++) sp.rp_off[p + 1] = sp.rp_off[p] + sp.lens[a] + 2;
          int64_t total = 0;
          check(ctx, mlp_csr_total(ctx, &total), "sparse set", 255);
          sp.row_ptr.resize(sp.rp_off[P]);
          sp.ent_off.resize(P + 1);
          sp.cols.resize(std::max<int64_t>(total, 1));
          sp.vals.resize(std::max<int64_t>(total, 1));
          check(ctx, mlp_csr_export(ctx, sp.row_ptr.data(), sp.ent_off.data(), sp.cols.data(), sp.vals.data()),
                "sparse set", 255);
          sp.build_views();
        }
        return *host_sp;
      };
      aln = qph::construct_and_refine(seqs, be, tree, opt, threads);
      stage("construction + refinement");
      if (getenv("MLP_CLI_TIMES")) fprintf(stderr, "[host] device MEA calls: labels and residue maps %.3f s\n", t_maps);
    }
  } catch (const RunError& e) {
    err = e.what();
    return e.status;
  } catch (const std::runtime_error& e) {
    err = e.what();
    return 255;
  }
  qph::write_fasta(out, aln);
  return 0;
}

}  // namespace mlpr
