// c_p_np_aln -- drop-in for kuangmeng/MLProbs' baseMSA/C_P_NP_Aln/c_p_np_aln
// with the all-pairs stages on the GPU (libmlpgpu, include/mlpgpu.h).
//
// Argument grammar and exit behaviour follow MSA::ParseParams
// (CPNP/MSA.cpp:248-435): unknown options, bad values, -help and -version
// print to stderr and exit(1); success is silent on stderr, exit 0.
//   -G            the family-test feature line (Alter_ModelAdjustmentTest)
//   -p 0          progressive alignment (pdoAlign, CPNP/MSA.cpp:895-1081)
//   -p 1          non-progressive alignment (npdoAlign, CPNP/MSA.cpp:1084-1140):
//                 alignment graph + similarity-set refinement (np_host.cpp)
//   -c N, -ir N, -co F, -o FILE, -a, -v, -annot FILE, -clustalw, -timeon/-timeoff
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <chrono>
#include <iostream>
#include <string>
#include <vector>

#include "mlpgpu.h"
#include "msa_host.h"

using cpnp::Row;

static const char* kVersion = "2.0";   // printed like the reference's "PNPProbs version"

static void usage() {
  std::cerr << "c_p_np_aln (MI355X build)\n\n"
               "Usage:\n\tc_p_np_aln [OPTION]... [infile]...\n\n"
               "Options:\n"
               "\t-p, --program <0|1>\t0 progressive (default), 1 non-progressive\n"
               "\t-G, --getPID\tprint the family-test features and exit\n"
               "\t-c, --consistency REPS\t0..5 (default 2)\n"
               "\t-ir, --iterative-refinement REPS\t0..1000 (default 100)\n"
               "\t-co, --cutoff CUT\t0..1 (default 0)\n"
               "\t-o, --outfile FILE\twrite the alignment to FILE\n"
               "\t-a, --alignment-order\tkeep the alignment order\n"
               "\t-v, --verbose\n"
               "\t-annot FILE, -clustalw, -timeon, -timeoff\t(accepted)\n"
               "\t-version, -help\n";
}

static bool get_int(const char* s, int* v) {   // MSA::GetInteger (CPNP/MSA.cpp:2093-2116)
  if (!s) return false;
  char* end;
  const long r = strtol(s, &end, 10);
  if (end == s || *end) return false;
  *v = (int)r;
  return true;
}
static bool get_float(const char* s, float* v) {   // MSA::GetFloat (CPNP/MSA.cpp:2118-2140)
  if (!s) return false;
  char* end;
  const double r = strtod(s, &end);
  if (end == s || *end) return false;
  *v = (float)r;
  return true;
}

// MLP_CLI_TIMES=1 prints stage times to stderr (off by default: the
// reference is silent on stderr on success).
static void stage(const char* name) {
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
    return;
  }
  const auto t1 = std::chrono::steady_clock::now();
  std::cerr << "[stage] " << name << " " << std::chrono::duration<double>(t1 - t0).count() << " s" << std::endl;
  t0 = t1;
}

[[noreturn]] static void fail(const std::string& msg) {
  std::cerr << msg << std::endl;
  exit(1);
}

static void check(mlp_ctx* ctx, int rc, const char* what) {
  if (rc != MLP_OK) fail(std::string("ERROR: ") + what + ": " + (ctx ? mlp_last_error(ctx) : "no context"));
}

// Device 0 by default.  MLP_DEVICES=<mask> (bit k = HIP device k, e.g. 0xff)
// opts in to one context over several GPUs, which shards families of >= 1e9
// pair-cells over them (mlp_ctx_create_mask); that path is verified with
// virtual shards on one GPU only, so it is not the default.
static int open_device(mlp_ctx** ctx) {
  if (const char* m = getenv("MLP_DEVICES")) {
    const unsigned long long mask = strtoull(m, nullptr, 0);
    if (mask) return mlp_ctx_create_mask(mask, ctx);
  }
  return mlp_ctx_create(0, ctx);
}

int main(int argc, char** argv) {
  stage(nullptr);  // start the stage clock
  if (argc < 2) {
    usage();
    return 1;
  }
  std::vector<std::string> files;
  std::string outname;
  bool progressive = true, just_features = false;
  cpnp::Options opt;
  for (int i = 1; i < argc; i++) {
    const char* a = argv[i];
    if (a[0] != '-') {
      files.push_back(a);
      continue;
    }
    int iv;
    float fv;
    if (!strcmp(a, "-help") || !strcmp(a, "-?")) {
      usage();
      return 1;
    } else if (!strcmp(a, "-o") || !strcmp(a, "--outfile")) {
      if (i < argc - 1) outname = argv[++i];
      else fail(std::string("ERROR: String expected for option ") + a);
    } else if (!strcmp(a, "-p") || !strcmp(a, "--program")) {
      const char* v = i + 1 < argc ? argv[++i] : nullptr;
      if (!get_int(v, &iv)) fail(std::string("ERROR: Invalid integer following option ") + a + ": " + (v ? v : ""));
      if (iv > 1 || iv < 0) fail(std::string("ERROR: For option ") + a + ", integer must be 0 or 1.");
      progressive = iv == 0;
    } else if (!strcmp(a, "-G") || !strcmp(a, "--getPID")) {
      just_features = true;
    } else if (!strcmp(a, "-c") || !strcmp(a, "--consistency")) {
      if (i >= argc - 1) fail(std::string("ERROR: Integer expected for option ") + a);
      if (!get_int(argv[++i], &iv)) fail(std::string("ERROR: Invalid integer following option ") + a + ": " + argv[i]);
      if (iv < 0 || iv > 5) fail(std::string("ERROR: For option ") + a + ", integer must be between 0 and 5.");
      opt.consistency = iv;
    } else if (!strcmp(a, "-ir") || !strcmp(a, "--iterative-refinement")) {
      if (i >= argc - 1) fail(std::string("ERROR: Integer expected for option ") + a);
      if (!get_int(argv[++i], &iv)) fail(std::string("ERROR: Invalid integer following option ") + a + ": " + argv[i]);
      if (iv < 0 || iv > 1000) fail(std::string("ERROR: For option ") + a + ", integer must be between 0 and 1000.");
      opt.refinement = iv;
    } else if (!strcmp(a, "-annot")) {
      if (i >= argc - 1) fail(std::string("ERROR: FILENAME expected for option ") + a);
      ++i;   // annotation output is not produced by this build
    } else if (!strcmp(a, "-clustalw") || !strcmp(a, "-timeoff") || !strcmp(a, "-timeon")) {
      // accepted; no effect on the MFA output
    } else if (!strcmp(a, "-co") || !strcmp(a, "--cutoff")) {
      if (i >= argc - 1) fail(std::string("ERROR: Floating-point value expected for option ") + a);
      if (!get_float(argv[++i], &fv))
        fail(std::string("ERROR: Invalid floating-point value following option ") + a + ": " + argv[i]);
      if (fv < 0 || fv > 1) fail(std::string("ERROR: For option ") + a + ", floating-point value must be between 0 and 1.");
      opt.cutoff = fv;
    } else if (!strcmp(a, "-v") || !strcmp(a, "--verbose")) {
      opt.verbose = true;
    } else if (!strcmp(a, "-a") || !strcmp(a, "--alignment-order")) {
      opt.align_order = true;
    } else if (!strcmp(a, "-version")) {
      fail(std::string("PNPProbs version ") + kVersion);
    } else {
      fail(std::string("ERROR: Unrecognized option: ") + a);
    }
  }
  // sequences of all input files, in order (MSA::MSA, CPNP/MSA.cpp:130-136)
  std::vector<Row> seqs;
  for (const std::string& f : files) {
    std::vector<Row> part;
    std::string err;
    if (!cpnp::load_fasta(f, part, err)) fail(err);
    for (Row& r : part) {
      r.label = r.sort_label = (int)seqs.size();
      seqs.push_back(std::move(r));
    }
  }
  if (seqs.empty()) fail("ERROR: No sequences read.");
  const int n = (int)seqs.size();

  mlp_ctx* ctx = nullptr;
  stage("parse");
  // Small families run on the host (mlp_ctx_create_host: the same stages,
  // bit for bit, without initialising the GPU runtime, whose start-up and
  // teardown alone cost 0.2-0.4 s per process); at ~2e7 pair-cells/s on the
  // host threads, families up to MLP_HOST_MAX_CELLS pair-cells (default 4e6,
  // 0: always the GPU) finish there before a device would be ready.
  double pair_cells = 0;
  for (size_t a = 0; a < seqs.size(); a++)
    for (size_t b = a + 1; b < seqs.size(); b++)
      pair_cells += (double)(seqs[a].length() + 1) * (double)(seqs[b].length() + 1);
  const double host_max = getenv("MLP_HOST_MAX_CELLS") ? atof(getenv("MLP_HOST_MAX_CELLS")) : 4e6;
  if (pair_cells <= host_max) {
    check(nullptr, mlp_ctx_create_host(&ctx), "host context");
    stage("host context");
  } else {
    check(nullptr, open_device(&ctx), "device");
    stage("device init");
    // one family per process: a moderate batch scratch.  A fresh process's
    // allocation waits for the driver to clear memory the previous process
    // released; back to back at C3 (512 x 400) the posterior stage took 1.09 s
    // at 32 GB, 1.39 s at 16 GB, 7.4-10.5 s at 64 GB
    if (!getenv("MLP_SCRATCH_GB")) check(ctx, mlp_set_scratch(ctx, 32ull << 30), "device");
  }
  std::string res;
  std::vector<int64_t> off(1, 0);
  for (const Row& r : seqs) {
    res.append(r.data, 1, std::string::npos);
    off.push_back((int64_t)res.size());
  }
  check(ctx, mlp_family_load(ctx, n, res.data(), off.data()), "family");
  stage("load");

  if (just_features) {   // CPNP/MSA.cpp:153-166 (theta = 1.0)
    float f[5];
    int32_t ints[2];
    check(ctx, mlp_family_features(ctx, 1.0f, f, ints), "family test");
    char line[512];
    snprintf(line, sizeof line, "%f\t%f\t%d\t%d\t%f\t%f\t%f", f[0], f[1], ints[0], ints[1], f[2], f[3], f[4]);
    std::cout << line << std::endl;
    mlp_ctx_destroy(ctx);
    return 0;
  }
  cpnp::Profile aln;
  if (n == 1) {
    aln.push_back(seqs[0]);
  } else {
    // ModelAdjustmentTest (CPNP/MSA.cpp:775-882) -> pid, delta
    float identity, variance, delta;
    int32_t code;
    check(ctx, mlp_model_adjustment(ctx, &identity, &variance, &delta, &code), "family test");
    stage("family test (Viterbi)");
    const int pid = code % 10, vpid = code / 10;
    // pdoAlign (CPNP/MSA.cpp:895-1081): posteriors, distances, tree, consistency;
    // npdoAlign (CPNP/MSA.cpp:1084-1140): ArrangePosteriorProbs' pair body,
    // consistency, alignment graph, refinement
    const int64_t P = mlp_family_npairs(ctx);
    check(ctx, mlp_posteriors(ctx, progressive ? pid : pid | MLP_PID_NPDO, delta, 0, P), "posteriors");
    std::vector<float> dist(P);
    check(ctx, mlp_pair_results(ctx, 0, P, dist.data(), nullptr, nullptr), "results");
    std::vector<std::vector<float>> D(n, std::vector<float>(n, 0.f));
    for (int a = 0, p = 0; a < n; a++)
      for (int b = a + 1; b < n; b++, p++) D[a][b] = D[b][a] = dist[p];
    stage("posteriors");
    cpnp::GuideTree tree;
    if (progressive) {
      tree = cpnp::build_tree(D, vpid);
      stage("guide tree");
    }
    if (opt.consistency > 0) check(ctx, mlp_relax(ctx, opt.consistency), "consistency");
    check(ctx, mlp_synchronize(ctx), "consistency");
    stage("consistency");
    cpnp::SparseSet sp;
    sp.n = n;
    sp.lens.resize(n);
    for (int k = 0; k < n; k++) sp.lens[k] = seqs[k].length();
    sp.rp_off.assign(P + 1, 0);
    for (int a = 0, p = 0; a < n; a++)
      for (int b = a + 1; b < n; b++, p++) sp.rp_off[p + 1] = sp.rp_off[p] + sp.lens[a] + 2;
    int64_t total = 0;
    check(ctx, mlp_csr_total(ctx, &total), "sparse set");
    sp.row_ptr.resize(sp.rp_off[P]);
    sp.ent_off.resize(P + 1);
    sp.cols.resize(std::max<int64_t>(total, 1));
    sp.vals.resize(std::max<int64_t>(total, 1));
    check(ctx, mlp_csr_export(ctx, sp.row_ptr.data(), sp.ent_off.data(), sp.cols.data(), sp.vals.data()),
          "sparse set");
    stage("sparse set to host");
    // BuildPosterior of the merges and refinement passes on the GPU
    // (mlp_profile_posterior_cpnp) once the profile pair holds enough sparse
    // entries to pay for a device round trip (~0.1-0.2 ms; the host adds
    // ~5e4 entries in that time); the sparse set stays resident.  After
    // consistency a divergent family's set is nearly empty (C2: 5e4 entries
    // over 8128 pairs), a similar family's is not.
    static const int64_t gpu_min = getenv("MLP_PROFILE_GPU_MIN") ? atoll(getenv("MLP_PROFILE_GPU_MIN")) : 100000;
    std::vector<int32_t> lab1, lab2, map1, map2;
    cpnp::set_profile_backend([&](const cpnp::Profile& a, const cpnp::Profile& b, const int* w) -> const float* {
      int64_t entries = 0;
      for (const Row& x : a)
        for (const Row& y : b) {
          const int64_t p = sp.pair(std::min(x.label, y.label), std::max(x.label, y.label));
          entries += sp.ent_off[p + 1] - sp.ent_off[p];
        }
      if (entries < gpu_min) return nullptr;
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
      fill(a, lab1, map1);
      fill(b, lab2, map2);
      const int rc = mlp_profile_posterior_cpnp(ctx, w, (int)a.size(), lab1.data(), a[0].length(), map1.data(),
                                                (int)b.size(), lab2.data(), b[0].length(), map2.data(), nullptr);
      if (rc == MLP_ERR_STATE) return nullptr;   // a profile wider than an LDS row: the host computes it
      check(ctx, rc, "profile posterior");
      return mlp_profile_result(ctx);
    });
    // Profile posterior and MEA both on the device (mlp_profile_mea): only
    // the path (and the few cells a refinement scores) come back.  Opt-in:
    // the device MEA is a chain of dependent steps (8 waves over 64-row
    // strips) and measured slower than the host's at C3 (QuickProbs
    // refinement: 1.52 ms a call against ~1 ms), so by default
    // (MLP_MEA_GPU_MIN unset) every MEA runs on the host.
    static const int64_t mea_min = getenv("MLP_MEA_GPU_MIN") ? atoll(getenv("MLP_MEA_GPU_MIN")) : INT64_MAX;
    cpnp::set_mea_backend([&](const cpnp::Profile& a, const cpnp::Profile& b, const int* w,
                              const std::vector<int64_t>* cells, std::vector<float>* vals, std::string& path,
                              float* score) -> bool {
      if (mlp_ctx_is_host(ctx) || mea_min == INT64_MAX) return false;
      const int L1 = a[0].length(), L2 = b[0].length();
      if ((int64_t)L1 * L2 < mea_min) return false;
      auto fill = [](const cpnp::Profile& p, std::vector<int32_t>& lab, std::vector<int32_t>& map) {
        lab.clear();
        map.clear();
        for (const Row& r : p) {
          lab.push_back(r.label);
          map.push_back(0);
          for (int c = 1; c <= r.length(); c++)
            if (r.data[c] != '-') map.push_back(c);
        }
      };
      fill(a, lab1, map1);
      fill(b, lab2, map2);
      check(ctx, mlp_profile_defer(ctx, 1), "profile posterior");
      const int rc = mlp_profile_posterior_cpnp(ctx, w, (int)a.size(), lab1.data(), L1, map1.data(), (int)b.size(),
                                                lab2.data(), L2, map2.data(), nullptr);
      if (rc == MLP_ERR_STATE) {   // a profile wider than an LDS row: the host computes it
        check(ctx, mlp_profile_defer(ctx, 0), "profile posterior");
        return false;
      }
      check(ctx, rc, "profile posterior");
      if (cells && !cells->empty())
        check(ctx, mlp_profile_gather(ctx, (int64_t)cells->size(), cells->data(), vals->data()), "profile posterior");
      path.resize((size_t)L1 + L2);
      int32_t n = 0;
      check(ctx, mlp_profile_mea(ctx, &path[0], &n, score), "MEA");
      path.resize(n);
      check(ctx, mlp_profile_defer(ctx, 0), "profile posterior");
      return true;
    });
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
    fprintf(stderr, "[host] profile posteriors %.3f s (%lld calls, %lld on the GPU), MEA %.3f s\n", tp, (long long)nc,
            (long long)nd, tm);
  }
  mlp_ctx_destroy(ctx);
  stage("context teardown");
  std::string out;
  cpnp::write_mfa(out, aln);
  if (outname.empty()) {
    fwrite(out.data(), 1, out.size(), stdout);
  } else {
    FILE* f = fopen(outname.c_str(), "wb");
    if (!f) fail("ERROR: Could not open file '" + outname + "' for writing.");
    fwrite(out.data(), 1, out.size(), f);
    fclose(f);
  }
  stage("output");
  return 0;
}
