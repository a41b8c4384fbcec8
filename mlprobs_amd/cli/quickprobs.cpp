// quickprobs -- drop-in for realign/QuickProbs/bin/quickprobs (QuickProbs 2,
// the realigner MLProbs.py calls) with the all-pairs posterior and
// consistency stages on the GPU (libmlpgpu, include/mlpgpu.h).
//
// ExtendedMSA::doAlign (QP/Alignment/Multiple/ExtendedMSA.cpp:67-213) with the
// default configuration (Configuration::setDefaults, Configuration.cpp:86-160):
//   posteriors (GPU, MLP_PID_QP) -> UPGMA guide tree + weights (host)
//   -> consistency with subtree-size selectivity 200 (GPU, mlp_relax_qp_selective)
//   -> progressive construction + column refinement (host) -> FASTA on stdout.
// Options (ProgramOptions::parse, QP/Common/ProgramOptions.cpp:9-64: any
// number of leading '-', values in the next argument, the first remaining
// argument is the input file):
//   -o/--outfile FILE, -c/--con-iters N, -r/--ref-count N, -t/--num-threads N,
//   -p/--platform N, -d/--device N, --mem-limit N (accepted; OpenCL / memory
//   settings of the reference), -v/--verbose (accepted).
//   -n/--nucleotide and -l/--clustalw are not in this build (exit 255).
// No input file: the usage text on stdout, exit 0 (main.cpp:31-37).  Errors
// the reference throws are printed on stderr with exit status 255.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <iostream>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "mlpgpu.h"
#include "qp_host.h"

static void stage(const char* name) {  // MLP_CLI_TIMES=1: stage times on stderr
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

[[noreturn]] static void fail(const std::string& msg) {  // main.cpp:61-64
  std::cerr << msg << std::endl;
  exit(255);
}

static void check(mlp_ctx* ctx, int rc, const char* what) {
  if (rc != MLP_OK) fail(std::string("ERROR: ") + what + ": " + (ctx ? mlp_last_error(ctx) : "no context"));
}

static void usage() {
  std::cout << "Usage:\n\t quickprobs [OPTION]... [infile]...\n\n"
               "Options:\n"
               "\tclustalw,l            \tuse CLUSTALW output format instead of FASTA format\n"
               "\tcon-iters,c           \tnumber of consistency repetitions\n"
               "\tdevice,d              \tOpenCL device id (use CPU mode if not specified)\n"
               "\tmem-limit             \tmemory limit\n"
               "\tnucleotide,n          \trun QuickProbs in the nucleotide mode\n"
               "\tnum-threads,t         \tnumber of threads (detect automatically if not specified)\n"
               "\toutfile,o             \toutput file name (STDOUT by default)\n"
               "\tplatform,p            \tOpenCL platform id (use CPU mode if not specified)\n"
               "\tref-count,r           \tnumber of iterative refinement passes\n"
               "\tverbose,v             \treport progress while aligning\n\n\n";
}

static bool parse_int(const std::string& s, long long* v) {
  if (s.empty()) return false;
  char* end;
  const long long r = strtoll(s.c_str(), &end, 10);
  if (*end) return false;
  *v = r;
  return true;
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
  std::vector<std::string> args(argv + 1, argv + argc), rest;
  std::string outname;
  qph::Options opt;
  int threads = 0;
  for (size_t i = 0; i < args.size(); i++) {
    std::string a = args[i];
    if (a.empty() || a[0] != '-') {
      rest.push_back(a);
      continue;
    }
    while (!a.empty() && a[0] == '-') a.erase(0, 1);
    if (a == "v" || a == "verbose") continue;
    if (a == "n" || a == "nucleotide") fail("ERROR: the nucleotide mode is not available in this build");
    if (a == "l" || a == "clustalw") fail("ERROR: CLUSTALW output is not available in this build");
    const bool is_int = a == "c" || a == "con-iters" || a == "r" || a == "ref-count" || a == "t" ||
                        a == "num-threads" || a == "p" || a == "platform" || a == "d" || a == "device" ||
                        a == "mem-limit";
    if (a == "o" || a == "outfile") {
      if (i + 1 < args.size()) outname = args[++i];
      continue;
    }
    if (!is_int) fail("ERROR: unrecognised option: -" + a);
    long long v;
    if (i + 1 < args.size() && parse_int(args[i + 1], &v)) {  // an unparsable value stays positional
      ++i;
      if (a == "c" || a == "con-iters") opt.consistency = (int)v;
      else if (a == "r" || a == "ref-count") opt.refinement = (int)v;
      else if (a == "t" || a == "num-threads") threads = (int)v;
    }
  }
  if (rest.empty()) {
    usage();
    return 0;
  }
  const std::string infile = rest[0];
  if (threads <= 0) threads = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));

  std::vector<qph::Seq> seqs;
  std::string msg, err;
  if (!qph::load_fasta(infile, seqs, msg, err)) {
    std::cout << msg;
    std::cout.flush();
    fail(err);
  }
  const int n = (int)seqs.size();
  for (const qph::Seq& s : seqs)
    if (s.data.find('-') != std::string::npos)
      fail("ERROR: gapped input ('.' in a sequence) is not available in this build");
  stage("load");

  qph::Profile aln;
  try {
    if (n == 1) {
      aln.push_back(seqs[0]);
    } else {
      mlp_ctx* ctx = nullptr;
      stage("parse");
      // Small families (MLProbs realigns one column region per call) run on
      // the host context: the same stages bit for bit on host threads, no
      // HIP runtime start-up (0.14-0.22 s per process); above
      // MLP_HOST_MAX_CELLS pair-cells (default 4e6, 0: always the GPU) the GPU.
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
        // one family per process: a 16 GB batch scratch.  A fresh process's
        // allocation waits for the driver to clear memory the previous process
        // released: measured at C3 (512 x 400) 0.82 s posteriors at 16 GB vs
        // 6.9-7.2 s at 64 GB, 1.16 s at 8 GB
        if (!getenv("MLP_SCRATCH_GB")) check(ctx, mlp_set_scratch(ctx, 16ull << 30), "device");
      }
      std::string res;
      std::vector<int64_t> off(1, 0);
      for (const qph::Seq& s : seqs) {
        res.append(s.data, 1, std::string::npos);
        off.push_back((int64_t)res.size());
      }
      check(ctx, mlp_family_load(ctx, n, res.data(), off.data()), "family");
      // PosteriorStage::run (QP/Alignment/Multiple/PosteriorStage.cpp:58-117)
      const int64_t P = mlp_family_npairs(ctx);
      check(ctx, mlp_posteriors(ctx, MLP_PID_QP, 0.f, 0, P), "posteriors");
      std::vector<float> dist(P);
      check(ctx, mlp_pair_results(ctx, 0, P, dist.data(), nullptr, nullptr), "results");
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
        check(ctx, mlp_relax_qp_selective(ctx, opt.consistency, wc.data(), seld.data(), 200.f), "consistency");
      check(ctx, mlp_synchronize(ctx), "consistency");
      stage("consistency");
      // construction + refinement: profile posteriors on the GPU from the
      // device-resident sparse set; the host copy of the set is fetched only
      // if a profile is too wide for the kernel's LDS row
      std::unique_ptr<qph::Sparse> host_sp;
      qph::PosteriorBackend be;
      be.device = [&](const std::vector<float>& w, const qph::Profile& A, const qph::Profile& B) -> const float* {
        const int L1 = A[0].length(), L2 = B[0].length();
        std::vector<int32_t> l1, l2;
        for (const qph::Seq& q : A) l1.push_back(q.label);
        for (const qph::Seq& q : B) l2.push_back(q.label);
        const std::vector<int32_t> m1 = qph::profile_maps(A), m2 = qph::profile_maps(B);
        // out = NULL: the matrix stays in the library's pinned buffer
        const int rc = mlp_profile_posterior(ctx, w.data(), (int)A.size(), l1.data(), L1, m1.data(), (int)B.size(),
                                             l2.data(), L2, m2.data(), nullptr);
        if (rc == MLP_ERR_STATE) return nullptr;  // too wide: the host restatement
        check(ctx, rc, "profile posterior");
        return mlp_profile_result(ctx);
      };
      // posterior and MEA both on the device, only the path comes back
      // (opt-in, MLP_MEA_DEVICE=1: measured slower than the host MEA at C3,
      // 1.52 ms a call against ~1 ms)
      if (getenv("MLP_MEA_DEVICE") && atoi(getenv("MLP_MEA_DEVICE")) > 0) {
        be.device_mea = [&](const std::vector<float>& w, const qph::Profile& A, const qph::Profile& B,
                            std::string& path, float* score) -> bool {
          const int L1 = A[0].length(), L2 = B[0].length();
          std::vector<int32_t> l1, l2;
          for (const qph::Seq& q : A) l1.push_back(q.label);
          for (const qph::Seq& q : B) l2.push_back(q.label);
          const std::vector<int32_t> m1 = qph::profile_maps(A), m2 = qph::profile_maps(B);
          check(ctx, mlp_profile_defer(ctx, 1), "profile posterior");
          const int rc = mlp_profile_posterior(ctx, w.data(), (int)A.size(), l1.data(), L1, m1.data(), (int)B.size(),
                                               l2.data(), L2, m2.data(), nullptr);
          if (rc == MLP_ERR_STATE) {  // too wide: the host restatement
            check(ctx, mlp_profile_defer(ctx, 0), "profile posterior");
            return false;
          }
          check(ctx, rc, "profile posterior");
          path.resize((size_t)L1 + L2);
          int32_t n = 0;
          check(ctx, mlp_profile_mea(ctx, &path[0], &n, score), "MEA");
          path.resize(n);
          check(ctx, mlp_profile_defer(ctx, 0), "profile posterior");
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
          check(ctx, mlp_csr_total(ctx, &total), "sparse set");
          sp.row_ptr.resize(sp.rp_off[P]);
          sp.ent_off.resize(P + 1);
          sp.cols.resize(std::max<int64_t>(total, 1));
          sp.vals.resize(std::max<int64_t>(total, 1));
          check(ctx, mlp_csr_export(ctx, sp.row_ptr.data(), sp.ent_off.data(), sp.cols.data(), sp.vals.data()),
                "sparse set");
          sp.build_views();
        }
        return *host_sp;
      };
      aln = qph::construct_and_refine(seqs, be, tree, opt, threads);
      mlp_ctx_destroy(ctx);
      stage("construction + refinement");
    }
  } catch (const std::runtime_error& e) {
    fail(e.what());
  }
  std::string out;
  qph::write_fasta(out, aln);
  if (outname.empty()) {
    fwrite(out.data(), 1, out.size(), stdout);
  } else {
    FILE* f = fopen(outname.c_str(), "wb");
    if (!f) fail("ERROR: unable to open output file " + outname);
    fwrite(out.data(), 1, out.size(), f);
    fclose(f);
  }
  return 0;
}
