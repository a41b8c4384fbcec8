// mlprobs -- the MLProbs pipeline driver (kuangmeng/MLProbs MLProbs.py) over
// the MI355X aligners, one process per family:
//
//   mlprobs [options] in.fa [out.msa]      (MLProbs.py in.fa out.msa)
//
// writes the final MSA to out.msa (default result.msa, MLProbs.py:33) and the
// reference's "[MAIN STEP]" / "[ELAPSED TIME]" progress on stdout.  The
// aligners run in-process (pipeline.h, runners.h); options:
//   --models DIR      forests + normalisation files (default: the
//                     classifier/ directory next to this binary's package)
//   --cpnp CMD --quickprobs CMD
//                     run the stages as external commands instead, exactly
//                     as MLProbs.py does (the reference CLIs built from
//                     source: the pipeline's CPU baseline)
//   --tmp DIR         scratch for the external commands' region files
//   --trace FILE      a JSON record of the stages (features, classes, column
//                     scores, regions, per-stage seconds)
//   -q                no progress lines
// Exit status 0; 1 where the reference pipeline raises a Python exception
// (no output written).
//
//   mlprobs --batch LIST [--devices D0,D1,..] [--report FILE] [options]
//
// runs many families (the reference's harness loops over a benchmark's
// families, one MLProbs.py process each: script.py:38-62): LIST holds one
// family per line, "in.fa out.msa [trace.json]" (whitespace separated).  One
// worker process per entry of --devices (default 0; an id may repeat) is
// forked before any GPU call, sees only its device (HIP_VISIBLE_DEVICES),
// keeps one device context for all its families and takes the next family,
// largest first, from a counter shared with the others.  Each family's
// output (and trace) is written exactly as a separate run writes it.  The
// report (JSON: per family seconds, status, worker, device runs; the wall
// time) goes to FILE or stdout.  Exit status 0 when every family succeeded.
#include <limits.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <numeric>
#include <sstream>
#include <string>

#include "pipeline.h"

static std::string self_dir() {
  char buf[PATH_MAX];
  const ssize_t n = readlink("/proc/self/exe", buf, sizeof buf - 1);
  if (n <= 0) return ".";
  buf[n] = 0;
  std::string p(buf);
  return p.substr(0, p.rfind('/'));
}

static std::string json_str(const std::string& s) {
  std::string r = "\"";
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') r += '\\', r += (char)c;
    else if (c < 0x20) {
      char b[8];
      snprintf(b, sizeof b, "\\u%04x", c);
      r += b;
    } else r += (char)c;
  }
  return r + "\"";
}

static std::string json_num(double v) {
  char b[40];
  snprintf(b, sizeof b, "%.17g", v);
  return b;
}

static void write_trace(const std::string& path, const mlpp::Trace& tr, const std::string& tools,
                        const mlpr::Session& session) {
  std::string j = "{";
  j += "\"tools\": " + json_str(tools);
  j += ", \"features_line\": " + json_str(tr.features_line);
  j += ", \"features1\": [";
  for (size_t i = 0; i < tr.features1.size(); i++) j += (i ? ", " : "") + json_num(tr.features1[i]);
  j += "], \"class1\": " + std::to_string(tr.class1);
  j += ", \"killed_stage\": " + std::to_string(tr.killed_stage);
  j += ", \"un_sp\": " + json_num(tr.cs.un_sp) + ", \"sd_un_sp\": " + json_num(tr.cs.sd) +
       ", \"peak_length_ratio\": " + json_num(tr.cs.peak) + ", \"len_seqs\": " + std::to_string(tr.cs.lens) +
       ", \"len_family\": " + std::to_string(tr.cs.nkeys);
  j += ", \"col_score\": [";
  for (size_t i = 0; i < tr.cs.col.size(); i++) j += (i ? ", " : "") + json_num(tr.cs.col[i]);
  j += "], \"class_region\": " + std::to_string(tr.class_region) + ", \"class_lens\": " + std::to_string(tr.class_lens);
  j += ", \"regions\": [";
  for (size_t i = 0; i < tr.regions.size(); i++)
    j += (i ? ", [" : "[") + std::to_string(tr.regions[i].first) + ", " + std::to_string(tr.regions[i].second) + "]";
  j += "], \"realigned\": [";
  for (size_t i = 0; i < tr.realigned.size(); i++) j += (i ? ", " : "") + json_str(tr.realigned[i]);
  j += "], \"kept_original\": [";
  for (size_t i = 0; i < tr.kept_original.size(); i++) j += (i ? ", " : "") + std::to_string(tr.kept_original[i]);
  j += "], \"path\": " + json_str(tr.path) + ", \"quickprobs_calls\": " + std::to_string(tr.quickprobs_calls);
  j += ", \"device_runs\": " + std::to_string(session.device_runs) +
       ", \"host_runs\": " + std::to_string(session.host_runs);
  j += ", \"times\": {";
  bool first = true;
  for (const auto& kv : tr.times) {
    j += (first ? "" : ", ") + json_str(kv.first) + ": " + json_num(kv.second);
    first = false;
  }
  j += "}}\n";
  FILE* f = fopen(path.c_str(), "wb");
  if (f) {
    fwrite(j.data(), 1, j.size(), f);
    fclose(f);
  }
}

// Stage probes for the tests (tests/test_pipeline.py):
//   --classify NAME   feature rows (whitespace separated) on stdin -> per row
//                     "class p_0 .. p_k" (the normalised inputs, as the
//                     classifiers receive them)
//   --scores FILE     calculateColScore on FILE's text (one trailing newline
//                     removed, as getstatusoutput gives it) and getAvgColScore
//                     on FILE, as JSON
//   --regions         one score vector per stdin line -> the unreliable
//                     regions for class_lens 0..3 and the reliable regions,
//                     one JSON line each
static int probe(const std::string& mode, const std::string& arg, const std::string& models) {
  if (mode == "--classify") {
    mlpp::Forest f;
    std::string err;
    if (!f.load(models + "/" + arg + ".forest", err)) {
      fprintf(stderr, "%s\n", err.c_str());
      return 1;
    }
    char line[1 << 16];
    while (fgets(line, sizeof line, stdin)) {
      std::vector<double> x;
      char* p = line;
      char* end;
      for (double v; (v = strtod(p, &end)), end != p; p = end) x.push_back(v);
      if ((int)x.size() != f.n_features) continue;
      const std::vector<double> pr = f.predict_proba(x);
      printf("%.17g", f.predict(x));
      for (double v : pr) printf(" %.17g", v);
      printf("\n");
    }
    return 0;
  }
  if (mode == "--scores") {
    FILE* fh = fopen(arg.c_str(), "rb");
    if (!fh) return 1;
    std::string text;
    char buf[1 << 16];
    size_t got;
    while ((got = fread(buf, 1, sizeof buf, fh)) > 0) text.append(buf, got);
    fclose(fh);
    std::string t = text;
    if (!t.empty() && t.back() == '\n') t.pop_back();
    const mlpp::ColScores cs = mlpp::column_scores(mlpp::parse_dic(mlpp::split_newline(t)));
    std::string j = "{\"col_score\": [";
    for (size_t i = 0; i < cs.col.size(); i++) j += (i ? ", " : "") + json_num(cs.col[i]);
    j += "], \"un_sp\": " + json_num(cs.un_sp) + ", \"sd_un_sp\": " + json_num(cs.sd) +
         ", \"peak_length_ratio\": " + json_num(cs.peak) + ", \"len_seqs\": " + std::to_string(cs.lens) +
         ", \"len_family\": " + std::to_string(cs.nkeys) + ", \"error\": " + (cs.error ? "true" : "false") +
         ", \"avg_col_score\": " + json_num(mlpp::avg_col_score(text)) + "}\n";
    fwrite(j.data(), 1, j.size(), stdout);
    return 0;
  }
  if (mode == "--regions") {
    std::string line;
    char buf[1 << 16];
    while (fgets(buf, sizeof buf, stdin)) {
      line = buf;
      std::vector<double> col;
      const char* p = line.c_str();
      char* end;
      for (double v; (v = strtod(p, &end)), end != p; p = end) col.push_back(v);
      auto emit = [](const std::vector<std::pair<int64_t, int64_t>>& r) {
        std::string s = "[";
        for (size_t i = 0; i < r.size(); i++)
          s += (i ? ", [" : "[") + std::to_string(r[i].first) + ", " + std::to_string(r[i].second) + "]";
        return s + "]";
      };
      std::string j = "{\"unreliable\": {";
      for (int cl = 0; cl < 4; cl++)
        j += (cl ? ", \"" : "\"") + std::to_string(cl) + "\": " + emit(mlpp::unreliable_regions(col, 1.2, 0.0, cl));
      j += "}, \"reliable\": " + emit(mlpp::reliable_regions(col, 2.0, 0, 0)) + "}\n";
      fwrite(j.data(), 1, j.size(), stdout);
    }
    return 0;
  }
  return 2;
}

// pair-cells of a family as the aligners read it (0 when it cannot be read)
static double family_cells(const std::string& path) {
  std::vector<cpnp::Row> rows;
  std::string err;
  if (!cpnp::load_fasta(path, rows, err)) return 0;
  std::vector<int> lens;
  for (const cpnp::Row& r : rows) lens.push_back(r.length());
  return mlpr::pair_cells(lens);
}

// one family of a run: the pipeline, its output file and trace
static int run_family(const std::string& in, const std::string& out, const std::string& trace, mlpp::Tools& tools,
                      const mlpp::Models& M, const mlpr::Session& session, bool verbose) {
  std::string result, err;
  mlpp::Trace tr;
  const bool ok = mlpp::run_pipeline(in, tools, M, result, tr, err, verbose);
  if (!trace.empty()) write_trace(trace, tr, tools.name(), session);
  if (!ok) {
    fprintf(stderr, "mlprobs: %s: %s\n", in.c_str(), err.c_str());
    return 1;
  }
  FILE* f = fopen(out.c_str(), "wb");
  if (!f) {
    fprintf(stderr, "mlprobs: cannot write %s\n", out.c_str());
    return 1;
  }
  fwrite(result.data(), 1, result.size(), f);
  fclose(f);
  return 0;
}

struct BatchSlot {   // one family's record in the workers' shared memory
  double seconds;
  int status, worker, device_runs, done;
};

static int run_batch(const std::string& list, const std::string& devices, const std::string& report,
                     const std::string& models, const std::string& cpnp_cmd, const std::string& qp_cmd,
                     const std::string& tmp, bool verbose) {
  struct Fam { std::string in, out, trace; double cells; };
  std::vector<Fam> fams;
  {
    FILE* f = fopen(list.c_str(), "rb");
    if (!f) {
      fprintf(stderr, "mlprobs: cannot read %s\n", list.c_str());
      return 2;
    }
    char line[8192];
    while (fgets(line, sizeof line, f)) {
      std::istringstream ss(line);
      Fam x;
      if (!(ss >> x.in >> x.out)) continue;
      ss >> x.trace;
      fams.push_back(x);
    }
    fclose(f);
  }
  std::vector<int> devs;
  {
    std::stringstream ss(devices);
    std::string tok;
    while (std::getline(ss, tok, ',')) devs.push_back(atoi(tok.c_str()));
    if (devs.empty()) devs.push_back(0);
  }
  const int n = (int)fams.size(), nw = (int)devs.size();
  for (Fam& x : fams) x.cells = family_cells(x.in);
  std::vector<int> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return fams[a].cells > fams[b].cells; });
  const double host_max = mlpr::Session().host_max();
  // the shared counter and per-family records (anonymous shared memory,
  // mapped before the fork)
  const size_t bytes = 64 + sizeof(BatchSlot) * (size_t)std::max(n, 1);
  void* shm = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  if (shm == MAP_FAILED) {
    perror("mlprobs: mmap");
    return 2;
  }
  int* next = (int*)shm;
  BatchSlot* slot = (BatchSlot*)((char*)shm + 64);
  memset(shm, 0, bytes);
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<pid_t> kids;
  for (int w = 0; w < nw; w++) {
    fflush(nullptr);
    const pid_t pid = fork();
    if (pid < 0) {
      perror("mlprobs: fork");
      return 2;
    }
    if (pid > 0) {
      kids.push_back(pid);
      continue;
    }
    // ---- worker w: its device only (nothing above touched the GPU); the
    // worker's scope ends (its context torn down) before the process exits
    setenv("HIP_VISIBLE_DEVICES", std::to_string(devs[w]).c_str(), 1);
    const int code = [&]() {
      mlpr::Session session;
      std::unique_ptr<mlpp::Tools> tools;
      const std::string wtmp = tmp + "/w" + std::to_string(w);
      if (!cpnp_cmd.empty()) {
        mkdir(wtmp.c_str(), 0755);
        tools = mlpp::external_tools(cpnp_cmd, qp_cmd, wtmp);
      } else {
        tools = mlpp::in_process_tools(&session);
        if (n && fams[order[0]].cells > host_max) session.prewarm();   // overlaps the models' load
      }
      mlpp::Models M;
      std::string err;
      if (!M.load(models, err)) {
        fprintf(stderr, "mlprobs: %s\n", err.c_str());
        return 2;
      }
      for (int k; (k = __atomic_fetch_add(next, 1, __ATOMIC_RELAXED)) < n;) {
        const Fam& x = fams[order[k]];
        const int dev0 = session.device_runs;
        const auto f0 = std::chrono::steady_clock::now();
        const int st = run_family(x.in, x.out, x.trace, *tools, M, session, verbose);
        BatchSlot& r = slot[order[k]];
        r.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - f0).count();
        r.status = st;
        r.worker = w;
        r.device_runs = session.device_runs - dev0;
        __atomic_store_n(&r.done, 1, __ATOMIC_RELEASE);
      }
      return 0;
    }();
    fflush(nullptr);
    exit(code);
  }
  int bad = 0;
  for (pid_t p : kids) {
    int ws = 0;
    waitpid(p, &ws, 0);
    if (!WIFEXITED(ws) || WEXITSTATUS(ws) != 0) bad++;
  }
  const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::string j = "{\"families\": " + std::to_string(n) + ", \"workers\": " + std::to_string(nw) +
                  ", \"devices\": " + json_str(devices) + ", \"wall_s\": " + json_num(wall) + ", \"runs\": [";
  int failed = 0;
  for (int i = 0; i < n; i++) {
    const BatchSlot& r = slot[i];
    const bool done = __atomic_load_n(&r.done, __ATOMIC_ACQUIRE) != 0;
    if (!done || r.status) failed++;
    j += std::string(i ? ", " : "") + "{\"in\": " + json_str(fams[i].in) + ", \"cells\": " + json_num(fams[i].cells) +
         ", \"s\": " + json_num(done ? r.seconds : -1) + ", \"status\": " + std::to_string(done ? r.status : -1) +
         ", \"worker\": " + std::to_string(done ? r.worker : -1) + ", \"device_runs\": " +
         std::to_string(done ? r.device_runs : 0) + "}";
  }
  j += "], \"failed\": " + std::to_string(failed) + ", \"workers_failed\": " + std::to_string(bad) + "}\n";
  munmap(shm, bytes);
  if (report.empty()) {
    fwrite(j.data(), 1, j.size(), stdout);
  } else if (FILE* f = fopen(report.c_str(), "wb")) {
    fwrite(j.data(), 1, j.size(), f);
    fclose(f);
  }
  return failed || bad ? 1 : 0;
}

int main(int argc, char** argv) {
  std::string models = self_dir() + "/../classifier", cpnp_cmd, qp_cmd, tmp = "/tmp", trace, batch, devices = "0",
              report;
  bool verbose = true;
  std::vector<std::string> pos;
  for (int i = 1; i < argc; i++) {
    const std::string a = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) {
        fprintf(stderr, "mlprobs: %s needs a value\n", a.c_str());
        exit(2);
      }
      return argv[++i];
    };
    if (a == "--models") models = val();
    else if (a == "--cpnp") cpnp_cmd = val();
    else if (a == "--quickprobs") qp_cmd = val();
    else if (a == "--tmp") tmp = val();
    else if (a == "--trace") trace = val();
    else if (a == "--batch") batch = val();
    else if (a == "--devices") devices = val();
    else if (a == "--report") report = val();
    else if (a == "-q") verbose = false;
    else if (a == "--classify" || a == "--scores") {
      const std::string v = val();
      return probe(a, v, models);
    } else if (a == "--regions") return probe(a, "", models);
    else if (a == "-h" || a == "--help") {
      printf("usage: mlprobs [--models DIR] [--cpnp CMD --quickprobs CMD] [--tmp DIR] [--trace FILE] [-q] in.fa [out.msa]\n"
             "       mlprobs --batch LIST [--devices D0,D1,..] [--report FILE] [options]\n");
      return 0;
    } else pos.push_back(a);
  }
  if ((!cpnp_cmd.empty()) != (!qp_cmd.empty())) {
    fprintf(stderr, "mlprobs: --cpnp and --quickprobs go together\n");
    return 2;
  }
  if (!batch.empty()) return run_batch(batch, devices, report, models, cpnp_cmd, qp_cmd, tmp, verbose);
  if (pos.empty()) {
    fprintf(stderr, "usage: mlprobs [options] in.fa [out.msa]\n");
    return 2;
  }
  const std::string in = pos[0], out = pos.size() > 1 ? pos[1] : "result.msa";
  mlpr::Session session;
  std::unique_ptr<mlpp::Tools> tools;
  if (!cpnp_cmd.empty()) {
    tools = mlpp::external_tools(cpnp_cmd, qp_cmd, tmp);
  } else {
    tools = mlpp::in_process_tools(&session);
    // a family the aligners run on the device: its context starts while the
    // models are read (the first stage, the -G line, needs it)
    if (family_cells(in) > session.host_max()) session.prewarm();
  }
  mlpp::Models M;
  std::string err;
  if (!M.load(models, err)) {
    fprintf(stderr, "mlprobs: %s\n", err.c_str());
    return 1;
  }
  return run_family(in, out, trace, *tools, M, session, verbose);
}
