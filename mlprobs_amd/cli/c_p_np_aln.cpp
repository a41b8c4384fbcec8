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
#include "runners.h"

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

[[noreturn]] static void fail(const std::string& msg) {
  std::cerr << msg << std::endl;
  exit(1);
}

int main(int argc, char** argv) {
  mlpr::stage(nullptr);  // start the stage clock
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
  std::string out, err;
  const int status = mlpr::run_cpnp(std::move(seqs), just_features, progressive, opt, nullptr, out, err);
  if (status) {
    std::cerr << err << std::endl;
    return status;
  }
  if (outname.empty() || just_features) {   // the -G line always goes to stdout (CPNP/MSA.cpp:163)
    fwrite(out.data(), 1, out.size(), stdout);
  } else {
    FILE* f = fopen(outname.c_str(), "wb");
    if (!f) fail("ERROR: Could not open file '" + outname + "' for writing.");
    fwrite(out.data(), 1, out.size(), f);
    fclose(f);
  }
  mlpr::stage("output");
  return 0;
}
