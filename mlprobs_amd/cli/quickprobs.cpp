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
#include "runners.h"

[[noreturn]] static void fail(const std::string& msg) {  // main.cpp:61-64
  std::cerr << msg << std::endl;
  exit(255);
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

int main(int argc, char** argv) {
  mlpr::stage(nullptr);  // start the stage clock
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
  for (const qph::Seq& s : seqs)
    if (s.data.find('-') != std::string::npos)
      fail("ERROR: gapped input ('.' in a sequence) is not available in this build");
  mlpr::stage("load");
  std::string out;
  const int status = mlpr::run_qp(std::move(seqs), opt, threads, nullptr, out, err);
  if (status) {
    std::cerr << err << std::endl;
    return status;
  }
  if (outname.empty()) {
    fwrite(out.data(), 1, out.size(), stdout);
  } else {
    FILE* f = fopen(outname.c_str(), "wb");
    if (!f) fail("ERROR: unable to open output file " + outname);
    fwrite(out.data(), 1, out.size(), f);
    fclose(f);
  }
  mlpr::stage("output");
  return 0;
}
