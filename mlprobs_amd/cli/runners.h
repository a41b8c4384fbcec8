// runners.h -- the two drop-in aligners as in-process calls: what
// `c_p_np_aln` (baseMSA/C_P_NP_Aln, MSA::MSA, CPNP/MSA.cpp:123-187) and
// `quickprobs` (realign/QuickProbs, QP/Console/main.cpp:18-68) do after
// reading their input file, on already parsed sequences.  The CLIs are thin
// wrappers over these; the pipeline driver (`mlprobs`, pipeline.h) calls them
// once per family and once per realigned column region without starting a
// process, sharing one device context through a Session.
#pragma once
#include <string>
#include <thread>
#include <vector>

#include "mlpgpu.h"
#include "msa_host.h"
#include "qp_host.h"

namespace mlpr {

// Contexts for a sequence of runs.  Small families (at most host_max_cells
// pair-cells: MLP_HOST_MAX_CELLS, default 4e6) get a host context of their
// own (no HIP call); larger ones share one device context, created on first
// use (device 0; MLP_DEVICES=<mask> opts in to the multi-GPU context).
struct Session {
  mlp_ctx* dev = nullptr;
  size_t scratch_bytes = 0;   // 0: the caller's default (16 GB, both aligners)
  double host_max_cells = -1; // < 0: MLP_HOST_MAX_CELLS or 4e6
  int device_runs = 0, host_runs = 0;  // aligner runs per context kind (the pipeline's trace)
  ~Session();
  double host_max() const;
  // Start creating the device context now, on a thread: HIP's start-up
  // (~0.2 s a process) overlaps the caller's host work (reading the models,
  // the family); the first run that needs the device waits for it.  A failed
  // creation is reported by that run, as without the prewarm.
  void prewarm();
  void ready();
  std::thread warm;
};

// A failed run: the exit status the reference CLI would return and the
// message it would print on stderr (stdout: `out`, possibly partial).
struct Failure {
  int status;
  std::string msg;
};

// c_p_np_aln on `seqs` (rows as cpnp::load_fasta gives them, labels in
// input order): the `-G` feature line when `features`, else the MFA of
// `-p 0` (progressive) or `-p 1`.  Returns 0 and the stdout bytes in `out`;
// or the reference's exit status (1) with the stderr text in `err`.
// session = nullptr: a context of its own, released before returning.
int run_cpnp(std::vector<cpnp::Row> seqs, bool features, bool progressive, cpnp::Options opt, Session* session,
             std::string& out, std::string& err);

// quickprobs on `seqs` (qph::load_fasta rows): the FASTA it writes on stdout.
// threads <= 0: min(16, hardware threads).  Failures: status 255 with the
// exception text (QP/Console/main.cpp:61-64).
int run_qp(std::vector<qph::Seq> seqs, const qph::Options& opt, int threads, Session* session, std::string& out,
           std::string& err);

// Pair-cells sum_{a<b} (L_a + 1)(L_b + 1) of a family.
double pair_cells(const std::vector<int>& lens);

// MLP_CLI_TIMES=1: stage times on stderr (off by default: the references
// are silent on stderr on success).  stage(nullptr) starts the clock.
void stage(const char* name);

}  // namespace mlpr
