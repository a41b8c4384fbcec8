// mlp_knobs.h -- every environment variable libmlpgpu reads, in one registry
// (mlp_knobs.cpp holds the table and the only getenv of the library).
//
// Settings (product):
//   MLP_SCRATCH_GB            cap of a device context's batch scratch, GiB (default:
//                             free HBM less max(16 GiB, 7%); mlp_set_scratch overrides)
//   MLP_HOST_THREADS          threads of a host context (default: hardware threads)
//   MLP_POOL_KEEP_GB          device pool bytes a process keeps once its last context on
//                             the device closes, GiB (default 32)
// Test hooks (MLP_TEST_*): force one side of a decision the library makes by
// itself, so the GPU suite checks both sides bit-identical:
//   MLP_TEST_PG_SEPARATE      0/1: PF posterior in the Zm slots / its own array
//   MLP_TEST_TOT_LANEFOLD     0/1: one-wave-per-pair local totals / the lane fold
//   MLP_TEST_TOT_FOLDBOUND    0/1: running-maximum / folded chunk-maximum listing bound
//   MLP_TEST_TOT_BESIDE       0/1/2: local totals after / beside the backward sweeps
//   MLP_TEST_TOT_FORCE_REPAIR every pair through the local totals' repair path
//   MLP_TEST_DEFER_FINISH     0: finish each batch before the next is launched
//   MLP_TEST_FORCE_PEER       peer copies between contexts on one device
//   MLP_TEST_ALLGATHER_FORCE  the grouped RCCL all-gather body at one rank
//   MLP_TEST_MEA_SPINS        device MEA: polls before a strip gives up (0: at once)
//   MLP_TEST_RELAX_PATH       tasks | pairs: row tasks only / fail on any row task
//   MLP_TEST_RELAX_TILE       outputs per relaxation tile (1..kTileMax)
//   MLP_TEST_RELAX_KP         the relaxation's large-prefetch instantiation
//   MLP_TEST_RELAX_LDS_KB     LDS staging of the one-workgroup class
//   MLP_TEST_RELAX_SMALL_KB   LDS staging of the two-workgroup class
//   MLP_TEST_RELAX_SPLIT_Z    z's per tile staged in passes
//   MLP_TEST_RELAX_GLOBAL_Z   z's per output read in place from HBM
//   MLP_TEST_PROFILE_STAGE    profile posterior: entries staged per lane round
//   MLP_TEST_PROFILE_SPLIT    profile posterior: rows per workgroup split
// Diagnosis (stderr):
//   MLP_LOG_RELAX             wall time of a consistency round's phases
//   MLP_LOG_PLAN              the relaxation's tile plan
//   MLP_LOG_PROFILE           profile posterior host / device seconds at teardown
#pragma once

namespace mlp {
// the variable's value, read at the call (callers on hot paths keep it in a
// static); the default when unset or empty.  Names outside the registry abort.
double knob(const char* name, double dflt);
bool knob_set(const char* name);
const char* knob_str(const char* name);  // nullptr when unset
}  // namespace mlp
