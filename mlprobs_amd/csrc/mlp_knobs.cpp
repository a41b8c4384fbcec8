// mlp_knobs.cpp -- the registry of mlp_knobs.h: the one place libmlpgpu reads
// its environment.
#include "mlp_knobs.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace mlp {
namespace {

const char* const kKnobs[] = {
    // settings
    "MLP_SCRATCH_GB", "MLP_HOST_THREADS", "MLP_POOL_KEEP_GB",
    // test hooks
    "MLP_TEST_PG_SEPARATE", "MLP_TEST_TOT_LANEFOLD", "MLP_TEST_TOT_FOLDBOUND", "MLP_TEST_TOT_BESIDE",
    "MLP_TEST_TOT_FORCE_REPAIR", "MLP_TEST_DEFER_FINISH", "MLP_TEST_FORCE_PEER", "MLP_TEST_ALLGATHER_FORCE",
    "MLP_TEST_MEA_SPINS", "MLP_TEST_RELAX_PATH", "MLP_TEST_RELAX_TILE", "MLP_TEST_RELAX_KP", "MLP_TEST_RELAX_LDS_KB",
    "MLP_TEST_RELAX_SMALL_KB", "MLP_TEST_RELAX_SPLIT_Z", "MLP_TEST_RELAX_GLOBAL_Z", "MLP_TEST_PROFILE_STAGE",
    "MLP_TEST_PROFILE_SPLIT",
    // diagnosis
    "MLP_LOG_RELAX", "MLP_LOG_PLAN", "MLP_LOG_PROFILE",
};

const char* lookup(const char* name) {
  for (const char* k : kKnobs)
    if (!strcmp(k, name)) {
      const char* v = getenv(name);
      return v && *v ? v : nullptr;
    }
  fprintf(stderr, "libmlpgpu: %s is not in the knob registry (mlp_knobs.h)\n", name);
  abort();
}

}  // namespace

double knob(const char* name, double dflt) {
  const char* v = lookup(name);
  return v ? atof(v) : dflt;
}

bool knob_set(const char* name) { return lookup(name) != nullptr; }

const char* knob_str(const char* name) { return lookup(name); }

}  // namespace mlp
