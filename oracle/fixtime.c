/* oracle/fixtime.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A clock for the reference CLI's -p 1 refinement, which reseeds rand() with
 * srand(time(0)) on every pass (CPNP/MSA.cpp:1896): linked into
 * _ref/c_p_np_aln_ft ahead of the C library, time() returns REF_FIXED_TIME
 * (seconds) so a golden output is reproducible.  The drop-in reads the same
 * value from MLP_SRAND_TIME.
 */
#include <stdlib.h>
#include <time.h>

time_t time(time_t *t) {
  const char *e = getenv("REF_FIXED_TIME");
  const time_t v = e ? (time_t)atoll(e) : (time_t)1700000000;
  if (t) *t = v;
  return v;
}
