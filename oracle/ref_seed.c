/*
 * ORACLE TEST INFRASTRUCTURE -- seed hook for oracle/_ref/refharness only.
 * See ref_seed_shim.h.  RFX_SPHERE_SEED pins the Vector3.cpp stream
 * (trace_math.h:34 via Vector3.cpp), RFX_JITTER_SEED the Render.cpp stream.
 * Unset -> the real glibc rand() value, i.e. the unmodified behaviour.
 */
#include <stdlib.h>
#include <string.h>

static int ends_with(const char *s, const char *suffix)
{
  size_t n = strlen(s), m = strlen(suffix);
  return n >= m && !strcmp(s + n - m, suffix);
}

int rfx_ref_seed(const char *tu)
{
  int real = rand();  /* keep the glibc sequence advancing exactly as unshimmed */
  const char *env = NULL;
  if (ends_with(tu, "/Vector3.cpp")) env = getenv("RFX_SPHERE_SEED");
  else if (ends_with(tu, "/Render.cpp")) env = getenv("RFX_JITTER_SEED");
  if (env && *env) return (int)(unsigned)strtoul(env, NULL, 0);
  return real;
}
