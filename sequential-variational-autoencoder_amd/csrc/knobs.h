// Tuning switches for same-box A/B experiments.
//
// The shipping library (the default build) compiles every switch to its default value: it reads no
// environment variable, so nothing in a caller's environment can change what a step computes or how
// it is scheduled.  A build with -DSVAE_KNOBS (libsvae_hip_knobs.so, built by build.py --knobs; used by
// tools/gpu/ab.sh and by the tests that hold an alternative path bitwise to the default) reads
// SVAE_<NAME> instead: once per process where the call site caches it in a static, per context where
// svae_create stores it.
#pragma once
#include <cstdlib>

#ifdef SVAE_KNOBS
static inline int svae_knob(const char* name, int def) {
  const char* e = getenv(name);
  return e ? atoi(e) : def;
}
#else
static constexpr int svae_knob(const char*, int def) { return def; }
#endif
