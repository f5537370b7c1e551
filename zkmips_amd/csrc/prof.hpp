// Opt-in stage timing with HIP events recorded on the stream that launches the work
// (zkm_profile_* in include/zkm_hip.h).  Disabled: one relaxed atomic load per scope.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>

namespace zkm {

extern std::atomic<bool> g_prof_on;

struct ProfScope {
    const char *name;
    hipStream_t s;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    double units;
    ProfScope(const char *n, hipStream_t st, double u = 0);
    ~ProfScope();
};

// host wall-clock of a scope (recorded as stage "host:<name>")
struct HostScope {
    const char *name;
    double t0 = -1;
    explicit HostScope(const char *n);
    ~HostScope();
};

// adds work units to a stage without timing it (e.g. permutations behind a timed stage)
void prof_add(const char *name, double units);

#define ZKM_PROF_CAT2(a, b) a##b
#define ZKM_PROF_CAT(a, b) ZKM_PROF_CAT2(a, b)
#define HPROF(name) ::zkm::HostScope ZKM_PROF_CAT(_hprof_, __LINE__)(name)
#define PROF(name, stream, units) ::zkm::ProfScope ZKM_PROF_CAT(_prof_, __LINE__)(name, stream, units)

}  // namespace zkm
