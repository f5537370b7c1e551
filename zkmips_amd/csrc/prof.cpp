// Stage timing: events are resolved lazily (zkm_profile_flush) so profiling adds no host syncs.
#include "prof.hpp"

#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/zkm_hip.h"

namespace zkm {

std::atomic<bool> g_prof_on{false};

namespace {
struct Rec { std::string name; hipEvent_t e0, e1; double units; };
struct Tot { uint64_t count = 0; double ms = 0, units = 0; };
std::mutex g_mu;
std::vector<Rec> g_pending;
std::map<std::string, Tot> g_tot;

void flush_locked() {
    for (auto &r : g_pending) {
        float ms = 0;
        if (hipEventSynchronize(r.e1) == hipSuccess && hipEventElapsedTime(&ms, r.e0, r.e1) == hipSuccess) {
            Tot &t = g_tot[r.name];
            t.count++;
            t.ms += ms;
            t.units += r.units;
        }
        (void)hipEventDestroy(r.e0);
        (void)hipEventDestroy(r.e1);
    }
    g_pending.clear();
}
}  // namespace

ProfScope::ProfScope(const char *n, hipStream_t st, double u) : name(n), s(st), units(u) {
    if (!g_prof_on.load(std::memory_order_relaxed)) return;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) { e0 = e1 = nullptr; return; }
    (void)hipEventRecord(e0, s);
}
ProfScope::~ProfScope() {
    if (!e0) return;
    (void)hipEventRecord(e1, s);
    std::lock_guard<std::mutex> g(g_mu);
    g_pending.push_back(Rec{name, e0, e1, units});
}

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
HostScope::HostScope(const char *n) : name(n) {
    if (g_prof_on.load(std::memory_order_relaxed)) t0 = now_ms();
}
HostScope::~HostScope() {
    if (t0 < 0) return;
    const double ms = now_ms() - t0;
    std::lock_guard<std::mutex> g(g_mu);
    Tot &t = g_tot[std::string("host:") + name];
    t.count++;
    t.ms += ms;
}

void prof_add(const char *name, double units) {
    if (!g_prof_on.load(std::memory_order_relaxed)) return;
    std::lock_guard<std::mutex> g(g_mu);
    Tot &t = g_tot[name];
    t.count++;
    t.units += units;
}

}  // namespace zkm

extern "C" {
void zkm_profile_enable(int on) { zkm::g_prof_on.store(on != 0); }
void zkm_profile_reset(void) {
    std::lock_guard<std::mutex> g(zkm::g_mu);
    zkm::flush_locked();
    zkm::g_tot.clear();
}
size_t zkm_profile_dump(char *buf, size_t len) {
    std::lock_guard<std::mutex> g(zkm::g_mu);
    zkm::flush_locked();
    std::string out;
    for (auto &kv : zkm::g_tot) {
        char line[256];
        snprintf(line, sizeof line, "%s %llu %.6f %.1f\n", kv.first.c_str(), (unsigned long long)kv.second.count,
                 kv.second.ms, kv.second.units);
        out += line;
    }
    if (buf && len) {
        size_t n = out.size() < len - 1 ? out.size() : len - 1;
        memcpy(buf, out.data(), n);
        buf[n] = 0;
    }
    return out.size() + 1;
}
}
