#include "common/sampler.h"

#include <cxxabi.h>
#include <dlfcn.h>
#include <signal.h>
#include <sys/time.h>
#include <ucontext.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

namespace adp {
namespace {

constexpr size_t kMaxSamples = 1 << 20;
uintptr_t* g_samples = nullptr;
std::atomic<size_t> g_count{0};
std::string* g_out = nullptr;
int g_hz = 1000;

void OnProf(int, siginfo_t*, void* ctx) {
  auto* uc = static_cast<ucontext_t*>(ctx);
  size_t i = g_count.fetch_add(1, std::memory_order_relaxed);
  if (i < kMaxSamples) g_samples[i] = static_cast<uintptr_t>(uc->uc_mcontext.gregs[REG_RIP]);
}

std::string Demangle(const char* s) {
  int status = 0;
  char* d = abi::__cxa_demangle(s, nullptr, nullptr, &status);
  std::string out = (status == 0 && d) ? d : s;
  free(d);
  return out;
}

}  // namespace

bool StartSamplerFromEnv() {
  const char* out = getenv("ADP_PROFILE_OUT");
  if (!out || !*out || g_samples) return false;
  if (const char* hz = getenv("ADP_PROFILE_HZ")) g_hz = std::max(1, atoi(hz));
  g_samples = new uintptr_t[kMaxSamples];
  g_out = new std::string(out);
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = OnProf;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGPROF, &sa, nullptr);
  itimerval it{};
  it.it_interval.tv_usec = 1000000 / g_hz;
  it.it_value = it.it_interval;
  setitimer(ITIMER_PROF, &it, nullptr);
  return true;
}

void StopSamplerAndReport() {
  if (!g_samples) return;
  itimerval it{};
  setitimer(ITIMER_PROF, &it, nullptr);
  signal(SIGPROF, SIG_IGN);
  size_t n = std::min(g_count.load(), kMaxSamples);
  std::map<std::string, size_t> by_sym, by_obj;
  for (size_t i = 0; i < n; ++i) {
    Dl_info info;
    std::string sym = "??", obj = "??";
    if (dladdr(reinterpret_cast<void*>(g_samples[i]), &info)) {
      if (info.dli_fname) {
        obj = info.dli_fname;
        size_t slash = obj.rfind('/');
        if (slash != std::string::npos) obj = obj.substr(slash + 1);
      }
      sym = info.dli_sname ? Demangle(info.dli_sname) : ("[" + obj + "]");
    }
    ++by_sym[sym];
    ++by_obj[obj];
  }
  FILE* f = fopen(g_out->c_str(), "w");
  if (f) {
    auto dump = [&](const char* title, const std::map<std::string, size_t>& m) {
      std::vector<std::pair<size_t, std::string>> v;
      for (const auto& [k, c] : m) v.emplace_back(c, k);
      std::sort(v.rbegin(), v.rend());
      fprintf(f, "== %s ==\n", title);
      for (const auto& [c, k] : v) fprintf(f, "%8zu %6.2f%%  %s\n", c, n ? 100.0 * c / n : 0.0, k.c_str());
    };
    fprintf(f, "samples %zu at %d Hz of process CPU time (%.3f CPU-s)\n", n, g_hz,
            static_cast<double>(n) / g_hz);
    dump("by shared object", by_obj);
    dump("by symbol", by_sym);
    fclose(f);
  }
  delete[] g_samples;
  g_samples = nullptr;
}

}  // namespace adp
