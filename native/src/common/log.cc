#include "common/log.h"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <mutex>
#include <string>
#include <sys/time.h>

#include "common/status.h"

namespace adp {
namespace {

LogLevel InitialLevel() {
  const char* e = std::getenv("ADP_LOG_LEVEL");
  if (!e) return LogLevel::kInfo;
  if (!strcasecmp(e, "debug")) return LogLevel::kDebug;
  if (!strcasecmp(e, "warn") || !strcasecmp(e, "warning")) return LogLevel::kWarn;
  if (!strcasecmp(e, "error")) return LogLevel::kError;
  return LogLevel::kInfo;
}

std::atomic<int> g_level{static_cast<int>(InitialLevel())};
std::mutex g_mu;
// ADP_LOG_FORMAT=json: one JSON object per line for log pipelines.
const bool g_json = [] {
  const char* e = std::getenv("ADP_LOG_FORMAT");
  return e && !strcasecmp(e, "json");
}();

const char* LevelWord(LogLevel l) {
  switch (l) {
    case LogLevel::kDebug: return "debug";
    case LogLevel::kInfo: return "info";
    case LogLevel::kWarn: return "warn";
    case LogLevel::kError: return "error";
  }
  return "unknown";
}

std::string JsonStr(const char* s) {
  std::string o = "\"";
  for (const char* p = s; *p; ++p) {
    unsigned char c = static_cast<unsigned char>(*p);
    if (c == '"' || c == '\\') { o += '\\'; o += static_cast<char>(c); }
    else if (c == '\n') o += "\\n";
    else if (c == '\t') o += "\\t";
    else if (c < 0x20) { char b[8]; snprintf(b, sizeof(b), "\\u%04x", c); o += b; }
    else o += static_cast<char>(c);
  }
  return o + "\"";
}

const char* LevelName(LogLevel l) {
  switch (l) {
    case LogLevel::kDebug: return "D";
    case LogLevel::kInfo: return "I";
    case LogLevel::kWarn: return "W";
    case LogLevel::kError: return "E";
  }
  return "?";
}

}  // namespace

void SetLogLevel(LogLevel l) { g_level.store(static_cast<int>(l)); }
namespace {
thread_local int t_quiet = 0;
}  // namespace

QuietLogs::QuietLogs() { ++t_quiet; }
QuietLogs::~QuietLogs() { --t_quiet; }

bool LogEnabled(LogLevel l) {
  if (t_quiet > 0 && l < LogLevel::kError) return false;
  return static_cast<int>(l) >= g_level.load(std::memory_order_relaxed);
}

void Logf(LogLevel l, const char* component, const char* fmt, ...) {
  // Most lines fit the stack buffer; longer ones (SIGUSR1 stats with a
  // latency histogram) are formatted again into a string, never truncated.
  char small[4096];
  std::string big;
  const char* msg = small;
  va_list ap, ap2;
  va_start(ap, fmt);
  va_copy(ap2, ap);
  int n = vsnprintf(small, sizeof(small), fmt, ap);
  va_end(ap);
  if (n >= static_cast<int>(sizeof(small))) {
    big.resize(static_cast<size_t>(n));
    vsnprintf(big.data(), big.size() + 1, fmt, ap2);
    msg = big.c_str();
  }
  va_end(ap2);
  struct timeval tv;
  gettimeofday(&tv, nullptr);
  struct tm tm;
  gmtime_r(&tv.tv_sec, &tm);
  char ts[32];
  strftime(ts, sizeof(ts), "%Y-%m-%dT%H:%M:%S", &tm);
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_json) {
    fprintf(stderr, "{\"ts\": \"%s.%06ldZ\", \"level\": \"%s\", \"component\": %s, \"msg\": %s}\n", ts,
            static_cast<long>(tv.tv_usec), LevelWord(l), JsonStr(component).c_str(), JsonStr(msg).c_str());
  } else {
    fprintf(stderr, "%s.%06ldZ %s %s: %s\n", ts, static_cast<long>(tv.tv_usec), LevelName(l), component, msg);
  }
  fflush(stderr);
}

const char* CodeName(Code c) {
  switch (c) {
    case Code::kOk: return "OK";
    case Code::kInvalidArgument: return "INVALID_ARGUMENT";
    case Code::kNotFound: return "NOT_FOUND";
    case Code::kAlreadyExists: return "ALREADY_EXISTS";
    case Code::kFailedPrecondition: return "FAILED_PRECONDITION";
    case Code::kUnavailable: return "UNAVAILABLE";
    case Code::kUnimplemented: return "UNIMPLEMENTED";
    case Code::kInternal: return "INTERNAL";
    case Code::kDeadlineExceeded: return "DEADLINE_EXCEEDED";
    case Code::kNotSupported: return "NOT_SUPPORTED";
    case Code::kPermissionDenied: return "PERMISSION_DENIED";
  }
  return "UNKNOWN";
}

std::string Status::ToString() const {
  if (ok()) return "OK";
  return std::string(CodeName(code_)) + ": " + msg_;
}

}  // namespace adp
