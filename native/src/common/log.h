// Structured, thread-safe logging.
//
// The reference logs with Go's `log` package to stdout/stderr
// (cmd/nvidia-device-plugin/main.go:134,221,272; server.go:105,261,326). We log
// one line per event as `ts level component: message`, to stderr, with a level
// threshold taken from ADP_LOG_LEVEL (debug|info|warn|error; default info).
// Logging must never sit on the Allocate hot path at info level: the reference
// prints a line per Allocate call (server.go:326); we print it at debug.
#pragma once

#include <cstdarg>

namespace adp {

enum class LogLevel { kDebug = 0, kInfo = 1, kWarn = 2, kError = 3 };

void SetLogLevel(LogLevel l);
bool LogEnabled(LogLevel l);
void Logf(LogLevel l, const char* component, const char* fmt, ...)
    __attribute__((format(printf, 3, 4)));

// While one lives, this thread logs errors only (e.g. objects built just to
// look at what they would do; other threads log as before).
class QuietLogs {
 public:
  QuietLogs();
  ~QuietLogs();
  QuietLogs(const QuietLogs&) = delete;
  QuietLogs& operator=(const QuietLogs&) = delete;
};

}  // namespace adp

#define ADP_LOG(level, comp, ...)                                  \
  do {                                                             \
    if (::adp::LogEnabled(level)) ::adp::Logf(level, comp, __VA_ARGS__); \
  } while (0)
#define LOG_DEBUG(comp, ...) ADP_LOG(::adp::LogLevel::kDebug, comp, __VA_ARGS__)
#define LOG_INFO(comp, ...) ADP_LOG(::adp::LogLevel::kInfo, comp, __VA_ARGS__)
#define LOG_WARN(comp, ...) ADP_LOG(::adp::LogLevel::kWarn, comp, __VA_ARGS__)
#define LOG_ERROR(comp, ...) ADP_LOG(::adp::LogLevel::kError, comp, __VA_ARGS__)
