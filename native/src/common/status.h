// Error model for the whole daemon: nothing below main() panics or exits.
//
// The reference crashes the process on any device-library error
// (cmd/nvidia-device-plugin/nvidia.go:65-69, `check()` -> log.Panicln) and relies
// on the DaemonSet restarting it (defect B16). Every fallible call here returns a
// Status or a Result<T> instead, and the supervisor decides what to do.
#pragma once

#include <string>
#include <utility>
#include <variant>

namespace adp {

enum class Code {
  kOk = 0,
  kInvalidArgument,
  kNotFound,
  kAlreadyExists,
  kFailedPrecondition,
  kUnavailable,
  kUnimplemented,
  kInternal,
  kDeadlineExceeded,
  kNotSupported,
  kPermissionDenied,
};

const char* CodeName(Code c);

class Status {
 public:
  Status() = default;
  Status(Code code, std::string msg) : code_(code), msg_(std::move(msg)) {}

  static Status Ok() { return Status(); }
  bool ok() const { return code_ == Code::kOk; }
  Code code() const { return code_; }
  const std::string& message() const { return msg_; }
  std::string ToString() const;

 private:
  Code code_ = Code::kOk;
  std::string msg_;
};

inline Status InvalidArgument(std::string m) { return Status(Code::kInvalidArgument, std::move(m)); }
inline Status NotFound(std::string m) { return Status(Code::kNotFound, std::move(m)); }
inline Status FailedPrecondition(std::string m) { return Status(Code::kFailedPrecondition, std::move(m)); }
inline Status Unavailable(std::string m) { return Status(Code::kUnavailable, std::move(m)); }
inline Status Internal(std::string m) { return Status(Code::kInternal, std::move(m)); }
inline Status Unimplemented(std::string m) { return Status(Code::kUnimplemented, std::move(m)); }
inline Status DeadlineExceeded(std::string m) { return Status(Code::kDeadlineExceeded, std::move(m)); }
inline Status NotSupported(std::string m) { return Status(Code::kNotSupported, std::move(m)); }

// Minimal expected<T, Status>.
template <typename T>
class Result {
 public:
  Result(T value) : v_(std::move(value)) {}            // NOLINT(implicit)
  Result(Status status) : v_(std::move(status)) {}     // NOLINT(implicit)

  bool ok() const { return v_.index() == 0; }
  const Status& status() const {
    static const Status kOk;
    return ok() ? kOk : std::get<1>(v_);
  }
  T& value() & { return std::get<0>(v_); }
  const T& value() const& { return std::get<0>(v_); }
  T&& value() && { return std::get<0>(std::move(v_)); }
  T* operator->() { return &std::get<0>(v_); }
  const T* operator->() const { return &std::get<0>(v_); }
  T& operator*() & { return std::get<0>(v_); }
  const T& operator*() const& { return std::get<0>(v_); }

 private:
  std::variant<T, Status> v_;
};

#define ADP_RETURN_IF_ERROR(expr)           \
  do {                                      \
    ::adp::Status _st = (expr);             \
    if (!_st.ok()) return _st;              \
  } while (0)

}  // namespace adp
