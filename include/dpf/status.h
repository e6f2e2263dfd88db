// status.h -- Status / StatusOr with absl's codes and semantics, so that the
// DistributedPointFunction API keeps the reference's error contract
// (dpf/status_macros.h:24-49; error codes listed in SURVEY.md section 5).
#ifndef DPF_STATUS_H_
#define DPF_STATUS_H_

#include <optional>
#include <string>
#include <utility>

namespace distributed_point_functions {

enum class StatusCode : int {
  kOk = 0,
  kCancelled = 1,
  kUnknown = 2,
  kInvalidArgument = 3,
  kDeadlineExceeded = 4,
  kNotFound = 5,
  kAlreadyExists = 6,
  kPermissionDenied = 7,
  kResourceExhausted = 8,
  kFailedPrecondition = 9,
  kAborted = 10,
  kOutOfRange = 11,
  kUnimplemented = 12,
  kInternal = 13,
  kUnavailable = 14,
  kDataLoss = 15,
  kUnauthenticated = 16,
};

const char* StatusCodeToString(StatusCode code);

class [[nodiscard]] Status {
 public:
  Status() = default;
  Status(StatusCode code, std::string message)
      : code_(code), message_(code == StatusCode::kOk ? std::string() : std::move(message)) {}
  bool ok() const { return code_ == StatusCode::kOk; }
  StatusCode code() const { return code_; }
  int raw_code() const { return static_cast<int>(code_); }
  const std::string& message() const { return message_; }
  std::string ToString() const {
    if (ok()) return "OK";
    return std::string(StatusCodeToString(code_)) + ": " + message_;
  }
  friend bool operator==(const Status& a, const Status& b) {
    return a.code_ == b.code_ && a.message_ == b.message_;
  }

 private:
  StatusCode code_ = StatusCode::kOk;
  std::string message_;
};

inline Status OkStatus() { return Status(); }
inline Status InvalidArgumentError(std::string m) {
  return Status(StatusCode::kInvalidArgument, std::move(m));
}
inline Status FailedPreconditionError(std::string m) {
  return Status(StatusCode::kFailedPrecondition, std::move(m));
}
inline Status UnimplementedError(std::string m) {
  return Status(StatusCode::kUnimplemented, std::move(m));
}
inline Status InternalError(std::string m) { return Status(StatusCode::kInternal, std::move(m)); }
inline Status ResourceExhaustedError(std::string m) {
  return Status(StatusCode::kResourceExhausted, std::move(m));
}
inline Status OutOfRangeError(std::string m) {
  return Status(StatusCode::kOutOfRange, std::move(m));
}

template <typename T>
class [[nodiscard]] StatusOr {
 public:
  StatusOr(const Status& s) : status_(s) {}                 // NOLINT
  StatusOr(Status&& s) : status_(std::move(s)) {}           // NOLINT
  StatusOr(const T& v) : value_(v) {}                       // NOLINT
  StatusOr(T&& v) : value_(std::move(v)) {}                 // NOLINT
  template <typename U,
            typename = std::enable_if_t<std::is_constructible_v<T, U&&> &&
                                        !std::is_same_v<std::decay_t<U>, T> &&
                                        !std::is_same_v<std::decay_t<U>, Status> &&
                                        !std::is_same_v<std::decay_t<U>, StatusOr<T>>>>
  StatusOr(U&& v) : value_(T(std::forward<U>(v))) {}        // NOLINT
  bool ok() const { return value_.has_value(); }
  const Status& status() const { return status_; }
  const T& value() const& { return *value_; }
  T& value() & { return *value_; }
  T&& value() && { return std::move(*value_); }
  const T& operator*() const& { return *value_; }
  T& operator*() & { return *value_; }
  T&& operator*() && { return std::move(*value_); }
  const T* operator->() const { return &*value_; }
  T* operator->() { return &*value_; }

 private:
  Status status_;
  std::optional<T> value_;
};

}  // namespace distributed_point_functions

#define DPF_STATUS_CONCAT_INNER_(a, b) a##b
#define DPF_STATUS_CONCAT_(a, b) DPF_STATUS_CONCAT_INNER_(a, b)

#define DPF_RETURN_IF_ERROR(expr)                                           \
  do {                                                                      \
    ::distributed_point_functions::Status _dpf_st = (expr);                 \
    if (!_dpf_st.ok()) return _dpf_st;                                      \
  } while (0)

#define DPF_ASSIGN_OR_RETURN_IMPL_(tmp, lhs, expr) \
  auto tmp = (expr);                               \
  if (!tmp.ok()) return tmp.status();              \
  lhs = std::move(tmp).value()

#define DPF_ASSIGN_OR_RETURN(lhs, expr) \
  DPF_ASSIGN_OR_RETURN_IMPL_(DPF_STATUS_CONCAT_(_dpf_statusor_, __LINE__), lhs, expr)

#endif  // DPF_STATUS_H_
