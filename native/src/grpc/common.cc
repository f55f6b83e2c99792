#include <cctype>
#include <cstdio>

#include "grpc/grpc.h"

namespace adp::grpc {

int ToGrpcCode(Code c) {
  switch (c) {
    case Code::kOk: return kGrpcOk;
    case Code::kInvalidArgument: return kGrpcInvalidArgument;
    case Code::kNotFound: return kGrpcNotFound;
    case Code::kAlreadyExists: return kGrpcAlreadyExists;
    case Code::kFailedPrecondition: return kGrpcFailedPrecondition;
    case Code::kUnavailable: return kGrpcUnavailable;
    case Code::kUnimplemented: return kGrpcUnimplemented;
    case Code::kInternal: return kGrpcInternal;
    case Code::kDeadlineExceeded: return kGrpcDeadlineExceeded;
    case Code::kNotSupported: return kGrpcUnimplemented;
    case Code::kPermissionDenied: return kGrpcPermissionDenied;
  }
  return kGrpcUnknown;
}

Code FromGrpcCode(int g) {
  switch (g) {
    case kGrpcOk: return Code::kOk;
    case kGrpcInvalidArgument: return Code::kInvalidArgument;
    case kGrpcNotFound: return Code::kNotFound;
    case kGrpcAlreadyExists: return Code::kAlreadyExists;
    case kGrpcFailedPrecondition: return Code::kFailedPrecondition;
    case kGrpcUnavailable: return Code::kUnavailable;
    case kGrpcUnimplemented: return Code::kUnimplemented;
    case kGrpcDeadlineExceeded: return Code::kDeadlineExceeded;
    case kGrpcPermissionDenied: return Code::kPermissionDenied;
    default: return Code::kInternal;
  }
}

void FrameMessage(std::string_view msg, std::string* out) {
  uint32_t n = static_cast<uint32_t>(msg.size());
  char hdr[5] = {0, static_cast<char>(n >> 24), static_cast<char>(n >> 16),
                 static_cast<char>(n >> 8), static_cast<char>(n)};
  out->append(hdr, 5);
  out->append(msg.data(), msg.size());
}

std::string PercentEncode(std::string_view s) {
  // grpc-message: printable ASCII except '%' passes through (gRPC HTTP/2 spec).
  std::string out;
  for (unsigned char c : s) {
    if (c >= 0x20 && c <= 0x7e && c != '%') {
      out += static_cast<char>(c);
    } else {
      char buf[4];
      snprintf(buf, sizeof(buf), "%%%02X", c);
      out += buf;
    }
  }
  return out;
}

std::string PercentDecode(std::string_view s) {
  std::string out;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size() &&
        std::isxdigit(static_cast<unsigned char>(s[i + 1])) &&
        std::isxdigit(static_cast<unsigned char>(s[i + 2]))) {
      out += static_cast<char>(std::stoi(std::string(s.substr(i + 1, 2)), nullptr, 16));
      i += 2;
    } else {
      out += s[i];
    }
  }
  return out;
}

}  // namespace adp::grpc
