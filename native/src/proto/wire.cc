#include "proto/wire.h"

namespace adp::pb {

void PutMapEntry(std::string* o, uint32_t field, std::string_view k, std::string_view v) {
  // Map entries always carry both key and value on the wire (golang/grpc-go and
  // C++ protobuf both emit them even when empty), so use PutLen, not PutStr.
  size_t body = 1 + VarintSize(k.size()) + k.size() + 1 + VarintSize(v.size()) + v.size();
  PutTag(o, field, kLen);
  PutVarint(o, body);
  PutLen(o, 1, k);
  PutLen(o, 2, v);
}

bool Reader::ReadVarintSlow(uint64_t* v) {
  uint64_t r = 0;
  for (int shift = 0; shift < 64; shift += 7) {
    if (p_ >= end_) { ok_ = false; return false; }
    uint8_t b = static_cast<uint8_t>(*p_++);
    r |= static_cast<uint64_t>(b & 0x7f) << shift;
    if (!(b & 0x80)) { *v = r; return true; }
  }
  ok_ = false;
  return false;
}

bool Reader::Skip(WireType wt) {
  switch (wt) {
    case kVarint: { uint64_t d; return ReadVarint(&d); }
    case kFixed64:
      if (end_ - p_ < 8) { ok_ = false; return false; }
      p_ += 8;
      return true;
    case kLen: { std::string_view d; return ReadLen(&d); }
    case kFixed32:
      if (end_ - p_ < 4) { ok_ = false; return false; }
      p_ += 4;
      return true;
  }
  ok_ = false;  // groups (3/4) are not valid in proto3
  return false;
}

}  // namespace adp::pb
