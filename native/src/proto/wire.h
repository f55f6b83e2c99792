// Protocol-buffers wire format (proto3 subset) -- hand-written, no libprotobuf.
//
// The reference links gogo/golang protobuf runtimes (~26k LoC vendored, SURVEY
// V15). The kubelet device-plugin API only needs varints, length-delimited
// fields, nested messages and map<string,string> entries, so this is a few
// hundred lines. Encoding is append-only into a std::string so the Allocate path
// can splice pre-encoded fragments (see plugin/plugin.cc).
#pragma once

#include <cstdint>
#include <string>
#include <string_view>

namespace adp::pb {

enum WireType : uint32_t { kVarint = 0, kFixed64 = 1, kLen = 2, kFixed32 = 5 };

inline void PutVarint(std::string* o, uint64_t v) {
  char buf[10];
  int n = 0;
  while (v >= 0x80) {
    buf[n++] = static_cast<char>((v & 0x7f) | 0x80);
    v >>= 7;
  }
  buf[n++] = static_cast<char>(v);
  o->append(buf, n);
}
inline size_t VarintSize(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) { v >>= 7; ++n; }
  return n;
}
inline void PutTag(std::string* o, uint32_t field, WireType wt) {
  PutVarint(o, (static_cast<uint64_t>(field) << 3) | wt);
}
// Length-delimited field, always emitted (repeated elements, sub-messages).
inline void PutLen(std::string* o, uint32_t field, std::string_view bytes) {
  PutTag(o, field, kLen);
  PutVarint(o, bytes.size());
  o->append(bytes.data(), bytes.size());
}
// proto3 singular string: omitted when empty.
inline void PutStr(std::string* o, uint32_t field, std::string_view s) {
  if (!s.empty()) PutLen(o, field, s);
}
inline void PutBool(std::string* o, uint32_t field, bool v) {
  if (v) { PutTag(o, field, kVarint); o->push_back(1); }
}
inline void PutInt64(std::string* o, uint32_t field, int64_t v) {
  if (v) { PutTag(o, field, kVarint); PutVarint(o, static_cast<uint64_t>(v)); }
}
inline void PutInt32(std::string* o, uint32_t field, int32_t v) {
  // int32 is sign-extended to 64 bits on the wire.
  if (v) { PutTag(o, field, kVarint); PutVarint(o, static_cast<uint64_t>(static_cast<int64_t>(v))); }
}
// One map<string,string> entry (a length-delimited {1: key, 2: value} message).
void PutMapEntry(std::string* o, uint32_t field, std::string_view k, std::string_view v);

class Reader {
 public:
  explicit Reader(std::string_view buf) : p_(buf.data()), end_(buf.data() + buf.size()) {}
  // Advances to the next field. Returns false at end of buffer or on error
  // (check ok()).
  bool Next(uint32_t* field, WireType* wt) {
    if (!ok_ || p_ >= end_) return false;
    uint64_t tag;
    if (!ReadVarint(&tag)) return false;
    *field = static_cast<uint32_t>(tag >> 3);
    *wt = static_cast<WireType>(tag & 7);
    if (*field == 0) { ok_ = false; return false; }
    return true;
  }
  // Inline one-byte fast path: every tag and most lengths in the kubelet API
  // (device IDs are < 128 bytes) are single-byte varints.
  bool ReadVarint(uint64_t* v) {
    if (p_ < end_ && !(static_cast<uint8_t>(*p_) & 0x80)) {
      *v = static_cast<uint8_t>(*p_++);
      return true;
    }
    return ReadVarintSlow(v);
  }
  bool ReadLen(std::string_view* v) {
    uint64_t n;
    if (!ReadVarint(&n)) return false;
    if (n > static_cast<uint64_t>(end_ - p_)) { ok_ = false; return false; }
    *v = std::string_view(p_, n);
    p_ += n;
    return true;
  }
  bool Skip(WireType wt);
  bool ok() const { return ok_; }
  size_t remaining() const { return static_cast<size_t>(end_ - p_); }

 private:
  bool ReadVarintSlow(uint64_t* v);
  const char* p_;
  const char* end_;
  bool ok_ = true;
};

}  // namespace adp::pb
