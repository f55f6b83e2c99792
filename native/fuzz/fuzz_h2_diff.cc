// Differential fuzzing (libFuzzer) of the two HTTP/2 engines of the plugin
// sockets: the native one (grpc/h2_conn.cc, the default) and nghttp2's session
// layer (--http2-server nghttp2). The same client bytes go to both; when both
// connections survive the input, every call that completed on either (its
// trailers sent) must have completed on both with the same grpc-status and the
// same response message bytes. Inputs one engine refuses and the other
// tolerates are not compared (nghttp2 validates more of HTTP messaging), nor
// are streams either side reset: a stream error (e.g. a window update past
// 2^31-1) or the client's RST_STREAM may land before or after the answer went
// out, depending on when an engine writes.
//
// Seeds: tools/gen_fuzz_seeds.py (shared with fuzz_h2).
#include <nghttp2/nghttp2.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <memory>
#include <string>

#include "common/log.h"
#include "grpc/grpc.h"
#include "grpc/server_conn.h"

using namespace adp;

namespace {

grpc::Server& Srv() {
  static grpc::Server* s = [] {
    SetLogLevel(LogLevel::kError);
    auto* srv = new grpc::Server("fuzz-diff");
    srv->AddUnary("/t.S/Echo", [](std::string_view q, std::string* r) {
      r->assign(q);
      return Status::Ok();
    });
    srv->AddUnary("/t.S/Fail", [](std::string_view, std::string*) { return InvalidArgument("no"); });
    srv->AddServerStream("/t.S/Watch", [](std::string_view, std::shared_ptr<grpc::ServerStream> st) {
      st->Send("first");
      st->Send(std::string(3000, 'w'));
      return Status::Ok();
    });
    return srv;
  }();
  return *s;
}

struct Call {
  std::string data;         // DATA payloads, padding removed
  std::string grpc_status;  // from the trailers ("" = not completed)
  bool reset = false;       // the server reset the stream (RST_STREAM)
};

struct Outcome {
  bool alive = false;
  std::map<uint32_t, Call> calls;
};

// Splits the server's bytes into frames and decodes its header blocks.
void ParseServerBytes(const std::string& out, Outcome* o) {
  nghttp2_hd_inflater* inf = nullptr;
  if (nghttp2_hd_inflate_new(&inf) != 0) return;
  size_t off = 0;
  std::string block;
  uint32_t block_sid = 0;
  while (off + 9 <= out.size()) {
    const auto* h = reinterpret_cast<const uint8_t*>(out.data() + off);
    size_t len = (size_t{h[0]} << 16) | (size_t{h[1]} << 8) | h[2];
    uint8_t type = h[3], flags = h[4];
    uint32_t sid = ((uint32_t{h[5]} << 24) | (uint32_t{h[6]} << 16) | (uint32_t{h[7]} << 8) | h[8]) & 0x7fffffffu;
    if (off + 9 + len > out.size()) break;
    std::string payload = out.substr(off + 9, len);
    off += 9 + len;
    if (type == 3 /*RST_STREAM*/) {
      o->calls[sid].reset = true;
    } else if (type == 0 /*DATA*/) {
      if (flags & 0x8) {  // PADDED
        if (payload.empty()) continue;
        size_t pad = static_cast<uint8_t>(payload[0]);
        payload = pad + 1 <= payload.size() ? payload.substr(1, payload.size() - 1 - pad) : "";
      }
      o->calls[sid].data += payload;
    } else if (type == 1 /*HEADERS*/ || type == 9 /*CONTINUATION*/) {
      if (type == 1) {
        size_t skip = 0, pad = 0;
        if (flags & 0x8) { pad = payload.empty() ? 0 : static_cast<uint8_t>(payload[0]); skip = 1; }
        if (flags & 0x20) skip += 5;
        payload = skip + pad <= payload.size() ? payload.substr(skip, payload.size() - skip - pad) : "";
        block.clear();
        block_sid = sid;
      }
      block += payload;
      if (!(flags & 0x4)) continue;  // END_HEADERS
      const auto* in = reinterpret_cast<const uint8_t*>(block.data());
      size_t left = block.size();
      while (true) {
        nghttp2_nv nv;
        int iflags = 0;
        ssize_t rv = nghttp2_hd_inflate_hd2(inf, &nv, &iflags, in, left, 1);
        if (rv < 0) break;
        in += rv;
        left -= static_cast<size_t>(rv);
        if (iflags & NGHTTP2_HD_INFLATE_EMIT) {
          std::string name(reinterpret_cast<const char*>(nv.name), nv.namelen);
          if (name == "grpc-status")
            o->calls[block_sid].grpc_status.assign(reinterpret_cast<const char*>(nv.value), nv.valuelen);
        }
        if (iflags & NGHTTP2_HD_INFLATE_FINAL) {
          nghttp2_hd_inflate_end_headers(inf);
          break;
        }
        if (rv == 0 && left == 0) break;
      }
    }
  }
  nghttp2_hd_inflate_del(inf);
}

// Streams the client itself reset (RST_STREAM in its bytes, read frame by
// frame as far as they parse): whether an answer went out first is timing.
std::set<uint32_t> ClientResets(const std::string& in, size_t preface) {
  std::set<uint32_t> out;
  for (size_t off = preface; off + 9 <= in.size();) {
    const auto* h = reinterpret_cast<const uint8_t*>(in.data() + off);
    size_t len = (size_t{h[0]} << 16) | (size_t{h[1]} << 8) | h[2];
    uint32_t sid = ((uint32_t{h[5]} << 24) | (uint32_t{h[6]} << 16) | (uint32_t{h[7]} << 8) | h[8]) & 0x7fffffffu;
    if (h[3] == 3 /*RST_STREAM*/) out.insert(sid);
    off += 9 + len;
  }
  return out;
}

Outcome Run(bool native, const std::string& in, size_t chunk) {
  Outcome o;
  int sv[2];
  if (socketpair(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0, sv) != 0) return o;
  auto conn = native ? grpc::MakeH2Conn(&Srv(), 0, sv[1]) : grpc::MakeNghttp2Conn(&Srv(), 0, sv[1]);
  if (!conn->Init()) {
    close(sv[0]);
    return o;
  }
  std::string out;
  char sink[1 << 16];
  auto drain = [&] {
    ssize_t r;
    while ((r = read(sv[0], sink, sizeof(sink))) > 0) out.append(sink, static_cast<size_t>(r));
  };
  bool alive = true;
  for (size_t off = 0; alive && off < in.size();) {
    ssize_t w = write(sv[0], in.data() + off, std::min(chunk, in.size() - off));
    if (w > 0) off += static_cast<size_t>(w);
    alive = conn->OnReadable() && !conn->Done();
    drain();
    if (w <= 0) alive = alive && conn->Flush();
  }
  for (int i = 0; alive && i < 8; ++i) {
    alive = conn->Flush() && !conn->Done();
    drain();
  }
  o.alive = alive;
  conn.reset();
  drain();
  close(sv[0]);
  ParseServerBytes(out, &o);
  return o;
}

}  // namespace

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  static const char kPreface[] = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n\0\0\0\4\0\0\0\0\0";
  std::string in(kPreface, sizeof(kPreface) - 1);
  size_t chunk = size ? (size_t{1} << (data[0] & 15)) : 1;
  if (size) in.append(reinterpret_cast<const char*>(data + 1), size - 1);
  Outcome a = Run(true, in, chunk), b = Run(false, in, chunk);
  static const bool verbose = getenv("ADP_FUZZ_VERBOSE") != nullptr;
  if (verbose)
    for (const Outcome* x : {&a, &b})
      for (const auto& [sid, call] : x->calls)
        fprintf(stderr, "%s alive=%d stream %u status '%s' %zu bytes\n", x == &a ? "native" : "nghttp2", x->alive,
                sid, call.grpc_status.c_str(), call.data.size());
  if (!a.alive || !b.alive) return 0;
  const std::set<uint32_t> client_reset = ClientResets(in, sizeof(kPreface) - 1 - 9);
  for (const Outcome* x : {&a, &b}) {
    const Outcome* y = x == &a ? &b : &a;
    for (const auto& [sid, call] : x->calls) {
      if (call.grpc_status.empty() || call.reset || client_reset.count(sid)) continue;
      auto it = y->calls.find(sid);
      if (it != y->calls.end() && it->second.reset) continue;
      if (it == y->calls.end() || it->second.grpc_status != call.grpc_status || it->second.data != call.data) {
        fprintf(stderr, "engines disagree on stream %u: native status '%s' %zu bytes, nghttp2 status '%s' %zu bytes\n",
                sid, a.calls[sid].grpc_status.c_str(), a.calls[sid].data.size(), b.calls[sid].grpc_status.c_str(),
                b.calls[sid].data.size());
        abort();
      }
    }
  }
  return 0;
}
