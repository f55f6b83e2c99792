// Coverage-guided fuzzing (libFuzzer) of the native HTTP/2 + gRPC server
// connection (grpc/h2_conn.cc) -- the bytes a kubelet, or anything else that
// can reach the plugin socket, sends. The input follows the client preface and
// an empty SETTINGS frame and is delivered in chunks whose sizes come from the
// input; the server answers into a socketpair that is drained as it goes. The
// connection may end at any point (a GOAWAY, a protocol error) but must never
// crash, read out of bounds, leak or hang. Handlers: a unary echo and a server
// stream that sends more than one flow-control window.
#include <sys/socket.h>
#include <unistd.h>

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
    auto* srv = new grpc::Server("fuzz");
    srv->AddUnary("/t.S/Echo", [](std::string_view q, std::string* r) {
      r->assign(q);
      return Status::Ok();
    });
    srv->AddUnary("/t.S/Fail", [](std::string_view, std::string*) { return InvalidArgument("no"); });
    srv->AddServerStream("/t.S/Watch", [](std::string_view, std::shared_ptr<grpc::ServerStream> st) {
      st->Send(std::string(70000, 'w'));
      st->Send("tail");
      return Status::Ok();
    });
    return srv;
  }();
  return *s;
}

}  // namespace

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  int sv[2];
  if (socketpair(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0, sv) != 0) return 0;
  auto conn = grpc::MakeH2Conn(&Srv(), 0, sv[1]);  // owns sv[1]
  if (!conn->Init()) {
    close(sv[0]);
    return 0;
  }
  static const char kPreface[] = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n\0\0\0\4\0\0\0\0\0";
  std::string in(kPreface, sizeof(kPreface) - 1);
  // First input byte: chunk size shift (1 << 0..15 bytes per write).
  size_t chunk = size ? (size_t{1} << (data[0] & 15)) : 1;
  if (size) in.append(reinterpret_cast<const char*>(data + 1), size - 1);
  char sink[1 << 16];
  bool alive = true;
  for (size_t off = 0; alive && off < in.size();) {
    ssize_t w = write(sv[0], in.data() + off, std::min(chunk, in.size() - off));
    if (w > 0) off += static_cast<size_t>(w);
    alive = conn->OnReadable() && !conn->Done();
    while (read(sv[0], sink, sizeof(sink)) > 0) {
    }
    if (w <= 0) alive = alive && conn->Flush();
  }
  // Whatever is queued (a long stream, window updates) drains or the peer goes.
  for (int i = 0; alive && i < 64 && conn->want_epollout(); ++i) {
    alive = conn->Flush();
    while (read(sv[0], sink, sizeof(sink)) > 0) {
    }
  }
  conn.reset();
  close(sv[0]);
  return 0;
}
