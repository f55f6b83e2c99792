// Coverage-guided fuzzing (libFuzzer) of the daemon's gRPC client
// (grpc/client.cc) -- what a kubelet, or anything bound at the kubelet or
// PodResources socket path, answers the daemon. The input follows the server's
// empty SETTINGS frame on a socketpair whose far end is then shut for writing;
// the client runs one unary call (input byte 0 even) or one server stream (odd)
// against it. Invariants: no crash, no out-of-bounds read, no leak, no hang;
// a successful call's message is within the client's receive bound, and a
// stream yields at most as many messages as the input could frame.
#include <sys/socket.h>
#include <unistd.h>

#include <cstdlib>
#include <string>

#include "common/log.h"
#include "grpc/grpc.h"

using namespace adp;

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  static bool quiet = [] {
    SetLogLevel(LogLevel::kError);
    return true;
  }();
  (void)quiet;
  int sv[2];
  if (socketpair(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0, sv) != 0) return 0;
  static const char kSettings[] = "\0\0\0\4\0\0\0\0\0";
  std::string in(kSettings, sizeof(kSettings) - 1);
  const bool stream = size && (data[0] & 1);
  if (size) in.append(reinterpret_cast<const char*>(data + 1), size - 1);
  for (size_t off = 0; off < in.size();) {
    ssize_t w = write(sv[0], in.data() + off, in.size() - off);
    if (w <= 0) break;  // the socket buffer is full: the rest is dropped
    off += static_cast<size_t>(w);
  }
  shutdown(sv[0], SHUT_WR);
  auto ch = grpc::Channel::FromFd(sv[1], 50);  // owns sv[1]
  if (ch.ok()) {
    if (!stream) {
      std::string resp;
      Status st = (*ch)->Unary("/t.S/Echo", "ping", &resp, 50);
      if (st.ok() && resp.size() > in.size()) abort();  // a message is never more than the peer sent
    } else {
      auto sid = (*ch)->StartStream("/t.S/Watch", "ping");
      size_t n = 0;
      std::string msg;
      while (sid.ok() && (*ch)->Recv(*sid, &msg, 50).ok()) {
        if (++n > in.size() / 5 + 1) abort();  // every message costs a 5-byte prefix
      }
    }
  }  // (a failed handshake closed sv[1] with the channel)
  close(sv[0]);
  return 0;
}
