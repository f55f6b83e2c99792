// One accepted gRPC connection (internal to the grpc module). Server owns a
// ServerConn per accepted socket on the loop that serves it; the HTTP/2 engine
// behind it is either the native one (h2_conn.cc, the default) or nghttp2's
// session layer (server.cc, --http2-server nghttp2).
#pragma once

#include <memory>
#include <string>
#include <string_view>
#include <time.h>

#include "grpc/grpc.h"

namespace adp::grpc {

class ServerConn {
 public:
  ServerConn(Server* srv, int loop, int fd) : srv_(srv), loop_(loop), fd_(fd) {}
  virtual ~ServerConn() = default;
  ServerConn(const ServerConn&) = delete;
  ServerConn& operator=(const ServerConn&) = delete;

  // Queues the server preface. False: the connection is unusable (fd closed).
  virtual bool Init() = 0;
  // Reads what the socket has, processes it, writes what can be written.
  // False: close the connection.
  virtual bool OnReadable() = 0;
  // Writes queued bytes. False: close the connection.
  virtual bool Flush() = 0;
  // Nothing left to do: the peer went away cleanly or a connection error was sent.
  virtual bool Done() const = 0;
  virtual bool want_epollout() const = 0;
  // Used by ServerStream (loop thread only).
  virtual bool QueueMessage(int32_t sid, std::string_view msg) = 0;
  virtual void Finish(int32_t sid, const Status& st) = 0;

  int fd() const { return fd_; }
  uint32_t epoll_events = 0;  // interest set currently registered with epoll

 protected:
  // Server and ServerStream internals; this base class is their friend.
  const UnaryHandler* FindUnary(std::string_view path) const {
    auto it = srv_->unary_.find(path);
    return it == srv_->unary_.end() ? nullptr : &it->second;
  }
  const StreamHandler* FindStreamHandler(std::string_view path) const {
    auto it = srv_->streams_.find(path);
    return it == srv_->streams_.end() ? nullptr : &it->second;
  }
  bool tracing() const { return srv_->trace_; }
  const std::string& server_name() const { return srv_->name_; }
  void CountCall() { srv_->stats_.calls.Add(1); }
  void CountError() { srv_->stats_.errors.Add(1); }
  std::shared_ptr<ServerStream> OpenStream(int32_t sid) {
    auto s = std::make_shared<ServerStream>();
    s->conn_ = this;
    s->stream_id_ = sid;
    s->id_ = srv_->next_stream_id_.fetch_add(1, std::memory_order_relaxed);
    s->loop_ = loop_;
    return s;
  }
  static void Detach(ServerStream* s) {
    if (s) {
      s->closed_ = true;
      s->conn_ = nullptr;
    }
  }
  static bool StreamClosed(const ServerStream& s) { return s.closed_; }

  // The request of a call as gRPC frames it: exactly one uncompressed
  // length-prefixed message (an empty body is an empty message). On a bad
  // request returns false with the gRPC status to answer in *code / *msg.
  static bool ParseRequest(bool grpc_content_type, std::string_view content_type, std::string_view body,
                           std::string_view* req, int* code, std::string* msg);
  // Runs a unary handler into *resp (cleared first), logging it when traced.
  Status RunUnary(const UnaryHandler& h, std::string_view path, std::string_view req, std::string* resp);

  // Residency of unary calls in the daemon, from the read that carried them to
  // their reply handed to send() (ServerStats::residency): the engine calls
  // ReadStarted() when a readable event starts, Answered() when a unary call
  // got its reply queued and Sending() before writing the queued bytes. One
  // sample per batch of calls answered together, from the start of the read
  // that carried the first of them. The send itself is left out: on a UDS it
  // wakes the peer inside the syscall, so the client can be running with the
  // reply before send() returns.
  static uint64_t MonoNs() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return static_cast<uint64_t>(ts.tv_sec) * 1000000000ull + static_cast<uint64_t>(ts.tv_nsec);
  }
  void ReadStarted() { read_ns_ = MonoNs(); }
  void Answered() {
    if (!answers_++) batch_ns_ = read_ns_;
  }
  void Sending() {
    if (answers_) {
      srv_->stats_.residency.Observe(MonoNs() - batch_ns_);
      answers_ = 0;
    }
  }

  Server* srv_;
  int loop_;
  int fd_;
  uint64_t read_ns_ = 0, batch_ns_ = 0;
  uint32_t answers_ = 0;
};

std::unique_ptr<ServerConn> MakeH2Conn(Server* srv, int loop, int fd);
std::unique_ptr<ServerConn> MakeNghttp2Conn(Server* srv, int loop, int fd);

}  // namespace adp::grpc
