// gRPC over HTTP/2 cleartext (h2c) on Unix-domain sockets, built on nghttp2.
//
// The kubelet talks to device plugins with gRPC over UDS (reference
// cmd/nvidia-device-plugin/server.go:113-240, grpc-go v1.29 vendored). There is
// no grpc++ in this toolchain, and a full gRPC stack is not needed: the plugin
// serves five unary/server-streaming methods and makes one unary call. This
// module implements exactly the gRPC-over-HTTP/2 protocol subset they use:
//   * 5-byte length-prefixed messages (uncompressed),
//   * `content-type: application/grpc`, `te: trailers`,
//   * status in trailers (`grpc-status`, percent-encoded `grpc-message`),
//     trailers-only responses for errors,
//   * unary and server-streaming calls (ListAndWatch stays open for the life of
//     the plugin and pushes a new device list on every health transition).
// The server's HTTP/2 connection layer is native (h2_conn.cc: framing, flow
// control, SETTINGS/PING/GOAWAY; nghttp2 only for HPACK decoding); nghttp2's
// session layer remains selectable for the server and drives the client.
//
// Threading: a Server runs N epoll loop threads; every connection is owned by
// one loop and its handlers execute inline on that loop (they are O(k)
// in-memory work, so an inline call is cheaper than any hand-off). Handlers
// may therefore run concurrently on different loops and must only read shared
// state or synchronise. Other threads inject work with Post()/PostAll().
#pragma once

#include <sched.h>
#include <sys/types.h>

#include <atomic>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

#include "common/status.h"
#include "metrics/metrics.h"

namespace adp::grpc {

// gRPC status codes (https://grpc.github.io/grpc/core/md_doc_statuscodes.html).
enum GrpcCode : int {
  kGrpcOk = 0,
  kGrpcCancelled = 1,
  kGrpcUnknown = 2,
  kGrpcInvalidArgument = 3,
  kGrpcDeadlineExceeded = 4,
  kGrpcNotFound = 5,
  kGrpcAlreadyExists = 6,
  kGrpcPermissionDenied = 7,
  kGrpcResourceExhausted = 8,
  kGrpcFailedPrecondition = 9,
  kGrpcAborted = 10,
  kGrpcOutOfRange = 11,
  kGrpcUnimplemented = 12,
  kGrpcInternal = 13,
  kGrpcUnavailable = 14,
};
int ToGrpcCode(Code c);
Code FromGrpcCode(int g);

// 5-byte gRPC message framing.
void FrameMessage(std::string_view msg, std::string* out);
std::string PercentEncode(std::string_view s);
std::string PercentDecode(std::string_view s);

class ServerConn;

// A server-streaming call that the handler keeps open. All methods must be
// called on the server's loop thread (use Server::Post from elsewhere).
class ServerStream {
 public:
  // Queues one message. Returns false once the peer has gone away. Messages are
  // state snapshots: if the peer is slow, unsent older messages are replaced by
  // the newest one (latest wins), bounding the memory a stuck client can pin.
  bool Send(std::string_view message);
  // Ends the call with trailers carrying `st`.
  void Finish(const Status& st);
  bool closed() const { return closed_; }
  uint64_t id() const { return id_; }
  int loop() const { return loop_; }  // the server loop that owns this stream

 private:
  friend class Server;
  friend class ServerConn;
  ServerConn* conn_ = nullptr;
  int32_t stream_id_ = 0;
  uint64_t id_ = 0;
  int loop_ = 0;
  bool closed_ = false;
};

using UnaryHandler = std::function<Status(std::string_view request, std::string* response)>;
using StreamHandler =
    std::function<Status(std::string_view request, std::shared_ptr<ServerStream> stream)>;

struct ServerStats {
  std::atomic<uint64_t> connections{0};  // per accept: not on the call path
  std::atomic<uint64_t> shed_connections{0};  // refused for lack of file descriptors
  metrics::Counter calls;                // per call, from every loop: sharded
  metrics::Counter errors;
  // Unary calls from the read that carried them to their reply fully written
  // (the daemon's share of what any client sees, whatever its gRPC stack).
  metrics::FineHistogram residency;
};

class Server {
 public:
  // `threads` epoll loops serve the connections: the listener lives on loop 0 and
  // accepted connections are dealt round-robin, so concurrent clients are served
  // in parallel (each connection stays on one loop for its lifetime).
  explicit Server(std::string name, int threads = 1);
  ~Server();
  Server(const Server&) = delete;
  Server& operator=(const Server&) = delete;

  void AddUnary(const std::string& path, UnaryHandler h);
  void AddServerStream(const std::string& path, StreamHandler h);

  // Removes a stale socket file, binds and listens.
  Status Listen(const std::string& socket_path);
  // Starts the loop threads. `on_fatal` runs (on a loop thread) if a loop fails
  // more than 5 times with less than an hour between failures -- the
  // reference's crash budget (server.go:177-205).
  Status Start(std::function<void()> on_fatal = nullptr);
  // Closes every connection and the listener, joins the threads. Idempotent.
  void Stop();
  // Runs `fn` on loop 0. Safe from any thread; queued before Start(), dropped
  // after Stop().
  void Post(std::function<void()> fn);
  // Runs `fn(loop)` on every loop.
  void PostAll(std::function<void(int loop)> fn);
  int loops() const { return static_cast<int>(loops_.size()); }
  bool OnLoopThread() const;
  // Per loop: the CPU it last served from (-1 = never) and its busy iterations.
  std::vector<std::pair<int, uint64_t>> LoopPlacement() const;
  const std::string& socket_path() const { return socket_path_; }
  // The socket file at socket_path() is still the one Listen() bound (not
  // removed, not replaced by another process binding the same path).
  bool OwnsSocketPath() const;
  const ServerStats& stats() const { return stats_; }
  // Log every unary call (method, status, sizes, handler time). Set before Start().
  void set_trace(bool on) { trace_ = on; }
  // Keep polling (no sleep) for this long after each burst of activity. Set before Start().
  void set_busy_poll_us(int us) { busy_poll_us_ = us < 0 ? 0 : us; }
  // HTTP/2 engine for accepted connections: the native one (default) or
  // nghttp2's session layer. Set before Start().
  void set_native_http2(bool on) { native_http2_ = on; }
  // Serve each connection from a loop thread on the L3 of the peer process's
  // last CPU (see FollowPeerL3). Set before Start().
  void set_follow_peer_l3(bool on) { follow_peer_l3_ = on; }
  // Runs on a loop after it has written what its handlers queued (once per
  // busy iteration): work that must not delay a response. Set before Start().
  void set_after_flush(std::function<void()> fn) { after_flush_ = std::move(fn); }

  // Test hook: make the next iteration of loop 0 fail as if epoll_wait errored.
  void InjectLoopFailureForTest() { inject_failure_.store(true); }

  struct Loop;

 private:
  friend class ServerConn;
  friend class ServerStream;
  Status RunLoop(Loop& l);
  void LoopMain(Loop& l);
  void AcceptAll();
  void AddConn(Loop& l, int fd);
  void FollowPeerL3(Loop& l, int pid);
  void CloseConn(Loop& l, int fd);
  void DrainPosted(Loop& l);
  void PostTo(Loop& l, std::function<void()> fn);

  std::string name_;
  std::string socket_path_;
  dev_t sock_dev_ = 0;  // identity of the socket file Listen() created
  ino_t sock_ino_ = 0;
  // std::less<>: looked up by string_view straight from the HPACK-decoded :path.
  std::map<std::string, UnaryHandler, std::less<>> unary_;
  std::map<std::string, StreamHandler, std::less<>> streams_;
  int listen_fd_ = -1;
  int spare_fd_ = -1;  // reserve descriptor for shedding connections at EMFILE
  std::vector<std::unique_ptr<Loop>> loops_;
  std::atomic<unsigned> next_loop_{0};
  std::atomic<bool> stopping_{false};
  std::atomic<bool> inject_failure_{false};
  std::function<void()> on_fatal_;
  std::atomic<uint64_t> next_stream_id_{1};
  bool trace_ = false;
  int busy_poll_us_ = 0;
  bool native_http2_ = true;
  bool follow_peer_l3_ = true;
  std::function<void()> after_flush_;
  cpu_set_t process_cpus_;  // CPUs the process may run on (at construction)
  ServerStats stats_;
};

// Blocking client (one HTTP/2 connection). Used for kubelet registration, the
// self-dial readiness probe, and the native benchmark/stub-kubelet tools.
class Channel {
 public:
  ~Channel();
  static Result<std::unique_ptr<Channel>> Dial(const std::string& uds_path, int timeout_ms);
  // Takes over a connected socket (non-blocking; closed with the channel) and
  // runs the HTTP/2 handshake on it. For tests and fuzzing.
  static Result<std::unique_ptr<Channel>> FromFd(int fd, int timeout_ms);

  Status Unary(const std::string& path, std::string_view request, std::string* response,
               int timeout_ms);
  // Opens a server-streaming call; returns the stream id.
  Result<int32_t> StartStream(const std::string& path, std::string_view request);
  // Next message of a stream. Returns NotFound("end of stream") after a clean end,
  // DeadlineExceeded on timeout, or the call's error status.
  Status Recv(int32_t stream_id, std::string* message, int timeout_ms);
  // Processes pending input without blocking (or up to timeout_ms).
  Status Pump(int timeout_ms);

  // Client frame pattern of the kubelet's grpc-go transport (BDP estimation on,
  // the default for a kubelet dial): a PING with an 8-byte payload after the
  // first DATA frame received while no such ping is outstanding -- i.e. about
  // one per sequential unary call -- and a grpc-go user-agent. grpc-go's loopy
  // writer goroutine writes that ping on its own while the application already
  // has its response, so here the caller writes it with SendBdpPing() after the
  // call returns (its own write, outside a timed call). Reference peer: the
  // kubelet's grpc-go client of cmd/nvidia-device-plugin/server.go:168-240.
  void EmulateGrpcGo(bool on) { grpc_go_ = on; }
  Status SendBdpPing();
  uint64_t bdp_pings_sent() const { return bdp_pings_; }

 private:
  struct CallState;
  Channel() = default;
  static Result<std::unique_ptr<Channel>> Start(std::unique_ptr<Channel> ch, int64_t deadline_ms,
                                                const std::string& peer);
  Status Flush();
  Status WaitFor(const std::function<bool()>& done, int timeout_ms);
  Result<int32_t> Submit(const std::string& path, std::string_view request);

  int fd_ = -1;
  void* session_ = nullptr;  // nghttp2_session*
  bool dead_ = false;
  bool got_settings_ = false;
  bool grpc_go_ = false;
  bool bdp_outstanding_ = false;
  bool bdp_due_ = false;
  uint64_t bdp_pings_ = 0;
  std::string wbuf_;  // frames gathered by Flush() for one write
  std::map<int32_t, std::unique_ptr<CallState>> calls_;
  friend struct ChannelCallbacks;
};

}  // namespace adp::grpc
