// gRPC h2c server on a Unix-domain socket (see grpc.h for the protocol subset).
//
// Parity: reference cmd/nvidia-device-plugin/server.go:168-215 (Serve: remove stale
// socket, listen on unix:<socket>, register the service, restart the serve loop on
// failure with a crash budget of 5 failures within an hour each).
#include <errno.h>
#include <fcntl.h>
#include <nghttp2/nghttp2.h>
#include <pthread.h>
#include <sched.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <fstream>
#include <sstream>

#include "common/log.h"
#include "grpc/grpc.h"
#include "grpc/server_conn.h"

namespace adp::grpc {
namespace {

constexpr size_t kMaxRequestBytes = 16u << 20;  // 16 MiB, >> any kubelet request
constexpr const char* kComp = "grpc-server";

bool StartsWithGrpc(std::string_view ct) { return ct.substr(0, 16) == "application/grpc"; }

nghttp2_nv MakeNv(std::string_view name, std::string_view value) {
  nghttp2_nv nv;
  nv.name = reinterpret_cast<uint8_t*>(const_cast<char*>(name.data()));
  nv.namelen = name.size();
  nv.value = reinterpret_cast<uint8_t*>(const_cast<char*>(value.data()));
  nv.valuelen = value.size();
  nv.flags = NGHTTP2_NV_FLAG_NONE;
  return nv;
}

}  // namespace

struct StreamState {
  // Resolved from :path as the header arrives; `path` itself is only kept when
  // it names no method (for the error) or calls are traced.
  const UnaryHandler* unary = nullptr;
  const StreamHandler* stream_handler = nullptr;
  std::string path;
  bool grpc_content_type = false;
  std::string content_type;  // only kept when it is not application/grpc*
  std::string body;
  bool dispatched = false;
  std::string out;       // framed response bytes not yet handed to nghttp2
  size_t out_off = 0;
  // Server streams carry state snapshots (ListAndWatch): while `out` is still
  // being sent, only the newest queued message is kept here (latest wins), so a
  // peer that stops reading costs at most two messages of memory.
  std::string pending;
  bool finishing = false;  // send trailers once `out` drains
  bool deferred = false;
  int grpc_status = 0;
  std::string grpc_message;
  std::shared_ptr<ServerStream> stream;
};

class Nghttp2Conn final : public ServerConn {
 public:
  Nghttp2Conn(Server* srv, int loop, int fd) : ServerConn(srv, loop, fd) {}
  ~Nghttp2Conn() override {
    for (auto& [_, st] : streams_) Detach(st.stream.get());
    if (session_) nghttp2_session_del(session_);
    if (fd_ >= 0) close(fd_);
  }

  bool Init() override;
  bool OnReadable() override;
  bool Flush() override;
  bool Done() const override {
    return !nghttp2_session_want_read(session_) && !nghttp2_session_want_write(session_) &&
           wbuf_.size() == woff_;
  }
  bool want_epollout() const override { return wbuf_.size() > woff_; }

  // --- called from nghttp2 callbacks ---
  StreamState* Find(int32_t sid) {
    auto it = streams_.find(sid);
    return it == streams_.end() ? nullptr : &it->second;
  }
  void Dispatch(int32_t sid);
  void OnPath(StreamState* st, std::string_view v) {
    st->unary = FindUnary(v);
    if (!st->unary) st->stream_handler = FindStreamHandler(v);
    if ((!st->unary && !st->stream_handler) || tracing()) st->path.assign(v);
  }
  void OnContentType(StreamState* st, std::string_view v) {
    st->grpc_content_type = StartsWithGrpc(v);
    if (!st->grpc_content_type) st->content_type.assign(v);
  }
  void OnStreamClose(int32_t sid) {
    auto it = streams_.find(sid);
    if (it == streams_.end()) return;
    Detach(it->second.stream.get());
    streams_.erase(it);
  }
  ssize_t ReadData(int32_t sid, uint8_t* buf, size_t len, uint32_t* flags);

  // --- used by ServerStream ---
  bool QueueMessage(int32_t sid, std::string_view msg) override;
  void Finish(int32_t sid, const Status& st) override;

  std::map<int32_t, StreamState> streams_;

 private:
  void SubmitTrailersOnly(int32_t sid, int code, const std::string& msg);
  void SubmitResponse(int32_t sid);
  void SubmitTrailers(int32_t sid, StreamState* st);

  nghttp2_session* session_ = nullptr;
  std::string wbuf_;
  std::string resp_buf_;  // unary handler output, framed into the stream's `out`
  size_t woff_ = 0;
};

// ------------------------- nghttp2 callbacks -------------------------

static int OnBeginHeaders(nghttp2_session*, const nghttp2_frame* frame, void* ud) {
  auto* c = static_cast<Nghttp2Conn*>(ud);
  if (frame->hd.type == NGHTTP2_HEADERS && frame->headers.cat == NGHTTP2_HCAT_REQUEST) {
    c->streams_[frame->hd.stream_id];
  }
  return 0;
}

static int OnHeader(nghttp2_session*, const nghttp2_frame* frame, const uint8_t* name,
                    size_t namelen, const uint8_t* value, size_t valuelen, uint8_t, void* ud) {
  auto* c = static_cast<Nghttp2Conn*>(ud);
  // The request's own header block only: a trailer block (HCAT_HEADERS) naming
  // :path or content-type again must not change the call (found by
  // native/fuzz/fuzz_h2_diff.cc; the native engine reads the first block only).
  if (frame->hd.type != NGHTTP2_HEADERS || frame->headers.cat != NGHTTP2_HCAT_REQUEST) return 0;
  StreamState* st = c->Find(frame->hd.stream_id);
  if (!st) return 0;
  std::string_view n(reinterpret_cast<const char*>(name), namelen);
  std::string_view v(reinterpret_cast<const char*>(value), valuelen);
  if (n == ":path") c->OnPath(st, v);
  else if (n == "content-type") c->OnContentType(st, v);
  return 0;
}

static int OnDataChunk(nghttp2_session* s, uint8_t, int32_t sid, const uint8_t* data, size_t len,
                       void* ud) {
  auto* c = static_cast<Nghttp2Conn*>(ud);
  StreamState* st = c->Find(sid);
  if (!st) return 0;
  if (st->dispatched) return 0;
  if (st->body.size() + len > kMaxRequestBytes) {
    nghttp2_submit_rst_stream(s, NGHTTP2_FLAG_NONE, sid, NGHTTP2_REFUSED_STREAM);
    st->dispatched = true;  // never hand a truncated request to a handler
    st->body.clear();
    st->body.shrink_to_fit();
    return 0;
  }
  st->body.append(reinterpret_cast<const char*>(data), len);
  return 0;
}

static int OnFrameRecv(nghttp2_session*, const nghttp2_frame* frame, void* ud) {
  auto* c = static_cast<Nghttp2Conn*>(ud);
  if ((frame->hd.type == NGHTTP2_DATA || frame->hd.type == NGHTTP2_HEADERS) &&
      (frame->hd.flags & NGHTTP2_FLAG_END_STREAM)) {
    c->Dispatch(frame->hd.stream_id);
  }
  return 0;
}

static int OnStreamCloseCb(nghttp2_session*, int32_t sid, uint32_t, void* ud) {
  static_cast<Nghttp2Conn*>(ud)->OnStreamClose(sid);
  return 0;
}

static ssize_t ReadCallback(nghttp2_session*, int32_t sid, uint8_t* buf, size_t length,
                            uint32_t* data_flags, nghttp2_data_source*, void* ud) {
  return static_cast<Nghttp2Conn*>(ud)->ReadData(sid, buf, length, data_flags);
}

// ------------------------- Nghttp2Conn -------------------------

bool Nghttp2Conn::Init() {
  nghttp2_session_callbacks* cbs;
  nghttp2_session_callbacks_new(&cbs);
  nghttp2_session_callbacks_set_on_begin_headers_callback(cbs, OnBeginHeaders);
  nghttp2_session_callbacks_set_on_header_callback(cbs, OnHeader);
  nghttp2_session_callbacks_set_on_data_chunk_recv_callback(cbs, OnDataChunk);
  nghttp2_session_callbacks_set_on_frame_recv_callback(cbs, OnFrameRecv);
  nghttp2_session_callbacks_set_on_stream_close_callback(cbs, OnStreamCloseCb);
  // Closed streams are not retained for the RFC 7540 priority tree (gRPC never
  // uses priorities); keeping them roughly doubles nghttp2's per-call cost.
  nghttp2_option* opt;
  nghttp2_option_new(&opt);
  nghttp2_option_set_no_closed_streams(opt, 1);
  // No per-header RFC 7540 §8 validation: the server only reads :path and
  // content-type and answers anything else with a gRPC status (saves a pass over
  // every header name and value per call).
  nghttp2_option_set_no_http_messaging(opt, 1);
  int rv = nghttp2_session_server_new2(&session_, cbs, this, opt);
  nghttp2_option_del(opt);
  nghttp2_session_callbacks_del(cbs);
  if (rv != 0) return false;
  nghttp2_settings_entry iv[] = {
      {NGHTTP2_SETTINGS_MAX_CONCURRENT_STREAMS, 1024},
      {NGHTTP2_SETTINGS_INITIAL_WINDOW_SIZE, 1u << 20},
      {NGHTTP2_SETTINGS_MAX_FRAME_SIZE, 1u << 16},
  };
  if (nghttp2_submit_settings(session_, NGHTTP2_FLAG_NONE, iv, sizeof(iv) / sizeof(iv[0])) != 0)
    return false;
  nghttp2_session_set_local_window_size(session_, NGHTTP2_FLAG_NONE, 0, 8 << 20);
  return Flush();
}

bool Nghttp2Conn::OnReadable() {
  char buf[64 * 1024];
  ReadStarted();
  // At most this much per readiness wake-up, then the loop's other
  // connections (epoll is level-triggered: the rest is reported again).
  size_t budget = size_t{1} << 20;
  while (true) {
    ssize_t n = read(fd_, buf, sizeof(buf));
    if (n > 0) {
      ssize_t rv = nghttp2_session_mem_recv(session_, reinterpret_cast<uint8_t*>(buf), n);
      if (rv < 0) {
        LOG_DEBUG(kComp, "nghttp2 recv error: %s", nghttp2_strerror(static_cast<int>(rv)));
        return false;
      }
      budget -= std::min(budget, static_cast<size_t>(n));
      if (static_cast<size_t>(n) < sizeof(buf) || budget == 0) break;
      continue;
    }
    if (n == 0) return false;  // peer closed
    if (errno == EINTR) continue;
    if (errno == EAGAIN || errno == EWOULDBLOCK) break;
    return false;
  }
  return Flush();
}

bool Nghttp2Conn::Flush() {
  // Pull frames out of nghttp2 until it has nothing more (flow control bounds
  // how much it produces), then write as much as the socket takes.
  while (true) {
    const uint8_t* data;
    ssize_t n = nghttp2_session_mem_send(session_, &data);
    if (n < 0) return false;
    if (n == 0) break;
    if (woff_ == wbuf_.size()) { wbuf_.clear(); woff_ = 0; }
    wbuf_.append(reinterpret_cast<const char*>(data), n);
  }
  if (woff_ < wbuf_.size()) Sending();
  while (woff_ < wbuf_.size()) {
    ssize_t n = send(fd_, wbuf_.data() + woff_, wbuf_.size() - woff_, MSG_NOSIGNAL);
    if (n > 0) { woff_ += n; continue; }
    if (n < 0 && errno == EINTR) continue;
    if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
    return false;
  }
  if (woff_ == wbuf_.size()) {
    wbuf_.clear();
    woff_ = 0;
  }
  return true;
}

ssize_t Nghttp2Conn::ReadData(int32_t sid, uint8_t* buf, size_t len, uint32_t* flags) {
  StreamState* st = Find(sid);
  if (!st) return NGHTTP2_ERR_TEMPORAL_CALLBACK_FAILURE;
  size_t avail = st->out.size() - st->out_off;
  size_t n = avail < len ? avail : len;
  if (n) {
    memcpy(buf, st->out.data() + st->out_off, n);
    st->out_off += n;
    if (st->out_off == st->out.size()) {
      st->out.clear();
      st->out_off = 0;
      if (!st->pending.empty()) st->out.swap(st->pending);  // next (latest) message
    }
  }
  if (st->out.size() == st->out_off) {
    if (st->finishing) {
      *flags |= NGHTTP2_DATA_FLAG_EOF | NGHTTP2_DATA_FLAG_NO_END_STREAM;
      SubmitTrailers(sid, st);
      return static_cast<ssize_t>(n);
    }
    if (n == 0) {
      st->deferred = true;
      return NGHTTP2_ERR_DEFERRED;
    }
  }
  return static_cast<ssize_t>(n);
}

void Nghttp2Conn::SubmitTrailers(int32_t sid, StreamState* st) {
  std::string code = std::to_string(st->grpc_status);
  std::string msg = PercentEncode(st->grpc_message);
  nghttp2_nv nva[2] = {MakeNv("grpc-status", code), MakeNv("grpc-message", msg)};
  nghttp2_submit_trailer(session_, sid, nva, msg.empty() ? 1 : 2);
}

void Nghttp2Conn::SubmitTrailersOnly(int32_t sid, int code, const std::string& msg) {
  std::string c = std::to_string(code);
  std::string m = PercentEncode(msg);
  nghttp2_nv nva[4] = {MakeNv(":status", "200"), MakeNv("content-type", "application/grpc"),
                       MakeNv("grpc-status", c), MakeNv("grpc-message", m)};
  nghttp2_submit_response(session_, sid, nva, m.empty() ? 3 : 4, nullptr);
  CountError();
}

void Nghttp2Conn::SubmitResponse(int32_t sid) {
  nghttp2_nv nva[2] = {MakeNv(":status", "200"), MakeNv("content-type", "application/grpc")};
  nghttp2_data_provider prd;
  prd.source.ptr = nullptr;
  prd.read_callback = ReadCallback;
  nghttp2_submit_response(session_, sid, nva, 2, &prd);
}

void Nghttp2Conn::Dispatch(int32_t sid) {
  StreamState* st = Find(sid);
  if (!st || st->dispatched) return;
  st->dispatched = true;
  CountCall();

  std::string_view req;
  int code = 0;
  std::string msg;
  if (!ParseRequest(st->grpc_content_type, st->content_type, st->body, &req, &code, &msg)) {
    SubmitTrailersOnly(sid, code, msg);
    return;
  }
  if (st->unary) {
    Answered();
    std::string& resp = resp_buf_;  // reused across calls: no allocation once warm
    Status s = RunUnary(*st->unary, st->path, req, &resp);
    st = Find(sid);  // handler cannot erase streams, but be defensive
    if (!st) return;
    if (!s.ok()) {
      SubmitTrailersOnly(sid, ToGrpcCode(s.code()), s.message());
      return;
    }
    FrameMessage(resp, &st->out);
    st->finishing = true;
    SubmitResponse(sid);
    return;
  }
  if (st->stream_handler) {
    auto stream = OpenStream(sid);
    st->stream = stream;
    SubmitResponse(sid);
    Status s = (*st->stream_handler)(req, stream);
    if (!s.ok() && !StreamClosed(*stream)) stream->Finish(s);
    return;
  }
  SubmitTrailersOnly(sid, kGrpcUnimplemented, "unknown method " + st->path);
}

bool Nghttp2Conn::QueueMessage(int32_t sid, std::string_view msg) {
  StreamState* st = Find(sid);
  if (!st || st->finishing) return false;
  if (st->out.size() == st->out_off) {
    st->out.clear();
    st->out_off = 0;
    FrameMessage(msg, &st->out);
  } else if (st->out_off == 0) {
    st->out.clear();  // nothing of the queued message went out yet: replace it
    FrameMessage(msg, &st->out);
  } else {
    st->pending.clear();  // finish the message in flight, then send only the newest
    FrameMessage(msg, &st->pending);
  }
  if (st->deferred) {
    st->deferred = false;
    nghttp2_session_resume_data(session_, sid);
  }
  return true;
}

void Nghttp2Conn::Finish(int32_t sid, const Status& s) {
  StreamState* st = Find(sid);
  if (!st || st->finishing) return;
  st->finishing = true;
  st->grpc_status = ToGrpcCode(s.code());
  st->grpc_message = s.ok() ? "" : s.message();
  if (st->deferred) {
    st->deferred = false;
    nghttp2_session_resume_data(session_, sid);
  }
}

bool ServerConn::ParseRequest(bool grpc_content_type, std::string_view content_type, std::string_view body,
                              std::string_view* req, int* code, std::string* msg) {
  if (!grpc_content_type) {
    *code = kGrpcInternal;
    *msg = "invalid content-type: " + std::string(content_type);
    return false;
  }
  *req = std::string_view();
  if (body.empty()) return true;
  const auto* b = reinterpret_cast<const uint8_t*>(body.data());
  if (body.size() < 5) {
    *code = kGrpcInternal;
    *msg = "truncated gRPC message header";
    return false;
  }
  if (b[0] != 0) {
    *code = kGrpcUnimplemented;
    *msg = "compressed messages are not supported";
    return false;
  }
  uint32_t n = (uint32_t(b[1]) << 24) | (uint32_t(b[2]) << 16) | (uint32_t(b[3]) << 8) | b[4];
  if (body.size() != 5 + static_cast<size_t>(n)) {
    *code = kGrpcInternal;
    *msg = "gRPC message length mismatch";
    return false;
  }
  *req = body.substr(5);
  return true;
}

Status ServerConn::RunUnary(const UnaryHandler& h, std::string_view path, std::string_view req, std::string* resp) {
  resp->clear();
  if (!tracing()) return h(req, resp);
  auto t0 = std::chrono::steady_clock::now();
  Status s = h(req, resp);
  double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  Logf(LogLevel::kInfo, "trace", "%s %.*s %s req=%zuB resp=%zuB handler=%.2fus", server_name().c_str(),
       static_cast<int>(path.size()), path.data(), s.ok() ? "OK" : s.ToString().c_str(), req.size(),
       resp->size(), us);
  return s;
}

std::unique_ptr<ServerConn> MakeNghttp2Conn(Server* srv, int loop, int fd) {
  return std::make_unique<Nghttp2Conn>(srv, loop, fd);
}

// ------------------------- ServerStream -------------------------

// Send/Finish only queue: they may run inside an nghttp2 callback (a handler
// sending its first message), where nghttp2_session_mem_send must not be
// re-entered. The loop flushes every connection after each iteration.
bool ServerStream::Send(std::string_view message) {
  if (closed_ || !conn_) return false;
  return conn_->QueueMessage(stream_id_, message);
}

void ServerStream::Finish(const Status& st) {
  if (closed_ || !conn_) return;
  conn_->Finish(stream_id_, st);
  closed_ = true;
}

// ------------------------- Server -------------------------

struct Server::Loop {
  int index = 0;
  int epoll_fd = -1;
  int event_fd = -1;
  std::thread thread;
  std::thread::id tid;
  std::mutex post_mu;
  std::vector<std::function<void()>> posted;
  std::map<int, std::unique_ptr<ServerConn>> conns;
  // --loop-affinity peer-l3: the peer process this loop follows and the L3 it
  // is pinned to (first CPU of that L3's list), re-checked while busy.
  int follow_pid = 0;
  int follow_l3 = -1;
  std::chrono::steady_clock::time_point next_follow_check{};
  std::map<int, int> peer_pid;  // fd -> visible peer pid (connections that may be followed)
  // Placement report (LoopPlacement): the CPU the loop ran on when it last
  // served something (sampled every 256 busy iterations) and how many busy
  // iterations it has had.
  std::atomic<int> cpu{-1};
  std::atomic<uint64_t> busy{0};
};

Server::Server(std::string name, int threads) : name_(std::move(name)) {
  if (sched_getaffinity(0, sizeof(process_cpus_), &process_cpus_) != 0) CPU_ZERO(&process_cpus_);
  // Loops (epoll + eventfd) exist from construction so Post() works before
  // Start(): work posted in between runs as soon as the loops start.
  if (threads < 1) threads = 1;
  for (int i = 0; i < threads; ++i) {
    auto l = std::make_unique<Loop>();
    l->index = i;
    l->epoll_fd = epoll_create1(EPOLL_CLOEXEC);
    l->event_fd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = l->event_fd;
    epoll_ctl(l->epoll_fd, EPOLL_CTL_ADD, l->event_fd, &ev);
    loops_.push_back(std::move(l));
  }
}

Server::~Server() { Stop(); }

void Server::AddUnary(const std::string& path, UnaryHandler h) { unary_[path] = std::move(h); }
void Server::AddServerStream(const std::string& path, StreamHandler h) {
  streams_[path] = std::move(h);
}

Status Server::Listen(const std::string& socket_path) {
  socket_path_ = socket_path;
  struct sockaddr_un addr;
  if (socket_path.size() >= sizeof(addr.sun_path))
    return InvalidArgument("socket path too long: " + socket_path);
  unlink(socket_path.c_str());  // stale socket from a previous run (server.go:169)
  listen_fd_ = socket(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (listen_fd_ < 0) return Internal(std::string("socket: ") + strerror(errno));
  memset(&addr, 0, sizeof(addr));
  addr.sun_family = AF_UNIX;
  memcpy(addr.sun_path, socket_path.c_str(), socket_path.size());
  if (bind(listen_fd_, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0) {
    Status s = Unavailable("bind " + socket_path + ": " + strerror(errno));
    close(listen_fd_);
    listen_fd_ = -1;
    return s;
  }
  struct stat st;
  if (stat(socket_path.c_str(), &st) == 0) {
    sock_dev_ = st.st_dev;
    sock_ino_ = st.st_ino;
  }
  if (listen(listen_fd_, 128) != 0) {
    Status s = Unavailable("listen " + socket_path + ": " + strerror(errno));
    close(listen_fd_);
    listen_fd_ = -1;
    return s;
  }
  // Held in reserve for AcceptAll(): with no descriptor left, a pending
  // connection keeps the (level-triggered) listener readable forever.
  if (spare_fd_ < 0) spare_fd_ = open("/dev/null", O_RDONLY | O_CLOEXEC);
  return Status::Ok();
}

bool Server::OwnsSocketPath() const {
  struct stat st;
  return sock_ino_ != 0 && stat(socket_path_.c_str(), &st) == 0 && st.st_dev == sock_dev_ &&
         st.st_ino == sock_ino_;
}

Status Server::Start(std::function<void()> on_fatal) {
  if (listen_fd_ < 0) return FailedPrecondition("Start() before Listen()");
  if (stopping_.load()) return FailedPrecondition("server already stopped");
  on_fatal_ = std::move(on_fatal);
  for (auto& l : loops_)
    if (l->epoll_fd < 0 || l->event_fd < 0) return Internal("epoll/eventfd setup failed");
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = listen_fd_;
  epoll_ctl(loops_[0]->epoll_fd, EPOLL_CTL_ADD, listen_fd_, &ev);
  for (auto& l : loops_) {
    Loop* lp = l.get();
    l->thread = std::thread([this, lp] { LoopMain(*lp); });
  }
  return Status::Ok();
}

void Server::Stop() {
  stopping_.store(true);  // later Post() calls are dropped
  for (auto& l : loops_) {
    if (!l->thread.joinable()) continue;
    uint64_t one = 1;
    ssize_t w = write(l->event_fd, &one, sizeof(one));
    (void)w;
    l->thread.join();
  }
  for (auto& l : loops_) {
    l->conns.clear();  // loops are gone; safe to tear down here
    std::lock_guard<std::mutex> lk(l->post_mu);
    l->posted.clear();
  }
  if (spare_fd_ >= 0) {
    close(spare_fd_);
    spare_fd_ = -1;
  }
  if (listen_fd_ >= 0) {
    close(listen_fd_);
    listen_fd_ = -1;
    // Only our own file: another instance of the plugin (a DaemonSet rollout
    // with maxSurge) may have bound the same path since.
    if (!socket_path_.empty() && OwnsSocketPath()) unlink(socket_path_.c_str());
  }
  for (auto& l : loops_) {
    if (l->epoll_fd >= 0) { close(l->epoll_fd); l->epoll_fd = -1; }
    if (l->event_fd >= 0) { close(l->event_fd); l->event_fd = -1; }
  }
}

void Server::PostTo(Loop& l, std::function<void()> fn) {
  if (stopping_.load() || l.event_fd < 0) return;
  {
    std::lock_guard<std::mutex> lk(l.post_mu);
    l.posted.push_back(std::move(fn));
  }
  uint64_t one = 1;
  ssize_t w = write(l.event_fd, &one, sizeof(one));
  (void)w;
}

void Server::Post(std::function<void()> fn) { PostTo(*loops_[0], std::move(fn)); }

void Server::PostAll(std::function<void(int)> fn) {
  for (auto& l : loops_) {
    int i = l->index;
    PostTo(*l, [fn, i] { fn(i); });
  }
}

std::vector<std::pair<int, uint64_t>> Server::LoopPlacement() const {
  std::vector<std::pair<int, uint64_t>> out;
  for (const auto& l : loops_)
    out.emplace_back(l->cpu.load(std::memory_order_relaxed), l->busy.load(std::memory_order_relaxed));
  return out;
}

bool Server::OnLoopThread() const {
  for (const auto& l : loops_)
    if (std::this_thread::get_id() == l->tid) return true;
  return false;
}

void Server::DrainPosted(Loop& l) {
  uint64_t v;
  ssize_t r = read(l.event_fd, &v, sizeof(v));
  (void)r;
  std::vector<std::function<void()>> work;
  {
    std::lock_guard<std::mutex> lk(l.post_mu);
    work.swap(l.posted);
  }
  for (auto& fn : work) fn();
}

namespace {

// CPU the process `pid` last ran on (/proc/<pid>/stat field 39), -1 if unknown.
int LastCpuOf(pid_t pid) {
  std::ifstream f("/proc/" + std::to_string(pid) + "/stat");
  std::string all((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  size_t rp = all.rfind(')');
  if (rp == std::string::npos) return -1;
  std::istringstream in(all.substr(rp + 1));
  std::string tok;
  for (int field = 3; in >> tok; ++field)
    if (field == 39) return atoi(tok.c_str());
  return -1;
}

// A sysfs CPU list ("0-7,128-135") of `cpu`, e.g. cache/index3/shared_cpu_list.
bool SysfsCpuList(int cpu, const char* rel, cpu_set_t* set) {
  std::ifstream f("/sys/devices/system/cpu/cpu" + std::to_string(cpu) + "/" + rel);
  std::string list;
  if (!std::getline(f, list)) return false;
  CPU_ZERO(set);
  std::istringstream in(list);
  std::string part;
  while (std::getline(in, part, ',')) {
    int a = -1, b = -1;
    if (sscanf(part.c_str(), "%d-%d", &a, &b) == 2) {
    } else if (sscanf(part.c_str(), "%d", &a) == 1) {
      b = a;
    } else {
      continue;
    }
    for (int c = a; c <= b && c < CPU_SETSIZE; ++c) CPU_SET(c, set);
  }
  return CPU_COUNT(set) > 0;
}

}  // namespace

void Server::FollowPeerL3(Loop& l, int pid) {
  // A request and its reply cross the socket twice; when caller and loop sit on
  // different CCDs every crossing pays an L3-to-L3 transfer (on the MI355X box's
  // EPYC 9575F: 4.4 us p50 on one L3 vs 5.0-5.3 us across, profiles/r1/session33/).
  // So the loop moves onto the L3 of the CPU the peer process last ran on --
  // within the CPUs this process may use -- and re-checks while it is busy, in
  // case the peer was moved to another CCD.
  int cpu = LastCpuOf(pid);
  cpu_set_t l3, core;
  if (cpu < 0 || !SysfsCpuList(cpu, "cache/index3/shared_cpu_list", &l3)) return;
  int l3_id = -1;
  for (int c = 0; c < CPU_SETSIZE && l3_id < 0; ++c)
    if (CPU_ISSET(c, &l3)) l3_id = c;
  if (l.follow_pid == pid && l.follow_l3 == l3_id) return;  // already there
  // The process-wide mask, not this thread's (it may already follow another peer).
  CPU_AND(&l3, &l3, &process_cpus_);
  // Not the peer's own core: a spinning loop on its SMT sibling slows both
  // (5.9 us p50 measured), a neighbouring core on the same L3 does not.
  if (SysfsCpuList(cpu, "topology/thread_siblings_list", &core)) {
    cpu_set_t rest;
    CPU_XOR(&rest, &l3, &core);
    CPU_AND(&rest, &rest, &l3);
    if (CPU_COUNT(&rest) > 0) l3 = rest;
  }
  if (CPU_COUNT(&l3) == 0) return;
  if (pthread_setaffinity_np(pthread_self(), sizeof(l3), &l3) == 0) {
    LOG_DEBUG(kComp, "'%s': connection from pid %d (cpu %d) served from its L3 (%d CPUs)%s", name_.c_str(), pid,
              cpu, CPU_COUNT(&l3), l.follow_pid == pid ? " after the peer moved" : "");
    l.follow_pid = pid;
    l.follow_l3 = l3_id;
  }
}

void Server::AddConn(Loop& l, int fd) {
  if (follow_peer_l3_) {
    ucred cr{};
    socklen_t len = sizeof(cr);
    // Only a visible peer (same PID namespace) that is not this process.
    if (getsockopt(fd, SOL_SOCKET, SO_PEERCRED, &cr, &len) == 0 && cr.pid > 0 && cr.pid != getpid()) {
      l.peer_pid[fd] = cr.pid;
      FollowPeerL3(l, cr.pid);
    }
  }
  auto conn = native_http2_ ? MakeH2Conn(this, l.index, fd) : MakeNghttp2Conn(this, l.index, fd);
  if (!conn->Init()) {  // closes fd
    l.peer_pid.erase(fd);
    return;
  }
  epoll_event ev{};
  ev.events = EPOLLIN | (conn->want_epollout() ? static_cast<uint32_t>(EPOLLOUT) : 0u);
  ev.data.fd = fd;
  epoll_ctl(l.epoll_fd, EPOLL_CTL_ADD, fd, &ev);
  conn->epoll_events = ev.events;
  stats_.connections.fetch_add(1, std::memory_order_relaxed);
  l.conns[fd] = std::move(conn);
}

void Server::AcceptAll() {
  while (true) {
    int fd = accept4(listen_fd_, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
    if (fd < 0) {
      if (errno == EINTR) continue;
      if ((errno == EMFILE || errno == ENFILE) && spare_fd_ >= 0) {
        // Out of descriptors: the listener would stay readable and the loop
        // would spin on it. Free the reserve, accept the connection and close
        // it (the client sees a reset and retries), then take the reserve back.
        close(spare_fd_);
        int shed = accept4(listen_fd_, nullptr, nullptr, SOCK_CLOEXEC);
        if (shed >= 0) close(shed);
        spare_fd_ = open("/dev/null", O_RDONLY | O_CLOEXEC);
        uint64_t n = stats_.shed_connections.fetch_add(1, std::memory_order_relaxed);
        if ((n & (n + 1)) == 0)  // 1st, 2nd, 4th, 8th ... time
          LOG_WARN(kComp, "'%s': out of file descriptors; refused connection #%llu (raise the open-files limit)",
                   name_.c_str(), static_cast<unsigned long long>(n + 1));
        if (shed >= 0) continue;
      }
      return;  // EAGAIN or transient: retry on next readiness
    }
    Loop& target = *loops_[next_loop_.fetch_add(1, std::memory_order_relaxed) % loops_.size()];
    if (&target == loops_[0].get()) {
      AddConn(target, fd);
    } else {
      // The fd travels in an owner that closes it if the hand-off is dropped
      // (server stopping, or the queue cleared before the loop ran it).
      struct OwnedFd {
        explicit OwnedFd(int f) : fd(f) {}
        OwnedFd(const OwnedFd&) = delete;
        OwnedFd& operator=(const OwnedFd&) = delete;
        ~OwnedFd() { if (fd >= 0) close(fd); }
        int fd;
      };
      auto owned = std::make_shared<OwnedFd>(fd);
      Loop* t = &target;
      PostTo(target, [this, t, owned] {
        int f = owned->fd;
        owned->fd = -1;
        AddConn(*t, f);
      });
    }
  }
}

void Server::CloseConn(Loop& l, int fd) {
  auto it = l.conns.find(fd);
  if (it == l.conns.end()) return;
  epoll_ctl(l.epoll_fd, EPOLL_CTL_DEL, fd, nullptr);
  l.conns.erase(it);
  auto pp = l.peer_pid.find(fd);
  if (pp == l.peer_pid.end()) return;
  int pid = pp->second;
  l.peer_pid.erase(pp);
  if (pid != l.follow_pid) return;
  for (const auto& [_, other] : l.peer_pid)
    if (other == pid) return;  // the followed peer still has a connection here
  // The last connection of the followed peer closed: give the loop back the
  // whole process mask instead of leaving it pinned to that peer's L3.
  pthread_setaffinity_np(pthread_self(), sizeof(process_cpus_), &process_cpus_);
  LOG_DEBUG(kComp, "'%s': followed peer %d disconnected; loop unpinned", name_.c_str(), pid);
  l.follow_pid = 0;
  l.follow_l3 = -1;
}

Status Server::RunLoop(Loop& l) {
#ifdef ADP_TEST_HOOKS
  // Tests: loop 0 fails every time it starts -- the crash budget end to end
  // (the reference exits after more than 5 crashes within an hour,
  // server.go:191-203). Compiled out of image builds.
  static const bool crash_hook = getenv("ADP_DEBUG_GRPC_LOOP_CRASH") != nullptr;
  if (crash_hook && l.index == 0) return Internal("ADP_DEBUG_GRPC_LOOP_CRASH");
#endif
  epoll_event events[64];
  // Adaptive busy-poll: after serving a request, keep polling without sleeping
  // for busy_poll_us_ so the kubelet's follow-up call (Allocate after
  // GetPreferredAllocation, the next pod of a burst) does not pay a scheduler
  // wake-up. An idle loop blocks in epoll_wait as usual (no CPU when idle).
  using Clock = std::chrono::steady_clock;
  const auto spin = std::chrono::microseconds(busy_poll_us_);
  Clock::time_point spin_until{};
  bool spinning = false;
  while (!stopping_.load()) {
    int n = epoll_wait(l.epoll_fd, events, 64, spinning ? 0 : -1);
    if (l.index == 0 && inject_failure_.exchange(false)) return Internal("injected loop failure");
    if (n < 0) {
      if (errno == EINTR) continue;
      return Internal(std::string("epoll_wait: ") + strerror(errno));
    }
    if (n == 0) {
      if (spinning && Clock::now() >= spin_until) spinning = false;
      continue;
    }
    uint64_t busy = l.busy.load(std::memory_order_relaxed) + 1;  // this loop is the only writer
    l.busy.store(busy, std::memory_order_relaxed);
    if ((busy & 255) == 1) l.cpu.store(sched_getcpu(), std::memory_order_relaxed);
    if (busy_poll_us_ > 0) {
      spinning = true;
      spin_until = Clock::now() + spin;
    }
    if (l.follow_pid > 0) {  // busy: is the peer still on the L3 we follow? (every 50 ms)
      auto now = Clock::now();
      if (now >= l.next_follow_check) {
        l.next_follow_check = now + std::chrono::milliseconds(50);
        FollowPeerL3(l, l.follow_pid);
      }
    }
    for (int i = 0; i < n; ++i) {
      int fd = events[i].data.fd;
      if (fd == listen_fd_ && l.index == 0) { AcceptAll(); continue; }
      if (fd == l.event_fd) { DrainPosted(l); continue; }
      auto it = l.conns.find(fd);
      if (it == l.conns.end()) continue;
      ServerConn* c = it->second.get();
      bool ok = true;
      if (events[i].events & (EPOLLIN | EPOLLHUP | EPOLLERR)) ok = c->OnReadable();
      else if (events[i].events & EPOLLOUT) ok = c->Flush();
      if (!ok || c->Done()) { CloseConn(l, fd); continue; }
    }
    // Flush every connection (handlers and posted work may have queued data on
    // any of them) and refresh EPOLLOUT interest.
    std::vector<int> dead;
    for (auto& [fd, c] : l.conns) {
      if (!c->Flush() || c->Done()) { dead.push_back(fd); continue; }
      uint32_t want = EPOLLIN | (c->want_epollout() ? static_cast<uint32_t>(EPOLLOUT) : 0u);
      if (want == c->epoll_events) continue;  // no syscall on the common path
      epoll_event ev{};
      ev.events = want;
      ev.data.fd = fd;
      epoll_ctl(l.epoll_fd, EPOLL_CTL_MOD, fd, &ev);
      c->epoll_events = want;
    }
    for (int fd : dead) CloseConn(l, fd);
    if (after_flush_) after_flush_();
  }
  return Status::Ok();
}

void Server::LoopMain(Loop& l) {
  l.tid = std::this_thread::get_id();
  using Clock = std::chrono::steady_clock;
  auto last_crash = Clock::now();
  int restarts = 0;
  while (!stopping_.load()) {
    LOG_DEBUG(kComp, "starting gRPC loop %d for '%s'", l.index, name_.c_str());
    Status st = RunLoop(l);
    if (st.ok() || stopping_.load()) break;
    LOG_ERROR(kComp, "gRPC server for '%s' crashed: %s", name_.c_str(), st.ToString().c_str());
    if (restarts > 5) {
      LOG_ERROR(kComp, "gRPC server for '%s' has repeatedly crashed recently; giving up",
                name_.c_str());
      if (on_fatal_) on_fatal_();
      break;
    }
    double since = std::chrono::duration<double>(Clock::now() - last_crash).count();
    last_crash = Clock::now();
    restarts = since > 3600 ? 1 : restarts + 1;
  }
}

}  // namespace adp::grpc
