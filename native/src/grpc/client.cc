// Blocking gRPC h2c client over a Unix-domain socket.
//
// Parity: reference cmd/nvidia-device-plugin/server.go:361-374 (`dial`: insecure,
// blocking, 5 s timeout, unix dialer) used for the self-dial readiness probe
// (server.go:207-213) and the kubelet Register call (server.go:218-240).
#include <errno.h>
#include <nghttp2/nghttp2.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <deque>

#include "grpc/grpc.h"

namespace adp::grpc {

struct Channel::CallState {
  int http_status = 0;
  int grpc_status = -1;
  std::string grpc_message;
  std::string buf;  // raw DATA not yet split into messages
  std::deque<std::string> msgs;
  bool closed = false;
  uint32_t rst_code = 0;
  std::string req;  // framed request
  size_t req_off = 0;
  bool bad_frame = false;
  bool too_large = false;  // a message, or the call's buffered messages, over kMaxRecvBytes
  size_t buffered = 0;     // bytes held in msgs
};

namespace {

nghttp2_nv Nv(const char* n, const char* v) {
  nghttp2_nv nv;
  nv.name = reinterpret_cast<uint8_t*>(const_cast<char*>(n));
  nv.namelen = strlen(n);
  nv.value = reinterpret_cast<uint8_t*>(const_cast<char*>(v));
  nv.valuelen = strlen(v);
  nv.flags = NGHTTP2_NV_FLAG_NONE;
  return nv;
}

// What one call may hold of its peer's messages: the kubelet's own PodResources
// client allows 16 MiB (podresources.DefaultMaxMsgSize); grpc-go's default is
// 4 MiB. A peer that sends more fails the call instead of growing the daemon.
constexpr size_t kMaxRecvBytes = 16u << 20;
// What Pump() reads per call before it returns, so WaitFor() sees its deadline
// even while a peer keeps the socket full.
constexpr size_t kReadBudgetPerPump = 1u << 20;

int64_t NowMs() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

}  // namespace

struct ChannelCallbacks {
  static Channel::CallState* Find(Channel* ch, int32_t sid) {
    auto it = ch->calls_.find(sid);
    return it == ch->calls_.end() ? nullptr : it->second.get();
  }
  static int OnHeader(nghttp2_session*, const nghttp2_frame* frame, const uint8_t* name,
                      size_t namelen, const uint8_t* value, size_t valuelen, uint8_t, void* ud) {
    auto* ch = static_cast<Channel*>(ud);
    if (frame->hd.type != NGHTTP2_HEADERS) return 0;
    Channel::CallState* c = Find(ch, frame->hd.stream_id);
    if (!c) return 0;
    std::string_view n(reinterpret_cast<const char*>(name), namelen);
    std::string v(reinterpret_cast<const char*>(value), valuelen);
    if (n == ":status") c->http_status = atoi(v.c_str());
    else if (n == "grpc-status") c->grpc_status = atoi(v.c_str());
    else if (n == "grpc-message") c->grpc_message = PercentDecode(v);
    return 0;
  }
  static int OnData(nghttp2_session* s, uint8_t, int32_t sid, const uint8_t* data, size_t len,
                    void* ud) {
    auto* ch = static_cast<Channel*>(ud);
    // grpc-go's bdpEstimator.add(): the first DATA after the last ping's ACK
    // starts a new sample (written by SendBdpPing()).
    if (ch->grpc_go_ && !ch->bdp_outstanding_) ch->bdp_due_ = true;
    Channel::CallState* c = Find(ch, sid);
    if (!c || c->too_large) return 0;
    c->buf.append(reinterpret_cast<const char*>(data), len);
    while (c->buf.size() >= 5) {
      const auto* b = reinterpret_cast<const uint8_t*>(c->buf.data());
      if (b[0] != 0) { c->bad_frame = true; c->buf.clear(); break; }
      uint32_t n = (uint32_t(b[1]) << 24) | (uint32_t(b[2]) << 16) | (uint32_t(b[3]) << 8) | b[4];
      if (c->buffered + n > kMaxRecvBytes) {
        // Hold nothing more of this call and cancel it: the caller gets an
        // error, never a partial answer.
        c->too_large = true;
        c->closed = true;
        c->buf.clear();
        c->buf.shrink_to_fit();
        c->msgs.clear();
        nghttp2_submit_rst_stream(s, NGHTTP2_FLAG_NONE, sid, NGHTTP2_CANCEL);
        break;
      }
      if (c->buf.size() < 5 + static_cast<size_t>(n)) break;
      c->msgs.emplace_back(c->buf.substr(5, n));
      c->buffered += n;
      c->buf.erase(0, 5 + static_cast<size_t>(n));
    }
    return 0;
  }
  static int OnFrameRecv(nghttp2_session*, const nghttp2_frame* frame, void* ud) {
    auto* ch = static_cast<Channel*>(ud);
    if (frame->hd.type == NGHTTP2_SETTINGS && !(frame->hd.flags & NGHTTP2_FLAG_ACK))
      ch->got_settings_ = true;
    if (frame->hd.type == NGHTTP2_GOAWAY) ch->dead_ = true;
    if (frame->hd.type == NGHTTP2_PING && (frame->hd.flags & NGHTTP2_FLAG_ACK)) ch->bdp_outstanding_ = false;
    return 0;
  }
  static int OnStreamClose(nghttp2_session*, int32_t sid, uint32_t code, void* ud) {
    auto* ch = static_cast<Channel*>(ud);
    Channel::CallState* c = Find(ch, sid);
    if (c) { c->closed = true; c->rst_code = code; }
    return 0;
  }
  static ssize_t Read(nghttp2_session*, int32_t sid, uint8_t* buf, size_t len, uint32_t* flags,
                      nghttp2_data_source*, void* ud) {
    auto* ch = static_cast<Channel*>(ud);
    Channel::CallState* c = Find(ch, sid);
    if (!c) { *flags |= NGHTTP2_DATA_FLAG_EOF; return 0; }
    size_t n = std::min(len, c->req.size() - c->req_off);
    memcpy(buf, c->req.data() + c->req_off, n);
    c->req_off += n;
    if (c->req_off == c->req.size()) *flags |= NGHTTP2_DATA_FLAG_EOF;
    return static_cast<ssize_t>(n);
  }
};

Channel::~Channel() {
  if (session_) nghttp2_session_del(static_cast<nghttp2_session*>(session_));
  if (fd_ >= 0) close(fd_);
}


Result<std::unique_ptr<Channel>> Channel::Dial(const std::string& uds_path, int timeout_ms) {
  std::unique_ptr<Channel> ch(new Channel());
  int64_t deadline = NowMs() + timeout_ms;
  struct sockaddr_un addr;
  if (uds_path.size() >= sizeof(addr.sun_path)) return InvalidArgument("socket path too long");
  memset(&addr, 0, sizeof(addr));
  addr.sun_family = AF_UNIX;
  memcpy(addr.sun_path, uds_path.c_str(), uds_path.size());
  // Like grpc.WithBlock: keep retrying connect until the deadline (the server
  // may not have bound yet).
  while (true) {
    ch->fd_ = socket(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    if (ch->fd_ < 0) return Internal(std::string("socket: ") + strerror(errno));
    if (connect(ch->fd_, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) == 0) break;
    int err = errno;
    if (err == EINPROGRESS || err == EAGAIN) {
      pollfd p{ch->fd_, POLLOUT, 0};
      int left = static_cast<int>(deadline - NowMs());
      if (left > 0 && poll(&p, 1, left) == 1) {
        int soerr = 0;
        socklen_t sl = sizeof(soerr);
        getsockopt(ch->fd_, SOL_SOCKET, SO_ERROR, &soerr, &sl);
        if (soerr == 0) break;
      }
    }
    close(ch->fd_);
    ch->fd_ = -1;
    // No socket file at all: nobody will bind it within a dial timeout (kubelet
    // re-creating kubelet.sock is picked up by the daemon's inotify watch), so
    // fail fast instead of blocking signal handling for the whole timeout.
    if (err == ENOENT || NowMs() >= deadline)
      return Unavailable("connect " + uds_path + ": " + strerror(err));
    usleep(20 * 1000);
  }
  return Start(std::move(ch), deadline, uds_path);
}

Result<std::unique_ptr<Channel>> Channel::FromFd(int fd, int timeout_ms) {
  std::unique_ptr<Channel> ch(new Channel());
  ch->fd_ = fd;
  return Start(std::move(ch), NowMs() + timeout_ms, "fd " + std::to_string(fd));
}

Result<std::unique_ptr<Channel>> Channel::Start(std::unique_ptr<Channel> ch, int64_t deadline,
                                                const std::string& peer) {
  nghttp2_session_callbacks* cbs;
  nghttp2_session_callbacks_new(&cbs);
  nghttp2_session_callbacks_set_on_header_callback(cbs, ChannelCallbacks::OnHeader);
  nghttp2_session_callbacks_set_on_data_chunk_recv_callback(cbs, ChannelCallbacks::OnData);
  nghttp2_session_callbacks_set_on_frame_recv_callback(cbs, ChannelCallbacks::OnFrameRecv);
  nghttp2_session_callbacks_set_on_stream_close_callback(cbs, ChannelCallbacks::OnStreamClose);
  nghttp2_session* s = nullptr;
  int rv = nghttp2_session_client_new(&s, cbs, ch.get());
  nghttp2_session_callbacks_del(cbs);
  if (rv != 0) return Internal("nghttp2_session_client_new failed");
  ch->session_ = s;
  nghttp2_settings_entry iv[] = {
      {NGHTTP2_SETTINGS_ENABLE_PUSH, 0},
      {NGHTTP2_SETTINGS_INITIAL_WINDOW_SIZE, 4u << 20},
      {NGHTTP2_SETTINGS_MAX_FRAME_SIZE, 1u << 16},
  };
  nghttp2_submit_settings(s, NGHTTP2_FLAG_NONE, iv, 3);
  nghttp2_session_set_local_window_size(s, NGHTTP2_FLAG_NONE, 0, 16 << 20);
  Channel* raw = ch.get();
  Status st = ch->WaitFor([raw] { return raw->got_settings_; },
                          std::max<int>(1, static_cast<int>(deadline - NowMs())));
  if (!st.ok()) return Unavailable("HTTP/2 handshake with " + peer + ": " + st.message());
  return ch;
}

Status Channel::Flush() {
  // Every frame nghttp2 has ready (a request's HEADERS + DATA, WINDOW_UPDATEs,
  // SETTINGS acks) goes out in one write, like grpc-go's batching writer: the
  // peer wakes up once per request instead of once per frame.
  auto* s = static_cast<nghttp2_session*>(session_);
  wbuf_.clear();
  while (true) {
    const uint8_t* data;
    ssize_t n = nghttp2_session_mem_send(s, &data);
    if (n < 0) { dead_ = true; return Internal(nghttp2_strerror(static_cast<int>(n))); }
    if (n == 0) break;
    wbuf_.append(reinterpret_cast<const char*>(data), static_cast<size_t>(n));
  }
  size_t off = 0;
  while (off < wbuf_.size()) {
    ssize_t w = send(fd_, wbuf_.data() + off, wbuf_.size() - off, MSG_NOSIGNAL);
    if (w > 0) { off += static_cast<size_t>(w); continue; }
    if (w < 0 && errno == EINTR) continue;
    if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
      // A peer that takes nothing for a second is not reading at all: give up
      // rather than hold the caller's thread for ever (no deadline reaches
      // this loop).
      pollfd p{fd_, POLLOUT, 0};
      if (poll(&p, 1, 1000) == 0) {
        dead_ = true;
        return Unavailable("peer took no bytes for 1 s");
      }
      continue;
    }
    dead_ = true;
    return Unavailable(std::string("write: ") + strerror(errno));
  }
  return Status::Ok();
}

Status Channel::Pump(int timeout_ms) {
  if (dead_) return Unavailable("connection closed");
  pollfd p{fd_, POLLIN, 0};
  int r = poll(&p, 1, timeout_ms);
  if (r < 0 && errno != EINTR) { dead_ = true; return Unavailable("poll failed"); }
  if (r <= 0) return Status::Ok();
  char buf[64 * 1024];
  for (size_t budget = kReadBudgetPerPump; budget > 0;) {
    ssize_t n = read(fd_, buf, sizeof(buf));
    if (n > 0) {
      ssize_t rv = nghttp2_session_mem_recv(static_cast<nghttp2_session*>(session_),
                                            reinterpret_cast<uint8_t*>(buf), n);
      if (rv < 0) { dead_ = true; return Internal(nghttp2_strerror(static_cast<int>(rv))); }
      if (static_cast<size_t>(n) < sizeof(buf)) break;
      budget -= std::min(budget, static_cast<size_t>(n));
      continue;
    }
    if (n == 0) { dead_ = true; break; }
    if (errno == EINTR) continue;
    if (errno == EAGAIN || errno == EWOULDBLOCK) break;
    dead_ = true;
    return Unavailable(std::string("read: ") + strerror(errno));
  }
  return Flush();
}

Status Channel::WaitFor(const std::function<bool()>& done, int timeout_ms) {
  int64_t deadline = NowMs() + timeout_ms;
  ADP_RETURN_IF_ERROR(Flush());
  while (!done()) {
    if (dead_) return Unavailable("connection closed by peer");
    int left = static_cast<int>(deadline - NowMs());
    if (left <= 0) return DeadlineExceeded("timed out");
    ADP_RETURN_IF_ERROR(Pump(left));
  }
  return Status::Ok();
}

Status Channel::SendBdpPing() {
  if (!bdp_due_ || dead_) return Status::Ok();
  static const uint8_t kBdpPayload[8] = {2, 4, 16, 16, 9, 14, 7, 7};  // grpc-go's bdpPing data
  bdp_due_ = false;
  if (nghttp2_submit_ping(static_cast<nghttp2_session*>(session_), NGHTTP2_FLAG_NONE, kBdpPayload) != 0)
    return Internal("nghttp2_submit_ping failed");
  bdp_outstanding_ = true;
  ++bdp_pings_;
  return Flush();
}

Result<int32_t> Channel::Submit(const std::string& path, std::string_view request) {
  if (dead_) return Unavailable("connection closed");
  auto call = std::make_unique<CallState>();
  FrameMessage(request, &call->req);
  nghttp2_nv hdrs[] = {
      Nv(":method", "POST"),       Nv(":scheme", "http"),
      Nv(":path", path.c_str()),   Nv(":authority", "localhost"),
      Nv("content-type", "application/grpc"), Nv("te", "trailers"),
      Nv("user-agent", grpc_go_ ? "grpc-go/1.65.0" : "amdgpu-dp-grpc/1.0"),
  };
  nghttp2_data_provider prd;
  prd.source.ptr = nullptr;
  prd.read_callback = ChannelCallbacks::Read;
  int32_t sid = nghttp2_submit_request(static_cast<nghttp2_session*>(session_), nullptr, hdrs,
                                       sizeof(hdrs) / sizeof(hdrs[0]), &prd, nullptr);
  if (sid < 0) return Internal(nghttp2_strerror(sid));
  calls_[sid] = std::move(call);
  ADP_RETURN_IF_ERROR(Flush());
  return sid;
}

Status Channel::Unary(const std::string& path, std::string_view request, std::string* response,
                      int timeout_ms) {
  auto sid = Submit(path, request);
  if (!sid.ok()) return sid.status();
  CallState* c = calls_[*sid].get();
  Status st = WaitFor([c] { return c->closed; }, timeout_ms);
  std::unique_ptr<CallState> hold = std::move(calls_[*sid]);
  calls_.erase(*sid);
  if (!st.ok()) {
    if (!dead_) {
      nghttp2_submit_rst_stream(static_cast<nghttp2_session*>(session_), NGHTTP2_FLAG_NONE, *sid,
                                NGHTTP2_CANCEL);
      Flush();
    }
    return st;
  }
  if (c->too_large) return Internal("response larger than " + std::to_string(kMaxRecvBytes) + " bytes");
  if (c->http_status != 200)
    return Unavailable("HTTP status " + std::to_string(c->http_status));
  if (c->grpc_status < 0) return Internal("missing grpc-status (stream reset code " +
                                          std::to_string(c->rst_code) + ")");
  if (c->grpc_status != 0) return Status(FromGrpcCode(c->grpc_status), c->grpc_message);
  if (c->bad_frame) return Unimplemented("compressed response");
  if (c->msgs.empty()) return Internal("no response message");
  *response = std::move(c->msgs.front());
  return Status::Ok();
}

Result<int32_t> Channel::StartStream(const std::string& path, std::string_view request) {
  return Submit(path, request);
}

Status Channel::Recv(int32_t stream_id, std::string* message, int timeout_ms) {
  auto it = calls_.find(stream_id);
  if (it == calls_.end()) return NotFound("unknown stream");
  CallState* c = it->second.get();
  Status st = WaitFor([c] { return !c->msgs.empty() || c->closed; }, timeout_ms);
  if (!st.ok()) return st;
  if (!c->msgs.empty()) {
    *message = std::move(c->msgs.front());
    c->msgs.pop_front();
    c->buffered -= message->size();
    return Status::Ok();
  }
  Status end = c->too_large ? Internal("stream message larger than " + std::to_string(kMaxRecvBytes) + " bytes")
               : (c->grpc_status == 0) ? NotFound("end of stream")
               : (c->grpc_status > 0) ? Status(FromGrpcCode(c->grpc_status), c->grpc_message)
                                      : Unavailable("stream reset");
  calls_.erase(it);
  return end;
}

}  // namespace adp::grpc
