// Native HTTP/2 server connection for the plugin's gRPC endpoints (RFC 7540 /
// RFC 7541 subset a gRPC server needs), the default engine behind ServerConn.
//
// Why not nghttp2's session layer: per call it allocates a stream object, copies
// and HPACK-deflates the response headers, runs the data-provider callback and
// queues frames through its outbound priority queue -- about a quarter of the
// daemon's CPU per RPC on the MI355X box (profiles/r1/session21/). A gRPC server
// needs far less: here a unary call is parsed straight out of the read buffer
// (HEADERS with END_HEADERS and a DATA frame with END_STREAM are handled
// without copying), the handler runs inline, and the response -- HEADERS from
// a constant HPACK block, DATA, trailers -- is appended to one write buffer.
// nghttp2 is still used for HPACK *decoding* (its inflater handles Huffman
// strings and the dynamic table the peer's encoder drives).
//
// Protocol coverage: client preface; SETTINGS (both directions, ACKs,
// INITIAL_WINDOW_SIZE deltas, MAX_FRAME_SIZE, HEADER_TABLE_SIZE with the HPACK
// size update it implies); PING/ACK; GOAWAY (received: finish open streams;
// sent on connection errors); RST_STREAM; WINDOW_UPDATE; connection and stream
// flow control in both directions; HEADERS with PADDED/PRIORITY and
// CONTINUATION; padded DATA; unknown frame types ignored. The response encoder
// indexes only content-type and grpc-status 0 (see PutContentType).
// Peer compatibility: exercised against grpcio (gRPC C-core) and nghttp2
// clients by the end-to-end and robustness suites.
#include <errno.h>
#include <nghttp2/nghttp2.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <algorithm>
#include <cstring>
#include <map>

#include "common/log.h"
#include "grpc/server_conn.h"

namespace adp::grpc {
namespace {

constexpr const char* kComp = "grpc-server";

enum FrameType : uint8_t {
  kData = 0, kHeaders = 1, kPriority = 2, kRstStream = 3, kSettings = 4,
  kPushPromise = 5, kPing = 6, kGoaway = 7, kWindowUpdate = 8, kContinuation = 9,
};
constexpr uint8_t kFlagEndStream = 0x1, kFlagAck = 0x1, kFlagEndHeaders = 0x4, kFlagPadded = 0x8,
                  kFlagPriority = 0x20;
enum H2Error : uint32_t {
  kNoError = 0, kProtocolError = 1, kInternalError = 2, kFlowControlError = 3, kStreamClosed = 5,
  kFrameSizeError = 6, kRefusedStream = 7, kCancel = 8, kCompressionError = 9, kEnhanceYourCalm = 11,
};

constexpr char kPreface[] = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n";
constexpr size_t kPrefaceLen = 24;
constexpr uint32_t kDefaultWindow = 65535;
constexpr uint32_t kMaxWindow = 0x7fffffff;
constexpr uint32_t kOurMaxFrame = 1u << 16;        // SETTINGS_MAX_FRAME_SIZE we announce
constexpr uint32_t kOurStreamWindow = 1u << 20;    // SETTINGS_INITIAL_WINDOW_SIZE we announce
constexpr uint32_t kOurConnWindow = 8u << 20;      // connection receive window
constexpr uint32_t kStreamAckBytes = 32u << 10;    // stream WINDOW_UPDATE threshold
constexpr uint32_t kConnAckBytes = 1u << 20;       // connection WINDOW_UPDATE threshold
constexpr uint32_t kMaxStreams = 1024;             // SETTINGS_MAX_CONCURRENT_STREAMS
constexpr size_t kMaxHeaderBlock = 64u << 10;      // HEADERS + CONTINUATION bytes per block
constexpr size_t kMaxRequestBytes = 16u << 20;     // >> any kubelet request
constexpr size_t kMaxGrpcMessageHeader = 4096;     // grpc-message is truncated beyond this
// A peer that keeps sending (PINGs, SETTINGS, requests) without reading our
// replies is cut off once this much output is queued (ENHANCE_YOUR_CALM).
constexpr size_t kMaxQueuedOutput = 16u << 20;
// After a connection error the peer's bytes are read and dropped until it
// stops sending (then the GOAWAY is written and the connection closed, so it
// can read why); a peer that keeps sending is cut off after this much
// (otherwise the loop would read and drop for ever, never seeing EAGAIN).
constexpr size_t kMaxDiscardAfterError = 64u << 20;
// Bytes one readiness wake-up reads from a connection before the loop turns to
// its other connections (epoll is level-triggered: the rest is reported again).
constexpr size_t kReadBudgetPerWake = 1u << 20;
// Request bytes buffered over all of a connection's open streams (each stream
// is also capped at kMaxRequestBytes): beyond it the peer is cut off.
constexpr size_t kMaxBufferedRequests = 64u << 20;

bool StartsWithGrpc(std::string_view ct) { return ct.substr(0, 16) == "application/grpc"; }

uint32_t Get24(const uint8_t* p) { return (uint32_t(p[0]) << 16) | (uint32_t(p[1]) << 8) | p[2]; }
uint32_t Get32(const uint8_t* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3];
}

void PutFrameHeader(std::string* o, size_t len, uint8_t type, uint8_t flags, uint32_t sid) {
  const char h[9] = {static_cast<char>(len >> 16), static_cast<char>(len >> 8), static_cast<char>(len),
                     static_cast<char>(type),      static_cast<char>(flags),    static_cast<char>((sid >> 24) & 0x7f),
                     static_cast<char>(sid >> 16), static_cast<char>(sid >> 8), static_cast<char>(sid)};
  o->append(h, 9);
}

void Put32(std::string* o, uint32_t v) {
  const char b[4] = {static_cast<char>(v >> 24), static_cast<char>(v >> 16), static_cast<char>(v >> 8),
                     static_cast<char>(v)};
  o->append(b, 4);
}

// HPACK integer with an N-bit prefix (RFC 7541 §5.1).
void PutHpackInt(std::string* o, uint8_t first, int prefix_bits, size_t v) {
  const size_t max = (size_t(1) << prefix_bits) - 1;
  if (v < max) {
    o->push_back(static_cast<char>(first | v));
    return;
  }
  o->push_back(static_cast<char>(first | max));
  v -= max;
  while (v >= 128) {
    o->push_back(static_cast<char>((v & 0x7f) | 0x80));
    v >>= 7;
  }
  o->push_back(static_cast<char>(v));
}

// Literal header field without indexing, new name, raw (non-Huffman) strings.
void PutLiteral(std::string* o, std::string_view name, std::string_view value) {
  o->push_back(0);
  PutHpackInt(o, 0, 7, name.size());
  o->append(name);
  PutHpackInt(o, 0, 7, value.size());
  o->append(value);
}

// The two header fields every response repeats. The encoder inserts each into
// the HPACK dynamic table the first time it sends it (literal with incremental
// indexing) and refers to it by index afterwards, so the peer's decoder does a
// table lookup instead of copying strings -- what nghttp2's deflater would do.
// Nothing else is ever inserted, so the table holds at most these two entries
// (32 + 12 + 16 and 32 + 11 + 1 = 104 bytes) and never evicts.
constexpr size_t kDynEntriesSize = 104;

struct H2Stream {
  const UnaryHandler* unary = nullptr;
  const StreamHandler* stream_handler = nullptr;
  std::string path;          // kept only when unresolved or traced
  bool grpc_content_type = false;
  std::string content_type;  // kept only when not application/grpc*
  std::string body;
  bool dispatched = false;
  bool remote_closed = false;  // END_STREAM received
  bool finishing = false;      // trailers go out once `out` drains
  bool trailers_sent = false;
  int grpc_status = 0;
  std::string grpc_message;
  std::string out;  // framed gRPC message(s) not yet sent as DATA
  size_t out_off = 0;
  std::string pending;  // server streams: newest message while `out` is in flight
  int64_t send_window = kDefaultWindow;
  uint32_t recv_unacked = 0;
  std::shared_ptr<ServerStream> stream;
};

class H2Conn final : public ServerConn {
 public:
  H2Conn(Server* srv, int loop, int fd) : ServerConn(srv, loop, fd) {}
  ~H2Conn() override {
    for (auto& [_, st] : streams_) Detach(st.stream.get());
    if (inflater_) nghttp2_hd_inflate_del(inflater_);
    if (fd_ >= 0) close(fd_);
  }

  bool Init() override;
  bool OnReadable() override;
  bool Flush() override;
  bool Done() const override {
    return woff_ == wbuf_.size() && (closing_ || (peer_goaway_ && streams_.empty()));
  }
  bool want_epollout() const override { return wbuf_.size() > woff_; }
  bool QueueMessage(int32_t sid, std::string_view msg) override;
  void Finish(int32_t sid, const Status& st) override;

 private:
  // Processes whole frames; returns the bytes consumed (all of them after a
  // connection error, which queues GOAWAY and sets closing_).
  size_t Consume(const uint8_t* p, size_t n);
  bool OnFrame(uint8_t type, uint8_t flags, uint32_t sid, const uint8_t* p, size_t len);
  bool OnData(uint8_t flags, uint32_t sid, const uint8_t* p, size_t len);
  bool OnHeaders(uint8_t flags, uint32_t sid, const uint8_t* p, size_t len);
  bool OnContinuation(uint8_t flags, uint32_t sid, const uint8_t* p, size_t len);
  bool OnSettings(uint8_t flags, uint32_t sid, const uint8_t* p, size_t len);
  bool OnWindowUpdate(uint32_t sid, const uint8_t* p, size_t len);
  bool DecodeHeaderBlock(const uint8_t* p, size_t len);
  bool ConnError(uint32_t code, const char* why);

  H2Stream* Find(uint32_t sid) {
    auto it = streams_.find(sid);
    return it == streams_.end() ? nullptr : &it->second;
  }
  void Erase(uint32_t sid);
  void MaybeErase(uint32_t sid, H2Stream& st) {
    if (st.remote_closed && st.trailers_sent) Erase(sid);
  }
  void Dispatch(uint32_t sid, H2Stream& st, std::string_view body);
  void SendHeaderBlock(uint32_t sid, std::string_view block, bool end_stream);
  void SendResponseHeaders(uint32_t sid);
  void SendTrailersOnly(uint32_t sid, int code, std::string_view msg);
  void SendTrailers(uint32_t sid, H2Stream& st);
  void RstStream(uint32_t sid, uint32_t code);
  void WindowUpdate(uint32_t sid, uint32_t inc);
  // Moves as much of the stream's queued data as the windows allow into wbuf_,
  // then its trailers once everything went out.
  void Pump(uint32_t sid, H2Stream& st);
  void PumpAll();

  nghttp2_hd_inflater* inflater_ = nullptr;
  bool preface_ok_ = false;
  bool closing_ = false;      // connection error: GOAWAY queued, close after the write
  bool peer_goaway_ = false;  // peer sent GOAWAY: finish open streams, then close
  bool aborted_ = false;      // close now, dropping queued output
  size_t discarded_ = 0;      // bytes read and dropped since closing_ (bounded: kMaxDiscardAfterError)
  std::string rbuf_;          // incomplete frame carried over to the next read
  std::string wbuf_;
  size_t woff_ = 0;
  std::string resp_buf_;      // unary handler output (reused)
  std::string hblock_;        // scratch for header blocks we send

  std::map<uint32_t, H2Stream> streams_;
  uint32_t last_sid_ = 0;  // highest client stream id seen
  size_t buffered_ = 0;    // sum of the open streams' request bodies

  // Peer settings / send side.
  uint32_t peer_max_frame_ = 16384;
  int64_t peer_initial_window_ = kDefaultWindow;
  int64_t conn_send_window_ = kDefaultWindow;
  uint32_t hpack_table_size_ = 4096;  // our encoder's table limit as the peer set it
  bool hpack_size_update_ = false;    // emit a table size update in the next block
  // HPACK encoder dynamic table: insertion number of content-type / grpc-status 0
  // (-1 = not inserted); index = 62 + (inserted - 1 - number).
  int dyn_ct_ = -1, dyn_status0_ = -1, dyn_inserted_ = 0;
  void PutContentType(std::string* b);
  void PutStatusOk(std::string* b);

  // Receive side.
  uint32_t conn_recv_unacked_ = 0;

  // Header block being received (HEADERS [+ CONTINUATION]).
  bool expect_continuation_ = false;
  uint32_t hb_sid_ = 0;
  bool hb_end_stream_ = false;
  bool hb_request_ = false;  // opens a new stream (vs. client trailers / ignored)
  bool hb_refuse_ = false;   // new stream beyond MAX_CONCURRENT_STREAMS
  std::string hb_buf_;
  H2Stream* hb_stream_ = nullptr;  // target of :path / content-type while decoding
};

bool H2Conn::Init() {
  if (nghttp2_hd_inflate_new(&inflater_) != 0) return false;
  // Server preface: SETTINGS, then open the connection receive window.
  PutFrameHeader(&wbuf_, 18, kSettings, 0, 0);
  const uint16_t ids[3] = {0x3 /*MAX_CONCURRENT_STREAMS*/, 0x4 /*INITIAL_WINDOW_SIZE*/,
                           0x5 /*MAX_FRAME_SIZE*/};
  const uint32_t vals[3] = {kMaxStreams, kOurStreamWindow, kOurMaxFrame};
  for (int i = 0; i < 3; ++i) {
    wbuf_.push_back(static_cast<char>(ids[i] >> 8));
    wbuf_.push_back(static_cast<char>(ids[i]));
    Put32(&wbuf_, vals[i]);
  }
  WindowUpdate(0, kOurConnWindow - kDefaultWindow);
  return Flush();
}

bool H2Conn::OnReadable() {
  uint8_t buf[64 * 1024];
  ReadStarted();
  bool eof = false;
  size_t budget = kReadBudgetPerWake;
  while (!eof && !aborted_) {
    ssize_t n = read(fd_, buf, sizeof(buf));
    if (n > 0) {
      if (closing_) {
        // Draining after a connection error until the peer stops sending (then
        // the GOAWAY is written) -- but a peer that keeps sending would keep
        // this loop here for ever (it never sees EAGAIN): cut off past a bound.
        discarded_ += static_cast<size_t>(n);
        if (discarded_ > kMaxDiscardAfterError) aborted_ = true;
        continue;
      }
      budget -= std::min(budget, static_cast<size_t>(n));
      if (rbuf_.empty()) {
        // Common case: whole frames in this read, parsed in place.
        size_t used = Consume(buf, static_cast<size_t>(n));
        if (used < static_cast<size_t>(n) && !closing_) rbuf_.assign(reinterpret_cast<char*>(buf) + used, n - used);
      } else {
        rbuf_.append(reinterpret_cast<char*>(buf), static_cast<size_t>(n));
        size_t used = Consume(reinterpret_cast<const uint8_t*>(rbuf_.data()), rbuf_.size());
        rbuf_.erase(0, used);
      }
      if (static_cast<size_t>(n) < sizeof(buf) || (budget == 0 && !closing_)) break;
      continue;
    }
    if (n == 0) {
      eof = true;
      break;
    }
    if (errno == EINTR) continue;
    if (errno == EAGAIN || errno == EWOULDBLOCK) break;
    return false;
  }
  if (eof || aborted_) return false;  // peer closed the connection, or it is cut off
  return Flush();
}

size_t H2Conn::Consume(const uint8_t* p, size_t n) {
  size_t off = 0;
  if (!preface_ok_) {
    size_t k = n < kPrefaceLen ? n : kPrefaceLen;
    if (memcmp(p, kPreface, k) != 0) {
      ConnError(kProtocolError, "bad client preface");
      return n;
    }
    if (n < kPrefaceLen) return 0;
    preface_ok_ = true;
    off = kPrefaceLen;
  }
  while (!closing_ && n - off >= 9) {
    const uint8_t* h = p + off;
    uint32_t len = Get24(h);
    if (len > kOurMaxFrame) {
      ConnError(kFrameSizeError, "frame larger than SETTINGS_MAX_FRAME_SIZE");
      return n;
    }
    if (n - off - 9 < len) break;
    if (wbuf_.size() - woff_ > kMaxQueuedOutput) {
      ConnError(kEnhanceYourCalm, "peer does not read its replies");
      aborted_ = true;  // the GOAWAY could never be written either: just close
      return n;
    }
    if (!OnFrame(h[3], h[4], Get32(h + 5) & 0x7fffffff, h + 9, len)) return n;
    off += 9 + len;
  }
  return closing_ ? n : off;
}

bool H2Conn::ConnError(uint32_t code, const char* why) {
  if (closing_) return false;
  LOG_DEBUG(kComp, "HTTP/2 connection error %u: %s", code, why);
  PutFrameHeader(&wbuf_, 8, kGoaway, 0, 0);
  Put32(&wbuf_, last_sid_);
  Put32(&wbuf_, code);
  closing_ = true;
  rbuf_.clear();
  return false;
}

bool H2Conn::OnFrame(uint8_t type, uint8_t flags, uint32_t sid, const uint8_t* p, size_t len) {
  if (expect_continuation_ && type != kContinuation)
    return ConnError(kProtocolError, "expected CONTINUATION");
  switch (type) {
    case kData:
      return OnData(flags, sid, p, len);
    case kHeaders:
      return OnHeaders(flags, sid, p, len);
    case kContinuation:
      return OnContinuation(flags, sid, p, len);
    case kPriority:
      if (sid == 0) return ConnError(kProtocolError, "PRIORITY on stream 0");
      return true;
    case kRstStream:
      if (sid == 0) return ConnError(kProtocolError, "RST_STREAM on stream 0");
      if (len != 4) return ConnError(kFrameSizeError, "RST_STREAM length");
      if (sid > last_sid_) return ConnError(kProtocolError, "RST_STREAM on idle stream");
      Erase(sid);
      return true;
    case kSettings:
      return OnSettings(flags, sid, p, len);
    case kPushPromise:
      return ConnError(kProtocolError, "PUSH_PROMISE from a client");
    case kPing:
      if (sid != 0) return ConnError(kProtocolError, "PING on a stream");
      if (len != 8) return ConnError(kFrameSizeError, "PING length");
      if (!(flags & kFlagAck)) {
        PutFrameHeader(&wbuf_, 8, kPing, kFlagAck, 0);
        wbuf_.append(reinterpret_cast<const char*>(p), 8);
      }
      return true;
    case kGoaway:
      if (sid != 0) return ConnError(kProtocolError, "GOAWAY on a stream");
      if (len < 8) return ConnError(kFrameSizeError, "GOAWAY length");
      peer_goaway_ = true;
      return true;
    case kWindowUpdate:
      return OnWindowUpdate(sid, p, len);
    default:
      return true;  // unknown frame types are ignored (RFC 7540 §4.1)
  }
}

bool H2Conn::OnData(uint8_t flags, uint32_t sid, const uint8_t* p, size_t len) {
  if (sid == 0) return ConnError(kProtocolError, "DATA on stream 0");
  // Flow control counts the whole payload, padding included.
  conn_recv_unacked_ += static_cast<uint32_t>(len);
  if (conn_recv_unacked_ >= kConnAckBytes) {
    WindowUpdate(0, conn_recv_unacked_);
    conn_recv_unacked_ = 0;
  }
  const uint8_t* data = p;
  size_t dlen = len;
  if (flags & kFlagPadded) {
    if (len < 1 || p[0] >= len) return ConnError(kProtocolError, "bad DATA padding");
    data = p + 1;
    dlen = len - 1 - p[0];
  }
  H2Stream* st = Find(sid);
  if (!st) {
    if (sid > last_sid_) return ConnError(kProtocolError, "DATA on idle stream");
    return true;  // stream already closed or reset: dropped
  }
  if (st->remote_closed) {
    RstStream(sid, kStreamClosed);
    return true;
  }
  const bool end = flags & kFlagEndStream;
  if (!end) {
    st->recv_unacked += static_cast<uint32_t>(len);
    if (st->recv_unacked >= kStreamAckBytes) {
      WindowUpdate(sid, st->recv_unacked);
      st->recv_unacked = 0;
    }
  }
  if (!st->dispatched) {
    if (st->body.size() + dlen > kMaxRequestBytes) {
      RstStream(sid, kRefusedStream);  // never hand a truncated request to a handler
      return true;
    }
    if (end && st->body.empty()) {
      st->remote_closed = true;
      Dispatch(sid, *st, std::string_view(reinterpret_cast<const char*>(data), dlen));  // zero-copy
      if ((st = Find(sid))) MaybeErase(sid, *st);
      return true;
    }
    if (buffered_ + dlen > kMaxBufferedRequests)
      return ConnError(kEnhanceYourCalm, "too many request bytes buffered");
    st->body.append(reinterpret_cast<const char*>(data), dlen);
    buffered_ += dlen;
  }
  if (end) {
    st->remote_closed = true;
    if (!st->dispatched) Dispatch(sid, *st, st->body);
    if ((st = Find(sid))) MaybeErase(sid, *st);
  }
  return true;
}

bool H2Conn::OnHeaders(uint8_t flags, uint32_t sid, const uint8_t* p, size_t len) {
  if (sid == 0 || (sid & 1) == 0) return ConnError(kProtocolError, "HEADERS on an invalid stream id");
  size_t off = 0, pad = 0;
  if (flags & kFlagPadded) {
    if (len < 1) return ConnError(kProtocolError, "bad HEADERS padding");
    pad = p[0];
    off = 1;
  }
  if (flags & kFlagPriority) off += 5;
  if (off + pad > len) return ConnError(kProtocolError, "bad HEADERS padding");
  hb_sid_ = sid;
  hb_end_stream_ = flags & kFlagEndStream;
  hb_request_ = false;
  hb_refuse_ = false;
  hb_stream_ = nullptr;
  if (H2Stream* st = Find(sid)) {
    // Trailers from the client: must end the stream; their fields are ignored.
    if (!hb_end_stream_ || st->remote_closed) return ConnError(kProtocolError, "unexpected HEADERS");
  } else if (sid > last_sid_) {
    last_sid_ = sid;
    hb_request_ = true;
    if (streams_.size() >= kMaxStreams || peer_goaway_) {
      hb_refuse_ = true;
    } else {
      H2Stream& ns = streams_[sid];
      ns.send_window = peer_initial_window_;
      hb_stream_ = &ns;
    }
  }
  // (HEADERS on a closed stream: decoded for the HPACK state, then dropped.)
  const uint8_t* frag = p + off;
  size_t flen = len - off - pad;
  if (flags & kFlagEndHeaders) return DecodeHeaderBlock(frag, flen);
  expect_continuation_ = true;
  hb_buf_.assign(reinterpret_cast<const char*>(frag), flen);
  return true;
}

bool H2Conn::OnContinuation(uint8_t flags, uint32_t sid, const uint8_t* p, size_t len) {
  if (!expect_continuation_ || sid != hb_sid_) return ConnError(kProtocolError, "unexpected CONTINUATION");
  if (hb_buf_.size() + len > kMaxHeaderBlock) return ConnError(kEnhanceYourCalm, "header block too large");
  hb_buf_.append(reinterpret_cast<const char*>(p), len);
  if (!(flags & kFlagEndHeaders)) return true;
  expect_continuation_ = false;
  std::string block = std::move(hb_buf_);
  hb_buf_.clear();
  return DecodeHeaderBlock(reinterpret_cast<const uint8_t*>(block.data()), block.size());
}

bool H2Conn::DecodeHeaderBlock(const uint8_t* in, size_t inlen) {
  for (;;) {
    nghttp2_nv nv;
    int inflate_flags = 0;
    ssize_t rv = nghttp2_hd_inflate_hd2(inflater_, &nv, &inflate_flags, in, inlen, 1);
    if (rv < 0) return ConnError(kCompressionError, "HPACK decoding failed");
    in += rv;
    inlen -= static_cast<size_t>(rv);
    if ((inflate_flags & NGHTTP2_HD_INFLATE_EMIT) && hb_stream_) {
      std::string_view n(reinterpret_cast<const char*>(nv.name), nv.namelen);
      std::string_view v(reinterpret_cast<const char*>(nv.value), nv.valuelen);
      H2Stream& st = *hb_stream_;
      if (n == ":path") {
        st.unary = FindUnary(v);
        if (!st.unary) st.stream_handler = FindStreamHandler(v);
        if ((!st.unary && !st.stream_handler) || tracing()) st.path.assign(v);
      } else if (n == "content-type") {
        st.grpc_content_type = StartsWithGrpc(v);
        if (!st.grpc_content_type) st.content_type.assign(v);
      }
    }
    if (inflate_flags & NGHTTP2_HD_INFLATE_FINAL) {
      nghttp2_hd_inflate_end_headers(inflater_);
      break;
    }
    if ((inflate_flags & NGHTTP2_HD_INFLATE_EMIT) == 0 && inlen == 0) break;
  }
  const uint32_t sid = hb_sid_;
  hb_stream_ = nullptr;
  if (hb_refuse_) {
    RstStream(sid, kRefusedStream);
    return true;
  }
  H2Stream* st = Find(sid);
  if (!st || !hb_end_stream_) return true;
  st->remote_closed = true;
  if (!st->dispatched) Dispatch(sid, *st, st->body);
  if ((st = Find(sid))) MaybeErase(sid, *st);
  return true;
}

bool H2Conn::OnSettings(uint8_t flags, uint32_t sid, const uint8_t* p, size_t len) {
  if (sid != 0) return ConnError(kProtocolError, "SETTINGS on a stream");
  if (flags & kFlagAck) {
    if (len != 0) return ConnError(kFrameSizeError, "SETTINGS ACK with payload");
    return true;
  }
  if (len % 6 != 0) return ConnError(kFrameSizeError, "SETTINGS length");
  for (size_t i = 0; i < len; i += 6) {
    uint16_t id = static_cast<uint16_t>((p[i] << 8) | p[i + 1]);
    uint32_t v = Get32(p + i + 2);
    switch (id) {
      case 0x1:  // HEADER_TABLE_SIZE: our encoder must not exceed it
        if (v < hpack_table_size_) {
          hpack_table_size_ = v;
          hpack_size_update_ = true;  // next block: size update 0 + v, table restarts empty
          dyn_ct_ = dyn_status0_ = -1;
          dyn_inserted_ = 0;
        }
        break;
      case 0x2:  // ENABLE_PUSH
        if (v > 1) return ConnError(kProtocolError, "bad ENABLE_PUSH");
        break;
      case 0x4: {  // INITIAL_WINDOW_SIZE: applies the delta to every open stream
        if (v > kMaxWindow) return ConnError(kFlowControlError, "bad INITIAL_WINDOW_SIZE");
        int64_t delta = static_cast<int64_t>(v) - peer_initial_window_;
        peer_initial_window_ = v;
        for (auto& [_, st] : streams_) {
          st.send_window += delta;
          if (st.send_window > kMaxWindow) return ConnError(kFlowControlError, "stream window overflow");
        }
        break;
      }
      case 0x5:  // MAX_FRAME_SIZE
        if (v < 16384 || v > 0xffffff) return ConnError(kProtocolError, "bad MAX_FRAME_SIZE");
        peer_max_frame_ = v;
        break;
      default:  // MAX_CONCURRENT_STREAMS, MAX_HEADER_LIST_SIZE, unknown: nothing to do
        break;
    }
  }
  PutFrameHeader(&wbuf_, 0, kSettings, kFlagAck, 0);
  PumpAll();  // a larger initial window may unblock queued data
  return true;
}

bool H2Conn::OnWindowUpdate(uint32_t sid, const uint8_t* p, size_t len) {
  if (len != 4) return ConnError(kFrameSizeError, "WINDOW_UPDATE length");
  uint32_t inc = Get32(p) & 0x7fffffff;
  if (sid == 0) {
    if (inc == 0) return ConnError(kProtocolError, "WINDOW_UPDATE of 0");
    conn_send_window_ += inc;
    if (conn_send_window_ > kMaxWindow) return ConnError(kFlowControlError, "connection window overflow");
    PumpAll();
    return true;
  }
  H2Stream* st = Find(sid);
  if (!st) {
    if (sid > last_sid_) return ConnError(kProtocolError, "WINDOW_UPDATE on idle stream");
    return true;
  }
  if (inc == 0) {
    RstStream(sid, kProtocolError);
    return true;
  }
  st->send_window += inc;
  if (st->send_window > kMaxWindow) {
    RstStream(sid, kFlowControlError);
    return true;
  }
  Pump(sid, *st);
  return true;
}

void H2Conn::Erase(uint32_t sid) {
  auto it = streams_.find(sid);
  if (it == streams_.end()) return;
  buffered_ -= it->second.body.size();
  Detach(it->second.stream.get());
  streams_.erase(it);
}

void H2Conn::RstStream(uint32_t sid, uint32_t code) {
  PutFrameHeader(&wbuf_, 4, kRstStream, 0, sid);
  Put32(&wbuf_, code);
  Erase(sid);
}

void H2Conn::WindowUpdate(uint32_t sid, uint32_t inc) {
  PutFrameHeader(&wbuf_, 4, kWindowUpdate, 0, sid);
  Put32(&wbuf_, inc);
}

void H2Conn::PutContentType(std::string* b) {
  if (dyn_ct_ >= 0) {
    PutHpackInt(b, 0x80, 7, 62 + (dyn_inserted_ - 1 - dyn_ct_));
  } else if (hpack_table_size_ >= kDynEntriesSize) {
    b->append("\x5f\x10" "application/grpc");  // incremental indexing, name = static 31
    dyn_ct_ = dyn_inserted_++;
  } else {
    b->append("\x0f\x10\x10" "application/grpc");  // without indexing
  }
}

void H2Conn::PutStatusOk(std::string* b) {
  if (dyn_status0_ >= 0) {
    PutHpackInt(b, 0x80, 7, 62 + (dyn_inserted_ - 1 - dyn_status0_));
  } else if (hpack_table_size_ >= kDynEntriesSize) {
    b->append("\x40\x0bgrpc-status\x01" "0", 15);  // incremental indexing, new name
    dyn_status0_ = dyn_inserted_++;
  } else {
    PutLiteral(b, "grpc-status", "0");
  }
}

void H2Conn::SendHeaderBlock(uint32_t sid, std::string_view block, bool end_stream) {
  // `block` was encoded against the table state after any pending size update
  // (the callers build it after this connection's SETTINGS were applied).
  std::string_view prefix;
  std::string upd;
  if (hpack_size_update_) {
    // RFC 7541 §4.2: first block after the peer lowered SETTINGS_HEADER_TABLE_SIZE.
    // Size 0 first (evicts everything), then the new limit.
    upd.push_back(0x20);
    if (hpack_table_size_ > 0) PutHpackInt(&upd, 0x20, 5, hpack_table_size_);
    prefix = upd;
    hpack_size_update_ = false;
  }
  const size_t total = prefix.size() + block.size();
  const uint8_t es = end_stream ? kFlagEndStream : 0;
  if (total <= peer_max_frame_) {
    PutFrameHeader(&wbuf_, total, kHeaders, es | kFlagEndHeaders, sid);
    wbuf_.append(prefix);
    wbuf_.append(block);
    return;
  }
  std::string all(prefix);
  all.append(block);
  size_t off = 0;
  bool first = true;
  while (off < all.size()) {
    size_t n = std::min<size_t>(peer_max_frame_, all.size() - off);
    bool last = off + n == all.size();
    PutFrameHeader(&wbuf_, n, first ? kHeaders : kContinuation,
                   static_cast<uint8_t>((first ? es : 0) | (last ? kFlagEndHeaders : 0)), sid);
    wbuf_.append(all, off, n);
    off += n;
    first = false;
  }
}

void H2Conn::SendResponseHeaders(uint32_t sid) {
  hblock_.assign(1, '\x88');  // :status 200 (static index 8)
  PutContentType(&hblock_);
  SendHeaderBlock(sid, hblock_, false);
}

void H2Conn::SendTrailersOnly(uint32_t sid, int code, std::string_view msg) {
  hblock_.assign(1, '\x88');
  PutContentType(&hblock_);
  PutLiteral(&hblock_, "grpc-status", std::to_string(code));
  std::string m = PercentEncode(msg.substr(0, kMaxGrpcMessageHeader));
  if (!m.empty()) PutLiteral(&hblock_, "grpc-message", m);
  SendHeaderBlock(sid, hblock_, true);
  CountError();
}

void H2Conn::SendTrailers(uint32_t sid, H2Stream& st) {
  if (st.grpc_status == 0 && st.grpc_message.empty()) {
    hblock_.clear();
    PutStatusOk(&hblock_);
    SendHeaderBlock(sid, hblock_, true);
  } else {
    hblock_.clear();
    PutLiteral(&hblock_, "grpc-status", std::to_string(st.grpc_status));
    std::string m = PercentEncode(std::string_view(st.grpc_message).substr(0, kMaxGrpcMessageHeader));
    if (!m.empty()) PutLiteral(&hblock_, "grpc-message", m);
    SendHeaderBlock(sid, hblock_, true);
  }
  st.trailers_sent = true;
}

void H2Conn::Pump(uint32_t sid, H2Stream& st) {
  while (st.out_off < st.out.size()) {
    int64_t n = static_cast<int64_t>(st.out.size() - st.out_off);
    n = std::min<int64_t>(n, peer_max_frame_);
    n = std::min<int64_t>(n, conn_send_window_);
    n = std::min<int64_t>(n, st.send_window);
    if (n <= 0) return;  // blocked until the peer opens a window
    PutFrameHeader(&wbuf_, static_cast<size_t>(n), kData, 0, sid);
    wbuf_.append(st.out, st.out_off, static_cast<size_t>(n));
    st.out_off += static_cast<size_t>(n);
    conn_send_window_ -= n;
    st.send_window -= n;
    if (st.out_off == st.out.size()) {
      st.out.clear();
      st.out_off = 0;
      if (!st.pending.empty()) st.out.swap(st.pending);  // next (latest) message
    }
  }
  if (st.finishing && !st.trailers_sent) {
    SendTrailers(sid, st);
    MaybeErase(sid, st);
  }
}

void H2Conn::PumpAll() {
  for (auto it = streams_.begin(); it != streams_.end();) {
    uint32_t sid = it->first;
    ++it;  // Pump may erase the current stream
    H2Stream* st = Find(sid);
    if (st && (st->out_off < st->out.size() || (st->finishing && !st->trailers_sent))) Pump(sid, *st);
  }
}

void H2Conn::Dispatch(uint32_t sid, H2Stream& st, std::string_view body) {
  st.dispatched = true;
  CountCall();
  std::string_view req;
  int code = 0;
  std::string msg;
  if (!ParseRequest(st.grpc_content_type, st.content_type, body, &req, &code, &msg)) {
    SendTrailersOnly(sid, code, msg);
    st.trailers_sent = true;
    return;
  }
  if (st.unary) {
    Answered();
    std::string& resp = resp_buf_;
    Status s = RunUnary(*st.unary, st.path, req, &resp);
    if (!s.ok()) {
      SendTrailersOnly(sid, ToGrpcCode(s.code()), s.message());
      st.trailers_sent = true;
      return;
    }
    SendResponseHeaders(sid);
    FrameMessage(resp, &st.out);
    st.finishing = true;
    Pump(sid, st);  // DATA + trailers when the windows allow (a small reply: at once)
    return;
  }
  if (st.stream_handler) {
    auto stream = OpenStream(static_cast<int32_t>(sid));
    st.stream = stream;
    SendResponseHeaders(sid);
    Status s = (*st.stream_handler)(req, stream);
    if (!s.ok() && !StreamClosed(*stream)) stream->Finish(s);
    return;
  }
  SendTrailersOnly(sid, kGrpcUnimplemented, "unknown method " + st.path);
  st.trailers_sent = true;
}

bool H2Conn::QueueMessage(int32_t sid, std::string_view msg) {
  H2Stream* st = Find(static_cast<uint32_t>(sid));
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
  Pump(static_cast<uint32_t>(sid), *st);
  return true;
}

void H2Conn::Finish(int32_t sid, const Status& s) {
  H2Stream* st = Find(static_cast<uint32_t>(sid));
  if (!st || st->finishing) return;
  st->finishing = true;
  st->grpc_status = ToGrpcCode(s.code());
  st->grpc_message = s.ok() ? "" : s.message();
  Pump(static_cast<uint32_t>(sid), *st);
}

bool H2Conn::Flush() {
  if (woff_ < wbuf_.size()) Sending();
  while (woff_ < wbuf_.size()) {
    ssize_t n = send(fd_, wbuf_.data() + woff_, wbuf_.size() - woff_, MSG_NOSIGNAL);
    if (n > 0) {
      woff_ += static_cast<size_t>(n);
      continue;
    }
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

}  // namespace

std::unique_ptr<ServerConn> MakeH2Conn(Server* srv, int loop, int fd) {
  return std::make_unique<H2Conn>(srv, loop, fd);
}

}  // namespace adp::grpc
