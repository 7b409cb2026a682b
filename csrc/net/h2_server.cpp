#include "net/h2_server.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <deque>
#include <stdexcept>
#include <unordered_map>

#include "net/hpack.h"
#include "runtime/batcher.h"  // now_us()

namespace dtfs {
namespace net {

namespace {

enum : uint8_t {
  kData = 0,
  kHeaders = 1,
  kPriority = 2,
  kRstStream = 3,
  kSettings = 4,
  kPushPromise = 5,
  kPing = 6,
  kGoaway = 7,
  kWindowUpdate = 8,
  kContinuation = 9,
};
enum : uint8_t { kEndStream = 0x1, kAck = 0x1, kEndHeaders = 0x4, kPadded = 0x8, kPrioFlag = 0x20 };
enum : uint32_t {
  kNoError = 0,
  kProtocolError = 1,
  kInternalError = 2,
  kFlowControlError = 3,
  kStreamClosed = 5,
  kFrameSizeError = 6,
  kRefusedStream = 7,
  kCompressionError = 9,
  kEnhanceYourCalm = 11,
};

const char kPreface[] = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n";  // 24 bytes
constexpr uint32_t kOurMaxFrame = 1u << 20;                // SETTINGS_MAX_FRAME_SIZE we accept
constexpr int64_t kOurStreamWindow = 16 << 20;             // SETTINGS_INITIAL_WINDOW_SIZE we grant
constexpr int64_t kOurConnWindow = int64_t(1) << 30;       // connection window we grant
constexpr int64_t kMaxWindow = (int64_t(1) << 31) - 1;
constexpr uint64_t kListenTag = 0, kWakeTag = 1;
// Per-connection memory bounds (a client that never finishes a header block,
// or never reads what it asks for, must not grow the server without limit):
// a header block (HEADERS + CONTINUATION) and its decoded list are capped at
// SETTINGS_MAX_HEADER_LIST_SIZE (advertised; GOAWAY ENHANCE_YOUR_CALM past
// it), and while more than kMaxOutBacklog bytes wait unsent the connection's
// input is not read (no PING / SETTINGS acks queue up behind a stalled reader).
constexpr uint32_t kMaxHeaderList = 64 << 10;
constexpr size_t kMaxOutBacklog = size_t(16) << 20;

uint32_t be32(const uint8_t* p) { return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3]; }

void put_frame_header(std::string* out, uint32_t len, uint8_t type, uint8_t flags, uint32_t sid) {
  const char h[9] = {char(len >> 16), char(len >> 8), char(len), char(type), char(flags),
                     char((sid >> 24) & 0x7f), char(sid >> 16), char(sid >> 8), char(sid)};
  out->append(h, 9);
}

void put_u32(std::string* out, uint32_t v) {
  const char b[4] = {char(v >> 24), char(v >> 16), char(v >> 8), char(v)};
  out->append(b, 4);
}

struct Stream {
  uint32_t id = 0;
  bool headers_done = false, dispatched = false, too_big = false;
  std::string path, method, content_type, encoding;
  int64_t deadline_us = 0;
  std::string body;
  int64_t recv_unacked = 0;  // DATA bytes not yet granted back (stream window)
  int64_t send_window = 65535;
  std::string pending;   // reply DATA payload not yet sent (flow control)
  size_t pending_off = 0;
  std::string trailers;  // header block sent once pending is out
  bool replying = false;
};

struct Conn {
  uint64_t id = 0;
  int fd = -1;
  std::string in, out;
  size_t in_off = 0, out_off = 0;
  bool preface = false, want_write = false, peer_goaway = false, dead = false;
  HpackDecoder hpack{4096};
  std::unordered_map<uint32_t, Stream> streams;
  // header block in progress (HEADERS then CONTINUATION until END_HEADERS)
  uint32_t block_sid = 0;
  bool block_end_stream = false;
  std::string block;
  uint32_t last_sid = 0;
  int64_t send_window = 65535;  // peer's connection window for our DATA
  int64_t peer_initial = 65535;
  uint32_t peer_max_frame = 16384;
  int64_t recv_unacked = 0;
  std::deque<uint32_t> blocked;  // streams waiting for window
  bool read_paused = false;      // out backlog over kMaxOutBacklog: EPOLLIN off
  // lingering close after our GOAWAY: the GOAWAY goes out, then our write side
  // shuts (FIN) and what the peer still sends is read and dropped until it
  // closes or the deadline passes. Closing a socket with unread input sends an
  // RST, which can destroy the GOAWAY in the peer's receive queue.
  bool closing = false, shut_wr = false;
  std::chrono::steady_clock::time_point close_by{};
  size_t backlog() const { return out.size() - out_off; }
};

}  // namespace

struct Posted {
  uint64_t conn;
  uint32_t stream;
  int status;
  std::string message, body;
};

class Loop : public std::enable_shared_from_this<Loop> {
 public:
  Loop(const H2Config& cfg, const GrpcHandler* handler, int lfd, int index)
      : cfg_(cfg), handler_(handler), lfd_(lfd), next_id_((uint64_t(index) << 48) + 2) {
    ep_ = epoll_create1(EPOLL_CLOEXEC);
    efd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    if (ep_ < 0 || efd_ < 0) throw std::runtime_error("epoll / eventfd failed");
    add(lfd_, kListenTag, EPOLLIN);
    add(efd_, kWakeTag, EPOLLIN);
  }
  ~Loop() {
    for (auto& kv : conns_) ::close(kv.second->fd);
    ::close(lfd_);
    ::close(efd_);
    ::close(ep_);
  }

  void post(Posted&& p) {
    {
      std::lock_guard<std::mutex> lk(q_mu_);
      if (stop_) {
        ++st_.dropped_replies;
        return;
      }
      q_.push_back(std::move(p));
    }
    const uint64_t one = 1;
    (void)!::write(efd_, &one, 8);
  }

  void stop() {
    {
      std::lock_guard<std::mutex> lk(q_mu_);
      stop_ = true;
    }
    const uint64_t one = 1;
    (void)!::write(efd_, &one, 8);
  }

  H2Stats stats() const {
    std::lock_guard<std::mutex> lk(q_mu_);
    return st_;
  }

  void run() {
    epoll_event evs[128];
    for (;;) {
      {
        std::lock_guard<std::mutex> lk(q_mu_);
        if (stop_) break;
      }
      const int n = epoll_wait(ep_, evs, 128, 200);
      for (int i = 0; i < n; ++i) {
        const uint64_t tag = evs[i].data.u64;
        if (tag == kListenTag) {
          accept_all();
        } else if (tag == kWakeTag) {
          uint64_t v;
          (void)!::read(efd_, &v, 8);
        } else {
          auto it = conns_.find(tag);
          if (it == conns_.end()) continue;
          Conn& c = *it->second;
          if (evs[i].events & (EPOLLERR | EPOLLHUP)) c.dead = true;
          if (!c.dead && c.closing) {
            if (evs[i].events & EPOLLOUT) flush(c);
            if (!c.dead && (evs[i].events & EPOLLIN)) discard_input(c);
            if (!c.dead) shut_when_flushed(c);
            if (c.dead) close_conn(tag);
            continue;
          }
          if (!c.dead && (evs[i].events & EPOLLIN)) on_readable(c);
          if (!c.dead && (evs[i].events & EPOLLOUT)) flush(c);
          if (c.dead || (!c.closing && c.peer_goaway && c.streams.empty() && c.out_off == c.out.size()))
            close_conn(tag);
        }
      }
      drain_replies();
      resume_paused();
      reap_closing();
    }
    // graceful-ish stop: GOAWAY to every client, then close
    for (auto& kv : conns_) {
      Conn& c = *kv.second;
      std::string g;
      put_frame_header(&g, 8, kGoaway, 0, 0);
      put_u32(&g, c.last_sid);
      put_u32(&g, kNoError);
      c.out.append(g);
      flush(c);
    }
  }

 private:
  void add(int fd, uint64_t tag, uint32_t events) {
    epoll_event e{};
    e.events = events;
    e.data.u64 = tag;
    if (epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &e) != 0) throw std::runtime_error("epoll_ctl add failed");
  }

  void set_write_interest(Conn& c, bool on) {
    if (c.want_write == on) return;
    c.want_write = on;
    update_events(c);
  }

  void update_events(Conn& c) {
    epoll_event e{};
    e.events = (c.read_paused ? 0u : uint32_t(EPOLLIN)) | (c.want_write ? uint32_t(EPOLLOUT) : 0u);
    e.data.u64 = c.id;
    epoll_ctl(ep_, EPOLL_CTL_MOD, c.fd, &e);
  }

  void accept_all() {
    for (;;) {
      const int fd = accept4(lfd_, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;  // EAGAIN (or a transient error: the next readiness retries)
      const int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      auto c = std::make_unique<Conn>();
      c->id = next_id_++;
      c->fd = fd;
      // our SETTINGS + the connection window grant (the client's preface comes first on
      // the wire from its side; ours may be sent immediately)
      std::string& o = c->out;
      put_frame_header(&o, 24, kSettings, 0, 0);
      o.append("\x00\x03", 2);
      put_u32(&o, cfg_.max_concurrent_streams);
      o.append("\x00\x04", 2);
      put_u32(&o, uint32_t(kOurStreamWindow));
      o.append("\x00\x05", 2);
      put_u32(&o, kOurMaxFrame);
      o.append("\x00\x06", 2);
      put_u32(&o, kMaxHeaderList);
      put_frame_header(&o, 4, kWindowUpdate, 0, 0);
      put_u32(&o, uint32_t(kOurConnWindow - 65535));
      const uint64_t id = c->id;
      add(fd, id, EPOLLIN);
      Conn& cr = *c;
      conns_.emplace(id, std::move(c));
      {
        std::lock_guard<std::mutex> lk(q_mu_);
        ++st_.connections;
        ++st_.open_connections;
      }
      flush(cr);
    }
  }

  void close_conn(uint64_t id) {
    auto it = conns_.find(id);
    if (it == conns_.end()) return;
    epoll_ctl(ep_, EPOLL_CTL_DEL, it->second->fd, nullptr);
    ::close(it->second->fd);
    conns_.erase(it);
    std::lock_guard<std::mutex> lk(q_mu_);
    --st_.open_connections;
  }

  void flush(Conn& c) {
    while (c.out_off < c.out.size()) {
      const ssize_t w = ::send(c.fd, c.out.data() + c.out_off, c.out.size() - c.out_off, MSG_NOSIGNAL);
      if (w < 0) {
        if (errno == EAGAIN || errno == EWOULDBLOCK) break;
        if (errno == EINTR) continue;
        c.dead = true;
        return;
      }
      c.out_off += size_t(w);
      bytes_out_ += w;
    }
    if (c.out_off == c.out.size()) {
      c.out.clear();
      c.out_off = 0;
      set_write_interest(c, false);
    } else {
      if (c.out_off > (1 << 20)) {
        c.out.erase(0, c.out_off);
        c.out_off = 0;
      }
      set_write_interest(c, true);
    }
    // Every flush, from whichever call site (readiness, drain_replies, goaway):
    // a closing connection sends its FIN once the GOAWAY is out, and a
    // connection whose reads were paused resumes once the reader caught up.
    // Resuming only from the EPOLLOUT branch hung a connection whose backlog
    // drained inside drain_replies (no EPOLLIN, no EPOLLOUT interest left).
    if (c.closing) {
      shut_when_flushed(c);
    } else if (c.read_paused && c.backlog() <= kMaxOutBacklog / 2) {
      c.read_paused = false;
      update_events(c);
      resume_.push_back(c.id);  // frames already buffered: processed by resume_paused()
    }
  }

  // Connections whose reads resumed: parse the frames they buffered while
  // paused (outside flush(), which process() paths call).
  void resume_paused() {
    while (!resume_.empty()) {
      std::vector<uint64_t> ids;
      ids.swap(resume_);
      for (uint64_t id : ids) {
        auto it = conns_.find(id);
        if (it == conns_.end()) continue;
        Conn& c = *it->second;
        if (c.dead || c.closing || c.read_paused) continue;
        process(c);
        if (!c.dead && !c.out.empty()) flush(c);
        if (c.dead) close_conn(id);
      }
    }
  }

  void goaway(Conn& c, uint32_t code, const std::string& why) {
    put_frame_header(&c.out, uint32_t(8 + why.size()), kGoaway, 0, 0);
    put_u32(&c.out, c.last_sid);
    put_u32(&c.out, code);
    c.out.append(why);
    c.closing = true;
    c.close_by = std::chrono::steady_clock::now() + std::chrono::seconds(2);
    closing_.push_back(c.id);
    c.streams.clear();  // replies still in the handler are dropped
    c.blocked.clear();
    if (c.read_paused) {
      c.read_paused = false;
      update_events(c);
    }
    flush(c);
    if (!c.dead) shut_when_flushed(c);
    std::lock_guard<std::mutex> lk(q_mu_);
    ++st_.protocol_errors;
  }

  void shut_when_flushed(Conn& c) {
    if (!c.shut_wr && c.out_off == c.out.size()) {
      ::shutdown(c.fd, SHUT_WR);
      c.shut_wr = true;
    }
  }

  void discard_input(Conn& c) {
    char buf[16384];
    for (;;) {
      const ssize_t r = ::recv(c.fd, buf, sizeof(buf), 0);
      if (r > 0) continue;
      if (r < 0 && errno == EINTR) continue;
      if (r == 0 || (errno != EAGAIN && errno != EWOULDBLOCK)) c.dead = true;
      return;
    }
  }

  // Lingering closes past their deadline (only the connections in closing_,
  // not every connection on every loop iteration).
  void reap_closing() {
    if (closing_.empty()) return;
    const auto now = std::chrono::steady_clock::now();
    size_t keep = 0;
    for (uint64_t id : closing_) {
      auto it = conns_.find(id);
      if (it == conns_.end()) continue;  // closed already
      if (now >= it->second->close_by) {
        close_conn(id);
      } else {
        closing_[keep++] = id;
      }
    }
    closing_.resize(keep);
  }

  void rst(Conn& c, uint32_t sid, uint32_t code) {
    put_frame_header(&c.out, 4, kRstStream, 0, sid);
    put_u32(&c.out, code);
    c.streams.erase(sid);
  }

  void on_readable(Conn& c) {
    char buf[65536];
    for (;;) {
      const ssize_t r = ::recv(c.fd, buf, sizeof(buf), 0);
      if (r > 0) {
        c.in.append(buf, size_t(r));
        bytes_in_ += r;
        continue;
      }
      if (r == 0) {
        c.dead = true;  // peer closed
        break;
      }
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      if (errno == EINTR) continue;
      c.dead = true;
      break;
    }
    process(c);
    if (c.in_off == c.in.size()) {
      c.in.clear();
      c.in_off = 0;
    } else if (c.in_off > (1 << 20)) {
      c.in.erase(0, c.in_off);
      c.in_off = 0;
    }
    if (!c.out.empty()) flush(c);
  }

  void process(Conn& c) {
    while (!c.dead && !c.closing) {
      if (c.backlog() > kMaxOutBacklog) {  // stalled reader: stop consuming its frames
        if (!c.read_paused) {
          c.read_paused = true;
          update_events(c);
          std::lock_guard<std::mutex> lk(q_mu_);
          ++st_.paused_reads;
        }
        return;
      }
      const size_t avail = c.in.size() - c.in_off;
      const uint8_t* p = reinterpret_cast<const uint8_t*>(c.in.data()) + c.in_off;
      if (!c.preface) {
        if (avail < 24) return;
        if (std::memcmp(p, kPreface, 24) != 0) return goaway(c, kProtocolError, "bad connection preface");
        c.in_off += 24;
        c.preface = true;
        continue;
      }
      if (avail < 9) return;
      const uint32_t len = (uint32_t(p[0]) << 16) | (uint32_t(p[1]) << 8) | p[2];
      const uint8_t type = p[3], flags = p[4];
      const uint32_t sid = be32(p + 5) & 0x7fffffffu;
      if (len > kOurMaxFrame) return goaway(c, kFrameSizeError, "frame larger than SETTINGS_MAX_FRAME_SIZE");
      if (avail < 9 + size_t(len)) return;
      c.in_off += 9 + len;
      const uint8_t* pl = p + 9;
      if (c.block_sid && type != kContinuation) return goaway(c, kProtocolError, "CONTINUATION expected");
      switch (type) {
        case kData:
          on_data(c, sid, flags, pl, len);
          break;
        case kHeaders:
          on_headers(c, sid, flags, pl, len);
          break;
        case kContinuation:
          if (!c.block_sid || sid != c.block_sid) return goaway(c, kProtocolError, "unexpected CONTINUATION");
          if (c.block.size() + len > kMaxHeaderList) return goaway(c, kEnhanceYourCalm, "header block too large");
          c.block.append(reinterpret_cast<const char*>(pl), len);
          if (flags & kEndHeaders) end_block(c);
          break;
        case kSettings:
          on_settings(c, sid, flags, pl, len);
          break;
        case kPing:
          if (sid != 0 || len != 8) return goaway(c, kProtocolError, "bad PING");
          if (!(flags & kAck)) {
            put_frame_header(&c.out, 8, kPing, kAck, 0);
            c.out.append(reinterpret_cast<const char*>(pl), 8);
          }
          break;
        case kWindowUpdate:
          on_window_update(c, sid, pl, len);
          break;
        case kRstStream:
          if (sid == 0 || len != 4) return goaway(c, kProtocolError, "bad RST_STREAM");
          if (c.streams.erase(sid)) {
            std::lock_guard<std::mutex> lk(q_mu_);
            ++st_.resets;
          }
          break;
        case kGoaway:
          c.peer_goaway = true;
          break;
        case kPushPromise:
          return goaway(c, kProtocolError, "PUSH_PROMISE from a client");
        default:  // PRIORITY and unknown types are ignored (RFC 7540 4.1, 5.5)
          break;
      }
    }
  }

  void on_settings(Conn& c, uint32_t sid, uint8_t flags, const uint8_t* pl, uint32_t len) {
    if (sid != 0) return goaway(c, kProtocolError, "SETTINGS on a stream");
    if (flags & kAck) {
      if (len != 0) goaway(c, kFrameSizeError, "SETTINGS ACK with payload");
      return;
    }
    if (len % 6) return goaway(c, kFrameSizeError, "SETTINGS length");
    for (uint32_t i = 0; i < len; i += 6) {
      const uint16_t id = uint16_t((pl[i] << 8) | pl[i + 1]);
      const uint32_t v = be32(pl + i + 2);
      if (id == 4) {  // INITIAL_WINDOW_SIZE: applies to every open stream's send window (6.9.2)
        if (int64_t(v) > kMaxWindow) return goaway(c, kFlowControlError, "INITIAL_WINDOW_SIZE too large");
        const int64_t delta = int64_t(v) - c.peer_initial;
        c.peer_initial = v;
        for (auto& kv : c.streams) kv.second.send_window += delta;
      } else if (id == 5) {
        if (v < 16384 || v > 16777215) return goaway(c, kProtocolError, "MAX_FRAME_SIZE out of range");
        c.peer_max_frame = v;
      }
      // HEADER_TABLE_SIZE: the server's encoder never indexes; ENABLE_PUSH,
      // MAX_CONCURRENT_STREAMS, MAX_HEADER_LIST_SIZE: nothing to do for a server
    }
    put_frame_header(&c.out, 0, kSettings, kAck, 0);
    flush_blocked(c);
  }

  void on_window_update(Conn& c, uint32_t sid, const uint8_t* pl, uint32_t len) {
    if (len != 4) return goaway(c, kFrameSizeError, "WINDOW_UPDATE length");
    const uint32_t inc = be32(pl) & 0x7fffffffu;
    if (sid == 0) {
      if (inc == 0) return goaway(c, kProtocolError, "zero connection WINDOW_UPDATE");
      c.send_window += inc;
      if (c.send_window > kMaxWindow) return goaway(c, kFlowControlError, "connection window overflow");
      flush_blocked(c);
      return;
    }
    auto it = c.streams.find(sid);
    if (it == c.streams.end()) return;  // closed stream: ignore
    if (inc == 0) return rst(c, sid, kProtocolError);
    it->second.send_window += inc;
    if (it->second.send_window > kMaxWindow) return rst(c, sid, kFlowControlError);
    if (it->second.replying) send_pending(c, it->second);
  }

  void on_headers(Conn& c, uint32_t sid, uint8_t flags, const uint8_t* pl, uint32_t len) {
    if (sid == 0 || (sid & 1) == 0) return goaway(c, kProtocolError, "HEADERS on an invalid stream id");
    uint32_t off = 0, pad = 0;
    if (flags & kPadded) {
      if (len < 1) return goaway(c, kProtocolError, "HEADERS padding");
      pad = pl[0];
      off = 1;
    }
    if (flags & kPrioFlag) off += 5;
    if (off + pad > len) return goaway(c, kProtocolError, "HEADERS padding exceeds the frame");
    if (len - off - pad > kMaxHeaderList) return goaway(c, kEnhanceYourCalm, "header block too large");
    c.block_sid = sid;
    c.block_end_stream = (flags & kEndStream) != 0;
    c.block.assign(reinterpret_cast<const char*>(pl + off), len - off - pad);
    if (flags & kEndHeaders) end_block(c);
  }

  // A complete header block: always decoded (HPACK state is per connection),
  // then applied to its stream - new (request headers) or open (trailers).
  void end_block(Conn& c) {
    const uint32_t sid = c.block_sid;
    const bool es = c.block_end_stream;
    c.block_sid = 0;
    std::vector<Header> hs;
    std::string err;
    if (!c.hpack.decode(reinterpret_cast<const uint8_t*>(c.block.data()), c.block.size(), &hs, &err,
                        kMaxHeaderList))
      return goaway(c, err.rfind("header list", 0) == 0 ? kEnhanceYourCalm : kCompressionError, "HPACK: " + err);
    c.block.clear();
    auto it = c.streams.find(sid);
    if (it == c.streams.end()) {
      if (sid <= c.last_sid) return;  // a stream we reset / finished: headers ignored (5.1)
      c.last_sid = sid;
      if (c.peer_goaway || c.streams.size() >= cfg_.max_concurrent_streams) {
        put_frame_header(&c.out, 4, kRstStream, 0, sid);
        put_u32(&c.out, kRefusedStream);
        return;
      }
      Stream s;
      s.id = sid;
      s.send_window = c.peer_initial;
      for (auto& h : hs) {
        if (h.first == ":path") s.path = std::move(h.second);
        else if (h.first == ":method") s.method = std::move(h.second);
        else if (h.first == "content-type") s.content_type = std::move(h.second);
        else if (h.first == "grpc-encoding") s.encoding = std::move(h.second);
        else if (h.first == "grpc-timeout") {
          const int64_t us = parse_grpc_timeout(h.second);
          if (us >= 0) s.deadline_us = runtime::now_us() + us;
        }
      }
      s.headers_done = true;
      it = c.streams.emplace(sid, std::move(s)).first;
    } else if (it->second.dispatched) {
      return rst(c, sid, kStreamClosed);  // nothing may follow the end of the request
    } else if (!es) {
      return rst(c, sid, kProtocolError);  // trailers must end the stream
    }
    if (es) end_stream(c, it->second);
  }

  void on_data(Conn& c, uint32_t sid, uint8_t flags, const uint8_t* pl, uint32_t len) {
    if (sid == 0) return goaway(c, kProtocolError, "DATA on stream 0");
    // flow control counts the whole payload, padding included (6.9.1)
    c.recv_unacked += len;
    if (c.recv_unacked >= kOurConnWindow / 2) {
      put_frame_header(&c.out, 4, kWindowUpdate, 0, 0);
      put_u32(&c.out, uint32_t(c.recv_unacked));
      c.recv_unacked = 0;
    }
    auto it = c.streams.find(sid);
    if (it == c.streams.end()) {
      if (sid > c.last_sid) return goaway(c, kProtocolError, "DATA on an idle stream");
      return;  // reset / closed: discard
    }
    Stream& s = it->second;
    if (s.dispatched) return rst(c, sid, kStreamClosed);
    uint32_t off = 0, pad = 0;
    if (flags & kPadded) {
      if (len < 1) return goaway(c, kProtocolError, "DATA padding");
      pad = pl[0];
      off = 1;
    }
    if (off + pad > len) return goaway(c, kProtocolError, "DATA padding exceeds the frame");
    const uint32_t n = len - off - pad;
    if (!s.too_big) {
      if (int64_t(s.body.size()) + n > cfg_.max_message + 5) {
        s.too_big = true;
        s.body.clear();
        s.body.shrink_to_fit();
      } else {
        s.body.append(reinterpret_cast<const char*>(pl + off), n);
      }
    }
    if (flags & kEndStream) return end_stream(c, s);
    s.recv_unacked += len;
    if (s.recv_unacked >= kOurStreamWindow / 2) {
      put_frame_header(&c.out, 4, kWindowUpdate, 0, sid);
      put_u32(&c.out, uint32_t(s.recv_unacked));
      s.recv_unacked = 0;
    }
  }

  // The client half-closed: validate, strip the gRPC message prefix, dispatch.
  void end_stream(Conn& c, Stream& s) {
    s.dispatched = true;
    Responder rsp(shared_from_this(), c.id, s.id);
    {
      std::lock_guard<std::mutex> lk(q_mu_);
      ++st_.calls;
    }
    if (s.method != "POST" || s.content_type.compare(0, 16, "application/grpc") != 0)
      return rsp.reply(13, "not a gRPC request (method " + s.method + ", content-type " + s.content_type + ")", "");
    if (s.too_big)
      return rsp.reply(8, "request message larger than " + std::to_string(cfg_.max_message) + " bytes", "");
    if (s.body.size() < 5) return rsp.reply(13, "request carries no gRPC message", "");
    const uint8_t* b = reinterpret_cast<const uint8_t*>(s.body.data());
    const uint32_t mlen = be32(b + 1);
    if (b[0] != 0)
      return rsp.reply(12, "compressed messages (grpc-encoding " + s.encoding + ") are not supported", "");
    if (size_t(mlen) + 5 != s.body.size()) return rsp.reply(13, "a unary call carries exactly one message", "");
    GrpcCall call;
    call.path = std::move(s.path);
    call.deadline_us = s.deadline_us;
    call.message.assign(s.body, 5, mlen);
    std::string().swap(s.body);
    (*handler_)(std::move(call), std::move(rsp));
  }

  void drain_replies() {
    std::vector<Posted> q;
    {
      std::lock_guard<std::mutex> lk(q_mu_);
      q.swap(q_);
    }
    std::vector<uint64_t> touched;
    for (auto& r : q) {
      auto it = conns_.find(r.conn);
      Stream* s = nullptr;
      if (it != conns_.end()) {
        auto si = it->second->streams.find(r.stream);
        if (si != it->second->streams.end() && !si->second.replying) s = &si->second;
      }
      if (!s) {
        std::lock_guard<std::mutex> lk(q_mu_);
        ++st_.dropped_replies;
        continue;
      }
      Conn& c = *it->second;
      write_reply(c, *s, r);
      touched.push_back(r.conn);
    }
    for (uint64_t id : touched) {
      auto it = conns_.find(id);
      if (it == conns_.end()) continue;
      flush(*it->second);
      if (it->second->dead) close_conn(id);
    }
    std::lock_guard<std::mutex> lk(q_mu_);
    st_.bytes_in = bytes_in_;
    st_.bytes_out = bytes_out_;
  }

  void write_reply(Conn& c, Stream& s, Posted& r) {
    {
      std::lock_guard<std::mutex> lk(q_mu_);
      ++st_.replies;
    }
    std::string hb;
    hpack_put_indexed(&hb, 8);                                     // :status 200
    hpack_put_literal(&hb, "", "application/grpc", 31);            // content-type
    if (r.status != 0) {  // trailers-only reply
      hpack_put_literal(&hb, "grpc-status", std::to_string(r.status));
      if (!r.message.empty()) hpack_put_literal(&hb, "grpc-message", grpc_percent_encode(r.message));
      put_headers(c, s.id, hb, true);
      c.streams.erase(s.id);
      return;
    }
    put_headers(c, s.id, hb, false);
    s.pending.clear();
    s.pending.reserve(5 + r.body.size());
    s.pending.push_back('\0');
    const uint32_t n = uint32_t(r.body.size());
    const char pfx[4] = {char(n >> 24), char(n >> 16), char(n >> 8), char(n)};
    s.pending.append(pfx, 4);
    s.pending.append(r.body);
    s.pending_off = 0;
    s.trailers.clear();
    hpack_put_literal(&s.trailers, "grpc-status", "0");
    s.replying = true;
    send_pending(c, s);
  }

  void put_headers(Conn& c, uint32_t sid, const std::string& block, bool end_stream) {
    // a reply header block is far below any MAX_FRAME_SIZE: one HEADERS frame
    put_frame_header(&c.out, uint32_t(block.size()), kHeaders, uint8_t(kEndHeaders | (end_stream ? kEndStream : 0)),
                     sid);
    c.out.append(block);
  }

  // DATA as the windows allow, then the trailers (END_STREAM); a stream that
  // runs out of window waits in c.blocked for a WINDOW_UPDATE / SETTINGS.
  void send_pending(Conn& c, Stream& s) {
    while (s.pending_off < s.pending.size()) {
      const int64_t left = int64_t(s.pending.size() - s.pending_off);
      const int64_t n = std::min<int64_t>({left, int64_t(c.peer_max_frame), c.send_window, s.send_window});
      if (n <= 0) {
        c.blocked.push_back(s.id);
        return;
      }
      put_frame_header(&c.out, uint32_t(n), kData, 0, s.id);
      c.out.append(s.pending, s.pending_off, size_t(n));
      s.pending_off += size_t(n);
      c.send_window -= n;
      s.send_window -= n;
    }
    put_headers(c, s.id, s.trailers, true);
    c.streams.erase(s.id);  // s is gone
  }

  void flush_blocked(Conn& c) {
    std::deque<uint32_t> b;
    b.swap(c.blocked);
    for (uint32_t sid : b) {
      auto it = c.streams.find(sid);
      if (it != c.streams.end() && it->second.replying) send_pending(c, it->second);
    }
  }

  const H2Config cfg_;
  const GrpcHandler* handler_;
  int lfd_, ep_ = -1, efd_ = -1;
  uint64_t next_id_;
  std::unordered_map<uint64_t, std::unique_ptr<Conn>> conns_;
  std::vector<uint64_t> resume_;   // reads resumed in flush(): buffered frames to process
  std::vector<uint64_t> closing_;  // lingering closes (GOAWAY sent), reaped at close_by
  mutable std::mutex q_mu_;
  std::vector<Posted> q_;
  bool stop_ = false;
  H2Stats st_;
  int64_t bytes_in_ = 0, bytes_out_ = 0;
};

void Responder::reply(int status, std::string message, std::string body) const {
  if (!loop_) return;
  loop_->post(Posted{conn_, stream_, status, std::move(message), std::move(body)});
}

namespace {

int listen_socket(const std::string& host, int port) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_flags = AI_PASSIVE | AI_NUMERICSERV;
  const std::string ps = std::to_string(port);
  if (getaddrinfo(host.empty() ? nullptr : host.c_str(), ps.c_str(), &hints, &res) != 0 || !res)
    throw std::runtime_error("cannot resolve " + host);
  int fd = -1;
  for (addrinfo* a = res; a; a = a->ai_next) {
    fd = ::socket(a->ai_family, a->ai_socktype | SOCK_NONBLOCK | SOCK_CLOEXEC, a->ai_protocol);
    if (fd < 0) continue;
    const int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof(one));
    if (::bind(fd, a->ai_addr, a->ai_addrlen) == 0 && ::listen(fd, 1024) == 0) break;
    ::close(fd);
    fd = -1;
  }
  freeaddrinfo(res);
  if (fd < 0) throw std::runtime_error("cannot listen on " + host + ":" + std::to_string(port) + ": " +
                                       std::strerror(errno));
  return fd;
}

int bound_port(int fd) {
  sockaddr_storage ss{};
  socklen_t l = sizeof(ss);
  getsockname(fd, reinterpret_cast<sockaddr*>(&ss), &l);
  if (ss.ss_family == AF_INET6) return ntohs(reinterpret_cast<sockaddr_in6*>(&ss)->sin6_port);
  return ntohs(reinterpret_cast<sockaddr_in*>(&ss)->sin_port);
}

}  // namespace

H2GrpcServer::H2GrpcServer(H2Config cfg, GrpcHandler handler)
    : cfg_(std::move(cfg)), handler_(new GrpcHandler(std::move(handler))) {
  const GrpcHandler* h = handler_.get();
  const int n = std::max(1, cfg_.threads);
  std::vector<int> fds;
  try {
    fds.push_back(listen_socket(cfg_.host, cfg_.port));
    port_ = bound_port(fds[0]);
    for (int i = 1; i < n; ++i) fds.push_back(listen_socket(cfg_.host, port_));
  } catch (...) {
    for (int fd : fds) ::close(fd);
    throw;
  }
  for (int i = 0; i < n; ++i) loops_.push_back(std::make_shared<Loop>(cfg_, h, fds[size_t(i)], i));
  for (auto& l : loops_) threads_.emplace_back([l] { l->run(); });
}

H2GrpcServer::~H2GrpcServer() { stop(); }

void H2GrpcServer::stop() {
  if (stopped_.exchange(true)) return;
  for (auto& l : loops_) l->stop();
  for (auto& t : threads_) t.join();
  threads_.clear();
  // the loops may outlive this object (Responders hold them) but no longer
  // call the handler
}

H2Stats H2GrpcServer::stats() const {
  H2Stats s;
  for (auto& l : loops_) {
    const H2Stats x = l->stats();
    s.connections += x.connections;
    s.open_connections += x.open_connections;
    s.calls += x.calls;
    s.replies += x.replies;
    s.dropped_replies += x.dropped_replies;
    s.resets += x.resets;
    s.protocol_errors += x.protocol_errors;
    s.paused_reads += x.paused_reads;
    s.bytes_in += x.bytes_in;
    s.bytes_out += x.bytes_out;
  }
  return s;
}

int64_t parse_grpc_timeout(const std::string& v) {
  if (v.size() < 2 || v.size() > 9) return -1;
  int64_t n = 0;
  for (size_t i = 0; i + 1 < v.size(); ++i) {
    if (v[i] < '0' || v[i] > '9') return -1;
    n = n * 10 + (v[i] - '0');
  }
  switch (v.back()) {
    case 'H': return n * 3600LL * 1000000LL;
    case 'M': return n * 60LL * 1000000LL;
    case 'S': return n * 1000000LL;
    case 'm': return n * 1000LL;
    case 'u': return n;
    case 'n': return (n + 999) / 1000;
    default: return -1;
  }
}

std::string grpc_percent_encode(const std::string& s) {
  static const char* hex = "0123456789ABCDEF";
  std::string o;
  for (unsigned char c : s) {
    if (c >= 0x20 && c <= 0x7e && c != '%') {
      o.push_back(char(c));
    } else {
      o.push_back('%');
      o.push_back(hex[c >> 4]);
      o.push_back(hex[c & 15]);
    }
  }
  return o;
}

}  // namespace net
}  // namespace dtfs
