#include "net/h2_client.h"

#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <thread>

#include "net/h2_server.h"    // parse_grpc_timeout (shared grammar)
#include "runtime/batcher.h"  // now_us()

namespace dtfs {
namespace net {

namespace {

enum : uint8_t { kData = 0, kHeaders = 1, kRstStream = 3, kSettings = 4, kPing = 6, kGoaway = 7, kWindowUpdate = 8,
                 kContinuation = 9 };
enum : uint8_t { kEndStream = 0x1, kAck = 0x1, kEndHeaders = 0x4, kPadded = 0x8, kPrioFlag = 0x20 };
const char kPreface[] = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n";
constexpr int64_t kRecvWindow = 16 << 20;

void frame_header(std::string* out, uint32_t len, uint8_t type, uint8_t flags, uint32_t sid) {
  const char h[9] = {char(len >> 16), char(len >> 8), char(len), char(type), char(flags),
                     char((sid >> 24) & 0x7f), char(sid >> 16), char(sid >> 8), char(sid)};
  out->append(h, 9);
}
void u32(std::string* out, uint32_t v) {
  const char b[4] = {char(v >> 24), char(v >> 16), char(v >> 8), char(v)};
  out->append(b, 4);
}
uint32_t be32(const uint8_t* p) { return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3]; }

std::string timeout_value(int64_t us) {
  if (us <= 0) return "";
  if (us < 100000000) return std::to_string(us) + "u";
  return std::to_string(us / 1000) + "m";
}

int percent_hex(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  return -1;
}

std::string percent_decode(const std::string& s) {
  std::string o;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size() + 0 && percent_hex(s[i + 1]) >= 0 && percent_hex(s[i + 2]) >= 0) {
      o.push_back(char(percent_hex(s[i + 1]) * 16 + percent_hex(s[i + 2])));
      i += 2;
    } else {
      o.push_back(s[i]);
    }
  }
  return o;
}

}  // namespace

H2Client::H2Client(const std::string& host, int port, int64_t connect_timeout_us) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  const std::string ps = std::to_string(port);
  if (getaddrinfo(host.c_str(), ps.c_str(), &hints, &res) != 0 || !res)
    throw std::runtime_error("cannot resolve " + host);
  for (addrinfo* a = res; a && fd_ < 0; a = a->ai_next) {
    fd_ = ::socket(a->ai_family, a->ai_socktype | SOCK_CLOEXEC, a->ai_protocol);
    if (fd_ < 0) continue;
    timeval tv{long(connect_timeout_us / 1000000), long(connect_timeout_us % 1000000)};
    setsockopt(fd_, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
    if (::connect(fd_, a->ai_addr, a->ai_addrlen) != 0) {
      ::close(fd_);
      fd_ = -1;
    }
  }
  freeaddrinfo(res);
  if (fd_ < 0) throw std::runtime_error("cannot connect to " + host + ":" + ps);
  const int one = 1;
  setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  authority_ = host + ":" + ps;
  std::string o(kPreface, 24);
  frame_header(&o, 12, kSettings, 0, 0);
  o.append("\x00\x02", 2);  // ENABLE_PUSH 0
  u32(&o, 0);
  o.append("\x00\x04", 2);  // INITIAL_WINDOW_SIZE
  u32(&o, uint32_t(kRecvWindow));
  frame_header(&o, 4, kWindowUpdate, 0, 0);
  u32(&o, uint32_t(kRecvWindow - 65535));
  std::string err;
  if (!send_all(o, &err)) throw std::runtime_error("h2 client: " + err);
  // the server's SETTINGS come first on its side: read until they are in
  for (;;) {
    uint8_t type, flags;
    uint32_t sid;
    std::string pl;
    if (!read_frame(&type, &flags, &sid, &pl, &err)) throw std::runtime_error("h2 client: " + err);
    if (!handle_control(type, flags, sid, pl, &err)) throw std::runtime_error("h2 client: " + err);
    if (type == kSettings && !(flags & kAck)) break;
  }
}

H2Client::~H2Client() {
  if (fd_ >= 0) {
    std::string g;
    frame_header(&g, 8, kGoaway, 0, 0);
    u32(&g, 0);
    u32(&g, 0);
    std::string err;
    send_all(g, &err);
    ::close(fd_);
  }
}

bool H2Client::send_all(const std::string& b, std::string* err) {
  size_t off = 0;
  while (off < b.size()) {
    const ssize_t w = ::send(fd_, b.data() + off, b.size() - off, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      *err = std::string("send: ") + std::strerror(errno);
      return false;
    }
    off += size_t(w);
  }
  return true;
}

bool H2Client::read_frame(uint8_t* type, uint8_t* flags, uint32_t* sid, std::string* payload, std::string* err) {
  auto need = [&](size_t n) {
    while (rbuf_.size() - roff_ < n) {
      if (roff_ > 0 && roff_ == rbuf_.size()) {
        rbuf_.clear();
        roff_ = 0;
      }
      char buf[65536];
      const ssize_t r = ::recv(fd_, buf, sizeof(buf), 0);
      if (r > 0) {
        rbuf_.append(buf, size_t(r));
      } else if (r == 0) {
        *err = "connection closed by the server";
        return false;
      } else if (errno != EINTR) {
        *err = std::string("recv: ") + std::strerror(errno);
        return false;
      }
    }
    return true;
  };
  if (!need(9)) return false;
  const uint8_t* p = reinterpret_cast<const uint8_t*>(rbuf_.data()) + roff_;
  const uint32_t len = (uint32_t(p[0]) << 16) | (uint32_t(p[1]) << 8) | p[2];
  *type = p[3];
  *flags = p[4];
  *sid = be32(p + 5) & 0x7fffffffu;
  if (!need(9 + size_t(len))) return false;
  payload->assign(rbuf_, roff_ + 9, len);
  roff_ += 9 + len;
  if (roff_ > (1 << 20)) {
    rbuf_.erase(0, roff_);
    roff_ = 0;
  }
  return true;
}

bool H2Client::handle_control(uint8_t type, uint8_t flags, uint32_t sid, const std::string& pl, std::string* err) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(pl.data());
  if (type == kSettings && !(flags & kAck)) {
    for (size_t i = 0; i + 6 <= pl.size(); i += 6) {
      const uint16_t id = uint16_t((p[i] << 8) | p[i + 1]);
      const uint32_t v = be32(p + i + 2);
      if (id == 4) {
        stream_window_ += int64_t(v) - peer_initial_;
        peer_initial_ = v;
      } else if (id == 5) {
        peer_max_frame_ = v;
      }
    }
    std::string a;
    frame_header(&a, 0, kSettings, kAck, 0);
    return send_all(a, err);
  }
  if (type == kPing && !(flags & kAck)) {
    std::string a;
    frame_header(&a, 8, kPing, kAck, 0);
    a.append(pl);
    return send_all(a, err);
  }
  if (type == kWindowUpdate && pl.size() == 4) {
    const uint32_t inc = be32(p) & 0x7fffffffu;
    if (sid == 0) send_conn_window_ += inc;
    else if (sid == next_sid_ - 2) stream_window_ += inc;  // the call in progress
    return true;
  }
  if (type == kGoaway) {
    *err = "server sent GOAWAY";
    return false;
  }
  return true;
}

bool H2Client::call(const std::string& path, const std::string& request, int64_t timeout_us, int* status,
                    std::string* message, std::string* body) {
  const uint32_t sid = next_sid_;
  next_sid_ += 2;
  stream_window_ = peer_initial_;
  std::string o, hb;
  hpack_put_indexed(&hb, 3);                                  // :method POST
  hpack_put_indexed(&hb, 6);                                  // :scheme http
  hpack_put_literal(&hb, "", path, 4);                        // :path
  hpack_put_literal(&hb, "", authority_, 1);                  // :authority
  hpack_put_literal(&hb, "", "application/grpc", 31);         // content-type
  hpack_put_literal(&hb, "te", "trailers");
  if (timeout_us > 0) hpack_put_literal(&hb, "grpc-timeout", timeout_value(timeout_us));
  frame_header(&o, uint32_t(hb.size()), kHeaders, kEndHeaders, sid);
  o.append(hb);
  std::string msg;
  msg.reserve(request.size() + 5);
  msg.push_back('\0');
  u32(&msg, uint32_t(request.size()));
  msg.append(request);
  size_t off = 0;
  std::string err;
  // request DATA under the server's windows (read control frames while blocked)
  while (off < msg.size()) {
    const int64_t n = std::min<int64_t>({int64_t(msg.size() - off), int64_t(peer_max_frame_), send_conn_window_,
                                         stream_window_});
    if (n <= 0) {
      if (!send_all(o, &err)) break;
      o.clear();
      uint8_t type, flags;
      uint32_t fsid;
      std::string pl;
      if (!read_frame(&type, &flags, &fsid, &pl, &err) || !handle_control(type, flags, fsid, pl, &err)) break;
      if (type == kRstStream && fsid == sid) {
        err = "stream reset by the server";
        break;
      }
      continue;
    }
    const bool last = off + size_t(n) == msg.size();
    frame_header(&o, uint32_t(n), kData, last ? kEndStream : 0, sid);
    o.append(msg, off, size_t(n));
    off += size_t(n);
    send_conn_window_ -= n;
    stream_window_ -= n;
  }
  if (!err.empty() || !send_all(o, &err)) {
    *message = err;
    return false;
  }
  // response: HEADERS, DATA..., trailers (or trailers-only)
  body->clear();
  std::string resp;
  *status = -1;
  message->clear();
  std::string block;
  bool in_block = false, block_end = false;
  for (;;) {
    uint8_t type, flags;
    uint32_t fsid;
    std::string pl;
    if (!read_frame(&type, &flags, &fsid, &pl, &err)) {
      *message = err;
      return false;
    }
    if (fsid != sid || (type != kHeaders && type != kData && type != kContinuation && type != kRstStream)) {
      if (!handle_control(type, flags, fsid, pl, &err)) {
        *message = err;
        return false;
      }
      continue;
    }
    if (type == kRstStream) {
      *message = "stream reset by the server";
      return false;
    }
    const uint8_t* p = reinterpret_cast<const uint8_t*>(pl.data());
    size_t off2 = 0, pad = 0;
    if ((type == kData || type == kHeaders) && (flags & kPadded)) {
      pad = p[0];
      off2 = 1;
    }
    if (type == kHeaders && (flags & kPrioFlag)) off2 += 5;
    if (off2 + pad > pl.size()) {
      *message = "bad padding";
      return false;
    }
    if (type == kData) {
      resp.append(pl, off2, pl.size() - off2 - pad);
      recv_unacked_ += int64_t(pl.size());
      if (recv_unacked_ >= kRecvWindow / 2) {  // connection window (each call is a fresh stream)
        std::string w;
        frame_header(&w, 4, kWindowUpdate, 0, 0);
        u32(&w, uint32_t(recv_unacked_));
        recv_unacked_ = 0;
        if (!send_all(w, &err)) {
          *message = err;
          return false;
        }
      }
      if (flags & kEndStream) {
        *message = "stream ended without trailers";
        return false;
      }
      continue;
    }
    if (type == kHeaders) {
      block.assign(pl, off2, pl.size() - off2 - pad);
      in_block = true;
      block_end = (flags & kEndStream) != 0;
    } else {
      if (!in_block) {
        *message = "unexpected CONTINUATION";
        return false;
      }
      block.append(pl);
    }
    if (!(flags & kEndHeaders)) continue;
    in_block = false;
    std::vector<Header> hs;
    if (!hpack_.decode(reinterpret_cast<const uint8_t*>(block.data()), block.size(), &hs, &err)) {
      *message = "HPACK: " + err;
      return false;
    }
    for (auto& h : hs) {
      if (h.first == "grpc-status") *status = std::atoi(h.second.c_str());
      else if (h.first == "grpc-message") *message = percent_decode(h.second);
    }
    if (!block_end) continue;  // response headers; DATA and trailers follow
    if (*status < 0) {
      *message = "no grpc-status in the trailers";
      return false;
    }
    if (*status == 0) {
      if (resp.size() < 5 || resp[0] != 0 || be32(reinterpret_cast<const uint8_t*>(resp.data()) + 1) + 5 != resp.size()) {
        *message = "malformed gRPC response message";
        return false;
      }
      body->assign(resp, 5, std::string::npos);
    }
    return true;
  }
}

GrpcLoadResult run_grpc_load(const std::string& host, int port, const std::string& path,
                             const std::vector<std::string>& requests, const GrpcLoadSpec& spec) {
  if (requests.empty()) throw std::invalid_argument("no requests");
  const int C = std::max(1, spec.concurrency);
  const int64_t total = spec.warmup + spec.count;
  GrpcLoadResult res;
  std::mutex mu;
  std::atomic<int64_t> next{0}, done{0};
  double t_open = 0, t_close = 0;
  const double wall0 = double(runtime::now_us());
  if (spec.warmup == 0) t_open = wall0;
  std::vector<std::thread> ts;
  for (int c = 0; c < C; ++c) {
    ts.emplace_back([&, c] {
      std::unique_ptr<H2Client> cl;
      try {
        cl = std::make_unique<H2Client>(host, port);
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> lk(mu);
        if (res.first_error.empty()) res.first_error = e.what();
        return;
      }
      for (;;) {
        const int64_t k = next.fetch_add(1);
        if (k >= total) return;
        const std::string& r = requests[size_t((k + c) % int64_t(requests.size()))];
        const int64_t t0 = runtime::now_us();
        int st = -1;
        std::string msg, body;
        const bool ok = cl->call(path, r, spec.timeout_us, &st, &msg, &body) && st == 0;
        const int64_t t1 = runtime::now_us();
        const int64_t d = done.fetch_add(1) + 1;
        std::lock_guard<std::mutex> lk(mu);
        if (ok) ++res.ok;
        else if (res.errors++ == 0) res.first_error = msg.empty() ? "grpc-status " + std::to_string(st) : msg;
        if (d == spec.warmup) t_open = double(t1);
        if (d > spec.warmup) res.latency_us.push_back(double(t1 - t0));
        if (d == total) t_close = double(t1);
        if (!ok && st < 0) {  // transport failure: a fresh connection for the next call
          try {
            cl = std::make_unique<H2Client>(host, port);
          } catch (...) {
            return;
          }
        }
      }
    });
  }
  for (auto& t : ts) t.join();
  res.wall_us = double(runtime::now_us()) - wall0;
  res.window_us = t_close > t_open ? t_close - t_open : 0;
  return res;
}

}  // namespace net
}  // namespace dtfs
