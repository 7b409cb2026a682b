// Native gRPC front door: HTTP/2 over cleartext TCP (h2c, prior knowledge -
// what gRPC clients speak on an insecure channel) on epoll threads, unary
// calls only.
//
// The reference's whole transport is one gRPC-java channel per host, a
// blocking unary Predict per shard (reference DCNClient.java:111-112,
// :118-125; pom.xml:83-92). Here the server side of that call runs without
// Python: each event-loop thread owns its connections (SO_REUSEPORT listeners,
// the kernel spreads connections), parses frames, decodes HPACK, reassembles
// the request message and hands it to a handler - for Predict the live
// server's submit(), which copies the bytes into the pinned request arena. The
// handler answers from any thread (the live server's completer) through a
// Responder; the loop that owns the connection encodes and writes the reply.
//
// HTTP/2 coverage: connection preface, SETTINGS (+ACK, initial window,
// max frame size, header table size), HEADERS + CONTINUATION (padding,
// priority), DATA (padding), connection- and stream-level flow control in both
// directions (WINDOW_UPDATE), PING (+ACK), RST_STREAM (cancellation), GOAWAY
// (graceful close both ways), PRIORITY (ignored). gRPC: length-prefixed
// messages (uncompressed; a compressed one gets UNIMPLEMENTED), grpc-timeout
// deadlines, trailers with grpc-status / percent-encoded grpc-message,
// trailers-only error replies.
#pragma once

#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace dtfs {
namespace net {

struct GrpcCall {
  std::string path;         // "/package.Service/Method"
  std::string message;      // the request message (after the 5-byte gRPC prefix)
  int64_t deadline_us = 0;  // absolute runtime::now_us() from grpc-timeout, 0 = none
};

class Loop;

// Answers one call exactly once, from any thread; a reply for a connection or
// stream that is gone (closed, reset by the client, server stopped) is dropped.
class Responder {
 public:
  Responder() = default;
  Responder(std::shared_ptr<Loop> loop, uint64_t conn, uint32_t stream)
      : loop_(std::move(loop)), conn_(conn), stream_(stream) {}
  // status 0: `body` is the response message; else a gRPC status code + message
  void reply(int status, std::string message, std::string body) const;

 private:
  std::shared_ptr<Loop> loop_;
  uint64_t conn_ = 0;
  uint32_t stream_ = 0;
};

using GrpcHandler = std::function<void(GrpcCall&&, Responder)>;

struct H2Config {
  std::string host = "0.0.0.0";
  int port = 0;                      // 0: any free port (see H2GrpcServer::port)
  int threads = 4;                   // event-loop threads
  int64_t max_message = 64 << 20;    // larger requests: RESOURCE_EXHAUSTED
  uint32_t max_concurrent_streams = 1024;
};

struct H2Stats {
  int64_t connections = 0, open_connections = 0, calls = 0, replies = 0, dropped_replies = 0;
  int64_t resets = 0, protocol_errors = 0, bytes_in = 0, bytes_out = 0;
  int64_t paused_reads = 0;  // connections whose input was paused behind an unread reply backlog
};

class H2GrpcServer {
 public:
  H2GrpcServer(H2Config cfg, GrpcHandler handler);
  ~H2GrpcServer();
  H2GrpcServer(const H2GrpcServer&) = delete;
  H2GrpcServer& operator=(const H2GrpcServer&) = delete;

  int port() const { return port_; }
  // Stop accepting, GOAWAY every connection, join the loops. Replies that
  // arrive later are dropped.
  void stop();
  H2Stats stats() const;

 private:
  H2Config cfg_;
  std::unique_ptr<GrpcHandler> handler_;  // the loops call it until stop()
  int port_ = 0;
  std::vector<std::shared_ptr<Loop>> loops_;
  std::vector<std::thread> threads_;
  std::atomic<bool> stopped_{false};
};

// "1S" / "250m" / "100u" ... -> microseconds (grpc-timeout grammar); -1 = invalid.
int64_t parse_grpc_timeout(const std::string& v);
// grpc-message percent-encoding (the gRPC HTTP/2 spec).
std::string grpc_percent_encode(const std::string& s);

}  // namespace net
}  // namespace dtfs
