// Native gRPC unary client over h2c and a closed-loop load generator on it:
// the client side of the reference's transport (one gRPC channel per host,
// blocking unary Predict, reference DCNClient.java:111-112, :118-125) without
// a Python client in the measurement. Used to drive the native front door
// (net/h2_server.h) from another process (bench.py --reference-workload
// --over-grpc) and in tests; it speaks to any gRPC server (grpcio included).
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "net/hpack.h"

namespace dtfs {
namespace net {

class H2Client {
 public:
  H2Client(const std::string& host, int port, int64_t connect_timeout_us = 5'000'000);
  ~H2Client();
  H2Client(const H2Client&) = delete;
  H2Client& operator=(const H2Client&) = delete;

  // One unary call (this connection carries one call at a time). Returns
  // false on a transport failure (*message says why); otherwise the gRPC
  // status (0 = OK, `body` = the response message) or error + message.
  bool call(const std::string& path, const std::string& request, int64_t timeout_us, int* status,
            std::string* message, std::string* body);

 private:
  bool read_frame(uint8_t* type, uint8_t* flags, uint32_t* sid, std::string* payload, std::string* err);
  bool send_all(const std::string& b, std::string* err);
  bool handle_control(uint8_t type, uint8_t flags, uint32_t sid, const std::string& pl, std::string* err);
  int fd_ = -1;
  std::string authority_;
  uint32_t next_sid_ = 1;
  int64_t send_conn_window_ = 65535, peer_initial_ = 65535;
  int64_t stream_window_ = 0;
  uint32_t peer_max_frame_ = 16384;
  int64_t recv_unacked_ = 0;
  HpackDecoder hpack_;
  std::string rbuf_;
  size_t roff_ = 0;
};

struct GrpcLoadSpec {
  int concurrency = 6;        // client threads, one connection each, closed loop
  int64_t warmup = 0;         // calls before the timed window
  int64_t count = 1000;       // calls in the timed window
  int64_t timeout_us = 0;     // per-call deadline (grpc-timeout), 0 = none
};

struct GrpcLoadResult {
  std::vector<double> latency_us;  // timed calls, completion order
  int64_t ok = 0, errors = 0;
  double window_us = 0, wall_us = 0;
  std::string first_error;
};

GrpcLoadResult run_grpc_load(const std::string& host, int port, const std::string& path,
                             const std::vector<std::string>& requests, const GrpcLoadSpec& spec);

}  // namespace net
}  // namespace dtfs
