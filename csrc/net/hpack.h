// HPACK (RFC 7541) for the native gRPC front door: a full decoder (static
// and dynamic tables, table-size updates, Huffman-coded strings) and the small
// encoder subset the server needs for its replies (indexed static entries and
// literals without indexing - the server never adds to the client's table).
//
// Reference counterpart: the reference's transport is gRPC-java over Netty
// (reference pom.xml:83-92, DCNClient.java:111-112); the TF-Serving host it
// talks to decodes these headers in its gRPC core.
#pragma once

#include <cstdint>
#include <deque>
#include <string>
#include <utility>
#include <vector>

namespace dtfs {
namespace net {

using Header = std::pair<std::string, std::string>;

class HpackDecoder {
 public:
  // max_table: the SETTINGS_HEADER_TABLE_SIZE this endpoint advertised
  explicit HpackDecoder(size_t max_table = 4096) : limit_(max_table), max_(max_table) {}
  // Decode one complete header block (HEADERS + CONTINUATION payloads).
  // false on a compression error (a connection error: COMPRESSION_ERROR) or
  // when the decoded list outgrows max_list bytes (0 = no bound; indexed
  // references to large table entries make a small block decode to a large
  // list, so the bound is checked while decoding).
  bool decode(const uint8_t* p, size_t n, std::vector<Header>* out, std::string* err, size_t max_list = 0);
  size_t table_size() const { return size_; }
  size_t table_entries() const { return dyn_.size(); }

 private:
  bool lookup(uint64_t index, Header* h, std::string* err) const;
  void insert(Header h);
  void evict_to(size_t cap);
  std::deque<Header> dyn_;  // front = most recent (index 62)
  size_t size_ = 0;
  size_t limit_;            // current table size limit (encoder's size updates)
  size_t max_;              // the advertised maximum
};

// Huffman (Appendix B): decode `n` bytes; false on an invalid code / padding.
bool huffman_decode(const uint8_t* p, size_t n, std::string* out);
// Encoder side, for tests and the native client: the Huffman-coded bytes.
std::string huffman_encode(const std::string& s);

// Integer representation (section 5.1) with an N-bit prefix; `first` holds
// the representation's flag bits above the prefix.
void hpack_put_int(std::string* out, uint8_t first, int prefix, uint64_t v);
// Literal header field without indexing, name and value as raw strings
// (or the name by static index when name_index > 0).
void hpack_put_literal(std::string* out, const std::string& name, const std::string& value, int name_index = 0);
// Indexed header field (a static-table entry).
inline void hpack_put_indexed(std::string* out, int index) { hpack_put_int(out, 0x80, 7, uint64_t(index)); }

}  // namespace net
}  // namespace dtfs
