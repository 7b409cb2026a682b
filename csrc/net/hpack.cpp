#include "net/hpack.h"

#include <array>

#include "net/hpack_huffman.h"

namespace dtfs {
namespace net {

namespace {

// RFC 7541 Appendix A (names checked against libnghttp2's encoder: tools/derive_hpack_huffman.py)
const Header kStatic[61] = {
    {":authority", ""},
    {":method", "GET"},
    {":method", "POST"},
    {":path", "/"},
    {":path", "/index.html"},
    {":scheme", "http"},
    {":scheme", "https"},
    {":status", "200"},
    {":status", "204"},
    {":status", "206"},
    {":status", "304"},
    {":status", "400"},
    {":status", "404"},
    {":status", "500"},
    {"accept-charset", ""},
    {"accept-encoding", "gzip, deflate"},
    {"accept-language", ""},
    {"accept-ranges", ""},
    {"accept", ""},
    {"access-control-allow-origin", ""},
    {"age", ""},
    {"allow", ""},
    {"authorization", ""},
    {"cache-control", ""},
    {"content-disposition", ""},
    {"content-encoding", ""},
    {"content-language", ""},
    {"content-length", ""},
    {"content-location", ""},
    {"content-range", ""},
    {"content-type", ""},
    {"cookie", ""},
    {"date", ""},
    {"etag", ""},
    {"expect", ""},
    {"expires", ""},
    {"from", ""},
    {"host", ""},
    {"if-match", ""},
    {"if-modified-since", ""},
    {"if-none-match", ""},
    {"if-range", ""},
    {"if-unmodified-since", ""},
    {"last-modified", ""},
    {"link", ""},
    {"location", ""},
    {"max-forwards", ""},
    {"proxy-authenticate", ""},
    {"proxy-authorization", ""},
    {"range", ""},
    {"referer", ""},
    {"refresh", ""},
    {"retry-after", ""},
    {"server", ""},
    {"set-cookie", ""},
    {"strict-transport-security", ""},
    {"transfer-encoding", ""},
    {"user-agent", ""},
    {"vary", ""},
    {"via", ""},
    {"www-authenticate", ""},
};

// Binary decode tree of the canonical code: node 0 is the root; a leaf holds
// sym >= 0. 257 leaves -> 256 internal nodes.
struct HuffTree {
  struct Node {
    int16_t child[2] = {-1, -1};
    int16_t sym = -1;
  };
  std::array<Node, 520> nodes{};
  int used = 1;
  HuffTree() {
    for (int s = 0; s < 257; ++s) {
      const uint32_t code = kHuffTable[s].code;
      const int bits = kHuffTable[s].bits;
      int n = 0;
      for (int b = bits - 1; b >= 0; --b) {
        const int bit = (code >> b) & 1;
        if (nodes[size_t(n)].child[bit] < 0) nodes[size_t(n)].child[bit] = int16_t(used++);
        n = nodes[size_t(n)].child[bit];
      }
      nodes[size_t(n)].sym = int16_t(s);
    }
  }
};

const HuffTree& tree() {
  static const HuffTree t;
  return t;
}

bool get_int(const uint8_t*& p, const uint8_t* end, int prefix, uint64_t* v) {
  if (p >= end) return false;
  const uint64_t mask = (uint64_t(1) << prefix) - 1;
  uint64_t x = *p++ & mask;
  if (x < mask) {
    *v = x;
    return true;
  }
  for (int shift = 0; shift <= 56; shift += 7) {
    if (p >= end) return false;
    const uint8_t c = *p++;
    x += uint64_t(c & 0x7f) << shift;
    if (!(c & 0x80)) {
      *v = x;
      return true;
    }
  }
  return false;  // absurdly long integer
}

bool get_string(const uint8_t*& p, const uint8_t* end, std::string* out) {
  if (p >= end) return false;
  const bool huff = (*p & 0x80) != 0;
  uint64_t len;
  if (!get_int(p, end, 7, &len) || len > uint64_t(end - p)) return false;
  if (huff) {
    out->clear();
    if (!huffman_decode(p, size_t(len), out)) return false;
  } else {
    out->assign(reinterpret_cast<const char*>(p), size_t(len));
  }
  p += len;
  return true;
}

}  // namespace

bool huffman_decode(const uint8_t* p, size_t n, std::string* out) {
  const HuffTree& t = tree();
  out->reserve(out->size() + n * 8 / 5 + 1);
  int node = 0, depth = 0;
  bool all_ones = true;  // the bits since the last complete symbol
  for (size_t i = 0; i < n; ++i) {
    for (int b = 7; b >= 0; --b) {
      const int bit = (p[i] >> b) & 1;
      node = t.nodes[size_t(node)].child[bit];
      if (node < 0) return false;
      ++depth;
      all_ones = all_ones && bit;
      const int sym = t.nodes[size_t(node)].sym;
      if (sym >= 0) {
        if (sym == 256) return false;  // EOS inside a string is an error (5.2)
        out->push_back(char(sym));
        node = 0;
        depth = 0;
        all_ones = true;
      }
    }
  }
  // padding: fewer than 8 bits, the most significant bits of EOS (all ones)
  return depth < 8 && all_ones;
}

std::string huffman_encode(const std::string& s) {
  std::string out;
  uint64_t acc = 0;
  int nbits = 0;
  for (unsigned char c : s) {
    acc = (acc << kHuffTable[c].bits) | kHuffTable[c].code;
    nbits += kHuffTable[c].bits;
    while (nbits >= 8) {
      out.push_back(char((acc >> (nbits - 8)) & 0xff));
      nbits -= 8;
    }
  }
  if (nbits > 0) out.push_back(char(((acc << (8 - nbits)) | ((1u << (8 - nbits)) - 1)) & 0xff));
  return out;
}

void hpack_put_int(std::string* out, uint8_t first, int prefix, uint64_t v) {
  const uint64_t mask = (uint64_t(1) << prefix) - 1;
  if (v < mask) {
    out->push_back(char(first | uint8_t(v)));
    return;
  }
  out->push_back(char(first | uint8_t(mask)));
  v -= mask;
  while (v >= 128) {
    out->push_back(char(0x80 | (v & 0x7f)));
    v >>= 7;
  }
  out->push_back(char(v));
}

void hpack_put_literal(std::string* out, const std::string& name, const std::string& value, int name_index) {
  hpack_put_int(out, 0x00, 4, uint64_t(name_index));  // literal without indexing
  if (name_index == 0) {
    hpack_put_int(out, 0x00, 7, name.size());
    out->append(name);
  }
  hpack_put_int(out, 0x00, 7, value.size());
  out->append(value);
}

bool HpackDecoder::lookup(uint64_t index, Header* h, std::string* err) const {
  if (index == 0) {
    *err = "header index 0";
    return false;
  }
  if (index <= 61) {
    *h = kStatic[index - 1];
    return true;
  }
  const uint64_t d = index - 62;
  if (d >= dyn_.size()) {
    *err = "header index " + std::to_string(index) + " past the dynamic table";
    return false;
  }
  *h = dyn_[size_t(d)];
  return true;
}

void HpackDecoder::evict_to(size_t cap) {
  while (size_ > cap && !dyn_.empty()) {
    size_ -= dyn_.back().first.size() + dyn_.back().second.size() + 32;
    dyn_.pop_back();
  }
}

void HpackDecoder::insert(Header h) {
  const size_t sz = h.first.size() + h.second.size() + 32;
  if (sz > limit_) {  // larger than the table: empties it, not inserted (4.4)
    evict_to(0);
    return;
  }
  evict_to(limit_ - sz);
  size_ += sz;
  dyn_.push_front(std::move(h));
}

bool HpackDecoder::decode(const uint8_t* p, size_t n, std::vector<Header>* out, std::string* err, size_t max_list) {
  const uint8_t* end = p + n;
  bool field_seen = false;
  size_t list = 0;  // RFC 7540 6.5.2 header list size: name + value + 32 per field
  auto over = [&](const Header& h) {
    list += h.first.size() + h.second.size() + 32;
    if (max_list && list > max_list) {
      *err = "header list larger than SETTINGS_MAX_HEADER_LIST_SIZE";
      return true;
    }
    return false;
  };
  while (p < end) {
    const uint8_t c = *p;
    if (c & 0x80) {  // indexed
      uint64_t idx;
      Header h;
      if (!get_int(p, end, 7, &idx) || !lookup(idx, &h, err)) {
        if (err->empty()) *err = "truncated index";
        return false;
      }
      if (over(h)) return false;
      out->push_back(std::move(h));
      field_seen = true;
    } else if ((c & 0xe0) == 0x20) {  // dynamic table size update
      uint64_t sz;
      if (!get_int(p, end, 5, &sz)) {
        *err = "truncated table size update";
        return false;
      }
      if (field_seen) {
        *err = "table size update after a header field";
        return false;
      }
      if (sz > max_) {
        *err = "table size update above SETTINGS_HEADER_TABLE_SIZE";
        return false;
      }
      limit_ = size_t(sz);
      evict_to(limit_);
    } else {  // literal: with incremental indexing (01), without (0000) or never indexed (0001)
      const bool incremental = (c & 0xc0) == 0x40;
      const int prefix = incremental ? 6 : 4;
      uint64_t idx;
      if (!get_int(p, end, prefix, &idx)) {
        *err = "truncated literal";
        return false;
      }
      Header h;
      if (idx) {
        if (!lookup(idx, &h, err)) return false;
      } else if (!get_string(p, end, &h.first)) {
        *err = "bad literal name";
        return false;
      }
      if (!get_string(p, end, &h.second)) {
        *err = "bad literal value";
        return false;
      }
      if (over(h)) return false;
      if (incremental) insert(h);
      out->push_back(std::move(h));
      field_seen = true;
    }
  }
  return true;
}

}  // namespace net
}  // namespace dtfs
