#include "runtime/numa.h"

#include <dirent.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace dtfs {
namespace runtime {

namespace {

constexpr int kMpolPreferred = 1, kMpolBind = 2;
constexpr unsigned kMpolMfStrict = 1u << 0, kMpolMfMove = 1u << 1;
constexpr int kMaxNodes = 1024;

std::string read_file(const std::string& path) {
  std::ifstream f(path);
  if (!f) return std::string();
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

std::vector<int> parse_cpulist(const std::string& s) {
  std::vector<int> out;
  std::stringstream ss(s);
  std::string part;
  while (std::getline(ss, part, ',')) {
    part.erase(std::remove_if(part.begin(), part.end(), [](char c) { return std::isspace(uint8_t(c)); }),
               part.end());
    if (part.empty()) continue;
    const size_t dash = part.find('-');
    const int lo = std::atoi(part.c_str());
    const int hi = dash == std::string::npos ? lo : std::atoi(part.c_str() + dash + 1);
    for (int c = lo; c <= hi; ++c) out.push_back(c);
  }
  return out;
}

struct NodeMask {
  unsigned long bits[kMaxNodes / (8 * sizeof(unsigned long))] = {};
  explicit NodeMask(int node) { bits[size_t(node) / (8 * sizeof(unsigned long))] |= 1ul << (node % (8 * sizeof(unsigned long))); }
};

}  // namespace

int numa_node_count() {
  int n = 0;
  if (DIR* d = opendir("/sys/devices/system/node")) {
    while (dirent* e = readdir(d))
      if (std::strncmp(e->d_name, "node", 4) == 0 && std::isdigit(uint8_t(e->d_name[4]))) ++n;
    closedir(d);
  }
  return std::max(1, n);
}

std::vector<int> numa_node_cpus(int node) {
  if (node < 0) return {};
  return parse_cpulist(read_file("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist"));
}

int pci_numa_node(const std::string& bus_id) {
  std::string id = bus_id;
  std::transform(id.begin(), id.end(), id.begin(), [](char c) { return char(std::tolower(uint8_t(c))); });
  const std::string s = read_file("/sys/bus/pci/devices/" + id + "/numa_node");
  if (s.empty()) return -1;
  const int n = std::atoi(s.c_str());
  return n >= 0 ? n : -1;  // -1: the platform reports no affinity
}

int bind_process_cpus(const std::vector<int>& cpus) {
  if (cpus.empty()) return 0;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus)
    if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &set);
  int n = 0;
  if (DIR* d = opendir("/proc/self/task")) {
    while (dirent* e = readdir(d)) {
      if (!std::isdigit(uint8_t(e->d_name[0]))) continue;
      const pid_t tid = pid_t(std::atoi(e->d_name));
      if (sched_setaffinity(tid, sizeof(set), &set) == 0) ++n;
    }
    closedir(d);
  }
  return n;
}

bool prefer_numa_node(int node) {
  if (node < 0 || node >= kMaxNodes) return false;
  NodeMask m(node);
  return syscall(SYS_set_mempolicy, kMpolPreferred, m.bits, (unsigned long)kMaxNodes) == 0;
}

void* alloc_on_node(size_t bytes, int node) {
  const size_t pg = size_t(sysconf(_SC_PAGESIZE));
  bytes = (bytes + pg - 1) / pg * pg;
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) throw std::runtime_error("alloc_on_node: mmap failed");
  if (node >= 0 && node < kMaxNodes) {
    NodeMask m(node);
    // best effort: a kernel without NUMA (or one node) leaves the default policy
    syscall(SYS_mbind, p, bytes, kMpolBind, m.bits, (unsigned long)kMaxNodes, kMpolMfStrict | kMpolMfMove);
  }
  std::memset(p, 0, bytes);  // first touch: the pages are allocated now, under the policy
  return p;
}

bool bind_range_to_node(void* p, size_t bytes, int node) {
  if (!p || node < 0 || node >= kMaxNodes) return false;
  NodeMask m(node);
  return syscall(SYS_mbind, p, bytes, kMpolBind, m.bits, (unsigned long)kMaxNodes, 0u) == 0;
}

void free_on_node(void* p, size_t bytes) {
  if (!p) return;
  const size_t pg = size_t(sysconf(_SC_PAGESIZE));
  munmap(p, (bytes + pg - 1) / pg * pg);
}

int page_numa_node(const void* p) {
  const size_t pg = size_t(sysconf(_SC_PAGESIZE));
  void* page = reinterpret_cast<void*>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t(pg) - 1));
  int status = -1;
  if (syscall(SYS_move_pages, 0, 1ul, &page, nullptr, &status, 0) != 0) return -1;
  return status >= 0 ? status : -1;
}

}  // namespace runtime
}  // namespace dtfs
