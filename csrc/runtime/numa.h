// NUMA placement of a rank's host side (no libnuma: raw syscalls + sysfs).
//
// On an 8-GPU MI355X node half of the GPUs hang off each CPU socket. A rank
// whose request arenas (the pinned buffers every H2D step copy reads) and
// serving threads sit on the far socket pays the inter-socket link on every
// copy - and the H2D copy is most of the DeepFM step period. So each rank
// finds its GPU's NUMA node from the PCI bus id (sysfs), pins its threads to
// that node's CPUs (sched_setaffinity for every thread of the process, new
// threads inherit) and allocates its arenas on that node (mmap + mbind +
// first touch) before registering them with the GPU (hipHostRegister, in the
// _hip module). The reference has no host placement at all (a Java client
// against remote hosts, DCNClient.java:118-125).
#pragma once

#include <cstddef>
#include <string>
#include <vector>

namespace dtfs {
namespace runtime {

int numa_node_count();                                  // nodes under /sys/devices/system/node (>= 1)
std::vector<int> numa_node_cpus(int node);              // the node's cpulist (empty: unknown node)
int pci_numa_node(const std::string& bus_id);           // "0000:65:00.0" -> node, -1 unknown / none
// Bind every thread of this process to `cpus` (threads created later inherit
// the calling thread's mask). Returns the number of threads re-bound.
int bind_process_cpus(const std::vector<int>& cpus);
// This thread's future allocations prefer `node` (set_mempolicy MPOL_PREFERRED).
bool prefer_numa_node(int node);
// Anonymous memory whose pages live on `node` (mbind MPOL_BIND, touched).
// Page-aligned; free with free_on_node(p, bytes).
void* alloc_on_node(size_t bytes, int node);
void free_on_node(void* p, size_t bytes);
// Place the (not yet touched) pages of [p, p + bytes) on `node` (mbind
// MPOL_BIND; p page-aligned). false: no NUMA support / bad node.
bool bind_range_to_node(void* p, size_t bytes, int node);
// The NUMA node of the page holding `p` (move_pages query), -1 on error.
int page_numa_node(const void* p);

}  // namespace runtime
}  // namespace dtfs
