// kgs gpuinfo: native AMD GPU enumeration for the device plugin and the CLI.
//
// Source of truth is the KFD topology in sysfs (/sys/class/kfd/kfd/topology),
// which every ROCm host exposes without any library: one node per CPU socket and
// per GPU (or GPU partition), with the DRM render minor, PCI location, XCC
// count, HBM size, hive id and the io_links (type 11 = xGMI, 2 = PCIe) that
// form the xGMI mesh. amd-smi (libamd_smi.so, dlopen'ed, optional) enriches
// the records with the HIP UUID.
//
// Everything is parameterised by a filesystem `root` so tests run against a
// fake tree (tests/fixtures/) and the plugin can read the host's /sys mounted
// at any path.
//
// The reference has no device discovery: it patches a constant "2" into node
// capacity (kind-gpu-sim.sh:113). Its upstream ROCm plugin (Go) is the
// component this replaces.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace kgs {
namespace gpuinfo {

enum LinkType : int {
  LINK_UNKNOWN = 0,
  LINK_PCIE = 2,
  LINK_XGMI = 11,
};

struct Link {
  int to_node = -1;     // KFD node id of the peer
  int type = 0;         // KFD io_link type (11 = xGMI)
  int weight = 0;       // KFD link weight (lower = closer)
  uint64_t max_bandwidth_mbs = 0;
};

struct Gpu {
  int node_id = -1;           // KFD topology node
  uint32_t gpu_id = 0;        // KFD gpu_id
  int index = -1;             // ordinal among GPUs, by node id (== HIP order when all visible)
  int render_minor = -1;      // /dev/dri/renderD<minor>
  std::string bdf;            // 0000:5a:00.0
  uint64_t unique_id = 0;
  uint64_t hive_id = 0;
  uint32_t gfx_target_version = 0;  // 90500 for gfx950
  std::string gfx_arch;             // "gfx950"
  uint32_t vendor_id = 0, device_id = 0;
  int simd_count = 0, cu_count = 0, num_xcc = 0;
  int lds_kb = 0, wave_size = 0;
  int max_clock_mhz = 0;
  uint64_t vram_bytes = 0;
  int numa_node = -1;
  std::string uuid;           // from amd-smi when available
  bool properties_readable = false;
  bool render_node_present = false;
  bool healthy = false;
  std::string health_reason;
  std::vector<Link> links;    // io_links to other GPU nodes
};

struct Topology {
  std::string root;
  bool kfd_present = false;       // <root>/dev/kfd exists
  bool topology_present = false;  // KFD topology directory exists
  bool amdsmi_used = false;
  std::vector<Gpu> gpus;
  int cpu_nodes = 0;
  std::vector<std::string> warnings;
};

// Enumerate GPUs under `root` ("/" for the live system).
Topology discover(const std::string& root, bool use_amdsmi = true);

// Re-evaluate one GPU's health against the filesystem (device nodes present,
// KFD node still readable). Cheap; the plugin calls it on every health tick.
bool refresh_health(const std::string& root, Gpu& g);

// "gfx950" from 90500.
std::string gfx_name(uint32_t target_version);

// xGMI hop matrix: [i][j] = link type between GPU i and j (0 if none, -1 = self).
std::vector<std::vector<int>> link_matrix(const Topology& t);

std::string to_json(const Topology& t);

}  // namespace gpuinfo
}  // namespace kgs
