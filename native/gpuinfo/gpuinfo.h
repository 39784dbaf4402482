// kgs gpuinfo: native AMD GPU enumeration for the device plugin and the CLI.
//
// Source of truth is the KFD topology in sysfs (/sys/class/kfd/kfd/topology),
// which every ROCm host exposes without any library: one node per CPU socket and
// per GPU (or GPU partition), with the DRM render minor, PCI location, XCC
// count, HBM size, hive id and the io_links (type 11 = xGMI, 2 = PCIe) that
// form the xGMI mesh. amd-smi (libamd_smi.so, dlopen'ed, optional; smi.h)
// adds the HIP UUID, ECC/RAS error counts, xGMI link status and its own
// GPU-to-GPU link matrix, which is cross-checked against the KFD io_links;
// HealthMonitor turns the error counts and link status into the plugin's
// Healthy/Unhealthy signal.
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
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "smi.h"

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

// amd-smi's view of the link from this GPU to GPU `to_index`.
struct SmiPeer {
  int to_index = -1;
  int type = 0;  // KFD numbering: 11 xGMI, 2 PCIe, 0 other / unknown
  uint64_t hops = 0, weight = 0;
  int p2p = -1;  // 1 accessible, 0 not, -1 unknown
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
  // amd-smi health sample (-1 = not available)
  int64_t ecc_correctable = -1, ecc_uncorrectable = -1, ecc_deferred = -1;
  int xgmi_links_total = -1, xgmi_links_up = -1, xgmi_links_down = -1;
  std::vector<SmiPeer> smi_links;  // amd-smi link type / hops / weight / P2P to the other GPUs
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
  std::string amdsmi_library;
  // amd-smi's link matrix checked against the KFD io_links (xGMI both ways)
  bool smi_topology_checked = false;
  bool smi_topology_agrees = false;
  std::vector<Gpu> gpus;
  int cpu_nodes = 0;
  std::vector<std::string> warnings;
};

// Enumerate GPUs under `root` ("/" for the live system).
Topology discover(const std::string& root, bool use_amdsmi = true);

// Re-evaluate one GPU's health against the filesystem (device nodes present,
// KFD node still readable). Cheap; the plugin calls it on every health tick.
bool refresh_health(const std::string& root, Gpu& g);

// Stateful health for the device plugin's tick: the sysfs checks of
// refresh_health plus, when amd-smi is available, two hardware signals against a
// per-GPU baseline taken at the first check:
//   * uncorrectable ECC errors rising by more than `ecc_tolerance` -> Unhealthy
//     (a counter that drops -- GPU reset / driver reload -- re-baselines, so a
//     recovered GPU turns Healthy again);
//   * an xGMI link that was up at baseline reported down -> Unhealthy (Healthy
//     again once it is back up).
struct HealthState {
  bool healthy = false;
  std::string reason;
  bool smi = false;  // amd-smi sampled this GPU
  SmiHealth sample;
};

class HealthMonitor {
 public:
  HealthMonitor(const std::string& root, bool use_amdsmi, int64_t ecc_tolerance = 0);
  HealthState check(int node_id, int render_minor, const std::string& bdf = "");
  bool amdsmi_used() const { return smi_ != nullptr; }

 private:
  struct Base {
    int64_t uncorr = -1;
    std::vector<int> links;
  };
  std::string root_;
  std::unique_ptr<SmiSession> smi_;
  std::map<int, Base> base_;  // by render minor
  int64_t tol_;
};

// amd-smi is consulted for the live system ("/") and, for tests, whenever
// KGS_AMDSMI_LIB names a (stub) library.
bool amdsmi_allowed(const std::string& root, bool use_amdsmi);

// "gfx950" from 90500.
std::string gfx_name(uint32_t target_version);

// xGMI hop matrix: [i][j] = link type between GPU i and j (0 if none, -1 = self).
std::vector<std::vector<int>> link_matrix(const Topology& t);

std::string to_json(const Topology& t);

}  // namespace gpuinfo
}  // namespace kgs
