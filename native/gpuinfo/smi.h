// kgs gpuinfo: the amd-smi session (libamd_smi.so, dlopen'ed).
//
// Everything amd-smi contributes -- HIP UUID, ECC/RAS error counts, xGMI link
// status, and the GPU-to-GPU link type / hops / weight / P2P view -- comes
// through one SmiSession, keyed by DRM render minor (the identity KFD sysfs
// also reports). The library is resolved at run time: the device-plugin image
// needs no ROCm install, and tests point KGS_AMDSMI_LIB at a stub library
// (native/gpuinfo/testing/amdsmi_stub.cpp) that injects error counts.
//
// The reference has no health signal at all; its upstream plugin (Go, cloned at
// kind-gpu-sim.sh:212-217) is what this replaces.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace kgs {
namespace gpuinfo {

struct SmiGpu {
  int render_minor = -1;
  std::string bdf;
  std::string uuid;
  void* handle = nullptr;  // amdsmi_processor_handle
};

struct SmiHealth {
  bool ecc_ok = false;  // the ECC query succeeded
  int64_t ecc_correctable = -1, ecc_uncorrectable = -1, ecc_deferred = -1;
  bool links_ok = false;  // the xGMI link-status query succeeded
  int links_total = -1, links_up = -1, links_down = -1;
  std::vector<int> link_state;  // per link: 0 down, 1 up, 2 disabled
};

struct SmiLink {
  bool ok = false;
  int type = 0;       // in KFD io_link numbering: 11 xGMI, 2 PCIe, 0 other/unknown
  uint64_t hops = 0;
  uint64_t weight = 0;
  int p2p = -1;       // 1 accessible, 0 not, -1 unknown
};

class SmiSession {
 public:
  // nullptr if the library is missing, disabled (KGS_NO_AMDSMI) or init fails.
  static std::unique_ptr<SmiSession> open();
  ~SmiSession();

  const std::vector<SmiGpu>& gpus() const { return gpus_; }
  const SmiGpu* by_minor(int minor) const;
  const SmiGpu* by_bdf(const std::string& bdf) const;
  bool health(const SmiGpu& g, SmiHealth& out) const;
  SmiLink link(const SmiGpu& a, const SmiGpu& b) const;
  const std::string& library() const { return lib_; }

  struct Api;

 private:
  SmiSession() = default;
  void* dl_ = nullptr;
  std::string lib_;
  std::unique_ptr<Api> api_;
  std::vector<SmiGpu> gpus_;
};

}  // namespace gpuinfo
}  // namespace kgs
