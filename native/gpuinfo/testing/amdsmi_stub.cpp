// Test double for libamd_smi.so: the subset of the amd-smi C API that
// native/gpuinfo/smi.cpp resolves, driven by a text state file that tests
// rewrite while a plugin is running (ECC errors appear, xGMI links drop).
//
// State file ($KGS_AMDSMI_STUB_STATE), re-read on every call:
//   gpu <render_minor> <bdf> <uuid> <corr> <uncorr> <deferred> <link states, e.g. 1111111>
//   link <minor_a> <minor_b> <type: xgmi|pcie> <hops> <weight>
// A pair with no `link` line reports PCIe, 2 hops, weight 40. Link states:
// 1 = up, 0 = down, 2 = disabled.
//
// Loaded only through KGS_AMDSMI_LIB (never by production code); built into
// kgs/_native/libamd_smi_stub.so by kgs/utils/build.py.
#include <amd_smi/amdsmi.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

namespace {

struct StubGpu {
  int minor = -1;
  unsigned dom = 0, bus = 0, dev = 0, fn = 0;
  std::string uuid;
  unsigned long long corr = 0, uncorr = 0, deferred = 0;
  std::string links;
};

struct StubLink {
  int a = -1, b = -1;
  bool xgmi = false;
  unsigned long long hops = 0, weight = 0;
};

struct State {
  std::vector<StubGpu> gpus;
  std::vector<StubLink> links;
};

State load() {
  State s;
  const char* p = std::getenv("KGS_AMDSMI_STUB_STATE");
  if (!p) return s;
  std::ifstream f(p);
  std::string line;
  while (std::getline(f, line)) {
    std::istringstream is(line);
    std::string kind;
    is >> kind;
    if (kind == "gpu") {
      StubGpu g;
      std::string bdf;
      is >> g.minor >> bdf >> g.uuid >> g.corr >> g.uncorr >> g.deferred >> g.links;
      std::sscanf(bdf.c_str(), "%x:%x:%x.%x", &g.dom, &g.bus, &g.dev, &g.fn);
      s.gpus.push_back(g);
    } else if (kind == "link") {
      StubLink L;
      std::string t;
      is >> L.a >> L.b >> t >> L.hops >> L.weight;
      L.xgmi = t == "xgmi";
      s.links.push_back(L);
    }
  }
  return s;
}

// handles are 1-based GPU ordinals; the single socket handle is a constant
int ordinal(amdsmi_processor_handle h) { return (int)(reinterpret_cast<uintptr_t>(h)) - 1; }

bool gpu_at(amdsmi_processor_handle h, StubGpu& out) {
  State s = load();
  const int i = ordinal(h);
  if (i < 0 || i >= (int)s.gpus.size()) return false;
  out = s.gpus[i];
  return true;
}

const StubLink* find_link(const State& s, int a, int b) {
  for (auto& L : s.links)
    if ((L.a == a && L.b == b) || (L.a == b && L.b == a)) return &L;
  return nullptr;
}

int initialized = 0;

}  // namespace

extern "C" {

amdsmi_status_t amdsmi_init(uint64_t) {
  initialized = 1;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_shut_down() {
  initialized = 0;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_socket_handles(uint32_t* count, amdsmi_socket_handle* handles) {
  if (!initialized) return AMDSMI_STATUS_NOT_INIT;
  const bool any = !load().gpus.empty();
  if (!handles) {
    *count = any ? 1 : 0;
    return AMDSMI_STATUS_SUCCESS;
  }
  if (*count >= 1 && any) handles[0] = reinterpret_cast<amdsmi_socket_handle>(uintptr_t(0x5eed));
  *count = any ? 1 : 0;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_processor_handles(amdsmi_socket_handle, uint32_t* count,
                                             amdsmi_processor_handle* handles) {
  const uint32_t n = (uint32_t)load().gpus.size();
  if (!handles) {
    *count = n;
    return AMDSMI_STATUS_SUCCESS;
  }
  const uint32_t m = *count < n ? *count : n;
  for (uint32_t i = 0; i < m; ++i) handles[i] = reinterpret_cast<amdsmi_processor_handle>(uintptr_t(i + 1));
  *count = m;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_enumeration_info(amdsmi_processor_handle h, amdsmi_enumeration_info_t* info) {
  StubGpu g;
  if (!gpu_at(h, g)) return AMDSMI_STATUS_INVAL;
  std::memset(info, 0, sizeof *info);
  info->drm_render = (uint32_t)g.minor;
  info->hip_id = (uint32_t)ordinal(h);
  std::snprintf(info->hip_uuid, sizeof info->hip_uuid, "%s", g.uuid.c_str());
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_device_bdf(amdsmi_processor_handle h, amdsmi_bdf_t* bdf) {
  StubGpu g;
  if (!gpu_at(h, g)) return AMDSMI_STATUS_INVAL;
  std::memset(bdf, 0, sizeof *bdf);
  bdf->domain_number = g.dom;
  bdf->bus_number = g.bus;
  bdf->device_number = g.dev;
  bdf->function_number = g.fn;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_device_uuid(amdsmi_processor_handle h, unsigned int* len, char* uuid) {
  StubGpu g;
  if (!gpu_at(h, g)) return AMDSMI_STATUS_INVAL;
  std::snprintf(uuid, *len, "%s", g.uuid.c_str());
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_total_ecc_count(amdsmi_processor_handle h, amdsmi_error_count_t* ec) {
  StubGpu g;
  if (!gpu_at(h, g)) return AMDSMI_STATUS_INVAL;
  std::memset(ec, 0, sizeof *ec);
  ec->correctable_count = g.corr;
  ec->uncorrectable_count = g.uncorr;
  ec->deferred_count = g.deferred;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_xgmi_link_status(amdsmi_processor_handle h, amdsmi_xgmi_link_status_t* ls) {
  StubGpu g;
  if (!gpu_at(h, g)) return AMDSMI_STATUS_INVAL;
  std::memset(ls, 0, sizeof *ls);
  const size_t n = g.links.size() < AMDSMI_MAX_NUM_XGMI_LINKS ? g.links.size() : AMDSMI_MAX_NUM_XGMI_LINKS;
  ls->total_links = (uint32_t)n;
  for (size_t i = 0; i < n; ++i)
    ls->status[i] = g.links[i] == '1' ? AMDSMI_XGMI_LINK_UP
                    : g.links[i] == '0' ? AMDSMI_XGMI_LINK_DOWN
                                        : AMDSMI_XGMI_LINK_DISABLE;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_topo_get_link_type(amdsmi_processor_handle a, amdsmi_processor_handle b, uint64_t* hops,
                                          amdsmi_link_type_t* type) {
  StubGpu ga, gb;
  if (!gpu_at(a, ga) || !gpu_at(b, gb)) return AMDSMI_STATUS_INVAL;
  State s = load();
  const StubLink* L = find_link(s, ga.minor, gb.minor);
  *hops = L ? L->hops : 2;
  *type = (L && L->xgmi) ? AMDSMI_LINK_TYPE_XGMI : AMDSMI_LINK_TYPE_PCIE;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_topo_get_link_weight(amdsmi_processor_handle a, amdsmi_processor_handle b, uint64_t* weight) {
  StubGpu ga, gb;
  if (!gpu_at(a, ga) || !gpu_at(b, gb)) return AMDSMI_STATUS_INVAL;
  State s = load();
  const StubLink* L = find_link(s, ga.minor, gb.minor);
  *weight = L ? L->weight : 40;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_is_P2P_accessible(amdsmi_processor_handle a, amdsmi_processor_handle b, bool* accessible) {
  StubGpu ga, gb;
  if (!gpu_at(a, ga) || !gpu_at(b, gb)) return AMDSMI_STATUS_INVAL;
  State s = load();
  const StubLink* L = find_link(s, ga.minor, gb.minor);
  *accessible = L && L->xgmi;
  return AMDSMI_STATUS_SUCCESS;
}

}  // extern "C"
